"""Test helpers: Arrow-style columns <-> per-row Python values, column comparison."""
from __future__ import annotations

import struct
from typing import List, Sequence

import numpy as np

from fury_amd.types import (BINARY, BOOL, DATE32, DECIMAL, FLOAT32, FLOAT64, INT8, INT16, INT32,
                            INT64, LIST, MAP, STRING, STRUCT, TIMESTAMP, Field, type_width)

_NP = {INT8: np.int8, INT16: np.int16, INT32: np.int32, INT64: np.int64, FLOAT32: np.float32,
       FLOAT64: np.float64, DATE32: np.int32, TIMESTAMP: np.int64}


def _valid(c, i):
    return c.validity is None or bool((int(c.validity[i >> 3]) >> (i & 7)) & 1)


def value_at(f: Field, c, i: int):
    """Python value of entry i (None for null), matching oracle/bean_oracle.py conventions."""
    if not _valid(c, i):
        return None
    t = f.type_id
    if t == BOOL:
        return bool((int(np.asarray(c.values).view(np.uint8)[i >> 3]) >> (i & 7)) & 1)
    if type_width(t) > 0:
        v = np.asarray(c.values).view(np.uint8).view(_NP[t])[i]
        if t in (FLOAT32, FLOAT64):
            # keep the raw bits: return the float but through struct to preserve NaN payloads
            return float(v)
        return int(v)
    if t in (STRING, BINARY):
        b = bytes(np.asarray(c.values).view(np.uint8)[int(c.offsets[i]):int(c.offsets[i + 1])])
        return b.decode("utf-8") if t == STRING else b
    if t == DECIMAL:
        return bytes(np.asarray(c.values).view(np.uint8)[16 * i:16 * i + 16])
    if t == LIST:
        return [value_at(f.children[0], c.child[0], j)
                for j in range(int(c.offsets[i]), int(c.offsets[i + 1]))]
    if t == STRUCT:
        return {fc.name: value_at(fc, cc, i) for fc, cc in zip(f.children, c.child)}
    if t == MAP:
        return [(value_at(f.children[0], c.child[0], j), value_at(f.children[1], c.child[1], j))
                for j in range(int(c.offsets[i]), int(c.offsets[i + 1]))]
    raise ValueError(t)


def columns_to_beans(fields: Sequence[Field], cols, n: int) -> List[dict]:
    return [{f.name: value_at(f, c, i) for f, c in zip(fields, cols)} for i in range(n)]


def as_u8(a) -> np.ndarray:
    if a is None:
        return None
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(a)).view(np.uint8).reshape(-1)


def bits(a, n: int) -> np.ndarray:
    """First n bits (LSB-first) of a bitmap as bool array."""
    return np.unpackbits(as_u8(a), bitorder="little")[:n].astype(bool)


def assert_columns_equal(fields: Sequence[Field], got, want, n: int, path: str = ""):
    """Byte-exact comparison of decoded columns (values of null entries must be 0 on both)."""
    for f, g, w in zip(fields, got, want):
        p = f"{path}{f.name}"
        if w.validity is not None and g.validity is not None:
            assert np.array_equal(bits(g.validity, n), bits(w.validity, n)), f"{p}: validity"
        t = f.type_id
        if t == BOOL:
            assert np.array_equal(bits(g.values, n), bits(w.values, n)), f"{p}: bool values"
        elif type_width(t) > 0:
            nb = n * type_width(t)
            assert np.array_equal(as_u8(g.values)[:nb], as_u8(w.values)[:nb]), f"{p}: values"
        elif t == DECIMAL:
            assert np.array_equal(as_u8(g.values)[:16 * n], as_u8(w.values)[:16 * n]), p
        elif t in (STRING, BINARY):
            go = as_u8(g.offsets).view(np.int32)[:n + 1]
            wo = as_u8(w.offsets).view(np.int32)[:n + 1]
            assert np.array_equal(go - go[0], wo - wo[0]), f"{p}: offsets"
            m = int(wo[n] - wo[0])
            assert np.array_equal(as_u8(g.values)[go[0]:go[0] + m],
                                  as_u8(w.values)[wo[0]:wo[0] + m]), f"{p}: payload"
        elif t == LIST:
            go = as_u8(g.offsets).view(np.int32)[:n + 1]
            wo = as_u8(w.offsets).view(np.int32)[:n + 1]
            assert np.array_equal(go, wo), f"{p}: list offsets"
            assert_columns_equal(f.children, g.child, w.child, int(wo[n]), p + ".")
        elif t == STRUCT:
            assert_columns_equal(f.children, g.child, w.child, n, p + ".")
        else:
            raise ValueError(t)


def float_bits_equal(a: float, b: float, t: int) -> bool:
    fmt = "<f" if t == FLOAT32 else "<d"
    return struct.pack(fmt, a) == struct.pack(fmt, b)
