"""Test helpers: Arrow-style columns <-> per-row Python values, column comparison."""
from __future__ import annotations

import struct
from typing import List, Sequence

import numpy as np

from fury_amd.types import (BINARY, BOOL, DATE32, DECIMAL, FLOAT32, FLOAT64, INT8, INT16, INT32,
                            INT64, LIST, MAP, STRING, STRUCT, TIMESTAMP, Field, type_width)

from fury_amd.beans import columns_to_beans, value_at  # noqa: F401


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
        elif t == MAP:
            go = as_u8(g.offsets).view(np.int32)[:n + 1]
            wo = as_u8(w.offsets).view(np.int32)[:n + 1]
            assert np.array_equal(go, wo), f"{p}: map offsets"
            assert_columns_equal(f.children, g.child, w.child, int(wo[n]), p + ".")
        else:
            raise ValueError(t)


def float_bits_equal(a: float, b: float, t: int) -> bool:
    fmt = "<f" if t == FLOAT32 else "<d"
    return struct.pack(fmt, a) == struct.pack(fmt, b)
