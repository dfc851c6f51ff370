"""Host-side bean <-> column materialisation (the part of generated toRow/fromRow that touches
Java objects and therefore stays on the host).  A bean is a ``dict`` field name ->
value; None is null.  Values: bool, int, float, str (STRING), bytes (BINARY / 16-byte DECIMAL),
list (LIST).  Used by the single-object RowEncoder methods; batch paths hand columns directly.
"""
from __future__ import annotations

import struct
from typing import List, Sequence

import numpy as np

from .types import (BINARY, BOOL, DATE32, DECIMAL, FLOAT32, FLOAT64, INT8, INT16, INT32, INT64,
                    LIST, MAP, STRING, STRUCT, TIMESTAMP, Field, type_width)
from .workloads import Column

NP_DTYPE = {INT8: np.int8, INT16: np.int16, INT32: np.int32, INT64: np.int64, FLOAT32: np.float32,
            FLOAT64: np.float64, DATE32: np.int32, TIMESTAMP: np.int64}


def _bits(flags: Sequence[bool]) -> np.ndarray:
    return np.packbits(np.asarray(flags, dtype=np.uint8), bitorder="little")


def values_to_column(f: Field, vals: list) -> Column:
    """One field's values (one per row / element) -> Arrow-style host column."""
    valid = [v is not None for v in vals]
    validity = _bits(valid) if f.nullable or not all(valid) else None
    t = f.type_id
    if t == BOOL:
        return Column(values=_bits([bool(v) if v is not None else False for v in vals]),
                      validity=validity)
    if type_width(t) > 0:
        dt = NP_DTYPE[t]
        arr = np.array([v if v is not None else 0 for v in vals], dtype=dt)
        return Column(values=arr, validity=validity)
    if t in (STRING, BINARY):
        parts = [(v.encode("utf-8") if t == STRING else bytes(v)) if v is not None else b""
                 for v in vals]
        offs = np.zeros(len(parts) + 1, np.int32)
        np.cumsum([len(p) for p in parts], out=offs[1:])
        data = np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy()
        return Column(values=data, validity=validity, offsets=offs)
    if t == DECIMAL:
        data = b"".join(bytes(v) if v is not None else bytes(16) for v in vals)
        return Column(values=np.frombuffer(data or bytes(16), np.uint8).copy(), validity=validity)
    if t == LIST:
        flat: list = []
        offs = np.zeros(len(vals) + 1, np.int32)
        for i, v in enumerate(vals):
            if v is not None:
                flat.extend(v)
            offs[i + 1] = len(flat)
        return Column(validity=validity, offsets=offs,
                      child=[values_to_column(f.children[0], flat)])
    if t == STRUCT:
        return Column(validity=validity,
                      child=[values_to_column(c, [None if v is None else v.get(c.name)
                                                  for v in vals]) for c in f.children])
    if t == MAP:
        keys: list = []
        items: list = []
        offs = np.zeros(len(vals) + 1, np.int32)
        for i, v in enumerate(vals):
            if v is not None:
                for k, x in v:
                    keys.append(k)
                    items.append(x)
            offs[i + 1] = len(keys)
        return Column(validity=validity, offsets=offs,
                      child=[values_to_column(f.children[0], keys),
                             values_to_column(f.children[1], items)])
    raise ValueError(f"unsupported type {t}")


def beans_to_columns(fields: Sequence[Field], beans: Sequence[dict]) -> List[Column]:
    return [values_to_column(f, [b.get(f.name) for b in beans]) for f in fields]


def _valid(c: Column, i: int) -> bool:
    return c.validity is None or bool((int(np.asarray(c.validity)[i >> 3]) >> (i & 7)) & 1)


def value_at(f: Field, c: Column, i: int):
    if not _valid(c, i):
        return None
    t = f.type_id
    if t == BOOL:
        return bool((int(np.asarray(c.values).view(np.uint8)[i >> 3]) >> (i & 7)) & 1)
    if type_width(t) > 0:
        v = np.asarray(c.values).view(np.uint8).view(NP_DTYPE[t])[i]
        return float(v) if t in (FLOAT32, FLOAT64) else int(v)
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


def columns_to_beans(fields: Sequence[Field], cols: Sequence[Column], n: int) -> List[dict]:
    return [{f.name: value_at(f, c, i) for f, c in zip(fields, cols)} for i in range(n)]


def pack_float_bits(v: float, t: int) -> bytes:
    return struct.pack("<f" if t == FLOAT32 else "<d", v)
