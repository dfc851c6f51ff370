"""Host export of device-produced Arrow columns as a ``pyarrow.RecordBatch`` — the host end of
``ArrowWriter.finishAsRecordBatch`` (java/fury-format/.../vectorized/ArrowWriter.java:89-93).
The buffers are the ones the device kernels wrote (validity bit = 1 valid, int32 offsets);
pyarrow only wraps them (``Array.from_buffers``), nothing is recomputed here."""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import pyarrow as pa

from .types import (BINARY, BOOL, DATE32, DECIMAL, FLOAT32, FLOAT64, INT8, INT16, INT32, INT64,
                    LIST, MAP, STRING, STRUCT, TIMESTAMP, Field)
from .workloads import Column

_PA = {BOOL: pa.bool_(), INT8: pa.int8(), INT16: pa.int16(), INT32: pa.int32(),
       INT64: pa.int64(), FLOAT32: pa.float32(), FLOAT64: pa.float64(), STRING: pa.utf8(),
       BINARY: pa.binary(), DATE32: pa.date32(), TIMESTAMP: pa.timestamp("us"),
       DECIMAL: pa.decimal128(38, 18)}


def pa_type(f: Field) -> pa.DataType:
    if f.type_id in _PA:
        return _PA[f.type_id]
    if f.type_id == LIST:
        e = f.children[0]
        return pa.list_(pa.field(e.name, pa_type(e), e.nullable))
    if f.type_id == STRUCT:
        return pa.struct([pa.field(c.name, pa_type(c), c.nullable) for c in f.children])
    if f.type_id == MAP:
        k, v = f.children
        return pa.map_(pa.field(k.name, pa_type(k), False), pa.field(v.name, pa_type(v), v.nullable))
    raise NotImplementedError(f"no Arrow export for {f}")


def _buf(a) -> pa.Buffer:
    return pa.py_buffer(np.ascontiguousarray(np.asarray(a)).view(np.uint8))


def column_to_array(f: Field, c: Column, n: int) -> pa.Array:
    t = pa_type(f)
    vb = _buf(c.validity) if c.validity is not None else None
    if f.type_id in (STRING, BINARY):
        return pa.Array.from_buffers(t, n, [vb, _buf(c.offsets), _buf(c.values)])
    if f.type_id == LIST:
        m = int(np.asarray(c.offsets)[n])
        child = column_to_array(f.children[0], c.child[0], m)
        return pa.Array.from_buffers(t, n, [vb, _buf(c.offsets)], children=[child])
    if f.type_id == STRUCT:
        kids = [column_to_array(fc, cc, n) for fc, cc in zip(f.children, c.child)]
        return pa.Array.from_buffers(t, n, [vb], children=kids)
    if f.type_id == MAP:
        m = int(np.asarray(c.offsets)[n])
        k = column_to_array(f.children[0], c.child[0], m)
        v = column_to_array(f.children[1], c.child[1], m)
        offs = pa.Array.from_buffers(pa.int32(), n + 1, [None, _buf(c.offsets)])
        mask = None
        if c.validity is not None:
            valid = np.unpackbits(np.asarray(c.validity).view(np.uint8), bitorder="little")[:n]
            mask = pa.array(valid == 0)
        return pa.MapArray.from_arrays(offs, k, v, type=t, mask=mask)
    return pa.Array.from_buffers(t, n, [vb, _buf(c.values)])


def columns_to_record_batch(fields: Sequence[Field], cols: List[Column], n: int):
    arrays = [column_to_array(f, c, n) for f, c in zip(fields, cols)]
    schema = pa.schema([pa.field(f.name, pa_type(f), f.nullable) for f in fields])
    return pa.RecordBatch.from_arrays(arrays, schema=schema)
