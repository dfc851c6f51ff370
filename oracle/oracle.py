"""TEST INFRASTRUCTURE ONLY — ctypes front end of the C restatement in ``row_oracle.c``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.  It is the parity checker for the HIP path, never part of the product: the
``fury_amd`` package does not import it and fails loudly when its HIP library is missing.

Semantics restated (file:line in the reference, FMT = java/fury-format/.../format):
  * encode  = RowEncoder.toRow per row (FMT/encoder/Encoders.java:88-93), rows concatenated;
              ``reuse=True`` restates RowEncoder.encode(obj)'s reused buffer (Encoders.java:191-198)
  * decode  = generated fromRow (FMT/encoder/RowEncoderBuilder.java:185-217) into Arrow columns
  * hash    = DataTypes.computeSchemaHash (FMT/type/DataTypes.java:499-544)
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FURY_ORACLE_LIB: the sanitizer build (tools/sanitize, tests/test_sanitize.py)
LIB_PATH = os.environ.get("FURY_ORACLE_LIB") or os.path.join(HERE, "liborow_oracle.so")

# fury_type_id (include/fury_row.h) = ArrowType ids (FMT/type/ArrowType.java:25-148)
BOOL, INT8, INT16, INT32, INT64 = 1, 3, 5, 7, 9
FLOAT32, FLOAT64, STRING, BINARY = 11, 12, 13, 14
DATE32, TIMESTAMP, DECIMAL, LIST, STRUCT, MAP = 16, 18, 23, 25, 26, 30

WIDTH = {BOOL: 1, INT8: 1, INT16: 2, INT32: 4, INT64: 8, FLOAT32: 4, FLOAT64: 8, DATE32: 4,
         TIMESTAMP: 8}
NP_DTYPE = {INT8: np.int8, INT16: np.int16, INT32: np.int32, INT64: np.int64,
            FLOAT32: np.float32, FLOAT64: np.float64, DATE32: np.int32, TIMESTAMP: np.int64}


@dataclass
class F:
    """A schema field (Arrow pojo Field as TypeInference builds it)."""
    name: str
    type_id: int
    nullable: bool = True
    children: Sequence["F"] = ()


@dataclass
class Col:
    """Arrow-style column: see ``fury_column`` in include/fury_row.h."""
    values: Optional[np.ndarray] = None
    validity: Optional[np.ndarray] = None
    offsets: Optional[np.ndarray] = None
    child: Optional[List["Col"]] = None


class _CField(ctypes.Structure):
    pass


_CField._fields_ = [("name", ctypes.c_char_p), ("type_id", ctypes.c_int32),
                    ("nullable", ctypes.c_int32), ("num_children", ctypes.c_int32),
                    ("children", ctypes.POINTER(_CField))]


class _CColumn(ctypes.Structure):
    pass


_CColumn._fields_ = [("values", ctypes.c_void_p), ("validity", ctypes.c_void_p),
                     ("offsets", ctypes.c_void_p), ("capacity", ctypes.c_int64),
                     ("child", ctypes.POINTER(_CColumn))]

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.fo_schema_hash.restype = ctypes.c_int64
        L.fo_schema_hash.argtypes = [ctypes.POINTER(_CField), ctypes.c_int32]
        L.fo_encode_batch.restype = ctypes.c_int64
        L.fo_encode_batch.argtypes = [ctypes.POINTER(_CField), ctypes.c_int32,
                                      ctypes.POINTER(_CColumn), ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
        L.fo_decode_batch.restype = ctypes.c_int
        L.fo_decode_batch.argtypes = [ctypes.POINTER(_CField), ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_CColumn)]
        L.fo_decode_batch_cur.restype = ctypes.c_int
        L.fo_decode_batch_cur.argtypes = [ctypes.POINTER(_CField), ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.POINTER(_CColumn), ctypes.c_void_p]
        L.fo_encode_fixed_inplace.restype = ctypes.c_int64
        L.fo_encode_fixed_inplace.argtypes = [ctypes.POINTER(_CField), ctypes.c_int32,
                                              ctypes.POINTER(_CColumn), ctypes.c_int64,
                                              ctypes.c_void_p]
        L.fo_type_width.restype = ctypes.c_int32
        L.fo_last_flags.restype = ctypes.c_int32
        L.fo_count_walk.restype = ctypes.c_int32
        L.fo_count_walk.argtypes = [ctypes.POINTER(_CField), ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int64]
        _lib = L
    return _lib


def _c_fields(fields: Sequence[F], keep: list):
    arr = (_CField * max(len(fields), 1))()
    for i, f in enumerate(fields):
        name = f.name.encode()
        keep.append(name)
        arr[i].name = name
        arr[i].type_id = f.type_id
        arr[i].nullable = int(f.nullable)
        arr[i].num_children = len(f.children)
        if f.children:
            ch = _c_fields(f.children, keep)
            arr[i].children = ch
        else:
            arr[i].children = None
    keep.append(arr)
    return arr


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def _c_columns(cols: Sequence[Col], keep: list):
    arr = (_CColumn * max(len(cols), 1))()
    for i, c in enumerate(cols):
        arr[i].values = _ptr(c.values)
        arr[i].validity = _ptr(c.validity)
        arr[i].offsets = _ptr(c.offsets)
        arr[i].capacity = 0 if c.values is None else c.values.nbytes
        if c.child:
            arr[i].child = _c_columns(c.child, keep)
        else:
            arr[i].child = None
    keep.append(arr)
    return arr


def schema_hash(fields: Sequence[F]) -> int:
    keep: list = []
    return int(lib().fo_schema_hash(_c_fields(fields, keep), len(fields)))


def bitmap_bytes(n: int) -> int:
    return ((n + 63) // 64) * 8


def fixed_size(fields: Sequence[F]) -> int:
    return bitmap_bytes(len(fields)) + 8 * len(fields)


def encode(fields: Sequence[F], cols: Sequence[Col], nrows: int, reuse: bool = False):
    """Returns (rows uint8[total], row_offsets int64[nrows+1])."""
    keep: list = []
    cf = _c_fields(fields, keep)
    cc = _c_columns(cols, keep)
    offs = np.zeros(nrows + 1, np.int64)
    total = lib().fo_encode_batch(cf, len(fields), cc, nrows, None, 0, offs.ctypes.data,
                                  int(reuse))
    if total < 0:
        raise RuntimeError(f"oracle encode failed with status {-total}")
    out = np.zeros(max(total, 1), np.uint8)
    total2 = lib().fo_encode_batch(cf, len(fields), cc, nrows, out.ctypes.data, out.nbytes,
                                   offs.ctypes.data, int(reuse))
    assert total2 == total
    return out[:total], offs


def encode_fixed_inplace(fields: Sequence[F], cols: Sequence[Col], nrows: int,
                         out: np.ndarray) -> int:
    keep: list = []
    return int(lib().fo_encode_fixed_inplace(_c_fields(fields, keep), len(fields),
                                             _c_columns(cols, keep), nrows, out.ctypes.data))


def _alloc_out(f: F, n: int, rows_bytes: int, with_validity: bool) -> Col:
    """Output column sized by upper bounds (element counts are bounded by row bytes)."""
    vb = np.zeros((n + 7) // 8 + 1, np.uint8) if with_validity else None
    t = f.type_id
    if t == BOOL:
        return Col(values=np.zeros((n + 7) // 8 + 1, np.uint8), validity=vb)
    if t in WIDTH:
        return Col(values=np.zeros(n * WIDTH[t] + 8, np.uint8), validity=vb)
    if t in (STRING, BINARY):
        return Col(values=np.zeros(rows_bytes + 8, np.uint8), validity=vb,
                   offsets=np.zeros(n + 1, np.int32))
    if t == DECIMAL:
        return Col(values=np.zeros(n * 16 + 8, np.uint8), validity=vb)
    if t == LIST:
        m = rows_bytes + 1
        return Col(validity=vb, offsets=np.zeros(n + 1, np.int32),
                   child=[_alloc_out(f.children[0], m, rows_bytes, with_validity)])
    if t == STRUCT:
        return Col(validity=vb, child=[_alloc_out(c, n, rows_bytes, with_validity)
                                       for c in f.children])
    if t == MAP:
        m = rows_bytes + 1
        return Col(validity=vb, offsets=np.zeros(n + 1, np.int32),
                   child=[_alloc_out(c, m, rows_bytes, with_validity) for c in f.children])
    raise ValueError(f"unsupported type {t}")


def _trim(f: F, c: Col, n: int) -> Col:
    t = f.type_id
    vb = None if c.validity is None else c.validity[:(n + 7) // 8]
    if t == BOOL:
        return Col(values=c.values[:(n + 7) // 8], validity=vb)
    if t in WIDTH:
        return Col(values=c.values[:n * WIDTH[t]].view(NP_DTYPE[t]), validity=vb)
    if t in (STRING, BINARY):
        return Col(values=c.values[:int(c.offsets[n])], validity=vb, offsets=c.offsets)
    if t == DECIMAL:
        return Col(values=c.values[:n * 16], validity=vb)
    if t == LIST:
        return Col(validity=vb, offsets=c.offsets,
                   child=[_trim(f.children[0], c.child[0], int(c.offsets[n]))])
    if t == STRUCT:
        return Col(validity=vb, child=[_trim(fc, cc, n) for fc, cc in zip(f.children, c.child)])
    if t == MAP:
        m = int(c.offsets[n])
        return Col(validity=vb, offsets=c.offsets,
                   child=[_trim(fc, cc, m) for fc, cc in zip(f.children, c.child)])
    raise ValueError(t)


def _shape_only(f: F) -> Col:
    """A column tree with every buffer None (the sizing pass writes nothing)."""
    return Col(child=[_shape_only(c) for c in f.children] if f.children else None)


def _nodes_dfs(fields: Sequence[F]):
    out = []

    def walk(f):
        out.append(f)
        for c in f.children:
            walk(c)
    for f in fields:
        walk(f)
    return out


def _alloc_exact(f: F, n: int, cur: np.ndarray, node: int, with_validity: bool):
    """Output column of node `node` (depth-first id) with n entries, sized from the sizing pass's
    cursors; returns (column, next node id)."""
    vb = np.zeros((n + 7) // 8 + 1, np.uint8) if with_validity else None
    t = f.type_id
    if t == BOOL:
        return Col(values=np.zeros((n + 7) // 8 + 1, np.uint8), validity=vb), node + 1
    if t in WIDTH:
        return Col(values=np.zeros(n * WIDTH[t] + 8, np.uint8), validity=vb), node + 1
    if t in (STRING, BINARY):
        return Col(values=np.zeros(int(cur[node]) + 8, np.uint8), validity=vb,
                   offsets=np.zeros(n + 1, np.int32)), node + 1
    if t == DECIMAL:
        return Col(values=np.zeros(n * 16 + 8, np.uint8), validity=vb), node + 1
    m = n if t == STRUCT else int(cur[node])
    kids, nxt = [], node + 1
    for c in f.children:
        k, nxt = _alloc_exact(c, m, cur, nxt, with_validity)
        kids.append(k)
    if t == STRUCT:
        return Col(validity=vb, child=kids), nxt
    if t in (LIST, MAP):
        return Col(validity=vb, offsets=np.zeros(n + 1, np.int32), child=kids), nxt
    raise ValueError(f"unsupported type {t}")


def decode(fields: Sequence[F], rows: np.ndarray, row_offsets: Optional[np.ndarray], nrows: int,
           with_validity: bool = True, sizing: str = "exact") -> List[Col]:
    """Two passes, as fo_decode_batch prescribes: a sizing pass (nothing written) whose cursors
    give every node's exact payload / child-entry count -- slots may share bytes of the batch, so
    no bound from the row bytes holds -- then the decode into buffers of those sizes.
    sizing="bound" (the CPU baseline, rows written by an encoder: every value inside its own row)
    skips the sizing pass and sizes outputs by the row bytes, as the reference's fromRow has no
    sizing pass either."""
    keep: list = []
    cf = _c_fields(fields, keep)
    if sizing == "bound":
        outs = [_alloc_out(f, nrows, int(rows.nbytes), with_validity) for f in fields]
        st = lib().fo_decode_batch(cf, len(fields), _ptr(rows), _ptr(row_offsets), nrows,
                                   _c_columns(outs, keep))
        if st != 0:
            raise RuntimeError(f"oracle decode failed with status {st}")
        return [_trim(f, c, nrows) for f, c in zip(fields, outs)]
    cur = np.zeros(len(_nodes_dfs(fields)) + 1, np.int64)
    st = lib().fo_decode_batch_cur(cf, len(fields), _ptr(rows), _ptr(row_offsets), nrows,
                                   _c_columns([_shape_only(f) for f in fields], keep),
                                   cur.ctypes.data)
    if st != 0:
        raise RuntimeError(f"oracle decode failed with status {st}")
    outs, node = [], 0
    for f in fields:
        c, node = _alloc_exact(f, nrows, cur, node, with_validity)
        outs.append(c)
    st = lib().fo_decode_batch(cf, len(fields), _ptr(rows),
                               _ptr(row_offsets), nrows, _c_columns(outs, keep))
    if st != 0:
        raise RuntimeError(f"oracle decode failed with status {st}")
    return [_trim(f, c, nrows) for f, c in zip(fields, outs)]


# Decode errors (row_oracle.c FO_ERR_*): the reference's exception each stands for
ERR_OOB, ERR_MAP, ERR_BUDGET = 1, 2, 4


def decode_checked(fields: Sequence[F], rows: np.ndarray, row_offsets: Optional[np.ndarray],
                   nrows: int, with_validity: bool = True):
    """The decode with the reference's bounds rule (row_oracle.c header: MemoryBuffer.checkPosition
    / get / slice / copyToUnsafe restated per container): returns (flags, columns) -- flags the
    ERR_* bits found (ERR_OOB = IndexOutOfBoundsException, ERR_MAP = BinaryMap.pointTo's
    UnsupportedOperationException); columns None when any was found (the reference throws).  The
    batch must not alias itself beyond what count_walk_flags admits (nested schemas: call that
    first; it bounds the walk)."""
    keep: list = []
    cf = _c_fields(fields, keep)
    cur = np.zeros(len(_nodes_dfs(fields)) + 1, np.int64)
    lib().fo_decode_batch_cur(cf, len(fields), _ptr(rows), _ptr(row_offsets), nrows,
                              _c_columns([_shape_only(f) for f in fields], keep), cur.ctypes.data)
    flags = int(lib().fo_last_flags())
    if flags:
        return flags, None
    return 0, decode(fields, rows, row_offsets, nrows, with_validity)


def count_walk_flags(fields: Sequence[F], rows: np.ndarray, row_offsets: np.ndarray,
                     nrows: int) -> int:
    """ERR_* bits of the device row walk's COUNT pass (fury_decode_prepare), restated in
    row_oracle.c fo_count_walk: the container checks over the nodes that hold or contain a
    counted slot, and the item budget per top-level field of a row (ERR_BUDGET: a device limit)."""
    keep: list = []
    if nrows == 0:
        return 0
    offs = np.ascontiguousarray(row_offsets, np.int64)
    return int(lib().fo_count_walk(_c_fields(fields, keep), len(fields), _ptr(rows), _ptr(offs),
                                   nrows))
