"""Host-side mirror of ``org.apache.fury.format.encoder.Encoders`` / ``RowEncoder`` over the
device C ABI.

Reference surface (FMT = java/fury-format/src/main/java/org/apache/fury/format):
  Encoders.bean(beanClass) -> RowEncoder<T>     FMT/encoder/Encoders.java:60-219
  RowEncoder.schema / toRow / fromRow / encode / decode   FMT/encoder/RowEncoder.java:26-32,
                                                          FMT/encoder/Encoder.java:31-40
  ArrowWriter.write(row) / finishAsRecordBatch  FMT/vectorized/ArrowWriter.java:74-99

A Java bean cannot cross onto the GPU, so the batch methods take/return Arrow-style columns
(``workloads.Column`` of torch tensors on the device) and ``RowBatch`` objects holding packed
rows in HBM.  The single-object methods (to_row / from_row / encode / decode) accept a bean as
a ``dict`` and run through the same device kernels as a batch of one.

Errors raise the Python counterparts of the reference's exceptions (see ``errors``).
"""
from __future__ import annotations

import contextlib
import ctypes
import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .types import (BINARY, BOOL, DECIMAL, FLOAT32, FLOAT64, LIST, MAP, STRING, STRUCT, Field,
                    type_width)
from .workloads import Column

# ---------------------------------------------------------------------------------------------
# Errors (status codes of include/fury_row.h fury_status)
# ---------------------------------------------------------------------------------------------


class FuryError(Exception):
    status = -1


class IllegalArgumentException(FuryError, ValueError):
    status = 1


class UnsupportedOperationException(FuryError, NotImplementedError):
    status = 2


class ClassNotCompatibleException(FuryError):
    """Schema hash mismatch on decode (Encoders.java:170-178)."""
    status = 3


class IndexOutOfBoundsException(FuryError, IndexError):
    status = 4


class EncoderException(FuryError):
    status = 5


class FuryDeviceError(FuryError, RuntimeError):
    status = 6


class CapacityError(FuryError):
    status = 7


_ERRORS = {c.status: c for c in (IllegalArgumentException, UnsupportedOperationException,
                                 ClassNotCompatibleException, IndexOutOfBoundsException,
                                 EncoderException, FuryDeviceError, CapacityError)}


def _check(status: int):
    if status != 0:
        raise _ERRORS.get(status, FuryError)(N.last_error())


# ---------------------------------------------------------------------------------------------
# Schema
# ---------------------------------------------------------------------------------------------
def _c_fields(fields: Sequence[Field], keep: list):
    arr = (N.FuryField * max(len(fields), 1))()
    for i, f in enumerate(fields):
        nm = f.name.encode("utf-8")
        keep.append(nm)
        arr[i].name = nm
        arr[i].type_id = f.type_id
        arr[i].nullable = int(bool(f.nullable))
        arr[i].num_children = len(f.children)
        arr[i].children = _c_fields(f.children, keep) if f.children else None
    keep.append(arr)
    return arr


class Schema:
    """A schema handle (``fury_schema``): layout + ``DataTypes.computeSchemaHash``.
    ``collection=True``: the schema of an ArrayEncoder / MapEncoder (one LIST or MAP field whose
    batch entries are top-level BinaryArrays / BinaryMaps, ``fury_collection_schema_create``)."""

    def __init__(self, fields: Sequence[Field], collection: bool = False):
        self.fields: List[Field] = list(fields)
        self.collection = collection
        keep: list = []
        h = ctypes.c_void_p()
        if collection:
            if len(self.fields) != 1:
                raise IllegalArgumentException("a collection schema has exactly one field")
            _check(N.lib().fury_collection_schema_create(_c_fields(self.fields, keep),
                                                         ctypes.byref(h)))
        else:
            _check(N.lib().fury_schema_create(_c_fields(self.fields, keep), len(self.fields),
                                              ctypes.byref(h)))
        self._h = h
        info = N.FurySchemaInfo()
        _check(N.lib().fury_schema_get_info(h, ctypes.byref(info)))
        self.num_fields = info.num_fields
        self.bitmap_bytes = info.bitmap_bytes
        self.fixed_size = info.fixed_size
        self.is_fixed = bool(info.is_fixed)
        self.schema_hash = int(info.schema_hash)

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.lib().fury_schema_destroy(h)
            except Exception:
                pass
            self._h = None

    def __repr__(self):
        return f"Schema({self.fields}, hash={self.schema_hash})"


# ---------------------------------------------------------------------------------------------
# Device columns <-> C structs
# ---------------------------------------------------------------------------------------------
def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        raise IllegalArgumentException("device columns must be torch tensors")
    if t.device.type != "cuda":
        raise IllegalArgumentException(f"tensor on {t.device}, expected a GPU tensor")
    if not t.is_contiguous():
        raise IllegalArgumentException("tensor must be contiguous")
    return t.data_ptr()


def _c_columns(cols: Sequence[Column], keep: list):
    arr = (N.FuryColumn * max(len(cols), 1))()
    for i, c in enumerate(cols):
        arr[i].values = _ptr(c.values)
        arr[i].validity = _ptr(c.validity)
        arr[i].offsets = _ptr(c.offsets)
        arr[i].capacity = 0 if c.values is None else c.values.numel() * c.values.element_size()
        arr[i].child = _c_columns(c.child, keep) if c.child else None
    keep.append(arr)
    return arr


def _hptr(a) -> Optional[int]:
    """Address of a HOST buffer: a contiguous numpy array or CPU tensor (e.g. pinned)."""
    if a is None:
        return None
    if isinstance(a, torch.Tensor):
        if a.device.type != "cpu" or not a.is_contiguous():
            raise IllegalArgumentException("host buffers must be contiguous CPU tensors")
        return a.data_ptr()
    a = np.asarray(a)
    if not a.flags["C_CONTIGUOUS"]:
        raise IllegalArgumentException("host buffers must be contiguous")
    return a.ctypes.data


def _nbytes(a) -> int:
    if a is None:
        return 0
    if isinstance(a, torch.Tensor):
        return a.numel() * a.element_size()
    return np.asarray(a).nbytes


def _c_host_columns(cols: Sequence[Column], keep: list):
    arr = (N.FuryColumn * max(len(cols), 1))()
    for i, c in enumerate(cols):
        for a in (c.values, c.validity, c.offsets):
            if a is not None:
                keep.append(a)
        arr[i].values = _hptr(c.values)
        arr[i].validity = _hptr(c.validity)
        arr[i].offsets = _hptr(c.offsets)
        arr[i].capacity = _nbytes(c.values)
        arr[i].child = _c_host_columns(c.child, keep) if c.child else None
    keep.append(arr)
    return arr


class _PinnedBlock:
    """hipHostMalloc'd host memory (fury_host_alloc), freed when the last array over it goes."""

    def __init__(self, nbytes: int):
        self._ptr = ctypes.c_void_p()
        _check(N.lib().fury_host_alloc(max(nbytes, 1), ctypes.byref(self._ptr)))
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "version": 3,
                                    "data": (self._ptr.value, False)}

    def __del__(self):
        if self._ptr.value:
            try:
                N.lib().fury_host_free(self._ptr)
            except TypeError:           # interpreter shutdown: the module is already torn down
                pass
            self._ptr = ctypes.c_void_p()


def host_empty(nbytes: int, dtype=np.uint8) -> np.ndarray:
    """A pinned host buffer for the host-memory batch path (include/fury_row.h fury_host_alloc):
    the GPU reaches it directly, so fixed-width encode_host / decode_host run without staging
    (GpuRowEncoder.allocatePinned is the JVM's equivalent)."""
    return np.asarray(_PinnedBlock(nbytes)).view(dtype)


def _tree_bytes(cols: Sequence[Column]) -> int:
    return sum(_nbytes(c.values) + _nbytes(c.validity) + _nbytes(c.offsets) +
               (_tree_bytes(c.child) if c.child else 0) for c in cols)


def _stream_handle(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _on(stream: Optional[torch.cuda.Stream]):
    """Makes ``stream`` torch's current stream for the body: output allocations belong to it (the
    caching allocator does not hand them to other streams while the kernels run) and host reads
    (``.item()``, ``.cpu()``) wait for the kernels launched on it."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def column_to_device(c: Column, device) -> Column:
    def t(a):
        if a is None:
            return None
        if isinstance(a, torch.Tensor):
            return a.to(device)
        return torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return Column(values=t(c.values), validity=t(c.validity), offsets=t(c.offsets),
                  child=[column_to_device(x, device) for x in c.child] if c.child else None)


def column_to_host(c: Column) -> Column:
    def h(a):
        if a is None:
            return None
        return a.detach().cpu().numpy()
    return Column(values=h(c.values), validity=h(c.validity), offsets=h(c.offsets),
                  child=[column_to_host(x) for x in c.child] if c.child else None)


@dataclass
class RowBatch:
    """Packed rows in device memory: row i = rows[row_offsets[i]:row_offsets[i+1]] (or
    i * fixed_size for fixed-width schemas, where row_offsets is None)."""
    rows: torch.Tensor
    row_offsets: Optional[torch.Tensor]
    nrows: int
    schema_hash: int

    def row_bytes(self, i: int, fixed_size: int) -> bytes:
        if self.row_offsets is None:
            b, e = i * fixed_size, (i + 1) * fixed_size
        else:
            b, e = int(self.row_offsets[i]), int(self.row_offsets[i + 1])
        return bytes(self.rows[b:e].cpu().numpy())


# ---------------------------------------------------------------------------------------------
# RowEncoder
# ---------------------------------------------------------------------------------------------
class RowEncoder:
    """``RowEncoder<T>`` with batch methods; not thread-safe per instance (like the reference,
    Encoders.java:74,146)."""

    def __init__(self, fields: Sequence[Field], device=None):
        self._schema = Schema(fields)
        self.device = torch.device(device if device is not None else "cuda")

    # -- RowEncoder API ------------------------------------------------------------------
    def schema(self) -> Schema:
        return self._schema

    @property
    def schema_hash(self) -> int:
        return self._schema.schema_hash

    # -- batch API -----------------------------------------------------------------------
    def measure(self, columns: Sequence[Column], nrows: int, stream=None) -> Optional[torch.Tensor]:
        """Row offsets (int64[nrows+1], device) for variable-length schemas; None if fixed."""
        if self._schema.is_fixed:
            return None
        with _on(stream):
            offs = torch.empty(nrows + 1, dtype=torch.int64, device=self.device)
        keep: list = []
        _check(N.lib().fury_row_measure(self._schema.handle, _c_columns(columns, keep), nrows,
                                        offs.data_ptr(), _stream_handle(stream)))
        return offs

    def measure_into(self, columns: Sequence[Column], nrows: int, offs: torch.Tensor,
                     stream=None) -> None:
        keep: list = []
        _check(N.lib().fury_row_measure(self._schema.handle, _c_columns(columns, keep), nrows,
                                        _ptr(offs), _stream_handle(stream)))

    def encode_into(self, columns: Sequence[Column], nrows: int, rows: torch.Tensor,
                    row_offsets: Optional[torch.Tensor], stream=None) -> None:
        keep: list = []
        _check(N.lib().fury_row_encode(self._schema.handle, _c_columns(columns, keep), nrows,
                                       _ptr(row_offsets), _ptr(rows), _stream_handle(stream)))

    def encode_measured_into(self, columns: Sequence[Column], nrows: int, rows: torch.Tensor,
                             row_offsets: Optional[torch.Tensor], stream=None) -> None:
        """Measure + encode in one call (no host sync) into a reused buffer (``rows`` capacity =
        its size): writes ``row_offsets``; when ``row_offsets[nrows]`` exceeds the capacity the
        rows did not fit (nothing past the capacity is written) — grow and call again."""
        keep: list = []
        _check(N.lib().fury_row_encode_measured(
            self._schema.handle, _c_columns(columns, keep), nrows, _ptr(row_offsets), _ptr(rows),
            rows.numel() * rows.element_size(), _stream_handle(stream)))

    # -- bound calls: the argument block built once, for hot loops --------------------------
    def bind_encode(self, columns: Sequence[Column], nrows: int, rows: torch.Tensor,
                    row_offsets: Optional[torch.Tensor] = None, stream=None,
                    measured: bool = False):
        """``encode_into`` (``measured``: ``encode_measured_into``) with the column descriptors
        and pointers resolved once; the returned callable re-issues the same call.  Building the
        descriptors of 100 columns costs ~0.3 ms of Python per call -- more than the Struct-100
        kernel -- so a loop that re-encodes the same buffers should bind.  The buffers must stay
        alive and unmoved while the callable is used."""
        keep: list = []
        cc = _c_columns(columns, keep)
        L = N.lib()
        if measured:
            args = (self._schema.handle, cc, nrows, _ptr(row_offsets), _ptr(rows),
                    rows.numel() * rows.element_size(), _stream_handle(stream))
            fn = L.fury_row_encode_measured
        else:
            args = (self._schema.handle, cc, nrows, _ptr(row_offsets), _ptr(rows),
                    _stream_handle(stream))
            fn = L.fury_row_encode

        def call():
            _check(fn(*args))
        # the schema handle in args lives as long as the Schema object: keep it (and this
        # encoder) alive with the callable, or a dropped encoder would free it under the call
        call.keep = (keep, columns, rows, row_offsets, self, self._schema)
        return call

    def bind_decode(self, batch: RowBatch, cols: List[Column], stream=None, arrow: bool = False):
        """``decode_into`` bound like ``bind_encode``."""
        keep: list = []
        cc = _c_columns(cols, keep)
        fn = N.lib().fury_rows_to_arrow if arrow else N.lib().fury_row_decode
        args = (self._schema.handle, _ptr(batch.rows), _ptr(batch.row_offsets), batch.nrows, cc,
                _stream_handle(stream))

        def call():
            _check(fn(*args))
        call.keep = (keep, batch, cols, self, self._schema)
        return call

    def encode_batch(self, columns: Sequence[Column], nrows: int, stream=None) -> RowBatch:
        offs = self.measure(columns, nrows, stream)
        with _on(stream):
            if offs is None:
                total = nrows * self._schema.fixed_size
            else:
                total = int(offs[nrows].item())
            rows = torch.empty(max(total, 16), dtype=torch.uint8, device=self.device)
        self.encode_into(columns, nrows, rows, offs, stream)
        return RowBatch(rows[:total] if total else rows[:0], offs, nrows, self.schema_hash)

    def alloc_columns(self, nrows: int, validity: bool = True) -> List[Column]:
        """Output columns for fixed-width fields (variable ones are sized by decode_measure).
        Validity and BOOL bitmaps are whole 32-bit words (the kernels store / OR them as words,
        include/fury_row.h: 4-byte aligned, padded to a multiple of 4 bytes)."""
        out = []
        words = ((nrows + 31) // 32) * 4
        for f in self._schema.fields:
            vb = (torch.empty(words, dtype=torch.uint8, device=self.device)
                  if validity else None)
            if f.type_id == BOOL:
                out.append(Column(values=torch.empty(words, dtype=torch.uint8,
                                                     device=self.device), validity=vb))
            elif type_width(f.type_id) > 0:
                out.append(Column(values=torch.empty(nrows * type_width(f.type_id),
                                                     dtype=torch.uint8, device=self.device),
                                  validity=vb))
            elif f.type_id == DECIMAL:
                out.append(Column(values=torch.empty(nrows * 16, dtype=torch.uint8,
                                                     device=self.device), validity=vb))
            elif f.type_id in (STRING, BINARY):
                out.append(Column(offsets=torch.empty(nrows + 1, dtype=torch.int32,
                                                      device=self.device), validity=vb))
            elif f.type_id == LIST:
                out.append(Column(offsets=torch.empty(nrows + 1, dtype=torch.int32,
                                                      device=self.device), validity=vb,
                                  child=[Column()]))
            else:
                raise UnsupportedOperationException(f"no device decode for {f}")
        return out

    @property
    def nested(self) -> bool:
        """True when the schema has STRUCT / MAP / LIST-of-variable-length fields, or more than
        256 fields of which some are variable-length (decoded by the two-step plan API: the generic
        engine); always for collection schemas."""
        if getattr(self._schema, "collection", False):
            return True
        if len(self._schema.fields) > 256 and not self._schema.is_fixed:
            return True
        def deep(f: Field) -> bool:
            if f.type_id in (STRUCT, MAP):
                return True
            if f.type_id == LIST:
                e = f.children[0]
                return type_width(e.type_id) < 0 or deep(e)
            return False
        return any(deep(f) for f in self._schema.fields)

    def _decode_nested(self, batch: RowBatch, validity: bool, arrow: bool,
                       stream=None) -> List[Column]:
        L = N.lib()
        h = self._schema.handle
        nn = L.fury_schema_num_nodes(h)
        entries = (ctypes.c_int64 * max(nn, 1))()
        nbytes = (ctypes.c_int64 * max(nn, 1))()
        plan = ctypes.c_void_p()
        sh = _stream_handle(stream)
        _check(L.fury_decode_prepare(h, _ptr(batch.rows), _ptr(batch.row_offsets), batch.nrows,
                                     entries, nbytes, ctypes.byref(plan), sh))
        try:
            order = _bfs(self._schema.fields)
            cols: List[Column] = []
            with _on(stream):
                cols = _alloc_nodes(order, entries, nbytes, validity or arrow, self.device)
            for i, (f, first) in enumerate(order):
                if f.children:
                    cols[i].child = [cols[first + j] for j in range(len(f.children))]
            top = cols[:len(self._schema.fields)]
            keep: list = []
            _check(L.fury_decode_execute(plan, _c_columns(top, keep), int(arrow), sh))
        finally:
            L.fury_decode_plan_destroy(plan)
        return top

    def _decode_bound(self, batch: RowBatch, validity: bool, arrow: bool,
                      stream=None) -> List[Column]:
        """Variable-length outputs sized from a bound the rows give (a column's payload bytes and
        list elements <= the batch's row bytes: every byte of them is inside some row), decoded
        in one pass, then trimmed to the real sizes after ONE host read of every column's
        offsets[n] -- no fury_row_decode_measure pass over the rows.  Rows that break the bound
        (a slot pointing outside its row) fall back to the exact-size ("measure") decode."""
        n = batch.nrows
        bound = int(batch.rows.numel() * batch.rows.element_size())
        with _on(stream):
            cols = self.alloc_columns(n, validity)
            for f, c in zip(self._schema.fields, cols):
                if f.type_id in (STRING, BINARY):
                    c.values = torch.empty(max(bound, 1), dtype=torch.uint8, device=self.device)
                elif f.type_id == LIST:
                    e = f.children[0]
                    nbytes = (bound + 7) // 8 if e.type_id == BOOL else bound
                    c.child = [Column(
                        values=torch.empty(nbytes + 8, dtype=torch.uint8, device=self.device),
                        validity=(torch.zeros((bound + 7) // 8 + 4, dtype=torch.uint8,
                                              device=self.device) if validity else None))]
        self.decode_into(batch, cols, stream, arrow)
        var = [(f, c) for f, c in zip(self._schema.fields, cols)
               if f.type_id in (STRING, BINARY, LIST)]
        if not var or n == 0:
            return cols
        with _on(stream):
            totals = torch.stack([c.offsets[n] for _, c in var]).cpu().tolist()
        for (f, c), total in zip(var, totals):
            if f.type_id == LIST:
                e = f.children[0]
                ch = c.child[0]
                nbytes = (total + 7) // 8 if e.type_id == BOOL else total * type_width(e.type_id)
                have = ch.values.numel() - 8
                if total < 0 or nbytes > have:
                    return self._decode(batch, validity, arrow, stream, None, "measure")
                ch.values = ch.values[:nbytes + 8]
                if ch.validity is not None:
                    ch.validity = ch.validity[:(total + 7) // 8 + 4]
            else:
                if total < 0 or total > c.values.numel():
                    return self._decode(batch, validity, arrow, stream, None, "measure")
                c.values = c.values[:max(total, 1)]
        return cols

    def _decode(self, batch: RowBatch, validity: bool, arrow: bool, stream=None,
                out: Optional[List[Column]] = None, sizing: str = "measure") -> List[Column]:
        if self.nested:
            return self._decode_nested(batch, validity, arrow, stream)
        if sizing not in ("measure", "bound"):
            raise ValueError(f"sizing must be 'measure' or 'bound', not {sizing!r}")
        if sizing == "measure" and out is None and self._wide_plan():
            # 17-256 fields: the plan API keeps the count pass's tile bases for the write pass
            # (fury_decode_prepare sizes, fury_decode_execute writes; the rows are counted once)
            return self._decode_nested(batch, validity, arrow, stream)
        if sizing == "bound" and out is None and not self._schema.is_fixed:
            return self._decode_bound(batch, validity, arrow, stream)
        n = batch.nrows
        if out is not None:
            cols = out
        else:
            with _on(stream):
                cols = self.alloc_columns(n, validity)
        keep: list = []
        sh = _stream_handle(stream)
        if not self._schema.is_fixed:
            _check(N.lib().fury_row_decode_measure(self._schema.handle, _ptr(batch.rows),
                                                   _ptr(batch.row_offsets), n,
                                                   _c_columns(cols, keep), sh))
            self._size_var_outputs(cols, n, validity, stream)
            keep = []
        fn = N.lib().fury_rows_to_arrow if arrow else N.lib().fury_row_decode
        _check(fn(self._schema.handle, _ptr(batch.rows), _ptr(batch.row_offsets), n,
                  _c_columns(cols, keep), sh))
        return cols

    def _wide_plan(self) -> bool:
        """Flat variable-length schemas the wide kernels decode (17-256 fields, tuning var_wide)."""
        nf = len(self._schema.fields)
        return (not self._schema.is_fixed and 16 < nf <= 256
                and N.lib().fury_get_tuning(b"var_wide") == 1)

    def _size_var_outputs(self, cols: List[Column], n: int, validity: bool, stream) -> None:
        """Allocates the payload / element buffers of the variable-length outputs from the
        offsets fury_row_decode_measure wrote (host read on ``stream``)."""
        with _on(stream):
            for f, c in zip(self._schema.fields, cols):
                if f.type_id in (STRING, BINARY):
                    total = int(c.offsets[n].item()) if n else 0
                    c.values = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
                elif f.type_id == LIST:
                    total = int(c.offsets[n].item()) if n else 0
                    e = f.children[0]
                    nbytes = (total + 7) // 8 if e.type_id == BOOL else total * type_width(e.type_id)
                    c.child = [Column(
                        values=torch.empty(nbytes + 8, dtype=torch.uint8, device=self.device),
                        validity=(torch.zeros((total + 7) // 8 + 4, dtype=torch.uint8,
                                              device=self.device) if validity else None))]

    def decode_into(self, batch: RowBatch, cols: List[Column], stream=None,
                    arrow: bool = False) -> None:
        """Decode into preallocated columns in one device pass (the kernel computes the Arrow
        offsets itself): no host synchronisation, so the call can be captured/timed back to
        back.  Payloads past a buffer's capacity are not written; ``offsets[nrows]`` always holds
        the size the column needs (see ``check_capacity``)."""
        keep: list = []
        sh = _stream_handle(stream)
        fn = N.lib().fury_rows_to_arrow if arrow else N.lib().fury_row_decode
        _check(fn(self._schema.handle, _ptr(batch.rows), _ptr(batch.row_offsets), batch.nrows,
                  _c_columns(cols, keep), sh))

    def check_capacity(self, cols: List[Column], nrows: int) -> None:
        """Raises CapacityError when a decode into preallocated ``cols`` needed more payload
        (STRING/BINARY bytes, LIST child elements) than the buffers hold (synchronises)."""
        self.device_status()
        if self._schema.is_fixed or self.nested or nrows == 0:
            return
        for f, c in zip(self._schema.fields, cols):
            if f.type_id not in (STRING, BINARY, LIST) or c.offsets is None:
                continue
            need = int(c.offsets[nrows].item())
            if f.type_id == LIST:
                e = f.children[0]
                v = c.child[0].values if c.child else None
                have = 0 if v is None else v.numel() * v.element_size()
                have = have * 8 if e.type_id == BOOL else have // type_width(e.type_id)
            else:
                have = 0 if c.values is None else c.values.numel() * c.values.element_size()
            if need > have:
                raise CapacityError(f"column {f.name}: decode needs {need}, buffer holds {have}")

    def decode_batch(self, batch: RowBatch, validity: bool = True, stream=None,
                     out: Optional[List[Column]] = None, sizing: str = "measure") -> List[Column]:
        """Rows -> columns (generated fromRow semantics).  Variable-length outputs are sized by
        ``sizing``: "measure" (default) runs fury_row_decode_measure first and allocates exactly;
        "bound" allocates each from the batch's row bytes (HBM for speed: no sizing pass over the
        rows) and trims after one host read.  Memory cost of "bound": the returned columns are
        views of those row-sized buffers, so while they live every STRING / BINARY / LIST output
        holds about the batch's row bytes of HBM (K variable-length columns: ~K x row bytes).
        ``stream``: every kernel, output allocation and host read of the call runs on it."""
        if batch.schema_hash != self.schema_hash:
            raise ClassNotCompatibleException(
                f"Schema is not consistent, encoder schema is {self._schema}. self/peer schema "
                f"hash are {self.schema_hash}/{batch.schema_hash}. Please check writer schema.")
        cols = self._decode(batch, validity, False, stream, out, sizing)
        self.device_status(stream)
        return cols

    def device_status(self, stream=None) -> None:
        """Synchronises ``stream`` and raises FuryDeviceError if an earlier asynchronous call's
        kernel could not produce a valid result (``fury_device_status``)."""
        _check(N.lib().fury_device_status(_stream_handle(stream)))

    # -- host-memory batch path: the JNI boundary (off-heap buffers in, off-heap buffers out) --
    def encode_host(self, columns: Sequence[Column], nrows: int, rows=None, row_offsets=None,
                    device_index: int = 0):
        """Host columns (numpy arrays or CPU/pinned tensors, fury_row.h layout) -> host rows,
        through HBM inside the call (``fury_row_encode_host``).  Returns (rows, row_offsets);
        row_offsets is None for fixed-width schemas unless a buffer was passed."""
        keep: list = []
        cc = _c_host_columns(columns, keep)
        fixed = self._schema.is_fixed
        if rows is None:
            bound = nrows * self._schema.fixed_size
            if not fixed:
                bound += 2 * _tree_bytes(columns) + 64 * nrows * (len(self._schema.fields) + 1)
            rows = np.empty(max(bound, 16), dtype=np.uint8)
        if row_offsets is None and not fixed:
            row_offsets = np.empty(nrows + 1, dtype=np.int64)
        nb = ctypes.c_int64(0)
        st = N.lib().fury_row_encode_host(self._schema.handle, cc, nrows, _hptr(rows),
                                          _nbytes(rows), _hptr(row_offsets), ctypes.byref(nb),
                                          device_index)
        if st == 7:                               # FURY_ERR_CAPACITY: retry at the exact size
            rows = np.empty(max(nb.value, 16), dtype=np.uint8)
            st = N.lib().fury_row_encode_host(self._schema.handle, cc, nrows, _hptr(rows),
                                              _nbytes(rows), _hptr(row_offsets),
                                              ctypes.byref(nb), device_index)
        _check(st)
        return rows[:nb.value], row_offsets

    def decode_host(self, rows, row_offsets, nrows: int, out: Optional[List[Column]] = None,
                    device_index: int = 0, pinned: bool = False) -> List[Column]:
        """Host rows -> host columns (``fury_row_decode_host``; nested schemas through the
        two-step host decode).  Without ``out``, numpy columns are allocated (pinned ones with
        ``pinned``, nested schemas): validity for nullable fields, and payload / element buffers
        bounded by the row bytes (a row holds every byte it decodes to)."""
        from .workloads import Column as C
        if self.nested and out is None:
            return self._decode_host_nested(rows, row_offsets, nrows, device_index, pinned)
        if out is None:
            out = []
            rb = max(_nbytes(rows), 16)
            for f in self._schema.fields:
                vb = np.zeros((nrows + 7) // 8 + 8, dtype=np.uint8) if f.nullable else None
                if f.type_id in (STRING, BINARY):
                    out.append(C(values=np.empty(rb, dtype=np.uint8), validity=vb,
                                 offsets=np.empty(nrows + 1, dtype=np.int32)))
                elif f.type_id == LIST:
                    e = f.children[0]
                    ev = np.zeros(rb // 8 + 8, dtype=np.uint8) if e.nullable else None
                    out.append(C(validity=vb, offsets=np.empty(nrows + 1, dtype=np.int32),
                                 child=[C(values=np.empty(rb, dtype=np.uint8), validity=ev)]))
                elif f.type_id == BOOL:
                    out.append(C(values=np.empty((nrows + 7) // 8 + 8, dtype=np.uint8),
                                 validity=vb))
                elif f.type_id == DECIMAL:
                    out.append(C(values=np.empty(nrows * 16, dtype=np.uint8), validity=vb))
                else:
                    out.append(C(values=np.empty(max(nrows * type_width(f.type_id), 8),
                                                 dtype=np.uint8), validity=vb))
        keep: list = []
        _check(N.lib().fury_row_decode_host(self._schema.handle, _hptr(rows), _hptr(row_offsets),
                                            nrows, _c_host_columns(out, keep), device_index))
        return out

    def _decode_host_nested(self, rows, row_offsets, nrows: int, device_index: int = 0,
                            pinned: bool = False):
        """Nested schemas through fury_decode_host_prepare / fury_decode_host_execute: node
        sizes first, then host buffers of exactly those sizes (pinned: written in place by the
        kernels), filled in one call."""
        L = N.lib()
        h = self._schema.handle
        nn = L.fury_schema_num_nodes(h)
        entries = (ctypes.c_int64 * max(nn, 1))()
        nbytes = (ctypes.c_int64 * max(nn, 1))()
        plan = ctypes.c_void_p()
        _check(L.fury_decode_host_prepare(h, _hptr(rows), _hptr(row_offsets), nrows, entries,
                                          nbytes, ctypes.byref(plan), device_index))
        try:
            order = _bfs(self._schema.fields)
            zeros = _pinned_zeros if pinned else np.zeros
            cols = [_alloc_host_node(f, int(entries[i]), int(nbytes[i]), zeros)
                    for i, (f, _) in enumerate(order)]
            for i, (f, first) in enumerate(order):
                if f.children:
                    cols[i].child = [cols[first + j] for j in range(len(f.children))]
            top = cols[:len(self._schema.fields)]
            keep: list = []
            _check(L.fury_decode_host_execute(plan, _c_host_columns(top, keep)))
        finally:
            L.fury_decode_plan_destroy(plan)
        return top

    # -- framing (Encoders.java:165-182, 201-213) ------------------------------------------
    def frame(self, batch: RowBatch, stream=None):
        """Java ``encode(MemoryBuffer, T)`` stream for every row: returns (bytes, frame_offsets)."""
        n = batch.nrows
        total = batch.rows.numel() + 12 * n
        with _on(stream):
            out = torch.empty(max(total, 16), dtype=torch.uint8, device=self.device)
            fo = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        _check(N.lib().fury_frame_rows(self._schema.handle, _ptr(batch.rows),
                                       _ptr(batch.row_offsets), n, _ptr(out), _ptr(fo),
                                       _stream_handle(stream)))
        return out[:total], fo

    def unframe(self, stream_bytes: torch.Tensor, nrows: int, stream=None) -> RowBatch:
        """Parses a ``decode(MemoryBuffer)`` stream; raises ClassNotCompatibleException on a
        schema-hash mismatch."""
        with _on(stream):
            rows = torch.empty(max(stream_bytes.numel(), 16), dtype=torch.uint8,
                               device=self.device)
            offs = torch.empty(nrows + 1, dtype=torch.int64, device=self.device)
        _check(N.lib().fury_unframe_rows(self._schema.handle, _ptr(stream_bytes),
                                         stream_bytes.numel(), nrows, _ptr(rows), _ptr(offs),
                                         _stream_handle(stream)))
        with _on(stream):
            total = int(offs[nrows].item()) if nrows else 0
        return RowBatch(rows[:total], None if self._schema.is_fixed else offs, nrows,
                        self.schema_hash)

    def encode_stream(self, columns: Sequence[Column], nrows: int, stream=None) -> torch.Tensor:
        """Batch ``encode(MemoryBuffer, T)`` over every row: the byte stream a Java writer loop
        produces (``[int32 len][int64 hash][row]`` per row), in device memory."""
        out, _ = self.frame(self.encode_batch(columns, nrows, stream=stream), stream=stream)
        return out

    def decode_stream(self, stream_bytes: torch.Tensor, nrows: int, validity: bool = True,
                      stream=None) -> List[Column]:
        """Batch ``decode(MemoryBuffer)`` of nrows frames: parallel stream parse, then the
        columns (ClassNotCompatibleException on a schema-hash mismatch, like the reference)."""
        return self.decode_batch(self.unframe(stream_bytes, nrows, stream=stream),
                                 validity=validity, stream=stream)

    # -- single-object API (a bean is a dict name -> value) --------------------------------
    def to_row(self, bean: dict) -> bytes:
        """``toRow(obj).toBytes()``: canonical row bytes of one bean."""
        from .beans import beans_to_columns
        cols = [column_to_device(c, self.device)
                for c in beans_to_columns(self._schema.fields, [bean])]
        b = self.encode_batch(cols, 1)
        return b.row_bytes(0, self._schema.fixed_size)

    def from_row(self, row: bytes) -> dict:
        from .beans import columns_to_beans
        t = torch.frombuffer(bytearray(row), dtype=torch.uint8).to(self.device)
        offs = None if self._schema.is_fixed else torch.tensor([0, len(row)], dtype=torch.int64,
                                                              device=self.device)
        cols = self.decode_batch(RowBatch(t, offs, 1, self.schema_hash))
        return columns_to_beans(self._schema.fields, [column_to_host(c) for c in cols], 1)[0]

    def encode(self, bean: dict) -> bytes:
        """``encode(T)``: [int64 schemaHash][row] (Encoders.java:191-198)."""
        return struct.pack("<q", self.schema_hash) + self.to_row(bean)

    def decode(self, data: bytes) -> dict:
        """``decode(byte[])``: checks the 8-byte schema hash first (Encoders.java:169-188)."""
        if len(data) < 8:
            raise IndexOutOfBoundsException("buffer shorter than the schema hash")
        peer = struct.unpack_from("<q", data, 0)[0]
        if peer != self.schema_hash:
            raise ClassNotCompatibleException(
                f"Schema is not consistent, encoder schema is {self._schema}. self/peer schema "
                f"hash are {self.schema_hash}/{peer}. Please check writer schema.")
        return self.from_row(data[8:])


def _bfs(fields: Sequence[Field]):
    """Schema nodes in the C ABI's breadth-first order: [(field, first_child_index)]."""
    q = list(fields)
    out = []
    i = 0
    while i < len(q):
        f = q[i]
        out.append((f, len(q)))
        q.extend(f.children)
        i += 1
    return out


def _node_sizes(order, cols: List[Column], n: int, stream=None):
    """Arrow entries and STRING / BINARY payload bytes of every schema node (breadth-first
    ``order``) of decoded columns ``cols`` with n top-level entries (device offsets read back)."""
    nodes: List[Optional[Column]] = [None] * len(order)
    m = [0] * len(order)
    b = [0] * len(order)
    ntop = len(cols)
    for k in range(ntop):
        nodes[k] = cols[k]
        m[k] = n
    with _on(stream):
        for i, (f, first) in enumerate(order):
            c = nodes[i]
            t = f.type_id
            end = int(c.offsets[m[i]].item()) if (t in (STRING, BINARY, LIST, MAP) and m[i]) else 0
            if t in (STRING, BINARY):
                b[i] = end
            for j in range(len(f.children)):
                nodes[first + j] = c.child[j]
                m[first + j] = m[i] if t == STRUCT else end
    return m, b


def _pinned_zeros(n: int, dtype=np.uint8) -> np.ndarray:
    a = host_empty(max(int(n), 1) * np.dtype(dtype).itemsize, dtype)
    a[:] = 0
    return a[:n]


def _alloc_host_node(f: Field, m: int, nbytes: int, zeros=np.zeros) -> Column:
    """Host buffers for one schema node with m Arrow entries (fury_decode_host_execute contract:
    exact sizes); ``zeros=_pinned_zeros`` gives pinned ones (the execute writes them in place)."""
    vb = zeros((m + 7) // 8 + 8, np.uint8)
    t = f.type_id
    if t == BOOL:
        return Column(values=zeros((m + 7) // 8 + 8, np.uint8), validity=vb)
    if type_width(t) > 0:
        return Column(values=zeros(m * type_width(t) + 8, np.uint8), validity=vb)
    if t in (STRING, BINARY):
        return Column(values=zeros(max(nbytes, 1), np.uint8), validity=vb,
                      offsets=zeros(m + 1, np.int32))
    if t == DECIMAL:
        return Column(values=zeros(16 * m + 16, np.uint8), validity=vb)
    if t in (LIST, MAP):
        return Column(validity=vb, offsets=zeros(m + 1, np.int32))
    if t == STRUCT:
        return Column(validity=vb)
    raise UnsupportedOperationException(f"no device decode for {f}")


def _alloc_nodes(order, entries, nbytes, validity: bool, device) -> List[Column]:
    """The output buffers of every schema node (breadth-first ``order``) carved from ONE device
    allocation: bitmaps (validity, BOOL values; zeroed -- the decode only sets bits of shared
    words) first, so a single memset clears them, then the int32 Arrow offsets, then values /
    payloads, each 256-B aligned.  One allocation and one memset instead of a few per node (~17
    nodes: the per-tensor cost was a third of a 400k-row decode's wall time), and the views of
    each region cut by ONE split_with_sizes call (round 6: per-view slicing in Python cost ~1 ms
    for a 128-field bean)."""
    def al(x):
        return (x + 255) & ~255
    regions = {"z": [], "o": [], "e": []}       # per region: (node, name, nbytes)
    for i, (f, _first) in enumerate(order):
        m, nb, t = int(entries[i]), int(nbytes[i]), f.type_id
        if validity:
            regions["z"].append((i, "validity", (m + 7) // 8 + 4))
        if t == BOOL:
            regions["z"].append((i, "values", (m + 7) // 8 + 4))
        elif type_width(t) > 0:
            regions["e"].append((i, "values", m * type_width(t) + 8))
        elif t in (STRING, BINARY):
            regions["e"].append((i, "values", max(nb, 1)))
            regions["o"].append((i, "offsets", 4 * (m + 1)))
        elif t == DECIMAL:
            regions["e"].append((i, "values", 16 * m + 16))
        elif t in (LIST, MAP):
            regions["o"].append((i, "offsets", 4 * (m + 1)))
        elif t != STRUCT:
            raise UnsupportedOperationException(f"no device decode for {f}")
    size = {k: sum(al(n) for _, _, n in v) for k, v in regions.items()}
    arena = torch.empty(max(size["z"] + size["o"] + size["e"], 256), dtype=torch.uint8, device=device)
    if size["z"]:
        arena[:size["z"]].zero_()
    views = [dict() for _ in order]
    base = 0
    for k in ("z", "o", "e"):
        segs = regions[k]
        if segs:
            region = arena[base:base + size[k]]
            unit = 4 if k == "o" else 1
            if unit == 4:
                region = region.view(torch.int32)
            sizes = []
            for _, _, n in segs:                 # each view, then its padding to 256 B
                sizes += [n // unit, (al(n) - n) // unit]
            parts = region.split_with_sizes(sizes)
            for j, (i, name, _) in enumerate(segs):
                views[i][name] = parts[2 * j]
        base += size[k]
    return [Column(values=v.get("values"), validity=v.get("validity"), offsets=v.get("offsets"))
            for v in views]


class _CollectionEncoder(RowEncoder):
    """Batch codec of top-level collections over the device engine: batch entry i is one
    BinaryArray (ArrayEncoder) / BinaryMap (MapEncoder).  The batch methods of RowEncoder apply
    unchanged with ONE column, the collection column (no validity: toArray / toMap of a null
    collection is not defined)."""

    def __init__(self, field: Field, device=None):
        self._schema = Schema([field], collection=True)
        self.device = torch.device(device if device is not None else "cuda")
        self._field = field

    def _column(self, values: list) -> Column:
        from .beans import values_to_column
        c = values_to_column(self._field, list(values))
        c.validity = None
        return column_to_device(c, self.device)

    def _values(self, data: bytes) -> list:
        from .beans import value_at
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.device)
        offs = torch.tensor([0, len(data)], dtype=torch.int64, device=self.device)
        cols = self.decode_batch(RowBatch(t, offs, 1, 0))
        return value_at(self._field, column_to_host(cols[0]), 0)

    def _bytes(self, values: list) -> bytes:
        b = self.encode_batch([self._column([values])], 1)
        return bytes(b.rows.cpu().numpy())

    def encode_stream(self, values: list) -> bytes:
        """``encode(MemoryBuffer, T)``: [int32 size][bytes] (Encoders.java:372-386 / 575-590)."""
        body = self._bytes(values)
        return struct.pack("<i", len(body)) + body

    def decode_stream(self, data: bytes, offset: int = 0):
        """``decode(MemoryBuffer)`` at ``offset``: returns (value, next offset)."""
        size = struct.unpack_from("<i", data, offset)[0]
        return self._values(data[offset + 4:offset + 4 + size]), offset + 4 + size


class ArrayEncoder(_CollectionEncoder):
    """``Encoders.arrayEncoder`` (Encoders.java:230-386): List -> BinaryArray.  ``field`` is the
    LIST field TypeInference infers for the collection type (its element: a bean STRUCT, a LIST,
    a MAP, or a scalar)."""

    def field(self) -> Field:
        return self._field

    def to_array(self, values: list) -> bytes:
        """``toArray(obj)`` bytes: [int64 n][null bitmap][n slots][variable section]."""
        return self._bytes(values)

    def from_array(self, data: bytes) -> list:
        return self._values(data)

    def encode(self, values: list) -> bytes:
        """``encode(T)`` of a fresh encoder: ``writer.getBuffer().getBytes(0, 8 + size)``
        (Encoders.java:365-369) = the array followed by 8 bytes of the zeroed buffer -- the length
        ArrayEncoderTest pins (224 / 1576 / 10824).  The reference never rewinds its writer, so a
        second encode() on the same Java encoder returns the FIRST array's bytes (SURVEY §7 trap 5);
        that bug is not reproduced: every call here returns this fresh-encoder result."""
        return self._bytes(values) + bytes(8)

    def decode(self, data: bytes) -> list:
        """``decode(byte[])``: the array at offset 0 (trailing bytes ignored, as pointTo does)."""
        return self._values(data)


class MapEncoder(_CollectionEncoder):
    """``Encoders.mapEncoder`` (Encoders.java:420-600, MapEncoderBuilder.java:152-208): Map ->
    BinaryMap [int64 keyArrayBytes][key BinaryArray][value BinaryArray].  A map value is a list
    of (key, value) pairs in iteration order."""

    def key_field(self) -> Field:
        return self._field.children[0]

    def value_field(self) -> Field:
        return self._field.children[1]

    def to_map(self, pairs: list) -> bytes:
        return self._bytes(pairs)

    def from_map(self, data: bytes) -> list:
        return self._values(data)

    def encode(self, pairs: list) -> bytes:
        """``encode(T)``: ``map.getBuf().getBytes(baseOffset, sizeInBytes)`` = the BinaryMap."""
        return self._bytes(pairs)

    def decode(self, data: bytes) -> list:
        return self._values(data)


class Encoders:
    """``Encoders`` factory (Encoders.java:60-73, 230-420)."""

    @staticmethod
    def bean(fields: Sequence[Field], device=None) -> RowEncoder:
        return RowEncoder(fields, device)

    @staticmethod
    def array_encoder(elem: Field, device=None, name: str = "value") -> ArrayEncoder:
        """``arrayEncoder(List<elem>)``: the LIST field of element field ``elem``."""
        return ArrayEncoder(Field(name, LIST, True, (elem,)), device)

    @staticmethod
    def map_encoder(key: Field, value: Field, device=None, name: str = "value") -> MapEncoder:
        """``mapEncoder(Map<key, value>)``: the MAP field of the key / value fields."""
        return MapEncoder(Field(name, MAP, True, (key, value)), device)


class ArrowWriter:
    """``ArrowWriter`` (ArrowWriter.java:55-99) over RowBatches: ``write(batch)`` converts a whole
    batch on the device and APPENDS it after everything written since ``reset()`` -- the
    reference's write(row) appends at the vectors' rowCount -- so two writes then
    ``finish_as_record_batch()`` give the concatenation.  ``finish()`` returns the accumulated
    device Arrow columns; ``finish_as_record_batch()`` a pyarrow.RecordBatch on the host.

    The accumulated buffers grow like Arrow's setSafe (capacity doubling, amortised O(1) per
    row): a batch that does not fit moves the accumulation into buffers of twice the size first.
    Appends run on the device (``fury_arrow_append``: copies, offset rebasing, bit shifting)."""

    def __init__(self, encoder: RowEncoder):
        self._enc = encoder
        self.reset()

    def write(self, batch: RowBatch, stream=None) -> None:
        """Synchronous like the reference's write(row): a row whose values lie outside the batch
        raises IndexOutOfBoundsException here (nothing of the batch is appended then)."""
        cols = self._enc._decode(batch, True, True, stream)
        self._enc.device_status(stream)
        n = batch.nrows
        order = _bfs(self._enc.schema().fields)
        m, b = _node_sizes(order, cols, n, stream)
        if self._acc is None or self._n == 0:
            self._acc, self._m, self._b = cols, m, b
            self._cap_m, self._cap_b = list(m), list(b)
        else:
            need_m = [x + y for x, y in zip(self._m, m)]
            need_b = [x + y for x, y in zip(self._b, b)]
            if any(x > c for x, c in zip(need_m, self._cap_m)) or \
                    any(x > c for x, c in zip(need_b, self._cap_b)):
                self._grow(order, need_m, need_b, stream)
            keep: list = []
            _check(N.lib().fury_arrow_append(self._enc.schema().handle,
                                             _c_columns(self._acc[:len(cols)], keep), self._n,
                                             _c_columns(cols, keep), n, _stream_handle(stream)))
            self._m, self._b = need_m, need_b
        self._n += n

    def _grow(self, order, need_m, need_b, stream) -> None:
        cap_m = [max(2 * c, x) for c, x in zip(self._cap_m, need_m)]
        cap_b = [max(2 * c, x) for c, x in zip(self._cap_b, need_b)]
        with _on(stream):
            nodes = _alloc_nodes(order, cap_m, cap_b, True, self._enc.device)
        for i, (f, first) in enumerate(order):
            if f.children:
                nodes[i].child = [nodes[first + j] for j in range(len(f.children))]
        top = nodes[:len(self._enc.schema().fields)]
        keep: list = []
        _check(N.lib().fury_arrow_append(self._enc.schema().handle, _c_columns(top, keep), 0,
                                         _c_columns(self._acc, keep), self._n,
                                         _stream_handle(stream)))
        self._acc, self._cap_m, self._cap_b = top, cap_m, cap_b

    def finish(self) -> List[Column]:
        """The device Arrow columns of every row written since reset() (views trimmed to the
        written entries)."""
        if self._acc is None:
            return []
        order = _bfs(self._enc.schema().fields)
        flat: List[Column] = []

        def walk(c: Column, i: int):
            f, first = order[i]
            m, nb = self._m[i], self._b[i]
            t = f.type_id
            out = Column(validity=None if c.validity is None else c.validity[:((m + 31) // 32) * 4])
            if t == BOOL:
                out.values = c.values[:((m + 31) // 32) * 4]
            elif type_width(t) > 0:
                out.values = c.values[:m * type_width(t)]
            elif t == DECIMAL:
                out.values = c.values[:16 * m]
            elif t in (STRING, BINARY):
                out.values = c.values[:max(nb, 1)]
                out.offsets = c.offsets[:m + 1]
            elif t in (LIST, MAP):
                out.offsets = c.offsets[:m + 1]
            if f.children:
                out.child = [walk(c.child[j], first + j) for j in range(len(f.children))]
            return out

        return [walk(c, i) for i, c in enumerate(self._acc)]

    def finish_as_record_batch(self):
        from .arrow import columns_to_record_batch
        return columns_to_record_batch(self._enc.schema().fields,
                                       [column_to_host(c) for c in self.finish()], self._n)

    # -- Arrow IPC (ArrowUtils.serializeRecordBatch / ArrowSerializers, ArrowUtils.java:63-72,
    #    ArrowSerializers.java:128-167) ---------------------------------------------------------
    def ipc_schema(self) -> bytes:
        """Encapsulated IPC Schema message (host bytes)."""
        return ipc_schema_message(self._enc)

    def finish_as_ipc_message(self, stream=None) -> torch.Tensor:
        """The written batch as ONE encapsulated IPC RecordBatch message in device memory
        (``serializeRecordBatch`` of ``finishAsRecordBatch()``)."""
        return ipc_record_batch_message(self._enc, self.finish(), self._n, stream)

    def finish_as_ipc_stream(self, stream=None) -> bytes:
        """Schema message + the batch + end-of-stream marker, on the host: the bytes
        ``ArrowStreamWriter`` writes for the batch (ArrowSerializers.java:128-134)."""
        body = self.finish_as_ipc_message(stream).cpu().numpy().tobytes()
        return self.ipc_schema() + body + IPC_EOS

    def reset(self) -> None:
        """ArrowWriter.reset(): the next write starts a new batch (ArrowWriter.java:95-99)."""
        self._acc: Optional[List[Column]] = None
        self._n = 0
        self._m: List[int] = []
        self._b: List[int] = []
        self._cap_m: List[int] = []
        self._cap_b: List[int] = []


IPC_EOS = b"\xff\xff\xff\xff\x00\x00\x00\x00"


def ipc_schema_message(enc: "RowEncoder") -> bytes:
    n = ctypes.c_int64(0)
    _check(N.lib().fury_arrow_ipc_schema(enc._schema.handle, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value)
    _check(N.lib().fury_arrow_ipc_schema(enc._schema.handle, buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


def ipc_record_batch_message(enc: "RowEncoder", cols: List[Column], nrows: int,
                             stream=None) -> torch.Tensor:
    """Encapsulated IPC RecordBatch message of device columns, gathered on the device."""
    keep: list = []
    cc = _c_columns(cols, keep)
    n = ctypes.c_int64(0)
    sh = _stream_handle(stream)
    _check(N.lib().fury_arrow_ipc_record_batch(enc._schema.handle, cc, nrows, None, 0,
                                               ctypes.byref(n), sh))
    out = torch.empty(max(n.value, 16), dtype=torch.uint8, device=enc.device)
    _check(N.lib().fury_arrow_ipc_record_batch(enc._schema.handle, cc, nrows, _ptr(out), n.value,
                                               ctypes.byref(n), sh))
    return out[:n.value]
