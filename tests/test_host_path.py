"""Host-memory batch path (the JNI boundary, include/fury_row.h fury_row_encode_host /
fury_row_decode_host): host columns -> HBM -> host rows and back inside one call, bit-exact
against the oracle.  Fixed-width batches span several pipeline chunks (ragged last chunk).
Marked gpu."""
from __future__ import annotations

import numpy as np
import pytest

from fury_amd.workloads import SCHEMAS, gen_columns
from tests.helpers import assert_columns_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n", [("struct100", 130_001), ("docs_struct", 4097), ("narrow", 1000),
                                    ("mixed", 20_011), ("nested", 9_999), ("struct100", 1),
                                    ("mixed", 0)])
def test_host_roundtrip_bit_exact(oracle, name, n):
    from fury_amd.encoder import Encoders
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=17)
    enc = Encoders.bean(fields, device="cuda:0")
    rows, offs = enc.encode_host(host, n)
    want, want_offs = oracle.encode(fields, host, n)
    assert rows.shape == want.shape and np.array_equal(rows, want), f"{name}: rows differ"
    if offs is not None:
        assert np.array_equal(offs, want_offs)
    if n == 0:
        return
    dec = enc.decode_host(rows, offs, n)
    ref = oracle.decode(fields, want, want_offs, n)
    assert_columns_equal(fields, dec, ref, n)


@pytest.mark.parametrize("n", [1, 300, 5000])
def test_host_nested_encode_and_decode(oracle, n):
    """Nested beans (struct, map, list of lists / structs / strings) through the host-memory
    path: encode_host bit-exact, and the two-step host decode (fury_decode_host_prepare /
    execute) returns the oracle's columns -- what GpuRowEncoder.decodeBatch needs for beans with
    nested beans, maps and lists of structs."""
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders
    from tests.test_device import _nested_beans, _nested_fields
    fields = _nested_fields()
    beans = _nested_beans(n, seed=2)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device="cuda:0")
    rows, offs = enc.encode_host(host, n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(rows, want) and np.array_equal(offs, want_offs)
    dec = enc.decode_host(rows, offs, n)
    assert_columns_equal(fields, dec, oracle.decode(fields, want, want_offs, n), n)
    assert columns_to_beans(fields, dec, n) == beans


def test_host_nested_decode_capacity_and_foo(oracle):
    """RowEncoderTest.Foo rows decoded from host memory; a too small payload buffer is a
    CapacityError (IndexOutOfBounds family), nothing partial."""
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders
    fields = SCHEMAS["foo"]
    beans = [{"f1": i, "f2": "str" * (i % 3), "f3": [str(j) for j in range(i % 4)],
              "f4": [(str(i), i)], "f5": {"f1": i, "f2": None if i % 2 else "b"}}
             for i in range(700)]
    enc = Encoders.bean(fields, device="cuda:0")
    rows, offs = enc.encode_host(beans_to_columns(fields, beans), len(beans))
    assert columns_to_beans(fields, enc.decode_host(rows, offs, len(beans)), len(beans)) == beans
    import ctypes
    L = N.lib()
    nn = L.fury_schema_num_nodes(enc.schema().handle)
    e = (ctypes.c_int64 * nn)()
    b = (ctypes.c_int64 * nn)()
    plan = ctypes.c_void_p()
    assert L.fury_decode_host_prepare(enc.schema().handle, rows.ctypes.data, offs.ctypes.data,
                                      len(beans), e, b, ctypes.byref(plan), 0) == 0
    try:
        from fury_amd.encoder import _alloc_host_node, _bfs, _c_host_columns
        order = _bfs(fields)
        cols = [_alloc_host_node(f, int(e[i]), int(b[i])) for i, (f, _) in enumerate(order)]
        for i, (f, first) in enumerate(order):
            if f.children:
                cols[i].child = [cols[first + j] for j in range(len(f.children))]
        cols[1].values = cols[1].values[:max(int(b[1]) - 1, 0)]     # f2 payload one byte short
        keep = []
        assert L.fury_decode_host_execute(plan, _c_host_columns(cols[:len(fields)], keep)) == 7
    finally:
        L.fury_decode_plan_destroy(plan)


def test_host_pinned_buffers():
    """Pinned (fury_host_register) host buffers give the same bytes as pageable ones."""
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import Column
    fields = SCHEMAS["struct100"]
    n = 70_000
    host = gen_columns("struct100", fields, n, seed=3)
    pinned = [Column(values=torch.from_numpy(c.values.view(np.uint8).copy()).pin_memory())
              for c in host]
    enc = Encoders.bean(fields, device="cuda:0")
    rows_ref, _ = enc.encode_host(host, n)
    buf = np.empty(n * 816, dtype=np.uint8)
    assert N.lib().fury_host_register(buf.ctypes.data, buf.nbytes) == 0
    try:
        rows, _ = enc.encode_host(pinned, n, rows=buf)
    finally:
        N.lib().fury_host_unregister(buf.ctypes.data)
    assert np.array_equal(rows, rows_ref)


def _fixed_nullable():
    from fury_amd.types import (BOOL, DATE32, FLOAT32, FLOAT64, INT8, INT16, INT32, INT64,
                                TIMESTAMP, field, not_null_field)
    return [field("a_bool", BOOL), field("b_byte", INT8), field("c_short", INT16),
            not_null_field("d_int", INT32), field("e_float", FLOAT32), field("f_date", DATE32),
            field("g_ts", TIMESTAMP), not_null_field("i_flag", BOOL),
            field("j_double", FLOAT64), not_null_field("k_long", INT64)]


def enc_is_fixed(fields):
    from fury_amd.encoder import Schema
    return Schema(fields).is_fixed


def _pinned(a):
    import torch
    return None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).pin_memory()


@pytest.mark.parametrize("name,n", [("struct100", 70_001), ("fixed_nullable", 33_333),
                                    ("fixed_nullable", 1), ("fixed_nullable", 64)])
def test_host_direct_pinned_fixed(oracle, name, n):
    """Fixed-width schemas with every host buffer pinned run the kernel directly on host memory
    (fury_get_tuning("host_direct") counts it): rows bit-exact vs the oracle, decode into pinned
    outputs whose bitmaps are exactly (n + 7) / 8 bytes (the guard bytes after them untouched)."""
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import Column
    fields = SCHEMAS["struct100"] if name == "struct100" else _fixed_nullable()
    assert enc_is_fixed(fields)
    host = gen_columns(name, fields, n, seed=5)
    pinned = [Column(values=_pinned(c.values), validity=_pinned(c.validity)) for c in host]
    enc = Encoders.bean(fields, device="cuda:0")
    want, _ = oracle.encode(fields, host, n)
    L = N.lib()
    d0 = L.fury_get_tuning(b"host_direct")
    rows = torch.empty(want.size, dtype=torch.uint8).pin_memory()
    got, _ = enc.encode_host(pinned, n, rows=rows)
    assert L.fury_get_tuning(b"host_direct") == d0 + 1, "encode did not take the direct path"
    assert np.array_equal(got.numpy(), want)
    ref = oracle.decode(fields, want, None, n)
    nb = (n + 7) // 8
    out = []
    for f, c in zip(fields, host):
        from fury_amd.types import BOOL, type_width
        vb = nb if f.type_id == BOOL else n * (16 if type_width(f.type_id) <= 0 else type_width(f.type_id))
        v = torch.full((vb + 8,), 0xAB, dtype=torch.uint8).pin_memory()
        m = torch.full((nb + 8,), 0xAB, dtype=torch.uint8).pin_memory() if f.nullable else None
        out.append((v, m))
    cols = [Column(values=v[:-8], validity=None if m is None else m[:-8]) for v, m in out]
    enc.decode_host(rows, None, n, out=cols)
    assert L.fury_get_tuning(b"host_direct") == d0 + 2, "decode did not take the direct path"
    assert_columns_equal(fields, cols, ref, n)
    for v, m in out:
        assert bool((v[-8:] == 0xAB).all()), "decode wrote past a values buffer"
        if m is not None:
            assert bool((m[-8:] == 0xAB).all()), "decode wrote past a validity bitmap"


def test_host_direct_falls_back_for_pageable_and_misaligned(oracle):
    """One pageable column, or a pinned row buffer that is not 16-byte aligned, sends the call
    down the staged path (same bytes)."""
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import Column
    fields = SCHEMAS["struct100"]
    n = 3000
    host = gen_columns("struct100", fields, n, seed=9)
    want, _ = oracle.encode(fields, host, n)
    pinned = [Column(values=_pinned(c.values)) for c in host]
    mixed = pinned[:-1] + [host[-1]]
    enc = Encoders.bean(fields, device="cuda:0")
    L = N.lib()
    d0 = L.fury_get_tuning(b"host_direct")
    rows = torch.empty(want.size, dtype=torch.uint8).pin_memory()
    assert np.array_equal(enc.encode_host(mixed, n, rows=rows)[0].numpy(), want)
    shifted = torch.empty(want.size + 8, dtype=torch.uint8).pin_memory()[8:]
    assert np.array_equal(enc.encode_host(pinned, n, rows=shifted)[0].numpy(), want)
    assert L.fury_get_tuning(b"host_direct") == d0
    assert np.array_equal(enc.encode_host(pinned, n, rows=rows)[0].numpy(), want)
    assert L.fury_get_tuning(b"host_direct") == d0 + 1


def test_host_empty_buffers_take_direct_path(oracle):
    """fury_host_alloc buffers (encoder.host_empty) are device-visible: encode_host / decode_host
    on them run direct, bit-exact."""
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders, host_empty
    from fury_amd.workloads import Column
    fields = SCHEMAS["struct100"]
    n = 4099
    host = gen_columns("struct100", fields, n, seed=21)
    cols = []
    for c in host:
        b = host_empty(c.values.nbytes)
        b[:] = c.values.view(np.uint8)
        cols.append(Column(values=b))
    enc = Encoders.bean(fields, device="cuda:0")
    want, _ = oracle.encode(fields, host, n)
    d0 = N.lib().fury_get_tuning(b"host_direct")
    rows = host_empty(want.size)
    got, _ = enc.encode_host(cols, n, rows=rows)
    out = [Column(values=host_empty(n * 8)) for _ in fields]
    enc.decode_host(rows, None, n, out=out)
    assert N.lib().fury_get_tuning(b"host_direct") == d0 + 2
    assert np.array_equal(got, want)
    assert all(np.array_equal(o.values, c.values.view(np.uint8)) for o, c in zip(out, host))


def _page_tail(nbytes, dtype=np.uint8):
    """A pinned (fury_host_alloc) buffer of exactly `nbytes` whose last byte is the last byte of
    its allocation's last page: a kernel read past the buffer's last 16-byte block would leave the
    mapping."""
    from fury_amd.encoder import host_empty
    size = max(int(nbytes), 1)
    alloc = (size + 4095) // 4096 * 4096
    return host_empty(alloc)[alloc - size:].view(dtype)


def _tail_copy(a, dtype):
    if a is None:
        return None
    src = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    b = _page_tail(src.nbytes)[:src.nbytes]
    b[:] = src
    return b.view(dtype)


def _tail_tree(c, fill: bool):
    from fury_amd.workloads import Column
    ch = [_tail_tree(x, fill) for x in c.child] if c.child else None
    if fill:
        return Column(values=_tail_copy(c.values, np.uint8), validity=_tail_copy(c.validity, np.uint8),
                      offsets=_tail_copy(c.offsets, np.int32), child=ch)

    def empty(a, dtype):
        return None if a is None else _page_tail(np.asarray(a).nbytes, dtype)
    return Column(values=empty(c.values, np.uint8), validity=empty(c.validity, np.uint8),
                  offsets=empty(c.offsets, np.int32), child=ch)


@pytest.mark.parametrize("name,n", [("mixed", 20_011), ("nested", 9_999), ("narrow", 3000),
                                    ("beanb", 777), ("mixed", 1)])
def test_host_direct_var_page_edge(oracle, name, n):
    """Flat variable-length schemas on pinned buffers run their kernels on host memory
    (host_direct counts both calls), every input and output buffer exactly its size and ending at
    a page edge: rows, row offsets and decoded columns bit-exact vs the oracle."""
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=29)
    want, want_offs = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, want_offs, n)
    enc = Encoders.bean(fields, device="cuda:0")
    L = N.lib()
    d0 = L.fury_get_tuning(b"host_direct")
    cols = [_tail_tree(c, True) for c in host]
    rows = _page_tail((want.size + 15) // 16 * 16)      # rows must be 16-byte aligned
    roffs = _page_tail(8 * (n + 1), np.int64)
    got, offs = enc.encode_host(cols, n, rows=rows, row_offsets=roffs)
    assert L.fury_get_tuning(b"host_direct") == d0 + 1, "encode did not take the direct path"
    assert np.array_equal(got, want) and np.array_equal(offs, want_offs)
    out = [_tail_tree(c, False) for c in ref]
    enc.decode_host(rows, roffs, n, out=out)
    assert L.fury_get_tuning(b"host_direct") == d0 + 2, "decode did not take the direct path"
    assert_columns_equal(fields, out, ref, n)


def test_host_direct_var_capacity_short(oracle):
    """A payload buffer one byte short: the direct decode reports FURY_ERR_CAPACITY (it writes
    nothing past the capacity)."""
    from fury_amd.encoder import CapacityError, Encoders
    fields = SCHEMAS["mixed"]
    n = 3000
    host = gen_columns("mixed", fields, n, seed=31)
    want, want_offs = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, want_offs, n)
    enc = Encoders.bean(fields, device="cuda:0")
    rows = _page_tail((want.size + 15) // 16 * 16)
    rows[:want.size] = want
    roffs = _tail_copy(want_offs, np.int64)
    from fury_amd import _native as N
    d0 = N.lib().fury_get_tuning(b"host_direct")
    out = [_tail_tree(c, False) for c in ref]
    k = next(i for i, f in enumerate(fields) if ref[i].offsets is not None and len(ref[i].values) > 1)
    full = out[k].values
    guard = _page_tail(full.nbytes + 8)
    guard[:] = 0xAB
    out[k].values = guard[:full.nbytes - 1]
    with pytest.raises(CapacityError):
        enc.decode_host(rows, roffs, n, out=out)
    assert N.lib().fury_get_tuning(b"host_direct") == d0 + 1, "decode did not take the direct path"
    assert bool((guard[full.nbytes - 1:] == 0xAB).all()), "decode wrote past the capacity"


def _page_zeros(n, dtype=np.uint8):
    a = _page_tail(max(int(n), 1) * np.dtype(dtype).itemsize, dtype)
    a[:] = 0
    return a[:n]


@pytest.mark.parametrize("name,n", [("foo", 3001), ("beana", 1200), ("nested7", 5000),
                                    ("maps", 777), ("nested7", 1)])
def test_host_direct_nested_page_edge(oracle, name, n):
    """Nested schemas (RowEncoderTest's Foo and BeanA among them) on pinned buffers: the encode
    reads the column tree and writes rows in place (kernels on host memory); the decode stages the
    rows in HBM and, with tuning host_decode_inplace, writes values / offsets / payloads into the
    pinned outputs (bitmaps through HBM) -- host_direct counts both.  Every buffer ends at a page
    edge; rows, offsets and columns bit-exact vs the oracle."""
    import ctypes
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, _alloc_host_node, _bfs, _c_host_columns
    from tests.test_tree import _beans, _schemas
    fields = _schemas()[name]
    beans = _beans(fields, n, n + len(name))
    host = beans_to_columns(fields, beans)
    want, want_offs = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, want_offs, n)
    enc = Encoders.bean(fields, device="cuda:0")
    L = N.lib()
    d0 = L.fury_get_tuning(b"host_direct")
    cols = [_tail_tree(c, True) for c in host]
    rows = _page_tail((want.size + 15) // 16 * 16)
    roffs = _page_tail(8 * (n + 1), np.int64)
    got, offs = enc.encode_host(cols, n, rows=rows, row_offsets=roffs)
    assert L.fury_get_tuning(b"host_direct") == d0 + 1, "encode did not take the direct path"
    assert np.array_equal(got, want) and np.array_equal(offs, want_offs)
    nn = L.fury_schema_num_nodes(enc.schema().handle)
    e = (ctypes.c_int64 * nn)()
    b = (ctypes.c_int64 * nn)()
    plan = ctypes.c_void_p()
    assert L.fury_decode_host_prepare(enc.schema().handle, rows.ctypes.data, roffs.ctypes.data,
                                      n, e, b, ctypes.byref(plan), 0) == 0, N.last_error()
    assert L.fury_set_tuning(b"host_decode_inplace", 1) == 0
    try:
        order = _bfs(fields)
        out = [_alloc_host_node(f, int(e[i]), int(b[i]), _page_zeros) for i, (f, _) in enumerate(order)]
        for i, (f, first) in enumerate(order):
            if f.children:
                out[i].child = [out[first + j] for j in range(len(f.children))]
        keep = []
        assert L.fury_decode_host_execute(plan, _c_host_columns(out[:len(fields)], keep)) == 0, \
            N.last_error()
    finally:
        L.fury_set_tuning(b"host_decode_inplace", 0)
        L.fury_decode_plan_destroy(plan)
    assert L.fury_get_tuning(b"host_direct") == d0 + 2, "decode did not write in place"
    top = out[:len(fields)]
    assert_columns_equal(fields, top, ref, n)
    assert columns_to_beans(fields, top, n) == beans
