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
