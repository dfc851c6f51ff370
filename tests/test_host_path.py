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


def test_host_nested_encode_and_decode_unsupported(oracle):
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, UnsupportedOperationException
    from tests.test_device import _nested_beans, _nested_fields
    fields = _nested_fields()
    beans = _nested_beans(300, seed=2)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device="cuda:0")
    rows, offs = enc.encode_host(host, 300)
    want, want_offs = oracle.encode(fields, host, 300)
    assert np.array_equal(rows, want) and np.array_equal(offs, want_offs)
    with pytest.raises(UnsupportedOperationException):
        enc.decode_host(rows, offs, 300, out=[])


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
