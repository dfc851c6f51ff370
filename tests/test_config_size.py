"""BASELINE.json configurations at their full sizes on the GPU (the oracle finishes only small
cases in seconds, so these check size-independent properties plus oracle windows):
  C3 -- 10M rows of the mixed schema (int32 / int64 / double + 3 UTF-8 strings, all nullable):
        decode(encode(cols)) == cols, every buffer (validity, values, offsets, payloads);
  C4 -- 4M rows id / score / list<int64>: rows -> Arrow (fury_rows_to_arrow) == the input
        columns (null lists are zero-length Arrow entries, as the generator writes them);
and for both, 300-row windows at the start, middle and end of the device rows equal the oracle's
encode of the same global rows.  Columns are generated on the device (gen_columns_torch, bit-equal
to the numpy generator: tests/test_workloads.py).  Marked gpu."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from fury_amd.workloads import SCHEMAS, gen_columns, gen_columns_torch  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _bits_equal(a, b, n, what):
    """First n bits of two bitmaps (device uint8 tensors)."""
    full = n // 8
    assert torch.equal(a[:full], b[:full]), what
    if n % 8:
        m = (1 << (n % 8)) - 1
        assert int(a[full]) & m == int(b[full]) & m, what


def _u8(t):
    return t.contiguous().view(torch.uint8)


def _windows(oracle, name, fields, batch, n):
    for off in (0, n // 2, n - 300):
        host = gen_columns(name, fields, 300, seed=1234, start=off)
        want, want_offs = oracle.encode(fields, host, 300)
        o = batch.row_offsets[off:off + 301].cpu().numpy()
        assert np.array_equal(o - o[0], want_offs), (name, off)
        assert np.array_equal(batch.rows[int(o[0]):int(o[-1])].cpu().numpy(), want), (name, off)


def test_c3_mixed_10m(oracle, dev):
    from fury_amd.encoder import Encoders
    name, n = "mixed", 10_000_000
    fields = SCHEMAS[name]
    cols = gen_columns_torch(name, fields, n, seed=1234, device=dev)
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, n)
    _windows(oracle, name, fields, b, n)
    dec = enc.decode_batch(b, validity=True, sizing="bound")
    for f, c, d in zip(fields, cols, dec):
        _bits_equal(c.validity, d.validity, n, f.name)
        if c.offsets is None:
            assert torch.equal(_u8(c.values), _u8(d.values)[:_u8(c.values).numel()]), f.name
        else:
            assert torch.equal(c.offsets, d.offsets), f.name
            tot = int(c.offsets[n])
            assert torch.equal(c.values[:tot], d.values[:tot]), f.name
    assert enc.schema_hash == 15296648724


def test_c4_nested_4m_rows_to_arrow(oracle, dev):
    from fury_amd.encoder import ArrowWriter, Encoders
    name, n = "nested", 4_000_000
    fields = SCHEMAS[name]
    cols = gen_columns_torch(name, fields, n, seed=1234, device=dev)
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, n)
    _windows(oracle, name, fields, b, n)
    w = ArrowWriter(enc)
    w.write(b)
    out = w.finish()
    for f, c, d in zip(fields, cols, out):
        if c.validity is None:          # non-null field: Arrow validity all set
            assert int(_u8(d.validity)[:n // 8].min()) == 255, f.name
        else:
            _bits_equal(c.validity, d.validity, n, f.name)
        if c.offsets is None:
            assert torch.equal(_u8(c.values), _u8(d.values)[:_u8(c.values).numel()]), f.name
        else:
            assert torch.equal(c.offsets, d.offsets), f.name
            m = int(c.offsets[n])
            assert torch.equal(_u8(c.child[0].values)[:8 * m], _u8(d.child[0].values)[:8 * m])
            assert int(_u8(d.child[0].validity)[:m // 8].min()) == 255
    assert enc.schema_hash == 15980292
