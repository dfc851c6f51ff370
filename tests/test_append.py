"""ArrowWriter accumulation (GPU): write(batch) appends after every row written since reset(), as
the reference's write(row) appends at the vectors' rowCount (java/fury-format/.../vectorized/
ArrowWriter.java:74-99) -- through fury_arrow_append on the device.  Two or three writes then
finish_as_record_batch() must equal pyarrow's concatenation of the batches converted one by one.
Also: a bound call keeps its schema alive after its encoder is dropped.  Marked gpu."""
from __future__ import annotations

import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
pa = pytest.importorskip("pyarrow")

from fury_amd.workloads import SCHEMAS, gen_columns  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _batches(name, sizes, dev):
    from fury_amd.encoder import Encoders, column_to_device
    fields = SCHEMAS[name]
    enc = Encoders.bean(fields, device=dev)
    out = []
    for j, n in enumerate(sizes):
        if name == "foo":
            from fury_amd.beans import beans_to_columns
            from tests.test_device import _random_value
            rng = np.random.default_rng(j)
            host = beans_to_columns(fields, [{f.name: _random_value(f, rng) for f in fields}
                                             for _ in range(n)])
        else:
            host = gen_columns(name, fields, n, seed=100 + j)
        out.append(enc.encode_batch([column_to_device(c, dev) for c in host], n))
    return enc, out


@pytest.mark.parametrize("name", ["mixed", "nested", "narrow", "struct100", "foo"])
def test_arrow_writer_appends(dev, name):
    from fury_amd.encoder import ArrowWriter
    sizes = [1001, 77, 2050, 31]
    enc, batches = _batches(name, sizes, dev)
    singles = []
    for b in batches:
        w1 = ArrowWriter(enc)
        w1.write(b)
        singles.append(w1.finish_as_record_batch())
    w = ArrowWriter(enc)
    for b in batches:
        w.write(b)
    got = w.finish_as_record_batch()
    want = pa.Table.from_batches(singles).combine_chunks().to_batches()[0]
    assert got.num_rows == sum(sizes)
    assert got.equals(want), name
    # reset(): the next write starts over
    w.reset()
    w.write(batches[2])
    assert w.finish_as_record_batch().equals(singles[2])
    # device columns of finish() hold exactly the written rows
    w.reset()
    w.write(batches[1])
    w.write(batches[3])
    tail = pa.Table.from_batches([singles[1], singles[3]]).combine_chunks().to_batches()[0]
    assert w.finish_as_record_batch().equals(tail)


def test_arrow_writer_ipc_after_appends(dev):
    """The IPC message of an accumulated writer decodes (pyarrow) to the concatenation."""
    import pyarrow.ipc as ipc
    from fury_amd.encoder import ArrowWriter
    enc, batches = _batches("mixed", [500, 333], dev)
    w = ArrowWriter(enc)
    for b in batches:
        w.write(b)
    table = ipc.open_stream(w.finish_as_ipc_stream()).read_all()
    assert table.num_rows == 833
    assert table.combine_chunks().to_batches()[0].equals(w.finish_as_record_batch())


def test_bound_call_outlives_encoder(oracle, dev):
    from fury_amd.encoder import Encoders, column_to_device
    fields = SCHEMAS["mixed"]
    n = 999
    host = gen_columns("mixed", fields, n, seed=9)
    cols = [column_to_device(c, dev) for c in host]
    enc = Encoders.bean(fields, device=dev)
    offs = enc.measure(cols, n)
    rows = torch.zeros(int(offs[n].item()) + 64, dtype=torch.uint8, device=dev)
    call = enc.bind_encode(cols, n, rows, offs)
    del enc
    gc.collect()
    call()
    torch.cuda.synchronize()
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(rows[:len(want)].cpu().numpy(), want)
