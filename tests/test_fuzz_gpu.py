"""Corrupted rows of random schemas through every decode path on the device: random bytes of a
well-formed batch overwritten (the row offsets stay valid), decoded by the flat kernels, the row
walk and the level engine.  Each decode either succeeds or raises IndexOutOfBoundsException /
UnsupportedOperationException; nothing reads outside the batch (guard bytes after it), nothing
hangs (the walk's item budget, the level engine's element bound), and the stream is clean
afterwards (the intact rows decode to the oracle's columns).  Marked gpu."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from tests.helpers import assert_columns_equal  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _decode(enc, batch):
    from fury_amd.encoder import column_to_host
    if enc.nested:
        from tests.test_tree import _decode_plan
        return _decode_plan(enc, batch)
    return [column_to_host(c) for c in enc.decode_batch(batch)]


@pytest.mark.parametrize("seed", list(range(24)))
def test_corrupt_rows_random_schemas(oracle, dev, seed):
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, IndexOutOfBoundsException, UnsupportedOperationException
    from tests.test_bounds import _batch
    from tests.test_tree import _beans, _random_schema
    rng = np.random.default_rng(9000 + seed)
    fields = _random_schema(rng, int(rng.integers(0, 5)), int(rng.integers(1, 12)))
    n = int(rng.integers(2, 600))
    host = beans_to_columns(fields, _beans(fields, n, seed))
    enc = Encoders.bean(fields, device=dev)
    rows, offs = oracle.encode(fields, host, n)
    rows = rows.copy()
    offs = np.asarray(offs, np.int64).copy()
    ref = oracle.decode(fields, rows, offs, n)
    L = N.lib()
    old = L.fury_get_tuning(b"nested_decode")
    try:
        for trial in range(3):
            bad = rows.copy()
            if len(bad):
                pos = rng.integers(0, len(bad), int(rng.integers(1, 40)))
                bad[pos] = rng.integers(0, 256, len(pos)).astype(np.uint8)
            for mode in ((2, 1) if enc.nested else (2,)):
                L.fury_set_tuning(b"nested_decode", mode)
                try:
                    _decode(enc, _batch(enc, bad, offs, n, dev))
                except (IndexOutOfBoundsException, UnsupportedOperationException):
                    pass
        L.fury_set_tuning(b"nested_decode", 2)
        assert_columns_equal(fields, _decode(enc, _batch(enc, rows, offs, n, dev)), ref, n)
    finally:
        L.fury_set_tuning(b"nested_decode", old)
