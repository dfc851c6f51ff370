"""The torch column generator (device data for the bench and the configuration-size GPU tests)
equals the numpy generator bit for bit: fixed-width, bool, decimal, string, binary and list
columns, nulls, element nulls, a non-zero start row (shards).  CPU."""
from __future__ import annotations

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from fury_amd.workloads import SCHEMAS, gen_columns, gen_columns_torch  # noqa: E402


def _eq(a, b, what):
    if a is None or b is None:
        assert a is None and b is None, what
        return
    assert np.array_equal(np.asarray(a).view(np.uint8).reshape(-1),
                          b.cpu().contiguous().view(torch.uint8).numpy().reshape(-1)), what


@pytest.mark.parametrize("name", ["struct100", "mixed", "nested", "narrow"])
@pytest.mark.parametrize("start", [0, 1_000_003])
def test_torch_generator_matches_numpy(name, start):
    fields = SCHEMAS[name]
    n = 2053
    a = gen_columns(name, fields, n, seed=77, start=start)
    b = gen_columns_torch(name, fields, n, seed=77, start=start, device="cpu")
    for f, x, y in zip(fields, a, b):
        _eq(x.values, y.values, f"{f.name} values")
        _eq(x.validity, y.validity, f"{f.name} validity")
        _eq(x.offsets, y.offsets, f"{f.name} offsets")
        if x.child:
            _eq(x.child[0].values, y.child[0].values, f"{f.name} child values")
            _eq(x.child[0].validity, y.child[0].validity, f"{f.name} child validity")


@pytest.mark.parametrize("name", ["struct100", "mixed", "nested", "narrow"])
def test_slice_columns_encode_like_the_whole(oracle, name):
    """Row slices (the CPU baseline's per-thread batches) encode to exactly the rows of the whole
    batch's encode between the slice's row offsets."""
    from fury_amd.workloads import slice_columns
    fields = SCHEMAS[name]
    n = 1037
    cols = gen_columns(name, fields, n, seed=5)
    rows, offs = oracle.encode(fields, cols, n)
    for b, e in ((0, 300), (300, 301), (301, 1037), (17, 999)):
        part = slice_columns(fields, cols, b, e)
        r, o = oracle.encode(fields, part, e - b)
        if offs is None:
            fs = len(rows) // n
            assert np.array_equal(r, rows[b * fs:e * fs])
        else:
            assert np.array_equal(r, rows[offs[b]:offs[e]])
            assert np.array_equal(o, offs[b:e + 1] - offs[b])
