"""The row-staged variable-length decode (decode_var_reg, var_dev.h) on LIST columns under the three
conditions round 3's unexplained fault could have reached:

* stage window -- a tile's row bytes beyond the LDS stage (dec_tile_plan sizes tiles from the
  batch average, so tiles of long lists read their tail rows from HBM);
* image capacity -- a tile's list elements beyond its LDS output image (the column goes straight
  to HBM, element by element);
* list-run indexing -- element runs of 0 / 1 / 63 / 64 / 65 / 127 / 129 elements starting at
  every bit position of the validity words, BOOL / INT16 / INT64 elements, nulls.

Each case is checked byte for byte against the oracle's decode, through fury_row_decode (exact
"measure" and row-sized "bound" output buffers) and ArrowWriter (fury_rows_to_arrow).  Marked
gpu."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from fury_amd import types as T  # noqa: E402
from tests.helpers import assert_columns_equal  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _c4_like(elem_type, elem_nullable=True):
    return [T.not_null_field("id", T.INT64), T.not_null_field("score", T.FLOAT64),
            T.array_field("vals", elem_type, elem_nullable=elem_nullable)]


def _value(t, i, j):
    if t == T.BOOL:
        return (i + j) % 3 == 0
    if t == T.INT16:
        return ((i * 131 + j * 7) % 65536) - 32768
    return (i << 20) + j * 0x9E3779B9 - (1 << 40)


def _beans(fields, lens, null_every=17, elem_null_every=5):
    et = fields[2].children[0].type_id
    out = []
    for i, m in enumerate(lens):
        vals = None if (null_every and i % null_every == 3 % null_every) else [
            None if (elem_null_every and fields[2].children[0].nullable and (i + j) % elem_null_every == 1)
            else _value(et, i, j) for j in range(m)]
        out.append({"id": i, "score": i * 0.5, "vals": vals})
    return out


def _check(oracle, dev, fields, beans):
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device, column_to_host
    n = len(beans)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    assert not enc.nested
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    ref = oracle.decode(fields, want, want_offs, n)
    for sizing in ("measure", "bound"):
        got = [column_to_host(c) for c in enc.decode_batch(batch, sizing=sizing)]
        assert_columns_equal(fields, got, ref, n)
    from fury_amd.encoder import ArrowWriter
    w = ArrowWriter(enc)
    w.write(batch)
    arrow = [column_to_host(c) for c in w.finish()]
    assert_columns_equal(fields, arrow, ref, n)


@pytest.mark.parametrize("elem", [T.INT64, T.INT16, T.BOOL])
def test_lists_beyond_stage_and_image(oracle, dev, elem):
    """Long-list rows among short ones: most tiles hold ~avg-sized rows, the tiles around the
    long rows exceed both the stage and the element image."""
    rng = np.random.default_rng(int(elem))
    lens = [int(rng.integers(0, 4)) for _ in range(30_000)]
    for i in range(0, len(lens), 997):
        for k in range(i, min(i + 40, len(lens))):
            lens[k] = int(rng.integers(300, 700))
    _check(oracle, dev, _c4_like(elem), _beans(_c4_like(elem), lens))


@pytest.mark.parametrize("elem", [T.INT64, T.INT16, T.BOOL])
def test_list_runs_every_bit_position(oracle, dev, elem):
    """Element runs whose lengths walk 0, 1, 63, 64, 65, 127, 129 while their start moves through
    every bit position of the element validity words (and of BOOL value words)."""
    pattern = [0, 1, 63, 64, 65, 127, 129, 2, 31, 32, 33]
    lens = [pattern[i % len(pattern)] + (i // len(pattern)) % 3 for i in range(9000)]
    _check(oracle, dev, _c4_like(elem), _beans(_c4_like(elem), lens, elem_null_every=3))


def test_non_nullable_elements_all_empty_and_all_null(oracle, dev):
    """int[]-style lists (non-null elements), a batch of only empty lists, a batch of only null
    lists."""
    f = _c4_like(T.INT64, elem_nullable=False)
    _check(oracle, dev, f, _beans(f, [(i * 7) % 40 for i in range(5000)], elem_null_every=0))
    _check(oracle, dev, f, _beans(f, [0] * 3000, null_every=0))
    _check(oracle, dev, f, _beans(f, [5] * 3000, null_every=1))
