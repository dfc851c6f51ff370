"""Corrupted rows of random schemas, device against the oracle's bounds rule.  Random bytes of a
well-formed batch are overwritten (the row offsets stay valid) and the batch is decoded by the
flat kernels, the row walk and the level engine.  Per trial the oracle -- the reference's decode
bounds rule restated in row_oracle.c (MemoryBuffer.checkPosition / get / slice / copyToUnsafe,
java/fury-core/.../memory/MemoryBuffer.java:303-309,2451-2455,2515-2518, per container) --
predicts the outcome and the device must produce it:
  * the oracle raises IndexOutOfBoundsException (or the map-count UnsupportedOperationException,
    BinaryMap.java:73-75) -> the device raises the same exception;
  * the oracle decodes -> the device decodes to identical columns, or raises the nested decode's
    item-budget error (a device limit with its own message, never a bounds error: rows whose slots
    alias other bytes).  The row walk's budget is restated too (fo_count_walk), so for the walk the
    budget error is predicted exactly; the level engine bounds each node's elements by the batch's
    bytes instead and may report it for rows the walk's budget admits.
The batch sits in a buffer with 0xAB guard bytes after it: a read past the batch would show as a
difference from the oracle, which never reads there.  The stream is clean afterwards (the intact
rows decode to the oracle's columns).  Marked gpu."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from fury_amd import types as T  # noqa: E402
from tests.helpers import assert_columns_equal  # noqa: E402

COUNTED = (T.STRING, T.BINARY, T.LIST, T.MAP)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _decode(enc, batch):
    from fury_amd.encoder import column_to_host
    if enc.nested:
        from tests.test_tree import _decode_plan
        cols = _decode_plan(enc, batch)
    else:
        cols = [column_to_host(c) for c in enc.decode_batch(batch)]
    enc.device_status()                      # errors the execute raised asynchronously
    return cols


def _shape(fields):
    """(levels, counted nodes) of a schema: the row walk takes <= 5 levels, <= 256 counted nodes."""
    def walk(f, d):
        lv, k = d + 1, int(f.type_id in COUNTED)
        for c in f.children:
            a, b = walk(c, d + 1)
            lv, k = max(lv, a), k + b
        return lv, k
    lv, k = 0, 0
    for f in fields:
        a, b = walk(f, 0)
        lv, k = max(lv, a), k + b
    return lv, k


def _expected(O, fields, nested, engine, rows, offs, n):
    """What the device must report: "oob", "map", "budget", "any" (an engine on a batch the walk's
    budget refuses: the oracle's full walk of it is not bounded), or the oracle's columns.
    engine: "walk" (its count pass is restated exactly, budget included), "bfs" (the same count-pass
    containers without a budget; a batch whose tiles overflow the arena goes to the walk) or
    "levels"."""
    if nested:
        cw = O.count_walk_flags(fields, rows, offs, n)
        if engine == "walk" and cw:                  # the walk's prepare reports these
            return "oob" if cw & O.ERR_OOB else "map" if cw & O.ERR_MAP else "budget"
        if cw & O.ERR_BUDGET:
            return "any"
        if engine == "bfs" and cw:                   # the tile BFS count pass: the same checks
            return "oob" if cw & O.ERR_OOB else "map"
    flags, cols = O.decode_checked(fields, rows, offs, n)
    if flags:
        return "oob" if flags & O.ERR_OOB else "map"
    return cols


@pytest.mark.parametrize("seed", list(range(24)))
def test_corrupt_rows_random_schemas(oracle, dev, seed):
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, IndexOutOfBoundsException, UnsupportedOperationException
    from oracle import oracle as O
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
    levels, counted = _shape(fields)
    L = N.lib()
    old = L.fury_get_tuning(b"nested_decode")
    old_gk = L.fury_get_tuning(b"walk_group_k")
    old_gmin = L.fury_get_tuning(b"walk_group_min")
    seen = []
    try:
        for trial in range(3):
            bad = rows.copy()
            if len(bad):
                pos = rng.integers(0, len(bad), int(rng.integers(1, 40)))
                bad[pos] = rng.integers(0, 256, len(pos)).astype(np.uint8)
            # 21: the row walk in field groups of one counted slot (walk_group_k 1)
            for mode in ((4, 3, 2, 21, 1) if enc.nested else (3,)):
                L.fury_set_tuning(b"walk_group_k", 1 if mode == 21 else old_gk)
                L.fury_set_tuning(b"walk_group_min", 0 if mode == 21 else old_gmin)
                L.fury_set_tuning(b"nested_decode", 2 if mode == 21 else mode)
                walkable = levels <= 5 and counted <= 256
                engine = ("bfs" if mode == 4 or (mode == 3 and not walkable)
                          else "walk" if mode in (2, 3, 21) and walkable else "levels")
                walk = engine != "levels" and walkable
                want = _expected(O, fields, enc.nested, engine, bad, offs, n)
                try:
                    got = _decode(enc, _batch(enc, bad, offs, n, dev))
                    err = None
                except IndexOutOfBoundsException:
                    err = "oob"
                except UnsupportedOperationException as e:
                    err = "budget" if "decode budget" in str(e) else "map"
                where = f"trial {trial}, engine {engine}"
                seen.append(err or "decoded")
                if want == "any" or (err == "budget" and not walk):
                    # the level engine's own bound (elements of a node vs the batch's bytes) is
                    # checked level by level and may pre-empt errors in deeper levels
                    continue
                if isinstance(want, str):
                    assert err == want, f"{where}: oracle says {want}, device {err or 'decoded'}"
                elif err is not None:
                    raise AssertionError(f"{where}: oracle decodes, device raises {err}")
                else:
                    assert_columns_equal(fields, got, want, n)
        L.fury_set_tuning(b"nested_decode", 3)
        assert_columns_equal(fields, _decode(enc, _batch(enc, rows, offs, n, dev)), ref, n)
    finally:
        L.fury_set_tuning(b"nested_decode", old)
        L.fury_set_tuning(b"walk_group_k", old_gk)
        L.fury_set_tuning(b"walk_group_min", old_gmin)
    print(f"seed {seed}: {seen}")


@pytest.mark.parametrize("seed", list(range(8)))
def test_corrupt_rows_wide_flat_engines(oracle, dev, seed):
    """Corrupted rows of 17-40-field flat schemas through the plan decode's two engines (round 6,
    tuning wide_engine): the wide tiles (1) must give the oracle's flat outcome, the row walk (2)
    the oracle's walk outcome (its count pass and item budget restated) -- the same exceptions or
    the same columns."""
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders, IndexOutOfBoundsException, UnsupportedOperationException
    from fury_amd.workloads import gen_columns
    from oracle import oracle as O
    from tests.test_bounds import _batch
    from tests.test_device import _wide_fields
    from fury_amd.encoder import column_to_host
    rng = np.random.default_rng(11000 + seed)
    fields = _wide_fields(int(rng.integers(17, 41)))
    n = int(rng.integers(50, 500))
    host = gen_columns("wide", fields, n, seed=seed, null_pct=10, str_max=40, list_max=8,
                       list_null_pct=10, elem_null_pct=10)
    enc = Encoders.bean(fields, device=dev)
    rows, offs = oracle.encode(fields, host, n)
    offs = np.asarray(offs, np.int64).copy()
    L = N.lib()
    old = L.fury_get_tuning(b"wide_engine")
    seen = []
    try:
        for trial in range(3):
            bad = rows.copy()
            pos = rng.integers(0, len(bad), int(rng.integers(1, 30)))
            bad[pos] = rng.integers(0, 256, len(pos)).astype(np.uint8)
            for engine in (1, 2):
                assert L.fury_set_tuning(b"wide_engine", engine) == 0
                want = _expected(O, fields, engine == 2, "walk" if engine == 2 else "levels",
                                 bad, offs, n)
                try:
                    got = [column_to_host(c) for c in enc.decode_batch(_batch(enc, bad, offs, n, dev))]
                    enc.device_status()
                    err = None
                except IndexOutOfBoundsException:
                    err = "oob"
                except UnsupportedOperationException as e:
                    err = "budget" if "decode budget" in str(e) else "map"
                where = f"trial {trial}, engine {engine}"
                seen.append(f"{engine}:{err or 'decoded'}")
                if isinstance(want, str):
                    assert err == want, f"{where}: oracle says {want}, device {err or 'decoded'}"
                else:
                    assert err is None, f"{where}: oracle decodes, device raises {err}"
                    assert_columns_equal(fields, got, want, n)
    finally:
        L.fury_set_tuning(b"wide_engine", old)
    print(f"seed {seed}: {len(fields)} fields, {seen}")
