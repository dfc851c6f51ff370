"""The nested engines against the oracle: the row-walk decode (walk.hip, tuning "nested_decode" = 2,
the default: the level engine past its limits; 3 takes the tile BFS past them), the tile-BFS decode
(bfs.hip, 4) and the level engine (levels.hip, 1) on the same rows, and the
row-walk encode (rowenc.hip; deep schemas through its explicit-stack continuation): every nested
schema shape the tests know, the reference's BeanA, collections (ArrayEncoder / MapEncoder
batches), schemas nested up to the 64-level limit, and LDS budgets small enough to force rows
read from HBM past the stage.  Marked gpu."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from fury_amd import types as T  # noqa: E402
from fury_amd.workloads import SCHEMAS  # noqa: E402
from tests.helpers import assert_columns_equal  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _tune(key, v):
    from fury_amd import _native as N
    assert N.lib().fury_set_tuning(key.encode(), v) == 0, N.last_error()


@pytest.fixture
def engines():
    """Restores the default engine and LDS budgets after the test."""
    from fury_amd import _native as N
    L = N.lib()
    old = {k: L.fury_get_tuning(k.encode()) for k in ("nested_decode", "walk_threads", "walk_stage", "walk_pool",
                                                       "walk_stage_write", "walk_threads_write",
                                                       "walk_out", "bfs_threads", "bfs_rows",
                                                       "bfs_stage", "bfs_arena", "walk_group_k",
                                                       "walk_group_min")}
    yield
    for k, v in old.items():
        _tune(k, v)


def _groups(gk):
    """Row-walk field groups of about gk counted slots on every schema (None: the defaults --
    groups of 8 slots past 16 slots)."""
    _tune("walk_group_min", 16 if gk is None else 0)
    _tune("walk_group_k", 8 if gk is None else gk)


def _schemas():
    from tests.test_device import _engine_schemas, _nested_fields
    out = dict(_engine_schemas())
    out["beana"] = SCHEMAS["beana"]
    out["nested7"] = _nested_fields()
    out["flat_mixed"] = SCHEMAS["mixed"]
    return out


def _beans(fields, n, seed):
    from tests.test_device import _random_value
    rng = np.random.default_rng(seed)
    return [{f.name: _random_value(f, rng) for f in fields} for _ in range(n)]


def _decode_plan(enc, batch):
    from fury_amd.encoder import column_to_host
    return [column_to_host(c) for c in enc._decode_nested(batch, True, False, None)]


@pytest.mark.parametrize("name", ["nested7", "foo", "deep_lists", "struct_chain", "maps", "beana",
                                  "flat_mixed"])
@pytest.mark.parametrize("budget", ["default", "tiny"])
def test_tree_decode_equals_oracle_and_level_engine(oracle, dev, engines, name, budget):
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_device
    fields = _schemas()[name]
    n = 2999
    beans = _beans(fields, n, len(name) * 31)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    ref = oracle.decode(fields, want, want_offs, n)
    _tune("nested_decode", 1)
    lv = _decode_plan(enc, batch)
    assert_columns_equal(fields, lv, ref, n)
    assert columns_to_beans(fields, lv, n) == beans
    if budget == "tiny":              # row walk: 1 KB stage (rows from HBM), no bitmap windows
        _tune("walk_stage", 1024)
        _tune("walk_stage_write", 2048)
        _tune("walk_pool", 0)
        _tune("walk_threads", 128)
        _tune("walk_threads_write", 128)
    _tune("nested_decode", 2)
    # output windows of the write pass (walk_out bytes): off, too small for most nodes (mixed
    # LDS / HBM stores), the default; write tiles of 512 (default, unstaged) and 256 rows
    legs = ([(128, 0), (128, 256), (128, 16384)] if budget == "tiny"
            else [(512, 0), (512, 40960), (256, 16384)])
    for tw, wo in legs:
        _tune("walk_threads_write", tw)
        _tune("walk_out", wo)
        walk = _decode_plan(enc, batch)
        assert_columns_equal(fields, walk, ref, n)
    # field groups (walk_group_k): a workgroup per (tile, group of top-level fields); 1 = about one
    # counted slot per group, the most groups the schema splits into
    for gk in (1, 2):
        _groups(gk)
        assert_columns_equal(fields, _decode_plan(enc, batch), ref, n)
    _groups(None)
    # tile BFS: threads / tile rows, a stage far smaller than the tile (rows read from HBM), an
    # arena too small for the tile (the batch falls back to the row walk), and the defaults
    from fury_amd import _native as N
    L = N.lib()
    _tune("nested_decode", 4)
    bfs_legs = ([(64, 64, 1024, 0), (256, 200, 2048, 0), (128, 128, 0, 1024)] if budget == "tiny"
                else [(128, 128, 0, 0), (64, 64, 0, 0), (256, 256, 0, 0), (128, 300, 0, 0)])
    for th, tr, stg, arena in bfs_legs:
        _tune("bfs_threads", th)
        _tune("bfs_rows", tr)
        _tune("bfs_stage", stg)
        _tune("bfs_arena", arena)
        fb = L.fury_get_tuning(b"bfs_fallbacks")
        got = _decode_plan(enc, batch)
        assert_columns_equal(fields, got, ref, n)
        if arena == 1024 and name in ("nested7", "deep_lists", "maps"):
            assert L.fury_get_tuning(b"bfs_fallbacks") > fb     # the arena leg really fell back


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 21])
def test_tree_decode_large_batch(oracle, dev, engines, mode):
    """400k depth-3 rows (thousands of tiles, multi-chunk tile scans) == the oracle's decode, level
    engine (1), row walk (2), row walk in field groups of one counted slot (21) and tile BFS (4)."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    from tests.test_device import _nested_beans, _nested_fields
    fields = _nested_fields()
    base = _nested_beans(20_000, seed=5)
    n = 400_000
    host = beans_to_columns(fields, (base * (n // len(base) + 1))[:n])
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    if mode == 21:                             # the row walk in field groups of one counted slot
        _groups(1)
    _tune("nested_decode", 2 if mode == 21 else mode)
    got = _decode_plan(enc, batch)
    assert_columns_equal(fields, got, oracle.decode(fields, want, want_offs, n), n)


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("kind", ["list_bar", "list_long", "list_str", "list_list", "map"])
def test_collections_both_engines(oracle, dev, engines, mode, kind):
    """ArrayEncoder / MapEncoder batches (root 1 / 2: each entry a top-level BinaryArray /
    BinaryMap) through the level engine (mode 1) and the row walk (mode 2)."""
    from tests.test_device import test_array_encoder_batch_vs_oracle, test_map_encoder_batch_vs_oracle
    _tune("nested_decode", mode)
    if kind == "map":
        test_map_encoder_batch_vs_oracle(oracle, dev)
    else:
        test_array_encoder_batch_vs_oracle(oracle, dev, kind)


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 21])
def test_tree_decode_skewed_rows(oracle, dev, engines, mode):
    """Tiles whose bytes exceed the stage (rows of very different sizes): the rows past the stage
    are read from HBM, the result is the oracle's."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = [T.field("a", T.INT32), T.array_field("l", T.STRING),
              T.struct_field("s", [T.field("x", T.INT64), T.array_field("y", T.INT16)])]
    rng = np.random.default_rng(9)
    beans = []
    for i in range(5000):
        big = i % 97 == 3
        k = int(rng.integers(200, 400)) if big else int(rng.integers(0, 3))
        beans.append({"a": i, "l": ["x" * int(rng.integers(0, 40)) for _ in range(k)],
                      "s": None if i % 11 == 5 else {"x": i * 3, "y": list(range(k % 50))}})
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    n = len(beans)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    if mode == 21:                             # the row walk in field groups of one counted slot
        _groups(1)
    _tune("nested_decode", 2 if mode == 21 else mode)
    got = _decode_plan(enc, batch)
    assert_columns_equal(fields, got, oracle.decode(fields, want, want_offs, n), n)


@pytest.fixture
def enc_engines():
    from fury_amd import _native as N
    L = N.lib()
    old = {k: L.fury_get_tuning(k.encode()) for k in ("rowenc_rows", "rowenc_img", "rowenc_tile")}
    yield
    for k, v in old.items():
        _tune(k, v)


def _encode_both_ways(oracle, dev, enc, dcols, host, fields, n):
    """encode_batch (measure + encode) and encode_measured_into == the oracle's bytes / offsets."""
    want, want_offs = oracle.encode(fields, host, n)
    b = enc.encode_batch(dcols, n)
    assert np.array_equal(b.row_offsets.cpu().numpy(), want_offs)
    assert np.array_equal(b.rows.cpu().numpy(), want)
    total = int(want_offs[-1])
    rows = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    enc.encode_measured_into(dcols, n, rows, offs)
    torch.cuda.synchronize()
    assert np.array_equal(rows[:total].cpu().numpy(), want)
    return b, want, want_offs


@pytest.mark.parametrize("name", ["nested7", "foo", "deep_lists", "struct_chain", "maps", "beana"])
@pytest.mark.parametrize("budget", ["default", "small", "tiny"])
def test_tree_encode_equals_oracle(oracle, dev, enc_engines, name, budget):
    """The row-walk nested encode (measure + encode) == the C restatement's bytes and offsets;
    "small" budgets build 128-row tiles in 8 KB chunks, "tiny" ones leave most rows to the
    HBM-direct path (a row alone past the image)."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = _schemas()[name]
    n = 3001
    beans = _beans(fields, n, len(name) * 17 + 5)
    host = beans_to_columns(fields, beans)
    dcols = [column_to_device(c, dev) for c in host]
    enc = Encoders.bean(fields, device=dev)
    if budget == "small":
        _tune("rowenc_rows", 128)
        _tune("rowenc_img", 8192)
    elif budget == "tiny":
        _tune("rowenc_img", 1024)
        _tune("rowenc_tile", 64)
    _encode_both_ways(oracle, dev, enc, dcols, host, fields, n)


@pytest.mark.parametrize("img", [0, 1024])
def test_tree_encode_capacity(oracle, dev, enc_engines, img):
    """encode_measured with a short buffer: offsets complete, no byte at or past the capacity
    written (guard bytes intact), the bytes before it equal to the oracle's; LDS-built rows and
    HBM-direct rows (img = 1024)."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = _schemas()["nested7"]
    n = 2000
    host = beans_to_columns(fields, _beans(fields, n, 77))
    dcols = [column_to_device(c, dev) for c in host]
    enc = Encoders.bean(fields, device=dev)
    want, want_offs = oracle.encode(fields, host, n)
    if img:
        _tune("rowenc_img", img)
    cap = (int(want_offs[n // 2]) + 13) & ~7
    rows = torch.full((cap + 4096,), 0xAB, dtype=torch.uint8, device=dev)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    from fury_amd import _native as N
    from fury_amd.encoder import _c_columns, _ptr, _stream_handle
    keep: list = []
    st = N.lib().fury_row_encode_measured(enc.schema().handle, _c_columns(dcols, keep), n,
                                          _ptr(offs), _ptr(rows), cap, _stream_handle(None))
    assert st == 0, N.last_error()
    torch.cuda.synchronize()
    got = rows.cpu().numpy()
    assert np.array_equal(offs.cpu().numpy(), want_offs)
    assert (got[cap:] == 0xAB).all()
    full = int(np.searchsorted(want_offs, cap, side="right")) - 1
    assert np.array_equal(got[:want_offs[full]], want[:want_offs[full]])


# ---- schemas nested past the inlined walk (depth 9 .. 64) -------------
def _deep_fields(levels):
    """`levels` levels of nesting: a struct chain with a LIST every third level and one MAP, so a
    row stays small (at most ~3 entries per collection)."""
    f = T.field("leaf", T.INT64)
    depth = 1
    d = 0
    while depth < levels:
        if d % 3 == 1:
            f = T.Field(f"l{d}", T.LIST, True, (f,))
            depth += 1
        elif d == 3:
            f = T.map_field(f"m{d}", T.field("k", T.STRING), f)
            depth += 1
        else:
            f = T.struct_field(f"s{d}", [T.field(f"v{d}", T.INT32 if d % 2 else T.STRING), f])
            depth += 1
        d += 1
    return [T.not_null_field("id", T.INT64), f, T.array_field("tail", T.INT16)]


def _schema_levels(fields):
    def lv(f):
        return 1 + max((lv(c) for c in f.children), default=0)
    return max(lv(f) for f in fields)


@pytest.mark.parametrize("levels", [6, 9, 12, 20, 64])
@pytest.mark.parametrize("dec_mode", [1, 2, 3, 4])
def test_deep_schema_round_trip(oracle, dev, engines, enc_engines, levels, dec_mode):
    """Depth 6 .. 64 schemas (64 = the schema limit): the row-walk encode continues past its
    inlined levels on an explicit stack, both decode settings read the rows back (the row walk
    hands schemas past kWalkMaxDepth to the level engine by itself); bytes, offsets and columns ==
    the oracle's."""
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_device
    fields = _deep_fields(levels)
    assert _schema_levels(fields) == levels
    n = 2500 if levels < 64 else 600
    beans = _beans(fields, n, levels * 7 + dec_mode)
    host = beans_to_columns(fields, beans)
    dcols = [column_to_device(c, dev) for c in host]
    enc = Encoders.bean(fields, device=dev)
    assert enc.nested
    b, want, want_offs = _encode_both_ways(oracle, dev, enc, dcols, host, fields, n)
    _tune("nested_decode", dec_mode)
    ref = oracle.decode(fields, want, want_offs, n)
    got = _decode_plan(enc, b)
    assert_columns_equal(fields, got, ref, n)
    assert columns_to_beans(fields, got, n) == beans


@pytest.mark.parametrize("levels", [7, 12])
@pytest.mark.parametrize("img", [0, 2048])
def test_deep_schema_large_rows(oracle, dev, enc_engines, levels, img):
    """Deep rows of several KB (long lists at every LIST level): rows past the LDS image take
    the HBM-direct path of the explicit-stack walk, == the oracle's bytes."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = _deep_fields(levels)
    n = 700 if levels < 12 else 200
    rng = np.random.default_rng(levels + img)

    def big(f):
        if f.type_id == T.LIST:
            return [big(f.children[0]) for _ in range(int(rng.integers(0, 7)))]
        if f.type_id == T.MAP:
            return [(f"k{i}", big(f.children[1])) for i in range(int(rng.integers(0, 4)))]
        if f.type_id == T.STRUCT:
            return {c.name: big(c) for c in f.children}
        if f.type_id == T.STRING:
            return "s" * int(rng.integers(0, 30))
        return int(rng.integers(-1000, 1000))
    beans = [{"id": i, fields[1].name: big(fields[1]), "tail": list(range(i % 20))} for i in range(n)]
    host = beans_to_columns(fields, beans)
    dcols = [column_to_device(c, dev) for c in host]
    enc = Encoders.bean(fields, device=dev)
    if img:
        _tune("rowenc_img", img)
    _, _, want_offs = _encode_both_ways(oracle, dev, enc, dcols, host, fields, n)
    assert int(np.diff(want_offs).max()) > 2048     # some rows past the small image


@pytest.mark.parametrize("levels", [2, 3, 4, 5, 6, 7, 9])
def test_row_walk_encode_depths(oracle, dev, enc_engines, levels):
    """The row-walk encode (rowenc.hip: one inlined instance per depth up to 5 levels, the
    explicit-stack instance past them) == the oracle's bytes and offsets."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = _deep_fields(levels)
    assert _schema_levels(fields) == levels
    n = 2100
    host = beans_to_columns(fields, _beans(fields, n, levels * 11))
    enc = Encoders.bean(fields, device=dev)
    want, want_offs = oracle.encode(fields, host, n)
    b = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    assert np.array_equal(b.row_offsets.cpu().numpy(), want_offs)
    assert np.array_equal(b.rows.cpu().numpy(), want)


@pytest.mark.parametrize("kind", ["list_bar", "list_long", "list_str", "list_list", "map"])
def test_collections_encode(oracle, dev, enc_engines, kind):
    """ArrayEncoder / MapEncoder batches (root 1 / 2) encoded by the row walk == the oracle."""
    from tests.test_device import test_array_encoder_batch_vs_oracle, test_map_encoder_batch_vs_oracle
    if kind == "map":
        test_map_encoder_batch_vs_oracle(oracle, dev)
    else:
        test_array_encoder_batch_vs_oracle(oracle, dev, kind)


@pytest.mark.parametrize("levels", [4, 5, 9])
def test_deep_schema_corrupt_rows(oracle, dev, engines, levels):
    """Rows of a nested schema with random bytes overwritten: the row walk (nested_decode 2, up to
    5 levels; deeper schemas take the level engine either way) and the level engine (1) finish --
    no walk through aliased slots grows without bound (the walk's item budget) -- decode to the
    same columns when both succeed, read nothing outside the batch (bounds checks shared: tcheck)
    and leave no error behind for the intact rows."""
    from fury_amd.encoder import IndexOutOfBoundsException, UnsupportedOperationException
    from fury_amd.encoder import column_to_host
    from tests.test_bounds import _batch, _nested_batch
    fields = _deep_fields(levels)
    n = 600
    enc, rows, offs = _nested_batch(oracle, fields, n, levels, dev)
    rng = np.random.default_rng(levels)
    for trial in range(4):
        bad = rows.copy()
        lo = int(offs[n // 2])
        pos = rng.integers(lo, len(bad), 24)
        bad[pos] = rng.integers(0, 256, len(pos)).astype(np.uint8)
        res = {}
        for mode in (4, 3, 2, 21, 1):          # 21: the row walk in field groups of one slot
            _groups(1 if mode == 21 else None)
            _tune("nested_decode", 2 if mode == 21 else mode)
            try:
                res[mode] = [column_to_host(c) for c in enc.decode_batch(_batch(enc, bad, offs, n, dev))]
            except (IndexOutOfBoundsException, UnsupportedOperationException) as e:
                res[mode] = type(e)
        _groups(None)
        # the grouped walk checks and charges exactly what the one-group walk does
        if isinstance(res[2], type) or isinstance(res[21], type):
            assert res[21] == res[2], (res[2], res[21])
        else:
            assert_columns_equal(fields, res[21], res[2], n)
        # a raise need not agree: the walk reports rows whose aliased slots would make it visit
        # more items than the row has bytes (its item budget), the level engine batches whose
        # elements or payload bytes outnumber the batch's row bytes; two decodes agree
        if not isinstance(res[2], type) and not isinstance(res[1], type):
            assert_columns_equal(fields, res[2], res[1], n)
        for m in (3, 4):
            if not isinstance(res[m], type) and not isinstance(res[1], type):
                assert_columns_equal(fields, res[m], res[1], n)
    _tune("nested_decode", 2)
    good = [column_to_host(c) for c in enc.decode_batch(_batch(enc, rows, offs, n, dev))]
    assert_columns_equal(fields, good, oracle.decode(fields, rows, offs, n), n)


def test_walk_budget_no_false_positive(oracle, dev, engines):
    """Well-formed rows at the edge of the count pass's item budget (2 x a row's bytes + 64):
    thousands of 1-byte list elements, lists of null structs (free) and of empty lists, maps of
    1-byte keys and values -- decoded by the row walk without a report, == the oracle."""
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_device
    S = T.struct_field
    fields = [T.not_null_field("id", T.INT64),
              T.Field("bits", T.LIST, True, (T.not_null_field("item", T.BOOL),)),
              T.Field("nulls", T.LIST, True, (S("item", [T.field(f"x{i:02d}", T.INT32) for i in range(20)]),)),
              T.Field("empties", T.LIST, True, (T.Field("item", T.LIST, True, (T.field("item", T.INT8),)),)),
              T.map_field("m", T.not_null_field("k", T.INT8), T.not_null_field("v", T.INT8))]
    rng = np.random.default_rng(3)
    n = 64
    beans = [{"id": i,
              "bits": [bool(x) for x in rng.integers(0, 2, 3000 + 17 * i)],
              "nulls": [None] * (500 + i),
              "empties": [[] for _ in range(400 + i)],
              "m": [(int(k), int(k) // 2) for k in range(-60, 60)]} for i in range(n)]
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    _tune("nested_decode", 2)
    got = _decode_plan(enc, batch)
    assert_columns_equal(fields, got, oracle.decode(fields, want, want_offs, n), n)
    assert columns_to_beans(fields, got, n) == beans


def test_walk_many_counted_nodes_fits_lds(oracle, dev, engines):
    """A schema at the row walk's counted-node limit (62 STRING fields + a LIST of a STRING struct:
    64 counted nodes): the write pass's per-row cursors (64 x rows) would overflow the LDS at the
    default 512-row tiles, so the plan steps down to 256-row tiles; the decode == the oracle."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = ([T.not_null_field("id", T.INT64)] + [T.field(f"s{i:02d}", T.STRING) for i in range(62)]
              + [T.Field("t", T.LIST, True, (T.struct_field("item", [T.field("x", T.STRING)]),))])
    n = 3000
    beans = _beans(fields, n, 64)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    _tune("nested_decode", 2)
    got = _decode_plan(enc, batch)
    assert_columns_equal(fields, got, oracle.decode(fields, want, want_offs, n), n)


def _random_schema(rng, depth_left, nfields, prefix="f"):
    """Random fields: scalars of every width, STRING / BINARY / DECIMAL, and (while depth_left)
    STRUCT / LIST / MAP of random children."""
    scal = [T.BOOL, T.INT8, T.INT16, T.INT32, T.INT64, T.FLOAT32, T.FLOAT64, T.DATE32,
            T.TIMESTAMP, T.STRING, T.BINARY, T.DECIMAL]
    out = []
    for i in range(nfields):
        name = f"{prefix}{i:02d}"
        kind = int(rng.integers(0, 6)) if depth_left > 0 else 0
        nullable = bool(rng.integers(0, 4))
        if kind <= 2:
            out.append(T.Field(name, scal[int(rng.integers(0, len(scal)))], nullable, ()))
        elif kind == 3:
            out.append(T.Field(name, T.STRUCT, nullable,
                               tuple(_random_schema(rng, depth_left - 1, int(rng.integers(1, 4)), name + "s"))))
        elif kind == 4:
            e = _random_schema(rng, depth_left - 1, 1, name + "e")[0]
            out.append(T.Field(name, T.LIST, nullable, (T.Field("item", e.type_id, e.nullable, e.children),)))
        else:
            k = T.Field("key", [T.INT32, T.STRING, T.INT64][int(rng.integers(0, 3))], False, ())
            v = _random_schema(rng, depth_left - 1, 1, name + "v")[0]
            out.append(T.Field(name, T.MAP, nullable, (k, T.Field("value", v.type_id, v.nullable, v.children))))
    return out


@pytest.mark.parametrize("seed", list(range(40)))
def test_random_nested_schemas(oracle, dev, engines, seed):
    """Random nested schemas (up to 5 levels, every type) with random beans: the device encode ==
    the oracle's bytes, and the row walk and the level engine both decode them to the oracle's
    columns."""
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_device
    rng = np.random.default_rng(1000 + seed)
    fields = _random_schema(rng, int(rng.integers(1, 5)), int(rng.integers(2, 9)))
    n = int(rng.integers(1, 900))
    beans = _beans(fields, n, seed)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    ref = oracle.decode(fields, want, want_offs, n)
    for mode in (4, 3, 2, 21, 1):              # 21: the row walk in field groups of one slot
        _groups(1 if mode == 21 else None)
        _tune("nested_decode", 2 if mode == 21 else mode)
        got = _decode_plan(enc, batch) if enc.nested else None
        if got is None:
            from fury_amd.encoder import column_to_host
            got = [column_to_host(c) for c in enc.decode_batch(batch)]
        assert_columns_equal(fields, got, ref, n)
    assert columns_to_beans(fields, got, n) == beans


@pytest.mark.parametrize("seed", list(range(16)))
def test_random_deep_schemas(oracle, dev, engines, seed):
    """Random schemas nested 6-10 levels (the encode's explicit-stack levels, the level-engine
    decode): bytes and columns == the oracle."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    rng = np.random.default_rng(7000 + seed)
    fields = []
    while not fields or max(_levels(f) for f in fields) < 6:
        fields = _random_schema(rng, int(rng.integers(6, 11)), int(rng.integers(1, 4)))
    n = int(rng.integers(1, 300))
    beans = _beans(fields, n, seed)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    assert_columns_equal(fields, _decode_plan(enc, batch), oracle.decode(fields, want, want_offs, n), n)


def _levels(f):
    return 1 + max((_levels(c) for c in f.children), default=0)


@pytest.mark.parametrize("nstr", [126, 254])
def test_walk_wide_counted_nodes(oracle, dev, engines, nstr):
    """Beans with 128 / 256 counted nodes (STRING fields + a LIST of a STRING struct): round 6 lifts
    the row walk's 64-counted-node limit to 256 and walks such beans in field groups (a workgroup
    per tile and group of top-level fields, walk_group_k slots each: 16 / 32 groups at the default
    8, 32 at 4 -- the cap, reached by doubling the group size --, 8 / 16 at 16, one group at 0), so these
    decode through the walk (nested_decode 2) -- and the tile BFS (4) and the level engine (1) --
    to the oracle's columns."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    fields = ([T.not_null_field("id", T.INT64)] + [T.field(f"s{i:03d}", T.STRING) for i in range(nstr)]
              + [T.Field("t", T.LIST, True, (T.struct_field("item", [T.field("x", T.STRING)]),))])
    n = 1500
    beans = _beans(fields, n, nstr)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    ref = oracle.decode(fields, want, want_offs, n)
    for mode, gk in ((2, 4), (2, 16), (2, 0), (4, 4), (1, 4)):
        _tune("walk_group_k", gk)
        _tune("nested_decode", mode)
        assert_columns_equal(fields, _decode_plan(enc, batch), ref, n)
