"""Pins the CPU oracle (oracle/row_oracle.c + oracle/bean_oracle.py) against the reference's own
known answers and reference-produced schema hashes (tests/golden/), and cross-checks the two
independent restatements against each other.  CPU only."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from fury_amd import types as T
from fury_amd.workloads import SCHEMAS, docs_struct_values, gen_columns
from oracle import bean_oracle as B
from tests.helpers import assert_columns_equal, columns_to_beans

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _known():
    return json.load(open(os.path.join(GOLDEN, "known_answers.json")))


def test_schema_hash_matches_reference_infer_py(oracle):
    """DataTypes.computeSchemaHash restatement == the reference's own infer.py output."""
    d = json.load(open(os.path.join(GOLDEN, "schema_hashes.json")))
    assert d["schemas"], "no golden schemas"
    for name, rec in d["schemas"].items():
        fields = T.schema_from_spec(rec["fields"])
        assert oracle.schema_hash(fields) == rec["hash"], name
        assert T.schema_spec(SCHEMAS[name]) == rec["fields"], name


def test_schema_hash_overflow_shift(oracle):
    """computeHash's ArithmeticException path (h >>= 2 then retry) is exercised by wide schemas:
    the docs Struct hash is the reference's value (checked above) and must be positive."""
    h = oracle.schema_hash(SCHEMAS["docs_struct"])
    assert h == 2926194988097786773


def test_bar_row_bytes_known_answer(oracle):
    fields = SCHEMAS["bar"]
    from fury_amd.workloads import Column
    cols = [Column(values=np.array([1], np.int32)),
            Column(values=np.frombuffer(b"str", np.uint8).copy(),
                   offsets=np.array([0, 3], np.int32))]
    rows, offs = oracle.encode(fields, cols, 1)
    assert rows.tobytes().hex() == _known()["bar_row_hex"]["value"]
    assert B.encode_row(fields, {"f1": 1, "f2": "str"}).hex() == _known()["bar_row_hex"]["value"]


def test_array_encoder_list_bar_224():
    """ArrayEncoderTest.testListEncoder: encode(5 bars).length == 224 (8 + array bytes, see
    SURVEY §7 trap 5: ArrayEncoder.encode returns getBytes(0, 8 + size))."""
    elem = T.struct_field("item", SCHEMAS["bar"])
    bars = [{"f1": k, "f2": f"i{k}"} for k in range(5)]
    assert 8 + len(B.encode_array(elem, bars)) == _known()["array_encoder_list_bar_bytes"]["value"]


def test_array_encoder_nested_1576():
    bar = T.struct_field("item", SCHEMAS["bar"])
    l1 = T.Field("item", T.LIST, True, (bar,))
    l2 = T.Field("item", T.LIST, True, (l1,))
    vals = [[[{"f1": k, "f2": f"s{k}"} for k in range(3)] for _ in range(i)] for i in range(5)]
    n = 8 + len(B.encode_array(l2, vals))
    assert n == _known()["array_encoder_nested_list_bar_bytes"]["value"]


def test_array_encoder_list_list_map_10824():
    bar = T.struct_field("item", SCHEMAS["bar"])
    foo = SCHEMAS["foo"]
    key = T.Field("key", T.STRUCT, False, tuple(foo))
    value = T.Field("value", T.LIST, True, (bar,))
    m = T.Field("item", T.MAP, True, (key, value))
    l1 = T.Field("item", T.LIST, True, (m,))
    foo_val = {"f1": 2, "f2": "str", "f3": ["a", "b", "c"], "f4": [("k1", 1), ("k2", 2)],
               "f5": {"f1": 1, "f2": "str"}}
    vals = [[[(foo_val, [{"f1": j, "f2": f"x{j}"}])] for j in range(3)] for _ in range(10)]
    n = 8 + len(B.encode_array(l1, vals))
    assert n == _known()["array_encoder_list_list_map_bytes"]["value"]


def test_cpp_row_to_string_known_answer():
    """cpp/fury/row/row_test.cc:96-98 (C++ sibling, same wire format)."""
    fields = [T.field("f1", T.STRING), T.field("f2", T.INT32),
              T.array_field("f3", T.INT32),
              T.map_field("f4", T.field("key", T.STRING), T.field("value", T.FLOAT32)),
              T.struct_field("f5", [T.field("n1", T.STRING), T.field("n2", T.INT32)])]
    row = B.encode_row(fields, {"f1": "str", "f2": 1, "f3": [2, 2],
                                "f4": [("key1", 1.0), ("key2", 1.0)],
                                "f5": {"n1": "str", "n2": 1}})
    assert B.row_to_string(fields, row) == _known()["cpp_row_to_string"]["value"]


def test_docs_struct_848(oracle):
    fields = SCHEMAS["docs_struct"]
    rows, offs = oracle.encode(fields, docs_struct_values(fields), 1)
    assert len(rows) + 8 == _known()["docs_struct_encode_bytes"]["value"]
    assert [f.name for f in fields][:8] == ["f0", "f1", "f10", "f100", "f101", "f102", "f103",
                                            "f11"]


@pytest.mark.parametrize("name,n", [("bar", 40), ("beanb", 60), ("mixed", 200), ("nested", 200),
                                    ("narrow", 150), ("struct100", 20)])
def test_columnar_oracle_matches_bean_oracle(oracle, name, n):
    """Two independent restatements (columnar C / value-level Python) give identical bytes."""
    fields = SCHEMAS[name]
    cols = gen_columns(name, fields, n, seed=99)
    rows, offs = oracle.encode(fields, cols, n)
    beans = columns_to_beans(fields, cols, n)
    for i, bean in enumerate(beans):
        want = B.encode_row(fields, bean)
        got = rows[offs[i]:offs[i + 1]].tobytes()
        assert got == want, f"{name} row {i}"


@pytest.mark.parametrize("name,n", [("mixed", 300), ("nested", 300), ("narrow", 200),
                                    ("struct100", 50), ("beanb", 80)])
def test_oracle_roundtrip(oracle, name, n):
    fields = SCHEMAS[name]
    cols = gen_columns(name, fields, n, seed=5)
    rows, offs = oracle.encode(fields, cols, n)
    dec = oracle.decode(fields, rows, offs, n)
    assert_columns_equal(fields, dec, cols, n)


def test_foo_struct_and_map_roundtrip(oracle):
    """Nested bean + map + list<string> through the columnar oracle vs the value oracle."""
    fields = SCHEMAS["foo"]
    bean = {"f1": 2, "f2": "str", "f3": ["a", "b", "c"], "f4": [("k1", 1), ("k2", 2)],
            "f5": {"f1": 1, "f2": "str"}}
    row = B.encode_row(fields, bean)
    assert B.read_row(row, 0, fields) == bean
    from fury_amd.workloads import Column
    cols = [
        Column(values=np.array([2], np.int32)),
        Column(values=np.frombuffer(b"str", np.uint8).copy(), offsets=np.array([0, 3], np.int32)),
        Column(offsets=np.array([0, 3], np.int32),
               child=[Column(values=np.frombuffer(b"abc", np.uint8).copy(),
                             offsets=np.array([0, 1, 2, 3], np.int32))]),
        Column(offsets=np.array([0, 2], np.int32),
               child=[Column(values=np.frombuffer(b"k1k2", np.uint8).copy(),
                             offsets=np.array([0, 2, 4], np.int32)),
                      Column(values=np.array([1, 2], np.int32))]),
        Column(child=[Column(values=np.array([1], np.int32)),
                      Column(values=np.frombuffer(b"str", np.uint8).copy(),
                             offsets=np.array([0, 3], np.int32))]),
    ]
    rows, offs = oracle.encode(fields, cols, 1)
    assert rows.tobytes() == row


def test_encode_reuse_differs_only_in_null_slots(oracle):
    """RowEncoder.encode(obj) reuses one buffer (Encoders.java:146,191-198): a null slot keeps the
    previous row's slot bytes.  Canonical (toRow) bytes zero it.  Everything else is equal."""
    fields = SCHEMAS["mixed"]
    n = 200
    cols = gen_columns("mixed", fields, n, seed=11)
    fresh, offs = oracle.encode(fields, cols, n)
    reused, offs2 = oracle.encode(fields, cols, n, reuse=True)
    assert np.array_equal(offs, offs2)
    diff_rows = 0
    for i in range(n):
        a = fresh[offs[i]:offs[i + 1]]
        b = reused[offs[i]:offs[i + 1]]
        if a.tobytes() != b.tobytes():
            diff_rows += 1
            nb = T.bitmap_bytes(len(fields))
            for k in range(len(fields)):
                s = slice(nb + 8 * k, nb + 8 * k + 8)
                if a[s].tobytes() != b[s].tobytes():
                    assert (a[k >> 3] >> (k & 7)) & 1, "only null slots may differ"
                    assert not a[s].any()
    assert diff_rows > 0


@pytest.mark.parametrize("name", ["struct100", "mixed", "nested", "narrow", "docs_struct"])
def test_golden_fixture_regression(oracle, name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    fields = SCHEMAS[name]
    if name == "docs_struct":
        cols, n = docs_struct_values(fields), 1
    else:
        n = len(d["row_offsets"]) - 1
        cols = gen_columns(name, fields, n, seed=1234)
    rows, offs = oracle.encode(fields, cols, n)
    assert np.array_equal(offs, d["row_offsets"])
    assert np.array_equal(rows, d["rows"])


def test_map_encoder_restatement_round_trips(oracle):
    """MapEncoderTest-shaped maps through the bean restatement of MapEncoderBuilder: toMap bytes
    decode back (BinaryMap.pointTo), and equal the MAP field's bytes inside a row written by the
    columnar C restatement (a top-level BinaryMap is laid out exactly as a map in a row's variable
    section: row = [bitmap 8][slot 8][map])."""
    from fury_amd.beans import beans_to_columns
    bar = T.struct_field("value", SCHEMAS["bar"])
    key = T.field("key", T.STRING)
    pairs = [(f"i{k}", {"f1": k, "f2": f"i{k}"}) for k in range(5)]
    data = B.encode_map(key, bar, pairs)
    assert B.decode_map(key, bar, data) == pairs
    lbar = T.Field("value", T.LIST, True, (T.Field("item", T.LIST, True,
                                                   (T.struct_field("item", SCHEMAS["bar"]),)),))
    nested = [(str(i), [[{"f1": k, "f2": f"s{k}"} for k in range(3)] for _ in range(i)])
              for i in range(5)]
    for kf, vf, v in ((key, bar, pairs), (key, lbar, nested)):
        m = T.Field("m", T.MAP, True, (kf, vf))
        rows, offs = oracle.encode([m], beans_to_columns([m], [{"m": v}]), 1)
        assert rows[16:offs[1]].tobytes() == B.encode_map(kf, vf, v)


def test_array_encoder_restatement_matches_row_restatement(oracle):
    """Top-level BinaryArray bytes (bean restatement of ArrayEncoderBuilder) == the LIST field's
    bytes inside a row (columnar C restatement), for lists of beans, strings, lists and maps."""
    from fury_amd.beans import beans_to_columns
    bar = T.struct_field("item", SCHEMAS["bar"])
    cases = [
        (bar, [{"f1": k, "f2": f"i{k}"} for k in range(5)]),
        (T.field("item", T.STRING), ["a", None, "bcdefghij", ""]),
        (T.Field("item", T.LIST, True, (T.field("item", T.INT32),)), [[1, 2], None, [], [3]]),
        (T.map_field("item", T.field("key", T.STRING), T.field("value", T.INT64)),
         [[("x", 1), ("yy", None)], []]),
    ]
    for elem, vals in cases:
        lf = T.Field("l", T.LIST, True, (elem,))
        rows, offs = oracle.encode([lf], beans_to_columns([lf], [{"l": vals}]), 1)
        got = B.encode_array(elem, vals)
        assert rows[16:offs[1]].tobytes() == got
        assert B.decode_array(elem, got) == vals


def test_null_struct_chain_decode(oracle):
    """A null struct appends a null entry to EVERY descendant (StructWriter.appendNull,
    ArrowWriter.java:577-584, recursive through child StructWriters): decode of struct-in-struct
    chains with strings / binary / decimal / lists under them equals the Arrow columns built from
    the beans."""
    from tests.test_device import _engine_schemas, _random_value
    from fury_amd.beans import beans_to_columns
    for name in ("struct_chain", "nested7", "maps"):
        fields = _engine_schemas()[name]
        rng = np.random.default_rng(3)
        n = 400
        beans = [{f.name: _random_value(f, rng) for f in fields} for _ in range(n)]
        cols = beans_to_columns(fields, beans)
        rows, offs = oracle.encode(fields, cols, n)
        assert_columns_equal(fields, oracle.decode(fields, rows, offs, n), cols, n)


def test_oracle_decode_bounds_rule():
    """The oracle's decode checks every container against the batch as the reference's
    MemoryBuffer does (row_oracle.c header): a STRING slot past the end, a negative element
    count, a struct header past the end and map arrays of different lengths are each reported
    (ERR_OOB / ERR_MAP) instead of read; the intact batch decodes with no flag."""
    from oracle import oracle as O
    from fury_amd import types as T
    from fury_amd.beans import beans_to_columns
    inner = [T.field("a", T.INT32), T.field("s", T.STRING)]
    fields = [T.field("s", T.STRING), T.array_field("l", T.INT64), T.struct_field("st", inner),
              T.map_field("m", T.field("key", T.STRING), T.field("value", T.INT32))]
    beans = [{"s": "hello", "l": [1, 2, 3], "st": {"a": 1, "s": "x"}, "m": [("k", 1), ("j", 2)]}
             for _ in range(3)]
    host = beans_to_columns(fields, beans)
    rows, offs = O.encode(fields, host, 3)
    flags, cols = O.decode_checked(fields, rows, offs, 3)
    assert flags == 0 and cols is not None
    assert O.count_walk_flags(fields, rows, offs, 3) == 0
    hb, last = 8, int(offs[2])
    total = int(offs[3])

    def slot(k):
        return last + hb + 8 * k

    def put(buf, at, v):
        buf[at:at + 8] = np.frombuffer(np.int64(v).tobytes(), np.uint8)

    def word(buf, at):
        return int(np.frombuffer(buf[at:at + 8].tobytes(), np.int64)[0])

    # STRING payload past the batch
    bad = rows.copy()
    put(bad, slot(0), ((total - last) << 32) | 16)
    assert O.decode_checked(fields, bad, offs, 3)[0] == O.ERR_OOB
    # negative element count of the list
    bad = rows.copy()
    arr = last + (word(rows, slot(1)) >> 32)
    put(bad, arr, -2)
    assert O.decode_checked(fields, bad, offs, 3)[0] == O.ERR_OOB
    assert O.count_walk_flags(fields, bad, offs, 3) == O.ERR_OOB
    # struct header straddling the end of the batch
    bad = rows.copy()
    put(bad, slot(2), ((total - 8 - last) << 32) | 24)
    assert O.decode_checked(fields, bad, offs, 3)[0] == O.ERR_OOB
    # map: the value array claims one element fewer than the key array
    bad = rows.copy()
    mp = last + (word(rows, slot(3)) >> 32)
    vals = mp + 8 + word(rows, mp)
    put(bad, vals, 1)
    assert O.decode_checked(fields, bad, offs, 3)[0] == O.ERR_MAP
    assert O.count_walk_flags(fields, bad, offs, 3) == O.ERR_MAP


def test_oracle_count_walk_budget():
    """The row walk's item budget, restated (fo_count_walk): a list of lists whose inner slots all
    alias one long inner array visits m x k items from a row of far fewer bytes -> ERR_BUDGET; the
    full decode (no budget) of the same rows still succeeds."""
    from oracle import oracle as O
    from fury_amd import types as T
    from fury_amd.beans import beans_to_columns
    fields = [T.Field("ll", T.LIST, True, (T.Field("item", T.LIST, True, (T.field("item", T.INT64),)),))]
    beans = [{"ll": [list(range(60)), [1]]}]
    host = beans_to_columns(fields, beans)
    rows, offs = O.encode(fields, host, 1)
    assert O.count_walk_flags(fields, rows, offs, 1) == 0
    # outer array at rel offset from the row's slot; element 1's slot -> element 0's inner array
    outer = int(np.frombuffer(rows[8:16].tobytes(), np.int64)[0]) >> 32   # row-relative
    m = int(np.frombuffer(rows[outer:outer + 8].tobytes(), np.int64)[0])
    assert m == 2
    slots = outer + 8 + 8
    s0 = int(np.frombuffer(rows[slots:slots + 8].tobytes(), np.int64)[0])
    # the outer count raised to 40 elements, all of them pointing at inner array 0 (60 items):
    # the elements' slots must lie inside the row, so reuse the row's own bytes as slots
    bad = np.zeros(len(rows) + 40 * 8 + 64, np.uint8)
    bad[:len(rows)] = rows
    offs2 = np.array([0, len(bad)], np.int64)
    newarr = len(rows)
    bad[newarr:newarr + 8] = np.frombuffer(np.int64(40).tobytes(), np.uint8)
    for j in range(40):
        at = newarr + 8 + 8 + 8 * j
        rel0 = (s0 >> 32) + outer - newarr                  # element slots are array-relative
        bad[at:at + 8] = np.frombuffer(np.int64((rel0 << 32) | (s0 & 0xffffffff)).tobytes(), np.uint8)
    slot = (np.int64(newarr - 0) << 32) | np.int64(8 + 8 + 8 * 40)
    bad[8:16] = np.frombuffer(np.int64(slot).tobytes(), np.uint8)
    assert O.count_walk_flags(fields, bad, offs2, 1) == O.ERR_BUDGET
    flags, cols = O.decode_checked(fields, bad, offs2, 1)
    assert flags == 0 and int(cols[0].offsets[1]) == 40
