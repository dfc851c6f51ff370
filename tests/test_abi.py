"""CPU checks of the C-ABI library: it loads, exports every symbol include/fury_row.h declares
with the signatures the bindings use, and its host-side schema logic (layout, schema hash,
field order, name conversion, argument errors) matches the reference.  No GPU compute."""
from __future__ import annotations

import ctypes
import json
import os
import re
import subprocess

import pytest

from fury_amd import types as T
from fury_amd.workloads import SCHEMAS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fury_row.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(fury_[a-z_0-9]+)\s*\(", src, re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = _declared_functions()
    assert "fury_row_encode" in names and "fury_rows_to_arrow" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from fury_amd import _native as N
    L = N.lib()
    for name in _declared_functions():
        assert hasattr(L, name), f"{name} declared in fury_row.h but not exported"
    assert set(_declared_functions()) == set(N.SIGNATURES), "bindings table out of sync"
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (fury_[a-z_0-9]+)$", out, re.M))
    assert set(_declared_functions()) <= exported


def test_abi_version():
    from fury_amd import _native as N
    assert N.lib().fury_abi_version() == 1


def test_type_width_matches_datatypes():
    from fury_amd import _native as N
    for tid in (T.BOOL, T.INT8, T.INT16, T.INT32, T.INT64, T.FLOAT32, T.FLOAT64, T.DATE32,
                T.TIMESTAMP, T.STRING, T.BINARY, T.DECIMAL, T.LIST, T.STRUCT, T.MAP):
        assert N.lib().fury_type_width(tid) == T.type_width(tid)


def test_schema_layout_and_hash_match_golden():
    from fury_amd.encoder import Schema
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "schema_hashes.json")))
    for name, rec in d["schemas"].items():
        s = Schema(T.schema_from_spec(rec["fields"]))
        assert s.schema_hash == rec["hash"], name
        assert s.fixed_size == T.fixed_size(s.fields)
        assert s.is_fixed == T.is_fixed_schema(s.fields)
    s = Schema(SCHEMAS["struct100"])
    assert (s.bitmap_bytes, s.fixed_size, s.num_fields) == (16, 816, 100)
    s = Schema(SCHEMAS["docs_struct"])
    assert s.fixed_size == 848


def test_sort_bean_fields_like_descriptor():
    from fury_amd import _native as N
    names = [f"f{i}" for i in range(104)] + ["beanB", "b", "Z", "élan", "a\U0001F600", "a￿"]
    arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
    order = (ctypes.c_int32 * len(names))()
    assert N.lib().fury_sort_bean_fields(arr, len(names), order) == 0
    got = [names[i] for i in order]
    # String.compareTo = UTF-16 code-unit order (surrogate pair D83D < FFFF)
    assert got == sorted(names, key=lambda s: s.encode("utf-16-be"))
    assert got[:3] == ["Z", "a\U0001F600", "a￿"]
    assert [f.name for f in T.infer_bean_schema([(n, T.field(n, T.INT32)) for n in
                                                 ("intList", "f1", "intArr")])] == \
        ["f1", "int_arr", "int_list"]


@pytest.mark.parametrize("src,want", [("doubleList", "double_list"), ("f1", "f1"),
                                      ("beanBIterable", "bean_b_iterable"),
                                      ("stringBeanBMap", "string_bean_b_map"), ("ABC", "_a_b_c")])
def test_lower_camel_to_lower_underscore(src, want):
    from fury_amd import _native as N
    out = ctypes.create_string_buffer(2 * len(src) + 1)
    n = N.lib().fury_lower_camel_to_lower_underscore(src.encode(), out, len(out))
    assert out.value.decode() == want and n == len(want)
    assert T.lower_camel_to_lower_underscore(src) == want


def test_schema_create_errors():
    from fury_amd.encoder import IllegalArgumentException, Schema, UnsupportedOperationException
    with pytest.raises(UnsupportedOperationException):
        Schema([T.Field("x", 99)])
    with pytest.raises(IllegalArgumentException):
        Schema([T.Field("l", T.LIST, True, ())])       # list without element field


def test_device_calls_reject_bad_arguments_without_touching_gpu():
    """Argument validation happens on the host before any HIP call."""
    from fury_amd import _native as N
    from fury_amd.encoder import Schema, UnsupportedOperationException
    L = N.lib()
    assert L.fury_row_encode(None, None, 1, None, None, None) == 1
    s = Schema(SCHEMAS["foo"])       # nested struct + map: generic engine; rows is null
    cols = (N.FuryColumn * 5)()
    assert L.fury_row_encode(s.handle, cols, 1, None, None, None) == 1
    deep = T.field("x", T.INT32)
    for d in range(9):               # 10 levels of nesting: the row walk's explicit stack
        deep = T.struct_field(f"s{d}", [deep])
    assert L.fury_row_encode(Schema([deep]).handle, cols, 1, None, None, None) == 1  # rows null
    for d in range(9, 70):           # 71 levels: beyond the schema limit (64)
        deep = T.struct_field(f"s{d}", [deep])
    with pytest.raises(UnsupportedOperationException):
        Schema([deep])
    wide = [T.struct_field(f"w{i}", [T.field("a", T.INT32), T.field("b", T.INT64)])
            for i in range(100)]     # > 256 nodes and 10 levels deep: the row walk (round 5;
    deep = T.field("x", T.INT32)     # round 4 refused it: no engine took both)
    for d in range(9):
        deep = T.struct_field(f"s{d}", [deep])
    assert L.fury_row_encode(Schema(wide + [deep]).handle, cols, 1, None, None, None) == 1  # rows null
    assert "rows is null" in N.last_error()
    assert L.fury_schema_num_nodes(s.handle) == 5 + 1 + 2 + 2
    s2 = Schema(SCHEMAS["struct100"])
    cols2 = (N.FuryColumn * 100)()
    assert L.fury_row_encode(s2.handle, cols2, 4, None, None, None) == 1   # rows is null
    assert L.fury_row_encode(s2.handle, cols2, -1, None, None, None) == 1  # nrows < 0


def test_new_entry_points_reject_bad_arguments_without_touching_gpu():
    """IPC, host-memory path, framing and tuning: argument errors are reported on the host
    (status codes = the reference's exception types) before any HIP call."""
    from fury_amd import _native as N
    from fury_amd.encoder import Schema
    L = N.lib()
    n = ctypes.c_int64(0)
    s = Schema(SCHEMAS["struct100"])
    cols = (N.FuryColumn * 100)()
    # Arrow IPC
    assert L.fury_arrow_ipc_schema(None, None, 0, ctypes.byref(n)) == 1
    assert L.fury_arrow_ipc_schema(s.handle, None, 0, None) == 1
    assert L.fury_arrow_ipc_schema(s.handle, None, 0, ctypes.byref(n)) == 0 and n.value > 0
    small = ctypes.create_string_buffer(8)
    assert L.fury_arrow_ipc_schema(s.handle, small, 8, ctypes.byref(n)) == 7      # CAPACITY
    assert L.fury_arrow_ipc_record_batch(None, cols, 1, None, 0, ctypes.byref(n), None) == 1
    assert L.fury_arrow_ipc_record_batch(s.handle, cols, -1, None, 0, ctypes.byref(n), None) == 1
    assert L.fury_arrow_ipc_record_batch(s.handle, None, 1, None, 0, ctypes.byref(n), None) == 1
    # host-memory path
    nb = ctypes.c_int64(0)
    assert L.fury_row_encode_host(None, cols, 1, None, 0, None, ctypes.byref(nb), 0) == 1
    assert L.fury_row_encode_host(s.handle, cols, -1, None, 0, None, ctypes.byref(nb), 0) == 1
    assert L.fury_row_encode_host(s.handle, cols, 10, None, 100, None, ctypes.byref(nb), 0) == 7
    assert nb.value == 10 * 816                                   # bytes the rows need
    m = Schema(SCHEMAS["mixed"])
    mcols = (N.FuryColumn * 6)()
    assert L.fury_row_encode_host(m.handle, mcols, 3, None, 0, None, ctypes.byref(nb), 0) == 1
    assert L.fury_row_decode_host(None, None, None, 1, cols, 0) == 1
    assert L.fury_row_decode_host(s.handle, None, None, 1, cols, 0) == 1       # rows null
    assert L.fury_row_decode_host(m.handle, small, None, 1, mcols, 0) == 1     # offsets null
    assert L.fury_row_decode_host(s.handle, None, None, 0, cols, 0) == 0       # empty batch
    assert L.fury_host_register(None, 16) == 1 and L.fury_host_unregister(None) == 1
    # framing
    assert L.fury_frame_rows(None, None, None, 1, None, None, None) == 1
    assert L.fury_frame_rows(m.handle, small, None, 1, small, None, None) == 1  # offsets null
    assert L.fury_unframe_rows(s.handle, None, 10, 1, None, None, None) == 1
    assert L.fury_unframe_rows(s.handle, None, -1, 1, None, None, None) == 1
    # tuning knobs: range checks, unknown keys
    assert L.fury_set_tuning(b"lookback_help", 2) == 1
    assert L.fury_set_tuning(b"unframe", 2) == 1
    assert L.fury_set_tuning(b"no_such_knob", 0) == 1
    # the measured-slower kernel variants were removed in round 3: their keys are unknown now
    assert L.fury_set_tuning(b"fixed_variant", 54) == 1
    assert L.fury_set_tuning(b"var_decode", 0) == 1
    assert L.fury_set_tuning(b"gen_decode", 0) == 1
    assert L.fury_get_tuning(b"no_such_knob") == -1
    assert L.fury_get_tuning(b"lookback_help") == 0


def test_host_decode_empty_batch_writes_arrow_offsets():
    """fury_row_decode_host with nrows = 0 (the JNI path) leaves valid Arrow offsets
    (offsets[0] = 0) in every top-level column that has an offsets buffer, like the device
    decode; it touches no GPU."""
    import numpy as np
    from fury_amd import _native as N
    from fury_amd.encoder import Schema
    L = N.lib()
    m = Schema(SCHEMAS["mixed"])
    cols = (N.FuryColumn * 6)()
    offs = [np.full(4, 77, np.int32) for _ in range(6)]
    for k in range(3, 6):                      # s1..s3: STRING
        cols[k].offsets = offs[k].ctypes.data
    assert L.fury_row_decode_host(m.handle, None, None, 0, cols, 0) == 0
    for k in range(3, 6):
        assert offs[k][0] == 0 and offs[k][1] == 77


def test_collection_schema_create():
    """fury_collection_schema_create: LIST -> ArrayEncoder, MAP -> MapEncoder schemas (no hash,
    no row header); anything else is an IllegalArgumentException; row framing is refused."""
    from fury_amd import _native as N
    from fury_amd.encoder import IllegalArgumentException, Schema
    s = Schema([T.Field("v", T.LIST, True, (T.struct_field("item", SCHEMAS["bar"]),))],
               collection=True)
    assert (s.schema_hash, s.fixed_size, s.is_fixed, s.num_fields) == (0, 0, False, 1)
    m = Schema([T.map_field("v", T.field("key", T.STRING), T.field("value", T.INT32))],
               collection=True)
    assert m.schema_hash == 0
    with pytest.raises(IllegalArgumentException):
        Schema([T.field("x", T.INT32)], collection=True)
    with pytest.raises(IllegalArgumentException):
        Schema([T.field("x", T.INT32), T.field("y", T.INT32)], collection=True)
    L = N.lib()
    buf = ctypes.create_string_buffer(64)
    assert L.fury_frame_rows(s.handle, buf, buf, 1, buf, buf, None) == 2
    assert L.fury_unframe_rows(m.handle, buf, 64, 1, buf, buf, None) == 2


def test_wide_schemas_accepted():
    """No field limit (RowEncoderBuilder.java:154-217 emits a statement per field for any N): 316+
    fixed-width fields take the column-block kernels, 257+ variable-length fields the generic
    engine; argument errors are still reported on the host."""
    import numpy as np
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders, Schema
    L = N.lib()
    buf = np.zeros(64, np.uint64)
    for n, kind in ((400, T.INT64), (300, T.STRING)):
        fields = [T.field(f"f{i:03d}", kind) for i in range(n)]
        s = Schema(fields)
        cols = (N.FuryColumn * n)()
        for k in range(n):
            cols[k].values = buf.ctypes.data
            cols[k].offsets = buf.ctypes.data
        assert L.fury_row_encode(s.handle, cols, 1, buf.ctypes.data, None, None) == 1   # rows null
        assert "rows is null" in N.last_error()
        assert Encoders.bean(fields, device="cpu").nested == (kind == T.STRING)
