"""The JNI-free core of GpuRowEncoder's native methods (fury_jni_*, fury_amd/csrc/jnicore.cpp),
driven with GpuRowEncoder's exact array layouts built here in Python:
  flattenField  -> names + int32 {typeId, nullable, numChildren} per node, pre-order;
  describe()    -> int64 {values, validity, offsets, capacity, numChildren} per node, pre-order;
  counts        -> int64 {entries, payload bytes} per node, breadth-first.
CPU: status -> Java exception class, schema creation (hash equals the Schema's), malformed
descriptors rejected before any device work, and a syntax check of fury_row_jni.cc against a
minimal jni.h declaring only the JNIEnv functions it calls (the image has no JDK).  GPU: Struct-100,
mixed and Foo encoded and decoded through the core equal the oracle."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from fury_amd import _native as N
from fury_amd.types import LIST
from fury_amd.workloads import SCHEMAS, gen_columns
from tests.helpers import assert_columns_equal

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def flatten(fields):
    names, meta = [], []

    def walk(f):
        names.append(f.name.encode())
        meta.extend([f.type_id, int(bool(f.nullable)), len(f.children)])
        for c in f.children:
            walk(c)
    for f in fields:
        walk(f)
    return names, meta


def _addr(a):
    return 0 if a is None else np.asarray(a).ctypes.data


def _cap(a):
    return 0 if a is None else np.asarray(a).nbytes


def describe(fields, cols, keep):
    d = []

    def walk(f, c):
        for a in (c.values, c.validity, c.offsets):
            if a is not None:
                keep.append(a)
        d.extend([_addr(c.values), _addr(c.validity), _addr(c.offsets), _cap(c.values),
                  len(f.children)])
        for fc, cc in zip(f.children, c.child or []):
            walk(fc, cc)
    for f, c in zip(fields, cols):
        walk(f, c)
    return np.array(d, np.int64)


def _i64p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def jni_schema(fields):
    names, meta = flatten(fields)
    L = N.lib()
    arr = (ctypes.c_char_p * len(names))(*names)
    m = np.array(meta, np.int32)
    h = ctypes.c_void_p()
    st = L.fury_jni_schema_create(arr, m.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                  len(names), len(fields), ctypes.byref(h))
    return st, h


def test_exception_classes():
    L = N.lib()
    assert L.fury_jni_exception_class(0) is None
    want = {1: b"java/lang/IllegalArgumentException", 2: b"java/lang/UnsupportedOperationException",
            3: b"org/apache/fury/exception/ClassNotCompatibleException",
            4: b"java/lang/IndexOutOfBoundsException",
            5: b"org/apache/fury/format/encoder/EncoderException",
            6: b"java/lang/RuntimeException", 7: b"java/lang/IndexOutOfBoundsException",
            99: b"java/lang/RuntimeException"}
    for st, cls in want.items():
        assert L.fury_jni_exception_class(st) == cls


@pytest.mark.parametrize("name", ["struct100", "mixed", "nested", "foo", "beanb"])
def test_jni_schema_matches_schema(name):
    from fury_amd.encoder import Schema
    fields = SCHEMAS[name]
    st, h = jni_schema(fields)
    assert st == 0, N.last_error()
    info = N.FurySchemaInfo()
    L = N.lib()
    assert L.fury_schema_get_info(h, ctypes.byref(info)) == 0
    assert info.schema_hash == Schema(fields).schema_hash
    L.fury_schema_destroy(h)


def test_jni_malformed_descriptors_rejected_without_device():
    L = N.lib()
    fields = SCHEMAS["foo"]
    names, meta = flatten(fields)
    arr = (ctypes.c_char_p * len(names))(*names)
    h = ctypes.c_void_p()
    bad = np.array(meta, np.int32)
    bad[2] = 5                                    # f1 (int) claims 5 children
    assert L.fury_jni_schema_create(arr, bad.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    len(names), len(fields), ctypes.byref(h)) == 1
    m = np.array(meta, np.int32)
    assert L.fury_jni_schema_create(arr, m.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    len(names) + 1, len(fields), ctypes.byref(h)) == 1
    st, h = jni_schema(fields)
    assert st == 0
    nodes = L.fury_schema_num_nodes(h)
    desc = np.zeros(5 * nodes, np.int64)
    rows = np.zeros(64, np.uint8)
    offs = np.zeros(2, np.int64)
    nb = ctypes.c_int64()
    # too short
    assert L.fury_jni_encode_host(h, _i64p(desc), 5 * nodes - 1, 1, rows.ctypes.data, 64,
                                  offs.ctypes.data, ctypes.byref(nb), 0) == 1
    # child counts all 0 where the schema has children
    assert L.fury_jni_encode_host(h, _i64p(desc), 5 * nodes, 1, rows.ctypes.data, 64,
                                  offs.ctypes.data, ctypes.byref(nb), 0) == 1
    assert "children" in N.last_error()
    # trailing entries past the schema's nodes
    long_desc = np.zeros(5 * nodes + 5, np.int64)
    assert L.fury_jni_decode_host(h, rows.ctypes.data, offs.ctypes.data, 1, _i64p(long_desc),
                                  5 * nodes + 5, 0) == 1
    L.fury_schema_destroy(h)


def test_jni_glue_compiles_against_minimal_jni_h(tmp_path):
    """fury_row_jni.cc (JNIEnv marshalling only) compiles against a jni.h declaring just the
    JNIEnv functions it calls, with the JNI specification's signatures."""
    inc = tmp_path / "jni.h"
    inc.write_text("""
#pragma once
#include <cstdint>
typedef int32_t jint; typedef int64_t jlong; typedef int32_t jsize; typedef uint8_t jboolean;
class _jobject {}; typedef _jobject* jobject; typedef jobject jclass; typedef jobject jstring;
typedef jobject jarray; typedef jobject jobjectArray; typedef jobject jintArray;
typedef jobject jlongArray;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
struct JNIEnv {
  jclass FindClass(const char*);
  jint ThrowNew(jclass, const char*);
  jsize GetArrayLength(jarray);
  jobject GetObjectArrayElement(jobjectArray, jsize);
  const char* GetStringUTFChars(jstring, jboolean*);
  void ReleaseStringUTFChars(jstring, const char*);
  void GetIntArrayRegion(jintArray, jsize, jsize, jint*);
  void GetLongArrayRegion(jlongArray, jsize, jsize, jlong*);
  void SetLongArrayRegion(jlongArray, jsize, jsize, const jlong*);
};
""")
    src = os.path.join(ROOT, "fury_amd", "csrc", "jni", "fury_row_jni.cc")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I", str(tmp_path),
                        src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


# ---- GPU: the core's host-memory batch path against the oracle --------------------------------

def _host_out(fields, n, rows_bytes):
    from fury_amd.workloads import Column
    out = []
    from fury_amd.types import BOOL, BINARY, DECIMAL, STRING, type_width
    for f in fields:
        vb = np.zeros((n + 7) // 8 + 8, np.uint8)
        if f.type_id in (STRING, BINARY):
            out.append(Column(values=np.zeros(max(rows_bytes, 16), np.uint8), validity=vb,
                              offsets=np.zeros(n + 1, np.int32)))
        elif f.type_id == LIST:
            out.append(Column(validity=vb, offsets=np.zeros(n + 1, np.int32),
                              child=[Column(values=np.zeros(max(rows_bytes, 16), np.uint8),
                                            validity=np.zeros(rows_bytes // 8 + 16, np.uint8))]))
        elif f.type_id == BOOL:
            out.append(Column(values=np.zeros((n + 7) // 8 + 8, np.uint8), validity=vb))
        elif f.type_id == DECIMAL:
            out.append(Column(values=np.zeros(16 * n + 16, np.uint8), validity=vb))
        else:
            out.append(Column(values=np.zeros(n * type_width(f.type_id) + 8, np.uint8),
                              validity=vb))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("struct100", 1001), ("mixed", 3001), ("nested", 2000)])
def test_jni_core_flat_roundtrip(oracle, name, n):
    L = N.lib()
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=21)
    st, h = jni_schema(fields)
    assert st == 0, N.last_error()
    keep: list = []
    desc = describe(fields, host, keep)
    want, want_offs = oracle.encode(fields, host, n)
    rows = np.zeros(len(want) + 64, np.uint8)
    offs = np.zeros(n + 1, np.int64)
    nb = ctypes.c_int64()
    assert L.fury_jni_encode_host(h, _i64p(desc), len(desc), n, rows.ctypes.data, rows.nbytes,
                                  offs.ctypes.data, ctypes.byref(nb), 0) == 0, N.last_error()
    assert nb.value == len(want)
    assert np.array_equal(rows[:nb.value], want)
    out = _host_out(fields, n, nb.value)
    keep2: list = []
    d2 = describe(fields, out, keep2)
    assert L.fury_jni_decode_host(h, rows.ctypes.data, offs.ctypes.data, n, _i64p(d2), len(d2),
                                  0) == 0, N.last_error()
    assert_columns_equal(fields, out, oracle.decode(fields, want, want_offs, n), n)
    L.fury_schema_destroy(h)


@pytest.mark.gpu
def test_jni_core_nested_foo(oracle):
    """Foo (list<string>, map<string,int>, nested Bar): encode through the core, then the two-step
    decode (prepare -> counts -> host buffers of those sizes -> execute), as decodeNested does."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import _alloc_host_node, _bfs
    from tests.test_device import _random_value
    L = N.lib()
    fields = SCHEMAS["foo"]
    n = 1200
    rng = np.random.default_rng(5)
    host = beans_to_columns(fields, [{f.name: _random_value(f, rng) for f in fields}
                                     for _ in range(n)])
    st, h = jni_schema(fields)
    assert st == 0, N.last_error()
    keep: list = []
    desc = describe(fields, host, keep)
    want, want_offs = oracle.encode(fields, host, n)
    rows = np.zeros(len(want) + 64, np.uint8)
    offs = np.zeros(n + 1, np.int64)
    nb = ctypes.c_int64()
    assert L.fury_jni_encode_host(h, _i64p(desc), len(desc), n, rows.ctypes.data, rows.nbytes,
                                  offs.ctypes.data, ctypes.byref(nb), 0) == 0, N.last_error()
    assert np.array_equal(rows[:nb.value], want)
    nn = L.fury_schema_num_nodes(h)
    counts = np.zeros(2 * nn, np.int64)
    plan = ctypes.c_void_p()
    short = np.zeros(2 * nn - 1, np.int64)
    assert L.fury_jni_decode_host_prepare(h, rows.ctypes.data, offs.ctypes.data, n,
                                          _i64p(short), len(short), ctypes.byref(plan),
                                          0) == 1          # FURY_ERR_INVALID_ARGUMENT
    assert not short.any() and not plan.value
    assert L.fury_jni_decode_host_prepare(h, rows.ctypes.data, offs.ctypes.data, n,
                                          _i64p(counts), len(counts), ctypes.byref(plan), 0) == 0
    order = _bfs(fields)
    cols = [_alloc_host_node(f, int(counts[2 * i]), int(counts[2 * i + 1]))
            for i, (f, _) in enumerate(order)]
    for i, (f, first) in enumerate(order):
        if f.children:
            cols[i].child = [cols[first + j] for j in range(len(f.children))]
    top = cols[:len(fields)]
    keep2: list = []
    d2 = describe(fields, top, keep2)
    assert L.fury_jni_decode_host_execute(h, plan, _i64p(d2), len(d2)) == 0, N.last_error()
    L.fury_decode_plan_destroy(plan)
    assert_columns_equal(fields, top, oracle.decode(fields, want, want_offs, n), n)
    L.fury_schema_destroy(h)
