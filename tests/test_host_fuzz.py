"""Randomised host-logic inputs (CPU, no device work): nested schemas of random shape through
fury_schema_create / fury_jni_schema_create (hash and layout agree between the two, and with the
oracle), truncated and corrupted JNI field / column descriptors (rejected with a status, never a
crash), and random batches through the oracle's encode -> decode.  Run plainly here and again by
tests/test_sanitize.py against the ASan/UBSan builds of the library and the oracle."""
from __future__ import annotations

import ctypes
import random

import numpy as np

from fury_amd import _native as N
from fury_amd import types as T
from tests.helpers import assert_columns_equal
from tests.test_jni_core import _i64p, flatten, jni_schema

SCALARS = [T.BOOL, T.INT8, T.INT16, T.INT32, T.INT64, T.FLOAT32, T.FLOAT64, T.STRING, T.BINARY,
           T.DATE32, T.TIMESTAMP]


def random_field(rnd, name, depth):
    nullable = rnd.random() < 0.7
    k = rnd.random()
    if depth < 4 and k < 0.15:
        kids = [random_field(rnd, f"s{j}", depth + 1) for j in range(rnd.randint(1, 4))]
        return T.field(name, T.STRUCT, nullable, kids)
    if depth < 4 and k < 0.3:
        return T.field(name, T.LIST, nullable, [random_field(rnd, "item", depth + 1)])
    if depth < 4 and k < 0.38:
        key = T.field("key", rnd.choice([T.INT32, T.INT64, T.STRING]), False)
        return T.field(name, T.MAP, nullable, [key, random_field(rnd, "value", depth + 1)])
    return T.field(name, rnd.choice(SCALARS), nullable)


def random_schema(rnd):
    return [random_field(rnd, f"f{k:02d}", 0) for k in range(rnd.randint(1, 12))]


def test_random_schemas_agree_between_entry_points(oracle):
    from fury_amd.encoder import Schema
    rnd = random.Random(20261018)
    L = N.lib()
    for _ in range(60):
        fields = random_schema(rnd)
        s = Schema(fields)
        st, h = jni_schema(fields)
        assert st == 0, N.last_error()
        info = N.FurySchemaInfo()
        assert L.fury_schema_get_info(h, ctypes.byref(info)) == 0
        assert info.schema_hash == s.schema_hash
        assert info.fixed_size == s.fixed_size
        assert L.fury_schema_num_nodes(h) == len(flatten(fields)[0])
        L.fury_schema_destroy(h)


def test_random_corrupted_jni_descriptors_are_rejected():
    rnd = random.Random(7)
    L = N.lib()
    for _ in range(200):
        fields = random_schema(rnd)
        names, meta = flatten(fields)
        m = np.array(meta, np.int32)
        how = rnd.randrange(4)
        nodes = len(names)
        if how == 0:                                  # a child count past the node list
            m[3 * rnd.randrange(nodes) + 2] = rnd.choice([-1, nodes + 1, 1 << 30])
        elif how == 1:                                # fewer nodes than the top level needs
            nodes = rnd.randrange(nodes)
        elif how == 2:                                # an unknown type id
            m[3 * rnd.randrange(nodes)] = rnd.choice([0, 2, 99, -5])
        arr = (ctypes.c_char_p * max(len(names), 1))(*names)
        h = ctypes.c_void_p()
        st = L.fury_jni_schema_create(arr, m.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      nodes, len(fields), ctypes.byref(h))
        if how == 3:
            assert st == 0, N.last_error()
        if st != 0:
            assert N.last_error()
            continue
        # column descriptors: random lengths and child counts, rejected before any device work
        n = L.fury_schema_num_nodes(h)
        ln = rnd.choice([0, 5 * n - 1, 5 * n + 5, rnd.randrange(5 * n + 1)])
        desc = np.zeros(max(ln, 1), np.int64)
        desc[4::5] = rnd.randrange(3)
        rows = np.zeros(64, np.uint8)
        offs = np.zeros(2, np.int64)
        nb = ctypes.c_int64()
        if ln != 5 * n:
            assert L.fury_jni_encode_host(h, _i64p(desc), ln, 1, rows.ctypes.data, 64,
                                          offs.ctypes.data, ctypes.byref(nb), 0) != 0
            assert L.fury_jni_decode_host(h, rows.ctypes.data, offs.ctypes.data, 1, _i64p(desc),
                                          ln, 0) != 0
        L.fury_schema_destroy(h)


def test_random_batches_oracle_round_trip(oracle):
    from fury_amd.beans import beans_to_columns
    from fury_amd.workloads import JavaRandom
    from tests.test_reference_beans import random_bean
    rnd = random.Random(3)
    for i in range(25):
        fields = random_schema(rnd)
        n = rnd.choice([0, 1, 7, 64, 65, 300])
        jr = JavaRandom(i)
        host = beans_to_columns(fields, [random_bean(fields, jr) for _ in range(n)])
        rows, offs = oracle.encode(fields, host, n)
        ref = oracle.decode(fields, rows, offs, n)
        again, again_offs = oracle.encode(fields, ref, n)
        assert np.array_equal(again, rows)
        assert_columns_equal(fields, oracle.decode(fields, again, again_offs, n), ref, n)
