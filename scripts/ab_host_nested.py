"""End-to-end host-memory path of NESTED schemas (the JNI boundary: fury_row_encode_host,
fury_decode_host_prepare / execute): host columns -> host rows -> host columns, timed per call,
direct (every buffer pinned: kernels on host memory) vs staged (pageable: copies through HBM).
GB/s = algorithmic bytes (column bytes + row bytes) per direction / wall time.

    python scripts/ab_host_nested.py --rows 1000000 --schema nested7
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pinned_tree(c, host_empty):
    from fury_amd.workloads import Column

    def cp(a, dt):
        if a is None:
            return None
        src = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        b = host_empty(max(src.nbytes, 16))[:src.nbytes]
        b[:] = src
        return b.view(dt)
    return Column(values=cp(c.values, np.uint8), validity=cp(c.validity, np.uint8),
                  offsets=cp(c.offsets, np.int32),
                  child=[pinned_tree(x, host_empty) for x in c.child] if c.child else None)


_OUT = {}


def decode(enc, fields, rows, offs, n, pinned):
    """fury_decode_host_prepare + fury_decode_host_execute into output buffers allocated once
    (pinned or pageable) and reused, as a JVM caller would keep its off-heap buffers."""
    import ctypes
    from fury_amd import _native as N
    from fury_amd.encoder import _alloc_host_node, _bfs, _c_host_columns, _pinned_zeros
    L = N.lib()
    h = enc.schema().handle
    nn = L.fury_schema_num_nodes(h)
    e = (ctypes.c_int64 * nn)()
    b = (ctypes.c_int64 * nn)()
    plan = ctypes.c_void_p()
    assert L.fury_decode_host_prepare(h, rows.ctypes.data, offs.ctypes.data, n, e, b,
                                      ctypes.byref(plan), 0) == 0, N.last_error()
    try:
        key = (pinned, n)
        if key not in _OUT:
            order = _bfs(fields)
            zeros = _pinned_zeros if pinned else np.zeros
            out = [_alloc_host_node(f, int(e[i]), int(b[i]), zeros) for i, (f, _) in enumerate(order)]
            for i, (f, first) in enumerate(order):
                if f.children:
                    out[i].child = [out[first + j] for j in range(len(f.children))]
            _OUT[key] = out[:len(fields)]
        keep = []
        assert L.fury_decode_host_execute(plan, _c_host_columns(_OUT[key], keep)) == 0, N.last_error()
    finally:
        L.fury_decode_plan_destroy(plan)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--schema", default="nested7")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, _tree_bytes, host_empty
    from fury_amd.workloads import SCHEMAS
    from tests.test_device import _nested_beans, _nested_fields
    if args.schema == "nested7":
        fields = _nested_fields()
        base = _nested_beans(20_000, seed=3)
    else:
        from tests.test_tree import _beans
        fields = SCHEMAS[args.schema]
        base = _beans(fields, 20_000, 3)
    n = args.rows
    host = beans_to_columns(fields, (base * (n // len(base) + 1))[:n])
    enc = Encoders.bean(fields, device="cuda:0")
    col_bytes = _tree_bytes(host)
    rows_ref, offs_ref = enc.encode_host(host, n)
    row_bytes = int(rows_ref.nbytes)
    alg = col_bytes + row_bytes
    pin = [pinned_tree(c, host_empty) for c in host]
    prow = host_empty((row_bytes + 15) // 16 * 16)
    poff = host_empty(8 * (n + 1), np.int64)

    def timed(fn):
        fn()
        ts = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return min(ts)
    res = {"schema": args.schema, "rows": n, "column_bytes": col_bytes, "row_bytes": row_bytes}
    res["encode_direct_s"] = timed(lambda: enc.encode_host(pin, n, rows=prow, row_offsets=poff))
    assert np.array_equal(prow[:row_bytes], rows_ref)
    res["encode_staged_s"] = timed(lambda: enc.encode_host(host, n))
    from fury_amd import _native as N
    d0 = N.lib().fury_get_tuning(b"host_direct")
    res["decode_direct_s"] = timed(lambda: decode(enc, fields, prow, poff, n, True))
    res["decode_staged_s"] = timed(lambda: decode(enc, fields, rows_ref, offs_ref, n, False))
    res["direct_calls"] = N.lib().fury_get_tuning(b"host_direct") - d0
    for k in ("encode_direct", "encode_staged", "decode_direct", "decode_staged"):
        res[k + "_GBps"] = round(alg / res[k + "_s"] / 1e9, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
