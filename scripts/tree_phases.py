"""Phase times of the row-walk decode passes (tuning "tree_debug"): thread 0 of every workgroup adds the
time between phase marks; printed as the mean microseconds per workgroup per phase (thread 0's
timeline: barrier waits included).  Depth-3 nested schema of the tests, --rows rows.

    python scripts/tree_phases.py --rows 4000000 [--tune key=value ...]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WALK_C = {0: "stage + barrier", 1: "walk (thread 0)", 2: "walk tail + scans", 3: "epilogue"}
WALK_W = {0: "prologue + stage + windows", 1: "walk (thread 0)", 2: "walk tail (barrier)",
          3: "window flush"}
# tile BFS (nested_decode 3, bfs.hip BClock)
BFS = {0: "stage + row / node bases", 1: "top-level nodes", 2: "nested nodes", 3: "owner arrays",
       4: "node table + barrier"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--tune", action="append", default=[])
    args = ap.parse_args()
    import torch
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    from tests.test_device import _nested_beans, _nested_fields
    L = N.lib()
    fn = L.fury_internal_tree_debug
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
    for kv in args.tune:
        k, v = kv.split("=")
        assert L.fury_set_tuning(k.encode(), int(v)) == 0, N.last_error()
    fields = _nested_fields()
    base = _nested_beans(50_000, seed=1)
    beans = (base * (args.rows // len(base) + 1))[:args.rows]
    dev = torch.device("cuda:0")
    cols = [column_to_device(c, dev) for c in beans_to_columns(fields, beans)]
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, args.rows)
    enc.decode_batch(batch)
    torch.cuda.synchronize()
    assert L.fury_set_tuning(b"tree_debug", 1) == 0
    out = (ctypes.c_int64 * 80)()
    fn(out, 80)                                     # zero
    enc.encode_batch(cols, args.rows)
    enc.decode_batch(batch)
    assert fn(out, 80) == 0
    res = {}
    bfs = L.fury_get_tuning(b"nested_decode") == 3 and L.fury_get_tuning(b"bfs_fallbacks") == 0
    for name, off, cnt_i, names in (("decode_pass1", 0, 64, BFS if bfs else WALK_C),
                                    ("decode_pass2", 16, 65, BFS if bfs else WALK_W)):
        wg = max(out[cnt_i], 1)
        res[name] = {"workgroups": out[cnt_i],
                     "us_per_wg": {names.get(i, str(i)): round(out[off + i] / wg / 100.0, 2)
                                   for i in range(15) if out[off + i]}}
    print(json.dumps({"rows": args.rows, "tune": args.tune, "phases": res}, indent=1))
    assert L.fury_set_tuning(b"tree_debug", 0) == 0


if __name__ == "__main__":
    main()
