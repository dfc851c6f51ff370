"""DIAGNOSTIC: time the var encode / decode kernels with phases switched off (FURY_VAR_DBG bits;
outputs are wrong when a bit is set — timing only).

    python scripts/diag_var.py [--workload mixed|nested] [--rows N]

encode bits: 1 skip payload staging, 2 skip row build, 4 skip the image store, 64 input loads
only (register-staged kernel).
decode bits: 8 skip fixed fields, 16 skip string/list payload, 32 skip look-back (base 0), 128
row loads only.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="mixed")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mode", type=int, default=0, help="tuning var_decode for the decode legs")
    ap.add_argument("--decode-only", action="store_true")
    args = ap.parse_args()
    os.environ["FURY_DIAGNOSTIC"] = "1"      # the phase-skipping bits are diagnostic only
    import torch
    from bench import DEFAULT_ROWS, make_device_columns
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import SCHEMAS
    dev = torch.device("cuda:0")
    fields = SCHEMAS[args.workload]
    n = args.rows or DEFAULT_ROWS[args.workload]
    cols = make_device_columns(args.workload, fields, n, 0, dev)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, n)
    out = enc.decode_batch(batch)
    torch.cuda.synchronize()

    def t(f):
        f()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        xs = []
        for _ in range(3):
            a.record()
            for _ in range(args.iters):
                f()
            b.record()
            torch.cuda.synchronize()
            xs.append(a.elapsed_time(b) / args.iters)
        return round(statistics.median(xs) * 1e3, 1)

    res = {"workload": args.workload, "rows": n, "encode_us": {}, "decode_us": {}}
    for d in (() if args.decode_only else (0, 2, 4, 6, 64)):
        os.environ["FURY_VAR_DBG"] = str(d)
        res["encode_us"][d] = t(lambda: enc.encode_into(cols, n, batch.rows, batch.row_offsets))
    os.environ["FURY_VAR_DBG"] = "0"          # restore valid rows before the decode legs
    enc.encode_into(cols, n, batch.rows, batch.row_offsets)
    torch.cuda.synchronize()
    from fury_amd import _native as N
    N.lib().fury_set_tuning(b"var_decode", args.mode)
    res["mode"] = args.mode
    for d in (0, 8, 16, 32, 56, 128) + (() if args.mode >= 4 else (4096, 4096 + 32)):
        os.environ["FURY_VAR_DBG"] = str(d)
        res["decode_us"][d] = t(lambda: enc.decode_into(batch, out))
    os.environ["FURY_VAR_DBG"] = "0"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
