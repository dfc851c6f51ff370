"""DIAGNOSTIC: HIP-event timing of the variable-length decode under each (var_decode mode,
FURY_VAR_DBG bits) leg, through bound calls (argument block built once, so host overhead per
call is a few us), interleaved rounds in one process.  Outputs are wrong when dbg bits are set.

    python scripts/time_decode.py [--workload mixed] [--rows N] [--legs 3:0,5:0,5:128]
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
    ap.add_argument("--legs", default="0:0,3:0,4:0,5:0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    os.environ["FURY_DIAGNOSTIC"] = "1"
    import torch
    from bench import DEFAULT_ROWS, _nbytes, make_device_columns
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import SCHEMAS
    dev = torch.device("cuda:0")
    fields = SCHEMAS[args.workload]
    n = args.rows or DEFAULT_ROWS[args.workload]
    cols = make_device_columns(args.workload, fields, n, 0, dev)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, n)
    out = enc.decode_batch(batch)
    call = enc.bind_decode(batch, out)
    L = N.lib()
    legs = [tuple(int(x) for x in leg.split(":")) for leg in args.legs.split(",")]

    def run(leg, k):
        L.fury_set_tuning(b"var_decode", leg[0])
        os.environ["FURY_VAR_DBG"] = str(leg[1])
        for _ in range(k):
            call()

    for leg in legs:
        run(leg, 2)
    torch.cuda.synchronize()
    times = {leg: [] for leg in legs}
    for _ in range(args.rounds):
        for leg in legs:
            L.fury_set_tuning(b"var_decode", leg[0])
            os.environ["FURY_VAR_DBG"] = str(leg[1])
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                call()
            b.record()
            torch.cuda.synchronize()
            times[leg].append(a.elapsed_time(b) / args.iters * 1e3)
    os.environ["FURY_VAR_DBG"] = "0"
    L.fury_set_tuning(b"var_decode", 0)
    nbytes = _nbytes(cols) + batch.rows.numel() + batch.row_offsets.numel() * 8
    res = {"workload": args.workload, "rows": n, "bytes": nbytes,
           "env": {k: v for k, v in os.environ.items() if k.startswith("FURY_LDS_")},
           "us": {f"{m}:{d}": round(statistics.median(v), 1) for (m, d), v in times.items()}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
