"""A/B timing of the variable-length decode (or, --encode, the measured encode) under fury_set_tuning legs (or one leg), HIP events
over bound calls, interleaved rounds in one process; every leg's output is checked equal to leg 0's.

    python scripts/ab_dec.py --workload mixed [--key lookback_help --legs 0,1]
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
    ap.add_argument("--legs", default="0")
    ap.add_argument("--key", default="none", help="fury_set_tuning key of the legs (none: one leg)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-check", action="store_true", help="timing-only legs (outputs differ)")
    ap.add_argument("--encode", action="store_true",
                    help="time the measured encode (rows + row offsets checked) instead")
    args = ap.parse_args()
    import torch
    from bench import DEFAULT_ROWS, make_device_columns
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
    if args.encode:
        from fury_amd.encoder import Column
        out = [Column(values=batch.rows), Column(values=batch.row_offsets)]
        call = enc.bind_encode(cols, n, batch.rows, batch.row_offsets, measured=True)
    L = N.lib()
    key = args.key.encode()

    def tune(v):
        if args.key != "none":
            assert L.fury_set_tuning(key, v) == 0
    legs = [int(x) for x in args.legs.split(",")]

    def flat(cs):
        ts = []
        for c in cs:
            for t in (c.values, c.validity, c.offsets):
                if t is not None:
                    ts.append(t.clone())
            if c.child:
                ts.extend(flat(c.child))
        return ts

    ref = None
    for leg in legs:
        tune(leg)
        for t in flat(out):
            pass
        call()
        torch.cuda.synchronize()
        got = flat(out)
        if ref is None:
            ref = got
        else:
            same = all(torch.equal(x, y) for x, y in zip(ref, got))
            print(json.dumps({"leg": leg, "equal_to_leg0": same}), flush=True)
            assert same or args.no_check, f"leg {leg} output differs"
    times = {leg: [] for leg in legs}
    for _ in range(args.rounds):
        for leg in legs:
            tune(leg)
            call()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                call()
            b.record()
            torch.cuda.synchronize()
            times[leg].append(a.elapsed_time(b) / args.iters)
    tune(0)
    print(json.dumps({"workload": args.workload, "rows": n, "key": args.key,
                      "ms": {str(k): round(statistics.median(v), 4) for k, v in times.items()},
                      "min_ms": {str(k): round(min(v), 4) for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
