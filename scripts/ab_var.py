"""Timing of the variable-length path's pieces in ONE process (HIP events, interleaved rounds).

    python scripts/ab_var.py [--workload mixed|nested|narrow] [--rows N] [--rounds 5] [--iters 10]

Legs: measure (fury_row_measure), encode (fury_row_encode at known offsets), encode_measured
(fury_row_encode_measured = measure + encode).  Prints a
JSON line with the median ms of each leg and the algorithmic GB/s of the encode/decode legs.
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders, _c_columns, _ptr, _stream_handle
    from bench import DEFAULT_ROWS, _nbytes, make_device_columns
    from fury_amd.workloads import SCHEMAS
    dev = torch.device("cuda:0")
    name = args.workload
    fields = SCHEMAS[name]
    n = args.rows or DEFAULT_ROWS[name]
    cols = make_device_columns(name, fields, n, 0, dev)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, n)
    offs = batch.row_offsets
    rows = batch.rows
    out = enc.decode_batch(batch)
    torch.cuda.synchronize()
    legs = {
        "measure": lambda: enc.measure_into(cols, n, offs),
        "encode": lambda: enc.encode_into(cols, n, rows, offs),
        "encode_measured": lambda: enc.encode_measured_into(cols, n, rows, offs),
    }
    if os.environ.get("AB_LEGS"):
        legs = {k: v for k, v in legs.items() if k in os.environ["AB_LEGS"].split(",")}
    times = {k: [] for k in legs}
    for _ in range(2):
        for f in legs.values():
            f()
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k, f in legs.items():
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                f()
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b) / args.iters)
    enc.check_capacity(out, n)

    col_bytes = _nbytes(cols)
    row_bytes = rows.numel() + offs.numel() * 8
    med = {k: round(statistics.median(v), 4) for k, v in times.items()}
    res = {"workload": name, "rows": n, "ms": med,
           "GBps": {k: round((col_bytes + row_bytes) / (med[k] * 1e-3) / 1e9, 1)
                    for k in med if k != "measure" and k != "decode_measure"}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
