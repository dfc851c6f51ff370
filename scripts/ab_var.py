"""Timing of the variable-length path's pieces in ONE process (HIP events, interleaved rounds).

    python scripts/ab_var.py [--workload mixed|nested|narrow] [--rows N] [--rounds 5] [--iters 10]

Legs: measure (fury_row_measure), encode (fury_row_encode at known offsets), encode_measured
(fury_row_encode_measured = measure + encode), decode one-pass (look-back) and two-pass (tuning
var_decode=1), decode_measure (sizing pass only).  Prints a
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
    keep = []
    sh = _stream_handle(None)
    ccols = _c_columns(out, keep)
    L = N.lib()
    legs = {
        "measure": lambda: enc.measure_into(cols, n, offs),
        "encode": lambda: enc.encode_into(cols, n, rows, offs),
        "encode_measured": lambda: enc.encode_measured_into(cols, n, rows, offs),
        "encode_tile": lambda: (os.environ.__setitem__("FURY_VAR_DBG", "1024"),
                                enc.encode_into(cols, n, rows, offs),
                                os.environ.__setitem__("FURY_VAR_DBG", "0")),
        "decode_1pass": lambda: (L.fury_set_tuning(b"var_decode", 3),
                                 enc.decode_into(batch, out)),
        "decode_2pass": lambda: (L.fury_set_tuning(b"var_decode", 1),
                                 enc.decode_into(batch, out)),
        "decode_512": lambda: (L.fury_set_tuning(b"var_decode", 2),
                               enc.decode_into(batch, out), L.fury_set_tuning(b"var_decode", 3)),
        "decode_measure": lambda: L.fury_row_decode_measure(enc._schema.handle, _ptr(rows),
                                                            _ptr(offs), n, ccols, sh),
        # round 2: tile order by ticket (default) vs blockIdx (4096); the LDS-DMA kernel (1024)
        "decode_ticket": lambda: (L.fury_set_tuning(b"var_decode", 0), enc.decode_into(batch, out)),
        "decode_order": lambda: (L.fury_set_tuning(b"var_decode", 0),
                                 os.environ.__setitem__("FURY_VAR_DBG", "4096"),
                                 enc.decode_into(batch, out),
                                 os.environ.__setitem__("FURY_VAR_DBG", "0")),
        "decode_maximg": lambda: (L.fury_set_tuning(b"var_decode", 0),
                                  os.environ.__setitem__("FURY_VAR_DBG", "8192"),
                                  enc.decode_into(batch, out),
                                  os.environ.__setitem__("FURY_VAR_DBG", "0")),
        "decode_lds": lambda: (L.fury_set_tuning(b"var_decode", 0),
                               os.environ.__setitem__("FURY_VAR_DBG", "1024"),
                               enc.decode_into(batch, out),
                               os.environ.__setitem__("FURY_VAR_DBG", "0")),
        # round 2: LDS-staged decode (var_lds.hip)
        "decode_lds_tile": lambda: (L.fury_set_tuning(b"var_decode", 4), enc.decode_into(batch, out)),
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
    L.fury_set_tuning(b"var_decode", 0)

    col_bytes = _nbytes(cols)
    row_bytes = rows.numel() + offs.numel() * 8
    med = {k: round(statistics.median(v), 4) for k, v in times.items()}
    res = {"workload": name, "rows": n, "ms": med,
           "GBps": {k: round((col_bytes + row_bytes) / (med[k] * 1e-3) / 1e9, 1)
                    for k in med if k != "measure" and k != "decode_measure"}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
