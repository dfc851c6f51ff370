"""A/B of the fixed-width kernel variants in ONE process (interleaved rounds), Struct-100.

    python scripts/ab_fixed.py [--rows 1000000] [--rounds 5] [--iters 20]

Prints per-variant median encode / decode times and algorithmic GB/s, next to a torch D2D copy
of the same byte volume (the achievable streaming reference on this device), and checks that
every variant produces identical rows and round-trips the columns.
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
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="0,1,2,3,6,7")
    ap.add_argument("--layout", default="separate",
                    help="separate: one allocation per column; arrow: one contiguous body, "
                         "columns back to back (an Arrow RecordBatch body)")
    args = ap.parse_args()
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders, RowBatch
    from fury_amd.workloads import SCHEMAS, Column
    dev = torch.device("cuda:0")
    fields = SCHEMAS["struct100"]
    n = args.rows
    g = torch.Generator(device=dev).manual_seed(1)
    if args.layout == "arrow":
        body = torch.randint(-2**63, 2**63 - 1, (len(fields) * n,), dtype=torch.int64, device=dev,
                             generator=g)
        cols = [Column(values=body[i * n:(i + 1) * n]) for i in range(len(fields))]
    else:
        cols = [Column(values=torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64,
                                            device=dev, generator=g)) for _ in fields]
    enc = Encoders.bean(fields, device=dev)
    rows = torch.empty(n * 816, dtype=torch.uint8, device=dev)
    out = enc.alloc_columns(n, validity=False)
    if args.layout == "arrow":
        obody = torch.empty(len(fields) * n * 8, dtype=torch.uint8, device=dev)
        out = [Column(values=obody[i * n * 8:(i + 1) * n * 8]) for i in range(len(fields))]
    batch = RowBatch(rows, None, n, enc.schema_hash)
    variants = [int(v) for v in args.variants.split(",")]
    ref_rows = None
    for v in variants:
        assert N.lib().fury_set_tuning(b"fixed_variant", v) == 0
        rows.zero_()
        enc.encode_into(cols, n, rows, None)
        enc.decode_batch(batch, validity=False, out=out)
        torch.cuda.synchronize()
        if ref_rows is None:
            ref_rows = rows.clone()
        assert torch.equal(rows, ref_rows), f"variant {v} rows differ"
        for c, o in zip(cols, out):
            assert torch.equal(c.values.view(torch.uint8), o.values), f"variant {v} decode"
    res = {v: {"enc": [], "dec": []} for v in variants}
    res["copy"] = {"enc": [], "dec": []}
    src = torch.empty(n * 808, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    for _ in range(args.rounds):
        for v in variants + ["copy"]:
            if v != "copy":
                N.lib().fury_set_tuning(b"fixed_variant", v)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(args.iters):
                if v == "copy":
                    dst.copy_(src)
                else:
                    enc.encode_into(cols, n, rows, None)
            ev[1].record()
            for _ in range(args.iters):
                if v == "copy":
                    src.copy_(dst)
                else:
                    enc.decode_batch(batch, validity=False, out=out)
            ev[2].record()
            torch.cuda.synchronize()
            res[v]["enc"].append(ev[0].elapsed_time(ev[1]) / args.iters)
            res[v]["dec"].append(ev[1].elapsed_time(ev[2]) / args.iters)
    nbytes = n * (800 + 816)
    report = {}
    for v, d in res.items():
        e, dd = statistics.median(d["enc"]), statistics.median(d["dec"])
        report[str(v)] = {"encode_ms": round(e, 4), "decode_ms": round(dd, 4),
                          "encode_GBps": round(nbytes / e / 1e6, 1),
                          "decode_GBps": round(nbytes / dd / 1e6, 1),
                          "encdec_GBps": round(2 * nbytes / (e + dd) / 1e6, 1),
                          "enc_min_ms": round(min(d["enc"]), 4), "dec_min_ms": round(min(d["dec"]), 4)}
    print(json.dumps({"rows": n, "variants": report}, indent=1))


if __name__ == "__main__":
    main()
