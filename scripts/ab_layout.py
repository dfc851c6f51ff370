"""Column placement A/B in ONE process (interleaved rounds), Struct-100, default kernel variant.

    python scripts/ab_layout.py [--rows 1000000] [--rounds 7] [--iters 20]

Layouts of the 100 input (and decoded output) columns:
  separate  one torch allocation per column (the caching allocator rounds 8 MB up to 2 MiB
            multiples: every column starts at the same offset modulo 2 MiB)
  arrow     one contiguous body, columns back to back (an Arrow RecordBatch / IPC body:
            8,000,000 B apart)
  stagger   one body, column c at c * (8 MB + 4 KB + 256 B)
Prints median encode / decode ms and algorithmic GB/s per layout; rows must be identical.
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch
    from fury_amd.encoder import Encoders, RowBatch
    from fury_amd.workloads import SCHEMAS, Column
    dev = torch.device("cuda:0")
    fields = SCHEMAS["struct100"]
    n = args.rows
    nc = len(fields)
    g = torch.Generator(device=dev).manual_seed(1)
    src = [torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device=dev, generator=g)
           for _ in fields]

    def layout(kind):
        if kind == "separate":
            ins = [Column(values=s.clone()) for s in src]
            outs = [Column(values=torch.empty(n * 8, dtype=torch.uint8, device=dev)) for _ in src]
            return ins, outs
        stride = n * 8 if kind == "arrow" else n * 8 + 4096 + 256
        body = torch.empty(nc * stride + 256, dtype=torch.uint8, device=dev)
        obody = torch.empty(nc * stride + 256, dtype=torch.uint8, device=dev)
        ins, outs = [], []
        for c, s in enumerate(src):
            v = body[c * stride:c * stride + n * 8]
            v.copy_(s.view(torch.uint8))
            ins.append(Column(values=v.view(torch.int64)))
            outs.append(Column(values=obody[c * stride:c * stride + n * 8]))
        return ins, outs

    enc = Encoders.bean(fields, device=dev)
    rows = torch.empty(n * 816, dtype=torch.uint8, device=dev)
    batch = RowBatch(rows, None, n, enc.schema_hash)
    kinds = ["separate", "arrow", "stagger"]
    sets = {k: layout(k) for k in kinds}
    ref = None
    for k in kinds:
        enc.encode_into(sets[k][0], n, rows, None)
        enc.decode_batch(batch, validity=False, out=sets[k][1])
        torch.cuda.synchronize()
        if ref is None:
            ref = rows.clone()
        assert torch.equal(rows, ref), k
        assert torch.equal(sets[k][1][3].values, src[3].view(torch.uint8)), k
    res = {k: {"enc": [], "dec": []} for k in kinds}
    for _ in range(args.rounds):
        for k in kinds:
            ins, outs = sets[k]
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(args.iters):
                enc.encode_into(ins, n, rows, None)
            ev[1].record()
            for _ in range(args.iters):
                enc.decode_batch(batch, validity=False, out=outs)
            ev[2].record()
            torch.cuda.synchronize()
            res[k]["enc"].append(ev[0].elapsed_time(ev[1]) / args.iters)
            res[k]["dec"].append(ev[1].elapsed_time(ev[2]) / args.iters)
    nb = n * (800 + 816)
    rep = {}
    for k, d in res.items():
        e, dd = statistics.median(d["enc"]), statistics.median(d["dec"])
        rep[k] = {"encode_ms": round(e, 4), "decode_ms": round(dd, 4),
                  "encode_GBps": round(nb / e / 1e6, 1), "decode_GBps": round(nb / dd / 1e6, 1)}
    print(json.dumps({"rows": n, "layouts": rep}))


if __name__ == "__main__":
    main()
