"""Host-memory batch path timing (fury_row_encode_host / fury_row_decode_host), Struct-100,
pinned host buffers, for several pipeline chunk counts (env FURY_HOST_CHUNKS, read per call).

    python scripts/ab_host.py [--rows 1000000] [--chunks 1,2,3,6,12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--chunks", default="1,2,3,6,12")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import SCHEMAS, Column
    fields = SCHEMAS["struct100"]
    n = args.rows
    g = torch.Generator().manual_seed(1)
    host = [Column(values=torch.randint(0, 255, (n * 8,), dtype=torch.uint8, generator=g)
                   .pin_memory()) for _ in fields]
    rows = torch.empty(n * 816, dtype=torch.uint8).pin_memory()
    out = [Column(values=torch.empty(n * 8, dtype=torch.uint8).pin_memory()) for _ in fields]
    enc = Encoders.bean(fields, device="cuda:0")
    res = {}
    # naive reference: whole-column H2D, encode, D2H on one stream (torch copies)
    dcols = [Column(values=torch.empty(n * 8, dtype=torch.uint8, device="cuda:0")) for _ in fields]
    drows = torch.empty(n * 816, dtype=torch.uint8, device="cuda:0")
    for c in [int(x) for x in args.chunks.split(",")] + [0]:
        os.environ["FURY_HOST_CHUNKS"] = str(max(c, 1))
        enc.encode_host(host, n, rows=rows)
        te = td = 0.0
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if c:
                enc.encode_host(host, n, rows=rows)
            else:
                for h, d in zip(host, dcols):
                    d.values.copy_(h.values, non_blocking=True)
                enc.encode_into(dcols, n, drows, None)
                rows.copy_(drows, non_blocking=True)
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            if c:
                enc.decode_host(rows, None, n, out=out)
            t2 = time.perf_counter()
            te += t1 - t0
            td += t2 - t1
        te /= args.reps
        td /= args.reps
        b = n * (800 + 816)
        key = f"chunks{c}" if c else "naive_torch_encode"
        res[key] = {"encode_ms": round(te * 1e3, 2), "encode_GBps": round(b / te / 1e9, 2)}
        if c:
            res[key].update({"decode_ms": round(td * 1e3, 2), "decode_GBps": round(b / td / 1e9, 2)})
    assert torch.equal(out[7].values, host[7].values)
    print(json.dumps({"rows": n, "results": res}))


if __name__ == "__main__":
    main()
