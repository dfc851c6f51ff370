"""EXPERIMENT: zero-copy host path for Struct-100 — the encode / decode kernels reading and
writing pinned host memory directly over PCIe (no HBM staging, reads and writes in flight
together), against the staged fury_row_encode_host / fury_row_decode_host.

    python scripts/ab_host_zc.py [--rows 1000000]

Legs (each one batch, ms + algorithmic GB/s = (column bytes + row bytes) / time):
  staged_{enc,dec}       the host API forced onto its staged path (H2D / kernel / D2H)
  api_{enc,dec}          the host API on pinned buffers (fixed_direct)
  zc_{enc,dec}           kernel on host pointers for input AND output
  zc_in_{enc,dec}        host input, HBM output (PCIe reads only)
  zc_out_{enc,dec}       HBM input, host output (PCIe writes only)
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders, _c_host_columns, _c_columns
    from fury_amd.workloads import SCHEMAS, Column
    fields = SCHEMAS["struct100"]
    n = args.rows
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(1)
    host = [Column(values=torch.randint(0, 255, (n * 8,), dtype=torch.uint8, generator=g)
                   .pin_memory()) for _ in fields]
    rows = torch.empty(n * 816, dtype=torch.uint8).pin_memory()
    out = [Column(values=torch.empty(n * 8, dtype=torch.uint8).pin_memory()) for _ in fields]
    dcols = [Column(values=h.values.to(dev)) for h in host]
    drows = torch.empty(n * 816, dtype=torch.uint8, device=dev)
    enc = Encoders.bean(fields, device=dev)
    sh = enc._schema.handle
    lib = N.lib()
    keep: list = []
    hc = _c_host_columns(host, keep)
    ho = _c_host_columns(out, keep)
    dc = _c_columns(dcols, keep)
    s = torch.cuda.current_stream().cuda_stream
    b = n * (800 + 816)

    def ok(st):
        assert st == 0, N.last_error()

    def zc_enc():
        ok(lib.fury_row_encode(sh, hc, n, None, rows.data_ptr(), s))
        torch.cuda.synchronize()

    def zc_dec():
        ok(lib.fury_row_decode(sh, rows.data_ptr(), None, n, ho, s))
        torch.cuda.synchronize()

    def zc_in_enc():
        ok(lib.fury_row_encode(sh, hc, n, None, drows.data_ptr(), s))
        torch.cuda.synchronize()

    def zc_in_dec():
        ok(lib.fury_row_decode(sh, rows.data_ptr(), None, n, dc, s))
        torch.cuda.synchronize()

    def zc_out_enc():
        ok(lib.fury_row_encode(sh, dc, n, None, rows.data_ptr(), s))
        torch.cuda.synchronize()

    def zc_out_dec():
        ok(lib.fury_row_decode(sh, drows.data_ptr(), None, n, ho, s))
        torch.cuda.synchronize()

    def staged_enc():
        os.environ["FURY_HOST_STAGED"] = "1"
        enc.encode_host(host, n, rows=rows)
        del os.environ["FURY_HOST_STAGED"]

    def staged_dec():
        os.environ["FURY_HOST_STAGED"] = "1"
        enc.decode_host(rows, None, n, out=out)
        del os.environ["FURY_HOST_STAGED"]

    def api_enc():                      # the shipped API: pinned buffers -> fixed_direct
        enc.encode_host(host, n, rows=rows)

    def api_dec():
        enc.decode_host(rows, None, n, out=out)

    # correctness first: zero-copy encode == staged encode, zero-copy decode == columns
    staged_enc()
    ref = rows.clone()
    rows.zero_()
    zc_enc()
    assert torch.equal(rows, ref), "zero-copy encode differs"
    zc_dec()
    assert all(torch.equal(o.values, h.values) for o, h in zip(out, host)), "zero-copy decode"
    drows.copy_(rows)
    # the same API on ordinary (malloc'd) buffers pinned by fury_host_register, as a JVM's
    # DirectByteBuffers are, plain 4 KB pages and transparent huge pages (2 MB mappings)
    import mmap
    import numpy as np

    def registered(nbytes, huge):
        if huge:
            m = mmap.mmap(-1, nbytes + (2 << 20))
            m.madvise(mmap.MADV_HUGEPAGE)
            a = np.frombuffer(m, dtype=np.uint8)
            off = (-a.ctypes.data) % (2 << 20)
            a = a[off:off + nbytes]
            a[:] = 0                            # fault the pages in (huge where the kernel can)
        else:
            a = np.empty(nbytes, dtype=np.uint8)
        assert lib.fury_host_register(a.ctypes.data, a.nbytes) == 0, N.last_error()
        return a

    reg = {}
    for huge in (False, True):
        rc = [Column(values=registered(n * 8, huge)) for _ in fields]
        for c, h in zip(rc, host):
            c.values[:] = h.values.numpy()
        rr = registered(n * 816, huge)
        ro = [Column(values=registered(n * 8, huge)) for _ in fields]
        reg[huge] = (rc, rr, ro)

    def reg_leg(huge, dec):
        rc, rr, ro = reg[huge]
        if dec:
            return lambda: enc.decode_host(rr, None, n, out=ro)
        return lambda: enc.encode_host(rc, n, rows=rr)

    tiny = [Column(values=h.values[:64 * 8]) for h in host]

    def api_tiny():                     # per-call overhead: 64 rows through the direct path
        enc.encode_host(tiny, 64, rows=rows[:64 * 816])

    legs = {"staged_enc": staged_enc, "staged_dec": staged_dec, "api_enc": api_enc,
            "api_dec": api_dec, "zc_enc": zc_enc,
            "zc_dec": zc_dec, "zc_in_enc": zc_in_enc, "zc_in_dec": zc_in_dec,
            "zc_out_enc": zc_out_enc, "zc_out_dec": zc_out_dec,
            "reg4k_enc": reg_leg(False, False), "reg4k_dec": reg_leg(False, True),
            "reg2m_enc": reg_leg(True, False), "reg2m_dec": reg_leg(True, True),
            "api_tiny": api_tiny}
    res = {k: [] for k in legs}
    for _ in range(args.reps):
        for k, f in legs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            res[k].append(time.perf_counter() - t0)
    for huge in (False, True):
        assert np.array_equal(reg[huge][2][7].values, host[7].values.numpy()), "registered legs"
    ms = {k: round(statistics.median(v) * 1e3, 3) for k, v in res.items()}
    gb = {k: round(b / (ms[k] * 1e-3) / 1e9, 1) for k in legs}
    line = {"rows": n, "ms": ms, "GBps_algorithmic": gb}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
