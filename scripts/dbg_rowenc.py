"""Row-walk encode (nested_encode 3 / 4) against the interpreter (2) on the depth-3 nested rows of
the tests: first differing bytes, their rows and tiles.

    python scripts/dbg_rowenc.py --rows 4000000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--modes", default="3,4")
    args = ap.parse_args()
    import numpy as np
    import torch
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    from tests.test_device import _nested_beans, _nested_fields
    L = N.lib()
    fields = _nested_fields()
    base = _nested_beans(50_000, seed=1)
    n = args.rows
    beans = (base * (n // len(base) + 1))[:n]
    dev = torch.device("cuda:0")
    cols = [column_to_device(c, dev) for c in beans_to_columns(fields, beans)]
    enc = Encoders.bean(fields, device=dev)
    assert L.fury_set_tuning(b"nested_encode", 2) == 0
    ref = enc.encode_batch(cols, n)
    torch.cuda.synchronize()
    dref = enc.decode_batch(ref)
    torch.cuda.synchronize()
    dref = [(x.clone() if x is not None else None) for c in dref for x in (c.values, c.validity, c.offsets)]
    ro = ref.row_offsets.cpu().numpy()
    rr = ref.rows.cpu().numpy()
    for m in [int(x) for x in args.modes.split(",")]:
        assert L.fury_set_tuning(b"nested_encode", m) == 0
        b = enc.encode_batch(cols, n)
        torch.cuda.synchronize()
        go = b.row_offsets.cpu().numpy()
        gr = b.rows.cpu().numpy()
        out = {"mode": m, "offsets_equal": bool(np.array_equal(go, ro)),
               "rows_len": [int(gr.size), int(rr.size)]}
        if gr.size == rr.size:
            d = np.nonzero(gr != rr)[0]
            out["diff_bytes"] = int(d.size)
            if d.size:
                rows_hit = np.searchsorted(ro, d, side="right") - 1
                ur = np.unique(rows_hit)
                out["diff_rows"] = int(ur.size)
                out["first_rows"] = ur[:10].tolist()
                tiles = np.unique(ur // 256)
                out["diff_tiles"] = int(tiles.size)
                spans = [int(ro[min((t + 1) * 256, n)] - ro[t * 256]) for t in tiles[:10]]
                out["tile_spans"] = spans
                r = int(ur[0])
                lo, hi = int(ro[r]), int(ro[r + 1])
                out["row0"] = {"row": r, "size": hi - lo,
                               "at": (d[d < hi][:8] - lo).tolist(),
                               "want": rr[lo:hi][:160].tolist(), "got": gr[lo:hi][:160].tolist()}
                out["bean"] = str(beans[r])
        dd = enc.decode_batch(b)
        torch.cuda.synchronize()
        dd = [x for c in dd for x in (c.values, c.validity, c.offsets)]
        cd = []
        for i, (x, y) in enumerate(zip(dref, dd)):
            if (x is None) != (y is None):
                cd.append([i, "none"])
            elif x is not None and not torch.equal(x, y):
                if x.shape != y.shape:
                    cd.append([i, "shape", list(x.shape), list(y.shape)])
                else:
                    xv, yv = x.cpu().numpy().view(np.uint8), y.cpu().numpy().view(np.uint8)
                    w = np.nonzero(xv != yv)[0]
                    cd.append([i, int(w.size), int(xv.size), w[:6].tolist(), xv[w[:6]].tolist(), yv[w[:6]].tolist()])
        out["decode_diffs"] = cd
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
