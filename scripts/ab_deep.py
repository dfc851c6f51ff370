"""Deep-schema decode A/B: nested_decode 2 against 1 on the tests' _deep_fields(levels) schema.  A
base batch of --base beans is encoded once and its rows tiled on the device to --rows rows.
(profiles/r05_deep_walk_vs_levels.jsonl: a build whose row walk continued past 5 levels on an
explicit stack -- mode 2 -- against the level engine -- mode 1; that walk was removed.)

    python scripts/ab_deep.py --levels 9,12,20 --rows 1000000
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
    ap.add_argument("--levels", default="9,12,20")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--base", type=int, default=20_000)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--wide", default="", help="comma list of counted-node counts: a bean of that "
                    "many STRING fields plus a list of structs (the walk's 64-counted-node limit)")
    ap.add_argument("--modes", default="3,1", help="nested_decode settings (3 tile BFS, 2 row "
                    "walk -- at most 5 levels, else the level engine --, 1 level engine)")
    ap.add_argument("--flat", default="", help="comma list of STRING-field counts: a flat bean of "
                    "id + that many STRING fields (--modes: wide_engine settings, 1 wide tiles, "
                    "2 row walk)")
    ap.add_argument("--wide33", action="store_true", help="also tests' _wide_fields(33) (wide_engine "
                    "legs as --flat)")
    ap.add_argument("--tune", default="", help="key=value,... tunings set first (e.g. walk_group_k=8)")
    args = ap.parse_args()
    import numpy as np
    import torch
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, RowBatch, column_to_device
    from tests.test_tree import _beans, _deep_fields
    dev = torch.device("cuda:0")
    L = N.lib()
    for kv in [x for x in args.tune.split(",") if x]:
        k, v = kv.split("=")
        assert L.fury_set_tuning(k.encode(), int(v)) == 0, N.last_error()
    from fury_amd import types as T
    cases = [("levels", int(x)) for x in args.levels.split(",") if x]
    cases += [("counted", int(x)) for x in args.wide.split(",") if x]
    cases += [("flat", int(x)) for x in args.flat.split(",") if x]
    if args.wide33:
        cases.append(("wide33", 33))
    for kind, levels in cases:
        if kind == "levels":
            fields = _deep_fields(levels)
        elif kind == "flat":
            fields = ([T.not_null_field("id", T.INT64)] +
                      [T.field(f"s{i:03d}", T.STRING) for i in range(levels)])
        elif kind == "wide33":
            from tests.test_device import _wide_fields
            fields = _wide_fields(33)
        else:
            fields = ([T.not_null_field("id", T.INT64)] +
                      [T.field(f"s{i:03d}", T.STRING) for i in range(levels - 2)] +
                      [T.Field("t", T.LIST, True, (T.struct_field("item", [T.field("x", T.STRING),
                                                                         T.field("y", T.INT32)]),))])
        beans = _beans(fields, args.base, levels)
        enc = Encoders.bean(fields, device=dev)
        b0 = enc.encode_batch([column_to_device(c, dev) for c in beans_to_columns(fields, beans)],
                              args.base)
        reps = max(1, args.rows // args.base)
        n = reps * args.base
        tot = int(b0.row_offsets[-1].item())
        rows = b0.rows.repeat(reps)
        offs = torch.cat([b0.row_offsets[:-1] + i * tot for i in range(reps)] +
                         [torch.tensor([reps * tot], dtype=torch.int64, device=dev)])
        batch = RowBatch(rows, offs, n, enc.schema_hash)
        res = {kind: levels, "rows": n, "row_bytes": reps * tot, "tune": args.tune}
        ref = None
        key = b"wide_engine" if kind in ("flat", "wide33") else b"nested_decode"
        for mode in [int(x) for x in args.modes.split(",")]:
            assert L.fury_set_tuning(key, mode) == 0
            out = enc.decode_batch(batch)
            torch.cuda.synchronize()
            got = [x for c in out for x in (c.values, c.validity, c.offsets)]
            if ref is None:
                ref = got
            else:
                res[f"equal_mode{mode}"] = all((x is None and y is None) or (
                    x is not None and y is not None and x.shape == y.shape and
                    torch.equal(x[:max(x.numel() - 16, 0)], y[:max(y.numel() - 16, 0)]))
                    for x, y in zip(ref, got))
            xs = []
            for _ in range(3):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.iters):
                    enc.decode_batch(batch)
                b.record()
                torch.cuda.synchronize()
                xs.append(a.elapsed_time(b) / args.iters)
            res[f"decode_ms_mode{mode}"] = round(statistics.median(xs), 3)
        assert L.fury_set_tuning(b"nested_decode", 2) == 0
        assert L.fury_set_tuning(b"wide_engine", 1) == 0
        res["bfs_fallbacks"] = L.fury_get_tuning(b"bfs_fallbacks")
        print(json.dumps(res), flush=True)
    del np


if __name__ == "__main__":
    main()
