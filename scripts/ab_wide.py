"""Wide flat variable-length schemas (17..256 fields): the 33-field schema of
tests/test_device.py::_wide_fields at --rows rows, timed with HIP events over bound-free calls:
encode (fury_row_encode_measured), flat decode (fury_row_decode: decode_var_kernel) and the plan
decode (fury_decode_prepare + execute: the row walk) -- GB/s of column + row bytes.

    python scripts/ab_wide.py --rows 5000000 --ncols 33
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=5_000_000)
    ap.add_argument("--ncols", type=int, default=33)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--str-max", type=int, default=24)
    ap.add_argument("--tune", action="append", default=[],
                    help="key=value fury_set_tuning before timing (repeatable)")
    ap.add_argument("--no-plan", action="store_true", help="skip the plan-API decode leg")
    ap.add_argument("--flat", type=int, default=0, help="id + this many STRING fields instead of "
                    "tests' _wide_fields(--ncols)")
    ap.add_argument("--enc-engines", default="", help="comma list of wide_enc_engine settings: "
                    "encode_ms per setting, rows checked equal to the first")
    args = ap.parse_args()
    import torch
    from fury_amd.encoder import Encoders, _tree_bytes, column_to_device
    from fury_amd.workloads import gen_columns
    from tests.test_device import _wide_fields
    from fury_amd import _native as N
    for kv in args.tune:
        k, v = kv.split("=")
        assert N.lib().fury_set_tuning(k.encode(), int(v)) == 0, N.last_error()
    from fury_amd import types as T
    fields = (([T.not_null_field("id", T.INT64)] + [T.field(f"s{i:03d}", T.STRING) for i in range(args.flat)])
              if args.flat else _wide_fields(args.ncols))
    n = args.rows
    host = gen_columns("wide", fields, n, seed=7, null_pct=10, str_max=args.str_max, list_max=6)
    dev = torch.device("cuda:0")
    cols = [column_to_device(c, dev) for c in host]
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, n)
    row_bytes = int(batch.rows.numel())
    col_bytes = _tree_bytes(host)
    alg = row_bytes + col_bytes
    rows = torch.empty_like(batch.rows)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(args.iters):
            s.record()
            fn()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e))
        return best
    res = {"ncols": len(fields), "rows": n, "row_bytes": row_bytes, "column_bytes": col_bytes}
    if args.enc_engines:
        ref = None
        for m in [int(x) for x in args.enc_engines.split(",")]:
            assert N.lib().fury_set_tuning(b"wide_enc_engine", m) == 0
            rows.zero_()
            res[f"encode_ms_engine{m}"] = timed(lambda: enc.encode_measured_into(cols, n, rows, offs))
            torch.cuda.synchronize()
            got = rows[:row_bytes].clone()
            if ref is None:
                ref = got
            else:
                res[f"rows_equal_engine{m}"] = bool(torch.equal(ref, got))
        assert N.lib().fury_set_tuning(b"wide_enc_engine", 1) == 0
    out = enc.decode_batch(batch)                       # allocated once (bound sizing)
    res["encode_ms"] = timed(lambda: enc.encode_measured_into(cols, n, rows, offs))
    res["decode_flat_ms"] = timed(lambda: enc.decode_batch(batch, out=out))
    # the API users call: sizing included (round 6: the plan API -- count pass once)
    res["decode_batch_ms"] = timed(lambda: enc.decode_batch(batch))
    # one device pass into the preallocated columns (no sizing pass, no host sync): the kernels
    res["decode_into_ms"] = timed(lambda: enc.decode_into(batch, out))
    legs = ["encode", "decode_flat", "decode_batch", "decode_into"]
    if not args.no_plan:
        res["decode_plan_ms"] = timed(lambda: enc._decode_nested(batch, True, False, None))
        legs.append("decode_plan")
    res["tune"] = args.tune
    for k in legs:
        res[k + "_TBps"] = round(alg / (res[k + "_ms"] * 1e-3) / 1e12, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
