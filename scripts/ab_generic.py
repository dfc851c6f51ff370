"""Timing of the nested-schema engines (rowenc.hip encode, walk.hip / levels.hip decode), on the
tests' 7-field nested schema (struct with list + string, list<list<int>>, map<string,int>,
list<struct>, list<string>, bool).  Columns come from beans (host, slow), repeated to --rows.

    python scripts/ab_generic.py [--rows 400000]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bytes(cols):
    t = 0
    for c in cols:
        for a in (c.values, c.validity, c.offsets):
            if a is not None:
                t += a.numel() * a.element_size()
        if c.child:
            t += _bytes(c.child)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=400_000)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--legs", default="2",
                    help="decode engines: 1 level engine, 2 row walk (tuning nested_decode), or a "
                         "JSON list of {tuning key: value} legs")
    args = ap.parse_args()
    import torch
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_device
    from tests.test_device import _nested_beans, _nested_fields
    fields = _nested_fields()
    base = _nested_beans(50_000, seed=1)
    beans = (base * (args.rows // len(base) + 1))[:args.rows]
    n = len(beans)
    dev = torch.device("cuda:0")
    cols = [column_to_device(c, dev) for c in beans_to_columns(fields, beans)]
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, n)
    out = enc.decode_batch(batch)
    torch.cuda.synchronize()

    def t(f):
        f()
        torch.cuda.synchronize()
        xs = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                f()
            b.record()
            torch.cuda.synchronize()
            xs.append(a.elapsed_time(b) / args.iters)
        return statistics.median(xs)
    import ctypes
    from fury_amd import _native as N
    if args.legs.startswith("["):          # JSON list of {tuning key: value} legs
        legs = json.loads(args.legs)
    else:
        legs = [{"nested_decode": int(x)} for x in args.legs.split(",")]
    ref = None
    keys = {k for leg in legs for k in leg}
    defaults = {k: N.lib().fury_get_tuning(k.encode()) for k in keys}
    for leg in legs:
        for k, v in defaults.items():         # every leg starts from the defaults
            assert N.lib().fury_set_tuning(k.encode(), int(v)) == 0, N.last_error()
        for k, v in leg.items():
            assert N.lib().fury_set_tuning(k.encode(), int(v)) == 0, N.last_error()
        b2 = enc.encode_batch(cols, n)
        d2 = enc.decode_batch(b2)
        torch.cuda.synchronize()
        got = (b2.rows.clone(), [x for c in d2 for x in (c.values, c.validity, c.offsets)])
        if ref is None:
            ref = got
        else:
            # value buffers carry an uninitialised pad past the last entry (<= 16 B): not compared
            same = torch.equal(ref[0], got[0]) and all(
                (x is None and y is None) or (x is not None and y is not None and x.shape == y.shape
                                              and torch.equal(x[:max(x.numel() - 16, 0)],
                                                              y[:max(y.numel() - 16, 0)]))
                for x, y in zip(ref[1], got[1]))
            print(json.dumps({"leg": leg, "equal_to_first": same}), flush=True)
        leg_run(args, t, enc, cols, n, batch, out, leg)


def leg_run(args, t, enc, cols, n, batch, out, leg):
    import ctypes
    import torch
    from fury_amd import _native as N
    enc_ms = t(lambda: enc.encode_batch(cols, n))
    dec_ms = t(lambda: enc.decode_batch(batch))
    # the pieces: measure (row sizes + scan), encode into sized rows, decode count pass
    # (fury_decode_prepare incl. its host read of the node totals), decode execute alone
    from fury_amd.encoder import _c_columns, _ptr
    L = N.lib()
    h = enc._schema.handle
    sh = torch.cuda.current_stream().cuda_stream
    offs = batch.row_offsets
    meas_ms = t(lambda: enc.measure_into(cols, n, offs))
    enc_only_ms = t(lambda: enc.encode_into(cols, n, batch.rows, offs))
    nn = L.fury_schema_num_nodes(h)
    e = (ctypes.c_int64 * nn)()
    b = (ctypes.c_int64 * nn)()

    def prep():
        p = ctypes.c_void_p()
        assert L.fury_decode_prepare(h, _ptr(batch.rows), _ptr(offs), n, e, b,
                                     ctypes.byref(p), sh) == 0
        return p

    def prep_destroy():
        L.fury_decode_plan_destroy(prep())

    prep_ms = t(prep_destroy)
    plan = prep()
    keep: list = []
    cc = _c_columns(out, keep)
    exec_ms = t(lambda: L.fury_decode_execute(plan, cc, 0, sh))
    L.fury_decode_plan_destroy(plan)
    cb = _bytes(cols)
    rb = batch.rows.numel() + 8 * (n + 1)
    print(json.dumps({"leg": leg, "pieces_ms": {"measure": round(meas_ms, 3), "encode": round(enc_only_ms, 3),
                                    "decode_prepare": round(prep_ms, 3),
                                    "decode_execute": round(exec_ms, 3)},
                      "execute_GBps": round((cb + rb) / exec_ms / 1e6, 1),"schema": "tests _nested_fields (7 fields, depth 3)", "rows": n,
                      "column_bytes": cb, "row_bytes": rb,
                      "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
                      "encode_GBps": round((cb + rb) / enc_ms / 1e6, 1),
                      "decode_GBps": round((cb + rb) / dec_ms / 1e6, 1),
                      "note": "wall per call incl. host syncs (measure + size reads)"}))


if __name__ == "__main__":
    main()
