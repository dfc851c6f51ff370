"""Timing of the stream framing path in ONE process (HIP events, interleaved rounds).

    python scripts/ab_frame.py [--workload struct100|mixed|nested] [--rows N] [--rounds 5]

Legs: frame (Encoders.encode(MemoryBuffer, T) for every row), unframe by the speculative parallel
parse (tuning unframe=0), and — on a bounded prefix, since it is one dependent HBM round trip
per frame — by the sequential walk (unframe=1).  Algorithmic bytes: frame reads the rows (+ row
offsets) and writes rows + 12 B per frame; unframe reads the stream and writes rows + row offsets.
Also times the Arrow IPC RecordBatch message of the decoded columns (leg "ipc": body gathered on
the device, reads the columns and writes the message).  Prints one JSON line with median ms
and GB/s per leg.
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
    ap.add_argument("--workload", default="struct100")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--walk-rows", type=int, default=20000)
    args = ap.parse_args()
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import ArrowWriter, Encoders, ipc_record_batch_message
    from bench import DEFAULT_ROWS, make_device_columns
    from fury_amd.workloads import SCHEMAS
    dev = torch.device("cuda:0")
    name = args.workload
    fields = SCHEMAS[name]
    n = args.rows or DEFAULT_ROWS[name]
    cols = make_device_columns(name, fields, n, 0, dev)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(cols, n)
    stream, _ = enc.frame(batch)
    got = enc.unframe(stream, n)
    assert torch.equal(got.rows, batch.rows), "unframe round trip"
    walks0 = N.lib().fury_get_tuning(b"unframe_walks")
    nw = min(n, args.walk_rows)
    wstream = stream[:int(batch.row_offsets[nw].item()) + 12 * nw] if batch.row_offsets is not None \
        else stream[:(batch.rows.numel() // n) * nw + 12 * nw]
    row_bytes = batch.rows.numel()
    offs_bytes = 0 if batch.row_offsets is None else 8 * (n + 1)
    aw = ArrowWriter(enc)
    aw.write(batch)
    dcols = aw.finish()
    ipc_len = ipc_record_batch_message(enc, dcols, n).numel()
    # round 2: the same stream at a 1-byte offset (Java frames at any writerIndex), and a stream
    # whose payloads spell a plausible header every ~100 frames (parallel repair, no walk)
    shifted_buf = torch.empty(stream.numel() + 64, dtype=torch.uint8, device=dev)
    shifted_buf[1:1 + stream.numel()] = stream
    shifted = shifted_buf[1:1 + stream.numel()]
    assert torch.equal(enc.unframe(shifted, n).rows, batch.rows), "unframe at offset 1"
    fake = stream.clone()
    if batch.row_offsets is not None:
        fo = (batch.row_offsets[:-1] + 12 * torch.arange(n, device=dev))
    else:
        fo = torch.arange(n, device=dev, dtype=torch.int64) * (batch.rows.numel() // n + 12)
    pick = fo[3::97] + 12 + 16                      # 8-byte slot 1 of every 97th row
    hdr = torch.tensor(list((24).to_bytes(4, "little")) +
                       list((enc.schema_hash & (2**64 - 1)).to_bytes(8, "little")),
                       dtype=torch.uint8, device=dev)
    for j in range(12):
        fake[pick + j] = hdr[j]
    rep0 = N.lib().fury_get_tuning(b"unframe_repairs")
    fr = enc.unframe(fake, n)
    assert N.lib().fury_get_tuning(b"unframe_repairs") == rep0 + 1, "fake headers not repaired"
    fake_rows = fr.rows.clone()
    legs = {
        "ipc": (lambda: ipc_record_batch_message(enc, dcols, n), 2 * ipc_len),
        "frame": (lambda: enc.frame(batch), row_bytes + offs_bytes + stream.numel() + 8 * (n + 1)),
        "unframe": (lambda: enc.unframe(stream, n), stream.numel() + row_bytes + 8 * (n + 1)),
        "unframe_offset1": (lambda: enc.unframe(shifted, n),
                            stream.numel() + row_bytes + 8 * (n + 1)),
        "unframe_repair": (lambda: enc.unframe(fake, n), stream.numel() + row_bytes + 8 * (n + 1)),
    }
    res = {k: [] for k in legs}
    res["unframe_walk"] = []
    for _ in range(args.rounds):
        for k, (fn, _b) in legs.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / args.iters)
        N.lib().fury_set_tuning(b"unframe", 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        enc.unframe(wstream, nw)
        e1.record()
        torch.cuda.synchronize()
        N.lib().fury_set_tuning(b"unframe", 0)
        res["unframe_walk"].append(e0.elapsed_time(e1))
    assert torch.equal(enc.unframe(fake, n).rows, fake_rows)
    walks = N.lib().fury_get_tuning(b"unframe_walks") - walks0
    assert walks == args.rounds, f"speculative parse fell back {walks - args.rounds} times"
    ms = {k: round(statistics.median(v), 4) for k, v in res.items()}
    gbps = {k: round(b / (ms[k] * 1e-3) / 1e9, 1) for k, (_f, b) in legs.items()}
    wb = wstream.numel() + (wstream.numel() - 12 * nw) + 8 * (nw + 1)
    gbps["unframe_walk"] = round(wb / (ms["unframe_walk"] * 1e-3) / 1e9, 3)
    print(json.dumps({"workload": name, "rows": n, "stream_bytes": stream.numel(),
                      "walk_rows": nw, "ms": ms, "GBps": gbps,
                      "note": "ms include the host sync of unframe's status return"}))


if __name__ == "__main__":
    main()
