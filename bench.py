"""Headline benchmark: device-resident Fury row-format encode+decode throughput (BASELINE.json).

One step = encode one batch of Arrow-style columns into Fury rows (HBM -> HBM) + decode those
rows back into columns, through the HIP kernels behind the C ABI.  Default workload is
configs[1]: 1M rows of Struct-100 (f00..f99, int64/float64, non-null) per GPU.  With --gpus N
there is one process per GPU: started by torch.distributed.run (RANK/WORLD_SIZE in the
environment, which must agree with --gpus), or, when run directly, spawned by this script
through fury_amd.shard.launch before it touches the GPU.  Every rank runs its own independent
shard of global rows, no data-path collective (rows are independent): --rows R per GPU (weak
scaling, default) or --total-rows T split into contiguous shards (strong scaling; C5 =
--total-rows 100000000 --gpus 8).

Prints ONE JSON line (rank 0).  `value` = total algorithmic bytes of all ranks / max-over-ranks
time (encode reads 800 B + writes 816 B per row, decode the reverse; 3,232 B/row).
Also reports the dominant kernel's roofline (HIP events on the launch stream) and the CPU
baseline (oracle C restatement of the Java writer/reader, 1 thread, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "row-format encode+decode GB/s (device-resident), Struct-100, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# CPU baseline threads: the GPU box's CPU share of one GPU job -- OMP_NUM_THREADS, which the box
# sets to that share (16; nproc and the affinity mask show the whole 256-thread machine, and jobs
# must size their pools to the share), else the affinity mask split over a node's 8 GPUs.
def cpu_threads():
    mine, _ = _host_cpus()
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return min(int(env), mine)
    return max(1, mine // 8)
DEFAULT_ROWS = {"struct100": 1_000_000, "mixed": 10_000_000, "nested": 4_000_000}


def _parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rows", type=int, default=None,
                   help="rows per GPU, weak scaling (default: BASELINE config size: struct100 1M, "
                        "mixed 10M, nested 4M)")
    p.add_argument("--total-rows", type=int, default=None,
                   help="strong scaling: this many rows in total, split into contiguous "
                        "near-equal shards over the GPUs (C5: --total-rows 100000000 --gpus 8)")
    p.add_argument("--share-gpus", action="store_true",
                   help="rehearsal only: allow more ranks than visible GPUs (ranks share them)")
    p.add_argument("--workload", default="struct100", choices=["struct100", "mixed", "nested"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-rows", type=int, default=None,
                   help="rows of the CPU baseline's batch (default: the bench batch, C2 = 1M)")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-verify", action="store_true",
                   help="diagnostic runs only: skip the post-timing correctness spot check")
    a = p.parse_args(argv)
    if a.rows is None:
        a.rows = DEFAULT_ROWS[a.workload]
    return a


def _buffers(col):
    out = [t for t in (col.values, col.validity, col.offsets) if t is not None]
    for c in col.child or []:
        out.extend(_buffers(c))
    return out


def _nbytes(cols):
    return sum(t.numel() * t.element_size() for c in cols for t in _buffers(c))


def make_device_columns(name, fields, rows, start, dev):
    """Synthetic columns resident in HBM, SplitMix64 keyed by (column, GLOBAL row index), so a
    shard holds exactly the rows a single-GPU run over the whole range would.  Struct-100 is
    generated on the device (fury_amd.workloads.gen_columns_torch, bit-identical to the host
    generator, tests/test_workloads.py)."""
    from fury_amd.workloads import gen_columns_torch
    return gen_columns_torch(name, fields, rows, seed=1234, start=start, device=dev)


def _host_cpus():
    """(CPUs this process may run on, CPUs the machine has): the box's nproc shows the whole
    machine, the affinity mask the share a GPU job gets."""
    try:
        mine = len(os.sched_getaffinity(0))
    except AttributeError:
        mine = os.cpu_count() or 1
    return mine, os.cpu_count() or 1


def cpu_baseline(name, fields, budget_s, sample_rows):
    """Oracle C restatement of the Java writer/reader (kind "port") timed on this host on the
    bench workload's own batch (``sample_rows`` rows, default = the full C2 batch of 1M rows;
    1M rows of the mixed / nested batches): 1 thread over the whole batch, then cpu_threads()
    threads each encoding + decoding a contiguous slice of it (one encoder per thread, like the
    reference's thread-confined RowEncoder; variable-length slices carry rebased offsets; ctypes
    releases the GIL inside the C calls)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    from fury_amd.workloads import gen_columns, slice_columns
    var = name != "struct100"
    host = gen_columns(name, fields, sample_rows, seed=99)

    def nbytes(cols):
        return sum(a.nbytes for c in cols for a in (c.values, c.validity, c.offsets)
                   if a is not None) + sum(nbytes(c.child) for c in cols if c.child)

    rows, offs = O.encode(fields, host, sample_rows)
    per_pass = 2 * (nbytes(host) + rows.nbytes + (offs.nbytes if var else 0))
    del rows, offs
    t0 = time.perf_counter()
    reps = 0
    while True:
        r, o = O.encode(fields, host, sample_rows)
        O.decode(fields, r, o if var else None, sample_rows, with_validity=False, sizing="bound")
        del r, o
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    mine, machine = _host_cpus()
    out = {"value": round(per_pass * reps / dt / 1e9, 4), "unit": "GB/s", "cores": 1,
           "kind": "port",
           "sample": f"{reps} x encode+decode of the {sample_rows}-row {name} batch "
                     f"(oracle/row_oracle.c, toRow/fromRow restatement, 1 thread) in {dt:.1f} s",
           "host_cpus": {"affinity": mine, "nproc": machine}}
    threads = cpu_threads()
    bounds = [(sample_rows * t // threads, sample_rows * (t + 1) // threads) for t in range(threads)]
    parts = [slice_columns(fields, host, b, e) for b, e in bounds]
    stop = time.perf_counter() + budget_s / 2

    def work(t):
        k, m = 0, bounds[t][1] - bounds[t][0]
        while time.perf_counter() < stop:
            r, o = O.encode(fields, parts[t], m)
            O.decode(fields, r, o if var else None, m, with_validity=False, sizing="bound")
            k += 1
        return k
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        laps = list(ex.map(work, range(threads)))
    dt = time.perf_counter() - t0
    done = sum(laps) / threads            # whole-batch passes (every slice the same size +-1)
    out["threads"] = {"value": round(per_pass * done / dt / 1e9, 4), "unit": "GB/s",
                      "cores": threads,
                      "sample": f"{sum(laps)} x encode+decode of 1/{threads} slices of the "
                                f"{sample_rows}-row batch on {threads} threads in {dt:.1f} s",
                      "why_cores": "the box's CPU share of one GPU job (OMP_NUM_THREADS); "
                                   "host_cpus shows the machine"}
    return out


def _worker(argv):
    """One rank of a `bench.py --gpus N` run started by fury_amd.shard.launch."""
    run(_parse(argv))


def main():
    args = _parse()
    if "RANK" not in os.environ and args.gpus > 1:
        # started directly with --gpus N: one worker process per GPU (spawned before this
        # process touches the GPU), rank 0 prints the JSON line
        from fury_amd.shard import launch
        launch(args.gpus, _worker, (sys.argv[1:],))
        return
    run(args)


def run(args):
    import torch

    from fury_amd.shard import Orchestrator, from_env, strong_shard, weak_shard
    r = from_env()
    world, rank, local = r.world, r.rank, r.local
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # orchestration only (gloo barrier + max of timings); the data path has no collective
    orch = Orchestrator(r)
    # one process per GPU; sharing a GPU between ranks only as an explicit rehearsal
    ndev = torch.cuda.device_count()
    if ndev < world and not args.share_gpus:
        raise SystemExit(f"bench.py: {world} ranks but {ndev} visible GPUs "
                         "(--share-gpus for a rehearsal)")
    shared = ndev < world                       # --share-gpus rehearsal: ranks share devices
    local = local % ndev if ndev else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from fury_amd.encoder import Encoders
    from fury_amd.workloads import SCHEMAS
    fields = SCHEMAS[args.workload]
    enc = Encoders.bean(fields, device=dev)
    if args.total_rows is not None:
        start, n = strong_shard(args.total_rows, world, rank)
        scaling = "strong"
    else:
        start, n = weak_shard(args.rows, rank)
        scaling = "weak"
    cols = make_device_columns(args.workload, fields, n, start, dev)
    out_cols = enc.alloc_columns(n, validity=False) if enc.schema().is_fixed else None
    stream = torch.cuda.current_stream()

    # pre-size the row buffer once (measure for var-length schemas)
    offs = enc.measure(cols, n)
    total_row_bytes = n * enc.schema().fixed_size if offs is None else int(offs[n].item())
    rows = torch.empty(max(total_row_bytes, 16), dtype=torch.uint8, device=dev)
    from fury_amd.encoder import RowBatch
    batch = RowBatch(rows[:total_row_bytes], offs, n, enc.schema_hash)

    var_out = None
    if out_cols is None:      # size the variable-length outputs once (first decode syncs)
        enc.encode_into(cols, n, batch.rows, batch.row_offsets, stream=stream)
        var_out = enc.decode_batch(batch, validity=True, stream=stream)
    col_bytes = _nbytes(cols)
    row_bytes = total_row_bytes + (0 if offs is None else offs.numel() * 8)
    enc_bytes = col_bytes + row_bytes           # read columns, write rows
    dec_bytes = row_bytes + col_bytes           # read rows, write columns
    step_bytes = enc_bytes + dec_bytes

    # the same calls as encode_measured_into / encode_into / decode_into, argument blocks built
    # once (RowEncoder.bind_*): per-call Python work must not starve the GPU between launches
    if offs is not None:           # variable-length rows: one pass computes sizes + rows
        encode = enc.bind_encode(cols, n, batch.rows, offs, stream=stream, measured=True)
    else:
        encode = enc.bind_encode(cols, n, batch.rows, None, stream=stream)
    # fixed width: the decode into preallocated columns; C4 names row->Arrow conversion
    # (ArrowWriter's fury_rows_to_arrow)
    decode = enc.bind_decode(batch, out_cols if out_cols is not None else var_out, stream=stream,
                             arrow=args.workload == "nested")

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        encode()
        if ev is not None:
            ev[1].record(stream)
        decode()
        if ev is not None:
            ev[2].record(stream)

    # the box's achievable streaming copy, same device, same stream, before the timed loop
    # (VERDICT r5 item 6): separates a slow box from a slow kernel in the roofline line
    copy = copy_rate(dev, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    orch.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0       # this rank's K steps; the max over ranks is taken below
    orch.barrier()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps

    dt_max = orch.max(dt)

    # correctness spot check after timing (cheap, device-side): decoded == input
    if args.no_verify:
        pass
    elif args.workload == "struct100":
        for c, d in zip(cols[:4], out_cols[:4]):
            assert torch.equal(c.values.view(torch.uint8), d.values), "decode mismatch"
    else:
        assert int(offs[n].item()) == total_row_bytes, "row buffer overflow"
        enc.check_capacity(var_out, n)
        from fury_amd import _native as N
        assert N.lib().fury_get_tuning(b"lookback_timeouts") == 0, "look-back gave up"
        for c, d in zip(cols, var_out):
            if c.offsets is not None and c.child is None:
                assert torch.equal(c.offsets, d.offsets), "decode offsets mismatch"

    e2e = None
    if world == 1 and not args.no_e2e and args.workload == "struct100":
        e2e = end_to_end(enc, cols, n, dev, stream)
    elif world == 1 and not args.no_e2e:
        e2e = end_to_end_var(enc, cols, n, int(offs[n].item()))

    # every rank's bytes and rows (shards may differ by one row under strong scaling)
    all_bytes = sum(orch.gather_ints(int(step_bytes)))
    all_rows = sum(orch.gather_ints(int(n)))
    all_row_bytes = sum(orch.gather_ints(int(total_row_bytes)))
    if rank != 0:
        orch.close()
        return
    dominant = ("encode", enc_ms, enc_bytes) if enc_ms >= dec_ms else ("decode", dec_ms, dec_bytes)
    achieved = dominant[2] / (dominant[1] * 1e-3) / 1e9
    traffic = None
    # PMC traffic (scripts/pmc.sh, scripts/pmc_var_traffic.sh) applies to the same workload and size
    pmc_file = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc_file) and n == DEFAULT_ROWS[args.workload]:
        pm = json.load(open(pmc_file))
        traffic = pm.get(f"{dominant[0]}_hbm_bytes_per_launch")
    data = "synthetic SplitMix64 columns keyed by (column, global row) generated in HBM; no dataset"
    config = {"workload": {"struct100": "Struct-100 encode+decode (configs[1])",
                           "mixed": "mixed int32/int64/double + 3 utf8 + nulls (configs[2])",
                           "nested": "id/score + list<int64>: encode + row->Arrow columns "
                                     "(ArrowWriter = fury_rows_to_arrow) (configs[3])"
                           }[args.workload],
              "rows_per_gpu": n, "row_bytes": enc.schema().fixed_size if offs is None
              else round(total_row_bytes / max(n, 1), 2),
              "algorithmic_bytes_per_step_per_gpu": step_bytes,
              "parallelism": f"{world} independent shard(s), no collective"}
    if args.total_rows is not None:
        config["total_rows"] = args.total_rows
        if args.workload == "struct100" and args.total_rows == 100_000_000:
            config["workload"] = "Struct-100 encode+decode, 100M rows sharded over the GPUs " \
                                 "(configs[4])"
    line = {
        "metric": METRIC,
        "value": round(all_bytes * args.steps / dt_max / 1e9, 2),
        "unit": "GB/s",
        # distinct devices: a --share-gpus rehearsal runs `world` ranks on fewer GPUs and is marked
        # so that it cannot be read as a scaling point
        "n_gpus": min(world, ndev) if shared else world,
        "ranks": world,
        "shared_gpus": shared,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int64" if args.workload == "struct100" else "u8",
        "data": data,
        "config": config,
        # row bytes per second beside the algorithmic bytes (information only)
        "rows": {"rows_per_s": round(all_rows * args.steps / dt_max, 1),
                 "row_GBps": round(2 * all_row_bytes * args.steps / dt_max / 1e9, 2),
                 "what": "rows encoded+decoded per second; row bytes written+read per second"},
        "roofline": {"bound": "hbm", "kernel": dominant[0], "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                     "encode_GBps": round(enc_bytes / (enc_ms * 1e-3) / 1e9, 1),
                     "decode_GBps": round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1),
                     "copy_GBps": copy["GBps"],
                     "frac_of_copy": round(achieved / copy["GBps"], 4),
                     "copy": copy["what"]},
    }
    if shared:
        line["rehearsal"] = (f"{world} ranks shared {min(world, ndev)} GPU(s) (--share-gpus): a "
                             "check of the multi-rank path, not a multi-GPU measurement")
    if e2e is not None:
        line["e2e_pcie"] = e2e
    if world == 1 and not args.no_cpu_baseline:     # the CPU baseline is an N=1 figure
        line["cpu_baseline"] = cpu_baseline(args.workload, fields, args.cpu_seconds,
                                            args.cpu_rows or min(n, 1_000_000))
    print(json.dumps(line), flush=True)
    orch.close()


def copy_rate(dev, stream, nbytes=1 << 30, reps=10):
    """Achievable HBM copy on this box: fury_hbm_copy (16-B non-temporal loads + stores, the
    library's own kernel) of a 1 GiB buffer, read + write bytes per second, HIP events on the bench
    stream, median of `reps` launches after one warm-up."""
    import statistics
    import torch
    from fury_amd import _native as N
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    src.fill_(7)
    L = N.lib()
    sh = stream.cuda_stream

    def launch():
        assert L.fury_hbm_copy(dst.data_ptr(), src.data_ptr(), nbytes, sh) == 0, N.last_error()
    launch()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        launch()
        b.record(stream)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    t = statistics.median(ms)
    del src, dst
    torch.cuda.empty_cache()
    return {"GBps": round(2 * nbytes / (t * 1e-3) / 1e9, 1),
            "what": f"fury_hbm_copy of {nbytes >> 20} MiB (read + write bytes / s, 16-B "
                    f"non-temporal, median of {reps} launches, same device and stream)"}


def end_to_end(enc, cols, n, dev, stream):
    """Host columns -> rows in host memory -> columns in host memory through the host-memory
    batch path a JVM caller uses (fury_row_encode_host / fury_row_decode_host).  Two kinds of
    host buffers: pinned allocations (fury_host_alloc = hipHostMalloc; GpuRowEncoder.allocatePinned
    on the JVM) — the headline `GBps_algorithmic` — and ordinary 4 KB-page allocations pinned in
    place with fury_host_register (hipHostRegister; a DirectByteBuffer registered as is).  Both
    take the direct path (the kernels read and write host memory over PCIe).  The
    PCIe-inclusive rate reported in DESIGN.md, never `value`."""
    import numpy as np
    import torch
    from fury_amd import _native as N
    from fury_amd.encoder import host_empty
    from fury_amd.workloads import Column
    fixed = enc.schema().fixed_size
    L = N.lib()
    src = [c.values.view(torch.uint8).cpu().numpy() for c in cols]

    def run(alloc):
        host_cols = [Column(values=alloc(n * 8)) for _ in cols]
        for h, v in zip(host_cols, src):
            h.values[:] = v
        host_rows = alloc(n * fixed)
        out = [Column(values=alloc(n * 8)) for _ in cols]
        d0 = L.fury_get_tuning(b"host_direct")
        enc.encode_host(host_cols, n, rows=host_rows)      # warm-up (streams, pool)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            enc.encode_host(host_cols, n, rows=host_rows)
            enc.decode_host(host_rows, None, n, out=out)
        dt = (time.perf_counter() - t0) / reps
        assert L.fury_get_tuning(b"host_direct") == d0 + 1 + 2 * reps, "staged, not direct"
        for k in (0, len(cols) // 2, len(cols) - 1):
            assert np.array_equal(out[k].values, host_cols[k].values), "host-path round trip"
        return dt

    registered = []

    def reg_alloc(nbytes):
        a = np.empty(nbytes, dtype=np.uint8)
        assert L.fury_host_register(a.ctypes.data, a.nbytes) == 0, N.last_error()
        registered.append(a)
        return a

    alg = 2 * (n * 800 + n * fixed)
    dt = run(host_empty)
    try:
        dt_reg = run(reg_alloc)
    finally:
        for a in registered:
            L.fury_host_unregister(a.ctypes.data)
    return {"GBps_algorithmic": round(alg / dt / 1e9, 2), "ms_per_step": round(dt * 1e3, 2),
            "registered_GBps_algorithmic": round(alg / dt_reg / 1e9, 2),
            "what": "host columns in fury_host_alloc (hipHostMalloc) buffers -> "
                    "fury_row_encode_host -> host rows -> fury_row_decode_host -> host columns, "
                    "direct (kernels on host memory over PCIe); registered_*: the same with "
                    "malloc'd buffers pinned by fury_host_register (4 KB pages)"}


def end_to_end_var(enc, cols, n, total_rows):
    """The variable-length workloads' host-memory round trip: host columns -> fury_row_encode_host
    -> host rows + row offsets -> fury_row_decode_host -> host columns, every buffer a
    fury_host_alloc (pinned) allocation of exactly the size the batch needs.  PCIe-inclusive, for
    DESIGN.md; never `value`."""
    import numpy as np
    import torch
    from fury_amd.encoder import host_empty
    from fury_amd.workloads import Column

    def pinned(t, dtype=np.uint8):
        if t is None:
            return None
        a = host_empty(t.numel() * t.element_size())
        a[:] = t.contiguous().view(torch.uint8).cpu().numpy()
        return a.view(dtype)

    def tree(c, fill):
        ch = [tree(x, fill) for x in c.child] if c.child else None
        if fill:
            return Column(values=pinned(c.values), validity=pinned(c.validity),
                          offsets=pinned(c.offsets, np.int32), child=ch)
        def empty(t, dtype=np.uint8):
            return None if t is None else host_empty(t.numel() * t.element_size()).view(dtype)
        return Column(values=empty(c.values), validity=empty(c.validity),
                      offsets=empty(c.offsets, np.int32), child=ch)

    host_cols = [tree(c, True) for c in cols]
    out = [tree(c, False) for c in cols]
    rows = host_empty(total_rows)
    roffs = host_empty(8 * (n + 1)).view(np.int64)
    enc.encode_host(host_cols, n, rows=rows, row_offsets=roffs)          # warm-up
    enc.decode_host(rows, roffs, n, out=out)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        enc.encode_host(host_cols, n, rows=rows, row_offsets=roffs)
        enc.decode_host(rows, roffs, n, out=out)
    dt = (time.perf_counter() - t0) / reps

    def same(a, b):
        if a.child:
            if not all(same(x, y) for x, y in zip(a.child, b.child)):
                return False
        return all((x is None) == (y is None) and (x is None or np.array_equal(x, y))
                   for x, y in ((a.offsets, b.offsets), (a.values, b.values)))
    assert all(same(a, b) for a, b in zip(host_cols, out)), "host-path round trip"
    alg = 2 * (_nbytes(cols) + total_rows)
    return {"GBps_algorithmic": round(alg / dt / 1e9, 2), "ms_per_step": round(dt * 1e3, 2),
            "what": "host columns in fury_host_alloc (pinned) buffers -> fury_row_encode_host -> "
                    "host rows -> fury_row_decode_host -> host columns (variable-length path)"}


if __name__ == "__main__":
    main()
