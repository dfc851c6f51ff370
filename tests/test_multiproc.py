"""World-size-2 gloo tests of the multi-GPU orchestration on CPU, through the same launcher
``bench.py --gpus N`` uses (fury_amd.shard.launch): independent shards keyed by global row index
reproduce the single-process batch exactly (so N GPUs need no collective), the host-side offset
scan places the shards, and the barrier / max-reduce / gather timing works."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(name, total, outdir):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from fury_amd.shard import Orchestrator, from_env, global_row_base, strong_shard
    from fury_amd.workloads import SCHEMAS, gen_columns
    from oracle import oracle as O
    r = from_env()
    orch = Orchestrator(r)
    fields = SCHEMAS[name]
    start, n = strong_shard(total, r.world, r.rank)
    cols = gen_columns(name, fields, n, seed=77, start=start)
    rows, offs = O.encode(fields, cols, n)
    orch.barrier()
    t = orch.max(float(r.rank + 1))
    sizes = orch.gather_ints(int(rows.nbytes))
    base = global_row_base(sizes)
    np.save(os.path.join(outdir, f"rows{r.rank}.npy"), rows)
    np.save(os.path.join(outdir, f"meta{r.rank}.npy"),
            np.array([t, base[r.rank], start, n, r.world, int(os.environ["LOCAL_RANK"])]))
    orch.close()


@pytest.mark.parametrize("name,total", [("mixed", 1001), ("struct100", 130), ("nested", 257)])
def test_two_rank_shards_reproduce_single_batch(tmp_path, oracle, name, total):
    from fury_amd.shard import launch
    world = 2
    launch(world, _worker, (name, total, str(tmp_path)))
    from fury_amd.workloads import SCHEMAS, gen_columns
    fields = SCHEMAS[name]
    whole, _ = oracle.encode(fields, gen_columns(name, fields, total, seed=77), total)
    parts = [np.load(tmp_path / f"rows{r}.npy") for r in range(world)]
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert all(m[0] == world for m in metas)                 # max-reduce of (rank + 1)
    assert [int(m[4]) for m in metas] == [world] * world      # WORLD_SIZE set by the launcher
    assert [int(m[5]) for m in metas] == list(range(world))   # LOCAL_RANK = rank on one node
    glued = np.concatenate(parts)
    assert np.array_equal(glued, whole)
    for r in range(world):
        b = int(metas[r][1])
        assert np.array_equal(whole[b:b + parts[r].nbytes], parts[r])


def test_shard_ranges():
    from fury_amd.shard import strong_shard, weak_shard
    assert [strong_shard(100_000_000, 8, r) for r in range(8)][-1] == (87_500_000, 12_500_000)
    spans = [strong_shard(10, 3, r) for r in range(3)]
    assert spans == [(0, 4), (4, 3), (7, 3)]
    assert weak_shard(1_000_000, 3) == (3_000_000, 1_000_000)


def test_bench_launches_one_worker_per_gpu_and_checks_the_world():
    """`bench.py --gpus 2` started directly spawns two ranks through fury_amd.shard.launch; each
    rank checks WORLD_SIZE against --gpus and refuses to run more ranks than visible GPUs (no GPU
    here), and a torch.distributed.run-style environment that disagrees with --gpus is refused."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=300)
    assert p.returncode != 0
    assert "2 ranks but 0 visible GPUs" in p.stderr, p.stderr[-2000:]
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=300)
    assert p.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in p.stderr, p.stderr[-2000:]


def test_device_generator_matches_host_generator():
    """gen_columns_torch (the bench's in-HBM Struct-100 generator, run here on the CPU) is bit
    for bit the host SplitMix64 generator the oracle checks, for any global row range."""
    import torch
    from fury_amd.workloads import SCHEMAS, gen_columns, gen_columns_torch
    from fury_amd import types as T
    fields = SCHEMAS["struct100"][:6] + [T.not_null_field("i", T.INT32),
                                         T.not_null_field("f", T.FLOAT32),
                                         T.not_null_field("h", T.INT16),
                                         T.not_null_field("b", T.INT8)]
    for start, n in ((0, 1000), (12_499_990, 37)):
        want = gen_columns("struct100", fields, n, seed=1234, start=start)
        got = gen_columns_torch("struct100", fields, n, seed=1234, start=start,
                                device=torch.device("cpu"))
        for w, g in zip(want, got):
            assert np.array_equal(np.ascontiguousarray(w.values).view(np.uint8),
                                  g.values.numpy().view(np.uint8))
