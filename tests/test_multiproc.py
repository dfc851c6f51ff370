"""World-size-2 gloo test of the multi-GPU orchestration on CPU: independent shards keyed by
global row index reproduce the single-process batch exactly (so N GPUs need no collective),
the host-side offset scan places the shards, and the barrier / max-reduce timing works."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, total, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from fury_amd.shard import Orchestrator, from_env, global_row_base, strong_shard
    from fury_amd.workloads import SCHEMAS, gen_columns
    from oracle import oracle as O
    orch = Orchestrator(from_env())
    fields = SCHEMAS[name]
    start, n = strong_shard(total, world, rank)
    cols = gen_columns(name, fields, n, seed=77, start=start)
    rows, offs = O.encode(fields, cols, n)
    orch.barrier()
    t = orch.max(float(rank + 1))
    sizes = orch.gather_ints(int(rows.nbytes))
    base = global_row_base(sizes)
    np.save(os.path.join(outdir, f"rows{rank}.npy"), rows)
    np.save(os.path.join(outdir, f"meta{rank}.npy"), np.array([t, base[rank], start, n]))
    orch.close()


@pytest.mark.parametrize("name,total", [("mixed", 1001), ("struct100", 130), ("nested", 257)])
def test_two_rank_shards_reproduce_single_batch(tmp_path, oracle, name, total):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), name, total, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    from fury_amd.workloads import SCHEMAS, gen_columns
    fields = SCHEMAS[name]
    whole, _ = oracle.encode(fields, gen_columns(name, fields, total, seed=77), total)
    parts = [np.load(tmp_path / f"rows{r}.npy") for r in range(world)]
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert all(m[0] == world for m in metas)                 # max-reduce of (rank + 1)
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
