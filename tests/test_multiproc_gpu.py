"""Multi-rank HIP parity on one GPU: the launcher `bench.py --gpus N` uses
(fury_amd.shard.launch) starts two ranks that SHARE the box's one GPU (--share-gpus rehearsal),
each rank encodes its own contiguous shard of global rows through the HIP library and decodes it
again.  Each rank's rows equal the oracle's encoding of exactly those global rows, the rank
decodes its rows back to the oracle's columns, and the two shards glued in rank order equal the
single-rank HIP encoding of the whole batch (independent shards keyed by global row: N GPUs need
no collective).  The ranks are fresh spawned interpreters (the launcher never forks
a process that has touched the GPU).  Also runs `bench.py --gpus 2 --share-gpus` itself and
checks that the line marks the rehearsal (n_gpus = distinct devices, shared_gpus).  Marked gpu."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _hip_worker(name, total, outdir):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import torch
    from fury_amd.encoder import Encoders, column_to_device, column_to_host
    from fury_amd.shard import Orchestrator, from_env, strong_shard
    from fury_amd.workloads import SCHEMAS, gen_columns
    from oracle import oracle as O
    from tests.helpers import assert_columns_equal
    r = from_env()
    orch = Orchestrator(r)
    ndev = torch.cuda.device_count()
    local = r.local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    fields = SCHEMAS[name]
    start, n = strong_shard(total, r.world, r.rank)
    host = gen_columns(name, fields, n, seed=77, start=start)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    dec = [column_to_host(c) for c in enc.decode_batch(batch)]
    torch.cuda.synchronize()
    rows = batch.rows.cpu().numpy()
    offs = None if batch.row_offsets is None else batch.row_offsets.cpu().numpy()
    want, want_offs = O.encode(fields, host, n)
    assert np.array_equal(rows, want), f"rank {r.rank}: rows differ from the oracle"
    assert_columns_equal(fields, dec, O.decode(fields, want, want_offs, n), n)
    orch.barrier()
    np.save(os.path.join(outdir, f"rows{r.rank}.npy"), rows)
    np.save(os.path.join(outdir, f"meta{r.rank}.npy"),
            np.array([start, n, local, ndev, torch.cuda.current_device()]))
    if offs is not None:
        np.save(os.path.join(outdir, f"offs{r.rank}.npy"), offs)
    orch.close()


_LAUNCH = """
import sys
sys.path.insert(0, {root!r})
from fury_amd.shard import launch
from tests.test_multiproc_gpu import _hip_worker
launch(2, _hip_worker, ({name!r}, {total}, {out!r}))
"""


@pytest.mark.parametrize("name,total", [("struct100", 20001), ("mixed", 30001), ("nested", 25003)])
def test_two_hip_ranks_share_one_gpu(tmp_path, oracle, name, total):
    import torch
    from fury_amd.encoder import Encoders, column_to_device
    from fury_amd.workloads import SCHEMAS, gen_columns
    # the ranks run in a fresh launcher process (this pytest process has used the GPU)
    p = subprocess.run([sys.executable, "-c", _LAUNCH.format(root=ROOT, name=name, total=total,
                                                             out=str(tmp_path))],
                       capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    fields = SCHEMAS[name]
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(2)]
    assert [int(m[0]) for m in metas] == [0, total // 2 + total % 2]
    assert sum(int(m[1]) for m in metas) == total
    assert all(int(m[2]) == 0 and int(m[4]) == 0 for m in metas), metas   # both on device 0
    dev = torch.device("cuda:0")
    host = gen_columns(name, fields, total, seed=77)
    enc = Encoders.bean(fields, device=dev)
    whole = enc.encode_batch([column_to_device(c, dev) for c in host], total)
    torch.cuda.synchronize()
    glued = np.concatenate([np.load(tmp_path / f"rows{r}.npy") for r in range(2)])
    assert np.array_equal(glued, whole.rows.cpu().numpy())
    if whole.row_offsets is not None:      # shard offsets rebased by the host-side scan
        o0, o1 = (np.load(tmp_path / f"offs{r}.npy") for r in range(2))
        glued_offs = np.concatenate([o0[:-1], o1 + o0[-1]])
        assert np.array_equal(glued_offs, whole.row_offsets.cpu().numpy())


def test_bench_share_gpus_line_is_marked_rehearsal():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--share-gpus", "--steps", "3", "--warmup", "1", "--rows", "200000",
                        "--no-cpu-baseline", "--no-e2e"],
                       capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["shared_gpus"] is True and line["ranks"] == 2
    assert line["n_gpus"] == 1, line
    assert "not a multi-GPU measurement" in line["rehearsal"]
    assert line["value"] > 0
