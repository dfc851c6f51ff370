"""Multi-GPU orchestration for the row codec: one process per GPU, independent row shards.

Rows are independent, so there is NO data-path collective: every rank encodes and
decodes its own contiguous global row range.  The only inter-process traffic is orchestration —
a barrier around the timed region and a max-reduce of the elapsed time — over gloo (CPU), so
xGMI/RCCL stay idle.  A concatenated global row buffer, if ever wanted, needs only a host-side
exclusive scan of per-shard byte totals (``global_row_base``).
"""
from __future__ import annotations

import os
import sys
import socket
from dataclasses import dataclass
from typing import Callable, List, Sequence, Tuple


@dataclass
class Rank:
    rank: int
    world: int
    local: int


def from_env() -> Rank:
    return Rank(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                int(os.environ.get("LOCAL_RANK", "0")))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker_entry(index: int, world: int, port: int, target: Callable, args: Sequence) -> None:
    os.environ.update(RANK=str(index), LOCAL_RANK=str(index), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    target(*args)


def launch(world: int, target: Callable, args: Sequence = ()) -> None:
    """Starts `world` worker processes (one per GPU), each with the torch.distributed.run
    environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), and runs
    ``target(*args)`` in every one; raises if any worker fails.

    Workers are spawned (fresh interpreters), so the caller must not have initialised the GPU:
    the parent only waits for its children.  ``bench.py --gpus N`` and the CPU gloo tests go
    through this same launcher."""
    if world < 1:
        raise ValueError("world must be >= 1")
    import torch.multiprocessing as mp
    mp.start_processes(_worker_entry, args=(world, free_port(), target, tuple(args)),
                       nprocs=world, join=True, start_method="spawn")


def weak_shard(rows_per_rank: int, rank: int) -> Tuple[int, int]:
    """Weak scaling: rank r owns global rows [r * rows_per_rank, (r + 1) * rows_per_rank)."""
    return rank * rows_per_rank, rows_per_rank


def strong_shard(total_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Strong scaling (C5: 100M rows over 8 GPUs): contiguous near-equal ranges."""
    base, extra = divmod(total_rows, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def global_row_base(shard_bytes: List[int]) -> List[int]:
    """Exclusive scan of per-shard row-byte totals: where each shard's rows would start in a
    concatenated batch (8-element host scan at 8 GPUs)."""
    out, acc = [], 0
    for b in shard_bytes:
        out.append(acc)
        acc += b
    return out


def _with_stdout_on_stderr(fn):
    """Runs fn with file descriptor 1 duplicated from 2 (C-level prints included: libc's buffers
    are flushed before fd 1 is restored)."""
    import ctypes
    libc = ctypes.CDLL(None)
    sys.stdout.flush()
    libc.fflush(None)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn()
    finally:
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


class Orchestrator:
    """Barrier + max-over-ranks timing for the bench contract."""

    def __init__(self, r: Rank):
        self.r = r
        self._dist = None
        if r.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                # gloo reports its mesh connections on stdout; the bench contract keeps stdout
                # for rank 0's one JSON line, so the rendezvous (and a first barrier, where the
                # mesh may be connected lazily) runs with fd 1 pointed at stderr
                _with_stdout_on_stderr(lambda: (
                    dist.init_process_group("gloo", rank=r.rank, world_size=r.world),
                    dist.barrier()))
            self._dist = dist

    def barrier(self) -> None:
        if self._dist is not None:
            self._dist.barrier()

    def max(self, value: float) -> float:
        if self._dist is None:
            return value
        import torch
        t = torch.tensor([value], dtype=torch.float64)
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX)
        return float(t[0])

    def gather_ints(self, value: int) -> List[int]:
        if self._dist is None:
            return [value]
        import torch
        t = torch.tensor([value], dtype=torch.int64)
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(self.r.world)]
        self._dist.all_gather(out, t)
        return [int(x[0]) for x in out]

    def close(self) -> None:
        if self._dist is not None and self._dist.is_initialized():
            self._dist.destroy_process_group()
