"""Multi-GPU plumbing: one process per GPU, contiguous codeword shards, no
data-path collective.

The decode has no exchange step (codewords are independent), so
ranks only need (a) their shard of the global codeword range -- the
reference's dormant per-rank frame split, DNA_main.cpp:629-651 -- and (b) a
barrier plus MAX/SUM of a few scalars for timing and counters -- its
commented-out MPI_Reduce of counters, DNA_main.cpp:1187-1193.  Those run on
the gloo backend over CPU tensors, so no GPU context is touched by torch.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple


def shard(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, start+count) share of `total` codewords for `rank`
    (balanced: sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    start = total * rank // world
    return start, total * (rank + 1) // world - start


class Group:
    """Thin wrapper over torch.distributed (gloo) or a single process."""

    def __init__(self, world: int, rank: int, local: int, pg=None):
        self.world, self.rank, self.local, self._pg = world, rank, local, pg

    @classmethod
    def from_env(cls) -> "Group":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        pg = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo announces its connections on fd 1; keep stdout for the
            # benchmark's single JSON line
            import sys
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=rank, world_size=world)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            pg = dist
        return cls(world, rank, local, pg)

    def _reduce(self, x: float, op: str) -> float:
        if self._pg is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self._pg.all_reduce(t, op=getattr(self._pg.ReduceOp, op))
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def sum(self, x: float) -> float:
        return self._reduce(x, "SUM")

    def gather(self, obj) -> list:
        """Every rank's `obj` (a small picklable value), in rank order."""
        if self._pg is None:
            return [obj]
        out = [None] * self.world
        self._pg.all_gather_object(out, obj)
        return out

    def barrier(self):
        if self._pg is not None:
            self._pg.barrier()

    def close(self):
        if self._pg is not None:
            self._pg.destroy_process_group()
            self._pg = None


def launch_local(fn, world: int, port: Optional[int] = None, args=()):
    """Run fn(group, *args) in `world` CPU processes with gloo (tests)."""
    import torch.multiprocessing as mp
    port = port or 29500 + os.getpid() % 1000
    mp.spawn(_entry, args=(world, port, fn, args), nprocs=world, join=True)


def _entry(rank, world, port, fn, args):
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    g = Group.from_env()
    try:
        fn(g, *args)
    finally:
        g.close()
