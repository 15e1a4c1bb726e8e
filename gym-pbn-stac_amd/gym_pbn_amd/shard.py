"""Multi-GPU sharding of env batches (one process per GPU).

Envs are independent, so the batch is partitioned into contiguous shards of
global env ids ``[rank * n_local, (rank + 1) * n_local)``; Philox counters are
keyed by the global id, so a trajectory does not depend on the GPU count. The
stepping path has no collective. The only exchange is the optional trajectory
all-gather over ``torch.distributed`` -- RCCL when the tensors live
on GPUs, gloo on CPU -- gathered per T-step chunk, not per step.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    n_local: int

    @property
    def env_base(self) -> int:
        return self.rank * self.n_local

    @property
    def n_global(self) -> int:
        return self.world * self.n_local


def shard_for(rank: int, world: int, n_local: int) -> Shard:
    if not (0 <= rank < world) or n_local < 1:
        raise ValueError("bad shard spec")
    return Shard(rank, world, n_local)


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """The slowest rank's time (bench contract: MAX over ranks)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_chunks(local: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather equal-sized per-rank chunks ``[n_local, ...]`` into ``[world * n_local, ...]``.

    ``local`` is a host array (e.g. a T-step chunk of packed observations); it is
    moved to ``device`` (a GPU for RCCL over xGMI) for the collective.
    """
    import torch

    world = dist.get_world_size()
    src = torch.from_numpy(np.ascontiguousarray(local).view(np.int64 if local.dtype == np.uint64 else local.dtype))
    if device is not None:
        src = src.to(device)
    out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src)
    res = out.cpu().numpy()
    return res.view(np.uint64) if local.dtype == np.uint64 else res
