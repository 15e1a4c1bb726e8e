"""Multi-GPU sharding of env batches (one process per GPU).

Envs are independent, so the batch is partitioned into contiguous shards of
global env ids ``[rank * n_local, (rank + 1) * n_local)``; Philox counters are
keyed by the global id, so a trajectory does not depend on the GPU count. The
stepping path has no collective. The only exchange is the optional trajectory
all-gather over ``torch.distributed`` -- RCCL when the tensors live
on GPUs, gloo on CPU -- gathered per T-step chunk, not per step.

Self-check of a sharded run (bench.py at any N): every rank recomputes the envs of
``sampled_env_ids`` that fall in its shard on their own (a 2-env batch with the same global ids,
seed and launch sequence: what a one-GPU run gives those ids), compares, and rank 0 digests every
rank's rows in global-id order (``rows_digest`` over ``gather_rows``), so the digest of a global
batch is the same at 1, 2, 4 or 8 GPUs.
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


def sampled_env_ids(n_global: int, n_samples: int) -> list:
    """Global env ids spread evenly over a global batch (even ids: the step stream's envs 2m and
    2m + 1 share a Philox call). The same ids for the same global batch at any GPU count."""
    n = max(1, min(n_samples, n_global // 2))
    return sorted({(k * n_global // n) & ~1 for k in range(n)})


def rows_digest(rows) -> str:
    """Digest of ``(global id, bytes)`` rows in global-id order (blake2b-64, hex)."""
    import hashlib

    h = hashlib.blake2b(digest_size=8)
    for gid, data in sorted(rows, key=lambda r: r[0]):
        h.update(int(gid).to_bytes(8, "little"))
        h.update(bytes(data))
    return h.hexdigest()


def gather_rows(local_rows, dist=None) -> list:
    """Every rank's ``(global id, bytes)`` rows on every rank (one small all_gather_object)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return list(local_rows)
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, [(int(g), bytes(d)) for g, d in local_rows])
    return [r for p in parts for r in p]


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
