"""Trajectory collection for the multi-flip env.

Each rank owns a shard of envs (``shard.py``) and runs T-step chunks of
``PBNTargetMultiEnv.step`` (R6, ``pbn_target_multi.py:119-154``) on its GPU, the
kernel writing every step's outputs straight into a device-resident chunk:

* ``obs``       [T][B_local][W]  int64 (packed state words, bit i of word i/64 = node i)
* ``reward``    [T][B_local]     int32
* ``flags``     [T][B_local]     uint8 (terminated | truncated << 1 | capped << 2)
* ``n_updates`` [T][B_local]     int32 (node updates the env step took)

The finished chunk is all-gathered across ranks with one
``all_gather_into_tensor`` per field (RCCL over xGMI on GPUs, gloo on CPU), giving
``[world][T][B_local]...`` (rank-major: rank r holds global envs
``[r*B_local, (r+1)*B_local)``). Chunks are double-buffered so the gather of chunk
k overlaps the env steps of chunk k+1: the collective runs on the process group's
own stream while the env kernel runs on the batch stream. There is no collective
inside the stepping path -- only this per-chunk exchange.
"""

from __future__ import annotations

from typing import Dict, Optional

from .batch import EnvConfig, PBNBatch

FIELDS = ("obs", "reward", "flags", "n_updates")


def alloc_chunk(T: int, n_envs: int, n_words: int, device) -> Dict[str, "torch.Tensor"]:  # noqa: F821
    import torch

    return {"obs": torch.empty((T, n_envs, n_words), dtype=torch.int64, device=device),
            "reward": torch.empty((T, n_envs), dtype=torch.int32, device=device),
            "flags": torch.empty((T, n_envs), dtype=torch.uint8, device=device),
            "n_updates": torch.empty((T, n_envs), dtype=torch.int32, device=device)}


def gather_chunk(chunk: Dict[str, "torch.Tensor"], dist, out: Optional[Dict] = None, async_op: bool = False):  # noqa: F821
    """All-gather every field of a chunk: ``[T][B_local]...`` -> ``[world][T][B_local]...``.

    Returns ``(gathered, works)``; with ``async_op`` the caller waits on ``works``.
    """
    import torch

    world = dist.get_world_size()
    if out is None:
        out = {k: torch.empty((world,) + tuple(v.shape), dtype=v.dtype, device=v.device) for k, v in chunk.items()}
    works = []
    for k in FIELDS:
        src = chunk[k]
        # uint8 is not an RCCL/gloo all-gather type everywhere; move flags as int8 bits
        if src.dtype == torch.uint8:
            src, dst = src.view(torch.int8), out[k].view(torch.int8)
        else:
            dst = out[k]
        w = dist.all_gather_into_tensor(dst.view(-1), src.contiguous().view(-1), async_op=async_op)
        if async_op:
            works.append(w)
    return out, works


class TrajectoryCollector:
    """T-step R6 chunks on one GPU; optional cross-rank gather of every chunk."""

    def __init__(self, batch: PBNBatch, cfg: EnvConfig, T: int, A: int, device, update_cap: int = 1 << 20,
                 dist=None, offset: int = 1, dedup: bool = True, fused: bool = True):
        self.batch, self.cfg = batch, cfg
        self.T, self.A = int(T), int(A)
        self.device = device
        self.update_cap = int(update_cap)
        self.offset, self.dedup = int(offset), bool(dedup)
        self.fused = bool(fused)  # one launch for the chunk's T steps (else one launch per step)
        self.dist = dist if (dist is not None and dist.is_initialized() and dist.get_world_size() > 1) else None
        B, W = batch.n_envs, batch.n_words
        self.bufs = [alloc_chunk(self.T, B, W, device) for _ in range(2)]
        self.gathered = None
        if self.dist is not None:
            import torch

            world = self.dist.get_world_size()
            self.gathered = [{k: torch.empty((world,) + tuple(v.shape), dtype=v.dtype, device=device)
                              for k, v in buf.items()} for buf in self.bufs]
        self._pending = [None, None]
        self._k = 0

    def run_chunk(self, actions, buf: Dict) -> None:
        """``actions``: device int32 tensor [T][B][A]. Asynchronous on the batch stream."""
        T, B, A = self.T, self.batch.n_envs, self.A
        if tuple(actions.shape) != (T, B, A) or not actions.is_contiguous() or actions.dtype.itemsize != 4:
            raise ValueError(f"actions must be a contiguous int32 [{T}][{B}][{A}] device tensor")
        o, r, f, n = buf["obs"], buf["reward"], buf["flags"], buf["n_updates"]
        so, sr, sf, sn = (o.stride(0) * o.element_size(), r.stride(0) * r.element_size(),
                          f.stride(0) * f.element_size(), n.stride(0) * n.element_size())
        sa = actions.stride(0) * actions.element_size()
        pa, po, pr, pf, pn = (actions.data_ptr(), o.data_ptr(), r.data_ptr(), f.data_ptr(), n.data_ptr())
        if self.fused:
            self.batch.env_rollout_multi_device(self.cfg, T, pa, A, po, pr, pf, pn, offset=self.offset,
                                                dedup=self.dedup, update_cap=self.update_cap)
            return
        for t in range(T):
            self.batch.env_step_multi_device(self.cfg, pa + t * sa, A, po + t * so, pr + t * sr, pf + t * sf,
                                             pn + t * sn, offset=self.offset, dedup=self.dedup,
                                             update_cap=self.update_cap)

    def step_chunk(self, actions, reset: bool = True):
        """Reset (optional), run one chunk, start its gather; returns the chunk index's buffers.

        With a process group the gather is asynchronous; :meth:`finish` waits for it.
        """
        i = self._k % 2
        if self._pending[i] is not None:  # the buffer's previous gather must be done before reuse
            self._drain(i)
        buf = self.bufs[i]
        if reset:
            self.batch.env_reset(self.cfg)
        self.run_chunk(actions, buf)
        self.batch.sync()  # the kernels ran on the batch stream; the collective reads the chunk next
        if self.dist is not None:
            _, works = gather_chunk(buf, self.dist, out=self.gathered[i], async_op=True)
            self._pending[i] = works
        self._k += 1
        return buf, (self.gathered[i] if self.dist is not None else None)

    def _drain(self, i: int) -> None:
        """Block the host until buffer ``i``'s gather has finished reading it.

        With RCCL (tensors on a GPU) ``Work.wait()`` only makes torch's *current* stream wait for
        the collective's stream; the host returns at once, and the env kernel that overwrites the
        buffer next runs on the batch's own stream, which that wait does not order. A rank can be
        two chunks ahead of a slower peer, so the collective may still be sending the buffer:
        synchronising the current stream (it now carries the wait) closes that window. The
        gather was started a whole chunk earlier, so this costs nothing in the steady state.
        With gloo ``wait()`` already blocks the host.
        """
        for w in self._pending[i]:
            w.wait()
        self._pending[i] = None
        buf = self.bufs[i]["obs"]
        if buf.is_cuda:
            import torch

            torch.cuda.current_stream(buf.device).synchronize()

    def finish(self) -> None:
        for i in range(2):
            if self._pending[i] is not None:
                self._drain(i)
