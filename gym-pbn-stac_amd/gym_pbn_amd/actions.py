"""Synthetic agent actions for the multi-flip env, keyed by GLOBAL env id (bench config 5).

SURVEY §8(d) config 5 draws the agent's flip actions from "Philox seed 0xAC7 keyed by env": the
reference's agent acts through ``PBNTargetMultiEnv.step(action)`` (pbn_target_multi.py:119-131),
one action row of A node indices (0 = no flip, node ``k`` = index ``k - 1`` with ``offset`` 1) per env
step. Keying the draw by (global env id, env step, slot) makes the global batch the same workload at
any GPU count: rank r generates only its own shard ``[env_base, env_base + B)`` and gets the rows a
one-GPU run would give those envs.

Stream (build-defined, shared by the CPU and GPU paths -- plain torch integer ops, so it runs the
same on either device): Philox4x32-10 with key = seed, counter ``{t, c1, gid_lo, (gid_hi & 0xFFFFFF) |
STREAM_ACTIONS << 24}`` (the kernels' counter layout, pbn_device.hpp ``philox_draw``); c1 = 0 gives the
node words of slots 0..3, c1 = 1 the keep words: slot a flips node ``1 + mulhi(w0[a], N)`` if
``w1[a] >= ceil(p_none * 2^32)``, else 0. A <= 4.
"""

from __future__ import annotations

STREAM_ACTIONS = 9
_M32 = 0xFFFFFFFF
_PM0, _PM1 = 0xD2511F53, 0xCD9E8D57
_PW0, _PW1 = 0x9E3779B9, 0xBB67AE85


def _mulhilo(a: int, b):
    """(hi, lo) of the 64-bit product of the u32 constant ``a`` and the u32 values in int64 tensor
    ``b``, from 16-bit halves so that no intermediate exceeds 2^34 (no int64 wrap-around)."""
    ah, al = a >> 16, a & 0xFFFF
    bh, bl = b >> 16, b & 0xFFFF
    mid = bl * ah + bh * al
    lo_full = bl * al + ((mid & 0xFFFF) << 16)
    return bh * ah + (mid >> 16) + (lo_full >> 32), lo_full & _M32


def philox4x32_10(c0, c1, c2, c3, key: int):
    """Random123 Philox4x32-10 on int64 tensors holding u32 counters (broadcastable); returns the
    four output words. Same rounds as pbn_device.hpp ``philox4x32_10`` (KAT: tests/test_actions.py)."""
    k0, k1 = key & _M32, (key >> 32) & _M32
    for r in range(10):
        if r:
            k0, k1 = (k0 + _PW0) & _M32, (k1 + _PW1) & _M32
        hi0, lo0 = _mulhilo(_PM0, c0)
        hi1, lo1 = _mulhilo(_PM1, c2)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def env_actions(n_steps: int, env_base: int, n_envs: int, n_actions: int, n_nodes: int, seed: int = 0xAC7,
                p_none: float = 0.75, step_base: int = 0, device=None):
    """int32 ``[n_steps][n_envs][n_actions]`` action rows for envs ``env_base .. env_base + n_envs - 1``
    at env steps ``step_base .. step_base + n_steps - 1`` (see the module docstring)."""
    import torch

    if not 1 <= n_actions <= 4:
        raise ValueError("n_actions must be 1..4 (one Philox call's words per row)")
    gid = torch.arange(env_base, env_base + n_envs, dtype=torch.int64, device=device)
    t = torch.arange(step_base, step_base + n_steps, dtype=torch.int64, device=device)[:, None]
    c0 = t.expand(n_steps, n_envs)
    c2 = (gid & _M32)[None, :].expand(n_steps, n_envs)
    c3 = (((gid >> 32) & 0xFFFFFF) | (STREAM_ACTIONS << 24))[None, :].expand(n_steps, n_envs)
    zero = torch.zeros((), dtype=torch.int64, device=device)
    node_w = philox4x32_10(c0, zero, c2, c3, seed)
    keep_w = philox4x32_10(c0, zero + 1, c2, c3, seed)
    thr = min(int(-(-p_none * 4294967296.0 // 1)), 1 << 32)  # ceil(p_none * 2^32)
    cols = []
    for a in range(n_actions):
        node = 1 + ((node_w[a] * n_nodes) >> 32)
        cols.append(torch.where(keep_w[a] >= thr, node, zero))
    return torch.stack(cols, dim=-1).to(torch.int32).contiguous()


__all__ = ["env_actions", "philox4x32_10", "STREAM_ACTIONS"]
