"""Batched device objects over the C ABI: networks, env batches, env configs.

A :class:`PBNBatch` is B independent copies of one network (the reference holds
one ``base.Graph`` / ``PBN`` per env and parallelises only by processes,
``utils/eval.py:41-53``). State lives in HBM as bit-packed uint64 words
``[B][W]``; every transition runs in the gfx950 kernels of libpbnsim.
"""

from __future__ import annotations

import functools

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib as L
from .network import KIND_PREDICTOR_MIX, PredictorNetwork, TruthTableNetwork, load_network


def pack_bits(bits) -> np.ndarray:
    """[..., N] 0/1 -> [..., W] uint64 (node i in bit i%64 of word i//64)."""
    bits = np.asarray(bits).astype(np.uint64, copy=False)
    n = bits.shape[-1]
    W = (n + 63) // 64
    pad = W * 64 - n
    if pad:
        bits = np.concatenate([bits, np.zeros(bits.shape[:-1] + (pad,), dtype=np.uint64)], axis=-1)
    b = bits.reshape(bits.shape[:-1] + (W, 64))
    shifts = np.arange(64, dtype=np.uint64)
    return np.bitwise_or.reduce(b << shifts, axis=-1).astype(np.uint64)


@functools.lru_cache(maxsize=64)
def _bit_index(n: int):
    idx = np.arange(n)
    return idx // 64, (idx % 64).astype(np.uint64)


def unpack_bits(words, n: int) -> np.ndarray:
    """[..., W] uint64 -> [..., N] uint8."""
    words = np.asarray(words, dtype=np.uint64)
    wi, sh = _bit_index(int(n))
    return ((words[..., wi] >> sh) & np.uint64(1)).astype(np.uint8)


class Net:
    """A network uploaded to the library (tables are copied; arrays may be freed)."""

    def __init__(self, network):
        if isinstance(network, (str, bytes)) or hasattr(network, "__fspath__"):
            network = load_network(network)
        network.validate()
        self.network = network
        self.n_nodes = network.n_nodes
        self.n_words = network.n_words
        self.kind = network.kind
        d = L.NetDesc()
        d.kind = network.kind
        d.n_nodes = network.n_nodes
        keep = []

        def arr(a, dt, t):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return L.ptr(a, t)

        if isinstance(network, PredictorNetwork):
            d.n_preds = network.n_preds
            d.pred_offsets = arr(network.pred_offsets, np.int32, L._i32p)
            d.pred_inputs = arr(network.pred_inputs, np.int32, L._i32p)
            d.pred_tt = arr(network.pred_tt, np.uint16, L._u16p)
            d.pred_thr = arr(network.pred_thr, np.uint64, L._u64p)
        elif isinstance(network, TruthTableNetwork):
            d.node_k = arr(network.node_k, np.int32, L._i32p)
            d.input_offsets = arr(network.input_offsets, np.int32, L._i32p)
            d.inputs = arr(network.inputs if network.inputs.size else np.zeros(1, np.int32), np.int32, L._i32p)
            d.thr_offsets = arr(network.thr_offsets, np.int64, L._i64p)
            d.thr = arr(network.thr, np.uint64, L._u64p)
        else:
            raise TypeError("unsupported network type")
        h = C.c_void_p()
        L.check(L.lib.pbn_net_create(C.byref(d), C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(L, "lib", None) is not None:  # not at interpreter exit
            L.lib.pbn_net_destroy(h)
            self._h = None


class EnvConfig:
    """Attractor/goal description for the multi-flip env (pbn_target_multi.py:437-458).

    ``attractors`` is the reference's ``all_attractors``: a list of attractors,
    each a list of hypercube tuples over the N nodes with ints and ``'*'``
    (cabean output, ``get_attractors_from_cabean.py:14-36``). The attracting
    set is the union of all cubes; reset draws from ``attractors[0]``; the
    target is ``attractors[-1][0]`` (``in_target`` only tests ``target[0]``).
    """

    def __init__(self, net: Net, attractors, horizon: int = 100, reward_success: int = 1000, action_cost: int = 1,
                 first_update_tested: bool = False):
        self.net = net
        N, W = net.n_nodes, net.n_words
        self.attractors = [list(a) for a in attractors]
        if not self.attractors or not all(self.attractors):
            raise ValueError("need at least one non-empty attractor")
        cubes = [c for a in self.attractors for c in a]
        care, val = cube_arrays(cubes, N)
        rc_, rv_ = cube_arrays(self.attractors[0], N)
        tc_, tv_ = cube_arrays([self.attractors[-1][0]], N)
        self.cube_care, self.cube_value = care, val
        self.reset_care, self.reset_value = rc_, rv_
        self.target_care, self.target_value = tc_[0].copy(), tv_[0].copy()
        self.horizon = int(horizon)
        self.reward_success = int(reward_success)
        self.action_cost = int(action_cost)
        d = L.EnvCfgDesc()
        d.n_cubes = care.shape[0]
        d.cube_care = L.ptr(care, L._u64p)
        d.cube_value = L.ptr(val, L._u64p)
        d.n_reset_cubes = rc_.shape[0]
        d.reset_care = L.ptr(rc_, L._u64p)
        d.reset_value = L.ptr(rv_, L._u64p)
        d.target_care = L.ptr(self.target_care, L._u64p)
        d.target_value = L.ptr(self.target_value, L._u64p)
        d.horizon = self.horizon
        d.reward_success = self.reward_success
        d.action_cost = self.action_cost
        self.first_update_tested = bool(first_update_tested)
        d.first_update_tested = int(self.first_update_tested)
        h = C.c_void_p()
        L.check(L.lib.pbn_envcfg_create(net.handle, C.byref(d), C.byref(h)))
        self._h = h
        del W

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(L, "lib", None) is not None:
            L.lib.pbn_envcfg_destroy(h)
            self._h = None


def flip_gap_table(n_nodes: int, p: float):
    """Geometric-gap thresholds for independent Bernoulli(p) node flips.

    ``T_k = floor((1-p)^k * 2^32)`` for k = 1..N, so that a 32-bit uniform u gives
    ``gap = #{k >= 1 : u < T_k}`` with ``P(gap >= k) = (1-p)^k``. ``None`` for p == 0.
    """
    if not (0.0 <= p <= 1.0):
        raise ValueError("Invalid Bit Flip Probability value.")  # eval.py:32-34
    if p == 0.0:
        return None
    k = np.arange(1, n_nodes + 1, dtype=np.float64)
    t = np.floor(np.power(1.0 - p, k) * 4294967296.0)
    return np.minimum(t, 4294967295.0).astype(np.uint32)


def cube_arrays(cubes: Sequence, n_nodes: int):
    """Hypercube tuples (ints / '*') -> (care, value) [H][W] uint64."""
    W = (n_nodes + 63) // 64
    care = np.zeros((len(cubes), W), dtype=np.uint64)
    val = np.zeros((len(cubes), W), dtype=np.uint64)
    for h, c in enumerate(cubes):
        if len(c) != n_nodes:
            raise ValueError(f"hypercube {h} has length {len(c)}, expected {n_nodes}")
        for i, x in enumerate(c):
            if x == "*" or x == "-":
                continue
            bit = np.uint64(1) << np.uint64(i % 64)
            care[h, i // 64] |= bit
            if int(x):
                val[h, i // 64] |= bit
    return care, val


def attractors_from_cubes(care, value, attractor_of, n_nodes: int):
    """Rebuild ``all_attractors`` (lists of int / '*' tuples) from packed cube arrays.

    ``care``/``value`` [H][W] uint64 as :func:`cube_arrays` makes them, ``attractor_of`` [H]
    the attractor index of every cube (the layout of the r6 fixtures).
    """
    c = unpack_bits(np.asarray(care, np.uint64), n_nodes)
    v = unpack_bits(np.asarray(value, np.uint64), n_nodes)
    out = {}
    for h, a in enumerate(np.asarray(attractor_of).tolist()):
        out.setdefault(int(a), []).append(tuple(int(x) if m else "*" for m, x in zip(c[h], v[h])))
    return [out[k] for k in sorted(out)]


class PBNBatch:
    """B independent envs of one network on one GPU."""

    def __init__(self, net, n_envs: int, device: int = 0, env_id_base: int = 0, seed: int = 0):
        self.net = net if isinstance(net, Net) else Net(net)
        self.n_envs = int(n_envs)
        self.n_nodes = self.net.n_nodes
        self.n_words = self.net.n_words
        self.device = int(device)
        h = C.c_void_p()
        L.check(L.lib.pbn_batch_create(self.net.handle, self.device, self.n_envs, int(env_id_base), int(seed),
                                       C.byref(h)))
        self._h = h

    # -- lifecycle --------------------------------------------------------
    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(L, "lib", None) is not None:
            L.lib.pbn_batch_destroy(h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        i = L.BatchInfo()
        L.check(L.lib.pbn_batch_get_info(self._h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in L.BatchInfo._fields_}

    def sync(self):
        L.check(L.lib.pbn_sync(self._h))

    # -- state ------------------------------------------------------------
    def set_state(self, words):
        w = np.ascontiguousarray(words, dtype=np.uint64).reshape(self.n_envs, self.n_words)
        L.check(L.lib.pbn_set_state(self._h, L.ptr(w, L._u64p)))

    def get_state(self) -> np.ndarray:
        w = np.empty((self.n_envs, self.n_words), dtype=np.uint64)
        L.check(L.lib.pbn_get_state(self._h, L.ptr(w, L._u64p)))
        return w

    def set_bits(self, bits):
        bits = np.asarray(bits)
        if bits.shape[-1] != self.n_nodes:
            raise ValueError(f"state length {bits.shape[-1]} != N={self.n_nodes}")
        self.set_state(pack_bits(bits.reshape(self.n_envs, self.n_nodes)))

    def get_bits(self) -> np.ndarray:
        return unpack_bits(self.get_state(), self.n_nodes)

    def set_state_device(self, dev_ptr: int):
        L.check(L.lib.pbn_set_state_device(self._h, C.c_void_p(dev_ptr)))

    def get_state_device(self, dev_ptr: int):
        L.check(L.lib.pbn_get_state_device(self._h, C.c_void_p(dev_ptr)))

    def randomize(self):
        L.check(L.lib.pbn_randomize_state(self._h))

    # -- dynamics ---------------------------------------------------------
    def flip(self, actions, offset: int = 1, dedup: bool = True):
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.n_envs, -1)
        L.check(L.lib.pbn_flip(self._h, L.ptr(a, L._i32p), a.shape[1], int(offset), int(bool(dedup))))

    def flip_device(self, d_actions: int, A: int, offset: int = 1, dedup: bool = True, check: bool = True):
        """``flip`` with device actions (``d_actions``: pointer to int32 ``[B][A]`` on this GPU).
        ``check=False`` returns at once; range errors are then raised by the next checked call."""
        L.check(L.lib.pbn_flip_device(self._h, C.c_void_p(int(d_actions)), int(A), int(offset), int(bool(dedup)),
                                      int(bool(check))))

    def step(self, n_updates: int = 1):
        L.check(L.lib.pbn_step(self._h, int(n_updates)))

    def prepare_steps(self, n_updates: int):
        """Capture the HIP graph for ``step(n_updates)`` now (setup; nothing runs)."""
        L.check(L.lib.pbn_step_prepare(self._h, int(n_updates)))

    def rollout(self, n_updates: int):
        L.check(L.lib.pbn_rollout(self._h, int(n_updates)))

    def step_replay(self, node_idx, k53):
        ni = np.ascontiguousarray(node_idx, dtype=np.uint32).reshape(-1, self.n_envs)
        kk = np.ascontiguousarray(k53, dtype=np.uint64).reshape(-1, self.n_envs)
        if ni.shape != kk.shape:
            raise ValueError("node_idx and k53 shapes differ")
        L.check(L.lib.pbn_step_replay(self._h, L.ptr(ni, L._u32p), L.ptr(kk, L._u64p), ni.shape[0]))

    def step_forced(self, node_idx):
        """Updates with caller-chosen nodes (``node_idx`` ``[T][B]``) and the Philox choice draws
        ``step`` would use for those updates; the update counter advances by T (pbn_step_forced)."""
        ni = np.ascontiguousarray(node_idx, dtype=np.uint32).reshape(-1, self.n_envs)
        L.check(L.lib.pbn_step_forced(self._h, L.ptr(ni, L._u32p), ni.shape[0]))

    def mt_seed(self, seeds, init_state: bool = True):
        s = np.ascontiguousarray(seeds, dtype=np.uint64).reshape(self.n_envs)
        L.check(L.lib.pbn_mt_seed(self._h, L.ptr(s, L._u64p), int(bool(init_state))))

    def mt_step(self, n_updates: int = 1):
        L.check(L.lib.pbn_mt_step(self._h, int(n_updates)))

    # -- R6 env -----------------------------------------------------------
    def env_reset(self, cfg: EnvConfig, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8).reshape(self.n_envs)
        L.check(L.lib.pbn_env_reset(self._h, cfg.handle, L.ptr(m, L._u8p)))

    def unpack_bits_device(self, d_bits: int, d_words: int = 0):
        """Device uint8 [B][N] node values from device words [B][W] (0 = the batch's state); async."""
        L.check(L.lib.pbn_unpack_bits_device(self._h, C.c_void_p(d_words or None), C.c_void_p(d_bits)))

    def env_reset_device(self, cfg: EnvConfig, d_mask: int = 0):
        """Asynchronous reset on the batch stream; ``d_mask``: device uint8 [B] pointer (0 = all)."""
        L.check(L.lib.pbn_env_reset_device(self._h, cfg.handle, C.c_void_p(d_mask or None)))

    def set_stream(self, stream=None):
        """Run this batch's calls on a HIP stream handle (e.g. ``torch.cuda.current_stream().cuda_stream``,
        0 being the default stream); ``None`` = the batch's own stream again."""
        own = stream is None
        L.check(L.lib.pbn_batch_set_stream(self._h, int(own), C.c_void_p(None if own or not stream else stream)))

    def set_n_steps(self, n_steps):
        a = np.ascontiguousarray(n_steps, dtype=np.int64).reshape(self.n_envs)
        L.check(L.lib.pbn_set_n_steps(self._h, L.ptr(a, L._i64p)))

    def get_n_steps(self) -> np.ndarray:
        a = np.empty(self.n_envs, dtype=np.int64)
        L.check(L.lib.pbn_get_n_steps(self._h, L.ptr(a, L._i64p)))
        return a

    def env_step_multi(self, cfg: EnvConfig, actions, offset: int = 1, dedup: bool = True,
                       update_cap: int = 1 << 20, replay: Optional[tuple] = None):
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.n_envs, -1)
        obs = np.empty((self.n_envs, self.n_words), dtype=np.uint64)
        rew = np.empty(self.n_envs, dtype=np.int32)
        flags = np.empty(self.n_envs, dtype=np.uint8)
        nup = np.empty(self.n_envs, dtype=np.uint32)
        if replay is None:
            rc = L.lib.pbn_env_step_multi(self._h, cfg.handle, L.ptr(a, L._i32p), a.shape[1], int(bool(dedup)),
                                          int(offset), int(update_cap), L.ptr(obs, L._u64p), L.ptr(rew, L._i32p),
                                          L.ptr(flags, L._u8p), L.ptr(nup, L._u32p))
        else:
            off = np.ascontiguousarray(replay[0], dtype=np.int64)
            di = np.ascontiguousarray(replay[1], dtype=np.uint32)
            dk = np.ascontiguousarray(replay[2], dtype=np.uint64)
            if di.size == 0:
                di = np.zeros(1, np.uint32)
                dk = np.zeros(1, np.uint64)
            rc = L.lib.pbn_env_step_multi_replay(self._h, cfg.handle, L.ptr(a, L._i32p), a.shape[1],
                                                 int(bool(dedup)), int(offset), L.ptr(off, L._i64p),
                                                 L.ptr(di, L._u32p), L.ptr(dk, L._u64p), L.ptr(obs, L._u64p),
                                                 L.ptr(rew, L._i32p), L.ptr(flags, L._u8p), L.ptr(nup, L._u32p))
        L.check(rc)
        return obs, rew, flags, nup

    def env_step_multi_device(self, cfg: EnvConfig, d_actions: int, A: int, d_obs: int, d_reward: int, d_flags: int,
                              d_n_updates: int, offset: int = 1, dedup: bool = True, update_cap: int = 1 << 20):
        """Asynchronous R6 step on device buffers (e.g. ``tensor.data_ptr()`` of torch cuda tensors)."""
        L.check(L.lib.pbn_env_step_multi_device(self._h, cfg.handle, C.c_void_p(d_actions), int(A),
                                                int(bool(dedup)), int(offset), int(update_cap),
                                                C.c_void_p(d_obs), C.c_void_p(d_reward), C.c_void_p(d_flags),
                                                C.c_void_p(d_n_updates)))

    def env_rollout_multi_device(self, cfg: EnvConfig, n_steps: int, d_actions: int, A: int, d_obs: int,
                                 d_reward: int, d_flags: int, d_n_updates: int, offset: int = 1, dedup: bool = True,
                                 update_cap: int = 1 << 20):
        """``n_steps`` R6 env steps in one launch (actions known up front, e.g. open-loop or
        exploration trajectories): device arrays actions ``[n_steps][B][A]`` int32 and outputs
        ``[n_steps][B][W]`` / ``[n_steps][B]``. Same results as ``n_steps`` calls of
        :meth:`env_step_multi_device` on the slices; each env walks its steps without waiting
        for the rest of the batch between them."""
        L.check(L.lib.pbn_env_rollout_multi_device(self._h, cfg.handle, int(n_steps), C.c_void_p(d_actions), int(A),
                                                   int(bool(dedup)), int(offset), int(update_cap),
                                                   C.c_void_p(d_obs), C.c_void_p(d_reward), C.c_void_p(d_flags),
                                                   C.c_void_p(d_n_updates)))

    def synch_step(self, n_steps: int = 1, perturbation_prob: float = 0.0):
        """Synchronous update (base.py:286-303); perturbation_prob > 0 enables perturbations (p=0.001 there)."""
        gap = flip_gap_table(self.n_nodes, perturbation_prob)
        L.check(L.lib.pbn_synch_step(self._h, int(n_steps), L.ptr(gap, L._u32p)))

    # -- SSD histogram (utils/eval.py:20-103) -------------------------------
    def ssd_counts(self, target_nodes, iters: int, bit_flip_prob: float = 0.01) -> np.ndarray:
        """Run ``iters`` SSD iterations on every env; returns counts [2^g] (first target = MSB)."""
        t = np.ascontiguousarray(target_nodes, dtype=np.int32)
        gap = flip_gap_table(self.n_nodes, bit_flip_prob)
        hist = np.zeros(1 << t.size, dtype=np.uint64)
        L.check(L.lib.pbn_ssd_run(self._h, L.ptr(t, L._i32p), int(t.size), L.ptr(gap, L._u32p), int(iters),
                                  L.ptr(hist, L._u64p)))
        return hist

    # -- timing -----------------------------------------------------------
    def timing(self, mode):
        """0 off; 1 an event pair around every launch; 2 one event region over all launches."""
        L.check(L.lib.pbn_timing_enable(self._h, int(mode)))

    def timing_read(self):
        ms = C.c_double(0)
        n = C.c_uint64(0)
        L.check(L.lib.pbn_timing_read(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def timing_read_each(self, cap: int = 1 << 16):
        """Timing mode 1: every timed launch's kernel ms since the last read, in launch order."""
        buf = (C.c_double * cap)()
        n = C.c_uint64(0)
        L.check(L.lib.pbn_timing_read_each(self._h, buf, cap, C.byref(n)))
        return [buf[k] for k in range(min(n.value, cap))]

    def env_tail_helpers(self) -> int:
        """Tail helpers the last R6 launch recruited (idle waves preparing a long tail session's blocks)."""
        n = C.c_uint32(0)
        L.check(L.lib.pbn_env_tail_helpers(self._h, C.byref(n)))
        return n.value

    def env_tail_stats(self) -> dict:
        """The last R6 launch's tail counters (hand-offs, helpers, ring blocks, ring blocks waited for)."""
        st = (C.c_uint32 * 4)()
        L.check(L.lib.pbn_env_tail_stats(self._h, st))
        return {"handoffs": st[0], "helpers": st[1], "ring_blocks": st[2], "ring_waits": st[3]}

    def env_grid_stats(self) -> dict:
        """The last R6 launch's grid-pool counters: envs handed to workgroups that had run out of work,
        tickets those workgroups took, waits given up (0), live count at the end (0)."""
        st = (C.c_uint32 * 4)()
        L.check(L.lib.pbn_env_grid_stats(self._h, st))
        return {"pushed": st[0], "tickets": st[1], "gave_up": st[2], "live_at_end": st[3]}

    def env_handoffs(self) -> int:
        """Envs the last R6 launch handed from tail-mode waves to idle ones (0 with the hand-off off)."""
        n = C.c_uint32(0)
        L.check(L.lib.pbn_env_handoffs(self._h, C.byref(n)))
        return n.value


__all__ = ["Net", "EnvConfig", "PBNBatch", "pack_bits", "unpack_bits", "cube_arrays", "attractors_from_cubes",
           "KIND_PREDICTOR_MIX"]
