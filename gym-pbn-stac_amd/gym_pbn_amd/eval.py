"""Evaluation on top of the device batch: the steady-state-distribution histogram.

Mirrors ``compute_ssd_hist`` (``gym_PBN/utils/eval.py:20-72``) without the
process pool: the reference deep-copies the env ``resets`` times and runs
``iters // resets`` transitions in each copy (``:41-53``); here each copy is one
env of a device batch and all of them run in one kernel (``pbn_ssd_run``).

Semantics per iteration (``_ssd_run``, ``:80-101``): count the bucket of the
target nodes (first target = most significant bit), flip every node with
probability ``bit_flip_prob``, take one transition. The reference's own
``getTargetIdx`` indexes the state tuple by gene ID and ``PBNTargetEnv.step`` is
broken at HEAD, so ``target_nodes`` are node *indices* here and the
transition is one async update (R1/R4) -- build-defined, documented in DESIGN.md.
"""

from __future__ import annotations

import itertools
from typing import Optional, Sequence

import numpy as np

from .batch import PBNBatch


def _bit_seq_to_str(seq) -> str:  # eval.py:16-17
    return "".join(str(i) for i in seq)


def ssd_counts(network, target_nodes: Sequence[int], iters: int, resets: int, bit_flip_prob: float = 0.01,
               seed: int = 0, device: int = 0, initial_states: Optional[np.ndarray] = None) -> np.ndarray:
    """Raw counts [2^g] over ``resets`` envs x ``iters`` iterations each."""
    b = PBNBatch(network, resets, device=device, seed=seed)
    if initial_states is None:
        b.randomize()
    else:
        b.set_state(initial_states)
    return b.ssd_counts(target_nodes, iters, bit_flip_prob)


def _predict(model, obs: np.ndarray) -> np.ndarray:
    """``model.predict(state, target, deterministic=True)`` as ``_ssd_run`` calls it (eval.py:97-100:
    ``target`` is the state again), on the whole batch; a returned tuple is (actions, ...)."""
    out = model.predict(obs, obs, deterministic=True)
    if type(out) is tuple:
        out = out[0]
    return np.asarray(out).reshape(obs.shape[0], -1)


def ssd_counts_controlled(network, target_nodes: Sequence[int], iters: int, resets: int, model, seed: int = 0,
                          device: int = 0, initial_states: Optional[np.ndarray] = None) -> np.ndarray:
    """Raw counts [2^g] of the model-controlled run (``_ssd_run`` with a model, eval.py:80-101):
    per iteration count the bucket, ask the model for an action on every env at once (a
    batched ``predict``, one call for the ``resets`` envs), flip node ``action - 1`` (0 = none,
    ``pbn_target.py:266-267``), one async transition (R1/R4, Philox, no bit-flip noise)."""
    b = PBNBatch(network, resets, device=device, seed=seed)
    if initial_states is None:
        b.randomize()
    else:
        b.set_state(initial_states)
    t = np.asarray(target_nodes, dtype=np.int64)
    weights = (1 << np.arange(t.size - 1, -1, -1)).astype(np.int64)  # first target = MSB
    counts = np.zeros(1 << t.size, dtype=np.uint64)
    for _ in range(iters):
        obs = b.get_bits()
        np.add.at(counts, obs[:, t].astype(np.int64) @ weights, 1)
        b.flip(_predict(model, obs).astype(np.int32), offset=1, dedup=True)
        b.step(1)
    b.close()
    return counts


def ssd_counts_controlled_device(network, target_nodes: Sequence[int], iters: int, resets: int, policy,
                                 seed: int = 0, device: int = 0, initial_states: Optional[np.ndarray] = None):
    """``ssd_counts_controlled`` with the whole loop on the GPU: ``policy`` is a torch callable
    taking the observations as a uint8 tensor ``[resets][N]`` on the device and returning the
    actions (node + 1, 0 = none) as an integer tensor ``[resets]`` or ``[resets][A]`` there. Per
    iteration (eval.py:84-101): bucket counted on the device, ``policy`` called once for every
    reset, flip (``pbn_flip_device``), one transition -- everything on torch's current stream,
    no observation or action crosses PCIe. Same counts as ``ssd_counts_controlled`` with a
    ``model.predict`` computing the same actions."""
    import torch

    b = PBNBatch(network, resets, device=device, seed=seed)
    if initial_states is None:
        b.randomize()
    else:
        b.set_state(initial_states)
    dev = torch.device("cuda", device)
    b.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    try:
        N = b.n_nodes
        t = torch.as_tensor(np.asarray(target_nodes, dtype=np.int64), device=dev)
        g = t.numel()
        weights = (2.0 ** torch.arange(g - 1, -1, -1, device=dev)).float()  # first target = MSB; exact (g <= 12)
        span = min(iters, 256)  # iterations whose buckets are counted together
        buckets = torch.empty((span, resets), dtype=torch.int16, device=dev)
        counts = torch.zeros(1 << g, dtype=torch.int64, device=dev)
        obs = torch.empty((resets, N), dtype=torch.uint8, device=dev)
        for k in range(iters):
            b.unpack_bits_device(obs.data_ptr())
            buckets[k % span] = obs[:, t].float().matmul(weights).to(torch.int16)
            if k % span == span - 1 or k == iters - 1:
                counts += torch.bincount(buckets[:k % span + 1].reshape(-1).long(), minlength=1 << g)
            act = torch.as_tensor(policy(obs), device=dev)
            act = act.reshape(resets, -1).to(torch.int32).contiguous()
            # range errors surface at the last iteration's checked call (the reference would
            # raise at the first; rows with a bad action are left untouched either way)
            b.flip_device(act.data_ptr(), act.shape[1], offset=1, dedup=True, check=k == iters - 1)
            b.step(1)
        out = counts.cpu().numpy().astype(np.uint64)
    finally:
        torch.cuda.current_stream(dev).synchronize()
        b.set_stream(None)
        b.close()
    return out


def compute_ssd_hist(network, target_nodes: Sequence[int], iters: int = 1_200_000, resets: int = 300,
                     bit_flip_prob: float = 0.01, seed: int = 0, device: int = 0,
                     initial_states: Optional[np.ndarray] = None, model=None, policy=None):
    """Normalised SSD histogram as a DataFrame indexed by the bucket bit strings (eval.py:62-69).

    ``model`` given: the controlled SSD (actions from ``model.predict``, no bit-flip noise,
    eval.py:96-101); ``policy`` given: the same with a torch policy on the device
    (``ssd_counts_controlled_device``); otherwise the uncontrolled run with Bernoulli bit flips,
    all on the device."""
    assert 0 <= bit_flip_prob <= 1, "Invalid Bit Flip Probability value."  # eval.py:32-34
    assert resets > 0, "Invalid resets value."
    assert iters > 0, "Invalid iterations value."
    assert iters // resets, "Resets does not divide the iterations."
    per = iters // resets
    if policy is not None:
        counts = ssd_counts_controlled_device(network, target_nodes, per, resets, policy, seed, device, initial_states)
    elif model is None:
        counts = ssd_counts(network, target_nodes, per, resets, bit_flip_prob, seed, device, initial_states)
    else:
        counts = ssd_counts_controlled(network, target_nodes, per, resets, model, seed, device, initial_states)
    ssd = counts.astype(np.float64) / resets / per  # mean over resets, then / (iters // resets)
    g = len(target_nodes)
    states = list(map(_bit_seq_to_str, itertools.product([0, 1], repeat=g)))
    import pandas as pd

    return pd.DataFrame(list(ssd), index=states, columns=["Value"])


def eval_increase(network, target_nodes: Sequence[int], model, target_node_values, original_ssd=None,
                  iters: int = 1_200_000, resets: int = 300, bit_flip_prob: float = 0.01, seed: int = 0,
                  device: int = 0, policy=None) -> float:
    """Total increase of the favourable buckets between the uncontrolled and the controlled
    SSD (``eval_increase``, eval.py:106-136). ``target_node_values`` are the favourable
    target-node value tuples (the reference's ``env.target_node_values``). ``policy`` (a torch
    policy on the device) replaces ``model`` for the controlled run when given."""
    if original_ssd is None:  # cache, as the reference
        original_ssd = compute_ssd_hist(network, target_nodes, iters, resets, bit_flip_prob, seed, device)
    model_ssd = compute_ssd_hist(network, target_nodes, iters, resets, bit_flip_prob, seed, device, model=model,
                                 policy=policy)
    states_of_interest = [_bit_seq_to_str(s) for s in target_node_values]
    return float((model_ssd - original_ssd).loc[states_of_interest, "Value"].sum())
