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


def compute_ssd_hist(network, target_nodes: Sequence[int], iters: int = 1_200_000, resets: int = 300,
                     bit_flip_prob: float = 0.01, seed: int = 0, device: int = 0,
                     initial_states: Optional[np.ndarray] = None):
    """Normalised SSD histogram as a DataFrame indexed by the bucket bit strings (eval.py:62-69)."""
    assert 0 <= bit_flip_prob <= 1, "Invalid Bit Flip Probability value."  # eval.py:32-34
    assert resets > 0, "Invalid resets value."
    assert iters > 0, "Invalid iterations value."
    assert iters // resets, "Resets does not divide the iterations."
    per = iters // resets
    counts = ssd_counts(network, target_nodes, per, resets, bit_flip_prob, seed, device, initial_states)
    ssd = counts.astype(np.float64) / resets / per  # mean over resets, then / (iters // resets)
    g = len(target_nodes)
    states = list(map(_bit_seq_to_str, itertools.product([0, 1], repeat=g)))
    import pandas as pd

    return pd.DataFrame(list(ssd), index=states, columns=["Value"])
