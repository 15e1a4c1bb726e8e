"""actions.env_actions (bench config 5's agent actions, keyed by global env id): its torch
Philox4x32-10 equals the oracle's (Random123 KAT-checked in test_oracle.py) word for word, and the
draws of an env do not depend on the batch it sits in."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

from gym_pbn_amd.actions import STREAM_ACTIONS, env_actions, philox4x32_10  # noqa: E402


def test_torch_philox_matches_oracle(oracle_mod):
    rng = np.random.default_rng(3)
    ctr = rng.integers(0, 2**32, size=(300, 4), dtype=np.uint64)
    keys = rng.integers(0, 2**63, size=300, dtype=np.uint64)
    for c, k in zip(ctr, keys):
        want = oracle_mod.philox4x32_10([int(x) for x in c], [int(k) & 0xFFFFFFFF, int(k) >> 32])
        got = philox4x32_10(*[torch.tensor(int(x), dtype=torch.int64) for x in c], int(k))
        assert [int(g) for g in got] == want
    # extreme counters (all ones) through the 16-bit split multiply
    want = oracle_mod.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF, 0xFFFFFFFF])
    got = philox4x32_10(*[torch.tensor(0xFFFFFFFF, dtype=torch.int64)] * 4, (1 << 64) - 1)
    assert [int(g) for g in got] == want


def test_env_actions_keyed_by_global_id(oracle_mod):
    T, N, seed = 6, 199, 0xAC7
    big = env_actions(T, 1000, 64, 4, N, seed=seed)
    assert big.dtype == torch.int32 and big.shape == (T, 64, 4)
    for base, n in ((1000, 1), (1017, 5), (1062, 2)):
        assert torch.equal(env_actions(T, base, n, 4, N, seed=seed), big[:, base - 1000:base - 1000 + n])
    assert torch.equal(env_actions(2, 1000, 64, 4, N, seed=seed, step_base=3), big[3:5])
    # one row by hand from the oracle's Philox: node words (c1 = 0), keep words (c1 = 1)
    t, g = 4, 1033
    ctr = lambda c1: [t, c1, g & 0xFFFFFFFF, ((g >> 32) & 0xFFFFFF) | (STREAM_ACTIONS << 24)]
    w0 = oracle_mod.philox4x32_10(ctr(0), [seed, 0])
    w1 = oracle_mod.philox4x32_10(ctr(1), [seed, 0])
    row = [(1 + ((w0[a] * N) >> 32)) if w1[a] >= 3 << 30 else 0 for a in range(4)]
    assert big[t, g - 1000].tolist() == row
