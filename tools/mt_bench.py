#!/usr/bin/env python3
"""MT mode (the reference's own CPython MT19937 per env, seeded from the Python seed alone:
pbn_mt_seed / pbn_mt_step, csrc/pbn_mt.hip) on Bittner-199: node-updates/s per GPU and the bytes the
generator state must move (measurement only).

Algorithmic bytes per node update: Graph.step draws randint(0, 198) (CPython _randbelow: 8-bit
getrandbits with rejection, 256/199 = 1.286 words on average) + random() (2 words) = 3.286 MT words;
every 624 words the env's 2,496-B table is twisted (read + written once): 8 B per word = 26.3 B per
update, plus the packed state read + written once per launch (64 B / T). Usage: python tools/mt_bench.py"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
import numpy as np  # noqa: E402

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

WORDS = 256 / 199 + 2.0
net = load_network("bittner199")
res = []
for B in (65536, 1 << 20):
    b = PBNBatch(net, B, seed=1)
    b.mt_seed(np.arange(B, dtype=np.uint64) + 12345)
    for T in (64, 512):
        b.mt_step(T)  # warm
        b.sync()
        b.timing(2)
        reps = 3
        for _ in range(reps):
            b.mt_step(T)
        b.timing(0)
        ms, n = b.timing_read()
        s = ms / 1e3 / reps
        ups = B * T / s
        alg = B * T * WORDS * 8 + 64 * B
        res.append({"B": B, "T": T, "ms_per_launch": ms / reps, "node_updates_per_s": ups,
                    "alg_GBs": alg / s / 1e9, "frac_of_8TBs": alg / s / 8e12})
        print(json.dumps(res[-1]), flush=True)
    b.close()
print(json.dumps({"mt_mode": res, "words_per_update": WORDS}))
