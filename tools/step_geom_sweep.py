#!/usr/bin/env python3
"""Step kernel (1M and 8M Bittner-200 envs) under launch-geometry settings, measurement only.

Usage: step_geom_sweep.py K:SB [K:SB ...]   (K = PBNSIM_ENVS_PER_THREAD, SB = PBNSIM_STEP_BLOCK)
For each setting: a fresh batch (Philox fair-bit states, seed 0x5EED), 5 warm-up launches, then
20-launch windows timed with HIP events on the batch stream, early in the trajectory (about 43 % of
envs change per launch) and after 1,000 further launches (about 10 %). PBNSIM_LIB picks the library."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

import numpy as np  # noqa: E402

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

net = load_network("bittner199")


def win(b, n=20):
    b.timing(2)
    b.step(n)
    b.timing(0)
    ms, L = b.timing_read()
    return round(ms * 1e3 / L, 2)


def changed(b):
    a = b.get_state()
    b.step(1)
    return round(float(np.any(a != b.get_state(), axis=1).mean()), 3)


res = {}
for spec in sys.argv[1:]:
    k, sb = spec.split(":")
    os.environ["PBNSIM_ENVS_PER_THREAD"] = k
    os.environ["PBNSIM_STEP_BLOCK"] = sb
    for B in (1 << 20, 1 << 23):
        b = PBNBatch(net, B, seed=0x5EED)
        b.randomize()
        b.step(5)
        early = [win(b) for _ in range(3)]
        q_early = changed(b)
        b.step(1000)
        late = [win(b) for _ in range(3)]
        q_late = changed(b)
        b.close()
        res[f"{spec}:{B}"] = {"early": early, "late": late, "changed_early": q_early, "changed_late": q_late}
print(json.dumps({"lib": os.environ.get("PBNSIM_LIB", "in-tree"), "res": res}))
