#!/usr/bin/env python3
"""Latency of the single-env surfaces (the reference's own use: one Graph, one env) on one GPU.
Reference: Graph.step on Bittner-200 ~49 us, PBNTargetMultiEnv.step ~69 ms."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.envs import Graph, PBNTargetMultiEnv  # noqa: E402


def per_call(f, n):
    for _ in range(20):
        f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t0) / n


out = {}
for name in ("bittner28", "bittner199"):
    g = Graph(name, seed=1)
    g.genRandState()
    out[f"Graph.step {name} us"] = per_call(g.step, 2000) * 1e6
z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
env = PBNTargetMultiEnv("bittner199", cubes_to_attractors(z, 199), horizon=100)
env.reset(seed=3)
rng = np.random.default_rng(0)
acts = [[int(x)] for x in rng.integers(0, 200, size=500)]
it = iter(acts * 100)
out["PBNTargetMultiEnv.step bittner199 us"] = per_call(lambda: env.step(next(it)), 300) * 1e6
print(json.dumps(out))
