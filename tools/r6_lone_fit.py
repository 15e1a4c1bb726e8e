#!/usr/bin/env python3
"""Tail-block cost of ONE env alone (its workgroup's other waves idle: tail helpers available), from a
regression of each launch's kernel time (HIP events) on its env step's length: B = 1 env, one workgroup
(PBNSIM_ENV_GRID=1), two lanes per wave taking envs (PBNSIM_ENV_LANES=2: the workgroup hand-off and the
tail helpers are on), fixture attractors, cap 2^20, T env steps with random flips; fit kernel_us =
a + b * ceil(updates / 64): b = us per 64-update block, a = fixed cost. Env knobs (PBNSIM_ENV_*) apply.
Measurement only: python tools/r6_lone_fit.py [T]"""
import json
import os
import sys
from pathlib import Path

os.environ.setdefault("PBNSIM_ENV_GRID", "1")
os.environ.setdefault("PBNSIM_ENV_LANES", "2")
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 80
z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
net = Net(load_network("bittner199"))
cfg = EnvConfig(net, cubes_to_attractors(z, 199), horizon=1000)
rng = np.random.default_rng(7)
acts = rng.integers(1, 200, size=(T, 1, 4)).astype(np.int32)
b = PBNBatch(net, 1, seed=0xAC7)
b.env_reset(cfg)
rows = []
for t in range(T):
    b.sync()
    b.timing(1)
    _, _, _, nup = b.env_step_multi(cfg, acts[t], update_cap=1 << 20)
    kms, _ = b.timing_read()
    b.timing(0)
    st = b.env_tail_stats()
    rows.append((int(nup[0]), kms * 1e3, st["helpers"], st["ring_blocks"], st["ring_waits"]))
n = np.array([r[0] for r in rows], float)
k = np.array([r[1] for r in rows], float)
blk = np.ceil(n / 64)
m = n >= 1024
slope, icpt = np.polyfit(blk[m], k[m], 1) if m.sum() >= 3 else (None, None)
print(json.dumps({"env_steps": T, "fit_steps": int(m.sum()), "us_per_block": slope, "fixed_us": icpt,
                  "updates_median": float(np.median(n)), "updates_max": int(n.max()),
                  "helpers_per_launch_median": float(np.median([r[2] for r in rows])),
                  "ring_blocks": int(sum(r[3] for r in rows)), "ring_waits": int(sum(r[4] for r in rows)),
                  "env": {k2: v for k2, v in os.environ.items() if k2.startswith("PBNSIM_")},
                  "rows": rows}))
