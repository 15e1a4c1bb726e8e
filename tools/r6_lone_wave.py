#!/usr/bin/env python3
"""Per-update latency of one R6 env chain when its wave runs alone: B envs (one or a few waves),
one launch per env step, T steps; reports ms per step, the longest env step's updates and us per
update of that chain (measurement only). Env knobs (PBNSIM_ENV_*) apply."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T, A = 20, 4
CAP = int(__import__('os').environ.get('R6_CAP', '4096'))  # update cap (the slope over caps: time per block)
z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
net = Net(load_network("bittner199"))
cfg = EnvConfig(net, cubes_to_attractors(z, 199), horizon=100)
rng = np.random.default_rng(1)
acts = rng.integers(1, 200, size=(T, B, A)).astype(np.int32)
acts[rng.random((T, B, A)) < 0.75] = 0
b = PBNBatch(net, B, seed=0xAC7)
b.env_reset(cfg)
b.env_step_multi(cfg, acts[0], update_cap=CAP)  # warm-up
rows = []
for t in range(1, T):
    b.sync()
    b.timing(1)  # HIP events around the launch: the kernel alone
    t0 = time.perf_counter()
    _, _, _, nup = b.env_step_multi(cfg, acts[t], update_cap=CAP)
    dt = time.perf_counter() - t0
    kms, _ = b.timing_read()
    b.timing(0)
    rows.append((dt, int(nup.max()), kms / 1e3))
us = [dt * 1e6 / m for dt, m, _ in rows if m >= 1024]
kus_all = [k * 1e6 for _, _, k in rows]
kus = [k * 1e6 / m for _, m, k in rows if m >= 1024]
print(json.dumps({"B": B, "ms_per_step_median": float(np.median([r[0] for r in rows]) * 1e3),
                  "kernel_ms_per_step_median": float(np.median([r[2] for r in rows]) * 1e3), "cap": CAP,
                  "max_updates_median": float(np.median([r[1] for r in rows])),
                  "us_per_update_of_longest_chain": float(np.median(us)) if us else None,
                  "kernel_us_per_update_of_longest_chain": float(np.median(kus)) if kus else None,
                  "note": "us_per_update_of_longest_chain: host wall time of the env_step_multi call (action copy in, "
                          "launch, outputs copied out) / the longest env step's updates; kernel_us_*: HIP events around "
                          "the launch alone (includes the kernel's staging prologue)",
                  "lanes": b.info()["env_lanes"]}))
