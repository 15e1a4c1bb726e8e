#!/usr/bin/env python3
"""Device RL loop: TorchVecPBNTargetMultiEnv.step with a random torch policy, B envs on one GPU
(Bittner-200, r6_bittner199 cubes, A = 4 slots, 0 w.p. 0.75); env-steps/s incl. observation
unpacking and on-device auto-reset. Measurement only."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.torch_env import TorchVecPBNTargetMultiEnv  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
env = TorchVecPBNTargetMultiEnv("bittner199", cubes_to_attractors(z, 199), B, horizon=100, update_cap=4096,
                                auto_reset=True, seed=7)
g = torch.Generator(device="cuda")
g.manual_seed(7)


def policy(obs):
    v = torch.randint(1, 200, (B, 4), device="cuda", generator=g, dtype=torch.int32)
    return v * (torch.rand((B, 4), device="cuda", generator=g) >= 0.75)


obs = env.reset()
ups = torch.zeros((), dtype=torch.int64, device="cuda")
for _ in range(3):  # the whole loop body: torch loads its kernels lazily on first use
    obs, r, te, tr, info = env.step(policy(obs))
    ups += info["n_updates"].to(torch.int64).sum()
torch.cuda.synchronize()
ups.zero_()
t0 = time.perf_counter()
for _ in range(K):
    obs, r, te, tr, info = env.step(policy(obs))
    ups += info["n_updates"].to(torch.int64).sum()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"B": B, "steps": K, "s_per_step": dt / K, "env_steps_per_s": B * K / dt,
                  "node_updates_per_s": float(ups.item()) / dt}))
