#!/usr/bin/env python3
"""Config 5 per GPU (131,072 Bittner-199 envs, A = 4, cap 4,096): one chunk of T = 100 env steps
as one fused launch and as 100 per-step launches, in lane mode (G = 1) and group modes G = 2/4/8
(PBNSIM_ENV_GROUP). Prints ms per env step for each (measurement only)."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
groups = [int(g) for g in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
T, A, CAP = 100, 4, 4096
z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
net = Net(load_network("bittner199"))
cfg = EnvConfig(net, cubes_to_attractors(z, 199), horizon=T)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(0xAC7)
v = torch.randint(1, 200, (T, B, A), device=dev, generator=g, dtype=torch.int32)
acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()
outs = [torch.empty((T, B, 4), dtype=torch.int64, device=dev), torch.empty((T, B), dtype=torch.int32, device=dev),
        torch.empty((T, B), dtype=torch.uint8, device=dev), torch.empty((T, B), dtype=torch.int32, device=dev)]
res = {}
for G in groups:
    os.environ["PBNSIM_ENV_GROUP"] = str(G)
    for fused in (True, False):
        b = PBNBatch(net, B, seed=0xAC7)
        best = None
        for rep in range(2):
            b.env_reset(cfg)
            b.sync()
            t0 = time.perf_counter()
            if fused:
                b.env_rollout_multi_device(cfg, T, acts.data_ptr(), A, *[x.data_ptr() for x in outs], update_cap=CAP)
            else:
                for t in range(T):
                    b.env_step_multi_device(cfg, acts[t].data_ptr(), A, *[x[t].data_ptr() for x in outs],
                                            update_cap=CAP)
            b.sync()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        lanes = b.info()["env_lanes"]
        b.close()
        res[f"G{G}:{'fused' if fused else 'per_step'}"] = {"ms_per_env_step": round(best * 1e3 / T, 3),
                                                           "env_steps_per_s": B * T / best, "lanes": lanes}
print(json.dumps(res))
