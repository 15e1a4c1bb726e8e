#!/usr/bin/env python3
"""Config-5 one-launch-per-env-step: raw loop of pbn_env_step_multi_device vs TrajectoryCollector
(fused=False), with and without per-launch event timing (measurement only). Prints ms per env step."""
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
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402
from gym_pbn_amd.rollout import TrajectoryCollector  # noqa: E402

B, T, A, CAP = 131072, 100, 4, 4096
z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
net = Net(load_network("bittner199"))
cfg = EnvConfig(net, cubes_to_attractors(z, 199), horizon=T)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(0xAC7)
v = torch.randint(1, 200, (T, B, A), device=dev, generator=g, dtype=torch.int32)
acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()
res = {}
for rep in range(2):
    for mode in ("raw", "raw_timing1", "collector", "collector_timing1"):
        b = PBNBatch(net, B, seed=0xAC7)
        col = TrajectoryCollector(b, cfg, T, A, dev, update_cap=CAP, fused=False)
        col.step_chunk(acts)
        col.finish()
        torch.cuda.synchronize()
        if mode.endswith("timing1"):
            b.timing(1)
        t0 = time.perf_counter()
        for _ in range(2):
            if mode.startswith("raw"):
                b.env_reset(cfg)
                col.run_chunk(acts, col.bufs[0])
            else:
                col.step_chunk(acts)
        col.finish()
        b.sync()
        dt = time.perf_counter() - t0
        k = None
        if mode.endswith("timing1"):
            kms, n = b.timing_read()
            b.timing(0)
            k = round(kms / 200, 3)
        res[f"{mode}:{rep}"] = {"ms_per_step": round(dt * 1e3 / 200, 3), "kernel_ms_per_step": k}
        b.close()
print(json.dumps(res))
