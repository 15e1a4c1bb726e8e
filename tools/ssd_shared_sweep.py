#!/usr/bin/env python3
"""SSD reference default (300 envs x 4,000 iterations, p = 0.01) and 4,096 envs x 640 in shared
mode with 4 vs 8 waves per env (PBNSIM_SSD_SHARED) and one wave per env. Measurement helper only."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
import torch  # noqa: E402,F401

from gym_pbn_amd.batch import Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

for name in ("bittner199", "tt200"):
    net = Net(load_network(name))
    for B, iters in ((300, 4000), (1024, 2048), (4096, 640)):
        for w in ("0", "4", "8"):
            os.environ["PBNSIM_SSD_SHARED"] = w
            b = PBNBatch(net, B, seed=1)
            b.randomize()
            b.ssd_counts(list(range(7)), 64, 0.01)
            b.sync()
            b.timing(2)
            b.ssd_counts(list(range(7)), iters, 0.01)
            b.sync()
            ms, _ = b.timing_read()
            print(f"{name} B={B} iters={iters} waves_per_env={w} ms={ms:.3f} G_per_s={B * iters / ms / 1e6:.2f}",
                  flush=True)
            b.close()
