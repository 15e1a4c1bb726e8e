#!/usr/bin/env python3
"""SSD throughput (transitions/s, HIP events) by batch size in lane mode (PBNSIM_SSD_WAVE=0),
one wave per env (WAVE=1, SHARED=0) and four waves per env (WAVE=1, SHARED=1); Bittner-200,
p = 0.01, 7 targets, ~40 M transitions per point. Measurement helper only."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
import torch  # noqa: E402,F401

from gym_pbn_amd.batch import Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

net = Net(load_network("bittner199"))
modes = {"lane": ("0", "0"), "wave": ("1", "0"), "shared": ("1", "1")}
for B in (1024, 4096, 16384, 65536, 262144):
    iters = max(64, (40_000_000 // B) // 64 * 64)
    for m, (wave, shared) in modes.items():
        if m == "shared" and B > 16384:
            continue
        os.environ["PBNSIM_SSD_WAVE"], os.environ["PBNSIM_SSD_SHARED"] = wave, shared
        b = PBNBatch(net, B, seed=1)
        b.randomize()
        b.ssd_counts(list(range(7)), 64, 0.01)
        b.sync()
        b.timing(2)
        b.ssd_counts(list(range(7)), iters, 0.01)
        b.sync()
        ms, _ = b.timing_read()
        print(f"B={B} iters={iters} mode={m} ms={ms:.3f} G_transitions_per_s={B * iters / ms / 1e6:.2f}", flush=True)
        b.close()
