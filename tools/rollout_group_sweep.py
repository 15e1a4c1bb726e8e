#!/usr/bin/env python3
"""Rollout throughput (node-updates/s, HIP events) in lane mode vs group mode (PBNSIM_ROLL_GROUP,
read at batch creation) over batch sizes. Measurement helper only."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
import torch  # noqa: E402,F401

from gym_pbn_amd.batch import Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

cases = [("bittner28", 65536, 256), ("bittner28", 16384, 256), ("bittner28", 262144, 256),
         ("bittner199", 65536, 256), ("bittner199", 131072, 128), ("bittner199", 262144, 64),
         ("bittner199", 1 << 20, 64)]
for name, B, T in cases:
    net = Net(load_network(name))
    for g in ("1", "2", "4", "8"):
        os.environ["PBNSIM_ROLL_GROUP"] = g
        b = PBNBatch(net, B, seed=3)
        b.randomize()
        b.rollout(T)
        b.sync()
        b.timing(2)
        for _ in range(5):
            b.rollout(T)
        b.sync()
        ms, _ = b.timing_read()
        print(f"{name} B={B} T={T} group={g} ms={ms / 5:.3f} G_updates_per_s={B * T * 5 / ms / 1e6:.1f}", flush=True)
        b.close()
