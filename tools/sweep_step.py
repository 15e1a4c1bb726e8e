#!/usr/bin/env python3
"""Sweep step-kernel variants (envs per thread R, store mode) on one GPU; wall-clock per launch.

Run under `rocprofv3 --kernel-trace --stats` to get per-variant kernel durations
(the template arguments in the kernel names tell the variants apart).
"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

import torch  # noqa: E402,F401

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402


def run(net, B, R, store, steps=200, warm=20, rollout=0, sb=1024):
    os.environ["PBNSIM_STEP_BLOCK"] = str(sb)
    os.environ["PBNSIM_ENVS_PER_THREAD"] = str(R)
    os.environ["PBNSIM_STORE_MODE"] = str(store)
    b = PBNBatch(net, B, seed=11)
    b.randomize()
    if rollout:
        b.rollout(rollout)
        b.sync()
        t0 = time.perf_counter()
        for _ in range(5):
            b.rollout(rollout)
        b.sync()
        dt = (time.perf_counter() - t0) / 5
        print(f"{net.name:11s} B={B:8d} K={R} SB={sb} rollout T={rollout}: {dt*1e6:9.1f} us/launch  "
              f"{B*rollout/dt/1e9:8.1f} G upd/s", flush=True)
    else:
        b.step(warm)
        b.sync()
        t0 = time.perf_counter()
        b.step(steps)
        b.sync()
        dt = (time.perf_counter() - t0) / steps
        W = net.n_words
        print(f"{net.name:11s} B={B:8d} K={R} SB={sb} store={store}: {dt*1e6:7.2f} us/step  {B/dt/1e9:7.1f} G env-steps/s  "
              f"alg {16*W*B/dt/1e9:7.0f} GB/s", flush=True)
    b.close()


if __name__ == "__main__":
    nets = {n: load_network(n) for n in ("bittner199", "bittner28", "tt200")}
    if len(sys.argv) > 1 and sys.argv[1] == "sbcmp":
        for rep in range(2):
            for sb in (256, 1024):
                for K in (1, 2, 4):
                    run(nets["bittner199"], 1 << 20, K, 1, sb=sb)
        for sb in (256, 1024):
            run(nets["bittner199"], 1 << 23, 2, 1, steps=50, warm=5, sb=sb)
            run(nets["tt200"], 1 << 20, 2, 1, sb=sb)
            run(nets["bittner28"], 65536, 1, 1, sb=sb)
            run(nets["bittner199"], 1 << 20, 1, 1, rollout=64, sb=sb)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "kcmp":
        for rep in range(3):
            for K in (1, 2, 3, 4):
                run(nets["bittner199"], 1 << 20, K, 1)
        sys.exit(0)
    for K in (1, 2, 4, 8, 16):
        for store in (0, 1):
            run(nets["bittner199"], 1 << 20, K, store)
    for K in (1, 4):
        run(nets["bittner199"], 1 << 20, K, 1, rollout=64)
    for B in (1 << 22, 1 << 23):
        for K in (4, 16):
            run(nets["bittner199"], B, K, 1, steps=50, warm=5)
    for K in (1, 4):
        run(nets["tt200"], 1 << 20, K, 1)
        run(nets["bittner28"], 65536, K, 1)
        run(nets["bittner28"], 65536, K, 1, rollout=256)
