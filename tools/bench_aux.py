#!/usr/bin/env python3
"""Throughput of the secondary kernels (one GPU): SSD histogram, synchronous step, MT mode.

* SSD (``compute_ssd_hist``, utils/eval.py:20-103): the reference default -- 300 resets x
  4,000 iterations (1.2M transitions, bit-flip p=0.01, 7 target genes) -- and a wide run
  (1M envs x 200 iterations) on Bittner-200.
* synchronous step (``Graph.synch_step``, base.py:286-303): 1M envs x 20 steps, perturbation
  p=0.001 (base.py:191) -> node-updates/s (N updates per env-step).
* MT mode (seed-only parity): 65,536 envs x 2,000 R1 updates.
* BASELINE config 2 (Bittner-28, 65,536 envs): step mode and rollout (256 updates per launch).

Prints one JSON line. Timing: HIP events over the region (``PBNBatch.timing(2)``).
"""

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from gym_pbn_amd.batch import Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402


def timed(b, fn):
    fn()  # warm (module load, first launch)
    b.sync()
    b.timing(2)
    t0 = time.perf_counter()
    fn()
    b.sync()
    wall = time.perf_counter() - t0
    ms, n = b.timing_read()
    b.timing(0)
    return ms / 1e3, wall, n


def main():
    net = Net(load_network("bittner199"))
    N = net.n_nodes
    targets = list(range(7))
    out = {}
    b = PBNBatch(net, 300, seed=1)
    b.randomize()
    s, wall, _ = timed(b, lambda: b.ssd_counts(targets, 4000, 0.01))
    out["ssd_reference_default"] = {"envs": 300, "iters": 4000, "transitions": 1.2e6, "s": s, "wall_s": wall,
                                    "transitions_per_s": 1.2e6 / s}
    b.close()
    B, it = 1 << 20, 200
    b = PBNBatch(net, B, seed=2)
    b.randomize()
    s, wall, _ = timed(b, lambda: b.ssd_counts(targets, it, 0.01))
    out["ssd_wide"] = {"envs": B, "iters": it, "s": s, "transitions_per_s": B * it / s}
    T = 20
    s, wall, _ = timed(b, lambda: b.synch_step(T, 0.001))
    out["synch_step"] = {"envs": B, "steps": T, "s": s, "env_steps_per_s": B * T / s,
                         "node_updates_per_s": B * T * N / s, "perturbation_p": 0.001}
    b.close()
    B, T = 1 << 16, 2000
    b = PBNBatch(net, B, seed=3)
    b.mt_seed(np.arange(B, dtype=np.uint64))
    s, wall, _ = timed(b, lambda: b.mt_step(T))
    out["mt_step"] = {"envs": B, "updates": T, "s": s, "node_updates_per_s": B * T / s}
    b.close()
    # BASELINE config 2: Bittner-28, 65,536 envs (state 512 KiB: launch-bound in step mode)
    n28 = Net(load_network("bittner28"))
    b = PBNBatch(n28, 1 << 16, seed=5)
    b.randomize()

    def steps28():
        for _ in range(200):
            b.step(1)

    s, wall, n = timed(b, steps28)
    s2, _, n2 = timed(b, lambda: b.rollout(256))
    out["bittner28_64k"] = {"envs": 1 << 16, "step_us_per_launch": s / n * 1e6,
                            "step_env_steps_per_s": (1 << 16) * n / s,
                            "rollout256_node_updates_per_s": (1 << 16) * 256 * n2 / s2}
    b.close()
    B = 8 << 20
    b = PBNBatch(net, B, seed=4)
    b.randomize()

    def steps():
        for _ in range(100):
            b.step(1)

    s, wall, n = timed(b, steps)
    out["step_8M"] = {"envs": B, "launches": n, "us_per_launch": s / n * 1e6, "env_steps_per_s": B * n / s,
                      "alg_GBs": 64 * B * n / s / 1e9}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
