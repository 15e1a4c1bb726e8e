#!/usr/bin/env python3
"""Child for rocprofv3 --pmc (measurement only): MT-mode steps of bench.py's workload (Bittner-199, 1,048,576
envs seeded 12345 + id, T = 256 per launch, 3 launches after one warm-up) on the library PBNSIM_LIB names."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
import numpy as np  # noqa: E402

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
b = PBNBatch(load_network("bittner199"), B, seed=1)
b.mt_seed(np.arange(B, dtype=np.uint64) + 12345, init_state=True)
for _ in range(4):
    b.mt_step(256)
b.sync()
b.close()
