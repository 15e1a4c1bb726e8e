#!/usr/bin/env python3
"""Step-mode launch time at small batches (Bittner-28, 65,536 envs: BASELINE config 2) per
envs-per-thread K and workgroup size; wall clock over 2,000 launches (measurement only)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from sweep_step import load_network, run  # noqa: E402

n28 = load_network("bittner28")
for rep in range(2):
    for sb in (256, 1024):
        for K in (1, 2, 4):
            run(n28, 65536, K, 1, steps=2000, warm=500, sb=sb)
