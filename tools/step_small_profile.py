#!/usr/bin/env python3
"""Config 2 step mode (Bittner-28, 65,536 envs): 640 launches, for rocprofv3 --kernel-trace
(per-kernel duration vs the per-launch wall time). Measurement helper only."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
import torch  # noqa: E402,F401

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

b = PBNBatch(load_network("bittner28"), 65536, seed=1)
b.randomize()
b.step(640)
b.sync()
b.timing(2)
b.step(640)
b.timing(0)
ms, n = b.timing_read()
print(f"us_per_launch={ms * 1e3 / n:.3f}")
