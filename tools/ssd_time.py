#!/usr/bin/env python3
"""Times the SSD reference default (300 envs x 4,000 iterations, p=0.01, 7 targets) on
Bittner-200 and TT-200, chunk-parallel wave mode vs serial apply (PBNSIM_SSD_SERIAL), with HIP
events; PBNSIM_LIB selects a measurement build. Measurement helper only."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
import torch  # noqa: E402,F401

from gym_pbn_amd.batch import Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

for name in ("bittner199", "tt200"):
    net = Net(load_network(name))
    for serial in ("0", "1"):
        os.environ["PBNSIM_SSD_SERIAL"] = serial  # read at batch creation
        for p in (0.01, 0.0):
            b = PBNBatch(net, 300, seed=1)
            b.randomize()
            b.ssd_counts(list(range(7)), 4000, p)
            b.sync()
            b.timing(2)
            b.ssd_counts(list(range(7)), 4000, p)
            b.sync()
            ms, _ = b.timing_read()
            print(f"{name} serial={serial} p={p} ssd_ms={ms:.3f}")
            b.close()
