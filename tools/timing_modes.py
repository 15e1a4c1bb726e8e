#!/usr/bin/env python3
"""The headline's timed window (fresh 1M-env batch, 5 warm-up launches, 20 timed) with the 20
launches as one prepared graph replay vs plain launches: HIP-event region per launch and host wall
per launch. Kernel-only durations come from a rocprofv3 trace of the same run (measurement only)."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

net = load_network("bittner199")
res = {}
for mode in ("graph", "plain", "graph", "plain"):
    os.environ["PBNSIM_STEP_GRAPH"] = "1" if mode == "graph" else "0"
    b = PBNBatch(net, 1 << 20, seed=0x5EED)
    b.randomize()
    b.step(5)
    b.prepare_steps(20)
    b.sync()
    b.timing(2)
    t0 = time.perf_counter()
    b.step(20)
    b.timing(0)
    b.sync()
    t1 = time.perf_counter()
    ms, n = b.timing_read()
    b.close()
    res.setdefault(mode, []).append({"event_us": round(ms * 1e3 / n, 3), "wall_us": round((t1 - t0) * 1e6 / 20, 3)})
print(json.dumps(res))
