#!/usr/bin/env python3
"""Step-kernel time in the driver's window (measurement only): Bittner-200, 1,048,576 fresh envs,
5 warm-up launches, then 20 launches inside one HIP-event region -- repeated on R fresh batches;
prints the median and all us-per-launch figures plus a digest of the final state (builds must agree).
Usage: PBNSIM_LIB=... python tools/step_time.py [R]"""
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 7
net = load_network("bittner199")
us, dig = [], None
for r in range(R):
    b = PBNBatch(net, 1 << 20, seed=0x5EED)
    b.randomize()
    b.step(5)
    b.prepare_steps(20)
    b.sync()
    b.timing(2)
    b.step(20)
    b.timing(0)
    ms, n = b.timing_read()
    us.append(ms * 1e3 / n)
    if r == 0:
        dig = hashlib.blake2b(b.get_state().tobytes(), digest_size=8).hexdigest()
    b.close()
print(json.dumps({"us_per_launch_median": sorted(us)[len(us) // 2], "us": [round(x, 3) for x in us], "state_digest": dig}))
