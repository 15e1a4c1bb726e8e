#!/usr/bin/env python3
"""What the bench headline's short window (--warmup 5 --steps 20) sees after each supplement:
20-launch windows of the 1M-env step kernel on a FRESH batch, right after heavy R6 compute,
after the 8M-env step run, after the copy-bandwidth probe. Prints one JSON object."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

net = load_network("bittner199")


def fresh_windows(k=6, warm=5):
    b = PBNBatch(net, 1 << 20, seed=0x5EED)
    b.randomize()
    b.step(warm)
    b.sync()
    out = []
    for _ in range(k):
        b.timing(2)
        b.step(20)
        b.timing(0)
        ms, n = b.timing_read()
        out.append(round(ms * 1e3 / n, 2))
    b.close()
    return out


class A:
    r6_batch = 131072
    r6_chunks = 2


res = {}
res["fresh_process"] = fresh_windows()
t0 = time.perf_counter()
bench.r6_supplement(A, 1, 0, 0, None, {})
res["r6_s"] = round(time.perf_counter() - t0, 2)
res["after_r6"] = fresh_windows()
bench.r6_supplement(A, 1, 0, 0, None, {})
big = PBNBatch(net, 1 << 23, seed=2)
big.randomize()
big.step(250)
big.sync()
big.close()
res["after_r6_then_8M_250"] = fresh_windows()
bench.r6_supplement(A, 1, 0, 0, None, {})
bench.copy_bandwidth(0)
res["after_r6_then_copy"] = fresh_windows()
b = PBNBatch(net, 1 << 20, seed=1)
b.randomize()
b.step(3000)
b.sync()
b.close()
res["after_3000_steps"] = fresh_windows()
time.sleep(2.0)
res["after_2s_idle"] = fresh_windows()
print(json.dumps(res))
