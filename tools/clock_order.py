#!/usr/bin/env python3
"""How the 1M-env step kernel's launch time depends on what ran before it (DVFS / fabric clock
ramp). Prints avg us per launch of 20-launch windows after different preceding work."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

net = load_network("bittner199")
b = PBNBatch(net, 1 << 20, seed=1)
b.randomize()
b.sync()


def win(n=20, k=1):
    out = []
    for _ in range(k):
        b.timing(2)
        b.step(n)
        b.timing(0)
        ms, l = b.timing_read()
        out.append(round(ms * 1e3 / l, 2))
    return out


res = {}
res["fresh_5_then_20"] = (b.step(5), win())[1]
res["ramp_50x20"] = win(20, 50)
time.sleep(1.0)
res["after_1s_idle_20x20"] = win(20, 20)
big = PBNBatch(net, 1 << 23, seed=2)
big.randomize()
big.step(250)
big.sync()
res["after_8M_250"] = win(20, 5)
time.sleep(0.5)
big.step(250)
big.sync()
b.step(5)
res["after_8M_250_then_5"] = win(20, 3)
big.close()
x = torch.empty(1 << 31, dtype=torch.uint8, device="cuda")
y = torch.empty_like(x)
time.sleep(0.5)
for _ in range(10):
    y.copy_(x)
torch.cuda.synchronize()
res["after_copy_2GiBx10"] = win(20, 3)
del x, y
time.sleep(0.5)
b.step(2000)
b.sync()
res["after_2000_steps"] = win(20, 3)
time.sleep(0.5)
b.rollout(64)
for _ in range(50):
    b.rollout(64)
b.sync()
res["after_rollout_50"] = win(20, 3)
print(json.dumps(res))
