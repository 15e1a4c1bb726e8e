#!/usr/bin/env python3
"""Does the config-5 per-step figure in bench.py depend on what ran before it? (measurement only)
Runs bench.r6_supplement alone, then after the rollout / config-2 / 8M supplements."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
import bench  # noqa: E402
import torch  # noqa: E402

from gym_pbn_amd.network import load_network  # noqa: E402

sys.argv = ["bench.py"]
args = bench.parse()
torch.cuda.set_device(0)
net = load_network(args.network)
out = {}


def r6(tag):
    t0 = time.perf_counter()
    r = bench.r6_supplement(args, 1, 0, 0, None, {})
    out[tag] = {"per_step_M": round(r["value_one_launch_per_env_step"] / 1e6, 1), "fused_M": round(r["value"] / 1e6, 1),
                "wall_s": round(time.perf_counter() - t0, 2)}
    print(tag, out[tag], flush=True)


r6("alone")
r6("alone_again")
bench.rollout_supplement(net, args.batch, 0, args.seed, args.rollout, {})
r6("after_rollout")
bench.config2_supplement(0)
r6("after_config2")
bench.beyond_mall_supplement(net, 0, args.seed, None)
r6("after_8m")
print(json.dumps(out))
