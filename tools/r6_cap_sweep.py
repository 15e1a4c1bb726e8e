"""How far the R6 until-attractor loop runs (pbn_target_multi.py:135-146, unbounded in the reference)
at config 5's shard: Bittner-200, B envs (131,072), A = 4 actions (0 w.p. 0.75), T env steps in one
fused launch per update cap, for both attractor specs bench.py reports:
  fixture -- the r6_bittner199 fixture's cubes (fix 165 of 199 bits);
  spec    -- SURVEY §8(d): 4 cubes over the 7 target genes (pbn_target_multi.py:354,415: nodes 0-6 of
             the exported network), the reference's own sample cabean attractors, other bits '*'.
Prints per (spec, cap): capped fraction, mean / p99 / max updates per env step, kernel ms.
Output of `python tools/r6_cap_sweep.py` -> profiles/r03_r6_cap_sweep.json."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT))
from bench import r6_attractors  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402


def main():
    import torch

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    caps = [int(c) for c in sys.argv[3].split(",")] if len(sys.argv) > 3 else [4096, 65536, 1 << 20]
    net = Net(load_network("bittner199"))
    dev = torch.device("cuda", 0)
    A, W = 4, net.n_words
    g = torch.Generator(device=dev)
    g.manual_seed(0xAC7)
    v = torch.randint(1, net.n_nodes + 1, (T, B, A), device=dev, generator=g, dtype=torch.int32)
    acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()
    o = torch.empty((T, B, W), dtype=torch.int64, device=dev)
    r = torch.empty((T, B), dtype=torch.int32, device=dev)
    f = torch.empty((T, B), dtype=torch.uint8, device=dev)
    n = torch.empty((T, B), dtype=torch.int32, device=dev)
    out = []
    for spec in ("fixture", "spec"):
        atts, desc = r6_attractors(spec, net.n_nodes)
        cfg = EnvConfig(net, atts, horizon=100)
        for cap in caps:
            b = PBNBatch(net, B, seed=0xAC7)
            b.env_reset(cfg)
            b.timing(1)
            b.env_rollout_multi_device(cfg, T, acts.data_ptr(), A, o.data_ptr(), r.data_ptr(), f.data_ptr(),
                                       n.data_ptr(), update_cap=cap)
            b.sync()
            ms, _ = b.timing_read()
            b.timing(0)
            nu = n.cpu().numpy().astype(np.int64)
            fl = f.cpu().numpy()
            row = {"attractors": spec, "update_cap": cap, "B": B, "T": T, "kernel_ms": ms,
                   "capped_frac": float(((fl & 4) != 0).mean()), "mean_updates": float(nu.mean()),
                   "p99_updates": float(np.percentile(nu, 99)), "max_updates": int(nu.max()),
                   "env_steps_per_s": B * T / (ms / 1e3)}
            print(json.dumps(row), flush=True)
            out.append(row)
            b.close()
    print(json.dumps({"sweep": out}))


if __name__ == "__main__":
    main()
