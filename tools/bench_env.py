#!/usr/bin/env python3
"""R6 multi-flip until-attractor env step throughput (per GPU).

Bittner-200 (199 nodes), B envs, A=4 action slots per env (0 w.p. 0.75, else uniform
node+1, Philox-like numpy stream seeded 0xAC7), attractor cubes = the r6_bittner199
fixture's synthetic hypercubes (165 fixed bits; cabean is unavailable), update cap 4096.
Reports env-steps/s and node-updates/s (sum of n_updates) over K env-step calls.
"""

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    net = load_network("bittner199")
    z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
    gnet = Net(net)
    cfg = EnvConfig(gnet, cubes_to_attractors(z, net.n_nodes), horizon=100)
    b = PBNBatch(gnet, B, seed=0xAC7)
    b.env_reset(cfg)
    rng = np.random.default_rng(0xAC7)
    acts = [rng.integers(1, net.n_nodes + 1, size=(B, 4)).astype(np.int32) for _ in range(K + 1)]
    for a in acts:
        a[rng.random(a.shape) < 0.75] = 0
    d_act = [torch.from_numpy(a).cuda() for a in acts]
    obs = torch.empty((B, net.n_words), dtype=torch.int64, device="cuda")
    rew = torch.empty(B, dtype=torch.int32, device="cuda")
    flg = torch.empty(B, dtype=torch.uint8, device="cuda")
    nup = torch.empty(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def call(a):
        b.env_step_multi_device(cfg, a.data_ptr(), 4, obs.data_ptr(), rew.data_ptr(), flg.data_ptr(),
                                nup.data_ptr(), update_cap=4096)

    call(d_act[0])
    b.sync()
    int(nup.to(torch.int64).sum().item())  # load torch's reduction kernels outside the timed loop
    tot_up = 0
    t0 = time.perf_counter()
    for k in range(K):
        call(d_act[k + 1])
        b.sync()
        tot_up += int(nup.to(torch.int64).sum().item())
    dt = time.perf_counter() - t0
    n = nup.cpu().numpy()
    f = flg.cpu().numpy()
    print(json.dumps({"B": B, "calls": K, "s_per_call": dt / K, "env_steps_per_s": B * K / dt,
                      "node_updates_per_s": tot_up / dt, "mean_updates": float(n.mean()),
                      "max_updates": int(n.max()), "capped_frac": float(((f & 4) != 0).mean()),
                      "terminated_frac": float(((f & 1) != 0).mean())}))


if __name__ == "__main__":
    main()
