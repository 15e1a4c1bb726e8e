#!/usr/bin/env python3
"""Child of tools/valu_pmc.py (runs under rocprofv3 --pmc): the VALU-bound kernels of the bench
line with its sizes and seeds. Logs, in launch order, the node updates of every k_env launch and
of every k_rollout launch to gpurun_out/valu_child.json so the parent can divide the counters."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_pbn_amd.actions import env_actions  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch, attractors_from_cubes  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402


def main():
    log = []
    net = load_network("bittner199")
    B, T = 1 << 20, 64  # bench.py rollout supplement
    b = PBNBatch(net, B, seed=0x5EED)
    b.randomize()
    for _ in range(3):
        b.rollout(T)
        log.append(["k_rollout", f"k_rollout:bittner199:{B}:{T}", B * T])
    b.close()
    # bench.py r6_supplement, rank 0 of 1: same cubes, actions, seeds
    T, B, A, CAP = 100, 131072, 4, 4096
    z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz", allow_pickle=False)
    gnet = Net(net)
    cfg = EnvConfig(gnet, attractors_from_cubes(z["cube_care"], z["cube_value"], z["cube_attractor"], 199), horizon=T)
    dev = torch.device("cuda", 0)
    acts = env_actions(T, 0, B, A, 199, seed=0xAC7, device=dev)  # bench.py r6_figure's actions (rank 0)
    outs = [torch.empty((T, B, gnet.n_words), dtype=torch.int64, device=dev),
            torch.empty((T, B), dtype=torch.int32, device=dev),
            torch.empty((T, B), dtype=torch.uint8, device=dev),
            torch.empty((T, B), dtype=torch.int32, device=dev)]
    for fused in (False, True):
        b = PBNBatch(gnet, B, seed=0xAC7)
        for chunk in range(2):
            b.env_reset(cfg)
            if fused:
                b.env_rollout_multi_device(cfg, T, acts.data_ptr(), A, *[x.data_ptr() for x in outs], update_cap=CAP)
                b.sync()
                log.append(["k_env", f"k_env:bittner199:{B}:fused{T}", int(outs[3].to(torch.int64).sum())])
            else:
                for t in range(T):
                    b.env_step_multi_device(cfg, acts[t].data_ptr(), A, *[x[t].data_ptr() for x in outs],
                                            update_cap=CAP)
                    b.sync()
                    log.append(["k_env", f"k_env:bittner199:{B}:per_step", int(outs[3][t].to(torch.int64).sum())])
        b.close()
    out = ROOT / "gpurun_out" / "valu_child.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(log))


if __name__ == "__main__":
    main()
