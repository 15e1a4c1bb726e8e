#!/usr/bin/env python3
"""Config 5: R6 multi-flip env trajectories on every GPU + RCCL all-gather of each chunk.

SURVEY §8d config 5: ``PBNTargetMultiEnv.step`` (pbn_target_multi.py:119-154) on
Bittner-200, B_local envs per GPU (default 131,072; 8 GPUs = 1,048,576), A=4 action
slots per env (0 w.p. 0.75, else a uniform node+1), the r6_bittner199 fixture's
synthetic attractor hypercubes (cabean is unavailable), horizon 100, update cap 4096.
One chunk = reset + T env steps (T = horizon: one episode per env) written to a
device chunk, then all-gathered across ranks while the next chunk runs
(``gym_pbn_amd.rollout.TrajectoryCollector``).

Run: ``python tools/bench_r6.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_r6.py``.
Prints one JSON line on rank 0: env-steps/s and node-updates/s over all ranks, and the
all-gather volume per GPU.
"""

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402
from gym_pbn_amd.rollout import TrajectoryCollector  # noqa: E402
from gym_pbn_amd.shard import max_over_ranks, shard_for  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=131072, help="envs per GPU")
    p.add_argument("--T", type=int, default=100, help="env steps per chunk (= horizon)")
    p.add_argument("--chunks", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--cap", type=int, default=4096)
    p.add_argument("--per-step", action="store_true", help="one launch per env step (closed-loop shape)")
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
    sh = shard_for(rank, world, a.batch)
    net = load_network("bittner199")
    z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz")
    gnet = Net(net)
    cfg = EnvConfig(gnet, cubes_to_attractors(z, net.n_nodes), horizon=a.T)
    b = PBNBatch(gnet, a.batch, device=local, env_id_base=sh.env_base, seed=0xAC7)
    col = TrajectoryCollector(b, cfg, a.T, 4, dev, update_cap=a.cap, dist=dist, fused=not a.per_step)
    g = torch.Generator(device=dev)
    g.manual_seed(0xAC7 + rank)

    def actions():
        v = torch.randint(1, net.n_nodes + 1, (a.T, a.batch, 4), device=dev, generator=g, dtype=torch.int32)
        keep = torch.rand((a.T, a.batch, 4), device=dev, generator=g) >= 0.75
        return (v * keep).to(torch.int32).contiguous()

    acts = [actions() for _ in range(2)]
    for k in range(a.warmup):
        col.step_chunk(acts[k % 2])
    col.finish()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    tot_up = torch.zeros((), dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    for k in range(a.chunks):
        buf, _ = col.step_chunk(acts[k % 2])
        tot_up += buf["n_updates"].to(torch.int64).sum()
    col.finish()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = max_over_ranks(time.perf_counter() - t0, dist, device=dev)
    ups = float(tot_up.item())
    if dist is not None:
        t = torch.tensor([ups], dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        ups = float(t.item())
    f = buf["flags"].cpu().numpy()
    n = buf["n_updates"].cpu().numpy()
    chunk_bytes = sum(v.numel() * v.element_size() for v in buf.values())
    if rank == 0:
        print(json.dumps({
            "metric": "R6 env-steps/sec (whole node), Bittner-200 multi-flip until-attractor, trajectories gathered",
            "value": world * a.batch * a.T * a.chunks / dt, "unit": "env-steps/s", "n_gpus": world,
            "node_updates_per_s": ups / dt, "s_per_chunk": dt / a.chunks,
            "config": {"batch_per_gpu": a.batch, "global_batch": world * a.batch, "T": a.T, "A": 4,
                       "update_cap": a.cap, "launch": "one per env step" if a.per_step else "one per chunk",
                       "env_lanes": b.info()["env_lanes"], "gather": "all_gather_into_tensor per chunk (rccl)" if world > 1
                       else "none (1 rank)"},
            "chunk_bytes_per_gpu": chunk_bytes, "gathered_bytes_per_gpu_per_chunk": chunk_bytes * world,
            "last_chunk": {"mean_updates": float(n.mean()), "max_updates": int(n.max()),
                           "capped_frac": float(((f & 4) != 0).mean()),
                           "terminated_frac": float(((f & 1) != 0).mean())}}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
