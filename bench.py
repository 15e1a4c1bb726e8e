#!/usr/bin/env python3
"""Benchmark: env-steps/s of the async PBN update on Bittner-200 at 1M envs per GPU.

Workload (BASELINE.json configs[2], metric "env-steps/sec (whole node), Bittner-200,
batch=1M; achieved HBM GB/s"): the exported ``predictor_sets_200_5_kmeans`` network
(N=199 nodes, 994 predictors, W=4 state words), 1,048,576 independent envs per GPU
resident in HBM as bit-packed uint64 words. One bench *step* = one R1 async
transition (``Graph.step``, base.py:306-312) for every env = one ``pbn_step`` launch
(state read from and written back to HBM). Philox4x32-10 RNG in-register.

Multi-GPU (``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``):
each rank owns 1,048,576 envs with global ids [rank*B, (rank+1)*B) -- weak scaling,
no data-path collective (envs are independent); barrier + max-over-ranks timing.

Prints ONE JSON line (rank 0) with ``roofline`` (algorithmic bytes / kernel time from
HIP events on the batch stream) and ``cpu_baseline`` (the oracle's C restatement on
host cores, rank 0 only).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--network", default="bittner199")
    p.add_argument("--batch", type=int, default=1 << 20, help="envs per GPU")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-events", action="store_true", help="time without per-launch HIP events")
    p.add_argument("--rollout", type=int, default=64, help="updates per launch for the supplementary rollout line")
    p.add_argument("--pmc-file", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    p.add_argument("--kernel-only", action="store_true", help="just run steps (for rocprofv3 child runs)")
    p.add_argument("--r6-chunks", type=int, default=2, help="config-5 supplement: timed T=100 chunks (0 = off)")
    p.add_argument("--r6-batch", type=int, default=131072, help="config-5 supplement: envs per GPU")
    p.add_argument("--no-config2", dest="config2", action="store_false", help="skip the Bittner-28 supplement")
    p.add_argument("--beyond-mall", action="store_true",
                   help="add the 8M-env (state past the MALL) step-mode supplement (off by default: it launches "
                        "the bench kernel at another size, which would mix into a rocprof average of the line)")
    p.add_argument("--dist-backend", default="nccl",
                   help="process group for the barrier / max-over-ranks timing (nccl = RCCL); gloo lets several "
                        "ranks share one GPU for rehearsals")
    return p.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return world, rank, local


def cpu_baseline(net, seconds: float):
    """Oracle (C restatement, same semantics and Philox stream) timed on host cores; bounded sample."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O

    O.build()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    o = O.Oracle(net)
    B = 65536
    st = o.init_philox(B, seed=1)
    T = 8
    t0 = time.perf_counter()
    o.step_philox(st, 1, 0, 0, T, n_threads=threads)
    dt = time.perf_counter() - t0
    T = max(8, int(T * seconds / max(dt, 1e-6)))
    t0 = time.perf_counter()
    o.step_philox(st, 1, 0, 0, T, n_threads=threads)
    dt = time.perf_counter() - t0
    return {"value": B * T / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pbn_oracle.c orc_step_philox, {net.name}, {B} envs x {T} updates "
                      f"({dt:.1f} s, OpenMP {threads} threads)",
            "reference_python_1core_measured_in_build_container": "20-28k env-steps/s (BASELINE.md)"}


def beyond_mall_supplement(net, device, seed):
    """Step mode on 8,388,608 envs on ONE GPU (BASELINE config 4's whole batch): 256 MiB of
    state, past the 256 MB MALL, so every launch streams the state from HBM. Algorithmic bytes
    / HIP-event kernel time, as for the main line."""
    from gym_pbn_amd.batch import PBNBatch

    B = 1 << 23
    b = PBNBatch(net, B, device=device, seed=seed)
    b.randomize()
    b.step(20)
    b.sync()
    b.timing(2)
    n = 100
    b.step(n)
    b.timing(0)
    ms, launches = b.timing_read()
    b.close()
    s = ms / 1e3 / max(launches, 1)
    alg = 16 * net.n_words * B
    return {"workload": "Bittner-200 step mode, 8,388,608 envs on one GPU (state 256 MiB > MALL)",
            "env_steps_per_s": B / s, "avg_kernel_us": s * 1e6, "alg_bytes_per_launch": alg,
            "achieved_GBs": alg / s / 1e9, "frac": alg / s / 1e9 / HBM_PEAK_GBS}


def copy_bandwidth(device, gib: float = 2.0, reps: int = 10):
    """Achievable HBM rate on this box: a device-to-device copy of a buffer far past the MALL,
    (read + write bytes) / time from CUDA events. Context for the roofline's fractions."""
    import torch

    n = int(gib * (1 << 30))
    src = torch.empty(n, dtype=torch.uint8, device=f"cuda:{device}")
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        dst.copy_(src)
    t1.record()
    torch.cuda.synchronize()
    s = t0.elapsed_time(t1) / 1e3 / reps
    del src, dst
    torch.cuda.empty_cache()
    return 2 * n / s / 1e9


def config2_supplement(device):
    """BASELINE config 2 beside the main line: Bittner-28 (predictor_sets_28_15_median, N = 28,
    one state word), 65,536 envs on one GPU (512 KiB of state: launch-bound in step mode), step
    mode (one Graph.step per env per launch) and rollout (256 updates per launch)."""
    from gym_pbn_amd.batch import PBNBatch
    from gym_pbn_amd.network import load_network

    B = 65536
    b = PBNBatch(load_network("bittner28"), B, device=device, seed=0x5EED)
    b.randomize()
    b.step(500)
    b.sync()
    b.timing(2)
    n = 2000
    b.step(n)
    b.timing(0)
    ms, launches = b.timing_read()
    b.rollout(256)
    b.sync()
    b.timing(2)
    for _ in range(5):
        b.rollout(256)
    b.timing(0)
    rms, rl = b.timing_read()
    lanes = b.info()["roll_lanes"]
    b.close()
    return {"workload": "Bittner-28, 65,536 envs, 1 GPU (BASELINE config 2)",
            "step_env_steps_per_s": B * n / (ms / 1e3), "step_us_per_launch": ms * 1e3 / max(launches, 1),
            "rollout_updates_per_launch": 256, "rollout_node_updates_per_s": B * 256 * 5 / (rms / 1e3),
            "rollout_lanes_per_env": lanes}


def r6_supplement(args, world, rank, device, dist):
    """BASELINE config 5 beside the main line: the multi-flip until-attractor env
    (pbn_target_multi.py:119-154) on Bittner-200, ``--r6-batch`` envs per GPU (131,072: 1M
    over 8 GPUs), T = horizon = 100 env steps per chunk written to a device chunk and
    all-gathered across ranks (RCCL) while the next chunk runs. Synthetic attractors: the
    r6_bittner199 fixture's cubes; A = 4 action slots (0 w.p. 0.75); update cap 4,096."""
    import numpy as np
    import torch

    from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch, attractors_from_cubes
    from gym_pbn_amd.network import load_network
    from gym_pbn_amd.rollout import TrajectoryCollector, gather_chunk
    from gym_pbn_amd.shard import max_over_ranks, shard_for

    T, B, A = 100, args.r6_batch, 4
    z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz", allow_pickle=False)
    net = Net(load_network("bittner199"))
    cfg = EnvConfig(net, attractors_from_cubes(z["cube_care"], z["cube_value"], z["cube_attractor"], net.n_nodes),
                    horizon=T)
    sh = shard_for(rank, world, B)
    dev = torch.device("cuda", device)
    g = torch.Generator(device=dev)
    g.manual_seed(0xAC7 + rank)
    v = torch.randint(1, net.n_nodes + 1, (T, B, A), device=dev, generator=g, dtype=torch.int32)
    acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()

    def run(fused):
        b = PBNBatch(net, B, device=device, env_id_base=sh.env_base, seed=0xAC7)
        col = TrajectoryCollector(b, cfg, T, A, dev, update_cap=4096, dist=dist, fused=fused)
        col.step_chunk(acts)  # warm-up chunk
        col.finish()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        ups = torch.zeros((), dtype=torch.int64, device=dev)
        t0 = time.perf_counter()
        for _ in range(args.r6_chunks):
            buf, _ = col.step_chunk(acts)
            ups += buf["n_updates"].to(torch.int64).sum()
        col.finish()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        dt = max_over_ranks(time.perf_counter() - t0, dist, device=dev)
        if dist is not None:
            dist.all_reduce(ups)
        lanes = b.info()["env_lanes"]
        return b, buf, dt, float(ups.item()), lanes

    # closed-loop shape first (one launch per env step, as an agent in the loop needs), then the
    # open-loop collector (actions known for the chunk: one launch walks each env through T steps)
    b, buf, dt_step, ups_step, _ = run(False)
    b.close()
    b, buf, dt, ups, lanes = run(True)
    out = {"metric": "R6 env-steps/s (whole node) incl. per-chunk trajectory all-gather", "unit": "env-steps/s",
           "value": world * B * T * args.r6_chunks / dt, "node_updates_per_s": ups / dt,
           "launch": "one per chunk (T env steps per env in one launch; actions known for the chunk)",
           "value_one_launch_per_env_step": world * B * T * args.r6_chunks / dt_step,
           "node_updates_per_s_one_launch_per_env_step": ups_step / dt_step,
           "batch_per_gpu": B, "global_batch": world * B, "T": T, "A": A, "update_cap": 4096, "env_lanes": lanes,
           "chunks": args.r6_chunks, "s_per_chunk": dt / args.r6_chunks,
           "chunk_bytes_per_gpu": sum(t.numel() * t.element_size() for t in buf.values())}
    if dist is not None:  # the gather alone: bytes received per GPU / time
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        gather_chunk(buf, dist)
        torch.cuda.synchronize()
        tg = max_over_ranks(time.perf_counter() - t0, dist, device=dev)
        out["all_gather_GBs_per_gpu"] = out["chunk_bytes_per_gpu"] * (world - 1) / tg / 1e9
        out["all_gather_s"] = tg
    b.close()
    return out


def main():
    args = parse()
    world, rank, local = dist_env()
    import numpy as np
    import torch

    from gym_pbn_amd import _lib
    from gym_pbn_amd.batch import PBNBatch
    from gym_pbn_amd.network import load_network
    from gym_pbn_amd.shard import max_over_ranks, shard_for

    dist = None
    if world > 1:
        import torch.distributed as dist

        ndev = max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local % ndev)
        dist.init_process_group(args.dist_backend)
    device = (local % max(torch.cuda.device_count(), 1)) if world > 1 else 0
    if torch.cuda.is_available():
        torch.cuda.set_device(device)

    net = load_network(args.network)
    B = args.batch
    shard = shard_for(rank, world, B)  # contiguous global env ids; Philox keyed by global id
    batch = PBNBatch(net, B, device=device, env_id_base=shard.env_base, seed=args.seed)
    batch.randomize()
    batch.sync()

    if args.kernel_only:
        batch.step(args.warmup + args.steps)
        batch.sync()
        return

    def barrier():
        if dist is not None:
            dist.barrier()

    batch.step(args.warmup)
    batch.sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    if not args.no_events:
        batch.timing(2)  # HIP events on the batch stream bracketing the timed launches
    t0 = time.perf_counter()
    batch.step(args.steps)
    if not args.no_events:
        batch.timing(0)  # closes the event region right behind the last launch
    batch.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    kernel_ms, launches = batch.timing_read() if not args.no_events else (float("nan"), 0)
    elapsed = max_over_ranks(t1 - t0, dist, device=f"cuda:{device}")
    kernel_ms = max_over_ranks(kernel_ms, dist, device=f"cuda:{device}")

    # supplementary: rollout mode (several updates per launch, state in registers)
    rollout = None
    if args.rollout > 1:
        batch.rollout(args.rollout)
        batch.sync()
        batch.timing(2)
        reps = 5
        for _ in range(reps):
            batch.rollout(args.rollout)
        batch.timing(0)
        rms, rl = batch.timing_read()
        rollout = {"updates_per_launch": args.rollout,
                   "node_updates_per_s_per_gpu": B * args.rollout * reps / (rms / 1e3),
                   "kernel_ms": rms / max(rl, 1)}

    beyond = None
    if rank == 0 and args.beyond_mall and B == 1 << 20:
        try:
            beyond = beyond_mall_supplement(net, device, args.seed)
        except Exception as exc:  # a supplement must not cost the main line
            beyond = {"error": f"{type(exc).__name__}: {exc}"}

    W = net.n_words
    alg_bytes = 16 * W * B  # read + write the packed state of every env
    avg_kernel_s = kernel_ms / 1e3 / max(launches, 1)
    achieved = alg_bytes / avg_kernel_s / 1e9 if launches else None
    traffic = None
    pmc_src = None
    try:
        pmc = json.loads(Path(args.pmc_file).read_text())
        key = f"{args.network}:{B}"
        if key in pmc.get("per_launch_bytes", {}):
            traffic = pmc["per_launch_bytes"][key]
            pmc_src = pmc.get("source")
    except (OSError, ValueError):
        pass

    total_steps = world * B * args.steps
    value = total_steps / elapsed
    if rank == 0:
        out = {
            "metric": "env-steps/sec (whole node), Bittner-200, batch=1M; achieved HBM GB/s",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (Philox fair-bit initial states; network exported from the reference's "
                    "predictor_sets_200_5_kmeans.pkl)",
            "config": {
                "workload": "Bittner-200 async node update (R1 Graph.step), step mode: one update per env per "
                            "launch, state resident in HBM",
                "network": args.network, "n_nodes": net.n_nodes, "state_words": W,
                "batch_per_gpu": B, "global_batch": world * B, "updates_per_step": 1,
                "parallelism": f"dp{world} (env shards, no collective)", "rng": "philox4x32-10",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "kernel": "pbn::k_step<4,1,1,0,1024> (W=4, predictor mix, dirty store, Philox, 1024-thread groups)",
                "timing": "HIP events on the batch stream bracketing the timed launches (launch gaps included)",
                "alg_bytes_per_launch": alg_bytes,
                "avg_kernel_us": avg_kernel_s * 1e6 if launches else None,
                "traffic_source": pmc_src,
                # measured HBM-side bytes per launch / launch time: the kernel stores only the
                # envs that changed and re-reads a 32 MiB state the 256 MB MALL can hold,
                # so the algorithmic rate above can exceed the HBM peak
                "traffic_GBs": (traffic / avg_kernel_s / 1e9) if (traffic and launches) else None,
                "traffic_frac": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if (traffic and launches) else None,
            },
            "node_updates_per_s": value,
            "rollout": rollout,
            "beyond_mall_8m": beyond,
        }
    batch.close()
    cfg2 = None
    if rank == 0 and args.config2:
        try:
            cfg2 = config2_supplement(device)
        except Exception as exc:  # a supplement must not cost the main line
            cfg2 = {"error": f"{type(exc).__name__}: {exc}"}
    r6 = None
    if args.r6_chunks > 0:
        try:
            r6 = r6_supplement(args, world, rank, device, dist)
        except Exception as exc:  # a supplement must not cost the main line
            r6 = {"error": f"{type(exc).__name__}: {exc}"}
    if rank == 0:
        try:  # achievable-copy rate on this box beside the spec peak
            copy = copy_bandwidth(device)
            rf = out["roofline"]
            rf["achievable_copy_GBs"] = copy
            rf["achievable_copy_source"] = ("torch device-to-device copy of 2 GiB (past the MALL), read + write "
                                            "bytes / CUDA-event time; the kernel's traffic_GBs also counts "
                                            "MALL-served fetches, so it can exceed this")
        except Exception as exc:  # a supplement must not cost the main line
            out["roofline"]["achievable_copy_GBs"] = f"error: {type(exc).__name__}: {exc}"
        out["config2_bittner28"] = cfg2
        out["config5_r6"] = r6
        if not args.no_cpu_baseline and world == 1:  # the host-core baseline: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline(net, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    del np, _lib


if __name__ == "__main__":
    main()
