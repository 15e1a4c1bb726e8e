"""bench.py's multi-rank bookkeeping rehearsed on CPU: two gloo ranks run bench.main() end to end --
headline window, supplements, config 5's three R6 figures with their per-chunk trajectory
all-gathers (rollout.TrajectoryCollector, the real class, on CPU tensors) -- with only the GPU
work stubbed (a stand-in PBNBatch; bench's device/process-group helpers on CPU). Every collective
each rank issues is recorded: both ranks must issue the same sequence (a rank that skipped or
reordered one would hang the other on RCCL), and it must contain the gathers and the max-over-ranks
reductions the line is built from. Also: a process group that cannot start (nccl on a host without
GPUs) ends ``bench.py --gpus 2`` promptly with a non-zero exit instead of hanging at a barrier."""

import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
COLLECTIVES = ("barrier", "all_reduce", "all_gather_into_tensor", "broadcast", "all_gather")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeBatch:
    """PBNBatch stand-in: the calls bench.py makes, no device."""

    def __init__(self, net, n_envs, device=0, env_id_base=0, seed=0):
        self.n_envs, self.n_words = int(n_envs), int(getattr(net, "n_words", 4))
        self._launches = 0

    def __getattr__(self, name):  # randomize, step, prepare_steps, sync, rollout, env_reset, *_device ...
        def call(*a, **k):
            if name in ("step",):
                self._launches += int(a[0]) if a else 1
        return call

    def timing(self, mode):
        self._launches = 0

    def timing_read(self):
        return 0.01 * max(self._launches, 1), max(self._launches, 1)

    def timing_read_each(self):
        return [0.01] * max(self._launches, 1)

    def env_handoffs(self):
        return 0

    def info(self):
        return {"env_lanes": 1, "roll_lanes": 1}

    def get_state(self):
        import numpy as np

        return np.zeros((self.n_envs, self.n_words), dtype=np.uint64)


class _FakeNet:
    def __init__(self, net):
        self.n_nodes, self.n_words, self.name = net.n_nodes, net.n_words, net.name


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    for p in (ROOT, ROOT / "gym-pbn-stac_amd"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as tdist

    import bench
    import gym_pbn_amd.batch as gb

    calls = []

    class _RecDist:
        def __getattr__(self, name):
            f = getattr(tdist, name)
            if name in COLLECTIVES:
                def rec(*a, **k):
                    shapes = [tuple(x.shape) for x in a if hasattr(x, "shape")]
                    calls.append([name, shapes])
                    return f(*a, **k)
                return rec
            return f

    def init_dist(backend, timeout_s):
        tdist.init_process_group("gloo", rank=rank, world_size=world)
        return _RecDist()

    bench._dev = lambda d: torch.device("cpu")
    bench._sync = lambda: None
    bench._set_device = lambda local: 0
    bench._init_dist = init_dist
    bench.window_changed_fraction = lambda *a: 0.4
    bench.copy_bandwidth = lambda device: 1000.0
    gb.PBNBatch = _FakeBatch
    gb.Net = _FakeNet
    gb.EnvConfig = lambda net, atts, horizon=100, **k: ("cfg", len(atts), horizon)
    sys.argv = ["bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "4096", "--r6-batch", "256",
                "--r6-chunks", "2", "--no-probe", "--dist-backend", "gloo", "--no-cpu-baseline"]
    out = Path(out_dir)
    with open(out / f"stdout{rank}.txt", "w") as fh:
        old, sys.stdout = sys.stdout, fh
        try:
            bench.main()
        finally:
            sys.stdout = old
    (out / f"calls{rank}.json").write_text(json.dumps(calls))


def test_two_rank_bench_bookkeeping_on_cpu(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    c0 = json.loads((tmp_path / "calls0.json").read_text())
    c1 = json.loads((tmp_path / "calls1.json").read_text())
    assert c0 == c1  # same collectives, same order, same shapes on both ranks
    names = [c[0] for c in c0]
    # three R6 figures (fixture/4096 with 2 chunks, high cap and spec attractors with 1), each run
    # per step and fused, each run once untimed (warm-up) and once timed: 4 fields gathered per
    # chunk, plus the standalone gather of each figure's last chunk
    n_chunks = 2 * 2 * (2 + 1 + 1)
    assert names.count("all_gather_into_tensor") == 4 * n_chunks + 4 * 3
    assert names.count("all_reduce") >= 2 + 3 * 2 * 2  # headline: time and kernel time; per R6 run: time, updates
    assert names[-1] == "barrier"
    lines = [ln for ln in (tmp_path / "stdout0.txt").read_text().splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not (tmp_path / "stdout1.txt").read_text().strip()
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * 4096
    r6 = d["config5_r6"]
    assert r6["global_batch"] == 512 and r6["attractors"] == "fixture" and r6["update_cap"] == 4096
    assert "all_gather_GBs_per_gpu" in r6
    assert r6["high_cap"]["attractors"] == "fixture" and r6["high_cap"]["update_cap"] > 4096
    assert r6["spec_attractors"]["attractors"] == "spec" and r6["spec_attractors"]["update_cap"] > 4096
    # the N > 1 line names its process group and checks its shards itself
    assert d["dist"]["backend"] == "gloo" and d["dist"]["world_size"] == 2
    assert [p["rank"] for p in d["dist"]["per_rank"]] == [0, 1]
    sc = d["shard_check"]
    assert sc["ranks"] == 2 and sc["match"] is True and sc["sampled_env_pairs"] == 32
    assert r6["shard_check"]["ranks"] == 2 and r6["shard_check"]["sampled_env_pairs"] == 16
    assert len(r6["chunk_diag"]) == 2 and "slowest_env_updates" in r6["chunk_diag"][0]
    assert "handoffs_last_fused_launch" in r6
    assert "process_census" in d


def test_failed_process_group_exits_nonzero_promptly():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    t0 = time.perf_counter()
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "nccl",
                        "--check-launch", "--dist-timeout", "60"], capture_output=True, text=True, timeout=240,
                       env=env)
    assert p.returncode != 0
    assert time.perf_counter() - t0 < 120
