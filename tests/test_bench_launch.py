"""bench.py's multi-rank launch path (CPU, gloo): ``--gpus N`` without torch.distributed.run starts
N ranks as a child process; the line's ``n_gpus`` is the process group's world size; a ``--gpus``
that disagrees with an existing ``WORLD_SIZE`` is an error, not a silent one-rank run."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_2_spawns_two_ranks():
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--check-launch"], capture_output=True, text=True, timeout=300, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # one line, from rank 0
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["max_over_ranks_of_rank"] == 1.0


def test_gpus_mismatch_with_world_size_fails():
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--check-launch"],
                       capture_output=True, text=True, timeout=120, env=_env(WORLD_SIZE="1", RANK="0"))
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


@pytest.mark.gpu
def test_window_changed_fraction_matches_host_count():
    """The roofline's write-back fraction: the twin-batch measurement (device compares on one stream)
    equals counting changed envs from host copies of the same trajectory, launch by launch."""
    import numpy as np

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    import bench
    from gym_pbn_amd.batch import PBNBatch
    from gym_pbn_amd.network import load_network

    net = load_network("bittner199")
    B, seed, base, W, K = 5000, 0x5EED, 77, 5, 20
    q = bench.window_changed_fraction(net, B, 0, seed, base, W, K)
    b = PBNBatch(net, B, seed=seed, env_id_base=base)
    b.randomize()
    b.step(W)
    n = 0
    for _ in range(K):
        a = b.get_state()
        b.step(1)
        n += int(np.any(a != b.get_state(), axis=1).sum())
    b.close()
    assert q == n / (B * K) and 0.2 < q < 0.6
