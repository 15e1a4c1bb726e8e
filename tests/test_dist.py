"""The N>1 path on CPU: world_size-2 gloo processes (no GPU).

Each rank steps its contiguous shard of global env ids (here with the oracle,
the same Philox stream the kernels use), then the trajectory chunks are
all-gathered; the result must equal one process stepping the whole batch.
This is the partitioning bench.py uses across GPUs (weak scaling, no
collective in the stepping path).
"""

import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_local, T, out_dir):
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    import oracle as O
    from gym_pbn_amd.network import load_network
    from gym_pbn_amd.shard import gather_chunks, max_over_ranks, shard_for

    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = shard_for(rank, world, n_local)
    o = O.Oracle(load_network("bittner28"))
    st = o.init_philox(n_local, seed=99, env_base=sh.env_base)
    chunk = np.empty((n_local, T, o.W), dtype=np.uint64)
    for t in range(T):
        st = o.step_philox(st, 99, sh.env_base, t, 1)
        chunk[:, t] = st
    full = gather_chunks(chunk, dist)
    slowest = max_over_ranks(float(rank + 1), dist)
    if rank == 0:
        np.save(Path(out_dir) / "gathered.npy", full)
        np.save(Path(out_dir) / "slowest.npy", np.array([slowest]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_match_single_process(tmp_path, oracle_mod):
    from gym_pbn_amd.network import load_network

    n_local, T, world = 300, 12, 2
    mp.spawn(_worker, args=(world, _free_port(), n_local, T, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "gathered.npy")
    o = oracle_mod.Oracle(load_network("bittner28"))
    st = o.init_philox(world * n_local, seed=99, env_base=0)
    ref = np.empty_like(got)
    for t in range(T):
        st = o.step_philox(st, 99, 0, t, 1)
        ref[:, t] = st
    assert np.array_equal(got, ref)
    assert float(np.load(tmp_path / "slowest.npy")[0]) == 2.0


def test_shard_ranges():
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    from gym_pbn_amd.shard import shard_for

    shards = [shard_for(r, 8, 1 << 20) for r in range(8)]
    assert [s.env_base for s in shards] == [r << 20 for r in range(8)]
    assert shards[0].n_global == 8 << 20


def _gather_worker(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from gym_pbn_amd.rollout import alloc_chunk, gather_chunk

    dist.init_process_group("gloo", rank=rank, world_size=world)
    T, B, W = 3, 5, 4
    c = alloc_chunk(T, B, W, "cpu")
    g = torch.Generator().manual_seed(rank)
    c["obs"].copy_(torch.randint(-2**62, 2**62, (T, B, W), generator=g))
    c["reward"].copy_(torch.arange(T * B, dtype=torch.int32).view(T, B) + 1000 * rank)
    c["flags"].copy_(torch.randint(0, 8, (T, B), generator=g).to(torch.uint8))
    c["n_updates"].copy_(torch.randint(0, 5000, (T, B), generator=g).to(torch.int32))
    out, works = gather_chunk(c, dist, async_op=True)
    for w in works:
        w.wait()
    torch.save({k: v.clone() for k, v in c.items()}, Path(out_dir) / f"local{rank}.pt")
    if rank == 0:
        torch.save(out, Path(out_dir) / "gathered.pt")
    dist.barrier()
    dist.destroy_process_group()


def test_trajectory_chunk_gather_is_rank_major(tmp_path):
    """rollout.gather_chunk: [T][B_local]... per rank -> [world][T][B_local]..., every field (config 5)."""
    import torch

    world = 2
    mp.spawn(_gather_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = torch.load(tmp_path / "gathered.pt", weights_only=True)
    for r in range(world):
        loc = torch.load(tmp_path / f"local{r}.pt", weights_only=True)
        for k, v in loc.items():
            assert got[k].dtype == v.dtype and torch.equal(got[k][r], v), k


def _digest_worker(rank, world, port, n_global, T, out_dir):
    """bench.py's N > 1 self-check on CPU: rank r steps its shard (oracle = the kernels' Philox
    stream), re-runs the sampled global ids in its shard as 2-env batches (the bench's check, with the
    oracle in place of the GPU), digests every rank's rows in global-id order, and draws config 5's
    actions for its shard (actions.env_actions, keyed by global env id)."""
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import oracle as O
    from gym_pbn_amd.actions import env_actions
    from gym_pbn_amd.network import load_network
    from gym_pbn_amd.shard import gather_chunks, gather_rows, rows_digest, sampled_env_ids, shard_for

    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = shard_for(rank, world, n_global // world)
    net = load_network("bittner28")
    o = O.Oracle(net)
    st = o.step_philox(o.init_philox(sh.n_local, seed=7, env_base=sh.env_base), 7, sh.env_base, 0, T)
    rows, bad = [], 0
    for g in sampled_env_ids(sh.n_global, 16):
        if sh.env_base <= g < sh.env_base + sh.n_local - 1:
            mine = o.step_philox(o.init_philox(2, seed=7, env_base=g), 7, g, 0, T)
            ref = np.ascontiguousarray(st[g - sh.env_base:g - sh.env_base + 2])
            bad += 0 if np.array_equal(mine, ref) else 1
            rows.append((g, ref.tobytes()))
    all_rows = gather_rows(rows, dist)
    acts = env_actions(5, sh.env_base, sh.n_local, 4, net.n_nodes).numpy()  # [T][B_local][A]
    acts_all = gather_chunks(np.ascontiguousarray(acts.transpose(1, 0, 2)), dist)  # [B_global][T][A]
    bad_t = torch.tensor([float(bad)])
    dist.all_reduce(bad_t, op=dist.ReduceOp.MAX)
    if rank == 0:
        (Path(out_dir) / "digest.txt").write_text(f"{rows_digest(all_rows)} {len(all_rows)} {int(bad_t.item())}")
        np.save(Path(out_dir) / "actions.npy", acts_all)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_check_digest_and_actions_same_at_world_1_and_2(tmp_path, oracle_mod):
    n_global, T = 1000, 9
    res = {}
    for world in (1, 2):
        d = tmp_path / f"w{world}"
        d.mkdir()
        mp.spawn(_digest_worker, args=(world, _free_port(), n_global, T, str(d)), nprocs=world, join=True)
        dig, n, bad = (d / "digest.txt").read_text().split()
        assert int(bad) == 0 and int(n) == 16  # every sampled pair re-run alone equals its shard's rows
        res[world] = (dig, np.load(d / "actions.npy"))
    assert res[1][0] == res[2][0]  # one digest for one global batch, at any rank count
    assert np.array_equal(res[1][1], res[2][1])  # identical actions for the same global env ids
    a = res[1][1]
    assert a.shape == (n_global, 5, 4) and a.min() == 0 and a.max() <= 28 and 0.7 < (a == 0).mean() < 0.8
