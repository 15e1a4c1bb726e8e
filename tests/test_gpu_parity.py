"""Parity of the gfx950 kernels (through the C ABI) with the oracle and the reference fixtures.

Bit-exact everywhere: the path is integer-only. Sizes are small enough for the
oracle to finish in seconds; the 1M-env cases check size-independent
properties (shard invariance, step == rollout, sampled envs vs the oracle).
"""

import os
import zlib

import numpy as np
import pytest

from conftest import cubes_to_attractors, golden, r6_config
from gym_pbn_amd.network import load_network

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    from gym_pbn_amd import _lib, batch

    assert _lib.device_count() >= 1, "gpu tests need a HIP device"
    return batch


# ----------------------------------------------------------------- replay vs reference fixtures
@pytest.mark.parametrize("name,kind", [("bittner28", "r1"), ("bittner199", "r1"), ("bittner70", "r1"),
                                       ("tt200", "r4"), ("tt8", "r4")])
def test_replay_matches_reference_trajectories(G, name, kind):
    """Feed the reference's own draws; every intermediate state must equal the reference's."""
    z = golden(f"{kind}_{name}.npz")
    S, T = z["node_idx"].shape
    b = G.PBNBatch(name, S)
    b.set_state(z["init"])
    # one update per call for the first 64 steps (state round-trips HBM), then the rest in one launch
    for t in range(64):
        b.step_replay(z["node_idx"][:, t][None], z["k53"][:, t][None])
        assert np.array_equal(b.get_state(), z["states"][:, t]), t
    b.step_replay(z["node_idx"][:, 64:].T.copy(), z["k53"][:, 64:].T.copy())
    assert np.array_equal(b.get_state(), z["states"][:, -1])


def test_single_env_b1_plumbing(G):
    """Config 1 (B=1, Bittner-28): the reference trajectory, one env, update by update."""
    z = golden("r1_bittner28.npz")
    b = G.PBNBatch("bittner28", 1)
    b.set_state(z["init"][:1])
    for t in range(300):
        b.step_replay(z["node_idx"][0, t:t + 1][None], z["k53"][0, t:t + 1][None])
        assert np.array_equal(b.get_state()[0], z["states"][0, t])


@pytest.mark.parametrize("name,B,base", [("bittner199", 4099, 77), ("bittner28", 1024, 64), ("tt200", 2048, 9)])
def test_step_forced_matches_oracle(G, oracle_mod, name, B, base):
    """``Graph.step(i=k)`` (base.py:306-309): the caller's node, the Philox choice draw of that update;
    forced updates interleave with ``step`` / ``rollout`` on one update counter."""
    net = load_network(name)
    o = oracle_mod.Oracle(net)
    b = G.PBNBatch(net, B, seed=99, env_id_base=base)
    b.randomize()
    st = b.get_state()
    lo = 1 if net.kind == 2 else 0
    ni = np.random.default_rng(B).integers(lo, net.n_nodes, size=(5, B)).astype(np.uint32)
    b.step_forced(ni)
    st = o.step_forced(st, ni, 99, base, 0)
    assert np.array_equal(b.get_state(), st)
    b.step(3)  # continues at update 5
    st = o.step_philox(st, 99, base, 5, 3)
    assert np.array_equal(b.get_state(), st)
    b.step_forced(ni[:1])  # update 8
    assert np.array_equal(b.get_state(), o.step_forced(st, ni[:1], 99, base, 8))
    with pytest.raises(Exception):
        b.step_forced(np.full((1, B), net.n_nodes, np.uint32))


def test_graph_step_forced_node(G, oracle_mod):
    """Single env: ``Graph.step(i=k)`` changes at most node k, equals the oracle, takes Python list
    indexing (negative k) and raises IndexError out of range like ``self.nodes[i]``."""
    from gym_pbn_amd.envs import Graph

    net = load_network("bittner199")
    o = oracle_mod.Oracle(net)
    g = Graph(net, seed=5, env_id=3)
    g.genRandState()
    words = o.init_philox(1, seed=5, env_base=3)
    assert g.getState() == tuple(oracle_mod.unpack_bits(words, net.n_nodes)[0].tolist())
    u = 0
    for k in [0, 17, 198, -1, -199, 42, 42, 42]:
        s0 = g.getState()
        s1 = g.step(i=k)
        node = k % net.n_nodes
        assert all(a == b for j, (a, b) in enumerate(zip(s0, s1)) if j != node)
        words = o.step_forced(words, np.array([[node]], np.uint32), 5, 3, u)
        u += 1
        assert s1 == tuple(oracle_mod.unpack_bits(words, net.n_nodes)[0].tolist()), k
    s = g.step()  # the unforced step draws update u's node
    assert s == tuple(oracle_mod.unpack_bits(o.step_philox(words, 5, 3, u, 1), net.n_nodes)[0].tolist())
    for bad in (199, -200):
        with pytest.raises(IndexError):
            g.step(i=bad)


# ----------------------------------------------------------------- Philox mode vs oracle
# an even env base puts envs 2m / 2m + 1 (which share a Philox call) in lane pairs that swap words
# over DPP; an odd base takes the one-call-per-env path
@pytest.mark.parametrize("base", [77, 64])
@pytest.mark.parametrize("name,B,T", [("bittner28", 4096, 64), ("bittner199", 8192, 40), ("tt200", 4096, 40),
                                      ("bittner70", 3001, 33), ("tt8", 1000, 50), ("syn500", 2048, 24)])
def test_philox_step_matches_oracle(G, oracle_mod, name, B, T, base):
    if name == "syn500":  # W = 8 state words: the largest network the build takes (N <= 512)
        from gym_pbn_amd.network import PredictorNetwork, synthetic_predictor_sets

        net = PredictorNetwork.from_predictor_sets(*synthetic_predictor_sets(500, 4, seed=500), name="syn500")
        assert net.n_words == 8
    else:
        net = load_network(name)
    o = oracle_mod.Oracle(net)
    b = G.PBNBatch(net, B, seed=1234, env_id_base=base)
    b.randomize()
    init = b.get_state()
    assert np.array_equal(init, o.init_philox(B, seed=1234, env_base=base))
    b.step(T)  # T launches, one update each
    assert np.array_equal(b.get_state(), o.step_philox(init, 1234, base, 0, T))
    b.rollout(T)  # T updates in registers, counters continue (odd T: the last pair half-used)
    assert np.array_equal(b.get_state(), o.step_philox(init, 1234, base, 0, 2 * T))


@pytest.mark.parametrize("graph", ["1", "0"])
@pytest.mark.parametrize("name", ["bittner199", "tt200"])
def test_step_graph_replays_match_oracle(G, oracle_mod, monkeypatch, graph, name):
    """pbn_step sends runs of launches as captured HIP graphs of 64, 32, ..., 2 launches (update
    counter read from device memory): replays continue the counter exactly for every run length,
    across calls and mixed with plain launches and rollouts; region timing counts every launch."""
    monkeypatch.setenv("PBNSIM_STEP_GRAPH", graph)
    net = load_network(name)
    o = oracle_mod.Oracle(net)
    B = 5000
    b = G.PBNBatch(net, B, seed=71, env_id_base=13)
    b.randomize()
    init = b.get_state()
    b.step(64 * 3 + 7)  # three 64-replays, then the 4- and 2-graphs and one plain launch
    b.rollout(5)
    b.step(64)
    assert np.array_equal(b.get_state(), o.step_philox(init, 71, 13, 0, 64 * 4 + 12))
    b.timing(2)
    b.step(128)
    b.timing(0)
    ms, launches = b.timing_read()
    assert launches == 128 and ms > 0
    assert np.array_equal(b.get_state(), o.step_philox(init, 71, 13, 0, 64 * 6 + 12))
    done = 64 * 6 + 12
    for n in (1, 2, 3, 5, 20, 63, 127, 1):  # every binary digit of a run below 64 is its own graph
        b.timing(2)
        b.step(n)
        b.timing(0)
        assert b.timing_read()[1] == n
        done += n
        assert np.array_equal(b.get_state(), o.step_philox(init, 71, 13, 0, done)), n
    b.close()


@pytest.mark.parametrize("block", ["256", "1024"])
def test_step_block_sizes_match_oracle(G, oracle_mod, monkeypatch, block):
    """Step mode with the workgroup size forced (PBNSIM_STEP_BLOCK: 1,024-thread groups are picked for
    batches that fill the GPU, 256 below): both sizes at a ragged batch, every env against the oracle."""
    monkeypatch.setenv("PBNSIM_STEP_BLOCK", block)
    net = load_network("bittner199")
    o = oracle_mod.Oracle(net)
    B = 300001
    b = G.PBNBatch(net, B, seed=17, env_id_base=5)
    b.randomize()
    init = b.get_state()
    b.step(7)
    assert np.array_equal(b.get_state(), o.step_philox(init, 17, 5, 0, 7, n_threads=16))
    b.close()


@pytest.mark.parametrize("base", [9, 10])
@pytest.mark.parametrize("k", ["1", "2", "4", "8"])
@pytest.mark.parametrize("name,B", [("bittner199", 70001), ("bittner28", 300001), ("tt200", 40000)])
def test_envs_per_thread_match_oracle(G, oracle_mod, monkeypatch, k, name, B, base):
    """Step mode with 1, 2, 4 or 8 envs per thread (the grid-stride pairs of k_step_single): ragged
    batches (the last env's DPP partner lane has left the loop), odd and even env bases, every env
    against the oracle, graph-replayed and plain launches."""
    monkeypatch.setenv("PBNSIM_ENVS_PER_THREAD", k)
    net = load_network(name)
    o = oracle_mod.Oracle(net)
    b = G.PBNBatch(net, B, seed=404, env_id_base=base)
    b.randomize()
    init = b.get_state()
    b.step(3)
    b.step(1)
    assert np.array_equal(b.get_state(), o.step_philox(init, 404, base, 0, 4))
    b.close()


def test_exact_length_step_graphs_match_oracle(G, oracle_mod):
    """pbn_step_prepare(n) captures one graph of exactly n launches without running anything; a
    length called twice in a row gets one too; the batch keeps four lengths (least recently used
    evicted). Every replay continues the update counter exactly."""
    net = load_network("bittner199")
    o = oracle_mod.Oracle(net)
    b = G.PBNBatch(net, 4099, seed=19, env_id_base=7)
    b.randomize()
    init = b.get_state()
    b.prepare_steps(20)
    b.prepare_steps(1)  # no-op
    assert np.array_equal(b.get_state(), init)  # setup only
    done = 0
    for n in (20, 20, 7, 7, 7, 33, 33, 5, 5, 9, 9, 20, 3, 20):  # 5 lengths through 4 slots
        b.timing(2)
        b.step(n)
        b.timing(0)
        ms, launches = b.timing_read()
        assert launches == n and ms > 0
        done += n
        assert np.array_equal(b.get_state(), o.step_philox(init, 19, 7, 0, done)), n
    b.timing(2)  # a region mixing an exact graph with plain launches and other graphs
    b.step(20)
    b.step(1)
    b.step(20)
    b.rollout(3)
    b.timing(0)
    ms, launches = b.timing_read()
    assert launches == 42 and ms > 0  # 41 step launches + one rollout launch (3 updates)
    done += 44
    assert np.array_equal(b.get_state(), o.step_philox(init, 19, 7, 0, done))
    b.prepare_steps(200)  # above 64: the power-of-two graphs
    b.step(200)
    done += 200
    assert np.array_equal(b.get_state(), o.step_philox(init, 19, 7, 0, done))
    with pytest.raises(Exception):
        b.prepare_steps(4097)
    b.close()


def test_config2_exact_size_matches_oracle(G, oracle_mod):
    """BASELINE config 2 at its exact size: 65,536 Bittner-28 envs (Graph.step, base.py:306-312).
    The library's own choices at this size, no overrides: step runs of 20 launches go out as one
    graph replay, and rollout picks the 2-lanes-per-env group kernel (k_rollout_grp<1,2>). Every env
    against the oracle."""
    net = load_network("bittner28")
    o = oracle_mod.Oracle(net)
    B, seed = 65536, 0x5EED
    b = G.PBNBatch(net, B, seed=seed)
    b.randomize()
    init = b.get_state()
    assert np.array_equal(init, o.init_philox(B, seed=seed))
    b.step(20)
    b.step(20)  # the second call of the same length replays its captured graph
    assert np.array_equal(b.get_state(), o.step_philox(init, seed, 0, 0, 40, n_threads=8))
    b.rollout(256)
    assert b.info()["roll_lanes"] == 2
    assert np.array_equal(b.get_state(), o.step_philox(init, seed, 0, 0, 40 + 256, n_threads=8))
    b.close()


def test_exact_graph_eviction_without_host_sync(G, oracle_mod):
    """Six lengths cycled through the four exact-length slots with no host sync between calls: every
    capture past the fourth evicts a graph whose replay may still be queued on the batch stream
    (pbn_abi.cpp exact_graph_build drains the stream before destroying it). The state after the
    whole run equals the oracle's."""
    net = load_network("bittner199")
    o = oracle_mod.Oracle(net)
    b = G.PBNBatch(net, 20001, seed=23, env_id_base=2)
    b.randomize()
    init = b.get_state()
    done = 0
    for _ in range(2):
        for n in (4, 6, 9, 12, 17, 25):  # each length twice in a row: captured at its second call
            b.step(n)
            b.step(n)
            done += 2 * n
    assert np.array_equal(b.get_state(), o.step_philox(init, 23, 2, 0, done))
    b.close()


def _syn_cubes(rng, n_nodes, n_cubes, n_care):
    """Random attractor cubes over n_care nodes each (attractor h = cube h), packed [H][W]."""
    W = (n_nodes + 63) // 64
    care = np.zeros((n_cubes, W), np.uint64)
    value = np.zeros((n_cubes, W), np.uint64)
    for h in range(n_cubes):
        for i in rng.choice(n_nodes, n_care, replace=False):
            care[h, i // 64] |= np.uint64(1) << np.uint64(i % 64)
            if rng.random() < 0.5:
                value[h, i // 64] |= np.uint64(1) << np.uint64(i % 64)
    return care, value


@pytest.mark.parametrize("n_nodes", [150, 500])
def test_small_pmax_network_matches_oracle(G, oracle_mod, n_nodes):
    """pmax = 2 (every node two predictors): the compact image of the Philox kernels is larger than
    the u64 image here, so k_step / k_rollout place their planes past it (NetLayout.plane_off) while
    the env kernel stages the u64 image's size. Step, rollout and the R6 env step vs the oracle."""
    from gym_pbn_amd.network import PredictorNetwork, synthetic_predictor_sets

    net = PredictorNetwork.from_predictor_sets(*synthetic_predictor_sets(n_nodes, 2, seed=n_nodes, ragged=False),
                                               name=f"syn{n_nodes}p2")
    o = oracle_mod.Oracle(net)
    B, seed, base = 6000, 31, 4
    b = G.PBNBatch(net, B, seed=seed, env_id_base=base)
    b.randomize()
    init = b.get_state()
    b.step(5)
    b.rollout(7)
    assert np.array_equal(b.get_state(), o.step_philox(init, seed, base, 0, 12))
    # R6: three cubes over 5 nodes each; attractor 0 for reset, the last as target
    care, value = _syn_cubes(np.random.default_rng(n_nodes), n_nodes, 3, 5)
    gnet = G.Net(net)
    cfg = G.EnvConfig(gnet, G.attractors_from_cubes(care, value, np.arange(3), n_nodes), horizon=10)
    cfgd = dict(care=care, value=value, target_care=care[2], target_value=value[2], reset_care=care[:1],
                reset_value=value[:1], horizon=10)
    e = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    e.env_reset(cfg)
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), care[:1], value[:1],
                                seed=seed, env_base=base, reset_count=0)
    assert np.array_equal(e.get_state(), st)
    rng = np.random.default_rng(1)
    for t in range(3):
        acts = rng.integers(0, n_nodes + 1, size=(B, 2)).astype(np.int32)
        obs, rew, flags, nup = e.env_step_multi(cfg, acts, update_cap=2048)
        ref = o.env_step_multi(cfgd, st, ns, acts, seed=seed, env_base=base, call_idx=t, update_cap=2048)
        assert np.array_equal(nup, ref["n_updates"]) and np.array_equal(obs, ref["obs"]), t
        assert np.array_equal(rew, ref["reward"]) and np.array_equal(flags, ref["flags"]), t
        st, ns = ref["state"], ref["n_steps"]
    b.close()
    e.close()


def test_step_inside_a_torch_graph_capture(G, oracle_mod):
    """pbn_step on a stream the caller is capturing (torch.cuda.graph) launches plainly into the
    caller's graph instead of capturing one of its own; replaying the caller's graph repeats the
    captured launches (same update counters), as any captured launch does."""
    import torch

    net = load_network("bittner199")
    o = oracle_mod.Oracle(net)
    b = G.PBNBatch(net, 3000, seed=5, env_id_base=1)
    b.randomize()
    init = b.get_state()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        b.set_stream(s.cuda_stream)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            b.step(70)  # >= 64: would use the batch's own graph outside a capture
        s.synchronize()
        b.set_stream(None)
    assert np.array_equal(b.get_state(), init)  # captured, not run
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(b.get_state(), o.step_philox(init, 5, 1, 0, 70))
    b.step(1)  # the host counter moved on by 70 during the capture
    assert np.array_equal(b.get_state(), o.step_philox(init, 5, 1, 0, 71))
    b.close()


@pytest.mark.parametrize("group", ["2", "4", "8"])
@pytest.mark.parametrize("name", ["bittner28", "bittner199", "syn5", "tt200"])
def test_rollout_group_mode_matches_oracle(G, oracle_mod, monkeypatch, group, name):
    """k_rollout_grp (G lanes per env, blocks of G updates resolved at once): the same states as
    the oracle for update counts that are not a multiple of G and ragged batches; tt200 (truth
    tables) ignores the knob and stays in lane mode; syn5 has long in-block dependency chains."""
    monkeypatch.setenv("PBNSIM_ROLL_GROUP", group)
    if name == "syn5":
        from gym_pbn_amd.network import PredictorNetwork, synthetic_predictor_sets

        net = PredictorNetwork.from_predictor_sets(*synthetic_predictor_sets(5, 4, seed=5), name="syn5")
    else:
        net = load_network(name)
    o = oracle_mod.Oracle(net)
    for B, T in ((1, 37), (65, 2), (1000, 61)):
        b = G.PBNBatch(net, B, seed=31, env_id_base=9)
        assert b.info()["roll_lanes"] == (1 if name == "tt200" else int(group))  # group mode really ran
        b.randomize()
        init = b.get_state()
        b.rollout(T)
        b.rollout(3)  # counters continue across calls
        assert np.array_equal(b.get_state(), o.step_philox(init, 31, 9, 0, T + 3)), (B, T)
        b.close()


@pytest.mark.parametrize("case", range(4))
def test_rollout_random_shapes_all_lane_counts(G, oracle_mod, monkeypatch, case):
    """Seeded random batch sizes and update counts: rollout with 1, 2, 4 and 8 lanes per env and
    step mode (plain and graph-replayed launches) all give the oracle's states."""
    rng = np.random.default_rng(77 + case)
    net = load_network(["bittner28", "bittner199"][case % 2])
    o = oracle_mod.Oracle(net)
    B = int(rng.integers(1, 3000))
    T = int(rng.integers(2, 200))
    ref = None
    for group in ("1", "2", "4", "8"):
        monkeypatch.setenv("PBNSIM_ROLL_GROUP", group)
        b = G.PBNBatch(net, B, seed=case, env_id_base=case * 11)
        b.randomize()
        init = b.get_state()
        if ref is None:
            ref = o.step_philox(init, case, case * 11, 0, 2 * T)
        b.rollout(T)
        b.step(T)
        assert np.array_equal(b.get_state(), ref), (group, B, T)
        b.close()


@pytest.mark.parametrize("name", ["bittner199", "bittner28"])
def test_ragged_batches_and_zero_updates(G, oracle_mod, name):
    """Batch sizes that fill no wave / workgroup / pair evenly (1, 63, 65, 1023, 1025, 4097, 70001):
    step, rollout and the R6 env step equal the oracle; zero-update calls change nothing."""
    net = load_network(name)
    o = oracle_mod.Oracle(net)
    rng = np.random.default_rng(3)
    for B in (1, 63, 65, 1023, 1025, 4097, 70001):
        b = G.PBNBatch(net, B, seed=99, env_id_base=5)
        b.randomize()
        init = b.get_state()
        b.step(0)
        b.rollout(0)
        assert np.array_equal(b.get_state(), init)
        b.step(3)
        b.rollout(5)
        assert np.array_equal(b.get_state(), o.step_philox(init, 99, 5, 0, 8)), B
        b.close()
    z = golden(f"r6_{name}.npz")
    gnet = G.Net(net)
    cfg = G.EnvConfig(gnet, cubes_to_attractors(z, net.n_nodes), horizon=4)
    cfgd = dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care,
                target_value=cfg.target_value, horizon=4, first_tested=False)
    for B in (1, 65, 1025):
        b = G.PBNBatch(gnet, B, seed=8, env_id_base=3)
        b.env_reset(cfg)
        st, ns = b.get_state(), np.zeros(B, np.int64)
        acts = rng.integers(0, net.n_nodes + 1, size=(B, 2)).astype(np.int32)
        obs, rew, flags, nup = b.env_step_multi(cfg, acts, update_cap=2048)
        ref = o.env_step_multi(cfgd, st, ns, acts, seed=8, env_base=3, call_idx=0, update_cap=2048)
        assert np.array_equal(nup, ref["n_updates"]) and np.array_equal(obs, ref["obs"]), B
        assert np.array_equal(b.get_state(), ref["state"]), B
        b.close()



def _oracle_threads():
    """OpenMP threads for whole-batch oracle checks: the box's CPU share (at most 16)."""
    import os

    return max(1, min(16, len(os.sched_getaffinity(0))))

@pytest.mark.parametrize("store_mode", ["0", "1"])
def test_store_modes_identical(G, monkeypatch, store_mode):
    monkeypatch.setenv("PBNSIM_STORE_MODE", store_mode)
    b = G.PBNBatch("bittner199", 50000, seed=5)
    b.randomize()
    s0 = b.get_state()
    b.step(10)
    r = G.PBNBatch("bittner199", 50000, seed=5)
    r.set_state(s0)
    r.rollout(10)
    assert np.array_equal(b.get_state(), r.get_state())


def test_full_size_shard_invariance_and_sampled_oracle(G, oracle_mod):
    """Bittner-200 at B=1,048,576: the two halves stepped as separate batches (global env ids)
    equal the full batch; EVERY env equals the oracle (one whole-batch orc_step_philox call, OpenMP);
    step x T == rollout(T)."""
    B, T = 1 << 20, 8
    net = load_network("bittner199")
    full = G.PBNBatch(net, B, seed=2024)
    full.randomize()
    init = full.get_state()
    full.step(T)
    got = full.get_state()
    halves = []
    for k in range(2):
        h = G.PBNBatch(net, B // 2, seed=2024, env_id_base=k * B // 2)
        h.set_state(init[k * B // 2:(k + 1) * B // 2])
        h.rollout(T)
        halves.append(h.get_state())
        h.close()
    assert np.array_equal(np.concatenate(halves), got)
    o = oracle_mod.Oracle(net)
    ref = o.step_philox(init, 2024, 0, 0, T, n_threads=_oracle_threads())
    bad = np.flatnonzero((ref != got).any(axis=1))
    assert bad.size == 0, (bad.size, bad[:8])
    # bits beyond node 198 stay clear
    assert not (got[:, 3] >> np.uint64(199 - 192)).any()


@pytest.mark.parametrize("B,base", [(1_000_003, 77), (1_000_001, 64)])
def test_large_ragged_batch_step_matches_oracle(G, oracle_mod, B, base):
    """The 1024-thread step path (image staged ahead of the state loads, clamped loads for lanes
    past B) on ragged batches of ~1M envs with an odd env base (one Philox call per env) and an even
    one (paired calls): every env equals the oracle after T steps (one whole-batch oracle call)."""
    T = 3
    net = load_network("bittner199")
    b = G.PBNBatch(net, B, seed=4242, env_id_base=base)
    b.randomize()
    init = b.get_state()
    b.step(T)
    got = b.get_state()
    b.close()
    o = oracle_mod.Oracle(net)
    ref = o.step_philox(init, 4242, base, 0, T, n_threads=_oracle_threads())
    bad = np.flatnonzero((ref != got).any(axis=1))
    assert bad.size == 0, (bad.size, bad[:8])
    assert not (got[:, 3] >> np.uint64(199 - 192)).any()


def test_max_batch_single_gpu_sampled_oracle(G, oracle_mod):
    """BASELINE config 4's whole batch (8,388,608 envs, 256 MiB of state) on one GPU: step and
    rollout equal the oracle on EVERY env (one whole-batch oracle call), bits past node 198 stay clear."""
    B, T = 1 << 23, 4
    net = load_network("bittner199")
    b = G.PBNBatch(net, B, seed=808)
    b.randomize()
    init = b.get_state()
    b.step(T)
    b.rollout(T)
    got = b.get_state()
    b.close()
    o = oracle_mod.Oracle(net)
    ref = o.step_philox(init, 808, 0, 0, 2 * T, n_threads=_oracle_threads())
    bad = np.flatnonzero((ref != got).any(axis=1))
    assert bad.size == 0, (bad.size, bad[:8])
    del ref
    assert not (got[:, 3] >> np.uint64(199 - 192)).any()


# ----------------------------------------------------------------- interventions
def test_flip_semantics(G):
    b = G.PBNBatch("bittner28", 4)
    b.set_state(np.zeros((4, 1), np.uint64))
    b.flip(np.array([[1, 1, 0], [3, 0, 3], [28, 5, 0], [-1 + 1, 0, 0]]), offset=1, dedup=True)
    bits = b.get_bits()
    assert bits[0, 0] == 1 and bits[1, 2] == 1 and bits[2, 27] == 1 and bits[2, 4] == 1 and bits[3].sum() == 0
    b.flip(np.array([[1, 1, 0], [0, 0, 0], [0, 0, 0], [0, 0, 0]]), offset=1, dedup=False)  # list input flips twice
    assert b.get_bits()[0, 0] == 1
    before = b.get_state()
    with pytest.raises(ValueError):
        b.flip(np.array([[29, 0, 0]] * 4), offset=1)  # base.py:283-284
    assert np.array_equal(b.get_state(), before)
    b.flip(np.array([[-3, 0, 0]] + [[0, 0, 0]] * 3), offset=1)  # Python negative indexing: node N-4
    assert b.get_bits()[0, 24] == 1


# ----------------------------------------------------------------- R6 env step
@pytest.mark.parametrize("name", ["bittner28", "bittner199"])
def test_env_step_multi_replay_matches_reference(G, name):
    z = golden(f"r6_{name}.npz")
    net = load_network(name)
    attractors = cubes_to_attractors(z, net.n_nodes)
    gnet = G.Net(net)
    cfg = G.EnvConfig(gnet, attractors, horizon=int(z["horizon"]))
    b = G.PBNBatch(gnet, 1)
    for r in range(len(z["seed"])):
        if z["t"][r] == 0:
            b.set_state(z["reset_state"][r][None])
            b.set_n_steps(np.zeros(1, np.int64))
        a, e = z["draw_offsets"][r], z["draw_offsets"][r + 1]
        rep = (np.array([0, e - a]), z["draws_i"][a:e], z["draws_k"][a:e])
        obs, rew, flags, nup = b.env_step_multi(cfg, z["actions"][r][None], dedup=not z["is_list"][r], replay=rep)
        assert np.array_equal(obs[0], z["obs"][r]), r
        assert np.array_equal(b.get_state()[0], z["state_after"][r]), r
        assert rew[0] == z["reward"][r] and (flags[0] & 1) == z["terminated"][r]
        assert ((flags[0] >> 1) & 1) == z["truncated"][r] and not (flags[0] & 4)
        assert nup[0] == e - a and b.get_n_steps()[0] == z["n_steps"][r]


@pytest.mark.parametrize("name,B", [("bittner28", 2048), ("bittner199", 512)])
def test_env_step_multi_philox_matches_oracle(G, oracle_mod, name, B):
    z = golden(f"r6_{name}.npz")
    net = load_network(name)
    o = oracle_mod.Oracle(net)
    cfgd = r6_config(z)
    gnet = G.Net(net)
    cfg = G.EnvConfig(gnet, cubes_to_attractors(z, net.n_nodes), horizon=cfgd["horizon"])
    b = G.PBNBatch(gnet, B, seed=31, env_id_base=1000)
    b.env_reset(cfg)
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), cfgd["reset_care"],
                                cfgd["reset_value"], seed=31, env_base=1000, reset_count=0)
    assert np.array_equal(b.get_state(), st) and np.array_equal(b.get_n_steps(), ns)
    rng = np.random.default_rng(8)
    for call in range(4):
        acts = rng.integers(0, net.n_nodes + 1, size=(B, 3)).astype(np.int32)
        acts[rng.random((B, 3)) < 0.6] = 0
        obs, rew, flags, nup = b.env_step_multi(cfg, acts, update_cap=20000)
        ref = o.env_step_multi(cfgd, st, ns, acts, seed=31, env_base=1000, call_idx=call, update_cap=20000)
        assert np.array_equal(obs, ref["obs"]) and np.array_equal(rew, ref["reward"])
        assert np.array_equal(flags, ref["flags"]) and np.array_equal(nup, ref["n_updates"])
        st, ns = ref["state"], ref["n_steps"]
        assert np.array_equal(b.get_state(), st)
    mask = (np.arange(B) % 3 == 0).astype(np.uint8)
    b.env_reset(cfg, mask)
    st, ns = o.env_reset_philox(st, ns, cfgd["reset_care"], cfgd["reset_value"], mask=mask, seed=31,
                                env_base=1000, reset_count=1)
    assert np.array_equal(b.get_state(), st) and np.array_equal(b.get_n_steps(), ns)


def test_env_step_rejects_bad_actions_without_side_effects(G):
    z = golden("r6_bittner28.npz")
    gnet = G.Net(load_network("bittner28"))
    cfg = G.EnvConfig(gnet, cubes_to_attractors(z, 28), horizon=7)
    b = G.PBNBatch(gnet, 8, seed=1)
    b.env_reset(cfg)
    before, nb = b.get_state(), b.get_n_steps()
    acts = np.zeros((8, 2), np.int32)
    acts[3, 1] = 40
    with pytest.raises(ValueError):
        b.env_step_multi(cfg, acts)
    assert np.array_equal(b.get_state(), before) and np.array_equal(b.get_n_steps(), nb)


def test_vec_env_and_single_env_adapters(G):
    from gym_pbn_amd.envs import Graph, PBNTargetMultiEnv, VecPBNTargetMultiEnv

    z = golden("r6_bittner28.npz")
    attractors = cubes_to_attractors(z, 28)
    v = VecPBNTargetMultiEnv("bittner28", attractors, 64, horizon=5, seed=3, auto_reset=True)
    obs = v.reset()
    assert obs.shape == (64, 28)
    for _ in range(6):
        obs, rew, term, trunc, info = v.step(np.zeros((64, 2), np.int32))
        assert obs.shape == (64, 28) and rew.dtype == np.int32
        assert (rew[~term] == -1).all() and (rew[term] == 999).all()
    env = PBNTargetMultiEnv("bittner28", attractors, horizon=3, seed=4)
    (s, t), info = env.reset()
    assert len(s) == 28 and info["observation_idx"] == int("".join(map(str, s)), 2)
    o, r, term, trunc, info = env.step([0, 0])
    assert r in (-2, 998) and isinstance(o, tuple)
    g = Graph("bittner28", seed=1)
    with pytest.raises(Exception):
        g.step()
    g.genRandState()
    s0 = g.getState()
    s1 = g.step()
    assert sum(a != b for a, b in zip(s0, s1)) <= 1
    with pytest.raises(ValueError):
        g.flipNode(28)


# ----------------------------------------------------------------- MT mode: reference streams on device
@pytest.mark.parametrize("walk", ["staged", "lanes"])
@pytest.mark.parametrize("name", ["bittner28", "bittner199"])
def test_mt_mode_reproduces_reference_from_seed(G, monkeypatch, name, walk):
    """random.seed(s); genRandState(); T x Graph.step() -- reproduced on the GPU from s alone, by the walk with
    LDS-staged windows (k_mt_staged, the default for these networks) and the per-lane loads (k_mt_step,
    PBNSIM_MT_LANES=1)."""
    monkeypatch.setenv("PBNSIM_MT_LANES", "1" if walk == "lanes" else "0")
    z = golden(f"r1_mt_{name}.npz")
    b = G.PBNBatch(name, len(z["seeds"]))
    b.mt_seed(z["seeds"], init_state=True)
    assert np.array_equal(b.get_state(), z["init"])
    cp = z["checkpoints"]
    for k in range(cp.shape[1]):
        b.mt_step(1000)
        assert np.array_equal(b.get_state(), cp[:, k]), k
    assert np.array_equal(b.get_state(), z["final"])


@pytest.mark.parametrize("name", ["tt200", "tt8"])
def test_mt_mode_truth_table_reproduces_reference(G, name):
    """random.seed(s); np.random.seed(s); PBN.reset(); T x PBN.step() on the GPU."""
    z = golden(f"r4_{name}.npz")
    b = G.PBNBatch(name, len(z["seeds"]))
    b.mt_seed(z["seeds"], init_state=True)
    assert np.array_equal(b.get_state(), z["init"])
    T = z["states"].shape[1]
    b.mt_step(7)
    assert np.array_equal(b.get_state(), z["states"][:, 6])
    b.mt_step(T - 7)
    assert np.array_equal(b.get_state(), z["states"][:, -1])


@pytest.mark.parametrize("walk", ["staged", "lanes"])
def test_mt_mode_many_seeds_vs_oracle(G, oracle_mod, monkeypatch, walk):
    """65,536 envs with spread seeds (crossing many MT twists, rows running out in different iterations):
    EVERY env vs the oracle's CPython MT (OpenMP over the envs), both walks; T = 700 in launches of 1, 2, 97
    and 600 updates (launches end mid-row, mid-window and mid-chunk)."""
    monkeypatch.setenv("PBNSIM_MT_LANES", "1" if walk == "lanes" else "0")
    net = load_network("bittner199")
    B, T = 65536, 700
    seeds = np.arange(B, dtype=np.uint64) * np.uint64(2654435761) + np.uint64(3)
    b = G.PBNBatch(net, B)
    b.mt_seed(seeds, init_state=True)
    for n in (1, 2, 97, 600):
        b.mt_step(n)
    got = b.get_state()
    b.close()
    o = oracle_mod.Oracle(net)
    assert np.array_equal(got, o.run_mt(seeds, T, n_threads=16))
    with pytest.raises(ValueError):
        G.PBNBatch("tt8", 2).mt_seed(np.array([1, 2**33], dtype=np.uint64))


@pytest.mark.parametrize("walk", ["staged", "lanes"])
def test_mt_mode_bench_workload_vs_oracle(G, oracle_mod, monkeypatch, walk):
    """bench.py's MT workload itself (mt_supplement: Bittner-199, 1,048,576 envs seeded 12345 + id, the
    state from genRandState, T = 256 updates per pbn_mt_step launch): two launches, every env vs the oracle's
    run_mt from the seeds alone (16 threads); both walks."""
    monkeypatch.setenv("PBNSIM_MT_LANES", "1" if walk == "lanes" else "0")
    net = load_network("bittner199")
    B, T = 1 << 20, 256
    seeds = np.arange(B, dtype=np.uint64) + np.uint64(12345)
    b = G.PBNBatch(net, B, seed=1)
    b.mt_seed(seeds, init_state=True)
    b.mt_step(T)
    b.mt_step(T)
    got = b.get_state()
    b.close()
    assert np.array_equal(got, oracle_mod.Oracle(net).run_mt(seeds, 2 * T, n_threads=16))


# ----------------------------------------------------------------- config 5: device trajectory chunks
@pytest.mark.parametrize("net_name,fused,group", [("bittner28", True, "1"), ("bittner28", False, "1"),
                                                   ("bittner28", True, "4"), ("bittner199", True, "1"),
                                                   ("bittner199", True, "8"), ("bittner199", False, "2")])
def test_trajectory_collector_matches_host_api(G, monkeypatch, net_name, fused, group):
    """rollout.TrajectoryCollector writes step t of a chunk into slice t; same results as T calls
    of the host API -- with the chunk as one fused launch (each env walks its T steps alone) or
    one launch per step, in lane mode and in group mode."""
    import torch

    from gym_pbn_amd.rollout import TrajectoryCollector

    monkeypatch.setenv("PBNSIM_ENV_GROUP", group)
    N = 28 if net_name == "bittner28" else 199
    z = golden(f"r6_{net_name}.npz")
    net = G.Net(load_network(net_name))
    cfg = G.EnvConfig(net, cubes_to_attractors(z, N), horizon=6)
    B, T, A = 3000, 6, 3
    rng = np.random.default_rng(5)
    acts = rng.integers(0, N + 1, size=(T, B, A)).astype(np.int32)
    acts[rng.random(acts.shape) < 0.6] = 0
    dev = torch.device("cuda", 0)
    b1 = G.PBNBatch(net, B, seed=77, env_id_base=123)
    col = TrajectoryCollector(b1, cfg, T, A, dev, update_cap=1 << 14, fused=fused)
    buf, gathered = col.step_chunk(torch.from_numpy(acts).to(dev))
    col.finish()
    assert gathered is None
    assert b1.info()["env_lanes"] == int(group)
    monkeypatch.setenv("PBNSIM_ENV_GROUP", "1")  # read at batch creation
    b2 = G.PBNBatch(net, B, seed=77, env_id_base=123)
    b2.env_reset(cfg)
    for t in range(T):
        obs, rew, flags, nup = b2.env_step_multi(cfg, acts[t], update_cap=1 << 14)
        assert np.array_equal(buf["obs"][t].cpu().numpy().view(np.uint64), obs), t
        assert np.array_equal(buf["reward"][t].cpu().numpy(), rew), t
        assert np.array_equal(buf["flags"][t].cpu().numpy(), flags), t
        assert np.array_equal(buf["n_updates"][t].cpu().numpy().view(np.uint32), nup), t
    assert (flags & 2).all()  # truncated at the horizon == T
    assert np.array_equal(b1.get_state(), b2.get_state())
    assert np.array_equal(b1.get_n_steps(), b2.get_n_steps())
    assert b1.info()["env_call_count"] == b2.info()["env_call_count"] == T


@pytest.mark.parametrize("group", ["1", "4"])
def test_env_rollout_skips_invalid_action_steps(G, monkeypatch, group):
    """An out-of-range action (the reference's flipNode ValueError, base.py:283-284) skips that env
    step for that env in the fused launch exactly as a per-step device call does: outputs left as
    they were, state and step count untouched, the error flag raised."""
    import torch

    from gym_pbn_amd import _lib as L

    monkeypatch.setenv("PBNSIM_ENV_GROUP", group)
    z = golden("r6_bittner199.npz")
    net = G.Net(load_network("bittner199"))
    cfg = G.EnvConfig(net, cubes_to_attractors(z, 199), horizon=100)
    B, T, A, W = 640, 5, 2, net.n_words
    rng = np.random.default_rng(9)
    acts = rng.integers(0, 200, size=(T, B, A)).astype(np.int32)
    acts[rng.random(acts.shape) < 0.5] = 0
    acts[2, 7, 1] = 250   # invalid at step 2 for env 7
    acts[0, 100, 0] = -300  # invalid at step 0 for env 100
    dev = torch.device("cuda", 0)
    d_acts = torch.from_numpy(acts).to(dev)

    def out():
        return (torch.full((T, B, W), -1, dtype=torch.int64, device=dev),
                torch.full((T, B), -7, dtype=torch.int32, device=dev),
                torch.full((T, B), 0xEE, dtype=torch.uint8, device=dev),
                torch.full((T, B), -1, dtype=torch.int32, device=dev))

    res = []
    for fused in (True, False):
        b = G.PBNBatch(net, B, seed=3, env_id_base=40)
        b.env_reset(cfg)
        o, r, f, n = out()
        if fused:
            b.env_rollout_multi_device(cfg, T, d_acts.data_ptr(), A, o.data_ptr(), r.data_ptr(), f.data_ptr(),
                                       n.data_ptr(), update_cap=4096)
        else:
            for t in range(T):
                b.env_step_multi_device(cfg, d_acts[t].data_ptr(), A, o[t].data_ptr(), r[t].data_ptr(),
                                        f[t].data_ptr(), n[t].data_ptr(), update_cap=4096)
        b.sync()
        res.append((o.cpu().numpy(), r.cpu().numpy(), f.cpu().numpy(), n.cpu().numpy(), b.get_state(),
                    b.get_n_steps()))
    for x, y in zip(*res):
        assert np.array_equal(x, y)
    o, r, f, n, st, ns = res[0]
    assert r[2, 7] == -7 and f[0, 100] == 0xEE and (o[0, 100] == -1).all()  # skipped steps left untouched
    assert ns[7] == T - 1 and ns[100] == T - 1 and ns[0] == T


# ----------------------------------------------------------------- env kernel variants vs the oracle
def _random_cubes(rng, N, H, n_care):
    cubes = []
    for _ in range(H):
        c = ["*"] * N
        for j in rng.choice(N, size=n_care, replace=False):
            c[int(j)] = int(rng.integers(0, 2))
        cubes.append(tuple(c))
    return cubes


@pytest.mark.parametrize("case", ["b28_gen_cap", "b28_h8_gen", "b199_h6_gen_first_tested", "b28_h12_general",
                                  "b199_nogen", "tt200_fast", "syn500_gen",
                                  "syn300_wide_cube", "b28_first_tested", "b28_h12_first_tested",
                                  "tt200_first_tested", "b199_grp2", "b199_grp4", "b199_grp8", "b28_grp4_cap",
                                  "b28_grp8_first_tested", "b28_grp2_h8", "b199_grp4_long",
                                  "b28_gen_cap41", "b199_gen_long", "b199_gen_long_first_tested",
                                  "b28_gen_cap41_tail32", "b199_gen_long_tail32", "b199_gen_long_tail16",
                                  "b199_gen_long_tail8", "b199_gen_long_tail1", "b199_gen_long_first_tested_tail32",
                                  "b28_first_tested_tail32", "b28_gen_cap41_tail3", "b199_gen_long_tail0",
                                  "b199_gen_long_lanes16", "b199_gen_long_lanes1", "b28_gen_cap41_lanes4",
                                  "b199_gen_long_first_tested_lanes8"])
def test_env_kernel_variants_match_oracle(G, oracle_mod, monkeypatch, case):
    """Every k_env variant (cooperative draw generation, byte counters without it, general
    cube matching, truth-table kind, W = 8) against the oracle's R6 step, incl. capped envs and
    long until-attractor loops (thousands of updates per env step, odd caps). ``_tailK``: the
    cooperative-draw kernel's tail mode (a wave whose queue ran dry resolves its envs one at a time,
    64 updates per block) from K live envs per wave (32: early, many envs queued behind the one
    resolved; 1: the last env only; 0: never; the default is ENV_TAIL_DEFAULT)."""
    from gym_pbn_amd.network import PredictorNetwork, synthetic_predictor_sets

    if "_tail" in case:  # the same inputs as the base case, another tail-mode threshold
        monkeypatch.setenv("PBNSIM_ENV_TAIL", case.split("_tail")[1])
        case = case.split("_tail")[0]
    # lane mode proper (every lane takes envs) unless the case names K lanes per wave taking envs
    # (tail mode from the first env; batches this small default to K = 1)
    monkeypatch.setenv("PBNSIM_ENV_LANES", "64")
    if "_lanes" in case:
        monkeypatch.setenv("PBNSIM_ENV_LANES", case.split("_lanes")[1])
        case = case.split("_lanes")[0]
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    cap, A, B = 3000, 3, 1024
    first = case.endswith("first_tested")  # PBNTargetEnv.step(force=False) semantics
    # k_env_grp (G lanes per env, blocks of G updates resolved in parallel) or lane mode (1)
    monkeypatch.setenv("PBNSIM_ENV_GROUP", case.split("_grp")[1][0] if "_grp" in case else "1")
    if case.startswith("b199_grp") or case.startswith("b199_gen_long"):
        net = load_network("bittner199")
    elif case.startswith("b28"):
        net = load_network("bittner28")
    elif case == "b199_h6_gen_first_tested":
        net = load_network("bittner199")
    elif case == "b199_nogen":
        net = load_network("bittner199")
        monkeypatch.setenv("PBNSIM_ENV_NO_GEN", "1")
    elif case.startswith("tt200"):
        net = load_network("tt200")
    else:
        n = 500 if case == "syn500_gen" else 300
        net = PredictorNetwork.from_predictor_sets(*synthetic_predictor_sets(n, 4, seed=n), name=f"syn{n}")
    N = net.n_nodes
    if case in ("b28_gen_cap", "b28_grp4_cap", "b28_gen_cap41"):
        cap = 41 if ("grp" in case or "cap41" in case) else 40  # not a multiple of the group size
        attractors = [_random_cubes(rng, N, 2, 5), _random_cubes(rng, N, 2, 5)]
    elif case.startswith("b199_gen_long"):  # long loops: thousands of updates per env step
        cap = 2001
        attractors = [_random_cubes(rng, N, 2, 12), _random_cubes(rng, N, 2, 4)]
    elif case == "b199_grp4_long":  # long until-attractor loops, many capped envs
        cap = 2001
        attractors = [_random_cubes(rng, N, 4, 12), _random_cubes(rng, N, 2, 4)]
    elif case in ("b28_grp2_h8", "b28_h8_gen"):  # 8 cubes: the most the byte counters hold
        attractors = [_random_cubes(rng, N, 4, 4), _random_cubes(rng, N, 4, 4)]
    elif case == "b199_h6_gen_first_tested":  # 5..8 cubes: both packed counter words
        attractors = [_random_cubes(rng, N, 3, 3), _random_cubes(rng, N, 3, 3)]
    elif case.startswith("b28_h12"):
        attractors = [_random_cubes(rng, N, 6, 4), _random_cubes(rng, N, 6, 4)]
    elif case == "syn300_wide_cube":  # one cube caring about 260 > 255 nodes: general matching
        attractors = [_random_cubes(rng, N, 1, 260) + _random_cubes(rng, N, 2, 3), _random_cubes(rng, N, 1, 3)]
    else:
        attractors = [_random_cubes(rng, N, 2, 4), _random_cubes(rng, N, 2, 4)]
    gnet = G.Net(net)
    cfg = G.EnvConfig(gnet, attractors, horizon=3, first_update_tested=first)
    o = oracle_mod.Oracle(net)
    cfgd = dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care,
                target_value=cfg.target_value, horizon=3, first_tested=first)
    b = G.PBNBatch(gnet, B, seed=5, env_id_base=77)
    b.randomize()
    st, ns = b.get_state(), np.zeros(B, np.int64)
    b.set_n_steps(ns)
    for call in range(3):
        acts = rng.integers(0, N + 1, size=(B, A)).astype(np.int32)
        acts[rng.random((B, A)) < 0.5] = 0
        obs, rew, flags, nup = b.env_step_multi(cfg, acts, update_cap=cap)
        ref = o.env_step_multi(cfgd, st, ns, acts, seed=5, env_base=77, call_idx=call, update_cap=cap)
        assert np.array_equal(nup, ref["n_updates"]), case
        assert np.array_equal(obs, ref["obs"]) and np.array_equal(rew, ref["reward"]), case
        assert np.array_equal(flags, ref["flags"]), case
        st, ns = ref["state"], ref["n_steps"]
        assert np.array_equal(b.get_state(), st), case
        if "_grp" in case:
            assert b.info()["env_lanes"] == int(case.split("_grp")[1][0])  # group mode really ran
        if case in ("b28_gen_cap", "b28_first_tested", "b28_gen_cap41") or case.startswith("b199_gen_long"):
            assert b.info()["env_kernel"] == 4  # wave-generated draws, one counter word (<= 4 cubes)
            assert b.info()["env_lane_limit"] == int(os.environ["PBNSIM_ENV_LANES"])
        if case in ("b28_h8_gen", "b199_h6_gen_first_tested"):
            assert b.info()["env_kernel"] == 2  # wave-generated draws, two counter words
    if case in ("b28_gen_cap", "b28_grp4_cap", "b199_grp4_long", "b28_gen_cap41") or case.startswith("b199_gen_long"):
        assert (flags & 4).any() and not (flags & 4).all()  # some envs capped, some reached an attractor
    assert (nup > 1).any()


def test_torch_vec_env_matches_host_vec_env(G):
    """Device-resident env (torch tensors in/out, batch on torch's stream) == the host API env,
    step for step, including on-device auto-reset of the envs that ended."""
    import torch

    from gym_pbn_amd.envs import VecPBNTargetMultiEnv
    from gym_pbn_amd.torch_env import TorchVecPBNTargetMultiEnv

    z = golden("r6_bittner28.npz")
    att = cubes_to_attractors(z, 28)
    B, A = 777, 2
    tv = TorchVecPBNTargetMultiEnv("bittner28", att, B, horizon=3, seed=21, update_cap=4096, auto_reset=True)
    hv = VecPBNTargetMultiEnv(load_network("bittner28"), att, B, horizon=3, seed=21, update_cap=4096, auto_reset=True)
    assert tv.observation_space.shape == (28,)
    o_t = tv.reset()
    o_h = hv.reset()
    assert o_t.is_cuda and o_t.dtype == torch.uint8 and np.array_equal(o_t.cpu().numpy(), o_h)
    rng = np.random.default_rng(4)
    for t in range(8):
        a = rng.integers(0, 29, size=(B, A)).astype(np.int32)
        a[rng.random(a.shape) < 0.6] = 0
        ot, rt, tt, trt, it = tv.step(torch.from_numpy(a).cuda())
        oh, rh, th, trh, ih = hv.step(a)
        assert np.array_equal(ot.cpu().numpy(), oh), t
        assert np.array_equal(rt.cpu().numpy(), rh) and np.array_equal(tt.cpu().numpy(), th), t
        assert np.array_equal(trt.cpu().numpy(), trh), t
        assert np.array_equal(it["n_updates"].cpu().numpy().view(np.uint32), ih["n_updates"]), t
    assert trh.any()  # horizon 3: truncations (and auto-resets) happened
    assert np.array_equal(tv.batch.get_state(), hv.batch.get_state())
    tv.close()


def test_sb3_vec_env_adapter(G):
    """SB3 VecEnv conventions over the batched multi-flip env: dones = terminated | truncated,
    ended envs reset at once (obs = their first observation of the next episode), the last
    observation in infos["terminal_observation"], truncations marked "TimeLimit.truncated"."""
    from gym_pbn_amd.envs import VecPBNTargetMultiEnv
    from gym_pbn_amd.sb3 import PBNVecEnv

    z = golden("r6_bittner28.npz")
    att = cubes_to_attractors(z, 28)
    B = 300
    ve = PBNVecEnv(VecPBNTargetMultiEnv(load_network("bittner28"), att, B, horizon=4, seed=2, update_cap=4096),
                   n_action_slots=2)
    twin = VecPBNTargetMultiEnv(load_network("bittner28"), att, B, horizon=4, seed=2, update_cap=4096)
    assert ve.num_envs == B and ve.action_space.shape == (2,) and ve.observation_space.shape == (28,)
    obs = ve.reset()
    assert np.array_equal(obs, twin.reset())
    rng = np.random.default_rng(8)
    n_done = 0
    for t in range(10):
        a = rng.integers(0, 29, size=(B, 2))
        a[rng.random(a.shape) < 0.7] = 0
        obs, rew, done, infos = ve.step(a)
        o, r, term, trunc, _ = twin.step(a)
        assert np.array_equal(done, term | trunc) and np.allclose(rew, r) and rew.dtype == np.float32
        for i in np.nonzero(done)[0]:
            assert np.array_equal(infos[i]["terminal_observation"], o[i])
            assert infos[i]["TimeLimit.truncated"] == bool(trunc[i] and not term[i])
        if done.any():
            fresh = twin.reset(done)
            o = o.copy()
            o[done] = fresh[done]
            n_done += int(done.sum())
        assert np.array_equal(obs, o), t
    assert n_done > B  # the horizon of 4 ends every episode at least twice
    ve.close()
