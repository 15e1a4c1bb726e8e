"""The oracle itself, pinned against the reference (CPU only).

Every expectation here comes from the reference or its RNGs: golden vectors
captured by tests/golden/make_golden.py from gym_PBN's own Graph.step /
PBN.step / PBNTargetMultiEnv.step, CPython's ``random`` and numpy's legacy
``RandomState`` (the generators base.py:7 and common/node.py:2 draw from), and
Random123's published Philox4x32-10 known-answer vectors.
"""

import random

import numpy as np
import pytest

from conftest import golden, r6_config
from gym_pbn_amd.network import load_network


@pytest.mark.parametrize("seed", [0, 1, 42, 12345, 2**32 + 7, 2**63 + 11])
def test_mt_matches_cpython(oracle_mod, seed):
    O = oracle_mod
    m, r = O.mt_python(seed), random.Random(seed)
    assert [O.mt_next(m) for _ in range(1500)] == [r.getrandbits(32) for _ in range(1500)]
    m, r = O.mt_python(seed), random.Random(seed)
    for n in (1, 2, 28, 199, 200, 1000):
        assert [O.mt_randbelow(m, n) for _ in range(300)] == [r.randint(0, n - 1) for _ in range(300)]
    assert [O.mt_k53(m) for _ in range(300)] == [int(r.random() * 2**53) for _ in range(300)]


@pytest.mark.parametrize("seed", [0, 1, 7, 2**32 - 1])
def test_mt_matches_numpy_legacy(oracle_mod, seed):
    O = oracle_mod
    m, rs = O.mt_numpy(seed), np.random.RandomState(seed)
    assert [O.mt_k53(m) for _ in range(2000)] == [int(rs.uniform(0, 1) * 2**53) for _ in range(2000)]


def test_philox_kat(oracle_mod):
    # Random123 kat_vectors, philox4x32 10 rounds
    f = oracle_mod.philox4x32_10
    assert f([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert f([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert f([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


@pytest.mark.parametrize("name", ["bittner28", "bittner199", "bittner70"])
def test_r1_replay_matches_reference(oracle_mod, name):
    z = golden(f"r1_{name}.npz")
    o = oracle_mod.Oracle(load_network(name))
    for si in range(len(z["seeds"])):
        st = z["init"][si][None]
        for t in range(z["states"].shape[1]):
            st = o.step_replay(st, z["node_idx"][si][t:t + 1], z["k53"][si][t:t + 1])
            assert np.array_equal(st[0], z["states"][si][t]), (si, t)


@pytest.mark.parametrize("name", ["tt200", "tt8"])
def test_r4_replay_matches_reference(oracle_mod, name):
    z = golden(f"r4_{name}.npz")
    o = oracle_mod.Oracle(load_network(name))
    for si in range(len(z["seeds"])):
        st = z["init"][si][None]
        for t in range(z["states"].shape[1]):
            st = o.step_replay(st, z["node_idx"][si][t:t + 1], z["k53"][si][t:t + 1])
            assert np.array_equal(st[0], z["states"][si][t]), (si, t)


@pytest.mark.parametrize("name", ["bittner28", "bittner199"])
def test_r1_mt_seed_only_matches_reference(oracle_mod, name):
    """random.seed(s); genRandState(); T x Graph.step() reproduced from the seed alone."""
    z = golden(f"r1_mt_{name}.npz")
    o = oracle_mod.Oracle(load_network(name))
    assert np.array_equal(o.run_mt(z["seeds"], 0), z["init"])
    assert np.array_equal(o.run_mt(z["seeds"], int(z["T"])), z["final"])
    cp = z["checkpoints"]
    st = o.run_mt(z["seeds"], 0)
    for k in range(cp.shape[1]):
        st = o.run_mt(z["seeds"], 1000 * (k + 1))
        assert np.array_equal(st, cp[:, k])


@pytest.mark.parametrize("name", ["tt200", "tt8"])
def test_r4_mt_seed_only_matches_reference(oracle_mod, name):
    z = golden(f"r4_{name}.npz")
    o = oracle_mod.Oracle(load_network(name))
    assert np.array_equal(o.run_mt(z["seeds"], 0), z["init"])
    assert np.array_equal(o.run_mt(z["seeds"], z["states"].shape[1]), z["states"][:, -1])


@pytest.mark.parametrize("name", ["bittner28", "bittner199"])
def test_r6_replay_matches_reference(oracle_mod, name):
    z = golden(f"r6_{name}.npz")
    o = oracle_mod.Oracle(load_network(name))
    cfg = r6_config(z)
    st = ns = None
    for r in range(len(z["seed"])):
        if z["t"][r] == 0:
            st, ns = z["reset_state"][r][None], np.zeros(1, np.int64)
        a, b = z["draw_offsets"][r], z["draw_offsets"][r + 1]
        rep = (np.array([0, b - a]), z["draws_i"][a:b], z["draws_k"][a:b])
        out = o.env_step_multi(cfg, st, ns, z["actions"][r][None], dedup=not z["is_list"][r], replay=rep)
        assert np.array_equal(out["obs"][0], z["obs"][r])
        assert np.array_equal(out["state"][0], z["state_after"][r])
        assert out["reward"][0] == z["reward"][r]
        assert (out["flags"][0] & 1) == z["terminated"][r]
        assert ((out["flags"][0] >> 1) & 1) == z["truncated"][r]
        assert out["n_updates"][0] == b - a and not (out["flags"][0] & 4)
        assert out["n_steps"][0] == z["n_steps"][r]
        st, ns = out["state"], out["n_steps"]


def test_r6_fixture_covers_quirks():
    """The fixtures exercise Q6 (obs != graph state), Q8 (list vs tensor), truncation and termination."""
    z = golden("r6_bittner28.npz")
    assert z["terminated"].any() and z["truncated"].any() and z["is_list"].any()
    assert (z["obs"] != z["state_after"]).any(axis=1).any()  # discarded first update (Q6)
    assert (np.diff(z["draw_offsets"]) == 1).any()


def test_philox_step_is_batch_and_shard_invariant(oracle_mod):
    """Philox counters are keyed by global env id: a shard reproduces its slice of the full batch."""
    o = oracle_mod.Oracle(load_network("bittner199"))
    full = o.init_philox(1024, seed=9)
    out = o.step_philox(full, seed=9, env_base=0, update_base=0, T=50)
    part = o.step_philox(full[512:], seed=9, env_base=512, update_base=0, T=50)
    assert np.array_equal(out[512:], part)
    two = o.step_philox(o.step_philox(full, 9, 0, 0, 20), 9, 0, 20, 30)
    assert np.array_equal(two, out)


def test_philox_transition_statistics(oracle_mod):
    """Philox mode samples the reference's transition law: P(Y=1|x) = sum of COD masses voting 1."""
    net = load_network("bittner28")
    o = oracle_mod.Oracle(net)
    B = 20000
    rng = np.random.default_rng(3)
    from gym_pbn_amd.batch import pack_bits, unpack_bits

    x = rng.integers(0, 2, net.n_nodes)
    st = np.repeat(pack_bits(x)[None], B, axis=0)
    out = unpack_bits(o.step_philox(st, seed=77, env_base=0, update_base=0, T=1), net.n_nodes)
    changed_node = np.argmax(out != x, axis=1)
    # node choice ~ uniform; next value of a node given x ~ Bernoulli(update_probability)
    for i in range(net.n_nodes):
        p = net.update_probability(x, i)
        # envs whose update hit node i: only those with a visible change are identifiable;
        # check the flip rate against p (x_i=0) or 1-p (x_i=1) over all envs at 1/N
        flips = np.sum((out[:, i] != x[i]))
        expect = B / net.n_nodes * (p if x[i] == 0 else 1 - p)
        assert abs(flips - expect) <= 5 * np.sqrt(expect + 1) + 2, (i, flips, expect)
    assert changed_node.shape == (B,)


@pytest.mark.parametrize("name", ["bittner199", "tt200"])
def test_forced_step_with_the_drawn_nodes_is_the_philox_step(oracle_mod, name):
    """``orc_step_forced`` (Graph.step(i=k)) fed the nodes the Philox step would draw (``mulhi(w, N)`` /
    ``1 + mulhi(w, N - 1)`` of the node word) reproduces ``orc_step_philox``: the choice word is the same."""
    net = load_network(name)
    o = oracle_mod.Oracle(net)
    B, T, seed, base = 257, 6, 31, 1001
    st = o.init_philox(B, seed=seed, env_base=base)
    ni = np.zeros((T, B), np.uint32)
    for t in range(T):
        for e in range(B):
            g = base + e
            w = oracle_mod.philox4x32_10([t, 0, (g >> 1) & 0xFFFFFFFF, ((g >> 1) >> 32) | (1 << 24)],
                                         [seed & 0xFFFFFFFF, seed >> 32])
            wn = w[2 * (g & 1)]
            ni[t, e] = (wn * net.n_nodes) >> 32 if net.kind == 1 else 1 + ((wn * (net.n_nodes - 1)) >> 32)
    assert np.array_equal(o.step_forced(st, ni, seed, base, 0), o.step_philox(st, seed, base, 0, T))
    # another node sequence gives another trajectory
    assert not np.array_equal(o.step_forced(st, (ni + 1) % net.n_nodes | (net.kind == 2), seed, base, 0),
                              o.step_philox(st, seed, base, 0, T))


def test_env_step_multi_threads_do_not_change_results(oracle_mod):
    """The OpenMP env loop of ``orc_env_step_multi`` gives the single-threaded results."""
    net = load_network("bittner28")
    z = golden("r6_bittner28.npz")
    cfg = r6_config(z)
    o = oracle_mod.Oracle(net)
    B = 3000
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.zeros(B, np.int64), cfg["reset_care"],
                                cfg["reset_value"], seed=4, env_base=11)
    rng = np.random.default_rng(4)
    acts = rng.integers(0, net.n_nodes + 1, size=(B, 2)).astype(np.int32)
    r1 = o.env_step_multi(cfg, st, ns, acts, seed=4, env_base=11, update_cap=4096, n_threads=1)
    r4 = o.env_step_multi(cfg, st, ns, acts, seed=4, env_base=11, update_cap=4096, n_threads=4)
    for k in r1:
        assert np.array_equal(r1[k], r4[k]), k
