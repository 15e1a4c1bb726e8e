"""SSD histogram (utils/eval.py:20-103): flip process statistics (CPU) and device parity (GPU)."""

import numpy as np
import pytest

from gym_pbn_amd.network import load_network


def _gap_positions(u_stream, T, N):
    """The kernel/oracle flip procedure: successive gaps = #{k>=1 : u < T_k}."""
    out, pos, first = [], 0, True
    for u in u_stream:
        gap = int(np.searchsorted(-T.astype(np.int64), -int(u), side="right"))  # #{k : T_k > u}
        pos = gap if first else pos + 1 + gap
        first = False
        if pos >= N:
            return out
        out.append(pos)
    raise AssertionError("stream exhausted")


def test_flip_gap_table_is_bernoulli_process():
    from gym_pbn_amd.batch import flip_gap_table

    N, p, R = 40, 0.05, 40000
    T = flip_gap_table(N, p)
    assert T.shape == (N,) and np.all(np.diff(T.astype(np.int64)) <= 0)
    rng = np.random.default_rng(0)
    counts = np.zeros(N)
    pair = 0
    for _ in range(R):
        pos = _gap_positions(rng.integers(0, 2**32, size=64, dtype=np.uint64), T, N)
        counts[pos] += 1
        pair += (3 in pos) and (17 in pos)
    # each node flips with probability p, independently
    assert np.all(np.abs(counts / R - p) < 5 * np.sqrt(p * (1 - p) / R))
    assert abs(pair / R - p * p) < 5 * np.sqrt(p * p / R)
    assert flip_gap_table(N, 0.0) is None
    assert np.all(flip_gap_table(N, 1.0) == 0)


GPU_CASES = [("bittner28", [0, 1, 2, 3, 6, 7, 9], 3000, 0.01), ("bittner199", [0, 1, 2, 3, 4, 5, 6], 2000, 0.01),
             ("tt200", [5, 50, 150], 1500, 0.02), ("bittner70", [1, 2], 1000, 0.0),
             ("bittner199", [3, 9], 1000, 0.09),  # ~18 flips per iteration: past the per-iteration buffer
             ("syn5", [0, 2, 4], 700, 0.05),  # 5 nodes: long in-chunk dependency chains (wave mode rounds)
             ("syn500", [7, 300, 499], 600, 0.01),  # W = 8
             ("tt8", [1, 3, 7], 900, 0.05),  # 8 nodes, 3 inputs each
             ("ttk7_40", [0, 5, 39], 700, 0.02),  # 7 inputs per node: past the chunk DAG's 6 (serial apply)
             ("bittner199", list(range(0, 120, 10)), 650, 0.02),  # 12 targets: the most the host takes
             ("bittner28", [4, 5], 10, 0.05)]  # fewer iterations than one chunk


def _net(name):
    if name.startswith("ttk"):  # ttk<k>_<n>: synthetic truth-table PBN
        from gym_pbn_amd.network import TruthTableNetwork, synthetic_truth_table_pbn

        k, n = (int(v) for v in name[3:].split("_"))
        return TruthTableNetwork.from_pbn_data(synthetic_truth_table_pbn(n, k, seed=n), name=name)
    if name.startswith("syn"):
        from gym_pbn_amd.network import PredictorNetwork, synthetic_predictor_sets

        n = int(name[3:])
        return PredictorNetwork.from_predictor_sets(*synthetic_predictor_sets(n, 4, seed=n), name=name)
    return load_network(name)


@pytest.mark.gpu
# one lane per env / one wave per env (chunk resolved in parallel) / four waves per env (chunks
# prepared in parallel, resolved in order) / one wave per env, serial apply
@pytest.mark.parametrize("mode", ["lane", "wave", "shared", "shared8", "wave_serial"])
@pytest.mark.parametrize("name,targets,iters,p", GPU_CASES)
def test_ssd_matches_oracle(oracle_mod, monkeypatch, mode, name, targets, iters, p):
    from gym_pbn_amd.batch import PBNBatch, flip_gap_table

    monkeypatch.setenv("PBNSIM_SSD_WAVE", "0" if mode == "lane" else "1")
    monkeypatch.setenv("PBNSIM_SSD_SERIAL", "1" if mode == "wave_serial" else "0")
    monkeypatch.setenv("PBNSIM_SSD_SHARED", {"shared": "4", "shared8": "8"}.get(mode, "0"))
    net = _net(name)
    B = 600
    b = PBNBatch(net, B, seed=17, env_id_base=5)
    b.randomize()
    s0 = b.get_state()
    h1 = b.ssd_counts(targets, iters, p)
    h2 = b.ssd_counts(targets, iters // 2, p)  # continues the iteration counter
    o = oracle_mod.Oracle(net)
    gap = flip_gap_table(net.n_nodes, p)
    st, r1 = oracle_mod.ssd_philox(o, s0, targets, gap, 17, 5, 0, iters)
    st, r2 = oracle_mod.ssd_philox(o, st, targets, gap, 17, 5, iters, iters // 2)
    assert np.array_equal(h1, r1) and np.array_equal(h2, r2)
    assert np.array_equal(b.get_state(), st)
    assert int(h1.sum()) == B * iters


@pytest.mark.gpu
def test_compute_ssd_hist_normalised():
    from gym_pbn_amd.eval import compute_ssd_hist

    df = compute_ssd_hist("bittner28", [0, 1, 2, 3, 6, 7, 9], iters=120_000, resets=300, seed=3)
    assert list(df.index[:2]) == ["0000000", "0000001"] and len(df) == 128
    assert abs(df["Value"].sum() - 1.0) < 1e-9


class _RulePolicy:
    """A deterministic stand-in agent: flip node 3 (action 4) when node 0 is set, else nothing;
    returns (actions, None) like a Stable-Baselines model."""

    def __init__(self):
        self.calls = 0

    def predict(self, obs, target, deterministic=True):
        assert deterministic and obs.shape == target.shape
        self.calls += 1
        return np.where(obs[:, 0] == 1, 4, 0), None


@pytest.mark.gpu
def test_controlled_ssd_matches_stepwise_oracle(oracle_mod):
    """Model-in-the-loop SSD (eval.py:96-101): bucket, batched predict, flip action-1, one R1
    update -- replayed with the oracle's Philox step and numpy flips."""
    from gym_pbn_amd.batch import PBNBatch
    from gym_pbn_amd.eval import compute_ssd_hist, eval_increase, ssd_counts_controlled

    net = load_network("bittner28")
    targets, B, iters = [0, 1, 2, 3, 6, 7, 9], 64, 40
    b = PBNBatch(net, B, seed=11)
    b.randomize()
    s0 = b.get_state()
    pol = _RulePolicy()
    got = ssd_counts_controlled(net, targets, iters, B, pol, seed=11, initial_states=s0)
    assert pol.calls == iters
    o = oracle_mod.Oracle(net)
    st, want = s0.copy(), np.zeros(1 << len(targets), np.uint64)
    for u in range(iters):
        bits = ((st[:, :1] >> np.arange(28, dtype=np.uint64)) & np.uint64(1)).astype(np.int64)
        np.add.at(want, bits[:, targets] @ (1 << np.arange(len(targets) - 1, -1, -1)), 1)
        st[bits[:, 0] == 1, 0] ^= np.uint64(1 << 3)  # action 4 flips node 3
        st = o.step_philox(st, 11, 0, u, 1)
    assert np.array_equal(got, want)
    df = compute_ssd_hist(net, targets, iters=iters * B, resets=B, seed=11, model=_RulePolicy())
    assert abs(df["Value"].sum() - 1.0) < 1e-9
    inc = eval_increase(net, targets, _RulePolicy(), [(0,) * 7, (1,) * 7], iters=iters * B, resets=B, seed=11)
    assert np.isfinite(inc)


@pytest.mark.gpu
def test_controlled_ssd_device_policy_matches_host_model():
    """The device-resident controlled SSD (torch policy on the GPU, pbn_flip_device) gives the
    same counts as the host path with an SB3-style model.predict computing the same actions;
    an out-of-range device action raises ValueError and leaves its row untouched."""
    import torch

    from gym_pbn_amd.batch import PBNBatch
    from gym_pbn_amd.eval import ssd_counts_controlled, ssd_counts_controlled_device

    net = load_network("bittner28")
    N = net.n_nodes

    class Model:
        def predict(self, obs, target, deterministic=True):
            return (obs[:, :6].astype(np.int64) * np.arange(1, 7)).sum(1) % (N + 1), None

    def policy(obs):
        return (obs[:, :6].long() * torch.arange(1, 7, device=obs.device)).sum(1) % (N + 1)

    targets = [0, 1, 2, 3, 6, 7, 9]
    host = ssd_counts_controlled(net, targets, 300, 64, Model(), seed=11)
    dev = ssd_counts_controlled_device(net, targets, 300, 64, policy, seed=11)
    assert np.array_equal(host, dev) and int(dev.sum()) == 300 * 64

    b = PBNBatch(net, 4, seed=2)
    b.randomize()
    s0 = b.get_state()
    acts = torch.tensor([[1, 0], [N + 1, 0], [3, 3], [0, 0]], dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        b.flip_device(acts.data_ptr(), 2)
    s1 = b.get_state()
    assert s1[1] == s0[1] and s1[3] == s0[3]  # the bad row and the no-op row
    assert s1[0] == s0[0] ^ np.uint64(1) and s1[2] == s0[2] ^ np.uint64(1 << 2)  # dedup: [3, 3] flips once
    b.flip_device(acts.data_ptr(), 2, check=False)  # asynchronous: the error waits for a checked call
    ok = torch.zeros((4, 1), dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        b.flip_device(ok.data_ptr(), 1)
    b.flip_device(ok.data_ptr(), 1)  # the flag was cleared by the check
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(6))
def test_ssd_random_shapes_all_modes_agree(oracle_mod, monkeypatch, case):
    """Seeded random batch sizes, run lengths, flip rates and target sets: every mode (lane,
    one wave, four and eight waves per env) gives the oracle's counts and states."""
    from gym_pbn_amd.batch import PBNBatch, flip_gap_table

    rng = np.random.default_rng(1000 + case)
    name = ["bittner28", "bittner199", "tt200"][case % 3]
    net = _net(name)
    B = int(rng.integers(1, 700))
    iters = int(rng.integers(1, 900))
    p = float(rng.choice([0.0, 0.005, 0.05]))
    targets = sorted(rng.choice(net.n_nodes, size=int(rng.integers(1, 9)), replace=False).tolist())
    rng.shuffle(targets)  # any order: the first target is the most significant bucket bit
    o = oracle_mod.Oracle(net)
    gap = flip_gap_table(net.n_nodes, p)
    ref = None
    for wave, shared in (("0", "0"), ("1", "0"), ("1", "4"), ("1", "8")):
        monkeypatch.setenv("PBNSIM_SSD_WAVE", wave)
        monkeypatch.setenv("PBNSIM_SSD_SHARED", shared)
        b = PBNBatch(net, B, seed=case, env_id_base=3 * case)
        b.randomize()
        s0 = b.get_state()
        h = b.ssd_counts(targets, iters, p)
        if ref is None:
            st, r = oracle_mod.ssd_philox(o, s0, targets, gap, case, 3 * case, 0, iters)
            ref = (st, r)
        assert np.array_equal(h, ref[1]), (wave, shared)
        assert np.array_equal(b.get_state(), ref[0]), (wave, shared)
        b.close()
