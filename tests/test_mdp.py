"""R7 PBNEnv and the macro-action MDP envs vs the reference (tests/golden/mdp_kat.json).

The fixtures run the reference env classes themselves (pbn_env.py, pbcn_env.py,
sampled_data.py, self_triggering.py) and log every draw. The device envs must
reproduce reset(seed) from the seed alone (its ``random.choice`` draws happen on
the host), then replay each step's transition draws (stdlib ``randint``, numpy
``uniform``) and self-triggering termination draws, and return the same
observation, reward, terminated, truncated and interval.
"""

import json
import random

import numpy as np
import pytest

from conftest import GOLDEN

KAT = json.loads((GOLDEN / "mdp_kat.json").read_text())


def _source(name):
    net = KAT["networks"][name]
    if net["PBN_data"] is not None:
        data = [(np.array(d["mask"], dtype=bool), np.array(d["table"]).reshape((2,) * sum(d["mask"])), d["name"],
                 d["control"]) for d in net["PBN_data"]]
        return {"PBN_data": data, "logic_func_data": None}
    nodes, funcs = net["logic_func_data"]
    return {"PBN_data": None, "logic_func_data": (nodes, [[tuple(f) for f in fs] for fs in funcs])}


def _network(name):
    from gym_pbn_amd.network import TruthTableNetwork

    src = _source(name)
    if src["PBN_data"] is not None:
        return TruthTableNetwork.from_pbn_data(src["PBN_data"])
    return TruthTableNetwork.from_logic_funcs(*src["logic_func_data"])


@pytest.mark.parametrize("name", sorted(KAT["networks"]))
def test_stg_attractors_match_reference(name):
    """compute_attractors == PBNEnv.compute_attractors (pbn_env.py:233-240) as a set of sets.

    The order is not comparable: networkx returns the components as sets of state
    *strings*, whose iteration order follows the per-process string hash seed
    (PYTHONHASHSEED), so the reference's own attractor order varies between runs."""
    from gym_pbn_amd.stg import compute_attractors

    ref = next(c["attractors"] for c in KAT["cases"] if c["network"] == name)
    got = compute_attractors(_network(name))
    canon = lambda atts: sorted(sorted(tuple(s) for s in a) for a in atts)  # noqa: E731
    assert canon(got) == canon(ref)


class _ReplayUniform:
    def __init__(self, values):
        self.values = list(values)

    def uniform(self, a, b):
        assert (a, b) == (0, 1)
        return self.values.pop(0)


def _env(case):
    from gym_pbn_amd import envs, mdp

    cls = {"PBNEnv": envs.PBNEnv, "PBNSampledDataEnv": mdp.PBNSampledDataEnv,
           "PBNSelfTriggeringEnv": mdp.PBNSelfTriggeringEnv, "PBCNEnv": mdp.PBCNEnv,
           "PBCNSampledDataEnv": mdp.PBCNSampledDataEnv, "PBCNSelfTriggeringEnv": mdp.PBCNSelfTriggeringEnv}[case["kind"]]
    target = {tuple(t) for t in case["target"]}
    # the attractors in the order the reference process held them (see the STG test), so that
    # reset(seed)'s random.choice over them picks the same state
    atts = [[tuple(s) for s in a] for a in case["attractors"]]
    return cls(goal_config={"all_attractors": [], "target_nodes": target}, **_source(case["network"]),
               **case["extra"], all_attractors=atts)


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(KAT["cases"])),
                         ids=[f'{c["network"]}-{c["kind"]}' for c in KAT["cases"]])
def test_env_replay_matches_reference(ci):
    case = KAT["cases"][ci]
    env = _env(case)
    for ep in case["episodes"]:
        env._rng = random.Random()  # the host RNG reset(seed) seeds (replaced by a replayer during steps)
        if ep.get("reset_error"):
            with pytest.raises(ValueError):
                env.reset(seed=ep["seed"])
            continue
        obs, info = env.reset(seed=ep["seed"])
        assert [int(x) for x in obs] == ep["reset_obs"], (ep["seed"], "reset")
        for t, st in enumerate(ep["steps"]):
            env.PBN.queue_replay(st["node_idx"], st["k53"])
            env._rng = _ReplayUniform(st["term_u"])
            a = tuple(st["action"]) if isinstance(st["action"], list) else st["action"]
            o, r, term, trunc, info = env.step(a)
            where = (ep["seed"], t, a)
            assert not env.PBN._replay and not env._rng.values, where  # every draw consumed
            assert [int(x) for x in o] == st["obs"], where
            assert r == st["reward"] and type(r) is type(st["reward"]), where
            assert (bool(term), bool(trunc)) == (st["terminated"], st["truncated"]), where
            assert info.get("interval") == st["interval"], where
            assert info["observation_idx"] == st["observation_idx"], where


@pytest.mark.gpu
def test_vec_pbn_env_matches_single_env_rules():
    """VecPBNEnv: B envs of PBN-v0 in one launch; rewards/termination as PBNEnv._get_reward
    (pbn_env.py:156-188) on the same device transitions (a twin batch stepped by hand)."""
    from gym_pbn_amd.batch import Net, PBNBatch, unpack_bits
    from gym_pbn_amd.envs import VecPBNEnv

    case = next(c for c in KAT["cases"] if c["network"] == "tt6" and c["kind"] == "PBNEnv")
    src = _source("tt6")
    target = {tuple(t) for t in case["target"]}
    B = 257
    v = VecPBNEnv(src["PBN_data"], goal_config={"target_nodes": target}, n_envs=B, seed=3)
    twin = PBNBatch(Net(v.network), B, seed=3)
    obs = v.reset()
    twin.set_bits(obs)
    rng = np.random.default_rng(0)
    for t in range(20):
        a = rng.integers(0, v.N, size=B)
        a[rng.random(B) < 0.5] = 0
        o, r, term, trunc, info = v.step(a)
        bits = twin.get_bits()
        for e in np.nonzero(a)[0]:
            bits[e, a[e]] ^= 1  # PBNEnv flips node `action` (pbn_env.py:141-142)
        twin.set_bits(bits)
        twin.step(1)
        ref = twin.get_bits()
        assert np.array_equal(o, ref), t
        exp_term = np.array([tuple(int(x) for x in row) in v.target_nodes for row in ref])
        assert np.array_equal(term, exp_term) and not trunc.any()
        assert np.array_equal(r, np.where(exp_term, 20, -4 - (a != 0)))
    with pytest.raises(Exception):
        v.step(np.full(B, v.N))


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(KAT["cases"])),
                         ids=[f'{c["network"]}-{c["kind"]}' for c in KAT["cases"]])
def test_env_spaces_match_reference_constructors(ci):
    """observation / action / discrete-action spaces as the reference constructors build them
    (pbn_env.py:81-83, pbcn_env.py:41-45, sampled_data.py:43-49,118-129,
    self_triggering.py:44-48,122-127), and invalid actions rejected through them."""
    case = KAT["cases"][ci]
    env = _env(case)
    kind, N = case["kind"], env.PBN.N
    assert env.observation_space.shape == (N,)
    if kind == "PBNEnv":
        assert env.action_space.n == N and env.action_space.start == 0
        with pytest.raises(Exception, match="not in action space"):
            env.step(N)
        with pytest.raises(Exception, match="not in action space"):
            env.step(1.0)  # Discrete.contains rejects floats
    elif kind in ("PBNSampledDataEnv", "PBNSelfTriggeringEnv"):
        second = env.interval_space if kind == "PBNSampledDataEnv" else env.prob_space
        assert env.primitive_action_space.n == N + 1 and second.start == 1
        assert second.n == (env.T if kind == "PBNSampledDataEnv" else 10)
        assert env.discrete_action_space.n == (N + 1) * second.n
        assert env.action_space.contains((N, int(second.start)))
        with pytest.raises(Exception, match="not in action space"):
            env.step((N + 1, 1))
        with pytest.raises(Exception, match="not in action space"):
            env.step((0, 0))
    else:
        M = env.M
        if kind == "PBCNEnv":
            assert env.action_space.n == M and env.discrete_action_space.n == 2 ** M
        else:
            second = env.interval_space if kind == "PBCNSampledDataEnv" else env.prob_space
            assert env.primitive_action_space.n == M and second.start == 1
            assert env.discrete_action_space.n == (2 ** M) * second.n
            with pytest.raises(Exception, match="not in action space"):
                env.step(env.discrete_action_space.n)
            with pytest.raises(Exception, match="not in action space"):
                env.step(([0] * (M + 1), 1))
