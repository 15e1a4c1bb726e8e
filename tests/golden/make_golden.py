"""Generate the golden vectors under tests/golden/ from the reference itself.

Run in the build container only (``python tests/golden/make_golden.py``); the
outputs are committed, and tests read only those files.

What is captured (SURVEY §8c "Golden vectors to commit"):

* ``r1_<net>.npz`` -- R1 ``Graph.step`` (``base.py:306-312``) on the exported
  Bittner networks. Per seed: ``random.seed(s); graph.genRandState()``
  (``base.py:368-370``), then T steps. Every draw the reference makes is logged
  through a forwarding proxy on ``base.random`` (the real global MT19937 stream),
  giving the replay stream ``(node_idx_t, k53_t)`` with ``random() == k53*2**-53``,
  and the state tuple each step returns.
* ``r4_<net>.npz`` -- R4 ``PBN.step`` (``common/pbn.py:129-133``,
  ``common/node.py:34-38``) on synthetic truth-table PBNs. Per seed:
  ``random.seed(s); np.random.seed(s); pbn.reset()`` (``pbn.py:96-119``), then T
  steps; stdlib ``randint(1, N-1)`` and numpy ``uniform(0, 1)`` are logged.
* ``r6_<net>.npz`` -- R6 ``PBNTargetMultiEnv.step`` (``pbn_target_multi.py:119-154``)
  with ``BittnerMulti7.is_attracting_state`` (``:489-492``): ``reset(seed)``
  (``:227-259``) then a sequence of multi-flip action rows (torch tensors, so
  de-duplicated as at ``:120-121``; plus list rows, not de-duplicated). The
  attractor hypercubes are synthetic (cabean is unavailable) and expanded into
  ``attracting_states`` exactly as ``:437-455`` does.
* ``r1_mt_<net>.npz`` -- long R1 runs keyed only by the Python seed, for the
  device MT19937 mode (``random.seed(s)`` + ``genRandState`` + T steps; final
  states and a digest of every intermediate state).
"""

from __future__ import annotations

import hashlib
import json
import os
import random
import subprocess
import sys
from itertools import product
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(REPO / "gym-pbn-stac_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import refload  # noqa: E402
from gym_pbn_amd.io.safe_pickle import load_pickle_safely  # noqa: E402
from gym_pbn_amd.network import load_network, synthetic_truth_table_pbn  # noqa: E402

BITTNER = Path("/root/reference/gym_PBN/envs/bittner/data")
PICKLES = {"bittner28": "predictor_sets_28_15_median.pkl", "bittner199": "predictor_sets_200_5_kmeans.pkl",
           "bittner70": "predictor_sets_70_5_kmeans.pkl"}
TWO53 = float(1 << 53)


def pack(bits) -> np.ndarray:
    bits = np.asarray(bits, dtype=np.uint64)
    W = (bits.shape[-1] + 63) // 64
    out = np.zeros(bits.shape[:-1] + (W,), dtype=np.uint64)
    for i in range(bits.shape[-1]):
        out[..., i // 64] |= bits[..., i] << np.uint64(i % 64)
    return out


def k53_of(u: float) -> int:
    k = u * TWO53
    assert k == int(k) and 0 <= k < TWO53
    return int(k)


def pairs(log, first="i", second="u"):
    assert len(log) % 2 == 0, log
    out = []
    for a, b in zip(log[0::2], log[1::2]):
        assert a[0] == first and b[0] == second, (a, b)
        out.append((int(a[1]), k53_of(b[1])))
    return out


def gen_r1(base, name, seeds=(0, 1, 2, 3), T=2000):
    net = load_network(name)
    ps = load_pickle_safely(BITTNER / PICKLES[name])
    g = refload.build_graph(base, ps, net.node_ids)
    rec = refload.DrawRecorder(random)
    base.random = rec
    out = {"seeds": np.array(seeds, dtype=np.int64)}
    inits, idx, k53, states = [], [], [], []
    try:
        for s in seeds:
            random.seed(s)
            g.genRandState()
            inits.append(pack([n.value for n in g.nodes]))
            rec.log.clear()
            st = []
            for _ in range(T):
                st.append(g.step())
            pr = pairs(rec.log)
            idx.append([p[0] for p in pr])
            k53.append([p[1] for p in pr])
            states.append(pack(np.array(st)))
    finally:
        base.random = random
    out["init"] = np.stack(inits)  # [S][W]
    out["node_idx"] = np.array(idx, dtype=np.uint32)  # [S][T]
    out["k53"] = np.array(k53, dtype=np.uint64)  # [S][T]
    out["states"] = np.stack(states)  # [S][T][W]
    np.savez_compressed(HERE / f"r1_{name}.npz", **out)
    print("r1", name, out["states"].shape)


def gen_r1_mt(base, name, seeds=(0, 1, 7, 12345), T=5000):
    """Seed-only fixtures: the device MT19937 mode must reproduce these from the seed alone."""
    net = load_network(name)
    ps = load_pickle_safely(BITTNER / PICKLES[name])
    g = refload.build_graph(base, ps, net.node_ids)
    finals, inits, digests, checkpoints = [], [], [], []
    for s in seeds:
        random.seed(s)
        g.genRandState()
        inits.append(pack([n.value for n in g.nodes]))
        h = hashlib.sha256()
        cps = []
        for t in range(T):
            st = g.step()
            w = pack(np.array(st))
            h.update(w.tobytes())
            if (t + 1) % 1000 == 0:
                cps.append(w)
        finals.append(pack(np.array(g.getState())))
        digests.append(h.hexdigest())
        checkpoints.append(np.stack(cps))
    np.savez_compressed(HERE / f"r1_mt_{name}.npz", seeds=np.array(seeds, dtype=np.int64),
                        init=np.stack(inits), final=np.stack(finals), checkpoints=np.stack(checkpoints),
                        T=np.int64(T), digests=np.array(digests))
    print("r1_mt", name)


def gen_r4(pbn_mod, node_mod, name, n, k, data_seed, seeds=(0, 1, 2, 3), T=2000):
    data = synthetic_truth_table_pbn(n, k, data_seed)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        p = pbn_mod.PBN(PBN_data=data)
    rec_std = refload.DrawRecorder(random)
    rec_np = refload.DrawRecorder(np.random)
    pbn_mod.random = rec_std
    node_mod.random = rec_np
    inits, idx, k53, states = [], [], [], []
    try:
        for s in seeds:
            random.seed(s)
            np.random.seed(s)
            p.reset()
            inits.append(pack(p.state.astype(np.uint8)))
            rec_std.log.clear()
            rec_np.log.clear()
            st = []
            for _ in range(T):
                p.step()
                st.append(p.state.astype(np.uint8).copy())
            assert all(e[0] == "i" for e in rec_std.log) and all(e[0] == "u" for e in rec_np.log)
            idx.append([e[1] for e in rec_std.log])
            k53.append([k53_of(e[1]) for e in rec_np.log])
            states.append(pack(np.array(st)))
    finally:
        pbn_mod.random = random
        node_mod.random = np.random
    np.savez_compressed(HERE / f"r4_{name}.npz", seeds=np.array(seeds, dtype=np.int64), init=np.stack(inits),
                        node_idx=np.array(idx, dtype=np.uint32), k53=np.array(k53, dtype=np.uint64),
                        states=np.stack(states))
    print("r4", name)


def cube_from_bias(mean, fixed_bits, overrides=None):
    """Hypercube tuple: fixed bits at their majority value, '*' elsewhere."""
    cube = ["*"] * len(mean)
    for b in fixed_bits:
        cube[b] = int(mean[b] >= 0.5)
    for b, v in (overrides or {}).items():
        cube[b] = v
    return tuple(cube)


def expand(all_attractors):
    """Verbatim semantics of pbn_target_multi.py:437-455 (expansion of '*')."""
    attracting = set()
    for attractor in all_attractors:
        for state in attractor:
            stars, positions = 0, []
            for i, s in enumerate(state):
                if s == "*":
                    stars += 1
                    positions.append(i)
            if stars == 0:
                attracting.add(tuple(state))
            for p in product([0, 1], repeat=stars):
                sm = list(state)
                for i, pos in enumerate(positions):
                    sm[pos] = p[i]
                    attracting.add(tuple(sm))
    return attracting


class HypercubeSet:
    """Membership-equivalent stand-in for the expanded set of :func:`expand`."""

    def __init__(self, cubes):
        self.cubes = cubes

    def __contains__(self, state):
        return any(all(c == "*" or c == x for c, x in zip(cube, state)) for cube in self.cubes)


def cube_arrays(cubes, N):
    W = (N + 63) // 64
    care = np.zeros((len(cubes), W), dtype=np.uint64)
    val = np.zeros((len(cubes), W), dtype=np.uint64)
    for h, c in enumerate(cubes):
        for i in range(N):
            if c[i] != "*":
                care[h, i // 64] |= np.uint64(1) << np.uint64(i % 64)
                if c[i]:
                    val[h, i // 64] |= np.uint64(1) << np.uint64(i % 64)
    return care, val


def gen_r6(base, multi, name, n_fixed, horizon, seeds, n_steps, list_every=0, max_stars=12):
    net = load_network(name)
    N = net.n_nodes
    ps = load_pickle_safely(BITTNER / PICKLES[name])
    g = refload.build_graph(base, ps, net.node_ids)
    # bias statistics from a reference run decide which bits the synthetic attractors fix
    random.seed(99)
    g.genRandState()
    S = np.array([g.step() for _ in range(30000)])[2000:]
    mean = S.mean(0)
    order = np.argsort(-np.abs(mean - 0.5), kind="stable")
    fixed = sorted(order[:n_fixed].tolist())
    extra = sorted(order[n_fixed:n_fixed + 4].tolist())
    c0 = cube_from_bias(mean, fixed)
    c1 = cube_from_bias(mean, fixed, {b: 1 - int(mean[b] >= 0.5) for b in extra[:1]})
    c2 = cube_from_bias(mean, fixed + extra[:2])
    c3 = cube_from_bias(mean, fixed + extra[:3], {b: 1 - int(mean[b] >= 0.5) for b in extra[1:2]})
    all_attractors = [[c0], [c1, c2], [c3]]
    env = object.__new__(multi.BittnerMulti7)
    env.graph = g
    env.horizon = horizon
    env.n_steps = 0
    env.all_attractors = all_attractors
    if N - n_fixed <= max_stars:
        env.attracting_states = expand(all_attractors)  # the reference's own expansion
    else:
        # 2**stars states cannot be enumerated; the expansion's membership test is
        # exactly "matches some hypercube", which HypercubeSet implements.
        env.attracting_states = HypercubeSet([c for a in all_attractors for c in a])
    env.attractor_count = len(all_attractors)
    env.probabilities = [1 / 3] * 3
    from collections import defaultdict
    env.recent_actions = defaultdict(lambda: 10)
    env.target = None
    rec = refload.DrawRecorder(random)
    base.random = rec
    rng = np.random.default_rng(1234)
    rows = []
    try:
        for s in seeds:
            (st, tg), info = env.reset(seed=s)
            reset_state = pack(np.array(g.getState()))
            for t in range(n_steps):
                a = rng.integers(0, N + 1, size=4)
                a[rng.random(4) < 0.5] = 0
                use_list = list_every and (t % list_every == list_every - 1)
                rec.log.clear()
                if use_list:
                    obs, reward, term, trunc, info = env.step([int(x) for x in a])
                else:
                    obs, reward, term, trunc, info = env.step(torch.tensor(a))
                dr = pairs(rec.log)
                rows.append(dict(seed=s, t=t, reset_state=reset_state, actions=a.astype(np.int32),
                                 is_list=int(bool(use_list)), obs=pack(np.array(obs)),
                                 state_after=pack(np.array(g.getState())), reward=int(reward),
                                 terminated=int(term), truncated=int(trunc), n_steps=int(env.n_steps),
                                 obs_idx=str(info["observation_idx"]),
                                 draws_i=[d[0] for d in dr], draws_k=[d[1] for d in dr]))
    finally:
        base.random = random
    care, val = cube_arrays([c for a in all_attractors for c in a], N)
    cube_attr = np.array([ai for ai, a in enumerate(all_attractors) for _ in a], dtype=np.int32)
    offs = np.cumsum([0] + [len(r["draws_i"]) for r in rows]).astype(np.int64)
    out = dict(
        cube_care=care, cube_value=val, cube_attractor=cube_attr, horizon=np.int64(horizon),
        seed=np.array([r["seed"] for r in rows], dtype=np.int64), t=np.array([r["t"] for r in rows], dtype=np.int64),
        reset_state=np.stack([r["reset_state"] for r in rows]), actions=np.stack([r["actions"] for r in rows]),
        is_list=np.array([r["is_list"] for r in rows], dtype=np.int32), obs=np.stack([r["obs"] for r in rows]),
        state_after=np.stack([r["state_after"] for r in rows]),
        reward=np.array([r["reward"] for r in rows], dtype=np.int32),
        terminated=np.array([r["terminated"] for r in rows], dtype=np.int32),
        truncated=np.array([r["truncated"] for r in rows], dtype=np.int32),
        n_steps=np.array([r["n_steps"] for r in rows], dtype=np.int64),
        obs_idx=np.array([r["obs_idx"] for r in rows]),
        draw_offsets=offs,
        draws_i=np.array([x for r in rows for x in r["draws_i"]], dtype=np.uint32),
        draws_k=np.array([x for r in rows for x in r["draws_k"]], dtype=np.uint64),
    )
    np.savez_compressed(HERE / f"r6_{name}.npz", **out)
    lens = np.diff(offs)
    print("r6", name, len(rows), "updates/step min/med/max", lens.min(), int(np.median(lens)), lens.max(),
          "terminated", int(out["terminated"].sum()), "truncated", int(out["truncated"].sum()))


def gen_r5_reset(base):
    """R5 reset KAT: PBNTargetEnv.reset (pbn_target.py:328-352) -- reset works at HEAD, step does not."""
    tgt = refload.load_target_env()
    net = load_network("bittner28")
    ps = load_pickle_safely(BITTNER / PICKLES["bittner28"])
    g = refload.build_graph(base, ps, net.node_ids)
    env = object.__new__(tgt.PBNTargetEnv)
    env.graph = g
    env.horizon = 100
    N = net.n_nodes
    rng = np.random.default_rng(3)
    atts = []
    for a in range(4):
        cubes = []
        for _ in range(1 + a % 2):
            c = ["*"] * N
            for j in rng.choice(N, size=10, replace=False):
                c[int(j)] = int(rng.integers(0, 2))
            cubes.append(tuple(c))
        atts.append(cubes)
    env.all_attractors = atts
    cases = []
    for seed in (1, 2, 3, 11, 12345):
        (st, tg), info = env.reset(seed=seed)
        cases.append({"seed": seed, "state": list(st), "target": list(tg), "graph": [int(x) for x in g.getState()],
                      "target_attractor": [list(c) for c in env.target]})
    doc = {"attractors": [[list(c) for c in a] for a in atts], "cases": cases}
    (HERE / "r5_reset_kat.json").write_text(json.dumps(doc) + "\n")
    print("r5 reset kat", len(cases))


def gen_cabean_kat(multi):
    """KAT: parse_attractors(sample_cabean_out) (get_attractors_from_cabean.py:57-81)."""
    cab = sys.modules["gym_PBN.utils.get_attractors_from_cabean"]
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        parsed = cab.parse_attractors(cab.sample_cabean_out)
    doc = {"input": cab.sample_cabean_out,
           "expected": {str(k): [list(t) for t in v] for k, v in parsed.items()}}
    (HERE / "cabean_parse_kat.json").write_text(json.dumps(doc, indent=1) + "\n")
    print("cabean kat", doc["expected"])


LOGIC_EXPRS = [
    "(a)", "(a and b)", "((a or b) and c)", "not not a", "a and not b or c", "True", "False", "a or True and b",
    "not (a or b)", "(not a)", "a and (b or (c and d))", "x1 and x2", "a and", "and a", "a b", "((a)", "a))",
    "not a and b", "a or b and c", "True or a", "a and True", "True and a", "not True", "(True)", "gene_1 and x",
    "a1b2 and c", "(a or b) and (c or d)", "not", "a or", ")", "( a )", "not (a and (b or not c)) or d and not a",
    "a and b or c and d or not e", "((a and b))", "(a or (b))", "a not b", "a (b)", "1a", "a or not (b and c)",
    "not a or not b and not c", "(a or b) and not (c or d) or (e and not a)", "False or a", "a and False",
]
LOGIC_NETS = [
    (["u", "x1", "x2", "x3", "x4"],  # example.py:24-35 (test_example_1)
     [[], [("not x2 and not x4", 1)], [("not x4 and not u and (x2 or x3)", 1)],
      [("not x2 and not x4 and x1", 0.7), ("False", 0.3)], [("not x2 and not x3", 1)]]),
    (["a", "b", "c", "d"],
     [[("b or c", 0.25), ("not d", 0.35), ("b and c and d", 0.4)], [("True", 0.5), ("a", 0.5)],
      [("(a or b) and (d or a)", 0.1), ("not a", 0.2), ("b", 0.3), ("d", 0.15)], [("a and b and c", 1)]]),
    (["p", "q"], [[("q", 0.3)], [("p", 0.1), ("p", 0.2), ("not p", 0.7)]]),
    (["a", "b"], [[("c", 1)], [("a", 1)]]),  # unknown symbol
]


def gen_logic():
    """Logic evaluator + converter KATs (utils/logic/eval.py, utils/converters.py:9-40)."""
    ev = sys.modules["gym_PBN.utils.logic.eval"]
    conv = sys.modules["gym_PBN.utils.converters"]
    exprs = []
    for e in LOGIC_EXPRS:
        rec = {"expr": e}
        try:
            syms = ev.LogicExpressionEvaluator.get_symbols(e)
            rec["symbols"] = syms
            order = sorted(set(syms))
            vals = []
            for bits in product([0, 1], repeat=len(order)):
                vals.append(int(ev.LogicExpressionEvaluator(dict(zip(order, bits))).evaluate(e)))
            rec["values"] = vals
        except Exception as exc:  # the reference rejects it
            rec["error"] = type(exc).__name__
        exprs.append(rec)
    nets = []
    for nodes, funcs in LOGIC_NETS:
        rec = {"nodes": nodes, "functions": [[list(f) for f in fs] for fs in funcs]}
        try:
            data = conv.logic_funcs_to_PBN_data(nodes, funcs)
            rec["expected"] = [{"mask": [int(x) for x in d[0]], "table": np.asarray(d[1]).reshape(-1).tolist(),
                                "name": d[2], "control": bool(d[3])} for d in data]
        except Exception as exc:
            rec["error"] = type(exc).__name__
        nets.append(rec)
    (HERE / "logic_kat.json").write_text(json.dumps({"expressions": exprs, "networks": nets}, indent=1) + "\n")
    print("logic kat", sum("error" in r for r in exprs), "rejected of", len(exprs))


def _mdp_networks():
    """(name, PBN_data or None, logic_func_data or None) used for the env fixtures.

    ``PBNEnv.reset`` loops until it draws an attractor of at most 10 states
    (``pbn_env.py:204-206``), so every network here has one.
    """
    rng = np.random.default_rng(35)
    data = []
    N = 6
    for i in range(N):
        others = [j for j in range(N) if j != i]
        k = 2 if i else 0  # node 0: no inputs -> a control node for the PBCN envs
        inp = sorted(rng.choice(others, size=k, replace=False).tolist())
        mask = np.zeros(N, dtype=bool)
        mask[inp] = True
        tt = rng.choice([0.0, 1.0, 0.0, 1.0, 0.8], size=(2,) * k) if k else np.array(0.0)
        data.append((mask, tt, f"G{i}", k == 0))
    logic4 = (["u", "a", "b", "c"], [[], [("not b", 1)], [("a and not u", 1)], [("b or c", 0.5), ("a", 0.5)]])
    return [("tt6", data, None), ("logic5", None, LOGIC_NETS[0]), ("logic4", None, logic4)]


def _to_json_data(data):
    return [{"mask": [int(x) for x in d[0]], "table": np.asarray(d[1]).reshape(-1).tolist(), "name": d[2],
             "control": bool(d[3])} for d in data]


def gen_mdp(node_mod, pbn_mod):
    """R7 + macro-action env KATs: PBNEnv, PBCNEnv, sampled-data and self-triggering envs.

    Each env is the reference class itself (gymnasium spaces are inert stand-ins whose
    ``contains`` accepts everything; only valid actions are fed). Transition draws
    (stdlib ``randint``, numpy ``uniform``) and the self-triggering termination draws
    (stdlib ``uniform``) are logged per env step so the device envs can replay them;
    ``reset(seed)``'s own ``random.choice`` draws are not replayed -- the device env
    must reproduce the reset state from the seed.
    """
    import contextlib
    import io
    pbn_env, pbcn_env, sampled, selftrig, pbcn = refload.load_mdp_envs()
    kinds = [("PBNEnv", pbn_env.PBNEnv, {}), ("PBNSampledDataEnv", sampled.PBNSampledDataEnv, {"T": 4}),
             ("PBNSelfTriggeringEnv", selftrig.PBNSelfTriggeringEnv, {}), ("PBCNEnv", pbcn_env.PBCNEnv, {}),
             ("PBCNSampledDataEnv", sampled.PBCNSampledDataEnv, {"T": 3}),
             ("PBCNSelfTriggeringEnv", selftrig.PBCNSelfTriggeringEnv, {"T": 6})]
    rec_std, rec_np, rec_st = (refload.DrawRecorder(random), refload.DrawRecorder(np.random),
                               refload.DrawRecorder(random))
    out = []
    for net_name, data, logic in _mdp_networks():
        src = {"PBN_data": list(data) if data is not None else [], "logic_func_data": logic}
        with contextlib.redirect_stdout(io.StringIO()):
            probe = pbn_env.PBNEnv(goal_config={"all_attractors": [], "target_nodes": set()}, **src)
        attractors = [list(a) for a in probe.all_attractors]
        target = {attractors[-1][0]}
        rng = np.random.default_rng(11)
        for kind, cls, extra in kinds:
            with contextlib.redirect_stdout(io.StringIO()):
                env = cls(goal_config={"all_attractors": [], "target_nodes": set(target)}, **src, **extra)
            N = env.PBN.N
            M = getattr(env.PBN, "M", 0)
            rec = {"network": net_name, "kind": kind, "extra": extra, "attractors": [[list(s) for s in a]
                                                                                    for a in attractors],
                   "target": [list(t) for t in target], "episodes": []}
            pbn_mod.random, pbcn.randint, node_mod.random, selftrig.random = (rec_std, rec_std.randint, rec_np,
                                                                              rec_st)
            try:
                for seed in (0, 1, 2, 5, 9):
                    ep = {"seed": seed}
                    try:
                        with contextlib.redirect_stdout(io.StringIO()):
                            obs, info = env.reset(seed=seed)
                    except ValueError:
                        ep["reset_error"] = True
                        rec["episodes"].append(ep)
                        continue
                    ep["reset_obs"] = [int(x) for x in obs]
                    steps = []
                    for t in range(12):
                        if kind == "PBNEnv" or kind == "PBCNEnv":
                            a = int(rng.integers(0, N)) if rng.random() < 0.6 else 0
                        elif kind == "PBNSampledDataEnv":
                            a = (int(rng.integers(0, N + 1)), int(rng.integers(1, 5)))
                        elif kind == "PBNSelfTriggeringEnv":
                            a = (int(rng.integers(0, N + 1)), int(rng.integers(1, 11)))
                        elif kind == "PBCNSampledDataEnv":
                            a = int(rng.integers(0, (2 ** M) * 3))
                        else:
                            a = int(rng.integers(0, (2 ** M) * 10))
                        for r in (rec_std, rec_np, rec_st):
                            r.log.clear()
                        with contextlib.redirect_stdout(io.StringIO()):
                            o, reward, term, trunc, info = env.step(a)
                        assert all(e[0] == "i" for e in rec_std.log) and len(rec_std.log) == len(rec_np.log)
                        steps.append({"action": list(a) if isinstance(a, tuple) else a,
                                      "obs": [int(x) for x in o], "reward": reward, "terminated": bool(term),
                                      "truncated": bool(trunc), "interval": info.get("interval"),
                                      "observation_idx": int(info["observation_idx"]),
                                      "node_idx": [int(e[1]) for e in rec_std.log],
                                      "k53": [k53_of(e[1]) for e in rec_np.log],
                                      "term_u": [float(e[1]) for e in rec_st.log]})
                    ep["steps"] = steps
                    rec["episodes"].append(ep)
            finally:
                pbn_mod.random, pbcn.randint, node_mod.random, selftrig.random = (random, random.randint, np.random,
                                                                                  random)
            out.append(rec)
    nets = {n: {"PBN_data": _to_json_data(d) if d is not None else None, "logic_func_data": lf}
            for n, d, lf in _mdp_networks()}
    (HERE / "mdp_kat.json").write_text(json.dumps({"networks": nets, "cases": out}) + "\n")
    print("mdp kat", len(out), "cases;", sum(len(e.get("steps", [])) for r in out for e in r["episodes"]), "steps")


def main():
    base, node_mod, pbn_mod = refload.load_hot_path()
    only = set(sys.argv[1:])
    if not only or "r1" in only:
        gen_r1(base, "bittner28")
        gen_r1(base, "bittner199")
        gen_r1(base, "bittner70", seeds=(5,), T=1000)
    if not only or "r4" in only:
        gen_r4(pbn_mod, node_mod, "tt200", 200, 4, 0)
        gen_r4(pbn_mod, node_mod, "tt8", 8, 3, 1, T=3000)
    if not only or "mt" in only:
        gen_r1_mt(base, "bittner28")
        gen_r1_mt(base, "bittner199", T=3000)
    if not only or "logic" in only:
        gen_logic()
    if not only or "mdp" in only:
        if os.environ.get("PYTHONHASHSEED") == "0":
            gen_mdp(node_mod, pbn_mod)
        else:
            # PBNEnv.compute_attractors returns networkx sets of state strings whose iteration order
            # follows the string-hash seed, and reset(seed) picks by position: the fixture is only
            # reproducible under a fixed PYTHONHASHSEED, which must be set before the interpreter
            # starts -- so the mdp cases run in a child process with PYTHONHASHSEED=0
            subprocess.run([sys.executable, str(Path(__file__).resolve()), "mdp"],
                           env={**os.environ, "PYTHONHASHSEED": "0"}, check=True)
    if not only or "r6" in only or "cabean" in only:
        multi = refload.load_multi_env()
        if not only or "r6" in only:
            gen_r6(base, multi, "bittner28", n_fixed=16, horizon=7, seeds=(1, 2, 3), n_steps=40, list_every=5)
            gen_r6(base, multi, "bittner199", n_fixed=165, horizon=100, seeds=(4, 5), n_steps=10)
        gen_cabean_kat(multi)
    if not only or "r5" in only:
        gen_r5_reset(base)


if __name__ == "__main__":
    main()
