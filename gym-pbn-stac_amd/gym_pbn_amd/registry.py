"""``make(id, **kwargs)`` for the reference's environment ids (``gym_PBN/__init__.py:1-134``).

gymnasium is not a dependency here, so this is a plain registry with the same ids.
Networks the reference builds from ``genedata.xls`` by predictor inference
(``bittner/utils.py:54-91``) are the exported networks bundled in ``gym_pbn_amd/data``
where the reference ships their predictor sets; attractors (the reference runs the
external ``cabean`` binary, ``get_attractors_from_cabean.py:39-54``) must be passed as
``all_attractors`` (``gym_pbn_amd.io.cabean.attractors_list`` parses cabean's output).
``max_episode_steps=100`` (a gymnasium TimeLimit in the reference) is the envs'
``horizon``.
"""

from __future__ import annotations

from typing import Callable, Dict

from . import envs, mdp

# id -> (factory, default kwargs). Bittner ids map to the bundled network of that size.
_BITTNER = {28: "bittner28", 70: "bittner70", 100: "bittner100", 200: "bittner199"}


def _target(n):
    def f(all_attractors=None, **kw):
        if all_attractors is None:
            raise ValueError("all_attractors is required (cabean output; see gym_pbn_amd.io.cabean)")
        return envs.PBNTargetEnv(kw.pop("network", _BITTNER[n]), all_attractors, **kw)

    return f


def _multi(n):
    def f(all_attractors=None, **kw):
        if all_attractors is None:
            raise ValueError("all_attractors is required (cabean output; see gym_pbn_amd.io.cabean)")
        return envs.PBNTargetMultiEnv(kw.pop("network", _BITTNER[n]), all_attractors, **kw)

    return f


def _missing(n, what):
    def f(network=None, all_attractors=None, **kw):
        if network is None:
            raise NotImplementedError(
                f"{what}: the reference builds this {n}-gene network from genedata.xls by predictor inference "
                "(out of scope); pass network= (a PredictorNetwork or a bundled name) and all_attractors=")
        return (envs.PBNTargetEnv if what.startswith("Bittner-") else envs.PBNTargetMultiEnv)(
            network, all_attractors, **kw)

    return f


def _general(N=200, all_attractors=None, **kw):  # pbn_target_multi.py:531-536 (N=200 -> the 199-node network)
    net = kw.pop("network", "bittner199" if N in (199, 200) else None)
    if net is None:
        raise NotImplementedError(f"BittnerMultiGeneral(N={N}): only N=200 ships (predictor_sets_200_5_kmeans)")
    if all_attractors is None:
        raise ValueError("all_attractors is required (cabean output; see gym_pbn_amd.io.cabean)")
    return envs.PBNTargetMultiEnv(net, all_attractors, **kw)


def _pbn_target(graph=None, goal_config=None, render_mode=None, render_no_cache=False, name=None,
                reward_config=None, end_episode_on_success=False, *, all_attractors=None, **kw):
    """``gym-PBN/PBN-target-v0`` -> ``PBNTargetEnv`` (``gym_PBN/__init__.py:5``) with the reference
    constructor (``pbn_target.py:26-110``): ``graph`` (here a network: a ``PredictorNetwork`` or a
    bundled name), ``goal_config`` with ``target_nodes`` / ``target_node_values`` /
    ``undesired_node_values`` / ``intervene_on`` (more than one missing raises, as ``_check_config``
    does; an empty config raises ``ValueError``), optional ``goal_config["horizon"]`` (default 100),
    ``reward_config`` (defaults 10 / 2 / 1; kept as attributes -- the reward itself is +20 / -5,
    ``:303-326``). The base class starts with no attractors (``:101``), so ``reset`` could never run
    there; here they are the keyword ``all_attractors`` (cabean output), required."""
    if graph is None:
        raise TypeError("PBNTargetEnv() missing required argument: 'graph'")
    goal_config = envs.PBNEnv._check_config(
        goal_config, "goal", {"target_nodes", "target_node_values", "undesired_node_values", "intervene_on"})
    if goal_config is None:
        raise ValueError("Target nodes, target values and intervention nodes need to be specified.")
    reward_config = envs.PBNEnv._check_config(
        reward_config, "reward", {"successful_reward", "wrong_attractor_cost", "action_cost"},
        default_values={"successful_reward": 10, "wrong_attractor_cost": 2, "action_cost": 1})
    # subscripts, as pbn_target.py:61-64: with exactly one key missing _check_config passes and
    # the subscript raises KeyError
    goal = (goal_config["target_nodes"], goal_config["target_node_values"],
            goal_config["undesired_node_values"], goal_config["intervene_on"])
    if all_attractors is None:
        raise ValueError("all_attractors is required (cabean output; see gym_pbn_amd.io.cabean)")
    env = envs.PBNTargetEnv(graph, all_attractors, horizon=goal_config.get("horizon", 100), name=name, **kw)
    env.target_nodes, env.target_node_values, env.undesired_node_values, env.intervene_on = goal
    env.successful_reward = reward_config["successful_reward"]
    env.wrong_attractor_cost = reward_config["wrong_attractor_cost"]
    env.action_cost = reward_config["action_cost"]
    env.end_episode_on_success = end_episode_on_success
    env.render_mode, env.render_no_cache = render_mode, render_no_cache
    return env


REGISTRY: Dict[str, Callable] = {
    "gym-PBN/PBN-v0": envs.PBNEnv,
    "gym-PBN/PBN-target-v0": _pbn_target,
    "gym-PBN/PBN-sampled-data-v0": mdp.PBNSampledDataEnv,
    "gym-PBN/PBN-self-triggering-v0": mdp.PBNSelfTriggeringEnv,
    "gym-PBN/PBCN-v0": mdp.PBCNEnv,
    "gym-PBN/PBCN-sampled-data-v0": mdp.PBCNSampledDataEnv,
    "gym-PBN/PBCN-self-triggering-v0": mdp.PBCNSelfTriggeringEnv,
    "gym-PBN/BittnerMultiGeneral-v0": _general,
}
for _n in (7, 10, 30, 50):
    REGISTRY[f"gym-PBN/Bittner-{_n}-v0"] = _missing(_n, f"Bittner-{_n}-v0")
for _n in (28, 70, 100, 200):
    REGISTRY[f"gym-PBN/Bittner-{_n}-v0"] = _target(_n)
for _n in (7, 10, 20, 25, 50):
    REGISTRY[f"gym-PBN/BittnerMulti-{_n}-v0"] = _missing(_n, f"BittnerMulti-{_n}-v0")
REGISTRY["gym-PBN/BittnerMulti-28-v0"] = _multi(28)
REGISTRY["gym-PBN/BittnerMulti-30-v0"] = _multi(28)  # __init__.py:115-120 registers BittnerMulti28 under -30 (Q15)


def make(env_id: str, **kwargs):
    if env_id not in REGISTRY:
        raise KeyError(f"unknown env id {env_id!r}; known: {sorted(REGISTRY)}")
    return REGISTRY[env_id](**kwargs)


__all__ = ["make", "REGISTRY"]
