"""Drop-in env surfaces over the device batch (gym_PBN.envs conventions).

* :class:`Graph`            -- ``gym_PBN/envs/bittner/base.py`` ``Graph`` (step/flipNode/setState/getState/...).
* :class:`PBN`              -- ``gym_PBN/envs/common/pbn.py`` ``PBN`` (reset/flip/step/state).
* :class:`PBNTargetMultiEnv` -- ``gym_PBN/envs/pbn_target_multi.py`` single env (reset/step, R6).
* :class:`VecPBNTargetMultiEnv` -- the same MDP over B envs in one call (Stable-Baselines3 VecEnv shaped).
* :class:`PBNEnv`           -- ``gym_PBN/envs/pbn_env.py`` ``PBNEnv`` step/reward conventions (R7).

Every transition runs on the GPU through libpbnsim (Philox mode). Return
conventions follow the reference: observations of the multi env are tuples,
rewards ints, ``info["observation_idx"]`` the state as an int with node 0 as
the most significant bit (``pbn_target_multi.py:295-298``).
"""

from __future__ import annotations

from typing import Optional

import numpy as np

from . import _lib as L
from .batch import EnvConfig, Net, PBNBatch, pack_bits, unpack_bits
from .network import PredictorNetwork, TruthTableNetwork, load_network


def state_to_idx(bits) -> int:
    """``int("".join(str(x) for x in state), 2)`` (pbn_target_multi.py:295-298)."""
    v = 0
    for x in bits:
        v = (v << 1) | int(x)
    return v


class Graph:
    """Single-env mirror of ``base.Graph`` backed by a one-env device batch."""

    def __init__(self, network, device: int = 0, seed: int = 0, env_id: int = 0):
        if not isinstance(network, PredictorNetwork):
            network = load_network(network)
        self.network = network
        self._b = PBNBatch(Net(network), 1, device=device, env_id_base=env_id, seed=seed)
        self._initialised = False

    @property
    def N(self) -> int:  # base.py:195-197
        return self.network.n_nodes

    def getIDs(self):  # base.py:332-334
        return [int(x) for x in self.network.node_ids]

    def genRandState(self):  # base.py:368-370
        self._b.randomize()
        self._initialised = True

    def setState(self, state):  # base.py:364-366
        bits = np.array([int(x) for x in state], dtype=np.uint8)
        if bits.shape[0] != self.N:
            raise ValueError(f"state has {bits.shape[0]} values, graph has {self.N} nodes")
        self._b.set_bits(bits[None])
        self._initialised = True

    def getState(self) -> tuple:  # base.py:320-324
        return tuple(int(x) for x in self._b.get_bits()[0])

    def getLabeledState(self) -> dict:  # base.py:314-318
        return dict(zip(self.getIDs(), self.getState()))

    def flipNode(self, index: int):  # base.py:280-284
        if index >= self.N:
            raise ValueError(f"Invalid action, no node at index {index}")
        self._b.flip(np.array([[index + 1]], dtype=np.int32), offset=1, dedup=True)

    def step(self, changed_nodes=None, i=None) -> tuple:  # base.py:306-312 (changed_nodes is ignored there too)
        if not self._initialised:
            raise Exception("Forgot to initialise the states")  # base.py:90-91
        if i is not None:
            raise NotImplementedError("a forced node index is not supported by the Philox device stream")
        self._b.step(1)
        return self.getState()


class PBN:
    """Single-env mirror of ``common.pbn.PBN`` (truth-table engine)."""

    def __init__(self, PBN_data=None, network: Optional[TruthTableNetwork] = None, device: int = 0, seed: int = 0,
                 env_id: int = 0):
        if network is None:
            network = TruthTableNetwork.from_pbn_data(PBN_data)
        self.network = network
        self.N = network.n_nodes
        self._b = PBNBatch(Net(network), 1, device=device, env_id_base=env_id, seed=seed)

    @property
    def state(self) -> np.ndarray:
        return self._b.get_bits()[0].astype(bool)

    def reset(self, state=None) -> np.ndarray:  # pbn.py:96-119
        if state is None:
            self._b.randomize()  # also clears node 0
        else:
            if len(state) != self.N:
                raise Exception(
                    f"The length of the state given ({len(state)}) is different from the PBN size ({self.N})."
                )
            bits = np.array(state, dtype=bool).astype(np.uint8)
            bits[0] = 0
            self._b.set_bits(bits[None])
        return self.state

    def flip(self, index: int):  # pbn.py:121-127
        if not (-self.N <= index < self.N):
            raise IndexError(index)
        self._b.flip(np.array([[index]], dtype=np.int32), offset=0, dedup=True)

    def step(self):  # pbn.py:129-133
        self._b.step(1)


class VecPBNTargetMultiEnv:
    """B copies of the multi-flip until-attractor MDP (pbn_target_multi.py:119-259) in one launch.

    ``step(actions)`` takes ``[B][A]`` int actions (node+1, 0 = none; de-duplicated
    per row like a torch tensor input) and returns numpy arrays
    ``(obs [B][N] uint8, reward [B] int32, terminated [B] bool, truncated [B] bool, info)``
    with ``info["n_updates"]`` (node updates per env) and ``info["capped"]``.
    ``auto_reset`` resets envs that ended (SB3 VecEnv semantics); the reference
    env itself never resets on its own.
    """

    def __init__(self, network, attractors, n_envs: int, horizon: int = 100, device: int = 0, seed: int = 0,
                 env_id_base: int = 0, update_cap: int = 1 << 20, auto_reset: bool = False):
        net = network if isinstance(network, Net) else Net(network)
        self.net = net
        self.num_envs = int(n_envs)
        self.N = net.n_nodes
        self.cfg = EnvConfig(net, attractors, horizon=horizon)
        self.batch = PBNBatch(net, n_envs, device=device, env_id_base=env_id_base, seed=seed)
        self.update_cap = int(update_cap)
        self.auto_reset = auto_reset

    def reset(self, mask=None) -> np.ndarray:
        self.batch.env_reset(self.cfg, mask)
        return self.batch.get_bits()

    def step(self, actions):
        a = np.asarray(actions)
        if a.ndim == 1:
            a = a[:, None]
        obs, rew, flags, nup = self.batch.env_step_multi(self.cfg, a, offset=1, dedup=True,
                                                         update_cap=self.update_cap)
        term = (flags & L.FLAG_TERMINATED) != 0
        trunc = (flags & L.FLAG_TRUNCATED) != 0
        info = {"n_updates": nup, "capped": (flags & L.FLAG_CAPPED) != 0, "obs_words": obs}
        if self.auto_reset and (term | trunc).any():
            self.batch.env_reset(self.cfg, (term | trunc).astype(np.uint8))
        return unpack_bits(obs, self.N), rew, term, trunc, info


class PBNTargetMultiEnv:
    """Single-env mirror of ``PBNTargetMultiEnv`` with ``BittnerMulti7`` attractor handling."""

    def __init__(self, network, attractors, horizon: int = 100, device: int = 0, seed: int = 0,
                 update_cap: int = 1 << 20, name: Optional[str] = None):
        if not isinstance(network, PredictorNetwork):
            network = load_network(network)
        self.network = network
        self.name = name or network.name
        self._v = VecPBNTargetMultiEnv(network, attractors, 1, horizon=horizon, device=device, seed=seed,
                                       update_cap=update_cap)
        self.all_attractors = self._v.cfg.attractors
        self.horizon = horizon
        self.target = self.all_attractors[-1]
        self.n_steps = 0

    @property
    def graph_state(self) -> tuple:
        return tuple(int(x) for x in self._v.batch.get_bits()[0])

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):  # :227-259
        if options is not None and "state" in options:
            bits = np.array([int(x) for x in options["state"]], dtype=np.uint8)
            self._v.batch.set_bits(bits[None])
            self._v.batch.set_n_steps(np.zeros(1, np.int64))
        else:
            self._v.reset()
        self.n_steps = 0
        obs = self.graph_state
        tgt = tuple(x if x != "*" else 0 for x in self.target[0])
        info = {"observation_idx": state_to_idx(obs), "observation_dict": obs}
        return (obs, tgt), info

    def step(self, actions):  # :119-154
        dedup = not isinstance(actions, list)
        if hasattr(actions, "detach"):
            actions = actions.detach().cpu().numpy()
        a = np.asarray(actions, dtype=np.int32).reshape(1, -1)
        b = self._v.batch
        obs, rew, flags, nup = b.env_step_multi(self._v.cfg, a, offset=1, dedup=dedup,
                                                update_cap=self._v.update_cap)
        self.n_steps += 1
        if flags[0] & L.FLAG_CAPPED:
            raise RuntimeError(f"update cap ({self._v.update_cap}) reached before an attracting state")
        o = tuple(int(x) for x in unpack_bits(obs, self.network.n_nodes)[0])
        info = {"observation_idx": state_to_idx(o), "observation_dict": o, "n_updates": int(nup[0])}
        return o, int(rew[0]), bool(flags[0] & L.FLAG_TERMINATED), bool(flags[0] & L.FLAG_TRUNCATED), info


class PBNEnv:
    """``PBNEnv`` step conventions (pbn_env.py:125-188) over the truth-table engine.

    ``all_attractors``: list of sets of state tuples (the reference derives them
    from the full STG at construction, pbn_env.py:54 -- out of scope here, so
    they are passed in). ``target_nodes``: set of target state tuples.
    """

    def __init__(self, PBN_data, all_attractors, target_nodes, device: int = 0, seed: int = 0):
        self.PBN = PBN(PBN_data, device=device, seed=seed)
        self.all_attractors = [set(tuple(int(v) for v in s) for s in a) for a in all_attractors]
        self.target_nodes = set(tuple(int(v) for v in s) for s in target_nodes)
        for attractor in self.all_attractors:  # pbn_env.py:57-59
            if self.target_nodes & attractor:
                self.target_nodes = self.target_nodes.union(attractor)
        self.attracting_states = set.union(*self.all_attractors)

    def reset(self, seed=None, options=None):
        state = options["state"] if options is not None and "state" in options else None
        if state is None:
            attr = sorted(self.all_attractors[0])
            state = attr[0]
        obs = self.PBN.reset(state)
        return obs, {"observation_idx": state_to_idx(obs.astype(int))}

    def step(self, action: int):
        if not (0 <= int(action) < self.PBN.N):
            raise Exception(f"Invalid action {action}, not in action space.")  # pbn_env.py:138-139
        if action != 0:
            self.PBN.flip(int(action))  # flips node `action`, not action-1 (pbn_env.py:141-142)
        self.PBN.step()
        obs = self.PBN.state
        t = tuple(int(x) for x in obs)
        reward, terminated = 0, False
        if t in self.target_nodes:  # pbn_env.py:171-183
            reward += 20
            terminated = True
        else:
            reward -= 4
            if action != 0:
                reward -= 1
        return obs, reward, terminated, False, {"observation_idx": state_to_idx(t)}


__all__ = ["Graph", "PBN", "PBNTargetMultiEnv", "VecPBNTargetMultiEnv", "PBNEnv", "state_to_idx", "pack_bits"]
