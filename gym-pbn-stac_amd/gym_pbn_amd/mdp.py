"""Macro-action MDP wrappers over the truth-table engine.

Mirrors of ``gym_PBN/envs/pbcn_env.py``, ``common/pbcn.py``, ``sampled_data.py`` and
``self_triggering.py``, with the reference constructors. They are host-side loops
over ``PBN.step()`` (R4); every transition runs on the GPU through
:class:`gym_pbn_amd.envs.PBN`. Stochastic termination draws ``uniform(0, 1)`` from
the env's host ``random.Random`` (the reference uses the global ``random``, seeded by
``reset(seed)``). Reward rules and quirks are those of the reference at HEAD:

* ``PBNEnv._get_reward`` uses literal +20 / -4 / -1 (``pbn_env.py:171-181``);
* ``PBCNEnv._get_reward`` uses ``successful_reward`` and ``wrong_attractor_cost``
  times the number of attractors containing the state (``pbcn_env.py:48-58``);
* ``PBCN.step`` ignores the control input (``common/pbcn.py:51-66``), so
  ``apply_control`` only records it;
* the sampled-data PBN env flips ``action - 1`` (``sampled_data.py:62``) while
  ``PBNEnv`` flips ``action`` (``pbn_env.py:141-142``);
* ``PBCNEnv`` keeps the *unexpanded* ``goal_config["target_nodes"]`` (``pbcn_env.py:43``).

One deliberate difference: a ``(control, interval)`` tuple given to the PBCN
macro-action envs is used as is; the reference first calls ``np.isreal`` on it
(``sampled_data.py:140``), which numpy >= 1.24 rejects for a ragged tuple.
"""

from __future__ import annotations

from typing import Sequence, Tuple, Union

import numpy as np

from . import spaces
from .envs import PBN, PBNEnv
from .network import TruthTableNetwork


def booleanize(X: int, length: int) -> np.ndarray:  # gym_PBN/utils/__init__.py:4-12
    out = np.zeros(length, dtype=bool)
    for i in range(length):
        h = 2 ** (length - i - 1)
        if X >= h:
            X -= h
            out[i] = 1
    return out


class PBCN(PBN):
    """``common/pbcn.py`` ``PBCN``: the PBN plus M control nodes (``is_control``, :23-34).

    ``step`` is ``PBN.step`` (``pbcn.py:51-66`` updates ``randint(1, N-1)`` from the
    same draws); the control input is only recorded (the reference never reads it).
    """

    def __init__(self, PBN_data=None, logic_func_data=None, **kw):
        if PBN_data is None or len(PBN_data) == 0:
            from .io.logic import logic_funcs_to_pbn_data

            PBN_data = logic_funcs_to_pbn_data(*logic_func_data)
        super().__init__(network=TruthTableNetwork.from_pbn_data(PBN_data), **kw)
        self.M = sum(1 for nd in PBN_data if nd[3])
        self.control_state = np.zeros(self.M, dtype=bool)

    def apply_control(self, control: Sequence[Union[int, bool]]):  # pbcn.py:40-49
        if len(control) != self.M:
            raise ValueError(f"Control for {len(control)} control nodes provided, when there are {self.M} "
                             f"in the network.")
        self.control_state = np.array(control, dtype=bool)

    def reset(self, state=None):  # pbcn.py:68-70
        self.control_state = np.zeros(self.M, dtype=bool)
        return super().reset(state)


class PBNSampledDataEnv(PBNEnv):
    """``PBNSampledDataEnv.step((action, interval))`` (sampled_data.py:15-85)."""

    def __init__(self, render_mode="human", render_no_cache=False, PBN_data=None, logic_func_data=None, name=None,
                 goal_config=None, reward_config=None, gamma: float = 0.99, T: int = None, **kw):
        super().__init__(render_mode, render_no_cache, PBN_data, logic_func_data, name, goal_config, reward_config,
                         **kw)
        self.gamma = gamma
        self.T = T if T is not None else 2 ** self.PBN.N
        self.primitive_action_space = spaces.Discrete(self.PBN.N + 1)  # sampled_data.py:43-49
        self.interval_space = spaces.Discrete(self.T, start=1)
        self.action_space = spaces.Tuple((self.primitive_action_space, self.interval_space))
        self.discrete_action_space = spaces.Discrete(self.primitive_action_space.n * self.interval_space.n)

    def step(self, action: Tuple[int, int]):
        if not self.action_space.contains(action):  # :52-53
            raise Exception(f"Invalid action {action}, not in action space.")
        control_action, interval = action
        total_reward = 0
        for i in range(interval):
            if control_action != 0:
                self.PBN.flip(control_action - 1)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._get_reward(observation, control_action)
            total_reward += reward
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i, "observation_idx": self._state_to_idx(observation)}


class PBNSelfTriggeringEnv(PBNEnv):
    """``PBNSelfTriggeringEnv.step((action, prob))`` (self_triggering.py:15-92): repeat until
    ``uniform(0, 1) <= prob / 10`` or T steps, discounting rewards by gamma^i."""

    def __init__(self, render_mode="human", render_no_cache=False, PBN_data=None, logic_func_data=None, name=None,
                 goal_config=None, reward_config=None, gamma: float = 0.99, T: int = 5, **kw):
        super().__init__(render_mode, render_no_cache, PBN_data, logic_func_data, name, goal_config, reward_config,
                         **kw)
        self.gamma = gamma
        self.T = T
        self.primitive_action_space = spaces.Discrete(self.PBN.N + 1)  # self_triggering.py:44-49
        self.prob_space = spaces.Discrete(10, start=1)  # {0.1, ..., 1.0}
        self.action_space = spaces.Tuple((self.primitive_action_space, self.prob_space))
        self.discrete_action_space = spaces.Discrete(self.primitive_action_space.n * self.prob_space.n)
        self.successful_reward, self.wrong_attractor_cost, self.action_cost = 1, 0, 1  # :51-54

    def step(self, action: Tuple[int, int]):
        if not self.action_space.contains(action):  # :56-57
            raise Exception(f"Invalid action {action}, not in action space.")
        control_action, prob = action
        prob /= 10
        total_reward, i, end = 0, 0, False
        while not end:
            if control_action != 0:
                self.PBN.flip(control_action - 1)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._get_reward(observation, control_action)
            total_reward += (self.gamma ** i) * reward
            i += 1
            end = self._rng.uniform(0, 1) <= prob or i == self.T
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i, "observation_idx": self._state_to_idx(observation),
            "T": self.T}


class PBCNEnv(PBNEnv):
    """``PBCNEnv`` (pbcn_env.py): control nodes recorded, reward by attractor membership."""

    def __init__(self, render_mode="human", render_no_cache=False, PBN_data=None, logic_func_data=None, name=None,
                 goal_config=None, reward_config=None, **kw):
        super().__init__(render_mode, render_no_cache, PBN_data, logic_func_data, name, goal_config, reward_config,
                         **kw)
        self.PBN = PBCN(PBN_data, logic_func_data, device=kw.get("device", 0), seed=kw.get("seed", 0))
        self.target_nodes = goal_config["target_nodes"]  # pbcn_env.py:43 (unexpanded)
        self.observation_space = spaces.bool_multibinary(self.PBN.N)  # pbcn_env.py:41-45
        self.action_space = spaces.bool_multibinary(self.PBN.M)
        self.discrete_action_space = spaces.Discrete(2 ** self.PBN.M)

    @property
    def M(self) -> int:
        return self.PBN.M

    def getTargetIdx(self) -> int:  # pbcn_env.py:45-47
        return int(tuple(int(x) for x in self.PBN.state) in self.target_nodes)

    def _get_reward(self, observation):  # pbcn_env.py:49-60
        t = tuple(int(x) for x in observation)
        if t in self.target_nodes:
            return self.successful_reward, True, False
        matched = sum(t in a for a in self.all_attractors)
        return -self.wrong_attractor_cost * matched, False, False

    def step(self, action: int = 0):  # pbcn_env.py:62-74
        if action != 0:
            self.PBN.flip(action)
        self.PBN.step()
        observation = self.PBN.state
        reward, terminated, truncated = self._get_reward(observation)
        return observation, reward, terminated, truncated, {"observation_idx": self._state_to_idx(observation)}


def _discrete(action) -> bool:
    return not isinstance(action, (tuple, list)) and bool(np.isreal(action))


class PBCNSampledDataEnv(PBCNEnv):
    """``PBCNSampledDataEnv.step((control, interval) | int)`` (sampled_data.py:88-179)."""

    def __init__(self, render_mode="human", render_no_cache=False, PBN_data=None, logic_func_data=None, name=None,
                 goal_config=None, reward_config=None, gamma: float = 0.99, T: int = None, **kw):
        super().__init__(render_mode, render_no_cache, PBN_data, logic_func_data, name, goal_config, reward_config,
                         **kw)
        self.gamma = gamma
        self.T = T if T is not None else 2 ** self.PBN.N
        self.primitive_action_space = spaces.bool_multibinary(self.M)  # sampled_data.py:118-129
        self.interval_space = spaces.Discrete(self.T, start=1)
        self.action_space = spaces.Tuple((self.primitive_action_space, self.interval_space))
        self.discrete_action_space = spaces.Discrete((2 ** self.M) * self.interval_space.n)

    def _idx_to_macro_action(self, i: int):
        action = booleanize(i % (2 ** self.M), self.M).tolist()
        return action, i // (2 ** self.M) + 1

    def step(self, action):
        if action is None:
            raise Exception("You need to provide a macro action with either `macro_action` or "
                            "`macro_action_discrete`.")
        if _discrete(action):
            if not self.discrete_action_space.contains(action):  # :145-147
                raise Exception(f"Invalid action {action}, not in action space.")
            action = self._idx_to_macro_action(int(action))
        if not self.action_space.contains(action):  # :151-152
            raise Exception(f"Invalid action {action}, not in action space.")
        control_action, interval = action
        time_step_cost = 1
        total_reward, terminated_step = 0, None
        for i in range(interval):
            self.PBN.apply_control(control_action)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._get_reward(observation)
            reward -= time_step_cost
            if terminated_step is not None:  # penalise overshooting the attractor
                reward -= self.successful_reward
            elif terminated:
                terminated_step = i
            total_reward += reward
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i + 1,
            "observation_idx": self._state_to_idx(observation)}


class PBCNSelfTriggeringEnv(PBCNEnv):
    """``PBCNSelfTriggeringEnv`` (self_triggering.py:95-189): PBCN rewards, stochastic termination."""

    def __init__(self, render_mode="human", render_no_cache=False, PBN_data=None, logic_func_data=None, name=None,
                 goal_config=None, reward_config=None, gamma: float = 0.99, T: int = None, **kw):
        super().__init__(render_mode, render_no_cache, PBN_data, logic_func_data, name, goal_config, reward_config,
                         **kw)
        self.gamma = gamma
        self.T = T
        self.primitive_action_space = spaces.bool_multibinary(self.M)  # self_triggering.py:122-130
        self.prob_space = spaces.Discrete(10, start=1)
        self.action_space = spaces.Tuple((self.primitive_action_space, self.prob_space))
        self.discrete_action_space = spaces.Discrete((2 ** self.M) * self.prob_space.n)
        self.successful_reward, self.wrong_attractor_cost, self.action_cost = 1, 1, 1  # :135-138

    def _idx_to_macro_action(self, i: int):
        return booleanize(i % (2 ** self.M), self.M).tolist(), i // (2 ** self.M) + 1

    def step(self, action):
        if action is None:
            raise Exception("You need to provide a macro action with either `macro_action` or "
                            "`macro_action_discrete`.")
        if _discrete(action):
            if not self.discrete_action_space.contains(action):  # :150-152
                raise Exception(f"Invalid action {action}, not in action space.")
            action = self._idx_to_macro_action(int(action))
        if type(action[1]) is float:  # self_triggering.py:155-156
            action = (action[0], int(action[1] * 10))
        if not self.action_space.contains(action):  # :158-159
            raise Exception(f"Invalid action {action}, not in action space.")
        control_action, prob = action
        prob /= 10
        total_reward, i, end = 0, 0, False
        while not end:
            self.PBN.apply_control(control_action)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._get_reward(observation)
            reward -= 1  # time step cost (self_triggering.py:170)
            total_reward += (self.gamma ** i) * reward
            i += 1
            end = self._rng.uniform(0, 1) <= prob or i == self.T
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i, "observation_idx": self._state_to_idx(observation),
            "T": self.T}
