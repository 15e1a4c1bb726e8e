"""Macro-action MDP wrappers over the truth-table engine.

Mirrors of ``gym_PBN/envs/pbcn_env.py``, ``sampled_data.py`` and
``self_triggering.py``. They are host-side loops over ``PBN.step()`` (R4); every
transition runs on the GPU through :class:`gym_pbn_amd.envs.PBN`. Reward rules and
quirks are those of the reference at HEAD:

* ``PBNEnv._get_reward`` uses literal +20 / -4 / -1 (``pbn_env.py:171-181``);
* ``PBCNEnv._get_reward`` uses ``successful_reward`` and ``wrong_attractor_cost``
  times the number of attractors containing the state (``pbcn_env.py:48-58``);
* ``PBCN.step`` ignores the control input (``common/pbcn.py:51-66``), so
  ``apply_control`` only records it;
* the sampled-data PBN env flips ``action - 1`` (``sampled_data.py:62``) while
  ``PBNEnv`` flips ``action`` (``pbn_env.py:141-142``).
"""

from __future__ import annotations

import random
from typing import Sequence, Tuple, Union

import numpy as np

from .envs import PBNEnv, state_to_idx


def booleanize(X: int, length: int) -> np.ndarray:  # gym_PBN/utils/__init__.py:4-12
    out = np.zeros(length, dtype=bool)
    for i in range(length):
        h = 2 ** (length - i - 1)
        if X >= h:
            X -= h
            out[i] = 1
    return out


class PBNSampledDataEnv(PBNEnv):
    """``PBNSampledDataEnv.step((action, interval))`` (sampled_data.py:50-85)."""

    def __init__(self, PBN_data, all_attractors, target_nodes, T=None, gamma=0.99, **kw):
        super().__init__(PBN_data, all_attractors, target_nodes, **kw)
        self.gamma = gamma
        self.T = T if T is not None else 2 ** self.PBN.N

    def step(self, action: Tuple[int, int]):
        control_action, interval = action
        if not (0 <= control_action <= self.PBN.N and 1 <= interval <= self.T):
            raise Exception(f"Invalid action {action}, not in action space.")
        total_reward = 0
        for i in range(interval):
            if control_action != 0:
                self.PBN.flip(control_action - 1)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._reward(observation, control_action)
            total_reward += reward
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i,
            "observation_idx": state_to_idx(observation.astype(int))}

    def _reward(self, observation, action):
        t = tuple(int(x) for x in observation)
        if t in self.target_nodes:
            return 20, True, False
        return -4 - (1 if action != 0 else 0), False, False


class PBNSelfTriggeringEnv(PBNSampledDataEnv):
    """``PBNSelfTriggeringEnv.step((action, prob))`` (self_triggering.py:56-92): repeat until
    ``random.uniform(0, 1) <= prob / 10`` or T steps, discounting rewards by gamma^i."""

    def __init__(self, PBN_data, all_attractors, target_nodes, T=5, gamma=0.99, rng_seed=None, **kw):
        super().__init__(PBN_data, all_attractors, target_nodes, T=T, gamma=gamma, **kw)
        self._rng = random.Random(rng_seed)

    def step(self, action: Tuple[int, int]):
        control_action, prob = action
        if not (0 <= control_action <= self.PBN.N and 1 <= prob <= 10):
            raise Exception(f"Invalid action {action}, not in action space.")
        prob /= 10
        total_reward, i, end = 0.0, 0, False
        while not end:
            if control_action != 0:
                self.PBN.flip(control_action - 1)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._reward(observation, control_action)
            total_reward += (self.gamma ** i) * reward
            i += 1
            end = self._rng.uniform(0, 1) <= prob or i == self.T
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i,
            "observation_idx": state_to_idx(observation.astype(int)), "T": self.T}


class PBCNEnv(PBNEnv):
    """``PBCNEnv`` (pbcn_env.py): control nodes recorded, reward by attractor membership."""

    def __init__(self, PBN_data, all_attractors, target_nodes, successful_reward=10, wrong_attractor_cost=2,
                 **kw):
        super().__init__(PBN_data, all_attractors, target_nodes, **kw)
        self.M = sum(1 for nd in PBN_data if nd[3])  # pbcn.py:23-34
        self.control_state = np.zeros(self.M, dtype=bool)
        self.successful_reward = successful_reward
        self.wrong_attractor_cost = wrong_attractor_cost

    def apply_control(self, control: Sequence[Union[int, bool]]):  # pbcn.py:40-49
        if len(control) != self.M:
            raise ValueError(f"Control for {len(control)} control nodes provided, when there are {self.M} "
                             f"in the network.")
        self.control_state = np.array(control, dtype=bool)

    def _get_reward(self, observation):  # pbcn_env.py:48-58
        t = tuple(int(x) for x in observation)
        if t in self.target_nodes:
            return self.successful_reward, True, False
        matched = sum(t in a for a in self.all_attractors)
        return -self.wrong_attractor_cost * matched, False, False

    def step(self, action: int = 0):  # pbcn_env.py:60-70
        if action != 0:
            self.PBN.flip(action)
        self.PBN.step()
        observation = self.PBN.state
        reward, terminated, truncated = self._get_reward(observation)
        return observation, reward, terminated, truncated, {"observation_idx": state_to_idx(observation.astype(int))}


class PBCNSampledDataEnv(PBCNEnv):
    """``PBCNSampledDataEnv.step((control, interval) | int)`` (sampled_data.py:120-179)."""

    def __init__(self, PBN_data, all_attractors, target_nodes, T=None, gamma=0.99, **kw):
        super().__init__(PBN_data, all_attractors, target_nodes, **kw)
        self.gamma = gamma
        self.T = T if T is not None else 2 ** self.PBN.N

    def _idx_to_macro_action(self, i: int):
        action = booleanize(i % (2 ** self.M), self.M).tolist()
        return action, i // (2 ** self.M) + 1

    def step(self, action):
        if action is None:
            raise Exception("You need to provide a macro action with either `macro_action` or "
                            "`macro_action_discrete`.")
        if not isinstance(action, (tuple, list)) and np.isreal(action):
            action = self._idx_to_macro_action(int(action))
        control_action, interval = action
        time_step_cost = 1
        total_reward, terminated_step = 0, None
        for i in range(interval):
            self.apply_control(control_action)
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
            "observation_idx": state_to_idx(observation.astype(int))}


class PBCNSelfTriggeringEnv(PBCNSampledDataEnv):
    """``PBCNSelfTriggeringEnv`` (self_triggering.py:96-189): PBCN rewards, stochastic termination."""

    def __init__(self, PBN_data, all_attractors, target_nodes, T=None, gamma=0.99, rng_seed=None, **kw):
        super().__init__(PBN_data, all_attractors, target_nodes, T=T, gamma=gamma, successful_reward=1,
                         wrong_attractor_cost=1, **kw)
        self._rng = random.Random(rng_seed)

    def step(self, action):
        if not isinstance(action, (tuple, list)) and np.isreal(action):
            action = self._idx_to_macro_action(int(action))
        if type(action[1]) is float:  # self_triggering.py:155-156
            action = (action[0], int(action[1] * 10))
        control_action, prob = action
        prob /= 10
        total_reward, i, end = 0.0, 0, False
        while not end:
            self.apply_control(control_action)
            self.PBN.step()
            observation = self.PBN.state
            reward, terminated, truncated = self._get_reward(observation)
            reward -= 1  # time step cost (self_triggering.py:170)
            total_reward += (self.gamma ** i) * reward
            i += 1
            end = self._rng.uniform(0, 1) <= prob or (self.T is not None and i == self.T)
        return observation, total_reward, terminated, truncated, {
            "control_action": control_action, "interval": i,
            "observation_idx": state_to_idx(observation.astype(int)), "T": self.T}
