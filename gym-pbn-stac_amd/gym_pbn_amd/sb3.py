"""Stable-Baselines3 ``VecEnv`` face of the batched envs (the north star's "SB3 reset()/step()
surface": B envs stepped by one kernel launch behave as SB3's vectorised env).

SB3 conventions (``stable_baselines3/common/vec_env/base_vec_env.py``): ``reset() -> obs``;
``step_async(actions)`` + ``step_wait() -> (obs, rewards, dones, infos)``; an env that ends
is reset at once, ``obs`` holds its first observation of the next episode and
``infos[i]["terminal_observation"]`` the last one of the ended episode;
``infos[i]["TimeLimit.truncated"]`` marks an end by truncation. When stable_baselines3 is
importable the adapter subclasses its ``VecEnv``; otherwise it is a plain class with the same
methods. The wrapped env keeps ``auto_reset`` off: resets happen here, after the terminal
observations were taken.
"""

from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import spaces

try:
    from stable_baselines3.common.vec_env import VecEnv as _VecEnvBase  # type: ignore

    SB3 = True
except ImportError:  # pragma: no cover - this image has no stable_baselines3
    _VecEnvBase = object
    SB3 = False


class PBNVecEnv(_VecEnvBase):
    """SB3 ``VecEnv`` over :class:`~gym_pbn_amd.envs.VecPBNTargetMultiEnv` (actions: node + 1,
    0 = none; ``n_action_slots`` > 1 flips several nodes per step as the BDQ branches do) or
    :class:`~gym_pbn_amd.envs.VecPBNEnv` (actions: node index, ``pbn_env.py:141-142``)."""

    def __init__(self, venv, n_action_slots: int = 1):
        self.venv = venv
        venv.auto_reset = False
        N = venv.N
        observation_space = spaces.MultiBinary(N)
        if hasattr(venv, "cfg"):  # multi-flip env
            action_space = (spaces.Discrete(N + 1) if n_action_slots == 1
                            else spaces.MultiDiscrete([N + 1] * int(n_action_slots)))
        else:
            action_space = spaces.Discrete(N)
        self.n_action_slots = int(n_action_slots)
        if SB3:
            super().__init__(venv.num_envs, observation_space, action_space)
        else:
            self.num_envs = venv.num_envs
            self.observation_space = observation_space
            self.action_space = action_space
        self._actions = None

    # -- SB3 VecEnv API ----------------------------------------------------------------------
    def reset(self) -> np.ndarray:
        return np.asarray(self.venv.reset(), dtype=np.uint8)

    def step_async(self, actions) -> None:
        self._actions = np.asarray(actions)

    def step_wait(self):
        obs, reward, term, trunc, _ = self.venv.step(self._actions)
        obs = np.array(obs, dtype=np.uint8)
        done = np.asarray(term, bool) | np.asarray(trunc, bool)
        infos = [{} for _ in range(self.num_envs)]
        if done.any():
            for i in np.nonzero(done)[0]:
                infos[i]["terminal_observation"] = obs[i].copy()
                infos[i]["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
            fresh = np.asarray(self.venv.reset(done))
            obs[done] = fresh[done]
        return obs, np.asarray(reward, dtype=np.float32), done, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        self.venv.batch.close()

    def seed(self, seed: Optional[int] = None):
        """Transitions use the Philox stream fixed at construction (``seed=`` of the env)."""
        return [None] * self.num_envs

    def _indices(self, indices) -> Sequence[int]:
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name: str, indices=None):
        return [getattr(self.venv, attr_name) for _ in self._indices(indices)]

    def set_attr(self, attr_name: str, value, indices=None) -> None:
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name: str, *args, indices=None, **kwargs):
        raise NotImplementedError("the envs are one device batch; call methods on PBNVecEnv.venv")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_images(self):
        return [None] * self.num_envs


__all__ = ["PBNVecEnv", "SB3"]
