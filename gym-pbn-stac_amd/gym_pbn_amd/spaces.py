"""Action / observation spaces of the env classes (gymnasium 0.27 shapes, ``setup.py:28``).

The reference builds ``gymnasium.spaces`` objects in every env constructor
(``pbn_env.py:81-83``, ``pbn_target.py:90-93``, ``pbn_target_multi.py:56-59``,
``pbcn_env.py:41-45``, ``sampled_data.py:43-49,118-129``, ``self_triggering.py:44-48,122-127``)
and validates actions with ``action_space.contains`` (``pbn_env.py:138``,
``sampled_data.py:53,146,151``, ``self_triggering.py:57,...``). Agents read ``.n`` /
``.shape`` from them. When gymnasium is importable its classes are used as they are;
otherwise these stand-ins keep the same constructor arguments, attributes and
``contains`` rules (gymnasium 0.27 ``Discrete`` / ``MultiBinary`` / ``MultiDiscrete`` /
``Tuple``), plus ``sample`` / ``seed`` from a numpy Generator.
"""

from __future__ import annotations

from collections.abc import Sequence

import numpy as np

try:  # the real thing when present
    from gymnasium.spaces import Discrete, MultiBinary, MultiDiscrete, Space, Tuple  # type: ignore

    GYMNASIUM = True
except ImportError:  # pragma: no cover - exercised in this image (gymnasium absent)
    GYMNASIUM = False

    class Space:
        def __init__(self, shape=None, dtype=None, seed=None):
            self._shape = None if shape is None else tuple(int(s) for s in shape)
            self.dtype = None if dtype is None else np.dtype(dtype)
            self._np_random = None
            if seed is not None:
                self.seed(seed)

        @property
        def shape(self):
            return self._shape

        @property
        def np_random(self) -> np.random.Generator:
            if self._np_random is None:
                self.seed()
            return self._np_random

        def seed(self, seed=None):
            self._np_random = np.random.default_rng(seed)
            return [seed]

        def __contains__(self, x) -> bool:
            return self.contains(x)

    class Discrete(Space):
        """{start, ..., start + n - 1}; ``contains`` takes Python ints (bool included) and
        0-d integer numpy values only, as gymnasium's does."""

        def __init__(self, n: int, seed=None, start: int = 0):
            assert int(n) > 0, "n (counts) have to be positive"
            self.n = np.int64(n)
            self.start = np.int64(start)
            super().__init__((), np.int64, seed)

        def sample(self, mask=None) -> np.int64:
            return np.int64(self.start + self.np_random.integers(self.n))

        def contains(self, x) -> bool:
            if isinstance(x, int):
                v = np.int64(x)
            elif isinstance(x, (np.generic, np.ndarray)) and np.issubdtype(x.dtype, np.integer) and x.shape == ():
                v = np.int64(x)
            else:
                return False
            return bool(self.start <= v < self.start + self.n)

        def __repr__(self):
            return f"Discrete({self.n})" if self.start == 0 else f"Discrete({self.n}, start={self.start})"

        def __eq__(self, other):
            return isinstance(other, Discrete) and self.n == other.n and self.start == other.start

    class MultiBinary(Space):
        def __init__(self, n, seed=None):
            self.n = n
            shape = (int(n),) if np.isscalar(n) else tuple(int(v) for v in n)
            super().__init__(shape, np.int8, seed)

        def sample(self, mask=None) -> np.ndarray:
            return self.np_random.integers(0, 2, size=self.shape, dtype=self.dtype)

        def contains(self, x) -> bool:
            if isinstance(x, Sequence):
                x = np.array(x)
            return bool(isinstance(x, np.ndarray) and self.shape == x.shape and np.all((x == 0) | (x == 1)))

        def __repr__(self):
            return f"MultiBinary({self.n})"

        def __eq__(self, other):
            return isinstance(other, MultiBinary) and self.n == other.n

    class MultiDiscrete(Space):
        def __init__(self, nvec, dtype=np.int64, seed=None):
            self.nvec = np.array(nvec, dtype=dtype, copy=True)
            assert (self.nvec > 0).all(), "nvec (counts) have to be positive"
            super().__init__(self.nvec.shape, dtype, seed)

        def sample(self, mask=None) -> np.ndarray:
            return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

        def contains(self, x) -> bool:
            if isinstance(x, Sequence):
                x = np.array(x)
            return bool(isinstance(x, np.ndarray) and x.shape == self.shape and x.dtype != object
                        and np.all(0 <= x) and np.all(x < self.nvec))

        def __repr__(self):
            return f"MultiDiscrete({self.nvec})"

        def __eq__(self, other):
            return isinstance(other, MultiDiscrete) and np.all(self.nvec == other.nvec)

    class Tuple(Space):
        def __init__(self, spaces, seed=None):
            self.spaces = tuple(spaces)
            super().__init__(None, None, seed)

        def seed(self, seed=None):
            super().seed(seed)
            for i, s in enumerate(getattr(self, "spaces", ())):
                s.seed(None if seed is None else int(seed) + i)
            return [seed]

        def sample(self, mask=None):
            return tuple(s.sample() for s in self.spaces)

        def contains(self, x) -> bool:
            if isinstance(x, (list, np.ndarray)):
                x = tuple(x)
            return isinstance(x, tuple) and len(x) == len(self.spaces) and all(
                s.contains(p) for s, p in zip(self.spaces, x))

        def __getitem__(self, i):
            return self.spaces[i]

        def __len__(self):
            return len(self.spaces)

        def __repr__(self):
            return "Tuple(" + ", ".join(str(s) for s in self.spaces) + ")"

        def __eq__(self, other):
            return isinstance(other, Tuple) and self.spaces == other.spaces


def bool_multibinary(n: int) -> "MultiBinary":
    """``MultiBinary(n)`` with ``dtype = bool``, as the reference sets it (``pbn_env.py:81-82``)."""
    s = MultiBinary(n)
    s.dtype = bool if GYMNASIUM else np.dtype(bool)
    return s


__all__ = ["Discrete", "MultiBinary", "MultiDiscrete", "Tuple", "Space", "GYMNASIUM", "bool_multibinary"]
