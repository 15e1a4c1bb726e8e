"""Spaces of the env classes (gymnasium 0.27 semantics; stand-ins when gymnasium is absent).

The reference validates actions with ``action_space.contains`` (pbn_env.py:138,
sampled_data.py:53/146/151, self_triggering.py:57/150/158): ints (bool included) and 0-d
integer numpy values only, in ``[start, start + n)``; MultiBinary takes sequences /
arrays of 0/1 of the right shape; Tuple takes tuples (lists / arrays converted).
"""

import numpy as np
import pytest

from gym_pbn_amd import spaces


def test_discrete_contains_follows_gymnasium():
    d = spaces.Discrete(5)
    assert d.contains(0) and d.contains(4) and not d.contains(5) and not d.contains(-1)
    assert d.contains(True) and d.contains(np.int64(3)) and d.contains(np.array(2, dtype=np.int32))
    assert not d.contains(2.0) and not d.contains(np.float64(1)) and not d.contains("1")
    assert not d.contains(np.array([1])) and not d.contains([1])
    s = spaces.Discrete(10, start=1)
    assert s.n == 10 and s.start == 1 and s.contains(1) and s.contains(10) and not s.contains(0)
    assert 3 in d


def test_multibinary_and_multidiscrete():
    mb = spaces.MultiBinary(4)
    assert mb.shape == (4,) and mb.n == 4
    assert mb.contains([0, 1, 1, 0]) and mb.contains(np.array([True, False, True, True]))
    assert not mb.contains([0, 2, 1, 0]) and not mb.contains([0, 1, 1]) and not mb.contains(3)
    b = spaces.bool_multibinary(3)
    assert np.dtype(b.dtype) == np.dtype(bool)
    md = spaces.MultiDiscrete(7)  # PBNTargetMultiEnv: MultiDiscrete(N + 1), a scalar nvec
    assert md.shape == () and md.contains(np.array(6)) and not md.contains(np.array(7))


def test_tuple_and_sampling():
    t = spaces.Tuple((spaces.Discrete(29), spaces.Discrete(10, start=1)))
    assert t.contains((3, 10)) and t.contains([0, 1]) and not t.contains((3, 0)) and not t.contains((3,))
    assert not t.contains((3.0, 2))
    t.seed(5)
    draws = [t.sample() for _ in range(200)]
    assert all(t.contains(x) for x in draws)
    t2 = spaces.Tuple((spaces.Discrete(29), spaces.Discrete(10, start=1)))
    t2.seed(5)
    assert draws[:10] == [t2.sample() for _ in range(10)]
    mb = spaces.MultiBinary(8)
    mb.seed(1)
    assert all(mb.contains(mb.sample()) for _ in range(20))
    d = spaces.Discrete(3, start=-1)
    d.seed(0)
    assert {int(d.sample()) for _ in range(100)} == {-1, 0, 1}


@pytest.mark.skipif(spaces.GYMNASIUM, reason="stand-ins only when gymnasium is absent")
def test_stand_ins_compare_by_value():
    assert spaces.Discrete(4) == spaces.Discrete(4) and spaces.Discrete(4) != spaces.Discrete(4, start=1)
    assert repr(spaces.Discrete(10, start=1)) == "Discrete(10, start=1)"
