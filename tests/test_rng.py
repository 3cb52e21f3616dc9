"""The native loops' numpy-legacy RandomState restatement (csrc/gdd_rng.hpp) against numpy itself,
draw for draw, including the state left behind. Host-only library calls: runs on CPU."""
import ctypes

import numpy as np
import pytest

from gdd import _lib


@pytest.fixture(scope="module")
def lib():
    return _lib.load()


def _pair(seed):
    rs = np.random.RandomState(seed)
    return rs, _lib.MTState.from_random_state(rs)


def _same_state(rs, st):
    a = rs.get_state()
    return np.array_equal(a[1], np.ctypeslib.as_array(st.key)) and a[2] == st.pos


@pytest.mark.parametrize("low,high,count", [(0, 169343, 1000), (0, 3000, 5000), (0, 2, 64),
                                            (5, 6, 10), (0, 2**32, 100), (0, 2**40, 50),
                                            (-7, 1000003, 333)])
def test_randint(lib, low, high, count):
    rs, st = _pair(15)
    for _ in range(3):  # several calls, to cross state regenerations
        ref = rs.randint(low, high, count)
        out = np.empty(count, np.int64)
        assert lib.gdd_rng_randint(ctypes.addressof(st), low, high, count, out.ctypes.data) == 0
        assert np.array_equal(out, ref)
    assert _same_state(rs, st)


def test_random_sample_and_uniform(lib):
    rs, st = _pair(7)
    ref = np.concatenate([rs.uniform(size=8) for _ in range(100)])
    out = np.empty(800, np.float64)
    lib.gdd_rng_random_sample(ctypes.addressof(st), 800, out.ctypes.data)
    assert np.array_equal(out, ref)
    assert _same_state(rs, st)


@pytest.mark.parametrize("n,size", [(1000, 17), (1000, 1000), (7, 3), (1, 1)])
def test_choice_without_replacement(lib, n, size):
    rs, st = _pair(3)
    ref = rs.choice(n, replace=False, size=size)
    out = np.empty(n, np.int64)
    lib.gdd_rng_permutation(ctypes.addressof(st), n, out.ctypes.data)
    assert np.array_equal(out[:size], ref)
    assert _same_state(rs, st)


@pytest.mark.parametrize("n", [3000, 2708, 17730, 1])
def test_choice_unit_weights(lib, n):
    rs, st = _pair(11)
    w = np.ones(n, np.float32)
    ref = rs.choice(n, p=w / w.sum())
    out = np.empty(1, np.int64)
    lib.gdd_rng_choice_unit_weights(ctypes.addressof(st), n, out.ctypes.data)
    assert out[0] == ref
    assert _same_state(rs, st)


def test_state_round_trip():
    rs = np.random.RandomState(123)
    rs.randint(0, 10, 700)
    st = _lib.MTState.from_random_state(rs)
    rs2 = np.random.RandomState(0)
    st.to_random_state(rs2)
    assert np.array_equal(rs.randint(0, 1000, 50), rs2.randint(0, 1000, 50))
