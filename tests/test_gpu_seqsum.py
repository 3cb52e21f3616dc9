"""gdd_inertia / gdd_inertia_ws — the sequential fp32 sum evaluated in parallel — vs the oracle's
one-term-at-a-time loop (sklearn _inertia_dense with one OpenMP thread, _k_means_common.pyx:92-121),
bit for bit.

The cases aim at what the parallel form has to get right (gdd_seqsum.hip's header): exact
round-to-even ties, whose outcome depends on the running sum's parity (odd integers added to a sum
in [2^24, 2^25), halves to a sum in [2^23, 2^24)); sums that cross many binades (a first term far
below the rest, ascending terms); zero and subnormal terms; single huge terms; an overflow to inf;
NaN and negative terms (the one-term tail); sample weights; lengths around the chunk (4096) and
segment (2048) boundaries; more segments than one resolve window (> 1024).
"""
import numpy as np
import pytest
import torch

from golden_util import bits
from oracle import oracle as O

pytestmark = pytest.mark.gpu

from gdd import _lib  # noqa: E402


def _dev_sums(x, w=None):
    lib = _lib.device_lib()
    xd = torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()
    wd = None if w is None else torch.from_numpy(np.ascontiguousarray(w, np.float32)).cuda()
    n = x.shape[0]
    out = torch.full((2,), -1.0, dtype=torch.float32, device="cuda")
    s = _lib.stream_ptr(xd.device)
    _lib.check(lib.gdd_inertia(n, xd.data_ptr(), _lib.ptr(wd), out.data_ptr(), s))
    ws = _lib.workspace(lib.gdd_inertia_ws_bytes(n), xd.device)
    _lib.check(lib.gdd_inertia_ws(n, xd.data_ptr(), _lib.ptr(wd), out.data_ptr() + 4, ws.data_ptr(),
                                  ws.numel(), s))
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _case(name, n, rng):
    f32 = np.float32
    if name == "uniform":
        return rng.random(n).astype(f32) * 100
    if name == "sqdist":  # inertia-like terms: chi-square with 40 degrees of freedom
        return (rng.standard_normal((n, 40)).astype(f32) ** 2).sum(1).astype(f32)
    if name == "ties_odd":  # a sum in [2^24, 2^25): odd integers tie, parity decides
        x = rng.integers(0, 8, n).astype(f32)
        x[0] = 2.0 ** 24
        return x
    if name == "ties_half":  # halves onto a sum in [2^23, 2^24)
        x = (rng.integers(0, 8, n) + 0.5).astype(f32)
        x[0] = 2.0 ** 23
        return x
    if name == "ties_mixed":  # ties at several binades as the sum climbs
        return (rng.integers(0, 3, n) * f32(0.5) + f32(2.0 ** 22) * (rng.random(n) < 0.001)).astype(f32)
    if name == "heavy_tail":  # |N(0,1)|^8: terms spanning many binades
        return (np.abs(rng.standard_normal(n)) ** 8).astype(f32)
    if name == "ascending":  # sorted: binade crossings spread over the whole array
        return np.sort(rng.random(n).astype(f32) ** 4)
    if name == "tiny_first":  # a first term 2^-120 below the rest: ~130 binades in the first chunk
        x = rng.random(n).astype(f32) + f32(0.5)
        x[0] = f32(2.0 ** -120)
        return x
    if name == "subnormal":
        return (rng.integers(0, 5, n) * f32(2.0 ** -140)).astype(f32)
    if name == "zeros":
        return np.zeros(n, f32)
    if name == "ones":
        return np.ones(n, f32)
    if name == "big_term":  # one term near FLT_MAX in the middle, small ones around it
        x = rng.random(n).astype(f32)
        x[n // 2] = f32(3e38)
        return x
    if name == "overflow":  # the sum overflows to inf
        x = np.full(n, f32(1e38))
        return x
    if name == "nan":
        x = rng.random(n).astype(f32)
        x[(2 * n) // 3] = np.nan
        return x
    if name == "negative":
        x = rng.random(n).astype(f32)
        x[n // 3] = f32(-0.75)
        return x
    if name == "neg_zero":
        x = rng.random(n).astype(f32)
        x[::7] = f32(-0.0)
        return x
    raise KeyError(name)


NAMES = ["uniform", "sqdist", "ties_odd", "ties_half", "ties_mixed", "heavy_tail", "ascending",
         "tiny_first", "subnormal", "zeros", "ones", "big_term", "overflow", "nan", "negative",
         "neg_zero"]
SIZES = [1, 2, 63, 4095, 4096, 4097, 6145, 20000, 169343]


def _same(a, b):
    a, b = np.float32(a), np.float32(b)
    if np.isnan(a) or np.isnan(b):
        return bool(np.isnan(a) and np.isnan(b))
    return bits(np.array([a]))[0] == bits(np.array([b]))[0]


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("n", SIZES)
def test_inertia_parallel_equals_sequential(name, n):
    rng = np.random.default_rng(n * 31 + len(name))
    x = _case(name, n, rng)
    ref = O.inertia(x)
    assert np.float32(ref) == np.cumsum(x, dtype=np.float32)[-1] or np.isnan(ref)
    got = _dev_sums(x)
    assert _same(got[0], ref), (name, n, got[0], ref)
    assert _same(got[1], ref), (name, n, got[1], ref)


@pytest.mark.parametrize("name", ["sqdist", "ties_odd", "heavy_tail", "ascending", "tiny_first"])
def test_inertia_parallel_weighted(name):
    n = 50001
    rng = np.random.default_rng(7)
    x = _case(name, n, rng)
    w = rng.choice(np.array([0.0, 0.5, 1.0, 2.0, 3.0], np.float32), n)
    ref = O.inertia(x, w)
    got = _dev_sums(x, w)
    assert _same(got[0], ref) and _same(got[1], ref), (name, got, ref)


@pytest.mark.parametrize("n", [2_449_029, 20_000_001])
def test_inertia_parallel_long(n):
    """The products shape (599 segments of 4096) and more segments than one resolve window."""
    rng = np.random.default_rng(n)
    x = (rng.standard_normal((n,)).astype(np.float32) ** 2 * 47).astype(np.float32)
    x[:: 1009] = np.float32(0.5)  # some exact halves
    ref = O.inertia(x)
    got = _dev_sums(x)
    assert _same(got[0], ref) and _same(got[1], ref), (got, ref)
