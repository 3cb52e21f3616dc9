"""CPU model of the exact parallel form of a sequential fp32 sum of SIGNED terms (csrc/gdd_colsum.hip,
r05): numpy's column sums of a C-contiguous float32 matrix (`X.mean(axis=0)`, `X.var(axis=0)` in
KMeans.fit's centring and _tolerance, sklearn/cluster/_kmeans.py:1476-1487 and :279-288) are one
sequential fp32 chain per column. While the running sum s stays in one signed binade (sign sigma,
|s| in [2^e, 2^(e+1))), s = S*u with u = 2^(e-23) and S a signed integer; a term t moves S by
round(t/u), ties to the even S — an advance that depends only on S's parity. A run of terms is then a
two-state transducer (per start parity: the advance, and the least and greatest partial advance), runs
compose associatively, and the composed run applies exactly when its path stays strictly inside the
binade (one unit of margin at the edge nearer zero, where the grid halves). The model follows the
kernels' arithmetic (candidate binades from an fp64 prefix, per-segment transducers, a resolve that
re-walks a segment whose transducer does not apply) and must give the sequential sum bit for bit."""
import numpy as np
import pytest
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from signed_chain import (IDENT, applies, binade, compose, guess, run_tr, seq_sum,  # noqa: E402,F401
                          segmented, term_tr, walk)


def cases():
    rng = np.random.default_rng(7)
    yield "zero-mean", rng.standard_normal(3000).astype(np.float32)
    yield "drift", (rng.standard_normal(3000) + 0.3).astype(np.float32)
    yield "negative drift", (rng.standard_normal(3000) - 2.0).astype(np.float32)
    yield "ties", (rng.integers(-4, 5, 3000) * 0.5 + 2 ** 23).astype(np.float32)
    yield "integers past 2^24", rng.integers(-3, 9, 3000).astype(np.float32) * np.float32(4096.0)
    yield "cancel to zero", np.concatenate([np.full(500, 0.1, np.float32), np.full(500, -0.1, np.float32),
                                            rng.standard_normal(1000).astype(np.float32)])
    yield "subnormals", (rng.standard_normal(2000) * 1e-40).astype(np.float32)
    yield "decades", (rng.standard_normal(3000) * 10.0 ** rng.integers(-12, 12, 3000)).astype(np.float32)
    yield "zeros and signed zeros", np.array([0.0, -0.0] * 300 + [1e-3, -1e-3] * 200, np.float32)
    x = rng.standard_normal(2000).astype(np.float32)
    x[777] = np.inf
    yield "infinity", x
    x = rng.standard_normal(2000).astype(np.float32)
    x[1500] = np.nan
    yield "nan", x


@pytest.mark.parametrize("name,t", list(cases()), ids=[c[0] for c in cases()])
@pytest.mark.parametrize("L", [64, 256])
def test_segmented_matches_sequential(name, t, L):
    ref = seq_sum(t)
    got, rewalks = segmented(t, L)
    assert (np.isnan(ref) and np.isnan(got)) or ref.view(np.uint32) == got.view(np.uint32), (name, ref, got)


def test_walk_matches_sequential_term_by_term():
    rng = np.random.default_rng(3)
    for _ in range(20):
        t = (rng.standard_normal(400) * 10.0 ** rng.integers(-3, 4)).astype(np.float32)
        s0 = np.float32(rng.standard_normal() * 10.0 ** rng.integers(-3, 4))
        assert seq_sum(t, s0).view(np.uint32) == walk(t, s0).view(np.uint32)


def test_drifting_sums_rarely_rewalk():
    t = (np.random.default_rng(5).standard_normal(20000) + 1.0).astype(np.float32)
    s, rewalks = segmented(t, 256)
    assert s.view(np.uint32) == seq_sum(t).view(np.uint32)
    assert rewalks <= 20  # the binade changes (~log2 of the sum's range), not every segment
