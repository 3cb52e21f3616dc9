"""CPU model of the rank-split Lloyd M-step fold (tests/signed_chain.py
rank_split_fold): one (cluster, column) chain of sklearn's M-step (_k_means_lloyd.pyx:140-152, a
sequential fp32 sum of the members' values in sample order) split over R ranks' contiguous row
blocks. Each rank ships per segment either two-binade transducer records or — where its fp64 path
nears a binade edge — the raw terms; the resolver composes them in rank order from +0. The result
must be the sequential sum bit for bit whenever no fallback is reported, over ties, cancellation to
zero, binade crossings, signed zeros, subnormals, decades of magnitude and non-finite terms, at
1–4 ranks with uneven and empty blocks."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from signed_chain import rank_split_fold, seq_sum  # noqa: E402


def cases():
    rng = np.random.default_rng(11)
    yield "zero-mean", rng.standard_normal(4000).astype(np.float32)
    yield "drift", (rng.standard_normal(4000) + 0.3).astype(np.float32)
    yield "negative drift", (rng.standard_normal(4000) - 2.0).astype(np.float32)
    yield "ties", (rng.integers(-4, 5, 3000) * 0.5 + 2 ** 23).astype(np.float32)
    yield "cancel to zero", np.concatenate([np.full(700, 0.1, np.float32), np.full(700, -0.1, np.float32),
                                            rng.standard_normal(1200).astype(np.float32)])
    yield "subnormals", (rng.standard_normal(2000) * 1e-40).astype(np.float32)
    yield "decades", (rng.standard_normal(3000) * 10.0 ** rng.integers(-12, 12, 3000)).astype(np.float32)
    yield "signed zeros", np.array([0.0, -0.0] * 300 + [1e-3, -1e-3] * 200, np.float32)
    yield "logit-like cluster column", (rng.standard_normal(6000) * 0.8 + 1.7).astype(np.float32)
    x = rng.standard_normal(2000).astype(np.float32)
    x[1777] = np.inf
    yield "infinity", x
    x = rng.standard_normal(2000).astype(np.float32)
    x[333] = np.nan
    yield "nan", x


def splits(m, R, rng):
    if R == 1:
        return [0, m]
    cuts = np.sort(rng.integers(0, m + 1, R - 1))
    return [0, *cuts.tolist(), m]


@pytest.mark.parametrize("name,t", list(cases()), ids=[c[0] for c in cases()])
@pytest.mark.parametrize("R", [1, 2, 3, 4])
@pytest.mark.parametrize("L", [64, 256])
def test_rank_split_fold_matches_sequential(name, t, R, L):
    rng = np.random.default_rng(R * 7 + L)
    ref = seq_sum(t)
    for trial in range(2):
        cut = splits(len(t), R, rng) if trial else [len(t) * r // R for r in range(R + 1)]
        blocks = [t[cut[r]:cut[r + 1]] for r in range(R)]
        got, st = rank_split_fold(blocks, L)
        if got is None:  # a record did not apply: the fallback (labels all-gather) path runs instead
            assert st["fallback"]
            continue
        assert (np.isnan(ref) and np.isnan(got)) or ref.view(np.uint32) == got.view(np.uint32), (name, R, L)


def test_rank_split_fold_empty_blocks_and_fallback_rare():
    rng = np.random.default_rng(2)
    t = (rng.standard_normal(20000) * 0.8 + 1.7).astype(np.float32)
    blocks = [t[:0], t[:9000], t[9000:9000], t[9000:]]
    got, st = rank_split_fold(blocks, 256)
    assert not st["fallback"] and got.view(np.uint32) == seq_sum(t).view(np.uint32)
    assert st["raw"] <= st["records"] // 4  # most segments ship two records, not their terms
