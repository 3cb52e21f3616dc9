"""k-means++ on the device vs the oracle, bit for bit, across every summation-order regime.

The oracle's distance and potential orders are pinned element-wise against scikit-learn/numpy/
OpenBLAS (tests/test_oracle_golden.py::test_kmeans_plusplus_vs_sklearn_duplicates and the grid in
oracle/gdd_oracle.c's header). Here the device must reproduce them:
  * gdd_skl_sqdist over shapes that select each OpenBLAS kernel: ddot (one-row chunk), dgemv_t
    (first centre, incl. the threaded column split), the TN small-matrix dgemm (trial order
    remainders), the regular dgemm (K split above 384, the single-threaded edge kernels for
    >= 12 trials);
  * full seedings with duplicated rows (potential driven to ~0), the 4096-entry sgemv_t block
    boundaries, the n % 4 tail, a single trial (sdot potentials), dims 1 / 33 / 400.
"""
import numpy as np
import pytest
import torch

from golden_util import bits
from oracle import oracle as O

pytestmark = pytest.mark.gpu

from gdd import _lib, synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402


def _skl_sqdist_dev(C, X):
    lib = _lib.device_lib()
    Cd, Xd = torch.from_numpy(C).cuda(), torch.from_numpy(X).cuda()
    out = torch.empty((C.shape[0], X.shape[0]), dtype=torch.float32, device="cuda")
    _lib.check(lib.gdd_skl_sqdist(C.shape[0], Cd.data_ptr(), X.shape[0], X.shape[1], Xd.data_ptr(),
                                  out.data_ptr(), _lib.stream_ptr(Xd.device)))
    torch.cuda.synchronize()
    return out.cpu().numpy()


SQDIST_CASES = [
    # (n, dim, T)
    (1, 40, 1), (2, 40, 1), (1106, 40, 1), (1105 + 1, 40, 3),  # one-row chunks: ddot / gemv by row
    (5000, 40, 1), (3001, 128, 1), (12503, 64, 1), (4707, 128, 1),  # dgemv_t, threaded split
    (150, 33, 3), (150, 64, 7), (37, 40, 9), (20, 100, 13), (94, 130, 13),  # small-matrix TN
    (301, 400, 7), (601, 400, 2), (241, 385, 5), (200, 512, 3),  # K split
    (511, 48, 13), (511, 33, 12), (500, 40, 13), (509, 37, 16), (1105, 40, 13),  # edge kernels
    (3000, 40, 6), (169, 7, 4), (4099, 3, 2), (2000, 1, 5),  # the plain chain
]


@pytest.mark.parametrize("n,dim,T", SQDIST_CASES)
def test_skl_sqdist_every_mode(n, dim, T):
    rng = np.random.default_rng(n * 7 + dim + T)
    X = (rng.standard_normal((n, dim)) * 2).astype(np.float32)
    X[1::5] = X[0]
    C = X[rng.integers(0, n, T)]
    ref = O.skl_sqdist_upcast(C, X)
    got = _skl_sqdist_dev(C, X)
    assert np.array_equal(bits(got), bits(ref))


KPP_CASES = [
    # (n, dim, k, dup, trials)
    (50, 4, 50, 7, None),       # k = n with duplicates: the potential reaches 0
    (300, 33, 300, 7, None),    # small-matrix kernel, duplicates
    (611, 17, 80, 11, None),
    (4095, 8, 40, None, None),  # sgemv_t block boundaries and the n % 4 tail
    (4096, 8, 40, None, None),
    (4097, 8, 40, None, None),
    (8195, 5, 30, 3, None),
    (2000, 400, 20, None, None),  # K split
    (1500, 1, 25, None, None),
    (1000, 12, 30, None, 1),    # one trial: sdot potentials
    (3000, 40, 120, None, None),
    (3000, 48, 60, None, None),   # fused rounds: the 48-feature register chain, and one past it
    (3000, 49, 60, None, None),
    (700, 600, 30, None, None),   # rows wider than the fused kernel's 512: two launches per round
    (10, 3, 2, None, None),       # k = 2: a single round, no centre gather
    (2708, 7, 70, None, None),    # Cora shape: T = 6, two trials on the 4-lane sgemv_t kernel
]


@pytest.mark.parametrize("n,dim,k,dup,trials", KPP_CASES)
def test_kmeans_plusplus_orders(n, dim, k, dup, trials):
    X = synth.blobs(n, dim, max(2, k // 4), seed=n + dim)
    if dup:
        X[1::dup] = X[0]
    X = np.ascontiguousarray(X - X.mean(axis=0), np.float32)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(5), n_local_trials=trials)
    ops = _Ops("cuda", n, k, dim)
    c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(5),
                                 n_local_trials=trials)
    assert np.array_equal(idx.cpu().numpy(), idx_ref)
    assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


def test_kmeans_plusplus_two_launch_path(monkeypatch):
    """The two-launch rounds (GDD_KPP_TWO_LAUNCH) give the same seeding as the fused ones."""
    n, dim, k = 3000, 40, 90
    X = np.ascontiguousarray(synth.blobs(n, dim, 20, seed=9), np.float32)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(3))
    monkeypatch.setenv("GDD_KPP_TWO_LAUNCH", "1")
    monkeypatch.setenv("GDD_KPP_NO_TABLE", "1")
    ops = _Ops("cuda", n, k, dim)
    c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(3))
    assert np.array_equal(idx.cpu().numpy(), idx_ref)
    assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


@pytest.mark.parametrize("n,dim,k", [(3000, 40, 454), (2708, 7, 70), (4096, 48, 40), (1999, 20, 100),
                                     (4095, 3, 1000), (37, 5, 16),
                                     # an even number of rounds: the last launch is a pair
                                     (3000, 40, 455), (2708, 7, 71), (1999, 20, 17), (37, 5, 17),
                                     (4095, 3, 1097)])  # T = 9: one round per launch
def test_kmeans_plusplus_round_forms(monkeypatch, n, dim, k):
    """Every single-block round form gives the oracle's seeding, bit for bit: two rounds per launch
    over the distance table (default for plain-chain plans, dim <= 48, k >= 16, T <= 8), one round
    per launch over the table (GDD_KPP_SINGLE_ROUND), the one-workgroup persistent rounds over the
    table (GDD_KPP_PERSIST, T <= 8), and the fused distance + fold rounds (GDD_KPP_NO_TABLE)."""
    X = np.ascontiguousarray(synth.blobs(n, dim, max(2, k // 4), seed=n + dim + 1), np.float32)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(15))
    for var in (None, "GDD_KPP_SINGLE_ROUND", "GDD_KPP_PERSIST", "GDD_KPP_NO_TABLE"):
        if var:
            monkeypatch.setenv(var, "1")
        ops = _Ops("cuda", n, k, dim)
        c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(15))
        assert np.array_equal(idx.cpu().numpy(), idx_ref), var
        assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref)), var
