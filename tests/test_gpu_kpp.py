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


def force(monkeypatch, *tokens):
    """GDD_FORCE (gdd_common.hpp): force the listed k-means++ paths for the next calls."""
    if tokens:
        monkeypatch.setenv("GDD_FORCE", ",".join(tokens))
    else:
        monkeypatch.delenv("GDD_FORCE", raising=False)


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
    (3706, 64, 371, None, None),  # ML-1M items (recsys SVD dim 64): the 64-slot distance table
    (3000, 57, 120, 5, None),     # a table chain with 7 zero slots, duplicates
    (4096, 64, 60, None, None),
    (6040, 64, 200, None, None),  # ML-1M users' shape: multi-block rounds over the n x n table
    (9001, 49, 100, 5, None),     # three blocks, duplicates
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
    """The two-launch rounds (the single-block path for rows wider than 512 features or more than 256
    distance workgroups; GDD_FORCE=kpp_two_launch) give the same seeding as the fused ones."""
    n, dim, k = 3000, 40, 90
    X = np.ascontiguousarray(synth.blobs(n, dim, 20, seed=9), np.float32)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(3))
    force(monkeypatch, "kpp_two_launch", "kpp_no_table")
    ops = _Ops("cuda", n, k, dim)
    c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(3))
    assert np.array_equal(idx.cpu().numpy(), idx_ref)
    assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


@pytest.mark.parametrize("n,dim,k", [(3000, 40, 454), (2708, 7, 70), (4096, 48, 40), (1999, 20, 100),
                                     (4095, 3, 1000), (37, 5, 16),
                                     # an even number of rounds: the last launch is a pair
                                     (3000, 40, 455), (2708, 7, 71), (1999, 20, 17), (37, 5, 17),
                                     (4095, 3, 1097),  # T = 9: one round per launch
                                     (3706, 64, 371), (2000, 49, 101)])  # the 64-slot table
def test_kmeans_plusplus_round_forms(monkeypatch, n, dim, k):
    """Every single-block round form gives the oracle's seeding, bit for bit: two rounds per launch
    over the distance table (default for plain-chain plans, dim <= 64, k >= 16, T <= 8; the two
    folds overlapped, or one after the other with GDD_FORCE=kpp_pair_serial), one round
    per launch over the table (the default for T > 8; GDD_FORCE=kpp_single_round), and the fused
    distance + fold rounds (the default for k < 16; GDD_FORCE=kpp_no_table)."""
    X = np.ascontiguousarray(synth.blobs(n, dim, max(2, k // 4), seed=n + dim + 1), np.float32)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(15))
    for toks in ((), ("kpp_pair_serial",), ("kpp_single_round",), ("kpp_no_table",)):
        force(monkeypatch, *toks)
        ops = _Ops("cuda", n, k, dim)
        c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(15))
        assert np.array_equal(idx.cpu().numpy(), idx_ref), toks
        assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref)), toks


# ---- the cumulative potential: numpy's left-to-right fp64 cumsum, exactly ---------------------------
def adversarial_points(n):
    """1-D points whose distances to the first centre (x = 0, index 0) are [0, 1, s, ..., s, 1, 1]
    with s = 2^-58: numpy's sequential fp64 cumsum absorbs every s into the leading 1, while any
    blocked evaluation adds the s's together first and climbs past 1 + 2^-52 (kernel prefix trees)."""
    X = np.full((n, 1), 2.0 ** -29, np.float32)
    X[0], X[1], X[n - 2], X[n - 1] = 0.0, -1.0, -1.0, 1.0
    return X


def adversarial_uniforms(k, T, rnd):
    """Round `rnd`'s trial 0 draws r = u * pot = 1 + 2^-50 (pot = 3 in round 1; 2 in round 2 once
    the point +1 is a centre): numpy's index is the second -1 point (n - 2); a blocked prefix says
    an s entry. The round's other trials draw the first -1 point (index 1, the same potential), so
    numpy's seeding takes index n - 2 (trial 0 wins the tie) and a blocked one index 1. Round 1's
    draws before an adversarial round 2 all pick the +1 point; the later rounds are ordinary."""
    u = np.random.RandomState(k + T).uniform(size=(k - 1, T))
    u[0, :] = 0.9999
    u[rnd - 1, :] = 0.25  # r < 1: the first -1 point (index 1), a tie with numpy's pick that trial 0 wins
    u[rnd - 1, 0] = (1.0 + 2.0 ** -50) / (3.0 if rnd == 1 else 2.0)
    return u.ravel()


def _kpp_dev(X, k, T, first, u, w=None):
    lib = _lib.device_lib()
    n, dim = X.shape
    Xd = torch.from_numpy(X).cuda()
    ud = torch.from_numpy(np.ascontiguousarray(u, np.float64)).cuda()
    wd = None if w is None else torch.from_numpy(w).cuda()
    centers = torch.empty((k, dim), dtype=torch.float32, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    ws = _lib.workspace(lib.gdd_kmeans_plusplus_ws_bytes(n, dim, T), Xd.device)
    _lib.check(lib.gdd_kmeans_plusplus(n, dim, Xd.data_ptr(), _lib.ptr(wd), k, T, first, ud.data_ptr(),
                                       centers.data_ptr(), idx.data_ptr(), ws.data_ptr(), ws.numel(),
                                       _lib.stream_ptr(Xd.device)))
    torch.cuda.synchronize()
    return centers.cpu().numpy(), idx.cpu().numpy()


# (n, forced paths): every search form — the pick count (round 0 of the single-block paths and the
# two-launch rounds), the fold's two-ballot search in the table pair / single rounds and the fused
# rounds, the multi-block round (per-(block, trial) and the split pick launch), k_kpp1_big's
# speculative draws and their regular fallback, in one round per launch and two (k_kpp1_big2, n <= 8192)
CUMSUM_FORMS = [
    (1000, ()), (4096, ()), (1000, ("kpp_single_round",)), (1000, ("kpp_no_table",)),
    (1000, ("kpp_no_table", "kpp_two_launch")), (4096, ("kpp_single_round",)),
    (1000, ("kpp_pair_serial",)), (6000, ()),
    (6000, ("kpp_single_round",)), (9000, ()),
    (9000, ("kpp_no_big1",)), (20000, ()), (20000, ("kpp_big1_max=32768",)), (530000, ()),
    (530000, ("kpp_no_split",)),
]


@pytest.mark.parametrize("rnd", [1, 2])
@pytest.mark.parametrize("n,env", CUMSUM_FORMS)
def test_kpp_cumsum_adversarial(monkeypatch, n, env, rnd):
    """A draw that lands between numpy's sequential cumulative potential and the kernels' blocked
    one. With the rounding check (default) and with the replay forced on every draw the seeding is
    numpy's; with the check disabled (GDD_KPP_EXACT=0) it is not — so the case is adversarial for
    that form and the check is what makes it exact."""
    k, T = 16, 4
    force(monkeypatch, "kpp_force_table", *env)  # the multi-block table rounds at k = 16 too
    X = adversarial_points(n)
    u = adversarial_uniforms(k, T, rnd)
    c_ref, idx_ref = O.kmeans_plusplus_draws(X, k, T, 0, u)
    assert idx_ref[rnd] == n - 2
    for mode in ("1", "2"):
        monkeypatch.setenv("GDD_KPP_EXACT", mode)
        c, idx = _kpp_dev(X, k, T, 0, u)
        assert np.array_equal(idx, idx_ref), (mode, idx[:4], idx_ref[:4])
        assert np.array_equal(bits(c), bits(c_ref)), mode
    monkeypatch.setenv("GDD_KPP_EXACT", "0")
    _, idx = _kpp_dev(X, k, T, 0, u)
    assert idx[rnd] != idx_ref[rnd], "the blocked prefix did not cross the threshold"


@pytest.mark.parametrize("n", [1000, 6000, 9000, 20000])
def test_kpp_cumsum_adversarial_weighted(monkeypatch, n):
    """The same with sample weights (w * closest in fp32, then the fp64 sum)."""
    force(monkeypatch, "kpp_big1_max=32768", "kpp_force_table")
    k, T = 16, 4
    X = adversarial_points(n)
    w = np.ones(n, np.float32)
    w[1] = 0.5
    w[n - 2] = 2.0
    u = adversarial_uniforms(k, T, 1)
    u[0] = (0.5 + 2.0 ** -50) / 3.5  # w * closest = [0, 0.5, s, ..., s, 2, 1]
    c_ref, idx_ref = O.kmeans_plusplus_draws(X, k, T, 0, u, w=w)
    assert idx_ref[1] == n - 2
    monkeypatch.setenv("GDD_KPP_EXACT", "1")
    c, idx = _kpp_dev(X, k, T, 0, u, w=w)
    assert np.array_equal(idx, idx_ref)
    assert np.array_equal(bits(c), bits(c_ref))


@pytest.mark.parametrize("n,dim,k", [(3000, 40, 454), (9000, 8, 60), (2708, 7, 70)])
def test_kpp_replay_every_draw(monkeypatch, n, dim, k):
    """GDD_KPP_EXACT=2 replays numpy's cumsum for every draw: the seeding must not change."""
    X = np.ascontiguousarray(synth.blobs(n, dim, max(2, k // 4), seed=n + dim + 5), np.float32)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(15))
    monkeypatch.setenv("GDD_KPP_EXACT", "2")
    c, idx = _Ops("cuda", n, k, dim).kmeans_plusplus(torch.from_numpy(X).cuda(), k,
                                                     np.random.RandomState(15))
    assert np.array_equal(idx.cpu().numpy(), idx_ref)
    assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


# ---- table rounds with one 1024-thread workgroup per trial (k_kpp1_big, 4096 < n <= 32768) ----------
@pytest.mark.parametrize("n,dim,k,oracle", [
    (4097, 64, 40, True), (6040, 64, 604, True),  # ML-1M users' shape, its k
    (8192, 40, 100, True), (8193, 33, 50, True),  # the 8- / 16-entry segment boundary
    (12003, 64, 120, True), (16384, 7, 30, True), (16385, 64, 25, False),
    (17730, 64, 1773, False),  # Ali-Display users' shape and k: T = 9
    (32768, 16, 40, False)])
def test_kmeans_plusplus_big_rounds(monkeypatch, n, dim, k, oracle):
    """k_kpp1_big (the default for table plans with 4096 < n <= 16384; two rounds per launch,
    k_kpp1_big2, up to n = 8192 with T <= 8) gives the seeding of the per-(block, trial) table rounds
    (the default above 16,384; GDD_FORCE=kpp_no_big1), of one round per launch (kpp_single_round)
    and, where the oracle is run, the oracle's — bit for bit, over the 8-, 16- and 32-entry segment
    forms, odd n (the sgemv_t tail), even and odd k (a trailing round alone) and T = 9."""
    X = synth.blobs(n, dim, max(2, k // 4), seed=n + dim + 3)
    X = np.ascontiguousarray(X - X.mean(axis=0), np.float32)
    # the 32-entry segments too (default limit 16,384); small k: the table although it does not pay
    force(monkeypatch, "kpp_big1_max=32768", "kpp_force_table")
    ops = _Ops("cuda", n, k, dim)
    Xd = torch.from_numpy(X).cuda()
    c, idx = ops.kmeans_plusplus(Xd, k, np.random.RandomState(42))
    force(monkeypatch, "kpp_big1_max=32768", "kpp_force_table", "kpp_no_big1")
    c2, idx2 = ops.kmeans_plusplus(Xd, k, np.random.RandomState(42))
    assert np.array_equal(idx.cpu().numpy(), idx2.cpu().numpy())
    assert np.array_equal(bits(c.cpu().numpy()), bits(c2.cpu().numpy()))
    # one round per launch against two (k_kpp1_big2: n <= 8192, T <= 8 — the default there)
    force(monkeypatch, "kpp_big1_max=32768", "kpp_force_table", "kpp_single_round")
    c3, idx3 = ops.kmeans_plusplus(Xd, k, np.random.RandomState(42))
    assert np.array_equal(idx.cpu().numpy(), idx3.cpu().numpy())
    assert np.array_equal(bits(c.cpu().numpy()), bits(c3.cpu().numpy()))
    if oracle:
        c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(42))
        assert np.array_equal(idx.cpu().numpy(), idx_ref)
        assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


@pytest.mark.parametrize("n", [9001, 6001])
def test_kmeans_plusplus_big_rounds_weighted_and_replayed(monkeypatch, n):
    """Sample weights (w * row in fp32 for the cumulative, the weighted sgemv_t lane chains) and
    every draw replayed (GDD_KPP_EXACT=2) on the one-workgroup-per-trial rounds (6,001 points: two
    rounds per launch, k_kpp1_big2)."""
    dim, k, T = 24, 40, 5
    force(monkeypatch, "kpp_force_table")
    X = np.ascontiguousarray(synth.blobs(n, dim, 10, seed=77), np.float32)
    w = np.random.default_rng(3).uniform(0.5, 2.0, n).astype(np.float32)
    u = np.random.RandomState(9).uniform(size=(k - 1) * T)
    c_ref, idx_ref = O.kmeans_plusplus_draws(X, k, T, 17, u, w=w)
    for mode in ("1", "2"):
        monkeypatch.setenv("GDD_KPP_EXACT", mode)
        c, idx = _kpp_dev(X, k, T, 17, u, w=w)
        assert np.array_equal(idx, idx_ref), mode
        assert np.array_equal(bits(c), bits(c_ref)), mode


@pytest.mark.parametrize("n,dim,k", [(16384, 64, 20), (32768, 16, 40)])
def test_kmeans_plusplus_small_k_skips_the_table(monkeypatch, n, dim, k):
    """with few centres the n x n table does not pay (its build costs more than the
    rounds it saves), so neither the workspace nor the fit builds it; the per-block rounds give the
    same seeding as the forced table rounds."""
    lib = _lib.device_lib()
    T = 2 + int(np.log(k))
    assert lib.gdd_kmeans_plusplus_ws_bytes_k(n, dim, T, k) < 4 * n * n // 4
    X = synth.blobs(n, dim, max(2, k // 4), seed=n + dim + 11)
    X = np.ascontiguousarray(X - X.mean(axis=0), np.float32)
    ops = _Ops("cuda", n, k, dim)
    Xd = torch.from_numpy(X).cuda()
    c, idx = ops.kmeans_plusplus(Xd, k, np.random.RandomState(5))
    force(monkeypatch, "kpp_force_table")
    c2, idx2 = ops.kmeans_plusplus(Xd, k, np.random.RandomState(5))
    assert np.array_equal(idx.cpu().numpy(), idx2.cpu().numpy())
    assert np.array_equal(bits(c.cpu().numpy()), bits(c2.cpu().numpy()))


def _hard_points(case, n, dim, seed):
    rng = np.random.default_rng(seed)
    if case == "integers":  # exact integer distances: the running sums pass 2^24, so ties are common
        return rng.integers(-300, 300, (n, dim)).astype(np.float32)
    X = synth.blobs(n, dim, 24, seed=seed)
    if case == "dupes":  # zero distances, long runs of them
        X[1::3] = X[0]
        X[n // 2:n // 2 + 400] = X[5]
    elif case == "range":  # twelve decades: crossings everywhere, tiny terms absorbed
        X *= (10.0 ** rng.uniform(-6, 6, (n, 1))).astype(np.float32)
    return np.ascontiguousarray(X, np.float32)


@pytest.mark.parametrize("case", ["blobs", "integers", "dupes", "range"])
@pytest.mark.parametrize("n,dim,k", [(3000, 40, 454), (2708, 7, 70), (1001, 5, 33), (6040, 64, 604),
                                     (5003, 33, 60), (4093, 3, 200), (3706, 64, 371)])
def test_kmeans_plusplus_hard_data(case, n, dim, k):
    """The n x n distance table (k_kpp_dmat_t's 4 x 4 register tiles), the table's pair and big
    rounds and the sgemv_t lane chains on data with exact ties (integer distances past 2^24), zero
    distances and twelve decades of magnitudes, 8- and 4-lane trials (T = 6 at the Cora shape), n % 4
    tails and dim 64 (the 64 KB tile): the oracle's seeding, bit for bit."""
    X = _hard_points(case, n, dim, n + dim + k)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(15))
    ops = _Ops("cuda", n, k, dim)
    c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(15))
    assert np.array_equal(idx.cpu().numpy(), idx_ref)
    assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


@pytest.mark.parametrize("case", ["blobs", "integers", "dupes", "range"])
@pytest.mark.parametrize("n,dim,k,toks", [(9001, 24, 200, ()), (12003, 7, 120, ()),
                                          (6040, 64, 604, ("kpp_no_big1",)),
                                          (9001, 24, 200, ("kpp_no_big1",)),
                                          (17730, 64, 300, ()),  # Ali-Display users' n: per-block rounds
                                          (8195, 5, 30, ("kpp_no_table",))])  # distances per round
def test_kmeans_plusplus_hard_data_multi_block(monkeypatch, case, n, dim, k, toks):
    """The multi-block forms on the same hard data: k_kpp1_big and the per-(block, trial) rounds
    (with and without the table) against the one-workgroup-per-trial table rounds (both compute every
    potential with the sequential lane chains), and against the oracle where it is quick."""
    X = _hard_points(case, n, dim, n + dim + k + 1)
    force(monkeypatch, "kpp_force_table", *toks)
    c, idx = _Ops("cuda", n, k, dim).kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(15))
    force(monkeypatch, "kpp_force_table", "kpp_big1_max=32768")
    c2, idx2 = _Ops("cuda", n, k, dim).kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(15))
    assert np.array_equal(idx.cpu().numpy(), idx2.cpu().numpy())
    assert np.array_equal(bits(c.cpu().numpy()), bits(c2.cpu().numpy()))
    if n * k <= 6040 * 604:
        c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(15))
        assert np.array_equal(idx.cpu().numpy(), idx_ref)
        assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


@pytest.mark.parametrize("n,dim,k,weighted", [(524289, 5, 12, False), (600001, 33, 20, True),
                                              (530000, 47, 9, False)])
def test_kmeans_plusplus_split_rounds_match_block_rounds(monkeypatch, n, dim, k, weighted):
    """The split rounds (k_kpp_dists: every trial's distances per 4096-point block, the feature rows
    by LDS-DMA through a ring, r06) against the per-(block, trial) rounds (GDD_FORCE=kpp_no_split),
    bit for bit: odd n (the last block's short tail and the XT row padding), dims below and above the
    ring depth, sample weights."""
    rng = np.random.default_rng(n + dim)
    X = np.ascontiguousarray(rng.standard_normal((n, dim)), np.float32)
    w = rng.uniform(0.5, 2.0, n).astype(np.float32) if weighted else None
    T = 2 + int(np.log(k))
    u = np.random.RandomState(n).uniform(size=(k - 1) * T)
    c, idx = _kpp_dev(X, k, T, 7, u, w=w)
    force(monkeypatch, "kpp_no_split")
    c2, idx2 = _kpp_dev(X, k, T, 7, u, w=w)
    assert np.array_equal(idx, idx2)
    assert np.array_equal(bits(c), bits(c2))
