"""HIP k-means primitives and estimators vs the CPU oracle (bit-exact) — needs a gfx950 GPU."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import _lib, synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402


def force(monkeypatch, *tokens):
    """GDD_FORCE (gdd_common.hpp): force the listed paths for the next calls (none: the defaults)."""
    if tokens:
        monkeypatch.setenv("GDD_FORCE", ",".join(tokens))
    else:
        monkeypatch.delenv("GDD_FORCE", raising=False)


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("n,dim,k", [(1000, 40, 454), (5000, 7, 70), (777, 64, 1773),
                                     (4096, 41, 769), (300, 47, 196), (129, 3, 5), (64, 300, 33)])
def test_assign_bitexact(n, dim, k):
    X = synth.blobs(n, dim, max(2, k // 3), seed=n + dim)
    C = X[np.random.default_rng(1).choice(n, size=k, replace=k > n)] + 0.01
    lab_ref, sq_ref = O.assign(X, C)
    ops = _Ops("cuda", n, k, dim)
    Xd, Cd = torch.from_numpy(X).cuda(), torch.from_numpy(np.ascontiguousarray(C)).cuda()
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    sq = torch.empty(n, dtype=torch.float32, device="cuda")
    ops.assign(Xd, Cd, labels=lab, sq=sq)
    assert np.array_equal(ops.cn2.cpu().numpy().view(np.uint32), bits(O.row_norms(C)))
    assert np.array_equal(lab.cpu().numpy(), lab_ref)
    assert np.array_equal(bits(sq.cpu().numpy()), bits(sq_ref))
    assert float(ops.inertia(sq).item()) == O.lib().oracle_inertia(n, sq_ref, None)


def test_assign_ties_lowest_index():
    """Duplicate centres: the first (lowest-index) one must win (strict '<' scan)."""
    X = synth.blobs(500, 8, 4, seed=3)
    C = np.repeat(X[:10], 3, axis=0)  # every centre present three times
    lab_ref, _ = O.assign(X, C)
    ops = _Ops("cuda", 500, C.shape[0], 8)
    lab = torch.empty(500, dtype=torch.int32, device="cuda")
    ops.assign(torch.from_numpy(X).cuda(), torch.from_numpy(C).cuda(), labels=lab)
    assert np.array_equal(lab.cpu().numpy(), lab_ref)
    assert (lab_ref % 3 == 0).all()


def test_gathered_rows():
    X = synth.blobs(4000, 40, 30, seed=5)
    rows = np.random.default_rng(2).integers(0, 4000, 1000)
    C = X[:50].copy()
    lab_ref, sq_ref = O.assign(X, C, rows=rows)
    ops = _Ops("cuda", 1000, 50, 40)
    lab = torch.empty(1000, dtype=torch.int32, device="cuda")
    sq = torch.empty(1000, dtype=torch.float32, device="cuda")
    ops.assign(torch.from_numpy(X).cuda(), torch.from_numpy(C).cuda(),
               rows=torch.from_numpy(rows).cuda(), labels=lab, sq=sq)
    assert np.array_equal(lab.cpu().numpy(), lab_ref)
    assert np.array_equal(bits(sq.cpu().numpy()), bits(sq_ref))


@pytest.mark.parametrize("n,dim,k", [(3000, 40, 454), (2708, 7, 70), (5000, 64, 300)])
def test_kmeans_plusplus_bitexact(n, dim, k):
    X = synth.blobs(n, dim, max(2, k // 4), seed=11)
    c_ref, idx_ref = O.kmeans_plusplus(X, k, np.random.RandomState(15))
    ops = _Ops("cuda", n, k, dim)
    c, idx = ops.kmeans_plusplus(torch.from_numpy(X).cuda(), k, np.random.RandomState(15))
    assert np.array_equal(idx.cpu().numpy(), idx_ref)
    assert np.array_equal(bits(c.cpu().numpy()), bits(c_ref))


def test_minibatch_update_bitexact():
    rng = np.random.default_rng(4)
    X = synth.blobs(3000, 40, 20, seed=4)
    k = 60
    C = X[:k].copy()
    W = rng.integers(0, 5, k).astype(np.float32)
    rows = rng.integers(0, 3000, 1000)
    lab = rng.integers(0, k, 1000).astype(np.int32)
    W_ref = W.copy()
    C_ref = O.minibatch_update(X[rows], lab, C, W_ref)
    lib = _lib.device_lib()
    Xd = torch.from_numpy(X).cuda()
    Cd = torch.from_numpy(C).cuda()
    Cn = torch.empty_like(Cd)
    Wd = torch.from_numpy(W).cuda()
    ws = _lib.workspace(lib.gdd_minibatch_update_ws_bytes(1000, k), "cuda")
    rows_d = torch.from_numpy(rows).cuda()  # keep the device buffers alive across the launch
    lab_d = torch.from_numpy(lab).cuda()
    _lib.check(lib.gdd_minibatch_update(1000, 40, Xd.data_ptr(), rows_d.data_ptr(), None,
                                        lab_d.data_ptr(), k, Cd.data_ptr(), Cn.data_ptr(),
                                        Wd.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_ptr()))
    assert np.array_equal(bits(Cn.cpu().numpy()), bits(C_ref))
    assert np.array_equal(bits(Wd.cpu().numpy()), bits(W_ref))


@pytest.mark.parametrize("n,dim,k,bs", [(5000, 40, 50, 1000), (20000, 41, 300, 1000),
                                        (3000, 16, 700, 256)])
def test_minibatch_kmeans_bitexact(n, dim, k, bs):
    X = synth.blobs(n, dim, k, seed=7)
    ref = O.minibatch_kmeans(X, k, random_state=15, batch_size=bs)
    m = gdd.MiniBatchKMeans(n_clusters=k, random_state=15, batch_size=bs).fit(X)
    assert m.n_steps_ == ref["n_steps_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))
    assert m.inertia_ == ref["inertia_"]


@pytest.mark.parametrize("n,dim,k,n_init", [(2708, 7, 70, "auto"), (2000, 64, 200, "auto"),
                                            (1500, 10, 30, 3)])
def test_kmeans_lloyd_bitexact(n, dim, k, n_init):
    X = synth.blobs(n, dim, k // 2, seed=8)
    np.random.seed(15)
    ref = O.kmeans(X, k, n_init=n_init)
    np.random.seed(15)
    m = gdd.KMeans(n_clusters=k, n_init=n_init).fit(X)
    assert m.n_iter_ == ref["n_iter_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))
    assert m.inertia_ == ref["inertia_"]


def test_cluster_mean_and_argmax():
    n, d, k = 5000, 96, 40
    feat = synth.features(n, d, 3)
    lab = np.random.default_rng(3).integers(0, k, n).astype(np.int32)
    lab[lab == 17] = 18  # one empty cluster -> NaN row
    ref, cnt_ref = O.cluster_mean(feat, lab, k)
    out, cnt = gdd.cluster_mean(torch.from_numpy(feat).cuda(), lab, k)
    o = out.cpu().numpy()
    assert np.array_equal(cnt.cpu().numpy(), cnt_ref)
    assert np.isnan(o[17]).all() and np.isnan(ref[17]).all()
    m = np.arange(k) != 17
    assert np.array_equal(bits(o[m]), bits(ref[m]))
    ref0, _ = O.cluster_mean(feat, lab, k, empty_as_zero=True)
    out0, _ = gdd.cluster_mean(torch.from_numpy(feat).cuda(), lab, k, empty_as_zero=True)
    assert np.array_equal(bits(out0.cpu().numpy()), bits(ref0))
    C = synth.blobs(k, 40, 5, seed=2)
    assert np.array_equal(gdd.argmax_rows(torch.from_numpy(C).cuda()).cpu().numpy(), np.argmax(C, -1))


def test_minibatch_rng_state_after_fit():
    """A shared RandomState ends in the same state as under scikit-learn (early stop rewinds)."""
    X = synth.blobs(20000, 40, 100, seed=9)
    rs_ref, rs = np.random.RandomState(3), np.random.RandomState(3)
    ref = O.minibatch_kmeans(X, 100, random_state=rs_ref, batch_size=1000)
    m = gdd.MiniBatchKMeans(n_clusters=100, random_state=rs, batch_size=1000).fit(X)
    assert m.n_steps_ == ref["n_steps_"] < (100 * 20000) // 1000  # stopped early
    assert np.array_equal(m.labels_, ref["labels_"])
    s1, s2 = rs_ref.get_state(), rs.get_state()
    assert np.array_equal(s1[1], s2[1]) and s1[2] == s2[2]


def test_minibatch_tol_path():
    X = synth.blobs(5000, 16, 20, seed=2)
    ref = O.minibatch_kmeans(X, 20, random_state=1, batch_size=500, tol=1e-3)
    m = gdd.MiniBatchKMeans(n_clusters=20, random_state=1, batch_size=500, tol=1e-3).fit(X)
    # the centre-shift sum is an fp32 device reduction (numpy's pairwise order is not restated):
    # same result unless the stop test sits within rounding of the tolerance
    assert abs(m.n_steps_ - ref["n_steps_"]) <= 1


@pytest.mark.parametrize("n,dim,k,form", [(50000, 40, 454, ""), (3000, 7, 70, ""), (20000, 64, 200, ""),
                                          (1000, 47, 1, ""), (40000, 41, 769, ""), (40000, 41, 769, "bf16_w4"),
                                          (9000, 45, 100, "bf16_w8"), (9000, 45, 100, "bf16_v1"),
                                          (3000, 200, 30, ""), (33, 41, 5, ""), (95, 47, 3, ""),
                                          (64, 45, 40, "bf16_w8")])
def test_assign_bf16_within_rounding(n, dim, k, form, monkeypatch):
    # the bf16 distance variant: labels equal the exact fp32 ones except where two
    # centres' distances lie within the bf16 rounding of the dot products (2^-7 ||x|| ||c|| each).
    # form: the 4- or 8-wave block form of the r06 kernel, or the r03 kernel (gdd_bf16.hip)
    from gdd.kmeans import _Ops
    force(monkeypatch, *([form] if form else []))
    rng = np.random.default_rng(n + k)
    X = (rng.standard_normal((n, dim)) + rng.integers(0, 5, (n, 1))).astype(np.float32)
    C = X[rng.choice(n, k, replace=False)] + rng.standard_normal((k, dim)).astype(np.float32) * 0.1
    Xd, Cd = torch.from_numpy(X).cuda(), torch.from_numpy(C).cuda()
    ops = _Ops("cuda", n, k, dim)
    l32 = torch.empty(n, dtype=torch.int32, device="cuda")
    l16 = torch.empty(n, dtype=torch.int32, device="cuda")
    sq16 = torch.empty(n, dtype=torch.float32, device="cuda")
    ops.assign(Xd, Cd, labels=l32)
    ops.assign(Xd, Cd, labels=l16, sq=sq16, precision="bf16")
    a, b = l32.cpu().numpy(), l16.cpu().numpy()
    assert b.min() >= 0 and b.max() < k
    if n >= 1000:  # near-ties are common here (centres sit among the points); tiny n: the bound alone
        assert (a == b).mean() >= 0.95
    diff = np.nonzero(a != b)[0]
    X64, C64 = X.astype(np.float64), C.astype(np.float64)
    xn = np.linalg.norm(X64, axis=1)
    cn = np.linalg.norm(C64, axis=1)
    for i in diff[:2000]:
        di = ((X64[i] - C64) ** 2).sum(-1)
        bound = 2 * 2.0 ** -7 * xn[i] * (cn[a[i]] + cn[b[i]]) + 1e-3 * (1 + di[a[i]])
        assert di[b[i]] - di[a[i]] <= bound
    # sq_dist is the exact fp32 distance to the chosen centre (the fp32 finalize path)
    i = rng.integers(0, n, 64)
    ref = ((X[i] - C[b[i]]) ** 2).sum(-1)
    np.testing.assert_allclose(sq16.cpu().numpy()[i], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,dim,k,weighted", [(5000, 1, 7, False), (20000, 7, 70, True), (30000, 47, 5, False),
                                              (3000, 256, 9, True), (2000, 300, 4, False), (1500, 512, 3, True)])
def test_segment_sum_f32_sequential(n, dim, k, weighted):
    # Lloyd's M-step sums (sklearn lloyd_iter_chunked_dense, one thread): per cluster, sequential fp32
    # in sample order (sum + x*w); an empty cluster gives zeros
    rng = np.random.default_rng(dim)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    lab = rng.integers(0, k - 1, n).astype(np.int32)  # cluster k-1 stays empty
    w = (rng.random(n) + 0.5).astype(np.float32) if weighted else None
    lib = _lib.device_lib()
    Xd, ld = torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda()
    wd = torch.from_numpy(w).cuda() if weighted else None
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    offs = torch.empty(k + 1, dtype=torch.int32, device="cuda")
    ws = _lib.workspace(lib.gdd_group_ws_bytes(n, k), "cuda")
    st = _lib.stream_ptr("cuda")
    _lib.check(lib.gdd_group_by_label(n, ld.data_ptr(), k, perm.data_ptr(), offs.data_ptr(), ws.data_ptr(),
                                      ws.numel(), st))
    sums = torch.empty(k, dim, dtype=torch.float32, device="cuda")
    wsum = torch.empty(k, dtype=torch.float32, device="cuda")
    _lib.check(lib.gdd_segment_sum_f32(n, dim, Xd.data_ptr(), _lib.ptr(wd), perm.data_ptr(), offs.data_ptr(), k,
                                       sums.data_ptr(), wsum.data_ptr(), st))
    ref = np.zeros((k, dim), np.float32)
    wref = np.zeros(k, np.float32)
    for c in range(k):
        idx = np.nonzero(lab == c)[0]
        if idx.size == 0:
            continue
        terms = X[idx] * (w[idx][:, None] if weighted else np.float32(1.0))
        ref[c] = np.add.accumulate(terms.astype(np.float32), axis=0, dtype=np.float32)[-1]
        wt = w[idx] if weighted else np.ones(idx.size, np.float32)
        wref[c] = np.add.accumulate(wt, dtype=np.float32)[-1]
    assert np.array_equal(sums.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(wsum.cpu().numpy().view(np.uint32), wref.view(np.uint32))


@pytest.mark.parametrize("n,dim", [(1, 3), (1000, 7), (100000, 47), (20000, 64), (333, 5), (777, 300),
                                   (768, 5), (1536, 8), (831, 9), (63, 2), (64, 3), (65, 17),
                                   (2000, 600), (5, 1), (64, 1), (129, 1), (8192, 1), (30001, 1)])
def test_center_columns_matches_numpy(n, dim):
    # KMeans.fit's X.mean(axis=0), X - mean and X.var(axis=0) (sklearn _tolerance) bit for bit
    rng = np.random.default_rng(n + dim)
    X = (rng.standard_normal((n, dim)) * 3 + 1).astype(np.float32)
    Xd = torch.from_numpy(X).cuda()
    out = torch.empty_like(Xd)
    mean = torch.empty(dim, dtype=torch.float32, device="cuda")
    var = torch.empty(dim, dtype=torch.float32, device="cuda")
    _lib.check(_lib.device_lib().gdd_center_columns(n, dim, Xd.data_ptr(), out.data_ptr(), mean.data_ptr(),
                                                    var.data_ptr(), _lib.stream_ptr("cuda")))
    m = X.mean(axis=0)
    assert np.array_equal(mean.cpu().numpy().view(np.uint32), m.view(np.uint32))
    assert np.array_equal(var.cpu().numpy().view(np.uint32), np.var(X, axis=0).view(np.uint32))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), (X - m).view(np.uint32))


def _colsum_cases():
    rng = np.random.default_rng(11)
    yield "gaussian", 100000, 47, (rng.standard_normal((100000, 47)) * 3 + 1).astype(np.float32)
    # zero-mean columns: the running sums wander across binades and signs (many re-walked segments)
    yield "zero-mean", 70001, 64, rng.standard_normal((70001, 64)).astype(np.float32)
    X = rng.standard_normal((131072, 5)).astype(np.float32)
    X[:, 1] = (rng.integers(-4, 5, 131072) * 0.5 + 2 ** 22).astype(np.float32)  # ties past 2^24
    X[:, 2] = np.float32(0.1)                                                 # constant
    X[::2, 3] = np.float32(1e-3)                                              # cancel to zero
    X[1::2, 3] = np.float32(-1e-3)
    X[:, 4] = (rng.standard_normal(131072) * 10.0 ** rng.integers(-20, 20, 131072)).astype(np.float32)
    yield "adversarial", 131072, 5, X
    X = rng.standard_normal((65536, 3)).astype(np.float32)
    X[4097, 1] = np.inf
    X[60000, 2] = np.nan
    yield "non-finite", 65536, 3, X
    yield "wide", 66000, 256, (rng.standard_normal((66000, 256)) + 0.01).astype(np.float32)
    yield "two columns", 300000, 2, (rng.standard_normal((300000, 2)) - 0.2).astype(np.float32)


@pytest.mark.parametrize("name,n,dim,X", list(_colsum_cases()), ids=[c[0] for c in _colsum_cases()])
def test_center_columns_parallel_matches_numpy(monkeypatch, name, n, dim, X):
    """gdd_center_columns_ws (r05): from 65,536 rows the column chains run in the exact parallel form
    (per-segment transducers of the sequential fp32 sum of signed terms, gdd_colsum.hip; CPU model in
    tests/test_signed_chain_model.py): mean, var and X - mean bit for bit against numpy and against
    the sequential chains (GDD_FORCE=center_seq)."""
    lib = _lib.device_lib()
    Xd = torch.from_numpy(X).cuda()
    res = []
    for par in ("1", "0"):
        force(monkeypatch, *(() if par == "1" else ("center_seq",)))
        out = torch.empty_like(Xd)
        mean = torch.empty(dim, dtype=torch.float32, device="cuda")
        var = torch.empty(dim, dtype=torch.float32, device="cuda")
        ws = _lib.workspace(lib.gdd_center_columns_ws_bytes(n, dim), "cuda")
        _lib.check(lib.gdd_center_columns_ws(n, dim, Xd.data_ptr(), out.data_ptr(), mean.data_ptr(),
                                             var.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_ptr("cuda")))
        res.append((mean.cpu().numpy(), var.cpu().numpy(), out.cpu().numpy()))
    with np.errstate(all="ignore"):
        m = X.mean(axis=0)
        v = np.var(X, axis=0)
        o = X - m
    def same(a, b):  # bit for bit; NaNs compare by position (their sign and payload are the FPU's)
        na, nb = np.isnan(a), np.isnan(b)
        return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))

    for mean, var, out in res:
        assert same(mean, m) and same(var, v) and same(out, o), name


# The device-resident MiniBatch loop: bit-identical to scikit-learn on centres, labels, inertia,
# n_steps_ and the RandomState left behind — across key-buffer groups (G = 1 and 4), row forms
# (dim % 4 != 0), with and without reassignment, early stopping and running to max_iter.
@pytest.mark.parametrize("n,dim,k,bs,ratio,max_iter", [
    (20000, 40, 454, 1000, 0.01, 100),
    (5000, 40, 50, 1000, 0.01, 100),
    (8000, 7, 70, 300, 0.01, 100),
    (6000, 64, 200, 512, 0.01, 100),
    (20000, 40, 454, 1000, 0.0, 100),
    (3000, 12, 100, 2048, 0.5, 100),
    (12000, 40, 300, 1000, 0.01, 1),
])
def test_minibatch_device_loop_shapes(n, dim, k, bs, ratio, max_iter):
    X = synth.blobs(n, dim, k, seed=n + k)
    rs_ref = np.random.RandomState(15)
    ref = O.minibatch_kmeans(X, k, random_state=rs_ref, batch_size=bs, reassignment_ratio=ratio,
                             max_iter=max_iter)
    rs = np.random.RandomState(15)
    m = gdd.MiniBatchKMeans(n_clusters=k, random_state=rs, batch_size=bs,
                            reassignment_ratio=ratio, max_iter=max_iter).fit(X)
    assert m.n_steps_ == ref["n_steps_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))
    assert m.inertia_ == ref["inertia_"]
    s1, s2 = rs_ref.get_state(), rs.get_state()
    assert np.array_equal(s1[1], s2[1]) and s1[2] == s2[2]


# Bounded Lloyd E-steps (on by default where the top-2 pass fits; GDD_FORCE=lloyd_no_prune: off): a row whose
# bounds prove its label skips the distance pass. Labels, centres, inertia and n_iter_ must equal
# the unbounded loop's bit for bit (and the oracle's where it is quick), also on data made of
# near-ties: duplicated rows, rows on the midpoint of two others, a symmetric lattice.
def _near_tie_data(n, dim, seed):
    rng = np.random.default_rng(seed)
    X = synth.blobs(n, dim, 12, seed=seed)
    q = n // 8
    X[:q] = X[q:2 * q]                                  # duplicated rows
    a, b = rng.integers(2 * q, n, q), rng.integers(2 * q, n, q)
    X[2 * q:3 * q] = (X[a] + X[b]) * np.float32(0.5)    # midpoints
    g = np.stack(np.meshgrid(*[np.arange(3, dtype=np.float32)] * min(dim, 3)), -1).reshape(-1, min(dim, 3))
    m = min(len(g), q)
    X[3 * q:3 * q + m, :g.shape[1]] = g[:m]             # a lattice: exact distance ties
    return np.ascontiguousarray(X, np.float32)


@pytest.mark.parametrize("n,dim,k,near_ties", [(40000, 47, 196, False), (30000, 40, 454, False),
                                               (20000, 7, 70, True), (16000, 3, 27, True),
                                               (12000, 16, 1, False), (24000, 48, 100, True)])
def test_kmeans_lloyd_bounded_estep_matches(monkeypatch, n, dim, k, near_ties):
    X = _near_tie_data(n, dim, n + dim) if near_ties else synth.blobs(n, dim, max(2, k // 2), seed=n + k)
    fits = []
    for prune in ("1", "0"):
        force(monkeypatch, *(() if prune == "1" else ("lloyd_no_prune",)))
        np.random.seed(15)
        fits.append(gdd.KMeans(n_clusters=k, n_init=1).fit(X))
    a, b = fits
    assert a.n_iter_ == b.n_iter_
    assert np.array_equal(a.labels_, b.labels_)
    assert np.array_equal(bits(a.cluster_centers_), bits(b.cluster_centers_))
    assert a.inertia_ == b.inertia_
    if n * k <= 2_000_000:
        np.random.seed(15)
        ref = O.kmeans(X, k, n_init=1)
        assert a.n_iter_ == ref["n_iter_"]
        assert np.array_equal(a.labels_, ref["labels_"])
        assert np.array_equal(bits(a.cluster_centers_), bits(ref["cluster_centers_"]))


@pytest.mark.parametrize("prune", ["1", "0"])
def test_kmeans_lloyd_relocation_with_bounds(monkeypatch, prune):
    """Fewer distinct points than clusters: k-means++ picks duplicate centres, so clusters go empty
    and are relocated (sklearn _relocate_empty_clusters) — the loop resumes and the bounds restart."""
    rng = np.random.default_rng(21)
    base = rng.standard_normal((40, 8)).astype(np.float32)
    X = np.ascontiguousarray(np.repeat(base, 60, axis=0)[rng.permutation(2400)])  # 40 distinct rows
    k = 48  # > 40: duplicate centres, empty clusters, relocation (oracle == single-thread sklearn)
    force(monkeypatch, *(() if prune == "1" else ("lloyd_no_prune",)))
    np.random.seed(15)
    ref = O.kmeans(X, k, n_init=1)
    np.random.seed(15)
    m = gdd.KMeans(n_clusters=k, n_init=1).fit(X)
    assert m.n_iter_ == ref["n_iter_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))
    assert m.inertia_ == ref["inertia_"]


@pytest.mark.parametrize("dim", [47, 48])
def test_kmeans_lloyd_sliced_fold_matches(monkeypatch, dim):
    """Large clusters (>= 1.5x the mean size and >= 4096 members) fold in 16-column slices, one
    workgroup each; every column's sequential chain is unchanged, so the fit is bit-identical to the
    unsliced fold and to the oracle (dim 47: scalar staging, 48: 16-byte staging)."""
    rng = np.random.default_rng(dim)
    sizes = [14000, 9000, 2500, 1500, 1000, 700, 500, 400, 250, 150]  # skewed: two big clusters
    centres = rng.standard_normal((len(sizes), dim)).astype(np.float32) * np.float32(4.0)
    X = np.concatenate([c + rng.standard_normal((m, dim)).astype(np.float32) for c, m in zip(centres, sizes)])
    X = np.ascontiguousarray(X[rng.permutation(len(X))], np.float32)
    k = 10
    fits = []
    for sl in ("1.5", "0"):
        force(monkeypatch, f"fold_slice={sl}")
        np.random.seed(15)
        fits.append(gdd.KMeans(n_clusters=k, n_init=1).fit(X))
    a, b = fits
    assert np.bincount(a.labels_, minlength=k).max() >= 1.5 * len(X) / k  # some cluster is sliced
    assert a.n_iter_ == b.n_iter_ and a.inertia_ == b.inertia_
    assert np.array_equal(a.labels_, b.labels_)
    assert np.array_equal(bits(a.cluster_centers_), bits(b.cluster_centers_))
    np.random.seed(15)
    ref = O.kmeans(X, k, n_init=1)
    assert a.n_iter_ == ref["n_iter_"]
    assert np.array_equal(a.labels_, ref["labels_"])
    assert np.array_equal(bits(a.cluster_centers_), bits(ref["cluster_centers_"]))


@pytest.mark.parametrize("dim,prune", [(47, "1"), (47, "0"), (30, "1"), (5, "0"), (101, "0")])
def test_kmeans_lloyd_padded_fold_matches(monkeypatch, dim, prune):
    """From 65,536 rows with dim % 4 != 0 the M-step folds a zero-padded copy of X (rows of
    round4(dim) floats, 16-byte gathers; r05) and writes only the real columns, and the bounded
    E-step reads its row lists from the same copy: the fit is bit-identical to the passes over X
    itself (GDD_FORCE=fold_no_pad / estep_no_pad), sliced large clusters included, and to the oracle."""
    rng = np.random.default_rng(100 + dim)
    sizes = [30000, 16000, 9000, 6000, 4000, 2500, 1500, 800, 400, 200]  # skewed: sliced clusters
    centres = rng.standard_normal((len(sizes), dim)).astype(np.float32) * np.float32(3.0)
    X = np.concatenate([c + rng.standard_normal((m, dim)).astype(np.float32) for c, m in zip(centres, sizes)])
    X = np.ascontiguousarray(X[rng.permutation(len(X))], np.float32)
    assert len(X) >= 65536
    k = 10
    fits = []
    # the bounded E-step's row lists also read the padded copy (r05)
    for pad, epad in (("1", "1"), ("1", "0"), ("0", "0")):
        force(monkeypatch, *([] if prune == "1" else ["lloyd_no_prune"]) + ([] if pad == "1" else ["fold_no_pad"]) +
              ([] if epad == "1" else ["estep_no_pad"]))
        np.random.seed(15)
        fits.append(gdd.KMeans(n_clusters=k, n_init=1).fit(X))
    a = fits[0]
    for b in fits[1:]:
        assert a.n_iter_ == b.n_iter_ and a.inertia_ == b.inertia_
        assert np.array_equal(a.labels_, b.labels_)
        assert np.array_equal(bits(a.cluster_centers_), bits(b.cluster_centers_))
    if dim == 47 and prune == "1":
        np.random.seed(15)
        ref = O.kmeans(X, k, n_init=1)
        assert a.n_iter_ == ref["n_iter_"]
        assert np.array_equal(a.labels_, ref["labels_"])
        assert np.array_equal(bits(a.cluster_centers_), bits(ref["cluster_centers_"]))


@pytest.mark.parametrize("case", ["ml1m_users", "ml1m_items", "relocation", "tol0", "large_n"])
def test_kmeans_lloyd_update_shapes(case):
    """The device loop's update (the average with the empty check folded in, labels changed, the
    convergence test) against the oracle: recsys shapes, empty-cluster relocation (the resumed
    iteration's update runs without the check), a strict convergence run (tol = 0) and a larger n."""
    rng = np.random.default_rng(5)
    kw = {}
    if case == "ml1m_users":
        X, k = synth.blobs(6040, 64, 151, seed=6040), 604
    elif case == "ml1m_items":
        X, k = synth.blobs(3706, 64, 92, seed=3706), 371
    elif case == "relocation":
        base = rng.standard_normal((40, 8)).astype(np.float32)
        X, k = np.repeat(base, 60, axis=0)[rng.permutation(2400)], 48
    elif case == "tol0":
        X, k = synth.blobs(5000, 16, 20, seed=50), 30
        kw = {"tol": 0.0}
    else:
        X, k = synth.blobs(140000, 8, 10, seed=14), 12
    X = np.ascontiguousarray(X, np.float32)
    np.random.seed(15)
    a = gdd.KMeans(n_clusters=k, n_init=1, **kw).fit(X)
    if X.shape[0] * k <= 4_000_000:
        np.random.seed(15)
        ref = O.kmeans(X, k, n_init=1, **kw)
        assert a.n_iter_ == ref["n_iter_"]
        assert np.array_equal(a.labels_, ref["labels_"])
        assert np.array_equal(bits(a.cluster_centers_), bits(ref["cluster_centers_"]))


@pytest.mark.parametrize("n,dim,k,bs", [(20000, 40, 454, 1000), (30000, 8, 200, 2048), (6000, 12, 400, 200),
                                        (8000, 10, 120, 64)])
def test_minibatch_reassign_forms(monkeypatch, n, dim, k, bs):
    """k_mb_reassign: the row copies in three block trips beside a one-wave next-batch draw (the
    parallel-copy form; r05), and with GDD_HOST_LOOP=1 the host-driven loop's reassignment. Blob
    inputs with fewer blobs than centres leave many clusters empty, so reassignments fire often and
    large (m up to b/2; b = 2048 takes two 2048-word passes). Both equal the oracle: labels, centres,
    inertia, n_steps_ and the generator's final state."""
    X = synth.blobs(n, dim, max(2, k // 4), seed=n + k)
    rs_ref = np.random.RandomState(5)
    ref = O.minibatch_kmeans(X, k, random_state=rs_ref, batch_size=bs)
    s_ref = rs_ref.get_state()
    for host in (False, True):
        if host:
            monkeypatch.setenv("GDD_HOST_LOOP", "1")
        rs = np.random.RandomState(5)
        m = gdd.MiniBatchKMeans(n_clusters=k, random_state=rs, batch_size=bs).fit(X)
        assert m.n_steps_ == ref["n_steps_"], host
        assert np.array_equal(m.labels_, ref["labels_"]), host
        assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"])), host
        assert m.inertia_ == ref["inertia_"], host
        s = rs.get_state()
        assert np.array_equal(s[1], s_ref[1]) and s[2] == s_ref[2], host


@pytest.mark.parametrize("n,dim,k,bs", [(6000, 12, 400, 200), (20000, 8, 300, 500), (3000, 16, 700, 256),
                                        (8000, 10, 120, 64)])
def test_minibatch_k_above_half_batch(monkeypatch, n, dim, k, bs):
    """k > b/2 (config 3's k = 769 > b/2 = 500): the device loop runs these fits too.
    A reassignment with more than b/2 centres due (np.argsort's branch — certain at step 0 when
    k >= 2b, since a batch leaves at least k - b clusters empty) stops the device loop at that step;
    the host runs its convergence test and reassignment, steps on while a weight sum is zero, and
    resumes the device loop. Labels, centres, inertia, n_steps_ and the generator's final state equal
    the oracle's and the host-driven loop's (GDD_HOST_LOOP=1)."""
    X = synth.blobs(n, dim, max(2, k // 3), seed=n + k)
    rs_ref = np.random.RandomState(11)
    ref = O.minibatch_kmeans(X, k, random_state=rs_ref, batch_size=bs)
    s_ref = rs_ref.get_state()
    for host in (False, True):
        if host:
            monkeypatch.setenv("GDD_HOST_LOOP", "1")
        rs = np.random.RandomState(11)
        m = gdd.MiniBatchKMeans(n_clusters=k, random_state=rs, batch_size=bs).fit(X)
        assert m.n_steps_ == ref["n_steps_"], host
        assert np.array_equal(m.labels_, ref["labels_"]), host
        assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"])), host
        assert m.inertia_ == ref["inertia_"], host
        s = rs.get_state()
        assert np.array_equal(s[1], s_ref[1]) and s[2] == s_ref[2], host


@pytest.mark.parametrize("mni", [1, 2, 3])
@pytest.mark.parametrize("n,dim,k,bs", [(3000, 16, 700, 256), (6000, 12, 400, 200)])
def test_minibatch_handoff_then_convergence_stop(n, dim, k, bs, mni):
    """the k > b/2 hand-off followed closely by a convergence stop. With k >= 2b the
    argsort branch fires at step 0 (the device loop hands that step to the host and resumes); a small
    max_no_improvement then stops the fit within a few steps of the hand-off, on the resumed segment.
    n_steps_, labels, centres, inertia and the generator's final state equal the oracle's."""
    X = synth.blobs(n, dim, max(2, k // 3), seed=n + k + mni)
    rs_ref = np.random.RandomState(23)
    ref = O.minibatch_kmeans(X, k, random_state=rs_ref, batch_size=bs, max_no_improvement=mni)
    s_ref = rs_ref.get_state()
    assert ref["n_steps_"] < 100 * n // bs  # the convergence stop fired
    rs = np.random.RandomState(23)
    m = gdd.MiniBatchKMeans(n_clusters=k, random_state=rs, batch_size=bs, max_no_improvement=mni).fit(X)
    assert m.n_steps_ == ref["n_steps_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))
    assert m.inertia_ == ref["inertia_"]
    s = rs.get_state()
    assert np.array_equal(s[1], s_ref[1]) and s[2] == s_ref[2]


def test_assign_bf16_gathered_rows_unaligned_and_predict():
    """The bf16 pass's other entries: a row list (the chunked kernel + finalize), an X that is not
    16-byte aligned (a view one row in, dim 41), and KMeans.predict(precision="bf16") — each label
    the exact fp32 one or within the bf16 rounding bound; predict at fp32 gives the exact labels."""
    from gdd.kmeans import _Ops
    rng = np.random.default_rng(12)
    n, dim, k = 20001, 41, 97
    Xall = (rng.standard_normal((n + 1, dim)) + rng.integers(0, 4, (n + 1, 1))).astype(np.float32)
    C = Xall[rng.choice(n, k, replace=False)] + rng.standard_normal((k, dim)).astype(np.float32) * 0.1
    Xd_all = torch.from_numpy(Xall).cuda()
    Xu = Xd_all[1:]  # 164 bytes in: not 16-byte aligned
    assert Xu.data_ptr() % 16 != 0
    Cd = torch.from_numpy(C).cuda()
    ops = _Ops("cuda", n + 1, k, dim)
    lab = {}
    for name, X, rows in (("unaligned", Xu, None), ("rows", Xd_all, torch.arange(1, n + 1, device="cuda"))):
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        ops.assign(X, Cd, rows=rows, labels=out, precision="bf16")
        lab[name] = out.cpu().numpy()
    exact = torch.empty(n, dtype=torch.int32, device="cuda")
    ops.assign(Xu.contiguous(), Cd, labels=exact)
    a = exact.cpu().numpy()
    X64, C64 = Xall[1:].astype(np.float64), C.astype(np.float64)
    xn, cn = np.linalg.norm(X64, axis=1), np.linalg.norm(C64, axis=1)
    for name, b in lab.items():
        assert b.min() >= 0 and b.max() < k
        for i in np.nonzero(a != b)[0][:2000]:
            di = ((X64[i] - C64) ** 2).sum(-1)
            assert di[b[i]] - di[a[i]] <= 2 * 2.0 ** -7 * xn[i] * (cn[a[i]] + cn[b[i]]) + 1e-3 * (1 + di[a[i]]), name
    km = gdd.KMeans(n_clusters=k)
    km.cluster_centers_ = C
    p = km.predict(Xall[1:], precision="bf16")
    for i in np.nonzero(a != p)[0][:2000]:
        di = ((X64[i] - C64) ** 2).sum(-1)
        assert di[p[i]] - di[a[i]] <= 2 * 2.0 ** -7 * xn[i] * (cn[a[i]] + cn[p[i]]) + 1e-3 * (1 + di[a[i]])
    assert np.array_equal(km.predict(Xall[1:]), a)  # fp32 predict: the exact labels
