"""Edge cases of the k-means kernels and fits (GPU vs the oracle, bit-exact).

Shapes the reference's inputs can take but the main tests do not: a single sample or centre,
partial 32-row tiles, dim 1 and the 512 maximum, duplicated rows (distance ties), k = n,
batch larger than n, reassignment disabled, early stopping disabled (max_no_improvement=None).
"""
import numpy as np
import pytest
import torch

from golden_util import bits
from oracle import oracle as O

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402


@pytest.mark.parametrize("n,dim,k", [(1, 3, 1), (31, 5, 4), (33, 1, 33), (200, 512, 7),
                                     (1000, 40, 1), (4097, 2, 600)])
def test_assign_edges(n, dim, k):
    rng = np.random.default_rng(n + dim + k)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    C = X[rng.choice(n, size=k, replace=k > n)].copy() if k <= n else rng.standard_normal((k, dim)).astype(np.float32)
    lab_ref, sq_ref = O.assign(X, C)
    Xd, Cd = torch.from_numpy(X).cuda(), torch.from_numpy(C).cuda()
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    sq = torch.empty(n, dtype=torch.float32, device="cuda")
    _Ops("cuda", n, k, dim).assign(Xd, Cd, labels=lab, sq=sq)
    assert np.array_equal(lab.cpu().numpy(), lab_ref)
    assert np.array_equal(bits(sq.cpu().numpy()), bits(sq_ref))


@pytest.mark.parametrize("n,dim,k,mode", [
    (40001, 47, 196, "contig"),   # products' row width: 12 waves per block, ragged last tile
    (20003, 1, 33, "contig"),     # n * dim not a multiple of 4: the scalar tail of the float4 fetch
    (30000, 3, 454, "contig"),
    (16385, 48, 900, "contig"),   # centres past one LDS chunk: chunked, atomically merged keys
    (25000, 41, 769, "contig"),   # Reddit's shape class
    (33000, 40, 454, "rows"),     # a row list: two lanes per gathered row
    (20001, 47, 196, "offset"),   # X not 16-byte aligned: the per-row fetch without a row list
])
def test_assign_large_n_wave_tiles(n, dim, k, mode):
    """The large-n labels pass (wave tiles, k_assign_waves) is the oracle's assignment bit for bit."""
    rng = np.random.default_rng(n + k)
    X = (rng.standard_normal((n, dim)) * 3).astype(np.float32)
    C = X[rng.choice(n, size=k, replace=False)] + np.float32(0.01)
    rows = rng.integers(0, n, n).astype(np.int64) if mode == "rows" else None
    lab_ref, sq_ref = O.assign(X, C, rows=rows)
    if mode == "offset":
        buf = torch.empty(n * dim + 1, dtype=torch.float32, device="cuda")
        Xd = buf[1:].view(n, dim)
        Xd.copy_(torch.from_numpy(X))
        assert Xd.data_ptr() % 16 != 0
    else:
        Xd = torch.from_numpy(X).cuda()
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    sq = torch.empty(n, dtype=torch.float32, device="cuda")
    _Ops("cuda", n, k, dim).assign(Xd, torch.from_numpy(np.ascontiguousarray(C)).cuda(),
                                   rows=None if rows is None else torch.from_numpy(rows).cuda(),
                                   labels=lab, sq=sq)
    assert np.array_equal(lab.cpu().numpy(), lab_ref)
    assert np.array_equal(bits(sq.cpu().numpy()), bits(sq_ref))


def test_assign_ties_between_tiles_and_zero_signs():
    # identical centres in different 32-centre tiles and chunks: the lowest index must win, also
    # when the distance is exactly zero (the packed key treats -0.0 and +0.0 as one value)
    rng = np.random.default_rng(1)
    base = rng.standard_normal((5, 16)).astype(np.float32)
    C = np.tile(base, (140, 1))  # 700 centres, every row repeated 140 times
    X = np.concatenate([base, np.zeros((3, 16), np.float32), base * 0.5]).astype(np.float32)
    lab_ref, sq_ref = O.assign(X, C)
    lab = torch.empty(X.shape[0], dtype=torch.int32, device="cuda")
    sq = torch.empty(X.shape[0], dtype=torch.float32, device="cuda")
    _Ops("cuda", X.shape[0], C.shape[0], 16).assign(torch.from_numpy(X).cuda(),
                                                     torch.from_numpy(C).cuda(), labels=lab, sq=sq)
    assert np.array_equal(lab.cpu().numpy(), lab_ref)
    assert lab_ref.max() < 5


@pytest.mark.parametrize("n,dim,k,n_init", [(50, 4, 50, 1), (300, 3, 12, 2), (64, 1, 5, 1)])
def test_kmeans_edges(n, dim, k, n_init):
    X = synth.blobs(n, dim, max(1, k // 3), seed=n)
    X[1::7] = X[0]  # duplicated rows
    np.random.seed(3)
    ref = O.kmeans(X, k, n_init=n_init)
    np.random.seed(3)
    m = gdd.KMeans(n_clusters=k, n_init=n_init).fit(X)
    assert m.n_iter_ == ref["n_iter_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))


@pytest.mark.parametrize("kw", [dict(batch_size=5000), dict(reassignment_ratio=0.0),
                                dict(max_no_improvement=None, max_iter=3), dict(n_clusters=1),
                                dict(init_size=40)])
def test_minibatch_edges(kw):
    n, dim = 3000, 9
    X = synth.blobs(n, dim, 20, seed=2)
    args = dict(n_clusters=20, random_state=7, batch_size=256)
    args.update(kw)
    ref = O.minibatch_kmeans(X, args.pop("n_clusters"), **args)
    args = dict(n_clusters=20, random_state=7, batch_size=256)
    args.update(kw)
    m = gdd.MiniBatchKMeans(**args).fit(X)
    assert m.n_steps_ == ref["n_steps_"]
    assert np.array_equal(m.labels_, ref["labels_"])
    assert np.array_equal(bits(m.cluster_centers_), bits(ref["cluster_centers_"]))
    assert m.inertia_ == ref["inertia_"]


def test_cluster_mean_single_cluster_and_mostly_empty():
    feat = synth.features(1000, 33, 4)
    for lab in (np.zeros(1000, np.int32), np.full(1000, 6, np.int32)):
        ref, cnt_ref = O.cluster_mean(feat, lab, 9)
        out, cnt = gdd.cluster_mean(torch.from_numpy(feat).cuda(), lab, 9)
        assert np.array_equal(cnt.cpu().numpy(), cnt_ref)
        o = out.cpu().numpy()
        assert np.array_equal(np.isnan(o), np.isnan(ref))
        m = ~np.isnan(ref)
        assert np.array_equal(bits(o[m]), bits(ref[m]))


@pytest.mark.parametrize("nbytes", [16, 4096 + 48, 1 << 20, (1 << 24) + 16 * 1023])
def test_stream_copy_exact(nbytes):
    # the bench's copy-peak kernel: every byte copied, nothing past the end touched
    from gdd import _lib
    lib = _lib.device_lib()
    src = torch.randint(-2**31, 2**31 - 1, (nbytes // 4 + 4,), dtype=torch.int32, device="cuda")
    dst = torch.zeros_like(src)
    _lib.check(lib.gdd_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, _lib.stream_ptr("cuda")))
    torch.cuda.synchronize()
    m = nbytes // 4
    assert torch.equal(src[:m], dst[:m]) and int(dst[m:].abs().sum()) == 0


def test_cluster_mean_more_clusters_than_one_launch():
    # k above the 65,535 clusters one fold launch's grid.y holds: the launches are chunked, each
    # writing its slice of the means and counts
    n, d, k = 200_000, 4, 70_001
    feat = synth.features(n, d, 8)
    lab = np.random.default_rng(3).integers(0, k, n).astype(np.int32)
    lab[:5] = k - 1
    ref, cnt_ref = O.cluster_mean(feat, lab, k)
    out, cnt = gdd.cluster_mean(torch.from_numpy(feat).cuda(), lab, k)
    assert np.array_equal(cnt.cpu().numpy(), cnt_ref)
    o = out.cpu().numpy()
    assert np.array_equal(np.isnan(o), np.isnan(ref))
    m = ~np.isnan(ref)
    assert np.array_equal(bits(o[m]), bits(ref[m]))


def test_lloyd_run_k_above_counting_sort():
    # k > 32,768: the device Lloyd loop groups the labels with the radix path (no LDS counters).
    # One iteration from given centres (distinct data points far apart, no cluster empty) against the
    # oracle's _lloyd_iter: labels, new centres, weights and shifts bit for bit.
    from gdd import _lib
    import ctypes
    n, dim, k = 34_000, 8, 33_000
    X = np.random.default_rng(11).standard_normal((n, dim)).astype(np.float32)
    C0 = X[:k].copy()
    lab_ref, c_ref, wic_ref, shift_ref = O._lloyd_iter(X, C0)
    assert (wic_ref > 0).all()  # 8-d points far apart: every centre keeps its own point
    lib = _lib.device_lib()
    dev = torch.device("cuda")
    Xd = torch.from_numpy(X).to(dev)
    Cb = (torch.from_numpy(C0).to(dev), torch.empty((k, dim), dtype=torch.float32, device=dev))
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    labels_old = torch.full((n,), -1, dtype=torch.int32, device=dev)
    wic = torch.empty(k, dtype=torch.float32, device=dev)
    shift = torch.empty(k, dtype=torch.float32, device=dev)
    ws = _lib.workspace(lib.gdd_kmeans_lloyd_ws_bytes(n, dim, k), dev)
    hws = _lib.pinned_workspace(lib.gdd_kmeans_lloyd_host_ws_bytes())
    state = torch.zeros(lib.gdd_lloyd_state_bytes(), dtype=torch.uint8, device=dev)
    done, reason = ctypes.c_int32(0), ctypes.c_int32(0)
    _lib.check(lib.gdd_kmeans_lloyd_run(n, dim, Xd.data_ptr(), k, Cb[0].data_ptr(), Cb[1].data_ptr(),
                                        labels.data_ptr(), labels_old.data_ptr(), wic.data_ptr(),
                                        shift.data_ptr(), 0, 0, 1, 0.0, state.data_ptr(),
                                        ctypes.addressof(done), ctypes.addressof(reason), ws.data_ptr(),
                                        ws.numel(), hws.data_ptr(), hws.numel(), _lib.stream_ptr(dev)))
    assert done.value == 1 and reason.value == 0
    assert np.array_equal(labels.cpu().numpy(), lab_ref)
    assert np.array_equal(bits(wic.cpu().numpy()), bits(wic_ref))
    assert np.array_equal(bits(Cb[1].cpu().numpy()), bits(c_ref))
    assert np.array_equal(bits(shift.cpu().numpy()), bits(shift_ref))
