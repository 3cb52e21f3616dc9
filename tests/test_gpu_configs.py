"""Parity at the BASELINE configs' own shapes (VERDICT r1 "untested configs").

* config 5 (ogbn-products): KMeans(k=196) on a 200,000 x 47 products-shaped input against
  scikit-learn's own result on the same input (fixture G9: labels hash, centres, inertia, n_iter) —
  this runs the multi-block k-means++ rounds, the persistent MFMA assignment and the device Lloyd
  loop; and the bf16 distance variant at the full 2,449,029 x 47, k=196 assignment shape;
* config 4 (ML-1M recsys): distill_recsys.kmeans_cluster on 6,040 x 64 (k=604) and 3,706 x 64
  (k=371) SVD-shaped embeddings, seed 42, against the reference function's output (G9);
* config 1 (Cora): 2,708 x 1,433 propagation (T=5, alpha=0.8), KMeans(k=70) on the 7-class logits
  and the cluster means, against the oracle bit for bit;
* config 2 (ogbn-arxiv): the full 169,343-node, 128-d propagation (T=18, alpha=0.91) against the
  oracle bit for bit.
"""
import hashlib

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import bits, load, load_json
from oracle import oracle as O

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import _lib, synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402
from gdd.pipeline import kmeans_cluster  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_products_shape_kmeans_matches_sklearn():
    rec = load_json("golden_configs.json")
    z = load("golden_configs.npz")
    X = synth.blobs(200000, 47, 196, seed=5)
    np.random.seed(15)  # the agents' KMeans(random_state=None) draws from the global RNG
    m = gdd.KMeans(n_clusters=196).fit(X)
    assert m.n_iter_ == rec["products_n_iter"]
    assert sha(m.labels_.astype(np.int32)) == rec["products_labels_sha256"]
    assert np.array_equal(bits(m.cluster_centers_), bits(z["products_centers"]))
    assert m.inertia_ == rec["products_inertia"]


def test_products_shape_bf16_assignment_within_rounding():
    # config 5's "fp32 vs bf16 MFMA distance kernel" at its full assignment shape: every label that
    # differs from the exact fp32 one lies within the bf16 rounding of the dot products
    n, dim, k = 2449029, 47, 196
    rng = np.random.default_rng(196)
    X = synth.blobs(n, dim, k, seed=47)
    C = X[rng.choice(n, k, replace=False)] + rng.standard_normal((k, dim)).astype(np.float32) * 0.05
    Xd, Cd = torch.from_numpy(X).cuda(), torch.from_numpy(C).cuda()
    ops = _Ops("cuda", n, k, dim)
    l32 = torch.empty(n, dtype=torch.int32, device="cuda")
    l16 = torch.empty(n, dtype=torch.int32, device="cuda")
    ops.assign(Xd, Cd, labels=l32)
    ops.assign(Xd, Cd, labels=l16, precision="bf16")
    a, b = l32.cpu().numpy(), l16.cpu().numpy()
    assert b.min() >= 0 and b.max() < k
    assert (a == b).mean() >= 0.99
    diff = np.nonzero(a != b)[0]
    X64, C64 = X.astype(np.float64), C.astype(np.float64)
    cn = np.linalg.norm(C64, axis=1)
    for i in diff[:4000]:
        di = ((X64[i] - C64) ** 2).sum(-1)
        bound = 2 * 2.0 ** -7 * np.linalg.norm(X64[i]) * (cn[a[i]] + cn[b[i]]) + 1e-3 * (1 + di[a[i]])
        assert di[b[i]] - di[a[i]] <= bound
    # the exact labels themselves equal the oracle's on a sample of rows
    rows = rng.integers(0, n, 20000)
    lab_ref, _ = O.assign(X[rows], C)
    assert np.array_equal(a[rows], lab_ref)


@pytest.mark.parametrize("name,n,k", [("users", 6040, 604), ("items", 3706, 371)])
def test_recsys_ml1m_kmeans_cluster_matches_reference(name, n, k):
    z = load("golden_configs.npz")
    E = synth.svd_like(n, 64, seed=n)
    lab, cen = kmeans_cluster(E, n_clusters=k, seed=42, minibatch=True)
    assert np.array_equal(lab, z[f"ml1m_{name}_labels"].astype(np.int64))
    assert np.array_equal(bits(cen), bits(z[f"ml1m_{name}_centers"]))


def test_cora_shape_propagate_kmeans_cluster_mean():
    n, d, C, k = 2708, 1433, 7, 70
    A = sp.csr_matrix(synth.chung_lu(n, 3.9, 15))
    X = synth.bag_of_words(n, d, 15)
    ro, co, vo = O.normalize_csr(A.indptr, A.indices, None, -1)
    t_ref, p_ref = O.propagate(ro, co, vo, X, 5, 0.8)
    g = gdd.normalize_adj(gdd.to_csr(A, device="cuda"))
    t, p = gdd.propagate(g, torch.from_numpy(X).cuda(), 5, 0.8)
    assert np.array_equal(bits(t.cpu().numpy()), bits(t_ref))
    assert np.array_equal(bits(p.cpu().numpy()), bits(p_ref))
    logits = synth.linear_logits(t_ref, C, 15)
    np.random.seed(15)
    ref = O.kmeans(logits, k)
    np.random.seed(15)
    km = gdd.KMeans(n_clusters=k).fit(logits)
    assert km.n_iter_ == ref["n_iter_"]
    assert np.array_equal(km.labels_, ref["labels_"])
    fs_ref, cnt_ref = O.cluster_mean(t_ref, ref["labels_"], k)
    fs, cnt = gdd.cluster_mean(t, km.labels_device_, k)
    assert np.array_equal(cnt.cpu().numpy(), cnt_ref)
    assert np.array_equal(bits(fs.cpu().numpy()), bits(fs_ref))  # NaN rows share one bit pattern


def test_arxiv_shape_propagate_matches_oracle():
    n, d = 169343, 128
    A = sp.csr_matrix(synth.chung_lu(n, 13.7, 15))
    X = synth.features(n, d, 15)
    ro, co, vo = O.normalize_csr(A.indptr, A.indices, None, -1)
    t_ref, p_ref = O.propagate(ro, co, vo, X, 18, 0.91)
    g = gdd.normalize_adj(gdd.to_csr(A, device="cuda"))
    assert g.nnz == co.shape[0]
    t, p = gdd.propagate(g, torch.from_numpy(X).cuda(), 18, 0.91)
    assert np.array_equal(bits(t.cpu().numpy()), bits(t_ref))
    assert np.array_equal(bits(p.cpu().numpy()), bits(p_ref))


def test_arxiv_shape_cluster_mean_matches_oracle():
    n, d, k = 169343, 128, 454
    feat = synth.features(n, d, 9)
    lab = np.random.default_rng(9).integers(0, k, n).astype(np.int32)
    lab[lab == 77] = 78  # an empty cluster -> NaN row
    ref, cnt_ref = O.cluster_mean(feat, lab, k)
    out, cnt = gdd.cluster_mean(torch.from_numpy(feat).cuda(), torch.from_numpy(lab).cuda(), k)
    assert np.array_equal(cnt.cpu().numpy(), cnt_ref)
    assert np.array_equal(bits(out.cpu().numpy()), bits(ref))


def test_average_centers_empty_cluster_copies_first_heaviest_in_loop_order():
    # _average_centers: cluster 1 (< argmax 2) copies the raw sums of cluster 2, cluster 4 (> 2)
    # its averaged row; ties for the heaviest weight go to the first index
    k, dim = 6, 37
    rng = np.random.default_rng(6)
    sums = rng.standard_normal((k, dim)).astype(np.float32) * 7
    w = np.array([3, 0, 5, 5, 0, 2], np.float32)
    old = rng.standard_normal((k, dim)).astype(np.float32)
    ref = sums.copy()
    shift_ref = np.empty(k, np.float32)
    O.lib().oracle_average_centers(k, dim, ref, w, old, shift_ref.ctypes.data_as(O.vp))
    Cn = torch.from_numpy(sums).cuda()
    shift = torch.empty(k, dtype=torch.float32, device="cuda")
    lib = _lib.device_lib()
    wd, od = torch.from_numpy(w).cuda(), torch.from_numpy(old).cuda()
    _lib.check(lib.gdd_average_centers(k, dim, Cn.data_ptr(), wd.data_ptr(), od.data_ptr(),
                                       shift.data_ptr(), _lib.stream_ptr("cuda")))
    got = Cn.cpu().numpy()
    assert np.array_equal(bits(got), bits(ref))
    assert np.array_equal(bits(shift.cpu().numpy()), bits(shift_ref))
    assert not np.array_equal(got[1], got[4])  # raw vs averaged copy


@pytest.mark.parametrize("n,k", [(1, 1), (1000, 3), (70000, 454), (2500000, 196), (5000, 9000),
                                 # the one-workgroup form (n <= 32,768, k <= 2,048): both tile sizes,
                                 # odd k, the limits
                                 (6040, 604), (16384, 2048), (16385, 1773), (32768, 1), (32768, 2047),
                                 (17730, 1773), (3706, 371)])
def test_group_by_label_is_a_stable_sort(n, k):
    rng = np.random.default_rng(n + k)
    lab = rng.integers(0, k, n).astype(np.int32)
    if n > 10:
        lab[::97] = -1  # outside [0, k): in no cluster
        lab[5::101] = k
    perm, offs = gdd.group_by_label(torch.from_numpy(lab).cuda(), k)
    valid = (lab >= 0) & (lab < k)
    order = np.argsort(np.where(valid, lab, k), kind="stable")[: valid.sum()]
    o = offs.cpu().numpy()
    assert o[-1] == valid.sum()
    assert np.array_equal(perm.cpu().numpy()[: valid.sum()], order.astype(np.int32))
    assert np.array_equal(o[:-1], np.searchsorted(np.sort(lab[valid]), np.arange(k), side="left"))


def _device_chung_lu(n, avg_degree, seed):
    """synth.chung_lu_device (the host generator needs minutes at the products shape)."""
    return synth.chung_lu_device(n, avg_degree, seed)


def test_products_shape_propagate_matches_oracle():
    """Config 5's propagation: N = 2,449,029, ~126M entries, d = 100, T = 3, alpha =
    0.91 — the normalised graph and every bit of target and the last hop against the oracle (hub
    rows split over many 256-entry segments, the fix-up pass, the d <= 112 lane group)."""
    n, d = 2449029, 100
    gr = _device_chung_lu(n, 50.5, 5)
    X = synth.features(n, d, 5)
    rp, co = gr.rowptr.cpu().numpy(), gr.col.cpu().numpy()
    assert co.shape[0] > 120_000_000
    ro, cn, vo = O.normalize_csr(rp, co, None, -1)
    g = gdd.normalize_adj(gr)
    assert np.array_equal(g.rowptr.cpu().numpy(), ro) and np.array_equal(g.col.cpu().numpy(), cn)
    assert np.array_equal(bits(g.val.cpu().numpy()), bits(vo))
    del gr
    t, p = gdd.propagate(g, torch.from_numpy(X).cuda(), 3, 0.91)
    t_ref, p_ref = O.propagate(ro, cn, vo, X, 3, 0.91)
    assert np.array_equal(bits(t.cpu().numpy()), bits(t_ref))
    assert np.array_equal(bits(p.cpu().numpy()), bits(p_ref))


def test_reddit_shape_minibatch_matches_sklearn():
    """Config 3's clustering at its full train shape (fixture G9b): MiniBatchKMeans(k=769, b=1000,
    random_state=15) on 153,932 x 41 — k > b/2, so the fit takes the host-driven step loop whose
    reassignment may take the argsort branch — labels, centres, inertia and n_steps_ as sklearn's."""
    rec = load_json("golden_full_shapes.json")
    X = synth.blobs(153932, 41, 769, seed=41)
    m = gdd.MiniBatchKMeans(n_clusters=769, random_state=15, batch_size=1000).fit(X)
    assert m.n_steps_ == rec["reddit_n_steps"]
    assert sha(m.labels_.astype(np.int32)) == rec["reddit_labels_sha256"]
    assert sha(np.ascontiguousarray(m.cluster_centers_, np.float32)) == rec["reddit_centers_sha256"]
    assert m.inertia_ == rec["reddit_inertia"]


def test_products_full_shape_kmeans_matches_sklearn():
    """Config 5's clustering at its full shape (fixture G9b): KMeans(k=196) on 2,449,029 x 47 after
    np.random.seed(15) — the multi-block (split) k-means++ rounds over 598 point blocks, the device
    Lloyd loop — labels, centres, inertia and n_iter_ as sklearn's."""
    rec = load_json("golden_full_shapes.json")
    X = synth.blobs(2449029, 47, 196, seed=5)
    np.random.seed(15)
    m = gdd.KMeans(n_clusters=196).fit(X)
    assert m.n_iter_ == rec["products_n_iter"]
    assert sha(m.labels_.astype(np.int32)) == rec["products_labels_sha256"]
    assert sha(np.ascontiguousarray(m.cluster_centers_, np.float32)) == rec["products_centers_sha256"]
    assert m.inertia_ == rec["products_inertia"]


def test_reddit_shape_propagate_matches_oracle():
    """Config 3's propagation at the Reddit train graph's full shape: N = 153,932,
    ~10M entries, d = 602, T = 3, alpha = 0.95 (main_induct.sh:16-21; the induct loops
    clustgdd_agent_induct.py:72-94) — the d > 128 float2 lanes with split hub rows and the fix-up,
    every bit of target and the last hop against the oracle."""
    n, d = 153932, 602
    gr = _device_chung_lu(n, 65.0, 3)
    X = synth.features(n, d, 3)
    rp, co = gr.rowptr.cpu().numpy(), gr.col.cpu().numpy()
    assert co.shape[0] > 9_000_000
    assert np.diff(rp).max() > 256  # hub rows span several segments
    ro, cn, vo = O.normalize_csr(rp, co, None, -1)
    g = gdd.normalize_adj(gr)
    assert np.array_equal(g.rowptr.cpu().numpy(), ro) and np.array_equal(g.col.cpu().numpy(), cn)
    assert np.array_equal(bits(g.val.cpu().numpy()), bits(vo))
    del gr
    t, p = gdd.propagate(g, torch.from_numpy(X).cuda(), 3, 0.95)
    t_ref, p_ref = O.propagate(ro, cn, vo, X, 3, 0.95)
    assert np.array_equal(bits(t.cpu().numpy()), bits(t_ref))
    assert np.array_equal(bits(p.cpu().numpy()), bits(p_ref))
