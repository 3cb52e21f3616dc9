"""The HIP path against the reference's golden vectors (tools/make_golden.py) — needs a GPU."""
import hashlib

import numpy as np
import pytest
import torch
from sklearn.preprocessing import StandardScaler

from golden_util import (MEAN_ATOL, MEAN_RTOL, PROP_ATOL, PROP_RTOL, bits, csr_to_sorted_coo,
                         graph_names, load, load_json, rng_from_fixture)

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import synth  # noqa: E402


def _graph(rowptr, col, val=None):
    n = len(rowptr) - 1
    import scipy.sparse as sp
    v = np.ones(len(col), np.float32) if val is None else val
    return gdd.to_csr(sp.csr_matrix((v, col, rowptr), shape=(n, n)), binary=val is None)


@pytest.mark.parametrize("name", graph_names())
def test_normalize_vs_reference(name):
    z = load("golden_normalize.npz")
    binary = name != "weighted"
    g = _graph(z[f"{name}_rowptr"], z[f"{name}_col"], None if binary else z[f"{name}_val"])
    gn = gdd.normalize_adj(g)
    r, c, v = csr_to_sorted_coo(gn.rowptr.cpu().numpy(), gn.col.cpu().numpy(), gn.val.cpu().numpy())
    assert np.array_equal(r, z[f"{name}_out_row"]) and np.array_equal(c, z[f"{name}_out_col"])
    if name == "selfloop0":
        np.testing.assert_allclose(v, z[f"{name}_out_val"], rtol=3e-7, atol=0)
    else:
        assert np.array_equal(bits(v), bits(z[f"{name}_out_val"]))


@pytest.mark.parametrize("T", [5, 18])
def test_propagate_vs_reference(T):
    z = load("golden_propagate.npz")
    gn = gdd.normalize_adj(_graph(z["rowptr"], z["col"]))
    alpha = {5: 0.8, 18: 0.91}[T]
    t, p = gdd.propagate(gn, torch.from_numpy(z["X"]).cuda(), T, alpha)
    np.testing.assert_allclose(t.cpu().numpy(), z[f"target_T{T}"], rtol=PROP_RTOL, atol=PROP_ATOL)
    np.testing.assert_allclose(p.cpu().numpy(), z[f"prop_T{T}"], rtol=PROP_RTOL, atol=PROP_ATOL)


def test_minibatch_kmeans_vs_sklearn():
    z = load("golden_kmeans.npz")
    m = gdd.MiniBatchKMeans(n_clusters=50, random_state=15, batch_size=1000).fit(z["mb_X"])
    assert m.n_steps_ == int(z["mb_n_steps"])
    assert np.array_equal(m.labels_, z["mb_labels"])
    assert np.array_equal(bits(m.cluster_centers_), bits(z["mb_centers"]))
    assert m.inertia_ == float(z["mb_inertia"])


@pytest.mark.parametrize("tag,n_init", [("km1", "auto"), ("km10", 10)])
def test_kmeans_vs_sklearn(tag, n_init):
    z = load("golden_kmeans.npz")
    np.random.seed(15)
    m = gdd.KMeans(n_clusters=70, n_init=n_init).fit(z["km_X"])
    assert m.n_iter_ == int(z[f"{tag}_n_iter"])
    assert np.array_equal(m.labels_, z[f"{tag}_labels"])
    assert np.array_equal(bits(m.cluster_centers_), bits(z[f"{tag}_centers"]))
    assert m.inertia_ == float(z[f"{tag}_inertia"])


def test_recsys_kmeans_cluster_vs_reference():
    z = load("golden_kmeans.npz")
    Xs = StandardScaler(with_mean=True, with_std=True).fit_transform(z["rs_X"])
    m = gdd.KMeans(n_clusters=200, random_state=42, n_init="auto").fit(Xs)
    assert np.array_equal(m.labels_.astype(np.int64), z["rs_labels"])
    assert np.array_equal(bits(m.cluster_centers_), bits(z["rs_centers"]))


def test_minibatch_arxiv_scale_hash():
    g = load_json("golden_kmeans_arxiv.json")
    X = synth.blobs(169343, 40, 454, seed=34)
    m = gdd.MiniBatchKMeans(n_clusters=454, random_state=15, batch_size=1000).fit(X)
    assert m.n_steps_ == g["n_steps"]
    assert hashlib.sha256(m.labels_.astype(np.int32).tobytes()).hexdigest() == g["labels_sha256"]
    assert hashlib.sha256(m.cluster_centers_.astype(np.float32).tobytes()).hexdigest() == g["centers_sha256"]
    assert m.inertia_ == g["inertia"]


@pytest.mark.parametrize("tag", ["cora", "arxiv"])
def test_pretrained_clustering_vs_reference(tag):
    z = load(f"golden_clustgdd_{tag}.npz")
    gn = gdd.normalize_adj(_graph(z["rowptr"], z["col"]))
    r, c, v = csr_to_sorted_coo(gn.rowptr.cpu().numpy(), gn.col.cpu().numpy(), gn.val.cpu().numpy())
    assert np.array_equal(r, z["norm_row"]) and np.array_equal(c, z["norm_col"])
    assert np.array_equal(bits(v), bits(z["norm_val"]))
    target, _ = gdd.propagate(gn, torch.from_numpy(z["feat"]).cuda(), int(z["T"]), float(z["alpha"]))
    np.testing.assert_allclose(target.cpu().numpy(), z["target_feat"], rtol=PROP_RTOL, atol=PROP_ATOL)
    k = int(z["n_syn"])
    if tag == "arxiv":
        km = gdd.MiniBatchKMeans(n_clusters=k, random_state=15, batch_size=100).fit(z["kmeans_X"])
    else:
        km = gdd.KMeans(n_clusters=k, random_state=rng_from_fixture(z)).fit(z["kmeans_X"])
    assert np.array_equal(km.labels_, z["cluster_labels"])
    feat_syn, _ = gdd.cluster_mean(torch.from_numpy(z["target_feat"]).cuda(), km.labels_device_, k)
    np.testing.assert_allclose(feat_syn.cpu().numpy(), z["feat_syn"], rtol=MEAN_RTOL, atol=MEAN_ATOL)
    labels_syn = gdd.argmax_rows(km.cluster_centers_device_)
    assert np.array_equal(labels_syn.cpu().numpy(), z["labels_syn"])


def test_recsys_kmeans_cluster_device_scaler():
    # distill_recsys.kmeans_cluster end to end on the device (StandardScaler included)
    from gdd import pipeline
    z = load("golden_kmeans.npz")
    lab, cen = pipeline.kmeans_cluster(z["rs_X"], n_clusters=200, seed=42, minibatch=False)
    assert np.array_equal(lab, z["rs_labels"])
    assert np.array_equal(bits(cen), bits(z["rs_centers"]))


@pytest.mark.parametrize("n,dim", [(17730, 64), (6040, 64), (6041, 100), (129, 3), (1, 5), (128, 64),
                                   (20000, 602), (100003, 41), (767, 9), (1537, 1)])
def test_standard_scaler_vs_oracle(n, dim):
    """The device scaler equals the oracle's numpy-order statistics: partial staged chunks (768 rows)
    and 64-row fold groups, 8-column groups with a partial last group, the Reddit feature width, a
    single row or column, a constant column."""
    from oracle import oracle as O
    from gdd import pipeline
    X = (np.random.default_rng(6).standard_normal((n, dim)) * 2 - 1).astype(np.float32)
    X[:, min(5, dim - 1)] = 3.0  # a constant column: scale 1
    out, mean, scale = pipeline.standard_scaler(X)
    ref, m_ref, s_ref = O.standard_scaler(X)
    assert np.array_equal(bits(out.cpu().numpy()), bits(ref))
    assert np.array_equal(mean.cpu().numpy(), m_ref) and np.array_equal(scale.cpu().numpy(), s_ref)


@pytest.mark.parametrize("tag", ["flickr", "reddit"])
def test_pretrained_clustering_induct_vs_reference(tag):
    """DataGraphSAINT's preparation + the inductive pretrained_clustering on the device (G7)."""
    from gdd import pipeline
    z = load(f"golden_clustgdd_induct_{tag}.npz")
    data = pipeline.graphsaint_split(_graph(z["rowptr"], z["col"]), z["feat_raw"], z["idx_train"],
                                     z["idx_val"], z["idx_test"])
    assert np.array_equal(bits(data.feat_full.cpu().numpy()), bits(z["feat_full"]))
    for name in ("train", "val", "test"):
        g = getattr(data, "adj_" + name)
        assert g.val is None  # binary stays binary
        assert np.array_equal(g.rowptr.cpu().numpy(), z[f"sub_{name}_rowptr"])
        assert np.array_equal(g.col.cpu().numpy(), z[f"sub_{name}_col"])
    k = int(z["n_syn"])
    np.random.set_state(rng_from_fixture(z).get_state())  # KMeans(random_state=None): global RNG
    feat_syn, labels_syn, cl, tgt, gn, tv, tt = pipeline.pretrained_clustering_induct_hot_path(
        data, int(z["T"]), float(z["alpha"]), z["kmeans_X"], k, dataset=tag, seed=15,
        cluster_minibatch=100)
    r, c, v = csr_to_sorted_coo(gn.rowptr.cpu().numpy(), gn.col.cpu().numpy(), gn.val.cpu().numpy())
    assert np.array_equal(r, z["norm_train_row"]) and np.array_equal(c, z["norm_train_col"])
    assert np.array_equal(bits(v), bits(z["norm_train_val"]))
    np.testing.assert_allclose(tgt.cpu().numpy(), z["target_train"], rtol=PROP_RTOL, atol=PROP_ATOL)
    np.testing.assert_allclose(tv.cpu().numpy(), z["target_val"], rtol=PROP_RTOL, atol=PROP_ATOL)
    assert tt.shape == (len(z["idx_test"]), z["feat_raw"].shape[1])
    assert np.array_equal(cl.cpu().numpy(), z["cluster_labels"])
    np.testing.assert_allclose(feat_syn.cpu().numpy(), z["feat_syn"], rtol=MEAN_RTOL, atol=MEAN_ATOL,
                               equal_nan=True)
    assert np.array_equal(labels_syn.cpu().numpy(), z["labels_syn"])
