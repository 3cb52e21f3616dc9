"""Induced sub-graphs on the device (gdd_subgraph_count/fill) against the oracle's restatement of
adj_full[np.ix_(idx, idx)] (utils_graphsaint.py:34-36). Integer work: bit-exact."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import bits

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _random_graph(n, deg, seed, weighted):
    rng = np.random.default_rng(seed)
    m = n * deg
    A = sp.coo_matrix((rng.random(m).astype(np.float32) + 0.5 if weighted else np.ones(m, np.float32),
                       (rng.integers(0, n, m), rng.integers(0, n, m))), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.sort_indices()
    return A


@pytest.mark.parametrize("n,deg,frac,weighted", [(1000, 5, 0.5, False), (20000, 12, 0.3, True),
                                                 (5000, 200, 0.6, False), (300, 2, 0.02, True)])
def test_induced_subgraph_matches_oracle(n, deg, frac, weighted):
    A = _random_graph(n, deg, n + deg, weighted)
    rng = np.random.default_rng(n)
    idx = np.sort(rng.choice(n, max(1, int(n * frac)), replace=False))
    g = gdd.to_csr(A, binary=not weighted)
    s = gdd.induced_subgraph(g, idx)
    rp, c, v = O.induced_subgraph(A.indptr, A.indices, A.data if weighted else None, idx)
    assert s.n == len(idx)
    assert np.array_equal(s.rowptr.cpu().numpy(), rp)
    assert np.array_equal(s.col.cpu().numpy(), c)
    if weighted:
        assert np.array_equal(bits(s.val.cpu().numpy()), bits(v))
    else:
        assert s.val is None
    ref = A[np.ix_(idx, idx)].tocsr()
    ref.sort_indices()
    assert np.array_equal(ref.indptr, rp) and np.array_equal(ref.indices, c)


def test_induced_subgraph_edge_cases():
    A = _random_graph(200, 3, 1, False)
    g = gdd.to_csr(A)
    # all nodes: identity
    s = gdd.induced_subgraph(g, np.arange(200))
    assert torch.equal(s.rowptr, g.rowptr) and torch.equal(s.col, g.col)
    # isolated selection: no surviving edge
    iso = np.where(np.asarray(A.sum(0)).ravel() + np.asarray(A.sum(1)).ravel() == 0)[0]
    one = gdd.induced_subgraph(g, np.array([5]))
    assert one.n == 1 and one.nnz == int(A[5, 5] != 0)
    if len(iso) > 1:
        e = gdd.induced_subgraph(g, iso)
        assert e.nnz == 0 and int(e.rowptr[-1]) == 0
    # device index tensor
    d = gdd.induced_subgraph(g, torch.arange(0, 200, 3, device="cuda"))
    ref = A[np.ix_(np.arange(0, 200, 3), np.arange(0, 200, 3))].tocsr()
    assert np.array_equal(d.col.cpu().numpy(), ref.indices)
    for bad in ([3, 2], [1, 1], [0, 200], [-1, 4]):
        with pytest.raises(ValueError):
            gdd.induced_subgraph(g, np.array(bad))
        # the same through a device index tensor: caught by the kernels' flag, no stray access
        with pytest.raises(ValueError):
            gdd.induced_subgraph(g, torch.tensor(bad, device="cuda"))


def test_graphsaint_split_scaler_matches_oracle():
    from gdd import pipeline
    rng = np.random.default_rng(3)
    n, d = 3000, 37
    A = _random_graph(n, 6, 2, False)
    X = (rng.standard_normal((n, d)) * 4 + 2).astype(np.float32)
    X[:, 3] = 1.5
    role = rng.choice(3, n)
    tr, va, te = (np.where(role == r)[0] for r in range(3))
    ns = pipeline.graphsaint_split(A, X, tr, va, te)
    _, mean, scale = O.standard_scaler(X[tr])
    full = O.scaler_transform(X, mean, scale)
    assert np.array_equal(bits(ns.feat_full.cpu().numpy()), bits(full))
    assert np.array_equal(bits(ns.feat_val.cpu().numpy()), bits(full[va]))
    for name, idx in (("train", tr), ("val", va), ("test", te)):
        ref = A[np.ix_(idx, idx)].tocsr()
        ref.sort_indices()
        sub = getattr(ns, "adj_" + name)
        assert np.array_equal(sub.rowptr.cpu().numpy(), ref.indptr)
        assert np.array_equal(sub.col.cpu().numpy(), ref.indices)


def test_load_graphsaint_files_vs_reference(tmp_path):
    # the G7 dataset written back in GraphSAINT's file format, read by load_graphsaint: the same
    # scaled features and role sub-graphs DataGraphSAINT produced (bit-exact)
    import json
    from gdd import pipeline
    from golden_util import load
    z = load("golden_clustgdd_induct_flickr.npz")
    n = len(z["rowptr"]) - 1
    A = sp.csr_matrix((np.ones(len(z["col"]), np.float32), z["col"], z["rowptr"]), shape=(n, n))
    sp.save_npz(tmp_path / "adj_full.npz", A)
    np.save(tmp_path / "feats.npy", z["feat_raw"])
    json.dump({"tr": z["idx_train"].tolist(), "va": z["idx_val"].tolist(), "te": z["idx_test"].tolist()},
              open(tmp_path / "role.json", "w"))
    json.dump({str(i): int(z["labels"][i]) for i in range(n)}, open(tmp_path / "class_map.json", "w"))
    ns = pipeline.load_graphsaint(str(tmp_path), "flickr")
    assert np.array_equal(bits(ns.feat_full.cpu().numpy()), bits(z["feat_full"]))
    assert ns.nclass == int(z["labels"].max()) + 1
    assert np.array_equal(ns.labels_train, z["labels"][z["idx_train"]])
    for name in ("train", "val", "test"):
        g = getattr(ns, "adj_" + name)
        assert np.array_equal(g.rowptr.cpu().numpy(), z[f"sub_{name}_rowptr"])
        assert np.array_equal(g.col.cpu().numpy(), z[f"sub_{name}_col"])
