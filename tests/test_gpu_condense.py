"""HIP condensation (graph_sparse / graph_compress / ER estimators) vs the CPU restatement
(bit-exact) and vs the reference fixture (golden_condense.npz) — needs a gfx950 GPU."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import load
from oracle import condense as O

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import condense as GC  # noqa: E402
from gdd import synth  # noqa: E402


def _bits(t):
    return np.ascontiguousarray(t.cpu().numpy() if isinstance(t, torch.Tensor) else t,
                                dtype=np.float32).view(np.uint32)


def _normalized(n, deg, seed):
    A = synth.chung_lu(n, deg, seed)
    gn = gdd.normalize_adj(gdd.to_csr(A))
    return gn, gn.rowptr.cpu().numpy(), gn.col.cpu().numpy(), gn.val.cpu().numpy()


def _fixture_graph(z):
    r, c, v = z["norm_row"], z["norm_col"], z["norm_val"]
    n = z["ebd"].shape[0]
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))
    A.sort_indices()
    return gdd.to_csr(A, binary=False), A.indptr.astype(np.int32), r, c, v


@pytest.mark.parametrize("n,deg,C", [(500, 8.0, 5), (20000, 10.0, 41), (3000, 6.0, 7)])
def test_er_and_softmax_bitexact(n, deg, C):
    gn, rp, col, val = _normalized(n, deg, 71)
    ebd = (np.random.default_rng(n).standard_normal((n, C)) * 2).astype(np.float32)
    er_ref, rew_ref = O.attaw_er(rp, col, val, ebd)
    er, g = GC.attaw_ER_estimator(gn, torch.from_numpy(ebd).cuda())
    assert np.array_equal(_bits(g.val), _bits(rew_ref))
    assert np.array_equal(_bits(er), _bits(er_ref))
    assert np.array_equal(_bits(GC.ER_estimator(gn)), _bits(O.vanilla_er(rp, col, val)))
    p = GC.softmax_rows(torch.from_numpy(ebd).cuda())
    assert np.array_equal(_bits(p), _bits(O.softmax_rows(ebd)))


@pytest.mark.parametrize("sp_type", ["attaw", "vanilla", "single"])
@pytest.mark.parametrize("n,deg,C,ratio", [(500, 8.0, 5, 0.4), (20000, 10.0, 41, 0.1)])
def test_graph_sparse_bitexact(sp_type, n, deg, C, ratio):
    gn, rp, col, val = _normalized(n, deg, 72)
    ebd = (np.random.default_rng(n + 1).standard_normal((n, C)) * 2).astype(np.float32)
    sels, vals = O.graph_sparse(rp, col, val, ratio, ebd, sp_type)
    out = GC.graph_sparse(gn, ratio, torch.from_numpy(ebd).cuda(), sp_type)
    assert len(out) == len(sels)
    rows = O.coo_rows(rp)
    for g, s in zip(out, sels):
        gr = g.rowptr.cpu().numpy()
        assert np.array_equal(O.coo_rows(gr), rows[s])
        assert np.array_equal(g.col.cpu().numpy(), col[s])
        assert np.array_equal(_bits(g.val), _bits(vals[s]))


def test_topk_ties_nan_and_zero():
    n = 64
    A = sp.random(n, n, density=0.3, random_state=3, format="csr", dtype=np.float32)
    A.data[:] = 1.0
    A.sort_indices()
    g = gdd.to_csr(A, binary=False)
    w = np.random.default_rng(4).integers(0, 5, g.nnz).astype(np.float32)
    w[::17] = np.nan
    w[3::29] = -0.0
    for m in (0, 1, 7, g.nnz // 2, g.nnz):
        sel = GC.topk_edges(g, torch.from_numpy(w).cuda(), m)[0].cpu().numpy()
        assert np.array_equal(sel, O.topk_edges(w, m)), m


@pytest.mark.parametrize("k,empty", [(40, None), (40, 17), (454, None), (7, 6)])
def test_graph_compress_bitexact(k, empty):
    n = 20000 if k == 454 else 3000
    gn, rp, col, val = _normalized(n, 10.0, 73)
    lab = np.random.default_rng(k).integers(0, k, n).astype(np.int32)
    lab[: k] = np.arange(k)
    if empty is not None:  # an empty cluster below the largest label -> NaN row/column
        lab[lab == empty] = (empty + 1) % k
    ebd = np.random.default_rng(5).standard_normal((n, 5)).astype(np.float32)
    sels, rew = O.graph_sparse(rp, col, val, 0.3, ebd, "attaw")
    subs = GC.graph_sparse(gn, 0.3, torch.from_numpy(ebd).cuda(), "attaw")
    comp, adj_syn = GC.graph_compress(torch.from_numpy(lab), gn, subs)
    rows = O.coo_rows(rp)
    ref_syn = O.compress(lab, rows, col, val)
    assert np.array_equal(_bits(adj_syn.to_dense()), _bits(ref_syn))
    for c_dev, s in zip(comp, sels):
        ref = O.compress(lab, rows[s], col[s], rew[s])
        assert np.array_equal(_bits(c_dev.to_dense()), _bits(ref))
    d = adj_syn.to_dense().cpu().numpy()
    if empty == k - 1:  # the largest cluster empty: cluster_num = max + 1 shrinks P (transduct:236)
        assert d.shape == (k - 1, k - 1)
    elif empty is not None:
        assert np.isnan(d[empty]).all() and np.isnan(d[:, empty]).all()


def test_against_reference_fixture():
    """Device vs the reference's own graph_sparse('attaw'/'vanilla') and graph_compress."""
    z = load("golden_condense.npz")
    g, rp, r, c, v = _fixture_graph(z)
    ebd = torch.from_numpy(z["ebd"]).cuda()
    ratio = float(z["ratio"])
    for sp_type in ("attaw", "vanilla"):
        out = GC.graph_sparse(g, ratio, ebd, sp_type)
        assert len(out) == int(z[f"{sp_type}_count"])
        for q, s in enumerate(out):
            rows = O.coo_rows(s.rowptr.cpu().numpy())
            assert np.array_equal(rows, z[f"{sp_type}{q}_row"])
            assert np.array_equal(s.col.cpu().numpy(), z[f"{sp_type}{q}_col"])
            assert np.max(np.abs(s.val.cpu().numpy() - z[f"{sp_type}{q}_val"])) <= 1e-6
    subs = GC.graph_sparse(g, ratio, ebd, "attaw")
    for tag in ("full", "gap"):
        comp, adj_syn = GC.graph_compress(torch.from_numpy(z[f"{tag}_labels"]), g, subs)
        pairs = [(adj_syn, z[f"{tag}_adj_syn"])] + [(cc, z[f"{tag}_compressed{q}"])
                                                  for q, cc in enumerate(comp)]
        for dev, ref in pairs:
            a = dev.to_dense().cpu().numpy()
            assert np.array_equal(np.isnan(a), np.isnan(ref))
            m = ~np.isnan(ref)
            assert np.all(np.abs(a[m] - ref[m]) <= 1e-5 * np.abs(ref[m]) + 1e-9)


def test_no_sp_and_rand():
    """'no_sp' hands the graph back; 'rand' (clustgdd_agent_transduct.py:207-222) takes, per class, the
    first int(nnz * ratio) edges of torch.randperm(nnz) on torch's global CPU generator, carrying their
    ER_estimator weights (the reference's "tried version" values)."""
    gn, rp, col, val = _normalized(300, 5.0, 74)
    assert GC.graph_sparse(gn, 0.5, None, "no_sp")[0] is gn
    with pytest.raises(ValueError):
        GC.graph_sparse(gn, 0.5, None, "rand")
    ebd = torch.zeros((300, 3))
    torch.manual_seed(7)
    graphs = GC.graph_sparse(gn, 0.5, ebd, "rand")
    er = O.vanilla_er(rp, col, val)
    rows = np.repeat(np.arange(300), np.diff(rp))
    torch.manual_seed(7)
    m = int(gn.nnz * 0.5)
    assert len(graphs) == 3
    for g in graphs:
        pick = np.sort(torch.randperm(gn.nnz)[:m].numpy())
        A = g.to_scipy().tocoo()
        o = np.lexsort((A.col, A.row))
        assert np.array_equal(A.row[o], rows[pick]) and np.array_equal(A.col[o], col[pick])
        assert np.array_equal(_bits(A.data[o].astype(np.float32)), _bits(er[pick]))
