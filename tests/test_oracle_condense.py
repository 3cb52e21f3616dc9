"""CPU: the condensation restatement (oracle/condense.py) against the reference's own
graph_sparse / graph_compress / ER estimators run on golden_condense.npz (tools/make_golden.py G6).

What is bit-exact and what is a tolerance (and why) is stated per test."""
import numpy as np
import pytest

from golden_util import load
from oracle import condense as O

# cosine: torch reduces the C products (and the norms) in ATen's vectorised order, the
# restatement sequentially -> the reweighted values agree to a few fp32 ulps
REW_ATOL = 1e-6
# graph_compress: the reference's two fp32 products (P^T A, then (.) P) vs exact integer sums
COMPRESS_RTOL = 1e-5


@pytest.fixture(scope="module")
def z():
    return load("golden_condense.npz")


def _csr(z):
    r, c, v = z["norm_row"], z["norm_col"], z["norm_val"]
    n = z["ebd"].shape[0]
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, r.astype(np.int64) + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), r, c, v


def test_vanilla_er_bitexact(z):
    rowptr, r, c, v = _csr(z)
    assert np.array_equal(O.vanilla_er(rowptr, c, v).view(np.uint32), z["er_vanilla"].view(np.uint32))


def test_attaw_reweight_and_er(z):
    rowptr, r, c, v = _csr(z)
    er, rew = O.attaw_er(rowptr, c, v, z["ebd"])
    assert np.max(np.abs(rew - z["reweighted_val"])) <= REW_ATOL
    # given the reference's reweighted values, degrees and ER are bit-exact
    ref_rew = z["reweighted_val"]
    deg = O.row_sums(rowptr, ref_rew)
    er_ref = (ref_rew / deg[r] + ref_rew / deg[c]).astype(np.float32)
    assert np.array_equal(er_ref.view(np.uint32), z["er_attaw"].view(np.uint32))


@pytest.mark.parametrize("sp_type", ["attaw", "vanilla"])
def test_selection_matches_reference(z, sp_type):
    rowptr, r, c, v = _csr(z)
    sels, vals = O.graph_sparse(rowptr, c, v, float(z["ratio"]), z["ebd"], sp_type)
    assert len(sels) == int(z[f"{sp_type}_count"])
    for q, s in enumerate(sels):
        assert np.array_equal(r[s], z[f"{sp_type}{q}_row"])
        assert np.array_equal(c[s], z[f"{sp_type}{q}_col"])
        assert np.max(np.abs(vals[s] - z[f"{sp_type}{q}_val"])) <= REW_ATOL


def test_single_selection_up_to_boundary_ties(z):
    """'single' weighs by ER alone, which is symmetric: (i,j) and (j,i) tie exactly, and
    torch.topk's choice at the boundary is unspecified (libstdc++ introselect order). The
    selections may differ only by swapping edges whose weight equals the boundary weight."""
    rowptr, r, c, v = _csr(z)
    m = int(len(r) * float(z["ratio"]))
    s = O.topk_edges(z["er_attaw"], m)
    ref = set(zip(z["single0_row"].tolist(), z["single0_col"].tolist()))
    mine = set(zip(r[s].tolist(), c[s].tolist()))
    w = z["er_attaw"]
    idx = {(int(a), int(b)): e for e, (a, b) in enumerate(zip(r, c))}
    boundary = w[s].min()
    for edge in ref ^ mine:
        assert w[idx[edge]] == boundary
    assert len(ref ^ mine) <= 2


@pytest.mark.parametrize("tag", ["full", "gap"])
def test_compress_matches_reference(z, tag):
    rowptr, r, c, v = _csr(z)
    lab = z[f"{tag}_labels"]
    sels, rew = O.graph_sparse(rowptr, c, v, float(z["ratio"]), z["ebd"], "attaw")
    pairs = [(O.compress(lab, r, c, v), z[f"{tag}_adj_syn"])]
    pairs += [(O.compress(lab, r[s], c[s], rew[s]), z[f"{tag}_compressed{q}"])
              for q, s in enumerate(sels)]
    for a, ref in pairs:
        assert a.shape == ref.shape
        assert np.array_equal(np.isnan(a), np.isnan(ref))
        m = ~np.isnan(ref)
        assert np.all(np.abs(a[m] - ref[m]) <= COMPRESS_RTOL * np.abs(ref[m]) + 1e-9)
        assert np.all(np.diag(a)[~np.isnan(np.diag(a))] == 0)
    if tag == "gap":  # cluster 17 empty: NaN row and column, as the reference's 0/0 column of P
        a = pairs[0][0]
        assert np.isnan(a[17]).all() and np.isnan(a[:, 17]).all()


def test_topk_rule():
    w = np.array([1, 3, 3, np.nan, 2, 3, -0.0, 0.0], np.float32)
    assert O.topk_edges(w, 1).tolist() == [3]                 # NaN is largest
    assert O.topk_edges(w, 3).tolist() == [1, 2, 3]           # ties to the lower index
    assert O.topk_edges(w, 7).tolist() == [0, 1, 2, 3, 4, 5, 6]  # -0 ties with +0


def test_fixed_shift_headroom():
    vals = np.array([1.0, -0.5, 0.25], np.float32)
    s = O.fixed_shift(vals)
    q = np.rint(np.ldexp(np.abs(vals).astype(np.float64), s))
    assert q.sum() * (len(vals) + 1) < 2.0 ** 63
