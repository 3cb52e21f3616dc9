"""The GCN evaluator's SpMM on libgdd (gdd.gcn; SURVEY §8(f) row 3, models/gcn.py:36-51).

* CSR transpose: integer/index work, bit-exact against scipy's ``A.T.tocsr()``;
* forward and backward products: bit-exact against the oracle's canonical-order SpMM (oracle/), and
  within fp32 rounding of torch's own sparse product on the device (the reference's ``torch.spmm``),
  rtol 1e-5 / atol 1e-6;
* the reference layer (GraphConvolution) and a two-layer GCN forward against the same computation in
  plain torch with the same parameters.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import bits

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import gcn  # noqa: E402
from oracle import oracle as O  # noqa: E402

RTOL, ATOL = 1e-5, 1e-6


def _graph(n, deg, seed, weighted=True, sym=False):
    rng = np.random.default_rng(seed)
    m = n * deg
    r, c = rng.integers(0, n, m), rng.integers(0, n, m)
    v = (rng.random(m) + 0.1).astype(np.float32) if weighted else np.ones(m, np.float32)
    A = sp.coo_matrix((v, (r, c)), shape=(n, n)).tocsr()
    if sym:
        A = (A + A.T).tocsr()
    A.sum_duplicates()
    A.sort_indices()
    return A


def _torch_sparse(A):
    coo = A.tocoo()
    idx = torch.from_numpy(np.vstack([coo.row, coo.col]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(coo.data.astype(np.float32)), A.shape).coalesce().cuda()


@pytest.mark.parametrize("n,deg,weighted", [(1, 1, True), (500, 3, True), (4000, 9, False),
                                            (30000, 20, True)])
def test_transpose_matches_scipy(n, deg, weighted):
    A = _graph(n, deg, n, weighted)
    A[min(3, n - 1), :] = 0  # an empty row -> an empty column of the transpose
    A.eliminate_zeros()
    g = gdd.to_csr(A, binary=not weighted)
    t = gcn.transpose(g)
    ref = A.T.tocsr()
    ref.sort_indices()
    assert np.array_equal(t.rowptr.cpu().numpy(), ref.indptr)
    assert np.array_equal(t.col.cpu().numpy(), ref.indices)
    if weighted:
        assert np.array_equal(bits(t.val.cpu().numpy()), bits(ref.data))
    else:
        assert t.val is None
    assert gcn.transpose(t) is g  # cached both ways


@pytest.mark.parametrize("n,deg,d", [(700, 4, 7), (20000, 12, 256), (20000, 12, 40)])
def test_spmm_forward_backward(n, deg, d):
    A = _graph(n, deg, d)
    g = gdd.to_csr(A)
    rng = np.random.default_rng(d)
    xh = rng.standard_normal((n, d)).astype(np.float32)
    wh = rng.standard_normal((n, d)).astype(np.float32)
    x = torch.from_numpy(xh).cuda().requires_grad_(True)
    y = gcn.spmm(g, x)
    (y * torch.from_numpy(wh).cuda()).sum().backward()
    # canonical order: bit-exact vs the oracle (forward A @ x, backward Aᵀ @ w)
    assert np.array_equal(bits(y.detach().cpu().numpy()), bits(O.spmm(A.indptr, A.indices, A.data, xh)))
    At = A.T.tocsr()
    At.sort_indices()
    assert np.array_equal(bits(x.grad.cpu().numpy()), bits(O.spmm(At.indptr, At.indices, At.data, wh)))
    # the reference's torch.spmm on the device, same inputs
    xt = torch.from_numpy(xh).cuda().requires_grad_(True)
    yt = torch.sparse.mm(_torch_sparse(A), xt)
    (yt * torch.from_numpy(wh).cuda()).sum().backward()
    np.testing.assert_allclose(y.detach().cpu().numpy(), yt.detach().cpu().numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(x.grad.cpu().numpy(), xt.grad.cpu().numpy(), rtol=RTOL, atol=ATOL)


def test_graph_convolution_two_layer_gcn():
    # GCN.forward (models/gcn.py:101-113) with with_relu, eval mode (no dropout): log_softmax of
    # adj @ (relu(adj @ (X W1) + b1) W2) + b2, on the normalised adjacency
    A = _graph(5000, 6, 5, weighted=False, sym=True)
    gn = gdd.normalize_adj(gdd.to_csr(A))
    adj_t = _torch_sparse(gn.to_scipy())
    torch.manual_seed(0)
    l1, l2 = gcn.GraphConvolution(64, 256).cuda(), gcn.GraphConvolution(256, 10).cuda()
    X = torch.randn(5000, 64, device="cuda")
    with torch.no_grad():
        out = torch.log_softmax(l2(torch.relu(l1(X, gn)), gn), dim=1)
        ref = torch.log_softmax(torch.spmm(adj_t, torch.relu(torch.spmm(adj_t, X @ l1.weight) + l1.bias)
                                           @ l2.weight) + l2.bias, dim=1)
    np.testing.assert_allclose(out.cpu().numpy(), ref.cpu().numpy(), rtol=1e-4, atol=1e-5)
    # torch sparse adj keeps the reference path
    with torch.no_grad():
        same = l1(X, adj_t)
        plain = torch.spmm(adj_t, X @ l1.weight) + l1.bias
    np.testing.assert_allclose(same.cpu().numpy(), plain.cpu().numpy(), rtol=0, atol=0)
    # training step: gradients reach W through the libgdd backward
    loss = l2(torch.relu(l1(X, gn)), gn).square().mean()
    loss.backward()
    assert l1.weight.grad is not None and torch.isfinite(l1.weight.grad).all()
    assert repr(l1) == "GraphConvolution (64 -> 256)"
