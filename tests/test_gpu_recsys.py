"""The recommender condensation and refinement model on libgdd (gdd.recsys).

* build_condensed_bipartite: integer work, bit-exact against the reference's output (G8) and the
  oracle (oracle/recsys.py) on larger random inputs, with empty super-nodes, all-duplicate input
  and out-of-range ids;
* LightGCNCondensed.propagate / bpr_loss / every parameter gradient against the reference model run
  on CPU with the same parameters (G8): the message passing sums in CSR order instead of index_add_'s,
  so fp32 tolerances (outputs rtol 1e-5 / atol 1e-6, gradients rtol 1e-4 / atol 1e-7).
"""
import numpy as np
import pytest
import torch

from golden_util import load

pytestmark = pytest.mark.gpu

from gdd import recsys  # noqa: E402
from oracle import recsys as R  # noqa: E402


def _check(C, rp, c, v):
    assert np.array_equal(C.rowptr.cpu().numpy(), rp)
    assert np.array_equal(C.col.cpu().numpy(), c)
    assert np.array_equal(C.val.cpu().numpy(), v)


def test_condense_vs_reference():
    z = load("golden_recsys.npz")
    C = recsys.build_condensed_bipartite(z["train_u"], z["train_i"], z["u2cu"], z["i2ci"],
                                         int(z["num_cu"]), int(z["num_ci"]))
    _check(C, z["C_indptr"], z["C_indices"], z["C_data"])
    ref = C.to_scipy()
    assert ref.shape == (int(z["num_cu"]), int(z["num_ci"]))
    ei, w = recsys.condensed_csr_to_edge_index(C)
    assert np.array_equal(ei.cpu().numpy(), z["edge_index"]) and np.array_equal(w.cpu().numpy(), z["w0"])


@pytest.mark.parametrize("nu,ni,E,ncu,nci", [(6040, 3706, 1_000_209, 604, 371),
                                             (20, 10, 5000, 3, 2), (50000, 80000, 300000, 5000, 8000)])
def test_condense_vs_oracle(nu, ni, E, ncu, nci):
    rng = np.random.default_rng(E)
    tu = rng.integers(0, nu, E)
    ti = (rng.zipf(1.5, E) % ni)
    u2cu = rng.integers(0, ncu, nu)
    i2ci = rng.integers(0, nci, ni)
    C = recsys.build_condensed_bipartite(tu, ti, u2cu, i2ci, ncu, nci)
    _check(C, *R.build_condensed_bipartite(tu, ti, u2cu, i2ci, ncu, nci))


def test_condense_edge_cases():
    # one pair repeated: a single stored count
    C = recsys.build_condensed_bipartite(np.zeros(1000, int), np.zeros(1000, int), [1], [0], 3, 1)
    _check(C, np.array([0, 0, 1, 1]), np.array([1 - 1]), np.array([1000.0], np.float32))
    with pytest.raises(IndexError):
        recsys.build_condensed_bipartite([0, 5], [0, 0], [0, 1], [0], 2, 1)  # user 5 unknown
    with pytest.raises(IndexError):
        recsys.build_condensed_bipartite([0, 1], [0, 0], [0, 7], [0], 2, 1)  # cluster 7 >= num_cu


def _model(z):
    ei = torch.from_numpy(z["edge_index"]).cuda()
    m = recsys.LightGCNCondensed(int(z["num_cu"]), int(z["num_ci"]), int(z["dim"]), int(z["layers"]), ei,
                                 torch.from_numpy(z["w0"]).cuda(), device=torch.device("cuda")).cuda()
    with torch.no_grad():
        for k, p in m.named_parameters():
            p.copy_(torch.from_numpy(z["param_" + k.replace(".", "_")]))
    return m


def test_lightgcn_propagate_and_grads_vs_reference():
    z = load("golden_recsys.npz")
    m = _model(z)
    u_out, i_out = m.propagate()
    np.testing.assert_allclose(u_out.detach().cpu().numpy(), z["u_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(i_out.detach().cpu().numpy(), z["i_out"], rtol=1e-5, atol=1e-6)
    loss = m.bpr_loss(torch.from_numpy(z["bpr_u"]).cuda(), torch.from_numpy(z["bpr_pos"]).cuda(),
                      torch.from_numpy(z["bpr_neg"]).cuda(), reg_lambda=1e-4)
    assert abs(loss.item() - float(z["loss"])) <= 1e-6
    loss.backward()
    for k, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), z["grad_" + k.replace(".", "_")], rtol=1e-4,
                                   atol=1e-7, err_msg=k)


def test_lightgcn_rejects_unsorted_edges():
    z = load("golden_recsys.npz")
    ei = torch.from_numpy(z["edge_index"][:, ::-1].copy()).cuda()
    m = recsys.LightGCNCondensed(int(z["num_cu"]), int(z["num_ci"]), 4, 1, ei,
                                 torch.from_numpy(z["w0"][::-1].copy()).cuda(), device=torch.device("cuda"))
    with pytest.raises(ValueError):
        m.cuda().propagate()
