"""HIP normalisation / propagation vs the CPU oracle (bit-exact) — needs a gfx950 GPU."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import synth  # noqa: E402


def _graph(n, deg, seed, kind="chung_lu"):
    return synth.chung_lu(n, deg, seed) if kind == "chung_lu" else synth.uniform_graph(n, deg, seed)


def _csr_host(A):
    A = sp.csr_matrix(A)
    return A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data.astype(np.float32)


@pytest.mark.parametrize("case", ["binary", "selfloop0", "weighted", "isolated", "empty_rows"])
def test_normalize_bitexact(case):
    n = 700
    A = _graph(n, 6.0, 3).tolil()
    self_loops = -1
    if case == "selfloop0":  # A[0,0] != 0 -> reference keeps fp32 and adds no I
        A[0, 0] = 1.0
    if case == "weighted":
        A = sp.csr_matrix(A)
        A.data = np.random.default_rng(0).uniform(0.1, 3.0, A.nnz).astype(np.float32)
    if case == "isolated":
        A = sp.csr_matrix(A)
        A[5, :] = 0
        A[:, 5] = 0
        A.eliminate_zeros()
    if case == "empty_rows":
        self_loops = 0
        A = sp.csr_matrix(A)
        A[7, :] = 0
        A.eliminate_zeros()
    A = sp.csr_matrix(A)
    A.sort_indices()
    rp, col, val = _csr_host(A)
    binary = case in ("binary", "isolated", "empty_rows")
    ro, co, vo = O.normalize_csr(rp, col, None if binary else val, self_loops)
    g = gdd.to_csr(A, binary=binary)
    gn = gdd.normalize_adj(g, self_loops=self_loops)
    assert np.array_equal(gn.rowptr.cpu().numpy(), ro)
    assert np.array_equal(gn.col.cpu().numpy(), co)
    assert np.array_equal(gn.val.cpu().numpy().view(np.uint32), vo.view(np.uint32))


# T >= 4 runs paired target updates (one hop defers its term to the next); float4 / float2 / float
# rows, odd and even hop counts, and the split hub row's fix-up path all take part
@pytest.mark.parametrize("d,T,alpha", [(128, 18, 0.91), (64, 5, 0.8), (7, 3, 0.5), (41, 4, 0.95),
                                       (602, 3, 0.95), (602, 6, 0.95), (100, 2, 0.91), (1, 1, 0.8),
                                       (3, 7, 0.8)])
def test_propagate_bitexact(d, T, alpha):
    n = 3000
    A = _graph(n, 12.0, 5)
    # a hub row long enough to be split into several segments (GDD_PROP_SEG = 256)
    A = A.tolil()
    A[11, :] = 0
    A[11, np.arange(0, n, 4)] = 1
    A = sp.csr_matrix(A)
    A.sort_indices()
    rp, col, _ = _csr_host(A)
    ro, co, vo = O.normalize_csr(rp, col, None, -1)
    X = synth.features(n, d, 9)
    t_ref, p_ref = O.propagate(ro, co, vo, X, T, alpha)
    g = gdd.normalize_adj(gdd.to_csr(A))
    t, p = gdd.propagate(g, torch.from_numpy(X).cuda(), T, alpha)
    assert np.array_equal(t.cpu().numpy().view(np.uint32), t_ref.view(np.uint32))
    assert np.array_equal(p.cpu().numpy().view(np.uint32), p_ref.view(np.uint32))


def test_propagate_vs_torch_reference_loop():
    """The reference loop with torch sparse mm (transduct:59-65) agrees within fp32 tolerance."""
    n, d, T, alpha = 2000, 32, 10, 0.9
    A = _graph(n, 8.0, 2)
    g = gdd.normalize_adj(gdd.to_csr(A))
    adj = g.to_torch_sparse()
    X = torch.from_numpy(synth.features(n, d, 4)).cuda()
    prop = X
    target = (1 - alpha) * prop
    for _ in range(1, T):
        prop = alpha * adj @ prop
        target = target + (1 - alpha) * prop
    t, p = gdd.propagate(g, X, T, alpha)
    torch.testing.assert_close(t, target, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p, prop, rtol=1e-5, atol=1e-6)


def test_spmm_matches_oracle():
    n, d = 1500, 48
    A = _graph(n, 10.0, 8)
    rp, col, _ = _csr_host(A)
    ro, co, vo = O.normalize_csr(rp, col, None, -1)
    x = synth.features(n, d, 1)
    y_ref = O.spmm(ro, co, vo, x, scale=0.7)
    g = gdd.normalize_adj(gdd.to_csr(A))
    y = gdd.spmm(g, torch.from_numpy(x).cuda(), 0.7)
    assert np.array_equal(y.cpu().numpy().view(np.uint32), y_ref.view(np.uint32))


@pytest.mark.parametrize("sched", ["", "hop_row_order", "hop_row_order,hop_xcd_contig"])
@pytest.mark.parametrize("d", [128, 40, 7])
def test_planned_hop_matches_oracle_and_accumulates(d, sched, monkeypatch):
    # gdd_spmm_plan once, then gdd_spmm_planned hops (the unit bench.py times): bit-exact with the
    # oracle's canonical order, including a hub row split into several segments; under each work-list
    # schedule (GDD_FORCE)
    if sched:
        monkeypatch.setenv("GDD_FORCE", sched)
    else:
        monkeypatch.delenv("GDD_FORCE", raising=False)
    n = 3000
    A = _graph(n, 12.0, 21)
    A = A.tolil()
    A[5, :] = 1.0  # a hub row of n entries (> GDD_PROP_SEG): the split-row fix-up path
    A = A.tocsr()
    rp, col, _ = _csr_host(A)
    ro, co, vo = O.normalize_csr(rp, col, None, -1)
    x = synth.features(n, d, 2)
    acc0 = synth.features(n, d, 3)
    y_ref = O.spmm(ro, co, vo, x, scale=0.91)
    acc_ref = (acc0 + np.float32(0.09) * y_ref).astype(np.float32)
    g = gdd.normalize_adj(gdd.to_csr(A))
    plan = gdd.graph.SpMMPlan(g, d)
    xd = torch.from_numpy(x).cuda()
    for _ in range(2):  # the plan is reusable
        y = torch.empty_like(xd)
        acc = torch.from_numpy(acc0).cuda()
        plan.hop(xd, y, 0.91, acc, 0.09)
        assert np.array_equal(y.cpu().numpy().view(np.uint32), y_ref.view(np.uint32))
        assert np.array_equal(acc.cpu().numpy().view(np.uint32), acc_ref.view(np.uint32))


@pytest.mark.parametrize("sched", ["", "hop_relabel_len", "hop_row_order,hop_xcd_contig"])
@pytest.mark.parametrize("relabel", ["degree", "rcm", "random"])
@pytest.mark.parametrize("d,T,alpha", [(128, 18, 0.91), (64, 5, 0.8), (41, 4, 0.95), (602, 3, 0.95),
                                       (100, 2, 0.91), (3, 7, 0.8)])
def test_propagate_relabeled_bitexact(relabel, d, T, alpha, sched, monkeypatch):
    """gdd_propagate_relabeled: the intermediate hops in another node order (rows of
    p at rho[r], gathers through rho[col], every row's entries in CSR order), the first hop reading
    X and the last storing p_last by the original ids, target by them throughout — target and p_last
    bit-identical to the oracle's, with the split hub row's fix-up and paired updates. sched: the
    work list in the new order (default, r06), longest first, or row order with XCD-contiguous
    ranges (GDD_FORCE; a schedule changes timing, never bits)."""
    if sched:
        monkeypatch.setenv("GDD_FORCE", sched)
    else:
        monkeypatch.delenv("GDD_FORCE", raising=False)
    n = 3000
    A = _graph(n, 12.0, 5).tolil()
    A[11, :] = 0
    A[11, np.arange(0, n, 4)] = 1
    A = sp.csr_matrix(A)
    A.sort_indices()
    rp, col, _ = _csr_host(A)
    ro, co, vo = O.normalize_csr(rp, col, None, -1)
    X = synth.features(n, d, 9)
    t_ref, p_ref = O.propagate(ro, co, vo, X, T, alpha)
    g = gdd.normalize_adj(gdd.to_csr(A))
    rho = np.random.default_rng(1).permutation(n).astype(np.int32) if relabel == "random" else relabel
    t, p = gdd.propagate(g, torch.from_numpy(X).cuda(), T, alpha, relabel=rho)
    assert np.array_equal(t.cpu().numpy().view(np.uint32), t_ref.view(np.uint32))
    assert np.array_equal(p.cpu().numpy().view(np.uint32), p_ref.view(np.uint32))
    with pytest.raises(ValueError):
        gdd.propagate(g, torch.from_numpy(X).cuda(), T, alpha, relabel=np.zeros(n, np.int32))


def test_locality_probe_schedule_bits(monkeypatch):
    """The hop's locality probe (r06, graphs of >= 1M rows): a community graph whose ids are in
    community order walks its rows in order, a shuffled one longest first — the schedule changes
    timing only: both equal the forced longest-first (hop_no_probe) and row-order results bit for bit."""
    for shuffle in (False, True):
        g = synth.sbm_device(1_050_000, 8.0, 3, block=1024, p_in=0.9, shuffle=shuffle)
        gn = gdd.normalize_adj(g)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(1)
        X = torch.randn(g.n, 12, device="cuda", generator=gen)
        outs = []
        for tok in ("", "hop_no_probe", "hop_row_order"):
            if tok:
                monkeypatch.setenv("GDD_FORCE", tok)
            else:
                monkeypatch.delenv("GDD_FORCE", raising=False)
            t, p = gdd.propagate(gn, X, 4, 0.9)
            outs.append((t.view(torch.int32).clone(), p.view(torch.int32).clone()))
        for t, p in outs[1:]:
            assert torch.equal(t, outs[0][0]) and torch.equal(p, outs[0][1])
