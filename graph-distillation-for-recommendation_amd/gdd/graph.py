"""Graph side of the ClustGDD hot path on MI355X: CSR upload, normalisation, propagation.

Drop-in for
* ``deep_robust_utils.to_tensor`` / ``sparse_mx_to_torch_sparse_tensor`` (ClustGDD/deep_robust_utils.py:85-113,
  :389-396) — :func:`to_csr` takes the same inputs (scipy sparse, torch sparse, dense array) and
  keeps CSR (int32 rowptr/col, fp32 values) resident in HBM instead of an int64 COO tensor;
* ``deep_robust_utils.normalize_adj_tensor(adj, sparse=True)`` (:245-256) — :func:`normalize_adj_tensor`;
* the propagation loop of ``ClustGDD.pretrained_clustering`` (clustgdd_agent_transduct.py:55-65,
  clustgdd_agent_induct.py:67-94) — :func:`propagate`.
All arithmetic runs in libgdd (HIP, gfx950); this module only moves buffers and checks shapes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib


@dataclass
class CSRGraph:
    """A square sparse matrix resident on the GPU as canonical CSR."""

    rowptr: torch.Tensor  # int32 [n+1]
    col: torch.Tensor  # int32 [nnz]
    val: Optional[torch.Tensor]  # fp32 [nnz]; None = all ones (binary adjacency)
    n: int

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    @property
    def shape(self):
        return (self.n, self.n)

    def values(self) -> torch.Tensor:
        if self.val is None:
            return torch.ones(self.nnz, dtype=torch.float32, device=self.device)
        return self.val

    def to_scipy(self) -> sp.csr_matrix:
        return sp.csr_matrix((self.values().cpu().numpy(), self.col.cpu().numpy(),
                              self.rowptr.cpu().numpy()), shape=self.shape)

    def to_torch_sparse(self) -> torch.Tensor:
        """COO view with the reference's index/value dtypes (int64 / fp32)."""
        rp = self.rowptr.long()
        rows = torch.repeat_interleave(torch.arange(self.n, device=self.device),
                                       rp[1:] - rp[:-1])
        idx = torch.stack([rows, self.col.long()])
        return torch.sparse_coo_tensor(idx, self.values(), self.shape).coalesce()


def to_csr(adj, device="cuda", binary: Optional[bool] = None) -> CSRGraph:
    """Upload an adjacency matrix (scipy sparse / torch sparse / dense) as canonical CSR.

    Duplicates are summed and columns sorted, as scipy's csr_matrix construction in
    ``deep_robust_utils.to_scipy`` (:408-417) does. ``binary=None`` detects an all-ones value
    array and then stores no values (the kernels read 1.0f).
    """
    if isinstance(adj, torch.Tensor):
        if adj.is_sparse:
            a = adj.coalesce()
            idx = a.indices().cpu().numpy()
            m = sp.csr_matrix((a.values().cpu().numpy().astype(np.float32), (idx[0], idx[1])),
                              shape=tuple(a.shape))
        elif adj.layout == torch.sparse_csr:
            m = sp.csr_matrix((adj.values().cpu().numpy(), adj.col_indices().cpu().numpy(),
                               adj.crow_indices().cpu().numpy()), shape=tuple(adj.shape))
        else:
            m = sp.csr_matrix(adj.detach().cpu().numpy())
    elif sp.issparse(adj):
        m = sp.csr_matrix(adj)
    else:
        m = sp.csr_matrix(np.asarray(adj))
    if m.shape[0] != m.shape[1]:
        raise ValueError(f"adjacency must be square, got {m.shape}")
    m = m.astype(np.float32)
    m.sum_duplicates()
    m.sort_indices()
    if m.nnz >= 2**31 - m.shape[0]:
        raise ValueError("graph too large for int32 CSR")
    dev = torch.device(device)
    vals = m.data
    if binary is None:
        binary = bool(np.all(vals == 1.0))
    rowptr = torch.from_numpy(m.indptr.astype(np.int32)).to(dev)
    col = torch.from_numpy(m.indices.astype(np.int32)).to(dev)
    val = None if binary else torch.from_numpy(vals.astype(np.float32)).to(dev)
    return CSRGraph(rowptr, col, val, m.shape[0])


def normalize_adj(adj: CSRGraph, self_loops: int = -1) -> CSRGraph:
    """Â = D^-1/2 (A + I) D^-1/2 (deep_robust_utils.normalize_adj, :180-207).

    self_loops=-1 is the reference rule: I is added only if A[0,0] == 0 (:199-200); fp64 math
    then, fp32 otherwise. Output is canonical CSR with fp32 values.
    """
    lib = _lib.device_lib()
    dev = adj.device
    n, nnz = adj.n, adj.nnz
    rowptr_out = torch.empty(n + 1, dtype=torch.int32, device=dev)
    col_out = torch.empty(nnz + n, dtype=torch.int32, device=dev)
    val_out = torch.empty(nnz + n, dtype=torch.float32, device=dev)
    ws = _lib.workspace(lib.gdd_normalize_ws_bytes(n, nnz), dev)
    _lib.check(lib.gdd_normalize_csr(n, nnz, adj.rowptr.data_ptr(), _lib.ptr(adj.col),
                                     _lib.ptr(adj.val), int(self_loops), rowptr_out.data_ptr(),
                                     col_out.data_ptr(), val_out.data_ptr(), ws.data_ptr(),
                                     ws.numel(), _lib.stream_ptr(dev)))
    nnz_out = int(rowptr_out[n].item())
    return CSRGraph(rowptr_out, col_out[:nnz_out], val_out[:nnz_out], n)


def induced_subgraph(adj: CSRGraph, idx) -> CSRGraph:
    """``adj[np.ix_(idx, idx)]`` on the device, canonical CSR (utils_graphsaint.py:34-36: the
    inductive agent's ``adj_train/val/test``, clustgdd_agent_induct.py:38-94).

    ``idx`` (host array or device tensor of node ids) must be strictly increasing, as GraphSAINT's
    role lists are; the kernels flag any other order and this raises ValueError. Values are kept
    (a binary graph stays binary).
    """
    lib = _lib.device_lib()
    dev = adj.device
    if isinstance(idx, torch.Tensor):
        ix = idx.to(device=dev, dtype=torch.int32).contiguous()
    else:
        h = np.asarray(idx, dtype=np.int64)
        if h.size and (h.min() < 0 or h.max() >= adj.n or np.any(np.diff(h) <= 0)):
            raise ValueError("induced_subgraph: idx must be strictly increasing node ids in [0, n)")
        ix = torch.from_numpy(np.ascontiguousarray(h.astype(np.int32))).to(dev)
    m = int(ix.numel())
    if m == 0:
        raise ValueError("induced_subgraph: empty node set")
    rowptr = torch.empty(m + 1, dtype=torch.int32, device=dev)
    ws = _lib.workspace(lib.gdd_subgraph_ws_bytes(adj.n, m), dev)
    st = _lib.stream_ptr(dev)
    _lib.check(lib.gdd_subgraph_count(adj.n, adj.rowptr.data_ptr(), _lib.ptr(adj.col), m,
                                      ix.data_ptr(), rowptr.data_ptr(), ws.data_ptr(), ws.numel(), st))
    nnz = int(rowptr[m].item())
    col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    val = None if adj.val is None else torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(lib.gdd_subgraph_fill(adj.n, adj.rowptr.data_ptr(), _lib.ptr(adj.col),
                                     _lib.ptr(adj.val), m, ix.data_ptr(), rowptr.data_ptr(),
                                     col.data_ptr(), _lib.ptr(val), bad.data_ptr(), ws.data_ptr(),
                                     ws.numel(), st))
    if int(bad.item()):
        raise ValueError("induced_subgraph: idx must be strictly increasing node ids in [0, n)")
    return CSRGraph(rowptr, col[:nnz], None if val is None else val[:nnz], m)


def normalize_adj_tensor(adj, sparse: bool = True, device=None) -> CSRGraph:
    """Drop-in for deep_robust_utils.normalize_adj_tensor(adj, sparse=True) (:245-256)."""
    if not sparse:
        raise NotImplementedError("dense normalisation is outside the MI355X hot path")
    if not isinstance(adj, CSRGraph):
        adj = to_csr(adj, device=device or "cuda")
    return normalize_adj(adj)


def _ws_propagate(adj: CSRGraph, d: int):
    lib = _lib.device_lib()
    return lib, _lib.workspace(lib.gdd_propagate_ws_bytes(adj.n, adj.nnz, d), adj.device)


def locality_order(adj: CSRGraph, kind: str = "degree") -> torch.Tensor:
    """A node relabelling for :func:`propagate`'s ``relabel`` (rho: node r's row of the intermediate
    hops at rho[r], int32 on the graph's device). ``"degree"``: rows by descending length, ties by id
    (the hubs every hop gathers most sit together); ``"rcm"``: reverse Cuthill-McKee of the pattern
    (scipy, on the host), which recovers the community blocks of a graph whose ids were shuffled."""
    dev = adj.device
    n = adj.n
    if kind == "degree":
        deg = (adj.rowptr[1:] - adj.rowptr[:-1]).to(torch.int64)
        order = torch.sort(-deg, stable=True).indices
    elif kind == "rcm":
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        order = torch.from_numpy(np.ascontiguousarray(
            reverse_cuthill_mckee(adj.to_scipy().tocsr(), symmetric_mode=True), np.int64)).to(dev)
    else:
        raise ValueError(f"unknown locality order {kind!r}")
    rho = torch.empty(n, dtype=torch.int32, device=dev)
    rho[order] = torch.arange(n, dtype=torch.int32, device=dev)
    return rho


def propagate(adj_norm: CSRGraph, features: torch.Tensor, T: int, alpha: float, group=None,
              relabel=None):
    """The closed-form feature denoising loop of pretrained_clustering (transduct:55-65).

    Returns ``(target_feat, prop_feat)`` exactly as the loop leaves them: ``target_feat =
    (1-α)·Σ_{t<T} (αÂ)^t X`` accumulated hop by hop in fp32, ``prop_feat`` = the last hop.
    ``group`` (a torch.distributed group over the GPUs of a node): when the size model of
    :func:`gdd.sharded.propagation_shards_pay` says the gathers outweigh a per-hop all-gather
    (ogbn-products, not ogbn-arxiv), the rows are partitioned over the ranks
    (:func:`gdd.sharded.sharded_propagate`, bit-identical); otherwise every rank propagates.
    ``relabel`` (opt-in): ``"degree"``, ``"rcm"`` or a permutation rho (node r -> row rho[r]): the
    intermediate hops run in that node order (gdd_propagate_relabeled) — same bits, different
    gather locality.
    """
    # the same input checks for both paths (the sharded dispatch used to come first)
    if T < 1:
        raise ValueError("prop_num must be >= 1 (the reference loop leaves target undefined)")
    X = features.contiguous()
    if X.dtype != torch.float32:
        raise TypeError("features must be float32")
    if X.device != adj_norm.device:
        raise ValueError("features and adjacency must be on the same device")
    n, d = X.shape
    if n != adj_norm.n:
        raise ValueError(f"features have {n} rows, adjacency {adj_norm.n}")
    if group is not None:
        from .sharded import propagation_shards_pay, sharded_propagate, world_of
        world = world_of(group)[1]
        if world > 1 and propagation_shards_pay(adj_norm.n, adj_norm.nnz, d, world):
            if relabel is not None:  # never drop a caller's relabel silently
                raise ValueError("relabel cannot be combined with the row-partitioned propagation "
                                 "this group selects (pass group=None, or relabel=None)")
            return sharded_propagate(adj_norm, X, T, alpha, group=group)
    if relabel is not None:
        rho = locality_order(adj_norm, relabel) if isinstance(relabel, str) else relabel
        rho = torch.as_tensor(rho, device=X.device).to(torch.int32).contiguous()
        if rho.shape != (n,) or not torch.equal(torch.sort(rho).values,
                                               torch.arange(n, dtype=torch.int32, device=X.device)):
            raise ValueError("relabel must be a permutation of range(n)")
        lib = _lib.device_lib()
        ws = _lib.workspace(lib.gdd_propagate_relabeled_ws_bytes(n, adj_norm.nnz, d), X.device)
        target = torch.empty_like(X)
        p_last = torch.empty_like(X)
        p_tmp = torch.empty_like(X) if T > 2 else None
        _lib.check(lib.gdd_propagate_relabeled(
            n, adj_norm.nnz, adj_norm.rowptr.data_ptr(), _lib.ptr(adj_norm.col),
            _lib.ptr(adj_norm.values()), rho.data_ptr(), d, X.data_ptr(), int(T), float(alpha),
            target.data_ptr(), p_last.data_ptr(), _lib.ptr(p_tmp), ws.data_ptr(), ws.numel(),
            _lib.stream_ptr(X.device)))
        return target, p_last
    lib, ws = _ws_propagate(adj_norm, d)
    target = torch.empty_like(X)
    p_last = torch.empty_like(X)
    p_tmp = torch.empty_like(X) if T > 2 else None
    _lib.check(lib.gdd_propagate(n, adj_norm.nnz, adj_norm.rowptr.data_ptr(),
                                 _lib.ptr(adj_norm.col), _lib.ptr(adj_norm.values()), d,
                                 X.data_ptr(), int(T), float(alpha), target.data_ptr(),
                                 p_last.data_ptr(), _lib.ptr(p_tmp), ws.data_ptr(), ws.numel(),
                                 _lib.stream_ptr(X.device)))
    return target, p_last


def spmm(adj: CSRGraph, x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """y = (scale·A) @ x in the canonical order (also the GCN evaluator's torch.spmm)."""
    x = x.contiguous()
    lib, ws = _ws_propagate(adj, x.shape[1])
    y = torch.empty_like(x)
    _lib.check(lib.gdd_spmm(adj.n, adj.nnz, adj.rowptr.data_ptr(), _lib.ptr(adj.col),
                            _lib.ptr(adj.values()), x.shape[1], float(scale), x.data_ptr(),
                            y.data_ptr(), None, 0.0, ws.data_ptr(), ws.numel(),
                            _lib.stream_ptr(x.device)))
    return y


class SpMMPlan:
    """A CSR structure's row-segment work list, built once (gdd_spmm_plan); each :meth:`hop`
    is then one planned SpMM launch pair (gdd_spmm_planned) with the canonical summation order."""

    def __init__(self, adj: CSRGraph, d: int):
        self.adj, self.d = adj, d
        self.lib, self.ws = _ws_propagate(adj, d)
        _lib.check(self.lib.gdd_spmm_plan(adj.n, adj.nnz, adj.rowptr.data_ptr(), d,
                                          self.ws.data_ptr(), self.ws.numel(),
                                          _lib.stream_ptr(adj.device)))

    def hop(self, x: torch.Tensor, y: torch.Tensor, scale: float = 1.0, acc: torch.Tensor = None,
            acc_scale: float = 0.0) -> torch.Tensor:
        """y = (scale·A) @ x; with acc also acc = acc + acc_scale * y (two fp32 roundings)."""
        a = self.adj
        _lib.check(self.lib.gdd_spmm_planned(
            a.n, a.nnz, a.rowptr.data_ptr(), _lib.ptr(a.col), _lib.ptr(a.values()), self.d,
            float(scale), x.data_ptr(), y.data_ptr(), _lib.ptr(acc), float(acc_scale),
            self.ws.data_ptr(), self.ws.numel(), _lib.stream_ptr(x.device)))
        return y
