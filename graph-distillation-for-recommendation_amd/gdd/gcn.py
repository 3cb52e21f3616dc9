"""The GCN evaluator's sparse product on MI355X.

The reference scores a distilled graph by training a GCN on it and evaluating every epoch on the full
graph: ``GraphConvolution.forward`` (ClustGDD/models/gcn.py:36-51) computes ``torch.spmm(adj, X @ W)``
with ``adj`` the normalised full adjacency (``_train_with_val``, :293-336: 600 epochs x 5 runs). That
product is the propagation hop's SpMM, so it runs on libgdd's planned hop (csrc/gdd_propagate.hip):

* :func:`spmm` — ``adj @ x`` for a :class:`gdd.graph.CSRGraph`, differentiable: the backward is
  ``adjᵀ @ grad`` on the transposed CSR (``gdd_csr_transpose``, built once per graph and cached);
* :class:`GraphConvolution` — the reference layer (same parameters, initialisation and forward) whose
  product goes through :func:`spmm` when ``adj`` is a CSRGraph (torch sparse / dense ``adj`` keep
  ``torch.spmm``, e.g. the small dense synthetic graph the GCN trains on).

Summation order: the canonical row-segment order of the hop (parity with torch's sparse kernels is a
tolerance, tests/test_gpu_gcn.py). The MLP/GCN training loop itself stays the caller's (out of scope).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib
from .graph import CSRGraph, SpMMPlan


def _plan(adj: CSRGraph, d: int) -> SpMMPlan:
    plans = adj.__dict__.setdefault("_plans", {})
    p = plans.get(d)
    if p is None:
        p = plans[d] = SpMMPlan(adj, d)
    return p


def transpose(adj: CSRGraph) -> CSRGraph:
    """Aᵀ as canonical CSR on the device (cached on ``adj``)."""
    t = adj.__dict__.get("_transpose")
    if t is not None:
        return t
    lib = _lib.device_lib()
    dev = adj.device
    rowptr = torch.empty(adj.n + 1, dtype=torch.int32, device=dev)
    col = torch.empty(max(adj.nnz, 1), dtype=torch.int32, device=dev)
    val = None if adj.val is None else torch.empty(max(adj.nnz, 1), dtype=torch.float32, device=dev)
    ws = _lib.workspace(lib.gdd_csr_transpose_ws_bytes(adj.n, adj.n, adj.nnz), dev)
    _lib.check(lib.gdd_csr_transpose(adj.n, adj.n, adj.nnz, adj.rowptr.data_ptr(), _lib.ptr(adj.col),
                                     _lib.ptr(adj.val), rowptr.data_ptr(), col.data_ptr(),
                                     _lib.ptr(val), None, ws.data_ptr(), ws.numel(),
                                     _lib.stream_ptr(dev)))
    t = CSRGraph(rowptr, col[:adj.nnz], None if val is None else val[:adj.nnz], adj.n)
    t.__dict__["_transpose"] = adj
    adj.__dict__["_transpose"] = t
    return t


def _product(adj: CSRGraph, x: torch.Tensor) -> torch.Tensor:
    x = x.detach().to(torch.float32).contiguous()
    if x.dim() != 2 or x.shape[0] != adj.n:
        raise ValueError(f"spmm: x must be [{adj.n}, d], got {tuple(x.shape)}")
    y = torch.empty_like(x)
    _plan(adj, x.shape[1]).hop(x, y)
    return y


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, adj):
        ctx.adj = adj
        return _product(adj, x)

    @staticmethod
    def backward(ctx, grad):
        return _product(transpose(ctx.adj), grad), None


def spmm(adj: CSRGraph, x: torch.Tensor) -> torch.Tensor:
    """``torch.spmm(adj, x)`` for a CSRGraph on libgdd (autograd: backward = adjᵀ @ grad)."""
    if x.requires_grad and torch.is_grad_enabled():
        return _SpMM.apply(x, adj)
    return _product(adj, x)


class GraphConvolution(nn.Module):
    """models/gcn.py:13-51: ``output = adj @ (input @ W) (+ bias)``; W in_features x out_features,
    both initialised uniform(-1/sqrt(out_features), +1/sqrt(out_features)) (:30-34)."""

    def __init__(self, in_features: int, out_features: int, with_bias: bool = True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(in_features, out_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if with_bias else None
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.weight.T.size(1))
        self.weight.data.uniform_(-stdv, stdv)
        if self.bias is not None:
            self.bias.data.uniform_(-stdv, stdv)

    def forward(self, input, adj):
        support = torch.spmm(input, self.weight) if input.is_sparse else torch.mm(input, self.weight)
        output = spmm(adj, support) if isinstance(adj, CSRGraph) else torch.spmm(adj, support)
        return output + self.bias if self.bias is not None else output

    def __repr__(self):
        return f"{self.__class__.__name__} ({self.in_features} -> {self.out_features})"
