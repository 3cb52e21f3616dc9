"""Range-partitioned Lloyd k-means across ranks: one all-reduce per iteration.

The reference runs ``KMeans(n_clusters=k).fit(X)`` on one host (clustgdd_agent_transduct.py:104-105,
distill_recsys.py:178). For graphs whose rows are spread over the GPUs of a node, each rank holds a
contiguous shard of X and the centres are replicated:

* init: the shards are all-gathered once and every rank runs the same k-means++ with the same
  RandomState (sklearn _kmeans_plusplus, ``gdd_kmeans_plusplus``), so the initial centres agree
  bit for bit without a broadcast — the one up-front exchange;
* iteration: local MFMA assignment (``gdd_kmeans_assign``), local per-cluster sums in int64 fixed
  point (``gdd_segment_sum_fixed``: llrint(x·2^s), exact integer adds), ONE all-reduce of
  [k·dim sums ‖ k counts ‖ labels-changed], then ``gdd_fixed_to_centers``. Integer sums are
  associative, so every world size — 1, 2, 4, 8 — produces the same centres and labels;
* stop: labels unchanged on every rank (strict convergence), or Σ‖ΔC‖² ≤ tol·mean(var(X))
  (sklearn _kmeans.py:717-734), followed by the final E-step when the stop was not strict.

Scikit-learn's single-threaded fp32 M-step sums (which ``gdd.KMeans`` reproduces bit for bit on one
GPU) cannot be split across ranks without changing their rounding; this class instead guarantees
rank-count invariance, with centres within fp32 rounding of the sequential ones. Empty clusters
keep their previous centre (sklearn relocates them to far points; documented deviation).

The device primitives come from an ``ops`` object: :class:`DeviceOps` (libgdd, the product path)
by default. Tests substitute a CPU implementation of the same five methods to exercise the
distributed logic with the gloo backend on hosts without a GPU.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .kmeans import _Ops, check_random_state


class DeviceOps:
    """libgdd primitives on one device (no CPU fallback)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.lib = _lib.device_lib()

    def tensor(self, a, dtype=None):
        return torch.as_tensor(a, dtype=dtype, device=self.device)

    def assign(self, X, C, labels, sq):
        ops = _Ops(self.device, X.shape[0], C.shape[0], X.shape[1])
        ops.assign(X, C, labels=labels, sq=sq)

    def segment_sum_fixed(self, X, labels, k, scale_exp):
        n, dim = X.shape
        sums = torch.zeros((k, dim), dtype=torch.int64, device=self.device)
        counts = torch.zeros(k, dtype=torch.int64, device=self.device)
        _lib.check(self.lib.gdd_segment_sum_fixed(n, dim, X.data_ptr(), None, labels.data_ptr(), k,
                                                  scale_exp, sums.data_ptr(), counts.data_ptr(),
                                                  _lib.stream_ptr(self.device)))
        return sums, counts

    def fixed_to_centers(self, sums, counts, scale_exp, C):
        k, dim = C.shape
        _lib.check(self.lib.gdd_fixed_to_centers(k, dim, sums.data_ptr(), counts.data_ptr(),
                                                 scale_exp, C.data_ptr(),
                                                 _lib.stream_ptr(self.device)))

    def kmeans_plusplus(self, X, k, rs):
        ops = _Ops(self.device, X.shape[0], k, X.shape[1])
        centers, _ = ops.kmeans_plusplus(X, k, rs)
        return centers


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _all_reduce(t: torch.Tensor, op, group):
    """all_reduce that also works for device tensors under gloo (staged through the host)."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    if t.is_cuda and dist.get_backend(group) != "nccl":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def _fixed_col_sum(V: torch.Tensor, n_total: int, group) -> torch.Tensor:
    """Column sums of V (fp64) over every rank, via int64 fixed point (exact and order-free)."""
    amax = torch.tensor([float(V.abs().max().item()) if V.numel() else 0.0], dtype=torch.float64,
                        device=V.device)
    bound = max(float(_all_reduce(amax, dist.ReduceOp.MAX, group).item()), 1e-300) * max(n_total, 1)
    s = int(min(60, 61 - math.ceil(math.log2(bound))))
    fx = torch.round(V * (2.0 ** s)).to(torch.int64).sum(0)
    _all_reduce(fx, dist.ReduceOp.SUM, group)
    return fx.to(torch.float64) * (2.0 ** -s)


def _all_gather_rows(X: torch.Tensor, group) -> torch.Tensor:
    """Concatenate every rank's rows in rank order (shards may differ in length)."""
    rank, world = _world(group)
    if world == 1:
        return X
    n_local = torch.tensor([X.shape[0]], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    host = X.detach().cpu()
    pad = torch.zeros((m, X.shape[1]), dtype=X.dtype)
    pad[:host.shape[0]] = host
    parts = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    full = torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
    return full.to(X.device)


class ShardedKMeans:
    """KMeans(n_clusters, max_iter, tol, random_state).fit over the rows of every rank."""

    def __init__(self, n_clusters=8, *, max_iter=300, tol=1e-4, random_state=None, group=None,
                 ops=None, device="cuda"):
        self.n_clusters = n_clusters
        self.max_iter = max_iter
        self.tol = tol
        self.random_state = random_state
        self.group = group
        self.ops = ops
        self.device = device

    def fit(self, X_local):
        ops = self.ops or DeviceOps(self.device)
        group = self.group
        X = ops.tensor(np.ascontiguousarray(X_local, dtype=np.float32)
                       if not isinstance(X_local, torch.Tensor) else X_local, dtype=torch.float32)
        X = X.contiguous()
        n_local, dim = X.shape
        k = self.n_clusters
        SUM, MAX = dist.ReduceOp.SUM, dist.ReduceOp.MAX
        nt = torch.tensor([n_local], dtype=torch.int64, device=X.device)
        n_total = int(_all_reduce(nt, SUM, group).item())
        if k > n_total:
            raise ValueError(f"n_samples={n_total} should be >= n_clusters={k}.")
        # global column mean and mean(var(X)) from fixed-point integer sums: exact, so identical
        # for every partition of the rows (sklearn centres X by its mean, _kmeans.py:1480-1484)
        mean = _fixed_col_sum(X.to(torch.float64), n_total, group) / n_total
        Xc = (X.to(torch.float64) - mean).to(torch.float32).contiguous()
        var = _fixed_col_sum(Xc.to(torch.float64) ** 2, n_total, group) / n_total
        tol_ = float(var.mean().item()) * self.tol
        # fixed-point scale of the M-step sums: |x| * n_total * 2^s < 2^62
        amax = torch.tensor([float(Xc.abs().max().item()) if n_local else 0.0],
                            dtype=torch.float64, device=X.device)
        bound = max(float(_all_reduce(amax, MAX, group).item()), 1e-30) * n_total
        scale_exp = int(min(60, 61 - math.ceil(math.log2(bound))))
        # replicated k-means++ on the gathered rows (same RandomState on every rank)
        rs = check_random_state(self.random_state)
        X_full = _all_gather_rows(Xc, group)
        C = ops.kmeans_plusplus(X_full, k, rs).contiguous()
        del X_full
        labels = ops.tensor(torch.zeros(n_local, dtype=torch.int32), dtype=torch.int32)
        labels_old = ops.tensor(torch.full((n_local,), -1, dtype=torch.int32), dtype=torch.int32)
        sq = ops.tensor(torch.zeros(n_local, dtype=torch.float32), dtype=torch.float32)
        strict = False
        it = 0
        for it in range(self.max_iter):
            ops.assign(Xc, C, labels, sq)
            sums, counts = ops.segment_sum_fixed(Xc, labels, k, scale_exp)
            changed = int(bool((labels != labels_old).any().item())) if n_local else 0
            pack = torch.cat([sums.reshape(-1), counts,
                              torch.tensor([changed], dtype=torch.int64, device=sums.device)])
            _all_reduce(pack, SUM, group)
            sums = pack[:k * dim].reshape(k, dim).contiguous()
            counts = pack[k * dim:k * dim + k].contiguous()
            any_changed = int(pack[-1].item()) > 0
            if not any_changed:
                strict = True  # labels identical to the previous iteration's on every rank
                break
            C_new = C.clone()
            ops.fixed_to_centers(sums, counts, scale_exp, C_new)
            shift = float(((C_new.to(torch.float64) - C.to(torch.float64)) ** 2).sum().item())
            C = C_new
            labels_old.copy_(labels)
            if shift <= tol_:
                break
        if not strict:
            ops.assign(Xc, C, labels, sq)  # final E-step (_kmeans.py:736-747)
        inertia = torch.tensor([float(sq.to(torch.float64).sum().item())], dtype=torch.float64,
                               device=X.device)
        _all_reduce(inertia, SUM, group)
        self.n_iter_ = it + 1
        self.labels_device_ = labels
        self.cluster_centers_device_ = (C.to(torch.float64) + mean).to(torch.float32)
        self.labels_ = labels.cpu().numpy()
        self.cluster_centers_ = self.cluster_centers_device_.cpu().numpy()
        self.inertia_ = float(inertia.item())
        self.scale_exp_ = scale_exp
        return self


def shard_rows(n: int, rank: int, world: int):
    """Contiguous range partition of n rows: (start, stop) of `rank`."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)
