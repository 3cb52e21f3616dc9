"""The recommender side of ClustGDD on MI355X (ClustGDD/distill_recsys.py).

Drop-ins, same names and argument meaning:

* :func:`build_condensed_bipartite` (distill_recsys.py:184-201) — interactions (u, i) aggregated to
  super-node pairs (u2cu[u], i2ci[i]), counts as values: ``gdd_bipartite_condense`` (two stable
  radix sorts and a run-length pass on the device). Returns a :class:`BipartiteCSR` (``.to_scipy()``
  gives the reference's ``sp.csr_matrix``, bit-identical);
* :func:`condensed_csr_to_edge_index` (:387-395) — the COO edge list in CSR order;
* :class:`LightGCNCondensed` (:275-384) — same parameters, initialisation, ``edge_weight``,
  ``propagate`` and ``bpr_loss``; the per-layer message passing (two ``index_add_`` scatters over the
  edges, :336-346) runs as two planned SpMMs over the condensed CSR and its transpose, with an
  autograd backward (the transposed products, and the edge gradient as per-edge dot products,
  ``gdd_edge_dots``). Degrees and normalisation stay the reference's torch expressions;
* :func:`save_distilled` (:736-764) — the artefacts in the reference's formats: ``condensed_graph.npz``
  {cu, ci, w, num_cu, num_ci}, ``u2cu.npy``, ``i2ci.npy``, ``condensed_embeddings.pt``;
* the refinement loop's helpers (:641-733): :func:`sample_bpr_triplets_from_condensed` (:217-272) as
  native host code drawing the same numbers from the same ``RandomState`` (``gdd_bpr_sample``), and
  :func:`recall_at_k` (:446-497) with the masking, top-k and hit count on the device
  (``gdd_recall_at_k``; the score GEMM is one library matmul). The driver is
  :mod:`gdd.distill_recsys`.

The message passing sums each row's edges as an fp32 fma chain in CSR order (the canonical hop order);
the reference's ``index_add_`` (sequential on CPU, atomic on GPU) is matched to fp32 tolerance.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F
from torch import nn

from . import _lib


def _i32(a, dev) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=torch.int32).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a), dtype=np.int32)).to(dev)


@dataclass
class BipartiteCSR:
    """A num_cu x num_ci matrix as canonical CSR on the device."""

    rowptr: torch.Tensor  # int32 [num_cu + 1]
    col: torch.Tensor  # int32 [nnz]
    val: torch.Tensor  # fp32 [nnz]
    num_cu: int
    num_ci: int

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    @property
    def shape(self):
        return (self.num_cu, self.num_ci)

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def rows(self) -> torch.Tensor:
        """The row (cu) of every stored entry, int64 [nnz]."""
        rp = self.rowptr.long()
        return torch.repeat_interleave(torch.arange(self.num_cu, device=self.device), rp[1:] - rp[:-1])

    def to_scipy(self) -> sp.csr_matrix:
        return sp.csr_matrix((self.val.cpu().numpy(), self.col.cpu().numpy(), self.rowptr.cpu().numpy()),
                             shape=self.shape)


def build_condensed_bipartite(train_u, train_i, u2cu, i2ci, num_cu: int, num_ci: int,
                              device="cuda") -> BipartiteCSR:
    """distill_recsys.build_condensed_bipartite on the device (values: pair counts, fp32)."""
    lib = _lib.device_lib()
    dev = torch.device(device)
    u, it = _i32(train_u, dev), _i32(train_i, dev)
    a, b = _i32(u2cu, dev), _i32(i2ci, dev)
    E = int(u.numel())
    if E != int(it.numel()):
        raise ValueError("train_u and train_i differ in length")
    num_cu, num_ci = int(num_cu), int(num_ci)
    rowptr = torch.empty(num_cu + 1, dtype=torch.int32, device=dev)
    if E == 0:
        rowptr.zero_()
        return BipartiteCSR(rowptr, torch.empty(0, dtype=torch.int32, device=dev),
                            torch.empty(0, dtype=torch.float32, device=dev), num_cu, num_ci)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    val = torch.empty(E, dtype=torch.float32, device=dev)
    nnz = torch.zeros(1, dtype=torch.int32, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = _lib.workspace(lib.gdd_bipartite_condense_ws_bytes(E, num_cu), dev)
    _lib.check(lib.gdd_bipartite_condense(E, u.data_ptr(), it.data_ptr(), int(a.numel()), int(b.numel()),
                                          a.data_ptr(), b.data_ptr(), num_cu, num_ci, rowptr.data_ptr(),
                                          col.data_ptr(), val.data_ptr(), nnz.data_ptr(), bad.data_ptr(),
                                          ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev)))
    flag, m = int(bad.item()), int(nnz.item())
    if flag & 1:
        raise IndexError("build_condensed_bipartite: a user/item id is outside u2cu/i2ci")
    if flag & 2:
        raise IndexError("build_condensed_bipartite: a cluster id is outside [0, num_cu/num_ci)")
    return BipartiteCSR(rowptr, col[:m], val[:m], num_cu, num_ci)


def condensed_csr_to_edge_index(C, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(edge_index int64 [2, E] over (cu, ci) in CSR order, edge weights fp32 [E])."""
    if isinstance(C, BipartiteCSR):
        dev = torch.device(device) if device is not None else C.device
        ei = torch.stack([C.rows(), C.col.long()]).to(dev)
        return ei, C.val.to(dev)
    C = sp.coo_matrix(C)
    ei = torch.stack([torch.from_numpy(C.row.astype(np.int64)), torch.from_numpy(C.col.astype(np.int64))])
    return ei.to(device or "cpu"), torch.from_numpy(C.data.astype(np.float32)).to(device or "cpu")


class _Bipartite:
    """The condensed graph's structure for message passing: B (rows cu) and Bᵀ (rows ci) as CSR,
    the permutation from Bᵀ entries to B entries (edge values change every step), and one SpMM plan
    per (side, width)."""

    def __init__(self, edge_index: torch.Tensor, num_cu: int, num_ci: int):
        lib = _lib.device_lib()
        dev = edge_index.device
        cu, ci = edge_index[0], edge_index[1]
        E = int(cu.numel())
        if E:
            key = cu * num_ci + ci
            if bool((key[1:] <= key[:-1]).any()):
                raise ValueError("edge_index must list distinct (cu, ci) pairs in CSR order "
                                 "(what condensed_csr_to_edge_index returns)")
            if int(cu.min()) < 0 or int(cu.max()) >= num_cu or int(ci.min()) < 0 or int(ci.max()) >= num_ci:
                raise IndexError("edge_index out of range")
        self.E, self.num_cu, self.num_ci, self.dev = E, num_cu, num_ci, dev
        self.cu = cu.to(torch.int32).contiguous()
        self.ci = ci.to(torch.int32).contiguous()
        counts = torch.bincount(cu, minlength=num_cu) if E else torch.zeros(num_cu, dtype=torch.int64,
                                                                             device=dev)
        self.rowptr = torch.zeros(num_cu + 1, dtype=torch.int32, device=dev)
        self.rowptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        self.rowptr_t = torch.empty(num_ci + 1, dtype=torch.int32, device=dev)
        self.col_t = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
        self.perm = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
        ws = _lib.workspace(lib.gdd_csr_transpose_ws_bytes(num_cu, num_ci, E), dev)
        _lib.check(lib.gdd_csr_transpose(num_cu, num_ci, E, self.rowptr.data_ptr(), _lib.ptr(self.ci),
                                         None, self.rowptr_t.data_ptr(), self.col_t.data_ptr(), None,
                                         self.perm.data_ptr(), ws.data_ptr(), ws.numel(),
                                         _lib.stream_ptr(dev)))
        self.perm_l = self.perm[:E].long()
        self._plans: Dict[Tuple[int, int], torch.Tensor] = {}
        self.bad = torch.zeros(1, dtype=torch.int32, device=dev)  # set by gdd_edge_dots on a bad row id

    def _plan(self, side: int, d: int) -> torch.Tensor:
        ws = self._plans.get((side, d))
        if ws is None:
            lib = _lib.device_lib()
            n, rp = (self.num_cu, self.rowptr) if side == 0 else (self.num_ci, self.rowptr_t)
            ws = _lib.workspace(lib.gdd_propagate_ws_bytes(n, self.E, d), self.dev)
            _lib.check(lib.gdd_spmm_plan(n, self.E, rp.data_ptr(), d, ws.data_ptr(), ws.numel(),
                                         _lib.stream_ptr(self.dev)))
            self._plans[(side, d)] = ws
        return ws

    def product(self, side: int, vals: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        """side 0: B @ x (x: num_ci rows); side 1: Bᵀ @ x (x: num_cu rows). vals: B's edge values."""
        lib = _lib.device_lib()
        x = x.detach().to(torch.float32).contiguous()
        n_out = self.num_cu if side == 0 else self.num_ci
        d = int(x.shape[1])
        y = torch.empty(n_out, d, dtype=torch.float32, device=x.device)
        if self.E == 0:
            return y.zero_()
        ws = self._plan(side, d)
        if side == 0:
            rp, col, v = self.rowptr, self.ci, vals.detach().contiguous()
        else:
            rp, col, v = self.rowptr_t, self.col_t, vals.detach()[self.perm_l].contiguous()
        _lib.check(lib.gdd_spmm_planned(n_out, self.E, rp.data_ptr(), col.data_ptr(), v.data_ptr(), d, 1.0,
                                        x.data_ptr(), y.data_ptr(), None, 0.0, ws.data_ptr(), ws.numel(),
                                        _lib.stream_ptr(x.device)))
        return y

    def edge_dots(self, a_rows: torch.Tensor, a: torch.Tensor, b_rows: torch.Tensor,
                  b: torch.Tensor) -> torch.Tensor:
        lib = _lib.device_lib()
        a, b = a.detach().float().contiguous(), b.detach().float().contiguous()
        out = torch.empty(self.E, dtype=torch.float32, device=a.device)
        _lib.check(lib.gdd_edge_dots(self.E, int(a.shape[1]), a_rows.data_ptr(), a.data_ptr(),
                                     int(a.shape[0]), b_rows.data_ptr(), b.data_ptr(), int(b.shape[0]),
                                     out.data_ptr(), self.bad.data_ptr(), _lib.stream_ptr(a.device)))
        return out

    def check(self) -> None:
        """Raise if an edge gradient met a row id outside its embedding table (one host read)."""
        if int(self.bad.item()):
            raise IndexError("gdd_edge_dots: edge row id out of range")


class _BiMessage(torch.autograd.Function):
    """(u_msg, i_msg) = (B(norm) @ it, B(norm)ᵀ @ u): one layer of distill_recsys.py:336-346."""

    @staticmethod
    def forward(ctx, norm, u, it, g):
        ctx.g = g
        ctx.save_for_backward(norm, u, it)
        return g.product(0, norm, it), g.product(1, norm, u)

    @staticmethod
    def backward(ctx, gu, gi):
        norm, u, it = ctx.saved_tensors
        g = ctx.g
        gu = gu.contiguous() if gu is not None else torch.zeros(g.num_cu, u.shape[1], device=u.device)
        gi = gi.contiguous() if gi is not None else torch.zeros(g.num_ci, it.shape[1], device=u.device)
        d_it = g.product(1, norm, gu) if ctx.needs_input_grad[2] else None
        d_u = g.product(0, norm, gi) if ctx.needs_input_grad[1] else None
        d_norm = None
        if ctx.needs_input_grad[0]:
            d_norm = g.edge_dots(g.cu, gu, g.ci, it) + g.edge_dots(g.ci, gi, g.cu, u)
        return d_norm, d_u, d_it, None


class LightGCNCondensed(nn.Module):
    """distill_recsys.LightGCNCondensed (:275-384) with the message passing on libgdd."""

    def __init__(self, num_cu: int, num_ci: int, dim: int, num_layers: int, edge_index: torch.Tensor,
                 edge_weight_init: torch.Tensor, device):
        super().__init__()
        self.num_cu, self.num_ci = int(num_cu), int(num_ci)
        self.dim, self.num_layers = int(dim), int(num_layers)
        self.device = device
        self.user_emb = nn.Embedding(self.num_cu, self.dim)
        self.item_emb = nn.Embedding(self.num_ci, self.dim)
        nn.init.normal_(self.user_emb.weight, std=0.1)
        nn.init.normal_(self.item_emb.weight, std=0.1)
        self.edge_index = edge_index.to(device)
        y = edge_weight_init.clamp_min(1e-6)
        inv_sp = torch.where(y > 20.0, y, torch.log(torch.expm1(y)))
        self.edge_logit = nn.Parameter(inv_sp)
        self.user_delta = nn.Parameter(torch.zeros(self.num_cu, self.dim, device=device))
        self.item_delta = nn.Parameter(torch.zeros(self.num_ci, self.dim, device=device))
        self._graph: Optional[_Bipartite] = None

    def graph(self) -> _Bipartite:
        if self._graph is None:
            self._graph = _Bipartite(self.edge_index, self.num_cu, self.num_ci)
        return self._graph

    def edge_weight(self) -> torch.Tensor:
        return F.softplus(self.edge_logit) + 1e-8

    def propagate(self) -> Tuple[torch.Tensor, torch.Tensor]:
        u0 = self.user_emb.weight + self.user_delta
        i0 = self.item_emb.weight + self.item_delta
        cu, ci = self.edge_index[0], self.edge_index[1]
        w = self.edge_weight()
        deg_u = torch.zeros(self.num_cu, device=w.device).index_add_(0, cu, w)
        deg_i = torch.zeros(self.num_ci, device=w.device).index_add_(0, ci, w)
        norm = w / (torch.sqrt(deg_u[cu] + 1e-8) * torch.sqrt(deg_i[ci] + 1e-8))
        g = self.graph()
        u, it = u0, i0
        u_layers, i_layers = [u], [it]
        for _ in range(self.num_layers):
            u, it = _BiMessage.apply(norm, u, it, g)
            u_layers.append(u)
            i_layers.append(it)
        return torch.stack(u_layers, dim=0).mean(dim=0), torch.stack(i_layers, dim=0).mean(dim=0)

    def bpr_loss(self, u: torch.Tensor, pos_i: torch.Tensor, neg_i: torch.Tensor,
                 reg_lambda: float = 1e-4) -> torch.Tensor:
        u_z, i_z = self.propagate()
        u_vec, pos_vec, neg_vec = u_z[u], i_z[pos_i], i_z[neg_i]
        pos_score = (u_vec * pos_vec).sum(dim=-1)
        neg_score = (u_vec * neg_vec).sum(dim=-1)
        loss_rank = F.softplus(neg_score - pos_score).mean()
        reg = (self.user_emb(u).norm(2).pow(2) + self.item_emb(pos_i).norm(2).pow(2)
               + self.item_emb(neg_i).norm(2).pow(2)) / max(1, u.shape[0])
        reg = reg + 1e-3 * (self.user_delta.norm(2).pow(2) + self.item_delta.norm(2).pow(2)) / (
            self.num_cu + self.num_ci)
        reg = reg + 1e-6 * self.edge_weight().norm(2).pow(2)
        return loss_rank + reg_lambda * reg


def save_distilled(out_dir: str, model: LightGCNCondensed, u2cu, i2ci, num_cu: int, num_ci: int) -> None:
    """The reference's artefacts (distill_recsys.py:736-764), same file names, keys and dtypes."""
    os.makedirs(out_dir, exist_ok=True)
    with torch.no_grad():
        w = model.edge_weight().detach().cpu().numpy()
        ei = model.edge_index.detach().cpu().numpy()
    np.savez_compressed(os.path.join(out_dir, "condensed_graph.npz"), cu=ei[0], ci=ei[1], w=w,
                        num_cu=np.int64(num_cu), num_ci=np.int64(num_ci))
    np.save(os.path.join(out_dir, "u2cu.npy"), np.asarray(u2cu).astype(np.int64))
    np.save(os.path.join(out_dir, "i2ci.npy"), np.asarray(i2ci).astype(np.int64))
    torch.save({"user_emb": model.user_emb.weight.detach().cpu(),
                "item_emb": model.item_emb.weight.detach().cpu(),
                "user_delta": model.user_delta.detach().cpu(),
                "item_delta": model.item_delta.detach().cpu()},
               os.path.join(out_dir, "condensed_embeddings.pt"))


# ---- refinement loop (distill_recsys.py:641-733) ---------------------------------------------------
class PositiveLists(list):
    """``_csr_row_to_set_list`` (distill_recsys.py:208-214): row r's column indices, as a list of
    arrays like the reference's, also held as one CSR (``indptr`` int64, ``indices`` int32) for the
    native sampler."""

    def __init__(self, indptr, indices):
        self.indptr = np.ascontiguousarray(indptr, dtype=np.int64)
        self.indices = np.ascontiguousarray(indices, dtype=np.int32)
        super().__init__(self.indices[self.indptr[r]:self.indptr[r + 1]].astype(np.int64)
                         for r in range(self.indptr.shape[0] - 1))
        rows_sorted = all(np.all(np.diff(a) >= 0) for a in self)
        self.sorted = None if rows_sorted else np.concatenate(
            [np.sort(a) for a in self] or [np.zeros(0)]).astype(np.int32)


def _csr_row_to_set_list(mat) -> PositiveLists:
    if isinstance(mat, BipartiteCSR):
        mat = mat.to_scipy()
    mat = sp.csr_matrix(mat)
    return PositiveLists(mat.indptr, mat.indices)


def sample_bpr_triplets_from_condensed(pos_items_by_user, num_items: int, batch_size: int,
                                       rng: np.random.RandomState):
    """(u, pos_i, neg_i) int64 arrays, drawn from ``rng`` (advanced in place) in the reference's
    order (:217-272). ``pos_items_by_user``: a :class:`PositiveLists`, a list of arrays, or a CSR."""
    if not isinstance(pos_items_by_user, PositiveLists):
        if sp.issparse(pos_items_by_user) or isinstance(pos_items_by_user, BipartiteCSR):
            pos_items_by_user = _csr_row_to_set_list(pos_items_by_user)
        else:
            rows = [np.asarray(a, dtype=np.int64).ravel() for a in pos_items_by_user]
            ptr = np.zeros(len(rows) + 1, np.int64)
            np.cumsum([r.shape[0] for r in rows], out=ptr[1:])
            pos_items_by_user = PositiveLists(ptr, np.concatenate(rows or [np.zeros(0, np.int64)]))
    pl = pos_items_by_user
    lib = _lib.load()
    st = _lib.MTState.from_random_state(rng)
    b = int(batch_size)
    u, pos, neg = (np.empty(b, np.int64) for _ in range(3))
    _lib.check(lib.gdd_bpr_sample(pl.indptr.ctypes.data, pl.indices.ctypes.data,
                                  None if pl.sorted is None else pl.sorted.ctypes.data,
                                  len(pl), int(num_items), b, ctypes.addressof(st), u.ctypes.data,
                                  pos.ctypes.data, neg.ctypes.data))
    st.to_random_state(rng)
    return u, pos, neg


def _csr_rows(ptr: np.ndarray, idx: np.ndarray, rows: np.ndarray):
    """CSR of the selected rows (int32), in the given row order."""
    lens = (ptr[rows + 1] - ptr[rows]).astype(np.int64)
    out_ptr = np.zeros(rows.shape[0] + 1, np.int64)
    np.cumsum(lens, out=out_ptr[1:])
    gather = np.repeat(ptr[rows] - out_ptr[:-1], lens) + np.arange(out_ptr[-1])
    return out_ptr.astype(np.int32), idx[gather].astype(np.int32)


class RecallEvaluator:
    """``recall_at_k`` (distill_recsys.py:446-497) with its host preparation done once: the evaluated
    users (sorted test users, the first ``max_users``), their training positives and their
    de-duplicated test items as device CSRs, and the denominator. Each call is one score GEMM plus
    ``gdd_recall_at_k`` (mask, top-k, hits) and one 8-byte read."""

    def __init__(self, train_R, test_u, test_i, k: int, device, max_users: int = 5000):
        train_R = sp.csr_matrix(train_R)
        self.device = torch.device(device)
        test_u = np.asarray(test_u, np.int64)
        test_i = np.asarray(test_i, np.int64)
        users = np.unique(test_u)
        if users.size > max_users:
            users = users[:max_users]
        self.users = users
        self.num_items = int(train_R.shape[1])
        self.k = min(int(k), self.num_items)
        pairs = np.unique(np.stack([test_u, test_i], 1), axis=0) if test_u.size else np.zeros((0, 2), np.int64)
        pairs = pairs[np.isin(pairs[:, 0], users)]
        te_ptr = np.searchsorted(pairs[:, 0], np.concatenate([users, [np.iinfo(np.int64).max]]))
        self.total = int(pairs.shape[0])
        tr_ptr, tr_col = _csr_rows(train_R.indptr.astype(np.int64), train_R.indices, users)
        dev = self.device
        self.users_t = torch.from_numpy(users).to(dev)
        self.tr_ptr, self.tr_col = torch.from_numpy(tr_ptr).to(dev), torch.from_numpy(tr_col).to(dev)
        self.te_ptr = torch.from_numpy(te_ptr.astype(np.int32)).to(dev)
        self.te_col = torch.from_numpy(pairs[:, 1].astype(np.int32)).to(dev)

    @torch.no_grad()
    def __call__(self, user_emb: torch.Tensor, item_emb: torch.Tensor) -> float:
        if self.users.size == 0:
            return 0.0
        lib = _lib.device_lib()
        scores = (user_emb[self.users_t] @ item_emb.t()).float().contiguous()  # [B, I] (:475-476)
        if self.k > _RECALL_KERNEL_MAX_K:
            return self._sorted_hits(scores)
        hits = torch.zeros(1, dtype=torch.int64, device=self.device)
        _lib.check(lib.gdd_recall_at_k(int(self.users.size), self.num_items, self.k, scores.data_ptr(),
                                       self.tr_ptr.data_ptr(), _lib.ptr(self.tr_col),
                                       self.te_ptr.data_ptr(), _lib.ptr(self.te_col), hits.data_ptr(),
                                       _lib.stream_ptr(self.device)))
        return float(int(hits.item()) / max(1, self.total))

    def _sorted_hits(self, scores: torch.Tensor, chunk: int = 1024) -> float:
        """k above gdd_recall_at_k's one-pick-per-thread limit: the same mask, then per user the k-th
        largest score t (one top-k); a test item is a hit when its score is above t, or equal to t and
        among the first k - #{score > t} items scoring t in ascending item order (the kernel's tie
        rule). Test items are read through their CSR, chunks of users at a time."""
        B, I = scores.shape
        dev = self.device
        tr_row = torch.repeat_interleave(torch.arange(B, device=dev),
                                         (self.tr_ptr[1:] - self.tr_ptr[:-1]).long())
        scores[tr_row, self.tr_col.long()] = -1e9
        te_row = torch.repeat_interleave(torch.arange(B, device=dev),
                                         (self.te_ptr[1:] - self.te_ptr[:-1]).long())
        te_col = self.te_col.long()
        hits = torch.zeros((), dtype=torch.int64, device=dev)
        for b0 in range(0, B, chunk):
            b1 = min(B, b0 + chunk)
            sc = scores[b0:b1]
            t = torch.topk(sc, self.k, dim=1, largest=True, sorted=False).values.min(dim=1).values
            need = self.k - (sc > t[:, None]).sum(dim=1)  # tie slots left at the threshold
            sel = (te_row >= b0) & (te_row < b1)
            r, c = te_row[sel] - b0, te_col[sel]
            s, tr = sc[r, c], t[r]
            hit = s > tr
            tie = s == tr
            if bool(tie.any()):
                eq_rank = torch.cumsum((sc == t[:, None]).to(torch.int32), dim=1)  # 1-based among ties
                hit |= tie & (eq_rank[r, c] <= need[r])
            hits += hit.sum()
        return float(int(hits.item()) / max(1, self.total))


_RECALL_KERNEL_MAX_K = 256  # gdd_recall_at_k: one pick per thread of a 256-thread workgroup


def recall_at_k(user_emb: torch.Tensor, item_emb: torch.Tensor, train_R, test_u, test_i, k: int,
                device, max_users: int = 5000) -> float:
    """Drop-in for distill_recsys.recall_at_k (:446-497); equal scores rank in ascending item order."""
    return RecallEvaluator(train_R, test_u, test_i, k, device, max_users)(user_emb, item_emb)


@torch.no_grad()
def manual_adam_step(params, state: Dict[int, Dict[str, torch.Tensor]], lr: float, betas=(0.9, 0.999),
                     eps: float = 1e-8, weight_decay: float = 0.0, step: int = 1) -> None:
    """distill_recsys.manual_adam_step (:402-439): Adam with bias correction, the same tensor
    expressions in the same order (so the parameter trajectory is the reference's)."""
    b1, b2 = betas
    for p in params:
        if p.grad is None:
            continue
        g = p.grad if weight_decay == 0.0 else p.grad.add(p, alpha=weight_decay)
        slot = state.setdefault(id(p), {"m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        m, v = slot["m"], slot["v"]
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        p.addcdiv_(m / (1 - b1 ** step), (v / (1 - b2 ** step)).sqrt().add_(eps), value=-lr)
