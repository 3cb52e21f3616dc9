"""CPU restatement of ClustGDD's graph condensation — TEST INFRASTRUCTURE ONLY.

The parity checker for libgdd's condensation kernels (``csrc/gdd_condense.hip``). Only
``tests/`` and ``bench.py``'s ``cpu_baseline`` leg import it; the product never does.

Restated from the reference (file:line):

* ``utils_clustgdd.attaw_ER_estimator`` (ClustGDD/utils_clustgdd.py:162-182): per-edge cosine
  similarity of the MLP logits, reweighted values ``val * cos``, degrees of the reweighted graph
  (``reweighted @ ones``), and the effective-resistance lower bound ``v/deg[src] + v/deg[dst]``;
* ``utils_clustgdd.ER_estimator`` (:149-159): the same bound on the unweighted-by-cosine graph;
* ``ClustGDD.graph_sparse`` (clustgdd_agent_transduct.py:131-232): per class ``i`` the edge weight
  ``softmax(ebd)[src, i] * softmax(ebd)[dst, i] * ER`` and ``torch.topk(weight, int(nnz*ratio))``;
  sp_type 'vanilla' and 'single' select on ``ER`` alone;
* ``ClustGDD.graph_compress`` (:234-250): ``P^T A P`` with ``P = onehot(labels) / cluster sizes``
  and the diagonal removed.

Orders this restatement fixes (the device follows them, so the two agree bit for bit):

* norms ``sqrtf`` of the sequential fp32 sum of squares, clamped at 1e-8 (torch's eps); cosine
  the sequential fp32 sum of ``(x/|x|) * (y/|y|)`` — torch reduces in a vectorised order, so
  against the reference this is a tolerance (1e-6), not bit parity;
* degrees: the sequential fp32 row sum in CSR order (torch's sparse @ ones: bit-exact);
* softmax: ``e = fp32(exp_f64(x - max))``, sequential fp32 sum, ``e / s`` (torch: tolerance);
* top-k: largest first, NaN largest, ties to the lower edge index (torch.topk leaves ties
  unspecified; on the reference fixtures the selections agree exactly);
* compress: each edge value as int64 fixed point ``llrint(v * 2^s)`` with
  ``s = 62 - ceil(log2(max|v|)) - ceil(log2(nnz + 1))``, exact integer sums per cluster pair,
  then ``sum * 2^-s / (|a| |b|)`` in fp64 rounded to fp32 (the reference's two fp32 products:
  tolerance 1e-5). An empty cluster below the largest label gives a NaN row and column, as the
  reference's ``0/0`` column of P does.
"""
from __future__ import annotations

import math

import numpy as np

EPS = 1e-8


def coo_rows(rowptr: np.ndarray) -> np.ndarray:
    n = len(rowptr) - 1
    return np.repeat(np.arange(n, dtype=np.int32), np.diff(rowptr).astype(np.int64))


def row_unit(ebd: np.ndarray) -> np.ndarray:
    """x / clamp_min(|x|, eps) per row (sequential fp32 sum of squares)."""
    x = np.ascontiguousarray(ebd, dtype=np.float32)
    s = np.zeros(x.shape[0], np.float32)
    for j in range(x.shape[1]):
        s = (s + x[:, j] * x[:, j]).astype(np.float32)
    nrm = np.maximum(np.sqrt(s), np.float32(EPS)).astype(np.float32)
    return (x / nrm[:, None]).astype(np.float32)


def edge_cosine(xu: np.ndarray, rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    a, b = xu[rows], xu[cols]
    s = np.zeros(len(rows), np.float32)
    for j in range(xu.shape[1]):
        s = (s + a[:, j] * b[:, j]).astype(np.float32)
    return s


def row_sums(rowptr: np.ndarray, v: np.ndarray) -> np.ndarray:
    """Sequential fp32 sum of each CSR row (torch sparse COO @ ones on the CPU)."""
    n = len(rowptr) - 1
    deg = np.zeros(n, np.float32)
    rows = coo_rows(rowptr)
    cnt = np.diff(rowptr)
    pos = np.arange(len(v)) - np.repeat(rowptr[:-1], cnt)
    for q in range(int(cnt.max()) if n else 0):
        m = pos == q
        deg[rows[m]] = (deg[rows[m]] + v[m]).astype(np.float32)
    return deg


def attaw_er(rowptr, col, val, ebd):
    """attaw_ER_estimator (utils_clustgdd.py:162-182) -> (ER_lower, reweighted values)."""
    rows = coo_rows(rowptr)
    cos = edge_cosine(row_unit(ebd), rows, col)
    rew = (val.astype(np.float32) * cos).astype(np.float32)
    deg = row_sums(rowptr, rew)
    with np.errstate(divide="ignore", invalid="ignore"):
        er = (rew / deg[rows] + rew / deg[col]).astype(np.float32)
    return er, rew


def vanilla_er(rowptr, col, val):
    """ER_estimator (utils_clustgdd.py:149-159)."""
    rows = coo_rows(rowptr)
    v = val.astype(np.float32)
    deg = row_sums(rowptr, v)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (v / deg[rows] + v / deg[col]).astype(np.float32)


def softmax_rows(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    m = x.max(axis=1)
    e = np.exp((x - m[:, None]).astype(np.float32).astype(np.float64)).astype(np.float32)
    s = np.zeros(x.shape[0], np.float32)
    for j in range(x.shape[1]):
        s = (s + e[:, j]).astype(np.float32)
    return (e / s[:, None]).astype(np.float32)


def topk_edges(w: np.ndarray, m: int) -> np.ndarray:
    """Edge ids of the m largest weights (NaN largest, ties to the lower id), ascending."""
    key = np.where(np.isnan(w), np.inf, w).astype(np.float64)
    nan_first = np.isnan(w)
    order = np.lexsort((np.arange(len(w)), -key, ~nan_first))
    return np.sort(order[:m]).astype(np.int32)


def class_weights(probs, er, rows, cols, i):
    return ((probs[rows, i] * probs[cols, i]).astype(np.float32) * er).astype(np.float32)


def graph_sparse(rowptr, col, val, ratio, ebd=None, sp_type="vanilla"):
    """ClustGDD.graph_sparse -> list of selected edge-id arrays (ascending) and the values the
    selected edges carry."""
    nnz = len(col)
    m = int(nnz * ratio)
    rows = coo_rows(rowptr)
    if sp_type == "no_sp":
        return [np.arange(nnz, dtype=np.int32)], val
    if sp_type == "vanilla":
        return [topk_edges(vanilla_er(rowptr, col, val), m)], val
    er, rew = attaw_er(rowptr, col, val, ebd)
    if sp_type == "single":
        return [topk_edges(er, m)], rew
    if sp_type == "attaw":
        p = softmax_rows(ebd)
        return [topk_edges(class_weights(p, er, rows, col, i), m) for i in range(p.shape[1])], rew
    raise ValueError(sp_type)


def fixed_shift(vals: np.ndarray) -> int:
    mx = float(np.max(np.abs(vals))) if len(vals) else 0.0
    if not np.isfinite(mx):
        raise ValueError("non-finite edge values")
    e1 = math.frexp(mx)[1] if mx > 0 else 0  # mx < 2^e1
    e2 = math.frexp(float(len(vals) + 1))[1]
    return 62 - e1 - e2


def compress(labels, rows, cols, vals, k=None):
    """graph_compress on one edge list: k x k fp32 with the diagonal zeroed (NaN for empty
    clusters)."""
    labels = np.asarray(labels, dtype=np.int64)
    kk = int(labels.max()) + 1 if k is None else int(k)
    size = np.bincount(labels, minlength=kk).astype(np.float64)
    s = fixed_shift(vals)
    q = np.rint(np.ldexp(vals.astype(np.float64), s)).astype(np.int64)
    acc = np.zeros(kk * kk, np.int64)
    np.add.at(acc, labels[rows] * kk + labels[cols], q)
    with np.errstate(divide="ignore", invalid="ignore"):
        out = (np.ldexp(acc.astype(np.float64), -s).reshape(kk, kk) / np.outer(size, size))
    out = out.astype(np.float32)
    empty = size == 0
    out[empty, :] = np.nan
    out[:, empty] = np.nan
    d = np.arange(kk)
    out[d, d] = out[d, d] - out[d, d]
    return out
