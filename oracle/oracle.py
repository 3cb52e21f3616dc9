"""CPU restatement of the ClustGDD hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the HIP path. Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg import it; the product package never does (and must fail
loudly rather than fall back to it).

Arithmetic lives in ``gdd_oracle.c`` (compiled to ``oracle/_build/liboracle.so`` by
``oracle/Makefile``); this file holds the ctypes bindings and the host-side control flow of the
reference algorithms, restated from:

* ``ClustGDD/clustgdd_agent_transduct.py:38-129`` — ``pretrained_clustering`` (normalise,
  propagate, k-means on the MLP logits, per-cluster feature means, argmax labels);
* scikit-learn 1.7.2 ``sklearn/cluster/_kmeans.py`` — ``MiniBatchKMeans.fit`` (:2046-2200,
  ``_mini_batch_step`` :1556-1669, ``_mini_batch_convergence`` :1960-2027) and ``KMeans.fit``
  (:1427-1530, ``_kmeans_single_lloyd`` :624-752), run with one OpenMP thread.

The RNG is numpy's legacy ``RandomState`` — the reference's own generator — so every draw
(validation/init subsets, k-means++ ``choice``/``uniform``, per-step ``randint``, reassignment
``choice``) happens in the same order as in scikit-learn.

Parity status: pinned. ``tests/test_oracle_golden.py`` checks this module bit-for-bit against the
golden vectors in ``tests/golden/`` that ``tools/make_golden.py`` produced by running the
reference code and scikit-learn in the build container.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
vp = ctypes.c_void_p
i64 = ctypes.c_int64
ci = ctypes.c_int
cf = ctypes.c_float


def build() -> str:
    """Compile gdd_oracle.c (gcc) into oracle/_build/liboracle.so."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_normalize_csr.restype = i64
        L.oracle_normalize_csr.argtypes = [i64, i32p, i32p, vp, ci, i32p, i32p, f32p]
        L.oracle_spmm.argtypes = [i64, i32p, i32p, f32p, ci, cf, f32p, f32p, vp, cf]
        L.oracle_propagate.argtypes = [i64, i32p, i32p, f32p, ci, f32p, ci, cf, f32p, f32p]
        L.oracle_row_norms.argtypes = [i64, ci, f32p, f32p]
        L.oracle_assign.argtypes = [i64, ci, f32p, vp, ci, f32p, f32p, i32p, vp]
        L.oracle_inertia.restype = cf
        L.oracle_inertia.argtypes = [i64, f32p, vp]
        L.oracle_minibatch_update.argtypes = [i64, ci, f32p, vp, vp, i32p, ci, f32p, f32p, f32p]
        L.oracle_segment_sum_f32.argtypes = [i64, ci, f32p, vp, i32p, ci, f32p, f32p]
        L.oracle_average_centers.argtypes = [ci, ci, f32p, f32p, f32p, vp]
        L.oracle_cluster_mean.argtypes = [i64, ci, f32p, i32p, ci, ci, f32p, i64p]
        L.oracle_sdot_skx.restype = cf
        L.oracle_sdot_skx.argtypes = [f32p, f32p, i64]
        L.oracle_kmeans_plusplus.argtypes = [i64, ci, f32p, vp, ci, ci, i64, f64p, f32p, i64p]
        L.oracle_labels_sqdist.argtypes = [i64, ci, f32p, f32p, i32p, f32p]
        L.oracle_sgemv_t_row.restype = cf
        L.oracle_sgemv_t_row.argtypes = [f32p, f32p, i64, ci, ci]
        L.oracle_skl_sqdist_upcast.argtypes = [ci, f32p, i64, ci, f32p, f32p]
        L.oracle_skl_batch_size.restype = i64
        L.oracle_skl_batch_size.argtypes = [i64, i64, ci]
        L.oracle_skl_dot_mode.argtypes = [ci, i64, ci, ci, i64, ctypes.POINTER(ci)]
        L.oracle_cr_rsqrt.restype = ctypes.c_double
        L.oracle_cr_rsqrt.argtypes = [ctypes.c_double]
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


# ------------------------------------------------------------------------------------------------
# graph side
# ------------------------------------------------------------------------------------------------
def normalize_csr(rowptr, col, val=None, self_loops: int = -1):
    """deep_robust_utils.normalize_adj restated on a canonical CSR (deep_robust_utils.py:180-207)."""
    rowptr, col = _c(rowptr, np.int32), _c(col, np.int32)
    n = rowptr.shape[0] - 1
    nnz = col.shape[0]
    v = None if val is None else _c(val, np.float32)
    ro = np.zeros(n + 1, np.int32)
    co = np.zeros(nnz + n, np.int32)
    vo = np.zeros(nnz + n, np.float32)
    m = lib().oracle_normalize_csr(n, rowptr, col, _ptr(v), self_loops, ro, co, vo)
    return ro, co[:m].copy(), vo[:m].copy()


def spmm(rowptr, col, val, x, scale=1.0, acc=None, acc_scale=0.0):
    rowptr, col, val, x = _c(rowptr, np.int32), _c(col, np.int32), _c(val, np.float32), _c(x, np.float32)
    d = x.shape[1]
    y = np.empty((rowptr.shape[0] - 1, d), np.float32)
    if acc is not None:
        assert acc.dtype == np.float32 and acc.flags.c_contiguous
    lib().oracle_spmm(rowptr.shape[0] - 1, rowptr, col, val, d, scale, x, y, _ptr(acc), acc_scale)
    return y


def propagate(rowptr, col, val, X, T: int, alpha: float):
    """The propagation loop of clustgdd_agent_transduct.py:59-65 -> (target_feat, prop_feat)."""
    rowptr, col, val, X = _c(rowptr, np.int32), _c(col, np.int32), _c(val, np.float32), _c(X, np.float32)
    n, d = X.shape
    target = np.empty_like(X)
    plast = np.empty_like(X)
    lib().oracle_propagate(n, rowptr, col, val, d, X, T, alpha, target, plast)
    return target, plast


# ------------------------------------------------------------------------------------------------
# k-means primitives
# ------------------------------------------------------------------------------------------------
def row_norms(X):
    X = _c(X, np.float32)
    out = np.empty(X.shape[0], np.float32)
    lib().oracle_row_norms(X.shape[0], X.shape[1], X, out)
    return out


def assign(X, C, rows=None, with_sq=True):
    X, C = _c(X, np.float32), _c(C, np.float32)
    cn2 = row_norms(C)
    r = None if rows is None else _c(rows, np.int64)
    n = X.shape[0] if r is None else r.shape[0]
    labels = np.empty(n, np.int32)
    sq = np.empty(n, np.float32) if with_sq else None
    lib().oracle_assign(n, X.shape[1], X, _ptr(r), C.shape[0], C, cn2, labels, _ptr(sq))
    return labels, sq


def labels_inertia(X, C):
    labels, sq = assign(X, C)
    return labels, float(lib().oracle_inertia(sq.shape[0], sq, None))


def inertia(sq, w=None) -> np.float32:
    """sklearn _inertia_dense with one OpenMP thread (_k_means_common.pyx:92-121): the sequential fp32
    sum of sq[i] * w[i] in sample order (w None: ones)."""
    sq = _c(sq, np.float32)
    wc = None if w is None else _c(w, np.float32)
    return np.float32(lib().oracle_inertia(sq.shape[0], sq, _ptr(wc)))


def sdot_skx(x, y):
    x, y = _c(x, np.float32), _c(y, np.float32)
    return float(lib().oracle_sdot_skx(x, y, x.shape[0]))


def minibatch_update(Xb, labels, C_old, weight_sums):
    """_minibatch_update_dense on an already-gathered batch; weight_sums updated in place."""
    Xb, C_old = _c(Xb, np.float32), _c(C_old, np.float32)
    C_new = np.empty_like(C_old)
    lib().oracle_minibatch_update(Xb.shape[0], Xb.shape[1], Xb, None, None, _c(labels, np.int32),
                                  C_old.shape[0], C_old, C_new, weight_sums)
    return C_new


def cluster_mean(feat, labels, k: int, empty_as_zero: bool = False):
    feat = _c(feat, np.float32)
    out = np.empty((k, feat.shape[1]), np.float32)
    counts = np.empty(k, np.int64)
    lib().oracle_cluster_mean(feat.shape[0], feat.shape[1], feat, _c(labels, np.int32), k,
                              int(empty_as_zero), out, counts)
    return out, counts


def _check_random_state(seed):
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, (int, np.integer)):
        return np.random.RandomState(seed)
    if isinstance(seed, np.random.RandomState):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a RandomState")


def skl_sqdist_upcast(Cx, X):
    """sklearn _euclidean_distances(Cx, X, Y_norm_squared=fp32 norms, squared=True), fp32 inputs
    (pairwise.py _euclidean_distances_upcast with OpenBLAS 0.3.29 SkylakeX summation orders)."""
    Cx, X = _c(np.atleast_2d(Cx), np.float32), _c(X, np.float32)
    out = np.empty((Cx.shape[0], X.shape[0]), np.float32)
    lib().oracle_skl_sqdist_upcast(Cx.shape[0], Cx, X.shape[0], X.shape[1], X, out)
    return out


def kmeans_plusplus(X, k: int, rs: np.random.RandomState, n_local_trials=None):
    """_kmeans_plusplus with unit sample weights; draws from `rs` in sklearn's order."""
    X = _c(X, np.float32)
    n, dim = X.shape
    w = np.ones(n, np.float32)
    T = 2 + int(np.log(k)) if n_local_trials is None else n_local_trials
    first = rs.choice(n, p=w / w.sum())
    u = np.concatenate([rs.uniform(size=T) for _ in range(k - 1)]) if k > 1 else np.zeros(1)
    centers = np.empty((k, dim), np.float32)
    idx = np.empty(k, np.int64)
    lib().oracle_kmeans_plusplus(n, dim, X, None, k, T, int(first), _c(u, np.float64), centers, idx)
    return centers, idx


def kmeans_plusplus_draws(X, k: int, T: int, first: int, u, w=None):
    """_kmeans_plusplus with the draws given: the first centre's index and the (k-1)*T uniforms
    (sklearn/cluster/_kmeans.py:226-268; cumsum strictly left to right, as np.cumsum)."""
    X = _c(X, np.float32)
    n, dim = X.shape
    wp = None if w is None else _c(w, np.float32)
    centers = np.empty((k, dim), np.float32)
    idx = np.empty(k, np.int64)
    lib().oracle_kmeans_plusplus(n, dim, X, None if wp is None else wp.ctypes.data, k, T, int(first),
                                 _c(u, np.float64), centers, idx)
    return centers, idx


# ------------------------------------------------------------------------------------------------
# MiniBatchKMeans.fit (sklearn/cluster/_kmeans.py:2046-2200), one OpenMP thread
# ------------------------------------------------------------------------------------------------
def minibatch_kmeans(X, n_clusters: int, random_state=None, batch_size: int = 1024,
                     max_iter: int = 100, n_init="auto", max_no_improvement=10, init_size=None,
                     reassignment_ratio: float = 0.01, tol: float = 0.0, compute_labels=True):
    X = _c(X, np.float32)
    n, dim = X.shape
    k = n_clusters
    rs = _check_random_state(random_state)
    bs = min(batch_size, n)
    isz = init_size
    if isz is None:
        isz = 3 * bs
        if isz < k:
            isz = 3 * k
    elif isz < k:
        isz = 3 * k
    isz = min(isz, n)
    n_init_ = 1 if n_init == "auto" else int(n_init)  # 'auto' + k-means++ -> 1 (sklearn >= 1.4)
    w = np.ones(n, np.float32)

    validation_indices = rs.randint(0, n, isz)
    X_valid = X[validation_indices]
    best_inertia, init_centers = None, None
    for _ in range(n_init_):
        if isz < n:
            init_indices = rs.randint(0, n, isz)
            Xi = X[init_indices]
        else:
            Xi = X
        centers, _ = kmeans_plusplus(Xi, k, rs)
        _, inertia = labels_inertia(X_valid, centers)
        if best_inertia is None or inertia < best_inertia:
            init_centers, best_inertia = centers, inertia

    centers = init_centers
    counts = np.zeros(k, np.float32)
    ewa = ewa_min = None
    no_improvement = 0
    n_since = 0
    n_steps = (max_iter * n) // bs
    tol_ = 0.0
    if tol > 0:
        tol_ = float(np.mean(np.var(X, axis=0)) * tol)
    i = 0
    for i in range(n_steps):
        mb = rs.randint(0, n, bs)
        n_since += bs
        if (counts == 0).any() or n_since >= 10 * k:
            n_since = 0
            random_reassign = True
        else:
            random_reassign = False
        Xb = X[mb]
        labels, batch_inertia = labels_inertia(Xb, centers)
        centers_new = minibatch_update(Xb, labels, centers, counts)
        if random_reassign and reassignment_ratio > 0:
            to_reassign = counts < reassignment_ratio * counts.max()
            if to_reassign.sum() > 0.5 * bs:
                dont = np.argsort(counts)[int(0.5 * bs):]
                to_reassign[dont] = False
            n_re = to_reassign.sum()
            if n_re:
                new_centers = rs.choice(bs, replace=False, size=n_re)
                centers_new[to_reassign] = Xb[new_centers]
            counts[to_reassign] = np.min(counts[~to_reassign])
        sq_diff = np.sum((centers_new - centers) ** 2) if tol_ > 0 else 0
        centers, centers_new = centers_new, centers
        # _mini_batch_convergence (Python floats, :1960-2027)
        bi = batch_inertia / bs
        step = i + 1
        if step == 1:
            continue
        if ewa is None:
            ewa = bi
        else:
            a = min(bs * 2.0 / (n + 1), 1)
            ewa = ewa * (1 - a) + bi * a
        if tol_ > 0.0 and sq_diff <= tol_:
            break
        if ewa_min is None or ewa < ewa_min:
            no_improvement = 0
            ewa_min = ewa
        else:
            no_improvement += 1
        if max_no_improvement is not None and no_improvement >= max_no_improvement:
            break
    n_steps_done = i + 1
    res = {"cluster_centers_": centers, "n_steps_": n_steps_done,
           "n_iter_": int(np.ceil((n_steps_done * bs) / n))}
    if compute_labels:
        labels, inertia = labels_inertia(X, centers)
        res["labels_"], res["inertia_"] = labels, inertia
    return res


# ------------------------------------------------------------------------------------------------
# KMeans.fit, lloyd (sklearn/cluster/_kmeans.py:1427-1530, :624-752), one OpenMP thread
# ------------------------------------------------------------------------------------------------
def _relocate_empty(X, centers_old, centers_new, wic, labels):
    """_relocate_empty_clusters_dense (_k_means_common.pyx:124-164), numpy as in sklearn."""
    empty = np.where(np.equal(wic, 0))[0].astype(np.int32)
    ne = empty.shape[0]
    if ne == 0:
        return
    distances = ((np.asarray(X) - np.asarray(centers_old)[labels]) ** 2).sum(axis=1)
    far = np.argpartition(distances, -ne)[:-ne - 1:-1].astype(np.int32)
    if np.max(distances) == 0:
        return
    for idx in range(ne):
        new_id = empty[idx]
        far_idx = far[idx]
        old_id = labels[far_idx]
        centers_new[old_id] -= X[far_idx] * np.float32(1.0)
        centers_new[new_id] = X[far_idx] * np.float32(1.0)
        wic[new_id] = np.float32(1.0)
        wic[old_id] -= np.float32(1.0)


def _lloyd_iter(X, centers, update_centers=True):
    n, dim = X.shape
    k = centers.shape[0]
    labels, _ = assign(X, centers, with_sq=False)
    if not update_centers:
        return labels, None, None, None
    sums = np.empty((k, dim), np.float32)
    wic = np.empty(k, np.float32)
    lib().oracle_segment_sum_f32(n, dim, X, None, labels, k, sums, wic)
    _relocate_empty(X, centers, sums, wic, labels)
    shift = np.empty(k, np.float32)
    lib().oracle_average_centers(k, dim, sums, wic, centers, _ptr(shift))
    return labels, sums, wic, shift


def _same_clustering(l1, l2, k):
    mapping = np.full(k, -1, np.int32)
    for a, b in zip(l1, l2):
        if mapping[a] == -1:
            mapping[a] = b
        elif mapping[a] != b:
            return False
    return True


def kmeans(X, n_clusters: int, random_state=None, n_init="auto", max_iter: int = 300,
           tol: float = 1e-4):
    X = np.array(X, dtype=np.float32, order="C", copy=True)
    k = n_clusters
    rs = _check_random_state(random_state)
    n_init_ = 1 if n_init == "auto" else int(n_init)
    tol_ = 0 if tol == 0 else np.mean(np.var(X, axis=0)) * tol  # _tolerance on the input (:279-288)
    X_mean = X.mean(axis=0)
    X -= X_mean
    best = None
    for _ in range(n_init_):
        centers, _ = kmeans_plusplus(X, k, rs)
        labels_old = np.full(X.shape[0], -1, np.int32)
        strict = False
        it = 0
        for it in range(max_iter):
            labels, cnew, wic, shift = _lloyd_iter(X, centers)
            centers = cnew
            if np.array_equal(labels, labels_old):
                strict = True
                break
            if (shift ** 2).sum() <= tol_:
                break
            labels_old[:] = labels
        if not strict:
            labels, _, _, _ = _lloyd_iter(X, centers, update_centers=False)
        # _inertia(X, w, centers, labels): the labels of the last E-step, the centers after it
        inertia = float(lib().oracle_inertia(X.shape[0], labels_sqdist(X, centers, labels), None))
        if best is None or (inertia < best[1] and not _same_clustering(labels, best[0], k)):
            best = (labels, inertia, centers, it + 1)
    labels, inertia, centers, n_iter = best
    return {"labels_": labels, "inertia_": inertia, "cluster_centers_": centers + X_mean,
            "n_iter_": n_iter}


def labels_sqdist(X, C, labels):
    """per-sample _euclidean_dense_dense(X[i], C[labels[i]]) (_k_means_common.pyx:26-48)"""
    X, C = _c(X, np.float32), _c(C, np.float32)
    out = np.empty(X.shape[0], np.float32)
    lib().oracle_labels_sqdist(X.shape[0], X.shape[1], X, C, _c(labels, np.int32), out)
    return out


# ------------------------------------------------------------------------------------------------
# ClustGDD.pretrained_clustering hot path (clustgdd_agent_transduct.py:38-129) on given logits
# ------------------------------------------------------------------------------------------------
def cluster_features(target_feat, logits, n_syn: int, dataset: str, seed: int,
                     cluster_minibatch: int = 1000):
    """k-means on the MLP logits then per-cluster means of target_feat (transduct:100-127)."""
    if dataset == "ogbn-arxiv":
        res = minibatch_kmeans(logits, n_syn, random_state=seed, batch_size=cluster_minibatch)
    else:
        res = kmeans(logits, n_syn)
    labels = res["labels_"]
    feat_syn, _ = cluster_mean(target_feat, labels, n_syn)
    labels_syn = np.argmax(res["cluster_centers_"], axis=-1)
    return feat_syn, labels_syn, labels.astype(np.int32), res


# ------------------------------------------------------------------------------------------------
# StandardScaler().fit_transform (sklearn/preprocessing/_data.py, utils/extmath.py
# _incremental_mean_and_var, first call): distill_recsys.py:172
# ------------------------------------------------------------------------------------------------
def standard_scaler(X):
    """(X_scaled fp32, mean fp64, scale fp64) with fp64 column sums accumulated row by row."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n = X.shape[0]
    s = np.zeros(X.shape[1], np.float64)
    for i in range(n):
        s = s + X[i].astype(np.float64)
    mean = s / n
    corr = np.zeros_like(s)
    ssq = np.zeros_like(s)
    for i in range(n):
        t = X[i].astype(np.float64) - mean
        corr = corr + t
        ssq = ssq + t * t
    var = (ssq - (corr * corr) / n) / n
    eps = np.finfo(np.float64).eps
    constant = var <= (n * eps) * var + ((n * mean) * eps) ** 2
    scale = np.where(constant, 1.0, np.sqrt(var))
    c = (X.astype(np.float64) - mean).astype(np.float32)
    out = (c.astype(np.float64) / scale).astype(np.float32)
    return out, mean, scale


# ------------------------------------------------------------------------------------------------
# GraphSAINT preparation (utils_graphsaint.py:34-48): induced sub-graphs adj_full[np.ix_(idx, idx)]
# and a StandardScaler fitted on the train rows, applied to every row
# ------------------------------------------------------------------------------------------------
def induced_subgraph(rowptr, col, val, idx):
    """CSR (rowptr, col, val) of A[idx][:, idx] for strictly increasing idx; val None = binary."""
    rowptr = np.asarray(rowptr, np.int64)
    col = np.asarray(col, np.int64)
    idx = np.asarray(idx, np.int64)
    n = len(rowptr) - 1
    if len(idx) and (np.any(np.diff(idx) <= 0) or idx[0] < 0 or idx[-1] >= n):
        raise ValueError("idx must be strictly increasing node ids")
    pos = np.full(n, -1, np.int64)
    pos[idx] = np.arange(len(idx))
    out_rp = [0]
    out_c, out_v = [], []
    for r in idx:
        cs = col[rowptr[r]:rowptr[r + 1]]
        q = pos[cs]
        keep = q >= 0
        out_c.append(q[keep])
        if val is not None:
            out_v.append(np.asarray(val, np.float32)[rowptr[r]:rowptr[r + 1]][keep])
        out_rp.append(out_rp[-1] + int(keep.sum()))
    c = np.concatenate(out_c).astype(np.int32) if out_c else np.zeros(0, np.int32)
    v = None if val is None else (np.concatenate(out_v) if out_v else np.zeros(0, np.float32))
    return np.asarray(out_rp, np.int32), c, v


def scaler_transform(X, mean, scale):
    """StandardScaler.transform on fp32 X: fp32(fp32(x - mean) / scale) (two fp64 ufuncs, fp32 out)."""
    c = (np.asarray(X, np.float32).astype(np.float64) - mean).astype(np.float32)
    return (c.astype(np.float64) / scale).astype(np.float32)
