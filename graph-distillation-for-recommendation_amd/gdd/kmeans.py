"""scikit-learn-compatible KMeans / MiniBatchKMeans whose arithmetic runs in libgdd on MI355X.

Drop-in for the estimators the reference constructs at
``clustgdd_agent_transduct.py:102-105``, ``clustgdd_agent_induct.py:131-134`` and
``distill_recsys.py:174-180``: same constructor arguments, ``fit`` / ``fit_predict`` /
``predict``, and the fitted attributes ``labels_``, ``cluster_centers_``, ``inertia_``,
``n_iter_`` (and ``n_steps_`` for MiniBatchKMeans) as numpy arrays/scalars.

Semantics are scikit-learn 1.7.2's (sklearn/cluster/_kmeans.py) run with one OpenMP thread:
* the RNG is numpy's legacy RandomState from ``check_random_state(random_state)`` — the
  reference's own generator — drawn in sklearn's order on the host;
* every O(n·k·d) and O(n·d) step runs on the device: k-means++ seeding, the MFMA distance GEMM
  with row argmin, inertia, the minibatch/Lloyd centre updates, the full labels pass;
* the host keeps the O(k) control: early stopping on the EWA inertia, the low-count reassignment
  test (numpy on a k-vector), Lloyd's convergence test.
Under those conditions labels, centres, inertia and step counts equal scikit-learn's bit for bit
(tests/test_gpu_kmeans.py against tests/golden/).

``n_init="auto"`` follows sklearn >= 1.4 (one init for k-means++). The README of the reference
pins scikit-learn 1.3.2, whose default was 10 (KMeans) / 3 (MiniBatchKMeans); pass ``n_init``
explicitly to reproduce that.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def check_random_state(seed):
    """sklearn.utils.check_random_state."""
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, (int, np.integer)):
        return np.random.RandomState(seed)
    if isinstance(seed, np.random.RandomState):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a numpy.random.RandomState instance")


def _as_device_f32(X, device):
    if isinstance(X, torch.Tensor):
        return X.detach().to(device=device, dtype=torch.float32).contiguous()
    return torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(device)


class _Ops:
    """Device primitives with their workspaces (one instance per fit)."""

    def __init__(self, device, n_max: int, k: int, dim: int):
        self.lib = _lib.device_lib()
        self.device = torch.device(device)
        self.k, self.dim = k, dim
        self.ws_assign = _lib.workspace(self.lib.gdd_kmeans_assign_ws_bytes(n_max), self.device)
        self.cn2 = torch.empty(k, dtype=torch.float32, device=self.device)
        self.scalar = torch.empty(1, dtype=torch.float32, device=self.device)

    @property
    def stream(self):
        return _lib.stream_ptr(self.device)

    def row_norms(self, C):
        _lib.check(self.lib.gdd_row_norms(C.shape[0], self.dim, C.data_ptr(), self.cn2.data_ptr(),
                                          self.stream))
        return self.cn2

    def assign(self, X, C, rows=None, labels=None, sq=None, n=None, precision="fp32"):
        n = (rows.shape[0] if rows is not None else X.shape[0]) if n is None else n
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        # bf16: the library takes the centres' norms itself (c_norm2 NULL, gdd.h)
        cn2 = self.row_norms(C) if precision == "fp32" else None
        fn = self.lib.gdd_kmeans_assign if precision == "fp32" else self.lib.gdd_kmeans_assign_bf16
        _lib.check(fn(
            n, self.dim, X.data_ptr(), _lib.ptr(rows), C.shape[0], C.data_ptr(), _lib.ptr(cn2),
            labels.data_ptr(), _lib.ptr(sq), self.ws_assign.data_ptr(), self.ws_assign.numel(),
            self.stream))

    def inertia(self, sq, n=None):
        n = sq.shape[0] if n is None else n
        _lib.check(self.lib.gdd_inertia(n, sq.data_ptr(), None, self.scalar.data_ptr(), self.stream))
        return self.scalar

    def kmeans_plusplus(self, Xi, k, rs, n_local_trials=None):
        """_kmeans_plusplus (sklearn/cluster/_kmeans.py:174-272) with unit sample weights."""
        n = Xi.shape[0]
        T = 2 + int(np.log(k)) if n_local_trials is None else int(n_local_trials)
        first = choice_unit_weights(rs, n)
        if k > 1:
            # sklearn draws rs.uniform(size=T) once per round (_kmeans.py:247); the legacy stream gives
            # the same doubles in one call (tests/test_kmeans_host.py), ~2 ms less host time at k = 604
            u = rs.uniform(size=(k - 1) * T)
        else:
            u = np.zeros(1)
        u_d = torch.from_numpy(u.astype(np.float64)).to(self.device)
        centers = torch.empty((k, self.dim), dtype=torch.float32, device=self.device)
        idx = torch.empty(k, dtype=torch.int64, device=self.device)
        ws = _lib.workspace(self.lib.gdd_kmeans_plusplus_ws_bytes_k(n, self.dim, T, k), self.device)
        _lib.check(self.lib.gdd_kmeans_plusplus(n, self.dim, Xi.data_ptr(), None, k, T, int(first),
                                                u_d.data_ptr(), centers.data_ptr(), idx.data_ptr(),
                                                ws.data_ptr(), ws.numel(), self.stream))
        return centers, idx


def choice_unit_weights(rs, n):
    """`rs.choice(n, p=w / w.sum())` for unit float32 weights (sklearn/cluster/_kmeans.py:226, the
    first centre) without numpy's O(n) host arrays (~15 ms at 2.45M points). numpy draws one double u
    (random_sample) and returns searchsorted(cdf, u, 'right'), cdf = cumsum(p) / cumsum(p)[-1] in fp64,
    p_i = c = float32(1 / float32(n)). Below 2^24 points every partial sum (i + 1) * c is exact in fp64
    (c has 24 significant bits, its lowest at or above 2^-45, every partial sum below 2), so
    cdf[i] = fl64((i + 1) / n), which Python's int division rounds the same way: the index is the first
    i with (i + 1) / n > u. Pinned against numpy in tests/test_kmeans_host.py."""
    if n >= 1 << 24:
        w = np.ones(n, dtype=np.float32)
        return int(rs.choice(n, p=w / w.sum()))
    u = rs.random_sample()
    i = min(n - 1, int(u * n))
    while i > 0 and i / n > u:  # cdf[i - 1] = i / n > u: step left
        i -= 1
    while (i + 1) / n <= u:  # cdf[i] <= u: step right
        i += 1
    return i


_SIDE_STREAMS = {}

# Diagnostics: when a dict, KMeans.fit synchronises between its stages and adds their wall times
# (ms) to it — "center_columns", "kmeans_plusplus", "lloyd_loop", "final_estep" — plus "lloyd_calls"
# (host round trips of the device loop). None (the default) adds no synchronisation.
PHASE_TIMING = None


def _phase(name, t0):
    import time
    if PHASE_TIMING is None:
        return t0
    torch.cuda.synchronize()
    now = time.perf_counter()
    PHASE_TIMING[name] = PHASE_TIMING.get(name, 0.0) + (now - t0) * 1e3
    return now


def _side_inertia(sq: torch.Tensor):
    """gdd_inertia(sq) on a per-device side stream, ordered after the caller's stream; returns the
    device scalar and the event that marks it ready."""
    dev = sq.device
    side = _SIDE_STREAMS.get(dev)
    if side is None:
        side = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    out = torch.empty(1, dtype=torch.float32, device=dev)
    lib = _lib.device_lib()
    n = sq.shape[0]
    ws = _lib.workspace(lib.gdd_inertia_ws_bytes(n), dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    _lib.check(lib.gdd_inertia_ws(n, sq.data_ptr(), None, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                  side.cuda_stream))
    sq.record_stream(side)
    out.record_stream(side)
    ws.record_stream(side)
    ev = torch.cuda.Event()
    ev.record(side)
    return out, ev


class _BaseKMeans:
    def __init__(self, n_clusters=8, *, init="k-means++", n_init="auto", max_iter=300, tol=1e-4,
                 verbose=0, random_state=None, device="cuda"):
        if init != "k-means++":
            raise NotImplementedError("only init='k-means++' (the reference's) is implemented")
        self.n_clusters = n_clusters
        self.init = init
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.verbose = verbose
        self.random_state = random_state
        self.device = device

    def _n_init(self, default):
        if self.n_init == "auto":
            return 1  # k-means++ with 'auto' (sklearn >= 1.4, _kmeans.py:879-889)
        return int(self.n_init)

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).labels_

    # fitted attributes as scikit-learn exposes them (host numpy / Python float), copied from the
    # device tensors on first access so the fit itself never waits on a device-to-host copy
    @property
    def cluster_centers_(self):
        if getattr(self, "_centers_np", None) is None:
            self._centers_np = self.cluster_centers_device_.cpu().numpy()
        return self._centers_np

    @cluster_centers_.setter
    def cluster_centers_(self, value):
        self._centers_np = np.asarray(value)

    @property
    def labels_(self):
        if getattr(self, "_labels_np", None) is None:
            self._labels_np = self.labels_device_.cpu().numpy()
        return self._labels_np

    @labels_.setter
    def labels_(self, value):
        self._labels_np = np.asarray(value)

    @property
    def inertia_(self):
        pending = getattr(self, "_inertia_async", None)
        if pending is not None:
            out, ev = pending
            ev.synchronize()
            self._inertia_value = float(out.item())
            self._inertia_async = None
        return self._inertia_value

    @inertia_.setter
    def inertia_(self, value):
        self._inertia_async = None
        self._inertia_value = value

    def predict(self, X, precision: str = "fp32"):
        """Nearest centre of each row. precision='fp32' is sklearn's predict bit for bit;
        'bf16' rounds the dot products' operands to bf16 (MFMA bf16 path) and may
        differ where two centres are within that rounding."""
        Xd = _as_device_f32(X, self.device)
        C = torch.from_numpy(np.ascontiguousarray(self.cluster_centers_, np.float32)).to(Xd.device)
        ops = _Ops(Xd.device, Xd.shape[0], C.shape[0], Xd.shape[1])
        labels = torch.empty(Xd.shape[0], dtype=torch.int32, device=Xd.device)
        ops.assign(Xd, C, labels=labels, precision=precision)
        return labels.cpu().numpy()

    @staticmethod
    def _check_weights(sample_weight):
        if sample_weight is not None and not np.all(np.asarray(sample_weight) == 1):
            raise NotImplementedError("non-unit sample_weight is not used by the reference")


class MiniBatchKMeans(_BaseKMeans):
    """sklearn.cluster.MiniBatchKMeans.fit (sklearn/cluster/_kmeans.py:2046-2200) on the device."""

    def __init__(self, n_clusters=8, *, init="k-means++", max_iter=100, batch_size=1024, verbose=0,
                 compute_labels=True, random_state=None, tol=0.0, max_no_improvement=10,
                 init_size=None, n_init="auto", reassignment_ratio=0.01, device="cuda", group=None):
        super().__init__(n_clusters, init=init, n_init=n_init, max_iter=max_iter, tol=tol,
                         verbose=verbose, random_state=random_state, device=device)
        # group: a torch.distributed group over the GPUs of a node. The steps run replicated on
        # every rank (same RandomState); the final labels pass is partitioned by rows (gdd.sharded)
        self.group = group
        self.batch_size = batch_size
        self.compute_labels = compute_labels
        self.max_no_improvement = max_no_improvement
        self.init_size = init_size
        self.reassignment_ratio = reassignment_ratio

    def _sizes(self, n):
        bs = min(self.batch_size, n)
        isz = self.init_size
        if isz is None:
            isz = 3 * bs
            if isz < self.n_clusters:
                isz = 3 * self.n_clusters
        elif isz < self.n_clusters:
            isz = 3 * self.n_clusters
        return bs, min(isz, n)

    def fit(self, X, y=None, sample_weight=None):
        self._check_weights(sample_weight)
        Xd = _as_device_f32(X, self.device)
        n, dim = Xd.shape
        k = self.n_clusters
        if k > n:
            raise ValueError(f"n_samples={n} should be >= n_clusters={k}.")
        rs = check_random_state(self.random_state)
        if self.tol > 0:
            return self._fit_host_loop(Xd, rs)
        bs, isz = self._sizes(n)
        lib = _lib.device_lib()
        dev = Xd.device
        st = _lib.MTState.from_random_state(rs)
        ws = _lib.workspace(lib.gdd_minibatch_kmeans_fit_ws_bytes(n, dim, k, bs, isz), dev)
        hws = _lib.pinned_workspace(lib.gdd_minibatch_kmeans_fit_host_ws_bytes(n, k, bs, isz))
        centers = torch.empty((k, dim), dtype=torch.float32, device=dev)
        n_steps, ewa = ctypes.c_int64(0), ctypes.c_double(0.0)
        max_ni = -1 if self.max_no_improvement is None else int(self.max_no_improvement)
        # compute_labels: the native fit enqueues the full labels pass (:2191-2197) as soon as the
        # loop stops and leaves the per-sample distances in `sq`; their inertia (the sequential
        # fp32 sum, evaluated in parallel by gdd_inertia_ws) runs on a side stream, read on first
        # access of inertia_
        from .sharded import world_of
        # only an explicit group shards: with group=None a process in some other job's default
        # group (e.g. a DDP run clustering per rank) fits on its own data
        sharded = self.compute_labels and self.group is not None and world_of(self.group)[1] > 1
        native_labels = self.compute_labels and not sharded
        labels = sq = None
        if native_labels:
            labels = torch.empty(n, dtype=torch.int32, device=dev)
            sq = torch.empty(n, dtype=torch.float32, device=dev)
        _lib.check(lib.gdd_minibatch_kmeans_fit(
            n, dim, Xd.data_ptr(), k, bs, int(self.max_iter), max_ni, float(self.reassignment_ratio),
            isz, self._n_init(3), 2 if native_labels else 0, ctypes.addressof(st),
            ctypes.cast(_lib.argsort_callback, ctypes.c_void_p).value, centers.data_ptr(),
            labels.data_ptr() if labels is not None else None, sq.data_ptr() if sq is not None else None,
            ctypes.addressof(n_steps), None if native_labels else ctypes.addressof(ewa),
            ws.data_ptr(), ws.numel(), hws.data_ptr(), hws.numel(), _lib.stream_ptr(dev)))
        st.to_random_state(rs)  # leave the generator where sklearn leaves it
        self.n_steps_ = int(n_steps.value)
        self.n_iter_ = int(np.ceil((self.n_steps_ * bs) / n))
        self.cluster_centers_device_ = centers
        if sharded:  # the final labels pass (:2191-2197) with the rows partitioned over the ranks
            from .sharded import sharded_labels
            labels, sq, _ = sharded_labels(Xd, centers, group=self.group, with_inertia=True,
                                           fold_inertia=False)
        if self.compute_labels:
            self.labels_device_ = labels
            self._inertia_async = _side_inertia(sq)
        else:
            self._inertia_value = ewa.value * n
        return self

    def _fit_host_loop(self, Xd, rs):
        """tol > 0: the centre-shift test needs the host every step (Python loop over the same
        device primitives)."""
        dev = Xd.device
        n, dim = Xd.shape
        k = self.n_clusters
        bs, isz = self._sizes(n)
        n_init = self._n_init(3)
        ops = _Ops(dev, max(n, isz, bs), k, dim)
        validation_indices = rs.randint(0, n, isz)
        best_inertia, init_centers = None, None
        for _ in range(n_init):
            if isz < n:
                init_indices = torch.from_numpy(rs.randint(0, n, isz)).to(dev)
                Xi = Xd.index_select(0, init_indices)
            else:
                Xi = Xd
            centers, _ = ops.kmeans_plusplus(Xi, k, rs)
            if n_init > 1:
                vrows = torch.from_numpy(validation_indices).to(dev)
                lab = torch.empty(isz, dtype=torch.int32, device=dev)
                sq = torch.empty(isz, dtype=torch.float32, device=dev)
                ops.assign(Xd, centers, rows=vrows, labels=lab, sq=sq)
                inertia = float(ops.inertia(sq).item())
            else:
                inertia = 0.0
            if best_inertia is None or inertia < best_inertia:
                init_centers, best_inertia = centers, inertia
        n_steps = (self.max_iter * n) // bs
        C, i, ewa = self._steps_sync(ops, Xd, init_centers, rs, n, bs, n_steps)
        self.n_steps_ = i + 1
        self.n_iter_ = int(np.ceil(((i + 1) * bs) / n))
        self.cluster_centers_device_ = C
        self.cluster_centers_ = C.cpu().numpy()
        if self.compute_labels:
            labels = torch.empty(n, dtype=torch.int32, device=dev)
            sq = torch.empty(n, dtype=torch.float32, device=dev)
            ops.assign(Xd, C, labels=labels, sq=sq)
            self.inertia_ = float(ops.inertia(sq).item())
            self.labels_device_ = labels
            self.labels_ = labels.cpu().numpy()
        else:
            self.inertia_ = ewa * n if ewa is not None else 0.0
        return self

    # -- the step loop -------------------------------------------------------------------------
    def _reassign(self, ops, Xd, rows_d, C_new, counts, rs, bs):
        """Low-count reassignment of _mini_batch_step (:1640-1667): numpy on the k-vector of counts
        (same expressions as sklearn, so argsort tie order and RNG use are identical)."""
        dev = Xd.device
        W = counts.cpu().numpy()
        to_reassign = W < self.reassignment_ratio * W.max()
        if to_reassign.sum() > 0.5 * bs:
            dont = np.argsort(W)[int(0.5 * bs):]
            to_reassign[dont] = False
        n_re = int(to_reassign.sum())
        if n_re:
            new_centers = rs.choice(bs, replace=False, size=n_re)
            dst = torch.from_numpy(np.where(to_reassign)[0]).to(dev)
            src = rows_d.index_select(0, torch.from_numpy(new_centers).to(dev))
            C_new.index_copy_(0, dst, Xd.index_select(0, src))
        W[to_reassign] = np.min(W[~to_reassign])
        counts.copy_(torch.from_numpy(W))
        return bool((W == 0).any())

    def _steps_sync(self, ops, Xd, C0, rs, n, bs, n_steps):
        """tol > 0: one synchronisation per step (the centre-shift test needs the host)."""
        dev, k, dim = Xd.device, self.n_clusters, Xd.shape[1]
        C = C0.contiguous()
        C_new = torch.empty_like(C)
        counts = torch.zeros(k, dtype=torch.float32, device=dev)
        ws_mb = _lib.workspace(ops.lib.gdd_minibatch_update_ws_bytes(bs, k), dev)
        labels_b = torch.empty(bs, dtype=torch.int32, device=dev)
        sq_b = torch.empty(bs, dtype=torch.float32, device=dev)
        rows_d = torch.empty(bs, dtype=torch.int64, device=dev)
        tol_ = float(torch.var(Xd, dim=0, unbiased=False).mean().item()) * self.tol
        any_zero, n_since = True, 0
        ewa = ewa_min = None
        no_improvement = 0
        i = 0
        for i in range(n_steps):
            mb = rs.randint(0, n, bs)
            n_since += bs
            rr = any_zero or n_since >= 10 * k
            if rr:
                n_since = 0
            rows_d.copy_(torch.from_numpy(mb))
            ops.assign(Xd, C, rows=rows_d, labels=labels_b, sq=sq_b)
            bi_d = ops.inertia(sq_b)
            _lib.check(ops.lib.gdd_minibatch_update(bs, dim, Xd.data_ptr(), rows_d.data_ptr(), None,
                                                    labels_b.data_ptr(), k, C.data_ptr(),
                                                    C_new.data_ptr(), counts.data_ptr(),
                                                    ws_mb.data_ptr(), ws_mb.numel(), ops.stream))
            if rr and self.reassignment_ratio > 0:
                any_zero = self._reassign(ops, Xd, rows_d, C_new, counts, rs, bs)
            sq_diff = float(((C_new - C) ** 2).sum().item())
            C, C_new = C_new, C
            bi = float(bi_d.item()) / bs
            if i == 0:
                continue
            if ewa is None:
                ewa = bi
            else:
                a = min(bs * 2.0 / (n + 1), 1)
                ewa = ewa * (1 - a) + bi * a
            if sq_diff <= tol_:
                break
            if ewa_min is None or ewa < ewa_min:
                no_improvement, ewa_min = 0, ewa
            else:
                no_improvement += 1
            if self.max_no_improvement is not None and no_improvement >= self.max_no_improvement:
                break
        return C, i, ewa


class KMeans(_BaseKMeans):
    """sklearn.cluster.KMeans(algorithm='lloyd').fit (sklearn/cluster/_kmeans.py:1427-1530)."""

    def __init__(self, n_clusters=8, *, init="k-means++", n_init="auto", max_iter=300, tol=1e-4,
                 verbose=0, random_state=None, copy_x=True, algorithm="lloyd", device="cuda"):
        super().__init__(n_clusters, init=init, n_init=n_init, max_iter=max_iter, tol=tol,
                         verbose=verbose, random_state=random_state, device=device)
        if algorithm != "lloyd":
            raise NotImplementedError("only algorithm='lloyd' (the default) is implemented")
        self.copy_x = copy_x
        self.algorithm = algorithm

    def fit(self, X, y=None, sample_weight=None):
        self._check_weights(sample_weight)
        X0 = _as_device_f32(X, self.device)
        n, dim = X0.shape
        k = self.n_clusters
        if k > n:
            raise ValueError(f"n_samples={n} should be >= n_clusters={k}.")
        rs = check_random_state(self.random_state)
        dev = X0.device
        import time
        tph = time.perf_counter() if PHASE_TIMING is not None else 0.0
        # sklearn's centring and _tolerance on the device (numpy's sequential column sums): X - mean,
        # mean and var of the INPUT (sklearn/cluster/_kmeans.py:1476-1487, :279-288)
        Xd = torch.empty_like(X0)
        mean_d = torch.empty(dim, dtype=torch.float32, device=dev)
        var_d = torch.empty(dim, dtype=torch.float32, device=dev)
        clib = _lib.device_lib()
        cws = _lib.workspace(clib.gdd_center_columns_ws_bytes(n, dim), dev)
        _lib.check(clib.gdd_center_columns_ws(n, dim, X0.data_ptr(), Xd.data_ptr(), mean_d.data_ptr(),
                                              var_d.data_ptr(), cws.data_ptr(), cws.numel(),
                                              _lib.stream_ptr(dev)))
        X_mean = mean_d.cpu().numpy()
        tol_ = 0 if self.tol == 0 else np.mean(var_d.cpu().numpy()) * self.tol
        del X0
        tph = _phase("center_columns", tph)
        ops = _Ops(dev, n, k, dim)
        lib = ops.lib
        stream = ops.stream
        ws = _lib.workspace(lib.gdd_kmeans_lloyd_ws_bytes(n, dim, k), dev)
        hws = _lib.pinned_workspace(lib.gdd_kmeans_lloyd_host_ws_bytes())
        state = torch.zeros(lib.gdd_lloyd_state_bytes(), dtype=torch.uint8, device=dev)
        labels = torch.empty(n, dtype=torch.int32, device=dev)
        labels_old = torch.empty(n, dtype=torch.int32, device=dev)
        wic = torch.empty(k, dtype=torch.float32, device=dev)
        shift = torch.empty(k, dtype=torch.float32, device=dev)
        sq = torch.empty(n, dtype=torch.float32, device=dev)
        done, reason = ctypes.c_int32(0), ctypes.c_int32(0)

        best = None
        n_inits = self._n_init(10)
        for _ in range(n_inits):
            C0, _ = ops.kmeans_plusplus(Xd, k, rs)
            tph = _phase("kmeans_plusplus", tph)
            Cb = (C0, torch.empty_like(C0))
            labels_old.fill_(-1)
            it0, resume = 0, 0
            while True:  # _kmeans_single_lloyd (:690-735), device-resident
                _lib.check(lib.gdd_kmeans_lloyd_run(
                    n, dim, Xd.data_ptr(), k, Cb[0].data_ptr(), Cb[1].data_ptr(), labels.data_ptr(),
                    labels_old.data_ptr(), wic.data_ptr(), shift.data_ptr(), it0, resume,
                    int(self.max_iter), float(tol_), state.data_ptr(), ctypes.addressof(done),
                    ctypes.addressof(reason), ws.data_ptr(), ws.numel(), hws.data_ptr(), hws.numel(),
                    stream))
                if PHASE_TIMING is not None:
                    PHASE_TIMING["lloyd_calls"] = PHASE_TIMING.get("lloyd_calls", 0) + 1
                if reason.value != 3:
                    break
                it = done.value  # an empty cluster at iteration `it`: relocate, then resume there
                self._relocate(Xd, Cb[it % 2], Cb[(it + 1) % 2], wic, labels, ops)
                it0, resume = it, 1
            n_iter = done.value
            tph = _phase("lloyd_loop", tph)
            strict = reason.value == 1
            C = Cb[n_iter % 2]  # iteration i writes C[(i+1) % 2]
            if not strict:  # the final E-step with the last centres (:736-747)
                ops.assign(Xd, C, labels=labels)
            _lib.check(lib.gdd_point_center_sqdist(n, dim, Xd.data_ptr(), labels.data_ptr(),
                                                   C.data_ptr(), sq.data_ptr(), stream))
            tph = _phase("final_estep", tph)
            if n_inits == 1:
                # one init: nothing to compare, so the fit returns without waiting on the device.
                # The inertia (the sequential fp32 sum over n, gdd_inertia_ws) runs on a side
                # stream and is read on first access of inertia_; labels and centres stay on the
                # device until their host attributes are read. cluster_centers_ = C + X_mean is the
                # same fp32 add numpy makes.
                self._inertia_async = _side_inertia(sq)
                self._inertia_value = None
                self.labels_device_ = labels
                self._labels_np = None
                self.cluster_centers_device_ = C + mean_d
                self._centers_np = None
                self.n_iter_ = n_iter
                return self
            inertia = float(ops.inertia(sq).item())
            lab_h = labels.cpu().numpy()
            if best is None or (inertia < best[1] and not _same_clustering(lab_h, best[0], k)):
                best = (lab_h, inertia, C.clone(), n_iter)
        lab_h, inertia, C, n_iter = best
        self.labels_ = lab_h
        self.inertia_ = inertia
        self.cluster_centers_ = C.cpu().numpy() + X_mean
        self.cluster_centers_device_ = torch.from_numpy(self.cluster_centers_).to(dev)
        self.labels_device_ = torch.from_numpy(lab_h).to(dev)
        self.n_iter_ = n_iter
        return self

    @staticmethod
    def _relocate(Xd, C_old, C_new, wic, labels, ops):
        """_relocate_empty_clusters_dense (_k_means_common.pyx:124-164). Rare. The far-point distances
        are computed on the device in numpy's order (gdd_relocate_distances), so the host's
        np.argpartition over them ranks exactly as sklearn's; only the chosen rows and the k-sized
        sums/weights cross to the host and back."""
        n, dim = Xd.shape
        wic_h = wic.cpu().numpy()
        empty = np.where(np.equal(wic_h, 0))[0].astype(np.int32)
        ne = empty.shape[0]
        if ne == 0:
            return
        dist = torch.empty(n, dtype=torch.float32, device=Xd.device)
        _lib.check(ops.lib.gdd_relocate_distances(n, dim, Xd.data_ptr(), labels.data_ptr(),
                                                  C_old.data_ptr(), dist.data_ptr(), ops.stream))
        distances = dist.cpu().numpy()
        far = np.argpartition(distances, -ne)[:-ne - 1:-1].astype(np.int32)
        if np.max(distances) == 0:
            return
        lab = labels.index_select(0, torch.from_numpy(far.astype(np.int64)).to(Xd.device)).cpu().numpy()
        rows = Xd.index_select(0, torch.from_numpy(far.astype(np.int64)).to(Xd.device)).cpu().numpy()
        cn = C_new.cpu().numpy()
        for idx in range(ne):
            new_id, old_id = empty[idx], lab[idx]
            cn[old_id] -= rows[idx] * np.float32(1.0)
            cn[new_id] = rows[idx] * np.float32(1.0)
            wic_h[new_id] = np.float32(1.0)
            wic_h[old_id] -= np.float32(1.0)
        C_new.copy_(torch.from_numpy(cn))
        wic.copy_(torch.from_numpy(wic_h))


def _same_clustering(l1, l2, k):
    """sklearn _is_same_clustering (_k_means_common.pyx:254-266): the map l1 -> l2 taken at each
    label's first occurrence must hold for every sample (vectorised; same answer as the loop)."""
    l1 = np.asarray(l1, np.int64)
    l2 = np.asarray(l2, np.int64)
    mapping = np.full(k, -1, np.int64)
    first = np.unique(l1, return_index=True)[1]
    mapping[l1[first]] = l2[first]
    return bool(np.array_equal(mapping[l1], l2))
