"""Multi-GPU distillation of one graph over the ranks of a node (BASELINE north star).

Every rank holds the whole graph, the features and the k-means input: the T-hop propagation's halo
is the whole graph after a few hops, so normalisation and propagation run
replicated, and so do the ~260 latency-bound MiniBatchKMeans steps (same RNG on every rank). The
k-means work that scales with n is partitioned:

* rows: the E-step of every Lloyd iteration and the final labels pass assign rows
  [r·m, (r+1)·m) on rank r (m = ceil(n / R)); ONE all-gather of the int32 labels (and, for the
  inertia, of the per-sample distances) follows;
* clusters: the Lloyd M-step sums and the cluster means are computed for clusters
  [r·q, (r+1)·q) (q = ceil(k / R)) over ALL their members in sample order — the single-GPU order —
  and ONE all-gather of the k-row slices follows.

Each value is therefore computed by the same kernel on the same operands as on one GPU:
labels, centres, inertia, iteration counts and cluster means are bit-identical for every world
size, and equal scikit-learn's (fixtures G3/G9) — the reference's call sites
``clustgdd_agent_transduct.py:102-125``, ``clustgdd_agent_induct.py:131-152`` and
``distill_recsys.py:172-180``. Empty clusters are relocated exactly as ``_relocate_empty_clusters``
(replicated: every rank holds X, the labels and the centres).

Collectives are ``torch.distributed`` all-gathers: RCCL over xGMI for device tensors (one process
per GPU), gloo for the CPU tests (device tensors under gloo are staged through the host). The
primitives come from an ``ops`` object — :class:`DeviceOps` (libgdd, the product path) by default;
tests substitute a CPU stand-in with the same methods to run the distributed logic without a GPU.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .kmeans import KMeans, _Ops, _same_clustering, check_random_state


# ------------------------------------------------------------------------------------------------
# partitions and collectives
# ------------------------------------------------------------------------------------------------
def world_of(group=None):
    """(rank, world size) of `group`, (0, 1) without an initialised process group."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def part(n: int, rank: int, world: int):
    """Equal-chunk partition used by the all-gathers: rank r owns [r*m, min(n, (r+1)*m)), m=ceil(n/R)."""
    m = -(-n // world) if n else 0
    a = min(n, rank * m)
    return a, min(n, a + m), m


def shard_rows(n: int, rank: int, world: int):
    """(start, stop) of `rank` in the row partition."""
    a, b, _ = part(n, rank, world)
    return a, b


def all_gather_parts(t: torch.Tensor, m: int, n: int, group=None, out: torch.Tensor = None) -> torch.Tensor:
    """Concatenate every rank's slice (rank r's first dim holds at most m rows) into the first n rows
    of the whole, in rank order. ``out`` (optional, world * m rows, not aliasing ``t``) receives the
    RCCL gather, so a loop can reuse one buffer instead of allocating a fresh one per call."""
    rank, world = world_of(group)
    if world == 1:
        return t[:n]
    if t.shape[0] == m and t.is_contiguous():  # already a full slot (e.g. a padded hop output)
        pad = t
    else:
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
    if t.is_cuda and dist.get_backend(group) == "nccl":
        if out is None:
            out = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, pad, group=group)
        return out[:n]
    host = pad.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    whole = torch.cat(parts, 0)
    if out is not None:
        out.copy_(whole)
        return out[:n]
    return whole[:n].to(t.device)


def assemble_cols(parts: torch.Tensor, k: int, dim: int, fw: int, world: int) -> torch.Tensor:
    """The k x dim sums from the ranks' column slices (slot r: a row-major k x w_r block, w_r =
    min(fw, dim - r*fw)), as gdd_lloyd_update's k_assemble_cols places them."""
    cols = []
    for r in range(world):
        w = min(fw, dim - r * fw)
        if w > 0:
            cols.append(parts[r * k * fw:r * k * fw + k * w].view(k, w))
    return torch.cat(cols, 1)


def all_gather_slots(buf: torch.Tensor, m: int, group=None) -> None:
    """In place: buf holds world * m rows (elements) and rank r's own slot is buf[r*m:(r+1)*m]; every
    rank ends with every slot. RCCL for device tensors (stream-ordered, no host sync); gloo host-stages."""
    rank, world = world_of(group)
    if world == 1:
        return
    mine = buf[rank * m:(rank + 1) * m]
    if buf.is_cuda and dist.get_backend(group) == "nccl":
        # a copy of the own slot as the input: the in-place form (input a view into the
        # output) is NCCL-legal but untested on hardware here; the copy is m elements
        dist.all_gather_into_tensor(buf, mine.clone(), group=group)
        return
    host = mine.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    buf.copy_(torch.cat(parts, 0).to(buf.device))


def global_rank(group, r: int) -> int:
    """The default-group rank of `group`'s rank r (collectives name their source by global rank)."""
    if group is None or group is dist.group.WORLD:
        return r
    return dist.get_global_rank(group, r)


_SUBGROUPS = {}


def subgroup(ranks, group=None):
    """A process group over `ranks` (ranks of `group`), created once per (group, ranks). Every rank
    of `group` must call this with the same arguments, members or not (dist.new_group's rule)."""
    key = (None if group is None or group is dist.group.WORLD else id(group), tuple(ranks))
    if key not in _SUBGROUPS:
        _SUBGROUPS[key] = dist.new_group([global_rank(group, r) for r in ranks])
    return _SUBGROUPS[key]


def broadcast_from(tensors, owner: int, group=None) -> None:
    """In place: every rank's `tensors` (contiguous, same shapes on every rank) end with the values
    that `group`'s rank `owner` holds. RCCL for device tensors (stream-ordered, no host sync); gloo
    stages through the host."""
    rank, world = world_of(group)
    if world == 1:
        return
    src = global_rank(group, owner)
    nccl = dist.get_backend(group) == "nccl"
    for t in tensors:
        if t.is_cuda and nccl:
            dist.broadcast(t, src=src, group=group)
            continue
        h = t.cpu() if t.is_cuda else t
        dist.broadcast(h, src=src, group=group)
        if h is not t:
            t.copy_(h)


def comm_device(group, device):
    """Where a tensor that crosses `group` lives: the GPU under RCCL, the host under gloo."""
    if world_of(group)[1] > 1 and dist.get_backend(group) != "nccl":
        return torch.device("cpu")
    return torch.device(device)


# ------------------------------------------------------------------------------------------------
# independent work over the ranks: the recsys pair (config 4) and the role graphs (config 3)
# ------------------------------------------------------------------------------------------------
def pair_owners(world: int):
    """Owners of distill_recsys's two kmeans_cluster calls (users, items): ranks 0 and 1 (one rank
    runs both). The fits share nothing (each its own random_state, distill_recsys.py:569-583)."""
    return (0, 1 % world)


def split_pair(jobs, group=None, device="cuda"):
    """Run independent jobs on their owner ranks and broadcast the results: ``jobs`` is a list of
    (fn, spec) where fn() returns arrays/tensors matching spec = [(shape, torch dtype), ...]; job j
    runs on rank ``pair_owners(R)[j]`` only. Returns, on every rank, one tuple of tensors per job
    (on the communication device: the GPU under RCCL, the host under gloo) — bit-identical to
    running every job on one rank, since each job is the single-rank computation itself."""
    rank, world = world_of(group)
    owners = pair_owners(world) if len(jobs) == 2 else tuple(j % world for j in range(len(jobs)))
    cdev = comm_device(group, device)
    outs = []
    for j, (fn, spec) in enumerate(jobs):
        if rank == owners[j]:
            res = fn()
            ts = tuple(torch.as_tensor(np.ascontiguousarray(r) if not isinstance(r, torch.Tensor) else r)
                       .to(device=cdev, dtype=dt).reshape(shape).contiguous()
                       for r, (shape, dt) in zip(res, spec))
        else:
            ts = tuple(torch.empty(shape, dtype=dt, device=cdev) for shape, dt in spec)
        outs.append(ts)
    for j, ts in enumerate(outs):  # the same broadcast order on every rank
        broadcast_from(list(ts), owners[j], group)
    return outs


ROLES = ("train", "val", "test")


def role_owners(world: int):
    """The ranks that propagate each GraphSAINT role graph (config 3, clustgdd_agent_induct.py:72-94:
    three independent loops): train on rank 0 and on every rank past the third, val on rank 1, test on
    rank 2; with two ranks val and test both go to rank 1 (train is ~80% of the hops' bytes at the
    Reddit split: 66% of the nodes and ~44% of the entries of the full graph)."""
    if world == 1:
        return {"train": [0], "val": [0], "test": [0]}
    if world == 2:
        return {"train": [0], "val": [1], "test": [1]}
    return {"train": [0] + list(range(3, world)), "val": [1], "test": [2]}


def propagate_roles(adjs, feats, T: int, alpha: float, group=None, ops=None, phases=None):
    """The three propagations of the inductive agent over the ranks: each role graph is normalised
    and propagated by its owners (:func:`role_owners`); train is row-partitioned over its owners
    (:func:`sharded_propagate` on a sub-group) where :func:`propagation_shards_pay` says so; then one
    broadcast per role's target. Every target is the single-GPU loop's, bit for bit. ``adjs`` and
    ``feats`` map role -> graph / N_role x d features (val/test read only on their owners).
    Returns (normalised train graph — computed on every rank, the agent keeps it — and a dict role ->
    target on every rank). ``phases`` (optional dict): synchronised wall ms per stage of this rank."""
    import time
    ops = ops or DeviceOps(feats["train"].device)
    rank, world = world_of(group)
    owners = role_owners(world)
    sync = getattr(ops, "synchronize", lambda: None)
    t_prev = [time.perf_counter()]

    def mark(name):
        if phases is not None:
            sync()
            now = time.perf_counter()
            phases[name] = phases.get(name, 0.0) + (now - t_prev[0]) * 1e3
            t_prev[0] = now

    if phases is not None:
        sync()
        t_prev[0] = time.perf_counter()
    norm_train = ops.normalize(adjs["train"])          # induct:56-64, every rank
    mark("normalize_train")
    targets = {}
    tr = owners["train"]
    X = feats["train"]
    if len(tr) > 1 and propagation_shards_pay(norm_train.n, norm_train.nnz, X.shape[1], len(tr)):
        sub = subgroup(tr, group)  # every rank creates it; only the members use it
        if rank in tr:
            targets["train"] = sharded_propagate(norm_train, X, T, alpha, group=sub, ops=ops)[0]
    elif rank == tr[0]:
        targets["train"] = ops.propagate(norm_train, X, T, alpha)[0]
    mark("propagate_train")
    for role in ("val", "test"):
        if rank == owners[role][0]:
            gn = ops.normalize(adjs[role])
            mark("normalize_" + role)
            targets[role] = ops.propagate(gn, feats[role], T, alpha)[0]
            mark("propagate_" + role)
    if world > 1:
        cdev = comm_device(group, ops.device)
        for role in ROLES:  # the same order on every rank
            n_r, d_r = int(feats[role].shape[0]), int(feats[role].shape[1])
            t = targets.get(role)
            if t is None:
                t = torch.empty((n_r, d_r), dtype=torch.float32, device=cdev)
            elif t.device != cdev:
                t = t.to(cdev)
            broadcast_from([t], owners[role][0], group)
            targets[role] = t.to(ops.device)
        mark("broadcast_targets")
    return norm_train, targets


# ------------------------------------------------------------------------------------------------
# the device primitives (libgdd)
# ------------------------------------------------------------------------------------------------
class DeviceOps:
    """libgdd primitives on one device (no CPU fallback)."""

    def __init__(self, device):
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.lib = _lib.device_lib()

    @property
    def stream(self):
        return _lib.stream_ptr(self.device)

    def tensor(self, a, dtype=None):
        if isinstance(a, torch.Tensor):
            return a.to(device=self.device, dtype=dtype or a.dtype).contiguous()
        return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=self.device)

    def synchronize(self):
        torch.cuda.synchronize(self.device)

    def normalize(self, adj):
        from .graph import CSRGraph, normalize_adj, to_csr
        g = adj if isinstance(adj, CSRGraph) else to_csr(adj, device=self.device)
        return normalize_adj(g)

    def propagate(self, adj_norm, X, T, alpha):
        from .graph import propagate
        X = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X, np.float32))
        return propagate(adj_norm, X.to(device=self.device, dtype=torch.float32).contiguous(), T, alpha)

    def center(self, X):
        n, dim = X.shape
        Xc = torch.empty_like(X)
        mean = torch.empty(dim, dtype=torch.float32, device=self.device)
        var = torch.empty(dim, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.gdd_center_columns(n, dim, X.data_ptr(), Xc.data_ptr(), mean.data_ptr(),
                                               var.data_ptr(), self.stream))
        return Xc, mean.cpu().numpy(), var.cpu().numpy()

    def kmeans_plusplus(self, X, k, rs):
        centers, _ = _Ops(self.device, X.shape[0], k, X.shape[1]).kmeans_plusplus(X, k, rs)
        return centers

    def assign(self, X, C, r0, r1, with_sq=False):
        n = r1 - r0
        labels = torch.empty(n, dtype=torch.int32, device=self.device)
        sq = torch.empty(n, dtype=torch.float32, device=self.device) if with_sq else None
        if n:
            _Ops(self.device, n, C.shape[0], X.shape[1]).assign(X[r0:r1], C, labels=labels, sq=sq)
        return labels, sq

    def group(self, labels, k):
        from .cluster import group_by_label
        return group_by_label(labels, k)

    def mstep(self, X, grp, k, c0, c1):
        n, dim = X.shape
        perm, offsets = grp
        sums = torch.empty((c1 - c0, dim), dtype=torch.float32, device=self.device)
        wsum = torch.empty(c1 - c0, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.gdd_segment_sum_f32_part(n, dim, X.data_ptr(), None, perm.data_ptr(),
                                                     offsets.data_ptr(), k, c0, c1, _lib.ptr(sums),
                                                     _lib.ptr(wsum), self.stream))
        return sums, wsum

    def relocate(self, X, C_old, sums, wsum, labels):
        KMeans._relocate(X, C_old, sums, wsum, labels, _Ops(self.device, 1, C_old.shape[0], X.shape[1]))

    def average(self, sums, wsum, C_old):
        k, dim = sums.shape
        C_new = sums.clone()
        shift = torch.empty(k, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.gdd_average_centers(k, dim, C_new.data_ptr(), wsum.data_ptr(),
                                                C_old.data_ptr(), shift.data_ptr(), self.stream))
        return C_new, shift

    def point_sqdist(self, X, labels, C, r0, r1):
        out = torch.empty(r1 - r0, dtype=torch.float32, device=self.device)
        if r1 > r0:
            _lib.check(self.lib.gdd_point_center_sqdist(r1 - r0, X.shape[1], X[r0:r1].data_ptr(),
                                                        labels[r0:r1].data_ptr(), C.data_ptr(),
                                                        out.data_ptr(), self.stream))
        return out

    def inertia(self, sq):
        out = torch.empty(1, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.gdd_inertia(sq.shape[0], sq.data_ptr(), None, out.data_ptr(), self.stream))
        return float(out.item())

    # -- the Lloyd loop in phases (gdd_lloyd_estep / _mstep / _update) ------------------------------
    def lloyd_begin(self, n, dim, k, world, m, fw):
        """Per-fit buffers: the workspace (bounds persist across iterations), the state word, labels
        padded to world * m slots, labels_old, wsum, shift, and the column-slice exchange buffer."""
        from types import SimpleNamespace
        dev = self.device
        return SimpleNamespace(
            n=n, dim=dim, k=k,
            ws=_lib.workspace(self.lib.gdd_kmeans_lloyd_ws_bytes(n, dim, k), dev),
            state=torch.zeros(self.lib.gdd_lloyd_state_bytes(), dtype=torch.uint8, device=dev),
            labels=torch.zeros(world * m, dtype=torch.int32, device=dev),
            labels_old=torch.empty(n, dtype=torch.int32, device=dev),
            wsum=torch.empty(k, dtype=torch.float32, device=dev),
            shift=torch.zeros(k, dtype=torch.float32, device=dev),
            parts=torch.zeros(world * k * fw, dtype=torch.float32, device=dev))

    def lloyd_clear(self, ctx, resume):
        ctx.state[:12].zero_()  # stop_at, reason, iter
        if not resume:
            ctx.state[12:16].zero_()  # the labels-changed flag
            ctx.labels_old.fill_(-1)

    def lloyd_estep(self, ctx, X, C, r0, r1, first, it):
        _lib.check(self.lib.gdd_lloyd_estep(ctx.n, r0, r1, ctx.dim, X.data_ptr(), ctx.k, C.data_ptr(),
                                            ctx.shift.data_ptr(), int(first), ctx.labels.data_ptr(),
                                            ctx.state.data_ptr(), it, ctx.ws.data_ptr(), ctx.ws.numel(),
                                            self.stream))

    def lloyd_mstep(self, ctx, X, f0, f1, out, it):
        _lib.check(self.lib.gdd_lloyd_mstep(ctx.n, ctx.dim, X.data_ptr(), ctx.labels.data_ptr(), ctx.k,
                                            f0, f1, out.data_ptr(), ctx.wsum.data_ptr(),
                                            ctx.state.data_ptr(), it, ctx.ws.data_ptr(), ctx.ws.numel(),
                                            self.stream))

    def lloyd_update(self, ctx, parts, fw, C_new, C_old, tol, it):
        _lib.check(self.lib.gdd_lloyd_update(ctx.n, ctx.dim, ctx.k, _lib.ptr(parts), fw, C_new.data_ptr(),
                                             ctx.wsum.data_ptr(), C_old.data_ptr(), ctx.shift.data_ptr(),
                                             ctx.labels.data_ptr(), ctx.labels_old.data_ptr(), float(tol),
                                             ctx.state.data_ptr(), it, self.stream))

    def lloyd_state_begin(self, ctx):
        """Start the state's device-to-host copy (pinned, stream-ordered); lloyd_state_end waits."""
        h = torch.empty(8, dtype=torch.int32, pin_memory=True)
        h.copy_(ctx.state[:32].view(torch.int32), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return h, ev

    def lloyd_state_end(self, handle):
        """(stop_at, reason, iter, done) of the copy lloyd_state_begin started."""
        h, ev = handle
        ev.synchronize()
        return int(h[0]), int(h[1]), int(h[2]), int(h[4])

    def rows_plan(self, rows_graph, d):
        from .graph import SpMMPlan
        return SpMMPlan(rows_graph, d)

    def rows_hop(self, plan, x, y, scale, acc, acc_scale):
        plan.hop(x, y, scale, acc, acc_scale)

    def cluster_mean(self, feat, grp, k, c0, c1, empty_as_zero):
        n, d = feat.shape
        perm, offsets = grp
        out = torch.empty((c1 - c0, d), dtype=torch.float32, device=self.device)
        counts = torch.empty(c1 - c0, dtype=torch.int64, device=self.device)
        _lib.check(self.lib.gdd_cluster_mean_part(n, d, feat.data_ptr(), perm.data_ptr(),
                                                  offsets.data_ptr(), k, c0, c1, int(empty_as_zero),
                                                  _lib.ptr(out), _lib.ptr(counts), self.stream))
        return out, counts


# ------------------------------------------------------------------------------------------------
# row-partitioned propagation
# ------------------------------------------------------------------------------------------------
HOP_GATHER_GBS = 5500.0  # random whole-row gathers from HBM (MI355X_MICROARCH.md), GB/s
ALLGATHER_GBS = 300.0    # RCCL all-gather bus bandwidth per GPU over xGMI (planning figure), GB/s


def propagation_shards_pay(n: int, nnz: int, d: int, world: int) -> bool:
    """Size model for row-partitioned propagation: a hop's gathers (nnz rows of d fp32, whole 128-B
    lines, at the HBM gather rate) shrink by (R-1)/R; each hop then all-gathers the N x d output
    ((R-1)/R of it crosses xGMI). ogbn-products (130M entries, d=100): ~12 ms of gathers vs ~2.9 ms
    of all-gather at R=8 -> shard; ogbn-arxiv (2.6M, d=128): 0.21 vs 0.25 ms -> replicate.
    GDD_SHARD_PROP=1/0 forces the choice."""
    import os
    env = os.environ.get("GDD_SHARD_PROP")
    if env is not None:
        return env == "1" and world > 1
    if world <= 1:
        return False
    line = 128
    row_bytes = -(-4 * d // line) * line
    frac = (world - 1) / world
    hop_ms = nnz * row_bytes / (HOP_GATHER_GBS * 1e9) * 1e3
    gather_ms = n * d * 4 * frac / (ALLGATHER_GBS * 1e9) * 1e3
    return hop_ms * frac > gather_ms


def sharded_propagate(adj_norm, X, T: int, alpha: float, group=None, ops=None):
    """gdd.propagate with the rows partitioned over the ranks (north star: "graph nodes range-
    partitioned across the 8 GPUs"; the loop of clustgdd_agent_transduct.py:59-65). Rank r computes
    rows [r*m, (r+1)*m) of every hop from the whole previous hop and keeps those rows of target; ONE
    all-gather of the hop's N x d output follows each hop, and one of target at the end. Every row's
    arithmetic is the single-GPU hop's (its own entries, the same segment chains, the same two target
    roundings; the first hop's initial target fp32(1-alpha)*X is the same single rounding), so
    target and the last hop are bit-identical for every world size. Returns (target, p_last)."""
    ops = ops or DeviceOps(X.device)
    rank, world = world_of(group)
    n, d = X.shape
    if T < 1:
        raise ValueError("prop_num must be >= 1 (the reference loop leaves target undefined)")
    # gdd_propagate's constants: alpha crosses the C ABI as fp32; 1 - alpha in fp64, then fp32
    a32 = float(np.float32(alpha))
    w32 = np.float32(1.0 - a32)
    r0, r1, m = part(n, rank, world)
    rp = adj_norm.rowptr
    e0, e1 = int(rp[r0]), int(rp[r1])
    target_loc = torch.zeros((m, d), dtype=torch.float32, device=X.device)
    target_loc[: r1 - r0] = X[r0:r1] * w32  # fp32(1 - alpha) * X (agent :59), one rounding
    if T == 1:
        return all_gather_parts(target_loc, m, n, group), X.clone()
    plan = None
    if r1 > r0:
        from .graph import CSRGraph
        rows = CSRGraph((rp[r0:r1 + 1] - rp[r0]).contiguous(), adj_norm.col[e0:e1],
                        adj_norm.values()[e0:e1], r1 - r0)
        plan = ops.rows_plan(rows, d)
    x = X.contiguous()
    # one hop-output slot and two gathered N x d buffers for the whole loop (a fresh slot
    # and a fresh output per hop went through the caching allocator, ~1 GB per rank per hop at
    # ogbn-products); hop h reads gathered buffer (h - 1) % 2 and its gather fills h % 2
    # (one rank: the hop output is the next hop's input, so two slots alternate instead)
    ys = [torch.empty((m, d), dtype=torch.float32, device=X.device) for _ in range(1 if world > 1 else 2)]
    gathered = [torch.empty((world * m, d), dtype=torch.float32, device=X.device) for _ in range(2)] \
        if world > 1 else [None, None]
    for h in range(T - 1):
        y = ys[h % len(ys)]
        if plan is not None:
            ops.rows_hop(plan, x, y[: r1 - r0], a32, target_loc[: r1 - r0], float(w32))
        x = all_gather_parts(y, m, n, group, out=gathered[h % 2])
    return all_gather_parts(target_loc, m, n, group), x


# ------------------------------------------------------------------------------------------------
# partitioned labels pass and cluster means
# ------------------------------------------------------------------------------------------------
def sharded_labels(X, C, group=None, ops=None, with_inertia=True, fold_inertia=True):
    """Nearest centre of every row, rows partitioned over the ranks, labels all-gathered.
    Returns (labels int32 [n], per-sample squared distances [n], inertia) — the inertia is the
    sequential fp32 fold over all n in sample order (sklearn _inertia_dense, one thread);
    ``fold_inertia=False`` leaves that fold to the caller (None)."""
    ops = ops or DeviceOps(X.device)
    rank, world = world_of(group)
    n = X.shape[0]
    r0, r1, m = part(n, rank, world)
    lab, sq = ops.assign(X, C, r0, r1, with_sq=with_inertia)
    labels = all_gather_parts(lab, m, n, group)
    if not with_inertia:
        return labels, None, None
    sq_full = all_gather_parts(sq, m, n, group)
    return labels, sq_full, ops.inertia(sq_full) if fold_inertia else None


def sharded_cluster_mean(feat, labels, k: int, empty_as_zero: bool = False, group=None, ops=None):
    """gdd.cluster_mean with clusters partitioned over the ranks (bit-identical to one GPU):
    every rank groups the (replicated) labels, folds its clusters' members in sample order, and the
    k-row slices are all-gathered -> (feat_syn [k, d], counts [k] int64)."""
    ops = ops or DeviceOps(feat.device)
    rank, world = world_of(group)
    c0, c1, q = part(k, rank, world)
    grp = ops.group(labels, k)
    out, counts = ops.cluster_mean(feat, grp, k, c0, c1, empty_as_zero)
    return all_gather_parts(out, q, k, group), all_gather_parts(counts, q, k, group)


# ------------------------------------------------------------------------------------------------
# Lloyd KMeans over the ranks
# ------------------------------------------------------------------------------------------------
ESTEP_TFLOPS = 50.0  # the unbounded E-step's MFMA rate at large n (measured 46-88 TF/s)


def lloyd_rows_pay(n: int, dim: int, k: int, world: int) -> bool:
    """Size model for ShardedKMeans: splitting the E-step's rows over R ranks saves (R-1)/R of it and
    adds an all-gather of the n int32 labels per iteration (~25 us + 4n(R-1)/R bytes at ~300 GB/s).
    With the bounded E-step (dim <= 48) an iteration's E-step is the bounds test plus the
    listed rows' exact pass, ~0.23 ms at 2.45M rows (r06 trace; r04's model took it for a 40 us bounds
    test), so ogbn-products splits at N >= 2 while the recsys shapes (a ~30 us E-step) replicate; an
    unbounded E-step (2 n k dim flops) of 1 ms and more shards. The M-step is not split: its ordered per-cluster folds are bound by the longest member
    chain, not by the rows' bytes (a column split measured 1.53 -> 1.49 / 1.57 / 1.59 ms at 1/2, 1/4,
    1/8 of the columns, `profiles/r04_fold_cols.txt`). GDD_SHARD_LLOYD=1/0 forces the choice."""
    import os
    env = os.environ.get("GDD_SHARD_LLOYD")
    if env is not None:
        return env == "1" and world > 1
    if world <= 1:
        return False
    bounded = dim <= 48  # the bounded E-step's shapes (gdd_lloyd.hip lloyd_prune_ok)
    # bounded: the bounds test plus the listed rows' exact pass, measured 233 us per iteration at the
    # products shape (2.45M rows, a third of them listed; r06 kernel trace, tools/prof_products_lloyd.py)
    # the part of the E-step that shrinks with the rows (its launch floor does not)
    estep_ms = n * 9.5e-8 if bounded else 2.0 * n * k * dim / (ESTEP_TFLOPS * 1e12) * 1e3
    frac = (world - 1) / world
    gather_ms = 0.025 + 4.0 * n * frac / 300e9 * 1e3
    return estep_ms * frac > gather_ms


class ShardedKMeans:
    """sklearn KMeans(n_clusters, n_init, max_iter, tol, random_state).fit (Lloyd, _kmeans.py:
    1427-1530 / :624-752) over a process group. ``fit`` takes the whole input on every rank; every
    rank ends with the same fitted attributes, bit-identical to one GPU. Where :func:`lloyd_rows_pay`
    says a row split pays, the device loop runs in phases — the E-step on this rank's rows, an
    all-gather of the labels, the replicated M-step (or, with ``split_columns``, this rank's feature
    columns and an all-gather of the column slices) and update; otherwise every rank runs the
    single-GPU device loop (`gdd.KMeans`) on the replicated input, with no collective at all."""

    def __init__(self, n_clusters=8, *, n_init="auto", max_iter=300, tol=1e-4, random_state=None,
                 group=None, ops=None, device="cuda", split_columns=False):
        self.n_clusters = n_clusters
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.random_state = random_state
        self.group = group
        self.ops = ops
        self.device = device
        self.split_columns = split_columns

    def fit(self, X, y=None, sample_weight=None):
        if sample_weight is not None and not np.all(np.asarray(sample_weight) == 1):
            raise NotImplementedError("non-unit sample_weight is not used by the reference")
        group = self.group
        rank, world = world_of(group)
        n_all, dim_all = X.shape
        if self.ops is None and not lloyd_rows_pay(n_all, dim_all, self.n_clusters, world):
            # replicated: the single-GPU device loop on every rank (same RandomState, same bits)
            km = KMeans(n_clusters=self.n_clusters, n_init=self.n_init, max_iter=self.max_iter,
                        tol=self.tol, random_state=self.random_state, device=self.device).fit(X)
            for a in ("labels_", "labels_device_", "inertia_", "cluster_centers_",
                      "cluster_centers_device_", "n_iter_"):
                setattr(self, a, getattr(km, a))
            self.mode_ = "replicated"
            return self
        self.mode_ = "rows"
        ops = self.ops or DeviceOps(self.device)
        X = ops.tensor(X, dtype=torch.float32)
        n, dim = X.shape
        k = self.n_clusters
        if k > n:
            raise ValueError(f"n_samples={n} should be >= n_clusters={k}.")
        r0, r1, m = part(n, rank, world)
        split = self.split_columns and world > 1
        # this rank's feature columns of the M-step (all of them unless split_columns)
        f0, f1, fw = part(dim, rank, world) if split else (0, dim, dim)
        rs = check_random_state(self.random_state)
        # centring and _tolerance on the whole (replicated) input, numpy's orders (:1476-1487, :279-288)
        Xc, X_mean, var = ops.center(X)
        tol_ = 0 if self.tol == 0 else np.mean(var) * self.tol
        n_init = 1 if self.n_init == "auto" else int(self.n_init)
        ctx = ops.lloyd_begin(n, dim, k, world, m, fw if split else 1)
        labels = ctx.labels[:n]
        mine = ctx.parts[rank * k * fw:(rank + 1) * k * fw].view(k, fw) if split else None
        best = None
        for _ in range(n_init):
            C0 = ops.kmeans_plusplus(Xc, k, rs)  # same RandomState on every rank: same centres
            Cb = (C0.contiguous(), torch.empty_like(C0))
            it0, resume, first_e = 0, False, 0
            while True:  # _kmeans_single_lloyd (:690-735), enqueued in chunks of iterations
                ops.lloyd_clear(ctx, resume)
                stop_at, reason, it_r, done = self._run_chunks(ops, ctx, Xc, Cb, it0, resume, first_e,
                                                              (r0, r1, m), (f0, f1, fw, split), mine,
                                                              tol_, group)
                if reason != 3:
                    break
                # an empty cluster at iteration it_r (rare): the sums to C[(it+1) % 2], sklearn's
                # relocation on the host (replicated, identical on every rank), then resume there
                it = it_r
                C_new = Cb[(it + 1) % 2]
                if split:  # otherwise the M-step wrote the sums there itself
                    C_new.copy_(assemble_cols(ctx.parts, k, dim, fw, world))
                ops.relocate(Xc, Cb[it % 2], C_new, ctx.wsum, labels)
                it0, resume, first_e = it, True, it + 1
            n_iter = done
            strict = reason == 1
            C = Cb[n_iter % 2]  # iteration i writes C[(i+1) % 2]
            if not strict:  # the final E-step with the last centres (:736-747)
                lab, _ = ops.assign(Xc, C, r0, r1)
                lab_full = all_gather_parts(lab, m, n, group)
            else:
                lab_full = labels.clone()
            sq = all_gather_parts(ops.point_sqdist(Xc, lab_full, C, r0, r1), m, n, group)
            inertia = ops.inertia(sq)
            lab_h = lab_full.cpu().numpy()
            if best is None or (inertia < best[1] and not _same_clustering(lab_h, best[0], k)):
                best = (lab_h, inertia, C.clone(), n_iter, lab_full.clone())
        lab_h, inertia, C, n_iter, labels_best = best
        self.labels_ = lab_h
        self.labels_device_ = labels_best
        self.inertia_ = inertia
        self.cluster_centers_ = C.cpu().numpy() + X_mean
        self.cluster_centers_device_ = ops.tensor(self.cluster_centers_, dtype=torch.float32)
        self.n_iter_ = n_iter
        return self

    def _run_chunks(self, ops, ctx, Xc, Cb, it0, resume, first_e, rows, cols, mine, tol_, group):
        """Iterations it0.. until the state's stop word is set or max_iter: each iteration is the
        E-step on this rank's rows, ONE all-gather of the labels, the M-step (all columns, into the
        next centres' buffer; or this rank's columns and ONE all-gather of the column slices), the
        replicated update; the host reads the state once per chunk (2, 4, then 8 iterations), one
        chunk behind, as gdd_kmeans_lloyd_run does. The M-step and update kernels are gated by the
        stop word, so iterations enqueued past a stop change nothing."""
        r0, r1, m = rows
        f0, f1, fw, split = cols
        i, ch, pending = it0, 2, None
        while i < self.max_iter:
            for _ in range(min(ch, self.max_iter - i)):
                if not (resume and i == it0):
                    ops.lloyd_estep(ctx, Xc, Cb[i % 2], r0, r1, i == first_e, i)
                    all_gather_slots(ctx.labels, m, group)
                    if split:
                        ops.lloyd_mstep(ctx, Xc, f0, f1, mine, i)
                        all_gather_slots(ctx.parts, ctx.k * fw, group)
                        ops.lloyd_update(ctx, ctx.parts, fw, Cb[(i + 1) % 2], Cb[i % 2], tol_, i)
                    else:
                        ops.lloyd_mstep(ctx, Xc, 0, ctx.dim, Cb[(i + 1) % 2], i)
                        ops.lloyd_update(ctx, None, ctx.dim, Cb[(i + 1) % 2], Cb[i % 2], tol_, i)
                else:  # resume after a relocation: C[(i+1) % 2] already holds the relocated sums
                    ops.lloyd_update(ctx, None, fw, Cb[(i + 1) % 2], Cb[i % 2], tol_, i)
                i += 1
            handle = ops.lloyd_state_begin(ctx)
            if pending is not None:
                st = ops.lloyd_state_end(pending)  # the previous chunk's decision, read while this one runs
                if st[0]:
                    return st
            pending = handle
            ch = min(ch * 2, 8)
        st = ops.lloyd_state_end(pending) if pending is not None else (0, 0, 0, 0)
        if st[0]:
            return st
        return 0, 0, 0, self.max_iter  # ran out of iterations (sklearn's loop end)

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).labels_

