"""Test helpers for gdd.sharded: a CPU stand-in for the device primitives (the oracle's arithmetic and
numpy's, test-only) and a gloo process-group runner."""
import os
import socket

import numpy as np
import torch

from oracle import oracle as O


def _np(t):
    return t.numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


class OracleOps:
    """The primitives gdd.sharded needs, computed on the host by the oracle (scikit-learn's orders)."""

    device = torch.device("cpu")

    def tensor(self, a, dtype=None):
        if isinstance(a, torch.Tensor):
            return a.to(dtype=dtype or a.dtype).contiguous()
        return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype)

    def center(self, X):
        x = _np(X)
        mean = x.mean(axis=0)
        return torch.from_numpy(x - mean), mean, np.var(x, axis=0)

    def kmeans_plusplus(self, X, k, rs):
        centers, _ = O.kmeans_plusplus(_np(X), k, rs)
        return torch.from_numpy(centers)

    def assign(self, X, C, r0, r1, with_sq=False):
        if r1 <= r0:
            return torch.zeros(0, dtype=torch.int32), torch.zeros(0, dtype=torch.float32)
        lab, sq = O.assign(_np(X)[r0:r1], _np(C))
        return torch.from_numpy(lab), torch.from_numpy(sq) if with_sq else None

    def group(self, labels, k):
        return _np(labels).astype(np.int32)

    def mstep(self, X, grp, k, c0, c1):
        x = np.ascontiguousarray(_np(X), np.float32)
        sums = np.empty((k, x.shape[1]), np.float32)
        wic = np.empty(k, np.float32)
        O.lib().oracle_segment_sum_f32(x.shape[0], x.shape[1], x, None, grp, k, sums, wic)
        return torch.from_numpy(sums[c0:c1].copy()), torch.from_numpy(wic[c0:c1].copy())

    def relocate(self, X, C_old, sums, wsum, labels):
        s, w = sums.numpy(), wsum.numpy()  # views: modified in place
        O._relocate_empty(_np(X), _np(C_old), s, w, _np(labels))

    def average(self, sums, wsum, C_old):
        cn = np.ascontiguousarray(_np(sums), np.float32).copy()
        shift = np.empty(cn.shape[0], np.float32)
        O.lib().oracle_average_centers(cn.shape[0], cn.shape[1], cn, _np(wsum), _np(C_old),
                                       shift.ctypes.data_as(O.vp))
        return torch.from_numpy(cn), torch.from_numpy(shift)

    def point_sqdist(self, X, labels, C, r0, r1):
        if r1 <= r0:
            return torch.zeros(0, dtype=torch.float32)
        return torch.from_numpy(O.labels_sqdist(_np(X)[r0:r1], _np(C), _np(labels)[r0:r1]))

    def inertia(self, sq):
        s = np.ascontiguousarray(_np(sq), np.float32)
        return float(O.lib().oracle_inertia(s.shape[0], s, None))

    # -- the Lloyd loop in phases: the oracle's arithmetic with the device's stop-word gating ------
    def lloyd_begin(self, n, dim, k, world, m, fw):
        from types import SimpleNamespace
        return SimpleNamespace(n=n, dim=dim, k=k, state=np.zeros(16, np.int32),
                               labels=torch.zeros(world * m, dtype=torch.int32),
                               labels_old=torch.empty(n, dtype=torch.int32),
                               wsum=torch.empty(k, dtype=torch.float32),
                               shift=torch.zeros(k, dtype=torch.float32),
                               parts=torch.zeros(world * k * fw, dtype=torch.float32))

    @staticmethod
    def _stopped(ctx, step):
        v = int(ctx.state[0])
        return v != 0 and v - 1 < step

    def lloyd_clear(self, ctx, resume):
        ctx.state[:3] = 0
        if not resume:
            ctx.state[3] = 0
            ctx.labels_old.fill_(-1)

    def lloyd_estep(self, ctx, X, C, r0, r1, first, it):
        if self._stopped(ctx, 2 * it) or r1 <= r0:
            return
        lab, _ = O.assign(_np(X)[r0:r1], _np(C))
        ctx.labels[r0:r1] = torch.from_numpy(lab)

    def lloyd_mstep(self, ctx, X, f0, f1, out, it):
        if self._stopped(ctx, 2 * it):
            return
        x = np.ascontiguousarray(_np(X), np.float32)
        k = ctx.k
        sums = np.empty((k, x.shape[1]), np.float32)
        wic = np.empty(k, np.float32)
        lab = np.ascontiguousarray(ctx.labels[:ctx.n].numpy())
        O.lib().oracle_segment_sum_f32(x.shape[0], x.shape[1], x, None, lab, k, sums, wic)
        if f1 > f0:
            out.view(-1)[:k * (f1 - f0)] = torch.from_numpy(np.ascontiguousarray(sums[:, f0:f1]).ravel())
        ctx.wsum[:] = torch.from_numpy(wic)
        if np.any(wic == 0):  # k_lloyd_check_empty
            ctx.state[1], ctx.state[2], ctx.state[0] = 3, it, 2 * it + 1

    def lloyd_update(self, ctx, parts, fw, C_new, C_old, tol, it):
        if self._stopped(ctx, 2 * it + 1):
            return
        from gdd.sharded import assemble_cols
        k, dim = ctx.k, ctx.dim
        if parts is not None:
            C_new.copy_(assemble_cols(parts, k, dim, fw, -(-dim // fw)))
        cn, shift = self.average(C_new, ctx.wsum, C_old)
        C_new.copy_(cn)
        ctx.shift.copy_(shift)
        lab = ctx.labels[:ctx.n]
        if bool((lab != ctx.labels_old).any()):  # k_lloyd_changed
            ctx.state[3] = 1
            ctx.labels_old.copy_(lab)
        reason = 0
        if ctx.state[3] == 0:
            reason = 1
        elif float((shift.numpy() ** 2).sum()) <= tol:  # numpy's pairwise fp32 sum
            reason = 2
        ctx.state[3] = 0
        ctx.state[4] = it + 1
        if reason:
            ctx.state[1], ctx.state[2], ctx.state[0] = reason, it, 2 * it + 2

    def lloyd_state_begin(self, ctx):
        return ctx.state.copy()

    def lloyd_state_end(self, h):
        return int(h[0]), int(h[1]), int(h[2]), int(h[4])

    def rows_plan(self, rows_graph, d):
        return (_np(rows_graph.rowptr), _np(rows_graph.col), _np(rows_graph.values()))

    def rows_hop(self, plan, x, y, scale, acc, acc_scale):
        rowptr, col, val = plan
        a = acc.numpy()  # a view: the oracle adds acc_scale * y into it in place
        y.copy_(torch.from_numpy(O.spmm(rowptr, col, val, _np(x), scale, a, acc_scale)))

    def cluster_mean(self, feat, grp, k, c0, c1, empty_as_zero):
        out, counts = O.cluster_mean(_np(feat), grp, k, empty_as_zero=empty_as_zero)
        return torch.from_numpy(out[c0:c1].copy()), torch.from_numpy(counts[c0:c1].copy())


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_gloo(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
