#!/usr/bin/env python3
"""Propagation-hop locality experiment: time the planned hop (with the target update) on the
normalised graph in its own node order and after order-preserving relabels (rows of x/p/target
renumbered, each row's entry order kept, so the summation order and the result are unchanged).

usage: micro_reorder.py [arxiv|products] [orders...]   orders: orig degree rcm random
Prints one line per order: us per hop and the bit-exactness of the un-permuted output."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402
from gdd.graph import CSRGraph, SpMMPlan  # noqa: E402


def relabel_host(indptr, col, val, order):
    n = indptr.shape[0] - 1
    rank = np.empty(n, np.int64)
    rank[order] = np.arange(n)
    lens = np.diff(indptr)[order]
    nptr = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=nptr[1:])
    starts = indptr[:-1][order]
    idx = np.repeat(starts - nptr[:-1], lens) + np.arange(nptr[-1])
    return nptr.astype(np.int32), rank[col[idx]].astype(np.int32), val[idx], rank


def hop_time(g, x, reps=10):
    plan = SpMMPlan(g, x.shape[1])
    y = torch.empty_like(x)
    acc = x.clone()
    for _ in range(2):
        plan.hop(x, y, 0.91, acc, 0.09)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        plan.hop(x, y, 0.91, acc, 0.09)
    e1.record()
    torch.cuda.synchronize()
    acc = x.clone()
    plan.hop(x, y, 0.91, acc, 0.09)
    return e0.elapsed_time(e1) / reps * 1e3, y, acc


def main(cfg_name="arxiv", *orders):
    orders = orders or ("orig", "degree", "rcm")
    cfg = synth.CONFIGS[cfg_name]
    t = time.perf_counter()
    A = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
    print(f"{cfg_name}: graph {A.shape[0]} nodes {A.nnz} entries ({time.perf_counter() - t:.1f} s)",
          flush=True)
    x0 = torch.from_numpy(synth.features(cfg.n, cfg.d, cfg.seed)).cuda()
    gn = gdd.normalize_adj(gdd.to_csr(A))
    indptr = gn.rowptr.cpu().numpy().astype(np.int64)
    col = gn.col.cpu().numpy().astype(np.int64)
    val = gn.values().cpu().numpy()
    n, d, nnz = cfg.n, cfg.d, gn.nnz
    bytes_hop = 4 * (n + 1) + 8 * nnz + 16 * n * d
    ref_y = ref_acc = None
    for name in orders:
        t = time.perf_counter()
        if name == "orig":
            order = np.arange(n)
        elif name == "degree":
            order = np.argsort(-np.diff(indptr), kind="stable")
        elif name == "rcm":
            from scipy.sparse.csgraph import reverse_cuthill_mckee
            m = sp.csr_matrix((val, col, indptr), shape=(n, n))
            order = reverse_cuthill_mckee(m, symmetric_mode=True).astype(np.int64)
        elif name == "random":
            order = np.random.default_rng(0).permutation(n)
        else:
            raise SystemExit(f"unknown order {name}")
        p, c, v, rank = relabel_host(indptr, col, val, order)
        g = CSRGraph(torch.from_numpy(p).cuda(), torch.from_numpy(c).cuda(),
                     torch.from_numpy(v).cuda(), n)
        tprep = time.perf_counter() - t
        xo = x0[torch.from_numpy(order).cuda()].contiguous()
        us, y, acc = hop_time(g, xo)
        back = torch.from_numpy(rank).cuda()
        y, acc = y[back], acc[back]
        if ref_y is None:
            ref_y, ref_acc = y, acc
            same = "ref"
        else:
            same = "bit-exact" if torch.equal(y, ref_y) and torch.equal(acc, ref_acc) else \
                f"DIFFERS max {float((y - ref_y).abs().max()):.3g}"
        print(f"{cfg_name} {name:7s}: {us:8.1f} us/hop  {bytes_hop / us / 1e3:7.0f} GB/s algorithmic  "
              f"(host relabel {tprep:.1f} s)  {same}", flush=True)
        del g, xo, y, acc


if __name__ == "__main__":
    main(*sys.argv[1:])
