#!/usr/bin/env python3
"""Condensation timing at the ogbn-arxiv shape: ClustGDD.graph_sparse(sp_type='attaw') over the
40 classes + graph_compress of the 41 graphs (the 40 class graphs and adj_norm), on the device,
beside the CPU restatement (oracle/condense.py, numpy) on a bounded sample.

Prints one JSON line. Inputs: the bench's Chung-Lu arxiv-shaped graph, random logits (C=40) as
``ebd``, random cluster labels (k=454), sp_ratio 0.1 (main_transduct.sh:61-68 for ogbn-arxiv).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import condense as GC  # noqa: E402
from gdd import synth  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


def main(reps=5, cpu=True):
    cfg = synth.CONFIGS["arxiv"]
    A = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
    gn = gdd.normalize_adj(gdd.to_csr(A))
    rng = np.random.default_rng(7)
    ebd_h = (rng.standard_normal((cfg.n, cfg.n_classes)) * 2).astype(np.float32)
    lab_h = rng.integers(0, cfg.k, cfg.n).astype(np.int32)
    ebd = torch.from_numpy(ebd_h).cuda()
    lab = torch.from_numpy(lab_h).cuda()
    ratio = 0.1
    GC.coo_rows(gn)
    t_er, _ = timed(lambda: GC.attaw_ER_estimator(gn, ebd), reps)
    t_sparse, subs = timed(lambda: GC.graph_sparse(gn, ratio, ebd, "attaw"), reps)
    t_comp, _ = timed(lambda: GC.graph_compress(lab, gn, subs), reps)
    t_comp_dense, _ = timed(lambda: GC.graph_compress(lab, gn, subs, dense=True), reps)
    kk = int(lab_h.max()) + 1
    t_one, _ = timed(lambda: GC.compress_dense(lab, gn, kk), reps * 4)
    # algorithmic bytes of one compress over adj_norm: rows, col, val (12 B/edge), two label
    # gathers (8 B/edge), one 8-B atomic per edge, the kk x kk output and labels once
    nnz = gn.nnz
    comp_bytes = 20 * nnz + 8 * nnz + 4 * kk * kk + 4 * cfg.n
    res = {
        "workload": "graph_sparse('attaw', ratio 0.1, C=40) + graph_compress(k=454) at the "
                    "ogbn-arxiv shape (N=169,343, nnz=%d)" % nnz,
        "attaw_er_ms": t_er, "graph_sparse_ms": t_sparse, "graph_compress_41_ms": t_comp,
        "graph_compress_41_dense_ms": t_comp_dense,
        "compress_adj_norm_ms": t_one,
        "compress_adj_norm_GBps": comp_bytes / (t_one * 1e-3) / 1e9,
        "device_total_ms": t_sparse + t_comp,
    }
    if cpu:
        from oracle import condense as O
        rp = gn.rowptr.cpu().numpy()
        col = gn.col.cpu().numpy()
        val = gn.val.cpu().numpy()
        t = time.perf_counter()
        er, rew = O.attaw_er(rp, col, val, ebd_h)
        p = O.softmax_rows(ebd_h)
        rows = O.coo_rows(rp)
        m = int(nnz * ratio)
        sels = [O.topk_edges(O.class_weights(p, er, rows, col, i), m) for i in range(4)]
        t_cpu_sel4 = time.perf_counter() - t
        t = time.perf_counter()
        O.compress(lab_h, rows, col, val)
        t_cpu_comp = time.perf_counter() - t
        est = t_cpu_sel4 / 4 * cfg.n_classes + t_cpu_comp * (cfg.n_classes * ratio + 1)
        res["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "sample": "numpy restatement: ER + 4 of 40 class selections, one "
                                         "full compress; extrapolated to 40 classes and 41 graphs",
                               "est_ms": est * 1e3}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(cpu="--no-cpu" not in sys.argv)
