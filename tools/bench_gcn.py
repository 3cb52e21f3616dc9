#!/usr/bin/env python3
"""The GCN evaluator's full-graph product at the ogbn-arxiv shape: one eval
forward of the reference GCN (models/gcn.py:101-113, nhid 256, C 40) per epoch, 600 epochs x 5 runs
(clustgdd_agent_transduct.py:417-425). Times each SpMM (d = 256 and d = 40) and the whole eval
forward on libgdd (gdd.gcn) against torch's own sparse product on the same GPU (COO and CSR), and the
reference's CPU torch.spmm on a bounded sample. Prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import gcn, synth  # noqa: E402


def dev_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    cfg = synth.CONFIGS["arxiv"]
    A = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
    gn = gdd.normalize_adj(gdd.to_csr(A))
    S = gn.to_scipy().tocoo()
    idx = torch.from_numpy(np.vstack([S.row, S.col]).astype(np.int64))
    vals = torch.from_numpy(S.data.astype(np.float32))
    coo = torch.sparse_coo_tensor(idx, vals, S.shape).coalesce().cuda()
    csr = coo.to_sparse_csr()
    X = torch.from_numpy(synth.features(cfg.n, cfg.d, cfg.seed)).cuda()
    torch.manual_seed(0)
    l1 = gcn.GraphConvolution(cfg.d, 256).cuda()
    l2 = gcn.GraphConvolution(256, cfg.n_classes).cuda()
    res = {"workload": f"GCN eval forward on the ogbn-arxiv-shaped graph (N={cfg.n}, nnz={gn.nnz}, "
                       f"d={cfg.d} -> 256 -> {cfg.n_classes})"}
    with torch.no_grad():
        for d in (256, cfg.n_classes):
            x = torch.randn(cfg.n, d, device="cuda")
            res[f"spmm_d{d}_gdd_ms"] = dev_ms(lambda: gcn.spmm(gn, x))
            res[f"spmm_d{d}_torch_coo_ms"] = dev_ms(lambda: torch.sparse.mm(coo, x))
            res[f"spmm_d{d}_torch_csr_ms"] = dev_ms(lambda: torch.sparse.mm(csr, x))
            bytes_ = 4 * (cfg.n + 1) + 8 * gn.nnz + 8 * cfg.n * d
            res[f"spmm_d{d}_gdd_algorithmic_GBps"] = bytes_ / (res[f"spmm_d{d}_gdd_ms"] * 1e-3) / 1e9

        def fwd(adj):
            h = torch.relu(l1(X, adj))
            return torch.log_softmax(l2(h, adj), dim=1)

        res["eval_forward_gdd_ms"] = dev_ms(lambda: fwd(gn))
        res["eval_forward_torch_coo_ms"] = dev_ms(lambda: fwd(coo))
        a = fwd(gn)
        b = fwd(coo)
        res["eval_forward_max_abs_diff"] = float((a - b).abs().max())
        # the reference's CPU path (torch.spmm on the host), one layer-1 product
        Xc = (X @ l1.weight).cpu()
        coo_c = coo.cpu()
        t = time.perf_counter()
        torch.spmm(coo_c, Xc)
        res["cpu_spmm_d256_ms"] = (time.perf_counter() - t) * 1e3
        res["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
