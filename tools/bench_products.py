#!/usr/bin/env python3
"""Config 5: the transductive hot path at the ogbn-products shape on the device.

Chung-Lu graph, N = 2,449,029, mean degree 50.5 (~124M entries before self-loops), d = 100, C = 47,
T = 18, alpha = 0.91 (arxiv's; the reference gives none), k = 196 with KMeans (Lloyd: the agent uses
MiniBatchKMeans only for ogbn-arxiv), random linear logits. Phase times (device-synchronised) and the
k-means iteration count. Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402


def main(reps=2):
    cfg = synth.CONFIGS["products"]
    t = time.perf_counter()
    A = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
    X = torch.from_numpy(synth.features(cfg.n, cfg.d, cfg.seed)).cuda()
    res = {"workload": f"ogbn-products shape: N={cfg.n}, nnz={A.nnz}, d={cfg.d}, C={cfg.n_classes}, "
                       f"T={cfg.T}, alpha={cfg.alpha}, KMeans(k={cfg.k}) Lloyd",
           "host_generation_s": time.perf_counter() - t}
    rng = np.random.default_rng(cfg.seed + 3)
    W = torch.from_numpy((rng.standard_normal((cfg.d, cfg.n_classes)) / np.sqrt(cfg.d)).astype(np.float32)).cuda()
    g = gdd.to_csr(A)
    del A
    for rep in range(reps + 1):
        ph = {}
        torch.cuda.synchronize()
        s = time.perf_counter()
        gn = gdd.normalize_adj(g)
        torch.cuda.synchronize()
        ph["normalize_ms"] = (time.perf_counter() - s) * 1e3
        s = time.perf_counter()
        target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha)
        torch.cuda.synchronize()
        ph["propagate_ms"] = (time.perf_counter() - s) * 1e3
        logits = target @ W
        np.random.seed(15)
        s = time.perf_counter()
        km = gdd.KMeans(n_clusters=cfg.k).fit(logits)
        torch.cuda.synchronize()
        ph["kmeans_ms"] = (time.perf_counter() - s) * 1e3
        s = time.perf_counter()
        gdd.cluster_mean(target, km.labels_device_, cfg.k)
        torch.cuda.synchronize()
        ph["cluster_mean_ms"] = (time.perf_counter() - s) * 1e3
        ph["kmeans_iters"] = int(km.n_iter_)
        if rep:
            res.setdefault("reps", []).append(ph)
        del gn, target, logits
    res["nnz_norm"] = int(gdd.normalize_adj(g).nnz)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
