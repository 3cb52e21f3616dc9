#!/usr/bin/env python3
"""Per-phase wall times of one bench step (device-synchronised between phases)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402


def main(cfg_name="arxiv", reps=3):
    cfg = synth.CONFIGS[cfg_name]
    A = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
    X = torch.from_numpy(synth.features(cfg.n, cfg.d, cfg.seed)).cuda()
    rng = np.random.default_rng(cfg.seed + 3)
    W = torch.from_numpy((rng.standard_normal((cfg.d, cfg.n_classes)) / np.sqrt(cfg.d)).astype(np.float32)).cuda()
    b = torch.from_numpy((rng.standard_normal(cfg.n_classes) * 0.1).astype(np.float32)).cuda()
    g = gdd.to_csr(A)
    torch.cuda.synchronize()
    for r in range(reps):
        t = {}
        s = time.perf_counter()
        gn = gdd.normalize_adj(g); torch.cuda.synchronize(); t["normalize"] = time.perf_counter() - s
        s = time.perf_counter()
        target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha); torch.cuda.synchronize()
        t["propagate"] = time.perf_counter() - s
        s = time.perf_counter()
        logits = torch.addmm(b, target, W); torch.cuda.synchronize(); t["logits"] = time.perf_counter() - s
        s = time.perf_counter()
        km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch).fit(logits)
        torch.cuda.synchronize(); t["minibatch_kmeans"] = time.perf_counter() - s
        s = time.perf_counter()
        fs, _ = gdd.cluster_mean(target, km.labels_device_, cfg.k)
        ls = gdd.argmax_rows(km.cluster_centers_device_); torch.cuda.synchronize()
        t["cluster_mean"] = time.perf_counter() - s
        print(f"rep {r}: " + ", ".join(f"{k}={v*1e3:.2f}ms" for k, v in t.items()),
              f"steps={km.n_steps_}", flush=True)


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["arxiv"]))
