#!/usr/bin/env python3
"""One bench-shaped MiniBatchKMeans fit (arxiv logits shape), repeated, for kernel traces."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402

cfg = synth.CONFIGS["arxiv"]
A = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
X = torch.from_numpy(synth.features(cfg.n, cfg.d, cfg.seed)).cuda()
rng = np.random.default_rng(cfg.seed + 3)
W = torch.from_numpy((rng.standard_normal((cfg.d, cfg.n_classes)) / np.sqrt(cfg.d)).astype(np.float32)).cuda()
b = torch.from_numpy((rng.standard_normal(cfg.n_classes) * 0.1).astype(np.float32)).cuda()
target, _ = gdd.propagate(gdd.normalize_adj(gdd.to_csr(A)), X, cfg.T, cfg.alpha)
logits = torch.addmm(b, target, W)
for r in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch).fit(logits)
    torch.cuda.synchronize()
    print(f"fit {r}: {1e3 * (time.perf_counter() - t):.2f} ms steps={km.n_steps_}", flush=True)
