#!/usr/bin/env python3
"""MiniBatchKMeans fit at the bench shape, three times, for a kernel-trace gap analysis
(run under rocprofv3 --kernel-trace; tools/gap_report.py reads the trace)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402


def main():
    cfg = synth.CONFIGS["arxiv"]
    X = torch.from_numpy(synth.blobs(cfg.n, cfg.n_classes, cfg.k, seed=1)).cuda()
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch).fit(X)
        torch.cuda.synchronize()
        print(f"fit {rep}: {(time.perf_counter() - t) * 1e3:.2f} ms wall, steps {km.n_steps_}", flush=True)


if __name__ == "__main__":
    main()
