#!/usr/bin/env python3
"""MiniBatchKMeans fits at the bench shape (169,343 x 40 logits, k=454, b=1000) repeated on the same
input, eager launches (GDD_GRAPH=0) against recorded-graph replay (GDD_GRAPH=1, recorded on a key's
second occurrence): per-fit wall time of each repetition, and a k-means++-only timing."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402


def main():
    X = torch.from_numpy(synth.blobs(169343, 40, 454, seed=34)).cuda()
    for mode in ("0", "1", "0", "1"):
        os.environ["GDD_GRAPH"] = mode
        ts = []
        for _ in range(8):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = gdd.MiniBatchKMeans(n_clusters=454, random_state=15, batch_size=1000).fit(X)
            _ = m.labels_device_
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"GDD_GRAPH={mode}: fit ms per repetition " + " ".join(f"{t:.2f}" for t in ts)
              + f"  (n_steps {m.n_steps_})", flush=True)
    Xi = X[:3000].contiguous()
    ops = _Ops("cuda", 3000, 454, 40)
    for mode in ("0", "1", "0", "1"):
        os.environ["GDD_GRAPH"] = mode
        ts = []
        for _ in range(6):
            rs = np.random.RandomState(15)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ops.kmeans_plusplus(Xi, 454, rs)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"GDD_GRAPH={mode}: k-means++ (3000 x 40, k=454) ms " + " ".join(f"{t:.2f}" for t in ts),
              flush=True)


if __name__ == "__main__":
    main()
