#!/usr/bin/env python3
"""Lloyd KMeans at the ogbn-products k-means shape (2,449,029 x 47, k = 196) for a fixed number of
iterations: wall time per iteration (run under rocprofv3 --kernel-trace --stats for the kernels)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402


def main(n=2449029, dim=47, k=196, iters=20):
    X = torch.from_numpy(synth.blobs(n, dim, k, seed=2)).cuda()
    for _ in range(2):
        np.random.seed(15)
        torch.cuda.synchronize()
        t = time.perf_counter()
        km = gdd.KMeans(n_clusters=k, max_iter=iters, tol=0.0).fit(X)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(f"KMeans {n}x{dim} k={k}: {km.n_iter_} iterations in {dt * 1e3:.1f} ms "
          f"({dt * 1e3 / km.n_iter_:.2f} ms/iteration incl. k-means++)", flush=True)


if __name__ == "__main__":
    main()
