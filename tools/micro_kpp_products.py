#!/usr/bin/env python3
"""k-means++ alone at the products KMeans shape (2,449,029 x 47, k = 196: the multi-block split
rounds), event-timed; run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gdd import synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402


def main(n=2449029, dim=47, k=196, reps=3):
    X = torch.from_numpy(synth.blobs(n, dim, k, seed=2)).cuda()
    ops = _Ops("cuda", n, k, dim)
    ops.kmeans_plusplus(X, k, np.random.RandomState(0))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.kmeans_plusplus(X, k, np.random.RandomState(0))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"products k-means++: {ms:.2f} ms per seeding, {ms * 1e3 / (k - 1):.1f} us per round", flush=True)


if __name__ == "__main__":
    main()
