#!/usr/bin/env python3
"""The recsys KMeans fits (distill_recsys.kmeans_cluster's KMeans on StandardScaled SVD-like
embeddings: ML-1M users 6,040 x 64 with k = 604, items 3,706 x 64 with k = 371) with the Lloyd loop's
forms on and off, same process: default (one-workgroup grouping; the average with the empty check
folded in), GDD_LLOYD_UPDATE_SMALL (the one-workgroup update), GDD_GROUP_SPLIT (the three-launch
grouping). Prints the median Lloyd-loop wall time
(gdd.kmeans.PHASE_TIMING) and whole-fit time over 5 fits per variant, twice."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import torch  # noqa: E402

from gdd import kmeans as gk  # noqa: E402
from gdd import synth  # noqa: E402
from gdd.pipeline import standard_scaler  # noqa: E402

VARIANTS = [(), ("GDD_LLOYD_UPDATE_SMALL",), ("GDD_GROUP_SPLIT",)]


def fit_times(Xs, k, reps=5):
    loop, whole, it = [], [], 0
    for _ in range(reps):
        ph = {}
        gk.PHASE_TIMING = ph
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        km = gk.KMeans(n_clusters=k, random_state=42, n_init="auto", device="cuda").fit(Xs)
        torch.cuda.synchronize()
        whole.append((time.perf_counter() - t0) * 1e3)
        gk.PHASE_TIMING = None
        loop.append(ph.get("lloyd_loop", 0.0))
        it = int(km.n_iter_)
    return statistics.median(loop), statistics.median(whole), it


def main():
    shapes = [("users", 6040, 604), ("items", 3706, 371)]
    data = {name: standard_scaler(synth.svd_like(n, 64, seed=n), device="cuda")[0] for name, n, _ in shapes}
    for name, n, k in shapes:  # warm-up
        gk.KMeans(n_clusters=k, random_state=42, n_init="auto", device="cuda").fit(data[name])
    for rep in range(2):
        for env in VARIANTS:
            for v in ("GDD_LLOYD_UPDATE_SMALL", "GDD_GROUP_SPLIT"):
                os.environ.pop(v, None)
            for v in env:
                os.environ[v] = "1"
            parts = []
            for name, n, k in shapes:
                lp, wh, it = fit_times(data[name], k)
                parts.append(f"{name}: lloyd {lp:.3f} ms ({it} it, {lp * 1e3 / max(it, 1):.1f} us/it), fit {wh:.3f} ms")
            print(f"rep {rep} {'+'.join(env) or 'default':45s} " + "; ".join(parts), flush=True)


if __name__ == "__main__":
    main()
