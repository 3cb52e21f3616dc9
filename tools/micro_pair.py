#!/usr/bin/env python3
"""The recsys clustering pair at the ML-1M shape (bench.py recsys_record): users' fit alone, items'
fit alone, the serial pair and the two-stream pair (gdd.pipeline.kmeans_cluster_pair), warm, wall
ms (min of 5; the two-stream pair: min of 10, every call printed on a second line)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import torch  # noqa: E402

from gdd import synth  # noqa: E402
from gdd.pipeline import kmeans_cluster, kmeans_cluster_pair  # noqa: E402

Eu, Ei = synth.svd_like(6040, 64, seed=6040), synth.svd_like(3706, 64, seed=3706)


ALL = {}


def wall(fn, reps=5, name=None):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    if name:
        ALL[name] = [round(x, 2) for x in ts]
    return min(ts)


res = {"users": wall(lambda: kmeans_cluster(Eu, 604, seed=42, device="cuda")),
       "items": wall(lambda: kmeans_cluster(Ei, 371, seed=42, device="cuda")),
       "serial_pair": wall(lambda: kmeans_cluster_pair(Eu, Ei, 604, 371, seed=42, device="cuda", concurrent=False)),
       "two_stream_pair": wall(lambda: kmeans_cluster_pair(Eu, Ei, 604, 371, seed=42, device="cuda"), 10,
                               "two_stream_pair")}
print(json.dumps(res))
print(json.dumps({"every_call_ms": ALL}))
