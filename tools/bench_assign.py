#!/usr/bin/env python3
"""The full k-means assignment pass ("MFMA-bound at fp32 for k >~ 40"; configs 2, 3, 5
carry fp32 and bf16 distance variants) at the arxiv, reddit and products shapes: fp32 (bit-exact with
sklearn) vs bf16 MFMA, device time per pass, TFLOP/s on 2*N*k*C, and the fraction of labels that agree.
Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gdd import synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402

SHAPES = {"arxiv": (169343, 40, 454), "reddit": (153932, 41, 769), "products": (2449029, 47, 196)}


def timed(fn, reps=10):
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
    res = {}
    for name, (n, dim, k) in SHAPES.items():
        X = torch.from_numpy(synth.blobs(n, dim, k, seed=3)).cuda()
        C = X[torch.randperm(n, device="cuda")[:k]].contiguous()
        ops = _Ops("cuda", n, k, dim)
        l32 = torch.empty(n, dtype=torch.int32, device="cuda")
        l16 = torch.empty(n, dtype=torch.int32, device="cuda")
        t32 = timed(lambda: ops.assign(X, C, labels=l32))
        t16 = timed(lambda: ops.assign(X, C, labels=l16, precision="bf16"))
        fl = 2.0 * n * k * dim
        res[name] = {"n": n, "dim": dim, "k": k, "fp32_ms": t32, "bf16_ms": t16,
                     "fp32_TFLOPs": fl / (t32 * 1e-3) / 1e12, "bf16_TFLOPs": fl / (t16 * 1e-3) / 1e12,
                     # the bf16 pass is HBM-bound (2 n k dim flops on 4 n dim bytes: ~2k/4 flop/B
                     # below the bf16 ridge): X's bytes per call time, against 8 TB/s
                     "bf16_X_GBs": 4.0 * n * dim / (t16 * 1e-3) / 1e9,
                     "bf16_hbm_frac": 4.0 * n * dim / (t16 * 1e-3) / 8e12,
                     "label_agreement": float((l32 == l16).float().mean())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
