#!/usr/bin/env python3
"""Statistics of the rank-split Lloyd M-step fold (the CPU model
tests/signed_chain.py rank_split_fold, pinned bit-exact by tests/test_lloyd_rank_split_model.py) at
the products shape: 2,449,029 x 47 logit-like rows (N(0,1) features through a random 100 x 47 map plus
a bias, centred as KMeans.fit centres them), labels from 196 centres drawn from the rows; MODEL_CHAINS
random (cluster, column) chains, each split over R ranks' contiguous row blocks. Prints, per (R, L):
the fallback rate, the share of segments shipped raw, and the bytes each rank ships per iteration
(extrapolated to all k x C chains) against the labels all-gather it would replace (1 byte per row at
k <= 256). One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from signed_chain import rank_split_fold, seq_sum  # noqa: E402

N, D, C, K = 2449029, 100, 47, 196
CHAINS = int(os.environ.get("MODEL_CHAINS", "24"))


def main():
    t0 = time.time()
    g = torch.Generator().manual_seed(5)
    W = torch.randn(D, C, generator=g) / 10.0
    b = torch.randn(C, generator=g)
    X = torch.empty(N, C)
    for i in range(0, N, 1 << 18):
        X[i:i + (1 << 18)] = torch.randn(min(1 << 18, N - i), D, generator=g) @ W + b
    X -= X.mean(0)
    cent = X[torch.randperm(N, generator=g)[:K]]
    cn = (cent * cent).sum(1)
    lab = torch.empty(N, dtype=torch.int64)
    for i in range(0, N, 1 << 17):
        xb = X[i:i + (1 << 17)]
        lab[i:i + (1 << 17)] = (cn[None, :] - 2.0 * xb @ cent.T).argmin(1)
    Xn, labn = X.numpy(), lab.numpy()
    rng = np.random.default_rng(3)
    picks = [(int(rng.integers(0, K)), int(rng.integers(0, C))) for _ in range(CHAINS)]
    out = {"shape": [N, C, K], "chains_sampled": CHAINS, "setup_s": time.time() - t0, "by_config": []}
    for R in (2, 4, 8):
        bounds = [N * r // R for r in range(R + 1)]
        for L in (256, 1024):
            fb = raw = rec = 0
            members = 0
            for c, j in picks:
                rows = np.nonzero(labn == c)[0]
                terms = Xn[rows, j]
                members += len(rows)
                blocks = [terms[(rows >= bounds[r]) & (rows < bounds[r + 1])] for r in range(R)]
                s, st = rank_split_fold(blocks, L)
                if s is not None:
                    assert s.view(np.uint32) == seq_sum(terms).view(np.uint32)
                fb += int(st["fallback"])
                raw += st["raw"]
                rec += st["records"]
            scale = K * C / CHAINS
            rec_bytes = rec * (2 * 24 + 2) * scale / R      # two 24-byte transducers + binade ids
            raw_bytes = raw * L * 4 * scale / R
            cfg = {"R": R, "L": L, "fallback_chains": fb, "fallback_rate": fb / CHAINS,
                   "segments_raw_share": raw / max(1, raw + rec),
                   "bytes_per_rank_per_iteration": rec_bytes + raw_bytes,
                   "of_which_raw": raw_bytes,
                   "labels_allgather_bytes_per_rank": N / R, "mean_members_per_chain": members / CHAINS}
            out["by_config"].append(cfg)
            print(json.dumps(cfg), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
