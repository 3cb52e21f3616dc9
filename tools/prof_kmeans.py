#!/usr/bin/env python3
"""MiniBatchKMeans at the arxiv shape, repeated (for rocprofv3 kernel traces)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import torch
import gdd
from gdd import synth
X = torch.from_numpy(synth.blobs(169343, 40, 454, seed=34)).cuda()
for r in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    m = gdd.MiniBatchKMeans(n_clusters=454, random_state=15, batch_size=1000).fit(X)
    torch.cuda.synchronize(); print(f"fit {r}: {1e3*(time.perf_counter()-t):.2f} ms steps={m.n_steps_}", flush=True)
