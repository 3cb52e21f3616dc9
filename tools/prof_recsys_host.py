#!/usr/bin/env python3
"""Host-side profile (cProfile, by own time) of five warm distill_recsys.kmeans_cluster fits at the ML-1M
users shape: where the fit spends Python / driver time around its device work."""
import cProfile, pstats, io, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-distillation-for-recommendation_amd"))
import torch
from gdd import synth
from gdd.pipeline import kmeans_cluster
Eu = synth.svd_like(6040, 64, seed=6040)
for _ in range(3):
    kmeans_cluster(Eu, 604, seed=42, device="cuda")
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    kmeans_cluster(Eu, 604, seed=42, device="cuda")
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:6000])
