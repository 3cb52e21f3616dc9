import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-distillation-for-recommendation_amd"))
import numpy as np, torch, gdd
from gdd import synth
X = synth.blobs(20000, 41, 300, seed=34)
print(os.environ.get("GDD_DBG"), os.environ.get("GDD_HOST_LOOP"), gdd.MiniBatchKMeans(n_clusters=300, random_state=15, batch_size=1000).fit(X).n_steps_, flush=True)
