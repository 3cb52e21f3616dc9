import os, sys, time, ctypes
sys.path.insert(0, os.path.join(os.getcwd(), "graph-distillation-for-recommendation_amd"))
import numpy as np, torch
import gdd
from gdd import _lib, synth
calls = []
def cb(w_ptr, k, out_ptr):
    t = time.perf_counter()
    _lib._np_argsort(w_ptr, k, out_ptr)
    calls.append(time.perf_counter() - t)
_lib.argsort_callback = _lib.ARGSORT_CB(cb)
dev = torch.device("cuda", 0)
cfg = synth.CONFIGS["reddit"]
g = synth.chung_lu_device(cfg.n, cfg.avg_degree, cfg.seed, device=dev)
gen = torch.Generator(device=dev); gen.manual_seed(cfg.seed)
X = torch.randn(cfg.n, cfg.d, device=dev, generator=gen)
W = torch.randn(cfg.d, cfg.n_classes, device=dev, generator=gen) / float(np.sqrt(cfg.d))
target, _ = gdd.propagate(gdd.normalize_adj(g), X, cfg.T, cfg.alpha)
L = target @ W
for rep in range(3):
    calls.clear()
    torch.cuda.synchronize(); t = time.perf_counter()
    km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch).fit(L)
    torch.cuda.synchronize()
    print(f"fit {1e3*(time.perf_counter()-t):.2f} ms, steps {km.n_steps_}, argsort callbacks {len(calls)} ({1e3*sum(calls):.2f} ms in numpy)", flush=True)
