#!/usr/bin/env python3
"""The bench's products record k-means (bench.py products_record: the device Chung-Lu graph, N(0,1)
features, random linear logits, KMeans(k=196, random_state=15)) fitted twice, with the final cluster
sizes: where a Lloyd iteration goes at that shape. Run under rocprofv3 --kernel-trace --stats for the
per-kernel split (E-step, bounds, grouping, the ordered M-step fold, the update)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import kmeans as gk  # noqa: E402
from gdd import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = synth.CONFIGS["products"]
    g = synth.chung_lu_device(cfg.n, cfg.avg_degree, cfg.seed, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(cfg.seed)
    X = torch.randn(cfg.n, cfg.d, device=dev, generator=gen)
    W = torch.randn(cfg.d, cfg.n_classes, device=dev, generator=gen) / float(np.sqrt(cfg.d))
    bias = torch.randn(cfg.n_classes, device=dev, generator=gen) * 0.1
    gn = gdd.normalize_adj(g)
    target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha)
    logits = torch.addmm(bias, target, W)
    del g, gn, target, X
    torch.cuda.synchronize()
    # PADS="11,10,11,10": an A/B of the zero-padded copy of X for the fold and for the E-step's row lists
    # (GDD_FORCE=fold_no_pad / estep_no_pad) on the same data
    pads = os.environ.get("PADS", "")
    forms = pads.split(",") if pads else [None] * int(os.environ.get("REPS", "2"))
    for r, pad in enumerate(forms):
        if pad is not None:  # "f" or "fe": the fold's padded copy, and the E-step's row lists on it
            toks = (["fold_no_pad"] if pad[0] == "0" else []) + \
                (["estep_no_pad"] if (pad[1] if len(pad) > 1 else pad[0]) == "0" else [])
            os.environ["GDD_FORCE"] = ",".join(toks)
        kph = {}
        gk.PHASE_TIMING = kph
        t = time.perf_counter()
        km = gdd.KMeans(n_clusters=cfg.k, random_state=cfg.seed, device=dev).fit(logits)
        lab = km.labels_device_
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        gk.PHASE_TIMING = None
        cnt = torch.bincount(lab.long(), minlength=cfg.k).cpu().numpy()
        top = np.sort(cnt)[::-1]
        print(f"rep {r}{'' if pad is None else ' pads=' + pad}: fit {ms:.1f} ms, {int(km.n_iter_)} iterations, phases "
              + " ".join(f"{k}={v:.1f}" if isinstance(v, float) else f"{k}={v}" for k, v in kph.items())
              + f"; cluster sizes max {top[0]} mean {cnt.mean():.0f} top5 {top[:5].tolist()} "
              f"min {top[-1]}", flush=True)
    np.save(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/products_cluster_sizes.npy", cnt)


if __name__ == "__main__":
    main()
