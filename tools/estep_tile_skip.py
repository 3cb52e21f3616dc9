#!/usr/bin/env python3
"""Feasibility of centre-tile skipping in the bounded Lloyd E-step at the products record's shape
(diagnostic): after a KMeans fit on the bench's logits, for every row with label c and
ub = ||x - C[c]||, tile g (32 consecutive centres) can hold no closer centre when
min_{c' in g} ||C[c] - C[c']|| > 2 ub (triangle inequality). Reports the fraction of (row, tile)
pairs skippable for all rows and for the rows a Hamerly-style test would list (second distance within
10% of the first), and the union over 32-row tiles in row order and in label order."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
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
    target, _ = gdd.propagate(gdd.normalize_adj(g), X, cfg.T, cfg.alpha)
    L = torch.addmm(bias, target, W)
    del g, X, target
    for it in (10, 300):
        km = gdd.KMeans(n_clusters=cfg.k, random_state=cfg.seed, max_iter=it, device=dev).fit(L)
        C = km.cluster_centers_device_.double()
        Lc = L.double() - L.double().mean(0)
        Cc = C - L.double().mean(0)
        lab = km.labels_device_.long()
        k = C.shape[0]
        G = (k + 31) // 32
        cc = torch.cdist(Cc, Cc)
        dtile = torch.stack([cc[:, 32 * t:min(k, 32 * t + 32)].masked_fill(
            (torch.arange(k, device=dev)[:, None] == torch.arange(32 * t, min(k, 32 * t + 32), device=dev)[None, :]),
            float("inf")).min(1).values for t in range(G)], 1)  # k x G
        n = Lc.shape[0]
        ub = torch.empty(n, dtype=torch.float64, device=dev)
        d2 = torch.empty(n, dtype=torch.float64, device=dev)
        for s in range(0, n, 200000):
            d = torch.cdist(Lc[s:s + 200000], Cc)
            top = d.topk(2, largest=False).values
            ub[s:s + 200000] = d.gather(1, lab[s:s + 200000, None])[:, 0]
            d2[s:s + 200000] = top[:, 1]
        need = dtile[lab] <= 2 * ub[:, None]  # n x G: tile may hold a closer centre
        need[torch.arange(n, device=dev), lab // 32] = True
        listed = d2 <= 1.1 * ub
        def union_frac(mask_rows, order):
            idx = order[mask_rows[order]]
            m = need[idx]
            t = (m.shape[0] // 32) * 32
            u = m[:t].view(-1, 32, G).any(1)
            return float(u.float().mean())
        print(f"max_iter {it}: listed {float(listed.float().mean()):.3f} of rows; tiles needed per listed row "
              f"{float(need[listed].float().mean()):.3f}; union over 32 listed rows: row order "
              f"{union_frac(listed, torch.arange(n, device=dev)):.3f}, label order "
              f"{union_frac(listed, torch.argsort(lab, stable=True)):.3f}", flush=True)


if __name__ == "__main__":
    main()
