#!/usr/bin/env python3
"""The propagation's work-list schedule (r06): the default (longest rows first, or row order where the
locality probe finds the ids local), longest first always (GDD_FORCE=hop_no_probe), row order
(hop_row_order) and row order with each XCD walking a contiguous eighth of the list
(hop_row_order,hop_xcd_contig), on the bench's graphs — arxiv (config 1/2, the headline), the
Reddit-train shape and the products shape (Chung-Lu, device-sampled) — same process, alternating,
device events, three rounds. Prints one JSON line per graph."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402

SCHEDULES = {"default": "", "noprobe": "hop_no_probe", "roworder": "hop_row_order",
             "contig": "hop_row_order,hop_xcd_contig"}
if os.environ.get("HOP_AB"):  # HOP_AB=<GDD_FORCE token>: the default against that token alone
    SCHEDULES = {"default": "", os.environ["HOP_AB"]: os.environ["HOP_AB"]}


def timed(gn, X, T, alpha, reps):
    gdd.propagate(gn, X, T, alpha)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        gdd.propagate(gn, X, T, alpha)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    graphs = []
    cfg = synth.CONFIGS["arxiv"]
    graphs.append(("arxiv chung-lu", gdd.to_csr(synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)), cfg, 20))
    if os.environ.get("HOP_AB"):
        graphs = graphs * 2
    rc = synth.CONFIGS["reddit"]
    graphs.append(("reddit-train chung-lu", synth.chung_lu_device(153932, rc.avg_degree, rc.seed), rc, 10))
    pc = synth.CONFIGS["products"]
    graphs.append(("products chung-lu", synth.chung_lu_device(pc.n, pc.avg_degree, pc.seed), pc, 2))
    graphs.append(("products-shape SBM (ids in community order)",
                   synth.sbm_device(pc.n, pc.avg_degree, 11, block=2048, p_in=0.9, shuffle=False), pc, 2))
    for name, g, c, reps in graphs:
        gn = gdd.normalize_adj(g)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(5)
        X = torch.randn(g.n, c.d, device="cuda", generator=gen)
        times = {k: [] for k in SCHEDULES}
        for _ in range(3):
            for k, tok in SCHEDULES.items():
                if tok:
                    os.environ["GDD_FORCE"] = tok
                else:
                    os.environ.pop("GDD_FORCE", None)
                times[k].append(timed(gn, X, c.T, c.alpha, reps))
        os.environ.pop("GDD_FORCE", None)
        us = {k: min(v) * 1e3 / (c.T - 1) for k, v in times.items()}
        print(json.dumps({"graph": name, "n": g.n, "nnz": int(gn.nnz), "d": c.d, "hops": c.T - 1,
                          "us_per_hop_min": us, "all_ms_per_call": times}), flush=True)
        del gn, X, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
