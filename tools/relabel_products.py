#!/usr/bin/env python3
"""Propagation locality at the products shape: gdd.propagate(T = 18, d = 100) on
2,449,029-node graphs with the intermediate hops in other node orders (gdd_propagate_relabeled:
bit-identical results), device events, same process.

Graphs: a community-structured stochastic block model of the products shape (~126M entries, blocks
of 2,048 nodes, 90% of each node's edges inside its block) with shuffled ids (real graphs' ids carry
no locality) and with contiguous blocks (the order a perfect relabel would recover), and the bench's
products-shaped Chung-Lu graph. Orders: the original ids, "degree", "rcm" (scipy, host) and, for
the shuffled SBM, the true community order.

Each order runs under three hop schedules (GDD_FORCE): "default" (original ids: longest rows first,
or row order where the locality probe finds the ids local; relabelled: the new order), "noprobe"
(hop_no_probe: longest first for original ids) and "contig" (hop_row_order,hop_xcd_contig: each XCD
walks a contiguous eighth of the list, so a row range's gathers stay in one L2). Prints one JSON line per (graph, order, schedule) and a summary line. RELABEL_REPS
(default 3) timed calls per configuration. Between configurations it launches a marker fill of (i + 1) * 1,000,000 floats, so a
rocprofv3 --pmc FETCH_SIZE pass of this script can be split per configuration
(tools/relabel_products_pmc.py)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import synth  # noqa: E402

REPS = int(os.environ.get("RELABEL_REPS", "3"))
SCHEDULES = {"default": "", "noprobe": "hop_no_probe", "contig": "hop_row_order,hop_xcd_contig"}
_marks = [0]


def marker():
    _marks[0] += 1
    torch.empty(_marks[0] * 1000000, device="cuda").fill_(0.0)
    torch.cuda.synchronize()
    return _marks[0]


def timed(gn, X, T, alpha, relabel):
    out = gdd.propagate(gn, X, T, alpha, relabel=relabel)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        gdd.propagate(gn, X, T, alpha, relabel=relabel)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS, out


def run(name, g, cfg, orders, res):
    gn = gdd.normalize_adj(g)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    X = torch.randn(g.n, cfg.d, device="cuda", generator=gen)
    hops = cfg.T - 1
    ref = None
    for kind, rho_fn in orders:
        t0 = time.time()
        rho = rho_fn(gn) if rho_fn else None
        order_s = time.time() - t0
        for sched, tok in SCHEDULES.items():
            if tok:
                os.environ["GDD_FORCE"] = tok
            else:
                os.environ.pop("GDD_FORCE", None)
            mk = marker()
            ms, (t, p) = timed(gn, X, cfg.T, cfg.alpha, rho)
            if ref is None:
                ref = (t, p)
            same = torch.equal(t.view(torch.int32), ref[0].view(torch.int32)) and \
                torch.equal(p.view(torch.int32), ref[1].view(torch.int32))
            rec = {"graph": name, "order": kind, "schedule": sched, "n": g.n, "nnz": int(gn.nnz),
                   "d": cfg.d, "hops": hops, "ms_per_call": ms, "us_per_hop": ms * 1e3 / hops,
                   "order_build_s": order_s, "bit_identical_to_original_order": bool(same), "marker": mk,
                   "calls": 1 + REPS}
            res.append(rec)
            print(json.dumps(rec), flush=True)
        os.environ.pop("GDD_FORCE", None)
    del gn, X


def main():
    pc = synth.CONFIGS["products"]
    res = []
    rcm = ("rcm", lambda gn: gdd.graph.locality_order(gn, "rcm"))
    deg = ("degree", lambda gn: gdd.graph.locality_order(gn, "degree"))
    for shuffle in (True, False):
        g, perm = synth.sbm_device(pc.n, pc.avg_degree, 11, block=2048, p_in=0.9, shuffle=shuffle,
                                   return_perm=True)
        orders = [("original", None), deg, rcm] if shuffle else [("original", None)]
        if shuffle:  # node perm[i] sits in block i // 2048: the community order puts it at row i
            def community(gn, perm=perm):
                rho = torch.empty(gn.n, dtype=torch.int32, device="cuda")
                rho[perm] = torch.arange(gn.n, dtype=torch.int32, device="cuda")
                return rho
            orders.append(("community", community))
        run(f"products-shape SBM ({'shuffled ids' if shuffle else 'contiguous blocks'})", g, pc,
            orders, res)
        del g, perm
        torch.cuda.empty_cache()
    g = synth.chung_lu_device(pc.n, pc.avg_degree, pc.seed)
    run("products chung-lu (bench graph)", g, pc, [("original", None), deg], res)
    print(json.dumps({"summary": [(r["graph"], r["order"], r["schedule"], round(r["us_per_hop"], 1))
                                  for r in res]}), flush=True)


if __name__ == "__main__":
    main()
