#!/usr/bin/env python3
"""bench.py — the ClustGDD distillation hot path on MI355X (BASELINE.json metric).

One *step* = one pass of the hot path of ``ClustGDD.pretrained_clustering``
(clustgdd_agent_transduct.py:38-129) over one ogbn-arxiv-shaped graph already resident in HBM:

    normalise Â (a2) -> 17 propagation hops (a3) -> linear "MLP" logits (a4 stand-in, one GEMM)
    -> MiniBatchKMeans(k=454, batch 1000, seed 15) on the logits (a5) -> per-cluster feature means
    and argmax labels (a7)

Synthetic data of the arxiv shape (N=169,343, d=128, ~2.4M nnz Chung-Lu power-law graph, C=40),
because the dataset cannot be downloaded here. ``value`` = nodes distilled per second over the
whole job (N x steps x ranks / max-over-ranks wall time); ``ms_per_step`` is the distill
wallclock. Multi-GPU: one process per GPU, each rank distils its own graph (independent
objects, no data-path collective): weak scaling.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config arxiv] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="arxiv")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=60,
                    help="minibatch steps the CPU baseline sample runs (extrapolated)")
    return ap.parse_args()


def setup_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus and world != 1:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def main():
    args = parse()
    rank, world, local = setup_dist(args.gpus)
    import gdd
    from gdd import synth

    cfg = synth.CONFIGS[args.config]
    seed = cfg.seed + 1000 * rank
    dev = torch.device("cuda", local)
    A = synth.chung_lu(cfg.n, cfg.avg_degree, seed)
    X_h = synth.features(cfg.n, cfg.d, seed)
    rng = np.random.default_rng(seed + 3)
    W = torch.from_numpy((rng.standard_normal((cfg.d, cfg.n_classes)) / np.sqrt(cfg.d)).astype(np.float32)).to(dev)
    b = torch.from_numpy((rng.standard_normal(cfg.n_classes) * 0.1).astype(np.float32)).to(dev)
    graph = gdd.to_csr(A, device=dev)
    X = torch.from_numpy(X_h).to(dev)
    nnz_in = graph.nnz
    torch.cuda.synchronize()

    prop_ev = []

    def step(record=False):
        gn = gdd.normalize_adj(graph)
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha)
        if record:
            e1.record()
            prop_ev.append((e0, e1, gn.nnz))
        logits = torch.addmm(b, target, W)
        if cfg.kmeans == "minibatch":
            km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed,
                                     batch_size=cfg.batch, device=dev).fit(logits)
        else:
            km = gdd.KMeans(n_clusters=cfg.k, device=dev).fit(logits)
        feat_syn, _ = gdd.cluster_mean(target, km.labels_device_, cfg.k)
        labels_syn = gdd.argmax_rows(km.cluster_centers_device_)
        return feat_syn, labels_syn, km

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_steps_km = []
    for _ in range(args.steps):
        _, _, km = step(record=True)
        n_steps_km.append(getattr(km, "n_steps_", getattr(km, "n_iter_", 0)))
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())

    # roofline of the dominant HBM kernel: one propagation hop (k_hop + its split-row fix-up), timed
    # per launch with HIP events on the stream it runs on, against a plan built once (the same
    # plan gdd_propagate builds per call)
    gn = gdd.normalize_adj(graph)
    n, d, hops = cfg.n, cfg.d, cfg.T - 1
    nnz = gn.nnz
    plan = gdd.graph.SpMMPlan(gn, d)
    bufs = [X.clone(), torch.empty_like(X)]
    acc = torch.zeros_like(X)
    w32 = float(np.float32(1.0 - cfg.alpha))
    for h in range(3):
        plan.hop(bufs[h % 2], bufs[(h + 1) % 2], cfg.alpha, acc, w32)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for h in range(hops):
        plan.hop(bufs[h % 2], bufs[(h + 1) % 2], cfg.alpha, acc, w32)
    ev[1].record()
    torch.cuda.synchronize()
    hop_ms = ev[0].elapsed_time(ev[1]) / hops
    prop_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1, _ in prop_ev]))
    bytes_hop = 4 * (n + 1) + 8 * nnz + 16 * n * d  # rowptr, col, val, p_in, p_out, target r/w
    achieved = bytes_hop / (hop_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic()
    copy_gbs = copy_peak(dev)

    out = {
        "metric": "distill wallclock (SpMM+k-means) & test-acc parity, ogbn-arxiv r=0.5% @1-8 GPU",
        "value": cfg.n * args.steps * world / t_max,
        "unit": "nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * t_max / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (Chung-Lu power-law graph + N(0,1) features of the ogbn-arxiv shape; "
                "random linear logits)",
        "config": {"workload": f"{cfg.name} pretrained_clustering hot path: normalize + "
                               f"{hops} SpMM hops + MiniBatchKMeans(k={cfg.k}, b={cfg.batch}) + "
                               "cluster means",
                   "nodes": cfg.n, "nnz_in": nnz_in, "nnz_norm": nnz, "feat_dim": d,
                   "k": cfg.k, "parallelism": f"replicas x{world} (one graph per GPU)",
                   "kmeans_steps": n_steps_km},
        "roofline": {"bound": "hbm", "kernel": "k_hop (+ k_fixup): one propagation hop",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": bytes_hop, "avg_launch_ms": hop_ms,
                     "traffic_source": traffic_src, "propagate_call_ms": prop_ms,
                     "copy_peak_measured": copy_gbs, "frac_of_copy_peak": achieved / copy_gbs},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, A, X_h, args.cpu_steps, n_steps_km[-1])
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def copy_peak(dev, nbytes=1 << 30, reps=10):
    """Achievable HBM bandwidth on this box: libgdd's streaming copy of 1 GiB (read + write bytes
    per copy), timed with HIP events on the stream it runs on."""
    from gdd import _lib
    lib = _lib.device_lib()
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    st = _lib.stream_ptr(dev)
    for _ in range(3):
        _lib.check(lib.gdd_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, st))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        _lib.check(lib.gdd_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, st))
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    if not torch.equal(src[:1024], dst[:1024]) or not torch.equal(src[-1024:], dst[-1024:]):
        raise RuntimeError("stream copy mismatch")
    del src, dst
    return 2 * nbytes / (ms * 1e-3) / 1e9


def pmc_traffic():
    """HBM-side bytes per k_hop launch from the newest committed rocprofv3 PMC summary
    (profiles/<round>_khop_traffic.json, written by tools/pmc_summary.py from FETCH_SIZE and
    WRITE_SIZE passes of this same bench command), or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_khop_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        rec = json.load(f)
    return rec.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def cpu_baseline(cfg, A, X_h, cpu_steps, gpu_km_steps):
    """The oracle (single-threaded C restatement) on a bounded sample of the same workload:
    full normalise + propagation, k-means++ + `cpu_steps` minibatch steps (extrapolated to the
    step count the GPU run took) + full labels pass + cluster means."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    import scipy.sparse as sp
    from gdd import synth
    A = sp.csr_matrix(A)
    t0 = time.perf_counter()
    ro, co, vo = O.normalize_csr(A.indptr, A.indices, None, -1)
    target, _ = O.propagate(ro, co, vo, X_h, cfg.T, cfg.alpha)
    t_graph = time.perf_counter() - t0
    rng = np.random.default_rng(cfg.seed + 3)
    W = (rng.standard_normal((cfg.d, cfg.n_classes)) / np.sqrt(cfg.d)).astype(np.float32)
    b = (rng.standard_normal(cfg.n_classes) * 0.1).astype(np.float32)
    logits = target @ W + b
    t1 = time.perf_counter()
    res = O.minibatch_kmeans(logits, cfg.k, random_state=cfg.seed, batch_size=cfg.batch,
                             max_iter=max(1, (cpu_steps * cfg.batch) // cfg.n + 1),
                             compute_labels=False)
    t_km_sample = time.perf_counter() - t1
    steps_done = res["n_steps_"]
    t2 = time.perf_counter()
    labels, _ = O.labels_inertia(logits, res["cluster_centers_"])
    O.cluster_mean(target, labels, cfg.k)
    t_tail = time.perf_counter() - t2
    # extrapolate the minibatch loop to the GPU run's step count (the init is paid once)
    t_est = t_graph + t_km_sample * max(gpu_km_steps, 1) / max(steps_done, 1) + t_tail
    sample_s = t_graph + t_km_sample + t_tail
    return {"value": cfg.n / t_est, "unit": "nodes/s", "cores": 1, "kind": "port",
            "sample": f"oracle/ C restatement, 1 thread: normalise + {cfg.T - 1} hops on the full "
                      f"graph, k-means++ and {steps_done} of {gpu_km_steps} minibatch steps "
                      f"(extrapolated), full labels pass + cluster means; {sample_s:.1f} s measured",
            "est_seconds_per_step": t_est}


if __name__ == "__main__":
    main()
