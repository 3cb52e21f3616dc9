#!/usr/bin/env python3
"""bench.py — the ClustGDD distillation hot path on MI355X (BASELINE.json metric).

One *step* = one pass of the hot path of ``ClustGDD.pretrained_clustering``
(clustgdd_agent_transduct.py:38-129) over one ogbn-arxiv-shaped graph already resident in HBM:

    normalise Â (a2) -> 17 propagation hops (a3) -> linear "MLP" logits (a4 stand-in, one GEMM)
    -> MiniBatchKMeans(k=454, batch 1000, seed 15) on the logits (a5) -> per-cluster feature means
    and argmax labels (a7)

Synthetic data of the arxiv shape (N=169,343, d=128, ~2.4M nnz Chung-Lu power-law graph, C=40),
because the dataset cannot be downloaded here. ``value`` = nodes distilled per second over the
whole job (graphs x N x steps / max-over-ranks wall time); ``ms_per_step`` is the distill
wallclock.

Multi-GPU, one process per GPU. The arxiv step does not shard: its T-hop halo is the
whole graph and MiniBatchKMeans is ~260 latency-bound sequential steps, so ``--mode replicas``
(default) runs N independent distillations, one graph per GPU (seed + rank), with no collective in
the data path ("scaling": "weak"). ``--mode one-graph`` distils ONE graph over all ranks as the north
star partitions it (gdd.sharded: labels pass by rows, cluster means by clusters, RCCL all-gathers,
bit-identical to one GPU; "scaling": "strong"); at N > 1 the replicas line also carries that mode's
time for the same graph under ``one_graph``.

The same line carries sub-records measured in this run: ``recsys`` (config 4's kmeans_cluster pair),
``products`` (config 5 at full shape; at N = 1 also fp32 vs bf16 labels pass), ``reddit`` (config
3's whole inductive path: GraphSAINT split, three role graphs, fit, means), and at N = 1 ``e2e``
(the drop-in agent with main_transduct.sh's arxiv flags: stage times and the five GCN accuracies)
and the CPU baselines. At N > 1 the recsys/products/reddit records distil ONE instance over all
ranks as north_star splits it.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config arxiv] [--mode replicas|one-graph]
                       [--no-cpu-baseline] [--no-extra] [--no-e2e]
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
    ap.add_argument("--mode", choices=("replicas", "one-graph"), default="replicas")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the recsys / products / reddit / e2e sub-records (quick A/B runs)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the drop-in agent run")
    return ap.parse_args()


def setup_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus and world != 1:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    # GDD_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with fewer GPUs than ranks (ranks
    # then share devices round-robin); the measured configuration is RCCL, one GPU per rank
    backend = os.environ.get("GDD_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
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
    one_graph = args.mode == "one-graph"
    seed = cfg.seed + (0 if one_graph else rank)  # replicas: an independent graph per rank
    dev = torch.device("cuda", local)
    group = None
    if world > 1 and one_graph:
        import torch.distributed as dist
        group = dist.group.WORLD
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

    def step(record=False, group=group):
        gn = gdd.normalize_adj(graph)
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha, group=group)
        if record:
            e1.record()
            prop_ev.append((e0, e1, gn.nnz))
        logits = torch.addmm(b, target, W)
        if cfg.kmeans == "minibatch":
            km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed,
                                     batch_size=cfg.batch, device=dev, group=group).fit(logits)
        else:
            from gdd.pipeline import _lloyd
            km = _lloyd(cfg.k, group, device=dev).fit(logits)
        feat_syn, _ = gdd.cluster_mean(target, km.labels_device_, cfg.k, group=group)
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
    t_max = max_over_ranks(elapsed, world, dev)
    one_graph_rec = None
    if world > 1 and not one_graph:
        # the same graph (rank 0's) distilled over all ranks, for the strong-scaling comparison
        import torch.distributed as dist
        if rank != 0:
            A1 = synth.chung_lu(cfg.n, cfg.avg_degree, cfg.seed)
            graph_1, X_1 = gdd.to_csr(A1, device=dev), torch.from_numpy(synth.features(cfg.n, cfg.d, cfg.seed)).to(dev)
            graph, X = graph_1, X_1
        g_all = dist.group.WORLD
        for _ in range(args.warmup):
            step(group=g_all)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(group=g_all)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        t1_max = max_over_ranks(time.perf_counter() - t1, world, dev)
        one_graph_rec = {"ms_per_step": 1e3 * t1_max / args.steps, "value": cfg.n * args.steps / t1_max,
                         "unit": "nodes/s", "scaling": "strong",
                         "parallelism": f"one graph over {world} ranks (gdd.sharded)"}
        if rank != 0:
            graph, X = gdd.to_csr(A, device=dev), torch.from_numpy(X_h).to(dev)

    # per-phase wall times of one more (untimed) step, synchronised between phases (SURVEY §8(d):
    # hot-path wallclock by stage and nodes clustered per second = N / k-means wallclock)
    phases = {}
    for _ in range(2):
        ph = {}

        def mark(name, t_prev):
            torch.cuda.synchronize()
            now = time.perf_counter()
            ph[name] = (now - t_prev) * 1e3
            return now
        torch.cuda.synchronize()
        tp = time.perf_counter()
        gn_p = gdd.normalize_adj(graph)
        tp = mark("normalize", tp)
        target_p, _ = gdd.propagate(gn_p, X, cfg.T, cfg.alpha, group=group)
        tp = mark("propagate", tp)
        logits_p = torch.addmm(b, target_p, W)
        tp = mark("logits", tp)
        if cfg.kmeans == "minibatch":
            km_p = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch,
                                       device=dev, group=group).fit(logits_p)
        else:
            from gdd.pipeline import _lloyd
            km_p = _lloyd(cfg.k, group, device=dev).fit(logits_p)
        tp = mark("kmeans", tp)
        gdd.cluster_mean(target_p, km_p.labels_device_, cfg.k, group=group)
        gdd.argmax_rows(km_p.cluster_centers_device_)
        mark("cluster_mean", tp)
        phases = ph
        del gn_p, target_p, logits_p, km_p

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
    mfma = assign_mfma(cfg, dev)
    with_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    # configs 4, 5 and 3 at their full shapes, measured in this run: at N = 1 on one GPU; at N > 1
    # ONE instance over all ranks as north_star splits it (recsys: the users' and items' fits on
    # ranks 0 and 1; products: row-partitioned propagation; Reddit: the role graphs on different
    # ranks) — VERDICT r5 #1/#5. The drop-in agent end to end runs at N = 1.
    extra = cfg.name == "ogbn-arxiv" and not args.no_extra
    g_all = None
    if world > 1:
        import torch.distributed as dist
        g_all = dist.group.WORLD
    recsys = recsys_record(dev, with_cpu=with_cpu, group=g_all, world=world) if extra else None
    products = products_record(dev, with_cpu=with_cpu, group=g_all, world=world) if extra else None
    reddit = reddit_record(dev, with_cpu=with_cpu, group=g_all, world=world) if extra else None
    e2e = e2e_record(dev) if extra and world == 1 and not args.no_e2e else None

    out = {
        "metric": "distill wallclock (SpMM+k-means) & test-acc parity, ogbn-arxiv r=0.5% @1-8 GPU",
        "value": cfg.n * args.steps * (1 if one_graph else world) / t_max,
        "unit": "nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * t_max / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if one_graph else "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (Chung-Lu power-law graph + N(0,1) features of the ogbn-arxiv shape; "
                "random linear logits)",
        "config": {"workload": f"{cfg.name} pretrained_clustering hot path: normalize + "
                               f"{hops} SpMM hops + MiniBatchKMeans(k={cfg.k}, b={cfg.batch}) + "
                               "cluster means",
                   "nodes": cfg.n, "nnz_in": nnz_in, "nnz_norm": nnz, "feat_dim": d,
                   "k": cfg.k,
                   "parallelism": ("single GPU" if world == 1 else
                                   (f"one graph over {world} ranks: labels pass by rows, cluster "
                                    "means by clusters (RCCL all-gathers); normalise, propagation "
                                    "and minibatch steps replicated") if one_graph else
                                   f"replicas x{world}: one graph per GPU, no data-path collective"),
                   "kmeans_steps": n_steps_km},
        # what `value` counts at this world size: replicas are N independent graphs
        # (aggregate throughput; ms_per_step stays one graph's distill wallclock); one-graph mode is
        # the strong-scaling distillation of a single graph over all ranks
        "value_basis": ("one graph on one GPU" if world == 1 else
                        f"one graph distilled over {world} ranks (strong scaling)" if one_graph else
                        f"{world} independent graphs, one per GPU (aggregate nodes/s over all ranks; "
                        "ms_per_step is one graph's wallclock; the strong-scaling time of rank 0's "
                        "graph over all ranks is under one_graph)"),
        "phases_ms": phases,
        "nodes_clustered_per_s": cfg.n / (phases["kmeans"] * 1e-3) if phases.get("kmeans") else None,
        "roofline": {"bound": "hbm", "kernel": "k_hop (+ k_fixup): one propagation hop",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": bytes_hop, "avg_launch_ms": hop_ms,
                     "traffic_source": traffic_src, "propagate_call_ms": prop_ms,
                     "copy_peak_measured": copy_gbs, "frac_of_copy_peak": achieved / copy_gbs},
        "mfma_assign": mfma,
        "recsys": recsys,
        "products": products,
        "reddit": reddit,
        "e2e": e2e,
        "cpu_baseline": None,
        "test_acc": {"parity_test": "tests/test_agent_cpu.py (G10: the reference agent's Train/Test "
                                    "Mean Accuracy reproduced exactly on CPU)",
                     "measured_here": ("e2e.train_test_mean: this run's drop-in agent on the "
                                       "synthetic arxiv-shaped dataset") if e2e else None},
    }
    if one_graph_rec is not None:
        out["one_graph"] = one_graph_rec
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, A, X_h)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def recsys_record(dev, with_cpu, reps=10, group=None, world=1):
    """Config 4's clustering stage on the bipartite recsys graph (north_star's second target):
    distill_recsys.kmeans_cluster (distill_recsys.py:158-181) as main() calls it (:565-583) — users
    then items, StandardScaler + KMeans(n_clusters=k, random_state=42, n_init="auto") — on
    ML-1M-shaped synthetic SVD embeddings (6,040 users x 64 with k = 604, 3,706 items x 64 with
    k = 371: reduction 0.1, svd 64), through gdd.pipeline.kmeans_cluster_pair: at N > 1 the users' fit
    on rank 0 and the items' on rank 1, results broadcast over RCCL (bit-identical to one GPU). Warm
    calls; wallclock per pair (max over ranks), nodes clustered per second; at N = 1 also a
    synchronised phase split of one more call each, the Lloyd assignment's MFMA use, and the
    reference's own scikit-learn calls on the host cores beside it."""
    from gdd import kmeans as gk
    from gdd import synth
    from gdd.pipeline import kmeans_cluster_pair, standard_scaler
    shapes = [("users", 6040, 604), ("items", 3706, 371)]
    E = {name: synth.svd_like(n, 64, seed=n) for name, n, _ in shapes}

    def pair():
        return kmeans_cluster_pair(E["users"], E["items"], 604, 371, seed=42, minibatch=True,
                                   device=dev, group=group)
    ms = _timed_ms(pair, reps, world, dev)
    nodes = sum(n for _, n, _ in shapes)
    rec = {"workload": "distill_recsys.kmeans_cluster x2 (users 6040x64 k=604, items 3706x64 k=371; "
                       "StandardScaler + KMeans(random_state=42, n_init='auto')), ML-1M shape",
           "data": "synthetic SVD-like embeddings (gdd.synth.svd_like)",
           "parallelism": ("single GPU" if world == 1 else
                           f"{world} ranks: users' fit on rank 0, items' on rank 1 (independent "
                           f"random_state each), labels and centres broadcast over {_backend_name(group)}"),
           "ms_per_pair": ms, "nodes_clustered_per_s": nodes / (ms * 1e-3), "cpu_baseline": None}
    if world > 1:
        return rec
    phases = {}
    for name, n, k in shapes:
        ph = {}
        torch.cuda.synchronize()
        tp = time.perf_counter()
        Xs, _, _ = standard_scaler(E[name], device=dev)  # includes the H2D copy of the embeddings
        torch.cuda.synchronize()
        ph["scaler"] = (time.perf_counter() - tp) * 1e3
        gk.PHASE_TIMING = ph
        try:
            tp = time.perf_counter()
            km = gk.KMeans(n_clusters=k, random_state=42, n_init="auto", device=dev).fit(Xs)
            lab, cen = km.labels_, km.cluster_centers_  # the host copies kmeans_cluster returns
            ph["to_host"] = (time.perf_counter() - tp) * 1e3 - sum(
                v for key, v in ph.items() if key not in ("scaler", "lloyd_calls"))
        finally:
            gk.PHASE_TIMING = None
        ph["n_iter"] = int(km.n_iter_)
        phases[name] = ph
        del lab, cen
    # the Lloyd E-step's distance GEMM at the users shape (2 n k d flops per call)
    from gdd.kmeans import _Ops
    n, k = shapes[0][1], shapes[0][2]
    Xs, _, _ = standard_scaler(E["users"], device=dev)
    C = Xs[:k].clone()
    ops = _Ops(dev, n, k, 64)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(3):
        ops.assign(Xs, C, labels=lab)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        ops.assign(Xs, C, labels=lab)
    ev[1].record()
    torch.cuda.synchronize()
    a_ms = ev[0].elapsed_time(ev[1]) / 20
    tf = 2.0 * n * k * 64 / (a_ms * 1e-3) / 1e12
    rec.update(phases_ms=phases,
               lloyd_assign_mfma={"achieved": tf, "peak": FP32_MATRIX_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": tf / FP32_MATRIX_PEAK_TFLOPS, "avg_launch_ms": a_ms,
                                  "shape": "6040 x 64 against 604 centres"})
    if with_cpu:
        rec["cpu_baseline"] = recsys_cpu_baseline(E, shapes)
    return rec


def _timed_ms(fn, reps, world, dev, warm=1):
    """ms per call of fn(): `warm` untimed calls, then `reps` timed ones bracketed by a barrier and a
    device sync on both sides, the max over ranks."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    return 1e3 * max_over_ranks(time.perf_counter() - t0, world, dev) / reps


def recsys_cpu_baseline(E, shapes):
    """distill_recsys.kmeans_cluster's own library calls (StandardScaler().fit_transform, then
    KMeans(n_clusters=k, random_state=42, n_init="auto").fit) for users and items, on the threads
    this process may use (min of the affinity mask and OMP_NUM_THREADS, the box's policy)."""
    from sklearn.cluster import KMeans as SkKMeans
    from sklearn.preprocessing import StandardScaler
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)
    threads = min(affinity, omp) if omp else affinity
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=threads)
    except ImportError:  # pragma: no cover
        limiter = None
    t0 = time.perf_counter()
    iters = {}
    for name, n, k in shapes:
        Xs = StandardScaler().fit_transform(E[name])
        km = SkKMeans(n_clusters=k, random_state=42, n_init="auto").fit(Xs)
        iters[name] = int(km.n_iter_)
    total = time.perf_counter() - t0
    if limiter is not None and hasattr(limiter, "unregister"):
        limiter.unregister()
    nodes = sum(n for _, n, _ in shapes)
    return {"value": nodes / total, "unit": "nodes/s", "seconds": total, "cores": threads,
            "kind": "reference-library", "affinity_cpus": affinity, "omp_num_threads": omp or None,
            "cpu_model": _cpu_model(), "n_iter": iters,
            "sample": "both kmeans_cluster calls once (StandardScaler + scikit-learn KMeans), "
                      f"{threads} threads"}


def max_over_ranks(seconds, world, dev):
    t = torch.tensor([seconds], dtype=torch.float64, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


FP32_MATRIX_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)


def assign_mfma(cfg, dev, reps=20):
    """MFMA use of the distance GEMM (north_star): the MiniBatchKMeans final labels pass at the bench
    shape (n x C logits against k centres: ||C||^2, the fp32 MFMA distance tiles with the fused
    argmin, the label/distance finalize), timed per call with HIP events on the launching stream;
    2 n k C flops per call."""
    from gdd.kmeans import _Ops
    g = torch.Generator(device=dev).manual_seed(cfg.seed)
    Xl = torch.randn(cfg.n, cfg.n_classes, device=dev, generator=g)
    C = Xl[: cfg.k].clone()
    ops = _Ops(dev, cfg.n, cfg.k, cfg.n_classes)
    lab = torch.empty(cfg.n, dtype=torch.int32, device=dev)
    for _ in range(3):
        ops.assign(Xl, C, labels=lab)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        ops.assign(Xl, C, labels=lab)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    flops = 2.0 * cfg.n * cfg.k * cfg.n_classes
    tf = flops / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "kernel": "labels pass: k_assign_waves (v_mfma_f32_32x32x2_f32 chains + "
                                     "argmin) + finalize", "achieved": tf,
            "peak": FP32_MATRIX_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP32_MATRIX_PEAK_TFLOPS,
            "flops_per_launch": flops, "avg_launch_ms": ms,
            "note": "exact fp32 k-ordered chains (sklearn's sgemm bits); K = C = 40"}


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


def _threads():
    """(threads, affinity, omp): the host threads a CPU baseline may use — min of the affinity mask
    and OMP_NUM_THREADS (the GPU box's lease sets the latter to its CPU share)."""
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)
    return (min(affinity, omp) if omp else affinity), affinity, omp


class _CpuThreads:
    """torch + BLAS/OpenMP limited to `threads` inside the block."""

    def __init__(self, threads):
        self.threads = threads

    def __enter__(self):
        self.prev = torch.get_num_threads()
        torch.set_num_threads(self.threads)
        try:
            from threadpoolctl import threadpool_limits
            self.lim = threadpool_limits(limits=self.threads)
        except ImportError:  # pragma: no cover
            self.lim = None
        return self

    def __exit__(self, *exc):
        if self.lim is not None and hasattr(self.lim, "unregister"):
            self.lim.unregister()
        torch.set_num_threads(self.prev)


def _sync_mark(ph, name, t_prev):
    torch.cuda.synchronize()
    now = time.perf_counter()
    ph[name] = (now - t_prev) * 1e3
    return now


def _products_pmc_traffic():
    """HBM bytes per products hop from the latest committed PMC record (profiles/<round>_hop_products_pmc.json,
    tools/pmc_summary.py over three separate rocprofv3 --pmc passes; a counter run cannot share this
    process), or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hop_products_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        rec = json.load(f)
    return rec.get("default", {}).get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def _hop_roofline(gn, X, alpha, reps=10):
    """One unpaired planned hop (SpMMPlan.hop with the target update, the same plan gdd_propagate
    builds per call), timed with HIP events on the stream gdd launches on (torch's current stream):
    average launch duration and its algorithmic bytes 4(N+1) + 8 nnz + 16 N d."""
    import gdd
    n, d = X.shape
    plan = gdd.graph.SpMMPlan(gn, d)
    bufs = [X.clone(), torch.empty_like(X)]
    acc = torch.zeros_like(X)
    w32 = float(np.float32(1.0 - alpha))
    for h in range(2):
        plan.hop(bufs[h % 2], bufs[(h + 1) % 2], alpha, acc, w32)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for h in range(reps):
        plan.hop(bufs[h % 2], bufs[(h + 1) % 2], alpha, acc, w32)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    nbytes = 4 * (n + 1) + 8 * gn.nnz + 16 * n * d
    gbs = nbytes / (ms * 1e-3) / 1e9
    del plan, bufs, acc
    return {"bound": "hbm", "kernel": "k_hop (+ k_fixup): one propagation hop", "achieved": gbs,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": ms}


def _cpu_hop_seconds(gn, X, alpha, threads):
    """The reference's hop on the host: torch CPU sparse COO @ dense (clustgdd_agent_transduct.py:63,
    `alpha * adj_norm @ prop`, adj_norm a coalesced fp32 COO tensor as sparse_mx_to_torch_sparse_tensor
    builds it) on `threads` threads; one hop timed (after one untimed hop when the hop is short)."""
    crow = gn.rowptr.to(torch.int64).cpu()
    rows = torch.repeat_interleave(torch.arange(gn.n, dtype=torch.int64), crow[1:] - crow[:-1])
    idx = torch.stack([rows, gn.col.to(torch.int64).cpu()])
    A = torch.sparse_coo_tensor(idx, gn.values().cpu(), (gn.n, gn.n)).coalesce()
    del rows, idx
    Xh = X.cpu()
    with _CpuThreads(threads):
        if gn.nnz * X.shape[1] < 2e9:
            y = alpha * (A @ Xh)
        t0 = time.perf_counter()
        y = alpha * (A @ Xh)
        s = time.perf_counter() - t0
    del A, Xh, y
    return s


def products_record(dev, with_cpu, group=None, world=1):
    """Config 5 at its full shape on one GPU (BASELINE configs[4]): ogbn-products'
    N = 2,449,029 nodes, mean degree 50.5 (~126M entries), d = 100, C = 47, T = 18, alpha = 0.91,
    KMeans(k = 196) (Lloyd: clustgdd_agent_transduct.py:104-105 for every dataset but arxiv) — the
    graph generated on the device (synth.chung_lu_device), N(0,1) features, random linear logits.
    Reports the synchronised phases of one warm pass, the hop's roofline, the k-means phases, and the
    fp32 vs bf16 MFMA labels pass (north_star: "fp32 vs bf16 MFMA distance kernel"); the CPU baseline
    is per unit (one torch CPU hop, one scikit-learn Lloyd iteration), not a whole run."""
    import gdd
    from gdd import kmeans as gk
    from gdd import synth
    from gdd.kmeans import _Ops
    cfg = synth.CONFIGS["products"]
    t0 = time.perf_counter()
    g = synth.chung_lu_device(cfg.n, cfg.avg_degree, cfg.seed, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(cfg.seed)
    X = torch.randn(cfg.n, cfg.d, device=dev, generator=gen)
    W = torch.randn(cfg.d, cfg.n_classes, device=dev, generator=gen) / float(np.sqrt(cfg.d))
    bias = torch.randn(cfg.n_classes, device=dev, generator=gen) * 0.1
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    if world > 1:
        return _products_group_record(cfg, g, X, W, bias, gen_s, dev, group, world)
    for _ in range(2):  # the first pass loads code objects and fills the caching allocator
        ph, kph = {}, {}
        torch.cuda.synchronize()
        tp = time.perf_counter()
        gn = gdd.normalize_adj(g)
        tp = _sync_mark(ph, "normalize", tp)
        target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha)
        tp = _sync_mark(ph, "propagate", tp)
        logits = torch.addmm(bias, target, W)
        tp = _sync_mark(ph, "logits", tp)
        gk.PHASE_TIMING = kph
        try:
            km = gdd.KMeans(n_clusters=cfg.k, random_state=cfg.seed, device=dev).fit(logits)
        finally:
            gk.PHASE_TIMING = None
        tp = _sync_mark(ph, "kmeans", tp)
        gdd.cluster_mean(target, km.labels_device_, cfg.k)
        gdd.argmax_rows(km.cluster_centers_device_)
        _sync_mark(ph, "cluster_mean", tp)
    n_iter = int(km.n_iter_)
    total_ms = sum(ph.values())
    hop = _hop_roofline(gn, X, cfg.alpha)
    hop["traffic"], hop["traffic_source"] = _products_pmc_traffic()
    # the labels pass at fp32 (exact, sklearn's bits) and bf16 (opt-in, config 5), same centres
    C = km.cluster_centers_device_.contiguous()
    ops = _Ops(dev, cfg.n, cfg.k, cfg.n_classes)
    # three alternating rounds, the best of each: the two passes draw different power, and the one
    # timed right after the other inherits its clock state (r06: ~10% either way)
    labs, times = {}, {}
    for _ in range(3):
        for prec in ("fp32", "bf16"):
            lab = torch.empty(cfg.n, dtype=torch.int32, device=dev)
            for _ in range(3):
                ops.assign(logits, C, labels=lab, precision=prec)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                ops.assign(logits, C, labels=lab, precision=prec)
            ev[1].record()
            torch.cuda.synchronize()
            times[prec] = min(times.get(prec, 1e9), ev[0].elapsed_time(ev[1]) / 10)
            labs[prec] = lab
    flops = 2.0 * cfg.n * cfg.k * cfg.n_classes
    agree = float((labs["fp32"] == labs["bf16"]).float().mean().item())
    peaks = {"fp32": FP32_MATRIX_PEAK_TFLOPS, "bf16": BF16_DENSE_PEAK_TFLOPS}
    assign = {p: {"avg_launch_ms": times[p], "achieved": flops / (times[p] * 1e-3) / 1e12,
                  "peak": peaks[p], "unit": "TFLOP/s",
                  "frac": flops / (times[p] * 1e-3) / 1e12 / peaks[p],
                  "x_read_gbs": 4.0 * cfg.n * cfg.n_classes / (times[p] * 1e-3) / 1e9,
                  "x_read_frac_of_hbm": 4.0 * cfg.n * cfg.n_classes / (times[p] * 1e-3) / 1e9 / HBM_PEAK_GBS}
              for p in ("fp32", "bf16")}
    rec = {"workload": f"ogbn-products shape (config 5): N={cfg.n}, nnz_norm={gn.nnz}, d={cfg.d}, "
                       f"C={cfg.n_classes}, {cfg.T - 1} hops (alpha {cfg.alpha}), KMeans(k={cfg.k}, "
                       f"random_state={cfg.seed}) Lloyd, cluster means",
           "data": "synthetic: Chung-Lu power-law graph sampled on the device, N(0,1) features, random "
                   "linear logits",
           "graph_generation_s": gen_s, "ms_total": total_ms, "phases_ms": ph,
           "kmeans_phases_ms": kph, "kmeans_n_iter": n_iter,
           "nodes_per_s": cfg.n / (total_ms * 1e-3),
           "hop_roofline": hop,
           "labels_pass": {"flops_per_launch": flops, "fp32": assign["fp32"], "bf16": assign["bf16"],
                           "bf16_speedup": times["fp32"] / times["bf16"],
                           "label_agreement": agree,
                           "note": "fp32 = k-ordered v_mfma_f32_32x32x2_f32 chains (sklearn's bits); "
                                   "bf16 = v_mfma_f32_32x32x16_bf16, every differing label within the "
                                   "bf16 rounding bound (tests/test_gpu_configs.py)"},
           "cpu_baseline": None}
    if with_cpu:
        threads, affinity, omp = _threads()
        hop_s = _cpu_hop_seconds(gn, X, cfg.alpha, threads)
        from sklearn.cluster import KMeans as SkKMeans
        L = logits.cpu().numpy()
        C0 = L[np.random.RandomState(cfg.seed).choice(cfg.n, cfg.k, replace=False)]
        it_s = {}
        with _CpuThreads(threads):
            for it in (1, 3):
                t0 = time.perf_counter()
                SkKMeans(n_clusters=cfg.k, init=C0, n_init=1, max_iter=it, tol=0.0,
                         algorithm="lloyd").fit(L)
                it_s[it] = time.perf_counter() - t0
        lloyd_s = (it_s[3] - it_s[1]) / 2
        rec["cpu_baseline"] = {
            "kind": "reference-library", "cores": threads, "affinity_cpus": affinity,
            "omp_num_threads": omp or None, "cpu_model": _cpu_model(),
            "hop_s": hop_s, "hop_gbs_algorithmic": hop["algorithmic_bytes_per_launch"] / hop_s / 1e9,
            "lloyd_iteration_s": lloyd_s,
            "modelled_step_s": (cfg.T - 1) * hop_s + n_iter * lloyd_s,
            "value": cfg.n / ((cfg.T - 1) * hop_s + n_iter * lloyd_s), "unit": "nodes/s (modelled)",
            "sample": (f"per unit on {threads} threads: one torch CPU sparse hop (COO @ dense, "
                       f"{cfg.n} x {cfg.d}); one scikit-learn Lloyd iteration = (fit(max_iter=3) - "
                       f"fit(max_iter=1)) / 2 on the same logits (k = {cfg.k}); modelled_step_s = "
                       f"{cfg.T - 1} hops + {n_iter} iterations (GPU's iteration count), "
                       "normalisation and k-means++ excluded")}
    del g, gn, X, target, logits, km, ops, labs
    torch.cuda.empty_cache()
    return rec


def _products_group_record(cfg, g, X, W, bias, gen_s, dev, group, world):
    """Config 5's pass distilling ONE graph over all ranks (every rank generates the same graph):
    propagation row-partitioned when gdd.sharded.propagation_shards_pay says so (one all-gather of
    each hop's output), KMeans as gdd.sharded.ShardedKMeans (its size model picks rows or
    replication), cluster means by cluster slices. Bit-identical to one GPU (tests/test_gpu_sharded.py)."""
    import gdd
    from gdd.pipeline import _lloyd
    from gdd.sharded import lloyd_rows_pay, propagation_shards_pay

    def one_pass(ph=None):
        tp = time.perf_counter()
        gn = gdd.normalize_adj(g)
        tp = _sync_mark(ph, "normalize", tp) if ph is not None else tp
        target, _ = gdd.propagate(gn, X, cfg.T, cfg.alpha, group=group)
        tp = _sync_mark(ph, "propagate", tp) if ph is not None else tp
        logits = torch.addmm(bias, target, W)
        km = _lloyd(cfg.k, group, random_state=cfg.seed, device=dev).fit(logits)
        tp = _sync_mark(ph, "logits_kmeans", tp) if ph is not None else tp
        gdd.cluster_mean(target, km.labels_device_, cfg.k, group=group)
        gdd.argmax_rows(km.cluster_centers_device_)
        if ph is not None:
            _sync_mark(ph, "cluster_mean", tp)
        return int(km.n_iter_), gn.nnz
    ms = _timed_ms(one_pass, 2, world, dev)
    ph = {}
    n_iter, nnz = one_pass(ph)
    return {"workload": f"ogbn-products shape (config 5): N={cfg.n}, nnz_norm={nnz}, d={cfg.d}, "
                        f"{cfg.T - 1} hops, KMeans(k={cfg.k}), cluster means — ONE graph over {world} ranks",
            "data": "synthetic: Chung-Lu power-law graph sampled on the device (same seed on every rank)",
            "parallelism": (f"{world} ranks (gdd.sharded): propagation "
                            f"{'row-partitioned, one all-gather per hop' if propagation_shards_pay(cfg.n, nnz, cfg.d, world) else 'replicated'}"
                            f"; Lloyd {'rows' if lloyd_rows_pay(cfg.n, cfg.n_classes, cfg.k, world) else 'replicated'}"
                            "; cluster means by cluster slices"),
            "graph_generation_s": gen_s, "ms_total": ms, "nodes_per_s": cfg.n / (ms * 1e-3),
            "phases_ms_rank0": ph, "kmeans_n_iter": n_iter, "cpu_baseline": None}


def _backend_name(group):
    """The collective library a group's broadcasts use: RCCL under the nccl backend, else gloo."""
    import torch.distributed as dist
    return "RCCL" if dist.get_backend(group) == "nccl" else dist.get_backend(group)


REDDIT_ROLES = (153932, 23699, 55334)  # GraphSAINT Reddit role.json sizes (train, val, test)
REDDIT_FULL_DEGREE = 101.7  # 232,965 nodes; the induced train graph then holds ~10.4M entries


def reddit_record(dev, with_cpu, group=None, world=1, reps=2):
    """Config 3's whole inductive hot path at full shape (BASELINE configs[2]; main_induct.sh:16-21:
    T = 20, alpha = 0.95; clustgdd_agent_induct.py:37-156): a 232,965-node graph (~23.7M entries)
    split with GraphSAINT's Reddit role sizes (153,932 train / 23,699 val / 55,334 test), d = 602 raw
    features; one pass = gdd.pipeline.graphsaint_split (train-fitted StandardScaler, three induced
    role graphs) + pretrained_clustering_induct_hot_path (three normalisations, 3 x 19 hops, 41
    logits from the train targets, MiniBatchKMeans(k = 769, b = 1000, random_state = 15), cluster
    means). At N > 1 the role graphs propagate on different ranks (gdd.sharded.role_owners: train on
    rank 0 — row-partitioned over ranks 0, 3.. where that pays — val on 1, test on 2) and the
    targets are broadcast; bit-identical to one GPU. Per-role phases of one more pass on rank 0; at
    N = 1 also the train hop's roofline, the fit split (k-means++ on the 3,000-point init subset, the
    final labels pass) and per-unit CPU baselines (one torch CPU hop per role graph, scikit-learn's
    MiniBatchKMeans.fit(max_iter=1))."""
    from gdd import synth
    from gdd.kmeans import _Ops
    from gdd.pipeline import graphsaint_split, pretrained_clustering_induct_hot_path
    from gdd.sharded import role_owners
    cfg = synth.CONFIGS["reddit"]
    n_tr, n_va, n_te = REDDIT_ROLES
    N = n_tr + n_va + n_te
    t0 = time.perf_counter()
    g_full = synth.chung_lu_device(N, REDDIT_FULL_DEGREE, cfg.seed, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(cfg.seed)
    perm = torch.randperm(N, device=dev, generator=gen)
    idx = {"train": torch.sort(perm[:n_tr]).values, "val": torch.sort(perm[n_tr:n_tr + n_va]).values,
           "test": torch.sort(perm[n_tr + n_va:]).values}
    feat = torch.randn(N, cfg.d, device=dev, generator=gen) * 3.0 + 1.0  # raw: the scaler centres it
    W = torch.randn(cfg.d, cfg.n_classes, device=dev, generator=gen) / float(np.sqrt(cfg.d))
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    last = {}

    def one_pass(ph=None):
        tp = time.perf_counter()
        data = graphsaint_split(g_full, feat, idx["train"], idx["val"], idx["test"], device=dev)
        if ph is not None:
            _sync_mark(ph, "graphsaint_split", tp)
        out = pretrained_clustering_induct_hot_path(
            data, cfg.T, cfg.alpha, lambda t_tr, t_va: t_tr @ W, cfg.k, dataset="reddit",
            seed=cfg.seed, cluster_minibatch=cfg.batch, device=dev, group=group, phases=ph)
        last.update(data=data, out=out)
    ms = _timed_ms(one_pass, reps, world, dev)
    ph = {}
    one_pass(ph)
    data, out = last["data"], last["out"]
    gn_tr, t_tr = out[4], out[3]
    nnz = {r: int(getattr(data, "adj_" + r).nnz) for r in ("train", "val", "test")}
    rec = {"workload": (f"Reddit inductive hot path (config 3): graphsaint_split of a {N}-node graph "
                        f"(roles {n_tr}/{n_va}/{n_te}, role-graph entries {nnz}), d={cfg.d}, 3 x "
                        f"{cfg.T - 1} hops (alpha {cfg.alpha}), logits C={cfg.n_classes}, "
                        f"MiniBatchKMeans(k={cfg.k}, b={cfg.batch}, random_state={cfg.seed}), cluster means"),
           "data": "synthetic: Chung-Lu power-law graph sampled on the device, random role split of "
                   "GraphSAINT's Reddit sizes, N(1, 9) raw features, random linear logits",
           "parallelism": ("single GPU" if world == 1 else
                           f"{world} ranks: each role graph propagated by its owners "
                           f"{role_owners(world)} (train row-partitioned over its owners when "
                           f"propagation_shards_pay), targets broadcast over {_backend_name(group)}; MiniBatchKMeans "
                           "steps replicated, labels pass by rows, cluster means by clusters"),
           "graph_generation_s": gen_s, "ms_total": ms, "nodes_per_s": N / (ms * 1e-3),
           "phases_ms" if world == 1 else "phases_ms_rank0": ph,
           "minibatch_steps": None, "cpu_baseline": None}
    if world > 1:
        del last, data, out
        return rec
    n_steps = None
    logits = t_tr @ W
    from gdd import MiniBatchKMeans
    km = MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch, device=dev).fit(logits)
    n_steps = int(km.n_steps_)
    rec["minibatch_steps"] = n_steps
    rec["hop_roofline"] = _hop_roofline(gn_tr, data.feat_train, cfg.alpha)
    # the fit's first and last stages as separate calls: k-means++ on a 3,000-point subset (k = 769,
    # T = 8) and the full labels pass against the fitted centres
    ops = _Ops(dev, n_tr, cfg.k, cfg.n_classes)
    Xi = logits[torch.randperm(n_tr, device=dev, generator=gen)[:3 * cfg.batch]].contiguous()
    ops_i = _Ops(dev, Xi.shape[0], cfg.k, cfg.n_classes)
    ops_i.kmeans_plusplus(Xi, cfg.k, np.random.RandomState(0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops_i.kmeans_plusplus(Xi, cfg.k, np.random.RandomState(1))
    torch.cuda.synchronize()
    kpp_ms = (time.perf_counter() - t0) * 1e3
    lab = torch.empty(n_tr, dtype=torch.int32, device=dev)
    C = km.cluster_centers_device_.contiguous()
    ops.assign(logits, C, labels=lab)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops.assign(logits, C, labels=lab)
    torch.cuda.synchronize()
    labels_ms = (time.perf_counter() - t0) * 1e3
    steps_ms = ph["kmeans"] - kpp_ms - labels_ms
    rec["minibatch_split_ms"] = {"kmeans_plusplus_init_subset": kpp_ms, "labels_pass": labels_ms,
                                 "steps_and_reassignment": steps_ms,
                                 "per_step_us": 1e3 * steps_ms / max(n_steps, 1)}
    if with_cpu:
        threads, affinity, omp = _threads()
        hop_s = {"train": _cpu_hop_seconds(gn_tr, data.feat_train, cfg.alpha, threads)}
        from gdd.graph import normalize_adj
        for r in ("val", "test"):
            hop_s[r] = _cpu_hop_seconds(normalize_adj(getattr(data, "adj_" + r)),
                                        getattr(data, "feat_" + r), cfg.alpha, threads)
        from sklearn.cluster import MiniBatchKMeans as SkMB
        L = logits.cpu().numpy()
        with _CpuThreads(threads):
            t0 = time.perf_counter()
            skm = SkMB(n_clusters=cfg.k, batch_size=cfg.batch, random_state=cfg.seed, max_iter=1).fit(L)
            mb_s = time.perf_counter() - t0
        model_s = (cfg.T - 1) * sum(hop_s.values()) + mb_s * n_steps / max(int(skm.n_steps_), 1)
        rec["cpu_baseline"] = {
            "kind": "reference-library", "cores": threads, "affinity_cpus": affinity,
            "omp_num_threads": omp or None, "cpu_model": _cpu_model(),
            "hop_s": hop_s, "minibatch_fit_max_iter1_s": mb_s, "minibatch_fit_steps": int(skm.n_steps_),
            "modelled_step_s": model_s, "value": N / model_s, "unit": "nodes/s (modelled)",
            "sample": (f"per unit on {threads} threads: one torch CPU sparse hop per role graph; "
                       f"scikit-learn MiniBatchKMeans(k={cfg.k}, b={cfg.batch}).fit(max_iter=1) "
                       f"({int(skm.n_steps_)} steps incl. its k-means++ init) on the same logits; "
                       f"modelled_step_s = {cfg.T - 1} hops of each role graph + the fit scaled to "
                       f"the GPU's {n_steps} steps (graphsaint_split and normalisation excluded)")}
    del g_full, feat, last, data, out, logits, km, ops, ops_i
    torch.cuda.empty_cache()
    return rec


def e2e_record(dev):
    """§8(d)'s end-to-end half, measured in this run: the drop-in agent
    (gdd.train_clustgdd_transduct -> gdd.agent.ClustGDD.train, clustgdd_agent_transduct.py:395-429)
    with main_transduct.sh:73-79's ogbn-arxiv r = 0.5% flags, on gdd.data.synthetic('ogbn-arxiv')
    (OGB's split sizes: 90,941 train nodes -> k = 454; class-conditioned features + homophilous
    graph, because OGB cannot be downloaded). Reports the reference's own printed stage times
    (pretraining = pretrained_clustering, refinement = sparsify + compress + refusion, Total = t2-t1),
    max memory and the five [train, test] test_with_val accuracies. The accuracy measures the
    synthetic data, not real arxiv."""
    import contextlib
    import io
    from gdd import train_clustgdd_transduct as drv
    argv = ["--gpu_id", str(dev.index or 0), "--dataset", "ogbn-arxiv", "--reduction_rate", "0.005",
            "--prop_num", "18", "--postprop_num", "10", "--alpha", "0.91", "--predropout", "0.6",
            "--sp_ratio", "0.1", "--preep", "1000", "--postep", "1000", "--frcoe", "1.9",
            "--predcoe", "0.025", "--save", "1"]
    out = io.StringIO()
    torch.cuda.reset_peak_memory_stats(dev)  # the agent's own peak (the records before it used more)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(out):
        agent = drv.main(argv)
    wall = time.perf_counter() - t0
    res = agent.results
    tail = [ln for ln in out.getvalue().splitlines() if ln.strip()][-5:]
    rec = {"command": "python -m gdd.train_clustgdd_transduct " + " ".join(argv),
           "reference_flags": "ClustGDD/main_transduct.sh:73-79 (ogbn-arxiv, r = 0.5%)",
           "data": "gdd.data.synthetic('ogbn-arxiv'): OGB's split sizes, learnable synthetic "
                   "features/graph (not comparable with published arxiv accuracies)",
           "nnodes_syn": int(agent.nnodes_syn), **agent.times,
           "train_test_mean": None if res is None else res.mean(0).tolist(),
           "train_test_std": None if res is None else res.std(0).tolist(),
           "runs": None if res is None else res.tolist(),
           "wall_s_including_5_evaluations": wall, "stdout_tail": tail}
    del agent
    torch.cuda.empty_cache()
    return rec


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, A, X_h):
    """The reference's own CPU path, whole step, no extrapolation: the library calls
    ClustGDD.pretrained_clustering makes, on the same synthetic inputs, with every host core the
    process may use —
      * normalize_adj_tensor(sparse=True) (deep_robust_utils.py:180-207, 245-256): scipy, A + I only
        if A[0,0] == 0, D^-1/2 (A+I) D^-1/2 in fp64, cast to an fp32 torch sparse COO tensor;
      * the propagation loop (clustgdd_agent_transduct.py:59-65): torch CPU sparse `@`, T-1 hops;
      * the logits (the MLP stand-in: one fp32 GEMM, as on the GPU);
      * MiniBatchKMeans(n_clusters=k, random_state=seed, batch_size=1000).fit (transduct:102-103),
        scikit-learn with its OpenMP/BLAS threads;
      * the cluster-mean loop (transduct:116-127): target[torch.where(labels == i)[0]].mean(0) per i.
    """
    import scipy.sparse as sp
    from sklearn.cluster import MiniBatchKMeans
    # the cores this process may run on (affinity mask; os.cpu_count() ignores it) and the OpenMP
    # share the box sets: the baseline runs min of the two threads (= all the lease's cores)
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)
    threads = min(affinity, omp) if omp else affinity
    torch.set_num_threads(threads)
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=threads)
    except ImportError:  # pragma: no cover
        limiter = None
    A = sp.coo_matrix(A, dtype=np.float32)
    n = A.shape[0]
    # the agent's adjacency arrives as a torch sparse COO tensor (to_tensor, deep_robust_utils.py:85-113)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((A.row, A.col)).astype(np.int64)),
                                  torch.from_numpy(A.data), (n, n))
    t0 = time.perf_counter()
    # normalize_adj_tensor(adj, sparse=True): to_scipy (CSR from the COO values/indices), then
    # normalize_adj on a LIL matrix (A + I only if A[0,0] == 0; fp64 row sums; inf -> 0; two diagonal
    # scalings), then back to an fp32 torch COO tensor (sparse_mx_to_torch_sparse_tensor)
    vals, ind = adj._values().numpy(), adj._indices().numpy()
    M = sp.csr_matrix((vals, ind), shape=(n, n)).tolil()
    if M[0, 0] == 0:
        M = M + sp.eye(n)
    deg = np.array(M.sum(1))
    with np.errstate(divide="ignore"):
        r = np.power(deg, -0.5).flatten()
    r[np.isinf(r)] = 0.0
    D = sp.diags(r)
    M = D.dot(M).dot(D).tocoo().astype(np.float32)
    idx = torch.cat((torch.LongTensor(M.row).unsqueeze(1), torch.LongTensor(M.col).unsqueeze(1)), 1)
    adj_norm = torch.sparse_coo_tensor(idx.t(), torch.FloatTensor(M.data), (n, n))
    t1 = time.perf_counter()
    feats = torch.from_numpy(X_h)
    prop = feats
    target = (1 - cfg.alpha) * prop
    for _ in range(1, cfg.T):
        prop = cfg.alpha * adj_norm @ prop
        target = target + (1 - cfg.alpha) * prop
    t2 = time.perf_counter()
    rng = np.random.default_rng(cfg.seed + 3)
    W = torch.from_numpy((rng.standard_normal((cfg.d, cfg.n_classes)) / np.sqrt(cfg.d)).astype(np.float32))
    b = torch.from_numpy((rng.standard_normal(cfg.n_classes) * 0.1).astype(np.float32))
    logits = torch.addmm(b, target, W).numpy()
    t3 = time.perf_counter()
    km = MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch).fit(logits)
    t4 = time.perf_counter()
    lab = torch.from_numpy(km.labels_.astype(np.int64))
    feat_syn = torch.stack([target[torch.where(lab == i)[0]].mean(dim=0) for i in range(cfg.k)])
    labels_syn = torch.argmax(torch.from_numpy(km.cluster_centers_), dim=-1)
    t5 = time.perf_counter()
    del feat_syn, labels_syn
    if limiter is not None:
        limiter.unregister() if hasattr(limiter, "unregister") else None
    total = t5 - t0
    return {"value": n / total, "unit": "nodes/s", "cores": threads, "kind": "reference-library",
            "affinity_cpus": affinity, "omp_num_threads": omp or None, "cpu_model": _cpu_model(),
            "threads_policy": ("min(affinity mask, OMP_NUM_THREADS): the GPU box's lease sets "
                               "OMP_NUM_THREADS to its CPU share (16 on a one-GPU box) although the "
                               "affinity mask shows the whole machine; the baseline runs that share"),
            "sample": (f"one whole step of the reference's CPU path on the bench's graph ({n} nodes): "
                       f"scipy normalize_adj, {cfg.T - 1} torch CPU sparse hops, logits GEMM, sklearn "
                       f"MiniBatchKMeans(k={cfg.k}, b={cfg.batch}, seed {cfg.seed}, {km.n_steps_} steps), "
                       f"torch where/mean loop; {threads} threads; {total:.1f} s measured"),
            "seconds_per_step": total,
            "stages_s": {"normalize": t1 - t0, "propagate": t2 - t1, "logits": t3 - t2,
                         "minibatch_kmeans": t4 - t3, "cluster_mean": t5 - t4}}


if __name__ == "__main__":
    main()
