#!/usr/bin/env python3
"""The reference's own CPU path for config 4 (ClustGDD/distill_recsys.py main, device='cpu'), timed on
the same synthetic ML-1M-shaped dataset as tools/bench_recsys_e2e.py, for a bounded number of
refinement epochs (the per-epoch cost is flat: sampler loop + CPU LightGCN step). Needs
/root/reference (build container only: the GPU box has no reference), so its numbers are this
container's CPU. Prints one JSON line: per-stage seconds, the per-epoch refinement cost, threads.

usage: ref_recsys_cpu.py [epochs]"""
import contextlib
import io
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from bench_recsys_e2e import write_dataset  # noqa: E402
from make_golden import import_reference  # noqa: E402


def main(epochs=20):
    _, _, ref = import_reference()
    stamps = {}

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            stamps[name] = stamps.get(name, 0.0) + time.perf_counter() - t
            return r
        return w
    for name in ("compute_svd_embeddings", "kmeans_cluster", "build_condensed_bipartite",
                 "sample_bpr_triplets_from_condensed", "recall_at_k", "manual_adam_step"):
        setattr(ref, name, timed(name, getattr(ref, name)))
    with tempfile.TemporaryDirectory() as tmp:
        n = write_dataset(tmp)
        old, cwd = sys.argv, os.getcwd()
        sys.argv = ["distill_recsys.py", "--data_dir", tmp, "--dataset", "ml1m", "--device", "cpu",
                    "--refine_epochs", str(epochs), "--log_every", str(10 ** 6)]
        os.chdir(tmp)
        buf = io.StringIO()
        t0 = time.perf_counter()
        try:
            with contextlib.redirect_stdout(buf):
                ref.main()
        finally:
            sys.argv = old
            os.chdir(cwd)
        total = time.perf_counter() - t0
    refine = total - sum(stamps.get(k, 0.0) for k in ("compute_svd_embeddings", "kmeans_cluster",
                                                       "build_condensed_bipartite"))
    # refine includes the data load and the two evaluations (before training and at the last epoch)
    evals = stamps.get("recall_at_k", 0.0)
    print(json.dumps({"workload": f"reference distill_recsys main (CPU), ML-1M shape, {n} interactions, "
                                  f"{epochs} BPR epochs b=4096", "torch_threads": torch.get_num_threads(),
                      "cpu_count": os.cpu_count(), "stages_s": stamps, "total_s": total,
                      "refine_ms_per_epoch": (refine - evals) / epochs * 1e3,
                      "recall_eval_s_each": evals / 2}), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:2]))
