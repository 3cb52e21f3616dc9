#!/usr/bin/env python3
"""Ordered per-cluster fold (Lloyd M-step sums, cluster means) at the ogbn-products k-means shape:
event-timed launches for random vs sorted cluster layouts (random row gathers vs contiguous rows),
and for the arxiv cluster-mean shape."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import _lib  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    lib = _lib.device_lib()
    st = _lib.stream_ptr()
    for (n, dim, k) in [(2449029, 47, 196), (2449029, 48, 196), (169343, 128, 454), (200000, 47, 196)]:
        X = torch.randn(n, dim, device="cuda")
        for layout in ("random", "sorted"):
            lab = np.random.default_rng(1).integers(0, k, n).astype(np.int32)
            if layout == "sorted":
                lab = np.sort(lab)
            ld = torch.from_numpy(lab).cuda()
            perm, offs = gdd.group_by_label(ld, k)
            sums = torch.empty(k, dim, device="cuda")
            w = torch.empty(k, device="cuda")
            t_sum = timeit(lambda: _lib.check(lib.gdd_segment_sum_f32(n, dim, X.data_ptr(), None, perm.data_ptr(),
                                                                     offs.data_ptr(), k, sums.data_ptr(),
                                                                     w.data_ptr(), st)))
            t_grp = timeit(lambda: gdd.group_by_label(ld, k))
            t_mean = timeit(lambda: gdd.cluster_mean(X, ld, k))
            gb = n * dim * 4 / 1e9
            print(f"n={n} dim={dim} k={k} {layout:6s}: fold_f32 {t_sum:.3f} ms ({gb / t_sum:.2f} TB/s) "
                  f"group {t_grp:.3f} ms  cluster_mean(total) {t_mean:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
