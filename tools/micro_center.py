#!/usr/bin/env python3
"""KMeans.fit's centring (gdd_center_columns: X - mean and the column variances in numpy's order) at
the products k-means shape (2,449,029 x 47) and the ML-1M shape, device events."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gdd import _lib  # noqa: E402


def main(reps=3):
    lib = _lib.device_lib()
    for n, d in ((2449029, 47), (6040, 64), (169343, 40)):
        X = torch.randn(n, d, device="cuda") * 3 + 1
        Y = torch.empty_like(X)
        m = torch.empty(d, device="cuda")
        v = torch.empty(d, device="cuda")
        call = lambda: _lib.check(lib.gdd_center_columns(n, d, X.data_ptr(), Y.data_ptr(), m.data_ptr(),  # noqa
                                                         v.data_ptr(), _lib.stream_ptr()))
        call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        ref = X.cpu().numpy().mean(axis=0)
        ok = np.array_equal(ref, m.cpu().numpy())
        print(f"center_columns n={n} d={d}: {ms:.3f} ms ({ms * 1e6 / n / 2:.2f} ns per row per pass), "
              f"mean {'== numpy' if ok else 'DIFFERS from numpy'}", flush=True)


if __name__ == "__main__":
    main()
