#!/usr/bin/env python3
"""StandardScaler statistics (gdd_standard_scaler) at the Reddit train shape (153,932 x 602) and the
ML-1M users shape (6,040 x 64): the column groups on one XCD against spread over all
(GDD_FORCE=scaler_one_xcd / scaler_spread), same process, device events. One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import torch  # noqa: E402

from gdd import pipeline  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
for n, d, reps in ((153932, 602, 3), (6040, 64, 20), (2449029, 47, 2)):
    X = torch.randn(n, d, device="cuda")
    r = {}
    outs = {}
    for name, tok in (("one_xcd", "scaler_one_xcd"), ("spread", "scaler_spread")):
        os.environ["GDD_FORCE"] = tok
        r[name] = min(timed(lambda: pipeline.standard_scaler(X), reps) for _ in range(2))
        outs[name] = pipeline.standard_scaler(X)
    os.environ.pop("GDD_FORCE", None)
    r["identical"] = all(torch.equal(a, b) for a, b in zip(outs["one_xcd"], outs["spread"]))
    res[f"{n}x{d}"] = r
    print(f"{n}x{d}", json.dumps(r), flush=True)
print(json.dumps(res))
