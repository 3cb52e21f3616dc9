#!/usr/bin/env python3
"""The bf16 full labels pass (config 5: 2,449,029 x 47 logits against k = 196 centres; also the arxiv
and Reddit shapes) — the r06 kernel (gdd_bf16.hip k_assign_bf16q, the default) and its A/B forms
against the r03 one (GDD_FORCE=bf16_v1), same process, alternating: device ms per pass (HIP events on
the launching stream), X's read rate against 8 TB/s, and whether each variant's labels equal the r03
kernel's. BF16_VARIANTS="name=tokens;..." (must hold v1), MICRO_SHAPES="products,reddit". Prints one
JSON line per shape and one for all."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-distillation-for-recommendation_amd"))
import torch  # noqa: E402

from gdd.kmeans import _Ops  # noqa: E402

SHAPES = {"products": (2449029, 47, 196), "arxiv": (169343, 40, 454), "reddit": (153932, 41, 769)}
SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ.get("MICRO_SHAPES", ",".join(SHAPES)).split(",")}
# variant -> GDD_FORCE tokens (A/B of the r06 kernel's forms; "" = the library default)
VARIANTS = dict(v.split("=", 1) for v in os.environ.get(
    "BF16_VARIANTS", "v1=bf16_v1;q=").split(";"))


def timed(fn, reps=20):
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
    res = {}
    for name, (n, dim, k) in SHAPES.items():
        g = torch.Generator(device="cuda").manual_seed(n)
        X = (torch.randn(n, 100, device="cuda", generator=g) @
             (torch.randn(100, dim, device="cuda", generator=g) / 10.0)).contiguous()
        C = X[torch.randperm(n, device="cuda", generator=g)[:k]].contiguous()
        ops = _Ops("cuda", n, k, dim)
        labs, times = {}, {v: [] for v in VARIANTS}
        for rnd in range(3):
            for v, tok in VARIANTS.items():
                if tok:
                    os.environ["GDD_FORCE"] = tok
                else:
                    os.environ.pop("GDD_FORCE", None)
                lab = torch.empty(n, dtype=torch.int32, device="cuda")
                times[v].append(timed(lambda: ops.assign(X, C, labels=lab, precision="bf16")))
                labs[v] = lab
        os.environ.pop("GDD_FORCE", None)
        l32 = torch.empty(n, dtype=torch.int32, device="cuda")
        ops.assign(X, C, labels=l32)
        xs = X.view(-1)
        floor_ms = min(timed(lambda: xs.sum()) for _ in range(3))  # torch's own read of X: the HBM floor
        ms = {v: min(t) for v, t in times.items()}
        res[name] = {"n": n, "dim": dim, "k": k, "ms": ms, "all_ms": times, "torch_sum_ms": floor_ms,
                     "x_read_frac_of_8TBs": {v: 4.0 * n * dim / (m * 1e-3) / 8e12 for v, m in ms.items()},
                     "labels_identical": {v: bool(torch.equal(labs[v], labs["v1"])) for v in labs},
                     "agreement_with_fp32": float((labs["v1"] == l32).float().mean())}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
