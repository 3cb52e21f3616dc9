#!/usr/bin/env python3
"""MFMA evidence for the k-means assignment ("MFMA utilisation for the
distance GEMM") from one rocprofv3 --pmc pass over tools/bench_assign.py (shapes arxiv, reddit,
products in that order; per shape and precision 11 launches: 1 warm-up + 10 timed).

Counters: SQ_INSTS_VALU_MFMA_MOPS_{F32,BF16} (MFMA math ops / 512), SQ_VALU_MFMA_BUSY_CYCLES (summed
over SIMDs), GRBM_GUI_ACTIVE (summed over the 8 XCDs). Per dispatch: counter FLOPs = MOPS x 512,
MFMA utilisation = BUSY / (GUI_ACTIVE / 8 x 1024 SIMDs), achieved TFLOP/s = algorithmic 2 n k dim /
the dispatch's duration (its timestamps).

usage: python tools/pmc_mfma_summary.py <counter_collection.csv> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict

SHAPES = [("arxiv", 169343, 40, 454), ("reddit", 153932, 41, 769), ("products", 2449029, 47, 196)]
PEAK = {"fp32": 157.3, "bf16": 2500.0}  # MI355X dense TF/s (MI355X_MICROARCH.md, matrix cores)


def main(path, out):
    disp = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = disp[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    res = {}
    for kind, key in (("fp32", "k_assign_persist"), ("bf16", "k_assign_bf16p")):
        ds = [disp[i] for i in sorted(disp) if key in disp[i]["name"]]
        per = len(ds) // len(SHAPES)
        for si, (name, n, dim, k) in enumerate(SHAPES):
            part = ds[si * per:(si + 1) * per][1:]  # drop the warm-up launch
            ns = sum(d["ns"] for d in part) / len(part)
            mops = sum(d["SQ_INSTS_VALU_MFMA_MOPS_F32"] + d["SQ_INSTS_VALU_MFMA_MOPS_BF16"] for d in part) / len(part)
            busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in part) / len(part)
            gui = sum(d["GRBM_GUI_ACTIVE"] for d in part) / len(part)
            alg = 2.0 * n * k * dim
            res.setdefault(name, {})[kind] = {
                "kernel": key, "avg_us": ns / 1e3, "algorithmic_gflop": alg / 1e9,
                "counter_gflop": mops * 512 / 1e9, "achieved_tflops": alg / ns / 1e3,
                "peak_tflops": PEAK[kind], "frac_of_peak": alg / ns / 1e3 / PEAK[kind],
                "mfma_busy_util": busy / (gui / 8 * 1024)}
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 "
                             "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 "
                             "tools/bench_assign.py", "shapes": res}, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
