#!/usr/bin/env python3
"""HBM-side traffic of the SpMM hop kernel from separate rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE, and optionally TCC_HIT_sum + TCC_MISS_sum for the L2 hit rate).

Applies the gfx950 corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the
bytes of 16-byte-per-lane reads (doubled here); WRITE_SIZE is exact for 16-byte stores. Both are
KiB per dispatch. Writes profiles/<tag>_khop_traffic.json, which bench.py reports as
roofline.traffic (bytes per launch).

usage: python tools/pmc_summary.py <run_dir> <out.json> [csv_prefix] [label] [algorithmic_bytes]
  run_dir holds pmc_fetch/, pmc_write/ and (optional) pmc_hit/, each with <prefix>_counter_collection.csv
"""
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and "k_hop" in r["Kernel_Name"]]


def main(run_dir, out_path, prefix="bench", label="k_hop (one propagation hop, ogbn-arxiv shape, d=128)",
         algorithmic=None):
    f = lambda sub: os.path.join(run_dir, sub, f"{prefix}_counter_collection.csv")  # noqa: E731
    fetch = per_dispatch(f("pmc_fetch"), "FETCH_SIZE")
    write = per_dispatch(f("pmc_write"), "WRITE_SIZE")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    read_bytes = 2.0 * f_kib * 1024.0
    write_bytes = w_kib * 1024.0
    out = {
        "kernel": label,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB_per_launch": f_kib,
        "WRITE_SIZE_KiB_per_launch": w_kib,
        "read_bytes_per_launch": read_bytes,
        "write_bytes_per_launch": write_bytes,
        "traffic_bytes_per_launch": read_bytes + write_bytes,
        "correction": "read = 2 x FETCH_SIZE (gfx950 reports half of 16-B/lane reads); write = WRITE_SIZE",
        "source": run_dir,
    }
    if algorithmic:
        out["algorithmic_bytes_per_launch"] = int(algorithmic)
        out["traffic_over_algorithmic"] = (read_bytes + write_bytes) / float(algorithmic)
    if os.path.exists(f("pmc_hit")):
        hit = per_dispatch(f("pmc_hit"), "TCC_HIT_sum")
        miss = per_dispatch(f("pmc_hit"), "TCC_MISS_sum")
        if hit and miss:
            h, m = sum(hit) / len(hit), sum(miss) / len(miss)
            out["TCC_HIT_per_launch"], out["TCC_MISS_per_launch"] = h, m
            out["l2_hit_rate"] = h / (h + m)
    with open(out_path, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:6])
