#!/usr/bin/env python3
"""HBM-side traffic of the SpMM hop kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Applies the gfx950 corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the
bytes of 16-byte-per-lane reads (doubled here); WRITE_SIZE is exact for 16-byte stores. Both are
KiB per dispatch. Writes profiles/<tag>_khop_traffic.json, which bench.py reports as
roofline.traffic (bytes per launch).

usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<tag>_khop_traffic.json
"""
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and "k_hop" in r["Kernel_Name"]]
    return vals


def main(run_dir, out_path):
    fetch = per_dispatch(os.path.join(run_dir, "pmc_fetch", "bench_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(run_dir, "pmc_write", "bench_counter_collection.csv"), "WRITE_SIZE")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    read_bytes = 2.0 * f_kib * 1024.0
    write_bytes = w_kib * 1024.0
    out = {
        "kernel": "k_hop (one propagation hop, ogbn-arxiv shape, d=128)",
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB_per_launch": f_kib,
        "WRITE_SIZE_KiB_per_launch": w_kib,
        "read_bytes_per_launch": read_bytes,
        "write_bytes_per_launch": write_bytes,
        "traffic_bytes_per_launch": read_bytes + write_bytes,
        "correction": "read = 2 x FETCH_SIZE (gfx950 reports half of 16-B/lane reads); write = WRITE_SIZE",
        "source": run_dir,
    }
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:3])
