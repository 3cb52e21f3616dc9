#!/usr/bin/env python3
"""Joins tools/relabel_products.py's timings (its JSON lines) with a rocprofv3 --pmc FETCH_SIZE pass
of the same script (RELABEL_REPS=1): per configuration, the mean FETCH_SIZE (KiB, summed over the
XCDs by rocprofv3) of the hop kernel's dispatches between that configuration's marker fill (a fill of
marker * 1,000,000 floats) and the next one (doubled: the gfx950 correction for 16-byte reads),
against the hop's algorithmic bytes as DESIGN §4 counts them
(4 (N + 1) + 8 nnz + 16 N d: the CSR once, the previous hop read once, this hop written, target read
and written).

usage: relabel_products_pmc.py TIMINGS.log COUNTERS.csv OUT.json"""
import csv
import json
import sys


def main(tlog, ccsv, out):
    recs = [json.loads(line) for line in open(tlog) if line.startswith("{") and '"summary"' not in line]
    rows = sorted(csv.DictReader(open(ccsv)), key=lambda r: int(r["Dispatch_Id"]))
    # marker fills: elementwise fill kernels whose grid covers marker * 1e6 floats
    seg, cur = {}, None
    for r in rows:
        name = r["Kernel_Name"]
        if "fill" in name.lower() or "FillFunctor" in name:
            g = int(r["Grid_Size"])
            for rec in recs:  # a float4-vectorised fill: one thread per 4 floats
                if abs(g * 4 - rec["marker"] * 1000000) <= 4096:
                    cur = rec["marker"]
                    break
            continue
        if cur is not None and "k_hop" in name:
            seg.setdefault(cur, []).append(float(r["Counter_Value"]))
    for rec in recs:
        v = seg.get(rec["marker"], [])
        n, nnz, d = rec["n"], rec["nnz"], rec["d"]
        rec["hop_dispatches"] = len(v)
        # FETCH_SIZE in KiB, doubled: gfx950 reports half the bytes of 16-byte-per-lane reads (the hop's
        # row gathers; MI355X_MICROARCH.md HBM section, as tools/pmc_summary.py)
        rec["fetch_bytes_per_hop"] = (2.0 * sum(v) / len(v) * 1024.0) if v else None
        rec["ideal_bytes_per_hop"] = 4 * (n + 1) + 8 * nnz + 16 * n * d  # DESIGN §4's algorithmic bytes
        if v:
            rec["fetch_over_ideal"] = rec["fetch_bytes_per_hop"] / rec["ideal_bytes_per_hop"]
    json.dump({"what": "products-shape propagation (T = 18, d = 100) in other node orders: hop time "
                       "(device events) and HBM fetch per hop (rocprofv3 --pmc FETCH_SIZE, separate "
                       "pass) — tools/relabel_products.py, tools/relabel_products_pmc.py",
               "records": recs}, open(out, "w"), indent=1)
    for rec in recs:
        print(rec["graph"][:42], rec["order"], rec.get("schedule"), round(rec["us_per_hop"], 1),
              rec.get("fetch_over_ideal"), rec["hop_dispatches"])


if __name__ == "__main__":
    main(*sys.argv[1:4])
