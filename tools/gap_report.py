#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of the last MiniBatchKMeans fit in a rocprofv3 kernel trace."""
import csv
import sys
from collections import Counter


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    firsts = [i for i, r in enumerate(rows) if "k_kpp_init" in r["Kernel_Name"]]
    seg = rows[firsts[-1]:]
    t0, prev_end, prev_name = int(seg[0]["Start_Timestamp"]), None, ""
    busy, gaps = 0, Counter()
    gap_total = 0
    for r in seg:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += en - st
        if prev_end is not None and st > prev_end:
            g = st - prev_end
            gap_total += g
            if g > 5000:
                gaps[(prev_name[:50], r["Kernel_Name"][:50])] += g
        prev_end = en if prev_end is None else max(prev_end, en)
        prev_name = r["Kernel_Name"]
    print(f"last fit: span {(prev_end - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, gaps {gap_total / 1e3:.1f} us")
    for (a, b), g in gaps.most_common(12):
        print(f"  {g / 1e3:8.1f} us  after {a}  before {b}")


if __name__ == "__main__":
    main(sys.argv[1])
