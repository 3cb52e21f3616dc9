#!/usr/bin/env python3
"""Where a bench step's wall time goes, from a rocprofv3 kernel trace of bench.py: steps start at
each normalisation (k_probe or k_fast_count); per step the span, the busy time of the main stream's
kernels, and the largest idle gaps with the kernels on either side.

usage: python tools/step_gaps.py <kernel_trace.csv> [steps to show]
"""
import csv
import re
import sys
from collections import Counter


def short(name):
    m = re.search(r"::(k_\w+|__amd_\w+)", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def main(path, show=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if re.search(r"k_probe|k_fast_count", r["Kernel_Name"])]
    # a step's normalisation launches one of these; keep the first of each adjacent pair
    starts = [s for j, s in enumerate(starts) if j == 0 or s - starts[j - 1] > 10]
    for a, b in list(zip(starts, starts[1:] + [len(rows)]))[-show - 1:-1]:
        seg = rows[a:b]
        t0 = int(seg[0]["Start_Timestamp"])
        prev_end, prev = None, ""
        busy, gaps, gap_total = 0, Counter(), 0
        for r in seg:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            busy += en - st
            if prev_end is not None and st > prev_end:
                g = st - prev_end
                gap_total += g
                if g > 3000:
                    gaps[(short(prev), short(r["Kernel_Name"]))] += g
            prev_end = en if prev_end is None else max(prev_end, en)
            prev = r["Kernel_Name"]
        print(f"step: span {(prev_end - t0) / 1e3:.1f} us, kernels {len(seg)}, busy {busy / 1e3:.1f} us, "
              f"idle {gap_total / 1e3:.1f} us")
        for (x, y), g in gaps.most_common(12):
            print(f"  {g / 1e3:8.1f} us idle  after {x}  before {y}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
