#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-fit span, busy time per kernel, idle gaps.

usage: python tools/timeline.py <kernel_trace.csv> [first-kernel-regex]
A 'segment' starts at every dispatch matching the regex (default: k_gather_rows, the first kernel
of a MiniBatchKMeans fit) and runs to the next one.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"::(k_\w+|__amd_\w+)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][-40:]


def main(path, start_re="k_gather_rows"):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    segs, cur = [], []
    for e in ev:
        if re.search(start_re, e[2]) and cur:
            segs.append(cur)
            cur = []
        cur.append(e)
    if cur:
        segs.append(cur)
    for si, seg in enumerate(segs):
        span = (seg[-1][1] - seg[0][0]) / 1e3
        busy = defaultdict(float)
        count = defaultdict(int)
        gaps = []
        for a, b in zip(seg, seg[1:]):
            gaps.append((b[0] - a[1]) / 1e3)
        for s, e, n in seg:
            busy[n] += (e - s) / 1e3
            count[n] += 1
        tot = sum(busy.values())
        big = sorted(gaps, reverse=True)[:5]
        small = sum(g for g in gaps if g < 20)
        print(f"segment {si}: span {span:.1f} us, kernels {tot:.1f} us, gaps<20us {small:.1f} us, "
              f"gaps>=20us {sum(g for g in gaps if g >= 20):.1f} us (largest {', '.join(f'{g:.0f}' for g in big)})")
        for n, t in sorted(busy.items(), key=lambda x: -x[1])[:12]:
            print(f"    {n:28s} {count[n]:5d} x {t / count[n]:8.2f} = {t:9.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
