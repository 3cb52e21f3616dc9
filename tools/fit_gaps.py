#!/usr/bin/env python3
"""Device idle time inside the last MiniBatchKMeans fit of a rocprofv3 kernel trace (k_kpp_init ..
k_assign_finalize): span, busy time, the gaps between kernels and the kernels they precede."""
import csv
import statistics
import sys
from collections import defaultdict


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    i0 = [i for i, n in enumerate(names) if "k_kpp_init" in n][-1]
    i1 = next(i for i in range(i0, len(rows)) if "k_assign_finalize" in names[i])
    seg = rows[i0:i1 + 1]
    t0, end = int(seg[0]["Start_Timestamp"]), int(seg[0]["Start_Timestamp"])
    busy, gaps, per = 0, [], defaultdict(lambda: [0, 0.0])
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            gaps.append(((s - end) / 1000, r["Kernel_Name"][:40]))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        k = r["Kernel_Name"][:40]
        per[k][0] += 1
        per[k][1] += (e - s) / 1000
    print(f"fit span {(end - t0) / 1000:.1f} us, busy {busy / 1000:.1f} us, gaps {sum(g for g, _ in gaps):.1f} us "
          f"in {len(gaps)} (median {statistics.median([g for g, _ in gaps]) if gaps else 0:.1f}), {len(seg)} kernels")
    by = defaultdict(float)
    for g, n in gaps:
        by[n] += g
    print("gap time by the kernel it precedes:", {n: round(v, 1) for n, v in sorted(by.items(), key=lambda x: -x[1])[:6]})
    print("kernel time:", {n: (c, round(t, 1)) for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:8]})


if __name__ == "__main__":
    main(sys.argv[1])
