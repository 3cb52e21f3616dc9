#!/usr/bin/env python3
"""Per-dispatch durations of one kernel from a rocprofv3 --kernel-trace CSV: the count, the mean,
the sum, and the largest dispatches (the reassignments that fire stand out from the checks that
do not).

usage: python tools/kernel_durations.py <kernel_trace.csv> <name substring> [top]
"""
import csv
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    d = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if key in r["Kernel_Name"]:
                d.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    if not d:
        print(f"{key}: no dispatches")
        return
    s = sorted(d, reverse=True)
    small = [x for x in d if x < 4.0]
    print(f"{key}: {len(d)} dispatches, mean {sum(d) / len(d):.2f} us, sum {sum(d):.1f} us; "
          f"< 4 us: {len(small)} (mean {sum(small) / max(1, len(small)):.2f}); "
          f"largest: " + " ".join(f"{x:.1f}" for x in s[:top]))


if __name__ == "__main__":
    main()
