#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace (CSV) into segments separated by GPU-idle
gaps (default 150 ms) and print per-kernel time per segment: separates a
bench run's warm-up batches from its timed regions.
usage: tools/trace_segments.py <kernel_trace.csv> [gap_ms]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 150.0
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(path)))
    segs, end = [], None
    for e in ev:
        if end is None or e[0] - end > gap * 1e6:
            segs.append([])
        segs[-1].append(e)
        end = e[1] if end is None else max(end, e[1])
    for s in segs:
        span = (max(x[1] for x in s) - s[0][0]) / 1e6
        agg = collections.defaultdict(lambda: [0, 0])
        for a, b, n in s:
            k = n.split("(")[0].replace("void ", "").replace("mpcx::", "")
            agg[k][0] += 1
            agg[k][1] += b - a
        busy = sum(v[1] for v in agg.values()) / 1e6
        print(f"segment: {len(s)} kernels, span {span:.1f} ms, kernel time {busy:.1f} ms")
        for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:6]:
            print(f"   {k:36s} {v[0]:5d} {v[1] / 1e6:9.1f} ms  {100 * v[1] / 1e6 / max(busy, 1e-9):5.1f}%")


if __name__ == "__main__":
    main()
