#!/usr/bin/env python3
"""Occupancy timeline of a rocprofv3 kernel trace: for every bin, the time-
weighted number of resident wavefronts of the mpcx kernels in flight, as a
fraction of the chip's resident capacity for each kernel's geometry (waves
per SIMD x 1024 SIMDs, from the kernel's VGPR count), summed over concurrent
kernels and capped at 1.
usage: tools/trace_occupancy.py <kernel_trace.csv> [bin_ms] [t0_ms] [t1_ms]"""
import csv
import sys


def waves_per_simd(vgpr):
    return max(1, min(8, 512 // max(1, vgpr)))


def main():
    path = sys.argv[1]
    bin_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
    ev = []
    for r in csv.DictReader(open(path)):
        if "mpcx::" not in r["Kernel_Name"]:
            continue
        waves = int(r["Grid_Size_X"]) // 64
        cap = waves_per_simd(int(r["VGPR_Count"]) + int(r.get("Accum_VGPR_Count") or 0)) * 1024
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), min(1.0, waves / cap),
                   r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mpcx::", "")))
    ev.sort()
    base = ev[0][0]
    t0 = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    t1 = float(sys.argv[4]) if len(sys.argv) > 4 else (max(e[1] for e in ev) - base) / 1e6
    b = t0
    tot_busy = tot_occ = 0.0
    while b < t1:
        lo, hi = base + b * 1e6, base + (b + bin_ms) * 1e6
        occ = busy = 0.0
        n = 0
        segs = []
        for s, e, f, name in ev:
            if e <= lo or s >= hi:
                continue
            ov = (min(e, hi) - max(s, lo)) / (hi - lo)
            occ += f * ov
            n += 1
            segs.append((max(s, lo), min(e, hi)))
        segs.sort()
        cur = None
        for s, e in segs:
            if cur is None or s > cur[1]:
                if cur:
                    busy += cur[1] - cur[0]
                cur = [s, e]
            else:
                cur[1] = max(cur[1], e)
        if cur:
            busy += cur[1] - cur[0]
        busy /= (hi - lo)
        tot_busy += busy * bin_ms
        tot_occ += min(1.0, occ) * bin_ms
        print(f"{b:8.0f} ms  kernels {n:3d}  busy {busy:4.2f}  occupancy {min(1.0, occ):4.2f}")
        b += bin_ms
    print(f"total: busy {tot_busy / (t1 - t0):.3f}, mean occupancy {tot_occ / (t1 - t0):.3f} over {t1 - t0:.0f} ms")


if __name__ == "__main__":
    main()
