#!/usr/bin/env python3
"""Per-kernel roofline of a workload from two files of the same run:
a rocprofv3 kernel trace (CSV) and libmpcx's launch log (MPCX_LAUNCH_LOG=path:
kind, geometry, operands, modulus bits, exponent bits, Go-equivalent MACs per
launch). For each kernel: launches, operands, the Go-equivalent work
(SURVEY.md 8(d) W summed over the operands' own exponents), the summed kernel
time from the trace, and work / time against the nominal INT32 MAD peak
(256 CU x 64 lanes x 2.4 GHz = 39.3 T/s). Kernels that overlap on the GPU
(concurrent lanes) share it, so a kernel's summed time over-counts its share
and its frac is a lower bound.
usage: tools/kernel_frac.py <kernel_trace.csv> <launch_log.csv> [t0_ns t1_ns]"""
import collections
import csv
import sys

PEAK = 256 * 64 * 2.4e9
# geometry id -> (P, K, G) (mpcx_internal.h MPCX_GEOM_P/K/G)
GEOM = {0: (1, 37, 64), 1: (4, 19, 16), 2: (4, 37, 16), 3: (16, 5, 4), 4: (32, 5, 2), 5: (3, 25, 21), 6: (8, 19, 8)}


def kname(kind, geom):
    if kind == "ec_combine":
        return "k_ec_combine"
    P, K, G = GEOM[geom]
    return f"k_{kind}<{P}, {K}, {G},"


def main():
    trace, log = sys.argv[1], sys.argv[2]
    t0 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    t1 = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 62
    work = collections.defaultdict(lambda: [0, 0, 0.0])
    for r in csv.DictReader(open(log)):
        k = kname(r["kind"], int(r["geom"]))
        w = work[k]
        w[0] += 1
        w[1] += int(r["operands"])
        w[2] += float(r["alg_macs"])
    tm = collections.defaultdict(lambda: [0, 0])
    for r in csv.DictReader(open(trace)):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if a < t0 or b > t1:
            continue
        name = r["Kernel_Name"].replace("void ", "").replace("mpcx::", "")
        for k in work:
            if name.startswith(k):
                tm[k][0] += 1
                tm[k][1] += b - a
    print(f"{'kernel':28s} {'launches':>8s} {'traced':>7s} {'operands':>10s} {'Go-eq MACs':>12s} {'time ms':>9s} {'frac':>6s}")
    for k, (n, ops, alg) in sorted(work.items(), key=lambda x: -tm[x[0]][1]):
        ms = tm[k][1] / 1e6
        frac = alg / (ms * 1e-3) / PEAK if ms > 0 and alg > 0 else float("nan")
        print(f"{k:28s} {n:8d} {tm[k][0]:7d} {ops:10d} {alg:12.4g} {ms:9.1f} {frac:6.3f}")


if __name__ == "__main__":
    main()
