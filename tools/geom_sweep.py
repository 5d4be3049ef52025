#!/usr/bin/env python3
"""Batch-size sweep of one class's geometries: 4096-bit (main 4x37, mid 8x19,
narrow 32x5; x^N mod N^2) or, with --class 1, 2048-bit (main 2x37, 4x19,
narrow 16x5; x^N mod N): wall time of the shared 2048-bit exponent and of
per-operand 768-bit exponents for each forced geometry, interleaved, min of
`reps`; a few outputs checked against CPython pow.
GPU box: python tools/geom_sweep.py [counts] [--class 1]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mpcium_amd import mpcx as M  # noqa: E402


def main():
    reps = 3
    args = [a for a in sys.argv[1:] if a != "--class" and a != "1"]
    cls1 = "--class" in sys.argv
    key = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")))
    N = int(key["N"], 16)
    m = N if cls1 else N * N
    M.init(0)
    mod = M.Modulus(m)
    rng = np.random.default_rng(7)
    counts = [int(c) for c in (args[0].split(",") if args else
                               "1250,2500,5000,7500,10000,15000,20000,25000,30000,40000".split(","))]
    geoms = [5, 1, 3] if cls1 else [2, 6, 4]
    W = mod.words
    ew = M.int_to_words(N, 64)
    res = []
    for count in counts:
        bases = rng.integers(0, 2 ** 32, size=(count, W), dtype=np.uint32)
        bases[:, -1] &= 0x0FFFFFFF if not cls1 else 0x3FFFFFFF  # < m
        pexp = rng.integers(0, 2 ** 32, size=(count, 24), dtype=np.uint32)  # 768-bit per-operand
        row = {"count": count}
        for shape, ex, shared in (("yN", ew, True), ("e768", pexp, False)):
            best = {g: 1e9 for g in geoms}
            for r in range(reps):
                for g in geoms:
                    M.set_option("force_geom", g)
                    t0 = time.perf_counter()
                    out = mod.exp_words(bases, ex, shared)
                    best[g] = min(best[g], time.perf_counter() - t0)
                    if r == 0:
                        for i in (0, count // 2, count - 1):
                            x = int.from_bytes(bases[i].tobytes(), "little")
                            e = N if shared else int.from_bytes(pexp[i].tobytes(), "little")
                            assert int.from_bytes(out[i].tobytes(), "little") == pow(x, e, m), (g, i)
            M.set_option("force_geom", -1)
            row[shape] = {str(g): round(best[g] * 1e3, 2) for g in geoms}
        res.append(row)
        print(json.dumps(row), flush=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "geom_sweep%s.json" % ("_c1" if cls1 else "")), "w"), indent=1)


if __name__ == "__main__":
    main()
