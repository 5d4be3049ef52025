#!/usr/bin/env python3
"""Isolated timing of the fixed-base comb kernel (k_fixedbase) on one GPU:
h1^a (one table) and h1^a h2^b (two tables) mod a 2048-bit N~ with 2048-bit
and 2816-bit exponents (DLN proofs, MtA range proofs), at several batch sizes,
kernel time from libmpcx's per-launch HIP events (mpcx_kernel_stats). Checked
against pow() on a sample. MPCX_LIB_PATH selects another libmpcx build (A/B).

    python tools/comb_bench.py [--reps 5]
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sizes", default="2048,16384,131072")
    ap.add_argument("--split", type=int, default=None, help="option fb_split (0: by launch size)")
    args = ap.parse_args()
    from mpcium_amd import mpcx
    mpcx.init(0)
    if args.split is not None:
        mpcx.set_option("fb_split", args.split)
    nodes = json.load(open(os.path.join(ROOT, "tests", "golden", "node_preparams.json")))["nodes"]
    Nt, h1, h2 = (int(nodes[0][k], 16) for k in ("NTildei", "H1i", "H2i"))
    mod = mpcx.Modulus(Nt)
    f1, f2 = mpcx.FixedBase(mod, h1, 3072), mpcx.FixedBase(mod, h2, 3072)
    rng = random.Random(5)
    out = {"lib": os.environ.get("MPCX_LIB_PATH", "mpcium_amd/libmpcx.so"), "split": args.split, "rows": []}
    for n in (int(x) for x in args.sizes.split(",")):
        for bits, nb in ((2048, 1), (2816, 2)):
            es = [[rng.getrandbits(bits) for _ in range(n)] for _ in range(nb)]
            fbs = [f1, f2][:nb]
            got = mpcx.fixedbase_exp(fbs, es)  # warm-up + check
            for i in range(0, n, max(1, n // 4)):
                w = 1
                for t in range(nb):
                    w = w * pow([h1, h2][t], es[t][i], Nt) % Nt
                assert got[i] == w, (n, bits, i)
            mpcx.set_option("kernel_stats", 1)
            mpcx.kernel_stats(reset=True)
            for _ in range(args.reps):
                mpcx.fixedbase_exp(fbs, es)
            ks = mpcx.kernel_stats()
            mpcx.set_option("kernel_stats", 0)
            k = [x for x in ks["kernels"] if x["kind"].startswith("fixedbase")][0]
            ms = k["kernel_ms"] / k["launches"]
            prods = n * nb * ((bits + 11) // 12)
            row = {"ops": n, "exp_bits": bits, "bases": nb, "kernel_ms": round(ms, 3), "ops_per_s": round(n / ms * 1e3),
                   "products_per_s": round(prods / ms * 1e3), "exec_frac": round(k["alg_macs"] / (k["kernel_ms"] / 1e3)
                                                                               / (256 * 64 * 2.4e9), 3)}
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
