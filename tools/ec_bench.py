#!/usr/bin/env python3
"""Isolated timing of k_ec_combine (secp256k1 a G + b P + c Q, one thread per
item) at signing's batch shapes, kernel time from libmpcx's per-launch HIP
events (mpcx_kernel_stats), checked against the oracle on a sample.
MPCX_LIB_PATH selects another libmpcx build (A/B).

    python tools/ec_bench.py [--reps 5] [--sizes 2048,11264,65536]
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
    ap.add_argument("--sizes", default="2048,11264,65536")
    args = ap.parse_args()
    from mpcium_amd import mpcx
    from oracle import tss_ref as T
    mpcx.init(0)
    rng = random.Random(7)
    n = T.SECP_N
    pts = [T.scalar_base_mult(rng.randrange(1, n)) for _ in range(64)]
    out = {"lib": os.environ.get("MPCX_LIB_PATH", "mpcium_amd/libmpcx.so"), "rows": []}
    for size in (int(x) for x in args.sizes.split(",")):
        for shape in ("aG+bP", "aG+bP+cQ"):
            items = []
            for i in range(size):
                P, Q = pts[i % 64], pts[(i * 7 + 3) % 64]
                c = rng.randrange(n) if shape == "aG+bP+cQ" else 0
                items.append((rng.randrange(n), rng.randrange(n), c, P, Q if c else None))
            got = mpcx.ec_combine_batch(items)  # warm-up + check
            for i in range(0, size, max(1, size // 6)):
                a, b, c, P, Q = items[i]
                want = T.ec_add(T.scalar_base_mult(a), T.ec_mul(b, P))
                if Q is not None:
                    want = T.ec_add(want, T.ec_mul(c, Q))
                assert got[i] == want, (size, shape, i)
            mpcx.set_option("kernel_stats", 1)
            mpcx.kernel_stats(reset=True)
            for _ in range(args.reps):
                mpcx.ec_combine_batch(items)
            ks = mpcx.kernel_stats()
            mpcx.set_option("kernel_stats", 0)
            k = [x for x in ks["kernels"] if x["kind"].startswith("ec")][0]
            ms = k["kernel_ms"] / k["launches"]
            row = {"items": size, "shape": shape, "kernel_ms": round(ms, 3), "items_per_s": round(size / ms * 1e3)}
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
