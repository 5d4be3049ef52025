#!/usr/bin/env python3
"""Where config 1's time goes: Encrypt + HomoMult batches of 1,024 through the
host mirror (libmpcx_host.so), one at a time and `--inflight` at a time from
their own threads; per-call wall times, the Python conversion share, and
libmpcx's kernel stats. Run under rocprofv3 --kernel-trace to see overlap.

    python tools/paillier_probe.py [--reps 10] [--inflight 4]
"""
import argparse
import json
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    from mpcium_amd import host as mhost, mpcx
    mhost.init(0)
    N = int(json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")))["N"], 16)
    pk = mhost.PublicKey(N)
    rng = random.Random(5)
    Q = mpcx.SECP_N
    ms = [rng.randrange(N) for _ in range(args.batch)]
    rs = [rng.randrange(1, N) for _ in range(args.batch)]
    bs = [rng.randrange(Q) for _ in range(args.batch)]
    cs, _ = pk.encrypt(ms, rs)
    pk.homo_mult(bs, cs)
    out = {}
    t = {"enc": [], "hm": []}
    t0 = time.perf_counter()
    for _ in range(args.reps):
        a = time.perf_counter()
        c, _ = pk.encrypt(ms, rs)
        b = time.perf_counter()
        pk.homo_mult(bs, c)
        t["enc"].append(b - a)
        t["hm"].append(time.perf_counter() - b)
    el = time.perf_counter() - t0
    out["sequential"] = {"ops_per_s": args.batch * args.reps / el, "enc_ms": 1e3 * sum(t["enc"]) / args.reps,
                         "homomult_ms": 1e3 * sum(t["hm"]) / args.reps}
    a = time.perf_counter()
    for _ in range(args.reps):
        W = mpcx.ints_to_words(ms, 64), mpcx.ints_to_words(rs, 64)
        mpcx.words_to_ints(mpcx.ints_to_words(cs, 128))
        mpcx.ints_to_words(bs, 8), mpcx.ints_to_words(cs, 128)
        mpcx.words_to_ints(mpcx.ints_to_words(cs, 128))
    out["python_conversions_ms_per_batch"] = 1e3 * (time.perf_counter() - a) / args.reps
    per = [[] for _ in range(args.inflight)]

    def worker(k):
        for _ in range(args.reps):
            a = time.perf_counter()
            c, _ = pk.encrypt(ms, rs)
            pk.homo_mult(bs, c)
            per[k].append(time.perf_counter() - a)
    mpcx.set_option("kernel_stats", 1)
    mpcx.kernel_stats(reset=True)
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(args.inflight)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    ks = mpcx.kernel_stats()
    mpcx.set_option("kernel_stats", 0)
    out["inflight"] = {"n": args.inflight, "ops_per_s": args.batch * args.reps * args.inflight / el,
                       "batch_ms_mean": 1e3 * sum(sum(p) for p in per) / (args.reps * args.inflight),
                       "kernels": ks["kernels"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
