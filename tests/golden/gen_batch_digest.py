#!/usr/bin/env python3
"""Generate tests/golden/batch_digest.json: SHA-256 over the whole config-2
batch of bench.py (65,536 bases x^N mod N^2 of the 2048-bit golden Paillier
key, bench.synth_bases with rank 0's seed), every output computed by the
oracle's C restatement of Go's expNN (oracle/gomodexp.c, 64-bit words) and a
1/64 sample cross-checked with GMP mpz_powm. Test infrastructure, run offline
(~6 min on 8 processes): tests/test_gpu_modexp.py and bench.py compare the
GPU's outputs with this digest.

Digest input: the outputs as `words` little-endian uint32 words each (the
device output layout), operand order.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "batch_digest.json")
COUNT = 65536
WORDS = 128          # MPCX_CLASS_WORDS of the 4096-bit class (bench.py: mod.class_words)
SEED = 0x6D706332    # bench.py: synth_bases(N2, count, 0x6D706332 + rank, words), rank 0
CHUNK = 256

_lib = None


def _init():
    global _lib
    from oracle import crosscheck as cc
    _lib = cc.load_c_oracle(64)


def _work(args):
    from oracle import crosscheck as cc
    lo, xs, N, N2 = args
    out = []
    for j, x in enumerate(xs):
        z = cc.c_expnn(_lib, x, N, N2)
        if (lo + j) % 64 == 0:
            g = cc.gmp_powm(x, N, N2)
            assert g is None or g == z, (lo + j)
        out.append(z)
    return lo, out


def synth_bases(N2: int, count: int, seed: int, words: int) -> np.ndarray:
    # same construction as bench.synth_bases
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 1 << 32, size=(count, words), dtype=np.uint64).astype(np.uint32)
    top = (N2 >> (32 * (words - 1))) & 0xFFFFFFFF
    x[:, words - 1] = x[:, words - 1] % max(top, 1)
    return x


def main():
    t0 = time.time()
    key = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")))
    N = int(key["N"], 16)
    N2 = N * N
    B = synth_bases(N2, COUNT, SEED, WORDS)
    xs = [int.from_bytes(B[i].astype("<u4").tobytes(), "little") for i in range(COUNT)]
    jobs = [(lo, xs[lo:lo + CHUNK], N, N2) for lo in range(0, COUNT, CHUNK)]
    res = [None] * COUNT
    with Pool(min(8, os.cpu_count() or 1), initializer=_init) as pool:
        for lo, out in pool.imap_unordered(_work, jobs):
            res[lo:lo + len(out)] = out
    h = hashlib.sha256()
    for z in res:
        h.update(z.to_bytes(4 * WORDS, "little"))
    doc = {"description": "SHA-256 of bench.py's config-2 batch outputs (x^N mod N^2, 65536 operands, rank-0 "
                          "seed), computed by oracle/gomodexp.c (64-bit words), GMP cross-checked on 1/64; "
                          "tests/golden/gen_batch_digest.py",
           "count": COUNT, "words": WORDS, "seed": SEED, "sha256": h.hexdigest(),
           "first_output": format(res[0], "x"), "gen_seconds": round(time.time() - t0, 1)}
    json.dump(doc, open(OUT, "w"), indent=1)
    print("wrote", OUT, doc["sha256"], doc["gen_seconds"], "s")


if __name__ == "__main__":
    main()
