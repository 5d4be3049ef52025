#!/usr/bin/env python3
"""Kernel-time A/B of libmpcx builds in one process each: python tools/ab_time.py <libmpcx.so> [reps]
times 65,536 x^N mod N^2 (4096-bit, shared 2048-bit exponent) through the
device-buffer-free host API (best of reps, wall time of the call) -- for
timing-only variants whose results are not checked."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpcium_amd import mpcx as M  # noqa: E402

M._LIB_PATH = os.path.abspath(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
key = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")))
N = int(key["N"], 16)
M.init(0)
mod = M.Modulus(N * N)
rng = np.random.default_rng(1)
B = rng.integers(0, 2 ** 32, size=(65536, mod.words), dtype=np.uint32)
B[:, -1] &= 0x0FFFFFFF
E = M.int_to_words(N, 64)
best = 1e9
for _ in range(reps):
    t0 = time.perf_counter()
    mod.exp_words(B, E, True)
    best = min(best, time.perf_counter() - t0)
print(json.dumps({"lib": sys.argv[1], "ms": round(best * 1e3, 2)}))
