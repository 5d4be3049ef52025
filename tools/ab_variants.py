"""A/B compile-time variants of libmpcx.so in ONE process (guide rule 24).

  python tools/ab_variants.py build            # here: builds build/ab/<name>/libmpcx.so
  python tools/ab_variants.py run [rounds]     # GPU box: interleaved timing

Each variant is a separate .so (same C-ABI) loaded side by side with ctypes.
"""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "ab")

VARIANTS = json.loads(os.environ.get("AB_VARIANTS", "null")) or {
    "base": [],
    "nosb": ["-DMPCX_SCHED_BARRIER=0"],
    "nopf": ["-DMPCX_PREFETCH_B=0"],
    "c2w2": ["-DMPCX_WAVES_PER_EU_C2=2"],
    "c1w3": ["-DMPCX_WAVES_PER_EU_C1=3"],
}


def build():
    csrc = os.path.join(ROOT, "mpcium_amd", "csrc")
    procs = []
    for name, flags in VARIANTS.items():
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wno-unused-result", "-I", os.path.join(ROOT, "include")] + flags + [
            "-o", os.path.join(d, "libmpcx.so"), os.path.join(csrc, "mpcx_kernels.hip"), os.path.join(csrc, "mpcx_api.cpp")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0
    json.dump(VARIANTS, open(os.path.join(OUT, "variants.json"), "w"))


def run(rounds=3):
    from mpcium_amd import mpcx as M
    variants = json.load(open(os.path.join(OUT, "variants.json")))
    key = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")))
    N = int(key["N"], 16)
    cases = [("c2_N2_yN", N * N, N, 65536), ("c1_N_y2048", N, N - 1, 65536)]
    libs = {}
    for name in variants:
        l = ctypes.CDLL(os.path.join(OUT, name, "libmpcx.so"))
        for fn, res, args in M.SIGNATURES:
            getattr(l, fn).restype = res
            getattr(l, fn).argtypes = args
        assert l.mpcx_init(0) == 0, l.mpcx_last_error()
        libs[name] = l
    results = {}
    for cname, m, e, count in cases:
        words = (m.bit_length() + 31) // 32
        rng = np.random.default_rng(1)
        bases = rng.integers(0, 1 << 32, size=(count, words), dtype=np.uint64).astype(np.uint32)
        bases[:, -1] %= max((m >> (32 * (words - 1))), 1)
        ew = M.nwords(e)
        ex = M.int_to_words(e, ew)
        state = {}
        for name, l in libs.items():
            h = ctypes.c_void_p()
            mw = M.int_to_words(m, words)
            assert l.mpcx_modulus_register(mw.ctypes.data, words, ctypes.byref(h)) == 0
            ptrs = []
            for nbytes in (bases.nbytes, ex.nbytes, bases.nbytes):
                p = ctypes.c_void_p()
                assert l.mpcx_dev_alloc(nbytes, ctypes.byref(p)) == 0
                ptrs.append(p)
            l.mpcx_memcpy_h2d(ptrs[0], bases.ctypes.data, bases.nbytes)
            l.mpcx_memcpy_h2d(ptrs[1], ex.ctypes.data, ex.nbytes)
            state[name] = (h, ptrs)
        times = {n: [] for n in libs}
        outs = {}
        for r in range(rounds + 1):
            for name, l in libs.items():
                h, ptrs = state[name]
                t0 = time.perf_counter()
                rc = l.mpcx_modexp_batch_device(h, count, ptrs[0], words, ptrs[1], ew, 1, e.bit_length(), ptrs[2], words, None)
                assert rc == 0, l.mpcx_last_error()
                l.mpcx_stream_sync(None)
                dt = time.perf_counter() - t0
                if r > 0:
                    times[name].append(dt)
                if r == 0:
                    o = np.zeros_like(bases)
                    l.mpcx_memcpy_d2h(o.ctypes.data, ptrs[2], o.nbytes)
                    outs[name] = o
        ref = outs[next(iter(outs))]
        idx = [0, 1, count // 2, count - 1]
        xs = M.words_to_ints(bases[idx]); zs = M.words_to_ints(ref[idx])
        ok_pow = all(pow(x, e, m) == z for x, z in zip(xs, zs))
        for name in libs:
            med = sorted(times[name])[len(times[name]) // 2]
            results.setdefault(cname, {})[name] = {"ms_median": med * 1e3, "ms_min": min(times[name]) * 1e3,
                                                   "rate": count / med, "same_as_ref": bool((outs[name] == ref).all()),
                                                   "ref_matches_pow": ok_pow}
        print(cname, json.dumps(results[cname]), flush=True)
    return results


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        res = run(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        json.dump(res, open(os.path.join(ROOT, "gpurun_out", "ab_results.json"), "w"), indent=1)
