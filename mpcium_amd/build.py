"""Build the gfx950 extension libraries in-tree (no JIT cache, no pip install).

libmpcx.so       -- C-ABI engine (include/mpcx.h): HIP kernels + host API.
libmpcx_host.so  -- C++ host mirror of the reference interfaces (ModInt.Exp,
                    crypto/paillier, safe-prime search) layered on the C-ABI.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

NUM_GEOMS = 7  # kernel geometries (mpcx_internal.h), one translation unit each
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result"]
KERNEL_HDRS = ["mpcx_device.hpp", "mpcx_mx.hpp", "mpcx_internal.h"]
HOST_SRCS = ["host/bignum.cpp", "host/engine.cpp", "host/modint.cpp", "host/paillier.cpp", "host/safeprime.cpp",
             "host/tsscommon.cpp", "host/secp256k1.cpp", "host/mta.cpp", "host/proofs.cpp", "host/signing.cpp", "host/keygenload.cpp",
             "host/hostprof.cpp", "host/gorand.cpp", "host/capi.cpp"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("[mpcium_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _objects():
    """(object, source, extra flags) of libmpcx.so: one k_modexp geometry per
    object (compiled in parallel: the unrolled Montgomery loops make each
    geometry ~30-60 s of hipcc), the prime kernels, and the C-ABI host code."""
    objdir = os.path.join(HERE, "build")
    objs = [(os.path.join(objdir, f"mpcx_geom{g}.o"), "mpcx_geom.hip", [f"-DMPCX_GEOM_ID={g}"])
            for g in range(NUM_GEOMS)]
    objs.append((os.path.join(objdir, "mpcx_prime.o"), "mpcx_prime.hip", []))
    objs.append((os.path.join(objdir, "mpcx_ec.o"), "mpcx_ec.hip", []))
    objs.append((os.path.join(objdir, "mpcx_api.o"), "mpcx_api.cpp", []))
    return objs


def build(force: bool = False, verbose: bool = True, jobs: int = 0) -> dict:
    from concurrent.futures import ThreadPoolExecutor
    out = {}
    lib = os.path.join(HERE, "libmpcx.so")
    common = [os.path.join(CSRC, h) for h in KERNEL_HDRS] + [os.path.join(ROOT, "include", "mpcx.h")]
    objs = _objects()
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    todo = [(o, s, f) for o, s, f in objs if force or _newer(o, [os.path.join(CSRC, s)] + common)]
    if todo:
        def one(item):
            o, src, flags = item
            _run([HIPCC, f"--offload-arch={ARCH}"] + HIP_FLAGS + flags +
                 ["-I", os.path.join(ROOT, "include"), "-c", "-o", o, os.path.join(CSRC, src)])
        n = jobs or min(len(todo), max(1, (os.cpu_count() or 2)), 16)
        with ThreadPoolExecutor(n) as ex:
            list(ex.map(one, todo))
    if force or todo or _newer(lib, [o for o, _, _ in objs]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + [o for o, _, _ in objs])
    out["libmpcx"] = lib
    host_srcs = [os.path.join(CSRC, s) for s in HOST_SRCS if os.path.exists(os.path.join(CSRC, s))]
    if host_srcs:
        # one object per host source (compiled in parallel), then one link
        hlib = os.path.join(HERE, "libmpcx_host.so")
        hdrs = [os.path.join(CSRC, "host", h) for h in os.listdir(os.path.join(CSRC, "host"))
                if h.endswith(".hpp")] + [os.path.join(ROOT, "include", "mpcx_host.h"),
                                          os.path.join(ROOT, "include", "mpcx.h")]
        hdir = os.path.join(HERE, "build", "host")
        os.makedirs(hdir, exist_ok=True)
        hobjs = [(os.path.join(hdir, os.path.basename(src)[:-4] + ".o"), src) for src in host_srcs]
        htodo = [(o, src) for o, src in hobjs if force or _newer(o, [src] + hdrs)]
        if htodo:
            def hone(item):
                o, src = item
                _run(["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-pthread",
                      "-I", os.path.join(ROOT, "include"), "-I", os.path.join(CSRC, "host"), "-c", "-o", o, src])
            n = jobs or min(len(htodo), max(1, (os.cpu_count() or 2)), 16)
            with ThreadPoolExecutor(n) as ex:
                list(ex.map(hone, htodo))
        if force or htodo or _newer(hlib, [o for o, _ in hobjs] + [lib]):
            _run(["g++", "-shared", "-pthread", "-o", hlib] + [o for o, _ in hobjs] +
                 ["-L", HERE, "-lmpcx", "-lcrypto", "-Wl,-rpath,$ORIGIN"])
        out["libmpcx_host"] = hlib
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
