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

KERNEL_SRCS = ["mpcx_kernels.hip", "mpcx_api.cpp"]
HOST_SRCS = ["host/bignum.cpp", "host/engine.cpp", "host/modint.cpp", "host/paillier.cpp", "host/safeprime.cpp",
             "host/capi.cpp"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("[mpcium_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force: bool = False, verbose: bool = True) -> dict:
    out = {}
    lib = os.path.join(HERE, "libmpcx.so")
    deps = [os.path.join(CSRC, s) for s in KERNEL_SRCS] + [
        os.path.join(CSRC, "mpcx_internal.h"), os.path.join(ROOT, "include", "mpcx.h")]
    if force or _newer(lib, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-result", "-fvisibility=default",
              "-I", os.path.join(ROOT, "include"), "-o", lib] + [os.path.join(CSRC, s) for s in KERNEL_SRCS])
    out["libmpcx"] = lib
    host_srcs = [os.path.join(CSRC, s) for s in HOST_SRCS if os.path.exists(os.path.join(CSRC, s))]
    if host_srcs:
        hlib = os.path.join(HERE, "libmpcx_host.so")
        hdeps = host_srcs + [os.path.join(CSRC, "host", h) for h in os.listdir(os.path.join(CSRC, "host"))
                             if h.endswith(".hpp")] + [os.path.join(ROOT, "include", "mpcx_host.h")]
        if force or _newer(hlib, hdeps + [lib]):
            _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-pthread",
                  "-I", os.path.join(ROOT, "include"), "-I", os.path.join(CSRC, "host"),
                  "-o", hlib] + host_srcs + ["-L", HERE, "-lmpcx", "-Wl,-rpath,$ORIGIN"])
        out["libmpcx_host"] = hlib
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
