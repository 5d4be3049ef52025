#!/usr/bin/env python3
"""Build a variant libmpcx.so for an interleaved A/B (tools/gpu.sh ab):
recompile ONE translation unit with extra flags and link it with the current
build's other objects.
usage: tools/build_variant.py <out_dir> <source under mpcium_amd/csrc> [-Dflag ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpcium_amd import build as b  # noqa: E402


def main():
    out_dir, src, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
    os.makedirs(out_dir, exist_ok=True)
    b.build()  # the current objects
    objs = []
    for o, s, f in b._objects():
        if s == src:
            vo = os.path.join(out_dir, os.path.basename(o))
            subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}"] + b.HIP_FLAGS + f + flags +
                           ["-I", os.path.join(ROOT, "include"), "-c", "-o", vo, os.path.join(b.CSRC, s)], check=True)
            objs.append(vo)
        else:
            objs.append(o)
    lib = os.path.join(out_dir, "libmpcx.so")
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
