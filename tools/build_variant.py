#!/usr/bin/env python3
"""Build a variant libmpcx.so for an interleaved A/B (tools/gpu.sh ab):
recompile ONE translation unit with extra flags and link it with the current
build's other objects.
usage: tools/build_variant.py <out_dir> <source under mpcium_amd/csrc | src1,src2 | all> [-Dflag ...]
("all": every HIP translation unit, e.g. for a flag read by mpcx_device.hpp)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpcium_amd import build as b  # noqa: E402


def main():
    out_dir, src, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
    srcs = set(src.split(","))
    os.makedirs(out_dir, exist_ok=True)
    b.build()  # the current objects
    objs, jobs = [], []
    for o, s, f in b._objects():
        if s in srcs or (src == "all" and s.endswith(".hip")):
            vo = os.path.join(out_dir, os.path.basename(o))
            jobs.append([b.HIPCC, f"--offload-arch={b.ARCH}"] + b.HIP_FLAGS + f + flags +
                        ["-I", os.path.join(ROOT, "include"), "-c", "-o", vo, os.path.join(b.CSRC, s)])
            objs.append(vo)
        else:
            objs.append(o)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(8, max(1, len(jobs)))) as ex:
        list(ex.map(lambda c: subprocess.run(c, check=True), jobs))
    lib = os.path.join(out_dir, "libmpcx.so")
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
