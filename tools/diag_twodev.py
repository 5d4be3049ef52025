#!/usr/bin/env python3
"""Diagnostic (GPU box): keygen proof batches with one HIP ordinal bound as two
logical devices vs one, with and without the launch coalescers, small waves
(the tests/test_gpu_multidev.py::test_two_logical_devices shape).
    python tools/diag_twodev.py <dup 0|1>   (MPCX_COALESCE=0 in the env turns coalescing off)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden  # noqa: E402
from mpcium_amd import host, mpcx, proofs  # noqa: E402

dup = sys.argv[1] == "1"
if dup:
    mpcx.set_option("duplicate_device", 1)
host.init(0)
if dup:
    host.init(0)
d = load_golden("node_preparams.json")
nodes = [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]
res = []
for rep in range(3):
    st = proofs.bench_keygen_proofs(nodes, 24, seed=0x10E + rep, wave=12)
    res.append(int(st["failures"]))
print(json.dumps({"dup": dup, "coalesce": os.environ.get("MPCX_COALESCE", "default"), "failures": res}), flush=True)
