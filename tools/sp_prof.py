#!/usr/bin/env python3
"""Host-time profile of the config-3 search (MPCX_HOST_PROFILE=1 in the
environment): warm-up, then `num` 1024-bit safe primes; prints the wall time
and the profile scopes (sp.step, sp.join_wait, sp.stage_b, ...)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpcium_amd import host as H  # noqa: E402

num = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H.init(0)
H.safe_primes(1024, int(sys.argv[2]) if len(sys.argv) > 2 else 1, seed=0x5AFE + 1)
H.profile_report(reset=True)
t0 = time.perf_counter()
res, st = H.safe_primes(1024, num, seed=0x5AFE)
el = time.perf_counter() - t0
print(f"{num} safe primes in {el:.4f} s = {num / el:.1f}/s; {st}")
print(H.profile_report())
