import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpcium_amd import host, mpcx
mpcx.init(0); host.init(0)
for seed in (1, 2):
    t = time.time()
    got, st = host.safe_primes(1024, 4, seed=seed)
    el = time.time() - t
    print(json.dumps({"seed": seed, "seconds": el, **st, "fermat_per_s": st["fermat_tests"] / el}), flush=True)
