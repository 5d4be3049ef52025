"""Fixed-base comb vs generic per-operand modexp on the N~ shape (2048-bit
modulus, h1^a h2^b with 2048/2816-bit exponents). Prints one JSON line."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpcium_amd import mpcx  # noqa: E402


def main(count=32768):
    mpcx.init(0)
    with open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "node_preparams.json")) as f:
        node = json.load(f)["nodes"][0]
    Nt, h1, h2 = (int(node[k], 16) for k in ("NTildei", "H1i", "H2i"))
    rng = random.Random(5)
    mod = mpcx.Modulus(Nt)
    t0 = time.perf_counter()
    f1, f2 = mpcx.FixedBase(mod, h1, 2816), mpcx.FixedBase(mod, h2, 2816)
    t_reg = time.perf_counter() - t0
    a = [rng.getrandbits(2048) for _ in range(count)]
    b = [rng.getrandbits(2816) for _ in range(count)]
    res = {"count": count, "register_s_two_tables": t_reg, "table_bytes": f1.table_bytes}
    for rep in range(2):
        t0 = time.perf_counter()
        z = mpcx.fixedbase_exp([f1, f2], [a, b])
        res["fixedbase_h1a_h2b_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        x = mod.exp([h1] * count, a)
        y = mod.exp_mul([h2] * count, b, x)
        res["generic_h1a_h2b_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        z1 = mpcx.fixedbase_exp([f1], [a])
        res["fixedbase_h1a_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        x1 = mod.exp([h1] * count, a)
        res["generic_h1a_s"] = time.perf_counter() - t0
    assert z == y and z1 == x1
    idx = rng.sample(range(count), 8)
    assert all(z[i] == pow(h1, a[i], Nt) * pow(h2, b[i], Nt) % Nt for i in idx)
    res["speedup_h1a_h2b"] = res["generic_h1a_h2b_s"] / res["fixedbase_h1a_h2b_s"]
    res["speedup_h1a"] = res["generic_h1a_s"] / res["fixedbase_h1a_s"]
    print(json.dumps(res))


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
