"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/gen_golden.py
(test infrastructure: imports oracle/, never the product path)

Every modexp vector is computed with CPython pow and cross-checked against GMP
mpz_powm, OpenSSL BN_mod_exp and the C restatement of Go expNNMontgomery
(oracle/libgomodexp.so); the generator aborts on any disagreement.  The
reference's own test suite holds no vectors for this path,
so these independent implementations are what pins the oracle.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import crosscheck as cc  # noqa: E402
from oracle import gomath as gm  # noqa: E402
from oracle import safeprime_ref as sp  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED_KEY = 0x6D706331  # BASELINE.md config 1 key seed ("mpc1")
SEED_VEC = 0x6D706332  # BASELINE.md config 2 operand seed ("mpc2")


def h(v: int) -> str:
    return "%x" % v if v >= 0 else "-%x" % (-v)


def checked_pow(x: int, y: int, m: int, c_lib) -> int:
    z = pow(x, y, m)
    checks = {"gmp": cc.gmp_powm(x, y, m), "openssl": cc.openssl_mod_exp(x, y, m)}
    if c_lib is not None:
        checks["c_restatement"] = cc.c_expnn(c_lib, x, y, m)
    for k, v in checks.items():
        if v is not None and v != z:
            raise SystemExit(f"cross-check mismatch ({k}) for m={m:x} x={x:x} y={y:x}")
    return z


def gen_key():
    path = os.path.join(OUT, "paillier_key_2048.json")
    if os.path.exists(path):
        return json.load(open(path))
    t0 = time.time()
    primes = []
    seed = SEED_KEY
    # tss-lib GenerateKeyPair: two 1024-bit safe primes with |P-Q| >= 2^(1024-3)
    while len(primes) < 2:
        got = sp.first_safe_primes(seed, 1024, 1)
        idx, p, q = got[0]
        if primes and abs(primes[0]["p"] - p).bit_length() < 1024 - 3:
            seed += 1
            continue
        primes.append({"seed": seed, "index": idx, "p": p, "q": q})
        seed += 1
    P, Q = primes[0]["p"], primes[1]["p"]
    N = P * Q
    lam = gm.paillier_lambda(P, Q)
    key = {
        "description": "Synthetic node Paillier key: two 1024-bit safe primes from the tss-lib safe-prime "
                       "candidate stream (oracle/safeprime_ref.py) over the CounterDRBG",
        "P": h(P), "Q": h(Q), "N": h(N), "LambdaN": h(lam), "PhiN": h((P - 1) * (Q - 1)),
        "P_seed": primes[0]["seed"], "P_index": primes[0]["index"],
        "Q_seed": primes[1]["seed"], "Q_index": primes[1]["index"],
        "gen_seconds": round(time.time() - t0, 1),
    }
    json.dump(key, open(path, "w"), indent=1)
    return key


def gen_modexp(key, c_lib):
    N = int(key["N"], 16)
    N2 = N * N
    rng = gm.CounterDRBG(SEED_VEC)
    vecs = []

    def add(name, x, y, m):
        vecs.append({"name": name, "m": h(m), "x": h(x), "y": h(y), "z": h(checked_pow(x, y, m, c_lib))})

    # config-2 shapes: mod N^2 (4096-bit) with the exponent lengths of the MtA inventory
    for eb in (0, 1, 2, 64, 65, 256, 768, 1792, 2048, 2304, 4096):
        for i in range(3):
            y = rng.randbits(eb) | (1 << (eb - 1)) if eb > 0 else 0
            add(f"N2_e{eb}_{i}", rng.randbelow(N2), y, N2)
    for i in range(4):
        add(f"N2_yN_{i}", rng.randbelow(N2), N, N2)  # r^N / s^N / beta^N shape
    # mod N (2048-bit) and a 2048-bit random odd modulus (N~ shape) up to 4.9 kbit exponents
    Nt = rng.randbits(2048) | 1 | (1 << 2047)
    for eb in (256, 2048, 2816, 4900):
        for i in range(2):
            add(f"N_e{eb}_{i}", rng.randbelow(N), rng.randbits(eb) | (1 << (eb - 1)), N)
            add(f"Nt_e{eb}_{i}", rng.randbelow(Nt), rng.randbits(eb) | (1 << (eb - 1)), Nt)
    # 1024-bit: Fermat shape on the key's primes and random bases
    P = int(key["P"], 16)
    add("P_fermat", 2, P - 1, P)
    for i in range(3):
        add(f"P_rand_{i}", rng.randbelow(P), rng.randbits(1023), P)
    # moduli that do not fill their kernel class, and class boundaries
    for bits in (3, 17, 31, 32, 33, 63, 64, 65, 500, 1000, 1023, 1024, 1025, 2047, 2080, 2081, 3000, 4095, 4096):
        m = rng.randbits(bits) | 1 | (1 << (bits - 1))
        add(f"mbits{bits}", rng.randbelow(1 << min(bits + 3, 4096)) if bits < 4096 else rng.randbelow(m),
            rng.randbits(300) | 1, m)
    # edge cases of nat.expNN
    add("edge_m1", 12345, 678, 1)
    add("edge_x0", 0, 99, N2)
    add("edge_x1", 1, N, N2)
    add("edge_xm", N2, N, N2)             # x == m
    add("edge_xm1", N2 - 1, N, N2)        # x == m-1 (-1): result +-1
    add("edge_xbig", (1 << 4096) - 1, N, N2)  # len(x) == len(m), x >= m
    add("edge_y1", rng.randbelow(N2), 1, N2)
    add("edge_allones", (1 << 4096) - 1, (1 << 2048) - 1, N2)
    return vecs


def gen_go_semantics(key):
    """Go Int.Exp sign rules (nil for non-invertible negative exponents)."""
    N = int(key["N"], 16)
    N2 = N * N
    rng = gm.CounterDRBG(SEED_VEC + 1)
    cases = []
    for x, y, m in [(-3, 5, 7), (-rng.randbelow(N2), N, N2), (rng.randbelow(N2), -rng.randbits(256), N2),
                    (N, -5, N2), (2, -1, 8), (3, -1, 8), (-(N2 + 5), 3, N2), (5, 0, N2), (-5, 0, N2)]:
        z = gm.go_exp(x, y, m)
        cases.append({"x": h(x), "y": h(y), "m": h(m), "z": None if z is None else h(z)})
    return cases


def gen_paillier(key):
    N = int(key["N"], 16)
    lam = int(key["LambdaN"], 16)
    N2 = N * N
    rng = gm.CounterDRBG(SEED_KEY + 100)
    ops = []
    for i in range(8):
        m = rng.randbelow(N) if i else 0
        r = rng.rand_coprime(N)
        c = gm.paillier_encrypt(N, m, r)
        b = rng.randbelow(gm.SECP256K1_N)
        hm = gm.paillier_homo_mult(N, b, c)
        m2 = rng.randbelow(N)
        c2 = gm.paillier_encrypt(N, m2, rng.rand_coprime(N))
        ha = gm.paillier_homo_add(N, c, c2)
        assert gm.paillier_decrypt(N, lam, c) == m
        assert gm.paillier_decrypt(N, lam, hm) == (m * b) % N
        assert gm.paillier_decrypt(N, lam, ha) == (m + m2) % N
        ops.append({"m": h(m), "r": h(r), "c": h(c), "b": h(b), "homo_mult": h(hm), "c2": h(c2), "m2": h(m2),
                    "homo_add": h(ha)})
    assert N2 > 0
    return ops


def gen_safeprimes():
    """First safe primes of small bit lengths from the tss-lib candidate stream."""
    out = []
    for bits, seed in ((64, 11), (128, 12), (256, 13), (512, 14)):
        idx, p, q = sp.first_safe_primes(seed, bits, 1)[0]
        out.append({"bits": bits, "seed": seed, "index": idx, "p": h(p), "q": h(q)})
    return out


def main():
    c_lib = cc.load_c_oracle()
    print("cross-check backends: gmp=%s openssl=%s c=%s" % (cc._gmp is not None, cc._ssl is not None, c_lib is not None))
    key = gen_key()
    print("key ok", key["gen_seconds"], "s")
    json.dump({"seed": SEED_VEC, "vectors": gen_modexp(key, c_lib)}, open(os.path.join(OUT, "modexp_vectors.json"), "w"),
              indent=0)
    json.dump({"cases": gen_go_semantics(key)}, open(os.path.join(OUT, "go_exp_semantics.json"), "w"), indent=1)
    json.dump({"seed": SEED_KEY + 100, "ops": gen_paillier(key)}, open(os.path.join(OUT, "paillier_vectors.json"), "w"),
              indent=0)
    json.dump({"primes": gen_safeprimes()}, open(os.path.join(OUT, "safeprime_vectors.json"), "w"), indent=1)
    print("done")


if __name__ == "__main__":
    main()
