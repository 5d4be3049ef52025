"""CPU tests: the oracle (test infrastructure) against the committed golden
vectors, which were cross-checked at generation time against GMP, OpenSSL
and the C restatement of Go expNNMontgomery (tests/golden/gen_golden.py)."""
import math
import subprocess

import pytest

from conftest import H, ROOT, load_golden
from oracle import crosscheck as cc
from oracle import gomath as gm
from oracle import safeprime_ref as sp


@pytest.fixture(scope="module")
def c_oracle():
    subprocess.run(["make", "-s", "-C", f"{ROOT}/oracle"], check=True)
    lib = cc.load_c_oracle()
    assert lib is not None
    return lib


def test_golden_vectors_python(golden_modexp):
    assert len(golden_modexp) > 60
    for v in golden_modexp:
        x, y, m, z = H(v["x"]), H(v["y"]), H(v["m"]), H(v["z"])
        assert gm.go_exp(x, y, m) == z, v["name"]


def test_golden_vectors_c_restatement(golden_modexp, c_oracle):
    for v in golden_modexp:
        x, y, m, z = H(v["x"]), H(v["y"]), H(v["m"]), H(v["z"])
        assert cc.c_expnn(c_oracle, x, y, m) == z, v["name"]


def test_golden_vectors_gmp_openssl_sample(golden_modexp):
    for v in golden_modexp[::5]:
        x, y, m, z = H(v["x"]), H(v["y"]), H(v["m"]), H(v["z"])
        for f in (cc.gmp_powm, cc.openssl_mod_exp):
            r = f(x, y, m)
            assert r is None or r == z, (f.__name__, v["name"])


def test_c_restatement_forced_montgomery_matches(c_oracle):
    # the Montgomery path Go takes for multi-word exponents, on odd moduli of every class
    import ctypes
    rng = gm.CounterDRBG(7)
    for bits in (1024, 2048, 4096):
        m = rng.randbits(bits) | 1 | (1 << (bits - 1))
        n = bits // 32
        x, y = rng.randbelow(m), rng.randbits(300)
        out = (ctypes.c_uint32 * n)()
        rc = c_oracle.gomodexp_montgomery(out, cc._words(x, n), n, cc._words(y, 10), 10, cc._words(m, n), n)
        assert rc == 0 and cc._from_words(out, n) == pow(x, y, m)


def test_go_exp_semantics():
    for c in load_golden("go_exp_semantics.json")["cases"]:
        assert gm.go_exp(H(c["x"]), H(c["y"]), H(c["m"])) == H(c["z"])
    assert gm.go_exp(2, -1, 8) is None  # Go returns nil: 2 has no inverse mod 8
    assert gm.go_exp(3, -1, 8) == 3
    assert gm.go_exp(-3, 5, 7) == pow(-3, 5, 7)


def test_paillier_restatement(paillier_key):
    N, lam = paillier_key["N"], paillier_key["LambdaN"]
    P, Q = paillier_key["P"], paillier_key["Q"]
    assert P * Q == N and N.bit_length() == 2048
    assert lam == (P - 1) * (Q - 1) // math.gcd(P - 1, Q - 1)
    for op in load_golden("paillier_vectors.json")["ops"]:
        m, r, c = H(op["m"]), H(op["r"]), H(op["c"])
        assert gm.paillier_encrypt(N, m, r) == c
        assert gm.paillier_decrypt(N, lam, c) == m
        assert gm.paillier_homo_mult(N, H(op["b"]), c) == H(op["homo_mult"])
        assert gm.paillier_homo_add(N, c, H(op["c2"])) == H(op["homo_add"])
    with pytest.raises(gm.ErrMessageTooLong):
        gm.paillier_encrypt(N, N, 1)
    with pytest.raises(gm.ErrMessageMalFormed):
        gm.paillier_decrypt(N, lam, P)  # gcd(c, N^2) != 1


def test_paillier_key_primes_are_safe(paillier_key):
    for k in ("P", "Q"):
        p = paillier_key[k]
        assert p.bit_length() == 1024
        assert pow(2, p - 1, p) == 1 and sp.miller_rabin((p - 1) // 2, 8)


def test_safeprime_stream_vectors():
    for v in load_golden("safeprime_vectors.json")["primes"]:
        if v["bits"] > 256:
            continue  # covered by the fixture itself; keep the CPU suite fast
        idx, p, q = sp.first_safe_primes(v["seed"], v["bits"], 1)[0]
        assert (idx, p, q) == (v["index"], H(v["p"]), H(v["q"]))


def test_candidate_layout():
    # tss-lib masking: top two bits set, odd, qBitLen bits (before the delta walk)
    q = sp.candidate_from_bytes(b"\x00" * 128, 1023)
    assert q.bit_length() == 1023 and q & 1 and (q >> 1021) == 3
    for p in sp.SMALL_PRIMES:
        assert q % p != 0
