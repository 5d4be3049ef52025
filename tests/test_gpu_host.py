"""GPU parity tests of the C++ host mirror (ModInt.Exp, crypto/paillier,
safe primes, GeneratePreParams) against the oracle and golden fixtures."""
import math
import random

import pytest

from conftest import H, load_golden
from oracle import gomath as gm
from oracle import safeprime_ref as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def host(gpu):
    from mpcium_amd import host as h
    h.init(0)
    return h


def test_modint_go_semantics_golden(host):
    for c in load_golden("go_exp_semantics.json")["cases"]:
        x, y, m = H(c["x"]), H(c["y"]), H(c["m"])
        if m % 2 == 0:
            continue  # math/big's even-modulus path stays with the caller
        assert host.modint_exp(m, [x], [y], shared=False)[0] == H(c["z"]), c


def test_modint_go_semantics_random(host, paillier_key):
    N = paillier_key["N"]
    rng = random.Random(8)
    for m in (N * N, N, 65537, 3, 1):
        xs = [rng.randrange(-m * 3, m * 3) for _ in range(30)] + [0, 1, -1, m, -m]
        ys = [rng.randrange(-2 ** 300, 2 ** 300) for _ in xs]
        got = host.modint_exp(m, xs, ys, shared=False)
        assert got == [gm.go_exp(x, y, m) for x, y in zip(xs, ys)], m
        got = host.modint_exp(m, xs, -5)
        assert got == [gm.go_exp(x, -5, m) for x in xs]


def test_modint_rejects_even_modulus(host):
    from mpcium_amd.mpcx import MpcxError
    with pytest.raises(MpcxError):
        host.modint_exp(1 << 64, [3], 5)


def test_paillier_golden(host, paillier_key):
    N, lam, P, Q = paillier_key["N"], paillier_key["LambdaN"], paillier_key["P"], paillier_key["Q"]
    sk = host.PrivateKey(N, lam, P, Q)
    ops = load_golden("paillier_vectors.json")["ops"]
    ms = [H(o["m"]) for o in ops]
    rs = [H(o["r"]) for o in ops]
    cs, err = sk.encrypt(ms, rs)
    assert err == [0] * len(ops) and cs == [H(o["c"]) for o in ops]
    hm, err = sk.homo_mult([H(o["b"]) for o in ops], cs)
    assert err == [0] * len(ops) and hm == [H(o["homo_mult"]) for o in ops]
    ha, err = sk.homo_add(cs, [H(o["c2"]) for o in ops])
    assert err == [0] * len(ops) and ha == [H(o["homo_add"]) for o in ops]
    dm, err = sk.decrypt(cs + hm + ha)
    assert err == [0] * (3 * len(ops))
    assert dm == ms + [m * H(o["b"]) % N for m, o in zip(ms, ops)] + [(m + H(o["m2"])) % N for m, o in zip(ms, ops)]


def test_paillier_errors(host, paillier_key):
    N, lam, P, Q = paillier_key["N"], paillier_key["LambdaN"], paillier_key["P"], paillier_key["Q"]
    sk = host.PrivateKey(N, lam, P, Q)
    N2 = N * N
    _, err = sk.encrypt([N, -1, 5], [3, 3, 3])
    assert err == [host.ERR_MESSAGE_TOO_LONG, host.ERR_MESSAGE_TOO_LONG, 0]
    _, err = sk.homo_mult([5, N, 5], [N2, 7, -1])
    assert err == [1, 1, 1]
    _, err = sk.homo_add([N2, 5], [5, N2 + 1])
    assert err == [1, 1]
    _, err = sk.decrypt([N2, -3, P * 5, Q, 0, 12345])
    assert err == [1, 1, 2, 2, 2, 0]
    # a key without its factors: tss-lib's lambda formula, gcd checked up front
    m, err = host.PrivateKey(N, lam, 0, 0).decrypt([N2, P * 5, Q * 7, 0, 12345])
    assert err == [1, 2, 2, 2, 0]
    assert m[4] == gm.paillier_decrypt(N, lam, 12345)


def test_paillier_random_roundtrip(host, paillier_key):
    N, lam, P, Q = paillier_key["N"], paillier_key["LambdaN"], paillier_key["P"], paillier_key["Q"]
    sk = host.PrivateKey(N, lam, P, Q)
    rng = gm.CounterDRBG(1234)
    n = 200
    ms = [rng.randbelow(N) for _ in range(n)]
    rs = [rng.rand_coprime(N) for _ in range(n)]
    cs, _ = sk.encrypt(ms, rs)
    assert cs == [gm.paillier_encrypt(N, m, r) for m, r in zip(ms, rs)]
    dm, _ = sk.decrypt(cs)
    assert dm == ms


def test_config1_full_batch_matches_c_oracle(host, paillier_key):
    """BASELINE config 1 at its stated size: one batch of 1,024 Encrypt +
    HomoMult ops (the bench's paillier line: m < N, r < N, b < q) through
    crypto/paillier's host mirror, EVERY output compared with tss-lib's
    formulas evaluated by the C restatement of Go's expNN (Gamma^m as a full
    Exp, as tss-lib computes it, not the GPU's 1 + mN shortcut)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import crosscheck as cc
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    N = paillier_key["N"]
    N2 = N * N
    pk = host.PublicKey(N)
    rng = random.Random(0x6D706331)  # bench.py paillier_line's draws
    n = 1024
    ms = [rng.randrange(N) for _ in range(n)]
    rs = [rng.randrange(1, N) for _ in range(n)]
    bs = [rng.randrange(gm.SECP256K1_N) for _ in range(n)]
    cs, err = pk.encrypt(ms, rs)
    assert err == [0] * n
    hm, err = pk.homo_mult(bs, cs)
    assert err == [0] * n

    def want(i):
        c = cc.c_expnn(lib, N + 1, ms[i], N2) * cc.c_expnn(lib, rs[i], N, N2) % N2
        return c, cc.c_expnn(lib, c, bs[i], N2)

    with ThreadPoolExecutor(8) as ex:  # ctypes releases the GIL
        ref = list(ex.map(want, range(n)))
    assert cs == [c for c, _ in ref]
    assert hm == [h for _, h in ref]


def test_safe_primes_match_oracle_stream(host):
    for v in load_golden("safeprime_vectors.json")["primes"]:
        got, stats = host.safe_primes(v["bits"], 1, seed=v["seed"])
        p, q, idx = got[0]
        assert (p, q, idx) == (H(v["p"]), H(v["q"]), v["index"]), v["bits"]
        assert stats["fermat_tests"] > 0


def test_safe_primes_small_multi(host):
    got, _ = host.safe_primes(128, 3, seed=77)
    want = sp.first_safe_primes(77, 128, 3)
    assert [(p, q, i) for p, q, i in got] == [(p, q, i) for i, p, q in want]


def test_generate_preparams_relations(host):
    pp, stats = host.generate_preparams(seed=0x6D706333)
    N, P, Q = pp["N"], pp["P"], pp["Q"]
    assert N == P * Q and N.bit_length() == 2048
    assert abs(P - Q).bit_length() >= 1024 - 3
    assert pp["PhiN"] == (P - 1) * (Q - 1)
    assert pp["LambdaN"] == pp["PhiN"] // math.gcd(P - 1, Q - 1)
    p, q = pp["p"], pp["q"]
    assert pp["NTildei"] == (2 * p + 1) * (2 * q + 1)
    for sp_ in (P, Q, 2 * p + 1, 2 * q + 1):
        assert pow(2, sp_ - 1, sp_) == 1 and sp.miller_rabin((sp_ - 1) // 2, 4)
    Nt = pp["NTildei"]
    assert pp["H2i"] == pow(pp["H1i"], pp["Alpha"], Nt)
    assert pp["Alpha"] * pp["Beta"] % (p * q) == 1
    assert math.gcd(pp["H1i"], Nt) == 1
    assert stats["candidates"] > 0


_SIEVE_PRIMES = [v for v in range(59, 2048, 2) if all(v % d for d in range(3, int(v ** 0.5) + 1, 2))]


@pytest.mark.parametrize("q_bits", [63, 255, 511, 1023])
def test_gpu_sieve_fermat_matches_oracle(gpu, q_bits):
    """mpcx_safeprime_sieve_fermat vs the oracle candidate layout
    (oracle/safeprime_ref.candidate_from_bytes), exact trial division of q and
    2q+1 by 59..2039, and pow(2, p-1, p) for every survivor."""
    nb = (q_bits + 7) // 8
    count = 3000
    raw = gm.CounterDRBG(0x51E7E + q_bits).read(nb * count)
    # a few crafted candidates: all-ones, all-zeros, a top-bit-overflowing walk
    raw = b"\xff" * nb + b"\x00" * nb + raw[2 * nb:]
    got = gpu.safeprime_sieve_fermat(raw, q_bits)
    want = []
    for i in range(count):
        q = sp.candidate_from_bytes(raw[i * nb:(i + 1) * nb], q_bits)
        if q.bit_length() != q_bits:
            continue
        p = 2 * q + 1
        if any(q % t == 0 or p % t == 0 for t in _SIEVE_PRIMES):
            continue
        want.append((i, pow(2, p - 1, p) == 1))
    assert got == want
    assert any(ok for _, ok in got) or q_bits == 1023


def test_safe_primes_1024_gpu_sieve(host):
    """One GeneratePreParams-size search through the GPU sieve path: p = 2q+1
    with p, q passing Fermat spot checks and the index's stream bytes giving
    q.  Bit-exact first indices at 1024 bits (every earlier candidate
    rejected) are pinned by tests/test_gpu_primes.py against the golden
    stream vector."""
    got, stats = host.safe_primes(1024, 2, seed=0x5AFE)
    nb = 128
    for p, q, idx in got:
        assert p == 2 * q + 1 and p.bit_length() == 1024
        assert all(pow(a, q - 1, q) == 1 for a in (2, 3, 5, 7)) and pow(2, p - 1, p) == 1
        raw = gm.CounterDRBG(0x5AFE).read(nb * (idx + 1))[idx * nb:]
        assert sp.candidate_from_bytes(raw, 1023) == q
    assert got[0][2] < got[1][2]
    assert stats["fermat_tests"] > 0 and stats["candidates"] >= got[1][2]


@pytest.mark.parametrize("bits,batch", [(128, 1000), (100, 777), (1024, 0)])
def test_safe_prime_batches_sharded_equal_stream_order(host, bits, batch):
    """Config-3 sharding: batches of the seeked CounterDRBG stream
    (mpcxh_safe_prime_batch) dealt to G ranks round-robin give the same first
    safe primes as the single-stream search, for G = 1, 2, 3 (ranks emulated in
    one process; the gather itself is covered by tests/test_shard_gloo.py).
    Batch sizes whose byte length is not a multiple of the DRBG block exercise
    the mid-block seek."""
    from mpcium_amd.shard import safe_primes_sharded
    num = 3 if bits < 1024 else 2
    seed = 0x5AFE + bits
    want, _ = host.safe_primes(bits, num, seed=seed)
    cache = {}

    def fn(b):
        if b not in cache:
            cache[b], _ = host.safe_prime_batch(bits, seed, b, batch)
        return cache[b]

    for world in (1, 2, 3):
        found = []
        for r in range(1 << 12):   # all ranks' round-r batches, then the gather
            for g in range(world):
                found += fn(r * world + g)
            if len(found) >= num:
                break
        assert sorted(found, key=lambda t: t[2])[:num] == want, world
    assert safe_primes_sharded(num, 0, 1, fn) == want
