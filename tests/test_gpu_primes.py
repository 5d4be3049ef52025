"""GPU tests of the safe-prime / primality path (A2, A7, A11, A12) against the
oracle (oracle/safeprime_ref.py, pinned to OEIS A217719 / A001262 in
tests/test_primes_cpu.py):

* k_mr (base 2) on the base-2 strong pseudoprimes and Carmichael numbers;
* k_lucas on the extra strong Lucas pseudoprimes, primes and composites;
* ProbablyPrime decisions (small-prime exits, MR, Lucas; a 2048-bit N);
* one safe-prime step (device DRBG, sieve, Pocklington, ride-along base-2
  strong test) against the oracle walk of the same stream;
* the first two 1024-bit safe primes of a stream and a whole
  GeneratePreParams, bit-exact against tests/golden/preparams_vectors.json,
  with the stream drawn on the GPU and through a host reader callback.
"""
import math

import pytest

from conftest import H, load_golden
from oracle import safeprime_ref as S

pytestmark = pytest.mark.gpu

A217719 = [989, 3239, 5777, 10877, 27971, 29681, 30739, 31631, 39059, 72389, 73919, 75077]
A001262 = [2047, 3277, 4033, 4681, 8321, 15841, 29341, 42799, 49141, 52633, 65281, 74665, 80581, 85489, 88357,
           90751]
CARMICHAEL = [561, 1105, 1729, 2465, 2821, 6601, 8911, 10585, 15841, 29341, 41041, 46657, 52633, 62745, 63973]
# the GPU sieve's exact trial division primes (mpcx_api.cpp TrialTables)
TRIAL = [t for t in range(59, 2048, 2) if all(t % d for d in range(3, math.isqrt(t) + 1, 2))]


class FastDRBG:
    """The CounterDRBG byte stream (oracle/gomath.py), read in large chunks."""

    def __init__(self, seed):
        import hashlib
        self._h = hashlib.sha256
        self.prefix = b"mpcx-drbg" + (seed & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")
        self.pos = 0

    def read(self, n):
        c0, c1 = self.pos // 32, (self.pos + n + 31) // 32
        out = b"".join(self._h(self.prefix + c.to_bytes(8, "little")).digest() for c in range(c0, c1))
        s = self.pos % 32
        self.pos += n
        return out[s:s + n]


@pytest.fixture(scope="module")
def h(gpu):
    from mpcium_amd import host
    host.init(0)
    return host


def test_mr_base2_pseudoprimes(gpu):
    ns = A001262 + CARMICHAEL + [3825123056546413051, (1 << 521) - 1, 101, 7919]
    got = gpu.mr_batch(ns, [2] * len(ns))
    assert got == [S.strong_probable_prime(n, 2) for n in ns]
    assert all(got[:len(A001262)])


@pytest.mark.parametrize("coop", [1, 0])
def test_fermat_and_mr_kernels_both_geometries(gpu, coop):
    """The cooperative kernels (k_prime2c: 2 lanes per candidate; k_mrc: 16
    lanes per test, 4-bit window) and the thread-per-candidate ones give the
    same decisions as CPython pow on primes, pseudoprimes, Carmichael numbers
    and random odd candidates of 3..1024 bits (bit lengths mixed in one wave)."""
    import random
    rng = random.Random(11 + coop)
    ns = A001262 + CARMICHAEL + [5, 7, 9, 15, 101, 7919, 3825123056546413051, (1 << 521) - 1, (1 << 607) - 1]
    ns += [rng.getrandbits(rng.randrange(3, 1025)) | 1 for _ in range(150)]
    ns += [(rng.getrandbits(1023) | (1 << 1023) | 1) for _ in range(50)]
    ns = [n for n in ns if n >= 5]
    key = load_golden("paillier_key_2048.json")
    ns += [int(key["P"], 16), int(key["Q"], 16)]
    gpu.set_option("prime_coop", coop)
    try:
        assert gpu.fermat2_batch(ns) == [pow(2, n - 1, n) == 1 for n in ns]
        bases = [rng.randrange(2, n - 1) if n > 4 else 2 for n in ns]
        assert gpu.mr_batch(ns, bases) == [S.strong_probable_prime(n, a) for n, a in zip(ns, bases)]
        assert gpu.mr_batch(ns, [2] * len(ns)) == [S.strong_probable_prime(n, 2) for n in ns]
    finally:
        gpu.set_option("prime_coop", 1)


@pytest.mark.parametrize("coop", [1, 0])
def test_lucas_kernel(gpu, coop):
    """k_lucasc (16 lanes per candidate) and k_lucas (thread per candidate)
    against the oracle: the extra strong Lucas pseudoprimes pass (as in Go),
    primes pass, composites of mixed sizes fail."""
    import random
    rng = random.Random(3 + coop)
    ns = A217719 + [3825123056546413051, (1 << 521) - 1, (1 << 607) - 1, 1000003, 999983 * 1000003]
    ns += [rng.getrandbits(1023) | (1 << 1022) | 1 for _ in range(40)]
    ns += [rng.getrandbits(rng.randrange(5, 1024)) | 1 for _ in range(40)]
    ns += [(1 << 89) - 1, (1 << 127) - 1, 2 ** 64 - 59]
    runs, Ps = [], []
    for n in ns:
        if n < 5:
            continue
        r, P = S.lucas_param(n)
        if r == 1:
            runs.append(n)
            Ps.append(P)
    gpu.set_option("prime_coop", coop)
    try:
        got = gpu.lucas_batch(runs, Ps)
    finally:
        gpu.set_option("prime_coop", 1)
    assert got == [S.probably_prime_lucas(n) for n in runs]
    assert all(got[:len(A217719)])  # the pseudoprimes pass, as in Go


def _prime_near(rng, bits):
    small = [p for p in range(3, 2000, 2) if all(p % d for d in range(3, int(p ** 0.5) + 1, 2))]
    n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    while any(n % p == 0 for p in small) or not S.probably_prime(n, 5):
        n += 2
    return n


def test_lucas_kernel_wide(gpu):
    """The wide Lucas geometry (16 x 5 digits, candidates up to 2048 bits):
    a batch with a candidate above 1024 bits runs every candidate there --
    the extra strong Lucas pseudoprimes, 1024-bit and 2048-bit composites,
    Mersenne prime 2^1279 - 1 and generated 1536/2048-bit primes, against the
    oracle."""
    import random
    rng = random.Random(11)
    key = load_golden("paillier_key_2048.json")
    ns = A217719 + [(1 << 1279) - 1, int(key["N"], 16), int(key["P"], 16), _prime_near(rng, 1536),
                    _prime_near(rng, 2048), _prime_near(rng, 1025)]
    ns += [rng.getrandbits(2048) | (1 << 2047) | 1 for _ in range(12)]
    ns += [rng.getrandbits(rng.randrange(1025, 2049)) | 1 for _ in range(12)]
    ns += [rng.getrandbits(1024) | 1 for _ in range(8)]
    runs, Ps = [], []
    for n in ns:
        r, P = S.lucas_param(n)
        if r == 1:
            runs.append(n)
            Ps.append(P)
    got = gpu.lucas_batch(runs, Ps)
    want = [S.probably_prime_lucas(n) for n in runs]
    assert got == want
    assert sum(want) >= len(A217719) + 4  # pseudoprimes and primes pass


def test_probably_prime_decisions(h):
    import random
    rng = random.Random(4)
    ns = A217719 + A001262 + CARMICHAEL + [3825123056546413051, 2, 3, 4, 61, 63, 64, 65, 67]
    ns += [(1 << 521) - 1, (1 << 607) - 1, ((1 << 89) - 1) * ((1 << 107) - 1)]
    ns += [rng.getrandbits(512) | 1 for _ in range(30)]
    key = load_golden("paillier_key_2048.json")
    ns += [int(key["N"], 16), int(key["P"], 16)]  # 2048-bit composite and a 1024-bit prime
    ns += [(1 << 1279) - 1, _prime_near(random.Random(12), 2048)]  # wide: MR with Go's bases, then Lucas
    got = h.probably_prime(ns, 20)
    assert got == [S.probably_prime(n, 20) for n in ns]


def test_safeprime_step_matches_oracle_walk(gpu):
    """4,096 candidates of a CounterDRBG stream at 1024 bits: the device DRBG,
    sieve and Pocklington passes equal the oracle's candidate walk, and q of
    some passes riding along get the oracle's base-2 verdicts."""
    seed, count, qb = 0x5AFE7, 4096, 1023
    nb = (qb + 7) // 8
    off = 3 * 1000 * nb  # an arbitrary stream position
    rng = FastDRBG(seed)
    rng.pos = off
    raw = rng.read(count * nb)
    want = []
    for i in range(count):
        q = S.candidate_from_bytes(raw[i * nb:(i + 1) * nb], qb)
        p = 2 * q + 1
        if q.bit_length() == qb and all(q % t and p % t for t in TRIAL) and pow(2, p - 1, p) == 1:
            want.append((i, p))
    ns, passes, _ = gpu.safeprime_step(seed, off, count, qb)
    assert passes == want
    assert 0 < ns < count
    qs = [p >> 1 for _, p in want] + [(1 << 521) - 1, 2047 * 3]
    _, _, sp = gpu.safeprime_step(seed, off, 0, qb, sprp_q=qs)
    assert sp == [S.strong_probable_prime(q, 2) for q in qs]


def test_first_1024_bit_safe_primes_golden(h):
    g = load_golden("preparams_vectors.json")["safe_primes_1024"]
    res, st = h.safe_primes(1024, 2, seed=g["seed"])
    assert [(i, p, q) for p, q, i in res] == [(v["index"], H(v["p"]), H(v["q"])) for v in g["primes"]]
    assert st["lucas_tests"] >= 2


def test_generate_preparams_golden_gpu_stream_and_host_reader(h):
    """GeneratePreParams on one stream, bit-exact in all 12 fields: once with
    the candidates drawn on the GPU (CounterDRBG seed), once through a host
    reader callback serving the same bytes -- equal only if each search gives
    back exactly the bytes after its last accepted candidate."""
    g = load_golden("preparams_vectors.json")["preparams"]
    want = {k: H(v) for k, v in g.items() if k not in ("seed", "consumed_bytes")}
    pp, _ = h.generate_preparams(seed=g["seed"])
    assert pp == want
    rd = FastDRBG(g["seed"])
    pp2, _ = h.generate_preparams(seed=0, rand_fn=lambda _ctx, buf, n: _fill(buf, rd.read(n)))
    assert pp2 == want


def _fill(buf, data):
    import ctypes
    ctypes.memmove(buf, data, len(data))
