"""GPU parity tests: every result through libmpcx.so (C-ABI) must equal the
oracle bit for bit (integer arithmetic, no tolerance)."""
import random

import numpy as np
import pytest

from conftest import H
from oracle import gomath as gm

pytestmark = pytest.mark.gpu


def by_modulus(vectors):
    groups = {}
    for v in vectors:
        groups.setdefault(H(v["m"]), []).append(v)
    return groups


def test_golden_vectors_gpu(gpu, golden_modexp):
    for m, vs in by_modulus(golden_modexp).items():
        if m % 2 == 0:
            continue
        mod = gpu.Modulus(m)
        # per-operand exponents in one batch
        xs = [H(v["x"]) for v in vs]
        ys = [H(v["y"]) for v in vs]
        lim = 1 << (32 * mod.class_words)
        xs_in = [x if x < lim else x % m for x in xs]
        got = mod.exp(xs_in, ys)
        for v, g in zip(vs, got):
            assert g == H(v["z"]), v["name"]
        # and each one with a shared exponent
        for v, x in zip(vs, xs_in):
            assert mod.exp([x], H(v["y"]))[0] == H(v["z"]), v["name"] + " shared"
        mod.release()


@pytest.mark.parametrize("bits", [64, 1024, 2048, 4096])
def test_ragged_batches_shared_exponent(gpu, bits):
    rng = random.Random(bits)
    m = rng.getrandbits(bits) | 1 | (1 << (bits - 1))
    mod = gpu.Modulus(m)
    e = rng.getrandbits(bits // 2) | 1
    for count in (1, mod.G - 1, mod.G, mod.G + 1, 3 * mod.G + 5):
        xs = [rng.randrange(m) for _ in range(count)]
        assert mod.exp(xs, e) == [pow(x, e, m) for x in xs], count
    mod.release()


def test_empty_batch(gpu):
    mod = gpu.Modulus((1 << 127) - 1)
    assert mod.exp([], 5) == []


def test_zero_and_small_exponents(gpu, paillier_key):
    N2 = paillier_key["N"] ** 2
    mod = gpu.Modulus(N2)
    rng = random.Random(3)
    xs = [rng.randrange(N2) for _ in range(20)] + [0, 1, N2 - 1]
    for e in (0, 1, 2, 3, 15, 16, 17, (1 << 64) - 1, 1 << 64):
        assert mod.exp(xs, e) == [gm.go_exp(x, e, N2) for x in xs], e


def test_shared_exponent_N_config2_sample(gpu, paillier_key):
    """Config-2 shape (x^N mod N^2) at a reduced count; full size runs in bench.py."""
    N = paillier_key["N"]
    N2 = N * N
    mod = gpu.Modulus(N2)
    rng = gm.CounterDRBG(0x6D706332)
    xs = [rng.randbelow(N2) for _ in range(2 * mod.G * 7 + 3)]
    got = mod.exp(xs, N)
    for x, g in zip(xs, got):
        assert g == pow(x, N, N2)


def test_config2_full_batch_digest(gpu, paillier_key):
    """The whole config-2 batch (bench.py's 65,536 synthetic bases, x^N mod
    N^2) through the host-buffer entry: SHA-256 of all outputs equals the
    digest computed by the oracle's C restatement of Go's expNN
    (tests/golden/batch_digest.json, tests/golden/gen_batch_digest.py)."""
    import hashlib
    import json
    import os
    from conftest import GOLDEN
    gd = json.load(open(os.path.join(GOLDEN, "batch_digest.json")))
    N = paillier_key["N"]
    N2 = N * N
    mod = gpu.Modulus(N2)
    words = gd["words"]
    rng = np.random.default_rng(gd["seed"])  # bench.synth_bases
    x = rng.integers(0, 1 << 32, size=(gd["count"], words), dtype=np.uint64).astype(np.uint32)
    top = (N2 >> (32 * (words - 1))) & 0xFFFFFFFF
    x[:, words - 1] = x[:, words - 1] % max(top, 1)
    e = gpu.int_to_words(N, gpu.nwords(N))
    out = mod.exp_words(x, e, shared=True, out_words=words)
    assert int.from_bytes(out[0].astype("<u4").tobytes(), "little") == int(gd["first_output"], 16)
    assert hashlib.sha256(out.astype("<u4").tobytes()).hexdigest() == gd["sha256"]


def test_per_operand_exponents_mixed_lengths(gpu, paillier_key):
    N = paillier_key["N"]
    N2 = N * N
    mod = gpu.Modulus(N2)
    rng = random.Random(11)
    xs = [rng.randrange(N2) for _ in range(40)]
    ys = [rng.getrandbits(rng.choice([0, 1, 5, 256, 768, 2048, 4096])) for _ in xs]
    assert mod.exp(xs, ys) == [pow(x, y, N2) for x, y in zip(xs, ys)]


def test_fermat2_batch(gpu, paillier_key):
    rng = random.Random(5)
    P, Q = paillier_key["P"], paillier_key["Q"]
    cands = [P, Q, (P - 1) // 2 * 2 + 1]
    cands += [rng.getrandbits(1024) | 1 | (1 << 1023) for _ in range(100)]
    cands += [rng.getrandbits(b) | 1 | (1 << (b - 1)) for b in (8, 64, 300, 512, 1000) for _ in range(3)]
    cands += [101, 65537, 561, 1105]  # primes and Carmichael numbers (which pass base 2)
    got = gpu.fermat2_batch(cands)
    assert got == [pow(2, p - 1, p) == 1 for p in cands]
    assert got[0] and got[1]


def test_rejects_even_and_oversized_modulus(gpu):
    with pytest.raises(gpu.MpcxError):
        gpu.Modulus(1 << 100)
    with pytest.raises(gpu.MpcxError):
        gpu.Modulus((1 << 4097) + 1)


def test_exp_mul_and_mulmod(gpu, paillier_key):
    N = paillier_key["N"]
    N2 = N * N
    rng = random.Random(21)
    for m in (N2, N, paillier_key["P"]):
        mod = gpu.Modulus(m)
        n = mod.G + 3
        xs = [rng.randrange(m) for _ in range(n)]
        cs = [rng.randrange(m) for _ in range(n)]
        assert mod.mulmod(xs, cs) == [x * c % m for x, c in zip(xs, cs)]
        assert mod.exp_mul(xs, N, cs) == [c * pow(x, N, m) % m for x, c in zip(xs, cs)]
        es = [rng.getrandbits(rng.choice([0, 3, 256, 2048])) for _ in xs]
        assert mod.exp_mul(xs, es, cs) == [c * pow(x, e, m) % m for x, e, c in zip(xs, es, cs)]
        assert mod.exp_mul(xs, 0, cs) == [c % m for c in cs]
        mod.release()


@pytest.mark.parametrize("geom", [1, 2, 3, 4, 5, 6])
def test_each_geometry_forced(gpu, paillier_key, geom):
    """Every geometry of the 2048-bit (1, 3, 5) and 4096-bit (2, 4, 6) classes:
    quad-per-operand, lane-pair (5: the 2048-bit main geometry), narrow and
    mid layouts, each forced for shared and per-operand exponents and the
    fused multiplier."""
    N = paillier_key["N"]
    m = N * N if geom in (2, 4, 6) else N
    rng = random.Random(geom)
    gpu.set_option("force_geom", geom)
    try:
        mod = gpu.Modulus(m)
        xs = [rng.randrange(m) for _ in range(40)]
        es = [rng.getrandbits(rng.choice([1, 17, 256, 2048])) for _ in xs]
        assert mod.exp(xs, N) == [pow(x, N, m) for x in xs]
        assert mod.exp(xs, es) == [pow(x, e, m) for x, e in zip(xs, es)]
        cs = [rng.randrange(m) for _ in xs]
        assert mod.exp_mul(xs, es, cs) == [c * pow(x, e, m) % m for x, e, c in zip(xs, es, cs)]
        mod.release()
    finally:
        gpu.set_option("force_geom", -1)


@pytest.mark.parametrize("force", [-1, 5])
def test_lane_pair_geometry_limits(gpu, paillier_key, force):
    """Geometry 5 (2 x 37 digits, R = 2^2072) serves moduli below 2^2070 with
    operands below 2^2072; a wider modulus of the class (up to 2080 bits), or
    bases / multipliers of 2072..2080 bits (allowed by the class width, not
    reduced by the caller), must run on geometry 1 instead -- default and
    forced alike -- with results equal to pow()."""
    N = paillier_key["N"]
    rng = random.Random(2072)
    gpu.set_option("force_geom", force)
    try:
        for m in (N, (1 << 2079) + rng.getrandbits(2078) | 1, (1 << 2069) + 1 + 2 * rng.getrandbits(2060)):
            mod = gpu.Modulus(m)
            top = 1 << (32 * mod.class_words)
            xs = [rng.randrange(m) for _ in range(33)] + [top - 1 - rng.getrandbits(20) for _ in range(3)]
            es = [rng.getrandbits(rng.choice([1, 64, 2048])) for _ in xs]
            assert mod.exp(xs, N) == [pow(x, N, m) for x in xs], m.bit_length()
            assert mod.exp(xs, es) == [pow(x, e, m) for x, e in zip(xs, es)], m.bit_length()
            cs = [rng.randrange(m) for _ in xs[:-1]] + [top - 5]
            assert mod.exp_mul(xs, es, cs) == [c * pow(x, e, m) % m for x, e, c in zip(xs, es, cs)]
            mod.release()
    finally:
        gpu.set_option("force_geom", -1)


@pytest.mark.parametrize("m_kind", ["N2", "N", "p"])
def test_fixed_window_widths_agree(gpu, paillier_key, m_kind):
    """Per-operand exponents above 1024 bits take a 5-bit fixed window (Go's is
    4 bits): both widths give pow's results on exponents around the window
    and word boundaries, with and without the fused multiplier."""
    N = paillier_key["N"]
    m = {"N2": N * N, "N": N, "p": paillier_key["P"]}[m_kind]
    rng = random.Random(77)
    lens = [320, 321, 1023, 1024, 1025, 1026, 1029, 1030, 2047, 2048, 2049, 2050, 3000, 4095, 4096, 4100]
    xs = [rng.randrange(m) for _ in lens * 2]
    es = [rng.getrandbits(b) | (1 << (b - 1)) for b in lens] + [(1 << b) - 1 for b in lens]
    cs = [rng.randrange(m) for _ in xs]
    want = [pow(x, e, m) for x, e in zip(xs, es)]
    mod = gpu.Modulus(m)
    try:
        for w in (4, 5):
            gpu.set_option("fixed_window", w)
            assert mod.exp(xs, es) == want, w
            assert mod.exp_mul(xs, es, cs) == [c * v % m for c, v in zip(cs, want)], w
    finally:
        gpu.set_option("fixed_window", 5)
        mod.release()


def test_split_plan_large_batch(gpu, paillier_key):
    """A batch that spans >1 round of resident wavefronts takes the main +
    narrow split; spot-check results across the split point."""
    N = paillier_key["N"]
    N2 = N * N
    mod = gpu.Modulus(N2)
    count = 30000  # ~1.1 rounds of the main 4096-bit geometry on MI355X
    rng = np.random.default_rng(3)
    words = mod.class_words
    B = rng.integers(0, 1 << 32, size=(count, words), dtype=np.uint64).astype(np.uint32)
    B[:, -1] %= (N2 >> (32 * (words - 1)))
    E = gpu.int_to_words(N, gpu.nwords(N))
    out = mod.exp_words(B, E, True)
    idx = list(range(0, count, 997)) + [count - 1]
    xs = gpu.words_to_ints(B[idx])
    zs = gpu.words_to_ints(out[idx])
    assert zs == [pow(x, N, N2) for x in xs]


SCHED_EXPONENTS = [1, 2, 3, 5, 7, 31, 32, 33, 63, (1 << 64) - 1, 1 << 64, (1 << 64) + 1, 0xAAAA_AAAA_AAAA_AAAA_AAAA,
                   (1 << 2047) | 1, (1 << 1000) | (1 << 500) | (1 << 37), (1 << 4900) - 1]


@pytest.mark.parametrize("width", [0, 1, 2, 3, 4, 5, 6])
def test_shared_exponent_window_schedules(gpu, paillier_key, width):
    """Shared exponents take the device-built sliding-window schedule
    (k_expsched; width capped by the "sched_width" option, 0 = Go's fixed
    window): sparse, dense, word-boundary and long exponents, with and
    without the fused multiplier, in the 4096-bit and 2048-bit classes."""
    N = paillier_key["N"]
    rng = random.Random(100 + width)
    gpu.set_option("sched_width", width)
    try:
        for m in (N * N, N):
            mod = gpu.Modulus(m)
            xs = [rng.randrange(m) for _ in range(mod.G + 1)] + [0, 1, m - 1]
            for e in SCHED_EXPONENTS + [N, rng.getrandbits(2048), rng.getrandbits(300)]:
                assert mod.exp(xs, e) == [pow(x, e, m) for x in xs], (width, m.bit_length(), e.bit_length())
            cs = [rng.randrange(m) for _ in xs]
            assert mod.exp_mul(xs, N - 1, cs) == [c * pow(x, N - 1, m) % m for x, c in zip(xs, cs)]
            mod.release()
    finally:
        gpu.set_option("sched_width", 6)


@pytest.mark.parametrize("wbits", [12, 11, 8])
def test_fixed_base_tables(gpu, paillier_key, wbits):
    """Fixed-base comb (h1^a h2^b mod N~ shape) with w-bit windows (12: the
    default; 11: windows straddling 32-bit words at varying offsets; 8: round
    2's): one and two bases, with and without a multiplier, zero/one/boundary
    exponents, ragged batches, and exponents past the table rejected."""
    N = paillier_key["N"]
    rng = random.Random(77 + wbits)
    mod = gpu.Modulus(N)
    h1, h2 = rng.randrange(N), rng.randrange(N)
    gpu.set_option("fb_window", wbits)
    try:
        f1, f2 = gpu.FixedBase(mod, h1, 2816), gpu.FixedBase(mod, h2, 300)
    finally:
        gpu.set_option("fb_window", 12)
    cap = lambda b: -(-b // wbits) * wbits  # noqa: E731
    assert f1.max_exp_bits == cap(2816) and f2.max_exp_bits == cap(300)
    for count in (1, mod.G - 1, mod.G + 1, 3 * mod.G + 5):
        a = [rng.getrandbits(rng.choice([0, 1, 8, 9, 256, 2048, 2816])) for _ in range(count)]
        b = [rng.getrandbits(rng.choice([0, 7, 64, 300])) for _ in range(count)]
        assert gpu.fixedbase_exp([f1], [a]) == [pow(h1, x, N) for x in a], count
        want = [pow(h1, x, N) * pow(h2, y, N) % N for x, y in zip(a, b)]
        assert gpu.fixedbase_exp([f1, f2], [a, b]) == want, count
        cs = [rng.randrange(N) for _ in range(count)]
        assert gpu.fixedbase_exp([f1, f2], [a, b], cs) == [c * w % N for c, w in zip(cs, want)], count
    edge = [0, 1, 255, 256, 4095, 4096, (1 << 2816) - 1, 1 << 2815, (1 << cap(2816)) - 1]
    assert gpu.fixedbase_exp([f1], [edge]) == [pow(h1, x, N) for x in edge]
    with pytest.raises(gpu.MpcxError):
        gpu.fixedbase_exp([f2], [[1 << cap(300)]])
    # a multiplier up to the class width (2080 bits) is served by a full-width table
    big = (1 << 2075) + 3
    assert gpu.fixedbase_exp([f1], [[5]], [big]) == [big * pow(h1, 5, N) % N]
    # N~-shape modulus from the node fixtures and the 1024-bit class
    for m in (paillier_key["P"], rng.getrandbits(1500) | 1 | (1 << 1499)):
        md = gpu.Modulus(m)
        fb = gpu.FixedBase(md, 3, 600)
        es = [rng.getrandbits(600) for _ in range(70)]
        assert gpu.fixedbase_exp([fb], [es]) == [pow(3, e, m) for e in es]
        fb.release()
        md.release()
    f2.release()
    f1.release()
    mod.release()


@pytest.mark.parametrize("split", [1, 2, 4, 0])
def test_fixed_base_window_split(gpu, paillier_key, split):
    """Option "fb_split": 1, 2 or 4 wavefronts share one comb operand's
    windows (j = w, w + S, ...; partials multiplied in by wave 0), 0 picks by
    launch size. Products equal pow() for one and two bases, multipliers,
    exponents shorter than S windows, zero exponents, ragged batches, and the
    multi-segment launch; the 1024-bit class (thread-per-operand layout) too."""
    N, P = paillier_key["N"], paillier_key["P"]
    rng = random.Random(900 + split)
    mod, modp = gpu.Modulus(N), gpu.Modulus(P)
    h1, h2, hp = rng.randrange(N), rng.randrange(N), rng.randrange(P)
    f1, f2, fp = gpu.FixedBase(mod, h1, 2816), gpu.FixedBase(mod, h2, 2048), gpu.FixedBase(modp, hp, 1024)
    gpu.set_option("fb_split", split)
    try:
        for count in (1, 17, 100, 3000):
            a = [rng.getrandbits(rng.choice([0, 5, 12, 13, 30, 2048, 2816])) for _ in range(count)]
            b = [rng.getrandbits(rng.choice([0, 24, 2048])) for _ in range(count)]
            cs = [rng.randrange(N) for _ in range(count)]
            assert gpu.fixedbase_exp([f1], [a]) == [pow(h1, x, N) for x in a], count
            want = [c * pow(h1, x, N) * pow(h2, y, N) % N for c, x, y in zip(cs, a, b)]
            assert gpu.fixedbase_exp([f1, f2], [a, b], cs) == want, count
            ep = [rng.getrandbits(rng.choice([0, 11, 1024])) for _ in range(count)]
            assert gpu.fixedbase_exp([fp], [ep]) == [pow(hp, x, P) for x in ep], count
        got = gpu.fixedbase_multi([([f1], [[3, 0, 1 << 2000]], None), ([f2, f1], [[7] * 40, list(range(40))], None)])
        assert got[0] == [pow(h1, e, N) for e in (3, 0, 1 << 2000)]
        assert got[1] == [pow(h2, 7, N) * pow(h1, e, N) % N for e in range(40)]
    finally:
        gpu.set_option("fb_split", 0)
        for f in (fp, f2, f1):
            f.release()
        modp.release()
        mod.release()
    with pytest.raises(gpu.MpcxError):
        gpu.set_option("fb_split", 3)


def test_fixed_base_multi_batch(gpu, paillier_key):
    """mpcx_fixedbase_multi_batch: comb groups of two different 2048-bit moduli
    (other tables, one and two bases, with and without multipliers, an empty
    and a one-operand group) as the segments of ONE launch equal pow(); groups
    of two classes are refused; a group's exponent past its table fails."""
    N, P = paillier_key["N"], paillier_key["P"]
    rng = random.Random(4242)
    m2 = rng.getrandbits(2046) | 1 | (1 << 2045)
    mods = [gpu.Modulus(N), gpu.Modulus(m2)]
    hs = [(rng.randrange(N), rng.randrange(N)), (rng.randrange(m2), rng.randrange(m2))]
    fbs = [(gpu.FixedBase(mods[0], hs[0][0], 2816), gpu.FixedBase(mods[0], hs[0][1], 2816)),
           (gpu.FixedBase(mods[1], hs[1][0], 1024), gpu.FixedBase(mods[1], hs[1][1], 1024))]
    groups, want = [], []
    for k, (count, nb, mul) in enumerate([(70, 2, False), (0, 1, False), (33, 1, True), (1, 2, True), (200, 2, True)]):
        mi = k % 2
        m = mods[mi].m
        bits = 2816 if mi == 0 else 1024
        es = [[rng.getrandbits(rng.choice([0, 5, bits // 2, bits])) for _ in range(count)] for _ in range(nb)]
        cs = [rng.randrange(m) for _ in range(count)] if mul else None
        groups.append((list(fbs[mi][:nb]), es, cs))
        w = []
        for i in range(count):
            v = cs[i] if mul else 1
            for t in range(nb):
                v = v * pow(hs[mi][t], es[t][i], m) % m
            w.append(v)
        want.append(w)
    assert gpu.fixedbase_multi(groups) == want
    pm = gpu.Modulus(P)
    fp = gpu.FixedBase(pm, 5, 64)
    with pytest.raises(gpu.MpcxError):  # 1024-bit and 2048-bit classes in one launch
        gpu.fixedbase_multi([([fp], [[3]], None), ([fbs[0][0]], [[3]], None)])
    with pytest.raises(gpu.MpcxError):
        gpu.fixedbase_multi([([fbs[1][0]], [[1 << 1100]], None)])
    fp.release()
    pm.release()
    for pair in fbs:
        for f in pair:
            f.release()
    for md in mods:
        md.release()


def test_multi_batch_groups_of_different_moduli(gpu):
    """mpcx_modexp_multi_batch: groups of three different 4096-bit moduli (the
    nodes' N^2), shared and per-operand exponents, with and without
    multipliers, an empty group and a one-operand group, in ONE launch; every
    result equals pow(). Groups of two classes are refused."""
    import json
    import os
    import random
    from conftest import GOLDEN
    from mpcium_amd import mpcx
    mpcx.init(0)
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    Ns = [int(n["N"], 16) for n in d["nodes"]]
    rng = random.Random(0x3A17)
    mods = [mpcx.Modulus(N * N) for N in Ns]
    try:
        groups, want = [], []
        for k, (N, mod) in enumerate(zip(Ns, mods)):
            N2 = N * N
            xs = [rng.randrange(N2) for _ in range(37 + 50 * k)]
            es = [rng.getrandbits(rng.choice([256, 768, 2048])) for _ in xs]
            ms = [rng.randrange(N2) for _ in xs]
            groups += [(mod, xs, N, None), (mod, xs, es, ms), (mod, xs[:1], es[:1], None), (mod, [], N, None)]
            want += [[pow(x, N, N2) for x in xs], [m * pow(x, e, N2) % N2 for x, e, m in zip(xs, es, ms)],
                     [pow(xs[0], es[0], N2)], []]
        got = mpcx.modexp_multi(groups)
        assert got == want
        modn = mpcx.Modulus(Ns[0])
        try:
            with pytest.raises(mpcx.MpcxError):
                mpcx.modexp_multi([(mods[0], [3], 5, None), (modn, [3], 5, None)])
        finally:
            modn.release()
    finally:
        for m in mods:
            m.release()


def test_kernel_stats_count_launches_and_work(gpu, paillier_key):
    """mpcx_kernel_stats: the launches of a shared-exponent batch are timed and
    carry the Go-equivalent work (E + ceil(E/4)) 2 L^2 per operand."""
    from mpcium_amd import mpcx
    N = paillier_key["N"]
    N2 = N * N
    mod = gpu.Modulus(N2)
    rng = random.Random(11)
    xs = [rng.randrange(N2) for _ in range(3000)]
    mpcx.set_option("kernel_stats", 1)
    try:
        mpcx.kernel_stats(reset=True)
        got = mod.exp(xs, N)
        ks = mpcx.kernel_stats(reset=True)
    finally:
        mpcx.set_option("kernel_stats", 0)
    assert got[:4] == [pow(x, N, N2) for x in xs[:4]]
    assert ks["enabled"] == 1
    mods = [k for k in ks["kernels"] if k["kind"].startswith("modexp")]
    assert sum(k["operands"] for k in mods) == len(xs)
    E, L = N.bit_length(), 128
    assert sum(k["alg_macs"] for k in mods) == pytest.approx(len(xs) * (E + (E + 3) // 4) * 2 * L * L, rel=1e-6)
    assert all(k["kernel_ms"] > 0 for k in mods)
    assert 0 < ks["busy_ms"] <= sum(k["kernel_ms"] for k in ks["kernels"]) + 1e-3
    # disabled: nothing is collected
    mod.exp(xs[:64], N)
    assert mpcx.kernel_stats()["kernels"] == []
