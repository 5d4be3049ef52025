"""Lane-accurate Python model of the wave-cooperative radix-2^28 Montgomery
multiply used by mpcium_amd/csrc/mpcx_kernels.hip (design check, not shipped).
G groups x P lanes x K slots; lane p of a group holds digits p*K .. p*K+K-1."""
import random
D = 28; M28 = (1 << D) - 1; U64 = (1 << 64) - 1

def to_digits(v, L): return [(v >> (D * i)) & M28 for i in range(L)]
def from_digits(ds): return sum(d << (D * i) for i, d in enumerate(ds))

def montmul_model(A, B, Nd, n0inv, P, K, mid):
    """A, B, Nd: lists (per lane) of K digits for ONE group. Returns per-lane acc (K each)."""
    L = P * K
    acc = [[0] * K for _ in range(P)]
    bdig = [B[i // K][i % K] for i in range(L)]
    maxv = 0
    for o in range(P):
        for u in range(K):
            i = o * K + u
            bi = bdig[i]
            for p in range(P):
                for k in range(K):
                    acc[p][k] += A[p][k] * bi
            m = ((acc[0][0] & 0xFFFFFFFF) * n0inv) & M28
            for p in range(P):
                for k in range(K):
                    acc[p][k] += m * Nd[p][k]
                    maxv = max(maxv, acc[p][k])
                    assert acc[p][k] <= U64, "overflow"
            assert acc[0][0] & M28 == 0
            # fold slot0 hi into slot1, cross-lane the lo part
            lo = [0] * P
            for p in range(P):
                a0 = acc[p][0]
                if K > 1:
                    acc[p][1] += a0 >> D
                lo[p] = a0 & M28
            new = []
            for p in range(P):
                inc = lo[p + 1] if p + 1 < P else 0
                if K == 1:  # carry goes to the next lane's slot (only P==... not used)
                    raise NotImplementedError
                new.append(acc[p][1:] + [inc])
            acc = new
        if o == mid:
            carries = [[a >> D for a in row] for row in acc]
            for p in range(P):
                for k in range(K):
                    acc[p][k] &= M28
            for p in range(P):
                for k in range(K):
                    if k > 0:
                        acc[p][k] += carries[p][k - 1]
                    elif p > 0:
                        acc[p][k] += carries[p - 1][K - 1]
            assert carries[P - 1][K - 1] == 0
    return acc, maxv

def normalize2(acc, P, K):
    for _ in range(2):
        carries = [[a >> D for a in row] for row in acc]
        acc = [[a & M28 for a in row] for row in acc]
        for p in range(P):
            for k in range(K):
                if k > 0: acc[p][k] += carries[p][k - 1]
                elif p > 0: acc[p][k] += carries[p - 1][K - 1]
        assert carries[P - 1][K - 1] == 0
    return acc

def check(P, K, nbits, trials=3, worst=False):
    L = P * K
    R = 1 << (D * L)
    rng = random.Random(P * 1000 + K)
    mid = P // 2 - 1
    worstmax = 0
    for t in range(trials):
        N = rng.getrandbits(nbits) | 1 | (1 << (nbits - 1))
        assert R > 4 * N
        n0inv = (-pow(N, -1, 1 << D)) % (1 << D)
        Nd = to_digits(N, L)
        if worst:
            a = 2 * N - 1; b = 2 * N - 1
        else:
            a = rng.randrange(2 * N); b = rng.randrange(2 * N)
        A = [[to_digits(a, L)[p * K + k] for k in range(K)] for p in range(P)]
        B = [[to_digits(b, L)[p * K + k] for k in range(K)] for p in range(P)]
        Ndl = [[Nd[p * K + k] for k in range(K)] for p in range(P)]
        acc, maxv = montmul_model(A, B, Ndl, n0inv, P, K, mid)
        worstmax = max(worstmax, maxv)
        acc = normalize2(acc, P, K)
        digs = [acc[p][k] for p in range(P) for k in range(K)]
        assert max(digs) <= M28 + (1 << 10)
        T = from_digits(digs)
        assert T == (a * b * pow(R, -1, N)) % N or T == (a * b * pow(R, -1, N)) % N + N, (P, K)
        assert T < 2 * N
    return worstmax.bit_length()

for (P, K, nb) in [(7, 21, 4096), (3, 25, 2048), (2, 19, 1024), (4, 5, 500)]:
    print(P, K, nb, "max acc bits", check(P, K, nb), "worst-case", check(P, K, nb, 1, True))
