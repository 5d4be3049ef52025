"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (mpcium_amd/) never imports it.

Pure-Python restatement of the tss-lib v2.0.2 keygen / reshare proofs whose
cost is modular exponentiation ("up:" =
github.com/bnb-chain/tss-lib/v2, pinned at /root/reference/go.mod:10, source
absent from the image):

* up:crypto/dlnproof/proof.go   NewDLNProof / (*Proof).Verify, Iterations = 128
  (keygen round 1 proves h2 = h1^alpha and h1 = h2^beta over the node's N~;
  up:ecdsa/keygen/dln_verifier.go verifies the peers' proofs)
* up:crypto/modproof/proof.go   NewProof / (*ProofMod).Verify, Iterations = 80
  (Paillier-Blum modulus proof of the node's Paillier N, CGGMP Fig. 16)
* up:crypto/facproof/proof.go   NewProof / (*ProofFac).Verify
  (no-small-factor proof of N0 = the Paillier N over the verifier's N^ = N~,
  s = h1, t = h2, CGGMP Fig. 28)

Randomness comes from a per-proof Reader in the order the upstream functions
draw it; the draw order, hash inputs and validity checks are restated from the
published algorithm (upstream, verify): parity with tss-lib itself is UNPINNED
(SURVEY.md 8(c)); the GPU path is checked bit-exactly against THIS
restatement.  Deliberately not restated (unverifiable detail): FacProof's
range checks on z1, z2.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

from . import tss_ref as T

Q = T.SECP_N
DLN_ITERATIONS = 128
MOD_ITERATIONS = 80

_pw = pow


def _exp(x: int, y: int, m: int) -> Optional[int]:
    """Go (*Int).Exp(x, y, m) with a negative y through ModInverse (None = nil)."""
    if y < 0:
        if math.gcd(x % m, m) != 1:
            return None
        return _pw(pow(x, -1, m), -y, m)
    return _pw(x, y, m)


# ----------------------------------------------------------------- Jacobi
def jacobi(a: int, n: int) -> int:
    """math/big Jacobi(x, y) for odd y > 0."""
    if n <= 0 or n % 2 == 0:
        raise ValueError("Jacobi: n must be odd and positive")
    a %= n
    j = 1
    while a:
        while a % 2 == 0:
            a //= 2
            if n % 8 in (3, 5):
                j = -j
        a, n = n, a
        if a % 4 == 3 and n % 4 == 3:
            j = -j
        a %= n
    return j if n == 1 else 0


def get_random_quadratic_non_residue(rd: T.Reader, n: int) -> int:
    """common.GetRandomQuadraticNonResidue(rand, n): GetRandomPositiveInt(n)
    until Jacobi(w, n) == -1 (upstream, verify)."""
    while True:
        w = T.get_random_positive_int(rd, n)
        if jacobi(w, n) == -1:
            return w


# ----------------------------------------------------------------- DLN
@dataclass
class DLNProof:
    Alpha: List[int]
    T: List[int]


def dln_prove(h1: int, h2: int, x: int, p: int, q: int, N: int, rd: T.Reader) -> DLNProof:
    """NewDLNProof(h1, h2, x, p, q, N, rand): alpha_i = h1^a_i mod N, a_i < pq;
    c = SHA512_256i(h1, h2, N, alpha...); t_i = a_i + c_i x mod pq."""
    pq = p * q
    a = []
    alpha = []
    for _ in range(DLN_ITERATIONS):
        ai = T.get_random_positive_int(rd, pq)
        a.append(ai)
        alpha.append(_pw(h1, ai, N))
    c = T.sha512_256i(h1, h2, N, *alpha)
    t = [(a[i] + ((c >> i) & 1) * x) % pq for i in range(DLN_ITERATIONS)]
    return DLNProof(alpha, t)


def dln_verify(pf: DLNProof, h1: int, h2: int, N: int) -> bool:
    """(*Proof).Verify(h1, h2, N)."""
    if pf is None or N <= 0:
        return False
    h1_, h2_ = h1 % N, h2 % N
    if not (1 < h1_ < N) or not (1 < h2_ < N) or h1_ == h2_:
        return False
    for v in list(pf.T) + list(pf.Alpha):
        if not (1 < v % N < N):
            return False
    c = T.sha512_256i(h1, h2, N, *pf.Alpha)
    for i in range(DLN_ITERATIONS):
        ci = (c >> i) & 1
        if _pw(h1, pf.T[i], N) != pf.Alpha[i] * _pw(h2, ci, N) % N:
            return False
    return True


# ----------------------------------------------------------------- Mod (Paillier-Blum)
@dataclass
class ModProof:
    W: int
    X: List[int]
    A: int
    B: int
    Z: List[int]


def _mod_challenges(session: bytes, W: int, N: int) -> List[int]:
    Y: List[int] = []
    for i in range(MOD_ITERATIONS):
        ei = T.sha512_256i_tagged(session, W, N, *Y[:i])
        Y.append(T.rejection_sample(N, ei))
    return Y


def mod_prove(session: bytes, N: int, P: int, Qf: int, rd: T.Reader) -> ModProof:
    """modproof.NewProof(Session, N, P, Q, rand) (CGGMP Fig. 16)."""
    phi = (P - 1) * (Qf - 1)
    W = get_random_quadratic_non_residue(rd, N)
    Y = _mod_challenges(session, W, N)
    inv_n = pow(N, -1, phi)
    A = 1 << MOD_ITERATIONS
    B = 1 << MOD_ITERATIONS
    expo = ((phi + 4) >> 3)
    expo = expo * expo % phi
    X, Z = [0] * MOD_ITERATIONS, [0] * MOD_ITERATIONS
    for i in range(MOD_ITERATIONS):
        for j in range(4):
            a, b = j & 1, (j & 2) >> 1
            yi = Y[i]
            if a:
                yi = (-yi) % N
            if b:
                yi = W * yi % N
            if jacobi(yi, P) == 1 and jacobi(yi, Qf) == 1:
                X[i] = _pw(yi, expo, N)
                Z[i] = _pw(Y[i], inv_n, N)
                A |= a << i
                B |= b << i
                break
    return ModProof(W, X, A, B, Z)


def mod_verify(pf: ModProof, session: bytes, N: int) -> bool:
    """(*ProofMod).Verify(Session, N): a probable-prime N is rejected first
    (Go: N.ProbablyPrime(30), restated in safeprime_ref.probably_prime with Go's
    math/rand Miller-Rabin bases and the extra strong Lucas test)."""
    from .safeprime_ref import probably_prime
    if pf is None or N <= 0 or N % 2 == 0:
        return False
    if probably_prime(N, 30):
        return False
    if jacobi(pf.W, N) != -1:
        return False
    if not T.is_in_interval(pf.W, N):
        return False
    for v in list(pf.X) + list(pf.Z):
        if not T.is_in_interval(v, N):
            return False
    if pf.A.bit_length() != MOD_ITERATIONS + 1 or pf.B.bit_length() != MOD_ITERATIONS + 1:
        return False
    Y = _mod_challenges(session, pf.W, N)
    for i in range(MOD_ITERATIONS):
        if _pw(pf.Z[i], N, N) != Y[i]:
            return False
        a, b = (pf.A >> i) & 1, (pf.B >> i) & 1
        right = Y[i]
        if a:
            right = (-right) % N
        if b:
            right = pf.W * right % N
        if _pw(pf.X[i], 4, N) != right:
            return False
    return True


def mod_proof_for_prime(session: bytes, p: int, rd: T.Reader) -> ModProof:
    """A ModProof for a PRIME p = 3 (mod 4) that satisfies every equation of
    the verifier (Z_i^p = Y_i by Fermat, X_i^4 = (-1)^a W^b Y_i via the
    ((p+1)/4)^2 power of a quadratic residue): only the N.ProbablyPrime(30)
    check rejects it. Test helper for that check in isolation."""
    assert p % 4 == 3
    W = get_random_quadratic_non_residue(rd, p)
    Y = _mod_challenges(session, W, p)
    e4 = ((p + 1) // 4) ** 2 % (p - 1)
    A = B = 1 << MOD_ITERATIONS
    X, Z = [], []
    for i, y in enumerate(Y):
        for j in range(4):
            a, b = j & 1, (j & 2) >> 1
            yi = (-y) % p if a else y
            yi = W * yi % p if b else yi
            if jacobi(yi, p) == 1:
                X.append(pow(yi, e4, p))
                Z.append(y % p)
                A |= a << i
                B |= b << i
                break
    return ModProof(W, X, A, B, Z)


# ----------------------------------------------------------------- Fac (no small factor)
@dataclass
class FacProof:
    P: int
    Q: int
    A: int
    B: int
    T: int
    Sigma: int
    Z1: int
    Z2: int
    W1: int
    W2: int
    V: int  # may be negative (sigma - nu*N0p < 0)


def fac_prove(session: bytes, N0: int, NCap: int, s: int, t: int, N0p: int, N0q: int, rd: T.Reader) -> FacProof:
    """facproof.NewProof(Session, ec, N0, NCap, s, t, N0p, N0q, rand) (CGGMP Fig. 28)."""
    q = Q
    q3 = q ** 3
    sqrtN0 = math.isqrt(N0)
    q3sqrtN0 = q3 * sqrtN0
    alpha = T.get_random_positive_int(rd, q3sqrtN0)
    beta = T.get_random_positive_int(rd, q3sqrtN0)
    mu = T.get_random_positive_int(rd, q * NCap)
    nu = T.get_random_positive_int(rd, q * NCap)
    sigma = T.get_random_positive_int(rd, q * N0 * NCap)
    r = T.get_random_positive_relatively_prime_int(rd, q3 * N0 * NCap)
    x = T.get_random_positive_int(rd, q3 * NCap)
    y = T.get_random_positive_int(rd, q3 * NCap)
    M = NCap
    P = _pw(s, N0p, M) * _pw(t, mu, M) % M
    Qc = _pw(s, N0q, M) * _pw(t, nu, M) % M
    A = _pw(s, alpha, M) * _pw(t, x, M) % M
    B = _pw(s, beta, M) * _pw(t, y, M) % M
    Tc = _pw(Qc, alpha, M) * _pw(t, r, M) % M
    e = T.rejection_sample(q, T.sha512_256i_tagged(session, N0, NCap, s, t, P, Qc, A, B, Tc, sigma))
    z1 = e * N0p + alpha
    z2 = e * N0q + beta
    w1 = e * mu + x
    w2 = e * nu + y
    v = e * (sigma - nu * N0p) + r
    return FacProof(P, Qc, A, B, Tc, sigma, z1, z2, w1, w2, v)


def fac_verify(pf: FacProof, session: bytes, N0: int, NCap: int, s: int, t: int) -> bool:
    """(*ProofFac).Verify(Session, ec, N0, NCap, s, t)."""
    if pf is None or N0 <= 0 or NCap <= 0:
        return False
    # z1, z2 range, CGGMP Fig. 28 form (+-sqrt(N0) 2^(l+eps) with 2^(l+eps) ->
    # q^3 plus the e*N0p slack of an honest response); tss-lib's exact
    # expression is not in this image: parity of the bound is unpinned
    zbound = (Q ** 3 + 2 * Q) * math.isqrt(N0)
    if not (0 <= pf.Z1 <= zbound and 0 <= pf.Z2 <= zbound):
        return False
    for v in (pf.P, pf.Q, pf.A, pf.B, pf.T):
        if not T.is_in_interval(v, NCap):
            return False
    e = T.rejection_sample(Q, T.sha512_256i_tagged(session, N0, NCap, s, t, pf.P, pf.Q, pf.A, pf.B, pf.T,
                                                   pf.Sigma))
    M = NCap
    if _pw(s, pf.Z1, M) * _pw(t, pf.W1, M) % M != pf.A * _pw(pf.P, e, M) % M:
        return False
    if _pw(s, pf.Z2, M) * _pw(t, pf.W2, M) % M != pf.B * _pw(pf.Q, e, M) % M:
        return False
    R = _pw(s, N0, M) * _exp(t, pf.Sigma, M) % M
    tv = _exp(t, pf.V, M)
    if tv is None:
        return False
    return _pw(pf.Q, pf.Z1, M) * tv % M == pf.T * _pw(R, e, M) % M
