"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (mpcium_amd/) never imports it.

Pure-Python restatement of tss-lib v2.0.2's MtA / MtAwc sub-protocol of GG18
ECDSA signing:

* up:crypto/mta/share_protocol.go   AliceInit, BobMid, BobMidWC, AliceEnd, AliceEndWC
* up:crypto/mta/range_proof.go      ProveRangeAlice, (*RangeProofAlice).Verify
* up:crypto/mta/proofs.go           ProveBob, ProveBobWC, (*ProofBob).Verify,
                                    (*ProofBobWC).Verify
* up:crypto/paillier/paillier.go    EncryptAndReturnRandomness, HomoMult,
                                    HomoAdd, Decrypt

Exponentiations are CPython ``pow`` (negative exponents through the modular
inverse, as Go (*Int).Exp); randomness is drawn from a per-session Reader in
the order the upstream functions draw it; hashing and random helpers are in
tss_ref.py.  The order of random draws, the hash inputs and the validity checks
of the Verify functions are restated from the published tss-lib algorithm
(upstream, verify): parity of this restatement with tss-lib itself is
UNPINNED (no Go toolchain, tss-lib absent -- SURVEY.md 8(c)); the build's GPU
path is checked bit-exactly against THIS restatement.

Where Go would dereference a nil Exp result (c^-e with c not invertible) and
panic, the restatement returns False (verification failure).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Tuple

from . import tss_ref as T

Q = T.SECP_N  # ec.Params().N for tss.EC() = secp256k1

# Modular exponentiation used by the restatement: CPython pow by default;
# use_go_modexp() switches to the C restatement of Go's nat.expNN
# (oracle/gomodexp.c) -- the CPU baseline of bench.py's signing line.
_pw = pow


def use_go_modexp(word_bits: int = 32) -> bool:
    """Route exponentiations through the C restatement of Go's expNN
    (word_bits 64: Go's amd64 word size, the CPU baseline)."""
    global _pw
    from .crosscheck import c_expnn, load_c_oracle
    lib = load_c_oracle(word_bits)
    if lib is None:
        return False
    _pw = lambda x, y, m: c_expnn(lib, x % m, y, m)  # noqa: E731
    return True


class ErrMessageTooLong(ValueError):
    pass


class ErrMessageMalFormed(ValueError):
    pass


def _exp(x: int, y: int, m: int) -> Optional[int]:
    """common.ModInt(m).Exp(x, y) = Go (*Int).Exp(x, y, m); None where Go returns nil."""
    if y < 0:
        if math.gcd(x % m, m) != 1:
            return None
        return _pw(pow(x, -1, m), -y, m)
    return _pw(x, y, m)


# ----------------------------------------------------------------- Paillier
def encrypt_and_return_randomness(rd: T.Reader, N: int, m: int) -> Tuple[int, int]:
    """PublicKey.EncryptAndReturnRandomness(rand, m)."""
    if m < 0 or m >= N:
        raise ErrMessageTooLong()
    x = T.get_random_positive_relatively_prime_int(rd, N)
    N2 = N * N
    c = _pw(N + 1, m, N2) * _pw(x, N, N2) % N2
    return c, x


def homo_mult(N: int, m: int, c1: int) -> int:
    N2 = N * N
    if m < 0 or m >= N or c1 < 0 or c1 >= N2:
        raise ErrMessageTooLong()
    return _pw(c1, m, N2)


def homo_add(N: int, c1: int, c2: int) -> int:
    N2 = N * N
    if c1 < 0 or c1 >= N2 or c2 < 0 or c2 >= N2:
        raise ErrMessageTooLong()
    return c1 * c2 % N2


def decrypt(N: int, lam: int, c: int) -> int:
    N2 = N * N
    if c < 0 or c >= N2:
        raise ErrMessageTooLong()
    if math.gcd(c, N2) > 1:
        raise ErrMessageMalFormed()
    lc = (_pw(c, lam, N2) - 1) // N
    lg = (_pw(N + 1, lam, N2) - 1) // N
    return lc * pow(lg, -1, N) % N


# ----------------------------------------------------------------- proofs
@dataclass
class RangeProofAlice:
    Z: int
    U: int
    W: int
    S: int
    S1: int
    S2: int


@dataclass
class ProofBob:
    Z: int
    ZPrm: int
    T: int
    V: int
    W: int
    S: int
    S1: int
    S2: int
    T1: int
    T2: int
    U: T.Point = None  # ProofBobWC.U (None for the plain ProofBob)


def prove_range_alice(pkN: int, c: int, NTilde: int, h1: int, h2: int, m: int, r: int,
                      rd: T.Reader) -> RangeProofAlice:
    """ProveRangeAlice(ec, pk, c, NTilde, h1, h2, m, r, rand) (up:crypto/mta/range_proof.go)."""
    q3 = Q ** 3
    qNt, q3Nt = Q * NTilde, q3 * NTilde
    alpha = T.get_random_positive_int(rd, q3)
    beta = T.get_random_positive_relatively_prime_int(rd, pkN)
    gamma = T.get_random_positive_int(rd, q3Nt)
    rho = T.get_random_positive_int(rd, qNt)
    z = _pw(h1, m, NTilde) * _pw(h2, rho, NTilde) % NTilde
    N2 = pkN * pkN
    u = _pw(pkN + 1, alpha, N2) * _pw(beta, pkN, N2) % N2
    w = _pw(h1, alpha, NTilde) * _pw(h2, gamma, NTilde) % NTilde
    e = T.rejection_sample(Q, T.sha512_256i(pkN, pkN + 1, c, z, u, w))
    s = _pw(r, e, pkN) * beta % pkN
    return RangeProofAlice(z, u, w, s, e * m + alpha, e * rho + gamma)


def verify_range_alice(pf: RangeProofAlice, pkN: int, NTilde: int, h1: int, h2: int, c: int) -> bool:
    """(*RangeProofAlice).Verify(ec, pk, NTilde, h1, h2, c)."""
    if pf is None or None in (pf.Z, pf.U, pf.W, pf.S, pf.S1, pf.S2):
        return False
    N2 = pkN * pkN
    q3 = Q ** 3
    if not (T.is_in_interval(pf.Z, NTilde) and T.is_in_interval(pf.U, N2) and T.is_in_interval(pf.W, NTilde)
            and T.is_in_interval(pf.S, pkN)):
        return False
    if math.gcd(pf.Z, NTilde) != 1 or math.gcd(pf.U, N2) != 1 or math.gcd(pf.W, NTilde) != 1 \
            or math.gcd(pf.S, pkN) != 1:
        return False
    if pf.S1 > q3:
        return False
    e = T.rejection_sample(Q, T.sha512_256i(pkN, pkN + 1, c, pf.Z, pf.U, pf.W))
    c_me = _exp(c, -e, N2)
    if c_me is None:
        return False
    prod = _pw(pkN + 1, pf.S1, N2) * _pw(pf.S, pkN, N2) % N2 * c_me % N2
    if pf.U != prod:
        return False
    z_me = _exp(pf.Z, -e, NTilde)
    if z_me is None:
        return False
    prod = _pw(h1, pf.S1, NTilde) * _pw(h2, pf.S2, NTilde) % NTilde * z_me % NTilde
    return pf.W == prod


def prove_bob_wc(session: bytes, pkN: int, NTilde: int, h1: int, h2: int, c1: int, c2: int, x: int, y: int,
                 r: int, X: T.Point, rd: T.Reader) -> ProofBob:
    """ProveBobWC(Session, ec, pk, NTilde, h1, h2, c1, c2, x, y, r, X, rand)
    (up:crypto/mta/proofs.go); X = None is ProveBob."""
    q3, q7 = Q ** 3, Q ** 7
    qNt, q3Nt = Q * NTilde, q3 * NTilde
    alpha = T.get_random_positive_int(rd, q3)
    rho = T.get_random_positive_int(rd, qNt)
    sigma = T.get_random_positive_int(rd, qNt)
    tau = T.get_random_positive_int(rd, q3Nt)
    rho_prm = T.get_random_positive_int(rd, q3Nt)
    beta = T.get_random_positive_relatively_prime_int(rd, pkN)
    gamma = T.get_random_positive_int(rd, q7)
    u = T.scalar_base_mult(alpha) if X is not None else None
    Nt = NTilde
    z = _pw(h1, x, Nt) * _pw(h2, rho, Nt) % Nt
    z_prm = _pw(h1, alpha, Nt) * _pw(h2, rho_prm, Nt) % Nt
    t = _pw(h1, y, Nt) * _pw(h2, sigma, Nt) % Nt
    N2 = pkN * pkN
    v = _pw(c1, alpha, N2) * _pw(pkN + 1, gamma, N2) % N2 * _pw(beta, pkN, N2) % N2
    w = _pw(h1, gamma, Nt) * _pw(h2, tau, Nt) % Nt
    if X is None:
        eh = T.sha512_256i_tagged(session, pkN, pkN + 1, c1, c2, z, z_prm, t, v, w)
    else:
        eh = T.sha512_256i_tagged(session, pkN, pkN + 1, X[0], X[1], c1, c2, u[0], u[1], z, z_prm, t, v, w)
    e = T.rejection_sample(Q, eh)
    s = _pw(r, e, pkN) * beta % pkN
    return ProofBob(z, z_prm, t, v, w, s, e * x + alpha, e * rho + rho_prm, e * y + gamma, e * sigma + tau, u)


def verify_bob_wc(pf: ProofBob, session: bytes, pkN: int, NTilde: int, h1: int, h2: int, c1: int, c2: int,
                  X: T.Point) -> bool:
    """(*ProofBobWC).Verify / (*ProofBob).Verify (X = None) (up:crypto/mta/proofs.go)."""
    if pf is None or None in (pf.Z, pf.ZPrm, pf.T, pf.V, pf.W, pf.S, pf.S1, pf.S2, pf.T1, pf.T2):
        return False
    if X is not None and not T.ec_on_curve(pf.U):
        return False
    N2 = pkN * pkN
    q3, q7 = Q ** 3, Q ** 7
    Nt = NTilde
    for v_, bound in ((pf.Z, Nt), (pf.ZPrm, Nt), (pf.T, Nt), (pf.V, N2), (pf.W, Nt), (pf.S, pkN)):
        if not T.is_in_interval(v_, bound) or math.gcd(v_, bound) != 1:
            return False
    # s1 <= q^3 and t1 <= q^7 (the Alpha-Rays range checks of tss-lib v2: BobMid
    # draws betaPrm < q^5 and ProveBob gamma < q^7, so an honest t1 = e*betaPrm +
    # gamma < q^6 + q^7 passes except with probability ~1/q).
    if pf.S1 > q3 or pf.T1 > q7:
        return False
    if X is None:
        eh = T.sha512_256i_tagged(session, pkN, pkN + 1, c1, c2, pf.Z, pf.ZPrm, pf.T, pf.V, pf.W)
    else:
        eh = T.sha512_256i_tagged(session, pkN, pkN + 1, X[0], X[1], c1, c2, pf.U[0], pf.U[1],
                                  pf.Z, pf.ZPrm, pf.T, pf.V, pf.W)
    e = T.rejection_sample(Q, eh)
    if X is not None:
        g_s1 = T.scalar_base_mult(pf.S1 % Q)
        xeu = T.ec_add(T.ec_mul(e, X), pf.U)
        if xeu is None or g_s1 != xeu:
            return False
    left = _pw(h1, pf.S1, Nt) * _pw(h2, pf.S2, Nt) % Nt
    if left != _pw(pf.Z, e, Nt) * pf.ZPrm % Nt:
        return False
    left = _pw(h1, pf.T1, Nt) * _pw(h2, pf.T2, Nt) % Nt
    if left != _pw(pf.T, e, Nt) * pf.W % Nt:
        return False
    left = _pw(c1, pf.S1, N2) * _pw(pf.S, pkN, N2) % N2 * _pw(pkN + 1, pf.T1, N2) % N2
    return left == _pw(c2, e, N2) * pf.V % N2


# ----------------------------------------------------------------- protocol
def alice_init(pkA: int, a: int, NTildeB: int, h1B: int, h2B: int, rd: T.Reader):
    """AliceInit(ec, pkA, a, NTildeB, h1B, h2B, rand) -> (cA, pf)."""
    cA, rA = encrypt_and_return_randomness(rd, pkA, a)
    pf = prove_range_alice(pkA, cA, NTildeB, h1B, h2B, a, rA, rd)
    return cA, pf


def bob_mid(session: bytes, pkA: int, pf: RangeProofAlice, b: int, cA: int, NTildeA: int, h1A: int, h2A: int,
            NTildeB: int, h1B: int, h2B: int, rd: T.Reader, B: T.Point = None, wc: bool = False):
    """BobMid / BobMidWC(Session, ec, pkA, pf, b, cA, NTildeA, h1A, h2A, NTildeB, h1B, h2B[, B], rand)
    -> (beta, cB, betaPrm, piB); raises ValueError where Go returns an error."""
    if not verify_range_alice(pf, pkA, NTildeB, h1B, h2B, cA):
        raise ValueError("RangeProofAlice.Verify() returned false")
    beta_prm = T.get_random_positive_int(rd, Q ** 5)  # betaPrm < q^5 (tss-lib v2, Alpha-Rays fix)
    c_beta_prm, c_rand = encrypt_and_return_randomness(rd, pkA, beta_prm)
    cB = homo_mult(pkA, b, cA)
    cB = homo_add(pkA, cB, c_beta_prm)
    beta = (0 - beta_prm) % Q
    piB = prove_bob_wc(session, pkA, NTildeA, h1A, h2A, cA, cB, b, beta_prm, c_rand, B if wc else None, rd)
    return beta, cB, beta_prm, piB


def alice_end(session: bytes, pkA: int, pf: ProofBob, h1A: int, h2A: int, cA: int, cB: int, NTildeA: int,
              lam: int, B: T.Point = None, wc: bool = False) -> int:
    """AliceEnd / AliceEndWC(Session, ec, pkA, pf, h1A, h2A, cA, cB, NTildeA[, B], sk) -> alpha mod q."""
    if not verify_bob_wc(pf, session, pkA, NTildeA, h1A, h2A, cA, cB, B if wc else None):
        raise ValueError("ProofBob.Verify() returned false")
    return decrypt(pkA, lam, cB) % Q
