"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (mpcium_amd/) never imports it.

Pure-Python restatement of one wallet of the config-4 signing driver
(mpcium_amd/csrc/host/signing.hpp): the wallet's random draws, every ordered
signer pair's MtA / MtAwc session (oracle/mta_ref.py: AliceInit, BobMid,
BobMidWC, AliceEnd, AliceEndWC of tss-lib up:crypto/mta), and the GG18
signature algebra of tss-lib's up:ecdsa/signing rounds 4-9 + finalize:

    delta = sum_i (k_i gamma_i + sum_j alpha_ij + beta_ij) = k gamma
    sigma = sum_i (k_i w_i + sum_j mu_ij + nu_ij)          = k x
    R = delta^-1 * sum_i gamma_i G,  r = R.x mod q,  s = m k + r sigma (mod q),
    low-s normalisation with the recovery id (bit 0 = R.y odd, bit 1 = R.x >= q)
    (upstream, verify)

and ecdsa.Verify(X, m, r, s) as mpcium calls it when the party ends
(/root/reference/pkg/mpc/ecdsa_signing_session.go:162).  The per-session
digest is SHA512_256i over the session's transcript fields (tss_ref.py), the
same record the GPU driver's trace holds.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from . import mta_ref as M
from . import tss_ref as T

Q = T.SECP_N
_M64 = (1 << 64) - 1


def mix(seed: int, a: int, b: int, c: int) -> int:
    """signing.cpp mix(): the per-wallet / per-pair CounterDRBG seed."""
    x = (seed ^ (a * 0x9E3779B97F4A7C15) ^ (b * 0xC2B2AE3D27D4EB4F) ^ (c * 0x165667B19E3779F9)) & _M64
    x ^= x >> 31
    x = (x * 0xBF58476D1CE4E5B9) & _M64
    x ^= x >> 29
    return x


def wallet_setup(seed: int, wi: int, signers: int):
    """Session id, per-signer (k_i, gamma_i, w_i) and the message, in the
    driver's draw order."""
    rd = T.Reader(mix(seed, wi, 0xFFFF, 0))
    sess = rd.read(32)
    shares = []
    for _ in range(signers):
        k = T.get_random_positive_int(rd, Q)
        g = T.get_random_positive_int(rd, Q)
        w = T.get_random_positive_int(rd, Q)
        shares.append((k, g, w))
    m = T.get_random_positive_int(rd, Q)
    return sess, shares, m


def _digest(cA, pfA, bob, bob_wc) -> int:
    ints = [cA, pfA.Z, pfA.U, pfA.W, pfA.S, pfA.S1, pfA.S2, bob[1]]
    for pf, nxt in ((bob[3], bob_wc[1]), (bob_wc[3], None)):
        ints += [pf.Z, pf.ZPrm, pf.T, pf.V, pf.W, pf.S, pf.S1, pf.S2, pf.T1, pf.T2]
        if nxt is not None:
            ints.append(nxt)
    ints += [bob_wc[3].U[0], bob_wc[3].U[1]]
    return T.sha512_256i(*ints)


def sign_wallet(nodes: Sequence[Dict[str, int]], signers: int, seed: int, wi: int):
    """-> (pairs: {(i, j): {alpha, beta, mu, nu, digest}}, (r, s, recid), verified)."""
    sess, shares, m = wallet_setup(seed, wi, signers)
    W = [T.scalar_base_mult(w) for _, _, w in shares]
    pairs: Dict[Tuple[int, int], dict] = {}
    for i in range(signers):
        for j in range(signers):
            if i == j:
                continue
            A, B = nodes[i], nodes[j]
            ki, gj, wj = shares[i][0], shares[j][1], shares[j][2]
            cA, pfA = M.alice_init(A["N"], ki, B["NTildei"], B["H1i"], B["H2i"],
                                   T.Reader(mix(seed, wi, i * 16 + j, 1)))
            bob = M.bob_mid(sess, A["N"], pfA, gj, cA, A["NTildei"], A["H1i"], A["H2i"], B["NTildei"], B["H1i"],
                            B["H2i"], T.Reader(mix(seed, wi, i * 16 + j, 2)))
            bob_wc = M.bob_mid(sess, A["N"], pfA, wj, cA, A["NTildei"], A["H1i"], A["H2i"], B["NTildei"],
                               B["H1i"], B["H2i"], T.Reader(mix(seed, wi, i * 16 + j, 3)), B=W[j], wc=True)
            alpha = M.alice_end(sess, A["N"], bob[3], A["H1i"], A["H2i"], cA, bob[1], A["NTildei"], A["LambdaN"])
            mu = M.alice_end(sess, A["N"], bob_wc[3], A["H1i"], A["H2i"], cA, bob_wc[1], A["NTildei"],
                             A["LambdaN"], B=W[j], wc=True)
            pairs[(i, j)] = {"alpha": alpha, "beta": bob[0], "mu": mu, "nu": bob_wc[0],
                             "digest": _digest(cA, pfA, bob, bob_wc)}
    delta = sigma = s_part = 0
    Gam = X = None
    for i, (k, g, w) in enumerate(shares):
        di, si = k * g, k * w
        for j in range(signers):
            if j != i:
                di += pairs[(i, j)]["alpha"] + pairs[(j, i)]["beta"]
                si += pairs[(i, j)]["mu"] + pairs[(j, i)]["nu"]
        delta, sigma = (delta + di) % Q, (sigma + si) % Q
        Gam = T.ec_add(Gam, T.scalar_base_mult(g))
        X = T.ec_add(X, W[i])
        s_part = (s_part + m * k) % Q
    R = T.ec_mul(pow(delta, -1, Q), Gam)
    r = R[0] % Q
    s = (s_part + r * sigma) % Q
    recid = (2 if R[0] >= Q else 0) | (R[1] & 1)
    if s > Q // 2:
        s, recid = Q - s, recid ^ 1
    return pairs, (r, s, recid), ecdsa_verify(X, m, r, s)


def ecdsa_verify(X, e: int, r: int, s: int) -> bool:
    """crypto/ecdsa Verify for a secp256k1 key with hash integer e < 2^256."""
    if not (0 < r < Q and 0 < s < Q) or X is None:
        return False
    w = pow(s, -1, Q)
    P = T.ec_add(T.scalar_base_mult(e * w % Q), T.ec_mul(r * w % Q, X))
    return P is not None and P[0] % Q == r


def pair_order(signers: int) -> List[Tuple[int, int]]:
    """Ordered signer pairs in the driver's trace order (i-major, j != i)."""
    return [(i, j) for i in range(signers) for j in range(signers) if i != j]
