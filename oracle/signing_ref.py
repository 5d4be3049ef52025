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

The rest of GG18 (tss-lib up:ecdsa/signing round_1.go .. round_9.go,
finalize.go; upstream, verify) is replayed per signer i from its own GG18
reader CounterDRBG(mix(seed, wallet, 0x100 + i, 4)), in this draw order:
  round 1: Gamma_i = gamma_i G; (C1_i, D1_i) = NewHashCommitment(Gamma_i.x, Gamma_i.y)
  round 4: pi_i = schnorr.NewZKProof(Session, gamma_i, Gamma_i)
  round 5: every peer's D1_j against C1_j and pi_j verified; R = theta^-1 (Gamma_i + sum_j Gamma_j),
           s_i = m k_i + R.x sigma_i (mod q); l_i, rho_i < q; V_i = s_i R + l_i G, A_i = rho_i G;
           (C5_i, D5_i) = NewHashCommitment(V_i.x, V_i.y, A_i.x, A_i.y)
  round 6: piA_i = NewZKProof(Session, rho_i, A_i), piV_i = NewZKVProof(Session, V_i, R, s_i, l_i)
  round 7: every peer's D5_j, piA_j, piV_j verified; V = -m G - r X + sum V, A = sum A;
           U_i = rho_i V, T_i = l_i A; (C7_i, D7_i) = NewHashCommitment(U_i.x, U_i.y, T_i.x, T_i.y)
  round 9: every peer's D7_j verified; sum U == sum T; s_i broadcast
  finalize: s = sum s_i, low-s, recovery id, ecdsa.Verify by every signer (tss-lib's finalize) and
           once more by every node's mpcium session (ecdsa_signing_session.go:162).
A wallet whose transcript fails any check is aborted (no signature); the
others are unaffected.
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


def sign_wallet(nodes: Sequence[Dict[str, int]], signers: int, seed: int, wi: int, tamper: int = 0):
    """-> (pairs: {(i, j): {alpha, beta, mu, nu, digest}}, (r, s, recid) or None
    (aborted), verified, GG18 transcript digest of rounds 1, 4-9)."""
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
    deltas, sigmas = [], []
    X = None
    for i, (k, g, w) in enumerate(shares):  # round 3: delta_i, sigma_i
        di, si = k * g, k * w
        for j in range(signers):
            if j != i:
                di += pairs[(i, j)]["alpha"] + pairs[(j, i)]["beta"]
                si += pairs[(i, j)]["mu"] + pairs[(j, i)]["nu"]
        deltas.append(di % Q)
        sigmas.append(si % Q)
        X = T.ec_add(X, W[i])
    digest, sig = gg18_rounds(sess, shares, m, deltas, sigmas, X, seed, wi, tamper)
    if sig is None:
        return pairs, None, False, digest
    return pairs, sig, ecdsa_verify(X, m, sig[0], sig[1]), digest


# ------------------------------------------------------------ GG18 rounds 1, 4-9
G = T.SECP_G


def hash_commit(rd: T.Reader, *secrets: int):
    """commitments.NewHashCommitment(rand, secrets...): r = MustGetRandomInt(256),
    C = SHA512_256i(r, secrets...), D = [r, secrets...]."""
    D = [T.must_get_random_int(rd, 256), *secrets]
    return T.sha512_256i(*D), D


def hash_decommit(C: int, D):
    """HashCommitDecommit{C, D}.DeCommit(): the secrets, or None."""
    if C is None or not D or T.sha512_256i(*D) != C:
        return None
    return list(D[1:])


def _point(xy) -> T.Point:
    """crypto.NewECPoint(ec, x, y): None unless (x, y) is on the curve."""
    P = (xy[0], xy[1])
    return P if T.ec_on_curve(P) else None


def zk_prove(session: bytes, x: int, X: T.Point, rd: T.Reader):
    """schnorr.NewZKProof(Session, x, X, rand) -> (alpha, t)."""
    a = T.get_random_positive_int(rd, Q)
    alpha = T.scalar_base_mult(a)
    c = T.rejection_sample(Q, T.sha512_256i_tagged(session, X[0], X[1], G[0], G[1], alpha[0], alpha[1]))
    return alpha, (a + c * x) % Q


def zk_verify(session: bytes, pf, X: T.Point) -> bool:
    """(*ZKProof).Verify(Session, X): t G == alpha + c X."""
    alpha, t = pf
    if alpha is None or t is None or not T.ec_on_curve(alpha) or X is None:
        return False
    c = T.rejection_sample(Q, T.sha512_256i_tagged(session, X[0], X[1], G[0], G[1], alpha[0], alpha[1]))
    aXc = T.ec_add(alpha, T.ec_mul(c, X))
    return aXc is not None and T.scalar_base_mult(t) == aXc


def zkv_prove(session: bytes, V: T.Point, R: T.Point, s: int, l: int, rd: T.Reader):
    """schnorr.NewZKVProof(Session, V, R, s, l, rand) -> (alpha, t, u)."""
    a = T.get_random_positive_int(rd, Q)
    b = T.get_random_positive_int(rd, Q)
    alpha = T.ec_add(T.ec_mul(a, R), T.scalar_base_mult(b))
    c = T.rejection_sample(Q, T.sha512_256i_tagged(session, V[0], V[1], R[0], R[1], G[0], G[1], alpha[0],
                                                     alpha[1]))
    return alpha, (a + c * s) % Q, (b + c * l) % Q


def zkv_verify(session: bytes, pf, V: T.Point, R: T.Point) -> bool:
    """(*ZKVProof).Verify(Session, V, R): t R + u G == alpha + c V."""
    alpha, t, u = pf
    if alpha is None or not T.ec_on_curve(alpha) or V is None or R is None:
        return False
    c = T.rejection_sample(Q, T.sha512_256i_tagged(session, V[0], V[1], R[0], R[1], G[0], G[1], alpha[0],
                                                     alpha[1]))
    left = T.ec_add(T.ec_mul(t, R), T.scalar_base_mult(u))
    right = T.ec_add(alpha, T.ec_mul(c, V))
    return left is not None and left == right


TAMPER_R4_SCHNORR, TAMPER_R6_ZKV, TAMPER_R7_DECOMMIT = 1, 2, 3


def gg18_rounds(sess: bytes, shares, m: int, deltas, sigmas, X: T.Point, seed: int, wi: int, tamper: int = 0):
    """Rounds 1, 4-9 and finalize for one wallet (module header). deltas /
    sigmas: every signer's delta_i, sigma_i from rounds 1-3. tamper: corrupt
    signer 0's round-4 Schnorr proof (1), its round-6 ZKV proof (2) or its
    round-7 decommitment (3). -> (transcript digest, (r, s, recid) or None)."""
    S = len(shares)
    rd = [T.Reader(mix(seed, wi, 0x100 + i, 4)) for i in range(S)]
    Gam = [T.scalar_base_mult(g) for _, g, _ in shares]
    c1 = [hash_commit(rd[i], Gam[i][0], Gam[i][1]) for i in range(S)]
    theta = sum(deltas) % Q
    theta_inv = pow(theta, -1, Q)
    pf4 = [zk_prove(sess, shares[i][1], Gam[i], rd[i]) for i in range(S)]
    if tamper == TAMPER_R4_SCHNORR:
        pf4[0] = (pf4[0][0], (pf4[0][1] + 1) % Q)
    ok = True
    R, si, li, roi, Vi, Ai, c5 = [None] * S, [0] * S, [0] * S, [0] * S, [None] * S, [None] * S, [None] * S
    for i in range(S):  # round 5
        Ri = Gam[i]
        for j in range(S):
            if j == i:
                continue
            g = hash_decommit(*c1[j])
            Gj = _point(g) if g is not None and len(g) == 2 else None
            if Gj is None or not zk_verify(sess, pf4[j], Gj):
                ok = False
                continue
            Ri = T.ec_add(Ri, Gj)
        R[i] = T.ec_mul(theta_inv, Ri)
        si[i] = (m * shares[i][0] + R[i][0] * sigmas[i]) % Q
        li[i] = T.get_random_positive_int(rd[i], Q)
        roi[i] = T.get_random_positive_int(rd[i], Q)
        Vi[i] = T.ec_add(T.ec_mul(si[i], R[i]), T.scalar_base_mult(li[i]))
        Ai[i] = T.scalar_base_mult(roi[i])
        c5[i] = hash_commit(rd[i], Vi[i][0], Vi[i][1], Ai[i][0], Ai[i][1])
    if not ok:
        return None, None
    pfA = [zk_prove(sess, roi[i], Ai[i], rd[i]) for i in range(S)]  # round 6
    pfV = [None] * S
    for i in range(S):
        pfV[i] = zkv_prove(sess, Vi[i], R[i], si[i], li[i], rd[i])
    if tamper == TAMPER_R6_ZKV:
        pfV[0] = (pfV[0][0], (pfV[0][1] + 1) % Q, pfV[0][2])
    Ui, Ti, c7 = [None] * S, [None] * S, [None] * S
    for i in range(S):  # round 7
        V = T.ec_add(T.scalar_base_mult((0 - m) % Q), T.ec_mul((0 - R[i][0]) % Q, X))
        V, A = T.ec_add(V, Vi[i]), Ai[i]
        for j in range(S):
            if j == i:
                continue
            v = hash_decommit(*c5[j])
            Vj = _point(v[0:2]) if v is not None and len(v) == 4 else None
            Aj = _point(v[2:4]) if v is not None and len(v) == 4 else None
            if Vj is None or Aj is None or not zk_verify(sess, pfA[j], Aj) or not zkv_verify(sess, pfV[j], Vj, R[i]):
                ok = False
                continue
            V, A = T.ec_add(V, Vj), T.ec_add(A, Aj)
        if not ok:
            continue
        Ui[i], Ti[i] = T.ec_mul(roi[i], V), T.ec_mul(li[i], A)
        c7[i] = hash_commit(rd[i], Ui[i][0], Ui[i][1], Ti[i][0], Ti[i][1])
    if not ok:
        return None, None
    if tamper == TAMPER_R7_DECOMMIT:
        c7[0] = (c7[0][0], [c7[0][1][0], c7[0][1][1] ^ 1] + c7[0][1][2:])
    for i in range(S):  # round 9
        U, Tt = Ui[i], Ti[i]
        for j in range(S):
            if j == i:
                continue
            v = hash_decommit(*c7[j])
            if v is None or len(v) != 4:
                ok = False
                continue
            U, Tt = T.ec_add(U, (v[0], v[1])), T.ec_add(Tt, (v[2], v[3]))
        if U != Tt:
            ok = False
    if not ok:
        return None, None
    ints = []
    for i in range(S):
        ints += [c1[i][0], Gam[i][0], Gam[i][1], pf4[i][0][0], pf4[i][0][1], pf4[i][1], c5[i][0], Vi[i][0], Vi[i][1],
                 Ai[i][0], Ai[i][1], pfA[i][0][0], pfA[i][0][1], pfA[i][1], pfV[i][0][0], pfV[i][0][1], pfV[i][1],
                 pfV[i][2], c7[i][0], Ui[i][0], Ui[i][1], Ti[i][0], Ti[i][1], si[i]]
    digest = T.sha512_256i(*ints)
    s = sum(si) % Q  # finalize (every signer: the same R, r, s)
    r = R[0][0] % Q
    recid = (2 if R[0][0] >= Q else 0) | (R[0][1] & 1)
    if s > Q // 2:
        s, recid = Q - s, recid ^ 1
    if not all(ecdsa_verify(X, m, r, s) for _ in range(2 * S)):  # tss-lib finalize + mpcium, per signer
        return digest, None
    return digest, (r, s, recid)


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
