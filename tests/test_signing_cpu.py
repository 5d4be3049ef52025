"""CPU tests of the signing oracle (oracle/signing_ref.py): one wallet signed
by 2 of the fixture nodes produces an ECDSA signature that verifies, the MtA
relations hold on every ordered pair, and tampering with the message or
signature fails verification. Exponentiations use the C restatement of Go's
expNN (64-bit Words) for speed; results are the same integers as pow()."""
import json
import os

import pytest

from conftest import GOLDEN
from oracle import crosscheck as cc
from oracle import mta_ref as M
from oracle import signing_ref as S
from oracle import tss_ref as T


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


@pytest.fixture()
def fast_exp():
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    old = M._pw
    M._pw = lambda x, y, m: cc.c_expnn(lib, x % m, y, m)
    yield
    M._pw = old


def test_mix_matches_driver_constants():
    # spot values of the driver's seed mixer (signing.cpp mix), fixed here so a change on either side is caught
    assert S.mix(0, 0, 0, 0) == 0
    assert S.mix(1, 2, 3, 4) == S.mix(1, 2, 3, 4) and S.mix(1, 2, 3, 4) != S.mix(1, 2, 3, 5)


def test_two_signer_wallet_signature_verifies(nodes, fast_exp):
    pairs, (r, s, recid), ok, digest = S.sign_wallet(nodes, 2, 0x5163, 0)
    assert ok and 0 < r < S.Q and 0 < s <= S.Q // 2 and recid in (0, 1, 2, 3)
    _, shares, m = S.wallet_setup(0x5163, 0, 2)
    for (i, j), p in pairs.items():
        assert (p["alpha"] + p["beta"]) % S.Q == shares[i][0] * shares[j][1] % S.Q
        assert (p["mu"] + p["nu"]) % S.Q == shares[i][0] * shares[j][2] % S.Q
    X = None
    for _, _, w in shares:
        X = T.ec_add(X, T.scalar_base_mult(w))
    assert S.ecdsa_verify(X, m, r, s)
    assert S.ecdsa_verify(X, m, r, S.Q - s)          # ECDSA accepts both s forms
    assert not S.ecdsa_verify(X, m + 1, r, s)
    assert not S.ecdsa_verify(X, m, r, (s + 1) % S.Q)


def test_schnorr_proofs_and_commitments():
    """tss-lib's round 1/4-9 building blocks (oracle/signing_ref.py): honest
    ZK / ZKV proofs verify, a proof for another point, another session or a
    shifted response does not; a hash commitment opens only to its own D."""
    rd = T.Reader(77)
    x, s_, l_ = 12345678901234567890, 987654321, 555
    X = T.scalar_base_mult(x)
    ss = b"session-0123456789abcdef-0123456"
    pf = S.zk_prove(ss, x, X, rd)
    assert S.zk_verify(ss, pf, X)
    assert not S.zk_verify(ss, pf, T.scalar_base_mult(x + 1))
    assert not S.zk_verify(ss[:-1] + b"7", pf, X)
    assert not S.zk_verify(ss, (pf[0], (pf[1] + 1) % S.Q), X)
    R = T.scalar_base_mult(99)
    V = T.ec_add(T.ec_mul(s_, R), T.scalar_base_mult(l_))
    pv = S.zkv_prove(ss, V, R, s_, l_, rd)
    assert S.zkv_verify(ss, pv, V, R)
    assert not S.zkv_verify(ss, (pv[0], pv[1], (pv[2] + 1) % S.Q), V, R)
    assert not S.zkv_verify(ss, pv, V, T.scalar_base_mult(98))
    C, D = S.hash_commit(rd, X[0], X[1])
    assert S.hash_decommit(C, D) == [X[0], X[1]]
    assert S.hash_decommit(C, [D[0], D[1] + 1, D[2]]) is None


@pytest.mark.parametrize("tamper", [S.TAMPER_R4_SCHNORR, S.TAMPER_R6_ZKV, S.TAMPER_R7_DECOMMIT])
def test_tampered_gg18_transcript_aborts_wallet(nodes, fast_exp, tamper):
    """A corrupted round-4 Schnorr proof, round-6 ZKV proof or round-7
    decommitment of one signer aborts the wallet: no signature."""
    pairs, sig, ok, digest = S.sign_wallet(nodes, 2, 0x5163, 1, tamper=tamper)
    assert sig is None and not ok


def test_openssl_ec_matches_restatement():
    """The OpenSSL-backed secp256k1 of the CPU baseline (oracle/ossl_ec.py)
    returns the same points as the pure-Python restatement."""
    from oracle import ossl_ec
    ec = ossl_ec._Ec()
    rd = T.Reader(5)
    for _ in range(8):
        k1, k2 = (T.get_random_positive_int(rd, S.Q) for _ in range(2))
        P = T.scalar_base_mult(k1)
        assert ec.base(k1) == P
        assert ec.mul(k2, P) == T.ec_mul(k2, P)
        assert ec.add(P, ec.base(k2)) == T.ec_add(P, T.scalar_base_mult(k2))
    assert ec.mul(S.Q, T.SECP_G) is None and ec.add(P, (P[0], T.SECP_P - P[1])) is None
