"""GPU tests of BASELINE configs 4 and 5 through the C-ABI drivers.

Config 4 (csrc/host/signing.hpp, mpcxh_bench_signing): 1,000 wallets signed by
2 and by 3 of the 3 fixture nodes (3 = every ready peer, mpcium's default:
/root/reference/pkg/mpc/node.go:148). The driver checks alpha + beta = k gamma
and mu + nu = k w on every session and ecdsa.Verify on every signature; sampled
wallets are recomputed by the oracle (oracle/signing_ref.py) and compared field
by field: every pair's alpha, beta, mu, nu, a digest of the whole session
transcript (cA, both proofs, cB, cB'), and the signature (r, s, recid).

Config 5 (csrc/host/keygenload.hpp): 5-party keygen / reshare proof work
(3-of-5), every proof verified."""
import json
import os

import pytest

from conftest import GOLDEN
from oracle import crosscheck as cc
from oracle import mta_ref as M
from oracle import signing_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


@pytest.fixture(scope="module")
def drv(gpu):
    from mpcium_amd import host, mta
    host.init(0)
    return mta


@pytest.fixture()
def fast_exp():
    lib = cc.load_c_oracle(64)
    if lib is None:
        pytest.skip("oracle/libgomodexp64.so not built")
    old = M._pw
    M._pw = lambda x, y, m: cc.c_expnn(lib, x % m, y, m)
    yield
    M._pw = old


@pytest.mark.parametrize("signers,wallets,trace", [(2, 10000, 6), (3, 1000, 3)])
def test_signing_wallets_match_oracle(drv, nodes, fast_exp, signers, wallets, trace):
    """Config 4 at its stated size for 2 signers (10,000 wallets, three
    concurrent wallet pipelines by default): traced wallets are spread over the
    batch, so every pipeline's sessions are compared with the oracle."""
    seed = 0x516E + signers
    st, tr = drv.bench_signing(nodes, signers, wallets, seed=seed, trace_wallets=trace)
    assert st["errors"] == 0 and st["relation_failures"] == 0
    assert st["signatures"] == wallets and st["verified"] == wallets
    assert st["sessions"] == wallets * signers * (signers - 1)
    order = S.pair_order(signers)
    assert tr["wallets"] == [t * wallets // trace for t in range(trace)]
    if signers == 2:  # one traced wallet in each third (the default pipelines' chunks)
        assert {wi * 3 // wallets for wi in tr["wallets"]} == {0, 1, 2}
    for t, wi in enumerate(tr["wallets"]):
        pairs, sig, ok = S.sign_wallet(nodes, signers, seed, wi)
        assert ok
        assert tr["sigs"][t] == sig, wi
        for p, ij in enumerate(order):
            assert tr["pairs"][p][t] == pairs[ij], (wi, ij)


def test_keygen_reshare_5_parties(gpu, nodes):
    """Config 5's shape: 3-of-5 keygen / reshare proof work. The 3 fixture nodes
    plus 2 nodes whose preparams come from the GPU GeneratePreParams; every
    party proves DLN x2, Mod and a Fac proof per peer, and verifies every
    peer's proofs."""
    from mpcium_amd import host as mhost
    from mpcium_amd import proofs as mproofs
    mhost.init(0)
    parties = list(nodes)
    for seed in (0x6D706335, 0x6D706336):
        pp, _ = mhost.generate_preparams(seed=seed)
        assert pp["N"] == pp["P"] * pp["Q"] and pp["NTildei"] == (2 * pp["p"] + 1) * (2 * pp["q"] + 1)
        parties.append(pp)
    n, sessions = 5, 16
    st = mproofs.bench_keygen_proofs(parties, sessions, seed=0x6B69)
    assert st["failures"] == 0
    assert st["proofs"] == sessions * n * (2 + 1 + (n - 1))
    assert st["verifications"] == sessions * n * (n - 1) * 4
