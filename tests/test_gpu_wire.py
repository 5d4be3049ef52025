"""GPU test of the F4 formats feeding the batch entry points: the golden MtA
sessions (tests/golden/mta_vectors.json) travel as mpcium TssMessage JSON
around tss-lib wire bytes, key material comes from LocalPartySaveData JSON,
and the decoded batches go through libmpcx: RangeProofAlice.Verify accepts
every session and AliceEnd / AliceEndWC reproduce the golden alphas."""
import json
import os

import pytest

from conftest import GOLDEN, H
from mpcium_amd import wire
from test_wire_cpu import party, r1_msg, r2_msg, save_data

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mta(gpu):
    from mpcium_amd import host, mta
    host.init(0)
    return mta


def test_wire_batches_through_gpu(mta):
    vec = [v for v in json.load(open(os.path.join(GOLDEN, "mta_vectors.json")))["sessions"]
           if (v["alice_node"], v["bob_node"]) == (0, 1)]
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    nodes = [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"}
             for n in d["nodes"]]
    # node 0 = Alice, node 1 = Bob, each loads its own save data from JSON
    sdA = wire.LocalPartySaveData.from_json(save_data(nodes, 0).to_json())
    sdB = wire.LocalPartySaveData.from_json(save_data(nodes, 1).to_json())
    alice, bob = party(0), party(1)

    # Round 1 at Bob: Alice's SignRound1Message1 for every wallet
    raws = [wire.TssMessage(f"w{k}", wire.wire_bytes(r1_msg(v), alice, [bob]), False, alice, [bob]).marshal()
            for k, v in enumerate(vec)]
    r1, _, skipped = wire.collect_signing_rounds(raws, bob)
    assert skipped == 0
    b1 = r1[alice.id]
    ok = mta.verify_range_alice(sdB.peer_paillier_n(0), sdB.own_dln(), b1.c, b1.proofs)
    assert ok == [True] * len(vec)

    # Round 2 at Alice: Bob's SignRound2Message (c1 = MtA, c2 = MtAwc)
    raws = [wire.TssMessage(f"w{k}", wire.wire_bytes(r2_msg(v), bob, [alice]), False, bob, [alice]).marshal()
            for k, v in enumerate(vec)]
    _, r2, _ = wire.collect_signing_rounds(raws, alice)
    b2 = r2[bob.id]
    ss = [bytes.fromhex(v["session"]) for v in vec]
    cA = [H(v["cA"]) for v in vec]
    alpha, err = mta.alice_end(ss, sdA.paillier_sk_tuple(), b2.proof_bob, sdA.own_dln(), cA, b2.c1)
    assert err == [0] * len(vec)
    assert alpha == [H(v["alpha"]) for v in vec]
    Bpts = [(H(v["Bx"]), H(v["By"])) for v in vec]
    alpha, err = mta.alice_end(ss, sdA.paillier_sk_tuple(), b2.proof_bob_wc, sdA.own_dln(), cA, b2.c2, B=Bpts)
    assert err == [0] * len(vec)
    assert alpha == [H(v["alpha_wc"]) for v in vec]
