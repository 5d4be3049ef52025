"""CPU tests of the wire / at-rest formats around the MtA path (SURVEY.md §8(f)
row F4; mpcium_amd/wire.py): mpcium's TssMessage JSON envelope
(ref:pkg/types/tss.go:13-24), tss-lib's MessageWrapper protobuf and the round
payloads that carry Paillier / N~ work, and LocalPartySaveData JSON.

Parity is unpinned against the reference for the protobuf field numbers and
the save-data field layout (tss-lib is not vendored in /root/reference): the
tests pin hand-computed protobuf bytes, Go encoding/json conventions, round
trips of the golden MtA sessions and node preparams, and tss-lib's rejection
rules (part counts, empty parts)."""
import base64
import json
import os

import pytest

from conftest import GOLDEN, H
from mpcium_amd import wire


@pytest.fixture(scope="module")
def vec():
    return [v for v in json.load(open(os.path.join(GOLDEN, "mta_vectors.json")))["sessions"]
            if (v["alice_node"], v["bob_node"]) == (0, 1)]


@pytest.fixture(scope="module")
def nodes():
    d = json.load(open(os.path.join(GOLDEN, "node_preparams.json")))
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"} for n in d["nodes"]]


def party(i):
    return wire.PartyID(id=str(i + 1), moniker=f"node{i}", key=(1000 + i).to_bytes(2, "big"), index=i)


def r1_msg(v):
    return wire.SignRound1Message1(H(v["cA"]), {k: H(x) for k, x in v["pfA"].items()})


def r2_msg(v):
    pb = {k: H(v["bob"]["pf"][k]) for k in wire.BOB_FIELDS}
    pb["U"] = None
    wc = {k: H(v["bob_wc"]["pf"][k]) for k in wire.BOB_FIELDS}
    wc["U"] = (H(v["bob_wc"]["pf"]["Ux"]), H(v["bob_wc"]["pf"]["Uy"]))
    return wire.SignRound2Message(H(v["bob"]["cB"]), H(v["bob_wc"]["cB"]), pb, wc)


def test_protobuf_known_bytes():
    # PartyID{id:"1", moniker:"a", key:0x01}: tags 0x0a, 0x12, 0x1a, length 1 each
    assert wire.PartyID("1", "a", b"\x01").to_pb() == bytes.fromhex("0a0131120161" "1a0101")
    # proto3 defaults are not emitted
    assert wire.PartyID().to_pb() == b""
    # varints across the 7-bit boundary
    assert wire._varint(300) == bytes.fromhex("ac02")
    assert wire._read_varint(bytes.fromhex("ac02"), 0) == (300, 2)
    # MessageWrapper{is_broadcast, from, message=Any{url, value}}
    w = wire.MessageWrapper("t/x", b"\x07", is_broadcast=True, from_=wire.PartyID("1"))
    assert w.to_bytes() == bytes.fromhex("0801" "1a030a0131" "5208" "0a03742f78" "120107")
    back = wire.MessageWrapper.from_bytes(w.to_bytes())
    assert back.is_broadcast and back.from_.id == "1" and back.type_url == "t/x" and back.content == b"\x07"


def test_protobuf_malformed():
    for bad in (b"\x0a", b"\x0a\x05ab", b"\x80", b"\x0b", bytes([0x00, 0x01])):
        with pytest.raises(wire.WireError):
            wire.pb_fields(bad)


def test_big_int_bytes():
    assert wire.int_bytes(0) == b""
    assert wire.int_bytes(255) == b"\xff" and wire.int_bytes(256) == b"\x01\x00"
    assert wire.bytes_int(b"\x00\x01") == 1
    with pytest.raises(wire.WireError):
        wire.int_bytes(-1)


def test_signing_payloads_round_trip(vec):
    for v in vec:
        m1 = r1_msg(v)
        raw = wire.wire_bytes(m1, party(0), [party(1)])
        w, c = wire.parse_wire(raw)
        assert w.type_url == "type.googleapis.com/binance.tsslib.ecdsa.signing.SignRound1Message1"
        assert not w.is_broadcast and w.from_.id == "1" and [p.id for p in w.to] == ["2"]
        assert c == m1
        m2 = r2_msg(v)
        w, c = wire.parse_wire(wire.wire_bytes(m2, party(1), [party(0)]))
        assert w.type_name == wire.SignRound2Message.TYPE and c == m2


def test_payload_part_rules(vec):
    m1 = r1_msg(vec[0])
    # a zero field has an empty big.Int.Bytes(): NonEmptyMultiBytes rejects it
    pf = dict(m1.range_proof_alice)
    pf["S1"] = 0
    raw = wire.wire_bytes(wire.SignRound1Message1(m1.c, pf), party(0), [party(1)])
    with pytest.raises(wire.WireError, match="empty part"):
        wire.parse_wire(raw)
    # wrong part count
    content = m1.to_content() + wire._pb_bytes(2, b"\x01")
    with pytest.raises(wire.WireError, match="expected 6 parts"):
        wire.SignRound1Message1.from_content(content)
    m2 = r2_msg(vec[0])
    content = m2.to_content()
    fs = [f for f in wire.pb_fields(content)]
    trimmed = b"".join(wire._pb_bytes(n, x, keep_empty=True) for n, _, x in fs[:-1])  # drop U.Y
    with pytest.raises(wire.WireError, match="ProofBobWC"):
        wire.SignRound2Message.from_content(trimmed)
    # unknown content types come back raw
    w = wire.MessageWrapper("type.googleapis.com/binance.tsslib.ecdsa.signing.SignRound3Message", b"\x0a\x01\x05")
    _, c = wire.parse_wire(w.to_bytes())
    assert c == b"\x0a\x01\x05"


def test_keygen_round1_round_trip(nodes):
    import random
    rng = random.Random(5)
    n = nodes[0]
    dln = lambda: {"Alpha": [rng.getrandbits(2048) | 1 for _ in range(128)],
                   "T": [rng.getrandbits(2046) | 1 for _ in range(128)]}
    m = wire.KGRound1Message(rng.getrandbits(256), n["N"], n["NTildei"], n["H1i"], n["H2i"], dln(), dln())
    w, c = wire.parse_wire(wire.wire_bytes(m, party(2), is_broadcast=True))
    assert w.is_broadcast and w.to == [] and c == m
    with pytest.raises(wire.WireError):
        wire.KGRound1Message(1, 1, 1, 1, 1, {"Alpha": [1], "T": [1]}, dln()).to_content()


def test_tss_message_json_go_conventions(vec):
    raw_wire = wire.wire_bytes(r1_msg(vec[0]), party(0), [party(1)])
    m = wire.TssMessage("wallet-7", raw_wire, False, party(0), [party(1)], signature=b"\x01\x02\x03")
    js = m.marshal()
    d = json.loads(js)
    # struct order, Go tag names, base64 []byte, compact separators
    assert list(d) == ["sessionID", "msgBytes", "isBroadcast", "from", "to", "isToOldCommittee",
                       "isToOldAndNewCommittees", "signature"]
    assert b": " not in js and b", " not in js
    assert base64.b64decode(d["msgBytes"]) == raw_wire and d["signature"] == "AQID"
    assert d["from"] == {"id": "1", "moniker": "node0", "key": base64.b64encode(b"\x03\xe8").decode(), "index": 0}
    assert wire.TssMessage.unmarshal(js) == m
    # nil slices / pointers are null; a broadcast without recipients
    b = wire.TssMessage("w", None, True)
    d = json.loads(b.marshal())
    assert d["msgBytes"] is None and d["from"] is None and d["to"] is None and d["signature"] is None
    assert wire.TssMessage.unmarshal(b.marshal()) == b
    for bad in (b"{", b"[]", b'{"msgBytes": "###"}'):
        with pytest.raises(wire.WireError):
            wire.TssMessage.unmarshal(bad)


def test_addressing_matches_receive_tss_message():
    me, other = party(0), party(1)
    assert wire.TssMessage("w", b"", True, other, None).addressed_to(me)
    assert wire.TssMessage("w", b"", True, other, []).addressed_to(me)
    assert wire.TssMessage("w", b"", False, other, [me]).addressed_to(me)
    assert not wire.TssMessage("w", b"", False, other, [other]).addressed_to(me)
    assert not wire.TssMessage("w", b"", False, other, [me, other]).addressed_to(me)
    assert not wire.TssMessage("w", b"", True, other, [other]).addressed_to(me)


def save_data(nodes, i):
    n = nodes[i]
    return wire.LocalPartySaveData(
        paillier_sk={"N": n["N"], "LambdaN": n["LambdaN"], "PhiN": n["PhiN"], "P": n["P"], "Q": n["Q"]},
        NTildei=n["NTildei"], H1i=n["H1i"], H2i=n["H2i"], Alpha=n["Alpha"], Beta=n["Beta"], P=n["p"], Q=n["q"],
        Xi=12345 + i, ShareID=100 + i, Ks=[100 + j for j in range(len(nodes))],
        NTildej=[m["NTildei"] for m in nodes], H1j=[m["H1i"] for m in nodes], H2j=[m["H2i"] for m in nodes],
        BigXj=[(j + 1, j + 2) for j in range(len(nodes))], PaillierPKs=[m["N"] for m in nodes], ECDSAPub=(7, 8))


def test_save_data_round_trip_and_key_material(nodes):
    for i in range(len(nodes)):
        sd = save_data(nodes, i)
        js = sd.to_json()
        d = json.loads(js)
        assert list(d)[:10] == ["PaillierSK", "NTildei", "H1i", "H2i", "Alpha", "Beta", "P", "Q", "Xi", "ShareID"]
        assert isinstance(d["NTildei"], int)  # big.Int as a bare JSON number
        assert d["ECDSAPub"] == {"Curve": "secp256k1", "Coords": [7, 8]}
        back = wire.LocalPartySaveData.from_json(js)
        assert back == sd
        assert back.party_index() == i
        pp = back.node_preparams()
        for k in ("N", "LambdaN", "P", "Q", "NTildei", "H1i", "H2i", "p", "q"):
            assert pp[k] == nodes[i][k]
        own = back.own_dln()
        assert own["P"] * own["Q"] == nodes[i]["NTildei"]
        for j in range(len(nodes)):
            assert back.peer_dln(j) == {"NTilde": nodes[j]["NTildei"], "h1": nodes[j]["H1i"], "h2": nodes[j]["H2i"]}
            assert back.peer_paillier_n(j) == nodes[j]["N"]


def test_save_data_incomplete():
    sd = wire.LocalPartySaveData.from_json(b'{"PaillierSK":null,"NTildei":5,"Ks":null,"PaillierPKs":[null]}')
    assert sd.Ks == [] and sd.PaillierPKs == [None]
    with pytest.raises(wire.WireError):
        sd.paillier_sk_tuple()
    with pytest.raises(wire.WireError):
        sd.own_dln()
    with pytest.raises(wire.WireError):
        sd.peer_paillier_n(0)
    with pytest.raises(wire.WireError):
        wire.LocalPartySaveData.from_json(b'{"ECDSAPub":{"Coords":[1]}}')


def test_collect_signing_rounds(vec):
    me, alice, carol = party(1), party(0), party(2)
    raws = []
    for k, v in enumerate(vec):
        raws.append(wire.TssMessage(f"w{k}", wire.wire_bytes(r1_msg(v), alice, [me]), False, alice, [me]).marshal())
        raws.append(wire.TssMessage(f"w{k}", wire.wire_bytes(r2_msg(v), carol, [me]), False, carol, [me]).marshal())
        # addressed to someone else / another round: not MtA work for me
        raws.append(wire.TssMessage(f"w{k}", wire.wire_bytes(r1_msg(v), alice, [carol]), False, alice,
                                    [carol]).marshal())
        w3 = wire.MessageWrapper("type.googleapis.com/" + wire.SIGNING_PKG + "SignRound3Message", b"\x0a\x01\x01",
                                 is_broadcast=True, from_=alice)
        raws.append(wire.TssMessage(f"w{k}", w3.to_bytes(), True, alice, None).marshal())
    r1, r2, skipped = wire.collect_signing_rounds(raws, me)
    assert skipped == 2 * len(vec)
    assert list(r1) == ["1"] and list(r2) == ["3"]
    assert r1["1"].wallet_ids == [f"w{k}" for k in range(len(vec))]
    assert r1["1"].c == [H(v["cA"]) for v in vec]
    assert r1["1"].proofs == [{k: H(x) for k, x in v["pfA"].items()} for v in vec]
    assert r2["3"].c1 == [H(v["bob"]["cB"]) for v in vec] and r2["3"].c2 == [H(v["bob_wc"]["cB"]) for v in vec]
    assert [p["U"] for p in r2["3"].proof_bob_wc] == [(H(v["bob_wc"]["pf"]["Ux"]), H(v["bob_wc"]["pf"]["Uy"]))
                                                      for v in vec]
