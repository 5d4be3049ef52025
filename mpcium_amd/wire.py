"""Wire and at-rest formats on either side of the batched MtA path (SURVEY.md
§8(f) row F4): what mpcium hands to tss-lib, decoded into the batch inputs the
GPU entry points take, and encoded back.

Three layers, outermost first:

1. ``TssMessage`` — mpcium's JSON envelope on NATS
   (ref:pkg/types/tss.go:13-24; marshalled by ``MarshalTssMessage`` at
   ref:pkg/types/tss.go:66-73, parsed by ``UnmarshalTssMessage`` at
   ref:pkg/types/tss.go:98-106, consumed by ``Session.receiveTssMessage`` at
   ref:pkg/mpc/session.go:164-205). Go ``encoding/json``: ``[]byte`` as
   padded standard base64, nil slices/pointers as ``null``, ``tss.PartyID`` as
   the promoted fields of its embedded ``*MessageWrapper_PartyID`` plus
   ``index``.
2. ``MsgBytes`` — tss-lib's ``MessageWrapper`` protobuf (``msg.WireBytes()``,
   parsed by ``tss.ParseWireMessage`` inside ``party.UpdateFromBytes``) with the
   round content in a ``google.protobuf.Any``. Field numbers follow tss-lib
   v2.0.2 ``protob/message.proto`` and ``ecdsa-signing.proto`` /
   ``ecdsa-keygen.proto`` (upstream, verify: tss-lib is not vendored in
   /root/reference).
3. Round payloads that carry Paillier / N~ work: ``SignRound1Message1`` (c_A and
   ``RangeProofAlice.Bytes()``, 6 parts), ``SignRound2Message`` (c1, c2 and
   ``ProofBob.Bytes()`` 10 parts, ``ProofBobWC.Bytes()`` 12 parts),
   ``KGRound1Message`` (Paillier N, N~, h1, h2, two DLN proofs of 2x128
   parts). Every part is a big-endian ``big.Int.Bytes()``; tss-lib's
   ``*FromBytes`` constructors reject empty parts (``common.NonEmptyMultiBytes``)
   and so does this decoder.

``LocalPartySaveData`` — the keygen output mpcium stores as JSON in Badger
(ref:pkg/mpc/ecdsa_keygen_session.go:102-108) and reloads for signing
(ref:pkg/mpc/ecdsa_signing_session.go:128-132) and resharing — decodes into
the key material the batch entry points take (``node_preparams`` / ``dln`` /
``paillier_pk`` below).

Pure host code: no GPU, no oracle. Go's ``math/big`` JSON form (bare decimal
numbers) round-trips through Python ints without loss.
"""
from __future__ import annotations

import base64
import json
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

TYPE_URL_PREFIX = "type.googleapis.com/"
SIGNING_PKG = "binance.tsslib.ecdsa.signing."
KEYGEN_PKG = "binance.tsslib.ecdsa.keygen."

RANGE_PROOF_ALICE_PARTS = 6   # Z, U, W, S, S1, S2
PROOF_BOB_PARTS = 10          # Z, ZPrm, T, V, W, S, S1, S2, T1, T2
PROOF_BOB_WC_PARTS = 12       # ProofBob + U.X, U.Y
DLN_ITERATIONS = 128          # dlnproof.Iterations: Alpha[128] then T[128]

RANGE_FIELDS = ["Z", "U", "W", "S", "S1", "S2"]
BOB_FIELDS = ["Z", "ZPrm", "T", "V", "W", "S", "S1", "S2", "T1", "T2"]


class WireError(ValueError):
    """A message tss-lib would refuse to parse (malformed protobuf, wrong part
    count, an empty part, an unexpected type URL)."""


# --------------------------------------------------------------------------
# big.Int <-> bytes (big-endian, minimal: Go's (*big.Int).Bytes / SetBytes)
# --------------------------------------------------------------------------

def int_bytes(v: int) -> bytes:
    if v < 0:
        raise WireError("big.Int.Bytes() carries the absolute value; negative ints are not on the wire")
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def bytes_int(b: bytes) -> int:
    return int.from_bytes(b, "big")


def _non_empty_parts(parts: Sequence[bytes], n: int, what: str) -> List[int]:
    """common.NonEmptyMultiBytes(bzs, n) then new(big.Int).SetBytes per part."""
    if len(parts) != n:
        raise WireError(f"{what}: expected {n} parts, got {len(parts)}")
    if any(len(p) == 0 for p in parts):
        raise WireError(f"{what}: empty part")
    return [bytes_int(p) for p in parts]


# --------------------------------------------------------------------------
# Minimal proto3 codec (varint + length-delimited are all these messages use)
# --------------------------------------------------------------------------

def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    v = shift = 0
    while True:
        if i >= len(buf):
            raise WireError("truncated varint")
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7
        if shift > 63:
            raise WireError("varint overflow")


def pb_fields(buf: bytes) -> List[Tuple[int, int, object]]:
    """Decode one message level into (field number, wire type, value) in wire
    order. Unknown fields are kept (proto3 parsers skip them)."""
    out = []
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if num == 0:
            raise WireError("field number 0")
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            if i + ln > len(buf):
                raise WireError("truncated length-delimited field")
            v = bytes(buf[i:i + ln])
            i += ln
        elif wt == 1:
            if i + 8 > len(buf):
                raise WireError("truncated fixed64")
            v, i = int.from_bytes(buf[i:i + 8], "little"), i + 8
        elif wt == 5:
            if i + 4 > len(buf):
                raise WireError("truncated fixed32")
            v, i = int.from_bytes(buf[i:i + 4], "little"), i + 4
        else:
            raise WireError(f"unsupported wire type {wt}")
        out.append((num, wt, v))
    return out


def _pb_bytes(num: int, b: bytes, keep_empty: bool = False) -> bytes:
    if not b and not keep_empty:   # proto3 scalar default is not emitted
        return b""
    return _varint(num << 3 | 2) + _varint(len(b)) + b


def _pb_bool(num: int, v: bool) -> bytes:
    return _varint(num << 3) + b"\x01" if v else b""


def _one_bytes(fs, num) -> bytes:
    v = b""
    for n, wt, x in fs:
        if n == num:
            if wt != 2:
                raise WireError(f"field {num}: expected bytes")
            v = x   # proto3: last one wins
    return v


def _rep_bytes(fs, num) -> List[bytes]:
    out = []
    for n, wt, x in fs:
        if n == num:
            if wt != 2:
                raise WireError(f"field {num}: expected bytes")
            out.append(x)
    return out


def _one_bool(fs, num) -> bool:
    v = False
    for n, wt, x in fs:
        if n == num:
            if wt != 0:
                raise WireError(f"field {num}: expected varint")
            v = bool(x)
    return v


# --------------------------------------------------------------------------
# tss.PartyID and the MessageWrapper
# --------------------------------------------------------------------------

@dataclass
class PartyID:
    """tss.PartyID: embedded *MessageWrapper_PartyID {id=1, moniker=2, key=3}
    plus Index (not on the protobuf wire; JSON ``index``)."""
    id: str = ""
    moniker: str = ""
    key: bytes = b""
    index: int = 0

    @property
    def key_int(self) -> int:
        return bytes_int(self.key)

    def to_pb(self) -> bytes:
        return (_pb_bytes(1, self.id.encode()) + _pb_bytes(2, self.moniker.encode()) + _pb_bytes(3, self.key))

    @classmethod
    def from_pb(cls, buf: bytes) -> "PartyID":
        fs = pb_fields(buf)
        return cls(_one_bytes(fs, 1).decode(), _one_bytes(fs, 2).decode(), _one_bytes(fs, 3))

    def to_json(self) -> dict:
        # Go: promoted fields with `json:",omitempty"`, then Index.
        d = {}
        if self.id:
            d["id"] = self.id
        if self.moniker:
            d["moniker"] = self.moniker
        if self.key:
            d["key"] = base64.b64encode(self.key).decode()
        d["index"] = self.index
        return d

    @classmethod
    def from_json(cls, d: Optional[dict]) -> Optional["PartyID"]:
        if d is None:
            return None
        return cls(d.get("id", ""), d.get("moniker", ""), _b64d(d.get("key")), int(d.get("index", 0)))


@dataclass
class MessageWrapper:
    """tss-lib protob/message.proto ``MessageWrapper``: is_broadcast=1,
    is_to_old_committee=2, from=3, to=4, is_to_old_and_new_committees=5,
    message=10 (google.protobuf.Any{type_url=1, value=2})."""
    type_url: str
    content: bytes
    is_broadcast: bool = False
    is_to_old_committee: bool = False
    is_to_old_and_new_committees: bool = False
    from_: Optional[PartyID] = None
    to: List[PartyID] = field(default_factory=list)

    @property
    def type_name(self) -> str:
        return self.type_url.rsplit("/", 1)[-1]

    def to_bytes(self) -> bytes:
        any_ = _pb_bytes(1, self.type_url.encode()) + _pb_bytes(2, self.content)
        out = _pb_bool(1, self.is_broadcast) + _pb_bool(2, self.is_to_old_committee)
        if self.from_ is not None:
            out += _pb_bytes(3, self.from_.to_pb(), keep_empty=True)
        for p in self.to:
            out += _pb_bytes(4, p.to_pb(), keep_empty=True)
        out += _pb_bool(5, self.is_to_old_and_new_committees)
        out += _pb_bytes(10, any_, keep_empty=True)
        return out

    @classmethod
    def from_bytes(cls, buf: bytes) -> "MessageWrapper":
        fs = pb_fields(buf)
        frm = [x for n, wt, x in fs if n == 3]
        anys = [x for n, wt, x in fs if n == 10]
        if not anys:
            raise WireError("MessageWrapper without message")
        afs = pb_fields(anys[-1])
        return cls(type_url=_one_bytes(afs, 1).decode(), content=_one_bytes(afs, 2),
                   is_broadcast=_one_bool(fs, 1), is_to_old_committee=_one_bool(fs, 2),
                   is_to_old_and_new_committees=_one_bool(fs, 5),
                   from_=PartyID.from_pb(frm[-1]) if frm else None,
                   to=[PartyID.from_pb(x) for x in _rep_bytes(fs, 4)])


# --------------------------------------------------------------------------
# Round payloads with Paillier / N~ work
# --------------------------------------------------------------------------

@dataclass
class SignRound1Message1:
    """ecdsa-signing.proto: c=1, range_proof_alice=2 (repeated). P2P, Alice -> Bob:
    the AliceInit output c_A and RangeProofAlice (row A8)."""
    c: int
    range_proof_alice: Dict[str, int]
    TYPE = SIGNING_PKG + "SignRound1Message1"

    def to_content(self) -> bytes:
        out = _pb_bytes(1, int_bytes(self.c))
        for f in RANGE_FIELDS:
            out += _pb_bytes(2, int_bytes(self.range_proof_alice[f]), keep_empty=True)
        return out

    @classmethod
    def from_content(cls, buf: bytes) -> "SignRound1Message1":
        fs = pb_fields(buf)
        vals = _non_empty_parts(_rep_bytes(fs, 2), RANGE_PROOF_ALICE_PARTS, "RangeProofAlice")
        return cls(bytes_int(_one_bytes(fs, 1)), dict(zip(RANGE_FIELDS, vals)))


@dataclass
class SignRound2Message:
    """ecdsa-signing.proto: c1=1, c2=2, proof_bob=3, proof_bob_wc=4. P2P, Bob ->
    Alice: BobMid's c_B with ProofBob and BobMidWC's c_B with ProofBobWC (row A9),
    consumed by AliceEnd / AliceEndWC (row A10)."""
    c1: int
    c2: int
    proof_bob: Dict[str, object]
    proof_bob_wc: Dict[str, object]
    TYPE = SIGNING_PKG + "SignRound2Message"

    def to_content(self) -> bytes:
        out = _pb_bytes(1, int_bytes(self.c1)) + _pb_bytes(2, int_bytes(self.c2))
        for f in BOB_FIELDS:
            out += _pb_bytes(3, int_bytes(self.proof_bob[f]), keep_empty=True)
        for f in BOB_FIELDS:
            out += _pb_bytes(4, int_bytes(self.proof_bob_wc[f]), keep_empty=True)
        ux, uy = self.proof_bob_wc["U"]
        out += _pb_bytes(4, int_bytes(ux), keep_empty=True) + _pb_bytes(4, int_bytes(uy), keep_empty=True)
        return out

    @classmethod
    def from_content(cls, buf: bytes) -> "SignRound2Message":
        fs = pb_fields(buf)
        pb = _non_empty_parts(_rep_bytes(fs, 3), PROOF_BOB_PARTS, "ProofBob")
        wc = _non_empty_parts(_rep_bytes(fs, 4), PROOF_BOB_WC_PARTS, "ProofBobWC")
        proof_bob = dict(zip(BOB_FIELDS, pb))
        proof_bob["U"] = None
        proof_bob_wc = dict(zip(BOB_FIELDS, wc[:10]))
        proof_bob_wc["U"] = (wc[10], wc[11])
        return cls(bytes_int(_one_bytes(fs, 1)), bytes_int(_one_bytes(fs, 2)), proof_bob, proof_bob_wc)


@dataclass
class KGRound1Message:
    """ecdsa-keygen.proto: commitment=1, paillier_n=2, n_tilde=3, h1=4, h2=5,
    dlnproof_1=6, dlnproof_2=7 (repeated; dlnproof.Proof.Serialize: Alpha[128]
    then T[128]). Broadcast; every receiver verifies both DLN proofs (row A13)."""
    commitment: int
    paillier_n: int
    n_tilde: int
    h1: int
    h2: int
    dlnproof_1: Dict[str, List[int]]
    dlnproof_2: Dict[str, List[int]]
    TYPE = KEYGEN_PKG + "KGRound1Message"

    @staticmethod
    def _dln_parts(p: Dict[str, List[int]]) -> List[bytes]:
        if len(p["Alpha"]) != DLN_ITERATIONS or len(p["T"]) != DLN_ITERATIONS:
            raise WireError("DLN proof needs 128 Alpha and 128 T values")
        return [int_bytes(v) for v in list(p["Alpha"]) + list(p["T"])]

    @staticmethod
    def _dln_from(parts: List[bytes]) -> Dict[str, List[int]]:
        vals = _non_empty_parts(parts, 2 * DLN_ITERATIONS, "DLNProof")
        return {"Alpha": vals[:DLN_ITERATIONS], "T": vals[DLN_ITERATIONS:]}

    def to_content(self) -> bytes:
        out = (_pb_bytes(1, int_bytes(self.commitment)) + _pb_bytes(2, int_bytes(self.paillier_n)) +
               _pb_bytes(3, int_bytes(self.n_tilde)) + _pb_bytes(4, int_bytes(self.h1)) +
               _pb_bytes(5, int_bytes(self.h2)))
        for b in self._dln_parts(self.dlnproof_1):
            out += _pb_bytes(6, b, keep_empty=True)
        for b in self._dln_parts(self.dlnproof_2):
            out += _pb_bytes(7, b, keep_empty=True)
        return out

    @classmethod
    def from_content(cls, buf: bytes) -> "KGRound1Message":
        fs = pb_fields(buf)
        return cls(bytes_int(_one_bytes(fs, 1)), bytes_int(_one_bytes(fs, 2)), bytes_int(_one_bytes(fs, 3)),
                   bytes_int(_one_bytes(fs, 4)), bytes_int(_one_bytes(fs, 5)),
                   cls._dln_from(_rep_bytes(fs, 6)), cls._dln_from(_rep_bytes(fs, 7)))


CONTENT_TYPES = {c.TYPE: c for c in (SignRound1Message1, SignRound2Message, KGRound1Message)}


def wire_bytes(content, from_: PartyID, to: Sequence[PartyID] = (), is_broadcast: bool = False) -> bytes:
    """tss.MessageImpl.WireBytes() for one of the payloads above."""
    return MessageWrapper(TYPE_URL_PREFIX + content.TYPE, content.to_content(), is_broadcast=is_broadcast,
                          from_=from_, to=list(to)).to_bytes()


def parse_wire(buf: bytes):
    """tss.ParseWireMessage: returns (MessageWrapper, decoded content). Content
    types outside this path come back as raw bytes."""
    w = MessageWrapper.from_bytes(buf)
    cls = CONTENT_TYPES.get(w.type_name)
    return w, (cls.from_content(w.content) if cls else w.content)


# --------------------------------------------------------------------------
# mpcium's TssMessage JSON envelope
# --------------------------------------------------------------------------

def _b64e(b: Optional[bytes]) -> Optional[str]:
    return None if b is None else base64.b64encode(b).decode()


def _b64d(s: Optional[str]) -> bytes:
    if s is None:
        return b""
    try:
        return base64.b64decode(s, validate=True)
    except Exception as e:  # Go: "illegal base64 data at input byte N"
        raise WireError(f"illegal base64 data: {e}") from None


@dataclass
class TssMessage:
    """ref:pkg/types/tss.go:13-24 (JSON tags as there)."""
    wallet_id: str
    msg_bytes: Optional[bytes]
    is_broadcast: bool = False
    from_: Optional[PartyID] = None
    to: Optional[List[PartyID]] = None
    is_to_old_committee: bool = False
    is_to_old_and_new_committees: bool = False
    signature: Optional[bytes] = None

    def marshal(self) -> bytes:
        """types.MarshalTssMessage (ref:pkg/types/tss.go:66-73): Go's compact
        json.Marshal, keys in struct order."""
        d = {
            "sessionID": self.wallet_id,
            "msgBytes": _b64e(self.msg_bytes),
            "isBroadcast": self.is_broadcast,
            "from": None if self.from_ is None else self.from_.to_json(),
            "to": None if self.to is None else [p.to_json() for p in self.to],
            "isToOldCommittee": self.is_to_old_committee,
            "isToOldAndNewCommittees": self.is_to_old_and_new_committees,
            "signature": _b64e(self.signature),
        }
        return json.dumps(d, separators=(",", ":")).encode()

    @classmethod
    def unmarshal(cls, raw: bytes) -> "TssMessage":
        """types.UnmarshalTssMessage (ref:pkg/types/tss.go:98-106)."""
        try:
            d = json.loads(raw)
        except ValueError as e:
            raise WireError(f"invalid JSON: {e}") from None
        if not isinstance(d, dict):
            raise WireError("TssMessage must be a JSON object")
        to = d.get("to")
        return cls(wallet_id=d.get("sessionID", ""),
                   msg_bytes=None if d.get("msgBytes") is None else _b64d(d["msgBytes"]),
                   is_broadcast=bool(d.get("isBroadcast", False)),
                   from_=PartyID.from_json(d.get("from")),
                   to=None if to is None else [PartyID.from_json(p) for p in to],
                   is_to_old_committee=bool(d.get("isToOldCommittee", False)),
                   is_to_old_and_new_committees=bool(d.get("isToOldAndNewCommittees", False)),
                   signature=None if d.get("signature") is None else _b64d(d["signature"]))

    def addressed_to(self, me: PartyID) -> bool:
        """ref:pkg/mpc/session.go:190-192: broadcast with no recipients, or
        exactly one recipient that is this party (ComparePartyIDs: same Id)."""
        if self.is_broadcast and not self.to:
            return True
        return bool(self.to) and len(self.to) == 1 and self.to[0].id == me.id


# --------------------------------------------------------------------------
# LocalPartySaveData (Badger value, JSON)
# --------------------------------------------------------------------------

def _point_json(p: Optional[Tuple[int, int]]):
    return None if p is None else {"Curve": "secp256k1", "Coords": [p[0], p[1]]}


def _point(d) -> Optional[Tuple[int, int]]:
    if d is None:
        return None
    c = d.get("Coords")
    if not isinstance(c, list) or len(c) != 2:
        raise WireError("ECPoint needs two coordinates")
    return int(c[0]), int(c[1])


def _ints(v) -> Optional[List[Optional[int]]]:
    return None if v is None else [None if x is None else int(x) for x in v]


def _opt_int(v) -> Optional[int]:
    return None if v is None else int(v)


@dataclass
class LocalPartySaveData:
    """tss-lib v2.0.2 ecdsa/keygen/save_data.go ``LocalPartySaveData``: the
    embedded LocalPreParams {PaillierSK{N, LambdaN, PhiN, P, Q}, NTildei, H1i,
    H2i, Alpha, Beta, P, Q} and LocalSecrets {Xi, ShareID} promoted to the top
    level, then Ks, NTildej, H1j, H2j, BigXj, PaillierPKs ([{N}]) and ECDSAPub
    ({"Curve", "Coords"}) (upstream, verify). big.Int fields are bare JSON
    numbers (Go big.Int.MarshalJSON)."""
    paillier_sk: Optional[Dict[str, int]]
    NTildei: Optional[int]
    H1i: Optional[int]
    H2i: Optional[int]
    Alpha: Optional[int]
    Beta: Optional[int]
    P: Optional[int]
    Q: Optional[int]
    Xi: Optional[int]
    ShareID: Optional[int]
    Ks: List[Optional[int]]
    NTildej: List[Optional[int]]
    H1j: List[Optional[int]]
    H2j: List[Optional[int]]
    BigXj: List[Optional[Tuple[int, int]]]
    PaillierPKs: List[Optional[int]]
    ECDSAPub: Optional[Tuple[int, int]]

    SK_FIELDS = ("N", "LambdaN", "PhiN", "P", "Q")

    @classmethod
    def from_json(cls, raw) -> "LocalPartySaveData":
        try:
            d = json.loads(raw) if isinstance(raw, (bytes, str)) else raw
        except ValueError as e:
            raise WireError(f"invalid JSON: {e}") from None
        sk = d.get("PaillierSK")
        sk = None if sk is None else {k: _opt_int(sk.get(k)) for k in cls.SK_FIELDS}
        pks = d.get("PaillierPKs")
        out = cls(paillier_sk=sk,
                  **{k: _opt_int(d.get(k)) for k in ("NTildei", "H1i", "H2i", "Alpha", "Beta", "P", "Q", "Xi",
                                                     "ShareID")},
                  Ks=_ints(d.get("Ks")) or [], NTildej=_ints(d.get("NTildej")) or [],
                  H1j=_ints(d.get("H1j")) or [], H2j=_ints(d.get("H2j")) or [],
                  BigXj=[_point(p) for p in (d.get("BigXj") or [])],
                  PaillierPKs=[None if p is None else _opt_int(p.get("N")) for p in (pks or [])],
                  ECDSAPub=_point(d.get("ECDSAPub")))
        return out

    def to_json(self) -> bytes:
        d = {"PaillierSK": None if self.paillier_sk is None else {k: self.paillier_sk.get(k)
                                                                   for k in self.SK_FIELDS}}
        for k in ("NTildei", "H1i", "H2i", "Alpha", "Beta", "P", "Q", "Xi", "ShareID", "Ks", "NTildej", "H1j",
                  "H2j"):
            d[k] = getattr(self, k)
        d["BigXj"] = [_point_json(p) for p in self.BigXj]
        d["PaillierPKs"] = [None if n is None else {"N": n} for n in self.PaillierPKs]
        d["ECDSAPub"] = _point_json(self.ECDSAPub)
        return json.dumps(d, separators=(",", ":")).encode()

    # ---- key material for the batch entry points ----------------------

    def party_index(self) -> int:
        """Position of this party in Ks (tss-lib: the sorted party keys)."""
        try:
            return self.Ks.index(self.ShareID)
        except ValueError:
            raise WireError("ShareID not found in Ks") from None

    def paillier_sk_tuple(self) -> Tuple[int, int, int, int]:
        """(N, LambdaN, P, Q): the `skA` argument of mta.alice_end."""
        sk = self.paillier_sk
        if sk is None or any(sk.get(k) is None for k in ("N", "LambdaN", "P", "Q")):
            raise WireError("PaillierSK incomplete")
        return sk["N"], sk["LambdaN"], sk["P"], sk["Q"]

    def own_dln(self) -> Dict[str, int]:
        """This node's (N~, h1, h2) with its safe primes, the `dlnA` argument of
        mta.alice_end (P = 2p+1, Q = 2q+1 of LocalPreParams.P/Q)."""
        if None in (self.NTildei, self.H1i, self.H2i):
            raise WireError("LocalPreParams incomplete")
        d = {"NTilde": self.NTildei, "h1": self.H1i, "h2": self.H2i}
        if self.P is not None and self.Q is not None:
            d["P"], d["Q"] = 2 * self.P + 1, 2 * self.Q + 1
        return d

    def peer_dln(self, j: int) -> Dict[str, int]:
        """Party j's (N~_j, h1_j, h2_j) as stored in NTildej/H1j/H2j."""
        return {"NTilde": self.NTildej[j], "h1": self.H1j[j], "h2": self.H2j[j]}

    def peer_paillier_n(self, j: int) -> int:
        n = self.PaillierPKs[j]
        if n is None:
            raise WireError(f"PaillierPKs[{j}] missing")
        return n

    def node_preparams(self) -> Dict[str, int]:
        """This node's key material in the form the config-4 driver takes
        (mta.bench_signing_mta nodes; tests/golden/node_preparams.json)."""
        N, lam, P, Q = self.paillier_sk_tuple()
        return {"N": N, "LambdaN": lam, "P": P, "Q": Q, "PhiN": self.paillier_sk.get("PhiN"),
                "NTildei": self.NTildei, "H1i": self.H1i, "H2i": self.H2i, "Alpha": self.Alpha,
                "Beta": self.Beta, "p": self.P, "q": self.Q}


# --------------------------------------------------------------------------
# Batch collection across wallets
# --------------------------------------------------------------------------

@dataclass
class Round1Batch:
    """SignRound1Message1s from one sender, across wallets: the inputs of
    mta.verify_range_alice / mta.bob_mid for that sender's Paillier key."""
    sender: str
    wallet_ids: List[str] = field(default_factory=list)
    c: List[int] = field(default_factory=list)
    proofs: List[Dict[str, int]] = field(default_factory=list)


@dataclass
class Round2Batch:
    """SignRound2Messages from one sender, across wallets: the inputs of
    mta.alice_end (c1 with proof_bob) and mta.alice_end WC (c2 with proof_bob_wc)."""
    sender: str
    wallet_ids: List[str] = field(default_factory=list)
    c1: List[int] = field(default_factory=list)
    c2: List[int] = field(default_factory=list)
    proof_bob: List[Dict[str, object]] = field(default_factory=list)
    proof_bob_wc: List[Dict[str, object]] = field(default_factory=list)


def collect_signing_rounds(raw_msgs: Iterable[bytes], me: PartyID):
    """Decode a stream of TssMessage JSON blobs (any mix of wallets, senders and
    rounds) into per-sender batches of MtA work for this party, keeping the
    messages receiveTssMessage would deliver (ref:pkg/mpc/session.go:190-205).
    Returns (round1 {sender id: Round1Batch}, round2 {sender id: Round2Batch},
    skipped count). Messages that tss-lib would reject raise WireError."""
    r1: Dict[str, Round1Batch] = {}
    r2: Dict[str, Round2Batch] = {}
    skipped = 0
    for raw in raw_msgs:
        m = TssMessage.unmarshal(raw)
        if not m.addressed_to(me) or m.msg_bytes is None or m.from_ is None:
            skipped += 1
            continue
        _, content = parse_wire(m.msg_bytes)
        sender = m.from_.id
        if isinstance(content, SignRound1Message1):
            b = r1.setdefault(sender, Round1Batch(sender))
            b.wallet_ids.append(m.wallet_id)
            b.c.append(content.c)
            b.proofs.append(content.range_proof_alice)
        elif isinstance(content, SignRound2Message):
            b = r2.setdefault(sender, Round2Batch(sender))
            b.wallet_ids.append(m.wallet_id)
            b.c1.append(content.c1)
            b.c2.append(content.c2)
            b.proof_bob.append(content.proof_bob)
            b.proof_bob_wc.append(content.proof_bob_wc)
        else:
            skipped += 1
    return r1, r2, skipped
