// mta.hpp -- batched mirror of tss-lib v2.0.2's MtA / MtAwc sub-protocol of
// GG18 ECDSA signing ("up:" =
// github.com/bnb-chain/tss-lib/v2, pinned at /root/reference/go.mod:10):
//
//   AliceInit          up:crypto/mta/share_protocol.go  (Encrypt + ProveRangeAlice)
//   BobMid / BobMidWC  up:crypto/mta/share_protocol.go  (Verify + Encrypt + HomoMult
//                                                        + HomoAdd + ProveBob[WC])
//   AliceEnd[WC]       up:crypto/mta/share_protocol.go  (ProofBob[WC].Verify + Decrypt)
//   ProveRangeAlice, RangeProofAlice.Verify             up:crypto/mta/range_proof.go
//   ProveBob[WC], ProofBob[WC].Verify                   up:crypto/mta/proofs.go
//
// Each function takes a batch of independent sessions that share key material
// (one Paillier key, one verifier's N~, h1, h2) -- the shape of mpcium's
// signing sessions, which all reuse the nodes' preparams
// (/root/reference/pkg/mpc/node.go:69,109) -- and runs every exponentiation of
// the batch on the GPU in a few launches per protocol step (ExpSet). Per
// session results are identical to the per-session Go functions for the same
// io.Reader stream (oracle/mta_ref.py restates them; parity vs tss-lib itself
// is unpinned).
//
// Bit-exact rewrites (no change to any output or decision):
//   * Gamma^k mod N^2 = 1 + (k mod N)*N  (Gamma = N + 1), not a modexp;
//   * products of two powers run as one fused launch (base^e * mul);
//   * RangeProofAlice.Verify's u == Gamma^s1 s^N c^-e (resp. w == h1^s1 h2^s2
//     z^-e) is checked as u c^e == Gamma^s1 s^N (resp. w z^e == h1^s1 h2^s2):
//     equivalent for invertible c, z (z by the gcd check; c is checked here --
//     where Go's Exp returns nil for a non-invertible c and the following Mul
//     panics, this mirror reports a verification failure);
//   * gcd(x, N~) == 1 for the caller's OWN N~ (factors known) is tested as
//     P' !| x and Q' !| x.
#pragma once

#include <cstdint>
#include <vector>

#include "bignum.hpp"
#include "paillier.hpp"
#include "secp256k1.hpp"
#include "tsscommon.hpp"

namespace mpcx::host::mta {

// A verifier's DLN parameters (N~, h1, h2). P, Q: the safe-prime factors of
// N~ when the caller owns them (own preparams: faster gcd checks), else 0.
struct DLNParams {
  Nat NTilde, h1, h2;
  Nat P, Q;
};

struct RangeProofAlice {
  Nat Z, U, W, S, S1, S2;
};

struct ProofBob {
  Nat Z, ZPrm, T, V, W, S, S1, S2, T1, T2;
  secp::Affine U;  // ProofBobWC.U (infinity for the plain ProofBob)
};

enum Status : uint8_t {
  OK = 0,
  ErrMessageTooLong = 1,   // paillier.ErrMessageTooLong
  ErrMessageMalFormed = 2, // paillier.ErrMessageMalFormed
  ErrProofVerify = 3,      // "RangeProofAlice.Verify() returned false" / "ProofBob.Verify() returned false"
};

// Session ids (the tss-lib `Session []byte` of BobMid/AliceEnd).
using Bytes = std::vector<uint8_t>;

// ---- proofs (batches; rand[i] is session i's io.Reader)
void ProveRangeAliceBatch(const paillier::PublicKey& pk, const DLNParams& dln, const std::vector<Nat>& c,
                          const std::vector<Nat>& m, const std::vector<Nat>& r, const std::vector<RandFn>& rand,
                          std::vector<RangeProofAlice>* out);
std::vector<uint8_t> VerifyRangeAliceBatch(const paillier::PublicKey& pk, const DLNParams& dln,
                                           const std::vector<Nat>& c, const std::vector<RangeProofAlice>& pf);

// X == nullptr: ProveBob; else ProveBobWC with X[i]
void ProveBobBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pk, const DLNParams& dln,
                   const std::vector<Nat>& c1, const std::vector<Nat>& c2, const std::vector<Nat>& x,
                   const std::vector<Nat>& y, const std::vector<Nat>& r, const std::vector<secp::Affine>* X,
                   const std::vector<RandFn>& rand, std::vector<ProofBob>* out);
// own_sk: the caller's Paillier key when pk is its own (gcd shortcuts), else nullptr
std::vector<uint8_t> VerifyBobBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pk,
                                    const DLNParams& dln, const std::vector<Nat>& c1, const std::vector<Nat>& c2,
                                    const std::vector<ProofBob>& pf, const std::vector<secp::Affine>* X,
                                    const paillier::PrivateKey* own_sk = nullptr);

// ---- protocol
// AliceInit(ec, pkA, a, NTildeB, h1B, h2B, rand) -> (cA, pf, err). skA: Alice's
// own private key when the caller holds it (it always does in tss-lib: AliceInit
// runs on Alice's node): Encrypt's r^N and the proof's beta^N then run mod P^2 and
// Q^2 with a CRT recombination -- bit-exact, half the GPU work.
void AliceInitBatch(const paillier::PublicKey& pkA, const std::vector<Nat>& a, const DLNParams& dlnB,
                    const std::vector<RandFn>& rand, std::vector<Nat>* cA, std::vector<RangeProofAlice>* pf,
                    std::vector<uint8_t>* err, const paillier::PrivateKey* skA = nullptr);

struct BobMidResult {
  Nat beta, cB, betaPrm;
  ProofBob pf;
};
// BobMid (B == nullptr) / BobMidWC (B[i] = Bob's public point) -- dlnA: Alice's
// N~ (for ProveBob), dlnB: Bob's own (for RangeProofAlice.Verify).
void BobMidBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pkA,
                 const std::vector<RangeProofAlice>& pf, const std::vector<Nat>& b, const std::vector<Nat>& cA,
                 const DLNParams& dlnA, const DLNParams& dlnB, const std::vector<secp::Affine>* B,
                 const std::vector<RandFn>& rand, std::vector<BobMidResult>* out, std::vector<uint8_t>* err);

// BobMid (b, rand) and BobMidWC (bwc, Bwc, randwc) on the same Alice message,
// as tss-lib's signing round 2 runs both per peer (up:ecdsa/signing/round_2.go):
// RangeProofAlice.Verify once for both (the same pure decision twice in Go),
// then the two halves as concurrent tasks; every output equals the two
// separate calls'. serial_halves: the halves share reader objects (one
// io.Reader per session for both) -- BobMid runs to completion first, so the
// draws are those of BobMid then BobMidWC called in that order.
void BobMidPairBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pkA,
                     const std::vector<RangeProofAlice>& pf, const std::vector<Nat>& b, const std::vector<Nat>& bwc,
                     const std::vector<Nat>& cA, const DLNParams& dlnA, const DLNParams& dlnB,
                     const std::vector<secp::Affine>& Bwc, const std::vector<RandFn>& rand,
                     const std::vector<RandFn>& randwc, std::vector<BobMidResult>* out,
                     std::vector<BobMidResult>* outwc, std::vector<uint8_t>* err, std::vector<uint8_t>* errwc,
                     bool serial_halves = false);

// AliceEnd (B == nullptr) / AliceEndWC -> alpha = Decrypt(cB) mod q
void AliceEndBatch(const std::vector<Bytes>& session, const paillier::PrivateKey& skA,
                   const std::vector<ProofBob>& pf, const DLNParams& dlnA, const std::vector<Nat>& cA,
                   const std::vector<Nat>& cB, const std::vector<secp::Affine>* B, std::vector<Nat>* alpha,
                   std::vector<uint8_t>* err);

// AliceEnd (pf, cB -> alpha) and AliceEndWC (pfwc, cBwc, Bwc -> mu) of one
// pair, as signing round 3 runs both per peer (up:ecdsa/signing/round_3.go):
// the two halves as concurrent tasks.
void AliceEndPairBatch(const std::vector<Bytes>& session, const paillier::PrivateKey& skA,
                       const std::vector<ProofBob>& pf, const std::vector<ProofBob>& pfwc, const DLNParams& dlnA,
                       const std::vector<Nat>& cA, const std::vector<Nat>& cB, const std::vector<Nat>& cBwc,
                       const std::vector<secp::Affine>& Bwc, std::vector<Nat>* alpha, std::vector<Nat>* mu,
                       std::vector<uint8_t>* err, std::vector<uint8_t>* errwc);

// q = secp256k1 group order (ec.Params().N)
const Nat& Q();

}  // namespace mpcx::host::mta
