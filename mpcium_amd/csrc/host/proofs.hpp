// proofs.hpp -- batched mirror of the tss-lib v2.0.2 keygen / reshare proofs
// whose cost is modular exponentiation ("up:" =
// github.com/bnb-chain/tss-lib/v2, pinned at /root/reference/go.mod:10):
//
//   DLN   up:crypto/dlnproof/proof.go   NewDLNProof / (*Proof).Verify (128 iterations;
//         keygen round 1 and up:ecdsa/keygen/dln_verifier.go)
//   Mod   up:crypto/modproof/proof.go   NewProof / (*ProofMod).Verify (80 iterations;
//         Paillier-Blum modulus proof of a node's Paillier N)
//   Fac   up:crypto/facproof/proof.go   NewProof / (*ProofFac).Verify (no small
//         factor proof of N0 = Paillier N over a verifier's (N~, h1, h2))
//
// Each batch holds many proofs over the same public parameters (a node's N~ /
// N and a peer's N~ are fixed for the node's lifetime,
// /root/reference/pkg/mpc/node.go:69,109): keygen and reshare sessions under
// load (BASELINE.json config 5) prove and verify these for every session.
// Every exponentiation runs on the GPU (ExpSet). Results equal the per-proof
// Go functions for the same io.Reader stream (oracle/proofs_ref.py restates
// them; parity vs tss-lib itself is unpinned).
//
// Bit-exact shortcuts: h2^c with c in {0, 1} is 1 or h2 (DLN verify); the
// quadratic-residue tests of the Mod prover run as Euler-criterion Legendre
// symbols mod P and Q on the GPU (equal to Go's Jacobi for prime moduli),
// combined multiplicatively over the four candidates (-1)^a W^b Y; N's
// compositeness in Mod verify (Go: N.ProbablyPrime(30) -> reject) is
// ProbablyPrimeBatch(N, 30): Miller-Rabin with base 2 and 30 further bases on
// the GPU (a 2048-bit N is beyond the Lucas kernel's class; a composite N
// passing 31 rounds is the only divergence from Go, and would make the
// verifier reject, never accept).
#pragma once

#include <cstdint>
#include <vector>

#include "bignum.hpp"
#include "tsscommon.hpp"

namespace mpcx::host::proofs {

using Bytes = std::vector<uint8_t>;

constexpr int kDLNIterations = 128;
constexpr int kModIterations = 80;

struct DLNProof {
  std::vector<Nat> Alpha, T;  // kDLNIterations each
};

// NewDLNProof(h1, h2, x, p, q, N, rand[i]) for i < rand.size()
std::vector<DLNProof> DLNProveBatch(const Nat& h1, const Nat& h2, const Nat& x, const Nat& p, const Nat& q,
                                    const Nat& N, const std::vector<RandFn>& rand);
// (*Proof).Verify(h1, h2, N) for every proof
std::vector<uint8_t> DLNVerifyBatch(const Nat& h1, const Nat& h2, const Nat& N, const std::vector<DLNProof>& pf);

struct ModProof {
  Nat W, A, B;
  std::vector<Nat> X, Z;  // kModIterations each
};

// modproof.NewProof(Session[i], N, P, Q, rand[i])
std::vector<ModProof> ModProveBatch(const std::vector<Bytes>& session, const Nat& N, const Nat& P, const Nat& Q,
                                    const std::vector<RandFn>& rand);
// (*ProofMod).Verify(Session[i], N)
std::vector<uint8_t> ModVerifyBatch(const std::vector<Bytes>& session, const Nat& N, const std::vector<ModProof>& pf);

struct FacProof {
  Nat P, Q, A, B, T, Sigma, Z1, Z2, W1, W2;
  Int V;  // e (sigma - nu N0p) + r: negative when sigma < nu N0p
};

// facproof.NewProof(Session[i], ec, N0, NCap, s, t, N0p, N0q, rand[i])
std::vector<FacProof> FacProveBatch(const std::vector<Bytes>& session, const Nat& N0, const Nat& NCap, const Nat& s,
                                    const Nat& t, const Nat& N0p, const Nat& N0q, const std::vector<RandFn>& rand);
// (*ProofFac).Verify(Session[i], ec, N0, NCap, s, t)
std::vector<uint8_t> FacVerifyBatch(const std::vector<Bytes>& session, const Nat& N0, const Nat& NCap, const Nat& s,
                                    const Nat& t, const std::vector<FacProof>& pf);

}  // namespace mpcx::host::proofs
