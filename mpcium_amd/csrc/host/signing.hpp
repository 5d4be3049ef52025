// signing.hpp -- the MtA phase of GG18 signing for many wallets at once
// (BASELINE.json config 4: "2-of-3 ECDSA signing across 10k wallets with MtA
// Paillier + range proofs offloaded").
//
// tss-lib v2.0.2 signing (up:ecdsa/signing/round_1.go .. round_3.go), as
// mpcium runs it per wallet (/root/reference/pkg/mpc/ecdsa_signing_session.go:134-147):
//   round 1: every signer i, for every other signer j:
//            (cA_ij, pfA_ij) = AliceInit(pk_i, k_i, N~_j, h1_j, h2_j)
//   round 2: signer j for every i: (beta_ji, cB_ij, piB) = BobMid(pf, gamma_j, cA_ij, ...)
//                                  (nu_ji, cB'_ij, piB') = BobMidWC(pf, w_j, cA_ij, ..., W_j = w_j G)
//   round 3: signer i for every j: alpha_ij = AliceEnd(piB, cA_ij, cB_ij),
//                                  mu_ij = AliceEndWC(piB', cA_ij, cB'_ij, W_j)
// with alpha_ij + beta_ji = k_i gamma_j and mu_ij + nu_ji = k_i w_j (mod q).
// Here one process plays every signer of every wallet: each protocol step is
// one batch per ordered signer pair across all wallets (the nodes' preparams
// are shared by all wallets, /root/reference/pkg/mpc/node.go:69,109), so the
// measured time is the cluster's whole MtA work per signature on one GPU.
// The remaining GG18 rounds (commitments, Schnorr proofs, delta/sigma, the
// final signature) are secp256k1 work outside the Paillier path.
#pragma once

#include <cstdint>
#include <vector>

#include "mta.hpp"
#include "paillier.hpp"

namespace mpcx::host::signing {

struct NodeKeys {
  paillier::PrivateKey sk;  // Paillier key (N, LambdaN, P, Q)
  mta::DLNParams dln;       // own N~, h1, h2 with factors P', Q'
};

struct MtaStats {
  double round1_s = 0, round2_s = 0, round3_s = 0, total_s = 0;
  double engine_busy_s = 0;  // inside libmpcx calls (GPU + transfers), summed over the concurrent tasks
  uint64_t wallets = 0, pairs = 0, sessions = 0;  // sessions = wallets x ordered pairs
  uint64_t errors = 0;                            // non-OK status codes
  uint64_t relation_failures = 0;                 // alpha + beta != k gamma (or mu + nu != k w)
};

// The MtA / MtAwc work of one GG18 signature per wallet, for `signers` of the
// nodes (2 = 2-of-3 with a minimal quorum, 3 = every ready peer, mpcium's default).
MtaStats RunSigningMtA(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed);

}  // namespace mpcx::host::signing
