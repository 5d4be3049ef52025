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
// Then the signature, from the MtA outputs (GG18 phase 4-5 algebra, tss-lib's
// up:ecdsa/signing round 4-9 + finalize):
//   delta_i = k_i gamma_i + sum_j (alpha_ij + beta_ij),  delta = sum delta_i = k gamma
//   sigma_i = k_i w_i + sum_j (mu_ij + nu_ij),           sigma = k x
//   R = delta^-1 * sum_i gamma_i G = k^-1 G,  r = R.x mod q
//   s = sum_i (m k_i + r sigma_i) = k (m + r x) mod q, normalised to s <= q/2
//       (recovery id bit 0 = R.y odd, flipped with s; bit 1 = R.x >= q)
// and every signature is checked as mpcium does after the party ends:
// ecdsa.Verify(X, m.Bytes(), r, s) with the wallet key X = sum_i w_i G
// (/root/reference/pkg/mpc/ecdsa_signing_session.go:162). (r, s) is a
// deterministic function of (k_i, gamma_i, w_i, m): phase 5's commitments and
// Schnorr proofs (round 5-9) check consistency without changing it and carry
// no Paillier work, so they are not replayed here.
// One process plays every signer of every wallet: each protocol step is one
// batch per ordered signer pair across a chunk of wallets (the nodes'
// preparams are shared by all wallets, /root/reference/pkg/mpc/node.go:69,109),
// so the measured time is the cluster's whole signing work per signature on
// one GPU. Wallet chunks run as concurrent pipelines (rounds 1-3, then the
// finalize), so one chunk's host work overlaps another's GPU batches.
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
  double round1_s = 0, round2_s = 0, round3_s = 0, total_s = 0;  // rounds: per pair chain (mean over pairs), summed over chunks
  double engine_busy_s = 0;  // wall time with >= 1 libmpcx call in flight (GPU + transfers)
  double alg_macs = 0;       // Go-equivalent algorithmic work sent to the GPU (Engine::alg_macs)
  uint64_t wallets = 0, pairs = 0, sessions = 0;  // sessions = wallets x ordered pairs
  uint64_t errors = 0;                            // non-OK status codes
  uint64_t relation_failures = 0;                 // alpha + beta != k gamma (or mu + nu != k w)
  double finalize_s = 0;                          // rounds 4-9 + ecdsa.Verify on the host (summed over chunks)
  uint64_t signatures = 0, verified = 0;          // signatures produced / passing ecdsa.Verify
};

// Per-session record of `trace_wallets` wallets (parity tests), spread evenly
// over the batch so every concurrent wallet pipeline is sampled: traced wallet
// t is TraceWallet(t, trace_wallets, wallets) = floor(t * wallets / trace_wallets).
// Per ordered pair p (Alice i, Bob j, i-major order) and traced wallet:
//   kTracePairWords words = alpha, beta, mu, nu (8 words each) and
//   SHA512_256i(cA, pfA fields, cB, pfB fields, cB', pfB' fields, u.x, u.y);
// then per wallet kTraceSigWords words = r, s (8 words each), recid.
constexpr uint32_t kTracePairWords = 40;
constexpr uint32_t kTraceSigWords = 17;
inline size_t TraceWallet(size_t t, size_t traced, size_t wallets) { return t * wallets / traced; }

// One GG18 signature per wallet for `signers` of the nodes (2 = 2-of-3 with a
// minimal quorum, 3 = every ready peer, mpcium's default): the MtA / MtAwc
// work on the GPU, then the signature and its verification on the host.
MtaStats RunSigning(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed,
                    size_t trace_wallets = 0, std::vector<uint32_t>* trace = nullptr);

}  // namespace mpcx::host::signing
