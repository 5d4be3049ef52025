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
// Then the rest of GG18 (tss-lib up:ecdsa/signing round_1.go .. round_9.go,
// finalize.go; every step upstream, verify), replayed per wallet and signer i
// from its own GG18 reader CounterDRBG(mix(seed, wallet, 0x100 + i, 4)):
//   round 1: Gamma_i = gamma_i G, (C1_i, D1_i) = commitments.NewHashCommitment(Gamma_i)
//   round 3: delta_i = k_i gamma_i + sum_j (alpha_ij + beta_ji),
//            sigma_i = k_i w_i + sum_j (mu_ij + nu_ji); theta = sum delta_i
//   round 4: schnorr.NewZKProof(Session, gamma_i, Gamma_i)
//   round 5: every peer's D1_j opened against C1_j and its proof verified;
//            R = theta^-1 (Gamma_i + sum_j Gamma_j) = k^-1 G; s_i = m k_i + R.x sigma_i;
//            V_i = s_i R + l_i G, A_i = rho_i G, (C5_i, D5_i) = commitment to (V_i, A_i)
//   round 6: NewZKProof(Session, rho_i, A_i), NewZKVProof(Session, V_i, R, s_i, l_i)
//   round 7: every peer's (V_j, A_j) opened and both proofs verified;
//            V = -m G - r X + sum V_j, A = sum A_j; U_i = rho_i V, T_i = l_i A, commitment C7_i
//   round 9: every peer's (U_j, T_j) opened; sum U == sum T
//   finalize: s = sum s_i (= k (m + r x)), low-s with the recovery id (bit 0 =
//            R.y odd, flipped with s; bit 1 = R.x >= q), ecdsa.Verify(X, m, r, s)
//            by every signer in tss-lib's finalize and again by every node's
//            mpcium session (/root/reference/pkg/mpc/ecdsa_signing_session.go:162),
//            with the wallet key X = sum_i W_i.
// A wallet whose transcript fails any check is aborted (no signature); the
// others are unaffected. Every point equation is a secp::Combine a G + b P +
// c Q, issued as one batch per step over a chunk's wallets.
// One process plays every signer of every wallet: each protocol step is one
// batch per ordered signer pair across a chunk of wallets (the nodes'
// preparams are shared by all wallets, /root/reference/pkg/mpc/node.go:69,109),
// so the measured time is the cluster's whole signing work per signature on
// one GPU. Wallet chunks run as concurrent pipelines (rounds 1-3, then rounds
// 4-9), so one chunk's host work overlaps another chunk's GPU batches.
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
  double finalize_s = 0;                          // rounds 4-9 + finalize (summed over chunks)
  uint64_t signatures = 0, verified = 0;          // signatures produced / passing ecdsa.Verify
  uint64_t aborted = 0;                           // wallets whose GG18 transcript failed a check
};

// Per-session record of `trace_wallets` wallets (parity tests), spread evenly
// over the batch so every concurrent wallet pipeline is sampled: traced wallet
// t is TraceWallet(t, trace_wallets, wallets) = floor(t * wallets / trace_wallets).
// Per ordered pair p (Alice i, Bob j, i-major order) and traced wallet:
//   kTracePairWords words = alpha, beta, mu, nu (8 words each) and
//   SHA512_256i(cA, pfA fields, cB, pfB fields, cB', pfB' fields, u.x, u.y);
// then per traced wallet kTraceSigWords words = r, s (8 words each), recid,
// and the 8-word SHA512_256i of its GG18 transcript: per signer C1, Gamma,
// round-4 proof (alpha, t), C5, V, A, round-6 proofs (alpha, t; alpha, t, u),
// C7, U, T, s_i (oracle/signing_ref.py gg18_rounds); zero when aborted.
constexpr uint32_t kTracePairWords = 40;
constexpr uint32_t kTraceSigWords = 25;
inline size_t TraceWallet(size_t t, size_t traced, size_t wallets) { return t * wallets / traced; }

// Test hooks: corrupt signer 0's round-4 Schnorr proof, round-6 ZKV proof or
// round-7 decommitment in wallet `tamper_wallet` (that wallet must abort).
constexpr int kTamperR4Schnorr = 1, kTamperR6Zkv = 2, kTamperR7Decommit = 3;

// One GG18 signature per wallet for `signers` of the nodes (2 = 2-of-3 with a
// minimal quorum, 3 = every ready peer, mpcium's default): the MtA / MtAwc
// work on the GPU, then rounds 4-9, the signature and its verifications.
MtaStats RunSigning(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed,
                    size_t trace_wallets = 0, std::vector<uint32_t>* trace = nullptr, int64_t tamper_wallet = -1,
                    int tamper_kind = 0);

}  // namespace mpcx::host::signing
