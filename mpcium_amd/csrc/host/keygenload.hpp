// keygenload.hpp -- the proof work of ECDSA keygen / reshare sessions under
// load (BASELINE.json config 5: "3-of-5 ECDSA reshare + keygen under load
// (mixed proof verification batches)").
//
// tss-lib v2.0.2 keygen (up:ecdsa/keygen/round_1.go .. round_3.go), as mpcium
// runs it per wallet (/root/reference/pkg/mpc/ecdsa_keygen_session.go:85-92),
// and resharing's new committee (up:ecdsa/resharing, mpcium:
// /root/reference/pkg/mpc/ecdsa_resharing_session.go:135-143) give every
// party i of n, per session:
//   prove : two DLN proofs over its own (N~_i, h1_i, h2_i) -- (h1, h2, alpha)
//           and (h2, h1, beta) (up:crypto/dlnproof, 128 iterations);
//           a Paillier-Blum modulus proof of N_i (up:crypto/modproof, 80 it.);
//           a no-small-factor proof of N_i to every peer j over
//           (N~_j, h1_j, h2_j) (up:crypto/facproof);
//   verify: every peer's two DLN proofs and Mod proof, and the Fac proof the
//           peer addressed to it.
// The node key material (Paillier keys, N~, h1, h2) is fixed per node
// (/root/reference/pkg/mpc/node.go:69,109), so a node's proofs across
// sessions are batches over the same public parameters. One process plays
// all n parties of all sessions, so the time is the whole cluster's proof
// work per session on one GPU. Which round sends which proof, and the
// resharing rounds' exact mix, are upstream details not checkable here
// (tss-lib is not vendored); the per-party mix above is what DESIGN.md
// measures.
#pragma once

#include <cstdint>
#include <vector>

#include "paillier.hpp"

namespace mpcx::host::keygenload {

struct PartyKeys {
  paillier::PrivateKey sk;                  // N, LambdaN, P, Q
  Nat NTilde, h1, h2, alpha, beta, p, q;    // DLN params: h2 = h1^alpha, N~ = (2p+1)(2q+1)
};

struct ProofStats {
  double prove_s = 0, verify_s = 0, total_s = 0, engine_busy_s = 0;
  double alg_macs = 0;  // Go-equivalent algorithmic work sent to the GPU (Engine::alg_macs)
  uint64_t sessions = 0, parties = 0, proofs = 0, verifications = 0;
  uint64_t failures = 0;  // verifications that did not pass (honest proofs: must be 0)
  uint64_t waves = 0, wave_sessions = 0;
  double max_wave_s = 0;  // slowest wave, prove + verify
  // mixed runs (reshare_mix): sessions and summed wave wall time per kind, and
  // the old committee's VSS checks (decommitment + share + public key)
  uint64_t keygen_sessions = 0, reshare_sessions = 0;
  double keygen_wave_s = 0, reshare_wave_s = 0;
  uint64_t vss_checks = 0, vss_failures = 0;
};

// ---- resharing as mpcium runs it: every node runs TWO resharing sessions per
// wallet, as an old party and as a new party
// (/root/reference/pkg/eventconsumer/event_consumer.go:407-416,
// /root/reference/pkg/mpc/ecdsa_resharing_session.go:114-138). Old = new
// committee = the n ready peers (ids 1..n), new threshold kReshareThreshold
// (3-of-5). Per session, as recalled from tss-lib v2.0.2 up:ecdsa/resharing
// (not vendored: "upstream, verify"):
//   old party i: w_i = lambda_i x_i (its Lagrange-weighted share of the wallet
//     key), vss.Create(t, w_i): coefficients a_1..a_t < q drawn from its
//     reader, then a hash commitment to V_ik = a_k G (r = MustGetRandomInt(256)
//     drawn after them); shares s_ij = f_i(j) to every new party j;
//   new party j: the new-committee proof work (identical to keygen's: DLN x2,
//     Mod, Fac per peer, proved and verified) and, for every old party i, the
//     decommitment and s_ij G == sum_k V_ik j^k, then x'_j = sum_i s_ij and
//     sum_i V_i0 == X (the wallet key).
// The wallet's old shares are a degree-t polynomial of a seeded stream.
constexpr size_t kReshareThreshold = 2;
// extra trace words of a reshare wave's traced session: per old party an 8-word
// SHA512_256i(C_i, V_i0.x, V_i0.y, .., V_it.y, s_i1 .. s_in), the 8-word digest
// of the new shares x'_1 .. x'_n, and the number of VSS checks that passed
inline size_t TraceVssWords(size_t n) { return n * 8 + 8 + 1; }

// Sessions stream through in waves of `wave_sessions` (<= 0: kDefaultWave),
// kWavesInFlight at a time: a wave's proofs are built, verified by every peer
// and dropped before a later wave starts, so host memory is bounded by the
// waves in flight (~0.9 MB of proofs per 5-party session), not by `sessions`
// -- mpcium's keygen / reshare consumers run sessions as they arrive
// (/root/reference/pkg/eventconsumer/event_consumer.go:103-204,375-518).
// Every session's streams and session id are functions of (seed, session
// index), so the wave size changes no proof.
constexpr size_t kDefaultWave = 1024;
constexpr size_t kWavesInFlight = 2;

// Trace of one session per wave (parity tests): session
// TracedSession(w, lo, hi) of wave w = [lo, hi), then per party i: 8-word
// digests SHA512_256i of its DLN proof (h1, h2, alpha) (Alpha[], T[]), its DLN
// proof (h2, h1, beta), its ModProof (W, A, B, X[], Z[]), and per peer j != i
// (ascending) of its FacProof to j (P, Q, A, B, T, Sigma, Z1, Z2, W1, W2, |V|,
// V < 0); a final word = the number of that session's verifications that
// passed.
inline size_t TraceSessionWords(size_t n) { return 1 + n * (3 + (n - 1)) * 8 + 1; }
inline size_t TracedSession(size_t wave, size_t lo, size_t hi) { return lo + (wave * 7919u) % (hi - lo); }

// reshare_mix: 0 -- every wave a keygen wave; 1 -- odd waves are resharing
// waves (the new committee's proof work + the old committee's VSS), so the two
// waves in flight are one of each kind (config 5: "reshare + keygen under
// load"). Trace: TraceSessionWords(n) + (reshare_mix ? TraceVssWords(n) : 0)
// words per wave (the VSS words zero on keygen waves).
// tamper_session >= 0 (test hook): in that resharing session old party 0 sends
// new party 1 a share off by one -- exactly one VSS check fails, nothing else.
ProofStats RunKeygenProofs(const std::vector<PartyKeys>& parties, size_t sessions, uint64_t seed,
                           size_t wave_sessions = 0, std::vector<uint32_t>* trace = nullptr, int reshare_mix = 0,
                           int64_t tamper_session = -1);

}  // namespace mpcx::host::keygenload
