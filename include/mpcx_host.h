/*
 * mpcx_host.h -- C surface of libmpcx_host.so, the C++ mirror of the
 * reference's modexp-calling interfaces (tss-lib v2.0.2, pinned at
 * /root/reference/go.mod:10; Go/tss-lib are absent from this image, so the
 * host side that would be Go is C++ here). Every exponentiation goes through
 * libmpcx.so (include/mpcx.h). Integers: little-endian 32-bit words with a
 * separate sign byte array where Go accepts negative *big.Int values.
 * Return codes are the MPCX_* codes of mpcx.h; mpcxh_last_error() has text.
 *
 * Reference interface each entry point mirrors:
 *   mpcxh_modint_exp_batch       up:common/int.go (*modInt).Exp -> Go (*Int).Exp
 *   mpcxh_paillier_*_batch       up:crypto/paillier/paillier.go
 *                                (EncryptAndReturnRandomness, HomoMult,
 *                                 HomoAdd, Decrypt; per-op error codes
 *                                 1 = ErrMessageTooLong, 2 = ErrMessageMalFormed)
 *   mpcxh_safe_primes            up:common/safe_prime.go GetRandomSafePrimesConcurrent
 *   mpcxh_safe_prime_batch       up:common/safe_prime.go runGenPrimeRoutine (one stream batch, sharded)
 *   mpcxh_generate_preparams     up:ecdsa/keygen/prepare.go GeneratePreParams,
 *                                called at /root/reference/pkg/mpc/node.go:69
 *   mpcxh_dln_*, mpcxh_mod_*,    up:crypto/dlnproof, up:crypto/modproof,
 *   mpcxh_fac_*_batch            up:crypto/facproof (keygen / reshare proofs)
 *   mpcxh_mta_*_batch            up:crypto/mta/{share_protocol,range_proof,proofs}.go
 *                                (AliceInit, BobMid[WC], AliceEnd[WC], the
 *                                 range / Bob proofs and their Verify)
 */
#ifndef MPCX_HOST_H_
#define MPCX_HOST_H_

#include <stddef.h>
#include <stdint.h>

#include "mpcx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* io.Reader stand-in: fill buf[0..n) with random bytes (io.ReadFull). */
typedef void (*mpcxh_rand_fn)(void* ctx, uint8_t* buf, size_t n);

/* One session's randomness source: tss-lib draws every MtA / proof random
 * value from the party's io.Reader inside party.UpdateFromBytes
 * (/root/reference/pkg/mpc/session.go:199). fn != NULL: fn(ctx, ...) is that
 * reader (a cgo export wrapping the Go io.Reader); it is
 * called from libmpcx_host's worker threads, never concurrently for one
 * session, but concurrently across sessions (a reader shared by several
 * sessions must be thread-safe, as crypto/rand.Reader is). fn == NULL: the
 * build's CounterDRBG stream seeded with `seed` (tests, benchmarks). */
typedef struct {
  mpcxh_rand_fn fn;
  void* ctx;
  uint64_t seed;
} mpcxh_reader_t;

#define MPCXH_PREPARAM_FIELDS 12

const char* mpcxh_last_error(void);
/* Bind one more GPU (mpcx_init) / GPUs 0..n_gpus-1 (mpcx_init_devices, n_gpus
 * <= 0: all visible). Every batch below spreads over the bound GPUs. */
int mpcxh_init(int device);
int mpcxh_init_devices(int n_gpus);

/* z_i = x_i^y_i mod m with Go semantics; ok[i] = 0 where Go returns nil
 * (y < 0 and x not invertible). y_shared != 0: one y for every x. m odd,
 * 1 <= m < 2^4096. */
int mpcxh_modint_exp_batch(const uint32_t* m, uint32_t mw, uint32_t count,
                           const uint32_t* xs, uint32_t xw, const uint8_t* x_neg,
                           const uint32_t* ys, uint32_t yw, const uint8_t* y_neg, int y_shared,
                           uint32_t* out, uint32_t ow, uint8_t* ok);

int mpcxh_paillier_encrypt_batch(const uint32_t* N, uint32_t nw, uint32_t count,
                                 const uint32_t* m, uint32_t mw, const uint8_t* m_neg,
                                 const uint32_t* r, uint32_t rw,
                                 uint32_t* c, uint32_t cw, uint8_t* err);
int mpcxh_paillier_homomult_batch(const uint32_t* N, uint32_t nw, uint32_t count,
                                  const uint32_t* m, uint32_t mw, const uint8_t* m_neg,
                                  const uint32_t* c1, uint32_t c1w, const uint8_t* c1_neg,
                                  uint32_t* out, uint32_t ow, uint8_t* err);
int mpcxh_paillier_homoadd_batch(const uint32_t* N, uint32_t nw, uint32_t count,
                                 const uint32_t* c1, uint32_t c1w, const uint8_t* c1_neg,
                                 const uint32_t* c2, uint32_t c2w, const uint8_t* c2_neg,
                                 uint32_t* out, uint32_t ow, uint8_t* err);
int mpcxh_paillier_decrypt_batch(const uint32_t* N, uint32_t nw, const uint32_t* lambda, uint32_t lw,
                                 const uint32_t* P, uint32_t pw, const uint32_t* Q, uint32_t qw,
                                 uint32_t count, const uint32_t* c, uint32_t cw, const uint8_t* c_neg,
                                 uint32_t* m, uint32_t mw, uint8_t* err);

/* First `num` safe primes p = 2q+1 of bit_len bits in candidate-stream order.
 * Random source: rand_fn(rand_ctx, ...) if non-NULL (read on the host), else
 * the CounterDRBG seeded with `seed` (drawn on the GPU). p_out/q_out: num x
 * words. index_out: stream positions. stats_out[6]: candidates, sieved out,
 * GPU Fermat tests, GPU Miller-Rabin rounds, usec, GPU strong Lucas tests. */
int mpcxh_safe_primes(int bit_len, int num, uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx,
                      uint32_t* p_out, uint32_t* q_out, uint32_t words, uint64_t* index_out,
                      uint64_t* stats_out);

/* One batch of the same search for sharding across GPUs (up:common/safe_prime.go
 * runGenPrimeRoutine, one batch of its candidate stream): candidates
 * [batch_no*batch, (batch_no+1)*batch) of the CounterDRBG(seed) stream
 * (batch 0 = default 196608). Writes up to max_out accepted primes in stream
 * order and their count to *n_found. Rank g of G takes batch_no = g (mod G);
 * the first `num` indices over all ranks equal mpcxh_safe_primes' output. */
int mpcxh_safe_prime_batch(int bit_len, uint64_t seed, uint64_t batch_no, uint32_t batch, uint32_t max_out,
                           uint32_t* p_out, uint32_t* q_out, uint32_t words, uint64_t* index_out,
                           uint32_t* n_found, uint64_t* stats_out);

/* LocalPreParams as 12 fields x 64 words: N, LambdaN, PhiN, P, Q (Paillier),
 * NTildei, H1i, H2i, Alpha, Beta, P, Q (Germain primes of N~). One stream:
 * the Paillier search, then N~'s, then f and alpha; each search consumes the
 * stream up to its last accepted candidate, as tss-lib at concurrency 1.
 * stats_out[6] as mpcxh_safe_primes. */
int mpcxh_generate_preparams(uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx,
                             uint32_t* out, uint64_t* stats_out);

/* ---------------------------------------------------------------- MtA
 * Batched mirror of tss-lib v2.0.2's MtA / MtAwc (up:crypto/mta/share_protocol.go,
 * range_proof.go, proofs.go), the Paillier work of GG18 signing that mpcium's
 * signing sessions (/root/reference/pkg/mpc/ecdsa_signing_session.go:134-147)
 * run through party.UpdateFromBytes (/root/reference/pkg/mpc/session.go:199).
 * One call = a batch of independent sessions sharing key material. Every
 * integer is `w` little-endian 32-bit words (w >= 128: N^2 fits); proofs are
 * count x fields x w words:
 *   RangeProofAlice (6 fields): Z, U, W, S, S1, S2
 *   ProofBob[WC]   (12 fields): Z, ZPrm, T, V, W, S, S1, S2, T1, T2, U.x, U.y
 *                               (U = 0, 0 for the plain ProofBob)
 * Points (B, the MtAwc public value) are count x 16 words: x (8), y (8).
 * Session ids are count x session_len bytes. readers[i]: session i's
 * io.Reader. err[i]: 0 ok, 1 ErrMessageTooLong, 2
 * ErrMessageMalFormed, 3 proof verification failed. */
typedef struct {
  const uint32_t* N;       /* Paillier N */
  const uint32_t* LambdaN; /* private-key fields: NULL for a peer's public key */
  const uint32_t* P;
  const uint32_t* Q;
} mpcxh_paillier_t;

typedef struct {
  const uint32_t* NTilde;
  const uint32_t* h1;
  const uint32_t* h2;
  const uint32_t* P; /* safe-prime factors of NTilde when the caller owns it, else NULL */
  const uint32_t* Q;
} mpcxh_dln_t;

#define MPCXH_RANGE_PROOF_FIELDS 6
#define MPCXH_PROOF_BOB_FIELDS 12

/* mta.AliceInit(ec, pkA, a, NTildeB, h1B, h2B, rand) -> cA, RangeProofAlice */
int mpcxh_mta_alice_init_batch(uint32_t w, const mpcxh_paillier_t* pkA, const mpcxh_dln_t* dlnB, uint32_t count,
                               const uint32_t* a, const mpcxh_reader_t* readers, uint32_t* cA, uint32_t* pf,
                               uint8_t* err);
/* (*RangeProofAlice).Verify(ec, pk, NTilde, h1, h2, c) */
int mpcxh_mta_verify_range_alice_batch(uint32_t w, const mpcxh_paillier_t* pk, const mpcxh_dln_t* dln,
                                       uint32_t count, const uint32_t* c, const uint32_t* pf, uint8_t* ok);
/* mta.BobMid (B == NULL) / BobMidWC(Session, ec, pkA, pf, b, cA, NTildeA, h1A, h2A,
 * NTildeB, h1B, h2B[, B], rand) -> beta, cB, betaPrm, ProofBob[WC] */
int mpcxh_mta_bob_mid_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const mpcxh_paillier_t* pkA,
                            const mpcxh_dln_t* dlnA, const mpcxh_dln_t* dlnB, uint32_t count, const uint32_t* pfA,
                            const uint32_t* b, const uint32_t* cA, const uint32_t* B,
                            const mpcxh_reader_t* readers, uint32_t* beta, uint32_t* cB, uint32_t* betaPrm,
                            uint32_t* pfB, uint8_t* err);
/* (*ProofBob).Verify / (*ProofBobWC).Verify(Session, ec, pk, NTilde, h1, h2, c1, c2[, X]) */
int mpcxh_mta_verify_bob_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const mpcxh_paillier_t* pk,
                               const mpcxh_dln_t* dln, uint32_t count, const uint32_t* c1, const uint32_t* c2,
                               const uint32_t* pfB, const uint32_t* X, uint8_t* ok);
/* mta.AliceEnd (B == NULL) / AliceEndWC(Session, ec, pkA, pf, h1A, h2A, cA, cB, NTildeA[, B], sk) -> alpha */
int mpcxh_mta_alice_end_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const mpcxh_paillier_t* skA,
                              const mpcxh_dln_t* dlnA, uint32_t count, const uint32_t* pfB, const uint32_t* cA,
                              const uint32_t* cB, const uint32_t* B, uint32_t* alpha, uint8_t* err);

/* Signing round 2 runs BobMid and BobMidWC on every peer's round-1 message
 * (up:ecdsa/signing/round_2.go): both halves of each session in one call,
 * RangeProofAlice.Verify once for both. b / readers / beta / cB / betaPrm /
 * pfB / err: the BobMid half; bwc, Bwc, readers_wc, *_wc: the BobMidWC half.
 * With distinct readers the two halves run concurrently (readers[i] and
 * readers_wc[i] may then be called at the same time); when readers[i] and
 * readers_wc[i] are the same callback (same fn and ctx) for any session, the
 * halves run one after the other, BobMid first. Every output equals the two
 * separate calls' (BobMid, then BobMidWC). */
int mpcxh_mta_bob_mid_pair_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len,
                                 const mpcxh_paillier_t* pkA, const mpcxh_dln_t* dlnA, const mpcxh_dln_t* dlnB,
                                 uint32_t count, const uint32_t* pfA, const uint32_t* cA, const uint32_t* b,
                                 const mpcxh_reader_t* readers, const uint32_t* bwc, const uint32_t* Bwc,
                                 const mpcxh_reader_t* readers_wc, uint32_t* beta, uint32_t* cB, uint32_t* betaPrm,
                                 uint32_t* pfB, uint8_t* err, uint32_t* beta_wc, uint32_t* cB_wc,
                                 uint32_t* betaPrm_wc, uint32_t* pfB_wc, uint8_t* err_wc);
/* Signing round 3's AliceEnd and AliceEndWC per peer (up:ecdsa/signing/round_3.go)
 * in one call: each half's ProofBob[WC] verification and Decrypt batch, the two
 * halves as concurrent tasks (no reader is involved). */
int mpcxh_mta_alice_end_pair_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len,
                                   const mpcxh_paillier_t* skA, const mpcxh_dln_t* dlnA, uint32_t count,
                                   const uint32_t* cA, const uint32_t* pfB, const uint32_t* cB,
                                   const uint32_t* pfB_wc, const uint32_t* cB_wc, const uint32_t* Bwc,
                                   uint32_t* alpha, uint8_t* err, uint32_t* mu, uint8_t* err_wc);

/* ---------------------------------------------------------------- keygen proofs
 * Batched mirror of tss-lib v2.0.2's DLN (up:crypto/dlnproof, 128 iterations),
 * Paillier-Blum modulus (up:crypto/modproof, 80 iterations) and no-small-factor
 * (up:crypto/facproof) proofs: keygen round 1-3 and reshare
 * (/root/reference/pkg/mpc/ecdsa_keygen_session.go:85-92,
 * /root/reference/pkg/mpc/ecdsa_resharing_session.go:132-143). A batch holds
 * `count` proofs over the same public parameters; integers are `w` words
 * (w >= 160: FacProof's v and sigma reach ~4.9 kbit), readers[i] is proof i's
 * io.Reader, sessions are count x session_len bytes.
 *   DLN proof: alpha (count x 128 x w), t (count x 128 x w)
 *   Mod proof: W (count x w), X (count x 80 x w), A, B (count x w), Z (count x 80 x w)
 *   Fac proof: count x 11 x w fields P, Q, A, B, T, Sigma, Z1, Z2, W1, W2, |V|
 *              and v_neg[count] (sign of V) */
#define MPCXH_PROOF_WORDS 160
#define MPCXH_DLN_ITERATIONS 128
#define MPCXH_MOD_ITERATIONS 80
#define MPCXH_FAC_FIELDS 11
int mpcxh_dln_prove_batch(uint32_t w, const uint32_t* h1, const uint32_t* h2, const uint32_t* x, const uint32_t* p,
                          const uint32_t* q, const uint32_t* N, uint32_t count, const mpcxh_reader_t* readers,
                          uint32_t* alpha, uint32_t* t);
int mpcxh_dln_verify_batch(uint32_t w, const uint32_t* h1, const uint32_t* h2, const uint32_t* N, uint32_t count,
                           const uint32_t* alpha, const uint32_t* t, uint8_t* ok);
int mpcxh_mod_prove_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N,
                          const uint32_t* P, const uint32_t* Q, uint32_t count, const mpcxh_reader_t* readers,
                          uint32_t* W, uint32_t* X, uint32_t* A, uint32_t* B, uint32_t* Z);
int mpcxh_mod_verify_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N,
                           uint32_t count, const uint32_t* W, const uint32_t* X, const uint32_t* A, const uint32_t* B,
                           const uint32_t* Z, uint8_t* ok);
int mpcxh_fac_prove_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N0,
                          const uint32_t* NCap, const uint32_t* s, const uint32_t* t, const uint32_t* N0p,
                          const uint32_t* N0q, uint32_t count, const mpcxh_reader_t* readers, uint32_t* pf,
                          uint8_t* v_neg);
int mpcxh_fac_verify_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N0,
                           const uint32_t* NCap, const uint32_t* s, const uint32_t* t, uint32_t count,
                           const uint32_t* pf, const uint8_t* v_neg, uint8_t* ok);

/* Config-4 driver: one GG18 signature for each of `wallets` wallets, signed by
 * the first `signers` of `n_nodes` nodes (keys: Paillier private keys + own
 * DLN params with factors, width w). Plays every signer through all of tss-lib
 * v2's signing rounds (csrc/host/signing.hpp): rounds 1-3 MtA / MtAwc of
 * up:ecdsa/signing on the GPU, checking alpha + beta = k gamma and mu + nu = k w
 * (mod q) for every session; the round-1 commitments, round-4 Schnorr proofs,
 * round 5-9 commitments, Schnorr / ZKV proofs and their checks; then s
 * (low-s) and ecdsa.Verify of every signature by every signer, twice (tss-lib's
 * finalize and mpcium's session: /root/reference/pkg/mpc/ecdsa_signing_session.go:162).
 * stats_out[MPCXH_SIGNING_STATS]: round1_s, round2_s, round3_s, total_s,
 * wallets, sessions, errors, relation_failures, engine_busy_s (time inside
 * libmpcx calls), finalize_s (rounds 4-9 + finalize), signatures, verified,
 * alg_macs (Go-equivalent algorithmic work of the exponentiations sent to the
 * GPU), aborted (wallets whose transcript failed a check).
 * trace_wallets > 0: trace_out receives, for the wallets floor(t * wallets /
 * trace_wallets), t = 0 .. trace_wallets-1 (spread over every wallet pipeline),
 * per ordered pair (i-major) and wallet 40 words (alpha, beta, mu, nu as 8
 * words each, SHA512_256i over the session's cA, RangeProofAlice, cB,
 * ProofBob, cB', ProofBobWC fields), then per wallet 25 words (r, s, recid,
 * SHA512_256i of the GG18 round 1/4-9 transcript). tamper_wallet >= 0 (test
 * hook): corrupt signer 0's round-4 Schnorr proof (tamper_kind 1), round-6
 * ZKV proof (2) or round-7 decommitment (3) in that wallet, which must abort. */
#define MPCXH_SIGNING_STATS 14
int mpcxh_bench_signing(uint32_t w, const mpcxh_paillier_t* sks, const mpcxh_dln_t* dlns, uint32_t n_nodes,
                        uint32_t signers, uint32_t wallets, uint64_t seed, double* stats_out, uint32_t trace_wallets,
                        uint32_t* trace_out, int64_t tamper_wallet, int tamper_kind);

/* Config-5 driver: the proof work of `sessions` keygen / reshare sessions of
 * n_parties nodes (csrc/host/keygenload.hpp): every party proves DLN x2,
 * Paillier-Blum Mod, and a Fac proof to each peer; every party verifies
 * every peer's proofs. Integers are w words wide (w >= 64). Sessions stream in
 * waves of wave_sessions (0: 1024), two waves in flight, every proof chain of a
 * wave (each party's proofs and their verification by every peer) at once:
 * host memory is bounded by the waves, not by `sessions`.
 * stats_out[MPCXH_KEYGEN_STATS]: prove_s, verify_s, total_s, sessions, parties,
 * proofs, verifications, failures, engine_busy_s, alg_macs, waves,
 * wave_sessions, max_wave_s.
 * trace_out (NULL: none): per wave, one traced session of
 * 1 + n(n+2)*8 + 1 words: its index, per party the 8-word SHA512_256i digests of
 * its DLN (h1, h2, alpha), DLN (h2, h1, beta), Mod proof and its Fac proof to
 * each peer (ascending), then the count of its verifications that passed
 * (keygenload.hpp TraceSessionWords). */
#define MPCXH_KEYGEN_STATS 13
typedef struct {
  mpcxh_paillier_t paillier;  /* the party's own Paillier private key */
  const uint32_t* NTilde;
  const uint32_t* h1;
  const uint32_t* h2;
  const uint32_t* alpha;      /* h2 = h1^alpha mod N~ */
  const uint32_t* beta;       /* alpha^-1 mod pq */
  const uint32_t* p;          /* N~ = (2p+1)(2q+1) */
  const uint32_t* q;
} mpcxh_party_t;
int mpcxh_bench_keygen_proofs(uint32_t w, const mpcxh_party_t* parties, uint32_t n_parties, uint32_t sessions,
                              uint64_t seed, uint32_t wave_sessions, double* stats_out, uint32_t* trace_out);
/* Config 5 with resharing as mpcium runs it (two resharing sessions per node
 * per wallet: old party and new party, /root/reference/pkg/eventconsumer/
 * event_consumer.go:407-416): reshare_mix = 1 makes every odd wave a resharing
 * wave -- the new committee's proof work (as keygen) plus the old committee's
 * VSS of its Lagrange-weighted share with new threshold 2 and the new
 * committee's decommitment, share and public-key checks (keygenload.hpp);
 * 0: keygen waves only (= mpcxh_bench_keygen_proofs).
 * stats_out[MPCXH_KEYGEN_RESHARE_STATS]: the MPCXH_KEYGEN_STATS values, then
 * keygen_sessions, reshare_sessions, keygen_wave_s, reshare_wave_s (summed
 * wave wall times per kind), vss_checks, vss_failures.
 * trace_out: per wave the keygen trace words, then n*8 + 9 VSS words (per old
 * party the 8-word digest of its commitment, points and shares; the digest of
 * the new shares; the count of VSS checks that passed; zero on keygen waves).
 * tamper_session >= 0 (test hook; -1: none): in that resharing session old party
 * 0 sends new party 1 a share off by one, so exactly one VSS check fails. */
#define MPCXH_KEYGEN_RESHARE_STATS 19
int mpcxh_bench_keygen_reshare(uint32_t w, const mpcxh_party_t* parties, uint32_t n_parties, uint32_t sessions,
                               uint64_t seed, uint32_t wave_sessions, int reshare_mix, int64_t tamper_session,
                               double* stats_out, uint32_t* trace_out);

/* Host-side helpers of the MtA path, exported as test hooks (no GPU needed):
 * common.SHA512_256i / SHA512_256i_TAGGED (tag == NULL: untagged) over count
 * integers of w words -> 32-byte digest; secp256k1 k*G and k*P (k: w words,
 * points 16 words x|y, all-zero = infinity); the first `count` draws of
 * common.GetRandomPositiveInt(rand, lessThan) (relprime != 0:
 * GetRandomPositiveRelativelyPrimeInt) from the CounterDRBG `seed`. */
int mpcxh_sha512_256i(const uint8_t* tag, size_t tag_len, uint32_t count, const uint32_t* ints, uint32_t w,
                      uint8_t* digest32);
int mpcxh_secp_scalar_base_mult(const uint32_t* k, uint32_t w, uint32_t* out16);
int mpcxh_secp_scalar_mult(const uint32_t* p16, const uint32_t* k, uint32_t w, uint32_t* out16);
/* u1*G + u2*P (the ecdsa.Verify combination) */
int mpcxh_secp_lincomb(const uint32_t* u1, const uint32_t* p16, const uint32_t* u2, uint32_t w, uint32_t* out16);
int mpcxh_random_draws(uint64_t seed, const uint32_t* less_than, uint32_t w, int relprime, uint32_t count,
                       uint32_t* out);

/* Go (*Int).ProbablyPrime(reps) for count odd or even n of `words` words
 * (go:src/math/big/prime.go: small-prime exits, Miller-Rabin with base 2 and
 * `reps` further bases drawn as Go draws them -- math/rand seeded with n's low
 * word, nat.random below n - 3, plus 2 -- and the extra strong Lucas test with
 * Baillie-OEIS parameter P, both on the GPU for n of up to 2048 bits). The same
 * tests as Go; only their order differs (base 2 first). ok[i] = 1: probably prime. */
int mpcxh_probably_prime_batch(uint32_t count, const uint32_t* n, uint32_t words, int reps, uint8_t* ok);
/* ok[i] = gcd(x[i], m[i]) == 1 for odd m[i] (math/big GCD(nil, nil, x, m).Cmp(one)
 * == 0, the coprimality test behind common.GetRandomPositiveRelativelyPrimeInt
 * and the proof verifiers' gcd checks); host-side, count operands of `words`
 * words each. MPCX_EINVAL for an even modulus. */
int mpcxh_coprime_batch(uint32_t count, const uint32_t* x, const uint32_t* m, uint32_t words, uint8_t* ok);

/* Host-time profile (environment MPCX_HOST_PROFILE=1 at process start, else
 * empty): "label: seconds (calls)" lines summed over threads, largest first,
 * written NUL-terminated into buf (truncated to cap); reset != 0 clears it. */
int mpcxh_profile_report(char* buf, size_t cap, int reset);

/* Host worker pool size: *threads = the threads parallel loops use now
 * (MPCX_HOST_THREADS, else min(usable CPUs, 16 per bound GPU)); *usable = the
 * CPUs this process may run on (affinity mask capped by the cgroup CPU quota). */
int mpcxh_host_threads(int* threads, int* usable);
/* The engine's page-locked staging pool (no GPU needed): bytes held (in use +
 * cached), peak bytes in use, and the pageable fallbacks taken when pinning
 * failed (count, bytes; each is also logged to stderr). Any pointer may be NULL. */
int mpcxh_pinned_pool_stats(uint64_t* held_bytes, uint64_t* peak_in_use_bytes, uint64_t* fallbacks,
                            uint64_t* fallback_bytes);
/* Pool self-test (no GPU): `tasks` threads each run a parallel loop of `outer`
 * indices, each index a nested parallel loop of `inner` indices adding
 * (task+1)(o+1)(i+1); *sum = the total. */
int mpcxh_pool_selftest(uint32_t tasks, uint32_t outer, uint32_t inner, uint64_t* sum);

/* Host bignum arithmetic (test hook, no GPU): op 0: a * b, 1: a / b, 2: a mod b,
 * 3: a^-1 mod b (Go ModInverse; MPCX_EINVAL when none), 4: gcd(a, b). Little-endian
 * words; *out_words = the result's normalized length (<= nout). */
int mpcxh_nat_arith(int op, const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* out,
                    uint32_t nout, uint32_t* out_words);

/* tss-lib candidate q from raw stream bytes (masking + delta walk; test hook). */
int mpcxh_candidate_from_bytes(const uint8_t* bytes, size_t n, int q_bit_len, uint32_t* q_out, uint32_t words);

/* n bytes of the CounterDRBG stream for `seed` (test hook). */
int mpcxh_drbg_read(uint64_t seed, uint8_t* out, size_t n);

/* Go math/rand (test hooks): count Int63() values of rand.New(rand.NewSource(seed)),
 * and the `reps` Miller-Rabin bases big.Int.ProbablyPrime(reps) draws for the odd
 * n (w words, n > 3), in Go's order, w words each (go:src/math/big/prime.go). */
int mpcxh_go_rand_int63(int64_t seed, uint32_t count, int64_t* out);
int mpcxh_go_mr_bases(const uint32_t* n, uint32_t w, uint32_t reps, uint32_t* out);

#ifdef __cplusplus
}
#endif

#endif /* MPCX_HOST_H_ */
