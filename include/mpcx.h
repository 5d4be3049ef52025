/*
 * mpcx.h -- C-ABI of libmpcx.so, the MI355X (gfx950) batched modular
 * exponentiation engine behind mpcium's tss-lib hot path.
 *
 * This is the drop-in boundary: plain pointers and sizes, no C++ or torch
 * types, no exceptions across the ABI. Every entry point returns an int
 * status (MPCX_OK == 0); mpcx_last_error() gives the thread's last message.
 *
 * Integers cross the boundary as little-endian arrays of 32-bit words
 * (Go: big.Int.Bits() on a 32-bit-word view, i.e. the natural layout a cgo
 * shim builds from big.Int.Bytes()); batches are operand-major (operand i
 * occupies words [i*stride, (i+1)*stride)). Results are the canonical
 * residue in [0, m), bit-identical to Go math/big (*Int).Exp for the same
 * non-negative inputs.
 *
 * Which reference interface each entry point replaces (the reference's
 * arithmetic lives in tss-lib v2.0.2, pinned at /root/reference/go.mod:10,
 * and Go math/big; "up:" = github.com/bnb-chain/tss-lib/v2, absent from the
 * image -- see SURVEY.md section 0):
 *   mpcx_modulus_register      -- the per-call setup inside math/big
 *                                 nat.expNNMontgomery (k0, RR), hoisted to
 *                                 once per node modulus (N^2, N~, N, p, q),
 *                                 which mpcium keeps for the process
 *                                 lifetime (/root/reference/pkg/mpc/node.go:69,109,170).
 *   mpcx_modexp_batch          -- up:common/int.go  (*modInt).Exp(x, y)
 *                                 = new(big.Int).Exp(x, y, m), for a batch of
 *                                 x with one shared y (e.g. y = N for r^N,
 *                                 y = lambda for c^lambda) or per-operand y
 *                                 (e.g. HomoMult c1^m), coalesced across the
 *                                 sessions /root/reference/pkg/mpc/session.go:199
 *                                 drives through party.UpdateFromBytes.
 *   mpcx_modexp_batch_device   -- same, device-resident buffers + stream
 *                                 (pipelines that keep operands in HBM).
 *   mpcx_modexp_submit/_job_*  -- the same batch, asynchronous (the Go
 *                                 batcher's submit / wait)
 *   mpcx_init_devices          -- one node process driving all its GPUs
 *   mpcx_fermat2_batch         -- up:common/safe_prime.go
 *                                 isPocklingtonCriterionSatisfied(p):
 *                                 2^(p-1) mod p == 1 for a batch of
 *                                 candidate moduli (keygen.GeneratePreParams,
 *                                 /root/reference/pkg/mpc/node.go:69).
 */
#ifndef MPCX_H_
#define MPCX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCX_OK 0
#define MPCX_EINVAL 1   /* bad argument (null pointer, even/zero modulus, size out of range) */
#define MPCX_ENODEV 2   /* no HIP device, or mpcx_init not called */
#define MPCX_EHIP 3     /* HIP runtime error or failed device self-test */
#define MPCX_ENOMEM 4   /* device or host allocation failed */

#define MPCX_MAX_MODULUS_BITS 4096 /* largest odd modulus a kernel class accepts */

typedef struct mpcx_modulus_s* mpcx_mod_t;

/* Library version (major*10000 + minor*100 + patch). */
int mpcx_version(void);

/* Text of the calling thread's last error ("" if none). */
const char* mpcx_last_error(void);

/* Number of visible HIP devices (0 without a GPU; never initialises one). */
int mpcx_device_count(int* out_count);

#define MPCX_MAX_DEVICES 16

/* Bind HIP device `device` (adds it to the process's set of bound GPUs) and
 * run its self-test. Idempotent per device. One process drives every GPU of
 * the node: an mpcium node is one Go process whose sessions share one set of
 * preparams (/root/reference/pkg/mpc/node.go:69,109,170). */
int mpcx_init(int device);

/* Bind devices 0 .. n_gpus-1 (n_gpus <= 0: every visible device). The
 * host-buffer entry points then spread over all bound devices: a batch of at
 * least 2 x "device_split_min" operands (mpcx_set_option, default 4096) is cut
 * into one contiguous operand range per device, run concurrently and
 * gathered into the caller's buffers (independent operands: no collective);
 * smaller batches go to one device, round-robin across calls. */
int mpcx_init_devices(int n_gpus);

/* The slice plan the host-buffer entry points use for a batch of `count`
 * operands over n_devices bound devices (pure function, no GPU needed):
 * *n_slices contiguous ranges [first[s], first[s] + n[s]) (arrays sized
 * >= n_devices), one per device 0..n_slices-1; one range (run on one device,
 * round-robin) unless every range gets >= min_slice operands. */
int mpcx_partition(uint32_t count, int n_devices, uint32_t min_slice, uint32_t* first, uint32_t* n,
                   uint32_t* n_slices);

/* Number of bound devices and (optionally) their HIP ordinals, bind order. */
int mpcx_bound_devices(int* out_count, int* ordinals, int max_ordinals);

/* Kernel launches issued so far by the batch entry points on bound device
 * `index` (modexp, fixed-base, secp256k1 batches): which devices a workload
 * actually used. */
int mpcx_device_launches(int index, uint64_t* out);

/* Kernel statistics of the batch entry points (modexp, multi-batch,
 * fixed-base, secp256k1), collected while option "kernel_stats" is 1: an
 * event pair around every launch, resolved at the lane's host wait. Writes a
 * JSON object to buf (NUL-terminated; MPCX_EINVAL if cap is too small):
 *   {"enabled":0|1,"busy_ms":B,"alg_macs":A,"kernels":[{"kind":..,"geom":g,
 *    "launches":n,"operands":n,"alg_macs":a,"kernel_ms":t},...]}
 * alg_macs: Go-equivalent work (SURVEY.md 8(d) W per exponentiation) for
 * the exponentiation kernels -- within ~5% of what they execute (same
 * squarings; 5-bit or sliding windows instead of 4-bit) -- and the executed
 * products x 2 L^2 for the fixed-base comb (one per w-bit window, far below
 * Go's work for the same Exp); 0 for secp256k1;
 * kernel_ms: summed launch durations (lanes overlap, so the kinds' sum can
 * exceed busy_ms, the union of all launches' intervals per device, summed
 * over devices). reset != 0: clear after reading and start a new time
 * origin on every bound device (call while no launch is in flight). */
int mpcx_kernel_stats(char* buf, size_t cap, int reset);

/* Device (index into the bound set, default 0) used by THIS thread's
 * device-buffer calls, modulus registration, comb-table builds, mpcx_dev_alloc
 * and mpcx_stream_create. Moduli and comb tables are usable on every bound
 * device (their constants are uploaded to a device on first use there). */
int mpcx_select_device(int index);

/* Release all device resources (registered moduli become invalid). */
int mpcx_shutdown(void);

/* Register an odd modulus m (m_words little-endian 32-bit words, leading zero
 * words allowed) with 1 <= m < 2^MPCX_MAX_MODULUS_BITS. Precomputes the
 * Montgomery constants and uploads them. *out stays valid until
 * mpcx_modulus_release / mpcx_shutdown. Even m returns MPCX_EINVAL: math/big
 * takes a different (CRT/windowed) path for even moduli, which the hot path
 * never uses; callers keep those on the host. */
int mpcx_modulus_register(const uint32_t* m_words, uint32_t m_len, mpcx_mod_t* out);
int mpcx_modulus_release(mpcx_mod_t mod);

/* Bits of the registered modulus, and the operand width (words) of the kernel
 * class serving it: bases may have up to that many words. */
int mpcx_modulus_info(mpcx_mod_t mod, uint32_t* out_bits, uint32_t* out_class_words);

/* out[i] = bases[i] ^ e_i mod m for i < count, host buffers.
 *   bases:    count x base_words words, base_words <= class words
 *             (mpcx_modulus_info); any value below 2^(32*class words),
 *             including values >= m, is accepted (math/big likewise accepts
 *             len(x) == len(m) without reducing first)
 *   exps:     exp_shared != 0: ONE exponent of exp_words words (e_i = exps)
 *             exp_shared == 0: count x exp_words words (e_i = exps[i*exp_words ...])
 *             exponents are non-negative (Go's y < 0 inverse path is the
 *             caller's); exp_words may be 0 (y = 0)
 *   out:      count x out_words words, out_words >= words(m); zero-padded.
 * Synchronous: returns after the results are in `out`. */
int mpcx_modexp_batch(mpcx_mod_t mod, uint32_t count,
                      const uint32_t* bases, uint32_t base_words,
                      const uint32_t* exps, uint32_t exp_words, int exp_shared,
                      uint32_t* out, uint32_t out_words);

/* Same contract with device pointers (d_*) on HIP stream `stream` (a
 * hipStream_t of the thread's selected device, NULL = default stream).
 * Asynchronous: the results are valid after the stream is synchronised.
 * exp_bits is the bit length of the largest exponent (any value >= it and <=
 * 32*exp_words is correct; per-operand exponents are processed as
 * ceil(exp_bits/4) 4-bit windows; a shared exponent's sliding-window schedule
 * is built on `stream` by a one-lane kernel, so the call stays asynchronous).
 * Every (device, stream) pair has its own kernel workspace, so calls on
 * different streams may run concurrently; the first call on a stream with a
 * larger batch than before grows that stream's workspace (hipMalloc, after
 * synchronising the stream). */
int mpcx_modexp_batch_device(mpcx_mod_t mod, uint32_t count,
                             const uint32_t* d_bases, uint32_t base_words,
                             const uint32_t* d_exps, uint32_t exp_words, int exp_shared,
                             uint32_t exp_bits,
                             uint32_t* d_out, uint32_t out_words, void* stream);

/* Fused variant: out[i] = muls[i] * bases[i]^e_i mod m (muls: count x
 * mul_words words, mul_words <= class words). Replaces the
 * "Exp then ModInt.Mul" pairs of the reference: Paillier Encrypt
 * c = (1 + m*N) * r^N mod N^2 (up:crypto/paillier/paillier.go
 * EncryptAndReturnRandomness) and the MtA proof terms. */
int mpcx_modexp_mul_batch(mpcx_mod_t mod, uint32_t count,
                          const uint32_t* bases, uint32_t base_words,
                          const uint32_t* exps, uint32_t exp_words, int exp_shared,
                          const uint32_t* muls, uint32_t mul_words,
                          uint32_t* out, uint32_t out_words);
int mpcx_modexp_mul_batch_device(mpcx_mod_t mod, uint32_t count,
                                 const uint32_t* d_bases, uint32_t base_words,
                                 const uint32_t* d_exps, uint32_t exp_words, int exp_shared,
                                 uint32_t exp_bits,
                                 const uint32_t* d_muls, uint32_t mul_words,
                                 uint32_t* d_out, uint32_t out_words, void* stream);

/* Asynchronous host-buffer submission (SURVEY.md 8(b) "async submit +
 * mpcx_sync"): the same work as mpcx_modexp_mul_batch (muls may be NULL:
 * mpcx_modexp_batch), run by libmpcx's submission threads. The caller keeps
 * every buffer alive and unmodified until mpcx_job_wait returns. *job is
 * released by mpcx_job_wait, which returns the batch's status. */
typedef struct mpcx_job_s* mpcx_job_t;
int mpcx_modexp_submit(mpcx_mod_t mod, uint32_t count,
                       const uint32_t* bases, uint32_t base_words,
                       const uint32_t* exps, uint32_t exp_words, int exp_shared,
                       const uint32_t* muls, uint32_t mul_words,
                       uint32_t* out, uint32_t out_words, mpcx_job_t* job);
int mpcx_job_test(mpcx_job_t job, int* done);
int mpcx_job_wait(mpcx_job_t job);

/* out[i] = a[i] * b[i] mod m -- up:common/int.go (*modInt).Mul and
 * paillier.(*PublicKey).HomoAdd (c1*c2 mod N^2), batched. */
int mpcx_mulmod_batch(mpcx_mod_t mod, uint32_t count,
                      const uint32_t* a, uint32_t a_words,
                      const uint32_t* b, uint32_t b_words,
                      uint32_t* out, uint32_t out_words);

/* Pocklington/Fermat check for safe-prime candidates: ok[i] = (2^(p_i - 1)
 * mod p_i == 1) for count odd candidates p_i of p_words words each
 * (5 <= p_i < 2^1024, p_words <= 32). Each candidate is its own modulus. */
int mpcx_fermat2_batch(uint32_t count, const uint32_t* p, uint32_t p_words, uint8_t* ok);

/* Several batches in ONE kernel launch: each group has its own registered
 * modulus (all of one size class), bases, shared or per-operand exponents,
 * optional multipliers and output, exactly as one mpcx_modexp_batch /
 * mpcx_modexp_mul_batch call (same semantics per group). The groups become
 * segments of one launch, so the concurrent small batches of many sessions
 * and moduli (an MtA step of every signer pair of every wallet pipeline) run
 * in the main, widest geometry instead of as many small launches. */
typedef struct {
  mpcx_mod_t mod;
  uint32_t count;
  const uint32_t* bases;
  uint32_t base_words;
  const uint32_t* exps;
  uint32_t exp_words;
  int exp_shared;
  const uint32_t* muls; /* NULL: no multiplier */
  uint32_t mul_words;
  uint32_t* out;
  uint32_t out_words;
} mpcx_modexp_group_t;
int mpcx_modexp_multi_batch(uint32_t n_groups, const mpcx_modexp_group_t* groups);

/* secp256k1 (btcec/v2 S256, /root/reference/go.mod:29): out_i = a_i G + b_i P_i
 * + c_i Q_i for count independent items, one GPU thread each -- every point
 * equation of tss-lib's GG18 signing outside the MtA (up:ecdsa/signing
 * round_1.go .. finalize.go: Gamma_i = gamma_i G, Schnorr / ZKV proofs and their
 * checks, R = theta^-1 sum Gamma, V_i = s_i R + l_i G, U_i = rho_i V, and
 * ecdsa.Verify's u1 G + u2 X; up:crypto/schnorr).
 * scalars: count x 24 words (a, b, c: 8 little-endian words each, any 256-bit
 * value, i.e. taken mod the group order); points: count x 32 words (P.x, P.y,
 * Q.x, Q.y, 8 little-endian words each; an all-zero point is the point at
 * infinity; others must be on the curve -- the caller checks, as
 * crypto.NewECPoint does); out: count x 16 words (x, y; all zero = infinity). */
int mpcx_ec_combine_batch(uint32_t count, const uint32_t* scalars, const uint32_t* points, uint32_t* out);

/* Miller-Rabin: ok[i] = n_i is a strong probable prime to base bases[i]
 * (5 <= n_i < 2^1024 odd, bases[i] < 2^(32*n_words); a base that is 0 mod
 * n_i reports "composite"). Each candidate is its own modulus. Serves
 * q.ProbablyPrime(20) of up:common/safe_prime.go (Go: math/big
 * probablyPrimeMillerRabin, go:src/math/big/prime.go). */
int mpcx_mr_batch(uint32_t count, const uint32_t* n, uint32_t n_words, const uint32_t* bases, uint8_t* ok);

/* Strong Lucas probable-prime test, the last step of Go's ProbablyPrime
 * (go:src/math/big/prime.go probablyPrimeLucas, the "extra strong" test):
 * ok[i] = n_i passes with parameters P[i], Q = 1 (Baillie-OEIS method C: the
 * caller supplies the smallest P >= 3 with Jacobi(P^2 - 4, n_i) = -1 and
 * handles the Jacobi = 0 / perfect-square exits). 5 <= n_i < 2^2048 odd
 * (n_words <= 64; a batch with a candidate above 1024 bits runs in the wide
 * 16 x 5-digit geometry), 3 <= P[i] < 2^14. Each candidate is its own modulus. */
int mpcx_lucas_batch(uint32_t count, const uint32_t* n, uint32_t n_words, const uint32_t* P, uint8_t* ok);

/* One pipelined step of the safe-prime search (up:common/safe_prime.go
 * runGenPrimeRoutine) on one bound device, all in one stream:
 *  - count candidates of nbytes = (q_bits+7)/8 stream bytes each: raw !=
 *    NULL: count x nbytes bytes from the host reader; raw == NULL: the
 *    CounterDRBG(seed) stream's bytes [stream_off, stream_off + count*nbytes),
 *    drawn on the device (no host hashing, no PCIe copy);
 *  - masks, delta walk, bit-length check and exact trial division of q and
 *    p = 2q+1 (as mpcx_safeprime_sieve_fermat);
 *  - in ONE launch: the Pocklington test 2^(p-1) == 1 (mod p) on every sieve
 *    survivor, and the base-2 strong probable-prime test on n_sprp given q
 *    (sprp_q: n_sprp x 32 words -- an earlier step's Fermat passes riding
 *    along).
 * Out: *n_sieved survivors (Fermat tests); *n_pass Fermat passes in stream
 * order: pass_idx (candidate index within the step) and pass_p (p, 32 words each;
 * both sized >= max_pass, else MPCX_ENOMEM); sprp_ok[n_sprp]. count may be 0
 * (ride-along only). 63 <= q_bits <= 1023. */
int mpcx_safeprime_step(uint64_t seed, const uint8_t* raw, uint64_t stream_off, uint32_t count, uint32_t q_bits,
                        const uint32_t* sprp_q, uint32_t n_sprp, uint32_t max_pass, uint32_t* n_sieved,
                        uint32_t* n_pass, uint32_t* pass_idx, uint32_t* pass_p, uint8_t* sprp_ok);

/* Safe-prime candidate batch on the GPU (up:common/safe_prime.go
 * runGenPrimeRoutine steps 1-5): raw = count candidates' (q_bits+7)/8 random
 * bytes each, in stream order (63 <= q_bits <= 1023). Each candidate q is
 * masked / delta-walked / length-checked exactly as tss-lib does, q and
 * p = 2q+1 are trial-divided by the primes 59..2039 (exact: only composites
 * are dropped), and every survivor gets the Pocklington test 2^(p-1) mod p.
 * Output, ascending candidate index: *n_out survivors of the sieve, their
 * indices idx_out[j] and Fermat verdicts ok_out[j] (both sized >= count). */
int mpcx_safeprime_sieve_fermat(const uint8_t* raw, uint32_t nbytes, uint32_t count, uint32_t q_bits,
                                uint32_t* n_out, uint32_t* idx_out, uint8_t* ok_out);

/* Fixed-base comb tables for long-lived bases of a <= 2080-bit modulus (the
 * h1, h2 of a node's N~ that every MtA range proof and DLN proof
 * exponentiates: up:crypto/mta/range_proof.go, up:crypto/mta/proofs.go,
 * up:crypto/dlnproof/proof.go; SURVEY.md 8(b) "_fixed_base"). Registration
 * precomputes b^(v 2^(wj)) R mod m for every w-bit window j below
 * max_exp_bits on the GPU (2^w entries per window; w = 12 by default, option
 * "fb_window", narrowed while the table would exceed 512 MB: ~320 MB for
 * 3072-bit exponents of a 2048-bit modulus, a small share of 288 GB of HBM);
 * the table lives until mpcx_fixedbase_release (release it before its
 * modulus). */
typedef struct mpcx_fixedbase_s* mpcx_fb_t;
#define MPCX_FB_MAX_EXP_BITS 65536
int mpcx_fixedbase_register(mpcx_mod_t mod, const uint32_t* base, uint32_t base_words,
                            uint32_t max_exp_bits, mpcx_fb_t* out);
int mpcx_fixedbase_release(mpcx_fb_t fb);
/* Largest exponent a table serves and its device footprint. */
int mpcx_fixedbase_info(mpcx_fb_t fb, uint32_t* max_exp_bits, size_t* table_bytes);

/* out[i] = (muls ? muls[i] : 1) * prod_{t < nbases} b_t^(e_t,i) mod m, with
 * 1 <= nbases <= 2 tables of the SAME modulus (e.g. z = h1^m h2^rho mod N~
 * as one product: one Montgomery product per w-bit window, no squarings).
 * exps[t]: count x exp_words[t] words (exp_words[t] may be 0: e = 0); every
 * exponent must fit its table (EINVAL otherwise). Synchronous. */
int mpcx_fixedbase_exp_batch(uint32_t nbases, const mpcx_fb_t* fbs, uint32_t count,
                             const uint32_t* const* exps, const uint32_t* exp_words,
                             const uint32_t* muls, uint32_t mul_words,
                             uint32_t* out, uint32_t out_words);

/* Several comb batches in ONE launch (kernel k_fixedbase_multi): each group is
 * exactly one mpcx_fixedbase_exp_batch call (its own tables -- any moduli of
 * one size class --, exponents, multipliers, output). Concurrent callers'
 * batches (h1, h2 of every peer's N~ in every wallet pipeline) become the
 * segments of one launch that fills the GPU, instead of many launches of a
 * fraction of a resident round each (the replaced surface is the same
 * common.ModInt.Exp on h1/h2, up:crypto/mta/range_proof.go). Synchronous. */
#define MPCX_FB_MAX_BASES 2
typedef struct {
  uint32_t nbases;                          /* 1 or 2 tables of one modulus */
  mpcx_fb_t fbs[MPCX_FB_MAX_BASES];
  uint32_t count;
  const uint32_t* exps[MPCX_FB_MAX_BASES];  /* count x exp_words[t] words */
  uint32_t exp_words[MPCX_FB_MAX_BASES];
  const uint32_t* muls;                     /* NULL: no multiplier */
  uint32_t mul_words;
  uint32_t* out;
  uint32_t out_words;
} mpcx_fixedbase_group_t;
int mpcx_fixedbase_multi_batch(uint32_t n_groups, const mpcx_fixedbase_group_t* groups);

/* Device memory helpers for callers without their own HIP allocator. */
int mpcx_dev_alloc(size_t bytes, void** out_ptr);
int mpcx_dev_free(void* ptr);
/* Page-locked host memory (portable across the bound devices): host-buffer
 * batches staged here are copied by DMA. Every other host range a call reads
 * or writes goes through the lane's own page-locked bounce buffer, copied by
 * libmpcx in the calling thread: no pageable pointer reaches the HIP runtime's
 * copy engine. A range that starts inside an mpcx_host_alloc block and runs
 * past its end is rejected with MPCX_EINVAL. */
int mpcx_host_alloc(size_t bytes, void** out_ptr);
int mpcx_host_free(void* ptr);
/* Host-copy counters since load: bytes DMA'd directly from/to mpcx_host_alloc
 * blocks, bytes bounced through the lanes' pinned buffers, and bounce-buffer
 * (re)allocations. Any pointer may be NULL. */
int mpcx_copy_stats(uint64_t* direct_bytes, uint64_t* bounced_bytes, uint64_t* bounce_allocs);
int mpcx_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes);
int mpcx_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes);
int mpcx_stream_create(void** out_stream);
int mpcx_stream_destroy(void* stream);
int mpcx_stream_sync(void* stream);
/* SURVEY.md 8(b) name of mpcx_stream_sync. */
int mpcx_sync(void* stream);

/* Tuning knobs (process-wide). Every default is the winner of a measured,
 * interleaved A/B on MI355X (DESIGN.md section 6 cites each):
 *   "narrow_rounds" 0..100 (default 15): batches under this many hundredths of
 *                a resident round of the main geometry run in the class's
 *                narrow geometry (3 was slower for signing, profiles/r03/narrow_ab).
 *   "geom_policy" 1 (default): 4096-bit batches pick the main, mid (8 x 19)
 *                or narrow geometry by a measured launch-time model of
 *                wavefronts per SIMD; 0: the "narrow_rounds" threshold only;
 *                2: every batch in its class's main geometry.
 *   "main_geom"  geometry id: make it the main (throughput) geometry of its
 *                class (A/B of kernel layouts: 5 vs 1 for the 2048-bit class).
 *   "sched_width" 0..6 (default 6): cap on the sliding-window width used for
 *                shared exponents; 0 selects Go's 4-bit fixed window.
 *   "fixed_window" 4 or 5 (default 5): widest fixed window for per-operand
 *                exponents (5 bits above 1024-bit exponents, else Go's 4).
 *   "fb_window"  4..12 (default 12): window width of comb tables registered
 *                from now on.
 *   "fb_split"   0 (default), 1, 2 or 4: wavefronts sharing one comb
 *                operand's windows (each takes every S-th window; wave 0
 *                multiplies the partials in); 0 picks the largest that keeps a
 *                launch within 4 wavefronts per SIMD (round 5, three interleaved
 *                rounds vs 1: keygen/reshare 437.6 vs 419.7 sessions/s, signing
 *                7,110 vs 6,874 and 3,225 vs 3,039 sigs/s, profiles/r05/fbsplit).
 *   "mx"         1 (default), 0 or 2: batches of the 4096-bit main geometry
 *                (>= "mx_min" operands, default 2048) run k_modexp_mx, the
 *                Montgomery reduction on the i8 matrix cores (round 5: config 2
 *                457K vs 378K modexp/s, profiles/r05/mx/); 2 adds the 2048-bit
 *                lane-pair geometry, which measured slower (1.22M vs 1.40M
 *                2048-bit modexp/s, keygen -7%: profiles/r05/mx/g5/).
 *                Multi-batch launches of the 4096-bit main geometry use it too
 *                (k_modexp_multi_mx) when every group has >= "mx_seg_min"
 *                operands (default 64 since round 6: six interleaved rounds
 *                against 256, 2 signers 7,454 vs 7,022 sigs/s, 3 signers 3,435
 *                vs 3,318, keygen 417 vs 425 sessions/s, profiles/r06/segmin*;
 *                round 5: the multi-batch kernel itself, signing +10%,
 *                profiles/r05/mx/multi/).
 *                Environment: MPCX_MX.
 *   "mx_step"    10..200 (default 81): the launch-time model's wave-round time
 *                of a 4096-bit main-geometry launch that will run on the
 *                matrix cores, in percent of the CIOS kernel's (config 2: 139.5
 *                vs 172.5 ms); 100 ignores the matrix cores (round 5's model).
 *                Round 6, three interleaved rounds against 100: 2 signers 7,418
 *                vs 7,237 sigs/s, 3 signers 3,398 vs 3,296, keygen 424 vs 419
 *                (profiles/r06/geomtput/). Environment: MPCX_MX_STEP.
 *   "geom_tput"  0..1000 (default 0): weight, in percent, of a launch's share of
 *                the GPU's SIMD time in the launch-time model (latency +
 *                weight x share). 150 / 300 measured neutral to slower (same
 *                A/B). Environment: MPCX_GEOM_TPUT.
 *   "prime_coop" 1 (default): cooperative per-candidate prime kernels; 0:
 *                thread per candidate.
 *   "lanes"      1..8 (default 6, or MPCX_LANES): execution lanes (streams
 *                with their own workspaces) per device used from now on.
 *   "device_split_min" operands (default 4096): smallest per-device slice
 *                of a host-buffer batch split across the bound devices
 *                (0: never split).
 * Test and measurement hooks:
 *   "force_geom" -1 (default) or a geometry id (0..6, see mpcx_internal.h) to
 *                run every batch of the matching class in that geometry (a
 *                geometry that cannot serve a modulus or its operands falls
 *                back to the class's full-width geometry).
 *   "duplicate_device" 0 (default) / 1: mpcx_init of an already bound
 *                ordinal binds it again as another logical device (own lanes,
 *                constants, workspaces), so the multi-device split and gather
 *                run concurrently on a one-GPU box.
 *   "kernel_stats" 0 (default) / 1: time every batch-entry-point launch
 *                with an event pair for mpcx_kernel_stats.
 * Environment, read at mpcx_init / mpcx_init_devices: MPCX_LANES (1..8,
 * default 6: execution lanes per device), MPCX_GEOM_POLICY, MPCX_NARROW_ROUNDS,
 * MPCX_PRIME_COOP, MPCX_FB_WINDOW, MPCX_MX, MPCX_MX_STEP, MPCX_GEOM_TPUT. */
int mpcx_set_option(const char* key, int value);
/* Current value of "mx", "mx_min", "mx_seg_min", "mx_step", "geom_tput",
 * "geom_policy", "sched_width", "fixed_window", "fb_split" or "lanes"
 * (benchmarks record which kernel path ran). */
int mpcx_get_option(const char* key, int* value);

/* The constant tables of k_modexp_mx (the 4096- and 2048-bit main geometries
 * with their Montgomery reduction on the i8 matrix cores,
 * mpcium_amd/csrc/mpcx_mx.hpp) for the odd modulus m and the geometry's digit
 * count L (148: R = 2^4144; 74: R = 2^2072; 4m < R): the LDS image of the
 * Toeplitz tables of m'' = -m^-1 mod R and of m, 2 x 16 row copies of the
 * reversed radix-2^7 digit strings (23,040 or 13,824 bytes). Host-only (no
 * device needed); for tests and tools. */
int mpcx_mx_tables(const uint32_t* m_words, uint32_t m_len, uint32_t L, uint8_t* out, size_t cap);

/* Kernel-class geometry of a modulus (for benchmarks and roofline math):
 * digits L (radix 2^28), lanes per operand P, digits per lane K, operands per
 * 64-lane wavefront G. */
int mpcx_modulus_geometry(mpcx_mod_t mod, uint32_t* L, uint32_t* P, uint32_t* K, uint32_t* G);

#ifdef __cplusplus
}
#endif

#endif /* MPCX_H_ */
