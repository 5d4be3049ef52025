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
 *   mpcxh_generate_preparams     up:ecdsa/keygen/prepare.go GeneratePreParams,
 *                                called at /root/reference/pkg/mpc/node.go:69
 */
#ifndef MPCX_HOST_H_
#define MPCX_HOST_H_

#include <stddef.h>
#include <stdint.h>

#include "mpcx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* io.Reader stand-in: fill buf[0..n) with random bytes. */
typedef void (*mpcxh_rand_fn)(void* ctx, uint8_t* buf, size_t n);

#define MPCXH_PREPARAM_FIELDS 12

const char* mpcxh_last_error(void);
int mpcxh_init(int device);

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
 * Random source: rand_fn(rand_ctx, ...) if non-NULL, else the CounterDRBG
 * seeded with `seed`. p_out/q_out: num x words. index_out: stream positions.
 * stats_out[5]: candidates, sieved out, GPU Fermat tests, GPU MR tests, usec. */
int mpcxh_safe_primes(int bit_len, int num, uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx,
                      uint32_t* p_out, uint32_t* q_out, uint32_t words, uint64_t* index_out,
                      uint64_t* stats_out);

/* LocalPreParams as 12 fields x 64 words: N, LambdaN, PhiN, P, Q (Paillier),
 * NTildei, H1i, H2i, Alpha, Beta, P, Q (Germain primes of N~). */
int mpcxh_generate_preparams(uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx,
                             uint32_t* out, uint64_t* stats_out);

/* tss-lib candidate q from raw stream bytes (masking + delta walk; test hook). */
int mpcxh_candidate_from_bytes(const uint8_t* bytes, size_t n, int q_bit_len, uint32_t* q_out, uint32_t words);

/* n bytes of the CounterDRBG stream for `seed` (test hook). */
int mpcxh_drbg_read(uint64_t seed, uint8_t* out, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* MPCX_HOST_H_ */
