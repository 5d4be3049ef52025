// mpcx_prime.hip -- launchers of the safe-prime kernels (candidate stream
// DRBG, sieve, base-2 Fermat / strong tests, Miller-Rabin, strong Lucas;
// thread per candidate), the shared-exponent window schedule (k_expsched) and
// the device self-test.
#ifndef MPCX_BLOCK_FENCE
#define MPCX_BLOCK_FENCE 1  // see montmul: keeps k_prime2c within its register budget
#endif
#include "mpcx_device.hpp"

namespace mpcx {

// Device self-test of the cross-lane primitives the kernels rely on.
__global__ void k_selftest(uint32_t* out) {
  const int lane = threadIdx.x;
  out[lane] = from_next_lane(1000u + lane);
  out[64 + lane] = from_prev_lane(1000u + lane);
  out[128 + lane] = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane / 7) * 7) * 4, (int)(2000 + lane));
  const uint64_t acc = (uint64_t)(0xFFFFFFF0u + lane) * (0xFFFFFFF7u - lane) + 0xFFFFFFFFFFFFull;
  out[192 + lane] = (uint32_t)(acc >> 32);
}

// ------------------------------------------------- sliding-window schedule
// The left-to-right sliding-window decomposition of a shared exponent
// (layout: MPCX_SCHED_* in mpcx_internal.h), built on the launch stream so
// the device-buffer API stays asynchronous. One lane: ~E scalar steps over a
// two-word cache of the exponent, microseconds against the exponentiation.
// Width w minimises table + multiplies: 2^(w-1) products for x^2 and the odd
// powers (none for w = 1), plus ~E/(w+1) window multiplies.
__global__ __launch_bounds__(64) void k_expsched(const ExpSchedArgs a) {
  if (threadIdx.x != 0) return;
  const uint32_t* e = a.exp;
  uint32_t* s = a.sched;
  int top = -1;
  for (int i = (int)a.exp_words - 1; i >= 0; --i) {
    const uint32_t v = e[i];
    if (v) {
      top = 32 * i + 31 - __builtin_clz(v);
      break;
    }
  }
  if (top < 0) {  // e = 0: the kernel takes Go's fixed-window path (z = 1)
    s[MPCX_SCHED_TOP] = MPCX_SCHED_NONE;
    s[MPCX_SCHED_TN] = 0;
    s[MPCX_SCHED_N] = 0;
    s[MPCX_SCHED_WIDTH] = 0;
    return;
  }
  const int E = top + 1;
  int w = 1;
  float best = (float)E / 2.0f;
  for (int c = 2; c <= (int)a.max_width && c <= MPCX_SCHED_MAX_WIDTH; ++c) {
    const float cost = (float)(1 << (c - 1)) + (float)E / (float)(c + 1);
    if (cost < best) {
      best = cost;
      w = c;
    }
  }
  uint32_t c0i = ~0u, c0 = 0, c1i = ~0u, c1 = 0;  // two most recent exponent words
  auto word = [&](uint32_t wi) -> uint32_t {
    if (wi == c0i) return c0;
    if (wi == c1i) return c1;
    const uint32_t v = e[wi];
    c1i = c0i;
    c1 = c0;
    c0i = wi;
    c0 = v;
    return v;
  };
  auto bit = [&](int i) -> uint32_t { return (word((uint32_t)i >> 5) >> (i & 31)) & 1u; };
  auto bits = [&](int lo, int len) -> uint32_t {
    uint32_t v = 0;
    for (int b = len - 1; b >= 0; --b) v = (v << 1) | bit(lo + b);
    return v;
  };
  // top window: bits [lo, top], lo the lowest set bit within w bits of top
  int lo = top - w + 1 > 0 ? top - w + 1 : 0;
  while (!bit(lo)) ++lo;
  const uint32_t top_ent = (bits(lo, top - lo + 1) - 1u) >> 1;
  uint32_t tn = top_ent, n = 0, sq = 0;
  int pos = lo - 1;
  while (pos >= 0) {
    if (!bit(pos)) {
      ++sq;
      --pos;
      continue;
    }
    lo = pos - w + 1 > 0 ? pos - w + 1 : 0;
    while (!bit(lo)) ++lo;
    const int len = pos - lo + 1;
    const uint32_t ent = (bits(lo, len) - 1u) >> 1;
    sq += (uint32_t)len;
    s[MPCX_SCHED_STEPS + n++] = (sq << 8) | ent;
    tn = ent > tn ? ent : tn;
    sq = 0;
    pos = lo - 1;
  }
  if (sq) s[MPCX_SCHED_STEPS + n++] = (sq << 8) | 0xFFu;
  s[MPCX_SCHED_TOP] = top_ent;
  s[MPCX_SCHED_TN] = tn;
  s[MPCX_SCHED_N] = n;
  s[MPCX_SCHED_WIDTH] = (uint32_t)w;
}


// ----------------------------------------------------- candidate stream
// The build's CounterDRBG (csrc/host/tsscommon.cpp, oracle/gomath.py) on the
// device: 32-byte block c = SHA-256("mpcx-drbg" || seed LE64 || c LE64). One
// thread per block; the safe-prime search draws its candidates' bytes here
// instead of hashing ~25 MB per batch on the host and copying them over PCIe.
namespace {
__device__ __forceinline__ uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
}  // namespace

__global__ __launch_bounds__(256) void k_drbg(const DrbgArgs a) {
  const uint64_t b0 = a.off >> 5, b1 = (a.off + a.n + 31) >> 5;
  const uint64_t c = b0 + (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (c >= b1) return;
  // one padded block: "mpcx-drbg" (9) | seed (8, LE) | c (8, LE) | 0x80 | zeros | bit length 200
  uint8_t m[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) m[i] = 0;
  const char tag[9] = {'m', 'p', 'c', 'x', '-', 'd', 'r', 'b', 'g'};
#pragma unroll
  for (int i = 0; i < 9; ++i) m[i] = (uint8_t)tag[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[9 + i] = (uint8_t)(a.seed >> (8 * i));
    m[17 + i] = (uint8_t)(c >> (8 * i));
  }
  m[25] = 0x80;
  m[62] = 0x00;
  m[63] = 200;  // 25 bytes * 8
  uint32_t w[64];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)m[4 * i] << 24 | (uint32_t)m[4 * i + 1] << 16 | (uint32_t)m[4 * i + 2] << 8 | m[4 * i + 3];
#pragma unroll
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t A = h[0], B = h[1], C = h[2], D = h[3], E = h[4], F = h[5], G = h[6], H = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint32_t S1 = ror32(E, 6) ^ ror32(E, 11) ^ ror32(E, 25);
    const uint32_t ch = (E & F) ^ (~E & G);
    const uint32_t t1 = H + S1 + ch + kSha256K[i] + w[i];
    const uint32_t S0 = ror32(A, 2) ^ ror32(A, 13) ^ ror32(A, 22);
    const uint32_t mj = (A & B) ^ (A & C) ^ (B & C);
    const uint32_t t2 = S0 + mj;
    H = G;
    G = F;
    F = E;
    E = D + t1;
    D = C;
    C = B;
    B = A;
    A = t1 + t2;
  }
  h[0] += A; h[1] += B; h[2] += C; h[3] += D; h[4] += E; h[5] += F; h[6] += G; h[7] += H;
  const uint64_t pos0 = c << 5;
  if (pos0 >= a.off && pos0 + 32 <= a.off + a.n && ((pos0 - a.off) & 3u) == 0) {
    // whole block inside the range, 4-byte aligned: 8 word stores (big-endian digest bytes)
    uint32_t* o = (uint32_t*)(a.out + (pos0 - a.off));
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = __builtin_bswap32(h[i]);
    return;
  }
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const uint64_t pos = pos0 + i;
    if (pos >= a.off && pos < a.off + a.n) a.out[pos - a.off] = (uint8_t)(h[i >> 2] >> (24 - 8 * (i & 3)));
  }
}

// ----------------------------------------------------- safe-prime sieve
// One thread per candidate of tss-lib's runGenPrimeRoutine stream
// (up:common/safe_prime.go; restated in csrc/host/safeprime.cpp
// CandidateFromBytes and oracle/safeprime_ref.py):
//  1. (qBitLen+7)/8 big-endian bytes, masked to qBitLen bits with the top two
//     bits set, made odd;
//  2. delta walk (+2) until q + delta is coprime to 3..53 (Go's old
//     crypto/rand.Prime walk over q mod smallPrimesProduct: the residues mod
//     each prime carry the same information);
//  3. bit length == qBitLen;
//  + exact trial division of q and p = 2q+1 by the primes 59..2039 (never
//     rejects a prime, so the first accepted candidate is unchanged).
// Survivors p = 2q+1 (32 words) go to an atomically allocated slot with the
// candidate index; the host restores stream order.
namespace {
__device__ __forceinline__ uint32_t mod_step(uint32_t r, uint32_t w, uint32_t d, uint64_t inv) {
  // (r 2^32 + w) mod d for r < d < 2^32: Barrett with inv = floor((2^64-1)/d)
  const uint64_t x = ((uint64_t)r << 32) | w;
  const uint64_t q = __umul64hi(x, inv);
  uint64_t rem = x - q * d;
  while (rem >= d) rem -= d;
  return (uint32_t)rem;
}
}  // namespace

__global__ __launch_bounds__(256) void k_sieve(const SieveArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.count) return;
  constexpr int W = MPCX_SIEVE_MAX_BYTES / 4;
  uint32_t q[W];
#pragma unroll
  for (int w = 0; w < W; ++w) q[w] = 0;
  const uint8_t* b = a.raw + (size_t)i * a.nbytes;
  const uint32_t n = a.nbytes;
  uint32_t bm = a.q_bits % 8u;
  if (bm == 0) bm = 8;
  // big-endian bytes -> little-endian words, with the masks of step 1
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t v = b[j];
    if (j == 0) {
      v &= (1u << bm) - 1u;
      v |= bm >= 2 ? (3u << (bm - 2)) : 1u;
    }
    if (j == 1 && bm < 2) v |= 0x80u;
    if (j == n - 1) v |= 1u;
    const uint32_t pos = n - 1 - j;  // byte position from the least significant end
#pragma unroll
    for (int w = 0; w < W; ++w)
      if ((uint32_t)w == (pos >> 2)) q[w] |= v << (8u * (pos & 3u));
  }
  // step 2: residues mod 3..53, delta walk
  constexpr uint32_t sp[15] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53};
  uint32_t r[15];
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int w = W - 1; w >= 0; --w) acc = ((acc << 32) | q[w]) % sp[k];
    r[k] = (uint32_t)acc;
  }
  uint32_t delta = 0;
  for (uint32_t d = 0; d < (1u << 20); d += 2) {
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 15; ++k) bad |= (r[k] + d) % sp[k] == 0;
    if (!bad) {
      delta = d;
      break;
    }
  }
  {
    uint64_t c = delta;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      c += q[w];
      q[w] = (uint32_t)c;
      c >>= 32;
    }
  }
  // step 3: bit length
  uint32_t bits = 0;
#pragma unroll
  for (int w = 0; w < W; ++w)
    if (q[w]) bits = 32u * w + 32u - __builtin_clz(q[w]);
  if (bits != a.q_bits) return;
  // trial division of q and 2q+1
  for (uint32_t g = 0; g < a.ngroups; ++g) {
    const uint32_t d = a.tprod[g];
    const uint64_t inv = a.tinv[g];
    uint32_t rr = 0;
#pragma unroll
    for (int w = W - 1; w >= 0; --w) rr = mod_step(rr, q[w], d, inv);
    for (uint32_t t = a.tstart[g]; t < a.tstart[g + 1]; ++t) {
      const uint32_t pr = a.tprimes[t];
      const uint32_t rq = rr % pr;
      if (rq == 0 || (2u * rq + 1u) % pr == 0) return;
    }
  }
  const uint32_t slot = atomicAdd(a.out_count, 1u);
  a.out_idx[slot] = i;
  uint32_t* o = a.out_p + (size_t)slot * W;
  uint32_t c = 1;  // p = 2q + 1
#pragma unroll
  for (int w = 0; w < W; ++w) {
    o[w] = (q[w] << 1) | c;
    c = q[w] >> 31;
  }
}

}  // namespace mpcx

extern "C" {

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_prime2(const mpcx::Prime2Args* a, uint32_t blocks,
                                                                   hipStream_t st) {
  hipLaunchKernelGGL((mpcx::k_prime2<MPCX_C0_K, MPCX_WAVES_PER_EU_FERMAT>), dim3(blocks), dim3(64), 0, st, *a);
  return hipGetLastError();
}

// cooperative base-2 tests: per-item constants, then P lanes per candidate
// (the caller sets f_blocks = ceil(count_f / (64 / MPCX_PRIME_P)) and
// fp_blocks = ceil(count_f / 64))
__attribute__((visibility("hidden"))) hipError_t mpcx_launch_prime2c(const mpcx::Prime2Args* a, hipStream_t st) {
  constexpr uint32_t G = 64 / MPCX_PRIME_P;
  const uint32_t pb = a->fp_blocks + (a->count_s + 63) / 64;
  const uint32_t cb = a->f_blocks + (a->count_s + G - 1) / G;
  if (pb) hipLaunchKernelGGL((mpcx::k_pprep_prime2<MPCX_PRIME_L>), dim3(pb), dim3(64), 0, st, *a);
  if (cb)
    hipLaunchKernelGGL((mpcx::k_prime2c<MPCX_PRIME_P, MPCX_PRIME_K, MPCX_WAVES_PER_EU_PRIME2C>), dim3(cb), dim3(64), 0,
                       st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_mrc(const mpcx::MrArgs* a, hipStream_t st) {
  constexpr uint32_t G = 64 / MPCX_MR_P;
  if (a->count == 0) return hipSuccess;
  hipLaunchKernelGGL((mpcx::k_pprep_mr<MPCX_MR_L>), dim3((a->count + 63) / 64), dim3(64), 0, st, *a);
  hipLaunchKernelGGL((mpcx::k_mrc<MPCX_MR_P, MPCX_MR_K, MPCX_WAVES_PER_EU_MRC>), dim3((a->count + G - 1) / G), dim3(64),
                     0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_lucasc(const mpcx::LucasArgs* a, hipStream_t st) {
  constexpr uint32_t G = 64 / MPCX_MR_P;
  if (a->count == 0) return hipSuccess;
  hipLaunchKernelGGL((mpcx::k_pprep_lucas<MPCX_MR_L>), dim3((a->count + 63) / 64), dim3(64), 0, st, *a);
  hipLaunchKernelGGL((mpcx::k_lucasc<MPCX_MR_P, MPCX_MR_K, MPCX_WAVES_PER_EU_MRC>), dim3((a->count + G - 1) / G),
                     dim3(64), 0, st, *a);
  return hipGetLastError();
}

// candidates of 1025..2048 bits (consts: count x 4 x MPCX_LUCASW_L digits)
__attribute__((visibility("hidden"))) hipError_t mpcx_launch_lucasc_wide(const mpcx::LucasArgs* a, hipStream_t st) {
  constexpr uint32_t G = 64 / MPCX_MR_P;
  if (a->count == 0) return hipSuccess;
  hipLaunchKernelGGL((mpcx::k_pprep_lucas<MPCX_LUCASW_L>), dim3((a->count + 63) / 64), dim3(64), 0, st, *a);
  hipLaunchKernelGGL((mpcx::k_lucasc<MPCX_MR_P, MPCX_LUCASW_K, MPCX_WAVES_PER_EU_MRC>), dim3((a->count + G - 1) / G),
                     dim3(64), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_lucas(const mpcx::LucasArgs* a, uint32_t blocks,
                                                                  hipStream_t st) {
  hipLaunchKernelGGL((mpcx::k_lucas<MPCX_C0_K, MPCX_WAVES_PER_EU_MR>), dim3(blocks), dim3(64), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_drbg(const mpcx::DrbgArgs* a, hipStream_t st) {
  const uint64_t blocks = ((a->off + a->n + 31) >> 5) - (a->off >> 5);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(mpcx::k_drbg, dim3((uint32_t)((blocks + 255) / 256)), dim3(256), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_mr(const mpcx::MrArgs* a, uint32_t blocks,
                                                               hipStream_t st) {
  hipLaunchKernelGGL((mpcx::k_mr<MPCX_C0_K, MPCX_WAVES_PER_EU_MR>), dim3(blocks), dim3(64), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_expsched(const mpcx::ExpSchedArgs* a,
                                                                      hipStream_t st) {
  hipLaunchKernelGGL(mpcx::k_expsched, dim3(1), dim3(64), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_sieve(const mpcx::SieveArgs* a, hipStream_t st) {
  hipLaunchKernelGGL(mpcx::k_sieve, dim3((a->count + 255) / 256), dim3(256), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_selftest(uint32_t* d_out, hipStream_t st) {
  hipLaunchKernelGGL(mpcx::k_selftest, dim3(1), dim3(64), 0, st, d_out);
  return hipGetLastError();
}

}  // extern "C"
