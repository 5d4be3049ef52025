// mpcx_prime.hip -- launchers of the safe-prime kernels (Fermat base 2,
// Miller-Rabin; thread per candidate), the shared-exponent window schedule
// (k_expsched) and the device self-test.
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

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_fermat2(const mpcx::FermatArgs* a, uint32_t blocks,
                                                                    hipStream_t st) {
  hipLaunchKernelGGL((mpcx::k_fermat2<MPCX_C0_K, MPCX_WAVES_PER_EU_FERMAT>), dim3(blocks), dim3(64), 0, st, *a);
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
