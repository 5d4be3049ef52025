// mpcx_device.hpp -- gfx950 (MI355X, CDNA4) batched modular exponentiation:
// device code shared by the per-geometry translation units (mpcx_geom.hip)
// and the primality kernels (mpcx_prime.hip).
//
// Replaces the arithmetic of Go math/big (*Int).Exp -> nat.expNNMontgomery
// (go1.23.5, go:src/math/big/nat.go) as reached through tss-lib v2.0.2
// common.ModInt(m).Exp (up:common/int.go) on mpcium's hot path
// (/root/reference/pkg/mpc/session.go:199 -> party.UpdateFromBytes -> Paillier /
// MtA proofs; /root/reference/pkg/mpc/node.go:69 -> GeneratePreParams).
//
// Design (DESIGN.md section "Kernels"):
//  * Radix 2^28 digits held in 64-bit lazy accumulators. A 28x28-bit product
//    is < 2^56, so an accumulator absorbs > 100 products before it can
//    overflow: every multiply-accumulate is ONE v_mad_u64_u32 (half rate on
//    gfx950, measured ~33.8 T/s/GPU), with no per-MAC carry instruction --
//    the carry-writing v_add_co/v_addc are half rate as well, so a 32-bit-limb
//    carry chain would cost >= 2 half-rate ops per MAC.
//  * Wavefront-cooperative operands: one 64-lane wavefront holds G operands;
//    operand g is spread over P lanes, each lane holding K consecutive digits
//    (L = P*K digits, R = 2^(28L) > 4m so no conditional subtraction is ever
//    needed inside the exponentiation: almost-Montgomery, results < 2m).
//  * Row-wise (CIOS) Montgomery: per digit b_i of the multiplier, every lane
//    does K mads for a*b_i, the group's lane 0 derives m_i, one ds_bpermute
//    broadcasts it, K more mads for m_i*N, then the accumulator window shifts
//    one digit: within a lane by register renaming (the K-iteration block is
//    unrolled), across lanes by ONE DPP wave_shl of a 28-bit value (the slot's
//    high part is folded into the next slot first).
//  * Exponentiation: a shared exponent follows a sliding-window schedule (odd
//    powers, windows of up to 6 bits, built on the device by k_expsched);
//    per-operand exponents use Go's fixed 4-bit window. Tables (<= 33 entries
//    per operand) live in a global workspace, lane-coalesced; b operands are
//    staged in LDS and read as group-broadcast ds_read_b32.
//  * The per-operand product is not a dense contraction. The REDUCTION of a
//    batch that shares its modulus is (fixed Toeplitz matrices of m'' and m):
//    geometry 2 runs it on the i8 matrix cores, k_modexp_mx (mpcx_mx.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "mpcx_internal.h"

#ifndef MPCX_SCHED_BARRIER
#define MPCX_SCHED_BARRIER 0
#endif
#ifndef MPCX_SQR_OPT
#define MPCX_SQR_OPT 1  // half-product squarings (montmul<..., true>)
#endif
#ifndef MPCX_PREFETCH2_KMAX
#define MPCX_PREFETCH2_KMAX 24  // montmul reads b two digits ahead for K below this
#endif
#ifndef MPCX_PREFETCH_B
#define MPCX_PREFETCH_B 1
#endif
#ifndef MPCX_SQR_B2
#define MPCX_SQR_B2 1  // k_modexp / k_prime2c squarings read 2*b from LDS (no per-iteration doubling)
#endif
#ifndef MPCX_BLOCK_FENCE
#define MPCX_BLOCK_FENCE 0  // scheduling fence between montmul's P blocks (1: all, 2: K >= 16; the prime kernels' TU sets 1)
#endif
#ifndef MPCX_PRIME2C_DBL_FOLD
#define MPCX_PRIME2C_DBL_FOLD 1  // k_prime2c: the square-and-double step as one product with B = 2^bit x
#endif
#ifndef MPCX_WAVES_PER_EU_FERMAT
#define MPCX_WAVES_PER_EU_FERMAT 1
#endif
#ifndef MPCX_WAVES_PER_EU_PRIME2C
#define MPCX_WAVES_PER_EU_PRIME2C 3
#endif
#ifndef MPCX_WAVES_PER_EU_MRC
#define MPCX_WAVES_PER_EU_MRC 3
#endif
#ifndef MPCX_WAVES_PER_EU_MR
#define MPCX_WAVES_PER_EU_MR 1
#endif

namespace mpcx {

// Compile-time loop: f(std::integral_constant<int, i>) for i in [B, E).
// Guarantees constant register-array indices (a partially unrolled loop
// would demote the accumulators to scratch memory).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

constexpr int DB = 28;
constexpr uint32_t M28 = (1u << DB) - 1u;

// lane l receives lane l+1's value; lane 63 receives 0 (DPP wave_shl:1, bound_ctrl zero).
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}
// lane l receives lane l-1's value; lane 0 receives 0 (DPP wave_shr:1).
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}

// Broadcast lane 0 of each P-lane operand group to the whole group. Quads
// (P = 4) and pairs (P = 2) use a DPP quad_perm, 8-lane groups a quad_perm plus
// row_shr:4 into the upper quad, 16-lane groups (one DPP row)
// DPP row_newbcast, 32-lane groups row_newbcast + row_bcast:15 -- a VALU move with a few cycles of latency on the
// per-iteration serial path; other group widths go through the LDS crossbar
// (ds_bpermute, ~100+ cycles of latency).
template <int P>
__device__ __forceinline__ uint32_t group_bcast(uint32_t v, int src_addr) {
  if constexpr (P == 4) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);  // quad_perm [0,0,0,0]
  } else if constexpr (P == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
  } else if constexpr (P == 8) {
    // each quad takes its lane 0, then the upper quad of every 8-lane group
    // (DPP banks 1 and 3) takes the lower quad's value by row_shr:4
    const int t = __builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(t, t, 0x114, 0xF, 0xA, false);
  } else if constexpr (P == 16) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150, 0xF, 0xF, false);  // row_newbcast:0
  } else if constexpr (P == 32) {
    // every row takes its lane 0, then rows 1 and 3 take lane 15 of the row
    // below (= lane 0 of rows 0 and 2) by row_bcast:15
    const int t = __builtin_amdgcn_mov_dpp((int)v, 0x150, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(t, t, 0x142, 0xA, 0xF, false);
  } else {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_addr, (int)v);
  }
}

// acc += a * b (32x32 -> 64 plus 64-bit addend): hipcc lowers this to ONE
// v_mad_u64_u32. (Inline asm would force ~20 s_nop hazard pads per digit
// iteration around its SGPR carry-out.)
__device__ __forceinline__ void mad64(uint64_t& acc, uint32_t a, uint32_t b) {
  acc += (uint64_t)a * b;
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One carry pass over 64-bit redundant digits: digit k keeps its low 28 bits
// and receives the high part of digit k-1 (across lanes via DPP). The carry
// out of a group's top digit is provably zero (value < R), so group
// boundaries need no masking.
template <int P, int K>
__device__ __forceinline__ void carry_pass64(uint64_t (&acc)[K]) {
  // in place, top slot first, so only one carry is live at a time
  const uint64_t ctop = acc[K - 1] >> DB;
#pragma unroll
  for (int k = K - 1; k >= 1; --k) acc[k] = (acc[k] & M28) + (acc[k - 1] >> DB);
  acc[0] &= M28;
  if constexpr (P > 1) {
    const uint32_t clo = from_prev_lane((uint32_t)ctop);
    const uint32_t chi = from_prev_lane((uint32_t)(ctop >> 32));
    acc[0] += ((uint64_t)chi << 32) | clo;
  }
}

template <int P, int K>
__device__ __forceinline__ void carry_pass32(uint32_t (&d)[K]) {
  const uint32_t ctop = d[K - 1] >> DB;
#pragma unroll
  for (int k = K - 1; k >= 1; --k) d[k] = (d[k] & M28) + (d[k - 1] >> DB);
  d[0] &= M28;
  if constexpr (P > 1) d[0] += from_prev_lane(ctop);
}

// A <- A * B * R^-1 (almost Montgomery, result < 2N given A, B < 2N), with
// B's L digits in LDS at bl[0..L) (p = this lane's index in its group).
// Result digits are <= 2^28 + 2^8 (two carry passes at the end), which keeps
// every product below 2^56.01 (2^57.02 for the doubled squaring products);
// each accumulator register restarts every K iterations (see the end of the
// block loop), so it stays below 2^63 with no carry pass inside the product.
//
// SQR (B == A, squaring): each unordered digit pair {i, j} needs ONE product
// 2*a_i*a_j (plus a_i^2 on the diagonal). In iteration t the product of
// multiplicand register k (digit s = p*K + k) is needed iff d = (k - t) mod K
// lies in [1, (K-1)/2] (doubled), or d == 0 with a per-lane factor
// (2 above the diagonal lane, 1 on it, 0 below); every other register is
// skipped for ALL lanes -- a compile-time decision, since t mod K is the
// unrolled index. Each pair lands in its column before that column is
// reduced (both orientations use an iteration <= i + j). K must be odd.
// Saves (K-1)/2 of the K a*b mads of every squaring iteration.
// B2IN (squarings only): the LDS row holds 2*b (digits < 2^30.01), stored so
// by the caller, which saves the per-iteration doubling.
template <int P, int K, bool SQR, bool B2IN = false>
__device__ __forceinline__ void montmul(uint32_t (&A)[K], const uint32_t* bl, const uint32_t (&Nd)[K],
                                        uint32_t n0inv, int m_src_addr, int p) {
  static_assert(SQR || !B2IN, "doubled multiplier rows are for squarings");
  static_assert(!SQR || (K % 2) == 1, "squaring schedule needs an odd digit count per lane");
  uint64_t acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0;
  // b digits are read from LDS ahead of use: one iteration ahead, or two for
  // short iterations (K < MPCX_PREFETCH2_KMAX: half an iteration of a K = 19
  // squaring is ~60 cycles, under the LDS read latency). Rows carry 2 digits
  // of padding for the reads past their end.
  constexpr bool PF2 = K < MPCX_PREFETCH2_KMAX;
  uint32_t bnext = bl[0];
  uint32_t bnext2 = PF2 ? bl[1] : 0u;
  // one copy of the K-iteration block (unrolling the P blocks would multiply
  // the code and the live ranges: k_prime2c spilled with P = 2 unrolled)
#pragma nounroll
  for (int o = 0; o < P; ++o) {
    const uint32_t* bo = bl + o * K;
    // diagonal-register factor of this lane for the whole block (2 above the
    // diagonal lane, 1 on it, 0 below) as a right shift of b2 = 2*b_i: digits
    // are < 2^29, so b2 < 2^30 and b2 >> 31 == 0. One v_lshrrev_b32 instead of
    // a v_mul_lo_u32 (which issues at MAD rate) per squaring iteration.
    const uint32_t dsh = p > o ? 0u : (p == o ? 1u : 31u);
    static_for<0, K>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const uint32_t bi = bnext;
      if constexpr (PF2) {
        bnext = bnext2;
        bnext2 = bo[u + 2];
      }
      const uint32_t b2 = B2IN ? bi : bi << 1;
      const uint32_t bd = b2 >> dsh;
      auto ab = [&](auto kc) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        if constexpr (!SQR) {
          mad64(acc[(k + u) % K], A[k], bi);
        } else {
          constexpr int d = ((k - u) % K + K) % K;
          if constexpr (d == 0) {
            mad64(acc[(k + u) % K], A[k], bd);
          } else if constexpr (d <= (K - 1) / 2) {
            mad64(acc[(k + u) % K], A[k], b2);
          }
        }
      };
      // slot 0 first: it feeds m_i, the only serial dependency of the iteration
      ab(std::integral_constant<int, 0>{});
      uint32_t m = ((uint32_t)acc[u] * n0inv) & M28;
      if constexpr (P > 1) m = group_bcast<P>(m, m_src_addr);
#if MPCX_PREFETCH_B
      // next digit of b, in flight behind the bpermute and the a*b_i mads
      // (the last read of the last block touches the neighbour row: unused)
      if constexpr (!PF2) bnext = bo[u + 1];
#endif
      static_for<1, K>(ab);
#if !MPCX_PREFETCH_B
      if constexpr (!PF2) bnext = bo[u + 1];
#endif
      static_for<0, K>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        mad64(acc[(k + u) % K], m, Nd[k]);
      });
      const uint64_t a0 = acc[u];
      acc[(u + 1) % K] += a0 >> DB;
      if constexpr (P > 1) {
        acc[u] = from_next_lane((uint32_t)a0 & M28);
      } else {
        acc[u] = 0;
      }
#if MPCX_SCHED_BARRIER
      // keep iterations from being interleaved by the machine scheduler: it
      // otherwise hoists b loads and mads across iterations and blows the
      // register budget (occupancy) for no issue-rate gain
      __builtin_amdgcn_sched_barrier(0);
#endif
    });
    // No mid-way carry pass is needed: a register is reset (slot 0 retires to
    // a 28-bit value) once every K iterations, so it sums at most K iterations
    // of one a*b and one m*N product (< 2^58.02 + 2^56 for the doubled
    // squaring row of k_prime2c, whose digits reach 2^30.01) plus a < 2^35
    // fold: < 2^62.8 for K <= 37. profiles/r03/kernel_ab: dropping the pass
    // took the config-2 kernel from 176.3 to 171.7 ms.
    // block boundary as a scheduling fence (mpcx_prime.hip: without it
    // k_prime2c's live ranges grew past its 3-wave budget and spilled; the
    // k_modexp geometries fit better without it). 2: long blocks only (K >= 16).
    if constexpr (MPCX_BLOCK_FENCE == 1 || (MPCX_BLOCK_FENCE == 2 && K >= 16)) __builtin_amdgcn_sched_barrier(0);
  }
  carry_pass64<P, K>(acc);
  // digits are now < 2^28 + 2^37: one more pass brings them to <= 2^28 + 2^10
  const uint32_t ctop = (uint32_t)(acc[K - 1] >> DB);
#pragma unroll
  for (int k = K - 1; k >= 1; --k) A[k] = ((uint32_t)acc[k] & M28) + (uint32_t)(acc[k - 1] >> DB);
  A[0] = (uint32_t)acc[0] & M28;
  if constexpr (P > 1) A[0] += from_prev_lane(ctop);
}

// Canonical digits (< 2^28): repeat carry passes until no digit overflows.
template <int P, int K>
__device__ __forceinline__ void canonicalize(uint32_t (&A)[K]) {
  for (int it = 0; it < P * K + 2; ++it) {
    bool over = false;
#pragma unroll
    for (int k = 0; k < K; ++k) over |= A[k] > M28;
    if (!__any(over)) break;
    carry_pass32<P, K>(A);
  }
}

template <int K>
__device__ __forceinline__ void lds_store_digits(uint32_t* bl, int p, const uint32_t (&A)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) bl[p * K + k] = A[k];
}

// the squaring's multiplier row: 2*A when montmul reads it as B2IN, else A
template <int K>
__device__ __forceinline__ void lds_store_sqr(uint32_t* bl, int p, const uint32_t (&A)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) bl[p * K + k] = MPCX_SQR_B2 ? A[k] << 1 : A[k];
}

// bits [wb*j, wb*j + wb) of the ew-word exponent e (wb <= 32; bits past the
// top word read as 0)
__device__ __forceinline__ uint32_t window_of(const uint32_t* e, uint32_t j, uint32_t wb, uint32_t ew) {
  const uint32_t bit = wb * j, w = bit >> 5, sh = bit & 31u;
  uint32_t v = e[w] >> sh;
  if (sh + wb > 32u && w + 1u < ew) v |= e[w + 1u] << (32u - sh);
  return v & ((1u << wb) - 1u);
}

// Leaves A (<= m after the Montgomery-domain exit mont(z R, 1)) canonical,
// maps m -> 0, and writes the operand's out_words words (digits -> words
// through the group's LDS row).
template <int P, int K>
__device__ __forceinline__ void store_result(uint32_t (&A)[K], const uint32_t (&Nd)[K], uint32_t* bl, int p,
                                             int g_raw, bool idle, bool active, uint32_t* o, uint32_t out_words) {
  constexpr int L = P * K;
  canonicalize<P, K>(A);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < K; ++k) eq &= (A[k] == Nd[k]);
  const uint64_t bal = __ballot(eq || idle);
  const uint64_t gmask = (P == 64 ? ~0ull : (((1ull << P) - 1ull) << (g_raw * P)));
  if (!idle && (bal & gmask) == gmask) {
#pragma unroll
    for (int k = 0; k < K; ++k) A[k] = 0;
  }
  wave_lds_fence();
  lds_store_digits<K>(bl, p, A);
  wave_lds_fence();
  if (active) {
    for (uint32_t w = (uint32_t)p; w < out_words; w += P) {
      const uint32_t bit = w * 32u;
      const uint32_t d0 = bit / DB, s0 = bit % DB;
      uint32_t v = 0;
      if (d0 < (uint32_t)L) {
        // s0 = 32w mod 28 <= 24, so bits [s0, s0+32) lie in two digits
        const uint64_t lo = bl[d0];
        const uint64_t hi = (d0 + 1 < (uint32_t)L) ? bl[d0 + 1] : 0u;
        v = (uint32_t)((lo | (hi << DB)) >> s0);
      }
      o[w] = v;
    }
  }
}

}  // namespace mpcx
#include "mpcx_mx.hpp"
namespace mpcx {

// Batched x_i^e_i mod m for one registered odd modulus m: wavefront `blk` of
// the batch described by a (k_modexp: one batch per launch; k_modexp_multi:
// several batches, each its own segment of the launch's wavefronts).
// MX (geometry 2 only, a.mx_img set; MX_WG wavefronts per workgroup): every
// product but the final exit runs as montmul_mx (reduction on the matrix cores,
// mpcx_mx.hpp) with the workgroup's LDS copy of the Toeplitz tables; the
// multiplier row is montmul_mx's scratch, so a row that the state machine reuses
// across products is staged again before each (`restage`).
template <int P, int K, int G, bool MX = false>
__device__ __forceinline__ void modexp_wave(const ModexpArgs& a, const uint32_t blk) {
  constexpr int L = P * K;
  using S = MxShape<P, K, G>;
  static_assert(!MX || (P == 4 && K == 37 && G == 16) || (P == 2 && K == 37 && G == 32),
                "montmul_mx serves geometries 2 and 5");
  // +2: the b prefetch reads up to two past a row; MX: tables, m's digits, rows
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[MX ? S::LDS_WORDS_WG : (G + 1) * L + 2];
  uint32_t* lds = lds_all;
  if constexpr (MX) {
    // the workgroup's tables and m's digits, then the wavefronts part
    const uint32_t* img = static_cast<const uint32_t*>(a.mx_img);
    for (int i = (int)threadIdx.x; i < S::IMG_BYTES / 4; i += 64 * MX_WG) lds_all[i] = img[i];
    for (int i = (int)threadIdx.x; i < L; i += 64 * MX_WG) lds_all[S::IMG_BYTES / 4 + i] = a.nd[i];
    __syncthreads();
    if (blk >= a.nwaves) return;  // the last workgroup's spare wavefronts
    lds = lds_all + S::IMG_BYTES / 4 + L + 4 + (threadIdx.x >> 6) * S::WAVE_WORDS;
  }
  const int lane = MX ? (int)(threadIdx.x & 63u) : (int)threadIdx.x;
  const int g_raw = lane / P;
  const bool idle = g_raw >= G;  // lanes beyond G*P carry zeros
  const int g = idle ? G : g_raw;
  const int p = lane - g_raw * P;
  const uint32_t op = blk * G + (idle ? 0 : g_raw);
  const bool active = !idle && op < a.count;
  uint32_t* bl = lds + g * (MX ? S::ROW : L);
  const int m_src_addr = (idle ? lane : g_raw * P) * 4;

  uint32_t Nd[K], A[K];
  // L digits of a constant (m, R^2 mod m) into registers; MX: through an opaque
  // pointer and lane index, so the per-digit addresses are not hoisted out of
  // the step loop and held live across every product (as load_digits)
  auto load_const = [&] __attribute__((always_inline))(const uint32_t* src, uint32_t (&v)[K]) {
    if constexpr (MX) asm volatile("" : "+s"(src));
    int pp = p;
    if constexpr (MX) asm volatile("" : "+v"(pp));
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = idle ? 0u : src[pp * K + k];
  };
  auto load_nd = [&] __attribute__((always_inline))() { load_const(a.nd, Nd); };
  if constexpr (!MX) load_nd();  // MX: only the exit product and store_result need m in registers
  MxConsts mxc{};
  const uint32_t* mx_md = lds_all + S::IMG_BYTES / 4;  // MX: m's digits (LDS)
  if constexpr (MX) mxc = mx_consts<S>(reinterpret_cast<const uint8_t*>(lds_all), lane);

  // operand words -> radix-2^28 digits (inactive operands compute on zero)
  auto load_digits = [&] __attribute__((always_inline))(const uint32_t* src, uint32_t words) {
    // opaque pointer and lane index: keeps the per-digit address/shift math
    // from being hoisted out of the step loop and held live across every
    // montmul (it cost ~3K registers and forced spills)
    asm volatile("" : "+s"(src));
    int pp = p;
    asm volatile("" : "+v"(pp));
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t bit = (uint32_t)(pp * K + k) * DB;
      const uint32_t w = bit >> 5, sh = bit & 31u;
      uint64_t v = 0;
      if (active) {
        const uint32_t* x = src + (size_t)op * words;
        const uint32_t lo = w < words ? x[w] : 0u;
        const uint32_t hi = (w + 1) < words ? x[w + 1] : 0u;
        v = ((uint64_t)hi << 32) | lo;
      }
      A[k] = (uint32_t)(v >> sh) & M28;
    }
  };

  // fixed window of wb bits (4, or 5 for long per-operand exponents): a step is
  // wb squarings and one multiply by the operand's own window's table entry
  const uint32_t wb = a.win_bits;
  const uint32_t nw = (a.exp_bits + wb - 1u) / wb;
  const uint32_t* ex = a.exp_shared ? a.exps : a.exps + (size_t)(active ? op : 0) * a.exp_words;
  // Per-wavefront table of MPCX_TABLE_ENTRIES entries x K digit-slots x 64 lanes, accessed
  // through a buffer descriptor: lane offset in one VGPR, entry/slot offset
  // in an SGPR (no per-slot address registers live across the montmuls).
  uint32_t* tbl = a.table + (size_t)blk * MPCX_TABLE_ENTRIES * K * 64u;
  const auto tbl_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(tbl, (short)0, (int)(MPCX_TABLE_ENTRIES * K * 64u * 4u), 0x00020000);
  const int tbl_lane_off = lane * 4;
  // entry offset (possibly per-lane) in voffset, slot offset k*256 as a constant soffset
  auto tbl_store = [&](uint32_t e, const uint32_t (&v)[K]) __attribute__((always_inline)) {
    const int voff = tbl_lane_off + (int)(e * K * 256u);
#pragma unroll
    for (int k = 0; k < K; ++k) __builtin_amdgcn_raw_buffer_store_b32(v[k], tbl_rsrc, voff, k * 256, 0);
  };
  auto tbl_load = [&](uint32_t e, uint32_t (&v)[K]) __attribute__((always_inline)) {
    const int voff = tbl_lane_off + (int)(e * K * 256u);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b32(tbl_rsrc, voff, k * 256, 0);
  };
  auto lds_from_table = [&] __attribute__((always_inline))(uint32_t e) {
    uint32_t tv[K];
    tbl_load(e, tv);
    lds_store_digits<K>(bl, p, tv);
  };
  auto lds_one = [&] __attribute__((always_inline))() {
    uint32_t one[K];
#pragma unroll
    for (int k = 0; k < K; ++k) one[k] = (p == 0 && k == 0 && !idle) ? 1u : 0u;
    lds_store_digits<K>(bl, p, one);
  };

  // table[0] = R mod m (Montgomery one); LDS <- R^2 mod m for the conversions
  {
    uint32_t r1[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r1[k] = idle ? 0u : a.r1d[p * K + k];
    tbl_store(0, r1);
  }
  {
    uint32_t r2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r2[k] = idle ? 0u : a.r2d[p * K + k];
    lds_store_digits<K>(bl, p, r2);
  }
  const bool has_mul = a.mul != nullptr;
  // Control state must stay provably wave-uniform (SGPRs): the schedule and a
  // shared exponent are read through readfirstlane, so the compiler keeps the
  // step machine and the table offsets off the VGPR file.
  //
  // A shared exponent e >= 1 follows the sliding-window schedule k_expsched
  // built from it on the same stream (ExpSched layout in mpcx_internal.h):
  // odd powers x^1, x^3, ..., x^(2 Tn + 1) in table[0..Tn], z = x^top, then
  // per entry s squarings and one multiply by an odd power. Windows of up to
  // 6 bits cost ~E/7 multiplies against Go's E/4 * 15/16; every decision
  // depends on e only, so the wave stays uniform. Per-operand exponents (and
  // e = 0) keep a fixed window (wb bits, every operand multiplies every step):
  // sliding windows would diverge.
  const bool sched = a.exp_shared != 0 && a.sched != nullptr &&
                     __builtin_amdgcn_readfirstlane(a.sched[MPCX_SCHED_TOP]) != MPCX_SCHED_NONE;
  const uint32_t wt = nw > 0 ? window_of(ex, nw - 1u, wb, a.exp_words) : 0u;
  // table entries built: fixed window p_1..p_T (a shared e < 2^wb needs p_1..p_e only)
  const uint32_t wt_u = __builtin_amdgcn_readfirstlane(wt);
  const uint32_t T = sched ? __builtin_amdgcn_readfirstlane(a.sched[MPCX_SCHED_TN])
                           : (a.exp_shared && nw <= 1u ? (wt_u > 1u ? wt_u : 1u) : (1u << wb) - 1u);
  // exponent steps: schedule entries, or windows below the top one
  const uint32_t nsteps = sched ? __builtin_amdgcn_readfirstlane(a.sched[MPCX_SCHED_N]) : (nw > 0 ? nw - 1u : 0u);

  // Montgomery-step state machine (ONE montmul call site keeps the code small):
  //   PRE : mul*R   = mont(mul, R^2)           -> table[MPCX_MUL_ENTRY]   (only with a multiplier)
  //   TAB : fixed window: p_i = mont(x, R^2), mont(p_{i-1}, p_1)  i = 1..T -> table[i]
  //         schedule:     x R = mont(x, R^2) -> table[0]
  //   TSQ : x^2 R (schedule, Tn > 0)
  //   STAB: x^(2i+1) R = mont(x^(2i-1) R, x^2 R) -> table[i], i = 1..Tn
  //   EXP : per step: s squarings, then mont(z, table entry)
  //         (fixed window: s = 4 and the operand's window, p_0 = R mod m)
  //   MULF: z*mul*R = mont(z*R, mul*R)                          (only with a multiplier)
  //   FIN : z       = mont(z*R, 1) <= m
  enum { ST_PRE, ST_TAB, ST_TSQ, ST_STAB, ST_EXP, ST_MULF, ST_FIN };
  int st;
  uint32_t idx = 1;
  bool sqr = false;  // next montmul is a squaring (B == A)
  if (has_mul) {
    load_digits(a.mul, a.mul_words);
    st = ST_PRE;
  } else {
    load_digits(a.base, a.base_words);
    st = ST_TAB;
  }
  wave_lds_fence();

  // Exponent steps (one inlined instance): a step is sq_left squarings, then
  // one multiply by table[pend] (pend < 0: none).
  uint32_t sq_left = 0;
  int pend = -1;  // uniform: table entry, or 0x100 for the operand's own window
  auto prepare_exp = [&] __attribute__((always_inline))() {
    for (;;) {
      if (sq_left) {
        --sq_left;
        lds_store_sqr<K>(bl, p, A);
        sqr = true;
        return;
      }
      if (pend >= 0) {
        // fixed window: the operand's window of the step just scheduled (idx - 1)
        lds_from_table(pend == 0x100 ? window_of(ex, nw - 1u - idx, wb, a.exp_words) : (uint32_t)pend);
        pend = -1;
        return;
      }
      if (idx == nsteps) {
        if (has_mul) {
          st = ST_MULF;
          lds_from_table(MPCX_MUL_ENTRY);
        } else {
          st = ST_FIN;
          lds_one();
        }
        return;
      }
      if (sched) {
        const uint32_t s = __builtin_amdgcn_readfirstlane(a.sched[MPCX_SCHED_STEPS + idx]);
        sq_left = s >> 8;
        pend = (s & 0xFFu) == 0xFFu ? -1 : (int)(s & 0xFFu);
      } else {
        sq_left = wb;
        pend = 0x100;
      }
      ++idx;
    }
  };

  int restage = -1;  // MX: table entry (or MX_RESTAGE_R2) to put back in the row before the next product
  constexpr int MX_RESTAGE_R2 = -2;
  for (;;) {
    if constexpr (MX) {
      if (restage != -1) {
        if (restage == MX_RESTAGE_R2) {
          uint32_t r2[K];
          load_const(a.r2d, r2);
          lds_store_digits<K>(bl, p, r2);
        } else {
          lds_from_table((uint32_t)restage);
        }
        restage = -1;
        wave_lds_fence();
      }
      if (st == ST_FIN) break;  // the exit product runs after the loop (m's digits live only there)
      if (sqr) {
        montmul_mx<S, true, (bool)MPCX_SQR_B2>(A, lds, mx_md, mxc, lane);
      } else {
        montmul_mx<S, false, false>(A, lds, mx_md, mxc, lane);
      }
    } else if (MPCX_SQR_OPT && sqr) {
      montmul<P, K, true, (bool)MPCX_SQR_B2>(A, bl, Nd, a.n0inv, m_src_addr, p);
    } else {
      montmul<P, K, false>(A, bl, Nd, a.n0inv, m_src_addr, p);
    }
    sqr = false;
    wave_lds_fence();
    bool start_exp = false, run_exp = false;
    if (st == ST_PRE) {
      tbl_store(MPCX_MUL_ENTRY, A);
      load_digits(a.base, a.base_words);  // LDS still holds R^2
      if constexpr (MX) restage = MX_RESTAGE_R2;
      st = ST_TAB;
      idx = 1;
    } else if (st == ST_TAB) {
      tbl_store(sched ? 0u : idx, A);
      if (sched && T > 0u) {
        lds_store_sqr<K>(bl, p, A);
        sqr = true;
        st = ST_TSQ;
      } else if (!sched && idx == 1) {
        lds_store_digits<K>(bl, p, A);  // B = p_1 for the remaining table steps
      } else if (MX && !sched && idx < T) {
        restage = 1;  // the next table step multiplies by p_1 again
      }
      if (!sched && idx < T) {
        ++idx;
      } else if (st == ST_TAB) {
        start_exp = true;  // table complete
      }
    } else if (st == ST_TSQ) {
      lds_store_digits<K>(bl, p, A);  // B = x^2 R for the odd-power chain
      if constexpr (MX) tbl_store(MPCX_SQ_ENTRY, A);
      tbl_load(0, A);
      st = ST_STAB;
      idx = 1;
    } else if (st == ST_STAB) {
      tbl_store(idx, A);
      if (MX && idx < T) restage = MPCX_SQ_ENTRY;  // the next odd power multiplies by x^2 R again
      if (idx < T) {
        ++idx;
      } else {
        start_exp = true;
      }
    } else if (st == ST_EXP) {
      run_exp = true;
    } else if (st == ST_MULF) {
      st = ST_FIN;
      lds_one();
    } else {
      break;  // ST_FIN done
    }
    if (start_exp) {
      // z = x^top (schedule) or p_top (fixed window; Montgomery one if e = 0)
      tbl_load(sched ? __builtin_amdgcn_readfirstlane(a.sched[MPCX_SCHED_TOP]) : wt, A);
      st = ST_EXP;
      idx = 0;
      run_exp = true;
    }
    if (run_exp) prepare_exp();
    wave_lds_fence();
  }

  if constexpr (MX) {
    load_nd();  // exit product mont(z R, 1) <= m by the CIOS loop: canonical as store_result needs
    montmul<P, K, false>(A, bl, Nd, a.n0inv, m_src_addr, p);
  }
  store_result<P, K>(A, Nd, bl, p, g_raw, idle, active, a.out + (size_t)op * a.out_words, a.out_words);
}

template <int P, int K, int G, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_modexp(const ModexpArgs a) {
  modexp_wave<P, K, G>(a, blockIdx.x);
}

// k_modexp_multi with the reduction on the matrix cores: every segment starts on
// a workgroup boundary (first[] counts MX_WG-wavefront workgroups), so the
// workgroup's waves share the segment's tables
template <int P, int K, int G, int WPE>
__global__ __launch_bounds__(64 * MX_WG) __attribute__((amdgpu_waves_per_eu(WPE))) void k_modexp_multi_mx(
    const ModexpArgs* __restrict__ segs, const uint32_t* __restrict__ first, uint32_t nsegs) {
  const uint32_t b = blockIdx.x;
  uint32_t s = 0;
  while (s + 1u < nsegs && __builtin_amdgcn_readfirstlane(first[s + 1u]) <= b) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  modexp_wave<P, K, G, true>(segs[s], (b - __builtin_amdgcn_readfirstlane(first[s])) * MX_WG + (threadIdx.x >> 6));
}

// geometry 2 with the reduction on the matrix cores (a.mx_img set): MX_WG
// wavefronts per workgroup share the tables in LDS
template <int P, int K, int G, int WPE>
__global__ __launch_bounds__(64 * MX_WG) __attribute__((amdgpu_waves_per_eu(WPE))) void k_modexp_mx(
    const ModexpArgs a) {
  modexp_wave<P, K, G, true>(a, blockIdx.x * MX_WG + (threadIdx.x >> 6));
}

// Several batches of one modulus class in one launch (mpcx_modexp_multi_batch:
// different moduli, shared or per-operand exponents, multipliers): segment s
// owns wavefronts [first[s], first[s+1]) and its own ModexpArgs (constants,
// schedule, window-table region), read wave-uniformly.
template <int P, int K, int G, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_modexp_multi(
    const ModexpArgs* __restrict__ segs, const uint32_t* __restrict__ first, uint32_t nsegs) {
  const uint32_t b = blockIdx.x;
  uint32_t s = 0;
  while (s + 1u < nsegs && __builtin_amdgcn_readfirstlane(first[s + 1u]) <= b) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  modexp_wave<P, K, G>(segs[s], b - __builtin_amdgcn_readfirstlane(first[s]));
}

// Fixed-base multi-exponentiation: out_i = mul_i * prod_t b_t^(e_t,i) mod m
// for up to MPCX_FB_MAX_BASES registered bases (h1, h2 of a node's N~;
// up:crypto/mta/range_proof.go z = h1^m h2^rho, up:crypto/dlnproof/proof.go
// alpha_i = h1^a_i). With the comb table b^(v 2^(wj)) per w-bit window there
// are no squarings at all: one Montgomery product per window of each
// exponent, z <- mont(z, T[j][v]), against Go's E squarings + E/4 multiplies
// for the same Exp. Every operand multiplies in every window (v = 0 reads
// the Montgomery one), so the wave never diverges; windows above every
// operand's exponent are skipped by a wave-uniform ballot.
//
// Window split: a workgroup is S = blockDim.x / 64 wavefronts (1, 2 or 4) for
// the SAME G operands; wave w takes windows j = w, w + S, ... of every base
// (interleaved: balanced for short exponents too), waves 1..S-1 leave their
// partial products (Montgomery form) in their LDS rows, and wave 0 multiplies
// them in before leaving the Montgomery domain: S - 1 extra products per
// operand for S times the wavefronts of a launch below a resident round.
// LDS: S slices of (G + 1) L + 2 words (dynamic, sized by the launch).
template <int P, int K, int G>
constexpr uint32_t fb_lds_slice_words() {
  return (uint32_t)((G + 1) * P * K + 2);
}

template <int P, int K, int G>
__device__ __forceinline__ void fixedbase_wave(const FixedBaseArgs& a, const uint32_t blk) {
  constexpr int L = P * K;
  constexpr uint32_t kSlice = fb_lds_slice_words<P, K, G>();
  extern __shared__ uint32_t fb_lds[];
  const uint32_t S = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // lane id from mbcnt: threadIdx.x & 63 made these kernels spill 48-264 B
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int g_raw = lane / P;
  const bool idle = g_raw >= G;
  const int g = idle ? G : g_raw;
  const int p = lane - g_raw * P;
  const uint32_t op = blk * G + (idle ? 0 : g_raw);
  const bool active = !idle && op < a.count;
  uint32_t* bl = fb_lds + wv * kSlice + g * L;
  const int m_src_addr = (idle ? lane : g_raw * P) * 4;

  uint32_t Nd[K], A[K];
#pragma unroll
  for (int k = 0; k < K; ++k) Nd[k] = idle ? 0u : a.nd[p * K + k];
  auto lds_digits = [&](const uint32_t* src) __attribute__((always_inline)) {  // L digits, [p*K + k]
    uint32_t t[K];
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = idle ? 0u : src[p * K + k];
    lds_store_digits<K>(bl, p, t);
  };
  // ONE montmul call site (three would triple the unrolled product and its
  // register allocation); its B operand is this wave's LDS row. The next
  // product's table entry is
  // loaded after the current product: loading it during the product into
  // registers measured 6% slower on config 5 (profiles/r03/fb_prefetch), and
  // staging it into a second LDS row set by LDS DMA (global_load_lds) 5-15%
  // slower in isolation (profiles/r04/fb_dma_ab/isolated). Issue priority for
  // the fetch or for the products: no change (profiles/r06/fbab).
  uint32_t t = 0, j = wv;  // next window: base t, window j
  uint32_t part = 1;  // wave 0: next partial to multiply in
  bool own = true, fin = false;
  // B <- the next window's entry (some operand of the wave has bits there),
  // then the other waves' partials (wave 0), then the exit multiplier 1; false
  // once the exit product has been handed out (waves > 0: once their windows
  // are done). Stored at once: no digits held in registers across a product.
  auto fetch = [&] __attribute__((always_inline))() -> bool {
    for (; t < a.nbases; ++t, j = wv) {
      const uint32_t ew = a.exp_words[t], wb = a.wbits[t];
      const uint32_t* ex = a.exps[t] + (size_t)(active ? op : 0) * ew;
      for (; j < a.nwin[t]; j += S) {
        const uint32_t v = (active && ew) ? window_of(ex, j, wb, ew) : 0u;
        if (__ballot(v != 0u) == 0ull) continue;  // no operand of the wave has bits here
        const uint32_t* e = a.tables[t] + (((size_t)j << wb) + v) * L;
        uint32_t nx[K];
#pragma unroll
        for (int k = 0; k < K; ++k) nx[k] = idle ? 0u : e[k * P + p];
        lds_store_digits<K>(bl, p, nx);
        j += S;
        return true;
      }
    }
    if (own) {  // this wave's windows are done
      own = false;
      if (S > 1u) {
        if (wv) lds_store_digits<K>(bl, p, A);  // the partial, for wave 0
        __syncthreads();
        if (wv) return false;
      }
    }
    if (part < S) {  // wave 0: B <- wave part's partial (copied into this wave's row)
      const uint32_t* src = fb_lds + part * kSlice + g * L;
      uint32_t nx[K];
#pragma unroll
      for (int k = 0; k < K; ++k) nx[k] = src[p * K + k];
      lds_store_digits<K>(bl, p, nx);
      ++part;
      return true;
    }
    if (fin) return false;
    fin = true;  // leave the Montgomery domain: z = mont(z R, 1) <= m
    uint32_t one[K];
#pragma unroll
    for (int k = 0; k < K; ++k) one[k] = (p == 0 && k == 0 && !idle) ? 1u : 0u;
    lds_store_digits<K>(bl, p, one);
    return true;
  };

  // B of the first product: R^2 already in LDS (z = mul R = mont(mul, R^2),
  // wave 0), or the first fetched entry
  bool more = true;
  if (a.mul && wv == 0u) {
    lds_digits(a.r2d);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t bit = (uint32_t)(p * K + k) * DB;
      const uint32_t w = bit >> 5, sh = bit & 31u;
      uint64_t v = 0;
      if (active) {
        const uint32_t* x = a.mul + (size_t)op * a.mul_words;
        const uint32_t lo = w < a.mul_words ? x[w] : 0u;
        const uint32_t hi = (w + 1) < a.mul_words ? x[w + 1] : 0u;
        v = ((uint64_t)hi << 32) | lo;
      }
      A[k] = (uint32_t)(v >> sh) & M28;
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) A[k] = idle ? 0u : a.r1d[p * K + k];  // z = R mod m
    more = fetch();
  }
  while (more) {
    wave_lds_fence();
    montmul<P, K, false>(A, bl, Nd, a.n0inv, m_src_addr, p);
    wave_lds_fence();
    more = fetch();
  }
  if (wv == 0u)
    store_result<P, K>(A, Nd, bl, p, g_raw, idle, active, a.out + (size_t)op * a.out_words, a.out_words);
}

template <int P, int K, int G, int WPE>
__global__ __launch_bounds__(64 * MPCX_FB_MAX_SPLIT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_fixedbase(
    const FixedBaseArgs a) {
  fixedbase_wave<P, K, G>(a, blockIdx.x);
}

// Several comb batches in one launch (mpcx_fixedbase_multi_batch: concurrent
// callers' batches -- other tables, other moduli of the class, muls or not):
// segment s owns workgroups [first[s], first[s+1]) and its own FixedBaseArgs,
// read wave-uniformly, as k_modexp_multi does for exponentiations.
template <int P, int K, int G, int WPE>
__global__ __launch_bounds__(64 * MPCX_FB_MAX_SPLIT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_fixedbase_multi(
    const FixedBaseArgs* __restrict__ segs, const uint32_t* __restrict__ first, uint32_t nsegs) {
  const uint32_t b = blockIdx.x;
  uint32_t s = 0;
  while (s + 1u < nsegs && __builtin_amdgcn_readfirstlane(first[s + 1u]) <= b) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  fixedbase_wave<P, K, G>(segs[s], b - __builtin_amdgcn_readfirstlane(first[s]));
}

// ------------------------------------------- per-candidate-modulus helpers
// Thread-per-operand kernels (P = 1, K digits per lane) whose modulus differs
// per lane: safe-prime candidates. Every Montgomery constant is derived on the
// device from the candidate itself.
template <int K>
__device__ __forceinline__ bool ge_digits(const uint32_t (&x)[K], const uint32_t (&y)[K]) {
  // branch-free lexicographic compare from the top digit
  int r = 0;  // 0 = equal so far, 1 = x > y, -1 = x < y
#pragma unroll
  for (int k = K - 1; k >= 0; --k) {
    const int c = (x[k] > y[k]) - (x[k] < y[k]);
    r = r != 0 ? r : c;
  }
  return r >= 0;
}
template <int K>
__device__ __forceinline__ void sub_digits(uint32_t (&x)[K], const uint32_t (&y)[K]) {
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t t = x[k] - y[k] - br;
    br = (t >> 31) & 1u;  // digits < 2^28: a borrow shows as the sign bit
    x[k] = t & M28;
  }
}
template <int K>
__device__ __forceinline__ void norm_serial(uint32_t (&x)[K]) {
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t t = x[k] + c;
    x[k] = t & M28;
    c = t >> DB;
  }
}
template <int K>
__device__ __forceinline__ void canon_serial(uint32_t (&x)[K], const uint32_t (&n)[K]) {
  norm_serial<K>(x);
  for (int it = 0; it < 8 && ge_digits<K>(x, n); ++it) sub_digits<K>(x, n);
}
template <int K>
__device__ __forceinline__ bool eq_digits(const uint32_t (&x)[K], const uint32_t (&y)[K]) {
  bool e = true;
#pragma unroll
  for (int k = 0; k < K; ++k) e &= x[k] == y[k];
  return e;
}
// x = (x + y) mod-lazy: digit sum, normalised (no reduction)
template <int K>
__device__ __forceinline__ void add_digits(uint32_t (&x)[K], const uint32_t (&y)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] += y[k];
  norm_serial<K>(x);
}
// candidate words -> radix-2^28 digits (inactive lanes: the odd dummy 1)
template <int K>
__device__ __forceinline__ void load_candidate(const uint32_t* w, uint32_t words, bool active, uint32_t (&Nd)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t bit = (uint32_t)k * DB, wi = bit >> 5, sh = bit & 31u;
    uint64_t v = 0;
    if (active) v = ((uint64_t)((wi + 1) < words ? w[wi + 1] : 0u) << 32) | (wi < words ? w[wi] : 0u);
    Nd[k] = (uint32_t)(v >> sh) & M28;
  }
  if (!active) Nd[0] = 1;
}
// -n^-1 mod 2^28 (Newton on 32 bits)
__device__ __forceinline__ uint32_t neg_inv28(uint32_t n0) {
  uint32_t inv = n0;
  for (int i = 0; i < 5; ++i) inv *= 2u - n0 * inv;
  return (0u - inv) & M28;
}
template <int K>
__device__ __forceinline__ int bitlen_digits(const uint32_t (&Nd)[K]) {
  int nbits = 1;  // unrolled: no dynamic register indexing
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (Nd[k] != 0u) nbits = k * DB + (32 - __builtin_clz(Nd[k]));
  return nbits;
}
// R mod n (canonical), R = 2^(28K): 2^nbits - n (< n), then doublings mod n
template <int K>
__device__ __forceinline__ void r_mod(const uint32_t (&Nd)[K], int nbits, uint32_t (&A)[K]) {
  uint32_t c = 1;  // two's complement of n within nbits bits
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int lo = k * DB;
    uint32_t maskk = 0;
    if (nbits >= lo + DB) maskk = M28;
    else if (nbits > lo) maskk = (1u << (nbits - lo)) - 1u;
    const uint32_t t = ((~Nd[k]) & maskk) + c;
    c = t >> DB;
    A[k] = t & maskk;
  }
  for (int i = nbits; i < DB * K; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) A[k] <<= 1;
    norm_serial<K>(A);
    if (ge_digits<K>(A, Nd)) sub_digits<K>(A, Nd);
  }
}
// bit j of the candidate (from its words in memory: no dynamic register index)
__device__ __forceinline__ uint32_t word_bit(const uint32_t* w, int j) { return (w[j >> 5] >> (j & 31)) & 1u; }

// -------------------------------------------- base-2 tests (k_prime2)
// Fermat items: ok = 2^(n-1) == 1 (mod n) -- tss-lib's Pocklington check on
// p = 2q+1 (up:common/safe_prime.go isPocklingtonCriterionSatisfied).
// Strong items: n - 1 = 2^s d, x = 2^d; ok iff x == 1, or x^(2^j) == n-1
// for some j < s -- the base-2 Miller-Rabin round of q.ProbablyPrime
// (go:src/math/big/prime.go, its forced last base), run first so the other
// rounds only see its survivors. One wave-uniform mode per block.
// Square-and-double: squarings are Montgomery squarings and the "multiply by
// 2" a digit doubling without reduction (values < 4n, and R > 16n keeps every
// almost-Montgomery output below 2n).
template <int K, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_prime2(const Prime2Args a) {
  constexpr int L = K;
  __shared__ uint32_t lds[65 * L + 2];
  const int lane = threadIdx.x;
  const bool strong = blockIdx.x >= a.f_blocks;
  uint32_t op, cnt;
  const uint32_t* src;
  if (!strong) {
    cnt = a.count_dev ? min(a.count_f, *a.count_dev) : a.count_f;
    if (blockIdx.x * 64u >= cnt) return;  // whole wave beyond the sieve's survivors
    op = blockIdx.x * 64u + lane;
    src = a.nf;
  } else {
    cnt = a.count_s;
    if ((blockIdx.x - a.f_blocks) * 64u >= cnt) return;
    op = (blockIdx.x - a.f_blocks) * 64u + lane;
    src = a.ns;
  }
  const bool active = op < cnt;
  uint32_t* bl = lds + lane * L;
  const uint32_t* nw = src + (size_t)(active ? op : 0) * a.n_words;
  uint32_t Nd[K], A[K], R1[K];
  load_candidate<K>(nw, a.n_words, active, Nd);
  const uint32_t n0inv = neg_inv28(Nd[0]);
  const int nbits = bitlen_digits<K>(Nd);
  r_mod<K>(Nd, nbits, R1);
  int s = 0;  // Fermat: e = n - 1; strong: e = (n - 1) >> s, s = v2(n - 1)
  if (strong && active) {
    s = 1;
    while (s < nbits && !word_bit(nw, s)) ++s;
  }
  // the top bit of e is the top bit of n: start from Montgomery 2
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = R1[k] << 1;
  norm_serial<K>(A);
  const int m_src_addr = lane * 4;
  for (int i = nbits - s - 2; i >= 0; --i) {
    lds_store_digits<K>(bl, 0, A);
    wave_lds_fence();
    montmul<1, K, true>(A, bl, Nd, n0inv, m_src_addr, 0);
    wave_lds_fence();
    const int j = i + s;  // bit j of n - 1: bit j of n, except bit 0 (n odd)
    if (j > 0 && active && word_bit(nw, j)) {
#pragma unroll
      for (int k = 0; k < K; ++k) A[k] <<= 1;
      norm_serial<K>(A);
    }
  }
  canon_serial<K>(A, Nd);
  bool pass = eq_digits<K>(A, R1);  // 2^e == 1
  if (strong) {
    uint32_t NR1[K];  // Montgomery form of n - 1
#pragma unroll
    for (int k = 0; k < K; ++k) NR1[k] = Nd[k];
    sub_digits<K>(NR1, R1);
    pass = pass || eq_digits<K>(A, NR1);
    for (int j = 1; j < s && !pass; ++j) {
      lds_store_digits<K>(bl, 0, A);
      wave_lds_fence();
      montmul<1, K, true>(A, bl, Nd, n0inv, m_src_addr, 0);
      wave_lds_fence();
      canon_serial<K>(A, Nd);
      if (eq_digits<K>(A, R1)) break;  // nontrivial square root of 1: composite
      pass = eq_digits<K>(A, NR1);
    }
  }
  if (!active) return;
  if (strong) {
    a.ok_s[op] = pass ? 1 : 0;
    return;
  }
  if (a.ok_f) a.ok_f[op] = pass ? 1 : 0;
  if (pass && a.pass_count) {
    const uint32_t slot = atomicAdd(a.pass_count, 1u);
    a.pass_idx[slot] = a.sieve_idx ? a.sieve_idx[op] : op;
    for (uint32_t w = 0; w < a.n_words; ++w) a.pass_n[(size_t)slot * a.n_words + w] = nw[w];
  }
}

// -------------------------------------------- strong Lucas test (k_lucas)
// Go math/big probablyPrimeLucas (go:src/math/big/prime.go), the last step of
// ProbablyPrime: with P from Baillie-OEIS method C (the smallest P >= 3 with
// Jacobi(P^2 - 4, n) = -1, found by the caller; Q = 1), n + 1 = 2^r s (s odd):
// n passes iff V_s == +-2 and U_s == 0 (checked as P V_s == 2 V_{s+1},
// Crandall-Pomerance 3.13), or V_{2^t s} == 0 for some 0 <= t < r - 1.
// V is built by the binary ladder V_2k = V_k^2 - 2, V_2k+1 = V_k V_k+1 - P in
// the Montgomery domain: each step is one product and one squaring for every
// lane (the bit only selects where the two results go, so the wave never
// diverges); the subtractions are additions of 2n - c (values stay < 4n).
template <int K, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_lucas(const LucasArgs a) {
  constexpr int L = K;
  __shared__ uint32_t lds[65 * L + 2];
  const int lane = threadIdx.x;
  const uint32_t op = blockIdx.x * 64u + lane;
  if (blockIdx.x * 64u >= a.count) return;
  const bool active = op < a.count;
  uint32_t* bl = lds + lane * L;
  const int m_src_addr = lane * 4;
  const uint32_t* nw = a.n + (size_t)(active ? op : 0) * a.n_words;
  uint32_t Nd[K], R1[K];
  load_candidate<K>(nw, a.n_words, active, Nd);
  const uint32_t n0inv = neg_inv28(Nd[0]);
  const int nbits = bitlen_digits<K>(Nd);
  r_mod<K>(Nd, nbits, R1);
  const uint32_t P = active ? a.P[op] : 3u;
  // PR = P R mod n (Horner over P's bits), TwoR = 2 R mod n
  uint32_t PR[K], TwoR[K], N2[K], CP[K], C2[K];
#pragma unroll
  for (int k = 0; k < K; ++k) PR[k] = 0;
  for (int b = 13; b >= 0; --b) {
#pragma unroll
    for (int k = 0; k < K; ++k) PR[k] <<= 1;
    norm_serial<K>(PR);
    if (ge_digits<K>(PR, Nd)) sub_digits<K>(PR, Nd);
    if ((P >> b) & 1u) {
      add_digits<K>(PR, R1);
      if (ge_digits<K>(PR, Nd)) sub_digits<K>(PR, Nd);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    TwoR[k] = R1[k] << 1;
    N2[k] = Nd[k] << 1;
  }
  norm_serial<K>(TwoR);
  if (ge_digits<K>(TwoR, Nd)) sub_digits<K>(TwoR, Nd);
  norm_serial<K>(N2);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    CP[k] = N2[k];
    C2[k] = N2[k];
  }
  sub_digits<K>(CP, PR);    // 2n - P R: adding it subtracts P
  sub_digits<K>(C2, TwoR);  // 2n - 2 R
  // n + 1 = 2^r s: r = trailing ones of n; bit j of n + 1 is 0 below r, 1 at
  // r, and bit j of n above
  int r = 0;
  if (active)
    while (r < nbits && word_bit(nw, r)) ++r;
  const int sbits = (r == nbits) ? 1 : nbits - r;
  uint32_t vk[K], vk1[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    vk[k] = TwoR[k];  // V_0 = 2
    vk1[k] = PR[k];   // V_1 = P
  }
  for (int i = sbits - 1; i >= 0; --i) {
    const int j = i + r;
    const bool bit = (j == r) || (active && word_bit(nw, j));
    // X = V_k V_k+1 - P; Y = (bit ? V_k+1 : V_k)^2 - 2
    uint32_t X[K], Y[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      X[k] = vk[k];
      Y[k] = bit ? vk1[k] : vk[k];
    }
    lds_store_digits<K>(bl, 0, vk1);
    wave_lds_fence();
    montmul<1, K, false>(X, bl, Nd, n0inv, m_src_addr, 0);
    wave_lds_fence();
    add_digits<K>(X, CP);
    lds_store_digits<K>(bl, 0, Y);
    wave_lds_fence();
    montmul<1, K, true>(Y, bl, Nd, n0inv, m_src_addr, 0);
    wave_lds_fence();
    add_digits<K>(Y, C2);
    // bit: k' = 2k+1 -> (V_2k+1, V_2k+2) = (X, Y); else k' = 2k -> (V_2k, V_2k+1) = (Y, X)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      vk[k] = bit ? X[k] : Y[k];
      vk1[k] = bit ? Y[k] : X[k];
    }
  }
  uint32_t NTwoR[K];  // Montgomery form of n - 2
#pragma unroll
  for (int k = 0; k < K; ++k) NTwoR[k] = Nd[k];
  sub_digits<K>(NTwoR, TwoR);
  canon_serial<K>(vk, Nd);
  bool pass = false;
  if (eq_digits<K>(vk, TwoR) || eq_digits<K>(vk, NTwoR)) {
    // U_s == 0  <=>  P V_s == 2 V_s+1 (mod n)
    uint32_t U1[K], U2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      U1[k] = vk[k];
      U2[k] = vk1[k];
    }
    lds_store_digits<K>(bl, 0, PR);
    wave_lds_fence();
    montmul<1, K, false>(U1, bl, Nd, n0inv, m_src_addr, 0);  // P V_s R
    wave_lds_fence();
    canon_serial<K>(U1, Nd);
    add_digits<K>(U2, vk1);  // 2 V_s+1 R (< 8n)
    canon_serial<K>(U2, Nd);
    pass = eq_digits<K>(U1, U2);
  }
  for (int t = 0; t < r - 1 && !pass; ++t) {
    bool zero = true;
#pragma unroll
    for (int k = 0; k < K; ++k) zero &= vk[k] == 0u;
    if (zero) {
      pass = true;
      break;
    }
    if (eq_digits<K>(vk, TwoR)) break;  // V = 2 is a fixed point of V^2 - 2: never 0
    lds_store_digits<K>(bl, 0, vk);
    wave_lds_fence();
    montmul<1, K, true>(vk, bl, Nd, n0inv, m_src_addr, 0);
    wave_lds_fence();
    add_digits<K>(vk, C2);
    canon_serial<K>(vk, Nd);
  }
  if (active) a.ok[op] = pass ? 1 : 0;
}

// ---------------------------------------------------------- Miller-Rabin
// ok[i] = n_i is a strong probable prime to base a_i (one candidate per lane,
// per-lane modulus): n - 1 = 2^s d, x = a^d; pass iff x == 1 or x^(2^j) == n-1
// for some j < s. Serves q.ProbablyPrime(20) in the safe-prime search
// (up:common/safe_prime.go). All Montgomery constants are derived on the
// device: R mod n by doubling, R^2 mod n = Mont(2^(28K)) by square-and-double.
template <int K, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_mr(const MrArgs a) {
  constexpr int L = K;
  __shared__ uint32_t lds[2 * 65 * L + 2];
  const int lane = threadIdx.x;
  const uint32_t op = blockIdx.x * 64u + lane;
  const bool active = op < a.count;
  uint32_t* bt = lds + lane * L;             // row for the running value (squarings)
  uint32_t* bm = lds + (65 + lane) * L;      // row for a*R (multiplies)
  const int m_src_addr = lane * 4;
  const uint32_t* nw = a.n + (size_t)(active ? op : 0) * a.n_words;
  const uint32_t* aw = a.a + (size_t)(active ? op : 0) * a.n_words;
  uint32_t Nd[K], A[K], X[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t bit = (uint32_t)k * DB, w = bit >> 5, sh = bit & 31u;
    uint64_t v = 0, u = 0;
    if (active) {
      v = ((uint64_t)((w + 1) < a.n_words ? nw[w + 1] : 0u) << 32) | (w < a.n_words ? nw[w] : 0u);
      u = ((uint64_t)((w + 1) < a.n_words ? aw[w + 1] : 0u) << 32) | (w < a.n_words ? aw[w] : 0u);
    }
    Nd[k] = (uint32_t)(v >> sh) & M28;
    X[k] = (uint32_t)(u >> sh) & M28;
  }
  if (!active) Nd[0] = 1;
  uint32_t inv = Nd[0];
  for (int i = 0; i < 5; ++i) inv *= 2u - Nd[0] * inv;
  const uint32_t n0inv = (0u - inv) & M28;
  int nbits = 1;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (Nd[k] != 0u) nbits = k * DB + (32 - __builtin_clz(Nd[k]));
  // R mod n
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = 0;
  {
    uint32_t c = 1;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int lo = k * DB;
      uint32_t maskk = 0;
      if (nbits >= lo + DB) maskk = M28;
      else if (nbits > lo) maskk = (1u << (nbits - lo)) - 1u;
      const uint32_t t = ((~Nd[k]) & maskk) + c;
      c = t >> DB;
      A[k] = t & maskk;
    }
  }
  for (int i = nbits; i < DB * K; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) A[k] <<= 1;
    norm_serial<K>(A);
    if (ge_digits<K>(A, Nd)) sub_digits<K>(A, Nd);
  }
  uint32_t R1[K];  // R mod n, canonical: Montgomery form of 1
#pragma unroll
  for (int k = 0; k < K; ++k) R1[k] = A[k];
  // R^2 mod n = Mont(2^(28K)): square-and-double over the bits of E = 28K
  constexpr int E = DB * K;
  constexpr int ETOP = 31 - __builtin_clz((unsigned)E);
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] <<= 1;  // Mont(2) (top bit of E)
  norm_serial<K>(A);
  for (int i = ETOP - 1; i >= 0; --i) {
    lds_store_digits<K>(bt, 0, A);
    wave_lds_fence();
    montmul<1, K, true>(A, bt, Nd, n0inv, m_src_addr, 0);
    wave_lds_fence();
    if ((E >> i) & 1) {
#pragma unroll
      for (int k = 0; k < K; ++k) A[k] <<= 1;
    }
    norm_serial<K>(A);
  }
  // a*R = mont(a, R^2)
  lds_store_digits<K>(bt, 0, A);
  wave_lds_fence();
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = X[k];
  montmul<1, K, false>(A, bt, Nd, n0inv, m_src_addr, 0);
  wave_lds_fence();
  lds_store_digits<K>(bm, 0, A);
  // n - 1 = 2^s d (n odd, n >= 5): s = number of trailing zero bits of n-1
  int s = 1;
  while (s < nbits && !((nw[s >> 5] >> (s & 31)) & 1u)) ++s;
  if (!active) s = 1;
  const int dbits = nbits - s;  // bit length of d
  // x = a^d, left to right binary (d's top bit is set)
  for (int i = dbits - 2; i >= 0; --i) {
    wave_lds_fence();
    lds_store_digits<K>(bt, 0, A);
    wave_lds_fence();
    montmul<1, K, true>(A, bt, Nd, n0inv, m_src_addr, 0);
    const uint32_t bit = active ? (nw[(i + s) >> 5] >> ((i + s) & 31)) & 1u : 0u;
    if (bit) {
      wave_lds_fence();
      montmul<1, K, false>(A, bm, Nd, n0inv, m_src_addr, 0);
    }
  }
  // compare in the Montgomery domain: 1 -> R1, n-1 -> n - R1
  uint32_t NR1[K];
#pragma unroll
  for (int k = 0; k < K; ++k) NR1[k] = Nd[k];
  {
    uint32_t br = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t t = NR1[k] - R1[k] - br;
      br = (t >> 31) & 1u;
      NR1[k] = t & M28;
    }
  }
  auto eq = [&](const uint32_t (&x)[K], const uint32_t (&y)[K]) __attribute__((always_inline)) {
    bool e = true;
#pragma unroll
    for (int k = 0; k < K; ++k) e &= x[k] == y[k];
    return e;
  };
  canon_serial<K>(A, Nd);
  bool pass = eq(A, R1) || eq(A, NR1);
  for (int j = 1; j < s && !pass; ++j) {
    wave_lds_fence();
    lds_store_digits<K>(bt, 0, A);
    wave_lds_fence();
    montmul<1, K, true>(A, bt, Nd, n0inv, m_src_addr, 0);
    canon_serial<K>(A, Nd);
    if (eq(A, R1)) break;  // nontrivial square root of 1: composite
    pass = eq(A, NR1);
  }
  if (active) a.ok[op] = pass ? 1 : 0;
}

// ------------------------------------ cooperative per-candidate kernels
// The thread-per-candidate kernels above hold K = 37 digits per lane and run
// one wavefront per SIMD, where a lone wave issues v_mad_u64_u32 at ~45% of
// the SIMD peak (profiles/r01): a Fermat launch is capped there, and a small
// Miller-Rabin or Lucas batch is one thread's full serial latency. The
// kernels below give each candidate P lanes (K digits each, the k_modexp
// montmul with a per-group modulus and -n^-1): P = 2 x K = 19 for the base-2
// throughput tests (32 candidates and 3 waves per SIMD), P = 16 x K = 3 for
// general-base Miller-Rabin (4 tests per wave, 1/8 of the serial chain).
// Per-item constants come from a thread-per-item prep kernel.

// R mod n (canonical, L digits), -n^-1 mod 2^28 and nbits | s << 16
// (s = v2(n - 1)) of one odd n >= 5 for R = 2^(28 L): 28 L - nbits doublings,
// a few % of the exponentiation that follows.
template <int L>
__device__ __forceinline__ void pprep_item(const uint32_t* nw, uint32_t n_words, uint32_t* r1_out, uint32_t* meta_out) {
  uint32_t Nd[L], R1[L];
  load_candidate<L>(nw, n_words, true, Nd);
  const int nbits = bitlen_digits<L>(Nd);
  r_mod<L>(Nd, nbits, R1);
  int s = 1;
  while (s < nbits && !word_bit(nw, s)) ++s;
#pragma unroll
  for (int d = 0; d < L; ++d) r1_out[d] = R1[d];
  meta_out[0] = neg_inv28(Nd[0]);
  meta_out[1] = (uint32_t)nbits | ((uint32_t)s << 16);
}

template <int L>
__global__ __launch_bounds__(64) void k_pprep_prime2(const Prime2Args a) {
  const bool strong = blockIdx.x >= a.fp_blocks;
  uint32_t cnt, i;
  const uint32_t* src;
  size_t base;
  if (!strong) {
    cnt = a.count_dev ? min(a.count_f, *a.count_dev) : a.count_f;
    i = blockIdx.x * 64u + threadIdx.x;
    src = a.nf;
    base = 0;
  } else {
    cnt = a.count_s;
    i = (blockIdx.x - a.fp_blocks) * 64u + threadIdx.x;
    src = a.ns;
    base = a.count_f;
  }
  if (i >= cnt) return;
  pprep_item<L>(src + (size_t)i * a.n_words, a.n_words, a.r1 + (base + i) * L, a.meta + (base + i) * 2);
}

template <int L>
__global__ __launch_bounds__(64) void k_pprep_mr(const MrArgs a) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= a.count) return;
  pprep_item<L>(a.n + (size_t)i * a.n_words, a.n_words, a.r1 + (size_t)i * L, a.meta + (size_t)i * 2);
}

// digits p*K .. p*K+K-1 of a little-endian word array (radix 2^28)
template <int K>
__device__ __forceinline__ void load_group_digits(const uint32_t* w, uint32_t words, int p, uint32_t (&D)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t bit = (uint32_t)(p * K + k) * DB, wi = bit >> 5, sh = bit & 31u;
    const uint64_t v = ((uint64_t)((wi + 1) < words ? w[wi + 1] : 0u) << 32) | (wi < words ? w[wi] : 0u);
    D[k] = (uint32_t)(v >> sh) & M28;
  }
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
  return v;
}

// all P lanes of this lane's group have v set
template <int P>
__device__ __forceinline__ bool group_all(bool v, int g) {
  const uint64_t bal = __ballot(v);
  const uint64_t gmask = (P == 64 ? ~0ull : (((1ull << P) - 1ull) << (g * P)));
  return (bal & gmask) == gmask;
}

// Leave the Montgomery domain on a copy and compare with 1 and n - 1:
// Y = mont(X, 1) <= n, canonical digits (uses the group's LDS row bl).
template <int P, int K>
__device__ __forceinline__ void exit_compare(const uint32_t (&X)[K], const uint32_t (&Nd)[K], uint32_t n0inv,
                                             uint32_t* bl, int p, int g, bool* is_one, bool* is_nm1) {
  uint32_t Y[K], one[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Y[k] = X[k];
    one[k] = (p == 0 && k == 0) ? 1u : 0u;
  }
  wave_lds_fence();
  lds_store_digits<K>(bl, p, one);
  wave_lds_fence();
  montmul<P, K, false>(Y, bl, Nd, n0inv, 0, p);
  wave_lds_fence();
  canonicalize<P, K>(Y);
  bool e1 = true, em = true;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const bool d0 = p == 0 && k == 0;
    e1 &= Y[k] == (d0 ? 1u : 0u);
    em &= Y[k] == (d0 ? Nd[0] - 1u : Nd[k]);  // n odd: n - 1 only changes digit 0
  }
  *is_one = group_all<P>(e1, g);
  *is_nm1 = group_all<P>(em, g);
}

// x <- 2x (digits doubled, one carry pass; values stay < R / 4)
template <int P, int K>
__device__ __forceinline__ void double_digits(uint32_t (&A)[K], bool on) {
  const uint32_t sh = on ? 1u : 0u;
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] <<= sh;
  carry_pass32<P, K>(A);
}

// Base-2 tests of k_prime2, P lanes per candidate: Fermat items
// (2^(n-1) == 1) in blocks [0, f_blocks), strong items (n - 1 = 2^s d:
// 2^d == 1, or 2^(2^j d) == n - 1 for some j < s) after them. Square and
// double as in k_prime2 (values < 4n, R > 16n); the exponent bits differ per
// candidate, so the doubling is a per-lane shift by 0 or 1.
template <int P, int K, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_prime2c(const Prime2Args a) {
  constexpr int L = P * K, G = 64 / P;
  __shared__ uint32_t lds[2 * G * L + 2];  // per group: work row, saved-x row
  const int lane = threadIdx.x, g = lane / P, p = lane - g * P;
  const bool strong = blockIdx.x >= a.f_blocks;
  uint32_t cnt, item;
  const uint32_t* src;
  size_t base;
  if (!strong) {
    cnt = a.count_dev ? min(a.count_f, *a.count_dev) : a.count_f;
    if (blockIdx.x * (uint32_t)G >= cnt) return;  // whole wave beyond the sieve's survivors
    item = blockIdx.x * G + g;
    src = a.nf;
    base = 0;
  } else {
    cnt = a.count_s;
    if ((blockIdx.x - a.f_blocks) * (uint32_t)G >= cnt) return;
    item = (blockIdx.x - a.f_blocks) * G + g;
    src = a.ns;
    base = a.count_f;
  }
  const bool active = item < cnt;
  const uint32_t it = active ? item : item - g;  // idle groups recompute the block's first item
  uint32_t* bl = lds + 2 * g * L;
  uint32_t* sv = bl + L;
  const uint32_t* nw = src + (size_t)it * a.n_words;
  uint32_t Nd[K], A[K];
  load_group_digits<K>(nw, a.n_words, p, Nd);
  {
    const uint32_t* r1 = a.r1 + (base + it) * L + p * K;
#pragma unroll
    for (int k = 0; k < K; ++k) A[k] = r1[k];  // Montgomery 1
  }
  const uint32_t n0inv = a.meta[(base + it) * 2];
  const uint32_t mt = a.meta[(base + it) * 2 + 1];
  const int nbits = (int)(mt & 0xFFFFu), s = (int)(mt >> 16);
  const int sh = strong ? s : 0;  // strong: e = (n - 1) >> s; Fermat: e = n - 1
  // Left to right from the wave's highest exponent bit, starting at
  // Montgomery 1: above a candidate's own top bit its exponent bits are 0 and
  // squaring 1 changes nothing, so no lane needs a predicated select.
  // Two montmul call sites (squaring, exit product) as in k_modexp: states
  //   SQ : x <- x^2, then x <- 2x on an exponent bit
  //   EX : y = mont(x, 1) <= n (x saved in the group's second row), compare
  //        y with 1 and n - 1, restore x
  //   SS : strong-test squaring x <- x^2, then EX again
  enum { SQ, EX, SS };
  int st = SQ;
  int i = wave_max(nbits - sh - 1), j = 0;
  const int smax = strong ? wave_max(s) : 1;
  bool pass = false, done = false;
  for (;;) {
    wave_lds_fence();
    if (st == EX) {
      uint32_t one[K];
#pragma unroll
      for (int k = 0; k < K; ++k) one[k] = (p == 0 && k == 0) ? 1u : 0u;
      lds_store_digits<K>(sv, p, A);
      lds_store_digits<K>(bl, p, one);
    } else if (MPCX_PRIME2C_DBL_FOLD && st == SQ) {
      // x <- 2^bit x^2 as ONE squaring product: B = 2^bit x in LDS, x in
      // registers -- the half-product schedule then sums x_i (2 x_j) pairs
      // (digits of B < 2^29 + 2^11, b2 < 2^31: the schedule's bounds hold, and
      // x (2x) < 8n^2 < nR keeps the result < 2n); no separate doubling pass
      const int jb = i + sh;  // bit jb of n - 1: bit jb of n except bit 0 (n odd)
      const uint32_t dsh = (jb > 0 && jb < nbits && word_bit(nw, jb)) ? 1u : 0u;
      uint32_t B2[K];
#pragma unroll
      for (int k = 0; k < K; ++k) B2[k] = A[k] << (dsh + (MPCX_SQR_B2 ? 1u : 0u));  // montmul reads 2B
      lds_store_digits<K>(bl, p, B2);
    } else {
      lds_store_sqr<K>(bl, p, A);  // SS (or SQ without the fold): a plain squaring
    }
    wave_lds_fence();
    if (st == EX) {
      montmul<P, K, false>(A, bl, Nd, n0inv, 0, p);
    } else {
      montmul<P, K, true, (bool)MPCX_SQR_B2>(A, bl, Nd, n0inv, 0, p);
    }
    if (st == SQ) {
      if (!MPCX_PRIME2C_DBL_FOLD) {
        const int jb = i + sh;  // bit jb of n - 1: bit jb of n except bit 0 (n odd)
        double_digits<P, K>(A, jb > 0 && jb < nbits && word_bit(nw, jb));
      }
      if (--i < 0) st = EX;
    } else if (st == SS) {
      st = EX;
    } else {
      canonicalize<P, K>(A);
      bool e1 = true, em = true;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const bool d0 = p == 0 && k == 0;
        e1 &= A[k] == (d0 ? 1u : 0u);
        em &= A[k] == (d0 ? Nd[0] - 1u : Nd[k]);  // n odd: n - 1 only changes digit 0
      }
      const bool one = group_all<P>(e1, g), nm1 = group_all<P>(em, g);
      if (j == 0) {
        pass = one || (strong && nm1);
        done = pass;
      } else if (!done && j < s) {
        if (one) {
          done = true;  // nontrivial square root of 1: composite
        } else if (nm1) {
          pass = true;
          done = true;
        }
      }
      if (++j >= smax) break;
      wave_lds_fence();
#pragma unroll
      for (int k = 0; k < K; ++k) A[k] = sv[p * K + k];
      st = SS;
    }
  }
  if (!active || p != 0) return;
  if (strong) {
    a.ok_s[item] = pass ? 1 : 0;
    return;
  }
  if (a.ok_f) a.ok_f[item] = pass ? 1 : 0;
  if (pass && a.pass_count) {
    const uint32_t slot = atomicAdd(a.pass_count, 1u);
    a.pass_idx[slot] = a.sieve_idx ? a.sieve_idx[item] : item;
    for (uint32_t w = 0; w < a.n_words; ++w) a.pass_n[(size_t)slot * a.n_words + w] = nw[w];
  }
}

// Miller-Rabin to arbitrary bases, P lanes per test: R^2 mod n by
// square-and-double from Mont(2), a R = mont(a, R^2), a 16-entry table
// T[v] = a^v R in the group's LDS rows, then x = a^d by Go's 4-bit fixed
// window (4 squarings and one table product per window for every lane: the
// wave never diverges) and the strong check. ok[i] as k_mr.
template <int P, int K, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_mrc(const MrArgs a) {
  constexpr int L = P * K, G = 64 / P, ROWS = 17;  // table rows 0..15, work row 16
  __shared__ uint32_t lds[G * ROWS * L + 2];
  const int lane = threadIdx.x, g = lane / P, p = lane - g * P;
  if (blockIdx.x * (uint32_t)G >= a.count) return;
  const uint32_t item = blockIdx.x * G + g;
  const bool active = item < a.count;
  const uint32_t it = active ? item : item - g;
  uint32_t* rows = lds + g * ROWS * L;
  uint32_t* wl = rows + 16 * L;
  const uint32_t* nw = a.n + (size_t)it * a.n_words;
  uint32_t Nd[K], R1[K], A[K], X[K];
  load_group_digits<K>(nw, a.n_words, p, Nd);
  load_group_digits<K>(a.a + (size_t)it * a.n_words, a.n_words, p, X);
  const uint32_t* r1 = a.r1 + (size_t)it * L + p * K;
#pragma unroll
  for (int k = 0; k < K; ++k) R1[k] = r1[k];
  const uint32_t n0inv = a.meta[(size_t)it * 2];
  const uint32_t mt = a.meta[(size_t)it * 2 + 1];
  const int nbits = (int)(mt & 0xFFFFu), s = (int)(mt >> 16);
  auto sqr = [&] __attribute__((always_inline))() {
    wave_lds_fence();
    lds_store_digits<K>(wl, p, A);
    wave_lds_fence();
    montmul<P, K, true>(A, wl, Nd, n0inv, 0, p);
  };
  // R^2 mod n = Mont(2^(28 L)): square-and-double over E = 28 L from Mont(2)
  constexpr int E = DB * L;
  constexpr int ETOP = 31 - __builtin_clz((unsigned)E);
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = R1[k];
  double_digits<P, K>(A, true);
  for (int i = ETOP - 1; i >= 0; --i) {
    sqr();
    double_digits<P, K>(A, ((E >> i) & 1) != 0);
  }
  // T[1] = a R = mont(a, R^2); T[0] = R mod n; T[v] = mont(T[v-1], T[1])
  wave_lds_fence();
  lds_store_digits<K>(wl, p, A);
  wave_lds_fence();
  montmul<P, K, false>(X, wl, Nd, n0inv, 0, p);
  wave_lds_fence();
  lds_store_digits<K>(rows, p, R1);
  lds_store_digits<K>(rows + L, p, X);
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = X[k];
  for (int v = 2; v < 16; ++v) {
    wave_lds_fence();
    montmul<P, K, false>(A, rows + L, Nd, n0inv, 0, p);
    wave_lds_fence();
    lds_store_digits<K>(rows + v * L, p, A);
  }
  // x = a^d, d = (n - 1) >> s = bits [s, nbits) of n, 4-bit windows from the top
  const int dbits = nbits - s;
  const int nwin = (dbits + 3) / 4;
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = R1[k];  // Montgomery one: leading zero windows keep it
  for (int w = wave_max(nwin) - 1; w >= 0; --w) {
#pragma unroll 1
    for (int q = 0; q < 4; ++q) sqr();
    uint32_t v = 0;
#pragma unroll
    for (int b = 3; b >= 0; --b) {
      const int j = s + 4 * w + b;
      v = (v << 1) | ((j < nbits) ? word_bit(nw, j) : 0u);
    }
    wave_lds_fence();
    montmul<P, K, false>(A, rows + v * L, Nd, n0inv, 0, p);
  }
  bool one, nm1;
  exit_compare<P, K>(A, Nd, n0inv, wl, p, g, &one, &nm1);
  bool pass = one || nm1, done = pass;
  const int smax = wave_max(s);
  for (int j = 1; j < smax; ++j) {
    sqr();
    exit_compare<P, K>(A, Nd, n0inv, wl, p, g, &one, &nm1);
    const bool live = !done && j < s;
    if (live && one) done = true;  // nontrivial square root of 1: composite
    else if (live && nm1) {
      pass = true;
      done = true;
    }
  }
  if (active && p == 0) a.ok[item] = pass ? 1 : 0;
}

// Strong Lucas test (k_lucas's ladder and checks), P lanes per candidate.
// Per-item Montgomery constants from a thread-per-item prep (the serial
// Horner / doubling steps), then the V ladder: every bit is one product and
// one squaring for every lane; bits above a candidate's own top keep
// (V_0, V_1) = (2, P) fixed (2^2 - 2 = 2, 2P - P = P), so the wave needs no
// predication. The checks compare canonical values after leaving the
// Montgomery domain.
template <int L>
__global__ __launch_bounds__(64) void k_pprep_lucas(const LucasArgs a) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= a.count) return;
  const uint32_t* nw = a.n + (size_t)i * a.n_words;
  uint32_t Nd[L], R1[L], PR[L], T[L];
  load_candidate<L>(nw, a.n_words, true, Nd);
  const int nbits = bitlen_digits<L>(Nd);
  r_mod<L>(Nd, nbits, R1);
  const uint32_t P = a.P[i];
#pragma unroll
  for (int k = 0; k < L; ++k) PR[k] = 0;
  for (int b = 13; b >= 0; --b) {  // P R mod n, Horner over P's bits
#pragma unroll
    for (int k = 0; k < L; ++k) PR[k] <<= 1;
    norm_serial<L>(PR);
    if (ge_digits<L>(PR, Nd)) sub_digits<L>(PR, Nd);
    if ((P >> b) & 1u) {
      add_digits<L>(PR, R1);
      if (ge_digits<L>(PR, Nd)) sub_digits<L>(PR, Nd);
    }
  }
  uint32_t* c = a.consts + (size_t)i * 4 * L;
  // [0] P R, [1] 2 R, [2] 2n - P R, [3] 2n - 2 R (all canonical, < 2n)
#pragma unroll
  for (int k = 0; k < L; ++k) c[k] = PR[k];
#pragma unroll
  for (int k = 0; k < L; ++k) T[k] = R1[k] << 1;
  norm_serial<L>(T);
  if (ge_digits<L>(T, Nd)) sub_digits<L>(T, Nd);
#pragma unroll
  for (int k = 0; k < L; ++k) c[L + k] = T[k];
  uint32_t N2[L];
#pragma unroll
  for (int k = 0; k < L; ++k) N2[k] = Nd[k] << 1;
  norm_serial<L>(N2);
  {
    uint32_t X[L];
#pragma unroll
    for (int k = 0; k < L; ++k) X[k] = N2[k];
    sub_digits<L>(X, PR);
#pragma unroll
    for (int k = 0; k < L; ++k) c[2 * L + k] = X[k];
#pragma unroll
    for (int k = 0; k < L; ++k) X[k] = N2[k];
    sub_digits<L>(X, T);
#pragma unroll
    for (int k = 0; k < L; ++k) c[3 * L + k] = X[k];
  }
  int r = 0;  // n + 1 = 2^r s: r = trailing ones of n
  while (r < nbits && word_bit(nw, r)) ++r;
  a.meta[(size_t)i * 2] = neg_inv28(Nd[0]);
  a.meta[(size_t)i * 2 + 1] = (uint32_t)nbits | ((uint32_t)r << 16);
}

// canonical value of Montgomery-form X in [0, n): y = mont(X, 1) <= n, with
// n mapped to 0
template <int P, int K>
__device__ __forceinline__ void exit_canonical(const uint32_t (&X)[K], const uint32_t (&Nd)[K], uint32_t n0inv,
                                               uint32_t* bl, int p, int g, uint32_t (&Y)[K]) {
  uint32_t one[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Y[k] = X[k];
    one[k] = (p == 0 && k == 0) ? 1u : 0u;
  }
  wave_lds_fence();
  lds_store_digits<K>(bl, p, one);
  wave_lds_fence();
  montmul<P, K, false>(Y, bl, Nd, n0inv, 0, p);
  wave_lds_fence();
  canonicalize<P, K>(Y);
  bool en = true;
#pragma unroll
  for (int k = 0; k < K; ++k) en &= Y[k] == Nd[k];
  if (group_all<P>(en, g)) {
#pragma unroll
    for (int k = 0; k < K; ++k) Y[k] = 0;
  }
}

// canonical Y equals the small constant c
template <int P, int K>
__device__ __forceinline__ bool group_eq_small(const uint32_t (&Y)[K], uint32_t c, int p, int g) {
  bool e = true;
#pragma unroll
  for (int k = 0; k < K; ++k) e &= Y[k] == ((p == 0 && k == 0) ? c : 0u);
  return group_all<P>(e, g);
}

template <int P, int K, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_lucasc(const LucasArgs a) {
  constexpr int L = P * K, G = 64 / P;
  __shared__ uint32_t lds[G * L + 2];
  const int lane = threadIdx.x, g = lane / P, p = lane - g * P;
  if (blockIdx.x * (uint32_t)G >= a.count) return;
  const uint32_t item = blockIdx.x * G + g;
  const bool active = item < a.count;
  const uint32_t it = active ? item : item - g;
  uint32_t* bl = lds + g * L;
  const uint32_t* nw = a.n + (size_t)it * a.n_words;
  uint32_t Nd[K], PR[K], CP[K], C2[K], vk[K], vk1[K];
  load_group_digits<K>(nw, a.n_words, p, Nd);
  {
    const uint32_t* c = a.consts + (size_t)it * 4 * L + p * K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      PR[k] = c[k];
      vk[k] = c[L + k];  // V_0 = 2
      CP[k] = c[2 * L + k];
      C2[k] = c[3 * L + k];
      vk1[k] = PR[k];  // V_1 = P
    }
  }
  const uint32_t n0inv = a.meta[(size_t)it * 2];
  const uint32_t mt = a.meta[(size_t)it * 2 + 1];
  const int nbits = (int)(mt & 0xFFFFu), r = (int)(mt >> 16);
  const int sbits = (r == nbits) ? 1 : nbits - r;  // bit length of s = (n + 1) >> r
  auto add_const = [&](uint32_t (&X)[K], const uint32_t (&C)[K]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < K; ++k) X[k] += C[k];
    carry_pass32<P, K>(X);  // < 4n < R: no carry leaves the group
  };
  for (int i = wave_max(sbits) - 1; i >= 0; --i) {
    const int j = i + r;  // bit i of s = bit j of n + 1: 1 at j == r, n's bit above
    const bool bit = i < sbits && (j == r || (j < nbits && word_bit(nw, j)));
    // X = V_k V_k+1 - P; Y = (bit ? V_k+1 : V_k)^2 - 2
    uint32_t X[K], Y[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      X[k] = vk[k];
      Y[k] = bit ? vk1[k] : vk[k];
    }
    wave_lds_fence();
    lds_store_digits<K>(bl, p, vk1);
    wave_lds_fence();
    montmul<P, K, false>(X, bl, Nd, n0inv, 0, p);
    add_const(X, CP);
    wave_lds_fence();
    lds_store_digits<K>(bl, p, Y);
    wave_lds_fence();
    montmul<P, K, true>(Y, bl, Nd, n0inv, 0, p);
    add_const(Y, C2);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      vk[k] = bit ? X[k] : Y[k];
      vk1[k] = bit ? Y[k] : X[k];
    }
  }
  // V_s == +-2 and U_s == 0 (P V_s == 2 V_s+1), or V_(2^t s) == 0, t < r - 1
  uint32_t Y[K];
  exit_canonical<P, K>(vk, Nd, n0inv, bl, p, g, Y);
  bool pass = false;
  {
    const bool is2 = group_eq_small<P, K>(Y, 2u, p, g);
    uint32_t Z[K];  // Y + 2 == n  <=>  V_s == n - 2
#pragma unroll
    for (int k = 0; k < K; ++k) Z[k] = Y[k] + ((p == 0 && k == 0) ? 2u : 0u);
    carry_pass32<P, K>(Z);
    bool en = true;
#pragma unroll
    for (int k = 0; k < K; ++k) en &= Z[k] == Nd[k];
    const bool isn2 = group_all<P>(en, g);
    uint32_t U1[K], U2[K], A1[K], A2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      U1[k] = vk[k];
      U2[k] = vk1[k] << 1;  // 2 V_s+1 R (< 4n)
    }
    carry_pass32<P, K>(U2);
    wave_lds_fence();
    lds_store_digits<K>(bl, p, PR);
    wave_lds_fence();
    montmul<P, K, false>(U1, bl, Nd, n0inv, 0, p);  // P V_s R
    exit_canonical<P, K>(U1, Nd, n0inv, bl, p, g, A1);
    exit_canonical<P, K>(U2, Nd, n0inv, bl, p, g, A2);
    bool eu = true;
#pragma unroll
    for (int k = 0; k < K; ++k) eu &= A1[k] == A2[k];
    pass = (is2 || isn2) && group_all<P>(eu, g);
  }
  bool done = pass;
  const int tmax = wave_max(r - 1);
  for (int t = 0; t < tmax; ++t) {
    const bool live = !done && t < r - 1;
    exit_canonical<P, K>(vk, Nd, n0inv, bl, p, g, Y);
    if (live && group_eq_small<P, K>(Y, 0u, p, g)) {
      pass = true;
      done = true;
    } else if (live && group_eq_small<P, K>(Y, 2u, p, g)) {
      done = true;  // V = 2 is a fixed point of V^2 - 2: never 0
    }
    wave_lds_fence();
    lds_store_digits<K>(bl, p, vk);
    wave_lds_fence();
    montmul<P, K, true>(vk, bl, Nd, n0inv, 0, p);
    add_const(vk, C2);
  }
  if (active && p == 0) a.ok[item] = pass ? 1 : 0;
}

}  // namespace mpcx

