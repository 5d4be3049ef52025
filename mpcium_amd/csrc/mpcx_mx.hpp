// mpcx_mx.hpp -- gfx950 Montgomery products with the REDUCTION on the matrix
// cores (v_mfma_i32_16x16x64_i8) and the product A*B on the VALU, for the two
// main geometries whose batches share one modulus: geometry 2 (4 x 37 lanes,
// 16 operands per wave, 4096-bit class: Paillier N^2) and geometry 5 (2 x 37,
// 32 operands per wave, 2048-bit class: N, N~).
//
// Every operand of a k_modexp batch shares the modulus m (config 2: 65,536 x
// r^N mod N^2; ModProof's Z_i^N mod N in keygen), so the two reduction products
// of a Montgomery multiplication in separated form,
//     q = (T mod R) * m'' mod R     (m'' = -m^-1 mod R)
//     U = (T + q m) / R,
// are products of a batch of rows with FIXED Toeplitz matrices of m'' and m:
// dense contractions. The VALU keeps what is per operand -- T = A*B, the same
// lazy radix-2^28 row loop as montmul<P, 37> (mpcx_device.hpp) without its
// m_i N half -- and the matrix cores take the reduction (two thirds of a
// CIOS squaring's multiply-accumulates).
//
// Layout (R = 2^(28 L), the same Montgomery domain as the CIOS geometry, so
// tables, constants and the CIOS exit product mix):
//  * VALU ("block") layout: operand g on lanes Pg..Pg+P-1, lane p holds radix-2^28
//    digits 37p..37p+36 -- montmul's layout.
//  * MFMA layout, per 16 operands (a geometry-5 wave runs two halves): operand
//    n = lane & 15, quarter h = lane >> 4. Radix-2^7 digits (4 per radix-2^28
//    digit, one byte each, so the conversion is a bit spread) are the K index; a
//    16x16x64 MFMA takes B = 64 digits of 16 operands (lane (n, h): bytes
//    16h..16h+15 of the K block -- one ds_read_b128 of radix-2^28 digits
//    16kb + 4h .. +3) and A = the Toeplitz block of m'' or m for output positions
//    16o..16o+15 (precomputed per modulus in the same lane map, so the hardware's
//    k order inside a lane never matters), and accumulates column sums
//    C[4h + r][n] = output position 16o + 4h + r of operand n: one lane holds 4
//    consecutive radix-2^7 positions = ONE radix-2^28 digit.
//  * Column sums are exact in i32: <= 4L products of 7-bit digits.
//  * q is normalised to balanced radix-2^28 digits in [-2^27 - 2^17, 2^27 + 2^17]
//    (one carry step, the neighbour digit's carry by ds_bpermute), whose top
//    radix-2^7 digit is in [-65, 64]: a valid signed i8, so |q| <= R/2 and
//    U + m, not U, is the result: U + m in (m/2, 3m/2) for A, B < 2m, the
//    bound the VALU product needs.
//  * The carry out of the low half of T + q m (an exact multiple of R) is the
//    rounded value of its top four column sums (the rest is < 2^-5 of a unit).
//
// One LDS row per operand: the multiplier (2A for squarings), overwritten by T's
// low digits as the product loop passes them, then T's high digits + m, then
// U + m. q goes from the accumulator layout to B fragments by permlane swaps.
// Included by mpcx_device.hpp (after montmul, before modexp_wave); not on its own.
#pragma once

namespace mpcx {

typedef int mx_v4i __attribute__((ext_vector_type(4)));

// MxShape, MxG2, MxG5, MX_WG: mpcx_internal.h (the C-ABI builds the tables with them)

struct MxConsts {
  const uint8_t* t1;  // LDS: table of m'' = -m^-1 mod R, pre-offset to this lane's row copy
  const uint8_t* t2;  // LDS: table of m, likewise
};
// lane (i = lane & 15, h = lane >> 4): fragment j at t + 16 (JMAX - j)
template <class S>
__device__ __forceinline__ MxConsts mx_consts(const uint8_t* img, int lane) {
  const int off = (lane & 15) * S::TAB_STRIDE + 16 * (lane >> 4);
  return MxConsts{img + off, img + S::TAB_BYTES + off};
}

// radix-2^28 digit (two's complement, |x| < 2^28) -> 4 radix-2^7 digits, one per
// byte (the top one signed): open a 1-bit gap above bits 6, 13 and 20
// (round 6: the closed form x + 2^7 (x >> 7) + 2^15 (x >> 14) + 2^23 (x >> 21) on the
// MAD pipe measured slower, profiles/r06/spab/)
__device__ __forceinline__ uint32_t mx_spread7(uint32_t x) {
  x += x & 0xFFFFFF80u;
  x += x & 0xFFFF8000u;
  x += x & 0xFF800000u;
  return x;
}

// T = A * B (B == A for SQR; B2IN: the row holds 2B) in montmul's row loop without
// the m_i N half: T's low L digits are emitted to tl[] as the window passes them
// (lane p == 0 of the group), the high L digits end in A (<= 2^28 + 2^10).
//
// Emission (MX_EMIT): 0 = lane p == 0 stores under an exec mask (two exec writes
// per iteration, and the SALU mask ops serialise against the MADs' carry-out
// SGPRs); 1 = every lane stores, lanes p != 0 into a per-lane trash slot of the
// wave's LDS area (tr: that lane's slots, L words from lane + 0), so the loop
// body has no exec changes.
#ifndef MX_EMIT
#define MX_EMIT 1
#endif
template <int P, int K, bool SQR, bool B2IN>
__device__ __forceinline__ void mx_product(uint32_t (&A)[K], const uint32_t* bl, uint32_t* tl, uint32_t* tr, int p) {
  static_assert(!SQR || (K % 2) == 1, "squaring schedule needs an odd digit count per lane");
  uint64_t acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0;
  uint32_t bnext = bl[0];
#pragma nounroll
  for (int o = 0; o < P; ++o) {
    const uint32_t* bo = bl + o * K;
    uint32_t* to = ((MX_EMIT == 0 || p == 0) ? tl : tr) + o * K;
    const uint32_t dsh = p > o ? 0u : (p == o ? 1u : 31u);
    static_for<0, K>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const uint32_t bi = bnext;
      bnext = bo[u + 1];
      const uint32_t b2 = B2IN ? bi : bi << 1;
      const uint32_t bd = b2 >> dsh;
      static_for<0, K>([&](auto kc) {
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
      });
      const uint64_t a0 = acc[u];
      acc[(u + 1) % K] += a0 >> DB;
      // lane 0's digit leaves the window as T's digit i (in CIOS it is zero);
      // it must not shift into the previous group's top slot
      const uint32_t lo = (uint32_t)a0 & M28;
      if constexpr (MX_EMIT == 1) {
        to[u] = lo;
      } else {
        if (p == 0) to[u] = lo;
      }
      acc[u] = from_next_lane(p == 0 ? 0u : lo);
#ifndef MX_ITER_FENCE
#define MX_ITER_FENCE 0
#endif
      if constexpr (MX_ITER_FENCE) __builtin_amdgcn_sched_barrier(0);
    });
  }
  carry_pass64<P, K>(acc);
  const uint32_t ctop = (uint32_t)(acc[K - 1] >> DB);
#pragma unroll
  for (int k = K - 1; k >= 1; --k) A[k] = ((uint32_t)acc[k] & M28) + (uint32_t)(acc[k - 1] >> DB);
  A[0] = (uint32_t)acc[0] & M28;
  A[0] += from_prev_lane(ctop);
}

// lane (n, h) <- lane (n, h - 1) (h = 0: lane (n, 3)); one LDS-crossbar permute
__device__ __forceinline__ int mx_from_prev_quarter(int v, int lane) {
  return __builtin_amdgcn_ds_bpermute(((lane - 16) & 63) << 2, v);
}

// split of the radix-2^28 digit sum c0 + c1 2^7 + c2 2^14 + c3 2^21 (+ add) into
// lo (bits 0..27 of the sum, as a signed remainder of lo_sum) and the carry:
// lo_sum = the low parts (< 2^31 for the bounds above), hi_sum = the high parts
__device__ __forceinline__ void mx_split(const mx_v4i c, int add, int& lo_sum, int& hi_sum) {
  lo_sum = c[0] + ((c[1] & 0x1FFFFF) << 7) + ((c[2] & 0x3FFF) << 14) + ((c[3] & 0x7F) << 21) + add;
  hi_sum = (c[1] >> 21) + (c[2] >> 14) + (c[3] >> 7);
}

// MX_SPLIT_MAD: the same digit sum as one 64-bit value V = c0 + add + c1 2^7 +
// c2 2^14 + c3 2^21 built by three v_mad_i64_i32 (the MAD pipe idles during the
// reduction) instead of masks, shifts and adds on the VALU; lo = V mod 2^28 and
// the carry V >> 28 (arithmetic) follow from V directly. Multipliers in SGPRs
// (VOP3 takes no literal), so the compiler cannot turn them back into shifts.
#ifndef MX_SPLIT_MAD
#define MX_SPLIT_MAD 1
#endif
__device__ __forceinline__ int64_t mx_sum64(const mx_v4i c, int add) {
  int64_t v = (int64_t)(c[0] + add);
  uint64_t cy;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(v), "=s"(cy) : "v"(c[1]), "s"(1 << 7));
  asm("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(v), "=s"(cy) : "v"(c[2]), "s"(1 << 14));
  asm("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(v), "=s"(cy) : "v"(c[3]), "s"(1 << 21));
  return v;
}
// V >> 28 as a 32-bit int (|V| < 2^59): one v_alignbit_b32 of the two halves
__device__ __forceinline__ int mx_hi28(int64_t v) {
  return (int)__builtin_amdgcn_alignbit((uint32_t)((uint64_t)v >> 32), (uint32_t)v, 28);
}

// acc[o - O0] += sum over K blocks kb of F_j (j = o - 4 kb) x bf[kb], for output
// blocks O0 <= o < O1; Toeplitz block j is read once and used for every kb it
// pairs with (one block ahead of its MFMAs)
template <class S, int NJ, int O0, int O1>
__device__ __forceinline__ void mx_toeplitz(mx_v4i (&acc)[O1 - O0], const uint8_t* f, const mx_v4i (&bf)[S::KB]) {
  // one ds_read_b128 per block: lane base in a VGPR, block offset an immediate
  auto ld = [&](int j) __attribute__((always_inline)) {
    return *reinterpret_cast<const mx_v4i*>(f + 16 * (S::JMAX - j));
  };
  static_for<0, O1 - O0>([&](auto oc) { acc[decltype(oc)::value] = mx_v4i{0, 0, 0, 0}; });
  // first and last Toeplitz block with an MFMA in this chunk
  constexpr int JLO = (O0 - 4 * (S::KB - 1)) > 0 ? (O0 - 4 * (S::KB - 1)) : 0;
  constexpr int JHI = (O1 - 1) < (NJ - 1) ? (O1 - 1) : (NJ - 1);
  mx_v4i fnext = ld(JLO);
  static_for<JLO, JHI + 1>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const mx_v4i fj = fnext;
    if constexpr (j + 1 <= JHI) fnext = ld(j + 1);
    // the next block's read stays one block ahead: ALU and MFMA may move
    // across, LDS reads may not (hoisting them all costs 4 VGPRs per block)
#ifndef MX_READ_FENCE
#define MX_READ_FENCE 1
#endif
    if constexpr (MX_READ_FENCE) __builtin_amdgcn_sched_barrier(0x000F);
    static_for<0, S::KB>([&](auto kc) {
      constexpr int kb = decltype(kc)::value;
      constexpr int o = j + 4 * kb;
      if constexpr (o >= O0 && o < O1) acc[o - O0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fj, bf[kb], acc[o - O0], 0, 0, 0);
    });
  });
}

// 4x4 transpose between the register index and the lane quarter (h): on return
// y[i] in lane (n, h) is x[h] of lane (n, i). Two permlane32 and two permlane16
// swaps (gfx950), no LDS.
__device__ __forceinline__ mx_v4i mx_transpose4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  auto r02 = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);
  auto r13 = __builtin_amdgcn_permlane32_swap(x1, x3, false, false);
  auto r01 = __builtin_amdgcn_permlane16_swap(r02[0], r13[0], false, false);
  auto r23 = __builtin_amdgcn_permlane16_swap(r02[1], r13[1], false, false);
  return mx_v4i{(int)r01[0], (int)r01[1], (int)r23[0], (int)r23[1]};
}

// Round 6 measured and removed: a workgroup barrier pairing one
// wave's product loop with its SIMD partner's reduction (slower), and each chunk's
// normalisation interleaved with the next chunk's MFMAs (equal).
// A <- A * B * R^-1 + m (mod-m class preserved; result in (m/2, 3m/2) for A, B < 2m).
// rows: this wavefront's G operand rows (S::ROW words each); operand g's row holds
// B (2B for squarings) on entry and is the scratch of the whole product: T's low
// digits overwrite B as the loop consumes it, then T's high digits + m, then
// U + m. md: m's L radix-2^28 digits (LDS).
// MX_PROF (microbench builds only): s_memtime stamps at the phase boundaries,
// accumulated per wave in MxProf (the stamps fence the scheduler around them)
#ifdef MX_PROF
struct MxProf {
  uint64_t t[7];
  uint64_t last;
};
#define MX_STAMP(i)                                          \
  do {                                                       \
    __builtin_amdgcn_sched_barrier(0);                       \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
    if ((i) > 0) pf->t[(i) - 1] += now_ - pf->last;          \
    pf->last = now_;                                         \
    __builtin_amdgcn_sched_barrier(0);                       \
  } while (0)
#define MX_PROF_ARG , MxProf* pf
#else
#define MX_STAMP(i) \
  do {              \
  } while (0)
#define MX_PROF_ARG
#endif
template <class S, bool SQR, bool B2IN>
__device__ __forceinline__ void montmul_mx(uint32_t (&A)[S::K], uint32_t* rows, const uint32_t* md,
                                           const MxConsts& c, int lane MX_PROF_ARG) {
  constexpr int P = S::P, K = S::K, L = S::L, ROW = S::ROW, KB = S::KB;
  const int g = lane / P, p = lane % P;    // block layout
  const int n = lane & 15, h = lane >> 4;  // MFMA layout
  uint32_t* rg = rows + g * ROW;
  // ---- T = A B on the VALU: low digits -> the row (behind the multiplier digits
  // the loop has read), high digits -> A
#ifndef MPCX_MX_TIMING
#define MPCX_MX_TIMING 0  // microbench builds only: 1 = product loop alone, 2 = reduction alone
#endif
  // MX_PRIO, the wave's issue priority by phase of the Montgomery product
  // (s_setprio; the two waves of a SIMD are mostly in different phases):
  // product loop P, fragment build F, q products R, q m products R2, carry
  // passes C. Presets: 0 none; 1 R = 1 (138.7 vs 139.6 ms, profiles/r06/libab1);
  // 2 P = 1; 3 P = F = 1; 4 P 2 > F = R = R2 1 > C 0; 5 (default) P 3 > F 2 >
  // R 1 > R2 = C 0. Config 2, three interleaved rounds per A/B
  // (profiles/r06/prioab2..4): 1 133.5 -> 4 128.2 (2, 3: 129.1) -> 5 123.3 ms.
  // The levels must fall along the product: equal levels for P and F (126.5) or
  // for R and R2 (124.9) lose, and so does the product loop's second half one
  // level down (126.0-126.6 vs 125.2, prioab5). Whenever the two waves are in
  // different phases, the one that is earlier in its product issues first; the
  // other fills the slots it leaves (a product-loop wave alone issues a MAD only
  // every ~10 cycles).
#ifndef MX_PRIO
#define MX_PRIO 5
#endif
  // -DMX_PRIO_P=.. etc. override one phase for an A/B
#ifndef MX_PRIO_P
#define MX_PRIO_P (MX_PRIO == 5 ? 3 : MX_PRIO == 4 ? 2 : (MX_PRIO == 2 || MX_PRIO == 3) ? 1 : 0)
#endif
#ifndef MX_PRIO_F
#define MX_PRIO_F (MX_PRIO == 5 ? 2 : (MX_PRIO == 3 || MX_PRIO == 4) ? 1 : 0)
#endif
#ifndef MX_PRIO_R
#define MX_PRIO_R ((MX_PRIO == 1 || MX_PRIO == 4 || MX_PRIO == 5) ? 1 : 0)
#endif
#ifndef MX_PRIO_R2
#define MX_PRIO_R2 (MX_PRIO == 5 ? 0 : MX_PRIO_R)
#endif
#ifndef MX_PRIO_C
#define MX_PRIO_C 0
#endif
  constexpr bool PRIO_ON = (MX_PRIO_P | MX_PRIO_F | MX_PRIO_R | MX_PRIO_R2 | MX_PRIO_C) != 0;
  MX_STAMP(0);
  if constexpr (PRIO_ON) __builtin_amdgcn_s_setprio(MX_PRIO_P);
  if constexpr (MPCX_MX_TIMING != 2) mx_product<P, K, SQR, B2IN>(A, rg, rg, rows + S::TRASH_OFF + lane, p);
  if constexpr (PRIO_ON) __builtin_amdgcn_s_setprio(MX_PRIO_F);
  MX_STAMP(1);
  if constexpr (MPCX_MX_TIMING == 1) return;
  wave_lds_fence();
  // ---- T's low half as B fragments (radix-2^7 bytes), every half of the wave
  mx_v4i bf[S::HALVES][KB];
  int ttop[S::HALVES];  // T's digit L - 1: the top 4 positions of the carry estimate
  static_for<0, S::HALVES>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    const uint32_t* rn = rows + (16 * s + n) * ROW;
    static_for<0, KB>([&](auto kc) {
      constexpr int kb = decltype(kc)::value;
      mx_v4i v = {0, 0, 0, 0};
      if (16 * kb + 4 * h < L) v = *reinterpret_cast<const mx_v4i*>(rn + 16 * kb + 4 * h);
      if constexpr (16 * kb + 15 >= L) {  // the digits past L in the last K block
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (16 * kb + 4 * h + i >= L) v[i] = 0;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (int)mx_spread7((uint32_t)v[i]);
      bf[s][kb] = v;
    });
    ttop[s] = (int)rn[L - 1];
  });
  wave_lds_fence();
  MX_STAMP(2);
  // ---- the row <- T's high digits + m (block layout)
#pragma unroll
  for (int k = 0; k < K; ++k) rg[p * K + k] = A[k] + md[p * K + k];
  if constexpr (PRIO_ON && MX_PRIO_R != MX_PRIO_F) __builtin_amdgcn_s_setprio(MX_PRIO_R);
  static_for<0, S::HALVES>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    uint32_t* rn = rows + (16 * s + n) * ROW;
    if constexpr (PRIO_ON && MX_PRIO_R2 != MX_PRIO_R && s > 0) __builtin_amdgcn_s_setprio(MX_PRIO_R);
    // ---- q column sums (o = j + 4 kb; chunks of output blocks bound the live
    // accumulators), balanced radix-2^28 digits with one carry step, as bytes;
    // every 4 blocks transposed in registers into one B fragment of phase 2
    mx_v4i qf[KB];
    {
      int xprev = 0;
      uint32_t X[4] = {0u, 0u, 0u, 0u};
      auto norm = [&](const mx_v4i& cs, int o) __attribute__((always_inline)) -> uint32_t {
        int lo, hi;
        if constexpr (MX_SPLIT_MAD) {
          const int64_t v = mx_sum64(cs, 1 << 27);
          lo = ((int)(uint32_t)v & (int)M28) - (1 << 27);
          hi = mx_hi28(v);
        } else {
          int lo_sum, hi_sum;
          mx_split(cs, 1 << 27, lo_sum, hi_sum);
          lo = (lo_sum & (int)M28) - (1 << 27);
          hi = hi_sum + (lo_sum >> 28);
        }
        const int x = mx_from_prev_quarter(hi, lane);
        int e = lo + (h == 0 ? xprev : x);
        xprev = x;
        if (4 * o + 3 >= L && 4 * o + h >= L) e = 0;  // digits past L: q is mod R
        return mx_spread7((uint32_t)e);
      };
      auto norm_block = [&](const mx_v4i& cs, auto oc) __attribute__((always_inline)) {
        constexpr int o = decltype(oc)::value;
        X[o & 3] = norm(cs, o);
        if constexpr ((o & 3) == 3) {
          qf[o >> 2] = mx_transpose4(X[0], X[1], X[2], X[3]);
        } else if constexpr (o == S::O1 - 1) {
          qf[o >> 2] = mx_transpose4(X[0], (o & 3) >= 1 ? X[1] : 0u, (o & 3) >= 2 ? X[2] : 0u, 0u);
        }
      };
      constexpr int NC = (S::O1 + S::CS1 - 1) / S::CS1;
      static_for<0, NC>([&](auto cc) {
        constexpr int O0 = S::CS1 * decltype(cc)::value;
        constexpr int O1 = O0 + S::CS1 < S::O1 ? O0 + S::CS1 : S::O1;
        mx_v4i acc[O1 - O0];
        mx_toeplitz<S, S::NJ1, O0, O1>(acc, c.t1, bf[s]);
        static_for<0, O1 - O0>([&](auto oc) {
          norm_block(acc[decltype(oc)::value], std::integral_constant<int, O0 + decltype(oc)::value>{});
        });
        __builtin_amdgcn_sched_barrier(0);  // one chunk's accumulators live at a time
      });
    }
    MX_STAMP(3);
    if constexpr (PRIO_ON && MX_PRIO_R2 != MX_PRIO_R) __builtin_amdgcn_s_setprio(MX_PRIO_R2);
    // ---- q m column sums for blocks O2LO.. : the lane whose 4 positions are the
    // low half's top (N7 - 4 .. N7 - 1) gives the carry out of the low half, the
    // lanes at positions N7 + 4d the digits d of U + m, adding T's high digit + m
    // from the row; the carry chain runs through the quarters as in q
    {
      int xprev = 0;
      auto emit = [&](const mx_v4i& cs, int o) __attribute__((always_inline)) {
        const int pos = 16 * o + 4 * h;
        const bool carry_lane = pos == S::N7 - 4;
        const int d = (pos - S::N7) >> 2;  // U's digit (< 0: the low half)
        const int dc = d < 0 ? 0 : d;
        const int add = carry_lane ? ttop[s] + (1 << 27) : (int)rn[dc];
        int hi, dig, top;  // dig: the sum's bits 0..27; top: the sum mod 2^32
        if constexpr (MX_SPLIT_MAD) {
          const int64_t v = mx_sum64(cs, add);
          hi = mx_hi28(v);  // on the carry lane: round(low half / R)
          top = (int)(uint32_t)v;
          dig = top & (int)M28;
        } else {
          int lo_sum, hi_sum;
          mx_split(cs, add, lo_sum, hi_sum);
          hi = hi_sum + (lo_sum >> 28);
          top = (int)((uint32_t)lo_sum + ((uint32_t)hi_sum << 28));
          dig = lo_sum & (int)M28;
        }
        const int x = mx_from_prev_quarter(hi, lane);
        const int cin = h == 0 ? xprev : x;
        xprev = x;
        // the top digit keeps its carry (the value is < 2m < 2^(28 L - 47))
        const int u = d == L - 1 ? top + cin : dig + cin;
        if (d >= 0) rn[dc] = (uint32_t)u;
      };
      constexpr int NC = (S::O2HI - S::O2LO + S::CS2 - 1) / S::CS2;
      static_for<0, NC>([&](auto cc) {
        constexpr int O0 = S::O2LO + S::CS2 * decltype(cc)::value;
        constexpr int O1 = O0 + S::CS2 < S::O2HI ? O0 + S::CS2 : S::O2HI;
        mx_v4i acc[O1 - O0];
        mx_toeplitz<S, S::NJ2, O0, O1>(acc, c.t2, qf);
        static_for<0, O1 - O0>([&](auto oc) { emit(acc[decltype(oc)::value], O0 + decltype(oc)::value); });
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  });
  if constexpr (PRIO_ON) __builtin_amdgcn_s_setprio(MX_PRIO_C);
  MX_STAMP(4);
  wave_lds_fence();
  // ---- back to the block layout; signed carry passes until every digit is >= 0
#pragma unroll
  for (int k = 0; k < K; ++k) A[k] = rg[p * K + k];
  MX_STAMP(5);
  // MX_CARRY_SKIP: the emitted digits lie in (-2^16, 2^28 + 2^16) (one carry step
  // of |carry| < 2^16); the next product takes any non-negative digits of that
  // size (its 64-bit accumulators have the room), so the passes run only when
  // some digit of the wave is negative (~1 wave in 4)
#ifndef MX_CARRY_SKIP
#define MX_CARRY_SKIP 1
#endif
  bool need = true;
  if constexpr (MX_CARRY_SKIP) {
    uint32_t sg = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) sg |= A[k];
    need = __any((int)sg < 0);
  }
  for (int it = 0; need && it < L + 2; ++it) {
    const int top = (int)A[K - 1];
    const int ctop = (p == P - 1) ? 0 : (top >> DB);
#pragma unroll
    for (int k = K - 1; k >= 1; --k) {
      const int cur = (int)A[k];
      const bool keep = (k == K - 1) && (p == P - 1);
      A[k] = (uint32_t)((keep ? cur : (cur & (int)M28)) + ((int)A[k - 1] >> DB));
    }
    const int c0 = (int)from_prev_lane((uint32_t)ctop);
    A[0] = (uint32_t)(((int)A[0] & (int)M28) + (p == 0 ? 0 : c0));
    bool neg = false;
#pragma unroll
    for (int k = 0; k < K; ++k) neg |= (int)A[k] < 0;
    if (!__any(neg)) break;
  }
  MX_STAMP(6);
}

}  // namespace mpcx
