// mpcx_mx.hpp -- gfx950 Montgomery products of the 4096-bit class with the
// REDUCTION on the matrix cores (v_mfma_i32_16x16x64_i8), the product A*B on
// the VALU.
//
// Every operand of a k_modexp batch shares the modulus m (Paillier N^2 of one
// key; config 2: 65,536 x r^N mod N^2), so the two reduction products of a
// Montgomery multiplication in separated form,
//     q = (T mod R) * m'' mod R     (m'' = -m^-1 mod R)
//     U = (T + q m) / R,
// are products of a batch of rows with FIXED Toeplitz matrices of m'' and m:
// dense contractions. The VALU keeps what is per operand -- T = A*B, the same
// lazy radix-2^28 row loop as montmul<4, 37> (mpcx_device.hpp) without its
// m_i N half -- and the matrix cores take the reduction (two thirds of a
// CIOS squaring's multiply-accumulates).
//
// Layout (one wavefront, G = 16 operands; R = 2^(28*148) = 2^4144, the same
// Montgomery domain as geometry 2, so tables, constants and the CIOS path mix):
//  * VALU ("block") layout: operand g on lanes 4g..4g+3, lane p holds radix-2^28
//    digits 37p..37p+36 -- montmul's layout.
//  * MFMA layout: operand n = lane & 15, quarter h = lane >> 4. Radix-2^7 digits
//    (4 per radix-2^28 digit, one byte each, so the conversion is a bit spread)
//    are the K index; a 16x16x64 MFMA takes B = 64 digits of 16 operands (lane
//    (n, h): bytes 16h..16h+15 of the K block -- one ds_read_b128 of radix-2^28
//    digits 16kb + 4h .. +3) and A = the Toeplitz block of m'' or m for output
//    positions 16o..16o+15 (precomputed per modulus in the same lane map, so the
//    hardware's k order inside a lane never matters), and accumulates column
//    sums C[4h + r][n] = output position 16o + 4h + r of operand n: one lane
//    holds 4 consecutive radix-2^7 positions = ONE radix-2^28 digit.
//  * Column sums are exact in i32: <= 592 products of 7-bit digits.
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

constexpr int MX_P = 4, MX_K = 37, MX_L = 148, MX_G = 16;
constexpr int MX_ROW = 148;  // dwords per operand row: b128 reads of 16 rows and b32 writes conflict-free
constexpr int MX_KB = 10;    // K blocks of 64 radix-2^7 digits (the last holds 16 of 592)
constexpr int MX_O1 = 37;    // output blocks of q (positions 0..591)
constexpr int MX_NJ1 = 37;   // Toeplitz blocks of m'' (delta = 16 j, j < 37)
constexpr int MX_NJ2 = 41;   // Toeplitz blocks of m (delta = 16 j, j < 41)
constexpr int MX_O2LO = 36, MX_O2HI = 74;  // output blocks of q m kept: positions 576..1183
// output-block chunks (live accumulators: one chunk at a time)
#ifndef MX_C1A
#define MX_C1A 12  // phase-1 chunks end on 4-block boundaries (one B fragment of q per 4 blocks)
#define MX_C1B 24
#define MX_C2A 49
#define MX_C2B 62
#endif
// LDS words per wavefront: the 16 operand rows, +4 for the product loop's read
// one past the last row
constexpr int MX_WAVE_WORDS = MX_G * MX_ROW + 4;
// Toeplitz tables in LDS, shared by the workgroup: per table (m'' for q, m for
// q m) 16 copies, one per fragment row i, of the digit string reversed and
// shifted so that lane (i, h)'s 16 bytes of block j start 16-aligned at
// i * MX_TAB_STRIDE + 16 (40 - j + h): copy_i[x] = v7[640 - x + i]. The stride
// (45 x 16 B) puts the 16 rows of a ds_read_b128 lane group on distinct banks.
constexpr int MX_TAB_STRIDE = 720;
constexpr int MX_TAB_BYTES = 16 * MX_TAB_STRIDE;  // one table
constexpr int MX_IMG_BYTES = 2 * MX_TAB_BYTES;    // the LDS image of both (the C-ABI uploads it)
// workgroup: MX_WG wavefronts share the image and m's digits
#ifndef MX_WG
#define MX_WG 4
#endif
constexpr int MX_LDS_WORDS_WG = MX_IMG_BYTES / 4 + MX_L + 4 + MX_WG * MX_WAVE_WORDS;

struct MxConsts {
  const uint8_t* t1;  // LDS: table of m'' = -m^-1 mod R, pre-offset to this lane's row copy
  const uint8_t* t2;  // LDS: table of m, likewise
};
// lane (i = lane & 15, h = lane >> 4): fragment j at t + 16 (40 - j)
__device__ __forceinline__ MxConsts mx_consts(const uint8_t* img, int lane) {
  const int off = (lane & 15) * MX_TAB_STRIDE + 16 * (lane >> 4);
  return MxConsts{img + off, img + MX_TAB_BYTES + off};
}

// radix-2^28 digit (two's complement, |x| < 2^28) -> 4 radix-2^7 digits, one per
// byte (the top one signed): open a 1-bit gap above bits 6, 13 and 20
__device__ __forceinline__ uint32_t mx_spread7(uint32_t x) {
  x += x & 0xFFFFFF80u;
  x += x & 0xFFFF8000u;
  x += x & 0xFF800000u;
  return x;
}

// T = A * B (B == A for SQR; B2IN: the row holds 2B) in montmul's row loop without
// the m_i N half: T's low 148 digits are emitted to tl[] as the window passes them
// (lane p == 0 of the group), the high 148 digits end in A (<= 2^28 + 2^10).
template <int K, bool SQR, bool B2IN>
__device__ __forceinline__ void mx_product(uint32_t (&A)[K], const uint32_t* bl, uint32_t* tl, int p) {
  constexpr int P = MX_P;
  static_assert(!SQR || (K % 2) == 1, "squaring schedule needs an odd digit count per lane");
  uint64_t acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0;
  uint32_t bnext = bl[0];
#ifndef MPCX_MX_EMIT_REG
#define MPCX_MX_EMIT_REG 0  // 1: T's low digits gathered in registers, stored once per block
#endif
#if MPCX_MX_EMIT_REG
  uint32_t em[K];
  const uint32_t shmask = p == 0 ? 0u : M28;
#endif
#pragma nounroll
  for (int o = 0; o < P; ++o) {
    const uint32_t* bo = bl + o * K;
    uint32_t* to = tl + o * K;
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
#if MPCX_MX_EMIT_REG
      em[u] = (uint32_t)a0;
      acc[u] = from_next_lane((uint32_t)a0 & shmask);
#else
      const uint32_t lo = (uint32_t)a0 & M28;
      if (p == 0) to[u] = lo;
      acc[u] = from_next_lane(p == 0 ? 0u : lo);
#endif
    });
#if MPCX_MX_EMIT_REG
    // the block's 37 digits of T, written once under one exec mask
    if (p == 0) {
#pragma unroll
      for (int u = 0; u < K; ++u) to[u] = em[u] & M28;
    }
#endif
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

// acc[o - O0] += sum over K blocks kb of F_j (j = o - 4 kb) x bf[kb], for output
// blocks O0 <= o < O1; Toeplitz block j (1 KB of fragments) is loaded once and
// used for every kb it pairs with (one load ahead of its MFMAs)
template <int NJ, int O0, int O1>
__device__ __forceinline__ void mx_toeplitz(mx_v4i (&acc)[O1 - O0], const uint8_t* f,
                                            const mx_v4i (&bf)[MX_KB], int lane) {
  // one ds_read_b128 per block: lane base in a VGPR, block offset an immediate
  auto ld = [&](int j) __attribute__((always_inline)) {
    return *reinterpret_cast<const mx_v4i*>(f + 16 * (40 - j));
  };
  static_for<0, O1 - O0>([&](auto oc) { acc[decltype(oc)::value] = mx_v4i{0, 0, 0, 0}; });
  // first and last Toeplitz block with an MFMA in this chunk
  constexpr int JLO = (O0 - 4 * (MX_KB - 1)) > 0 ? (O0 - 4 * (MX_KB - 1)) : 0;
  constexpr int JHI = (O1 - 1) < (NJ - 1) ? (O1 - 1) : (NJ - 1);
  mx_v4i fnext = ld(JLO);
  static_for<JLO, JHI + 1>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const mx_v4i fj = fnext;
    if constexpr (j + 1 <= JHI) fnext = ld(j + 1);
    // the next block's read stays one block ahead: ALU and MFMA may move
    // across, LDS reads may not (hoisting them all costs 4 VGPRs per block)
    __builtin_amdgcn_sched_barrier(0x000F);
    static_for<0, MX_KB>([&](auto kc) {
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

// A <- A * B * R^-1 + m (mod-m class preserved; result in (m/2, 3m/2) for A, B < 2m).
// rows: this wavefront's 16 operand rows (MX_ROW words each); operand g's row
// holds B (2B for squarings) on entry and is the scratch of the whole product:
// T's low digits overwrite B as the loop consumes it, then T's high digits + m,
// then U + m. md: m's 148 radix-2^28 digits (LDS).
template <bool SQR, bool B2IN>
__device__ __forceinline__ void montmul_mx(uint32_t (&A)[MX_K], uint32_t* rows, const uint32_t* md,
                                           const MxConsts& c, int lane) {
  const int g = lane >> 2, p = lane & 3;  // block layout
  const int n = lane & 15, h = lane >> 4;  // MFMA layout
  uint32_t* rg = rows + g * MX_ROW;
  uint32_t* rn = rows + n * MX_ROW;
  // ---- T = A B on the VALU: low digits -> the row (behind the multiplier digits
  // the loop has read), high digits -> A
#ifndef MPCX_MX_TIMING
#define MPCX_MX_TIMING 0  // microbench builds only: 1 = product loop alone, 2 = reduction alone
#endif
  if constexpr (MPCX_MX_TIMING != 2) mx_product<MX_K, SQR, B2IN>(A, rg, rg, p);
  if constexpr (MPCX_MX_TIMING == 1) return;
  wave_lds_fence();
  // ---- T's low half as B fragments (radix-2^7 bytes)
  mx_v4i bf[MX_KB];
  static_for<0, MX_KB>([&](auto kc) {
    constexpr int kb = decltype(kc)::value;
    mx_v4i v = {0, 0, 0, 0};
    if (kb < MX_KB - 1 || h == 0) v = *reinterpret_cast<const mx_v4i*>(rn + 16 * kb + 4 * h);
    bf[kb] = v;
  });
  const int t147 = (int)rn[MX_L - 1];  // T's digit 147: positions 588..591 of the carry estimate
  static_for<0, MX_KB>([&](auto kc) {
    constexpr int kb = decltype(kc)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i) bf[kb][i] = (int)mx_spread7((uint32_t)bf[kb][i]);
  });
  wave_lds_fence();
  // ---- the row <- T's high digits + m (block layout)
#pragma unroll
  for (int k = 0; k < MX_K; ++k) rg[p * MX_K + k] = A[k] + md[p * MX_K + k];
  // ---- q column sums (o = j + 4 kb; chunks of output blocks bound the live
  // accumulators), balanced radix-2^28 digits with one carry step, as bytes;
  // every 4 blocks transposed in registers into one B fragment of phase 2
  mx_v4i qf[MX_KB];
  {
    int xprev = 0;
    uint32_t X[4] = {0u, 0u, 0u, 0u};
    auto norm = [&](const mx_v4i& cs) __attribute__((always_inline)) -> uint32_t {
      int lo_sum, hi_sum;
      mx_split(cs, 1 << 27, lo_sum, hi_sum);
      const int lo = (lo_sum & (int)M28) - (1 << 27);
      const int hi = hi_sum + (lo_sum >> 28);
      const int x = mx_from_prev_quarter(hi, lane);
      const int e = lo + (h == 0 ? xprev : x);
      xprev = x;
      return mx_spread7((uint32_t)e);
    };
    auto chunk = [&](auto o0c, auto o1c) __attribute__((always_inline)) {
      constexpr int O0 = decltype(o0c)::value, O1 = decltype(o1c)::value;
      mx_v4i acc[O1 - O0];
      mx_toeplitz<MX_NJ1, O0, O1>(acc, c.t1, bf, lane);
      static_for<0, O1 - O0>([&](auto oc) {
        constexpr int o = O0 + decltype(oc)::value;
        X[o & 3] = norm(acc[decltype(oc)::value]);
        if constexpr ((o & 3) == 3) {
          qf[o >> 2] = mx_transpose4(X[0], X[1], X[2], X[3]);
        } else if constexpr (o == MX_O1 - 1) {
          qf[o >> 2] = mx_transpose4(X[0], (o & 3) >= 1 ? X[1] : 0u, (o & 3) >= 2 ? X[2] : 0u, 0u);
        }
      });
      __builtin_amdgcn_sched_barrier(0);  // one chunk's accumulators live at a time
    };
    chunk(std::integral_constant<int, 0>{}, std::integral_constant<int, MX_C1A>{});
    chunk(std::integral_constant<int, MX_C1A>{}, std::integral_constant<int, MX_C1B>{});
    chunk(std::integral_constant<int, MX_C1B>{}, std::integral_constant<int, MX_O1>{});
  }
  // ---- q m column sums for positions 576..1183, in chunks; block 36 gives the
  // carry out of the low half (lane h = 3), blocks 37.. the digits
  // d = 4 (o - 37) + h of U + m, adding T's high digit + m from the row
  {
    int xprev = 0;
    auto emit = [&](const mx_v4i& cs, int o) __attribute__((always_inline)) {
      int lo_sum, hi_sum;
      if (o == MX_O2LO) {
        mx_split(cs, t147 + (1 << 27), lo_sum, hi_sum);
        const int carry = hi_sum + (lo_sum >> 28);  // round(low half / R), meaningful on h = 3
        xprev = mx_from_prev_quarter(carry, lane);   // lane (n, 0) <- lane (n, 3)
        return;
      }
      const int d = 4 * (o - MX_O2LO - 1) + h;
      mx_split(cs, (int)rn[d], lo_sum, hi_sum);
      const int hi = hi_sum + (lo_sum >> 28);
      const int x = mx_from_prev_quarter(hi, lane);
      const int cin = h == 0 ? xprev : x;
      xprev = x;
      int u = (lo_sum & (int)M28) + cin;
      // the top digit keeps its carry (the value is < 2m < 2^4097)
      if (o == MX_O2HI - 1 && h == 3) u = (int)((uint32_t)lo_sum + ((uint32_t)hi_sum << 28)) + cin;
      rn[d] = (uint32_t)u;
    };
    auto chunk = [&](auto o0c, auto o1c) __attribute__((always_inline)) {
      constexpr int O0 = decltype(o0c)::value, O1 = decltype(o1c)::value;
      mx_v4i acc[O1 - O0];
      mx_toeplitz<MX_NJ2, O0, O1>(acc, c.t2, qf, lane);
      static_for<0, O1 - O0>([&](auto oc) { emit(acc[decltype(oc)::value], O0 + decltype(oc)::value); });
      __builtin_amdgcn_sched_barrier(0);
    };
    chunk(std::integral_constant<int, MX_O2LO>{}, std::integral_constant<int, MX_C2A>{});
    chunk(std::integral_constant<int, MX_C2A>{}, std::integral_constant<int, MX_C2B>{});
    chunk(std::integral_constant<int, MX_C2B>{}, std::integral_constant<int, MX_O2HI>{});
  }
  wave_lds_fence();
  // ---- back to the block layout; signed carry passes until every digit is >= 0
#pragma unroll
  for (int k = 0; k < MX_K; ++k) A[k] = rg[p * MX_K + k];
  for (int it = 0; it < MX_L + 2; ++it) {
    const int top = (int)A[MX_K - 1];
    const int ctop = (p == MX_P - 1) ? 0 : (top >> DB);
#pragma unroll
    for (int k = MX_K - 1; k >= 1; --k) {
      const int cur = (int)A[k];
      const bool keep = (k == MX_K - 1) && (p == MX_P - 1);
      A[k] = (uint32_t)((keep ? cur : (cur & (int)M28)) + ((int)A[k - 1] >> DB));
    }
    const int c0 = (int)from_prev_lane((uint32_t)ctop);
    A[0] = (uint32_t)(((int)A[0] & (int)M28) + (p == 0 ? 0 : c0));
    bool neg = false;
#pragma unroll
    for (int k = 0; k < MX_K; ++k) neg |= (int)A[k] < 0;
    if (!__any(neg)) break;
  }
}

}  // namespace mpcx
