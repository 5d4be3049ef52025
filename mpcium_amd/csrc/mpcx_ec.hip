// mpcx_ec.hip -- batched secp256k1 point combinations on gfx950:
//   out_i = a_i G + b_i P_i + c_i Q_i
// Every point equation of tss-lib's GG18 signing outside the MtA is one of
// these (up:ecdsa/signing round_1.go .. finalize.go; btcec/v2 S256 arithmetic,
// /root/reference/go.mod:29): Gamma_i = gamma_i G, the Schnorr / ZKV proofs'
// alpha = a G (+ b R) and their checks t G - c X == alpha, R = theta^-1 sum
// Gamma, V_i = s_i R + l_i G, U_i = rho_i V, and ecdsa.Verify's u1 G + u2 X.
// One thread per item: the batch is thousands of independent small
// computations (wallets x signers), integer work with no shared operand.
//
// Field: p = 2^256 - 2^32 - 977, eight 32-bit limbs, values kept < p; a product
// is folded with 2^256 = 2^32 + 977 (mod p). Points: Jacobian (X, Y, Z) with
// a = 0 formulas (dbl-2009-l, add-2007-bl, madd-2007-bl). a G uses a fixed-base
// comb of 8-bit windows (32 x 255 affine points, 522 KB in HBM, built once per
// device by this kernel itself as plain multiples of G: 32 mixed additions, no
// doublings); b P + c Q share
// 256 doublings with 4-bit windows (Shamir's trick; 15-entry Jacobian tables per
// thread in a lane-coalesced global workspace). One field inversion per item
// returns the affine result.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpcx_internal.h"

namespace mpcx {
namespace {

struct Fe {
  uint32_t v[8];
};

__device__ __constant__ const uint32_t kP[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                                0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

__device__ __forceinline__ bool fe_is_zero(const Fe& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i];
  return o == 0;
}
// a >= p (a < 2^256)
__device__ __forceinline__ bool fe_geq_p(const Fe& a) {
  // p's limbs 2..7 are all ones: a >= p iff those are all ones and (a1, a0) >= (p1, p0)
  uint32_t hi = 0xFFFFFFFFu;
#pragma unroll
  for (int i = 2; i < 8; ++i) hi &= a.v[i];
  if (hi != 0xFFFFFFFFu) return false;
  if (a.v[1] != kP[1]) return a.v[1] > kP[1];
  return a.v[0] >= kP[0];
}
// a + k (k < 2^40) * (2^32 + 977) folded into a 256-bit value, then < p
__device__ __forceinline__ void fe_fold(Fe& r, uint64_t k) {
  while (k) {
    // r += k * 977 + (k << 32)
    uint64_t lo = k * 977u;  // < 2^50
    uint64_t c = (uint64_t)r.v[0] + (uint32_t)lo;
    r.v[0] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)r.v[1] + (uint32_t)(lo >> 32) + (uint32_t)k;
    r.v[1] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)r.v[2] + (uint32_t)(k >> 32);
    r.v[2] = (uint32_t)c;
    c >>= 32;
#pragma unroll
    for (int i = 3; i < 8; ++i) {
      c += r.v[i];
      r.v[i] = (uint32_t)c;
      c >>= 32;
    }
    k = c;  // 2^256 wrapped: fold once more (at most twice in total)
  }
  if (fe_geq_p(r)) {  // r - p = r + (2^32 + 977) - 2^256
    uint64_t c = (uint64_t)r.v[0] + 977u;
    r.v[0] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)r.v[1] + 1u;
    r.v[1] = (uint32_t)c;
    c >>= 32;
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      c += r.v[i];
      r.v[i] = (uint32_t)c;
      c >>= 32;
    }
  }
}
__device__ __forceinline__ Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  fe_fold(r, c);
  return r;
}
__device__ __forceinline__ Fe fe_sub(const Fe& a, const Fe& b) {
  Fe r;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t d = (int64_t)a.v[i] - (int64_t)b.v[i] + br;
    r.v[i] = (uint32_t)d;
    br = d >> 32;  // 0 or -1
  }
  if (br) {  // a < b: add p back (mod 2^256)
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)r.v[i] + kP[i];
      r.v[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  return r;
}
__device__ __forceinline__ Fe fe_dbl(const Fe& a) { return fe_add(a, a); }
// t (512 bits, 16 limbs) mod p: two folds of the high half by
// 2^256 = 2^32 + 977
__device__ __forceinline__ Fe fe_reduce512(const uint32_t (&t)[16]) {
  // r = lo + hi * 977 + (hi << 32)
  Fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)t[i] + (uint64_t)t[8 + i] * 977u + (i ? t[7 + i] : 0u);
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  c += t[15];  // the last shifted limb
  fe_fold(r, c);
  return r;
}
// a * b mod p: 8 x 8 schoolbook rows into 16 limbs, then the fold
__device__ __forceinline__ Fe fe_mul(const Fe& a, const Fe& b) {
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c += (uint64_t)a.v[i] * b.v[j] + t[i + j];
      t[i + j] = (uint32_t)c;
      c >>= 32;
    }
    t[i + 8] = (uint32_t)c;
  }
  return fe_reduce512(t);
}
// a^2 mod p: the 28 products a_i a_j (i < j) once, doubled by a shift, plus
// the 8 squares on the diagonal (36 limb products against fe_mul's 64)
__device__ __forceinline__ Fe fe_sqr(const Fe& a) {
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; ++j) {
      c += (uint64_t)a.v[i] * a.v[j] + t[i + j];
      t[i + j] = (uint32_t)c;
      c >>= 32;
    }
    t[i + 8] = (uint32_t)c;  // no earlier row reaches limb i + 8
  }
  uint32_t top = 0;  // off-diagonal sum < 2^511: doubling fits 16 limbs
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t v = t[k];
    t[k] = (v << 1) | top;
    top = v >> 31;
  }
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t sq = (uint64_t)a.v[i] * a.v[i];
    c += (uint64_t)t[2 * i] + (uint32_t)sq;
    t[2 * i] = (uint32_t)c;
    c >>= 32;
    c += (uint64_t)t[2 * i + 1] + (sq >> 32);
    t[2 * i + 1] = (uint32_t)c;
    c >>= 32;
  }
  return fe_reduce512(t);
}
__device__ Fe fe_sqr_n(Fe r, int n) {
  for (int i = 0; i < n; ++i) r = fe_sqr(r);
  return r;
}
// a^(p-2) by an addition chain: p - 2 = 2^256 - 2^32 - 979 is 223 ones, a
// zero, then 0xFFFFFC2D = 22 ones, 00001, 011, 01. x_k = a^(2^k - 1) built
// up to x223 (x_{i+j} = x_i^(2^j) x_j), then the low 33 bits appended:
// 255 squarings and 15 multiplications (square-and-multiply: 255 + 238)
__device__ Fe fe_inv(const Fe& a) {
  const Fe x2 = fe_mul(fe_sqr(a), a);
  const Fe x3 = fe_mul(fe_sqr(x2), a);
  const Fe x6 = fe_mul(fe_sqr_n(x3, 3), x3);
  const Fe x9 = fe_mul(fe_sqr_n(x6, 3), x3);
  const Fe x11 = fe_mul(fe_sqr_n(x9, 2), x2);
  const Fe x22 = fe_mul(fe_sqr_n(x11, 11), x11);
  const Fe x44 = fe_mul(fe_sqr_n(x22, 22), x22);
  const Fe x88 = fe_mul(fe_sqr_n(x44, 44), x44);
  const Fe x176 = fe_mul(fe_sqr_n(x88, 88), x88);
  const Fe x220 = fe_mul(fe_sqr_n(x176, 44), x44);
  const Fe x223 = fe_mul(fe_sqr_n(x220, 3), x3);
  Fe r = fe_mul(fe_sqr_n(x223, 23), x22);  // 223 ones, 0, 22 ones
  r = fe_mul(fe_sqr_n(r, 5), a);           // 00001
  r = fe_mul(fe_sqr_n(r, 3), x2);          // 011
  r = fe_mul(fe_sqr_n(r, 2), a);           // 01
  return r;
}

struct Jac {
  Fe X, Y, Z;  // Z == 0: infinity
};

__device__ __forceinline__ bool jac_inf(const Jac& p) { return fe_is_zero(p.Z); }

// dbl-2009-l (a = 0)
__device__ Jac jac_dbl(const Jac& p) {
  if (jac_inf(p) || fe_is_zero(p.Y)) return Jac{};
  const Fe A = fe_sqr(p.X), B = fe_sqr(p.Y), C = fe_sqr(B);
  const Fe D = fe_dbl(fe_sub(fe_sqr(fe_add(p.X, B)), fe_add(A, C)));
  const Fe E = fe_add(fe_dbl(A), A), F = fe_sqr(E);
  Jac r;
  r.X = fe_sub(F, fe_dbl(D));
  const Fe C8 = fe_dbl(fe_dbl(fe_dbl(C)));
  r.Y = fe_sub(fe_mul(E, fe_sub(D, r.X)), C8);
  r.Z = fe_dbl(fe_mul(p.Y, p.Z));
  return r;
}
// add-2007-bl
__device__ Jac jac_add(const Jac& p, const Jac& q) {
  if (jac_inf(p)) return q;
  if (jac_inf(q)) return p;
  const Fe Z1Z1 = fe_sqr(p.Z), Z2Z2 = fe_sqr(q.Z);
  const Fe U1 = fe_mul(p.X, Z2Z2), U2 = fe_mul(q.X, Z1Z1);
  const Fe S1 = fe_mul(fe_mul(p.Y, q.Z), Z2Z2), S2 = fe_mul(fe_mul(q.Y, p.Z), Z1Z1);
  const Fe H = fe_sub(U2, U1), R = fe_sub(S2, S1);
  if (fe_is_zero(H)) {
    if (fe_is_zero(R)) return jac_dbl(p);
    return Jac{};
  }
  const Fe HH = fe_sqr(H), HHH = fe_mul(H, HH), V = fe_mul(U1, HH);
  Jac r;
  r.X = fe_sub(fe_sub(fe_sqr(R), HHH), fe_dbl(V));
  r.Y = fe_sub(fe_mul(R, fe_sub(V, r.X)), fe_mul(S1, HHH));
  r.Z = fe_mul(fe_mul(p.Z, q.Z), H);
  return r;
}
// p + (x, y) affine (madd-2007-bl style, Z2 = 1)
__device__ Jac jac_madd(const Jac& p, const Fe& x, const Fe& y) {
  if (jac_inf(p)) {
    Jac r;
    r.X = x;
    r.Y = y;
    r.Z = Fe{{1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};
    return r;
  }
  const Fe Z1Z1 = fe_sqr(p.Z);
  const Fe U2 = fe_mul(x, Z1Z1), S2 = fe_mul(fe_mul(y, p.Z), Z1Z1);
  const Fe H = fe_sub(U2, p.X), R = fe_sub(S2, p.Y);
  if (fe_is_zero(H)) {
    if (fe_is_zero(R)) return jac_dbl(p);
    return Jac{};
  }
  const Fe HH = fe_sqr(H), HHH = fe_mul(H, HH), V = fe_mul(p.X, HH);
  Jac r;
  r.X = fe_sub(fe_sub(fe_sqr(R), HHH), fe_dbl(V));
  r.Y = fe_sub(fe_mul(R, fe_sub(V, r.X)), fe_mul(p.Y, HHH));
  r.Z = fe_mul(p.Z, H);
  return r;
}

__device__ __forceinline__ Fe load_fe(const uint32_t* w) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = w[i];
  return r;
}

// per-thread table workspace: entry e (0..29: P's 1..15, Q's 1..15), coordinate
// word k (24 per Jacobian point), lane-coalesced across the block
__device__ __forceinline__ void tbl_put(uint32_t* ws, int e, const Jac& p) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ws[((e * 24) + i) * 64 + lane] = p.X.v[i];
    ws[((e * 24) + 8 + i) * 64 + lane] = p.Y.v[i];
    ws[((e * 24) + 16 + i) * 64 + lane] = p.Z.v[i];
  }
}
__device__ __forceinline__ Jac tbl_get(const uint32_t* ws, int e) {
  const int lane = threadIdx.x;
  Jac p;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    p.X.v[i] = ws[((e * 24) + i) * 64 + lane];
    p.Y.v[i] = ws[((e * 24) + 8 + i) * 64 + lane];
    p.Z.v[i] = ws[((e * 24) + 16 + i) * 64 + lane];
  }
  return p;
}

__device__ __forceinline__ uint32_t nibble(const uint32_t* k, int w) { return (k[w >> 3] >> ((w & 7) * 4)) & 15u; }

}  // namespace

// a: count x 24 words (a, b, c), pts: count x 32 words (P.x, P.y, Q.x, Q.y;
// all-zero = infinity), out: count x 16 words (x, y; all-zero = infinity),
// gtab: 32 x 255 affine points (x, y as 8 words each) of d 256^w G, ws: the
// per-thread tables (blocks x 30 x 24 x 64 words)
__global__ __launch_bounds__(64) void k_ec_combine(const uint32_t* __restrict__ sc, const uint32_t* __restrict__ pts,
                                                   uint32_t* __restrict__ out, const uint32_t* __restrict__ gtab,
                                                   uint32_t* __restrict__ ws_all, uint32_t count) {
  const uint32_t item = blockIdx.x * 64u + threadIdx.x;
  const bool active = item < count;
  uint32_t* ws = ws_all + (size_t)blockIdx.x * (30u * 24u * 64u);
  const uint32_t* s = sc + (size_t)(active ? item : 0u) * 24u;
  const uint32_t* pp = pts + (size_t)(active ? item : 0u) * 32u;
  uint32_t kb[8], kc[8];
  bool usep = false, useq = false;
  {
    uint32_t ob = 0, oc = 0, op = 0, oq = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      kb[i] = active ? s[8 + i] : 0u;
      kc[i] = active ? s[16 + i] : 0u;
      ob |= kb[i];
      oc |= kc[i];
      op |= pp[i] | pp[8 + i];
      oq |= pp[16 + i] | pp[24 + i];
    }
    usep = ob && op;
    useq = oc && oq;
  }
  // tables kP, kQ for k = 1..15
  for (int t = 0; t < 2; ++t) {
    if (!(t ? useq : usep)) continue;
    Jac base;
    base.X = load_fe(pp + 16 * t);
    base.Y = load_fe(pp + 16 * t + 8);
    base.Z = Fe{{1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};
    Jac acc = base;
    tbl_put(ws, 15 * t, acc);
    for (int k = 2; k <= 15; ++k) {
      acc = jac_madd(acc, base.X, base.Y);
      tbl_put(ws, 15 * t + k - 1, acc);
    }
  }
  Jac acc = {};
  if (usep || useq) {
    for (int w = 63; w >= 0; --w) {
      if (!jac_inf(acc)) {
        acc = jac_dbl(acc);
        acc = jac_dbl(acc);
        acc = jac_dbl(acc);
        acc = jac_dbl(acc);
      }
      if (usep) {
        const uint32_t d = nibble(kb, w);
        if (d) acc = jac_add(acc, tbl_get(ws, (int)d - 1));
      }
      if (useq) {
        const uint32_t d = nibble(kc, w);
        if (d) acc = jac_add(acc, tbl_get(ws, 15 + (int)d - 1));
      }
    }
  }
  // + a G: one mixed addition per nonzero byte of a
  for (int j = 0; j < 32; ++j) {
    const uint32_t d = active ? (s[j >> 2] >> ((j & 3) * 8)) & 0xFFu : 0u;
    if (!d) continue;
    const uint32_t* e = gtab + ((size_t)j * 255u + (d - 1u)) * 16u;
    acc = jac_madd(acc, load_fe(e), load_fe(e + 8));
  }
  if (!active) return;
  uint32_t* o = out + (size_t)item * 16u;
  if (jac_inf(acc)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = 0u;
    return;
  }
  const Fe zi = fe_inv(acc.Z), zi2 = fe_sqr(zi), zi3 = fe_mul(zi2, zi);
  const Fe x = fe_mul(acc.X, zi2), y = fe_mul(acc.Y, zi3);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    o[i] = x.v[i];
    o[8 + i] = y.v[i];
  }
}

}  // namespace mpcx

extern "C" __attribute__((visibility("hidden"))) hipError_t mpcx_launch_ec_combine(const uint32_t* sc, const uint32_t* pts,
                                                                        uint32_t* out, const uint32_t* gtab,
                                                                        uint32_t* ws, uint32_t count,
                                                                        hipStream_t st) {
  const uint32_t blocks = (count + 63u) / 64u;
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(mpcx::k_ec_combine, dim3(blocks), dim3(64), 0, st, sc, pts, out, gtab, ws, count);
  return hipGetLastError();
}
