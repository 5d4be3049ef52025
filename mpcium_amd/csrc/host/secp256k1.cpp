// secp256k1.cpp -- see secp256k1.hpp.
#include "secp256k1.hpp"

#include "hostprof.hpp"
#include "tsscommon.hpp"
#include "mpcx.h"

#include <stdexcept>
#include <string>

#include <algorithm>
#include <vector>

namespace mpcx::host::secp {
namespace {

using u128 = unsigned __int128;

constexpr Fe P = {0xFFFFFFFEFFFFFC2Full, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull};
constexpr uint64_t PC = 0x1000003D1ull;  // 2^256 mod p = 2^32 + 977

bool fe_geq_p(const Fe& a) {
  for (int i = 3; i >= 0; --i)
    if (a[i] != P[i]) return a[i] > P[i];
  return true;
}

// With p = 2^256 - PC, x >= p iff x + PC carries out of 256 bits, and then
// x - p = (x + PC) mod 2^256: the reductions below are branch-free selects.

// r + c*2^256 (c in {0, 1}, r + c*2^256 < 2p) reduced mod p
Fe fe_norm(const Fe& r, uint64_t c) {
  Fe t;
  u128 s = (u128)r[0] + PC;
  t[0] = (uint64_t)s;
  for (int i = 1; i < 4; ++i) {
    s = (u128)r[i] + (uint64_t)(s >> 64);
    t[i] = (uint64_t)s;
  }
  const uint64_t m = 0 - ((uint64_t)(s >> 64) | c);  // all ones: take t
  Fe o;
  for (int i = 0; i < 4; ++i) o[i] = (t[i] & m) | (r[i] & ~m);
  return o;
}

Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)a[i] + b[i] + (uint64_t)(c >> 64);
    r[i] = (uint64_t)c;
  }
  return fe_norm(r, (uint64_t)(c >> 64));
}

// a - b mod p: on borrow add p back, i.e. subtract PC mod 2^256
Fe fe_sub(const Fe& a, const Fe& b) {
  Fe r;
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  const uint64_t k = PC & (0 - br);
  u128 d = (u128)r[0] - k;
  r[0] = (uint64_t)d;
  for (int i = 1; i < 4; ++i) {
    d = (u128)r[i] - ((uint64_t)(d >> 64) & 1);
    r[i] = (uint64_t)d;
  }
  return r;
}

Fe fe_neg(const Fe& a) { return fe_sub(Fe{0, 0, 0, 0}, a); }
Fe fe_dbl(const Fe& a) { return fe_add(a, a); }

// 512-bit t -> t mod p: t = hi*2^256 + lo == hi*PC + lo
Fe fe_reduce512(const uint64_t t[8]) {
  uint64_t r[4];
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c = (u128)t[4 + i] * PC + t[i] + (uint64_t)(c >> 64);
    r[i] = (uint64_t)c;
  }
  // r + h*2^256, h < 2^34: fold h*PC (< 2^67) once more
  const u128 hp = (u128)(uint64_t)(c >> 64) * PC;
  Fe o;
  u128 s = (u128)r[0] + (uint64_t)hp;
  o[0] = (uint64_t)s;
  s = (u128)r[1] + (uint64_t)(hp >> 64) + (uint64_t)(s >> 64);
  o[1] = (uint64_t)s;
  for (int i = 2; i < 4; ++i) {
    s = (u128)r[i] + (uint64_t)(s >> 64);
    o[i] = (uint64_t)s;
  }
  // o + carry*2^256 < 2p (the carry leaves o tiny)
  return fe_norm(o, (uint64_t)(s >> 64));
}

Fe fe_mul(const Fe& a, const Fe& b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a[i] * b[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  return fe_reduce512(t);
}

// 10 limb products: the 6 cross products once, doubled, plus the 4 squares
Fe fe_sqr(const Fe& a) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 3; ++i) {
    u128 c = 0;
    for (int j = i + 1; j < 4; ++j) {
      c += (u128)a[i] * a[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  uint64_t top = 0;  // sum of cross products < a^2 / 2 < 2^511: doubling cannot overflow
  for (int k = 0; k < 8; ++k) {
    const uint64_t v = t[k];
    t[k] = (v << 1) | top;
    top = v >> 63;
  }
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 sq = (u128)a[i] * a[i];
    c += (u128)t[2 * i] + (uint64_t)sq;
    t[2 * i] = (uint64_t)c;
    c >>= 64;
    c += (u128)t[2 * i + 1] + (uint64_t)(sq >> 64);
    t[2 * i + 1] = (uint64_t)c;
    c >>= 64;
  }
  return fe_reduce512(t);
}

Fe fe_sqr_n(Fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sqr(a);
  return a;
}

bool fe_is_zero(const Fe& a) { return !(a[0] | a[1] | a[2] | a[3]); }

// a^(p-2) mod p. p - 2 in binary: 223 ones, a zero, 22 ones, then 0000101101;
// the chain builds a^(2^k - 1) for k = 2, 3, 6, 9, 11, 22, 44, 88, 176, 220,
// 223 and appends the tail: 255 squarings, 15 multiplications.
Fe fe_inv(const Fe& a) {
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
  Fe t = fe_mul(fe_sqr_n(x223, 23), x22);  // ...1 0 (22 ones)
  t = fe_mul(fe_sqr_n(t, 5), a);           // 00001
  t = fe_mul(fe_sqr_n(t, 3), x2);          // 011
  return fe_mul(fe_sqr_n(t, 2), a);        // 01
}

struct Jac {
  Fe X{}, Y{}, Z{};  // Z == 0: infinity
};

bool jac_inf(const Jac& p) { return fe_is_zero(p.Z); }

Jac jac_neg(const Jac& p) { return Jac{p.X, fe_neg(p.Y), p.Z}; }

// a = 0: dbl-2009-l (2M + 5S)
Jac jac_dbl(const Jac& p) {
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

// add-2007-bl (11M + 5S)
Jac jac_add(const Jac& p, const Jac& q) {
  if (jac_inf(p)) return q;
  if (jac_inf(q)) return p;
  const Fe Z1Z1 = fe_sqr(p.Z), Z2Z2 = fe_sqr(q.Z);
  const Fe U1 = fe_mul(p.X, Z2Z2), U2 = fe_mul(q.X, Z1Z1);
  const Fe S1 = fe_mul(fe_mul(p.Y, q.Z), Z2Z2), S2 = fe_mul(fe_mul(q.Y, p.Z), Z1Z1);
  const Fe H = fe_sub(U2, U1), Rr = fe_sub(S2, S1);
  if (fe_is_zero(H)) {
    if (fe_is_zero(Rr)) return jac_dbl(p);
    return Jac{};
  }
  const Fe HH = fe_sqr(H), HHH = fe_mul(H, HH), V = fe_mul(U1, HH);
  Jac r;
  r.X = fe_sub(fe_sub(fe_sqr(Rr), HHH), fe_dbl(V));
  r.Y = fe_sub(fe_mul(Rr, fe_sub(V, r.X)), fe_mul(S1, HHH));
  r.Z = fe_mul(fe_mul(p.Z, q.Z), H);
  return r;
}

Jac to_jac(const Affine& a) {
  Jac j;
  if (a.inf) return j;
  j.X = a.x;
  j.Y = a.y;
  j.Z = {1, 0, 0, 0};
  return j;
}

// Jacobian + affine q (q not infinity): madd-2007-bl (7M + 4S)
Jac jac_madd(const Jac& p, const Affine& q) {
  if (jac_inf(p)) return to_jac(q);
  const Fe Z1Z1 = fe_sqr(p.Z);
  const Fe U2 = fe_mul(q.x, Z1Z1), S2 = fe_mul(q.y, fe_mul(p.Z, Z1Z1));
  const Fe H = fe_sub(U2, p.X), r0 = fe_sub(S2, p.Y);
  if (fe_is_zero(H)) {
    if (fe_is_zero(r0)) return jac_dbl(p);
    return Jac{};
  }
  const Fe HH = fe_sqr(H), I = fe_dbl(fe_dbl(HH)), J = fe_mul(H, I);
  const Fe r = fe_dbl(r0), V = fe_mul(p.X, I);
  Jac o;
  o.X = fe_sub(fe_sub(fe_sqr(r), J), fe_dbl(V));
  o.Y = fe_sub(fe_mul(r, fe_sub(V, o.X)), fe_dbl(fe_mul(p.Y, J)));
  o.Z = fe_sub(fe_sub(fe_sqr(fe_add(p.Z, H)), Z1Z1), HH);
  return o;
}

Affine to_affine(const Jac& j) {
  Affine a;
  if (jac_inf(j)) return a;
  const Fe zi = fe_inv(j.Z), zi2 = fe_sqr(zi);
  a.x = fe_mul(j.X, zi2);
  a.y = fe_mul(j.Y, fe_mul(zi2, zi));
  a.inf = false;
  return a;
}

using Scalar = std::array<uint64_t, 4>;

Scalar scalar_limbs(const Nat& k) {
  const Nat r = k < CurveN() ? k : k % CurveN();
  Scalar s{};
  const auto& w = r.limbs();
  for (size_t i = 0; i < w.size() && i < 8; ++i) s[i / 2] |= (uint64_t)w[i] << (32 * (i % 2));
  return s;
}

const Affine& generator() {
  static const Affine g = [] {
    Affine a;
    a.x = NatToFe(Nat::from_hex("79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798"));
    a.y = NatToFe(Nat::from_hex("483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8"));
    a.inf = false;
    return a;
  }();
  return g;
}

// Fixed-base table: entry [w][d - 1] = d * 256^w * G in affine form, w < 32,
// 1 <= d <= 255 (522 KB), so k*G is at most 32 mixed additions. Built once;
// the affine conversion shares one inversion (Montgomery's batch trick).
constexpr int kBaseWindows = 32, kBaseDigits = 255;
const std::vector<Affine>& base_table() {
  static const std::vector<Affine> t = [] {
    const size_t n = (size_t)kBaseWindows * kBaseDigits;
    std::vector<Jac> jt(n);
    Jac b = to_jac(generator());
    for (int w = 0; w < kBaseWindows; ++w) {
      Jac* row = &jt[(size_t)w * kBaseDigits];
      row[0] = b;
      for (int d = 1; d < kBaseDigits; ++d) row[d] = jac_add(row[d - 1], b);
      for (int i = 0; i < 8; ++i) b = jac_dbl(b);
    }
    // batch inversion of every Z (none is zero: d * 256^w < n)
    std::vector<Fe> pre(n);
    Fe acc = {1, 0, 0, 0};
    for (size_t i = 0; i < n; ++i) {
      pre[i] = acc;
      acc = fe_mul(acc, jt[i].Z);
    }
    Fe inv = fe_inv(acc);
    std::vector<Affine> out(n);
    for (size_t i = n; i-- > 0;) {
      const Fe zi = fe_mul(inv, pre[i]);  // 1 / Z_i
      inv = fe_mul(inv, jt[i].Z);
      const Fe zi2 = fe_sqr(zi);
      out[i].x = fe_mul(jt[i].X, zi2);
      out[i].y = fe_mul(jt[i].Y, fe_mul(zi2, zi));
      out[i].inf = false;
    }
    return out;
  }();
  return t;
}

// acc + s*G (s < n) by the fixed-base table
Jac add_base_mult(Jac acc, const Scalar& s) {
  const auto& tab = base_table();
  for (int w = 0; w < kBaseWindows; ++w) {
    const unsigned d = (unsigned)((s[w / 8] >> (8 * (w % 8))) & 0xFFu);
    if (d) acc = jac_madd(acc, tab[(size_t)w * kBaseDigits + d - 1]);
  }
  return acc;
}

// width-5 NAF of s (< 2^256): digits in {0, +-1, +-3, ..., +-15}; returns length
int wnaf5(const Scalar& s, int8_t out[258]) {
  uint64_t k[5] = {s[0], s[1], s[2], s[3], 0};
  int len = 0;
  auto nonzero = [&] { return (k[0] | k[1] | k[2] | k[3] | k[4]) != 0; };
  while (nonzero()) {
    int d = 0;
    if (k[0] & 1) {
      d = (int)(k[0] & 31);
      if (d >= 16) d -= 32;
      if (d > 0) {  // k -= d
        u128 br = (u128)k[0] - (uint64_t)d;
        k[0] = (uint64_t)br;
        for (int i = 1; i < 5 && (br >> 64); ++i) {
          br = (u128)k[i] - 1;
          k[i] = (uint64_t)br;
        }
      } else {  // k += -d
        u128 c = (u128)k[0] + (uint64_t)(-d);
        k[0] = (uint64_t)c;
        for (int i = 1; i < 5 && (c >> 64); ++i) {
          c = (u128)k[i] + 1;
          k[i] = (uint64_t)c;
        }
      }
    }
    out[len++] = (int8_t)d;
    for (int i = 0; i < 4; ++i) k[i] = (k[i] >> 1) | (k[i + 1] << 63);
    k[4] >>= 1;
  }
  return len;
}

// GLV endomorphism: lambda*(x, y) = (beta*x, y) with lambda^3 = 1 (mod n),
// beta^3 = 1 (mod p). k = k1 + k2*lambda (mod n) with |k1|, |k2| <= ~2^128 from
// the reduced lattice basis (a1, b1), (a2, b2): c1 = round(b2 k / n),
// c2 = round(-b1 k / n), k1 = k - c1 a1 - c2 a2, k2 = -c1 b1 - c2 b2 (any c1,
// c2 satisfy k1 + k2 lambda = k mod n; the rounding only keeps them short).
// Constants checked by tests/test_mta_cpu.py (lambda*G against the oracle).
struct Glv {
  Fe beta;
  Nat a1, b1abs, a2, n_half;  // b1 < 0, b2 = a1
};
const Glv& glv() {
  static const Glv g = [] {
    Glv v;
    v.beta = NatToFe(Nat::from_hex("7ae96a2b657c07106e64479eac3434e99cf0497512f58995c1396c28719501ee"));
    v.a1 = Nat::from_hex("3086d221a7d46bcde86c90e49284eb15");
    v.b1abs = Nat::from_hex("e4437ed6010e88286f547fa90abfe4c3");
    v.a2 = Nat::from_hex("114ca50f7a8e2f3f657c1108d9d44cfd8");
    v.n_half = CurveN() >> 1;
    return v;
  }();
  return g;
}

Scalar limbs_of(const Nat& r) {
  Scalar s{};
  const auto& w = r.limbs();
  for (size_t i = 0; i < w.size() && i < 8; ++i) s[i / 2] |= (uint64_t)w[i] << (32 * (i % 2));
  return s;
}

// k = k1 + k2*lambda: magnitudes and signs
void glv_split(const Nat& k, Nat* k1, bool* neg1, Nat* k2, bool* neg2) {
  const Glv& g = glv();
  const Nat& n = CurveN();
  const Nat c1 = (g.a1 * k + g.n_half) / n;     // round(b2 k / n), b2 = a1
  const Nat c2 = (g.b1abs * k + g.n_half) / n;  // round(-b1 k / n)
  const Nat sub = c1 * g.a1 + c2 * g.a2;         // k1 = k - sub
  if (k >= sub) {
    *k1 = k - sub;
    *neg1 = false;
  } else {
    *k1 = sub - k;
    *neg1 = true;
  }
  const Nat pos = c1 * g.b1abs, neg = c2 * g.a1;  // k2 = c1 |b1| - c2 b2
  if (pos >= neg) {
    *k2 = pos - neg;
    *neg2 = false;
  } else {
    *k2 = neg - pos;
    *neg2 = true;
  }
}

// s*p for a variable point (Jacobian result): GLV split, then one doubling
// chain over both halves' width-5 NAFs (odd multiples p, 3p, ..., 15p and
// their lambda images)
Jac var_mult(const Affine& p, const Scalar& s) {
  if (p.inf) return Jac{};
  uint32_t w[8];
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = (uint32_t)s[i];
    w[2 * i + 1] = (uint32_t)(s[i] >> 32);
  }
  Nat k1, k2;
  bool neg1, neg2;
  glv_split(Nat::from_words(w, 8), &k1, &neg1, &k2, &neg2);
  int8_t naf1[258], naf2[258];
  const int len1 = wnaf5(limbs_of(k1), naf1), len2 = wnaf5(limbs_of(k2), naf2);
  Jac odd[8], lodd[8];
  odd[0] = to_jac(p);
  if (neg1) odd[0] = jac_neg(odd[0]);
  const Jac p2 = jac_dbl(odd[0]);
  for (int i = 1; i < 8; ++i) odd[i] = jac_add(odd[i - 1], p2);
  const Fe beta = glv().beta;
  for (int i = 0; i < 8; ++i) {  // lambda * (odd multiple of +-p), sign fixed for k2
    lodd[i] = Jac{fe_mul(odd[i].X, beta), odd[i].Y, odd[i].Z};
    if (neg1 != neg2) lodd[i] = jac_neg(lodd[i]);
  }
  Jac r;
  for (int i = std::max(len1, len2) - 1; i >= 0; --i) {
    r = jac_dbl(r);
    const int d1 = i < len1 ? naf1[i] : 0, d2 = i < len2 ? naf2[i] : 0;
    if (d1 > 0) r = jac_add(r, odd[d1 / 2]);
    else if (d1 < 0) r = jac_add(r, jac_neg(odd[(-d1) / 2]));
    if (d2 > 0) r = jac_add(r, lodd[d2 / 2]);
    else if (d2 < 0) r = jac_add(r, jac_neg(lodd[(-d2) / 2]));
  }
  return r;
}

}  // namespace

const Nat& CurveN() {
  static const Nat n = Nat::from_hex("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141");
  return n;
}

Nat FeToNat(const Fe& a) {
  uint32_t w[8];
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = (uint32_t)a[i];
    w[2 * i + 1] = (uint32_t)(a[i] >> 32);
  }
  return Nat::from_words(w, 8);
}

Fe NatToFe(const Nat& a) {
  Fe f{};
  const auto& w = a.limbs();
  for (size_t i = 0; i < w.size() && i < 8; ++i) f[i / 2] |= (uint64_t)w[i] << (32 * (i % 2));
  return f;
}

bool IsOnCurve(const Affine& p) {
  if (p.inf) return false;
  if (fe_geq_p(p.x) || fe_geq_p(p.y)) return false;
  const Fe lhs = fe_sqr(p.y);
  const Fe rhs = fe_add(fe_mul(fe_sqr(p.x), p.x), Fe{7, 0, 0, 0});
  return lhs == rhs;
}

bool Equal(const Affine& a, const Affine& b) {
  if (a.inf || b.inf) return a.inf == b.inf;
  return a.x == b.x && a.y == b.y;
}

Affine Add(const Affine& a, const Affine& b) {
  if (b.inf) return a;
  return to_affine(jac_madd(to_jac(a), b));
}

Affine ScalarBaseMult(const Nat& k) {
  MPCX_PROF("ec.base_mult");
  return to_affine(add_base_mult(Jac{}, scalar_limbs(k)));
}

Affine ScalarMult(const Affine& p, const Nat& k) {
  MPCX_PROF("ec.var_mult");
  return to_affine(var_mult(p, scalar_limbs(k)));
}

Affine LinComb(const Nat& u1, const Affine& X, const Nat& u2) {
  MPCX_PROF("ec.lincomb");
  return to_affine(add_base_mult(var_mult(X, scalar_limbs(u2)), scalar_limbs(u1)));
}

const Affine& Generator() { return generator(); }

const Nat& FieldP() {
  static const Nat p = Nat::from_hex("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F");
  return p;
}

Affine Combine(const Nat& a, const Affine& P, const Nat& b, const Affine& Q, const Nat& c) {
  MPCX_PROF("ec.combine");
  Jac acc;
  if (!b.is_zero() && !P.inf) acc = var_mult(P, scalar_limbs(b));
  if (!c.is_zero() && !Q.inf) acc = jac_add(acc, var_mult(Q, scalar_limbs(c)));
  if (!a.is_zero()) acc = add_base_mult(acc, scalar_limbs(a));
  return to_affine(acc);
}

std::vector<Affine> CombineBatch(const std::vector<Comb>& items) {
  MPCX_TRACE("gpu.ec", items.size());
  MPCX_PROF("ec.combine_batch");
  const size_t n = items.size();
  std::vector<Affine> out(n);
  if (!n) return out;
  // one GPU thread per item (mpcx_ec_combine_batch, libmpcx's k_ec_combine)
  std::vector<uint32_t> sc(n * 24, 0), pt(n * 32, 0), res(n * 16, 0);
  auto put_scalar = [&](const Nat& k, uint32_t* w) {
    if (k.bit_len() > 256) (k % CurveN()).to_words(w, 8);
    else k.to_words(w, 8);
  };
  auto put_point = [&](const Affine& p, uint32_t* w) {
    if (p.inf) return;  // all zero = infinity
    FeToNat(p.x).to_words(w, 8);
    FeToNat(p.y).to_words(w + 8, 8);
  };
  parallel_for((n + 255) / 256, [&](size_t blk) {
    for (size_t i = blk * 256; i < std::min(n, blk * 256 + 256); ++i) {
      const Comb& t = items[i];
      put_scalar(t.a, &sc[i * 24]);
      put_scalar(t.b, &sc[i * 24 + 8]);
      put_scalar(t.c, &sc[i * 24 + 16]);
      put_point(t.P, &pt[i * 32]);
      put_point(t.Q, &pt[i * 32 + 16]);
    }
  });
  const int rc = mpcx_ec_combine_batch((uint32_t)n, sc.data(), pt.data(), res.data());
  if (rc != MPCX_OK) throw std::runtime_error(std::string("mpcx_ec_combine_batch: ") + mpcx_last_error());
  parallel_for((n + 255) / 256, [&](size_t blk) {
    for (size_t i = blk * 256; i < std::min(n, blk * 256 + 256); ++i) {
      const uint32_t* w = &res[i * 16];
      uint32_t o = 0;
      for (int k = 0; k < 16; ++k) o |= w[k];
      if (!o) continue;  // infinity
      out[i].x = NatToFe(Nat::from_words(w, 8));
      out[i].y = NatToFe(Nat::from_words(w + 8, 8));
      out[i].inf = false;
    }
  });
  return out;
}

}  // namespace mpcx::host::secp
