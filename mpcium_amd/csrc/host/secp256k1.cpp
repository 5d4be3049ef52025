// secp256k1.cpp -- see secp256k1.hpp.
#include "secp256k1.hpp"

#include <mutex>
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

Fe fe_sub_p(const Fe& a) {
  Fe r;
  u128 br = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 d = (u128)a[i] - P[i] - br;
    r[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  return r;
}

Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a[i] + b[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  // r + c*2^256: fold the carry (2^256 = PC mod p)
  if (c) {
    u128 t = (u128)r[0] + PC;
    r[0] = (uint64_t)t;
    t >>= 64;
    for (int i = 1; i < 4 && t; ++i) {
      t += r[i];
      r[i] = (uint64_t)t;
      t >>= 64;
    }
  }
  if (fe_geq_p(r)) r = fe_sub_p(r);
  return r;
}

Fe fe_neg(const Fe& a) {
  bool z = !(a[0] | a[1] | a[2] | a[3]);
  if (z) return a;
  Fe r;
  u128 br = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 d = (u128)P[i] - a[i] - br;
    r[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  return r;
}

Fe fe_sub(const Fe& a, const Fe& b) { return fe_add(a, fe_neg(b)); }

// 512-bit t -> t mod p: t = hi*2^256 + lo == hi*PC + lo
Fe fe_reduce512(const uint64_t t[8]) {
  uint64_t r[5];
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)t[4 + i] * PC + t[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  r[4] = (uint64_t)c;  // < 2^34
  Fe o;
  c = (u128)r[4] * PC + r[0];
  o[0] = (uint64_t)c;
  c >>= 64;
  for (int i = 1; i < 4; ++i) {
    c += r[i];
    o[i] = (uint64_t)c;
    c >>= 64;
  }
  if (c) {  // at most one more 2^256 wrap
    u128 s = (u128)o[0] + PC;
    o[0] = (uint64_t)s;
    s >>= 64;
    for (int i = 1; i < 4 && s; ++i) {
      s += o[i];
      o[i] = (uint64_t)s;
      s >>= 64;
    }
  }
  if (fe_geq_p(o)) o = fe_sub_p(o);
  return o;
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

Fe fe_sqr(const Fe& a) { return fe_mul(a, a); }

bool fe_is_zero(const Fe& a) { return !(a[0] | a[1] | a[2] | a[3]); }

// a^(p-2) mod p
Fe fe_inv(const Fe& a) {
  // p - 2 = FFFFFFFF...FFFFFFFE FFFFFC2D
  Fe e = P;
  e[0] -= 2;
  Fe r = {1, 0, 0, 0}, b = a;
  for (int i = 0; i < 256; ++i) {
    if ((e[i / 64] >> (i % 64)) & 1) r = fe_mul(r, b);
    b = fe_sqr(b);
  }
  return r;
}

struct Jac {
  Fe X{}, Y{}, Z{};  // Z == 0: infinity
};

bool jac_inf(const Jac& p) { return fe_is_zero(p.Z); }

Jac jac_dbl(const Jac& p) {
  if (jac_inf(p) || fe_is_zero(p.Y)) return Jac{};
  // a = 0: dbl-2009-l
  const Fe A = fe_sqr(p.X), B = fe_sqr(p.Y), C = fe_sqr(B);
  Fe D = fe_sub(fe_sqr(fe_add(p.X, B)), fe_add(A, C));
  D = fe_add(D, D);
  const Fe E = fe_add(fe_add(A, A), A), F = fe_sqr(E);
  Jac r;
  r.X = fe_sub(F, fe_add(D, D));
  Fe C8 = fe_add(C, C);
  C8 = fe_add(C8, C8);
  C8 = fe_add(C8, C8);
  r.Y = fe_sub(fe_mul(E, fe_sub(D, r.X)), C8);
  const Fe YZ = fe_mul(p.Y, p.Z);
  r.Z = fe_add(YZ, YZ);
  return r;
}

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
  r.X = fe_sub(fe_sub(fe_sqr(Rr), HHH), fe_add(V, V));
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

Affine to_affine(const Jac& j) {
  Affine a;
  if (jac_inf(j)) return a;
  const Fe zi = fe_inv(j.Z), zi2 = fe_sqr(zi);
  a.x = fe_mul(j.X, zi2);
  a.y = fe_mul(j.Y, fe_mul(zi2, zi));
  a.inf = false;
  return a;
}

std::array<uint64_t, 4> scalar_limbs(const Nat& k) {
  const Nat r = k % CurveN();
  std::array<uint64_t, 4> s{};
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

// table[w][d] = d * 16^w * G (Jacobian), w < 64, d < 16
const std::vector<Jac>& base_table() {
  static const std::vector<Jac> t = [] {
    std::vector<Jac> tab(64 * 16);
    Jac b = to_jac(generator());
    for (int w = 0; w < 64; ++w) {
      tab[w * 16] = Jac{};
      tab[w * 16 + 1] = b;
      for (int d = 2; d < 16; ++d) tab[w * 16 + d] = jac_add(tab[w * 16 + d - 1], b);
      for (int i = 0; i < 4; ++i) b = jac_dbl(b);
    }
    return tab;
  }();
  return t;
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

Affine Add(const Affine& a, const Affine& b) { return to_affine(jac_add(to_jac(a), to_jac(b))); }

Affine ScalarBaseMult(const Nat& k) {
  const auto s = scalar_limbs(k);
  const auto& tab = base_table();
  Jac r;
  for (int w = 0; w < 64; ++w) {
    const unsigned d = (unsigned)((s[w / 16] >> (4 * (w % 16))) & 15u);
    if (d) r = jac_add(r, tab[w * 16 + d]);
  }
  return to_affine(r);
}

Affine ScalarMult(const Affine& p, const Nat& k) {
  const auto s = scalar_limbs(k);
  Jac tab[16];
  tab[0] = Jac{};
  tab[1] = to_jac(p);
  for (int d = 2; d < 16; ++d) tab[d] = jac_add(tab[d - 1], tab[1]);
  Jac r;
  for (int w = 63; w >= 0; --w) {
    for (int i = 0; i < 4; ++i) r = jac_dbl(r);
    const unsigned d = (unsigned)((s[w / 16] >> (4 * (w % 16))) & 15u);
    if (d) r = jac_add(r, tab[d]);
  }
  return to_affine(r);
}

}  // namespace mpcx::host::secp
