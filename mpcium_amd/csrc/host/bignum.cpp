// bignum.cpp -- see bignum.hpp.
#include "bignum.hpp"

#include "hostprof.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace mpcx::host {

Nat::Nat(uint64_t v) {
  if (v) w_.push_back((uint32_t)v);
  if (v >> 32) w_.push_back((uint32_t)(v >> 32));
}

void Nat::norm() {
  while (!w_.empty() && w_.back() == 0) w_.pop_back();
}

Nat Nat::from_words(const uint32_t* w, size_t n) {
  Nat r;
  r.w_.assign(w, w + n);
  r.norm();
  return r;
}

void Nat::set_words(const uint32_t* w, size_t n) {
  while (n && !w[n - 1]) --n;
  w_.assign(w, w + n);
}

Nat Nat::from_bytes_be(const uint8_t* b, size_t n) {
  Nat r;
  r.w_.assign((n + 3) / 4, 0);
  for (size_t i = 0; i < n; ++i) {
    const size_t pos = n - 1 - i;  // byte significance
    r.w_[pos / 4] |= (uint32_t)b[i] << (8 * (pos % 4));
  }
  r.norm();
  return r;
}

Nat Nat::from_hex(const std::string& s) {
  Nat r;
  for (char c : s) {
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else throw std::invalid_argument("bad hex digit");
    r = (r << 4) + Nat((uint64_t)d);
  }
  return r;
}

std::vector<uint8_t> Nat::to_bytes_be() const {
  std::vector<uint8_t> out;
  const uint32_t nb = (bit_len() + 7) / 8;
  out.resize(nb);
  for (uint32_t i = 0; i < nb; ++i) out[nb - 1 - i] = (uint8_t)(w_[i / 4] >> (8 * (i % 4)));
  return out;
}

void Nat::to_words(uint32_t* out, size_t n) const {
  if (w_.size() > n) throw std::length_error("Nat::to_words: value does not fit");
  std::fill(out, out + n, 0u);
  std::copy(w_.begin(), w_.end(), out);
}

std::string Nat::to_hex() const {
  if (w_.empty()) return "0";
  static const char* hx = "0123456789abcdef";
  std::string s;
  for (int i = (int)w_.size() - 1; i >= 0; --i)
    for (int sh = 28; sh >= 0; sh -= 4) s.push_back(hx[(w_[i] >> sh) & 15]);
  size_t nz = s.find_first_not_of('0');
  return s.substr(nz);
}

uint32_t Nat::bit_len() const {
  if (w_.empty()) return 0;
  return (uint32_t)(32 * (w_.size() - 1) + (32 - __builtin_clz(w_.back())));
}

bool Nat::bit(uint32_t i) const {
  const size_t wi = i / 32;
  return wi < w_.size() && ((w_[wi] >> (i % 32)) & 1u);
}

uint64_t Nat::low64() const {
  uint64_t v = w_.empty() ? 0 : w_[0];
  if (w_.size() > 1) v |= (uint64_t)w_[1] << 32;
  return v;
}

int cmp(const Nat& a, const Nat& b) {
  if (a.w_.size() != b.w_.size()) return a.w_.size() < b.w_.size() ? -1 : 1;
  for (int i = (int)a.w_.size() - 1; i >= 0; --i)
    if (a.w_[i] != b.w_[i]) return a.w_[i] < b.w_[i] ? -1 : 1;
  return 0;
}

Nat operator+(const Nat& a, const Nat& b) {
  const Nat& x = a.w_.size() >= b.w_.size() ? a : b;
  const Nat& y = a.w_.size() >= b.w_.size() ? b : a;
  Nat r;
  r.w_.resize(x.w_.size() + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < x.w_.size(); ++i) {
    c += (uint64_t)x.w_[i] + (i < y.w_.size() ? y.w_[i] : 0u);
    r.w_[i] = (uint32_t)c;
    c >>= 32;
  }
  r.w_[x.w_.size()] = (uint32_t)c;
  r.norm();
  return r;
}

Nat operator-(const Nat& a, const Nat& b) {
  if (cmp(a, b) < 0) throw std::domain_error("Nat subtraction underflow");
  Nat r;
  r.w_.resize(a.w_.size());
  int64_t br = 0;
  for (size_t i = 0; i < a.w_.size(); ++i) {
    int64_t d = (int64_t)a.w_[i] - (i < b.w_.size() ? b.w_[i] : 0u) + br;
    r.w_[i] = (uint32_t)d;
    br = d >> 32;
  }
  r.norm();
  return r;
}

namespace {
using u128 = unsigned __int128;

// 64-bit limb view of a normalized word vector: ceil(n / 2) limbs (x86-64 is
// little-endian, so word pairs are the limbs; an odd top word is zero-padded)
inline size_t limbs64(size_t n32) { return (n32 + 1) / 2; }
inline void load64(const std::vector<uint32_t>& w, uint64_t* out) {
  const size_t n = w.size();
  if (!n) return;
  out[(n - 1) / 2] = 0;
  std::memcpy(out, w.data(), n * 4);
}
// words [0, n32) of a limb array into a normalized word vector
inline void store64(const uint64_t* l, size_t n32, std::vector<uint32_t>* w) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(l);
  while (n32 && !p[n32 - 1]) --n32;
  w->assign(p, p + n32);
}

// Per-thread scratch limbs: the protocol mirrors run millions of products and
// reductions from the host pool, so no allocation per operation.
uint64_t* scratch(size_t n) {
  thread_local std::vector<uint64_t> buf;
  if (buf.size() < n) buf.resize(std::max<size_t>(n, 2 * buf.size()));
  return buf.data();
}

// r[0, na + nb) = a * b (schoolbook on 64-bit limbs, mulx chains)
void mul_limbs(const uint64_t* a, size_t na, const uint64_t* b, size_t nb, uint64_t* r) {
  std::fill(r, r + na + nb, 0ull);
  for (size_t i = 0; i < nb; ++i) {
    const uint64_t bi = b[i];
    if (!bi) continue;
    uint64_t c = 0;
    uint64_t* ri = r + i;
    for (size_t j = 0; j < na; ++j) {
      const u128 t = (u128)a[j] * bi + ri[j] + c;
      ri[j] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
    ri[na] = c;
  }
}
}  // namespace

Nat operator*(const Nat& a, const Nat& b) {
  Nat r;
  if (a.is_zero() || b.is_zero()) return r;
  const size_t na = limbs64(a.w_.size()), nb = limbs64(b.w_.size());
  uint64_t* s = scratch(2 * (na + nb));
  uint64_t *x = s, *y = s + na, *z = s + na + nb;
  load64(a.w_, x);
  load64(b.w_, y);
  if (na >= nb) mul_limbs(x, na, y, nb, z);
  else mul_limbs(y, nb, x, na, z);
  store64(z, a.w_.size() + b.w_.size(), &r.w_);
  return r;
}

Nat operator<<(const Nat& a, uint32_t s) {
  if (a.is_zero()) return a;
  Nat r;
  const uint32_t ws = s / 32, bs = s % 32;
  r.w_.assign(a.w_.size() + ws + 1, 0);
  for (size_t i = 0; i < a.w_.size(); ++i) {
    r.w_[i + ws] |= a.w_[i] << bs;
    if (bs) r.w_[i + ws + 1] |= a.w_[i] >> (32 - bs);
  }
  r.norm();
  return r;
}

Nat operator>>(const Nat& a, uint32_t s) {
  const uint32_t ws = s / 32, bs = s % 32;
  Nat r;
  if (ws >= a.w_.size()) return r;
  r.w_.assign(a.w_.size() - ws, 0);
  for (size_t i = 0; i < r.w_.size(); ++i) {
    r.w_[i] = a.w_[i + ws] >> bs;
    if (bs && i + ws + 1 < a.w_.size()) r.w_[i] |= a.w_[i + ws + 1] << (32 - bs);
  }
  r.norm();
  return r;
}

uint32_t Nat::mod_u32(uint32_t m) const {
  uint64_t r = 0;
  for (int i = (int)w_.size() - 1; i >= 0; --i) r = ((r << 32) | w_[i]) % m;
  return (uint32_t)r;
}

// Knuth, TAOCP vol. 2, 4.3.1, Algorithm D, on 64-bit limbs (128-bit trial
// quotients).
void Nat::divmod(const Nat& u, const Nat& v, Nat* q, Nat* r) {
  if (v.is_zero()) throw std::domain_error("division by zero");
  if (cmp(u, v) < 0) {
    if (q) *q = Nat();
    if (r) *r = u;
    return;
  }
  const size_t nu = limbs64(u.w_.size()), n = limbs64(v.w_.size()), m = nu - n;
  uint64_t* s = scratch(nu + 1 + n + (m + 1) + nu);
  uint64_t *un = s, *vn = s + nu + 1, *qq = vn + n, *tmp = qq + m + 1;
  if (n == 1) {
    load64(u.w_, tmp);
    load64(v.w_, vn);
    const uint64_t d = vn[0];
    u128 rem = 0;
    for (size_t i = nu; i-- > 0;) {
      const u128 cur = (rem << 64) | tmp[i];
      qq[i] = (uint64_t)(cur / d);
      rem = cur % d;
    }
    if (q) store64(qq, 2 * nu, &q->w_);
    if (r) *r = Nat((uint64_t)rem);
    return;
  }
  load64(v.w_, vn);
  load64(u.w_, tmp);
  const int sh = __builtin_clzll(vn[n - 1]);
  if (sh) {
    for (size_t i = n - 1; i > 0; --i) vn[i] = (vn[i] << sh) | (vn[i - 1] >> (64 - sh));
    vn[0] <<= sh;
    un[nu] = tmp[nu - 1] >> (64 - sh);
    for (size_t i = nu - 1; i > 0; --i) un[i] = (tmp[i] << sh) | (tmp[i - 1] >> (64 - sh));
    un[0] = tmp[0] << sh;
  } else {
    std::memcpy(un, tmp, nu * 8);
    un[nu] = 0;
  }
  const uint64_t vt = vn[n - 1], vs = vn[n - 2];
  for (size_t j = m + 1; j-- > 0;) {
    // trial quotient from the top two limbs, corrected by the third (at most
    // two decrements; then at most one add-back below)
    const u128 num = ((u128)un[j + n] << 64) | un[j + n - 1];
    u128 qhat = num / vt, rhat = num % vt;
    while ((qhat >> 64) || (u128)(uint64_t)qhat * vs > ((rhat << 64) | un[j + n - 2])) {
      --qhat;
      rhat += vt;
      if (rhat >> 64) break;
    }
    const uint64_t qh = (uint64_t)qhat;
    uint64_t mc = 0, br = 0;
    for (size_t i = 0; i < n; ++i) {
      const u128 p = (u128)qh * vn[i] + mc;
      mc = (uint64_t)(p >> 64);
      const uint64_t pl = (uint64_t)p, ui = un[i + j];
      const uint64_t d = ui - pl - br;
      br = (ui < pl || (ui - pl) < br) ? 1u : 0u;
      un[i + j] = d;
    }
    const uint64_t top = un[j + n];
    const uint64_t d = top - mc - br;
    const bool neg = top < mc || (top - mc) < br;
    un[j + n] = d;
    qq[j] = qh;
    if (neg) {  // qhat was one too large: add v back
      --qq[j];
      uint64_t c = 0;
      for (size_t i = 0; i < n; ++i) {
        const u128 t = (u128)un[i + j] + vn[i] + c;
        un[i + j] = (uint64_t)t;
        c = (uint64_t)(t >> 64);
      }
      un[j + n] += c;
    }
  }
  if (q) store64(qq, 2 * (m + 1), &q->w_);
  if (r) {
    for (size_t i = 0; i < n; ++i) tmp[i] = sh ? (un[i] >> sh) | (un[i + 1] << (64 - sh)) : un[i];
    store64(tmp, 2 * n, &r->w_);
  }
}

Nat operator/(const Nat& a, const Nat& b) {
  Nat q;
  Nat::divmod(a, b, &q, nullptr);
  return q;
}

Nat operator%(const Nat& a, const Nat& b) {
  Nat r;
  Nat::divmod(a, b, nullptr, &r);
  return r;
}

Nat gcd(Nat a, Nat b) {
  while (!b.is_zero()) {
    Nat r = a % b;
    a = b;
    b = r;
  }
  return a;
}

Nat mod_signed(const Int& x, const Nat& m) {
  Nat r = x.mag % m;
  if (x.neg && !r.is_zero()) r = m - r;
  return r;
}

bool mod_inverse(const Int& g, const Nat& n, Nat* out) {
  if (n.is_zero()) return false;
  Nat a = mod_signed(g, n);
  if (n == Nat(1)) {
    *out = Nat();
    return true;
  }
  // extended Euclid with sign-tracked coefficients: s0*a == r0 (mod n)
  Nat r0 = n, r1 = a;
  Int s0(Nat(), false), s1(Nat(1), false);
  while (!r1.is_zero()) {
    Nat q, r;
    Nat::divmod(r0, r1, &q, &r);
    // s2 = s0 - q*s1
    Nat qs = q * s1.mag;
    Int s2;
    if (s0.neg == !s1.neg) {  // s0 and -q*s1 have the same sign
      s2 = Int(s0.mag + qs, s0.neg);
    } else if (cmp(s0.mag, qs) >= 0) {
      s2 = Int(s0.mag - qs, s0.neg);
    } else {
      s2 = Int(qs - s0.mag, !s0.neg);
    }
    r0 = r1;
    r1 = r;
    s0 = s1;
    s1 = s2;
  }
  if (r0 != Nat(1)) return false;
  *out = mod_signed(s0, n);
  return true;
}

}  // namespace mpcx::host

namespace mpcx::host {
namespace {

using V64 = std::vector<uint64_t>;

V64 to64(const Nat& a) {
  const auto& w = a.limbs();
  V64 r((w.size() + 1) / 2, 0);
  for (size_t i = 0; i < w.size(); ++i) r[i / 2] |= (uint64_t)w[i] << (32 * (i % 2));
  while (!r.empty() && r.back() == 0) r.pop_back();
  return r;
}

int cmp64(const V64& a, const V64& b) {
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  for (size_t i = a.size(); i-- > 0;)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}

// a -= b (a > b), then a >>= ctz(a), trimmed
void sub_shift(V64& a, const V64& b) {
  unsigned __int128 br = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    const unsigned __int128 d = (unsigned __int128)a[i] - (i < b.size() ? b[i] : 0) - br;
    a[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  size_t z = 0;
  while (z < a.size() && a[z] == 0) ++z;
  if (z) a.erase(a.begin(), a.begin() + (long)z);
  const int s = __builtin_ctzll(a[0]);
  if (s) {
    for (size_t i = 0; i + 1 < a.size(); ++i) a[i] = (a[i] >> s) | (a[i + 1] << (64 - s));
    a.back() >>= s;
  }
  while (!a.empty() && a.back() == 0) a.pop_back();
}

}  // namespace

namespace {

constexpr size_t kGcdMaxWords = 128;  // 8192-bit operands on the batched path

size_t bitlen64(const uint64_t* a, size_t n) {
  for (size_t i = n; i-- > 0;)
    if (a[i]) return i * 64 + 64 - (size_t)__builtin_clzll(a[i]);
  return 0;
}

// bits [nb-64, nb) of a (nb >= 64)
uint64_t top64(const uint64_t* a, size_t nb) {
  const size_t lo = nb - 64, w = lo / 64, s = lo % 64;
  return s ? (a[w] >> s) | (a[w + 1] << (64 - s)) : a[w];
}

// out = |a f + b g| / 2^31 (the combination is divisible by 2^31 by
// construction); n words in, n words out
void lincomb_shift31(const uint64_t* a, const uint64_t* b, size_t n, int64_t f, int64_t g, uint64_t* out) {
  uint64_t t[kGcdMaxWords + 1];
  __int128 carry = 0;
  for (size_t i = 0; i < n; ++i) {
    const __int128 v = carry + (__int128)a[i] * f + (__int128)b[i] * g;
    t[i] = (uint64_t)v;
    carry = v >> 64;
  }
  t[n] = (uint64_t)carry;
  if (carry < 0) {  // two's complement negate
    unsigned __int128 c = 1;
    for (size_t i = 0; i <= n; ++i) {
      c += (uint64_t)~t[i];
      t[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  for (size_t i = 0; i < n; ++i) out[i] = (t[i] >> 31) | (t[i + 1] << 33);
}

// plain binary GCD of u and odd v (word arrays of n words): gcd == 1?
bool coprime_binary(V64 u, V64 v) {
  while (!u.empty() && u.back() == 0) u.pop_back();
  while (!v.empty() && v.back() == 0) v.pop_back();
  if (u.empty()) return v.size() == 1 && v[0] == 1;
  {
    size_t z = 0;
    while (u[z] == 0) ++z;
    u.erase(u.begin(), u.begin() + (long)z);
    const int s = __builtin_ctzll(u[0]);
    if (s) {
      for (size_t i = 0; i + 1 < u.size(); ++i) u[i] = (u[i] >> s) | (u[i + 1] << (64 - s));
      u.back() >>= s;
    }
    while (!u.empty() && u.back() == 0) u.pop_back();
  }
  for (;;) {
    if (u.size() == 1 && v.size() == 1) {
      uint64_t a64 = u[0], b64 = v[0];
      while (a64 != b64) {
        if (a64 > b64) {
          a64 -= b64;
          a64 >>= __builtin_ctzll(a64);
        } else {
          b64 -= a64;
          b64 >>= __builtin_ctzll(b64);
        }
      }
      return a64 == 1;
    }
    const int c = cmp64(u, v);
    if (c == 0) return u.size() == 1 && u[0] == 1;
    if (c > 0) sub_shift(u, v);
    else sub_shift(v, u);
  }
}

}  // namespace

bool coprime_odd(const Nat& x, const Nat& m) {
  MPCX_PROF("gcd.coprime_odd");
  if (m.is_zero() || !m.is_odd()) throw std::invalid_argument("coprime_odd: modulus must be odd");
  if (m == Nat(1)) return true;
  const Nat a = x >= m ? x % m : x;
  if (a.is_zero()) return false;
  V64 u = to64(a), v = to64(m);
  const size_t n = v.size();
  if (n > kGcdMaxWords) return coprime_binary(u, v);
  u.resize(n, 0);
  // Binary GCD with v odd throughout, 31 steps at a time: the steps' parity
  // tests read the exact low 31 bits and their comparisons read the top 33
  // bits, so they run on one 64-bit register per operand; the resulting
  // transition matrix (entries < 2^31 in magnitude, determinant +-2^31) is
  // then applied to the full operands. Every step keeps gcd(u, v) (v stays
  // odd), an approximate comparison only costs a sign flip, and u reaches 0
  // with v = gcd after about 2 * bits / 31 rounds.
  std::vector<uint64_t> nu(n), nv(n);
  const size_t bits = bitlen64(v.data(), n);
  const size_t cap = 2 * (2 * bits / 31 + 8);
  for (size_t round = 0;; ++round) {
    const size_t nb = std::max(bitlen64(u.data(), n), bitlen64(v.data(), n));
    if (bitlen64(u.data(), n) == 0) break;
    if (round == cap) return coprime_binary(u, v);  // not reached in practice
    uint64_t xa, xb;
    if (nb <= 64) {
      xa = u[0];
      xb = v[0];
    } else {
      constexpr uint64_t lo31 = (1ull << 31) - 1;
      xa = (top64(u.data(), nb) & ~lo31) | (u[0] & lo31);
      xb = (top64(v.data(), nb) & ~lo31) | (v[0] & lo31);
    }
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    for (int i = 0; i < 31; ++i) {  // branch-free: odd -> (swap if xa < xb), xa -= xb; then xa /= 2
      const uint64_t odd = 0 - (xa & 1);
      const uint64_t sw = odd & (0 - (uint64_t)(xa < xb));
      const uint64_t tx = (xa ^ xb) & sw;
      xa ^= tx;
      xb ^= tx;
      const int64_t tf = (f0 ^ f1) & (int64_t)sw, tg = (g0 ^ g1) & (int64_t)sw;
      f0 ^= tf;
      f1 ^= tf;
      g0 ^= tg;
      g1 ^= tg;
      xa -= xb & odd;
      f0 -= f1 & (int64_t)odd;
      g0 -= g1 & (int64_t)odd;
      xa >>= 1;
      f1 *= 2;
      g1 *= 2;
    }
    lincomb_shift31(u.data(), v.data(), n, f0, g0, nu.data());
    lincomb_shift31(u.data(), v.data(), n, f1, g1, nv.data());
    u.swap(nu);
    v.swap(nv);
  }
  // gcd = v
  if (v[0] != 1) return false;
  for (size_t i = 1; i < n; ++i)
    if (v[i]) return false;
  return true;
}

namespace {

// t = a b R^-1 mod m (CIOS on 64-bit limbs, R = 2^(64 n)), result < m
void mont_mul64(const uint64_t* a, const uint64_t* b, const uint64_t* m, size_t n, uint64_t minv, uint64_t* out) {
  using u128 = unsigned __int128;
  uint64_t t[kGcdMaxWords + 2] = {};
  for (size_t i = 0; i < n; ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < n; ++j) {
      const u128 v = (u128)a[j] * b[i] + t[j] + c;
      t[j] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
    u128 v = (u128)t[n] + c;
    t[n] = (uint64_t)v;
    t[n + 1] = (uint64_t)(v >> 64);
    const uint64_t q = t[0] * minv;
    v = (u128)q * m[0] + t[0];
    c = (uint64_t)(v >> 64);
    for (size_t j = 1; j < n; ++j) {
      v = (u128)q * m[j] + t[j] + c;
      t[j - 1] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
    v = (u128)t[n] + c;
    t[n - 1] = (uint64_t)v;
    t[n] = t[n + 1] + (uint64_t)(v >> 64);
  }
  // t < 2m: one conditional subtraction
  bool ge = t[n] != 0;
  if (!ge) {
    ge = true;
    for (size_t j = n; j-- > 0;)
      if (t[j] != m[j]) {
        ge = t[j] > m[j];
        break;
      }
  }
  if (ge) {
    uint64_t br = 0;
    for (size_t j = 0; j < n; ++j) {
      const u128 d = (u128)t[j] - m[j] - br;
      t[j] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1;
    }
  }
  for (size_t j = 0; j < n; ++j) out[j] = t[j];
}

}  // namespace

bool coprime_product_odd(const Nat* const* xs, size_t k, const Nat& m) {
  if (m.is_zero() || !m.is_odd()) throw std::invalid_argument("coprime_product_odd: modulus must be odd");
  if (m == Nat(1) || k == 0) return true;
  if (k == 1) return coprime_odd(*xs[0], m);
  const V64 mv = to64(m);
  const size_t n = mv.size();
  if (n > kGcdMaxWords) {
    for (size_t i = 0; i < k; ++i)
      if (!coprime_odd(*xs[i], m)) return false;
    return true;
  }
  uint64_t minv = 1;  // -m^-1 mod 2^64 by Newton iteration
  for (int i = 0; i < 6; ++i) minv *= 2 - mv[0] * minv;
  minv = 0 - minv;
  // acc = prod x_i R^-(k-1) mod m; R is a unit mod odd m, so gcd(acc, m) ==
  // gcd(prod x_i, m), which is 1 iff every x_i is coprime to m
  auto load = [&](const Nat& x, V64* out) {
    *out = to64(x < m ? x : x % m);
    out->resize(n, 0);
  };
  V64 acc, xv, tmp(n);
  load(*xs[0], &acc);
  for (size_t i = 1; i < k; ++i) {
    load(*xs[i], &xv);
    mont_mul64(acc.data(), xv.data(), mv.data(), n, minv, tmp.data());
    acc.swap(tmp);
  }
  Nat a;
  {
    std::vector<uint32_t> w(2 * n);
    for (size_t i = 0; i < n; ++i) {
      w[2 * i] = (uint32_t)acc[i];
      w[2 * i + 1] = (uint32_t)(acc[i] >> 32);
    }
    a = Nat::from_words(w.data(), w.size());
  }
  return coprime_odd(a, m);
}

}  // namespace mpcx::host

namespace mpcx::host {

Nat isqrt(const Nat& n) {
  if (n.is_zero()) return Nat();
  // Newton from above: x0 = 2^ceil(bits/2) >= sqrt(n)
  Nat x = Nat(1) << ((n.bit_len() + 1) / 2);
  for (;;) {
    Nat y = (x + n / x) >> 1;
    if (!(y < x)) return x;
    x = y;
  }
}

int jacobi(const Nat& a_in, const Nat& n_in) {
  if (!n_in.is_odd()) throw std::invalid_argument("jacobi: n must be odd");
  Nat a = a_in % n_in, n = n_in;
  int j = 1;
  while (!a.is_zero()) {
    uint32_t z = 0;
    while (!a.bit(z)) ++z;
    if (z) {
      a = a >> z;
      const uint32_t n8 = (uint32_t)(n.low64() & 7u);
      if ((z & 1u) && (n8 == 3 || n8 == 5)) j = -j;
    }
    // reciprocity: swap, flip if both are 3 mod 4
    if ((a.low64() & 3u) == 3 && (n.low64() & 3u) == 3) j = -j;
    Nat r = n % a;
    n = a;
    a = r;
  }
  return n == Nat(1) ? j : 0;
}

}  // namespace mpcx::host
