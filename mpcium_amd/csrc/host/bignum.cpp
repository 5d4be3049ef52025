// bignum.cpp -- see bignum.hpp.
#include "bignum.hpp"

#include "hostprof.hpp"

#include <algorithm>
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

Nat operator*(const Nat& a, const Nat& b) {
  Nat r;
  if (a.is_zero() || b.is_zero()) return r;
  r.w_.assign(a.w_.size() + b.w_.size(), 0);
  for (size_t i = 0; i < b.w_.size(); ++i) {
    uint64_t c = 0;
    const uint64_t bi = b.w_[i];
    for (size_t j = 0; j < a.w_.size(); ++j) {
      c += (uint64_t)a.w_[j] * bi + r.w_[i + j];
      r.w_[i + j] = (uint32_t)c;
      c >>= 32;
    }
    r.w_[i + a.w_.size()] = (uint32_t)c;
  }
  r.norm();
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

// Knuth, TAOCP vol. 2, 4.3.1, Algorithm D.
void Nat::divmod(const Nat& u, const Nat& v, Nat* q, Nat* r) {
  if (v.is_zero()) throw std::domain_error("division by zero");
  if (cmp(u, v) < 0) {
    if (q) *q = Nat();
    if (r) *r = u;
    return;
  }
  const size_t n = v.w_.size(), m = u.w_.size() - n;
  if (n == 1) {
    Nat qq;
    qq.w_.assign(u.w_.size(), 0);
    uint64_t rem = 0;
    for (int i = (int)u.w_.size() - 1; i >= 0; --i) {
      const uint64_t cur = (rem << 32) | u.w_[i];
      qq.w_[i] = (uint32_t)(cur / v.w_[0]);
      rem = cur % v.w_[0];
    }
    qq.norm();
    if (q) *q = qq;
    if (r) *r = Nat(rem);
    return;
  }
  const int s = __builtin_clz(v.w_.back());
  std::vector<uint32_t> vn(n), un(u.w_.size() + 1);
  for (size_t i = n - 1; i > 0; --i) vn[i] = s ? (v.w_[i] << s) | (v.w_[i - 1] >> (32 - s)) : v.w_[i];
  vn[0] = v.w_[0] << s;
  un[u.w_.size()] = s ? u.w_.back() >> (32 - s) : 0;
  for (size_t i = u.w_.size() - 1; i > 0; --i) un[i] = s ? (u.w_[i] << s) | (u.w_[i - 1] >> (32 - s)) : u.w_[i];
  un[0] = u.w_[0] << s;
  Nat qq;
  qq.w_.assign(m + 1, 0);
  for (int j = (int)m; j >= 0; --j) {
    const uint64_t num = ((uint64_t)un[j + n] << 32) | un[j + n - 1];
    uint64_t qhat = num / vn[n - 1], rhat = num % vn[n - 1];
    while (qhat >= (1ull << 32) || qhat * vn[n - 2] > ((rhat << 32) | un[j + n - 2])) {
      --qhat;
      rhat += vn[n - 1];
      if (rhat >= (1ull << 32)) break;
    }
    int64_t borrow = 0;
    uint64_t carry = 0;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t p = qhat * vn[i] + carry;
      carry = p >> 32;
      const int64_t t = (int64_t)un[i + j] - (int64_t)(uint32_t)p + borrow;
      un[i + j] = (uint32_t)t;
      borrow = t >> 32;
    }
    const int64_t t = (int64_t)un[j + n] - (int64_t)carry + borrow;
    un[j + n] = (uint32_t)t;
    if (t < 0) {
      --qhat;
      uint64_t c = 0;
      for (size_t i = 0; i < n; ++i) {
        const uint64_t sum = (uint64_t)un[i + j] + vn[i] + c;
        un[i + j] = (uint32_t)sum;
        c = sum >> 32;
      }
      un[j + n] += (uint32_t)c;
    }
    qq.w_[j] = (uint32_t)qhat;
  }
  qq.norm();
  if (q) *q = qq;
  if (r) {
    Nat rr;
    rr.w_.assign(n, 0);
    for (size_t i = 0; i < n; ++i) rr.w_[i] = s ? (un[i] >> s) | (un[i + 1] << (32 - s)) : un[i];
    rr.norm();
    *r = rr;
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

bool coprime_odd(const Nat& x, const Nat& m) {
  MPCX_PROF("gcd.coprime_odd");
  if (m.is_zero() || !m.is_odd()) throw std::invalid_argument("coprime_odd: modulus must be odd");
  if (m == Nat(1)) return true;
  const Nat a = x >= m ? x % m : x;
  if (a.is_zero()) return false;
  V64 u = to64(a), v = to64(m);
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
  // binary GCD of odd u, v (gcd(x, m) = gcd(x / 2^k, m) for odd m)
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
