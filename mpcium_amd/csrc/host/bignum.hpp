// bignum.hpp -- minimal host-side arbitrary-precision integers for the glue
// around the GPU engine (sign handling, reductions, L(u) = (u-1)/N, modular
// inverses, byte/word conversion). No modular exponentiation lives here: every
// Exp of the hot path goes through libmpcx.so.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mpcx::host {

// Non-negative integer, little-endian 32-bit words, normalized (no leading zeros).
class Nat {
 public:
  Nat() = default;
  explicit Nat(uint64_t v);
  static Nat from_words(const uint32_t* w, size_t n);
  void set_words(const uint32_t* w, size_t n);  // = from_words(w, n), one exact-size allocation
  static Nat from_bytes_be(const uint8_t* b, size_t n);  // Go big.Int.SetBytes
  static Nat from_hex(const std::string& s);

  std::vector<uint8_t> to_bytes_be() const;  // Go big.Int.Bytes (empty for 0)
  void to_words(uint32_t* out, size_t n) const;  // zero-padded; requires words() <= n
  std::string to_hex() const;

  size_t words() const { return w_.size(); }
  const std::vector<uint32_t>& limbs() const { return w_; }
  uint32_t bit_len() const;
  bool is_zero() const { return w_.empty(); }
  bool is_odd() const { return !w_.empty() && (w_[0] & 1u); }
  bool bit(uint32_t i) const;
  uint64_t low64() const;

  friend int cmp(const Nat& a, const Nat& b);
  friend Nat operator+(const Nat& a, const Nat& b);
  friend Nat operator-(const Nat& a, const Nat& b);  // requires a >= b
  friend Nat operator*(const Nat& a, const Nat& b);
  friend Nat operator<<(const Nat& a, uint32_t s);
  friend Nat operator>>(const Nat& a, uint32_t s);
  static void divmod(const Nat& u, const Nat& v, Nat* q, Nat* r);  // v != 0
  friend Nat operator/(const Nat& a, const Nat& b);
  friend Nat operator%(const Nat& a, const Nat& b);
  uint32_t mod_u32(uint32_t m) const;

  bool operator==(const Nat& o) const { return w_ == o.w_; }
  bool operator!=(const Nat& o) const { return w_ != o.w_; }
  bool operator<(const Nat& o) const { return cmp(*this, o) < 0; }
  bool operator<=(const Nat& o) const { return cmp(*this, o) <= 0; }
  bool operator>(const Nat& o) const { return cmp(*this, o) > 0; }
  bool operator>=(const Nat& o) const { return cmp(*this, o) >= 0; }

 private:
  void norm();
  std::vector<uint32_t> w_;
};

Nat gcd(Nat a, Nat b);
// gcd(x, m) == 1 for odd m > 0 (binary GCD on 64-bit limbs; the validity
// checks of the MtA proofs and GetRandomPositiveRelativelyPrimeInt)
bool coprime_odd(const Nat& x, const Nat& m);
// gcd(x_0 * ... * x_{k-1}, m) == 1 for odd m, i.e. every x_i coprime to m: one
// gcd of a Montgomery product (64-bit CIOS) instead of k gcds
bool coprime_product_odd(const Nat* const* xs, size_t k, const Nat& m);
// floor(sqrt(n)) (Go (*Int).Sqrt)
Nat isqrt(const Nat& n);
// Jacobi symbol (a | n) for odd n > 0 (Go big.Jacobi)
int jacobi(const Nat& a, const Nat& n);

// Signed integer (sign-magnitude like Go's big.Int; zero is never negative).
struct Int {
  Nat mag;
  bool neg = false;
  Int() = default;
  Int(const Nat& m, bool n = false) : mag(m), neg(n && !m.is_zero()) {}
  bool is_zero() const { return mag.is_zero(); }
};

// x mod m in [0, m) for signed x (Go (*Int).Mod semantics, m > 0).
Nat mod_signed(const Int& x, const Nat& m);

// Go (*Int).ModInverse(g, n): inverse of g in Z/nZ; returns false if none.
bool mod_inverse(const Int& g, const Nat& n, Nat* out);

}  // namespace mpcx::host
