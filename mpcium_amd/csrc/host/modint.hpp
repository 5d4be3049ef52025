// modint.hpp -- mirror of tss-lib v2.0.2 common.ModInt (up:common/int.go) and
// the Go math/big (*Int).Exp semantics it inherits (go1.23.5 int.go):
//   Exp(x, y) = x^y mod |m| in [0, |m|); y < 0 uses ModInverse(x, m) and
//   yields nil (Exp returns false) when x is not invertible; the result takes
//   x's sign for odd y and is then made positive mod |m|.
// Every exponentiation runs on the GPU (libmpcx.so). Even moduli and m == 0
// are rejected with EngineError(MPCX_EINVAL): math/big takes a different
// (windowed / CRT / unreduced) path for them that the hot path never uses, so
// a Go integration keeps calling math/big for those.
#pragma once

#include <vector>

#include "bignum.hpp"
#include "engine.hpp"

namespace mpcx::host {

class ModInt {
 public:
  explicit ModInt(const Nat& m) : m_(m) {}
  const Nat& modulus() const { return m_; }

  // z = x^y mod m (Go semantics); returns false where Go returns nil.
  bool Exp(const Int& x, const Int& y, Nat* z) const;

  // Batched Exp: ok[i] == 0 marks a nil result. A single y is shared by all x.
  void ExpBatch(const std::vector<Int>& xs, const std::vector<Int>& ys, std::vector<Nat>* z,
                std::vector<uint8_t>* ok) const;

  // (*modInt).Mul / Add / Sub / ModInverse of up:common/int.go
  Nat Mul(const Nat& x, const Nat& y) const;
  std::vector<Nat> MulBatch(const std::vector<Nat>& x, const std::vector<Nat>& y) const;
  Nat Add(const Int& x, const Int& y) const;
  Nat Sub(const Int& x, const Int& y) const;
  bool ModInverse(const Int& g, Nat* out) const { return mod_inverse(g, m_, out); }

 private:
  Nat m_;
};

}  // namespace mpcx::host
