// modint.cpp -- see modint.hpp.
#include "modint.hpp"

namespace mpcx::host {

void ModInt::ExpBatch(const std::vector<Int>& xs, const std::vector<Int>& ys, std::vector<Nat>* z,
                      std::vector<uint8_t>* ok) const {
  if (ys.size() != 1 && ys.size() != xs.size()) throw std::invalid_argument("ys: 1 or one per x");
  if (m_.is_zero()) throw EngineError(MPCX_EINVAL, "ModInt: m == 0 is not supported");
  const size_t n = xs.size();
  z->assign(n, Nat());
  ok->assign(n, 1);
  // Go (*Int).exp: for y < 0, xWords = ModInverse(x, m).abs (nil if none);
  // otherwise xWords = x.abs. The GPU computes xWords^|y| mod m.
  std::vector<Nat> bases(n);
  for (size_t i = 0; i < n; ++i) {
    const Int& y = ys.size() == 1 ? ys[0] : ys[i];
    if (y.neg) {
      Nat inv;
      if (!mod_inverse(xs[i], m_, &inv)) {
        (*ok)[i] = 0;
        continue;
      }
      bases[i] = inv;
    } else {
      bases[i] = xs[i].mag;
    }
  }
  std::vector<Nat> exps;
  for (const auto& y : ys) exps.push_back(y.mag);
  std::vector<Nat> r = Engine::get().exp(m_, bases, exps);
  for (size_t i = 0; i < n; ++i) {
    if (!(*ok)[i]) continue;
    const Int& y = ys.size() == 1 ? ys[0] : ys[i];
    // z.neg = len(z.abs) > 0 && x.neg && len(yWords) > 0 && yWords[0]&1 == 1
    const bool neg = !r[i].is_zero() && xs[i].neg && !y.mag.is_zero() && y.mag.is_odd();
    (*z)[i] = neg ? m_ - r[i] : r[i];
  }
}

bool ModInt::Exp(const Int& x, const Int& y, Nat* z) const {
  std::vector<Nat> zs;
  std::vector<uint8_t> ok;
  ExpBatch({x}, {y}, &zs, &ok);
  if (!ok[0]) return false;
  *z = zs[0];
  return true;
}

Nat ModInt::Mul(const Nat& x, const Nat& y) const { return MulBatch({x}, {y})[0]; }

std::vector<Nat> ModInt::MulBatch(const std::vector<Nat>& x, const std::vector<Nat>& y) const {
  return Engine::get().mulmod(m_, x, y);
}

Nat ModInt::Add(const Int& x, const Int& y) const {
  Nat a = mod_signed(x, m_), b = mod_signed(y, m_);
  Nat s = a + b;
  return s >= m_ ? s - m_ : s;
}

Nat ModInt::Sub(const Int& x, const Int& y) const {
  Nat a = mod_signed(x, m_), b = mod_signed(y, m_);
  return a >= b ? a - b : (a + m_) - b;
}

}  // namespace mpcx::host
