// Property check of the host Nat arithmetic under ASAN + UBSAN (CPU only; tools/nat_asan.sh):
// u = q v + r with r < v, and (u v) / v == u, (u v) % v == 0, on random and all-ones operands of
// 1..260 / 1..140 words (odd and even word counts, the 64-bit-limb padding paths).
#include "bignum.hpp"
#include <cstdio>
#include <random>
using namespace mpcx::host;
static Nat rnd(std::mt19937_64& g, int words, bool ones) {
  std::vector<uint32_t> w(words);
  for (auto& x : w) x = ones ? 0xFFFFFFFFu : (uint32_t)g();
  if (words) w.back() |= 1u << (g() % 32);
  return Nat::from_words(w.data(), w.size());
}
int main() {
  std::mt19937_64 g(7);
  long bad = 0, n = 0;
  for (int it = 0; it < 20000; ++it) {
    const int wu = 1 + g() % 260, wv = 1 + g() % 140;
    Nat u = rnd(g, wu, (g() % 16) == 0), v = rnd(g, wv, (g() % 16) == 0);
    if (v.is_zero()) continue;
    Nat q, r;
    Nat::divmod(u, v, &q, &r);
    if (!(r < v) || q * v + r != u) ++bad;
    Nat p = u * v;
    if (p / v != u || !(p % v).is_zero()) ++bad;
    ++n;
  }
  std::printf("checked %ld, bad %ld\n", n, bad);
  return bad != 0;
}
