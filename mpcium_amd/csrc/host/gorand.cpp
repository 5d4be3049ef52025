// gorand.cpp -- see gorand.hpp.
#include "gorand.hpp"

#include <array>
#include <mutex>

namespace mpcx::host {
namespace {

constexpr int L = GoRand::kLen, T = GoRand::kTap;
constexpr int32_t kInt32Max = 0x7FFFFFFF;

// x[n+1] = 48271 x[n] mod (2^31 - 1), Schrage's method as rng.go
int32_t seedrand(int32_t x) {
  const int32_t hi = x / 44488, lo = x % 44488;
  x = 48271 * lo - 3399 * hi;
  if (x < 0) x += kInt32Max;
  return x;
}

using Poly = std::array<uint64_t, L>;

// a * b mod (x^607 - x^334 - 1) over Z/2^64
Poly polymulmod(const Poly& a, const Poly& b) {
  std::array<uint64_t, 2 * L - 1> p{};
  for (int i = 0; i < L; ++i) {
    if (!a[i]) continue;
    const uint64_t ai = a[i];
    for (int j = 0; j < L; ++j) p[i + j] += ai * b[j];
  }
  for (int k = 2 * L - 2; k >= L; --k) {  // x^k = x^(k-273) + x^(k-607)
    p[k - T] += p[k];
    p[k - L] += p[k];
  }
  Poly r;
  for (int i = 0; i < L; ++i) r[i] = p[i];
  return r;
}

// rngCooked: gen_cooked.go's ring after 7.8e12 steps from srand(1)
const std::array<uint64_t, L>& cooked() {
  static std::array<uint64_t, L> c;
  static std::once_flag once;
  std::call_once(once, [] {
    constexpr uint64_t kSteps = 7800000000000ull;
    uint64_t vec[L];
    int32_t x = 1;
    for (int i = -20; i < L; ++i) {
      x = seedrand(x);
      if (i >= 0) {
        uint64_t u = (uint64_t)(int64_t)x << 20;
        x = seedrand(x);
        u ^= (uint64_t)(int64_t)x << 10;
        x = seedrand(x);
        u ^= (uint64_t)(int64_t)x;
        vec[i] = u;
      }
    }
    // sequence window: step t writes ring position (333 - t) mod 607, which
    // held s_(t-607); u_i = s_(i-607), i < 607, extended by the recurrence
    std::vector<uint64_t> u(2 * L);
    for (int i = 0; i < L; ++i) u[i] = vec[((333 - i) % L + L) % L];
    for (int i = L; i < 2 * L; ++i) u[i] = u[i - L] + u[i - T];
    // c(x) = x^M mod P: s_(M-607+i) = u_(M+i) = sum_k c_k u_(k+i)
    Poly res{}, base{};
    res[0] = 1;
    base[1] = 1;
    for (uint64_t n = kSteps; n;) {
      if (n & 1) res = polymulmod(res, base);
      n >>= 1;
      if (n) base = polymulmod(base, base);
    }
    for (int i = 0; i < L; ++i) {
      uint64_t v = 0;
      for (int k = 0; k < L; ++k) v += res[k] * u[k + i];
      const uint64_t t = kSteps - L + (uint64_t)i;  // step that wrote it
      c[(size_t)(((333 - (int64_t)(t % L)) % L + L) % L)] = v;
    }
  });
  return c;
}

}  // namespace

GoRand::GoRand(int64_t seed) {
  const auto& ck = cooked();
  tap_ = 0;
  feed_ = L - T;
  seed = seed % kInt32Max;
  if (seed < 0) seed += kInt32Max;
  if (seed == 0) seed = 89482311;
  int32_t x = (int32_t)seed;
  for (int i = -20; i < L; ++i) {
    x = seedrand(x);
    if (i >= 0) {
      uint64_t u = (uint64_t)(int64_t)x << 40;
      x = seedrand(x);
      u ^= (uint64_t)(int64_t)x << 20;
      x = seedrand(x);
      u ^= (uint64_t)(int64_t)x;
      u ^= ck[(size_t)i];
      vec_[i] = u;
    }
  }
}

uint64_t GoRand::Uint64() {
  if (--tap_ < 0) tap_ += L;
  if (--feed_ < 0) feed_ += L;
  const uint64_t x = vec_[feed_] + vec_[tap_];
  vec_[feed_] = x;
  return x;
}

Nat GoNatRandom(GoRand& r, const Nat& limit) {
  const uint32_t n = limit.bit_len();
  const uint32_t words64 = (n + 63) / 64;
  const uint32_t msw = n % 64 ? n % 64 : 64;
  const uint64_t mask = msw == 64 ? ~0ull : ((1ull << msw) - 1);
  std::vector<uint32_t> w(2 * (size_t)words64);
  for (;;) {
    for (uint32_t i = 0; i < words64; ++i) {
      const uint64_t lo = r.Uint32();
      uint64_t v = lo | ((uint64_t)r.Uint32() << 32);
      if (i == words64 - 1) v &= mask;
      w[2 * i] = (uint32_t)v;
      w[2 * i + 1] = (uint32_t)(v >> 32);
    }
    Nat z = Nat::from_words(w.data(), w.size());
    if (z < limit) return z;
  }
}

std::vector<Nat> GoMillerRabinBases(const Nat& n, int reps) {
  GoRand r((int64_t)n.low64());  // rand.NewSource(int64(n[0]))
  const Nat nm3 = n - Nat(3);
  std::vector<Nat> out;
  out.reserve((size_t)reps);
  for (int i = 0; i < reps; ++i) out.push_back(GoNatRandom(r, nm3) + Nat(2));
  return out;
}

}  // namespace mpcx::host
