// gorand.hpp -- Go math/rand's generator, as math/big's ProbablyPrime uses it
// for its Miller-Rabin bases (go1.23.5 math/big/prime.go
// probablyPrimeMillerRabin: rand.New(rand.NewSource(int64(n[0]))), bases
// x = nat.random(rand, n - 3) + 2, base 2 in the last round).
//
//   rngSource  go:src/math/rand/rng.go: additive lagged Fibonacci generator
//              s_t = s_(t-607) + s_(t-273) over Z/2^64 in a 607-word ring,
//              seeded by the Park-Miller stream x <- 48271 x mod 2^31 - 1
//              XORed with rngCooked
//   rngCooked  go:src/math/rand/gen_cooked.go: the same ring filled from
//              seed 1 (shifts 20 / 10), after 7.8e12 steps -- taken here as
//              one jump (x^7.8e12 mod x^607 - x^334 - 1), computed on first use
//   Uint32     Int63() >> 31
//   nat.random go:src/math/big/nat.go: 64-bit Words, Uint32() | Uint32() << 32
//              per word, top word masked to the limit's bit length, retried
//              until below the limit
// Restated in oracle/gorand.py, pinned there by Go's documented outputs for
// seed 1 (Int63 = 5577006791947779410, 8674665223082153551, ...).
#pragma once

#include <cstdint>
#include <vector>

#include "bignum.hpp"

namespace mpcx::host {

class GoRand {
 public:
  explicit GoRand(int64_t seed);  // rand.New(rand.NewSource(seed))
  uint64_t Uint64();
  int64_t Int63() { return (int64_t)(Uint64() & ((1ull << 63) - 1)); }
  uint32_t Uint32() { return (uint32_t)(Int63() >> 31); }

  static constexpr int kLen = 607;
  static constexpr int kTap = 273;

 private:
  int tap_, feed_;
  uint64_t vec_[kLen];
};

// nat.random(rand, limit, limit.BitLen()) with 64-bit Words: uniform in [0, limit)
Nat GoNatRandom(GoRand& r, const Nat& limit);

// The `reps` random Miller-Rabin bases ProbablyPrime(reps) draws for odd
// n > 3, in Go's order (Go runs base 2 after them).
std::vector<Nat> GoMillerRabinBases(const Nat& n, int reps);

}  // namespace mpcx::host
