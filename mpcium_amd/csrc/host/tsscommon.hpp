// tsscommon.hpp -- mirror of the tss-lib v2.0.2 common helpers on the MtA path
// (module pinned at /root/reference/go.mod:10; "up:" = github.com/bnb-chain/tss-lib/v2):
//   up:common/random.go      MustGetRandomInt, GetRandomPositiveInt,
//                            GetRandomPositiveRelativelyPrimeInt,
//                            IsNumberInMultiplicativeGroup (over Go
//                            crypto/rand.Int on a caller io.Reader)
//   up:common/hash.go        SHA512_256, SHA512_256i, SHA512_256i_TAGGED
//   up:common/hash_utils.go  RejectionSample
//   up:common/int.go         IsInInterval
// Restated in oracle/tss_ref.py (the parity oracle); details the restatement
// marks "upstream, verify" are unverifiable in this image.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "bignum.hpp"

namespace mpcx::host {

// io.Reader stand-in: fill buf[0..n) with random bytes.
using RandFn = std::function<void(uint8_t* buf, size_t n)>;

// Deterministic byte stream SHA-256(b"mpcx-drbg" || seed_le64 || ctr_le64),
// identical to oracle/tss_ref.py Reader (tests and synthetic inputs).
class CounterDRBG {
 public:
  explicit CounterDRBG(uint64_t seed) : seed_(seed) {}
  void read(uint8_t* out, size_t n);
  // Position the stream at byte `offset` (block c depends only on (seed, c)):
  // a reader seeked to k bytes yields what a fresh reader yields after k bytes.
  void seek(uint64_t offset);
  uint64_t seed() const { return seed_; }
  // bytes read so far (the next byte's stream offset)
  uint64_t position() const { return ctr_ * 32 - (buf_.size() - pos_); }
  RandFn fn() {
    return [this](uint8_t* b, size_t n) { read(b, n); };
  }

 private:
  uint64_t seed_, ctr_ = 0;
  std::vector<uint8_t> buf_;
  size_t pos_ = 0;
};

// crypto/rand.Int(rand, max)
Nat CryptoRandInt(const RandFn& rand, const Nat& max);
// common.MustGetRandomInt(rand, bits) = crypto/rand.Int(rand, 2^bits - 1)
Nat MustGetRandomInt(const RandFn& rand, uint32_t bits);
// common.GetRandomPositiveInt(rand, lessThan)
Nat GetRandomPositiveInt(const RandFn& rand, const Nat& lessThan);
// common.GetRandomPositiveRelativelyPrimeInt(rand, n), n odd
Nat GetRandomPositiveRelativelyPrimeInt(const RandFn& rand, const Nat& n);
// out[i] = GetRandomPositiveRelativelyPrimeInt(*rand[i], n) for every i; each
// reader makes the same reads as the scalar call, the coprimality decisions of
// each draw round are batched (CoprimeMany)
void GetRandomPositiveRelativelyPrimeIntBatch(const std::vector<const RandFn*>& rand, const Nat& n,
                                              const std::vector<Nat*>& out);
// ok[i] = gcd(*xs[i], m) == 1 (one gcd per chunk of a Montgomery product for odd m)
std::vector<uint8_t> CoprimeMany(const std::vector<const Nat*>& xs, const Nat& m);
// common.IsInInterval(b, bound): 0 <= b < bound (b non-negative here)
inline bool IsInInterval(const Nat& b, const Nat& bound) { return b < bound; }

// common.SHA512_256(in ...[]byte)
std::vector<uint8_t> SHA512_256(const std::vector<std::vector<uint8_t>>& in);
// common.SHA512_256i(in ...*big.Int)
Nat SHA512_256i(const std::vector<const Nat*>& in);
// common.SHA512_256i_TAGGED(tag, in ...*big.Int)
Nat SHA512_256i_TAGGED(const std::vector<uint8_t>& tag, const std::vector<const Nat*>& in);
// common.RejectionSample(q, eHash) = eHash mod q
Nat RejectionSample(const Nat& q, const Nat& eHash);

// Parallel loop over [0, n) on the host worker pool (host_threads() threads
// including the caller); fn must be thread-safe per index.
void parallel_for(size_t n, const std::function<void(size_t)>& fn);
// CPUs this process may run on: affinity mask capped by the cgroup CPU quota
int usable_cpus();
// pool size: MPCX_HOST_THREADS, else min(usable_cpus(), 16 per bound GPU)
int host_threads();

}  // namespace mpcx::host
