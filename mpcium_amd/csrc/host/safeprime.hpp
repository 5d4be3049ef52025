// safeprime.hpp -- mirror of tss-lib v2.0.2 common.GetRandomSafePrimesConcurrent
// (up:common/safe_prime.go), paillier.GenerateKeyPair
// (up:crypto/paillier/paillier.go) and keygen.GeneratePreParams
// (up:ecdsa/keygen/prepare.go), called by mpcium once per node at boot
// (/root/reference/pkg/mpc/node.go:69). Restated in SURVEY.md 8(a) A7, A11, A12.
//
// Candidate stream (per runGenPrimeRoutine): read (qBitLen+7)/8 bytes, mask to
// qBitLen with the top two bits set, make odd, delta-walk until q is coprime to
// the primes 3..53; p = 2q + 1. Accept iff bitlen(q) == qBitLen, 2^(p-1) == 1
// mod p (Pocklington) and q.ProbablyPrime(20) (Go: 20 Miller-Rabin rounds with
// pseudo-random bases plus base 2, then the strong Lucas test).
//
// GPU pipeline (q of 63..1023 bits), one mpcx_safeprime_step per batch of the
// stream: candidates drawn on the device (CounterDRBG streams) or copied from
// the host reader, sieved (exact trial division: never rejects a prime), the
// Pocklington test on every survivor -- and, in the same launch, the base-2
// Miller-Rabin round on the previous batch's Fermat passes. Their survivors
// (in practice the primes) get the remaining 20 Miller-Rabin bases and the
// strong Lucas test (mpcx_mr_batch, mpcx_lucas_batch) while the next batch's
// step runs. Output order = candidate-stream order, i.e. what tss-lib returns
// at concurrency 1 (its concurrent output order is scheduling-defined), and
// the stream is left right after the last accepted candidate (Stream).
//
// ProbablyPrime decisions are Go's: the n Miller-Rabin bases come from Go's
// math/rand seeded with the candidate's low word (gorand.hpp, as
// go:src/math/big/prime.go draws them), plus base 2 and the strong Lucas test.
#pragma once

#include <cstdint>
#include <functional>
#include <vector>

#include "bignum.hpp"
#include "paillier.hpp"
#include "tsscommon.hpp"

namespace mpcx::host {

struct GermainSafePrime {
  Nat p;  // safe prime p = 2q + 1
  Nat q;  // Sophie Germain prime
  uint64_t index;  // position in the candidate stream
};

struct SafePrimeStats {
  uint64_t candidates = 0;     // stream candidates drawn
  uint64_t sieved_out = 0;     // rejected by the sieve (masks, bit length, trial division)
  uint64_t fermat_tests = 0;   // GPU Pocklington/Fermat tests
  uint64_t mr_tests = 0;       // GPU Miller-Rabin rounds (base 2 + further bases)
  uint64_t lucas_tests = 0;    // GPU strong Lucas tests
  double seconds = 0;
};

// The io.Reader a search draws from, consumed exactly as tss-lib at
// concurrency 1 consumes its reader: after GetRandomSafePrimes the stream
// stands right after the last accepted candidate's bytes (the batches' extra
// bytes are given back: a CounterDRBG seeks, a host reader's bytes are pushed
// back and served first to the next draw). A CounterDRBG stream's candidate
// bytes are drawn on the GPU.
class Stream {
 public:
  explicit Stream(RandFn fn) : fn_(std::move(fn)) {}
  explicit Stream(CounterDRBG* drbg) : drbg_(drbg) {}
  void read(uint8_t* out, size_t n);
  void unread(const uint8_t* data, size_t n);  // n bytes back in front of the stream
  // the CounterDRBG the GPU may draw from at its current position (none while
  // pushed-back bytes are pending)
  CounterDRBG* device_stream() const { return pushback_.empty() ? drbg_ : nullptr; }
  RandFn fn() {
    return [this](uint8_t* b, size_t n) { read(b, n); };
  }

 private:
  RandFn fn_;
  CounterDRBG* drbg_ = nullptr;
  std::vector<uint8_t> pushback_;  // served from the front
  size_t pb_pos_ = 0;
};

// common.GetRandomSafePrimesConcurrent(ctx, bitLen, numPrimes, 1, rand)
std::vector<GermainSafePrime> GetRandomSafePrimes(int bitLen, int numPrimes, Stream& rand,
                                                  SafePrimeStats* stats = nullptr, size_t batch = 0,
                                                  uint64_t max_candidates = (1ull << 40));
// Same over a plain reader (the batches' extra bytes are consumed).
std::vector<GermainSafePrime> GetRandomSafePrimes(int bitLen, int numPrimes, const RandFn& rand,
                                                  SafePrimeStats* stats = nullptr, size_t batch = 0,
                                                  uint64_t max_candidates = (1ull << 40));

// Go (*Int).ProbablyPrime(reps) decisions for a batch of odd n (see the
// header comment on the bases): small-prime exits, Miller-Rabin with base 2 +
// `reps` further bases (Go's), and the strong Lucas test, on the GPU (n up to
// 2^2048: a 2048-bit Paillier N takes the wide Lucas geometry).
// base2_passed: every n is already known to pass the base-2 round (the safe-
// prime step decided it), which is then not repeated. The further bases and
// the Lucas test run as two concurrent GPU batches; the decision is their
// conjunction, as in Go.
std::vector<uint8_t> ProbablyPrimeBatch(const std::vector<Nat>& n, int reps, SafePrimeStats* stats = nullptr,
                                        bool base2_passed = false);
// Baillie-OEIS method C for Go's probablyPrimeLucas: 1 with *P (run the test),
// 0 (n composite: square, or Jacobi(P^2 - 4, n) = 0 with n != P + 2),
// 2 (n == P + 2 is prime).
int LucasParam(const Nat& n, uint32_t* P);

// One batch of the CounterDRBG(seed) candidate stream: candidates
// [batch_no*batch, (batch_no+1)*batch), drawn by seeking the stream to the
// batch's first byte. Every accepted safe prime of the batch, in stream order.
// The sharded search (mpcium_amd/shard.py safe_primes_sharded) gives rank g the
// batches b = g (mod G) and keeps the first numPrimes indices over all ranks:
// exactly GetRandomSafePrimes' output for the same seed and batch size.
std::vector<GermainSafePrime> SafePrimeBatch(int bitLen, uint64_t seed, uint64_t batch_no, size_t batch = 0,
                                             SafePrimeStats* stats = nullptr);

// Candidate q from raw bytes (steps 1-3); exposed for tests.
Nat CandidateFromBytes(const uint8_t* bytes, size_t n, int qBitLen);

// paillier.GenerateKeyPair(ctx, rand, modulusBitLen)
paillier::PrivateKey GenerateKeyPair(int modulusBitLen, Stream& rand, SafePrimeStats* stats = nullptr);

struct LocalPreParams {
  paillier::PrivateKey PaillierSK;
  Nat NTildei, H1i, H2i, Alpha, Beta, P, Q;
};

// keygen.GeneratePreParamsWithContextAndRandom (Paillier 2048 + N~ from two
// 1024-bit safe primes, h1 = f^2, h2 = h1^alpha mod N~, beta = alpha^-1 mod pq),
// the Paillier search first, then N~'s, then f and alpha, on one stream
LocalPreParams GeneratePreParams(Stream& rand, SafePrimeStats* stats = nullptr);

}  // namespace mpcx::host
