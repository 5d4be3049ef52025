// safeprime.hpp -- mirror of tss-lib v2.0.2 common.GetRandomSafePrimesConcurrent
// (up:common/safe_prime.go), paillier.GenerateKeyPair
// (up:crypto/paillier/paillier.go) and keygen.GeneratePreParams
// (up:ecdsa/keygen/prepare.go), called by mpcium once per node at boot
// (/root/reference/pkg/mpc/node.go:69). Restated in SURVEY.md 8(a) A7, A11, A12.
//
// Candidate stream (per runGenPrimeRoutine): read (qBitLen+7)/8 bytes, mask to
// qBitLen with the top two bits set, make odd, delta-walk until q is coprime to
// the primes 3..53; p = 2q + 1. Accept iff bitlen(q) == qBitLen, 2^(p-1) == 1
// mod p (Pocklington) and q passes Miller-Rabin (ProbablyPrime(20): base 2 plus
// 20 further bases). The host sieves candidates (exact trial division, which
// never changes which candidate is accepted first); the GPU runs the Fermat
// test on every survivor in large batches, then Miller-Rabin on the rare
// Fermat survivors. Output order = candidate-stream order, i.e. what tss-lib
// returns at concurrency 1 (its concurrent output order is scheduling-defined).
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
  uint64_t sieved_out = 0;     // rejected by host trial division
  uint64_t fermat_tests = 0;   // GPU Pocklington/Fermat tests
  uint64_t mr_tests = 0;       // GPU Miller-Rabin tests
  double seconds = 0;
};

// common.GetRandomSafePrimesConcurrent(ctx, bitLen, numPrimes, 1, rand)
std::vector<GermainSafePrime> GetRandomSafePrimes(int bitLen, int numPrimes, const RandFn& rand,
                                                  SafePrimeStats* stats = nullptr, size_t batch = 0,
                                                  uint64_t max_candidates = (1ull << 40));

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
paillier::PrivateKey GenerateKeyPair(int modulusBitLen, const RandFn& rand, SafePrimeStats* stats = nullptr);

struct LocalPreParams {
  paillier::PrivateKey PaillierSK;
  Nat NTildei, H1i, H2i, Alpha, Beta, P, Q;
};

// keygen.GeneratePreParamsWithContextAndRandom (Paillier 2048 + N~ from two
// 1024-bit safe primes, h1 = f^2, h2 = h1^alpha mod N~, beta = alpha^-1 mod pq)
LocalPreParams GeneratePreParams(const RandFn& rand, SafePrimeStats* stats = nullptr);

}  // namespace mpcx::host
