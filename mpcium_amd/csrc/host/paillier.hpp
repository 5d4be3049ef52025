// paillier.hpp -- batched mirror of tss-lib v2.0.2 crypto/paillier
// (up:crypto/paillier/paillier.go; formulas restated in SURVEY.md 8(a) rows
// A3-A7). Same names, argument meaning and error behaviour as the Go API,
// with a batch dimension: one GPU launch serves every operation of a batch.
//
//   Encrypt:   c = Gamma^m * r^N mod N^2,  Gamma = N + 1. Gamma^m is computed
//              as 1 + m*N mod N^2 (algebraic identity, bit-exact; not counted
//              as a modexp), r^N and the product run fused on the GPU.
//   HomoMult:  c1^m mod N^2                          (GPU, per-operand exponent)
//   HomoAdd:   c1 * c2 mod N^2                       (GPU mulmod)
//   Decrypt:   m = L(c^lambda mod N^2) * L(Gamma^lambda mod N^2)^-1 mod N
//              c^lambda on the GPU (shared exponent lambda); Gamma^lambda =
//              1 + lambda*N, so L(Gamma^lambda) = lambda and its inverse mod N
//              is cached per key; the final product mod N on the GPU. The
//              gcd(c, N^2) == 1 check is done as c mod P != 0 && c mod Q != 0
//              (same predicate, P and Q are private-key fields).
// Randomness: tss-lib draws r inside Encrypt from its io.Reader; the batch API
// takes r from the caller (the Go shim draws it from the same reader), which is
// what makes results reproducible for fixed randomness.
#pragma once

#include <vector>

#include "bignum.hpp"

namespace mpcx::host::paillier {

enum Err : uint8_t { OK = 0, ErrMessageTooLong = 1, ErrMessageMalFormed = 2 };

struct PublicKey {
  Nat N;
  Nat NSquare() const { return N * N; }
  Nat Gamma() const { return N + Nat(1); }

  // EncryptAndReturnRandomness with caller-supplied randomness r in Z*_N.
  void EncryptBatch(const std::vector<Int>& m, const std::vector<Nat>& r, std::vector<Nat>* c,
                    std::vector<uint8_t>* err) const;
  void HomoMultBatch(const std::vector<Int>& m, const std::vector<Int>& c1, std::vector<Nat>* out,
                     std::vector<uint8_t>* err) const;
  void HomoAddBatch(const std::vector<Int>& c1, const std::vector<Int>& c2, std::vector<Nat>* out,
                    std::vector<uint8_t>* err) const;
};

struct PrivateKey {
  PublicKey pub;
  Nat LambdaN, PhiN, P, Q;
  void DecryptBatch(const std::vector<Int>& c, std::vector<Nat>* m, std::vector<uint8_t>* err) const;
};

// The key holder's CRT decryption (DecryptBatch's CRT form) in two parts, so a
// caller can put the two exponentiations up = c^(P-1) mod P^2 and
// uq = c^(Q-1) mod Q^2 into a launch step it already runs (AliceEnd's
// verification, mta.cpp) instead of a step of their own. Same plaintext as
// tss-lib's L(c^lambda) * mu mod N for every c in Z*_{N^2}.
struct CrtDecrypt {
  Nat P, Q, P2, Q2, Pm1, Qm1, hP, hQ, qinv;
  explicit CrtDecrypt(const PrivateKey& sk);  // requires the factors P, Q of N
  // m from (up, uq); ErrMessageMalFormed when P | c or Q | c (gcd(c, N^2) != 1)
  uint8_t finish(const Nat& up, const Nat& uq, Nat* m) const;
};

// L(u) = (u - 1) / N
Nat L(const Nat& u, const Nat& N);

}  // namespace mpcx::host::paillier
