// secp256k1.hpp -- the curve arithmetic the MtAwc proofs need on the host
// (tss.EC() = btcec/v2 S256, /root/reference/go.mod:29): u = alpha*G in
// ProveBobWC and s1*G == e*X + u in (*ProofBobWC).Verify
// (up:crypto/mta/proofs.go), and the signature + ecdsa.Verify of signing.cpp.
// Fixed-width 4x64-bit field arithmetic mod p = 2^256 - 2^32 - 977 (dedicated
// squaring, 255S + 15M inversion chain), Jacobian coordinates, a 32 x 255
// affine table for the base point (k*G = at most 32 mixed additions), and
// width-5 NAF for variable points.
// ScalarBaseMult(k) = (k mod n)*G (crypto.ScalarBaseMult semantics under which
// the MtAwc check holds for alpha < q^3).
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "bignum.hpp"

namespace mpcx::host::secp {

using Fe = std::array<uint64_t, 4>;  // little-endian limbs, value < p

struct Affine {
  Fe x{}, y{};
  bool inf = true;  // point at infinity
};

extern const Nat& CurveN();  // group order n (= q in tss-lib)
const Affine& Generator();   // G
const Nat& FieldP();         // p = 2^256 - 2^32 - 977

// k*G, k reduced mod n
Affine ScalarBaseMult(const Nat& k);
// k*P, k reduced mod n
Affine ScalarMult(const Affine& P, const Nat& k);
Affine Add(const Affine& P, const Affine& Q);
// u1*G + u2*X (both scalars reduced mod n) with one affine conversion
Affine LinComb(const Nat& u1, const Affine& X, const Nat& u2);
// a*G + b*P + c*Q (scalars reduced mod n; a zero scalar or an infinite point
// drops its term): every point equation of GG18's rounds 5-9 and of the
// Schnorr proofs is one of these
Affine Combine(const Nat& a, const Affine& P, const Nat& b, const Affine& Q, const Nat& c);
struct Comb {
  Nat a, b, c;
  Affine P, Q;
};
// Combine over a batch of independent items, on the GPU (one thread per item:
// mpcx_ec_combine_batch); throws without a bound device
std::vector<Affine> CombineBatch(const std::vector<Comb>& items);
bool IsOnCurve(const Affine& P);
bool Equal(const Affine& P, const Affine& Q);

Nat FeToNat(const Fe& a);
Fe NatToFe(const Nat& a);  // requires a < 2^256 (reduced mod p)

}  // namespace mpcx::host::secp
