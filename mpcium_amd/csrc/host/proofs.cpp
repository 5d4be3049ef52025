// proofs.cpp -- see proofs.hpp. Each step cites the tss-lib v2.0.2 function it
// mirrors (restated in oracle/proofs_ref.py).
#include "proofs.hpp"

#include <stdexcept>

#include "expset.hpp"
#include "safeprime.hpp"
#include "secp256k1.hpp"

namespace mpcx::host::proofs {
namespace {

const Nat& q() { return secp::CurveN(); }

// Legendre symbol from the Euler criterion value r = x^((p-1)/2) mod p
int legendre_from(const Nat& r, const Nat& p) {
  if (r.is_zero()) return 0;
  if (r == Nat(1)) return 1;
  if (r == p - Nat(1)) return -1;
  throw std::runtime_error("Euler criterion: modulus is not prime");
}

Nat mulmod(const Nat& a, const Nat& b, const Nat& m) { return (a * b) % m; }

std::vector<Nat> mod_challenges(const Bytes& session, const Nat& W, const Nat& N) {
  std::vector<Nat> Y;
  Y.reserve(kModIterations);
  std::vector<const Nat*> in{&W, &N};
  for (int i = 0; i < kModIterations; ++i) {
    Y.push_back(RejectionSample(N, SHA512_256i_TAGGED(session, in)));
    in.push_back(&Y.back());
  }
  return Y;
}

}  // namespace

// ================================================================ DLN
std::vector<DLNProof> DLNProveBatch(const Nat& h1, const Nat& h2, const Nat& x, const Nat& p, const Nat& qq,
                                    const Nat& N, const std::vector<RandFn>& rand) {
  const size_t n = rand.size();
  const Nat pq = p * qq;
  const Nat xr = x % pq;
  std::vector<DLNProof> out(n);
  std::vector<std::vector<Nat>> a(n);
  parallel_for(n, [&](size_t i) {
    a[i].resize(kDLNIterations);
    for (auto& ai : a[i]) ai = GetRandomPositiveInt(rand[i], pq);  // a_i < pq
    out[i].Alpha.resize(kDLNIterations);
    out[i].T.resize(kDLNIterations);
  });
  ExpSet e(N);
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < kDLNIterations; ++k) e.add(h1, a[i][k], &out[i].Alpha[k]);  // alpha_i = h1^a_i mod N
  e.run();
  parallel_for(n, [&](size_t i) {
    std::vector<const Nat*> msg{&h1, &h2, &N};
    for (const auto& al : out[i].Alpha) msg.push_back(&al);
    const Nat c = SHA512_256i(msg);
    for (int k = 0; k < kDLNIterations; ++k) {
      Nat t = a[i][k];
      if (c.bit((uint32_t)k)) t = (t + xr) % pq;  // t_i = a_i + c_i x mod pq
      out[i].T[k] = t;
    }
  });
  return out;
}

std::vector<uint8_t> DLNVerifyBatch(const Nat& h1, const Nat& h2, const Nat& N, const std::vector<DLNProof>& pf) {
  const size_t n = pf.size();
  std::vector<uint8_t> ok(n, 0);
  if (N.is_zero()) return ok;
  const Nat one(1);
  const Nat h1_ = h1 % N, h2_ = h2 % N;
  if (!(one < h1_) || !(one < h2_) || h1_ == h2_) return ok;
  std::vector<Nat> c(n);
  std::vector<std::vector<Nat>> L(n), R(n);
  parallel_for(n, [&](size_t i) {
    const auto& p = pf[i];
    if ((int)p.T.size() != kDLNIterations || (int)p.Alpha.size() != kDLNIterations) return;
    for (const auto* v : {&p.T, &p.Alpha})
      for (const auto& x : *v)
        if (!(one < x % N)) return;
    std::vector<const Nat*> msg{&h1, &h2, &N};
    for (const auto& al : p.Alpha) msg.push_back(&al);
    c[i] = SHA512_256i(msg);
    L[i].resize(kDLNIterations);
    R[i].resize(kDLNIterations);
    ok[i] = 1;
  });
  ExpSet e(N);
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) continue;
    for (int k = 0; k < kDLNIterations; ++k) {
      e.add(h1, pf[i].T[k], &L[i][k]);  // h1^t_i
      // alpha_i h2^c_i with c_i in {0, 1}: alpha_i mod N or alpha_i h2 mod N
      if (c[i].bit((uint32_t)k)) e.add(pf[i].Alpha[k], one, &R[i][k], &h2);
      else R[i][k] = pf[i].Alpha[k] % N;
    }
  }
  e.run();
  for (size_t i = 0; i < n; ++i)
    if (ok[i])
      for (int k = 0; k < kDLNIterations && ok[i]; ++k) ok[i] = L[i][k] == R[i][k];
  return ok;
}

// ================================================================ Mod (Paillier-Blum)
std::vector<ModProof> ModProveBatch(const std::vector<Bytes>& session, const Nat& N, const Nat& P, const Nat& Q,
                                    const std::vector<RandFn>& rand) {
  const size_t n = rand.size();
  if (session.size() != n) throw std::invalid_argument("ModProof: sizes");
  const Nat one(1);
  const Nat Pm1 = P - one, Qm1 = Q - one, phi = Pm1 * Qm1;
  Nat invN;
  if (!mod_inverse(Int(N), phi, &invN)) throw std::invalid_argument("ModProof: N not invertible mod phi");
  Nat expo = (phi + Nat(4)) >> 3;
  expo = (expo * expo) % phi;  // fourth-root exponent
  const Nat eP = Pm1 >> 1, eQ = Qm1 >> 1;
  std::vector<ModProof> out(n);
  std::vector<std::vector<Nat>> Y(n);
  parallel_for(n, [&](size_t i) {
    // common.GetRandomQuadraticNonResidue(rand, N)
    for (;;) {
      Nat w = GetRandomPositiveInt(rand[i], N);
      if (jacobi(w, N) == -1) {
        out[i].W = w;
        break;
      }
    }
    Y[i] = mod_challenges(session[i], out[i].W, N);
    out[i].X.assign(kModIterations, Nat());
    out[i].Z.assign(kModIterations, Nat());
  });
  // Legendre symbols of W and every Y_i mod P and mod Q (Euler criterion on the GPU)
  std::vector<Nat> wP(n), wQ(n);
  std::vector<std::vector<Nat>> yP(n, std::vector<Nat>(kModIterations)), yQ(n, std::vector<Nat>(kModIterations));
  {
    ExpSet eP_(P), eQ_(Q);
    for (size_t i = 0; i < n; ++i) {
      eP_.add(out[i].W, eP, &wP[i]);
      eQ_.add(out[i].W, eQ, &wQ[i]);
      for (int k = 0; k < kModIterations; ++k) {
        eP_.add(Y[i][k], eP, &yP[i][k]);
        eQ_.add(Y[i][k], eQ, &yQ[i][k]);
      }
    }
    run_all({&eP_, &eQ_});
  }
  const int lmP = P.bit(1) ? -1 : 1, lmQ = Q.bit(1) ? -1 : 1;  // (-1 | p) = (-1)^((p-1)/2)
  std::vector<std::vector<Nat>> Yp(n, std::vector<Nat>(kModIterations));
  std::vector<std::vector<uint8_t>> found(n, std::vector<uint8_t>(kModIterations, 0));
  parallel_for(n, [&](size_t i) {
    const int lwP = legendre_from(wP[i], P), lwQ = legendre_from(wQ[i], Q);
    Nat A = one << kModIterations, B = one << kModIterations;
    for (int k = 0; k < kModIterations; ++k) {
      const int lyP = legendre_from(yP[i][k], P), lyQ = legendre_from(yQ[i][k], Q);
      for (int j = 0; j < 4; ++j) {
        const int a = j & 1, b = (j >> 1) & 1;
        const int sP = (a ? lmP : 1) * (b ? lwP : 1) * lyP, sQ = (a ? lmQ : 1) * (b ? lwQ : 1) * lyQ;
        if (sP == 1 && sQ == 1) {
          Nat yi = Y[i][k] % N;
          if (a && !yi.is_zero()) yi = N - yi;   // modN.Mul(-1, Yi)
          if (b) yi = mulmod(out[i].W, yi, N);   // modN.Mul(W, Yi)
          Yp[i][k] = yi;
          found[i][k] = 1;
          if (a) A = A + (one << (uint32_t)k);
          if (b) B = B + (one << (uint32_t)k);
          break;
        }
      }
    }
    out[i].A = A;
    out[i].B = B;
  });
  // X_i = Y'_i^expo mod N (fourth root), Z_i = Y_i^(N^-1 mod phi) mod N, by CRT
  // over the prover's P and Q (same integers: x^e mod p = x^e_p mod p with
  // e_p = ((e - 1) mod (p - 1)) + 1 for e >= 1, also when p | x): two 1024-bit
  // exponents mod 1024-bit primes instead of a 2048-bit one mod N.
  auto red = [&](const Nat& ex, const Nat& pm1) { return ex.is_zero() ? ex : (ex - one) % pm1 + one; };
  const Nat xP = red(expo, Pm1), xQ = red(expo, Qm1), zP = red(invN, Pm1), zQ = red(invN, Qm1);
  std::vector<std::vector<Nat>> rP(n, std::vector<Nat>(2 * kModIterations)),
      rQ(n, std::vector<Nat>(2 * kModIterations));
  {
    ExpSet sP(P), sQ(Q);
    for (size_t i = 0; i < n; ++i)
      for (int k = 0; k < kModIterations; ++k) {
        if (!found[i][k]) continue;
        sP.add(Yp[i][k], xP, &rP[i][2 * k]);
        sQ.add(Yp[i][k], xQ, &rQ[i][2 * k]);
        sP.add(Y[i][k], zP, &rP[i][2 * k + 1]);
        sQ.add(Y[i][k], zQ, &rQ[i][2 * k + 1]);
      }
    run_all({&sP, &sQ});
  }
  Nat qinv;
  if (!mod_inverse(Int(Q % P), P, &qinv)) throw std::invalid_argument("ModProof: P, Q not coprime");
  auto crt = [&](const Nat& a, const Nat& b) {  // x mod P = a, x mod Q = b -> x mod N
    const Nat bp = b % P;
    const Nat d = a < bp ? a + P - bp : a - bp;
    return b + Q * mulmod(d, qinv, P);
  };
  parallel_for(n, [&](size_t i) {
    for (int k = 0; k < kModIterations; ++k) {
      if (!found[i][k]) continue;
      out[i].X[k] = crt(rP[i][2 * k], rQ[i][2 * k]);
      out[i].Z[k] = crt(rP[i][2 * k + 1], rQ[i][2 * k + 1]);
    }
  });
  return out;
}

std::vector<uint8_t> ModVerifyBatch(const std::vector<Bytes>& session, const Nat& N, const std::vector<ModProof>& pf) {
  const size_t n = pf.size();
  if (session.size() != n) throw std::invalid_argument("ModProof.Verify: sizes");
  std::vector<uint8_t> ok(n, 0);
  if (N.is_zero() || !N.is_odd()) return ok;
  if (ProbablyPrimeBatch({N}, 30)[0]) return ok;  // Fig 16: N.ProbablyPrime(30) -> reject (see proofs.hpp)
  const Nat one(1);
  const Nat ref = one << kModIterations;
  std::vector<std::vector<Nat>> Y(n), ZN(n), X4(n);
  parallel_for(n, [&](size_t i) {
    const auto& p = pf[i];
    if ((int)p.X.size() != kModIterations || (int)p.Z.size() != kModIterations) return;
    if (jacobi(p.W, N) != -1) return;
    if (!IsInInterval(p.W, N)) return;
    for (const auto* v : {&p.Z, &p.X})
      for (const auto& x : *v)
        if (!IsInInterval(x, N)) return;
    if (p.A.bit_len() != ref.bit_len() || p.B.bit_len() != ref.bit_len()) return;
    Y[i] = mod_challenges(session[i], p.W, N);
    ZN[i].resize(kModIterations);
    X4[i].resize(kModIterations);
    ok[i] = 1;
  });
  const Nat four(4);
  ExpSet e(N);
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) continue;
    for (int k = 0; k < kModIterations; ++k) {
      e.add(pf[i].Z[k], N, &ZN[i][k]);   // Z_i^N
      e.add(pf[i].X[k], four, &X4[i][k]);  // X_i^4
    }
  }
  e.run();
  parallel_for(n, [&](size_t i) {
    if (!ok[i]) return;
    const auto& p = pf[i];
    for (int k = 0; k < kModIterations; ++k) {
      if (ZN[i][k] != Y[i][k]) {
        ok[i] = 0;
        return;
      }
      Nat right = Y[i][k];
      if (p.A.bit((uint32_t)k) && !right.is_zero()) right = N - right;
      if (p.B.bit((uint32_t)k)) right = mulmod(p.W, right, N);
      if (X4[i][k] != right) {
        ok[i] = 0;
        return;
      }
    }
  });
  return ok;
}

// ================================================================ Fac (no small factor)
std::vector<FacProof> FacProveBatch(const std::vector<Bytes>& session, const Nat& N0, const Nat& NCap, const Nat& s,
                                    const Nat& t, const Nat& N0p, const Nat& N0q, const std::vector<RandFn>& rand) {
  const size_t n = rand.size();
  if (session.size() != n) throw std::invalid_argument("FacProof: sizes");
  const Nat& Q_ = q();
  const Nat q3 = Q_ * Q_ * Q_;
  const Nat q3sqrtN0 = q3 * isqrt(N0);
  const Nat qNCap = Q_ * NCap, qN0NCap = qNCap * N0, q3NCap = q3 * NCap, q3N0NCap = q3NCap * N0;
  struct St {
    Nat alpha, beta, mu, nu, sigma, r, x, y, e;
  };
  std::vector<St> st(n);
  std::vector<FacProof> out(n);
  parallel_for(n, [&](size_t i) {  // Fig 28.1 sample
    auto& v = st[i];
    v.alpha = GetRandomPositiveInt(rand[i], q3sqrtN0);
    v.beta = GetRandomPositiveInt(rand[i], q3sqrtN0);
    v.mu = GetRandomPositiveInt(rand[i], qNCap);
    v.nu = GetRandomPositiveInt(rand[i], qNCap);
    v.sigma = GetRandomPositiveInt(rand[i], qN0NCap);
    v.r = GetRandomPositiveRelativelyPrimeInt(rand[i], q3N0NCap);
    v.x = GetRandomPositiveInt(rand[i], q3NCap);
    v.y = GetRandomPositiveInt(rand[i], q3NCap);
  });
  // Fig 28.1 compute, every value as ONE two-table comb product on (s, t) in
  // ONE launch step (round 4: four steps, s^alpha / s^beta first, then the t
  // products, then Q^alpha, then T):
  //   P = s^N0p t^mu, Q = s^N0q t^nu, A = s^alpha t^x, B = s^beta t^y,
  //   T = Q^alpha t^r = (s^N0q t^nu)^alpha t^r = s^(N0q alpha) t^(nu alpha + r)
  // -- exponent identities of the group Z*_NCap (any commutative monoid), so
  // the same residues bit for bit; the longest exponent, nu alpha + r, is
  // < q^3 N0 NCap + q NCap q^3 sqrt(N0) < 2^4900, inside the comb tables'
  // kFixedMaxBits (longer ones would take the per-operand path).
  std::vector<Nat> ea(n), eb(n);
  ExpSet e(NCap);
  for (size_t i = 0; i < n; ++i) {
    auto& v = st[i];
    ea[i] = N0q * v.alpha;
    eb[i] = v.nu * v.alpha + v.r;
    e.add2(s, N0p, t, v.mu, &out[i].P);
    e.add2(s, N0q, t, v.nu, &out[i].Q);
    e.add2(s, v.alpha, t, v.x, &out[i].A);
    e.add2(s, v.beta, t, v.y, &out[i].B);
    e.add2(s, ea[i], t, eb[i], &out[i].T);
  }
  e.run();
  parallel_for(n, [&](size_t i) {
    auto& o = out[i];
    auto& v = st[i];
    o.Sigma = v.sigma;
    v.e = RejectionSample(Q_, SHA512_256i_TAGGED(session[i], {&N0, &NCap, &s, &t, &o.P, &o.Q, &o.A, &o.B, &o.T,
                                                               &o.Sigma}));
    o.Z1 = v.e * N0p + v.alpha;  // Fig 28.3
    o.Z2 = v.e * N0q + v.beta;
    o.W1 = v.e * v.mu + v.x;
    o.W2 = v.e * v.nu + v.y;
    // v = e (sigma - nu N0p) + r, signed
    const Nat nuN0p = v.nu * N0p;
    if (!(v.sigma < nuN0p)) {
      o.V = Int(v.e * (v.sigma - nuN0p) + v.r);
    } else {
      const Nat neg = v.e * (nuN0p - v.sigma);
      o.V = v.r < neg ? Int(neg - v.r, true) : Int(v.r - neg);
    }
  });
  return out;
}

std::vector<uint8_t> FacVerifyBatch(const std::vector<Bytes>& session, const Nat& N0, const Nat& NCap, const Nat& s,
                                    const Nat& t, const std::vector<FacProof>& pf) {
  const size_t n = pf.size();
  if (session.size() != n) throw std::invalid_argument("FacProof.Verify: sizes");
  std::vector<uint8_t> ok(n, 0);
  if (N0.is_zero() || NCap.is_zero()) return ok;
  const Nat& Q_ = q();
  // z1, z2 range (CGGMP Fig. 28: z1, z2 in +-sqrt(N0) 2^(l+eps)), checked
  // before any exponentiation: an honest z = e N0p + alpha has alpha <
  // q^3 isqrt(N0) and e N0p < 2 q isqrt(N0) (N0p < sqrt(2 N0) for a balanced
  // N0), so z <= (q^3 + 2q) isqrt(N0); a prover hiding a small factor of N0
  // needs z ~ e N0/small far above it. The exact expression tss-lib uses is
  // not in this image: parity of this bound is unpinned.
  const Nat zbound = (Q_ * Q_ * Q_ + Q_ + Q_) * isqrt(N0);
  std::vector<Nat> e(n);
  bool any_neg = false;
  parallel_for(n, [&](size_t i) {
    const auto& p = pf[i];
    if (p.Z1 > zbound || p.Z2 > zbound) return;
    for (const Nat* v : {&p.P, &p.Q, &p.A, &p.B, &p.T})
      if (!IsInInterval(*v, NCap)) return;
    e[i] = RejectionSample(Q_, SHA512_256i_TAGGED(session[i], {&N0, &NCap, &s, &t, &p.P, &p.Q, &p.A, &p.B, &p.T,
                                                               &p.Sigma}));
    ok[i] = 1;
  });
  for (size_t i = 0; i < n; ++i) any_neg |= ok[i] && pf[i].V.neg;
  Nat tinv;
  const bool t_inv_ok = any_neg && mod_inverse(Int(t), NCap, &tinv);
  // Every check's exponentiations in ONE launch step (round 4: three):
  //   s^z1 t^w1 == A P^e,  s^z2 t^w2 == B Q^e,  Q^z1 t^v == T R^e with
  //   R = s^N0 t^sigma, so R^e = s^(N0 e) t^(sigma e) -- a two-table comb
  //   product with multiplier T instead of R first and R^e after it; Q^z1 and
  //   t^v run side by side and are multiplied on the host (2048-bit product).
  struct St {
    Nat qz1, tv, L1, R1, L2, R2, L3, R3, ne, se;
  };
  std::vector<St> st(n);
  ExpSet x(NCap);
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) continue;
    const auto& p = pf[i];
    if (p.V.neg && !t_inv_ok) {  // t^v undefined (Go: nil)
      ok[i] = 0;
      continue;
    }
    auto& v = st[i];
    v.ne = N0 * e[i];
    v.se = p.Sigma * e[i];
    x.add2(s, p.Z1, t, p.W1, &v.L1);       // s^z1 t^w1
    x.add2(s, p.Z2, t, p.W2, &v.L2);       // s^z2 t^w2
    x.add(p.P, e[i], &v.R1, &p.A);         // A P^e
    x.add(p.Q, e[i], &v.R2, &p.B);         // B Q^e
    x.add(p.Q, p.Z1, &v.qz1);              // Q^z1
    x.add(p.V.neg ? tinv : t, p.V.mag, &v.tv);  // t^v
    x.add2(s, v.ne, t, v.se, &v.R3, &p.T);  // T R^e = T s^(N0 e) t^(sigma e)
  }
  x.run();
  parallel_for(n, [&](size_t i) {
    if (ok[i]) st[i].L3 = (st[i].qz1 * st[i].tv) % NCap;  // Q^z1 t^v
  });
  for (size_t i = 0; i < n; ++i)
    ok[i] = ok[i] && st[i].L1 == st[i].R1 && st[i].L2 == st[i].R2 && st[i].L3 == st[i].R3;
  return ok;
}

}  // namespace mpcx::host::proofs
