// paillier.cpp -- see paillier.hpp.
#include "paillier.hpp"

#include "engine.hpp"
#include "expset.hpp"
#include "tsscommon.hpp"

namespace mpcx::host::paillier {

Nat L(const Nat& u, const Nat& N) { return (u - Nat(1)) / N; }

static Nat mulmod(const Nat& a, const Nat& b, const Nat& m) { return (a * b) % m; }

static bool in_range(const Int& v, const Nat& hi) { return !v.neg && v.mag < hi; }

void PublicKey::EncryptBatch(const std::vector<Int>& m, const std::vector<Nat>& r, std::vector<Nat>* c,
                             std::vector<uint8_t>* err) const {
  if (m.size() != r.size()) throw std::invalid_argument("one r per message");
  const Nat N2 = NSquare();
  c->assign(m.size(), Nat());
  err->assign(m.size(), OK);
  std::vector<Nat> rs, gm;
  std::vector<size_t> idx;
  for (size_t i = 0; i < m.size(); ++i) {
    if (!in_range(m[i], N)) {  // m < 0 || m >= N
      (*err)[i] = ErrMessageTooLong;
      continue;
    }
    idx.push_back(i);
    rs.push_back(r[i]);
    gm.push_back(Nat(1) + m[i].mag * N);  // Gamma^m = 1 + m*N (< N^2 since m < N)
  }
  if (idx.empty()) return;
  // c = Gamma^m * r^N mod N^2, fused on the GPU (shared exponent N)
  std::vector<Nat> out = Engine::get().exp(N2, rs, {N}, &gm);
  for (size_t j = 0; j < idx.size(); ++j) (*c)[idx[j]] = out[j];
}

void PublicKey::HomoMultBatch(const std::vector<Int>& m, const std::vector<Int>& c1, std::vector<Nat>* out,
                              std::vector<uint8_t>* err) const {
  if (m.size() != c1.size()) throw std::invalid_argument("length mismatch");
  const Nat N2 = NSquare();
  out->assign(m.size(), Nat());
  err->assign(m.size(), OK);
  std::vector<Nat> bs, es;
  std::vector<size_t> idx;
  for (size_t i = 0; i < m.size(); ++i) {
    if (!in_range(m[i], N) || !in_range(c1[i], N2)) {
      (*err)[i] = ErrMessageTooLong;
      continue;
    }
    idx.push_back(i);
    bs.push_back(c1[i].mag);
    es.push_back(m[i].mag);
  }
  if (idx.empty()) return;
  std::vector<Nat> r = Engine::get().exp(N2, bs, es);
  for (size_t j = 0; j < idx.size(); ++j) (*out)[idx[j]] = r[j];
}

void PublicKey::HomoAddBatch(const std::vector<Int>& c1, const std::vector<Int>& c2, std::vector<Nat>* out,
                             std::vector<uint8_t>* err) const {
  if (c1.size() != c2.size()) throw std::invalid_argument("length mismatch");
  const Nat N2 = NSquare();
  out->assign(c1.size(), Nat());
  err->assign(c1.size(), OK);
  std::vector<Nat> a, b;
  std::vector<size_t> idx;
  for (size_t i = 0; i < c1.size(); ++i) {
    if (!in_range(c1[i], N2) || !in_range(c2[i], N2)) {
      (*err)[i] = ErrMessageTooLong;
      continue;
    }
    idx.push_back(i);
    a.push_back(c1[i].mag);
    b.push_back(c2[i].mag);
  }
  if (idx.empty()) return;
  std::vector<Nat> r = Engine::get().mulmod(N2, a, b);
  for (size_t j = 0; j < idx.size(); ++j) (*out)[idx[j]] = r[j];
}

void PrivateKey::DecryptBatch(const std::vector<Int>& c, std::vector<Nat>* m, std::vector<uint8_t>* err) const {
  const Nat& N = pub.N;
  const Nat N2 = pub.NSquare();
  m->assign(c.size(), Nat());
  err->assign(c.size(), OK);
  std::vector<Nat> cs;
  std::vector<size_t> idx;
  const bool crt = !P.is_zero() && !Q.is_zero() && P * Q == N;
  for (size_t i = 0; i < c.size(); ++i) {
    if (!in_range(c[i], N2)) {
      (*err)[i] = ErrMessageTooLong;
      continue;
    }
    // gcd(c, N^2) > 1  <=>  P | c or Q | c: checked here on a key without
    // factors, from the CRT exponentiations below otherwise
    if (!crt && !coprime_odd(c[i].mag, N)) {
      (*err)[i] = ErrMessageMalFormed;
      continue;
    }
    idx.push_back(i);
    cs.push_back(c[i].mag);
  }
  if (idx.empty()) return;
  if (!crt) {
    // no factors on this key: tss-lib's formula as written
    // 1. L(c^lambda mod N^2) -- GPU, shared exponent lambda
    std::vector<Nat> u = Engine::get().exp(N2, cs, {LambdaN});
    std::vector<Nat> lc(u.size());
    for (size_t j = 0; j < u.size(); ++j) lc[j] = L(u[j], N);
    // 2. L(Gamma^lambda mod N^2) = lambda mod N (Gamma^lambda = 1 + lambda*N)
    Nat inv;
    if (!mod_inverse(Int(LambdaN % N), N, &inv)) throw EngineError(MPCX_EINVAL, "lambda not invertible mod N");
    // 3. m = L(c^lambda) * L(Gamma^lambda)^-1 mod N -- GPU mulmod
    std::vector<Nat> invs(lc.size(), inv);
    std::vector<Nat> r = Engine::get().mulmod(N, lc, invs);
    for (size_t j = 0; j < idx.size(); ++j) (*m)[idx[j]] = r[j];
    return;
  }
  const CrtDecrypt cd(*this);
  std::vector<Nat> up(cs.size()), uq(cs.size());
  run_concurrently({[&] { up = Engine::get().exp(cd.P2, cs, {cd.Pm1}); },
                    [&] { uq = Engine::get().exp(cd.Q2, cs, {cd.Qm1}); }});
  parallel_for(idx.size(), [&](size_t j) {
    const uint8_t e = cd.finish(up[j], uq[j], &(*m)[idx[j]]);
    if (e) (*err)[idx[j]] = e;
  });
}

// CRT form (same plaintext: every c in Z*_{N^2} is Gamma^m r^N for exactly one
// m in [0, N), and both formulas return that m). Per prime p of N:
//   m_p = L_p(c^(p-1) mod p^2) * h_p mod p,  L_p(u) = (u - 1) / p,
//   h_p = L_p(Gamma^(p-1) mod p^2)^-1 = ((p-1) * N / p mod p)^-1 mod p,
// then m = m_q + q * ((m_p - m_q) * q^-1 mod p). Two 1024-bit exponents mod
// 2048-bit moduli on the GPU instead of a 2047-bit exponent mod N^2: a
// quarter of the Montgomery work.
CrtDecrypt::CrtDecrypt(const PrivateKey& sk) : P(sk.P), Q(sk.Q) {
  const Nat one(1);
  P2 = P * P;
  Q2 = Q * Q;
  Pm1 = P - one;
  Qm1 = Q - one;
  auto h_of = [&](const Nat& p, const Nat& pm1, const Nat& other) {
    Nat h;  // (1 + N)^(p-1) = 1 + (p-1) N mod p^2, so L_p = (p-1) * other mod p
    if (!mod_inverse(Int(mulmod(pm1, other % p, p)), p, &h)) throw EngineError(MPCX_EINVAL, "Paillier key: bad factor");
    return h;
  };
  hP = h_of(P, Pm1, Q);
  hQ = h_of(Q, Qm1, P);
  if (!mod_inverse(Int(Q % P), P, &qinv)) throw EngineError(MPCX_EINVAL, "Paillier key: P, Q not coprime");
}

uint8_t CrtDecrypt::finish(const Nat& up, const Nat& uq, Nat* m) const {
  // p | c  <=>  c^(p-1) mod p^2 == 0 (p^2 | c^(p-1), p - 1 >= 2); otherwise it
  // is 1 mod p. tss-lib rejects such c (gcd(c, N^2) != 1) with ErrMessageMalFormed.
  if (up.is_zero() || uq.is_zero()) return ErrMessageMalFormed;
  const Nat mp = mulmod(L(up, P), hP, P), mq = mulmod(L(uq, Q), hQ, Q);
  const Nat mqp = mq % P;
  const Nat d = mp < mqp ? mp + P - mqp : mp - mqp;
  *m = mq + Q * mulmod(d, qinv, P);
  return OK;
}

}  // namespace mpcx::host::paillier
