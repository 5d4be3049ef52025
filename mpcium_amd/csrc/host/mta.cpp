// mta.cpp -- see mta.hpp. Every formula below cites the tss-lib v2.0.2 step it
// implements (restated in oracle/mta_ref.py and SURVEY.md 8(a) A8-A10).
#include "mta.hpp"

#include <algorithm>
#include <cstdlib>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <thread>

#include "engine.hpp"
#include "expset.hpp"
#include "hostprof.hpp"

namespace mpcx::host::mta {
namespace {

const Nat& q3() {
  static const Nat v = Q() * Q() * Q();
  return v;
}
const Nat& q5() {
  static const Nat v = q3() * Q() * Q();
  return v;
}
const Nat& q7() {
  static const Nat v = q3() * q3() * Q();
  return v;
}

// Gamma^k mod N^2 = (1 + N)^k = 1 + (k mod N) N  (binomial theorem; < N^2)
Nat gamma_pow(const Nat& k, const Nat& N) {
  MPCX_PROF("paillier.gamma_pow");
  return Nat(1) + (k % N) * N;
}

Nat affine_x(const secp::Affine& p) { return secp::FeToNat(p.x); }
Nat affine_y(const secp::Affine& p) { return secp::FeToNat(p.y); }

// mul * r^N mod N^2 requests of one launch step (Encrypt's c = Gamma^m r^N,
// the range proof's u = Gamma^alpha beta^N). With the key's factors at hand
// (Alice's own key in AliceInit) each runs as r^N mod P^2 and mod Q^2 --
// 2048-bit moduli, half the Montgomery work of one 4096-bit exponentiation,
// in the 2048-bit main geometry -- and is recombined on the host
// (x = x_Q + Q^2 ((x_P - x_Q) (Q^2)^-1 mod P^2)): the same residue mod N^2,
// bit-exact. Without them, mod N^2 as before. MPCX_INIT_CRT=0: always mod N^2
// (A/B runs).
class N2Step {
 public:
  N2Step(const paillier::PublicKey& pk, const paillier::PrivateKey* own) : N_(pk.N), N2_(pk.NSquare()) {
    static const bool on = [] {
      const char* e = std::getenv("MPCX_INIT_CRT");
      return !(e && e[0] == '0');
    }();
    crt_ = on && own && !own->P.is_zero() && !own->Q.is_zero() && own->P * own->Q == pk.N;
    if (crt_) {
      P2_ = own->P * own->P;
      Q2_ = own->Q * own->Q;
      if (!mod_inverse(Int(Q2_ % P2_), P2_, &q2inv_)) crt_ = false;
    }
    eN2_ = std::make_unique<ExpSet>(N2_);
    if (crt_) {
      eP2_ = std::make_unique<ExpSet>(P2_);
      eQ2_ = std::make_unique<ExpSet>(Q2_);
    }
  }
  // out = mul * r^N mod N^2; r, mul and out must outlive run()/finish()
  void add(const Nat& r, const Nat& mul, Nat* out) { reqs_.push_back({&r, &mul, out}); }
  // queue the launches (call run_all on sets() afterwards, then finish())
  void prepare() {
    if (!crt_) {
      for (const Req& q : reqs_) eN2_->add(*q.r, N_, q.out, q.mul);
      return;
    }
    const size_t n = reqs_.size();
    red_.assign(n, Red{});
    parallel_for(n, [&](size_t i) {
      const Req& q = reqs_[i];
      red_[i].rp = *q.r % P2_;
      red_[i].rq = *q.r % Q2_;
      red_[i].mp = *q.mul % P2_;
      red_[i].mq = *q.mul % Q2_;
    });
    for (size_t i = 0; i < n; ++i) {
      eP2_->add(red_[i].rp, N_, &red_[i].xp, &red_[i].mp);
      eQ2_->add(red_[i].rq, N_, &red_[i].xq, &red_[i].mq);
    }
  }
  std::vector<ExpSet*> sets() { return crt_ ? std::vector<ExpSet*>{eP2_.get(), eQ2_.get()} : std::vector<ExpSet*>{eN2_.get()}; }
  void finish() {
    if (crt_) {
      parallel_for(reqs_.size(), [&](size_t i) {
        const Red& r = red_[i];
        const Nat xqp = r.xq % P2_;
        const Nat d = r.xp < xqp ? r.xp + P2_ - xqp : r.xp - xqp;
        *reqs_[i].out = r.xq + Q2_ * ((d * q2inv_) % P2_);
      });
    }
    reqs_.clear();
    red_.clear();
  }

 private:
  struct Req {
    const Nat *r, *mul;
    Nat* out;
  };
  struct Red {
    Nat rp, rq, mp, mq, xp, xq;
  };
  const Nat N_, N2_;
  bool crt_ = false;
  Nat P2_, Q2_, q2inv_;
  std::unique_ptr<ExpSet> eN2_, eP2_, eQ2_;
  std::vector<Req> reqs_;
  std::vector<Red> red_;
};

// the launches of several sets and N2Steps of one protocol step at once
void run_step(std::initializer_list<ExpSet*> sets, N2Step* n2) {
  std::vector<std::function<void()>> fs;
  for (ExpSet* x : sets) x->collect(fs);
  if (n2) {
    n2->prepare();
    for (ExpSet* x : n2->sets()) x->collect(fs);
  }
  run_concurrently(fs);
  for (ExpSet* x : sets) x->clear();
  if (n2) {
    for (ExpSet* x : n2->sets()) x->clear();
    n2->finish();
  }
}

// ---- ProveRangeAlice in stages (shared by ProveRangeAliceBatch and AliceInitBatch)
struct RangeProveState {
  Nat alpha, beta, gamma, rho;
  Nat gam_alpha, e;
};

// steps 1-4 for every session, in each reader's draw order: alpha < q^3,
// beta in Z*_N (the batch's gcd decisions taken together), gamma < q^3 N~,
// rho < q N~; plus Gamma^alpha
void range_draw(std::vector<RangeProveState>& st, const paillier::PublicKey& pk, const DLNParams& dln,
                const std::vector<RandFn>& rand) {
  const size_t n = st.size();
  parallel_for(n, [&](size_t i) { st[i].alpha = GetRandomPositiveInt(rand[i], q3()); });
  std::vector<const RandFn*> rd(n);
  std::vector<Nat*> beta(n);
  for (size_t i = 0; i < n; ++i) {
    rd[i] = &rand[i];
    beta[i] = &st[i].beta;
  }
  GetRandomPositiveRelativelyPrimeIntBatch(rd, pk.N, beta);
  const Nat q3Nt = q3() * dln.NTilde, qNt = Q() * dln.NTilde;
  parallel_for(n, [&](size_t i) {
    st[i].gamma = GetRandomPositiveInt(rand[i], q3Nt);
    st[i].rho = GetRandomPositiveInt(rand[i], qNt);
    st[i].gam_alpha = gamma_pow(st[i].alpha, pk.N);
  });
}

}  // namespace

const Nat& Q() { return secp::CurveN(); }

// ================================================================ RangeProofAlice
namespace {
// Steps 5-11 of ProveRangeAlice for drawn states st (range_draw), c[i] the
// ciphertext session i proves. eN2 may already hold the caller's own requests
// (AliceInit's Encrypt): they run in the proof's first launches, and c[i] is
// read only after them (the challenge hashes it).
void range_prove_core(const paillier::PublicKey& pk, const DLNParams& dln, const std::vector<const Nat*>& c,
                      const std::vector<Nat>& m, const std::vector<Nat>& r, std::vector<RangeProveState>& st,
                      N2Step& eN2, std::vector<RangeProofAlice>* out) {
  const size_t n = st.size();
  out->assign(n, RangeProofAlice{});
  ExpSet eNt(dln.NTilde), eN(pk.N);
  for (size_t i = 0; i < n; ++i) {
    auto& s = st[i];
    auto& o = (*out)[i];
    eN2.add(s.beta, s.gam_alpha, &o.U);                      // 6. u = Gamma^alpha beta^N mod N^2
    eNt.add2(dln.h1, m[i], dln.h2, s.rho, &o.Z);             // 5. z = h1^m h2^rho mod N~
    eNt.add2(dln.h1, s.alpha, dln.h2, s.gamma, &o.W);        // 7. w = h1^alpha h2^gamma mod N~
  }
  run_step({&eNt}, &eN2);
  const Nat gamma = pk.Gamma();
  parallel_for(n, [&](size_t i) {  // 8-9. e = RejectionSample(q, SHA512_256i(N, Gamma, c, z, u, w))
    auto& o = (*out)[i];
    st[i].e = RejectionSample(Q(), SHA512_256i({&pk.N, &gamma, c[i], &o.Z, &o.U, &o.W}));
  });
  for (size_t i = 0; i < n; ++i) eN.add(r[i], st[i].e, &(*out)[i].S, &st[i].beta);  // s = r^e beta mod N
  eN.run();
  parallel_for(n, [&](size_t i) {
    auto& o = (*out)[i];
    o.S1 = st[i].e * m[i] + st[i].alpha;    // s1 = e m + alpha
    o.S2 = st[i].e * st[i].rho + st[i].gamma;  // s2 = e rho + gamma
  });
}
}  // namespace

void ProveRangeAliceBatch(const paillier::PublicKey& pk, const DLNParams& dln, const std::vector<Nat>& c,
                          const std::vector<Nat>& m, const std::vector<Nat>& r, const std::vector<RandFn>& rand,
                          std::vector<RangeProofAlice>* out) {
  const size_t n = c.size();
  if (m.size() != n || r.size() != n || rand.size() != n) throw std::invalid_argument("ProveRangeAlice: sizes");
  std::vector<RangeProveState> st(n);
  range_draw(st, pk, dln, rand);
  std::vector<const Nat*> cp(n);
  for (size_t i = 0; i < n; ++i) cp[i] = &c[i];
  N2Step eN2(pk, nullptr);
  range_prove_core(pk, dln, cp, m, r, st, eN2, out);
}

std::vector<uint8_t> VerifyRangeAliceBatch(const paillier::PublicKey& pk, const DLNParams& dln,
                                           const std::vector<Nat>& c, const std::vector<RangeProofAlice>& pf) {
  const size_t n = c.size();
  if (pf.size() != n) throw std::invalid_argument("RangeProofAlice.Verify: sizes");
  const Nat N2 = pk.NSquare();
  const Nat gamma = pk.Gamma();
  std::vector<uint8_t> ok(n, 0);
  std::vector<Nat> e(n), gs1(n), L1(n), R1(n), L2(n), R2(n), cr(n);
  parallel_for(n, [&](size_t i) {
    MPCX_PROF("mta.verify_range.checks");
    const auto& p = pf[i];
    if (!IsInInterval(p.Z, dln.NTilde) || !IsInInterval(p.U, N2) || !IsInInterval(p.W, dln.NTilde) ||
        !IsInInterval(p.S, pk.N))
      return;
    if (p.S1 > q3()) return;
    // Go's Exp(c, -e, N^2) accepts any c invertible mod N^2 (c >= N^2 is
    // reduced by ModInverse); a non-invertible c gives nil and the following
    // Mul panics -- reported here as a verification failure. The hash binds
    // the caller's c as given.
    cr[i] = c[i] < N2 ? c[i] : c[i] % N2;
    ok[i] = 1;
  });
  {  // z, w in Z*_N~ and u, s, c in Z*_N: the batch's gcd decisions together
    std::vector<size_t> sel;
    std::vector<const Nat*> xt, xn;
    for (size_t i = 0; i < n; ++i)
      if (ok[i]) {
        sel.push_back(i);
        xt.insert(xt.end(), {&pf[i].Z, &pf[i].W});
        xn.insert(xn.end(), {&pf[i].U, &pf[i].S, &cr[i]});
      }
    const std::vector<uint8_t> ct = CoprimeMany(xt, dln.NTilde), cn = CoprimeMany(xn, pk.N);
    for (size_t j = 0; j < sel.size(); ++j)
      ok[sel[j]] = ct[2 * j] && ct[2 * j + 1] && cn[3 * j] && cn[3 * j + 1] && cn[3 * j + 2];
  }
  parallel_for(n, [&](size_t i) {
    if (!ok[i]) return;
    const auto& p = pf[i];
    e[i] = RejectionSample(Q(), SHA512_256i({&pk.N, &gamma, &c[i], &p.Z, &p.U, &p.W}));
    gs1[i] = gamma_pow(p.S1, pk.N);
  });
  ExpSet eN2(N2), eNt(dln.NTilde);
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) continue;
    const auto& p = pf[i];
    eN2.add(cr[i], e[i], &L1[i], &p.U);     // u c^e
    eN2.add(p.S, pk.N, &R1[i], &gs1[i]);    // Gamma^s1 s^N
    eNt.add2(dln.h1, p.S1, dln.h2, p.S2, &R2[i]);  // h1^s1 h2^s2
    eNt.add(p.Z, e[i], &L2[i], &p.W);             // w z^e
  }
  run_all({&eN2, &eNt});
  for (size_t i = 0; i < n; ++i) ok[i] = ok[i] && L1[i] == R1[i] && L2[i] == R2[i];
  return ok;
}

// ================================================================ ProofBob[WC]
namespace {
struct BobProveState {
  Nat alpha, rho, sigma, tau, rhoPrm, beta, gamma;
  secp::Affine u;
  Nat bg, c1a, e;  // Gamma^gamma beta^N, c1^alpha
  bool wc = false;  // ProveBobWC (u = alpha*G)
};

// steps 1-4 (+5 for WC states) for the sessions st[js[k]] with readers rd[k],
// in each reader's draw order alpha, rho, sigma, tau, rhoPrm, beta, gamma (the
// beta gcd decisions taken together)
void bob_draw(std::vector<BobProveState>& st, const std::vector<size_t>& js, const std::vector<const RandFn*>& rd,
              const paillier::PublicKey& pk, const DLNParams& dln) {
  const size_t n = js.size();
  const Nat qNt = Q() * dln.NTilde, q3Nt = q3() * dln.NTilde;
  parallel_for(n, [&](size_t k) {
    BobProveState& s = st[js[k]];
    const RandFn& rand = *rd[k];
    s.alpha = GetRandomPositiveInt(rand, q3());
    s.rho = GetRandomPositiveInt(rand, qNt);
    s.sigma = GetRandomPositiveInt(rand, qNt);
    s.tau = GetRandomPositiveInt(rand, q3Nt);
    s.rhoPrm = GetRandomPositiveInt(rand, q3Nt);
  });
  std::vector<Nat*> beta(n);
  for (size_t k = 0; k < n; ++k) beta[k] = &st[js[k]].beta;
  GetRandomPositiveRelativelyPrimeIntBatch(rd, pk.N, beta);
  parallel_for(n, [&](size_t k) { st[js[k]].gamma = GetRandomPositiveInt(*rd[k], q7()); });
  // 5. u = alpha*G of every WC session, one GPU batch (k_ec_combine)
  std::vector<secp::Comb> cu;
  std::vector<size_t> wc;
  for (size_t k = 0; k < n; ++k)
    if (st[js[k]].wc) {
      wc.push_back(js[k]);
      cu.emplace_back();
      cu.back().a = st[js[k]].alpha;
    }
  const std::vector<secp::Affine> u = secp::CombineBatch(cu);
  for (size_t k = 0; k < wc.size(); ++k) st[wc[k]].u = u[k];
}

// the exponentiations of ProveBob before its challenge, one launch step:
// N^2 -> bg = Gamma^gamma beta^N and c1^alpha; N~ -> z, z', t, w (6-9, 10.),
// each h1^x h2^y one two-table comb product
void bob_stage_a(BobProveState& s, const paillier::PublicKey& pk, const DLNParams& dln, const Nat& c1, const Nat& x,
                 const Nat& y, ExpSet& eN2, ExpSet& eNt, Nat* gam_gamma, ProofBob& o) {
  *gam_gamma = gamma_pow(s.gamma, pk.N);
  eN2.add(s.beta, pk.N, &s.bg, gam_gamma);
  eN2.add(c1, s.alpha, &s.c1a);
  eNt.add2(dln.h1, x, dln.h2, s.rho, &o.Z);           // z = h1^x h2^rho
  eNt.add2(dln.h1, s.alpha, dln.h2, s.rhoPrm, &o.ZPrm);  // z' = h1^alpha h2^rhoPrm
  eNt.add2(dln.h1, y, dln.h2, s.sigma, &o.T);          // t = h1^y h2^sigma
  eNt.add2(dln.h1, s.gamma, dln.h2, s.tau, &o.W);      // w = h1^gamma h2^tau
}

// 9. v = c1^alpha Gamma^gamma beta^N: the two factors of stage A multiplied on
// the host (a 4096-bit product) instead of a second launch step that waited
// for bg (round 4)
void bob_stage_b(BobProveState& s, const Nat& N2, ProofBob& o) { o.V = (s.c1a * s.bg) % N2; }

// 11-12. e = RejectionSample(q, SHA512_256i_TAGGED(Session, N, Gamma, [X.x, X.y,] c1, c2, [u.x, u.y,] z, z', t, v, w))
Nat bob_challenge(const Bytes& session, const paillier::PublicKey& pk, const Nat& gamma, const secp::Affine* X,
                  const Nat& c1, const Nat& c2, const ProofBob& p) {
  if (!X) return RejectionSample(Q(), SHA512_256i_TAGGED(session, {&pk.N, &gamma, &c1, &c2, &p.Z, &p.ZPrm, &p.T,
                                                                     &p.V, &p.W}));
  const Nat Xx = affine_x(*X), Xy = affine_y(*X), ux = affine_x(p.U), uy = affine_y(p.U);
  return RejectionSample(Q(), SHA512_256i_TAGGED(session, {&pk.N, &gamma, &Xx, &Xy, &c1, &c2, &ux, &uy, &p.Z,
                                                           &p.ZPrm, &p.T, &p.V, &p.W}));
}

// 13. s1 = e x + alpha, s2 = e rho + rhoPrm, t1 = e y + gamma, t2 = e sigma + tau
void bob_responses(const BobProveState& s, const Nat& x, const Nat& y, ProofBob& o) {
  o.S1 = s.e * x + s.alpha;
  o.S2 = s.e * s.rho + s.rhoPrm;
  o.T1 = s.e * y + s.gamma;
  o.T2 = s.e * s.sigma + s.tau;
  o.U = s.u;
}
}  // namespace

void ProveBobBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pk, const DLNParams& dln,
                   const std::vector<Nat>& c1, const std::vector<Nat>& c2, const std::vector<Nat>& x,
                   const std::vector<Nat>& y, const std::vector<Nat>& r, const std::vector<secp::Affine>* X,
                   const std::vector<RandFn>& rand, std::vector<ProofBob>* out) {
  const size_t n = c1.size();
  if (session.size() != n || c2.size() != n || x.size() != n || y.size() != n || r.size() != n ||
      rand.size() != n || (X && X->size() != n))
    throw std::invalid_argument("ProveBob: sizes");
  const Nat N2 = pk.NSquare(), gamma = pk.Gamma();
  std::vector<BobProveState> st(n);
  std::vector<Nat> gg(n);
  out->assign(n, ProofBob{});
  {
    std::vector<size_t> js(n);
    std::vector<const RandFn*> rd(n);
    for (size_t i = 0; i < n; ++i) {
      js[i] = i;
      rd[i] = &rand[i];
      st[i].wc = X != nullptr;
    }
    bob_draw(st, js, rd, pk, dln);
  }
  ExpSet eN2(N2), eNt(dln.NTilde), eN(pk.N);
  for (size_t i = 0; i < n; ++i) bob_stage_a(st[i], pk, dln, c1[i], x[i], y[i], eN2, eNt, &gg[i], (*out)[i]);
  run_all({&eN2, &eNt});
  parallel_for(n, [&](size_t i) {
    bob_stage_b(st[i], N2, (*out)[i]);
    (*out)[i].U = st[i].u;
    st[i].e = bob_challenge(session[i], pk, gamma, X ? &(*X)[i] : nullptr, c1[i], c2[i], (*out)[i]);
  });
  for (size_t i = 0; i < n; ++i) eN.add(r[i], st[i].e, &(*out)[i].S, &st[i].beta);  // s = r^e beta mod N
  eN.run();
  parallel_for(n, [&](size_t i) { bob_responses(st[i], x[i], y[i], (*out)[i]); });
}

namespace {
// Decrypt(cB) mod q of every session whose proof verified
void alice_decrypt(const paillier::PrivateKey& skA, const std::vector<const Nat*>& cB, const std::vector<uint8_t>& ok,
                   const std::vector<Nat*>& alpha, const std::vector<uint8_t*>& err) {
  std::vector<Int> cs;
  std::vector<size_t> idx;
  for (size_t i = 0; i < cB.size(); ++i) {
    if (!ok[i]) {
      *err[i] = ErrProofVerify;
      continue;
    }
    idx.push_back(i);
    cs.push_back(Int(*cB[i]));
  }
  std::vector<Nat> m;
  std::vector<uint8_t> derr;
  skA.DecryptBatch(cs, &m, &derr);
  for (size_t j = 0; j < idx.size(); ++j) {
    if (derr[j]) *err[idx[j]] = derr[j];
    else *alpha[idx[j]] = m[j] % Q();
  }
}
// ProofBob[WC].Verify of session i's proof *pfp[i], X[i] == nullptr for a
// plain ProofBob: one batch may mix both kinds (AliceEnd and AliceEndWC of one
// pair share every modulus).
std::vector<uint8_t> verify_bob_core(const std::vector<const Bytes*>& session, const paillier::PublicKey& pk,
                                     const DLNParams& dln, const std::vector<const Nat*>& c1,
                                     const std::vector<const Nat*>& c2, const std::vector<const ProofBob*>& pfp,
                                     const std::vector<const secp::Affine*>& X, const paillier::PrivateKey* own,
                                     const std::vector<Nat*>* dec = nullptr,
                                     const std::vector<uint8_t*>* dec_err = nullptr) {
  const size_t n = c1.size();
  const Nat N2 = pk.NSquare(), gamma = pk.Gamma();
  std::vector<uint8_t> ok(n, 0);
  std::vector<Nat> e(n), gt1(n), r1(n), r2(n), q1(n), r3(n), l1(n), l2(n), l3(n);
  parallel_for(n, [&](size_t i) {
    MPCX_PROF("mta.verify_bob.checks");
    const auto& p = *pfp[i];
    if (X[i] && !secp::IsOnCurve(p.U)) return;
    const Nat& Nt = dln.NTilde;
    for (const Nat* v : {&p.Z, &p.ZPrm, &p.T, &p.W})
      if (!IsInInterval(*v, Nt)) return;
    if (!IsInInterval(p.V, N2) || !IsInInterval(p.S, pk.N)) return;
    // 3. s1 <= q^3, t1 <= q^7 (tss-lib v2's Alpha-Rays range checks: betaPrm < q^5,
    // gamma < q^7, so an honest t1 = e betaPrm + gamma < q^6 + q^7)
    if (p.S1 > q3() || p.T1 > q7()) return;
    ok[i] = 1;
  });
  {  // z, z', t, w in Z*_N~ and v, s in Z*_N: the batch's gcd decisions together
    std::vector<size_t> sel;
    std::vector<const Nat*> xt, xn;
    for (size_t i = 0; i < n; ++i)
      if (ok[i]) {
        sel.push_back(i);
        xt.insert(xt.end(), {&pfp[i]->Z, &pfp[i]->ZPrm, &pfp[i]->T, &pfp[i]->W});
        xn.insert(xn.end(), {&pfp[i]->V, &pfp[i]->S});
      }
    const std::vector<uint8_t> ct = CoprimeMany(xt, dln.NTilde), cn = CoprimeMany(xn, pk.N);
    for (size_t j = 0; j < sel.size(); ++j)
      ok[sel[j]] = ct[4 * j] && ct[4 * j + 1] && ct[4 * j + 2] && ct[4 * j + 3] && cn[2 * j] && cn[2 * j + 1];
  }
  // 4. (WC) s1*G == e*X + u, rejected when e*X + u is the point at infinity
  // (Go: xEU nil). Evaluated as one combination T = s1*G + (q - e)*X compared
  // with u: T == u  <=>  s1*G == e*X + u as group elements, and when that
  // holds, e*X + u = infinity  <=>  s1*G = infinity  <=>  s1 == 0 (mod q).
  // Every session's combination in one GPU batch (k_ec_combine).
  std::vector<secp::Comb> cw(n);
  std::vector<uint8_t> is_wc(n, 0);
  parallel_for(n, [&](size_t i) {
    if (!ok[i]) return;
    const auto& p = *pfp[i];
    e[i] = bob_challenge(*session[i], pk, gamma, X[i], *c1[i], *c2[i], p);
    if (X[i]) {
      const Nat s1q = p.S1 % Q();
      if (s1q.is_zero()) {
        ok[i] = 0;
        return;
      }
      const Nat eq = e[i] % Q();
      cw[i].a = s1q;
      cw[i].P = *X[i];
      cw[i].b = eq.is_zero() ? eq : Q() - eq;
      is_wc[i] = 1;
    }
    gt1[i] = gamma_pow(p.T1, pk.N);
  });
  {
    std::vector<secp::Comb> items;
    std::vector<size_t> idx;
    for (size_t i = 0; i < n; ++i)
      if (ok[i] && is_wc[i]) {
        idx.push_back(i);
        items.push_back(std::move(cw[i]));
      }
    const std::vector<secp::Affine> T = secp::CombineBatch(items);
    for (size_t k = 0; k < idx.size(); ++k)
      if (!secp::Equal(T[k], pfp[idx[k]]->U)) ok[idx[k]] = 0;
  }
  // Equation 7 holds mod N^2 iff it holds mod P^2 and mod Q^2 (CRT): the key
  // holder (AliceEnd) checks it on the two half-width moduli, a quarter of the
  // Montgomery work each; everyone else mod N^2.
  static const bool crt_on = [] {  // MPCX_VERIFY_CRT=0: mod N^2 also for the key holder (A/B runs)
    const char* e = std::getenv("MPCX_VERIFY_CRT");
    return !(e && e[0] == '0');
  }();
  // the factors must be the key's: otherwise mod N^2 for the
  // verification and alice_decrypt's own fallback for the plaintexts
  const bool crt = crt_on && own && !own->P.is_zero() && !own->Q.is_zero() && own->P * own->Q == pk.N;
  // With the key's factors every exponentiation of the verification -- and,
  // when asked (AliceEnd), the CRT decryption of c2 -- is independent of the
  // others: ONE launch step. c1^s1 runs without a multiplier and is multiplied
  // into s^N Gamma^t1 on the host (a 2048-bit product per half), where the
  // form below chains it behind the first step.
  std::unique_ptr<paillier::CrtDecrypt> cd;
  if (crt) cd = std::make_unique<paillier::CrtDecrypt>(*own);
  const Nat& P2 = crt ? cd->P2 : N2;
  const Nat& Q2 = crt ? cd->Q2 : N2;
  const bool decrypt = crt && dec;
  struct Red {  // s, c1, c2, v, Gamma^t1 reduced mod P^2 and Q^2
    Nat s, c1, c2, v, g;
  };
  std::vector<Red> rp(crt ? n : 0), rq(crt ? n : 0);
  std::vector<Nat> q1q(crt ? n : 0), r3q(crt ? n : 0), l3q(crt ? n : 0), up(decrypt ? n : 0), uq(decrypt ? n : 0);
  std::vector<uint8_t> dec_ok(decrypt ? n : 0, 0);  // c2 < N^2: Decrypt's range check
  if (crt) {
    parallel_for(n, [&](size_t i) {
      if (!ok[i]) return;
      const auto& p = *pfp[i];
      for (int h = 0; h < 2; ++h) {
        const Nat& m = h ? Q2 : P2;
        Red& r = h ? rq[i] : rp[i];
        r.s = p.S % m;
        r.c1 = *c1[i] % m;
        r.c2 = *c2[i] % m;
        r.v = p.V % m;
        r.g = gt1[i] % m;
      }
      if (decrypt) dec_ok[i] = *c2[i] < N2;
    });
  }
  ExpSet eN2(P2), eQ2(Q2), eNt(dln.NTilde);
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) continue;
    const auto& p = *pfp[i];
    eNt.add2(dln.h1, p.S1, dln.h2, p.S2, &l1[i]);  // 5. h1^s1 h2^s2
    eNt.add2(dln.h1, p.T1, dln.h2, p.T2, &l2[i]);  // 6. h1^t1 h2^t2
    eNt.add(p.Z, e[i], &r1[i], &p.ZPrm);    // 5. z^e z'
    eNt.add(p.T, e[i], &r2[i], &p.W);       // 6. t^e w
    if (crt) {
      eN2.add(rp[i].s, pk.N, &q1[i], &rp[i].g);   // 7. s^N Gamma^t1 mod P^2
      eN2.add(rp[i].c2, e[i], &r3[i], &rp[i].v);  // 7. c2^e v mod P^2
      eN2.add(rp[i].c1, p.S1, &l3[i]);            // 7. c1^s1 mod P^2
      eQ2.add(rq[i].s, pk.N, &q1q[i], &rq[i].g);  //    and mod Q^2
      eQ2.add(rq[i].c2, e[i], &r3q[i], &rq[i].v);
      eQ2.add(rq[i].c1, p.S1, &l3q[i]);
      if (decrypt && dec_ok[i]) {
        eN2.add(rp[i].c2, cd->Pm1, &up[i]);  // Decrypt(c2): c2^(P-1) mod P^2
        eQ2.add(rq[i].c2, cd->Qm1, &uq[i]);  //              c2^(Q-1) mod Q^2
      }
    } else {
      eN2.add(p.S, pk.N, &q1[i], &gt1[i]);    // 7. s^N Gamma^t1
      eN2.add(*c2[i], e[i], &r3[i], &p.V);    // 7. c2^e v
    }
  }
  run_all({&eN2, &eQ2, &eNt});
  if (crt) {
    parallel_for(n, [&](size_t i) {  // 7. c1^s1 s^N Gamma^t1 mod P^2 and mod Q^2
      if (!ok[i]) return;
      l3[i] = (l3[i] * q1[i]) % P2;
      l3q[i] = (l3q[i] * q1q[i]) % Q2;
    });
  } else {
    for (size_t i = 0; i < n; ++i)
      if (ok[i]) eN2.add(*c1[i], pfp[i]->S1, &l3[i], &q1[i]);  // 7. c1^s1 s^N Gamma^t1
    eN2.run();
  }
  for (size_t i = 0; i < n; ++i)
    ok[i] = ok[i] && l1[i] == r1[i] && l2[i] == r2[i] && l3[i] == r3[i] && (!crt || l3q[i] == r3q[i]);
  if (dec) {  // AliceEnd: Decrypt(c2) mod q of every session whose proof verified
    if (decrypt) {
      parallel_for(n, [&](size_t i) {
        if (!ok[i]) {
          *(*dec_err)[i] = ErrProofVerify;
        } else if (!dec_ok[i]) {
          *(*dec_err)[i] = ErrMessageTooLong;
        } else {
          Nat m;
          const uint8_t de = cd->finish(up[i], uq[i], &m);
          if (de) *(*dec_err)[i] = de;
          else *(*dec)[i] = m % Q();
        }
      });
    } else {
      alice_decrypt(*own, c2, ok, *dec, *dec_err);
    }
  }
  return ok;
}
}  // namespace

std::vector<uint8_t> VerifyBobBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pk,
                                    const DLNParams& dln, const std::vector<Nat>& c1, const std::vector<Nat>& c2,
                                    const std::vector<ProofBob>& pf, const std::vector<secp::Affine>* X,
                                    const paillier::PrivateKey* own_sk) {
  const size_t n = c1.size();
  if (session.size() != n || c2.size() != n || pf.size() != n || (X && X->size() != n))
    throw std::invalid_argument("ProofBob.Verify: sizes");
  // own_sk: the verifier's own key (equation 7 checked mod P^2 and Q^2)
  std::vector<const Bytes*> sp(n);
  std::vector<const Nat*> c1p(n), c2p(n);
  std::vector<const ProofBob*> pfp(n);
  std::vector<const secp::Affine*> Xp(n, nullptr);
  for (size_t i = 0; i < n; ++i) {
    sp[i] = &session[i];
    c1p[i] = &c1[i];
    c2p[i] = &c2[i];
    pfp[i] = &pf[i];
    if (X) Xp[i] = &(*X)[i];
  }
  return verify_bob_core(sp, pk, dln, c1p, c2p, pfp, Xp, own_sk);
}

// ================================================================ protocol
void AliceInitBatch(const paillier::PublicKey& pkA, const std::vector<Nat>& a, const DLNParams& dlnB,
                    const std::vector<RandFn>& rand, std::vector<Nat>* cA, std::vector<RangeProofAlice>* pf,
                    std::vector<uint8_t>* err, const paillier::PrivateKey* skA) {
  const size_t n = a.size();
  if (rand.size() != n) throw std::invalid_argument("AliceInit: sizes");
  cA->assign(n, Nat());
  err->assign(n, OK);
  // EncryptAndReturnRandomness: 0 <= a < N, then r in Z*_N
  std::vector<size_t> idx;
  for (size_t i = 0; i < n; ++i) {
    if (!(a[i] < pkA.N)) (*err)[i] = ErrMessageTooLong;
    else idx.push_back(i);
  }
  const size_t k = idx.size();
  std::vector<Nat> r(k), ga(k), c(k), m(k);
  std::vector<RandFn> rd(k);
  {
    std::vector<const RandFn*> rdr(k);
    std::vector<Nat*> rp(k);
    for (size_t j = 0; j < k; ++j) {
      rdr[j] = &rand[idx[j]];
      rp[j] = &r[j];
      m[j] = a[idx[j]];
      rd[j] = rand[idx[j]];
    }
    GetRandomPositiveRelativelyPrimeIntBatch(rdr, pkA.N, rp);
  }
  // every reader's ProveRangeAlice draws follow its Encrypt draw, so all are
  // taken before the first launch: c = Gamma^a r^N then runs in the proof's
  // first launches (same modulus and exponent as its u = Gamma^alpha beta^N)
  std::vector<RangeProveState> st(k);
  range_draw(st, pkA, dlnB, rd);
  parallel_for(k, [&](size_t j) { ga[j] = gamma_pow(m[j], pkA.N); });
  N2Step eN2(pkA, skA);  // Alice's own key: c and u by CRT mod P^2, Q^2
  std::vector<const Nat*> cp(k);
  for (size_t j = 0; j < k; ++j) {
    eN2.add(r[j], ga[j], &c[j]);  // c = Gamma^a r^N mod N^2
    cp[j] = &c[j];
  }
  std::vector<RangeProofAlice> p;
  range_prove_core(pkA, dlnB, cp, m, r, st, eN2, &p);
  pf->assign(n, RangeProofAlice{});
  for (size_t j = 0; j < k; ++j) {
    (*cA)[idx[j]] = c[j];
    (*pf)[idx[j]] = std::move(p[j]);
  }
}

namespace {
// f and g on two threads; rethrows the first failure
void both(const std::function<void()>& f, const std::function<void()>& g) {
  std::exception_ptr ef, eg;
  const int chain = prof::chain();
  std::thread t([&, chain] {
    MPCX_PROF_CPU("cpu.mta_halves");
    prof::set_chain(chain);
    try {
      g();
    } catch (...) {
      eg = std::current_exception();
    }
  });
  try {
    f();
  } catch (...) {
    ef = std::current_exception();
  }
  t.join();
  if (ef) std::rethrow_exception(ef);
  if (eg) std::rethrow_exception(eg);
}

// One BobMid[WC] half of a session whose RangeProofAlice verified: its b, its
// point B (nullptr: plain BobMid), its reader and its result slots.
struct BobHalf {
  size_t i;  // session index (session id, cA)
  const Nat* b;
  const secp::Affine* B;
  const RandFn* rd;
  BobMidResult* out;
  uint8_t* err;
};

// Everything of BobMid[WC] after pf.Verify, for any mix of plain and WC halves
// on one Alice key: every half's draws in its own reader's order, and each
// step's exponentiations of all halves in shared launches.
void bob_mid_halves(const std::vector<Bytes>& session, const paillier::PublicKey& pkA, const DLNParams& dlnA,
                    const std::vector<Nat>& cA, const std::vector<BobHalf>& h) {
  const size_t k = h.size();
  const Nat N2 = pkA.NSquare(), gamma = pkA.Gamma();
  std::vector<BobProveState> st(k);
  std::vector<Nat> cRand(k), gbp(k), cbp(k), gg(k);
  std::vector<uint8_t> live(k, 0);
  {
    MPCX_PROF("mta.bob_mid.draws");
    std::vector<const RandFn*> rd(k);
    std::vector<Nat*> cr(k);
    for (size_t j = 0; j < k; ++j) {
      rd[j] = h[j].rd;
      cr[j] = &cRand[j];
    }
    // betaPrm < q^5 (tss-lib v2 BobMid), then the Encrypt(betaPrm) randomness in Z*_N
    parallel_for(k, [&](size_t j) { h[j].out->betaPrm = GetRandomPositiveInt(*rd[j], q5()); });
    GetRandomPositiveRelativelyPrimeIntBatch(rd, pkA.N, cr);
    std::vector<size_t> js;
    std::vector<const RandFn*> rdj;
    for (size_t j = 0; j < k; ++j) {
      gbp[j] = gamma_pow(h[j].out->betaPrm, pkA.N);
      // HomoMult(b, cA): 0 <= b < N and 0 <= cA < N^2, else ErrMessageTooLong
      // (RangeProofAlice.Verify accepts any invertible cA, so a verified cA may
      // still be >= N^2); it fails after Encrypt's draws, before ProveBob's
      if (!(*h[j].b < pkA.N) || !(cA[h[j].i] < N2)) {
        *h[j].err = ErrMessageTooLong;
        continue;
      }
      live[j] = 1;
      st[j].wc = h[j].B != nullptr;
      js.push_back(j);
      rdj.push_back(rd[j]);
    }
    bob_draw(st, js, rdj, pkA, dlnA);  // ProveBob[WC] steps 1-5
  }
  // every exponentiation before the challenge in ONE launch step: Encrypt's
  // r^N, HomoMult's cA^b and ProveBob's stage A (c^b and cA^alpha multiplied
  // into their products on the host below)
  std::vector<Nat> cab(k);
  ExpSet eN2(N2), eNt(dlnA.NTilde), eN(pkA.N);
  for (size_t j = 0; j < k; ++j) {
    if (!live[j]) continue;
    const Nat& c = cA[h[j].i];
    eN2.add(cRand[j], pkA.N, &cbp[j], &gbp[j]);  // cBetaPrm = Gamma^betaPrm r^N
    eN2.add(c, *h[j].b, &cab[j]);                // HomoMult(b, cA) = cA^b
    bob_stage_a(st[j], pkA, dlnA, c, *h[j].b, h[j].out->betaPrm, eN2, eNt, &gg[j], h[j].out->pf);
  }
  run_all({&eN2, &eNt});
  parallel_for(k, [&](size_t j) {
    if (!live[j]) return;
    auto& o = *h[j].out;
    o.cB = (cab[j] * cbp[j]) % N2;  // cB = HomoAdd(HomoMult(b, cA), cBetaPrm)
    bob_stage_b(st[j], N2, o.pf);
    o.beta = (Q() - o.betaPrm % Q()) % Q();  // beta = ModInt(q).Sub(0, betaPrm)
    o.pf.U = st[j].u;
    st[j].e = bob_challenge(session[h[j].i], pkA, gamma, h[j].B, cA[h[j].i], o.cB, o.pf);
  });
  for (size_t j = 0; j < k; ++j)
    if (live[j]) eN.add(cRand[j], st[j].e, &h[j].out->pf.S, &st[j].beta);  // s = r^e beta mod N
  eN.run();
  parallel_for(k, [&](size_t j) {
    if (live[j]) bob_responses(st[j], *h[j].b, h[j].out->betaPrm, h[j].out->pf);
  });
}
}  // namespace

void BobMidBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pkA,
                 const std::vector<RangeProofAlice>& pf, const std::vector<Nat>& b, const std::vector<Nat>& cA,
                 const DLNParams& dlnA, const DLNParams& dlnB, const std::vector<secp::Affine>* B,
                 const std::vector<RandFn>& rand, std::vector<BobMidResult>* out, std::vector<uint8_t>* err) {
  const size_t n = cA.size();
  if (session.size() != n || pf.size() != n || b.size() != n || rand.size() != n || (B && B->size() != n))
    throw std::invalid_argument("BobMid: sizes");
  out->assign(n, BobMidResult{});
  err->assign(n, OK);
  // RangeProofAlice.Verify(ec, pkA, NTildeB, h1B, h2B, cA)
  const std::vector<uint8_t> ok = VerifyRangeAliceBatch(pkA, dlnB, cA, pf);
  // HomoMult's range checks (b < N, cA < N^2) follow the draws of betaPrm and
  // the Encrypt randomness, as in Go (bob_mid_halves).
  std::vector<BobHalf> h;
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) (*err)[i] = ErrProofVerify;
    else h.push_back({i, &b[i], B ? &(*B)[i] : nullptr, &rand[i], &(*out)[i], &(*err)[i]});
  }
  bob_mid_halves(session, pkA, dlnA, cA, h);
}

void BobMidPairBatch(const std::vector<Bytes>& session, const paillier::PublicKey& pkA,
                     const std::vector<RangeProofAlice>& pf, const std::vector<Nat>& b, const std::vector<Nat>& bwc,
                     const std::vector<Nat>& cA, const DLNParams& dlnA, const DLNParams& dlnB,
                     const std::vector<secp::Affine>& Bwc, const std::vector<RandFn>& rand,
                     const std::vector<RandFn>& randwc, std::vector<BobMidResult>* out,
                     std::vector<BobMidResult>* outwc, std::vector<uint8_t>* err, std::vector<uint8_t>* errwc,
                     bool serial_halves) {
  const size_t n = cA.size();
  if (session.size() != n || pf.size() != n || b.size() != n || bwc.size() != n || Bwc.size() != n ||
      rand.size() != n || randwc.size() != n)
    throw std::invalid_argument("BobMidPair: sizes");
  out->assign(n, BobMidResult{});
  outwc->assign(n, BobMidResult{});
  err->assign(n, OK);
  errwc->assign(n, OK);
  // Both halves verify the same (cA, pf) under the same key: one verification
  // decides both (Verify is a pure function of its inputs)
  const std::vector<uint8_t> ok = VerifyRangeAliceBatch(pkA, dlnB, cA, pf);
  std::vector<BobHalf> h, hwc;
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i]) {
      (*err)[i] = (*errwc)[i] = ErrProofVerify;
      continue;
    }
    h.push_back({i, &b[i], nullptr, &rand[i], &(*out)[i], &(*err)[i]});
    hwc.push_back({i, &bwc[i], &Bwc[i], &randwc[i], &(*outwc)[i], &(*errwc)[i]});
  }
  // the two halves as concurrent tasks: one half's host phases (draws, hashing,
  // gcd batches) overlap the other's launches (measured faster on MI355X than
  // one merged batch of both halves, whose host and GPU phases alternate)
  // (serial_halves: the caller passed one reader object for both halves of a
  // session -- BobMid's draws, then BobMidWC's, as two calls in that order)
  if (serial_halves) {
    bob_mid_halves(session, pkA, dlnA, cA, h);
    bob_mid_halves(session, pkA, dlnA, cA, hwc);
    return;
  }
  both([&] { bob_mid_halves(session, pkA, dlnA, cA, h); }, [&] { bob_mid_halves(session, pkA, dlnA, cA, hwc); });
}

void AliceEndBatch(const std::vector<Bytes>& session, const paillier::PrivateKey& skA,
                   const std::vector<ProofBob>& pf, const DLNParams& dlnA, const std::vector<Nat>& cA,
                   const std::vector<Nat>& cB, const std::vector<secp::Affine>* B, std::vector<Nat>* alpha,
                   std::vector<uint8_t>* err) {
  const size_t n = cA.size();
  if (session.size() != n || pf.size() != n || cB.size() != n || (B && B->size() != n))
    throw std::invalid_argument("AliceEnd: sizes");
  alpha->assign(n, Nat());
  err->assign(n, OK);
  std::vector<const Bytes*> sp(n);
  std::vector<const Nat*> c1(n), c2(n);
  std::vector<const ProofBob*> pp(n);
  std::vector<const secp::Affine*> Xp(n, nullptr);
  std::vector<Nat*> a(n);
  std::vector<uint8_t*> e(n);
  for (size_t i = 0; i < n; ++i) {
    sp[i] = &session[i];
    c1[i] = &cA[i];
    c2[i] = &cB[i];
    pp[i] = &pf[i];
    if (B) Xp[i] = &(*B)[i];
    a[i] = &(*alpha)[i];
    e[i] = &(*err)[i];
  }
  // ProofBob[WC].Verify, then Decrypt(cB) mod q: one launch step (verify_bob_core)
  verify_bob_core(sp, skA.pub, dlnA, c1, c2, pp, Xp, &skA, &a, &e);
}

void AliceEndPairBatch(const std::vector<Bytes>& session, const paillier::PrivateKey& skA,
                       const std::vector<ProofBob>& pf, const std::vector<ProofBob>& pfwc, const DLNParams& dlnA,
                       const std::vector<Nat>& cA, const std::vector<Nat>& cB, const std::vector<Nat>& cBwc,
                       const std::vector<secp::Affine>& Bwc, std::vector<Nat>* alpha, std::vector<Nat>* mu,
                       std::vector<uint8_t>* err, std::vector<uint8_t>* errwc) {
  const size_t n = cA.size();
  if (session.size() != n || pf.size() != n || pfwc.size() != n || cB.size() != n || cBwc.size() != n ||
      Bwc.size() != n)
    throw std::invalid_argument("AliceEndPair: sizes");
  alpha->assign(n, Nat());
  mu->assign(n, Nat());
  err->assign(n, OK);
  errwc->assign(n, OK);
  // each half verified and decrypted as its own batch, the two halves as
  // concurrent tasks (host phases of one overlap the other's launches)
  auto half = [&](const std::vector<ProofBob>& p, const std::vector<Nat>& c, const secp::Affine* X0,
                  std::vector<Nat>* res, std::vector<uint8_t>* er) {
    std::vector<const Bytes*> sp(n);
    std::vector<const Nat*> c1(n), c2(n);
    std::vector<const ProofBob*> pp(n);
    std::vector<const secp::Affine*> Xp(n, nullptr);
    std::vector<Nat*> a(n);
    std::vector<uint8_t*> e(n);
    for (size_t i = 0; i < n; ++i) {
      sp[i] = &session[i];
      c1[i] = &cA[i];
      c2[i] = &c[i];
      pp[i] = &p[i];
      if (X0) Xp[i] = X0 + i;
      a[i] = &(*res)[i];
      e[i] = &(*er)[i];
    }
    verify_bob_core(sp, skA.pub, dlnA, c1, c2, pp, Xp, &skA, &a, &e);
  };
  both([&] { half(pf, cB, nullptr, alpha, err); }, [&] { half(pfwc, cBwc, Bwc.data(), mu, errwc); });
}

}  // namespace mpcx::host::mta
