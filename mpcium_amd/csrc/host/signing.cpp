// signing.cpp -- see signing.hpp.
#include "signing.hpp"

#include "engine.hpp"
#include "hostprof.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace mpcx::host::signing {
namespace {
double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// runs every task on its own thread; rethrows the first failure
void run_tasks(const std::vector<std::function<void()>>& tasks) {
  std::vector<std::exception_ptr> errs(tasks.size());
  std::vector<std::thread> th;
  for (size_t t = 0; t < tasks.size(); ++t)
    th.emplace_back([&, t] {
      MPCX_PROF_CPU("cpu.sign_tasks");
      try {
        tasks[t]();
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
  for (auto& x : th) x.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}
uint64_t mix(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t x = seed ^ (a * 0x9E3779B97F4A7C15ull) ^ (b * 0xC2B2AE3D27D4EB4Full) ^ (c * 0x165667B19E3779F9ull);
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  return x;
}
mta::DLNParams public_dln(const mta::DLNParams& d) {
  mta::DLNParams p;
  p.NTilde = d.NTilde;
  p.h1 = d.h1;
  p.h2 = d.h2;
  return p;
}

Nat X_(const secp::Affine& p) { return secp::FeToNat(p.x); }
Nat Y_(const secp::Affine& p) { return secp::FeToNat(p.y); }

// ---------------------------------------------------------------- GG18 pieces
// commitments.NewHashCommitment(rand, secrets...): r = MustGetRandomInt(256),
// C = SHA512_256i(r, secrets...), D = [r, secrets...]
void hash_commit(const RandFn& rd, std::vector<Nat> secrets, Nat* C, std::vector<Nat>* D) {
  D->clear();
  D->push_back(MustGetRandomInt(rd, 256));
  for (auto& s : secrets) D->push_back(std::move(s));
  std::vector<const Nat*> in;
  for (const auto& x : *D) in.push_back(&x);
  *C = SHA512_256i(in);
}
// HashCommitDecommit{C, D}.DeCommit() with `len` secrets: true iff D opens C
bool hash_decommit(const Nat& C, const std::vector<Nat>& D, size_t len) {
  if (D.size() != len + 1) return false;
  std::vector<const Nat*> in;
  for (const auto& x : D) in.push_back(&x);
  return SHA512_256i(in) == C;
}
// crypto.NewECPoint(ec, x, y): the point if (x, y) is on the curve
bool point_from(const Nat& x, const Nat& y, secp::Affine* P) {
  const Nat& p = secp::FieldP();
  if (!(x < p) || !(y < p)) return false;
  P->x = secp::NatToFe(x);
  P->y = secp::NatToFe(y);
  P->inf = false;
  return secp::IsOnCurve(*P);
}
// schnorr ZKProof / ZKVProof challenges:
//   c = RejectionSample(q, SHA512_256i_TAGGED(Session, X.x, X.y, G.x, G.y, alpha.x, alpha.y))
//   c = RejectionSample(q, SHA512_256i_TAGGED(Session, V.x, V.y, R.x, R.y, G.x, G.y, alpha.x, alpha.y))
Nat zk_challenge(const mta::Bytes& session, const secp::Affine& X, const secp::Affine& alpha) {
  const secp::Affine& G = secp::Generator();
  const Nat xx = X_(X), xy = Y_(X), gx = X_(G), gy = Y_(G), ax = X_(alpha), ay = Y_(alpha);
  return RejectionSample(mta::Q(), SHA512_256i_TAGGED(session, {&xx, &xy, &gx, &gy, &ax, &ay}));
}
Nat zkv_challenge(const mta::Bytes& session, const secp::Affine& V, const secp::Affine& R,
                  const secp::Affine& alpha) {
  const secp::Affine& G = secp::Generator();
  const Nat vx = X_(V), vy = Y_(V), rx = X_(R), ry = Y_(R), gx = X_(G), gy = Y_(G), ax = X_(alpha), ay = Y_(alpha);
  return RejectionSample(mta::Q(), SHA512_256i_TAGGED(session, {&vx, &vy, &rx, &ry, &gx, &gy, &ax, &ay}));
}
Nat negq(const Nat& c) {
  const Nat r = c % mta::Q();
  return r.is_zero() ? r : mta::Q() - r;
}
Nat addq(const Nat& a, const Nat& b) { return (a + b) % mta::Q(); }

// One signer of one wallet through GG18 rounds 1, 4-9 (signing.hpp).
struct Signer {
  CounterDRBG rd{0};     // the signer's GG18 reader
  secp::Affine Gam;      // round 1: Gamma_i = gamma_i G
  Nat C1;                //          commitment to Gamma_i
  std::vector<Nat> D1;
  secp::Affine a4;       // round 4: ZKProof(gamma_i, Gamma_i) = (alpha, t)
  Nat t4;
  Nat delta, sigma;      // round 3
  secp::Affine Rsum, R;  // round 5: R = theta^-1 sum Gamma
  Nat s, l, rho;
  secp::Affine V, A;
  Nat C5;
  std::vector<Nat> D5;
  secp::Affine aA, aV;   // round 6: ZKProof(rho, A) = (aA, tA), ZKVProof(V, R, s, l) = (aV, tV, uV)
  Nat tA, tV, uV;
  secp::Affine U, T;     // round 7
  Nat C7;
  std::vector<Nat> D7;
  bool ok = true;
};

}  // namespace

MtaStats RunSigning(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed,
                    size_t trace_wallets, std::vector<uint32_t>* trace, int64_t tamper_wallet, int tamper_kind) {
  if (signers < 2 || (size_t)signers > nodes.size()) throw std::invalid_argument("signers must be in [2, nodes]");
  MPCX_TRACE("run", wallets);  // timeline window of this run
  const Nat& q = mta::Q();
  const size_t S = (size_t)signers, Wn = wallets;
  MtaStats st;
  st.wallets = Wn;
  // per wallet and signer: k_i, gamma_i, w_i < q; W_i = w_i G; one session id per wallet
  std::vector<std::vector<Nat>> k(S, std::vector<Nat>(Wn)), g(S, std::vector<Nat>(Wn)), w(S, std::vector<Nat>(Wn));
  std::vector<std::vector<secp::Affine>> Wp(S, std::vector<secp::Affine>(Wn));
  std::vector<mta::Bytes> sess(Wn);
  std::vector<Nat> msg(Wn);        // the message (tx hash as an integer < q) of each wallet's signature
  std::vector<Signer> sg(Wn * S);  // GG18 state of signer i of wallet wi at [wi * S + i]
  parallel_for(Wn, [&](size_t wi) {
    CounterDRBG d(mix(seed, wi, 0xFFFF, 0));
    const RandFn r = d.fn();
    sess[wi].resize(32);
    r(sess[wi].data(), 32);
    for (size_t i = 0; i < S; ++i) {
      k[i][wi] = GetRandomPositiveInt(r, q);
      g[i][wi] = GetRandomPositiveInt(r, q);
      w[i][wi] = GetRandomPositiveInt(r, q);
      sg[wi * S + i].rd = CounterDRBG(mix(seed, wi, 0x100 + i, 4));
    }
    msg[wi] = GetRandomPositiveInt(r, q);
  });
  // GG18 rounds 1 and 4 depend on no MtA output: W_i = w_i G, the wallet key
  // X = sum_i W_i, Gamma_i = gamma_i G with its round-1 commitment, and the
  // round-4 Schnorr proof of gamma_i run as a background task while round 1's
  // MtA batches run; round 2 (MtAwc needs W_j) waits for it.
  std::vector<secp::Affine> XW(Wn);
  std::exception_ptr ec_err;
  std::thread ec_task([&] {
    MPCX_PROF_CPU("cpu.sign_ec_task");
    try {
      MPCX_PROF("sign.rounds1_4_ec");
      std::vector<secp::Comb> c(2 * Wn * S);
      for (size_t wi = 0; wi < Wn; ++wi)
        for (size_t i = 0; i < S; ++i) {
          c[2 * (wi * S + i)].a = g[i][wi];
          c[2 * (wi * S + i) + 1].a = w[i][wi];
        }
      const std::vector<secp::Affine> p = secp::CombineBatch(c);
      std::vector<Nat> a4(Wn * S);
      std::vector<secp::Comb> ca(Wn * S);
      parallel_for(Wn, [&](size_t wi) {
        secp::Affine X;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = sg[wi * S + i];
          s.Gam = p[2 * (wi * S + i)];
          Wp[i][wi] = p[2 * (wi * S + i) + 1];
          X = secp::Add(X, Wp[i][wi]);
          const RandFn r = s.rd.fn();
          hash_commit(r, {X_(s.Gam), Y_(s.Gam)}, &s.C1, &s.D1);  // round 1
          a4[wi * S + i] = GetRandomPositiveInt(r, q);              // round 4: a < q, alpha = a G
          ca[wi * S + i].a = a4[wi * S + i];
        }
        XW[wi] = X;
      });
      const std::vector<secp::Affine> al = secp::CombineBatch(ca);
      parallel_for(Wn, [&](size_t wi) {
        for (size_t i = 0; i < S; ++i) {
          Signer& s = sg[wi * S + i];
          s.a4 = al[wi * S + i];
          s.t4 = addq(a4[wi * S + i], zk_challenge(sess[wi], s.Gam, s.a4) * g[i][wi]);  // t = a + c gamma
        }
        if ((int64_t)wi == tamper_wallet && tamper_kind == kTamperR4Schnorr) sg[wi * S].t4 = addq(sg[wi * S].t4, Nat(1));
      });
    } catch (...) {
      ec_err = std::current_exception();
    }
  });
  bool ec_joined = false;
  std::mutex ec_mu;
  auto join_ec = [&] {
    std::lock_guard<std::mutex> lk(ec_mu);
    if (!ec_joined) {
      ec_task.join();
      ec_joined = true;
    }
    if (ec_err) std::rethrow_exception(ec_err);
  };
  struct JoinGuard {  // an exception in round 1 must not leave the task joinable
    std::function<void()> f;
    ~JoinGuard() {
      try {
        f();
      } catch (...) {
      }
    }
  } join_guard{join_ec};
  struct Pair {
    size_t i, j;  // Alice i, Bob j
    std::vector<Nat> cA;
    std::vector<mta::RangeProofAlice> pfA;
    std::vector<mta::BobMidResult> bob, bobwc;
    std::vector<Nat> alpha, mu;
  };
  std::vector<Pair> pairs;
  for (size_t i = 0; i < S; ++i)
    for (size_t j = 0; j < S; ++j)
      if (i != j) pairs.push_back(Pair{i, j, {}, {}, {}, {}, {}, {}});
  st.pairs = pairs.size();
  st.sessions = pairs.size() * Wn;
  for (auto& p : pairs) {
    p.cA.resize(Wn);
    p.pfA.resize(Wn);
    p.bob.resize(Wn);
    p.bobwc.resize(Wn);
    p.alpha.resize(Wn);
    p.mu.resize(Wn);
  }
  std::atomic<uint64_t> errors{0};
  auto count_err = [&](const std::vector<uint8_t>& err) {
    uint64_t n = 0;
    for (auto e : err) n += e != 0;
    errors += n;
  };
  auto pidx = [&](size_t i, size_t j) { return i * (S - 1) + (j < i ? j : j - 1); };  // i-major, j != i
  const Nat half = q >> 1;
  std::vector<Nat> sig_r(Wn), sig_s(Wn);
  std::vector<uint32_t> recid(Wn, 0);
  std::vector<uint8_t> verified(Wn, 0);
  std::atomic<uint64_t> relation_failures{0};
  std::mutex tm;
  double r1 = 0, r2 = 0, r3 = 0, r4 = 0;  // per-round seconds summed over chunks

  // Wallets [lo, hi) through rounds 1-3 and then rounds 4-9 + finalize. The
  // ordered pairs are independent chains -- AliceInit, then BobMid || BobMidWC
  // (one paired batch), then AliceEnd || AliceEndWC -- with no barrier between
  // rounds, so one chain's host phases overlap another's GPU batches. Chunks
  // run as concurrent pipelines. Every session's reader is its own
  // CounterDRBG(mix(seed, wallet, pair, role)), so the split changes no value.
  auto run_chunk = [&](size_t lo, size_t hi) {
    const size_t n = hi - lo;
    const std::vector<mta::Bytes> cs(sess.begin() + (long)lo, sess.begin() + (long)hi);
    auto sl = [&](const std::vector<Nat>& v) { return std::vector<Nat>(v.begin() + (long)lo, v.begin() + (long)hi); };
    auto slp = [&](const std::vector<secp::Affine>& v) {
      return std::vector<secp::Affine>(v.begin() + (long)lo, v.begin() + (long)hi);
    };
    struct Local {
      std::vector<CounterDRBG> da, db, dbwc;
      std::vector<RandFn> ra, rb, rbwc;
      std::vector<Nat> cA;
      std::vector<mta::RangeProofAlice> pfA;
      std::vector<mta::BobMidResult> bob, bobwc;
      std::vector<Nat> alpha, mu;
    };
    std::vector<Local> L(pairs.size());
    for (size_t pi = 0; pi < pairs.size(); ++pi) {
      const Pair& p = pairs[pi];
      Local& l = L[pi];
      l.da.reserve(n);
      l.db.reserve(n);
      l.dbwc.reserve(n);
      for (size_t wi = lo; wi < hi; ++wi) {
        l.da.emplace_back(mix(seed, wi, p.i * 16 + p.j, 1));
        l.db.emplace_back(mix(seed, wi, p.i * 16 + p.j, 2));
        l.dbwc.emplace_back(mix(seed, wi, p.i * 16 + p.j, 3));
      }
      for (size_t x = 0; x < n; ++x) {
        l.ra.push_back(l.da[x].fn());
        l.rb.push_back(l.db[x].fn());
        l.rbwc.push_back(l.dbwc[x].fn());
      }
    }
    const double c0 = now(), b0 = Engine::get().busy_seconds_now();
    const size_t np = pairs.size();
    std::vector<double> st1(np), st2(np), st3(np);
    std::vector<std::function<void()>> tasks;
    for (size_t pi = 0; pi < np; ++pi)
      tasks.push_back([&, pi] {
        const Pair& p = pairs[pi];
        Local& l = L[pi];
        prof::set_chain((int)(lo * 64 + pi));  // timeline tag: chunk start x 64 + ordered pair
        const double a0 = now();
        {  // round 1: AliceInit(k_i) to Bob j
          MPCX_TRACE("round1", n);
          std::vector<uint8_t> err;
          mta::AliceInitBatch(nodes[p.i].sk.pub, sl(k[p.i]), public_dln(nodes[p.j].dln), l.ra, &l.cA, &l.pfA, &err,
                              &nodes[p.i].sk);
          count_err(err);
        }
        const double a1 = now();
        {  // round 2: BobMid(gamma_j) + BobMidWC(w_j, W_j)
          MPCX_TRACE("round2", n);
          std::vector<uint8_t> err, errwc;
          join_ec();
          const std::vector<secp::Affine> Wj = slp(Wp[p.j]);
          mta::BobMidPairBatch(cs, nodes[p.i].sk.pub, l.pfA, sl(g[p.j]), sl(w[p.j]), l.cA, public_dln(nodes[p.i].dln),
                               nodes[p.j].dln, Wj, l.rb, l.rbwc, &l.bob, &l.bobwc, &err, &errwc);
          count_err(err);
          count_err(errwc);
        }
        const double a2 = now();
        {  // round 3: AliceEnd + AliceEndWC
          MPCX_TRACE("round3", n);
          std::vector<mta::ProofBob> pf(n), pfwc(n);
          std::vector<Nat> cB(n), cBwc(n);
          for (size_t x = 0; x < n; ++x) {
            pf[x] = l.bob[x].pf;
            cB[x] = l.bob[x].cB;
            pfwc[x] = l.bobwc[x].pf;
            cBwc[x] = l.bobwc[x].cB;
          }
          std::vector<uint8_t> err, errwc;
          const std::vector<secp::Affine> Wj = slp(Wp[p.j]);
          mta::AliceEndPairBatch(cs, nodes[p.i].sk, pf, pfwc, nodes[p.i].dln, l.cA, cB, cBwc, Wj, &l.alpha, &l.mu, &err,
                                 &errwc);
          count_err(err);
          count_err(errwc);
        }
        st1[pi] = a1 - a0;
        st2[pi] = a2 - a1;
        st3[pi] = now() - a2;
      });
    run_tasks(tasks);
    const double c3 = now(), b3 = Engine::get().busy_seconds_now();
    for (size_t pi = 0; pi < pairs.size(); ++pi) {
      Pair& p = pairs[pi];
      Local& l = L[pi];
      for (size_t x = 0; x < n; ++x) {
        p.cA[lo + x] = std::move(l.cA[x]);
        p.pfA[lo + x] = std::move(l.pfA[x]);
        p.bob[lo + x] = std::move(l.bob[x]);
        p.bobwc[lo + x] = std::move(l.bobwc[x]);
        p.alpha[lo + x] = std::move(l.alpha[x]);
        p.mu[lo + x] = std::move(l.mu[x]);
      }
    }
    join_ec();
    {
      MPCX_PROF("sign.rounds4_9");
      prof::set_chain((int)(lo * 64 + 63));
      MPCX_TRACE("rounds4_9", n);
      auto at = [&](size_t x, size_t i) -> Signer& { return sg[(lo + x) * S + i]; };
      // round 3's outputs: delta_i = k_i gamma_i + sum_j (alpha_ij + beta_ji),
      // sigma_i = k_i w_i + sum_j (mu_ij + nu_ji); theta = sum delta_i
      std::vector<Nat> theta_inv(n);
      std::vector<uint8_t> live(n, 1);
      parallel_for(n, [&](size_t x) {
        const size_t wi = lo + x;
        uint64_t bad = 0;
        for (const auto& p : pairs) {
          bad += (p.alpha[wi] + p.bob[wi].beta) % q != (k[p.i][wi] * g[p.j][wi]) % q;
          bad += (p.mu[wi] + p.bobwc[wi].beta) % q != (k[p.i][wi] * w[p.j][wi]) % q;
        }
        if (bad) relation_failures += bad;
        Nat theta;
        for (size_t i = 0; i < S; ++i) {
          Nat di = k[i][wi] * g[i][wi], si = k[i][wi] * w[i][wi];
          for (size_t j = 0; j < S; ++j) {
            if (j == i) continue;
            const Pair& ij = pairs[pidx(i, j)];  // i as Alice
            const Pair& ji = pairs[pidx(j, i)];  // i as Bob
            di = di + ij.alpha[wi] + ji.bob[wi].beta;
            si = si + ij.mu[wi] + ji.bobwc[wi].beta;
          }
          at(x, i).delta = di % q;
          at(x, i).sigma = si % q;
          theta = (theta + at(x, i).delta) % q;
        }
        if (theta.is_zero() || !mod_inverse(Int(theta), q, &theta_inv[x])) live[x] = 0;
      });
      const size_t P = S - 1;  // peers
      // ---- round 5: every peer's Gamma_j decommitted and its Schnorr proof
      // verified (t G + (q - c) Gamma_j == alpha), R = theta^-1 sum Gamma
      std::vector<secp::Comb> c5(n * S * (P + 1));  // per (wallet, signer): P verifications, then R
      std::vector<secp::Affine> Gj(n * S * P);
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          s.Rsum = s.Gam;
          size_t pj = 0;
          for (size_t j = 0; j < S; ++j) {
            if (j == i) continue;
            const Signer& o = at(x, j);
            const size_t e = (x * S + i) * (P + 1) + pj;
            secp::Affine& G_ = Gj[(x * S + i) * P + pj];
            ++pj;
            if (!hash_decommit(o.C1, o.D1, 2) || !point_from(o.D1[1], o.D1[2], &G_) || !secp::IsOnCurve(o.a4)) {
              s.ok = false;
              continue;
            }
            c5[e].a = o.t4;
            c5[e].P = G_;
            c5[e].b = negq(zk_challenge(sess[lo + x], G_, o.a4));
            s.Rsum = secp::Add(s.Rsum, G_);
          }
          secp::Comb& cr = c5[(x * S + i) * (P + 1) + P];
          cr.P = s.Rsum;
          cr.b = theta_inv[x];
        }
      });
      const std::vector<secp::Affine> r5 = secp::CombineBatch(c5);
      std::vector<secp::Comb> c5b(n * S * 2);  // V_i = l_i G + s_i R, A_i = rho_i G
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          for (size_t pj = 0, j = 0; j < S; ++j) {
            if (j == i) continue;
            // tss-lib's ZKProof.Verify fails when alpha + cX is the point at
            // infinity; with tG - cX == alpha that is t = 0 mod q
            if (!secp::Equal(r5[(x * S + i) * (P + 1) + pj], at(x, j).a4) || (at(x, j).t4 % q).is_zero())
              s.ok = false;
            ++pj;
          }
          s.R = r5[(x * S + i) * (P + 1) + P];
          if (s.R.inf) {
            s.ok = false;
            continue;
          }
          s.s = (msg[lo + x] * k[i][lo + x] + X_(s.R) * s.sigma) % q;  // s_i = m k_i + r sigma_i
          const RandFn r = s.rd.fn();
          s.l = GetRandomPositiveInt(r, q);
          s.rho = GetRandomPositiveInt(r, q);
          secp::Comb& cv = c5b[2 * (x * S + i)];
          cv.a = s.l;
          cv.P = s.R;
          cv.b = s.s;
          c5b[2 * (x * S + i) + 1].a = s.rho;
        }
      });
      const std::vector<secp::Affine> va = secp::CombineBatch(c5b);
      // ---- round 5 commitments and round 6 proofs: ZKProof(rho, A): alpha = a G;
      // ZKVProof(V, R, s, l): alpha = a R + b G
      std::vector<secp::Comb> c6(n * S * 2);
      std::vector<Nat> aa(n * S), av(n * S), bv(n * S);
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          if (s.R.inf) continue;
          s.V = va[2 * (x * S + i)];
          s.A = va[2 * (x * S + i) + 1];
          const RandFn r = s.rd.fn();
          hash_commit(r, {X_(s.V), Y_(s.V), X_(s.A), Y_(s.A)}, &s.C5, &s.D5);
          const size_t e = x * S + i;
          aa[e] = GetRandomPositiveInt(r, q);
          av[e] = GetRandomPositiveInt(r, q);
          bv[e] = GetRandomPositiveInt(r, q);
          c6[2 * e].a = aa[e];
          c6[2 * e + 1].a = bv[e];
          c6[2 * e + 1].P = s.R;
          c6[2 * e + 1].b = av[e];
        }
      });
      const std::vector<secp::Affine> a6 = secp::CombineBatch(c6);
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          if (s.R.inf) continue;
          const size_t e = x * S + i;
          s.aA = a6[2 * e];
          s.aV = a6[2 * e + 1];
          const Nat cA = zk_challenge(sess[lo + x], s.A, s.aA), cV = zkv_challenge(sess[lo + x], s.V, s.R, s.aV);
          s.tA = addq(aa[e], cA * s.rho);
          s.tV = addq(av[e], cV * s.s);
          s.uV = addq(bv[e], cV * s.l);
        }
        if ((int64_t)(lo + x) == tamper_wallet && tamper_kind == kTamperR6Zkv) at(x, 0).tV = addq(at(x, 0).tV, Nat(1));
      });
      // ---- round 7: every peer's (V_j, A_j) decommitted, ZKProof(A_j) and
      // ZKVProof(V_j, R) verified; V = -m G - r X + sum V, A = sum A
      std::vector<secp::Comb> c7(n * S * (2 * P + 1));
      std::vector<secp::Affine> Vj(n * S * P), Aj(n * S * P);
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        const size_t wi = lo + x;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          if (s.R.inf) continue;
          const size_t base = (x * S + i) * (2 * P + 1);
          for (size_t pj = 0, j = 0; j < S; ++j) {
            if (j == i) continue;
            const Signer& o = at(x, j);
            const size_t e = (x * S + i) * P + pj;
            secp::Comb& ca = c7[base + 2 * pj];
            secp::Comb& cv = c7[base + 2 * pj + 1];
            ++pj;
            if (!hash_decommit(o.C5, o.D5, 4) || !point_from(o.D5[1], o.D5[2], &Vj[e]) ||
                !point_from(o.D5[3], o.D5[4], &Aj[e]) || !secp::IsOnCurve(o.aA) || !secp::IsOnCurve(o.aV)) {
              s.ok = false;
              continue;
            }
            ca.a = o.tA;  // tA G - cA A_j == alphaA
            ca.P = Aj[e];
            ca.b = negq(zk_challenge(sess[wi], Aj[e], o.aA));
            cv.a = o.uV;  // uV G + tV R - cV V_j == alphaV
            cv.P = s.R;
            cv.b = o.tV;
            cv.Q = Vj[e];
            cv.c = negq(zkv_challenge(sess[wi], Vj[e], s.R, o.aV));
          }
          secp::Comb& cm = c7[base + 2 * P];  // -m G - r X
          cm.a = negq(msg[wi]);
          cm.P = XW[wi];
          cm.b = negq(X_(s.R));
        }
      });
      const std::vector<secp::Affine> r7 = secp::CombineBatch(c7);
      std::vector<secp::Comb> c7b(n * S * 2);  // U_i = rho_i V, T_i = l_i A
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          if (s.R.inf) continue;
          const size_t base = (x * S + i) * (2 * P + 1);
          secp::Affine V = secp::Add(r7[base + 2 * P], s.V), A = s.A;
          for (size_t pj = 0, j = 0; j < S; ++j) {
            if (j == i) continue;
            const Signer& o = at(x, j);
            const size_t e = (x * S + i) * P + pj;
            // ZKProof: alpha + cA = infinity iff tA = 0 mod q (as in round 5).
            // ZKVProof: tss-lib fails when tR + uG is infinity; without the
            // discrete log of R (nobody knows k) that takes tV = uV = 0 mod q
            // (alpha = -cV otherwise needs a fixed point of the challenge hash)
            if (!secp::Equal(r7[base + 2 * pj], o.aA) || !secp::Equal(r7[base + 2 * pj + 1], o.aV) ||
                (o.tA % q).is_zero() || ((o.tV % q).is_zero() && (o.uV % q).is_zero()))
              s.ok = false;
            V = secp::Add(V, Vj[e]);
            A = secp::Add(A, Aj[e]);
            ++pj;
          }
          c7b[2 * (x * S + i)].P = V;
          c7b[2 * (x * S + i)].b = s.rho;
          c7b[2 * (x * S + i) + 1].P = A;
          c7b[2 * (x * S + i) + 1].b = s.l;
        }
      });
      const std::vector<secp::Affine> ut = secp::CombineBatch(c7b);
      // ---- round 7 commitments, round 9: every peer's (U_j, T_j) decommitted,
      // sum U == sum T; finalize: s = sum s_i, low-s, recovery id, and
      // ecdsa.Verify by every signer twice (tss-lib's finalize, then the node's
      // mpcium session: /root/reference/pkg/mpc/ecdsa_signing_session.go:162)
      std::vector<secp::Comb> cf(n * S * 2);
      std::vector<Nat> fin_s(n);
      std::vector<uint32_t> fin_rid(n);
      std::vector<uint8_t> fin_ok(n, 0);
      parallel_for(n, [&](size_t x) {
        if (!live[x]) return;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          if (s.R.inf) continue;
          s.U = ut[2 * (x * S + i)];
          s.T = ut[2 * (x * S + i) + 1];
          hash_commit(s.rd.fn(), {X_(s.U), Y_(s.U), X_(s.T), Y_(s.T)}, &s.C7, &s.D7);
        }
        if ((int64_t)(lo + x) == tamper_wallet && tamper_kind == kTamperR7Decommit && at(x, 0).D7.size() > 1) {
          Nat& u = at(x, 0).D7[1];  // U.x with its low bit flipped
          u = u.bit(0) ? u - Nat(1) : u + Nat(1);
        }
        bool all = true;
        for (size_t i = 0; i < S; ++i) {
          Signer& s = at(x, i);
          if (s.R.inf) {
            all = false;
            continue;
          }
          secp::Affine U = s.U, T = s.T;
          for (size_t j = 0; j < S; ++j) {
            if (j == i) continue;
            const Signer& o = at(x, j);
            secp::Affine Uj, Tj;
            if (!hash_decommit(o.C7, o.D7, 4) || !point_from(o.D7[1], o.D7[2], &Uj) ||
                !point_from(o.D7[3], o.D7[4], &Tj)) {
              s.ok = false;
              continue;
            }
            U = secp::Add(U, Uj);
            T = secp::Add(T, Tj);
          }
          if (!secp::Equal(U, T)) s.ok = false;
          all = all && s.ok;
        }
        if (!all) return;
        // finalize (signer 0's view; every signer holds the same R, r, s when all checks passed)
        const Signer& s0 = at(x, 0);
        Nat sum;
        for (size_t i = 0; i < S; ++i) sum = (sum + at(x, i).s) % q;
        const Nat rx = X_(s0.R), r = rx % q;
        if (r.is_zero() || sum.is_zero()) return;
        uint32_t rid = (rx >= q ? 2u : 0u) | (Y_(s0.R).bit(0) ? 1u : 0u);
        if (sum > half) {  // low-s form, recovery id flipped with it
          sum = q - sum;
          rid ^= 1u;
        }
        Nat sinv;
        if (!mod_inverse(Int(sum), q, &sinv)) return;
        const Nat u1 = (msg[lo + x] * sinv) % q, u2 = (r * sinv) % q;
        for (size_t v = 0; v < 2 * S; ++v) {  // ecdsa.Verify(X, m, r, s): u1 G + u2 X has x == r (mod q)
          secp::Comb& c = cf[x * 2 * S + v];
          c.a = u1;
          c.P = XW[lo + x];
          c.b = u2;
        }
        fin_s[x] = sum;
        fin_rid[x] = rid;
        fin_ok[x] = 1;
      });
      const std::vector<secp::Affine> vf = secp::CombineBatch(cf);
      parallel_for(n, [&](size_t x) {
        if (!fin_ok[x]) return;
        const size_t wi = lo + x;
        const Nat r = X_(at(x, 0).R) % q;
        bool good = true;
        for (size_t v = 0; v < 2 * S; ++v) {
          const secp::Affine& P_ = vf[x * 2 * S + v];
          good = good && !P_.inf && X_(P_) % q == r;
        }
        sig_r[wi] = r;
        sig_s[wi] = fin_s[x];
        recid[wi] = fin_rid[x];
        verified[wi] = good;
      });
    }
    const double c4 = now();
    if (prof::enabled()) {  // seconds with no libmpcx call in flight (one chunk: exact)
      static const int s13 = prof::slot_of("sign.gpu_idle.rounds1_3"), s4 = prof::slot_of("sign.gpu_idle.rounds4_9");
      prof::add(s13, (uint64_t)(std::max(0.0, (c3 - c0) - (b3 - b0)) * 1e9));
      prof::add(s4, (uint64_t)((c4 - c3) * 1e9));
    }
    auto mean = [&](const std::vector<double>& v) {
      double t = 0;
      for (double x : v) t += x;
      return v.empty() ? 0.0 : t / (double)v.size();
    };
    std::lock_guard<std::mutex> lk(tm);
    r1 += mean(st1);  // per pair chain, averaged over the pairs
    r2 += mean(st2);
    r3 += mean(st3);
    r4 += c4 - c3;
  };

  // Chunking: concurrent wallet pipelines whose host phases fall into each
  // other's GPU launches. 2 signers (2 ordered pairs): three pipelines --
  // three vs two mean 6,036 vs 5,770 sigs/s over four alternating pairs, then
  // 6,187 vs 5,766 (profiles/r02/pipe_ab/); round 3 re-measured 6,441 vs
  // 6,367, within the spread (profiles/r03/pipe_ab/). 3+ signers (6+ pairs):
  // two pipelines since round 3's coalesced launches and lighter host work --
  // 2,859 vs 2,673 sigs/s over seven runs each, t = 3.6 (profiles/r03/pipes3/,
  // profiles/r03/pipe_ab/, profiles/r03/lanes_ab/); round 2 measured them 15%
  // slower. MPCX_SIGN_PIPELINE = "chunks,workers" overrides (A/B runs).
  size_t n_chunks = pairs.size() <= 2 ? 3 : 2, n_workers = n_chunks;
  if (const char* e = std::getenv("MPCX_SIGN_PIPELINE")) {
    unsigned a = 0, b = 0;
    if (std::sscanf(e, "%u,%u", &a, &b) == 2 && a > 0 && b > 0) {
      n_chunks = a;
      n_workers = b;
    }
  }
  n_chunks = std::max<size_t>(1, std::min(n_chunks, Wn));
  n_workers = std::min(n_workers, n_chunks);
  Engine::get().reset_busy();
  const double t0 = now();
  {
    std::atomic<size_t> next{0};
    std::vector<std::function<void()>> workers;
    // MPCX_SIGN_STAGGER_MS: worker t starts t x this many ms late (A/B runs:
    // desynchronizes the pipelines' host and GPU phases)
    static const int stagger_ms = [] {
      const char* e = std::getenv("MPCX_SIGN_STAGGER_MS");
      return e ? std::max(0, std::atoi(e)) : 0;
    }();
    for (size_t t = 0; t < n_workers; ++t)
      workers.push_back([&, t] {
        if (stagger_ms && t) std::this_thread::sleep_for(std::chrono::milliseconds(stagger_ms * (int)t));
        for (;;) {
          const size_t c = next.fetch_add(1);
          if (c >= n_chunks) return;
          run_chunk(Wn * c / n_chunks, Wn * (c + 1) / n_chunks);
        }
      });
    if (Wn) run_tasks(workers);
  }
  join_ec();
  st.relation_failures = relation_failures.load();
  const double t5 = now();
  for (size_t wi = 0; wi < Wn; ++wi) {
    st.signatures += !sig_r[wi].is_zero();
    st.verified += verified[wi];
  }
  st.aborted = Wn - st.signatures;
  if (trace && trace_wallets) {
    const size_t tw = std::min(trace_wallets, Wn);
    trace->assign(pairs.size() * tw * kTracePairWords + tw * kTraceSigWords, 0);
    uint32_t* o = trace->data();
    for (const auto& p : pairs)
      for (size_t t = 0; t < tw; ++t, o += kTracePairWords) {
        const size_t wi = TraceWallet(t, tw, Wn);
        p.alpha[wi].to_words(o, 8);
        p.bob[wi].beta.to_words(o + 8, 8);
        p.mu[wi].to_words(o + 16, 8);
        p.bobwc[wi].beta.to_words(o + 24, 8);
        const auto& a = p.pfA[wi];
        const auto& b = p.bob[wi];
        const auto& c = p.bobwc[wi];
        const Nat ux = secp::FeToNat(c.pf.U.x), uy = secp::FeToNat(c.pf.U.y);
        std::vector<const Nat*> in{&p.cA[wi], &a.Z, &a.U, &a.W, &a.S, &a.S1, &a.S2, &b.cB};
        for (const auto* f : {&b.pf, &c.pf}) {
          for (const Nat* x : {&f->Z, &f->ZPrm, &f->T, &f->V, &f->W, &f->S, &f->S1, &f->S2, &f->T1, &f->T2})
            in.push_back(x);
          if (f == &b.pf) in.push_back(&c.cB);
        }
        in.push_back(&ux);
        in.push_back(&uy);
        SHA512_256i(in).to_words(o + 32, 8);
      }
    for (size_t t = 0; t < tw; ++t, o += kTraceSigWords) {
      const size_t wi = TraceWallet(t, tw, Wn);
      sig_r[wi].to_words(o, 8);
      sig_s[wi].to_words(o + 8, 8);
      o[16] = recid[wi];
      if (sig_r[wi].is_zero()) continue;  // aborted: no transcript digest
      std::vector<Nat> ints;
      for (size_t i = 0; i < S; ++i) {
        const Signer& s = sg[wi * S + i];
        for (const Nat& v : {s.C1, X_(s.Gam), Y_(s.Gam), X_(s.a4), Y_(s.a4), s.t4, s.C5, X_(s.V), Y_(s.V), X_(s.A),
                             Y_(s.A), X_(s.aA), Y_(s.aA), s.tA, X_(s.aV), Y_(s.aV), s.tV, s.uV, s.C7, X_(s.U), Y_(s.U),
                             X_(s.T), Y_(s.T), s.s})
          ints.push_back(v);
      }
      std::vector<const Nat*> in;
      for (const auto& v : ints) in.push_back(&v);
      SHA512_256i(in).to_words(o + 17, 8);
    }
  }
  st.round1_s = r1;
  st.round2_s = r2;
  st.round3_s = r3;
  st.finalize_s = r4;
  st.total_s = t5 - t0;
  st.errors = errors.load();
  st.engine_busy_s = Engine::get().busy_seconds();
  st.alg_macs = Engine::get().alg_macs();
  return st;
}

}  // namespace mpcx::host::signing
