// signing.cpp -- see signing.hpp.
#include "signing.hpp"

#include "engine.hpp"
#include "hostprof.hpp"

#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <stdexcept>

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
}  // namespace

MtaStats RunSigning(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed,
                    size_t trace_wallets, std::vector<uint32_t>* trace) {
  if (signers < 2 || (size_t)signers > nodes.size()) throw std::invalid_argument("signers must be in [2, nodes]");
  const Nat& q = mta::Q();
  const size_t S = (size_t)signers, Wn = wallets;
  MtaStats st;
  st.wallets = Wn;
  // per wallet and signer: k_i, gamma_i, w_i < q; W_i = w_i G; one session id per wallet
  std::vector<std::vector<Nat>> k(S, std::vector<Nat>(Wn)), g(S, std::vector<Nat>(Wn)), w(S, std::vector<Nat>(Wn));
  std::vector<std::vector<secp::Affine>> Wp(S, std::vector<secp::Affine>(Wn));
  std::vector<mta::Bytes> sess(Wn);
  std::vector<Nat> msg(Wn);  // the message (tx hash as an integer < q) of each wallet's signature
  parallel_for(Wn, [&](size_t wi) {
    CounterDRBG d(mix(seed, wi, 0xFFFF, 0));
    const RandFn r = d.fn();
    sess[wi].resize(32);
    r(sess[wi].data(), 32);
    for (size_t i = 0; i < S; ++i) {
      k[i][wi] = GetRandomPositiveInt(r, q);
      g[i][wi] = GetRandomPositiveInt(r, q);
      w[i][wi] = GetRandomPositiveInt(r, q);
      Wp[i][wi] = secp::ScalarBaseMult(w[i][wi]);
    }
    msg[wi] = GetRandomPositiveInt(r, q);
  });
  struct Pair {
    size_t i, j;  // Alice i, Bob j
    std::vector<CounterDRBG> drbg_a, drbg_b, drbg_bwc;
    std::vector<RandFn> ra, rb, rbwc;
    std::vector<Nat> cA;
    std::vector<mta::RangeProofAlice> pfA;
    std::vector<mta::BobMidResult> bob, bobwc;
    std::vector<Nat> alpha, mu;
  };
  std::vector<Pair> pairs;
  for (size_t i = 0; i < S; ++i)
    for (size_t j = 0; j < S; ++j)
      if (i != j) pairs.push_back(Pair{i, j, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}});
  st.pairs = pairs.size();
  st.sessions = pairs.size() * Wn;
  for (auto& p : pairs) {
    p.drbg_a.reserve(Wn);
    p.drbg_b.reserve(Wn);
    p.drbg_bwc.reserve(Wn);
    for (size_t wi = 0; wi < Wn; ++wi) {
      p.drbg_a.emplace_back(mix(seed, wi, p.i * 16 + p.j, 1));
      p.drbg_b.emplace_back(mix(seed, wi, p.i * 16 + p.j, 2));
      p.drbg_bwc.emplace_back(mix(seed, wi, p.i * 16 + p.j, 3));
    }
    for (size_t wi = 0; wi < Wn; ++wi) {
      p.ra.push_back(p.drbg_a[wi].fn());
      p.rb.push_back(p.drbg_b[wi].fn());
      p.rbwc.push_back(p.drbg_bwc[wi].fn());
    }
  }
  // Within a round the ordered pairs (and a pair's MtA / MtAwc halves) are
  // independent: they run as concurrent tasks, so one task's host work
  // (hashing, random draws, gcds, conversions) overlaps another's GPU batch.
  std::atomic<uint64_t> errors{0};
  auto count_err = [&](const std::vector<uint8_t>& err) {
    uint64_t n = 0;
    for (auto e : err) n += e != 0;
    errors += n;
  };
  Engine::get().reset_busy();
  const double t0 = now();
  // round 1: AliceInit(pk_i, k_i, N~_j, h1_j, h2_j)
  {
    std::vector<std::function<void()>> tasks;
    for (auto& p : pairs)
      tasks.push_back([&, pp = &p] {
        std::vector<uint8_t> err;
        mta::AliceInitBatch(nodes[pp->i].sk.pub, k[pp->i], public_dln(nodes[pp->j].dln), pp->ra, &pp->cA, &pp->pfA,
                            &err);
        count_err(err);
      });
    run_tasks(tasks);
  }
  const double t1 = now();
  // round 2: Bob j -- BobMid(gamma_j), BobMidWC(w_j, W_j)
  {
    std::vector<std::function<void()>> tasks;
    for (auto& p : pairs) {
      tasks.push_back([&, pp = &p] {
        std::vector<uint8_t> err;
        mta::BobMidBatch(sess, nodes[pp->i].sk.pub, pp->pfA, g[pp->j], pp->cA, public_dln(nodes[pp->i].dln),
                         nodes[pp->j].dln, nullptr, pp->rb, &pp->bob, &err);
        count_err(err);
      });
      tasks.push_back([&, pp = &p] {
        std::vector<uint8_t> err;
        mta::BobMidBatch(sess, nodes[pp->i].sk.pub, pp->pfA, w[pp->j], pp->cA, public_dln(nodes[pp->i].dln),
                         nodes[pp->j].dln, &Wp[pp->j], pp->rbwc, &pp->bobwc, &err);
        count_err(err);
      });
    }
    run_tasks(tasks);
  }
  const double t2 = now();
  // round 3: Alice i -- AliceEnd, AliceEndWC
  {
    std::vector<std::function<void()>> tasks;
    for (auto& p : pairs) {
      tasks.push_back([&, pp = &p] {
        std::vector<mta::ProofBob> pf(Wn);
        std::vector<Nat> cB(Wn);
        for (size_t wi = 0; wi < Wn; ++wi) {
          pf[wi] = pp->bob[wi].pf;
          cB[wi] = pp->bob[wi].cB;
        }
        std::vector<uint8_t> err;
        mta::AliceEndBatch(sess, nodes[pp->i].sk, pf, nodes[pp->i].dln, pp->cA, cB, nullptr, &pp->alpha, &err);
        count_err(err);
      });
      tasks.push_back([&, pp = &p] {
        std::vector<mta::ProofBob> pf(Wn);
        std::vector<Nat> cB(Wn);
        for (size_t wi = 0; wi < Wn; ++wi) {
          pf[wi] = pp->bobwc[wi].pf;
          cB[wi] = pp->bobwc[wi].cB;
        }
        std::vector<uint8_t> err;
        mta::AliceEndBatch(sess, nodes[pp->i].sk, pf, nodes[pp->i].dln, pp->cA, cB, &Wp[pp->j], &pp->mu, &err);
        count_err(err);
      });
    }
    run_tasks(tasks);
  }
  const double t3 = now();
  for (const auto& p : pairs)
    for (size_t wi = 0; wi < Wn; ++wi) {
      const bool ok1 = (p.alpha[wi] + p.bob[wi].beta) % q == (k[p.i][wi] * g[p.j][wi]) % q;
      const bool ok2 = (p.mu[wi] + p.bobwc[wi].beta) % q == (k[p.i][wi] * w[p.j][wi]) % q;
      st.relation_failures += !ok1 + !ok2;
    }
  // rounds 4-9 + finalize and ecdsa.Verify (see signing.hpp), per wallet
  auto pidx = [&](size_t i, size_t j) { return i * (S - 1) + (j < i ? j : j - 1); };  // i-major, j != i
  const Nat half = q >> 1;
  std::vector<Nat> sig_r(Wn), sig_s(Wn);
  std::vector<uint32_t> recid(Wn, 0);
  std::vector<uint8_t> verified(Wn, 0);
  const double t4 = now();
  parallel_for(Wn, [&](size_t wi) {
    MPCX_PROF("sign.finalize_verify");
    Nat delta, s_sum, sigma_sum;
    secp::Affine Gam, X;
    for (size_t i = 0; i < S; ++i) {
      Nat di = k[i][wi] * g[i][wi], si = k[i][wi] * w[i][wi];
      for (size_t j = 0; j < S; ++j) {
        if (j == i) continue;
        const Pair& ij = pairs[pidx(i, j)];  // i as Alice
        const Pair& ji = pairs[pidx(j, i)];  // i as Bob
        di = di + ij.alpha[wi] + ji.bob[wi].beta;
        si = si + ij.mu[wi] + ji.bobwc[wi].beta;
      }
      delta = (delta + di) % q;
      sigma_sum = (sigma_sum + si) % q;
      Gam = secp::Add(Gam, secp::ScalarBaseMult(g[i][wi]));  // Gamma_i = gamma_i G (decommitted in round 4)
      X = secp::Add(X, Wp[i][wi]);
      // s_i = m k_i + r sigma_i (round 5 on); r is known once R is: accumulate m k_i and sigma_i
      s_sum = (s_sum + msg[wi] * k[i][wi]) % q;
    }
    Nat dinv;
    if (delta.is_zero() || !mod_inverse(Int(delta), q, &dinv)) return;
    const secp::Affine R = secp::ScalarMult(Gam, dinv);  // R = delta^-1 Gamma = k^-1 G
    if (R.inf) return;
    const Nat rx = secp::FeToNat(R.x), ry = secp::FeToNat(R.y);
    const Nat r = rx % q;
    if (r.is_zero()) return;
    Nat sv = (s_sum + r * sigma_sum) % q;
    if (sv.is_zero()) return;
    uint32_t rid = (rx >= q ? 2u : 0u) | (ry.bit(0) ? 1u : 0u);
    if (sv > half) {  // low-s form, recovery id flipped with it
      sv = q - sv;
      rid ^= 1u;
    }
    sig_r[wi] = r;
    sig_s[wi] = sv;
    recid[wi] = rid;
    // ecdsa.Verify(X, m, r, s): (m s^-1) G + (r s^-1) X has x == r (mod q)
    Nat sinv;
    if (!mod_inverse(Int(sv), q, &sinv)) return;
    const secp::Affine P = secp::Add(secp::ScalarBaseMult((msg[wi] * sinv) % q), secp::ScalarMult(X, (r * sinv) % q));
    verified[wi] = !P.inf && secp::FeToNat(P.x) % q == r;
  });
  const double t5 = now();
  for (size_t wi = 0; wi < Wn; ++wi) {
    st.signatures += !sig_r[wi].is_zero();
    st.verified += verified[wi];
  }
  if (trace && trace_wallets) {
    const size_t tw = std::min(trace_wallets, Wn);
    trace->assign(pairs.size() * tw * kTracePairWords + tw * kTraceSigWords, 0);
    uint32_t* o = trace->data();
    for (const auto& p : pairs)
      for (size_t wi = 0; wi < tw; ++wi, o += kTracePairWords) {
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
    for (size_t wi = 0; wi < tw; ++wi, o += kTraceSigWords) {
      sig_r[wi].to_words(o, 8);
      sig_s[wi].to_words(o + 8, 8);
      o[16] = recid[wi];
    }
  }
  st.round1_s = t1 - t0;
  st.round2_s = t2 - t1;
  st.round3_s = t3 - t2;
  st.finalize_s = t5 - t4;
  st.total_s = t5 - t0;
  st.errors = errors.load();
  st.engine_busy_s = Engine::get().busy_seconds();
  st.alg_macs = Engine::get().alg_macs();
  return st;
}

}  // namespace mpcx::host::signing
