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
    }
    msg[wi] = GetRandomPositiveInt(r, q);
  });
  // The wallet points that do not depend on the MtA outputs -- W_i = w_i G,
  // Gamma = sum_i gamma_i G (round 4's decommitted Gamma_i), X = sum_i W_i --
  // are computed by a background task while round 1 runs; round 2 (MtAwc
  // needs W_j) waits for it.
  std::vector<secp::Affine> GamW(Wn), XW(Wn);
  std::exception_ptr ec_err;
  std::thread ec_task([&] {
    try {
      parallel_for(Wn, [&](size_t wi) {
        secp::Affine Gam, X;
        for (size_t i = 0; i < S; ++i) {
          Wp[i][wi] = secp::ScalarBaseMult(w[i][wi]);
          Gam = secp::Add(Gam, secp::ScalarBaseMult(g[i][wi]));
          X = secp::Add(X, Wp[i][wi]);
        }
        GamW[wi] = Gam;
        XW[wi] = X;
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

  // Wallets [lo, hi) through rounds 1-3 and the finalize. The ordered pairs
  // (and a pair's MtA / MtAwc halves) are independent tasks; chunks can run as
  // concurrent pipelines, so one chunk's host work (draws, hashing, gcds,
  // finalize + ecdsa.Verify) overlaps another chunk's GPU batches. Every session's reader is its own CounterDRBG(mix(seed, wallet,
  // pair, role)), so the split changes no value.
  // MPCX_SIGN_CHAINS=0: rounds with a barrier between them (A/B)
  const char* ce = std::getenv("MPCX_SIGN_CHAINS");
  const bool chains = !(ce && ce[0] == '0');
  // MPCX_SIGN_STAGGER_MS: chain k starts k times this late (A/B runs)
  const char* se = std::getenv("MPCX_SIGN_STAGGER_MS");
  const double stagger_ms = se ? std::atof(se) : 0.0;
  // MPCX_SIGN_PAIRED=0: BobMid / BobMidWC (AliceEnd / AliceEndWC) as two
  // concurrent batches instead of one paired batch (A/B)
  const char* pe = std::getenv("MPCX_SIGN_PAIRED");
  const bool paired = !(pe && pe[0] == '0');
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
    // One pair's protocol steps (Alice i, Bob j)
    auto alice_init = [&](size_t pi) {
      const Pair& p = pairs[pi];
      std::vector<uint8_t> err;
      mta::AliceInitBatch(nodes[p.i].sk.pub, sl(k[p.i]), public_dln(nodes[p.j].dln), L[pi].ra, &L[pi].cA, &L[pi].pfA,
                          &err);
      count_err(err);
    };
    auto bob_mid = [&](size_t pi, bool wc) {  // BobMid(gamma_j) / BobMidWC(w_j, W_j)
      const Pair& p = pairs[pi];
      std::vector<uint8_t> err;
      std::vector<secp::Affine> Wj;
      if (wc) {
        join_ec();
        Wj = slp(Wp[p.j]);
      }
      mta::BobMidBatch(cs, nodes[p.i].sk.pub, L[pi].pfA, sl(wc ? w[p.j] : g[p.j]), L[pi].cA,
                       public_dln(nodes[p.i].dln), nodes[p.j].dln, wc ? &Wj : nullptr, wc ? L[pi].rbwc : L[pi].rb,
                       wc ? &L[pi].bobwc : &L[pi].bob, &err);
      count_err(err);
    };
    auto alice_end = [&](size_t pi, bool wc) {  // AliceEnd / AliceEndWC
      const Pair& p = pairs[pi];
      const auto& bm = wc ? L[pi].bobwc : L[pi].bob;
      std::vector<mta::ProofBob> pf(n);
      std::vector<Nat> cB(n);
      for (size_t x = 0; x < n; ++x) {
        pf[x] = bm[x].pf;
        cB[x] = bm[x].cB;
      }
      std::vector<uint8_t> err;
      const std::vector<secp::Affine> Wj = wc ? slp(Wp[p.j]) : std::vector<secp::Affine>{};
      mta::AliceEndBatch(cs, nodes[p.i].sk, pf, nodes[p.i].dln, L[pi].cA, cB, wc ? &Wj : nullptr,
                         wc ? &L[pi].mu : &L[pi].alpha, &err);
      count_err(err);
    };
    // BobMid + BobMidWC (and AliceEnd + AliceEndWC) of a pair as one paired
    // batch: one RangeProofAlice verification, launches twice as large
    auto bob_mid_pair = [&](size_t pi) {
      const Pair& p = pairs[pi];
      std::vector<uint8_t> err, errwc;
      join_ec();
      const std::vector<secp::Affine> Wj = slp(Wp[p.j]);
      mta::BobMidPairBatch(cs, nodes[p.i].sk.pub, L[pi].pfA, sl(g[p.j]), sl(w[p.j]), L[pi].cA,
                           public_dln(nodes[p.i].dln), nodes[p.j].dln, Wj, L[pi].rb, L[pi].rbwc, &L[pi].bob,
                           &L[pi].bobwc, &err, &errwc);
      count_err(err);
      count_err(errwc);
    };
    auto alice_end_pair = [&](size_t pi) {
      const Pair& p = pairs[pi];
      std::vector<mta::ProofBob> pf(n), pfwc(n);
      std::vector<Nat> cB(n), cBwc(n);
      for (size_t x = 0; x < n; ++x) {
        pf[x] = L[pi].bob[x].pf;
        cB[x] = L[pi].bob[x].cB;
        pfwc[x] = L[pi].bobwc[x].pf;
        cBwc[x] = L[pi].bobwc[x].cB;
      }
      std::vector<uint8_t> err, errwc;
      const std::vector<secp::Affine> Wj = slp(Wp[p.j]);
      mta::AliceEndPairBatch(cs, nodes[p.i].sk, pf, pfwc, nodes[p.i].dln, L[pi].cA, cB, cBwc, Wj, &L[pi].alpha,
                             &L[pi].mu, &err, &errwc);
      count_err(err);
      count_err(errwc);
    };
    const size_t np = pairs.size();
    std::vector<double> st1(np), st2(np), st3(np);
    if (chains) {
      // Each ordered pair's chain -- AliceInit, then BobMid || BobMidWC, then
      // AliceEnd || AliceEndWC -- depends only on its own outputs: the chains
      // run concurrently with no barrier between rounds, so one chain's host
      // phases (draws, hashing, gcd batches, packing) overlap another chain's
      // GPU batches instead of every task reaching its host phase in lockstep.
      std::vector<std::function<void()>> tasks;
      for (size_t pi = 0; pi < np; ++pi)
        tasks.push_back([&, pi] {
          if (stagger_ms > 0 && pi) std::this_thread::sleep_for(std::chrono::microseconds((long)(stagger_ms * 1000 * pi)));
          const double a0 = now();
          alice_init(pi);
          const double a1 = now();
          if (paired) bob_mid_pair(pi);
          else run_tasks({[&] { bob_mid(pi, false); }, [&] { bob_mid(pi, true); }});
          const double a2 = now();
          if (paired) alice_end_pair(pi);
          else run_tasks({[&] { alice_end(pi, false); }, [&] { alice_end(pi, true); }});
          st1[pi] = a1 - a0;
          st2[pi] = a2 - a1;
          st3[pi] = now() - a2;
        });
      run_tasks(tasks);
    } else {  // rounds with a barrier between them (A/B: MPCX_SIGN_CHAINS=0)
      std::vector<std::function<void()>> t1, t2, t3;
      for (size_t pi = 0; pi < np; ++pi) {
        t1.push_back([&, pi] { alice_init(pi); });
        if (paired) {
          t2.push_back([&, pi] { bob_mid_pair(pi); });
          t3.push_back([&, pi] { alice_end_pair(pi); });
          continue;
        }
        t2.push_back([&, pi] { bob_mid(pi, false); });
        t2.push_back([&, pi] { bob_mid(pi, true); });
        t3.push_back([&, pi] { alice_end(pi, false); });
        t3.push_back([&, pi] { alice_end(pi, true); });
      }
      const double a0 = now();
      run_tasks(t1);
      const double a1 = now();
      run_tasks(t2);
      const double a2 = now();
      run_tasks(t3);
      const double a3 = now();
      std::fill(st1.begin(), st1.end(), a1 - a0);
      std::fill(st2.begin(), st2.end(), a2 - a1);
      std::fill(st3.begin(), st3.end(), a3 - a2);
    }
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
    // rounds 4-9 + finalize and ecdsa.Verify (see signing.hpp), per wallet
    parallel_for(n, [&](size_t x) {
      MPCX_PROF("sign.finalize_verify");
      const size_t wi = lo + x;
      uint64_t bad = 0;
      for (const auto& p : pairs) {
        bad += (p.alpha[wi] + p.bob[wi].beta) % q != (k[p.i][wi] * g[p.j][wi]) % q;
        bad += (p.mu[wi] + p.bobwc[wi].beta) % q != (k[p.i][wi] * w[p.j][wi]) % q;
      }
      if (bad) relation_failures += bad;
      Nat delta, s_sum, sigma_sum;
      const secp::Affine& Gam = GamW[wi];  // sum_i Gamma_i (decommitted in round 4)
      const secp::Affine& X = XW[wi];      // the wallet key sum_i W_i
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
      const secp::Affine P = secp::LinComb((msg[wi] * sinv) % q, X, (r * sinv) % q);
      verified[wi] = !P.inf && secp::FeToNat(P.x) % q == r;
    });
    const double c4 = now();
    if (prof::enabled()) {  // seconds with no libmpcx call in flight (one chunk: exact)
      static const int s13 = prof::slot_of("sign.gpu_idle.rounds1_3"), s4 = prof::slot_of("sign.gpu_idle.finalize");
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

  // chunking: MPCX_SIGN_PIPELINE="chunks,workers". Default: three concurrent
  // third-wallet pipelines for 2 signers (2 ordered pairs leave the GPU idle
  // while every chain is in a host phase; the halves' phases interleave), one
  // for more signers (their 6+ chains already keep the GPU ~75% busy, and half
  // launches cost more GPU time): measured on MI355X with the shared host pool,
  // profiles/r02/pipe_ab/ (before the pool, halves measured slower)
  // (three pipelines measured mean 6,036 vs 5,770 for two, four alternating pairs, profiles/r02/pipe_ab/)
  size_t n_chunks = pairs.size() <= 2 ? 3 : 1, n_workers = n_chunks;
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
    // MPCX_SIGN_CHUNK_STAGGER_MS: worker t starts t times this late, so the
    // pipelines' host phases fall into each other's launch phases
    // (default 60 ms with two pipelines: mean 5,699 vs 5,478 sigs/s unstaggered,
    // 150 ms 5,647, three alternating runs each, profiles/r02/stag_ab/)
    const char* cs = std::getenv("MPCX_SIGN_CHUNK_STAGGER_MS");
    const double chunk_stagger_ms = cs ? std::atof(cs) : (n_workers == 2 ? 60.0 : 0.0);
    for (size_t t = 0; t < n_workers; ++t)
      workers.push_back([&, t] {
        if (chunk_stagger_ms > 0 && t)
          std::this_thread::sleep_for(std::chrono::microseconds((long)(chunk_stagger_ms * 1000 * (double)t)));
        for (;;) {
          const size_t c = next.fetch_add(1);
          if (c >= n_chunks) return;
          run_chunk(Wn * c / n_chunks, Wn * (c + 1) / n_chunks);
        }
      });
    if (Wn) run_tasks(workers);
  }
  st.relation_failures = relation_failures.load();
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
