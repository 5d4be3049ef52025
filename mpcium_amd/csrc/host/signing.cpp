// signing.cpp -- see signing.hpp.
#include "signing.hpp"

#include "engine.hpp"

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

MtaStats RunSigningMtA(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed) {
  if (signers < 2 || (size_t)signers > nodes.size()) throw std::invalid_argument("signers must be in [2, nodes]");
  const Nat& q = mta::Q();
  const size_t S = (size_t)signers, Wn = wallets;
  MtaStats st;
  st.wallets = Wn;
  // per wallet and signer: k_i, gamma_i, w_i < q; W_i = w_i G; one session id per wallet
  std::vector<std::vector<Nat>> k(S, std::vector<Nat>(Wn)), g(S, std::vector<Nat>(Wn)), w(S, std::vector<Nat>(Wn));
  std::vector<std::vector<secp::Affine>> Wp(S, std::vector<secp::Affine>(Wn));
  std::vector<mta::Bytes> sess(Wn);
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
  st.round1_s = t1 - t0;
  st.round2_s = t2 - t1;
  st.round3_s = t3 - t2;
  st.total_s = t3 - t0;
  st.errors = errors.load();
  st.engine_busy_s = Engine::get().busy_seconds();
  return st;
}

}  // namespace mpcx::host::signing
