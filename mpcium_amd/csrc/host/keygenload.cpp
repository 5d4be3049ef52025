// keygenload.cpp -- see keygenload.hpp.
#include "keygenload.hpp"

#include <atomic>
#include <mutex>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <memory>
#include <stdexcept>
#include <thread>

#include "engine.hpp"
#include "proofs.hpp"

namespace mpcx::host::keygenload {
namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

uint64_t mix(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t x = seed ^ (a * 0x9E3779B97F4A7C15ull) ^ (b * 0xC2B2AE3D27D4EB4Full) ^ (c * 0x165667B19E3779F9ull);
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  return x;
}

// at most `width` tasks at a time (each task's host steps are parallel_for'd)
void run_bounded(const std::vector<std::function<void()>>& tasks, size_t width) {
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> errs(tasks.size());
  auto worker = [&] {
    for (;;) {
      const size_t t = next.fetch_add(1);
      if (t >= tasks.size()) return;
      try {
        tasks[t]();
      } catch (...) {
        errs[t] = std::current_exception();
      }
    }
  };
  std::vector<std::thread> th;
  for (size_t w = 0; w < std::min(width, tasks.size()); ++w) th.emplace_back(worker);
  for (auto& x : th) x.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// one random stream per (session, party, proof kind, peer)
struct Streams {
  std::vector<CounterDRBG> drbg;
  std::vector<RandFn> fn;
  Streams(uint64_t seed, size_t sessions, uint64_t party, uint64_t kind) {
    drbg.reserve(sessions);
    for (size_t s = 0; s < sessions; ++s) drbg.emplace_back(mix(seed, s, party, kind));
    for (auto& d : drbg) fn.push_back(d.fn());
  }
};

}  // namespace

ProofStats RunKeygenProofs(const std::vector<PartyKeys>& parties, size_t sessions, uint64_t seed) {
  const size_t n = parties.size();
  if (n < 2) throw std::invalid_argument("need at least two parties");
  ProofStats st;
  st.sessions = sessions;
  st.parties = n;
  // session ids (SSID bytes) shared by the parties of a session
  std::vector<proofs::Bytes> sess(sessions);
  {
    CounterDRBG d(mix(seed, 0xFFFF, 0, 0));
    for (auto& b : sess) {
      b.resize(32);
      d.read(b.data(), 32);
    }
  }
  std::vector<std::vector<proofs::DLNProof>> dln1(n), dln2(n);
  std::vector<std::vector<proofs::ModProof>> mod(n);
  std::vector<std::vector<std::vector<proofs::FacProof>>> fac(n, std::vector<std::vector<proofs::FacProof>>(n));
  std::vector<std::unique_ptr<Streams>> streams;
  auto stream = [&](uint64_t party, uint64_t kind) -> const std::vector<RandFn>& {
    streams.push_back(std::make_unique<Streams>(seed, sessions, party, kind));
    return streams.back()->fn;
  };
  // streams are created up front (the task bodies only read them)
  std::vector<const std::vector<RandFn>*> r_dln1(n), r_dln2(n), r_mod(n);
  std::vector<std::vector<const std::vector<RandFn>*>> r_fac(n, std::vector<const std::vector<RandFn>*>(n));
  for (size_t i = 0; i < n; ++i) {
    r_dln1[i] = &stream(i, 1);
    r_dln2[i] = &stream(i, 2);
    r_mod[i] = &stream(i, 3);
    for (size_t j = 0; j < n; ++j)
      if (j != i) r_fac[i][j] = &stream(i, 16 + j);
  }
  const size_t width = 8;
  const char* ce = std::getenv("MPCX_KEYGEN_CHAINS");
  const bool chains = !(ce && ce[0] == '0');
  std::atomic<uint64_t> fails{0};
  auto count = [&](const std::vector<uint8_t>& ok) {
    uint64_t f = 0;
    for (auto v : ok) f += v == 0;
    fails += f;
  };
  st.proofs = (uint64_t)sessions * n * (3 + (n - 1));
  st.verifications = (uint64_t)sessions * n * (n - 1) * 4;
  // One chain per proof batch: prove, then every peer's verification of it.
  // A verification depends only on its proof, so the chains run with no
  // barrier between proving and verifying: one chain's host steps overlap
  // another's GPU batches.
  std::mutex tm;
  double last_prove = 0;
  auto proved = [&] {
    std::lock_guard<std::mutex> lk(tm);
    last_prove = std::max(last_prove, now());
  };
  // lane budget of this workload (MPCX_KEYGEN_LANES, default 8: its many small
  // independent chains overlap better; measured +10-15% over 4), restored after
  const char* kl = std::getenv("MPCX_KEYGEN_LANES");
  const int lanes = kl ? std::atoi(kl) : 8;
  struct LaneBudget {
    int prev = 0;
    explicit LaneBudget(int n) {
      if (n >= 1 && n <= 8) prev = Engine::get().set_lanes(n);
    }
    ~LaneBudget() {
      try {
        if (prev) Engine::get().set_lanes(prev);
      } catch (...) {  // no throw from a destructor; the next call reports libmpcx's state
      }
    }
  } budget(lanes);
  Engine::get().reset_busy();
  const double t0 = now();
  {
    std::vector<std::function<void()>> tasks;
    for (size_t i = 0; i < n; ++i) {
      const PartyKeys& P = parties[i];
      tasks.push_back([&, i] {
        dln1[i] = proofs::DLNProveBatch(P.h1, P.h2, P.alpha, P.p, P.q, P.NTilde, *r_dln1[i]);
        proved();
        for (size_t j = 0; j < n; ++j)
          if (j != i) count(proofs::DLNVerifyBatch(P.h1, P.h2, P.NTilde, dln1[i]));
      });
      tasks.push_back([&, i] {
        dln2[i] = proofs::DLNProveBatch(P.h2, P.h1, P.beta, P.p, P.q, P.NTilde, *r_dln2[i]);
        proved();
        for (size_t j = 0; j < n; ++j)
          if (j != i) count(proofs::DLNVerifyBatch(P.h2, P.h1, P.NTilde, dln2[i]));
      });
      tasks.push_back([&, i] {
        mod[i] = proofs::ModProveBatch(sess, P.sk.pub.N, P.sk.P, P.sk.Q, *r_mod[i]);
        proved();
        for (size_t j = 0; j < n; ++j)
          if (j != i) count(proofs::ModVerifyBatch(sess, P.sk.pub.N, mod[i]));
      });
      for (size_t j = 0; j < n; ++j) {
        if (j == i) continue;
        tasks.push_back([&, i, j] {
          const PartyKeys& V = parties[j];
          fac[i][j] = proofs::FacProveBatch(sess, P.sk.pub.N, V.NTilde, V.h1, V.h2, P.sk.P, P.sk.Q, *r_fac[i][j]);
          proved();
          count(proofs::FacVerifyBatch(sess, P.sk.pub.N, V.NTilde, V.h1, V.h2, fac[i][j]));
        });
      }
    }
    if (chains) {
      run_bounded(tasks, width);
    } else {  // every proof first, then every verification (MPCX_KEYGEN_CHAINS=0)
      std::vector<std::function<void()>> prove, verify;
      for (size_t i = 0; i < n; ++i) {
        const PartyKeys& P = parties[i];
        prove.push_back([&, i] { dln1[i] = proofs::DLNProveBatch(P.h1, P.h2, P.alpha, P.p, P.q, P.NTilde, *r_dln1[i]); });
        prove.push_back([&, i] { dln2[i] = proofs::DLNProveBatch(P.h2, P.h1, P.beta, P.p, P.q, P.NTilde, *r_dln2[i]); });
        prove.push_back([&, i] { mod[i] = proofs::ModProveBatch(sess, P.sk.pub.N, P.sk.P, P.sk.Q, *r_mod[i]); });
        for (size_t j = 0; j < n; ++j) {
          if (j == i) continue;
          const PartyKeys& V = parties[j];
          prove.push_back([&, i, j] {
            fac[i][j] = proofs::FacProveBatch(sess, P.sk.pub.N, V.NTilde, V.h1, V.h2, P.sk.P, P.sk.Q, *r_fac[i][j]);
          });
          verify.push_back([&, i] { count(proofs::DLNVerifyBatch(P.h1, P.h2, P.NTilde, dln1[i])); });
          verify.push_back([&, i] { count(proofs::DLNVerifyBatch(P.h2, P.h1, P.NTilde, dln2[i])); });
          verify.push_back([&, i] { count(proofs::ModVerifyBatch(sess, P.sk.pub.N, mod[i])); });
          verify.push_back([&, i, j] { count(proofs::FacVerifyBatch(sess, P.sk.pub.N, V.NTilde, V.h1, V.h2, fac[i][j])); });
        }
      }
      run_bounded(prove, width);
      proved();
      run_bounded(verify, width);
    }
  }
  const double t2 = now();
  st.prove_s = last_prove - t0;  // until the last proof batch was done
  st.verify_s = t2 - last_prove;  // verification tail after it
  st.total_s = t2 - t0;
  st.failures = fails.load();
  st.engine_busy_s = Engine::get().busy_seconds();
  st.alg_macs = Engine::get().alg_macs();
  return st;
}

}  // namespace mpcx::host::keygenload
