// expset.hpp -- batches of modular exponentiations against one modulus,
// issued as few GPU launches (libmpcx.so through Engine). Used by the MtA
// (mta.cpp) and keygen-proof (proofs.cpp) batch mirrors.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <exception>
#include <functional>
#include <initializer_list>
#include <map>
#include <thread>
#include <vector>

#include "bignum.hpp"
#include "engine.hpp"
#include "hostprof.hpp"

namespace mpcx::host {

// Runs every closure concurrently (the last one on the calling thread) and
// rethrows the first failure once all have finished. libmpcx runs calls from
// different threads on different execution lanes (streams), so independent
// launches of one protocol step overlap on the GPU instead of queueing.
inline void run_concurrently(const std::vector<std::function<void()>>& fs) {
  if (fs.empty()) return;
  static const bool serial = [] {  // MPCX_EXPSET_SERIAL=1: one launch after another (A/B runs)
    const char* e = std::getenv("MPCX_EXPSET_SERIAL");
    return e && e[0] == '1';
  }();
  if (serial) {
    for (const auto& f : fs) f();
    return;
  }
  std::vector<std::exception_ptr> errs(fs.size());
  std::vector<std::thread> th;
  const int chain = prof::chain();
  for (size_t i = 0; i + 1 < fs.size(); ++i)
    th.emplace_back([&, i, chain] {
      MPCX_PROF_CPU("cpu.launch_threads");
      prof::set_chain(chain);
      try {
        fs[i]();
      } catch (...) {
        errs[i] = std::current_exception();
      }
    });
  try {
    fs.back()();
  } catch (...) {
    errs.back() = std::current_exception();
  }
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// ------------------------------------------------------------------ ExpSet
// Modexp requests against one modulus, issued as few GPU launches: large
// groups of requests that share one exponent object (y = N, y = lambda) go to
// a shared-exponent launch; the rest are grouped by exponent length (the kernel processes the
// group's longest exponent, so lengths within a group differ by <= 1/8).
// Products base^e * mul run fused (mpcx_modexp_mul_batch).
class ExpSet {
 public:
  explicit ExpSet(const Nat& m) : m_(m) {}
  void add(const Nat& base, const Nat& e, Nat* out, const Nat* mul = nullptr) {
    reqs_.push_back({&base, &e, mul, out});
  }
  // out = (mul ? mul : 1) * b1^e1 * b2^e2 mod m: two recurring bases (h1^x h2^y
  // of the range proofs) in ONE comb launch, both exponents' windows chained
  // into one accumulator (k_fixedbase with two tables), instead of a launch per
  // base with the second waiting on the first
  void add2(const Nat& b1, const Nat& e1, const Nat& b2, const Nat& e2, Nat* out, const Nat* mul = nullptr) {
    reqs2_.push_back({&b1, &e1, &b2, &e2, mul, out});
  }
  size_t size() const { return reqs_.size() + reqs2_.size(); }
  // Every launch of the pending requests, concurrently; the set is empty after.
  void run() {
    std::vector<std::function<void()>> fs;
    collect(fs);
    run_concurrently(fs);
    clear();
  }
  // Appends one closure per launch of the pending requests (run them, e.g. with
  // run_concurrently together with other sets' launches, then clear()).
  void collect(std::vector<std::function<void()>>& fs) {
    collect2(fs);
    if (reqs_.empty()) return;
    // A base recurring across many requests (h1, h2 of N~ in every session's
    // range proof) goes to the fixed-base comb path: no squarings, one
    // product per 8-bit window. Sorted by exponent length, so wavefronts are
    // homogeneous and skip the windows above their exponents.
    std::vector<uint8_t> done(reqs_.size(), 0);
    if (Engine::get().fixed_base_ok(m_)) {
      std::map<const Nat*, std::vector<size_t>> by_b;
      for (size_t i = 0; i < reqs_.size(); ++i)  // over-long (peer-supplied) exponents: per-operand path
        if (reqs_[i].e->bit_len() <= Engine::kFixedMaxBits) by_b[reqs_[i].b].push_back(i);
      for (auto& kv : by_b) {
        if (kv.second.size() < kFixedMin) continue;
        auto idx = kv.second;
        std::stable_sort(idx.begin(), idx.end(),
                         [&](size_t a, size_t b) { return reqs_[a].e->bit_len() < reqs_[b].e->bit_len(); });
        for (size_t i : idx) done[i] = 1;
        fs.push_back([this, idx] { launch_fixed(idx); });
      }
    }
    std::map<const Nat*, std::vector<size_t>> by_e;
    for (size_t i = 0; i < reqs_.size(); ++i)
      if (!done[i]) by_e[reqs_[i].e].push_back(i);
    std::vector<size_t> rest;
    for (auto& kv : by_e) {
      // a shared-exponent launch only for a large group (y = N, y = lambda);
      // a session's own e used by two requests stays in the per-operand groups
      if (kv.second.size() >= 64 || kv.second.size() == reqs_.size()) {
        auto idx = kv.second;
        fs.push_back([this, idx] { launch(idx, true); });
      } else {
        rest.insert(rest.end(), kv.second.begin(), kv.second.end());
      }
    }
    std::sort(rest.begin(), rest.end(),
              [&](size_t a, size_t b) { return reqs_[a].e->bit_len() < reqs_[b].e->bit_len(); });
    size_t g0 = 0;
    while (g0 < rest.size()) {
      const uint32_t lo = reqs_[rest[g0]].e->bit_len();
      size_t g1 = g0 + 1;
      while (g1 < rest.size() && reqs_[rest[g1]].e->bit_len() <= lo + lo / 8 + 32) ++g1;
      std::vector<size_t> idx(rest.begin() + (long)g0, rest.begin() + (long)g1);
      fs.push_back([this, idx] { launch(idx, false); });
      g0 = g1;
    }
  }
  void clear() {
    reqs_.clear();
    reqs2_.clear();
  }

 private:
  struct Req {
    const Nat* b;
    const Nat* e;
    const Nat* mul;
    Nat* out;
  };
  struct Req2 {
    const Nat *b1, *e1, *b2, *e2, *mul;
    Nat* out;
  };
  // two-base requests: per (b1, b2) pair one two-table comb launch when the
  // comb path takes them; otherwise b1^e1 first, then b2^e2 times it
  void collect2(std::vector<std::function<void()>>& fs) {
    if (reqs2_.empty()) return;
    std::map<std::pair<const Nat*, const Nat*>, std::vector<size_t>> by_b;
    for (size_t i = 0; i < reqs2_.size(); ++i) by_b[{reqs2_[i].b1, reqs2_[i].b2}].push_back(i);
    const bool comb = Engine::get().fixed_base_ok(m_);
    for (auto& kv : by_b) {
      // only the requests with an over-long (peer-supplied, unbounded) exponent
      // leave the comb path; the rest of the group stays on it
      std::vector<size_t> idx, longx;
      for (size_t i : kv.second)
        (reqs2_[i].e1->bit_len() <= Engine::kFixedMaxBits && reqs2_[i].e2->bit_len() <= Engine::kFixedMaxBits
             ? idx
             : longx)
            .push_back(i);
      if (!comb || idx.size() < kFixedMin) {
        idx.insert(idx.end(), longx.begin(), longx.end());
        longx.clear();
        std::sort(idx.begin(), idx.end());
        fs.push_back([this, idx] { launch_two_step(idx); });
        continue;
      }
      std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
        return std::max(reqs2_[a].e1->bit_len(), reqs2_[a].e2->bit_len()) <
               std::max(reqs2_[b].e1->bit_len(), reqs2_[b].e2->bit_len());
      });
      fs.push_back([this, idx] { launch_fixed2(idx); });
      if (!longx.empty()) fs.push_back([this, longx] { launch_two_step(longx); });
    }
  }
  void launch_fixed2(const std::vector<size_t>& idx) {
    MPCX_PROF("expset.launch_fixed2");
    const size_t n = idx.size();
    std::vector<const Nat*> e1(n), e2(n), muls;
    std::vector<Nat*> outs(n);
    bool any_mul = false;
    for (size_t i : idx) any_mul |= reqs2_[i].mul != nullptr;
    if (any_mul) muls.resize(n);
    for (size_t j = 0; j < n; ++j) {
      const Req2& r = reqs2_[idx[j]];
      e1[j] = r.e1;
      e2[j] = r.e2;
      outs[j] = r.out;
      if (any_mul) muls[j] = r.mul;
    }
    const Nat* bases[2] = {reqs2_[idx[0]].b1, reqs2_[idx[0]].b2};
    const Nat* const* exps[2] = {e1.data(), e2.data()};
    Engine::get().fixed_multi_into(m_, 2, bases, n, exps, any_mul ? muls.data() : nullptr, outs.data());
  }
  void launch_two_step(const std::vector<size_t>& idx) {
    MPCX_PROF("expset.launch_two_step");
    const size_t n = idx.size();
    std::vector<Nat> t(n);
    std::vector<const Nat*> b(n), e(n), muls;
    std::vector<Nat*> outs(n);
    bool any_mul = false;
    for (size_t i : idx) any_mul |= reqs2_[i].mul != nullptr;
    for (size_t j = 0; j < n; ++j) {
      b[j] = reqs2_[idx[j]].b1;
      e[j] = reqs2_[idx[j]].e1;
      outs[j] = &t[j];
    }
    if (any_mul) {
      muls.resize(n);
      for (size_t j = 0; j < n; ++j) muls[j] = reqs2_[idx[j]].mul;
    }
    Engine::get().exp_into(m_, n, b.data(), e.data(), n, any_mul ? muls.data() : nullptr, outs.data());
    std::vector<const Nat*> tm(n);
    for (size_t j = 0; j < n; ++j) {
      b[j] = reqs2_[idx[j]].b2;
      e[j] = reqs2_[idx[j]].e2;
      tm[j] = &t[j];
      outs[j] = reqs2_[idx[j]].out;
    }
    Engine::get().exp_into(m_, n, b.data(), e.data(), n, tm.data(), outs.data());
  }
  static constexpr size_t kFixedMin = 64;  // requests on one base before a comb table pays
  // the requests' own operands and outputs, through pointers: no copies
  void launch_fixed(const std::vector<size_t>& idx) {
    MPCX_PROF("expset.launch_fixed");
    std::vector<const Nat*> exps(idx.size()), muls;
    std::vector<Nat*> outs(idx.size());
    bool any_mul = false;
    for (size_t i : idx) any_mul |= reqs_[i].mul != nullptr;
    if (any_mul) muls.resize(idx.size());
    for (size_t j = 0; j < idx.size(); ++j) {
      const Req& r = reqs_[idx[j]];
      exps[j] = r.e;
      outs[j] = r.out;
      if (any_mul) muls[j] = r.mul;
    }
    Engine::get().fixed_exp_into(m_, *reqs_[idx[0]].b, idx.size(), exps.data(), any_mul ? muls.data() : nullptr,
                                 outs.data());
  }
  void launch(const std::vector<size_t>& idx, bool shared) {
    MPCX_PROF("expset.launch");
    std::vector<const Nat*> bases(idx.size()), exps(shared ? 1 : idx.size()), muls;
    std::vector<Nat*> outs(idx.size());
    bool any_mul = false;
    for (size_t i : idx) any_mul |= reqs_[i].mul != nullptr;
    if (any_mul) muls.resize(idx.size());
    for (size_t j = 0; j < idx.size(); ++j) {
      const Req& r = reqs_[idx[j]];
      bases[j] = r.b;
      if (!shared) exps[j] = r.e;
      outs[j] = r.out;
      if (any_mul) muls[j] = r.mul;
    }
    if (shared) exps[0] = reqs_[idx[0]].e;
    Engine::get().exp_into(m_, idx.size(), bases.data(), exps.data(), exps.size(), any_mul ? muls.data() : nullptr,
                           outs.data());
  }
  const Nat m_;  // by value: callers pass temporaries (pk.NSquare())
  std::vector<Req> reqs_;
  std::vector<Req2> reqs2_;
};

// Every launch of several sets (one protocol step's moduli: N^2, N~, N) at once.
inline void run_all(std::initializer_list<ExpSet*> sets) {
  std::vector<std::function<void()>> fs;
  for (ExpSet* s : sets) s->collect(fs);
  run_concurrently(fs);
  for (ExpSet* s : sets) s->clear();
}

}  // namespace mpcx::host
