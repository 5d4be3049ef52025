// expset.hpp -- batches of modular exponentiations against one modulus,
// issued as few GPU launches (libmpcx.so through Engine). Used by the MtA
// (mta.cpp) and keygen-proof (proofs.cpp) batch mirrors.
#pragma once

#include <algorithm>
#include <map>
#include <vector>

#include "bignum.hpp"
#include "engine.hpp"
#include "hostprof.hpp"

namespace mpcx::host {

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
  size_t size() const { return reqs_.size(); }
  void run() {
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
        auto& idx = kv.second;
        std::stable_sort(idx.begin(), idx.end(),
                         [&](size_t a, size_t b) { return reqs_[a].e->bit_len() < reqs_[b].e->bit_len(); });
        launch_fixed(idx);
        for (size_t i : idx) done[i] = 1;
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
        launch(kv.second, true);
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
      launch(std::vector<size_t>(rest.begin() + (long)g0, rest.begin() + (long)g1), false);
      g0 = g1;
    }
    reqs_.clear();
  }

 private:
  struct Req {
    const Nat* b;
    const Nat* e;
    const Nat* mul;
    Nat* out;
  };
  static constexpr size_t kFixedMin = 64;  // requests on one base before a comb table pays
  void launch_fixed(const std::vector<size_t>& idx) {
    MPCX_PROF("expset.launch_fixed");
    std::vector<Nat> exps, muls;
    exps.reserve(idx.size());
    bool any_mul = false;
    for (size_t i : idx) any_mul |= reqs_[i].mul != nullptr;
    for (size_t i : idx) {
      exps.push_back(*reqs_[i].e);
      if (any_mul) muls.push_back(reqs_[i].mul ? *reqs_[i].mul : Nat(1));
    }
    std::vector<Nat> r = Engine::get().fixed_exp(m_, *reqs_[idx[0]].b, exps, any_mul ? &muls : nullptr);
    for (size_t j = 0; j < idx.size(); ++j) *reqs_[idx[j]].out = std::move(r[j]);
  }
  void launch(const std::vector<size_t>& idx, bool shared) {
    MPCX_PROF("expset.launch");
    std::vector<Nat> bases, exps, muls;
    bases.reserve(idx.size());
    bool any_mul = false;
    for (size_t i : idx) any_mul |= reqs_[i].mul != nullptr;
    for (size_t i : idx) {
      bases.push_back(*reqs_[i].b);
      if (!shared) exps.push_back(*reqs_[i].e);
      if (any_mul) muls.push_back(reqs_[i].mul ? *reqs_[i].mul : Nat(1));
    }
    if (shared) exps.push_back(*reqs_[idx[0]].e);
    std::vector<Nat> r = Engine::get().exp(m_, bases, exps, any_mul ? &muls : nullptr);
    for (size_t j = 0; j < idx.size(); ++j) *reqs_[idx[j]].out = std::move(r[j]);
  }
  const Nat m_;  // by value: callers pass temporaries (pk.NSquare())
  std::vector<Req> reqs_;
};

}  // namespace mpcx::host
