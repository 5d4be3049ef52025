// Engine stress on the CPU (test infrastructure; tools/engine_stress.sh builds
// it under ASAN or TSAN against tools/mock_mpcx.cpp). Many threads issue
// comb (fixed_multi_into, one or two bases) and generic (exp_into) batches of
// random sizes over a few moduli and bases, with exponent lengths that grow
// over the run so comb tables are rebuilt (3,072 -> 5,120 bits) while other
// threads still launch on the old ones, the 2-GB-per-table mock footprint
// makes the cache evict under load, and the mock refuses a share of the
// pinned allocations (the pageable fallback). Every output is checked against
// the mock's result function: a group routed to another caller's buffer, a
// read past a caller's range, a table used after release or a data race fails
// the run (the coalescer with concurrent table growth and
// a forced pageable fallback).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "engine.hpp"

extern "C" uint64_t mock_launches();
extern "C" uint64_t mock_pin_refusals();

using namespace mpcx::host;

namespace {
Nat rand_nat(std::mt19937_64& rng, uint32_t bits) {
  std::vector<uint32_t> w((bits + 31) / 32);
  for (auto& x : w) x = (uint32_t)rng();
  if (bits % 32) w.back() &= (1u << (bits % 32)) - 1u;
  return Nat::from_words(w.data(), w.size());
}
Nat rand_below(std::mt19937_64& rng, const Nat& m) {
  for (;;) {
    Nat x = rand_nat(rng, m.bit_len());
    if (x < m) return x;
  }
}
uint32_t w_at(const Nat& x, size_t j) { return j < x.words() ? x.limbs()[j] : 0u; }
}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 12;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 60;
  Engine& eng = Engine::get();
  eng.init(0);
  std::mt19937_64 seed_rng(12345);
  // moduli: two 2048-bit (comb class) and one 4096-bit; bases below them
  std::vector<Nat> mods;
  for (uint32_t bits : {2048u, 2047u, 4096u}) {
    Nat m = rand_nat(seed_rng, bits) + (Nat(1) << (bits - 1));
    if (!m.is_odd()) m = m + Nat(1);
    if (m.bit_len() > bits) m = m - Nat(2);
    mods.push_back(m);
  }
  std::vector<Nat> bases;
  for (int i = 0; i < 4; ++i) bases.push_back(rand_below(seed_rng, mods[i % 2]));
  std::atomic<uint64_t> checked{0}, bad{0}, ops{0};
  std::atomic<int> phase{0};  // exponent growth: 3072 + 512 * phase bits (<= 5120)
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      std::mt19937_64 rng(1000 + t);
      for (int it = 0; it < iters; ++it) {
        if (t == 0 && it % std::max(1, iters / 5) == 0) phase.store(std::min(4, it / std::max(1, iters / 5)));
        const size_t n = 1 + rng() % (rng() % 4 == 0 ? 3000 : 300);
        const bool comb = rng() % 3 != 0;
        const bool with_mul = rng() % 2;
        if (comb) {
          const size_t mi = rng() % 2;
          const Nat& m = mods[mi];
          const size_t nb = 1 + rng() % 2;
          const Nat* bs[2] = {&bases[mi], &bases[mi + 2]};
          const uint32_t maxb = 3072 + 512 * (uint32_t)phase.load();
          std::vector<Nat> e[2], mul(with_mul ? n : 0), out(n);
          std::vector<const Nat*> ep[2], mp;
          std::vector<Nat*> op(n);
          for (size_t b = 0; b < nb; ++b) {
            e[b].resize(n);
            ep[b].resize(n);
            for (size_t i = 0; i < n; ++i) {
              e[b][i] = rand_nat(rng, 1 + (uint32_t)(rng() % maxb));
              ep[b][i] = &e[b][i];
            }
          }
          for (size_t i = 0; i < n; ++i) {
            if (with_mul) mul[i] = rand_below(rng, m);
            op[i] = &out[i];
          }
          if (with_mul)
            for (auto& x : mul) mp.push_back(&x);
          const Nat* const* eps[2] = {ep[0].data(), nb > 1 ? ep[1].data() : nullptr};
          eng.fixed_multi_into(m, nb, bs, n, eps, with_mul ? mp.data() : nullptr, op.data());
          uint32_t tag = 0;
          for (size_t b = 0; b < nb; ++b) tag ^= w_at(*bs[b], 0) ^ w_at(m, 0);
          for (size_t i = 0; i < n; ++i) {
            std::vector<uint32_t> w(m.words());
            for (size_t j = 0; j < w.size(); ++j) {
              uint32_t v = j == 0 ? tag : 0u;
              for (size_t b = 0; b < nb; ++b) v ^= w_at(e[b][i], j);
              v ^= with_mul ? w_at(mul[i], j) : (j == 0 ? 1u : 0u);
              w[j] = v;
            }
            if (Nat::from_words(w.data(), w.size()) != out[i]) bad++;
            checked++;
          }
        } else {
          const Nat& m = mods[rng() % 3];
          const bool shared = rng() % 2;
          std::vector<Nat> b(n), e(shared ? 1 : n), mul(with_mul ? n : 0), out(n);
          for (auto& x : b) x = rand_below(rng, m);
          for (auto& x : e) x = rand_nat(rng, 1 + (uint32_t)(rng() % 2100));
          for (auto& x : mul) x = rand_below(rng, m);
          std::vector<const Nat*> bp, ep, mp;
          std::vector<Nat*> op;
          for (auto& x : b) bp.push_back(&x);
          for (auto& x : e) ep.push_back(&x);
          for (auto& x : mul) mp.push_back(&x);
          for (auto& x : out) op.push_back(&x);
          eng.exp_into(m, n, bp.data(), ep.data(), ep.size(), with_mul ? mp.data() : nullptr, op.data());
          for (size_t i = 0; i < n; ++i) {
            std::vector<uint32_t> w(m.words());
            const Nat& ei = e[shared ? 0 : i];
            for (size_t j = 0; j < w.size(); ++j)
              w[j] = w_at(b[i], j) ^ w_at(ei, j) ^ (with_mul ? w_at(mul[i], j) : (j == 0 ? 1u : 0u));
            if (Nat::from_words(w.data(), w.size()) != out[i]) bad++;
            checked++;
          }
        }
        ops += n;
      }
    });
  for (auto& x : th) x.join();
  uint64_t held = 0, peak = 0, fb = 0, fbb = 0;
  pinned_pool_stats(&held, &peak, &fb, &fbb);
  std::printf("engine_stress: threads %d iters %d outputs %llu bad %llu launches %llu pin_refusals %llu "
              "fallbacks %llu pool_held %llu\n",
              threads, iters, (unsigned long long)checked.load(), (unsigned long long)bad.load(),
              (unsigned long long)mock_launches(), (unsigned long long)mock_pin_refusals(), (unsigned long long)fb,
              (unsigned long long)held);
  if (bad.load() || fb == 0) {
    std::printf("engine_stress: FAIL (%s)\n", bad.load() ? "wrong outputs" : "no pageable fallback exercised");
    return 1;
  }
  std::printf("engine_stress: OK\n");
  return 0;
}
