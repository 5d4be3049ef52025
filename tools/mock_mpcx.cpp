// CPU stand-in for libmpcx.so (test infrastructure, never shipped): the subset
// of include/mpcx.h that libmpcx_host's Engine calls, with the host-memory
// behaviour of the real library and a cheap, checkable "result" instead of
// the exponentiation. Linked only into tools/engine_stress.cpp, under ASAN or
// TSAN, so that the Engine's coalescers, pinned pool, table cache and error
// paths run on many threads without a GPU:
//   - every input byte of every group is read, and every output byte written,
//     after a random delay (the real copies run while other callers queue);
//   - a host range that starts inside an mpcx_host_alloc block must end inside
//     it (the real library's registry check) or the process aborts;
//   - mpcx_host_alloc fails at random (MOCK_PIN_FAIL per mille) and on each
//     thread's first two calls, forcing the Engine's pageable fallback;
//   - fixed-base tables are heap objects whose contents every launch reads
//     (a launch on a released table is a use-after-free ASAN reports), and
//     report 2 GB each so the Engine's 24 GB cache evicts under load.
// Result function (word-wise, out_words words): modexp  out = base ^ exp ^ mul;
// fixed-base out = (XOR_t exp_t) ^ mul ^ (XOR_t table tag), tag = base word 0
// ^ modulus word 0 in word 0 (mul absent: 1).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "mpcx.h"

struct mpcx_modulus_s {
  std::vector<uint32_t> m;
  uint32_t class_words;
};
struct mpcx_fixedbase_s {
  mpcx_mod_t mod;
  uint32_t max_bits;
  std::vector<uint32_t> table;  // table[0] = tag; the rest is read by launches
};

namespace {
thread_local std::string t_err;
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pins;
std::atomic<uint64_t> g_launches{0}, g_fallbacks{0};

int fail(int code, const char* msg) {
  t_err = msg;
  return code;
}
uint32_t rnd(uint32_t n) {
  thread_local std::mt19937 rng(std::random_device{}());
  return n ? rng() % n : 0;
}
void jitter() { std::this_thread::sleep_for(std::chrono::microseconds(rnd(300))); }

// the real library's pinned-range rule; reads the whole range
void read_range(const void* p, size_t bytes, std::vector<uint32_t>& dst) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.upper_bound((uintptr_t)p);
    if (it != g_pins.begin()) {
      --it;
      if ((uintptr_t)p < it->first + it->second && (uintptr_t)p + bytes > it->first + it->second) {
        std::fprintf(stderr, "mock: range %p+%zu overruns its pinned block\n", p, bytes);
        std::abort();
      }
    }
  }
  dst.resize(bytes / 4);
  if (bytes) std::memcpy(dst.data(), p, bytes);
}
uint32_t word(const std::vector<uint32_t>& v, size_t i) { return i < v.size() ? v[i] : 0u; }
uint32_t class_words_of(size_t words) { return words <= 32 ? 32 : words <= 65 ? 65 : 128; }
}  // namespace

extern "C" {
const char* mpcx_last_error(void) { return t_err.c_str(); }
int mpcx_init(int) { return MPCX_OK; }
int mpcx_init_devices(int) { return MPCX_OK; }
int mpcx_bound_devices(int* n, int* ords, int max) {
  if (n) *n = 1;
  if (ords && max > 0) ords[0] = 0;
  return MPCX_OK;
}
int mpcx_set_option(const char*, int) { return MPCX_OK; }
int mpcx_modulus_register(const uint32_t* m, uint32_t len, mpcx_mod_t* out) {
  auto* md = new mpcx_modulus_s();
  md->m.assign(m, m + len);
  md->class_words = class_words_of(len);
  *out = md;
  return MPCX_OK;
}
int mpcx_modulus_info(mpcx_mod_t mod, uint32_t* bits, uint32_t* cw) {
  if (bits) *bits = 32 * (uint32_t)mod->m.size();
  if (cw) *cw = mod->class_words;
  return MPCX_OK;
}
int mpcx_host_alloc(size_t bytes, void** out) {
  static const int fail_pm = [] {
    const char* e = std::getenv("MOCK_PIN_FAIL");
    return e ? std::atoi(e) : 100;
  }();
  // each thread's first two calls are refused too: the Engine's release-and-retry
  // then fails as well, so every run takes the pageable fallback at least once
  thread_local int t_calls = 0;
  if (++t_calls <= 2 || (int)rnd(1000) < fail_pm) {
    g_fallbacks++;
    return fail(MPCX_ENOMEM, "mock: pinned allocation refused");
  }
  void* p = std::malloc(bytes);
  if (!p) return fail(MPCX_ENOMEM, "mock: malloc");
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pins[(uintptr_t)p] = bytes;
  *out = p;
  return MPCX_OK;
}
int mpcx_host_free(void* p) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pins.erase((uintptr_t)p);
  }
  std::free(p);
  return MPCX_OK;
}
int mpcx_fixedbase_register(mpcx_mod_t mod, const uint32_t* base, uint32_t base_words, uint32_t max_bits,
                            mpcx_fb_t* out) {
  jitter();
  auto* fb = new mpcx_fixedbase_s();
  fb->mod = mod;
  fb->max_bits = max_bits;
  fb->table.assign(256, 0);
  fb->table[0] = (base_words ? base[0] : 0) ^ mod->m[0];
  *out = fb;
  return MPCX_OK;
}
int mpcx_fixedbase_release(mpcx_fb_t fb) {
  delete fb;
  return MPCX_OK;
}
int mpcx_fixedbase_info(mpcx_fb_t fb, uint32_t* max_bits, size_t* bytes) {
  if (max_bits) *max_bits = fb->max_bits;
  if (bytes) *bytes = size_t(2) << 30;
  return MPCX_OK;
}

int mpcx_modexp_multi_batch(uint32_t n, const mpcx_modexp_group_t* gs) {
  struct In {
    std::vector<uint32_t> b, e, m;
  };
  std::vector<In> in(n);
  for (uint32_t i = 0; i < n; ++i) {
    const auto& g = gs[i];
    read_range(g.bases, (size_t)g.count * g.base_words * 4, in[i].b);
    read_range(g.exps, (g.exp_shared ? 1 : (size_t)g.count) * g.exp_words * 4, in[i].e);
    if (g.muls) read_range(g.muls, (size_t)g.count * g.mul_words * 4, in[i].m);
  }
  jitter();
  for (uint32_t i = 0; i < n; ++i) {
    const auto& g = gs[i];
    std::vector<uint32_t> out((size_t)g.count * g.out_words);
    for (uint32_t k = 0; k < g.count; ++k)
      for (uint32_t j = 0; j < g.out_words; ++j) {
        uint32_t v = j < g.base_words ? in[i].b[(size_t)k * g.base_words + j] : 0u;
        const size_t eo = g.exp_shared ? 0 : (size_t)k * g.exp_words;
        if (j < g.exp_words) v ^= in[i].e[eo + j];
        if (g.muls) {
          if (j < g.mul_words) v ^= in[i].m[(size_t)k * g.mul_words + j];
        } else if (j == 0) {
          v ^= 1u;
        }
        out[(size_t)k * g.out_words + j] = v;
      }
    std::memcpy(g.out, out.data(), out.size() * 4);
  }
  g_launches++;
  return MPCX_OK;
}
int mpcx_modexp_batch(mpcx_mod_t mod, uint32_t count, const uint32_t* bases, uint32_t bw, const uint32_t* exps,
                      uint32_t ew, int shared, uint32_t* out, uint32_t ow) {
  mpcx_modexp_group_t g{mod, count, bases, bw, exps, ew, shared, nullptr, 0, out, ow};
  return mpcx_modexp_multi_batch(1, &g);
}
int mpcx_modexp_mul_batch(mpcx_mod_t mod, uint32_t count, const uint32_t* bases, uint32_t bw, const uint32_t* exps,
                          uint32_t ew, int shared, const uint32_t* muls, uint32_t mw, uint32_t* out, uint32_t ow) {
  mpcx_modexp_group_t g{mod, count, bases, bw, exps, ew, shared, muls, mw, out, ow};
  return mpcx_modexp_multi_batch(1, &g);
}

int mpcx_fixedbase_multi_batch(uint32_t n, const mpcx_fixedbase_group_t* gs) {
  struct In {
    std::vector<uint32_t> e[MPCX_FB_MAX_BASES], m;
    uint32_t tag = 0;
  };
  std::vector<In> in(n);
  for (uint32_t i = 0; i < n; ++i) {
    const auto& g = gs[i];
    for (uint32_t t = 0; t < g.nbases; ++t) {
      read_range(g.exps[t], (size_t)g.count * g.exp_words[t] * 4, in[i].e[t]);
      uint64_t s = 0;  // every launch reads its tables
      for (uint32_t v : g.fbs[t]->table) s += v;
      (void)s;
      in[i].tag ^= g.fbs[t]->table[0];
    }
    if (g.muls) read_range(g.muls, (size_t)g.count * g.mul_words * 4, in[i].m);
  }
  jitter();
  for (uint32_t i = 0; i < n; ++i) {
    const auto& g = gs[i];
    std::vector<uint32_t> out((size_t)g.count * g.out_words);
    for (uint32_t k = 0; k < g.count; ++k)
      for (uint32_t j = 0; j < g.out_words; ++j) {
        uint32_t v = j == 0 ? in[i].tag : 0u;
        for (uint32_t t = 0; t < g.nbases; ++t)
          if (j < g.exp_words[t]) v ^= in[i].e[t][(size_t)k * g.exp_words[t] + j];
        if (g.muls) {
          if (j < g.mul_words) v ^= in[i].m[(size_t)k * g.mul_words + j];
        } else if (j == 0) {
          v ^= 1u;
        }
        out[(size_t)k * g.out_words + j] = v;
      }
    std::memcpy(g.out, out.data(), out.size() * 4);
  }
  g_launches++;
  return MPCX_OK;
}
int mpcx_fixedbase_exp_batch(uint32_t nb, const mpcx_fb_t* fbs, uint32_t count, const uint32_t* const* exps,
                             const uint32_t* ew, const uint32_t* muls, uint32_t mw, uint32_t* out, uint32_t ow) {
  mpcx_fixedbase_group_t g{};
  g.nbases = nb;
  g.count = count;
  for (uint32_t t = 0; t < nb; ++t) {
    g.fbs[t] = fbs[t];
    g.exps[t] = exps[t];
    g.exp_words[t] = ew[t];
  }
  g.muls = muls;
  g.mul_words = mw;
  g.out = out;
  g.out_words = ow;
  return mpcx_fixedbase_multi_batch(1, &g);
}
// not exercised by the stress; present so the Engine links
int mpcx_fermat2_batch(uint32_t, const uint32_t*, uint32_t, uint8_t*) { return fail(MPCX_ENODEV, "mock"); }
int mpcx_mr_batch(uint32_t, const uint32_t*, uint32_t, const uint32_t*, uint8_t*) { return fail(MPCX_ENODEV, "mock"); }
int mpcx_lucas_batch(uint32_t, const uint32_t*, uint32_t, const uint32_t*, uint8_t*) {
  return fail(MPCX_ENODEV, "mock");
}
int mpcx_safeprime_step(uint64_t, const uint8_t*, uint64_t, uint32_t, uint32_t, const uint32_t*, uint32_t, uint32_t,
                        uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint8_t*) {
  return fail(MPCX_ENODEV, "mock");
}
uint64_t mock_launches() { return g_launches.load(); }
uint64_t mock_pin_refusals() { return g_fallbacks.load(); }
}
