// engine.hpp -- C++ host mirror of the reference's modexp-calling surfaces,
// layered on the libmpcx.so C-ABI (include/mpcx.h). This is the code a Go
// integration would put in its cgo package; Go is absent
// from this image, so the mirror is C++ (compiled reference -> compiled host).
#pragma once

#include <atomic>
#include <cstdint>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "bignum.hpp"
#include "mpcx.h"

namespace mpcx::host {

// Launch coalescing (engine.cpp Coalescer): at most kCoalesceInflight merged
// dispatches per bound GPU in flight (environment MPCX_COALESCE overrides;
// 0 turns coalescing off), each at most kCoalesceMaxOps operands; a call of
// kCoalesceAloneOps operands or more launches on its own.
constexpr int kCoalesceInflight = 3;
constexpr uint64_t kCoalesceMaxOps = 131072;
constexpr size_t kCoalesceAloneOps = 16384;  // wider calls launch on their own

class EngineError : public std::runtime_error {
 public:
  EngineError(int code, const std::string& msg) : std::runtime_error(msg), code(code) {}
  int code;
};

// Process-wide handle on the node's GPUs (libmpcx spreads every batch over
// the bound devices) plus a cache of registered moduli: a node's N^2, N, N~
// are registered once and reused by every session, exactly like mpcium
// reuses its preparams (/root/reference/pkg/mpc/node.go:69,109,170).
class Engine {
 public:
  static Engine& get();
  void init(int device);         // bind one more GPU
  void init_devices(int n_gpus);  // bind GPUs 0..n_gpus-1 (<= 0: all visible)
  bool initialized() const { return bound_; }
  // Longest exponent the fixed-base comb path takes: every honest protocol
  // exponent on h1, h2, s, t (MtA s2/t2 ~2.8 kbit, FacProof sigma/v ~4.9 kbit)
  // fits; a longer (peer-supplied) exponent runs on the per-operand path, so
  // one adversarial proof can neither force a huge table build nor fail the
  // whole batch.
  static constexpr uint32_t kFixedMaxBits = 5120;
  static constexpr size_t kFixedMaxBases = 2;  // tables per comb launch (mpcx_fixedbase_exp_batch)

  // out[i] = (muls ? muls[i] : 1) * bases[i]^e_i mod m, m odd, 1 <= m < 2^4096.
  // exps.size() == 1: shared exponent; else one per base. Bases of any size
  // (reduced mod m on the host first when wider than the kernel class).
  std::vector<Nat> exp(const Nat& m, const std::vector<Nat>& bases, const std::vector<Nat>& exps,
                       const std::vector<Nat>* muls = nullptr);
  // The same over pointer arrays, results written through outs (no copies of
  // the operands): n bases, n_exps == 1 (shared) or n exponents, muls null or
  // n entries (a null entry: 1), n outputs.
  void exp_into(const Nat& m, size_t n, const Nat* const* bases, const Nat* const* exps, size_t n_exps,
                const Nat* const* muls, Nat* const* outs);
  std::vector<Nat> mulmod(const Nat& m, const std::vector<Nat>& a, const std::vector<Nat>& b);
  // out[i] = (muls ? muls[i] : 1) * base^exps[i] mod m through a comb table of
  // `base` (mpcx_fixedbase_*), built on first use and cached: the bases that
  // recur across every session (h1, h2 of a node's N~) pay for it once.
  std::vector<Nat> fixed_exp(const Nat& m, const Nat& base, const std::vector<Nat>& exps,
                             const std::vector<Nat>* muls = nullptr);
  void fixed_exp_into(const Nat& m, const Nat& base, size_t n, const Nat* const* exps, const Nat* const* muls,
                      Nat* const* outs);
  // out[i] = (muls ? muls[i] : 1) * prod_t bases[t]^exps[t][i] mod m for nb <= 2
  // recurring bases, one comb launch (each base's table cached as above)
  void fixed_multi_into(const Nat& m, size_t nb, const Nat* const* bases, size_t n, const Nat* const* const* exps,
                        const Nat* const* muls, Nat* const* outs);
  // fixed-base path usable for m (odd, <= 2080 bits) and enabled
  // (environment MPCX_FIXED_BASE=0 turns it off, for A/B runs)
  bool fixed_base_ok(const Nat& m) const;
  // wall-clock seconds during which at least one libmpcx exponentiation call
  // (GPU + transfers) was in flight, since the last reset. Calls from
  // different threads run concurrently on libmpcx's lanes (streams).
  double busy_seconds() const { return (double)busy_ns_.load() * 1e-9; }
  // the same, including a busy interval still open now
  double busy_seconds_now();
  // Go-equivalent algorithmic work of the exponentiations sent to libmpcx
  // since the last reset: SURVEY.md 8(d) W = (E + ceil(E/4)) 2 L^2 32-bit
  // MACs per x^e mod m (E = bit length of e, L = 32-bit words of m), the
  // work Go's 4-bit-window expNNMontgomery does for it, whatever window,
  // comb table or geometry the GPU uses. Algebraic shortcuts the host takes
  // instead of an exponentiation (Gamma^m = 1 + mN, CRT halves) count only
  // what is actually launched.
  double alg_macs() const { return (double)alg_macs_.load(); }
  void reset_busy() {
    busy_ns_ = 0;
    alg_macs_ = 0;
  }
  // execution lanes per device libmpcx uses from now on (mpcx_set_option "lanes");
  // returns the previous count. Many small independent proof chains (config-5
  // keygen load) gain from 8; signing's latency-bound chains run best on 6.
  int set_lanes(int n);
  std::vector<uint8_t> fermat2(const std::vector<Nat>& cands);
  // mpcx_safeprime_step: sieve + Pocklington over `count` stream candidates
  // (raw bytes, or the CounterDRBG(seed) stream from byte stream_off), plus
  // the base-2 strong test on sprp_q riding along in the same launch
  struct StepOut {
    uint32_t sieved = 0;           // sieve survivors = Pocklington tests
    std::vector<uint32_t> idx;     // Fermat passes: candidate index within the step (ascending)
    std::vector<Nat> p;            //                 and their p = 2q + 1
    std::vector<uint8_t> sprp;     // verdicts for sprp_q
  };
  StepOut safeprime_step(uint64_t seed, const uint8_t* raw, uint64_t stream_off, uint32_t count, uint32_t q_bits,
                         const std::vector<Nat>& sprp_q);
  std::vector<uint8_t> strong_probable_prime(const std::vector<Nat>& n, const std::vector<Nat>& bases);
  // mpcx_lucas_batch: strong Lucas test with parameters P (n < 2^2048)
  std::vector<uint8_t> lucas(const std::vector<Nat>& n, const std::vector<uint32_t>& P);

 private:
  struct Mod {
    mpcx_mod_t h;
    uint32_t class_words;
    uint32_t words;
  };
  Mod& modulus(const Nat& m);
  // A comb table; released when the last user drops it (another thread may
  // grow or evict the cache entry while a batch still uses the table).
  struct FixedTable {
    mpcx_fb_t h = nullptr;
    uint32_t max_bits = 0;
    size_t bytes = 0;  // device footprint (mpcx_fixedbase_info)
    ~FixedTable() {
      if (h) mpcx_fixedbase_release(h);
    }
  };
  using Fixed = std::shared_ptr<FixedTable>;
  Fixed fixed(const Nat& m, const Nat& base, uint32_t need_bits);
  // busy-time accounting: union of in-flight intervals
  void enter_call();
  void leave_call();
  std::mutex mu_, busy_mu_;
  int inflight_ = 0;
  std::chrono::steady_clock::time_point busy_t0_;
  bool bound_ = false;
  bool fixed_enabled_ = true;
  std::atomic<uint64_t> busy_ns_{0};
  std::atomic<uint64_t> alg_macs_{0};
  std::atomic<int> lanes_{0};  // 0: libmpcx's default (MPCX_LANES or 6)
  void count_work(const Nat& m, const Nat* const* exps, size_t n_exps, size_t count);
  std::map<std::vector<uint32_t>, Mod> mods_;
  std::map<std::pair<std::vector<uint32_t>, std::vector<uint32_t>>, Fixed> fixed_;
  size_t fixed_bytes_ = 0;                                  // device bytes of the cached tables
  static constexpr size_t kFixedMaxBytes = size_t(24) << 30;  // of the 288 GB per GPU
};

[[noreturn]] void throw_last(int rc, const char* what);

// Engine's page-locked staging pool: bytes held (in use + cached), peak bytes
// in use, and the pageable fallbacks taken when pinning failed (count, bytes).
void pinned_pool_stats(uint64_t* held_bytes, uint64_t* peak_in_use_bytes, uint64_t* fallbacks,
                       uint64_t* fallback_bytes);

}  // namespace mpcx::host
