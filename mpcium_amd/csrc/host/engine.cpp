// engine.cpp -- see engine.hpp.
#include "engine.hpp"

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <malloc.h>
#include <string>

#include "hostprof.hpp"
#include "tsscommon.hpp"

#include <algorithm>
#include <functional>
#include <chrono>
#include <cstdlib>

namespace mpcx::host {

void throw_last(int rc, const char* what) {
  throw EngineError(rc, std::string(what) + ": " + mpcx_last_error());
}

Engine& Engine::get() {
  // never destroyed: releasing device tables from a static destructor could
  // run after the HIP runtime has been torn down at process exit
  static Engine* e = new Engine();
  return *e;
}

// The protocol mirrors allocate and free millions of small bignums per second
// from many threads. glibc's per-thread arenas then grow (mprotect) and trim
// their heaps back on nearly every batch: an eighth of a signing run's CPU
// (profiles/r03/sample1). A high trim threshold and top pad keep the arenas'
// heaps mapped instead (MPCX_MALLOC_TUNE=0: glibc defaults, for A/B runs).
static void tune_malloc() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("MPCX_MALLOC_TUNE");
    if (e && e[0] == '0') return;
    mallopt(M_TRIM_THRESHOLD, 512 << 20);
    mallopt(M_TOP_PAD, 8 << 20);
  });
}

void Engine::init(int device) {
  tune_malloc();
  std::lock_guard<std::mutex> lk(mu_);
  int rc = mpcx_init(device);
  if (rc) throw_last(rc, "mpcx_init");
  bound_ = true;
  const char* fb = std::getenv("MPCX_FIXED_BASE");
  fixed_enabled_ = !(fb && fb[0] == '0');
}

void Engine::init_devices(int n_gpus) {
  tune_malloc();
  std::lock_guard<std::mutex> lk(mu_);
  int rc = mpcx_init_devices(n_gpus);
  if (rc) throw_last(rc, "mpcx_init_devices");
  bound_ = true;
  const char* fb = std::getenv("MPCX_FIXED_BASE");
  fixed_enabled_ = !(fb && fb[0] == '0');
}

void Engine::enter_call() {
  std::lock_guard<std::mutex> lk(busy_mu_);
  if (inflight_++ == 0) busy_t0_ = std::chrono::steady_clock::now();
}

void Engine::leave_call() {
  std::lock_guard<std::mutex> lk(busy_mu_);
  if (--inflight_ == 0)
    busy_ns_ += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                               busy_t0_).count();
}

double Engine::busy_seconds_now() {
  std::lock_guard<std::mutex> lk(busy_mu_);
  uint64_t ns = busy_ns_;
  if (inflight_ > 0)
    ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - busy_t0_)
              .count();
  return (double)ns * 1e-9;
}

void Engine::count_work(const Nat& m, const Nat* const* exps, size_t n_exps, size_t count) {
  const uint64_t L = m.words(), l2 = 2 * L * L;
  uint64_t w = 0;
  auto one = [&](const Nat& e) {
    const uint64_t E = e.bit_len();
    return (E + (E + 3) / 4) * l2;
  };
  if (n_exps == 1 && count != 1) {
    w = one(*exps[0]) * count;
  } else {
    for (size_t i = 0; i < n_exps; ++i) w += one(*exps[i]);
  }
  alg_macs_ += w;
}

Engine::Mod& Engine::modulus(const Nat& m) {
  auto it = mods_.find(m.limbs());
  if (it != mods_.end()) return it->second;
  Mod md{};
  int rc = mpcx_modulus_register(m.limbs().data(), (uint32_t)m.words(), &md.h);
  if (rc) throw_last(rc, "mpcx_modulus_register");
  uint32_t bits = 0;
  mpcx_modulus_info(md.h, &bits, &md.class_words);
  md.words = (uint32_t)m.words();
  return mods_.emplace(m.limbs(), md).first->second;
}

// fn(lo, hi) over [0, n) in chunks of 2048 on the host pool (packing and
// unpacking a 40K-operand batch serially sat on its task's critical path)
static void par_chunks(size_t n, const std::function<void(size_t, size_t)>& fn) {
  constexpr size_t kChunk = 2048;
  if (n <= kChunk) {
    fn(0, n);
    return;
  }
  parallel_for((n + kChunk - 1) / kChunk, [&](size_t c) { fn(c * kChunk, std::min(n, (c + 1) * kChunk)); });
}

namespace {
// Pool of page-locked host buffers (mpcx_host_alloc) for the batches' inputs
// and outputs: libmpcx DMAs them directly (anything else it bounces through
// its lanes' own pinned buffers with a CPU copy). Buffers are reused across
// calls (size classes of powers of two); free buffers beyond cache_max() bytes
// are returned to the system. A failed pinned allocation first releases every
// cached free buffer and retries; only then does the batch fall back to a
// pageable buffer -- counted, and logged to stderr (the first 8 times, then
// every 1000th), never silent.
class PinnedPool {
 public:
  // free pinned bytes kept for reuse: MPCX_PINNED_CACHE_MB, else 8 GB shared by
  // the node's local ranks (LOCAL_WORLD_SIZE under torchrun), at least 1 GB
  static size_t cache_max() {
    static const size_t v = [] {
      if (const char* e = std::getenv("MPCX_PINNED_CACHE_MB")) return (size_t)std::max(0L, std::atol(e)) << 20;
      long ranks = 1;
      if (const char* w = std::getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1L, std::atol(w));
      return std::max((size_t)1 << 30, ((size_t)8 << 30) / (size_t)ranks);
    }();
    return v;
  }
  static PinnedPool& get() {
    static PinnedPool p;
    return p;
  }
  uint32_t* acquire(size_t words) {
    size_t cls = 1u << 16;  // 256 KB minimum
    while (cls < words) cls <<= 1;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto& fl = free_[cls];
      if (!fl.empty()) {
        uint32_t* p = fl.back();
        fl.pop_back();
        cached_bytes_ -= cls * 4;
        note_use(cls * 4);
        return p;
      }
    }
    void* p = nullptr;
    if (mpcx_host_alloc(cls * 4, &p) != MPCX_OK) {
      release_cached();
      if (mpcx_host_alloc(cls * 4, &p) != MPCX_OK) return nullptr;
    }
    std::lock_guard<std::mutex> lk(mu_);
    size_of_[(uint32_t*)p] = cls;
    held_bytes_ += cls * 4;
    note_use(cls * 4);
    return (uint32_t*)p;
  }
  void release(uint32_t* p) {
    if (!p) return;
    std::unique_lock<std::mutex> lk(mu_);
    const size_t cls = size_of_.at(p);
    in_use_bytes_ -= cls * 4;
    if (cached_bytes_ + cls * 4 > cache_max()) {
      size_of_.erase(p);
      held_bytes_ -= cls * 4;
      lk.unlock();
      mpcx_host_free(p);
      return;
    }
    free_[cls].push_back(p);
    cached_bytes_ += cls * 4;
  }
  void note_fallback(size_t words) {
    const uint64_t k = fallbacks_.fetch_add(1) + 1;
    fallback_bytes_ += words * 4;
    if (k <= 8 || k % 1000 == 0)
      std::fprintf(stderr, "[mpcx engine] pinned host allocation of %zu B failed (%s): pageable buffer #%llu\n",
                   words * 4, mpcx_last_error(), (unsigned long long)k);
  }
  void stats(uint64_t* held, uint64_t* peak_in_use, uint64_t* fallbacks, uint64_t* fallback_bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    if (held) *held = held_bytes_;
    if (peak_in_use) *peak_in_use = peak_in_use_;
    if (fallbacks) *fallbacks = fallbacks_.load();
    if (fallback_bytes) *fallback_bytes = fallback_bytes_.load();
  }

 private:
  void note_use(size_t bytes) {  // mu_ held
    in_use_bytes_ += bytes;
    peak_in_use_ = std::max(peak_in_use_, in_use_bytes_);
  }
  void release_cached() {
    std::vector<uint32_t*> drop;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& [cls, fl] : free_) {
        for (uint32_t* p : fl) {
          drop.push_back(p);
          size_of_.erase(p);
          held_bytes_ -= cls * 4;
        }
        fl.clear();
      }
      cached_bytes_ = 0;
    }
    for (uint32_t* p : drop) mpcx_host_free(p);
  }
  std::mutex mu_;
  std::map<size_t, std::vector<uint32_t*>> free_;
  std::map<uint32_t*, size_t> size_of_;
  size_t held_bytes_ = 0, cached_bytes_ = 0, in_use_bytes_ = 0, peak_in_use_ = 0;
  std::atomic<uint64_t> fallbacks_{0}, fallback_bytes_{0};
};

// a pinned buffer of `words` words (a counted, logged pageable fallback if
// pinning fails: libmpcx then bounces it, so the batch stays correct)
struct HostBuf {
  uint32_t* p = nullptr;
  std::vector<uint32_t> fallback;
  bool pinned = false;
  explicit HostBuf(size_t words) {
    static const bool off = [] {  // MPCX_PINNED=0: pageable staging (A/B runs)
      const char* e = std::getenv("MPCX_PINNED");
      return e && e[0] == '0';
    }();
    p = off ? nullptr : PinnedPool::get().acquire(words);
    if (!p) {
      if (!off) PinnedPool::get().note_fallback(words);
      fallback.resize(words);
      p = fallback.data();
    } else {
      pinned = true;
    }
  }
  ~HostBuf() {
    if (pinned) PinnedPool::get().release(p);
  }
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
};
}  // namespace

void pinned_pool_stats(uint64_t* held_bytes, uint64_t* peak_in_use_bytes, uint64_t* fallbacks,
                       uint64_t* fallback_bytes) {
  PinnedPool::get().stats(held_bytes, peak_in_use_bytes, fallbacks, fallback_bytes);
}

namespace {
// Launch coalescing across concurrent callers (ExpSets of different signer
// pairs, wallet pipelines and moduli): each exp() call is a group; a caller
// that finds fewer than max_inflight dispatches running becomes the leader
// and issues every pending group of its modulus class as ONE
// mpcx_modexp_multi_batch launch; the others wait for their results. Under
// load the GPU thus receives few large launches (the main geometry's
// throughput) instead of many narrow ones; alone, a call dispatches at once.
template <class Group, int (*Launch)(uint32_t, const Group*)>
class CoalescerT {
 public:
  struct Req {
    Group g{};
    bool taken = false, done = false;
    int rc = MPCX_OK;
    std::string err;
  };
  // min_ops > 0: while another dispatch of this coalescer is in flight, a
  // leader waits until the queue holds min_ops operands (a finishing dispatch
  // or a new arrival wakes it; with nothing in flight it always launches)
  int run(Req& r, int max_inflight, uint64_t max_ops, uint64_t min_ops = 0) {
    std::unique_lock<std::mutex> lk(mu_);
    q_.push_back(&r);
    queued_ += r.g.count;
    if (min_ops) cv_.notify_all();
    while (!r.done) {
      if (!r.taken && inflight_ < max_inflight && (inflight_ == 0 || queued_ >= min_ops)) {
        std::vector<Req*> batch{&r};  // the leader's own group first, then arrival order
        r.taken = true;
        uint64_t ops = r.g.count;
        queued_ -= r.g.count;
        for (auto it = q_.begin(); it != q_.end();) {
          if (*it == &r) {
            it = q_.erase(it);
          } else if (!(*it)->taken && ops + (*it)->g.count <= max_ops) {
            ops += (*it)->g.count;
            queued_ -= (*it)->g.count;
            (*it)->taken = true;
            batch.push_back(*it);
            it = q_.erase(it);
          } else {
            ++it;
          }
        }
        ++inflight_;
        lk.unlock();
        // whatever happens in the launch, every member of the batch gets an
        // rc and done, and inflight_ drops again (a throw here would
        // otherwise leave the followers waiting forever)
        int rc = MPCX_OK;
        std::string err;
        try {
          std::vector<Group> gs;
          gs.reserve(batch.size());
          for (Req* b : batch) gs.push_back(b->g);
          rc = Launch((uint32_t)gs.size(), gs.data());
          if (rc) err = mpcx_last_error();
        } catch (const std::bad_alloc&) {
          rc = MPCX_ENOMEM;
          err = "host allocation failed in a coalesced launch";
        } catch (const std::exception& ex) {
          rc = MPCX_EHIP;
          err = std::string("coalesced launch: ") + ex.what();
        }
        lk.lock();
        --inflight_;
        for (Req* b : batch) {
          b->rc = rc;
          b->err = err;
          b->done = true;
        }
        cv_.notify_all();
      } else {
        cv_.wait(lk);
      }
    }
    return r.rc;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Req*> q_;
  uint64_t queued_ = 0;  // operands of the groups in q_ not yet taken
  int inflight_ = 0;
};

using Coalescer = CoalescerT<mpcx_modexp_group_t, mpcx_modexp_multi_batch>;
// comb launches: concurrent fixed-base batches (h1, h2 of every peer's N~ in
// every wallet pipeline, proof chain) as the segments of one k_fixedbase_multi
using FixedCoalescer = CoalescerT<mpcx_fixedbase_group_t, mpcx_fixedbase_multi_batch>;

Coalescer& coalescer(uint32_t class_words) {
  static Coalescer c[3];
  return c[class_words <= 32 ? 0 : class_words <= 65 ? 1 : 2];
}
FixedCoalescer& fixed_coalescer(uint32_t class_words) {
  static FixedCoalescer c[2];
  return c[class_words <= 32 ? 0 : 1];
}

// MPCX_COALESCE = max coalesced dispatches in flight per bound device (0: off,
// each exp() call is its own launch); default kCoalesceInflight
// MPCX_COALESCE_MAXOPS: operands per merged launch (A/B runs); default kCoalesceMaxOps
uint64_t coalesce_max_ops() {
  static const uint64_t v = [] {
    const char* e = std::getenv("MPCX_COALESCE_MAXOPS");
    const long long x = e ? std::atoll(e) : 0;
    return x > 0 ? (uint64_t)x : kCoalesceMaxOps;
  }();
  return v;
}

// MPCX_COALESCE_MIN_OPS: queued operands a modexp leader waits for while a
// dispatch is in flight (0, the default: launch whenever the in-flight budget
// allows)
uint64_t coalesce_min_ops() {
  static const uint64_t v = [] {
    const char* e = std::getenv("MPCX_COALESCE_MIN_OPS");
    const long long x = e ? std::atoll(e) : 0;
    return x > 0 ? (uint64_t)x : (uint64_t)0;
  }();
  return v;
}

int coalesce_inflight() {
  static const int v = [] {
    const char* e = std::getenv("MPCX_COALESCE");
    return e ? std::atoi(e) : kCoalesceInflight;
  }();
  if (v <= 0) return 0;
  int dev = 1;  // per bound device
  if (mpcx_bound_devices(&dev, nullptr, 0) != MPCX_OK || dev < 1) dev = 1;
  return v * dev;
}
}  // namespace

static void pack_into(const std::vector<Nat>& v, uint32_t w, uint32_t* out) {
  par_chunks(v.size(), [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) v[i].to_words(out + i * w, w);
  });
}

static void pack_ptrs(const Nat* const* v, size_t n, uint32_t w, uint32_t* out) {
  par_chunks(n, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) v[i]->to_words(out + i * w, w);
  });
}

static std::vector<uint32_t> pack(const std::vector<Nat>& v, uint32_t w) {
  std::vector<uint32_t> out((size_t)v.size() * w);
  pack_into(v, w, out.data());
  return out;
}

static void unpack_into(const uint32_t* buf, size_t count, uint32_t w, Nat* const* outs) {
  MPCX_PROF("engine.unpack");
  par_chunks(count, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) outs[i]->set_words(buf + i * w, w);
  });
}

template <class T>
static std::vector<const T*> ptrs(const std::vector<T>& v) {
  std::vector<const T*> p(v.size());
  for (size_t i = 0; i < v.size(); ++i) p[i] = &v[i];
  return p;
}

static std::vector<Nat*> out_ptrs(std::vector<Nat>& v) {
  std::vector<Nat*> p(v.size());
  for (size_t i = 0; i < v.size(); ++i) p[i] = &v[i];
  return p;
}

std::vector<Nat> Engine::exp(const Nat& m, const std::vector<Nat>& bases, const std::vector<Nat>& exps,
                             const std::vector<Nat>* muls) {
  if (exps.size() != 1 && exps.size() != bases.size()) throw std::invalid_argument("exps: 1 or one per base");
  if (muls && muls->size() != bases.size()) throw std::invalid_argument("muls: one per base");
  std::vector<Nat> out(bases.size());
  const auto bp = ptrs(bases), ep = ptrs(exps);
  std::vector<const Nat*> mp;
  if (muls) mp = ptrs(*muls);
  exp_into(m, bases.size(), bp.data(), ep.data(), ep.size(), muls ? mp.data() : nullptr, out_ptrs(out).data());
  return out;
}

void Engine::exp_into(const Nat& m, size_t n, const Nat* const* bases, const Nat* const* exps, size_t n_exps,
                      const Nat* const* muls, Nat* const* outs) {
  if (n_exps != 1 && n_exps != n) throw std::invalid_argument("exps: 1 or one per base");
  if (!n) return;
  Mod md;
  {
    std::lock_guard<std::mutex> lk(mu_);
    md = modulus(m);
  }
  // Host-side packing runs outside the lock, so another thread's batch can
  // use the GPU meanwhile. math/big reduces x mod m first when
  // len(x) > len(m) (nat.expNNMontgomery); here: only when x does not fit
  // the kernel class width. A null multiplier is 1.
  auto packed = [&](const Nat* const* v, uint32_t* out) {
    par_chunks(n, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        uint32_t* o = out + i * md.class_words;
        if (!v[i]) {
          std::fill(o, o + md.class_words, 0u);
          o[0] = 1;
        } else if (v[i]->words() > md.class_words) {
          (*v[i] % m).to_words(o, md.class_words);
        } else {
          v[i]->to_words(o, md.class_words);
        }
      }
    });
  };
  const bool shared = n_exps == 1;
  uint32_t ew = 1;
  for (size_t i = 0; i < n_exps; ++i) ew = std::max<uint32_t>(ew, (uint32_t)exps[i]->words());
  HostBuf B(n * md.class_words), E(n_exps * ew), M(muls ? n * md.class_words : 1), out(n * md.words);
  {
    MPCX_PROF("engine.exp.pack");
    packed(bases, B.p);
    pack_ptrs(exps, n_exps, ew, E.p);
    if (muls) packed(muls, M.p);
  }
  count_work(m, exps, n_exps, n);
  int rc;
  {
    MPCX_PROF("engine.exp.gpu");
    MPCX_TRACE(md.class_words <= 32 ? "gpu.exp1024" : md.class_words <= 65 ? "gpu.exp2048" : "gpu.exp4096", n);
    enter_call();
    const int inflight = coalesce_inflight();
    // a batch already wide enough to fill the GPU gains nothing from merging
    // (config-5's 128-iteration DLN batches): it launches alone, outside the
    // coalescer's in-flight budget
    if (inflight > 0 && n < kCoalesceAloneOps) {
      Coalescer::Req r;
      r.g.mod = md.h;
      r.g.count = (uint32_t)n;
      r.g.bases = B.p;
      r.g.base_words = md.class_words;
      r.g.exps = E.p;
      r.g.exp_words = ew;
      r.g.exp_shared = shared ? 1 : 0;
      r.g.muls = muls ? M.p : nullptr;
      r.g.mul_words = muls ? md.class_words : 0;
      r.g.out = out.p;
      r.g.out_words = md.words;
      rc = coalescer(md.class_words).run(r, inflight, coalesce_max_ops(), coalesce_min_ops());
      if (rc) {
        leave_call();
        throw EngineError(rc, "mpcx_modexp_multi_batch: " + r.err);
      }
    } else if (muls) {
      rc = mpcx_modexp_mul_batch(md.h, (uint32_t)n, B.p, md.class_words, E.p, ew, shared ? 1 : 0, M.p,
                                 md.class_words, out.p, md.words);
    } else {
      rc = mpcx_modexp_batch(md.h, (uint32_t)n, B.p, md.class_words, E.p, ew, shared ? 1 : 0, out.p, md.words);
    }
    leave_call();
  }
  if (rc) throw_last(rc, "mpcx_modexp_batch");
  unpack_into(out.p, n, md.words, outs);
}

bool Engine::fixed_base_ok(const Nat& m) const {
  return fixed_enabled_ && m.is_odd() && m.bit_len() <= 2080;
}

Engine::Fixed Engine::fixed(const Nat& m, const Nat& base, uint32_t need_bits) {
  auto key = std::make_pair(m.limbs(), base.limbs());
  auto it = fixed_.find(key);
  if (it != fixed_.end() && it->second->max_bits >= need_bits) return it->second;
  if (it != fixed_.end()) {  // grow: rebuild for the longer exponent
    fixed_bytes_ -= std::min(fixed_bytes_, it->second->bytes);
    fixed_.erase(it);
  }
  // bound the device footprint (~320 MB per 12-bit table): drop every cached
  // table past kFixedMaxBytes (handles in use keep theirs alive)
  if (fixed_bytes_ >= kFixedMaxBytes || fixed_.size() >= 256) {
    fixed_.clear();
    fixed_bytes_ = 0;
  }
  if (need_bits > kFixedMaxBits) throw std::invalid_argument("fixed-base exponent above kFixedMaxBits");
  Mod& md = modulus(m);
  // MtA exponents on h1, h2 reach ~2818 bits (s2, t2 < q^3 N~ + e q N~); one size serves them all
  const uint32_t bits = std::max<uint32_t>(3072, (need_bits + 511) / 512 * 512);
  auto f = std::make_shared<FixedTable>();
  std::vector<uint32_t> bw(md.class_words, 0);
  base.to_words(bw.data(), md.class_words);
  int rc = mpcx_fixedbase_register(md.h, bw.data(), md.class_words, bits, &f->h);
  if (rc) throw_last(rc, "mpcx_fixedbase_register");
  f->max_bits = bits;
  if (mpcx_fixedbase_info(f->h, nullptr, &f->bytes) == MPCX_OK) fixed_bytes_ += f->bytes;
  fixed_.emplace(key, f);
  return f;
}

std::vector<Nat> Engine::fixed_exp(const Nat& m, const Nat& base, const std::vector<Nat>& exps,
                                   const std::vector<Nat>* muls) {
  if (muls && muls->size() != exps.size()) throw std::invalid_argument("muls: one per exponent");
  std::vector<Nat> out(exps.size());
  const auto ep = ptrs(exps);
  std::vector<const Nat*> mp;
  if (muls) mp = ptrs(*muls);
  fixed_exp_into(m, base, exps.size(), ep.data(), muls ? mp.data() : nullptr, out_ptrs(out).data());
  return out;
}

void Engine::fixed_exp_into(const Nat& m, const Nat& base, size_t n, const Nat* const* exps, const Nat* const* muls,
                            Nat* const* outs) {
  const Nat* bases[1] = {&base};
  const Nat* const* ex[1] = {exps};
  fixed_multi_into(m, 1, bases, n, ex, muls, outs);
}

void Engine::fixed_multi_into(const Nat& m, size_t nb, const Nat* const* bases, size_t n,
                              const Nat* const* const* exps, const Nat* const* muls, Nat* const* outs) {
  if (nb == 0 || nb > kFixedMaxBases) throw std::invalid_argument("fixed_multi_into: 1 or 2 bases");
  if (!n) return;
  Mod md;
  {
    std::lock_guard<std::mutex> lk(mu_);
    md = modulus(m);
  }
  uint32_t ew[kFixedMaxBases] = {1, 1}, need[kFixedMaxBases] = {1, 1};
  for (size_t t = 0; t < nb; ++t)
    for (size_t i = 0; i < n; ++i) {
      ew[t] = std::max<uint32_t>(ew[t], (uint32_t)exps[t][i]->words());
      need[t] = std::max<uint32_t>(need[t], exps[t][i]->bit_len());
    }
  HostBuf E0(n * ew[0]), E1(nb > 1 ? n * ew[1] : 1), Mw(muls ? n * md.class_words : 1), out(n * md.words);
  pack_ptrs(exps[0], n, ew[0], E0.p);
  if (nb > 1) pack_ptrs(exps[1], n, ew[1], E1.p);
  if (muls) {
    par_chunks(n, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        uint32_t* o = Mw.p + i * md.class_words;
        const Nat* x = muls[i];
        if (!x) {
          std::fill(o, o + md.class_words, 0u);
          o[0] = 1;
        } else {
          (x->words() > md.class_words ? *x % m : *x).to_words(o, md.class_words);
        }
      }
    });
  }
  Fixed f[kFixedMaxBases];
  mpcx_fb_t h[kFixedMaxBases] = {nullptr, nullptr};
  for (size_t t = 0; t < nb; ++t) {
    const Nat& base = *bases[t];
    const Nat b = base.words() > md.class_words || base >= m ? base % m : base;
    // look up (or build) under the lock; the shared handle keeps the table
    // alive while this batch uses it, even if another thread evicts it
    std::lock_guard<std::mutex> lk(mu_);
    f[t] = fixed(m, b, need[t]);
    h[t] = f[t]->h;
  }
  const uint32_t* ep[kFixedMaxBases] = {E0.p, E1.p};
  for (size_t t = 0; t < nb; ++t) count_work(m, exps[t], n, n);
  int rc;
  {
    MPCX_PROF("engine.fixed.gpu");
    MPCX_TRACE("gpu.comb", n);
    enter_call();
    const int inflight = coalesce_inflight();
    if (inflight > 0 && n < kCoalesceAloneOps) {
      FixedCoalescer::Req r;
      r.g.nbases = (uint32_t)nb;
      r.g.count = (uint32_t)n;
      for (size_t t = 0; t < nb; ++t) {
        r.g.fbs[t] = h[t];
        r.g.exps[t] = ep[t];
        r.g.exp_words[t] = ew[t];
      }
      r.g.muls = muls ? Mw.p : nullptr;
      r.g.mul_words = muls ? md.class_words : 0;
      r.g.out = out.p;
      r.g.out_words = md.words;
      rc = fixed_coalescer(md.class_words).run(r, inflight, coalesce_max_ops());
      if (rc) {
        leave_call();
        throw EngineError(rc, "mpcx_fixedbase_multi_batch: " + r.err);
      }
    } else {
      rc = mpcx_fixedbase_exp_batch((uint32_t)nb, h, (uint32_t)n, ep, ew, muls ? Mw.p : nullptr,
                                    muls ? md.class_words : 0, out.p, md.words);
    }
    leave_call();
  }
  if (rc) throw_last(rc, "mpcx_fixedbase_exp_batch");
  unpack_into(out.p, n, md.words, outs);
}

int Engine::set_lanes(int n) {
  int prev = lanes_.exchange(n);
  if (prev == 0) {
    const char* e = std::getenv("MPCX_LANES");
    prev = e ? std::max(1, std::min(8, std::atoi(e))) : 6;
  }
  int rc = mpcx_set_option("lanes", n);
  if (rc) throw_last(rc, "mpcx_set_option(lanes)");
  return prev;
}

std::vector<Nat> Engine::mulmod(const Nat& m, const std::vector<Nat>& a, const std::vector<Nat>& b) {
  std::vector<Nat> one{Nat(1)};
  return exp(m, a, one, &b);
}

std::vector<uint8_t> Engine::fermat2(const std::vector<Nat>& cands) {
  if (cands.empty()) return {};
  uint32_t w = 1;
  for (const auto& c : cands) w = std::max<uint32_t>(w, (uint32_t)c.words());
  HostBuf P(cands.size() * w);  // pinned: DMA'd directly (MR / Lucas batches of ModProof verification are GBs)
  pack_into(cands, w, P.p);
  std::vector<uint8_t> ok(cands.size());
  int rc = mpcx_fermat2_batch((uint32_t)cands.size(), P.p, w, ok.data());
  if (rc) throw_last(rc, "mpcx_fermat2_batch");
  return ok;
}

Engine::StepOut Engine::safeprime_step(uint64_t seed, const uint8_t* raw, uint64_t stream_off, uint32_t count,
                                       uint32_t q_bits, const std::vector<Nat>& sprp_q) {
  constexpr uint32_t W = 32;  // MPCX_SIEVE_MAX_BYTES / 4
  StepOut o;
  // Pocklington passes per candidate fall like 1 / bits: size the pass buffers
  // to the batch for small candidates, to 1/64 of it from 512-bit q up
  const uint32_t max_pass = q_bits >= 511 ? std::max<uint32_t>(1024, count / 64) : std::max<uint32_t>(count, 1);
  std::vector<uint32_t> pidx(max_pass), pp((size_t)max_pass * W), sq = pack(sprp_q, W);
  std::vector<uint8_t> sok(std::max<size_t>(sprp_q.size(), 1));
  uint32_t ns = 0, np = 0;
  enter_call();
  int rc = mpcx_safeprime_step(seed, raw, stream_off, count, q_bits, sprp_q.empty() ? nullptr : sq.data(),
                               (uint32_t)sprp_q.size(), max_pass, &ns, &np, pidx.data(), pp.data(), sok.data());
  leave_call();
  if (rc) throw_last(rc, "mpcx_safeprime_step");
  o.sieved = ns;
  o.idx.assign(pidx.begin(), pidx.begin() + np);
  o.p.resize(np);
  for (uint32_t j = 0; j < np; ++j) o.p[j] = Nat::from_words(pp.data() + (size_t)j * W, W);
  o.sprp.assign(sok.begin(), sok.begin() + sprp_q.size());
  return o;
}

std::vector<uint8_t> Engine::lucas(const std::vector<Nat>& n, const std::vector<uint32_t>& P) {
  if (n.size() != P.size()) throw std::invalid_argument("one P per candidate");
  if (n.empty()) return {};
  uint32_t w = 1;
  for (const auto& c : n) w = std::max<uint32_t>(w, (uint32_t)c.words());
  HostBuf N(n.size() * w);
  pack_into(n, w, N.p);
  std::vector<uint8_t> ok(n.size());
  enter_call();
  int rc = mpcx_lucas_batch((uint32_t)n.size(), N.p, w, P.data(), ok.data());
  leave_call();
  if (rc) throw_last(rc, "mpcx_lucas_batch");
  return ok;
}

std::vector<uint8_t> Engine::strong_probable_prime(const std::vector<Nat>& n, const std::vector<Nat>& bases) {
  if (n.size() != bases.size()) throw std::invalid_argument("one base per candidate");
  if (n.empty()) return {};
  uint32_t w = 1;
  for (const auto& c : n) w = std::max<uint32_t>(w, (uint32_t)c.words());
  std::vector<Nat> b(bases);
  for (size_t i = 0; i < b.size(); ++i)
    if (b[i].words() > w) b[i] = b[i] % n[i];
  HostBuf N(n.size() * w), A(n.size() * w);
  pack_into(n, w, N.p);
  pack_into(b, w, A.p);
  std::vector<uint8_t> ok(n.size());
  enter_call();
  int rc = mpcx_mr_batch((uint32_t)n.size(), N.p, w, A.p, ok.data());
  leave_call();
  if (rc) throw_last(rc, "mpcx_mr_batch");
  return ok;
}

}  // namespace mpcx::host
