// engine.cpp -- see engine.hpp.
#include "engine.hpp"

#include "hostprof.hpp"

#include <algorithm>
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

void Engine::init(int device) {
  std::lock_guard<std::mutex> lk(mu_);
  int rc = mpcx_init(device);
  if (rc) throw_last(rc, "mpcx_init");
  bound_ = true;
  const char* fb = std::getenv("MPCX_FIXED_BASE");
  fixed_enabled_ = !(fb && fb[0] == '0');
}

void Engine::init_devices(int n_gpus) {
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

void Engine::count_work(const Nat& m, const std::vector<Nat>& exps, size_t count) {
  const uint64_t L = m.words(), l2 = 2 * L * L;
  uint64_t w = 0;
  auto one = [&](const Nat& e) {
    const uint64_t E = e.bit_len();
    return (E + (E + 3) / 4) * l2;
  };
  if (exps.size() == 1 && count != 1) {
    w = one(exps[0]) * count;
  } else {
    for (const auto& e : exps) w += one(e);
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

static std::vector<uint32_t> pack(const std::vector<Nat>& v, uint32_t w) {
  std::vector<uint32_t> out((size_t)v.size() * w);
  for (size_t i = 0; i < v.size(); ++i) v[i].to_words(out.data() + i * w, w);
  return out;
}

static std::vector<Nat> unpack(const std::vector<uint32_t>& buf, size_t count, uint32_t w) {
  std::vector<Nat> out(count);
  for (size_t i = 0; i < count; ++i) out[i] = Nat::from_words(buf.data() + i * w, w);
  return out;
}

std::vector<Nat> Engine::exp(const Nat& m, const std::vector<Nat>& bases, const std::vector<Nat>& exps,
                             const std::vector<Nat>* muls) {
  if (exps.size() != 1 && exps.size() != bases.size()) throw std::invalid_argument("exps: 1 or one per base");
  if (muls && muls->size() != bases.size()) throw std::invalid_argument("muls: one per base");
  if (bases.empty()) return {};
  Mod md;
  {
    std::lock_guard<std::mutex> lk(mu_);
    md = modulus(m);
  }
  // Host-side packing runs outside the lock, so another thread's batch can
  // use the GPU meanwhile. math/big reduces x mod m first when
  // len(x) > len(m) (nat.expNNMontgomery); here: only when x does not fit
  // the kernel class width.
  auto packed = [&](const std::vector<Nat>& v) {
    std::vector<uint32_t> out((size_t)v.size() * md.class_words);
    for (size_t i = 0; i < v.size(); ++i) {
      if (v[i].words() > md.class_words) {
        (v[i] % m).to_words(out.data() + i * md.class_words, md.class_words);
      } else {
        v[i].to_words(out.data() + i * md.class_words, md.class_words);
      }
    }
    return out;
  };
  const bool shared = exps.size() == 1;
  uint32_t ew = 1;
  for (const auto& e : exps) ew = std::max<uint32_t>(ew, (uint32_t)e.words());
  std::vector<uint32_t> B, E, M;
  {
    MPCX_PROF("engine.exp.pack");
    B = packed(bases);
    E = pack(exps, ew);
    if (muls) M = packed(*muls);
  }
  std::vector<uint32_t> out((size_t)bases.size() * md.words);
  count_work(m, exps, bases.size());
  int rc;
  MPCX_PROF("engine.exp.gpu+unpack");
  enter_call();
  if (muls) {
    rc = mpcx_modexp_mul_batch(md.h, (uint32_t)bases.size(), B.data(), md.class_words, E.data(), ew, shared ? 1 : 0,
                               M.data(), md.class_words, out.data(), md.words);
  } else {
    rc = mpcx_modexp_batch(md.h, (uint32_t)bases.size(), B.data(), md.class_words, E.data(), ew, shared ? 1 : 0,
                           out.data(), md.words);
  }
  leave_call();
  if (rc) throw_last(rc, "mpcx_modexp_batch");
  return unpack(out, bases.size(), md.words);
}

bool Engine::fixed_base_ok(const Nat& m) const {
  return fixed_enabled_ && m.is_odd() && m.bit_len() <= 2080;
}

Engine::Fixed Engine::fixed(const Nat& m, const Nat& base, uint32_t need_bits) {
  auto key = std::make_pair(m.limbs(), base.limbs());
  auto it = fixed_.find(key);
  if (it != fixed_.end() && it->second->max_bits >= need_bits) return it->second;
  if (it != fixed_.end()) fixed_.erase(it);  // grow: rebuild for the longer exponent
  if (fixed_.size() >= 256) fixed_.clear();  // bound the device footprint (~30 MB per table)
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
  fixed_.emplace(key, f);
  return f;
}

std::vector<Nat> Engine::fixed_exp(const Nat& m, const Nat& base, const std::vector<Nat>& exps,
                                   const std::vector<Nat>* muls) {
  if (muls && muls->size() != exps.size()) throw std::invalid_argument("muls: one per exponent");
  if (exps.empty()) return {};
  Mod md;
  {
    std::lock_guard<std::mutex> lk(mu_);
    md = modulus(m);
  }
  uint32_t ew = 1, need = 1;
  for (const auto& e : exps) {
    ew = std::max<uint32_t>(ew, (uint32_t)e.words());
    need = std::max<uint32_t>(need, e.bit_len());
  }
  const Nat b = base.words() > md.class_words || base >= m ? base % m : base;
  auto E = pack(exps, ew);
  std::vector<uint32_t> Mw;
  if (muls) {
    Mw.assign((size_t)muls->size() * md.class_words, 0);
    for (size_t i = 0; i < muls->size(); ++i) {
      const Nat& x = (*muls)[i];
      (x.words() > md.class_words ? x % m : x).to_words(Mw.data() + i * md.class_words, md.class_words);
    }
  }
  std::vector<uint32_t> out((size_t)exps.size() * md.words);
  Fixed f;
  {
    // look up (or build) under the lock; the shared handle keeps the table
    // alive while this batch uses it, even if another thread evicts it
    std::lock_guard<std::mutex> lk(mu_);
    f = fixed(m, b, need);
  }
  const uint32_t* ep = E.data();
  count_work(m, exps, exps.size());
  MPCX_PROF("engine.fixed.gpu+unpack");
  enter_call();
  int rc = mpcx_fixedbase_exp_batch(1, &f->h, (uint32_t)exps.size(), &ep, &ew, muls ? Mw.data() : nullptr,
                                    muls ? md.class_words : 0, out.data(), md.words);
  leave_call();
  if (rc) throw_last(rc, "mpcx_fixedbase_exp_batch");
  return unpack(out, exps.size(), md.words);
}

std::vector<Nat> Engine::mulmod(const Nat& m, const std::vector<Nat>& a, const std::vector<Nat>& b) {
  std::vector<Nat> one{Nat(1)};
  return exp(m, a, one, &b);
}

std::vector<uint8_t> Engine::fermat2(const std::vector<Nat>& cands) {
  if (cands.empty()) return {};
  uint32_t w = 1;
  for (const auto& c : cands) w = std::max<uint32_t>(w, (uint32_t)c.words());
  auto P = pack(cands, w);
  std::vector<uint8_t> ok(cands.size());
  int rc = mpcx_fermat2_batch((uint32_t)cands.size(), P.data(), w, ok.data());
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
  auto N = pack(n, w);
  std::vector<uint8_t> ok(n.size());
  enter_call();
  int rc = mpcx_lucas_batch((uint32_t)n.size(), N.data(), w, P.data(), ok.data());
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
  auto N = pack(n, w);
  auto A = pack(b, w);
  std::vector<uint8_t> ok(n.size());
  enter_call();
  int rc = mpcx_mr_batch((uint32_t)n.size(), N.data(), w, A.data(), ok.data());
  leave_call();
  if (rc) throw_last(rc, "mpcx_mr_batch");
  return ok;
}

}  // namespace mpcx::host
