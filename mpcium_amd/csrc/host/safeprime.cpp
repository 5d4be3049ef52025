// safeprime.cpp -- see safeprime.hpp.
#include "safeprime.hpp"

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <future>
#include <thread>

#include "engine.hpp"
#include "gorand.hpp"
#include "hostprof.hpp"
#include "modint.hpp"

namespace mpcx::host {

// ------------------------------------------------------------ candidates
static const uint32_t kSmallPrimes[] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53};
static const uint64_t kSmallPrimesProduct = 16294579238595022365ull;

Nat CandidateFromBytes(const uint8_t* bytes_in, size_t n, int qBitLen) {
  if (n == 0) throw std::invalid_argument("empty candidate");
  std::vector<uint8_t> bytes(bytes_in, bytes_in + n);
  unsigned b = (unsigned)(qBitLen % 8);
  if (b == 0) b = 8;
  bytes[0] &= (uint8_t)((1u << b) - 1);
  if (b >= 2) {
    bytes[0] |= (uint8_t)(3u << (b - 2));
  } else {
    bytes[0] |= 1;
    if (bytes.size() > 1) bytes[1] |= 0x80;
  }
  bytes.back() |= 1;
  Nat q = Nat::from_bytes_be(bytes.data(), bytes.size());
  // bigMod.Mod(q, smallPrimesProduct); delta walk (Go's old crypto/rand.Prime)
  uint64_t mod = 0;
  for (int i = (int)q.words() - 1; i >= 0; --i)
    mod = (uint64_t)(((unsigned __int128)mod << 32 | q.limbs()[i]) % kSmallPrimesProduct);
  for (uint64_t delta = 0; delta < (1ull << 20); delta += 2) {
    const uint64_t m = mod + delta;
    bool bad = false;
    for (uint32_t p : kSmallPrimes) {
      if (m % p == 0 && (qBitLen > 6 || m != p)) {
        bad = true;
        break;
      }
    }
    if (bad) continue;
    if (delta > 0) q = q + Nat(delta);
    break;
  }
  return q;
}

namespace {
// trial-division groups: primes 59 .. 2039 packed into products < 2^32
struct TrialGroups {
  std::vector<uint32_t> prod;
  std::vector<std::vector<uint32_t>> primes;
  TrialGroups() {
    std::vector<uint32_t> ps;
    for (uint32_t v = 59; v < 2048; v += 2) {
      bool pr = true;
      for (uint32_t d = 3; d * d <= v; d += 2)
        if (v % d == 0) {
          pr = false;
          break;
        }
      if (pr) ps.push_back(v);
    }
    uint64_t cur = 1;
    std::vector<uint32_t> grp;
    for (uint32_t p : ps) {
      if (cur * p >= (1ull << 32)) {
        prod.push_back((uint32_t)cur);
        primes.push_back(grp);
        cur = 1;
        grp.clear();
      }
      cur *= p;
      grp.push_back(p);
    }
    if (!grp.empty()) {
      prod.push_back((uint32_t)cur);
      primes.push_back(grp);
    }
  }
};
const TrialGroups& trial_groups() {
  static TrialGroups t;
  return t;
}

// exact: true iff neither q nor 2q+1 has a prime factor in [59, 2048)
bool passes_trial(const Nat& q) {
  const auto& tg = trial_groups();
  for (size_t g = 0; g < tg.prod.size(); ++g) {
    const uint64_t r = q.mod_u32(tg.prod[g]);
    for (uint32_t p : tg.primes[g]) {
      const uint64_t rq = r % p;
      if (rq == 0 || (2 * rq + 1) % p == 0) return false;
    }
  }
  return true;
}

// Miller-Rabin bases of ProbablyPrime(reps): base 2 (Go's forced last round;
// the decision does not depend on the order) first, then Go's `reps` bases in
// [2, n-2] from math/rand seeded with the candidate's low word (gorand.hpp)
std::vector<Nat> mr_bases(const Nat& q, int reps) {
  std::vector<Nat> out{Nat(2)};
  for (auto& b : GoMillerRabinBases(q, reps)) out.push_back(std::move(b));
  return out;
}
}  // namespace

// ------------------------------------------------------------ Stream
void Stream::read(uint8_t* out, size_t n) {
  const size_t from_pb = std::min(n, pushback_.size() - pb_pos_);
  if (from_pb) {
    std::memcpy(out, pushback_.data() + pb_pos_, from_pb);
    pb_pos_ += from_pb;
    if (pb_pos_ == pushback_.size()) {
      pushback_.clear();
      pb_pos_ = 0;
    }
    out += from_pb;
    n -= from_pb;
  }
  if (!n) return;
  if (drbg_) drbg_->read(out, n);
  else fn_(out, n);
}

void Stream::unread(const uint8_t* data, size_t n) {
  if (!n) return;
  if (drbg_ && pushback_.empty()) {  // a CounterDRBG just steps back
    drbg_->seek(drbg_->position() - n);
    return;
  }
  std::vector<uint8_t> nb(data, data + n);
  nb.insert(nb.end(), pushback_.begin() + (long)pb_pos_, pushback_.end());
  pushback_.swap(nb);
  pb_pos_ = 0;
}

// ------------------------------------------------------------ ProbablyPrime
int LucasParam(const Nat& n, uint32_t* P) {
  // go:src/math/big/prime.go probablyPrimeLucas: smallest P >= 3 with
  // Jacobi(P^2 - 4, n) = -1; Jacobi 0 means p + 2 | n; a square n never gets -1
  for (uint32_t p = 3;; ++p) {
    if (p > 10000) throw std::runtime_error("LucasParam: no D with (D/n) = -1");
    const int j = jacobi(Nat((uint64_t)p * p - 4), n);
    if (j == -1) {
      *P = p;
      return 1;
    }
    if (j == 0) return n == Nat(p + 2) ? 2 : 0;
    if (p == 40) {
      const Nat r = isqrt(n);
      if (r * r == n) return 0;
    }
  }
}

std::vector<uint8_t> ProbablyPrimeBatch(const std::vector<Nat>& n, int reps, SafePrimeStats* stats,
                                        bool base2_passed) {
  const size_t cnt = n.size();
  std::vector<uint8_t> ok(cnt, 0);
  static const uint32_t kSmall[] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53};
  const uint64_t mask = (1ull << 2) | (1ull << 3) | (1ull << 5) | (1ull << 7) | (1ull << 11) | (1ull << 13) |
                        (1ull << 17) | (1ull << 19) | (1ull << 23) | (1ull << 29) | (1ull << 31) | (1ull << 37) |
                        (1ull << 41) | (1ull << 43) | (1ull << 47) | (1ull << 53) | (1ull << 59) | (1ull << 61);
  std::vector<size_t> live;
  for (size_t i = 0; i < cnt; ++i) {
    const Nat& x = n[i];
    if (x.bit_len() <= 6) {  // x < 64
      ok[i] = (uint8_t)((mask >> x.low64()) & 1u);
      continue;
    }
    if (!x.is_odd()) continue;
    bool div = false;
    for (uint32_t p : kSmall) div |= x.mod_u32(p) == 0;
    if (!div) live.push_back(i);
  }
  // Miller-Rabin: base 2 first; the other bases only for its survivors
  std::vector<size_t> small, large;  // GPU thread-per-candidate class (< 2^1024) / wider
  for (size_t i : live) (n[i].bit_len() <= 1024 ? small : large).push_back(i);
  uint64_t mr = 0, lt = 0;
  if (!small.empty()) {
    std::vector<Nat> nn, aa;
    std::vector<size_t> s2;  // base-2 survivors
    if (base2_passed) {
      s2 = small;
    } else {
      for (size_t i : small) {
        nn.push_back(n[i]);
        aa.push_back(Nat(2));
      }
      auto r2 = Engine::get().strong_probable_prime(nn, aa);
      mr += nn.size();
      for (size_t j = 0; j < small.size(); ++j)
        if (r2[j]) s2.push_back(small[j]);
      nn.clear();
      aa.clear();
    }
    std::vector<size_t> owner;
    for (size_t i : s2) {
      const auto bs = mr_bases(n[i], reps);
      for (size_t b = 1; b < bs.size(); ++b) {
        nn.push_back(n[i]);
        aa.push_back(bs[b]);
        owner.push_back(i);
      }
    }
    // strong Lucas test on the base-2 survivors, concurrently with their
    // further Miller-Rabin bases (two latency-bound batches on two lanes)
    std::vector<Nat> ln;
    std::vector<uint32_t> lp;
    std::vector<size_t> lo;
    std::vector<uint8_t> lucas_ok(cnt, 0);
    for (size_t i : s2) {
      uint32_t P = 0;
      const int lr = LucasParam(n[i], &P);
      if (lr != 1) {
        lucas_ok[i] = lr == 2;
        continue;
      }
      ln.push_back(n[i]);
      lp.push_back(P);
      lo.push_back(i);
    }
    std::future<std::vector<uint8_t>> lucas;
    if (!ln.empty()) lucas = std::async(std::launch::async, [&] { return Engine::get().lucas(ln, lp); });
    std::vector<uint8_t> pass(cnt, 0);
    for (size_t i : s2) pass[i] = 1;
    std::exception_ptr mr_err;
    try {
      if (!nn.empty()) {
        auto rr = Engine::get().strong_probable_prime(nn, aa);
        mr += nn.size();
        for (size_t j = 0; j < nn.size(); ++j)
          if (!rr[j]) pass[owner[j]] = 0;
      }
    } catch (...) {
      mr_err = std::current_exception();
    }
    if (lucas.valid()) {
      const auto lr = lucas.get();  // joined before any rethrow
      lt += ln.size();
      for (size_t j = 0; j < ln.size(); ++j) lucas_ok[lo[j]] = lr[j];
    }
    if (mr_err) std::rethrow_exception(mr_err);
    for (size_t i : s2) ok[i] = pass[i] && lucas_ok[i];
  }
  std::vector<Nat> wl;  // > 1024 bits passing every Miller-Rabin base: Lucas next
  std::vector<uint32_t> wp;
  std::vector<size_t> wo;
  for (size_t i : large) {
    // > 1024 bits: base 2 + reps bases as one shared-exponent launch (x^d for
    // every base), the s - 1 squarings on the host, then the strong Lucas test
    const Nat& x = n[i];
    const Nat nm1 = x - Nat(1);
    uint32_t s = 0;
    while (!nm1.bit(s)) ++s;
    const Nat d = nm1 >> s;
    const auto bs = mr_bases(x, reps);
    std::vector<Nat> ys = Engine::get().exp(x, bs, std::vector<Nat>{d});
    mr += bs.size();
    bool all = true;
    for (Nat y : ys) {
      if (y == Nat(1) || y == nm1) continue;
      bool hit = false;
      for (uint32_t j = 1; j < s && !hit; ++j) {
        y = (y * y) % x;
        if (y == Nat(1)) break;
        hit = y == nm1;
      }
      if (!hit) {
        all = false;
        break;
      }
    }
    if (!all) continue;
    uint32_t P = 0;
    const int lr = LucasParam(x, &P);
    if (lr != 1) {
      ok[i] = lr == 2;
      continue;
    }
    wl.push_back(x);
    wp.push_back(P);
    wo.push_back(i);
  }
  if (!wl.empty()) {
    const auto lr = Engine::get().lucas(wl, wp);
    lt += wl.size();
    for (size_t j = 0; j < wl.size(); ++j) ok[wo[j]] = lr[j];
  }
  if (stats) {
    stats->mr_tests += mr;
    stats->lucas_tests += lt;
  }
  return ok;
}

namespace {
void check_safe_prime_args(int bitLen) {
  if (bitLen < 6) throw std::invalid_argument("safe prime size must be at least 6 bits");
  if (bitLen > 1024) throw std::invalid_argument("GPU candidate class holds safe primes up to 1024 bits");
}

// candidates per batch: ~45K per 1024-bit safe prime, far fewer at small sizes
// (environment MPCX_SAFEPRIME_BATCH overrides it above 512 bits; the output
// and the stream consumption do not depend on the batch size)
size_t default_batch(int bitLen) {
  if (bitLen > 512) {
    static const size_t env = [] {
      const char* e = std::getenv("MPCX_SAFEPRIME_BATCH");
      const long v = e ? std::atol(e) : 0;
      return v >= 1024 && v <= (1l << 22) ? (size_t)v : (size_t)0;
    }();
    if (env) return env;
    // 3 * 2^18: ~228K sieve survivors per step, 2.3 resident rounds of
    // k_prime2c (MI355X, profiles/r02/sp_sweep: 256 safe primes at 2^19 /
    // 3 * 2^18 / 3.5 * 2^18 / 2^20 -> 486 / 518 / 514 / 499 per s; the bench's
    // 64 primes measure the same 400-412 per s for 2^19 .. 3 * 2^18, where the
    // last step's overshoot offsets the fuller rounds)
    return 786432;
  }
  if (bitLen > 256) return 65536;
  return 16384;
}

void add_stats(SafePrimeStats* stats, const SafePrimeStats& st) {
  if (!stats) return;
  stats->candidates += st.candidates;
  stats->sieved_out += st.sieved_out;
  stats->fermat_tests += st.fermat_tests;
  stats->mr_tests += st.mr_tests;
  stats->lucas_tests += st.lucas_tests;
  stats->seconds += st.seconds;
}

// Host-sieve path for q below the GPU sieve's 63 bits: one batch of raw
// stream bytes -> (candidate index, q) of its Fermat passes.
void small_batch(int bitLen, const uint8_t* raw, size_t batch, SafePrimeStats& st, std::vector<uint32_t>* fidx,
                 std::vector<Nat>* fq) {
  const int qBitLen = bitLen - 1;
  const size_t nbytes = (size_t)(qBitLen + 7) / 8;
  std::vector<Nat> qs(batch), ps;
  std::vector<uint8_t> keep(batch, 0);
  parallel_for(batch, [&](size_t i) {
    qs[i] = CandidateFromBytes(raw + i * nbytes, nbytes, qBitLen);
    keep[i] = (qs[i].bit_len() == (uint32_t)qBitLen) && (bitLen <= 12 || passes_trial(qs[i]));
  });
  std::vector<uint32_t> idx;
  for (size_t i = 0; i < batch; ++i) {
    if (!keep[i]) continue;
    idx.push_back((uint32_t)i);
    ps.push_back((qs[i] << 1) + Nat(1));
  }
  st.sieved_out += batch - idx.size();
  st.fermat_tests += ps.size();
  std::vector<uint8_t> f = bitLen >= 4 ? Engine::get().fermat2(ps) : std::vector<uint8_t>(ps.size(), 1);
  for (size_t j = 0; j < idx.size(); ++j)
    if (f[j]) {
      fidx->push_back(idx[j]);
      fq->push_back(qs[idx[j]]);
    }
}

// q (< 2^1023) that passed the base-2 Miller-Rabin round: the remaining
// ProbablyPrime(20) rounds and the strong Lucas test
std::vector<uint8_t> finish_q(const std::vector<Nat>& qs, SafePrimeStats& st) {
  MPCX_PROF("sp.stage_b");
  return ProbablyPrimeBatch(qs, 20, &st, /*base2_passed=*/true);
}
}  // namespace

std::vector<GermainSafePrime> GetRandomSafePrimes(int bitLen, int numPrimes, Stream& src, SafePrimeStats* stats,
                                                  size_t batch, uint64_t max_candidates) {
  check_safe_prime_args(bitLen);
  if (numPrimes < 1) throw std::invalid_argument("numPrimes should be > 0");
  const auto t0 = std::chrono::steady_clock::now();
  SafePrimeStats st;
  const int qBitLen = bitLen - 1;
  const size_t nbytes = (size_t)(qBitLen + 7) / 8;
  if (batch == 0) batch = default_batch(bitLen);
  const bool gpu = qBitLen >= 63;
  CounterDRBG* dev = gpu ? src.device_stream() : nullptr;
  const uint64_t off0 = dev ? dev->position() : 0;
  std::vector<std::vector<uint8_t>> raws;  // host-read batches (given back past the last accepted candidate)
  std::vector<GermainSafePrime> acc;        // accepted, stream order (decided candidates only)
  // Pipeline (one step per batch): step k runs the sieve + Pocklington of
  // batch k and the base-2 round of batch k-1's Fermat passes; batch k-1's
  // base-2 survivors then finish (other rounds + Lucas) while step k+1 runs.
  // Batches are decided in order, so `acc` only ever holds decided batches.
  struct Cand {
    uint64_t index;
    Nat q;
  };
  std::vector<Cand> fermat_prev;  // Fermat passes of the previous batch
  std::vector<Cand> running;      // stage B in flight
  std::future<std::vector<uint8_t>> job;
  SafePrimeStats stb;             // stage-B counters (joined before use)
  auto absorb = [&](const std::vector<Cand>& c, const std::vector<uint8_t>& v) {
    for (size_t j = 0; j < c.size(); ++j)
      if (v[j]) acc.push_back({(c[j].q << 1) + Nat(1), c[j].q, c[j].index});
  };
  auto join = [&] {
    MPCX_PROF("sp.join_wait");
    if (job.valid()) absorb(running, job.get());
    running.clear();
  };
  auto qs_of = [](const std::vector<Cand>& c) {
    std::vector<Nat> qs;
    for (const auto& x : c) qs.push_back(x.q);
    return qs;
  };
  uint64_t next = 0;  // next candidate index to draw
  for (;;) {
    const bool more = next < max_candidates;
    if (!more && fermat_prev.empty() && !job.valid()) break;
    const uint64_t first = next;
    const uint32_t count = more ? (uint32_t)batch : 0u;
    const std::vector<Nat> ride = qs_of(fermat_prev);
    std::vector<uint32_t> fidx;
    std::vector<Nat> fq;
    std::vector<uint8_t> sprp;
    if (gpu) {
      std::vector<uint8_t> raw;
      if (count && !dev) {
        raw.resize((size_t)count * nbytes);
        src.read(raw.data(), raw.size());
      }
      MPCX_PROF("sp.step");
      const auto o = Engine::get().safeprime_step(dev ? dev->seed() : 0, raw.empty() ? nullptr : raw.data(),
                                                  off0 + first * nbytes, count, (uint32_t)qBitLen, ride);
      st.sieved_out += count - o.sieved;
      st.fermat_tests += o.sieved;
      fidx = o.idx;
      for (const auto& p : o.p) fq.push_back(p >> 1);  // q = (p - 1) / 2
      sprp = o.sprp;
      if (!raw.empty()) raws.push_back(std::move(raw));
    } else {
      if (count) {
        std::vector<uint8_t> raw((size_t)count * nbytes);
        src.read(raw.data(), raw.size());
        small_batch(bitLen, raw.data(), count, st, &fidx, &fq);
        raws.push_back(std::move(raw));
      }
      const std::vector<Nat> two(ride.size(), Nat(2));
      sprp = Engine::get().strong_probable_prime(ride, two);
    }
    st.mr_tests += ride.size();
    st.candidates += count;
    next += count;
    std::vector<Cand> surv;  // previous batch's base-2 survivors
    for (size_t j = 0; j < fermat_prev.size(); ++j)
      if (sprp[j]) surv.push_back(fermat_prev[j]);
    join();  // the batch before the previous one is decided
    if (acc.size() >= (size_t)numPrimes) break;
    if (acc.size() + surv.size() >= (size_t)numPrimes || !more) {
      // its probable primes may suffice: finish them now rather than draw on
      MPCX_PROF("sp.finish_sync");
      absorb(surv, finish_q(qs_of(surv), stb));
      if (acc.size() >= (size_t)numPrimes) break;
    } else {
      running = std::move(surv);
      job = std::async(std::launch::async, [qs = qs_of(running), &stb] { return finish_q(qs, stb); });
    }
    fermat_prev.clear();
    for (size_t j = 0; j < fidx.size(); ++j) fermat_prev.push_back({first + fidx[j], fq[j]});
  }
  join();
  st.mr_tests += stb.mr_tests;
  st.lucas_tests += stb.lucas_tests;
  std::sort(acc.begin(), acc.end(), [](const auto& a, const auto& b) { return a.index < b.index; });
  if ((int)acc.size() < numPrimes) throw std::runtime_error("safe prime search exhausted max_candidates");
  acc.resize((size_t)numPrimes);
  // leave the stream right after the last accepted candidate
  const uint64_t consumed = (acc.back().index + 1) * nbytes;
  if (dev) {
    dev->seek(off0 + consumed);
  } else {
    uint64_t pos = 0;
    std::vector<uint8_t> back;
    for (const auto& r : raws) {
      const uint64_t lo = pos, hi = pos + r.size();
      if (hi > consumed) {
        const uint64_t from = consumed > lo ? consumed - lo : 0;
        back.insert(back.end(), r.begin() + (long)from, r.end());
      }
      pos = hi;
    }
    src.unread(back.data(), back.size());
  }
  st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  add_stats(stats, st);
  return acc;
}

std::vector<GermainSafePrime> GetRandomSafePrimes(int bitLen, int numPrimes, const RandFn& rand,
                                                  SafePrimeStats* stats, size_t batch, uint64_t max_candidates) {
  Stream s(rand);
  return GetRandomSafePrimes(bitLen, numPrimes, s, stats, batch, max_candidates);
}

std::vector<GermainSafePrime> SafePrimeBatch(int bitLen, uint64_t seed, uint64_t batch_no, size_t batch,
                                             SafePrimeStats* stats) {
  check_safe_prime_args(bitLen);
  const auto t0 = std::chrono::steady_clock::now();
  if (batch == 0) batch = default_batch(bitLen);
  const int qBitLen = bitLen - 1;
  const size_t nbytes = (size_t)(qBitLen + 7) / 8;
  SafePrimeStats st;
  std::vector<uint32_t> fidx;
  std::vector<Nat> fq;
  if (qBitLen >= 63) {
    const auto o = Engine::get().safeprime_step(seed, nullptr, batch_no * batch * nbytes, (uint32_t)batch,
                                                (uint32_t)qBitLen, {});
    st.sieved_out += batch - o.sieved;
    st.fermat_tests += o.sieved;
    fidx = o.idx;
    for (const auto& p : o.p) fq.push_back(p >> 1);
  } else {
    std::vector<uint8_t> raw(nbytes * batch);
    CounterDRBG drbg(seed);
    drbg.seek(batch_no * (uint64_t)raw.size());
    drbg.read(raw.data(), raw.size());
    small_batch(bitLen, raw.data(), batch, st, &fidx, &fq);
  }
  st.candidates += batch;
  const auto pr = ProbablyPrimeBatch(fq, 20, &st);
  std::vector<GermainSafePrime> out;
  for (size_t j = 0; j < fq.size(); ++j)
    if (pr[j]) out.push_back({(fq[j] << 1) + Nat(1), fq[j], batch_no * batch + fidx[j]});
  st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  add_stats(stats, st);
  return out;
}

paillier::PrivateKey GenerateKeyPair(int modulusBitLen, Stream& rand, SafePrimeStats* stats) {
  const int half = modulusBitLen / 2;
  Nat P, Q;
  for (;;) {
    auto sgps = GetRandomSafePrimes(half, 2, rand, stats);
    P = sgps[0].p;
    Q = sgps[1].p;
    const Nat d = P >= Q ? P - Q : Q - P;
    if ((int)d.bit_len() >= half - 3) break;  // KS-BTL-F-03: |P-Q| must be large
  }
  paillier::PrivateKey sk;
  sk.pub.N = P * Q;
  const Nat Pm1 = P - Nat(1), Qm1 = Q - Nat(1);
  sk.PhiN = Pm1 * Qm1;
  sk.LambdaN = sk.PhiN / gcd(Pm1, Qm1);
  sk.P = P;
  sk.Q = Q;
  return sk;
}

LocalPreParams GeneratePreParams(Stream& stream, SafePrimeStats* stats) {
  const RandFn rand = stream.fn();
  LocalPreParams pp;
  // tss-lib runs these two searches concurrently on one reader (stream
  // interleaving is scheduling-defined); here they run in a fixed order.
  pp.PaillierSK = GenerateKeyPair(2048, stream, stats);
  auto sgps = GetRandomSafePrimes(1024, 2, stream, stats);
  const Nat P = sgps[0].p, Q = sgps[1].p;
  pp.NTildei = P * Q;
  pp.P = sgps[0].q;
  pp.Q = sgps[1].q;
  const Nat pq = pp.P * pp.Q;
  const Nat f1 = GetRandomPositiveRelativelyPrimeInt(rand, pp.NTildei);
  pp.Alpha = GetRandomPositiveRelativelyPrimeInt(rand, pp.NTildei);
  if (!mod_inverse(Int(pp.Alpha), pq, &pp.Beta)) throw std::runtime_error("alpha not invertible mod pq");
  const ModInt modN(pp.NTildei);
  pp.H1i = modN.Mul(f1, f1);
  if (!modN.Exp(Int(pp.H1i), Int(pp.Alpha), &pp.H2i)) throw std::runtime_error("h2 = h1^alpha failed");
  return pp;
}

}  // namespace mpcx::host
