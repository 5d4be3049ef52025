// keygenload.cpp -- see keygenload.hpp.
#include "keygenload.hpp"

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <memory>
#include <stdexcept>
#include <thread>

#include "engine.hpp"
#include "hostprof.hpp"
#include "proofs.hpp"
#include "secp256k1.hpp"
#include "tsscommon.hpp"

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
    MPCX_PROF_CPU("cpu.keygen_tasks");
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

// one random stream per (session, party, proof kind, peer) for sessions [lo, hi)
struct Streams {
  std::vector<CounterDRBG> drbg;
  std::vector<RandFn> fn;
  Streams(uint64_t seed, size_t lo, size_t hi, uint64_t party, uint64_t kind) {
    drbg.reserve(hi - lo);
    for (size_t s = lo; s < hi; ++s) drbg.emplace_back(mix(seed, s, party, kind));
    for (auto& d : drbg) fn.push_back(d.fn());
  }
};

Nat digest(const std::vector<const Nat*>& v) { return SHA512_256i(v); }
Nat dln_digest(const proofs::DLNProof& p) {
  std::vector<const Nat*> v;
  for (const auto& x : p.Alpha) v.push_back(&x);
  for (const auto& x : p.T) v.push_back(&x);
  return digest(v);
}
Nat mod_digest(const proofs::ModProof& p) {
  std::vector<const Nat*> v{&p.W, &p.A, &p.B};
  for (const auto& x : p.X) v.push_back(&x);
  for (const auto& x : p.Z) v.push_back(&x);
  return digest(v);
}
Nat fac_digest(const proofs::FacProof& p) {
  const Nat vabs = p.V.mag, vneg(p.V.neg ? 1u : 0u);
  return digest({&p.P, &p.Q, &p.A, &p.B, &p.T, &p.Sigma, &p.Z1, &p.Z2, &p.W1, &p.W2, &vabs, &vneg});
}

secp::Affine negate(const secp::Affine& P) {
  if (P.inf) return P;
  secp::Affine r = P;
  const Nat y = secp::FeToNat(P.y);
  r.y = secp::NatToFe(y.is_zero() ? y : secp::FieldP() - y);
  return r;
}

// The old committee's side of a resharing wave [lo, hi) (keygenload.hpp) and
// the new committee's checks of it: two GPU EC batches (k_ec_combine) plus
// host hashing. vt: the traced session's TraceVssWords(n) words (or null).
void vss_wave(size_t lo, size_t hi, size_t n, uint64_t seed, size_t ts, uint32_t* vt, std::atomic<uint64_t>& checks,
              std::atomic<uint64_t>& fails, int64_t tamper) {
  MPCX_PROF("keygen.vss");
  constexpr size_t T = kReshareThreshold;
  static_assert(T == 2, "the share check is one a*G + b*P + c*Q combination");
  const size_t m = hi - lo;
  const Nat& q = secp::CurveN();
  // Lagrange coefficients of the old committee (ids 1..n) at 0
  std::vector<Nat> lam(n);
  for (size_t i = 0; i < n; ++i) {
    Nat num(1), den(1);
    for (size_t j = 0; j < n; ++j) {
      if (j == i) continue;
      num = (num * Nat(j + 1)) % q;
      den = (den * ((Nat(j + 1) + q - Nat(i + 1)) % q)) % q;
    }
    Nat inv;
    if (!mod_inverse(Int(den), q, &inv)) throw std::runtime_error("vss: Lagrange denominator");
    lam[i] = (num * inv) % q;
  }
  struct Old {
    std::vector<Nat> a, sh;  // coefficients a_0..a_T, shares s_i1..s_in
    Nat r, C;
    std::vector<secp::Affine> V;
  };
  std::vector<Nat> secret(m);
  std::vector<std::vector<Old>> od(m, std::vector<Old>(n));
  parallel_for(m, [&](size_t x) {
    const size_t s = lo + x;
    CounterDRBG wd(mix(seed, s, 0xEE, 0));  // the wallet's old sharing polynomial
    const RandFn wr = wd.fn();
    std::vector<Nat> c(T + 1);
    for (auto& ck : c) ck = GetRandomPositiveInt(wr, q);
    secret[x] = c[0];
    for (size_t i = 0; i < n; ++i) {
      Nat xi = c[T];  // x_i = f(i + 1) by Horner
      for (size_t k = T; k-- > 0;) xi = (xi * Nat(i + 1) + c[k]) % q;
      Old& o = od[x][i];
      CounterDRBG d(mix(seed, s, i, 9));
      const RandFn r = d.fn();
      o.a.resize(T + 1);
      o.a[0] = (lam[i] * xi) % q;  // w_i
      for (size_t k = 1; k <= T; ++k) o.a[k] = GetRandomPositiveInt(r, q);
      o.r = MustGetRandomInt(r, 256);
      o.sh.resize(n);
      for (size_t j = 0; j < n; ++j) {
        Nat v = o.a[T];
        for (size_t k = T; k-- > 0;) v = (v * Nat(j + 1) + o.a[k]) % q;
        o.sh[j] = v;
      }
    }
  });
  // EC batch 1: X = secret G, V_ik = a_k G
  std::vector<secp::Comb> c1(m * (1 + n * (T + 1)));
  for (size_t x = 0; x < m; ++x) {
    const size_t b = x * (1 + n * (T + 1));
    c1[b].a = secret[x];
    for (size_t i = 0; i < n; ++i)
      for (size_t k = 0; k <= T; ++k) c1[b + 1 + i * (T + 1) + k].a = od[x][i].a[k];
  }
  const std::vector<secp::Affine> p1 = secp::CombineBatch(c1);
  std::vector<secp::Affine> X(m);
  parallel_for(m, [&](size_t x) {
    const size_t b = x * (1 + n * (T + 1));
    X[x] = p1[b];
    for (size_t i = 0; i < n; ++i) {
      Old& o = od[x][i];
      o.V.assign(p1.begin() + (long)(b + 1 + i * (T + 1)), p1.begin() + (long)(b + 1 + (i + 1) * (T + 1)));
      std::vector<Nat> flat{o.r};
      for (const auto& v : o.V) {
        flat.push_back(secp::FeToNat(v.x));
        flat.push_back(secp::FeToNat(v.y));
      }
      std::vector<const Nat*> in;
      for (const auto& f : flat) in.push_back(&f);
      o.C = SHA512_256i(in);  // commitments.NewHashCommitment(rand, flatVs...)
    }
  });
  if (tamper >= (int64_t)lo && tamper < (int64_t)hi && n > 1) {  // old party 0 -> new party 1, off by one
    Nat& sh = od[(size_t)tamper - lo][0].sh[1];
    sh = (sh + Nat(1)) % q;
  }
  // EC batch 2: new party j's share check of old party i:
  // (q - s_ij) G + j V_i1 + j^2 V_i2 == -V_i0
  std::vector<secp::Comb> c2(m * n * n);
  std::vector<uint8_t> dec_ok(m * n * n, 0);
  parallel_for(m, [&](size_t x) {
    for (size_t i = 0; i < n; ++i) {
      const Old& o = od[x][i];
      std::vector<Nat> D{o.r};  // the decommitment as received, checked against C_i
      for (const auto& v : o.V) {
        D.push_back(secp::FeToNat(v.x));
        D.push_back(secp::FeToNat(v.y));
      }
      std::vector<const Nat*> in;
      for (const auto& f : D) in.push_back(&f);
      const bool dc = SHA512_256i(in) == o.C;
      for (size_t j = 0; j < n; ++j) {
        secp::Comb& cb = c2[(x * n + i) * n + j];
        const Nat& sij = o.sh[j];
        cb.a = sij.is_zero() ? sij : q - sij;
        cb.P = o.V[1];
        cb.b = Nat(j + 1);
        cb.Q = o.V[2];
        cb.c = Nat((j + 1) * (j + 1));
        dec_ok[(x * n + i) * n + j] = dc;
      }
    }
  });
  const std::vector<secp::Affine> p2 = secp::CombineBatch(c2);
  std::atomic<uint64_t> ok_total{0}, bad_total{0};
  parallel_for(m, [&](size_t x) {
    uint64_t good = 0, bad = 0;
    secp::Affine sumV;
    for (size_t i = 0; i < n; ++i) {
      const Old& o = od[x][i];
      sumV = secp::Add(sumV, o.V[0]);
      const secp::Affine nv0 = negate(o.V[0]);
      for (size_t j = 0; j < n; ++j) {
        const size_t k = (x * n + i) * n + j;
        (dec_ok[k] && secp::Equal(p2[k], nv0) ? good : bad) += 1;
      }
    }
    // every new party: sum_i V_i0 == X
    (secp::Equal(sumV, X[x]) ? good : bad) += n;
    ok_total += good;
    bad_total += bad;
    if (vt && lo + x == ts) {
      uint32_t* d = vt;
      for (size_t i = 0; i < n; ++i, d += 8) {
        const Old& o = od[x][i];
        std::vector<Nat> v{o.C};
        for (const auto& pt : o.V) {
          v.push_back(secp::FeToNat(pt.x));
          v.push_back(secp::FeToNat(pt.y));
        }
        for (const auto& sh : o.sh) v.push_back(sh);
        std::vector<const Nat*> in;
        for (const auto& f : v) in.push_back(&f);
        SHA512_256i(in).to_words(d, 8);
      }
      std::vector<Nat> xs(n);
      for (size_t j = 0; j < n; ++j) {
        Nat acc;
        for (size_t i = 0; i < n; ++i) acc = acc + od[x][i].sh[j];
        xs[j] = acc % q;  // x'_j
      }
      std::vector<const Nat*> in;
      for (const auto& f : xs) in.push_back(&f);
      SHA512_256i(in).to_words(d, 8);
      d[8] = (uint32_t)good;
    }
  });
  checks += ok_total.load() + bad_total.load();
  fails += bad_total.load();
}

}  // namespace

ProofStats RunKeygenProofs(const std::vector<PartyKeys>& parties, size_t sessions, uint64_t seed,
                           size_t wave_sessions, std::vector<uint32_t>* trace, int reshare_mix, int64_t tamper_session) {
  const size_t n = parties.size();
  if (n < 2) throw std::invalid_argument("need at least two parties");
  const size_t W = wave_sessions ? wave_sessions : kDefaultWave;
  const size_t n_waves = sessions ? (sessions + W - 1) / W : 0;
  ProofStats st;
  st.sessions = sessions;
  st.parties = n;
  st.waves = n_waves;
  st.wave_sessions = W;
  st.proofs = (uint64_t)sessions * n * (3 + (n - 1));
  st.verifications = (uint64_t)sessions * n * (n - 1) * 4;
  const size_t tk = TraceSessionWords(n), tw = tk + (reshare_mix ? TraceVssWords(n) : 0);
  if (trace) trace->assign(n_waves * tw, 0);
  std::atomic<uint64_t> fails{0}, vss_checks{0}, vss_fails{0};
  std::atomic<uint64_t> kg_sessions{0}, rs_sessions{0};
  double kg_wave_s = 0, rs_wave_s = 0;  // under tm
  std::mutex tm;
  double last_prove = 0, max_wave = 0;
  size_t waves_done = 0;  // under tm
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

  // One wave [lo, hi): one chain per proof batch -- prove, then every peer's
  // verification of it (no barrier between proving and verifying: one chain's
  // host steps overlap another's GPU batches); the wave's proofs are dropped
  // when it returns.
  auto run_wave = [&](size_t w) {
    const size_t lo = w * W, hi = std::min(sessions, lo + W), m = hi - lo;
    const bool reshare = reshare_mix && (w % 2 == 1);
    const double w0 = now();
    std::vector<proofs::Bytes> sess(m);  // SSID bytes shared by the parties of a session
    {
      CounterDRBG d(mix(seed, 0xFFFF, 0, 0));
      d.seek((uint64_t)lo * 32);
      for (auto& b : sess) {
        b.resize(32);
        d.read(b.data(), 32);
      }
    }
    std::vector<std::unique_ptr<Streams>> streams;
    auto stream = [&](uint64_t party, uint64_t kind) -> const std::vector<RandFn>& {
      streams.push_back(std::make_unique<Streams>(seed, lo, hi, party, kind));
      return streams.back()->fn;
    };
    std::vector<const std::vector<RandFn>*> r_dln1(n), r_dln2(n), r_mod(n);
    std::vector<std::vector<const std::vector<RandFn>*>> r_fac(n, std::vector<const std::vector<RandFn>*>(n));
    for (size_t i = 0; i < n; ++i) {
      r_dln1[i] = &stream(i, 1);
      r_dln2[i] = &stream(i, 2);
      r_mod[i] = &stream(i, 3);
      for (size_t j = 0; j < n; ++j)
        if (j != i) r_fac[i][j] = &stream(i, 16 + j);
    }
    std::vector<std::vector<proofs::DLNProof>> dln1(n), dln2(n);
    std::vector<std::vector<proofs::ModProof>> mod(n);
    std::vector<std::vector<std::vector<proofs::FacProof>>> fac(n, std::vector<std::vector<proofs::FacProof>>(n));
    const size_t ts = TracedSession(w, lo, hi) - lo;  // traced session within the wave
    std::atomic<uint32_t> traced_ok{0};
    auto count = [&](const std::vector<uint8_t>& ok) {
      uint64_t f = 0;
      for (auto v : ok) f += v == 0;
      fails += f;
      traced_ok += ok[ts] != 0;
    };
    auto proved = [&] {
      std::lock_guard<std::mutex> lk(tm);
      last_prove = std::max(last_prove, now());
    };
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
    if (reshare)  // the old committee's VSS beside the new committee's proof chains
      tasks.push_back([&, lo, hi] {
        vss_wave(lo, hi, n, seed, TracedSession(w, lo, hi), trace ? trace->data() + w * tw + tk : nullptr, vss_checks,
                 vss_fails, tamper_session);
      });
    // every proof chain of the wave at once (35 for 5 parties): their small
    // per-pair batches meet in the coalescers; 8 at a time measured 5% slower
    // with twice the narrow-geometry share (profiles/r04/keygen_tasks_ab/)
    run_bounded(tasks, tasks.size());
    (reshare ? rs_sessions : kg_sessions) += m;
    if (trace) {
      uint32_t* o = trace->data() + w * tw;
      o[0] = (uint32_t)(lo + ts);
      uint32_t* d = o + 1;
      for (size_t i = 0; i < n; ++i) {
        dln_digest(dln1[i][ts]).to_words(d, 8);
        dln_digest(dln2[i][ts]).to_words(d + 8, 8);
        mod_digest(mod[i][ts]).to_words(d + 16, 8);
        d += 24;
        for (size_t j = 0; j < n; ++j)
          if (j != i) {
            fac_digest(fac[i][j][ts]).to_words(d, 8);
            d += 8;
          }
      }
      *d = traced_ok.load();
    }
    std::lock_guard<std::mutex> lk(tm);
    max_wave = std::max(max_wave, now() - w0);
    (reshare ? rs_wave_s : kg_wave_s) += now() - w0;
    // MPCX_PROGRESS=1: a line on stderr every 10 finished waves and at the end
    // (long runs are otherwise silent for minutes)
    static const bool progress = [] {
      const char* e = std::getenv("MPCX_PROGRESS");
      return e && e[0] == '1';
    }();
    const size_t finished = ++waves_done;
    if (progress && (finished % 10 == 0 || finished == n_waves))
      std::fprintf(stderr, "[keygenload] %zu/%zu waves done (last %.1f s)\n", finished, n_waves, now() - w0);
  };

  Engine::get().reset_busy();
  const double t0 = now();
  {  // kWavesInFlight workers take the waves in order (MPCX_KEYGEN_WAVES: A/B runs)
    static const size_t in_flight = [] {
      const char* e = std::getenv("MPCX_KEYGEN_WAVES");
      const int v = e ? std::atoi(e) : 0;
      return v > 0 ? (size_t)v : kWavesInFlight;
    }();
    std::atomic<size_t> next{0};
    std::vector<std::function<void()>> workers;
    for (size_t k = 0; k < std::min(in_flight, n_waves); ++k)
      workers.push_back([&] {
        for (;;) {
          const size_t w = next.fetch_add(1);
          if (w >= n_waves) return;
          run_wave(w);
        }
      });
    run_bounded(workers, workers.size());
  }
  const double t2 = now();
  st.prove_s = std::max(0.0, last_prove - t0);  // until the last proof batch was done
  st.verify_s = t2 - std::max(t0, last_prove);  // verification tail after it
  st.total_s = t2 - t0;
  st.max_wave_s = max_wave;
  st.failures = fails.load();
  st.engine_busy_s = Engine::get().busy_seconds();
  st.alg_macs = Engine::get().alg_macs();
  st.keygen_sessions = kg_sessions.load();
  st.reshare_sessions = rs_sessions.load();
  st.keygen_wave_s = kg_wave_s;
  st.reshare_wave_s = rs_wave_s;
  st.vss_checks = vss_checks.load();
  st.vss_failures = vss_fails.load();
  return st;
}

}  // namespace mpcx::host::keygenload
