// capi.cpp -- extern "C" surface of libmpcx_host.so (include/mpcx_host.h):
// the C++ mirror of the reference interfaces, callable over any FFI (the
// parity tests drive it through ctypes; a Go integration would call
// libmpcx.so directly and keep its own ModInt/paillier code).
#include "mpcx_host.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <functional>
#include <string>
#include <vector>

#include "engine.hpp"
#include "gorand.hpp"
#include "hostprof.hpp"
#include "modint.hpp"
#include "paillier.hpp"
#include "mta.hpp"
#include "proofs.hpp"
#include "safeprime.hpp"
#include "keygenload.hpp"
#include "signing.hpp"

using namespace mpcx::host;

namespace {
thread_local std::string g_herr;

int guard(const std::function<void()>& f) {
  try {
    f();
    return MPCX_OK;
  } catch (const EngineError& e) {
    g_herr = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_herr = e.what();
    return MPCX_EINVAL;
  }
}

std::vector<Int> ints(const uint32_t* w, uint32_t nw, const uint8_t* neg, uint32_t count) {
  std::vector<Int> v(count);
  for (uint32_t i = 0; i < count; ++i) v[i] = Int(Nat::from_words(w + (size_t)i * nw, nw), neg ? neg[i] != 0 : false);
  return v;
}

std::vector<Nat> nats(const uint32_t* w, uint32_t nw, uint32_t count) {
  std::vector<Nat> v(count);
  for (uint32_t i = 0; i < count; ++i) v[i] = Nat::from_words(w + (size_t)i * nw, nw);
  return v;
}

void store(const std::vector<Nat>& v, uint32_t* out, uint32_t ow) {
  for (size_t i = 0; i < v.size(); ++i) v[i].to_words(out + i * ow, ow);
}

RandFn rand_from(uint64_t seed, mpcxh_rand_fn fn, void* ctx, CounterDRBG* drbg) {
  if (fn) return [fn, ctx](uint8_t* b, size_t n) { fn(ctx, b, n); };
  *drbg = CounterDRBG(seed);
  return drbg->fn();
}
Nat nat_or0(const uint32_t* p, uint32_t w) { return p ? Nat::from_words(p, w) : Nat(); }

paillier::PrivateKey paillier_from(const mpcxh_paillier_t* k, uint32_t w) {
  if (!k || !k->N) throw std::invalid_argument("null Paillier key");
  paillier::PrivateKey sk;
  sk.pub.N = Nat::from_words(k->N, w);
  sk.LambdaN = nat_or0(k->LambdaN, w);
  sk.P = nat_or0(k->P, w);
  sk.Q = nat_or0(k->Q, w);
  if (!sk.P.is_zero() && !sk.Q.is_zero()) sk.PhiN = (sk.P - Nat(1)) * (sk.Q - Nat(1));
  return sk;
}

mta::DLNParams dln_from(const mpcxh_dln_t* d, uint32_t w) {
  if (!d || !d->NTilde || !d->h1 || !d->h2) throw std::invalid_argument("null DLN parameters");
  mta::DLNParams p;
  p.NTilde = Nat::from_words(d->NTilde, w);
  p.h1 = Nat::from_words(d->h1, w);
  p.h2 = Nat::from_words(d->h2, w);
  p.P = nat_or0(d->P, w);
  p.Q = nat_or0(d->Q, w);
  return p;
}

void check_width(uint32_t w) {
  if (w < 128) throw std::invalid_argument("MtA integer width must be >= 128 words (N^2)");
}

// Per-session io.Readers: the caller's callback, or a CounterDRBG owned by
// `drbgs` (reserved up front: the RandFns point into it).
std::vector<RandFn> readers(const mpcxh_reader_t* rd, uint32_t count, std::vector<CounterDRBG>* drbgs) {
  if (!rd && count) throw std::invalid_argument("null readers");
  drbgs->clear();
  drbgs->reserve(count);
  std::vector<RandFn> r;
  r.reserve(count);
  for (uint32_t i = 0; i < count; ++i) {
    if (rd[i].fn) {
      const mpcxh_rand_fn fn = rd[i].fn;
      void* ctx = rd[i].ctx;
      r.push_back([fn, ctx](uint8_t* b, size_t n) { fn(ctx, b, n); });
    } else {
      drbgs->emplace_back(rd[i].seed);
      r.push_back(drbgs->back().fn());
    }
  }
  return r;
}

std::vector<mta::Bytes> sessions_from(const uint8_t* s, uint32_t len, uint32_t count) {
  std::vector<mta::Bytes> v(count);
  for (uint32_t i = 0; i < count; ++i) v[i].assign(s + (size_t)i * len, s + (size_t)(i + 1) * len);
  return v;
}

std::vector<secp::Affine> points_from(const uint32_t* p, uint32_t count) {
  std::vector<secp::Affine> v(count);
  for (uint32_t i = 0; i < count; ++i) {
    v[i].x = secp::NatToFe(Nat::from_words(p + (size_t)i * 16, 8));
    v[i].y = secp::NatToFe(Nat::from_words(p + (size_t)i * 16 + 8, 8));
    v[i].inf = false;
  }
  return v;
}

void put(const Nat& v, uint32_t* out, uint32_t w) { v.to_words(out, w); }

std::vector<mta::RangeProofAlice> range_from(const uint32_t* p, uint32_t count, uint32_t w) {
  std::vector<mta::RangeProofAlice> v(count);
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t* b = p + (size_t)i * MPCXH_RANGE_PROOF_FIELDS * w;
    Nat* f[] = {&v[i].Z, &v[i].U, &v[i].W, &v[i].S, &v[i].S1, &v[i].S2};
    for (int k = 0; k < MPCXH_RANGE_PROOF_FIELDS; ++k) *f[k] = Nat::from_words(b + (size_t)k * w, w);
  }
  return v;
}

void range_to(const std::vector<mta::RangeProofAlice>& v, uint32_t* p, uint32_t w) {
  for (size_t i = 0; i < v.size(); ++i) {
    uint32_t* b = p + i * MPCXH_RANGE_PROOF_FIELDS * w;
    const Nat* f[] = {&v[i].Z, &v[i].U, &v[i].W, &v[i].S, &v[i].S1, &v[i].S2};
    for (int k = 0; k < MPCXH_RANGE_PROOF_FIELDS; ++k) put(*f[k], b + (size_t)k * w, w);
  }
}

std::vector<mta::ProofBob> bob_from(const uint32_t* p, uint32_t count, uint32_t w, bool wc) {
  std::vector<mta::ProofBob> v(count);
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t* b = p + (size_t)i * MPCXH_PROOF_BOB_FIELDS * w;
    Nat* f[] = {&v[i].Z, &v[i].ZPrm, &v[i].T, &v[i].V, &v[i].W, &v[i].S, &v[i].S1, &v[i].S2, &v[i].T1, &v[i].T2};
    for (int k = 0; k < 10; ++k) *f[k] = Nat::from_words(b + (size_t)k * w, w);
    if (wc) {
      const Nat ux = Nat::from_words(b + (size_t)10 * w, w), uy = Nat::from_words(b + (size_t)11 * w, w);
      v[i].U.x = secp::NatToFe(ux);
      v[i].U.y = secp::NatToFe(uy);
      v[i].U.inf = ux.bit_len() > 256 || uy.bit_len() > 256;  // off the field: fails IsOnCurve
      if (v[i].U.inf) v[i].U.x = v[i].U.y = secp::Fe{};
    }
  }
  return v;
}

void bob_to(const std::vector<mta::ProofBob>& v, uint32_t* p, uint32_t w) {
  for (size_t i = 0; i < v.size(); ++i) {
    uint32_t* b = p + i * MPCXH_PROOF_BOB_FIELDS * w;
    const Nat* f[] = {&v[i].Z, &v[i].ZPrm, &v[i].T, &v[i].V, &v[i].W, &v[i].S, &v[i].S1, &v[i].S2, &v[i].T1, &v[i].T2};
    for (int k = 0; k < 10; ++k) put(*f[k], b + (size_t)k * w, w);
    put(v[i].U.inf ? Nat() : secp::FeToNat(v[i].U.x), b + (size_t)10 * w, w);
    put(v[i].U.inf ? Nat() : secp::FeToNat(v[i].U.y), b + (size_t)11 * w, w);
  }
}
}  // namespace

extern "C" {

const char* mpcxh_last_error(void) { return g_herr.c_str(); }

int mpcxh_init(int device) {
  return guard([&] { Engine::get().init(device); });
}

int mpcxh_init_devices(int n_gpus) {
  return guard([&] { Engine::get().init_devices(n_gpus); });
}

int mpcxh_modint_exp_batch(const uint32_t* m, uint32_t mw, uint32_t count, const uint32_t* xs, uint32_t xw,
                           const uint8_t* x_neg, const uint32_t* ys, uint32_t yw, const uint8_t* y_neg,
                           int y_shared, uint32_t* out, uint32_t ow, uint8_t* ok) {
  return guard([&] {
    ModInt mi(Nat::from_words(m, mw));
    std::vector<Nat> z;
    std::vector<uint8_t> okv;
    mi.ExpBatch(ints(xs, xw, x_neg, count), ints(ys, yw, y_neg, y_shared ? 1 : count), &z, &okv);
    store(z, out, ow);
    std::memcpy(ok, okv.data(), count);
  });
}

int mpcxh_paillier_encrypt_batch(const uint32_t* N, uint32_t nw, uint32_t count, const uint32_t* m, uint32_t mw,
                                 const uint8_t* m_neg, const uint32_t* r, uint32_t rw, uint32_t* c, uint32_t cw,
                                 uint8_t* err) {
  return guard([&] {
    paillier::PublicKey pk{Nat::from_words(N, nw)};
    std::vector<Nat> out;
    std::vector<uint8_t> e;
    pk.EncryptBatch(ints(m, mw, m_neg, count), nats(r, rw, count), &out, &e);
    store(out, c, cw);
    std::memcpy(err, e.data(), count);
  });
}

int mpcxh_paillier_homomult_batch(const uint32_t* N, uint32_t nw, uint32_t count, const uint32_t* m, uint32_t mw,
                                  const uint8_t* m_neg, const uint32_t* c1, uint32_t c1w, const uint8_t* c1_neg,
                                  uint32_t* out, uint32_t ow, uint8_t* err) {
  return guard([&] {
    paillier::PublicKey pk{Nat::from_words(N, nw)};
    std::vector<Nat> o;
    std::vector<uint8_t> e;
    pk.HomoMultBatch(ints(m, mw, m_neg, count), ints(c1, c1w, c1_neg, count), &o, &e);
    store(o, out, ow);
    std::memcpy(err, e.data(), count);
  });
}

int mpcxh_paillier_homoadd_batch(const uint32_t* N, uint32_t nw, uint32_t count, const uint32_t* c1, uint32_t c1w,
                                 const uint8_t* c1_neg, const uint32_t* c2, uint32_t c2w, const uint8_t* c2_neg,
                                 uint32_t* out, uint32_t ow, uint8_t* err) {
  return guard([&] {
    paillier::PublicKey pk{Nat::from_words(N, nw)};
    std::vector<Nat> o;
    std::vector<uint8_t> e;
    pk.HomoAddBatch(ints(c1, c1w, c1_neg, count), ints(c2, c2w, c2_neg, count), &o, &e);
    store(o, out, ow);
    std::memcpy(err, e.data(), count);
  });
}

int mpcxh_paillier_decrypt_batch(const uint32_t* N, uint32_t nw, const uint32_t* lambda, uint32_t lw,
                                 const uint32_t* P, uint32_t pw, const uint32_t* Q, uint32_t qw, uint32_t count,
                                 const uint32_t* c, uint32_t cw, const uint8_t* c_neg, uint32_t* m, uint32_t mw,
                                 uint8_t* err) {
  return guard([&] {
    paillier::PrivateKey sk;
    sk.pub.N = Nat::from_words(N, nw);
    sk.LambdaN = Nat::from_words(lambda, lw);
    sk.P = Nat::from_words(P, pw);
    sk.Q = Nat::from_words(Q, qw);
    // a key without its factors (P = Q = 0) decrypts by tss-lib's lambda formula
    if (!sk.P.is_zero() && !sk.Q.is_zero()) sk.PhiN = (sk.P - Nat(1)) * (sk.Q - Nat(1));
    std::vector<Nat> o;
    std::vector<uint8_t> e;
    sk.DecryptBatch(ints(c, cw, c_neg, count), &o, &e);
    store(o, m, mw);
    std::memcpy(err, e.data(), count);
  });
}

namespace {
void put_stats(const SafePrimeStats& st, uint64_t* out) {
  if (!out) return;
  out[0] = st.candidates;
  out[1] = st.sieved_out;
  out[2] = st.fermat_tests;
  out[3] = st.mr_tests;
  out[4] = (uint64_t)(st.seconds * 1e6);
  out[5] = st.lucas_tests;
}
}  // namespace

int mpcxh_safe_primes(int bit_len, int num, uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx, uint32_t* p_out,
                      uint32_t* q_out, uint32_t words, uint64_t* index_out, uint64_t* stats_out) {
  return guard([&] {
    CounterDRBG drbg(seed);
    // CounterDRBG streams are drawn on the GPU; a caller's reader on the host
    Stream src = rand_fn ? Stream(rand_from(seed, rand_fn, rand_ctx, &drbg)) : Stream(&drbg);
    SafePrimeStats st;
    auto v = GetRandomSafePrimes(bit_len, num, src, &st);
    for (int i = 0; i < num; ++i) {
      v[i].p.to_words(p_out + (size_t)i * words, words);
      v[i].q.to_words(q_out + (size_t)i * words, words);
      if (index_out) index_out[i] = v[i].index;
    }
    put_stats(st, stats_out);
  });
}

int mpcxh_safe_prime_batch(int bit_len, uint64_t seed, uint64_t batch_no, uint32_t batch, uint32_t max_out,
                           uint32_t* p_out, uint32_t* q_out, uint32_t words, uint64_t* index_out,
                           uint32_t* n_found, uint64_t* stats_out) {
  return guard([&] {
    if (!n_found) throw std::invalid_argument("n_found is NULL");
    SafePrimeStats st;
    auto v = SafePrimeBatch(bit_len, seed, batch_no, batch, &st);
    const uint32_t n = (uint32_t)std::min<size_t>(v.size(), max_out);
    for (uint32_t i = 0; i < n; ++i) {
      v[i].p.to_words(p_out + (size_t)i * words, words);
      v[i].q.to_words(q_out + (size_t)i * words, words);
      if (index_out) index_out[i] = v[i].index;
    }
    *n_found = n;
    put_stats(st, stats_out);
  });
}

int mpcxh_generate_preparams(uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx, uint32_t* out, uint64_t* stats_out) {
  return guard([&] {
    CounterDRBG drbg(seed);
    Stream src = rand_fn ? Stream(rand_from(seed, rand_fn, rand_ctx, &drbg)) : Stream(&drbg);
    SafePrimeStats st;
    LocalPreParams pp = GeneratePreParams(src, &st);
    const Nat* f[MPCXH_PREPARAM_FIELDS] = {&pp.PaillierSK.pub.N, &pp.PaillierSK.LambdaN, &pp.PaillierSK.PhiN,
                                           &pp.PaillierSK.P,     &pp.PaillierSK.Q,       &pp.NTildei,
                                           &pp.H1i,              &pp.H2i,                &pp.Alpha,
                                           &pp.Beta,             &pp.P,                  &pp.Q};
    for (int i = 0; i < MPCXH_PREPARAM_FIELDS; ++i) f[i]->to_words(out + (size_t)i * 64, 64);
    put_stats(st, stats_out);
  });
}

int mpcxh_probably_prime_batch(uint32_t count, const uint32_t* n, uint32_t words, int reps, uint8_t* ok) {
  return guard([&] {
    if (reps < 0) throw std::invalid_argument("negative reps");
    const auto v = ProbablyPrimeBatch(nats(n, words, count), reps);
    std::memcpy(ok, v.data(), count);
  });
}

int mpcxh_coprime_batch(uint32_t count, const uint32_t* x, const uint32_t* m, uint32_t words, uint8_t* ok) {
  return guard([&] {
    const auto xs = nats(x, words, count), ms = nats(m, words, count);
    parallel_for(count, [&](size_t i) {
      if (!ms[i].is_odd()) throw std::invalid_argument("coprime_batch: even modulus");
      ok[i] = coprime_odd(xs[i], ms[i]) ? 1 : 0;
    });
  });
}

int mpcxh_host_threads(int* threads, int* usable) {
  return guard([&] {
    if (threads) *threads = host_threads();
    if (usable) *usable = usable_cpus();
  });
}

int mpcxh_pinned_pool_stats(uint64_t* held_bytes, uint64_t* peak_in_use_bytes, uint64_t* fallbacks,
                            uint64_t* fallback_bytes) {
  return guard([&] { pinned_pool_stats(held_bytes, peak_in_use_bytes, fallbacks, fallback_bytes); });
}

int mpcxh_nat_arith(int op, const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* out,
                    uint32_t nout, uint32_t* out_words) {
  return guard([&] {
    if (!out || !out_words || (na && !a) || (nb && !b)) throw std::invalid_argument("null buffer");
    const Nat x = Nat::from_words(a, na), y = Nat::from_words(b, nb);
    Nat r;
    switch (op) {
      case 0: r = x * y; break;
      case 1: r = x / y; break;
      case 2: r = x % y; break;
      case 3:
        if (!mod_inverse(Int(x), y, &r)) throw EngineError(MPCX_EINVAL, "not invertible");
        break;
      case 4: r = gcd(x, y); break;
      default: throw std::invalid_argument("nat_arith: unknown op");
    }
    if (r.words() > nout) throw std::length_error("nat_arith: output buffer too small");
    r.to_words(out, nout);
    *out_words = (uint32_t)r.words();
  });
}

int mpcxh_pool_selftest(uint32_t tasks, uint32_t outer, uint32_t inner, uint64_t* sum) {
  return guard([&] {
    if (!sum) throw std::invalid_argument("null sum");
    // `tasks` threads each run a parallel loop of `outer` indices whose every
    // index runs a nested loop of `inner` indices (the drivers' shape: protocol
    // tasks issuing parallel loops from inside parallel loops)
    std::atomic<uint64_t> acc{0};
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < tasks; ++t)
      th.emplace_back([&, t] {
        parallel_for(outer, [&](size_t o) {
          std::atomic<uint64_t> part{0};
          parallel_for(inner, [&](size_t i) { part += (uint64_t)(t + 1) * (o + 1) * (i + 1); });
          acc += part.load();
        });
      });
    for (auto& x : th) x.join();
    *sum = acc.load();
  });
}

int mpcxh_profile_report(char* buf, size_t cap, int reset) {
  return guard([&] {
    if (!buf || !cap) throw std::invalid_argument("null buffer");
    const std::string r = prof::report();
    const size_t n = std::min(cap - 1, r.size());
    std::memcpy(buf, r.data(), n);
    buf[n] = 0;
    if (reset) prof::reset();
  });
}

int mpcxh_candidate_from_bytes(const uint8_t* bytes, size_t n, int q_bit_len, uint32_t* q_out, uint32_t words) {
  return guard([&] { CandidateFromBytes(bytes, n, q_bit_len).to_words(q_out, words); });
}

int mpcxh_go_rand_int63(int64_t seed, uint32_t count, int64_t* out) {
  return guard([&] {
    if (!out && count) throw std::invalid_argument("null out");
    GoRand r(seed);
    for (uint32_t i = 0; i < count; ++i) out[i] = r.Int63();
  });
}

int mpcxh_go_mr_bases(const uint32_t* n, uint32_t w, uint32_t reps, uint32_t* out) {
  return guard([&] {
    const Nat x = Nat::from_words(n, w);
    if (!x.is_odd() || x.bit_len() < 3 || x == Nat(3)) throw std::invalid_argument("need odd n > 3");
    const auto bs = GoMillerRabinBases(x, (int)reps);
    for (uint32_t i = 0; i < reps; ++i) bs[i].to_words(out + (size_t)i * w, w);
  });
}

int mpcxh_drbg_read(uint64_t seed, uint8_t* out, size_t n) {
  return guard([&] {
    CounterDRBG d(seed);
    d.read(out, n);
  });
}

// ------------------------------------------------------------------ MtA
int mpcxh_mta_alice_init_batch(uint32_t w, const mpcxh_paillier_t* pkA, const mpcxh_dln_t* dlnB, uint32_t count,
                               const uint32_t* a, const mpcxh_reader_t* seeds, uint32_t* cA, uint32_t* pf,
                               uint8_t* err) {
  return guard([&] {
    check_width(w);
    const auto sk = paillier_from(pkA, w);
    const auto dln = dln_from(dlnB, w);
    std::vector<CounterDRBG> drbgs;
    const auto rd = readers(seeds, count, &drbgs);
    std::vector<Nat> c;
    std::vector<mta::RangeProofAlice> p;
    std::vector<uint8_t> e;
    // a key with its factors (the caller is Alice): the CRT form
    mta::AliceInitBatch(sk.pub, nats(a, w, count), dln, rd, &c, &p, &e, sk.P.is_zero() ? nullptr : &sk);
    store(c, cA, w);
    range_to(p, pf, w);
    std::memcpy(err, e.data(), count);
  });
}

int mpcxh_mta_verify_range_alice_batch(uint32_t w, const mpcxh_paillier_t* pk, const mpcxh_dln_t* dln,
                                       uint32_t count, const uint32_t* c, const uint32_t* pf, uint8_t* ok) {
  return guard([&] {
    check_width(w);
    const auto sk = paillier_from(pk, w);
    const auto ok_v = mta::VerifyRangeAliceBatch(sk.pub, dln_from(dln, w), nats(c, w, count), range_from(pf, count, w));
    std::memcpy(ok, ok_v.data(), count);
  });
}

int mpcxh_mta_bob_mid_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const mpcxh_paillier_t* pkA,
                            const mpcxh_dln_t* dlnA, const mpcxh_dln_t* dlnB, uint32_t count, const uint32_t* pfA,
                            const uint32_t* b, const uint32_t* cA, const uint32_t* B,
                            const mpcxh_reader_t* seeds, uint32_t* beta, uint32_t* cB, uint32_t* betaPrm,
                            uint32_t* pfB, uint8_t* err) {
  return guard([&] {
    check_width(w);
    const auto sk = paillier_from(pkA, w);
    std::vector<CounterDRBG> drbgs;
    const auto rd = readers(seeds, count, &drbgs);
    std::vector<secp::Affine> Bv;
    if (B) Bv = points_from(B, count);
    std::vector<mta::BobMidResult> out;
    std::vector<uint8_t> e;
    mta::BobMidBatch(sessions_from(sessions, session_len, count), sk.pub, range_from(pfA, count, w), nats(b, w, count),
                     nats(cA, w, count), dln_from(dlnA, w), dln_from(dlnB, w), B ? &Bv : nullptr, rd, &out, &e);
    std::vector<mta::ProofBob> pfs(count);
    for (uint32_t i = 0; i < count; ++i) {
      put(out[i].beta, beta + (size_t)i * w, w);
      put(out[i].cB, cB + (size_t)i * w, w);
      put(out[i].betaPrm, betaPrm + (size_t)i * w, w);
      pfs[i] = out[i].pf;
    }
    bob_to(pfs, pfB, w);
    std::memcpy(err, e.data(), count);
  });
}

int mpcxh_mta_verify_bob_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const mpcxh_paillier_t* pk,
                               const mpcxh_dln_t* dln, uint32_t count, const uint32_t* c1, const uint32_t* c2,
                               const uint32_t* pfB, const uint32_t* X, uint8_t* ok) {
  return guard([&] {
    check_width(w);
    const auto sk = paillier_from(pk, w);
    std::vector<secp::Affine> Xv;
    if (X) Xv = points_from(X, count);
    const bool own = !sk.P.is_zero() && !sk.Q.is_zero();
    const auto ok_v = mta::VerifyBobBatch(sessions_from(sessions, session_len, count), sk.pub, dln_from(dln, w),
                                          nats(c1, w, count), nats(c2, w, count), bob_from(pfB, count, w, X != nullptr),
                                          X ? &Xv : nullptr, own ? &sk : nullptr);
    std::memcpy(ok, ok_v.data(), count);
  });
}

int mpcxh_mta_alice_end_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const mpcxh_paillier_t* skA,
                              const mpcxh_dln_t* dlnA, uint32_t count, const uint32_t* pfB, const uint32_t* cA,
                              const uint32_t* cB, const uint32_t* B, uint32_t* alpha, uint8_t* err) {
  return guard([&] {
    check_width(w);
    const auto sk = paillier_from(skA, w);
    if (sk.LambdaN.is_zero() || sk.P.is_zero() || sk.Q.is_zero())
      throw std::invalid_argument("AliceEnd needs the private key (LambdaN, P, Q)");
    std::vector<secp::Affine> Bv;
    if (B) Bv = points_from(B, count);
    std::vector<Nat> al;
    std::vector<uint8_t> e;
    mta::AliceEndBatch(sessions_from(sessions, session_len, count), sk, bob_from(pfB, count, w, B != nullptr),
                       dln_from(dlnA, w), nats(cA, w, count), nats(cB, w, count), B ? &Bv : nullptr, &al, &e);
    store(al, alpha, w);
    std::memcpy(err, e.data(), count);
  });
}

static void bob_results_out(const std::vector<mta::BobMidResult>& out, uint32_t w, uint32_t* beta, uint32_t* cB,
                            uint32_t* betaPrm, uint32_t* pfB) {
  std::vector<mta::ProofBob> pfs(out.size());
  for (size_t i = 0; i < out.size(); ++i) {
    put(out[i].beta, beta + i * w, w);
    put(out[i].cB, cB + i * w, w);
    put(out[i].betaPrm, betaPrm + i * w, w);
    pfs[i] = out[i].pf;
  }
  bob_to(pfs, pfB, w);
}

int mpcxh_mta_bob_mid_pair_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len,
                                 const mpcxh_paillier_t* pkA, const mpcxh_dln_t* dlnA, const mpcxh_dln_t* dlnB,
                                 uint32_t count, const uint32_t* pfA, const uint32_t* cA, const uint32_t* b,
                                 const mpcxh_reader_t* rdr, const uint32_t* bwc, const uint32_t* Bwc,
                                 const mpcxh_reader_t* rdr_wc, uint32_t* beta, uint32_t* cB, uint32_t* betaPrm,
                                 uint32_t* pfB, uint8_t* err, uint32_t* beta_wc, uint32_t* cB_wc,
                                 uint32_t* betaPrm_wc, uint32_t* pfB_wc, uint8_t* err_wc) {
  return guard([&] {
    check_width(w);
    if (!Bwc) throw std::invalid_argument("BobMidPair: Bwc is required");
    const auto sk = paillier_from(pkA, w);
    std::vector<CounterDRBG> d1, d2;
    const auto rd = readers(rdr, count, &d1);
    const auto rdwc = readers(rdr_wc, count, &d2);
    // one callback reader object for both halves of a session: the halves run
    // one after the other (the reader is never called concurrently for a session)
    bool shared = false;
    for (uint32_t i = 0; i < count && !shared; ++i)
      shared = rdr[i].fn && rdr[i].fn == rdr_wc[i].fn && rdr[i].ctx == rdr_wc[i].ctx;
    std::vector<mta::BobMidResult> out, outwc;
    std::vector<uint8_t> e, ewc;
    mta::BobMidPairBatch(sessions_from(sessions, session_len, count), sk.pub, range_from(pfA, count, w),
                         nats(b, w, count), nats(bwc, w, count), nats(cA, w, count), dln_from(dlnA, w),
                         dln_from(dlnB, w), points_from(Bwc, count), rd, rdwc, &out, &outwc, &e, &ewc, shared);
    bob_results_out(out, w, beta, cB, betaPrm, pfB);
    bob_results_out(outwc, w, beta_wc, cB_wc, betaPrm_wc, pfB_wc);
    std::memcpy(err, e.data(), count);
    std::memcpy(err_wc, ewc.data(), count);
  });
}

int mpcxh_mta_alice_end_pair_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len,
                                   const mpcxh_paillier_t* skA, const mpcxh_dln_t* dlnA, uint32_t count,
                                   const uint32_t* cA, const uint32_t* pfB, const uint32_t* cB,
                                   const uint32_t* pfB_wc, const uint32_t* cB_wc, const uint32_t* Bwc,
                                   uint32_t* alpha, uint8_t* err, uint32_t* mu, uint8_t* err_wc) {
  return guard([&] {
    check_width(w);
    if (!Bwc) throw std::invalid_argument("AliceEndPair: Bwc is required");
    const auto sk = paillier_from(skA, w);
    if (sk.LambdaN.is_zero() || sk.P.is_zero() || sk.Q.is_zero())
      throw std::invalid_argument("AliceEnd needs the private key (LambdaN, P, Q)");
    std::vector<Nat> al, m;
    std::vector<uint8_t> e, ewc;
    mta::AliceEndPairBatch(sessions_from(sessions, session_len, count), sk, bob_from(pfB, count, w, false),
                           bob_from(pfB_wc, count, w, true), dln_from(dlnA, w), nats(cA, w, count),
                           nats(cB, w, count), nats(cB_wc, w, count), points_from(Bwc, count), &al, &m, &e, &ewc);
    store(al, alpha, w);
    store(m, mu, w);
    std::memcpy(err, e.data(), count);
    std::memcpy(err_wc, ewc.data(), count);
  });
}

// ------------------------------------------------------------------ test hooks
int mpcxh_sha512_256i(const uint8_t* tag, size_t tag_len, uint32_t count, const uint32_t* ints, uint32_t w,
                      uint8_t* digest32) {
  return guard([&] {
    const std::vector<Nat> v = nats(ints, w, count);
    std::vector<const Nat*> ptrs;
    for (const auto& x : v) ptrs.push_back(&x);
    const Nat h = tag ? SHA512_256i_TAGGED(std::vector<uint8_t>(tag, tag + tag_len), ptrs) : SHA512_256i(ptrs);
    std::vector<uint8_t> b = h.to_bytes_be();
    std::memset(digest32, 0, 32);
    std::memcpy(digest32 + (32 - b.size()), b.data(), b.size());
  });
}

static void point_out(const secp::Affine& p, uint32_t* out16) {
  std::memset(out16, 0, 16 * sizeof(uint32_t));
  if (p.inf) return;
  secp::FeToNat(p.x).to_words(out16, 8);
  secp::FeToNat(p.y).to_words(out16 + 8, 8);
}

int mpcxh_secp_scalar_base_mult(const uint32_t* k, uint32_t w, uint32_t* out16) {
  return guard([&] { point_out(secp::ScalarBaseMult(Nat::from_words(k, w)), out16); });
}

int mpcxh_secp_scalar_mult(const uint32_t* p16, const uint32_t* k, uint32_t w, uint32_t* out16) {
  return guard([&] {
    const auto P = points_from(p16, 1)[0];
    point_out(secp::ScalarMult(P, Nat::from_words(k, w)), out16);
  });
}

int mpcxh_secp_lincomb(const uint32_t* u1, const uint32_t* p16, const uint32_t* u2, uint32_t w, uint32_t* out16) {
  return guard([&] {
    const auto P = points_from(p16, 1)[0];
    point_out(secp::LinComb(Nat::from_words(u1, w), P, Nat::from_words(u2, w)), out16);
  });
}

int mpcxh_random_draws(uint64_t seed, const uint32_t* less_than, uint32_t w, int relprime, uint32_t count,
                       uint32_t* out) {
  return guard([&] {
    CounterDRBG d(seed);
    const RandFn r = d.fn();
    const Nat lt = Nat::from_words(less_than, w);
    for (uint32_t i = 0; i < count; ++i)
      (relprime ? GetRandomPositiveRelativelyPrimeInt(r, lt) : GetRandomPositiveInt(r, lt)).to_words(out + (size_t)i * w, w);
  });
}

int mpcxh_bench_signing(uint32_t w, const mpcxh_paillier_t* sks, const mpcxh_dln_t* dlns, uint32_t n_nodes,
                        uint32_t signers, uint32_t wallets, uint64_t seed, double* stats_out, uint32_t trace_wallets,
                        uint32_t* trace_out, int64_t tamper_wallet, int tamper_kind) {
  return guard([&] {
    check_width(w);
    if (!stats_out) throw std::invalid_argument("null stats_out");
    if (trace_wallets && !trace_out) throw std::invalid_argument("null trace_out");
    std::vector<signing::NodeKeys> nodes(n_nodes);
    for (uint32_t i = 0; i < n_nodes; ++i) {
      nodes[i].sk = paillier_from(&sks[i], w);
      nodes[i].dln = dln_from(&dlns[i], w);
    }
    std::vector<uint32_t> tr;
    const auto st =
        signing::RunSigning(nodes, (int)signers, wallets, seed, trace_wallets, &tr, tamper_wallet, tamper_kind);
    const double v[MPCXH_SIGNING_STATS] = {st.round1_s, st.round2_s, st.round3_s, st.total_s, (double)st.wallets,
                                           (double)st.sessions, (double)st.errors, (double)st.relation_failures,
                                           st.engine_busy_s, st.finalize_s, (double)st.signatures,
                                           (double)st.verified, st.alg_macs, (double)st.aborted};
    std::memcpy(stats_out, v, sizeof v);
    if (trace_wallets) std::memcpy(trace_out, tr.data(), tr.size() * sizeof(uint32_t));
  });
}

// ------------------------------------------------------------------ keygen proofs
static void check_pw(uint32_t w) {
  if (w < MPCXH_PROOF_WORDS) throw std::invalid_argument("proof integer width must be >= 160 words");
}
static Nat one_nat(const uint32_t* p, uint32_t w) {
  if (!p) throw std::invalid_argument("null integer");
  return Nat::from_words(p, w);
}

int mpcxh_dln_prove_batch(uint32_t w, const uint32_t* h1, const uint32_t* h2, const uint32_t* x, const uint32_t* p,
                          const uint32_t* q, const uint32_t* N, uint32_t count, const mpcxh_reader_t* seeds,
                          uint32_t* alpha, uint32_t* t) {
  return guard([&] {
    check_pw(w);
    std::vector<CounterDRBG> drbgs;
    const auto rd = readers(seeds, count, &drbgs);
    const auto pf = proofs::DLNProveBatch(one_nat(h1, w), one_nat(h2, w), one_nat(x, w), one_nat(p, w),
                                          one_nat(q, w), one_nat(N, w), rd);
    for (uint32_t i = 0; i < count; ++i)
      for (int k = 0; k < proofs::kDLNIterations; ++k) {
        const size_t off = ((size_t)i * proofs::kDLNIterations + k) * w;
        put(pf[i].Alpha[k], alpha + off, w);
        put(pf[i].T[k], t + off, w);
      }
  });
}

int mpcxh_dln_verify_batch(uint32_t w, const uint32_t* h1, const uint32_t* h2, const uint32_t* N, uint32_t count,
                           const uint32_t* alpha, const uint32_t* t, uint8_t* ok) {
  return guard([&] {
    check_pw(w);
    std::vector<proofs::DLNProof> pf(count);
    for (uint32_t i = 0; i < count; ++i) {
      pf[i].Alpha = nats(alpha + (size_t)i * proofs::kDLNIterations * w, w, proofs::kDLNIterations);
      pf[i].T = nats(t + (size_t)i * proofs::kDLNIterations * w, w, proofs::kDLNIterations);
    }
    const auto v = proofs::DLNVerifyBatch(one_nat(h1, w), one_nat(h2, w), one_nat(N, w), pf);
    std::memcpy(ok, v.data(), count);
  });
}

int mpcxh_mod_prove_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N,
                          const uint32_t* P, const uint32_t* Q, uint32_t count, const mpcxh_reader_t* seeds,
                          uint32_t* W, uint32_t* X, uint32_t* A, uint32_t* B, uint32_t* Z) {
  return guard([&] {
    check_pw(w);
    std::vector<CounterDRBG> drbgs;
    const auto rd = readers(seeds, count, &drbgs);
    const auto pf = proofs::ModProveBatch(sessions_from(sessions, session_len, count), one_nat(N, w), one_nat(P, w),
                                          one_nat(Q, w), rd);
    for (uint32_t i = 0; i < count; ++i) {
      put(pf[i].W, W + (size_t)i * w, w);
      put(pf[i].A, A + (size_t)i * w, w);
      put(pf[i].B, B + (size_t)i * w, w);
      store(pf[i].X, X + (size_t)i * proofs::kModIterations * w, w);
      store(pf[i].Z, Z + (size_t)i * proofs::kModIterations * w, w);
    }
  });
}

int mpcxh_mod_verify_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N,
                           uint32_t count, const uint32_t* W, const uint32_t* X, const uint32_t* A, const uint32_t* B,
                           const uint32_t* Z, uint8_t* ok) {
  return guard([&] {
    check_pw(w);
    std::vector<proofs::ModProof> pf(count);
    for (uint32_t i = 0; i < count; ++i) {
      pf[i].W = Nat::from_words(W + (size_t)i * w, w);
      pf[i].A = Nat::from_words(A + (size_t)i * w, w);
      pf[i].B = Nat::from_words(B + (size_t)i * w, w);
      pf[i].X = nats(X + (size_t)i * proofs::kModIterations * w, w, proofs::kModIterations);
      pf[i].Z = nats(Z + (size_t)i * proofs::kModIterations * w, w, proofs::kModIterations);
    }
    const auto v = proofs::ModVerifyBatch(sessions_from(sessions, session_len, count), one_nat(N, w), pf);
    std::memcpy(ok, v.data(), count);
  });
}

int mpcxh_fac_prove_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N0,
                          const uint32_t* NCap, const uint32_t* s, const uint32_t* t, const uint32_t* N0p,
                          const uint32_t* N0q, uint32_t count, const mpcxh_reader_t* seeds, uint32_t* pf,
                          uint8_t* v_neg) {
  return guard([&] {
    check_pw(w);
    std::vector<CounterDRBG> drbgs;
    const auto rd = readers(seeds, count, &drbgs);
    const auto out = proofs::FacProveBatch(sessions_from(sessions, session_len, count), one_nat(N0, w),
                                           one_nat(NCap, w), one_nat(s, w), one_nat(t, w), one_nat(N0p, w),
                                           one_nat(N0q, w), rd);
    for (uint32_t i = 0; i < count; ++i) {
      uint32_t* b = pf + (size_t)i * MPCXH_FAC_FIELDS * w;
      const Nat* f[] = {&out[i].P, &out[i].Q, &out[i].A, &out[i].B, &out[i].T, &out[i].Sigma,
                        &out[i].Z1, &out[i].Z2, &out[i].W1, &out[i].W2, &out[i].V.mag};
      for (int k = 0; k < MPCXH_FAC_FIELDS; ++k) put(*f[k], b + (size_t)k * w, w);
      v_neg[i] = out[i].V.neg ? 1 : 0;
    }
  });
}

int mpcxh_fac_verify_batch(uint32_t w, const uint8_t* sessions, uint32_t session_len, const uint32_t* N0,
                           const uint32_t* NCap, const uint32_t* s, const uint32_t* t, uint32_t count,
                           const uint32_t* pf, const uint8_t* v_neg, uint8_t* ok) {
  return guard([&] {
    check_pw(w);
    std::vector<proofs::FacProof> in(count);
    for (uint32_t i = 0; i < count; ++i) {
      const uint32_t* b = pf + (size_t)i * MPCXH_FAC_FIELDS * w;
      Nat* f[] = {&in[i].P, &in[i].Q, &in[i].A, &in[i].B, &in[i].T, &in[i].Sigma,
                  &in[i].Z1, &in[i].Z2, &in[i].W1, &in[i].W2};
      for (int k = 0; k < 10; ++k) *f[k] = Nat::from_words(b + (size_t)k * w, w);
      in[i].V = Int(Nat::from_words(b + (size_t)10 * w, w), v_neg && v_neg[i]);
    }
    const auto v = proofs::FacVerifyBatch(sessions_from(sessions, session_len, count), one_nat(N0, w),
                                          one_nat(NCap, w), one_nat(s, w), one_nat(t, w), in);
    std::memcpy(ok, v.data(), count);
  });
}

}  // extern "C"

namespace {
keygenload::ProofStats bench_config5(uint32_t w, const mpcxh_party_t* parties, uint32_t n_parties, uint32_t sessions,
                                     uint64_t seed, uint32_t wave_sessions, int mix, uint32_t* trace_out,
                                     int64_t tamper = -1) {
  if (w < 64) throw std::invalid_argument("party integer width must be >= 64 words");
  if (!parties) throw std::invalid_argument("null argument");
  std::vector<keygenload::PartyKeys> ps(n_parties);
  for (uint32_t i = 0; i < n_parties; ++i) {
    const mpcxh_party_t& a = parties[i];
    if (!a.NTilde || !a.h1 || !a.h2 || !a.alpha || !a.beta || !a.p || !a.q)
      throw std::invalid_argument("null party field");
    ps[i].sk = paillier_from(&a.paillier, w);
    ps[i].NTilde = Nat::from_words(a.NTilde, w);
    ps[i].h1 = Nat::from_words(a.h1, w);
    ps[i].h2 = Nat::from_words(a.h2, w);
    ps[i].alpha = Nat::from_words(a.alpha, w);
    ps[i].beta = Nat::from_words(a.beta, w);
    ps[i].p = Nat::from_words(a.p, w);
    ps[i].q = Nat::from_words(a.q, w);
  }
  std::vector<uint32_t> tr;
  const auto st = keygenload::RunKeygenProofs(ps, sessions, seed, wave_sessions, trace_out ? &tr : nullptr, mix, tamper);
  if (trace_out) std::memcpy(trace_out, tr.data(), tr.size() * sizeof(uint32_t));
  return st;
}
void keygen_stats(const keygenload::ProofStats& st, double* v) {
  const double a[MPCXH_KEYGEN_RESHARE_STATS] = {
      st.prove_s, st.verify_s, st.total_s, (double)st.sessions, (double)st.parties, (double)st.proofs,
      (double)st.verifications, (double)st.failures, st.engine_busy_s, st.alg_macs, (double)st.waves,
      (double)st.wave_sessions, st.max_wave_s, (double)st.keygen_sessions, (double)st.reshare_sessions,
      st.keygen_wave_s, st.reshare_wave_s, (double)st.vss_checks, (double)st.vss_failures};
  std::memcpy(v, a, sizeof a);
}
}  // namespace

int mpcxh_bench_keygen_proofs(uint32_t w, const mpcxh_party_t* parties, uint32_t n_parties, uint32_t sessions,
                              uint64_t seed, uint32_t wave_sessions, double* stats_out, uint32_t* trace_out) {
  return guard([&] {
    if (!stats_out) throw std::invalid_argument("null argument");
    const auto st = bench_config5(w, parties, n_parties, sessions, seed, wave_sessions, 0, trace_out);
    double v[MPCXH_KEYGEN_RESHARE_STATS];
    keygen_stats(st, v);
    std::memcpy(stats_out, v, MPCXH_KEYGEN_STATS * sizeof(double));
  });
}

int mpcxh_bench_keygen_reshare(uint32_t w, const mpcxh_party_t* parties, uint32_t n_parties, uint32_t sessions,
                               uint64_t seed, uint32_t wave_sessions, int reshare_mix, int64_t tamper_session,
                               double* stats_out, uint32_t* trace_out) {
  return guard([&] {
    if (!stats_out) throw std::invalid_argument("null argument");
    if (reshare_mix != 0 && reshare_mix != 1) throw std::invalid_argument("reshare_mix: 0 or 1");
    const auto st =
        bench_config5(w, parties, n_parties, sessions, seed, wave_sessions, reshare_mix, trace_out, tamper_session);
    keygen_stats(st, stats_out);
  });
}
