// capi.cpp -- extern "C" surface of libmpcx_host.so (include/mpcx_host.h):
// the C++ mirror of the reference interfaces, callable over any FFI (the
// parity tests drive it through ctypes; a Go integration would call
// libmpcx.so directly and keep its own ModInt/paillier code).
#include "mpcx_host.h"

#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "engine.hpp"
#include "modint.hpp"
#include "paillier.hpp"
#include "safeprime.hpp"

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
}  // namespace

extern "C" {

const char* mpcxh_last_error(void) { return g_herr.c_str(); }

int mpcxh_init(int device) {
  return guard([&] { Engine::get().init(device); });
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
    sk.PhiN = (sk.P - Nat(1)) * (sk.Q - Nat(1));
    std::vector<Nat> o;
    std::vector<uint8_t> e;
    sk.DecryptBatch(ints(c, cw, c_neg, count), &o, &e);
    store(o, m, mw);
    std::memcpy(err, e.data(), count);
  });
}

int mpcxh_safe_primes(int bit_len, int num, uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx, uint32_t* p_out,
                      uint32_t* q_out, uint32_t words, uint64_t* index_out, uint64_t* stats_out) {
  return guard([&] {
    CounterDRBG drbg(seed);
    RandFn rnd = rand_from(seed, rand_fn, rand_ctx, &drbg);
    SafePrimeStats st;
    auto v = GetRandomSafePrimes(bit_len, num, rnd, &st);
    for (int i = 0; i < num; ++i) {
      v[i].p.to_words(p_out + (size_t)i * words, words);
      v[i].q.to_words(q_out + (size_t)i * words, words);
      if (index_out) index_out[i] = v[i].index;
    }
    if (stats_out) {
      stats_out[0] = st.candidates;
      stats_out[1] = st.sieved_out;
      stats_out[2] = st.fermat_tests;
      stats_out[3] = st.mr_tests;
      stats_out[4] = (uint64_t)(st.seconds * 1e6);
    }
  });
}

int mpcxh_generate_preparams(uint64_t seed, mpcxh_rand_fn rand_fn, void* rand_ctx, uint32_t* out, uint64_t* stats_out) {
  return guard([&] {
    CounterDRBG drbg(seed);
    RandFn rnd = rand_from(seed, rand_fn, rand_ctx, &drbg);
    SafePrimeStats st;
    LocalPreParams pp = GeneratePreParams(rnd, &st);
    const Nat* f[MPCXH_PREPARAM_FIELDS] = {&pp.PaillierSK.pub.N, &pp.PaillierSK.LambdaN, &pp.PaillierSK.PhiN,
                                           &pp.PaillierSK.P,     &pp.PaillierSK.Q,       &pp.NTildei,
                                           &pp.H1i,              &pp.H2i,                &pp.Alpha,
                                           &pp.Beta,             &pp.P,                  &pp.Q};
    for (int i = 0; i < MPCXH_PREPARAM_FIELDS; ++i) f[i]->to_words(out + (size_t)i * 64, 64);
    if (stats_out) {
      stats_out[0] = st.candidates;
      stats_out[1] = st.sieved_out;
      stats_out[2] = st.fermat_tests;
      stats_out[3] = st.mr_tests;
      stats_out[4] = (uint64_t)(st.seconds * 1e6);
    }
  });
}

int mpcxh_candidate_from_bytes(const uint8_t* bytes, size_t n, int q_bit_len, uint32_t* q_out, uint32_t words) {
  return guard([&] { CandidateFromBytes(bytes, n, q_bit_len).to_words(q_out, words); });
}

int mpcxh_drbg_read(uint64_t seed, uint8_t* out, size_t n) {
  return guard([&] {
    CounterDRBG d(seed);
    d.read(out, n);
  });
}

}  // extern "C"
