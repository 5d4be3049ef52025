// signing.cpp -- see signing.hpp.
#include "signing.hpp"

#include <chrono>
#include <stdexcept>

namespace mpcx::host::signing {
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
mta::DLNParams public_dln(const mta::DLNParams& d) {
  mta::DLNParams p;
  p.NTilde = d.NTilde;
  p.h1 = d.h1;
  p.h2 = d.h2;
  return p;
}
}  // namespace

MtaStats RunSigningMtA(const std::vector<NodeKeys>& nodes, int signers, size_t wallets, uint64_t seed) {
  if (signers < 2 || (size_t)signers > nodes.size()) throw std::invalid_argument("signers must be in [2, nodes]");
  const Nat& q = mta::Q();
  const size_t S = (size_t)signers, Wn = wallets;
  MtaStats st;
  st.wallets = Wn;
  // per wallet and signer: k_i, gamma_i, w_i < q; W_i = w_i G; one session id per wallet
  std::vector<std::vector<Nat>> k(S, std::vector<Nat>(Wn)), g(S, std::vector<Nat>(Wn)), w(S, std::vector<Nat>(Wn));
  std::vector<std::vector<secp::Affine>> Wp(S, std::vector<secp::Affine>(Wn));
  std::vector<mta::Bytes> sess(Wn);
  parallel_for(Wn, [&](size_t wi) {
    CounterDRBG d(mix(seed, wi, 0xFFFF, 0));
    const RandFn r = d.fn();
    sess[wi].resize(32);
    r(sess[wi].data(), 32);
    for (size_t i = 0; i < S; ++i) {
      k[i][wi] = GetRandomPositiveInt(r, q);
      g[i][wi] = GetRandomPositiveInt(r, q);
      w[i][wi] = GetRandomPositiveInt(r, q);
      Wp[i][wi] = secp::ScalarBaseMult(w[i][wi]);
    }
  });
  struct Pair {
    size_t i, j;  // Alice i, Bob j
    std::vector<CounterDRBG> drbg_a, drbg_b, drbg_bwc;
    std::vector<RandFn> ra, rb, rbwc;
    std::vector<Nat> cA;
    std::vector<mta::RangeProofAlice> pfA;
    std::vector<mta::BobMidResult> bob, bobwc;
    std::vector<Nat> alpha, mu;
  };
  std::vector<Pair> pairs;
  for (size_t i = 0; i < S; ++i)
    for (size_t j = 0; j < S; ++j)
      if (i != j) pairs.push_back(Pair{i, j, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}});
  st.pairs = pairs.size();
  st.sessions = pairs.size() * Wn;
  for (auto& p : pairs) {
    p.drbg_a.reserve(Wn);
    p.drbg_b.reserve(Wn);
    p.drbg_bwc.reserve(Wn);
    for (size_t wi = 0; wi < Wn; ++wi) {
      p.drbg_a.emplace_back(mix(seed, wi, p.i * 16 + p.j, 1));
      p.drbg_b.emplace_back(mix(seed, wi, p.i * 16 + p.j, 2));
      p.drbg_bwc.emplace_back(mix(seed, wi, p.i * 16 + p.j, 3));
    }
    for (size_t wi = 0; wi < Wn; ++wi) {
      p.ra.push_back(p.drbg_a[wi].fn());
      p.rb.push_back(p.drbg_b[wi].fn());
      p.rbwc.push_back(p.drbg_bwc[wi].fn());
    }
  }
  std::vector<uint8_t> err;
  const double t0 = now();
  // round 1: AliceInit(pk_i, k_i, N~_j, h1_j, h2_j)
  for (auto& p : pairs) {
    mta::AliceInitBatch(nodes[p.i].sk.pub, k[p.i], public_dln(nodes[p.j].dln), p.ra, &p.cA, &p.pfA, &err);
    for (auto e : err) st.errors += e != 0;
  }
  const double t1 = now();
  // round 2: Bob j -- BobMid(gamma_j), BobMidWC(w_j, W_j)
  for (auto& p : pairs) {
    const auto dlnA = public_dln(nodes[p.i].dln);
    mta::BobMidBatch(sess, nodes[p.i].sk.pub, p.pfA, g[p.j], p.cA, dlnA, nodes[p.j].dln, nullptr, p.rb, &p.bob, &err);
    for (auto e : err) st.errors += e != 0;
    mta::BobMidBatch(sess, nodes[p.i].sk.pub, p.pfA, w[p.j], p.cA, dlnA, nodes[p.j].dln, &Wp[p.j], p.rbwc, &p.bobwc,
                     &err);
    for (auto e : err) st.errors += e != 0;
  }
  const double t2 = now();
  // round 3: Alice i -- AliceEnd, AliceEndWC
  for (auto& p : pairs) {
    std::vector<mta::ProofBob> pf(Wn), pfwc(Wn);
    std::vector<Nat> cB(Wn), cBwc(Wn);
    for (size_t wi = 0; wi < Wn; ++wi) {
      pf[wi] = p.bob[wi].pf;
      pfwc[wi] = p.bobwc[wi].pf;
      cB[wi] = p.bob[wi].cB;
      cBwc[wi] = p.bobwc[wi].cB;
    }
    mta::AliceEndBatch(sess, nodes[p.i].sk, pf, nodes[p.i].dln, p.cA, cB, nullptr, &p.alpha, &err);
    for (auto e : err) st.errors += e != 0;
    mta::AliceEndBatch(sess, nodes[p.i].sk, pfwc, nodes[p.i].dln, p.cA, cBwc, &Wp[p.j], &p.mu, &err);
    for (auto e : err) st.errors += e != 0;
  }
  const double t3 = now();
  for (const auto& p : pairs)
    for (size_t wi = 0; wi < Wn; ++wi) {
      const bool ok1 = (p.alpha[wi] + p.bob[wi].beta) % q == (k[p.i][wi] * g[p.j][wi]) % q;
      const bool ok2 = (p.mu[wi] + p.bobwc[wi].beta) % q == (k[p.i][wi] * w[p.j][wi]) % q;
      st.relation_failures += !ok1 + !ok2;
    }
  st.round1_s = t1 - t0;
  st.round2_s = t2 - t1;
  st.round3_s = t3 - t2;
  st.total_s = t3 - t0;
  return st;
}

}  // namespace mpcx::host::signing
