// safeprime.cpp -- see safeprime.hpp.
#include "safeprime.hpp"

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>

#include "engine.hpp"
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

// 20 deterministic Miller-Rabin bases in [2, q-2] for candidate q, plus base 2
std::vector<Nat> mr_bases(const Nat& q) {
  std::vector<Nat> out{Nat(2)};
  CounterDRBG rng(q.low64() ^ 0x4d52u);
  const uint32_t bits = q.bit_len();
  const Nat lim = q - Nat(3);
  std::vector<uint8_t> buf((bits + 7) / 8);
  while (out.size() < 21) {
    rng.read(buf.data(), buf.size());
    Nat v = Nat::from_bytes_be(buf.data(), buf.size()) % lim;
    out.push_back(v + Nat(2));
  }
  return out;
}
}  // namespace

namespace {
void check_safe_prime_args(int bitLen) {
  if (bitLen < 6) throw std::invalid_argument("safe prime size must be at least 6 bits");
  if (bitLen > 1024) throw std::invalid_argument("GPU candidate class holds safe primes up to 1024 bits");
}

size_t default_batch(int bitLen) { return bitLen - 1 >= 63 ? 196608 : 16384; }

// One batch of the candidate stream (raw = batch x nbytes of stream bytes whose
// first candidate has stream index base_index): sieve, Pocklington, Miller-Rabin.
// Appends the accepted safe primes in stream order, at most `limit` of them.
void test_batch(int bitLen, const uint8_t* raw, size_t batch, uint64_t base_index, SafePrimeStats& st,
                std::vector<GermainSafePrime>& out, size_t limit) {
  const int qBitLen = bitLen - 1;
  const size_t nbytes = (size_t)(qBitLen + 7) / 8;
  // GPU sieve (mpcx_safeprime_sieve_fermat) for q of 63..1023 bits: candidate
  // masks, delta walk, trial division and the Pocklington test all on the
  // device; the host draws the stream and runs Miller-Rabin on the rare
  // Fermat survivors. Smaller sizes keep the host sieve.
  const bool gpu_sieve = qBitLen >= 63;
  const unsigned nthreads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // Fermat survivors (stream order): candidate index in the batch and q
  std::vector<size_t> fidx;
  std::vector<Nat> fq;
  if (gpu_sieve) {
    const auto sv = Engine::get().safeprime_sieve_fermat(raw, (uint32_t)nbytes, (uint32_t)batch, (uint32_t)qBitLen);
    st.sieved_out += batch - sv.size();
    st.fermat_tests += sv.size();
    for (const auto& [i, ok] : sv) {
      if (!ok) continue;
      fidx.push_back(i);
      fq.push_back(CandidateFromBytes(raw + (size_t)i * nbytes, nbytes, qBitLen));
    }
  } else {
    std::vector<Nat> qs(batch);
    std::vector<uint8_t> keep(batch, 0);
    auto work = [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        qs[i] = CandidateFromBytes(raw + i * nbytes, nbytes, qBitLen);
        keep[i] = (qs[i].bit_len() == (uint32_t)qBitLen) && (bitLen <= 12 || passes_trial(qs[i]));
      }
    };
    std::vector<std::thread> th;
    const size_t chunk = (batch + nthreads - 1) / nthreads;
    for (unsigned t = 0; t < nthreads; ++t) {
      const size_t lo = t * chunk, hi = std::min(batch, lo + chunk);
      if (lo < hi) th.emplace_back(work, lo, hi);
    }
    for (auto& t : th) t.join();
    std::vector<size_t> idx;
    std::vector<Nat> ps;
    for (size_t i = 0; i < batch; ++i) {
      if (!keep[i]) continue;
      idx.push_back(i);
      ps.push_back((qs[i] << 1) + Nat(1));
    }
    st.sieved_out += batch - idx.size();
    st.fermat_tests += ps.size();
    // GPU: Pocklington criterion 2^(p-1) == 1 mod p on every survivor
    std::vector<uint8_t> f = bitLen >= 4 ? Engine::get().fermat2(ps) : std::vector<uint8_t>(ps.size(), 1);
    for (size_t j = 0; j < idx.size(); ++j) {
      if (!f[j]) continue;
      fidx.push_back(idx[j]);
      fq.push_back(qs[idx[j]]);
    }
  }
  st.candidates += batch;
  // GPU: Miller-Rabin on q for the Fermat survivors, in stream order
  std::vector<Nat> mr_n, mr_a;
  for (const Nat& q : fq)
    for (const Nat& a : mr_bases(q)) {
      mr_n.push_back(q);
      mr_a.push_back(a);
    }
  st.mr_tests += mr_n.size();
  std::vector<uint8_t> mr = Engine::get().strong_probable_prime(mr_n, mr_a);
  for (size_t s = 0; s < fq.size() && out.size() < limit; ++s) {
    bool prime = true;
    for (size_t r = 0; r < 21; ++r) prime &= mr[s * 21 + r] != 0;
    if (!prime) continue;
    out.push_back({(fq[s] << 1) + Nat(1), fq[s], base_index + fidx[s]});
  }
}

void add_stats(SafePrimeStats* stats, const SafePrimeStats& st) {
  if (!stats) return;
  stats->candidates += st.candidates;
  stats->sieved_out += st.sieved_out;
  stats->fermat_tests += st.fermat_tests;
  stats->mr_tests += st.mr_tests;
  stats->seconds += st.seconds;
}
}  // namespace

std::vector<GermainSafePrime> SafePrimeBatch(int bitLen, uint64_t seed, uint64_t batch_no, size_t batch,
                                             SafePrimeStats* stats) {
  check_safe_prime_args(bitLen);
  const auto t0 = std::chrono::steady_clock::now();
  if (batch == 0) batch = default_batch(bitLen);
  const size_t nbytes = (size_t)(bitLen - 1 + 7) / 8;
  std::vector<uint8_t> raw(nbytes * batch);
  CounterDRBG drbg(seed);
  drbg.seek(batch_no * (uint64_t)raw.size());
  drbg.read(raw.data(), raw.size());
  SafePrimeStats st;
  std::vector<GermainSafePrime> out;
  test_batch(bitLen, raw.data(), batch, batch_no * batch, st, out, SIZE_MAX);
  st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  add_stats(stats, st);
  return out;
}

std::vector<GermainSafePrime> GetRandomSafePrimes(int bitLen, int numPrimes, const RandFn& rand,
                                                  SafePrimeStats* stats, size_t batch, uint64_t max_candidates) {
  check_safe_prime_args(bitLen);
  if (numPrimes < 1) throw std::invalid_argument("numPrimes should be > 0");
  const auto t0 = std::chrono::steady_clock::now();
  SafePrimeStats st;
  const size_t nbytes = (size_t)(bitLen - 1 + 7) / 8;
  if (batch == 0) batch = default_batch(bitLen);
  std::vector<GermainSafePrime> out;
  std::vector<uint8_t> raw(nbytes * batch);
  uint64_t index = 0;
  while ((int)out.size() < numPrimes && index < max_candidates) {
    // draw a batch from the stream: one read of batch candidates' bytes is the
    // same byte stream as batch sequential reads (stream order is the contract)
    rand(raw.data(), nbytes * batch);
    test_batch(bitLen, raw.data(), batch, index, st, out, (size_t)numPrimes);
    index += batch;
  }
  st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  add_stats(stats, st);
  if ((int)out.size() < numPrimes) throw std::runtime_error("safe prime search exhausted max_candidates");
  return out;
}

paillier::PrivateKey GenerateKeyPair(int modulusBitLen, const RandFn& rand, SafePrimeStats* stats) {
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

LocalPreParams GeneratePreParams(const RandFn& rand, SafePrimeStats* stats) {
  LocalPreParams pp;
  // tss-lib runs these two searches concurrently on one reader (stream
  // interleaving is scheduling-defined); here they run in a fixed order.
  pp.PaillierSK = GenerateKeyPair(2048, rand, stats);
  auto sgps = GetRandomSafePrimes(1024, 2, rand, stats);
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
