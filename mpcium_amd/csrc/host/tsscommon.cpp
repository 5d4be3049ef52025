// tsscommon.cpp -- see tsscommon.hpp.
#include "tsscommon.hpp"
#include <exception>
#include <mutex>
#include <condition_variable>
#include <sched.h>
#include <chrono>
#include <cstdio>

#include "mpcx.h"

#include "hostprof.hpp"

#include <cpuid.h>
#include <immintrin.h>
#include <openssl/evp.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace mpcx::host {

// ------------------------------------------------------------------ SHA-256 (CounterDRBG)
namespace {
// x86 SHA extensions (SHA-NI; every EPYC since Zen 1): one 64-byte block with
// sha256rnds2 (2 rounds per instruction) and sha256msg1/msg2 for the message
// schedule, W[4i..4i+3] = msg2(msg1(W[i-4], W[i-3]) + W[4i-7..4i-4], W[i-1]).
// Selected at run time (CPUID.7.0:EBX bit 29); the scalar block is the
// fallback, and tests/test_host_cpu.py checks the DRBG stream against hashlib.
bool has_sha_ni() {
  static const bool v = [] {
    unsigned a = 0, b = 0, c = 0, d = 0;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    if (!((b >> 29) & 1u)) return false;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
    return ((c >> 19) & 1u) && ((c >> 9) & 1u);  // SSE4.1, SSSE3
  }();
  return v;
}

__attribute__((target("sha,sse4.1,ssse3"))) void sha256_block_ni(uint32_t h[8], const uint8_t* p) {
  alignas(16) static const uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  // state as (A B E F), (C D G H)
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[0]), 0xB1);
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[4]), 0x1B);
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);
  s1 = _mm_blend_epi16(s1, t, 0xF0);
  const __m128i abef = s0, cdgh = s1;
  __m128i w[16];
  for (int i = 0; i < 16; ++i) {
    if (i < 4) {
      w[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), bswap);
    } else {
      __m128i x = _mm_sha256msg1_epu32(w[i - 4], w[i - 3]);
      x = _mm_add_epi32(x, _mm_alignr_epi8(w[i - 1], w[i - 2], 4));
      w[i] = _mm_sha256msg2_epu32(x, w[i - 1]);
    }
    __m128i m = _mm_add_epi32(w[i], _mm_load_si128((const __m128i*)&K[4 * i]));
    s1 = _mm_sha256rnds2_epu32(s1, s0, m);
    m = _mm_shuffle_epi32(m, 0x0E);
    s0 = _mm_sha256rnds2_epu32(s0, s1, m);
  }
  s0 = _mm_add_epi32(s0, abef);
  s1 = _mm_add_epi32(s1, cdgh);
  t = _mm_shuffle_epi32(s0, 0x1B);   // F E B A
  s1 = _mm_shuffle_epi32(s1, 0xB1);  // D C H G
  s0 = _mm_blend_epi16(t, s1, 0xF0); // D C B A
  s1 = _mm_alignr_epi8(s1, t, 8);    // H G F E
  _mm_storeu_si128((__m128i*)&h[0], s0);
  _mm_storeu_si128((__m128i*)&h[4], s1);
}

struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block_scalar(const uint8_t* p) {
    static const uint32_t k[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t S1 = ror(e, 6) ^ ror(e, 11) ^ ror(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + k[i] + w[i];
      const uint32_t S0 = ror(a, 2) ^ ror(a, 13) ^ ror(a, 22);
      const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void block(const uint8_t* p) {
    if (has_sha_ni()) sha256_block_ni(h, p);
    else block_scalar(p);
  }
  // one-shot digest of a short message (< 56 bytes)
  static void digest_short(const uint8_t* msg, size_t n, uint8_t out[32]) {
    Sha256 s;
    uint8_t blk[64] = {0};
    std::memcpy(blk, msg, n);
    blk[n] = 0x80;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; ++i) blk[63 - i] = (uint8_t)(bits >> (8 * i));
    s.block(blk);
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(s.h[i] >> (24 - 8 * j));
  }
};
}  // namespace

void CounterDRBG::seek(uint64_t offset) {
  ctr_ = offset / 32;
  buf_.clear();
  pos_ = 0;
  uint8_t skip[32];
  if (offset % 32) read(skip, offset % 32);
}

void CounterDRBG::read(uint8_t* out, size_t n) {
  // drain the current block, then -- for bulk reads (a safe-prime candidate
  // batch) -- compute whole counter blocks in parallel: block c depends only
  // on (seed, c), so the byte stream is identical to sequential reads
  if (n >= (64u << 10)) {
    const size_t take = std::min(n, buf_.size() - pos_);
    std::memcpy(out, buf_.data() + pos_, take);
    pos_ += take;
    out += take;
    n -= take;
    const size_t blocks = n / 32;
    const uint64_t c0 = ctr_;
    const size_t per = 4096;
    parallel_for((blocks + per - 1) / per, [&](size_t t) {
      uint8_t msg[25];
      std::memcpy(msg, "mpcx-drbg", 9);
      for (int i = 0; i < 8; ++i) msg[9 + i] = (uint8_t)(seed_ >> (8 * i));
      const size_t hi = std::min(blocks, (t + 1) * per);
      for (size_t b = t * per; b < hi; ++b) {
        const uint64_t c = c0 + b;
        for (int i = 0; i < 8; ++i) msg[17 + i] = (uint8_t)(c >> (8 * i));
        Sha256::digest_short(msg, sizeof msg, out + b * 32);
      }
    });
    ctr_ = c0 + blocks;
    out += blocks * 32;
    n -= blocks * 32;
  }
  while (n) {
    if (pos_ == buf_.size()) {
      uint8_t msg[25];
      std::memcpy(msg, "mpcx-drbg", 9);
      for (int i = 0; i < 8; ++i) msg[9 + i] = (uint8_t)(seed_ >> (8 * i));
      for (int i = 0; i < 8; ++i) msg[17 + i] = (uint8_t)(ctr_ >> (8 * i));
      ++ctr_;
      buf_.assign(32, 0);
      Sha256::digest_short(msg, sizeof msg, buf_.data());
      pos_ = 0;
    }
    const size_t take = std::min(n, buf_.size() - pos_);
    std::memcpy(out, buf_.data() + pos_, take);
    pos_ += take;
    out += take;
    n -= take;
  }
}


// ------------------------------------------------------------------ SHA-512/256
// FIPS 180-4 SHA-512/256 (Go crypto.SHA512_256) through OpenSSL's EVP digest
// (libcrypto's assembly SHA-512: ~4x the portable C block function this
// replaced on the signing path's ~5 KB transcripts). One context per thread,
// reset per hash.
namespace {
struct Sha512_256 {
  EVP_MD_CTX* ctx;
  Sha512_256() : ctx(thread_ctx()) {
    if (EVP_DigestInit_ex2(ctx, md(), nullptr) != 1) throw std::runtime_error("EVP_DigestInit_ex2(SHA512-256)");
  }
  void update(const uint8_t* p, size_t n) {
    if (n && EVP_DigestUpdate(ctx, p, n) != 1) throw std::runtime_error("EVP_DigestUpdate");
  }
  void finish(uint8_t out[32]) {
    unsigned len = 0;
    if (EVP_DigestFinal_ex(ctx, out, &len) != 1 || len != 32) throw std::runtime_error("EVP_DigestFinal_ex");
  }
  static const EVP_MD* md() {
    // fetched once: passing EVP_sha512_256() makes OpenSSL 3 look the
    // implementation up in its provider store on every init
    static const EVP_MD* m = [] {
      const EVP_MD* f = EVP_MD_fetch(nullptr, "SHA512-256", nullptr);
      return f ? f : EVP_sha512_256();
    }();
    return m;
  }
  static EVP_MD_CTX* thread_ctx() {
    struct Holder {
      EVP_MD_CTX* c = EVP_MD_CTX_new();
      ~Holder() { EVP_MD_CTX_free(c); }
    };
    static thread_local Holder h;
    if (!h.c) throw std::runtime_error("EVP_MD_CTX_new");
    return h.c;
  }
};

void put_le64(uint8_t* o, uint64_t v) {
  for (int i = 0; i < 8; ++i) o[i] = (uint8_t)(v >> (8 * i));
}

// 8-byte little-endian element count, then every element followed by '$' and
// its byte length as 8 little-endian bytes (up:common/hash.go)
void frame(Sha512_256& s, const std::vector<std::vector<uint8_t>>& parts) {
  uint8_t cnt[8];
  put_le64(cnt, parts.size());
  s.update(cnt, 8);
  uint8_t tail[9];
  tail[0] = '$';
  for (const auto& p : parts) {
    if (!p.empty()) s.update(p.data(), p.size());
    put_le64(tail + 1, p.size());
    s.update(tail, 9);
  }
}

// The same framing for integers (big-endian magnitude bytes, Go's
// big.Int.Bytes), written into one buffer so the digest sees one update.
void frame_ints(Sha512_256& s, const std::vector<const Nat*>& in) {
  static thread_local std::vector<uint8_t> buf;
  size_t total = 8;
  for (const Nat* n : in) total += (n ? (n->bit_len() + 7) / 8 : 0) + 9;
  buf.resize(total);
  uint8_t* o = buf.data();
  put_le64(o, in.size());
  o += 8;
  for (const Nat* n : in) {
    const uint32_t nb = n ? (n->bit_len() + 7) / 8 : 0;
    if (nb) {
      const auto& w = n->limbs();
      for (uint32_t i = 0; i < nb; ++i) o[nb - 1 - i] = (uint8_t)(w[i / 4] >> (8 * (i % 4)));
      o += nb;
    }
    *o++ = '$';
    put_le64(o, nb);
    o += 8;
  }
  s.update(buf.data(), total);
}
}  // namespace

std::vector<uint8_t> SHA512_256(const std::vector<std::vector<uint8_t>>& in) {
  if (in.empty()) return {};
  Sha512_256 s;
  frame(s, in);
  std::vector<uint8_t> out(32);
  s.finish(out.data());
  return out;
}

Nat SHA512_256i(const std::vector<const Nat*>& in) {
  MPCX_PROF("hash.sha512_256i");
  if (in.empty()) return Nat();
  Sha512_256 s;
  frame_ints(s, in);
  uint8_t out[32];
  s.finish(out);
  return Nat::from_bytes_be(out, 32);
}

Nat SHA512_256i_TAGGED(const std::vector<uint8_t>& tag, const std::vector<const Nat*>& in) {
  MPCX_PROF("hash.sha512_256i_tagged");
  const std::vector<uint8_t> tagBz = SHA512_256({tag});
  if (in.empty()) return Nat();
  Sha512_256 s;
  s.update(tagBz.data(), tagBz.size());
  s.update(tagBz.data(), tagBz.size());
  frame_ints(s, in);
  uint8_t out[32];
  s.finish(out);
  return Nat::from_bytes_be(out, 32);
}

Nat RejectionSample(const Nat& q, const Nat& eHash) { return eHash % q; }

// ------------------------------------------------------------------ random
Nat CryptoRandInt(const RandFn& rand, const Nat& max) {
  if (max.is_zero()) throw std::invalid_argument("crypto/rand: argument to Int is <= 0");
  const Nat n = max - Nat(1);
  const uint32_t bitLen = n.bit_len();
  if (bitLen == 0) return Nat();
  const size_t k = (bitLen + 7) / 8;
  unsigned b = bitLen % 8;
  if (b == 0) b = 8;
  std::vector<uint8_t> buf(k);
  for (;;) {
    rand(buf.data(), k);
    buf[0] &= (uint8_t)((1u << b) - 1);
    Nat v = Nat::from_bytes_be(buf.data(), k);
    if (v < max) return v;
  }
}

Nat MustGetRandomInt(const RandFn& rand, uint32_t bits) {
  if (bits == 0 || bits > 5000) throw std::invalid_argument("MustGetRandomInt: bits out of range");
  return CryptoRandInt(rand, (Nat(1) << bits) - Nat(1));
}

Nat GetRandomPositiveInt(const RandFn& rand, const Nat& lessThan) {
  MPCX_PROF("rand.positive_int");
  if (lessThan.is_zero()) throw std::invalid_argument("GetRandomPositiveInt: lessThan must be > 0");
  for (;;) {
    Nat t = MustGetRandomInt(rand, lessThan.bit_len());
    if (t < lessThan) return t;
  }
}

Nat GetRandomPositiveRelativelyPrimeInt(const RandFn& rand, const Nat& n) {
  MPCX_PROF("rand.relprime_int");
  if (n.is_zero()) throw std::invalid_argument("GetRandomPositiveRelativelyPrimeInt: n must be > 0");
  for (;;) {
    Nat t = MustGetRandomInt(rand, n.bit_len());
    if (t.is_zero() || !(t < n)) continue;
    if (n.is_odd() ? coprime_odd(t, n) : gcd(t, n) == Nat(1)) return t;
  }
}

std::vector<uint8_t> CoprimeMany(const std::vector<const Nat*>& xs, const Nat& m) {
  MPCX_PROF("gcd.coprime_many");
  const size_t n = xs.size();
  std::vector<uint8_t> ok(n, 0);
  if (n == 0) return ok;
  if (!m.is_odd()) {
    parallel_for(n, [&](size_t i) { ok[i] = gcd(*xs[i], m) == Nat(1); });
    return ok;
  }
  // one gcd per chunk of a product; a chunk holding a non-coprime x (never
  // for honest inputs) is decided element by element
  constexpr size_t kChunk = 48;
  const size_t chunks = (n + kChunk - 1) / kChunk;
  parallel_for(chunks, [&](size_t c) {
    const size_t b = c * kChunk, e = std::min(n, b + kChunk);
    if (coprime_product_odd(xs.data() + b, e - b, m)) {
      for (size_t i = b; i < e; ++i) ok[i] = 1;
    } else {
      for (size_t i = b; i < e; ++i) ok[i] = coprime_odd(*xs[i], m);
    }
  });
  return ok;
}

void GetRandomPositiveRelativelyPrimeIntBatch(const std::vector<const RandFn*>& rand, const Nat& n,
                                              const std::vector<Nat*>& out) {
  if (n.is_zero()) throw std::invalid_argument("GetRandomPositiveRelativelyPrimeInt: n must be > 0");
  if (rand.size() != out.size()) throw std::invalid_argument("GetRandomPositiveRelativelyPrimeIntBatch: sizes");
  // Each reader makes exactly the reads of its one-by-one call: a round draws
  // one candidate t in [1, n) per pending reader (zero / out-of-range draws
  // are redrawn on the spot, as in the scalar loop), the round's gcd
  // decisions are batched, and only readers whose t shares a factor with n
  // draw again.
  std::vector<size_t> pending(rand.size());
  for (size_t i = 0; i < pending.size(); ++i) pending[i] = i;
  while (!pending.empty()) {
    parallel_for(pending.size(), [&](size_t j) {
      const size_t i = pending[j];
      for (;;) {
        Nat t = MustGetRandomInt(*rand[i], n.bit_len());
        if (t.is_zero() || !(t < n)) continue;
        *out[i] = std::move(t);
        return;
      }
    });
    std::vector<const Nat*> xs(pending.size());
    for (size_t j = 0; j < pending.size(); ++j) xs[j] = out[pending[j]];
    const std::vector<uint8_t> ok = CoprimeMany(xs, n);
    std::vector<size_t> next;
    for (size_t j = 0; j < pending.size(); ++j)
      if (!ok[j]) next.push_back(pending[j]);
    pending.swap(next);
  }
}

// ------------------------------------------------------------------ threads
// CPUs this process may use: its affinity mask, capped by the cgroup v2 CPU
// quota (a GPU box gives a job a share of the machine: the affinity shows every
// CPU, cpu.max how many may run at once).
int usable_cpus() {
  static const int n = [] {
    int a = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) a = CPU_COUNT(&set);
    if (a <= 0) a = (int)std::max(1u, std::thread::hardware_concurrency());
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32] = {0};
      long period = 0;
      if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0) {
        const long q = std::atol(quota);
        if (q > 0) a = std::min(a, (int)std::max(1L, (q + period - 1) / period));
      }
      std::fclose(f);
    }
    return std::max(1, a);
  }();
  return n;
}

// Host threads for parallel loops: the usable CPUs, up to kThreadsPerDevice per
// bound GPU (one node process drives all of its GPUs, and each GPU's protocol
// batches need their own share of host work: /root/reference/pkg/mpc/node.go:69,109,170).
// MPCX_HOST_THREADS overrides the total.
int host_threads() {
  static const int env = [] {
    const char* e = std::getenv("MPCX_HOST_THREADS");
    return e ? std::atoi(e) : 0;
  }();
  if (env > 0) return env;
  constexpr int kThreadsPerDevice = 16;
  int dev = 0;
  if (mpcx_bound_devices(&dev, nullptr, 0) != MPCX_OK || dev < 1) dev = 1;
  return std::max(1, std::min(usable_cpus(), kThreadsPerDevice * dev));
}

namespace {
// One process-wide pool of host_threads() - 1 workers shared by every
// parallel_for: the signing and keygen drivers run several protocol tasks at
// once, each issuing parallel loops, and a thread set per loop oversubscribed
// the cores (tasks x 16 threads) and paid a spawn per loop. A loop is a task in
// the pool's list; the caller works on its own loop too, so a loop started from
// inside another one (or from any thread) always makes progress.
struct Loop {
  const std::function<void(size_t)>* fn;
  size_t n;
  std::atomic<size_t> next{0};
  std::atomic<size_t> done{0};
  std::atomic<bool> failed{false};
  std::atomic<int> users{0};  // pool workers inside work()
  std::exception_ptr err;
  std::mutex err_mu;
  // runs indices until none is left; returns after the last index it took
  // (true: it finished the loop's last index)
  bool work() {
    bool last = false;
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return last;
      if (!failed.load(std::memory_order_relaxed)) {
        try {
          (*fn)(i);
        } catch (...) {
          std::lock_guard<std::mutex> lk(err_mu);
          if (!failed.exchange(true)) err = std::current_exception();
        }
      }
      last = done.fetch_add(1) + 1 == n;
    }
  }
};

class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();  // never destroyed: workers outlive static teardown
    p->grow(host_threads() - 1);
    return *p;
  }
  void run(Loop& l) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      loops_.push_back(&l);
    }
    cv_.notify_all();
    l.work();
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = loops_.begin(); it != loops_.end(); ++it)
        if (*it == &l) {
          loops_.erase(it);
          break;
        }
    }
    // Every index was taken and no worker can pick the loop up any more: sleep
    // on the completion signal until the indices still running elsewhere finish
    // and the workers leave the loop (no spinning: many protocol tasks wait here
    // at once). The waiter does not run other loops' indices meanwhile: with
    // nested loops that recursion would be unbounded (a worker inside an outer
    // index helping the outer loop again, one stack frame set per index).
    // (finish() notifies under done_mu_ after every transition that can make
    // this true: the last index done, the last worker gone)
    std::unique_lock<std::mutex> lk(done_mu_);
    done_cv_.wait(lk, [&] { return l.done.load() >= l.n && l.users.load() == 0; });
  }

 private:
  HostPool() = default;
  void grow(int workers) {
    std::lock_guard<std::mutex> lk(grow_mu_);
    for (; workers_ < workers; ++workers_)
      std::thread([this] {
        for (;;) {
          Loop* l = nullptr;
          {
            // the loop is taken by the predicate itself: other threads advance
            // `next` without the lock, so a second look could find none left
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return (l = pending_locked()) != nullptr; });
            l->users.fetch_add(1);  // l stays alive (listed or waited for) until users drops back to 0
          }
          MPCX_PROF_CPU("cpu.pool_workers");
          finish(l, l->work());
        }
      }).detach();
  }
  Loop* pending_locked() {
    for (Loop* x : loops_)
      if (x->next.load() < x->n) return x;
    return nullptr;
  }
  // a worker leaves loop l (last: it completed l's final index)
  void finish(Loop* l, bool last) {
    const bool left_last = l->users.fetch_sub(1) == 1;
    if (last || left_last) {
      std::lock_guard<std::mutex> lk(done_mu_);
      done_cv_.notify_all();
    }
  }
  std::mutex mu_, grow_mu_, done_mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<Loop*> loops_;
  int workers_ = 0;
};

bool pool_enabled() {
  static const bool on = [] {  // MPCX_HOST_POOL=0: a thread set per loop (A/B runs)
    const char* e = std::getenv("MPCX_HOST_POOL");
    return !(e && e[0] == '0');
  }();
  return on;
}
}  // namespace

void parallel_for(size_t n, const std::function<void(size_t)>& fn) {
  const size_t nt = std::min<size_t>((size_t)host_threads(), n);
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  if (pool_enabled()) {
    Loop l;
    l.fn = &fn;
    l.n = n;
    HostPool::get().run(l);
    if (l.err) std::rethrow_exception(l.err);
    return;
  }
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::atomic<bool> failed{false};
  auto work = [&] {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n || failed.load()) return;
      try {
        fn(i);
      } catch (...) {
        if (!failed.exchange(true)) err = std::current_exception();
        return;
      }
    }
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
}

}  // namespace mpcx::host
