// tsscommon.cpp -- see tsscommon.hpp.
#include "tsscommon.hpp"

#include "hostprof.hpp"

#include <cpuid.h>
#include <immintrin.h>

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
// FIPS 180-4 SHA-512 with the SHA-512/256 initial hash value, truncated to 32 bytes
// (Go crypto.SHA512_256).
namespace {
struct Sha512_256 {
  uint64_t h[8] = {0x22312194FC2BF72Cull, 0x9F555FA3C84C64C2ull, 0x2393B86B6F53B151ull, 0x963877195940EABDull,
                   0x96283EE2A88EFFE3ull, 0xBE5E1E2553863992ull, 0x2B0199FC2C85B8AAull, 0x0EB72DDC81C52CA2ull};
  uint8_t buf[128];
  size_t blen = 0;
  uint64_t total = 0;
  static uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
  void block(const uint8_t* p) {
    static const uint64_t k[80] = {
        0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
        0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
        0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
        0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
        0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
        0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
        0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
        0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
        0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
        0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
        0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
        0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
        0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
        0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
        0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
        0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
    uint64_t w[80];
    for (int i = 0; i < 16; ++i) {
      uint64_t v = 0;
      for (int j = 0; j < 8; ++j) v = (v << 8) | p[8 * i + j];
      w[i] = v;
    }
    for (int i = 16; i < 80; ++i) {
      const uint64_t s0 = ror(w[i - 15], 1) ^ ror(w[i - 15], 8) ^ (w[i - 15] >> 7);
      const uint64_t s1 = ror(w[i - 2], 19) ^ ror(w[i - 2], 61) ^ (w[i - 2] >> 6);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 80; ++i) {
      const uint64_t S1 = ror(e, 14) ^ ror(e, 18) ^ ror(e, 41);
      const uint64_t ch = (e & f) ^ (~e & g);
      const uint64_t t1 = hh + S1 + ch + k[i] + w[i];
      const uint64_t S0 = ror(a, 28) ^ ror(a, 34) ^ ror(a, 39);
      const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint64_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    total += n;
    while (n) {
      const size_t take = std::min(n, 128 - blen);
      std::memcpy(buf + blen, p, take);
      blen += take;
      p += take;
      n -= take;
      if (blen == 128) {
        block(buf);
        blen = 0;
      }
    }
  }
  void finish(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    uint8_t pad = 0x80;
    update(&pad, 1);
    const uint8_t z = 0;
    while (blen != 112) update(&z, 1);
    uint8_t len[16] = {0};
    for (int i = 0; i < 8; ++i) len[15 - i] = (uint8_t)(bits >> (8 * i));
    update(len, 16);
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
  }
};

// 8-byte little-endian element count, then every element followed by '$'
void frame(Sha512_256& s, const std::vector<std::vector<uint8_t>>& parts) {
  uint8_t cnt[8];
  for (int i = 0; i < 8; ++i) cnt[i] = (uint8_t)((uint64_t)parts.size() >> (8 * i));
  s.update(cnt, 8);
  const uint8_t delim = '$';
  for (const auto& p : parts) {
    if (!p.empty()) s.update(p.data(), p.size());
    s.update(&delim, 1);
  }
}

std::vector<std::vector<uint8_t>> int_parts(const std::vector<const Nat*>& in) {
  std::vector<std::vector<uint8_t>> parts;
  parts.reserve(in.size());
  for (const Nat* n : in) parts.push_back(n ? n->to_bytes_be() : std::vector<uint8_t>{});
  return parts;
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
  frame(s, int_parts(in));
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
  frame(s, int_parts(in));
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
int host_threads() {
  static const int n = [] {
    const char* e = std::getenv("MPCX_HOST_THREADS");
    int v = e ? std::atoi(e) : 0;
    if (v <= 0) v = std::min(16, (int)std::max(1u, std::thread::hardware_concurrency()));
    return v;
  }();
  return n;
}

void parallel_for(size_t n, const std::function<void(size_t)>& fn) {
  const size_t nt = std::min<size_t>((size_t)host_threads(), n);
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
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
