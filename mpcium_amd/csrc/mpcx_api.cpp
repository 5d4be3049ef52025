// mpcx_api.cpp -- C-ABI host side of libmpcx.so (see include/mpcx.h).
//
// Owns device selection, the per-modulus Montgomery constants (what Go's
// nat.expNNMontgomery recomputes on every call: k0 and RR,
// go:src/math/big/nat.go), the kernel workspace and the staging buffers, and
// launches the gfx950 kernels of mpcx_kernels.hip. No CPU compute fallback:
// every modexp runs on the GPU or the call fails with an error code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mpcx.h"
#include "mpcx_internal.h"

// per-geometry kernels (mpcx_geom.hip, one translation unit per geometry id)
#define MPCX_GEOM_DECL(g)                                                                          \
  hipError_t mpcx_launch_modexp_g##g(const mpcx::ModexpArgs* a, uint32_t waves, hipStream_t st); \
  hipError_t mpcx_modexp_occupancy_g##g(int* blocks_per_cu);
#define MPCX_FOR_EACH_GEOM(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6)
static_assert(MPCX_NUM_GEOMS == 7, "update MPCX_FOR_EACH_GEOM and build.py GEOMS");
extern "C" {
MPCX_FOR_EACH_GEOM(MPCX_GEOM_DECL)
hipError_t mpcx_launch_fermat2(const mpcx::FermatArgs* a, uint32_t blocks, hipStream_t st);
hipError_t mpcx_launch_mr(const mpcx::MrArgs* a, uint32_t blocks, hipStream_t st);
hipError_t mpcx_launch_expsched(const mpcx::ExpSchedArgs* a, hipStream_t st);
hipError_t mpcx_launch_fixedbase_g0(const mpcx::FixedBaseArgs* a, uint32_t waves, hipStream_t st);
hipError_t mpcx_launch_fixedbase_g1(const mpcx::FixedBaseArgs* a, uint32_t waves, hipStream_t st);
hipError_t mpcx_launch_sieve(const mpcx::SieveArgs* a, hipStream_t st);
hipError_t mpcx_launch_selftest(uint32_t* d_out, hipStream_t st);
}

struct mpcx_modulus_s {
  int cls;
  uint32_t bits;
  uint32_t words;  // normalized length of m in 32-bit words
  uint32_t n0inv;
  uint32_t* d_const;  // per geometry of the class: 3*L_g digits N, R mod N, R^2 mod N
  uint32_t const_off[MPCX_NUM_GEOMS];  // digit offset of geometry g's block (class members only)
  std::vector<uint32_t> m;
};

struct mpcx_fixedbase_s {
  mpcx_mod_t mod;
  int geom;          // main geometry of the modulus class (table layout)
  uint32_t nwin;     // 8-bit windows: exponents of up to 8*nwin bits
  uint32_t* d_table; // nwin x 256 entries x L digits ([k][p] interleaved)
};

namespace {

constexpr int kDigitBits = 28;
constexpr uint32_t kM28 = (1u << kDigitBits) - 1u;

thread_local std::string g_err;
std::mutex g_mu;
int g_device = -1;
int g_num_cus = 0;
int g_geom_slots[MPCX_NUM_GEOMS] = {0};  // resident wavefronts per device, per geometry
bool g_split = false;                    // narrow-geometry tail launch (measured slower: off)
int g_force_geom = -1;                   // mpcx_set_option("force_geom", g): one geometry for everything
double g_narrow_rounds = 0.15;           // mpcx_set_option("narrow_rounds", 100x): narrow-geometry threshold
int g_sched_width = MPCX_SCHED_MAX_WIDTH;  // mpcx_set_option("sched_width", w): 0 = Go's fixed window
int g_main_geom[MPCX_NUM_CLASSES] = {MPCX_MAIN_GEOM(0), MPCX_MAIN_GEOM(1), MPCX_MAIN_GEOM(2)};
struct Staging {
  void* ptr = nullptr;
  size_t bytes = 0;
};
// An execution lane: one HIP stream with its own exponentiation-table
// workspace and staging buffers. Host-buffer calls from different threads run
// on different lanes concurrently, so small or partial-round batches (a
// latency-bound Fac-proof group, a 10k-wallet MtA step that fills 40% of the
// wavefront slots) overlap on the GPU instead of queueing behind one lock.
// kLanes matches the HW queues HIP gives a process by default.
struct Lane {
  std::mutex mu;
  hipStream_t st = nullptr;  // created on first use (non-blocking)
  uint32_t* ws = nullptr;    // exponentiation table workspace
  size_t ws_bytes = 0;
  Staging stage[4];  // bases, exps, out, misc
  Staging sieve[3];  // survivors' p words, survivors' indices, trial-division tables + counter
};
constexpr int kLanes = 4;
Lane g_lanes[kLanes];
// Workspace of the device-buffer entry points (caller's stream, under g_mu;
// callers order their own device-buffer calls) and of table builds.
Lane g_dev_lane;
std::atomic<unsigned> g_lane_rr{0};

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(MPCX_EHIP, "%s: %s", what, hipGetErrorString(e));
}

int class_for_bits(uint32_t bits) {
  for (int c = 0; c < MPCX_NUM_CLASSES; ++c)
    if ((int)bits <= MPCX_CLASS_MAXBITS(c)) return c;
  return -1;
}

uint32_t bit_length(const std::vector<uint32_t>& x) {
  for (int i = (int)x.size() - 1; i >= 0; --i)
    if (x[i]) return (uint32_t)(32 * i + (32 - __builtin_clz(x[i])));
  return 0;
}

uint32_t bit_length_words(const uint32_t* x, uint32_t n) {
  for (int i = (int)n - 1; i >= 0; --i)
    if (x[i]) return (uint32_t)(32 * i + (32 - __builtin_clz(x[i])));
  return 0;
}

// x >= m (same length)
bool geq(const std::vector<uint32_t>& x, const std::vector<uint32_t>& m) {
  for (int i = (int)x.size() - 1; i >= 0; --i)
    if (x[i] != m[i]) return x[i] > m[i];
  return true;
}

// 2^k mod m by doubling with conditional subtraction (once per registration).
std::vector<uint32_t> pow2_mod(uint32_t k, const std::vector<uint32_t>& m) {
  const size_t n = m.size();
  std::vector<uint32_t> x(n + 1, 0), mm(m);
  mm.push_back(0);
  x[0] = 1;
  if (n == 1 && m[0] == 1) return std::vector<uint32_t>(n, 0);
  for (uint32_t i = 0; i < k; ++i) {
    uint32_t c = 0;
    for (size_t j = 0; j <= n; ++j) {
      const uint32_t nc = x[j] >> 31;
      x[j] = (x[j] << 1) | c;
      c = nc;
    }
    if (geq(x, mm)) {
      uint64_t br = 0;
      for (size_t j = 0; j <= n; ++j) {
        const uint64_t d = (uint64_t)x[j] - mm[j] - br;
        x[j] = (uint32_t)d;
        br = (d >> 63) & 1;
      }
    }
  }
  x.resize(n);
  return x;
}

std::vector<uint32_t> to_digits(const std::vector<uint32_t>& w, uint32_t L) {
  std::vector<uint32_t> d(L, 0);
  for (uint32_t i = 0; i < L; ++i) {
    const uint32_t bit = i * kDigitBits, wi = bit >> 5, s = bit & 31;
    uint64_t v = 0;
    if (wi < w.size()) v = w[wi];
    if (wi + 1 < w.size()) v |= (uint64_t)w[wi + 1] << 32;
    d[i] = (uint32_t)(v >> s) & kM28;
  }
  return d;
}

hipError_t mpcx_launch_modexp(int geom, const mpcx::ModexpArgs* a, uint32_t waves, hipStream_t st) {
  switch (geom) {
#define MPCX_CASE(g) \
  case g:            \
    return mpcx_launch_modexp_g##g(a, waves, st);
    MPCX_FOR_EACH_GEOM(MPCX_CASE)
#undef MPCX_CASE
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t mpcx_modexp_occupancy(int geom, int* blocks_per_cu) {
  switch (geom) {
#define MPCX_CASE(g) \
  case g:            \
    return mpcx_modexp_occupancy_g##g(blocks_per_cu);
    MPCX_FOR_EACH_GEOM(MPCX_CASE)
#undef MPCX_CASE
    default:
      return hipErrorInvalidValue;
  }
}

// Every entry point runs on the caller's thread: bind that thread to the
// process's GPU (HIP's current device is per thread; a worker thread would
// otherwise submit to device 0 on a multi-GPU node).
int ensure_device() {
  if (g_device < 0) return fail(MPCX_ENODEV, "mpcx_init() has not been called");
  thread_local int t_dev = -1;
  if (t_dev != g_device) {
    hipError_t e = hipSetDevice(g_device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    t_dev = g_device;
  }
  return MPCX_OK;
}

// A free lane (round-robin start, first one not in use), else wait for one.
Lane& acquire_lane(std::unique_lock<std::mutex>& lk) {
  const unsigned start = g_lane_rr.fetch_add(1, std::memory_order_relaxed);
  for (int i = 0; i < kLanes; ++i) {
    Lane& l = g_lanes[(start + i) % kLanes];
    std::unique_lock<std::mutex> t(l.mu, std::try_to_lock);
    if (t.owns_lock()) {
      lk = std::move(t);
      return l;
    }
  }
  Lane& l = g_lanes[start % kLanes];
  lk = std::unique_lock<std::mutex>(l.mu);
  return l;
}

int lane_stream(Lane& l) {
  if (l.st) return MPCX_OK;
  hipError_t e = hipStreamCreateWithFlags(&l.st, hipStreamNonBlocking);
  if (e != hipSuccess) {
    l.st = nullptr;
    return hip_fail(e, "hipStreamCreate(lane)");
  }
  return MPCX_OK;
}

int h2d(void* d, const void* h, size_t bytes, hipStream_t st) {
  if (!bytes) return MPCX_OK;
  hipError_t e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "copy inputs");
}

int d2h_sync(void* h, const void* d, size_t bytes, hipStream_t st) {
  hipError_t e = bytes ? hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st) : hipSuccess;
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "copy results");
}

int ensure_buffer(Staging& s, size_t bytes) {
  if (s.bytes >= bytes && s.ptr) return MPCX_OK;
  if (s.ptr) (void)hipFree(s.ptr);
  s.ptr = nullptr;
  s.bytes = 0;
  size_t want = std::max<size_t>(bytes, 1 << 20);
  hipError_t e = hipMalloc(&s.ptr, want);
  if (e != hipSuccess) return fail(MPCX_ENOMEM, "hipMalloc(%zu): %s", want, hipGetErrorString(e));
  s.bytes = want;
  return MPCX_OK;
}

int ensure_workspace(Lane& l, size_t bytes) {
  if (l.ws_bytes >= bytes) return MPCX_OK;
  if (l.ws) {
    // the lane's previous kernels may still read the old workspace
    if (l.st) (void)hipStreamSynchronize(l.st);
    (void)hipFree(l.ws);
  }
  l.ws = nullptr;
  l.ws_bytes = 0;
  hipError_t e = hipMalloc((void**)&l.ws, bytes);
  if (e != hipSuccess) return fail(MPCX_ENOMEM, "hipMalloc(workspace %zu): %s", bytes, hipGetErrorString(e));
  l.ws_bytes = bytes;
  return MPCX_OK;
}

int run_selftest() {
  uint32_t* d = nullptr;
  hipError_t e = hipMalloc((void**)&d, 256 * sizeof(uint32_t));
  if (e != hipSuccess) return hip_fail(e, "selftest alloc");
  e = mpcx_launch_selftest(d, nullptr);
  std::vector<uint32_t> h(256);
  if (e == hipSuccess) e = hipMemcpy(h.data(), d, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(e, "selftest");
  for (uint32_t l = 0; l < 64; ++l) {
    const uint32_t nxt = l < 63 ? 1000 + l + 1 : 0;
    const uint32_t prv = l > 0 ? 1000 + l - 1 : 0;
    const uint32_t bp = 2000 + (l / 7) * 7;
    const uint64_t acc = (uint64_t)(0xFFFFFFF0u + l) * (0xFFFFFFF7u - l) + 0xFFFFFFFFFFFFull;
    if (h[l] != nxt || h[64 + l] != prv || h[128 + l] != bp || h[192 + l] != (uint32_t)(acc >> 32))
      return fail(MPCX_EHIP,
                  "device self-test failed at lane %u (dpp next %u/%u prev %u/%u bpermute %u/%u mad %u/%u)", l,
                  h[l], nxt, h[64 + l], prv, h[128 + l], bp, h[192 + l], (uint32_t)(acc >> 32));
  }
  return MPCX_OK;
}

}  // namespace

extern "C" {

int mpcx_version(void) { return 100; }

int mpcx_set_option(const char* key, int value) {
  if (!key) return fail(MPCX_EINVAL, "null option");
  std::lock_guard<std::mutex> lk(g_mu);
  if (std::strcmp(key, "split") == 0) {
    g_split = value != 0;
  } else if (std::strcmp(key, "force_geom") == 0) {
    if (value < -1 || value >= MPCX_NUM_GEOMS) return fail(MPCX_EINVAL, "force_geom %d out of range", value);
    g_force_geom = value;
  } else if (std::strcmp(key, "sched_width") == 0) {
    // cap on the sliding-window width of shared exponents; 0: Go's 4-bit fixed window
    if (value < 0 || value > MPCX_SCHED_MAX_WIDTH) return fail(MPCX_EINVAL, "sched_width %d out of range", value);
    g_sched_width = value;
  } else if (std::strcmp(key, "narrow_rounds") == 0) {
    // batches below value/100 of a resident round run in the narrow geometry
    if (value < 0 || value > 100) return fail(MPCX_EINVAL, "narrow_rounds %d out of range", value);
    g_narrow_rounds = value / 100.0;
  } else if (std::strcmp(key, "main_geom") == 0) {
    // main (throughput) geometry of the geometry's class
    if (value < 0 || value >= MPCX_NUM_GEOMS) return fail(MPCX_EINVAL, "main_geom %d out of range", value);
    g_main_geom[MPCX_GEOM_CLASS(value)] = value;
  } else {
    return fail(MPCX_EINVAL, "unknown option %s", key);
  }
  return MPCX_OK;
}

const char* mpcx_last_error(void) { return g_err.c_str(); }

int mpcx_device_count(int* out_count) {
  if (!out_count) return fail(MPCX_EINVAL, "null out_count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *out_count = n;
  return MPCX_OK;
}

int mpcx_init(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_device >= 0) {
    if (g_device == device) return MPCX_OK;
    return fail(MPCX_EINVAL, "already bound to device %d (one process per GPU)", g_device);
  }
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return fail(MPCX_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n) return fail(MPCX_EINVAL, "device %d out of range [0,%d)", device, n);
  e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MPCX_ENODEV, "device %d is %s; libmpcx is built for gfx950 only", device, prop.gcnArchName);
  g_device = device;
  g_num_cus = prop.multiProcessorCount;
  for (int g = 0; g < MPCX_NUM_GEOMS; ++g) {
    int b = 0;
    if (mpcx_modexp_occupancy(g, &b) != hipSuccess || b <= 0) b = 1;
    g_geom_slots[g] = b * g_num_cus;
  }
  const char* sp = std::getenv("MPCX_SPLIT");
  if (sp) g_split = sp[0] != '0';
  int rc = run_selftest();
  if (rc != MPCX_OK) g_device = -1;
  return rc;
}

int mpcx_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto drop = [](Lane& l) {
    std::lock_guard<std::mutex> ll(l.mu);
    if (l.st) {
      (void)hipStreamSynchronize(l.st);
      (void)hipStreamDestroy(l.st);
    }
    l.st = nullptr;
    if (l.ws) (void)hipFree(l.ws);
    l.ws = nullptr;
    l.ws_bytes = 0;
    for (auto* arr : {l.stage, l.sieve})
      for (int i = 0; i < (arr == l.stage ? 4 : 3); ++i) {
        if (arr[i].ptr) (void)hipFree(arr[i].ptr);
        arr[i] = Staging{};
      }
  };
  for (auto& l : g_lanes) drop(l);
  drop(g_dev_lane);
  g_device = -1;
  return MPCX_OK;
}

int mpcx_modulus_register(const uint32_t* m_words, uint32_t m_len, mpcx_mod_t* out) {
  if (!m_words || !out || m_len == 0) return fail(MPCX_EINVAL, "null modulus or output");
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = ensure_device();
  if (rc) return rc;
  std::vector<uint32_t> m(m_words, m_words + m_len);
  while (m.size() > 1 && m.back() == 0) m.pop_back();
  const uint32_t bits = bit_length(m);
  if (bits == 0) return fail(MPCX_EINVAL, "modulus is zero");
  if ((m[0] & 1u) == 0) return fail(MPCX_EINVAL, "modulus is even (math/big uses a non-Montgomery path; keep it on the host)");
  const int cls = class_for_bits(bits);
  if (cls < 0) return fail(MPCX_EINVAL, "modulus has %u bits > %d", bits, MPCX_MAX_MODULUS_BITS);
  auto* mod = new mpcx_modulus_s();
  mod->cls = cls;
  mod->bits = bits;
  mod->words = (uint32_t)m.size();
  mod->m = m;
  uint32_t inv = m[0];
  for (int i = 0; i < 5; ++i) inv *= 2u - m[0] * inv;
  mod->n0inv = (0u - inv) & kM28;
  std::vector<uint32_t> host;
  for (int g = 0; g < MPCX_NUM_GEOMS; ++g) {
    mod->const_off[g] = 0;
    if (MPCX_GEOM_CLASS(g) != cls) continue;
    const uint32_t L = (uint32_t)MPCX_GEOM_L(g);
    mod->const_off[g] = (uint32_t)host.size();
    auto nd = to_digits(m, L);
    auto r1 = to_digits(pow2_mod(kDigitBits * L, m), L);
    auto r2 = to_digits(pow2_mod(2 * kDigitBits * L, m), L);
    host.insert(host.end(), nd.begin(), nd.end());
    host.insert(host.end(), r1.begin(), r1.end());
    host.insert(host.end(), r2.begin(), r2.end());
  }
  hipError_t e = hipMalloc((void**)&mod->d_const, host.size() * sizeof(uint32_t));
  if (e != hipSuccess) {
    delete mod;
    return fail(MPCX_ENOMEM, "hipMalloc(modulus): %s", hipGetErrorString(e));
  }
  e = hipMemcpy(mod->d_const, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(mod->d_const);
    delete mod;
    return hip_fail(e, "upload modulus");
  }
  *out = mod;
  return MPCX_OK;
}

int mpcx_modulus_release(mpcx_mod_t mod) {
  if (!mod) return fail(MPCX_EINVAL, "null modulus");
  std::lock_guard<std::mutex> lk(g_mu);
  if (mod->d_const) (void)hipFree(mod->d_const);
  delete mod;
  return MPCX_OK;
}

int mpcx_modulus_info(mpcx_mod_t mod, uint32_t* out_bits, uint32_t* out_class_words) {
  if (!mod) return fail(MPCX_EINVAL, "null modulus");
  if (out_bits) *out_bits = mod->bits;
  if (out_class_words) *out_class_words = (uint32_t)MPCX_CLASS_WORDS(mod->cls);
  return MPCX_OK;
}

int mpcx_modulus_geometry(mpcx_mod_t mod, uint32_t* L, uint32_t* P, uint32_t* K, uint32_t* G) {
  if (!mod) return fail(MPCX_EINVAL, "null modulus");
  const int g = g_main_geom[mod->cls];
  if (L) *L = (uint32_t)MPCX_GEOM_L(g);
  if (P) *P = (uint32_t)MPCX_GEOM_P(g);
  if (K) *K = (uint32_t)MPCX_GEOM_K(g);
  if (G) *G = (uint32_t)MPCX_GEOM_G(g);
  return MPCX_OK;
}

static int modexp_device_locked(Lane& lane, mpcx_mod_t mod, uint32_t count, const uint32_t* d_bases,
                                uint32_t base_words, const uint32_t* d_exps, uint32_t exp_words, int exp_shared,
                                uint32_t exp_bits, const uint32_t* d_muls, uint32_t mul_words, uint32_t* d_out,
                                uint32_t out_words, hipStream_t st) {
  const uint32_t class_words = (uint32_t)MPCX_CLASS_WORDS(mod->cls);
  if (base_words == 0 || base_words > class_words)
    return fail(MPCX_EINVAL, "base_words %u outside [1, %u] (reduce mod m first)", base_words, class_words);
  if (d_muls && (mul_words == 0 || mul_words > class_words))
    return fail(MPCX_EINVAL, "mul_words %u outside [1, %u]", mul_words, class_words);
  if (out_words < mod->words) return fail(MPCX_EINVAL, "out_words %u < modulus words %u", out_words, mod->words);
  if (exp_bits > 32u * exp_words) return fail(MPCX_EINVAL, "exp_bits %u > 32*exp_words", exp_bits);
  if (count == 0) return MPCX_OK;
  if (!d_bases || !d_out || (exp_words && !d_exps)) return fail(MPCX_EINVAL, "null buffer");
  // Geometry plan: whole rounds of resident wavefronts in the main geometry,
  // the partial last round (or a small batch) in the narrow geometry.
  struct Part {
    int geom;
    uint32_t first, count;
  } parts[2];
  int nparts = 0;
  const int gm = g_main_geom[mod->cls], gn = MPCX_NARROW_GEOM(mod->cls);
  if (g_force_geom >= 0 && MPCX_GEOM_CLASS(g_force_geom) == mod->cls) {
    parts[nparts++] = {g_force_geom, 0, count};
  } else {
    const uint32_t G = (uint32_t)MPCX_GEOM_G(gm);
    const double waves = (double)((count + G - 1) / G);
    const double rounds = waves / (double)std::max(1, g_geom_slots[gm]);
    const double full = std::floor(rounds), frac = rounds - full;
    // Measured on MI355X (profiles/r01): a lone wavefront issues v_mad_u64_u32
    // at ~45% of SIMD peak, so tiny batches (< 0.15 of a round) finish sooner
    // spread over the narrow geometry's 3x more wavefronts; from ~0.3 rounds up
    // the main geometry wins, and a narrow tail launch did not pay.
    if (gn >= 0 && rounds < g_narrow_rounds) {
      parts[nparts++] = {gn, 0, count};
    } else if (!g_split || gn < 0 || rounds < 1.0 || frac == 0.0 || frac > 0.75) {
      parts[nparts++] = {gm, 0, count};
    } else {
      const uint32_t nmain = (uint32_t)full * (uint32_t)g_geom_slots[gm] * G;
      parts[nparts++] = {gm, 0, nmain};
      parts[nparts++] = {gn, nmain, count - nmain};
    }
  }
  size_t ws_words = 0;
  for (int i = 0; i < nparts; ++i) {
    const uint32_t G = (uint32_t)MPCX_GEOM_G(parts[i].geom), K = (uint32_t)MPCX_GEOM_K(parts[i].geom);
    ws_words += (size_t)((parts[i].count + G - 1) / G) * MPCX_TABLE_ENTRIES * K * 64u;
  }
  // a shared exponent's sliding-window schedule lives after the tables
  const bool use_sched = exp_shared && exp_bits > 0 && g_sched_width > 0;
  const size_t sched_off = ws_words;
  if (use_sched) ws_words += MPCX_SCHED_WORDS(32u * exp_words);
  int rc = ensure_workspace(lane, ws_words * sizeof(uint32_t));
  if (rc) return rc;
  if (use_sched) {
    mpcx::ExpSchedArgs sa{};
    sa.exp = d_exps;
    sa.exp_words = exp_words;
    sa.max_width = (uint32_t)g_sched_width;
    sa.sched = lane.ws + sched_off;
    hipError_t e = mpcx_launch_expsched(&sa, st);
    if (e != hipSuccess) return hip_fail(e, "launch k_expsched");
  }
  size_t ws_off = 0;
  for (int i = 0; i < nparts; ++i) {
    const Part& pt = parts[i];
    const uint32_t G = (uint32_t)MPCX_GEOM_G(pt.geom), K = (uint32_t)MPCX_GEOM_K(pt.geom);
    const uint32_t waves = (pt.count + G - 1) / G;
    mpcx::ModexpArgs a{};
    const uint32_t L = (uint32_t)MPCX_GEOM_L(pt.geom);
    a.nd = mod->d_const + mod->const_off[pt.geom];
    a.r1d = a.nd + L;
    a.r2d = a.nd + 2 * L;
    a.base = d_bases + (size_t)pt.first * base_words;
    a.exps = exp_shared ? d_exps : (d_exps ? d_exps + (size_t)pt.first * exp_words : nullptr);
    a.mul = d_muls ? d_muls + (size_t)pt.first * mul_words : nullptr;
    a.out = d_out + (size_t)pt.first * out_words;
    a.table = lane.ws + ws_off;
    a.count = pt.count;
    a.base_words = base_words;
    a.exp_words = exp_words;
    a.mul_words = d_muls ? mul_words : 0;
    a.exp_bits = exp_words ? exp_bits : 0;
    a.out_words = out_words;
    a.n0inv = mod->n0inv;
    a.exp_shared = exp_shared ? 1 : 0;
    a.sched = use_sched ? lane.ws + sched_off : nullptr;
    hipError_t e = mpcx_launch_modexp(pt.geom, &a, waves, st);
    if (e != hipSuccess) return hip_fail(e, "launch k_modexp");
    ws_off += (size_t)waves * MPCX_TABLE_ENTRIES * K * 64u;
  }
  return MPCX_OK;
}

static uint32_t max_exp_bits(const uint32_t* exps, uint32_t exp_words, int exp_shared, uint32_t count) {
  uint32_t bits = 0;
  if (!exp_words) return 0;
  if (exp_shared) return bit_length_words(exps, exp_words);
  for (uint32_t i = 0; i < count; ++i) bits = std::max(bits, bit_length_words(exps + (size_t)i * exp_words, exp_words));
  return bits;
}

// host-buffer path: stage inputs, launch, copy back (synchronous)
static int modexp_host(mpcx_mod_t mod, uint32_t count, const uint32_t* bases, uint32_t base_words,
                       const uint32_t* exps, uint32_t exp_words, int exp_shared, const uint32_t* muls,
                       uint32_t mul_words, uint32_t* out, uint32_t out_words) {
  if (!mod) return fail(MPCX_EINVAL, "null modulus");
  if (count == 0) return MPCX_OK;
  if (!bases || !out || (exp_words && !exps)) return fail(MPCX_EINVAL, "null buffer");
  int rc = ensure_device();
  if (rc) return rc;
  const uint32_t exp_bits = max_exp_bits(exps, exp_words, exp_shared, count);
  const size_t n_exp_words = exp_shared ? exp_words : (size_t)count * exp_words;
  const size_t bb = (size_t)count * base_words * 4, eb = std::max<size_t>(n_exp_words * 4, 4),
               ob = (size_t)count * out_words * 4, mb = muls ? (size_t)count * mul_words * 4 : 0;
  std::unique_lock<std::mutex> lk;
  Lane& l = acquire_lane(lk);
  if ((rc = lane_stream(l))) return rc;
  Staging* sg = l.stage;
  if ((rc = ensure_buffer(sg[0], bb)) || (rc = ensure_buffer(sg[1], eb)) || (rc = ensure_buffer(sg[2], ob)) ||
      (muls && (rc = ensure_buffer(sg[3], mb))))
    return rc;
  if ((rc = h2d(sg[0].ptr, bases, bb, l.st)) || (rc = h2d(sg[1].ptr, exps, n_exp_words * 4, l.st)) ||
      (muls && (rc = h2d(sg[3].ptr, muls, mb, l.st))))
    return rc;
  rc = modexp_device_locked(l, mod, count, (const uint32_t*)sg[0].ptr, base_words, (const uint32_t*)sg[1].ptr,
                            exp_words, exp_shared, exp_bits, muls ? (const uint32_t*)sg[3].ptr : nullptr, mul_words,
                            (uint32_t*)sg[2].ptr, out_words, l.st);
  if (rc) return rc;
  return d2h_sync(out, sg[2].ptr, ob, l.st);
}

int mpcx_modexp_batch_device(mpcx_mod_t mod, uint32_t count, const uint32_t* d_bases, uint32_t base_words,
                             const uint32_t* d_exps, uint32_t exp_words, int exp_shared, uint32_t exp_bits,
                             uint32_t* d_out, uint32_t out_words, void* stream) {
  if (!mod) return fail(MPCX_EINVAL, "null modulus");
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = ensure_device();
  if (rc) return rc;
  return modexp_device_locked(g_dev_lane, mod, count, d_bases, base_words, d_exps, exp_words, exp_shared, exp_bits,
                              nullptr, 0, d_out, out_words, (hipStream_t)stream);
}

int mpcx_modexp_mul_batch_device(mpcx_mod_t mod, uint32_t count, const uint32_t* d_bases, uint32_t base_words,
                                 const uint32_t* d_exps, uint32_t exp_words, int exp_shared, uint32_t exp_bits,
                                 const uint32_t* d_muls, uint32_t mul_words, uint32_t* d_out, uint32_t out_words,
                                 void* stream) {
  if (!mod) return fail(MPCX_EINVAL, "null modulus");
  if (!d_muls) return fail(MPCX_EINVAL, "null multipliers");
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = ensure_device();
  if (rc) return rc;
  return modexp_device_locked(g_dev_lane, mod, count, d_bases, base_words, d_exps, exp_words, exp_shared, exp_bits,
                              d_muls, mul_words, d_out, out_words, (hipStream_t)stream);
}

int mpcx_modexp_batch(mpcx_mod_t mod, uint32_t count, const uint32_t* bases, uint32_t base_words,
                      const uint32_t* exps, uint32_t exp_words, int exp_shared, uint32_t* out,
                      uint32_t out_words) {
  return modexp_host(mod, count, bases, base_words, exps, exp_words, exp_shared, nullptr, 0, out, out_words);
}

int mpcx_modexp_mul_batch(mpcx_mod_t mod, uint32_t count, const uint32_t* bases, uint32_t base_words,
                          const uint32_t* exps, uint32_t exp_words, int exp_shared, const uint32_t* muls,
                          uint32_t mul_words, uint32_t* out, uint32_t out_words) {
  if (!muls) return fail(MPCX_EINVAL, "null multipliers");
  return modexp_host(mod, count, bases, base_words, exps, exp_words, exp_shared, muls, mul_words, out, out_words);
}

int mpcx_mulmod_batch(mpcx_mod_t mod, uint32_t count, const uint32_t* a, uint32_t a_words, const uint32_t* b,
                      uint32_t b_words, uint32_t* out, uint32_t out_words) {
  if (!a || !b) return fail(MPCX_EINVAL, "null operands");
  const uint32_t one = 1;
  return modexp_host(mod, count, a, a_words, &one, 1, 1, b, b_words, out, out_words);
}

int mpcx_fermat2_batch(uint32_t count, const uint32_t* p, uint32_t p_words, uint8_t* ok) {
  if (count == 0) return MPCX_OK;
  if (!p || !ok || p_words == 0) return fail(MPCX_EINVAL, "null buffer");
  if (p_words > (uint32_t)MPCX_CLASS_WORDS(0))
    return fail(MPCX_EINVAL, "p_words %u > %d", p_words, MPCX_CLASS_WORDS(0));
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t* pi = p + (size_t)i * p_words;
    const uint32_t bits = bit_length_words(pi, p_words);
    if (bits > (uint32_t)MPCX_CLASS_MAXBITS(0))
      return fail(MPCX_EINVAL, "candidate %u has %u bits > %d", i, bits, MPCX_CLASS_MAXBITS(0));
    if (bits < 3 || (pi[0] & 1u) == 0) return fail(MPCX_EINVAL, "candidate %u is not an odd integer >= 5", i);
  }
  int rc = ensure_device();
  if (rc) return rc;
  std::unique_lock<std::mutex> lk;
  Lane& l = acquire_lane(lk);
  if ((rc = lane_stream(l))) return rc;
  const size_t pb = (size_t)count * p_words * 4;
  if ((rc = ensure_buffer(l.stage[0], pb)) || (rc = ensure_buffer(l.stage[3], count))) return rc;
  if ((rc = h2d(l.stage[0].ptr, p, pb, l.st))) return rc;
  mpcx::FermatArgs a{};
  a.p = (const uint32_t*)l.stage[0].ptr;
  a.ok = (uint8_t*)l.stage[3].ptr;
  a.count = count;
  a.p_words = p_words;
  hipError_t e = mpcx_launch_fermat2(&a, (count + 63) / 64, l.st);
  if (e != hipSuccess) return hip_fail(e, "launch k_fermat2");
  return d2h_sync(ok, l.stage[3].ptr, count, l.st);
}

int mpcx_mr_batch(uint32_t count, const uint32_t* n, uint32_t n_words, const uint32_t* bases, uint8_t* ok) {
  if (count == 0) return MPCX_OK;
  if (!n || !bases || !ok || n_words == 0) return fail(MPCX_EINVAL, "null buffer");
  if (n_words > (uint32_t)MPCX_CLASS_WORDS(0))
    return fail(MPCX_EINVAL, "n_words %u > %d", n_words, MPCX_CLASS_WORDS(0));
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t* ni = n + (size_t)i * n_words;
    if (bit_length_words(ni, n_words) < 3 || (ni[0] & 1u) == 0)
      return fail(MPCX_EINVAL, "candidate %u is not an odd integer >= 5", i);
  }
  int rc = ensure_device();
  if (rc) return rc;
  std::unique_lock<std::mutex> lk;
  Lane& l = acquire_lane(lk);
  if ((rc = lane_stream(l))) return rc;
  const size_t nb = (size_t)count * n_words * 4;
  if ((rc = ensure_buffer(l.stage[0], nb)) || (rc = ensure_buffer(l.stage[1], nb)) ||
      (rc = ensure_buffer(l.stage[3], count)))
    return rc;
  if ((rc = h2d(l.stage[0].ptr, n, nb, l.st)) || (rc = h2d(l.stage[1].ptr, bases, nb, l.st))) return rc;
  mpcx::MrArgs a{};
  a.n = (const uint32_t*)l.stage[0].ptr;
  a.a = (const uint32_t*)l.stage[1].ptr;
  a.ok = (uint8_t*)l.stage[3].ptr;
  a.count = count;
  a.n_words = n_words;
  hipError_t e = mpcx_launch_mr(&a, (count + 63) / 64, l.st);
  if (e != hipSuccess) return hip_fail(e, "launch k_mr");
  return d2h_sync(ok, l.stage[3].ptr, count, l.st);
}

int mpcx_dev_alloc(size_t bytes, void** out_ptr) {
  if (!out_ptr) return fail(MPCX_EINVAL, "null out_ptr");
  if (int rc = ensure_device()) return rc;
  hipError_t e = hipMalloc(out_ptr, bytes);
  if (e != hipSuccess) return fail(MPCX_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  return MPCX_OK;
}

int mpcx_dev_free(void* ptr) {
  hipError_t e = hipFree(ptr);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "hipFree");
}

int mpcx_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes) {
  hipError_t e = hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "hipMemcpy H2D");
}

int mpcx_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes) {
  hipError_t e = hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "hipMemcpy D2H");
}

int mpcx_stream_create(void** out_stream) {
  if (!out_stream) return fail(MPCX_EINVAL, "null out_stream");
  hipStream_t s;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
  *out_stream = (void*)s;
  return MPCX_OK;
}

int mpcx_stream_destroy(void* stream) {
  hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "hipStreamDestroy");
}

int mpcx_stream_sync(void* stream) {
  hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  return e == hipSuccess ? MPCX_OK : hip_fail(e, "hipStreamSynchronize");
}

}  // extern "C"

// ------------------------------------------------------------ fixed base
// Comb tables for a long-lived base (h1, h2 of a node's N~; SURVEY.md 8(a)
// "shared bases"): entry (j, v) = b^(v 2^(8j)) R mod m. Built on the GPU by
// the modexp kernels: b_j = b^(2^(8j)) (per-operand exponents), then
// T(j, v) = (R mod m) * b_j^v (fused multiplier), then reordered into the
// kernel geometry's digit layout on the host.
int mpcx_fixedbase_register(mpcx_mod_t mod, const uint32_t* base, uint32_t base_words, uint32_t max_exp_bits,
                            mpcx_fb_t* out) {
  if (!mod || !base || !out) return fail(MPCX_EINVAL, "null argument");
  if (mod->cls > 1) return fail(MPCX_EINVAL, "fixed-base tables serve moduli of <= %d bits", MPCX_CLASS_MAXBITS(1));
  const uint32_t cw = (uint32_t)MPCX_CLASS_WORDS(mod->cls);
  if (base_words == 0 || base_words > cw) return fail(MPCX_EINVAL, "base_words %u outside [1, %u]", base_words, cw);
  if (max_exp_bits == 0 || max_exp_bits > 65536) return fail(MPCX_EINVAL, "max_exp_bits %u outside [1, 65536]", max_exp_bits);
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = ensure_device();
  if (rc) return rc;
  // the build reuses the device-buffer workspace on the null stream: drain
  // any device-buffer call still reading it on a caller's stream (rare: once
  // per long-lived base)
  (void)hipDeviceSynchronize();
  const int geom = MPCX_MAIN_GEOM(mod->cls);
  const uint32_t L = (uint32_t)MPCX_GEOM_L(geom), P = (uint32_t)MPCX_GEOM_P(geom), K = (uint32_t)MPCX_GEOM_K(geom);
  const uint32_t nwin = (max_exp_bits + MPCX_FB_WINDOW_BITS - 1) / MPCX_FB_WINDOW_BITS;
  const uint32_t nv = MPCX_FB_ENTRIES - 1;  // v = 1..255 computed; v = 0 is R mod m
  const size_t n2 = (size_t)nwin * nv;
  if (n2 > 0xFFFFFFFFull) return fail(MPCX_EINVAL, "table too large");
  const uint32_t ew1 = (MPCX_FB_WINDOW_BITS * (nwin - 1)) / 32 + 1;  // 2^(8j) needs bit 8j
  // host inputs
  std::vector<uint32_t> hb((size_t)nwin * cw, 0), he1((size_t)nwin * ew1, 0);
  for (uint32_t j = 0; j < nwin; ++j) {
    std::memcpy(&hb[(size_t)j * cw], base, base_words * 4);
    const uint32_t bit = MPCX_FB_WINDOW_BITS * j;
    he1[(size_t)j * ew1 + bit / 32] = 1u << (bit % 32);
  }
  const std::vector<uint32_t> r1w = pow2_mod(kDigitBits * L, mod->m);  // R mod m, mod->words words
  std::vector<uint32_t> he2(n2), hm(n2 * mod->words);
  for (size_t i = 0; i < n2; ++i) {
    he2[i] = (uint32_t)(i % nv) + 1u;
    std::memcpy(&hm[i * mod->words], r1w.data(), mod->words * 4);
  }
  uint32_t *d_b = nullptr, *d_e1 = nullptr, *d_bj = nullptr, *d_e2 = nullptr, *d_m = nullptr, *d_t = nullptr;
  auto cleanup = [&] {
    for (uint32_t* ptr : {d_b, d_e1, d_bj, d_e2, d_m, d_t})
      if (ptr) (void)hipFree(ptr);
  };
  auto alloc = [&](uint32_t** ptr, size_t words) {
    return hipMalloc((void**)ptr, std::max<size_t>(words, 1) * 4) == hipSuccess;
  };
  if (!alloc(&d_b, hb.size()) || !alloc(&d_e1, he1.size()) || !alloc(&d_bj, (size_t)nwin * cw) ||
      !alloc(&d_e2, n2) || !alloc(&d_m, hm.size()) || !alloc(&d_t, n2 * cw)) {
    cleanup();
    return fail(MPCX_ENOMEM, "hipMalloc(fixed-base build)");
  }
  hipError_t e = hipMemcpy(d_b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_e1, he1.data(), he1.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_e2, he2.data(), he2.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_m, hm.data(), hm.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    cleanup();
    return hip_fail(e, "upload fixed-base inputs");
  }
  rc = modexp_device_locked(g_dev_lane, mod, nwin, d_b, cw, d_e1, ew1, 0, MPCX_FB_WINDOW_BITS * (nwin - 1) + 1,
                            nullptr, 0, d_bj, cw, nullptr);
  // T(j, v) = R * b_j^v: operand i = j*255 + (v-1) takes base b_j -> replicate b_j rows
  std::vector<uint32_t> hbj((size_t)nwin * cw), hb2;
  if (!rc) {
    e = hipMemcpy(hbj.data(), d_bj, hbj.size() * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = hip_fail(e, "copy b_j");
  }
  if (!rc) {
    hb2.resize(n2 * cw);
    for (size_t i = 0; i < n2; ++i) std::memcpy(&hb2[i * cw], &hbj[(i / nv) * cw], cw * 4);
    (void)hipFree(d_b);
    d_b = nullptr;
    if (!alloc(&d_b, hb2.size())) rc = fail(MPCX_ENOMEM, "hipMalloc(fixed-base bases)");
  }
  if (!rc) {
    e = hipMemcpy(d_b, hb2.data(), hb2.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) rc = hip_fail(e, "upload b_j");
  }
  if (!rc)
    rc = modexp_device_locked(g_dev_lane, mod, (uint32_t)n2, d_b, cw, d_e2, 1, 0, MPCX_FB_WINDOW_BITS, d_m,
                              mod->words, d_t, cw, nullptr);
  std::vector<uint32_t> ht(n2 * cw);
  if (!rc) {
    e = hipMemcpy(ht.data(), d_t, ht.size() * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = hip_fail(e, "copy table");
  }
  cleanup();
  if (rc) return rc;
  // digits, [k][p] interleaved per entry
  const size_t ent_words = L;
  std::vector<uint32_t> tab((size_t)nwin * MPCX_FB_ENTRIES * ent_words);
  auto put = [&](size_t ent, const std::vector<uint32_t>& words) {
    const std::vector<uint32_t> d = to_digits(words, L);
    uint32_t* dst = &tab[ent * ent_words];
    for (uint32_t pp = 0; pp < P; ++pp)
      for (uint32_t k = 0; k < K; ++k) dst[k * P + pp] = d[pp * K + k];
  };
  std::vector<uint32_t> w(cw);
  for (uint32_t j = 0; j < nwin; ++j) {
    put((size_t)j * MPCX_FB_ENTRIES, r1w);
    for (uint32_t v = 1; v < MPCX_FB_ENTRIES; ++v) {
      std::memcpy(w.data(), &ht[((size_t)j * nv + (v - 1)) * cw], cw * 4);
      put((size_t)j * MPCX_FB_ENTRIES + v, w);
    }
  }
  auto* fb = new mpcx_fixedbase_s();
  fb->mod = mod;
  fb->geom = geom;
  fb->nwin = nwin;
  e = hipMalloc((void**)&fb->d_table, tab.size() * 4);
  if (e != hipSuccess) {
    delete fb;
    return fail(MPCX_ENOMEM, "hipMalloc(fixed-base table %zu B)", tab.size() * 4);
  }
  e = hipMemcpy(fb->d_table, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(fb->d_table);
    delete fb;
    return hip_fail(e, "upload fixed-base table");
  }
  *out = fb;
  return MPCX_OK;
}

int mpcx_fixedbase_release(mpcx_fb_t fb) {
  if (!fb) return fail(MPCX_EINVAL, "null fixed base");
  std::lock_guard<std::mutex> lk(g_mu);
  if (fb->d_table) (void)hipFree(fb->d_table);
  delete fb;
  return MPCX_OK;
}

int mpcx_fixedbase_info(mpcx_fb_t fb, uint32_t* max_exp_bits, size_t* table_bytes) {
  if (!fb) return fail(MPCX_EINVAL, "null fixed base");
  if (max_exp_bits) *max_exp_bits = fb->nwin * MPCX_FB_WINDOW_BITS;
  if (table_bytes) *table_bytes = (size_t)fb->nwin * MPCX_FB_ENTRIES * MPCX_GEOM_L(fb->geom) * 4;
  return MPCX_OK;
}

int mpcx_fixedbase_exp_batch(uint32_t nbases, const mpcx_fb_t* fbs, uint32_t count, const uint32_t* const* exps,
                             const uint32_t* exp_words, const uint32_t* muls, uint32_t mul_words, uint32_t* out,
                             uint32_t out_words) {
  if (nbases == 0 || nbases > MPCX_FB_MAX_BASES) return fail(MPCX_EINVAL, "nbases %u outside [1, %d]", nbases, MPCX_FB_MAX_BASES);
  if (!fbs || !exps || !exp_words) return fail(MPCX_EINVAL, "null argument");
  for (uint32_t t = 0; t < nbases; ++t) {
    if (!fbs[t]) return fail(MPCX_EINVAL, "null fixed base %u", t);
    if (fbs[t]->mod != fbs[0]->mod) return fail(MPCX_EINVAL, "fixed bases of different moduli");
  }
  mpcx_mod_t mod = fbs[0]->mod;
  const uint32_t cw = (uint32_t)MPCX_CLASS_WORDS(mod->cls);
  if (out_words < mod->words) return fail(MPCX_EINVAL, "out_words %u < modulus words %u", out_words, mod->words);
  if (muls && (mul_words == 0 || mul_words > cw)) return fail(MPCX_EINVAL, "mul_words %u outside [1, %u]", mul_words, cw);
  if (count == 0) return MPCX_OK;
  if (!out) return fail(MPCX_EINVAL, "null output");
  uint32_t nwin[MPCX_FB_MAX_BASES] = {0, 0};
  for (uint32_t t = 0; t < nbases; ++t) {
    if (exp_words[t] && !exps[t]) return fail(MPCX_EINVAL, "null exponents %u", t);
    uint32_t bits = 0;
    for (uint32_t i = 0; i < count && exp_words[t]; ++i)
      bits = std::max(bits, bit_length_words(exps[t] + (size_t)i * exp_words[t], exp_words[t]));
    if (bits > fbs[t]->nwin * MPCX_FB_WINDOW_BITS)
      return fail(MPCX_EINVAL, "exponent of %u bits > fixed-base table's %u", bits, fbs[t]->nwin * MPCX_FB_WINDOW_BITS);
    nwin[t] = (bits + MPCX_FB_WINDOW_BITS - 1) / MPCX_FB_WINDOW_BITS;
  }
  int rc = ensure_device();
  if (rc) return rc;
  const size_t eb0 = (size_t)count * exp_words[0] * 4, eb1 = nbases > 1 ? (size_t)count * exp_words[1] * 4 : 0,
               ob = (size_t)count * out_words * 4, mb = muls ? (size_t)count * mul_words * 4 : 0;
  std::unique_lock<std::mutex> lk;
  Lane& l = acquire_lane(lk);
  if ((rc = lane_stream(l))) return rc;
  Staging* sg = l.stage;
  if ((rc = ensure_buffer(sg[0], eb0)) || (rc = ensure_buffer(sg[1], eb1)) ||
      (rc = ensure_buffer(sg[2], ob)) || (muls && (rc = ensure_buffer(sg[3], mb))))
    return rc;
  if ((rc = h2d(sg[0].ptr, exps[0], eb0, l.st)) || (rc = h2d(sg[1].ptr, exps[1], eb1, l.st)) ||
      (muls && (rc = h2d(sg[3].ptr, muls, mb, l.st))))
    return rc;
  hipError_t e;
  const int geom = fbs[0]->geom;
  mpcx::FixedBaseArgs a{};
  a.nd = mod->d_const + mod->const_off[geom];
  a.r1d = a.nd + MPCX_GEOM_L(geom);
  a.r2d = a.nd + 2 * MPCX_GEOM_L(geom);
  for (uint32_t t = 0; t < nbases; ++t) {
    a.tables[t] = fbs[t]->d_table;
    a.exps[t] = (const uint32_t*)sg[t].ptr;
    a.exp_words[t] = exp_words[t];
    a.nwin[t] = nwin[t];
  }
  a.nbases = nbases;
  a.mul = muls ? (const uint32_t*)sg[3].ptr : nullptr;
  a.mul_words = muls ? mul_words : 0;
  a.out = (uint32_t*)sg[2].ptr;
  a.out_words = out_words;
  a.count = count;
  a.n0inv = mod->n0inv;
  const uint32_t waves = (count + MPCX_GEOM_G(geom) - 1) / MPCX_GEOM_G(geom);
  e = geom == MPCX_MAIN_GEOM(0) ? mpcx_launch_fixedbase_g0(&a, waves, l.st)
                                : mpcx_launch_fixedbase_g1(&a, waves, l.st);
  if (e != hipSuccess) return hip_fail(e, "launch k_fixedbase");
  return d2h_sync(out, sg[2].ptr, ob, l.st);
}

// ------------------------------------------------------------ safe-prime sieve
namespace {
// trial-division groups: primes 59..2039 packed into products < 2^32 (the
// host sieve's grouping, csrc/host/safeprime.cpp)
struct TrialTables {
  std::vector<uint32_t> prod, start, primes;
  std::vector<uint64_t> inv;
  TrialTables() {
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
    start.push_back(0);
    for (uint32_t p : ps) {
      if (cur * p >= (1ull << 32)) {
        prod.push_back((uint32_t)cur);
        start.push_back((uint32_t)primes.size());
        cur = 1;
      }
      cur *= p;
      primes.push_back(p);
    }
    prod.push_back((uint32_t)cur);
    start.push_back((uint32_t)primes.size());
    for (uint32_t d : prod) inv.push_back(~0ull / d);
  }
};
}  // namespace

int mpcx_safeprime_sieve_fermat(const uint8_t* raw, uint32_t nbytes, uint32_t count, uint32_t q_bits,
                                uint32_t* n_out, uint32_t* idx_out, uint8_t* ok_out) {
  if (!n_out) return fail(MPCX_EINVAL, "null n_out");
  *n_out = 0;
  if (q_bits < 63 || q_bits > 1023) return fail(MPCX_EINVAL, "q_bits %u outside [63, 1023]", q_bits);
  if (nbytes != (q_bits + 7) / 8) return fail(MPCX_EINVAL, "nbytes %u != (q_bits + 7) / 8", nbytes);
  if (count == 0) return MPCX_OK;
  if (!raw || !idx_out || !ok_out) return fail(MPCX_EINVAL, "null buffer");
  static const TrialTables tt;
  int rc = ensure_device();
  if (rc) return rc;
  std::unique_lock<std::mutex> lk;
  Lane& l = acquire_lane(lk);
  if ((rc = lane_stream(l))) return rc;
  Staging *sg = l.stage, *sv = l.sieve;
  constexpr uint32_t W = MPCX_SIEVE_MAX_BYTES / 4;
  const size_t ng = tt.prod.size();
  // misc buffer: counter | prod | start | primes | inv (8-byte aligned)
  const size_t off_prod = 2, off_start = off_prod + ng, off_primes = off_start + tt.start.size();
  const size_t off_inv = (off_primes + tt.primes.size() + 1) / 2 * 2;
  const size_t misc_words = off_inv + 2 * ng;
  if ((rc = ensure_buffer(sg[0], (size_t)count * nbytes)) || (rc = ensure_buffer(sg[3], count)) ||
      (rc = ensure_buffer(sv[0], (size_t)count * W * 4)) || (rc = ensure_buffer(sv[1], (size_t)count * 4)) ||
      (rc = ensure_buffer(sv[2], misc_words * 4)))
    return rc;
  std::vector<uint32_t> misc(misc_words, 0);
  std::copy(tt.prod.begin(), tt.prod.end(), misc.begin() + off_prod);
  std::copy(tt.start.begin(), tt.start.end(), misc.begin() + off_start);
  std::copy(tt.primes.begin(), tt.primes.end(), misc.begin() + off_primes);
  std::memcpy(misc.data() + off_inv, tt.inv.data(), ng * 8);
  if ((rc = h2d(sv[2].ptr, misc.data(), misc_words * 4, l.st)) ||
      (rc = h2d(sg[0].ptr, raw, (size_t)count * nbytes, l.st)))
    return rc;
  uint32_t* dm = (uint32_t*)sv[2].ptr;
  mpcx::SieveArgs sa{};
  sa.raw = (const uint8_t*)sg[0].ptr;
  sa.nbytes = nbytes;
  sa.count = count;
  sa.q_bits = q_bits;
  sa.tprod = dm + off_prod;
  sa.tstart = dm + off_start;
  sa.tprimes = dm + off_primes;
  sa.tinv = (const uint64_t*)(dm + off_inv);
  sa.ngroups = (uint32_t)ng;
  sa.out_p = (uint32_t*)sv[0].ptr;
  sa.out_idx = (uint32_t*)sv[1].ptr;
  sa.out_count = dm;
  hipError_t e = mpcx_launch_sieve(&sa, l.st);
  if (e != hipSuccess) return hip_fail(e, "launch k_sieve");
  mpcx::FermatArgs fa{};
  fa.p = sa.out_p;
  fa.ok = (uint8_t*)sg[3].ptr;
  fa.count = count;
  fa.p_words = W;
  fa.count_dev = dm;
  e = mpcx_launch_fermat2(&fa, (count + 63) / 64, l.st);
  if (e != hipSuccess) return hip_fail(e, "launch k_fermat2");
  uint32_t n = 0;
  if ((rc = d2h_sync(&n, dm, 4, l.st))) return rc;
  if (n > count) return fail(MPCX_EHIP, "sieve survivor count %u > %u", n, count);
  std::vector<uint32_t> idx(n);
  std::vector<uint8_t> ok(n);
  if (n) {
    e = hipMemcpyAsync(idx.data(), sa.out_idx, (size_t)n * 4, hipMemcpyDeviceToHost, l.st);
    if (e != hipSuccess) return hip_fail(e, "copy survivors");
    if ((rc = d2h_sync(ok.data(), fa.ok, n, l.st))) return rc;
  }
  // stream order
  std::vector<uint32_t> ord(n);
  for (uint32_t j = 0; j < n; ++j) ord[j] = j;
  std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return idx[x] < idx[y]; });
  for (uint32_t j = 0; j < n; ++j) {
    idx_out[j] = idx[ord[j]];
    ok_out[j] = ok[ord[j]];
  }
  *n_out = n;
  return MPCX_OK;
}
