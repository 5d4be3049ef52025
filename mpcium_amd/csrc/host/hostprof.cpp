// hostprof.cpp -- see hostprof.hpp.
#include "hostprof.hpp"

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <mutex>
#include <vector>

namespace mpcx::host::prof {
namespace {
constexpr int kSlots = 128;
std::atomic<uint64_t> g_ns[kSlots];
std::atomic<uint64_t> g_calls[kSlots];
const char* g_label[kSlots];
int g_n = 0;
std::mutex g_mu;
}  // namespace

bool enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MPCX_HOST_PROFILE");
    return e && e[0] == '1';
  }();
  return on;
}

int slot_of(const char* label) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (int i = 0; i < g_n; ++i)
    if (std::strcmp(g_label[i], label) == 0) return i;
  if (g_n >= kSlots) return kSlots - 1;
  g_label[g_n] = label;
  return g_n++;
}

uint64_t thread_cpu_ns() {
  timespec ts{};
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

namespace {
thread_local int t_chain = -1;
std::mutex g_tr_mu;
FILE* trace_file() {
  static FILE* f = [] {
    const char* p = std::getenv("MPCX_HOST_TRACE");
    FILE* h = p && *p ? std::fopen(p, "w") : nullptr;
    if (h) std::fprintf(h, "chain,kind,n,t0_ns,t1_ns\n");
    return h;
  }();
  return f;
}
}  // namespace

bool trace_on() {
  static const bool on = trace_file() != nullptr;
  return on;
}
uint64_t now_ns() {
  timespec ts{};
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
void set_chain(int c) { t_chain = c; }
int chain() { return t_chain; }
void trace(const char* kind, uint64_t t0, uint64_t t1, int64_t n) {
  FILE* f = trace_file();
  if (!f) return;
  std::lock_guard<std::mutex> lk(g_tr_mu);
  std::fprintf(f, "%d,%s,%lld,%llu,%llu\n", t_chain, kind, (long long)n, (unsigned long long)t0,
               (unsigned long long)t1);
}

void add(int slot, uint64_t ns) {
  g_ns[slot].fetch_add(ns, std::memory_order_relaxed);
  g_calls[slot].fetch_add(1, std::memory_order_relaxed);
}


// ---------------------------------------------------------------- sampler
// MPCX_HOST_SAMPLE=<hz> with MPCX_HOST_SAMPLE_OUT=<file>: SIGPROF (process
// CPU time, so samples land on whichever thread burns CPU) records a call
// stack per tick; reset() (re)arms it, report() stops it and writes
// <file>.<k> (k counts the reports), one line per distinct stack, "count module+0xoff@dynsym;..." innermost first,
// for tools/host_samples.py to symbolize (addr2line on the same build).
namespace {
constexpr int kDepth = 24;
constexpr size_t kMaxSamples = 1 << 18;
struct Sample {
  int n;
  void* pc[kDepth];
};
Sample* g_samples = nullptr;
std::atomic<size_t> g_nsamp{0};
std::atomic<bool> g_armed{false};

int sample_hz() {
  static const int hz = [] {
    const char* e = std::getenv("MPCX_HOST_SAMPLE");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  return hz;
}

void on_prof(int, siginfo_t*, void*) {
  if (!g_armed.load(std::memory_order_relaxed)) return;
  const int saved = errno;
  const size_t i = g_nsamp.fetch_add(1, std::memory_order_relaxed);
  if (i < kMaxSamples) g_samples[i].n = backtrace(g_samples[i].pc, kDepth);
  errno = saved;
}

void set_timer(int hz) {
  itimerval it{};
  if (hz > 0) {
    it.it_interval.tv_usec = 1000000 / hz;
    it.it_value = it.it_interval;
  }
  setitimer(ITIMER_PROF, &it, nullptr);
}

void sampler_arm() {
  const int hz = sample_hz();
  if (hz <= 0) return;
  if (!g_samples) {
    g_samples = new Sample[kMaxSamples];
    void* warm[4];
    (void)backtrace(warm, 4);  // loads the unwinder outside the handler
    struct sigaction sa {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGPROF, &sa, nullptr);
  }
  g_nsamp = 0;
  g_armed = true;
  set_timer(hz);
}

void sampler_dump() {
  const char* path = std::getenv("MPCX_HOST_SAMPLE_OUT");
  if (sample_hz() <= 0 || !g_samples || !g_armed.exchange(false)) return;
  set_timer(0);
  const size_t n = std::min(g_nsamp.load(), kMaxSamples);
  std::map<std::vector<void*>, uint64_t> stacks;
  for (size_t i = 0; i < n; ++i) {
    const Sample& s = g_samples[i];
    // frames 0-1: this handler and the signal trampoline
    if (s.n > 2) ++stacks[std::vector<void*>(s.pc + 2, s.pc + s.n)];
  }
  static int seq = 0;
  const std::string file = path ? std::string(path) + "." + std::to_string(seq++) : std::string();
  std::FILE* f = path ? std::fopen(file.c_str(), "w") : nullptr;
  if (!f) return;
  std::map<void*, std::string> names;
  for (const auto& kv : stacks) {
    std::fprintf(f, "%llu ", (unsigned long long)kv.second);
    for (size_t j = 0; j < kv.first.size(); ++j) {
      void* pc = kv.first[j];
      auto it = names.find(pc);
      if (it == names.end()) {
        Dl_info di{};
        char buf[512];
        // return addresses point after the call: -1 lands inside it
        if (dladdr(pc, &di) && di.dli_fname)
          std::snprintf(buf, sizeof buf, "%s+0x%llx@%s", di.dli_fname,
                        (unsigned long long)((char*)pc - (char*)di.dli_fbase - (j ? 1 : 0)),
                        di.dli_sname ? di.dli_sname : "");
        else
          std::snprintf(buf, sizeof buf, "?+0x%llx", (unsigned long long)(uintptr_t)pc);
        it = names.emplace(pc, buf).first;
      }
      std::fprintf(f, "%s%s", j ? ";" : "", it->second.c_str());
    }
    std::fputc('\n', f);
  }
  std::fclose(f);
}
}  // namespace

void reset() {
  sampler_arm();
  for (int i = 0; i < kSlots; ++i) {
    g_ns[i] = 0;
    g_calls[i] = 0;
  }
}

std::string report() {
  sampler_dump();
  std::vector<int> idx;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (int i = 0; i < g_n; ++i) idx.push_back(i);
  }
  std::sort(idx.begin(), idx.end(), [](int a, int b) { return g_ns[a].load() > g_ns[b].load(); });
  std::string out;
  char line[256];
  for (int i : idx) {
    if (!g_calls[i].load()) continue;
    std::snprintf(line, sizeof line, "%s: %.4f s (%llu)\n", g_label[i], (double)g_ns[i].load() * 1e-9,
                  (unsigned long long)g_calls[i].load());
    out += line;
  }
  return out;
}

}  // namespace mpcx::host::prof
