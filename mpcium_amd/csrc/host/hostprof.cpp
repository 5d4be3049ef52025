// hostprof.cpp -- see hostprof.hpp.
#include "hostprof.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
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

void add(int slot, uint64_t ns) {
  g_ns[slot].fetch_add(ns, std::memory_order_relaxed);
  g_calls[slot].fetch_add(1, std::memory_order_relaxed);
}

void reset() {
  for (int i = 0; i < kSlots; ++i) {
    g_ns[i] = 0;
    g_calls[i] = 0;
  }
}

std::string report() {
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
