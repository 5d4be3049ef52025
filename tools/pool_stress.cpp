// Host worker-pool stress under ThreadSanitizer (CPU only): 12 threads issue
// nested parallel_for loops of random shapes, 30 rounds (tools/pool_tsan.sh).
#include <atomic>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>
#include "tsscommon.hpp"
using namespace mpcx::host;
int main() {
  std::atomic<uint64_t> total{0};
  for (int rep = 0; rep < 30; ++rep) {
    std::vector<std::thread> th;
    for (int t = 0; t < 12; ++t)
      th.emplace_back([&, t] {
        std::mt19937 rng(rep * 100 + t);
        for (int it = 0; it < 20; ++it) {
          size_t outer = rng() % 40, inner = rng() % 24;
          parallel_for(outer, [&](size_t o) {
            parallel_for(inner, [&](size_t i) { total += (o + 1) * (i + 1); });
          });
        }
      });
    for (auto& x : th) x.join();
  }
  std::printf("total %llu\n", (unsigned long long)total.load());
  return 0;
}
