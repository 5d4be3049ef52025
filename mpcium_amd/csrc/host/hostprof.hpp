// hostprof.hpp -- opt-in host-side time accounting (MPCX_HOST_PROFILE=1):
// scoped timers summed per label over all threads, to see where the host
// share of a protocol batch goes (hashing, random draws, gcds, packing, ...).
// Off by default: one relaxed load per scope.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <string>

namespace mpcx::host::prof {

bool enabled();
void add(int slot, uint64_t ns);
int slot_of(const char* label);  // registers the label on first use
std::string report();            // "label: seconds (calls)" lines, largest first
void reset();

class Scope {
 public:
  explicit Scope(int slot) : slot_(enabled() ? slot : -1) {
    if (slot_ >= 0) t0_ = std::chrono::steady_clock::now();
  }
  ~Scope() {
    if (slot_ >= 0)
      add(slot_, (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0_)
                     .count());
  }

 private:
  int slot_;
  std::chrono::steady_clock::time_point t0_;
};

// CPU seconds of the calling thread (CLOCK_THREAD_CPUTIME_ID)
uint64_t thread_cpu_ns();

// CPU time (not wall time) of this thread from construction to destruction,
// summed under `slot`: wraps a thread's entry function so the report splits
// the process's CPU by thread role (pool workers, protocol tasks, launch
// threads); whatever the roles do not cover is the HIP runtime's and Python's.
class ThreadCpu {
 public:
  explicit ThreadCpu(int slot) : slot_(enabled() ? slot : -1), t0_(slot_ >= 0 ? thread_cpu_ns() : 0) {}
  ~ThreadCpu() {
    if (slot_ >= 0) add(slot_, thread_cpu_ns() - t0_);
  }

 private:
  int slot_;
  uint64_t t0_;
};

// ---- timeline (MPCX_HOST_TRACE=<file>): one CSV line per traced interval,
// "chain,kind,n,t0_ns,t1_ns" on the steady clock (CLOCK_MONOTONIC, the clock
// libmpcx's MPCX_KTRACE kernel lines use), so a run's protocol chains can be
// laid against the kernels they waited for (tools/timeline.py). The chain tag
// is thread-local; run_concurrently hands it to its launch threads.
bool trace_on();
uint64_t now_ns();
void set_chain(int chain);
int chain();
void trace(const char* kind, uint64_t t0_ns, uint64_t t1_ns, int64_t n);
class TraceScope {
 public:
  TraceScope(const char* kind, int64_t n) : kind_(trace_on() ? kind : nullptr), n_(n), t0_(kind_ ? now_ns() : 0) {}
  ~TraceScope() {
    if (kind_) trace(kind_, t0_, now_ns(), n_);
  }

 private:
  const char* kind_;
  int64_t n_;
  uint64_t t0_;
};

}  // namespace mpcx::host::prof

#define MPCX_PROF_CAT2(a, b) a##b
#define MPCX_PROF_CAT(a, b) MPCX_PROF_CAT2(a, b)
// MPCX_PROF("label"): time the rest of the enclosing scope under `label`
#define MPCX_PROF(label)                                                       \
  static const int MPCX_PROF_CAT(mpcx_prof_slot_, __LINE__) = ::mpcx::host::prof::slot_of(label); \
  ::mpcx::host::prof::Scope MPCX_PROF_CAT(mpcx_prof_scope_, __LINE__)(MPCX_PROF_CAT(mpcx_prof_slot_, __LINE__))
// MPCX_TRACE("kind", n): a timeline interval over the rest of the scope
#define MPCX_TRACE(kind, n) ::mpcx::host::prof::TraceScope MPCX_PROF_CAT(mpcx_trace_, __LINE__)(kind, (int64_t)(n))
// MPCX_PROF_CPU("label"): this thread's CPU time over the rest of the scope
#define MPCX_PROF_CPU(label)                                                   \
  static const int MPCX_PROF_CAT(mpcx_profc_slot_, __LINE__) = ::mpcx::host::prof::slot_of(label); \
  ::mpcx::host::prof::ThreadCpu MPCX_PROF_CAT(mpcx_profc_scope_, __LINE__)(MPCX_PROF_CAT(mpcx_profc_slot_, __LINE__))
