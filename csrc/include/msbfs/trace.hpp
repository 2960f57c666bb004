// Observability: roctx ranges and per-level solver records.
//
// The reference's only instrumentation is two std::chrono phase timers (main.cu:235,297-301,
// 399-400; SURVEY §5 "Tracing / profiling"). Here:
//   * named roctx ranges around every phase (CLI: load / distribute / upload / compute / reduce;
//     solvers: batch, level "L3 BU", hybrid phases) — rocprofv3 --marker-trace shows them on the
//     timeline next to the kernels. Compiled in when the rocprofiler-sdk roctx library is present
//     (MSBFS_HAVE_ROCTX), otherwise the calls are empty inlines. MSBFS_ROCTX=0 disables them at
//     run time.
//   * LevelRec: one record per BFS level (direction, frontier / active sizes, host wall time of
//     the level including its counter read-back), kept in RunStats and exported through the C API
//     (msbfs_solver_levels) and the CLI's --json line.
#pragma once

#include <cstdint>

namespace msbfs {

struct LevelRec {
  int32_t batch = 0;       // batch index (groups beyond one pass run as further batches)
  int32_t level = 0;       // BFS level (1 = first expansion from the sources)
  char dir = 'T';          // 'T' top-down (push) or 'B' bottom-up (pull)
  int64_t nf = 0;          // union frontier entering the level (vertices)
  int64_t ef = 0;          // its degree sum
  int64_t nf_next = 0;     // vertices newly visited by some group at this level
  int64_t active = 0;      // bottom-up: unfinished vertices scanned; top-down: touched vertices
  double ms = 0;           // host wall time of the level (launches + counter read-back)
};

namespace trace {

bool enabled();
void push(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void pop();
void mark(const char* msg);

// RAII range: `trace::Range r("compute");` or `trace::Range r("level %u", l);`
struct Range {
  explicit Range(const char* name) { push("%s", name); }
  template <class A0, class... A>
  Range(const char* fmt, A0 a0, A... a) {
    if (enabled()) push(fmt, a0, a...);
  }
  ~Range() { pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

}  // namespace trace
}  // namespace msbfs
