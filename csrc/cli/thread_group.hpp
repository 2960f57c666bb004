// In-process collectives for N ranks that are N threads of one process (ThreadComm, the
// single-process multi-GPU mode `--spmd N`; also the in-process fake of the test
// plan). Host-only C++ so the sanitizer self-test (tests/host_selftest.cpp,
// ThreadSanitizer) can drive it directly.
//
// Every collective is: publish this rank's pointer / value in its slot, barrier, read the other
// slots, barrier (so no rank overwrites or frees a published buffer while a peer reads it).
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace msbfs {

struct ThreadGroup {
  explicit ThreadGroup(int n) : size(n), ptrs(n), cptrs(n), vals(n), dvals(n), counts(n) {}
  const int size;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  // per-rank slots published between two barriers
  std::vector<void*> ptrs;
  std::vector<const void*> cptrs;
  std::vector<uint64_t> vals;
  std::vector<double> dvals;
  std::vector<const std::vector<int64_t>*> counts;
  // generation-counted barrier (reusable back to back)
  void sync() {
    std::unique_lock<std::mutex> l(m);
    const uint64_t g = gen;
    if (++arrived == size) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(l, [&] { return gen != g; });
    }
  }
};

inline void tg_bcast(ThreadGroup& g, int rank, void* p, size_t bytes, int root) {
  if (rank == root) g.cptrs[root] = p;
  g.sync();
  if (rank != root && bytes) std::memcpy(p, g.cptrs[root], bytes);
  g.sync();  // the root's buffer stays valid until every copy is done
}

inline uint64_t tg_allreduce_min(ThreadGroup& g, int rank, uint64_t x) {
  g.vals[rank] = x;
  g.sync();
  uint64_t r = x;
  for (uint64_t v : g.vals) r = std::min(r, v);
  g.sync();
  return r;
}

inline double tg_allreduce_max(ThreadGroup& g, int rank, double x) {
  g.dvals[rank] = x;
  g.sync();
  double r = x;
  for (double v : g.dvals) r = std::max(r, v);
  g.sync();
  return r;
}

inline void tg_allreduce_sum(ThreadGroup& g, int rank, int64_t* p, size_t n) {
  g.cptrs[rank] = p;
  g.sync();
  std::vector<int64_t> t(n, 0);
  for (int r = 0; r < g.size; ++r) {
    const int64_t* q = (const int64_t*)g.cptrs[r];
    for (size_t i = 0; i < n; ++i) t[i] += q[i];
  }
  g.sync();  // everyone has read every input before anyone overwrites its own
  if (n) std::memcpy(p, t.data(), n * 8);
}

inline void tg_allgather(ThreadGroup& g, int rank, uint64_t x, std::vector<uint64_t>& out) {
  g.vals[rank] = x;
  g.sync();
  out = g.vals;
  g.sync();
}

// offset of rank r's block for rank `me` inside r's (destination-major) send buffer
inline int64_t tg_send_offset(const ThreadGroup& g, int r, int me) {
  int64_t o = 0;
  for (int k = 0; k < me; ++k) o += (*g.counts[r])[k];
  return o;
}

inline void tg_alltoallv(ThreadGroup& g, int rank, const uint64_t* send,
                         const std::vector<int64_t>& scount, uint64_t* recv,
                         const std::vector<int64_t>& rcount) {
  g.cptrs[rank] = send;
  g.counts[rank] = &scount;
  g.sync();
  int64_t ro = 0;
  bool ok = true;
  for (int r = 0; r < g.size; ++r) {
    if (rcount[r] != (*g.counts[r])[rank]) {
      ok = false;
      break;
    }
    if (rcount[r])
      std::memcpy(recv + ro, (const uint64_t*)g.cptrs[r] + tg_send_offset(g, r, rank),
                  rcount[r] * 8);
    ro += rcount[r];
  }
  g.sync();
  if (!ok) throw std::runtime_error("threads all-to-all: count mismatch");
}

}  // namespace msbfs
