// CPU multi-source BFS: BASELINE config 1 ("serial CPU BFS on 1 rank") and the test oracle.
// Semantics follow GPUMultiSourceBFS + ComputeFofU (main.cu:40-89): all valid sources of a group
// start at distance 0, out-of-range sources are ignored, F sums the finite distances only.
#include <algorithm>
#include <atomic>
#include <thread>

#include "msbfs/graph.hpp"

namespace msbfs {

int64_t cpu_msbfs_F(const HostCsr& g, const int32_t* src, int64_t nsrc, std::vector<int32_t>& dist,
                    std::vector<int64_t>& queue, int64_t* edges, int32_t* levels) {
  const int64_t n = g.n;
  dist.assign(n, -1);
  queue.resize(std::max<int64_t>(n, 1));
  int64_t head = 0, tail = 0;
  for (int64_t i = 0; i < nsrc; ++i) {
    const int64_t s = src[i];
    if (s >= 0 && s < n && dist[s] < 0) {
      dist[s] = 0;
      queue[tail++] = s;
    }
  }
  int64_t F = 0, deg_sum = 0;
  int32_t maxd = 0;
  while (head < tail) {
    const int64_t u = queue[head++];
    const int32_t du = dist[u];
    F += du;
    maxd = std::max(maxd, du);
    const int64_t b = g.rowptr[u], e = g.rowptr[u + 1];
    deg_sum += e - b;
    for (int64_t j = b; j < e; ++j) {
      const int32_t v = g.col[j];
      if (dist[v] < 0) {
        dist[v] = du + 1;
        queue[tail++] = v;
      }
    }
  }
  if (edges) *edges = deg_sum / 2;
  if (levels) *levels = tail ? maxd + 1 : 0;
  return F;
}

void cpu_msbfs_all(const HostCsr& g, const QuerySet& q, std::vector<int64_t>& F,
                   std::vector<int64_t>* edges, int nthreads) {
  const int64_t K = q.K();
  F.assign(K, 0);
  if (edges) edges->assign(K, 0);
  if (nthreads <= 0) nthreads = default_threads();
  nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, K));
  std::atomic<int64_t> next{0};
  auto worker = [&] {
    std::vector<int32_t> dist;
    std::vector<int64_t> queue;
    for (;;) {
      const int64_t k = next.fetch_add(1);
      if (k >= K) break;
      int64_t e = 0;
      F[k] = cpu_msbfs_F(g, q.ids.data() + q.off[k], q.off[k + 1] - q.off[k], dist, queue, &e);
      if (edges) (*edges)[k] = e;
    }
  };
  if (nthreads == 1) {
    worker();
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back(worker);
  for (auto& t : th) t.join();
}

}  // namespace msbfs
