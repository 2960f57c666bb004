// Host graph / query generators. The reference ships no generator and no data;
// BASELINE configs need RMAT (Graph500 A=.57 B=.19 C=.19 D=.05, edge factor 16), uniform random
// and high-diameter road-like graphs, plus random query sets. The RNG is the shared counter-based
// one in common.hpp so the device generator (kernels/gen.hip) produces the identical edge list.
#include <algorithm>
#include <thread>

#include "msbfs/graph.hpp"

namespace msbfs {

template <class F>
static void par(int nthreads, int64_t total, F&& fn) {
  if (nthreads <= 0) nthreads = default_threads();
  if (nthreads <= 1 || total < 65536) {
    fn(0, total);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (total + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t b = t * chunk, e = std::min(total, b + chunk);
    if (b >= e) break;
    th.emplace_back([&fn, b, e] { fn(b, e); });
  }
  for (auto& x : th) x.join();
}

EdgeList gen_rmat(int scale, int64_t edgefactor, uint64_t seed, double a, double b, double c,
                  bool scramble, int nthreads) {
  if (scale < 1 || scale > 31) fail("rmat scale must be in [1, 31] (int32 vertex ids)");
  EdgeList el;
  el.n = int64_t(1) << scale;
  const int64_t m = el.n * edgefactor;
  el.u.resize(m);
  el.v.resize(m);
  const RmatParams p = make_rmat_params(scale, seed, a, b, c, scramble ? 1 : 0);
  par(nthreads, m, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      uint32_t u, v;
      rmat_edge(p, (uint64_t)i, u, v);
      el.u[i] = (int32_t)u;
      el.v[i] = (int32_t)v;
    }
  });
  return el;
}

EdgeList gen_uniform(int64_t n, int64_t m, uint64_t seed, int nthreads) {
  if (n <= 0 || n > INT32_MAX) fail("uniform graph needs 0 < n <= INT32_MAX");
  EdgeList el;
  el.n = n;
  el.u.resize(m);
  el.v.resize(m);
  par(nthreads, m, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      uint32_t u, v;
      uniform_edge(seed, (uint64_t)i, (uint64_t)n, u, v);
      el.u[i] = (int32_t)u;
      el.v[i] = (int32_t)v;
    }
  });
  return el;
}

EdgeList gen_grid(int64_t rows, int64_t cols, double keep, int64_t shortcuts, uint64_t seed) {
  if (rows <= 0 || cols <= 0 || rows * cols > INT32_MAX) fail("bad grid size");
  EdgeList el;
  el.n = rows * cols;
  const uint64_t thr = keep >= 1.0 ? ~0ull : (uint64_t)(keep * 18446744073709551615.0);
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t c = 0; c < cols; ++c) {
      const int64_t id = r * cols + c;
      if (c + 1 < cols && mix64(seed ^ (uint64_t)(2 * id)) <= thr) {
        el.u.push_back((int32_t)id);
        el.v.push_back((int32_t)(id + 1));
      }
      if (r + 1 < rows && mix64(seed ^ (uint64_t)(2 * id + 1)) <= thr) {
        el.u.push_back((int32_t)id);
        el.v.push_back((int32_t)(id + cols));
      }
    }
  for (int64_t s = 0; s < shortcuts; ++s) {
    uint32_t u, v;
    uniform_edge(seed ^ 0x5107C075ull, (uint64_t)s, (uint64_t)el.n, u, v);
    el.u.push_back((int32_t)u);
    el.v.push_back((int32_t)v);
  }
  return el;
}

QuerySet gen_queries(int64_t n, int64_t K, int64_t size, uint64_t seed) {
  QuerySet q;
  q.off.reserve(K + 1);
  q.ids.reserve(K * size);
  for (int64_t k = 0; k < K; ++k) {
    for (int64_t j = 0; j < size; ++j)
      q.ids.push_back((int32_t)query_vertex(seed, (uint64_t)k, (uint64_t)j, (uint64_t)n));
    q.off.push_back((int64_t)q.ids.size());
  }
  return q;
}

}  // namespace msbfs
