// C API implementation (thin, exception-safe wrappers over the C++ engine).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "msbfs/device.hpp"
#include "msbfs/graph.hpp"
#include "msbfs/msbfs.h"

struct msbfs_graph_s {
  msbfs::DeviceGraph g;
};
struct msbfs_solver_s {
  msbfs_graph graph = nullptr;
  int algo = 0;
  std::unique_ptr<msbfs::Solver> impl;
  int nthreads = 0;
  std::vector<msbfs::LevelRec> recs;  // per-level records of the last run / phase
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  } catch (...) {
    g_err = "unknown error";
    return -1;
  }
}

template <class T>
T* dup(const std::vector<T>& v) {
  T* p = (T*)malloc(std::max<size_t>(1, v.size()) * sizeof(T));
  if (!p) msbfs::fail("out of host memory");
  if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

hipStream_t as_stream(void* s) { return (hipStream_t)s; }
}  // namespace

// run fn on the solver's device stream with event timing and fill st
template <class Fn>
void timed(msbfs_solver s, void* stream, msbfs_stats* st, const char* what, Fn&& fn) {
  MSBFS_HIP_CHECK(hipSetDevice(s->graph->g.device));
  msbfs::trace::Range range(what);
  msbfs::RunStats rs;
  hipStream_t hs = as_stream(stream);
  hipEvent_t e0, e1;
  MSBFS_HIP_CHECK(hipEventCreate(&e0));
  MSBFS_HIP_CHECK(hipEventCreate(&e1));
  MSBFS_HIP_CHECK(hipEventRecord(e0, hs));
  fn(&rs, hs);
  MSBFS_HIP_CHECK(hipEventRecord(e1, hs));
  MSBFS_HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0;
  MSBFS_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  s->recs = std::move(rs.recs);
  if (st) {
    st->levels = rs.levels;
    st->td_levels = rs.td_levels;
    st->bu_levels = rs.bu_levels;
    st->batches = rs.batches;
    st->device_ms = ms;
  }
}

extern "C" {

const char* msbfs_last_error(void) { return g_err.c_str(); }
const char* msbfs_version(void) { return "msbfs 0.1.0 (gfx950)"; }
void msbfs_free(void* p) { free(p); }

int msbfs_device_count(int* n) {
  return guard([&] {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
  });
}
int msbfs_set_device(int dev) { return guard([&] { MSBFS_HIP_CHECK(hipSetDevice(dev)); }); }
int msbfs_device_sync(void) { return guard([&] { MSBFS_HIP_CHECK(hipDeviceSynchronize()); }); }

int msbfs_read_graph_csr(const char* path, int use_cache, int64_t* n, int64_t* m,
                         int64_t** rowptr, int32_t** col) {
  return guard([&] {
    msbfs::HostCsr g = msbfs::load_graph(path, use_cache != 0);
    *n = g.n;
    *m = g.m;
    *rowptr = dup(g.rowptr);
    *col = dup(g.col);
  });
}

int msbfs_read_edge_list(const char* path, int64_t* n, int64_t* m, int32_t** u, int32_t** v) {
  return guard([&] {
    msbfs::EdgeList el = msbfs::read_edge_list_bin(path);
    *n = el.n;
    *m = el.m();
    *u = dup(el.u);
    *v = dup(el.v);
  });
}

int msbfs_write_edge_list(const char* path, int64_t n, int64_t m, const int32_t* u,
                          const int32_t* v) {
  return guard([&] {
    msbfs::EdgeList el;
    el.n = n;
    el.u.assign(u, u + m);
    el.v.assign(v, v + m);
    msbfs::write_edge_list_bin(path, el);
  });
}

int msbfs_read_queries(const char* path, int64_t* K, int64_t** off, int64_t* nids, int32_t** ids) {
  return guard([&] {
    msbfs::QuerySet q = msbfs::read_query_bin(path);
    *K = q.K();
    *off = dup(q.off);
    *nids = (int64_t)q.ids.size();
    *ids = dup(q.ids);
  });
}

int msbfs_write_queries(const char* path, int64_t K, const int64_t* off, const int32_t* ids,
                        int force_extended) {
  return guard([&] {
    msbfs::QuerySet q;
    q.off.assign(off, off + K + 1);
    q.ids.assign(ids, ids + off[K]);
    msbfs::write_query_bin(path, q, force_extended != 0);
  });
}

int msbfs_build_csr(int64_t n, int64_t m, const int32_t* u, const int32_t* v, int stable,
                    int64_t** rowptr, int32_t** col) {
  return guard([&] {
    msbfs::EdgeList el;
    el.n = n;
    el.u.assign(u, u + m);
    el.v.assign(v, v + m);
    for (int64_t i = 0; i < m; ++i)
      if ((uint32_t)el.u[i] >= (uint64_t)n || (uint32_t)el.v[i] >= (uint64_t)n)
        msbfs::fail("edge " + std::to_string(i) + " has a vertex id outside [0, n)");
    msbfs::HostCsr g = msbfs::build_csr(el, 0, stable != 0);
    *rowptr = dup(g.rowptr);
    *col = dup(g.col);
  });
}

int msbfs_gen_rmat_host(int scale, int64_t edgefactor, uint64_t seed, double a, double b, double c,
                        int scramble, int32_t** u, int32_t** v, int64_t* n, int64_t* m) {
  return guard([&] {
    msbfs::EdgeList el = msbfs::gen_rmat(scale, edgefactor, seed, a, b, c, scramble != 0);
    *n = el.n;
    *m = el.m();
    *u = dup(el.u);
    *v = dup(el.v);
  });
}

int msbfs_gen_uniform_host(int64_t n, int64_t m, uint64_t seed, int32_t** u, int32_t** v) {
  return guard([&] {
    msbfs::EdgeList el = msbfs::gen_uniform(n, m, seed);
    *u = dup(el.u);
    *v = dup(el.v);
  });
}

int msbfs_gen_grid_host(int64_t rows, int64_t cols, double keep, int64_t shortcuts, uint64_t seed,
                        int32_t** u, int32_t** v, int64_t* n, int64_t* m) {
  return guard([&] {
    msbfs::EdgeList el = msbfs::gen_grid(rows, cols, keep, shortcuts, seed);
    *n = el.n;
    *m = el.m();
    *u = dup(el.u);
    *v = dup(el.v);
  });
}

int msbfs_gen_queries(int64_t n, int64_t K, int64_t size, uint64_t seed, int64_t** off,
                      int32_t** ids) {
  return guard([&] {
    msbfs::QuerySet q = msbfs::gen_queries(n, K, size, seed);
    *off = dup(q.off);
    *ids = dup(q.ids);
  });
}

int msbfs_cpu_run(int64_t n, const int64_t* rowptr, const int32_t* col, int64_t K,
                  const int64_t* qoff, const int32_t* qids, int64_t* F, int64_t* edges,
                  int nthreads) {
  return guard([&] {
    msbfs::HostCsr g;
    g.n = n;
    g.rowptr.assign(rowptr, rowptr + n + 1);
    g.col.assign(col, col + rowptr[n]);
    g.m = rowptr[n] / 2;
    msbfs::QuerySet q;
    q.off.assign(qoff, qoff + K + 1);
    q.ids.assign(qids, qids + qoff[K]);
    std::vector<int64_t> f, e;
    msbfs::cpu_msbfs_all(g, q, f, edges ? &e : nullptr, nthreads);
    std::memcpy(F, f.data(), K * sizeof(int64_t));
    if (edges) std::memcpy(edges, e.data(), K * sizeof(int64_t));
  });
}

int msbfs_graph_from_host_csr(int device, int64_t n, const int64_t* rowptr, const int32_t* col,
                              msbfs_graph* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(device));
    auto h = std::make_unique<msbfs_graph_s>();
    h->g.device = device;
    msbfs::device_graph_from_host(h->g, n, rowptr, col, nullptr);
    *out = h.release();
  });
}

int msbfs_graph_from_device_edges(int device, int64_t n, int64_t m, const int32_t* d_u,
                                  const int32_t* d_v, msbfs_graph* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(device));
    auto h = std::make_unique<msbfs_graph_s>();
    h->g.device = device;
    msbfs::device_graph_from_edges(h->g, n, m, d_u, d_v, nullptr);
    *out = h.release();
  });
}

int msbfs_graph_wrap_device(int device, int64_t n, int64_t nnz, int64_t* d_rowptr, int32_t* d_col,
                            msbfs_graph* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(device));
    // (the one-lane-per-vertex pulls read column ids as aligned 16-byte words)
    if (reinterpret_cast<uintptr_t>(d_col) & 15)
      msbfs::fail("graph wrap: the column array must be 16-byte aligned");
    auto h = std::make_unique<msbfs_graph_s>();
    h->g.device = device;
    h->g.n = n;
    h->g.nnz = nnz;
    h->g.m = nnz / 2;
    h->g.rowptr = d_rowptr;
    h->g.col = d_col;
    msbfs::device_graph_stats(h->g, nullptr);
    *out = h.release();
  });
}

int msbfs_graph_gen_rmat(int device, int scale, int64_t edgefactor, uint64_t seed, double a,
                         double b, double c, int scramble, msbfs_graph* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(device));
    auto h = std::make_unique<msbfs_graph_s>();
    h->g.device = device;
    msbfs::device_graph_gen_rmat(h->g, scale, edgefactor, seed, a, b, c, scramble, nullptr);
    *out = h.release();
  });
}

int msbfs_graph_gen_uniform(int device, int64_t n, int64_t m, uint64_t seed, msbfs_graph* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(device));
    auto h = std::make_unique<msbfs_graph_s>();
    h->g.device = device;
    msbfs::device_graph_gen_uniform(h->g, n, m, seed, nullptr);
    *out = h.release();
  });
}

int msbfs_graph_from_edge_file(int device, const char* path, msbfs_graph* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(device));
    auto h = std::make_unique<msbfs_graph_s>();
    h->g.device = device;
    msbfs::device_graph_from_edge_file(h->g, path ? path : "", nullptr);
    *out = h.release();
  });
}

int msbfs_graph_sort_rows(msbfs_graph g) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(g->g.device));
    msbfs::device_graph_sort_rows(g->g, nullptr);
  });
}

int msbfs_graph_relabel_by_degree(msbfs_graph g) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(g->g.device));
    msbfs::device_graph_relabel_by_degree(g->g, nullptr);
  });
}

int msbfs_graph_relabel_map(msbfs_graph g, int32_t* old2new) {
  return guard([&] {
    if (!g->g.old2new) msbfs::fail("graph is not relabelled");
    MSBFS_HIP_CHECK(hipSetDevice(g->g.device));
    MSBFS_HIP_CHECK(hipMemcpy(old2new, g->g.old2new, g->g.n * sizeof(int32_t),
                              hipMemcpyDeviceToHost));
  });
}

int msbfs_graph_is_relabelled(msbfs_graph g) { return g->g.old2new ? 1 : 0; }

int msbfs_graph_info(msbfs_graph g, int64_t* n, int64_t* nnz, int64_t* m, int64_t* max_degree,
                     int64_t* isolated) {
  return guard([&] {
    if (n) *n = g->g.n;
    if (nnz) *nnz = g->g.nnz;
    if (m) *m = g->g.m;
    if (max_degree) *max_degree = g->g.max_degree;
    if (isolated) *isolated = g->g.isolated;
  });
}

int msbfs_graph_device_ptrs(msbfs_graph g, void** rowptr, void** col) {
  return guard([&] {
    *rowptr = g->g.rowptr;
    *col = g->g.col;
  });
}

int msbfs_graph_download(msbfs_graph g, int64_t* rowptr, int32_t* col) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(g->g.device));
    MSBFS_HIP_CHECK(hipMemcpy(rowptr, g->g.rowptr, (g->g.n + 1) * sizeof(int64_t),
                              hipMemcpyDeviceToHost));
    if (g->g.nnz)
      MSBFS_HIP_CHECK(hipMemcpy(col, g->g.col, g->g.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
  });
}

void msbfs_graph_free(msbfs_graph g) {
  if (!g) return;
  (void)hipSetDevice(g->g.device);
  delete g;
}

int msbfs_solver_create(msbfs_graph g, int algo, int64_t max_groups, msbfs_solver* out) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(g->g.device));
    auto s = std::make_unique<msbfs_solver_s>();
    s->graph = g;
    if (algo == MSBFS_ALGO_AUTO)
      algo = msbfs::auto_device_algo(g->g, max_groups) == 2 ? MSBFS_ALGO_DIST : MSBFS_ALGO_BITPAR;
    s->algo = algo;
    switch (algo) {
      case MSBFS_ALGO_BITPAR:
        s->impl = msbfs::make_bitpar_solver(g->g, (int)std::min<int64_t>(max_groups, 1024));
        break;
      case MSBFS_ALGO_DIST:
        s->impl = msbfs::make_dist_solver(g->g);
        break;
      case MSBFS_ALGO_TOPDOWN:
        s->impl = msbfs::make_dist_solver(g->g);
        s->impl->opt.force_dir = 1;
        break;
      case MSBFS_ALGO_SWEEP:
        s->impl = msbfs::make_sweep_solver(g->g);
        break;
      default:
        msbfs::fail("unknown/unsupported device algorithm " + std::to_string(algo));
    }
    *out = s.release();
  });
}

int msbfs_solver_set_options(msbfs_solver s, const msbfs_options* o) {
  return guard([&] {
    auto& opt = s->impl->opt;
    if (o->alpha > 0) opt.alpha = o->alpha;
    if (o->beta > 0) opt.beta = o->beta;
    if (o->wide_degree > 0) opt.wide_degree = o->wide_degree;
    opt.force_dir = o->force_dir;
    if (o->max_words > 0) opt.max_words = o->max_words;
  });
}

int msbfs_solver_prepare(msbfs_solver s, void* stream) {
  return guard([&] {
    MSBFS_HIP_CHECK(hipSetDevice(s->graph->g.device));
    s->impl->prepare((hipStream_t)stream);
  });
}

int msbfs_solver_prepare_hybrid(msbfs_solver s, int part, int nparts, void* stream) {
  return guard([&] {
    if (nparts < 1 || part < 0 || part >= nparts) msbfs::fail("prepare_hybrid: bad part index");
    MSBFS_HIP_CHECK(hipSetDevice(s->graph->g.device));
    s->impl->prepare_hybrid(part, nparts, (hipStream_t)stream);
  });
}

int msbfs_solver_tune(msbfs_solver s, const char* spec) {
  return guard([&] {
    if (!spec) msbfs::fail("msbfs_solver_tune: null spec");
    s->impl->tune(spec);
  });
}

int msbfs_solver_run(msbfs_solver s, int64_t K, const int64_t* qoff, const int32_t* qids,
                     int64_t* F, int64_t* edges2, msbfs_stats* st, void* stream) {
  return guard([&] {
    timed(s, stream, st, "solver run", [&](msbfs::RunStats* rs, hipStream_t hs) {
      s->impl->run(K, qoff, qids, F, edges2, rs, hs);
    });
  });
}

int msbfs_hybrid_extent(msbfs_graph g, int64_t* n_eff) {
  return guard([&] { *n_eff = msbfs::hybrid_extent(g->g); });
}

int64_t msbfs_solver_hybrid_max_groups(msbfs_solver s) {
  return s && s->impl ? s->impl->hybrid_max_groups() : 0;
}

int msbfs_solver_hybrid_phase_a(msbfs_solver s, int64_t K, const int64_t* qoff,
                                const int32_t* qids, int part, int nparts, int64_t n_eff,
                                int count_l1, const int32_t* wbeg, void* send_dev, int64_t* out,
                                msbfs_stats* st, void* stream) {
  return guard([&] {
    timed(s, stream, st, "hybrid phase A", [&](msbfs::RunStats* rs, hipStream_t hs) {
      s->impl->hybrid_phase_a(K, qoff, qids, part, nparts, n_eff, count_l1 != 0, wbeg,
                              (uint64_t*)send_dev, out, rs, hs);
    });
  });
}

int msbfs_solver_hybrid_phase_a_coded(msbfs_solver s, int64_t K, const int64_t* qoff,
                                      const int32_t* qids, int part, int nparts, int64_t n_eff,
                                      int count_l1, const int32_t* wbeg, void* send_dev,
                                      int64_t* out, int64_t* coded_len, msbfs_stats* st,
                                      void* stream) {
  return guard([&] {
    if (!coded_len) msbfs::fail("hybrid_phase_a_coded: coded_len is null");
    timed(s, stream, st, "hybrid phase A", [&](msbfs::RunStats* rs, hipStream_t hs) {
      s->impl->hybrid_phase_a(K, qoff, qids, part, nparts, n_eff, count_l1 != 0, wbeg,
                              (uint64_t*)send_dev, out, rs, hs, coded_len);
    });
  });
}

int msbfs_solver_hybrid_chunk_bounds(msbfs_solver s, int part, int nparts, int64_t n_eff,
                                     int chunks, int64_t* bounds) {
  return guard([&] {
    if (!s || !s->impl) msbfs::fail("null solver");
    if (chunks < 1 || chunks > 1024) msbfs::fail("hybrid: chunks must be in [1, 1024]");
    MSBFS_HIP_CHECK(hipSetDevice(s->graph->g.device));
    s->impl->hybrid_chunk_bounds(part, nparts, n_eff, chunks, bounds, nullptr);
    MSBFS_HIP_CHECK(hipDeviceSynchronize());
  });
}

int msbfs_solver_hybrid_phase_a_chunked(msbfs_solver s, int64_t K, const int64_t* qoff,
                                        const int32_t* qids, int part, int nparts,
                                        int64_t n_eff, int count_l1, const int32_t* wbeg,
                                        void* send_dev, int64_t* out, int chunks,
                                        msbfs_chunk_fn cb, void* user, msbfs_stats* st,
                                        void* stream) {
  return guard([&] {
    if (!cb) msbfs::fail("hybrid_phase_a_chunked: no chunk callback");
    timed(s, stream, st, "hybrid phase A", [&](msbfs::RunStats* rs, hipStream_t hs) {
      s->impl->hybrid_phase_a(K, qoff, qids, part, nparts, n_eff, count_l1 != 0, wbeg,
                              (uint64_t*)send_dev, out, rs, hs, nullptr, chunks, cb, user);
    });
  });
}

int msbfs_solver_hybrid_decode(msbfs_solver s, const void* coded_dev, const int64_t* coded_len,
                               int nparts, int64_t n_eff, int w_count, void* dense_dev,
                               void* stream) {
  return guard([&] {
    if (!s || !s->impl) msbfs::fail("null solver");
    MSBFS_HIP_CHECK(hipSetDevice(s->graph->g.device));
    msbfs::trace::Range range("hybrid decode");
    s->impl->hybrid_decode((const uint64_t*)coded_dev, coded_len, nparts, n_eff, w_count,
                           (uint64_t*)dense_dev, (hipStream_t)stream);
  });
}

int msbfs_solver_hybrid_phase_c(msbfs_solver s, int64_t K, int w_begin, int w_count, int nparts,
                                int64_t n_eff, const void* recv_dev, const int64_t* reduced,
                                int64_t* F_local, msbfs_stats* st, void* stream) {
  return guard([&] {
    timed(s, stream, st, "hybrid phase C", [&](msbfs::RunStats* rs, hipStream_t hs) {
      s->impl->hybrid_phase_c(K, w_begin, w_count, nparts, n_eff, (const uint64_t*)recv_dev,
                              reduced, F_local, rs, hs);
    });
  });
}

int64_t msbfs_solver_levels(msbfs_solver s, msbfs_level* out, int64_t cap) {
  if (!s) return -1;
  const int64_t n = (int64_t)s->recs.size();
  for (int64_t i = 0; out && i < std::min(n, cap); ++i) {
    const msbfs::LevelRec& r = s->recs[i];
    out[i] = msbfs_level{r.batch, r.level, r.dir, {0, 0, 0}, r.nf, r.ef, r.nf_next, r.active, r.ms};
  }
  return n;
}

void msbfs_solver_free(msbfs_solver s) {
  if (!s) return;
  (void)hipSetDevice(s->graph->g.device);
  delete s;
}

int64_t msbfs_argmin(const int64_t* F, int64_t K) {
  std::vector<int64_t> f(F, F + K);
  return msbfs::argmin_first(f);
}

}  // extern "C"
