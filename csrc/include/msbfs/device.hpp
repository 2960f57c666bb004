// Internal device-side infrastructure shared by the HIP translation units: error checks,
// device buffers, the device CSR, wave64 helpers and the solver interfaces.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "msbfs/common.hpp"
#include "msbfs/trace.hpp"

#define MSBFS_HIP_CHECK(expr)                                                                \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      ::msbfs::fail(std::string("HIP error '") + hipGetErrorString(_e) + "' at " __FILE__ ":" + \
                    std::to_string(__LINE__) + " in " #expr);                                \
  } while (0)

namespace msbfs {

// Owning device allocation (RAII). Graph-sized buffers are allocated once and reused for every
// query group / batch: the reference cudaMalloc/cudaFree's a flag per query (main.cu:57,72).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  explicit DevBuf(size_t b) { alloc(b); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    release();
    p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0;
    return *this;
  }
  ~DevBuf() { release(); }
  void alloc(size_t b) {
    release();
    if (b == 0) b = 16;
    MSBFS_HIP_CHECK(hipMalloc(&p, b));
    bytes = b;
  }
  void ensure(size_t b) { if (b > bytes) alloc(b); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T* as() const { return (T*)p; }
};

// Pinned host staging buffer (for per-level counter read-back without pageable copies; the
// reference does 1-byte synchronous pageable copies every level, main.cu:64,69).
struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  explicit PinnedBuf(size_t b) : bytes(b) { MSBFS_HIP_CHECK(hipHostMalloc(&p, b, hipHostMallocDefault)); }
  ~PinnedBuf() { if (p) (void)hipHostFree(p); }
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  template <class T> T* as() const { return (T*)p; }
};

// Device-resident symmetric CSR (int64 offsets, int32 columns). Either owns its arrays or
// borrows externally-owned ones (e.g. torch tensors handed over from Python).
struct DeviceGraph {
  int device = 0;
  int64_t n = 0, nnz = 0, m = 0;
  int64_t* rowptr = nullptr;
  int32_t* col = nullptr;
  DevBuf own_rowptr, own_col;
  int64_t max_degree = 0;
  int64_t isolated = 0;
  // Optional degree-descending relabelling: old2new[v] maps a user vertex id to the internal id
  // (null when the graph keeps the user's ids). Solvers map query sources through it.
  int32_t* old2new = nullptr;
  DevBuf own_old2new;
  // every row's neighbour ids ascending (device_graph_sort_rows; relabelling sorts too). Solvers
  // may binary-search rows only when this is set.
  bool rows_sorted = false;
  // How a device-generated graph was made (0 = not generated, 1 = RMAT, 2 = uniform): a
  // relabelling that has no room for a second column array regenerates the edges straight into
  // the new ids instead (the generators are deterministic functions of the edge index).
  int gen_kind = 0;
  RmatParams gen_rmat{};
  uint64_t gen_seed = 0;
  int64_t gen_edges = 0;
};

// Stats returned by solvers (mirrors msbfs_stats in msbfs.h). recs: one record per BFS level
// (bit-parallel solver; see trace.hpp), exported by msbfs_solver_levels.
struct RunStats {
  int64_t levels = 0, td_levels = 0, bu_levels = 0, batches = 0;
  double device_ms = 0;
  std::vector<LevelRec> recs;
};

// ---- device-graph construction (kernels/gen.hip) -------------------------------------------
void device_graph_from_host(DeviceGraph& g, int64_t n, const int64_t* rowptr, const int32_t* col,
                            hipStream_t s);
// The legacy graph file (main.cu:92-130) built into a CSR on the device: the mapped edge list is
// streamed to HBM through pinned staging, then degree count (atomics) -> scan -> scatter, ids
// validated on the device. Neighbour order is not the file's (F does not depend on it).
void device_graph_from_edge_file(DeviceGraph& g, const std::string& path, hipStream_t s);
void device_graph_from_edges(DeviceGraph& g, int64_t n, int64_t m, const int32_t* d_u,
                             const int32_t* d_v, hipStream_t s);
void device_graph_gen_rmat(DeviceGraph& g, int scale, int64_t edgefactor, uint64_t seed, double a,
                           double b, double c, int scramble, hipStream_t s);
void device_graph_gen_uniform(DeviceGraph& g, int64_t n, int64_t m, uint64_t seed, hipStream_t s);
void device_graph_stats(DeviceGraph& g, hipStream_t s);
void device_graph_sort_rows(DeviceGraph& g, hipStream_t s);
// Renumber vertices by descending degree (stable), rebuild the CSR with sorted rows and keep the
// old->new map in g.old2new. F(U) is invariant under relabelling.
void device_graph_relabel_by_degree(DeviceGraph& g, hipStream_t s);

// ---- solvers ---------------------------------------------------------------------------------
constexpr int kDefaultWideDegree = 32;
struct SolverOptions {
  double alpha = 14.0;  // top-down -> bottom-up when frontier edges > unexplored edges / alpha
  double beta = 24.0;   // bottom-up -> top-down when frontier vertices < active vertices / beta
  // first bottom-up level: vertices above this degree go to the chunk kernel (at the default,
  // bit-parallel passes of <= 4 words use the tuning key wide_few instead)
  int wide_degree = kDefaultWideDegree;
  int force_dir = 0;    // 0 auto, 1 top-down only, 2 bottom-up after level 0
  int max_words = 16;   // bit-parallel: at most 64*max_words groups per batch
  bool count_edges = false;
};

class Solver {
 public:
  virtual ~Solver() = default;
  // Runs groups [0,K) of a packed query set; F[k] and (optionally) edges2[k] (= sum of degrees
  // of reached vertices, i.e. 2x the Graph500 traversed-edge count) are written to host memory.
  virtual void run(int64_t K, const int64_t* qoff, const int32_t* qids, int64_t* F,
                   int64_t* edges2, RunStats* st, hipStream_t stream) = 0;
  // Groups one solver pass handles at once (bit-parallel: 64*W; per-group solvers run any
  // number in one call). Callers that overlap work between passes split runs at this size.
  virtual int64_t pass_groups() const { return INT64_MAX; }
  // Build graph-derived tables and worst-case scratch now (before a timed region) instead of on
  // the first run.
  virtual void prepare(hipStream_t stream) { (void)stream; }
  // The same for hybrid phase A as part `part` of `nparts` (its own vertices' tables)
  virtual void prepare_hybrid(int part, int nparts, hipStream_t stream) {
    (void)part;
    (void)nparts;
    (void)stream;
  }
  // Algorithm tuning, "key=value,key=value" (bit-parallel solver: see bp::Tuning in
  // kernels/bitpar/solver.hpp). Unknown keys are errors; solvers without tuning reject any.
  virtual void tune(const std::string& spec) {
    if (!spec.empty()) fail("this solver has no tuning keys (got '" + spec + "')");
  }

  // ---- hybrid multi-GPU mode (bit-parallel solver only) ------------------------------------
  // Levels 1-2 run vertex-partitioned (every rank: all K groups, pulls only for its residue
  // class of vertices v = part + i*nparts < n_eff); one all-to-all hands every rank its own
  // words (groups) for all vertices; the remaining levels run query-partitioned. See
  // kernels/bitpar/hybrid.hpp. Largest K one hybrid round supports (0: not supported).
  virtual int64_t hybrid_max_groups() const { return 0; }
  // Largest number of ranks (vertex parts) one hybrid round supports.
  static constexpr int kHybridMaxParts = 64;
  // Phase A. wbeg[0..nparts]: destination word split (rank j gets words [wbeg[j], wbeg[j+1]) of
  // ceil(K/64)). send_dev: cnt*wbeg[nparts] words, destination-major, cnt = own vertices.
  // out_host[2K+3]: F partial, per-group "new at level 2" flags, then frontier size / edges /
  // visited edges.
  // coded_len_host != nullptr: send_dev gets the zero-word coded segments instead (see
  // hybrid_coded_bound / kernels/bitpar.hip "zero-word coding"), coded_len_host[j] = words of
  // destination j's segment; the segments lie back to back in destination order.
  //
  // Overlapped (chunked) exchange, dense mode only: `chunks` > 1 splits the own vertices into
  // index ranges [bounds[c], bounds[c+1]) (hybrid_chunk_bounds: the same split on every call
  // for one part / nparts / n_eff / chunks). Phase A packs each range into its place in
  // send_dev as soon as the level-2 pull finished it and calls cb(user, c, bounds[c],
  // bounds[c+1]) with that pack enqueued on `stream`; the callback starts its piece of the
  // all-to-all ordered after that point (on the collective's own stream) while the next range
  // computes. cb runs exactly `chunks` times, in order; send_dev's layout is unchanged.
  using ChunkFn = void (*)(void* user, int chunk, int64_t i0, int64_t i1);
  virtual void hybrid_phase_a(int64_t K, const int64_t* qoff, const int32_t* qids, int part,
                              int nparts, int64_t n_eff, bool count_l1, const int32_t* wbeg,
                              uint64_t* send_dev, int64_t* out_host, RunStats* st,
                              hipStream_t stream, int64_t* coded_len_host = nullptr,
                              int chunks = 1, ChunkFn cb = nullptr, void* user = nullptr) {
    (void)K, (void)qoff, (void)qids, (void)part, (void)nparts, (void)n_eff, (void)count_l1,
        (void)wbeg, (void)send_dev, (void)out_host, (void)st, (void)stream, (void)coded_len_host,
        (void)chunks, (void)cb, (void)user;
    fail("this solver has no hybrid mode (use the bit-parallel solver)");
  }
  // bounds[0..chunks]: the own-vertex index ranges of a chunked phase A (see above)
  virtual void hybrid_chunk_bounds(int part, int nparts, int64_t n_eff, int chunks,
                                   int64_t* bounds, hipStream_t stream) {
    (void)stream;
    const int64_t cnt = n_eff > part ? (n_eff - part + nparts - 1) / nparts : 0;
    for (int c = 0; c <= chunks; ++c) bounds[c] = cnt * c / chunks;
  }
  // Receiver side of the coded exchange: coded_dev holds one coded segment per source part r
  // (coded_len_host[r] words each, back to back); dense_dev gets the layout hybrid_phase_c reads.
  virtual void hybrid_decode(const uint64_t* coded_dev, const int64_t* coded_len_host, int nparts,
                             int64_t n_eff, int w_count, uint64_t* dense_dev, hipStream_t stream) {
    (void)coded_dev, (void)coded_len_host, (void)nparts, (void)n_eff, (void)w_count,
        (void)dense_dev, (void)stream;
    fail("this solver has no hybrid mode (use the bit-parallel solver)");
  }
  // Phase C. recv_dev: for every source part r in order, w_count words of each of r's vertices;
  // reduced[2K+3]: out_host summed over ranks. F_out[64*w_count] (local groups): levels >= 3.
  virtual void hybrid_phase_c(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                              const uint64_t* recv_dev, const int64_t* reduced, int64_t* F_out,
                              RunStats* st, hipStream_t stream) {
    (void)K, (void)w_begin, (void)w_count, (void)nparts, (void)n_eff, (void)recv_dev,
        (void)reduced, (void)F_out, (void)st, (void)stream;
    fail("this solver has no hybrid mode (use the bit-parallel solver)");
  }
  SolverOptions opt;
};

// Largest coded size (words) of a segment of `dense_words` words: every word nonzero.
inline int64_t hybrid_coded_bound(int64_t dense_words) { return dense_words + (dense_words + 63) / 64; }

// Vertices taking part in the hybrid exchange: 1 + the last vertex with deg > 0 (after degree
// relabelling every isolated vertex is in the suffix [n_eff, n)).
int64_t hybrid_extent(const DeviceGraph& g);

std::unique_ptr<Solver> make_bitpar_solver(const DeviceGraph& g, int max_groups);

// MSBFS_ALGO_AUTO for `groups` groups per solver pass: the per-group distance BFS for up to 2
// groups (RMAT-26: 3.7 / 7.1 ms for 1 / 2 groups vs 10.1 / 12.4 ms bit-parallel, whose
// per-vertex work does not shrink with the group count; 3 groups: 9.5 vs 8.4 ms), bit-parallel
// otherwise and on low-degree graphs (road grid 4896^2, one group: 70 ms bit-parallel vs 114 ms
// distance BFS).
constexpr int64_t kAutoDistMaxGroups = 2;
inline int auto_device_algo(const DeviceGraph& g, int64_t groups) {
  return (groups <= kAutoDistMaxGroups && g.max_degree > 64) ? 2 /* dist */ : 1 /* bitpar */;
}
std::unique_ptr<Solver> make_dist_solver(const DeviceGraph& g);
std::unique_ptr<Solver> make_sweep_solver(const DeviceGraph& g);

// ---- common level-loop helpers (kernels/lbs.hip) ---------------------------------------------
// Inclusive prefix sum of ceil(degree / chunk) over `list[0..cnt)` into offs[0..cnt) (int64);
// chunk = 1 gives the frontier's edge prefix used by the load-balanced top-down expansions.
size_t frontier_scan_temp_bytes(int64_t max_items);
// plain inclusive prefix sum of int64 values (hipcub); temp >= inclusive_scan_temp_bytes(cnt)
size_t inclusive_scan_temp_bytes(int64_t max_items);
void inclusive_scan_i64(const int64_t* in, int64_t* out, int64_t cnt, void* temp,
                        size_t temp_bytes, hipStream_t s);
void frontier_degree_scan(const int64_t* rowptr, const int32_t* list, int64_t cnt, int64_t* offs,
                          void* temp, size_t temp_bytes, hipStream_t s, int64_t chunk = 1);

inline int grid_for(int64_t items, int per_block, int cap = 2048) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace msbfs

#if defined(__HIPCC__)
// ---- wave64 device helpers ---------------------------------------------------------------
namespace msbfs {
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l ? (~0ull >> (64 - l)) : 0ull;
}
// Wave-aggregated append: every lane with pred gets a unique slot of *counter. Must be called
// by all lanes that are active in the enclosing control flow.
__device__ __forceinline__ uint32_t wave_append(bool pred, uint32_t* counter) {
  const uint64_t mask = __ballot(pred);
  if (!mask) return 0;
  const int leader = __ffsll((unsigned long long)mask) - 1;
  uint32_t base = 0;
  if (lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
  base = __shfl(base, leader);
  return base + (uint32_t)__popcll(mask & lanemask_lt());
}
__device__ __forceinline__ int64_t upper_bound_i64(const int64_t* a, int64_t cnt, int64_t x) {
  int64_t lo = 0, hi = cnt;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
}  // namespace msbfs
#endif
