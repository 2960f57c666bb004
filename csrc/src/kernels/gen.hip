// Device graph construction: RMAT / uniform generation and count -> scan -> scatter CSR build.
//
// The reference builds the CSR serially on rank 0 from a vector<vector<int>> (main.cu:106-129)
// and broadcasts it through host MPI (main.cu:241-255). Here every GPU can build its own replica
// straight in HBM: the counter-based generator (common.hpp) is evaluated twice — once to count
// degrees, once to scatter — so no edge list is ever materialised (RMAT-30's 137 GB edge list
// would not fit next to its CSR). int64 offsets lift the reference's 2m <= INT_MAX limit.
#include <hipcub/hipcub.hpp>

#include "msbfs/device.hpp"
#include "msbfs/graph.hpp"

namespace msbfs {
namespace {

constexpr int kBlock = 256;

// map != nullptr: endpoints are renumbered through it (relabelled regeneration)
__global__ __launch_bounds__(kBlock) void k_rmat_pass(RmatParams p, int64_t m,
                                                      unsigned long long* cnt, int32_t* col,
                                                      int scatter, const int32_t* map = nullptr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    uint32_t u, v;
    rmat_edge(p, (uint64_t)i, u, v);
    if (map) {
      u = (uint32_t)map[u];
      v = (uint32_t)map[v];
    }
    if (!scatter) {
      atomicAdd(&cnt[u], 1ull);
      atomicAdd(&cnt[v], 1ull);
    } else {
      col[atomicAdd(&cnt[u], 1ull)] = (int32_t)v;
      col[atomicAdd(&cnt[v], 1ull)] = (int32_t)u;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_uniform_pass(uint64_t seed, int64_t n, int64_t m,
                                                         unsigned long long* cnt, int32_t* col,
                                                         int scatter, const int32_t* map = nullptr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    uint32_t u, v;
    uniform_edge(seed, (uint64_t)i, (uint64_t)n, u, v);
    if (map) {
      u = (uint32_t)map[u];
      v = (uint32_t)map[v];
    }
    if (!scatter) {
      atomicAdd(&cnt[u], 1ull);
      atomicAdd(&cnt[v], 1ull);
    } else {
      col[atomicAdd(&cnt[u], 1ull)] = (int32_t)v;
      col[atomicAdd(&cnt[v], 1ull)] = (int32_t)u;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_edges_pass(const int32_t* eu, const int32_t* ev,
                                                       int64_t m, unsigned long long* cnt,
                                                       int32_t* col, int scatter) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const int32_t u = eu[i], v = ev[i];
    if (!scatter) {
      atomicAdd(&cnt[u], 1ull);
      atomicAdd(&cnt[v], 1ull);
    } else {
      col[atomicAdd(&cnt[u], 1ull)] = v;
      col[atomicAdd(&cnt[v], 1ull)] = u;
    }
  }
}

// Edges of the legacy file format ({int32 u, int32 v} pairs, main.cu:108-112) from a device
// copy: count (scatter = 0) or scatter both directions (main.cu:113-115). An id outside [0, n)
// (UB in the reference) records the lowest offending edge index in *bad and is skipped.
__global__ __launch_bounds__(kBlock) void k_pairs_pass(const int2* e, int64_t m, int64_t e0,
                                                       int64_t n, unsigned long long* cnt,
                                                       int32_t* col, int scatter,
                                                       unsigned long long* bad) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const int2 uv = e[i];
    if ((uint32_t)uv.x >= (uint64_t)n || (uint32_t)uv.y >= (uint64_t)n) {
      atomicMin(bad, (unsigned long long)(e0 + i));
      continue;
    }
    if (!scatter) {
      atomicAdd(&cnt[uv.x], 1ull);
      atomicAdd(&cnt[uv.y], 1ull);
    } else {
      col[atomicAdd(&cnt[uv.x], 1ull)] = uv.y;
      col[atomicAdd(&cnt[uv.y], 1ull)] = uv.x;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_copy_i64(const int64_t* src, int64_t* dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = src[i];
}

__global__ __launch_bounds__(kBlock) void k_degree_stats(const int64_t* rowptr, int64_t n,
                                                         unsigned long long* out /*max, iso*/) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long mx = 0, iso = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const unsigned long long d = (unsigned long long)(rowptr[i + 1] - rowptr[i]);
    mx = d > mx ? d : mx;
    iso += d == 0;
  }
  // wave64 reduction then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long om = __shfl_xor(mx, off);
    mx = om > mx ? om : mx;
    iso += __shfl_xor(iso, off);
  }
  if (lane_id() == 0) {
    atomicMax(&out[0], mx);
    atomicAdd(&out[1], iso);
  }
}

// Per-row sort of neighbour lists: rows up to 1024 entries are bitonic-sorted in LDS by one
// block; longer rows by a per-row radix sort pass in chunks (rare: only hubs).
template <int CAP>
__global__ __launch_bounds__(256) void k_sort_rows_lds(const int64_t* rowptr, int32_t* col,
                                                      const int32_t* rows, int64_t nrows) {
  extern __shared__ __attribute__((aligned(16))) int32_t s[];
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int32_t v = rows[r];
    const int64_t b = rowptr[v];
    const int len = (int)(rowptr[v + 1] - b);
    for (int i = threadIdx.x; i < CAP; i += blockDim.x) s[i] = i < len ? col[b + i] : INT32_MAX;
    __syncthreads();
    for (int k = 2; k <= CAP; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < CAP; i += blockDim.x) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const int32_t a = s[i], c = s[ixj];
            const bool up = (i & k) == 0;
            if ((a > c) == up) { s[i] = c; s[ixj] = a; }
          }
        }
        __syncthreads();
      }
    for (int i = threadIdx.x; i < len; i += blockDim.x) col[b + i] = s[i];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_bucket_rows(const int64_t* rowptr, int64_t n,
                                                        int32_t* small, uint32_t* nsmall,
                                                        int32_t* mid, uint32_t* nmid,
                                                        int32_t* big, uint32_t* nbig,
                                                        int32_t* huge, uint32_t* nhuge) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t lim = (n + stride - 1) / stride * stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += stride) {
    const int64_t d = i < n ? rowptr[i + 1] - rowptr[i] : 0;
    const bool a = d > 1 && d <= 64, bm = d > 64 && d <= 1024, c = d > 1024 && d <= 16384;
    const uint32_t pa = wave_append(a, nsmall);
    const uint32_t pb = wave_append(bm, nmid);
    const uint32_t pc = wave_append(c, nbig);
    const bool h = d > 16384;
    const uint32_t ph = wave_append(h, nhuge);
    if (a) small[pa] = (int32_t)i;
    if (bm) mid[pb] = (int32_t)i;
    if (c) big[pc] = (int32_t)i;
    if (h) huge[ph] = (int32_t)i;
  }
}

// one lane per row, insertion sort (rows <= 64)
__global__ __launch_bounds__(kBlock) void k_sort_rows_small(const int64_t* rowptr, int32_t* col,
                                                           const int32_t* rows, int64_t nrows) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += stride) {
    const int32_t v = rows[r];
    int32_t* a = col + rowptr[v];
    const int len = (int)(rowptr[v + 1] - rowptr[v]);
    for (int i = 1; i < len; ++i) {
      const int32_t x = a[i];
      int j = i - 1;
      while (j >= 0 && a[j] > x) { a[j + 1] = a[j]; --j; }
      a[j + 1] = x;
    }
  }
}

void build_from_counts(DeviceGraph& g, DevBuf& cnt, hipStream_t s) {
  // cnt[0..n) holds degrees (int64). rowptr[0]=0, rowptr[1..n] = inclusive scan.
  const int64_t n = g.n;
  MSBFS_HIP_CHECK(hipMemsetAsync(g.rowptr, 0, sizeof(int64_t), s));
  size_t tb = 0;
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, cnt.as<int64_t>(), g.rowptr + 1,
                                                   (int)n, s));
  DevBuf tmp(tb);
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, cnt.as<int64_t>(), g.rowptr + 1,
                                                   (int)n, s));
  int64_t nnz = 0;
  MSBFS_HIP_CHECK(hipMemcpyAsync(&nnz, g.rowptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  g.nnz = nnz;
  // cursor := rowptr[0..n)
  k_copy_i64<<<grid_for(n, kBlock), kBlock, 0, s>>>(g.rowptr, cnt.as<int64_t>(), n);
  MSBFS_HIP_CHECK(hipGetLastError());
  g.own_col.alloc((size_t)std::max<int64_t>(nnz, 1) * sizeof(int32_t));
  g.col = g.own_col.as<int32_t>();
  g.rows_sorted = false;
}

void alloc_rowptr(DeviceGraph& g, int64_t n) {
  if (n < 0 || n > INT32_MAX) fail("vertex count must fit int32 ids");
  g.n = n;
  g.own_rowptr.alloc((size_t)(n + 1) * sizeof(int64_t));
  g.rowptr = g.own_rowptr.as<int64_t>();
}

}  // namespace

void device_graph_stats(DeviceGraph& g, hipStream_t s) {
  DevBuf out(2 * sizeof(unsigned long long));
  MSBFS_HIP_CHECK(hipMemsetAsync(out.p, 0, out.bytes, s));
  if (g.n > 0) {
    k_degree_stats<<<grid_for(g.n, kBlock), kBlock, 0, s>>>(g.rowptr, g.n,
                                                          out.as<unsigned long long>());
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  unsigned long long h[2];
  MSBFS_HIP_CHECK(hipMemcpyAsync(h, out.p, sizeof(h), hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  g.max_degree = (int64_t)h[0];
  g.isolated = (int64_t)h[1];
}

void device_graph_from_host(DeviceGraph& g, int64_t n, const int64_t* rowptr, const int32_t* col,
                            hipStream_t s) {
  alloc_rowptr(g, n);
  g.nnz = rowptr[n];
  g.m = g.nnz / 2;
  g.own_col.alloc((size_t)std::max<int64_t>(g.nnz, 1) * sizeof(int32_t));
  g.col = g.own_col.as<int32_t>();
  g.rows_sorted = false;
  MSBFS_HIP_CHECK(hipMemcpyAsync(g.rowptr, rowptr, (n + 1) * sizeof(int64_t),
                                 hipMemcpyHostToDevice, s));
  if (g.nnz)
    MSBFS_HIP_CHECK(hipMemcpyAsync(g.col, col, g.nnz * sizeof(int32_t), hipMemcpyHostToDevice, s));
  device_graph_stats(g, s);
}

void device_graph_from_edges(DeviceGraph& g, int64_t n, int64_t m, const int32_t* d_u,
                             const int32_t* d_v, hipStream_t s) {
  alloc_rowptr(g, n);
  g.m = m;
  DevBuf cnt((size_t)std::max<int64_t>(n, 1) * sizeof(int64_t));
  MSBFS_HIP_CHECK(hipMemsetAsync(cnt.p, 0, cnt.bytes, s));
  if (m) {
    k_edges_pass<<<grid_for(m, kBlock), kBlock, 0, s>>>(d_u, d_v, m, cnt.as<unsigned long long>(),
                                                       nullptr, 0);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  build_from_counts(g, cnt, s);
  if (m) {
    k_edges_pass<<<grid_for(m, kBlock), kBlock, 0, s>>>(d_u, d_v, m, cnt.as<unsigned long long>(),
                                                       g.col, 1);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  device_graph_stats(g, s);
}

// Host -> device upload of the mapped edge list through two pinned staging buffers: the
// threads copy piece i + 1 out of the page cache while the DMA engine moves piece i.
// fn(dev_ptr, first_edge, edges) runs on stream s after each piece landed in `dst` (dst =
// nullptr: one reused device piece buffer per staging buffer, fn consumes it in place).
template <class F>
static void stream_edges(const EdgeFileMap& f, int2* dst, hipStream_t s, F&& fn) {
  constexpr int64_t kPiece = int64_t(1) << 25;  // edges per piece (256 MB)
  const int64_t piece = std::min<int64_t>(kPiece, std::max<int64_t>(f.m, 1));
  PinnedBuf pin0((size_t)piece * 8), pin1((size_t)piece * 8);
  PinnedBuf* pin[2] = {&pin0, &pin1};
  DevBuf dpiece[2];
  if (!dst)
    for (auto& d : dpiece) d.alloc((size_t)piece * 8);
  hipEvent_t ev[2];
  for (auto& e : ev) MSBFS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  bool used[2] = {false, false};
  int k = 0;
  for (int64_t e0 = 0; e0 < f.m; e0 += piece, k ^= 1) {
    const int64_t len = std::min(piece, f.m - e0);
    if (used[k]) MSBFS_HIP_CHECK(hipEventSynchronize(ev[k]));  // staging k free again
    parallel_memcpy(pin[k]->p, f.edges + 8 * e0, (size_t)len * 8);
    int2* d = dst ? dst + e0 : dpiece[k].as<int2>();
    MSBFS_HIP_CHECK(hipMemcpyAsync(d, pin[k]->p, (size_t)len * 8, hipMemcpyHostToDevice, s));
    fn(d, e0, len);
    MSBFS_HIP_CHECK(hipEventRecord(ev[k], s));
    used[k] = true;
  }
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  for (auto& e : ev) (void)hipEventDestroy(e);
}

void device_graph_from_edge_file(DeviceGraph& g, const std::string& path, hipStream_t s) {
  const EdgeFileMap f = map_edge_file(path);
  alloc_rowptr(g, f.n);
  g.m = f.m;
  const int64_t n = f.n, m = f.m;
  DevBuf cnt((size_t)std::max<int64_t>(n, 1) * sizeof(int64_t));
  MSBFS_HIP_CHECK(hipMemsetAsync(cnt.p, 0, cnt.bytes, s));
  DevBuf bad(sizeof(unsigned long long));
  MSBFS_HIP_CHECK(hipMemsetAsync(bad.p, 0xFF, bad.bytes, s));
  // the whole edge list in HBM when it fits next to the CSR (one pass over the file: count and
  // scatter read the device copy); otherwise the file is streamed twice
  size_t fr = 0, tot = 0;
  MSBFS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
  const size_t ebytes = (size_t)m * 8, cbytes = (size_t)m * 8 + (size_t)n * 24;
  const bool resident = ebytes + cbytes + (size_t(4) << 30) < fr;
  DevBuf all;
  if (resident && m) all.alloc(ebytes);
  auto pass = [&](int scatter) {
    auto run = [&](const int2* d, int64_t e0, int64_t len) {
      k_pairs_pass<<<grid_for(len, kBlock, 8192), kBlock, 0, s>>>(
          d, len, e0, n, cnt.as<unsigned long long>(), scatter ? g.col : nullptr, scatter,
          bad.as<unsigned long long>());
      MSBFS_HIP_CHECK(hipGetLastError());
    };
    if (resident && scatter) {
      if (m) run(all.as<int2>(), 0, m);
    } else if (m) {
      // (count pass of the resident mode: upload into `all`, count each piece as it lands)
      stream_edges(f, resident ? all.as<int2>() : nullptr, s, run);
    }
    unsigned long long b = ~0ull;
    MSBFS_HIP_CHECK(hipMemcpyAsync(&b, bad.p, sizeof(b), hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    if (b != ~0ull)
      fail("graph file " + path + ": edge " + std::to_string(b) +
           " has a vertex id outside [0, n)");
  };
  pass(0);
  build_from_counts(g, cnt, s);
  pass(1);
  g.rows_sorted = false;
  device_graph_stats(g, s);
}

void device_graph_gen_rmat(DeviceGraph& g, int scale, int64_t edgefactor, uint64_t seed, double a,
                           double b, double c, int scramble, hipStream_t s) {
  if (scale < 1 || scale > 31) fail("rmat scale must be in [1, 31]");
  const int64_t n = int64_t(1) << scale, m = n * edgefactor;
  alloc_rowptr(g, n);
  g.m = m;
  const RmatParams p = make_rmat_params(scale, seed, a, b, c, scramble);
  DevBuf cnt((size_t)n * sizeof(int64_t));
  MSBFS_HIP_CHECK(hipMemsetAsync(cnt.p, 0, cnt.bytes, s));
  const int grid = grid_for(m, kBlock, 8192);
  k_rmat_pass<<<grid, kBlock, 0, s>>>(p, m, cnt.as<unsigned long long>(), nullptr, 0);
  MSBFS_HIP_CHECK(hipGetLastError());
  build_from_counts(g, cnt, s);
  k_rmat_pass<<<grid, kBlock, 0, s>>>(p, m, cnt.as<unsigned long long>(), g.col, 1);
  MSBFS_HIP_CHECK(hipGetLastError());
  g.gen_kind = 1;
  g.gen_rmat = p;
  g.gen_edges = m;
  device_graph_stats(g, s);
}

void device_graph_gen_uniform(DeviceGraph& g, int64_t n, int64_t m, uint64_t seed, hipStream_t s) {
  alloc_rowptr(g, n);
  g.m = m;
  DevBuf cnt((size_t)std::max<int64_t>(n, 1) * sizeof(int64_t));
  MSBFS_HIP_CHECK(hipMemsetAsync(cnt.p, 0, cnt.bytes, s));
  const int grid = grid_for(m, kBlock, 8192);
  if (m) {
    k_uniform_pass<<<grid, kBlock, 0, s>>>(seed, n, m, cnt.as<unsigned long long>(), nullptr, 0);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  build_from_counts(g, cnt, s);
  if (m) {
    k_uniform_pass<<<grid, kBlock, 0, s>>>(seed, n, m, cnt.as<unsigned long long>(), g.col, 1);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  g.gen_kind = 2;
  g.gen_seed = seed;
  g.gen_edges = m;
  device_graph_stats(g, s);
}

namespace {
__global__ __launch_bounds__(kBlock) void k_deg_iota(const int64_t* rowptr, int64_t n,
                                                     uint32_t* deg, int32_t* ids) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    deg[i] = (uint32_t)(rowptr[i + 1] - rowptr[i]);
    ids[i] = (int32_t)i;
  }
}
__global__ __launch_bounds__(kBlock) void k_invert_perm(const int32_t* perm, int64_t n,
                                                        int32_t* old2new, const uint32_t* sdeg,
                                                        int64_t* newdeg) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    old2new[perm[i]] = (int32_t)i;
    newdeg[i] = (int64_t)sdeg[i];
  }
}
// one wave per new row: copy the old row of perm[i], mapping every neighbour through old2new
__global__ __launch_bounds__(kBlock) void k_gather_rows(const int64_t* orow, const int32_t* ocol,
                                                        const int32_t* perm, const int64_t* nrow,
                                                        const int32_t* old2new, int32_t* ncol,
                                                        int64_t n) {
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int lane = lane_id();
  for (int64_t i = wave; i < n; i += nwaves) {
    const int32_t o = perm[i];
    const int64_t b = orow[o], len = orow[o + 1] - b, nb = nrow[i];
    for (int64_t j = lane; j < len; j += 64) ncol[nb + j] = old2new[ocol[b + j]];
  }
}
}  // namespace

void device_graph_relabel_by_degree(DeviceGraph& g, hipStream_t s) {
  const int64_t n = g.n;
  if (n == 0 || g.old2new) return;
  // The rebuild holds a second column array next to the first. A device-generated graph without
  // room for it (RMAT-30: 128 GiB of columns) is regenerated in the new ids instead: same rows,
  // and after the row sort the same CSR. MSBFS_RELABEL_REGEN=1 forces that path (tests).
  bool regen = false;
  {
    size_t free_b = 0, total_b = 0;
    const bool tight = hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                       (double)free_b < 1.05 * ((double)g.nnz * 4.0 + (double)n * 40.0);
    const char* force = getenv("MSBFS_RELABEL_REGEN");
    regen = g.gen_kind != 0 && (tight || (force && atoi(force) != 0));
    if (tight && !regen)
      fail("not enough device memory to relabel the graph (needs a second " +
           std::to_string(g.nnz * 4 >> 20) + " MiB column array)");
  }
  DevBuf deg(n * 4), sdeg(n * 4), ids(n * 4), perm(n * 4), newdeg(n * 8);
  k_deg_iota<<<grid_for(n, kBlock), kBlock, 0, s>>>(g.rowptr, n, deg.as<uint32_t>(),
                                                    ids.as<int32_t>());
  MSBFS_HIP_CHECK(hipGetLastError());
  size_t tb = 0;
  MSBFS_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(
      nullptr, tb, deg.as<uint32_t>(), sdeg.as<uint32_t>(), ids.as<int32_t>(), perm.as<int32_t>(),
      (int)n, 0, 32, s));
  {
    DevBuf temp(tb);
    MSBFS_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(
        temp.p, tb, deg.as<uint32_t>(), sdeg.as<uint32_t>(), ids.as<int32_t>(),
        perm.as<int32_t>(), (int)n, 0, 32, s));
  }
  deg.release();
  ids.release();
  g.own_old2new.alloc(n * 4);
  int32_t* o2n = g.own_old2new.as<int32_t>();
  k_invert_perm<<<grid_for(n, kBlock), kBlock, 0, s>>>(perm.as<int32_t>(), n, o2n,
                                                       sdeg.as<uint32_t>(), newdeg.as<int64_t>());
  MSBFS_HIP_CHECK(hipGetLastError());
  sdeg.release();
  // new rowptr = scan of the sorted degrees
  DevBuf nrow((n + 1) * 8);
  MSBFS_HIP_CHECK(hipMemsetAsync(nrow.p, 0, 8, s));
  size_t sb = 0;
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, sb, newdeg.as<int64_t>(),
                                                   nrow.as<int64_t>() + 1, (int)n, s));
  {
    DevBuf temp(sb);
    MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(temp.p, sb, newdeg.as<int64_t>(),
                                                     nrow.as<int64_t>() + 1, (int)n, s));
  }
  newdeg.release();
  DevBuf ncol;
  if (regen) {
    // scatter the regenerated edges into the new rows (cursor = new row starts)
    perm.release();
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    g.own_col.release();
    g.col = nullptr;
    ncol.alloc((size_t)std::max<int64_t>(g.nnz, 1) * 4);
    DevBuf cur((size_t)n * sizeof(int64_t));
    k_copy_i64<<<grid_for(n, kBlock), kBlock, 0, s>>>(nrow.as<int64_t>(), cur.as<int64_t>(), n);
    MSBFS_HIP_CHECK(hipGetLastError());
    const int64_t m = g.gen_edges;
    const int grid = grid_for(m, kBlock, 8192);
    if (m && g.gen_kind == 1)
      k_rmat_pass<<<grid, kBlock, 0, s>>>(g.gen_rmat, m, cur.as<unsigned long long>(),
                                          ncol.as<int32_t>(), 1, o2n);
    else if (m)
      k_uniform_pass<<<grid, kBlock, 0, s>>>(g.gen_seed, n, m, cur.as<unsigned long long>(),
                                             ncol.as<int32_t>(), 1, o2n);
    MSBFS_HIP_CHECK(hipGetLastError());
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  } else {
    ncol.alloc((size_t)std::max<int64_t>(g.nnz, 1) * 4);
    k_gather_rows<<<grid_for(n * 64, kBlock, 8192), kBlock, 0, s>>>(
        g.rowptr, g.col, perm.as<int32_t>(), nrow.as<int64_t>(), o2n, ncol.as<int32_t>(), n);
    MSBFS_HIP_CHECK(hipGetLastError());
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  g.own_rowptr = std::move(nrow);
  g.own_col = std::move(ncol);
  g.rowptr = g.own_rowptr.as<int64_t>();
  g.col = g.own_col.as<int32_t>();
  g.old2new = o2n;
  device_graph_sort_rows(g, s);
  device_graph_stats(g, s);
}

void device_graph_sort_rows(DeviceGraph& g, hipStream_t s) {
  // Sorted rows make the device CSR deterministic (the atomic scatter is not) and give bottom-up
  // sweeps ascending-id neighbour order. Rows > 1024 are sorted with a segmented radix sort.
  const int64_t n = g.n;
  if (n == 0) {
    g.rows_sorted = true;
    return;
  }
  DevBuf lists((size_t)4 * n * sizeof(int32_t)), cnts(4 * sizeof(uint32_t));
  int32_t* small = lists.as<int32_t>();
  int32_t* mid = small + n;
  int32_t* big = mid + n;
  int32_t* hugel = big + n;
  uint32_t* c = cnts.as<uint32_t>();
  MSBFS_HIP_CHECK(hipMemsetAsync(c, 0, cnts.bytes, s));
  k_bucket_rows<<<grid_for(n, kBlock), kBlock, 0, s>>>(g.rowptr, n, small, c, mid, c + 1, big,
                                                       c + 2, hugel, c + 3);
  MSBFS_HIP_CHECK(hipGetLastError());
  uint32_t h[4];
  MSBFS_HIP_CHECK(hipMemcpyAsync(h, c, sizeof(h), hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  if (h[0]) {
    k_sort_rows_small<<<grid_for(h[0], kBlock), kBlock, 0, s>>>(g.rowptr, g.col, small, h[0]);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  if (h[1]) {
    k_sort_rows_lds<1024><<<std::min<uint32_t>(h[1], 4096), 256, 1024 * 4, s>>>(g.rowptr, g.col,
                                                                             mid, h[1]);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  if (h[2]) {
    k_sort_rows_lds<16384><<<std::min<uint32_t>(h[2], 1024), 256, 16384 * 4, s>>>(
        g.rowptr, g.col, big, h[2]);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  if (h[3]) {
    std::vector<int32_t> rows(h[3]);
    MSBFS_HIP_CHECK(hipMemcpyAsync(rows.data(), hugel, h[3] * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    std::vector<int64_t> rp(n + 1);
    MSBFS_HIP_CHECK(hipMemcpyAsync(rp.data(), g.rowptr, (n + 1) * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    DevBuf tmpkeys, temp;
    for (int32_t v : rows) {
      const int64_t b = rp[v], len = rp[v + 1] - rp[v];
      tmpkeys.ensure(len * sizeof(int32_t));
      size_t tb = 0;
      MSBFS_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, g.col + b,
                                                        tmpkeys.as<int32_t>(), (int)len, 0, 32, s));
      temp.ensure(tb);
      MSBFS_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, tb, g.col + b,
                                                        tmpkeys.as<int32_t>(), (int)len, 0, 32, s));
      MSBFS_HIP_CHECK(hipMemcpyAsync(g.col + b, tmpkeys.p, len * sizeof(int32_t),
                                     hipMemcpyDeviceToDevice, s));
    }
  }
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  g.rows_sorted = true;
}

// ---- frontier degree scan (shared by the level loops) ----------------------------------------
namespace {
__global__ __launch_bounds__(kBlock) void k_list_degrees(const int64_t* rowptr, const int32_t* list,
                                                         int64_t cnt, int64_t* out, int64_t chunk) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += stride) {
    const int32_t v = list[i];
    const int64_t d = rowptr[v + 1] - rowptr[v];
    out[i] = chunk == 1 ? d : (d + chunk - 1) / chunk;
  }
}
}  // namespace

size_t frontier_scan_temp_bytes(int64_t max_items) {
  size_t tb = 0;
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, (int64_t*)nullptr,
                                                   (int64_t*)nullptr, (int)std::max<int64_t>(max_items, 1)));
  return tb + (size_t)std::max<int64_t>(max_items, 1) * sizeof(int64_t) + 256;
}

void frontier_degree_scan(const int64_t* rowptr, const int32_t* list, int64_t cnt, int64_t* offs,
                          void* temp, size_t temp_bytes, hipStream_t s, int64_t chunk) {
  if (cnt <= 0) return;
  int64_t* degs = (int64_t*)temp;
  char* t2 = (char*)temp + (((size_t)cnt * sizeof(int64_t) + 255) & ~size_t(255));
  size_t tb = temp_bytes - ((size_t)(t2 - (char*)temp));
  k_list_degrees<<<grid_for(cnt, kBlock), kBlock, 0, s>>>(rowptr, list, cnt, degs, chunk);
  MSBFS_HIP_CHECK(hipGetLastError());
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(t2, tb, degs, offs, (int)cnt, s));
}

size_t inclusive_scan_temp_bytes(int64_t max_items) {
  size_t tb = 0;
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, (int64_t*)nullptr,
                                                   (int64_t*)nullptr, (int)std::max<int64_t>(max_items, 1)));
  return tb + 256;
}

void inclusive_scan_i64(const int64_t* in, int64_t* out, int64_t cnt, void* temp,
                        size_t temp_bytes, hipStream_t s) {
  if (cnt <= 0) return;
  if (cnt > INT32_MAX) fail("inclusive_scan_i64: more than 2^31 items");
  MSBFS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, in, out, (int)cnt, s));
}

}  // namespace msbfs
