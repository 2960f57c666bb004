// Per-query distance-array multi-source BFS (one int32 distance per vertex, one group at a time).
//
// Two solvers:
//  * DistSolver — direction-optimising level-synchronous BFS: top-down is edge-parallel over a
//    compacted frontier queue (load-balanced search on the frontier's degree prefix) with
//    atomicCAS(-1 -> L+1) claims; bottom-up scans the shrinking list of unvisited vertices and stops
//    at the first neighbour on level L (hubs get a whole wave). F(U) = sum_L L*|frontier_L| is
//    accumulated from the per-level queue lengths, so no distance array is ever reduced or copied.
//    Every frontier is appended to ONE visit-order array (level L's frontier is a contiguous
//    slice), which gives (a) device-driven level batches on low-degree graphs: up to 64 top-down
//    levels per host round trip, each level reading its slice bounds from device counter slots
//    written by the previous level (road grid: thousands of levels, one host sync per batch
//    instead of three per level as in main.cu:61-71), and (b) a reset of the distance array by
//    scattering -1 over the visited prefix when a group reached few vertices, instead of the
//    4n-byte refill per group (the reference rebuilds and copies n ints per query, main.cu:42-53).
//  * SweepSolver — the reference algorithm (BFSKernal main.cu:16-38: one thread per vertex, every
//    level rescans all n distances; GPUMultiSourceBFS main.cu:40-73) done MI355X-style: device
//    source scatter instead of a host-built n-int array + H2D copy (main.cu:44-53), a pinned
//    termination flag instead of 1-byte pageable copies (main.cu:64-69), and an on-device wave64
//    distance-sum reduction (reduce_fsum) instead of the 4n-byte D2H copy + host loop
//    (ComputeFofU main.cu:75-89). Kept as the parity/baseline algorithm (--algo sweep).
#include <algorithm>
#include <cstring>

#include "msbfs/device.hpp"
#include "msbfs/device_lists.hpp"

namespace msbfs {
namespace dist {

constexpr int kBlock = 256;

struct Ctr {
  Slot32 fl2, ul2, ulw2, updated;
  Slot64 ef2, eu2;
};
struct HostCtr {
  uint32_t fl2, ul2, ulw2, updated;
  unsigned long long ef2, eu2;
};

constexpr int kWaves = kBlock / 64;

// Device-driven level batches (low-degree graphs): slot j describes level j's frontier, the
// slice ord[lo, lo + nf); the kernel of level j appends level j+1's vertices after it and fills
// slot j+1. stop = 1: the level's push -> pull test fired, the host continues from there.
struct alignas(128) LevelSlot {
  unsigned long long lo;
  uint32_t nf;
  uint32_t stop;
  unsigned long long ef;  // degree sum of the frontier
  uint32_t pad[26];
};
constexpr int kMaxBatch = 64;

// one top-down level of a device-driven batch: thread per frontier vertex (max degree <= 64)
__global__ __launch_bounds__(kBlock) void k_td_dd(int32_t* ord, LevelSlot* slots, int j,
                                                  int32_t level0, const int64_t* rowptr,
                                                  const int32_t* col, int32_t* dist,
                                                  unsigned long long ef_stop) {
  __shared__ LdsQueue q;
  __shared__ unsigned long long scratch[kWaves];
  const LevelSlot cur = slots[j];
  if (cur.nf == 0) return;  // frontier died (or an earlier level stopped the batch)
  if (j > 0 && cur.ef > ef_stop) {  // the host would pull here: stop the batch at this level
    if (blockIdx.x == 0 && threadIdx.x == 0) slots[j].stop = 1u;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) slots[j + 1].lo = cur.lo + cur.nf;
  q_init(q);
  __syncthreads();
  int32_t* out = ord + cur.lo + cur.nf;
  const int32_t nl = level0 + j + 1;  // slot 0 is level level0
  unsigned long long ef = 0;
  for (int64_t b = (int64_t)blockIdx.x * kBlock; b < cur.nf; b += (int64_t)gridDim.x * kBlock) {
    const int64_t i = b + threadIdx.x;
    int64_t e = 0, end = 0;
    if (i < cur.nf) {
      const int32_t u = ord[cur.lo + i];
      e = rowptr[u];
      end = rowptr[u + 1];
    }
    // one edge per step for every thread (block-uniform steps: the queue flushes every step)
    while (__syncthreads_or(e < end)) {
      bool app = false;
      int32_t v = 0;
      if (e < end) {
        v = col[e++];
        if (dist[v] < 0) app = atomicCAS(&dist[v], -1, nl) == -1;
        if (app) ef += (unsigned long long)(rowptr[v + 1] - rowptr[v]);
      }
      q_push(q, app, v);
      q_flush(q, out, &slots[j + 1].nf, kBlock, false);
    }
  }
  q_flush(q, out, &slots[j + 1].nf, 0, true);
  block_sum_add(ef, &slots[j + 1].ef, scratch);
}

// dist[ord[i]] = -1 for the visited prefix (the reset when a group reached few vertices)
__global__ __launch_bounds__(kBlock) void k_reset_visited(const int32_t* ord, int64_t cnt,
                                                          int32_t* dist) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < cnt;
       i += (int64_t)gridDim.x * kBlock)
    dist[ord[i]] = -1;
}

__global__ __launch_bounds__(kBlock) void k_init(const int32_t* src, int64_t ns, int64_t n,
                                                 const int64_t* rowptr, int32_t* dist, int32_t* fl,
                                                 Ctr* ctr, const int32_t* relabel) {
  __shared__ LdsQueue q;
  __shared__ unsigned long long scratch[kWaves];
  q_init(q);
  __syncthreads();
  unsigned long long ef = 0;
  for (int64_t b = (int64_t)blockIdx.x * kBlock; b < ns; b += (int64_t)gridDim.x * kBlock) {
    const int64_t i = b + threadIdx.x;
    bool app = false;
    int32_t v = -1;
    if (i < ns) {
      v = src[i];
      if (v >= 0 && v < n) {  // main.cu:49 range check
        if (relabel) v = relabel[v];
        app = atomicCAS(&dist[v], -1, 0) == -1;
        if (app) ef += (unsigned long long)(rowptr[v + 1] - rowptr[v]);
      }
    }
    q_push(q, app, v);
    q_flush(q, fl, &ctr->fl2.v, kBlock, false);
  }
  q_flush(q, fl, &ctr->fl2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
}

// top-down: thread per frontier edge (load-balanced search on the frontier's degree prefix)
__global__ __launch_bounds__(kBlock) void k_td(const int32_t* fl, int64_t nf, const int64_t* offs,
                                               const int64_t* rowptr, const int32_t* col,
                                               int32_t* dist, int32_t nl, int32_t* fl2, Ctr* ctr) {
  __shared__ LdsQueue q;
  __shared__ unsigned long long scratch[kWaves];
  q_init(q);
  __syncthreads();
  const int64_t total = offs[nf - 1];
  unsigned long long ef = 0;
  for (int64_t b = (int64_t)blockIdx.x * kBlock; b < total; b += (int64_t)gridDim.x * kBlock) {
    const int64_t e = b + threadIdx.x;
    bool app = false;
    int32_t v = 0;
    if (e < total) {
      const int64_t i = upper_bound_i64(offs, nf, e);
      const int32_t u = fl[i];
      const int64_t start = i ? offs[i - 1] : 0;
      v = col[rowptr[u] + (e - start)];
      if (dist[v] < 0) app = atomicCAS(&dist[v], -1, nl) == -1;
      if (app) ef += (unsigned long long)(rowptr[v + 1] - rowptr[v]);
    }
    q_push(q, app, v);
    q_flush(q, fl2, &ctr->fl2.v, kBlock, false);
  }
  q_flush(q, fl2, &ctr->fl2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
}

__global__ __launch_bounds__(kBlock) void k_build_unvisited(int64_t n, const int64_t* rowptr,
                                                            const int32_t* dist, int wide,
                                                            int32_t* ul, int32_t* ulw, Ctr* ctr) {
  __shared__ LdsQueue qn, qw;
  __shared__ unsigned long long scratch[kWaves];
  q_init(qn);
  q_init(qw);
  __syncthreads();
  unsigned long long eu = 0;
  for (int64_t b = (int64_t)blockIdx.x * kBlock; b < n; b += (int64_t)gridDim.x * kBlock) {
    const int64_t i = b + threadIdx.x;
    int64_t d = 0;
    bool ok = false;
    if (i < n) {
      d = rowptr[i + 1] - rowptr[i];
      ok = d > 0 && dist[i] < 0;
    }
    if (ok) eu += (unsigned long long)d;
    q_push(qn, ok && d <= wide, (int32_t)i);
    q_push(qw, ok && d > wide, (int32_t)i);
    q_flush(qn, ul, &ctr->ul2.v, kBlock, false);
    q_flush(qw, ulw, &ctr->ulw2.v, kBlock, false);
  }
  q_flush(qn, ul, &ctr->ul2.v, 0, true);
  q_flush(qw, ulw, &ctr->ulw2.v, 0, true);
  block_sum_add(eu, &ctr->eu2.v, scratch);
}

// bottom-up, thread per unvisited narrow vertex: stop at the first neighbour on level L
__global__ __launch_bounds__(kBlock) void k_bu(const int32_t* ul, int64_t nu, const int64_t* rowptr,
                                               const int32_t* col, int32_t* dist, int32_t L,
                                               int32_t* ul2, int32_t* fl2, Ctr* ctr) {
  __shared__ LdsQueue qf, qk;
  __shared__ unsigned long long scratch[kWaves];
  q_init(qf);
  q_init(qk);
  __syncthreads();
  unsigned long long ef = 0, eu = 0;
  for (int64_t b = (int64_t)blockIdx.x * kBlock; b < nu; b += (int64_t)gridDim.x * kBlock) {
    const int64_t i = b + threadIdx.x;
    bool found = false, keep = false;
    int32_t v = 0;
    if (i < nu && dist[ul[i]] < 0) {  // visited by an intervening top-down level: drop
      v = ul[i];
      const int64_t bb = rowptr[v], e = rowptr[v + 1];
      for (int64_t j = bb; j < e; ++j)
        if (dist[col[j]] == L) {
          found = true;
          break;
        }
      if (found) {
        dist[v] = L + 1;
        ef += (unsigned long long)(e - bb);
      } else {
        keep = true;
        eu += (unsigned long long)(e - bb);
      }
    }
    q_push(qf, found, v);
    q_push(qk, keep, v);
    q_flush(qf, fl2, &ctr->fl2.v, kBlock, false);
    q_flush(qk, ul2, &ctr->ul2.v, kBlock, false);
  }
  q_flush(qf, fl2, &ctr->fl2.v, 0, true);
  q_flush(qk, ul2, &ctr->ul2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(eu, &ctr->eu2.v, scratch);
}

// bottom-up, one wave per high-degree unvisited vertex (ballot early exit every 64 neighbours);
// rounds are block-uniform (one vertex per wave per round) so the block queues can flush
__global__ __launch_bounds__(kBlock) void k_bu_wide(const int32_t* ul, int64_t nu,
                                                    const int64_t* rowptr, const int32_t* col,
                                                    int32_t* dist, int32_t L, int32_t* ul2,
                                                    int32_t* fl2, Ctr* ctr) {
  __shared__ LdsQueue qf, qk;
  __shared__ unsigned long long scratch[kWaves];
  q_init(qf);
  q_init(qk);
  __syncthreads();
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  unsigned long long ef = 0, eu = 0;
  for (int64_t b = (int64_t)blockIdx.x * kWaves; b < nu; b += (int64_t)gridDim.x * kWaves) {
    const int64_t i = b + wv;
    bool found = false, keep = false;
    int32_t v = 0;
    if (i < nu) {
      v = ul[i];
      if (dist[v] < 0) {  // wave-uniform
        const int64_t bb = rowptr[v], e = rowptr[v + 1];
        for (int64_t j0 = bb; j0 < e; j0 += 64) {
          const int64_t j = j0 + lane;
          const bool hit = j < e && dist[col[j]] == L;
          if (__ballot(hit)) {
            found = true;
            break;
          }
        }
        keep = !found;
        if (lane == 0) {
          if (found) {
            dist[v] = L + 1;
            ef += (unsigned long long)(e - bb);
          } else {
            eu += (unsigned long long)(e - bb);
          }
        }
      }
    }
    q_push(qf, found && lane == 0, v);
    q_push(qk, keep && lane == 0, v);
    q_flush(qf, fl2, &ctr->fl2.v, kWaves, false);
    q_flush(qk, ul2, &ctr->ulw2.v, kWaves, false);
  }
  q_flush(qf, fl2, &ctr->fl2.v, 0, true);
  q_flush(qk, ul2, &ctr->ulw2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(eu, &ctr->eu2.v, scratch);
}

// ---- reference-algorithm sweep -------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sweep_level(const int64_t* rowptr, const int32_t* col,
                                                        int64_t n, int32_t* dist, int32_t L,
                                                        uint32_t* updated) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  bool upd = false;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
    if (dist[v] != L) continue;
    for (int64_t j = rowptr[v]; j < rowptr[v + 1]; ++j) {
      const int32_t u = col[j];
      // same benign race as the reference (main.cu:30-33): every writer stores L+1
      if (dist[u] == -1) {
        dist[u] = L + 1;
        upd = true;
      }
    }
  }
  // one plain store per wave that found work (the reference's `*d_updated = true`)
  if (__ballot(upd) && lane_id() == 0) *(volatile uint32_t*)updated = 1u;
}

// wave64 reduction of the distance sum (and the reached-degree sum for the TEPS numerator)
__global__ __launch_bounds__(kBlock) void k_reduce_fsum(const int32_t* dist, const int64_t* rowptr,
                                                        int64_t n, unsigned long long* out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long f = 0, e = 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
    const int32_t d = dist[v];
    if (d >= 0) {  // only reachable vertices count (main.cu:84-85)
      f += (unsigned long long)d;
      e += (unsigned long long)(rowptr[v + 1] - rowptr[v]);
    }
  }
  __shared__ unsigned long long sf[kBlock / 64], se[kBlock / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    f += __shfl_xor(f, off);
    e += __shfl_xor(e, off);
  }
  if (lane_id() == 0) {
    sf[threadIdx.x >> 6] = f;
    se[threadIdx.x >> 6] = e;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, b = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      a += sf[w];
      b += se[w];
    }
    atomicAdd(&out[0], a);
    atomicAdd(&out[1], b);
  }
}

class DistSolver final : public Solver {
 public:
  explicit DistSolver(const DeviceGraph& g) : g_(g) {
    const int64_t n = std::max<int64_t>(g.n, 1);
    dist_.alloc((size_t)n * sizeof(int32_t));
    MSBFS_HIP_CHECK(hipMemset(dist_.p, 0xFF, dist_.bytes));
    ord_.alloc((size_t)n * sizeof(int32_t));
    for (int i = 0; i < 2; ++i) {
      ul_[i].alloc((size_t)n * sizeof(int32_t));
      ulw_[i].alloc((size_t)n * sizeof(int32_t));
    }
    offs_.alloc((size_t)n * sizeof(int64_t));
    scan_bytes_ = frontier_scan_temp_bytes(n);
    scan_tmp_.alloc(scan_bytes_);
    ctr_.alloc(sizeof(Ctr));
    hctr_ = std::make_unique<PinnedBuf>(sizeof(Ctr));
    slots_.alloc((size_t)(kMaxBatch + 1) * sizeof(LevelSlot));
    hslots_ = std::make_unique<PinnedBuf>((size_t)(kMaxBatch + 1) * sizeof(LevelSlot));
  }

  void run(int64_t K, const int64_t* qoff, const int32_t* qids, int64_t* F, int64_t* edges2,
           RunStats* st, hipStream_t s) override {
    const int64_t n = g_.n;
    int64_t maxs = 1;
    for (int64_t k = 0; k < K; ++k) maxs = std::max(maxs, qoff[k + 1] - qoff[k]);
    src_.ensure((size_t)maxs * sizeof(int32_t));
    // device-driven top-down batches where every frontier vertex has few edges (road-like)
    const bool dd = g_.max_degree <= 64 && opt.force_dir != 2;
    for (int64_t k = 0; k < K; ++k) {
      const int64_t ns = qoff[k + 1] - qoff[k];
      // reset: the previous group's visited vertices are ord[0, visited_); scatter -1 over them
      // when that is cheaper than refilling all n ints
      if (visited_ * 8 < n) {
        if (visited_)
          k_reset_visited<<<grid_for(visited_, kBlock, 4096), kBlock, 0, s>>>(
              ord_.as<int32_t>(), visited_, dist_.as<int32_t>());
      } else {
        MSBFS_HIP_CHECK(hipMemsetAsync(dist_.p, 0xFF, (size_t)std::max<int64_t>(n, 1) * 4, s));
      }
      // until this group finishes, an exception (caught by the C API guard, the solver living
      // on) may leave any vertex marked: force the full refill for the next group
      visited_ = n;
      MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
      if (ns) {
        MSBFS_HIP_CHECK(hipMemcpyAsync(src_.p, qids + qoff[k], ns * sizeof(int32_t),
                                       hipMemcpyHostToDevice, s));
        k_init<<<grid_for(ns, kBlock), kBlock, 0, s>>>(src_.as<int32_t>(), ns, n, g_.rowptr,
                                                       dist_.as<int32_t>(), ord_.as<int32_t>(),
                                                       ctr_.as<Ctr>(), g_.old2new);
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      HostCtr c = read(s);
      // frontier of level L = ord[lo, lo + nf)
      int64_t lo = 0, nf = c.fl2, ef = (int64_t)c.ef2, Fk = 0, E2 = ef;
      int64_t na = n, ea = g_.nnz, nu = 0, nuw = 0;
      int uc = 0;
      bool bottom_up = false, have_ul = false;
      int32_t L = 0;
      int batch = 4;
      while (nf > 0) {
        if (opt.force_dir == 1) bottom_up = false;
        else if (opt.force_dir == 2) bottom_up = L > 0;
        else if (!bottom_up) bottom_up = (double)ef > (double)ea / opt.alpha;
        else bottom_up = !((double)nf < (double)na / opt.beta);
        if (dd && !bottom_up) {
          // ---- up to `batch` top-down levels, one host round trip
          MSBFS_HIP_CHECK(hipMemsetAsync(slots_.p, 0, slots_.bytes, s));
          LevelSlot s0{};
          s0.lo = (unsigned long long)lo;
          s0.nf = (uint32_t)nf;
          s0.ef = (unsigned long long)ef;
          MSBFS_HIP_CHECK(hipMemcpyAsync(slots_.p, &s0, sizeof(s0), hipMemcpyHostToDevice, s));
          const unsigned long long ef_stop =
              opt.force_dir == 1 ? ~0ull
                                 : (unsigned long long)std::max(0.0, std::min((double)ea / opt.alpha, 1.8e19));
          const int grid = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
          trace::Range range_batch("dist L%d-%d TD batch", L + 1, L + batch);
          for (int j = 0; j < batch; ++j)
            k_td_dd<<<grid, kBlock, 0, s>>>(ord_.as<int32_t>(), slots_.as<LevelSlot>(), j, L,
                                            g_.rowptr, g_.col, dist_.as<int32_t>(), ef_stop);
          // (slot j describes level L + j)
          MSBFS_HIP_CHECK(hipGetLastError());
          MSBFS_HIP_CHECK(hipMemcpyAsync(hslots_->p, slots_.p, (size_t)(batch + 1) * sizeof(LevelSlot),
                                         hipMemcpyDeviceToHost, s));
          MSBFS_HIP_CHECK(hipStreamSynchronize(s));
          const LevelSlot* h = hslots_->as<LevelSlot>();
          int real = 0;  // levels that expanded
          while (real < batch && h[real].nf > 0 && !h[real].stop) {
            Fk += (int64_t)(L + real + 1) * (int64_t)h[real + 1].nf;
            E2 += (int64_t)h[real + 1].ef;
            ++real;
          }
          if (st) {
            st->td_levels += real;
            st->levels += real;
          }
          L += real;
          lo = (int64_t)h[real].lo;
          nf = h[real].nf;
          ef = (int64_t)h[real].ef;
          if (real == batch) batch = std::min(batch * 2, kMaxBatch);
          if (real < batch && h[real].stop) bottom_up = true;  // the batch stopped for a pull
          if (nf == 0) break;
          if (!bottom_up) continue;
        }
        MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
        int32_t* out = ord_.as<int32_t>() + lo + nf;  // the next frontier follows this one
        if (!bottom_up) {
          frontier_degree_scan(g_.rowptr, ord_.as<int32_t>() + lo, nf, offs_.as<int64_t>(),
                               scan_tmp_.p, scan_bytes_, s);
          k_td<<<grid_for(ef, kBlock, 8192), kBlock, 0, s>>>(
              ord_.as<int32_t>() + lo, nf, offs_.as<int64_t>(), g_.rowptr, g_.col,
              dist_.as<int32_t>(), L + 1, out, ctr_.as<Ctr>());
          MSBFS_HIP_CHECK(hipGetLastError());
          if (st) st->td_levels++;
        } else {
          if (!have_ul) {
            k_build_unvisited<<<grid_for(n, kBlock), kBlock, 0, s>>>(
                n, g_.rowptr, dist_.as<int32_t>(), opt.wide_degree, ul_[0].as<int32_t>(),
                ulw_[0].as<int32_t>(), ctr_.as<Ctr>());
            MSBFS_HIP_CHECK(hipGetLastError());
            c = read(s);
            nu = c.ul2;
            nuw = c.ulw2;
            have_ul = true;
            uc = 0;
            MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
          }
          if (nu)
            k_bu<<<grid_for(nu, kBlock), kBlock, 0, s>>>(
                ul_[uc].as<int32_t>(), nu, g_.rowptr, g_.col, dist_.as<int32_t>(), L,
                ul_[uc ^ 1].as<int32_t>(), out, ctr_.as<Ctr>());
          if (nuw)
            k_bu_wide<<<grid_for(nuw, kBlock / 64), kBlock, 0, s>>>(
                ulw_[uc].as<int32_t>(), nuw, g_.rowptr, g_.col, dist_.as<int32_t>(), L,
                ulw_[uc ^ 1].as<int32_t>(), out, ctr_.as<Ctr>());
          MSBFS_HIP_CHECK(hipGetLastError());
          uc ^= 1;
          if (st) st->bu_levels++;
        }
        c = read(s);
        if (bottom_up) {
          nu = c.ul2;
          nuw = c.ulw2;
          na = nu + nuw;
          ea = (int64_t)c.eu2;
        }  // after a top-down level the lists may hold visited vertices: dropped lazily
        lo += nf;
        nf = c.fl2;
        ef = (int64_t)c.ef2;
        Fk += (int64_t)(L + 1) * nf;
        E2 += ef;
        ++L;
        if (st) st->levels++;
      }
      visited_ = lo + nf;  // every visited vertex sits in ord[0, lo + nf)
      F[k] = Fk;
      if (edges2) edges2[k] = E2;
    }
  }

 private:
  HostCtr read(hipStream_t s) {
    MSBFS_HIP_CHECK(hipMemcpyAsync(hctr_->p, ctr_.p, sizeof(Ctr), hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    const Ctr* c = hctr_->as<Ctr>();
    return HostCtr{c->fl2.v, c->ul2.v, c->ulw2.v, c->updated.v, c->ef2.v, c->eu2.v};
  }
  const DeviceGraph& g_;
  DevBuf dist_, ord_, ul_[2], ulw_[2], offs_, scan_tmp_, ctr_, src_, slots_;
  size_t scan_bytes_ = 0;
  int64_t visited_ = 0;  // vertices the last group reached (ord[0, visited_) to reset)
  std::unique_ptr<PinnedBuf> hctr_, hslots_;
};

class SweepSolver final : public Solver {
 public:
  explicit SweepSolver(const DeviceGraph& g) : g_(g) {
    const int64_t n = std::max<int64_t>(g.n, 1);
    dist_.alloc((size_t)n * sizeof(int32_t));
    fl_.alloc((size_t)n * sizeof(int32_t));
    ctr_.alloc(sizeof(Ctr));
    red_.alloc(2 * sizeof(unsigned long long));
    hctr_ = std::make_unique<PinnedBuf>(sizeof(Ctr));
  }
  void run(int64_t K, const int64_t* qoff, const int32_t* qids, int64_t* F, int64_t* edges2,
           RunStats* st, hipStream_t s) override {
    const int64_t n = g_.n;
    int64_t maxs = 1;
    for (int64_t k = 0; k < K; ++k) maxs = std::max(maxs, qoff[k + 1] - qoff[k]);
    src_.ensure((size_t)maxs * sizeof(int32_t));
    for (int64_t k = 0; k < K; ++k) {
      const int64_t ns = qoff[k + 1] - qoff[k];
      MSBFS_HIP_CHECK(hipMemsetAsync(dist_.p, 0xFF, (size_t)std::max<int64_t>(n, 1) * 4, s));
      MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
      if (ns) {
        MSBFS_HIP_CHECK(hipMemcpyAsync(src_.p, qids + qoff[k], ns * sizeof(int32_t),
                                       hipMemcpyHostToDevice, s));
        k_init<<<grid_for(ns, kBlock), kBlock, 0, s>>>(src_.as<int32_t>(), ns, n, g_.rowptr,
                                                       dist_.as<int32_t>(), fl_.as<int32_t>(),
                                                       ctr_.as<Ctr>(), g_.old2new);
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      // level loop: one launch per level + termination flag (main.cu:61-71)
      Ctr* hc = hctr_->as<Ctr>();
      for (int32_t L = 0;; ++L) {
        MSBFS_HIP_CHECK(hipMemsetAsync(&ctr_.as<Ctr>()->updated.v, 0, sizeof(uint32_t), s));
        if (n)
          k_sweep_level<<<grid_for(n, kBlock, 8192), kBlock, 0, s>>>(
              g_.rowptr, g_.col, n, dist_.as<int32_t>(), L, &ctr_.as<Ctr>()->updated.v);
        MSBFS_HIP_CHECK(hipGetLastError());
        MSBFS_HIP_CHECK(hipMemcpyAsync(&hc->updated.v, &ctr_.as<Ctr>()->updated.v, sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, s));
        MSBFS_HIP_CHECK(hipStreamSynchronize(s));
        if (st) st->levels++;
        if (!hc->updated.v) break;
      }
      MSBFS_HIP_CHECK(hipMemsetAsync(red_.p, 0, red_.bytes, s));
      if (n)
        k_reduce_fsum<<<grid_for(n, kBlock, 2048), kBlock, 0, s>>>(
            dist_.as<int32_t>(), g_.rowptr, n, red_.as<unsigned long long>());
      MSBFS_HIP_CHECK(hipGetLastError());
      unsigned long long h[2];
      MSBFS_HIP_CHECK(hipMemcpyAsync(h, red_.p, sizeof(h), hipMemcpyDeviceToHost, s));
      MSBFS_HIP_CHECK(hipStreamSynchronize(s));
      F[k] = (int64_t)h[0];
      if (edges2) edges2[k] = (int64_t)h[1];
    }
  }

 private:
  const DeviceGraph& g_;
  DevBuf dist_, fl_, ctr_, red_, src_;
  std::unique_ptr<PinnedBuf> hctr_;
};

}  // namespace dist

std::unique_ptr<Solver> make_dist_solver(const DeviceGraph& g) {
  return std::make_unique<dist::DistSolver>(g);
}
std::unique_ptr<Solver> make_sweep_solver(const DeviceGraph& g) {
  return std::make_unique<dist::SweepSolver>(g);
}

}  // namespace msbfs
