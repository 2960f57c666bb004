// Per-query distance-array multi-source BFS (one int32 distance per vertex, one group at a time).
//
// Two solvers:
//  * DistSolver — direction-optimising level-synchronous BFS: top-down is edge-parallel over a
//    compacted frontier queue (load-balanced search on the frontier's degree prefix) with
//    atomicCAS(-1 -> L+1) claims; bottom-up scans the shrinking list of unvisited vertices and stops
//    at the first neighbour on level L (hubs get a whole wave). F(U) = sum_L L*|frontier_L| is
//    accumulated from the per-level queue lengths, so no distance array is ever reduced or copied.
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
    for (int i = 0; i < 2; ++i) {
      fl_[i].alloc((size_t)n * sizeof(int32_t));
      ul_[i].alloc((size_t)n * sizeof(int32_t));
      ulw_[i].alloc((size_t)n * sizeof(int32_t));
    }
    offs_.alloc((size_t)n * sizeof(int64_t));
    scan_bytes_ = frontier_scan_temp_bytes(n);
    scan_tmp_.alloc(scan_bytes_);
    ctr_.alloc(sizeof(Ctr));
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
                                                       dist_.as<int32_t>(), fl_[0].as<int32_t>(),
                                                       ctr_.as<Ctr>(), g_.old2new);
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      HostCtr c = read(s);
      int64_t nf = c.fl2, ef = (int64_t)c.ef2, Fk = 0, E2 = ef;
      int64_t na = n, ea = g_.nnz, nu = 0, nuw = 0;
      int fc = 0, uc = 0;
      bool bottom_up = false, have_ul = false;
      int32_t L = 0;
      while (nf > 0) {
        if (opt.force_dir == 1) bottom_up = false;
        else if (opt.force_dir == 2) bottom_up = L > 0;
        else if (!bottom_up) bottom_up = (double)ef > (double)ea / opt.alpha;
        else bottom_up = !((double)nf < (double)na / opt.beta);
        MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
        if (!bottom_up) {
          frontier_degree_scan(g_.rowptr, fl_[fc].as<int32_t>(), nf, offs_.as<int64_t>(),
                               scan_tmp_.p, scan_bytes_, s);
          k_td<<<grid_for(ef, kBlock, 8192), kBlock, 0, s>>>(
              fl_[fc].as<int32_t>(), nf, offs_.as<int64_t>(), g_.rowptr, g_.col,
              dist_.as<int32_t>(), L + 1, fl_[fc ^ 1].as<int32_t>(), ctr_.as<Ctr>());
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
                ul_[uc ^ 1].as<int32_t>(), fl_[fc ^ 1].as<int32_t>(), ctr_.as<Ctr>());
          if (nuw)
            k_bu_wide<<<grid_for(nuw, kBlock / 64), kBlock, 0, s>>>(
                ulw_[uc].as<int32_t>(), nuw, g_.rowptr, g_.col, dist_.as<int32_t>(), L,
                ulw_[uc ^ 1].as<int32_t>(), fl_[fc ^ 1].as<int32_t>(), ctr_.as<Ctr>());
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
        nf = c.fl2;
        ef = (int64_t)c.ef2;
        Fk += (int64_t)(L + 1) * nf;
        E2 += ef;
        fc ^= 1;
        ++L;
        if (st) st->levels++;
      }
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
  DevBuf dist_, fl_[2], ul_[2], ulw_[2], offs_, scan_tmp_, ctr_, src_;
  size_t scan_bytes_ = 0;
  std::unique_ptr<PinnedBuf> hctr_;
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
