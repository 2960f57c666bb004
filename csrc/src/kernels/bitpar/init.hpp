// Bit-parallel MS-BFS: per-batch initialisation kernels (sources, lazy row resets) and the
// accumulator reset shared by the level kernels.
#pragma once

#include "common.hpp"

namespace msbfs {
namespace bp {

// ---------------------------------------------------------------------------------------------
// init: scatter the batch's sources (v, local group) into both visited buffers and the
// top-down accumulator; dedupe vertices into the first frontier list via stamps.
// ---------------------------------------------------------------------------------------------
// Only vis_[0] is cleared per batch (hipMemset of n*W words); vis_[1] still holds the previous
// batch's rows and is made valid row by row: k_init ORs sources into both buffers, so their
// rows are zeroed first; top-down finalize writes both buffers of every touched vertex; the
// first bottom-up level writes Wb for every active (deg > 0, not done) vertex. Rows of deg-0
// vertices are never read (no edges lead to them), so after the first bottom-up level both
// buffers are valid wherever a kernel looks. Saves one n*W*8-byte fill per batch.
template <int W>
__global__ __launch_bounds__(kBlock) void k_zero_src_rows(const int32_t* pv, int64_t np,
                                                         const int32_t* relabel, uint64_t* visA,
                                                         uint64_t* visB) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < np * W;
       i += (int64_t)gridDim.x * kBlock) {
    int32_t v = pv[i / W];
    if (relabel) v = relabel[v];
    visA[(int64_t)v * W + (i % W)] = 0;
    visB[(int64_t)v * W + (i % W)] = 0;
  }
}

// Lazy batches (every batch of the fused-count path and the hybrid phase A): no per-batch fill of
// vis_[0]. Until the first pull level a row is read only if its vertex is visited: the sources'
// rows (k_zero_src_rows), top-down targets and touched vertices through the anyvis guard (`lzv`,
// k_td_finalize's `lazy`: a vertex no group has visited has an all-zero row, so a stale row is
// never used). The first pull level filters every probe and reads its own rows through a
// snapshot of anyvis taken at the level start (k_bu_narrow `snap`), and writes the rows of all its
// active vertices; a top-down level right after it reads the old rows through the same snapshot
// (k_td_expand `osnap`). From then on both buffers hold valid rows for every vertex a kernel
// reads (a vertex finished at the first pull level and first visited there keeps a stale row in
// the other buffer, but no active vertex two levels later is its neighbour). Phase A with
// several parts instead zeroes its own rows here (its pulls cover only them).
// rows of the vertices v = part + i*nparts, i < cnt (G lanes per row, coalesced)
template <int W>
__global__ __launch_bounds__(kBlock) void k_zero_part_rows(int64_t cnt, int part, int nparts,
                                                          uint64_t* vis) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G;
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t x = t; x < cnt * G; x += stride) {
    const int64_t v = part + (x / G) * nparts;
    stv<VW>(vis + v * W + (x % G) * VW, vzero<VW>());
  }
}

template <int W, bool COUNT>
__global__ __launch_bounds__(kBlock) void k_init(const int32_t* pv, const int32_t* pk, int64_t np,
                                                 const int64_t* rowptr, uint64_t* visA,
                                                 uint64_t* visB, uint64_t* acc, int32_t* stamp,
                                                 int32_t epoch, int32_t* fl, Ctr* ctr,
                                                 unsigned long long* E, uint64_t* alive,
                                                 uint32_t* anyvis, const int32_t* relabel) {
  __shared__ LdsQueue q;
  __shared__ unsigned long long scratch[kWaves];
  q_init(q);
  __syncthreads();
  unsigned long long ef = 0;
  for (int64_t b = (int64_t)blockIdx.x * kBlock; b < np; b += (int64_t)gridDim.x * kBlock) {
    const int64_t i = b + threadIdx.x;
    bool app = false;
    int32_t v = 0;
    if (i < np) {
      v = pv[i];
      if (relabel) v = relabel[v];  // user id -> internal (degree-ordered) id
      const int k = pk[i];
      const int word = k >> 6;
      const uint64_t bit = 1ull << (k & 63);
      const uint64_t old = atomicOr((unsigned long long*)&visA[(int64_t)v * W + word], bit);
      if (!(old & bit)) {
        atomicOr((unsigned long long*)&visB[(int64_t)v * W + word], bit);
        atomicOr((unsigned long long*)&acc[(int64_t)v * W + word], bit);
        (void)alive;  // alive (groups with a valid source) is uploaded by the host
        const unsigned long long deg = (unsigned long long)(rowptr[v + 1] - rowptr[v]);
        if constexpr (COUNT) atomicAdd(&E[k], deg);
        app = atomicExch(&stamp[v], epoch) != epoch;
        if (app) {
          ef += deg;
          atomicOr(&anyvis[v >> 5], 1u << (v & 31));
        }
      }
    }
    q_push(q, app, v);
    q_flush(q, fl, &ctr->fl2.v, kBlock, false);
  }
  q_flush(q, fl, &ctr->fl2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ef, &ctr->ev2.v, scratch);
}


template <int W>
__global__ __launch_bounds__(kBlock) void k_zero_acc(const int32_t* fl, int64_t nf, uint64_t* acc) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = t; i < nf * G; i += stride) {
    const int64_t idx = i / G;
    const int slot = (int)(i % G);
    stv<VW>(acc + (int64_t)fl[idx] * W + slot * VW, vzero<VW>());
  }
}

}  // namespace bp
}  // namespace msbfs
