// Block-level list building for grid-stride level kernels (HIP only).
//
// Appending to a global list with one atomic per wave serialises on the counter's cache line
// (device-scope atomics on one address execute one at a time at the memory side); building
// frontiers / active lists that way cost more than the traversal itself. Here each block
// collects items in an LDS queue (wave-aggregated LDS atomics) and flushes it with ONE global
// atomic per ~kQCap items, writing the items out as a contiguous, coalesced run.
#pragma once

#include "msbfs/device.hpp"

namespace msbfs {

constexpr int kQCap = 1024;  // LDS queue capacity (items) per block

// CAP items; bigger queues (full-graph list builds) mean fewer flushes, i.e. fewer atomics on
// the one global counter, which the memory side executes one at a time
template <int CAP>
struct LdsQueueN {
  int32_t item[CAP];
  uint32_t n;
  uint32_t base;
};
using LdsQueue = LdsQueueN<kQCap>;

// Call from every thread, followed by a __syncthreads() before the first push.
template <int CAP>
__device__ __forceinline__ void q_init(LdsQueueN<CAP>& q) {
  if (threadIdx.x == 0) q.n = 0;
}

// wave-aggregated push into the block queue (call from converged wave code)
template <int CAP>
__device__ __forceinline__ void q_push(LdsQueueN<CAP>& q, bool pred, int32_t v) {
  const uint64_t mask = __ballot(pred);
  if (!mask) return;
  const int leader = __ffsll((unsigned long long)mask) - 1;
  uint32_t pos = 0;
  if (lane_id() == leader) pos = atomicAdd(&q.n, (uint32_t)__popcll(mask));
  pos = __shfl(pos, leader) + (uint32_t)__popcll(mask & lanemask_lt());
  if (pred) q.item[pos] = v;
}

// Flush each of NQ queues to its out[] when it may not hold another `room` items (or always, at
// the end), sharing the barriers: two when nothing is flushed, four otherwise (the pull kernels
// check three queues after every tile; flushed one at a time they paid up to 15 barriers a tile).
// Must be called by every thread of the block (block-uniform control flow); blockDim >= NQ.
template <int CAP, int NQ>
__device__ __forceinline__ void q_flush_n(LdsQueueN<CAP>* const (&q)[NQ], int32_t* const (&out)[NQ],
                                          uint32_t* const (&gcnt)[NQ], int room, bool force) {
  __syncthreads();
  uint32_t n[NQ];
  bool f[NQ], any = false;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    n[i] = q[i]->n;
    f[i] = n[i] != 0 && (force || n[i] + (uint32_t)room > (uint32_t)CAP);
    any |= f[i];
  }
  __syncthreads();  // every count read before any push or reset
  if (!any) return;
  // (no pushes until the last barrier: the counts may be reset here)
#pragma unroll
  for (int i = 0; i < NQ; ++i)
    if (f[i] && threadIdx.x == (unsigned)i) {
      q[i]->base = atomicAdd(gcnt[i], n[i]);
      q[i]->n = 0;
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if (!f[i]) continue;
    const uint32_t base = q[i]->base;
    for (uint32_t j = threadIdx.x; j < n[i]; j += blockDim.x) out[i][base + j] = q[i]->item[j];
  }
  __syncthreads();  // items read before the next pushes overwrite them
}

template <int CAP>
__device__ __forceinline__ void q_flush(LdsQueueN<CAP>& q, int32_t* out, uint32_t* gcnt, int room,
                                        bool force) {
  LdsQueueN<CAP>* const qs[1] = {&q};
  int32_t* const os[1] = {out};
  uint32_t* const cs[1] = {gcnt};
  q_flush_n<CAP, 1>(qs, os, cs, room, force);
}

// block-wide sum of per-thread values, one atomic per block; scratch holds blockDim/64 values
__device__ __forceinline__ void block_sum_add(unsigned long long val, unsigned long long* dst,
                                              unsigned long long* scratch) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) val += __shfl_xor(val, off);
  __syncthreads();
  if (lane_id() == 0) scratch[threadIdx.x >> 6] = val;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += scratch[w];
    if (t) atomicAdd(dst, t);
  }
}

// Device counters; every field on its own 128-B line so unrelated atomics never share a line.
struct alignas(128) Slot32 {
  uint32_t v;
  uint32_t pad[31];
};
struct alignas(128) Slot64 {
  unsigned long long v;
  uint32_t pad[30];
};

}  // namespace msbfs
