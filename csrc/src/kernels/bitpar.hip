// Bit-parallel, direction-optimising multi-source BFS over up to 64*W query groups at once.
//
// What it replaces: the reference runs each query group as its own level-synchronous BFS with a
// thread-per-vertex kernel that rescans all n distances every level (BFSKernal main.cu:16-38,
// driven by GPUMultiSourceBFS main.cu:40-73), then copies all n distances to the host to sum them
// (ComputeFofU main.cu:75-89). Queries run strictly one after another per rank
// (main.cu:312-322).
//
// Here one pass over the graph advances 64*W groups together (MS-BFS, Then et al. VLDB'15):
//  * every vertex owns W 64-bit words: bit k of word j = "visited by group 64j+k".
//  * top-down levels (small frontiers) push frontier bits along edges with 64-bit atomicOr into
//    an accumulator, edge-parallel via a load-balanced search over the frontier's degree prefix
//    (no hub serialisation);
//  * bottom-up levels (large frontiers) pull: an unfinished vertex ORs its neighbours' visited
//    words and stops as soon as every still-alive group is covered (early exit). Double-buffered
//    visited arrays make the pull race-free without a separate frontier array (a neighbour bit
//    visited at any level <= L can only have been set exactly at L if it is still missing here).
//    Low-degree vertices get G lanes each; high-degree vertices are cut into fixed-size edge
//    chunks that many waves scan in parallel (partial ORs merged with atomicOr, then a finalize
//    pass), so a 10^6-neighbour hub never serialises a level on one wave.
//  * per-group F(U) = sum_level level * |newly visited| is accumulated on chip: every new bit adds
//    to a per-group LDS counter; one global atomic per group per block at the end. Only 8 bytes
//    per group ever leave the device (vs 4n bytes per query in the reference).
//  * groups whose frontier died are masked out ("alive" words), so groups stuck in small
//    components never stop other groups' vertices from finishing.
//  * list building (active lists, frontiers, touched sets) goes through per-block LDS queues:
//    one global atomic per ~1K items instead of one per wave (same-line atomics serialise).
// Lane mapping for wave64: each lane owns VW (1-2) words = one 8-16 B load, a vertex's W words are
// spread over G = W/VW consecutive lanes, so W=16 reads a vertex's 128-B line in one coalesced
// wave-instruction slice.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>

#include "msbfs/device.hpp"
#include "msbfs/device_lists.hpp"

namespace msbfs {
namespace bp {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kChunk = 1024;      // bottom-up edge chunk for wide vertices
constexpr int kMaxGrid = 2048;    // blocks of the grid-stride level kernels
constexpr int kSmallDeg = 64;     // max degree for the vertex-parallel top-down expansion

template <int W>
struct Lay {
  static constexpr int VW = W >= 2 ? 2 : 1;
  static constexpr int G = W / VW;      // lanes per vertex
  static constexpr int VPW = 64 / G;    // vertices per wave
  static constexpr int TILE = kWaves * VPW;  // vertices per block iteration
  static constexpr uint64_t GBITS = (G == 64) ? ~0ull : ((1ull << G) - 1);
};

template <int VW>
struct V {
  uint64_t w[VW];
};

template <int VW>
__device__ __forceinline__ V<VW> ldv(const uint64_t* p) {
  V<VW> r;
  if constexpr (VW == 2) {
    typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
    const u2 x = *(const u2*)p;
    r.w[0] = x.x;
    r.w[1] = x.y;
  } else {
    r.w[0] = *p;
  }
  return r;
}
template <int VW>
__device__ __forceinline__ void stv(uint64_t* p, const V<VW>& v) {
  if constexpr (VW == 2) {
    typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
    u2 x;
    x.x = v.w[0];
    x.y = v.w[1];
    *(u2*)p = x;
  } else {
    *p = v.w[0];
  }
}
template <int VW>
__device__ __forceinline__ V<VW> vzero() {
  V<VW> r;
#pragma unroll
  for (int j = 0; j < VW; ++j) r.w[j] = 0;
  return r;
}

// Wave-uniform copies (SGPRs) of values every lane holds identically: keeps loops over them
// uniform (scalar branches) instead of exec-masked "divergent" loops.
__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int32_t uni32(int32_t x) {
  return (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

struct Ctr {
  Slot32 act2, actw2, fl2, touched;
  Slot64 ef2;  // sum of degrees of the next frontier
  Slot64 eu2;  // sum of degrees of the next active lists
  Slot64 ev2;  // sum of degrees of vertices visited for the first time (by any group)
};
// host view of the interesting fields
struct HostCtr {
  uint32_t act2, actw2, fl2, touched;
  unsigned long long ef2, eu2, ev2;
};

__device__ __forceinline__ bool is_done(const uint32_t* done, int32_t v) {
  return (done[v >> 5] >> (v & 31)) & 1u;
}
__device__ __forceinline__ void set_done(uint32_t* done, int32_t v) {
  atomicOr(&done[v >> 5], 1u << (v & 31));
}
// anyvis: bit v set once vertex v is visited by any group. A clear bit guarantees both visited
// buffers of v are all-zero (bits are set before/with the first non-zero store and never
// cleared within a batch), so pulls may skip the 8*W-byte load; a set bit only costs a load.
__device__ __forceinline__ bool any_visited(const uint32_t* anyvis, int32_t u) {
  return (anyvis[u >> 5] >> (u & 31)) & 1u;
}

// ---- per-group level counters in LDS ------------------------------------------------------------
template <int W, bool COUNT>
struct Lds {
  uint32_t f[64 * W];
  unsigned long long e[COUNT ? 64 * W : 1];
};

template <int W, bool COUNT>
__device__ __forceinline__ void lds_zero(Lds<W, COUNT>& s) {
  for (int i = threadIdx.x; i < 64 * W; i += blockDim.x) {
    s.f[i] = 0;
    if constexpr (COUNT) s.e[i] = 0;
  }
}

template <int W, bool COUNT>
__device__ __forceinline__ void count_bits(Lds<W, COUNT>& s, const V<Lay<W>::VW>& nw, int slot,
                                           uint32_t deg) {
  constexpr int VW = Lay<W>::VW;
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    uint64_t x = nw.w[j];
    const int base = (slot * VW + j) * 64;
    while (x) {
      const int b = __ffsll((unsigned long long)x) - 1;
      x &= x - 1;
      atomicAdd(&s.f[base + b], 1u);
      if constexpr (COUNT) atomicAdd(&s.e[base + b], (unsigned long long)deg);
    }
  }
}

// Per-block counter row -> slab row blockIdx.x (plain stores; no same-address atomics). The
// level's rows are summed by k_level_reduce.
template <int W, bool COUNT>
__device__ __forceinline__ void slab_store(Lds<W, COUNT>& s, uint32_t* slabF,
                                           unsigned long long* slabE) {
  __syncthreads();
  uint32_t* rf = slabF + (size_t)blockIdx.x * (64 * W);
  for (int i = threadIdx.x; i < 64 * W; i += blockDim.x) {
    rf[i] = s.f[i];
    if constexpr (COUNT) slabE[(size_t)blockIdx.x * (64 * W) + i] = s.e[i];
  }
}

// Register-resident bit-sliced (carry-save) counters: bit b of c[j][d] is bit d of the count of
// group (slot*VW + j)*64 + b. Adding a 64-bit new-bits word costs 2*D branch-free ops, vs one
// LDS atomic per set bit in a divergent loop. Spilled to LDS every < 2^D additions.
template <int VW, int DD = 6>
struct BitCounter {
  static constexpr int D = DD;
  uint64_t c[VW][D];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < VW; ++j)
#pragma unroll
      for (int d = 0; d < D; ++d) c[j][d] = 0;
  }
  __device__ __forceinline__ void add(const V<VW>& x) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      uint64_t carry = x.w[j];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const uint64_t t = c[j][d] & carry;
        c[j][d] ^= carry;
        carry = t;
      }
    }
  }
  template <int W, bool COUNT>
  __device__ __forceinline__ void spill(Lds<W, COUNT>& s, int slot) {
    spill(s.f, slot);
  }
  __device__ __forceinline__ void spill(uint32_t* f, int slot) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      uint64_t any = 0;
#pragma unroll
      for (int d = 0; d < D; ++d) any |= c[j][d];
      const int base = (slot * VW + j) * 64;
      while (any) {
        const int b = __ffsll((unsigned long long)any) - 1;
        any &= any - 1;
        uint32_t v = 0;
#pragma unroll
        for (int d = 0; d < D; ++d) v |= (uint32_t)((c[j][d] >> b) & 1ull) << d;
        atomicAdd(&f[base + b], v);
      }
#pragma unroll
      for (int d = 0; d < D; ++d) c[j][d] = 0;
    }
  }
  // Same, into rows of STRIDE words per 64 groups. STRIDE = 65 skews the groups of different
  // lane slots onto different LDS banks: with 64 every lane of the wave hit the bank of bit b
  // (level-3 k_bu_narrow counted ~5e8 bank-conflict cycles; RMAT-26 levels 3 / 4 6.46 / 2.53 ->
  // 6.22 / 2.46 ms with 65). Summing the sub-groups' counts with shuffles before one atomic per
  // slot measured slower (a 64-step wave-uniform bit loop: 27.2 ms/step).
  template <int STRIDE>
  __device__ __forceinline__ void spill_strided(uint32_t* f, int slot) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      uint64_t any = 0;
#pragma unroll
      for (int d = 0; d < D; ++d) any |= c[j][d];
      const int base = (slot * VW + j) * STRIDE;
      while (any) {
        const int b = __ffsll((unsigned long long)any) - 1;
        any &= any - 1;
        uint32_t v = 0;
#pragma unroll
        for (int d = 0; d < D; ++d) v |= (uint32_t)((c[j][d] >> b) & 1ull) << d;
        atomicAdd(&f[base + b], v);
      }
#pragma unroll
      for (int d = 0; d < D; ++d) c[j][d] = 0;
    }
  }
};

// Sum the level's slab rows: block (word, row-group); lane = group bit. F += level * count
// (`level` is the weight: 0 for a level another rank of the hybrid mode accounts for),
// alive_next |= groups with count > 0 (one ballot + one atomicOr per word per row-group).
template <int W, bool COUNT>
__global__ __launch_bounds__(kBlock) void k_level_reduce(const uint32_t* slabF,
                                                         const unsigned long long* slabE, int rows,
                                                         int rgroups, unsigned long long* F,
                                                         unsigned long long* E,
                                                         uint64_t* alive_next, uint32_t level) {
  __shared__ unsigned long long pf[kWaves][64], pe[kWaves][64];
  const int word = blockIdx.x % W, rg = blockIdx.x / W;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const int r0 = (int)((int64_t)rows * rg / rgroups);
  const int r1 = (int)((int64_t)rows * (rg + 1) / rgroups);
  const int i = word * 64 + lane;
  unsigned long long f = 0, e = 0;
  for (int r = r0 + wv; r < r1; r += kWaves) {
    f += slabF[(size_t)r * (64 * W) + i];
    if constexpr (COUNT) e += slabE[(size_t)r * (64 * W) + i];
  }
  pf[wv][lane] = f;
  pe[wv][lane] = e;
  __syncthreads();
  if (wv == 0) {
    for (int w = 1; w < kWaves; ++w) {
      f += pf[w][lane];
      e += pe[w][lane];
    }
    if (f) atomicAdd(&F[i], f * level);
    if constexpr (COUNT) {
      if (e) atomicAdd(&E[i], e);
    }
    const uint64_t m = __ballot(f != 0);
    if (lane == 0 && m) atomicOr((unsigned long long*)&alive_next[word], m);
  }
}

// k_level_reduce over the slab rows of nlev consecutive levels (`rows` rows each, level j's rows
// first-level-major) of the device-driven batches: F += sum_j weight(level_first + j) * count_j;
// alive_next + 16 * j = the groups with new vertices at level j (the mask after it). One launch
// per few levels (a launch costs ~5 us, a road-like graph's level 15-200 us); the levels in
// between read an older alive mask, a superset, which only lets them mark fewer vertices done.
template <int W>
__global__ __launch_bounds__(kBlock) void k_level_reduce_multi(const uint32_t* slabF, int rows,
                                                               int nlev, int rgroups,
                                                               uint32_t level_first, int weight_l1,
                                                               unsigned long long* F,
                                                               uint64_t* alive_next) {
  __shared__ uint32_t pl[kWaves][64];
  const int word = blockIdx.x % W, rg = blockIdx.x / W;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const int r0 = (int)((int64_t)rows * rg / rgroups);
  const int r1 = (int)((int64_t)rows * (rg + 1) / rgroups);
  const int i = word * 64 + lane;
  unsigned long long fw = 0;
  for (int j = 0; j < nlev; ++j) {
    uint32_t f = 0;
    for (int r = r0 + wv; r < r1; r += kWaves) f += slabF[((size_t)j * rows + r) * (64 * W) + i];
    pl[wv][lane] = f;
    __syncthreads();
    if (wv == 0) {
      for (int w = 1; w < kWaves; ++w) f += pl[w][lane];
      const uint32_t lvl = level_first + (uint32_t)j;
      fw += (unsigned long long)f * ((lvl == 1 && !weight_l1) ? 0u : lvl);
      const uint64_t m = __ballot(f != 0);
      if (lane == 0 && m) atomicOr((unsigned long long*)&alive_next[16 * j + word], m);
    }
    __syncthreads();
  }
  if (wv == 0 && fw) atomicAdd(&F[i], fw);
}

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

// ---------------------------------------------------------------------------------------------
// top-down expand: edge-parallel over the frontier (load-balanced search on offs = inclusive
// degree prefix). DIFF=true: frontier bits = visCur & ~visOld (frontier came from bottom-up);
// DIFF=false: frontier bits are in accCur (frontier came from top-down / init).
// ---------------------------------------------------------------------------------------------
template <int W, bool DIFF>
__global__ __launch_bounds__(kBlock) void k_td_expand(
    const int32_t* fl, int64_t nf, const int64_t* offs, const int64_t* rowptr, const int32_t* col,
    const uint64_t* visCur, const uint64_t* fsrc, const uint32_t* done, uint64_t* accNext,
    int32_t* stamp, int32_t epoch, int32_t* touched, Ctr* ctr, const uint32_t* lzv = nullptr,
    const uint32_t* osnap = nullptr) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  __shared__ LdsQueue q;
  q_init(q);
  __syncthreads();
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  const int64_t total = offs[nf - 1];
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < total; tb += (int64_t)gridDim.x * TILE) {
    const int64_t e = tb + wv * VPW + sub;
    bool touch = false;
    int32_t v = 0;
    if (e < total) {
      const int64_t i = upper_bound_i64(offs, nf, e);
      const int32_t u = fl[i];
      const int64_t start = i ? offs[i - 1] : 0;
      v = col[rowptr[u] + (e - start)];
      if (!is_done(done, v)) {
        const int64_t uo = (int64_t)u * W + slot * VW, vo = (int64_t)v * W + slot * VW;
        V<VW> fb = ldv<VW>(visCur + uo);
        if constexpr (DIFF) {
          // osnap: the old row of a vertex first visited at the previous (first, unfilled) pull
          // level was never written: it is all zero (see start_batch)
          const V<VW> old =
              (osnap && !any_visited(osnap, u)) ? vzero<VW>() : ldv<VW>(fsrc + uo);
#pragma unroll
          for (int j = 0; j < VW; ++j) fb.w[j] &= ~old.w[j];
        } else {
          fb = ldv<VW>(fsrc + uo);
        }
        // lzv: rows of never-visited vertices may be stale (lazy reset, see k_zero_part_rows)
        const V<VW> r = (lzv && !any_visited(lzv, v)) ? vzero<VW>() : ldv<VW>(visCur + vo);
        bool any = false, first = false;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const uint64_t mm = fb.w[j] & ~r.w[j];
          if (mm) {
            first |= atomicOr((unsigned long long*)&accNext[vo + j], mm) == 0ull;
            any = true;
          }
        }
        if constexpr (W == 1) {
          touch = first;  // (see k_td_expand_small)
        } else {
          // one lane per group decides the first touch of v in this level (the group shares v)
          const uint64_t gm = (__ballot(any) >> (sub * G)) & L::GBITS;
          if (gm && slot == 0) touch = atomicExch(&stamp[v], epoch) != epoch;
        }
      }
    }
    q_push(q, touch, v);
    q_flush(q, touched, &ctr->touched.v, TILE, false);
  }
  q_flush(q, touched, &ctr->touched.v, 0, true);
}

// top-down expand for low-degree frontiers (road-like graphs: a few edges per vertex, thousands
// of levels): G lanes per frontier vertex walk its row edge by edge. No degree prefix scan and no
// per-edge binary search (k_td_expand's load balancing costs more than it saves when every
// vertex has ~2-4 edges).
// nf_dev (device-driven level batches): the frontier size written by the previous level's
// finalize, read here instead of the host's nf_arg.
template <int W, bool DIFF>
__global__ __launch_bounds__(kBlock) void k_td_expand_small(
    const int32_t* fl, int64_t nf_arg, const uint32_t* nf_dev, const int64_t* rowptr,
    const int32_t* col, const uint64_t* visCur, const uint64_t* fsrc, const uint32_t* done,
    uint64_t* accNext, int32_t* stamp, int32_t epoch, int32_t* touched, Ctr* ctr,
    const uint32_t* lzv = nullptr, const uint32_t* osnap = nullptr, Ctr* cstop = nullptr,
    unsigned long long ef_stop = 0) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  // device-driven batch: stop where the host would pull (cstop = the slot of this level's
  // frontier, whose degree sum the previous finalize wrote; see k_td_fused)
  if (cstop && cstop->fl2.v > 0 && cstop->ef2.v > ef_stop) {
    if (blockIdx.x == 0 && threadIdx.x == 0) cstop->act2.v = 1u;
    return;
  }
  __shared__ LdsQueue q;
  q_init(q);
  __syncthreads();
  const int64_t nf = nf_dev ? (int64_t)*nf_dev : nf_arg;
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nf; tb += (int64_t)gridDim.x * TILE) {
    const int64_t idx = tb + wv * VPW + sub;
    int64_t e = 0, end = 0;
    V<VW> fb = vzero<VW>();
    if (idx < nf) {
      const int32_t u = fl[idx];
      e = rowptr[u];
      end = rowptr[u + 1];
      const int64_t uo = (int64_t)u * W + slot * VW;
      if constexpr (DIFF) {
        fb = ldv<VW>(visCur + uo);
        const V<VW> old =
            (osnap && !any_visited(osnap, u)) ? vzero<VW>() : ldv<VW>(fsrc + uo);  // see k_td_expand
#pragma unroll
        for (int j = 0; j < VW; ++j) fb.w[j] &= ~old.w[j];
      } else {
        fb = ldv<VW>(fsrc + uo);
      }
    }
    // one edge per step for every vertex of the block (block-uniform steps, so the queue can
    // flush every step; used only on graphs whose maximum degree is small)
    while (__syncthreads_or(e < end)) {
      bool touch = false;
      int32_t v = 0;
      if (e < end) {
        v = col[e];
        if (!is_done(done, v)) {
          const int64_t vo = (int64_t)v * W + slot * VW;
          const V<VW> r = (lzv && !any_visited(lzv, v)) ? vzero<VW>() : ldv<VW>(visCur + vo);
          bool any = false, first = false;
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const uint64_t mm = fb.w[j] & ~r.w[j];
            if (mm) {
              first |= atomicOr((unsigned long long*)&accNext[vo + j], mm) == 0ull;
              any = true;
            }
          }
          if constexpr (W == 1) {
            // one word per vertex: the accumulator is all zero at the level start, so the push
            // that finds it empty is v's first touch (no second atomic on the stamp)
            touch = first;
          } else {
            const uint64_t gm = (__ballot(any) >> (sub * G)) & L::GBITS;
            if (gm && slot == 0) touch = atomicExch(&stamp[v], epoch) != epoch;
          }
        }
        ++e;
      }
      q_push(q, touch, v);
      q_flush(q, touched, &ctr->touched.v, TILE, false);
    }
  }
  q_flush(q, touched, &ctr->touched.v, 0, true);
}

// device-driven level batch: seed slot 0 with the current frontier size and alive mask
__global__ void k_batch_seed(Ctr* c0, uint32_t nf, unsigned long long ef, const uint64_t* alive,
                             uint64_t* alive0) {
  if (threadIdx.x == 0) {
    c0->fl2.v = nf;
    c0->ef2.v = ef;
  }
  if (threadIdx.x < 16) alive0[threadIdx.x] = alive[threadIdx.x];
}

// top-down finalize: new = acc & ~vis; update both visited buffers; build the next frontier.
// FUSE: the level's new-bit counts go straight to this block's counter-slab row (as in the
// bottom-up kernels) instead of a k_count_frontier pass over the new frontier.
template <int W, bool COUNT, bool FUSE>
__global__ __launch_bounds__(kBlock) void k_td_finalize(
    const int32_t* touched, const int64_t* rowptr, uint64_t* visCur, uint64_t* visOld,
    uint64_t* accNext, const uint64_t* alive, const uint64_t* gmask, uint32_t* done, int32_t* fl2,
    Ctr* ctr, const int32_t* fl_old, int64_t nf_old_arg, const uint32_t* nfold_dev,
    uint64_t* accCur_zero, uint32_t* anyvis, uint32_t* slabF, int lazy, const uint32_t* stop) {
  static_assert(!(FUSE && COUNT), "the edge-counting pass uses k_count_frontier");
  if (stop && *stop) {  // the batch stopped at this level (k_td_expand_small)
    if constexpr (FUSE)
      for (int i = threadIdx.x; i < 64 * W; i += kBlock) slabF[(size_t)blockIdx.x * 64 * W + i] = 0u;
    return;
  }
  const int64_t nf_old = nfold_dev ? (int64_t)*nfold_dev : nf_old_arg;
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  __shared__ LdsQueue q;
  __shared__ unsigned long long scratch[kWaves];
  constexpr int CR = 65;  // bank-skewed counter rows (see BitCounter::spill_strided)
  __shared__ uint32_t cnt[FUSE ? CR * W : 1];
  if constexpr (FUSE)
    for (int i = threadIdx.x; i < CR * W; i += kBlock) cnt[i] = 0;
  q_init(q);
  __syncthreads();
  BitCounter<VW> bc;
  int nadd = 0;
  if constexpr (FUSE) bc.zero();
  const int64_t nt = ctr->touched.v;  // written by k_td_expand (previous kernel on the stream)
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  V<VW> am, gm;
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    am.w[j] = alive[slot * VW + j];
    gm.w[j] = gmask[slot * VW + j];
  }
  unsigned long long ef = 0, ev = 0;
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nt; tb += (int64_t)gridDim.x * TILE) {
    const int64_t idx = tb + wv * VPW + sub;
    const bool valid = idx < nt;
    int32_t v = 0;
    bool anynew = false, notfull = false, rnz = false;
    V<VW> nw = vzero<VW>();
    uint32_t deg = 0;
    if (valid) {
      v = touched[idx];
      const int64_t vo = (int64_t)v * W + slot * VW;
      const V<VW> a = ldv<VW>(accNext + vo);
      // lazy: a vertex no group has visited yet may have a stale row (see k_zero_part_rows)
      const V<VW> r = (lazy && !any_visited(anyvis, v)) ? vzero<VW>() : ldv<VW>(visCur + vo);
      V<VW> nv;
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        nw.w[j] = a.w[j] & ~r.w[j];
        nv.w[j] = r.w[j] | nw.w[j];
        anynew |= nw.w[j] != 0;
        notfull |= (~nv.w[j] & am.w[j] & gm.w[j]) != 0;
        rnz |= r.w[j] != 0;
      }
      stv<VW>(accNext + vo, nw);
      stv<VW>(visCur + vo, nv);
      stv<VW>(visOld + vo, nv);
      deg = (uint32_t)(rowptr[v + 1] - rowptr[v]);
    }
    if constexpr (FUSE) {  // nw is zero for invalid lanes
      bc.add(nw);
      if (++nadd == (1 << BitCounter<VW>::D) - 1) {
        bc.template spill_strided<CR>(cnt, slot);
        nadd = 0;
      }
    }
    const uint64_t bn = __ballot(anynew), bf = __ballot(notfull), br = __ballot(rnz);
    const bool g_new = (bn >> (sub * G)) & L::GBITS;
    const bool g_full = !((bf >> (sub * G)) & L::GBITS);
    const bool g_first = g_new && !((br >> (sub * G)) & L::GBITS);
    const bool leader = valid && slot == 0;
    if (leader && g_full) set_done(done, v);
    const bool app = leader && g_new;
    if (app) ef += deg;
    if (leader && g_first) {
      atomicOr(&anyvis[v >> 5], 1u << (v & 31));
      ev += deg;
    }
    q_push(q, app, v);
    q_flush(q, fl2, &ctr->fl2.v, TILE, false);
  }
  q_flush(q, fl2, &ctr->fl2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  if constexpr (FUSE) {
    bc.template spill_strided<CR>(cnt, slot);
    __syncthreads();
    uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
    for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = cnt[i + (i >> 6)];
  }
  // zero the consumed top-down frontier bits of the previous frontier
  if (accCur_zero) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t b = wave * VPW; b < nf_old; b += nwaves * VPW) {
      const int64_t idx = b + sub;
      if (idx < nf_old) stv<VW>(accCur_zero + (int64_t)fl_old[idx] * W + slot * VW, vzero<VW>());
    }
  }
}

// One-kernel top-down level for low-degree graphs (device-driven batches, td_batch; road-like
// graphs run thousands of levels of up to a few million frontier vertices, where the expand +
// finalize pair spent ~115 us per level, much of it on chains of dependent loads).
// The visited row itself is the claim: atomicOr(vis[v], frontier bits) returns the bits other
// pushers already set, so every (vertex, group) bit is counted exactly once, by the push that
// set it; the new bits go to accNext (the next frontier's bits) and the push that finds accNext
// empty (W = 1) or wins the stamp (W > 1) appends v to the next frontier. No touched list and
// no second pass; only vis[cur] is updated (the caller marks the other buffer stale, see
// Loop::old_stale). Each lane walks U edges of its vertex per step with all loads issued
// before the atomics. Requires fully valid rows of vis[cur] (no lazy batch) and frontier bits
// in accCur, which the lane that reads them clears (accCur is the level-after-next's accNext).
// The next frontier is written twice: as a list (flNext, its size is the next level's nf) and
// as a bitmap (fbmNext). Levels with at least bm_min frontier vertices walk the bitmap instead
// of the list: blocks expand the set bits of 256 consecutive words (8192 ids) in id order, so
// the rows, row offsets and neighbour rows a block touches are contiguous runs (a grid graph's
// neighbours are v +- 1 and v +- width) instead of the list's arrival order. The level consumes
// (zeroes) fbmCur either way. Frontier degree sums: level i adds its own frontier's (from the
// row offsets it loads anyway) to the previous slot's ef (own: that slot's frontier was written
// by a fused level); only the batch's last level (tail) sums the degrees of what it appends.
// Road grid 4896^2, 64 groups (MI355X): expand + finalize 562 ms; one kernel 371 ms; + bitmap
// walk 334 ms; + both atomics in flight, deferred degree sums, one reduction per 6 levels 319 ms.
template <int W>
__global__ __launch_bounds__(kBlock) void k_td_fused(
    const int32_t* fl, const uint32_t* nf_dev, int64_t bm_min, uint32_t* fbmCur,
    uint32_t* fbmNext, int64_t nwords, const int64_t* rowptr, const int32_t* col, uint64_t* vis,
    uint64_t* accCur, uint64_t* accNext, const uint64_t* alive, const uint64_t* gmask,
    uint32_t* done, uint32_t* anyvis, int32_t* stamp, int32_t epoch, int32_t* flNext, Ctr* ctr,
    uint32_t* slabF, Ctr* cprev, int own, int tail, const Ctr* cpp,
    unsigned long long ef_stop) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  constexpr int U = 4;
  constexpr int QC = 2 * kQCap;
  static_assert(TILE * U <= QC / 2, "queue room for one step");
  __shared__ LdsQueueN<QC> q;
  __shared__ unsigned long long scratch[kWaves];
  constexpr int CR = 65;  // bank-skewed counter rows (see BitCounter::spill_strided)
  __shared__ uint32_t cnt[CR * W];
  // bitmap mode: words per tile (8192 ids; 4096-id tiles measured 6 % slower on the road grid)
  constexpr int BW = kBlock;
  __shared__ uint16_t lst[BW * 32];  // bitmap mode: set bits of the tile's words
  __shared__ uint32_t wsum[kWaves];
  for (int i = threadIdx.x; i < CR * W; i += kBlock) cnt[i] = 0;
  q_init(q);
  __syncthreads();
  BitCounter<VW> bc;
  bc.zero();
  int nadd = 0;
  const int64_t nf = (int64_t)*nf_dev;
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  V<VW> amg;
#pragma unroll
  for (int j = 0; j < VW; ++j) amg.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  unsigned long long ef = 0, ev = 0, ef_own = 0;
  // direction check inside the batch (the host's test, on this frontier's degree sum estimated
  // from its size and the previous frontier's mean degree): a level the host would run as a pull
  // does nothing but record its frontier's degree sum and the stop; every later
  // level of the batch then sees an empty frontier, and the host resumes from this level
  // (cprev->act2 = 1)
  if (cpp && nf > 0 && cpp->fl2.v > 0 &&
      (double)nf * ((double)cpp->ef2.v / (double)cpp->fl2.v) > (double)ef_stop) {
    if (own) {
      for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nf;
           i += (int64_t)gridDim.x * kBlock) {
        const int32_t u = fl[i];
        ef_own += (unsigned long long)(rowptr[u + 1] - rowptr[u]);
      }
      block_sum_add(ef_own, &cprev->ef2.v, scratch);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) cprev->act2.v = 1u;  // (unused by top-down levels)
    uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
    for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = 0u;
    return;
  }

  // expand frontier vertex u (has) of this lane's row group; block-uniform call
  auto expand = [&](bool has, int32_t u) {
    int64_t e = 0, end = 0;
    V<VW> fb = vzero<VW>();
    if (has) {
      e = rowptr[u];
      end = rowptr[u + 1];
      if (slot == 0) ef_own += (unsigned long long)(end - e);
      const int64_t uo = (int64_t)u * W + slot * VW;
      fb = ldv<VW>(accCur + uo);
      stv<VW>(accCur + uo, vzero<VW>());
    }
    while (__syncthreads_or(e < end)) {
      int32_t v[U];
      uint32_t dw[U];
      V<VW> r[U];
#pragma unroll
      for (int j = 0; j < U; ++j) v[j] = e + j < end ? col[e + j] : -1;
#pragma unroll
      for (int j = 0; j < U; ++j) {
        dw[j] = ~0u;
        r[j] = vzero<VW>();
        if (v[j] >= 0) {
          dw[j] = done[v[j] >> 5];
          r[j] = ldv<VW>(vis + (int64_t)v[j] * W + slot * VW);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int32_t x = v[j];
        V<VW> nw = vzero<VW>();
        bool push = false, first = false, full = true, was0 = true;
        if (x >= 0 && !((dw[j] >> (x & 31)) & 1u)) {
          const int64_t xo = (int64_t)x * W + slot * VW;
#pragma unroll
          for (int k = 0; k < VW; ++k) {
            const uint64_t mm = fb.w[k] & ~r[j].w[k];
            uint64_t now = r[j].w[k];
            if (mm) {
              // both atomics in flight together: accNext may take a bit a concurrent push
              // claimed in vis first (that push adds it too: same union); the vis return
              // decides which push counts it
              const uint64_t ov = atomicOr((unsigned long long*)&vis[xo + k], mm);
              const uint64_t oa = atomicOr((unsigned long long*)&accNext[xo + k], mm);
              nw.w[k] = mm & ~ov;
              now = ov | mm;
              first |= oa == 0ull;
              was0 &= ov == 0ull;
              push = true;
            }
            full &= (~now & amg.w[k]) == 0;
          }
        }
        // one lane per row group decides for the vertex (the G lanes share x)
        const uint64_t bg = __ballot(push), bn = __ballot(!full);
        const bool g_push = (bg >> (sub * G)) & L::GBITS;
        const bool g_full = !((bn >> (sub * G)) & L::GBITS);
        const bool leader = slot == 0 && g_push;
        bool app = false, fresh = false;
        if (leader) {
          const uint32_t bit = 1u << (x & 31);
          if constexpr (W == 1) {
            app = first;  // accNext was empty: v's first touch this level
            // the whole row was empty (vis is cleared per batch): first visit by any group
            fresh = was0;
            if (fresh) atomicOr(&anyvis[x >> 5], bit);
          } else {
            app = atomicExch(&stamp[x], epoch) != epoch;
            if (!any_visited(anyvis, x)) fresh = !(atomicOr(&anyvis[x >> 5], bit) & bit);
          }
          if (g_full) set_done(done, x);
          if (app) atomicOr(&fbmNext[x >> 5], bit);
          // the next frontier's degree sum is taken by the next level from the row offsets it
          // loads anyway (ef_own), except after the batch's last level
          if ((app && tail) || fresh) {
            const unsigned long long deg = (unsigned long long)(rowptr[x + 1] - rowptr[x]);
            if (app && tail) ef += deg;
            if (fresh) ev += deg;
          }
        }
        bc.add(nw);
        if (++nadd == (1 << BitCounter<VW>::D) - 1) {
          bc.template spill_strided<CR>(cnt, slot);
          nadd = 0;
        }
        q_push(q, app, x);
      }
      q_flush(q, flNext, &ctr->fl2.v, TILE * U, false);
      e += U;
    }
  };

  if (nf < bm_min) {
    for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nf; tb += (int64_t)gridDim.x * TILE) {
      const int64_t idx = tb + wv * VPW + sub;
      const bool has = idx < nf;
      const int32_t u = has ? fl[idx] : 0;
      if (has && slot == 0) fbmCur[u >> 5] = 0u;  // (every bit of the word is in this list)
      expand(has, u);
    }
  } else {
    for (int64_t wb = (int64_t)blockIdx.x * BW; wb < nwords; wb += (int64_t)gridDim.x * BW) {
      const int64_t wi = wb + threadIdx.x;
      const uint32_t w = (threadIdx.x < BW && wi < nwords) ? fbmCur[wi] : 0u;
      if (!__syncthreads_or(w != 0u)) continue;
      if (w) fbmCur[wi] = 0u;
      // block exclusive scan of the words' popcounts -> positions in lst
      const uint32_t c = (uint32_t)__popc(w);
      uint32_t incl = c;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
      }
      if (lane == 63) wsum[wv] = incl;
      __syncthreads();
      uint32_t base = 0, total = 0;
#pragma unroll
      for (int k = 0; k < kWaves; ++k) {
        base += k < wv ? wsum[k] : 0u;
        total += wsum[k];
      }
      uint32_t pos = base + incl - c;
      for (uint32_t x = w; x; x &= x - 1)
        lst[pos++] = (uint16_t)((threadIdx.x << 5) + (__ffs(x) - 1));
      __syncthreads();
      for (uint32_t c0 = 0; c0 < total; c0 += TILE) {
        const uint32_t idx = c0 + wv * VPW + sub;
        const bool has = idx < total;
        expand(has, has ? (int32_t)(wb * 32 + lst[idx]) : 0);
      }
      __syncthreads();  // lst / wsum reused by the next tile
    }
  }
  q_flush(q, flNext, &ctr->fl2.v, 0, true);
  if (tail) block_sum_add(ef, &ctr->ef2.v, scratch);
  if (own) block_sum_add(ef_own, &cprev->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  bc.template spill_strided<CR>(cnt, slot);
  __syncthreads();
  uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
  for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = cnt[i + (i >> 6)];
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

// build the bottom-up active lists (deg > 0, not done) over the vertices v = part + i*nparts,
// i < cnt, split by degree (nparts = 1: every vertex; the hybrid mode's vertex-partitioned
// level pulls only for its own residue class)
template <int QCAP>
__global__ __launch_bounds__(kBlock) void k_build_active(int64_t cnt, int part, int nparts,
                                                         const int64_t* rowptr,
                                                         const uint32_t* done, int wide_deg,
                                                         int32_t* act, int32_t* actw, Ctr* ctr) {
  // Each block owns QCAP consecutive list positions j and flushes its narrow queue once at the
  // end (one counter atomic per QCAP vertices: atomics on one address serialise, and 64K of them
  // were most of this kernel's time on 33M vertices). Blocks are dispatched in order, so the
  // lists come out nearly ascending (hubs first in the wide list: the chunk kernel deals chunks
  // in list order, and a grid-stride build that interleaved distant ranges cost ~1 ms of level-2
  // tail on RMAT-26). The rare wide vertices go through a small queue flushed when needed.
  constexpr int VPT = 4;  // vertices per thread per step (loads first, pushes after)
  constexpr int64_t kStep = (int64_t)VPT * kBlock;
  static_assert(QCAP % kStep == 0, "whole steps per block");
  __shared__ LdsQueueN<QCAP> qn;
  __shared__ LdsQueue qw;
  __shared__ unsigned long long scratch[kWaves];
  q_init(qn);
  q_init(qw);
  __syncthreads();
  unsigned long long eu = 0;
  const int64_t b0 = (int64_t)blockIdx.x * QCAP, b1 = min(b0 + (int64_t)QCAP, cnt);
  for (int64_t b = b0; b < b1; b += kStep) {
    int64_t d[VPT];
    uint32_t dw[VPT];
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int64_t j = b + q * kBlock + threadIdx.x;
      const int64_t i = part + j * nparts;
      d[q] = 0;
      dw[q] = ~0u;
      if (j < b1) {
        d[q] = rowptr[i + 1] - rowptr[i];
        dw[q] = done[i >> 5];
      }
    }
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int64_t i = part + (b + q * kBlock + threadIdx.x) * nparts;
      const bool ok = d[q] > 0 && !((dw[q] >> (i & 31)) & 1u);
      if (ok) eu += (unsigned long long)d[q];
      q_push(qn, ok && d[q] <= wide_deg, (int32_t)i);
      q_push(qw, ok && d[q] > wide_deg, (int32_t)i);
    }
    q_flush(qw, actw, &ctr->actw2.v, (int)kStep, false);
  }
  q_flush(qn, act, &ctr->act2.v, 0, true);
  q_flush(qw, actw, &ctr->actw2.v, 0, true);
  block_sum_add(eu, &ctr->eu2.v, scratch);
}

// ---------------------------------------------------------------------------------------------
// Sparse row codes for the first bottom-up level. Its frontier is the level-1 frontier: outside
// the top hubs a vertex there was reached from one or two sources, so its visited row (8*W bytes)
// mostly holds a single set bit (RMAT-26, 1024 groups: ~1.2 bits per row below degree ~9K).
// Gathering those rows made the level bound by Infinity-Cache traffic (rocprofv3, k_bu_chunks at
// level 2: 44 % L2 hit rate, ~115 GB of L2 misses for 0.74e9 row gathers). code[u] (32 bit):
// 0 = row empty; else bits 30-31 = number of set groups c (1-3) and bits 10*i .. 10*i+9 their
// ids (groups < 1024); kDenseCode = anything else (gathered as before). Several slots: the
// multi-bit rows of the mid-degree ids (RMAT-26: degree 1K-8K, 1-2 expected bits) were most of
// the level's L2 misses (the dense rows left did not fit one XCD's 4 MB L2 next to the top hubs'
// rows; single-slot codes 7.5 ms for the level's chunk pulls, two slots 6.9 ms). The
// frontier's codes occupy a 64x smaller footprint than its rows, so the pulls mostly hit L2.
// Only ids >= code_from use codes: after degree relabelling the lower ids are the hubs, whose rows
// are dense and L2-resident. The codes live in the top-down touched buffer (unused by bottom-up
// levels, rebuilt by every top-down level).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kDenseCode = 0xFFFFFFFFu;  // (3 slots of group 1023: never a real code)
constexpr int kCodeSlots = 3;
// group of slot i of a sparse code, -1 for an unused slot
__device__ __forceinline__ int code_g(uint32_t c, int i) {
  return i < (int)(c >> 30) ? (int)((c >> (10 * i)) & 1023u) : -1;
}
constexpr int32_t kNoCodes = INT32_MAX;

template <int W>
// ids [lo, hi), then the list entries fl[0..nl) >= hi
__global__ __launch_bounds__(kBlock) void k_build_codes(const uint64_t* R, const uint32_t* anyvis,
                                                        int64_t lo, int64_t hi, const int32_t* fl,
                                                        int64_t nl, uint32_t* code) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < hi - lo + nl;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t u = i < hi - lo ? lo + i : (int64_t)fl[i - (hi - lo)];
    if (i >= hi - lo && u < hi) continue;
    uint32_t c = 0;
    if (any_visited(anyvis, (int32_t)u)) {
      int pc = 0;
#pragma unroll
      for (int j = 0; j < W; ++j) {
        uint64_t w = R[u * W + j];
        const int pw = __popcll(w);
        if (pc + pw <= kCodeSlots) {  // (dense hub rows skip the bit loop)
          while (w) {
            const int b = __ffsll((unsigned long long)w) - 1;
            w &= w - 1;
            c |= (uint32_t)(j * 64 + b) << (10 * pc);
            ++pc;
          }
        } else {
          pc += pw;
        }
      }
      c = pc == 0 ? 0u : pc <= kCodeSlots ? c | ((uint32_t)pc << 30) : kDenseCode;
    }
    code[u] = c;
  }
}

// first id with degree < min_deg (rows relabelled by descending degree; one thread)
__global__ void k_degree_bound(const int64_t* rowptr, int64_t n, int64_t min_deg, int32_t* out) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid + 1] - rowptr[mid] < min_deg) hi = mid;
    else lo = mid + 1;
  }
  *out = (int32_t)lo;
}


// ---------------------------------------------------------------------------------------------
// Prefix pull + tail push for the first bottom-up level (rows sorted by id, degree relabelled).
// The LDS hub bitmap covers the ids < H; a pull that scanned whole rows had to probe the global
// visited bitmap for every neighbour id >= H (the degree tail: ~40 % of the edge endpoints on
// RMAT-26, almost none of them in the level-1 frontier). Instead the pulls stop at the first id
// >= H, and the few level-1 frontier vertices u >= H push their bits to their neighbours here:
// acc[v] |= row(u) (atomicOr, mostly one word thanks to the sparse codes) and stamp[v] = epoch.
// The narrow pull folds acc[v] of stamped vertices into its accumulator (and clears it); wide
// vertices collect it with their chunk results in k_bu_wide_finalize. Sources need no push:
// every neighbour of a source was reached at level 1. Only own vertices (v % nparts == part) are
// targets (the hybrid mode's level 2 pulls only those), and done vertices are skipped, so every
// written acc entry is consumed and cleared within the level.
// ---------------------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(kBlock) void k_push_tail(
    const int32_t* fl, int64_t nf, int32_t H, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, const uint32_t* code, int32_t code_from, const uint32_t* done,
    int part, int nparts, uint64_t* acc, int32_t* stamp, int32_t epoch) {
  // 16 lanes per frontier entry, 4 entries per wave in flight (tail vertices have tens to a few
  // hundred neighbours; the lanes of an entry take consecutive row entries)
  constexpr int PG = 64;
  const int lane = lane_id(), slot = lane % PG;
  const int64_t grp = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / PG;
  const int64_t ngrp = ((int64_t)gridDim.x * kBlock) / PG;
  for (int64_t i = grp; i < nf; i += ngrp) {
    const int32_t u = fl[i];
    if (u < H) continue;
    const uint32_t c = (code && u >= code_from) ? code[u] : kDenseCode;
    if (c == 0) continue;
    const int64_t b = rowptr[u], e = rowptr[u + 1];
    for (int64_t k = b + slot; k < e; k += PG) {
      const int32_t v = col[k];
      if (nparts > 1 && v % nparts != part) continue;
      if (is_done(done, v)) continue;
      if (c != kDenseCode) {
        for (int i = 0; i < kCodeSlots; ++i) {
          const int g = code_g(c, i);
          if (g >= 0) atomicOr((unsigned long long*)&acc[(int64_t)v * W + (g >> 6)], 1ull << (g & 63));
        }
      } else {
        for (int j = 0; j < W; ++j) {
          const uint64_t w = R[(int64_t)u * W + j];
          if (w) atomicOr((unsigned long long*)&acc[(int64_t)v * W + j], (unsigned long long)w);
        }
      }
      stamp[v] = epoch;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// bottom-up, narrow vertices: G lanes per vertex, early exit when every alive group is covered.
// Each step takes C = 8 neighbours: the group's G lanes load and filter them cooperatively
// (8/G column ids + 8/G bitmap probes per lane instead of 8 + 8), then every lane pulls its
// slot of each surviving neighbour's row (ids broadcast inside the group by shuffles).
// BT = block size; HUBW > 0: probes of the HUBW*32 lowest ids (hubs) read an LDS snapshot of
// the visited bitmap (see k_bu_chunks; big blocks amortise the copy).
// ---------------------------------------------------------------------------------------------
//
// FUSE: the level's new-bit counts are accumulated here (register bit-sliced counters -> LDS ->
// this block's row of the counter slab, slabF = first row of this launch) instead of by a
// separate k_count_frontier pass that re-reads both rows of every new frontier vertex.
// PFX (prefix-pull level, see k_push_tail): rows are scanned only up to the first id >= HUBW*32,
// and pushed bits (acc of vertices with stamp == epoch) seed the accumulator.
// CS = neighbours per step (rows gathered between two coverage checks).
// C1 > 0 (unfiltered levels only): a first step of just C1 rows before the CS-wide steps; late
// levels are mostly covered by the first neighbour or two (sorted rows: hubs first).
template <int W, bool COUNT, int BT, int HUBW, bool FUSE, bool FILT = true, bool PFX = false,
          int CS = 8, int C1 = 0, int MINW = 4>
__global__ __launch_bounds__(BT, MINW) void k_bu_narrow(
    const int32_t* act, int64_t nact, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, uint64_t* Wb, const uint64_t* alive, const uint64_t* gmask, uint32_t* done,
    int32_t* act2, int32_t* fl2, Ctr* ctr, uint32_t* anyvis, int32_t filter_from, int32_t* actw2,
    int next_wide, uint32_t* slabF, uint64_t* pacc, const int32_t* stamp, int32_t epoch,
    const int32_t* plen, const uint32_t* nact_dev, const uint32_t* snap) {
  static_assert(!PFX || HUBW > 0, "the prefix pull relies on the LDS hub bitmap");
  // snap (first pull level of a batch that did not clear its visited buffer, see start_batch):
  // the any-visited bitmap as of the level start. Probes read it (a vertex first visited during
  // this level may still have a stale row) and an own row it does not mark is all zero.
  const uint32_t* pvis = snap ? snap : anyvis;
  if (nact_dev) nact = (int64_t)*nact_dev;  // (list length known only on the device)
  static_assert(!(FUSE && COUNT), "the edge-counting pass uses k_count_frontier");
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW;
  constexpr int NWV = BT / 64, TILE = NWV * VPW;
  constexpr int C = CS;                      // neighbours per step
  constexpr int Q = C / G > 0 ? C / G : 1;   // ids loaded per lane per step
  static_assert(G * Q == C || (C < G && Q == 1), "step = whole lane groups or part of one");
  __shared__ LdsQueue qa, qf, qw;
  __shared__ unsigned long long scratch[NWV];
  __shared__ uint32_t hub[HUBW > 0 ? HUBW : 1];
  // counter rows of CR words per 64 groups, bank-skewed (see BitCounter::spill_strided) except
  // on the prefix level: its sparse spills ran level 2 ~0.2 ms slower skewed (4 runs each)
  constexpr int CR = PFX ? 64 : 65;
  __shared__ uint32_t cnt[FUSE ? CR * W : 1];
  if constexpr (HUBW > 0)
    for (int i = threadIdx.x; i < HUBW; i += BT) hub[i] = pvis[i];
  if constexpr (FUSE)
    for (int i = threadIdx.x; i < CR * W; i += BT) cnt[i] = 0;
  q_init(qa);
  q_init(qf);
  q_init(qw);
  __syncthreads();
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  unsigned long long eu = 0, ef = 0, ev = 0;
  BitCounter<VW, PFX ? 5 : 6> bc;
  int nadd = 0;
  if constexpr (FUSE) bc.zero();
  // Software pipeline over the grid-stride tiles: the active-list entry is loaded two tiles
  // ahead and the vertex's visited row and row offsets one tile ahead, so a tile starts with
  // its column loads instead of two dependent round trips (list entry -> row / offsets).
  const int64_t stride = (int64_t)gridDim.x * TILE, lofs = wv * VPW + sub;
  int64_t tb = (int64_t)blockIdx.x * TILE;
  int32_t v1 = 0, v2 = 0;  // list entries of tiles tb and tb + stride
  V<VW> r1 = vzero<VW>();  // row of v1
  int64_t b1 = 0;          // row offsets of v1
  uint32_t d1 = 0;
  if (tb + lofs < nact) v1 = act[tb + lofs];
  if (tb + stride + lofs < nact) v2 = act[tb + stride + lofs];
  uint32_t p1 = 0;  // PFX: prefix length of v1's row (ids < H)
  if (tb + lofs < nact) {
    r1 = (snap && !any_visited(snap, v1)) ? vzero<VW>() : ldv<VW>(R + (int64_t)v1 * W + slot * VW);
    b1 = rowptr[v1];
    d1 = (uint32_t)(rowptr[v1 + 1] - b1);
    if constexpr (PFX) p1 = (uint32_t)plen[v1];
  }
  int32_t u1[Q];  // first-step column ids of the current tile's vertex (third pipeline stage)
#pragma unroll
  for (int q = 0; q < Q; ++q)
    u1[q] = (tb + lofs < nact && q * G + slot < C && (uint32_t)(q * G + slot) < (PFX ? p1 : d1))
                ? col[b1 + q * G + slot] : -1;
  for (; tb < nact; tb += stride) {
    const int64_t idx = tb + lofs;
    const bool valid = idx < nact;
    const int32_t v = valid ? v1 : 0;
    const V<VW> r = r1;
    const int64_t beg = b1, end = b1 + (PFX ? p1 : d1);  // PFX: pull only the prefix
    const uint32_t deg = d1;
    int32_t u0[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) u0[q] = u1[q];
    // prefetch: row / offsets of the next tile, list entry of the one after
    v1 = v2;
    if (idx + stride < nact) {
      r1 = (snap && !any_visited(snap, v1)) ? vzero<VW>() : ldv<VW>(R + (int64_t)v1 * W + slot * VW);
      b1 = rowptr[v1];
      d1 = (uint32_t)(rowptr[v1 + 1] - b1);
      if constexpr (PFX) p1 = (uint32_t)plen[v1];
    }
    if (idx + 2 * stride < nact) v2 = act[idx + 2 * stride];
    V<VW> unv = vzero<VW>(), acc = vzero<VW>();
    bool lane_open = false, rnz = false;
    if (valid) {
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        unv.w[j] = ~r.w[j] & am.w[j];
        lane_open |= unv.w[j] != 0;
        rnz |= r.w[j] != 0;
      }
    }
    if constexpr (PFX) {  // bits pushed from the tail frontier (k_push_tail)
      if (valid && stamp[v] == epoch) {
        acc = ldv<VW>(pacc + (int64_t)v * W + slot * VW);
        stv<VW>(pacc + (int64_t)v * W + slot * VW, vzero<VW>());
      }
    }
    const bool g_open = valid && ((__ballot(lane_open) >> (sub * G)) & L::GBITS);
    int64_t e0 = beg;
    bool g_cov = false;
    if constexpr (C1 > 0) {
      static_assert(!FILT, "the short first step skips the filter");
      if (g_open) {
        V<VW> x[C1];
#pragma unroll
        for (int c = 0; c < C1; ++c) {
          const int32_t uc = G == 1 ? u0[c] : __shfl(u0[c / G], sub * G + (c % G));
          x[c] = uc >= 0 ? ldv<VW>(R + (int64_t)uc * W + slot * VW) : vzero<VW>();
        }
        bool cov = true;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
#pragma unroll
          for (int c = 0; c < C1; ++c) acc.w[j] |= x[c].w[j];
          cov &= (acc.w[j] & unv.w[j]) == unv.w[j];
        }
        g_cov = !((__ballot(!cov) >> (sub * G)) & L::GBITS);
        e0 = beg + C1;
      }
    }
    if (g_open && !g_cov) {
      for (int64_t e = e0; e < end; e += C) {
        int32_t u[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int64_t ee = e + q * G + slot;
          // first step: preloaded (without the short first step)
          u[q] = (C1 == 0 && e == beg) ? u0[q]
                                       : ((q * G + slot < C && ee < end) ? col[ee] : -1);
        }

        // ids below filter_from are loaded without a probe (filter off: filter_from = INT_MAX)
        // probes: every load first, every use after (with the use next to the load inside the
        // branch the compiler waited for each probe before issuing the next)
        if (FILT && filter_from != INT32_MAX) {  // wave-uniform
          // (LDS and global results in separate registers: a shared destination made the LDS
          // read wait for the outstanding global probes)
          uint32_t pg[Q], ph[Q];
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            pg[q] = ~0u;
            if (u[q] >= filter_from && !(HUBW > 0 && u[q] < HUBW * 32)) pg[q] = pvis[u[q] >> 5];
          }
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            ph[q] = ~0u;
            if (HUBW > 0 && u[q] >= filter_from && u[q] < HUBW * 32) ph[q] = hub[u[q] >> 5];
          }
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (!(((pg[q] & ph[q]) >> (u[q] & 31)) & 1u)) u[q] = -1;
        }
        V<VW> x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          // candidate c = column entry e + c: lane (c % G) of this group holds it in u[c / G]
          const int32_t uc = G == 1 ? u[c] : __shfl(u[c / G], sub * G + (c % G));
          x[c] = uc >= 0 ? ldv<VW>(R + (int64_t)uc * W + slot * VW) : vzero<VW>();
        }
        bool cov = true;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
#pragma unroll
          for (int c = 0; c < C; ++c) acc.w[j] |= x[c].w[j];
          cov &= (acc.w[j] & unv.w[j]) == unv.w[j];
        }
        // the whole group runs this loop in lock step (same v); exit when all lanes covered
        if (!((__ballot(!cov) >> (sub * G)) & L::GBITS)) break;

      }
    }
    V<VW> nw;
    bool anynew = false, notfull = false;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      nw.w[j] = acc.w[j] & unv.w[j];
      anynew |= nw.w[j] != 0;
      notfull |= (unv.w[j] & ~nw.w[j]) != 0;
    }
    if (valid) {  // also when nothing is open: Wb may hold the previous batch's rows
      V<VW> nv;
#pragma unroll
      for (int j = 0; j < VW; ++j) nv.w[j] = r.w[j] | nw.w[j];
      stv<VW>(Wb + (int64_t)v * W + slot * VW, nv);
    }
    if constexpr (FUSE) {  // nw is zero for invalid lanes
      bc.add(nw);
      if (++nadd == (1 << BitCounter<VW, PFX ? 5 : 6>::D) - 1) {
        bc.template spill_strided<CR>(cnt, slot);
        nadd = 0;
      }
    }
    const uint64_t bn = __ballot(anynew), bf = __ballot(notfull);
    const bool g_new = (bn >> (sub * G)) & L::GBITS;
    const bool g_nf = (bf >> (sub * G)) & L::GBITS;
    const bool leader = valid && slot == 0;
    if (leader && !g_nf) set_done(done, v);
    const bool keep = leader && g_nf, app = leader && g_new;
    if (keep) eu += deg;
    if (app) ef += deg;
    {
      const bool g_first = g_new && !((__ballot(rnz) >> (sub * G)) & L::GBITS);
      if (leader && g_first) {
        atomicOr(&anyvis[v >> 5], 1u << (v & 31));
        ev += deg;
      }
    }
    // third stage: the next tile's first-step ids (its offsets arrived during this tile)
#pragma unroll
    for (int q = 0; q < Q; ++q)
      u1[q] = (idx + stride < nact && q * G + slot < C &&
               (uint32_t)(q * G + slot) < (PFX ? p1 : d1))
                  ? col[b1 + q * G + slot] : -1;
    q_push(qa, keep && (int)deg <= next_wide, v);
    q_push(qw, keep && (int)deg > next_wide, v);
    q_push(qf, app, v);
    q_flush(qa, act2, &ctr->act2.v, TILE, false);
    q_flush(qw, actw2, &ctr->actw2.v, TILE, false);
    q_flush(qf, fl2, &ctr->fl2.v, TILE, false);
  }
  q_flush(qa, act2, &ctr->act2.v, 0, true);
  q_flush(qw, actw2, &ctr->actw2.v, 0, true);
  q_flush(qf, fl2, &ctr->fl2.v, 0, true);
  block_sum_add(eu, &ctr->eu2.v, scratch);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  if constexpr (FUSE) {
    bc.template spill_strided<CR>(cnt, slot);
    __syncthreads();
    uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
    for (int i = threadIdx.x; i < 64 * W; i += BT) row[i] = cnt[CR == 65 ? i + (i >> 6) : i];
  }
}

// ---------------------------------------------------------------------------------------------
// Late pull levels, first pass: from the third bottom-up level on almost every
// active vertex is covered by its first neighbour (rows sorted: the biggest hub first), and the
// level is bound by the latency of its dependent loads (list entry -> row offsets -> first column
// id -> neighbour row). This lean kernel (no multi-step loop, no software pipeline) keeps few
// registers, so twice as many waves hide that latency. A vertex the first row covers is
// finished here exactly as k_bu_narrow would (row, counts, done bit, frontier, anyvis); the others
// go to an overflow list (ctr->touched, unused by pull levels) that k_bu_narrow then processes
// from scratch.
// ---------------------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(kBlock, 8) void k_bu_first(
    const int32_t* act, int64_t nact, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, uint64_t* Wb, const uint64_t* alive, const uint64_t* gmask, uint32_t* done,
    int32_t* ovf, int32_t* fl2, Ctr* ctr, uint32_t* anyvis, uint32_t* slabF, const int32_t* first) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  constexpr int CR = 65;  // bank-skewed counter rows (see BitCounter::spill_strided)
  __shared__ LdsQueue qo, qf;
  __shared__ unsigned long long scratch[kWaves];
  __shared__ uint32_t cnt[CR * W];
  for (int i = threadIdx.x; i < CR * W; i += kBlock) cnt[i] = 0;
  q_init(qo);
  q_init(qf);
  __syncthreads();
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  unsigned long long ef = 0, ev = 0;
  BitCounter<VW> bc;
  bc.zero();
  int nadd = 0;
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nact; tb += (int64_t)gridDim.x * TILE) {
    const int64_t idx = tb + wv * VPW + sub;
    const bool valid = idx < nact;
    int32_t v = 0;
    V<VW> r = vzero<VW>(), nw = vzero<VW>();
    uint32_t deg = 0;
    bool open = false, rnz = false;
    if (valid) {
      v = act[idx];
      const int32_t u = first ? first[v] : col[rowptr[v]];  // active vertices have deg > 0
      r = ldv<VW>(R + (int64_t)v * W + slot * VW);
      deg = (uint32_t)(rowptr[v + 1] - rowptr[v]);  // only counted, off the load chain
      const V<VW> x = ldv<VW>(R + (int64_t)u * W + slot * VW);
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const uint64_t unv = ~r.w[j] & am.w[j];
        nw.w[j] = x.w[j] & unv;
        open |= (unv & ~nw.w[j]) != 0;
        rnz |= r.w[j] != 0;
      }
    }
    const bool g_open = (__ballot(open) >> (sub * G)) & L::GBITS;
    const bool fin = valid && !g_open;  // covered by the first row: finished at this level
    if (!fin) nw = vzero<VW>();
    if (fin) {
      V<VW> nv;
#pragma unroll
      for (int j = 0; j < VW; ++j) nv.w[j] = r.w[j] | nw.w[j];
      stv<VW>(Wb + (int64_t)v * W + slot * VW, nv);
    }
    bc.add(nw);
    if (++nadd == (1 << BitCounter<VW>::D) - 1) {
      bc.template spill_strided<CR>(cnt, slot);
      nadd = 0;
    }
    bool anynew = false;
#pragma unroll
    for (int j = 0; j < VW; ++j) anynew |= nw.w[j] != 0;
    const bool g_new = (__ballot(anynew) >> (sub * G)) & L::GBITS;
    const bool g_first = g_new && !((__ballot(rnz) >> (sub * G)) & L::GBITS);
    const bool leader = valid && slot == 0;
    if (leader && fin) set_done(done, v);
    if (leader && g_new) ef += deg;
    if (leader && g_first) {
      atomicOr(&anyvis[v >> 5], 1u << (v & 31));
      ev += deg;
    }
    q_push(qo, leader && !fin, v);
    q_push(qf, leader && g_new, v);
    q_flush(qo, ovf, &ctr->touched.v, TILE, false);
    q_flush(qf, fl2, &ctr->fl2.v, TILE, false);
  }
  q_flush(qo, ovf, &ctr->touched.v, 0, true);
  q_flush(qf, fl2, &ctr->fl2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  bc.template spill_strided<CR>(cnt, slot);
  __syncthreads();
  uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
  for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = cnt[i + (i >> 6)];
}

// bottom-up, wide vertices, phase 1: one wave per edge chunk (<= kChunk edges), processed in
// tiles of 256 edges so the dependent loads are batched instead of chained per neighbour:
//   A) all 64 lanes load 4 column ids each (one coalesced 1-KB pass), optionally test them
//      against the visited-by-anyone bitmap (256 independent loads), and compact the survivors
//      into an LDS list (ballot + popcount prefix);
//   B) the S = 64/G lane groups pull 4 neighbour rows each per step (4*S rows in flight per
//      wave), OR-reduce across groups (xor shuffles) and stop once every alive group is covered.
// The chunk's new bits are merged into acc[v] with atomicOr (k_bu_wide_finalize folds them in).
// offs = inclusive prefix of chunk counts over the wide list.
//
// HUBW > 0 (levels that filter): the block first copies the visited bitmap of the HUBW*32
// lowest ids into LDS. After degree relabelling those are the hubs, which carry most edge
// endpoints (RMAT-26: the top 2^19 ids take roughly two thirds), so most filter probes become
// LDS reads instead of divergent global loads. The copy is a snapshot taken at kernel start; a
// bit another kernel of this level sets later belongs to a vertex first visited at this level,
// whose row in R is still zero, so skipping it is exact. Big blocks (BT threads, 2 per CU)
// amortise the copy; the grid is persistent (grid-stride over chunks).
// One wave pulls edges [beg, lim) of wide vertex v (a chunk) and publishes the new bits into
// acc[v] (k_bu_wide_finalize folds them in). coop: chunks of one vertex run concurrently and
// share progress through acc (see below); coop = 0 (first bottom-up level) skips that.
template <int W, int T, int HUBW>
__device__ __forceinline__ void chunk_pull(int32_t v, int64_t beg, int64_t lim, const int32_t* col,
                                           const uint64_t* R, const V<Lay<W>::VW>& am,
                                           uint64_t* acc, const uint32_t* anyvis,
                                           const uint32_t* hub, int32_t filter_from, int coop,
                                           int32_t* lst, const uint32_t* code,
                                           int32_t code_from, unsigned long long* wacc,
                                           const uint32_t* snap) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, S = L::VPW;
  constexpr int PB = VW == 2 ? 4 : 8;  // rows in flight per lane group in phase B
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int64_t vo = (int64_t)v * W + slot * VW;
  const V<VW> r = (snap && !any_visited(snap, v)) ? vzero<VW>() : ldv<VW>(R + vo);  // see k_bu_narrow
  // g = bits the vertex's other chunks have published so far. Chunks of one hub run
  // concurrently, so each tile publishes its partial OR with a RETURNING atomicOr that also
  // hands back the current union from the memory side (atomics bypass the non-coherent per-XCD
  // L2s); every chunk stops once the union covers all alive groups.
  V<VW> g = vzero<VW>();
  if (coop) {
    if (sub == 0) {
#pragma unroll
      for (int j = 0; j < VW; ++j) g.w[j] = atomicOr((unsigned long long*)&acc[vo + j], 0ull);
    }
#pragma unroll
    for (int j = 0; j < VW; ++j) g.w[j] = __shfl(g.w[j], slot);  // lane slot of sub-group 0
  }
  V<VW> unv, a = vzero<VW>();
  bool lane_open = false;
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    unv.w[j] = ~r.w[j] & am.w[j];
    lane_open |= (unv.w[j] & ~g.w[j]) != 0;
  }
  if (!__ballot(lane_open)) return;  // wave-uniform
  bool covered = false;
  for (int64_t t0 = beg; t0 < lim && !covered; t0 += T) {
    // ---- phase A: ids of this tile, filtered, compacted into lst[0..cnt)
    constexpr int Q = T / 64;
    int32_t u[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t e = t0 + q * 64 + lane;
      u[q] = e < lim ? col[e] : -1;
    }
    if (filter_from != INT32_MAX) {
      // probes: every load first, every use after (see k_bu_narrow)
      uint32_t pg[Q], ph[Q];  // separate destinations (see k_bu_narrow)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        pg[q] = ~0u;
        if (u[q] >= filter_from && !(HUBW > 0 && u[q] < HUBW * 32)) pg[q] = anyvis[u[q] >> 5];
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        ph[q] = ~0u;
        if (HUBW > 0 && u[q] >= 0 && u[q] < HUBW * 32) ph[q] = hub[u[q] >> 5];
      }
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (u[q] >= 0 && !(((pg[q] & ph[q]) >> (u[q] & 31)) & 1u)) u[q] = -1;
    }
    if (code_from != kNoCodes) {  // wave-uniform
      // single-group neighbours: their bit goes into this wave's LDS words (ds_or_b64) instead
      // of a row gather; the words are folded into every lane group's accumulator below
      if (lane < W) wacc[lane] = 0;
      __builtin_amdgcn_wave_barrier();
      uint32_t cd[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        cd[q] = kDenseCode;
        if (u[q] >= code_from) cd[q] = code[u[q]];
      }
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (cd[q] != kDenseCode) {
#pragma unroll
          for (int i = 0; i < kCodeSlots; ++i) {
            const int g = code_g(cd[q], i);
            if (g >= 0) atomicOr(&wacc[g >> 6], 1ull << (g & 63));
          }
          u[q] = -1;
        }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < VW; ++j) a.w[j] |= wacc[slot * VW + j];
    }
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint64_t m = __ballot(u[q] >= 0);
      if (u[q] >= 0) lst[cnt + __popcll(m & lanemask_lt())] = u[q];
      cnt += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    // ---- phase B: rows of the surviving neighbours, PB per lane group per step
    for (int b = 0; b < cnt; b += PB * S) {
      int32_t uu[PB];
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int k = b + q * S + sub;
        uu[q] = k < cnt ? lst[k] : -1;
      }
      {
        // loads first, ORs after: the compiler then keeps all PB loads in flight
        V<VW> x[PB];
#pragma unroll
        for (int q = 0; q < PB; ++q) {
          x[q] = vzero<VW>();
          if (uu[q] >= 0) x[q] = ldv<VW>(R + (int64_t)uu[q] * W + slot * VW);
        }
#pragma unroll
        for (int q = 0; q < PB; ++q)
#pragma unroll
          for (int j = 0; j < VW; ++j) a.w[j] |= x[q].w[j];
      }
#pragma unroll
      for (int off = G; off < 64; off <<= 1)
#pragma unroll
        for (int j = 0; j < VW; ++j) a.w[j] |= __shfl_xor(a.w[j], off);
      bool cov = true;
#pragma unroll
      for (int j = 0; j < VW; ++j) cov &= ((a.w[j] | g.w[j]) & unv.w[j]) == unv.w[j];
      if (!__ballot(!cov)) {
        covered = true;
        break;
      }
    }
    __builtin_amdgcn_wave_barrier();  // lst is rewritten by the next tile
    // publish this chunk's bits so far and pick up the other chunks' (one round trip)
    if (coop && !covered && t0 + T < lim) {
      bool cov = true;
      if (sub == 0) {
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const uint64_t nb = a.w[j] & unv.w[j] & ~g.w[j];
          g.w[j] |= nb ? atomicOr((unsigned long long*)&acc[vo + j], nb)
                       : atomicOr((unsigned long long*)&acc[vo + j], 0ull);
          g.w[j] |= nb;
          cov &= ((a.w[j] | g.w[j]) & unv.w[j]) == unv.w[j];
        }
      }
      if (!__ballot(!cov)) covered = true;
#pragma unroll
      for (int j = 0; j < VW; ++j) g.w[j] = __shfl(g.w[j], slot);
    }
  }
  if (sub == 0) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const uint64_t nb = a.w[j] & unv.w[j] & ~g.w[j];
      if (nb) atomicOr((unsigned long long*)&acc[vo + j], nb);
    }
  }
}

// Chunk descriptor: vertex, first column position, edge count (<= kChunk). Built once per level
// by k_chunk_desc; a wave reads its next descriptor with one scalar load while it pulls the
// current chunk (vs an owner -> list entry -> row offsets chain of dependent loads per chunk).
struct ChunkDesc {
  int32_t v;
  uint32_t beg_lo, beg_hi;
  int32_t len;
};

// first position in the sorted row [b, e) whose id is >= H
__device__ __forceinline__ int64_t row_lower_bound(const int32_t* col, int64_t b, int64_t e,
                                                   int32_t H) {
  while (b < e) {
    const int64_t mid = (b + e) >> 1;
    if (col[mid] < H) b = mid + 1;
    else e = mid;
  }
  return b;
}

// plen[v] = length of v's row prefix with ids < H (rows sorted; a graph property, computed once
// per graph and bound H, see BitparSolver::prefix_lens)
__global__ __launch_bounds__(kBlock) void k_prefix_lens(const int64_t* rowptr, const int32_t* col,
                                                        int64_t n, int32_t H, int32_t* plen) {
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n;
       v += (int64_t)gridDim.x * kBlock) {
    const int64_t b = rowptr[v];
    plen[v] = (int32_t)(row_lower_bound(col, b, rowptr[v + 1], H) - b);
  }
}

// first[v] = v's first neighbour (rows sorted: after degree relabelling its biggest hub), -1 for
// an isolated vertex: the lean first-row pass (k_bu_first) reads it with one coalesced 4-byte load
// instead of the rowptr -> col chain, whose col[rowptr[v]] touches one 128-byte line per vertex
__global__ __launch_bounds__(kBlock) void k_first_nbr(const int64_t* rowptr, const int32_t* col,
                                                      int64_t n, int32_t* first) {
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n;
       v += (int64_t)gridDim.x * kBlock) {
    const int64_t b = rowptr[v];
    first[v] = rowptr[v + 1] > b ? col[b] : -1;
  }
}

// chunk counts of the wide vertices' row prefixes (inclusive-scanned into offs by the host)
__global__ __launch_bounds__(kBlock) void k_prefix_chunks(const int32_t* wl, int64_t nw,
                                                          const int32_t* plen, int64_t* cnt) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nw;
       i += (int64_t)gridDim.x * kBlock)
    cnt[i] = ((int64_t)plen[wl[i]] + kChunk - 1) / kChunk;
}

// plen != nullptr: chunks cover only the row prefixes with ids < H (prefix-pull level)
__global__ __launch_bounds__(kBlock) void k_chunk_desc(const int32_t* wl, int64_t nw,
                                                       const int64_t* offs, const int64_t* rowptr,
                                                       const int32_t* plen, ChunkDesc* desc) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nw;
       i += (int64_t)gridDim.x * kBlock) {
    const int32_t v = wl[i];
    const int64_t b = rowptr[v];
    const int64_t e = plen ? b + plen[v] : rowptr[v + 1];
    const int64_t c0 = i ? offs[i - 1] : 0, c1 = offs[i];
    for (int64_t c = c0; c < c1; ++c) {
      const int64_t cb = b + (c - c0) * kChunk;
      desc[c] = ChunkDesc{v, (uint32_t)cb, (uint32_t)((uint64_t)cb >> 32),
                          (int32_t)min((int64_t)kChunk, e - cb)};
    }
  }
}

template <int W, int T, int BT, int HUBW>
__global__ __launch_bounds__(BT, (BT >= 1024 && HUBW <= 16384) ? 8 : 4) void k_bu_chunks(
    const ChunkDesc* __restrict__ desc, const int64_t* nchunks_p, const int32_t* col,
    const uint64_t* R,
    const uint64_t* alive, const uint64_t* gmask, uint64_t* acc, const uint32_t* anyvis,
    int32_t filter_from, int coop, const uint32_t* code, int32_t code_from,
    const uint32_t* snap) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G;
  __shared__ int32_t tile[BT / 64][T];
  __shared__ unsigned long long wacc[BT / 64][W];
  __shared__ uint32_t hub[HUBW > 0 ? HUBW : 1];
  if (snap) anyvis = snap;  // probes read the level-start bitmap (see k_bu_narrow)
  if constexpr (HUBW > 0) {
    for (int i = threadIdx.x; i < HUBW; i += BT) hub[i] = anyvis[i];
    __syncthreads();
  }
  const int slot = lane_id() % G;
  int32_t* lst = tile[threadIdx.x >> 6];
  const int64_t nchunks = uni64(*nchunks_p);  // inclusive chunk prefix of the last wide vertex
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  // Chunk order. Without early exit (coop = 0: the first bottom-up level, where hardly any row
  // is covered) chunks are dealt round robin over the waves, which balances the hubs' expensive
  // chunks. With early exit a wave takes a contiguous run, so a vertex's later chunks usually
  // come after its earlier ones have published their bits and are skipped at the first check.
  const int64_t cstart = uni64(coop ? nchunks * wave / nwaves : wave);
  const int64_t cend = uni64(coop ? nchunks * (wave + 1) / nwaves : nchunks);
  const int64_t cstep = uni64(coop ? 1 : nwaves);
  ChunkDesc d{0, 0, 0, 0};
  if (cstart < cend) d = desc[cstart];
  for (int64_t c = cstart; c < cend; c += cstep) {
    const int32_t v = uni32(d.v);
    const int64_t beg = uni64((int64_t)(((uint64_t)d.beg_hi << 32) | d.beg_lo));
    const int64_t lim = beg + uni32(d.len);
    if (c + cstep < cend) d = desc[c + cstep];  // next descriptor, in flight during the pull
    chunk_pull<W, T, HUBW>(v, beg, lim, col, R, am, acc, anyvis, hub, filter_from, coop,
                           lst, code, code_from, wacc[threadIdx.x >> 6], snap);
  }
}

// bottom-up, wide vertices, phase 2: G lanes per vertex fold acc[v] into the visited words.
template <int W, bool COUNT, bool FUSE>
__global__ __launch_bounds__(kBlock) void k_bu_wide_finalize(
    const int32_t* wl, int64_t nw, const int64_t* rowptr, const uint64_t* R, uint64_t* Wb,
    uint64_t* acc, const uint64_t* alive, const uint64_t* gmask, uint32_t* done, int32_t* actw2,
    int32_t* fl2, Ctr* ctr, uint32_t* anyvis, int32_t* act2n, int next_wide, uint32_t* slabF,
    const uint32_t* snap) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  __shared__ LdsQueue qa, qf, qn;
  __shared__ unsigned long long scratch[kWaves];
  // bank-skewed counter rows (see BitCounter::spill_strided): wide vertices gain many groups
  // at once, so every spill touches most counters
  constexpr int CR = 65;
  __shared__ uint32_t cnt[FUSE ? CR * W : 1];
  if constexpr (FUSE)
    for (int i = threadIdx.x; i < CR * W; i += kBlock) cnt[i] = 0;
  q_init(qa);
  q_init(qf);
  q_init(qn);
  __syncthreads();
  BitCounter<VW> bc;
  int nadd = 0;
  if constexpr (FUSE) bc.zero();
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  unsigned long long eu = 0, ef = 0, ev = 0;
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nw; tb += (int64_t)gridDim.x * TILE) {
    const int64_t idx = tb + wv * VPW + sub;
    const bool valid = idx < nw;
    int32_t v = 0;
    V<VW> nwb = vzero<VW>();
    bool anynew = false, notfull = false, rnz = false;
    uint32_t deg = 0;
    if (valid) {
      v = wl[idx];
      const int64_t vo = (int64_t)v * W + slot * VW;
      const V<VW> r = (snap && !any_visited(snap, v)) ? vzero<VW>() : ldv<VW>(R + vo);
      const V<VW> a = ldv<VW>(acc + vo);
      V<VW> nv;
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const uint64_t unv = ~r.w[j] & am.w[j];
        nwb.w[j] = a.w[j] & unv;
        nv.w[j] = r.w[j] | nwb.w[j];
        anynew |= nwb.w[j] != 0;
        notfull |= (unv & ~nwb.w[j]) != 0;
        rnz |= r.w[j] != 0;
      }
      stv<VW>(acc + vo, vzero<VW>());
      stv<VW>(Wb + vo, nv);
      deg = (uint32_t)(rowptr[v + 1] - rowptr[v]);
    }
    if constexpr (FUSE) {  // nwb is zero for invalid lanes
      bc.add(nwb);
      if (++nadd == (1 << BitCounter<VW>::D) - 1) {
        bc.template spill_strided<CR>(cnt, slot);
        nadd = 0;
      }
    }
    const uint64_t bn = __ballot(anynew), bf = __ballot(notfull);
    const bool g_new = (bn >> (sub * G)) & L::GBITS;
    const bool g_nf = (bf >> (sub * G)) & L::GBITS;
    const bool leader = valid && slot == 0;
    if (leader && !g_nf) set_done(done, v);
    const bool keep = leader && g_nf, app = leader && g_new;
    if (keep) eu += deg;
    if (app) ef += deg;
    {
      const bool g_first = g_new && !((__ballot(rnz) >> (sub * G)) & L::GBITS);
      if (leader && g_first) {
        atomicOr(&anyvis[v >> 5], 1u << (v & 31));
        ev += deg;
      }
    }
    q_push(qa, keep && (int)deg > next_wide, v);
    q_push(qn, keep && (int)deg <= next_wide, v);
    q_push(qf, app, v);
    q_flush(qa, actw2, &ctr->actw2.v, TILE, false);
    q_flush(qn, act2n, &ctr->act2.v, TILE, false);
    q_flush(qf, fl2, &ctr->fl2.v, TILE, false);
  }
  q_flush(qa, actw2, &ctr->actw2.v, 0, true);
  q_flush(qn, act2n, &ctr->act2.v, 0, true);
  q_flush(qf, fl2, &ctr->fl2.v, 0, true);
  block_sum_add(eu, &ctr->eu2.v, scratch);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  if constexpr (FUSE) {
    bc.template spill_strided<CR>(cnt, slot);
    __syncthreads();
    uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
    for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = cnt[i + (i >> 6)];
  }
}

// ---------------------------------------------------------------------------------------------
// Per-level accounting, once per level over the NEW frontier list (kept out of the traversal
// kernels so they keep their occupancy): new bits of v = visNew[v] & ~visOld[v] after a
// bottom-up level (DIFF) or acc[v] after a top-down level. G lanes per vertex; counts go to
// register bit-sliced counters (or, for the edge-count mode, per-bit LDS atomics weighted by
// degree), then to this block's slab row.
// ---------------------------------------------------------------------------------------------
template <int W, bool COUNT, bool DIFF>
__global__ __launch_bounds__(kBlock) void k_count_frontier(const int32_t* fl, const Ctr* ctr,
                                                           const int64_t* rowptr,
                                                           const uint64_t* a,
                                                           const uint64_t* b, uint32_t* slabF,
                                                           unsigned long long* slabE) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  __shared__ Lds<W, COUNT> s;
  lds_zero(s);
  __syncthreads();
  const int64_t nf = ctr->fl2.v;
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  BitCounter<VW> bc;
  bc.zero();
  int nadd = 0;
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nf; tb += (int64_t)gridDim.x * TILE) {
    const int64_t idx = tb + wv * VPW + sub;
    V<VW> nw = vzero<VW>();
    uint32_t deg = 0;
    if (idx < nf) {
      const int32_t v = fl[idx];
      const int64_t vo = (int64_t)v * W + slot * VW;
      nw = ldv<VW>(a + vo);
      if constexpr (DIFF) {
        const V<VW> o = ldv<VW>(b + vo);
#pragma unroll
        for (int j = 0; j < VW; ++j) nw.w[j] &= ~o.w[j];
      }
      if constexpr (COUNT) deg = (uint32_t)(rowptr[v + 1] - rowptr[v]);
    }
    if constexpr (COUNT) {
      count_bits<W, COUNT>(s, nw, slot, deg);
    } else {
      bc.add(nw);
      if (++nadd == (1 << BitCounter<VW>::D) - 1) {
        bc.spill(s, slot);
        nadd = 0;
      }
    }
  }
  if constexpr (!COUNT) bc.spill(s, slot);
  slab_store<W, COUNT>(s, slabF, slabE);
}

// ---------------------------------------------------------------------------------------------
// hybrid multi-GPU mode: kernels
//
// Why: with groups split round-robin over GPUs (main.cu:304-307) every GPU still scans the whole
// graph at the first bottom-up level, whose cost hardly depends on the number of groups (a row
// scan stops only once EVERY group is covered), so 8 GPUs each pay most of one GPU's time. Levels
// 1-2 need only the sources' neighbourhoods, which every rank can build for all groups, so level
// 2 is split by vertex (each rank pulls for its residue class v = part mod nparts, for all
// groups) and one all-to-all then gives every rank its own block of words for every vertex
// (hybrid 2D decomposition: vertex-partitioned for the explosive level, query-partitioned after
// it). The cyclic vertex split balances both the pull work (hubs and tail spread evenly) and the
// exchange (every rank sends the same number of rows); vertices >= n_eff (the deg-0 suffix of a
// degree-relabelled graph) are not exchanged at all.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxParts = Solver::kHybridMaxParts;
struct WordSplit {
  int32_t b[kMaxParts + 1];
};
struct PartPrefix {
  int64_t b[kMaxParts + 1];  // b[r] = number of vertices owned by parts < r
};

// own vertices of part `part` of `nparts` below n_eff: v = part + i*nparts
static inline int64_t part_count(int64_t n_eff, int part, int nparts) {
  return n_eff > part ? (n_eff - part + nparts - 1) / nparts : 0;
}

// ---- zero-word coding of the hybrid exchange -------------------------------------------------
// After level 2 about half of the exchanged 64-bit words are zero (RMAT-26, 1024 groups, 8
// ranks: 50.5 %). A segment of L words (one destination's share) travels as ceil(L/64) bitmap
// words (bit i of bitmap word c: word 64c+i is nonzero) followed by its nonzero words in order
// (parallel/hybrid.py encode_np/decode_np are the reference twins). The sender packs the dense
// segments (k_pack_words) and codes them 8 chunks of 64 words per wave (k_code_bits -> scan ->
// k_code_emit: coalesced 512-byte chunk reads; coding straight from the visited rows read each
// 128-byte row once per destination: 1.5 ms at 8 ranks); the receiver expands into the dense
// layout phase C reads (k_decode_pop -> scan -> k_decode_emit). Chunks (64 words) are numbered
// globally over the segments; a segment's chunks are [c0[j], c0[j+1]).
struct CodeSegs {
  int64_t c0[kMaxParts + 1];  // first global chunk of each segment; c0[nseg] = total chunks
  int64_t len[kMaxParts];     // dense words of each segment
  int64_t base[kMaxParts];    // decode: coded start of each segment in the received buffer
  int64_t dense[kMaxParts];   // decode: dense start of each segment
};

__device__ __forceinline__ int code_seg(const CodeSegs& cs, int nseg, int64_t c) {
  int j = 0;
  while (j + 1 < nseg && c >= cs.c0[j + 1]) ++j;
  return j;
}

// send[cnt*wbeg[j] + i*nw_j + (w-wbeg[j])] = vis[v*W + w], v = part + i*nparts: destination-major
// (rows of deg-0 vertices may be stale, see k_zero_src_rows: they are sent as zeros; phase C
// never reads them either)
template <int W>
__global__ __launch_bounds__(kBlock) void k_pack_words(const uint64_t* vis, const int64_t* rowptr,
                                                       int part, int nparts, int64_t cnt, int wt,
                                                       WordSplit ws, uint64_t* send) {
  const int64_t total = cnt * wt;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t i = t / wt;
    const int w = (int)(t - i * wt);
    const int64_t v = part + i * nparts;
    int j = 0;
    while (w >= ws.b[j + 1]) ++j;
    const int nw = ws.b[j + 1] - ws.b[j];
    const bool deg0 = rowptr[v + 1] == rowptr[v];
    send[cnt * ws.b[j] + i * nw + (w - ws.b[j])] = deg0 ? 0ull : vis[v * W + w];
  }
}

// Chunks per wave in the coding kernels: the loads of all of them are issued before any use
// (one chunk per wave left the kernels bound by wave launches and single dependent loads).
constexpr int kCodeCPW = 8;

// bitmap word and popcount of every chunk of the dense segments in `dense` (segment j starts at
// cs.dense[j])
__global__ __launch_bounds__(kBlock) void k_code_bits(const uint64_t* dense, CodeSegs cs, int nseg,
                                                      uint64_t* bits, int64_t* pop) {
  const int lane = lane_id();
  const int64_t nch = cs.c0[nseg];
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t cb = (((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * kCodeCPW; cb < nch;
       cb += nwaves * kCodeCPW) {
    uint64_t x[kCodeCPW];
    int j = code_seg(cs, nseg, cb);
#pragma unroll
    for (int k = 0; k < kCodeCPW; ++k) {
      const int64_t c = cb + k;
      while (j + 1 < nseg && c >= cs.c0[j + 1]) ++j;
      const int64_t t = (c - cs.c0[j]) * 64 + lane;
      x[k] = (c < nch && t < cs.len[j]) ? dense[cs.dense[j] + t] : 0ull;
    }
    uint64_t mine = 0;
#pragma unroll
    for (int k = 0; k < kCodeCPW; ++k) {
      const uint64_t bm = __ballot(x[k] != 0);
      if (lane == k) mine = bm;
    }
    if (lane < kCodeCPW && cb + lane < nch) {
      bits[cb + lane] = mine;
      pop[cb + lane] = __popcll(mine);
    }
  }
}

// incl = inclusive scan of pop. Segment j's coded start is c0[j] + X(c0[j]), X = exclusive
// prefix: bitmap word of chunk c at c + X(c0[j]), its nonzero words from c0[j+1] + X(c).
__global__ __launch_bounds__(kBlock) void k_code_emit(const uint64_t* dense, CodeSegs cs, int nseg,
                                                      const uint64_t* bits, const int64_t* incl,
                                                      uint64_t* out) {
  const int lane = lane_id();
  const int64_t nch = cs.c0[nseg];
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t cb = (((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * kCodeCPW; cb < nch;
       cb += nwaves * kCodeCPW) {
    // lane k < CPW holds chunk cb+k's bitmap, inclusive prefix and segment start offset
    uint64_t bml = 0;
    int64_t incl_l = 0, xj_l = 0;
    int jl = 0;
    if (lane < kCodeCPW && cb + lane < nch) {
      const int64_t c = cb + lane;
      jl = code_seg(cs, nseg, c);
      bml = bits[c];
      incl_l = incl[c];
      const int64_t cj = cs.c0[jl];
      xj_l = incl[cj] - __popcll(bits[cj]);
    }
    uint64_t x[kCodeCPW];
#pragma unroll
    for (int k = 0; k < kCodeCPW; ++k) {  // every data load first
      const uint64_t bm = __shfl(bml, k);
      const int j = __shfl(jl, k);
      const int64_t c = cb + k;
      x[k] = (c < nch && ((bm >> lane) & 1ull))
                 ? dense[cs.dense[j] + (c - cs.c0[j]) * 64 + lane] : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kCodeCPW; ++k) {
      const int64_t c = cb + k;
      if (c >= nch) break;
      const uint64_t bm = __shfl(bml, k);
      const int j = __shfl(jl, k);
      const int64_t xc = __shfl(incl_l, k) - __popcll(bm);
      const int64_t xj = __shfl(xj_l, k);
      if (lane == 0) out[c + xj] = bm;
      if ((bm >> lane) & 1ull) out[cs.c0[j + 1] + xc + __popcll(bm & lanemask_lt())] = x[k];
    }
  }
}

// coded length of every segment: its chunks (bitmap words) + its nonzero words
__global__ void k_code_lens(CodeSegs cs, int nseg, const uint64_t* bits, const int64_t* incl,
                            int64_t* lens) {
  const int j = threadIdx.x;
  if (j >= nseg) return;
  const int64_t a = cs.c0[j], b = cs.c0[j + 1];
  lens[j] = b > a ? (b - a) + incl[b - 1] - (incl[a] - __popcll(bits[a])) : 0;
}

// receiver: one thread per received chunk, popcount of its bitmap word
__global__ __launch_bounds__(kBlock) void k_decode_pop(const uint64_t* in, CodeSegs cs, int nseg,
                                                       int64_t* pop) {
  const int64_t nch = cs.c0[nseg];
  for (int64_t d = (int64_t)blockIdx.x * kBlock + threadIdx.x; d < nch;
       d += (int64_t)gridDim.x * kBlock) {
    const int r = code_seg(cs, nseg, d);
    pop[d] = __popcll(in[cs.base[r] + (d - cs.c0[r])]);
  }
}

// kCodeCPW received chunks per wave: their 64 dense words each (zeros included)
__global__ __launch_bounds__(kBlock) void k_decode_emit(const uint64_t* in, CodeSegs cs, int nseg,
                                                        const int64_t* incl, uint64_t* dense) {
  const int lane = lane_id();
  const int64_t nch = cs.c0[nseg];
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t db = (((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * kCodeCPW; db < nch;
       db += nwaves * kCodeCPW) {
    // lane k < CPW: chunk db+k's segment, bitmap word and data start
    uint64_t bml = 0;
    int64_t data_l = 0;
    int rl = 0;
    if (lane < kCodeCPW && db + lane < nch) {
      const int64_t d = db + lane;
      rl = code_seg(cs, nseg, d);
      const int64_t d0 = cs.c0[rl];
      const uint64_t* seg = in + cs.base[rl];
      bml = seg[d - d0];
      // nonzero words before this chunk in segment r
      const int64_t before = (incl[d] - __popcll(bml)) - (incl[d0] - __popcll(seg[0]));
      data_l = cs.base[rl] + (cs.c0[rl + 1] - d0) + before;
    }
    uint64_t x[kCodeCPW];
#pragma unroll
    for (int k = 0; k < kCodeCPW; ++k) {
      const uint64_t bm = __shfl(bml, k);
      const int64_t dl = __shfl(data_l, k);  // every lane takes part in the shuffle
      x[k] = (db + k < nch && ((bm >> lane) & 1ull)) ? in[dl + __popcll(bm & lanemask_lt())]
                                                     : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kCodeCPW; ++k) {
      const int64_t d = db + k;
      if (d >= nch) break;
      const int r = __shfl(rl, k);
      const int64_t t = (d - cs.c0[r]) * 64 + lane;
      if (t < cs.len[r]) dense[cs.dense[r] + t] = x[k];
    }
  }
}

// Phase C state from the received words: both visited buffers (stride W, zero padding beyond
// nw), done = every alive group present, anyvis = any bit. One thread per vertex; the bitmaps
// are written with plain stores from wave ballots (64 vertices = 2 words), so no memset.
// recv holds, per source part r (in order), nw words of each of r's vertices v = r + i*nparts.
// It also builds the first phase-C level's active lists (deg > 0, not done, split at wide_deg;
// what k_build_active would do in a second pass over the vertices). Vertices >= n_eff (no
// edges) are skipped: no phase-C kernel reads their rows or bits.
template <int W>
__global__ __launch_bounds__(kBlock) void k_hybrid_setup(const uint64_t* recv, int nw,
                                                         int64_t n_eff, int nparts, PartPrefix pre,
                                                         uint64_t* visA, uint64_t* visB,
                                                         const uint64_t* alive,
                                                         const uint64_t* gmask, uint32_t* done,
                                                         uint32_t* anyvis, const int64_t* rowptr,
                                                         int wide_deg, int32_t* act,
                                                         int32_t* actw, Ctr* ctr) {
  // G lanes per vertex (the solver's row layout): every row read and write is coalesced (with one
  // thread per vertex the W-word rows were written at a W*8-byte lane stride: 6.9 ms instead of
  // ~1 ms at W = 8). A block covers TILE consecutive vertices, a multiple of 32, so it writes whole
  // done / anyvis words with plain stores.
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  static_assert(TILE % 32 == 0, "whole bitmap words per block");
  __shared__ uint8_t fullf[TILE], nzf[TILE];
  __shared__ LdsQueueN<2048> qn, qw;
  __shared__ unsigned long long scratch[kWaves];
  q_init(qn);
  q_init(qw);
  __syncthreads();
  unsigned long long eu = 0;
  const int64_t nwords32 = (n_eff + 31) / 32;
  const int lane = lane_id(), slot = lane % G, sub = lane / G, wv = threadIdx.x >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < n_eff; tb += (int64_t)gridDim.x * TILE) {
    const int64_t v = tb + wv * VPW + sub;
    V<VW> x = vzero<VW>();
    int64_t deg = 0;
    if (v < n_eff) {
      const uint64_t* src = recv + (pre.b[v % nparts] + v / nparts) * nw;
      if (slot == 0) deg = rowptr[v + 1] - rowptr[v];
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const int w = slot * VW + j;
        x.w[j] = w < nw ? src[w] : 0ull;
      }
    }
    bool nz = false, full = true;
    if (v < n_eff) {
      stv<VW>(visA + v * W + slot * VW, x);
      stv<VW>(visB + v * W + slot * VW, x);
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        nz |= x.w[j] != 0;
        full &= (~x.w[j] & am.w[j]) == 0;
      }
    }
    const bool g_nz = (__ballot(nz) >> (sub * G)) & L::GBITS;
    const bool g_full = !((__ballot(!full) >> (sub * G)) & L::GBITS);
    if (slot == 0) {
      fullf[wv * VPW + sub] = v < n_eff && g_full;
      nzf[wv * VPW + sub] = g_nz;
    }
    const bool actv = slot == 0 && v < n_eff && deg > 0 && !g_full;
    if (actv) eu += (unsigned long long)deg;
    q_push(qn, actv && deg <= wide_deg, (int32_t)v);
    q_push(qw, actv && deg > wide_deg, (int32_t)v);
    q_flush(qn, act, &ctr->act2.v, TILE, false);
    q_flush(qw, actw, &ctr->actw2.v, TILE, false);
    for (int i = threadIdx.x; i < TILE / 32; i += kBlock) {
      const int64_t w32 = (tb >> 5) + i;
      if (w32 < nwords32) {
        uint32_t d = 0, a = 0;
        for (int b = 0; b < 32; ++b) {
          d |= (uint32_t)fullf[i * 32 + b] << b;
          a |= (uint32_t)nzf[i * 32 + b] << b;
        }
        done[w32] = d;
        anyvis[w32] = a;
      }
    }
    __syncthreads();
  }
  q_flush(qn, act, &ctr->act2.v, 0, true);
  q_flush(qw, actw, &ctr->actw2.v, 0, true);
  block_sum_add(eu, &ctr->eu2.v, scratch);
}

// n_eff = 1 + the last vertex with deg > 0 (0 if none): per-thread max, wave max, one atomic
// per wave (atomics on one address serialise)
__global__ void k_extent(const int64_t* rowptr, int64_t n, unsigned long long* out) {
  unsigned long long m = 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (int64_t)gridDim.x * blockDim.x)
    if (rowptr[v + 1] > rowptr[v]) m = (unsigned long long)(v + 1);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(m, off);
    m = o > m ? o : m;
  }
  if (lane_id() == 0 && m) atomicMax(out, m);
}

// ---------------------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------------------
class BitparSolver final : public Solver {
 public:
  BitparSolver(const DeviceGraph& g, int max_groups) : g_(g) {
    int w = 1;
    while (w * 64 < max_groups && w < 16) w <<= 1;
    const int64_t n = std::max<int64_t>(g.n, 1);
    // Size the batch width to free HBM: 4 visited/accumulator buffers of n*W words plus ~48 B
    // per vertex of lists; groups beyond 64*W run as further batches.
    {
      size_t free_b = 0, total_b = 0;
      if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
        const double fixed = 52.0 * (double)n + (double)g.nnz / 256.0 + 64.0 * (1 << 20);
        while (w > 1 && fixed + 32.0 * (double)n * w > 0.92 * (double)free_b) w >>= 1;
        if (fixed + 32.0 * (double)n * w > 0.92 * (double)free_b)
          fail("not enough device memory for the bit-parallel solver (n=" + std::to_string(n) + ")");
      }
    }
    maxW_ = w;
    const size_t vb = (size_t)n * maxW_ * sizeof(uint64_t);
    for (int i = 0; i < 2; ++i) {
      vis_[i].alloc(vb);
      acc_[i].alloc(vb);
      MSBFS_HIP_CHECK(hipMemset(acc_[i].p, 0, vb));
    }
    stamp_.alloc((size_t)n * sizeof(int32_t));
    MSBFS_HIP_CHECK(hipMemset(stamp_.p, 0xFF, stamp_.bytes));
    done_.alloc((size_t)((n + 31) / 32) * sizeof(uint32_t));
    anyvis_.alloc((size_t)((n + 31) / 32) * sizeof(uint32_t));
    asnap_.alloc((size_t)((n + 31) / 32) * sizeof(uint32_t));
    if (const char* f = getenv("MSBFS_FILTER_FRAC")) filter_frac_ = atof(f);
    if (const char* h = getenv("MSBFS_HUB_MB")) hub_bytes_ = atof(h) * (1 << 20);
    for (int i = 0; i < 2; ++i) {
      act_[i].alloc((size_t)n * sizeof(int32_t));
      actw_[i].alloc((size_t)n * sizeof(int32_t));
      fl_[i].alloc((size_t)n * sizeof(int32_t));
    }
    touched_.alloc((size_t)n * sizeof(int32_t));
    offs_.alloc((size_t)n * sizeof(int64_t));
    scan_bytes_ = frontier_scan_temp_bytes(n);
    scan_tmp_.alloc(scan_bytes_);
    ctr_.alloc(sizeof(Ctr));
    small_.alloc(64 * 16 * sizeof(unsigned long long) * 2 + 4 * 16 * sizeof(uint64_t));
    // per-level counter slab: <= 3 counting kernels per level x <= kMaxGrid blocks
    slabF_.alloc((size_t)3 * kMaxGrid * 64 * maxW_ * sizeof(uint32_t));
    slabE_.alloc((size_t)3 * kMaxGrid * 64 * maxW_ * sizeof(unsigned long long));
    hctr_ = std::make_unique<PinnedBuf>(sizeof(Ctr));
    hsmall_ = std::make_unique<PinnedBuf>(small_.bytes);
    if (const char* d = getenv("MSBFS_DIRS")) dirs_ = d;  // per-level T/B override (tuning)
    if (const char* w = getenv("MSBFS_WIDE_LATER")) wide_later_ = atoi(w);
    if (const char* t = getenv("MSBFS_TILE")) tile_ = atoi(t);
    if (const char* h = getenv("MSBFS_HUBLDS")) hub_lds_ = atoi(h);
    if (const char* f = getenv("MSBFS_FUSE_COUNT")) fuse_count_ = atoi(f);
    if (const char* x = getenv("MSBFS_CODES")) codes_ = atoi(x);
    if (const char* x = getenv("MSBFS_LEAN")) lean_ = atoi(x);
    if (const char* x = getenv("MSBFS_LEAN_MIN")) lean_min_ = atoll(x);
    if (const char* x = getenv("MSBFS_LEAN_LEVEL")) lean_level_ = atoi(x);
    if (const char* x = getenv("MSBFS_FIRST")) first_on_ = atoi(x);

    if (const char* x = getenv("MSBFS_HUBBIG")) hub_big_ = atoi(x);
    if (const char* x = getenv("MSBFS_PFX")) pfx_ = atoi(x);
    if (const char* x = getenv("MSBFS_NARROW_C")) narrow_c_ = atoi(x);
    if (const char* x = getenv("MSBFS_COOP")) coop_ = atoi(x);
    if (const char* x = getenv("MSBFS_GAMMA")) gamma_ = atof(x);
    if (const char* x = getenv("MSBFS_GAMMA2")) gamma2_ = atof(x);
    if (const char* x = getenv("MSBFS_LAZY")) lazy_ = atoi(x);
    if (const char* x = getenv("MSBFS_TD_FUSED")) td_fused_ = atoi(x);
    if (const char* x = getenv("MSBFS_TD_BM")) td_bm_min_ = atoll(x);
    if (const char* x = getenv("MSBFS_TD_RED")) td_red_ = atoi(x);
    if (const char* x = getenv("MSBFS_ALPHA_LOW")) alpha_low_ = atof(x);
    if (const char* x = getenv("MSBFS_TD_FUSED_DEG")) td_fused_deg_ = atof(x);
    if (const char* x = getenv("MSBFS_TD_GRID"))
      td_grid_ = std::max(1, std::min(3 * kMaxGrid, atoi(x)));  // (slab rows)
    if (const char* x = getenv("MSBFS_AQ")) aq_ = atoi(x);
    if (const char* x = getenv("MSBFS_PFX_H")) pfx_h_ = atoi(x);
    if (const char* x = getenv("MSBFS_CODE_DEG")) code_deg_ = atof(x);
    if (const char* b = getenv("MSBFS_BATCH")) batch_levels_ = std::max(1, std::min(kBatch, atoi(b)));
    bctr_.alloc((size_t)(kBatch + 1) * (sizeof(Ctr) + 16 * sizeof(uint64_t)));
    hbctr_ = std::make_unique<PinnedBuf>((size_t)(kBatch + 1) * sizeof(Ctr));
    MSBFS_HIP_CHECK(hipDeviceSynchronize());
  }

  void run(int64_t K, const int64_t* qoff, const int32_t* qids, int64_t* F, int64_t* edges2,
           RunStats* st, hipStream_t stream) override {
    int64_t k0 = 0;
    while (k0 < K) {
      int64_t remain = K - k0;
      int w = 1;
      while (w * 64 < remain && w < std::min(maxW_, opt.max_words)) w <<= 1;
      const int64_t nb = std::min<int64_t>(remain, 64 * w);
      run_batch(w, k0, nb, qoff, qids, F + k0, edges2 ? edges2 + k0 : nullptr, st, stream);
      k0 += nb;
      if (st) st->batches++;
    }
  }

  int64_t hybrid_max_groups() const override { return 64 * (int64_t)maxW_; }

  void hybrid_phase_a(int64_t K, const int64_t* qoff, const int32_t* qids, int part, int nparts,
                      int64_t n_eff, bool count_l1, const int32_t* wbeg, uint64_t* send,
                      int64_t* out, RunStats* st, hipStream_t s,
                      int64_t* coded_len = nullptr) override {
    if (K < 1 || K > hybrid_max_groups())
      fail("hybrid mode: K=" + std::to_string(K) + " groups exceeds one round (" +
           std::to_string(hybrid_max_groups()) + ")");
    if (nparts < 1 || nparts > kMaxParts) fail("hybrid mode: 1..64 ranks");
    if (part < 0 || part >= nparts) fail("hybrid mode: bad part index");
    if (n_eff < this->n_eff() || n_eff > g_.n) fail("hybrid mode: bad vertex extent");
    const int wt = (int)((K + 63) / 64);
    if (wbeg[0] != 0 || wbeg[nparts] != wt) fail("hybrid mode: word split must cover ceil(K/64)");
    for (int j = 0; j < nparts; ++j)
      if (wbeg[j + 1] < wbeg[j]) fail("hybrid mode: word split not monotone");
    int w = 1;
    while (w < wt) w <<= 1;
#define MSBFS_BP_CASE(WW)                                                                  \
  case WW:                                                                                 \
    phase_a_impl<WW>(K, qoff, qids, part, nparts, n_eff, count_l1, wbeg, send, out, st, s, \
                     coded_len);                                                             \
    break;
    switch (w) {
      MSBFS_BP_CASE(1)
      MSBFS_BP_CASE(2)
      MSBFS_BP_CASE(4)
      MSBFS_BP_CASE(8)
      MSBFS_BP_CASE(16)
      default: fail("bad word count");
    }
#undef MSBFS_BP_CASE
    if (st) st->batches++;
  }

  void hybrid_phase_c(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                      const uint64_t* recv, const int64_t* reduced, int64_t* F_out, RunStats* st,
                      hipStream_t s) override {
    if (w_count <= 0) return;
    if (w_begin < 0 || (int64_t)(w_begin + w_count) * 64 - 63 > K || w_count > maxW_)
      fail("hybrid mode: bad word block");
    if (nparts < 1 || nparts > kMaxParts) fail("hybrid mode: 1..64 ranks");
    if (n_eff < this->n_eff() || n_eff > g_.n) fail("hybrid mode: bad vertex extent");
    int w = 1;
    while (w < w_count) w <<= 1;
#define MSBFS_BP_CASE(WW)                                                               \
  case WW:                                                                              \
    phase_c_impl<WW>(K, w_begin, w_count, nparts, n_eff, recv, reduced, F_out, st, s);  \
    break;
    switch (w) {
      MSBFS_BP_CASE(1)
      MSBFS_BP_CASE(2)
      MSBFS_BP_CASE(4)
      MSBFS_BP_CASE(8)
      MSBFS_BP_CASE(16)
      default: fail("bad word count");
    }
#undef MSBFS_BP_CASE
  }

 private:
  // Level-loop state. The normal path runs one batch start to finish; the hybrid phases run
  // a capped / range-restricted piece of it (phase A) or resume it from exchanged state (C).
  struct Loop {
    int cur = 0;  // vis_[cur] = read buffer (up to date for every non-done vertex)
    int fc = 0;   // fl_[fc] = current frontier
    int ac = 0;   // acc_[ac] holds the current frontier bits when fsrc_acc
    int alv = 0;  // alive[alv] = groups with a non-empty frontier
    uint32_t level = 0;
    int64_t nf = 0, ef = 0, ev = 0, na = 0, ea = 0, nact = 0, nactw = 0;
    bool have_active = false, fsrc_acc = true, bottom_up = false;
    int bu_levels = 0;
    // limits
    uint32_t stop_level = 0xFFFFFFFFu;  // last level to run
    int64_t cnt = 0;                    // first active-list build: v = part + i*nparts, i < cnt
    int part = 0, nparts = 1;
    bool weight_l1 = true;              // add level-1 counts to F
    std::string plan;                   // plan[level] = 'T'/'B' forces the next level
    int64_t ev_l1 = 0;                  // ev after level 1
    int64_t ef0 = 0;                    // degree sum of the sources (level-0 frontier)
    bool lazy = false;                  // no vis_[0] fill (see start_batch)
    bool osnap_next = false;            // the previous level was the first pull of a lazy batch
    bool lean_off = false;              // a lean first-row pass overflowed (see k_bu_first)
    bool lean_ran = false;              // this level ran one (its overflow count is c.touched)
    bool old_stale = false;             // k_td_fused levels updated only vis_[cur]
  };
  struct Small {
    unsigned long long* F;
    unsigned long long* E;
    uint64_t* alive[2];
    uint64_t* gmask;
  };
  Small small() {
    Small r;
    r.F = small_.as<unsigned long long>();
    r.E = r.F + 64 * 16;
    r.alive[0] = (uint64_t*)(r.E + 64 * 16);
    r.alive[1] = r.alive[0] + 16;
    r.gmask = r.alive[1] + 16;
    return r;
  }

  template <int W, bool COUNT>
  void start_batch(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids, Loop& S,
                   hipStream_t s);
  template <int W, bool COUNT>
  void levels(Loop& S, RunStats* st, hipStream_t s);
  template <int W, bool COUNT>
  void td_batch(Loop& S, RunStats* st, hipStream_t s);
  // device-driven top-down batches run k_td_fused levels (needs every row of vis_[cur] valid,
  // i.e. no lazy batch; the edge-counting pass keeps expand + finalize + k_count_frontier)
  double alpha_eff() const {
    return fused_batches<false>() ? std::min(opt.alpha, alpha_low_) : opt.alpha;
  }
  template <bool COUNT>
  bool fused_batches() const {
    return !COUNT && td_fused_ && batch_levels_ > 1 && g_.max_degree <= kSmallDeg &&
           (double)g_.nnz <= td_fused_deg_ * (double)std::max<int64_t>(g_.n, 1);
  }
  template <int W, bool COUNT>
  void batch_impl(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids, int64_t* F,
                  int64_t* edges2, RunStats* st, hipStream_t s);
  template <int W>
  void phase_a_impl(int64_t K, const int64_t* qoff, const int32_t* qids, int part, int nparts,
                    int64_t n_eff, bool count_l1, const int32_t* wbeg, uint64_t* send,
                    int64_t* out, RunStats* st, hipStream_t s,
                    int64_t* coded_len);
  template <int W>
  void phase_c_impl(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                    const uint64_t* recv, const int64_t* reduced, int64_t* F_out, RunStats* st,
                    hipStream_t s);

  void run_batch(int w, int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids,
                 int64_t* F, int64_t* edges2, RunStats* st, hipStream_t s) {
    const bool c = edges2 != nullptr || opt.count_edges;
#define MSBFS_BP_CASE(WW)                                                   \
  case WW:                                                                  \
    if (c) batch_impl<WW, true>(k0, nb, qoff, qids, F, edges2, st, s);      \
    else batch_impl<WW, false>(k0, nb, qoff, qids, F, edges2, st, s);       \
    break;
    switch (w) {
      MSBFS_BP_CASE(1)
      MSBFS_BP_CASE(2)
      MSBFS_BP_CASE(4)
      MSBFS_BP_CASE(8)
      MSBFS_BP_CASE(16)
      default: fail("bad word count");
    }
#undef MSBFS_BP_CASE
  }


  // 1 + the last vertex with deg > 0 (cached per graph buffers: relabelling replaces them).
  // Vertices beyond it are never active, never neighbours: level loops and clears skip them.
  int64_t n_eff() {
    if (eff_key_[0] != (const void*)g_.rowptr || eff_key_[1] != (const void*)g_.col ||
        eff_key_[2] != (const void*)g_.old2new) {
      n_eff_ = hybrid_extent(g_);
      eff_key_[0] = g_.rowptr;
      eff_key_[1] = g_.col;
      eff_key_[2] = g_.old2new;
    }
    return n_eff_;
  }

  // plen[v] = row prefix length with ids < H for every vertex (cached per graph buffers and H)
  const int32_t* prefix_lens(int32_t H, hipStream_t s) {
    if (plen_key_[0] != (const void*)g_.rowptr || plen_key_[1] != (const void*)g_.col ||
        plen_h_ != H) {
      plen_.ensure((size_t)std::max<int64_t>(g_.n, 1) * sizeof(int32_t));
      k_prefix_lens<<<grid_for(g_.n, kBlock, 8192), kBlock, 0, s>>>(g_.rowptr, g_.col, g_.n, H,
                                                                     plen_.as<int32_t>());
      MSBFS_HIP_CHECK(hipGetLastError());
      plen_key_[0] = g_.rowptr;
      plen_key_[1] = g_.col;
      plen_h_ = H;
    }
    return plen_.as<int32_t>();
  }

  // scratch of the exchange coding: bitmap words, popcounts and their inclusive scan per chunk
  struct CodeWs {
    uint64_t* bits;
    int64_t* pop;
    int64_t* incl;
    void* tmp;
    size_t tmp_bytes;
    uint64_t* dense;  // sender: the dense segments (dense_words)
  };
  CodeWs code_ws(int64_t chunks, int64_t dense_words = 0) {
    const size_t a = ((size_t)chunks * 8 + 255) & ~size_t(255);
    const size_t tb = (inclusive_scan_temp_bytes(chunks) + 255) & ~size_t(255);
    code_ws_.ensure(3 * a + tb + (size_t)dense_words * 8);
    char* p = (char*)code_ws_.p;
    return CodeWs{(uint64_t*)p, (int64_t*)(p + a), (int64_t*)(p + 2 * a), p + 3 * a, tb,
                  (uint64_t*)(p + 3 * a + tb)};
  }

  // zero-word coded send segments of phase A (see k_code_bits); coded_len[j] (host) = words of
  // destination j's segment
  template <int W>
  void code_send(const uint64_t* vis, int64_t cnt, int part, int nparts, const WordSplit& ws,
                 uint64_t* send, int64_t* coded_len, hipStream_t s) {
    CodeSegs cs{};
    int64_t c = 0, dn = 0;
    for (int j = 0; j < nparts; ++j) {
      cs.c0[j] = c;
      cs.len[j] = cnt * (ws.b[j + 1] - ws.b[j]);
      cs.dense[j] = dn;
      c += (cs.len[j] + 63) / 64;
      dn += cs.len[j];
    }
    cs.c0[nparts] = c;
    for (int j = 0; j < nparts; ++j) coded_len[j] = 0;
    if (c == 0) return;
    const CodeWs w = code_ws(c, dn);
    k_pack_words<W><<<grid_for(cnt * ws.b[nparts], kBlock, 8192), kBlock, 0, s>>>(
        vis, g_.rowptr, part, nparts, cnt, ws.b[nparts], ws, w.dense);
    MSBFS_HIP_CHECK(hipGetLastError());
    const int gc = grid_for((c + kCodeCPW - 1) / kCodeCPW * 64, kBlock, 1 << 20);
    k_code_bits<<<gc, kBlock, 0, s>>>(w.dense, cs, nparts, w.bits, w.pop);
    MSBFS_HIP_CHECK(hipGetLastError());
    inclusive_scan_i64(w.pop, w.incl, c, w.tmp, w.tmp_bytes, s);
    k_code_emit<<<gc, kBlock, 0, s>>>(w.dense, cs, nparts, w.bits, w.incl, send);
    MSBFS_HIP_CHECK(hipGetLastError());
    k_code_lens<<<1, 64, 0, s>>>(cs, nparts, w.bits, w.incl, w.pop);  // pop is free again
    MSBFS_HIP_CHECK(hipGetLastError());
    MSBFS_HIP_CHECK(hipMemcpyAsync(coded_len, w.pop, nparts * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }

  void hybrid_decode(const uint64_t* coded, const int64_t* coded_len, int nparts, int64_t n_eff,
                     int w_count, uint64_t* dense, hipStream_t s) override {
    if (nparts < 1 || nparts > kMaxParts) fail("hybrid mode: 1..64 ranks");
    if (w_count < 0 || w_count > maxW_) fail("hybrid mode: bad word block");
    CodeSegs cs{};
    int64_t c = 0, base = 0, dn = 0;
    for (int r = 0; r < nparts; ++r) {
      const int64_t L = part_count(n_eff, r, nparts) * w_count, nch = (L + 63) / 64;
      if (coded_len[r] < nch || coded_len[r] > L + nch)
        fail("hybrid decode: coded segment " + std::to_string(r) + " has " +
             std::to_string(coded_len[r]) + " words, outside [" + std::to_string(nch) + ", " +
             std::to_string(L + nch) + "]");
      cs.c0[r] = c;
      cs.len[r] = L;
      cs.base[r] = base;
      cs.dense[r] = dn;
      c += nch;
      base += coded_len[r];
      dn += L;
    }
    cs.c0[nparts] = c;
    if (c == 0) return;
    const CodeWs w = code_ws(c);
    k_decode_pop<<<grid_for(c, kBlock, 1 << 20), kBlock, 0, s>>>(coded, cs, nparts, w.pop);
    MSBFS_HIP_CHECK(hipGetLastError());
    inclusive_scan_i64(w.pop, w.incl, c, w.tmp, w.tmp_bytes, s);
    k_decode_emit<<<grid_for((c + kCodeCPW - 1) / kCodeCPW * 64, kBlock, 1 << 20), kBlock, 0,
                    s>>>(coded, cs, nparts, w.incl, dense);
    MSBFS_HIP_CHECK(hipGetLastError());
  }

  // first[v] for every vertex (cached per graph buffers like prefix_lens); nullptr when the
  // 4n bytes do not fit comfortably (RMAT-30) or MSBFS_FIRST=0: k_bu_first then reads col
  const int32_t* first_nbr(hipStream_t s) {
    if (!first_on_) return nullptr;
    if (first_key_[0] != (const void*)g_.rowptr || first_key_[1] != (const void*)g_.col) {
      const size_t bytes = (size_t)std::max<int64_t>(g_.n, 1) * sizeof(int32_t);
      if (first_.bytes < bytes) {
        size_t fr = 0, tot = 0;
        MSBFS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
        if (fr < bytes + ((size_t)2 << 30)) {
          first_on_ = 0;
          return nullptr;
        }
      }
      first_.ensure(bytes);
      k_first_nbr<<<grid_for(g_.n, kBlock, 8192), kBlock, 0, s>>>(g_.rowptr, g_.col, g_.n,
                                                                   first_.as<int32_t>());
      MSBFS_HIP_CHECK(hipGetLastError());
      first_key_[0] = g_.rowptr;
      first_key_[1] = g_.col;
    }
    return first_.as<int32_t>();
  }

  HostCtr read_ctr(hipStream_t s) {
    MSBFS_HIP_CHECK(hipMemcpyAsync(hctr_->p, ctr_.p, sizeof(Ctr), hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    const Ctr* c = hctr_->as<Ctr>();
    return HostCtr{c->act2.v, c->actw2.v, c->fl2.v, c->touched.v, c->ef2.v, c->eu2.v, c->ev2.v};
  }

  // copy the small block (F, E, alive, gmask) to pinned host memory and wait
  const unsigned long long* read_small(hipStream_t s) {
    MSBFS_HIP_CHECK(hipMemcpyAsync(hsmall_->p, small_.p, small_.bytes, hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    return hsmall_->as<unsigned long long>();
  }

  const DeviceGraph& g_;
  int maxW_ = 1;
  DevBuf vis_[2], acc_[2], stamp_, done_, act_[2], actw_[2], fl_[2], touched_, offs_, scan_tmp_,
      ctr_, small_, pairs_, slabF_, slabE_, anyvis_, desc_;
  double filter_frac_ = 0.5;  // skip unvisited neighbours while visited edges < frac * nnz
  double hub_bytes_ = 0.0;    // MSBFS_HUB_MB: hub rows loaded without the bitmap test (off: best)
  size_t scan_bytes_ = 0;
  std::unique_ptr<PinnedBuf> hctr_, hsmall_;
  int32_t epoch_ = 0;
  std::string dirs_;
  int wide_later_ = 1024;
  int tile_ = 256;
  int hub_lds_ = 3;  // bit 0: chunks kernel, bit 1: narrow kernel (MSBFS_HUBLDS)
  int fuse_count_ = 1;  // MSBFS_FUSE_COUNT=0: separate k_count_frontier pass
  int64_t n_eff_ = 0;
  const void* eff_key_[3] = {nullptr, nullptr, nullptr};
  // sparse row codes on the first bottom-up level (MSBFS_CODES=0: off); ids with degree >=
  // code_deg_ * nnz / (source degree sum), i.e. expected >= code_deg_ set bits, keep row gathers
  int codes_ = 1;
  // lean first pass on the third and later pull levels (see k_bu_first; MSBFS_LEAN=0: off).
  // RMAT-26, 1024 groups: level 4 2.48 -> 2.07 ms (98 % of its vertices finish on the first
  // row); on the second pull level most vertices overflow (128 groups: level 3 3.5 -> 4.1 ms)
  int lean_ = 1;
  int64_t lean_min_ = 1 << 20;  // MSBFS_LEAN_MIN: smallest active list for the lean pass
  int lean_level_ = 3;          // MSBFS_LEAN_LEVEL: first pull level (1-based) that may run it
  DevBuf plen_;
  DevBuf first_;
  DevBuf code_ws_;
  const void* first_key_[2] = {nullptr, nullptr};
  int first_on_ = 1;  // MSBFS_FIRST=0: no first-neighbour array (A/B knob)
  const void* plen_key_[2] = {nullptr, nullptr};
  int32_t plen_h_ = 0;
  // MSBFS_PFX: 0 = the first bottom-up level pulls whole rows (no tail push); 1 = prefix bound at
  // the 128-KB hub bitmap (ids < 1M, one chunk block per CU); 2 (default) = at the 56-KB one
  // (ids < 458752, two blocks per CU): RMAT-26 level 2 16.8 ms vs 18.1 (1) vs 21.2 (0)
  int pfx_ = 2;
  int32_t pfx_h_ = 0;  // MSBFS_PFX_H: lower prefix bound (tuning; smaller measured slower)
  int aq_ = 4096;       // MSBFS_AQ: vertices per block of the active-list build (4096 or 1024)
  int lazy_ = 1;        // MSBFS_LAZY=0: every batch fills vis_[0] (see start_batch)
  int td_fused_ = 1;    // MSBFS_TD_FUSED=0: device-driven batches use expand + finalize
  int64_t td_bm_min_ = 65536;  // MSBFS_TD_BM: k_td_fused walks the frontier bitmap from this nf
  DevBuf fbm_[2];       // frontier bitmaps of the fused levels (n bits each)
  int td_grid_ = 1024;  // MSBFS_TD_GRID: blocks of the device-driven batches' kernels
  int td_red_ = 6;      // MSBFS_TD_RED: fused levels per k_level_reduce_multi launch
  // MSBFS_TD_FUSED_DEG: fused levels only below this mean degree (road-like graphs). Denser
  // low-degree graphs pull after a few levels, and their first pull runs faster after lazy push
  // levels (uniform n = 16M, m = 128M, 1024 groups: 29.6 ms vs 32.3 ms with fused levels)
  double td_fused_deg_ = 8.0;
  // MSBFS_ALPHA_LOW: push -> pull threshold (Beamer's alpha) on graphs with max degree <= kSmallDeg
  // (fused top-down levels). Road grid 4896^2, 256 groups: alpha 14 pulls from ~1.7M frontier
  // vertices on and takes 3030 ms, alpha 4 stays top-down (1648 ms batched); 1024 groups still pull
  // (8.8 s vs 12.5 s top-down only); uniform n = 16M, m = 128M, 1024 groups: pulls from level 2
  double alpha_low_ = 4.0;
  DevBuf asnap_;        // any-visited bitmap at the start of a lazy batch's first pull level
  double gamma_ = 1.0;  // MSBFS_GAMMA: push -> pull once frontier edges > gamma * n_eff
  // MSBFS_GAMMA2: the same test for level 2 (< 0: gamma_). Lower, because only level 2 can pull
  // with prefix pull + tail push: a push level 2 makes level 3 the first pull, which scans whole
  // rows (RMAT-30, 16 groups: level 3 277 ms; 296 -> 106 ms/step; RMAT-26, 4 groups 15.5 -> 8.7)
  double gamma2_ = 0.25;
  int coop_ = -1;      // MSBFS_COOP: cross-chunk early exit on the first pull level (-1 auto)
  int narrow_c_ = 2;   // MSBFS_NARROW_C: short first narrow step (0 off, 1 always, 2 by level)
  int hub_big_ = 3;  // MSBFS_HUBBIG: bit 0 narrow, bit 1 chunks use a 128-KB LDS hub bitmap
  double code_deg_ = 3.0;  // (3-slot codes: 6.58 ms level-2 chunk pulls vs 6.69 at 2.0, 6.62 at 4.0)
  std::map<int64_t, int32_t> code_bound_;
  const void* code_key_[2] = {nullptr, nullptr};
  // first id with degree < min_deg (rounded to a power of two, cached per graph); 0 when the
  // graph keeps the user's ids (no degree order to exploit)
  int32_t code_bound(double min_deg) {
    if (!g_.old2new) return 0;
    if (code_key_[0] != (const void*)g_.rowptr || code_key_[1] != (const void*)g_.col) {
      code_bound_.clear();
      code_key_[0] = g_.rowptr;
      code_key_[1] = g_.col;
    }
    int64_t d = 1;
    while (d < (int64_t)min_deg && d < ((int64_t)1 << 40)) d <<= 1;
    auto it = code_bound_.find(d);
    if (it != code_bound_.end()) return it->second;
    DevBuf b;
    b.alloc(sizeof(int32_t));
    k_degree_bound<<<1, 1>>>(g_.rowptr, g_.n, d, b.as<int32_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
    int32_t h = 0;
    MSBFS_HIP_CHECK(hipMemcpy(&h, b.p, sizeof(h), hipMemcpyDeviceToHost));
    code_bound_[d] = h;
    return h;
  }
  // device-driven top-down level batches (low-degree graphs): up to kBatch levels per host
  // round trip, doubling from 4 while the frontier lives (MSBFS_BATCH=1 turns them off)
  static constexpr int kBatch = 64;
  int batch_levels_ = kBatch;
  int batch_next_ = 4;
  DevBuf bctr_;  // (kBatch+1) Ctr slots, then (kBatch+1) x 16 alive words
  std::unique_ptr<PinnedBuf> hbctr_;
};

// per-batch reset + sources + level 0 (k_init); leaves the loop state ready for level 1
template <int W, bool COUNT>
void BitparSolver::start_batch(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids,
                               Loop& S, hipStream_t s) {
  const int64_t n = g_.n;
  // Rows of vertices >= n_eff (deg 0) are never read: only sources can be there, and their rows
  // are zeroed by k_zero_src_rows. vis_[1]: see k_zero_src_rows.
  const size_t vb = (size_t)std::max<int64_t>(n_eff(), 1) * W * sizeof(uint64_t);
  if (!S.lazy) MSBFS_HIP_CHECK(hipMemsetAsync(vis_[0].p, 0, vb, s));
  else if (S.cnt > 0 && S.nparts > 1)  // hybrid phase A: only the rows levels 1-2 read (see k_zero_part_rows)
    k_zero_part_rows<W><<<grid_for(S.cnt * Lay<W>::G, kBlock, 8192), kBlock, 0, s>>>(
        S.cnt, S.part, S.nparts, vis_[0].as<uint64_t>());
  MSBFS_HIP_CHECK(hipMemsetAsync(done_.p, 0, done_.bytes, s));
  MSBFS_HIP_CHECK(hipMemsetAsync(anyvis_.p, 0, anyvis_.bytes, s));
  MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
  MSBFS_HIP_CHECK(hipMemsetAsync(small_.p, 0, small_.bytes, s));
  const Small sm = small();
  // ---- sources: (vertex, local group) pairs, out-of-range ids dropped (main.cu:49)
  std::vector<int32_t> hp, hk;
  hp.reserve(2 * (qoff[k0 + nb] - qoff[k0]));
  for (int64_t k = 0; k < nb; ++k)
    for (int64_t j = qoff[k0 + k]; j < qoff[k0 + k + 1]; ++j) {
      const int32_t v = qids[j];
      if (v >= 0 && v < n) {
        hp.push_back(v);
        hk.push_back((int32_t)k);
      }
    }
  const int64_t np = (int64_t)hp.size();
  {
    // gmask = the batch's groups; alive = groups with at least one valid source (computed here:
    // an atomicOr per source pair onto 16 words serialised k_init, ~0.1 ms per batch)
    uint64_t hm[2][16] = {{0}};
    for (int64_t k = 0; k < nb; ++k) hm[0][k >> 6] |= 1ull << (k & 63);
    for (int64_t i = 0; i < np; ++i) hm[1][hk[i] >> 6] |= 1ull << (hk[i] & 63);
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.gmask, hm[0], sizeof(hm[0]), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[0], hm[1], sizeof(hm[1]), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));  // hm is a stack buffer
  }
  pairs_.ensure((size_t)std::max<int64_t>(np, 1) * 2 * sizeof(int32_t));
  int32_t* dpv = pairs_.as<int32_t>();
  int32_t* dpk = dpv + std::max<int64_t>(np, 1);
  hp.insert(hp.end(), hk.begin(), hk.end());
  if (np) {
    MSBFS_HIP_CHECK(hipMemcpyAsync(dpv, hp.data(), np * sizeof(int32_t), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipMemcpyAsync(dpk, hp.data() + np, np * sizeof(int32_t),
                                   hipMemcpyHostToDevice, s));
  }
  ++epoch_;
  if (np) {
    k_zero_src_rows<W><<<grid_for(np * W, kBlock), kBlock, 0, s>>>(
        dpv, np, g_.old2new, vis_[0].as<uint64_t>(), vis_[1].as<uint64_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
    k_init<W, COUNT><<<grid_for(np, kBlock), kBlock, 0, s>>>(
        dpv, dpk, np, g_.rowptr, vis_[0].as<uint64_t>(), vis_[1].as<uint64_t>(),
        acc_[S.ac].as<uint64_t>(), stamp_.as<int32_t>(), epoch_, fl_[S.fc].as<int32_t>(),
        ctr_.as<Ctr>(), sm.E, sm.alive[0], anyvis_.as<uint32_t>(), g_.old2new);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  const HostCtr c = read_ctr(s);  // also retires the pinned/host source copies
  S.nf = c.fl2;
  S.ef = (int64_t)c.ef2;
  S.ef0 = S.ef;
  S.ev = (int64_t)c.ev2;
  S.na = n;
  S.ea = g_.nnz;  // active estimate before the first bottom-up build
}

template <int W, bool COUNT>
void BitparSolver::levels(Loop& S, RunStats* st, hipStream_t s) {
  using L = Lay<W>;
  const int64_t n = g_.n;
  const Small sm = small();
  const int grid = kMaxGrid;
  static const bool trace = getenv("MSBFS_TRACE") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  HostCtr c{};
  while (S.nf > 0 && S.level < S.stop_level) {
    // direction choice (Beamer et al. SC'12, on the union frontier)
    bool& bottom_up = S.bottom_up;
    if (opt.force_dir == 1) bottom_up = false;
    else if (opt.force_dir == 2) bottom_up = S.level > 0;
    else if (!bottom_up)
      // Beamer's edge test, plus a vertex test: a pull level costs about one visit per
      // non-isolated vertex (prefix pulls, early exit), a push level one scattered atomic per
      // frontier edge, so pull once the frontier has more edges than the graph has vertices
      // (RMAT-30, 256 groups: 742 -> 294 ms/step; RMAT-26, 16 groups: 16.4 -> 9.3 ms; road
      // graphs never get there). MSBFS_GAMMA scales the vertex test (0 turns it off).
      bottom_up = (double)S.ef > (double)S.ea / alpha_eff() ||
                  (gamma_ > 0 && S.level >= 1 &&
                   (double)S.ef > (S.level == 1 && gamma2_ >= 0 ? gamma2_ : gamma_) *
                                      (double)n_eff());
    else bottom_up = !((double)S.nf < (double)S.na / opt.beta && (double)S.ef < (double)S.ea / alpha_eff());
    if (S.level < dirs_.size() && (dirs_[S.level] == 'T' || dirs_[S.level] == 'B'))
      bottom_up = dirs_[S.level] == 'B';
    if (S.level < S.plan.size() && (S.plan[S.level] == 'T' || S.plan[S.level] == 'B'))
      bottom_up = S.plan[S.level] == 'B';
    // low-degree graphs (road-like: thousands of small top-down levels): run a batch of levels
    // without host round trips (kernels read the frontier sizes from device counters)
    if (!bottom_up && batch_levels_ > 1 && g_.max_degree <= kSmallDeg && !trace &&
        S.level + 2 < S.stop_level && opt.force_dir != 2 && S.plan.empty() &&
        (dirs_.size() <= S.level)) {
      td_batch<W, COUNT>(S, st, s);
      tl = std::chrono::steady_clock::now();
      continue;
    }
    MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
    MSBFS_HIP_CHECK(hipMemsetAsync(sm.alive[S.alv ^ 1], 0, 16 * sizeof(uint64_t), s));
    ++S.level;
    trace::Range range_level(bottom_up ? "bitpar L%u BU" : "bitpar L%u TD", S.level);
    int rows = 0;  // slab rows written by this level's counting kernels
    auto slabF = [&](int r) { return slabF_.as<uint32_t>() + (size_t)r * 64 * W; };
    auto slabE = [&](int r) { return slabE_.as<unsigned long long>() + (size_t)r * 64 * W; };
    uint64_t* R = vis_[S.cur].as<uint64_t>();
    uint64_t* O = vis_[S.cur ^ 1].as<uint64_t>();
    const uint64_t* alive = sm.alive[S.alv];
    if (!bottom_up) {
      // ---- top-down
      ++epoch_;
      const uint32_t* lzv = S.lazy ? anyvis_.as<uint32_t>() : nullptr;  // see k_zero_part_rows
      if (g_.max_degree <= kSmallDeg) {
        // low-degree graph: vertex-parallel expansion, no degree scan
        const int eg = grid_for(S.nf, L::TILE, 4096);
        if (S.fsrc_acc)
          k_td_expand_small<W, false><<<eg, kBlock, 0, s>>>(
              fl_[S.fc].as<int32_t>(), S.nf, nullptr, g_.rowptr, g_.col, R,
              acc_[S.ac].as<uint64_t>(),
              done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
              touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv);
        else
          k_td_expand_small<W, true><<<eg, kBlock, 0, s>>>(
              fl_[S.fc].as<int32_t>(), S.nf, nullptr, g_.rowptr, g_.col, R, O,
              done_.as<uint32_t>(),
              acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
              touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv,
              S.osnap_next ? asnap_.as<uint32_t>() : nullptr);
      } else {
      frontier_degree_scan(g_.rowptr, fl_[S.fc].as<int32_t>(), S.nf, offs_.as<int64_t>(),
                           scan_tmp_.p, scan_bytes_, s);
      const int eg = grid_for(S.ef, L::TILE, 8192);
      if (S.fsrc_acc)
        k_td_expand<W, false><<<eg, kBlock, 0, s>>>(
            fl_[S.fc].as<int32_t>(), S.nf, offs_.as<int64_t>(), g_.rowptr, g_.col, R,
            acc_[S.ac].as<uint64_t>(), done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(),
            stamp_.as<int32_t>(), epoch_, touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv);
      else
        k_td_expand<W, true><<<eg, kBlock, 0, s>>>(
            fl_[S.fc].as<int32_t>(), S.nf, offs_.as<int64_t>(), g_.rowptr, g_.col, R, O,
            done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
            touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv,
            S.osnap_next ? asnap_.as<uint32_t>() : nullptr);
      }
      MSBFS_HIP_CHECK(hipGetLastError());
      // touched <= min(n, frontier edges); the kernel reads the exact count from ctr
      const int64_t nt_max = std::min<int64_t>(std::max<int64_t>(S.ef, S.nf), n);
      const int gf = grid_for(nt_max, L::TILE, grid);
      constexpr bool FUSE = !COUNT;
      const bool fuse = FUSE && fuse_count_;
      auto kf = fuse ? k_td_finalize<W, COUNT, FUSE> : k_td_finalize<W, COUNT, false>;
      kf<<<gf, kBlock, 0, s>>>(
          touched_.as<int32_t>(), g_.rowptr, R, O, acc_[S.ac ^ 1].as<uint64_t>(), alive,
          sm.gmask, done_.as<uint32_t>(), fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
          fl_[S.fc].as<int32_t>(), S.nf, nullptr,
          S.fsrc_acc ? acc_[S.ac].as<uint64_t>() : nullptr, anyvis_.as<uint32_t>(), slabF(rows),
          S.lazy ? 1 : 0, nullptr);
      MSBFS_HIP_CHECK(hipGetLastError());
      if (fuse) {
        rows += gf;
      } else {
        // new frontier bits are in acc_[ac ^ 1]
        const int gc = grid_for(nt_max, L::TILE, grid);
        k_count_frontier<W, COUNT, false><<<gc, kBlock, 0, s>>>(
            fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(), g_.rowptr, acc_[S.ac ^ 1].as<uint64_t>(),
            nullptr, slabF(rows), slabE(rows));
        rows += gc;
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      S.ac ^= 1;
      S.fsrc_acc = true;
      S.osnap_next = false;
      if (st) st->td_levels++;
    } else {
      // ---- bottom-up
      if (S.old_stale) {
        // fused top-down levels wrote only vis_[cur]; pulls write the other buffer's rows of the
        // active vertices and read both buffers' rows of the finished ones afterwards
        const size_t vb = (size_t)std::max<int64_t>(n_eff(), 1) * W * sizeof(uint64_t);
        MSBFS_HIP_CHECK(hipMemcpyAsync(O, R, vb, hipMemcpyDeviceToDevice, s));
        S.old_stale = false;
      }
      const int next_wide = std::max(opt.wide_degree, wide_later_);
      if (!S.have_active) {
        // after the first bottom-up level most vertices exit early: a whole wave per chunk pays
        // off only for much higher degrees, so later lists are split at a higher threshold
        const int wide0 = S.bu_levels == 0 ? opt.wide_degree : next_wide;
        auto kb = aq_ == 1024 ? k_build_active<1024> : k_build_active<4096>;
        kb<<<grid_for(S.cnt, aq_ == 1024 ? 1024 : 4096, INT32_MAX), kBlock, 0, s>>>(
            S.cnt, S.part, S.nparts, g_.rowptr, done_.as<uint32_t>(), wide0, act_[0].as<int32_t>(),
            actw_[0].as<int32_t>(), ctr_.as<Ctr>());
        MSBFS_HIP_CHECK(hipGetLastError());
        c = read_ctr(s);
        S.nact = c.act2;
        S.nactw = c.actw2;
        S.have_active = true;
        MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
      }
      const bool first_bu = S.bu_levels == 0;
      ++S.bu_levels;
      if (S.fsrc_acc) {
        // bottom-up does not read frontier bits; clear the pending top-down ones so acc_[ac]
        // is all-zero and can collect the wide vertices' chunk results
        k_zero_acc<W><<<grid_for(S.nf * L::G, kBlock), kBlock, 0, s>>>(
            fl_[S.fc].as<int32_t>(), S.nf, acc_[S.ac].as<uint64_t>());
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      // lazy batch, first pull level: rows of vertices nobody visited yet may be stale, so every
      // gathered row must be one of a visited vertex (always filter), and probes / own rows use a
      // snapshot of the any-visited bitmap (a vertex first visited during the level may be
      // probed before its row is written). From the next pull level on the read buffer holds
      // this level's rows, valid for every vertex a pull can reach (see start_batch).
      const bool lazy_first = S.lazy && first_bu;
      const uint32_t* snap = nullptr;
      if (lazy_first) {
        MSBFS_HIP_CHECK(hipMemcpyAsync(asnap_.p, anyvis_.p, anyvis_.bytes, hipMemcpyDeviceToDevice, s));
        snap = asnap_.as<uint32_t>();
      }
      const bool filter = lazy_first || (double)S.ev < filter_frac_ * (double)g_.nnz;
      // hub rows (lowest ids after degree relabelling) sized to ~hub_bytes_ are always loaded
      const int64_t hub_ids = g_.old2new && !S.lazy ? (int64_t)(hub_bytes_ / (8.0 * W)) : 0;
      const int32_t filter_from =
          filter ? (int32_t)std::min<int64_t>(hub_ids, INT32_MAX) : INT32_MAX;
      constexpr int kHubW = 14336;  // 56 KB of LDS: ids < 458752
      const bool hub_lds = hub_lds_ && filter_from == 0 && n > (int64_t)kHubW * 32 * 4;
      // counting fused into the traversal kernels (the edge-count pass keeps k_count_frontier)
      constexpr bool FUSE = !COUNT;
      const bool fuse = FUSE && fuse_count_;
      // prefix pull + tail push on the first bottom-up level (see k_push_tail): both pulls use
      // the 128-KB hub bitmap, whose range [0, H) is where the prefixes end
      constexpr int kHubBig = 32768;
      // MSBFS_PFX=2: prefix bound at the small hub bitmap (ids < 458752, two chunk blocks per CU,
      // more tail pushes); 1: at the big one (ids < 1M)
      const bool pfx_small = pfx_ == 2;
      int32_t kPfxH = (pfx_small ? kHubW : kHubBig) * 32;
      if (pfx_h_ > 0) kPfxH = std::min(kPfxH, pfx_h_);  // MSBFS_PFX_H: a lower bound (tuning)
      const bool pfx = pfx_ && first_bu && S.level == 2 && hub_lds && (hub_lds_ & 3) == 3 &&
                       (pfx_small || (hub_big_ & 3) == 3) && n > (int64_t)kHubBig * 32 * 4 &&
                       g_.rows_sorted && n <= INT32_MAX;
      // sparse row codes for the first bottom-up level after level 1 (see k_build_codes). With
      // the prefix pull only ids < H and the tail pushers' own codes are ever read: the codes of
      // [code_from, H) plus those of the frontier vertices >= H (not 4 bytes for every id).
      int32_t code_from = kNoCodes;
      const uint32_t* codes = nullptr;
      if (first_bu && S.level == 2 && codes_ && W >= 8 && S.ef0 > 0 && n <= INT32_MAX) {
        const int64_t ne = n_eff();
        code_from = (int32_t)std::min<int64_t>(
            code_bound(code_deg_ * (double)g_.nnz / (double)S.ef0), ne);
        if (code_from < ne) {
          uint32_t* cb = touched_.as<uint32_t>();  // n entries
          const int64_t hi = pfx ? std::min<int64_t>(std::max<int64_t>(kPfxH, code_from), ne) : ne;
          const int64_t nl = pfx ? S.nf : 0;
          k_build_codes<W><<<grid_for(hi - code_from + nl, kBlock, 8192), kBlock, 0, s>>>(
              R, anyvis_.as<uint32_t>(), code_from, hi, fl_[S.fc].as<int32_t>(), nl, cb);
          MSBFS_HIP_CHECK(hipGetLastError());
          codes = cb;
        } else {
          code_from = kNoCodes;
        }
      }
      const int32_t* plen = pfx ? prefix_lens(kPfxH, s) : nullptr;
      if (pfx) {
        ++epoch_;
        k_push_tail<W><<<grid_for(S.nf * 64, kBlock, 8192), kBlock, 0, s>>>(
            fl_[S.fc].as<int32_t>(), S.nf, kPfxH, g_.rowptr, g_.col, R, codes, code_from,
            done_.as<uint32_t>(), S.part, S.nparts, acc_[S.ac].as<uint64_t>(),
            stamp_.as<int32_t>(), epoch_);
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      if (S.nact) {
        if (pfx) {
          constexpr int BT = 1024;
          const int gn = grid_for(S.nact, (BT / 64) * L::VPW, 512);
          // 4-neighbour steps: 122 VGPRs, no spills (8-neighbour steps spilled at the 128-VGPR
          // bound): RMAT-26 5.17 -> 4.96 ms (the full pulls of level 3 keep 8: 5.8 vs 6.8 ms)
          auto kn = fuse ? (pfx_small ? k_bu_narrow<W, COUNT, BT, kHubW, FUSE, true, true, 4>
                                      : k_bu_narrow<W, COUNT, BT, kHubBig, FUSE, true, true>)
                         : (pfx_small ? k_bu_narrow<W, COUNT, BT, kHubW, false, true, true>
                                      : k_bu_narrow<W, COUNT, BT, kHubBig, false, true, true>);
          kn<<<gn, BT, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive,
                               sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                               fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
                               anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                               next_wide, slabF(rows), acc_[S.ac].as<uint64_t>(),
                               stamp_.as<int32_t>(), epoch_, plen, nullptr, snap);
          if (fuse) rows += gn;
        } else if (hub_lds && (hub_lds_ & 2)) {
          constexpr int BT = 1024;
          const int gn = grid_for(S.nact, (BT / 64) * L::VPW, 512);
          // the narrow kernel runs one 1024-thread block per CU anyway (VGPR-bound), so its LDS
          // has room for a 4x larger hub bitmap (MSBFS_HUBBIG bit 0)
          const bool big = (hub_big_ & 1) && n > (int64_t)kHubBig * 32 * 4;
          auto kn = fuse ? (big ? k_bu_narrow<W, COUNT, BT, kHubBig, FUSE>
                                : k_bu_narrow<W, COUNT, BT, kHubW, FUSE>)
                         : (big ? k_bu_narrow<W, COUNT, BT, kHubBig, false>
                                : k_bu_narrow<W, COUNT, BT, kHubW, false>);
          kn<<<gn, BT, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive,
                               sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                               fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
                               anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                               next_wide, slabF(rows), nullptr, nullptr, 0, nullptr, nullptr, snap);
          if (fuse) rows += gn;
        } else {
          const int gn = grid_for(S.nact, L::TILE, grid);
          // FILT = false: no probe code at all (fewer VGPRs) on the levels that load every row
          const bool filt = filter_from != INT32_MAX;
          // short first step (one row) from the third bottom-up level on, or with few words: by
          // then most vertices are covered by their first neighbour (RMAT-26, 1024 groups: level
          // 4 3.1 -> 2.5 ms; level 3 prefers full steps: 6.5 vs 6.7 ms). MSBFS_NARROW_C: 0 off,
          // 1 always, 2 (default) this rule
          const bool short1 = narrow_c_ == 1 || (narrow_c_ == 2 && (S.bu_levels >= 3 || W <= 4));
          if (lean_ && !S.lean_off && fuse && !filt && S.bu_levels >= lean_level_ &&
              S.nact >= lean_min_) {
            S.lean_ran = true;
            // lean first pass, then the regular pull over the vertices it could not finish
            const int gl = grid_for(S.nact, L::TILE, grid);
            k_bu_first<W><<<gl, kBlock, 0, s>>>(
                act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive, sm.gmask,
                done_.as<uint32_t>(), touched_.as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
                ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), slabF(rows), first_nbr(s));
            MSBFS_HIP_CHECK(hipGetLastError());
            rows += gl;
            k_bu_narrow<W, COUNT, kBlock, 0, FUSE, false, false, 8, 1><<<gn, kBlock, 0, s>>>(
                touched_.as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive, sm.gmask,
                done_.as<uint32_t>(), act_[1].as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
                ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                next_wide, slabF(rows), nullptr, nullptr, 0, nullptr, &ctr_.as<Ctr>()->touched.v,
                nullptr);
            MSBFS_HIP_CHECK(hipGetLastError());
            rows += gn;
          } else {
          auto kn = fuse ? (filt ? k_bu_narrow<W, COUNT, kBlock, 0, FUSE, true>
                                 : short1 ? k_bu_narrow<W, COUNT, kBlock, 0, FUSE, false, false, 8, 1>
                                          : k_bu_narrow<W, COUNT, kBlock, 0, FUSE, false>)
                         : (filt ? k_bu_narrow<W, COUNT, kBlock, 0, false, true>
                                 : k_bu_narrow<W, COUNT, kBlock, 0, false, false>);
          kn<<<gn, kBlock, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive,
                                   sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                                   fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
                                   anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                                   next_wide, slabF(rows), nullptr, nullptr, 0, nullptr, nullptr, snap);
          if (fuse) rows += gn;
          }
        }
        MSBFS_HIP_CHECK(hipGetLastError());
      }
      if (S.nactw) {
        if (pfx) {  // chunks of the row prefixes with ids < H only
          int64_t* cnt = scan_tmp_.as<int64_t>();
          char* t2 = (char*)scan_tmp_.p + (((size_t)S.nactw * sizeof(int64_t) + 255) & ~size_t(255));
          const size_t tb = scan_bytes_ - (size_t)(t2 - (char*)scan_tmp_.p);
          k_prefix_chunks<<<grid_for(S.nactw, kBlock), kBlock, 0, s>>>(
              actw_[0].as<int32_t>(), S.nactw, plen, cnt);
          MSBFS_HIP_CHECK(hipGetLastError());
          inclusive_scan_i64(cnt, offs_.as<int64_t>(), S.nactw, t2, tb, s);
        } else {
          frontier_degree_scan(g_.rowptr, actw_[0].as<int32_t>(), S.nactw, offs_.as<int64_t>(),
                               scan_tmp_.p, scan_bytes_, s, kChunk);
        }
        const int64_t chunks_max = S.nactw + S.ea / kChunk + 1;
        // Early exit across a vertex's chunks (coop) everywhere except on an explosive first
        // bottom-up level (level 2: hardly any row gets covered, and round-robin chunk dealing
        // balances the hubs better). When top-down ran longer (RMAT-30: first pull at level 3,
        // most of every hub's groups already visited) the early exit skips most chunks.
        // MSBFS_COOP: 1 always, 0 = never on the first bottom-up level (the old rule).
        const int coop = !first_bu ? 1 : coop_ == 1 ? 1 : coop_ == 0 ? 0 : (S.level == 2 ? 0 : 1);
        desc_.ensure((size_t)chunks_max * sizeof(ChunkDesc));
        k_chunk_desc<<<grid_for(S.nactw, kBlock), kBlock, 0, s>>>(
            actw_[0].as<int32_t>(), S.nactw, offs_.as<int64_t>(), g_.rowptr, plen,
            desc_.as<ChunkDesc>());
        MSBFS_HIP_CHECK(hipGetLastError());
        if (hub_lds && (hub_lds_ & 1)) {
          // exact chunk count = offs[nactw - 1], read on the device (no host round trip)
          // MSBFS_HUBBIG bit 1: one block per CU with a 128-KB hub bitmap (ids < 1M)
          const bool big = (hub_big_ & 2) && n > (int64_t)kHubBig * 32 * 4 && !(pfx && pfx_small);
          auto ck = big ? k_bu_chunks<W, 256, 1024, kHubBig> : k_bu_chunks<W, 256, 1024, kHubW>;
          ck<<<grid_for(chunks_max, 16, big ? 256 : 512), 1024, 0, s>>>(
              desc_.as<ChunkDesc>(), offs_.as<int64_t>() + S.nactw - 1, g_.col, R, alive,
              sm.gmask, acc_[S.ac].as<uint64_t>(), anyvis_.as<uint32_t>(), filter_from,
              coop, codes, code_from, snap);
        } else {
          auto ck = tile_ >= 1024 ? k_bu_chunks<W, 1024, kBlock, 0>
                    : tile_ >= 512 ? k_bu_chunks<W, 512, kBlock, 0> : k_bu_chunks<W, 256, kBlock, 0>;
          ck<<<grid_for(chunks_max, kWaves, 8192), kBlock, 0, s>>>(
              desc_.as<ChunkDesc>(), offs_.as<int64_t>() + S.nactw - 1, g_.col, R, alive, sm.gmask, acc_[S.ac].as<uint64_t>(),
              anyvis_.as<uint32_t>(), filter_from, coop, codes, code_from, snap);
        }
        MSBFS_HIP_CHECK(hipGetLastError());
        const int gw = grid_for(S.nactw, L::TILE, grid);
        auto kf = fuse ? k_bu_wide_finalize<W, COUNT, FUSE> : k_bu_wide_finalize<W, COUNT, false>;
        kf<<<gw, kBlock, 0, s>>>(
            actw_[0].as<int32_t>(), S.nactw, g_.rowptr, R, O, acc_[S.ac].as<uint64_t>(), alive,
            sm.gmask, done_.as<uint32_t>(), actw_[1].as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
            ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), act_[1].as<int32_t>(), next_wide,
            slabF(rows), snap);
        MSBFS_HIP_CHECK(hipGetLastError());
        if (fuse) rows += gw;
      }
      if (!fuse) {
        // new frontier bits = Wb & ~R (both still in place: the swap is below)
        const int gc = grid_for(S.nact + S.nactw, L::TILE, grid);
        k_count_frontier<W, COUNT, true><<<gc, kBlock, 0, s>>>(
            fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(), g_.rowptr, O, R, slabF(rows),
            slabE(rows));
        MSBFS_HIP_CHECK(hipGetLastError());
        rows += gc;
      }
      std::swap(act_[0], act_[1]);
      std::swap(actw_[0], actw_[1]);
      S.cur ^= 1;
      S.fsrc_acc = false;
      S.osnap_next = lazy_first;
      if (st) st->bu_levels++;
    }
    if (rows) {
      const int rg = std::max(1, std::min(64, rows / 32));
      const uint32_t weight = (S.level == 1 && !S.weight_l1) ? 0u : S.level;
      k_level_reduce<W, COUNT><<<W * rg, kBlock, 0, s>>>(slabF(0), slabE(0), rows, rg, sm.F, sm.E,
                                                         sm.alive[S.alv ^ 1], weight);
      MSBFS_HIP_CHECK(hipGetLastError());
    }
    c = read_ctr(s);
    if (S.lean_ran) {
      // (high-diameter graphs: most vertices need more than their first neighbour; once a lean
      // pass sends over a quarter of its vertices on, the batch keeps the regular pull)
      if ((int64_t)c.touched * 4 > S.nact) S.lean_off = true;
      S.lean_ran = false;
    }
    if (bottom_up) {
      S.nact = c.act2;
      S.nactw = c.actw2;
      S.na = S.nact + S.nactw;
      S.ea = (int64_t)c.eu2;
    }
    const auto t2 = std::chrono::steady_clock::now();
    const double lms = std::chrono::duration<double, std::milli>(t2 - tl).count();
    if (st) {
      LevelRec rec;
      rec.batch = (int32_t)st->batches;
      rec.level = (int32_t)S.level;
      rec.dir = bottom_up ? 'B' : 'T';
      rec.nf = S.nf;
      rec.ef = S.ef;
      rec.nf_next = (int64_t)c.fl2;
      rec.active = bottom_up ? S.na : (int64_t)c.touched;
      rec.ms = lms;
      st->recs.push_back(rec);
    }
    if (trace) {
      fprintf(stderr,
              "[msbfs bp W=%d] level %u %s nf=%lld ef=%lld -> nf'=%lld ef'=%lld touched=%u "
              "active=%lld (wide %lld) ea=%lld ev=%lld  %.3f ms\n",
              W, S.level, bottom_up ? "BU" : "TD", (long long)S.nf, (long long)S.ef,
              (long long)c.fl2, (long long)c.ef2, c.touched, (long long)S.na, (long long)S.nactw,
              (long long)S.ea, (long long)(S.ev + (long long)c.ev2), lms);
    }
    tl = t2;
    S.nf = c.fl2;
    S.ef = (int64_t)c.ef2;
    S.ev += (int64_t)c.ev2;
    if (S.level == 1) S.ev_l1 = S.ev;
    S.fc ^= 1;
    S.alv ^= 1;
    if (st) st->levels++;
  }
}

// A batch of up to batch_next_ top-down levels with no host synchronisation: level i of the
// batch reads its frontier size from counter slot i (slot 0 seeded from the host) and writes
// slot i + 1; alive masks likewise. Levels after the frontier dies are no-ops (every kernel
// sees a zero count). One copy of all slots afterwards restores the host's view.
template <int W, bool COUNT>
void BitparSolver::td_batch(Loop& S, RunStats* st, hipStream_t s) {
  using L = Lay<W>;
  const int64_t n = g_.n;
  const Small sm = small();
  int K = std::min<int>(batch_next_, batch_levels_);
  if (S.stop_level != 0xFFFFFFFFu) K = std::min<int64_t>(K, (int64_t)S.stop_level - S.level);
  K = std::max(K, 1);
  Ctr* slots = bctr_.as<Ctr>();
  uint64_t* aslot = (uint64_t*)(slots + kBatch + 1);
  MSBFS_HIP_CHECK(hipMemsetAsync(bctr_.p, 0, bctr_.bytes, s));
  const int64_t nwords = (n_eff() + 31) / 32;
  if (fused_batches<COUNT>()) {
    // the batch's first level reads the host's list; later ones may walk the bitmap its
    // predecessor wrote (levels outside the batch leave stale bits: start from zero)
    for (auto& b : fbm_) {
      b.ensure((size_t)std::max<int64_t>(nwords, 1) * sizeof(uint32_t));
      MSBFS_HIP_CHECK(hipMemsetAsync(b.p, 0, (size_t)std::max<int64_t>(nwords, 1) * 4, s));
    }
  }
  k_batch_seed<<<1, 64, 0, s>>>(slots, (uint32_t)S.nf, (unsigned long long)S.ef,
                                sm.alive[S.alv], aslot);
  MSBFS_HIP_CHECK(hipGetLastError());
  constexpr bool FUSE = !COUNT;
  const bool fuse = FUSE && fuse_count_;
  const int grid = (int)std::min<int64_t>(td_grid_, std::max<int64_t>(1, (n + L::TILE - 1) / L::TILE));
  uint64_t* R = vis_[S.cur].as<uint64_t>();
  uint64_t* O = vis_[S.cur ^ 1].as<uint64_t>();
  const uint32_t level0 = S.level;
  const auto t0 = std::chrono::steady_clock::now();
  bool bm_ok = false;  // the previous level of this batch wrote the frontier bitmap
  const int rg = std::max(1, std::min(64, grid / 32));
  // fused levels share a reduction launch: level i's counters go to slab rows (i - pend) * grid
  const int red = std::max(1, std::min(td_red_, 3 * kMaxGrid / grid));
  int pend = -1;  // first fused level not reduced yet
  // the host's push -> pull test, on the degree sum of the frontier entering a level
  double efs = (double)S.ea / alpha_eff();
  if (gamma_ > 0) efs = std::min(efs, gamma_ * (double)n_eff());
  const unsigned long long ef_stop =
      opt.force_dir == 1 ? ~0ull : (unsigned long long)std::max(0.0, std::min(efs, 1.8e19));
  int aidx = 0;   // alive slot the next level reads
  auto reduce_pending = [&](int upto) {
    if (pend < 0) return;
    k_level_reduce_multi<W><<<W * rg, kBlock, 0, s>>>(slabF_.as<uint32_t>(), grid, upto - pend,
                                                      rg, level0 + 1 + pend, S.weight_l1 ? 1 : 0,
                                                      sm.F, aslot + 16 * (pend + 1));
    MSBFS_HIP_CHECK(hipGetLastError());
    aidx = upto;
    pend = -1;
  };
  trace::Range range_batch("bitpar L%u-%u TD batch", level0 + 1, level0 + K);
  for (int i = 0; i < K; ++i) {
    Ctr* prev = slots + i;
    Ctr* cur = slots + i + 1;
    const uint32_t level = level0 + 1 + i;
    ++epoch_;
    const uint32_t weight = (level == 1 && !S.weight_l1) ? 0u : level;
    if (fused_batches<COUNT>() && S.fsrc_acc && !S.lazy) {
      if (pend < 0) pend = i;
      k_td_fused<W><<<grid, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), &prev->fl2.v, bm_ok ? td_bm_min_ : INT64_MAX,
          fbm_[S.fc & 1].as<uint32_t>(), fbm_[(S.fc & 1) ^ 1].as<uint32_t>(), nwords, g_.rowptr,
          g_.col, R, acc_[S.ac].as<uint64_t>(), acc_[S.ac ^ 1].as<uint64_t>(), aslot + 16 * aidx,
          sm.gmask, done_.as<uint32_t>(), anyvis_.as<uint32_t>(), stamp_.as<int32_t>(), epoch_,
          fl_[S.fc ^ 1].as<int32_t>(), cur,
          slabF_.as<uint32_t>() + (size_t)(i - pend) * grid * 64 * W, prev,
          bm_ok ? 1 : 0, i + 1 == K ? 1 : 0, i > 0 ? slots + i - 1 : nullptr, ef_stop);
      MSBFS_HIP_CHECK(hipGetLastError());
      if (i + 1 - pend == red || i + 1 == K) reduce_pending(i + 1);
      S.fc ^= 1;
      S.ac ^= 1;
      S.old_stale = true;
      bm_ok = true;
      continue;
    }
    reduce_pending(i);
    bm_ok = false;  // (this level writes no bitmap)
    if (S.fsrc_acc)
      k_td_expand_small<W, false><<<grid, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), 0, &prev->fl2.v, g_.rowptr, g_.col, R,
          acc_[S.ac].as<uint64_t>(), done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(),
          stamp_.as<int32_t>(), epoch_, touched_.as<int32_t>(), cur,
          S.lazy ? anyvis_.as<uint32_t>() : nullptr, nullptr, i > 0 ? prev : nullptr, ef_stop);
    else
      k_td_expand_small<W, true><<<grid, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), 0, &prev->fl2.v, g_.rowptr, g_.col, R, O,
          done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
          touched_.as<int32_t>(), cur, S.lazy ? anyvis_.as<uint32_t>() : nullptr,
          S.osnap_next ? asnap_.as<uint32_t>() : nullptr, i > 0 ? prev : nullptr, ef_stop);
    auto kf = fuse ? k_td_finalize<W, COUNT, FUSE> : k_td_finalize<W, COUNT, false>;
    kf<<<grid, kBlock, 0, s>>>(touched_.as<int32_t>(), g_.rowptr, R, O,
                               acc_[S.ac ^ 1].as<uint64_t>(), aslot + 16 * aidx, sm.gmask,
                               done_.as<uint32_t>(), fl_[S.fc ^ 1].as<int32_t>(), cur,
                               fl_[S.fc].as<int32_t>(), 0, &prev->fl2.v,
                               S.fsrc_acc ? acc_[S.ac].as<uint64_t>() : nullptr,
                               anyvis_.as<uint32_t>(), slabF_.as<uint32_t>(), S.lazy ? 1 : 0,
                               &prev->act2.v);
    if (!fuse)
      k_count_frontier<W, COUNT, false><<<grid, kBlock, 0, s>>>(
          fl_[S.fc ^ 1].as<int32_t>(), cur, g_.rowptr, acc_[S.ac ^ 1].as<uint64_t>(), nullptr,
          slabF_.as<uint32_t>(), slabE_.as<unsigned long long>());
    k_level_reduce<W, COUNT><<<W * rg, kBlock, 0, s>>>(slabF_.as<uint32_t>(),
                                                       slabE_.as<unsigned long long>(), grid, rg,
                                                       sm.F, sm.E, aslot + 16 * (i + 1), weight);
    MSBFS_HIP_CHECK(hipGetLastError());
    aidx = i + 1;
    S.fc ^= 1;
    S.ac ^= 1;
    S.fsrc_acc = true;
    S.osnap_next = false;
  }
  (void)aidx;
  MSBFS_HIP_CHECK(hipMemcpyAsync(hbctr_->p, bctr_.p, (size_t)(K + 1) * sizeof(Ctr),
                                 hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  const Ctr* h = hbctr_->as<Ctr>();
  int real = 0;
  for (int i = 0; i < K; ++i) {
    // frontier empty before level i, or level i stopped for a pull: the rest were no-ops
    if (h[i].fl2.v == 0 || h[i].act2.v) break;
    ++real;
    S.ev += (int64_t)h[i + 1].ev2.v;
    if (level0 + 1 + i == 1) S.ev_l1 = S.ev;
  }
  // alive after the last real level -> the host loop's current alive buffer
  MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[S.alv], aslot + 16 * real, 16 * sizeof(uint64_t),
                                 hipMemcpyDeviceToDevice, s));
  S.level = level0 + real;
  S.nf = h[real].fl2.v;
  S.ef = (int64_t)h[real].ef2.v;
  if ((K - real) % 2) {
    // the no-op levels flipped the list / accumulator parity (they touched no buffer)
    S.fc ^= 1;
    S.ac ^= 1;
  }
  if (st && real > 0) {  // per-level records; the batch's wall time is split evenly
    const double ms = std::chrono::duration<double, std::milli>(
                          std::chrono::steady_clock::now() - t0).count() / real;
    for (int i = 0; i < real; ++i) {
      LevelRec rec;
      rec.batch = (int32_t)st->batches;
      rec.level = (int32_t)(level0 + 1 + i);
      rec.dir = 'T';
      rec.nf = h[i].fl2.v;
      rec.ef = (int64_t)h[i].ef2.v;
      rec.nf_next = h[i + 1].fl2.v;
      rec.active = h[i + 1].touched.v;
      rec.ms = ms;
      st->recs.push_back(rec);
    }
  }
  if (st) {
    st->td_levels += real;
    st->levels += real;
  }
  batch_next_ = S.nf > 0 ? std::min(batch_next_ * 2, kBatch) : 4;
}

template <int W, bool COUNT>
void BitparSolver::batch_impl(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids,
                              int64_t* Fout, int64_t* edges2, RunStats* st, hipStream_t s) {
  Loop S;
  S.cnt = n_eff();
  // lazy: no per-batch fill of vis_[0] (n_eff * 8W bytes, ~0.8 ms on RMAT-26); the edge-counting
  // pass re-reads both rows of every new vertex (k_count_frontier), so it keeps the fill
  S.lazy = lazy_ && !COUNT && fuse_count_ && !fused_batches<COUNT>();
  start_batch<W, COUNT>(k0, nb, qoff, qids, S, s);
  levels<W, COUNT>(S, st, s);
  // frontier is empty: accumulator entries were cleared by finalize / zero_acc
  const unsigned long long* h = read_small(s);
  for (int64_t k = 0; k < nb; ++k) {
    Fout[k] = (int64_t)h[k];
    if (edges2) edges2[k] = (int64_t)h[64 * 16 + k];
  }
}

// Phase A: level 1 (top-down, every rank identical, only rank 0 adds it to F), level 2
// (bottom-up over this rank's residue class only), then pack its rows' words per destination.
template <int W>
void BitparSolver::phase_a_impl(int64_t K, const int64_t* qoff, const int32_t* qids, int part,
                                int nparts, int64_t n_eff, bool count_l1, const int32_t* wbeg,
                                uint64_t* send, int64_t* out, RunStats* st, hipStream_t s,
                                int64_t* coded_len) {
  Loop S;
  S.part = part;
  S.nparts = nparts;
  S.cnt = part_count(n_eff, part, nparts);
  S.stop_level = 2;
  S.weight_l1 = count_l1;
  S.plan = "TB";
  S.lazy = lazy_ && fuse_count_ && opt.force_dir == 0 && dirs_.empty();
  start_batch<W, false>(0, K, qoff, qids, S, s);
  levels<W, false>(S, st, s);
  if (S.fsrc_acc && S.nf > 0) {  // stopped after a top-down level: restore the zero accumulator
    k_zero_acc<W><<<grid_for(S.nf * Lay<W>::G, kBlock), kBlock, 0, s>>>(
        fl_[S.fc].as<int32_t>(), S.nf, acc_[S.ac].as<uint64_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  const int wt = (int)((K + 63) / 64);
  WordSplit ws{};
  for (int j = 0; j <= nparts; ++j) ws.b[j] = wbeg[j];
  for (int j = nparts + 1; j <= kMaxParts; ++j) ws.b[j] = wt + 1;  // never reached
  if (coded_len) {
    code_send<W>(vis_[S.cur].as<uint64_t>(), S.cnt, part, nparts, ws, send, coded_len, s);
  } else if (S.cnt > 0) {
    k_pack_words<W><<<grid_for(S.cnt * wt, kBlock, 8192), kBlock, 0, s>>>(
        vis_[S.cur].as<uint64_t>(), g_.rowptr, part, nparts, S.cnt, wt, ws, send);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  const bool ran_l2 = S.level >= 2;
  const Small sm = small();
  const unsigned long long* h = read_small(s);
  const unsigned long long* alive_h = h + (sm.alive[S.alv] - (uint64_t*)sm.F);
  for (int64_t k = 0; k < K; ++k) {
    out[k] = (int64_t)h[k];
    out[K + k] = ran_l2 ? (int64_t)((alive_h[k >> 6] >> (k & 63)) & 1ull) : 0;
  }
  out[2 * K] = ran_l2 ? S.nf : 0;
  out[2 * K + 1] = ran_l2 ? S.ef : 0;
  out[2 * K + 2] = count_l1 ? S.ev : (ran_l2 ? S.ev - S.ev_l1 : 0);
}

// Phase C: rebuild the level-2 state of this rank's groups from the exchanged words and run
// the remaining levels (the first one bottom-up: the frontier is only implicit in the words).
template <int W>
void BitparSolver::phase_c_impl(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                                const uint64_t* recv, const int64_t* reduced, int64_t* F_out,
                                RunStats* st, hipStream_t s) {
  MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
  MSBFS_HIP_CHECK(hipMemsetAsync(small_.p, 0, small_.bytes, s));
  const Small sm = small();
  {
    uint64_t ha[2][16] = {{0}};  // alive, gmask
    for (int w = 0; w < w_count; ++w)
      for (int b = 0; b < 64; ++b) {
        const int64_t k = (int64_t)(w_begin + w) * 64 + b;
        if (k >= K) break;
        ha[1][w] |= 1ull << b;
        if (reduced[K + k] > 0) ha[0][w] |= 1ull << b;
      }
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[0], ha[0], sizeof(ha[0]), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.gmask, ha[1], sizeof(ha[1]), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  if (n_eff > 0) {  // vertices >= n_eff have no edges: no kernel reads their rows or bits
    PartPrefix pre{};
    for (int r = 0; r < nparts; ++r) pre.b[r + 1] = pre.b[r] + part_count(n_eff, r, nparts);
    k_hybrid_setup<W><<<grid_for(n_eff, Lay<W>::TILE, 8192), kBlock, 0, s>>>(
        recv, w_count, n_eff, nparts, pre, vis_[0].as<uint64_t>(), vis_[1].as<uint64_t>(),
        sm.alive[0], sm.gmask, done_.as<uint32_t>(), anyvis_.as<uint32_t>(), g_.rowptr,
        std::max(opt.wide_degree, wide_later_), act_[0].as<int32_t>(), actw_[0].as<int32_t>(),
        ctr_.as<Ctr>());
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  Loop S;
  {
    // the setup built the level-3 active lists (see k_hybrid_setup)
    const HostCtr c = read_ctr(s);
    S.nact = c.act2;
    S.nactw = c.actw2;
    S.have_active = true;
    MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
  }
  S.cnt = n_eff;
  S.level = 2;
  S.nf = reduced[2 * K];
  S.ef = reduced[2 * K + 1];
  S.ev = reduced[2 * K + 2];
  S.na = S.nact + S.nactw;
  S.ea = g_.nnz;
  S.bu_levels = 1;
  S.fsrc_acc = false;
  S.bottom_up = true;
  S.plan = "..B";
  levels<W, false>(S, st, s);
  const unsigned long long* h = read_small(s);
  for (int64_t i = 0; i < (int64_t)w_count * 64; ++i) F_out[i] = (int64_t)h[i];
}

}  // namespace bp

std::unique_ptr<Solver> make_bitpar_solver(const DeviceGraph& g, int max_groups) {
  return std::make_unique<bp::BitparSolver>(g, max_groups);
}

int64_t hybrid_extent(const DeviceGraph& g) {
  MSBFS_HIP_CHECK(hipSetDevice(g.device));
  if (g.n <= 0) return 0;
  DevBuf d;
  d.alloc(sizeof(unsigned long long));
  MSBFS_HIP_CHECK(hipMemset(d.p, 0, sizeof(unsigned long long)));
  bp::k_extent<<<grid_for(g.n, 256, 2048), 256>>>(g.rowptr, g.n, d.as<unsigned long long>());
  MSBFS_HIP_CHECK(hipGetLastError());
  unsigned long long h = 0;
  MSBFS_HIP_CHECK(hipMemcpy(&h, d.p, sizeof(h), hipMemcpyDeviceToHost));
  return (int64_t)h;
}

}  // namespace msbfs
