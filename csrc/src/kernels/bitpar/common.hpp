// Bit-parallel MS-BFS: row layout, wave helpers, level counters and the per-level reductions
// shared by every translation unit of the solver (kernels/bitpar_*.hip). Design overview:
// solver.hpp.
#pragma once

#include <cstdint>

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

// One lane per vertex (G == 1): column entries [b, b + 4) of a row ending at e (-1 past it) from
// two aligned 16-byte loads, i.e. one address per four entries instead of one per entry (the
// address unit is the busy resource of these pulls). col must be 16-byte aligned (the graph
// constructors check it); the second load re-reads the first window when the row ends before
// it, and an aligned window never leaves the page of the valid entry it starts at.
__device__ __forceinline__ void col4_aligned(const int32_t* col, int64_t b, int64_t e,
                                             int32_t (&u)[4]) {
  typedef int32_t i4 __attribute__((ext_vector_type(4)));
  const int64_t a = b & ~(int64_t)3;
  const int sh = (int)(b - a);
  const i4 w0 = *(const i4*)(col + a);
  const i4 w1 = *(const i4*)(col + (a + 4 < e ? a + 4 : a));
  const int32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int32_t x = sh == 0 ? w[q] : sh == 1 ? w[q + 1] : sh == 2 ? w[q + 2] : w[q + 3];
    u[q] = b + q < e ? x : -1;
  }
}

// lanes below this one among the set bits of a wave mask (v_mbcnt)
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-private LDS queue: items of this wave only; the count is wave-uniform (kept in an SGPR),
// a flush takes one global atomic for the whole run and writes it out coalesced.
__device__ __forceinline__ void wq_push(int32_t* q, uint32_t& n, bool pred, int32_t v) {
  const uint64_t m = __ballot(pred);
  if (pred) q[n + mbcnt64(m)] = v;
  n += (uint32_t)__popcll(m);
}
__device__ __forceinline__ void wq_flush(int32_t* q, uint32_t& n, int32_t* out, uint32_t* gcnt) {
  if (!n) return;
  uint32_t base = 0;
  if (lane_id() == 0) base = atomicAdd(gcnt, n);
  base = __builtin_amdgcn_readfirstlane(base);
  for (uint32_t i = lane_id(); i < n; i += 64) out[base + i] = q[i];
  n = 0;
}

// The end-of-kernel flush of every wave's queue: the block's waves publish their counts, one
// lane takes the block's run with one atomic, each wave writes its items at its offset.
// Block-uniform (every thread calls it); wbase: kWaves + 1 LDS words.
__device__ __forceinline__ void wq_flush_block(int32_t* q, uint32_t& n, int32_t* out,
                                               uint32_t* gcnt, uint32_t* wbase) {
  const int wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) wbase[wv] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < nwv; ++w) {
      const uint32_t c = wbase[w];
      wbase[w] = t;
      t += c;
    }
    wbase[nwv] = t ? atomicAdd(gcnt, t) : 0u;
  }
  __syncthreads();
  const uint32_t base = wbase[nwv] + wbase[wv];
  for (uint32_t i = lane_id(); i < n; i += 64) out[base + i] = q[i];
  n = 0;
}

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
// Set bit v of bitmap bm for every lane with pred, one atomicOr per distinct word of the wave
// instead of one per lane (whole wave, uniform control flow). Device-scope atomics execute at the
// memory side (tens of G/s for the whole chip); the pull kernels' vertices come from list tiles
// in id order, so a wave's bits fall in a few words. The first kMaxWords distinct words are
// combined (OR across the lanes of the word by xor shuffles), any lanes left over (a scattered
// list) use their own atomic. RMAT-26, 128 groups: 13.3 -> 10.6 ms/step (level 4 1.66 -> 0.70 ms,
// ~1 ms of it done-bit atomics); 1024 groups: level 2 14.9 -> 14.6 ms (first-visit bits). Not for
// k_td_fused's appends: the road grid ran 321 -> 371 ms with it (its claims dominate, and the
// combining loops sit inside the unrolled edge loop).
template <bool COMBINE = true>
__device__ __forceinline__ void wave_set_bits(uint32_t* bm, int32_t v, bool pred) {
  if constexpr (!COMBINE) {
    if (pred) atomicOr(&bm[v >> 5], 1u << (v & 31));
    return;
  }
  constexpr int kMaxWords = 4;
  uint64_t pending = __ballot(pred);
  if (!pending) return;
  const int lane = lane_id();
  const int32_t w = v >> 5;
  const uint32_t bit = 1u << (v & 31);
#pragma unroll 1
  for (int it = 0; it < kMaxWords && pending; ++it) {
    const int l = __ffsll((unsigned long long)pending) - 1;
    const int32_t wl = __shfl(w, l);
    const bool mine = ((pending >> lane) & 1ull) && w == wl;
    uint32_t b = mine ? bit : 0u;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) b |= __shfl_xor(b, off);
    if (lane == l) atomicOr(&bm[wl], b);
    pending &= ~__ballot(mine);
  }
  if ((pending >> lane) & 1ull) atomicOr(&bm[w], bit);
}
// flags of the unfiltered pull kernels (k_bu_first, k_bu_full)
constexpr int kFlagSkipRows = 1;     // dskip: a vertex finishing here writes no row
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
  // spill_strided with 32-bit halves (~12 instead of ~21 VALU per set counter bit: the
  // first pull level sets about half the bits of every word between two spills)
  template <int STRIDE>
  __device__ __forceinline__ void spill_strided32(uint32_t* f, int slot) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint32_t sl[D], any = 0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          sl[d] = (uint32_t)(c[j][d] >> (32 * h));
          any |= sl[d];
        }
        uint32_t* row = f + (slot * VW + j) * STRIDE + 32 * h;
        while (any) {
          const int b = __ffs(any) - 1;
          any &= any - 1;
          uint32_t v = 0;
#pragma unroll
          for (int d = 0; d < D; ++d) v |= ((sl[d] >> b) & 1u) << d;
          atomicAdd(&row[b], v);
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) c[j][d] = 0;
    }
  }
};

// Gate of a level of a device-driven pull batch (BitparSolver::bu_batch): level i reads counter
// slot c (written by level i - 1, or seeded by the host for i = 0) and runs while the frontier
// entering it is non-empty and the host loop's pull -> push test (levels(): nf < na / beta and
// ef < ea / alpha, same double arithmetic) would keep pulling. Every kernel of the level
// evaluates it at its start, so a closed level is a no-op. c == nullptr: always open.
// The pull -> push test (Beamer et al. SC'12): switch back to push once the frontier is small
// against the active vertices (beta) and its edges against theirs (alpha). One definition for
// the host loop and the device gate, so both decide alike.
__host__ __device__ inline bool keep_pulling(double nf, double ef, double na, double ea,
                                             double beta, double alpha) {
  return !(nf < na / beta && ef < ea / alpha);
}
struct BuGate {
  const Ctr* c;
  double beta, alpha;
  int first;  // the batch's first level (the host already chose to pull)
};
__host__ __device__ inline bool bu_gate_eval(const Ctr& c, double beta, double alpha, int first) {
  if (c.fl2.v == 0) return false;
  return first || keep_pulling((double)c.fl2.v, (double)c.ef2.v,
                               (double)c.act2.v + (double)c.actw2.v, (double)c.eu2.v, beta, alpha);
}
__device__ __forceinline__ bool bu_gate_open(const BuGate& g) {
  return !g.c || bu_gate_eval(*g.c, g.beta, g.alpha, g.first);
}

// Sum the level's slab rows: block (word, row-group); lane = group bit. F += level * count
// (`level` is the weight: 0 for a level another rank of the hybrid mode accounts for),
// alive_next |= groups with count > 0 (one ballot + one atomicOr per word per row-group).
template <int W, bool COUNT>
__global__ __launch_bounds__(kBlock) void k_level_reduce(const uint32_t* slabF,
                                                         const unsigned long long* slabE, int rows,
                                                         int rgroups, unsigned long long* F,
                                                         unsigned long long* E,
                                                         uint64_t* alive_next, uint32_t level,
                                                         BuGate gate) {
  if (!bu_gate_open(gate)) return;  // (uniform: no barrier skipped by part of the block)
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

}  // namespace bp
}  // namespace msbfs
