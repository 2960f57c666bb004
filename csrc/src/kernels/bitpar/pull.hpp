// Bit-parallel MS-BFS: bottom-up (pull) level kernels — active lists, sparse row codes, prefix
// pull + tail push, the narrow lane-group pull, the lean first-row pass, hub edge chunks and the
// wide finalize.
#pragma once

#include "common.hpp"

namespace msbfs {
namespace bp {

// build the bottom-up active lists (deg > 0, not done) over the vertices v = part + i*nparts,
// i < cnt, split by degree, or by the row prefix length plen[v] when given (the untiled prefix
// level pulls only the prefix: a vertex of high degree with a short prefix is a narrow one)
// (nparts = 1: every vertex; the hybrid mode's vertex-partitioned level pulls only for its own
// residue class)
template <int QCAP>
__global__ __launch_bounds__(kBlock) void k_build_active(int64_t cnt, int part, int nparts,
                                                         const int64_t* rowptr,
                                                         const uint32_t* done, int wide_deg,
                                                         int32_t* act, int32_t* actw, Ctr* ctr,
                                                         const int32_t* plen = nullptr,
                                                         int64_t n_eff = -1) {
  // n_eff >= 0 (with plen, degree-relabelled rows: exactly the vertices < n_eff have edges): no
  // row offsets are read at all (RMAT-30: 8.6 GB), and eu2 stays 0 (its caller reads only the
  // list sizes)
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
    int64_t d[VPT], sd[VPT];
    uint32_t dw[VPT];
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int64_t j = b + q * kBlock + threadIdx.x;
      const int64_t i = part + j * nparts;
      d[q] = 0;
      sd[q] = 0;
      dw[q] = ~0u;
      if (j < b1) {
        if (n_eff >= 0) {
          d[q] = i < n_eff ? 1 : 0;
          if (i < n_eff) sd[q] = (int64_t)plen[i];
        } else {
          d[q] = rowptr[i + 1] - rowptr[i];
          sd[q] = plen ? (int64_t)plen[i] : d[q];
        }
        dw[q] = done[i >> 5];
      }
    }
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int64_t i = part + (b + q * kBlock + threadIdx.x) * nparts;
      const bool ok = d[q] > 0 && !((dw[q] >> (i & 31)) & 1u);
      if (ok && n_eff < 0) eu += (unsigned long long)d[q];
      q_push(qn, ok && sd[q] <= wide_deg, (int32_t)i);
      q_push(qw, ok && sd[q] > wide_deg, (int32_t)i);
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

// first id with degree < 2^k for k = 0..kDegBounds-1 (rows relabelled by descending degree: one
// binary search per k, one thread each)
constexpr int kDegBounds = 41;
static __global__ void k_degree_bounds(const int64_t* rowptr, int64_t n, int32_t* out) {
  const int k = threadIdx.x;
  if (k >= kDegBounds) return;
  const int64_t min_deg = (int64_t)1 << k;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid + 1] - rowptr[mid] < min_deg) hi = mid;
    else lo = mid + 1;
  }
  out[k] = (int32_t)lo;
}

// number of vertices with degree > d (bounds the wide list of any pull level)
static __global__ __launch_bounds__(kBlock) void k_count_wide(const int64_t* rowptr, int64_t n, int64_t d,
                                                       unsigned long long* out) {
  __shared__ unsigned long long scratch[kWaves];
  unsigned long long c = 0;
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n;
       v += (int64_t)gridDim.x * kBlock)
    c += rowptr[v + 1] - rowptr[v] > d;
  block_sum_add(c, out, scratch);
}

// ---------------------------------------------------------------------------------------------
// Prefix pull + tail push for the first bottom-up level (rows sorted by id, degree relabelled).
// The LDS hub bitmap covers the ids < H; a pull that scanned whole rows had to probe the global
// visited bitmap for every neighbour id >= H (the degree tail: ~40 % of the edge endpoints on
// RMAT-26, almost none of them in the level-1 frontier). Instead the pulls stop at the first id
// >= H, and the few level-1 frontier vertices u >= H push their bits to their neighbours here:
// acc[v] |= row(u) (atomicOr, mostly one word thanks to the sparse codes) and stamp[v] = epoch
// (stamp = nullptr: the consumer reads every vertex's acc row instead).
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
    int part, int nparts, uint64_t* acc, int32_t* stamp, int32_t epoch, int split) {
  constexpr int PG = 64;  // lanes per wave: an entry's lanes take consecutive row entries
  // `split` waves per frontier entry (wave s of entry i takes row entries s*64 + lane, step
  // split*64; the host splits small frontiers only), UN entries per lane in flight: a frontier
  // vertex of degree 30K otherwise kept one wave busy for ~470 dependent rounds of column id ->
  // done probe -> atomic while the rest of the grid had finished (RMAT-30 / 32 groups: ~10K
  // frontier vertices push; 1024 groups: ~100K+, mostly of low degree, one wave each)
  constexpr int UN = 4;
  const int SPLIT = split;
  // own targets: v % nparts == part (hybrid phase A); a power-of-two count tests the low bits
  // instead of dividing (v % nparts: ~40 VALU per neighbour entry)
  const uint32_t pmask = (nparts & (nparts - 1)) == 0 ? (uint32_t)(nparts - 1) : 0u;
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / PG;
  const int64_t nwave = ((int64_t)gridDim.x * kBlock) / PG;
  for (int64_t wi = wave; wi < nf * SPLIT; wi += nwave) {
    const int64_t i = wi / SPLIT;
    const int sp = (int)(wi % SPLIT);
    const int32_t u = fl[i];
    if (u < H) continue;
    const uint32_t c = (code && u >= code_from) ? code[u] : kDenseCode;
    if (c == 0) continue;
    const int64_t b = rowptr[u], e = rowptr[u + 1];
    const int64_t kStep = (int64_t)SPLIT * PG;
    for (int64_t k0 = b + sp * PG + lane; k0 < e; k0 += UN * kStep) {
      int32_t v[UN];
      bool ok[UN];
#pragma unroll
      for (int q = 0; q < UN; ++q) {  // loads first (clamped index), tests after
        const int64_t k = k0 + q * kStep;
        const int32_t x = col[k < e ? k : k0];
        v[q] = x;
        ok[q] = k < e;
      }
#pragma unroll
      for (int q = 0; q < UN; ++q)
        if (nparts > 1)
          ok[q] = ok[q] && (pmask ? ((uint32_t)v[q] & pmask) == (uint32_t)part
                                  : v[q] % nparts == part);
      if (done) {  // (nullptr: the consumer clears done rows too)
        uint32_t dw[UN];
#pragma unroll
        for (int q = 0; q < UN; ++q) dw[q] = done[v[q] >> 5];
#pragma unroll
        for (int q = 0; q < UN; ++q) ok[q] = ok[q] && !((dw[q] >> (v[q] & 31)) & 1u);
      }
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if (!ok[q]) continue;
        if (c != kDenseCode) {
          for (int s = 0; s < kCodeSlots; ++s) {
            const int g = code_g(c, s);
            if (g >= 0)
              atomicOr((unsigned long long*)&acc[(int64_t)v[q] * W + (g >> 6)], 1ull << (g & 63));
          }
        } else {
          for (int j = 0; j < W; ++j) {
            const uint64_t w = R[(int64_t)u * W + j];
            if (w)
              atomicOr((unsigned long long*)&acc[(int64_t)v[q] * W + j], (unsigned long long)w);
          }
        }
        if (stamp) stamp[v[q]] = epoch;  // (nullptr: the consumer reads every acc row)
      }
    }
  }
}

// 32-bit block sum, one atomic per block
__device__ __forceinline__ void block_sum_add32(uint32_t val, uint32_t* dst, uint32_t* scratch) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) val += __shfl_xor(val, off);
  __syncthreads();
  if (lane_id() == 0) scratch[threadIdx.x >> 6] = val;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += scratch[w];
    if (t) atomicAdd(dst, t);
  }
}

// The tail push AFTER the tiled prefix pull (tuning key push_after; one GPU, no chunked
// exchange): the pushed bits go straight into the level's output rows O, so the tile epilogue
// reads no acc row (4.2 GB on RMAT-26 / 1024 groups, every tile vertex) and a push whose bit
// the prefix pull already set costs a plain load instead of an atomic. The push then does the
// accounting of what it adds (the epilogue has run): per-group counts of the bits its
// atomicOr newly set (LDS counters -> this block's slab row), and for a vertex it gave its
// first new bit of the level, the frontier bit (+ count, degree sum), and for one it gave its
// first bit at all, the any-visited bit (+ degree sum). A vertex the pushed bits complete is
// left not done (the next pull finds it covered). Census (tools/tail_push_stats.py, RMAT-26):
// 179K tail pushers, 40.7M pushed edges, 42.5M code slots, 6.9M distinct targets.
template <int W>
__global__ __launch_bounds__(kBlock) void k_push_tail_after(
    const int32_t* fl, int64_t nf, int32_t H, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, const uint32_t* code, int32_t code_from, uint64_t* O, uint32_t* fbm,
    uint32_t* anyvis, Ctr* ctr, uint32_t* slabF) {
  __shared__ uint32_t cnt[64 * W];
  __shared__ unsigned long long scratch[kWaves];
  __shared__ uint32_t scratch32[kWaves];
  for (int i = threadIdx.x; i < 64 * W; i += kBlock) cnt[i] = 0;
  __syncthreads();
  unsigned long long ef = 0, ev = 0;
  uint32_t nfc = 0;
  const int lane = lane_id();
  const int64_t grp = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t ngrp = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t i = grp; i < nf; i += ngrp) {
    const int32_t u = fl[i];
    if (u < H) continue;
    const uint32_t c = (code && u >= code_from) ? code[u] : kDenseCode;
    if (c == 0) continue;
    const int64_t b = rowptr[u], e = rowptr[u + 1];
    for (int64_t k = b + lane; k < e; k += 64) {
      const int32_t v = col[k];
      // (every target has its output row: the tiles and the big vertices' finalize write one
      // for the vertices done before this level too, holding every alive group)
      bool added = false;
      if (c != kDenseCode) {
        for (int s = 0; s < kCodeSlots; ++s) {
          const int g = code_g(c, s);
          if (g < 0) continue;
          unsigned long long* p = (unsigned long long*)&O[(int64_t)v * W + (g >> 6)];
          const unsigned long long bit = 1ull << (g & 63);
          if (*p & bit) continue;  // (set by the pull or an earlier push: bits only get set)
          if (!(atomicOr(p, bit) & bit)) {
            atomicAdd(&cnt[g], 1u);
            added = true;
          }
        }
      } else {
        for (int j = 0; j < W; ++j) {
          const uint64_t w = R[(int64_t)u * W + j];
          if (!w) continue;
          uint64_t nb = w & ~(uint64_t)atomicOr((unsigned long long*)&O[(int64_t)v * W + j],
                                                (unsigned long long)w);
          added |= nb != 0;
          while (nb) {
            atomicAdd(&cnt[j * 64 + __ffsll((unsigned long long)nb) - 1], 1u);
            nb &= nb - 1;
          }
        }
      }
      if (added) {  // (plain loads first: most targets got new bits from the pull already)
        const uint32_t m = 1u << (v & 31);
        const bool in_f = (fbm[v >> 5] & m) != 0, seen = (anyvis[v >> 5] & m) != 0;
        if (!in_f || !seen) {
          const unsigned long long dv = (unsigned long long)(rowptr[v + 1] - rowptr[v]);
          if (!in_f && !(atomicOr(&fbm[v >> 5], m) & m)) {
            ++nfc;
            ef += dv;
          }
          if (!seen && !(atomicOr(&anyvis[v >> 5], m) & m)) ev += dv;
        }
      }
    }
  }
  block_sum_add32(nfc, &ctr->fl2.v, scratch32);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  __syncthreads();
  uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
  for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = cnt[i];
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
// PFX (prefix-pull level, see k_push_tail): rows are scanned only over their prefix plen[v] (the
// ids below the level's bound H <= HUBW*32, see BitparSolver::pfx_bound),
// and pushed bits (acc of vertices with stamp == epoch; every vertex's acc when stamp is
// nullptr) seed the accumulator.
// CS = neighbours per step (rows gathered between two coverage checks).
// C1 > 0 (unfiltered levels only): a first step of just C1 rows before the CS-wide steps; late
// levels are mostly covered by the first neighbour or two (sorted rows: hubs first).
// FBM: the new frontier goes into the bitmap fbm (passed as fl2) and its size into ctr->fl2, no
// frontier list (the prefix level at few words, whose next level pulls: see level_bu).
template <int W, bool COUNT, int BT, int HUBW, bool FUSE, bool FILT = true, bool PFX = false,
          int CS = 8, int C1 = 0, int MINW = 4, bool FBM = false>
__global__ __launch_bounds__(BT, MINW) void k_bu_narrow(
    const int32_t* act, int64_t nact, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, uint64_t* Wb, const uint64_t* alive, const uint64_t* gmask, uint32_t* done,
    int32_t* act2, int32_t* fl2, Ctr* ctr, uint32_t* anyvis, int32_t filter_from, int32_t* actw2,
    int next_wide, uint32_t* slabF, uint64_t* pacc, const int32_t* stamp, int32_t epoch,
    const int32_t* plen, const uint32_t* nact_dev, const uint32_t* snap, BuGate gate) {
  static_assert(!PFX || HUBW > 0, "the prefix pull relies on the LDS hub bitmap");
  if (!bu_gate_open(gate)) return;  // closed level of a device-driven batch (uniform)
  // snap (first pull level of a batch that did not clear its visited buffer, see start_batch):
  // the any-visited bitmap as of the level start. Probes read it (a vertex first visited during
  // this level may still have a stale row) and an own row it does not mark is all zero.
  const uint32_t* pvis = snap ? snap : anyvis;
  if (nact_dev) nact = (int64_t)*nact_dev;  // (list length known only on the device)
  static_assert(!(FUSE && COUNT), "the edge-counting pass uses k_count_frontier");
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW;
  // done / any-visited bits: one atomic per word of the wave (wave_set_bits) where a wave
  // holds many vertices or many first visits (W = 16 levels 3-4 measured ~0.4 ms slower each)
  constexpr bool kCombine = G <= 4 || PFX;
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
  uint32_t nfc = 0;  // FBM: new frontier vertices
  __shared__ uint32_t scratch32[FBM ? NWV : 1];
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
  // one lane per vertex, four-entry steps: aligned 16-byte id loads (col4_aligned, pull_full.hpp)
  constexpr bool A4 = G == 1 && Q == 4 && C == 4;
  int32_t u1[Q];  // first-step column ids of the current tile's vertex (third pipeline stage)
  auto first_ids = [&](bool ok, int32_t (&u)[Q]) {
    if constexpr (A4) {
      const int64_t n1 = ok ? (int64_t)(PFX ? p1 : d1) : 0;
      col4_aligned(col, ok ? b1 : 0, ok ? b1 + n1 : 0, u);
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        u[q] = (ok && q * G + slot < C && (uint32_t)(q * G + slot) < (PFX ? p1 : d1))
                   ? col[b1 + q * G + slot] : -1;
    }
  };
  first_ids(tb + lofs < nact, u1);
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
      if (!stamp) {  // (uniform) no stamps: every vertex reads its row, clears it if set
        const V<VW> a0 = ldv<VW>(pacc + (int64_t)(valid ? v : 0) * W + slot * VW);
        bool set = false;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          acc.w[j] = valid ? a0.w[j] : 0ull;
          set |= acc.w[j] != 0;
        }
        if (set) stv<VW>(pacc + (int64_t)v * W + slot * VW, vzero<VW>());
      } else if (valid && stamp[v] == epoch) {
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
        bool loaded = false;
        if constexpr (A4) {
          if (!(C1 == 0 && e == beg)) {
            col4_aligned(col, e, end, u);
            loaded = true;
          }
        }
        if (!loaded) {
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int64_t ee = e + q * G + slot;
            // first step: preloaded (without the short first step)
            u[q] = (C1 == 0 && e == beg) ? u0[q]
                                         : ((q * G + slot < C && ee < end) ? col[ee] : -1);
          }
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
    wave_set_bits<kCombine>(done, v, leader && !g_nf);
    const bool keep = leader && g_nf, app = leader && g_new;
    if (keep) eu += deg;
    if (app) ef += deg;
    {
      const bool g_first = g_new && !((__ballot(rnz) >> (sub * G)) & L::GBITS);
      wave_set_bits<kCombine>(anyvis, v, leader && g_first);
      if (leader && g_first) ev += deg;
    }
    // third stage: the next tile's first-step ids (its offsets arrived during this tile)
    first_ids(idx + stride < nact, u1);
    q_push(qa, keep && (int)deg <= next_wide, v);
    q_push(qw, keep && (int)deg > next_wide, v);
    if constexpr (FBM) {
      wave_set_bits<true>(reinterpret_cast<uint32_t*>(fl2), v, app);
      nfc += app ? 1u : 0u;
      q_flush_n<kQCap, 2>({&qa, &qw}, {act2, actw2}, {&ctr->act2.v, &ctr->actw2.v}, TILE, false);
    } else {
      q_push(qf, app, v);
      q_flush_n<kQCap, 3>({&qa, &qw, &qf}, {act2, actw2, fl2},
                          {&ctr->act2.v, &ctr->actw2.v, &ctr->fl2.v}, TILE, false);
    }
  }
  if constexpr (FBM) {
    q_flush_n<kQCap, 2>({&qa, &qw}, {act2, actw2}, {&ctr->act2.v, &ctr->actw2.v}, 0, true);
    block_sum_add32(nfc, &ctr->fl2.v, scratch32);
  } else {
    q_flush_n<kQCap, 3>({&qa, &qw, &qf}, {act2, actw2, fl2},
                        {&ctr->act2.v, &ctr->actw2.v, &ctr->fl2.v}, 0, true);
  }
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
// dsnap / skip (tuning dskip, see k_bu_full): a first neighbour done at the level start
// covers every alive group (probe instead of its row); every vertex this pass finishes is done,
// so with skip it writes no row at all.
template <int W>
__global__ __launch_bounds__(kBlock, W >= 16 ? 8 : 6) void k_bu_first(
    const int32_t* act, int64_t nact, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, uint64_t* Wb, const uint64_t* alive, const uint64_t* gmask, uint32_t* done,
    int32_t* ovf, int32_t* fl2, Ctr* ctr, uint32_t* anyvis, uint32_t* slabF, const int32_t* first,
    const uint32_t* dsnap, int flags) {
  const bool skip = flags & kFlagSkipRows;
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  // done / any-visited bits: one atomic per word of the wave (wave_set_bits) where a wave
  // holds many vertices or many first visits (W = 16 levels 3-4 measured ~0.4 ms slower each)
  constexpr bool kCombine = G <= 4;
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
      V<VW> x;
      r = ldv<VW>(R + (int64_t)v * W + slot * VW);
      deg = (uint32_t)(rowptr[v + 1] - rowptr[v]);  // only counted, off the load chain
      if (dsnap && ((dsnap[u >> 5] >> (u & 31)) & 1u)) x = am;  // (a done first neighbour)
      else x = ldv<VW>(R + (int64_t)u * W + slot * VW);
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
    if (fin && !skip) {
      V<VW> nv;
#pragma unroll
      for (int j = 0; j < VW; ++j) nv.w[j] = r.w[j] | nw.w[j];
      stv<VW>(Wb + (int64_t)v * W + slot * VW, nv);
    }
    bc.add(nw);
    if (++nadd == (1 << BitCounter<VW>::D) - 1) {
      bc.template spill_strided32<CR>(cnt, slot);
      nadd = 0;
    }
    bool anynew = false;
#pragma unroll
    for (int j = 0; j < VW; ++j) anynew |= nw.w[j] != 0;
    const bool g_new = (__ballot(anynew) >> (sub * G)) & L::GBITS;
    const bool g_first = g_new && !((__ballot(rnz) >> (sub * G)) & L::GBITS);
    const bool leader = valid && slot == 0;
    wave_set_bits<kCombine>(done, v, leader && fin);
    if (leader && g_new) ef += deg;
    wave_set_bits<kCombine>(anyvis, v, leader && g_first);
    if (leader && g_first) ev += deg;
    q_push(qo, leader && !fin, v);
    q_push(qf, leader && g_new, v);
    q_flush(qo, ovf, &ctr->touched.v, TILE, false);
    q_flush(qf, fl2, &ctr->fl2.v, TILE, false);
  }
  q_flush(qo, ovf, &ctr->touched.v, 0, true);
  q_flush(qf, fl2, &ctr->fl2.v, 0, true);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  bc.template spill_strided32<CR>(cnt, slot);
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
                                           const uint32_t* snap, const uint32_t* dsnap) {
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
  // each: OR the S lane groups' partial rows together and test coverage after every step of
  // PB*S rows; otherwise once per tile. Without early exit across chunks (coop = 0: the first
  // pull level, where hardly any row gets covered) the per-step reduction (3 x VW xor-shuffles)
  // was most of the kernel's LDS instructions: RMAT-26 level-2 chunk pulls 6.63 -> 6.41 ms.
  const bool each = coop != 0;
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
    if (dsnap) {  // (uniform) done neighbours: the alive mask instead of their rows (k_bu_full)
      bool hit = false;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (u[q] >= 0 && ((dsnap[u[q] >> 5] >> (u[q] & 31)) & 1u)) {
          u[q] = -1;
          hit = true;
        }
      if (__ballot(hit))
#pragma unroll
        for (int j = 0; j < VW; ++j) a.w[j] |= am.w[j];
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
      if (each) {
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
    }
    if (!each) {  // one cross-group OR and coverage check per tile (see `each`)
#pragma unroll
      for (int off = G; off < 64; off <<= 1)
#pragma unroll
        for (int j = 0; j < VW; ++j) a.w[j] |= __shfl_xor(a.w[j], off);
      bool cov = true;
#pragma unroll
      for (int j = 0; j < VW; ++j) cov &= ((a.w[j] | g.w[j]) & unv.w[j]) == unv.w[j];
      if (!__ballot(!cov)) covered = true;
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

// chunk_pull for the prefix-pull level without codes (fewer than 8 words, or codes off): every
// id of a row prefix is below the LDS hub bitmap's bound, so the probes are LDS reads only, and
// no chunk exits early (coop = 0 at the first pull level). The next tile's column ids are loaded
// while the current tile is probed and gathered; every load is unconditional (clamped index,
// result selected after), so the compiler waits for exactly the loads each use needs instead of
// all of them (RMAT-30 / 32 groups: the level's chunk pulls stream ~10^10 prefix entries at one
// word per vertex, and a wave otherwise waited for every tile's ids from HBM in turn).
template <int W, int T, int HUBW>
__device__ __forceinline__ void chunk_pull_pfx(int32_t v, int64_t beg, int64_t lim,
                                               const int32_t* col, const uint64_t* R,
                                               const V<Lay<W>::VW>& am, uint64_t* acc,
                                               const uint32_t* hub, int32_t* lst,
                                               const uint32_t* snap) {
  static_assert(HUBW > 0, "the prefix chunks probe the LDS hub bitmap");
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, S = L::VPW;
  constexpr int PB = VW == 2 ? 4 : 8;  // rows in flight per lane group in phase B
  constexpr int Q = T / 64;
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int64_t vo = (int64_t)v * W + slot * VW;
  const V<VW> r = (snap && !any_visited(snap, v)) ? vzero<VW>() : ldv<VW>(R + vo);
  V<VW> unv, a = vzero<VW>();
  bool lane_open = false;
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    unv.w[j] = ~r.w[j] & am.w[j];
    lane_open |= unv.w[j] != 0;
  }
  if (!__ballot(lane_open)) return;  // wave-uniform
  // ids of the tile at t0 (16-byte aligned): lane l takes entries t0 + 4l .. t0 + 4l + 3 with
  // one aligned 16-byte load (a quarter of the address work of four 4-byte loads; a window past
  // the chunk reads the chunk's first one instead, and an aligned window holding a valid entry
  // never leaves its page), entries outside [beg, lim) are -1
  static_assert(Q == 4, "one 16-byte window per lane");
  typedef int32_t i4 __attribute__((ext_vector_type(4)));
  const int64_t a0 = beg & ~(int64_t)3;
  auto load_ids = [&](int64_t t0, int32_t (&u)[Q]) {
    const int64_t e = t0 + 4 * lane;
    const i4 w = *(const i4*)(col + (e < lim ? e : a0));
    const int32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < Q; ++q) u[q] = (e + q >= beg && e + q < lim) ? x[q] : -1;
  };
  int32_t un[Q];
  load_ids(a0, un);
  bool covered = false;
  for (int64_t t0 = a0; t0 < lim && !covered; t0 += T) {
    int32_t u[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) u[q] = un[q];
    load_ids(t0 + T, un);  // (past the end: clamped, unused)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t h = hub[(u[q] >= 0 ? u[q] : 0) >> 5];
      if (u[q] >= 0 && !((h >> (u[q] & 31)) & 1u)) u[q] = -1;
    }
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint64_t m = __ballot(u[q] >= 0);
      if (u[q] >= 0) lst[cnt + __popcll(m & lanemask_lt())] = u[q];
      cnt += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    for (int b = 0; b < cnt; b += PB * S) {
      int32_t uu[PB];
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int k = b + q * S + sub;
        const int32_t x = lst[k < cnt ? k : 0];
        uu[q] = k < cnt ? x : -1;
      }
      // (idle lanes load nothing: their address costs the address unit as much as a row)
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
    // one cross-group OR and coverage check per tile
#pragma unroll
    for (int off = G; off < 64; off <<= 1)
#pragma unroll
      for (int j = 0; j < VW; ++j) a.w[j] |= __shfl_xor(a.w[j], off);
    bool cov = true;
#pragma unroll
    for (int j = 0; j < VW; ++j) cov &= (a.w[j] & unv.w[j]) == unv.w[j];
    if (!__ballot(!cov)) covered = true;
    __builtin_amdgcn_wave_barrier();  // lst is rewritten by the next tile
  }
  if (sub == 0) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const uint64_t nb = a.w[j] & unv.w[j];
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
static __global__ __launch_bounds__(kBlock) void k_prefix_lens(const int64_t* rowptr, const int32_t* col,
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
static __global__ __launch_bounds__(kBlock) void k_first_nbr(const int64_t* rowptr, const int32_t* col,
                                                      int64_t n, int32_t* first) {
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n;
       v += (int64_t)gridDim.x * kBlock) {
    const int64_t b = rowptr[v];
    first[v] = rowptr[v + 1] > b ? col[b] : -1;
  }
}

// chunk counts of the wide vertices' row prefixes (inclusive-scanned into offs by the host)
static __global__ __launch_bounds__(kBlock) void k_prefix_chunks(const int32_t* wl, int64_t nw,
                                                          const int32_t* plen, int64_t* cnt) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nw;
       i += (int64_t)gridDim.x * kBlock)
    cnt[i] = ((int64_t)plen[wl[i]] + kChunk - 1) / kChunk;
}

// plen != nullptr: chunks cover only the row prefixes with ids < H (prefix-pull level)
static __global__ __launch_bounds__(kBlock) void k_chunk_desc(const int32_t* wl, int64_t nw,
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

// Two-pass chunk scheduling on the early-exit levels (tuning key chunk2): pass 1 pulls only the
// first chunk of every wide vertex (most are covered by the hubs at the head of their sorted
// rows), pass 2 only the remaining chunks of the vertices pass 1 left open. In one pass every
// chunk of a covered vertex still cost its wave an own-row load and a returning atomic before
// it could skip (RMAT-26 level 3: 313K wide vertices, ~1M+ chunks, 0.5 ms).
static __global__ __launch_bounds__(kBlock) void k_chunk_first(const int32_t* wl, int64_t nw,
                                                               const int64_t* rowptr,
                                                               ChunkDesc* desc, int64_t* cnt) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nw;
       i += (int64_t)gridDim.x * kBlock) {
    const int32_t v = wl[i];
    const int64_t b = rowptr[v], e = rowptr[v + 1];
    desc[i] = ChunkDesc{v, (uint32_t)b, (uint32_t)((uint64_t)b >> 32),
                        (int32_t)min((int64_t)kChunk, e - b)};
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *cnt = nw;
}
// chunks left of wide vertex i after pass 1: 0 once acc[v] (the union its chunks published)
// covers every alive group v misses, else all but the first (G lanes per vertex)
template <int W>
__global__ __launch_bounds__(kBlock) void k_chunk_rest_count(
    const int32_t* wl, int64_t nw, const int64_t* rowptr, const uint64_t* R, const uint64_t* acc,
    const uint64_t* alive, const uint64_t* gmask, const uint32_t* snap, int64_t* cnt) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  const int lane = lane_id(), slot = lane % G, sub = lane / G, wv = threadIdx.x >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nw; tb += (int64_t)gridDim.x * TILE) {
    const int64_t i = tb + wv * VPW + sub;
    bool open = false;
    int32_t v = 0;
    if (i < nw) {
      v = wl[i];
      const int64_t vo = (int64_t)v * W + slot * VW;
      const V<VW> r = (snap && !any_visited(snap, v)) ? vzero<VW>() : ldv<VW>(R + vo);
      const V<VW> a = ldv<VW>(acc + vo);
#pragma unroll
      for (int j = 0; j < VW; ++j) open |= (~r.w[j] & am.w[j] & ~a.w[j]) != 0;
    }
    const bool g_open = (__ballot(open) >> (sub * G)) & L::GBITS;
    if (i < nw && slot == 0) {
      const int64_t d = rowptr[v + 1] - rowptr[v];
      const int64_t nc = (d + kChunk - 1) / kChunk;
      cnt[i] = g_open && nc > 1 ? nc - 1 : 0;
    }
  }
}
// descriptors of the pass-2 chunks (offs = inclusive prefix of k_chunk_rest_count)
static __global__ __launch_bounds__(kBlock) void k_chunk_rest_desc(const int32_t* wl, int64_t nw,
                                                                   const int64_t* offs,
                                                                   const int64_t* rowptr,
                                                                   ChunkDesc* desc) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nw;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t c0 = i ? offs[i - 1] : 0, c1 = offs[i];
    if (c0 == c1) continue;
    const int32_t v = wl[i];
    const int64_t b = rowptr[v], e = rowptr[v + 1];
    for (int64_t c = c0; c < c1; ++c) {
      const int64_t cb = b + (1 + c - c0) * kChunk;
      desc[c] = ChunkDesc{v, (uint32_t)cb, (uint32_t)((uint64_t)cb >> 32),
                          (int32_t)min((int64_t)kChunk, e - cb)};
    }
  }
}

// PFXL: the chunks of a prefix-pull level without codes (chunk_pull_pfx)
template <int W, int T, int BT, int HUBW, bool PFXL = false>
__global__ __launch_bounds__(BT, (BT >= 1024 && HUBW <= 16384) ? 8 : 4) void k_bu_chunks(
    const ChunkDesc* __restrict__ desc, const int64_t* nchunks_p, const int32_t* col,
    const uint64_t* R,
    const uint64_t* alive, const uint64_t* gmask, uint64_t* acc, const uint32_t* anyvis,
    int32_t filter_from, int coop, const uint32_t* code, int32_t code_from,
    const uint32_t* snap, const uint32_t* dsnap = nullptr) {
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
    if constexpr (PFXL)
      chunk_pull_pfx<W, T, HUBW>(v, beg, lim, col, R, am, acc, hub, lst, snap);
    else
      chunk_pull<W, T, HUBW>(v, beg, lim, col, R, am, acc, anyvis, hub, filter_from, coop,
                             lst, code, code_from, wacc[threadIdx.x >> 6], snap, dsnap);
  }
}

// bottom-up, wide vertices, phase 2: G lanes per vertex fold acc[v] into the visited words.
template <int W, bool COUNT, bool FUSE, bool FLB = false>
__global__ __launch_bounds__(kBlock) void k_bu_wide_finalize(
    const int32_t* wl, int64_t nw, const int64_t* rowptr, const uint64_t* R, uint64_t* Wb,
    uint64_t* acc, const uint64_t* alive, const uint64_t* gmask, uint32_t* done, int32_t* actw2,
    int32_t* fl2, Ctr* ctr, uint32_t* anyvis, int32_t* act2n, int next_wide, uint32_t* slabF,
    const uint32_t* snap, uint32_t* fbm = nullptr) {
  // fbm != nullptr (the tiled first pull level, see tiles.hpp): wl is the static big-vertex list,
  // so done vertices are skipped; no list queues: the new frontier goes into bitmap fbm and its
  // size into ctr->fl2, the next active lists come from k_build_active after the level.
  // FLB (with fbm, the narrow pull's FBM levels): wl is the level's wide active list; only the
  // frontier goes into fbm, the next active lists are built here as without fbm.
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  // done / any-visited bits: one atomic per word of the wave (wave_set_bits) where a wave
  // holds many vertices or many first visits (W = 16 levels 3-4 measured ~0.4 ms slower each)
  constexpr bool kCombine = G <= 4;
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
  uint32_t nfc = 0;
  __shared__ uint32_t scratch32[kWaves];
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nw; tb += (int64_t)gridDim.x * TILE) {
    const int64_t idx = tb + wv * VPW + sub;
    bool valid = idx < nw;
    int32_t v = 0;
    V<VW> nwb = vzero<VW>();
    bool anynew = false, notfull = false, rnz = false;
    uint32_t deg = 0;
    if (valid) {
      v = wl[idx];
      if (fbm && !FLB && is_done(done, v)) {
        // (the tiled level's tail push also pushes into done vertices: leave their acc row clean;
        // and give them their unchanged row in Wb, which k_push_tail_after filters against)
        const int64_t vo = (int64_t)v * W + slot * VW;
        stv<VW>(acc + vo, vzero<VW>());
        stv<VW>(Wb + vo, ldv<VW>(R + vo));
        valid = false;
      }
    }
    if (valid) {
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
    wave_set_bits<kCombine>(done, v, leader && !g_nf);
    const bool keep = leader && g_nf, app = leader && g_new;
    if (keep && (!fbm || FLB)) eu += deg;
    if (app) ef += deg;
    {
      const bool g_first = g_new && !((__ballot(rnz) >> (sub * G)) & L::GBITS);
      wave_set_bits<kCombine>(anyvis, v, leader && g_first);
      if (leader && g_first) ev += deg;
    }
    if (fbm) {  // (uniform)
      wave_set_bits<kCombine>(fbm, v, app);
      nfc += app ? 1u : 0u;
      if (!FLB) continue;
    } else {
      q_push(qf, app, v);
    }
    q_push(qa, keep && (int)deg > next_wide, v);
    q_push(qn, keep && (int)deg <= next_wide, v);
    q_flush_n<kQCap, 3>({&qa, &qn, &qf}, {actw2, act2n, fl2},
                        {&ctr->actw2.v, &ctr->act2.v, &ctr->fl2.v}, TILE, false);
  }
  q_flush_n<kQCap, 3>({&qa, &qn, &qf}, {actw2, act2n, fl2},
                      {&ctr->actw2.v, &ctr->act2.v, &ctr->fl2.v}, 0, true);
  if (fbm) block_sum_add32(nfc, &ctr->fl2.v, scratch32);
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

// counter slot 0 and alive mask 0 of a device-driven pull batch (bu_batch): the host's view
// after the level before the batch
static __global__ void k_bu_seed(Ctr* c0, uint32_t nf, unsigned long long ef, uint32_t nact,
                          uint32_t nactw, unsigned long long eu, const uint64_t* alive,
                          uint64_t* alive0) {
  if (threadIdx.x == 0) {
    c0->fl2.v = nf;
    c0->ef2.v = ef;
    c0->act2.v = nact;
    c0->actw2.v = nactw;
    c0->eu2.v = eu;
  }
  if (threadIdx.x < 16) alive0[threadIdx.x] = alive[threadIdx.x];
}

}  // namespace bp
}  // namespace msbfs
