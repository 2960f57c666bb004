// Bit-parallel MS-BFS: the full (unfiltered) pull of the later bottom-up levels — the second
// pull level on (RMAT-26 / 1024 groups: level 3, 32.5M active vertices, ~140M neighbour rows), the
// lean pass's overflow list and the device-driven pull batches (bu_batch).
//
// Same algorithm as k_bu_narrow without the probe / prefix / snapshot machinery (these levels load
// every neighbour row): G lanes per vertex, CS neighbours per step, early exit once every alive
// group is covered. Round-4 changes, from the level-3 ISA and counters of k_bu_narrow (5.6 ms,
// 3.0 TB/s, ~310 VALU per tile, six block barriers per tile):
//  * rows move branch-free: a neighbour slot past the end of the row (or a done neighbour) reads
//    the all-zero row n of the visited buffers (BitparSolver allocates n + 2 rows; levels()
//    clears rows n and n + 1 for the word count at hand);
//  * a step's column ids are broadcast inside the lane group with ds_swizzle (constant pattern,
//    all CS issued before the first use) instead of one ds_bpermute + wait + branch per row;
//  * the new lists (next active, next wide, new frontier) go through WAVE-private LDS queues with
//    one global atomic per flush (no __syncthreads in the tile loop: the four waves of a block
//    no longer wait for the slowest one every tile).
#pragma once

#include <utility>

#include "common.hpp"

namespace msbfs {
namespace bp {

// row u's slice of a lane at byte offset voff within the row (u < n + 2)
template <int W, int VW>
__device__ __forceinline__ V<VW> ld_row(const uint64_t* base, int32_t u, int voff) {
  return ldv<VW>(base + (int64_t)u * W + voff / 8);
}
template <int W, int VW>
__device__ __forceinline__ void st_row(uint64_t* base, int32_t u, int voff, const V<VW>& r) {
  stv<VW>(base + (int64_t)u * W + voff / 8, r);
}

// Value of lane (group base + K) for every lane of a group of G lanes (G <= 8 never crosses the
// 32-lane halves ds_swizzle's bitmask mode works in): and-mask keeps the group bits, or-mask
// selects the lane.
template <int G, int K>
__device__ __forceinline__ int32_t group_bcast(int32_t x) {
  static_assert(G >= 1 && G <= 32 && K < G, "group");
  if constexpr (G == 1) {
    return x;
  } else {
    constexpr int kAnd = 0x1F & ~(G - 1);
    return __builtin_amdgcn_ds_swizzle(x, kAnd | (K << 5));
  }
}
template <int G, int Q, int N, int... Ks>
__device__ __forceinline__ void bcast_ids(const int32_t (&u)[Q], int32_t (&uc)[N],
                                          std::integer_sequence<int, Ks...>) {
  ((uc[Ks] = group_bcast<G, Ks % G>(u[Ks / G])), ...);
}

// Done rows are never read (tuning key dskip, BitparSolver::level_bu): a vertex that is done (every
// alive group visited) has every group alive now, so a pull may OR the alive mask instead of its
// row. dsnap = the done bitmap as of the level start (a vertex done during this level may hold
// bits of this level; its row of the previous level is still valid and is read); a neighbour
// done in dsnap is probed (4 bytes) instead of gathered (8*W bytes), and with `skip` a vertex
// finishing at this level does not write its row at all (RMAT-26 levels 3-4: ~32M rows). The
// one reader that needs such a row, a push level right after, gets it from k_fix_done_rows.
__device__ __forceinline__ bool done_in(const uint32_t* snap, int32_t u) {
  return u >= 0 && ((snap[u >> 5] >> (u & 31)) & 1u);
}

// CS neighbours per step; C1 > 0: a first step of only C1 rows (late levels are mostly covered by
// the first neighbour, rows sorted hubs first). nact_dev: list length on the device (device-driven
// levels). gate: closed levels of a device-driven batch are no-ops. dsnap / skip: see above.
// Few words (W <= 4: phase C of the hybrid mode at 8 ranks, RMAT-30's 32-group passes): 4-row
// steps; up to 2 words also a 96-VGPR bound, five waves per SIMD (with 8-row steps: 110-128 VGPRs,
// four waves per SIMD, and the pull is latency-bound there).
template <int W>
constexpr int full_cs() { return W <= 4 ? 4 : 8; }
// PF: a step loads the column ids of the group's next step (from 4 words on; at 1-2 words the
// extra ids spilled registers). RMAT-26 / 1024 groups level 3: 5.30 -> 5.19 ms (round 5). (Five
// waves per SIMD with 512-entry queues spilled 37-47 VGPRs at 16 words: not kept.)
template <int W, int CS = full_cs<W>(), int C1 = 0>
__global__ __launch_bounds__(kBlock, W <= 2 ? 5 : 4) void k_bu_full(
    const int32_t* act, int64_t nact, const int64_t* rowptr, const int32_t* col,
    const uint64_t* R, uint64_t* Wb, int64_t n, const uint64_t* alive, const uint64_t* gmask,
    uint32_t* done, int32_t* act2, int32_t* fl2, Ctr* ctr, uint32_t* anyvis, int32_t* actw2,
    int next_wide, uint32_t* slabF, const uint32_t* nact_dev, BuGate gate,
    const uint32_t* dsnap, int flags) {
  if (!bu_gate_open(gate)) return;  // (uniform)
  const bool skip = flags & kFlagSkipRows;
  constexpr bool PF = W >= 4;
  if (nact_dev) nact = (int64_t)*nact_dev;
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  constexpr int C = CS;
  constexpr int Q = C / G > 0 ? C / G : 1;  // ids loaded per lane per step
  static_assert(G * Q == C, "a step is whole lane groups");
  static_assert(C1 == 0 || C1 <= C, "short first step");
  constexpr bool kCombine = G <= 4;
  // per-wave queues: next narrow active list, new frontier, next wide list. A flush (one
  // same-address atomic, ~12 ns each at the memory side, serialised per counter) comes when
  // another tile's pushes might not fit; 1024-item queues keep them at about the round-3 block
  // queues' count (448-item ones made level 3 pay ~170K of them) and fill the LDS of four
  // blocks per CU (the VGPR bound) exactly (768 for up to 2 words: five blocks per CU).
  constexpr int QA = W <= 2 ? 768 : 1024, QF = QA, QW = 2 * VPW > 128 ? 2 * VPW : 128;
  static_assert(QW >= 2 * VPW, "a wide push always fits after a flush");
  __shared__ int32_t qmem[kWaves][QA + QF + QW];
  __shared__ unsigned long long scratch[kWaves];
  __shared__ uint32_t wbase[kWaves + 1];
  constexpr int CR = 65;  // bank-skewed counter rows (BitCounter::spill_strided)
  __shared__ uint32_t cnt[CR * W];
  for (int i = threadIdx.x; i < CR * W; i += kBlock) cnt[i] = 0;
  __syncthreads();
  const int lane = lane_id(), slot = lane % G, sub = lane / G;
  const int wv = threadIdx.x >> 6;
  int32_t* qa = qmem[wv];
  int32_t* qf = qa + QA;
  int32_t* qw = qf + QF;
  uint32_t na = 0, nf = 0, nw = 0;  // (wave-uniform)
  const uint64_t* rR = R;
  uint64_t* rO = Wb;
  const int voff = slot * VW * 8;
  const int32_t zrow = (int32_t)n;  // the all-zero row (n <= INT32_MAX - 2, see the solver)
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  unsigned long long eu = 0, ef = 0, ev = 0;
  // Carry-save group counters: 7 slices (a spill every 127 tiles) at 16 words, spilled on
  // 32-bit halves (~12 VALU per set counter bit instead of ~28: level 3 spills find most
  // counter bits set, ~50 VALU per tile with 6 slices and 64-bit spills); 5 slices for few
  // words (one spill every 31 tiles, the 96-VGPR bound)
  BitCounter<VW, W <= 4 ? 5 : (W >= 16 ? 7 : 6)> bc;
  bc.zero();
  int nadd = 0;
  // software pipeline (as k_bu_narrow): list entry two tiles ahead, own row / offsets one tile
  // ahead, the first step's column ids one tile ahead (loaded at the end of the previous tile)
  const int64_t stride = (int64_t)gridDim.x * TILE, lofs = wv * VPW + sub;
  int64_t tb = (int64_t)blockIdx.x * TILE;
  int32_t v1 = -1, v2 = -1;
  if (tb + lofs < nact) v1 = act[tb + lofs];
  if (tb + stride + lofs < nact) v2 = act[tb + stride + lofs];
  // Every prefetch below is an unconditional load from a clamped index (an invalid lane reads
  // row / offsets / column entry 0) with the result selected after: a load under a branch made
  // the compiler wait for it at the branch's end (s_waitcnt vmcnt(0) across basic blocks), which
  // undid the pipeline (round-3 k_bu_narrow waited for its prefetched offsets on the spot).
  V<VW> r1 = ld_row<W, VW>(rR, v1 >= 0 ? v1 : zrow, voff);
  int64_t b1 = rowptr[v1 >= 0 ? v1 : 0], e1 = rowptr[(v1 >= 0 ? v1 : 0) + 1];
  if (v1 < 0) e1 = b1;
  constexpr int F1 = C1 > 0 ? C1 : C;  // neighbours of the first step
  // column entries [b, b + F1) of a row [b, e): slot q*G + lane's entry, -1 past the end
  // (one lane per vertex and four-entry steps: col4_aligned)
  constexpr bool A4 = G == 1 && Q == 4;
  auto first_ids = [&](int64_t b, int64_t e, int32_t (&u)[Q]) {
    if constexpr (A4 && F1 == 4) {
      col4_aligned(col, b, e, u);
      return;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int k = q * G + slot;
      const bool ok = k < F1 && b + k < e;
      const int32_t x = col[ok ? b + k : 0];
      u[q] = ok ? x : -1;
    }
  };
  // done-probe words of ids u (a dsnap word; 0 without probes or for -1)
  auto probe_words = [&](const int32_t (&u)[Q], uint32_t (&pd)[Q]) {
#pragma unroll
    for (int q = 0; q < Q; ++q) pd[q] = 0u;
    if (dsnap) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint32_t w = dsnap[(u[q] >= 0 ? u[q] : 0) >> 5];
        pd[q] = u[q] >= 0 ? w : 0u;
      }
    }
  };
  // column entries [e, e + C) of a row ending at `end`: slot q*G + lane's entry, -1 past the end
  auto step_ids = [&](int64_t e, int64_t end, int32_t (&u)[Q]) {
    if constexpr (A4) {
      col4_aligned(col, e < end ? e : 0, e < end ? end : 0, u);
      return;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t ee = e + q * G + slot;
      const int32_t x = col[ee < end ? ee : 0];
      u[q] = ee < end ? x : -1;
    }
  };
  int32_t un[Q];    // ids of the group's next continuation step (PF)
  int32_t u1[Q];
  uint32_t pd1[Q];  // dsnap words of u1 (the done probe, loaded a tile ahead too)
  first_ids(b1, e1, u1);
  probe_words(u1, pd1);
  for (; tb < nact; tb += stride) {
    const int64_t idx = tb + lofs;
    const bool valid = idx < nact;
    const int32_t v = valid ? v1 : 0;
    const V<VW> r = r1;
    const int64_t beg = b1, end = e1;
    const uint32_t deg = (uint32_t)(e1 - b1);
    int32_t u0[Q];
    uint32_t pd0[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      u0[q] = u1[q];
      pd0[q] = pd1[q];
    }
    // prefetch: row / offsets of the next tile, list entry of the one after
    v1 = idx + stride < nact ? v2 : -1;
    r1 = ld_row<W, VW>(rR, v1 >= 0 ? v1 : zrow, voff);
    b1 = rowptr[v1 >= 0 ? v1 : 0];
    e1 = rowptr[(v1 >= 0 ? v1 : 0) + 1];
    {
      const int64_t i2 = idx + 2 * stride;
      const int32_t a2 = act[i2 < nact ? i2 : 0];
      v2 = i2 < nact ? a2 : v2;
    }
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
    bool g_open = valid && ((__ballot(lane_open) >> (sub * G)) & L::GBITS);
    const bool g_first_step = g_open;
    if (g_open) {
      // first step: the preloaded ids (F1 of them)
      {
        if (dsnap) {  // (uniform) done neighbours: the alive mask instead of their rows
          bool hit = false;
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (u0[q] >= 0 && ((pd0[q] >> (u0[q] & 31)) & 1u)) {
              u0[q] = -1;
              hit = true;
            }
          if ((__ballot(hit) >> (sub * G)) & L::GBITS)
#pragma unroll
            for (int j = 0; j < VW; ++j) acc.w[j] = am.w[j];
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) u0[q] = u0[q] >= 0 ? u0[q] : zrow;
        int32_t uc[F1];
        bcast_ids<G, Q, F1>(u0, uc, std::make_integer_sequence<int, F1>{});
        V<VW> x[F1];
#pragma unroll
        for (int c = 0; c < F1; ++c) {
          // (only the slots some vertex of the wave has: degree-sorted lists make a wave's
          // degrees alike, and every issued slot costs the address unit a full instruction;
          // gathering all F1 slots ran level 3 at 76 % TA busy)
          x[c] = vzero<VW>();
          if (__ballot(beg + c < end)) x[c] = ld_row<W, VW>(rR, uc[c], voff);
        }
        // (the next tile's first-step ids behind the rows: waiting for the rows leaves them in
        // flight; their offsets were loaded at the top of this tile)
        if (v1 < 0) e1 = b1;
        first_ids(b1, e1, u1);
        // and the ids of this vertex's second step: a group the first step leaves open issues
        // its next rows without another round trip for the column ids
        if (PF) step_ids(beg + F1, end, un);
        bool cov = true;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
#pragma unroll
          for (int c = 0; c < F1; ++c) acc.w[j] |= x[c].w[j];
          cov &= (acc.w[j] & unv.w[j]) == unv.w[j];
        }
        g_open = (__ballot(!cov) >> (sub * G)) & L::GBITS;
      }
      for (int64_t e = beg + F1; g_open && e < end; e += C) {
        int32_t u[Q];
        if (PF) {  // (loaded one step ahead; the next step's now)
#pragma unroll
          for (int q = 0; q < Q; ++q) u[q] = un[q];
          step_ids(e + C, end, un);
        } else {
          step_ids(e, end, u);
        }
        if (dsnap) {
          uint32_t pd[Q];
          probe_words(u, pd);
          bool hit = false;
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (u[q] >= 0 && ((pd[q] >> (u[q] & 31)) & 1u)) {
              u[q] = -1;
              hit = true;
            }
          if ((__ballot(hit) >> (sub * G)) & L::GBITS)
#pragma unroll
            for (int j = 0; j < VW; ++j) acc.w[j] |= am.w[j];
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) u[q] = u[q] >= 0 ? u[q] : zrow;
        int32_t uc[C];
        bcast_ids<G, Q, C>(u, uc, std::make_integer_sequence<int, C>{});
        V<VW> x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          x[c] = vzero<VW>();
          if (__ballot(e + c < end)) x[c] = ld_row<W, VW>(rR, uc[c], voff);
        }
        bool cov = true;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
#pragma unroll
          for (int c = 0; c < C; ++c) acc.w[j] |= x[c].w[j];
          cov &= (acc.w[j] & unv.w[j]) == unv.w[j];
        }
        // the group runs this loop in lock step (same v); it stops when all its lanes are covered
        g_open = (__ballot(!cov) >> (sub * G)) & L::GBITS;
      }
    }
    if (!g_first_step) {  // (no first step ran for this group: the next tile's ids now)
      if (v1 < 0) e1 = b1;
      first_ids(b1, e1, u1);
    }
    V<VW> nwv;
    bool anynew = false, notfull = false;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      nwv.w[j] = acc.w[j] & unv.w[j];
      anynew |= nwv.w[j] != 0;
      notfull |= (unv.w[j] & ~nwv.w[j]) != 0;
    }
    const uint64_t bn = __ballot(anynew), bf = __ballot(notfull);
    const bool g_new = (bn >> (sub * G)) & L::GBITS;
    const bool g_nf = (bf >> (sub * G)) & L::GBITS;
    {  // also when nothing is open: Wb may hold the previous batch's rows
      // (skip: a vertex done now is never read again, see above; a store under a branch costs
      // no wait, and no idle lane hammers the scratch row's one cache line)
      V<VW> nv;
#pragma unroll
      for (int j = 0; j < VW; ++j) nv.w[j] = r.w[j] | nwv.w[j];
      if (valid && (g_nf || !skip)) st_row<W, VW>(rO, v, voff, nv);
    }
    bc.add(nwv);  // (zero for invalid lanes)
    if (++nadd == (1 << decltype(bc)::D) - 1) {
      bc.template spill_strided32<CR>(cnt, slot);
      nadd = 0;
    }
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
    // third stage: the done probe of the next tile's first-step ids (loaded during this tile)
    probe_words(u1, pd1);
    wq_push(qa, na, keep && (int)deg <= next_wide, v);
    wq_push(qw, nw, keep && (int)deg > next_wide, v);
    wq_push(qf, nf, app, v);
    if (na + VPW > QA) wq_flush(qa, na, act2, &ctr->act2.v);
    if (nw + VPW > QW) wq_flush(qw, nw, actw2, &ctr->actw2.v);
    if (nf + VPW > QF) wq_flush(qf, nf, fl2, &ctr->fl2.v);
  }
  // the rest of every wave's queues: one atomic per block and list (a block barrier is free at
  // the end; per-wave atomics here were 3 x 8192 on three addresses)
  wq_flush_block(qa, na, act2, &ctr->act2.v, wbase);
  wq_flush_block(qw, nw, actw2, &ctr->actw2.v, wbase);
  wq_flush_block(qf, nf, fl2, &ctr->fl2.v, wbase);
  block_sum_add(eu, &ctr->eu2.v, scratch);
  block_sum_add(ef, &ctr->ef2.v, scratch);
  block_sum_add(ev, &ctr->ev2.v, scratch);
  bc.template spill_strided32<CR>(cnt, slot);
  __syncthreads();
  uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
  for (int i = threadIdx.x; i < 64 * W; i += kBlock) row[i] = cnt[i + (i >> 6)];
}

// A push level after a pull level that skipped the rows of its finishing vertices (dskip) reads
// the frontier's new bits as Wrow & ~Rrow: restore Wrow[v] = Rrow[v] | am for the frontier
// vertices that finished (done) at that level (their new bits were exactly am & ~Rrow[v]).
template <int W>
__global__ __launch_bounds__(kBlock) void k_fix_done_rows(const int32_t* fl, const uint32_t* nf_dev,
                                                          int64_t nf, const uint32_t* done,
                                                          const uint64_t* Rrow, uint64_t* Wrow,
                                                          const uint64_t* alive,
                                                          const uint64_t* gmask) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  if (nf_dev) nf = (int64_t)*nf_dev;
  const int lane = lane_id(), slot = lane % G, sub = lane / G, wv = threadIdx.x >> 6;
  V<VW> am;
#pragma unroll
  for (int j = 0; j < VW; ++j) am.w[j] = alive[slot * VW + j] & gmask[slot * VW + j];
  for (int64_t tb = (int64_t)blockIdx.x * TILE; tb < nf; tb += (int64_t)gridDim.x * TILE) {
    const int64_t i = tb + wv * VPW + sub;
    if (i >= nf) continue;
    const int32_t v = fl[i];
    if (!is_done(done, v)) continue;
    const int64_t o = (int64_t)v * W + slot * VW;
    V<VW> r = ldv<VW>(Rrow + o);
#pragma unroll
    for (int j = 0; j < VW; ++j) r.w[j] |= am.w[j];
    stv<VW>(Wrow + o, r);
  }
}

}  // namespace bp
}  // namespace msbfs
