// Bit-parallel MS-BFS: top-down (push) level kernels — load-balanced edge-parallel expansion,
// the low-degree vertex-parallel expansion, finalize, and the one-kernel fused level of the
// device-driven batches (road-like graphs).
#pragma once

#include "common.hpp"

namespace msbfs {
namespace bp {

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

}  // namespace bp
}  // namespace msbfs

