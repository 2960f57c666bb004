// Bit-parallel MS-BFS: the first bottom-up level's prefix pull as an edge-streaming kernel over
// static vertex tiles (k_pfx_tiles), replacing the narrow lane-group pull and the hub chunks on
// that level.
//
// Why: the per-vertex pulls (k_bu_narrow, one lane group per vertex, 4-8 neighbours per step and
// a coverage ballot between steps) chain their loads (list entry -> offsets -> column ids ->
// probe -> rows) and sync the block for their list queues every tile; on RMAT-26 / 1024 groups
// the level-2 pulls run at about half the rate the chip gathers rows and codes at
// (profiles/gather_rates.md). The first pull level never exits early (hardly any vertex gets all
// its groups at level 2), so its work is a plain boolean SpMM over the row prefixes:
//     Y[v] = OR_{u in prefix(v), u visited} row(u)
// and can be streamed edge by edge with no per-vertex loop.
//
// Layout (built once per graph, prefix bound H and vertex partition; BitparSolver::pfx_tiles):
//   pent[] = every own vertex's prefix column ids (ids < H <= 2^19) in vertex order, packed as
//            u | vl << 19 with vl = the vertex's index inside its tile (< VT)
//   tiles  = consecutive own vertices (<= VT of them, ~kTileWeight entries + kVertexWeight per
//            vertex) with their entry range; a vertex with more than kBigPrefix entries gets
//            partial tiles of its own (kPartialEntries each) instead, whose results are OR-ed
//            into acc[v] and folded in by k_bu_wide_finalize over the big-vertex list.
// One wave per tile, no block barriers: entries are loaded 256 at a time (4 per lane,
// coalesced), probed against the LDS hub bitmap, single-group codes OR their bits into the
// wave's LDS accumulator rows, the rest are compacted and their rows gathered by lane groups
// (several rows in flight per group) and OR-ed into the accumulator rows. The epilogue is the
// narrow pull's (new bits, row store, counters, done / any-visited bits) minus the list
// queues: the frontier goes into a bitmap (materialised as a list only if a top-down level
// follows) and the next active lists come from one k_build_active pass after the level. The
// tail push before it (k_push_tail) runs without stamps or done tests: the level's acc rows are
// all-zero but the pushed ones, and every tile vertex (and big vertex) reads and clears its own.
// Used from 8 words on (4 words: no sparse codes, slower than the per-vertex pulls).
// RMAT-26 / 1024 groups: level 2 14.9 -> 12.3-12.5 ms (profiles/rmat26_tiles_counters.md).
#pragma once

#include "common.hpp"
#include "pull.hpp"

namespace msbfs {
namespace bp {

struct PfxTile {
  int32_t v0;   // first vertex
  int32_t nv;   // vertices (low 16 bits); kTilePartial: one vertex, a slice of its entries
  int64_t e0;   // first entry in pent (the next tile's e0 ends it)
};
constexpr int32_t kTilePartial = 1 << 16;
constexpr uint32_t kPentNone = 0xFFFFFFFFu;
constexpr int kPentUBits = 19;                     // u < 2^19 (H = 458752)
constexpr uint32_t kPentUMask = (1u << kPentUBits) - 1;
constexpr int kTileWeight = 1024;   // entries + kVertexWeight * vertices per tile (target)
constexpr int kBigPrefix = 1024;    // more prefix entries: partial tiles
constexpr int kPartialEntries = 1024;
constexpr int kTileBlock = 1024;    // one block per CU: the hub bitmap + 16 waves' rows
constexpr int kTileHubW = 14336;    // hub bitmap words (ids < 458752, the prefix bound)

// vertices per tile (the wave's accumulator rows: VT x W words, 4 KB at W = 16; the same tiles
// serve every word count) and the weight of a vertex besides its entries
constexpr int kTileVT = 32;
constexpr int kVertexWeight = kTileWeight / kTileVT;

// pent for the vertices of normal tiles (one wave per tile, the vertices one after another) and
// for the partial tiles of big vertices (their slice of the row prefix, vl = 0)
__global__ __launch_bounds__(256) void k_fill_pent(const PfxTile* tiles, int64_t ntiles,
                                                   int nparts, const int64_t* rowptr,
                                                   const int32_t* col, const int32_t* plen,
                                                   uint32_t* pent) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t = wave; t < ntiles; t += nw) {
    const PfxTile d = tiles[t];
    const int64_t e1 = tiles[t + 1].e0;
    if (d.nv & kTilePartial) {
      // slice [k0, k0 + (e1 - e0)) of the vertex's prefix: partial tiles of one vertex are
      // consecutive, the first one starts at the vertex's first entry
      int64_t first = t;
      while (first > 0 && (tiles[first - 1].nv & kTilePartial) && tiles[first - 1].v0 == d.v0)
        --first;
      const int64_t k0 = d.e0 - tiles[first].e0;
      const int64_t b = rowptr[d.v0] + k0;
      for (int64_t k = lane; k < e1 - d.e0; k += 64) pent[d.e0 + k] = (uint32_t)col[b + k];
      continue;
    }
    const int nv = d.nv & 0xFFFF;
    int64_t e = d.e0;
    for (int i = 0; i < nv; ++i) {
      const int32_t v = d.v0 + i * nparts;
      const int32_t p = plen[v];
      const int64_t b = rowptr[v];
      for (int k = lane; k < p; k += 64) pent[e + k] = (uint32_t)col[b + k] | ((uint32_t)i << kPentUBits);
      e += p;
    }
  }
}

// One round = up to kRound entries of one tile. Rounds are software-pipelined across the
// wave's tiles (tile t, t + nwaves, ...): while round r is processed, the packed entries of
// round r + 1 are in flight (the entry stream comes from HBM).
constexpr int kRoundQ = 4;                 // entries per lane per round
constexpr int kRound = 64 * kRoundQ;
struct TileRound {
  int64_t t, e, e0, e1;  // tile (>= ntiles: none), first entry, the tile's entry range
};
__device__ __forceinline__ TileRound tile_first_round(const PfxTile* tiles, int64_t ntiles,
                                                      int64_t t) {
  if (t >= ntiles) return TileRound{t, 0, 0, 0};
  const int64_t e0 = uni64(tiles[t].e0), e1 = uni64(tiles[t + 1].e0);
  return TileRound{t, e0, e0, e1};
}
__device__ __forceinline__ TileRound tile_next_round(const PfxTile* tiles, int64_t ntiles,
                                                     int64_t nwaves, const TileRound& r) {
  if (r.t >= ntiles) return r;
  if (r.e + kRound < r.e1) return TileRound{r.t, r.e + kRound, r.e0, r.e1};
  return tile_first_round(tiles, ntiles, r.t + nwaves);
}

// bit k = any lane of lane group k (G consecutive lanes) set in the wave mask m (uniform: SALU)
template <int G>
__device__ __forceinline__ uint32_t group_any(uint64_t m) {
  if constexpr (G == 8) {  // OR-fold each byte into its low bit, then gather the 8 bits
    m |= m >> 4;
    m |= m >> 2;
    m |= m >> 1;
    m &= 0x0101010101010101ull;
    m |= m >> 7;
    m |= m >> 14;
    m |= m >> 28;
    return (uint32_t)(m & 0xFFu);
  } else {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 64 / G; ++k)
      r |= (uint32_t)(((m >> (k * G)) & ((1ull << G) - 1)) != 0) << k;
    return r;
  }
}
// OR the bits of a 32-bit tile mask (bit i = vertex v0 + i) into bitmap bm (one lane)
__device__ __forceinline__ void tile_mask_or(uint32_t* bm, int32_t v0, uint32_t m) {
  if (!m) return;
  const int32_t w = v0 >> 5, sh = v0 & 31;
  atomicOr(&bm[w], m << sh);
  if (sh && (m >> (32 - sh))) atomicOr(&bm[w + 1], m >> (32 - sh));
}

// zrow: an all-zero row (the gather target of the idle lane groups of a batch)
// (One 1024-thread block per CU, bound by the LDS: the hub bitmap plus 16 waves' accumulator
// rows. Measured round 4: 256-thread blocks probing the global, L2-resident hub bitmap instead,
// 4 or 5 blocks per CU, ran level 2 in 14.1 / 15.4 ms against 12.5 ms here: the L2 round trip
// of every probe costs more than the extra waves hide.)
// ACC = false (tuning key push_after): the tail push runs after this kernel and ORs its bits
// into the output rows itself (k_push_tail_after), so no acc row is read here.
template <int W, bool ACC = true>
__global__ __launch_bounds__(kTileBlock, 1) void k_pfx_tiles(
    const PfxTile* __restrict__ tiles, int64_t ntiles, const uint32_t* __restrict__ pent,
    int nparts, const int64_t* rowptr, const uint64_t* R, uint64_t* O, uint64_t* acc,
    const uint32_t* pvis, const uint32_t* snap, const uint32_t* code, int32_t code_from,
    const uint64_t* alive, const uint64_t* gmask, uint32_t* done, uint32_t* anyvis, uint32_t* fbm,
    Ctr* ctr, uint32_t* slabF, const uint64_t* zrow) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, S = 64 / G, VT = kTileVT;
  static_assert(VPW <= kTileVT && kTileVT % VPW == 0, "whole epilogue passes per tile");
  constexpr int NWV = kTileBlock / 64;
  constexpr int PB = 4;       // rows in flight per lane group and batch
  constexpr int Q = kRoundQ;
  constexpr int CR = 65;      // bank-skewed counter rows (BitCounter::spill_strided)
  constexpr int YW = VT * W + 64;  // + one dummy word per lane (idle lanes' ORs, no conflicts)
  __shared__ uint32_t hub[kTileHubW];
  __shared__ unsigned long long Y[NWV][YW];
  __shared__ uint32_t lst[NWV][kRound];
  __shared__ uint32_t cnt[CR * W];
  for (int i = threadIdx.x; i < kTileHubW; i += kTileBlock) hub[i] = pvis[i];
  for (int i = threadIdx.x; i < CR * W; i += kTileBlock) cnt[i] = 0;
  __syncthreads();
  const int lane = lane_id(), slot = lane % G, sub = lane / G, wv = threadIdx.x >> 6;
  unsigned long long* y = Y[wv];
  const int dummy = VT * W + lane;
  uint32_t* ls = lst[wv];
  // alive & batch mask per word in LDS (read per epilogue pass: registers go to the counters)
  __shared__ unsigned long long amask[W];
  if (threadIdx.x < W) amask[threadIdx.x] = alive[threadIdx.x] & gmask[threadIdx.x];
  __syncthreads();
  // frontier count and degree sums per wave in LDS, added per tile from the tile masks (no
  // 64-bit per-lane accumulators live through the round loop: registers for the pipeline)
  __shared__ unsigned long long wef[NWV], wev[NWV];
  __shared__ uint32_t wnf[NWV];
  if (threadIdx.x < NWV) {
    wef[threadIdx.x] = 0;
    wev[threadIdx.x] = 0;
    wnf[threadIdx.x] = 0;
  }
  // 5 slices: a spill (one LDS add per set counter bit, ~100 per lane at level 2) every 31
  // passes (6 slices do not fit the 128 VGPRs of a 1024-thread block at 16 words)
  BitCounter<VW, 5> bc;
  bc.zero();
  int nadd = 0;
  const int64_t nwaves = (int64_t)gridDim.x * NWV;
  auto load_round = [&](const TileRound& r, uint32_t (&pk)[Q]) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t i = r.e + q * 64 + lane;
      pk[q] = (r.t < ntiles && i < r.e1) ? pent[i] : kPentNone;
    }
  };
  // probe (branch-free: the unused lanes read hub word 0) + code loads of a round
  auto probe_round = [&](uint32_t (&pk)[Q], uint32_t (&cd)[Q]) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t u = pk[q] != kPentNone ? pk[q] & kPentUMask : 0u;
      const bool hit = (hub[u >> 5] >> (u & 31)) & 1u;
      pk[q] = hit ? pk[q] : kPentNone;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) cd[q] = kDenseCode;
    if (code_from != INT32_MAX) {  // (uniform: no codes on this level, no code array)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint32_t u = pk[q] & kPentUMask;
        const bool coded = pk[q] != kPentNone && (int32_t)u >= code_from;
        const uint32_t c = code[coded ? u : (uint32_t)code_from];
        cd[q] = coded ? c : kDenseCode;
      }
    }
  };
  TileRound rc = tile_first_round(tiles, ntiles, (int64_t)blockIdx.x * NWV + wv);
  TileRound rb = tile_next_round(tiles, ntiles, nwaves, rc);  // (rc's successor)
  uint32_t pkc[Q], cdc[Q], pkb[Q];
  load_round(rc, pkc);
  while (rc.t < ntiles) {
    load_round(rb, pkb);    // entries of round r + 1 in flight
    probe_round(pkc, cdc);
    if (rc.e == rc.e0) {    // first round of a tile: clear the accumulator rows
#pragma unroll
      for (int k = lane; k < VT * W; k += 64) y[k] = 0;
      __builtin_amdgcn_wave_barrier();
    }
    // ---- round r: sparse codes straight into the accumulator rows (idle slots: dummy word)
    // (32-bit halves of the rows: one shift per bit; an idle slot ORs 0 into its lane's dummy)
    uint32_t* y32 = reinterpret_cast<uint32_t*>(y);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const bool coded = pkc[q] != kPentNone && cdc[q] != kDenseCode;
      const uint32_t vrow = (pkc[q] >> kPentUBits) * (2 * W);
      const uint32_t nset = cdc[q] >> 30;
#pragma unroll
      for (int i = 0; i < kCodeSlots; ++i) {
        const uint32_t g = (cdc[q] >> (10 * i)) & 1023u;
        const bool on = coded && (uint32_t)i < nset;
        atomicOr(&y32[on ? vrow + (g >> 5) : 2 * dummy], 1u << (g & 31));
      }
      pkc[q] = coded ? kPentNone : pkc[q];
    }
    // the rest: dense rows, compacted into the wave's list, gathered by lane groups
    int c = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const bool keep = pkc[q] != kPentNone;
      const uint64_t m = __ballot(keep);
      if (keep) ls[c + __popcll(m & lanemask_lt())] = pkc[q];
      c += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    for (int b = 0; b < c; b += PB * S) {
      uint32_t uu[PB];
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int k = b + q * S + sub;
        uu[q] = ls[k < c ? k : 0];
        uu[q] = k < c ? uu[q] : kPentNone;
      }
      V<VW> x[PB];
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const uint64_t* src = uu[q] != kPentNone
                                  ? R + (int64_t)(uu[q] & kPentUMask) * W + slot * VW
                                  : zrow + slot * VW;
        x[q] = ldv<VW>(src);
      }
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int base = uu[q] != kPentNone ? (int)(uu[q] >> kPentUBits) * W + slot * VW : -1;
#pragma unroll
        for (int j = 0; j < VW; ++j) atomicOr(&y[base >= 0 ? base + j : dummy], x[q].w[j]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (rc.e + kRound >= rc.e1) {  // last round of the tile
      const int32_t v0 = uni32(tiles[rc.t].v0);
      const int32_t nvf = uni32(tiles[rc.t].nv);
      if (nvf & kTilePartial) {
        // a slice of a big vertex: publish its bits (k_bu_wide_finalize folds them in)
        if (sub == 0) {
          const int64_t vo = (int64_t)v0 * W + slot * VW;
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const uint64_t a = y[slot * VW + j];
            if (a) atomicOr((unsigned long long*)&acc[vo + j], a);
          }
        }
      } else {
        // epilogue: VPW vertices per pass, G lanes each (the narrow pull's, without list
        // queues); done / frontier / first-visit bits collect in tile masks (bit i = vertex i).
        // Every load of the tile is issued before any is used: lane i fetches vertex i's row
        // offsets, stamp and bitmap words, every lane group its vertices' own rows; then the
        // pushed rows of the stamped vertices (one dependent round trip per tile, not per pass).
        const int nv = nvf & 0xFFFF;
        constexpr int NP = kTileVT / VPW;  // passes per tile
        const int32_t vlane = v0 + lane * nparts;
        int64_t rp0 = 0, rp1 = 0;
        uint32_t dwl = 0, swl = ~0u;
        if (lane < nv) {
          rp0 = rowptr[vlane];
          rp1 = rowptr[vlane + 1];
          dwl = done[vlane >> 5];
          swl = (snap ? snap : anyvis)[vlane >> 5];
        }
        const uint32_t degl = (uint32_t)(rp1 - rp0);
        const bool okl = lane < nv && degl > 0 && !((dwl >> (vlane & 31)) & 1u);
        // own row: only a vertex some group visited has a non-zero row (and in a lazy batch the
        // row of one nobody visited is stale): at level 2 that skips ~99 % of the own-row loads.
        // (anyvis bits of this tile's vertices change only in this epilogue, after the read)
        const bool visl = lane < nv && ((swl >> (vlane & 31)) & 1u);
        const uint64_t bok = __ballot(okl), bvis = __ballot(visl);
        // !ACC: vertices done before the level get their (unchanged) row in O as well, so the
        // tail push after the tiles needs no done probe (their rows already hold every alive
        // group: its plain-load filter skips them)
        const uint64_t bput = ACC ? bok : __ballot(lane < nv && degl > 0);
        uint32_t m_done = 0, m_new = 0, m_first = 0;
        // two passes per batch: own rows and pushed rows of 16 vertices in flight
        constexpr int NH = 1;
#pragma unroll
        for (int h = 0; h < NP; h += NH) {
          if (h * VPW >= nv) break;
          V<VW> rr[NH], pa[NH];
#pragma unroll
          for (int k = 0; k < NH; ++k) {
            const int i = (h + k) * VPW + sub;
            const int64_t vo = (int64_t)(v0 + i * nparts) * W + slot * VW;
            rr[k] = ((bvis >> i) & 1ull) ? ldv<VW>(R + vo) : vzero<VW>();
            // bits pushed by k_push_tail (no stamps: the level's acc rows are all-zero but
            // the pushed ones, and a tile's rows are one contiguous run; the push skips no done
            // vertex either, so every vertex of the tile reads and clears its row)
            pa[k] = ACC && i < nv ? ldv<VW>(acc + vo) : vzero<VW>();
          }
#pragma unroll
        for (int k = 0; k < NH; ++k) {
          const int pi = h + k;
          const int p = pi * VPW;
          if (p >= nv) break;
          const int i = p + sub;
          const int32_t v = v0 + i * nparts;
          const bool valid = (bok >> i) & 1ull;
          const bool put = (bput >> i) & 1ull;  // (valid, or done with edges when !ACC)
          V<VW> r = vzero<VW>(), a = vzero<VW>();
          if (put) r = rr[k];
          if (valid) {
#pragma unroll
            for (int j = 0; j < VW; ++j) a.w[j] = y[i * W + slot * VW + j] | pa[k].w[j];
          }
          {
            bool pushed = false;
#pragma unroll
            for (int j = 0; j < VW; ++j) pushed |= pa[k].w[j] != 0;
            if (ACC && pushed) stv<VW>(acc + (int64_t)v * W + slot * VW, vzero<VW>());
          }
          V<VW> nw, nvr;
          bool anynew = false, notfull = false, rnz = false;
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const uint64_t unv = ~r.w[j] & amask[slot * VW + j];
            nw.w[j] = valid ? a.w[j] & unv : 0;
            nvr.w[j] = r.w[j] | nw.w[j];
            anynew |= nw.w[j] != 0;
            notfull |= (unv & ~nw.w[j]) != 0;
            rnz |= r.w[j] != 0;
          }
          if (put) stv<VW>(O + (int64_t)v * W + slot * VW, nvr);
          bc.add(nw);
          if (++nadd == (1 << decltype(bc)::D) - 1) {
            bc.template spill_strided32<CR>(cnt, slot);
            nadd = 0;
          }
          // per-group flags (a group's lanes share validity; the others OR over its words),
          // compressed to one bit per group = per vertex of the pass
          const uint32_t gval = group_any<G>(__ballot(valid));
          const uint32_t gnew = group_any<G>(__ballot(anynew)) & gval;
          const uint32_t gnf = group_any<G>(__ballot(notfull));
          const uint32_t gfirst = gnew & ~group_any<G>(__ballot(rnz));
          m_done |= (gval & ~gnf) << p;
          m_new |= gnew << p;
          m_first |= gfirst << p;
        }
        }
        // (bit i of the masks = vertex i = lane i's degree; m_new / m_first hold valid vertices)
        if ((m_new >> lane) & 1u) atomicAdd(&wef[wv], (unsigned long long)degl);
        if ((m_first >> lane) & 1u) atomicAdd(&wev[wv], (unsigned long long)degl);
        if (lane == 0) wnf[wv] += (uint32_t)__popc(m_new);
        if (nparts == 1) {
          if (lane == 0) {
            tile_mask_or(done, v0, m_done);
            tile_mask_or(fbm, v0, m_new);
            tile_mask_or(anyvis, v0, m_first);
          }
        } else if (lane < nv) {  // (hybrid phase A: strided vertices, one bit each)
          const int32_t v = v0 + lane * nparts;
          if ((m_done >> lane) & 1u) atomicOr(&done[v >> 5], 1u << (v & 31));
          if ((m_new >> lane) & 1u) atomicOr(&fbm[v >> 5], 1u << (v & 31));
          if ((m_first >> lane) & 1u) atomicOr(&anyvis[v >> 5], 1u << (v & 31));
        }
      }
    }
    // shift the pipeline
    rc = rb;
    rb = tile_next_round(tiles, ntiles, nwaves, rb);
#pragma unroll
    for (int q = 0; q < Q; ++q) pkc[q] = pkb[q];
  }
  bc.template spill_strided32<CR>(cnt, slot);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    unsigned long long b = 0, c = 0;
    for (int w = 0; w < NWV; ++w) {
      a += wnf[w];
      b += wef[w];
      c += wev[w];
    }
    if (a) atomicAdd(&ctr->fl2.v, a);
    if (b) atomicAdd(&ctr->ef2.v, b);
    if (c) atomicAdd(&ctr->ev2.v, c);
  }
  uint32_t* row = slabF + (size_t)blockIdx.x * (64 * W);
  for (int i = threadIdx.x; i < 64 * W; i += kTileBlock) row[i] = cnt[i + (i >> 6)];
}

// frontier list from the frontier bitmap (LDS block queue; rare: only when a top-down level
// follows a tiled pull). Block-uniform loops: q_flush synchronises the block.
__global__ __launch_bounds__(kBlock) void k_bitmap_list(const uint32_t* bm, int64_t nwords,
                                                        int32_t* out, Ctr* ctr) {
  __shared__ LdsQueue q;
  q_init(q);
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t n = (nwords + stride - 1) / stride * stride;
  for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < n; w += stride) {
    uint32_t b = w < nwords ? bm[w] : 0u;
    for (int k = 0; k < 32; ++k) {  // at most one item per thread per step
      const bool has = b != 0;
      const int bit = has ? __ffs(b) - 1 : 0;
      if (has) b &= b - 1;
      q_push(q, has, (int32_t)(w * 32 + bit));
      q_flush(q, out, &ctr->touched.v, kBlock, false);
    }
  }
  q_flush(q, out, &ctr->touched.v, 0, true);
}

}  // namespace bp
}  // namespace msbfs
