// Bit-parallel MS-BFS: hybrid multi-GPU mode kernels (exchange packing, zero-word coding,
// receiver setup) and the vertex-extent reduction.
#pragma once

#include "common.hpp"

namespace msbfs {
namespace bp {

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
// never reads them either). G lanes per vertex (the row layout): one degree test and one 8*VW-byte
// row load per lane; a destination's words of consecutive vertices are contiguous, so the lanes
// of one slot store adjacent runs (one word per thread with a 64-bit divide and a degree test per
// word took 0.32 ms per rank at 8 ranks on RMAT-26)
// (only own-vertex indices i in [i0, i1): a chunked phase A packs each range when it is final)
template <int W>
__global__ __launch_bounds__(kBlock) void k_pack_words(const uint64_t* vis, const int64_t* rowptr,
                                                       int part, int nparts, int64_t cnt, int wt,
                                                       WordSplit ws, uint64_t* send, int64_t i0,
                                                       int64_t i1) {
  using L = Lay<W>;
  constexpr int VW = L::VW, G = L::G, VPW = L::VPW, TILE = L::TILE;
  const int lane = lane_id(), slot = lane % G, sub = lane / G, wv = threadIdx.x >> 6;
  // destination of each of this lane's words (fixed for the whole kernel)
  int dj[VW], doff[VW], dnw[VW];
#pragma unroll
  for (int k = 0; k < VW; ++k) {
    const int w = slot * VW + k;
    int j = 0;
    if (w < wt)
      while (w >= ws.b[j + 1]) ++j;  // (w < wt = ws.b[nparts]: ends at a real part)
    dj[k] = j;
    dnw[k] = ws.b[j + 1] - ws.b[j];
    doff[k] = w - ws.b[j];
  }
  for (int64_t tb = i0 + (int64_t)blockIdx.x * TILE; tb < i1; tb += (int64_t)gridDim.x * TILE) {
    const int64_t i = tb + wv * VPW + sub;
    if (i >= i1) continue;
    const int64_t v = part + i * nparts;
    const bool deg0 = rowptr[v + 1] == rowptr[v];
    const V<VW> r = deg0 ? vzero<VW>() : ldv<VW>(vis + v * W + slot * VW);
#pragma unroll
    for (int k = 0; k < VW; ++k)
      if (slot * VW + k < wt) send[cnt * ws.b[dj[k]] + i * dnw[k] + doff[k]] = r.w[k];
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
                                                         int32_t* actw, Ctr* ctr, int pshift) {
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
      // (a power-of-two part count splits v with a mask and a shift, not a 64-bit division)
      const int64_t part = pshift >= 0 ? (v & (nparts - 1)) : v % nparts;
      const int64_t idx = pshift >= 0 ? (v >> pshift) : v / nparts;
      const uint64_t* src = recv + (pre.b[part] + idx) * nw;
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
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        nz |= x.w[j] != 0;
        full &= (~x.w[j] & am.w[j]) == 0;
      }
    }
    const bool g_nz = (__ballot(nz) >> (sub * G)) & L::GBITS;
    const bool g_full = !((__ballot(!full) >> (sub * G)) & L::GBITS);
    // the level-3 output buffer needs the rows of the vertices done now only: every active one
    // gets its row from the level-3 pull (or is skipped there, dskip3, and never read again)
    if (v < n_eff && g_full) stv<VW>(visB + v * W + slot * VW, x);
    if (slot == 0) {
      fullf[wv * VPW + sub] = v < n_eff && g_full;
      nzf[wv * VPW + sub] = g_nz;
    }
    const bool actv = slot == 0 && v < n_eff && deg > 0 && !g_full;
    if (actv) eu += (unsigned long long)deg;
    q_push(qn, actv && deg <= wide_deg, (int32_t)v);
    q_push(qw, actv && deg > wide_deg, (int32_t)v);
    q_flush_n<2048, 2>({&qn, &qw}, {act, actw}, {&ctr->act2.v, &ctr->actw2.v}, TILE, false);
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

}  // namespace bp
}  // namespace msbfs
