// Bit-parallel MS-BFS solver: the first pull level's prefix pull over static vertex tiles
// (kernels and rationale: bitpar/tiles.hpp). Tiles are built once per graph, word count and
// vertex partition (prepare(), or the first hybrid phase A of a partition), outside any timed
// run.
#include <algorithm>
#include <vector>

#include "bitpar/init.hpp"
#include "bitpar/solver.hpp"
#include "bitpar/tiles.hpp"

namespace msbfs {
namespace bp {

namespace {
void greedy_tiles(const std::vector<int32_t>& plen, int64_t cnt, int part, int nparts,
                  std::vector<PfxTile>& tiles, std::vector<int32_t>& big, int64_t& nent) {
  constexpr int VT = kTileVT, VWT = kVertexWeight;
  int64_t e = 0;
  int32_t v0 = 0;
  int nv = 0;
  int64_t w = 0, te0 = 0;
  auto close = [&] {
    if (nv > 0) tiles.push_back(PfxTile{v0, nv, te0});
    nv = 0;
    w = 0;
  };
  for (int64_t i = 0; i < cnt; ++i) {
    const int32_t v = (int32_t)(part + i * nparts);
    const int64_t p = plen[(size_t)i];
    if (p > kBigPrefix) {
      close();
      big.push_back(v);
      for (int64_t k = 0; k < p; k += kPartialEntries) {
        tiles.push_back(PfxTile{v, kTilePartial | 1, e});
        e += std::min<int64_t>(kPartialEntries, p - k);
      }
      continue;
    }
    if (nv == VT || (nv > 0 && w + p + VWT > kTileWeight)) close();
    if (nv == 0) {
      v0 = v;
      te0 = e;
    }
    ++nv;
    w += p + VWT;
    e += p;
  }
  close();
  tiles.push_back(PfxTile{0, 0, e});  // sentinel: ends the last tile
  nent = e;
}

__global__ void k_gather_plen(const int32_t* plen, int64_t cnt, int part, int nparts,
                              int32_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = plen[part + i * nparts];
}
}  // namespace

const BitparSolver::TileSet* BitparSolver::pfx_tiles(int W, int part, int nparts, hipStream_t s) {
  if (!tiles_ok_ || !tun_.tiles) return nullptr;
  // (4 words: no sparse codes, every visited hub's row gathered: RMAT-26 / 256 groups ran
  // level 2 in 9.7 ms tiled vs 7.4 ms per vertex)
  if (W < 4 || W < tun_.tiles_w) return nullptr;
  for (auto it = tilesets_.begin(); it != tilesets_.end();) {
    TileSet& T = **it;
    if (T.key[0] != (const void*)g_.rowptr || T.key[1] != (const void*)g_.col) {
      it = tilesets_.erase(it);  // (an older graph buffer: relabelled or replaced)
      continue;
    }
    if (T.part == part && T.nparts == nparts) return &T;
    ++it;
  }
  constexpr int32_t kPfxH = kTileHubW * 32;
  const int32_t* plen = prefix_lens(kPfxH, s);
  const int64_t ne = n_eff(), cnt = ne > part ? (ne - part + nparts - 1) / nparts : 0;
  std::vector<int32_t> hp((size_t)std::max<int64_t>(cnt, 1));
  {
    DevBuf d((size_t)std::max<int64_t>(cnt, 1) * sizeof(int32_t));
    if (cnt > 0) {
      k_gather_plen<<<grid_for(cnt, 256, 8192), 256, 0, s>>>(plen, cnt, part, nparts,
                                                              d.as<int32_t>());
      MSBFS_HIP_CHECK(hipGetLastError());
      MSBFS_HIP_CHECK(hipMemcpyAsync(hp.data(), d.p, (size_t)cnt * sizeof(int32_t),
                                     hipMemcpyDeviceToHost, s));
    }
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  std::vector<PfxTile> tl;
  std::vector<int32_t> big;
  int64_t nent = 0;
  greedy_tiles(hp, cnt, part, nparts, tl, big, nent);
  const size_t pb = (size_t)std::max<int64_t>(nent, 1) * sizeof(uint32_t);
  const size_t tb = tl.size() * sizeof(PfxTile), bb = std::max<size_t>(big.size(), 1) * 4;
  size_t fr = 0, tot = 0;
  MSBFS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
  if (pb + tb + bb + ((size_t)4 << 30) > fr && !tilesets_.empty()) {
    tilesets_.clear();  // (another partition's tiles: make room)
    MSBFS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
  }
  if (pb + tb + bb + ((size_t)4 << 30) > fr) {  // (RMAT-30: keep the per-vertex pulls)
    tiles_ok_ = false;
    return nullptr;
  }
  tilesets_.push_back(std::make_unique<TileSet>());
  TileSet& T = *tilesets_.back();
  T.pent.alloc(pb);
  T.tiles.alloc(tb);
  T.big.alloc(bb);
  MSBFS_HIP_CHECK(hipMemcpyAsync(T.tiles.p, tl.data(), tb, hipMemcpyHostToDevice, s));
  if (!big.empty())
    MSBFS_HIP_CHECK(hipMemcpyAsync(T.big.p, big.data(), big.size() * 4, hipMemcpyHostToDevice, s));
  T.ntiles = (int64_t)tl.size() - 1;
  T.nbig = (int64_t)big.size();
  T.nent = nent;
  T.ti.resize((size_t)T.ntiles + 1);
  T.te.resize((size_t)T.ntiles + 1);
  for (int64_t t = 0; t < T.ntiles; ++t) {
    T.ti[(size_t)t] = ((int64_t)tl[(size_t)t].v0 - part) / nparts;
    T.te[(size_t)t] = tl[(size_t)t].e0;
    if (tl[(size_t)t].nv & kTilePartial) T.last_partial = t;
  }
  T.ti[(size_t)T.ntiles] = cnt;
  T.te[(size_t)T.ntiles] = nent;
  if (T.ntiles > 0) {
    k_fill_pent<<<grid_for(T.ntiles * 64, 256, 16384), 256, 0, s>>>(
        T.tiles.as<PfxTile>(), T.ntiles, nparts, g_.rowptr, g_.col, plen, T.pent.as<uint32_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));  // (tl / big are host vectors)
  T.part = part;
  T.nparts = nparts;
  T.key[0] = g_.rowptr;
  T.key[1] = g_.col;
  if (num_cus_ == 0) {
    hipDeviceProp_t prop;
    MSBFS_HIP_CHECK(hipGetDeviceProperties(&prop, g_.device));
    num_cus_ = prop.multiProcessorCount;
  }
  fbm_tile_.ensure((size_t)((g_.n + 31) / 32 + 1) * sizeof(uint32_t));
  if (!zrow_.p) {
    zrow_.alloc(16 * sizeof(uint64_t));
    MSBFS_HIP_CHECK(hipMemsetAsync(zrow_.p, 0, zrow_.bytes, s));
  }
  lcnt_.ensure(sizeof(Ctr));
  return &T;
}

// phase A of part `part` of `nparts` pulls its level 2 over the tiles of its own vertices
void BitparSolver::prepare_hybrid(int part, int nparts, hipStream_t s) {
  if (tiles_possible()) (void)pfx_tiles(maxW_, part, nparts, s);
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
}

// Own-vertex ranges of a chunked phase A (device.hpp): from the tile set, split at tile starts
// into pieces of about equal tile counts (a tile is ~kTileWeight of entries and vertices; equal
// prefix entries gave RMAT-26 / 8 parts pieces ready at 1.72, 1.72, 1.99 and 2.89 ms: the
// low-degree end is vertex-bound); the first piece holds every big vertex's partial tiles
// (k_bu_wide_finalize runs after it). Without tiles: an even split (the ranges are then packed
// after the level).
void BitparSolver::hybrid_chunk_bounds(int part, int nparts, int64_t n_eff, int chunks,
                                       int64_t* b, hipStream_t s) {
  if (chunks < 1) fail("hybrid: chunks must be >= 1");
  const int64_t cnt = n_eff > part ? (n_eff - part + nparts - 1) / nparts : 0;
  // (tile-aligned whenever any word count of this solver can take the tiled level: the tiles
  // are the same for every word count, and an untiled level packs its ranges afterwards)
  const TileSet* T = tiles_possible() ? pfx_tiles(maxW_, part, nparts, s) : nullptr;
  if (!T || T->ti.empty() || T->ti.back() != cnt) {
    for (int c = 0; c <= chunks; ++c) b[c] = cnt * c / chunks;
    return;
  }
  b[0] = 0;
  int64_t t = 0;
  for (int c = 1; c < chunks; ++c) {
    int64_t tc = T->ntiles * c / chunks;
    if (c == 1) tc = std::max(tc, T->last_partial + 1);
    t = std::max(t, std::min(tc, T->ntiles));
    b[c] = T->ti[(size_t)t];
  }
  b[chunks] = cnt;
}

// The first pull level of a batch over the tiles (see level_bu: called after the tail push).
// Returns the slab rows it wrote; leaves the next active lists in act_[1] / actw_[1] and the
// frontier in fbm_tile_ (S.fl_bitmap).
template <int W>
int BitparSolver::tiles_pull(Loop& S, hipStream_t s, const uint64_t* R, uint64_t* O,
                             const uint32_t* snap, const uint32_t* codes, int32_t code_from,
                             int rows) {
  if constexpr (W < 4) {
    fail("tiled pull: needs 4 or more words");
  } else {
  const TileSet* T = pfx_tiles(W, S.part, S.nparts, s);
  const Small sm = small();
  const uint64_t* alive = sm.alive[S.alv];
  const int64_t nwords = (g_.n + 31) / 32;
  MSBFS_HIP_CHECK(hipMemsetAsync(fbm_tile_.p, 0, (size_t)nwords * sizeof(uint32_t), s));
  const uint32_t* pvis = snap ? snap : anyvis_.as<uint32_t>();
  const int grid = std::max(1, num_cus_);
  // tile ranges: one launch for the whole level, or one per own-vertex range of a chunked
  // hybrid phase A (each range's rows are final once its launch and, for the first, the big
  // vertices' finalize ran; on_chunk then packs and sends them while the next range computes)
  const int nch = S.on_chunk && S.chunk_b.size() >= 2 ? (int)S.chunk_b.size() - 1 : 1;
  auto finalize_big = [&] {
    if (!T->nbig) return;
    const int gw = grid_for(T->nbig, Lay<W>::TILE, kMaxGrid);
    k_bu_wide_finalize<W, false, true><<<gw, kBlock, 0, s>>>(
        T->big.as<int32_t>(), T->nbig, g_.rowptr, R, O, acc_[S.ac].as<uint64_t>(), alive,
        sm.gmask, done_.as<uint32_t>(), nullptr, nullptr, ctr_.as<Ctr>(),
        anyvis_.as<uint32_t>(), nullptr, 0, slabF<W>(rows), snap, fbm_tile_.as<uint32_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
    rows += gw;
  };
  auto tile_at = [&](int c) -> int64_t {  // first tile of range c
    if (c <= 0) return 0;
    if (c >= nch) return T->ntiles;
    const int64_t t = std::lower_bound(T->ti.begin(), T->ti.end() - 1, S.chunk_b[(size_t)c]) -
                      T->ti.begin();
    // a range must start at a tile start: a tile straddling two ranges would be computed by the
    // launch of the earlier range, after the later range's piece had already left
    if (T->ti[(size_t)t] != S.chunk_b[(size_t)c] || (c == 1 && t <= T->last_partial))
      fail("tiled pull: exchange range " + std::to_string(c) + " does not start at a tile");
    return t;
  };
  // ranges from the last (low-degree end) to the first (hubs): pieces go out in the order
  // their words are packed and the low-degree ranges hold most own vertices, i.e. most bytes
  // per tile, so the big pieces overlap the remaining tiles and the exchange still running when
  // the level ends is the hubs' small piece. RMAT-26, 8 parts, 4 ranges: the first piece was
  // ready at 1.7 of 3.0 ms and 1.24 of the 1.75 ms exchange (at 300 GB/s) was exposed in
  // range order. (Every rank hands its pieces out in this same order: the collectives pair up.)
  for (int k = 0; k < nch; ++k) {
    const int c = nch - 1 - k;
    const int64_t t0 = tile_at(c), t1 = tile_at(c + 1);
    if (t1 > t0) {
      if (rows + grid > 3 * kMaxGrid) fail("tiled pull: counter slab rows exhausted");
      auto kt = S.push_after ? k_pfx_tiles<W, false> : k_pfx_tiles<W, true>;
      kt<<<grid, kTileBlock, 0, s>>>(
          T->tiles.as<PfxTile>() + t0, t1 - t0, T->pent.as<uint32_t>(), S.nparts, g_.rowptr, R,
          O, acc_[S.ac].as<uint64_t>(), pvis, snap, codes, codes ? code_from : INT32_MAX, alive,
          sm.gmask, done_.as<uint32_t>(), anyvis_.as<uint32_t>(), fbm_tile_.as<uint32_t>(),
          ctr_.as<Ctr>(), slabF<W>(rows), zrow_.as<uint64_t>());
      MSBFS_HIP_CHECK(hipGetLastError());
      rows += grid;
    }
    if (c == 0) finalize_big();
    if (nch > 1) {
      S.on_chunk(c);
      ++S.chunks_done;
    }
  }
  // next active lists (a hybrid phase A stops here: nothing reads them)
  if (S.level < S.stop_level) {
    const int next_wide = std::max(opt.wide_degree, kWideLater);
    k_build_active<4096><<<grid_for(S.cnt, 4096, INT32_MAX), kBlock, 0, s>>>(
        S.cnt, S.part, S.nparts, g_.rowptr, done_.as<uint32_t>(), next_wide,
        act_[1].as<int32_t>(), actw_[1].as<int32_t>(), ctr_.as<Ctr>());
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  S.fl_bitmap = true;
  }
  return rows;
}

// fl_[fc] from the frontier bitmap of a prefix level (only a top-down level reads the list)
void BitparSolver::materialize_frontier(Loop& S, hipStream_t s) {
  if (!S.fl_bitmap) return;
  S.fl_bitmap = false;
  if (S.nf <= 0) return;
  const int64_t nwords = (g_.n + 31) / 32;
  lcnt_.ensure(sizeof(Ctr));  // (also left by the untiled prefix level, see level_bu)
  MSBFS_HIP_CHECK(hipMemsetAsync(lcnt_.p, 0, sizeof(Ctr), s));
  k_bitmap_list<<<grid_for(nwords, kBlock, 2048), kBlock, 0, s>>>(
      fbm_tile_.as<uint32_t>(), nwords, fl_[S.fc].as<int32_t>(), lcnt_.as<Ctr>());
  MSBFS_HIP_CHECK(hipGetLastError());
}

#define MSBFS_BP_INST(WW)                                                                     \
  template int BitparSolver::tiles_pull<WW>(Loop&, hipStream_t, const uint64_t*, uint64_t*,   \
                                            const uint32_t*, const uint32_t*, int32_t, int);
MSBFS_BP_FOR_W(MSBFS_BP_INST)
#undef MSBFS_BP_INST

}  // namespace bp
}  // namespace msbfs
