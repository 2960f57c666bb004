// Bit-parallel MS-BFS solver: bottom-up (pull) levels — active lists, sparse row codes, prefix
// pull + tail push on the first pull level, narrow / lean / hub-chunk pulls after it
// (level_bu). Design overview: bitpar/solver.hpp; kernels: bitpar/pull.hpp.
#include <algorithm>

#include "bitpar/init.hpp"
#include "bitpar/pull.hpp"
#include "bitpar/pull_full.hpp"
#include "bitpar/solver.hpp"

namespace msbfs {
namespace bp {

// plen[v] = row prefix length with ids < H for every vertex (cached per graph buffers and H)
const int32_t* BitparSolver::prefix_lens(int32_t H, hipStream_t s) {
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

// first[v] for every vertex (cached per graph buffers like prefix_lens); nullptr when the 4n
// bytes do not fit comfortably (RMAT-30): k_bu_first then reads col[rowptr[v]]
const int32_t* BitparSolver::first_nbr(hipStream_t s) {
  if (!first_ok_) return nullptr;
  if (first_key_[0] != (const void*)g_.rowptr || first_key_[1] != (const void*)g_.col) {
    const size_t bytes = (size_t)std::max<int64_t>(g_.n, 1) * sizeof(int32_t);
    if (first_.bytes < bytes) {
      size_t fr = 0, tot = 0;
      MSBFS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
      if (fr < bytes + ((size_t)2 << 30)) {
        first_ok_ = false;
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

// first id with degree < min_deg (rounded up to a power of two; one table per graph); 0 when
// the graph keeps the user's ids (no degree order to exploit)
int32_t BitparSolver::code_bound(double min_deg) {
  if (!g_.old2new) return 0;
  if (code_key_[0] != (const void*)g_.rowptr || code_key_[1] != (const void*)g_.col ||
      deg_bounds_.empty()) {
    DevBuf b;
    b.alloc(kDegBounds * sizeof(int32_t));
    k_degree_bounds<<<1, 64>>>(g_.rowptr, g_.n, b.as<int32_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
    deg_bounds_.assign(kDegBounds, 0);
    MSBFS_HIP_CHECK(hipMemcpy(deg_bounds_.data(), b.p, kDegBounds * sizeof(int32_t),
                              hipMemcpyDeviceToHost));
    code_key_[0] = g_.rowptr;
    code_key_[1] = g_.col;
  }
  int k = 0;
  while (k + 1 < kDegBounds && ((int64_t)1 << k) < (int64_t)min_deg) ++k;
  return deg_bounds_[k];
}

// Prefix bound H of the untiled prefix level. Pulling the ids of [a, b) costs a column entry per
// edge into the range (every active vertex scans its prefix); pushing them costs a scattered
// atomic per edge of the range's frontier vertices only. A random source is adjacent to u with
// probability ~deg(u)/n, so with S sources u is a level-1 frontier vertex with probability
// ~S deg(u)/n: the pull pays where that is >= 1/(64 W) (a push is W atomics per edge). Measured
// with tuning pfx_h: RMAT-30 / 32 groups best at H = 32768 (level 2 33.0 -> 28.7 ms), RMAT-26 /
// 16 groups at 32768-131072 (3.38 -> 3.02 ms), RMAT-22 / 64 groups near 131072, RMAT-26 / 128
// groups (2 words) at the hub bitmap's bound.
template <int W>
int32_t BitparSolver::pfx_bound(const Loop& S) {
  constexpr int32_t kPfxH = 14336 * 32;  // (the LDS hub bitmap's bound, see level_bu)
  if (tun_.pfx_h > 0) return std::min(tun_.pfx_h, kPfxH);
  if (S.nsrc <= 0) return kPfxH;
  // (>= 2^28 vertices: 1 / 32 whatever the words, the pull's column stream and the push's
  // atomics both miss the caches there; RMAT-30 / 128-group passes: H 458752 -> the ~174K
  // vertices of degree >= 2^14, 209.0 -> 203.8 ms per 256-group step; 32 groups unchanged)
  const double md = n_eff() >= ((int64_t)1 << 28)
                        ? (double)g_.n / (32.0 * (double)S.nsrc)
                        : (double)g_.n / (64.0 * W * (double)S.nsrc);  // degree where the pull pays
  if (md < 2.0) return kPfxH;
  int k = 0;
  while (k + 1 < kDegBounds && (double)((int64_t)1 << (k + 1)) <= md) ++k;  // 2^k <= md
  const int32_t h = code_bound((double)((int64_t)1 << k));  // vertices of degree >= 2^k
  return h <= 0 ? kPfxH : std::min(std::max(h, 1024), kPfxH);
}

// Everything a run would otherwise build or allocate on first use, so that no timed run pays
// for it (the CLI's computation phase, main.cu:301-400): the vertex extent, the prefix
// lengths and first-neighbour array, the degree-bound table, and the worst-case chunk
// descriptor and source-pair buffers.
void BitparSolver::prepare(hipStream_t s) {
  const int64_t ne = n_eff();
  constexpr int32_t kPfxH = 14336 * 32;  // (the prefix pull's bound, see level_bu)
  if (g_.rows_sorted && g_.n <= INT32_MAX && tun_.pfx == 2) {
    prefix_lens(kPfxH, s);
    if (tiles_possible()) (void)pfx_tiles(maxW_, 0, 1, s);  // (the first pull level's tiles)
  }
  if (tun_.lean) first_nbr(s);
  (void)code_bound(1.0);
  DevBuf c;
  c.alloc(sizeof(unsigned long long));
  MSBFS_HIP_CHECK(hipMemsetAsync(c.p, 0, sizeof(unsigned long long), s));
  k_count_wide<<<grid_for(g_.n, kBlock, 2048), kBlock, 0, s>>>(g_.rowptr, g_.n, opt.wide_degree,
                                                               c.as<unsigned long long>());
  MSBFS_HIP_CHECK(hipGetLastError());
  unsigned long long nwide = 0;
  MSBFS_HIP_CHECK(hipMemcpyAsync(&nwide, c.p, sizeof(nwide), hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  const size_t db = (size_t)(nwide + g_.nnz / kChunk + 1) * sizeof(ChunkDesc);
  size_t fr = 0, tot = 0;
  MSBFS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
  if (db < fr / 8) desc_.ensure(db);  // (a graph filling HBM keeps the per-level sizing)
  pairs_.ensure((size_t)1 << 22);
  (void)ne;
}

// dskip (see pull_full.hpp). Rows are skipped only by the lean first-row pass (and its overflow
// pull): there ~98 % of the active vertices finish (RMAT-26 level 4: 24.4M rows not written).
// Measured (round 4, RMAT-26 / 1024 groups): probing on every unfiltered level cost level 3
// +0.55 ms (a dependent 4-byte load per step for vertices whose neighbours are never done) for
// -0.25 ms at level 4. A vertex done at a skipping level L keeps a stale row, so every later pull
// level of the batch probes a snapshot of the done bitmap taken at the start of level L + 1
// (one copy: vertices done after it wrote their rows); level L itself probes the snapshot of its
// own start (its first neighbours: a done hub covers the vertex without a row gather).
const uint32_t* BitparSolver::done_probe(Loop& S, bool skip_now, hipStream_t s) {
  if (!skip_now && !S.skipped_any) return nullptr;
  const size_t b = (size_t)((g_.n + 31) / 32) * sizeof(uint32_t);
  if (skip_now || S.resnap) {
    dsnap_.ensure(std::max<size_t>(b, 4));
    MSBFS_HIP_CHECK(hipMemcpyAsync(dsnap_.p, done_.p, b, hipMemcpyDeviceToDevice, s));
  }
  S.resnap = skip_now;
  S.skipped_any |= skip_now;
  return dsnap_.as<uint32_t>();
}

// rows of the last (dskip) pull level's frontier vertices that finished there (see
// k_fix_done_rows); the level's output buffer is vis_[cur], its input vis_[cur ^ 1]
template <int W>
void BitparSolver::fix_done_rows(Loop& S, hipStream_t s) {
  S.skip_pending = false;
  if (S.nf <= 0) return;
  const Small sm = small();
  k_fix_done_rows<W><<<grid_for(S.nf, Lay<W>::TILE, kMaxGrid), kBlock, 0, s>>>(
      fl_[S.fc].as<int32_t>(), nullptr, S.nf, done_.as<uint32_t>(),
      vis_[S.cur ^ 1].as<uint64_t>(), vis_[S.cur].as<uint64_t>(), S.skip_alive, sm.gmask);
  MSBFS_HIP_CHECK(hipGetLastError());
}

template <int W, bool COUNT>
int BitparSolver::level_bu(Loop& S, hipStream_t s) {
  using L = Lay<W>;
  const int64_t n = g_.n;
  const Small sm = small();
  const int grid = kMaxGrid;
  int rows = 0;  // slab rows written by this level's counting kernels
  uint64_t* R = vis_[S.cur].as<uint64_t>();
  uint64_t* O = vis_[S.cur ^ 1].as<uint64_t>();
  const uint64_t* alive = sm.alive[S.alv];
  if (S.old_stale) {
    // fused top-down levels wrote only vis_[cur]; pulls write the other buffer's rows of the
    // active vertices and read both buffers' rows of the finished ones afterwards
    const size_t vb = (size_t)std::max<int64_t>(n_eff(), 1) * W * sizeof(uint64_t);
    MSBFS_HIP_CHECK(hipMemcpyAsync(O, R, vb, hipMemcpyDeviceToDevice, s));
    S.old_stale = false;
  }
  const int next_wide = std::max(opt.wide_degree, kWideLater);
  // the first pull level at level 2 with the prefix pull streams static vertex tiles
  // (bitpar/tiles.hpp) instead of pulling per vertex from active lists
  constexpr int kHubW = 14336, kHubBig = 32768;
  const bool tiled = !COUNT && W >= 4 && W >= tun_.tiles_w && tun_.tiles && tun_.pfx == 2 && S.bu_levels == 0 &&
                     S.level == 2 && g_.rows_sorted && n <= INT32_MAX &&
                     n > (int64_t)kHubBig * 32 * 4 &&
                     ((S.lazy && S.bu_levels == 0) || (double)S.ev < tun_.filter_frac * (double)g_.nnz) &&
                     pfx_tiles(W, S.part, S.nparts, s) != nullptr;
  S.fl_bitmap = false;  // this level writes its own frontier (list, or bitmap when tiled)
  // The untiled prefix level with a low prefix bound (few sources, see pfx_bound) splits its
  // lists by prefix length (k_build_active): most vertices of degree > wide_few then have short
  // prefixes, which the per-vertex pull handles in a few steps instead of a hub chunk each.
  // RMAT-30 / 32 groups (H ~32K): 53.3 -> 51.2 ms per step (level 2 27.0 -> 23.5, levels 3-4
  // +1.4); RMAT-26 / 16 groups (H ~84K) 4.99 -> 4.92; with H >= ~300K (64+ groups on RMAT-26)
  // 0.4-0.6 ms slower, so only below H = 131072. (The predicate is `pfx` below, evaluated
  // before the level's state moves on.)
  constexpr int32_t kHubN = kHubW * 32;
  const bool pfx_lists = !tiled && tun_.pfx == 2 && S.bu_levels == 0 && S.level == 2 &&
                         pfx_bound<W>(S) <= 131072 &&
                         ((S.lazy && S.bu_levels == 0) ||
                          (double)S.ev < tun_.filter_frac * (double)g_.nnz) &&
                         n > (int64_t)kHubN * 4 && n > (int64_t)kHubBig * 32 * 4 &&
                         g_.rows_sorted && n <= INT32_MAX;
  if (!S.have_active && !tiled) {
    // after the first bottom-up level most vertices exit early: a whole wave per chunk pays
    // off only for much higher degrees, so later lists are split at a higher threshold
    // (wide_few only on big graphs: RMAT-22 / 64 groups ran level 2 in 0.66 ms at 32 or 64 and
    // 0.76-0.83 ms at 128; the narrow pull's long rows then have too few vertices to hide behind)
    // (lists split by prefix length on a graph of >= 2^28 non-isolated vertices: half of it;
    // RMAT-30 / 32 groups 51.1 -> 49.5 ms at 64, 49.8 at 48, 52.6 at 32 prefix entries, while
    // RMAT-26 / 16 groups keeps 128: 4.70 ms, 4.84 at 96, 4.95 at 64)
    const bool few = W <= 4 && tun_.wide_few > 0 && opt.wide_degree == kDefaultWideDegree &&
                     n_eff() >= ((int64_t)1 << 23);
    const int wide0 = S.bu_levels != 0 ? next_wide
                      : !few ? opt.wide_degree
                      : (pfx_lists && n_eff() >= ((int64_t)1 << 28)) ? std::max(1, tun_.wide_few / 2)
                                                                      : tun_.wide_few;
    k_build_active<4096><<<grid_for(S.cnt, 4096, INT32_MAX), kBlock, 0, s>>>(
        S.cnt, S.part, S.nparts, g_.rowptr, done_.as<uint32_t>(), wide0, act_[0].as<int32_t>(),
        actw_[0].as<int32_t>(), ctr_.as<Ctr>(),
        pfx_lists ? prefix_lens(pfx_bound<W>(S), s) : nullptr,
        (pfx_lists && g_.old2new) ? n_eff() : -1);  // (degree-relabelled: no isolated id < n_eff)
    MSBFS_HIP_CHECK(hipGetLastError());
    const HostCtr c = read_ctr(s);
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
  // filtered levels probe the any-visited bitmap before gathering a neighbour's row (while
  // fewer than filter_frac of the edges lead to visited vertices, and always on a lazy batch's
  // first pull); filter_from = first id that is probed (0) or INT32_MAX (no probes)
  const bool filter = lazy_first || (double)S.ev < tun_.filter_frac * (double)g_.nnz;
  const int32_t filter_from = filter ? 0 : INT32_MAX;
  // probes of the lowest ids (the hubs after degree relabelling) read an LDS copy of their
  // bitmap words: 56 KB (ids < 458752, two blocks per CU) or, where one 1024-thread block per CU
  // has the LDS to itself, 128 KB (ids < 1M)
  const bool hub_lds = filter_from == 0 && n > (int64_t)kHubW * 32 * 4;
  const bool hub_big = n > (int64_t)kHubBig * 32 * 4;
  // counting fused into the traversal kernels (the edge-count pass keeps k_count_frontier)
  constexpr bool FUSE = !COUNT;
  // prefix pull + tail push on the first bottom-up level (see k_push_tail): the pulls stop at
  // the small hub bitmap's bound H = 458752 (RMAT-26 level 2: 16.8 ms vs 18.1 at the 1M bound)
  constexpr int32_t kPfxH = kHubW * 32;
  const bool pfx = tun_.pfx == 2 && first_bu && S.level == 2 && hub_lds && hub_big &&
                   g_.rows_sorted && n <= INT32_MAX;
  // sparse row codes for the first bottom-up level after level 1 (see k_build_codes). With
  // the prefix pull only ids < H and the tail pushers' own codes are ever read: the codes of
  // [code_from, H) plus those of the frontier vertices >= H (not 4 bytes for every id).
  // dskip (see done_probe): the lean pass skips the rows of the vertices it finishes; a filtered
  // level never follows it in a batch (ev only grows), and the unfiltered kernels all probe
  // (k_bu_full, k_bu_first, the hub chunks; not the per-vertex pulls of tun_.full = 0)
  const bool lean_now = tun_.lean && !S.lean_off && FUSE && filter_from == INT32_MAX &&
                        !tiled && !pfx && S.bu_levels >= kLeanLevel &&
                        S.nact >= tun_.lean_min;
  const bool skip_now = lean_now && !COUNT && tun_.dskip && full_pull() && !S.keep_rows;
  // dskip3: the full pull of an unfiltered, non-lean level (RMAT-26 level 3) skips the rows of
  // the vertices it finishes too, but probes nothing itself while no earlier level skipped (its
  // input rows are all current); the later levels probe as after any skipping level
  const bool skip3 = !lean_now && tun_.dskip3 && tun_.dskip && !COUNT && full_pull() &&
                     !S.keep_rows && filter_from == INT32_MAX && !tiled && !pfx &&
                     S.bu_levels >= 1;
  const bool probed_before = S.skipped_any;
  const uint32_t* dsnap =
      (!COUNT && full_pull()) ? done_probe(S, skip_now || skip3, s) : nullptr;
  const uint32_t* dprobe = skip3 && !probed_before ? nullptr : dsnap;
  S.skip_pending = skip_now || skip3;
  S.skip_alive = alive;
  int32_t code_from = kNoCodes;
  const uint32_t* codes = nullptr;
  if (first_bu && S.level == 2 && tun_.codes && W >= 8 && S.ef0 > 0 && n <= INT32_MAX) {
    const int64_t ne = n_eff();
    code_from = (int32_t)std::min<int64_t>(
        code_bound((tiled ? tun_.tiles_code_deg : tun_.code_deg) * (double)g_.nnz /
                   (double)S.ef0), ne);
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
  // prefix bound: the tiles' fixed one, or pfx_bound for the per-vertex prefix pull (plen is
  // cached for one bound: a batch with another source count rebuilds it, one pass over the rows)
  // (the tiles hold their entries: no prefix lengths read at run time)
  const int32_t H = tiled ? kPfxH : pfx_bound<W>(S);
  const int32_t* plen = pfx && !tiled ? prefix_lens(H, s) : nullptr;
  // the untiled prefix level (few words) writes its frontier as a bitmap (fbm_tile_, as the tiled
  // one): the next level pulls and reads no list, a push materialises it (materialize_frontier)
  const bool fbm_out = pfx && FUSE && !tiled && S.nact + S.nactw > 0;
  if (fbm_out) {
    const int64_t nwords = (g_.n + 31) / 32;
    fbm_tile_.ensure((size_t)(nwords + 1) * sizeof(uint32_t));
    MSBFS_HIP_CHECK(hipMemsetAsync(fbm_tile_.p, 0, (size_t)nwords * sizeof(uint32_t), s));
  }
  // (see k_push_tail_after; needs the whole level in one tiles launch and vertex part 0 of 1)
  S.push_after = pfx && tiled && tun_.push_after && S.nparts == 1 && !S.on_chunk;
  // no stamps for the per-vertex prefix pull at <= 4 words: it reads every vertex's pushed row
  // (8W coalesced bytes) instead of a stamp, and the push stores no stamp per edge
  const bool pfx_nostamp = pfx && !tiled && W <= 4;
  if (pfx && !S.push_after) {
    ++epoch_;
    const int split = S.nf < 65536 ? 8 : 1;  // (see k_push_tail)
    k_push_tail<W><<<grid_for(S.nf * 64 * split, kBlock, 8192), kBlock, 0, s>>>(
        fl_[S.fc].as<int32_t>(), S.nf, H, g_.rowptr, g_.col, R, codes, code_from,
        tiled ? nullptr : done_.as<uint32_t>(), S.part, S.nparts, acc_[S.ac].as<uint64_t>(),
        (tiled || pfx_nostamp) ? nullptr : stamp_.as<int32_t>(), epoch_, split);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  if (tiled) {
    rows = tiles_pull<W>(S, s, R, O, snap, codes, code_from, rows);
    if (S.push_after) {
      const int gp = grid_for(S.nf * 64, kBlock, kMaxGrid);
      if (rows + gp > 3 * kMaxGrid) fail("tail push: counter slab rows exhausted");
      k_push_tail_after<W><<<gp, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), S.nf, kPfxH, g_.rowptr, g_.col, R, codes, code_from, O,
          fbm_tile_.as<uint32_t>(), anyvis_.as<uint32_t>(), ctr_.as<Ctr>(), slabF<W>(rows));
      MSBFS_HIP_CHECK(hipGetLastError());
      rows += gp;
      S.push_after = false;
    }
    S.have_active = S.level < S.stop_level;
  } else if (S.nact) {
    if (pfx) {
      // one word: 80 VGPRs, 6 waves per SIMD, so two 768-thread blocks per CU (the 56-KB hub
      // bitmap each) instead of one 1024-thread block: RMAT-30 / 32 groups level 2 35.9 -> 32.8
      // ms, RMAT-26 / 16 groups 3.53 -> 3.36 ms (a next-step column id prefetch measured slower:
      // 88 VGPRs)
      constexpr int BT = W == 1 ? 768 : 1024;
      const int gn = grid_for(S.nact, (BT / 64) * L::VPW, 512);
      // 4-neighbour steps: 122 VGPRs, no spills (8-neighbour steps spilled at the 128-VGPR
      // bound): RMAT-26 5.17 -> 4.96 ms (the full pulls of level 3 keep 8: 5.8 vs 6.8 ms)
      // (FBM: frontier bitmap in place of the list, see fbm_out)
      auto kn = FUSE ? k_bu_narrow<W, COUNT, BT, kHubW, FUSE, true, true, 4, 0, (W == 1 && BT < 1024 ? 6 : 4), true>
                     : k_bu_narrow<W, COUNT, BT, kHubW, false, true, true>;
      kn<<<gn, BT, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive,
                           sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                           FUSE ? reinterpret_cast<int32_t*>(fbm_tile_.p)
                                : fl_[S.fc ^ 1].as<int32_t>(),
                           ctr_.as<Ctr>(),
                           anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                           next_wide, slabF<W>(rows), acc_[S.ac].as<uint64_t>(),
                           pfx_nostamp ? nullptr : stamp_.as<int32_t>(), epoch_, plen, nullptr,
                           snap, BuGate{});
      if (FUSE) rows += gn;
    } else if (hub_lds) {
      constexpr int BT = 1024;
      const int gn = grid_for(S.nact, (BT / 64) * L::VPW, 512);
      // the narrow kernel runs one 1024-thread block per CU anyway (VGPR-bound), so its LDS
      // has room for a 4x larger hub bitmap
      auto kn = hub_big ? k_bu_narrow<W, COUNT, BT, kHubBig, FUSE>
                        : k_bu_narrow<W, COUNT, BT, kHubW, FUSE>;
      kn<<<gn, BT, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive,
                           sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                           fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
                           anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                           next_wide, slabF<W>(rows), nullptr, nullptr, 0, nullptr, nullptr, snap, BuGate{});
      if (FUSE) rows += gn;
    } else {
      const int gn = grid_for(S.nact, L::TILE, grid);
      // FILT = false: no probe code at all (fewer VGPRs) on the levels that load every row
      const bool filt = filter_from != INT32_MAX;
      // short first step (one row) from the third bottom-up level on, or with few words: by
      // then most vertices are covered by their first neighbour (RMAT-26, 1024 groups: level
      // 4 3.1 -> 2.5 ms; level 3 prefers full steps: 6.5 vs 6.7 ms)
      const bool short1 = S.bu_levels >= 3 || W <= 4;
      if (tun_.lean && !S.lean_off && FUSE && !filt && S.bu_levels >= kLeanLevel &&
          S.nact >= tun_.lean_min) {
        S.lean_ran = true;
        // lean first pass, then the regular pull over the vertices it could not finish
        const int gl = grid_for(S.nact, L::TILE, grid);
        k_bu_first<W><<<gl, kBlock, 0, s>>>(
            act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive, sm.gmask,
            done_.as<uint32_t>(), touched_.as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
            ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), slabF<W>(rows), first_nbr(s), dsnap,
            skip_now ? kFlagSkipRows : 0);
        MSBFS_HIP_CHECK(hipGetLastError());
        rows += gl;
        if (full_pull())
          k_bu_full<W, full_cs<W>(), 1><<<gn, kBlock, 0, s>>>(
              touched_.as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, n, alive, sm.gmask,
              done_.as<uint32_t>(), act_[1].as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
              ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), actw_[1].as<int32_t>(), next_wide,
              slabF<W>(rows), &ctr_.as<Ctr>()->touched.v, BuGate{}, dsnap,
              skip_now ? kFlagSkipRows : 0);
        else
          k_bu_narrow<W, COUNT, kBlock, 0, FUSE, false, false, 8, 1><<<gn, kBlock, 0, s>>>(
              touched_.as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive, sm.gmask,
              done_.as<uint32_t>(), act_[1].as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
              ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
              next_wide, slabF<W>(rows), nullptr, nullptr, 0, nullptr,
              &ctr_.as<Ctr>()->touched.v, nullptr, BuGate{});
        MSBFS_HIP_CHECK(hipGetLastError());
        rows += gn;
      } else if (FUSE && !filt && full_pull()) {
        auto kf = short1 ? k_bu_full<W, full_cs<W>(), 1> : k_bu_full<W, full_cs<W>(), 0>;
        kf<<<gn, kBlock, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, n, alive,
                                 sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                                 fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
                                 anyvis_.as<uint32_t>(), actw_[1].as<int32_t>(), next_wide,
                                 slabF<W>(rows), nullptr, BuGate{}, dprobe,
                                 (skip3 ? kFlagSkipRows : 0));
        rows += gn;
      } else {
        auto kn = FUSE ? (filt ? k_bu_narrow<W, COUNT, kBlock, 0, FUSE, true>
                               : short1 ? k_bu_narrow<W, COUNT, kBlock, 0, FUSE, false, false, 8, 1>
                                        : k_bu_narrow<W, COUNT, kBlock, 0, FUSE, false>)
                       : (filt ? k_bu_narrow<W, COUNT, kBlock, 0, false, true>
                               : k_bu_narrow<W, COUNT, kBlock, 0, false, false>);
        kn<<<gn, kBlock, 0, s>>>(act_[0].as<int32_t>(), S.nact, g_.rowptr, g_.col, R, O, alive,
                                 sm.gmask, done_.as<uint32_t>(), act_[1].as<int32_t>(),
                                 fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
                                 anyvis_.as<uint32_t>(), filter_from, actw_[1].as<int32_t>(),
                                 next_wide, slabF<W>(rows), nullptr, nullptr, 0, nullptr, nullptr,
                                 snap, BuGate{});
        if (FUSE) rows += gn;
      }
    }
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  // early exit across a vertex's chunks (coop) everywhere except on an explosive first
  // bottom-up level (level 2: hardly any row gets covered, and round-robin chunk dealing
  // balances the hubs better). When top-down ran longer (RMAT-30: first pull at level 3, most of
  // every hub's groups already visited) the early exit skips most chunks.
  const int coop = !first_bu || S.level != 2 ? 1 : 0;
  auto launch_chunks = [&](const ChunkDesc* d, const int64_t* np, int64_t maxc) {
    if (hub_lds) {
      // exact chunk count = *np, read on the device (no host round trip); one block per CU
      // with the 128-KB hub bitmap (ids < 1M) except on the prefix level, whose prefixes end
      // at the small one's bound (two blocks per CU)
      const bool big = hub_big && !pfx;
      // (the prefix level without codes: LDS probes only, the next tile's ids in flight)
      auto ck = big ? k_bu_chunks<W, 256, 1024, kHubBig>
                    : (pfx && !codes && filter_from == 0 && !dprobe && !coop)
                          ? k_bu_chunks<W, 256, 1024, kHubW, true>
                          : k_bu_chunks<W, 256, 1024, kHubW>;
      ck<<<grid_for(maxc, 16, big ? 256 : 512), 1024, 0, s>>>(
          d, np, g_.col, R, alive, sm.gmask, acc_[S.ac].as<uint64_t>(), anyvis_.as<uint32_t>(),
          filter_from, coop, codes, code_from, snap, dprobe);
    } else {
      k_bu_chunks<W, 256, kBlock, 0><<<grid_for(maxc, kWaves, 8192), kBlock, 0, s>>>(
          d, np, g_.col, R, alive, sm.gmask, acc_[S.ac].as<uint64_t>(), anyvis_.as<uint32_t>(),
          filter_from, coop, codes, code_from, snap, dprobe);
    }
    MSBFS_HIP_CHECK(hipGetLastError());
  };
  if (S.nactw && !tiled && coop && !pfx && tun_.chunk2) {
    // two passes (see k_chunk_first): first chunks, then the rest of the open vertices
    const int64_t chunks_max = S.nactw + S.ea / kChunk + 1;
    desc_.ensure((size_t)chunks_max * sizeof(ChunkDesc));
    chunk_cnt_.ensure(sizeof(int64_t));
    ChunkDesc* d = desc_.as<ChunkDesc>();
    k_chunk_first<<<grid_for(S.nactw, kBlock), kBlock, 0, s>>>(
        actw_[0].as<int32_t>(), S.nactw, g_.rowptr, d, chunk_cnt_.as<int64_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
    launch_chunks(d, chunk_cnt_.as<int64_t>(), S.nactw);
    int64_t* cnt = scan_tmp_.as<int64_t>();
    char* t2 = (char*)scan_tmp_.p + (((size_t)S.nactw * sizeof(int64_t) + 255) & ~size_t(255));
    const size_t tb = scan_bytes_ - (size_t)(t2 - (char*)scan_tmp_.p);
    k_chunk_rest_count<W><<<grid_for(S.nactw, L::TILE, grid), kBlock, 0, s>>>(
        actw_[0].as<int32_t>(), S.nactw, g_.rowptr, R, acc_[S.ac].as<uint64_t>(), alive,
        sm.gmask, snap, cnt);
    MSBFS_HIP_CHECK(hipGetLastError());
    inclusive_scan_i64(cnt, offs_.as<int64_t>(), S.nactw, t2, tb, s);
    k_chunk_rest_desc<<<grid_for(S.nactw, kBlock), kBlock, 0, s>>>(
        actw_[0].as<int32_t>(), S.nactw, offs_.as<int64_t>(), g_.rowptr, d + S.nactw);
    MSBFS_HIP_CHECK(hipGetLastError());
    launch_chunks(d + S.nactw, offs_.as<int64_t>() + S.nactw - 1, chunks_max - S.nactw);
  } else if (S.nactw && !tiled) {
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
    desc_.ensure((size_t)chunks_max * sizeof(ChunkDesc));
    k_chunk_desc<<<grid_for(S.nactw, kBlock), kBlock, 0, s>>>(
        actw_[0].as<int32_t>(), S.nactw, offs_.as<int64_t>(), g_.rowptr, plen,
        desc_.as<ChunkDesc>());
    MSBFS_HIP_CHECK(hipGetLastError());
    launch_chunks(desc_.as<ChunkDesc>(), offs_.as<int64_t>() + S.nactw - 1, chunks_max);
  }
  if (S.nactw && !tiled) {
    const int gw = grid_for(S.nactw, L::TILE, grid);
    auto kw = fbm_out ? k_bu_wide_finalize<W, COUNT, FUSE, true>
                      : k_bu_wide_finalize<W, COUNT, FUSE>;
    kw<<<gw, kBlock, 0, s>>>(
        actw_[0].as<int32_t>(), S.nactw, g_.rowptr, R, O, acc_[S.ac].as<uint64_t>(), alive,
        sm.gmask, done_.as<uint32_t>(), actw_[1].as<int32_t>(), fl_[S.fc ^ 1].as<int32_t>(),
        ctr_.as<Ctr>(), anyvis_.as<uint32_t>(), act_[1].as<int32_t>(), next_wide,
        slabF<W>(rows), snap, fbm_out ? fbm_tile_.as<uint32_t>() : nullptr);
    MSBFS_HIP_CHECK(hipGetLastError());
    if (FUSE) rows += gw;
  }
  if constexpr (!FUSE) {
    // new frontier bits = Wb & ~R (both still in place: the swap is below)
    const int gc = grid_for(S.nact + S.nactw, L::TILE, grid);
    k_count_frontier<W, COUNT, true><<<gc, kBlock, 0, s>>>(
        fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(), g_.rowptr, O, R, slabF<W>(rows),
        slabE<W>(rows));
    MSBFS_HIP_CHECK(hipGetLastError());
    rows += gc;
  }
  std::swap(act_[0], act_[1]);
  std::swap(actw_[0], actw_[1]);
  S.cur ^= 1;
  S.fsrc_acc = false;
  S.osnap_next = lazy_first;
  if (fbm_out) S.fl_bitmap = true;
  return rows;
}

// Pull levels that bu_batch may run: the third pull level on (lists split at kWideLater, every
// row pulled without probes, no lean pass), active lists of at most tun_.bu_max vertices, no
// forced directions and no edge counting (k_count_frontier needs per-level host sizes).
template <int W, bool COUNT>
bool BitparSolver::bu_batch_ok(const Loop& S) const {
  // (fsrc_acc: a push level came last; level_bu first clears the accumulator entries of its
  // frontier, which later pulls and the next batch expect all-zero)
  if (COUNT || tun_.bu_max <= 0 || tun_.batch <= 1 || !S.have_active || S.bu_levels < 2 ||
      S.old_stale || S.fsrc_acc || S.na > tun_.bu_max || !S.plan.empty() || tun_.dirs.size() > S.level)
    return false;
  if ((double)S.ev < tun_.filter_frac * (double)g_.nnz) return false;  // level_bu would filter
  if (tun_.lean && !S.lean_off && S.nact >= tun_.lean_min) return false;
  return S.stop_level == 0xFFFFFFFFu || S.level + 2 <= S.stop_level;
}

// A batch of up to bu_next_ pull levels with no host synchronisation (the late levels of
// scale-free graphs: RMAT levels 4+ cost ~10-50 us of GPU time each, less than a host round
// trip). Level i reads counter slot i (slot 0 seeded from the host) and writes slot i + 1; its
// kernels run only while the BuGate on slot i is open (frontier non-empty and the pull -> push
// test still says pull), so the levels after the frontier dies or the direction turns are
// no-ops and the host loop resumes exactly where the host-driven levels would be. Both lists
// (narrow, wide) go through the short-first-step narrow kernel (late levels: most vertices are
// covered by their first neighbour); the list lengths come from the slots.
template <int W, bool COUNT>
void BitparSolver::bu_batch(Loop& S, RunStats* st, hipStream_t s) {
  static_assert(!COUNT, "edge counting keeps host-driven pull levels (bu_batch_ok)");
  using L = Lay<W>;
  const Small sm = small();
  int K = std::max(2, std::min({bu_next_, tun_.batch, kBatch}));
  if (S.stop_level != 0xFFFFFFFFu) K = (int)std::min<int64_t>(K, (int64_t)S.stop_level - S.level);
  S.fl_bitmap = false;  // (the batch's levels write frontier lists)
  Ctr* slots = bctr_.as<Ctr>();
  uint64_t* aslot = (uint64_t*)(slots + kBatch + 1);
  MSBFS_HIP_CHECK(hipMemsetAsync(bctr_.p, 0, bctr_.bytes, s));
  k_bu_seed<<<1, 64, 0, s>>>(slots, (uint32_t)S.nf, (unsigned long long)S.ef, (uint32_t)S.nact,
                             (uint32_t)S.nactw, (unsigned long long)S.ea, sm.alive[S.alv], aslot);
  MSBFS_HIP_CHECK(hipGetLastError());
  // lists only shrink: a vertex stays active at most, and keeps its side of the kWideLater split
  const int gn = grid_for(S.nact + S.nactw, L::TILE, kMaxGrid);
  const int gw = S.nactw ? grid_for(S.nactw, L::TILE, kMaxGrid) : 0;
  const int rows = gn + gw, rg = std::max(1, std::min(64, rows / 32));
  const int next_wide = std::max(opt.wide_degree, kWideLater);
  const double alpha = alpha_eff();
  const uint32_t level0 = S.level;
  const auto t0 = std::chrono::steady_clock::now();
  trace::Range range_batch("bitpar L%u-%u BU batch", level0 + 1, level0 + K);
  auto kn = k_bu_narrow<W, false, kBlock, 0, true, false, false, 8, 1>;
  const bool full = full_pull();
  // dskip: after a skipping level the batch's levels probe the snapshot (taken once, before the
  // first of them); they skip nothing themselves
  const uint32_t* dsnap = full ? done_probe(S, false, s) : nullptr;
  auto launch = [&](int grid, const int32_t* list, const uint64_t* R, uint64_t* O,
                    const uint64_t* alive, int32_t* fl_out, Ctr* out, uint32_t* slab,
                    const uint32_t* len, const BuGate& gate, int p) {
    if (full)
      k_bu_full<W, full_cs<W>(), 1><<<grid, kBlock, 0, s>>>(
          list, 0, g_.rowptr, g_.col, R, O, g_.n, alive, sm.gmask, done_.as<uint32_t>(),
          act_[p ^ 1].as<int32_t>(), fl_out, out, anyvis_.as<uint32_t>(),
          actw_[p ^ 1].as<int32_t>(), next_wide, slab, len, gate, dsnap, 0);
    else
      kn<<<grid, kBlock, 0, s>>>(list, 0, g_.rowptr, g_.col, R, O, alive, sm.gmask,
                                 done_.as<uint32_t>(), act_[p ^ 1].as<int32_t>(), fl_out, out,
                                 anyvis_.as<uint32_t>(), INT32_MAX, actw_[p ^ 1].as<int32_t>(),
                                 next_wide, slab, nullptr, nullptr, 0, nullptr, len, nullptr, gate);
  };
  for (int i = 0; i < K; ++i) {
    const BuGate gate{slots + i, opt.beta, alpha, i == 0 ? 1 : 0};
    const int p = i & 1;
    const uint64_t* R = vis_[S.cur ^ p].as<uint64_t>();
    uint64_t* O = vis_[S.cur ^ p ^ 1].as<uint64_t>();
    int32_t* fl_out = fl_[S.fc ^ p ^ 1].as<int32_t>();
    const uint64_t* alive = aslot + 16 * i;
    launch(gn, act_[p].as<int32_t>(), R, O, alive, fl_out, slots + i + 1, slabF<W>(0),
           &slots[i].act2.v, gate, p);
    if (gw)
      launch(gw, actw_[p].as<int32_t>(), R, O, alive, fl_out, slots + i + 1, slabF<W>(gn),
             &slots[i].actw2.v, gate, p);
    k_level_reduce<W, false><<<W * rg, kBlock, 0, s>>>(slabF<W>(0), slabE<W>(0), rows, rg, sm.F,
                                                       sm.E, aslot + 16 * (i + 1), level0 + 1 + i,
                                                       gate);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  MSBFS_HIP_CHECK(hipMemcpyAsync(hbctr_->p, bctr_.p, (size_t)(K + 1) * sizeof(Ctr),
                                 hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  const Ctr* h = hbctr_->as<Ctr>();
  int real = 0;  // levels whose gate was open (the same test the kernels made)
  while (real < K && bu_gate_eval(h[real], opt.beta, alpha, real == 0 ? 1 : 0)) {
    S.ev += (int64_t)h[real + 1].ev2.v;
    ++real;
  }
  MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[S.alv], aslot + 16 * real, 16 * sizeof(uint64_t),
                                 hipMemcpyDeviceToDevice, s));
  if (st && real > 0) {  // per-level records; the batch's wall time is split evenly
    const double ms = std::chrono::duration<double, std::milli>(
                          std::chrono::steady_clock::now() - t0).count() / real;
    for (int i = 0; i < real; ++i) {
      LevelRec rec;
      rec.batch = (int32_t)st->batches;
      rec.level = (int32_t)(level0 + 1 + i);
      rec.dir = 'B';
      rec.nf = h[i].fl2.v;
      rec.ef = (int64_t)h[i].ef2.v;
      rec.nf_next = h[i + 1].fl2.v;
      rec.active = (int64_t)h[i + 1].act2.v + h[i + 1].actw2.v;  // (as levels(): the new lists)
      rec.ms = ms;
      st->recs.push_back(rec);
    }
    st->bu_levels += real;
    st->levels += real;
  }
  S.level = level0 + real;
  S.bu_levels += real;
  S.nf = h[real].fl2.v;
  S.ef = (int64_t)h[real].ef2.v;
  S.nact = h[real].act2.v;
  S.nactw = h[real].actw2.v;
  S.na = S.nact + S.nactw;
  S.ea = (int64_t)h[real].eu2.v;
  if (real & 1) {  // level i read list / row / frontier buffers of parity i
    std::swap(act_[0], act_[1]);
    std::swap(actw_[0], actw_[1]);
    S.cur ^= 1;
    S.fc ^= 1;
  }
  S.fsrc_acc = false;
  S.osnap_next = false;
  // (the last real level's alive mask stays in bctr_ until the next batch: a push level right
  // after restores the skipped rows of its frontier first, see levels())
  if (real > 0) S.skip_pending = false;  // (a skipping level's frontier: restored only if next)
  // the next batch: twice as long while the frontier lives, else this tail's length + 1
  bu_next_ = real == K ? std::min(2 * K, kBatch) : real + 1;
}

#define MSBFS_BP_INST(WW)                                                 \
  template void BitparSolver::fix_done_rows<WW>(Loop&, hipStream_t);     \
  template int BitparSolver::level_bu<WW, false>(Loop&, hipStream_t);    \
  template int BitparSolver::level_bu<WW, true>(Loop&, hipStream_t);     \
  template bool BitparSolver::bu_batch_ok<WW, false>(const Loop&) const; \
  template bool BitparSolver::bu_batch_ok<WW, true>(const Loop&) const;  \
  template void BitparSolver::bu_batch<WW, false>(Loop&, RunStats*, hipStream_t);
MSBFS_BP_FOR_W(MSBFS_BP_INST)
#undef MSBFS_BP_INST

}  // namespace bp
}  // namespace msbfs
