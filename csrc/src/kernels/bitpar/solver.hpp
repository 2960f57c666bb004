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
//
// Source layout (one class, four translation units that compile in parallel):
//   bitpar/common.hpp  init.hpp  push.hpp  pull.hpp  hybrid.hpp   kernels by family
//   bitpar_solver.hip  construction, batches, the level loop (direction choice, reductions)
//   bitpar_push.hip    top-down levels and the device-driven level batches
//   bitpar_pull.hip    bottom-up levels (prefix pull + tail push, narrow / lean / chunk pulls)
//   bitpar_hybrid.hip  the hybrid multi-GPU phases and the exchange coding
#pragma once

#include <chrono>
#include <functional>
#include <vector>
#include <memory>
#include <string>

#include "common.hpp"

namespace msbfs {
namespace bp {

// Algorithm tuning of the bit-parallel solver. Defaults are the measured best (RMAT-26 / 1024
// groups, RMAT-30, road grid, uniform graphs; see README). Set per solver through
// Solver::tune ("key=value,key=value"; msbfs_solver_tune in the C API, Solver(tuning=...) in
// Python) or process-wide through the one variable MSBFS_TUNE (same syntax; echoed on stderr).
// Unknown keys and malformed values are errors, never ignored. Every key is exercised by a GPU
// oracle test (tests/test_gpu_kernels.py).
struct Tuning {
  // push -> pull once the frontier's degree sum exceeds gamma x n_eff (0: off). Level 2, where
  // the prefix pull applies, uses gamma2 (< 0: gamma): RMAT-30 / 16 groups 296 -> 106 ms
  double gamma = 1.0, gamma2 = 0.25;
  bool gamma2_auto = true;  // gamma2 not set explicitly: only skewed graphs use it (gamma_for)
  // first bottom-up level: 0 = whole-row pull; 2 = prefix pull (ids < 458752, the 56-KB LDS hub
  // bitmap) + tail push (RMAT-26 level 2: 16.8 ms vs 21.2 for whole rows)
  int pfx = 2;
  // sparse single-group row codes on the first bottom-up level; ids with degree >=
  // code_deg * nnz / (source degree sum), i.e. >= code_deg expected set bits, keep row gathers
  int codes = 1;
  double code_deg = 3.0;
  // lean first-row pass on the third and later pull levels (k_bu_first) for active lists of at
  // least lean_min vertices (RMAT-26 level 4: 2.48 -> 2.07 ms)
  int lean = 1;
  int64_t lean_min = 1 << 20;
  int lazy = 1;        // no per-batch fill of the visited buffer (see start_batch)
  int td_fused = 1;    // device-driven batches run the one-kernel k_td_fused levels
  int64_t td_bm = 65536;  // k_td_fused walks the frontier bitmap from this frontier size on
  int batch = 64;      // top-down levels per device-driven batch (1 = host-driven levels)
  // pull levels from the third on run as device-driven batches (bu_batch) while the active lists
  // hold at most bu_max vertices (0 = host-driven pull levels; needs batch > 1)
  int64_t bu_max = 1 << 20;
  int tiles = 1;       // first pull level over static vertex tiles (bitpar/tiles.hpp)
  int tiles_w = 8;     // fewest words per vertex that take the tiled first pull level (4, 8 or 16)
  // unfiltered pull levels (the second pull level on, lean overflow, device-driven batches) run
  // k_bu_full (structured-buffer rows, wave-private list queues; bitpar/pull_full.hpp) instead
  // of k_bu_narrow
  int full = 1;
  // done rows are never read (k_bu_full): pulls probe a level-start snapshot of the done bitmap
  // instead of gathering done neighbours' rows, and the rows of vertices finishing on an
  // unfiltered pull level are not written (a push level right after gets them restored)
  int dskip = 1;
  // tiled first pull level: the tail push after the tiles, into the output rows (one GPU, no
  // chunked exchange; k_push_tail_after) instead of into acc rows every tile vertex reads
  // (RMAT-26 / 1024 groups: level 2 12.5 -> 10.95 ms, 20.7-21.3 -> 19.1-19.8 ms per step)
  int push_after = 1;
  // dskip on the non-lean unfiltered full pulls too (RMAT-26 level 3: 5.80 -> 5.68 ms, 1 GB of
  // row stores fewer; see level_bu)
  int dskip3 = 1;
  // two-pass chunk scheduling of the wide vertices on early-exit levels (k_chunk_first):
  // RMAT-26 / 1024 groups level 3 5.70 -> 5.30 ms
  int chunk2 = 1;
  // wide threshold of the first pull level for passes of <= 4 words (no tiles there) while
  // SolverOptions::wide_degree is at its default, on graphs of >= 2^23 non-isolated vertices:
  // RMAT-26, level 2, 128 groups 6.54 -> 6.01 ms, 256 groups 7.49 -> 7.11 ms (32 -> 128; 512 and
  // 2048 slower; RMAT-22 prefers 32-64). 0: wide_degree as given
  int wide_few = 128;
  // prefix bound of the untiled first pull level (ids below it are pulled, the frontier vertices
  // at or above it push; <= 458752, the LDS hub bitmap's bound). 0: from the batch's source
  // count (BitparSolver::pfx_bound)
  int pfx_h = 0;
  // pull levels probe the any-visited bitmap before a neighbour's row while fewer than this
  // fraction of the edges lead to visited vertices (ev < filter_frac * nnz)
  double filter_frac = 0.5;
  int tiles_bpc = 5;
  // code_deg of the tiled level: codes are cheap there (a 4-byte load and LDS ORs instead of a
  // row gather), so rows with up to ~12 expected bits are worth a try (RMAT-26 level 2: 3 ->
  // 12: 13.85 -> 13.32 ms)
  double tiles_code_deg = 12.0;
  std::string dirs;    // forced per-level directions 'T'/'B' (tests, experiments)

  void set(const std::string& key, const std::string& value);
  void parse(const std::string& spec);  // "k=v,k=v" (or ";")
  static const Tuning& process_default();  // defaults + MSBFS_TUNE, read once per process
};

class BitparSolver final : public Solver {
 public:
  BitparSolver(const DeviceGraph& g, int max_groups);

  void run(int64_t K, const int64_t* qoff, const int32_t* qids, int64_t* F, int64_t* edges2,
           RunStats* st, hipStream_t stream) override;
  void tune(const std::string& spec) override { tun_.parse(spec); }
  int64_t pass_groups() const override { return 64 * (int64_t)std::min(maxW_, opt.max_words); }
  // graph-derived tables and worst-case scratch, built before any timed run (bitpar_pull.hip)
  void prepare(hipStream_t s) override;
  void prepare_hybrid(int part, int nparts, hipStream_t s) override;

  int64_t hybrid_max_groups() const override { return 64 * (int64_t)maxW_; }
  void hybrid_phase_a(int64_t K, const int64_t* qoff, const int32_t* qids, int part, int nparts,
                      int64_t n_eff, bool count_l1, const int32_t* wbeg, uint64_t* send,
                      int64_t* out, RunStats* st, hipStream_t s, int64_t* coded_len = nullptr,
                      int chunks = 1, ChunkFn cb = nullptr, void* user = nullptr) override;
  void hybrid_chunk_bounds(int part, int nparts, int64_t n_eff, int chunks, int64_t* bounds,
                           hipStream_t s) override;
  void hybrid_phase_c(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                      const uint64_t* recv, const int64_t* reduced, int64_t* F_out, RunStats* st,
                      hipStream_t s) override;
  void hybrid_decode(const uint64_t* coded, const int64_t* coded_len, int nparts, int64_t n_eff,
                     int w_count, uint64_t* dense, hipStream_t s) override;

  // Level-loop state. The normal path runs one batch start to finish; the hybrid phases run
  // a capped / range-restricted piece of it (phase A) or resume it from exchanged state (C).
  struct Loop {
    int cur = 0;  // vis_[cur] = read buffer (up to date for every non-done vertex)
    int fc = 0;   // fl_[fc] = current frontier
    int ac = 0;   // acc_[ac] holds the current frontier bits when fsrc_acc
    int alv = 0;  // alive[alv] = groups with a non-empty frontier
    uint32_t level = 0;
    int64_t nf = 0, ef = 0, ev = 0, na = 0, ea = 0, nact = 0, nactw = 0;
    int64_t nsrc = 0;  // the batch's (source, group) pairs
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
    bool fl_bitmap = false;             // fl_[fc] not built yet: the frontier is in fbm_tile_
    // chunked hybrid phase A: the tiled level-2 pull runs the own-vertex ranges
    // [chunk_b[c], chunk_b[c+1]) one after another and calls on_chunk(c) after each (its rows
    // are final then); chunks_done counts the calls (phase A makes up the rest after the level)
    std::vector<int64_t> chunk_b;
    std::function<void(int)> on_chunk;
    int chunks_done = 0;
    // dskip: the last level skipped the rows of the vertices it finished; a push level next
    // restores those of its frontier (k_fix_done_rows) from the read buffer and this alive mask
    bool keep_rows = false;
    bool push_after = false;  // this tiled level's tail push runs after the tiles (k_push_tail_after)
    bool skip_pending = false;
    const uint64_t* skip_alive = nullptr;
    // a level skipped rows: every later pull level of the batch probes dsnap_ (re-snapshotted
    // at the start of the first pull level after each skipping level)
    bool skipped_any = false, resnap = false;
  };
  struct Small {
    unsigned long long* F;
    unsigned long long* E;
    uint64_t* alive[2];
    uint64_t* gmask;
  };

 private:
  Small small() {
    Small r;
    r.F = small_.as<unsigned long long>();
    r.E = r.F + 64 * 16;
    r.alive[0] = (uint64_t*)(r.E + 64 * 16);
    r.alive[1] = r.alive[0] + 16;
    r.gmask = r.alive[1] + 16;
    return r;
  }
  template <int W>
  uint32_t* slabF(int row) { return slabF_.as<uint32_t>() + (size_t)row * 64 * W; }
  template <int W>
  unsigned long long* slabE(int row) {
    return slabE_.as<unsigned long long>() + (size_t)row * 64 * W;
  }

  // ---- bitpar_solver.hip
  template <int W, bool COUNT>
  void start_batch(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids, Loop& S,
                   hipStream_t s);
  template <int W, bool COUNT>
  void levels(Loop& S, RunStats* st, hipStream_t s);
  template <int W, bool COUNT>
  void batch_impl(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids, int64_t* F,
                  int64_t* edges2, RunStats* st, hipStream_t s);
  void run_batch(int w, int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids,
                 int64_t* F, int64_t* edges2, RunStats* st, hipStream_t s);
  // ---- bitpar_push.hip: one top-down level (returns the counter-slab rows it wrote)
  template <int W, bool COUNT>
  int level_td(Loop& S, hipStream_t s);
  template <int W, bool COUNT>
  void td_batch(Loop& S, RunStats* st, hipStream_t s);
  // ---- bitpar_pull.hip: one bottom-up level (returns the counter-slab rows it wrote)
  template <int W, bool COUNT>
  int level_bu(Loop& S, hipStream_t s);
  template <int W, bool COUNT>
  bool bu_batch_ok(const Loop& S) const;
  template <int W, bool COUNT>
  void bu_batch(Loop& S, RunStats* st, hipStream_t s);
  const int32_t* prefix_lens(int32_t H, hipStream_t s);
  template <int W>
  int32_t pfx_bound(const Loop& S);  // prefix bound of the untiled prefix level
  // ---- bitpar_tiles.hip: the first pull level's prefix pull over static vertex tiles
  struct TileSet {
    DevBuf pent, tiles, big;
    int64_t ntiles = 0, nbig = 0, nent = 0;
    std::vector<int64_t> ti, te;  // host: own-vertex index and first entry of every tile (+ end)
    int64_t last_partial = -1;    // last tile of a big vertex (they all precede chunk 1)
    int part = -1, nparts = 0;
    const void* key[2] = {nullptr, nullptr};
  };
  // the tiles of the own vertices (part of nparts; built on first use and cached per graph
  // buffers; nullptr for fewer than 8 words, or when they do not fit in HBM)
  const TileSet* pfx_tiles(int W, int part, int nparts, hipStream_t s);
  // some word count of this solver may take the tiled first pull level (the graph-side half of
  // level_bu's `tiled` test; pfx_tiles adds the word-count half: W >= 4 and W >= tiles_w)
  bool tiles_possible() const {
    return tun_.tiles && tun_.pfx == 2 && g_.rows_sorted && g_.n <= INT32_MAX && maxW_ >= 4 &&
           maxW_ >= tun_.tiles_w;
  }
  template <int W>
  int tiles_pull(Loop& S, hipStream_t s, const uint64_t* R, uint64_t* O, const uint32_t* snap,
                 const uint32_t* codes, int32_t code_from, int rows);
  // the frontier list of a tiled level is only a bitmap until a top-down level needs it
  void materialize_frontier(Loop& S, hipStream_t s);
  const int32_t* first_nbr(hipStream_t s);
  int32_t code_bound(double min_deg);
  // ---- bitpar_hybrid.hip
  template <int W>
  void phase_a_impl(int64_t K, const int64_t* qoff, const int32_t* qids, int part, int nparts,
                    int64_t n_eff, bool count_l1, const int32_t* wbeg, uint64_t* send,
                    int64_t* out, RunStats* st, hipStream_t s, int64_t* coded_len, int chunks,
                    ChunkFn cb, void* user);
  template <int W>
  void phase_c_impl(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                    const uint64_t* recv, const int64_t* reduced, int64_t* F_out, RunStats* st,
                    hipStream_t s);
  template <int W>
  void code_send(const uint64_t* vis, uint64_t* staging, int64_t cnt, int part, int nparts,
                 const int32_t* wbeg, uint64_t* send, int64_t* coded_len, hipStream_t s);
  // scratch of the exchange coding: bitmap words, popcounts and their inclusive scan per chunk
  struct CodeWs {
    uint64_t* bits;
    int64_t* pop;
    int64_t* incl;
    void* tmp;
    size_t tmp_bytes;
  };
  CodeWs code_ws(int64_t chunks);

  // device-driven top-down batches run k_td_fused levels (needs every row of vis_[cur] valid,
  // i.e. no lazy batch; the edge-counting pass keeps expand + finalize + k_count_frontier)
  double alpha_eff() const {
    return fused_batches<false>() ? std::min(opt.alpha, kAlphaLow) : opt.alpha;
  }
  template <bool COUNT>
  bool fused_batches() const {
    return !COUNT && tun_.td_fused && tun_.batch > 1 && g_.max_degree <= kSmallDeg &&
           (double)g_.nnz <= kTdFusedDeg * (double)std::max<int64_t>(g_.n, 1);
  }
  // push -> pull test threshold on the frontier's degree sum for the level after `done_levels`
  // completed ones (the vertex half of the direction test, see levels())
  // gamma2 (the earlier pull at level 2) only on skewed graphs (max degree > 16x the mean): there
  // the level-1 frontier holds hubs and the prefix pull covers most edges cheaply. On a uniform
  // random graph (n = 16M, m = 128M, 1024 groups, ef / n_eff = 0.26 at level 2) it pulled where a
  // push was 2.5 ms cheaper (34.2 vs 29.1 ms per step, round 4).
  double gamma_for(uint32_t done_levels) {
    if (done_levels != 1 || tun_.gamma2 < 0) return tun_.gamma;
    if (!tun_.gamma2_auto) return tun_.gamma2;  // (set explicitly: applies to every graph)
    const double mean = (double)g_.nnz / (double)std::max<int64_t>(n_eff(), 1);
    return (double)g_.max_degree > 16.0 * mean ? tun_.gamma2 : tun_.gamma;
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

  // ---- fixed policy constants (formerly environment knobs; measured, see README)
  static constexpr int kWideLater = 1024;     // wide split after the first bottom-up level
  static constexpr int kTdGrid = 1024;        // blocks of the device-driven batches' kernels
  static constexpr int kTdRed = 6;            // fused levels per k_level_reduce_multi launch
  // push -> pull threshold (Beamer's alpha) on graphs with max degree <= kSmallDeg (fused
  // top-down levels). Road grid 4896^2, 256 groups: alpha 14 pulls from ~1.7M frontier vertices
  // on and takes 3030 ms, alpha 4 stays top-down (1648 ms batched)
  static constexpr double kAlphaLow = 4.0;
  // fused levels only below this mean degree (road-like graphs): denser low-degree graphs pull
  // after a few levels (uniform n = 16M, m = 128M, 1024 groups: 29.6 ms vs 32.3 ms fused)
  static constexpr double kTdFusedDeg = 8.0;
  static constexpr int kBatch = 64;  // most levels per device-driven batch
  static constexpr int kLeanLevel = 3;  // first pull level (1-based) that may run the lean pass
  // k_bu_full: the all-zero row n is an int32 vertex index (row n + 1 is scratch), so graphs
  // with n > INT32_MAX - 2 keep k_bu_narrow
  bool full_pull() const { return tun_.full && g_.n <= (int64_t)INT32_MAX - 2; }

  const DeviceGraph& g_;
  Tuning tun_;
  int maxW_ = 1;
  DevBuf vis_[2], acc_[2], stamp_, done_, act_[2], actw_[2], fl_[2], touched_, offs_, scan_tmp_,
      ctr_, small_, pairs_, slabF_, slabE_, anyvis_, desc_;
  size_t scan_bytes_ = 0;
  std::unique_ptr<PinnedBuf> hctr_, hsmall_, hsrc_;  // (hsrc_: start_batch's H2D staging)
  int32_t epoch_ = 0;
  int64_t n_eff_ = 0;
  const void* eff_key_[3] = {nullptr, nullptr, nullptr};
  DevBuf plen_;
  DevBuf chunk_cnt_;  // pass-1 chunk count of the two-pass wide pull (device int64)
  DevBuf first_;
  DevBuf code_ws_;
  const void* first_key_[2] = {nullptr, nullptr};
  bool first_ok_ = true;  // the first-neighbour array fits (RMAT-30: no room; col[rowptr[v]])
  const void* plen_key_[2] = {nullptr, nullptr};
  int32_t plen_h_ = 0;
  DevBuf fbm_[2];   // frontier bitmaps of the fused levels (n bits each)
  DevBuf asnap_;    // any-visited bitmap at the start of a lazy batch's first pull level
  std::vector<int32_t> deg_bounds_;  // first id with degree < 2^k (relabelled graphs)
  const void* code_key_[2] = {nullptr, nullptr};
  int batch_next_ = 4;  // levels of the next device-driven batch (doubles while the frontier lives)
  int bu_next_ = 4;     // levels of the next device-driven pull batch (the last run's pull tail + 1)
  std::vector<std::unique_ptr<TileSet>> tilesets_;  // per vertex partition (hybrid emulation: all)
  bool tiles_ok_ = true;  // false once the tiles did not fit
  DevBuf fbm_tile_, lcnt_, zrow_;  // frontier bitmap of a tiled level, list counter, zero row
  DevBuf dsnap_;                   // done bitmap as of a dskip level's start
  // dskip: the done-bitmap snapshot a pull level probes (nullptr: no probes); skip_now: this
  // level skips the rows of the vertices it finishes
  const uint32_t* done_probe(Loop& S, bool skip_now, hipStream_t s);
  template <int W>
  void fix_done_rows(Loop& S, hipStream_t s);
  int num_cus_ = 0;
  DevBuf bctr_;  // (kBatch+1) Ctr slots, then (kBatch+1) x 16 alive words
  std::unique_ptr<PinnedBuf> hbctr_;
};

// explicit instantiation of a member template for every word count (W) and counting mode
#define MSBFS_BP_FOR_W(X) X(1) X(2) X(4) X(8) X(16)

}  // namespace bp
}  // namespace msbfs
