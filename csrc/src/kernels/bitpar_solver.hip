// Bit-parallel MS-BFS solver: construction, tuning, batches and the level loop (direction
// choice, per-level reductions, host read-back). The level bodies live in bitpar_push.hip
// (top-down) and bitpar_pull.hip (bottom-up); design overview in bitpar/solver.hpp.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bitpar/init.hpp"
#include "bitpar/solver.hpp"

namespace msbfs {
namespace bp {

// ---- tuning ----------------------------------------------------------------------------------
namespace {
double to_num(const std::string& key, const std::string& v) {
  char* end = nullptr;
  const double x = strtod(v.c_str(), &end);
  if (v.empty() || !end || *end) fail("tuning: bad value '" + v + "' for " + key);
  return x;
}
}  // namespace

void Tuning::set(const std::string& key, const std::string& v) {
  if (key == "gamma") gamma = to_num(key, v);
  else if (key == "gamma2") {
    gamma2 = to_num(key, v);
    gamma2_auto = false;
  }
  else if (key == "pfx") {
    pfx = (int)to_num(key, v);
    if (pfx != 0 && pfx != 2) fail("tuning: pfx must be 0 (whole rows) or 2 (prefix pull)");
  } else if (key == "codes") codes = (int)to_num(key, v);
  else if (key == "code_deg") code_deg = to_num(key, v);
  else if (key == "lean") lean = (int)to_num(key, v);
  else if (key == "lean_min") lean_min = (int64_t)to_num(key, v);
  else if (key == "lazy") lazy = (int)to_num(key, v);
  else if (key == "td_fused") td_fused = (int)to_num(key, v);
  else if (key == "td_bm") td_bm = (int64_t)to_num(key, v);
  else if (key == "batch") {
    batch = (int)to_num(key, v);
    if (batch < 1 || batch > 64) fail("tuning: batch must be in [1, 64]");
  } else if (key == "bu_max") bu_max = (int64_t)to_num(key, v);
  else if (key == "tiles") tiles = (int)to_num(key, v);
  else if (key == "tiles_code_deg") tiles_code_deg = to_num(key, v);
  else if (key == "full") full = (int)to_num(key, v);
  else if (key == "dskip") dskip = (int)to_num(key, v);
  else if (key == "push_after") push_after = (int)to_num(key, v);
  else if (key == "dskip3") dskip3 = (int)to_num(key, v);
  else if (key == "chunk2") chunk2 = (int)to_num(key, v);
  else if (key == "wide_few") wide_few = (int)to_num(key, v);
  else if (key == "filter_frac") filter_frac = to_num(key, v);
  else if (key == "pfx_h") {
    pfx_h = (int)to_num(key, v);
    if (pfx_h < 0 || pfx_h > 458752) fail("tuning: pfx_h must be in [0, 458752]");
  }
  else if (key == "tiles_w") {
    tiles_w = (int)to_num(key, v);
    if (tiles_w != 4 && tiles_w != 8 && tiles_w != 16) fail("tuning: tiles_w must be 4, 8 or 16");
  }
  else if (key == "dirs") {
    for (char c : v)
      if (c != 'T' && c != 'B' && c != '.') fail("tuning: dirs takes T, B or . per level");
    dirs = v;
  } else {
    fail("tuning: unknown key '" + key +
         "' (gamma gamma2 pfx codes code_deg lean lean_min lazy td_fused td_bm batch bu_max tiles tiles_code_deg full dskip push_after dskip3 chunk2 wide_few pfx_h filter_frac tiles_w dirs)");
  }
}

void Tuning::parse(const std::string& spec) {
  size_t p = 0;
  while (p < spec.size()) {
    size_t e = spec.find_first_of(",;", p);  // (';' too: shell tools split env lists at ',')
    if (e == std::string::npos) e = spec.size();
    const std::string kv = spec.substr(p, e - p);
    p = e + 1;
    if (kv.empty()) continue;
    const size_t q = kv.find('=');
    if (q == std::string::npos) fail("tuning: expected key=value, got '" + kv + "'");
    set(kv.substr(0, q), kv.substr(q + 1));
  }
}

const Tuning& Tuning::process_default() {
  static const Tuning t = [] {
    Tuning d;
    if (const char* e = getenv("MSBFS_TUNE")) {
      d.parse(e);
      fprintf(stderr, "msbfs: MSBFS_TUNE=%s\n", e);  // never a silent algorithm change
    }
    return d;
  }();
  return t;
}

// ---- construction ----------------------------------------------------------------------------
BitparSolver::BitparSolver(const DeviceGraph& g, int max_groups)
    : g_(g), tun_(Tuning::process_default()) {
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
  // (+ 2 rows: the all-zero row n and the scratch row n + 1 of k_bu_full's branch-free gathers)
  const size_t vb = (size_t)(n + 2) * maxW_ * sizeof(uint64_t);
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
  // F, E, alive x 2, gmask, (spare) (see Small)
  small_.alloc(64 * 16 * sizeof(unsigned long long) * 3 + 4 * 16 * sizeof(uint64_t));
  // per-level counter slab: <= 3 counting kernels per level x <= kMaxGrid blocks
  slabF_.alloc((size_t)3 * kMaxGrid * 64 * maxW_ * sizeof(uint32_t));
  slabE_.alloc((size_t)3 * kMaxGrid * 64 * maxW_ * sizeof(unsigned long long));
  hctr_ = std::make_unique<PinnedBuf>(sizeof(Ctr));
  hsmall_ = std::make_unique<PinnedBuf>(small_.bytes);
  bctr_.alloc((size_t)(kBatch + 1) * (sizeof(Ctr) + 16 * sizeof(uint64_t)));
  hbctr_ = std::make_unique<PinnedBuf>((size_t)(kBatch + 1) * sizeof(Ctr));
  MSBFS_HIP_CHECK(hipDeviceSynchronize());
}

void BitparSolver::run(int64_t K, const int64_t* qoff, const int32_t* qids, int64_t* F,
                       int64_t* edges2, RunStats* st, hipStream_t stream) {
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

void BitparSolver::run_batch(int w, int64_t k0, int64_t nb, const int64_t* qoff,
                             const int32_t* qids, int64_t* F, int64_t* edges2, RunStats* st,
                             hipStream_t s) {
  const bool c = edges2 != nullptr || opt.count_edges;
#define MSBFS_BP_CASE(WW)                                                   \
  case WW:                                                                  \
    if (c) batch_impl<WW, true>(k0, nb, qoff, qids, F, edges2, st, s);      \
    else batch_impl<WW, false>(k0, nb, qoff, qids, F, edges2, st, s);       \
    break;
  switch (w) {
    MSBFS_BP_FOR_W(MSBFS_BP_CASE)
    default: fail("bad word count");
  }
#undef MSBFS_BP_CASE
}

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
  S.nsrc = np;
  // the batch's masks and source pairs go up from one pinned staging buffer (pageable copies
  // stage through the runtime and now and then stalled a step: RMAT-26 / 1024 groups, 1 step in
  // ~10-30 took +6 ms outside the level loop, tools/step_split.py); the read_ctr below retires
  // the copies before the buffer can be rewritten
  const int64_t np1 = std::max<int64_t>(np, 1);
  const size_t hbytes = 32 * sizeof(uint64_t) + (size_t)np1 * 2 * sizeof(int32_t);
  if (!hsrc_ || hsrc_->bytes < hbytes) hsrc_ = std::make_unique<PinnedBuf>(hbytes + hbytes / 2);
  {
    // gmask = the batch's groups; alive = groups with at least one valid source (computed here:
    // an atomicOr per source pair onto 16 words serialised k_init, ~0.1 ms per batch)
    uint64_t* hm = hsrc_->as<uint64_t>();
    std::fill(hm, hm + 32, 0ull);
    for (int64_t k = 0; k < nb; ++k) hm[k >> 6] |= 1ull << (k & 63);
    for (int64_t i = 0; i < np; ++i) hm[16 + (hk[i] >> 6)] |= 1ull << (hk[i] & 63);
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.gmask, hm, 16 * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[0], hm + 16, 16 * sizeof(uint64_t),
                                   hipMemcpyHostToDevice, s));
  }
  pairs_.ensure((size_t)np1 * 2 * sizeof(int32_t));
  int32_t* dpv = pairs_.as<int32_t>();
  int32_t* dpk = dpv + np1;
  if (np) {
    int32_t* hpp = reinterpret_cast<int32_t*>(hsrc_->as<uint64_t>() + 32);
    std::copy(hp.begin(), hp.end(), hpp);
    std::copy(hk.begin(), hk.end(), hpp + np1);
    MSBFS_HIP_CHECK(hipMemcpyAsync(dpv, hpp, (size_t)np1 * 2 * sizeof(int32_t),
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
  const Small sm = small();
  // rows n (all-zero) and n + 1 (scratch) of this word count (see bitpar/pull_full.hpp)
  for (int i = 0; i < 2; ++i)
    MSBFS_HIP_CHECK(hipMemsetAsync(vis_[i].as<uint64_t>() + (size_t)std::max<int64_t>(g_.n, 1) * W,
                                   0, 2 * W * sizeof(uint64_t), s));
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
      // graphs never get there). Tuning gamma scales the vertex test (0 turns it off).
      bottom_up = (double)S.ef > (double)S.ea / alpha_eff() ||
                  (tun_.gamma > 0 && S.level >= 1 &&
                   (double)S.ef > gamma_for(S.level) * (double)n_eff());
    else bottom_up = keep_pulling((double)S.nf, (double)S.ef, (double)S.na, (double)S.ea, opt.beta,
                                  alpha_eff());
    const std::string& dirs = tun_.dirs;
    if (S.level < dirs.size() && (dirs[S.level] == 'T' || dirs[S.level] == 'B'))
      bottom_up = dirs[S.level] == 'B';
    if (S.level < S.plan.size() && (S.plan[S.level] == 'T' || S.plan[S.level] == 'B'))
      bottom_up = S.plan[S.level] == 'B';
    // low-degree graphs (road-like: thousands of small top-down levels): run a batch of levels
    // without host round trips (kernels read the frontier sizes from device counters)
    if (!bottom_up) materialize_frontier(S, s);  // (a tiled pull left only its bitmap)
    if (!bottom_up && S.skip_pending) {
      // push after a dskip pull level: restore its frontier's skipped rows
      fix_done_rows<W>(S, s);
    }
    if (!bottom_up && tun_.batch > 1 && g_.max_degree <= kSmallDeg && !trace &&
        S.level + 2 < S.stop_level && opt.force_dir != 2 && S.plan.empty() &&
        (dirs.size() <= S.level)) {
      td_batch<W, COUNT>(S, st, s);
      tl = std::chrono::steady_clock::now();
      continue;
    }
    // late pull levels (small active lists: host round trips cost more than the level itself)
    if constexpr (!COUNT) {
      if (bottom_up && !trace && bu_batch_ok<W, COUNT>(S)) {
        bu_batch<W, COUNT>(S, st, s);
        tl = std::chrono::steady_clock::now();
        continue;
      }
    }
    MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
    MSBFS_HIP_CHECK(hipMemsetAsync(sm.alive[S.alv ^ 1], 0, 16 * sizeof(uint64_t), s));
    ++S.level;
    trace::Range range_level(bottom_up ? "bitpar L%u BU" : "bitpar L%u TD", S.level);
    // slab rows written by this level's counting kernels
    const int rows = bottom_up ? level_bu<W, COUNT>(S, s) : level_td<W, COUNT>(S, s);
    if (st) ++(bottom_up ? st->bu_levels : st->td_levels);
    if (rows) {
      const int rg = std::max(1, std::min(64, rows / 32));
      const uint32_t weight = (S.level == 1 && !S.weight_l1) ? 0u : S.level;
      k_level_reduce<W, COUNT><<<W * rg, kBlock, 0, s>>>(
          slabF<W>(0), slabE<W>(0), rows, rg, sm.F, sm.E, sm.alive[S.alv ^ 1], weight, BuGate{});
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

template <int W, bool COUNT>
void BitparSolver::batch_impl(int64_t k0, int64_t nb, const int64_t* qoff, const int32_t* qids,
                              int64_t* Fout, int64_t* edges2, RunStats* st, hipStream_t s) {
  Loop S;
  S.cnt = n_eff();
  // lazy: no per-batch fill of vis_[0] (n_eff * 8W bytes, ~0.8 ms on RMAT-26); the edge-counting
  // pass re-reads both rows of every new vertex (k_count_frontier), so it keeps the fill
  S.lazy = tun_.lazy && !COUNT && !fused_batches<COUNT>();
  start_batch<W, COUNT>(k0, nb, qoff, qids, S, s);
  levels<W, COUNT>(S, st, s);
  // frontier is empty: accumulator entries were cleared by finalize / zero_acc
  const unsigned long long* h = read_small(s);
  for (int64_t k = 0; k < nb; ++k) {
    Fout[k] = (int64_t)h[k];
    if (edges2) edges2[k] = (int64_t)h[64 * 16 + k];
  }
}


#define MSBFS_BP_INST(WW)                                                                         \
  template void BitparSolver::start_batch<WW, false>(int64_t, int64_t, const int64_t*,          \
                                                     const int32_t*, Loop&, hipStream_t);        \
  template void BitparSolver::start_batch<WW, true>(int64_t, int64_t, const int64_t*,           \
                                                    const int32_t*, Loop&, hipStream_t);         \
  template void BitparSolver::levels<WW, false>(Loop&, RunStats*, hipStream_t);                 \
  template void BitparSolver::levels<WW, true>(Loop&, RunStats*, hipStream_t);
MSBFS_BP_FOR_W(MSBFS_BP_INST)
#undef MSBFS_BP_INST

}  // namespace bp

std::unique_ptr<Solver> make_bitpar_solver(const DeviceGraph& g, int max_groups) {
  return std::make_unique<bp::BitparSolver>(g, max_groups);
}

}  // namespace msbfs
