// Bit-parallel MS-BFS solver: the hybrid multi-GPU phases (levels 1-2 vertex-partitioned, one
// all-to-all of visited words, the rest query-partitioned) and the zero-word coding of the
// exchange. Design overview: bitpar/solver.hpp and bitpar/hybrid.hpp; the caller (CLI,
// parallel/hybrid.py) does the communication.
#include <algorithm>

#include "bitpar/hybrid.hpp"
#include "bitpar/init.hpp"
#include "bitpar/solver.hpp"

namespace msbfs {
namespace bp {

namespace {
WordSplit word_split(const int32_t* wbeg, int nparts, int wt) {
  WordSplit ws{};
  for (int j = 0; j <= nparts; ++j) ws.b[j] = wbeg[j];
  for (int j = nparts + 1; j <= kMaxParts; ++j) ws.b[j] = wt + 1;  // never reached
  return ws;
}
}  // namespace

void BitparSolver::hybrid_phase_a(int64_t K, const int64_t* qoff, const int32_t* qids, int part,
                                  int nparts, int64_t n_eff, bool count_l1, const int32_t* wbeg,
                                  uint64_t* send, int64_t* out, RunStats* st, hipStream_t s,
                                  int64_t* coded_len, int chunks, ChunkFn cb, void* user) {
  if (K < 1 || K > hybrid_max_groups())
    fail("hybrid mode: K=" + std::to_string(K) + " groups exceeds one round (" +
         std::to_string(hybrid_max_groups()) + ")");
  if (nparts < 1 || nparts > kMaxParts) fail("hybrid mode: 1..64 ranks");
  if (part < 0 || part >= nparts) fail("hybrid mode: bad part index");
  if (n_eff < this->n_eff() || n_eff > g_.n) fail("hybrid mode: bad vertex extent");
  const int wt = (int)((K + 63) / 64);
  if (wbeg[0] != 0 || wbeg[nparts] != wt) fail("hybrid mode: word split must cover ceil(K/64)");
  for (int j = 0; j < nparts; ++j)
    if (wbeg[j + 1] < wbeg[j]) fail("hybrid mode: word split not monotone");
  if (chunks < 1 || (chunks > 1 && (coded_len || !cb)))
    fail("hybrid mode: a chunked exchange needs chunks >= 1, the dense layout and a callback");
  int w = 1;
  while (w < wt) w <<= 1;
#define MSBFS_BP_CASE(WW)                                                                  \
  case WW:                                                                                 \
      phase_a_impl<WW>(K, qoff, qids, part, nparts, n_eff, count_l1, wbeg, send, out, st, s, \
                       coded_len, chunks, cb, user);                                         \
    break;
  switch (w) {
    MSBFS_BP_FOR_W(MSBFS_BP_CASE)
    default: fail("bad word count");
  }
#undef MSBFS_BP_CASE
  if (st) st->batches++;
}

void BitparSolver::hybrid_phase_c(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                                  const uint64_t* recv, const int64_t* reduced, int64_t* F_out,
                                  RunStats* st, hipStream_t s) {
  if (w_count <= 0) return;
  if (w_begin < 0 || (int64_t)(w_begin + w_count) * 64 - 63 > K || w_count > maxW_)
    fail("hybrid mode: bad word block");
  if (nparts < 1 || nparts > kMaxParts) fail("hybrid mode: 1..64 ranks");
  if (n_eff < this->n_eff() || n_eff > g_.n) fail("hybrid mode: bad vertex extent");
  int w = 1;
  while (w < w_count) w <<= 1;
#define MSBFS_BP_CASE(WW)                                                               \
  case WW:                                                                              \
    phase_c_impl<WW>(K, w_begin, w_count, nparts, n_eff, recv, reduced, F_out, st, s);  \
    break;
  switch (w) {
    MSBFS_BP_FOR_W(MSBFS_BP_CASE)
    default: fail("bad word count");
  }
#undef MSBFS_BP_CASE
}

BitparSolver::CodeWs BitparSolver::code_ws(int64_t chunks) {
  const size_t a = ((size_t)chunks * 8 + 255) & ~size_t(255);
  const size_t tb = (inclusive_scan_temp_bytes(chunks) + 255) & ~size_t(255);
  code_ws_.ensure(3 * a + tb);
  char* p = (char*)code_ws_.p;
  return CodeWs{(uint64_t*)p, (int64_t*)(p + a), (int64_t*)(p + 2 * a), p + 3 * a, tb};
}

// zero-word coded send segments of phase A (see k_code_bits); the dense segments are packed
// into `staging` first; coded_len[j] (host) = words of destination j's segment
template <int W>
void BitparSolver::code_send(const uint64_t* vis, uint64_t* staging, int64_t cnt, int part,
                             int nparts, const int32_t* wbeg, uint64_t* send, int64_t* coded_len,
                             hipStream_t s) {
  const WordSplit ws = word_split(wbeg, nparts, wbeg[nparts]);
  CodeSegs cs{};
  int64_t c = 0, dn = 0;
  for (int j = 0; j < nparts; ++j) {
    cs.c0[j] = c;
    cs.len[j] = cnt * (ws.b[j + 1] - ws.b[j]);
    cs.dense[j] = dn;
    c += (cs.len[j] + 63) / 64;
    dn += cs.len[j];
  }
  cs.c0[nparts] = c;
  for (int j = 0; j < nparts; ++j) coded_len[j] = 0;
  if (c == 0) return;
  const CodeWs w = code_ws(c);
  k_pack_words<W><<<grid_for(cnt, Lay<W>::TILE, 8192), kBlock, 0, s>>>(
      vis, g_.rowptr, part, nparts, cnt, ws.b[nparts], ws, staging, 0, cnt);
  MSBFS_HIP_CHECK(hipGetLastError());
  const int gc = grid_for((c + kCodeCPW - 1) / kCodeCPW * 64, kBlock, 1 << 20);
  k_code_bits<<<gc, kBlock, 0, s>>>(staging, cs, nparts, w.bits, w.pop);
  MSBFS_HIP_CHECK(hipGetLastError());
  inclusive_scan_i64(w.pop, w.incl, c, w.tmp, w.tmp_bytes, s);
  k_code_emit<<<gc, kBlock, 0, s>>>(staging, cs, nparts, w.bits, w.incl, send);
  MSBFS_HIP_CHECK(hipGetLastError());
  k_code_lens<<<1, 64, 0, s>>>(cs, nparts, w.bits, w.incl, w.pop);  // pop is free again
  MSBFS_HIP_CHECK(hipGetLastError());
  MSBFS_HIP_CHECK(hipMemcpyAsync(coded_len, w.pop, nparts * sizeof(int64_t),
                                 hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
}

void BitparSolver::hybrid_decode(const uint64_t* coded, const int64_t* coded_len, int nparts,
                                 int64_t n_eff, int w_count, uint64_t* dense, hipStream_t s) {
  if (nparts < 1 || nparts > kMaxParts) fail("hybrid mode: 1..64 ranks");
  if (w_count < 0 || w_count > maxW_) fail("hybrid mode: bad word block");
  CodeSegs cs{};
  int64_t c = 0, base = 0, dn = 0;
  for (int r = 0; r < nparts; ++r) {
    const int64_t L = part_count(n_eff, r, nparts) * w_count, nch = (L + 63) / 64;
    if (coded_len[r] < nch || coded_len[r] > L + nch)
      fail("hybrid decode: coded segment " + std::to_string(r) + " has " +
           std::to_string(coded_len[r]) + " words, outside [" + std::to_string(nch) + ", " +
           std::to_string(L + nch) + "]");
    cs.c0[r] = c;
    cs.len[r] = L;
    cs.base[r] = base;
    cs.dense[r] = dn;
    c += nch;
    base += coded_len[r];
    dn += L;
  }
  cs.c0[nparts] = c;
  if (c == 0) return;
  const CodeWs w = code_ws(c);
  k_decode_pop<<<grid_for(c, kBlock, 1 << 20), kBlock, 0, s>>>(coded, cs, nparts, w.pop);
  MSBFS_HIP_CHECK(hipGetLastError());
  inclusive_scan_i64(w.pop, w.incl, c, w.tmp, w.tmp_bytes, s);
  k_decode_emit<<<grid_for((c + kCodeCPW - 1) / kCodeCPW * 64, kBlock, 1 << 20), kBlock, 0,
                  s>>>(coded, cs, nparts, w.incl, dense);
  MSBFS_HIP_CHECK(hipGetLastError());
}

// Phase A: level 1 (top-down, every rank identical, only rank 0 adds it to F), level 2
// (bottom-up over this rank's residue class only), then pack its rows' words per destination.
template <int W>
void BitparSolver::phase_a_impl(int64_t K, const int64_t* qoff, const int32_t* qids, int part,
                                int nparts, int64_t n_eff, bool count_l1, const int32_t* wbeg,
                                uint64_t* send, int64_t* out, RunStats* st, hipStream_t s,
                                int64_t* coded_len, int chunks, ChunkFn cb, void* user) {
  Loop S;
  S.part = part;
  S.nparts = nparts;
  S.cnt = part_count(n_eff, part, nparts);
  S.stop_level = 2;
  S.weight_l1 = count_l1;
  S.plan = "TB";
  S.lazy = tun_.lazy && opt.force_dir == 0 && tun_.dirs.empty();
  S.keep_rows = true;  // (every own row is packed after level 2)
  const int wt = (int)((K + 63) / 64);
  const WordSplit ws = word_split(wbeg, nparts, wt);
  // pack own-vertex range [i0, i1) of buffer vis into its place in send
  auto pack = [&](const uint64_t* vis, int64_t i0, int64_t i1) {
    if (i1 <= i0) return;
    k_pack_words<W><<<grid_for(i1 - i0, Lay<W>::TILE, 8192), kBlock, 0, s>>>(
        vis, g_.rowptr, part, nparts, S.cnt, wt, ws, send, i0, i1);
    MSBFS_HIP_CHECK(hipGetLastError());
  };
  if (chunks > 1) {
    S.chunk_b.resize((size_t)chunks + 1);
    hybrid_chunk_bounds(part, nparts, n_eff, chunks, S.chunk_b.data(), s);
    // (called by the tiled level-2 pull after each range: its output buffer is vis_[cur ^ 1])
    S.on_chunk = [&](int c) {
      pack(vis_[S.cur ^ 1].as<uint64_t>(), S.chunk_b[(size_t)c], S.chunk_b[(size_t)c + 1]);
      cb(user, c, S.chunk_b[(size_t)c], S.chunk_b[(size_t)c + 1]);
    };
  }
  start_batch<W, false>(0, K, qoff, qids, S, s);
  levels<W, false>(S, st, s);
  if (S.fsrc_acc && S.nf > 0) {  // stopped after a top-down level: restore the zero accumulator
    k_zero_acc<W><<<grid_for(S.nf * Lay<W>::G, kBlock), kBlock, 0, s>>>(
        fl_[S.fc].as<int32_t>(), S.nf, acc_[S.ac].as<uint64_t>());
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  if (chunks > 1) {
    // ranges the level did not hand out (no tiled level-2 pull): packed now, in the tiled
    // pull's order (last range first; every rank must start its pieces in the same order)
    for (int k = S.chunks_done; k < chunks; ++k) {
      const int c = chunks - 1 - k;
      pack(vis_[S.cur].as<uint64_t>(), S.chunk_b[(size_t)c], S.chunk_b[(size_t)c + 1]);
      cb(user, c, S.chunk_b[(size_t)c], S.chunk_b[(size_t)c + 1]);
    }
  } else if (coded_len) {
    // the dense segments are staged in the other visited buffer (n*maxW words >= cnt*wt; no
    // phase needs its rows any more: phase C and the next batch rewrite or guard every row)
    code_send<W>(vis_[S.cur].as<uint64_t>(), vis_[S.cur ^ 1].as<uint64_t>(), S.cnt, part,
                 nparts, wbeg, send, coded_len, s);
  } else {
    pack(vis_[S.cur].as<uint64_t>(), 0, S.cnt);
  }
  const bool ran_l2 = S.level >= 2;
  const Small sm = small();
  const unsigned long long* h = read_small(s);
  const unsigned long long* alive_h = h + (sm.alive[S.alv] - (uint64_t*)sm.F);
  for (int64_t k = 0; k < K; ++k) {
    out[k] = (int64_t)h[k];
    out[K + k] = ran_l2 ? (int64_t)((alive_h[k >> 6] >> (k & 63)) & 1ull) : 0;
  }
  out[2 * K] = ran_l2 ? S.nf : 0;
  out[2 * K + 1] = ran_l2 ? S.ef : 0;
  out[2 * K + 2] = count_l1 ? S.ev : (ran_l2 ? S.ev - S.ev_l1 : 0);
}

// Phase C: rebuild the level-2 state of this rank's groups from the exchanged words and run
// the remaining levels (the first one bottom-up: the frontier is only implicit in the words).
template <int W>
void BitparSolver::phase_c_impl(int64_t K, int w_begin, int w_count, int nparts, int64_t n_eff,
                                const uint64_t* recv, const int64_t* reduced, int64_t* F_out,
                                RunStats* st, hipStream_t s) {
  MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
  MSBFS_HIP_CHECK(hipMemsetAsync(small_.p, 0, small_.bytes, s));
  const Small sm = small();
  {
    // alive, gmask (pinned staging, as start_batch: a pageable copy now and then stalled ms)
    if (!hsrc_ || hsrc_->bytes < 32 * sizeof(uint64_t))
      hsrc_ = std::make_unique<PinnedBuf>(32 * sizeof(uint64_t));
    uint64_t* ha = hsrc_->as<uint64_t>();
    std::fill(ha, ha + 32, 0ull);
    for (int w = 0; w < w_count; ++w)
      for (int b = 0; b < 64; ++b) {
        const int64_t k = (int64_t)(w_begin + w) * 64 + b;
        if (k >= K) break;
        ha[16 + w] |= 1ull << b;
        if (reduced[K + k] > 0) ha[w] |= 1ull << b;
      }
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[0], ha, 16 * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipMemcpyAsync(sm.gmask, ha + 16, 16 * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    // (no wait here: the read_ctr after k_hybrid_setup retires these copies before hsrc_ is
    // written again)
  }
  if (n_eff > 0) {  // vertices >= n_eff have no edges: no kernel reads their rows or bits
    PartPrefix pre{};
    for (int r = 0; r < nparts; ++r) pre.b[r + 1] = pre.b[r] + part_count(n_eff, r, nparts);
    k_hybrid_setup<W><<<grid_for(n_eff, Lay<W>::TILE, 8192), kBlock, 0, s>>>(
        recv, w_count, n_eff, nparts, pre, vis_[0].as<uint64_t>(), vis_[1].as<uint64_t>(),
        sm.alive[0], sm.gmask, done_.as<uint32_t>(), anyvis_.as<uint32_t>(), g_.rowptr,
        std::max(opt.wide_degree, kWideLater), act_[0].as<int32_t>(), actw_[0].as<int32_t>(),
        ctr_.as<Ctr>(), (nparts & (nparts - 1)) == 0 ? __builtin_ctz((unsigned)nparts) : -1);
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  Loop S;
  {
    // the setup built the level-3 active lists (see k_hybrid_setup)
    const HostCtr c = read_ctr(s);
    S.nact = c.act2;
    S.nactw = c.actw2;
    S.have_active = true;
    MSBFS_HIP_CHECK(hipMemsetAsync(ctr_.p, 0, sizeof(Ctr), s));
  }
  S.cnt = n_eff;
  S.level = 2;
  S.nf = reduced[2 * K];
  S.ef = reduced[2 * K + 1];
  S.ev = reduced[2 * K + 2];
  S.na = S.nact + S.nactw;
  S.ea = g_.nnz;
  S.bu_levels = 1;
  S.fsrc_acc = false;
  S.bottom_up = true;
  S.plan = "..B";
  levels<W, false>(S, st, s);
  const unsigned long long* h = read_small(s);
  for (int64_t i = 0; i < (int64_t)w_count * 64; ++i) F_out[i] = (int64_t)h[i];
}

}  // namespace bp

int64_t hybrid_extent(const DeviceGraph& g) {
  MSBFS_HIP_CHECK(hipSetDevice(g.device));
  if (g.n <= 0) return 0;
  DevBuf d;
  d.alloc(sizeof(unsigned long long));
  MSBFS_HIP_CHECK(hipMemset(d.p, 0, sizeof(unsigned long long)));
  bp::k_extent<<<grid_for(g.n, 256, 2048), 256>>>(g.rowptr, g.n, d.as<unsigned long long>());
  MSBFS_HIP_CHECK(hipGetLastError());
  unsigned long long h = 0;
  MSBFS_HIP_CHECK(hipMemcpy(&h, d.p, sizeof(h), hipMemcpyDeviceToHost));
  return (int64_t)h;
}

}  // namespace msbfs
