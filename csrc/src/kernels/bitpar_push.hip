// Bit-parallel MS-BFS solver: top-down (push) levels — one host-driven level (level_td) and the
// device-driven level batches of low-degree graphs (td_batch). Design overview:
// bitpar/solver.hpp; kernels: bitpar/push.hpp.
#include <algorithm>

#include "bitpar/push.hpp"
#include "bitpar/solver.hpp"

namespace msbfs {
namespace bp {

template <int W, bool COUNT>
int BitparSolver::level_td(Loop& S, hipStream_t s) {
  using L = Lay<W>;
  const int64_t n = g_.n;
  const Small sm = small();
  const int grid = kMaxGrid;
  int rows = 0;  // slab rows written by this level's counting kernels
  uint64_t* R = vis_[S.cur].as<uint64_t>();
  uint64_t* O = vis_[S.cur ^ 1].as<uint64_t>();
  const uint64_t* alive = sm.alive[S.alv];
  ++epoch_;
  const uint32_t* lzv = S.lazy ? anyvis_.as<uint32_t>() : nullptr;  // see k_zero_part_rows
  if (g_.max_degree <= kSmallDeg) {
    // low-degree graph: vertex-parallel expansion, no degree scan
    const int eg = grid_for(S.nf, L::TILE, 4096);
    if (S.fsrc_acc)
      k_td_expand_small<W, false><<<eg, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), S.nf, nullptr, g_.rowptr, g_.col, R,
          acc_[S.ac].as<uint64_t>(),
          done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
          touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv);
    else
      k_td_expand_small<W, true><<<eg, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), S.nf, nullptr, g_.rowptr, g_.col, R, O,
          done_.as<uint32_t>(),
          acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
          touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv,
          S.osnap_next ? asnap_.as<uint32_t>() : nullptr);
  } else {
  frontier_degree_scan(g_.rowptr, fl_[S.fc].as<int32_t>(), S.nf, offs_.as<int64_t>(),
                       scan_tmp_.p, scan_bytes_, s);
  const int eg = grid_for(S.ef, L::TILE, 8192);
  if (S.fsrc_acc)
    k_td_expand<W, false><<<eg, kBlock, 0, s>>>(
        fl_[S.fc].as<int32_t>(), S.nf, offs_.as<int64_t>(), g_.rowptr, g_.col, R,
        acc_[S.ac].as<uint64_t>(), done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(),
        stamp_.as<int32_t>(), epoch_, touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv);
  else
    k_td_expand<W, true><<<eg, kBlock, 0, s>>>(
        fl_[S.fc].as<int32_t>(), S.nf, offs_.as<int64_t>(), g_.rowptr, g_.col, R, O,
        done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
        touched_.as<int32_t>(), ctr_.as<Ctr>(), lzv,
        S.osnap_next ? asnap_.as<uint32_t>() : nullptr);
  }
  MSBFS_HIP_CHECK(hipGetLastError());
  // touched <= min(n, frontier edges); the kernel reads the exact count from ctr
  const int64_t nt_max = std::min<int64_t>(std::max<int64_t>(S.ef, S.nf), n);
  const int gf = grid_for(nt_max, L::TILE, grid);
  constexpr bool FUSE = !COUNT;  // counts fused into finalize (the edge-count pass: k_count_frontier)
  k_td_finalize<W, COUNT, FUSE><<<gf, kBlock, 0, s>>>(
      touched_.as<int32_t>(), g_.rowptr, R, O, acc_[S.ac ^ 1].as<uint64_t>(), alive,
      sm.gmask, done_.as<uint32_t>(), fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(),
      fl_[S.fc].as<int32_t>(), S.nf, nullptr,
      S.fsrc_acc ? acc_[S.ac].as<uint64_t>() : nullptr, anyvis_.as<uint32_t>(), slabF<W>(rows),
      S.lazy ? 1 : 0, nullptr);
  MSBFS_HIP_CHECK(hipGetLastError());
  if constexpr (FUSE) {
    rows += gf;
  } else {
    // new frontier bits are in acc_[ac ^ 1]
    const int gc = grid_for(nt_max, L::TILE, grid);
    k_count_frontier<W, COUNT, false><<<gc, kBlock, 0, s>>>(
        fl_[S.fc ^ 1].as<int32_t>(), ctr_.as<Ctr>(), g_.rowptr, acc_[S.ac ^ 1].as<uint64_t>(),
        nullptr, slabF<W>(rows), slabE<W>(rows));
    rows += gc;
    MSBFS_HIP_CHECK(hipGetLastError());
  }
  S.ac ^= 1;
  S.fsrc_acc = true;
  S.osnap_next = false;
  return rows;
}

// A batch of up to batch_next_ top-down levels with no host synchronisation: level i of the
// batch reads its frontier size from counter slot i (slot 0 seeded from the host) and writes
// slot i + 1; alive masks likewise. Levels after the frontier dies are no-ops (every kernel
// sees a zero count). One copy of all slots afterwards restores the host's view.
template <int W, bool COUNT>
void BitparSolver::td_batch(Loop& S, RunStats* st, hipStream_t s) {
  using L = Lay<W>;
  const int64_t n = g_.n;
  const Small sm = small();
  int K = std::min<int>(batch_next_, tun_.batch);
  if (S.stop_level != 0xFFFFFFFFu) K = std::min<int64_t>(K, (int64_t)S.stop_level - S.level);
  K = std::max(K, 1);
  Ctr* slots = bctr_.as<Ctr>();
  uint64_t* aslot = (uint64_t*)(slots + kBatch + 1);
  MSBFS_HIP_CHECK(hipMemsetAsync(bctr_.p, 0, bctr_.bytes, s));
  const int64_t nwords = (n_eff() + 31) / 32;
  if (fused_batches<COUNT>()) {
    // the batch's first level reads the host's list; later ones may walk the bitmap its
    // predecessor wrote (levels outside the batch leave stale bits: start from zero)
    for (auto& b : fbm_) {
      b.ensure((size_t)std::max<int64_t>(nwords, 1) * sizeof(uint32_t));
      MSBFS_HIP_CHECK(hipMemsetAsync(b.p, 0, (size_t)std::max<int64_t>(nwords, 1) * 4, s));
    }
  }
  k_batch_seed<<<1, 64, 0, s>>>(slots, (uint32_t)S.nf, (unsigned long long)S.ef,
                                sm.alive[S.alv], aslot);
  MSBFS_HIP_CHECK(hipGetLastError());
  constexpr bool FUSE = !COUNT;
  const int grid = (int)std::min<int64_t>(kTdGrid, std::max<int64_t>(1, (n + L::TILE - 1) / L::TILE));
  uint64_t* R = vis_[S.cur].as<uint64_t>();
  uint64_t* O = vis_[S.cur ^ 1].as<uint64_t>();
  const uint32_t level0 = S.level;
  const auto t0 = std::chrono::steady_clock::now();
  bool bm_ok = false;  // the previous level of this batch wrote the frontier bitmap
  const int rg = std::max(1, std::min(64, grid / 32));
  // fused levels share a reduction launch: level i's counters go to slab rows (i - pend) * grid
  const int red = std::max(1, std::min(kTdRed, 3 * kMaxGrid / grid));
  int pend = -1;  // first fused level not reduced yet
  // the host's push -> pull test, on the degree sum of the frontier entering a level (level 2
  // uses gamma2, like the host loop: gamma_for)
  auto ef_stop_for = [&](uint32_t level) -> unsigned long long {
    if (opt.force_dir == 1) return ~0ull;
    double efs = (double)S.ea / alpha_eff();
    if (tun_.gamma > 0 && level >= 2) efs = std::min(efs, gamma_for(level - 1) * (double)n_eff());
    return (unsigned long long)std::max(0.0, std::min(efs, 1.8e19));
  };
  int aidx = 0;   // alive slot the next level reads
  auto reduce_pending = [&](int upto) {
    if (pend < 0) return;
    k_level_reduce_multi<W><<<W * rg, kBlock, 0, s>>>(slabF_.as<uint32_t>(), grid, upto - pend,
                                                      rg, level0 + 1 + pend, S.weight_l1 ? 1 : 0,
                                                      sm.F, aslot + 16 * (pend + 1));
    MSBFS_HIP_CHECK(hipGetLastError());
    aidx = upto;
    pend = -1;
  };
  trace::Range range_batch("bitpar L%u-%u TD batch", level0 + 1, level0 + K);
  for (int i = 0; i < K; ++i) {
    Ctr* prev = slots + i;
    Ctr* cur = slots + i + 1;
    const uint32_t level = level0 + 1 + i;
    ++epoch_;
    const uint32_t weight = (level == 1 && !S.weight_l1) ? 0u : level;
    if (fused_batches<COUNT>() && S.fsrc_acc && !S.lazy) {
      if (pend < 0) pend = i;
      k_td_fused<W><<<grid, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), &prev->fl2.v, bm_ok ? tun_.td_bm : INT64_MAX,
          fbm_[S.fc & 1].as<uint32_t>(), fbm_[(S.fc & 1) ^ 1].as<uint32_t>(), nwords, g_.rowptr,
          g_.col, R, acc_[S.ac].as<uint64_t>(), acc_[S.ac ^ 1].as<uint64_t>(), aslot + 16 * aidx,
          sm.gmask, done_.as<uint32_t>(), anyvis_.as<uint32_t>(), stamp_.as<int32_t>(), epoch_,
          fl_[S.fc ^ 1].as<int32_t>(), cur,
          slabF_.as<uint32_t>() + (size_t)(i - pend) * grid * 64 * W, prev,
          bm_ok ? 1 : 0, i + 1 == K ? 1 : 0, i > 0 ? slots + i - 1 : nullptr, ef_stop_for(level));
      MSBFS_HIP_CHECK(hipGetLastError());
      if (i + 1 - pend == red || i + 1 == K) reduce_pending(i + 1);
      S.fc ^= 1;
      S.ac ^= 1;
      S.old_stale = true;
      bm_ok = true;
      continue;
    }
    reduce_pending(i);
    bm_ok = false;  // (this level writes no bitmap)
    if (S.fsrc_acc)
      k_td_expand_small<W, false><<<grid, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), 0, &prev->fl2.v, g_.rowptr, g_.col, R,
          acc_[S.ac].as<uint64_t>(), done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(),
          stamp_.as<int32_t>(), epoch_, touched_.as<int32_t>(), cur,
          S.lazy ? anyvis_.as<uint32_t>() : nullptr, nullptr, i > 0 ? prev : nullptr, ef_stop_for(level));
    else
      k_td_expand_small<W, true><<<grid, kBlock, 0, s>>>(
          fl_[S.fc].as<int32_t>(), 0, &prev->fl2.v, g_.rowptr, g_.col, R, O,
          done_.as<uint32_t>(), acc_[S.ac ^ 1].as<uint64_t>(), stamp_.as<int32_t>(), epoch_,
          touched_.as<int32_t>(), cur, S.lazy ? anyvis_.as<uint32_t>() : nullptr,
          S.osnap_next ? asnap_.as<uint32_t>() : nullptr, i > 0 ? prev : nullptr, ef_stop_for(level));
    k_td_finalize<W, COUNT, FUSE><<<grid, kBlock, 0, s>>>(touched_.as<int32_t>(), g_.rowptr, R, O,
                               acc_[S.ac ^ 1].as<uint64_t>(), aslot + 16 * aidx, sm.gmask,
                               done_.as<uint32_t>(), fl_[S.fc ^ 1].as<int32_t>(), cur,
                               fl_[S.fc].as<int32_t>(), 0, &prev->fl2.v,
                               S.fsrc_acc ? acc_[S.ac].as<uint64_t>() : nullptr,
                               anyvis_.as<uint32_t>(), slabF_.as<uint32_t>(), S.lazy ? 1 : 0,
                               &prev->act2.v);
    if constexpr (!FUSE)
      k_count_frontier<W, COUNT, false><<<grid, kBlock, 0, s>>>(
          fl_[S.fc ^ 1].as<int32_t>(), cur, g_.rowptr, acc_[S.ac ^ 1].as<uint64_t>(), nullptr,
          slabF_.as<uint32_t>(), slabE_.as<unsigned long long>());
    k_level_reduce<W, COUNT><<<W * rg, kBlock, 0, s>>>(slabF_.as<uint32_t>(),
                                                       slabE_.as<unsigned long long>(), grid, rg,
                                                       sm.F, sm.E, aslot + 16 * (i + 1), weight, BuGate{});
    MSBFS_HIP_CHECK(hipGetLastError());
    aidx = i + 1;
    S.fc ^= 1;
    S.ac ^= 1;
    S.fsrc_acc = true;
    S.osnap_next = false;
  }
  (void)aidx;
  MSBFS_HIP_CHECK(hipMemcpyAsync(hbctr_->p, bctr_.p, (size_t)(K + 1) * sizeof(Ctr),
                                 hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  const Ctr* h = hbctr_->as<Ctr>();
  int real = 0;
  for (int i = 0; i < K; ++i) {
    // frontier empty before level i, or level i stopped for a pull: the rest were no-ops
    if (h[i].fl2.v == 0 || h[i].act2.v) break;
    ++real;
    S.ev += (int64_t)h[i + 1].ev2.v;
    if (level0 + 1 + i == 1) S.ev_l1 = S.ev;
  }
  // alive after the last real level -> the host loop's current alive buffer
  MSBFS_HIP_CHECK(hipMemcpyAsync(sm.alive[S.alv], aslot + 16 * real, 16 * sizeof(uint64_t),
                                 hipMemcpyDeviceToDevice, s));
  S.level = level0 + real;
  S.nf = h[real].fl2.v;
  S.ef = (int64_t)h[real].ef2.v;
  if ((K - real) % 2) {
    // the no-op levels flipped the list / accumulator parity (they touched no buffer)
    S.fc ^= 1;
    S.ac ^= 1;
  }
  if (st && real > 0) {  // per-level records; the batch's wall time is split evenly
    const double ms = std::chrono::duration<double, std::milli>(
                          std::chrono::steady_clock::now() - t0).count() / real;
    for (int i = 0; i < real; ++i) {
      LevelRec rec;
      rec.batch = (int32_t)st->batches;
      rec.level = (int32_t)(level0 + 1 + i);
      rec.dir = 'T';
      rec.nf = h[i].fl2.v;
      rec.ef = (int64_t)h[i].ef2.v;
      rec.nf_next = h[i + 1].fl2.v;
      rec.active = h[i + 1].touched.v;
      rec.ms = ms;
      st->recs.push_back(rec);
    }
  }
  if (st) {
    st->td_levels += real;
    st->levels += real;
  }
  batch_next_ = S.nf > 0 ? std::min(batch_next_ * 2, kBatch) : 4;
}


#define MSBFS_BP_INST(WW)                                                          \
  template int BitparSolver::level_td<WW, false>(Loop&, hipStream_t);             \
  template int BitparSolver::level_td<WW, true>(Loop&, hipStream_t);              \
  template void BitparSolver::td_batch<WW, false>(Loop&, RunStats*, hipStream_t); \
  template void BitparSolver::td_batch<WW, true>(Loop&, RunStats*, hipStream_t);
MSBFS_BP_FOR_W(MSBFS_BP_INST)
#undef MSBFS_BP_INST

}  // namespace bp
}  // namespace msbfs
