// msbfs CLI — drop-in for the reference binary:
//     mpirun -np <ranks> msbfs -g <graph.bin> -q <query.bin> -gn <numGPU>
// prints the identical 7-line report (main.cu:403-414). Control flow mirrors main() in
// main.cu:195-421: bootstrap (:197-201), usage (:204-212), flags (:214-224), device = rank % -gn
// (:227-228), rank-0 load + broadcast (:237-280), device setup (:282-295), round-robin queries
// (:303-322), result reduction + argmin (:324-397), report (:402-414).
//
// Opt-in extensions (unknown tokens are ignored, like the reference):
//   --algo {auto,bitpar,dist,topdown,sweep,cpu}   --comm {auto,mpi,rccl,local}
//   --gen rmat:SCALE:EF:SEED | uniform:N:M:SEED   (per-rank device generation, no broadcast)
//   --qgen K:SIZE:SEED                            (generated query groups)
//   --tune key=value,...   bit-parallel solver tuning (see msbfs_solver_tune in msbfs.h)
//   --threads N (cpu algo)  --cache (CSR sidecar, off by default like the reference's re-read;
//   --no-cache is accepted)  --json  --sort-rows  --no-relabel  --repeat R
//   --spmd N   (N >= 1) single-process multi-GPU: N ranks as N threads of this process (thread r on device
//              r % -gn), RCCL communicators from ncclCommInitAll when every rank owns a GPU
//   --dist {auto,roundrobin,hybrid,hybrid-coded}  multi-rank decomposition (auto: hybrid when > 1
//          rank, the bit-parallel solver and K <= one pass; see kernels/bitpar "hybrid";
//          hybrid-coded: the same with the zero-word coded all-to-all)
#include <hip/hip_runtime.h>

#include <algorithm>

#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "comm.hpp"
#include "msbfs/device.hpp"
#include "msbfs/graph.hpp"

using namespace msbfs;
using clk = std::chrono::high_resolution_clock;

namespace {

struct Args {
  std::string graph, query, algo = "auto", comm = "auto", gen, qgen, dist = "auto", tune;
  int numGPU = 1;
  int threads = 0;
  int repeat = 1;
  int spmd = 0;
  int max_words = 0;    // bit-parallel: at most 64*max_words groups per solver pass (0: all fit)
  int async_slots = 0;  // asynchronous MIN slots before a drain (0: Comm::kAsyncSlots; tests)
  int chunks = 0;       // hybrid: pieces of the overlapped exchange (0: 8 with RCCL, else 1)
  bool cache = false, json = false, sort_rows = false, relabel = true;
  bool host_csr = false;  // build the CSR of a graph file on the host (default: on the device)
};

std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, d)) out.push_back(t);
  return out;
}

// Fault injection for the failure-handling tests (the reference has none: a rank-0 exit() leaves
// the other ranks blocked in MPI_Bcast, main.cu:95-99). MSBFS_FAULT=<where>:<rank>
// makes rank <rank> throw at <where> in {load, compute}; every failure on any rank then takes
// the whole job down (MPI_Abort / ncclCommAbort) instead of leaving peers in a collective.
void maybe_inject(const char* where, int rank) {
  static const char* spec = getenv("MSBFS_FAULT");
  if (!spec) return;
  const std::string s(spec);
  const size_t c = s.find(':');
  if (s.substr(0, c) != where) return;
  if (c != std::string::npos && atoi(s.c_str() + c + 1) != rank) return;
  fail(std::string("injected fault: ") + where + " on rank " + std::to_string(rank));
}

// the communicator a failure must abort (world until the RCCL upgrade, then the upgraded one);
// per thread in single-process mode
thread_local Comm* g_active = nullptr;

int algo_id(const std::string& a) {
  if (a == "auto") return 0;
  if (a == "bitpar") return 1;
  if (a == "dist") return 2;
  if (a == "topdown") return 3;
  if (a == "sweep") return 4;
  if (a == "cpu") return 5;
  fail("unknown --algo " + a);
}

}  // namespace

// one rank of the job: the reference's main() body from device binding on (main.cu:226-421).
// `world` is this rank's communicator; `upgraded`: it already is the final one (single-process
// mode made the RCCL communicators up front with ncclCommInitAll).
int rank_main(Args a, std::unique_ptr<Comm> world, bool upgraded) {
  const int world_rank = world->rank();
  g_active = world.get();
  std::unique_ptr<Comm> comm;  // outlives the try block: the catch may have to abort it
  try {
    if (a.numGPU <= 0) fail("-gn must be >= 1 (the reference divides by it, main.cu:227)");
    const int algo = algo_id(a.algo);
    const bool cpu = algo == 5;

    int device = -1;
    if (!cpu) {  // device = world_rank % numGPU (main.cu:227-228), checked
      int ndev = 0;
      if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail("no GPU visible (use --algo cpu)");
      device = world_rank % a.numGPU;
      if (device >= ndev) {
        if (world_rank == 0)
          fprintf(stderr, "msbfs: -gn %d exceeds the %d visible GPU(s); using device %d\n",
                  a.numGPU, ndev, device % ndev);
        device %= ndev;
      }
      MSBFS_HIP_CHECK(hipSetDevice(device));
    }
    comm = (cpu || upgraded) ? std::move(world) : maybe_upgrade_rccl(std::move(world), a.comm, device);
    g_active = comm.get();

    const auto t_pre0 = clk::now();  // main.cu:235
    trace::push("preprocessing");
    maybe_inject("load", comm->rank());

    // ---- graph: rank-0 load + broadcast, or per-rank deterministic generation -----------------
    HostCsr hg;
    DeviceGraph dg;
    dg.device = std::max(device, 0);
    hipStream_t stream = nullptr;
    const bool gen = !a.gen.empty();
    if (gen) {
      auto f = split(a.gen, ':');
      if (f.size() < 2) fail("--gen expects rmat:SCALE:EF:SEED or uniform:N:M:SEED");
      if (f[0] == "rmat") {
        const int scale = std::stoi(f[1]);
        const int64_t ef = f.size() > 2 ? std::stoll(f[2]) : 16;
        const uint64_t seed = f.size() > 3 ? std::stoull(f[3]) : 1;
        if (cpu) hg = build_csr(gen_rmat(scale, ef, seed), a.threads);
        else device_graph_gen_rmat(dg, scale, ef, seed, 0.57, 0.19, 0.19, 1, stream);
      } else if (f[0] == "uniform") {
        const int64_t n = std::stoll(f[1]);
        const int64_t m = f.size() > 2 ? std::stoll(f[2]) : 10 * n;
        const uint64_t seed = f.size() > 3 ? std::stoull(f[3]) : 1;
        if (cpu) hg = build_csr(gen_uniform(n, m, seed), a.threads);
        else device_graph_gen_uniform(dg, n, m, seed, stream);
      } else {
        fail("unknown generator " + f[0]);
      }
      if (!a.graph.size()) a.graph = a.gen;
    } else {
      // rank 0 reads the file (main.cu:237-239). GPU runs build the CSR on the device straight
      // from the mapped edge list (device_graph_from_edge_file); --cache keeps the host build,
      // whose sidecar skips parsing altogether on the next run.
      int64_t hdr[3] = {0, 0, 0};  // n, m, CSR already on rank 0's device
      if (comm->rank() == 0) {
        try {
          if (!cpu && !a.cache && !a.host_csr) {
            device_graph_from_edge_file(dg, a.graph, stream);
            hdr[0] = dg.n;
            hdr[1] = dg.m;
            hdr[2] = 1;
          } else {
            hg = load_graph(a.graph, a.cache, a.threads);
            hdr[0] = hg.n;
            hdr[1] = hg.m;
          }
        } catch (const Error& e) {
          fprintf(stderr, "%s\n", e.what());  // "Could not open graph file %s" (main.cu:97)
          comm->abort(EXIT_FAILURE);
        }
      }
      comm->bcast_host(hdr, sizeof(hdr), 0);
      const int64_t n = hdr[0], m = hdr[1];
      const bool on_device = hdr[2] != 0;
      if (on_device && comm->rank() == 0 && !comm->device_collectives() && comm->size() > 1) {
        // host collectives: the other ranks get the device-built CSR through host memory
        hg.n = n;
        hg.m = m;
        hg.rowptr.resize(n + 1);
        hg.col.resize(2 * m);
        MSBFS_HIP_CHECK(hipMemcpy(hg.rowptr.data(), dg.rowptr, (n + 1) * sizeof(int64_t),
                                  hipMemcpyDeviceToHost));
        MSBFS_HIP_CHECK(hipMemcpy(hg.col.data(), dg.col, 2 * m * sizeof(int32_t),
                                  hipMemcpyDeviceToHost));
      }
      if (cpu) {
        if (comm->rank() != 0) {
          hg.n = n;
          hg.m = m;
          hg.rowptr.resize(n + 1);
          hg.col.resize(2 * m);
        }
        comm->bcast_host(hg.rowptr.data(), (n + 1) * sizeof(int64_t), 0);
        comm->bcast_host(hg.col.data(), 2 * m * sizeof(int32_t), 0);
      } else if (comm->device_collectives()) {
        // upload once on rank 0 (or built there), then HBM -> HBM broadcast over xGMI
        if (comm->rank() == 0) {
          if (!on_device) device_graph_from_host(dg, n, hg.rowptr.data(), hg.col.data(), stream);
          hg = HostCsr();
        } else {
          dg.n = n;
          dg.m = m;
          dg.nnz = 2 * m;
          dg.own_rowptr.alloc((n + 1) * sizeof(int64_t));
          dg.own_col.alloc(std::max<int64_t>(1, 2 * m) * sizeof(int32_t));
          dg.rowptr = dg.own_rowptr.as<int64_t>();
          dg.col = dg.own_col.as<int32_t>();
        }
        MSBFS_HIP_CHECK(hipStreamSynchronize(stream));
        comm->bcast_device(dg.rowptr, (n + 1) * sizeof(int64_t), 0, stream);
        comm->bcast_device(dg.col, 2 * m * sizeof(int32_t), 0, stream);
        if (comm->rank() != 0) device_graph_stats(dg, stream);
      } else {
        if (comm->rank() != 0) {
          hg.n = n;
          hg.m = m;
          hg.rowptr.resize(n + 1);
          hg.col.resize(2 * m);
        }
        if (comm->size() > 1) {
          comm->bcast_host(hg.rowptr.data(), (n + 1) * sizeof(int64_t), 0);
          comm->bcast_host(hg.col.data(), 2 * m * sizeof(int32_t), 0);
        }
        if (!(on_device && comm->rank() == 0))
          device_graph_from_host(dg, n, hg.rowptr.data(), hg.col.data(), stream);
        hg = HostCsr();
      }
    }
    const int64_t nverts = cpu ? hg.n : dg.n;
    if (!cpu && a.sort_rows) device_graph_sort_rows(dg, stream);
    // degree-descending ids (part of preprocessing, like the CSR build): the bit-parallel
    // solver's prefix pulls and hub bitmaps rely on them; F does not depend on the numbering.
    // Best effort (a graph without room for a second column array keeps its ids).
    bool relabelled = false;
    if (!cpu && a.relabel) {
      try {
        device_graph_relabel_by_degree(dg, stream);
        relabelled = true;
      } catch (const Error& e) {
        fprintf(stderr, "msbfs: rank %d keeps the file's vertex ids: %s\n", comm->rank(), e.what());
      }
    }

    // ---- queries: one packed broadcast instead of 2K+1 (main.cu:257-280) ---------------------
    QuerySet q;
    if (!a.qgen.empty()) {
      auto f = split(a.qgen, ':');
      const int64_t K = std::stoll(f.at(0));
      const int64_t sz = f.size() > 1 ? std::stoll(f[1]) : 16;
      const uint64_t seed = f.size() > 2 ? std::stoull(f[2]) : 7;
      q = gen_queries(nverts, K, sz, seed);
      if (!a.query.size()) a.query = a.qgen;
    } else {
      int64_t qh[2] = {0, 0};
      if (comm->rank() == 0) {
        try {
          q = read_query_bin(a.query);
        } catch (const Error& e) {
          fprintf(stderr, "%s\n", e.what());  // "Could not open query file %s" (main.cu:139)
          comm->abort(EXIT_FAILURE);
        }
        qh[0] = q.K();
        qh[1] = (int64_t)q.ids.size();
      }
      comm->bcast_host(qh, sizeof(qh), 0);
      if (comm->rank() != 0) {
        q.off.resize(qh[0] + 1);
        q.ids.resize(qh[1]);
      }
      comm->bcast_host(q.off.data(), q.off.size() * sizeof(int64_t), 0);
      comm->bcast_host(q.ids.data(), q.ids.size() * sizeof(int32_t), 0);
    }
    const int64_t K = q.K();

    if (a.dist != "auto" && a.dist != "roundrobin" && a.dist != "hybrid" &&
        a.dist != "hybrid-coded")
      fail("unknown --dist " + a.dist);
    // zero-word coded exchange (parallel/hybrid.py coding_default: it pays only below ~170 GB/s
    // of all-to-all per GPU): send/receive coded segments, decode into hrecv; the phase-A SUM
    // all-reduce also carries the P x P matrix of coded lengths. A command-line choice, agreed
    // below with the hybrid eligibility (every rank must size and call the same collectives).
    const bool want_coded = a.dist == "hybrid-coded";
    if (want_coded) a.dist = "hybrid";
    const int P = comm->size(), me = comm->rank();
    int dalgo = algo;
    if (!cpu && dalgo == 0)
      dalgo = a.dist == "hybrid" && K > 1 ? 1 : auto_device_algo(dg, (K + P - 1) / P);
    const bool want_hybrid =
        !cpu && dalgo == 1 && (a.dist == "hybrid" || (a.dist == "auto" && P > 1));

    std::unique_ptr<Solver> solver;
    if (!cpu) {
      const int64_t rr_local = (K + P - 1) / P;
      if (dalgo == 1)
        solver = make_bitpar_solver(
            dg, (int)std::min<int64_t>(std::max<int64_t>(want_hybrid ? K : rr_local, 1), 1024));
      else if (dalgo == 4) solver = make_sweep_solver(dg);
      else {
        solver = make_dist_solver(dg);
        if (dalgo == 3) solver->opt.force_dir = 1;
      }
      if (a.json) solver->opt.count_edges = true;
      if (a.max_words > 0) solver->opt.max_words = a.max_words;
      if (!a.tune.empty()) solver->tune(a.tune);
      solver->prepare(stream);  // graph-derived tables: preprocessing, not computation
      MSBFS_HIP_CHECK(hipDeviceSynchronize());
    }
    // Every rank must take the same branch (the two modes call different collectives), but
    // hybrid_max_groups() depends on the free HBM each rank saw when its solver was built (ranks
    // sharing a GPU see less): agree with a MIN all-reduce of the local eligibility.
    const bool hybrid_local = want_hybrid && K >= 1 && P <= Solver::kHybridMaxParts &&
                              K <= solver->hybrid_max_groups();
    // (the hybrid exchange moves rows by vertex id: every rank must number vertices alike)
    const bool same_ids = comm->allreduce_min_u64(relabelled ? 1 : 0) == 1 ||
                          comm->allreduce_min_u64(relabelled ? 0 : 1) == 1;
    // one MIN all-reduce: bit 1 = hybrid-eligible here, bit 0 = coded exchange requested here
    const uint64_t agree = comm->allreduce_min_u64((hybrid_local ? 2u : 0u) | (want_coded ? 1u : 0u));
    const bool hybrid = agree >= 2 && same_ids;
    const bool hcoded = hybrid && (agree & 1u);
    if (hybrid) solver->prepare_hybrid(me, P, stream);  // (preprocessing: phase A's tables)
    if (a.dist == "hybrid" && !hybrid && me == 0)
      fprintf(stderr,
              "msbfs: --dist hybrid needs --algo bitpar, <= %d ranks and K <= one pass on every "
              "rank; using round-robin\n",
              Solver::kHybridMaxParts);

    // ---- assignment: static round-robin (main.cu:304-307), or whole 64-group words (hybrid)
    std::vector<int32_t> wbeg(P + 1, 0);
    std::vector<int64_t> pcount(P, 0);  // vertices of each part (v = part + i*P < n_eff)
    int64_t n_eff = 0;
    if (hybrid) {
      const int wt = (int)((K + 63) / 64);
      for (int j = 0; j <= P; ++j) wbeg[j] = (int32_t)((int64_t)j * wt / P);
      n_eff = hybrid_extent(dg);
      for (int r = 0; r < P; ++r) pcount[r] = n_eff > r ? (n_eff - r + P - 1) / P : 0;
    }
    QuerySet local;
    std::vector<int64_t> local_to_global;
    auto take = [&](int64_t k) {
      local_to_global.push_back(k);
      local.ids.insert(local.ids.end(), q.ids.begin() + q.off[k], q.ids.begin() + q.off[k + 1]);
      local.off.push_back((int64_t)local.ids.size());
    };
    if (hybrid) {
      for (int64_t k = 64 * (int64_t)wbeg[me]; k < std::min<int64_t>(K, 64 * (int64_t)wbeg[me + 1]);
           ++k)
        take(k);
    } else {
      for (int64_t k = me; k < K; k += P) take(k);
    }
    const int64_t nlocal = (int64_t)local_to_global.size();
    // hybrid exchange buffers: send = own range x all words (destination-major), recv = all
    // vertices x own words
    DevBuf hsend, hrecv, hrcoded;
    std::vector<int64_t> scount(P, 0), rcount(P, 0), hout, hF, clen(P, 0);
    const int nw_me = hybrid ? wbeg[me + 1] - wbeg[me] : 0;
    if (hybrid) {
      const int64_t cnt = pcount[me];
      int64_t ns = 0, nr = 0;
      for (int j = 0; j < P; ++j) {
        scount[j] = cnt * (wbeg[j + 1] - wbeg[j]);
        rcount[j] = pcount[j] * nw_me;
        ns += scount[j];
        nr += rcount[j];
      }
      int64_t nsc = 0, nrc = 0;
      for (int j = 0; j < P; ++j) {
        nsc += hybrid_coded_bound(scount[j]);
        nrc += hybrid_coded_bound(rcount[j]);
      }
      hsend.alloc((size_t)std::max<int64_t>(hcoded ? nsc : ns, 1) * 8);
      hrecv.alloc((size_t)std::max<int64_t>(nr, 1) * 8);
      if (hcoded) hrcoded.alloc((size_t)std::max<int64_t>(nrc, 1) * 8);
      hout.resize(2 * K + 3 + (hcoded ? (size_t)P * P : 0));
      hF.resize((size_t)std::max(1, 64 * nw_me));
    }
    // Overlapped exchange (dense): phase A hands out its own-vertex ranges as they are done and
    // each range's piece of the all-to-all runs while the next one computes (RcclComm: on the
    // communicator's stream). Every rank's range bounds are agreed on here (one SUM all-reduce).
    const int nchunks = (hybrid && !hcoded)
                            ? std::max(1, std::min(a.chunks > 0 ? a.chunks
                                                                : (comm->device_collectives() ? 8 : 1),
                                                   256))
                            : 1;
    std::vector<int64_t> cbounds;  // [P][nchunks + 1]
    if (nchunks > 1) {
      cbounds.assign((size_t)P * (nchunks + 1), 0);
      solver->hybrid_chunk_bounds(me, P, n_eff, nchunks, cbounds.data() + (size_t)me * (nchunks + 1),
                                  stream);
      MSBFS_HIP_CHECK(hipStreamSynchronize(stream));
      comm->allreduce_sum_i64(cbounds.data(), cbounds.size());
    }

    const auto t_pre1 = clk::now();  // main.cu:297-298
    trace::pop();
    const double preprocessing_time = std::chrono::duration<double>(t_pre1 - t_pre0).count();

    // ---- computation (main.cu:301-400) ---------------------------------------------------------
    std::vector<int64_t> F(nlocal, 0), E2(nlocal, 0);
    double computation_time = 0;
    int64_t minF = -1, minK = -1;
    RunStats rs;
    if (hybrid && a.json && nlocal) {  // TEPS numerator: untimed counting pass of the own groups
      std::vector<int64_t> Ft(nlocal);
      solver->run(nlocal, local.off.data(), local.ids.data(), Ft.data(), E2.data(), nullptr, stream);
    }
    // Round robin runs its groups in passes of the solver's width (64*W groups); each pass's
    // packed key goes into an asynchronous MIN all-reduce on the communicator's own stream
    // while the next pass computes, so only the last pass's 8-byte reduction is exposed. Every
    // rank issues the same number of reductions (ranks with fewer passes send NONE).
    const int64_t pass = (cpu || hybrid || !solver) ? std::max<int64_t>(nlocal, 1)
                                                    : std::max<int64_t>(1, solver->pass_groups());
    const int npass_local = nlocal ? (int)(1 + (nlocal - 1) / pass) : 0;
    const int npass = hybrid ? 1 : (int)comm->allreduce_max_f64((double)npass_local);
    // more passes than asynchronous slots (small solver widths on huge graphs): the slots are
    // drained every kAsyncSlots passes and folded into the running minimum (every rank drains at
    // the same pass, since npass is agreed on)
    int nslots = std::min(npass, (int)Comm::kAsyncSlots);
    if (a.async_slots > 0) nslots = std::min(nslots, a.async_slots);
    nslots = std::max(nslots, 1);
    comm->reserve_device_scratch((size_t)std::max<int64_t>(hout.size(), a.json ? K : 0) * 8);
    int qbits = 1;
    while ((int64_t(1) << qbits) <= K) ++qbits;
    const uint64_t NONE = ~0ull;
    // packed key of F[i0, i1): 1 + (F << qbits | q), NONE for no groups, 0 when F does not fit
    auto pack = [&](int64_t i0, int64_t i1) -> uint64_t {
      int64_t maxF = 0;
      for (int64_t i = i0; i < i1; ++i) maxF = std::max(maxF, F[i]);
      if (qbits >= 63 || (maxF >> (63 - qbits)) != 0) return 0;
      uint64_t key = NONE;
      for (int64_t i = i0; i < i1; ++i)
        key = std::min(key, 1 + (((uint64_t)F[i] << qbits) | (uint64_t)local_to_global[i]));
      return key;
    };
    std::vector<uint64_t> keys(nslots);
    for (int rep = 0; rep < a.repeat; ++rep) {
      comm->barrier();
      trace::Range range_compute("computation");
      const auto t_c0 = clk::now();
      if (cpu) {
        HostCsr& g = hg;
        std::vector<int64_t> e;
        cpu_msbfs_all(g, local, F, a.json ? &e : nullptr, a.threads > 0 ? a.threads : default_threads());
        if (a.json)
          for (int64_t i = 0; i < nlocal; ++i) E2[i] = 2 * e[i];
      } else if (hybrid) {
        // levels 1-2 vertex-partitioned (all groups), one word all-to-all, the rest per rank
        rs = RunStats();
        if (nchunks > 1) {
          // piece c: own range [b(me, c), b(me, c + 1)) of every destination's word block of
          // hsend (destination-major), from every rank r its range c straight into r's block of
          // hrecv (source-major, the layout phase C reads)
          struct PieceCtx {
            Comm* comm;
            const std::vector<int64_t>* b;
            int P, me, nch, nw_me;
            const int32_t* wbeg;
            const std::vector<int64_t>* pcount;
            uint64_t *send, *recv;
            hipStream_t s;
          } pc{comm.get(), &cbounds, P, me, nchunks, nw_me, wbeg.data(), &pcount,
               hsend.as<uint64_t>(), hrecv.as<uint64_t>(), stream};
          auto piece = [](void* user, int c, int64_t i0, int64_t i1) {
            const PieceCtx& x = *(const PieceCtx*)user;
            std::vector<int64_t> soff(x.P), scnt(x.P), roff(x.P), rcnt(x.P);
            const int64_t cnt = (*x.pcount)[x.me];
            int64_t rb = 0;
            for (int j = 0; j < x.P; ++j) {
              const int64_t nwj = x.wbeg[j + 1] - x.wbeg[j];
              soff[j] = cnt * x.wbeg[j] + i0 * nwj;
              scnt[j] = (i1 - i0) * nwj;
              const int64_t a0 = (*x.b)[(size_t)j * (x.nch + 1) + c];
              const int64_t a1 = (*x.b)[(size_t)j * (x.nch + 1) + c + 1];
              roff[j] = rb + a0 * x.nw_me;
              rcnt[j] = (a1 - a0) * x.nw_me;
              rb += (*x.pcount)[j] * x.nw_me;
            }
            x.comm->alltoallv_piece_u64(x.send, soff, scnt, x.recv, roff, rcnt, x.s);
          };
          solver->hybrid_phase_a(K, q.off.data(), q.ids.data(), me, P, n_eff, me == 0,
                                 wbeg.data(), hsend.as<uint64_t>(), hout.data(), &rs, stream,
                                 nullptr, nchunks, piece, &pc);
        } else {
          solver->hybrid_phase_a(K, q.off.data(), q.ids.data(), me, P, n_eff, me == 0,
                                 wbeg.data(), hsend.as<uint64_t>(), hout.data(), &rs, stream,
                                 hcoded ? clen.data() : nullptr);
        }
        {
          trace::Range range_x("hybrid exchange");
          if (nchunks > 1) {
            comm->allreduce_sum_i64(hout.data(), hout.size());
            comm->exchange_wait(stream);  // (phase C's kernels follow on `stream`)
          } else if (hcoded) {
            int64_t* M = hout.data() + 2 * K + 3;
            std::fill(M, M + (size_t)P * P, 0);
            for (int j = 0; j < P; ++j) M[(size_t)me * P + j] = clen[j];
            comm->allreduce_sum_i64(hout.data(), hout.size());
            std::vector<int64_t> sc(P), rc(P);
            for (int j = 0; j < P; ++j) {
              sc[j] = M[(size_t)me * P + j];
              rc[j] = M[(size_t)j * P + me];
            }
            comm->alltoallv_device_u64(hsend.as<uint64_t>(), sc, hrcoded.as<uint64_t>(), rc,
                                       stream);
            if (nw_me > 0)
              solver->hybrid_decode(hrcoded.as<uint64_t>(), rc.data(), P, n_eff, nw_me,
                                    hrecv.as<uint64_t>(), stream);
          } else {
            comm->alltoallv_device_u64(hsend.as<uint64_t>(), scount, hrecv.as<uint64_t>(),
                                       rcount, stream);
            comm->allreduce_sum_i64(hout.data(), hout.size());
          }
        }
        solver->hybrid_phase_c(K, wbeg[me], nw_me, P, n_eff, hrecv.as<uint64_t>(), hout.data(),
                               hF.data(), &rs, stream);
        for (int64_t i = 0; i < nlocal; ++i) F[i] = hout[local_to_global[i]] + hF[i];
      }
      // ONE packed min-reduce of 1 + (F << qbits | q) per pass keeps the lowest-index tie-break
      // (main.cu:391-396); a rank whose F would not fit next to the query index sends 0, so
      // every rank sees 0 and takes the two-pass fallback together
      uint64_t key = NONE;
      int pending = 0;  // slots issued since the last drain
      auto drain = [&]() {
        comm->wait_async(keys.data(), pending);
        // (0 = some rank's F does not fit: it stays the minimum and forces the fallback)
        for (int b = 0; b < pending; ++b) key = std::min(key, keys[b]);
        pending = 0;
      };
      if (!cpu && !hybrid) {
        rs = RunStats();
        for (int b = 0; b < npass; ++b) {
          const int64_t i0 = std::min<int64_t>((int64_t)b * pass, nlocal);
          const int64_t i1 = std::min<int64_t>(i0 + pass, nlocal);
          if (i1 > i0)
            solver->run(i1 - i0, local.off.data() + i0, local.ids.data(), F.data() + i0,
                        a.json ? E2.data() + i0 : nullptr, &rs, stream);
          if (b + 1 == npass) maybe_inject("compute", comm->rank());
          if (pending == nslots) drain();
          comm->allreduce_min_u64_async(pack(i0, i1), pending++);
        }
      } else {
        maybe_inject("compute", comm->rank());
        comm->allreduce_min_u64_async(pack(0, nlocal), pending++);
      }
      drain();
      if (key == NONE) { minF = -1; minK = -1; }
      else if (key != 0) {
        --key;
        minF = (int64_t)(key >> qbits);
        minK = (int64_t)(key & ((1ull << qbits) - 1));
      } else {
        // two-pass fallback when F would not fit next to the query index
        uint64_t mf = NONE;
        for (int64_t f : F) mf = std::min(mf, (uint64_t)f);
        mf = comm->allreduce_min_u64(mf);
        uint64_t mk = NONE;
        for (int64_t i = 0; i < nlocal; ++i)
          if ((uint64_t)F[i] == mf) mk = std::min(mk, (uint64_t)local_to_global[i]);
        mk = comm->allreduce_min_u64(mk);
        if (mf == NONE) { minF = -1; minK = -1; }
        else { minF = (int64_t)mf; minK = (int64_t)mk; }
      }
      const auto t_c1 = clk::now();
      computation_time = std::chrono::duration<double>(t_c1 - t_c0).count();
    }

    if (comm->rank() == 0) {  // main.cu:403-414
      std::cout << std::fixed << std::setprecision(9);
      std::cout << "Graph: " << a.graph << "\n";
      std::cout << "Query: " << a.query << "\n";
      std::cout << "Query number (k) with minimum F value: " << (minK + 1) << "\n";
      std::cout << "Minimum F value: " << minF << "\n";
      std::cout << "GPU # : " << a.numGPU << " GPU\n";
      std::cout << "Preprocessing time: " << preprocessing_time << " s\n";
      std::cout << "Computation time: " << computation_time << " s\n";
      std::cout.flush();
    }
    if (a.json) {
      // full F vector + TEPS accounting (Graph500: traversed edges = reached degree sum / 2)
      std::vector<int64_t> allF(K, 0), allE(K, 0);
      for (int64_t i = 0; i < nlocal; ++i) {
        allF[local_to_global[i]] = F[i];
        allE[local_to_global[i]] = E2[i];
      }
      comm->allreduce_sum_i64(allF.data(), K);
      comm->allreduce_sum_i64(allE.data(), K);
      const double tmax = comm->allreduce_max_f64(computation_time);
      if (comm->rank() == 0) {
        double edges = 0;
        for (int64_t e : allE) edges += 0.5 * (double)e;
        std::cout << "{\"K\": " << K << ", \"n\": " << nverts << ", \"ranks\": " << comm->size()
                  << ", \"comm\": \"" << comm->name() << "\", \"algo\": \"" << a.algo
                  << "\", \"traversed_edges\": " << std::setprecision(0) << edges
                  << ", \"teps\": " << std::setprecision(3) << (tmax > 0 ? edges / tmax : 0)
                  << ", \"levels\": " << rs.levels << ", \"td_levels\": " << rs.td_levels
                  << ", \"bu_levels\": " << rs.bu_levels << ", \"dirs\": \"";
        for (const LevelRec& r : rs.recs) std::cout << r.dir;
        std::cout << "\", \"level_ms\": [" << std::setprecision(3);
        for (size_t i = 0; i < rs.recs.size(); ++i) std::cout << (i ? ", " : "") << rs.recs[i].ms;
        std::cout << "], \"F\": [";
        for (int64_t k = 0; k < K; ++k) std::cout << (k ? ", " : "") << allF[k];
        std::cout << "]}" << std::endl;
      }
    }
    solver.reset();
    comm.reset();
  } catch (const std::exception& e) {
    fprintf(stderr, "msbfs: %s\n", e.what());
    fflush(stderr);
    // peers may be blocked in a collective: abort the job rather than finalize (MPI_Finalize
    // would wait for them forever)
    if (g_active && g_active->size() > 1) g_active->abort(EXIT_FAILURE);
    return EXIT_FAILURE;
  }
  return 0;
}

int main(int argc, char* argv[]) {
  auto world = make_world_comm(&argc, &argv);
  if (argc < 5) {  // main.cu:204-212
    if (world->rank() == 0)
      std::cerr << "Usage: mpirun -np <ranks> " << argv[0]
                << " -g <graph.bin> -q <query.bin> -gn <numGPU>" << std::endl;
    finalize_world();
    return -1;
  }
  Args a;
  for (int i = 1; i < argc; i++) {  // exact strcmp flags, unknown tokens ignored (main.cu:216-224)
    const bool has = i + 1 < argc;
    if (!strcmp(argv[i], "-g") && has) a.graph = argv[++i];
    else if (!strcmp(argv[i], "-q") && has) a.query = argv[++i];
    else if (!strcmp(argv[i], "-gn") && has) a.numGPU = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--algo") && has) a.algo = argv[++i];
    else if (!strcmp(argv[i], "--comm") && has) a.comm = argv[++i];
    else if (!strcmp(argv[i], "--dist") && has) a.dist = argv[++i];
    else if (!strcmp(argv[i], "--gen") && has) a.gen = argv[++i];
    else if (!strcmp(argv[i], "--qgen") && has) a.qgen = argv[++i];
    else if (!strcmp(argv[i], "--tune") && has) a.tune = argv[++i];
    else if (!strcmp(argv[i], "--threads") && has) a.threads = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--repeat") && has) a.repeat = std::max(1, atoi(argv[++i]));
    else if (!strcmp(argv[i], "--spmd") && has) a.spmd = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--max-words") && has) a.max_words = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--async-slots") && has) a.async_slots = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--chunks") && has) a.chunks = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--cache")) a.cache = true;
    else if (!strcmp(argv[i], "--no-cache")) a.cache = false;
    else if (!strcmp(argv[i], "--json")) a.json = true;
    else if (!strcmp(argv[i], "--sort-rows")) a.sort_rows = true;
    else if (!strcmp(argv[i], "--no-relabel")) a.relabel = false;
    else if (!strcmp(argv[i], "--host-csr")) a.host_csr = true;
  }
  int rc = 0;
  if (a.spmd >= 1) {
    // single-process multi-GPU (the ncclCommInitAll bootstrap): one thread per rank
    try {
      if (world->size() != 1) fail("--spmd runs the whole job in one process (launch one rank)");
      if (a.numGPU <= 0) fail("-gn must be >= 1 (the reference divides by it, main.cu:227)");
      auto comms = make_thread_comms(a.spmd);
      // (one rank: RCCL only when asked for, like maybe_upgrade_rccl: a one-rank communicator
      // still runs every device collective)
      if (a.algo != "cpu" && (a.comm == "rccl" || (a.comm == "auto" && a.spmd > 1))) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail("no GPU visible (use --algo cpu)");
        std::vector<int> devs(a.spmd);
        for (int r = 0; r < a.spmd; ++r) devs[r] = (r % a.numGPU) % ndev;
        {
          std::vector<int> sd(devs);
          std::sort(sd.begin(), sd.end());
          const bool dup = std::adjacent_find(sd.begin(), sd.end()) != sd.end();
          if (dup && a.comm == "rccl")
            fail("--comm rccl needs one GPU per --spmd rank (RCCL rejects repeated devices); "
                 "lower --spmd or use --comm auto / host");
          if (dup)
            fprintf(stderr, "msbfs: --spmd %d shares GPUs: host collectives (no RCCL)\n", a.spmd);
        }
        comms = upgrade_thread_comms_rccl(std::move(comms), devs);
        // (as maybe_upgrade_rccl: RCCL needs one rank per GPU; never a silent fallback)
        if (a.comm == "rccl" && comms[0]->name() != "rccl")
          fprintf(stderr, "msbfs: --comm rccl needs one rank per GPU (--spmd %d over %d device(s)); "
                  "falling back to the in-process thread collectives\n", a.spmd,
                  std::min(a.numGPU, ndev));
      }
      std::vector<int> rcs(a.spmd, 0);
      std::vector<std::thread> th;
      for (int r = 0; r < a.spmd; ++r)
        th.emplace_back([&, r] { rcs[r] = rank_main(a, std::move(comms[r]), true); });
      for (auto& t : th) t.join();
      for (int x : rcs) rc = std::max(rc, x);
    } catch (const std::exception& e) {
      fprintf(stderr, "msbfs: %s\n", e.what());
      rc = EXIT_FAILURE;
    }
  } else {
    rc = rank_main(a, std::move(world), false);
  }
  finalize_world();
  return rc;
}
