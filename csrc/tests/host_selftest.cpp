// Host-code self test for the sanitizer builds (make -C csrc asan / tsan).
//
// The reference has no race detection or sanitizer story at all (its kernel relies on a benign
// data race, main.cu:16-38). GPU AddressSanitizer is not available on the target
// pool, so the sanitizers cover the native HOST code: the multi-threaded generators, the parallel
// CSR build (count -> scan -> scatter over threads), the mmap loaders / writers and the CSR
// sidecar cache, the query-parallel CPU BFS and the in-process thread collectives of the
// single-process multi-GPU mode. Every parallel result is compared with a
// single-thread run, so a data race that changes a value fails the test even without TSan.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <unistd.h>

#include "../cli/thread_group.hpp"
#include "msbfs/graph.hpp"

using namespace msbfs;

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

// The in-process communicator of the single-process multi-GPU mode (cli/thread_group.hpp): P
// threads run many rounds of every collective back to back (the slots and the barrier are
// reused immediately, the case a missing barrier would corrupt) and check every result.
static void thread_group_selftest() {
  const int P = 5, rounds = 300;
  ThreadGroup g(P);
  std::vector<int> bad(P, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r] {
      for (int it = 0; it < rounds; ++it) {
        int64_t buf[3] = {r == it % P ? (int64_t)it : -1, r == it % P ? (int64_t)(it * 7) : -1, 0};
        tg_bcast(g, r, buf, 2 * sizeof(int64_t), it % P);
        bad[r] += buf[0] != it || buf[1] != it * 7;
        bad[r] += tg_allreduce_min(g, r, (uint64_t)(1000 + r * 13 + it)) != (uint64_t)(1000 + it);
        bad[r] += tg_allreduce_max(g, r, (double)(r + it)) != (double)(P - 1 + it);
        int64_t v[4] = {r, 1, it, -r};
        tg_allreduce_sum(g, r, v, 4);
        bad[r] += v[0] != P * (P - 1) / 2 || v[1] != P || v[2] != (int64_t)P * it ||
                  v[3] != -P * (P - 1) / 2;
        std::vector<uint64_t> all;
        tg_allgather(g, r, (uint64_t)(r * r + it), all);
        for (int k = 0; k < P; ++k) bad[r] += all[k] != (uint64_t)(k * k + it);
        // all-to-all: rank r sends (j + 1 + it % 3) words of value r*100 + j to rank j
        std::vector<int64_t> sc(P), rc(P);
        std::vector<uint64_t> send, recv;
        for (int j = 0; j < P; ++j) {
          sc[j] = j + 1 + it % 3;
          rc[j] = r + 1 + it % 3;
          for (int64_t w = 0; w < sc[j]; ++w) send.push_back((uint64_t)(r * 100 + j));
        }
        recv.assign(P * (r + 1 + it % 3), ~0ull);
        tg_alltoallv(g, r, send.data(), sc, recv.data(), rc);
        for (int j = 0, o = 0; j < P; ++j)
          for (int64_t w = 0; w < rc[j]; ++w) bad[r] += recv[o++] != (uint64_t)(j * 100 + r);
      }
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < P; ++r) CHECK(bad[r] == 0);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const std::string gp = dir + "/selftest_g.bin", qp = dir + "/selftest_q.bin";
  const int T = 8;
  thread_group_selftest();
  // generators: threaded == serial
  EdgeList e1 = gen_rmat(12, 8, 5, 0.57, 0.19, 0.19, true, 1);
  EdgeList e8 = gen_rmat(12, 8, 5, 0.57, 0.19, 0.19, true, T);
  CHECK(e1.u == e8.u && e1.v == e8.v);
  EdgeList u1 = gen_uniform(3000, 20000, 9, 1), u8 = gen_uniform(3000, 20000, 9, T);
  CHECK(u1.u == u8.u && u1.v == u8.v);
  // CSR build: threaded (stable order) == serial
  HostCsr c1 = build_csr(e1, 1, true), c8 = build_csr(e1, T, true);
  CHECK(c1.rowptr == c8.rowptr && c1.col == c8.col);
  CHECK(c1.nnz() == 2 * e1.m());
  // file round trip + sidecar cache (written on the first load, read on the second)
  write_edge_list_bin(gp, e1);
  EdgeList r = read_edge_list_bin(gp);
  CHECK(r.n == e1.n && r.u == e1.u && r.v == e1.v);
  unlink((gp + ".csr").c_str());
  HostCsr l1 = load_graph(gp, true, T);
  HostCsr l2 = load_graph(gp, true, T);
  CHECK(l1.rowptr == c1.rowptr && l2.rowptr == c1.rowptr && l2.col == l1.col);
  // queries: legacy and extended formats
  QuerySet q = gen_queries(c1.n, 300, 5, 7);
  write_query_bin(qp, q, false);  // K > 255 -> extended
  QuerySet q2 = read_query_bin(qp);
  CHECK(q2.off == q.off && q2.ids == q.ids);
  // query-parallel CPU BFS: threaded == serial, F and traversed edges
  std::vector<int64_t> F1, F8, E1, E8;
  cpu_msbfs_all(l1, q, F1, &E1, 1);
  cpu_msbfs_all(l1, q, F8, &E8, T);
  CHECK(F1 == F8 && E1 == E8);
  CHECK(argmin_first(F1) >= 0);
  unlink(gp.c_str());
  unlink((gp + ".csr").c_str());
  unlink(qp.c_str());
  printf("host selftest: %s (%d failed checks)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
