// Host-side graph / query containers, binary formats, generators and the CPU BFS oracle.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "msbfs/common.hpp"

namespace msbfs {

// Symmetric CSR with 64-bit offsets (the reference uses int32 offsets, main.cu:121, which
// overflow at 2m > INT_MAX, i.e. RMAT-26 ef16). Column ids stay int32 because the
// legacy edge-list format stores int32 vertex ids (main.cu:102,108-112).
struct HostCsr {
  int64_t n = 0;
  int64_t m = 0;  // undirected input edges (duplicates and self-loops counted as in the file)
  std::vector<int64_t> rowptr;  // n+1
  std::vector<int32_t> col;     // 2m
  int64_t nnz() const { return rowptr.empty() ? 0 : rowptr.back(); }
};

// Query groups packed as CSR: group k = ids[off[k] .. off[k+1]).
struct QuerySet {
  std::vector<int64_t> off{0};
  std::vector<int32_t> ids;
  int64_t K() const { return (int64_t)off.size() - 1; }
  void add(const std::vector<int32_t>& g) {
    ids.insert(ids.end(), g.begin(), g.end());
    off.push_back((int64_t)ids.size());
  }
};

// Edge list as produced by generators / the legacy file (u[i], v[i]).
struct EdgeList {
  int64_t n = 0;
  std::vector<int32_t> u, v;
  int64_t m() const { return (int64_t)u.size(); }
};

// ---- legacy binary formats (main.cu:92-164) ----------------------------------------------
// graph: int32 n | int64 m | m x {int32 u, int32 v}, little endian, no header magic.
EdgeList read_edge_list_bin(const std::string& path);
void write_edge_list_bin(const std::string& path, const EdgeList& el);
// The legacy graph file mapped read-only and header-checked (size vs m), without copying the
// edges: the device CSR build (device_graph_from_edge_file) streams them straight to HBM.
struct EdgeFileMap {
  int64_t n = 0, m = 0;
  const uint8_t* edges = nullptr;  // m x {int32 u, int32 v}
  std::shared_ptr<void> keep;      // the mapping
};
EdgeFileMap map_edge_file(const std::string& path);
// memcpy split over nthreads host threads (page-cache -> pinned staging)
void parallel_memcpy(void* dst, const void* src, size_t bytes, int nthreads = 0);
// query: uint8 K | K x {uint8 size | size x int32}. Extended (K or a size > 255): byte 0 is 0
// (a legacy K=0 file is exactly one byte long), followed by magic "MSBFSQX1", uint32 K and
// K x {uint32 size | size x int32}. The legacy reader path is bit-exact with main.cu:134-164.
QuerySet read_query_bin(const std::string& path);
void write_query_bin(const std::string& path, const QuerySet& q, bool force_extended = false);

// Parallel count -> scan -> scatter CSR build (both directions of every edge, like
// main.cu:113-115). stable=true keeps per-vertex neighbour order = file order (main.cu:128).
HostCsr build_csr(const EdgeList& el, int nthreads = 0, bool stable = false);
// Load a graph file, using/refreshing an optional binary CSR sidecar cache (<path>.csr).
HostCsr load_graph(const std::string& path, bool use_cache, int nthreads = 0);
// Identity of a graph file for the sidecar cache: stat fields at ns resolution + a hash of the
// header and 64 sampled 4-KiB blocks. Plain data (no padding), compared bytewise.
struct CsrSourceKey {
  uint64_t size = 0, dev = 0, ino = 0;
  int64_t mtime_ns = 0, ctime_ns = 0;
  uint64_t sample_hash = 0;
};
CsrSourceKey csr_source_key(const std::string& path);
// best-effort: returns false (and leaves no file) on any failure
bool write_csr_cache(const std::string& path, const HostCsr& g, const CsrSourceKey& key);
// true only for a complete cache of the same source whose payload checksum matches
bool read_csr_cache(const std::string& path, HostCsr& g, const CsrSourceKey& key);

// ---- generators (host; device twins live in kernels/gen.hip) -------------------------------
EdgeList gen_rmat(int scale, int64_t edgefactor, uint64_t seed, double a = 0.57,
                  double b = 0.19, double c = 0.19, bool scramble = true, int nthreads = 0);
EdgeList gen_uniform(int64_t n, int64_t m, uint64_t seed, int nthreads = 0);
// rows x cols 4-neighbour grid (high-diameter "road-like" graph); each edge kept with
// probability keep (deterministic in seed), plus `shortcuts` random long edges.
EdgeList gen_grid(int64_t rows, int64_t cols, double keep, int64_t shortcuts, uint64_t seed);
QuerySet gen_queries(int64_t n, int64_t K, int64_t size, uint64_t seed);

// ---- CPU multi-source BFS oracle ------------------------------------------------------------
// F(U) = sum over vertices reachable from U of dist(U, v); sources outside [0,n) ignored
// (main.cu:49); unreachable vertices contribute nothing (main.cu:84-85).
// Also returns, if edges != nullptr, the traversed-edge count of the group (sum of degrees of
// reached vertices / 2 — the Graph500 TEPS numerator).
int64_t cpu_msbfs_F(const HostCsr& g, const int32_t* src, int64_t nsrc, std::vector<int32_t>& dist,
                    std::vector<int64_t>& queue, int64_t* edges = nullptr,
                    int32_t* levels = nullptr);
// All groups, query-parallel over nthreads host threads.
void cpu_msbfs_all(const HostCsr& g, const QuerySet& q, std::vector<int64_t>& F,
                   std::vector<int64_t>* edges, int nthreads);

// Reference tie-break (main.cu:381-397): first valid F, then strict '<'; returns -1 if K==0.
int64_t argmin_first(const std::vector<int64_t>& F);

int default_threads();

}  // namespace msbfs
