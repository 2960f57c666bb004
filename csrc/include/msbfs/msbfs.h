/* msbfs — MI355X-native multi-source BFS / distance-to-set engine. Public C API.
 *
 * Capability parity with the reference (irmakerkol/Parallel-Multi-Source-BFS-Implementation-
 * Using-MPI-and-CUDA, main.cu): binary edge-list graph + query loaders (main.cu:92-164),
 * symmetric CSR, per-group multi-source BFS + F(U) (main.cu:16-89), round-robin distribution
 * and global argmin (main.cu:303-397). All functions return 0 on success and a negative value
 * on error; msbfs_last_error() returns the thread-local message.
 */
#ifndef MSBFS_H_
#define MSBFS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct msbfs_graph_s* msbfs_graph;
typedef struct msbfs_solver_s* msbfs_solver;

enum msbfs_algo {
  MSBFS_ALGO_AUTO = 0,    /* dist for <= 2 groups on graphs with max degree > 64, else bit-parallel */
  MSBFS_ALGO_BITPAR = 1,  /* 64*W groups per pass, direction optimising */
  MSBFS_ALGO_DIST = 2,    /* one distance array per group, direction optimising */
  MSBFS_ALGO_TOPDOWN = 3, /* dist path, top-down only (queue + load-balanced edges) */
  MSBFS_ALGO_SWEEP = 4,   /* reference algorithm: thread per vertex, full sweep per level */
  MSBFS_ALGO_CPU = 5      /* host threads (oracle / "serial CPU BFS" config) */
};

typedef struct {
  int64_t levels, td_levels, bu_levels, batches;
  double device_ms;
} msbfs_stats;

/* one BFS level of the last run (bit-parallel solver): direction 'T' (top-down push) or 'B'
 * (bottom-up pull), union frontier size / degree sum entering the level, vertices newly visited
 * by some group, bottom-up active (or top-down touched) vertices, host wall time of the level */
typedef struct {
  int32_t batch, level;
  char dir, pad[3];
  int64_t nf, ef, nf_next, active;
  double ms;
} msbfs_level;

typedef struct {
  double alpha, beta;
  int wide_degree, force_dir, max_words;
} msbfs_options;

const char* msbfs_last_error(void);
const char* msbfs_version(void);
void msbfs_free(void* p);

/* ---- devices ---- */
int msbfs_device_count(int* n);
int msbfs_set_device(int dev);
int msbfs_device_sync(void);

/* ---- host formats / generators (buffers returned via malloc; free with msbfs_free) ---- */
int msbfs_read_graph_csr(const char* path, int use_cache, int64_t* n, int64_t* m,
                         int64_t** rowptr, int32_t** col);
int msbfs_read_edge_list(const char* path, int64_t* n, int64_t* m, int32_t** u, int32_t** v);
int msbfs_write_edge_list(const char* path, int64_t n, int64_t m, const int32_t* u,
                          const int32_t* v);
int msbfs_read_queries(const char* path, int64_t* K, int64_t** off, int64_t* nids, int32_t** ids);
int msbfs_write_queries(const char* path, int64_t K, const int64_t* off, const int32_t* ids,
                        int force_extended);
int msbfs_build_csr(int64_t n, int64_t m, const int32_t* u, const int32_t* v, int stable,
                    int64_t** rowptr, int32_t** col);
int msbfs_gen_rmat_host(int scale, int64_t edgefactor, uint64_t seed, double a, double b, double c,
                        int scramble, int32_t** u, int32_t** v, int64_t* n, int64_t* m);
int msbfs_gen_uniform_host(int64_t n, int64_t m, uint64_t seed, int32_t** u, int32_t** v);
int msbfs_gen_grid_host(int64_t rows, int64_t cols, double keep, int64_t shortcuts, uint64_t seed,
                        int32_t** u, int32_t** v, int64_t* n, int64_t* m);
int msbfs_gen_queries(int64_t n, int64_t K, int64_t size, uint64_t seed, int64_t** off,
                      int32_t** ids);

/* ---- CPU BFS (query-parallel host threads) ---- */
int msbfs_cpu_run(int64_t n, const int64_t* rowptr, const int32_t* col, int64_t K,
                  const int64_t* qoff, const int32_t* qids, int64_t* F, int64_t* edges,
                  int nthreads);

/* ---- device graphs ---- */
int msbfs_graph_from_host_csr(int device, int64_t n, const int64_t* rowptr, const int32_t* col,
                              msbfs_graph* out);
int msbfs_graph_from_device_edges(int device, int64_t n, int64_t m, const int32_t* d_u,
                                  const int32_t* d_v, msbfs_graph* out);
int msbfs_graph_wrap_device(int device, int64_t n, int64_t nnz, int64_t* d_rowptr, int32_t* d_col,
                            msbfs_graph* out);
int msbfs_graph_gen_rmat(int device, int scale, int64_t edgefactor, uint64_t seed, double a,
                         double b, double c, int scramble, msbfs_graph* out);
int msbfs_graph_gen_uniform(int device, int64_t n, int64_t m, uint64_t seed, msbfs_graph* out);
/* the legacy edge-list file (main.cu:92-130) built into a CSR on the device (streamed upload,
 * device count -> scan -> scatter; no host edge arrays) */
int msbfs_graph_from_edge_file(int device, const char* path, msbfs_graph* out);
int msbfs_graph_sort_rows(msbfs_graph g);
/* Renumber vertices by descending degree (hubs first, rows sorted). Queries keep using the
 * original ids: solvers map sources through the stored old->new map. */
int msbfs_graph_relabel_by_degree(msbfs_graph g);
int msbfs_graph_relabel_map(msbfs_graph g, int32_t* old2new);
int msbfs_graph_is_relabelled(msbfs_graph g);
int msbfs_graph_info(msbfs_graph g, int64_t* n, int64_t* nnz, int64_t* m, int64_t* max_degree,
                     int64_t* isolated);
int msbfs_graph_device_ptrs(msbfs_graph g, void** rowptr, void** col);
int msbfs_graph_download(msbfs_graph g, int64_t* rowptr, int32_t* col);
void msbfs_graph_free(msbfs_graph g);

/* ---- solvers ---- */
int msbfs_solver_create(msbfs_graph g, int algo, int64_t max_groups, msbfs_solver* out);
int msbfs_solver_set_options(msbfs_solver s, const msbfs_options* o);
/* Algorithm tuning "key=value,key=value" (bit-parallel solver keys: gamma gamma2 pfx codes
 * code_deg lean lean_min lazy td_fused td_bm batch dirs; defaults are the measured best).
 * Unknown keys or bad values fail with an error; other solvers accept only an empty spec. The
 * process-wide defaults come from MSBFS_TUNE (same syntax, read once, echoed on stderr). */
int msbfs_solver_tune(msbfs_solver s, const char* spec);
/* Build graph-derived tables and worst-case scratch now instead of in the first run (the CLI
 * calls it during preprocessing; optional). */
int msbfs_solver_prepare(msbfs_solver s, void* stream);
/* The same for the hybrid phase A of rank `part` of `nparts` (call it before timing hybrid runs). */
int msbfs_solver_prepare_hybrid(msbfs_solver s, int part, int nparts, void* stream);
/* F[k] for k in [0,K); edges2 (nullable) = per-group sum of reached degrees (2x the Graph500
 * traversed-edge count). stream = hipStream_t or NULL for the null stream. */
int msbfs_solver_run(msbfs_solver s, int64_t K, const int64_t* qoff, const int32_t* qids,
                     int64_t* F, int64_t* edges2, msbfs_stats* st, void* stream);
/* per-level records of the solver's last run / hybrid phase: copies min(n, cap) records to out
 * (nullable) and returns n (or -1 for a null solver) */
int64_t msbfs_solver_levels(msbfs_solver s, msbfs_level* out, int64_t cap);
void msbfs_solver_free(msbfs_solver s);

/* ---- hybrid multi-GPU mode (bit-parallel solver) ----
 * Levels 1-2 vertex-partitioned (each rank: all K groups, bottom-up pulls only for its vertices
 * v = part + i*nparts < n_eff), one all-to-all of visited words, remaining levels
 * query-partitioned (rank j owns the groups of words [wbeg[j], wbeg[j+1]) of ceil(K/64)). The
 * caller does the communication (cnt_r = number of vertices of part r):
 *   A: phase_a -> send_dev (device, cnt_me*ceil(K/64) u64, destination-major), out[2K+3]
 *   exchange: all-to-all send -> recv (rank j receives cnt_r*(wbeg[j+1]-wbeg[j]) u64 from each
 *             rank r, in rank order), all-reduce SUM of out -> reduced
 *   C: phase_c(recv, reduced) -> F_local[64*nwords] (levels >= 3 of the own groups)
 *   F[k] = reduced[k] + F_local[k - 64*wbeg[rank]] for the own groups. */
int msbfs_hybrid_extent(msbfs_graph g, int64_t* n_eff);
int64_t msbfs_solver_hybrid_max_groups(msbfs_solver s);
int msbfs_solver_hybrid_phase_a(msbfs_solver s, int64_t K, const int64_t* qoff,
                                const int32_t* qids, int part, int nparts, int64_t n_eff,
                                int count_l1, const int32_t* wbeg, void* send_dev, int64_t* out,
                                msbfs_stats* st, void* stream);
/* Zero-word coded exchange (about half the bytes after level 2): phase_a_coded writes one coded
 * segment per destination j back to back into send_dev (at most cnt_me*nw_j + ceil(cnt_me*nw_j/64)
 * u64 each; coded_len[j] = its length, host) and decode expands the received segments (coded_len[r]
 * u64 from each rank r, in rank order) into the dense recv layout phase_c reads. */
int msbfs_solver_hybrid_phase_a_coded(msbfs_solver s, int64_t K, const int64_t* qoff,
                                      const int32_t* qids, int part, int nparts, int64_t n_eff,
                                      int count_l1, const int32_t* wbeg, void* send_dev,
                                      int64_t* out, int64_t* coded_len, msbfs_stats* st,
                                      void* stream);
/* Overlapped exchange (dense layout): phase A in `chunks` own-vertex ranges
 * [bounds[c], bounds[c+1]) (msbfs_solver_hybrid_chunk_bounds, bounds[chunks+1]); after each
 * range's words are packed into send_dev (pack enqueued on `stream`), cb(user, c, i0, i1) runs
 * on the calling thread: it starts that piece of the all-to-all ordered after `stream` (e.g. an
 * asynchronous collective on the communicator's stream) while the next range computes. */
typedef void (*msbfs_chunk_fn)(void* user, int chunk, int64_t i0, int64_t i1);
int msbfs_solver_hybrid_chunk_bounds(msbfs_solver s, int part, int nparts, int64_t n_eff,
                                     int chunks, int64_t* bounds);
int msbfs_solver_hybrid_phase_a_chunked(msbfs_solver s, int64_t K, const int64_t* qoff,
                                        const int32_t* qids, int part, int nparts,
                                        int64_t n_eff, int count_l1, const int32_t* wbeg,
                                        void* send_dev, int64_t* out, int chunks,
                                        msbfs_chunk_fn cb, void* user, msbfs_stats* st,
                                        void* stream);
int msbfs_solver_hybrid_decode(msbfs_solver s, const void* coded_dev, const int64_t* coded_len,
                               int nparts, int64_t n_eff, int w_count, void* dense_dev,
                               void* stream);
int msbfs_solver_hybrid_phase_c(msbfs_solver s, int64_t K, int w_begin, int w_count, int nparts,
                                int64_t n_eff, const void* recv_dev, const int64_t* reduced,
                                int64_t* F_local, msbfs_stats* st, void* stream);

/* reference argmin (main.cu:381-397): first valid, strict '<', lowest index wins ties; -1 if K=0 */
int64_t msbfs_argmin(const int64_t* F, int64_t K);

#ifdef __cplusplus
}
#endif
#endif /* MSBFS_H_ */
