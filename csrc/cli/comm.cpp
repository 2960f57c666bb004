#include "comm.hpp"

#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>

#include "msbfs/device.hpp"
#include "thread_group.hpp"

#ifdef MSBFS_HAVE_MPI
#include <mpi.h>
#endif
#ifdef MSBFS_HAVE_RCCL
#include <rccl/rccl.h>
#endif

namespace msbfs {

void Comm::bcast_device(void* dptr, size_t bytes, int root, hipStream_t s) {
  if (size() == 1 || bytes == 0) return;
  std::vector<char> h(bytes);
  if (rank() == root) {
    MSBFS_HIP_CHECK(hipMemcpyAsync(h.data(), dptr, bytes, hipMemcpyDeviceToHost, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  bcast_host(h.data(), bytes, root);
  if (rank() != root) {
    MSBFS_HIP_CHECK(hipMemcpyAsync(dptr, h.data(), bytes, hipMemcpyHostToDevice, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
}

void Comm::alltoallv_device_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                                uint64_t* recv, const std::vector<int64_t>& rcount,
                                hipStream_t s) {
  int64_t ns = 0, nr = 0;
  for (int64_t c : scount) ns += c;
  for (int64_t c : rcount) nr += c;
  std::vector<uint64_t> hs(std::max<int64_t>(ns, 1)), hr(std::max<int64_t>(nr, 1));
  if (ns) MSBFS_HIP_CHECK(hipMemcpyAsync(hs.data(), send, ns * 8, hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  alltoallv_host_u64(hs.data(), scount, hr.data(), rcount);
  if (nr) MSBFS_HIP_CHECK(hipMemcpyAsync(recv, hr.data(), nr * 8, hipMemcpyHostToDevice, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
}

void Comm::alltoallv_piece_u64(const uint64_t* send, const std::vector<int64_t>& soff,
                               const std::vector<int64_t>& scount, uint64_t* recv,
                               const std::vector<int64_t>& roff,
                               const std::vector<int64_t>& rcount, hipStream_t s) {
  int64_t ns = 0, nr = 0;
  for (int64_t c : scount) ns += c;
  for (int64_t c : rcount) nr += c;
  std::vector<uint64_t> hs(std::max<int64_t>(ns, 1)), hr(std::max<int64_t>(nr, 1));
  int64_t o = 0;
  for (size_t j = 0; j < scount.size(); o += scount[j], ++j)
    if (scount[j])
      MSBFS_HIP_CHECK(hipMemcpyAsync(hs.data() + o, send + soff[j], scount[j] * 8,
                                     hipMemcpyDeviceToHost, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  alltoallv_host_u64(hs.data(), scount, hr.data(), rcount);
  o = 0;
  for (size_t r = 0; r < rcount.size(); o += rcount[r], ++r)
    if (rcount[r])
      MSBFS_HIP_CHECK(hipMemcpyAsync(recv + roff[r], hr.data() + o, rcount[r] * 8,
                                     hipMemcpyHostToDevice, s));
  MSBFS_HIP_CHECK(hipStreamSynchronize(s));
}

void Comm::allreduce_min_u64_async(uint64_t x, int slot) {
  if (slot < 0 || slot >= kAsyncSlots) fail("async all-reduce slot out of range");
  if ((int)async_vals_.size() <= slot) async_vals_.resize(slot + 1, ~0ull);
  async_vals_[slot] = allreduce_min_u64(x);
}

void Comm::wait_async(uint64_t* results, int nslots) {
  for (int i = 0; i < nslots; ++i) results[i] = i < (int)async_vals_.size() ? async_vals_[i] : ~0ull;
  async_vals_.clear();
}

namespace {

class LocalComm final : public Comm {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  std::string name() const override { return "local"; }
  void barrier() override {}
  void bcast_host(void*, size_t, int) override {}
  uint64_t allreduce_min_u64(uint64_t x) override { return x; }
  void allreduce_sum_i64(int64_t*, size_t) override {}
  double allreduce_max_f64(double x) override { return x; }
  void allgather_u64(uint64_t x, std::vector<uint64_t>& out) override { out.assign(1, x); }
  void alltoallv_host_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                          uint64_t* recv, const std::vector<int64_t>&) override {
    if (scount[0]) std::memcpy(recv, send, scount[0] * 8);
  }
  void alltoallv_device_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                            uint64_t* recv, const std::vector<int64_t>&, hipStream_t s) override {
    if (scount[0])
      MSBFS_HIP_CHECK(hipMemcpyAsync(recv, send, scount[0] * 8, hipMemcpyDeviceToDevice, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  [[noreturn]] void abort(int code) override { std::exit(code); }
};

}  // namespace

namespace {

class ThreadComm final : public Comm {
 public:
  ThreadComm(std::shared_ptr<ThreadGroup> g, int rank) : g_(std::move(g)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return g_->size; }
  std::string name() const override { return "threads"; }
  void barrier() override { g_->sync(); }
  void bcast_host(void* p, size_t bytes, int root) override {
    tg_bcast(*g_, rank_, p, bytes, root);
  }
  void bcast_device(void* dptr, size_t bytes, int root, hipStream_t s) override {
    if (rank_ == root) g_->cptrs[root] = dptr;
    int dev = 0;
    MSBFS_HIP_CHECK(hipGetDevice(&dev));
    g_->vals[rank_] = (uint64_t)dev;
    g_->sync();
    if (rank_ != root && bytes) {
      MSBFS_HIP_CHECK(hipMemcpyPeerAsync(dptr, dev, g_->cptrs[root], (int)g_->vals[root], bytes, s));
      MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    }
    g_->sync();
  }
  uint64_t allreduce_min_u64(uint64_t x) override { return tg_allreduce_min(*g_, rank_, x); }
  void allreduce_sum_i64(int64_t* p, size_t n) override { tg_allreduce_sum(*g_, rank_, p, n); }
  double allreduce_max_f64(double x) override { return tg_allreduce_max(*g_, rank_, x); }
  void allgather_u64(uint64_t x, std::vector<uint64_t>& out) override {
    tg_allgather(*g_, rank_, x, out);
  }
  void alltoallv_host_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                          uint64_t* recv, const std::vector<int64_t>& rcount) override {
    tg_alltoallv(*g_, rank_, send, scount, recv, rcount);
  }
  void alltoallv_device_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                            uint64_t* recv, const std::vector<int64_t>& rcount,
                            hipStream_t s) override {
    int dev = 0;
    MSBFS_HIP_CHECK(hipGetDevice(&dev));
    g_->cptrs[rank_] = send;
    g_->counts[rank_] = &scount;
    g_->vals[rank_] = (uint64_t)dev;
    g_->sync();
    // every receiver pulls its pieces (peer copies over xGMI when the ranks own different GPUs)
    int64_t ro = 0;
    for (int r = 0; r < g_->size; ++r) {
      if (rcount[r] != (*g_->counts[r])[rank_]) fail("threads all-to-all: count mismatch");
      if (rcount[r])
        MSBFS_HIP_CHECK(hipMemcpyPeerAsync(recv + ro, dev,
                                           (const uint64_t*)g_->cptrs[r] + tg_send_offset(*g_, r, rank_),
                                           (int)g_->vals[r], rcount[r] * 8, s));
      ro += rcount[r];
    }
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
    g_->sync();
  }
  [[noreturn]] void abort(int code) override {
    // one process is the whole job: end it (peer threads may be blocked in a collective)
    fflush(stdout);
    fflush(stderr);
    std::_Exit(code);
  }

 private:
  std::shared_ptr<ThreadGroup> g_;
  int rank_;
};

#ifdef MSBFS_HAVE_MPI
constexpr size_t kChunk = size_t(1) << 30;

class MpiComm : public Comm {
 public:
  MpiComm() {
    MPI_Comm_rank(MPI_COMM_WORLD, &rank_);
    MPI_Comm_size(MPI_COMM_WORLD, &size_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return "mpi"; }
  void barrier() override { MPI_Barrier(MPI_COMM_WORLD); }
  void bcast_host(void* p, size_t bytes, int root) override {
    char* c = (char*)p;
    for (size_t off = 0; off < bytes; off += kChunk) {
      const int cnt = (int)std::min(kChunk, bytes - off);
      MPI_Bcast(c + off, cnt, MPI_BYTE, root, MPI_COMM_WORLD);
    }
  }
  uint64_t allreduce_min_u64(uint64_t x) override {
    uint64_t r = x;
    MPI_Allreduce(&x, &r, 1, MPI_UINT64_T, MPI_MIN, MPI_COMM_WORLD);
    return r;
  }
  void allreduce_sum_i64(int64_t* p, size_t n) override {
    for (size_t off = 0; off < n; off += kChunk / 8) {
      const int cnt = (int)std::min(kChunk / 8, n - off);
      MPI_Allreduce(MPI_IN_PLACE, p + off, cnt, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
    }
  }
  double allreduce_max_f64(double x) override {
    double r = x;
    MPI_Allreduce(&x, &r, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    return r;
  }
  void allgather_u64(uint64_t x, std::vector<uint64_t>& out) override {
    out.resize(size_);
    MPI_Allgather(&x, 1, MPI_UINT64_T, out.data(), 1, MPI_UINT64_T, MPI_COMM_WORLD);
  }
  void alltoallv_host_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                          uint64_t* recv, const std::vector<int64_t>& rcount) override {
    // MPI counts are int: every peer block travels as <= 1 GiB pieces; both sides derive the
    // same piece count from the same block size, so nonblocking pieces pair up exactly
    std::vector<MPI_Request> req;
    const int64_t piece = (int64_t)(kChunk / 8);
    int64_t so = 0, ro = 0;
    for (int j = 0; j < size_; ++j) {
      for (int64_t o = 0; o < rcount[j]; o += piece) {
        req.emplace_back();
        MPI_Irecv(recv + ro + o, (int)std::min(piece, rcount[j] - o), MPI_UINT64_T, j, 7,
                  MPI_COMM_WORLD, &req.back());
      }
      for (int64_t o = 0; o < scount[j]; o += piece) {
        req.emplace_back();
        MPI_Isend(send + so + o, (int)std::min(piece, scount[j] - o), MPI_UINT64_T, j, 7,
                  MPI_COMM_WORLD, &req.back());
      }
      so += scount[j];
      ro += rcount[j];
    }
    if (!req.empty()) MPI_Waitall((int)req.size(), req.data(), MPI_STATUSES_IGNORE);
  }
  void allreduce_min_u64_async(uint64_t x, int slot) override {
    if (slot < 0 || slot >= kAsyncSlots) fail("async all-reduce slot out of range");
    if (in_.empty()) {  // fixed storage: buffers of in-flight requests never move
      in_.assign(kAsyncSlots, ~0ull);
      out_.assign(kAsyncSlots, ~0ull);
      req_.assign(kAsyncSlots, MPI_REQUEST_NULL);
    }
    in_[slot] = x;
    nused_ = std::max(nused_, slot + 1);
    MPI_Iallreduce(&in_[slot], &out_[slot], 1, MPI_UINT64_T, MPI_MIN, MPI_COMM_WORLD, &req_[slot]);
  }
  void wait_async(uint64_t* results, int nslots) override {
    if (nused_) MPI_Waitall(nused_, req_.data(), MPI_STATUSES_IGNORE);
    for (int i = 0; i < nslots; ++i) results[i] = i < nused_ ? out_[i] : ~0ull;
    nused_ = 0;
  }
  [[noreturn]] void abort(int code) override {
    // unlike main.cu:98,140 (exit without MPI_Abort -> peers hang in MPI_Bcast), take the job down
    MPI_Abort(MPI_COMM_WORLD, code);
    std::exit(code);
  }

 private:
  int rank_ = 0, size_ = 1;
  // in-flight asynchronous all-reduces (kAsyncSlots entries allocated once)
  std::vector<uint64_t> in_, out_;
  std::vector<MPI_Request> req_;
  int nused_ = 0;
};
#endif

#ifdef MSBFS_HAVE_RCCL
#define NCCL_CHECK(x)                                                                     \
  do {                                                                                    \
    ncclResult_t r_ = (x);                                                                \
    if (r_ != ncclSuccess) ::msbfs::fail(std::string("RCCL error: ") + ncclGetErrorString(r_)); \
  } while (0)

// RCCL prints a version banner on stdout at init; the report on stdout must stay the
// reference's 7 lines (main.cu:403-414), so the banner goes to stderr
template <class F>
ncclResult_t quiet_init(F&& f) {
  fflush(stdout);
  const int saved = dup(1);
  if (saved >= 0) dup2(2, 1);
  const ncclResult_t r = f();
  fflush(stdout);
  if (saved >= 0) {
    dup2(saved, 1);
    close(saved);
  }
  return r;
}

class RcclComm final : public Comm {
 public:
  // one process per GPU: unique id over the host communicator, ncclCommInitRank
  RcclComm(std::unique_ptr<Comm> host, int device) : host_(std::move(host)), device_(device) {
    ncclUniqueId id;
    if (host_->rank() == 0) NCCL_CHECK(ncclGetUniqueId(&id));
    host_->bcast_host(&id, sizeof(id), 0);
    MSBFS_HIP_CHECK(hipSetDevice(device_));
    NCCL_CHECK(quiet_init([&] { return ncclCommInitRank(&comm_, host_->size(), id, host_->rank()); }));
    setup();
  }
  // single-process mode: a communicator made by ncclCommInitAll for this rank's device
  RcclComm(std::unique_ptr<Comm> host, int device, ncclComm_t comm)
      : host_(std::move(host)), device_(device), comm_(comm) {
    MSBFS_HIP_CHECK(hipSetDevice(device_));
    setup();
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
    if (scratch_) (void)hipFree(scratch_);
    if (hstage_) (void)hipHostFree(hstage_);
    if (hkeys_) (void)hipHostFree(hkeys_);
    if (piece_ev_) (void)hipEventDestroy(piece_ev_);
    if (done_ev_) (void)hipEventDestroy(done_ev_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  int rank() const override { return host_->rank(); }
  int size() const override { return host_->size(); }
  std::string name() const override { return "rccl"; }
  bool device_collectives() const override { return true; }
  void barrier() override { host_->barrier(); }
  void bcast_host(void* p, size_t bytes, int root) override { host_->bcast_host(p, bytes, root); }
  void bcast_device(void* dptr, size_t bytes, int root, hipStream_t s) override {
    // chunked ring broadcast HBM -> HBM over xGMI
    const size_t chunk = size_t(1) << 30;
    for (size_t off = 0; off < bytes; off += chunk)
      NCCL_CHECK(ncclBroadcast((char*)dptr + off, (char*)dptr + off, std::min(chunk, bytes - off),
                               ncclInt8, root, comm_, s));
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  uint64_t allreduce_min_u64(uint64_t x) override {
    uint64_t* hk = hkeys_ + 2 * kAsyncSlots;  // a slot of its own (not an async slot)
    hk[0] = x;
    MSBFS_HIP_CHECK(hipMemcpyAsync(key_dev(kAsyncSlots), hk, 8, hipMemcpyHostToDevice, stream_));
    NCCL_CHECK(ncclAllReduce(key_dev(kAsyncSlots), key_dev(kAsyncSlots), 1, ncclUint64, ncclMin,
                             comm_, stream_));
    MSBFS_HIP_CHECK(hipMemcpyAsync(hk + 1, key_dev(kAsyncSlots), 8, hipMemcpyDeviceToHost, stream_));
    MSBFS_HIP_CHECK(hipStreamSynchronize(stream_));
    return hk[1];
  }
  void reserve_device_scratch(size_t bytes) override { ensure(bytes); }
  void allreduce_sum_i64(int64_t* p, size_t n) override {
    if (!n) return;
    ensure(n * 8);  // persistent: reserve_device_scratch() sizes it before any timed region
    std::memcpy(hstage_, p, n * 8);
    int64_t* d = (int64_t*)((char*)scratch_ + kKeyBytes);
    MSBFS_HIP_CHECK(hipMemcpyAsync(d, hstage_, n * 8, hipMemcpyHostToDevice, stream_));
    NCCL_CHECK(ncclAllReduce(d, d, n, ncclInt64, ncclSum, comm_, stream_));
    MSBFS_HIP_CHECK(hipMemcpyAsync(hstage_, d, n * 8, hipMemcpyDeviceToHost, stream_));
    MSBFS_HIP_CHECK(hipStreamSynchronize(stream_));
    std::memcpy(p, hstage_, n * 8);
  }
  // issued on the communicator's stream: runs beside the caller's next kernels
  void allreduce_min_u64_async(uint64_t x, int slot) override {
    if (slot < 0 || slot >= kAsyncSlots) fail("async all-reduce slot out of range");
    hkeys_[slot] = x;
    MSBFS_HIP_CHECK(hipMemcpyAsync(key_dev(slot), hkeys_ + slot, 8, hipMemcpyHostToDevice, stream_));
    NCCL_CHECK(ncclAllReduce(key_dev(slot), key_dev(slot), 1, ncclUint64, ncclMin, comm_, stream_));
    MSBFS_HIP_CHECK(hipMemcpyAsync(hkeys_ + kAsyncSlots + slot, key_dev(slot), 8,
                                   hipMemcpyDeviceToHost, stream_));
    nasync_ = std::max(nasync_, slot + 1);
  }
  void wait_async(uint64_t* results, int nslots) override {
    MSBFS_HIP_CHECK(hipStreamSynchronize(stream_));
    for (int i = 0; i < nslots; ++i) results[i] = i < nasync_ ? hkeys_[kAsyncSlots + i] : ~0ull;
    nasync_ = 0;
  }
  double allreduce_max_f64(double x) override { return host_->allreduce_max_f64(x); }
  void allgather_u64(uint64_t x, std::vector<uint64_t>& out) override {
    host_->allgather_u64(x, out);
  }
  void alltoallv_host_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                          uint64_t* recv, const std::vector<int64_t>& rcount) override {
    host_->alltoallv_host_u64(send, scount, recv, rcount);
  }
  // a piece of the overlapped exchange: the comm stream waits for the caller's stream (the pack
  // of this piece), then one grouped send/recv round runs there while the caller goes on
  void alltoallv_piece_u64(const uint64_t* send, const std::vector<int64_t>& soff,
                           const std::vector<int64_t>& scount, uint64_t* recv,
                           const std::vector<int64_t>& roff, const std::vector<int64_t>& rcount,
                           hipStream_t s) override {
    MSBFS_HIP_CHECK(hipEventRecord(piece_ev_, s));
    MSBFS_HIP_CHECK(hipStreamWaitEvent(stream_, piece_ev_, 0));
    const int P = size();
    NCCL_CHECK(ncclGroupStart());
    for (int j = 0; j < P; ++j) {
      if (scount[j])
        NCCL_CHECK(ncclSend(send + soff[j], (size_t)scount[j], ncclUint64, j, comm_, stream_));
      if (rcount[j])
        NCCL_CHECK(ncclRecv(recv + roff[j], (size_t)rcount[j], ncclUint64, j, comm_, stream_));
    }
    NCCL_CHECK(ncclGroupEnd());
  }
  void exchange_wait(hipStream_t s) override {
    MSBFS_HIP_CHECK(hipEventRecord(done_ev_, stream_));
    MSBFS_HIP_CHECK(hipStreamWaitEvent(s, done_ev_, 0));
  }
  void alltoallv_device_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                            uint64_t* recv, const std::vector<int64_t>& rcount,
                            hipStream_t s) override {
    // one grouped point-to-point round: every pair of GPUs talks over its own xGMI link at once
    const int P = size();
    int64_t so = 0, ro = 0;
    NCCL_CHECK(ncclGroupStart());
    for (int j = 0; j < P; ++j) {
      if (scount[j]) NCCL_CHECK(ncclSend(send + so, (size_t)scount[j], ncclUint64, j, comm_, s));
      if (rcount[j]) NCCL_CHECK(ncclRecv(recv + ro, (size_t)rcount[j], ncclUint64, j, comm_, s));
      so += scount[j];
      ro += rcount[j];
    }
    NCCL_CHECK(ncclGroupEnd());
    MSBFS_HIP_CHECK(hipStreamSynchronize(s));
  }
  [[noreturn]] void abort(int code) override {
    if (comm_) ncclCommAbort(comm_);
    comm_ = nullptr;
    host_->abort(code);
  }

 private:
  // device scratch: (kAsyncSlots + 1) key slots, then the all-reduce staging area
  static constexpr size_t kKeyBytes = ((size_t)(kAsyncSlots + 1) * 8 + 255) & ~size_t(255);
  uint64_t* key_dev(int slot) const { return (uint64_t*)scratch_ + slot; }
  void setup() {
    MSBFS_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    MSBFS_HIP_CHECK(hipEventCreateWithFlags(&piece_ev_, hipEventDisableTiming));
    MSBFS_HIP_CHECK(hipEventCreateWithFlags(&done_ev_, hipEventDisableTiming));
    MSBFS_HIP_CHECK(hipHostMalloc((void**)&hkeys_, (2 * kAsyncSlots + 2) * 8, hipHostMallocDefault));
    ensure(64 << 10);
  }
  void ensure(size_t bytes) {
    if (bytes <= cap_ && scratch_) return;
    const size_t cap = std::max(bytes, cap_ * 2);
    if (scratch_) (void)hipFree(scratch_);
    if (hstage_) (void)hipHostFree(hstage_);
    MSBFS_HIP_CHECK(hipMalloc(&scratch_, kKeyBytes + cap));
    MSBFS_HIP_CHECK(hipHostMalloc(&hstage_, cap, hipHostMallocDefault));
    cap_ = cap;
  }
  std::unique_ptr<Comm> host_;
  int device_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;  // the communicator's own stream (collectives, async keys)
  void* scratch_ = nullptr;
  void* hstage_ = nullptr;        // pinned staging of allreduce_sum_i64
  uint64_t* hkeys_ = nullptr;     // pinned: async inputs, async results, one sync slot pair
  size_t cap_ = 0;
  int nasync_ = 0;
  hipEvent_t piece_ev_ = nullptr, done_ev_ = nullptr;  // overlapped exchange ordering
};
#endif

bool g_mpi_inited = false;

}  // namespace

std::unique_ptr<Comm> make_world_comm(int* argc, char*** argv) {
#ifdef MSBFS_HAVE_MPI
  if (!getenv("MSBFS_NO_MPI")) {
    MPI_Init(argc, argv);
    g_mpi_inited = true;
    return std::make_unique<MpiComm>();
  }
#endif
  (void)argc;
  (void)argv;
  return std::make_unique<LocalComm>();
}

std::unique_ptr<Comm> maybe_upgrade_rccl(std::unique_ptr<Comm> host, const std::string& want,
                                         int device) {
  // one rank: plain host comm, unless RCCL is asked for explicitly (a one-rank communicator
  // still runs every device collective: the RCCL code paths on a one-GPU box)
  if (want == "mpi" || want == "local" || device < 0 || (host->size() == 1 && want != "rccl"))
    return host;
#ifdef MSBFS_HAVE_RCCL
  // RCCL needs one rank per GPU: check (host, device) pairs are unique across the job.
  char hn[256] = {0};
  gethostname(hn, sizeof(hn) - 1);
  const uint64_t key = (std::hash<std::string>{}(hn) & ~0xFFFFull) | (uint64_t)(device & 0xFFFF);
  std::vector<uint64_t> keys;
  host->allgather_u64(key, keys);
  std::sort(keys.begin(), keys.end());
  const bool unique = std::adjacent_find(keys.begin(), keys.end()) == keys.end();
  if (!unique) {
    if (want == "rccl" && host->rank() == 0)
      fprintf(stderr, "msbfs: --comm rccl needs one rank per GPU; falling back to MPI\n");
    return host;
  }
  return std::make_unique<RcclComm>(std::move(host), device);
#else
  if (want == "rccl" && host->rank() == 0)
    fprintf(stderr, "msbfs: built without RCCL/MPI; using %s\n", host->name().c_str());
  return host;
#endif
}

std::vector<std::unique_ptr<Comm>> make_thread_comms(int nranks) {
  auto g = std::make_shared<ThreadGroup>(nranks);
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < nranks; ++r) out.push_back(std::make_unique<ThreadComm>(g, r));
  return out;
}

std::vector<std::unique_ptr<Comm>> upgrade_thread_comms_rccl(
    std::vector<std::unique_ptr<Comm>> host, const std::vector<int>& devices) {
#ifdef MSBFS_HAVE_RCCL
  const int n = (int)host.size();
  std::vector<int> d(devices);
  std::sort(d.begin(), d.end());
  if (n < 1 || (int)devices.size() != n || std::adjacent_find(d.begin(), d.end()) != d.end())
    return host;  // RCCL needs one rank per GPU
  std::vector<ncclComm_t> comms(n);
  NCCL_CHECK(quiet_init([&] { return ncclCommInitAll(comms.data(), n, devices.data()); }));
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r)
    out.push_back(std::make_unique<RcclComm>(std::move(host[r]), devices[r], comms[r]));
  return out;
#else
  (void)devices;
  return host;
#endif
}

void finalize_world() {
#ifdef MSBFS_HAVE_MPI
  if (g_mpi_inited) MPI_Finalize();
#endif
}

}  // namespace msbfs
