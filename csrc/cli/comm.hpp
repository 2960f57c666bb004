// Process-group communication for the msbfs CLI.
//
// The reference's whole distributed layer is 13 blocking host-memory MPI call sites on
// MPI_COMM_WORLD (Bcast x(5+2K) main.cu:242-280, Gather + Gatherv with a custom
// struct datatype main.cu:328-368). Here:
//   * LocalComm — single process (also the fallback when the binary is built without MPI);
//   * ThreadComm — N ranks as N threads of one process (single-process multi-GPU mode,
//                 `--spmd N`, and the in-process fake of the test plan): shared-memory
//                 collectives, device exchanges by peer copies;
//   * MpiComm   — host MPI (MPICH): bootstrap, oversubscribed GPUs, CPU runs; large buffers are
//                 broadcast in <= 1 GiB chunks (the reference's int counts overflow at 2^31);
//   * RcclComm  — device collectives over xGMI when every rank owns a distinct GPU: the CSR is
//                 broadcast HBM -> HBM with ncclBroadcast and the result is ONE 8-byte
//                 ncclAllReduce(ncclMin) on a packed (F << qbits | q) key that keeps the
//                 reference's lowest-index tie-break (main.cu:391-396). Device scratch is
//                 persistent (no hipMalloc in the timed region) and the collectives run on the
//                 communicator's own HIP stream, so an asynchronous MIN all-reduce overlaps the
//                 next query batch's kernels on the compute stream. Bootstrap: ncclGetUniqueId
//                 over the host comm + ncclCommInitRank (one process per GPU), or
//                 ncclCommInitAll in single-process mode.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace msbfs {

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual std::string name() const = 0;
  virtual void barrier() = 0;
  virtual void bcast_host(void* p, size_t bytes, int root) = 0;
  // device broadcast; default stages through host memory
  virtual void bcast_device(void* dptr, size_t bytes, int root, hipStream_t s);
  virtual uint64_t allreduce_min_u64(uint64_t x) = 0;
  virtual void allreduce_sum_i64(int64_t* p, size_t n) = 0;
  virtual double allreduce_max_f64(double x) = 0;
  virtual void allgather_u64(uint64_t x, std::vector<uint64_t>& out) = 0;
  // all-to-all of 64-bit words between device buffers (hybrid mode's visited-word exchange):
  // scount[j] words go from send (destination-major) to rank j, rcount[r] words arrive from
  // rank r (source-major). Default: stage through host memory + alltoallv_host.
  virtual void alltoallv_device_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                                    uint64_t* recv, const std::vector<int64_t>& rcount,
                                    hipStream_t s);
  virtual void alltoallv_host_u64(const uint64_t* send, const std::vector<int64_t>& scount,
                                  uint64_t* recv, const std::vector<int64_t>& rcount) = 0;
  // One piece of a chunked all-to-all between device buffers (the overlapped hybrid exchange):
  // scount[j] words from send + soff[j] go to rank j, rcount[r] words from rank r land at
  // recv + roff[r]. Ordered after the work queued on `s` so far; may return before the words
  // moved (RcclComm: grouped ncclSend/ncclRecv on the communicator's stream while `s` goes on).
  // exchange_wait(s) orders `s` after every piece issued so far. Default: synchronous, staged
  // through host memory.
  virtual void alltoallv_piece_u64(const uint64_t* send, const std::vector<int64_t>& soff,
                                   const std::vector<int64_t>& scount, uint64_t* recv,
                                   const std::vector<int64_t>& roff,
                                   const std::vector<int64_t>& rcount, hipStream_t s);
  virtual void exchange_wait(hipStream_t s) { (void)s; }
  [[noreturn]] virtual void abort(int code) = 0;
  virtual bool device_collectives() const { return false; }
  // Size persistent device scratch for allreduce_sum_i64 of `bytes` (called before a timed
  // region so no collective allocates inside it)
  virtual void reserve_device_scratch(size_t bytes) { (void)bytes; }
  // Asynchronous MIN all-reduce of one u64 into result slot `slot` (< kAsyncSlots): issued
  // now, complete after wait_async(). RcclComm runs it on its own stream (overlapping the
  // caller's next kernels), MpiComm as MPI_Iallreduce; the default is synchronous.
  static constexpr int kAsyncSlots = 1024;
  virtual void allreduce_min_u64_async(uint64_t x, int slot);
  virtual void wait_async(uint64_t* results, int nslots);

 protected:
  std::vector<uint64_t> async_vals_;
};

// N ranks as N threads of one process (see above and thread_group.hpp). Every thread owns one
// ThreadComm of the same group; rank = thread index.
std::vector<std::unique_ptr<Comm>> make_thread_comms(int nranks);
// Single-process multi-GPU: one RCCL communicator per device (ncclCommInitAll), each wrapped
// around the thread comm of the same rank; returns the inputs unchanged without RCCL.
std::vector<std::unique_ptr<Comm>> upgrade_thread_comms_rccl(
    std::vector<std::unique_ptr<Comm>> host, const std::vector<int>& devices);

// Creates the world communicator. `want` in {"auto","mpi","rccl","local"}; `device` is this
// rank's GPU (or -1 for CPU-only runs).
std::unique_ptr<Comm> make_world_comm(int* argc, char*** argv);
std::unique_ptr<Comm> maybe_upgrade_rccl(std::unique_ptr<Comm> host, const std::string& want,
                                         int device);
void finalize_world();

}  // namespace msbfs
