// Process-group communication for the msbfs CLI.
//
// The reference's whole distributed layer is 13 blocking host-memory MPI call sites on
// MPI_COMM_WORLD (Bcast x(5+2K) main.cu:242-280, Gather + Gatherv with a custom
// struct datatype main.cu:328-368). Here:
//   * LocalComm — single process (also the fallback when the binary is built without MPI);
//   * MpiComm   — host MPI (MPICH): bootstrap, oversubscribed GPUs, CPU runs; large buffers are
//                 broadcast in <= 1 GiB chunks (the reference's int counts overflow at 2^31);
//   * RcclComm  — device collectives over xGMI when every rank owns a distinct GPU: the CSR is
//                 broadcast HBM -> HBM with ncclBroadcast and the result is ONE 8-byte
//                 ncclAllReduce(ncclMin) on a packed (F << qbits | q) key that keeps the
//                 reference's lowest-index tie-break (main.cu:391-396).
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
  [[noreturn]] virtual void abort(int code) = 0;
  virtual bool device_collectives() const { return false; }
};

// Creates the world communicator. `want` in {"auto","mpi","rccl","local"}; `device` is this
// rank's GPU (or -1 for CPU-only runs).
std::unique_ptr<Comm> make_world_comm(int* argc, char*** argv);
std::unique_ptr<Comm> maybe_upgrade_rccl(std::unique_ptr<Comm> host, const std::string& want,
                                         int device);
void finalize_world();

}  // namespace msbfs
