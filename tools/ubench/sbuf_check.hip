// Structured-buffer semantics the k_bu_full pull relies on (bitpar/pull_full.hpp), checked on the
// device before any solver uses them:
//  1. index == num_records reads zeros (the range check), although the allocation holds data there;
//  (an index 0xFFFFFFFF read is never tried: round 4 found no index range check, check 1)
//  3. index * stride beyond 4 GiB addresses the right row (a 5 GiB buffer);
//  4. a store at index == num_records is dropped.
// hipcc -O3 --offload-arch=gfx950 tools/ubench/sbuf_check.hip -o build/sbuf_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__device__ u4 sload(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");
__device__ void sstore(u4 v, __amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                       int aux) __asm("llvm.amdgcn.struct.ptr.buffer.store.v4i32");

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);      \
      return 2;                                                             \
    }                                                                       \
  } while (0)

// lane l reads the 16-byte slice (l % 8) of row idx[l / 8]
__global__ void k_read(const uint64_t* base, int nrec, const uint32_t* idx, u4* out) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)128, nrec, 0x00020000);
  const int l = threadIdx.x;
  out[l] = sload(r, (int)idx[l / 8], (l % 8) * 16, 0, 0);
}
__global__ void k_write(uint64_t* base, int nrec, uint32_t idx) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)128, nrec, 0x00020000);
  u4 v = {0xdeadbeefu, 0xdeadbeefu, 0xdeadbeefu, 0xdeadbeefu};
  sstore(v, r, (int)idx, (threadIdx.x % 8) * 16, 0, 0);
}
// row i, word j = i * 16 + j + 1 (never zero)
__global__ void k_fill(uint64_t* p, int64_t rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * 16;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (uint64_t)i + 1;
}

static int read_rows(const uint64_t* d, int nrec, std::vector<uint32_t> rows,
                     std::vector<uint64_t>& got) {
  uint32_t* di;
  u4* dout;
  std::vector<uint32_t> idx(64);
  for (int l = 0; l < 64; ++l) idx[l] = rows[l / 8];
  CK(hipMalloc(&di, 64 * 4));
  CK(hipMalloc(&dout, 64 * 16));
  CK(hipMemcpy(di, idx.data(), 64 * 4, hipMemcpyHostToDevice));
  k_read<<<1, 64>>>(d, nrec, di, dout);
  CK(hipGetLastError());
  got.assign(8 * 16, 0);
  CK(hipMemcpy(got.data(), dout, 64 * 16, hipMemcpyDeviceToHost));
  CK(hipFree(di));
  CK(hipFree(dout));
  return 0;
}

int main() {
  const int64_t rows = 40 * 1000 * 1000;  // 5.12 GB of 128-byte rows
  uint64_t* d;
  CK(hipMalloc(&d, (size_t)rows * 128));
  k_fill<<<4096, 256>>>(d, rows);
  CK(hipDeviceSynchronize());
  auto expect = [](int64_t r, int j) { return (uint64_t)(r * 16 + j + 1); };
  std::vector<uint64_t> got;
  int bad = 0;
  // 1. in-range rows and index == num_records (nrec = 1000: row 1000 holds data)
  if (read_rows(d, 1000, {0, 1, 999, 1000, 5, 1000, 7, 998}, got)) return 2;
  const int64_t want1[8] = {0, 1, 999, -1, 5, -1, 7, 998};
  for (int v = 0; v < 8; ++v)
    for (int j = 0; j < 16; ++j) {
      const uint64_t w = want1[v] < 0 ? 0 : expect(want1[v], j);
      if (got[v * 16 + j] != w) ++bad;
    }
  printf("check 1 (range check at index == num_records): %s\n", bad ? "FAIL" : "ok");
  for (int v = 0; v < 8; ++v)  // what each row read returned (word 0 and 15)
    printf("  row %lld: got %llu %llu want %llu %llu\n", (long long)want1[v],
           (unsigned long long)got[v * 16], (unsigned long long)got[v * 16 + 15],
           (unsigned long long)(want1[v] < 0 ? 0 : expect(want1[v], 0)),
           (unsigned long long)(want1[v] < 0 ? 0 : expect(want1[v], 15)));
  // (no index -1 read: without the range check it would address 512 GB past the base)
  bad = 0;
  // 3. rows beyond 4 GiB (row 33554432 starts at exactly 4 GiB; num_records = rows + 8, all
  // reads in bounds)
  if (read_rows(d, (int)rows + 8, {33554431, 33554432, 33554433, 39999999, 35000000, 0, 36000001,
                                   0}, got))
    return 2;
  const int64_t want3[8] = {33554431, 33554432, 33554433, 39999999, 35000000, 0, 36000001, 0};
  for (int v = 0; v < 8; ++v)
    for (int j = 0; j < 16; ++j) {
      const uint64_t w = want3[v] < 0 ? 0 : expect(want3[v], j);
      if (got[v * 16 + j] != w) ++bad;
    }
  printf("check 3 (index * stride beyond 4 GiB): %s\n", bad ? "FAIL" : "ok");
  for (int v = 0; v < 7; ++v)
    printf("  row %lld: got %llu want %llu\n", (long long)want3[v],
           (unsigned long long)got[v * 16], (unsigned long long)expect(want3[v], 0));
  if (bad) return 1;
  // 4. a store at index == num_records is dropped; one in range lands
  k_write<<<1, 64>>>(d, 1000, 1000);
  k_write<<<1, 64>>>(d, 1000, 10);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> h(16 * 2);
  CK(hipMemcpy(h.data(), d + 1000 * 16, 16 * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h.data() + 16, d + 10 * 16, 16 * 8, hipMemcpyDeviceToHost));
  for (int j = 0; j < 16; ++j) {
    if (h[j] != expect(1000, j)) ++bad;
    if (h[16 + j] != 0xdeadbeefdeadbeefull) ++bad;
  }
  printf("check 4 (out-of-range store dropped): %s\n", bad ? "FAIL" : "ok");
  CK(hipFree(d));
  return bad ? 1 : 0;
}
