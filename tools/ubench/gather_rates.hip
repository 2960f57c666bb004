// Gather-rate microbenchmark for the level-2 pull's access shapes (MI355X, gfx950).
//
// A table of R rows of 128 bytes (W = 16 visited words, 1024 groups) is gathered by a stream of
// random row indices, the way the first bottom-up level gathers the level-1 frontier rows of its
// hub neighbours. Shapes:
//   rows<G>   G lanes per row (16 B per lane for G = 8, 8 B for G = 16, 2 x 16 B for G = 4),
//             64/G rows per wave instruction, U instructions in flight per wave
//   code      one lane per index, one 4-byte word per row (the sparse row codes)
//   code8     one lane per index, one 8-byte word per row
//   code16    one lane per index, one 16-byte word per row
//   idx       the index stream alone (coalesced 4-byte loads)
//   ldsdma    rows<8> through global_load_lds_dwordx4 into a per-wave LDS buffer, then ds_read
// Prints G rows (or indices) per second and the gathered TB/s for each table size.
//
//   hipcc -O3 --offload-arch=gfx950 -o gather_rates gather_rates.hip && ./gather_rates
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kW = 16;  // words per row

// G lanes per row; each lane reads 16*8/G bytes of it
template <int G, int U>
__global__ __launch_bounds__(256) void k_rows(const uint64_t* __restrict__ X,
                                              const int32_t* __restrict__ idx, int64_t N,
                                              uint64_t* out) {
  constexpr int S = 64 / G;         // rows per wave instruction
  constexpr int LW = kW / G;        // words per lane
  const int lane = threadIdx.x & 63, slot = lane % G, sub = lane / G;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  uint64_t acc[LW];
#pragma unroll
  for (int j = 0; j < LW; ++j) acc[j] = 0;
  for (int64_t b = wave * (S * U); b < N; b += nw * (S * U)) {
    int32_t r[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t i = b + q * S + sub;
      r[q] = i < N ? idx[i] : -1;
    }
    uint64_t x[U][LW];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      if (r[q] >= 0) {
        const uint64_t* p = X + (int64_t)r[q] * kW + slot * LW;
        if constexpr (LW == 1) {
          x[q][0] = p[0];
        } else {
#pragma unroll
          for (int j = 0; j < LW; j += 2) {
            const ulonglong2 v = *(const ulonglong2*)(p + j);
            x[q][j] = v.x;
            x[q][j + 1] = v.y;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < LW; ++j) x[q][j] = 0;
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q)
#pragma unroll
      for (int j = 0; j < LW; ++j) acc[j] |= x[q][j];
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < LW; ++j) s ^= acc[j];
  if (s == 0x123456789ull) out[0] = s;  // keep the loads
}

// one lane per index, B bytes per row (4, 8 or 16)
template <int B, int U>
__global__ __launch_bounds__(256) void k_code(const uint32_t* __restrict__ X,
                                              const int32_t* __restrict__ idx, int64_t N,
                                              uint64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = (int64_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (int64_t b = t; b < N; b += nt * U) {
    int32_t r[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t i = b + q * nt;
      r[q] = i < N ? idx[i] : -1;
    }
    uint64_t x[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      x[q] = 0;
      if (r[q] >= 0) {
        if constexpr (B == 4) {
          x[q] = X[r[q]];
        } else if constexpr (B == 8) {
          x[q] = ((const uint64_t*)X)[r[q]];
        } else {
          const ulonglong2 v = ((const ulonglong2*)X)[r[q]];
          x[q] = v.x ^ v.y;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q) acc |= x[q];
  }
  if (acc == 0x123456789ull) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_idx(const int32_t* __restrict__ idx, int64_t N,
                                             uint64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = (int64_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (int64_t i = t; i < N; i += nt) acc += (uint32_t)idx[i];
  if (acc == 0x123456789ull) out[0] = acc;
}

// rows<8> through LDS DMA: each wave instruction lands 8 rows (1 KB) in the wave's LDS buffer
template <int U>
__global__ __launch_bounds__(256) void k_ldsdma(const uint64_t* __restrict__ X,
                                                const int32_t* __restrict__ idx, int64_t N,
                                                uint64_t* out) {
  constexpr int S = 8;
  __shared__ uint64_t buf[4][U][128];  // per wave: U slices of 8 rows x 16 words
  const int lane = threadIdx.x & 63, slot = lane % 8, sub = lane / 8, wv = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  uint64_t acc0 = 0, acc1 = 0;
  for (int64_t b = wave * (S * U); b < N; b += nw * (S * U)) {
    int32_t r[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t i = b + q * S + sub;
      r[q] = i < N ? idx[i] : 0;
    }
#pragma unroll
    for (int q = 0; q < U; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(X + (int64_t)r[q] * kW + slot * 2),
                                       (__attribute__((address_space(3))) void*)&buf[wv][q][0],
                                       16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const ulonglong2 v = *(const ulonglong2*)&buf[wv][q][lane * 2];
      acc0 |= v.x;
      acc1 |= v.y;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if ((acc0 ^ acc1) == 0x123456789ull) out[0] = acc0;
}

static uint64_t rng = 88172645463325252ull;
static uint64_t nxt() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

int main(int argc, char** argv) {
  const int64_t N = (int64_t)1 << 26;
  const int grid = 256 * 8;
  std::vector<int64_t> tables = {18000, 458752, 8 << 20};
  uint64_t* X;
  int32_t* idx;
  uint64_t* out;
  CK(hipMalloc(&X, (size_t)(8 << 20) * 128));
  CK(hipMemset(X, 0x5a, (size_t)(8 << 20) * 128));
  CK(hipMalloc(&idx, N * 4));
  CK(hipMalloc(&out, 64));
  std::vector<int32_t> h(N);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int64_t R : tables) {
    for (int64_t i = 0; i < N; ++i) h[i] = (int32_t)(nxt() % (uint64_t)R);
    CK(hipMemcpy(idx, h.data(), N * 4, hipMemcpyHostToDevice));
    auto run = [&](const char* name, auto launch, double bytes_per) {
      launch();
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("table %8lld rows (%7.1f MB)  %-10s %8.3f ms  %7.1f G/s  %6.2f TB/s\n",
             (long long)R, R * 128 / 1e6, name, best, N / best / 1e6,
             N * bytes_per / best / 1e9);
      fflush(stdout);
    };
    run("idx", [&] { k_idx<<<grid, 256>>>(idx, N, out); }, 4);
    run("rows<4>", [&] { k_rows<4, 4><<<grid, 256>>>(X, idx, N, out); }, 128);
    run("rows<8>", [&] { k_rows<8, 4><<<grid, 256>>>(X, idx, N, out); }, 128);
    run("rows<8>u8", [&] { k_rows<8, 8><<<grid, 256>>>(X, idx, N, out); }, 128);
    run("rows<16>", [&] { k_rows<16, 4><<<grid, 256>>>(X, idx, N, out); }, 128);
    run("code4", [&] { k_code<4, 4><<<grid, 256>>>((const uint32_t*)X, idx, N, out); }, 4);
    run("code8", [&] { k_code<8, 4><<<grid, 256>>>((const uint32_t*)X, idx, N, out); }, 8);
    run("code16", [&] { k_code<16, 4><<<grid, 256>>>((const uint32_t*)X, idx, N, out); }, 16);
    run("ldsdma<8>", [&] { k_ldsdma<4><<<grid, 256>>>(X, idx, N, out); }, 128);
  }
  return 0;
}
