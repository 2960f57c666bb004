// msbfs — MI355X-native multi-source BFS / distance-to-set engine.
// Shared host/device helpers: error handling, integer types, counter-based RNG.
//
// Reference parity notes: the reference (main.cu) checks no CUDA/MPI return codes at all
// (SURVEY §2 C18); every runtime call here goes through MSBFS_HIP_CHECK and errors are
// reported through msbfs::Error / msbfs_last_error().
#pragma once

#include <cstdint>
#include <cstddef>
#include <stdexcept>
#include <string>

#if defined(__HIPCC__)
#define MSBFS_HD __host__ __device__ __forceinline__
#else
#define MSBFS_HD inline
#endif

namespace msbfs {

struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

[[noreturn]] void fail(const std::string& msg);

// ---------------------------------------------------------------------------------------
// Counter-based RNG (splitmix64 finaliser). Identical on host and device so that a graph
// generated on the GPU is edge-for-edge the graph the host generator writes to a .bin file.
// ---------------------------------------------------------------------------------------
MSBFS_HD uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Bijective scramble of a `scale`-bit vertex id (Graph500 relabels RMAT vertices so that
// vertex id carries no degree information). Each step is a bijection on [0, 2^scale):
// odd multiply mod 2^s, add, xor-shift-right.
MSBFS_HD uint64_t scramble_id(uint64_t x, int scale, uint64_t seed) {
  const uint64_t mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1);
  const uint64_t k1 = (mix64(seed ^ 0x51ED27ull) | 1ull), k2 = (mix64(seed ^ 0xC0FFEEull) | 1ull);
  const uint64_t a1 = mix64(seed ^ 0xA11CEull), a2 = mix64(seed ^ 0xB0Bull);
  const int sh = scale / 2 + 1;
  x = (x * k1 + a1) & mask;
  x ^= x >> sh;
  x = (x * k2 + a2) & mask;
  x ^= x >> sh;
  x = (x * k1 + a2) & mask;
  return x;
}

// RMAT (Kronecker) edge i of a 2^scale graph. Thresholds are the cumulative quadrant
// probabilities A, A+B, A+B+C in 32-bit fixed point. Quadrant order (Graph500):
// [0,A) -> (0,0), [A,A+B) -> (0,1), [A+B,A+B+C) -> (1,0), rest -> (1,1).
struct RmatParams {
  uint32_t tA, tAB, tABC;
  int scale;
  uint64_t seed;
  int scramble;
};

MSBFS_HD void rmat_edge(const RmatParams& p, uint64_t i, uint32_t& u_out, uint32_t& v_out) {
  const uint64_t key = mix64(p.seed ^ mix64(i + 0x1234567ull));
  uint64_t u = 0, v = 0;
  for (int l = 0; l < p.scale; l += 2) {
    const uint64_t r = mix64(key + (uint64_t)l);
    const uint32_t x0 = (uint32_t)r, x1 = (uint32_t)(r >> 32);
    {
      const uint32_t bu = x0 >= p.tAB;
      const uint32_t bv = ((x0 >= p.tA) & (x0 < p.tAB)) | (x0 >= p.tABC);
      u = (u << 1) | bu;
      v = (v << 1) | bv;
    }
    if (l + 1 < p.scale) {
      const uint32_t bu = x1 >= p.tAB;
      const uint32_t bv = ((x1 >= p.tA) & (x1 < p.tAB)) | (x1 >= p.tABC);
      u = (u << 1) | bu;
      v = (v << 1) | bv;
    }
  }
  if (p.scramble) {
    u = scramble_id(u, p.scale, p.seed);
    v = scramble_id(v, p.scale, p.seed);
  }
  u_out = (uint32_t)u;
  v_out = (uint32_t)v;
}

inline RmatParams make_rmat_params(int scale, uint64_t seed, double a, double b, double c,
                                   int scramble) {
  auto fx = [](double p) -> uint32_t {
    double s = p * 4294967296.0;
    if (s >= 4294967295.0) return 0xFFFFFFFFu;
    if (s <= 0) return 0;
    return (uint32_t)s;
  };
  RmatParams p;
  p.tA = fx(a);
  p.tAB = fx(a + b);
  p.tABC = fx(a + b + c);
  p.scale = scale;
  p.seed = seed;
  p.scramble = scramble;
  return p;
}

// Uniform random edge i over n vertices (config "1K-vertex/10K-edge random").
MSBFS_HD void uniform_edge(uint64_t seed, uint64_t i, uint64_t n, uint32_t& u, uint32_t& v) {
  const uint64_t r = mix64(seed ^ mix64(i + 0x9876543ull));
  u = (uint32_t)(((r & 0xFFFFFFFFull) * n) >> 32);
  v = (uint32_t)(((r >> 32) * n) >> 32);
}

// Random query vertex j of group k (uniform in [0, n)).
MSBFS_HD uint32_t query_vertex(uint64_t seed, uint64_t k, uint64_t j, uint64_t n) {
  const uint64_t r = mix64(seed ^ mix64((k << 20) ^ j ^ 0xABCDEFull));
  return (uint32_t)(((r >> 32) * n) >> 32);
}

}  // namespace msbfs
