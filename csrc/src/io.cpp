// Binary graph/query I/O, parallel CSR build and the CSR sidecar cache.
//
// Reference: LoadGraphBin main.cu:92-130 (per-element fread, vector<vector<int>> adjacency,
// int32 offsets) and LoadQueryBin main.cu:134-164 (uint8 K, uint8 sizes). Here the file is
// mmap'd, validated (truncation, id range — UB in the reference), and turned into an
// int64-offset CSR by a multi-threaded count -> scan -> scatter.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <thread>

#include "msbfs/graph.hpp"

namespace msbfs {

void fail(const std::string& msg) { throw Error(msg); }

int default_threads() {
  unsigned hc = std::thread::hardware_concurrency();
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    int v = atoi(e);
    if (v > 0) return v;
  }
  return hc ? (int)std::min(hc, 64u) : 4;
}

template <class F>
static void parallel_for(int nthreads, int64_t total, F&& fn) {
  if (nthreads <= 1 || total < 65536) {
    fn(0, total, 0);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (total + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t b = t * chunk, e = std::min(total, b + chunk);
    if (b >= e) break;
    th.emplace_back([&fn, b, e, t] { fn(b, e, t); });
  }
  for (auto& x : th) x.join();
}

namespace {
struct MappedFile {
  int fd = -1;
  void* p = nullptr;
  size_t size = 0;
  int64_t mtime = 0;
  explicit MappedFile(const std::string& path, const char* what) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) fail(std::string("Could not open ") + what + " file " + path);
    struct stat st;
    if (fstat(fd, &st) != 0) fail("stat failed on " + path);
    size = (size_t)st.st_size;
    mtime = (int64_t)st.st_mtime;
    if (size) {
      p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) fail("mmap failed on " + path);
      madvise(p, size, MADV_SEQUENTIAL);
    }
  }
  ~MappedFile() {
    if (p && p != MAP_FAILED) munmap(p, size);
    if (fd >= 0) ::close(fd);
  }
  const uint8_t* bytes() const { return (const uint8_t*)p; }
};

void write_all(FILE* f, const void* p, size_t n, const std::string& path) {
  if (n && fwrite(p, 1, n, f) != n) fail("short write to " + path);
}
}  // namespace

EdgeFileMap map_edge_file(const std::string& path) {
  auto mf = std::make_shared<MappedFile>(path, "graph");
  if (mf->size < 12) fail("graph file " + path + " is truncated (need 12-byte header)");
  int32_t n;
  int64_t m;
  std::memcpy(&n, mf->bytes(), 4);
  std::memcpy(&m, mf->bytes() + 4, 8);
  if (n < 0 || m < 0) fail("graph file " + path + " has a negative n or m");
  const uint64_t need = 12ull + 8ull * (uint64_t)m;
  if (mf->size < need)
    fail("graph file " + path + " is truncated: header says m=" + std::to_string(m) +
         " edges but the file holds " + std::to_string((mf->size - 12) / 8));
  EdgeFileMap f;
  f.n = n;
  f.m = m;
  f.edges = mf->bytes() + 12;
  f.keep = mf;
  return f;
}

void parallel_memcpy(void* dst, const void* src, size_t bytes, int nthreads) {
  if (nthreads <= 0) nthreads = default_threads();
  constexpr size_t kGrain = size_t(1) << 22;
  const int64_t pieces = (int64_t)((bytes + kGrain - 1) / kGrain);
  if (pieces <= 1 || nthreads <= 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < std::min<int64_t>(nthreads, pieces); ++t)
    th.emplace_back([&] {
      for (int64_t i; (i = next.fetch_add(1)) < pieces;) {
        const size_t o = (size_t)i * kGrain;
        std::memcpy((char*)dst + o, (const char*)src + o, std::min(kGrain, bytes - o));
      }
    });
  for (auto& x : th) x.join();
}

EdgeList read_edge_list_bin(const std::string& path) {
  MappedFile mf(path, "graph");
  if (mf.size < 12) fail("graph file " + path + " is truncated (need 12-byte header)");
  int32_t n;
  int64_t m;
  std::memcpy(&n, mf.bytes(), 4);
  std::memcpy(&m, mf.bytes() + 4, 8);
  if (n < 0 || m < 0) fail("graph file " + path + " has a negative n or m");
  const uint64_t need = 12ull + 8ull * (uint64_t)m;
  if (mf.size < need)
    fail("graph file " + path + " is truncated: header says m=" + std::to_string(m) +
         " edges but the file holds " + std::to_string((mf.size - 12) / 8));
  EdgeList el;
  el.n = n;
  el.u.resize(m);
  el.v.resize(m);
  const uint8_t* base = mf.bytes() + 12;
  std::atomic<int64_t> bad{-1};
  parallel_for(default_threads(), m, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      int32_t uv[2];
      std::memcpy(uv, base + 8 * i, 8);
      el.u[i] = uv[0];
      el.v[i] = uv[1];
      if ((uint32_t)uv[0] >= (uint32_t)n || (uint32_t)uv[1] >= (uint32_t)n) {
        int64_t exp = -1;
        bad.compare_exchange_strong(exp, i);
      }
    }
  });
  if (bad.load() >= 0)
    fail("graph file " + path + ": edge " + std::to_string(bad.load()) +
         " has a vertex id outside [0, n)");
  return el;
}

void write_edge_list_bin(const std::string& path, const EdgeList& el) {
  if (el.n > INT32_MAX) fail("legacy graph format stores n as int32");
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) fail("Could not open graph file " + path + " for writing");
  const int32_t n = (int32_t)el.n;
  const int64_t m = el.m();
  write_all(f, &n, 4, path);
  write_all(f, &m, 8, path);
  std::vector<int32_t> buf;
  const int64_t B = 1 << 20;
  for (int64_t i = 0; i < m; i += B) {
    const int64_t e = std::min(m, i + B);
    buf.resize(2 * (e - i));
    for (int64_t j = i; j < e; ++j) {
      buf[2 * (j - i)] = el.u[j];
      buf[2 * (j - i) + 1] = el.v[j];
    }
    write_all(f, buf.data(), buf.size() * 4, path);
  }
  if (fclose(f) != 0) fail("close failed on " + path);
}

static const char kQxMagic[8] = {'M', 'S', 'B', 'F', 'S', 'Q', 'X', '1'};

QuerySet read_query_bin(const std::string& path) {
  MappedFile mf(path, "query");
  const uint8_t* p = mf.bytes();
  const size_t sz = mf.size;
  QuerySet q;
  if (sz < 1) fail("query file " + path + " is empty (need at least the K byte)");
  size_t pos = 0;
  auto need = [&](size_t k) {
    if (pos + k > sz) fail("query file " + path + " is truncated at byte " + std::to_string(pos));
  };
  if (p[0] == 0 && sz >= 1 + 8 + 4 && std::memcmp(p + 1, kQxMagic, 8) == 0) {
    // extended format
    pos = 9;
    uint32_t K;
    std::memcpy(&K, p + pos, 4);
    pos += 4;
    q.off.reserve(K + 1);
    for (uint32_t k = 0; k < K; ++k) {
      need(4);
      uint32_t s;
      std::memcpy(&s, p + pos, 4);
      pos += 4;
      need(4ull * s);
      const size_t base = q.ids.size();
      q.ids.resize(base + s);
      std::memcpy(q.ids.data() + base, p + pos, 4ull * s);
      pos += 4ull * s;
      q.off.push_back((int64_t)q.ids.size());
    }
    return q;
  }
  // legacy format: uint8 K, then K x {uint8 size, size x int32} (main.cu:143-160)
  const int K = p[0];
  pos = 1;
  for (int k = 0; k < K; ++k) {
    need(1);
    const int s = p[pos++];
    need(4ull * s);
    const size_t base = q.ids.size();
    q.ids.resize(base + s);
    std::memcpy(q.ids.data() + base, p + pos, 4ull * s);
    pos += 4ull * s;
    q.off.push_back((int64_t)q.ids.size());
  }
  return q;
}

void write_query_bin(const std::string& path, const QuerySet& q, bool force_extended) {
  const int64_t K = q.K();
  bool ext = force_extended || K > 255;
  for (int64_t k = 0; k < K && !ext; ++k) ext = (q.off[k + 1] - q.off[k]) > 255;
  if (ext && K == 0) ext = true;
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) fail("Could not open query file " + path + " for writing");
  if (!ext) {
    const uint8_t k8 = (uint8_t)K;
    write_all(f, &k8, 1, path);
    for (int64_t k = 0; k < K; ++k) {
      const uint8_t s = (uint8_t)(q.off[k + 1] - q.off[k]);
      write_all(f, &s, 1, path);
      write_all(f, q.ids.data() + q.off[k], 4ull * s, path);
    }
  } else {
    if (K > UINT32_MAX) fail("too many query groups");
    const uint8_t z = 0;
    const uint32_t k32 = (uint32_t)K;
    write_all(f, &z, 1, path);
    write_all(f, kQxMagic, 8, path);
    write_all(f, &k32, 4, path);
    for (int64_t k = 0; k < K; ++k) {
      const uint32_t s = (uint32_t)(q.off[k + 1] - q.off[k]);
      write_all(f, &s, 4, path);
      write_all(f, q.ids.data() + q.off[k], 4ull * s, path);
    }
  }
  if (fclose(f) != 0) fail("close failed on " + path);
}

HostCsr build_csr(const EdgeList& el, int nthreads, bool stable) {
  if (nthreads <= 0) nthreads = default_threads();
  HostCsr g;
  g.n = el.n;
  g.m = el.m();
  const int64_t n = el.n, m = el.m();
  g.rowptr.assign(n + 1, 0);
  int64_t* deg = g.rowptr.data() + 1;
  parallel_for(nthreads, m, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      __atomic_fetch_add(&deg[el.u[i]], 1, __ATOMIC_RELAXED);
      __atomic_fetch_add(&deg[el.v[i]], 1, __ATOMIC_RELAXED);
    }
  });
  for (int64_t i = 0; i < n; ++i) g.rowptr[i + 1] += g.rowptr[i];
  g.col.resize(2 * m);
  std::vector<int64_t> cur(g.rowptr.begin(), g.rowptr.end() - 1);
  if (stable || nthreads <= 1 || m < 65536) {
    // exact reference neighbour order: adj[u] += v; adj[v] += u in file order
    for (int64_t i = 0; i < m; ++i) {
      g.col[cur[el.u[i]]++] = el.v[i];
      g.col[cur[el.v[i]]++] = el.u[i];
    }
  } else {
    parallel_for(nthreads, m, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) {
        const int32_t u = el.u[i], v = el.v[i];
        g.col[__atomic_fetch_add(&cur[u], 1, __ATOMIC_RELAXED)] = v;
        g.col[__atomic_fetch_add(&cur[v], 1, __ATOMIC_RELAXED)] = u;
      }
    });
  }
  return g;
}

// ---- CSR sidecar cache (<graph>.csr) ---------------------------------------------------------
// Not in the reference (it re-reads the edge list every run); opt-in (`--cache`). A cache entry is
// only used when it was built from the very same source file: the key holds the file's size,
// device/inode, mtime and ctime with nanosecond resolution (a rewrite within the same second
// still changes ctime_ns) and a hash of the 12-byte header plus 64 sampled 4-KiB blocks of the
// edge list (two graphs with the same n and m differ there with overwhelming probability). The
// payload carries its own checksum, so a truncated or corrupted cache is rejected, not used.
static const char kCsrMagic[8] = {'M', 'S', 'B', 'F', 'S', 'C', 'R', '2'};

namespace {
inline uint64_t mix64(uint64_t h, uint64_t x) {
  h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0xFF51AFD7ED558CCDull;
  return h ^ (h >> 33);
}
uint64_t hash_bytes(const uint8_t* p, size_t n, uint64_t h) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x;
    std::memcpy(&x, p + i, 8);
    h = mix64(h, x);
  }
  uint64_t tail = 0;
  if (i < n) std::memcpy(&tail, p + i, n - i);
  return mix64(h, tail ^ ((uint64_t)n << 56));
}
// order-dependent hash of a large buffer, 64-MiB pieces hashed in parallel
uint64_t hash_parallel(const void* data, size_t bytes, uint64_t seed) {
  const size_t piece = 64ull << 20;
  const int64_t np = (int64_t)((bytes + piece - 1) / piece);
  std::vector<uint64_t> ph((size_t)std::max<int64_t>(np, 1), 0);
  const uint8_t* p = (const uint8_t*)data;
  const int T = (int)std::min<int64_t>(std::min(default_threads(), 16), np);
  auto work = [&](int t) {
    for (int64_t i = t; i < np; i += T) {
      const size_t off = (size_t)i * piece;
      ph[i] = hash_bytes(p + off, std::min(piece, bytes - off), seed + (uint64_t)i);
    }
  };
  if (T <= 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  uint64_t h = mix64(seed, bytes);
  for (int64_t i = 0; i < np; ++i) h = mix64(h, ph[i]);
  return h;
}
}  // namespace

CsrSourceKey csr_source_key(const std::string& path) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) fail("Could not open graph file " + path);
  CsrSourceKey k;
  k.size = (uint64_t)st.st_size;
  k.dev = (uint64_t)st.st_dev;
  k.ino = (uint64_t)st.st_ino;
  k.mtime_ns = (int64_t)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec;
  k.ctime_ns = (int64_t)st.st_ctim.tv_sec * 1000000000ll + st.st_ctim.tv_nsec;
  uint64_t h = 0x6D73626673ull;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) fail("Could not open graph file " + path);
  std::vector<uint8_t> buf(4096);
  auto sample = [&](uint64_t off, size_t len) {
    if (off >= k.size) return;
    len = (size_t)std::min<uint64_t>(len, k.size - off);
    if (fseeko(f, (off_t)off, SEEK_SET) != 0 || fread(buf.data(), 1, len, f) != len) {
      fclose(f);
      fail("read failed on " + path);
    }
    h = hash_bytes(buf.data(), len, mix64(h, off));
  };
  sample(0, 12);
  const int kSamples = 64;
  for (int i = 0; i < kSamples; ++i) sample(12 + (k.size > 12 ? (k.size - 12) / kSamples * i : 0), 4096);
  if (k.size > 4096) sample(k.size - 4096, 4096);
  fclose(f);
  k.sample_hash = h;
  return k;
}

bool write_csr_cache(const std::string& path, const HostCsr& g, const CsrSourceKey& key) {
  // best-effort: any failure leaves no file behind and is not an error of the load
  static std::atomic<uint64_t> seq{0};
  const std::string tmp = path + ".tmp." + std::to_string((long long)getpid()) + "." +
                          std::to_string((unsigned long long)seq.fetch_add(1));
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;
  bool ok = true;
  try {
    const uint64_t sum = mix64(hash_parallel(g.rowptr.data(), 8 * g.rowptr.size(), 1),
                               hash_parallel(g.col.data(), 4 * g.col.size(), 2));
    write_all(f, kCsrMagic, 8, tmp);
    write_all(f, &key, sizeof(key), tmp);
    write_all(f, &g.n, 8, tmp);
    write_all(f, &g.m, 8, tmp);
    write_all(f, &sum, 8, tmp);
    write_all(f, g.rowptr.data(), 8 * g.rowptr.size(), tmp);
    write_all(f, g.col.data(), 4 * g.col.size(), tmp);
  } catch (const Error&) {
    ok = false;
  }
  if (fclose(f) != 0) ok = false;
  if (ok && rename(tmp.c_str(), path.c_str()) != 0) ok = false;
  if (!ok) unlink(tmp.c_str());
  return ok;
}

bool read_csr_cache(const std::string& path, HostCsr& g, const CsrSourceKey& key) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  char magic[8];
  CsrSourceKey k;
  int64_t n, m;
  uint64_t sum;
  bool ok = fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kCsrMagic, 8) == 0 &&
            fread(&k, sizeof(k), 1, f) == 1 && std::memcmp(&k, &key, sizeof(k)) == 0 &&
            fread(&n, 8, 1, f) == 1 && fread(&m, 8, 1, f) == 1 && fread(&sum, 8, 1, f) == 1 &&
            n >= 0 && m >= 0 && n < (int64_t)1 << 40 && m < (int64_t)1 << 40;
  HostCsr c;
  if (ok) {
    c.n = n;
    c.m = m;
    c.rowptr.resize(n + 1);
    c.col.resize(2 * m);
    ok = fread(c.rowptr.data(), 8, n + 1, f) == (size_t)(n + 1) &&
         fread(c.col.data(), 4, 2 * m, f) == (size_t)(2 * m) && fgetc(f) == EOF &&
         c.rowptr.front() == 0 && c.rowptr.back() == 2 * m &&
         mix64(hash_parallel(c.rowptr.data(), 8 * c.rowptr.size(), 1),
               hash_parallel(c.col.data(), 4 * c.col.size(), 2)) == sum;
  }
  fclose(f);
  if (ok) g = std::move(c);
  return ok;
}

HostCsr load_graph(const std::string& path, bool use_cache, int nthreads) {
  HostCsr g;
  const std::string cpath = path + ".csr";
  CsrSourceKey key;
  if (use_cache) {
    key = csr_source_key(path);
    if (read_csr_cache(cpath, g, key)) return g;
  }
  EdgeList el = read_edge_list_bin(path);
  g = build_csr(el, nthreads, false);
  if (use_cache) {
    el = EdgeList();
    // the source must not have changed while it was parsed
    CsrSourceKey after;
    bool same = false;
    try {
      after = csr_source_key(path);
      same = std::memcmp(&after, &key, sizeof(key)) == 0;
    } catch (const Error&) {
    }
    if (same) write_csr_cache(cpath, g, key);
  }
  return g;
}

int64_t argmin_first(const std::vector<int64_t>& F) {
  int64_t minF = -1, minK = -1;
  for (size_t i = 0; i < F.size(); ++i)
    if (F[i] >= 0) {
      minF = F[i];
      minK = (int64_t)i;
      break;
    }
  for (size_t i = 0; i < F.size(); ++i)
    if (F[i] < minF && F[i] >= 0) {
      minF = F[i];
      minK = (int64_t)i;
    }
  return minK;
}

}  // namespace msbfs
