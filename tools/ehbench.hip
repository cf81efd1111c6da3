// ehbench.hip -- chunk-phase shapes of the encode + piece-id kernel
// (storb_amd/csrc/rs_encode_hash.hip): PF (prefetch the next data block
// before compressing), GS (shares compressed per basic block), CVL
// (chaining values in LDS). Config-2 geometry RS(4,2), 1024 x 1 MiB chunks,
// and the storb-faithful RS(2,1) of 256 KiB chunks; every variant's parity
// and digests compared with the first one; median of REPS samples of L
// back-to-back launches.
//
// build: make -C tools ehbench
// usage: ehbench [L] [REPS]
#include "../storb_amd/csrc/rs_encode_hash.hip"
#include "../storb_amd/csrc/blake3.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

using namespace storb_rs;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e_));                                     \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void fill(uint64_t *q, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
       i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    q[i] = z ^ (z >> 31);
  }
}

struct V {
  std::string name;
  std::function<hipError_t(const EncHashArgs &, hipStream_t)> go;
  std::vector<float> ms;
  bool diag = false;  // wrong output by design: timed, not compared
};

// Hash-only shapes of the same kernel (M = 0): the stripes' data shares then
// parity shares as B-pitched messages, G per lane (messages past the last
// whole group are skipped: timing only).
template <int G, int PF>
hipError_t hash_only(const EncHashArgs &e, int K, int M, hipStream_t s) {
  auto run = [&](const uint8_t *in, uint32_t count, uint8_t *out) {
    EncHashArgs a{};
    a.data = in;
    a.data_stride = uint64_t(G) * e.block;
    a.share_stride = e.block;
    a.hashes = out;
    a.block = e.block;
    a.nstripes = count / G;
    a.nchunks = e.nchunks;
    a.seg_log2 = e.seg_log2;
    return a.nstripes ? launch_eh<G, 0, PF, 1, false, 0, 0>(a, s) : hipSuccess;
  };
  hipError_t r = run(e.data, e.nstripes * K, e.hashes + 4096);
  if (r == hipSuccess) r = run(e.parity, e.nstripes * M, e.hashes + 4096 + size_t(e.nstripes) * K * 32);
  return r;
}

template <int K, int M>
std::vector<V> variants() {
  return {
      {"PF0 GS1 regs (round-4 first cut)", launch_eh<K, M, false, 1, false>, {}},
      {"PF1 GS1 regs", launch_eh<K, M, true, 1, false>, {}},
      {"PF0 GS2 regs", launch_eh<K, M, false, 2, false>, {}},
      {"PF1 GS2 regs", launch_eh<K, M, true, 2, false>, {}},
      {"PF0 GS1 cv in LDS", launch_eh<K, M, false, 1, true>, {}},
      {"PF1 GS1 cv in LDS", launch_eh<K, M, true, 1, true>, {}},
      {"PF0 GS2 cv in LDS", launch_eh<K, M, false, 2, true>, {}},
      {"PF1 GS2 cv in LDS", launch_eh<K, M, true, 2, true>, {}},
      {"PF1 GS1 regs, write-back stores", launch_eh<K, M, true, 1, false, 0, 1>, {}},
      {"PF0 GS1 regs, write-back stores", launch_eh<K, M, false, 1, false, 0, 1>, {}},
      {"PF1 GS2 regs, write-back stores", launch_eh<K, M, true, 2, false, 0, 1>, {}},
      {"PF1 GS1 cv in LDS, write-back stores", launch_eh<K, M, true, 1, true, 0, 1>, {}},
      {"PF2 (rolling) regs, nt stores", launch_eh<K, M, 2, 1, false, 0, 0>, {}},
      {"PF2 (rolling) regs, write-back stores", launch_eh<K, M, 2, 1, false, 0, 1>, {}},
      {"PF2 (rolling) cv in LDS, nt stores", launch_eh<K, M, 2, 1, true, 0, 0>, {}},
      {"PF2 (rolling) cv in LDS, write-back", launch_eh<K, M, 2, 1, true, 0, 1>, {}},
      {"diag PF1 GS1: no GF fold", launch_eh<K, M, true, 1, false, 1>, {}, true},
      {"diag PF1 GS1: no parity stores", launch_eh<K, M, true, 1, false, 2>, {}, true},
      {"diag PF1 GS1: neither", launch_eh<K, M, true, 1, false, 3>, {}, true},
      {"hash only, 4 per lane, PF2 write-back", [](const EncHashArgs &a, hipStream_t s) {
         return hash_only<4, 2>(a, K, M, s);
       }, {}, true},
      {"hash only, 4 per lane, PF1", [](const EncHashArgs &a, hipStream_t s) {
         return hash_only<4, 1>(a, K, M, s);
       }, {}, true},
      {"hash only, 6 per lane, PF1", [](const EncHashArgs &a, hipStream_t s) {
         return hash_only<6, 1>(a, K, M, s);
       }, {}, true},
      {"hash only, 2 per lane, PF1", [](const EncHashArgs &a, hipStream_t s) {
         return hash_only<2, 1>(a, K, M, s);
       }, {}, true},
      {"reference: blake3_batch_kernel, all n shares", [](const EncHashArgs &a, hipStream_t s) {
         hipError_t e = launch_blake3_batch(a.data, a.block, a.nstripes * K, a.block,
                                            a.hashes + 4096, s);
         if (e == hipSuccess)
           e = launch_blake3_batch(a.parity, a.block, a.nstripes * M, a.block,
                                   a.hashes + 4096 + size_t(a.nstripes) * K * 32, s);
         return e;
       }, {}, true},
  };
}

template <int K, int M>
int run(uint32_t N, size_t B, int L, int reps) {
  const uint32_t n = K + M;
  uint8_t *d, *p, *h;
  CK(hipMalloc(&d, size_t(N) * K * B));
  CK(hipMalloc(&p, size_t(N) * M * B));
  CK(hipMalloc(&h, size_t(N) * n * 32 + 4096 + size_t(N) * n * 32));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(d),
                     size_t(N) * K * B / 8, 0x5709Bull);
  EncHashArgs a{};
  a.data = d;
  a.data_stride = K * B;
  a.parity = p;
  a.parity_stride = M * B;
  a.hashes = h;
  a.block = B;
  a.share_stride = B;
  a.nstripes = N;
  a.nchunks = static_cast<uint32_t>(B / 1024);
  while ((1u << a.seg_log2) < a.nchunks) a.seg_log2++;
  const std::vector<uint8_t> enc = enc_matrix(K, n);
  for (int j = 0; j < K; j++)
    for (int i = 0; i < M; i++) {
      const PermTab t = perm_tab(enc[size_t(K + i) * K + j]);
      uint32_t *w = a.tab[j * M + i];
      w[0] = t.t0lo;
      w[1] = t.t0hi;
      w[2] = t.t1lo;
      w[3] = t.t1hi;
      w[4] = t.t2;
    }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto vs = variants<K, M>();
  std::vector<uint8_t> p0(size_t(N) * M * B), h0(size_t(N) * n * 32), pg(p0.size()), hg(h0.size());
  for (size_t vi = 0; vi < vs.size(); vi++) {
    CK(hipMemsetAsync(p, 0, p0.size(), s));
    CK(hipMemsetAsync(h, 0, h0.size(), s));
    CK(vs[vi].go(a, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? pg.data() : p0.data(), p, p0.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(vi ? hg.data() : h0.data(), h, h0.size(), hipMemcpyDeviceToHost));
    if (vi && !vs[vi].diag && (std::memcmp(p0.data(), pg.data(), p0.size()) ||
               std::memcmp(h0.data(), hg.data(), h0.size()))) {
      std::printf("%s: MISMATCH\n", vs[vi].name.c_str());
      return 1;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < reps; r++)
    for (auto &v : vs) {
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < L; i++) CK(v.go(a, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float x;
      CK(hipEventElapsedTime(&x, e0, e1));
      v.ms.push_back(x / L);
    }
  const double shard_bytes = double(N) * n * B;
  std::printf("RS(%d,%d), %u stripes x %zu KiB shares (%.2f GB of shares per launch)\n", K, M, N,
              B >> 10, shard_bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float m = v.ms[v.ms.size() / 2];
    std::printf("  %-44s %.4f ms  %.0f GB/s of shares  %.1f GiB/s of chunks  %s\n",
                v.name.c_str(), m, shard_bytes / (m * 1e-3) / 1e9,
                double(N) * K * B / (m * 1e-3) / (1ull << 30), v.diag ? "" : "(bit-exact)");
  }
  CK(hipFree(d));
  CK(hipFree(p));
  CK(hipFree(h));
  return 0;
}

int main(int argc, char **argv) {
  const int L = argc > 1 ? std::atoi(argv[1]) : 5;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  if (run<4, 2>(1024, 256u << 10, L, reps)) return 1;
  if (run<2, 1>(4096, 128u << 10, L, reps)) return 1;
  return 0;
}
