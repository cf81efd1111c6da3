// kbench.hip -- variant study for the RS(4,2) encode kernel on gfx950.
//
// One process, interleaved rounds (cdna_hip_programming.md 5.4 rule 24):
// each variant's parity is checked bit-exact against the product kernel
// (rs_apply_perm<4,2,true> from storb_amd/csrc), then timed with HIP events.
// A "copy" kernel with the same traffic shape (read 4 shards, write 2) but no
// GF math measures the memory ceiling for this access pattern.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../storb_amd/csrc \
//        kbench.hip ../storb_amd/csrc/rs_perm_k4.hip -o _build/kbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "rs_device.hpp"
#include "rs_kernels.hpp"

using namespace storb_rs;


#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,       \
                   hipGetErrorString(e));                                   \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

struct Enc42 {
  const uint8_t *data;
  uint8_t *parity;
  uint64_t B;  // shard bytes
  uint32_t nstripes;
  PermTab t[2][4];
};

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <int U, bool NTL, bool NTS, bool COPY>
__device__ __forceinline__ void enc_unit(const Enc42 &a, uint32_t stripe, uint32_t c0,
                                         uint32_t step) {
  const uint32_t cols = a.B >> 4;
  const u32x4 *in = reinterpret_cast<const u32x4 *>(a.data + (uint64_t)stripe * 4 * a.B);
  u32x4 *out = reinterpret_cast<u32x4 *>(a.parity + (uint64_t)stripe * 2 * a.B);
  u32x4 x[4][U];
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int u = 0; u < U; u++) x[j][u] = ld<NTL>(in + j * cols + c0 + u * step);
  u32x4 acc[2][U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    if constexpr (COPY) {
      acc[0][u] = x[0][u] ^ x[1][u];
      acc[1][u] = x[2][u] ^ x[3][u];
    } else {
      acc[0][u] = acc[1][u] = u32x4{0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int w = 0; w < 4; w++) {
          const uint32_t d = x[j][u][w];
          const uint32_t s0 = d & 0x07070707u, s1 = (d >> 3) & 0x07070707u,
                         s2 = (d >> 6) & 0x03030303u;
#pragma unroll
          for (int i = 0; i < 2; i++) acc[i][u][w] ^= gf_mul_perm(a.t[i][j], s0, s1, s2);
        }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(out + i * cols + c0 + u * step, acc[i][u]);
}

// One tile per block (like the product kernel), tables in kernel args.
template <int T, int U, bool NTL, bool NTS, bool COPY>
__global__ __launch_bounds__(T) void k_tile(const Enc42 a) {
  const uint32_t cols = a.B >> 4;
  const uint32_t tps = cols / (T * U);
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t c0 = (blockIdx.x - stripe * tps) * (T * U) + threadIdx.x;
  enc_unit<U, NTL, NTS, COPY>(a, stripe, c0, T);
}

// Persistent grid-stride over tiles.
template <int T, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(T) void k_persist(const Enc42 a) {
  const uint32_t cols = a.B >> 4;
  const uint32_t tps = cols / (T * U);
  const uint32_t ntiles = tps * a.nstripes;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t stripe = t / tps;
    const uint32_t c0 = (t - stripe * tps) * (T * U) + threadIdx.x;
    enc_unit<U, NTL, NTS, false>(a, stripe, c0, T);
  }
}

__global__ void k_fill(uint64_t *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

struct KVariant {
  std::string name;
  bool copy;
  std::function<void(hipStream_t)> run;
  std::vector<float> us;
};

int main(int argc, char **argv) {
  const uint32_t N = argc > 1 ? std::atoi(argv[1]) : 1024;
  const uint64_t B = 256 << 10;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  const int reps = 10;
  uint8_t *data, *par, *ref;
  CK(hipMalloc(&data, N * 4 * B));
  CK(hipMalloc(&par, N * 2 * B));
  CK(hipMalloc(&ref, N * 2 * B));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)data, N * 4 * B / 8);
  const std::vector<uint8_t> enc = enc_matrix(4, 6);
  Enc42 a{};
  a.data = data;
  a.parity = par;
  a.B = B;
  a.nstripes = N;
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 4; j++) a.t[i][j] = perm_tab(enc[(4 + i) * 4 + j]);
  // product kernel -> ref
  PermTab *dt;
  CK(hipMalloc(&dt, sizeof(a.t)));
  CK(hipMemcpy(dt, a.t, sizeof(a.t), hipMemcpyHostToDevice));
  ApplyArgs pa{};
  pa.k = 4;
  pa.r = 2;
  for (int j = 0; j < 4; j++) {
    pa.in[j] = data + j * B;
    pa.in_stride[j] = 4 * B;
  }
  for (int i = 0; i < 2; i++) {
    pa.out[i] = ref + i * B;
    pa.out_stride[i] = 2 * B;
  }
  pa.ptab = dt;
  pa.block = B;
  pa.nstripes = N;
  CK(dispatch_perm_k4(pa, 0));
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> href(N * 2 * B), hgot(N * 2 * B);
  CK(hipMemcpy(href.data(), ref, href.size(), hipMemcpyDeviceToHost));

  int cus = 256;
  std::vector<KVariant> vs;
  auto tiles = [&](int T, int U) { return (uint32_t)((B / 16) / (T * U) * N); };
  ApplyArgs pp = pa;
  pp.out[0] = par;
  pp.out[1] = par + B;
  vs.push_back({"product rs_apply_perm<4,2>", false, [&](hipStream_t s) { CK(dispatch_perm_k4(pp, s)); }, {}});
#define TILE(T, U, NL, NS)                                                           \
  vs.push_back({"tile T=" #T " U=" #U " ntL=" #NL " ntS=" #NS, false,               \
                [&](hipStream_t s) {                                                 \
                  hipLaunchKernelGGL((k_tile<T, U, NL, NS, false>), dim3(tiles(T, U)), \
                                     dim3(T), 0, s, a);                              \
                },                                                                   \
                {}});
  TILE(256, 2, false, false)
  TILE(256, 2, true, false)
  TILE(256, 2, false, true)
  TILE(256, 2, true, true)
  TILE(256, 4, true, true)
  TILE(256, 1, true, true)
  TILE(512, 2, true, true)
  TILE(512, 1, true, true)
  TILE(1024, 1, true, true)
  TILE(128, 2, true, true)
  TILE(64, 4, true, true)
#define PERS(T, U, NL, NS, G)                                                               \
  vs.push_back({"persist T=" #T " U=" #U " ntL=" #NL " ntS=" #NS " grid=" #G "xCU", false, \
                [&](hipStream_t s) {                                                        \
                  hipLaunchKernelGGL((k_persist<T, U, NL, NS>), dim3(G * cus), dim3(T), 0, \
                                     s, a);                                                 \
                },                                                                          \
                {}});
  PERS(256, 2, true, true, 8)
  PERS(256, 2, true, true, 16)
  PERS(256, 4, true, true, 8)
  vs.push_back({"COPY-shape (xor only) T=256 U=2", true, [&](hipStream_t s) {
                  hipLaunchKernelGGL((k_tile<256, 2, false, false, true>), dim3(tiles(256, 2)),
                                     dim3(256), 0, s, a);
                }, {}});
  vs.push_back({"COPY-shape (xor only) T=256 U=2 nt", true, [&](hipStream_t s) {
                  hipLaunchKernelGGL((k_tile<256, 2, true, true, true>), dim3(tiles(256, 2)),
                                     dim3(256), 0, s, a);
                }, {}});

  hipStream_t s;
  CK(hipStreamCreate(&s));
  // correctness
  for (auto &v : vs) {
    if (v.copy) continue;
    CK(hipMemset(par, 0, N * 2 * B));
    v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(hgot.data(), par, hgot.size(), hipMemcpyDeviceToHost));
    if (std::memcmp(hgot.data(), href.data(), href.size()) != 0) {
      std::printf("MISMATCH %s\n", v.name.c_str());
      return 2;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs) {
      v.run(s);  // warm
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; i++) v.run(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / reps);
    }
  const double bytes = (double)N * 6 * B;
  std::printf("RS(4,2) encode, %u x 1 MiB stripes, %.3f GB algorithmic per launch\n", N,
              bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2], mn = v.us[0];
    std::printf("%-46s median %8.1f us  min %8.1f us  %7.1f GB/s (%.1f%% of 8 TB/s)\n",
                v.name.c_str(), med, mn, bytes / med / 1e3, bytes / med / 1e3 / 80.0);
  }
  return 0;
}
