// k64pair.hip -- Storb's k = 64 encode (32 parity rows) as two 16-row
// bit-sliced blocks: two launches (the product, rs_jit.cpp row blocks) that
// each read all 64 inputs, against ONE launch whose workgroups come in pairs
// (same tile, rows 0-15 / 16-31) placed so the second of a pair can re-read
// the tile from cache instead of HBM:
//   xcd   the pair on the same XCD (workgroup b runs on XCD b % 8), so the
//         second hits that XCD's L2;
//   adj   the pair on neighbouring workgroups (different XCDs; the shared
//         Infinity Cache only).
// Built twice: -DSTORB_BS_LOAD_NT=1 (the product's non-temporal loads) and
// =0 (default-policy loads, which may allocate where nt ones do not).
// Every variant is compared bit-exactly with the two-launch product form.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../storb_amd/csrc \
//        -DSTORB_BS_LOAD_NT=1 k64pair.hip -o _build/k64pair_nt
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "rs_bitslice.hpp"

using namespace storb_rs;
using namespace storb_rs::bs;

int storb_rs::wg_cap_override() { return -1; }
int storb_rs::table_threads_override() { return 0; }

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e));                                      \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

template <class M, int R0, int R1>
struct RowSlice {
  static constexpr int K = M::K, R = R1 - R0;
  static constexpr unsigned long long copy_mask = 0;
  struct Net {
    uint8_t row[R][K][8];
  };
  static constexpr Net make() {
    Net n{};
    for (int p = 0; p < R; p++)
      for (int j = 0; j < K; j++)
        for (int b = 0; b < 8; b++) n.row[p][j][b] = M::net.row[R0 + p][j][b];
    return n;
  }
  static constexpr Net net = make();
};

using Enc = EncMat<64, 96>;
using Lo = RowSlice<Enc, 0, 16>;
using Hi = RowSlice<Enc, 16, 32>;
constexpr int G = bs_group(64, 16);
constexpr int T = 128;

struct OutB {
  uint8_t *out[16];
  uint64_t out_stride[16];
};

template <class M>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2))) void k_single(
    const ApplyArgs a) {
  bs_kernel_body<M, G, T, 0>(a);
}

// MODE 0: pair on one XCD; 1: neighbouring workgroups.
template <int MODE>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2))) void k_pair(
    const ApplyArgs a, const OutB b) {
  constexpr uint32_t CPT = bs_cols_per_tile(T);
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + CPT - 1) / CPT;
  const uint32_t nt = tps * a.nstripes;
  uint32_t t, half;
  if (MODE == 0) {
    const uint32_t x = blockIdx.x % 8, slot = blockIdx.x / 8;
    half = slot & 1;
    t = (slot >> 1) * 8 + x;
  } else {
    half = blockIdx.x & 1;
    t = blockIdx.x >> 1;
  }
  if (t >= nt) return;
  const uint32_t stripe = t / tps, tile = t - stripe * tps;
  const uint32_t v0 = tile * CPT + (threadIdx.x >> 6) * 128 + (threadIdx.x & 63);
  if (half == 0)
    bs_tile_to<Lo, G>(a, a.out, a.out_stride, stripe, v0, cols);
  else
    bs_tile_to<Hi, G>(a, b.out, b.out_stride, stripe, v0, cols);
}

template <auto Kern, typename... Args>
hipError_t launch(uint64_t blocks, int cap, hipStream_t s, Args... args) {
  const size_t dyn = cap_lds(cap, 0);
  if (dyn > (64u << 10))
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(Kern),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)));
  hipLaunchKernelGGL(Kern, dim3(blocks), dim3(T), dyn, s, args...);
  return hipGetLastError();
}

__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

struct V {
  std::string name;
  std::function<void(hipStream_t)> fn;
  std::vector<float> us;
};

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  const uint32_t ns = 8, K = 64, R = 32;
  const uint64_t B = 2 << 20;
  const uint64_t in_bytes = (uint64_t)ns * K * B, out_bytes = (uint64_t)ns * R * B;
  uint8_t *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, 64);
  ApplyArgs a{};
  a.k = K;
  a.r = 16;
  for (uint32_t j = 0; j < K; j++) {
    a.in[j] = in + j * B;
    a.in_stride[j] = K * B;
  }
  OutB b{};
  for (int i = 0; i < 16; i++) {
    a.out[i] = out + i * B;
    a.out_stride[i] = R * B;
    b.out[i] = out + (16 + i) * B;
    b.out_stride[i] = R * B;
  }
  a.block = B;
  a.nstripes = ns;
  ApplyArgs ahi = a;
  for (int i = 0; i < 16; i++) {
    ahi.out[i] = b.out[i];
    ahi.out_stride[i] = b.out_stride[i];
  }
  const uint64_t tiles = (B / 16 / bs_cols_per_tile(T)) * ns;
  std::vector<V> vs;
  for (int cap : {3, 4}) {
    vs.push_back({"two launches cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK(launch<k_single<Lo>>(tiles, cap, s, a));
                    CK(launch<k_single<Hi>>(tiles, cap, s, ahi));
                  }, {}});
    vs.push_back({"pair same-XCD cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK(launch<k_pair<0>>((2 * tiles + 15) / 16 * 16, cap, s, a, b));
                  }, {}});
    vs.push_back({"pair neighbours cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK(launch<k_pair<1>>(2 * tiles, cap, s, a, b));
                  }, {}});
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<uint8_t> ref(out_bytes), got(out_bytes);
  for (size_t vi = 0; vi < vs.size(); vi++) {
    CK(hipMemset(out, 0xA5, out_bytes));
    vs[vi].fn(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? got.data() : ref.data(), out, out_bytes, hipMemcpyDeviceToHost));
    if (vi && std::memcmp(got.data(), ref.data(), out_bytes)) {
      std::printf("MISMATCH %s\n", vs[vi].name.c_str());
      return 2;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs) {
      v.fn(s);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < 4; i++) v.fn(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / 4);
    }
  const double bytes = (double)in_bytes + out_bytes;
  std::printf("k=64 encode, 8 x 128 MiB chunks (loads nt=%d): %.3f GB algorithmic, bit-exact\n",
              STORB_BS_LOAD_NT, bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    std::printf("  %-26s %8.1f us  %7.1f GB/s  %.1f%% of 8 TB/s\n", v.name.c_str(), med,
                bytes / med / 1e3, bytes / med / 1e3 / 80.0);
  }
  return 0;
}
