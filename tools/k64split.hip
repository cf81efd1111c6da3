// k64split.hip -- Storb's k = 64 encode (32 parity rows): the product's two
// 16-row launches (rs_jit.cpp row blocks, each reading and bit-slicing all 64
// inputs) against ONE row-split launch (rs_bitslice_core.h bs_split_body: the
// two waves of a 128-lane workgroup share each input's bit-planes through
// LDS and fold 16 rows each), over load-group size G and the
// resident-workgroup cap. Also RS(32,16)-like 20- and 24-row decodes at k = 64
// (split vs two blocks). Every variant is compared bit-exactly with the
// two-launch form.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../storb_amd/csrc \
//        -fconstexpr-steps=100000000 k64split.hip -o _build/k64split
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

using Enc = EncMat<64, 96>;
using Lo = RowSlice<Enc, 0, 16>;
using Hi = RowSlice<Enc, 16, 32>;
constexpr int G16 = bs_group(64, 16);
constexpr int T = 128;

template <class M>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2))) void k_single(
    const ApplyArgs a) {
  bs_kernel_body<M, G16, T, 0>(a);
}

template <class M, int G>
__global__ __launch_bounds__(kSplitThreads) __attribute__((amdgpu_waves_per_eu(2))) void k_split(
    const ApplyArgs a) {
  bs_split_body<M, G, 0>(a);
}

template <auto Kern, typename... Args>
hipError_t launch(uint64_t blocks, int cap, size_t static_lds, hipStream_t s, Args... args) {
  const size_t dyn = cap_lds(cap, static_lds);
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
  const uint64_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (2u << 20);
  const uint32_t ns = argc > 3 ? std::atoi(argv[3]) : 8, K = 64, R = 32;
  const uint64_t in_bytes = (uint64_t)ns * K * B, out_bytes = (uint64_t)ns * R * B;
  uint8_t *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, 64);
  ApplyArgs a{};
  a.k = K;
  a.r = 32;
  for (uint32_t j = 0; j < K; j++) {
    a.in[j] = in + j * B;
    a.in_stride[j] = K * B;
  }
  for (int i = 0; i < 32; i++) {
    a.out[i] = out + i * B;
    a.out_stride[i] = R * B;
  }
  a.block = B;
  a.nstripes = ns;
  ApplyArgs alo = a, ahi = a;
  alo.r = ahi.r = 16;
  for (int i = 0; i < 16; i++) {
    ahi.out[i] = a.out[16 + i];
    ahi.out_stride[i] = a.out_stride[16 + i];
  }
  const uint64_t cols = B / 16;
  const uint64_t tiles1 = ((cols + bs_cols_per_tile(T) - 1) / bs_cols_per_tile(T)) * ns;
  const uint64_t tiles2 = ((cols + kSplitColsPerTile - 1) / kSplitColsPerTile) * ns;
  std::vector<V> vs;
  for (int cap : {3, 4}) {
    vs.push_back({"two launches cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK(launch<k_single<Lo>>(tiles1, cap, 0, s, alo));
                    CK(launch<k_single<Hi>>(tiles1, cap, 0, s, ahi));
                  }, {}});
  }
  for (int cap : {2, 3, 4, 0}) {
    vs.push_back({"split G=2 cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK((launch<k_split<Enc, 2>>(tiles2, cap, sizeof(SplitLds<2>), s, a)));
                  }, {}});
    vs.push_back({"split G=4 cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK((launch<k_split<Enc, 4>>(tiles2, cap, sizeof(SplitLds<4>), s, a)));
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
  std::printf("k=64 encode (32 rows), %u x %llu-B shares: %.3f GB algorithmic, bit-exact\n", ns,
              (unsigned long long)B, bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    std::printf("  %-26s %8.1f us  %7.1f GB/s  %.1f%% of 8 TB/s\n", v.name.c_str(), med,
                bytes / med / 1e3, bytes / med / 1e3 / 80.0);
  }
  return 0;
}
