// k64split.hip -- the row-split bit-sliced kernel (rs_bitslice_core.h
// bs_split_body: the two waves of a 128-lane workgroup share each input's
// bit-planes through LDS and fold half the rows each) over load-group size G
// and the resident-workgroup cap, against:
//   RS(64,32) encode: the two 16-row launches the product ran before (each
//     reading and bit-slicing all 64 inputs);
//   RS(32,16) / RS(16,8) encode: the product's one-wave-per-tile kernel (is
//     splitting 16 or 8 rows over two waves worth its extra table work?).
// Every variant is compared bit-exactly with the first of its geometry.
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

template <class M, int G, int T, int SWZ>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2))) void k_single(
    const ApplyArgs a) {
  bs_kernel_body<M, G, T, SWZ>(a);
}

template <class M, int G, bool TAB = false>
__global__ __launch_bounds__(kSplitThreads) __attribute__((amdgpu_waves_per_eu(2))) void k_split(
    const ApplyArgs a) {
  bs_split_body<M, G, 0, TAB>(a);
}

template <auto Kern, typename... Args>
hipError_t launch(uint64_t blocks, int threads, int cap, size_t static_lds, hipStream_t s,
                  Args... args) {
  const size_t dyn = cap_lds(cap, static_lds);
  if (dyn > (64u << 10))
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(Kern),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)));
  hipLaunchKernelGGL(Kern, dim3(blocks), dim3(threads), dyn, s, args...);
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

// Storb-sized batch of 1 GiB of data: (k, n) shares of B bytes, ns stripes.
template <int K, int N>
int run(int rounds, uint64_t B, uint32_t ns) {
  constexpr int R = N - K;
  using Enc = EncMat<K, N>;
  const uint64_t in_bytes = (uint64_t)ns * K * B, out_bytes = (uint64_t)ns * R * B;
  uint8_t *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, 64);
  ApplyArgs a{};
  a.k = K;
  a.r = R;
  for (uint32_t j = 0; j < K; j++) {
    a.in[j] = in + j * B;
    a.in_stride[j] = K * B;
  }
  for (int i = 0; i < R; i++) {
    a.out[i] = out + i * B;
    a.out_stride[i] = R * B;
  }
  a.block = B;
  a.nstripes = ns;
  const uint64_t cols = B / 16;
  const uint64_t tiles2 = ((cols + kSplitColsPerTile - 1) / kSplitColsPerTile) * ns;
  std::vector<V> vs;
  if constexpr (R > 16) {
    // the product before the row split: two 16-row launches
    using Lo = RowSlice<Enc, 0, R / 2>;
    using Hi = RowSlice<Enc, R / 2, R>;
    constexpr BsShape S = bs_shape(K, R / 2);
    constexpr int G = bs_group(K, R / 2);
    ApplyArgs alo = a, ahi = a;
    alo.r = ahi.r = R / 2;
    for (int i = 0; i < R / 2; i++) {
      ahi.out[i] = a.out[R / 2 + i];
      ahi.out_stride[i] = a.out_stride[R / 2 + i];
    }
    const uint64_t tiles1 = ((cols + bs_cols_per_tile(S.threads) - 1) / bs_cols_per_tile(S.threads)) * ns;
    vs.push_back({"two launches (old product)", [=](hipStream_t s) {
                    CK((launch<k_single<Lo, G, S.threads, S.swz>>(tiles1, S.threads, S.cap, 0, s, alo)));
                    CK((launch<k_single<Hi, G, S.threads, S.swz>>(tiles1, S.threads, S.cap, 0, s, ahi)));
                  }, {}});
  } else {
    // the product: one launch, every row in one wave
    constexpr BsShape S = bs_shape(K, R);
    constexpr int G = bs_group(K, R);
    const uint64_t tiles1 = ((cols + bs_cols_per_tile(S.threads) - 1) / bs_cols_per_tile(S.threads)) * ns;
    vs.push_back({"one wave per tile (product)", [=](hipStream_t s) {
                    CK((launch<k_single<Enc, G, S.threads, S.swz>>(tiles1, S.threads, S.cap, 0, s, a)));
                  }, {}});
  }
  for (int cap : {4, 0}) {
    vs.push_back({"split G=2 cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK((launch<k_split<Enc, 2>>(tiles2, kSplitThreads, cap, sizeof(SplitLds<2>), s, a)));
                  }, {}});
    vs.push_back({"split-tables G=2 cap=" + std::to_string(cap), [=](hipStream_t s) {
                    CK((launch<k_split<Enc, 2, true>>(tiles2, kSplitThreads, cap,
                                                      sizeof(SplitTabLds<2>), s, a)));
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
  std::printf("RS(%d,%d) encode (%d rows), %u x %llu-B shares: %.3f GB algorithmic, bit-exact\n",
              K, R, R, ns, (unsigned long long)B, bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    std::printf("  %-26s %8.1f us  %7.1f GB/s  %.1f%% of 8 TB/s\n", v.name.c_str(), med,
                bytes / med / 1e3, bytes / med / 1e3 / 80.0);
  }
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipStreamDestroy(s));
  return 0;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;  // argv[2]: also k = 32 / 16
  // 1 GiB of data per geometry: Storb's 8 / 32 / 128 MiB chunks
  int rc = run<64, 96>(rounds, 2u << 20, 8);
  if (!rc && argc > 2) rc = run<32, 48>(rounds, 1u << 20, 32);
  if (!rc && argc > 2) rc = run<16, 24>(rounds, 512u << 10, 128);
  return rc;
}
