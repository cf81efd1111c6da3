// bsbench.hip -- bit-sliced encode (rs_bitslice.hpp) vs the product v_perm
// kernel (rs_device.hpp) on Storb's wide encode geometries:
//   RS(16,8)  storb (k=16, m=24): 8 MiB chunks, B = 512 KiB  (config 5 shape)
//   RS(32,16) storb (k=32, m=48): 32 MiB chunks, B = 1 MiB
//   RS(8,4)   storb (k=8,  m=12): 2-4 MiB chunks, B = 256 KiB
// Outputs are compared bit-exactly (bit-sliced vs v_perm); timings are
// interleaved rounds in one process.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../storb_amd/csrc \
//        bsbench.hip -o _build/bsbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "rs_bitslice.hpp"
#include "rs_device.hpp"

using namespace storb_rs;


#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e));                                      \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

using Fn = std::function<hipError_t(const ApplyArgs &, hipStream_t)>;
struct V {
  std::string name;
  Fn fn;
  std::vector<float> us;
};

template <int K, int N>
void run(const char *name, uint32_t nstripes, uint64_t B, int rounds, int tail) {
  constexpr int R = N - K;
  std::vector<V> vs;
  vs.push_back({"v_perm product", [](const ApplyArgs &a, hipStream_t s) {
                  return go_perm_r<(K > 32 ? 32 : K)>(a, s);
                }, {}});
  vs.push_back({"bitslice", [](const ApplyArgs &a, hipStream_t s) {
                  return bs::launch_bitslice<K, N>(a, s);
                }, {}});
  for (int cap : {0, 2, 4, 6})  // resident-workgroup caps (rs_kernels.hpp wg_cap)
    vs.push_back({"bitslice wg/CU<=" + std::to_string(cap),
                  [cap](const ApplyArgs &a, hipStream_t s) {
                    const uint64_t blocks = ((a.block / 16 + 511) / 512) * a.nstripes;
                    return launch_lds<bs::rs_encode_bitslice<K, N>>(blocks, 256, cap_lds(cap, 0),
                                                                   s, a);
                  }, {}});
  B -= tail;  // ragged share size: exercises the guarded tail
  const uint64_t in_bytes = (uint64_t)nstripes * K * B, out_bytes = (uint64_t)nstripes * R * B;
  uint8_t *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, K);
  const std::vector<uint8_t> enc = enc_matrix(K, N);
  std::vector<PermTab> tabs;
  const uint32_t rp = rows_bucket(R);
  for (int j = 0; j < K; j++)
    for (uint32_t i = 0; i < rp; i++)
      tabs.push_back(i < (uint32_t)R ? perm_tab(enc[(K + i) * K + j]) : PermTab{});
  PermTab *dt;
  CK(hipMalloc(&dt, tabs.size() * sizeof(PermTab)));
  CK(hipMemcpy(dt, tabs.data(), tabs.size() * sizeof(PermTab), hipMemcpyHostToDevice));
  ApplyArgs a{};
  a.k = K;
  a.r = R;
  for (int j = 0; j < K; j++) {
    a.in[j] = in + j * B;
    a.in_stride[j] = K * B;
  }
  for (int i = 0; i < R; i++) {
    a.out[i] = out + i * B;
    a.out_stride[i] = R * B;
  }
  a.ptab = dt;
  a.tab_rows = rp;
  a.block = B;
  a.nstripes = nstripes;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<uint8_t> ref(out_bytes), got(out_bytes);
  for (size_t vi = 0; vi < vs.size(); vi++) {
    CK(hipMemset(out, 0xA5, out_bytes));
    CK(vs[vi].fn(a, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? got.data() : ref.data(), out, out_bytes, hipMemcpyDeviceToHost));
    if (vi && std::memcmp(got.data(), ref.data(), out_bytes)) {
      size_t first = 0;
      while (got[first] == ref[first]) first++;
      std::printf("MISMATCH %s %s at byte %zu (%02x vs %02x)\n", name, vs[vi].name.c_str(),
                  first, got[first], ref[first]);
      std::exit(2);
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 8;
  for (int rd = 0; rd < rounds; rd++)
    for (auto &v : vs) {
      CK(v.fn(a, s));
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; i++) CK(v.fn(a, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / reps);
    }
  const double bytes = (double)in_bytes + out_bytes;
  std::printf("%s (B=%llu): %.3f GB algorithmic per launch, bit-exact\n", name,
              (unsigned long long)B, bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    std::printf("  %-16s median %8.1f us  min %8.1f us  %7.1f GB/s  %.1f%% of 8 TB/s\n",
                v.name.c_str(), med, v.us[0], bytes / med / 1e3, bytes / med / 1e3 / 80.0);
  }
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipFree(dt));
  CK(hipStreamDestroy(s));
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  run<16, 24>("RS(16,8) encode 128 x 8 MiB", 128, 512 << 10, rounds, 0);
  run<32, 48>("RS(32,16) encode 32 x 32 MiB", 32, 1 << 20, rounds, 0);
  run<8, 12>("RS(8,4) encode 512 x 2 MiB", 512, 256 << 10, rounds, 0);
  run<16, 24>("RS(16,8) ragged", 7, 40000, 2, 16);
  return 0;
}
