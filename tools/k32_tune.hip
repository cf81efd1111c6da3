// k32_tune.hip -- launch shape of the table kernel rs_apply_perm at k = 32.
//
// The (T, U, G, TL, PAIR, cap) choices of rs_device.hpp Tune were swept in
// round 1 on k <= 16 shapes only (DESIGN.md "Tuning"); k = 32 inherits
// U = 1, G = 8, TL, uncapped. Here: config 6's geometry (32 chunks x 32 MiB,
// k = 32, B = 1 MiB) decoded with R = 1, 2, 4 rows through several shapes,
// every output compared bit-exactly with the product shape's, timings in
// interleaved rounds (median of reps, HIP events on one stream).
// Bytes = nstripes x (k + R) x B.
//
// build: make -C tools k32_tune
// usage: k32_tune [REPS] [ALL]: R = 3, 5, 6, 8, 16 (round 4); ALL = 1 adds R = 1, 2, 4
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "rs_device.hpp"

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

struct Var {
  std::string name;
  std::function<hipError_t(const ApplyArgs &, hipStream_t)> fn;
  std::vector<float> ms;
};

template <int R>
std::vector<Var> variants() {
  std::vector<Var> v;
  if constexpr (R > 4 || R == 3) {  // the round-4 sweep of the remaining row buckets
    v.push_back({"r3 product U1 G8 TL", [](const ApplyArgs &a, hipStream_t s) {
                   return launch_perm<32, R, 256, 1, false, 8, true>(a, s, 0);
                 }});
    v.push_back({"U1 G4 TL", [](const ApplyArgs &a, hipStream_t s) {
                   return launch_perm<32, R, 256, 1, false, 4, true>(a, s, 0);
                 }});
    v.push_back({"U1 G2 TL", [](const ApplyArgs &a, hipStream_t s) {
                   return launch_perm<32, R, 256, 1, false, 2, true>(a, s, 0);
                 }});
    v.push_back({"U1 G16 TL", [](const ApplyArgs &a, hipStream_t s) {
                   return launch_perm<32, R, 256, 1, false, 16, true>(a, s, 0);
                 }});
    v.push_back({"U1 G4 TL cap4", [](const ApplyArgs &a, hipStream_t s) {
                   return launch_perm<32, R, 256, 1, false, 4, true>(a, s, 4);
                 }});
    return v;
  }
  v.push_back({"product U1 G8 TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 1, false, 8, true>(a, s, Tune<32, R>::OCC);
               }});
  v.push_back({"U1 G8 TL cap4", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 1, false, 8, true>(a, s, 4);
               }});
  v.push_back({"U1 G4 TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 1, false, 4, true>(a, s, 0);
               }});
  v.push_back({"U1 G16 TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 1, false, 16, true>(a, s, 0);
               }});
  v.push_back({"U1 G8 TL PAIR", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 1, false, 8, true, true>(a, s, 0);
               }});
  v.push_back({"U2 G4 TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 2, false, 4, true>(a, s, 0);
               }});
  v.push_back({"U2 G8 TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 2, false, 8, true>(a, s, 0);
               }});
  v.push_back({"T512 U1 G8 TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 512, 1, false, 8, true>(a, s, 0);
               }});
  v.push_back({"U1 G8 BAR TL", [](const ApplyArgs &a, hipStream_t s) {
                 return launch_perm<32, R, 256, 1, true, 8, true>(a, s, 0);
               }});
  return v;
}

template <int R>
int run(int reps, uint8_t *d, uint8_t *p, uint8_t *o, PermTab *dt, uint32_t N, size_t B) {
  constexpr uint32_t k = 32;
  std::mt19937 rng(R * 7 + 1);
  std::vector<PermTab> tabs(k * R);
  for (auto &t : tabs) t = perm_tab(static_cast<uint8_t>(rng() | 1));
  CK(hipMemcpy(dt, tabs.data(), tabs.size() * sizeof(PermTab), hipMemcpyHostToDevice));
  ApplyArgs a{};
  // survivors: data shares R.. of each chunk, then the first R parity shares
  for (uint32_t j = 0; j < k; j++) {
    const uint32_t id = j + R;
    a.in[j] = id < k ? d + id * B : p + (id - k) * B;
    a.in_stride[j] = id < k ? k * B : 16 * B;
  }
  for (uint32_t i = 0; i < R; i++) {
    a.out[i] = o + i * B;
    a.out_stride[i] = R * B;
  }
  a.ptab = dt;
  a.k = k;
  a.r = R;
  a.tab_rows = R;
  a.block = B;
  a.nstripes = N;
  auto vs = variants<R>();
  const size_t ob = size_t(N) * R * B;
  std::vector<uint8_t> want(ob), got(ob);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t vi = 0; vi < vs.size(); vi++) {
    CK(hipMemsetAsync(o, 0xEE, ob, s));
    CK(vs[vi].fn(a, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? got.data() : want.data(), o, ob, hipMemcpyDeviceToHost));
    if (vi && std::memcmp(want.data(), got.data(), ob) != 0) {
      std::printf("R=%d %s: MISMATCH\n", R, vs[vi].name.c_str());
      return 1;
    }
  }
  for (int r = 0; r < reps; r++)
    for (auto &v : vs) {
      CK(hipEventRecord(e0, s));
      CK(v.fn(a, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float x = 0;
      CK(hipEventElapsedTime(&x, e0, e1));
      v.ms.push_back(x);
    }
  const double bytes = double(N) * (k + R) * B;
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float m = v.ms[v.ms.size() / 2];
    std::printf("R=%d %-20s %8.4f ms  %6.2f TB/s  %5.1f %%  (bit-exact)\n", R, v.name.c_str(), m,
                bytes / (m * 1e-3) / 1e12, 100.0 * bytes / (m * 1e-3) / 8e12);
  }
  CK(hipStreamDestroy(s));
  return 0;
}

__global__ void fill(uint64_t *q, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
       i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    q[i] = z ^ (z >> 31);
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const uint32_t N = 32, k = 32;
  const size_t B = 1u << 20;
  uint8_t *d, *p, *o;
  PermTab *dt;
  CK(hipMalloc(&d, N * k * B));
  CK(hipMalloc(&p, N * 16 * B));
  CK(hipMalloc(&o, N * 16 * B));
  CK(hipMalloc(&dt, k * 16 * sizeof(PermTab)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(d),
                     N * k * B / 8, 11);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(p),
                     N * 16 * B / 8, 12);
  CK(hipDeviceSynchronize());
  const bool all = argc > 2 && std::atoi(argv[2]) == 1;  // 1: R = 1, 2, 4 too (round 3's sweep)
  if (all && (run<1>(reps, d, p, o, dt, N, B) || run<2>(reps, d, p, o, dt, N, B) ||
              run<4>(reps, d, p, o, dt, N, B)))
    return 1;
  if (run<3>(reps, d, p, o, dt, N, B) || run<5>(reps, d, p, o, dt, N, B) ||
      run<6>(reps, d, p, o, dt, N, B) || run<8>(reps, d, p, o, dt, N, B) ||
      run<16>(reps, d, p, o, dt, N, B))
    return 1;
  return 0;
}
