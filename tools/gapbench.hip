// gapbench.hip -- what the launch boundary costs between back-to-back
// RS(4,2) launches (the default bench step is two of them: encode, then the
// decode of shares {0, 1} from {2..5}), and whether the size of the kernel
// argument block matters. ApplyArgs carries 64 input, 32 output and 64 copy
// slots (~2.6 KB of kernel arguments); SmallArgs the 4 + 2 a (4, 6) launch
// uses (~120 B). Same tile (perm_tile), same tables, outputs compared.
// Per variant: L back-to-back launches on one stream between two events;
// per-launch time = total / L, against the same launch timed alone.
//
// build: make -C tools gapbench
// usage: gapbench [L] [REPS]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
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

struct SmallArgs {
  const uint8_t *in[4];
  uint64_t in_stride[4];
  uint8_t *out[2];
  uint64_t out_stride[2];
  const PermTab *ptab;
  uint64_t block;
  uint32_t k, r, nstripes, pad;
};

struct SmallView {
  const SmallArgs &a;
  uint32_t stripe;
  __device__ __forceinline__ const u32x4 *in(int j) const {
    return reinterpret_cast<const u32x4 *>(a.in[j] + static_cast<uint64_t>(stripe) * a.in_stride[j]);
  }
  __device__ __forceinline__ u32x4 *out(int i) const {
    return reinterpret_cast<u32x4 *>(a.out[i] + static_cast<uint64_t>(stripe) * a.out_stride[i]);
  }
  __device__ __forceinline__ bool has_copy(int) const { return false; }
  __device__ __forceinline__ u32x4 *copy(int) const { return nullptr; }
  __device__ __forceinline__ bool accumulate() const { return false; }
};

// Output shares written through buffer stores with an explicit cache policy
// (aux: 16 = sc1, write-through: the line leaves the XCD's L2 at once, so
// the kernel-end release has no dirty lines to write back; 18 = sc1 nt;
// MI355X_MICROARCH.md "stores of each flavour": plain / nt keep the line in
// L2). perm_tile stores through st_stream(q + c, x): q is a BufOut here.
template <int AUX>
struct BufRef {
  __amdgpu_buffer_rsrc_t r;
  int off;
};
template <int AUX>
struct BufOut {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ BufRef<AUX> operator+(uint32_t c) const {
    return {r, static_cast<int>(c * 16u)};
  }
  __device__ __forceinline__ u32x4 operator[](uint32_t c) const {
    return __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(c * 16u), 0, 0);
  }
};
// found by argument-dependent lookup from perm_tile's st_stream(q + c, x)
template <int AUX>
__device__ __forceinline__ void st_stream(BufRef<AUX> p, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, p.r, p.off, 0, AUX);
}

template <int AUX>
struct SmallViewSt {
  const SmallArgs &a;
  uint32_t stripe;
  __device__ __forceinline__ const u32x4 *in(int j) const {
    return reinterpret_cast<const u32x4 *>(a.in[j] + static_cast<uint64_t>(stripe) * a.in_stride[j]);
  }
  __device__ __forceinline__ BufOut<AUX> out(int i) const {
    uint8_t *p = a.out[i] + static_cast<uint64_t>(stripe) * a.out_stride[i];
    return {__builtin_amdgcn_make_buffer_rsrc(p, 0, static_cast<int>(a.block), 0x00020000)};
  }
  __device__ __forceinline__ bool has_copy(int) const { return false; }
  __device__ __forceinline__ u32x4 *copy(int) const { return nullptr; }
  __device__ __forceinline__ bool accumulate() const { return false; }
};

template <int AUX>
__global__ __launch_bounds__(256) void rs_small42_st(const SmallArgs a) {
  constexpr uint32_t TILE = 256;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t base = (blockIdx.x - stripe * tps) * TILE;
  const SmallViewSt<AUX> v{a, stripe};
  if (base + TILE <= cols)
    perm_tile<4, 2, 256, 1, false, 4, false, false>(v, a.ptab, a.k, a.r, cols, base + threadIdx.x);
  else
    perm_tile<4, 2, 256, 1, false, 4, false, true>(v, a.ptab, a.k, a.r, cols, base + threadIdx.x);
}

__global__ __launch_bounds__(256) void rs_small42(const SmallArgs a) {
  constexpr uint32_t TILE = 256;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t stripe = blockIdx.x / tps;
  const uint32_t base = (blockIdx.x - stripe * tps) * TILE;
  const SmallView v{a, stripe};
  if (base + TILE <= cols)
    perm_tile<4, 2, 256, 1, false, 4, false, false>(v, a.ptab, a.k, a.r, cols, base + threadIdx.x);
  else
    perm_tile<4, 2, 256, 1, false, 4, false, true>(v, a.ptab, a.k, a.r, cols, base + threadIdx.x);
}

int main(int argc, char **argv) {
  const int L = argc > 1 ? std::atoi(argv[1]) : 40;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  const uint32_t N = 1024, k = 4, n = 6;
  const size_t B = 256u << 10;
  uint8_t *d, *p;
  CK(hipMalloc(&d, size_t(N) * k * B));
  CK(hipMalloc(&p, size_t(N) * (n - k) * B));
  CK(hipMemset(d, 0x5C, size_t(N) * k * B));
  std::vector<PermTab> tabs(k * 2);
  for (uint32_t j = 0; j < k; j++)
    for (uint32_t i = 0; i < 2; i++) tabs[j * 2 + i] = perm_tab(static_cast<uint8_t>(3 + 7 * j + 11 * i));
  PermTab *dt;
  CK(hipMalloc(&dt, tabs.size() * sizeof(PermTab)));
  CK(hipMemcpy(dt, tabs.data(), tabs.size() * sizeof(PermTab), hipMemcpyHostToDevice));
  ApplyArgs a{};
  SmallArgs sa{};
  for (uint32_t j = 0; j < k; j++) {
    a.in[j] = sa.in[j] = d + j * B;
    a.in_stride[j] = sa.in_stride[j] = k * B;
  }
  for (uint32_t i = 0; i < 2; i++) {
    a.out[i] = sa.out[i] = p + i * B;
    a.out_stride[i] = sa.out_stride[i] = (n - k) * B;
  }
  a.ptab = sa.ptab = dt;
  a.k = sa.k = k;
  a.r = sa.r = 2;
  a.tab_rows = 2;
  a.block = sa.block = B;
  a.nstripes = sa.nstripes = N;
  const uint64_t blocks = uint64_t(N) * (B / 16 / 256);
  using C = Tune<4, 2>;
  const size_t dyn = cap_lds(C::OCC, 0);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct V {
    const char *name;
    std::function<hipError_t()> go;
    std::vector<float> one, many;
  };
  std::vector<V> vs = {
      {"ApplyArgs (product kernel, 2.6 KB args)",
       [&] { return launch_perm<4, 2, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>(a, s, C::OCC); }, {}, {}},
      {"SmallArgs (same tile, ~120 B args)",
       [&] { return launch_lds<rs_small42>(blocks, 256, dyn, s, sa); }, {}, {}},
      {"SmallArgs, buffer stores sc1 (write-through)",
       [&] { return launch_lds<rs_small42_st<16>>(blocks, 256, dyn, s, sa); }, {}, {}},
      {"SmallArgs, buffer stores sc1 nt",
       [&] { return launch_lds<rs_small42_st<18>>(blocks, 256, dyn, s, sa); }, {}, {}},
      {"SmallArgs, buffer stores nt",
       [&] { return launch_lds<rs_small42_st<2>>(blocks, 256, dyn, s, sa); }, {}, {}},
      {"SmallArgs, buffer stores sc0 sc1",
       [&] { return launch_lds<rs_small42_st<17>>(blocks, 256, dyn, s, sa); }, {}, {}},
  };
  // same bytes out
  std::vector<uint8_t> w(size_t(N) * (n - k) * B), g(w.size());
  for (size_t vi = 0; vi < vs.size(); vi++) {
    CK(hipMemsetAsync(p, 0, w.size(), s));
    CK(vs[vi].go());
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? g.data() : w.data(), p, w.size(), hipMemcpyDeviceToHost));
    if (vi && std::memcmp(w.data(), g.data(), w.size())) {
      std::printf("%s: MISMATCH\n", vs[vi].name);
      return 1;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < reps; r++)
    for (auto &v : vs) {
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      CK(v.go());
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float x;
      CK(hipEventElapsedTime(&x, e0, e1));
      v.one.push_back(x);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < L; i++) CK(v.go());
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&x, e0, e1));
      v.many.push_back(x / L);
    }
  const double bytes = double(N) * n * B;
  for (auto &v : vs) {
    std::sort(v.one.begin(), v.one.end());
    std::sort(v.many.begin(), v.many.end());
    const float o = v.one[v.one.size() / 2], m = v.many[v.many.size() / 2];
    std::printf("%-42s alone %.4f ms  back-to-back %.4f ms/launch (%.2f TB/s, %.1f %%)  "
                "boundary %+.1f us\n",
                v.name, o, m, bytes / (m * 1e-3) / 1e12, 100 * bytes / (m * 1e-3) / 8e12,
                (m - o) * 1e3);
  }
  return 0;
}
