// bstune.hip -- launch-shape sweep of the bit-sliced core (rs_bitslice_core.h)
// that both the ahead-of-time encoders and the run-time-compiled decode
// kernels use: load-group size G (shares in flight per double-buffer half)
// x resident-workgroup cap (LDS reservation, rs_kernels.hpp cap_lds), on the
// wide geometries RS(16,8) (8 MiB chunks) and RS(32,16) (32 MiB chunks).
// Every variant's output is compared bit-exactly with the product kernel's;
// timings are interleaved rounds in one process (median of rounds).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../storb_amd/csrc \
//        bstune.hip -o _build/bstune
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

template <int K, int N, int G, int T, int SWZ>
__global__ __launch_bounds__(T) void k_bs(const ApplyArgs a) {
  bs::bs_kernel_body<bs::EncMat<K, N>, G, T, SWZ>(a);
}

template <int K, int N, int C, int W, int G, int SWZ>
__global__ __launch_bounds__(64 * C * W) void k_ks(const ApplyArgs a) {
  bs::bs_ksplit_body<bs::EncMat<K, N>, C, W, G, SWZ>(a);
}

// The access structure with (almost) no GF work: row 0 = XOR of the
// bit-sliced inputs (transposes kept), rows 1.. zero (stored). What a launch
// shape streams at when the folds cost nothing (BSTUNE_NOGF).
template <int K_, int N_>
struct ZeroMat {
  static constexpr int K = K_, R = N_ - K_;
  static constexpr unsigned long long copy_mask = 0;
  struct Net {
    unsigned char row[R][K][8];
  };
  static constexpr Net make() {
    Net n{};
    for (int j = 0; j < K; j++)
      for (int b = 0; b < 8; b++) n.row[0][j][b] = static_cast<unsigned char>(1u << b);
    return n;
  }
  static constexpr Net net = make();
};

template <int K, int N, int G, int T, int SWZ>
__global__ __launch_bounds__(T) void k_bs0(const ApplyArgs a) {
  bs::bs_kernel_body<ZeroMat<K, N>, G, T, SWZ>(a);
}

template <int K, int N, int C, int W, int G, int SWZ>
__global__ __launch_bounds__(64 * C * W) void k_ks0(const ApplyArgs a) {
  bs::bs_ksplit_body<ZeroMat<K, N>, C, W, G, SWZ>(a);
}

// 16 B per lane, every input loaded up front (the round-2 probe shape).
template <int K, int R, int T>
__global__ __launch_bounds__(T) void k_flat(const ApplyArgs a) {
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4), tps = cols / T;
  const uint32_t stripe = blockIdx.x / tps, t = blockIdx.x - stripe * tps;
  const uint32_t c = t * T + threadIdx.x;
  bs::v4 v[K];
#pragma unroll
  for (int j = 0; j < K; j++)
    v[j] = bs::ld_nt(reinterpret_cast<const bs::v4 *>(a.in[j] + (uint64_t)stripe * a.in_stride[j]) + c);
  bs::v4 acc = v[0];
#pragma unroll
  for (int j = 1; j < K; j++) acc ^= v[j];
#pragma unroll
  for (int i = 0; i < R; i++) {
    bs::v4 o = acc;
    o.x ^= i;
    bs::st_nt(reinterpret_cast<bs::v4 *>(a.out[i] + (uint64_t)stripe * a.out_stride[i]) + c, o);
  }
}

using Fn = std::function<hipError_t(const ApplyArgs &, hipStream_t)>;
struct V {
  std::string name;
  Fn fn;
  std::vector<float> us;
};

// Workgroup size T (lanes; each wave streams 2 KiB of every share) x
// tile rotation per stripe (SWZ) x resident-workgroup cap, for load group G.
template <int K, int N, int G, int T, int SWZ>
void add(std::vector<V> &vs, std::initializer_list<int> caps) {
  for (int cap : caps)
    vs.push_back({"G=" + std::to_string(G) + " T=" + std::to_string(T) + " swz=" +
                      std::to_string(SWZ) + " cap=" + std::to_string(cap),
                  [cap](const ApplyArgs &a, hipStream_t s) {
                    const uint64_t cpt = bs::bs_cols_per_tile(T);
                    const uint64_t blocks = ((a.block / 16 + cpt - 1) / cpt) * a.nstripes;
                    return launch_lds<k_bs<K, N, G, T, SWZ>>(blocks, T, cap_lds(cap, 0), s, a);
                  }, {}});
}

// Input-split workgroups (rs_bitslice_core.h bs_ksplit_body): W waves on the
// same 2 KiB of every share, each folding k / W inputs, G per load group.
template <int K, int N, int C, int W, int G, int SWZ>
void add_ks(std::vector<V> &vs, std::initializer_list<int> caps) {
  for (int cap : caps)
    vs.push_back({"ksplit C=" + std::to_string(C) + " W=" + std::to_string(W) + " G=" +
                      std::to_string(G) + " swz=" + std::to_string(SWZ) + " cap=" +
                      std::to_string(cap),
                  [cap](const ApplyArgs &a, hipStream_t s) {
                    const uint64_t cpt = 128 * C;
                    const uint64_t blocks = ((a.block / 16 + cpt - 1) / cpt) * a.nstripes;
                    return launch_lds<k_ks<K, N, C, W, G, SWZ>>(
                        blocks, 64 * C * W, cap_lds(cap, bs::ksplit_lds_bytes(C, W, N - K)), s, a);
                  }, {}});
}

template <int K, int N, int G, int T, int SWZ>
void add0(std::vector<V> &vs, std::initializer_list<int> caps) {
  for (int cap : caps)
    vs.push_back({"nogf G=" + std::to_string(G) + " T=" + std::to_string(T) + " swz=" +
                      std::to_string(SWZ) + " cap=" + std::to_string(cap),
                  [cap](const ApplyArgs &a, hipStream_t s) {
                    const uint64_t cpt = bs::bs_cols_per_tile(T);
                    const uint64_t blocks = ((a.block / 16 + cpt - 1) / cpt) * a.nstripes;
                    return launch_lds<k_bs0<K, N, G, T, SWZ>>(blocks, T, cap_lds(cap, 0), s, a);
                  }, {}});
}
template <int K, int N, int C, int W, int G, int SWZ>
void add_ks0(std::vector<V> &vs, std::initializer_list<int> caps) {
  for (int cap : caps)
    vs.push_back({"nogf ksplit C=" + std::to_string(C) + " W=" + std::to_string(W) + " G=" +
                      std::to_string(G) + " cap=" + std::to_string(cap),
                  [cap](const ApplyArgs &a, hipStream_t s) {
                    const uint64_t cpt = 128 * C;
                    const uint64_t blocks = ((a.block / 16 + cpt - 1) / cpt) * a.nstripes;
                    return launch_lds<k_ks0<K, N, C, W, G, SWZ>>(
                        blocks, 64 * C * W, cap_lds(cap, bs::ksplit_lds_bytes(C, W, N - K)), s, a);
                  }, {}});
}
template <int K, int N, int T>
void add_flat(std::vector<V> &vs, std::initializer_list<int> caps) {
  for (int cap : caps)
    vs.push_back({"flat16B T=" + std::to_string(T) + " cap=" + std::to_string(cap),
                  [cap](const ApplyArgs &a, hipStream_t s) {
                    const uint64_t blocks = (a.block / 16 / T) * a.nstripes;
                    return launch_lds<k_flat<K, N - K, T>>(blocks, T, cap_lds(cap, 0), s, a);
                  }, {}});
}

// dec = false: encode layout (k data shares in, n - k parity shares out, each
// region packed per stripe). dec = true: the in-place decode layout of
// bench.py --erase R (data shares 0..R-1 lost, rebuilt into their slots of the
// data region from data shares R..K-1 and parity shares 0..R-1), so reads and
// writes share the data region as they do in the product.
template <int K, int N>
void run(const char *name, uint32_t nstripes, uint64_t B, int rounds, bool dec = false) {
  constexpr int R = N - K;
  std::vector<V> vs;
  const bool nogf = std::getenv("BSTUNE_NOGF") != nullptr;
  if (!dec && !nogf)
    vs.push_back({"product", [](const ApplyArgs &a, hipStream_t s) {
                    return bs::launch_bitslice<K, N>(a, s);
                  }, {}});
  constexpr int G = bs::bs_group(K, R);
  if (nogf) {  // access-shape ceilings; not compared bit-exactly across shapes
    add0<K, N, G, 64, 1>(vs, {4, 6});
    if constexpr (R == 8) {
      add_ks0<K, N, 1, 4, 4, 1>(vs, {4, 6});
      add_ks0<K, N, 2, 2, 8, 1>(vs, {2, 3});
      add_ks0<K, N, 2, 2, 4, 1>(vs, {2, 3});
      add_ks0<K, N, 2, 4, 4, 1>(vs, {1});
    } else if constexpr (R == 16) {
      add_ks0<K, N, 2, 2, 2, 1>(vs, {2, 3});
    }
    add_flat<K, N, 256>(vs, {0, 1, 2});
    add_flat<K, N, 512>(vs, {1});
    add_flat<K, N, 128>(vs, {2, 4});
  } else if (std::getenv("BSTUNE_FEWROWS")) {  // decodes with few lost rows: G x (T, cap)
    if constexpr (R <= 8) {  // the product shape (bs_shape) first: the bit-exact reference
      constexpr bs::BsShape S = bs::bs_shape(K, R);
      add<K, N, G, S.threads, S.swz>(vs, {S.cap});
      add<K, N, 4, 128, 0>(vs, {2, 4, 5});
      add<K, N, 4, 64, 0>(vs, {3, 4, 6, 7, 8});
      add<K, N, 4, 64, 1>(vs, {4, 7});
      add<K, N, 4, 256, 0>(vs, {1, 2});
    }
  } else if (std::getenv("BSTUNE_KSPLIT")) {  // input-split workgroups x cap
    if (dec) {  // the JIT decode kernels' shape first (rs_args.h bs_shape): the reference
      constexpr bs::BsShape S = bs::bs_shape(K, R);
      add<K, N, G, S.threads, S.swz>(vs, {S.cap});
    }
    if constexpr (R == 8) {
      add_ks<K, N, 1, 4, 4, 1>(vs, {4});
      add_ks<K, N, 2, 2, 8, 1>(vs, {2, 3});
      add_ks<K, N, 2, 2, 4, 1>(vs, {2, 3});
    }
    if constexpr (R == 16) {
      add_ks<K, N, 2, 2, 4, 1>(vs, {2});
      add_ks<K, N, 2, 2, 2, 1>(vs, {2});
    }
    if constexpr (R == 2 || R == 4) {
      add_ks<K, N, 1, 2, 4, 1>(vs, {3, 4, 6, 8});
      add_ks<K, N, 2, 2, 4, 1>(vs, {2, 3, 4});
      if constexpr (K / 2 % 8 == 0) add_ks<K, N, 2, 2, 8, 1>(vs, {2, 3, 4});
      if constexpr (K % 4 == 0 && R == 4) add_ks<K, N, 1, 4, 4, 1>(vs, {2, 3, 4});
      if constexpr (K % 4 == 0 && R == 4) add_ks<K, N, 2, 4, 4, 1>(vs, {1, 2});
    }
  } else if (std::getenv("BSTUNE_LOWCAP")) {  // fewer bytes in flight per CU
    add<K, N, G, 64, 1>(vs, {2, 3, 4, 6});
    add<K, N, G, 128, 1>(vs, {1, 2, 3});
    add<K, N, G, 256, 1>(vs, {1});
    if constexpr (K % 4 == 0 && G != 4) {
      add<K, N, 4, 64, 1>(vs, {3, 4, 6, 8});
      add<K, N, 4, 128, 1>(vs, {2, 3});
    }
    if constexpr (K % 2 == 0 && G != 2) add<K, N, 2, 64, 1>(vs, {4, 6, 8});
  } else if (std::getenv("BSTUNE_GROUPS")) {  // load-group size at the product shapes
    add<K, N, G, 64, 1>(vs, {6});
    add<K, N, G, 128, 0>(vs, {3, 4});
    if constexpr (K == 16) {
      add<K, N, 16, 64, 1>(vs, {4, 6, 8});
      add<K, N, 16, 128, 0>(vs, {2, 3, 4});
      add<K, N, 2, 64, 1>(vs, {6, 8});
      add<K, N, 2, 128, 0>(vs, {3, 4});
      add<K, N, 4, 128, 0>(vs, {3, 4});
    }
  } else {
    add<K, N, G, 256, 0>(vs, {0, 2});
    add<K, N, G, 128, 0>(vs, {3, 4});
    add<K, N, G, 128, 1>(vs, {4});
    add<K, N, G, 64, 0>(vs, {4, 5, 6, 8});
    add<K, N, G, 64, 1>(vs, {4, 5, 6, 8});
  }
  // parity region: Storb's n - k = k / 2 shares per stripe in the decode layout
  constexpr int P = K / 2;
  const uint64_t in_bytes = (uint64_t)nstripes * K * B, out_bytes = (uint64_t)nstripes * R * B;
  const uint64_t par_bytes = dec ? (uint64_t)nstripes * P * B : out_bytes;
  uint8_t *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, par_bytes));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, K);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)out, par_bytes / 8, N);
  ApplyArgs a{};
  a.k = K;
  a.r = R;
  for (int j = 0; j < K; j++) {
    const bool par = dec && j >= K - R;
    a.in[j] = par ? out + (j - (K - R)) * B : in + (dec ? j + R : j) * B;
    a.in_stride[j] = par ? P * B : K * B;
  }
  for (int i = 0; i < R; i++) {
    a.out[i] = dec ? in + i * B : out + i * B;
    a.out_stride[i] = dec ? K * B : R * B;
  }
  a.block = B;
  a.nstripes = nstripes;
  uint8_t *res = dec ? in : out;
  const uint64_t res_bytes = dec ? in_bytes : out_bytes;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<uint8_t> ref(res_bytes), got(res_bytes);
  for (size_t vi = 0; vi < vs.size(); vi++) {
    if (!dec) CK(hipMemset(out, 0xA5, out_bytes));
    CK(vs[vi].fn(a, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? got.data() : ref.data(), res, res_bytes, hipMemcpyDeviceToHost));
    if (vi && !nogf && std::memcmp(got.data(), ref.data(), res_bytes)) {
      std::printf("MISMATCH %s %s\n", name, vs[vi].name.c_str());
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
  const double bytes = (double)in_bytes + out_bytes;  // k*B read + r*B written, either layout
  std::printf("%s: %.3f GB algorithmic per launch%s\n", name, bytes / 1e9,
              nogf ? " (no-GF shapes: outputs not compared)" : ", every variant bit-exact");
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    std::printf("  %-26s median %8.1f us  %7.1f GB/s  %.1f%% of 8 TB/s\n", v.name.c_str(), med,
                bytes / med / 1e3, bytes / med / 1e3 / 80.0);
  }
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipStreamDestroy(s));
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  const int which = argc > 2 ? std::atoi(argv[2]) : 0;  // 0 all, 1 encode, 2 decode, 3 k=16 only
  if (which == 4) {  // few-row decodes (BSTUNE_FEWROWS): config 5's decode shape
    run<16, 18>("decode k=16, 2 lost (in place)", 128, 512 << 10, rounds, true);
    run<16, 20>("decode k=16, 4 lost (in place)", 128, 512 << 10, rounds, true);
    return 0;
  }
  if (which == 5) {  // decodes for the input-split JIT shapes (BSTUNE_KSPLIT)
    run<16, 18>("decode k=16, 2 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<16, 20>("decode k=16, 4 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<16, 24>("decode k=16, 8 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<32, 34>("decode k=32, 2 lost, 32 x 32 MiB (in place)", 32, 1 << 20, rounds, true);
    run<32, 48>("decode k=32, 16 lost, 32 x 32 MiB (in place)", 32, 1 << 20, rounds, true);
    return 0;
  }
  if (which == 3) {
    run<16, 24>("RS(16,8) encode 128 x 8 MiB", 128, 512 << 10, rounds);
    run<16, 18>("decode k=16, 2 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<16, 24>("decode k=16, 8 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    return 0;
  }
  if (which != 2) {
    run<16, 24>("RS(16,8) encode 128 x 8 MiB", 128, 512 << 10, rounds);
    run<32, 48>("RS(32,16) encode 32 x 32 MiB", 32, 1 << 20, rounds);
  }
  if (which != 1) {
    run<16, 18>("decode k=16, 2 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<16, 20>("decode k=16, 4 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<16, 24>("decode k=16, 8 lost, 128 x 8 MiB (in place)", 128, 512 << 10, rounds, true);
    run<32, 34>("decode k=32, 2 lost, 32 x 32 MiB (in place)", 32, 1 << 20, rounds, true);
    run<32, 48>("decode k=32, 16 lost, 32 x 32 MiB (in place)", 32, 1 << 20, rounds, true);
  }
  return 0;
}
