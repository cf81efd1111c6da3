// hbm_probe.hip -- what access shape / cache policy streams HBM fastest on
// gfx950, for the byte-moving shape of the RS kernels (read k shares of a
// stripe at one column, write r shares).
//
// Every variant moves the same bytes: NS stripes x (KI input + RO output)
// shares of B bytes, each lane one 16-byte column of every share. Inputs are
// XOR-combined (no GF work) so nothing is dead code. Variants differ in:
//   * cache policy bits on the buffer loads / stores (aux: 1 = sc0,
//     2 = nt, 16 = sc1; gfx950 encodings),
//   * blockIdx -> tile mapping (stripe-major as in the product kernel, or
//     column-major: consecutive workgroups walk different stripes),
//   * shape: (KI, RO) = (4, 2) the RS(4,2) encode, (1, 1) copy, (4, 0) read
//     only (one dword per lane written only if a never-true test holds),
//     (0, 2) write only.
// One process, interleaved rounds, median of the rounds per variant; each
// sample times `reps` back-to-back launches (argv[3], default 8).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 hbm_probe.hip -o _build/hbm_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,                 \
                   hipGetErrorString(e));                                            \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const uint8_t *in;   // NS * KI * B
  uint8_t *out;        // NS * RO * B
  uint32_t *sink;
  uint64_t B;
  uint32_t ns;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

template <int KI, int RO, int LA, int SA, bool COLMAJOR, int T>
__global__ __launch_bounds__(T) void probe(const Args a) {
  const uint32_t cols = static_cast<uint32_t>(a.B >> 4);
  const uint32_t tps = cols / T;
  uint32_t stripe, tile;
  if (COLMAJOR) {
    stripe = blockIdx.x % a.ns;
    tile = blockIdx.x / a.ns;
  } else {
    stripe = blockIdx.x / tps;
    tile = blockIdx.x % tps;
  }
  const uint32_t off = (tile * T + threadIdx.x) * 16;
  u32x4 acc = {0, 0, 0, 0};
  if constexpr (KI > 0) {
    const uint8_t *base = a.in + static_cast<uint64_t>(stripe) * KI * a.B;
    const __amdgpu_buffer_rsrc_t r = rsrc(base, static_cast<uint32_t>(KI * a.B));
    u32x4 v[KI > 0 ? KI : 1];
#pragma unroll
    for (int j = 0; j < KI; j++)
      v[j] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off + j * static_cast<uint32_t>(a.B),
                                                        0, LA));
#pragma unroll
    for (int j = 0; j < KI; j++) acc ^= v[j];
  } else {
    acc = u32x4{off, stripe, off ^ 0x5a5a5a5au, stripe * 3u};
  }
  if constexpr (RO > 0) {
    uint8_t *base = a.out + static_cast<uint64_t>(stripe) * RO * a.B;
    const __amdgpu_buffer_rsrc_t r = rsrc(base, static_cast<uint32_t>(RO * a.B));
#pragma unroll
    for (int i = 0; i < RO; i++) {
      u32x4 o = acc;
      o.x ^= i;
      __builtin_amdgcn_raw_buffer_store_b128(o, r, off + i * static_cast<uint32_t>(a.B), 0, SA);
    }
  } else {
    if ((acc.x & acc.y & acc.z & acc.w) == 0xdeadbeefu) a.sink[threadIdx.x] = acc.x;
  }
}

// Same shape with global_load / global_store (what the product kernel
// emits): NTL / NTS = __builtin_nontemporal_load / _store.
template <int KI, int RO, bool NTL, bool NTS, int T>
__global__ __launch_bounds__(T) void probe_global(const Args a) {
  const uint32_t cols = static_cast<uint32_t>(a.B >> 4);
  const uint32_t tps = cols / T;
  const uint32_t stripe = blockIdx.x / tps, tile = blockIdx.x % tps;
  const uint32_t c = tile * T + threadIdx.x;
  const u32x4 *in = reinterpret_cast<const u32x4 *>(a.in + static_cast<uint64_t>(stripe) * KI * a.B);
  u32x4 *out = reinterpret_cast<u32x4 *>(a.out + static_cast<uint64_t>(stripe) * RO * a.B);
  u32x4 v[KI];
#pragma unroll
  for (int j = 0; j < KI; j++) v[j] = NTL ? __builtin_nontemporal_load(in + j * cols + c) : in[j * cols + c];
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < KI; j++) acc ^= v[j];
#pragma unroll
  for (int i = 0; i < RO; i++) {
    u32x4 o = acc;
    o.x ^= i;
    if (NTS)
      __builtin_nontemporal_store(o, out + i * cols + c);
    else
      out[i * cols + c] = o;
  }
}

// RS(4,2) traffic with W rounds of dummy VALU work per input dword (a
// v_perm + xor chain, ~2 ops per round), to see how the store policy
// interacts with the compute the product kernel does between its loads and
// stores (~60 VALU per dword of output for RS(4,2)).
template <int W, bool NTS, int U, int T>
__global__ __launch_bounds__(T) void probe_work(const Args a) {
  const uint32_t cols = static_cast<uint32_t>(a.B >> 4);
  const uint32_t tps = cols / (T * U);
  const uint32_t stripe = blockIdx.x / tps, tile = blockIdx.x % tps;
  const u32x4 *in = reinterpret_cast<const u32x4 *>(a.in + static_cast<uint64_t>(stripe) * 4 * a.B);
  u32x4 *out = reinterpret_cast<u32x4 *>(a.out + static_cast<uint64_t>(stripe) * 2 * a.B);
  u32x4 v[U][4];
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 0; j < 4; j++)
      v[u][j] = __builtin_nontemporal_load(in + j * cols + tile * T * U + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 p = {0, 0, 0, 0}, q = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int w = 0; w < 4; w++) {
        uint32_t x = v[u][j][w];
#pragma unroll
        for (int r = 0; r < W; r++) {
          x = __builtin_amdgcn_perm(x, 0x01234567u + r, 0x07060504u + j);
          x ^= 0x9e3779b9u * (r + 1);
        }
        p[w] ^= x;
        q[w] ^= x + j;
      }
    u32x4 *o0 = out + tile * T * U + u * T + threadIdx.x, *o1 = o0 + cols;
    if (NTS) {
      __builtin_nontemporal_store(p, o0);
      __builtin_nontemporal_store(q, o1);
    } else {
      *o0 = p;
      *o1 = q;
    }
  }
}

__global__ void fill_random(uint32_t *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x5709B;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = static_cast<uint32_t>(z ^ (z >> 31));
  }
}

// RS(4,2) traffic with the workgroup -> tile map made XCD-aware: the
// dispatcher deals workgroups round-robin over the 8 XCDs, so workgroup b
// runs on XCD b % 8; remapped, XCD x streams the contiguous x-th eighth of
// the tiles (tile = (b % 8) * (grid / 8) + b / 8) instead of every 8th tile.
template <bool NTS, int T>
__global__ __launch_bounds__(T) void probe_xcd(const Args a) {
  const uint32_t cols = static_cast<uint32_t>(a.B >> 4);
  const uint32_t tps = cols / T;
  const uint32_t per = gridDim.x / 8;
  const uint32_t bid = (blockIdx.x % 8) * per + blockIdx.x / 8;
  const uint32_t stripe = bid / tps, tile = bid % tps;
  const uint32_t c = tile * T + threadIdx.x;
  const u32x4 *in = reinterpret_cast<const u32x4 *>(a.in + static_cast<uint64_t>(stripe) * 4 * a.B);
  u32x4 *out = reinterpret_cast<u32x4 *>(a.out + static_cast<uint64_t>(stripe) * 2 * a.B);
  u32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; j++) v[j] = __builtin_nontemporal_load(in + j * cols + c);
  u32x4 acc = v[0] ^ v[1] ^ v[2] ^ v[3];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    u32x4 o = acc;
    o.x ^= i;
    if (NTS)
      __builtin_nontemporal_store(o, out + i * cols + c);
    else
      out[i * cols + c] = o;
  }
}

// Wide shapes with U columns per lane (U x 4 KiB of every share per
// workgroup): does a longer run per stream help when 16+ streams interleave?
template <int KI, int RO, int U, int T>
__global__ __launch_bounds__(T) void probe_u(const Args a) {
  const uint32_t cols = static_cast<uint32_t>(a.B >> 4);
  const uint32_t tps = cols / (T * U);
  const uint32_t stripe = blockIdx.x / tps, tile = blockIdx.x % tps;
  const u32x4 *in = reinterpret_cast<const u32x4 *>(a.in + static_cast<uint64_t>(stripe) * KI * a.B);
  u32x4 *out = reinterpret_cast<u32x4 *>(a.out + static_cast<uint64_t>(stripe) * RO * a.B);
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t c = tile * T * U + u * T + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < KI; j++) acc ^= __builtin_nontemporal_load(in + j * cols + c);
#pragma unroll
    for (int i = 0; i < RO; i++) {
      u32x4 o = acc;
      o.x ^= i;
      __builtin_nontemporal_store(o, out + i * cols + c);
    }
  }
}

struct Variant {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

int main(int argc, char **argv) {
  const uint64_t B = 256 << 10;          // 256 KiB shares, as RS(4,2) of 1 MiB chunks
  const uint32_t NS = 1024;              // 1 GiB of data shares
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  // Launches per timed sample: 1 measures a cold single launch (dirty lines
  // left in L2/MALL are written back after the end event); 8 measures the
  // steady state a stream of launches sees.
  const int reps = argc > 3 ? std::atoi(argv[3]) : 8;
  uint8_t *in, *out;
  uint32_t *sink;
  CK(hipMalloc(&in, NS * 4 * B));
  CK(hipMalloc(&out, NS * 2 * B));
  CK(hipMalloc(&sink, 4096));
  if (argc > 2 && std::atoi(argv[2]) == 1)
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0,
                       reinterpret_cast<uint32_t *>(in), NS * 4 * B / 4);
  else
    CK(hipMemset(in, 0x3c, NS * 4 * B));
  CK(hipDeviceSynchronize());
  CK(hipMemset(out, 0, NS * 2 * B));
  Args a{in, out, sink, B, NS};
  std::vector<Variant> vs;
  constexpr int T = 256;
  const uint32_t grid = static_cast<uint32_t>(NS * (B / 16 / T));

#define ADD(KI, RO, LA, SA, CM)                                                                \
  vs.push_back(Variant{std::string("KI=") + #KI + " RO=" + #RO + " la=" + #LA + " sa=" + #SA + \
                           (CM ? " colmajor" : " stripemajor"),                                \
                       static_cast<double>(NS) * ((KI) + (RO)) * B,                           \
                       [=](hipStream_t s) {                                                    \
                         hipLaunchKernelGGL((probe<KI, RO, LA, SA, CM, T>), dim3(grid),        \
                                            dim3(T), 0, s, a);                                 \
                       },                                                                      \
                       {}})

  // RS(4,2) shape over cache policies
  ADD(4, 2, 0, 0, false);
  ADD(4, 2, 2, 2, false);
  ADD(4, 2, 2, 0, false);
  ADD(4, 2, 0, 2, false);
  ADD(4, 2, 1, 2, false);
  ADD(4, 2, 3, 2, false);
  ADD(4, 2, 16, 2, false);
  ADD(4, 2, 18, 2, false);
  ADD(4, 2, 19, 19, false);
  ADD(4, 2, 2, 18, false);
  ADD(4, 2, 2, 3, false);
  ADD(4, 2, 2, 2, true);
  // other shapes, nt
  ADD(1, 1, 2, 2, false);
  ADD(1, 1, 0, 0, false);
  ADD(4, 0, 2, 0, false);
  ADD(4, 0, 0, 0, false);
  ADD(4, 0, 3, 0, false);
  ADD(0, 2, 0, 2, false);
  ADD(0, 2, 0, 0, false);

#define ADDG(KI, RO, NTL, NTS)                                                                 \
  vs.push_back(Variant{std::string("global KI=") + #KI + " RO=" + #RO + " ntl=" + #NTL +        \
                           " nts=" + #NTS,                                                     \
                       static_cast<double>(NS) * ((KI) + (RO)) * B,                           \
                       [=](hipStream_t s) {                                                    \
                         hipLaunchKernelGGL((probe_global<KI, RO, NTL, NTS, T>), dim3(grid),   \
                                            dim3(T), 0, s, a);                                 \
                       },                                                                      \
                       {}})
  ADDG(4, 2, true, true);
  ADDG(4, 2, true, false);
  ADDG(4, 2, false, false);
  ADDG(1, 1, true, false);
  ADDG(1, 1, false, false);

#define ADDW(W, NTS, U)                                                                        \
  vs.push_back(Variant{std::string("work W=") + #W + " nts=" + #NTS + " U=" + #U,              \
                       static_cast<double>(NS) * 6 * B,                                        \
                       [=](hipStream_t s) {                                                    \
                         hipLaunchKernelGGL((probe_work<W, NTS, U, T>), dim3(grid / (U)),      \
                                            dim3(T), 0, s, a);                                 \
                       },                                                                      \
                       {}})
  ADDW(0, true, 1);
  ADDW(0, false, 1);
  ADDW(4, true, 1);
  ADDW(4, false, 1);
  ADDW(8, true, 1);
  ADDW(8, false, 1);
  ADDW(16, true, 1);
  ADDW(16, false, 1);
  ADDW(8, true, 2);
  ADDW(8, false, 2);

  // wide stripes (Storb's k = 16 geometry): a quarter of the stripes, same bytes
  const Args a16{in, out, sink, B, NS / 4};
  const uint32_t grid16 = static_cast<uint32_t>((NS / 4) * (B / 16 / T));
#define ADD16(KI, RO)                                                                          \
  vs.push_back(Variant{std::string("wide KI=") + #KI + " RO=" + #RO + " nt/nt",                 \
                       static_cast<double>(NS / 4) * ((KI) + (RO)) * B,                       \
                       [=](hipStream_t s) {                                                    \
                         hipLaunchKernelGGL((probe<KI, RO, 2, 2, false, T>), dim3(grid16),     \
                                            dim3(T), 0, s, a16);                               \
                       },                                                                      \
                       {}})
#define ADDU(KI, RO, U)                                                                        \
  vs.push_back(Variant{std::string("wide KI=") + #KI + " RO=" + #RO + " U=" + #U,               \
                       static_cast<double>(NS / 4) * ((KI) + (RO)) * B,                       \
                       [=](hipStream_t s) {                                                    \
                         hipLaunchKernelGGL((probe_u<KI, RO, U, T>), dim3(grid16 / (U)),       \
                                            dim3(T), 0, s, a16);                               \
                       },                                                                      \
                       {}})
  ADDU(16, 2, 1);
  ADDU(16, 2, 2);
  ADDU(16, 2, 4);
  ADDU(16, 8, 2);
  ADD16(16, 2);
  ADD16(16, 8);
  ADD16(8, 4);
  ADD16(8, 3);
  vs.push_back(Variant{"xcd-remapped KI=4 RO=2 nt/nt", static_cast<double>(NS) * 6 * B,
                       [=](hipStream_t s) {
                         hipLaunchKernelGGL((probe_xcd<true, T>), dim3(grid), dim3(T), 0, s, a);
                       },
                       {}});
  vs.push_back(Variant{"xcd-remapped KI=4 RO=2 nt/default", static_cast<double>(NS) * 6 * B,
                       [=](hipStream_t s) {
                         hipLaunchKernelGGL((probe_xcd<false, T>), dim3(grid), dim3(T), 0, s, a);
                       },
                       {}});

  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &v : vs) v.run(s);  // warm
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; r++) {
    for (auto &v : vs) {
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; i++) v.run(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / reps);
    }
  }
  std::printf("B=%llu KiB, %u stripes, %d rounds (median), %d launches per sample\n",
              static_cast<unsigned long long>(B >> 10), NS, rounds, reps);
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    std::printf("%-44s %9.1f us  %7.1f GB/s  (min %7.1f GB/s)\n", v.name.c_str(), med * 1e3,
                v.bytes / (med * 1e-3) / 1e9, v.bytes / (v.ms[0] * 1e-3) / 1e9);
  }
  return 0;
}
