// wide_probe.hip -- why do the wide RS access shapes (16 or 32 input share
// streams + 8 or 16 output streams per stripe) stream HBM slower than
// RS(4,2)'s 4 + 2? (16 + 8 caps near 6.2 TB/s with no GF work
// at all, 4 + 2 reaches 6.45-6.7.)
//
// Every variant moves the config-5 bytes: 128 stripes of 16 x 512 KiB data
// shares (1 GiB) in, 8 x 512 KiB parity shares per stripe out, inputs XOR-
// combined so nothing is dead. Hypotheses, one variant family each:
//   pitch   share pitch B + 4 KiB / + 256 B instead of B (2^19): bank /
//           channel aliasing of the 24 streams that sit 512 KiB apart;
//   ro/wo   read-only / write-only of the same shape (is it the mix?);
//   cols    1, 2 or 4 columns per lane (8-32 KiB of a share per workgroup);
//   grp     loads issued all at once vs groups of 4/8 with a wait between;
//   pers    persistent grid (cap x 256 workgroups looping over tiles);
//   wg      512- and 1024-lane workgroups (same tile per lane);
//   swz     tile order rotated per stripe, so concurrently running
//           workgroups of neighbouring stripes sit at different offsets;
//   cap     resident-workgroup caps via LDS reservation (2, 4).
// One process, interleaved rounds, median; each sample times 8 launches.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 wide_probe.hip -o _build/wide_probe
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

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

struct Args {
  const uint8_t *in;  // ns stripes x KI shares, share pitch P
  uint8_t *out;       // ns stripes x RO shares, share pitch P
  uint32_t *sink;
  uint64_t B;         // share bytes
  uint64_t P;         // share pitch
  uint32_t ns;
};

// One tile = U columns per lane x T lanes of every share of a stripe. GRP:
// loads issued in groups of GRP shares, the group's XOR folded (forcing a
// vmcnt wait) before the next group is issued (0 = all at once).
template <int KI, int RO, int U, int T, int GRP, int SWZ>
__device__ __forceinline__ void tile_body(const Args &a, uint32_t stripe, uint32_t tile,
                                          uint32_t tps) {
  // tile order per stripe: 1 rotate by stripe * (tps/8 + 1), 2 rotate by
  // half a stripe on odd stripes, 3 XOR with a stripe hash
  if (SWZ == 1) tile = (tile + stripe * (tps / 8 + 1)) % tps;
  if (SWZ == 2) tile = (tile + (stripe & 1) * (tps / 2)) % tps;
  if (SWZ == 3) tile = tile ^ ((stripe * 0x9Du) & (tps - 1));
  const uint32_t c0 = tile * T * U + threadIdx.x;
  const uint8_t *ib = a.in + static_cast<uint64_t>(stripe) * KI * a.P;
  uint8_t *ob = a.out + static_cast<uint64_t>(stripe) * RO * a.P;
  v4 acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) acc[u] = v4{0, 0, 0, 0};
  if constexpr (KI > 0) {
    constexpr int G = GRP == 0 ? KI : GRP;
#pragma unroll
    for (int g0 = 0; g0 < KI; g0 += G) {
      v4 v[G][U];
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int u = 0; u < U; u++)
          v[g][u] = __builtin_nontemporal_load(
              reinterpret_cast<const v4 *>(ib + (g0 + g) * a.P) + c0 + u * T);
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= v[g][u];
      if (GRP) asm volatile("" : "+v"(acc[0]));
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = v4{c0, stripe, c0 ^ 0x5a5a5a5au, stripe * 3u + u};
  }
  if constexpr (RO > 0) {
#pragma unroll
    for (int i = 0; i < RO; i++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        v4 o = acc[u];
        o.x ^= i;
        __builtin_nontemporal_store(o, reinterpret_cast<v4 *>(ob + i * a.P) + c0 + u * T);
      }
  } else {
    v4 t = acc[0];
#pragma unroll
    for (int u = 1; u < U; u++) t ^= acc[u];
    if ((t.x & t.y & t.z & t.w) == 0xdeadbeefu) a.sink[threadIdx.x] = t.x;
  }
}

template <int KI, int RO, int U, int T, int GRP, int SWZ, int LDSB>
__global__ __launch_bounds__(T) void probe(const Args a) {
  if constexpr (LDSB > 0) {
    __shared__ uint32_t pad[LDSB / 4];
    asm volatile("" ::"v"(pad));
  }
  const uint32_t tps = static_cast<uint32_t>(a.B / 16 / (T * U));
  const uint32_t stripe = blockIdx.x / tps, tile = blockIdx.x % tps;
  tile_body<KI, RO, U, T, GRP, SWZ>(a, stripe, tile, tps);
}

template <int KI, int RO, int U, int T>
__global__ __launch_bounds__(T) void probe_pers(const Args a) {
  const uint32_t tps = static_cast<uint32_t>(a.B / 16 / (T * U));
  const uint32_t total = tps * a.ns;
  for (uint32_t b = blockIdx.x; b < total; b += gridDim.x)
    tile_body<KI, RO, U, T, 0, 0>(a, b / tps, b % tps, tps);
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

struct Variant {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

// LDS reservation that leaves `cap` 256-lane workgroups resident per CU
// (160 KiB LDS per CU; as rs_kernels.hpp cap_lds).
constexpr int lds_for(int cap) { return cap ? (160 * 1024) / cap - 1024 : 0; }

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const int reps = 8;
  const uint64_t B = 512 << 10;
  const uint32_t NS = 128;
  const uint64_t PMAX = B + 4096;
  uint8_t *in, *out;
  uint32_t *sink;
  // sized for the widest shape: 32 shares of 1 MiB x 32 stripes = 16 x 512 KiB x 128
  CK(hipMalloc(&in, NS * 16 * PMAX + (64 << 20)));
  CK(hipMalloc(&out, NS * 8 * PMAX + (64 << 20)));
  CK(hipMalloc(&sink, 4096));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(in),
                     (NS * 16 * PMAX) / 4);
  CK(hipDeviceSynchronize());
  CK(hipMemset(out, 0, NS * 8 * PMAX));
  std::vector<Variant> vs;
  int ncu = 256;
  {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    ncu = pr.multiProcessorCount;
  }

#define ADDV(NAME, KI, RO, U, T, GRP, SWZ, LDSB, PITCH, BB, NSS)                              \
  do {                                                                                       \
    const Args aa{in, out, sink, (BB), (PITCH), (NSS)};                                      \
    const uint32_t grid = static_cast<uint32_t>((NSS) * ((BB) / 16 / ((T) * (U))));          \
    vs.push_back(Variant{NAME, static_cast<double>(NSS) * ((KI) + (RO)) * (BB),             \
                         [=](hipStream_t s) {                                                \
                           hipLaunchKernelGGL((probe<KI, RO, U, T, GRP, SWZ, LDSB>),         \
                                              dim3(grid), dim3(T), 0, s, aa);                \
                         },                                                                  \
                         {}});                                                               \
  } while (0)

  // round 2 of the probe: combinations of what helped in round 1 (tile
  // rotation per stripe, resident-workgroup caps) and smaller per-workgroup
  // footprints (T = 64 / 128 lanes)
  const uint64_t K2 = 256 << 10, M1 = 1 << 20;
  ADDV("rs42 base", 4, 2, 1, 256, 0, 0, 0, K2, K2, 1024);
  ADDV("rs42 cap4", 4, 2, 1, 256, 0, 0, lds_for(4), K2, K2, 1024);
  ADDV("rs42 swz1", 4, 2, 1, 256, 0, 1, 0, K2, K2, 1024);
  ADDV("rs42 swz1 cap4", 4, 2, 1, 256, 0, 1, lds_for(4), K2, K2, 1024);
  ADDV("rs42 swz2 cap4", 4, 2, 1, 256, 0, 2, lds_for(4), K2, K2, 1024);
  ADDV("rs42 swz3 cap4", 4, 2, 1, 256, 0, 3, lds_for(4), K2, K2, 1024);
  ADDV("rs42 swz1 cap2", 4, 2, 1, 256, 0, 1, lds_for(2), K2, K2, 1024);
  ADDV("rs42 T128 cap8", 4, 2, 1, 128, 0, 0, lds_for(8), K2, K2, 1024);
  ADDV("rs42 T128 swz1 cap8", 4, 2, 1, 128, 0, 1, lds_for(8), K2, K2, 1024);
  ADDV("16+8 base", 16, 8, 1, 256, 0, 0, 0, B, B, NS);
  ADDV("16+8 cap2", 16, 8, 1, 256, 0, 0, lds_for(2), B, B, NS);
  ADDV("16+8 cap1", 16, 8, 1, 256, 0, 0, lds_for(1), B, B, NS);
  ADDV("16+8 swz1", 16, 8, 1, 256, 0, 1, 0, B, B, NS);
  ADDV("16+8 swz1 cap2", 16, 8, 1, 256, 0, 1, lds_for(2), B, B, NS);
  ADDV("16+8 swz2 cap2", 16, 8, 1, 256, 0, 2, lds_for(2), B, B, NS);
  ADDV("16+8 swz3 cap2", 16, 8, 1, 256, 0, 3, lds_for(2), B, B, NS);
  ADDV("16+8 swz1 cap4", 16, 8, 1, 256, 0, 1, lds_for(4), B, B, NS);
  ADDV("16+8 T128 cap4", 16, 8, 1, 128, 0, 0, lds_for(4), B, B, NS);
  ADDV("16+8 T128 swz1 cap4", 16, 8, 1, 128, 0, 1, lds_for(4), B, B, NS);
  ADDV("16+8 T128 swz1 cap2", 16, 8, 1, 128, 0, 1, lds_for(2), B, B, NS);
  ADDV("16+8 T64 swz1 cap4", 16, 8, 1, 64, 0, 1, lds_for(4), B, B, NS);
  ADDV("16+8 T64 swz1 cap8", 16, 8, 1, 64, 0, 1, lds_for(8), B, B, NS);
  // the bit-sliced kernels' lane shape: 2 columns per lane
  ADDV("16+8 2col cap2", 16, 8, 2, 256, 0, 0, lds_for(2), B, B, NS);
  ADDV("16+8 2col swz1 cap2", 16, 8, 2, 256, 0, 1, lds_for(2), B, B, NS);
  ADDV("16+8 2col swz1 cap1", 16, 8, 2, 256, 0, 1, lds_for(1), B, B, NS);
  ADDV("16+8 2col T128 swz1 cap2", 16, 8, 2, 128, 0, 1, lds_for(2), B, B, NS);
  ADDV("16+8 2col T128 swz1 cap4", 16, 8, 2, 128, 0, 1, lds_for(4), B, B, NS);
  ADDV("16+8 2col T64 swz1 cap4", 16, 8, 2, 64, 0, 1, lds_for(4), B, B, NS);
  ADDV("16+8 2col T64 swz1 cap8", 16, 8, 2, 64, 0, 1, lds_for(8), B, B, NS);
  ADDV("16+2 base", 16, 2, 1, 256, 0, 0, 0, B, B, NS);
  ADDV("16+2 cap2", 16, 2, 1, 256, 0, 0, lds_for(2), B, B, NS);
  ADDV("16+2 swz1 cap2", 16, 2, 1, 256, 0, 1, lds_for(2), B, B, NS);
  ADDV("16+2 swz1 cap4", 16, 2, 1, 256, 0, 1, lds_for(4), B, B, NS);
  ADDV("32+16 base", 32, 16, 1, 256, 0, 0, 0, M1, M1, 32);
  ADDV("32+16 swz1", 32, 16, 1, 256, 0, 1, 0, M1, M1, 32);
  ADDV("32+16 swz1 cap2", 32, 16, 1, 256, 0, 1, lds_for(2), M1, M1, 32);
  ADDV("32+16 2col swz1 cap2", 32, 16, 2, 256, 0, 1, lds_for(2), M1, M1, 32);
  ADDV("32+16 2col T128 swz1 cap2", 32, 16, 2, 128, 0, 1, lds_for(2), M1, M1, 32);
  ADDV("8+3 B=32K", 8, 3, 1, 256, 0, 0, 0, 32 << 10, 32 << 10, 2048);
  ADDV("8+3 B=32K cap4", 8, 3, 1, 256, 0, 0, lds_for(4), 32 << 10, 32 << 10, 2048);
  ADDV("8+3 B=32K swz1 cap4", 8, 3, 1, 256, 0, 1, lds_for(4), 32 << 10, 32 << 10, 2048);
  ADDV("8+3 B=32K swz3 cap4", 8, 3, 1, 256, 0, 3, lds_for(4), 32 << 10, 32 << 10, 2048);

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
    std::fprintf(stderr, "round %d done\n", r);
  }
  std::printf("wide_probe: %d rounds (median), %d launches per sample, %d CUs\n", rounds, reps,
              ncu);
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    std::printf("%-34s %9.1f us  %7.1f GB/s  (best %7.1f GB/s)\n", v.name.c_str(), med * 1e3,
                v.bytes / (med * 1e-3) / 1e9, v.bytes / (v.ms[0] * 1e-3) / 1e9);
  }
  return 0;
}
