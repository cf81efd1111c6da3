// dlprobe.hip -- the HBM ceiling of the download decode's access shape
// (VERDICT r4 item 4): per-stripe records, k inputs read (the present data
// shares in place in the chunk buffer + the first e parity shares), e
// missing data shares written in place, no GF work (inputs XOR-combined, so
// nothing is dead code). The stripes and their lost shares follow the bench
// lines' download mixes:
//   k4:  config 2's shape, 1024 x 1 MiB chunks (B = 256 KiB), the 675 chunks
//        that lost one data share (bench.py --erase-pattern download, seed
//        0x5709B) -- a 4 read : 1 write mix over a scattered subset;
//   k16: config 5's shape, 128 x 8 MiB chunks (B = 512 KiB), 48 / 58 / 9
//        chunks that lost 1 / 2 / 3 data shares -- 16 : 1-3;
//   k32: config 6's shape, 32 x 32 MiB chunks (B = 1 MiB), 14 / 13 / 1 chunks
//        that lost 1 / 2 / 3 data shares -- 32 : 1-3.
// Variants (all moving the same bytes): workgroup size T, 16-B columns per
// lane U, tiles per workgroup, resident-workgroup cap (LDS reservation),
// record read through scalar loads vs computed addresses (a uniform launch
// over contiguous stripes, the ceiling with no records at all). Each sample
// times `reps` back-to-back launches; interleaved rounds, median.
//
// build: make -C tools dlprobe   run: tools/_build/dlprobe [rounds] [reps] [k4|k16|k32]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
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
typedef const uint64_t __attribute__((address_space(4))) cu64;

constexpr int kMaxK = 32, kMaxR = 4;
// One item: r (low 32 bits of q[0] >> 32), k input pointers, kMaxR outputs.
constexpr int kRecQ = 1 + kMaxK + kMaxR;

struct Args {
  const uint64_t *rec;
  uint32_t k;
  uint32_t cols;  // 16-B columns per share
  uint32_t tpw;   // tiles per workgroup
};

__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

template <int K, int R, int T, int U>
__device__ __forceinline__ void tile(cu64 *q, uint32_t c0) {
  u32x4 acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) acc[u] = u32x4{0, 0, 0, 0};
  u32x4 v[K][U];
#pragma unroll
  for (int j = 0; j < K; j++) {
    const uint8_t *p = reinterpret_cast<const uint8_t *>(q[1 + j]);
#pragma unroll
    for (int u = 0; u < U; u++) v[j][u] = ld(p + (static_cast<uint64_t>(c0) + u * T) * 16);
  }
#pragma unroll
  for (int j = 0; j < K; j++)
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] ^= v[j][u];
#pragma unroll
  for (int i = 0; i < R; i++) {
    uint8_t *p = reinterpret_cast<uint8_t *>(q[1 + kMaxK + i]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      u32x4 o = acc[u];
      o.x ^= i;
      st(p + (static_cast<uint64_t>(c0) + u * T) * 16, o);
    }
  }
}

// Mixed row counts, records read with scalar loads (as rs_apply_desc_mix).
template <int K, int T, int U>
__global__ __launch_bounds__(T) void dl_mix(const Args a) {
  const uint32_t tiles = a.cols / (T * U);
  const uint32_t wpi = (tiles + a.tpw - 1) / a.tpw;
  const uint32_t item = blockIdx.x / wpi;
  const uint32_t t0 = (blockIdx.x - item * wpi) * a.tpw;
  cu64 *q = (cu64 *)(a.rec) + static_cast<uint64_t>(item) * kRecQ;
  const uint32_t r = static_cast<uint32_t>(q[0] >> 32);
  for (uint32_t t = t0; t < t0 + a.tpw && t < tiles; t++) {
    const uint32_t c0 = t * T * U + threadIdx.x;
    if (r <= 1)
      tile<K, 1, T, U>(q, c0);
    else if (r == 2)
      tile<K, 2, T, U>(q, c0);
    else if (r == 3)
      tile<K, 3, T, U>(q, c0);
    else
      tile<K, 4, T, U>(q, c0);
  }
}

// Persistent: gridDim.x workgroups (cap x CUs), each striding over the
// launch's tiles in order, so the resident set always covers a contiguous
// run of tiles and no workgroup is dispatched twice.
template <int K, int T, int U>
__global__ __launch_bounds__(T) void dl_persist(const Args a, uint32_t total) {
  const uint32_t tiles = a.cols / (T * U);
  for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
    const uint32_t item = g / tiles, t = g - item * tiles;
    cu64 *q = (cu64 *)(a.rec) + static_cast<uint64_t>(item) * kRecQ;
    const uint32_t r = static_cast<uint32_t>(q[0] >> 32);
    const uint32_t c0 = t * T * U + threadIdx.x;
    if (r <= 1)
      tile<K, 1, T, U>(q, c0);
    else if (r == 2)
      tile<K, 2, T, U>(q, c0);
    else if (r == 3)
      tile<K, 3, T, U>(q, c0);
    else
      tile<K, 4, T, U>(q, c0);
  }
}

// The uniform reference: contiguous stripes, addresses computed (k inputs
// then r outputs per stripe, each B bytes), no record.
template <int K, int R, int T>
__global__ __launch_bounds__(T) void dl_uniform(uint8_t *base, uint32_t cols) {
  const uint32_t tiles = cols / T;
  const uint32_t s = blockIdx.x / tiles, t = blockIdx.x % tiles;
  const uint64_t B = static_cast<uint64_t>(cols) * 16;
  uint8_t *p = base + static_cast<uint64_t>(s) * (K + R) * B;
  const uint64_t off = (static_cast<uint64_t>(t) * T + threadIdx.x) * 16;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 v[K];
#pragma unroll
  for (int j = 0; j < K; j++) v[j] = ld(p + j * B + off);
#pragma unroll
  for (int j = 0; j < K; j++) acc ^= v[j];
#pragma unroll
  for (int i = 0; i < R; i++) {
    u32x4 o = acc;
    o.x ^= i;
    st(p + (K + i) * B + off, o);
  }
}

struct Variant {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

static size_t cap_lds(int cap) { return cap > 0 ? (160u << 10) / cap / 1024 * 1024 : 0; }

template <auto Kern, class... A>
static void launch(uint32_t blocks, int T, size_t dyn, hipStream_t s, A... a) {
  if (dyn > (64u << 10))
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(Kern),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)));
  hipLaunchKernelGGL(Kern, dim3(blocks), dim3(T), dyn, s, a...);
}

struct Shape {
  const char *name;
  uint32_t k, n, nchunks;
  uint64_t B;
  std::vector<int> lost_hist;  // lost_hist[e] chunks lost e data shares
};

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 8;
  std::vector<Shape> shapes = {{"k4", 4, 6, 1024, 256u << 10, {349, 675}},
                               {"k16", 16, 24, 128, 512u << 10, {13, 48, 58, 9}},
                               {"k32", 32, 48, 32, 1u << 20, {4, 14, 13, 1}}};
  const char *only = argc > 3 ? argv[3] : nullptr;  // run one shape
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  if (only && std::string(only) == "c3") {
    // config 3's decode shape with no GF work: RS(8,4) decode of 3 rows, 8
    // in + 3 out, 4096 contiguous stripes of 32 KiB shares, over workgroup
    // sizes and caps (the product: rs_apply_perm<8,3> T=256 cap 4, 0.80)
    const uint64_t B = 32u << 10, ns = 4096, bytes = ns * 11 * B;
    const uint32_t cols = static_cast<uint32_t>(B / 16);
    uint8_t *u;
    CK(hipMalloc(&u, bytes));
    CK(hipMemset(u, 0x44, bytes));
    std::vector<Variant> vs;
    auto add83 = [&](int T, int cap) {
      const uint32_t blocks = static_cast<uint32_t>(ns * (cols / T));
      vs.push_back(Variant{"config3 8+3 T=" + std::to_string(T) + " cap=" + std::to_string(cap),
                           static_cast<double>(bytes),
                           [=](hipStream_t st) {
                             if (T == 256)
                               launch<dl_uniform<8, 3, 256>>(blocks, 256, cap_lds(cap), st, u, cols);
                             else if (T == 128)
                               launch<dl_uniform<8, 3, 128>>(blocks, 128, cap_lds(cap), st, u, cols);
                             else
                               launch<dl_uniform<8, 3, 64>>(blocks, 64, cap_lds(cap), st, u, cols);
                           },
                           {}});
    };
    for (int cap : {0, 2, 3, 4, 5, 6, 8}) add83(256, cap);
    for (int cap : {0, 6, 8, 10, 12}) add83(128, cap);
    for (int cap : {0, 12, 16, 20, 24}) add83(64, cap);
    for (auto &v : vs) v.run(s);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; r++)
      for (auto &v : vs) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; i++) v.run(s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms / reps);
      }
    std::printf("c3: 4096 x (8 + 3) x 32 KiB contiguous, %.1f MB per launch, %d rounds x %d launches\n",
                bytes / 1e6, rounds, reps);
    for (auto &v : vs) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      std::printf("  %-46s %8.1f us  %7.1f GB/s  frac %.3f (best %.3f)\n", v.name.c_str(),
                  med * 1e3, v.bytes / (med * 1e-3) / 1e9, v.bytes / (med * 1e-3) / 8e12,
                  v.bytes / (v.ms[0] * 1e-3) / 8e12);
    }
    CK(hipFree(u));
    return 0;
  }
  for (const Shape &sh : shapes) {
    if (only && std::string(only) != sh.name) continue;
    const uint64_t chunk = sh.k * sh.B;
    uint8_t *data, *par, *uni;
    CK(hipMalloc(&data, sh.nchunks * chunk));
    CK(hipMalloc(&par, sh.nchunks * (sh.n - sh.k) * sh.B));
    CK(hipMemset(data, 0x3c, sh.nchunks * chunk));
    CK(hipMemset(par, 0x5a, sh.nchunks * (sh.n - sh.k) * sh.B));
    // items: chunks in order, each with its lost set (seeded), as the bench
    std::mt19937_64 rng(0x5709B);
    std::vector<int> e_of;
    for (size_t e = 0; e < sh.lost_hist.size(); e++)
      for (int c = 0; c < sh.lost_hist[e]; c++) e_of.push_back(static_cast<int>(e));
    std::shuffle(e_of.begin(), e_of.end(), rng);
    std::vector<uint64_t> rec;
    double bytes = 0;
    uint32_t nitems = 0, rows_total = 0;
    for (uint32_t c = 0; c < sh.nchunks; c++) {
      const int e = e_of[c];
      if (e == 0) continue;
      std::vector<uint32_t> ids(sh.k);
      for (uint32_t j = 0; j < sh.k; j++) ids[j] = j;
      std::shuffle(ids.begin(), ids.end(), rng);
      std::vector<uint32_t> lost(ids.begin(), ids.begin() + e);
      std::sort(lost.begin(), lost.end());
      std::vector<uint64_t> q(kRecQ, 0);
      q[0] = static_cast<uint64_t>(e) << 32;
      uint32_t slot = 0, p = 0;
      for (uint32_t j = 0; j < sh.k; j++)  // present data shares, then parity 0.. in the lost slots
        if (!std::binary_search(lost.begin(), lost.end(), j))
          q[1 + slot++] = reinterpret_cast<uint64_t>(data + c * chunk + j * sh.B);
      while (slot < sh.k)
        q[1 + slot++] =
            reinterpret_cast<uint64_t>(par + (static_cast<uint64_t>(c) * (sh.n - sh.k) + p++) * sh.B);
      for (int i = 0; i < e; i++)
        q[1 + kMaxK + i] = reinterpret_cast<uint64_t>(data + c * chunk + lost[i] * sh.B);
      rec.insert(rec.end(), q.begin(), q.end());
      bytes += static_cast<double>(sh.k + e) * sh.B;
      nitems++;
      rows_total += e;
    }
    uint64_t *drec;
    CK(hipMalloc(&drec, rec.size() * 8));
    CK(hipMemcpy(drec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice));
    const uint32_t cols = static_cast<uint32_t>(sh.B / 16);
    std::vector<Variant> vs;
    auto add_mix = [&](const std::string &nm, auto kern, int T, int U, uint32_t tpw, int cap) {
      const uint32_t tiles = cols / (T * U);
      const uint32_t blocks = (tiles + tpw - 1) / tpw * nitems;
      Args a{drec, sh.k, cols, tpw};
      const size_t dyn = cap_lds(cap);
      vs.push_back(Variant{nm + " T=" + std::to_string(T) + " U=" + std::to_string(U) + " tpw=" +
                               std::to_string(tpw) + " cap=" + std::to_string(cap),
                           bytes, [=](hipStream_t st) { kern(blocks, T, dyn, st, a); }, {}});
    };
    auto add_persist = [&](int K, int T, int per_cu) {
      const uint32_t tiles = cols / T, total = tiles * nitems;
      const uint32_t grid = std::min<uint32_t>(total, 256u * per_cu);
      Args a{drec, sh.k, cols, 1};
      const size_t dyn = cap_lds(per_cu);
      vs.push_back(Variant{"persistent T=" + std::to_string(T) + " wg/CU=" + std::to_string(per_cu),
                           bytes,
                           [=](hipStream_t st) {
                             if (K == 4)
                               launch<dl_persist<4, 256, 1>>(grid, T, dyn, st, a, total);
                             else if (K == 16)
                               launch<dl_persist<16, 256, 1>>(grid, T, dyn, st, a, total);
                             else
                               launch<dl_persist<32, 256, 1>>(grid, T, dyn, st, a, total);
                           },
                           {}});
    };
    for (int pc : {2, 4, 6, 8}) add_persist(static_cast<int>(sh.k), 256, pc);
#define MIX(K, T, U)                                                                    \
  [](uint32_t b, int t, size_t d, hipStream_t st, Args a) {                             \
    launch<dl_mix<K, T, U>>(b, t, d, st, a);                                            \
  }
    if (sh.k == 4) {
      for (int cap : {0, 2, 3, 4, 5, 6, 8}) add_mix("mix", MIX(4, 256, 1), 256, 1, 1, cap);
      for (int cap : {0, 4}) add_mix("mix", MIX(4, 256, 2), 256, 2, 1, cap);
      for (int cap : {0, 8, 12, 16}) add_mix("mix", MIX(4, 128, 1), 128, 1, 1, cap);
      for (int cap : {0, 16, 24}) add_mix("mix", MIX(4, 64, 1), 64, 1, 1, cap);
      for (uint32_t tpw : {2u, 4u, 8u})
        for (int cap : {0, 4}) add_mix("mix", MIX(4, 256, 1), 256, 1, tpw, cap);
      // uniform ceiling: contiguous stripes of 4 in + 1 out, same bytes
      CK(hipMalloc(&uni, static_cast<uint64_t>(nitems) * 5 * sh.B));
      CK(hipMemset(uni, 0x11, static_cast<uint64_t>(nitems) * 5 * sh.B));
      // the headline encode's shape (RS(4,2): 4 in + 2 out, 1024 contiguous
      // stripes) over workgroup sizes and caps, for the table kernel's shape
      {
        uint8_t *u42;
        const uint64_t ns42 = 1024, bytes42 = ns42 * 6 * sh.B;
        CK(hipMalloc(&u42, bytes42));
        CK(hipMemset(u42, 0x22, bytes42));
        auto add42 = [&](int T, int cap) {
          const uint32_t blocks = static_cast<uint32_t>(ns42 * (cols / T));
          vs.push_back(Variant{"encode-shape 4+2 T=" + std::to_string(T) + " cap=" + std::to_string(cap),
                               static_cast<double>(bytes42),
                               [=](hipStream_t st) {
                                 if (T == 256)
                                   launch<dl_uniform<4, 2, 256>>(blocks, 256, cap_lds(cap), st, u42, cols);
                                 else if (T == 128)
                                   launch<dl_uniform<4, 2, 128>>(blocks, 128, cap_lds(cap), st, u42, cols);
                                 else
                                   launch<dl_uniform<4, 2, 64>>(blocks, 64, cap_lds(cap), st, u42, cols);
                               },
                               {}});
        };
        for (int cap : {0, 4, 5}) add42(256, cap);
        for (int cap : {0, 8, 10}) add42(128, cap);
        for (int cap : {0, 12, 16, 20}) add42(64, cap);
      }
      for (int cap : {0, 4})
        vs.push_back(Variant{"uniform contiguous 4+1 T=256 cap=" + std::to_string(cap),
                             static_cast<double>(nitems) * 5 * sh.B,
                             [=](hipStream_t st) {
                               launch<dl_uniform<4, 1, 256>>(nitems * (cols / 256), 256,
                                                             cap_lds(cap), st, uni, cols);
                             },
                             {}});
    } else if (sh.k == 32) {
      for (int cap : {0, 2, 3, 4}) add_mix("mix", MIX(32, 256, 1), 256, 1, 1, cap);
      for (int cap : {0, 4, 6, 8}) add_mix("mix", MIX(32, 128, 1), 128, 1, 1, cap);
      for (int cap : {0, 8, 12, 16}) add_mix("mix", MIX(32, 64, 1), 64, 1, 1, cap);
      const uint64_t per = 34ull * sh.B;  // 32 + 2, the mix's mean rows
      CK(hipMalloc(&uni, static_cast<uint64_t>(nitems) * per));
      CK(hipMemset(uni, 0x11, static_cast<uint64_t>(nitems) * per));
      for (int cap : {0, 3})
        vs.push_back(Variant{"uniform contiguous 32+2 T=256 cap=" + std::to_string(cap),
                             static_cast<double>(nitems) * per,
                             [=](hipStream_t st) {
                               launch<dl_uniform<32, 2, 256>>(nitems * (cols / 256), 256,
                                                              cap_lds(cap), st, uni, cols);
                             },
                             {}});
    } else {
      for (int cap : {0, 2, 3, 4, 6}) add_mix("mix", MIX(16, 256, 1), 256, 1, 1, cap);
      for (int cap : {0, 4, 6, 8}) add_mix("mix", MIX(16, 128, 1), 128, 1, 1, cap);
      for (int cap : {0, 8, 12, 16}) add_mix("mix", MIX(16, 64, 1), 64, 1, 1, cap);
      for (uint32_t tpw : {2u, 4u})
        for (int cap : {0, 3}) add_mix("mix", MIX(16, 256, 1), 256, 1, tpw, cap);
      // the (32, 48) encode's access shape (32 in + 16 out, 1 MiB shares, 32
      // contiguous stripes: config 6), over workgroup sizes and caps
      {
        uint8_t *u3216;
        const uint64_t B32 = 1u << 20, ns32 = 32, bytes32 = ns32 * 48 * B32;
        const uint32_t cols32 = static_cast<uint32_t>(B32 / 16);
        CK(hipMalloc(&u3216, bytes32));
        CK(hipMemset(u3216, 0x33, bytes32));
        auto add3216 = [&](int T, int cap) {
          const uint32_t blocks = static_cast<uint32_t>(ns32 * (cols32 / T));
          vs.push_back(Variant{"encode-shape 32+16 T=" + std::to_string(T) + " cap=" + std::to_string(cap),
                               static_cast<double>(bytes32),
                               [=](hipStream_t st) {
                                 if (T == 256)
                                   launch<dl_uniform<32, 16, 256>>(blocks, 256, cap_lds(cap), st, u3216, cols32);
                                 else if (T == 128)
                                   launch<dl_uniform<32, 16, 128>>(blocks, 128, cap_lds(cap), st, u3216, cols32);
                                 else
                                   launch<dl_uniform<32, 16, 64>>(blocks, 64, cap_lds(cap), st, u3216, cols32);
                               },
                               {}});
        };
        for (int cap : {0, 2, 3, 4}) add3216(256, cap);
        for (int cap : {0, 4, 6, 8}) add3216(128, cap);
        for (int cap : {0, 8, 12, 16}) add3216(64, cap);
      }
      const uint64_t per = 18ull * sh.B;  // 16 + 2, the mix's mean rows
      CK(hipMalloc(&uni, static_cast<uint64_t>(nitems) * per));
      CK(hipMemset(uni, 0x11, static_cast<uint64_t>(nitems) * per));
      for (int cap : {0, 3})
        vs.push_back(Variant{"uniform contiguous 16+2 T=256 cap=" + std::to_string(cap),
                             static_cast<double>(nitems) * per,
                             [=](hipStream_t st) {
                               launch<dl_uniform<16, 2, 256>>(nitems * (cols / 256), 256,
                                                              cap_lds(cap), st, uni, cols);
                             },
                             {}});
    }
#undef MIX
    for (auto &v : vs) v.run(s);  // warm
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; r++)
      for (auto &v : vs) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; i++) v.run(s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms / reps);
      }
    std::printf("%s: %u items (%u rows), B = %llu KiB, %.1f MB per launch, %d rounds x %d launches\n",
                sh.name, nitems, rows_total, static_cast<unsigned long long>(sh.B >> 10),
                bytes / 1e6, rounds, reps);
    for (auto &v : vs) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      std::printf("  %-46s %8.1f us  %7.1f GB/s  frac %.3f (best %.3f)\n", v.name.c_str(),
                  med * 1e3, v.bytes / (med * 1e-3) / 1e9, v.bytes / (med * 1e-3) / 8e12,
                  v.bytes / (v.ms[0] * 1e-3) / 8e12);
    }
    CK(hipFree(drec));
    CK(hipFree(uni));
    CK(hipFree(data));
    CK(hipFree(par));
  }
  return 0;
}
