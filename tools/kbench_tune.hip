// kbench_tune.hip -- pick the launch shape (threads T, dwordx4 columns per
// lane U, sched_barrier BAR) of the product kernel rs_apply_perm per (k, r)
// bucket, on the BASELINE shapes:
//   W1  RS(4,2) encode     1024 x 1 MiB   (k=4,  r=2, B=256 KiB)   config 2
//   W2  RS(8,4) decode e=3 4096 x 256 KiB (k=8,  r=3, B=32 KiB)    config 3
//   W3  RS(16,8) encode    128 x 8 MiB    (k=16, r=8, B=512 KiB)   config 5 shape
// Every variant's output is compared bit-exactly with the first variant's;
// timings are interleaved rounds in one process (guide 5.4 rule 24).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../storb_amd/csrc \
//        kbench_tune.hip -o _build/kbench_tune
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "gf256.hpp"
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

struct V {
  std::string name;
  std::function<hipError_t(const ApplyArgs &, hipStream_t)> fn;
  std::vector<float> us;
};

struct W {
  const char *name;
  uint32_t k, r, n_stripes;
  uint64_t B;
  std::vector<V> vs;
  bool inplace = false;  // decode layout of bench --config 3 (see below)
  int order = 0;  // survivor order: 0 index, 1 library slot order (parity in the holes), 2 parity first
  bool copy = false;  // inplace layout, but rebuilt into a separate chunk buffer (fused assembly)
};

template <int KM, int RM, int T, int U, bool BAR, int G, bool TL = false, bool PAIR = false>
V mk() {
  char buf[112];
  std::snprintf(buf, sizeof buf, "<%d,%d> T=%d U=%d BAR=%d G=%d TL=%d PAIR=%d", KM, RM, T, U,
                (int)BAR, G, (int)TL, (int)PAIR);
  return V{buf, [](const ApplyArgs &a, hipStream_t s) {
             return launch_perm<KM, RM, T, U, BAR, G, TL, PAIR>(a, s);
           }, {}};
}

// Occupancy cap: the same kernel launched with dynamic LDS so only
// `wg_per_cu` workgroups fit a CU's 160 KiB (does fewer waves in flight
// stream HBM better? argv[3] = "occ").
template <int KM, int RM, int T, int U, bool BAR, int G, bool TL = false, bool PAIR = false>
V mk_occ(int wg_per_cu) {
  V v = mk<KM, RM, T, U, BAR, G, TL, PAIR>();
  // per-WG LDS (static tables + dynamic) = 160 KiB / n rounded down to 1 KiB:
  // n workgroups fit a CU, n + 1 do not
  const size_t stat = TL ? sizeof(PermTab) * KM * RM : 0;
  const size_t lds = wg_per_cu ? ((160u << 10) / wg_per_cu) / 1024 * 1024 - stat : 0;
  v.name += " wg/CU<=" + std::to_string(wg_per_cu);
  v.fn = [lds](const ApplyArgs &a, hipStream_t s) {
    auto kern = rs_apply_perm<KM, RM, T, U, BAR, G, TL, PAIR>;
    if (lds > (64u << 10)) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         static_cast<int>(lds));
      if (e != hipSuccess) return e;
    }
    const uint64_t cols = a.block >> 4;
    const uint64_t blocks = ((cols + T * U - 1) / (T * U)) * a.nstripes;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(T), lds, s, a);
    return hipGetLastError();
  };
  return v;
}

// Fused-assembly (COPY) kernels under a cap: decode into a separate chunk
// buffer, config 3's assembly leg (argv[3] = "copy").
template <int KM, int RM, int T, bool BAR, int G, bool TL, bool PAIR>
V mk_copy(int wg_per_cu) {
  char buf[112];
  std::snprintf(buf, sizeof buf, "COPY <%d,%d> T=%d G=%d TL=%d PAIR=%d wg/CU<=%d", KM, RM, T, G,
                (int)TL, (int)PAIR, wg_per_cu);
  const size_t stat = TL ? sizeof(PermTab) * KM * RM : 0;
  const size_t lds = wg_per_cu ? ((160u << 10) / wg_per_cu) / 1024 * 1024 - stat : 0;
  return V{buf, [lds](const ApplyArgs &a, hipStream_t s) {
             auto kern = rs_apply_perm<KM, RM, T, 1, BAR, G, TL, PAIR, true>;
             if (lds > (64u << 10)) {
               hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  static_cast<int>(lds));
               if (e != hipSuccess) return e;
             }
             const uint64_t blocks = (((a.block >> 4) + T - 1) / T) * a.nstripes;
             hipLaunchKernelGGL(kern, dim3(blocks), dim3(T), lds, s, a);
             return hipGetLastError();
           }, {}};
}

template <int KM, int RM>
V product() {
  using C = Tune<KM, RM>;
  V v = mk<KM, RM, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>();
  v.name = "product " + v.name;
  return v;
}

template <int KM, int RM>
void add_occ(std::vector<V> &v) {
  using C = Tune<KM, RM>;
  v.push_back(product<KM, RM>());
  for (int n : {0, 2, 3, 4, 5, 6})
    v.push_back(mk_occ<KM, RM, C::T, C::U, C::BAR, C::G, C::TL, C::PAIR>(n));
}

template <int KM, int RM>
void add_all(std::vector<V> &v) {
  constexpr int GM = KM < 8 ? KM : 8;
  v.push_back(product<KM, RM>());
  v.push_back(mk<KM, RM, 256, 1, false, GM, KM >= 8, false>());
  v.push_back(mk<KM, RM, 256, 1, false, GM, KM >= 8, true>());
  v.push_back(mk<KM, RM, 256, 1, true, GM, KM >= 8, true>());
  v.push_back(mk<KM, RM, 256, 1, false, GM, !(KM >= 8), true>());
  v.push_back(mk<KM, RM, 128, 1, false, GM, KM >= 8, true>());
  v.push_back(mk<KM, RM, 256, 2, false, GM, KM >= 8, true>());
  if constexpr (KM >= 8) {
    v.push_back(mk<KM, RM, 256, 1, false, 4, true, true>());
    v.push_back(mk<KM, RM, 256, 1, false, 4, true, false>());
    v.push_back(mk<KM, RM, 128, 1, false, 8, true, false>());
  }
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const int reps = 8;
  std::vector<W> ws = {{"W1 RS(4,2) encode 1024 x 1 MiB", 4, 2, 1024, 256 << 10, {}},
                       {"W2 RS(8,4) decode e=3 4096 x 256 KiB", 8, 3, 4096, 32 << 10, {}},
                       {"W3 RS(16,8) encode 128 x 8 MiB", 16, 8, 128, 512 << 10, {}},
                       {"W2i RS(8,4) decode e=3 in place (bench config 3 layout)", 8, 3, 4096,
                        32 << 10, {}, true},
                       {"W2s RS(8,4) decode e=3 in place, survivors in the library's slot order",
                        8, 3, 4096, 32 << 10, {}, true, 1},
                       {"W2p RS(8,4) decode e=3 in place, parity survivors first",
                        8, 3, 4096, 32 << 10, {}, true, 2}};
  add_all<4, 2>(ws[0].vs);
  add_all<8, 3>(ws[1].vs);
  add_all<16, 8>(ws[2].vs);
  add_all<8, 3>(ws[3].vs);
  ws[3].vs.push_back(mk<8, 4, 256, 1, false, 8, true>());  // previous pow2 bucket
  ws[3].vs.back().name += " (r padded to 4)";
  ws[4].vs.push_back(product<8, 3>());
  ws[5].vs.push_back(product<8, 3>());
  if (argc > 3 && std::strcmp(argv[3], "occ") == 0) {  // occupancy sweep, product shapes
    std::vector<W> o = {ws[0], ws[3], ws[2],
                        {"W5 RS(16,2) decode 128 x 8 MiB (config 5 decode shape)", 16, 2, 128,
                         512 << 10, {}},
                        {"W6 RS(8,4) encode 4096 x 256 KiB", 8, 4, 4096, 32 << 10, {}}};
    for (auto &w : o) w.vs.clear();
    add_occ<4, 2>(o[0].vs);
    for (int n : {8, 9, 10, 11, 12})  // finer caps: 128-lane workgroups
      o[0].vs.push_back(mk_occ<4, 2, 128, 1, false, 4, false, false>(n));
    for (int n : {12, 14, 16, 18, 20, 22, 24})  // one wave per workgroup
      o[0].vs.push_back(mk_occ<4, 2, 64, 1, false, 4, false, false>(n));
    for (int n : {2, 3, 4})  // two columns per lane under a cap
      o[0].vs.push_back(mk_occ<4, 2, 256, 2, false, 4, false, false>(n));
    // round 6: around the one-wave product shape (PermShape<4,2>: T 64, G 4, 14 per CU)
    for (int n : {13, 14})
      o[0].vs.push_back(mk_occ<4, 2, 64, 1, false, 2, false, false>(n));
    for (int n : {13, 14})
      o[0].vs.push_back(mk_occ<4, 2, 64, 1, false, 4, false, true>(n));
    for (int n : {13, 14})
      o[0].vs.push_back(mk_occ<4, 2, 64, 1, true, 4, false, false>(n));
    for (int n : {6, 7, 8})
      o[0].vs.push_back(mk_occ<4, 2, 64, 2, false, 4, false, false>(n));
    for (int n : {2, 3})
      o[0].vs.push_back(mk_occ<4, 2, 512, 1, false, 4, false, false>(n));
    add_occ<8, 3>(o[1].vs);
    for (int n : {0, 8, 10, 12, 16})
      o[1].vs.push_back(mk_occ<8, 3, 128, 1, false, 8, true, true>(n));
    for (int n : {0, 10, 12, 14, 16, 20, 24, 32})
      o[1].vs.push_back(mk_occ<8, 3, 64, 1, false, 8, true, true>(n));
    for (int n : {10, 12, 14, 16})
      o[1].vs.push_back(mk_occ<8, 3, 64, 1, false, 4, true, true>(n));
    for (int n : {0, 3, 4, 5})
      o[1].vs.push_back(mk_occ<8, 3, 256, 1, false, 4, true, true>(n));
    add_occ<16, 8>(o[2].vs);
    add_occ<16, 2>(o[3].vs);
    add_occ<8, 4>(o[4].vs);
    for (int n : {12, 14, 16, 20})  // one-wave workgroups (config 3's <8,3> shape)
      o[4].vs.push_back(mk_occ<8, 4, 64, 1, false, 4, true, true>(n));
    for (int n : {14, 16})
      o[4].vs.push_back(mk_occ<8, 4, 64, 1, false, 8, true, true>(n));
    // round 6: Storb's (2, 3) encode (256 KiB chunks) and single-row rebuilds at k = 4
    o.push_back({"W7 RS(2,1) encode 4096 x 256 KiB (Storb's (2, 3))", 2, 1, 4096, 128 << 10, {}});
    o.push_back({"W8 RS(4,1) one row from 4, 1024 x 1 MiB", 4, 1, 1024, 256 << 10, {}});
    o[5].vs.push_back(product<2, 1>());
    o[6].vs.push_back(product<4, 1>());
    for (int n : {0, 4, 6, 8})
      o[5].vs.push_back(mk_occ<2, 1, 256, 1, false, 2, false, false>(n));
    for (int n : {12, 13, 14, 16, 20, 24, 28, 32, 0})
      o[5].vs.push_back(mk_occ<2, 1, 64, 1, false, 2, false, false>(n));
    for (int n : {12, 14, 16, 0})
      o[5].vs.push_back(mk_occ<2, 1, 128, 1, false, 2, false, false>(n));
    for (int n : {0, 4, 6})
      o[6].vs.push_back(mk_occ<4, 1, 256, 1, false, 4, false, false>(n));
    for (int n : {12, 13, 14, 16, 20, 24})
      o[6].vs.push_back(mk_occ<4, 1, 64, 1, false, 4, false, false>(n));
    ws = o;
    if (argc > 4) ws = {o[std::atoi(argv[4])]};  // one workload of the sweep
  } else if (argc > 3 && std::strcmp(argv[3], "copy") == 0) {
    W c{"W2c RS(8,4) decode e=3 into a separate chunk buffer (config 3 assembly)", 8, 3, 4096,
        32 << 10, {}, true, 0, true};
    for (int n : {0, 3, 4, 5, 6})
      c.vs.push_back(mk_copy<8, 3, 256, false, 8, true, true>(n));
    for (int n : {12, 14, 16, 20, 24})
      c.vs.push_back(mk_copy<8, 3, 64, false, 4, true, true>(n));
    for (int n : {14, 16, 20})
      c.vs.push_back(mk_copy<8, 3, 64, false, 8, true, true>(n));
    for (int n : {6, 8, 10})
      c.vs.push_back(mk_copy<8, 3, 128, false, 4, true, true>(n));
    ws = {c};
  } else if (argc > 2) {
    ws.erase(ws.begin(), ws.begin() + std::atoi(argv[2]));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &w : ws) {
    const uint64_t in_bytes = (uint64_t)w.n_stripes * w.k * w.B;
    const uint64_t out_bytes = (uint64_t)w.n_stripes * w.r * w.B;
    uint8_t *in, *out, *dst = nullptr;
    CK(hipMalloc(&in, in_bytes));
    if (w.copy) CK(hipMalloc(&dst, in_bytes));
    CK(hipMalloc(&out, w.inplace ? (uint64_t)w.n_stripes * 4 * w.B : out_bytes));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, w.k);
    if (w.inplace)  // random "parity" too: zero inputs raise the clock (DVFS)
      hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)out,
                         (uint64_t)w.n_stripes * 4 * w.B / 8, 77);
    // coefficients: enc rows of (k, k+r) -- shape is what matters
    const std::vector<uint8_t> enc = enc_matrix(w.k, w.k + w.r);
    std::vector<PermTab> tabs;
    const uint32_t rp = rows_bucket(w.r);  // [input][rows_bucket(r)], zero padded
    for (uint32_t j = 0; j < w.k; j++)
      for (uint32_t i = 0; i < rp; i++)
        tabs.push_back(i < w.r ? perm_tab(enc[(w.k + i) * w.k + j]) : PermTab{});
    PermTab *dt;
    CK(hipMalloc(&dt, (size_t)w.k * 16 * sizeof(PermTab)));  // room for any padded variant
    CK(hipMemcpy(dt, tabs.data(), tabs.size() * sizeof(PermTab), hipMemcpyHostToDevice));
    ApplyArgs a{};
    a.k = w.k;
    a.r = w.r;
    for (uint32_t j = 0; j < w.k; j++) {
      a.in[j] = in + j * w.B;
      a.in_stride[j] = w.k * w.B;
    }
    for (uint32_t i = 0; i < w.r; i++) {
      a.out[i] = out + i * w.B;
      a.out_stride[i] = w.r * w.B;
    }
    if (w.inplace) {
      // survivors {1,2,4,6,7} from the data region (stride 8B) and parity
      // {8,9,10} from the parity region (stride 4B); rebuilt {0,3,5} written
      // into the data region: exactly decode_batch_dev(..., d_out = d_data).
      // index order, or storb_rs.cpp select_shares' slot order: data share s
      // in slot s, parity shares filling the holes {0, 3, 5}
      const int orders[3][8] = {{1, 2, 4, 6, 7, 8, 9, 10}, {8, 1, 2, 9, 4, 10, 6, 7},
                                {8, 9, 10, 1, 2, 4, 6, 7}};
      const int *surv = orders[w.order];
      const int lost[3] = {0, 3, 5};
      for (int j = 0; j < 8; j++) {
        a.in[j] = surv[j] < 8 ? in + surv[j] * w.B : out + (surv[j] - 8) * w.B;
        a.in_stride[j] = surv[j] < 8 ? 8 * w.B : 4 * w.B;
      }
      for (int i = 0; i < 3; i++) {
        a.out[i] = (w.copy ? dst : in) + lost[i] * w.B;
        a.out_stride[i] = 8 * w.B;
      }
      if (w.copy) {  // the surviving data shares stored to their slots of dst as loaded
        for (int j = 0; j < 8; j++)
          if (surv[j] < 8) {
            a.copy[j] = dst + surv[j] * w.B;
            a.copy_stride[j] = 8 * w.B;
            a.ncopy++;
          }
      }
    }
    a.ptab = dt;
    a.tab_rows = rp;
    a.block = w.B;
    a.nstripes = w.n_stripes;
    std::vector<uint8_t> ref(out_bytes), got(out_bytes);
    for (size_t vi = 0; vi < w.vs.size() && !w.inplace; vi++) {
      CK(hipMemset(out, 0, out_bytes));
      CK(w.vs[vi].fn(a, s));
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(vi ? got.data() : ref.data(), out, out_bytes, hipMemcpyDeviceToHost));
      if (vi && std::memcmp(got.data(), ref.data(), out_bytes)) {
        std::printf("MISMATCH %s %s\n", w.name, w.vs[vi].name.c_str());
        return 2;
      }
    }
    for (int rd = 0; rd < rounds; rd++)
      for (auto &v : w.vs) {
        CK(v.fn(a, s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; i++) CK(v.fn(a, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.us.push_back(ms * 1000.f / reps);
      }
    // COPY: k*B read + k*B written per stripe (the bench's assembly leg)
    const double bytes = w.copy ? 2.0 * in_bytes : (double)in_bytes + out_bytes;
    if (w.copy) {  // every variant bit-exact against the first (the product shape)
      std::vector<uint8_t> r0(in_bytes), r1(in_bytes);
      for (size_t vi = 0; vi < w.vs.size(); vi++) {
        CK(hipMemset(dst, 0, in_bytes));
        CK(w.vs[vi].fn(a, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(vi ? r1.data() : r0.data(), dst, in_bytes, hipMemcpyDeviceToHost));
        if (vi && std::memcmp(r0.data(), r1.data(), in_bytes)) {
          std::printf("MISMATCH %s %s\n", w.name, w.vs[vi].name.c_str());
          return 2;
        }
      }
    }
    std::printf("%s: %.3f GB algorithmic per launch\n", w.name, bytes / 1e9);
    for (auto &v : w.vs) {
      std::sort(v.us.begin(), v.us.end());
      const float med = v.us[v.us.size() / 2];
      std::printf("  %-30s median %8.1f us  min %8.1f us  %7.1f GB/s  %.1f%%\n",
                  v.name.c_str(), med, v.us[0], bytes / med / 1e3, bytes / med / 1e3 / 80.0);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(dt));
    if (dst) CK(hipFree(dst));
  }
  return 0;
}
