// mixbench.hip -- the mixed-row descriptor decode kernel (rs_apply_desc_mix)
// against variants of where a workgroup gets its row count and its tables.
//
// Workload: a download's chunks, each with its own survivor set (download.rs
// :363-451 keeps the first k + 1 pieces to arrive; piece.rs:368-381 sorts and
// takes the first k): BASELINE config 5's geometry (128 x 8 MiB chunks,
// k = 16, B = 512 KiB; 13 / 48 / 58 / 9 chunks lost 0 / 1 / 2 / 3 data
// shares) or, with K = 32, config 6's (32 x 32 MiB, k = 32, B = 1 MiB;
// 4 / 14 / 13 / 1). Random coefficients per chunk (performance only; every
// variant's output is compared byte for byte with the product kernel's).
//
// The product kernel's workgroup does: s_load rec[0] (table offset | rows)
// -> branch on rows -> load its pattern's tables from global memory into LDS
// -> barrier -> first share loads. Variants:
//   noTL      the tables read with scalar loads where they are used (no LDS
//             staging, no barrier), offset still from rec[0];
//   sorted    items ordered by row count; a workgroup's count comes from the
//             launch arguments (blockIdx against per-count boundaries), so
//             nothing waits for rec[0] before the branch;
//   inline    the item's tables inside its record, at a fixed offset: the
//             pointer loads and the table loads issue together;
//   G         shares per load group.
// Bytes = sum over chunks with e > 0 of (k + e) * B.
//
// build: make -C tools mixbench
// usage: mixbench [REPS] [K]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <type_traits>
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

struct Bounds {
  uint32_t first[kMixR + 2];  // first workgroup of the items with r rows (sorted launches)
  uint32_t tab_q;             // qword offset of the inline tables in a record
};

typedef const PermTab __attribute__((address_space(4))) cPermTab;

// Shares per load group of the branch with R rows: GSET 0 = G everywhere;
// 1 = k = 32 {16, 16, 2, 4} / k = 16 {8, 8, 4, 4}; 2 = k = 32 {16, 16, 4, 4}
// / k = 16 {16, 8, 8, 8}.
template <int KM, int G, int GSET>
constexpr int gsel(int R) {
  if (GSET == 1) return KM == 32 ? (R <= 2 ? 16 : R == 3 ? 2 : 4) : (R <= 2 ? 8 : 4);
  if (GSET == 2) return KM == 32 ? (R <= 2 ? 16 : 4) : (R == 1 ? 16 : 8);
  return G;
}

template <int KM, int R, int G, bool TL, bool INL, int U = 1, bool PAIR = false>
__device__ __forceinline__ void vbody(const DescArgs &a, const Bounds &b, cu64 *rec,
                                      PermTab *lds) {
  constexpr uint32_t TILE = kThreads * U;
  const uint32_t cols = static_cast<uint32_t>(a.block >> 4);
  const uint32_t tps = (cols + TILE - 1) / TILE;
  const uint32_t t = blockIdx.x % tps;
  cPermTab *gt = INL ? (cPermTab *)(rec + b.tab_q) : (cPermTab *)(a.ptab) + (rec[0] & 0xFFFFFFFFu);
  const DescView v{rec, a.k, a.r};
  const uint32_t base = t * TILE;
  auto go = [&](auto tabs) {
    if (base + TILE <= cols)
      perm_tile<KM, R, kThreads, U, false, G, PAIR, false, false>(v, tabs, a.k, R, cols,
                                                                base + threadIdx.x);
    else
      perm_tile<KM, R, kThreads, U, false, G, PAIR, true, false>(v, tabs, a.k, R, cols,
                                                               base + threadIdx.x);
  };
  if constexpr (TL) {
    typedef const u32x4 __attribute__((address_space(1))) gcu32x4;
    const uint32_t n16 = a.k * R * (sizeof(PermTab) / 16);
    for (uint32_t i = threadIdx.x; i < n16; i += kThreads)
      reinterpret_cast<u32x4 *>(lds)[i] = ((gcu32x4 *)(gt))[i];
    __syncthreads();
    go(static_cast<const PermTab *>(lds));
  } else {
    go(gt);
  }
}

// Paired inputs per branch: PSET 0 none, 1 all, 2 R <= 3, 3 R <= 2, 4 R != 2,
// 5 R >= 3, 6 R == 1.
constexpr bool psel(int PSET, int R) {
  return PSET == 1 || (PSET == 2 && R <= 3) || (PSET == 3 && R <= 2) || (PSET == 4 && R != 2) ||
         (PSET == 5 && R >= 3) || (PSET == 6 && R == 1);
}

template <int KM, int G, bool TL, bool SORTED, bool INL, int U = 1, int GSET = 0,
          int PSET = 0>
__global__ __launch_bounds__(kThreads) void mixv(const DescArgs a, const Bounds b) {
  __shared__ __attribute__((aligned(16))) PermTab lds[TL ? KM * kMixR : 1];
  const uint32_t tps = (static_cast<uint32_t>(a.block >> 4) + kThreads * U - 1) / (kThreads * U);
  const uint32_t item = blockIdx.x / tps;
  cu64 *rec = (cu64 *)(a.desc) + static_cast<uint64_t>(item) * a.rec_qwords;
  uint32_t r;
  if constexpr (SORTED)
    r = blockIdx.x >= b.first[4] ? 4 : blockIdx.x >= b.first[3] ? 3 : blockIdx.x >= b.first[2] ? 2 : 1;
  else
    r = static_cast<uint32_t>(rec[0] >> 32);
  if (r <= 1) return vbody<KM, 1, gsel<KM, G, GSET>(1), TL, INL, U, psel(PSET, 1)>(a, b, rec, lds);
  if (r == 2) return vbody<KM, 2, gsel<KM, G, GSET>(2), TL, INL, U, psel(PSET, 2)>(a, b, rec, lds);
  if (r == 3) return vbody<KM, 3, gsel<KM, G, GSET>(3), TL, INL, U, psel(PSET, 3)>(a, b, rec, lds);
  return vbody<KM, 4, gsel<KM, G, GSET>(4), TL, INL, U, psel(PSET, 4)>(a, b, rec, lds);
}

struct Var {
  std::string name;
  bool sorted, inl;  // sorted: ascending row count, r from the launch arguments
  std::function<hipError_t(const DescArgs &, const Bounds &, hipStream_t)> fn;
  std::vector<float> ms;
  int U = 1;
  bool heavy_first = false;  // records ordered by descending row count (r still from rec[0])
};

template <int KM, int G, bool TL, bool SORTED, bool INL, int U = 1, int GSET = 0,
          int PSET = 0>
Var mk(const char *name, int cap) {
  return {name, SORTED, INL, [cap](const DescArgs &a, const Bounds &b, hipStream_t s) {
            const uint64_t tps = ((a.block >> 4) + kThreads * U - 1) / (kThreads * U);
            const size_t dyn = cap_lds(cap, TL ? sizeof(PermTab) * KM * kMixR : 0);
            return launch_lds<mixv<KM, G, TL, SORTED, INL, U, GSET, PSET>>(tps * a.nitems, kThreads,
                                                                           dyn, s, a, b);
          }, {}, U};
}

template <int KM>
std::vector<Var> variants() {
  std::vector<Var> v;
  v.push_back({"product rs_apply_desc_mix", false, false,
               [](const DescArgs &a, const Bounds &, hipStream_t s) { return launch_apply_desc(a, s); },
               {}});
  {
    Var h{"product kernel, heaviest items first", false, false,
          [](const DescArgs &a, const Bounds &, hipStream_t s) { return launch_apply_desc(a, s); },
          {}};
    h.heavy_first = true;
    v.push_back(h);
  }
  // input-split tiles (rs_device.hpp rs_apply_desc_mix_ks): W waves x cap
  auto ks = [&](auto WC, int cap, bool heavy) {
    constexpr int W = decltype(WC)::value;
    Var x{"input-split W=" + std::to_string(W) + " cap=" + std::to_string(cap) +
              (heavy ? " heavy first" : ""), false, false,
          [cap](const DescArgs &a, const Bounds &, hipStream_t s) {
            return launch_desc_mix_ks<KM, W>(a, s, cap);
          },
          {}};
    x.heavy_first = heavy;
    v.push_back(x);
  };
  // round 6: the caps around 14 waves per CU (the table kernel's best, rs_device.hpp
  // PermShape), records heaviest first as apply_desc orders them
  for (int cap : {0, 5, 6, 7, 8, 10}) ks(std::integral_constant<int, 2>{}, cap, true);
  for (int cap : {0, 3, 4, 5}) ks(std::integral_constant<int, 4>{}, cap, true);
  if constexpr (KM == 32)
    for (int cap : {2, 3}) ks(std::integral_constant<int, 8>{}, cap, true);
  constexpr int GP = Tune<KM, 1>::G;  // the product's group size
  v.push_back(mk<KM, GP, true, false, false>("same shape here (TL, rec[0])", 0));
  if constexpr (KM == 16) {
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 1>("G8 PAIR all", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 2>("G8 PAIR R<=3", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 3>("G8 PAIR R<=2", 0));
    v.push_back(mk<KM, 4, true, false, false, 1, 0, 1>("G4 PAIR all", 0));
    v.push_back(mk<KM, 4, true, false, false, 1, 0, 2>("G4 PAIR R<=3", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 1, 1>("GSET1 PAIR all", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 4>("G8 PAIR R!=2", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 5>("G8 PAIR R>=3", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 6>("G8 PAIR R==1", 0));
    v.push_back(mk<KM, 8, true, false, false, 1, 0, 1>("G8 PAIR all (again)", 0));
  } else {
    v.push_back(mk<KM, 16, true, false, false>("G16 (TL, rec[0])", 0));
    v.push_back(mk<KM, 16, true, false, false>("G16 cap3", 3));
    v.push_back(mk<KM, 16, true, false, false, 1, 0, 3>("G16 cap3 PAIR R<=2", 3));
  }
  return v;
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

template <int KM, int R>
int isolate(int reps, const std::vector<uint32_t> &es, uint32_t N, uint32_t k, uint32_t n,
            size_t B, uint8_t *d, uint8_t *p, uint8_t *o, size_t ob, hipStream_t s, hipEvent_t e0,
            hipEvent_t e1, std::mt19937 &rng, double &t_uni_sum, double &t_mix_sum) {
  uint32_t M = 0;
  for (uint32_t s2 = 0; s2 < N; s2++) M += es[s2] == R;
  if (!M) return 0;
  std::vector<PermTab> tabs(k * R);
  for (auto &t : tabs) t = perm_tab(uint8_t(rng() | 1));
  PermTab *dtab;
  CK(hipMalloc(&dtab, tabs.size() * sizeof(PermTab)));
  CK(hipMemcpy(dtab, tabs.data(), tabs.size() * sizeof(PermTab), hipMemcpyHostToDevice));
  // the uniform launch needs equally spaced stripes: the first M stripes
  auto slot_id = [&](uint32_t c) { return c < R ? k + c : c; };  // slots 0..R-1 <- parity
  std::vector<uint64_t> rec;
  for (uint32_t q = 0; q < M; q++) {
    rec.push_back(0 | (uint64_t(R) << 32));
    for (uint32_t c = 0; c < k; c++) {
      const uint32_t id = slot_id(c);
      rec.push_back(reinterpret_cast<uint64_t>(id < k ? d + q * k * B + id * B
                                                      : p + q * (n - k) * B + (id - k) * B));
    }
    for (uint32_t i = 0; i < kMixR; i++)
      rec.push_back(i < R ? reinterpret_cast<uint64_t>(o + (size_t(q) * kMixR + i) * B) : 0);
  }
  uint64_t *drec;
  CK(hipMalloc(&drec, rec.size() * 8));
  CK(hipMemcpy(drec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice));
  DescArgs da{};
  da.desc = drec;
  da.ptab = dtab;
  da.block = B;
  da.k = k;
  da.r = kMixR;
  da.tpw = 1;
  da.nitems = M;
  da.rec_qwords = 1 + k + kMixR;
  da.mix = 1;
  ApplyArgs aa{};
  for (uint32_t c = 0; c < k; c++) {
    const uint32_t id = slot_id(c);
    aa.in[c] = id < k ? d + id * B : p + (id - k) * B;
    aa.in_stride[c] = id < k ? k * B : (n - k) * B;
  }
  for (uint32_t i = 0; i < R; i++) {
    aa.out[i] = o + i * B;
    aa.out_stride[i] = kMixR * B;
  }
  aa.ptab = dtab;
  aa.k = k;
  aa.r = R;
  aa.tab_rows = R;
  aa.block = B;
  aa.nstripes = M;
  using C2 = Tune<KM, R>;
  auto uni = [&](int cap) {
    return launch_perm<KM, R, C2::T, C2::U, C2::BAR, C2::G, C2::TL, C2::PAIR>(aa, s, cap);
  };
  struct Iso {
    const char *name;
    std::function<hipError_t()> fn;
    std::vector<float> ms;
  };
  std::vector<Iso> iso = {
      {"mixed-row kernel (records)", [&] { return launch_apply_desc(da, s); }, {}},
      {"uniform rs_apply_perm, tuned cap", [&] { return uni(C2::OCC); }, {}},
      {"uniform rs_apply_perm, uncapped", [&] { return uni(0); }, {}},
  };
  std::vector<uint8_t> w2(ob), g2(ob);
  for (size_t vi = 0; vi < iso.size(); vi++) {
    CK(hipMemsetAsync(o, 0xEE, ob, s));
    CK(iso[vi].fn());
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? g2.data() : w2.data(), o, ob, hipMemcpyDeviceToHost));
    if (vi && std::memcmp(w2.data(), g2.data(), ob) != 0) {
      std::printf("isolation R=%d %s: MISMATCH\n", R, iso[vi].name);
      return 1;
    }
  }
  for (int r = 0; r < reps; r++)
    for (auto &v : iso) {
      CK(hipEventRecord(e0, s));
      CK(v.fn());
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float x = 0;
      CK(hipEventElapsedTime(&x, e0, e1));
      v.ms.push_back(x);
    }
  const double b2 = double(M) * (k + R) * B;
  for (size_t vi = 0; vi < iso.size(); vi++) {
    auto &v = iso[vi];
    std::sort(v.ms.begin(), v.ms.end());
    const float m = v.ms[v.ms.size() / 2];
    if (vi == 0) t_mix_sum += m;
    if (vi == 2) t_uni_sum += m;
    std::printf("k=%u R=%d subset (%u stripes): %-34s %8.4f ms  %6.2f TB/s  %5.1f %%  (bit-exact)\n",
                k, R, M, v.name, m, b2 / (m * 1e-3) / 1e12, 100.0 * b2 / (m * 1e-3) / 8e12);
  }
  CK(hipFree(drec));
  CK(hipFree(dtab));
  return 0;
}

template <int KM>
int run(int reps) {
  const bool c6 = KM == 32;
  const uint32_t k = KM, n = k + k / 2, N = c6 ? 32 : 128;
  const size_t B = c6 ? (1u << 20) : (512u << 10);
  const int hist[4] = {c6 ? 4 : 13, c6 ? 14 : 48, c6 ? 13 : 58, c6 ? 1 : 9};
  uint8_t *d, *p, *o;
  CK(hipMalloc(&d, size_t(N) * k * B));
  CK(hipMalloc(&p, size_t(N) * (n - k) * B));
  CK(hipMalloc(&o, size_t(N) * kMixR * B));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(d),
                     size_t(N) * k * B / 8, 11);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(p),
                     size_t(N) * (n - k) * B / 8, 12);
  CK(hipDeviceSynchronize());
  std::mt19937 rng(5);
  std::vector<uint32_t> es;
  for (uint32_t e = 0; e < 4; e++)
    for (int i = 0; i < hist[e]; i++) es.push_back(e);
  std::shuffle(es.begin(), es.end(), rng);
  // items (chunks with e > 0) in chunk order, and sorted by e
  struct Item {
    uint32_t s, e;
    std::vector<uint64_t> in;
    std::vector<PermTab> tabs;  // [j * e + i]
  };
  std::vector<Item> items;
  double bytes = 0;
  for (uint32_t s = 0; s < N; s++) {
    const uint32_t e = es[s];
    if (!e) continue;
    Item it{s, e, {}, {}};
    std::vector<uint32_t> all(k);
    for (uint32_t j = 0; j < k; j++) all[j] = j;
    std::shuffle(all.begin(), all.end(), rng);
    std::vector<uint32_t> lost(all.begin(), all.begin() + e), surv;
    for (uint32_t i = 0; i < n && surv.size() < k; i++)
      if (std::find(lost.begin(), lost.end(), i) == lost.end()) surv.push_back(i);
    for (uint32_t c = 0; c < k; c++) {
      const uint32_t id = surv[c];
      it.in.push_back(reinterpret_cast<uint64_t>(id < k ? d + s * k * B + id * B
                                                        : p + s * (n - k) * B + (id - k) * B));
    }
    for (uint32_t j = 0; j < k * e; j++) it.tabs.push_back(perm_tab(uint8_t(rng() | 1)));
    items.push_back(std::move(it));
    bytes += double(k + e) * B;
  }
  const uint32_t tps = static_cast<uint32_t>((B / 16 + kThreads - 1) / kThreads);
  const uint32_t tab_q = 1 + k + kMixR;
  const uint32_t rec_plain = 1 + k + kMixR, rec_inl = tab_q + 4 * k * kMixR;
  auto build = [&](bool sorted, bool inl, int U, bool heavy_first, std::vector<uint64_t> &rec,
                   std::vector<PermTab> &tab, Bounds &b) {
    const uint32_t tpsU = static_cast<uint32_t>((B / 16 + kThreads * U - 1) / (kThreads * U));
    std::vector<uint32_t> ord(items.size());
    for (uint32_t i = 0; i < ord.size(); i++) ord[i] = i;
    if (sorted)
      std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return items[x].e < items[y].e; });
    if (heavy_first)
      std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return items[x].e > items[y].e; });
    rec.clear();
    tab.clear();
    b = Bounds{};
    for (uint32_t r = 0; r <= kMixR + 1; r++) b.first[r] = UINT32_MAX;
    b.tab_q = tab_q;
    for (uint32_t q = 0; q < ord.size(); q++) {
      const Item &it = items[ord[q]];
      if (sorted && b.first[it.e] == UINT32_MAX)
        for (uint32_t r = 1; r <= it.e; r++) b.first[r] = std::min(b.first[r], q * tpsU);
      const size_t r0 = rec.size();
      rec.resize(r0 + (inl ? rec_inl : rec_plain), 0);
      rec[r0] = (inl ? 0 : tab.size()) | (uint64_t(it.e) << 32);
      for (uint32_t c = 0; c < k; c++) rec[r0 + 1 + c] = it.in[c];
      // output row i of chunk s -> o + ((s * kMixR) + i) * B
      for (uint32_t i = 0; i < it.e; i++)
        rec[r0 + 1 + k + i] = reinterpret_cast<uint64_t>(o + (size_t(it.s) * kMixR + i) * B);
      if (inl)
        std::memcpy(&rec[r0 + tab_q], it.tabs.data(), it.tabs.size() * sizeof(PermTab));
      else
        tab.insert(tab.end(), it.tabs.begin(), it.tabs.end());
    }
    // sorted: counts above the largest present start past the grid
    for (uint32_t r = 1; r <= kMixR; r++)
      if (b.first[r] == UINT32_MAX) b.first[r] = static_cast<uint32_t>(ord.size()) * tpsU;
  };
  auto vs = variants<KM>();
  struct Up {
    uint64_t *rec = nullptr;
    PermTab *tab = nullptr;
    Bounds b{};
    DescArgs a{};
  };
  std::vector<Up> ups(vs.size());
  for (size_t vi = 0; vi < vs.size(); vi++) {
    std::vector<uint64_t> rec;
    std::vector<PermTab> tab;
    build(vs[vi].sorted, vs[vi].inl, vs[vi].U, vs[vi].heavy_first, rec, tab, ups[vi].b);
    CK(hipMalloc(&ups[vi].rec, rec.size() * 8));
    CK(hipMemcpy(ups[vi].rec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&ups[vi].tab, std::max<size_t>(1, tab.size()) * sizeof(PermTab)));
    if (!tab.empty())
      CK(hipMemcpy(ups[vi].tab, tab.data(), tab.size() * sizeof(PermTab), hipMemcpyHostToDevice));
    DescArgs &a = ups[vi].a;
    a.desc = ups[vi].rec;
    a.ptab = ups[vi].tab;
    a.block = B;
    a.k = k;
    a.r = kMixR;
    a.tpw = 1;
    a.nitems = static_cast<uint32_t>(items.size());
    a.copy = 0;
    a.rec_qwords = vs[vi].inl ? rec_inl : rec_plain;
    a.mix = 1;
  }
  const size_t ob = size_t(N) * kMixR * B;
  std::vector<uint8_t> want(ob), got(ob);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (size_t vi = 0; vi < vs.size(); vi++) {
    CK(hipMemsetAsync(o, 0xEE, ob, s));
    CK(vs[vi].fn(ups[vi].a, ups[vi].b, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(vi ? got.data() : want.data(), o, ob, hipMemcpyDeviceToHost));
    if (vi && std::memcmp(want.data(), got.data(), ob) != 0) {
      std::printf("k=%u %s: MISMATCH\n", k, vs[vi].name.c_str());
      return 1;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < reps; r++)
    for (size_t vi = 0; vi < vs.size(); vi++) {
      CK(hipEventRecord(e0, s));
      CK(vs[vi].fn(ups[vi].a, ups[vi].b, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float x = 0;
      CK(hipEventElapsedTime(&x, e0, e1));
      vs[vi].ms.push_back(x);
    }
  std::printf("k=%u: %zu chunks decoded (%u with no loss), %.3f GB per launch\n", k, items.size(),
              hist[0], bytes / 1e9);
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float m = v.ms[v.ms.size() / 2];
    std::printf("k=%u %-34s %8.4f ms  %6.2f TB/s  %5.1f %%  (bit-exact)\n", k, v.name.c_str(), m,
                bytes / (m * 1e-3) / 1e12, 100.0 * bytes / (m * 1e-3) / 8e12);
  }
  // Isolation per row count R: the chunks that lost R data shares, each
  // with the same survivor slots (data shares 0..R-1 lost, rebuilt from the
  // first R parity shares): the mixed-row kernel over them (records) against
  // the uniform table kernel over the same stripes (pointers in kernel
  // arguments), same tables. The three uniform launches back to back against
  // the one mixed launch over all chunks: how much of the gap to the uniform
  // 2-lost figure is the mix of row counts rather than the descriptors.
  double t_uni_sum = 0, t_mix_sum = 0;
  if (isolate<KM, 1>(reps, es, N, k, n, B, d, p, o, ob, s, e0, e1, rng, t_uni_sum, t_mix_sum) ||
      isolate<KM, 2>(reps, es, N, k, n, B, d, p, o, ob, s, e0, e1, rng, t_uni_sum, t_mix_sum) ||
      isolate<KM, 3>(reps, es, N, k, n, B, d, p, o, ob, s, e0, e1, rng, t_uni_sum, t_mix_sum))
    return 1;
  std::printf("k=%u all row counts: sum of the uniform launches (uncapped) %.4f ms = %.1f %%, "
              "sum of the per-count mixed launches %.4f ms = %.1f %%\n", k, t_uni_sum,
              100.0 * bytes / (t_uni_sum * 1e-3) / 8e12, t_mix_sum,
              100.0 * bytes / (t_mix_sum * 1e-3) / 8e12);
  CK(hipStreamDestroy(s));
  for (auto &u : ups) {
    CK(hipFree(u.rec));
    CK(hipFree(u.tab));
  }
  CK(hipFree(d));
  CK(hipFree(p));
  CK(hipFree(o));
  return 0;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const int K = argc > 2 ? std::atoi(argv[2]) : 16;
  return K == 32 ? run<32>(reps) : run<16>(reps);
}
