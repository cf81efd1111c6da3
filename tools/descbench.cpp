// descbench.cpp -- per-stripe-pattern decode launches (rs_apply_desc) on a
// download-shaped workload: BASELINE config 5's geometry (128 x 8 MiB
// chunks, k = 16, n = 24) where each chunk lost 0-3 data shares in the
// proportions bench.py --erase-pattern download draws (13 / 48 / 58 / 9 of
// 128), random survivor sets. Times (hipEvents, median of reps):
//   * product: storb_rs_decode_stripes_dev (the library's own grouping,
//     stream fan-out and tiles-per-workgroup rule);
//   * the per-row-count launches sequential on one stream, tpw = 1, 2, 4, 8;
//   * the same fanned out over 3 streams;
//   * uniform reference: every stripe with 2 lost, one table-kernel launch
//     (storb_rs_decode_batch_dev with the PERM variant).
//   * one mixed-row launch (DescArgs::mix) over the resident-workgroup cap;
//   * the product call's host time;
// Bytes = sum over stripes with e > 0 of (k + e) * B. Performance only (the
// coefficients are random); bit-exactness is tests/test_gpu_patterns.py's.
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/descbench.cpp -Iinclude \
//   -Istorb_amd/csrc -Lstorb_amd/lib -lstorb_rs -Wl,-rpath,'$ORIGIN/../../storb_amd/lib' \
//   -o tools/_build/descbench
// usage: descbench [REPS] [K]; K = 4 runs the default line's download leg (config
// 2's geometry); K = 32 runs config 6's download shape instead
// (32 chunks x 32 MiB, k = 32, n = 48, B = 1 MiB; 4 / 14 / 13 / 1 chunks lost
// 0 / 1 / 2 / 3 data shares, the histogram of profiles/r3k_bench_c6_download.json).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "gf256.hpp"
#include "rs_kernels.hpp"
#include "storb_rs.h"

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                        \
    }                                                                  \
  } while (0)

using namespace storb_rs;

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const int karg = argc > 2 ? std::atoi(argv[2]) : 16;
  const bool c6 = karg == 32, c2 = karg == 4;
  const uint32_t k = c6 ? 32 : c2 ? 4 : 16, n = k + k / 2, N = c6 ? 32 : c2 ? 1024 : 128;
  const size_t B = c6 ? (1u << 20) : c2 ? (256u << 10) : (512u << 10);
  // K = 4: the default bench line's download leg (1024 x 1 MiB chunks, 349 /
  // 675 lost 0 / 1 data shares, BENCH download_decode histogram)
  const int hist[4] = {c6 ? 4 : c2 ? 349 : 13, c6 ? 14 : c2 ? 675 : 48, c6 ? 13 : c2 ? 0 : 58,
                       c6 ? 1 : c2 ? 0 : 9};
  uint8_t *d = nullptr, *p = nullptr;
  CK(hipMalloc(&d, N * k * B));
  CK(hipMalloc(&p, N * (n - k) * B));
  CK(hipMemset(d, 0x3C, N * k * B));
  CK(hipMemset(p, 0x5A, N * (n - k) * B));
  std::mt19937 rng(5);
  std::vector<uint32_t> es;
  for (uint32_t e = 0; e < 4; e++)
    for (int i = 0; i < hist[e]; i++) es.push_back(e);
  std::shuffle(es.begin(), es.end(), rng);
  // per stripe: survivors (first k of the shares not lost) and lost rows
  std::vector<std::vector<uint32_t>> surv(N), lost(N);
  std::vector<uint32_t> flat, cnt;
  double bytes = 0;
  for (uint32_t s = 0; s < N; s++) {
    std::vector<uint32_t> all(k);
    for (uint32_t j = 0; j < k; j++) all[j] = j;
    std::shuffle(all.begin(), all.end(), rng);
    lost[s].assign(all.begin(), all.begin() + es[s]);
    std::sort(lost[s].begin(), lost[s].end());
    for (uint32_t i = 0; i < n && surv[s].size() < k; i++)
      if (std::find(lost[s].begin(), lost[s].end(), i) == lost[s].end()) surv[s].push_back(i);
    flat.insert(flat.end(), surv[s].begin(), surv[s].end());
    cnt.push_back(k);
    if (es[s]) bytes += double(k + es[s]) * B;
  }
  storb_rs_ctx *ctx = nullptr;
  if (storb_rs_ctx_create(0, &ctx)) return 1;
  hipStream_t st[3];
  for (auto &x : st) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t e0, e1, fs, fe[2];
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fs, hipEventDisableTiming));
  for (auto &x : fe) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  auto timeit = [&](const char *name, auto &&go, double b) -> int {
    go();
    CK(hipStreamSynchronize(st[0]));
    std::vector<float> ms;
    for (int r = 0; r < reps; r++) {
      CK(hipEventRecord(e0, st[0]));
      go();
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float x = 0;
      CK(hipEventElapsedTime(&x, e0, e1));
      ms.push_back(x);
    }
    std::sort(ms.begin(), ms.end());
    const float m = ms[ms.size() / 2];
    std::printf("%-58s %8.4f ms  %6.2f TB/s  %5.1f %%\n", name, m, b / (m * 1e-3) / 1e12,
                100.0 * b / (m * 1e-3) / 8e12);
    return 0;
  };
  // product
  if (timeit("product storb_rs_decode_stripes_dev", [&] {
        storb_rs_decode_stripes_dev(ctx, k, n, B, N, flat.data(), cnt.data(), d, 0, p, 0, d, 0,
                                    st[0]);
      }, bytes))
    return 1;
  // hand-built groups: random tables per row count, records per stripe
  const uint64_t rb_max = 3;
  std::vector<std::vector<uint64_t>> recs(rb_max + 1);
  std::vector<std::vector<PermTab>> tabs(rb_max + 1);
  std::vector<uint32_t> nitems(rb_max + 1, 0);
  for (uint32_t s = 0; s < N; s++) {
    const uint32_t e = es[s];
    if (!e) continue;
    const uint64_t off = tabs[e].size();
    for (uint32_t j = 0; j < k * e; j++) tabs[e].push_back(perm_tab(uint8_t(rng() | 1)));
    recs[e].push_back(off);
    for (uint32_t c = 0; c < k; c++) {
      const uint32_t id = surv[s][c];
      recs[e].push_back(reinterpret_cast<uint64_t>(
          id < k ? d + s * k * B + id * B : p + s * (n - k) * B + (id - k) * B));
    }
    for (uint32_t r = 0; r < e; r++)
      recs[e].push_back(reinterpret_cast<uint64_t>(d + s * k * B + lost[s][r] * B));
    nitems[e]++;
  }
  std::vector<uint64_t *> drec(rb_max + 1, nullptr);
  std::vector<PermTab *> dtab(rb_max + 1, nullptr);
  for (uint32_t e = 1; e <= rb_max; e++) {
    CK(hipMalloc(&drec[e], recs[e].size() * 8));
    CK(hipMalloc(&dtab[e], tabs[e].size() * sizeof(PermTab)));
    CK(hipMemcpy(drec[e], recs[e].data(), recs[e].size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtab[e], tabs[e].data(), tabs[e].size() * sizeof(PermTab), hipMemcpyHostToDevice));
  }
  auto args = [&](uint32_t e, uint32_t tpw) {
    DescArgs a{};
    a.desc = drec[e];
    a.ptab = dtab[e];
    a.block = B;
    a.k = k;
    a.r = e;
    a.tpw = tpw;
    a.nitems = nitems[e];
    a.copy = 0;
    a.rec_qwords = 1 + k + e;
    return a;
  };
  const uint32_t order[3] = {2, 1, 3};  // biggest group first
  for (uint32_t tpw : {1u, 2u, 4u, 8u}) {
    char name[96];
    std::snprintf(name, sizeof(name), "per-row-count launches, 1 stream, tpw %u", tpw);
    if (timeit(name, [&] {
          for (uint32_t e : order) (void)launch_apply_desc(args(e, tpw), st[0]);
        }, bytes))
      return 1;
    std::snprintf(name, sizeof(name), "per-row-count launches, 3 streams, tpw %u", tpw);
    if (timeit(name, [&] {
          (void)hipEventRecord(fs, st[0]);
          (void)hipStreamWaitEvent(st[1], fs, 0);
          (void)hipStreamWaitEvent(st[2], fs, 0);
          for (int i = 0; i < 3; i++) (void)launch_apply_desc(args(order[i], tpw), st[i]);
          for (int i = 1; i < 3; i++) {
            (void)hipEventRecord(fe[i - 1], st[i]);
            (void)hipStreamWaitEvent(st[0], fe[i - 1], 0);
          }
        }, bytes))
      return 1;
  }
  // one mixed-row launch (DescArgs::mix): records with kMixR output slots,
  // rec[0] = table offset | rows << 32; resident-workgroup cap swept
  std::vector<uint64_t> mrec;
  std::vector<PermTab> mtab;
  for (uint32_t s = 0; s < N; s++) {
    const uint32_t e = es[s];
    if (!e) continue;
    const uint64_t off = mtab.size();
    for (uint32_t j = 0; j < k * e; j++) mtab.push_back(perm_tab(uint8_t(rng() | 1)));
    mrec.push_back(off | (uint64_t(e) << 32));
    for (uint32_t c = 0; c < k; c++) {
      const uint32_t id = surv[s][c];
      mrec.push_back(reinterpret_cast<uint64_t>(
          id < k ? d + s * k * B + id * B : p + s * (n - k) * B + (id - k) * B));
    }
    for (uint32_t r = 0; r < kMixR; r++)
      mrec.push_back(r < e ? reinterpret_cast<uint64_t>(d + s * k * B + lost[s][r] * B) : 0);
  }
  uint64_t *dmrec = nullptr;
  PermTab *dmtab = nullptr;
  CK(hipMalloc(&dmrec, mrec.size() * 8));
  CK(hipMalloc(&dmtab, mtab.size() * sizeof(PermTab)));
  CK(hipMemcpy(dmrec, mrec.data(), mrec.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dmtab, mtab.data(), mtab.size() * sizeof(PermTab), hipMemcpyHostToDevice));
  for (uint32_t cap : {0u, 2u, 3u, 4u, 6u, 8u}) {
    for (uint32_t tpw : {1u, 2u, 4u}) {
      DescArgs a{};
      a.desc = dmrec;
      a.ptab = dmtab;
      a.block = B;
      a.k = k;
      a.r = kMixR;
      a.tpw = tpw;
      a.nitems = N - hist[0];
      a.rec_qwords = 1 + k + kMixR;
      a.mix = 1;
      a.cap = cap;
      char name[96];
      std::snprintf(name, sizeof(name), "one mixed-row launch, cap %u%s, tpw %u", cap,
                    cap ? "" : " (default)", tpw);
      if (timeit(name, [&] { (void)launch_apply_desc(a, st[0]); }, bytes)) return 1;
    }
  }
  // host time of the product call (patterns, records, upload, launches)
  {
    std::vector<double> hus;
    for (int r = 0; r < reps; r++) {
      CK(hipStreamSynchronize(st[0]));
      const auto t0 = std::chrono::steady_clock::now();
      storb_rs_decode_stripes_dev(ctx, k, n, B, N, flat.data(), cnt.data(), d, 0, p, 0, d, 0, st[0]);
      hus.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(st[0]));
    std::sort(hus.begin(), hus.end());
    std::printf("product call host time (returns before the kernels end): median %.1f us\n",
                hus[hus.size() / 2]);
  }
  // uniform reference: 2 lost everywhere (K = 4: 1 lost, as the download),
  // table kernel
  storb_rs_set_kernel(ctx, STORB_RS_KERNEL_PERM);
  const uint32_t ul = c2 ? 1 : 2;
  std::vector<uint32_t> s2;
  for (uint32_t i = ul; i < n && s2.size() < k; i++) s2.push_back(i);
  char uname[96];
  const uint32_t un = c2 ? uint32_t(hist[1]) : N;
  std::snprintf(uname, sizeof(uname), "uniform: %u stripes, %u lost, rs_apply_perm<%u,%u>", un, ul,
                k, ul);
  if (timeit(uname, [&] {
        storb_rs_decode_batch_dev(ctx, k, n, B, un, s2.data(), k, d, 0, p, 0, d, 0, st[0]);
      }, double(un) * (k + ul) * B))
    return 1;
  storb_rs_ctx_destroy(ctx);
  return 0;
}
