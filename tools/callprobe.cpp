// callprobe.cpp -- one single-chunk call shape, back to back, for tracing.
//
// The zfec-rs shim calls storb_rs_encode / storb_rs_decode once per chunk
// (piece.rs:328-329, 383-386 through integration/zfec-rs-mi355x/src/lib.rs).
// This runs ONE geometry N times in a row (no oracle between calls, unlike
// tools/callbench.cpp) so that a rocprofv3 --kernel-trace --hip-runtime-trace
// of it shows where a call's time goes (packing, launches, waits, unpacking),
// and prints the median / p10 per-call latency.
//
// usage: callprobe K N CHUNK_BYTES ITERS [encode|decode] [pageable|pinned]
// build: g++ -O2 -std=c++17 tools/callprobe.cpp -Iinclude -Lstorb_amd/lib -lstorb_rs \
//          -Wl,-rpath,'$ORIGIN/../../storb_amd/lib' -o tools/_build/callprobe
// Stage timeline (library built with -DSTORB_RS_CALL_TRACE as
// tools/_build/libstorb_rs_trace.so, see tools/r3k_calltrace.sh): add
//   -DCALL_TRACE -Ltools/_build -lstorb_rs_trace (instead of -lstorb_rs), rpath '$ORIGIN'
// and each stage mark's median offset from the call's start is printed.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "storb_rs.h"

using clk = std::chrono::steady_clock;

#ifdef CALL_TRACE
extern "C" int storb_rs_debug_marks(const char **what, double *us, int max);
#include <map>
#include <string>
#endif

int main(int argc, char **argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: callprobe K N CHUNK ITERS [encode|decode] [pageable|pinned]\n");
    return 1;
  }
  const uint32_t k = std::atoi(argv[1]), n = std::atoi(argv[2]);
  const size_t chunk = std::strtoull(argv[3], nullptr, 10);
  const int iters = std::atoi(argv[4]);
  const bool dec = argc > 5 && std::strcmp(argv[5], "decode") == 0;
  const bool pinned = argc > 6 && std::strcmp(argv[6], "pinned") == 0;
  auto buf = [&](size_t len) {
    void *p = nullptr;
    if (pinned) {
      if (storb_rs_host_alloc(len, &p)) std::abort();
    } else {
      p = std::aligned_alloc(64, (len + 63) / 64 * 64);
    }
    std::memset(p, 0x11, len);
    return static_cast<uint8_t *>(p);
  };
  storb_rs_ctx *ctx = nullptr;
  if (storb_rs_ctx_create(0, &ctx)) return 1;
  const size_t B = storb_rs_block_size(k, chunk), pad = k * B - chunk;
  uint8_t *data = buf(chunk);
  for (size_t i = 0; i < chunk; i++) data[i] = static_cast<uint8_t>(i * 131 + (i >> 9));
  std::vector<uint8_t *> par(n - k);
  for (auto &p : par) p = buf(B);
  size_t bo, po;
  if (storb_rs_encode(ctx, k, n, data, chunk, par.data(), &bo, &po)) return 2;
  // decode inputs: data shares 0 and 1 lost, first k survivors by index
  std::vector<uint8_t *> ds(k);
  for (uint32_t j = 0; j < k; j++) {
    ds[j] = buf(B);
    const size_t o = static_cast<size_t>(j) * B;
    if (o < chunk) std::memcpy(ds[j], data + o, std::min(B, chunk - o));
  }
  std::vector<const uint8_t *> sh;
  std::vector<uint32_t> idx;
  for (uint32_t i = std::min<uint32_t>(2, n - k); i < n && sh.size() < k; i++) {
    sh.push_back(i < k ? ds[i] : par[i - k]);
    idx.push_back(i);
  }
  uint8_t *out = buf(chunk);
  std::vector<double> us;
#ifdef CALL_TRACE
  std::map<std::string, std::vector<double>> at;  // "i:stage" -> offsets from call start
#endif
  for (int r = 0; r < iters + 5; r++) {
    const auto t0 = clk::now();
    const int rc = dec ? storb_rs_decode(ctx, k, n, sh.data(), idx.data(), k, B, pad, out)
                       : storb_rs_encode(ctx, k, n, data, chunk, par.data(), &bo, &po);
    const auto t1 = clk::now();
    if (rc) return 3;
    if (r >= 5) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
#ifdef CALL_TRACE
    const char *w[64];
    double m[64];
    const int nm = storb_rs_debug_marks(w, m, 64);
    const double s0 = std::chrono::duration<double, std::micro>(t0.time_since_epoch()).count();
    for (int i = 0; r >= 5 && i < nm; i++) {
      char key[64];
      std::snprintf(key, sizeof(key), "%02d:%s", i, w[i]);
      at[key].push_back(m[i] - s0);
    }
#endif
  }
#ifdef CALL_TRACE
  for (auto &kv : at) {
    std::sort(kv.second.begin(), kv.second.end());
    std::printf("  %-12s at %8.2f us (median)\n", kv.first.c_str(), kv.second[kv.second.size() / 2]);
  }
#endif
  if (dec && std::memcmp(out, data, chunk) != 0) {
    std::fprintf(stderr, "decode mismatch\n");
    return 4;
  }
  std::sort(us.begin(), us.end());
  std::printf("{\"k\": %u, \"n\": %u, \"chunk\": %zu, \"op\": \"%s\", \"buffers\": \"%s\", "
              "\"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"GiBps\": %.2f}\n",
              k, n, chunk, dec ? "decode" : "encode", pinned ? "page-locked" : "pageable",
              us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10],
              chunk / us[us.size() / 2] * 1e6 / (1 << 30));
  storb_rs_ctx_destroy(ctx);
  return 0;
}
