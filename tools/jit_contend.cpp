// jit_contend.cpp -- does the JIT's compile thread make progress while the
// calling thread keeps the GPU busy? (tools/jit_fuzz.py saw 0 of 32 queued
// compiles finish in 6 s of decode calls on the GPU box, then all 32 in
// 11 s once the calls stopped.) Queues k = 16 decode patterns
// (storb_rs_jit_prepare_decode, no wait) and, for 12 s, either sleeps
// ("idle"), or issues small device calls back to back on one stream and
// waits for each ("gpu": encode_batch_dev of 4 x 64 KiB stripes + stream
// sync), printing the compile count every 2 s.
// build: hipcc -O2 -std=c++17 tools/jit_contend.cpp -Iinclude -Lstorb_amd/lib -lstorb_rs \
//          -Wl,-rpath,'$ORIGIN/../../storb_amd/lib' -o tools/_build/jit_contend
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "storb_rs.h"

int main(int argc, char **argv) {
  using clk = std::chrono::steady_clock;
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const int seed = argc > 2 ? std::atoi(argv[2]) : 0;
  storb_rs_ctx *ctx = nullptr;
  if (storb_rs_ctx_create(0, &ctx)) return 1;
  uint8_t *d = nullptr, *p = nullptr;
  if (hipMalloc(&d, 16 * 65536 * 4) || hipMalloc(&p, 8 * 65536 * 4)) return 1;
  hipStream_t s;
  if (hipStreamCreate(&s)) return 1;
  const uint32_t k = 16, n = 24;
  for (int q = 0; q < 24; q++) {  // 24 distinct 3-lost patterns (seeded so comgr's cache misses)
    std::vector<uint32_t> sv;
    const uint32_t a = (q + seed) % 16, b = (q * 5 + 3 + seed) % 16, c = (q * 11 + 7 + seed) % 16;
    for (uint32_t i = 0; i < n && sv.size() < k; i++)
      if (i != a && i != b && i != c) sv.push_back(i);
    storb_rs_jit_prepare_decode(k, n, sv.data(), k, 0, 0);
  }
  const auto t0 = clk::now();
  double last = -2;
  long calls = 0;
  for (;;) {
    if (gpu) {
      if (storb_rs_encode_batch_dev(ctx, 16, 24, 65536, 4, d, 0, p, 0, s)) return 2;
      if (hipStreamSynchronize(s)) return 3;
      calls++;
    } else {
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    if (el - last >= 2.0) {
      last = el;
      storb_rs_jit_stats_t st;
      storb_rs_jit_stats(&st);
      std::printf("%s t=%.1f calls=%ld compiled=%llu pending=%llu compile_ms=%.0f\n",
                  gpu ? "gpu " : "idle", el, calls, (unsigned long long)st.compiled,
                  (unsigned long long)st.pending, st.compile_ms);
      std::fflush(stdout);
    }
    if (el > 12) break;
  }
  storb_rs_ctx_destroy(ctx);
  return 0;
}
