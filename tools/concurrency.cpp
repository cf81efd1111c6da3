// concurrency.cpp -- many uploads at once, each on its own thread.
//
// Storb runs one tokio task per upload (upload.rs:418-420 encodes that
// upload's chunks one after another); through the zfec-rs shim every task's
// thread gets its own storb_rs_ctx (own stream, own pinned staging), so
// concurrent uploads become concurrent kernels on one GPU. This measures the
// aggregate rate of T threads each encoding R chunks of Storb's sizing for
// an object of OBJ bytes, pageable buffers, against the oracle's rate on
// the same T threads (the reference's CPU cost for the same work).
//
// usage: concurrency OBJ_BYTES [R=200] (prints one JSON line per T)
// build: g++ -O2 -std=c++17 -pthread concurrency.cpp -I../include -I../oracle \
//        -L../storb_amd/lib -lstorb_rs -L../oracle/_build -lzfec_oracle \
//        -Wl,-rpath,'$ORIGIN/../../storb_amd/lib:$ORIGIN/../../oracle/_build' -o _build/concurrency
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "storb_rs.h"
#include "zfec_oracle.h"

using clk = std::chrono::steady_clock;

int main(int argc, char **argv) {
  const uint64_t obj = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1ull << 20);
  const int R = argc > 2 ? std::atoi(argv[2]) : 200;
  const uint64_t chunk = storb_piece_length(obj, 0, 0);
  uint64_t k64, m64;
  storb_get_k_and_m(chunk, &k64, &m64);
  const uint32_t k = static_cast<uint32_t>(k64), n = static_cast<uint32_t>(m64);
  const size_t B = storb_rs_block_size(k, chunk);
  zo_init();
  // gpu = 1: a context per thread (the shim's layout); 0: the oracle
  for (int T : {1, 2, 4, 8, 16}) {
    for (int gpu = 1; gpu >= 0; gpu--) {
      std::atomic<int> bad{0}, ready{0};
      std::atomic<bool> go{false};
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
          // setup (context, staging, tables, one warm call) outside the clock
          storb_rs_ctx *ctx = nullptr;
          if (gpu == 1 && storb_rs_ctx_create(0, &ctx) != STORB_RS_OK) bad++;
          std::vector<uint8_t> data(chunk);
          zo_splitmix_fill(0x5709B + t, data.data(), chunk);
          std::vector<std::vector<uint8_t>> par(n - k, std::vector<uint8_t>(B));
          std::vector<uint8_t *> pp(n - k);
          for (uint32_t i = 0; i < n - k; i++) pp[i] = par[i].data();
          size_t bo, po;
          if (ctx) storb_rs_encode(ctx, k, n, data.data(), chunk, pp.data(), &bo, &po);
          ready++;
          while (!go.load()) std::this_thread::yield();
          for (int r = 0; r < R; r++) {
            const int rc = gpu ? storb_rs_encode(ctx, k, n, data.data(), chunk, pp.data(), &bo, &po)
                               : zo_encode_parity(k, n, data.data(), chunk, pp.data(), &bo, &po);
            if (rc) bad++;
          }
          ready--;  // signals the clock (the last thread out stops it)
          if (ctx) storb_rs_ctx_destroy(ctx);
        });
      while (ready.load() < T) std::this_thread::yield();
      auto t0 = clk::now();
      go = true;
      while (ready.load() > 0) std::this_thread::yield();
      const double s = std::chrono::duration<double>(clk::now() - t0).count();
      for (auto &x : th) x.join();  // context teardown outside the clock
      std::printf(
          "{\"path\": \"%s\", \"object_bytes\": %llu, \"chunk_bytes\": %llu, \"k\": %u, "
          "\"m_total\": %u, \"threads\": %d, \"calls_per_thread\": %d, \"GiBps\": %.3f, "
          "\"calls_per_s\": %.0f, \"errors\": %d}\n",
          gpu ? "storb_rs_encode (ctx per thread)" : "oracle (CPU)",
          static_cast<unsigned long long>(obj), static_cast<unsigned long long>(chunk), k, n, T,
          R, static_cast<double>(T) * R * chunk / s / (1 << 30), T * R / s, bad.load());
      std::fflush(stdout);
    }
  }
  return 0;
}
