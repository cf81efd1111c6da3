// asyncbench.cpp -- one upload task, async calls with D chunks in flight.
//
// upload.rs:418-420 encodes an upload's chunks one after another inside one
// tokio task; with storb_rs_encode_async the task can keep D chunks on the
// GPU while it stages the next (host_async.cpp). One thread, one context,
// Storb's sizing for an object of OBJ bytes, pageable buffers; D = 0 is the
// synchronous storb_rs_encode loop for comparison. Every op's parity is
// checked against the synchronous call's.
//
// usage: asyncbench OBJ_BYTES [R=200]   (one JSON line per depth)
// build: g++ -O2 -std=c++17 -pthread asyncbench.cpp -I../include \
//        -L../storb_amd/lib -lstorb_rs -Wl,-rpath,'$ORIGIN/../../storb_amd/lib' \
//        -o _build/asyncbench
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "storb_rs.h"

using clk = std::chrono::steady_clock;

int main(int argc, char **argv) {
  const uint64_t obj = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (16ull << 20);
  const int R = argc > 2 ? std::atoi(argv[2]) : 200;
  const uint64_t chunk = storb_piece_length(obj, 0, 0);
  uint64_t k64, m64;
  storb_get_k_and_m(chunk, &k64, &m64);
  const uint32_t k = static_cast<uint32_t>(k64), n = static_cast<uint32_t>(m64), p = n - k;
  const size_t B = storb_rs_block_size(k, chunk);
  storb_rs_ctx *ctx = nullptr;
  if (storb_rs_ctx_create(0, &ctx) != STORB_RS_OK) {
    std::fprintf(stderr, "no device\n");
    return 1;
  }
  std::vector<uint8_t> data(chunk);
  for (size_t i = 0; i < chunk; i++) data[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
  std::vector<std::vector<uint8_t>> ref(p, std::vector<uint8_t>(B));
  std::vector<uint8_t *> rp(p);
  for (uint32_t i = 0; i < p; i++) rp[i] = ref[i].data();
  size_t bo, po;
  if (storb_rs_encode(ctx, k, n, data.data(), chunk, rp.data(), &bo, &po)) return 1;
  for (int D : {0, 1, 2, 3, 4, 8, 16}) {
    const int slots = D ? D : 1;
    std::vector<std::vector<std::vector<uint8_t>>> par(
        slots, std::vector<std::vector<uint8_t>>(p, std::vector<uint8_t>(B)));
    std::vector<std::vector<uint8_t *>> pp(slots, std::vector<uint8_t *>(p));
    for (int s = 0; s < slots; s++)
      for (uint32_t i = 0; i < p; i++) pp[s][i] = par[s][i].data();
    std::vector<storb_rs_op *> ops(slots, nullptr);
    int bad = 0;
    auto check = [&](int s) {
      for (uint32_t i = 0; i < p; i++)
        if (std::memcmp(par[s][i].data(), ref[i].data(), B)) bad++;
    };
    // warm outside the clock: D ops in flight at once, so the context has D
    // slots (stream + staging) before the timed loop reuses them
    for (int s = 0; s < slots && D; s++)
      if (storb_rs_encode_async(ctx, k, n, data.data(), chunk, pp[s].data(), &bo, &po, nullptr,
                                nullptr, &ops[s]))
        bad++;
    for (int s = 0; s < slots && D; s++) {
      if (ops[s] && storb_rs_op_finish(ops[s])) bad++;
      ops[s] = nullptr;
    }
    const auto t0 = clk::now();
    for (int r = 0; r < R; r++) {
      const int s = r % slots;
      if (D == 0) {
        if (storb_rs_encode(ctx, k, n, data.data(), chunk, pp[0].data(), &bo, &po)) bad++;
        continue;
      }
      if (ops[s]) {  // the slot's previous chunk: collect it first
        if (storb_rs_op_finish(ops[s])) bad++;
        check(s);
        ops[s] = nullptr;
      }
      if (storb_rs_encode_async(ctx, k, n, data.data(), chunk, pp[s].data(), &bo, &po, nullptr,
                                nullptr, &ops[s]))
        bad++;
    }
    for (int s = 0; s < slots; s++)
      if (ops[s]) {
        if (storb_rs_op_finish(ops[s])) bad++;
        check(s);
      }
    const double sec = std::chrono::duration<double>(clk::now() - t0).count();
    if (D == 0) check(0);
    std::printf(
        "{\"path\": \"%s\", \"depth\": %d, \"object_bytes\": %llu, \"chunk_bytes\": %llu, "
        "\"k\": %u, \"m_total\": %u, \"calls\": %d, \"GiBps\": %.3f, \"us_per_chunk\": %.1f, "
        "\"mismatches\": %d}\n",
        D ? "storb_rs_encode_async" : "storb_rs_encode (sync)", D,
        static_cast<unsigned long long>(obj), static_cast<unsigned long long>(chunk), k, n, R,
        static_cast<double>(R) * chunk / sec / (1 << 30), sec / R * 1e6, bad);
    std::fflush(stdout);
  }
  storb_rs_ctx_destroy(ctx);
  return 0;
}
