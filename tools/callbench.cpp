// callbench.cpp -- the drop-in path one call at a time.
//
// Storb's unchanged piece.rs calls Fec::encode / Fec::decode once per chunk
// (upload.rs:418-420, download.rs:464); through the zfec-rs shim each is one
// storb_rs_encode / storb_rs_decode: host bytes in, host bytes out, blocking.
// For object sizes from 64 KiB to 1 GiB this sizes chunks exactly as Storb
// does (piece_length of the object, get_k_and_m of the chunk, piece.rs:
// 292-317), then times per call (median of reps):
//   * encode: storb_rs_encode of one chunk (parity to caller buffers),
//   * decode: storb_rs_decode with the first min(n-k, 2) data shares lost,
// next to the oracle (scalar zfec restatement, oracle/, single thread: the
// reference's own per-chunk CPU cost) on the same chunk, bit-exact checked.
// Output: one JSON line per object size. `callbench REPS pinned` puts every
// caller buffer in page-locked memory (storb_rs_host_alloc): the calls then
// run the kernel on them in place, with no staging copies.
//
// build: g++ -O2 -std=c++17 callbench.cpp -I../include -I../oracle \
//        -L../storb_amd/lib -lstorb_rs -L../oracle/_build -lzfec_oracle \
//        -Wl,-rpath,'$ORIGIN/../../storb_amd/lib:$ORIGIN/../../oracle/_build' -o _build/callbench
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "storb_rs.h"
#include "zfec_oracle.h"

using clk = std::chrono::steady_clock;

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static bool g_pinned = false;

// Caller buffer: pageable (heap) or page-locked, zero-filled.
static uint8_t *buf(size_t n) {
  void *p = nullptr;
  if (g_pinned) {
    if (storb_rs_host_alloc(n, &p) != STORB_RS_OK) std::abort();
  } else {
    p = std::aligned_alloc(64, (n + 63) / 64 * 64);
  }
  std::memset(p, 0, n);
  return static_cast<uint8_t *>(p);
}
static void unbuf(uint8_t *p) {
  if (g_pinned)
    storb_rs_host_free(p);
  else
    std::free(p);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 21;
  g_pinned = argc > 2 && std::strcmp(argv[2], "pinned") == 0;
  storb_rs_ctx *ctx = nullptr;
  if (storb_rs_ctx_create(0, &ctx) != STORB_RS_OK) {
    std::fprintf(stderr, "no device\n");
    return 1;
  }
  zo_init();
  for (uint64_t obj : {64ull << 10, 1ull << 20, 16ull << 20, 256ull << 20, 1ull << 30}) {
    const uint64_t chunk = storb_piece_length(obj, 0, 0);  // upload.rs:209 chunk size
    uint64_t k64, m64;
    storb_get_k_and_m(chunk, &k64, &m64);
    const uint32_t k = static_cast<uint32_t>(k64), n = static_cast<uint32_t>(m64);
    const size_t B = storb_rs_block_size(k, chunk);
    const size_t pad = static_cast<size_t>(k) * B - chunk;
    uint8_t *data = buf(chunk);
    zo_splitmix_fill(0x5709B + obj, data, chunk);
    std::vector<uint8_t *> pp(n - k), wp(n - k);
    for (uint32_t i = 0; i < n - k; i++) {
      pp[i] = buf(B);
      wp[i] = static_cast<uint8_t *>(std::calloc(B, 1));
    }
    size_t bo, po;
    std::vector<double> te, to_e, td, to_d;
    for (int r = 0; r < reps + 2; r++) {
      auto t0 = clk::now();
      if (storb_rs_encode(ctx, k, n, data, chunk, pp.data(), &bo, &po)) return 2;
      auto t1 = clk::now();
      zo_encode_parity(k, n, data, chunk, wp.data(), &bo, &po);
      auto t2 = clk::now();
      if (r >= 2) {
        te.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        to_e.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
      }
    }
    for (uint32_t i = 0; i < n - k; i++)
      if (std::memcmp(pp[i], wp[i], B) != 0) {
        std::fprintf(stderr, "parity mismatch obj=%llu\n", static_cast<unsigned long long>(obj));
        return 3;
      }
    // decode: lose the first e data shares, keep the rest (first k by index)
    const uint32_t e = std::min<uint32_t>(n - k, 2);
    std::vector<uint8_t *> dshare(k);
    for (uint32_t j = 0; j < k; j++) {
      dshare[j] = buf(B);
      const size_t o = static_cast<size_t>(j) * B;
      if (o < chunk) std::memcpy(dshare[j], data + o, std::min(B, chunk - o));
    }
    std::vector<const uint8_t *> sh;
    std::vector<uint32_t> idx;
    std::vector<unsigned> uidx;
    for (uint32_t i = e; i < n && sh.size() < k; i++) {
      sh.push_back(i < k ? dshare[i] : pp[i - k]);
      idx.push_back(i);
      uidx.push_back(i);
    }
    uint8_t *out = buf(chunk);
    std::vector<uint8_t> out2(chunk);
    for (int r = 0; r < reps + 2; r++) {
      auto t0 = clk::now();
      if (storb_rs_decode(ctx, k, n, sh.data(), idx.data(), k, B, pad, out)) return 4;
      auto t1 = clk::now();
      zo_decode(k, n, sh.data(), uidx.data(), k, B, pad, out2.data());
      auto t2 = clk::now();
      if (r >= 2) {
        td.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        to_d.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
      }
    }
    if (std::memcmp(out, data, chunk) != 0 || std::memcmp(out2.data(), data, chunk) != 0) {
      std::fprintf(stderr, "decode mismatch obj=%llu\n", static_cast<unsigned long long>(obj));
      return 5;
    }
    unbuf(data);
    unbuf(out);
    for (auto *q : pp) unbuf(q);
    for (auto *q : dshare) unbuf(q);
    for (auto *q : wp) std::free(q);
    const double me = median(te), moe = median(to_e), md = median(td), mod = median(to_d);
    std::printf(
        "{\"object_bytes\": %llu, \"chunk_bytes\": %llu, \"k\": %u, \"m_total\": %u, "
        "\"lost_data_shares\": %u, \"encode_us\": %.1f, \"encode_GiBps\": %.2f, "
        "\"oracle_encode_us\": %.1f, \"decode_us\": %.1f, \"decode_GiBps\": %.2f, "
        "\"oracle_decode_us\": %.1f, \"speedup_encode\": %.2f, \"speedup_decode\": %.2f, "
        "\"caller_buffers\": \"%s\"}\n",
        static_cast<unsigned long long>(obj), static_cast<unsigned long long>(chunk), k, n, e,
        me, chunk / me * 1e6 / (1 << 30), moe, md, chunk / md * 1e6 / (1 << 30), mod, moe / me,
        mod / md, g_pinned ? "page-locked" : "pageable");
    std::fflush(stdout);
  }
  storb_rs_ctx_destroy(ctx);
  return 0;
}
