// CPU unit test of the host copy pool (storb_amd/csrc/host_pool.hpp) used by
// the pipelined host path: parallel copies are byte-exact at odd sizes and
// every part of a run() executes exactly once, repeatedly.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../storb_amd/csrc/host_pool.hpp"

// copy_stream (non-temporal stores into staging): exact at every destination
// / source misalignment and length around the 4 KiB and 128-byte edges, no
// byte written outside [dst, dst + n); and copy_segs with nt segments.
static int check_copy_stream() {
  std::vector<unsigned char> src(70000), dst(70100);
  for (size_t i = 0; i < src.size(); i++) src[i] = static_cast<unsigned char>(i * 37 + 11);
  for (size_t doff : {0, 1, 15, 31, 32, 33}) {
    for (size_t soff : {0, 3, 32}) {
      for (size_t n : {0, 1, 127, 4095, 4096, 4097, 4096 + 127, 65536, 65536 + 33}) {
        std::fill(dst.begin(), dst.end(), 0xEE);
        storb_rs::copy_stream(dst.data() + doff, src.data() + soff, n);
        for (size_t i = 0; i < dst.size(); i++) {
          const bool in = i >= doff && i < doff + n;
          const unsigned char want = in ? src[soff + i - doff] : 0xEE;
          if (dst[i] != want) {
            std::printf("copy_stream mismatch doff=%zu soff=%zu n=%zu at %zu\n", doff, soff, n, i);
            return 1;
          }
        }
      }
    }
  }
  storb_rs::HostPool pool(4);
  std::vector<unsigned char> d2(3u << 20, 0xEE);
  std::vector<storb_rs::CopySeg> segs;
  segs.push_back({d2.data() + 5, src.data(), 60000, true});
  segs.push_back({d2.data() + 70000, nullptr, 5000});
  segs.push_back({d2.data() + 80000, src.data() + 7, 50000, false});
  pool.copy_segs(segs.data(), segs.size());
  for (size_t i = 0; i < 60000; i++)
    if (d2[5 + i] != src[i]) return std::printf("copy_segs nt mismatch at %zu\n", i), 1;
  for (size_t i = 0; i < 5000; i++)
    if (d2[70000 + i] != 0) return std::printf("copy_segs zero mismatch at %zu\n", i), 1;
  for (size_t i = 0; i < 50000; i++)
    if (d2[80000 + i] != src[7 + i]) return std::printf("copy_segs mismatch at %zu\n", i), 1;
  if (d2[4] != 0xEE || d2[60005] != 0xEE) return std::printf("copy_segs overrun\n"), 1;
  return 0;
}

int main() {
  if (check_copy_stream()) return 1;
  for (int threads : {1, 3, 8}) {
    storb_rs::HostPool pool(threads);
    for (size_t bytes : {size_t(0), size_t(1), size_t(4095), size_t(1) << 20,
                         (size_t(5) << 20) + 7, (size_t(33) << 20) + 4097}) {
      std::vector<unsigned char> src(bytes + 1), dst(bytes + 1, 0xEE);
      for (size_t i = 0; i < bytes; i++) src[i] = static_cast<unsigned char>(i * 131 + 7);
      pool.copy(dst.data(), src.data(), bytes);
      for (size_t i = 0; i < bytes; i++)
        if (dst[i] != src[i]) {
          std::printf("copy mismatch threads=%d bytes=%zu at %zu\n", threads, bytes, i);
          return 1;
        }
      if (dst[bytes] != 0xEE) {
        std::printf("copy overrun threads=%d bytes=%zu\n", threads, bytes);
        return 1;
      }
    }
    for (int rep = 0; rep < 200; rep++) {
      const int parts = 1 + rep % 37;
      std::vector<std::atomic<int>> hits(parts);
      for (auto &h : hits) h = 0;
      pool.run(parts, [&](int i) { hits[i]++; });
      for (int i = 0; i < parts; i++)
        if (hits[i] != 1) {
          std::printf("run part %d executed %d times (threads=%d)\n", i, hits[i].load(),
                      threads);
          return 1;
        }
    }
  }
  std::printf("host pool ok\n");
  return 0;
}
