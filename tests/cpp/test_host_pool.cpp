// CPU unit test of the host copy pool (storb_amd/csrc/host_pool.hpp) used by
// the pipelined host path: parallel copies are byte-exact at odd sizes and
// every part of a run() executes exactly once, repeatedly.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../storb_amd/csrc/host_pool.hpp"

int main() {
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
