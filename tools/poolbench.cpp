// poolbench.cpp -- host copy rates into page-locked staging: one thread vs
// the HostPool (host_pool.hpp) at several sizes, thread counts and spin
// windows, back to back and with a gap between jobs (the kernel's time in a
// single call). Picks the single-call pack/unpack split (host_calls.cpp).
// build: hipcc -O3 -std=c++17 -pthread tools/poolbench.cpp -o tools/_build/poolbench
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../storb_amd/csrc/host_pool.hpp"

using clk = std::chrono::steady_clock;

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const size_t sizes[] = {128u << 10, 256u << 10, 512u << 10, 1u << 20, 4u << 20};
  std::vector<uint8_t> src(8u << 20, 0x5A);
  uint8_t *dst = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&dst), 8u << 20, hipHostMallocDefault) != hipSuccess) return 1;
  std::memset(dst, 0, 8u << 20);
  for (int gap_us : {0, 20}) {
    for (size_t n : sizes) {
      // one thread
      std::vector<double> t1;
      for (int i = 0; i < 400; i++) {
        if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
        auto a = clk::now();
        std::memcpy(dst, src.data(), n);
        t1.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
      }
      std::printf("gap %2d us  %5zu KiB  1 thread memcpy  %7.2f us  %6.1f GB/s\n", gap_us, n >> 10,
                  median(t1), n / median(t1) / 1e3);
      for (int th : {2, 4, 8}) {
        for (int spin : {0, 60}) {
          for (size_t minp : {size_t(0)}) {
            storb_rs::HostPool pool(th, spin);
            std::vector<double> t;
            for (int i = 0; i < 400; i++) {
              if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
              storb_rs::CopySeg sg{dst, src.data(), n};
              auto a = clk::now();
              pool.copy_segs(&sg, 1);
              t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
            }
            std::printf("gap %2d us  %5zu KiB  pool %d thr spin %2d (parts_for %zu)  %7.2f us  %6.1f GB/s\n",
                        gap_us, n >> 10, th, spin, minp + pool.parts_for(n), median(t), n / median(t) / 1e3);
          }
        }
      }
    }
  }
  hipHostFree(dst);
  return 0;
}
