// host_pool.hpp -- a small persistent worker pool for the host-side copies
// around the device (pageable caller buffers <-> pinned staging).
//
// One host thread copies ~15-20 GB/s; the pipelined host path moves
// 1.5 x the input through memcpy (pack in, unpack parity), so a single
// thread capped it near 10 GiB/s of input. Splitting each copy over a few
// threads lets the PCIe DMA become the bound instead.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace storb_rs {

// A byte range to copy (src != nullptr) or to zero-fill (src == nullptr).
// (Non-temporal stores for the copies into staging were measured and not
// kept: equal at 1 MiB calls, slower at 8 MiB -- (16, 24) encode 315 ->
// 380 us -- tools/callprobe.cpp, profiles/r3u_copy_split_nt_ab.txt.)
struct CopySeg {
  uint8_t *dst;
  const uint8_t *src;
  size_t len;
};

// memcpy with non-temporal 32-byte stores (AVX2; plain memcpy without it or
// below 256 KiB): no read-for-ownership of the destination lines. The batch
// pipelines (host_batch.cpp) copy this way into staging and into the
// caller's output: pageable batch decode 18-25 -> 32-35 GiB/s, encode equal
// (tools/gpu/hostpath_ab.sh, profiles/r5nt_hostpath_nt_ab.jsonl, staging
// only, and r5nt_hostpath_nt_output_ab.jsonl, output rows too). The
// single-chunk calls keep memcpy (their 8 MiB encode lost with NT stores,
// below).
#if defined(__x86_64__)
__attribute__((target("avx2"))) inline void nt_copy_avx2(uint8_t *d, const uint8_t *s, size_t n) {
  size_t head = (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31;
  if (head > n) head = n;
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  const size_t m = n & ~static_cast<size_t>(127);
  for (size_t i = 0; i < m; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 96), e);
  }
  std::memcpy(d + m, s + m, n - m);
  _mm_sfence();
}
#endif
inline void copy_nt(void *dst, const void *src, size_t n) {
#if defined(__x86_64__)
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2 && n >= (256u << 10)) {
    nt_copy_avx2(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
    return;
  }
#endif
  std::memcpy(dst, src, n);
}


class HostPool {
 public:
  explicit HostPool(int nthreads, int spin_us = 60) : spin_us_(spin_us) {
    for (int i = 1; i < nthreads; i++) workers_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  HostPool(const HostPool &) = delete;
  HostPool &operator=(const HostPool &) = delete;

  int size() const { return static_cast<int>(workers_.size()) + 1; }

  // f(i) for every i in [0, parts); the caller takes part too. Blocking.
  // Workers that finished a job spin for spin_us before sleeping, so the
  // back-to-back jobs of one call (pack, launch, unpack of each slice) start
  // without a futex wake-up each (~5-20 us on a busy host).
  void run(int parts, const std::function<void(int)> &f) {
    if (parts <= 0) return;
    if (parts == 1 || workers_.empty()) {
      for (int i = 0; i < parts; i++) f(i);
      return;
    }
    bool wake;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      parts_ = parts;
      next_ = 0;
      done_.store(0, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
      wake = sleepers_ > 0;
    }
    if (wake) cv_.notify_all();
    work();
    for (unsigned spin = 0; done_.load(std::memory_order_acquire) != parts; spin++)
      if (spin > 4096) std::this_thread::yield();
    std::lock_guard<std::mutex> lk(mu_);
    job_ = nullptr;
  }

  // memcpy split over the pool (copy_segs' rule).
  void copy(void *dst, const void *src, size_t bytes, bool nt = false) {
    CopySeg s{static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), bytes};
    copy_segs(&s, 1, nt);
  }

  // How many threads a copy of `total` bytes into page-locked memory takes.
  // Measured (the removed poolbench, profiles/r3_poolbench.txt, GPU-box host):
  // one thread copies 256 KiB in 1.7 us and 1 MiB in 21 us; two threads 1 MiB
  // in 5.2 us, while 4 or 8 (waking, claiming parts) took 13-20 us; from
  // 4 MiB on 8 threads win (28-35 us against 44 for two, 84 for one). Inside
  // the single-chunk calls (the source hot in the caller's cache, the
  // staging just read by the GPU) one thread packed a 512 KiB slice in
  // 6.8 us against 13.2 with two and 13-14 with four or eight
  // (tools/callprobe.cpp stage marks, profiles/r3m_calltrace.txt): jobs up
  // to 1 MiB stay on the calling thread.
  int parts_for(size_t total) const {
#ifdef STORB_RS_FORCE_PARTS  // A/B builds of tools/callprobe.cpp only
    return std::max(1, std::min(STORB_RS_FORCE_PARTS, size()));
#endif
    if (total <= (1u << 20)) return 1;
    if (total < (4u << 20)) return std::min(2, size());
    return static_cast<int>(std::max<size_t>(2, std::min<size_t>(size(), total / (512u << 10))));
  }

  // Copy / zero-fill a list of byte ranges, the total split evenly over
  // parts_for(total) threads.
  void copy_segs(const CopySeg *segs, size_t nsegs, bool nt = false) {
    size_t total = 0;
    for (size_t i = 0; i < nsegs; i++) total += segs[i].len;
    if (total == 0) return;
    const int parts = parts_for(total);
    const size_t per = ((total + parts - 1) / parts + 63) & ~static_cast<size_t>(63);
    run(parts, [&](int p) {
      size_t lo = std::min(total, static_cast<size_t>(p) * per), hi = std::min(total, lo + per);
      size_t base = 0;
      for (size_t i = 0; i < nsegs && lo < hi; i++) {
        const CopySeg &sg = segs[i];
        if (base + sg.len > lo) {
          const size_t a = lo - base, b = std::min(sg.len, hi - base);
          if (sg.src && nt) copy_nt(sg.dst + a, sg.src + a, b - a);
          else if (sg.src) std::memcpy(sg.dst + a, sg.src + a, b - a);
          else std::memset(sg.dst + a, 0, b - a);
          lo = base + b;
        }
        base += sg.len;
      }
    });
  }

 private:
  const int spin_us_;  // how long a worker spins for the next job before sleeping

  void work() {
    for (;;) {
      int i;
      const std::function<void(int)> *f;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!job_ || next_ >= parts_) return;
        i = next_++;
        f = job_;
      }
      (*f)(i);
      done_.fetch_add(1, std::memory_order_acq_rel);
    }
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned spin = 1; gen_.load(std::memory_order_acquire) == seen; spin++) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        if ((spin & 255) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_))
          break;
      }
      {
        std::unique_lock<std::mutex> lk(mu_);
        sleepers_++;
        cv_.wait(lk, [&] { return gen_.load() != seen; });
        sleepers_--;
        if (stop_.load()) return;
        seen = gen_.load();
      }
      work();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  const std::function<void(int)> *job_ = nullptr;
  int parts_ = 0, next_ = 0, sleepers_ = 0;
  std::atomic<int> done_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

}  // namespace storb_rs
