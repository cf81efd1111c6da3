// host_pool.hpp -- a small persistent worker pool for the host-side copies
// around the device (pageable caller buffers <-> pinned staging).
//
// One host thread copies ~15-20 GB/s; the pipelined host path moves
// 1.5 x the input through memcpy (pack in, unpack parity), so a single
// thread capped it near 10 GiB/s of input. Splitting each copy over a few
// threads lets the PCIe DMA become the bound instead.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace storb_rs {

class HostPool {
 public:
  explicit HostPool(int nthreads) {
    for (int i = 1; i < nthreads; i++) workers_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  HostPool(const HostPool &) = delete;
  HostPool &operator=(const HostPool &) = delete;

  int size() const { return static_cast<int>(workers_.size()) + 1; }

  // f(i) for every i in [0, parts); the caller takes part too. Blocking.
  void run(int parts, const std::function<void(int)> &f) {
    if (parts <= 0) return;
    if (parts == 1 || workers_.empty()) {
      for (int i = 0; i < parts; i++) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      parts_ = parts;
      next_ = 0;
      done_ = 0;
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return done_ == parts_; });
    job_ = nullptr;
  }

  // memcpy split into >= 1 MiB slices over the pool.
  void copy(void *dst, const void *src, size_t bytes) {
    constexpr size_t kSlice = 1u << 20;
    const int parts = static_cast<int>(std::min<size_t>(size(), (bytes + kSlice - 1) / kSlice));
    if (parts <= 1) {
      std::memcpy(dst, src, bytes);
      return;
    }
    const size_t per = ((bytes + parts - 1) / parts + 4095) & ~static_cast<size_t>(4095);
    run(parts, [&](int i) {
      const size_t off = std::min(bytes, static_cast<size_t>(i) * per);
      const size_t cnt = std::min(per, bytes - off);
      if (cnt) std::memcpy(static_cast<uint8_t *>(dst) + off,
                           static_cast<const uint8_t *>(src) + off, cnt);
    });
  }

 private:
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
      std::lock_guard<std::mutex> lk(mu_);
      if (++done_ == parts_) done_cv_.notify_all();
    }
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)> *job_ = nullptr;
  int parts_ = 0, next_ = 0, done_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace storb_rs
