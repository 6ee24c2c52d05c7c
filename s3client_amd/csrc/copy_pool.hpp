// copy_pool.hpp -- host threads that fill pinned staging from pageable part memory or file
// ranges (one task per part slice).  DMA straight from pageable memory goes through the
// runtime's bounce buffer and serialises with the host; staging keeps the copy engine fed
// from pinned memory.  HIP-free (the host-concurrency sanitizer build runs it).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "topology.hpp"

namespace s3h::host {

class CopyPool {
 public:
  // `workers` threads beside the caller, bound to place.cpus (the device's node) when that set
  // is non-empty.
  CopyPool(unsigned workers, const Place& place) : bound_(place.ncpus > 0 ? place.node : -1) {
    for (unsigned i = 0; i < workers; ++i)
      threads_.emplace_back([this, place] {
        bind_self(place);
        loop();
      });
  }
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  int bound_node() const { return bound_; }
  unsigned size() const { return unsigned(threads_.size()); }
  // fn(i) for every i in [0, n), on the workers and the calling thread; returns when every
  // call has returned.  One run at a time per pool (callers serialise: a pool belongs to one
  // host context, or is taken under a lock).  fn must not throw.
  void run(uint64_t n, const std::function<void(uint64_t)>& fn) {
    {
      std::lock_guard<std::mutex> l(m_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      busy_ = threads_.size();
      ++gen_;
    }
    cv_.notify_all();
    work(&fn, n);
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work(const std::function<void(uint64_t)>* fn, uint64_t n) {
    for (uint64_t i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(uint64_t)>* fn;
      uint64_t n;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        fn = fn_;  // read under the lock: the run that published them
        n = n_;
      }
      work(fn, n);
      std::lock_guard<std::mutex> l(m_);
      if (--busy_ == 0) done_.notify_one();
    }
  }
  int bound_ = -1;
  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(uint64_t)>* fn_ = nullptr;
  std::atomic<uint64_t> next_{0};
  uint64_t n_ = 0, gen_ = 0;
  size_t busy_ = 0;
  bool stop_ = false;
};

}  // namespace s3h::host
