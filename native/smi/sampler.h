// Periodic sampler thread + bounded ring buffer (host-only, header-only).
//
// The reference's only sampler is a Python loop that polls `nvidia-smi` every second into a
// DataFrame (pkg/profiler/parse_smi_metrics.py:23-42).  Here the amd-smi layer samples on a
// C++ thread into a ring that Python drains.  Kept free of amd-smi so the concurrency
// contract (start / stop / drain from any thread) is tested under ThreadSanitizer on the
// host: native/tests/sampler_tsan.cpp.
#pragma once
#include <atomic>
#include <chrono>
#include <cstddef>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace gs {

template <class T>
class PeriodicSampler {
 public:
  PeriodicSampler() = default;
  PeriodicSampler(const PeriodicSampler&) = delete;
  PeriodicSampler& operator=(const PeriodicSampler&) = delete;
  ~PeriodicSampler() { stop(); }

  // (Re)start: any running thread is stopped and joined first.
  void start(std::function<T()> fn, double period_s, int capacity) {
    std::lock_guard<std::mutex> life(life_mu_);
    stop_locked();
    {
      std::lock_guard<std::mutex> g(ring_mu_);
      cap_ = capacity > 0 ? static_cast<size_t>(capacity) : 600;
    }
    running_.store(true, std::memory_order_release);
    th_ = std::thread([this, fn = std::move(fn), period_s]() {
      const auto period = std::chrono::duration<double>(period_s > 0 ? period_s : 0.0);
      while (running_.load(std::memory_order_acquire)) {
        T v = fn();
        {
          std::lock_guard<std::mutex> g(ring_mu_);
          ring_.push_back(std::move(v));
          while (ring_.size() > cap_) ring_.pop_front();
          ++produced_;
        }
        const auto until = std::chrono::steady_clock::now() + period;
        while (running_.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < until)
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    });
  }

  void stop() {
    std::lock_guard<std::mutex> life(life_mu_);
    stop_locked();
  }

  bool running() const { return running_.load(std::memory_order_acquire); }

  std::vector<T> drain() {
    std::lock_guard<std::mutex> g(ring_mu_);
    std::vector<T> out(std::make_move_iterator(ring_.begin()), std::make_move_iterator(ring_.end()));
    ring_.clear();
    return out;
  }

  size_t produced() const {
    std::lock_guard<std::mutex> g(ring_mu_);
    return produced_;
  }

 private:
  void stop_locked() {
    running_.store(false, std::memory_order_release);
    if (th_.joinable()) th_.join();
  }

  std::mutex life_mu_;               // serialises start/stop (thread handle ownership)
  mutable std::mutex ring_mu_;       // ring, capacity, counter
  std::thread th_;
  std::atomic<bool> running_{false};
  std::deque<T> ring_;
  size_t cap_ = 600;
  size_t produced_ = 0;
};

}  // namespace gs
