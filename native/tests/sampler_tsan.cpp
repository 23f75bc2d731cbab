// ThreadSanitizer test of the telemetry sampler (-fsanitize=thread variant of
// the host code).  A producer thread samples into the ring while readers drain it and a
// controller restarts / stops the sampler; TSan aborts the process on any data race.
//   g++ -std=c++17 -O1 -g -fsanitize=thread -pthread -Inative/smi native/tests/sampler_tsan.cpp
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "sampler.h"

int main() {
  gs::PeriodicSampler<std::vector<int>> s;
  std::atomic<int> seq{0};
  auto fn = [&seq]() { return std::vector<int>(4, seq.fetch_add(1)); };
  std::atomic<bool> done{false};
  std::atomic<size_t> drained{0};
  s.start(fn, 0.0005, 64);
  std::vector<std::thread> readers;
  for (int r = 0; r < 3; ++r)
    readers.emplace_back([&]() {
      while (!done.load()) {
        for (auto& v : s.drain()) {
          if (v.size() != 4 || v[0] != v[3]) {
            std::fprintf(stderr, "torn sample\n");
            std::abort();
          }
          drained.fetch_add(1);
        }
        std::this_thread::yield();
      }
    });
  std::thread controller([&]() {
    for (int i = 0; i < 20; ++i) {
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      if (i % 3 == 0) s.stop(); else s.start(fn, 0.0005, 16 + i);
    }
  });
  controller.join();
  s.start(fn, 0.0005, 64);
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  s.stop();
  done.store(true);
  for (auto& t : readers) t.join();
  drained += s.drain().size();
  if (drained.load() == 0 || drained.load() > s.produced()) {
    std::fprintf(stderr, "bad counts drained=%zu produced=%zu\n", drained.load(), s.produced());
    return 1;
  }
  std::printf("ok drained=%zu produced=%zu\n", drained.load(), s.produced());
  return 0;
}
