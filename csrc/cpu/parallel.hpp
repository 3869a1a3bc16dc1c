// Dynamic work distribution over std::threads for the batch entry points: one
// atomic ticket counter, each worker pulls the next policy index.  Workers
// share only read-only inputs (Workload, Programs) and write disjoint output
// rows, so the batch is race-free by construction; the ThreadSanitizer build
// of csrc/cpu/selftest.cpp (tools/sanitize_cpu.py --tsan) checks exactly that.
#pragma once

#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

namespace fks {

template <class Fn>
void parallel_for(int64_t n, int threads, Fn fn) {
  if (threads <= 1 || n <= 1) { for (int64_t i = 0; i < n; ++i) fn(i); return; }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&] { for (int64_t i; (i = next.fetch_add(1)) < n;) fn(i); });
  for (auto& th : pool) th.join();
}

}  // namespace fks
