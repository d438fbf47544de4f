// Internal helpers shared by the CPU core translation units (not part of the C ABI).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "svm355.h"

namespace svm355 {

// Thread-local last-error string surfaced through svm_last_error().
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Static-partition parallel for over [0, n): fn(begin, end). Deterministic partitioning,
// so any per-element result is independent of the thread count.
template <class F>
void parallel_for(int64_t n, int32_t n_threads, F&& fn) {
  if (n <= 0) return;
  int64_t t = std::max<int32_t>(1, n_threads);
  if (t > n) t = n;
  if (t == 1) {
    fn(int64_t(0), n);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(size_t(t - 1));
  const int64_t chunk = (n + t - 1) / t;
  for (int64_t w = 1; w < t; ++w) {
    const int64_t b = w * chunk, e = std::min(n, b + chunk);
    if (b < e) pool.emplace_back([&fn, b, e] { fn(b, e); });
  }
  fn(int64_t(0), std::min(n, chunk));
  for (auto& th : pool) th.join();
}

// Persistent worker team for loops that run many short parallel passes (an SMO iteration does two
// or three O(n) passes).  Spawning std::threads per pass costs tens of microseconds per thread,
// more than the pass itself; on a many-core host that turned a 1.5k-row solve into minutes.
// parallel_for() uses the same static partition as the free function above, so results are
// bit-identical to it and to the serial run.  Every worker runs every job (an empty range if it
// has no chunk) and checks in, so no worker can read the fields of a later job early.
class WorkerTeam {
 public:
  explicit WorkerTeam(int32_t n_threads) : nt_(std::max<int32_t>(1, n_threads)) {
    th_.reserve(size_t(nt_ - 1));
    for (int32_t w = 1; w < nt_; ++w) th_.emplace_back([this, w] { loop(w); });
  }
  ~WorkerTeam() {
    stop_.store(true, std::memory_order_relaxed);
    gen_.fetch_add(1, std::memory_order_release);
    for (auto& t : th_) t.join();
  }
  WorkerTeam(const WorkerTeam&) = delete;
  WorkerTeam& operator=(const WorkerTeam&) = delete;
  int32_t size() const { return nt_; }

  template <class F>
  void parallel_for(int64_t n, F&& fn) {
    if (n <= 0) return;
    const int64_t t = std::min<int64_t>(nt_, n);
    if (t == 1) {
      fn(int64_t(0), n);
      return;
    }
    const int64_t chunk = (n + t - 1) / t;
    auto body = [&](int32_t w) {
      const int64_t b = int64_t(w) * chunk, e = std::min(n, b + chunk);
      if (b < e) fn(b, e);
    };
    job_ctx_ = &body;
    job_fn_ = [](void* c, int32_t w) { (*static_cast<decltype(body)*>(c))(w); };
    pending_.store(nt_ - 1, std::memory_order_relaxed);
    gen_.fetch_add(1, std::memory_order_release);
    body(0);
    while (pending_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }

 private:
  void loop(int32_t w) {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g;
      int spins = 0;
      while ((g = gen_.load(std::memory_order_acquire)) == seen) {
        if (spins < 2048)
          ++spins;
        else
          std::this_thread::yield();
      }
      seen = g;
      if (stop_.load(std::memory_order_relaxed)) return;
      job_fn_(job_ctx_, w);
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  int32_t nt_;
  std::vector<std::thread> th_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int32_t> pending_{0};
  std::atomic<bool> stop_{false};
  void* job_ctx_ = nullptr;
  void (*job_fn_)(void*, int32_t) = nullptr;
};

inline int32_t resolve_threads(int32_t n_threads) {
  if (n_threads > 0) return n_threads;
  const unsigned hc = std::thread::hardware_concurrency();
  return hc ? int32_t(std::min(hc, 64u)) : 1;
}

// Reference RBF: exp(-gamma * sum_k (a_k - b_k)^2), summed in ascending k (main3.cpp:92-104).
inline double rbf_direct(const double* a, const double* b, int64_t d, double gamma) {
  double res = 0.0;
  for (int64_t k = 0; k < d; ++k) {
    const double t = a[k] - b[k];
    res += t * t;
  }
  return __builtin_exp(-gamma * res);
}

}  // namespace svm355
