// Internal helpers shared by the CPU core translation units (not part of the C ABI).
#pragma once
#include <algorithm>
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
