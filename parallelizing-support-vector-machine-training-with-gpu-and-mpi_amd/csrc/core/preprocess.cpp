// L1 preprocessing, L2 kernel evaluation and L4 evaluation on the CPU.
//
//   svm_minmax   <- find_min_max   main3.cpp:57-71 (column-wise, first row seeds min/max)
//   svm_scale    <- scale_features main3.cpp:74-89 (range < 1e-12 -> 1; x = (x - min) / range)
//   svm_rbf      <- kernel         main3.cpp:92-104 (gamma is a parameter here, not hard-coded)
//   svm_decision <- predict loop   main3.cpp:391-402 (sum from -b over SVs in order)
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>
#include <sys/stat.h>

#include "internal.h"

using namespace svm355;

extern "C" {

SVM_API int svm_minmax(const double* X, int64_t n, int64_t d, double* mn, double* mx) {
  if (n <= 0 || d <= 0 || !X || !mn || !mx) {
    set_error("svm_minmax: bad arguments (n=%lld d=%lld)", (long long)n, (long long)d);
    return SVM_ERR_ARG;
  }
  for (int64_t j = 0; j < d; ++j) {
    mn[j] = X[j];
    mx[j] = X[j];
  }
  // Row-outer order (cache friendly); min/max are order independent so results are identical.
  std::vector<char> nan(static_cast<size_t>(d), 0);  // std::min / max drop a NaN that is not the seed
  for (int64_t i = 0; i < n; ++i) {
    const double* r = X + i * d;
    for (int64_t j = 0; j < d; ++j) {
      mn[j] = std::min(mn[j], r[j]);
      mx[j] = std::max(mx[j], r[j]);
      nan[size_t(j)] |= r[j] != r[j];
    }
  }
  for (int64_t j = 0; j < d; ++j)  // a NaN anywhere in a column: both bounds NaN (callers reject them)
    if (nan[size_t(j)]) mn[j] = mx[j] = std::nan("");
  return SVM_OK;
}

SVM_API int svm_scale(double* X, int64_t n, int64_t d, const double* mn, const double* mx) {
  if (n < 0 || d <= 0 || (n > 0 && !X) || !mn || !mx) {
    set_error("svm_scale: bad arguments");
    return SVM_ERR_ARG;
  }
  std::vector<double> range(static_cast<size_t>(d));
  for (int64_t j = 0; j < d; ++j) {
    double r = mx[j] - mn[j];
    if (r < 1e-12) r = 1.0;
    range[size_t(j)] = r;
  }
  for (int64_t i = 0; i < n; ++i) {
    double* r = X + i * d;
    for (int64_t j = 0; j < d; ++j) r[j] = (r[j] - mn[j]) / range[size_t(j)];
  }
  return SVM_OK;
}

SVM_API double svm_rbf(const double* a, const double* b, int64_t d, double gamma) {
  return rbf_direct(a, b, d, gamma);
}

SVM_API int svm_rbf_matrix(const double* A, int64_t m, const double* B, int64_t n, int64_t d,
                           double gamma, double* K, int32_t n_threads) {
  if (m < 0 || n < 0 || d <= 0 || !K) {
    set_error("svm_rbf_matrix: bad arguments");
    return SVM_ERR_ARG;
  }
  parallel_for(m, resolve_threads(n_threads), [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i)
      for (int64_t j = 0; j < n; ++j) K[i * n + j] = rbf_direct(A + i * d, B + j * d, d, gamma);
  });
  return SVM_OK;
}

SVM_API int svm_decision(const double* Xs, const int32_t* ys, const double* alphas, int64_t nsv,
                         const double* Xq, int64_t m, int64_t d, double gamma, double b,
                         double* out, int32_t n_threads) {
  if (m < 0 || nsv < 0 || d <= 0 || (m > 0 && (!Xq || !out))) {
    set_error("svm_decision: bad arguments");
    return SVM_ERR_ARG;
  }
  parallel_for(m, resolve_threads(n_threads), [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      double curr = -b;
      for (int64_t k = 0; k < nsv; ++k)
        curr += alphas[k] * ys[k] * rbf_direct(Xq + i * d, Xs + k * d, d, gamma);
      out[i] = curr;
    }
  });
  return SVM_OK;
}

SVM_API int64_t svm_sv_indices(const double* alpha, int64_t n, double tol, int64_t* out) {
  int64_t c = 0;
  for (int64_t i = 0; i < n; ++i)
    if (alpha[i] > tol) {
      if (out) out[c] = i;
      ++c;
    }
  return c;
}

SVM_API int svm_model_save(const char* dir, const int64_t* ids, const int32_t* labels,
                           const double* alphas, int64_t nsv, double b) {
  if (!dir) {
    set_error("svm_model_save: null dir");
    return SVM_ERR_ARG;
  }
  if (mkdir(dir, 0755) != 0 && errno != EEXIST) {
    set_error("svm_model_save: cannot create %s", dir);
    return SVM_ERR_IO;
  }
  const std::string base(dir);
  auto open = [&](const char* name) { return fopen((base + "/" + name).c_str(), "wb"); };
  FILE* fi = open("final_sv_ids.txt");
  FILE* fl = open("final_sv_labels.txt");
  FILE* fa = open("final_sv_alphas.txt");
  FILE* fb = open("final_b.txt");
  if (!fi || !fl || !fa || !fb) {
    for (FILE* f : {fi, fl, fa, fb})
      if (f) fclose(f);
    set_error("svm_model_save: cannot write model files in %s", dir);
    return SVM_ERR_IO;
  }
  // One value per line, as the reference's commented writers (mpi_svm_main3.cpp:754-770).
  // Alphas and b use %.17g so a reload is bit-exact.
  for (int64_t i = 0; i < nsv; ++i) {
    fprintf(fi, "%lld\n", (long long)ids[i]);
    fprintf(fl, "%d\n", labels[i]);
    fprintf(fa, "%.17g\n", alphas[i]);
  }
  fprintf(fb, "%.17g\n", b);
  for (FILE* f : {fi, fl, fa, fb}) fclose(f);
  return SVM_OK;
}

}  // extern "C"
