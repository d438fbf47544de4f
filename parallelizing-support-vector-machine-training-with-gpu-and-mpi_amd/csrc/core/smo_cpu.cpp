// L3 SMO solver on the CPU — the correctness oracle and the "serial" baseline.
//
// Keerthi et al. first-order working-set selection with Platt's two-variable update, exactly as
// SMO_train in main3.cpp:162-294 (cold start) and mpi_svm_main3.cpp:155-290 (warm start):
//   I_high = {y=+1, a<C-eps} U {y=-1, a>eps}, i_high = argmin f over I_high (lowest index on ties)
//   I_low  = {y=+1, a>eps}   U {y=-1, a<C-eps}, i_low  = argmax f over I_low  (lowest index on ties)
//   stop when b_low <= b_high + 2*tau, no candidate, infeasible [U,V], eta <= eps, or iterations
//   exceed max_iter; b = (b_high + b_low)/2.
// Kernel rows of i_high / i_low are recomputed only when the index changes (main3.cpp:216-232).
//
// Opt-in (svm_params.wss = 2, not the reference): second-order selection of the second index
// (Fan, Chen & Lin 2005, WSS 2).  i_high and the stop test stay first-order; then
//   j = argmin over t in I_low with f_t > f_{i_high} of  -(f_t - f_{i_high})^2 / a_t,
//   a_t = K(i,i) + K(t,t) - 2 K(i,t)  (K(t,t) = 1 for the RBF kernel; a_t <= 0 -> eps),
// lowest index on ties, and the pair (i_high, j) gets the same two-variable update.
// With n_threads > 1 the O(n) loops are split into static chunks; each element is computed by the
// same expression, and the argmin/argmax merge keeps the serial lowest-index rule, so the result is
// bit-identical to the serial run.
#include <chrono>
#include <cmath>
#include <limits>

#include "internal.h"

using namespace svm355;

namespace {

struct Pick {
  double v;
  int64_t i;
};

// Row providers: fill row[j] = K(i, j) for all j.
struct XRows {
  const double* X;
  int64_t d;
  double gamma;
  void fill(int64_t i, double* row, int64_t n, WorkerTeam& team) const {
    const double* xi = X + i * d;
    team.parallel_for(n, [&](int64_t lo, int64_t hi) {
      for (int64_t j = lo; j < hi; ++j) row[j] = rbf_direct(xi, X + j * d, d, gamma);
    });
  }
  // K(x_i, x_j) with x_i as the reference's first argument.
  double k(int64_t i, int64_t j) const { return rbf_direct(X + i * d, X + j * d, d, gamma); }
};

struct GramRows {
  const double* K;
  int64_t ldk;
  void fill(int64_t i, double* row, int64_t n, WorkerTeam&) const {
    const double* src = K + i * ldk;
    for (int64_t j = 0; j < n; ++j) row[j] = src[j];
  }
  double k(int64_t i, int64_t j) const { return K[i * ldk + j]; }
};

template <class Rows>
int smo_solve(const Rows& rows, const int32_t* y, int64_t n, double* alpha, int32_t warm,
              const svm_params* pp, svm_result* res, int64_t* trace, int64_t trace_cap) {
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  if (n <= 0 || !y || !alpha) {
    set_error("svm_smo_train: empty problem");
    return SVM_ERR_EMPTY;
  }
  const auto t0 = std::chrono::steady_clock::now();
  // Worker count: the requested threads, but at least kMinPerThread elements each (the passes are
  // a few ns per element; below that the fork/join of a pass costs more than it saves).  The
  // result does not depend on the count (static chunks, serial tie-break in the merge).
  constexpr int64_t kMinPerThread = 256;
  const int32_t nt = int32_t(std::max<int64_t>(1, std::min<int64_t>(std::max(1, p.n_threads), n / kMinPerThread)));
  WorkerTeam team(nt);
  const double C = p.C, eps = p.eps, tau = p.tau;
  std::vector<double> f(size_t(n), 0.0);

  if (!warm) {
    for (int64_t i = 0; i < n; ++i) alpha[i] = 0.0;
    for (int64_t i = 0; i < n; ++i) f[size_t(i)] = -static_cast<double>(y[i]);
  } else {
    // f_i = sum_{alpha_j != 0} alpha_j y_j K(x_j, x_i) - y_i, j ascending (mpi_svm_main3.cpp:169-186)
    std::vector<int64_t> nz;
    for (int64_t j = 0; j < n; ++j)
      if (alpha[j] != 0.0) nz.push_back(j);
    team.parallel_for(n, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) {
        double sum = 0.0;
        for (int64_t j : nz) sum += alpha[j] * y[j] * rows.k(j, i);
        f[size_t(i)] = sum - static_cast<double>(y[i]);
      }
    });
  }

  std::vector<double> Kh(size_t(n), 0.0), Kl(size_t(n), 0.0);
  int64_t i_high_prev = n, i_low_prev = n;
  double b_high = 0.0, b_low = 0.0;  // reference leaves these uninitialised before iteration 1
  int64_t num_iter = 1;
  int32_t stop = SVM_STOP_RUNNING;
  int64_t n_trace = 0;

  const int64_t nchunks = std::min<int64_t>(nt, n);
  std::vector<Pick> ph(static_cast<size_t>(nchunks)), pl(static_cast<size_t>(nchunks));

  while (true) {
    // --- working-set selection (calc_i_high / calc_i_low, main3.cpp:107-142)
    const int64_t chunk = (n + nchunks - 1) / nchunks;
    auto scan = [&](int64_t c) {
      const int64_t lo = c * chunk, hi = std::min(n, lo + chunk);
      Pick h{std::numeric_limits<double>::infinity(), n};
      Pick l{-std::numeric_limits<double>::infinity(), n};
      for (int64_t i = lo; i < hi; ++i) {
        const double a = alpha[i], fi = f[size_t(i)];
        const bool in_high = (y[i] == 1 && a < C - eps) || (y[i] == -1 && a > 0.0 + eps);
        const bool in_low = (y[i] == 1 && a > 0.0 + eps) || (y[i] == -1 && a < C - eps);
        if (in_high && fi < h.v) h = {fi, i};
        if (in_low && fi > l.v) l = {fi, i};
      }
      ph[size_t(c)] = h;
      pl[size_t(c)] = l;
    };
    if (nchunks == 1) {
      scan(0);
    } else {
      team.parallel_for(nchunks, [&](int64_t lo, int64_t hi) {
        for (int64_t c = lo; c < hi; ++c) scan(c);
      });
    }
    Pick h = ph[0], l = pl[0];
    for (int64_t c = 1; c < nchunks; ++c) {  // chunk order + strict compare = serial tie-break
      if (ph[size_t(c)].v < h.v) h = ph[size_t(c)];
      if (pl[size_t(c)].v > l.v) l = pl[size_t(c)];
    }
    const int64_t i_high = h.i, i_low = l.i;
    if (i_high >= n || i_low >= n) {
      stop = SVM_STOP_NO_CANDIDATE;
      break;
    }
    b_high = f[size_t(i_high)];
    b_low = f[size_t(i_low)];
    if (b_low <= b_high + 2.0 * tau) {
      stop = SVM_STOP_CONVERGED;
      break;
    }
    // --- kernel rows on change
    if (i_high != i_high_prev) {
      i_high_prev = i_high;
      rows.fill(i_high, Kh.data(), n, team);
    }
    int64_t i_low_upd = i_low;  // the second index of the update
    double f_low = b_low;
    if (p.wss == 2) {  // second-order choice of the second index (needs row i_high)
      const double K11 = Kh[size_t(i_high)];
      auto scan2 = [&](int64_t c) {
        const int64_t lo = c * chunk, hi = std::min(n, lo + chunk);
        Pick g{std::numeric_limits<double>::infinity(), n};
        for (int64_t t = lo; t < hi; ++t) {
          const double a = alpha[t], ft = f[size_t(t)];
          const bool in_low = (y[t] == 1 && a > 0.0 + eps) || (y[t] == -1 && a < C - eps);
          if (!in_low || !(ft > b_high)) continue;
          const double bb = ft - b_high;
          double at = K11 + 1.0 - 2.0 * Kh[size_t(t)];
          if (at <= 0.0) at = eps;
          const double gain = -(bb * bb) / at;
          if (gain < g.v) g = {gain, t};
        }
        pl[size_t(c)] = g;
      };
      if (nchunks == 1) {
        scan2(0);
      } else {
        team.parallel_for(nchunks, [&](int64_t lo, int64_t hi) {
          for (int64_t c = lo; c < hi; ++c) scan2(c);
        });
      }
      Pick g = pl[0];
      for (int64_t c = 1; c < nchunks; ++c)
        if (pl[size_t(c)].v < g.v) g = pl[size_t(c)];
      i_low_upd = g.i;  // exists: the first-order i_low has f > b_high + 2 tau
      f_low = f[size_t(i_low_upd)];
    }
    if (i_low_upd != i_low_prev) {
      i_low_prev = i_low_upd;
      rows.fill(i_low_upd, Kl.data(), n, team);
    }
    // --- two-variable update (main3.cpp:235-266)
    const int s = y[i_high] * y[i_low_upd];
    const double K11 = Kh[size_t(i_high)];
    const double K22 = Kl[size_t(i_low_upd)];
    const double K12 = Kh[size_t(i_low_upd)];
    const double eta = K11 + K22 - 2.0 * K12;
    const double ah = alpha[i_high], al = alpha[i_low_upd];
    double U, V;
    if (s == -1) {
      U = std::max(0.0, al - ah);
      V = std::min(C, C + al - ah);
    } else {
      U = std::max(0.0, al + ah - C);
      V = std::min(C, al + ah);
    }
    if (!(U <= V + 1e-12)) {
      stop = SVM_STOP_INFEASIBLE;
      break;
    }
    if (eta <= eps) {
      stop = SVM_STOP_NONPOS_ETA;
      break;
    }
    double al_new = al + y[i_low_upd] * (b_high - f_low) / eta;
    if (al_new > V) al_new = V;
    if (al_new < U) al_new = U;
    const double ah_new = ah + s * (al - al_new);
    // --- f update (main3.cpp:268-275): f_i += (dh*y_h)*Kh_i + (dl*y_l)*Kl_i
    const double dh = ah_new - ah, dl = al_new - al;
    const int32_t yh = y[i_high], yl = y[i_low_upd];
    team.parallel_for(n, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) f[size_t(i)] += dh * yh * Kh[size_t(i)] + dl * yl * Kl[size_t(i)];
    });
    alpha[i_high] = ah_new;
    alpha[i_low_upd] = al_new;
    if (trace && n_trace < trace_cap) {
      trace[2 * n_trace] = i_high;
      trace[2 * n_trace + 1] = i_low_upd;
      ++n_trace;
    }
    ++num_iter;
    if (num_iter > p.max_iter) {
      stop = SVM_STOP_MAX_ITER;
      break;
    }
  }

  if (res) {
    res->iterations = num_iter;
    res->b_high = b_high;
    res->b_low = b_low;
    res->b = (b_high + b_low) / 2;
    res->stop_reason = stop;
    res->reserved = 0;
    res->n_sv = svm_sv_indices(alpha, n, p.sv_tol, nullptr);
    res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  if (p.verbose && stop != SVM_STOP_CONVERGED) fprintf(stderr, "%s\n", svm_stop_message(stop));
  return SVM_OK;
}

}  // namespace

extern "C" {

SVM_API int svm_smo_train(const double* X, const int32_t* y, int64_t n, int64_t d, double* alpha,
                          int32_t warm, const svm_params* p, svm_result* r, int64_t* trace,
                          int64_t trace_cap) {
  if (!X || d <= 0) {
    set_error("svm_smo_train: bad X/d");
    return SVM_ERR_ARG;
  }
  XRows rows{X, d, p ? p->gamma : 0.00125};
  return smo_solve(rows, y, n, alpha, warm, p, r, trace, trace_cap);
}

SVM_API int svm_smo_train_gram(const double* K, int64_t ldk, const int32_t* y, int64_t n,
                               double* alpha, int32_t warm, const svm_params* p, svm_result* r,
                               int64_t* trace, int64_t trace_cap) {
  if (!K || ldk < n) {
    set_error("svm_smo_train_gram: bad K/ldk");
    return SVM_ERR_ARG;
  }
  GramRows rows{K, ldk};
  return smo_solve(rows, y, n, alpha, warm, p, r, trace, trace_cap);
}

}  // extern "C"
