// Newton polish of a working set's free variables: the decomposition solver's end-game step, shared
// by the device solver (csrc/hip/decomp.hip, ws_newton_kernel) and its CPU oracle
// (csrc/core/decomp_cpu.cpp), which must stay bit-identical.
//
// Why.  The reference's SMO (main3.cpp:162-294) moves two variables per iteration.  Near the optimum
// the set of free support vectors (0 < alpha < C) no longer changes, and what is left is to equalise
// their f on the unknown b.  Pairwise steps do that at a linear rate: on the 60k headline solve the last
// 5 working sets take 6,868 of the 9,641 pair updates (71 %), with all 339 final free points already in
// them and the gap going from 0.05 to 7e-5 (CPU oracle, outer iterations 24-28).  With the free set F
// fixed, the rest is one linear system: for the signed changes u_j = dalpha_j y_j (j in F),
//     K_FF u - b 1 = -f_F,   1^T u = 0
// (f_F + K_FF u = b on F keeps every free point at the same f; 1^T u = y^T dalpha = 0 keeps the
// equality constraint).  With K_FF = L L^T (Cholesky), x1 = K_FF^-1 f_F, x2 = K_FF^-1 1:
//     b = 1^T x1 / 1^T x2,   u = b x2 - x1.
// The full step solves the QP restricted to F; if it would leave the box, the step is cut at the first
// bound (t < 1, lowest position on ties) and that variable lands on its bound.  The objective is convex
// along the step, so every cut still decreases it.  The working set's f is updated with the realised
// changes, and the pairwise SMO continues from there (new free points, bounded violators, the stop).
//
// When.  Inside the inner solve, once `every` iterations of the pairwise chain have passed without any
// updated point changing its bound status (the free set has settled), at most per_solve times; a step
// cut at a bound is repeated up to `repeat` steps; and right at the start of the inner solve when the
// previous one needed at least frac x m pair updates (the end game).  F must have 2 <= |F| <= max_free.
// On the 60k headline (CPU oracle) this takes the pair updates from 9,760 to ~4,200-4,700 with 14-20
// steps, in the last five working sets.
//
// Arithmetic (the bit-identity contract): the Cholesky is left-looking, every entry
//     s = A_ik;  for j = 0 .. k-1: s = fma(-L_ij, L_kj, s);  L_ik = s / L_kk  (L_kk = sqrt(s))
// in ascending j; the two right-hand sides are two extra rows of the same factorisation (so z = L^-1 r
// comes out of the same loop); the back substitution is column-oriented, j = nf-1 .. 0, each
// s_i = fma(-L_ji, x_j, s_i); the sums of x1 and x2 are sequential in ascending order; u_k = fma(b, x2_k,
// -x1_k); f_q += sum_k fma(K(q, F_k), ur_k, .) in ascending k.  The device kernel blocks the loops but
// applies every entry's operations in this order.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <limits>
#include <vector>

#include "svm355.h"

namespace svm355 {

struct NewtonCfg {
  bool on = false;         // opt-in (SVM355_DECOMP_NEWTON=1): a net loss on the headline, see below
  double frac = 0.5;       // a step at the start of the inner solve when the last one needed >= frac x m
  int32_t every = 50;      // a step after `every` chain iterations with no point changing its bound status
  int32_t per_solve = 8;   // at most this many triggers per inner solve
  int32_t repeat = 2;      // a trigger repeats the step while it is cut at a bound, up to this many steps
  int32_t max_free = 640;  // |F| above this: no step (the factorisation costs |F|^3 / 6 FMAs)
};

// Off by default.  The device step (newton_wg) costs ~0.67 ms at |F| = 302 (probe; ~0.86 ms in situ), and
// the inner-solve variant compiled with it (NWT) costs ~0.8 us more per pair update even when no step runs
// (its SGPR spills), against ~1.6 us per pair update saved: on the 60k headline 16 steps take the pair
// updates from 9,760 to 4,532 and the fit from 21.4 to 29.9 ms (profiles/newton.md).
// SVM355_DECOMP_NEWTON=1 turns the step on; SVM355_DECOMP_NEWTON_{FRAC,EVERY,PER_SOLVE,REPEAT,MAX} tune
// it (A/B runs; both sides read the same variables).
inline NewtonCfg newton_cfg(const svm_params& p) {
  (void)p;
  NewtonCfg c;
  if (const char* v = std::getenv("SVM355_DECOMP_NEWTON")) c.on = std::atoi(v) != 0;
  if (const char* v = std::getenv("SVM355_DECOMP_NEWTON_FRAC")) c.frac = std::max(0.0, std::atof(v));
  if (const char* v = std::getenv("SVM355_DECOMP_NEWTON_EVERY")) c.every = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("SVM355_DECOMP_NEWTON_PER_SOLVE")) c.per_solve = std::max(0, std::atoi(v));
  if (const char* v = std::getenv("SVM355_DECOMP_NEWTON_REPEAT")) c.repeat = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("SVM355_DECOMP_NEWTON_MAX")) c.max_free = std::max(2, std::min(1024, std::atoi(v)));
  return c;
}

// The inner solve's counter of chain iterations without a bound-status change starts at `every` (a step
// before the first pair) when the last inner solve was long.
inline int32_t newton_since0(const NewtonCfg& c, int64_t last_inner_it, int last_m) {
  return c.on && last_m > 0 && double(last_inner_it) >= c.frac * double(last_m) ? c.every : 0;
}

// A point's bound status: 0 at the lower bound, 2 at the upper, 1 free (the sets' eps thresholds).
inline int bound_status(double a, double C, double eps) { return a <= 0.0 + eps ? 0 : a >= C - eps ? 2 : 1; }

// The step on a working set of m points (host reference; the CPU oracle runs it as is).  a, f, yw: the
// working set's alpha, f and labels by position; Kw(q, k) the kernel value of positions q and k (row q,
// column k of K(W, W): the device reads rows F_i for K_FF and rows F_k for the f update).
// Returns 0 when no step was applied, 1 for a full step, 2 for a step cut at a bound (a and f updated).
template <class KFn>
int newton_step_ref(int m, double* a, double* f, const int32_t* yw, KFn&& Kw, double C, double eps, int32_t max_free) {
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  std::vector<int> F;
  for (int k = 0; k < m; ++k)
    if (a[k] > c_lo && a[k] < c_hi) F.push_back(k);
  const int nf = int(F.size());
  if (nf < 2 || nf > max_free) return 0;
  // rows 0 .. nf-1: K_FF (lower); rows nf, nf+1: the right-hand sides f_F and 1
  std::vector<double> A(size_t(nf + 2) * nf, 0.0);
  for (int i = 0; i < nf; ++i)
    for (int k = 0; k <= i; ++k) A[size_t(i) * nf + k] = Kw(F[i], F[k]);
  for (int k = 0; k < nf; ++k) {
    A[size_t(nf) * nf + k] = f[F[k]];
    A[size_t(nf + 1) * nf + k] = 1.0;
  }
  for (int k = 0; k < nf; ++k) {
    double s = A[size_t(k) * nf + k];
    for (int j = 0; j < k; ++j) s = std::fma(-A[size_t(k) * nf + j], A[size_t(k) * nf + j], s);
    if (!(s > 1e-12)) return 0;  // not positive definite in working precision (e.g. duplicate rows)
    const double lkk = std::sqrt(s);
    A[size_t(k) * nf + k] = lkk;
    for (int i = k + 1; i < nf + 2; ++i) {
      double t = A[size_t(i) * nf + k];
      for (int j = 0; j < k; ++j) t = std::fma(-A[size_t(i) * nf + j], A[size_t(k) * nf + j], t);
      A[size_t(i) * nf + k] = t / lkk;
    }
  }
  std::vector<double> s1(A.begin() + size_t(nf) * nf, A.begin() + size_t(nf + 1) * nf);
  std::vector<double> s2(A.begin() + size_t(nf + 1) * nf, A.begin() + size_t(nf + 2) * nf);
  std::vector<double> x1(static_cast<size_t>(nf)), x2(static_cast<size_t>(nf));
  for (int j = nf - 1; j >= 0; --j) {
    const double ljj = A[size_t(j) * nf + j];
    x1[size_t(j)] = s1[size_t(j)] / ljj;
    x2[size_t(j)] = s2[size_t(j)] / ljj;
    for (int i = 0; i < j; ++i) {
      s1[size_t(i)] = std::fma(-A[size_t(j) * nf + i], x1[size_t(j)], s1[size_t(i)]);
      s2[size_t(i)] = std::fma(-A[size_t(j) * nf + i], x2[size_t(j)], s2[size_t(i)]);
    }
  }
  double S1 = 0.0, S2 = 0.0;
  for (int k = 0; k < nf; ++k) {
    S1 += x1[size_t(k)];
    S2 += x2[size_t(k)];
  }
  if (!(S2 > 0.0) || !std::isfinite(S1)) return 0;
  const double b = S1 / S2;
  double t = 1.0;
  int blk = -1;
  std::vector<double> d(static_cast<size_t>(nf));
  for (int k = 0; k < nf; ++k) {
    const double u = std::fma(b, x2[size_t(k)], -x1[size_t(k)]);
    d[size_t(k)] = yw[F[k]] == 1 ? u : -u;  // dalpha = y u
    const double ak = a[F[k]], dk = d[size_t(k)];
    const double tk = dk > 0.0 ? (C - ak) / dk : dk < 0.0 ? (0.0 - ak) / dk : std::numeric_limits<double>::infinity();
    if (tk < t) {
      t = tk;
      blk = k;
    }
  }
  std::vector<double> ur(static_cast<size_t>(nf));
  for (int k = 0; k < nf; ++k) {
    const double ak = a[F[k]], dk = d[size_t(k)];
    double an = k == blk ? (dk > 0.0 ? C : 0.0) : std::fma(t, dk, ak);
    an = std::min(C, std::max(0.0, an));
    ur[size_t(k)] = yw[F[k]] == 1 ? an - ak : ak - an;  // (an - ak) y
    a[F[k]] = an;
  }
  for (int q = 0; q < m; ++q) {
    double s = 0.0;
    for (int k = 0; k < nf; ++k) s = std::fma(Kw(F[k], q), ur[size_t(k)], s);
    f[q] += s;
  }
  return blk >= 0 ? 2 : 1;
}

}  // namespace svm355
