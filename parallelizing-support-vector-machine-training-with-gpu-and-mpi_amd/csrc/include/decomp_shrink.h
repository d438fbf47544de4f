// Shrinking (an active set) of the working-set decomposition solver: the one schedule and rule that
// the device solver (csrc/hip/decomp.hip) and its CPU oracle (csrc/core/decomp_cpu.cpp) share, so the
// two trajectories stay bit-identical.
//
// The reference selects and tests over all n points every iteration (main3.cpp:203-214,
// gpu_svm_main3.cu:366-392).  At the end of a solve only ~2 % of the points are support vectors; the
// rest sit at alpha = 0 with f far from the open gap.  LIBSVM's rule (Fan, Chen & Lin 2005, sec. 5)
// drops such a point from selection and from the f update:
//   * a point only in I_high (at a bound) whose f is above b_low cannot be the i_high of any
//     violating pair, and
//   * a point only in I_low whose f is below b_high cannot be its i_low.
// The solve then runs on the active points.  When the active problem meets the stop test, f is
// recomputed for every point from alpha (the warm-start formula, f = -y + K (alpha y) over the
// nonzero alphas), every point is made active again, and the reference's stop test is applied to
// all n points.  If it fails, the solve continues.
//
// Schedule: a shrink pass runs after outer iteration `done` (done = outer iterations completed) when
// done - origin >= start and (done - origin - start) % period == 0.  origin is the start of the solve
// or the last unshrink.  The pass uses the bounds of that outer iteration's working-set build.
#pragma once
#include <cstdint>
#include <cstdlib>

#include "svm355.h"

namespace svm355 {

struct ShrinkCfg {
  bool on = false;
  int32_t start = 0, period = 0;
  double margin = 2.0;  // a point is shrunk only beyond the bounds by margin x the gap
  // a pass after `done` outer iterations (origin: the last unshrink)
  bool pass_after(int64_t done, int64_t origin) const {
    if (!on) return false;
    const int64_t k = done - origin - start;
    return k >= 0 && k % period == 0;
  }
};

// svm_params.shrink: 0 = the default (off), -1 = off, k > 0 = a pass every k outer iterations from the
// k-th.  Off by default: on the synthetic MNIST draws the gap stays wide for most of the solve, few points
// leave the active set before the last few outer iterations, and the unshrink (f recomputed from alpha)
// costs more than the smaller selections save -- 60k 21.2 vs 20.3 ms, 250k 98.3 vs 89.4 ms, 1M 319.8 vs
// 307.2 ms on / off (profiles/shrinking.md).  SVM355_DECOMP_SHRINK (0 off, k > 0 the period),
// SVM355_DECOMP_SHRINK_START and SVM355_DECOMP_SHRINK_MARGIN override it (A/B runs); both sides read the
// same variables.  The margin: LIBSVM's rule (margin 0) drops points as soon as they leave the bounds;
// on the synthetic MNIST draws that shrank points the solve needed again (60k: 12,566 pair updates and 2
// unshrinks against 9,641 unshrunk), margin 2 keeps the pair updates (9,760, 1 unshrink) and still ends
// with ~350 of the 60,000 points active (CPU oracle, scripts/shrink_sim.py).
inline ShrinkCfg shrink_cfg(const svm_params& p) {
  ShrinkCfg c;
  int32_t period = p.shrink > 0 ? p.shrink : -1;
  if (const char* v = std::getenv("SVM355_DECOMP_SHRINK")) period = std::atoi(v) > 0 ? std::atoi(v) : -1;
  c.on = period > 0;
  c.period = c.on ? period : 0;
  c.start = c.period;
  if (const char* v = std::getenv("SVM355_DECOMP_SHRINK_START"))
    if (c.on) c.start = std::atoi(v) > 0 ? std::atoi(v) : 1;
  if (const char* v = std::getenv("SVM355_DECOMP_SHRINK_MARGIN")) c.margin = std::atof(v) > 0.0 ? std::atof(v) : 0.0;
  return c;
}

// The rule, for a point with label y, alpha a, gradient f, against the build's bounds (b_high, b_low).
// The thresholds (hi_cut, lo_cut) = (b_low + margin gap, b_high - margin gap), computed once per pass.
inline void shrink_cuts(double b_high, double b_low, double margin, double* hi_cut, double* lo_cut) {
  const double g = margin * (b_low - b_high);
  *hi_cut = b_low + g;
  *lo_cut = b_high - g;
}
inline bool shrinkable(int32_t y, double a, double f, double C, double eps, double hi_cut, double lo_cut) {
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  const bool up = (y == 1 && a < c_hi) || (y == -1 && a > c_lo);
  const bool dn = (y == 1 && a > c_lo) || (y == -1 && a < c_hi);
  return (up && !dn && f > hi_cut) || (dn && !up && f < lo_cut);
}

// The stop code the build reports when the ACTIVE problem stops while points are shrunk: not a stop
// of the solve (never returned), the host unshrinks and continues.
constexpr int32_t kStopUnshrink = -200;

}  // namespace svm355
