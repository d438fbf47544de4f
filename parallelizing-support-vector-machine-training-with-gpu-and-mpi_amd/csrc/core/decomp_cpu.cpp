// CPU oracle of the working-set decomposition SMO (csrc/hip/decomp.hip), on a precomputed kernel
// matrix.  Given the device's own kernel values it reproduces the device trajectory bit for bit:
// every working set, every moved column and coefficient, alpha and f after every outer iteration
// (tests/test_gpu_decomp_oracle.py).  What has to match, and how:
//   * selection (ws_select_kernel): blocks of `per` points; per block T rounds of an arg-min over
//     I_high and an arg-max over I_low in (value, lowest index) order -- a total order, so the
//     device's thread / wave / workgroup reduction tree gives the lexicographic extreme and so does a
//     plain scan here;
//   * build (ws_build_kernel): b_high / b_low over the candidates, the reference's stop test
//     (main3.cpp:213), the working set = the candidates' ids sorted without duplicates;
//   * inner solve (ws_inner_kernel): i = argmin f over I_high, j second order (Fan, Chen & Lin gain
//     -(f_t - b_high)^2 / (2 - 2 K(i, t)), exact division as on the device) or first order, the
//     reference's clip / eta / update arithmetic (main3.cpp:235-275) with the same operation order
//     (both sides build with -ffp-contract=off), W's own stop max(tau, tau_frac * gap);
//   * f update (igram GEMV epilogue + ws_fsum_count_kernel): per row, per 64-column half, lane l's
//     two terms (columns l and 32 + l) summed from 0, a 32-lane xor butterfly (16, 8, 4, 2, 1), and
//     the halves added in index order before the one add into f.
//   * shrinking (decomp_shrink.h): the same schedule, rule and unshrink (f recomputed from alpha with
//     the warm start's chunked GEMV) -- which points are active is part of the trajectory; which rows the
//     device also keeps updating (its packed list lags the flags) is not, so the trace shows f only
//     for active points (NaN elsewhere).
// The kernel values themselves come from the caller (the device Gram on the exact-integer path).
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <limits>
#include <vector>

#include "../cascade/cascade_capi.h"
#include "decomp_newton.h"
#include "decomp_shrink.h"
#include "internal.h"

using namespace svm355;

namespace {

constexpr int kMaxWS = SVM_DECOMP_MAX_WS;
constexpr int64_t kSelPts = 256 * 16;  // points per selection block below the block cap (ws_select_kernel)
constexpr int kInnerNT = 256;           // the device's inner workgroup (ws_inner_kernel<256, 4>)

struct Shape {
  bool ok = false;
  int q = 0, T = 0;
  int64_t NB = 0, per = 0, L = 0;
};

// decomp_shape (decomp.hip): blocks a multiple of 8 (of 8 * world when world does not divide 8), so
// 1, 2, 4 or 8 ranks own whole blocks of the one-rank partition
Shape shape(int64_t n, int qws, int world) {
  Shape d;
  d.q = std::max(4, std::min(qws, kMaxWS));
  const int64_t nb0 = std::max<int64_t>((n + kSelPts - 1) / kSelPts, std::min<int64_t>(64, (n + 63) / 64));
  const int64_t mult = (8 % world == 0) ? 8 : int64_t(8) * world;
  d.NB = (nb0 + mult - 1) / mult * mult;
  d.NB = std::min<int64_t>(d.NB, int64_t(kMaxWS / 2) / mult * mult);  // past 2,097,152 rows: wider blocks
  d.per = d.NB > 0 ? (n + d.NB - 1) / d.NB : 0;
  d.T = d.NB > 0 ? int(std::max<int64_t>(1, d.q / (2 * d.NB))) : 0;
  d.L = 2 * d.NB * d.T;
  d.ok = n >= 2 && n < int64_t(INT32_MAX) && d.NB >= 1 && d.L <= kMaxWS && world >= 1;
  return d;
}

// One candidate record (ws_select_kernel's CandRec: f and the point id, -1 = none); 16 bytes with no
// padding, so the records cross the transport as plain bytes.
struct Cand {
  double f;
  int64_t id;
};
static_assert(sizeof(Cand) == 16, "candidate records are exchanged as 16-byte records");

// One device GEMV + half-sum pass: f[i] += sum over halves c of half(c, i) (see the header comment).
void gemv_update(const double* K, int64_t ldk, int64_t n, const int32_t* cols, const double* coef, int64_t cnt,
                 double* f, WorkerTeam& team) {
  if (cnt <= 0) return;
  const int64_t halves = (cnt + 63) / 64;
  team.parallel_for(n, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      const double* Ki = K + i * ldk;
      double s = 0.0;
      for (int64_t c = 0; c < halves; ++c) {
        double v[32];
        for (int l = 0; l < 32; ++l) {
          double r = 0.0;
          for (int bj = 0; bj < 2; ++bj) {
            const int64_t j = c * 64 + bj * 32 + l;
            r += j < cnt ? coef[j] * Ki[cols[j]] : 0.0;
          }
          v[l] = r;
        }
        for (int off = 16; off > 0; off >>= 1) {
          double w[32];
          for (int l = 0; l < 32; ++l) w[l] = v[l] + v[l ^ off];
          for (int l = 0; l < 32; ++l) v[l] = w[l];
        }
        s += v[0];
      }
      f[i] += s;
    }
  });
}

// The solve of one rank (t == nullptr: one rank).  Distributed (decomp.hip run_decomp, world > 1):
// this rank owns the blocks [rank NB / world, (rank + 1) NB / world) of the global block partition,
// keeps f for their points only, selects their candidates, and ONE all-gather of the candidate records
// per outer iteration (rank-major) gives every rank the same list; every rank then builds the same
// working set and runs the same inner solve on its alpha replica (K is all n x n on every rank), and
// updates f for its own rows.  The block partition is the one-rank partition for world | 8, so the
// trajectory is the one-rank trajectory bit for bit.  Returns SVM_OK or an error code (set_error);
// transport failures throw (TransportError / CascadeAborted).
int decomp_solve(const double* K, int64_t ldk, const int32_t* y, int64_t n, double* alpha, int32_t warm,
                 const svm_params& p, int32_t qws, double tau_frac, int32_t inner_wss, svm_result* res,
                 int64_t* stats, svm_decomp_trace* tr, Transport* t) {
  const int world = t ? t->world() : 1, rank = t ? t->rank() : 0;
  if (!K || !y || !alpha || n < 2 || ldk < n) {
    set_error("svm_decomp_train_gram: bad arguments");
    return SVM_ERR_ARG;
  }
  if (!(tau_frac >= 0.0 && tau_frac < 0.5)) {
    set_error("svm_decomp_train_gram: tau_frac must be in [0, 0.5)");
    return SVM_ERR_ARG;
  }
  if (tr && world != 1) {
    set_error("svm_decomp_train_gram: a trace needs one rank");
    return SVM_ERR_ARG;
  }
  const Shape sh = shape(n, qws > 0 ? qws : kMaxWS, world);
  if (!sh.ok) {
    set_error("svm_decomp_train_gram: n = %lld is outside the solver's shapes", (long long)n);
    return SVM_ERR_ARG;
  }
  const int64_t NBr = sh.NB / world, bb0 = rank * NBr;
  const int64_t lo = std::min<int64_t>(n, bb0 * sh.per), hi = std::min<int64_t>(n, (bb0 + NBr) * sh.per);
  const int64_t nloc = hi - lo, Lr = 2 * NBr * sh.T, LhR = NBr * sh.T;
  // fault injection (tests): rank SVM355_DECOMP_FAIL_RANK fails at the start of outer iteration
  // SVM355_DECOMP_FAIL_OUTER (default 0); its peers must leave their all-gather with an error
  int fail_outer = -1;
  if (const char* fr = getenv("SVM355_DECOMP_FAIL_RANK"); fr && world > 1 && atoi(fr) == rank) {
    const char* fo = getenv("SVM355_DECOMP_FAIL_OUTER");
    fail_outer = fo ? std::max(0, atoi(fo)) : 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  WorkerTeam team(std::max<int32_t>(1, std::min<int32_t>(resolve_threads(p.n_threads), int32_t(n / 256) + 1)));
  const double C = p.C, eps = p.eps, tau = p.tau, c_hi = C - eps, c_lo = 0.0 + eps;
  const double inf = std::numeric_limits<double>::infinity();
  auto in_high = [&](int32_t yi, double a) { return (yi == 1 && a < c_hi) || (yi == -1 && a > c_lo); };
  auto in_low = [&](int32_t yi, double a) { return (yi == 1 && a > c_lo) || (yi == -1 && a < c_hi); };

  // ---- start: cold (alpha = 0, f = -y: ws_init_kernel) or warm (f = -y + K (alpha y) over the
  // nonzero alphas, ascending, in chunks of kMaxWS columns: decomp.hip's warm start); f of this
  // rank's rows [lo, hi) only
  std::vector<double> f(static_cast<size_t>(std::max<int64_t>(nloc, 1)));
  int64_t warm_cols = 0;
  // f = -y + K (alpha y) over the nonzero alphas (ascending ids, chunks of kMaxWS columns): the warm
  // start, and the recomputation when the solve unshrinks
  auto f_from_alpha = [&]() -> int64_t {
    for (int64_t i = lo; i < hi; ++i) f[size_t(i - lo)] = -static_cast<double>(y[i]);
    std::vector<int32_t> nzc;
    std::vector<double> nzv;
    for (int64_t j = 0; j < n; ++j)
      if (alpha[j] != 0.0) {
        nzc.push_back(int32_t(j));
        nzv.push_back(alpha[j] * double(y[j]));
      }
    for (size_t c0 = 0; c0 < nzc.size(); c0 += kMaxWS)
      gemv_update(K + lo * ldk, ldk, nloc, nzc.data() + c0, nzv.data() + c0,
                  int64_t(std::min<size_t>(kMaxWS, nzc.size() - c0)), f.data(), team);
    return int64_t(nzc.size());
  };
  if (!warm) {
    for (int64_t i = lo; i < hi; ++i) f[size_t(i - lo)] = -static_cast<double>(y[i]);
    for (int64_t i = 0; i < n; ++i) alpha[i] = 0.0;
  } else {
    warm_cols = f_from_alpha();
  }
  // shrinking: shr[i - lo] = 1 while row i is out of the active set
  const ShrinkCfg shc = shrink_cfg(p);
  std::vector<uint8_t> shr(size_t(std::max<int64_t>(nloc, 1)), 0);
  bool shrunk = false;  // a shrink pass has run since the start / the last unshrink
  int64_t origin = 0, unshrinks = 0, passes = 0, min_active = nloc, n_active = nloc;

  int64_t outer = 0, inner_total = 0, changed_total = 0, last_inner_it = 0, newton_steps = 0;
  int64_t chain_it = 0;  // inner-solve loop iterations (each one or more pair updates)
  int last_m = 0;
  NewtonCfg nwc = newton_cfg(p);
  nwc.on = nwc.on && inner_wss == 3;  // the device polishes in its default inner solve (second order + second pair)
  int32_t last_reason = SVM_STOP_CONVERGED, stop = SVM_STOP_RUNNING;
  double bh = inf, bl = -inf;
  std::vector<Cand> cown(size_t(std::max<int64_t>(Lr, 1))), call(size_t(sh.L));
  std::vector<int32_t> W;
  std::vector<double> a, a0, ft, kh, kl;
  std::vector<int32_t> yw, cols;
  std::vector<double> coef;
  if (tr) tr->count = 0;
  for (;;) {
    if (outer == fail_outer) {
      set_error("decomposition SMO: injected failure of rank %d at outer iteration %lld", rank, (long long)outer);
      return SVM_ERR_INTERNAL;
    }
    // ---- selection over this rank's blocks: per block, T picks per side in (value, lowest index) order
    team.parallel_for(NBr, [&](int64_t blo, int64_t bhi) {
      std::vector<char> th, tl;
      for (int64_t bl_ = blo; bl_ < bhi; ++bl_) {
        const int64_t b = bb0 + bl_;
        const int64_t b0 = std::min<int64_t>(n, b * sh.per), b1 = std::min<int64_t>(n, b0 + sh.per);
        const int64_t cnt = std::max<int64_t>(0, b1 - b0);
        th.assign(size_t(cnt), 0);
        tl.assign(size_t(cnt), 0);
        for (int k = 0; k < sh.T; ++k) {
          double mv = inf, xv = -inf;
          int64_t mi = -1, xi = -1;
          for (int64_t i = b0; i < b1; ++i) {
            if (shr[size_t(i - lo)]) continue;
            const double ai = alpha[i], fi = f[size_t(i - lo)];
            if (!th[size_t(i - b0)] && in_high(y[i], ai) && fi < mv) {
              mv = fi;
              mi = i;
            }
            if (!tl[size_t(i - b0)] && in_low(y[i], ai) && fi > xv) {
              xv = fi;
              xi = i;
            }
          }
          cown[size_t(bl_ * sh.T + k)] = mi >= 0 ? Cand{mv, mi} : Cand{0.0, -1};
          cown[size_t(LhR + bl_ * sh.T + k)] = xi >= 0 ? Cand{xv, xi} : Cand{0.0, -1};
          if (mi >= 0) th[size_t(mi - b0)] = 1;
          if (xi >= 0) tl[size_t(xi - b0)] = 1;
        }
      }
    });
    // ---- the candidate exchange: rank-major [rank r: I_high picks of its blocks, then I_low picks]
    if (world > 1)
      t->allgather(cown.data(), Lr * int64_t(sizeof(Cand)), call.data());
    else
      std::copy(cown.begin(), cown.begin() + sh.L, call.begin());
    // ---- build: bounds, stop test, the sorted de-duplicated working set
    bh = inf;
    bl = -inf;
    std::vector<std::pair<int64_t, double>> ids;
    ids.reserve(call.size());
    for (int64_t u = 0; u < sh.L; ++u) {
      const Cand& c = call[size_t(u)];
      if (c.id < 0) continue;
      if (u % Lr < LhR)
        bh = std::fmin(bh, c.f);
      else
        bl = std::fmax(bl, c.f);
      ids.emplace_back(c.id, c.f);
    }
    std::sort(ids.begin(), ids.end(), [](const auto& u, const auto& v) { return u.first < v.first; });
    W.clear();
    std::vector<double> Wf;
    for (size_t q = 0; q < ids.size(); ++q)
      if (q == 0 || ids[q].first != ids[q - 1].first) {
        W.push_back(int32_t(ids[q].first));
        Wf.push_back(ids[q].second);
      }
    const int m = int(W.size());
    if (outer > 0 && last_inner_it == 0)
      stop = last_reason == SVM_STOP_CONVERGED ? SVM_STOP_NO_CANDIDATE : last_reason;
    else if (!(bh < inf) || !(bl > -inf))
      stop = SVM_STOP_NO_CANDIDATE;
    else if (bl <= bh + 2.0 * tau)
      stop = SVM_STOP_CONVERGED;
    else if (inner_total + 1 > p.max_iter)
      stop = SVM_STOP_MAX_ITER;
    else if (m < 2 || m > kMaxWS) {
      set_error("svm_decomp_train_gram: working set outside [2, %d]", kMaxWS);
      return SVM_ERR_INTERNAL;
    }
    if (stop != SVM_STOP_RUNNING && stop != SVM_STOP_MAX_ITER && shrunk) {
      // the ACTIVE problem stopped: every point active again, f recomputed from alpha, and the stop
      // test again on all n points (the next selection)
      stop = SVM_STOP_RUNNING;
      f_from_alpha();
      std::fill(shr.begin(), shr.end(), uint8_t(0));
      n_active = nloc;
      shrunk = false;
      origin = outer;
      last_inner_it = -1;  // the no-progress test looks at the next working set, not the last one
      last_m = 0;          // and the Newton polish waits for a long inner solve on the full problem
      ++unshrinks;
      continue;
    }
    if (stop != SVM_STOP_RUNNING) break;
    const double tau_in = std::fmax(tau, tau_frac * (bl - bh));
    const int64_t max_inner = std::min<int64_t>(int64_t(20) * m, p.max_iter - inner_total);

    // ---- inner solve on W (positions 0..m-1 = ascending ids)
    a.assign(size_t(m), 0.0);
    yw.assign(size_t(m), 0);
    ft.assign(Wf.begin(), Wf.end());
    for (int k = 0; k < m; ++k) {
      a[size_t(k)] = alpha[W[size_t(k)]];
      yw[size_t(k)] = y[W[size_t(k)]];
    }
    a0 = a;
    kh.assign(size_t(m), 0.0);
    kl.assign(size_t(m), 0.0);
    int64_t it = 0;
    int32_t reason = SVM_STOP_CONVERGED;
    // the Newton polish of W's free variables (decomp_newton.h): `since` counts chain iterations with no
    // bound-status change, and starts at `every` after a long inner solve
    int32_t since = newton_since0(nwc, last_inner_it, last_m), ntrig = 0;
    for (;;) {
      double hv = inf, lv = -inf;
      int ih = -1, il = -1;
      for (int k = 0; k < m; ++k) {
        if (in_high(yw[size_t(k)], a[size_t(k)]) && ft[size_t(k)] < hv) {
          hv = ft[size_t(k)];
          ih = k;
        }
        if (in_low(yw[size_t(k)], a[size_t(k)]) && ft[size_t(k)] > lv) {
          lv = ft[size_t(k)];
          il = k;
        }
      }
      if (ih < 0 || il < 0) {
        reason = SVM_STOP_NO_CANDIDATE;
        break;
      }
      if (lv <= hv + 2.0 * tau_in) break;
      if (it >= max_inner) {
        reason = SVM_STOP_MAX_ITER;
        break;
      }
      if (nwc.on && since >= nwc.every && ntrig < nwc.per_solve) {
        ++ntrig;
        since = 0;
        int code = 0, steps = 0;
        while (steps < nwc.repeat &&
               (code = newton_step_ref(m, a.data(), ft.data(), yw.data(),
                                       [&](int q, int k) { return K[int64_t(W[size_t(q)]) * ldk + W[size_t(k)]]; },
                                       C, eps, nwc.max_free)) != 0) {
          ++steps;
          if (code == 1) break;
        }
        if (steps > 0) {
          it += steps;  // a step counts as an iteration of the inner solve
          newton_steps += steps;
          continue;  // select again
        }
      }
      // inner_wss 3: the second pair from the same selection (ws_inner_kernel DP): i2 = the best I_high
      // point outside i_high's wave of the 256-thread inner workgroup (position k lies in wave
      // (k mod 512) / 128), j2 = the first-order j.  inner_wss 4 (ws_inner_kernel J2S): j2 by the
      // second-order gain of row i2 over I_low points above f(i2), from the same snapshot
      int i2 = -1;
      int j2 = il;
      if (inner_wss >= 3) {
        const int wih = (ih % (2 * kInnerNT)) / 128;
        double v2 = inf;
        for (int k = 0; k < m; ++k)
          if ((k % (2 * kInnerNT)) / 128 != wih && in_high(yw[size_t(k)], a[size_t(k)]) && ft[size_t(k)] < v2) {
            v2 = ft[size_t(k)];
            i2 = k;
          }
      }
      if (inner_wss == 4) {
        j2 = -1;
        if (i2 >= 0) {
          const double* K2 = K + int64_t(W[size_t(i2)]) * ldk;
          const double h2 = ft[size_t(i2)];
          double gv2 = inf;
          for (int k = 0; k < m; ++k) {
            if (!in_low(yw[size_t(k)], a[size_t(k)]) || !(ft[size_t(k)] > h2)) continue;
            const double bb = ft[size_t(k)] - h2;
            double at = 2.0 - 2.0 * K2[W[size_t(k)]];
            at = at <= 0.0 ? eps : at;
            const double gain = -(bb * bb) / at;
            if (gain < gv2) {
              gv2 = gain;
              j2 = k;
            }
          }
        }
      }
      const double* Ki = K + int64_t(W[size_t(ih)]) * ldk;
      for (int k = 0; k < m; ++k) kh[size_t(k)] = Ki[W[size_t(k)]];
      double bl_upd = lv;
      if (inner_wss != 1) {
        double gv = inf;
        int gj = -1;
        for (int k = 0; k < m; ++k) {
          if (!in_low(yw[size_t(k)], a[size_t(k)]) || !(ft[size_t(k)] > hv)) continue;
          const double bb = ft[size_t(k)] - hv;
          double at = 2.0 - 2.0 * kh[size_t(k)];
          at = at <= 0.0 ? eps : at;
          const double gain = -(bb * bb) / at;
          if (gain < gv) {
            gv = gain;
            gj = k;
          }
        }
        if (gj < 0) {
          reason = SVM_STOP_NO_CANDIDATE;
          break;
        }
        il = gj;
        bl_upd = ft[size_t(il)];
      }
      const double K12 = kh[size_t(il)];
      const double* Kj = K + int64_t(W[size_t(il)]) * ldk;
      for (int k = 0; k < m; ++k) kl[size_t(k)] = Kj[W[size_t(k)]];
      const double ah = a[size_t(ih)], al = a[size_t(il)];
      const int32_t yh = yw[size_t(ih)], yl = yw[size_t(il)];
      const int s = yh * yl;
      const double eta = 1.0 + 1.0 - 2.0 * K12;
      double U, V;
      if (s == -1) {
        U = std::fmax(0.0, al - ah);
        V = std::fmin(C, C + al - ah);
      } else {
        U = std::fmax(0.0, al + ah - C);
        V = std::fmin(C, al + ah);
      }
      if (!(U <= V + 1e-12)) {
        reason = SVM_STOP_INFEASIBLE;
        break;
      }
      if (eta <= eps) {
        reason = SVM_STOP_NONPOS_ETA;
        break;
      }
      double al_new = al + double(yl) * (hv - bl_upd) / eta;
      if (al_new > V) al_new = V;
      if (al_new < U) al_new = U;
      const double ah_new = ah + double(s) * (al - al_new);
      const double ch = (ah_new - ah) * double(yh);
      const double cl = (al_new - al) * double(yl);
      for (int k = 0; k < m; ++k) ft[size_t(k)] += ch * kh[size_t(k)] + cl * kl[size_t(k)];
      bool moved_status = bound_status(ah_new, C, eps) != bound_status(ah, C, eps) ||
                          bound_status(al_new, C, eps) != bound_status(al, C, eps);
      a[size_t(ih)] = ah_new;
      a[size_t(il)] = al_new;
      ++it;
      if (i2 >= 0 && j2 >= 0 && j2 != ih && i2 != j2 && il != j2 && il != i2 && it < max_inner) {
        const double fi2 = ft[size_t(i2)], fj2 = ft[size_t(j2)];  // after the first update
        const double a2h = a[size_t(i2)], a2l = a[size_t(j2)];
        const int32_t yh2 = yw[size_t(i2)], yl2 = yw[size_t(j2)];
        const int s2 = yh2 * yl2;
        const double eta2 = 1.0 + 1.0 - 2.0 * K[int64_t(W[size_t(i2)]) * ldk + W[size_t(j2)]];
        double U2, V2;
        if (s2 == -1) {
          U2 = std::fmax(0.0, a2l - a2h);
          V2 = std::fmin(C, C + a2l - a2h);
        } else {
          U2 = std::fmax(0.0, a2l + a2h - C);
          V2 = std::fmin(C, a2l + a2h);
        }
        if (fj2 > fi2 + 2.0 * tau_in && U2 <= V2 + 1e-12 && !(eta2 <= eps)) {
          double al2 = a2l + double(yl2) * (fi2 - fj2) / eta2;
          if (al2 > V2) al2 = V2;
          if (al2 < U2) al2 = U2;
          const double ah2 = a2h + double(s2) * (a2l - al2);
          const double ch2 = (ah2 - a2h) * double(yh2);
          const double cl2 = (al2 - a2l) * double(yl2);
          const double* Ki2 = K + int64_t(W[size_t(i2)]) * ldk;
          const double* Kj2 = K + int64_t(W[size_t(j2)]) * ldk;
          for (int k = 0; k < m; ++k) ft[size_t(k)] += ch2 * Ki2[W[size_t(k)]] + cl2 * Kj2[W[size_t(k)]];
          moved_status = moved_status || bound_status(ah2, C, eps) != bound_status(a2h, C, eps) ||
                         bound_status(al2, C, eps) != bound_status(a2l, C, eps);
          a[size_t(i2)] = ah2;
          a[size_t(j2)] = al2;
          ++it;
        }
      }
      ++chain_it;
      since = moved_status ? 0 : since + 1;
    }
    // ---- moved columns (ascending position = ascending id), alpha written back
    cols.clear();
    coef.clear();
    for (int k = 0; k < m; ++k)
      if (a[size_t(k)] != a0[size_t(k)]) {
        alpha[W[size_t(k)]] = a[size_t(k)];
        cols.push_back(W[size_t(k)]);
        coef.push_back((a[size_t(k)] - a0[size_t(k)]) * (yw[size_t(k)] == 1 ? 1.0 : -1.0));
      }
    ++outer;
    inner_total += it;
    changed_total += int64_t(cols.size());
    last_inner_it = it;
    last_m = m;
    last_reason = reason;
    gemv_update(K + lo * ldk, ldk, nloc, cols.data(), coef.data(), int64_t(cols.size()), f.data(), team);
    if (shc.pass_after(outer, origin)) {  // shrink pass with this outer iteration's bounds
      int64_t drop = 0;
      double hc, lc;
      shrink_cuts(bh, bl, shc.margin, &hc, &lc);
      for (int64_t i = lo; i < hi; ++i)
        if (!shr[size_t(i - lo)] && shrinkable(y[i], alpha[i], f[size_t(i - lo)], C, eps, hc, lc)) {
          shr[size_t(i - lo)] = 1;
          ++drop;
        }
      n_active -= drop;
      min_active = std::min(min_active, n_active);
      shrunk = true;
      ++passes;
      if (getenv("SVM355_DECOMP_SHRINK_LOG"))
        fprintf(stderr, "decomp oracle: rank %d outer %lld shrink pass: %lld active of %lld\n", rank,
                (long long)outer, (long long)n_active, (long long)nloc);
    }
    if (tr && tr->count < tr->cap) {
      const int64_t o = tr->count++;
      if (tr->m) tr->m[o] = m;
      if (tr->W)
        for (int k = 0; k < kMaxWS; ++k) tr->W[o * kMaxWS + k] = k < m ? W[size_t(k)] : -1;
      if (tr->moved) tr->moved[o] = int32_t(cols.size());
      for (int k = 0; k < kMaxWS; ++k) {
        const bool v = k < int(cols.size());
        if (tr->cols) tr->cols[o * kMaxWS + k] = v ? cols[size_t(k)] : -1;
        if (tr->coef) tr->coef[o * kMaxWS + k] = v ? coef[size_t(k)] : 0.0;
      }
      if (tr->inner) tr->inner[o] = it;
      if (tr->bounds) {
        tr->bounds[2 * o] = bh;
        tr->bounds[2 * o + 1] = bl;
      }
      if (tr->n == n && tr->alpha) std::copy(alpha, alpha + n, tr->alpha + o * n);
      if (tr->n == n && tr->f)
        for (int64_t i = 0; i < n; ++i)
          tr->f[o * n + i] = shr[size_t(i)] ? std::numeric_limits<double>::quiet_NaN() : f[size_t(i)];
    }
  }
  if (stats) {
    stats[0] = outer;
    stats[1] = inner_total;
    stats[2] = sh.L;
    stats[3] = int64_t(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    stats[4] = changed_total;
    stats[5] = 0;
    stats[6] = 0;
    stats[7] = warm_cols;
    stats[8] = unshrinks;
    stats[9] = passes;
    stats[10] = min_active;
    stats[11] = 0;
    stats[12] = newton_steps;
    stats[13] = chain_it;
  }
  if (res) {
    res->iterations = inner_total + 1;
    res->b_high = bh;
    res->b_low = bl;
    res->b = (bh + bl) / 2;
    res->stop_reason = stop;
    res->reserved = 0;
    res->n_sv = svm_sv_indices(alpha, n, p.sv_tol, nullptr);
    res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return SVM_OK;
}

svm_params params_or_default(const svm_params* pp) {
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  return p;
}

}  // namespace

extern "C" SVM_API int svm_decomp_train_gram(const double* K, int64_t ldk, const int32_t* y, int64_t n,
                                             double* alpha, int32_t warm, const svm_params* pp, int32_t qws,
                                             double tau_frac, int32_t inner_wss, svm_result* res, int64_t* stats,
                                             svm_decomp_trace* tr) {
  return decomp_solve(K, ldk, y, n, alpha, warm, params_or_default(pp), qws, tau_frac, inner_wss, res, stats, tr,
                      nullptr);
}

// This process's rank of the distributed form over caller-supplied host collectives (a gloo group
// under torchrun: the CPU twin of the per-process device rank, svmd_cascade_rank_decomp).
extern "C" SVM_API int svm_decomp_rank_train_gram(const svm_host_comm* comm, const double* K, int64_t ldk,
                                                  const int32_t* y, int64_t n, double* alpha, int32_t warm,
                                                  const svm_params* pp, int32_t qws, double tau_frac,
                                                  int32_t inner_wss, svm_result* res, int64_t* stats) {
  if (!host_comm_valid(comm)) {
    set_error("svm_decomp_rank_train_gram: bad communicator");
    return SVM_ERR_ARG;
  }
  try {
    auto t = make_hostcomm_transport(*comm, nullptr);
    return decomp_solve(K, ldk, y, n, alpha, warm, params_or_default(pp), qws, tau_frac, inner_wss, res, stats,
                        nullptr, comm->world > 1 ? t.get() : nullptr);
  } catch (const std::exception& e) {
    set_error("decomposition SMO: %s", e.what());
    return SVM_ERR_INTERNAL;
  }
}

// world thread-ranks of this process over a strict loopback group (the thread-rank twin; the ranks'
// alpha replicas must come out identical).  alpha / res / stats: rank 0's.
extern "C" SVM_API int svm_decomp_group_train_gram(int32_t world, const double* K, int64_t ldk, const int32_t* y,
                                                   int64_t n, double* alpha, int32_t warm, const svm_params* pp,
                                                   int32_t qws, double tau_frac, int32_t inner_wss, svm_result* res,
                                                   int64_t* stats, double comm_timeout_s) {
  if (world < 1 || !K || !y || !alpha || n < 2) {
    set_error("svm_decomp_group_train_gram: bad arguments");
    return SVM_ERR_ARG;
  }
  const svm_params p = params_or_default(pp);
  auto token = std::make_shared<AbortToken>();
  auto lg = std::make_shared<LoopbackGroup>(world, WaitPolicy{token, comm_timeout_s > 0 ? comm_timeout_s : 600.0});
  auto be = make_cpu_backend();
  std::vector<std::unique_ptr<LoopbackTransport>> tr;
  for (int r = 0; r < world; ++r) tr.push_back(std::make_unique<LoopbackTransport>(lg, r, be.get()));
  std::vector<std::vector<double>> replicas{size_t(world)};
  for (int r = 1; r < world; ++r) replicas[size_t(r)].assign(alpha, alpha + n);  // warm starts: the same start
  try {
    run_rank_threads(
        world, token,
        [&](int r) {
          double* a = r == 0 ? alpha : replicas[size_t(r)].data();
          const int rc = decomp_solve(K, ldk, y, n, a, warm, p, qws, tau_frac, inner_wss, r == 0 ? res : nullptr,
                                      r == 0 ? stats : nullptr, nullptr, world > 1 ? tr[size_t(r)].get() : nullptr);
          if (rc != SVM_OK) throw CascadeError(svm_last_error());
        },
        [&](int) {});
  } catch (const std::exception& e) {
    set_error("decomposition SMO: %s", e.what());
    return SVM_ERR_INTERNAL;
  }
  for (int r = 1; r < world; ++r)
    if (!std::equal(alpha, alpha + n, replicas[size_t(r)].begin())) {
      set_error("decomposition SMO: rank %d's alpha replica differs from rank 0's", r);
      return SVM_ERR_INTERNAL;
    }
  return SVM_OK;
}

// One Newton polish step on a working set of m points (tests): Kw (m x m, row stride ldk), labels,
// alpha and f by position (updated in place); *code = 0 (no step), 1 (full), 2 (cut at a bound).
extern "C" SVM_API int svm_decomp_newton_step(const double* Kw, int64_t ldk, const int32_t* y, int32_t m, double* a,
                                              double* f, double C, double eps, int32_t max_free, int32_t* code) {
  if (!Kw || !y || !a || !f || !code || m < 1 || ldk < m) {
    set_error("svm_decomp_newton_step: bad arguments");
    return SVM_ERR_ARG;
  }
  *code = newton_step_ref(m, a, f, y, [&](int q, int k) { return Kw[int64_t(q) * ldk + k]; }, C, eps, max_free);
  return SVM_OK;
}

// The device f-update GEMV's arithmetic alone (tests): f[i] += sum_k coef[k] K(i, cols[k]), k < cnt,
// for the n rows of K (row stride ldk), in the device's summation order (gemv_update).
extern "C" SVM_API int svm_decomp_gemv_ref(const double* K, int64_t ldk, int64_t n, const int32_t* cols,
                                           const double* coef, int64_t cnt, double* f) {
  if (!K || n < 0 || cnt < 0 || (cnt > 0 && (!cols || !coef)) || !f) {
    set_error("svm_decomp_gemv_ref: bad arguments");
    return SVM_ERR_ARG;
  }
  WorkerTeam team(std::max<int32_t>(1, std::min<int32_t>(resolve_threads(0), int32_t(n / 256) + 1)));
  gemv_update(K, ldk, n, cols, coef, cnt, f, team);
  return SVM_OK;
}
