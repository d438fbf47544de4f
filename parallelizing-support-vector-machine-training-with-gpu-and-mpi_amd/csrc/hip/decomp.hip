// Working-set decomposition SMO (opt-in, SVC(solver="decomp")): the reference's first-order SMO
// semantics per pair, but on a WORKING SET of up to q points at a time -- the SMO-type decomposition
// of LIBSVM / ThunderSVM re-designed for MI355X.
//
// The reference (main3.cpp:162-294, gpu_svm_main3.cu:318-483) updates ONE pair per iteration over
// all n points, so a GPU iteration is bound by a grid-wide exchange (~3.4 us at 60k even
// persistent).  Here one outer iteration is:
//   1. ws_select_kernel   per block of the points, its T most violating of I_high (smallest f) and
//                         of I_low (largest f), lowest index on ties -- the union always holds the
//                         globally maximal violating pair, so every outer iteration makes progress;
//   2. ws_build_kernel    one workgroup: the stop test on the global extremes (b_low <= b_high + 2 tau,
//                         main3.cpp:213), then the sorted, de-duplicated working set W (m <= q);
//   3. K(W, W)            the working set's rows gathered, its m x m Gram on the exact-integer path
//                         (the same kernel values as the full Gram, igram.hip);
//   4. ws_inner_kernel    ONE workgroup runs first-order SMO on W with the reference's update
//                         arithmetic (clip bounds, eta, stop reasons) -- an iteration is a workgroup
//                         reduction and two L2-resident row reads, no grid exchange -- until W's own
//                         gap is below max(tau, gap / 10);
//   5. f update           f += K(:, W) (delta alpha * y): the exact-integer kernel values of all n
//                         rows against W computed on int8 MFMA and reduced in the epilogue
//                         (igram_tri_kernel GEMV mode), never stored -- no n x n Gram at all.
// The stop test is the reference's, on all n points, so the model meets the same optimality bound
// (tests: the same support-vector set as the pairwise solve, b within the stop tolerance); the
// sequence of pair updates differs, so iteration counts and b differ in the last digits.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "decomp.h"
#include "decomp_newton.h"
#include "decomp_shrink.h"
#include "persist.h"
#include "svm355_device.h"
#include "trace.h"

namespace svm355 {
namespace {

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

struct DecompHost {  // pinned: the PROF build's phase totals (the loop state is DecompCtl, on the device)
  int64_t prof[12];  // clock64 ticks per phase summed over iterations; [6] kernel clock64, [7] wall ticks;
                     // [8..11] the second-order j phase split (row i, gains + wave reduction, publish +
                     // barrier, fold)
};

// The outer loop's state on the device: the kernels of an outer iteration read and advance it, so the
// host enqueues several outer iterations between synchronisations (a stopped solve turns the rest of
// the batch into no-op launches).  stop = SVM_STOP_RUNNING (0) while running; kStopInternal: the working
// set came out outside [2, kMaxWS] (a bug).
struct DecompCtl {
  int32_t stop, m;
  double b_high, b_low;      // of the last working-set build
  double tau_in;             // the next inner solve's stop tolerance
  int64_t max_inner;         // and its iteration cap
  int64_t outer, inner_total, changed_total, last_inner_it;
  int32_t last_inner_reason;
  int32_t shrunk;            // a shrink pass has run since the start or the last unshrink
  int64_t n_active;          // this GPU's points not shrunk
  int64_t passes;            // shrink passes run
  int32_t last_m, pad2;      // the last inner solve's working-set size (the Newton polish's arming)
  int64_t newton_steps;      // Newton polish steps applied (decomp_newton.h)
};

// The Newton polish's knobs on the device (NewtonCfg).
struct NwDev {
  int32_t on, every, per_solve, repeat, max_free, pad;
  double frac;
};
constexpr int32_t kStopInternal = -100;

// The control block's host copy, written by the kernel that last changes it in an outer iteration (the
// inner solve, or the build when it stops the solve) with plain vector stores into pinned host memory:
// visible to the host once the batch's event has completed, with no copy in the stream.
__device__ __forceinline__ void publish_ctl(const DecompCtl& c, DecompCtl* __restrict__ pub) {
  if (pub) *pub = c;
}

constexpr int kSelNT = 256, kSelE = 16;  // per-block selection: up to 4096 points per block
constexpr int kMaxWS = 1024;             // working-set capacity (one 1024-thread inner workgroup)

// A working-set candidate: global point id (-1 = none) and its f.  Candidates carry f because in the
// distributed solve a GPU holds f only for its own points (every GPU holds alpha and y for all).
struct CandRec {
  double f;
  int32_t id, pad;
};

// Per block b of `per` points of this GPU's slice (local rows [b per, (b + 1) per), global ids lo +
// local): the T most violating points of I_high (smallest f) and of I_low (largest f) in wave_arg's
// order (value, then lowest index): every wave's own T best by T wave arg-reductions (the winner
// masked out by its owner after each), then a 4-way merge of the sorted wave lists.  f is the slice's
// (local index); alpha and y are global.
// Shrinking (decomp_shrink.h): shr[i] = 1 excludes local row i; with a packed list (act: the rows in
// the active order, boff: selection block b's rows are act[boff[b] .. boff[b + 1])) the block walks its
// packed rows instead of [b per, (b + 1) per) -- the same points in the same ascending order, so the picks
// are those of the masked full block.
__global__ __launch_bounds__(kSelNT) void ws_select_kernel(const double* __restrict__ f,
                                                           const double* __restrict__ alpha,
                                                           const int32_t* __restrict__ y, int64_t lo, int64_t nloc,
                                                           int64_t per, int T, double C, double eps,
                                                           CandRec* __restrict__ cand_h, CandRec* __restrict__ cand_l,
                                                           const DecompCtl* __restrict__ ctl,
                                                           const int32_t* __restrict__ act,
                                                           const int32_t* __restrict__ boff,
                                                           const uint8_t* __restrict__ shr) {
  if (ctl->stop != SVM_STOP_RUNNING) return;
  constexpr int NW = kSelNT / 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t b0 = act ? int64_t(boff[blockIdx.x]) : int64_t(blockIdx.x) * per;
  const int64_t b1 = act ? int64_t(boff[blockIdx.x + 1]) : std::min<int64_t>(nloc, b0 + per);
  const double c_hi = C - eps, c_lo = 0.0 + eps, inf = __builtin_inf();
  double fh[kSelE], fl[kSelE];
  uint32_t gi[kSelE];  // global ids, ascending in e
#pragma unroll
  for (int e = 0; e < kSelE; ++e) {
    const int64_t k = b0 + t + int64_t(kSelNT) * e;
    fh[e] = inf;
    fl[e] = -inf;
    const int64_t i = k < b1 ? (act ? int64_t(act[k]) : k) : k;
    gi[e] = uint32_t(lo + i);
    if (k < b1 && !(shr && shr[i])) {
      const double a = alpha[lo + i], fi = f[i];
      const int32_t yi = y[lo + i];
      if ((yi == 1 && a < c_hi) || (yi == -1 && a > c_lo)) fh[e] = fi;
      if ((yi == 1 && a > c_lo) || (yi == -1 && a < c_hi)) fl[e] = fi;
    }
  }
  // Every wave takes its own T best of each side with wave reductions only (no barrier per pick), then
  // the block's T best are the first T of the merge of the four sorted wave lists: the same picks in
  // the same order as T rounds of a block arg-reduction (the keys (value, index) are distinct).
  constexpr int kTMax = 64;  // T <= q / (2 * 8 blocks)
  __shared__ double lv[2][NW][kTMax];
  __shared__ uint32_t li[2][NW][kTMax];
  for (int k = 0; k < T; ++k) {
    VI mn{inf, kSentinel}, mx{-inf, kSentinel};
#pragma unroll
    for (int e = 0; e < kSelE; ++e) {  // ascending index within a thread: strict compares keep the lowest
      const uint32_t i = gi[e];
      const bool ch = fh[e] < mn.v, cl = fl[e] > mx.v;
      mn = ch ? VI{fh[e], i} : mn;
      mx = cl ? VI{fl[e], i} : mx;
    }
    VIL a, b;
    wave_arg_pair(mn, mx, a, b);
    if (lane == 0) {
      lv[0][w][k] = a.v;
      li[0][w][k] = a.i;
      lv[1][w][k] = b.v;
      li[1][w][k] = b.i;
    }
#pragma unroll
    for (int e = 0; e < kSelE; ++e) {
      if (gi[e] == a.i) fh[e] = inf;
      if (gi[e] == b.i) fl[e] = -inf;
    }
  }
  __syncthreads();
  if (t == 0 || t == 64) {  // wave 0 merges I_high, wave 1 I_low
    const int sd = t == 0 ? 0 : 1;
    int ptr[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) ptr[q] = 0;
    CandRec* out = (sd == 0 ? cand_h : cand_l) + int64_t(blockIdx.x) * T;
    for (int k = 0; k < T; ++k) {
      int bq = 0;
      VI best{lv[sd][0][ptr[0]], li[sd][0][ptr[0]]};
#pragma unroll
      for (int q = 1; q < NW; ++q) {
        const VI c{lv[sd][q][ptr[q]], li[sd][q][ptr[q]]};
        const bool take = sd == 0 ? beats<true>(c, best) : beats<false>(c, best);
        if (take) {
          best = c;
          bq = q;
        }
      }
      ++ptr[bq];  // a wave's list holds T entries: no list runs out before T picks
      const bool ok = best.i != kSentinel && (sd == 0 ? best.v < inf : best.v > -inf);
      out[k] = CandRec{ok ? best.v : 0.0, ok ? int32_t(best.i) : -1, 0};
    }
  }
}

// ws_select_kernel's picks for blocks of any size, streamed from memory: past 2,097,152 rows the block
// count is capped at kMaxWS / 2 (the candidates must fit one working set, so T = 1) and a block holds
// more than the kSelNT x kSelE points the register-resident kernel takes (SVM355_DECOMP_WIDE_SELECT=1
// runs it at any n, for the equivalence tests).  Round k takes, per side, the best point strictly after
// round k - 1's block pick in (value, lowest index) order: the keys are distinct, so that is the next
// entry of the sorted list the T arg-reductions of ws_select_kernel (and the CPU oracle) produce.  One
// pass over the block per round; every thread merges the four wave winners itself.
__global__ __launch_bounds__(kSelNT) void ws_select_wide_kernel(const double* __restrict__ f,
                                                                const double* __restrict__ alpha,
                                                                const int32_t* __restrict__ y, int64_t lo,
                                                                int64_t nloc, int64_t per, int T, double C, double eps,
                                                                CandRec* __restrict__ cand_h,
                                                                CandRec* __restrict__ cand_l,
                                                                const DecompCtl* __restrict__ ctl,
                                                                const int32_t* __restrict__ act,
                                                                const int32_t* __restrict__ boff,
                                                                const uint8_t* __restrict__ shr) {
  if (ctl->stop != SVM_STOP_RUNNING) return;
  constexpr int NW = kSelNT / 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t b0 = act ? int64_t(boff[blockIdx.x]) : int64_t(blockIdx.x) * per;
  const int64_t b1 = act ? int64_t(boff[blockIdx.x + 1]) : std::min<int64_t>(nloc, b0 + per);
  const double c_hi = C - eps, c_lo = 0.0 + eps, inf = __builtin_inf();
  __shared__ double wv[2][NW];
  __shared__ uint32_t wi[2][NW];
  VI ph{-inf, 0}, pl{inf, 0};  // the previous round's block picks (round 0: nothing excluded)
  for (int k = 0; k < T; ++k) {
    VI mn{inf, kSentinel}, mx{-inf, kSentinel};
    for (int64_t kk = b0 + t; kk < b1; kk += kSelNT) {  // ascending index within a thread
      const int64_t i = act ? int64_t(act[kk]) : kk;
      if (shr && shr[i]) continue;
      const double a = alpha[lo + i], fi = f[i];
      const int32_t yi = y[lo + i];
      const uint32_t gi = uint32_t(lo + i);
      const bool up = (yi == 1 && a < c_hi) || (yi == -1 && a > c_lo);
      const bool dn = (yi == 1 && a > c_lo) || (yi == -1 && a < c_hi);
      const bool eh = k == 0 || fi > ph.v || (fi == ph.v && gi > ph.i);
      const bool el = k == 0 || fi < pl.v || (fi == pl.v && gi > pl.i);
      if (up && eh && fi < mn.v) mn = VI{fi, gi};
      if (dn && el && fi > mx.v) mx = VI{fi, gi};
    }
    VIL a, b;
    wave_arg_pair(mn, mx, a, b);
    if (lane == 0) {
      wv[0][w] = a.v;
      wi[0][w] = a.i;
      wv[1][w] = b.v;
      wi[1][w] = b.i;
    }
    __syncthreads();
    VI bh{wv[0][0], wi[0][0]}, bl{wv[1][0], wi[1][0]};
#pragma unroll
    for (int q = 1; q < NW; ++q) {
      const VI ch{wv[0][q], wi[0][q]}, cl{wv[1][q], wi[1][q]};
      if (beats<true>(ch, bh)) bh = ch;
      if (beats<false>(cl, bl)) bl = cl;
    }
    __syncthreads();  // every thread has read the wave winners before the next round writes them
    if (t == 0) {
      const bool ok = bh.i != kSentinel && bh.v < inf;
      cand_h[int64_t(blockIdx.x) * T + k] = CandRec{ok ? bh.v : 0.0, ok ? int32_t(bh.i) : -1, 0};
    } else if (t == 64) {
      const bool ok = bl.i != kSentinel && bl.v > -inf;
      cand_l[int64_t(blockIdx.x) * T + k] = CandRec{ok ? bl.v : 0.0, ok ? int32_t(bl.i) : -1, 0};
    }
    ph = bh;
    pl = bl;
  }
}

// One workgroup over the L gathered candidates (Lr per GPU, GPU-major; the first Lh of each GPU's
// are I_high picks, T per selection block, the rest I_low): b_high = min f over the I_high
// candidates, b_low = max f over the I_low ones (the global extremes: every block's first pick is its
// own extreme), the stop test, and the working set = the candidates' ids sorted, without duplicates (a
// free SV may be in both lists), with their f (Wf).  No sort: selection blocks are disjoint id ranges
// in candidate order (GPU-major, block-major), so a candidate's place in W is its block's offset (a
// scan of the blocks' distinct counts) plus the number of distinct ids of its own block (2T picks)
// below it -- four barriers instead of a 55-stage bitonic network.
__global__ __launch_bounds__(kMaxWS) void ws_build_kernel(const CandRec* __restrict__ cand, int L, int Lr, int Lh, int T,
                                                          double tau, double tau_frac, int64_t max_iter,
                                                          int32_t* __restrict__ W, double* __restrict__ Wf,
                                                          DecompCtl* __restrict__ ctl, int32_t* __restrict__ mcount,
                                                          DecompCtl* __restrict__ pub) {
  if (ctl->stop != SVM_STOP_RUNNING) return;
  __shared__ int32_t s[kMaxWS];
  __shared__ int8_t kf[kMaxWS];
  __shared__ int32_t bcnt[kMaxWS / 2];
  __shared__ int32_t wsum[kMaxWS / 64];
  __shared__ double red[2][kMaxWS / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const CandRec c = t < L ? cand[t] : CandRec{0.0, -1, 0};
  double vh = __builtin_inf(), vl = -__builtin_inf();
  if (c.id >= 0) {
    if (t % Lr < Lh)
      vh = c.f;
    else
      vl = c.f;
  }
  for (int off = 32; off > 0; off >>= 1) {
    vh = fmin(vh, __shfl_xor(vh, off, 64));
    vl = fmax(vl, __shfl_xor(vl, off, 64));
  }
  if (lane == 0) {
    red[0][w] = vh;
    red[1][w] = vl;
  }
  // this candidate's selection block: its T high picks start at hb, its T low picks at hb + Lh
  const int nb = L / (2 * T), nbr = Lh / T;
  int blk = 0, hb = 0;
  if (t < L) {
    const int r = t / Lr, o = t - r * Lr, lb = (o < Lh ? o : o - Lh) / T;
    blk = r * nbr + lb;
    hb = r * Lr + lb * T;
  }
  s[t] = c.id;
  if (t < kMaxWS / 2) bcnt[t] = 0;
  __syncthreads();
  // the block's first occurrence of an id is the one kept
  bool keep = c.id >= 0;
  if (keep)
    for (int half = 0; half < 2; ++half)
      for (int j = hb + half * Lh, je = j + T; j < je; ++j)
        if (j < t && s[j] == c.id) keep = false;
  kf[t] = keep;
  if (keep) atomicAdd(&bcnt[blk], 1);
  __syncthreads();
  // exclusive scan of the blocks' distinct counts (nb <= 512 blocks)
  const int bv = t < nb ? bcnt[t] : 0;
  const int incl = wave_incl_scan(bv);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int wpre = 0;
  for (int q = 0; q < w; ++q) wpre += wsum[q];
  if (t < nb) bcnt[t] = wpre + incl - bv;
  __syncthreads();
  if (keep) {
    int j = bcnt[blk];
    for (int half = 0; half < 2; ++half)
      for (int i = hb + half * Lh, ie = i + T; i < ie; ++i) j += (kf[i] != 0 && s[i] < c.id) ? 1 : 0;
    W[j] = c.id;
    Wf[j] = c.f;  // duplicates of an id carry the same f
  }
  if (t == 0) {
    int m = 0;
    double bh = __builtin_inf(), bl = -__builtin_inf();
    for (int q = 0; q < kMaxWS / 64; ++q) {
      m += wsum[q];
      bh = fmin(bh, red[0][q]);
      bl = fmax(bl, red[1][q]);
    }
    ctl->b_high = bh;
    ctl->b_low = bl;
    int32_t st = SVM_STOP_RUNNING;
    if (ctl->outer > 0 && ctl->last_inner_it == 0)  // no progress on the last W (a reference stop reason in it)
      st = ctl->last_inner_reason == SVM_STOP_CONVERGED ? SVM_STOP_NO_CANDIDATE : ctl->last_inner_reason;
    else if (!(bh < __builtin_inf()) || !(bl > -__builtin_inf()))  // "i_high or i_low not found" (main3.cpp:205-209)
      st = SVM_STOP_NO_CANDIDATE;
    else if (bl <= bh + 2.0 * tau)
      st = SVM_STOP_CONVERGED;
    else if (ctl->inner_total + 1 > max_iter)  // the reference counts num_iter from 1 (main3.cpp:283-287)
      st = SVM_STOP_MAX_ITER;
    else if (m < 2 || m > kMaxWS)
      st = kStopInternal;
    // the ACTIVE problem stopped while points are shrunk: not a stop -- the host unshrinks (f recomputed
    // from alpha, every point active) and the next build tests all n points (decomp_shrink.h)
    if (st != SVM_STOP_RUNNING && st != SVM_STOP_MAX_ITER && st != kStopInternal && ctl->shrunk) st = kStopUnshrink;
    if (st != SVM_STOP_RUNNING) {
      ctl->stop = st;
      *mcount = 0;  // the rest of the batch's f updates are no-ops
      publish_ctl(*ctl, pub);
    } else {
      ctl->m = m;
      ctl->tau_in = fmax(tau, tau_frac * (bl - bh));
      ctl->max_inner = min(int64_t(20) * m, max_iter - ctl->inner_total);
    }
  }
}

// Qw[k] = Q[W[k]] (kq bytes), N0w[k], WNw[k]: one workgroup per working-set row.
__global__ __launch_bounds__(64) void ws_gather_kernel(const int8_t* __restrict__ Q, const int32_t* __restrict__ N0,
                                                       const double* __restrict__ WN, int kq,
                                                       const int32_t* __restrict__ W, const DecompCtl* __restrict__ ctl,
                                                       int8_t* __restrict__ Qw, int32_t* __restrict__ N0w,
                                                       double* __restrict__ WNw) {
  const int k = blockIdx.x;
  if (ctl->stop != SVM_STOP_RUNNING || k >= ctl->m) return;
  const int64_t src = W[k];
  const int4* s = reinterpret_cast<const int4*>(Q + src * int64_t(kq));
  int4* d = reinterpret_cast<int4*>(Qw + int64_t(k) * kq);
  for (int c = threadIdx.x; c < kq / 16; c += 64) d[c] = s[c];
  if (threadIdx.x == 0) {
    N0w[k] = N0[src];
    WNw[k] = WN[src];
  }
}

// ---- Newton polish of the working set's free variables (decomp_newton.h) ---------------------------------
// The inner workgroup's step on W's free set F (positions with c_lo < alpha < c_hi): the Cholesky of
// K_FF with the right-hand sides f_F and 1 as two extra rows, the back substitution, b and u, the step
// cut at the first bound, alpha and f of every position of W updated.  gA / gF: W's alpha and f by
// position (the caller's registers spilled there around the call); Amat: (|F| + 2) x ldA scratch.
// Every entry's arithmetic is newton_step_ref's, in its order (decomp_newton.h):
//   * the factorisation is left-looking in panels of kNwPW columns: a row's panel entries first take the
//     terms of every earlier column (ascending j, from the panel's own rows staged in LDS), then wave 0
//     factors the panel in LDS column by column (the diagonal's sqrt, the divisions, the updates of the
//     panel's later columns) with no workgroup barrier;
//   * the back substitution goes by blocks of 64 columns from the last: wave 0 solves the block's
//     triangle (staged in LDS) one column at a time, then every thread applies the block's 64 x to its
//     entries below, in descending column order;
//   * sums and the step's arg-min in the sequential order (thread 0; wave_arg's value-then-lowest-index).
// Returns 0 (nothing changed), 1 (full step) or 2 (cut at a bound), the same in every thread.
constexpr int kNwPW = 16;      // panel width
constexpr int kNwMax = 512;    // |F| bound of the LDS buffers (NewtonCfg::max_free is clamped to it)
// The factorisation's row updates for one panel (newton_wg): pb[r][c] = A[p0 + r][p0 + c] - sum_{j < p0}
// L[p0 + r][j] L[p0 + c][j] (ascending j) for the panel's rows r < ract and columns c < pw (lower entries;
// the right-hand-side rows nf, nf + 1 take every column), lp[j][c] = L[p0 + c][j] -- on FP64 MFMA
// (v_mfma_f64_16x16x4f64): a wave per 16-row tile of the panel rows,
// 16 columns, k-steps of 4 columns j..j+3.  The instruction sums its four products into the accumulator
// as four fused multiply-adds in k order -- measured bit for bit against the chain c = fma(a0, b0, c);
// ... fma(a3, b3, c) on 512,000 random entries (bench_kernels/mfma_f64_order.hip) -- so with A = -L (exact)
// every entry takes exactly newton_step_ref's ascending fma chain.  Lane l: A = -L[p0 + row0 + (l & 15)]
// [j + (l >> 4)], B = L[p0 + (l & 15)][j + (l >> 4)] (lp[j][c]); D: col = l & 15, row = (l >> 4) + 4 r.
__device__ __forceinline__ void newton_rows_mfma(const double* __restrict__ Amat, int64_t ldA,
                                                 const double* __restrict__ lp, double* __restrict__ pb, int p0, int pw,
                                                 int nf, int ract, int lane, int w, int nw) {
  const int col = lane & 15, g = lane >> 4;
  const int ntile = (ract + 15) / 16;
  for (int tile = w; tile < ntile; tile += nw) {
    const int r0 = tile * 16;
    const int ar = r0 + col;                 // the A operand's row (panel-local)
    const bool arv = ar < ract;
    const double* arow = Amat + int64_t(p0 + (arv ? ar : 0)) * ldA;
    f64x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = r0 + g + 4 * r, i = p0 + rr;
      acc[r] = rr < ract && col < pw && (i >= nf || p0 + col <= i) ? Amat[int64_t(i) * ldA + p0 + col] : 0.0;
    }
    // A operands 16 k-steps (64 columns) at a time, the next 16 loaded while these run: one wave per SIMD,
    // so only loads in flight hide their latency; k-steps at or beyond p0 are skipped (uniform), never
    // run with zero operands (an added 0 could flip the sign of a zero)
    // (the loads are unconditional -- columns up to p0 + 127 < kMaxWS stay inside Amat's row, and what
    // lies beyond p0 is never used -- so all 16 are in flight together; a branch around each would make
    // the compiler wait for every load before the next)
    double nx[16];
    auto load16 = [&](int j) {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const double v = arow[j + 4 * s2 + g];
        nx[s2] = arv ? -v : 0.0;
      }
    };
    load16(0);
    for (int j = 0; j < p0; j += 64) {
      double av[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) av[s2] = nx[s2];
      load16(j + 64);
      if (j + 64 <= p0) {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], lp[(j + 4 * s2 + g) * kNwPW + col], acc, 0, 0, 0);
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          if (j + 4 * s2 < p0)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], lp[(j + 4 * s2 + g) * kNwPW + col], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = r0 + g + 4 * r;
      if (rr < ract) pb[rr * kNwPW + col] = acc[r];
    }
  }
}

__device__ __forceinline__ int newton_wg(int m, const double* __restrict__ Kw, int64_t ldw, const int8_t* __restrict__ sy,
                                      double* __restrict__ gA, double* __restrict__ gF, double* __restrict__ Amat,
                                      double C, double eps, int max_free, int64_t* __restrict__ prof = nullptr) {
  constexpr int64_t ldA = kMaxWS;
  __shared__ int32_t fidx[kMaxWS];
  __shared__ __attribute__((aligned(16))) double pb[(kNwMax + 2) * kNwPW];  // the panel's rows; later x1, x2, u
  __shared__ __attribute__((aligned(16))) double lp[kNwMax * kNwPW];        // the panel's own rows of L (as [j][c]); later s1, s2, the diagonal blocks
  __shared__ int32_t s_wc[16];
  __shared__ int32_t s_fail, s_blk;
  __shared__ double s_t, s_b;
  __shared__ double s_wv[16];
  __shared__ uint32_t s_wi[16];
  const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, w = t >> 6, nw = nt >> 6;
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  if (prof && t == 0) prof[7] = wall_clock64();
  // 1. the free positions in ascending order
  int base = 0;
  for (int c0 = 0; c0 < m; c0 += nt) {
    const int k = c0 + t;
    const double ak = k < m ? gA[k] : 0.0;
    const bool fr = k < m && ak > c_lo && ak < c_hi;
    const unsigned long long bal = __ballot(fr);
    if (lane == 0) s_wc[w] = __popcll(bal);
    __syncthreads();
    int r = __popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
    for (int q = 0; q < nw; ++q) {
      if (q < w) r += s_wc[q];
      tot += s_wc[q];
    }
    if (fr) fidx[base + r] = k;
    base += tot;
    __syncthreads();
  }
  const int nf = base;
  if (nf < 2 || nf > min(max_free, kNwMax)) return 0;
  if (prof && threadIdx.x == 0) prof[0] = wall_clock64();
  // 2. A = K_FF (lower) and the right-hand sides f_F, 1 (rows nf, nf + 1); the lower triangle as one flat
  // range of nf (nf + 1) / 2 entries (row i starts at i (i + 1) / 2), 32 independent gathers per thread
  {
    constexpr int U = 32;
    const int64_t ne = int64_t(nf) * (nf + 1) / 2;
    for (int64_t e0 = t; e0 < ne; e0 += U * int64_t(nt)) {
      double v[U];
      int64_t dst[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e1 = e0 + int64_t(u) * nt, e = min(e1, ne - 1);  // clamped: the gathers are unconditional
        int i = int((__builtin_sqrt(8.0 * double(e) + 1.0) - 1.0) * 0.5);
        i = int64_t(i) * (i + 1) / 2 > e ? i - 1 : int64_t(i + 1) * (i + 2) / 2 <= e ? i + 1 : i;
        const int k = int(e - int64_t(i) * (i + 1) / 2);
        v[u] = Kw[int64_t(fidx[i]) * ldw + fidx[k]];
        dst[u] = e1 < ne ? int64_t(i) * ldA + k : -1;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (dst[u] >= 0) Amat[dst[u]] = v[u];
    }
  }
  for (int k = t; k < nf; k += nt) {
    Amat[int64_t(nf) * ldA + k] = gF[fidx[k]];
    Amat[int64_t(nf + 1) * ldA + k] = 1.0;
  }
  if (t == 0) s_fail = 0;
  __threadfence_block();
  __syncthreads();
  if (prof && threadIdx.x == 0) prof[1] = wall_clock64();
  // 3. the factorisation, a panel of kNwPW columns at a time: every panel row takes the terms of the earlier
  // columns (newton_rows, ascending j; the panel's own rows of L staged in LDS as lp[j][c]) into pb, wave 0
  // factors the panel's diagonal block in registers (a lane per row, readlane broadcasts), and a thread per
  // row then solves the rows below the block against it (ascending kk) and stores the panel to Amat.
  double* dblk = pb;  // the panel's diagonal block, kNwPW x kNwPW
  int64_t pt0 = 0;
  auto pstamp = [&](int k) {
    if (prof && t == 0) {
      const int64_t now = wall_clock64();
      if (pt0) prof[k] += now - pt0;
      pt0 = now;
    }
  };
  if (prof && t == 0) prof[8] = prof[9] = prof[10] = prof[11] = 0;
  for (int p0 = 0; p0 < nf; p0 += kNwPW) {
    const int pw = min(kNwPW, nf - p0);
    pstamp(11);
    for (int e = t; e < kNwPW * p0; e += nt) {  // lp[j][c] = L[p0 + c][j], j < p0
      const int j = e / kNwPW, c = e - j * kNwPW;
      lp[e] = c < pw ? Amat[int64_t(p0 + c) * ldA + j] : 0.0;
    }
    __syncthreads();
    // the earlier columns' terms on the panel's rows [p0, nf + 2), into pb[r][c] (r = row - p0): a thread per
    // row below 129 rows... above 128 rows (up to 3 rows per thread), 2 threads per row (8 columns each)
    // up to 128, 4 (4 columns each) up to 64 -- every lane busy however few rows are left
    const int ract = nf + 2 - p0;
    newton_rows_mfma(Amat, ldA, lp, pb, p0, pw, nf, ract, lane, w, nw);
    pstamp(8);
    __syncthreads();
    if (w == 0) {  // the diagonal block in wave 0's registers: lane r = row p0 + r
      double dr[kNwPW];
#pragma unroll
      for (int c = 0; c < kNwPW; ++c) dr[c] = lane < pw ? dblk[lane * kNwPW + c] : 0.0;
      bool bad = false;
#pragma unroll
      for (int kk = 0; kk < kNwPW; ++kk) {
        if (kk < pw) {
          const double d = read_lane64(dr[kk], kk);  // row kk's updated diagonal
          bad = bad || !(d > 1e-12);
          const double lkk = d > 1e-12 ? __builtin_sqrt(d) : 1.0;
          if (lane == kk) dr[kk] = lkk;
          if (lane > kk) dr[kk] = dr[kk] / lkk;
#pragma unroll
          for (int k2 = kk + 1; k2 < kNwPW; ++k2)
            if (k2 < pw) {
              const double lk2 = read_lane64(dr[kk], k2);  // L[p0 + k2][p0 + kk]
              if (lane >= k2) dr[k2] = __builtin_fma(-dr[kk], lk2, dr[k2]);
            }
        }
      }
      if (lane < pw)
#pragma unroll
        for (int c = 0; c < kNwPW; ++c) dblk[lane * kNwPW + c] = dr[c];
      if (lane == 0 && bad) s_fail = 1;
    }
    __syncthreads();
    pstamp(9);
    if (s_fail) return 0;
    // the rows below the block (and the two right-hand sides) against it, a thread per row; then every
    // row to Amat
    for (int r = t; r < ract; r += nt) {
      const int i = p0 + r;
      double sv[kNwPW];
#pragma unroll
      for (int c2 = 0; c2 < kNwPW / 2; ++c2) {
        const f64x2 v = reinterpret_cast<const f64x2*>(pb + r * kNwPW)[c2];
        sv[2 * c2] = v[0];
        sv[2 * c2 + 1] = v[1];
      }
      if (r >= pw) {
#pragma unroll
        for (int kk = 0; kk < kNwPW; ++kk)
          if (kk < pw) {
            sv[kk] = sv[kk] / dblk[kk * kNwPW + kk];
#pragma unroll
            for (int k2 = kk + 1; k2 < kNwPW; ++k2)
              if (k2 < pw) sv[k2] = __builtin_fma(-sv[kk], dblk[k2 * kNwPW + kk], sv[k2]);
          }
      }
#pragma unroll
      for (int c = 0; c < kNwPW; ++c)
        if (c < pw && (i >= nf || p0 + c <= i)) Amat[int64_t(i) * ldA + p0 + c] = sv[c];
    }
    __threadfence_block();
    __syncthreads();
    pstamp(10);
  }
  if (prof && threadIdx.x == 0) prof[2] = wall_clock64();
  // 4. back substitution: s1 / s2 = z (the right-hand-side rows), x = L^-T z, by blocks of 64 columns
  double* s1 = lp;
  double* s2 = lp + kNwMax;
  double* dB = lp + 2 * kNwMax;  // the block's triangle, 64 x 64
  double* x1 = pb;
  double* x2 = pb + kNwMax;
  for (int k = t; k < nf; k += nt) {
    s1[k] = Amat[int64_t(nf) * ldA + k];
    s2[k] = Amat[int64_t(nf + 1) * ldA + k];
  }
  for (int jb = (nf - 1) / 64 * 64; jb >= 0; jb -= 64) {
    const int je = min(jb + 64, nf), bw = je - jb;
    for (int e = t; e < 64 * 64; e += nt) {
      const int r = e >> 6, c = e & 63;
      dB[e] = r < bw && c <= r ? Amat[int64_t(jb + r) * ldA + jb + c] : 0.0;
    }
    __syncthreads();
    if (w == 0) {  // the block's triangle in registers: lane i holds column i (L_ji, j >= i) and s_i
      double col[64];
#pragma unroll
      for (int r = 0; r < 64; ++r) col[r] = dB[r * 64 + lane];
      const int i = jb + lane;
      double a1 = i < je ? s1[i] : 0.0, a2 = i < je ? s2[i] : 0.0;
#pragma unroll
      for (int r = 63; r >= 0; --r) {
        if (r < bw) {  // j = jb + r, descending
          const double ljj = read_lane64(col[r], r);
          const double xa = read_lane64(a1, r) / ljj, xb = read_lane64(a2, r) / ljj;
          if (lane == r) {
            x1[jb + r] = xa;
            x2[jb + r] = xb;
          }
          if (lane < r) {
            a1 = __builtin_fma(-col[r], xa, a1);
            a2 = __builtin_fma(-col[r], xb, a2);
          }
        }
      }
    }
    __syncthreads();
    for (int i = t; i < jb; i += nt) {  // the block's columns on the entries below it, descending j
      double a1 = s1[i], a2 = s2[i];
      for (int j0 = je - 1; j0 >= jb; j0 -= 32) {
        double l[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) l[u] = Amat[int64_t(max(j0 - u, jb)) * ldA + i];  // unconditional: all in flight
#pragma unroll
        for (int u = 0; u < 32; ++u)
          if (j0 - u >= jb) {
            a1 = __builtin_fma(-l[u], x1[j0 - u], a1);
            a2 = __builtin_fma(-l[u], x2[j0 - u], a2);
          }
      }
      s1[i] = a1;
      s2[i] = a2;
    }
    __syncthreads();
  }
  if (prof && threadIdx.x == 0) prof[3] = wall_clock64();
  // 5. b = sum x1 / sum x2 (ascending)
  if (t == 0) {
    double S1 = 0.0, S2 = 0.0;
    for (int k = 0; k < nf; ++k) {
      S1 += x1[k];
      S2 += x2[k];
    }
    const bool ok = S2 > 0.0 && __builtin_isfinite(S1);
    s_fail = ok ? 0 : 1;
    s_b = ok ? S1 / S2 : 0.0;
  }
  __syncthreads();
  if (s_fail) return 0;
  // 6. the step's cut: min over k of the bound ratios (value, then lowest k)
  const double b = s_b;
  double* dal = lp;  // dalpha by F position (s1 / s2 are consumed)
  VI best{__builtin_inf(), kSentinel};
  for (int k = t; k < nf; k += nt) {
    const double u = __builtin_fma(b, x2[k], -x1[k]);
    const double dk = sy[fidx[k]] == 1 ? u : -u;
    dal[k] = dk;
    const double ak = gA[fidx[k]];
    const double tk = dk > 0.0 ? (C - ak) / dk : dk < 0.0 ? (0.0 - ak) / dk : __builtin_inf();
    if (tk < best.v) best = VI{tk, uint32_t(k)};  // ascending k within a thread: strict keeps the lowest
  }
  const VIL wb = wave_arg<true>(best);
  if (lane == 0) {
    s_wv[w] = wb.v;
    s_wi[w] = wb.i;
  }
  __syncthreads();
  if (t == 0) {
    VI bb{s_wv[0], s_wi[0]};
    for (int q = 1; q < nw; ++q) {
      const VI c{s_wv[q], s_wi[q]};
      if (beats<true>(c, bb)) bb = c;
    }
    s_t = bb.v < 1.0 ? bb.v : 1.0;
    s_blk = bb.v < 1.0 ? int(bb.i) : -1;
  }
  __syncthreads();
  // 7. alpha, and the realised changes (an - a) y
  const double tt = s_t;
  const int blk = s_blk;
  double* ur = x1;  // x1 / x2 are consumed after the reads above
  __syncthreads();
  for (int k = t; k < nf; k += nt) {
    const double ak = gA[fidx[k]], dk = dal[k];
    double an = k == blk ? (dk > 0.0 ? C : 0.0) : __builtin_fma(tt, dk, ak);
    an = fmin(C, fmax(0.0, an));
    ur[k] = sy[fidx[k]] == 1 ? an - ak : ak - an;
    gA[fidx[k]] = an;
  }
  __threadfence_block();
  __syncthreads();
  if (prof && threadIdx.x == 0) prof[4] = wall_clock64();
  // 8. f of every position of W: f_q += sum_k K(F_k, q) ur_k (ascending k), 16 loads per batch
  for (int q0 = 0; q0 < m; q0 += 4 * nt) {  // four positions per thread at once: 4 x 16 loads in flight
    double sacc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < nf; k0 += 16) {
      double kv[4][16];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int q = min(q0 + v * nt + t, m - 1);  // clamped: the loads are unconditional, all in flight
#pragma unroll
        for (int u = 0; u < 16; ++u) kv[v][u] = Kw[int64_t(fidx[min(k0 + u, nf - 1)]) * ldw + q];
      }
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (k0 + u < nf) sacc[v] = __builtin_fma(kv[v][u], ur[k0 + u], sacc[v]);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = q0 + v * nt + t;
      if (q < m) gF[q] += sacc[v];
    }
  }
  __threadfence_block();
  __syncthreads();
  if (prof && t == 0) {
    prof[5] = wall_clock64();
    prof[6] = nf;
  }
  return blk >= 0 ? 2 : 1;
}

// One Newton step on a given working set (tests / timing, svmd_decomp_newton_probe): K(W, W) in Kw (m x
// m, row stride ldw), alpha and f by position in gA / gF (updated), labels y; *code_out = the step's code.
__global__ __launch_bounds__(256) void ws_newton_probe_kernel(int m, const double* __restrict__ Kw, int64_t ldw,
                                                              const int32_t* __restrict__ y, double* __restrict__ gA,
                                                              double* __restrict__ gF, double* __restrict__ Amat,
                                                              double C, double eps, int max_free,
                                                              int32_t* __restrict__ code_out, int64_t* __restrict__ prof) {
  __shared__ int8_t sy[kMaxWS];
  for (int k = threadIdx.x; k < kMaxWS; k += blockDim.x) sy[k] = k < m ? int8_t(y[k]) : int8_t(0);
  __syncthreads();
  const int code = newton_wg(m, Kw, ldw, sy, gA, gF, Amat, C, eps, max_free, prof);
  if (threadIdx.x == 0) *code_out = code;
}

// First-order SMO on the working set in ONE workgroup of NT threads: thread t holds the PER contiguous
// points W[t PER + e] (f, alpha, y in registers; its entries of a K(W, W) row are PER / 2 16-byte loads).
// Per iteration:
//   select   branch-free thread-local (value, lowest position) minimum over I_high and maximum over
//            I_low, carrying the winner's alpha, then the wave64 arg-reductions (wave_arg);
//   publish  lane 0 of every wave writes its two candidates to LDS (double-buffered by iteration
//            parity) -- the iteration's ONE barrier;
//   merge    every lane folds the NW per-wave candidates itself (LDS broadcast reads, the same serial
//            order and tie rule everywhere), so all waves hold the identical (i_high, i_low, b_high,
//            b_low, alpha_h, alpha_l) with no second barrier; the pair's labels come from LDS;
//   rows     K12 and this thread's entries of the two rows of the L2-resident K(W, W);
//   update   the reference's clip / eta / update arithmetic on the same inputs in every thread
//            (persist_solve's sequence, main3.cpp:235-275) and f += ch K(i, .) + cl K(j, .).
// Stops at W's own gap <= 2 tau_in, at max_inner, or on a reference stop reason.  Then the points
// whose alpha changed are compacted in position order: cols[j] = their global ids, coef[j] =
// (alpha_new - alpha_old) y, *mcount = how many -- the f update of all n points reads only those.
// With packed rows (a shrunk solve, pos_of: local row -> packed position or -1), cdiag[j] = column j's
// packed position on this GPU (-1: none), the f update's unit diagonal.
//   DP (second order only): a second pair per iteration from the same selection -- i2 = the best
//            I_high candidate of the waves other than i_high's, j2 = the first-order j (max f over
//            I_low) -- whose rows load beside row i_high; after the first pair's update it is applied
//            if it is still a violating pair (f_j2 > f_i2 + 2 tau_in) and feasible.  32 % fewer
//            iterations of the chain at 60k for ~10 % more work per iteration.
//   J2S (with DP): j2 by the second-order gain of row i2 instead of the first-order j (row i2 loads
//            beside row i before the gains; both gains reduce in the same wave / barrier / fold).
template <int NT, int PER, bool PROF = false, bool W2 = false, bool DP = false, bool J2S = false, bool NWT = false>
__global__ __launch_bounds__(NT) void ws_inner_kernel(const double* __restrict__ Kw, int64_t ldw,
                                                      const int32_t* __restrict__ W, DecompCtl* __restrict__ ctl,
                                                      const int32_t* __restrict__ y, double* __restrict__ alpha,
                                                      const double* __restrict__ Wf, double C, double eps,
                                                      int32_t* __restrict__ cols, double* __restrict__ coef,
                                                      int32_t* __restrict__ mcount, DecompHost* __restrict__ hs,
                                                      DecompCtl* __restrict__ pub, const int32_t* __restrict__ pos_of,
                                                      int64_t lo, int64_t nloc, int32_t* __restrict__ cdiag,
                                                      double* __restrict__ gAw, double* __restrict__ gFw,
                                                      double* __restrict__ nAmat, NwDev nw) {
  if (ctl->stop != SVM_STOP_RUNNING) return;
  const int m = ctl->m;
  const double tau_in = ctl->tau_in;
  const int64_t max_inner = ctl->max_inner;
  constexpr int NW = NT / 64;
  static_assert(PER % 2 == 0, "row entries are loaded 16 bytes at a time");
  __shared__ double pv[2][2][NW], pa[2][2][NW];
  __shared__ uint32_t pi[2][2][NW];
  __shared__ double qv[2][NW], qa[2][NW], qf[2][NW], qk[2][NW];  // W2: the second index's candidates
  __shared__ uint32_t qi[2][NW];
  __shared__ double rv[2][NW], ra[2][NW], rf[2][NW], rk[2][NW];  // J2S: the second pair's j candidates
  __shared__ uint32_t ri2[2][NW];
  __shared__ int8_t sy[NT * PER];
  __shared__ int32_t wcnt[PER][NW];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // position of this thread's element e: pair h = e / 2 of every lane is one 16-byte piece; a wave's 64
  // pieces of pair h are one contiguous kilobyte, and the NT / 64 waves' kilobytes of pair h are adjacent
  const int pbase = w * 128 + 2 * lane;
  auto pos = [&](int e) { return pbase + (e >> 1) * (2 * NT) + (e & 1); };
  double a[PER], a0[PER], ft[PER];
  bool yp[PER], yn[PER];  // y = +1 / y = -1 (padding: neither, so in neither set)
  int64_t gid[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int k = pos(e);
    const bool valid = k < m;
    gid[e] = valid ? W[k] : 0;
    a[e] = valid ? alpha[gid[e]] : 0.0;
    a0[e] = a[e];
    const int32_t yk = valid ? y[gid[e]] : 0;
    yp[e] = yk == 1;
    yn[e] = yk == -1;
    sy[k] = int8_t(yk);
    ft[e] = valid ? Wf[k] : 0.0;
  }
  const double c_hi = C - eps, c_lo = 0.0 + eps, inf = __builtin_inf();
  int64_t it = 0;
  int32_t reason = SVM_STOP_CONVERGED;
  // the Newton polish (decomp_newton.h): chain iterations with no bound-status change, starting at `every`
  // after a long last inner solve (newton_since0)
  int32_t since = NWT && ctl->last_m > 0 && double(ctl->last_inner_it) >= nw.frac * double(ctl->last_m) ? nw.every : 0;
  int32_t ntrig = 0;
  int64_t nsteps = 0;
  // PROF: wave 0's clock at the phase boundaries (select | publish+barrier | merge | row loads | update)
  int64_t pacc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int64_t pt = PROF ? int64_t(clock64()) : 0;
  const int64_t pc0 = pt, pw0 = PROF ? int64_t(wall_clock64()) : 0;
  // this thread's PER contiguous entries of row r of K(W, W) as 16-byte loads (in bounds: t PER + e <
  // NT PER <= ldw; the row base is 16-byte aligned: ldw even), zero beyond m
  auto row = [&](int r, double* out) {
    const double2* src = reinterpret_cast<const double2*>(Kw + int64_t(r) * ldw + pbase);
#pragma unroll
    for (int h = 0; h < PER / 2; ++h) {
      const double2 v = src[NT * h];
      out[2 * h] = pos(2 * h) < m ? v.x : 0.0;
      out[2 * h + 1] = pos(2 * h + 1) < m ? v.y : 0.0;
    }
  };
  // a wave-uniform element of K(W, W) through a VECTOR load (in order with the row loads on vmcnt): a
  // scalar load would share lgkmcnt with the folds' LDS reads, which would then wait for it
  auto kval = [&](int r, int c) {
    int64_t off = int64_t(r) * ldw + c;
    asm volatile("" : "+v"(off));
    return Kw[off];
  };
  auto stamp = [&](int k) {
    if constexpr (PROF) {
      const int64_t now = int64_t(clock64());
      pacc[k] += now - pt;
      pt = now;
    }
  };
  for (int par = 0;; par ^= 1) {
    double hv = inf, lv = -inf, ha = 0.0, la = 0.0;
    uint32_t hi = kSentinel, li = kSentinel;
#pragma unroll
    for (int e = 0; e < PER; ++e) {  // ascending position within a thread: strict compares keep the lowest
      const bool below = a[e] < c_hi, above = a[e] > c_lo;
      const bool in_high = (yp[e] && below) || (yn[e] && above);
      const bool in_low = (yp[e] && above) || (yn[e] && below);
      const bool ch = in_high && ft[e] < hv, cl = in_low && ft[e] > lv;
      const uint32_t k = uint32_t(pos(e));
      hv = ch ? ft[e] : hv;
      ha = ch ? a[e] : ha;
      hi = ch ? k : hi;
      lv = cl ? ft[e] : lv;
      la = cl ? a[e] : la;
      li = cl ? k : li;
    }
    int lmn, lmx;  // the lanes holding the wave's winners publish them (no cross-lane reads)
    wave_arg_pair_lanes(VI{hv, hi}, VI{lv, li}, lmn, lmx);
    stamp(0);
    if (lane == lmn) {
      pv[par][0][w] = hv;
      pi[par][0][w] = hi;
      pa[par][0][w] = ha;
    }
    if (lane == lmx) {
      pv[par][1][w] = lv;
      pi[par][1][w] = li;
      pa[par][1][w] = la;
    }
    __syncthreads();
    stamp(1);
    // the same pairwise tree fold in every lane (value, then lowest position): log2(NW) dependent steps
    // fold (value, position) only, tracking the winning wave; its alpha is read from LDS afterwards
    double fv[2][NW];
    uint32_t fi[2][NW];
    int fw[2][NW];
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        fv[sd][q] = pv[par][sd][q];
        fi[sd][q] = pi[par][sd][q];
        fw[sd][q] = q;
      }
#pragma unroll
    for (int st = 1; st < NW; st <<= 1)
#pragma unroll
      for (int q = 0; q + st < NW; q += 2 * st) {
        // bitwise, not short-circuit: the compiler turned || / && on these uniform values into branches
        const bool th = (fv[0][q + st] < fv[0][q]) | ((fv[0][q + st] == fv[0][q]) & (fi[0][q + st] < fi[0][q]));
        const bool tl = (fv[1][q + st] > fv[1][q]) | ((fv[1][q + st] == fv[1][q]) & (fi[1][q + st] < fi[1][q]));
        fv[0][q] = th ? fv[0][q + st] : fv[0][q];
        fi[0][q] = th ? fi[0][q + st] : fi[0][q];
        fw[0][q] = th ? fw[0][q + st] : fw[0][q];
        fv[1][q] = tl ? fv[1][q + st] : fv[1][q];
        fi[1][q] = tl ? fi[1][q + st] : fi[1][q];
        fw[1][q] = tl ? fw[1][q + st] : fw[1][q];
      }
    double bh = fv[0][0], bl = fv[1][0];
    uint32_t uih = fi[0][0], uil = fi[1][0];
    stamp(2);
    if (uih == kSentinel || uil == kSentinel) {
      reason = SVM_STOP_NO_CANDIDATE;
      break;
    }
    if (bl <= bh + 2.0 * tau_in) break;  // W's own optimum (reason stays CONVERGED)
    if (it >= max_inner) {
      reason = SVM_STOP_MAX_ITER;
      break;
    }
    if (NWT && since >= nw.every && ntrig < nw.per_solve) {  // uniform: the polish, then select again
      ++ntrig;
      since = 0;
#pragma unroll
      for (int e = 0; e < PER; ++e)
        if (pos(e) < m) {
          gAw[pos(e)] = a[e];
          gFw[pos(e)] = ft[e];
        }
      __threadfence_block();
      __syncthreads();
      int steps = 0;
      while (NWT && steps < nw.repeat) {
        const int code = newton_wg(m, Kw, ldw, sy, gAw, gFw, nAmat, C, eps, nw.max_free);
        if (code == 0) break;
        ++steps;
        if (code == 1) break;
      }
      if (steps > 0) {
#pragma unroll
        for (int e = 0; e < PER; ++e)
          if (pos(e) < m) {
            a[e] = gAw[pos(e)];
            ft[e] = gFw[pos(e)];
          }
        it += steps;
        nsteps += steps;
        continue;
      }
    }
    int ih = int(uih), il = int(uil);
    double K12, bl_upd = bl, al;  // the second index's f in the update (first order: b_low)
    double kh[PER], kl[PER];
    // DP: the second pair (i2, j2) and what its update needs, from the same selection
    int i2 = -1;
    double f2h = 0.0, a2h = 0.0, f2l = bl, a2l = 0.0;
    double2 r2h[PER / 2], r2l[PER / 2];  // DP: rows i2 and j2, raw, consumed by the second pair only
    double Kh_i2 = 0.0, Kh_j2 = 0.0, Kl_i2 = 0.0, Kl_j2 = 0.0, K2_12 = 0.0;
    bool dp_ok = false;
    if constexpr (DP) {
      const int wih = fw[0][0];
      double bv = inf;
      uint32_t bi = kSentinel;
      int bq = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const double v = pv[par][0][q];
        const uint32_t ix = pi[par][0][q];
        const bool take = (q != wih) & ((v < bv) | ((v == bv) & (ix < bi)));
        bv = take ? v : bv;
        bi = take ? ix : bi;
        bq = take ? q : bq;
      }
      i2 = bi != kSentinel ? int(bi) : -1;
      f2h = bv;
      a2h = pa[par][0][bq];
      a2l = pa[par][1][fw[1][0]];
      dp_ok = J2S ? i2 >= 0 : i2 >= 0 && il != ih && i2 != il;  // (not J2S) il is still the first-order j = j2
    }
    int j2 = il;
    double2 rj[PER / 2];  // second order: row j's raw pieces, consumed only after the clip arithmetic
    if constexpr (!W2) {
      // one memory round trip: K12 and this thread's entries of the two rows; the labels from LDS
      K12 = Kw[int64_t(ih) * ldw + il];
      row(ih, kh);
      row(il, kl);
      al = pa[par][1][fw[1][0]];
    } else {
      // second-order choice of the second index (smo_cpu.cpp / persist_solve WSS2): row i_high, then
      // the maximum of (f_t - b_high)^2 / a_t over I_low points above b_high (a_t = 2 - 2 K(i, t),
      // floored at eps; reciprocal approximation: only the choice depends on it), a second barrier
      // and fold, then row j
      row(ih, kh);  // unconditional loads (no exec-mask branch per load)
      if constexpr (J2S) {  // row i2 now (its gains need it); row j2 and the K values after the fold
        const int ri = dp_ok ? i2 : ih;
        const double2* s2h = reinterpret_cast<const double2*>(Kw + int64_t(ri) * ldw + pbase);
#pragma unroll
        for (int h = 0; h < PER / 2; ++h) r2h[h] = s2h[NT * h];
        Kh_i2 = kval(ih, ri);
      } else if constexpr (DP) {
        {  // issued after row i (unconditionally -- row i again when there is no second pair: no branch
           // around loads, whose merge made the compiler wait for all of them before the gains)
          const int ri = dp_ok ? i2 : ih, rj2 = dp_ok ? j2 : ih;
          const double2* s2h = reinterpret_cast<const double2*>(Kw + int64_t(ri) * ldw + pbase);
          const double2* s2l = reinterpret_cast<const double2*>(Kw + int64_t(rj2) * ldw + pbase);
#pragma unroll
          for (int h = 0; h < PER / 2; ++h) r2h[h] = s2h[NT * h];
#pragma unroll
          for (int h = 0; h < PER / 2; ++h) r2l[h] = s2l[NT * h];
          Kh_i2 = kval(ih, ri);
          Kh_j2 = kval(ih, rj2);
          K2_12 = kval(ri, rj2);
        }
      }
      if constexpr (PROF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(8);
      }
      double gv = inf;
      int ge = 0;  // the element of the thread's best gain: its alpha, f and K(i, j) are read by the winner
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const bool below = a[e] < c_hi, above = a[e] > c_lo;
        const bool in_low = (yp[e] && above) || (yn[e] && below);
        const double bb = ft[e] - bh;
        double at = 2.0 - 2.0 * kh[e];
        at = at <= 0.0 ? eps : at;
        // IEEE division (not v_rcp_f64): the choice is then reproducible on the host bit for bit
        // (svm_decomp_train_gram, the CPU oracle)
        const double gain = -(bb * bb) / at;
        const bool c = in_low && ft[e] > bh && gain < gv;
        gv = c ? gain : gv;
        ge = c ? e : ge;
      }
      const uint32_t gi = gv < inf ? uint32_t(pos(ge)) : kSentinel;
      double gv2 = inf;
      int ge2 = 0;
      if constexpr (J2S) {  // the same gain over I_low points above f(i2), on row i2 (f2h = inf: none)
#pragma unroll
        for (int e = 0; e < PER; ++e) {
          const bool below = a[e] < c_hi, above = a[e] > c_lo;
          const bool in_low = (yp[e] && above) || (yn[e] && below);
          const double bb = ft[e] - f2h;
          const double k2 = pos(e) < m ? ((e & 1) ? r2h[e >> 1].y : r2h[e >> 1].x) : 0.0;
          double at = 2.0 - 2.0 * k2;
          at = at <= 0.0 ? eps : at;
          const double gain = -(bb * bb) / at;
          const bool c = in_low && ft[e] > f2h && gain < gv2;
          gv2 = c ? gain : gv2;
          ge2 = c ? e : ge2;
        }
      }
      const uint32_t gi2 = gv2 < inf ? uint32_t(pos(ge2)) : kSentinel;
      const int lc = wave_arg_lane<true>(VI{gv, gi});
      const int lc2 = J2S ? wave_arg_lane<true>(VI{gv2, gi2}) : -1;
      stamp(9);
      if (lane == lc) {
        double ga = a[0], gf = ft[0], gk = kh[0];
#pragma unroll
        for (int e = 1; e < PER; ++e) {
          ga = ge == e ? a[e] : ga;
          gf = ge == e ? ft[e] : gf;
          gk = ge == e ? kh[e] : gk;
        }
        qv[par][w] = gv;
        qi[par][w] = gi;
        qa[par][w] = ga;
        qf[par][w] = gf;
        qk[par][w] = gk;
      }
      if (J2S && lane == lc2) {
        double ga = a[0], gf = ft[0], gk = r2h[0].x;
#pragma unroll
        for (int e = 1; e < PER; ++e) {
          ga = ge2 == e ? a[e] : ga;
          gf = ge2 == e ? ft[e] : gf;
          gk = ge2 == e ? ((e & 1) ? r2h[e >> 1].y : r2h[e >> 1].x) : gk;
        }
        rv[par][w] = gv2;
        ri2[par][w] = gi2;
        ra[par][w] = ga;
        rf[par][w] = gf;
        rk[par][w] = gk;
      }
      __syncthreads();
      stamp(10);
      // the same (value, lowest position) order as a serial fold, as a tree over (value, position);
      // the winner's alpha, f and K(i, j) are read from its wave's slot afterwards
      double cv[NW];
      uint32_t cj[NW];
      int cw[NW];
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        cv[q] = qv[par][q];
        cj[q] = qi[par][q];
        cw[q] = q;
      }
#pragma unroll
      for (int st = 1; st < NW; st <<= 1)
#pragma unroll
        for (int q = 0; q + st < NW; q += 2 * st) {
          const bool tk = (cv[q + st] < cv[q]) | ((cv[q + st] == cv[q]) & (cj[q + st] < cj[q]));
          cv[q] = tk ? cv[q + st] : cv[q];
          cj[q] = tk ? cj[q + st] : cj[q];
          cw[q] = tk ? cw[q + st] : cw[q];
        }
      if (cj[0] == kSentinel) {  // no I_low point above b_high (cannot happen while the gap is open)
        reason = SVM_STOP_NO_CANDIDATE;
        break;
      }
      il = int(cj[0]);
      stamp(11);
      {  // issued now, consumed after the clip / division below, which then runs under the loads' latency
        const double2* src = reinterpret_cast<const double2*>(Kw + int64_t(il) * ldw + pbase);
#pragma unroll
        for (int h = 0; h < PER / 2; ++h) rj[h] = src[NT * h];
      }
      if constexpr (J2S) {  // the second pair's j: the same fold over the second gains
        double dv[NW];
        uint32_t dj[NW];
        int dw[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          dv[q] = rv[par][q];
          dj[q] = ri2[par][q];
          dw[q] = q;
        }
#pragma unroll
        for (int st = 1; st < NW; st <<= 1)
#pragma unroll
          for (int q = 0; q + st < NW; q += 2 * st) {
            const bool tk = (dv[q + st] < dv[q]) | ((dv[q + st] == dv[q]) & (dj[q + st] < dj[q]));
            dv[q] = tk ? dv[q + st] : dv[q];
            dj[q] = tk ? dj[q + st] : dj[q];
            dw[q] = tk ? dw[q + st] : dw[q];
          }
        const bool jok = dj[0] != kSentinel;
        j2 = jok ? int(dj[0]) : ih;
        dp_ok = dp_ok && jok && j2 != ih && il != j2 && il != i2;
        f2l = rf[par][dw[0]];
        a2l = ra[par][dw[0]];
        K2_12 = rk[par][dw[0]];
        const int rj2 = dp_ok ? j2 : ih;
        const double2* s2l = reinterpret_cast<const double2*>(Kw + int64_t(rj2) * ldw + pbase);
#pragma unroll
        for (int h = 0; h < PER / 2; ++h) r2l[h] = s2l[NT * h];
        Kh_j2 = kval(ih, rj2);
        Kl_i2 = kval(il, dp_ok ? i2 : il);
        Kl_j2 = kval(il, rj2);
      } else if constexpr (DP) {
        dp_ok = dp_ok && il != j2 && il != i2;  // the second-order j must leave the second pair alone
        Kl_i2 = kval(il, dp_ok ? i2 : il);
        Kl_j2 = kval(il, dp_ok ? j2 : il);
      }
      al = qa[par][cw[0]];
      bl_upd = qf[par][cw[0]];
      K12 = qk[par][cw[0]];
    }
    const double ah = pa[par][0][fw[0][0]];
    const int32_t yh = sy[ih], yl = sy[il];
    if constexpr (PROF) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      stamp(3);
    }
    const double K11 = 1.0, K22 = 1.0;  // the Gram's unit diagonal
    const int s = yh * yl;
    const double eta = K11 + K22 - 2.0 * K12;
    double U, V;
    if (s == -1) {
      U = fmax(0.0, al - ah);
      V = fmin(C, C + al - ah);
    } else {
      U = fmax(0.0, al + ah - C);
      V = fmin(C, al + ah);
    }
    if (!(U <= V + 1e-12)) {
      reason = SVM_STOP_INFEASIBLE;
      break;
    }
    if (eta <= eps) {
      reason = SVM_STOP_NONPOS_ETA;
      break;
    }
    double al_new = al + double(yl) * (bh - bl_upd) / eta;
    if (al_new > V) al_new = V;
    if (al_new < U) al_new = U;
    const double ah_new = ah + double(s) * (al - al_new);
    const double ch = (ah_new - ah) * double(yh);
    const double cl = (al_new - al) * double(yl);
    // a bound-status change of an updated point (bound_status): the Newton polish waits for a settled set
    auto bst = [&](double v) { return v <= c_lo ? 0 : v >= c_hi ? 2 : 1; };
    bool moved_status = NWT && (bst(ah_new) != bst(ah) || bst(al_new) != bst(al));
    if constexpr (W2) {
#pragma unroll
      for (int h = 0; h < PER / 2; ++h) {
        double x = rj[h].x, z = rj[h].y;
        // an empty asm reading cl: the wait for row j's data lands here, after the division, not inside it
        asm volatile("" : "+v"(x), "+v"(z) : "v"(cl));
        kl[2 * h] = pos(2 * h) < m ? x : 0.0;
        kl[2 * h + 1] = pos(2 * h + 1) < m ? z : 0.0;
      }
    }
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int k = pos(e);
      ft[e] += ch * kh[e] + cl * kl[e];  // main3.cpp:274 operation order
      a[e] = k == ih ? ah_new : k == il ? al_new : a[e];
    }
    ++it;
    if constexpr (DP) {
      if (dp_ok && it < max_inner) {
        // the second pair's f after the first update, as its owner thread computed it just now
        const double fi2 = f2h + (ch * Kh_i2 + cl * Kl_i2);
        const double fj2 = f2l + (ch * Kh_j2 + cl * Kl_j2);
        const int32_t yh2 = sy[i2], yl2 = sy[j2];
        const int s2 = yh2 * yl2;
        const double eta2 = K11 + K22 - 2.0 * K2_12;
        double U2, V2;
        if (s2 == -1) {
          U2 = fmax(0.0, a2l - a2h);
          V2 = fmin(C, C + a2l - a2h);
        } else {
          U2 = fmax(0.0, a2l + a2h - C);
          V2 = fmin(C, a2l + a2h);
        }
        if (fj2 > fi2 + 2.0 * tau_in && U2 <= V2 + 1e-12 && !(eta2 <= eps)) {  // still violating, feasible
          double al2 = a2l + double(yl2) * (fi2 - fj2) / eta2;
          if (al2 > V2) al2 = V2;
          if (al2 < U2) al2 = U2;
          const double ah2 = a2h + double(s2) * (a2l - al2);
          const double ch2 = (ah2 - a2h) * double(yh2);
          const double cl2 = (al2 - a2l) * double(yl2);
          double k2h[PER], k2l[PER];
#pragma unroll
          for (int h = 0; h < PER / 2; ++h) {
            double x = r2h[h].x, z = r2h[h].y, u = r2l[h].x, v = r2l[h].y;
            asm volatile("" : "+v"(x), "+v"(z), "+v"(u), "+v"(v) : "v"(cl2));  // consumed here, not at the load
            k2h[2 * h] = pos(2 * h) < m ? x : 0.0;
            k2h[2 * h + 1] = pos(2 * h + 1) < m ? z : 0.0;
            k2l[2 * h] = pos(2 * h) < m ? u : 0.0;
            k2l[2 * h + 1] = pos(2 * h + 1) < m ? v : 0.0;
          }
#pragma unroll
          for (int e = 0; e < PER; ++e) {
            const int k = pos(e);
            ft[e] += ch2 * k2h[e] + cl2 * k2l[e];
            a[e] = k == i2 ? ah2 : k == j2 ? al2 : a[e];
          }
          ++it;
          if constexpr (NWT) moved_status = moved_status || bst(ah2) != bst(a2h) || bst(al2) != bst(a2l);
        }
      }
    }
    if constexpr (NWT) since = moved_status ? 0 : since + 1;
    stamp(4);
  }
  // compaction in position order: pair h, then wave, then lane, then e & 1
  bool chg[PER];
  int below[PER / 2];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    chg[e] = pos(e) < m && a[e] != a0[e];
    if (chg[e]) alpha[gid[e]] = a[e];
  }
#pragma unroll
  for (int h = 0; h < PER / 2; ++h) {
    const unsigned long long b0 = __ballot(chg[2 * h]), b1 = __ballot(chg[2 * h + 1]);
    const unsigned long long lt = (1ull << lane) - 1ull;
    below[h] = __popcll(b0 & lt) + __popcll(b1 & lt);
    if (lane == 0) wcnt[h][w] = __popcll(b0) + __popcll(b1);
  }
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int h = 0; h < PER / 2; ++h) {
    int j = base + below[h];
    for (int q = 0; q < NW; ++q) {
      if (q < w) j += wcnt[h][q];
      base += wcnt[h][q];
    }
#pragma unroll
    for (int e = 2 * h; e < 2 * h + 2; ++e)
      if (chg[e]) {
        cols[j] = int32_t(gid[e]);
        coef[j] = (a[e] - a0[e]) * (yp[e] ? 1.0 : -1.0);
        // packed rows (shrinking): the column's row in the packed list, for the unit diagonal of the update
        if (cdiag) cdiag[j] = gid[e] >= lo && gid[e] < lo + nloc ? pos_of[gid[e] - lo] : -1;
        ++j;
      }
  }
  if (PROF && t == 0) {
    for (int k = 0; k < 5; ++k) hs->prof[k] += pacc[k];
    for (int k = 8; k < 12; ++k) hs->prof[k] += pacc[k];
    hs->prof[6] += int64_t(clock64()) - pc0;
    hs->prof[7] += int64_t(wall_clock64()) - pw0;
  }
  if (t == 0) {
    *mcount = base;
    ctl->outer += 1;
    ctl->inner_total += it;
    ctl->changed_total += base;
    ctl->last_inner_it = it;
    ctl->last_m = m;
    ctl->newton_steps += nsteps;
    ctl->last_inner_reason = reason;
    publish_ctl(*ctl, pub);
  }
}

// FP64 rows (real-valued data): Xo[k] = X[ids[k]] (ld doubles) and no[k] = nrm[ids[k]] for k < *count,
// one workgroup per row; no-op when gated (a stopped solve's remaining launches).
__global__ __launch_bounds__(64) void ws_gather_f64_kernel(const double* __restrict__ X, const double* __restrict__ nrm,
                                                           int64_t ld, const int32_t* __restrict__ ids,
                                                           const int32_t* __restrict__ count,
                                                           const int32_t* __restrict__ gate, double* __restrict__ Xo,
                                                           double* __restrict__ no) {
  const int k = blockIdx.x;
  if ((gate && *gate != 0) || k >= *count) return;
  const int64_t src = ids[k];
  const double2* s = reinterpret_cast<const double2*>(X + src * ld);
  double2* d = reinterpret_cast<double2*>(Xo + int64_t(k) * ld);
  for (int64_t c = threadIdx.x; c < ld / 2; c += 64) d[c] = s[c];
  if (threadIdx.x == 0) no[k] = nrm[src];
}

// FP64 rows: f[i] += sum_{k < *count} coef[k] Kc[i][k] (the block K(rows, moved columns)), one wave
// per row, lane-strided then a fixed butterfly (deterministic).
__global__ __launch_bounds__(256) void ws_rowsum_f64_kernel(const double* __restrict__ Kc, int64_t ldc,
                                                            const double* __restrict__ coef,
                                                            const int32_t* __restrict__ count, double* __restrict__ f,
                                                            int64_t nloc) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int cnt = *count;
  if (row >= nloc || cnt <= 0) return;
  const double* kr = Kc + row * ldc;
  double acc = 0.0;
  for (int k = lane; k < cnt; k += 64) acc += coef[k] * kr[k];
  acc = wave_sum(acc);
  if (lane == 0) f[row] += acc;
}

// Column cache bookkeeping of one f update (one 1024-thread workgroup): the moved columns cols[0..*count)
// the cache lacks get slots -- free persistent ones in moved order while the cache has room (slot_of
// keeps them for the rest of the fit), then, with `meta`, slots evicted by a CLOCK sweep, then scratch
// slots cap + position -- and are listed for the column store (miss_ids / miss_slots, state[1] of them);
// rd_slot[k] = every moved column's slot.  state[0] = the next free persistent slot; state[2] = 1 when
// the narrow column store takes the misses (at most 64: the tiled store's gate); state[3] = the clock
// hand, state[4] = the update's stamp.  meta (nullptr: fill-only) = owner[cap] (point id, -1 none),
// last[cap] (stamp of the last update that used the slot), ref[cap] (the CLOCK bit, set on every use):
// past ~2M rows the distinct moved columns outnumber the slots a quarter of the HBM holds, and the
// columns the solve moves late are not the ones it moved first.  A victim is a slot this update does not
// read whose bit the hand finds clear (the hand clears the bits it passes); a cached column is the
// recomputed one bit for bit, so the policy never changes a result.
__device__ __forceinline__ int block_excl_scan_1024(bool v, int32_t* wsum, int& total) {
  const int k = threadIdx.x, lane = k & 63, w = k >> 6;
  const unsigned long long bal = __ballot(v);
  if (lane == 0) wsum[w] = __popcll(bal);
  __syncthreads();
  int r = __popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
  for (int q = 0; q < 16; ++q) {
    if (q < w) r += wsum[q];
    tot += wsum[q];
  }
  __syncthreads();  // wsum is reused by the next scan
  total = tot;
  return r;
}

__global__ __launch_bounds__(1024) void ws_cache_plan_kernel(const int32_t* __restrict__ cols,
                                                             const int32_t* __restrict__ count,
                                                             int32_t* __restrict__ slot_of, int32_t cap,
                                                             int32_t* __restrict__ state, int32_t* __restrict__ rd_slot,
                                                             int32_t* __restrict__ miss_ids,
                                                             int32_t* __restrict__ miss_slots,
                                                             int32_t* __restrict__ meta,
                                                             const int32_t* __restrict__ cdiag,
                                                             int32_t* __restrict__ miss_diag) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t vict[kMaxWS];
  __shared__ int32_t s_nv, s_hand, s_stop;
  const int k = threadIdx.x;
  const int cnt = *count;
  const bool valid = k < cnt;
  const int32_t id = valid ? cols[k] : -1;
  int32_t sl = valid ? slot_of[id] : 0;
  const bool miss = valid && sl < 0;
  int32_t* owner = meta;
  int32_t* last = meta ? meta + cap : nullptr;
  int32_t* ref = meta ? meta + 2 * int64_t(cap) : nullptr;
  const int32_t E = state[4] + 1;
  if (meta && valid && !miss) {  // hits: read by this update (never a victim now) and referenced
    last[sl] = E;
    ref[sl] = 1;
  }
  int tot = 0;
  const int r = block_excl_scan_1024(miss, wsum, tot);  // its barriers publish the hits' stamps
  const int32_t next = state[0];
  const int fresh = max(0, min(tot, cap - next));
  const int need = meta ? tot - fresh : 0;
  if (k == 0) {
    s_nv = 0;
    s_hand = state[3];
  }
  __syncthreads();
  if (need > 0) {
    const int win = min(cap, kMaxWS);
    const int max_sweeps = 2 * ((cap + win - 1) / win) + 1;  // one full turn clears every unpinned bit
    for (int sweep = 0; sweep < max_sweeps; ++sweep) {
      const int have = s_nv, hand = s_hand;
      if (have >= need) break;  // uniform: read after a barrier
      const int32_t sx = int32_t((int64_t(hand) + k) % cap);
      // slots from `next` on are this update's fresh fills (the cache fills up in this very update)
      const bool cand = k < win && sx < next && last[sx] != E && ref[sx] == 0;
      int vtot = 0;
      const int vr = block_excl_scan_1024(cand, wsum, vtot);
      const bool take = cand && have + vr < need;
      if (take) {
        vict[have + vr] = sx;
        last[sx] = E;  // taken: not a candidate again when a small cache's next window wraps onto it
      }
      if (take && have + vr == need - 1) s_stop = k;  // the hand stops after the last victim it needs
      __syncthreads();
      const bool done = have + vtot >= need;
      const int passed = done ? s_stop + 1 : win;
      if (k < passed && !take && last[sx] != E) ref[sx] = 0;  // second chance used up
      __syncthreads();
      if (k == 0) {
        s_nv = min(need, have + vtot);
        s_hand = int32_t((int64_t(hand) + passed) % cap);
      }
      __syncthreads();
    }
  }
  const int nv = s_nv;
  if (miss) {
    if (r < fresh) {
      sl = next + r;
    } else if (r - fresh < nv) {
      sl = vict[r - fresh];
      const int32_t old = owner[sl];
      if (old >= 0) slot_of[old] = -1;  // not a column of this update: its slot would be pinned
    } else {
      sl = cap + k;  // no slot free or evictable: a scratch slot for this update only
    }
    if (sl < cap) {
      slot_of[id] = sl;
      if (meta) {
        owner[sl] = id;
        last[sl] = E;
        ref[sl] = 1;
      }
    }
    miss_ids[r] = id;
    miss_slots[r] = sl;
    if (cdiag) miss_diag[r] = cdiag[k];  // packed rows: the column's packed position (the unit diagonal)
  }
  if (valid) rd_slot[k] = sl;
  __syncthreads();  // every thread has read state[0] / state[3] / state[4]
  if (k == 0) {
    state[0] = next + fresh;
    state[1] = tot;
    state[2] = tot <= 64 ? 1 : 0;
    state[3] = s_hand;
    state[4] = E;
  }
}

// f[i] += sum_k coef[k] K(i, cols[k]) from the column cache, in the GEMV + half-sum order, bit for bit
// (igram GEMV epilogue + ws_fsum_count_kernel): per 64-column half, lane l's two terms (columns l and
// 32 + l) summed from 0, the 32-lane xor butterfly (16, 8, 4, 2, 1) as seen by lane 0 -- a binary tree
// whose leaves in evaluation order are the 5-bit bit-reversed lanes, so a 6-deep stack of completed
// subtrees replaces the 32 lane values --, the halves added in index order, then one add into f.
// A thread per RPT rows (16-byte loads: ldc is a multiple of 4); the 32 leaves of a half run as 4
// rolled groups of 8 (8 column pairs of loads in flight per group; unrolled, the compiler hoisted all
// 64 and ran at 3 waves / SIMD: 4.3 against 5.9 TB/s), the level of a group's last leaf depending on g.
// Packed rows (a shrunk solve): row i of the cache is f[act[i]], i < *nrows.
template <int RPT>
__global__ __launch_bounds__(256) void ws_cache_fsum_kernel(const double* __restrict__ cache, int64_t ldc,
                                                             const int32_t* __restrict__ rd_slot,
                                                             const double* __restrict__ coef,
                                                             const int32_t* __restrict__ count, double* __restrict__ f,
                                                             int64_t nloc, const int32_t* __restrict__ act = nullptr,
                                                             const int32_t* __restrict__ nrows = nullptr) {
  const int64_t i = RPT * (int64_t(blockIdx.x) * blockDim.x + threadIdx.x);
  const int cnt = *count;
  if (nrows) nloc = std::min<int64_t>(nloc, *nrows);
  if (i >= nloc || cnt <= 0) return;
  const int halves = (cnt + 63) / 64;
  const double* base = cache + i;
  double s[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) s[r] = 0.0;
  for (int c = 0; c < halves; ++c) {
    double st[6][RPT];
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = 8 * g + jj;
        const int l = ((j & 1) << 4) | ((j & 2) << 2) | (j & 4) | ((j & 8) >> 2) | ((j & 16) >> 4);
        const int k0 = c * 64 + l, k1 = k0 + 32;
        double x[RPT];
#pragma unroll
        for (int r = 0; r < RPT; ++r) x[r] = 0.0;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int k = kk ? k1 : k0;
          if (k < cnt) {
            const double cf = coef[k];
            const f64x2* src = reinterpret_cast<const f64x2*>(base + int64_t(rd_slot[k]) * ldc);
#pragma unroll
            for (int r2 = 0; r2 < RPT / 2; ++r2) {
              const f64x2 v = src[r2];
              x[2 * r2] += cf * v[0];
              x[2 * r2 + 1] += cf * v[1];
            }
          }
        }
        int lev = 0;
#pragma unroll
        for (int t = jj; t & 1; t >>= 1, ++lev)
#pragma unroll
          for (int r = 0; r < RPT; ++r) x[r] = st[lev][r] + x[r];
        if (jj == 7) {  // lev == 3: continue up through the trailing ones of g
          if (g & 1) {
#pragma unroll
            for (int r = 0; r < RPT; ++r) x[r] = st[3][r] + x[r];
            if (g & 2) {
#pragma unroll
              for (int r = 0; r < RPT; ++r) x[r] = st[4][r] + x[r];
#pragma unroll
              for (int r = 0; r < RPT; ++r) st[5][r] = x[r];
            } else {
#pragma unroll
              for (int r = 0; r < RPT; ++r) st[4][r] = x[r];
            }
          } else {
#pragma unroll
            for (int r = 0; r < RPT; ++r) st[3][r] = x[r];
          }
        } else {
#pragma unroll
          for (int r = 0; r < RPT; ++r) st[lev][r] = x[r];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) s[r] += st[5][r];
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r)
    if (i + r < nloc) f[act ? int64_t(act[i + r]) : i + r] += s[r];
}

// f[i] += the first ceil(*mcount / 64) column halves of part (the ones the GEMV wrote).  Packed rows
// (a shrunk solve): part row i is f[act[i]], i < *nrows.
__global__ __launch_bounds__(256) void ws_fsum_count_kernel(const double* __restrict__ part, int64_t ldp,
                                                            const int32_t* __restrict__ mcount,
                                                            double* __restrict__ f, int64_t n,
                                                            const int32_t* __restrict__ act = nullptr,
                                                            const int32_t* __restrict__ nrows = nullptr) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int npart = (*mcount + 63) / 64;
  if (nrows) n = std::min<int64_t>(n, *nrows);
  if (i >= n || npart == 0) return;
  const double* p = part + i * ldp;
  double s = 0.0;
  for (int c = 0; c < npart; ++c) s += p[c];
  f[act ? int64_t(act[i]) : i] += s;
}

// ---- shrinking (decomp_shrink.h) ----------------------------------------------------------------------
// The shrink pass after an outer iteration: every active row of this GPU (the packed list act[0 ..
// *nrows), or all nloc rows) that the rule drops gets shr = 1; ctl->n_active counts what is left and
// ctl->shrunk records that a pass ran (the build then unshrinks instead of stopping).  The bounds are the
// outer iteration's build's.
__global__ __launch_bounds__(256) void ws_shrink_pass_kernel(const double* __restrict__ f,
                                                             const double* __restrict__ alpha,
                                                             const int32_t* __restrict__ y, int64_t lo, int64_t nloc,
                                                             const int32_t* __restrict__ act,
                                                             const int32_t* __restrict__ nrows,
                                                             uint8_t* __restrict__ shr, double C, double eps,
                                                             double margin, DecompCtl* __restrict__ ctl) {
  if (ctl->stop != SVM_STOP_RUNNING) return;
  __shared__ int32_t wdrop[4];
  const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t nr = act ? std::min<int64_t>(nloc, *nrows) : nloc;
  const double g = margin * (ctl->b_low - ctl->b_high);  // shrink_cuts
  const double hi_cut = ctl->b_low + g, lo_cut = ctl->b_high - g;
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  bool drop = false;
  if (k < nr) {
    const int64_t i = act ? int64_t(act[k]) : k;
    if (!shr[i]) {
      const int32_t yi = y[lo + i];
      const double a = alpha[lo + i], fi = f[i];
      const bool up = (yi == 1 && a < c_hi) || (yi == -1 && a > c_lo);
      const bool dn = (yi == 1 && a > c_lo) || (yi == -1 && a < c_hi);
      drop = (up && !dn && fi > hi_cut) || (dn && !up && fi < lo_cut);  // shrinkable()
      if (drop) shr[i] = 1;
    }
  }
  const unsigned long long b = __ballot(drop);
  if ((threadIdx.x & 63) == 0) wdrop[threadIdx.x >> 6] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int d = wdrop[0] + wdrop[1] + wdrop[2] + wdrop[3];
    if (d) atomicAdd(reinterpret_cast<unsigned long long*>(&ctl->n_active), static_cast<unsigned long long>(-int64_t(d)));
    if (blockIdx.x == 0) {
      ctl->shrunk = 1;
      ctl->passes += 1;
    }
  }
}

// Repacking the active rows, 1 of 2 (one workgroup per selection block of this GPU): the block's rows
// still active -- its packed rows [boff[b], boff[b + 1]) of the current list act, or its full range
// [b per, (b + 1) per) before the first repack (act null) -- counted into bcnt[b].
__global__ __launch_bounds__(256) void ws_pack_count_kernel(const int32_t* __restrict__ act,
                                                            const int32_t* __restrict__ boff, int64_t per,
                                                            int64_t nloc, const uint8_t* __restrict__ shr,
                                                            int32_t* __restrict__ bcnt) {
  __shared__ int32_t wsum[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t b0 = act ? int64_t(boff[blockIdx.x]) : int64_t(blockIdx.x) * per;
  const int64_t b1 = act ? int64_t(boff[blockIdx.x + 1]) : std::min<int64_t>(nloc, b0 + per);
  int c = 0;
  for (int64_t k = b0 + t; k < b1; k += 256) c += shr[act ? int64_t(act[k]) : k] ? 0 : 1;
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if (lane == 0) wsum[w] = c;
  __syncthreads();
  if (t == 0) bcnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// Repacking, 2 of 2 (one workgroup per selection block): the block's new offset (the sum of the counts
// before it; the last block also writes the total to nboff[nb] and *nrows), then its active rows in
// order to the new list nact, pos_of[row] = the new position (-1 for the rows dropped), and the packed
// copies of their quantised rows (Qa, N0a, WNa: the GEMV / column store's row operand).  It reads the old
// list (act, boff) and writes the other buffer of the pair, so no block overwrites a list another reads.
__global__ __launch_bounds__(256) void ws_pack_write_kernel(const int32_t* __restrict__ act,
                                                            const int32_t* __restrict__ boff, int64_t per,
                                                            int64_t nloc, const uint8_t* __restrict__ shr,
                                                            const int32_t* __restrict__ bcnt,
                                                            int32_t* __restrict__ nboff, int32_t* __restrict__ nrows,
                                                            int32_t* __restrict__ nact, int32_t* __restrict__ pos_of,
                                                            const int8_t* __restrict__ Q, const int32_t* __restrict__ N0,
                                                            const double* __restrict__ WN, int64_t lo, int kq,
                                                            int8_t* __restrict__ Qa, int32_t* __restrict__ N0a,
                                                            double* __restrict__ WNa) {
  __shared__ int32_t wsum[4];
  __shared__ int32_t rows[256], dst[256];
  __shared__ int32_t s_n;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nb = int(gridDim.x), b = int(blockIdx.x);
  {  // this block's offset: the counts of the blocks before it (nb <= 512)
    int v = 0;
    for (int q = t; q < b; q += 256) v += bcnt[q];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) wsum[w] = v;
    __syncthreads();
    if (t == 0) {
      const int base = wsum[0] + wsum[1] + wsum[2] + wsum[3];
      nboff[b] = base;
      s_n = base;
      if (b == nb - 1) {
        nboff[nb] = base + bcnt[b];
        *nrows = base + bcnt[b];
      }
    }
    __syncthreads();
  }
  int base = s_n;
  const int64_t b0 = act ? int64_t(boff[b]) : int64_t(b) * per;
  const int64_t b1 = act ? int64_t(boff[b + 1]) : std::min<int64_t>(nloc, b0 + per);
  const int cpr = kq / 16;  // 16-byte chunks per quantised row
  for (int64_t c0 = b0; c0 < b1; c0 += 256) {
    const int64_t k = c0 + t;
    const int64_t i = k < b1 ? (act ? int64_t(act[k]) : k) : -1;
    const bool keep = i >= 0 && !shr[i];
    const unsigned long long bal = __ballot(keep);
    __syncthreads();  // the previous chunk is done with wsum / s_n / rows / dst
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int r = __popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
    for (int q = 0; q < 4; ++q) {
      if (q < w) r += wsum[q];
      tot += wsum[q];
    }
    if (keep) {
      nact[base + r] = int32_t(i);
      pos_of[i] = base + r;
      rows[r] = int32_t(i);
      dst[r] = base + r;
      N0a[base + r] = N0[lo + i];
      WNa[base + r] = WN[lo + i];
    } else if (i >= 0) {
      pos_of[i] = -1;
    }
    __syncthreads();  // rows / dst complete
    for (int64_t c = t; c < int64_t(tot) * cpr; c += 256) {  // the kept rows' bytes, 16 at a time
      const int rr = int(c / cpr), ch = int(c - int64_t(rr) * cpr);
      reinterpret_cast<int4*>(Qa + int64_t(dst[rr]) * kq)[ch] =
          reinterpret_cast<const int4*>(Q + (lo + int64_t(rows[rr])) * kq)[ch];
    }
    base += tot;
  }
}

// Unshrink, on the device side: every row active again (shr = 0; the host resets the packed list to the
// identity), the control block running with no shrink pass since (origin = now), and the no-progress test
// disarmed for the next working set (last_inner_it = -1: the last inner solve ran on the active problem).
__global__ void ws_unshrink_ctl_kernel(DecompCtl* __restrict__ ctl, int64_t nloc) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    ctl->stop = SVM_STOP_RUNNING;
    ctl->shrunk = 0;
    ctl->n_active = nloc;
    ctl->last_inner_it = -1;
    ctl->last_m = 0;
  }
}

// pos_of = the identity (the packed list before any repack, or after an unshrink).
__global__ void ws_iota_kernel(int32_t* __restrict__ v, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) v[i] = int32_t(i);
}

__global__ void ws_init_kernel(const int32_t* __restrict__ y, double* __restrict__ alpha, double* __restrict__ f,
                               int64_t lo, int64_t nloc, int64_t n, int warm, DecompCtl* __restrict__ ctl) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n && !warm) alpha[i] = 0.0;
  if (i < nloc) f[i] = -static_cast<double>(y[lo + i]);  // main3.cpp:165-172
  if (i == 0 && ctl) ctl->n_active = nloc;
}

// Warm start: the ascending ids j with alpha_j != 0 into cols, alpha_j y_j into coef, their number to
// *count (device) and *count_h (pinned host).  One 1024-thread workgroup; each thread takes 8
// consecutive points of a 8192-point chunk, a workgroup exclusive scan of the per-thread counts
// places them (ascending order preserved).
__global__ __launch_bounds__(1024) void ws_nz_compact_kernel(const double* __restrict__ alpha,
                                                             const int32_t* __restrict__ y, int64_t n,
                                                             int32_t* __restrict__ cols, double* __restrict__ coef,
                                                             int32_t* __restrict__ count, int64_t* __restrict__ count_h) {
  constexpr int E = 8, NW = 1024 / 64;
  __shared__ int32_t wtot[NW];
  __shared__ int64_t base;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) base = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += int64_t(1024) * E) {
    const int64_t i0 = c0 + int64_t(t) * E;
    int cnt = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) cnt += (i0 + e < n && alpha[i0 + e] != 0.0) ? 1 : 0;
    int incl = cnt;  // inclusive wave scan
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    int64_t pos = base + incl - cnt;
    for (int q = 0; q < w; ++q) pos += wtot[q];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = i0 + e;
      if (i < n && alpha[i] != 0.0) {
        cols[pos] = int32_t(i);
        coef[pos] = alpha[i] * double(y[i]);
        ++pos;
      }
    }
    __syncthreads();
    if (t == 0) {
      int64_t tot = 0;
      for (int q = 0; q < NW; ++q) tot += wtot[q];
      base += tot;
    }
    __syncthreads();
  }
  if (t == 0) {
    *count = int32_t(base);
    *count_h = base;
  }
}

// counts[c] = the columns of warm-start chunk c (kMaxWS per chunk; the last one partial).
__global__ void ws_chunk_counts_kernel(const int32_t* __restrict__ count, int32_t* __restrict__ counts, int nchunks) {
  const int c = int(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c < nchunks) counts[c] = max(0, min(kMaxWS, *count - c * kMaxWS));
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

DecompShape decomp_shape(int64_t n, int qws, int world) {
  DecompShape d;
  d.q = std::max(4, std::min(qws, kMaxWS));
  // blocks of <= 4096 points, at least 64 blocks (each gives its own top-T picks), a multiple of 8 so
  // 1, 2, 4 or 8 GPUs own whole blocks and the distributed trajectory is the one-GPU one (another
  // world rounds to a multiple of it)
  const int64_t nb0 = std::max<int64_t>((n + kSelNT * kSelE - 1) / (kSelNT * kSelE), std::min<int64_t>(64, (n + 63) / 64));
  const int64_t mult = (8 % world == 0) ? 8 : int64_t(8) * world;
  d.NB = (nb0 + mult - 1) / mult * mult;
  // at most kMaxWS / 2 blocks (past 2,097,152 rows): their extreme pairs fill one working set, and the
  // blocks grow beyond kSelNT x kSelE points (ws_select_wide_kernel)
  d.NB = std::min<int64_t>(d.NB, int64_t(kMaxWS / 2) / mult * mult);
  d.per = d.NB > 0 ? (n + d.NB - 1) / d.NB : 0;
  // T picks per block and side; at least one, so the working-set capacity L = 2 NB T is the
  // requested q rounded down to the blocks, or 2 NB when q < 2 NB (every block contributes its extreme
  // pair: the union must hold the globally maximal violating pair).  stats[2] reports L.
  d.T = d.NB > 0 ? int(std::max<int64_t>(1, d.q / (2 * d.NB))) : 0;
  d.L = 2 * d.NB * d.T;
  d.ok = n >= 2 && n < int64_t(kSentinel) && d.NB >= 1 && d.L <= kMaxWS && world >= 1;
  return d;
}

// Decomposition solve on quantised rows (Q, N0, WN: all n rows; the plan's step weights in stw on the
// device).  alpha: n doubles (cold start: zeroed here).  q: working-set size (<= 1024).
// Distributed (world > 1): this GPU owns the blocks [rank NB / world, (rank + 1) NB / world) of the
// selection's global block partition, keeps f for their points only, and exchanges its candidate
// records once per outer iteration through `allgather`; every GPU then builds the same working set and
// runs the same inner solve on the same inputs (alpha is replicated and updated identically), and
// updates f for its own points.  With world dividing 8 the trajectory is the one-GPU trajectory.
// stats (kDecompStats int64): outer iterations, inner iterations, working-set capacity, solve
// microseconds, columns of the f updates (points moved, summed over the outer iterations), inner
// workgroup size, kernel-value path (0 exact-integer int8 MFMA, 1 FP64 MFMA), warm-start columns.
int run_decomp(DeviceCtx* ctx, const DecompRows& R, const int32_t* y, double* alpha, int64_t n, const svm_params& p,
               int qws, svm_result* r, int64_t* stats, const DecompOpts& o) {
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = ctx->stream;
  const int world = o.world, rank = o.rank;
  const DecompAllGather& allgather = o.allgather;
  if (world < 1 || rank < 0 || rank >= world || (world > 1 && !allgather)) {
    set_error("decomposition SMO: bad world / rank / exchange");
    return SVM_ERR_ARG;
  }
  const bool f64 = R.fp64();
  if (f64 ? (R.ld % 16 != 0 || !R.nrm) : (!R.Q || !R.P)) {
    set_error("decomposition SMO: bad row source");
    return SVM_ERR_ARG;
  }
  static const QuantPlan kNoPlan;
  const QuantPlan& P = f64 ? kNoPlan : *R.P;
  const int8_t* Q = R.Q;
  const int32_t* N0 = R.N0;
  const double *WN = R.WN, *stw = R.stw;
  svm_decomp_trace* tr = o.trace;
  if (tr && (world != 1 || tr->cap < 0 || (tr->n != 0 && tr->n != n))) {
    set_error("decomposition SMO: a trace needs one GPU and snapshots of n = %lld", (long long)n);
    return SVM_ERR_ARG;
  }
  const DecompShape sh = decomp_shape(n, qws, world);
  if (!sh.ok) {
    set_error("decomposition SMO: n = %lld is outside the solver's shapes (2 <= n < 2^31 - 1, %lld candidates <= %d, "
              "world <= 64)", (long long)n, (long long)sh.L, kMaxWS);
    return SVM_ERR_ARG;
  }
  const int64_t NBr = sh.NB / world, b0 = rank * NBr;
  const int64_t lo = std::min<int64_t>(n, b0 * sh.per), hi = std::min<int64_t>(n, (b0 + NBr) * sh.per);
  const int64_t nloc = hi - lo;
  const int T = sh.T;
  const int64_t Lr = 2 * NBr * T;  // this GPU's candidate records (I_high picks, then I_low)
  const char* wide_env = getenv("SVM355_DECOMP_WIDE_SELECT");
  const bool wide_select = sh.per > int64_t(kSelNT) * kSelE || T > 64 || (wide_env && atoi(wide_env) == 1);
  // inner workgroup: NT threads x PER points (NT * PER = 1024); SVM355_DECOMP_NT = 64 | 128 | 256 | 512
  int inner_nt = 256;
  if (const char* v = getenv("SVM355_DECOMP_NT")) inner_nt = atoi(v);
  if (inner_nt != 64 && inner_nt != 128 && inner_nt != 512 && inner_nt != 65) inner_nt = 256;
  // 65: one wave x 6 points (A/B probe of a one-wave inner solve; needs a working set of <= 384)
  if (inner_nt == 65 && sh.L > 384) {
    set_error("decomposition SMO: SVM355_DECOMP_NT=65 needs a working set of <= 384 points");
    return SVM_ERR_ARG;
  }
  // inner stop: the working set's own gap <= max(2 tau, 2 tau_frac gap) (SVM355_DECOMP_TAU_FRAC)
  double tau_frac = 0.1;
  if (const char* v = getenv("SVM355_DECOMP_TAU_FRAC")) tau_frac = atof(v);
  // at 0.5 and above the working set's stop (its gap <= tau_frac x 2 gap) holds before any update, so the
  // solve could make no progress (it would stop at once with a zero model)
  if (!(tau_frac >= 0.0 && tau_frac < 0.5)) {
    set_error("decomposition SMO: SVM355_DECOMP_TAU_FRAC must be in [0, 0.5), got %g", tau_frac);
    return SVM_ERR_ARG;
  }
  // SVM355_DECOMP_PROF=1: clock64 phase totals of the inner solves on stderr (diagnostic build)
  const bool prof = getenv("SVM355_DECOMP_PROF") && atoi(getenv("SVM355_DECOMP_PROF")) == 1;
  // inner pair selection: second order for j (default; fewer, longer iterations: 8,206 vs 14,334 at
  // 60k, 12% faster) or first order (SVM355_DECOMP_WSS=1)
  const bool inner_wss2 = !(getenv("SVM355_DECOMP_WSS") && atoi(getenv("SVM355_DECOMP_WSS")) == 1);
  // SVM355_DECOMP_WSS = 3 (the default): second order plus the second pair per iteration (DP); 2: one
  // pair (40k 17.0 -> 15.5 ms, 60k 20.8 -> 19.2, 120k 43.9 -> 42.7, 250k 84.9 -> 83.1, 1M 296 -> 289)
  const char* wss_env = getenv("SVM355_DECOMP_WSS");
  const bool inner_dp = inner_wss2 && (wss_env ? atoi(wss_env) >= 3 : true);
  // SVM355_DECOMP_WSS = 4: the second pair's j by the second-order gain of row i2 (opt-in)
  const bool inner_j2s = inner_dp && wss_env && atoi(wss_env) == 4;
  const int64_t ldw = kMaxWS;              // K(W, W) row stride
  const int64_t ldp = 2 * (kMaxWS / 128);  // column halves of the f update
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += al(bytes);
    return o;
  };
  // Column cache (exact-integer rows): the f update's kernel columns K(this GPU's rows, j) stay in HBM
  // per point for the rest of the fit, so a column moved again is a read, not an int8-MFMA
  // recomputation (64 / 75 / 85 % of the column uses at 60k / 250k / 1M repeat an earlier one,
  // profiles/r4_decomp_column_cache.txt); bit-identical to the GEMV path (ws_cache_fsum_kernel).
  // SVM355_DECOMP_CCACHE = 0 off, 1 on; default on once this GPU's int8 rows (nloc x kq bytes, read by
  // every recomputation) outgrow the 256 MB last-level cache: the recomputation then streams them from
  // HBM (192 MiB: 60k MNIST rows, 46 MB, are 4 % faster without the cache, 250k rows 2 % with it).
  bool use_cache = false;
  int32_t cache_cap = 0;
  // Sizing and allocating the cache and the workspace is one step per process: thread ranks sharing a
  // GPU (the loopback rehearsal) would otherwise read the same free memory, each take half of it, and
  // leave a later rank without room for its workspace.
  static std::mutex alloc_mu;
  std::unique_lock<std::mutex> alloc_lock(alloc_mu);
  // evict by CLOCK once the slots are taken (SVM355_DECOMP_CCACHE_EVICT=0: fill-only, the round-4 cache)
  const char* ev_env = getenv("SVM355_DECOMP_CCACHE_EVICT");
  const bool cache_evict = !(ev_env && atoi(ev_env) == 0);
  int64_t ldc_cache = 0;
  double* cache = nullptr;
  if (!f64 && nloc > 0) {
    const char* cc = getenv("SVM355_DECOMP_CCACHE");
    use_cache = cc ? atoi(cc) != 0 : nloc * int64_t(P.kq) > (int64_t(192) << 20);
  }
  if (use_cache) {
    // slots: twice the distinct columns measured per fit (~1,686 (n / 60k)^0.46), within half the free
    // HBM, plus kMaxWS scratch slots (moved columns beyond a full cache, this update only)
    int64_t cap = int64_t(2.0 * 1686.0 * std::pow(double(n) / 60000.0, 0.46));
    cap = std::min<int64_t>(std::max<int64_t>(cap, 1024), n);
    size_t free_b = 0, total_b = 0;
    SVMD_CHECK(hipMemGetInfo(&free_b, &total_b));
    ldc_cache = (nloc + 3) & ~int64_t(3);  // a multiple of 4: 16-byte row pairs (or quads) in the reader
    const size_t slot_b = size_t(ldc_cache) * 8;
    // the workspace allocated below (f, the GEMV partials, the per-point slot map, a warm start's columns
    // and ~64 MB of fixed parts) comes out of the same free memory
    const size_t ws_need = size_t(nloc + 1) * 8 * size_t(1 + ldp) + size_t(n) * (o.warm ? 16 : 4) + (size_t(64) << 20);
    const size_t ws_grow = ws_need > ctx->ws_bytes ? ws_need - ctx->ws_bytes : 0;
    const size_t avail = free_b + ctx->rc_cache_bytes > ws_grow ? free_b + ctx->rc_cache_bytes - ws_grow : 0;
    cap = std::min<int64_t>(cap, int64_t(avail / 2 / slot_b) - kMaxWS);
    // and at most a quarter of the GPU's HBM (SVM355_DECOMP_CCACHE_FRAC): the slab is a grow-only
    // buffer of the context, kept for the next fit, that PyTorch's allocator cannot see -- it must leave
    // room for the caller's tensors and other contexts on the device.  At 1M rows that is
    // ~8,000 slots of 8 MB for ~6,100 distinct columns a fit moves, so no fit of n <= 1M loses a hit.
    // (a context's own share when several solve side by side, svmd_set_ccache_frac; the env var overrides)
    double frac = ctx->ccache_frac >= 0.0 ? ctx->ccache_frac : 0.25;
    // processes sharing this GPU (torchrun ranks over host-staged gloo on one device; alloc_mu orders the
    // sizing within a process only): each takes its share of the quarter
    if (ctx->ccache_frac < 0.0)
      if (const char* lw = getenv("LOCAL_WORLD_SIZE")) {
        int ndev = 1;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) ndev = 1;
        const int sharing = (std::max(1, atoi(lw)) + ndev - 1) / ndev;
        frac /= double(sharing);
      }
    if (const char* v = getenv("SVM355_DECOMP_CCACHE_FRAC")) frac = std::min(0.9, std::max(0.0, atof(v)));
    cap = std::min<int64_t>(cap, int64_t(double(total_b) * frac / double(slot_b)) - kMaxWS);
    int64_t min_cap = 256;
    if (const char* v = getenv("SVM355_DECOMP_CCACHE_SLOTS")) {  // tests: a small cache (its scratch path)
      cap = std::min<int64_t>(cap, atoll(v));
      min_cap = 1;
    }
    if (cap >= min_cap && cap < int64_t(INT32_MAX) - kMaxWS) {
      cache = ctx->ensure_rc_cache(size_t(cap + kMaxWS) * slot_b);
      cache_cap = int32_t(cap);
    }
    use_cache = cache != nullptr;
    if (!use_cache) (void)hipGetLastError();  // a failed allocation is not sticky: the GEMV path runs
  }
  const size_t nl1 = size_t(std::max<int64_t>(nloc, 1));
  const size_t o_f = take(nl1 * 8), o_own = take(size_t(Lr) * sizeof(CandRec)),
               o_all = take(size_t(sh.L) * sizeof(CandRec)), o_W = take(kMaxWS * 4), o_Wf = take(kMaxWS * 8),
               o_Kw = take(size_t(kMaxWS) * ldw * 8), o_coef = take(kMaxWS * 8), o_cols = take(kMaxWS * 4),
               o_mcount = take(256), o_ctl = take(sizeof(DecompCtl));
  // exact-integer rows: the working set's quantised rows and the GEMV's column-half partials;
  // FP64 rows: the working set's and the moved columns' rows (+ norms) and the block K(rows, columns)
  const size_t o_Qw = f64 ? 0 : take(size_t(kMaxWS) * P.kq), o_N0w = f64 ? 0 : take(kMaxWS * 4),
               o_WNw = f64 ? 0 : take(kMaxWS * 8), o_part = f64 ? 0 : take(nl1 * ldp * 8),
               o_Xw = f64 ? take(size_t(kMaxWS) * R.ld * 8) : 0, o_nw = f64 ? take(kMaxWS * 8) : 0,
               o_Xc = f64 ? take(size_t(kMaxWS) * R.ld * 8) : 0, o_nc = f64 ? take(kMaxWS * 8) : 0,
               o_Kc = f64 ? take(nl1 * kMaxWS * 8) : 0;
  // column cache state: slot per point (-1 = none), the update's slots, its misses, {next free, misses}
  const size_t o_cslot = use_cache ? take(size_t(n) * 4) : 0, o_crd = use_cache ? take(kMaxWS * 4) : 0,
               o_cmid = use_cache ? take(kMaxWS * 4) : 0, o_cmsl = use_cache ? take(kMaxWS * 4) : 0,
               o_cst = use_cache ? take(64) : 0,
               o_cmeta = use_cache && cache_evict ? take(size_t(cache_cap) * 12) : 0;
  // K(W, W) through the narrow column store: the identity ids 0 .. kMaxWS - 1 and the column count
  const size_t o_wid = f64 ? 0 : take(kMaxWS * 4 + 64);
  // warm start (and the recomputation of f when a shrunk solve unshrinks): the nonzero alphas' ids and
  // alpha y (all n at most), the per-chunk column counts
  const ShrinkCfg shc = shrink_cfg(p);
  const bool nzbuf = o.warm || shc.on;
  const int64_t nchunks = (n + kMaxWS - 1) / kMaxWS;
  const size_t o_wcols = nzbuf ? take(size_t(n) * 4) : 0, o_wcoef = nzbuf ? take(size_t(n) * 8) : 0,
               o_wcnt = nzbuf ? take(size_t(nchunks + 1) * 4) : 0;
  // shrinking (decomp_shrink.h): the per-row flags; with packing (exact-integer rows) the packed lists of
  // active rows (two buffers), the selection blocks' offsets into them (two), the blocks' counts, the
  // rows' packed positions, the device-side packed row count, the moved columns' (and misses') packed
  // positions for the unit diagonal, and the packed copies of the quantised rows
  const char* pk_env = getenv("SVM355_DECOMP_PACK");
  const bool pack_on = shc.on && !f64 && nloc > 0 && !(pk_env && atoi(pk_env) == 0);
  double repack_frac = 0.75;  // repack when the active rows are at most this share of the packed ones
  if (const char* v = getenv("SVM355_DECOMP_REPACK")) repack_frac = std::min(1.0, std::max(0.0, atof(v)));
  const size_t o_shr = shc.on ? take(nl1) : 0;
  // the Newton polish (decomp_newton.h): W's alpha by position and the factorisation's scratch
  const NewtonCfg nwc = newton_cfg(p);
  const NwDev nwd{nwc.on ? 1 : 0, nwc.every, nwc.per_solve, nwc.repeat, nwc.max_free, 0, nwc.frac};
  const size_t o_gaw = take(kMaxWS * 8), o_namat = nwc.on ? take(size_t(kMaxWS + 2) * kMaxWS * 8) : 0;
  const size_t o_act = pack_on ? take(nl1 * 4 * 2) : 0, o_boff = pack_on ? take(size_t(NBr + 1) * 4 * 2) : 0,
               o_bcnt = pack_on ? take(size_t(NBr + 1) * 4) : 0, o_pos = pack_on ? take(nl1 * 4) : 0,
               o_nrows = pack_on ? take(64) : 0, o_cdiag = pack_on ? take(kMaxWS * 4) : 0,
               o_mdiag = pack_on ? take(kMaxWS * 4) : 0, o_Qa = pack_on ? take(nl1 * size_t(P.kq)) : 0,
               o_N0a = pack_on ? take(nl1 * 4) : 0, o_WNa = pack_on ? take(nl1 * 8) : 0;
  int rc = ctx->ensure_ws(off);
  if (rc) return rc;
  rc = ctx->ensure_pinned(sizeof(DecompHost) * 2 + 2 * sizeof(DecompCtl) + 64);
  if (rc) return rc;
  alloc_lock.unlock();
  char* ws = static_cast<char*>(ctx->ws);
  auto* f = reinterpret_cast<double*>(ws + o_f);
  auto* cown = reinterpret_cast<CandRec*>(ws + o_own);
  auto* call = world > 1 ? reinterpret_cast<CandRec*>(ws + o_all) : cown;
  auto* W = reinterpret_cast<int32_t*>(ws + o_W);
  auto* Wf = reinterpret_cast<double*>(ws + o_Wf);
  auto* Qw = reinterpret_cast<int8_t*>(ws + o_Qw);
  auto* N0w = reinterpret_cast<int32_t*>(ws + o_N0w);
  auto* WNw = reinterpret_cast<double*>(ws + o_WNw);
  auto* Kw = reinterpret_cast<double*>(ws + o_Kw);
  auto* coef = reinterpret_cast<double*>(ws + o_coef);
  auto* cols = reinterpret_cast<int32_t*>(ws + o_cols);
  auto* mcount = reinterpret_cast<int32_t*>(ws + o_mcount);
  auto* part = reinterpret_cast<double*>(ws + o_part);
  auto* Xw = reinterpret_cast<double*>(ws + o_Xw);
  auto* nw = reinterpret_cast<double*>(ws + o_nw);
  auto* Xc = reinterpret_cast<double*>(ws + o_Xc);
  auto* nc = reinterpret_cast<double*>(ws + o_nc);
  auto* Kc = reinterpret_cast<double*>(ws + o_Kc);
  auto* cslot = reinterpret_cast<int32_t*>(ws + o_cslot);
  auto* crd = reinterpret_cast<int32_t*>(ws + o_crd);
  auto* cmid = reinterpret_cast<int32_t*>(ws + o_cmid);
  auto* cmsl = reinterpret_cast<int32_t*>(ws + o_cmsl);
  auto* cst = reinterpret_cast<int32_t*>(ws + o_cst);
  auto* cmeta = use_cache && cache_evict ? reinterpret_cast<int32_t*>(ws + o_cmeta) : nullptr;
  auto* wid = reinterpret_cast<int32_t*>(ws + o_wid);  // [kMaxWS] identity, then the count kMaxWS
  auto* ctl = reinterpret_cast<DecompCtl*>(ws + o_ctl);
  auto* shr = shc.on ? reinterpret_cast<uint8_t*>(ws + o_shr) : nullptr;
  auto* gAw = reinterpret_cast<double*>(ws + o_gaw);
  auto* nAmat = nwc.on ? reinterpret_cast<double*>(ws + o_namat) : nullptr;
  double* Wfw = Wf;  // the inner solve's W-local f, also the Newton polish's
  int32_t* pact[2] = {reinterpret_cast<int32_t*>(ws + o_act), reinterpret_cast<int32_t*>(ws + o_act) + nl1};
  int32_t* pboff[2] = {reinterpret_cast<int32_t*>(ws + o_boff), reinterpret_cast<int32_t*>(ws + o_boff) + (NBr + 1)};
  auto* pbcnt = reinterpret_cast<int32_t*>(ws + o_bcnt);
  auto* pos_of = reinterpret_cast<int32_t*>(ws + o_pos);
  auto* pk_rows = reinterpret_cast<int32_t*>(ws + o_nrows);
  auto* cdiag = reinterpret_cast<int32_t*>(ws + o_cdiag);
  auto* mdiag = reinterpret_cast<int32_t*>(ws + o_mdiag);
  auto* Qa = reinterpret_cast<int8_t*>(ws + o_Qa);
  auto* N0a = reinterpret_cast<int32_t*>(ws + o_N0a);
  auto* WNa = reinterpret_cast<double*>(ws + o_WNa);
  // the packed state (host side): pk = the current list's buffer (-1: none, the rows in place -- before
  // the first repack and after an unshrink), pk_bound = an upper bound of the device's packed row count
  // (the active count the host last read: passes only drop rows)
  int pk = -1;
  int64_t pk_bound = nloc;
  // f += K(this GPU's rows, cols[0:*cnt]) coef: the exact-integer GEMV (column-half partials summed in
  // order) or, for FP64 rows, the moved columns' rows gathered, their block on FP64 MFMA and a row sum
  // tiled: also launch the tiled column store for updates of more than 64 misses (it exits at once
  // otherwise, but a launch over every row tile costs ~5-8 us); off after the first outer iterations,
  // where the narrow store takes any count itself (only the cold start misses hundreds of columns)
  // Packed rows (a shrunk solve, pk >= 0): the row operand is the packed copy (Qa, N0a, WNa) of the active
  // rows, pk_bound of them by the host's bound (the device count pk_rows gates the sums), the unit
  // diagonal from the columns' packed positions (the inner solve's cdiag), and the sums go to f[act[k]].
  auto f_update = [&](const int32_t* cl, const double* cf, const int32_t* cnt, bool tiled = true) -> int {
    if (nloc <= 0) return SVM_OK;
    const bool packed = pk >= 0;
    const int8_t* Qr = packed ? Qa : Q + lo * int64_t(P.kq);
    const int32_t* N0r = packed ? N0a : N0 + lo;
    const double* WNr = packed ? WNa : WN + lo;
    const int64_t nr = packed ? pk_bound : nloc, roff = packed ? 0 : lo;
    const int32_t* pa = packed ? pact[pk] : nullptr;
    const int32_t* pn = packed ? pk_rows : nullptr;
    if (nr <= 0) return SVM_OK;
    if (use_cache) {  // plan the slots, compute and store the missing columns, sum every column from the cache
      hipLaunchKernelGGL(ws_cache_plan_kernel, dim3(1), dim3(kMaxWS), 0, s, cl, cnt, cslot, cache_cap, cst, crd, cmid,
                         cmsl, cmeta, packed ? cdiag : nullptr, mdiag);
      SVMD_LAUNCH_CHECK();
      const int rc2 = launch_igram_colstore(s, Qr, N0r, WNr, stw, nr, roff, Q, N0, WN, cmid, cmsl, cst + 1, kMaxWS, P,
                                            p.gamma, cache, ldc_cache, cst + 2, tiled, packed ? mdiag : nullptr);
      if (rc2) return rc2;
      hipLaunchKernelGGL((ws_cache_fsum_kernel<2>), dim3(unsigned((nr + 511) / 512)), dim3(256), 0, s, cache,
                         ldc_cache, crd, cf, cnt, f, nr, pa, pn);
      SVMD_LAUNCH_CHECK();
      return SVM_OK;
    }
    if (!f64) {
      const int rc2 = launch_igram_gemv(s, Qr, N0r, WNr, stw, nr, roff, Q, N0, WN, cl, cf, cnt, kMaxWS, P, p.gamma, part,
                                        ldp, packed ? cdiag : nullptr);
      if (rc2) return rc2;
      hipLaunchKernelGGL(ws_fsum_count_kernel, dim3(unsigned((nr + 255) / 256)), dim3(256), 0, s, part, ldp, cnt, f, nr,
                         pa, pn);
      SVMD_LAUNCH_CHECK();
      return SVM_OK;
    }
    hipLaunchKernelGGL(ws_gather_f64_kernel, dim3(unsigned(kMaxWS)), dim3(64), 0, s, R.X, R.nrm, R.ld, cl, cnt,
                       nullptr, Xc, nc);
    SVMD_LAUNCH_CHECK();
    const int rc2 = launch_rbf_block_dev(s, R.X + lo * R.ld, R.nrm + lo, nloc, R.ld, Xc, nc, kMaxWS, R.ld, R.ld,
                                         p.gamma, Kc, kMaxWS, false, nullptr, cnt, cl, lo);
    if (rc2) return rc2;
    hipLaunchKernelGGL(ws_rowsum_f64_kernel, dim3(unsigned((nloc + 3) / 4)), dim3(256), 0, s, Kc, int64_t(kMaxWS), cf,
                       cnt, f, nloc);
    SVMD_LAUNCH_CHECK();
    return SVM_OK;
  };
  auto* hs = static_cast<DecompHost*>(ctx->pinned);
  auto* ctl_h = reinterpret_cast<DecompCtl*>(static_cast<char*>(ctx->pinned) + sizeof(DecompHost) * 2);
  std::memset(hs, 0, sizeof(DecompHost));
  SVMD_CHECK(hipMemsetAsync(ctl, 0, sizeof(DecompCtl), s));  // stop = SVM_STOP_RUNNING, counters 0
  if (f64) SVMD_CHECK(hipMemsetAsync(Xw, 0, size_t(kMaxWS) * R.ld * 8, s));  // rows beyond m stay finite
  const char* kww = getenv("SVM355_DECOMP_KWW");  // "sym": the triangular Gram launch (A/B)
  const bool kww_narrow = !f64 && !(kww && std::strcmp(kww, "sym") == 0) && P.kq <= 1536;
  if (kww_narrow) {
    static const std::vector<int32_t> ident = [] {
      std::vector<int32_t> v(kMaxWS + 1);
      for (int k = 0; k < kMaxWS; ++k) v[k] = k;
      v[kMaxWS] = kMaxWS;
      return v;
    }();
    SVMD_CHECK(hipMemcpyAsync(wid, ident.data(), ident.size() * 4, hipMemcpyHostToDevice, s));
  }
  auto cache_reset = [&]() -> int {  // no point has a slot, the first free slot is 0
    if (!use_cache) return SVM_OK;
    SVMD_CHECK(hipMemsetAsync(cslot, 0xFF, size_t(n) * 4, s));
    SVMD_CHECK(hipMemsetAsync(cst, 0, 64, s));
    if (cmeta) {  // owners and stamps -1, CLOCK bits clear
      SVMD_CHECK(hipMemsetAsync(cmeta, 0xFF, size_t(cache_cap) * 8, s));
      SVMD_CHECK(hipMemsetAsync(cmeta + 2 * int64_t(cache_cap), 0, size_t(cache_cap) * 4, s));
    }
    return SVM_OK;
  };
  if ((rc = cache_reset())) return rc;  // a fresh cache per fit
  if (shr) SVMD_CHECK(hipMemsetAsync(shr, 0, nl1, s));
  hipLaunchKernelGGL(ws_init_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, y, alpha, f, lo, nloc, n,
                     int(o.warm), ctl);
  SVMD_LAUNCH_CHECK();
  // f += K(:, nz) (alpha y)_nz: the nonzero alphas compacted (ascending ids), then the GEMV in chunks of
  // kMaxWS columns, each summed into f in order (svm_decomp_train_gram does the same): a warm start, and
  // the recomputation of f when a shrunk solve unshrinks.  The one host read: how many chunks.
  auto nz_update = [&](int64_t* nz_out) -> int {
    auto* wcols = reinterpret_cast<int32_t*>(ws + o_wcols);
    auto* wcoef = reinterpret_cast<double*>(ws + o_wcoef);
    auto* wcnt = reinterpret_cast<int32_t*>(ws + o_wcnt);
    auto* nz_h = reinterpret_cast<int64_t*>(static_cast<char*>(ctx->pinned) + sizeof(DecompHost) * 2 +
                                            2 * sizeof(DecompCtl));
    *nz_h = -1;
    hipLaunchKernelGGL(ws_nz_compact_kernel, dim3(1), dim3(1024), 0, s, alpha, y, n, wcols, wcoef, wcnt + nchunks,
                       nz_h);
    SVMD_LAUNCH_CHECK();
    SVMD_CHECK(hipStreamSynchronize(s));
    const int64_t nz = *nz_h;
    if (nz < 0 || nz > n) {
      set_error("decomposition SMO: the nonzero-alpha compaction returned no count");
      return SVM_ERR_INTERNAL;
    }
    const int nch = int((nz + kMaxWS - 1) / kMaxWS);
    if (nch > 0) {
      hipLaunchKernelGGL(ws_chunk_counts_kernel, dim3(unsigned((nch + 255) / 256)), dim3(256), 0, s, wcnt + nchunks,
                         wcnt, nch);
      SVMD_LAUNCH_CHECK();
    }
    for (int c = 0; c < nch; ++c) {
      const int rc2 = f_update(wcols + int64_t(c) * kMaxWS, wcoef + int64_t(c) * kMaxWS, wcnt + c);
      if (rc2) return rc2;
    }
    if (nz_out) *nz_out = nz;
    return SVM_OK;
  };
  int64_t warm_cols = 0;
  if (o.warm && (rc = nz_update(&warm_cols))) return rc;
  // shrinking, host side: o_dev = the device's outer-iteration count when the next enqueued one runs
  // (exact: only a stop or an unshrink turns launches into no-ops, and the host re-reads the count at
  // an unshrink), origin = the outer count at the start or the last unshrink, seen_active = the active
  // rows the host last read back
  int64_t o_dev = 0, origin = 0, seen_active = nloc, min_active = nloc, unshrinks = 0, repacks = 0;
  // repack: the active rows (not shrunk) into the other list buffer, their quantised rows copied, the
  // column cache (whose rows are the packed ones) cleared
  auto repack = [&]() -> int {
    const int nb = pk < 0 ? 0 : pk ^ 1;
    const int32_t* ca = pk < 0 ? nullptr : pact[pk];
    const int32_t* cb = pk < 0 ? nullptr : pboff[pk];
    hipLaunchKernelGGL(ws_pack_count_kernel, dim3(unsigned(NBr)), dim3(256), 0, s, ca, cb, sh.per, nloc, shr, pbcnt);
    SVMD_LAUNCH_CHECK();
    hipLaunchKernelGGL(ws_pack_write_kernel, dim3(unsigned(NBr)), dim3(256), 0, s, ca, cb, sh.per, nloc, shr, pbcnt,
                       pboff[nb], pk_rows, pact[nb], pos_of, Q, N0, WN, lo, P.kq, Qa, N0a, WNa);
    SVMD_LAUNCH_CHECK();
    pk = nb;
    pk_bound = seen_active;
    ++repacks;
    return cache_reset();
  };
  if (tr) tr->count = 0;
  // Outer iterations are enqueued `batch` at a time (SVM355_DECOMP_BATCH, default 1): every kernel reads
  // the device control block, so after the stop the rest are no-op launches.  Each batch ends with a
  // readback of the control block and an event; the host waits for batch k's event only after it has
  // enqueued batch k + 1, so the GPU always has the next batch queued (no idle host round trip).
  int batch = 1;  // with one batch always queued ahead, 1 already hides the host; more only adds no-op tail
  if (const char* v = getenv("SVM355_DECOMP_BATCH")) batch = std::max(1, atoi(v));
  if (tr) batch = 1;  // the trace reads every outer iteration back
  int32_t* gate = &ctl->stop;
  // fault injection (tests, world > 1): rank SVM355_DECOMP_FAIL_RANK fails when it is about to enqueue
  // outer iteration SVM355_DECOMP_FAIL_OUTER (default 0: before the first selection), while its peers
  // wait in their candidate all-gathers (decomp_cpu.cpp has the same hook)
  int64_t fail_outer = -1;
  if (const char* fr = getenv("SVM355_DECOMP_FAIL_RANK"); fr && world > 1 && atoi(fr) == rank) {
    const char* fo = getenv("SVM355_DECOMP_FAIL_OUTER");
    fail_outer = fo ? std::max(0, atoi(fo)) : 0;
  }
  const int64_t max_batches = p.max_iter / std::max(1, batch) + 64;  // a stop comes well before: never spin
#define SVM_WS_INNER_(NT, PER, PR, S2)                                                                            \
  do {                                                                                                             \
    if (inner_j2s && S2)                                                                                           \
      hipLaunchKernelGGL((ws_inner_kernel<NT, PER, PR, S2, S2, S2>), dim3(1), dim3(NT), 0, s, Kw, ldw, W, ctl, y,  \
                         alpha, Wf, p.C, p.eps, cols, coef, mcount, hs, pub, ipos, lo, nloc, icdiag, gAw, Wfw, nAmat, \
                         nwd);                                                                                     \
    else if (inner_dp && S2 && nwc.on)                                                                             \
      hipLaunchKernelGGL((ws_inner_kernel<NT, PER, PR, S2, S2, false, true>), dim3(1), dim3(NT), 0, s, Kw, ldw, W,  \
                         ctl, y, alpha, Wf, p.C, p.eps, cols, coef, mcount, hs, pub, ipos, lo, nloc, icdiag, gAw, Wfw, \
                         nAmat, nwd);                                                                              \
    else if (inner_dp && S2)                                                                                       \
      hipLaunchKernelGGL((ws_inner_kernel<NT, PER, PR, S2, S2>), dim3(1), dim3(NT), 0, s, Kw, ldw, W, ctl, y,      \
                         alpha, Wf, p.C, p.eps, cols, coef, mcount, hs, pub, ipos, lo, nloc, icdiag, gAw, Wfw, nAmat, \
                         nwd);                                                                                     \
    else                                                                                                           \
      hipLaunchKernelGGL((ws_inner_kernel<NT, PER, PR, S2>), dim3(1), dim3(NT), 0, s, Kw, ldw, W, ctl, y, alpha,   \
                         Wf, p.C, p.eps, cols, coef, mcount, hs, pub, ipos, lo, nloc, icdiag, gAw, Wfw, nAmat, nwd); \
  } while (0)
#define SVM_WS_INNER(NT, PER)                \
  if (prof && inner_wss2)                    \
    SVM_WS_INNER_(NT, PER, true, true);      \
  else if (prof)                             \
    SVM_WS_INNER_(NT, PER, true, false);     \
  else if (inner_wss2)                       \
    SVM_WS_INNER_(NT, PER, false, true);     \
  else                                       \
    SVM_WS_INNER_(NT, PER, false, false)
  // solo timing (DecompSolo): the two device segments of an outer iteration under the shared mutex,
  // each timed alone and waited for before the mutex is released
  DecompSolo* solo = (world > 1 && !tr) ? o.solo : nullptr;
  hipEvent_t sev[4] = {nullptr, nullptr, nullptr, nullptr};
  struct SoloEvents {
    hipEvent_t* e;
    ~SoloEvents() {
      for (int i = 0; i < 4; ++i)
        if (e[i]) (void)hipEventDestroy(e[i]);
    }
  } sev_guard{sev};
  if (solo)
    for (auto& e : sev) SVMD_CHECK(hipEventCreate(&e));
  std::unique_lock<std::mutex> solo_lk;
  auto solo_begin = [&](int k) -> int {
    if (!solo) return SVM_OK;
    solo_lk = std::unique_lock<std::mutex>(*solo->mu);
    SVMD_CHECK(hipEventRecord(sev[2 * k], s));
    return SVM_OK;
  };
  auto solo_end = [&](int k) -> int {
    if (!solo) return SVM_OK;
    SVMD_CHECK(hipEventRecord(sev[2 * k + 1], s));
    SVMD_CHECK(hipEventSynchronize(sev[2 * k + 1]));
    float ms = 0.0f;
    SVMD_CHECK(hipEventElapsedTime(&ms, sev[2 * k], sev[2 * k + 1]));
    (k == 0 ? solo->sel_ms : solo->rest_ms).push_back(double(ms));
    solo_lk.unlock();
    return SVM_OK;
  };
  const DecompCtl* fin = nullptr;  // the readback that saw the stop
  DecompCtl* ctl_pub = nullptr;  // ctl_h as the device addresses it
  SVMD_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctl_pub), ctl_h, 0));
  // The unshrink (decomp_shrink.h), when a readback shows kStopUnshrink: the queued batch ran as no-ops and
  // `ev` (recorded after it) is waited for under the exchange's policy; then every row is active again, the
  // rows are in place again (no packed list), the column cache is cleared, f is recomputed from alpha (the
  // warm start's chunked update), and the outer loop resumes at the device's outer count.
  const bool shrink_log = getenv("SVM355_DECOMP_SHRINK_LOG") && atoi(getenv("SVM355_DECOMP_SHRINK_LOG")) == 1;
  auto unshrink = [&](const DecompCtl& seen, hipEvent_t ev) -> int {
    if (ev && !(world > 1 && allgather.wait && allgather.wait(ev))) SVMD_CHECK(hipEventSynchronize(ev));
    hipLaunchKernelGGL(ws_unshrink_ctl_kernel, dim3(1), dim3(64), 0, s, ctl, nloc);
    SVMD_LAUNCH_CHECK();
    SVMD_CHECK(hipMemsetAsync(shr, 0, nl1, s));
    pk = -1;
    pk_bound = nloc;
    seen_active = nloc;
    int rc2 = cache_reset();
    if (rc2) return rc2;
    hipLaunchKernelGGL(ws_init_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, y, alpha, f, lo, nloc, n, 1,
                       ctl);
    SVMD_LAUNCH_CHECK();
    if ((rc2 = nz_update(nullptr))) return rc2;
    o_dev = origin = seen.outer;
    ++unshrinks;
    if (shrink_log) {
      SVMD_CHECK(hipStreamSynchronize(s));
      fprintf(stderr, "decomp: rank %d unshrink at outer %lld (%.3f ms)\n", rank, (long long)seen.outer, ms_since(t0));
    }
    return SVM_OK;
  };
  bool queued = false;  // a batch is in flight whose readback the host has not checked
  for (int64_t bt = 0;; ++bt) {
    DecompCtl* pub = tr ? nullptr : ctl_pub + (bt & 1);  // the trace path copies the block itself
    for (int bi = 0; bi < batch; ++bi) {
      if (bt * batch + bi == fail_outer) {
        set_error("injected failure of rank %d at outer iteration %lld", rank, (long long)fail_outer);
        return SVM_ERR_INTERNAL;
      }
      if ((rc = solo_begin(0))) return rc;
      // repack once the active rows the host last read are at most repack_frac of the packed ones
      if (pack_on && NBr > 0 && bi == 0 && seen_active < pk_bound && double(seen_active) <= repack_frac * double(pk_bound))
        if ((rc = repack())) return rc;
      const int32_t* sact = pk >= 0 ? pact[pk] : nullptr;
      const int32_t* sboff = pk >= 0 ? pboff[pk] : nullptr;
      if (NBr > 0)
        hipLaunchKernelGGL(wide_select ? ws_select_wide_kernel : ws_select_kernel, dim3(unsigned(NBr)), dim3(kSelNT),
                           0, s, f, alpha, y, lo, nloc, sh.per, T, p.C, p.eps, cown, cown + NBr * T, ctl, sact, sboff,
                           shr);
      SVMD_LAUNCH_CHECK();
      if ((rc = solo_end(0))) return rc;
      if (world > 1) allgather.gather(cown, int64_t(Lr * sizeof(CandRec)), call);  // stream-ordered
      if ((rc = solo_begin(1))) return rc;
      hipLaunchKernelGGL(ws_build_kernel, dim3(1), dim3(kMaxWS), 0, s, call, int(sh.L), int(Lr), int(NBr * T), int(T),
                         p.tau, tau_frac, int64_t(p.max_iter), W, Wf, ctl, mcount, pub);
      SVMD_LAUNCH_CHECK();
      if (!f64) {
        hipLaunchKernelGGL(ws_gather_kernel, dim3(unsigned(kMaxWS)), dim3(64), 0, s, Q, N0, WN, P.kq, W, ctl, Qw, N0w,
                           WNw);
        SVMD_LAUNCH_CHECK();
        // K(W, W) over the full capacity (rows beyond m are never read); skipped once stopped
        bool ww = false;
        if (kww_narrow && (rc = launch_igram_ww(s, Qw, N0w, WNw, stw, kMaxWS, wid, wid + kMaxWS, P, p.gamma, Kw, ldw,
                                                gate, &ww)))
          return rc;
        if (!ww) {
          rc = launch_igram_sym(s, Qw, N0w, WNw, const_cast<double*>(stw), kMaxWS, P, p.gamma, Kw, ldw, false, gate);
          if (rc) return rc;
        }
      } else {
        hipLaunchKernelGGL(ws_gather_f64_kernel, dim3(unsigned(kMaxWS)), dim3(64), 0, s, R.X, R.nrm, R.ld, W, &ctl->m,
                           gate, Xw, nw);
        SVMD_LAUNCH_CHECK();
        // K(W, W) on FP64 MFMA, columns bounded by m, unit diagonal; skipped once stopped
        rc = launch_rbf_block_dev(s, Xw, nw, kMaxWS, R.ld, Xw, nw, kMaxWS, R.ld, R.ld, p.gamma, Kw, ldw, true, gate,
                                  &ctl->m, nullptr, 0);
        if (rc) return rc;
      }
      const int32_t* ipos = pk >= 0 ? pos_of : nullptr;
      int32_t* icdiag = pk >= 0 ? cdiag : nullptr;
      if (inner_nt == 65)
        SVM_WS_INNER(64, 6);
      else if (inner_nt == 64)
        SVM_WS_INNER(64, 16);
      else if (inner_nt == 128)
        SVM_WS_INNER(128, 8);
      else if (inner_nt == 256)
        SVM_WS_INNER(256, 4);
      else
        SVM_WS_INNER(512, 2);
      SVMD_LAUNCH_CHECK();
      rc = f_update(cols, coef, mcount, bt * batch + bi < 4);
      if (rc) return rc;
      ++o_dev;  // this outer iteration's count once it has run
      if (shc.pass_after(o_dev, origin) && nloc > 0) {  // the shrink pass, with this outer iteration's bounds
        const int64_t np = pk >= 0 ? pk_bound : nloc;
        hipLaunchKernelGGL(ws_shrink_pass_kernel, dim3(unsigned((np + 255) / 256)), dim3(256), 0, s, f, alpha, y, lo,
                           nloc, pk >= 0 ? pact[pk] : nullptr, pk_rows, shr, p.C, p.eps, shc.margin, ctl);
        SVMD_LAUNCH_CHECK();
      }
      if ((rc = solo_end(1))) return rc;
#undef SVM_WS_INNER
#undef SVM_WS_INNER_
    }
    if (tr) {  // trace: every outer iteration is read back before the next is enqueued
      SVMD_CHECK(hipMemcpyAsync(ctl_h, ctl, sizeof(DecompCtl), hipMemcpyDeviceToHost, s));
      SVMD_CHECK(hipStreamSynchronize(s));
      if (ctl_h->stop == kStopUnshrink) {
        const DecompCtl seen = *ctl_h;
        if ((rc = unshrink(seen, nullptr))) return rc;
        continue;
      }
      if (ctl_h->stop != SVM_STOP_RUNNING) {
        fin = ctl_h;
        break;
      }
      seen_active = ctl_h->n_active;
      min_active = std::min(min_active, seen_active);
      if (tr->count < tr->cap) {
        const int64_t oi = tr->count++;
        const int m = ctl_h->m;
        int32_t mv = 0;
        SVMD_CHECK(hipMemcpy(&mv, mcount, 4, hipMemcpyDeviceToHost));
        if (tr->m) tr->m[oi] = m;
        if (tr->W) {
          SVMD_CHECK(hipMemcpy(tr->W + oi * kMaxWS, W, size_t(m) * 4, hipMemcpyDeviceToHost));
          for (int k = m; k < kMaxWS; ++k) tr->W[oi * kMaxWS + k] = -1;
        }
        if (tr->moved) tr->moved[oi] = mv;
        if (tr->cols) {
          SVMD_CHECK(hipMemcpy(tr->cols + oi * kMaxWS, cols, size_t(mv) * 4, hipMemcpyDeviceToHost));
          for (int k = mv; k < kMaxWS; ++k) tr->cols[oi * kMaxWS + k] = -1;
        }
        if (tr->coef) {
          SVMD_CHECK(hipMemcpy(tr->coef + oi * kMaxWS, coef, size_t(mv) * 8, hipMemcpyDeviceToHost));
          for (int k = mv; k < kMaxWS; ++k) tr->coef[oi * kMaxWS + k] = 0.0;
        }
        if (tr->inner) tr->inner[oi] = ctl_h->last_inner_it;
        if (tr->bounds) {
          tr->bounds[2 * oi] = ctl_h->b_high;
          tr->bounds[2 * oi + 1] = ctl_h->b_low;
        }
        if (tr->n == n && tr->alpha)
          SVMD_CHECK(hipMemcpy(tr->alpha + oi * n, alpha, size_t(n) * 8, hipMemcpyDeviceToHost));
        if (tr->n == n && tr->f) {
          SVMD_CHECK(hipMemcpy(tr->f + oi * n, f, size_t(n) * 8, hipMemcpyDeviceToHost));
          if (shr) {  // shrunk rows: NaN (their f is not part of the trajectory; the oracle's trace agrees)
            std::vector<uint8_t> sh_h(static_cast<size_t>(n));
            SVMD_CHECK(hipMemcpy(sh_h.data(), shr, size_t(n), hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < n; ++i)
              if (sh_h[size_t(i)]) tr->f[oi * n + i] = __builtin_nan("");
          }
        }
      }
      if (bt >= max_batches) {
        set_error("decomposition SMO: no stop after %lld outer iterations", (long long)ctl_h->outer);
        return SVM_ERR_INTERNAL;
      }
      continue;
    }
    SVMD_CHECK(hipEventRecord(ctx->ev_ctl[bt & 1], s));  // the batch's kernels published into ctl_h[bt & 1]
    if (!queued) {  // keep one batch queued ahead of the wait
      queued = true;
      continue;
    }
    const int64_t pb = bt - 1;
    hipEvent_t ev = ctx->ev_ctl[pb & 1];
    const auto tw = std::chrono::steady_clock::now();
    if (!(world > 1 && allgather.wait && allgather.wait(ev))) SVMD_CHECK(hipEventSynchronize(ev));
    if (o.host_wait_ms) *o.host_wait_ms += ms_since(tw);
    if (ctl_h[pb & 1].stop == kStopUnshrink) {  // batch bt ran as no-ops: drain it, unshrink, restart the pipeline
      const DecompCtl seen = ctl_h[pb & 1];
      if ((rc = unshrink(seen, ctx->ev_ctl[bt & 1]))) return rc;
      queued = false;
      continue;
    }
    if (ctl_h[pb & 1].stop != SVM_STOP_RUNNING) {
      fin = ctl_h + (pb & 1);  // batch bt (queued) runs as no-ops; the state is final
      break;
    }
    seen_active = ctl_h[pb & 1].n_active;
    min_active = std::min(min_active, seen_active);
    if (shrink_log)
      fprintf(stderr, "decomp: rank %d outer %lld gap %.6g active %lld packed %lld (%.3f ms)\n", rank,
              (long long)ctl_h[pb & 1].outer, ctl_h[pb & 1].b_low - ctl_h[pb & 1].b_high, (long long)seen_active,
              (long long)(pk >= 0 ? pk_bound : nloc), ms_since(t0));
    if (bt >= max_batches) {
      set_error("decomposition SMO: no stop after %lld outer iterations", (long long)ctl_h[pb & 1].outer);
      return SVM_ERR_INTERNAL;
    }
  }
  if (fin->stop == kStopInternal) {
    set_error("decomposition SMO: working set outside [2, %d] points", kMaxWS);
    return SVM_ERR_INTERNAL;
  }
  const int64_t outer = fin->outer, inner_total = fin->inner_total, changed_total = fin->changed_total;
  const int32_t stop = fin->stop;
  const double bh = fin->b_high, bl = fin->b_low;
  if (prof && inner_total > 0) {
    const double it = double(inner_total);
    fprintf(stderr, "decomp prof (clock64 ticks / inner iteration): select %.0f  publish+barrier %.0f  merge %.0f  "
            "row loads %.0f  update %.0f  (%lld iterations; inner kernels %.3f ms wall = %lld clock64 ticks)\n",
            hs->prof[0] / it, hs->prof[1] / it, hs->prof[2] / it,
            (hs->prof[3] + hs->prof[8] + hs->prof[9] + hs->prof[10] + hs->prof[11]) / it, hs->prof[4] / it,
            (long long)inner_total, hs->prof[7] / 1e5, (long long)hs->prof[6]);
    if (inner_wss2)
      fprintf(stderr, "decomp prof second-order j (inside row loads): row i %.0f  gains + wave reduction %.0f  "
              "publish + barrier %.0f  fold %.0f  row j %.0f\n", hs->prof[8] / it, hs->prof[9] / it,
              hs->prof[10] / it, hs->prof[11] / it, hs->prof[3] / it);
  }
  if (stats) {
    stats[0] = outer;
    stats[1] = inner_total;
    stats[2] = sh.L;  // the working-set capacity actually used (see decomp_shape)
    stats[3] = int64_t(ms_since(t0) * 1000.0);
    stats[4] = changed_total;
    stats[5] = inner_nt;
    stats[6] = f64 ? 1 : 0;
    stats[7] = warm_cols;
    stats[8] = unshrinks;
    stats[9] = fin->passes;
    stats[10] = min_active;
    stats[11] = repacks;
    stats[12] = fin->newton_steps;
  }
  if (r) {
    r->iterations = inner_total + 1;
    r->b_high = bh;
    r->b_low = bl;
    r->b = (bh + bl) / 2;
    r->stop_reason = stop;
    r->reserved = 0;
    r->n_sv = -1;
    r->seconds = ms_since(t0) / 1e3;
  }
  return SVM_OK;
}

namespace {

// The solve after quantisation: step weights to the device, the decomposition, the SV count.
int decomp_solve(DeviceCtx* ctx, const DecompRows& R, const int32_t* y_d, double* alpha_d, int64_t n,
                 const svm_params& p, int q, svm_result* r, int64_t* stats, const DecompOpts& o) {
  {
    TraceRange ts("svm355:decomp");
    const int rc = run_decomp(ctx, R, y_d, alpha_d, n, p, q > 0 ? q : 1024, r, stats, o);
    if (rc) return rc;
  }
  if (r) {
    int64_t c = 0;
    const int rc = count_sv(ctx, alpha_d, n, 1, p.sv_tol, &c);
    if (rc) return rc;
    r->n_sv = c;
  }
  return SVM_OK;
}

// The context's grow-only buffer holds the quantised rows (the solver's workspace is ctx->ws):
// Q (n x kq), N0, WN, the step weights and the quantiser's column tables (aux_bytes).
int decomp_quant_buffers(DeviceCtx* ctx, int64_t n, const QuantPlan& P, size_t aux_bytes, int8_t** Q, int32_t** N0,
                         double** WN, double** stw, void** aux) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t need = al(size_t(n) * P.kq) + al(size_t(n) * 4) + al(size_t(n) * 8) + al(P.step_w.size() * 8) +
                      al(aux_bytes);
  if (need > ctx->gram_bytes) {
    if (ctx->gram) {
      SVMD_CHECK(hipStreamSynchronize(ctx->stream));
      SVMD_CHECK(hipFree(ctx->gram));
      ctx->gram = nullptr;
      ctx->gram_bytes = 0;
    }
    SVMD_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx->gram), need));
    ctx->gram_bytes = need;
  }
  char* base = reinterpret_cast<char*>(ctx->gram);
  *Q = reinterpret_cast<int8_t*>(base);
  *N0 = reinterpret_cast<int32_t*>(base + al(size_t(n) * P.kq));
  *WN = reinterpret_cast<double*>(reinterpret_cast<char*>(*N0) + al(size_t(n) * 4));
  *stw = reinterpret_cast<double*>(reinterpret_cast<char*>(*WN) + al(size_t(n) * 8));
  *aux = reinterpret_cast<char*>(*stw) + al(P.step_w.size() * 8);
  return SVM_OK;
}

// The quantised rows' solve: the step weights to the device, then the decomposition.
int decomp_after_quant(DeviceCtx* ctx, const int8_t* Q, const int32_t* N0, const double* WN, double* stw,
                       const QuantPlan& P, const int32_t* y_d, double* alpha_d, int64_t n, const svm_params& p, int q,
                       svm_result* r, int64_t* stats, const DecompOpts& o) {
  SVMD_CHECK(hipMemcpyAsync(stw, P.step_w.data(), P.step_w.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  DecompRows R;
  R.Q = Q;
  R.N0 = N0;
  R.WN = WN;
  R.stw = stw;
  R.P = &P;
  return decomp_solve(ctx, R, y_d, alpha_d, n, p, q, r, stats, o);
}

}  // namespace

// The same solve from scaled FP64 rows (X_d: n x ld, the reference's host format, already min-max
// scaled on the device with mn_h / mx_h): quantize_rows produces the same Q, N0, WN as the uint8
// path, so the trajectory and the model are the uint8 path's.  Rows whose statistics admit no
// exact-integer plan (real-valued data; SVM355_DECOMP_F64=1 forces it) are solved on the FP64 rows
// themselves, every kernel value on FP64 MFMA (gram_mfma.hip) -- gpu_svm_main3.cu:119-147's RBF on
// arbitrary doubles.
int decomp_fit_rows(DeviceCtx* ctx, const double* X_d, int64_t n, int64_t ld, int64_t d, const double* mn_h,
                    const double* mx_h, const int32_t* y_d, double* alpha_d, const svm_params& p, int q, svm_result* r,
                    int64_t* stats, bool* used, double* prep_ms, const DecompOpts& o) {
  const auto t0 = std::chrono::steady_clock::now();
  *used = false;
  if (!decomp_shape(n, q, o.world).ok) return SVM_OK;  // beyond the solver's shapes: the caller's fallback
  const char* fe = getenv("SVM355_DECOMP_F64");
  const bool force_f64 = fe && atoi(fe) == 1;
  QuantPlan P;
  if (!force_f64 && mn_h && mx_h && plan_quant(mn_h, mx_h, d, &P) && P.kq <= 32 * 128) {
    int8_t* Q;
    int32_t* N0;
    double *WN, *stw;
    void* aux;
    int rc = decomp_quant_buffers(ctx, n, P, quantize_aux_bytes(P), &Q, &N0, &WN, &stw, &aux);
    if (rc) return rc;
    bool ok = false;
    {
      TraceRange tr("svm355:quantise");
      rc = quantize_rows(ctx->stream, X_d, n, ld, P, aux, Q, N0, WN, &ok);
      if (rc) return rc;
    }
    if (ok) {
      if (prep_ms) *prep_ms = ms_since(t0);
      rc = decomp_after_quant(ctx, Q, N0, WN, stw, P, y_d, alpha_d, n, p, q, r, stats, o);
      if (rc) return rc;
      *used = true;
      return SVM_OK;
    }
  }
  if (ld % 16 != 0 || ld < d) return SVM_OK;  // the FP64 block kernel's k-steps
  // The FP64-row solve keeps the moved columns' block K(rows, <= 1024 columns) per f update: n x 1024
  // doubles of workspace (8 GB at 1M rows).  When that does not fit 80 % of what the device has free
  // (plus the context's current workspace, which it would replace), nothing runs (*used = false) and
  // the caller takes the pairwise solver (SVC(solver="auto")).
  {
    size_t free_b = 0, total_b = 0;
    SVMD_CHECK(hipMemGetInfo(&free_b, &total_b));
    const double need = double(n) / double(std::max(1, o.world)) * double(kMaxWS) * 8.0 +
                        double(size_t(kMaxWS) * ld * 16);  // this GPU's rows (distributed: ~n / world)
    if (need > 0.8 * double(free_b + ctx->ws_bytes)) return SVM_OK;
  }
  // FP64 rows: their squared norms in the context's grow-only buffer, then the solve
  const size_t need = size_t(n) * 8;
  if (need > ctx->gram_bytes) {
    if (ctx->gram) {
      SVMD_CHECK(hipStreamSynchronize(ctx->stream));
      SVMD_CHECK(hipFree(ctx->gram));
      ctx->gram = nullptr;
      ctx->gram_bytes = 0;
    }
    SVMD_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx->gram), need));
    ctx->gram_bytes = need;
  }
  auto* nrm = reinterpret_cast<double*>(ctx->gram);
  int rc = launch_scale_norms(ctx->stream, const_cast<double*>(X_d), n, d, ld, nullptr, nullptr, nrm);
  if (rc) return rc;
  if (prep_ms) *prep_ms = ms_since(t0);
  DecompRows R;
  R.X = X_d;
  R.nrm = nrm;
  R.ld = ld;
  rc = decomp_solve(ctx, R, y_d, alpha_d, n, p, q, r, stats, o);
  if (rc) return rc;
  *used = true;
  return SVM_OK;
}

int decomp_fit_u8(DeviceCtx* ctx, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h, const double* mx_h,
                  const int32_t* y_d, double* alpha_d, const svm_params& p, int q, svm_result* r, int64_t* stats,
                  bool* used, double* prep_ms, const DecompOpts& o) {
  const auto t0 = std::chrono::steady_clock::now();
  *used = false;
  // outside the solver's shapes (n < 2 or n >= 2^31 - 1, decomp_shape): nothing runs, the caller takes
  // the pairwise solver (SVC(solver="auto"))
  if (!decomp_shape(n, q, o.world).ok) return SVM_OK;
  QuantPlan P;
  if (!plan_quant(mn_h, mx_h, d, &P) || P.kq > 32 * 128) return SVM_OK;  // igram's LDS table bound
  int8_t* Q;
  int32_t* N0;
  double *WN, *stw;
  void* aux;
  int rc = decomp_quant_buffers(ctx, n, P, quantize_u8_aux_bytes(P), &Q, &N0, &WN, &stw, &aux);
  if (rc) return rc;
  bool ok = false;
  {
    TraceRange tr("svm355:quantise");
    rc = quantize_u8_rows(ctx->stream, Xu_d, n, d, mn_h, mx_h, P, aux, Q, N0, WN, &ok);
    if (rc) return rc;
  }
  if (!ok) return SVM_OK;
  if (prep_ms) *prep_ms = ms_since(t0);
  rc = decomp_after_quant(ctx, Q, N0, WN, stw, P, y_d, alpha_d, n, p, q, r, stats, o);
  if (rc) return rc;
  *used = true;
  return SVM_OK;
}

}  // namespace svm355

using namespace svm355;

extern "C" {

// Decomposition SMO straight from uint8 pixel rows (exact-integer kernel values, no stored Gram).
// *used = 0 and nothing done when the rows' statistics do not admit the integer plan.  stats
// (optional, 8 int64): see run_decomp.
SVM_API int svmd_train_decomp_u8(void* h, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h,
                                 const double* mx_h, const int32_t* y_d, double* alpha_d, const svm_params* pp,
                                 int32_t q, svm_result* r, svmd_timing* timing, int64_t* stats, int32_t* used_out) {
  SVMD_CTX(h);
  if (used_out) *used_out = 0;
  if (!Xu_d || n < 2 || d <= 0 || !mn_h || !mx_h || !y_d || !alpha_d) {
    set_error("svmd_train_decomp_u8: bad arguments");
    return SVM_ERR_ARG;
  }
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  const auto t0 = std::chrono::steady_clock::now();
  int rc = ctx->begin();
  if (rc) return rc;
  bool used = false;
  double prep = 0.0;
  rc = decomp_fit_u8(ctx, Xu_d, n, d, mn_h, mx_h, y_d, alpha_d, p, q, r, stats, &used, &prep);
  if (rc) return rc;
  if (used && timing) {
    timing->gram_ms = prep;  // quantisation only: no Gram is stored
    timing->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    timing->smo_ms = timing->total_ms - prep;
  }
  if (used_out) *used_out = used ? 1 : 0;
  return ctx->end();
}

// The same solve from min-max scaled FP64 rows on the device (X_d: n x ld; mn_h / mx_h the training
// statistics they were scaled with): quantised into the same integers as the uint8 path, so the
// trajectory and the model are identical.  *used = 0 when the values admit no exact-integer plan.
SVM_API int svmd_train_decomp_rows(void* h, const double* X_d, int64_t n, int64_t ld, int64_t d, const double* mn_h,
                                   const double* mx_h, const int32_t* y_d, double* alpha_d, const svm_params* pp,
                                   int32_t q, svm_result* r, svmd_timing* timing, int64_t* stats, int32_t* used_out) {
  SVMD_CTX(h);
  if (used_out) *used_out = 0;
  if (!X_d || n < 2 || d <= 0 || ld < d || !mn_h || !mx_h || !y_d || !alpha_d) {
    set_error("svmd_train_decomp_rows: bad arguments");
    return SVM_ERR_ARG;
  }
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  const auto t0 = std::chrono::steady_clock::now();
  int rc = ctx->begin();
  if (rc) return rc;
  bool used = false;
  double prep = 0.0;
  rc = decomp_fit_rows(ctx, X_d, n, ld, d, mn_h, mx_h, y_d, alpha_d, p, q, r, stats, &used, &prep);
  if (rc) return rc;
  if (used && timing) {
    timing->gram_ms = prep;
    timing->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    timing->smo_ms = timing->total_ms - prep;
  }
  if (used_out) *used_out = used ? 1 : 0;
  return ctx->end();
}

// The general entry: uint8 rows (is_u8, X_d n x d) or min-max scaled FP64 rows (X_d n x ld), cold or
// warm start (alpha_d holds the start), an optional per-outer-iteration trace (tests: one
// synchronisation per outer iteration).  *used = 0 and nothing done without an exact-integer plan.
SVM_API int svmd_train_decomp(void* h, const void* X_d, int32_t is_u8, int64_t n, int64_t ld, int64_t d,
                              const double* mn_h, const double* mx_h, const int32_t* y_d, double* alpha_d,
                              const svm_params* pp, int32_t q, int32_t warm, svm_result* r, svmd_timing* timing,
                              int64_t* stats, int32_t* used_out, svm_decomp_trace* trace) {
  SVMD_CTX(h);
  if (used_out) *used_out = 0;
  if (!X_d || n < 2 || d <= 0 || (!is_u8 && ld < d) || !mn_h || !mx_h || !y_d || !alpha_d) {
    set_error("svmd_train_decomp: bad arguments");
    return SVM_ERR_ARG;
  }
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  const auto t0 = std::chrono::steady_clock::now();
  int rc = ctx->begin();
  if (rc) return rc;
  bool used = false;
  double prep = 0.0;
  DecompOpts o;
  o.warm = warm != 0;
  o.trace = trace;
  rc = is_u8 ? decomp_fit_u8(ctx, static_cast<const uint8_t*>(X_d), n, d, mn_h, mx_h, y_d, alpha_d, p, q, r, stats,
                             &used, &prep, o)
             : decomp_fit_rows(ctx, static_cast<const double*>(X_d), n, ld, d, mn_h, mx_h, y_d, alpha_d, p, q, r,
                               stats, &used, &prep, o);
  if (rc) return rc;
  if (used && timing) {
    timing->gram_ms = prep;
    timing->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    timing->smo_ms = timing->total_ms - prep;
  }
  if (used_out) *used_out = used ? 1 : 0;
  return ctx->end();
}

// The decomposition solver's f-update GEMV alone (tests): the uint8 rows quantised as a solve would,
// then f_out[i] = sum_k coef[k] K(lo + i, cols[k]) over k < m for the rows [lo, lo + nloc) -- the GEMV
// kernel with the device-side count m, its partial halves summed in order (the f update of a solve,
// from f = 0).  cols / coef / f_out are host arrays; m <= 1024.  *used = 0 without an exact plan.
SVM_API int svmd_decomp_gemv_u8(void* h, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h,
                                const double* mx_h, double gamma, int64_t lo, int64_t nloc, const int32_t* cols_h,
                                const double* coef_h, int32_t m, double* f_out, int32_t* used_out) {
  SVMD_CTX(h);
  if (used_out) *used_out = 0;
  if (!Xu_d || n < 1 || d <= 0 || lo < 0 || nloc < 1 || lo + nloc > n || m < 1 || m > kMaxWS || !cols_h || !coef_h ||
      !f_out) {
    set_error("svmd_decomp_gemv_u8: bad arguments");
    return SVM_ERR_ARG;
  }
  for (int k = 0; k < m; ++k)
    if (cols_h[k] < 0 || cols_h[k] >= n) {
      set_error("svmd_decomp_gemv_u8: column %d out of range", cols_h[k]);
      return SVM_ERR_ARG;
    }
  int rc = ctx->begin();
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  QuantPlan P;
  if (!plan_quant(mn_h, mx_h, d, &P) || P.kq > 32 * 128) return ctx->end();
  int8_t* Q;
  int32_t* N0;
  double *WN, *stw;
  void* aux;
  rc = decomp_quant_buffers(ctx, n, P, quantize_u8_aux_bytes(P), &Q, &N0, &WN, &stw, &aux);
  if (rc) return rc;
  bool ok = false;
  rc = quantize_u8_rows(s, Xu_d, n, d, mn_h, mx_h, P, aux, Q, N0, WN, &ok);
  if (rc) return rc;
  if (!ok) return ctx->end();
  SVMD_CHECK(hipMemcpyAsync(stw, P.step_w.data(), P.step_w.size() * 8, hipMemcpyHostToDevice, s));
  const int64_t ldp = 2 * (kMaxWS / 128);
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t o_cols = 0, o_coef = al(kMaxWS * 4), o_cnt = o_coef + al(kMaxWS * 8), o_f = o_cnt + 256,
               o_part = o_f + al(size_t(nloc) * 8), need = o_part + size_t(nloc) * ldp * 8;
  rc = ctx->ensure_ws(need);
  if (rc) return rc;
  char* ws = static_cast<char*>(ctx->ws);
  auto* cols = reinterpret_cast<int32_t*>(ws + o_cols);
  auto* coef = reinterpret_cast<double*>(ws + o_coef);
  auto* cnt = reinterpret_cast<int32_t*>(ws + o_cnt);
  auto* f = reinterpret_cast<double*>(ws + o_f);
  auto* part = reinterpret_cast<double*>(ws + o_part);
  SVMD_CHECK(hipMemcpyAsync(cols, cols_h, size_t(m) * 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(coef, coef_h, size_t(m) * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(cnt, &m, 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemsetAsync(f, 0, size_t(nloc) * 8, s));
  const char* vc = getenv("SVM355_GEMV_VIA_CACHE");
  if (vc && atoi(vc) != 0) {
    // the column-cache form of the same update (tests / timing): a fresh cache of m persistent slots
    // (every column a miss: the narrow store up to 64 columns, the tiled one beyond), then the reader
    const int64_t ldc = (nloc + 3) & ~int64_t(3);
    double* cache = ctx->ensure_rc_cache(size_t(m + kMaxWS) * ldc * 8);
    if (!cache) {
      set_error("svmd_decomp_gemv_u8: no memory for the column cache");
      return SVM_ERR_DEVICE;
    }
    const size_t o_cs = need, o_rd = o_cs + al(size_t(n) * 4), o_mid = o_rd + al(kMaxWS * 4),
                 o_msl = o_mid + al(kMaxWS * 4), o_st = o_msl + al(kMaxWS * 4), need2 = o_st + 256;
    rc = ctx->ensure_ws(need2);
    if (rc) return rc;
    ws = static_cast<char*>(ctx->ws);  // (re)allocated: every pointer again
    cols = reinterpret_cast<int32_t*>(ws + o_cols);
    coef = reinterpret_cast<double*>(ws + o_coef);
    cnt = reinterpret_cast<int32_t*>(ws + o_cnt);
    f = reinterpret_cast<double*>(ws + o_f);
    auto* cslot = reinterpret_cast<int32_t*>(ws + o_cs);
    auto* crd = reinterpret_cast<int32_t*>(ws + o_rd);
    auto* cmid = reinterpret_cast<int32_t*>(ws + o_mid);
    auto* cmsl = reinterpret_cast<int32_t*>(ws + o_msl);
    auto* cst = reinterpret_cast<int32_t*>(ws + o_st);
    SVMD_CHECK(hipMemcpyAsync(cols, cols_h, size_t(m) * 4, hipMemcpyHostToDevice, s));
    SVMD_CHECK(hipMemcpyAsync(coef, coef_h, size_t(m) * 8, hipMemcpyHostToDevice, s));
    SVMD_CHECK(hipMemcpyAsync(cnt, &m, 4, hipMemcpyHostToDevice, s));
    SVMD_CHECK(hipMemsetAsync(f, 0, size_t(nloc) * 8, s));
    SVMD_CHECK(hipMemsetAsync(cslot, 0xFF, size_t(n) * 4, s));
    SVMD_CHECK(hipMemsetAsync(cst, 0, 256, s));
    hipLaunchKernelGGL(ws_cache_plan_kernel, dim3(1), dim3(kMaxWS), 0, s, cols, cnt, cslot, m, cst, crd, cmid, cmsl,
                       nullptr, nullptr, nullptr);
    SVMD_LAUNCH_CHECK();
    rc = launch_igram_colstore(s, Q + lo * int64_t(P.kq), N0 + lo, WN + lo, stw, nloc, lo, Q, N0, WN, cmid, cmsl,
                               cst + 1, kMaxWS, P, gamma, cache, ldc, cst + 2);
    if (rc) return rc;
    hipLaunchKernelGGL((ws_cache_fsum_kernel<2>), dim3(unsigned((nloc + 511) / 512)), dim3(256), 0, s, cache, ldc, crd,
                       coef, cnt, f, nloc);
    SVMD_LAUNCH_CHECK();
  } else {
    rc = launch_igram_gemv(s, Q + lo * int64_t(P.kq), N0 + lo, WN + lo, stw, nloc, lo, Q, N0, WN, cols, coef, cnt,
                           kMaxWS, P, gamma, part, ldp);
    if (rc) return rc;
    hipLaunchKernelGGL(ws_fsum_count_kernel, dim3(unsigned((nloc + 255) / 256)), dim3(256), 0, s, part, ldp, cnt, f,
                       nloc);
    SVMD_LAUNCH_CHECK();
  }
  SVMD_CHECK(hipMemcpyAsync(f_out, f, size_t(nloc) * 8, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  if (used_out) *used_out = 1;
  return ctx->end();
}

// One Newton polish step (decomp_newton.h) on the device for a host working set (tests / timing): Kw_h
// (m x m), y_h, a_h / f_h by position (overwritten with the result); *code = 0 / 1 / 2; prof (optional, 8
// int64): wall-clock stamps of the phases (free set, K_FF, factorisation, back substitution, step, f) of
// the last of `reps` runs (each from the same inputs), ticks at 100 MHz; ms_out: the mean time per step.
SVM_API int svmd_decomp_newton_probe(void* h, const double* Kw_h, const int32_t* y_h, int32_t m, double* a_h,
                                     double* f_h, double C, double eps, int32_t max_free, int32_t reps, int32_t* code,
                                     int64_t* prof_h, double* ms_out) {
  SVMD_CTX(h);
  if (!Kw_h || !y_h || !a_h || !f_h || !code || m < 1 || m > kMaxWS || reps < 1) {
    set_error("svmd_decomp_newton_probe: bad arguments (1 <= m <= %d)", kMaxWS);
    return SVM_ERR_ARG;
  }
  int rc = ctx->begin();
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t o_k = 0, o_y = al(size_t(kMaxWS) * kMaxWS * 8), o_a = o_y + al(kMaxWS * 4), o_f = o_a + al(kMaxWS * 8),
               o_a0 = o_f + al(kMaxWS * 8), o_f0 = o_a0 + al(kMaxWS * 8), o_c = o_f0 + al(kMaxWS * 8), o_p = o_c + 256,
               o_A = o_p + 256, need = o_A + size_t(kMaxWS + 2) * kMaxWS * 8;
  if ((rc = ctx->ensure_ws(need))) return rc;
  char* ws = static_cast<char*>(ctx->ws);
  auto* Kw = reinterpret_cast<double*>(ws + o_k);
  auto* yd = reinterpret_cast<int32_t*>(ws + o_y);
  auto* ad = reinterpret_cast<double*>(ws + o_a);
  auto* fd = reinterpret_cast<double*>(ws + o_f);
  auto* a0 = reinterpret_cast<double*>(ws + o_a0);
  auto* f0 = reinterpret_cast<double*>(ws + o_f0);
  auto* cd = reinterpret_cast<int32_t*>(ws + o_c);
  auto* pd = reinterpret_cast<int64_t*>(ws + o_p);
  auto* Ad = reinterpret_cast<double*>(ws + o_A);
  SVMD_CHECK(hipMemcpy2DAsync(Kw, kMaxWS * 8, Kw_h, size_t(m) * 8, size_t(m) * 8, size_t(m), hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(yd, y_h, size_t(m) * 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(a0, a_h, size_t(m) * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(f0, f_h, size_t(m) * 8, hipMemcpyHostToDevice, s));
  hipEvent_t e0, e1;
  SVMD_CHECK(hipEventCreate(&e0));
  SVMD_CHECK(hipEventCreate(&e1));
  float tot = 0.0f;
  for (int r = 0; r < reps; ++r) {
    SVMD_CHECK(hipMemcpyAsync(ad, a0, size_t(m) * 8, hipMemcpyDeviceToDevice, s));
    SVMD_CHECK(hipMemcpyAsync(fd, f0, size_t(m) * 8, hipMemcpyDeviceToDevice, s));
    SVMD_CHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(ws_newton_probe_kernel, dim3(1), dim3(256), 0, s, m, Kw, int64_t(kMaxWS), yd, ad, fd, Ad, C, eps,
                       max_free, cd, pd);
    SVMD_LAUNCH_CHECK();
    SVMD_CHECK(hipEventRecord(e1, s));
    SVMD_CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    SVMD_CHECK(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  SVMD_CHECK(hipMemcpyAsync(a_h, ad, size_t(m) * 8, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipMemcpyAsync(f_h, fd, size_t(m) * 8, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipMemcpyAsync(code, cd, 4, hipMemcpyDeviceToHost, s));
  if (prof_h) SVMD_CHECK(hipMemcpyAsync(prof_h, pd, 16 * 8, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  if (ms_out) *ms_out = double(tot) / reps;
  return ctx->end();
}

}  // extern "C"

SVMD_TU_WARM(decomp)
