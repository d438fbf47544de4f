// L3 device-resident SMO (gfx950).
//
// Reference host loop (gpu_svm_main3.cu:318-483) runs per iteration: 2 masking kernels, 2-4
// strided-tree argmin/argmax launches, 0-2 kernel-row launches + cudaDeviceSynchronize, 1 f-update
// kernel and 11 blocking scalar cudaMemcpy round trips.  Here one SMO iteration is exactly two
// kernels and no host involvement:
//
//   smo_select_kernel  (grid over n)  f += ch*K[ih,:] + cl*K[il,:] for the previous update, fused
//                      with the masked argmin over I_high / argmax over I_low of the new f
//                      (wave64 butterfly + LDS, packed (value,index) with lowest-index ties =
//                      the serial semantics; the reference GPU's bit-reversed tie preference is
//                      deliberately not replicated).
//   smo_step_kernel    (one workgroup) final reduction of the block partials, stop tests, clip
//                      bounds U/V, eta, the two-variable alpha update and the f-update
//                      coefficients, all in a device-side state block.
//
// The pair is captured CHUNK times into a hipGraph and replayed; the host only polls a pinned
// stop flag once per replay (two replays in flight).  Kernel rows come from the resident RBF Gram
// (gram_mfma.hip), so K11/K22/K12 are plain loads.  Arithmetic replicates main3.cpp:235-275
// operation by operation (built with -ffp-contract=off), so on an identical kernel matrix the
// trajectory is bit-identical to the CPU oracle.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ctx.h"
#include "qrows.h"

namespace svm355 {
namespace {

constexpr int kSelectThreads = 256;
constexpr int kChunk = 128;  // SMO iterations per graph replay

struct SmoState {
  int64_t ih, il;       // pair updated by the last step (consumed by the next select)
  double ch, cl;        // f-update coefficients (alpha_new - alpha) * y for ih / il
  double b_high, b_low;
  int64_t num_iter;     // reference counter (starts at 1)
  int32_t pending;      // 1 -> (ih, il, ch, cl) not yet applied to f
  int32_t stop;         // enum svm_stop
};

struct Partial {
  double vmin;
  int64_t imin;
  double vmax;
  int64_t imax;
};

constexpr int64_t kNoIdx = INT64_MAX;

__global__ __launch_bounds__(kSelectThreads) void smo_select_kernel(
    const double* __restrict__ K, int64_t ldk, const int32_t* __restrict__ y,
    const double* __restrict__ alpha, double* __restrict__ f, int64_t n,
    const SmoState* __restrict__ st, Partial* __restrict__ part, double C, double eps) {
  if (st->stop) return;
  const int32_t pending = st->pending;
  const double ch = st->ch, cl = st->cl;
  const double* Kh = K + st->ih * ldk;
  const double* Kl = K + st->il * ldk;
  const double c_hi = C - eps, c_lo = 0.0 + eps;

  double hv = __builtin_inf(), lv = -__builtin_inf();
  int64_t hi = kNoIdx, li = kNoIdx;
  const int64_t stride = int64_t(gridDim.x) * kSelectThreads;
  for (int64_t i = int64_t(blockIdx.x) * kSelectThreads + threadIdx.x; i < n; i += stride) {
    double fi = f[i];
    if (pending) {
      fi += ch * Kh[i] + cl * Kl[i];  // main3.cpp:274 operation order
      f[i] = fi;
    }
    const double a = alpha[i];
    const int32_t yi = y[i];
    const bool in_high = (yi == 1 && a < c_hi) || (yi == -1 && a > c_lo);
    const bool in_low = (yi == 1 && a > c_lo) || (yi == -1 && a < c_hi);
    if (in_high && fi < hv) {
      hv = fi;
      hi = i;
    }
    if (in_low && fi > lv) {
      lv = fi;
      li = i;
    }
  }
  wave_argmin(hv, hi);
  wave_argmax(lv, li);
  __shared__ Partial sp[kSelectThreads / kWave];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sp[w] = Partial{hv, hi, lv, li};
  __syncthreads();
  if (threadIdx.x == 0) {
    Partial r = sp[0];
#pragma unroll
    for (int k = 1; k < kSelectThreads / kWave; ++k) {
      if (better_min(r.vmin, r.imin, sp[k].vmin, sp[k].imin)) {
        r.vmin = sp[k].vmin;
        r.imin = sp[k].imin;
      }
      if (better_max(r.vmax, r.imax, sp[k].vmax, sp[k].imax)) {
        r.vmax = sp[k].vmax;
        r.imax = sp[k].imax;
      }
    }
    part[blockIdx.x] = r;
  }
}

__global__ __launch_bounds__(256) void smo_step_kernel(
    const Partial* __restrict__ part, int nparts, const double* __restrict__ K, int64_t ldk,
    const int32_t* __restrict__ y, double* __restrict__ alpha, int64_t n, SmoState* __restrict__ st,
    double C, double eps, double tau, int64_t max_iter, int64_t* __restrict__ trace, int64_t trace_cap) {
  if (st->stop) return;
  double hv = __builtin_inf(), lv = -__builtin_inf();
  int64_t hi = kNoIdx, li = kNoIdx;
  for (int k = threadIdx.x; k < nparts; k += blockDim.x) {
    const Partial p = part[k];
    if (better_min(hv, hi, p.vmin, p.imin)) {
      hv = p.vmin;
      hi = p.imin;
    }
    if (better_max(lv, li, p.vmax, p.imax)) {
      lv = p.vmax;
      li = p.imax;
    }
  }
  wave_argmin(hv, hi);
  wave_argmax(lv, li);
  __shared__ Partial sp[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sp[w] = Partial{hv, hi, lv, li};
  __syncthreads();
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    if (better_min(hv, hi, sp[k].vmin, sp[k].imin)) {
      hv = sp[k].vmin;
      hi = sp[k].imin;
    }
    if (better_max(lv, li, sp[k].vmax, sp[k].imax)) {
      lv = sp[k].vmax;
      li = sp[k].imax;
    }
  }
  if (hi >= n || li >= n) {  // main3.cpp:205-209 (b_high/b_low keep their previous values)
    st->pending = 0;
    st->stop = SVM_STOP_NO_CANDIDATE;
    return;
  }
  const double bh = hv, bl = lv;  // == f[i_high], f[i_low]
  st->b_high = bh;
  st->b_low = bl;
  if (bl <= bh + 2.0 * tau) {
    st->pending = 0;
    st->stop = SVM_STOP_CONVERGED;
    return;
  }
  // All scalar operands issued together: one memory round trip.
  const int32_t yh = y[hi], yl = y[li];
  const double K11 = K[hi * ldk + hi], K22 = K[li * ldk + li], K12 = K[hi * ldk + li];
  const double ah = alpha[hi], al = alpha[li];
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
    st->pending = 0;
    st->stop = SVM_STOP_INFEASIBLE;
    return;
  }
  if (eta <= eps) {
    st->pending = 0;
    st->stop = SVM_STOP_NONPOS_ETA;
    return;
  }
  double al_new = al + double(yl) * (bh - bl) / eta;
  if (al_new > V) al_new = V;
  if (al_new < U) al_new = U;
  const double ah_new = ah + double(s) * (al - al_new);
  st->ch = (ah_new - ah) * double(yh);
  st->cl = (al_new - al) * double(yl);
  st->ih = hi;
  st->il = li;
  st->pending = 1;
  alpha[hi] = ah_new;
  alpha[li] = al_new;
  const int64_t it = st->num_iter;
  if (trace && it - 1 < trace_cap) {
    trace[2 * (it - 1)] = hi;
    trace[2 * (it - 1) + 1] = li;
  }
  st->num_iter = it + 1;
  if (it + 1 > max_iter) st->stop = SVM_STOP_MAX_ITER;
}

// Cold start: alpha = 0, f = -y (main3.cpp:165-172 / init_alpha_f gpu_svm_main3.cu:152-161).
__global__ void smo_init_cold_kernel(const int32_t* __restrict__ y, double* __restrict__ alpha,
                                     double* __restrict__ f, int64_t n, SmoState* st) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) {
    alpha[i] = 0.0;
    f[i] = -static_cast<double>(y[i]);
  }
  if (i == 0) *st = SmoState{0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, SVM_STOP_RUNNING};
}

// Warm start, step 1: ascending list of j with alpha_j != 0 (single workgroup, ballot compaction),
// with coef_k = alpha_j * y_j next to it -- the first product of the reference's
// alpha_j * y_j * K(j, i), so step 2 computes the same bits.
__global__ __launch_bounds__(1024) void nonzero_compact_kernel(const double* __restrict__ alpha,
                                                               const int32_t* __restrict__ y, int64_t n,
                                                               int64_t* __restrict__ idx, double* __restrict__ coef,
                                                               int64_t* __restrict__ count, SmoState* st) {
  __shared__ int64_t wave_cnt[16];
  __shared__ int64_t base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += blockDim.x) {
    const int64_t i = c0 + threadIdx.x;
    const bool nz = i < n && alpha[i] != 0.0;
    const unsigned long long m = __ballot(nz);
    if (lane == 0) wave_cnt[w] = __popcll(m);
    __syncthreads();
    int64_t off = base;
    for (int k = 0; k < w; ++k) off += wave_cnt[k];
    if (nz) {
      const int64_t k = off + __popcll(m & ((1ull << lane) - 1ull));
      idx[k] = i;
      coef[k] = alpha[i] * double(y[i]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t tot = 0;
      for (int k = 0; k < nw; ++k) tot += wave_cnt[k];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *count = base;
    *st = SmoState{0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, SVM_STOP_RUNNING};
  }
}

// Warm start, step 2: f_i = sum_{j in nz, ascending} alpha_j y_j K[j][i] - y_i
// (mpi_svm_main3.cpp:169-186; column access K[j][i] is coalesced across i).  The sum stays serial in
// ascending j per point (the reference's order); the wave-uniform idx / coef loads are read kWarmU
// at a time and the kWarmU column loads issued before the adds consume them, so each group costs
// one memory round trip instead of a dependent chain per term.  64-thread blocks spread a
// cascade-sized n over many CUs.
constexpr int kWarmU = 8;
__global__ __launch_bounds__(64) void warm_f_kernel(const double* __restrict__ K, int64_t ldk,
                                                    const int32_t* __restrict__ y,
                                                    const int64_t* __restrict__ idx,
                                                    const double* __restrict__ coef,
                                                    const int64_t* __restrict__ count,
                                                    double* __restrict__ f, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t cnt = *count;
  const int64_t ic = i < n ? i : n - 1;  // tail lanes read a valid column, store nothing
  double sum = 0.0;
  int64_t k = 0;
  for (; k + kWarmU <= cnt; k += kWarmU) {
    double kv[kWarmU], c[kWarmU];
#pragma unroll
    for (int u = 0; u < kWarmU; ++u) {
      c[u] = coef[k + u];
      kv[u] = K[idx[k + u] * ldk + ic];
    }
#pragma unroll
    for (int u = 0; u < kWarmU; ++u) sum += c[u] * kv[u];
  }
  for (; k < cnt; ++k) sum += coef[k] * K[idx[k] * ldk + ic];
  if (i < n) f[i] = sum - static_cast<double>(y[i]);
}

// ------------------------------------------------------------------------------------------------
// Persistent SMO: the whole solve in ONE launch.
//
// G workgroups (G <= #CUs, all co-resident) each own a contiguous slice of the training points and
// keep f, alpha and y of that slice in registers for the entire solve.  One iteration:
//   1. local masked argmin over I_high / argmax over I_low of the slice (wave64 butterfly + LDS),
//      carrying alpha of the winners;
//   2. publish the workgroup's two candidates as ten 8-byte {epoch, 32-bit payload} granules with
//      agent-scope relaxed (sc1) stores — a granule is written by one store and needs no fence;
//   3. wave 0 of EVERY workgroup sweeps all G candidate records (relaxed agent loads, s_sleep
//      between polls) until every tag equals the epoch, and reduces them with the lowest-index
//      rule: every workgroup obtains the identical (i_high, i_low, b_high, b_low, alpha_h, alpha_l);
//   4. every workgroup evaluates the stop tests and the two-variable update redundantly (same
//      inputs, same instruction sequence -> same bits), issuing the K11/K22/K12 and y loads in the
//      same memory round trip as its slice of rows K[i_high,:] and K[i_low,:];
//   5. the owners of i_high / i_low update their register alpha; every slice applies the f update.
// Records are double-buffered by epoch parity (a workgroup can be at most one epoch ahead of the
// slowest reader).  Every spin is bounded; a timeout sets *err and all workgroups drain.
// Per iteration this costs one HBM round trip plus one all-to-all granule exchange, instead of two
// kernel boundaries and a single-workgroup tail (smo_select_kernel + smo_step_kernel).
constexpr int kGranules = 10;    // per candidate record
constexpr int kRecStride = 16;   // granules per record slot (128 B)
constexpr int kMaxG = 64;        // one sweep pass: lane L of wave 0 reads workgroup L's record
constexpr uint32_t kSentinel = 0x7FFFFFFFu;  // "no candidate" index (n < 2^31)

__device__ __forceinline__ uint32_t lo32(double x) { return uint32_t(__double_as_longlong(x)); }
__device__ __forceinline__ uint32_t hi32(double x) { return uint32_t(uint64_t(__double_as_longlong(x)) >> 32); }
__device__ __forceinline__ double mk64(uint32_t lo, uint32_t hi) {
  return __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
}

// ---- wave64 arg-reductions on (double value, uint32 index) without LDS traffic, with the serial
// tie rule (smallest value -- largest for MAX -- then the lowest index): the result is identical in
// every lane and independent of the schedule.  Values are compared through an order-preserving
// 64-bit key (sign-folded bits, -0 folded onto +0).  Its HIGH word is reduced with one DPP move and
// one v_min/max_u32 per step (quad_perm xor1, xor2, row_half_mirror (8), row_mirror (16), then the
// gfx950 v_permlane16_swap / v_permlane32_swap for the 32/64-lane halves); a ballot then finds the
// lanes holding the winning high word -- almost always exactly one, whose value, index and lane are
// read directly.  Only a tie of the high words costs a second 32-bit pass over the low words, and
// only an exact value tie a third pass for the lowest index.  (Replaces a 64-bit value pass plus an
// index pass on every reduction: about half the DPP steps.)
struct VI {
  double v;
  uint32_t i;
};
struct VIL {  // winner: value, index and the lane that holds it (read its other fields with readlane)
  double v;
  uint32_t i;
  int lane;
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ uint64_t order_key(double v) {
  const uint64_t u = uint64_t(__double_as_longlong(v == 0.0 ? 0.0 : v));
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
template <bool MIN>
__device__ __forceinline__ uint32_t pick32(uint32_t a, uint32_t b) {
  return MIN ? min(a, b) : max(a, b);
}
// v_permlane{16,32}_swap with both operands = x returns, in every lane, its own value and its
// partner's (in an order that depends on the row): combine both.
template <bool MIN, bool S32>
__device__ __forceinline__ uint32_t swap_pick32(uint32_t x) {
  if constexpr (S32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return pick32<MIN>(r[0], r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return pick32<MIN>(r[0], r[1]);
  }
}
// Butterfly over aligned groups of L lanes (L = 1..64, power of two); returns lane 0's group result
// (wave-uniform).
template <bool MIN, int L>
__device__ __forceinline__ uint32_t group_pick32(uint32_t x) {
  if (L > 1) x = pick32<MIN>(x, dpp32<0xB1>(x));   // quad_perm [1,0,3,2]
  if (L > 2) x = pick32<MIN>(x, dpp32<0x4E>(x));   // quad_perm [2,3,0,1]
  if (L > 4) x = pick32<MIN>(x, dpp32<0x141>(x));  // row_half_mirror
  if (L > 8) x = pick32<MIN>(x, dpp32<0x140>(x));  // row_mirror
  if (L > 16) x = swap_pick32<MIN, false>(x);
  if (L > 32) x = swap_pick32<MIN, true>(x);
  return uint32_t(__builtin_amdgcn_readfirstlane(int(x)));
}
__device__ __forceinline__ double read_lane64(double x, int src) {
  return mk64(uint32_t(__builtin_amdgcn_readlane(int(lo32(x)), src)),
              uint32_t(__builtin_amdgcn_readlane(int(hi32(x)), src)));
}
// Inclusive prefix sum over the 64 lanes (lane L gets x[0] + ... + x[L]); full wave.  DPP only:
// Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8; lanes shifted in from outside the row
// read 0), then row_bcast:15 adds row 0's total to row 1 and row 2's to row 3, and row_bcast:31
// adds lane 31's (rows 0-1 total) to rows 2 and 3.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int32_t dpp_add_src(int32_t x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x) {
  x += dpp_add_src<0x111>(x);  // row_shr:1
  x += dpp_add_src<0x112>(x);  // row_shr:2
  x += dpp_add_src<0x114>(x);  // row_shr:4
  x += dpp_add_src<0x118>(x);  // row_shr:8
  x += dpp_add_src<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp_add_src<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
// a strictly before b in wave_arg's order: the value key (smallest for MIN, largest for MAX), then
// the lowest index.  A lane merging several candidates with it holds the one wave_arg would pick.
template <bool MIN>
__device__ __forceinline__ bool beats(VI a, VI b) {
  const uint64_t ka = order_key(a.v), kb = order_key(b.v);
  if (ka != kb) return MIN ? ka < kb : ka > kb;
  return a.i < b.i;
}
// Requires a full wave (EXEC = all 64 lanes).  L = number of leading lanes that may hold candidates;
// lanes >= L must hold "no candidate" sentinels (value +inf for MIN / -inf for MAX, index
// kSentinel), which never beat a real candidate.
template <bool MIN, int L = 64>
__device__ __forceinline__ VIL wave_arg(VI a) {
  const uint64_t k = order_key(a.v);
  const uint32_t kh = uint32_t(k >> 32), kl = uint32_t(k);
  const uint32_t bh = group_pick32<MIN, L>(kh);
  unsigned long long tie = __ballot(kh == bh);
  if (__popcll(tie) != 1) {  // equal high words: compare the low words
    const uint32_t bl = group_pick32<MIN, L>(kh == bh ? kl : (MIN ? 0xFFFFFFFFu : 0u));
    const bool same = kh == bh && kl == bl;
    tie = __ballot(same);
    if (__popcll(tie) != 1) {  // exact value tie (e.g. the first iteration, f = -y): lowest index
      const uint32_t bi = group_pick32<true, L>(same ? a.i : 0xFFFFFFFFu);
      tie = __ballot(same && a.i == bi);
    }
  }
  const int src = __builtin_ctzll(tie);
  return VIL{read_lane64(a.v, src), uint32_t(__builtin_amdgcn_readlane(int(a.i), src)), src};
}

struct PersistShared {
  double wv[2][16], wa[2][16];  // per-wave candidates [min|max][wave]
  uint32_t wi[2][16];
  double gv[2], ga[2];          // global winners of the current epoch
  uint32_t gi[2];
  int timeout;
  int64_t rslot[2];             // cached row source: slots of rows (i_high, i_low) ...
  int32_t rmiss[2];             // ... and whether this epoch fills them
  double k12;                   // second-order selection: K(i_high, j) from the winner's record
};

// ---- Row sources of the persistent solver.  choose() runs on one lane of every workgroup once the
// pair is known (before the barrier that publishes it); fetch() then gives every thread the rows'
// values for its elements plus K11 / K22 / K12, issuing all loads in one memory round trip.
// Second-order selection reads the pair's rows one at a time (row i_high before the second exchange,
// row j after it): choose_one() (lane 0 of wave 0, `keep` = a slot that must survive) and fetch_one()
// (every thread: its elements of the row, and K(row, row)).
struct ResidentRows {  // the resident n x n Gram
  const double* __restrict__ K;
  int64_t ldk;
  __device__ __forceinline__ void choose(PersistShared&, uint32_t, uint32_t) const {}
  __device__ __forceinline__ void choose_one(PersistShared&, int, uint32_t, int64_t) const {}
  template <int NT, int E>
  __device__ __forceinline__ void fetch_one(const PersistShared&, int, int64_t row, int64_t lo, int t,
                                            int64_t hi_end, double (&k)[E], double& diag) const {
    const double* R = K + row * ldk;
    diag = R[row];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      k[e] = i < hi_end ? R[i] : 0.0;
    }
  }
  template <int NT, int E>
  __device__ __forceinline__ void fetch(const PersistShared&, int64_t ih, int64_t il, int64_t lo, int t,
                                        int64_t hi_end, double (&kh)[E], double (&kl)[E], double& K11,
                                        double& K22, double& K12) const {
    K11 = K[ih * ldk + ih];
    K22 = K[il * ldk + il];
    K12 = K[ih * ldk + il];
    const double* Kh = K + ih * ldk;
    const double* Kl = K + il * ldk;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      const bool ok = i < hi_end;
      kh[e] = ok ? Kh[i] : 0.0;
      kl[e] = ok ? Kl[i] : 0.0;
    }
  }
};

// Kernel rows held in an HBM row cache of nslots x ldc doubles, computed from the rows themselves
// on a miss (qrows.h).  The 2-way set-associative directory (int32 tags + MRU way per set) lives
// in LDS and is REPLICATED in every workgroup: all workgroups see the same pair sequence and run the
// same deterministic lookups, so they agree on every slot and miss without exchanging anything.  On
// a miss each workgroup computes its own slice of the row (kval2: both rows of the pair in one pass
// over each element's quantised row) and writes it into the slot; hits read the slot, exactly like
// the resident Gram.  Values are bit-identical to the exact-integer Gram, hence the trajectory.
template <bool INT>
struct CachedRows {
  QRows q;
  double* __restrict__ cache;
  int64_t ldc;
  int32_t* tags;    // LDS, nslots entries (-1 = empty)
  uint8_t* mru;     // LDS, nslots / 2 entries
  int64_t nsets;
  double neg_gamma;

  __device__ __forceinline__ int64_t lookup(int64_t row, int64_t keep, int32_t* miss) const {
    const int64_t set = uint32_t(row) % uint32_t(nsets), s0 = 2 * set;  // row < 2^31, nsets <= 8192
    const int2 tw = reinterpret_cast<const int2*>(tags)[set];           // both ways in one LDS read
    if (tw.x == int32_t(row)) {
      mru[set] = 0;
      *miss = 0;
      return s0;
    }
    if (tw.y == int32_t(row)) {
      mru[set] = 1;
      *miss = 0;
      return s0 + 1;
    }
    int way = 1 - int(mru[set]);
    if (s0 + way == keep) way = 1 - way;
    tags[s0 + way] = int32_t(row);
    mru[set] = uint8_t(way);
    *miss = 1;
    return s0 + way;
  }
  __device__ __forceinline__ void choose_one(PersistShared& sh, int which, uint32_t row, int64_t keep) const {
    int32_t m = 0;
    sh.rslot[which] = lookup(row, keep, &m);
    sh.rmiss[which] = m;
  }
  template <int NT, int E>
  __device__ __forceinline__ void fetch_one(const PersistShared& sh, int which, int64_t row, int64_t lo, int t,
                                            int64_t hi_end, double (&k)[E], double& diag) const {
    diag = 1.0;  // kval(a, a)
    double* Cr = cache + sh.rslot[which] * ldc;
    if (sh.rmiss[which]) {
      if constexpr (INT) {
        constexpr int EG = E < 4 ? E : 4;
#pragma unroll 1
        for (int e0 = 0; e0 < E; e0 += EG) fill<NT, EG, true, false>(lo + int64_t(NT) * e0, row, row, t, hi_end, Cr, Cr);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int64_t i = lo + t + NT * e;
          if (i < hi_end) Cr[i] = kval<false>(q, row, i, neg_gamma);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {  // this thread's own stores, or a filled slot from an earlier epoch
      const int64_t i = lo + t + NT * e;
      k[e] = i < hi_end ? Cr[i] : 0.0;
    }
  }
  __device__ __forceinline__ void choose(PersistShared& sh, uint32_t ih, uint32_t il) const {
    int32_t mh = 0, ml = 0;
    const int64_t sh_ = lookup(ih, -1, &mh);
    const int64_t sl_ = lookup(il, sh_, &ml);
    sh.rslot[0] = sh_;
    sh.rslot[1] = sl_;
    sh.rmiss[0] = mh;
    sh.rmiss[1] = ml;
  }
  // K(ih, il) of the exact-integer path, computed redundantly by every wave: lane s takes k-step s
  // (and s + 64), then the steps are combined in order with the igram group flushes -> kval bits.
  // mid() runs after K12's own loads are issued and before their data is used: loads it issues
  // (the hit path's row reads) stay in flight through K12's arithmetic, since the in-order vmcnt
  // wait for K12's operands does not cover loads issued after them.
  template <class Mid>
  __device__ __forceinline__ double k12(int64_t ih, int64_t il, Mid mid) const {
    if constexpr (INT) {
      const int lane = threadIdx.x & 63, nsteps = q.kq / 32;
      int32_t d[2] = {0, 0};
      double wl[2] = {0.0, 0.0};  // step s's flush weight in lane s & 63 (no loads in the serial loop)
      int4 a0[2], a1[2], b0[2], b1[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int s = lane + 64 * r;
        if (s < q.main_step0) wl[r] = q.step_w[s];
        a0[r] = a1[r] = b0[r] = b1[r] = int4{0, 0, 0, 0};
        if (s < nsteps) {
          const int4* pa = reinterpret_cast<const int4*>(q.Q + ih * int64_t(q.kq)) + 2 * s;
          const int4* pb = reinterpret_cast<const int4*>(q.Q + il * int64_t(q.kq)) + 2 * s;
          a0[r] = pa[0];
          a1[r] = pa[1];
          b0[r] = pb[0];
          b1[r] = pb[1];
        }
      }
      const int32_t n0h = q.N0[ih], n0l = q.N0[il];
      const double wnh = q.main_step0 > 0 ? q.WN[ih] : 0.0, wnl = q.main_step0 > 0 ? q.WN[il] : 0.0;
      mid();
#pragma unroll
      for (int r = 0; r < 2; ++r) {  // zero operands past nsteps give d = 0
        int32_t acc = 0;
        acc = __builtin_amdgcn_sdot4(a0[r].x, b0[r].x, acc, false);
        acc = __builtin_amdgcn_sdot4(a0[r].y, b0[r].y, acc, false);
        acc = __builtin_amdgcn_sdot4(a0[r].z, b0[r].z, acc, false);
        acc = __builtin_amdgcn_sdot4(a0[r].w, b0[r].w, acc, false);
        acc = __builtin_amdgcn_sdot4(a1[r].x, b1[r].x, acc, false);
        acc = __builtin_amdgcn_sdot4(a1[r].y, b1[r].y, acc, false);
        acc = __builtin_amdgcn_sdot4(a1[r].z, b1[r].z, acc, false);
        acc = __builtin_amdgcn_sdot4(a1[r].w, b1[r].w, acc, false);
        d[r] = acc;
      }
      // kval's serial walk is "acc += d[s]; at a flush step: x += w * acc, acc = 0".  The integer
      // group sums are exact, so they come from an inclusive prefix scan over the steps (group sum
      // = P[flush] - P[previous flush]); only the FP64 accumulation stays serial, over the flush
      // steps alone and in step order -- the same operands in the same order as kval.
      const int32_t P0 = wave_incl_scan(d[0]);
      const int32_t P1 = nsteps > 64 ? wave_incl_scan(d[1]) + __builtin_amdgcn_readlane(P0, 63) : 0;
      uint64_t m0 = __ballot(lane < q.main_step0 && wl[0] != 0.0);
      uint64_t m1 = __ballot(lane + 64 < q.main_step0 && wl[1] != 0.0);
      int32_t prev = 0;
      double x = 0.0;
      while (m0) {
        const int s = __builtin_ctzll(m0);
        m0 &= m0 - 1;
        const int32_t ps = __builtin_amdgcn_readlane(P0, s);
        x += read_lane64(wl[0], s) * double(ps - prev);
        prev = ps;
      }
      while (m1) {
        const int s = __builtin_ctzll(m1);
        m1 &= m1 - 1;
        const int32_t ps = __builtin_amdgcn_readlane(P1, s);
        x += read_lane64(wl[1], s) * double(ps - prev);
        prev = ps;
      }
      const int32_t acc = __builtin_amdgcn_readlane(nsteps > 64 ? P1 : P0, 63) - prev;
      const int32_t D0 = n0h + n0l - 2 * acc;
      double dist = q.w0 * double(D0);
      if (q.main_step0 > 0) dist += (wnh + wnl) - 2.0 * x;
      dist = dist > 0.0 ? dist : 0.0;
      return exp(neg_gamma * dist);
    } else {
      mid();
      return kval<false>(q, ih, il, neg_gamma);
    }
  }
  template <int NT, int E>
  __device__ __forceinline__ void fetch(const PersistShared& sh, int64_t ih, int64_t il, int64_t lo, int t,
                                        int64_t hi_end, double (&kh)[E], double (&kl)[E], double& K11,
                                        double& K22, double& K12) const {
    const int32_t mh = sh.rmiss[0], ml = sh.rmiss[1];
    double* Ch = cache + sh.rslot[0] * ldc;
    double* Cl = cache + sh.rslot[1] * ldc;
    K11 = 1.0;  // kval(a, a): the Gram's diagonal is exactly 1
    K22 = 1.0;
    if constexpr (INT) {
      if (!(mh | ml)) {  // hit: the row reads overlap K12's arithmetic
        K12 = k12(ih, il, [&] {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int64_t i = lo + t + NT * e;
            const bool ok = i < hi_end;
            kh[e] = ok ? Ch[i] : 0.0;
            kl[e] = ok ? Cl[i] : 0.0;
          }
        });
        return;
      }
      K12 = k12(ih, il, [] {});
      // A miss first writes this thread's elements of the missed row(s) into the slot, in groups of
      // EG elements with the group loop kept rolled, so the fill's registers do not stack on the
      // E-element solver state; then every element is read back from the slot like a hit (a
      // thread reading its own stores).
      constexpr int EG = E < 4 ? E : 4;
#pragma unroll 1
      for (int e0 = 0; e0 < E; e0 += EG) {
        if (mh && ml)
          fill<NT, EG, true, true>(lo + int64_t(NT) * e0, ih, il, t, hi_end, Ch, Cl);
        else if (mh)
          fill<NT, EG, true, false>(lo + int64_t(NT) * e0, ih, il, t, hi_end, Ch, Cl);
        else
          fill<NT, EG, false, true>(lo + int64_t(NT) * e0, ih, il, t, hi_end, Ch, Cl);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t i = lo + t + NT * e;
        const bool ok = i < hi_end;
        kh[e] = ok ? Ch[i] : 0.0;
        kl[e] = ok ? Cl[i] : 0.0;
      }
      return;
    }
    K12 = k12(ih, il, [] {});
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      const bool ok = i < hi_end;
      kh[e] = (ok && !mh) ? Ch[i] : 0.0;
      kl[e] = (ok && !ml) ? Cl[i] : 0.0;
    }
    if (mh | ml) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t i = lo + t + NT * e;
        if (i < hi_end) {
          double a, b;
          kval2<INT>(q, ih, il, i, neg_gamma, &a, &b);
          if (mh) {
            kh[e] = a;
            Ch[i] = a;
          }
          if (ml) {
            kl[e] = b;
            Cl[i] = b;
          }
        }
      }
    }
  }
  // Miss fill of the exact-integer rows for this thread's E elements: the k-step loop is outermost,
  // so every step issues the loads of all E elements' chunks at once (E-fold memory parallelism
  // against the one-element-at-a-time walk of kval2) -- per element the arithmetic and its order
  // are kval's, so the values are bit-identical.  DA / DB: rows ih / il missed.  Elements
  // lo + t + NT * e, e < EG.
  template <int NT, int EG, bool DA, bool DB>
  __device__ __forceinline__ void fill(int64_t lo, int64_t ih, int64_t il, int t, int64_t hi_end, double* Ch,
                                       double* Cl) const {
    const int4* pa = reinterpret_cast<const int4*>(q.Q + ih * int64_t(q.kq));
    const int4* pb = reinterpret_cast<const int4*>(q.Q + il * int64_t(q.kq));
    const int4* pq = q.Qt ? reinterpret_cast<const int4*>(q.Qt) : nullptr;
    const int64_t cs = q.Qt ? q.n_rows : 1;  // chunk stride (interleaved) or 1 (row-major rows)
    int32_t acca[EG], accb[EG];
    double xa[EG], xb[EG];
    const int4* pi[EG];
#pragma unroll
    for (int e = 0; e < EG; ++e) {
      const int64_t i = lo + t + NT * e;
      const int64_t ic = i < hi_end ? i : lo;  // clamped (valid) row for the tail's dummy loads
      pi[e] = pq ? pq + ic : reinterpret_cast<const int4*>(q.Q + ic * int64_t(q.kq));
      acca[e] = accb[e] = 0;
      xa[e] = xb[e] = 0.0;
    }
    const int nsteps = q.kq / 32;
    int4 c0[EG], c1[EG];
    for (int s = 0; s < nsteps; ++s) {
#pragma unroll
      for (int e = 0; e < EG; ++e) {
        c0[e] = pi[e][(2 * s) * cs];
        c1[e] = pi[e][(2 * s + 1) * cs];
      }
      int4 a0, a1, b0, b1;
      if (DA) {
        a0 = pa[2 * s];
        a1 = pa[2 * s + 1];
      }
      if (DB) {
        b0 = pb[2 * s];
        b1 = pb[2 * s + 1];
      }
#pragma unroll
      for (int e = 0; e < EG; ++e) {
        if (DA) {
          int32_t acc = acca[e];
          acc = __builtin_amdgcn_sdot4(a0.x, c0[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(a0.y, c0[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(a0.z, c0[e].z, acc, false);
          acc = __builtin_amdgcn_sdot4(a0.w, c0[e].w, acc, false);
          acc = __builtin_amdgcn_sdot4(a1.x, c1[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(a1.y, c1[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(a1.z, c1[e].z, acc, false);
          acca[e] = __builtin_amdgcn_sdot4(a1.w, c1[e].w, acc, false);
        }
        if (DB) {
          int32_t acc = accb[e];
          acc = __builtin_amdgcn_sdot4(b0.x, c0[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(b0.y, c0[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(b0.z, c0[e].z, acc, false);
          acc = __builtin_amdgcn_sdot4(b0.w, c0[e].w, acc, false);
          acc = __builtin_amdgcn_sdot4(b1.x, c1[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(b1.y, c1[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(b1.z, c1[e].z, acc, false);
          accb[e] = __builtin_amdgcn_sdot4(b1.w, c1[e].w, acc, false);
        }
      }
      if (s < q.main_step0) {
        const double wg = q.step_w[s];
        if (wg != 0.0) {  // igram_tri_kernel's group flush, same order and expression
#pragma unroll
          for (int e = 0; e < EG; ++e) {
            if (DA) {
              xa[e] += wg * double(acca[e]);
              acca[e] = 0;
            }
            if (DB) {
              xb[e] += wg * double(accb[e]);
              accb[e] = 0;
            }
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EG; ++e) {
      const int64_t i = lo + t + NT * e;
      if (i >= hi_end) continue;
      if (DA) {
        double dist = q.w0 * double(q.N0[ih] + q.N0[i] - 2 * acca[e]);
        if (q.main_step0 > 0) dist += (q.WN[ih] + q.WN[i]) - 2.0 * xa[e];
        dist = dist > 0.0 ? dist : 0.0;
        Ch[i] = ih == i ? 1.0 : exp(neg_gamma * dist);
      }
      if (DB) {
        double dist = q.w0 * double(q.N0[il] + q.N0[i] - 2 * accb[e]);
        if (q.main_step0 > 0) dist += (q.WN[il] + q.WN[i]) - 2.0 * xb[e];
        dist = dist > 0.0 ? dist : 0.0;
        Cl[i] = il == i ? 1.0 : exp(neg_gamma * dist);
      }
    }
  }
};

// Diagnostic build (STAMP = true, SVM355_PSMO_STAMP=1): workgroup 0 / lane 0 accumulates
// s_memtime deltas per phase over epochs [kStampFrom, kStampFrom + kStampCount) into stamps[0..7]
// (stamps[7] = s_memrealtime delta, 100 MHz, for the clock).  Never used in timed runs.
constexpr uint32_t kStampFrom = 200, kStampCount = 2000;
// Exchange-skew diagnostic (same STAMP builds): s_memrealtime (100 MHz, one clock for the whole chip)
// of every workgroup's record publication and of workgroup 0's sweep completion, for kSkewEpochs
// epochs from kStampFrom, at stamps[kSkewBase + g * kSkewEpochs + e] / [... + kMaxG * kSkewEpochs + e].
constexpr uint32_t kSkewEpochs = 64;
constexpr int kSkewBase = 16;
#define PSTAMP(k)                                                                   \
  do {                                                                              \
    if (STAMP && stamping) {                                                        \
      __builtin_amdgcn_sched_barrier(0);                                            \
      unsigned long long ts_;                                                       \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts_)::"memory");   \
      __builtin_amdgcn_sched_barrier(0);                                            \
      sacc[k] += ts_ - sprev;                                                       \
      sprev = ts_;                                                                  \
    }                                                                               \
  } while (0)

// XCD-local registration window (s_memrealtime ticks, 100 MHz): 2 ms, then the host falls back.
constexpr unsigned long long kRegisterTicks = 200000;

// One solve of the persistent SMO by G co-resident workgroups (this one is g), NT threads per
// workgroup (NW = NT/64 waves), E register-resident elements per thread: element e of thread t is
// training point lo + t + NT*e of the workgroup's slice.  Epochs continue from epoch0 (record tags
// must never repeat on a slot array); returns the last epoch used.  RPL = records per sweep lane:
// G <= 64 * RPL workgroups (lane L of wave 0 polls records L, L + 64, ...; slot arrays of 64 * RPL
// records per epoch parity).  The exchange-skew stamps exist for RPL = 1 only.
// WSS2 (opt-in, resident Gram, RPL = 1): second-order choice of the second index (smo_cpu.cpp):
// after the first exchange names i_high (and the first-order maximum for the stop test), every
// workgroup reads its slice of row i_high, computes -(f_t - f_ih)^2 / a_t over its I_low points
// above f_ih, and a second exchange (the next epoch) picks the minimum; its record carries the
// gain, j, alpha_j, f_j and K(i_high, j) (from the owner's row slice).
template <int NT, int E, bool STAMP, bool XLOCAL, class Rows, int RPL = 1, bool WSS2 = false>
__device__ __forceinline__ uint32_t persist_solve(
    PersistShared& sh, int G, int g, uint32_t epoch0, const Rows& rows,
    const int32_t* __restrict__ y, double* __restrict__ alpha, double* __restrict__ f, int64_t n, int64_t slice,
    unsigned long long* __restrict__ slots, SmoState* __restrict__ st, double C, double eps, double tau,
    int64_t max_iter, int64_t* __restrict__ trace, int64_t trace_cap, unsigned* __restrict__ err,
    int64_t spin_limit, unsigned long long* __restrict__ stamps) {
  constexpr int NW = NT / 64;
  unsigned long long sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sprev = 0, rt0 = 0;
  bool stamping = false;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t lo = int64_t(g) * slice, hi_end = std::min<int64_t>(n, lo + slice);
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  const double inf = __builtin_inf();

  double fr[E], ar[E];
  int32_t yr[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t i = lo + t + NT * e;
    const bool ok = i < hi_end;
    fr[e] = ok ? f[i] : 0.0;
    ar[e] = ok ? alpha[i] : 0.0;
    yr[e] = ok ? y[i] : 0;  // y = 0 is in neither set
  }
  if (t == 0) sh.timeout = 0;
  int64_t num_iter = st->num_iter;
  double b_high = st->b_high, b_low = st->b_low;
  int32_t stop = SVM_STOP_RUNNING;

  uint32_t epoch = epoch0 + 1;
  for (;; ++epoch) {
    if (STAMP) {
      // window start: stamps[8] when the host set it (SVM355_PSMO_STAMP_FROM), else kStampFrom
      const uint32_t from = stamps[8] ? uint32_t(stamps[8]) : kStampFrom;
      const bool on = g == 0 && threadIdx.x == 0 && epoch >= from && epoch < from + kStampCount;
      if (on && !stamping) rt0 = __builtin_amdgcn_s_memrealtime();
      if (!on && stamping) sacc[7] = __builtin_amdgcn_s_memrealtime() - rt0;
      stamping = on;
      if (stamping) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sprev)::"memory");
    }
    // ---- 1. local selection over the register slice (ascending index within a thread)
    VI mn{inf, kSentinel}, mx{-inf, kSentinel};
    double amn = 0.0, amx = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t i = uint32_t(lo + t + NT * e);
      const double a = ar[e], fi = fr[e];
      const int32_t yi = yr[e];
      const bool in_high = (yi == 1 && a < c_hi) || (yi == -1 && a > c_lo);
      const bool in_low = (yi == 1 && a > c_lo) || (yi == -1 && a < c_hi);
      if (in_high && fi < mn.v) {
        mn = VI{fi, i};
        amn = a;
      }
      if (in_low && fi > mx.v) {
        mx = VI{fi, i};
        amx = a;
      }
    }
    {
      const VIL wmn = wave_arg<true>(mn), wmx = wave_arg<false>(mx);
      const double awmn = read_lane64(amn, wmn.lane), awmx = read_lane64(amx, wmx.lane);
      PSTAMP(0);
      if (lane == 0) {
        sh.wv[0][w] = wmn.v;
        sh.wi[0][w] = wmn.i;
        sh.wa[0][w] = awmn;
        sh.wv[1][w] = wmx.v;
        sh.wi[1][w] = wmx.i;
        sh.wa[1][w] = awmx;
      }
    }
    __syncthreads();
    PSTAMP(1);
    unsigned long long* rec = slots + (size_t(epoch & 1) * (64 * RPL)) * kRecStride;
    if (w == 0) {
      // ---- 2. merge the NW waves and publish this workgroup's record (lanes 0..9, one granule each)
      VI a{inf, kSentinel}, b{-inf, kSentinel};
      double aa = 0.0, ba = 0.0;
      if (NW == 1) {
        a = VI{sh.wv[0][0], sh.wi[0][0]};
        b = VI{sh.wv[1][0], sh.wi[1][0]};
        aa = sh.wa[0][0];
        ba = sh.wa[1][0];
      } else {
        VI ca{inf, kSentinel}, cb{-inf, kSentinel};
        double caa = 0.0, cba = 0.0;
        if (lane < NW) {
          ca = VI{sh.wv[0][lane], sh.wi[0][lane]};
          cb = VI{sh.wv[1][lane], sh.wi[1][lane]};
          caa = sh.wa[0][lane];
          cba = sh.wa[1][lane];
        }
        // Lanes 0..NW-1 hold the wave results (sentinels above): log2(NW) steps; the winner is read
        // from its lane, so every publishing lane sees the same record.
        const VIL ra = wave_arg<true, NW>(ca), rb = wave_arg<false, NW>(cb);
        a = VI{ra.v, ra.i};
        b = VI{rb.v, rb.i};
        aa = read_lane64(caa, ra.lane);
        ba = read_lane64(cba, rb.lane);
      }
      if (lane < kGranules) {
        // Branch-free payload selection (no divergent switch).
        uint32_t pay = lo32(a.v);
        pay = lane == 1 ? hi32(a.v) : pay;
        pay = lane == 2 ? a.i : pay;
        pay = lane == 3 ? lo32(aa) : pay;
        pay = lane == 4 ? hi32(aa) : pay;
        pay = lane == 5 ? lo32(b.v) : pay;
        pay = lane == 6 ? hi32(b.v) : pay;
        pay = lane == 7 ? b.i : pay;
        pay = lane == 8 ? lo32(ba) : pay;
        pay = lane == 9 ? hi32(ba) : pay;
        // Memory-model note (XLOCAL).  The readers are other workgroups, but every participant runs
        // on XCD 0 (xcd_register checks HW_REG_XCC_ID), and HIP has no scope between workgroup and
        // agent.  On gfx950 the scopes differ only in the store's cache-coherence bits: workgroup
        // scope emits `global_store_dwordx2 ... sc0` (through the write-through vL1D into the
        // XCD's L2), agent scope `... sc1` (written through past the XCD-local L2 to the
        // device-coherent level, because the eight XCD L2s are not coherent with each other).  The
        // pollers' agent-scope loads (`global_load_dwordx2 ... sc1`) miss the vL1D and are served by
        // that same L2, the single point of coherence of one XCD, so the sc0 store is visible to
        // them.  Agent scope costs 16 % at the headline shape (3.42 -> 3.95 us/iter at n = 60k,
        // profiles/r2_psmo_store_scope_ab.txt); tests/test_isa_pins.py pins both encodings.
        if constexpr (XLOCAL)
          __hip_atomic_store(rec + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          __hip_atomic_store(rec + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      PSTAMP(2);
      if (STAMP && RPL == 1 && lane == 0 && epoch >= kStampFrom && epoch < kStampFrom + kSkewEpochs)
        stamps[kSkewBase + g * kSkewEpochs + (epoch - kStampFrom)] = __builtin_amdgcn_s_memrealtime();
      // ---- 3. lane L polls the records of workgroups L, L + 64, ... until their ten tags equal the
      // epoch (every spin round re-reads all of them: one round trip, not one per record), then
      // keeps the best of them under wave_arg's order (value key, then the lowest index)
      VI gm{inf, kSentinel}, gx{-inf, kSentinel};
      double agm = 0.0, agx = 0.0;
      bool timed_out = false;
      if (lane < G) {
        uint32_t v[RPL][kGranules];
        for (int64_t spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int rr = 0; rr < RPL; ++rr) {
            if (RPL == 1 || lane + 64 * rr < G) {
              const unsigned long long* r = rec + size_t(lane + 64 * rr) * kRecStride;
#pragma unroll
              for (int k = 0; k < kGranules; ++k) {
                const unsigned long long x = __hip_atomic_load(r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v[rr][k] = uint32_t(x);
                ok &= uint32_t(x >> 32) == epoch;
              }
            }
          }
          if (ok) break;
          if (spins > spin_limit) {
            timed_out = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (!timed_out) {
#pragma unroll
          for (int rr = 0; rr < RPL; ++rr) {
            if (RPL == 1 || lane + 64 * rr < G) {
              const VI cm{mk64(v[rr][0], v[rr][1]), v[rr][2]}, cx{mk64(v[rr][5], v[rr][6]), v[rr][7]};
              if (rr == 0 || beats<true>(cm, gm)) {
                gm = cm;
                agm = mk64(v[rr][3], v[rr][4]);
              }
              if (rr == 0 || beats<false>(cx, gx)) {
                gx = cx;
                agx = mk64(v[rr][8], v[rr][9]);
              }
            }
          }
        }
      }
      const bool any_to = __any(timed_out);
      if (STAMP && RPL == 1 && g == 0 && lane == 0 && epoch >= kStampFrom && epoch < kStampFrom + kSkewEpochs)
        stamps[kSkewBase + kMaxG * kSkewEpochs + (epoch - kStampFrom)] = __builtin_amdgcn_s_memrealtime();
      PSTAMP(3);
      const VIL wgm = wave_arg<true>(gm), wgx = wave_arg<false>(gx);
      const double awgm = read_lane64(agm, wgm.lane), awgx = read_lane64(agx, wgx.lane);
      if (lane == 0) {
        sh.gv[0] = wgm.v;
        sh.gi[0] = wgm.i;
        sh.ga[0] = awgm;
        sh.gv[1] = wgx.v;
        sh.gi[1] = wgx.i;
        sh.ga[1] = awgx;
        // a pair that will be updated: the row source prepares its rows (every workgroup alike;
        // second-order selection: row i_high now, the second row after the second exchange)
        if (!any_to && wgm.i != kSentinel && wgx.i != kSentinel && !(wgx.v <= wgm.v + 2.0 * tau)) {
          if constexpr (WSS2)
            rows.choose_one(sh, 0, wgm.i, -1);
          else
            rows.choose(sh, wgm.i, wgx.i);
        }
        if (any_to) {
          sh.timeout = 1;
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
    PSTAMP(4);
    if (sh.timeout) {
      stop = -1;
      break;
    }
    const uint32_t uih = sh.gi[0], uil = sh.gi[1];
    // ---- 4. stop tests and the two-variable update (identical in every workgroup)
    if (uih == kSentinel || uil == kSentinel) {
      stop = SVM_STOP_NO_CANDIDATE;
      break;
    }
    const int64_t ih = uih;
    int64_t il = uil;
    const double bh = sh.gv[0], bl = sh.gv[1];
    b_high = bh;
    b_low = bl;
    if (bl <= bh + 2.0 * tau) {
      stop = SVM_STOP_CONVERGED;
      break;
    }
    double K11, K22, K12;
    double kh[E], kl[E];
    int32_t yh, yl;
    double bl_upd = bl, al = sh.ga[1];  // the second index's f and alpha in the update
    if constexpr (WSS2) {
      // ---- 4b. row i_high, the local second-order candidate, a second exchange for j
      rows.template fetch_one<NT, E>(sh, 0, ih, lo, t, hi_end, kh, K11);
      VI cm{inf, kSentinel};
      double ca = 0.0, cf = 0.0, ck = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double a = ar[e], ft = fr[e];
        const int32_t yt = yr[e];
        const bool in_low = (yt == 1 && a > c_lo) || (yt == -1 && a < c_hi);
        if (!in_low || !(ft > bh)) continue;
        const double bb = ft - bh;
        double at = K11 + 1.0 - 2.0 * kh[e];  // K(t, t) = 1 for the RBF kernel
        if (at <= 0.0) at = eps;
        const double gain = -(bb * bb) / at;
        if (gain < cm.v) {  // ascending index within a thread: strict compare keeps the lowest
          cm = VI{gain, uint32_t(lo + t + NT * e)};
          ca = a;
          cf = ft;
          ck = kh[e];
        }
      }
      {
        const VIL wc = wave_arg<true>(cm);
        const double wa = read_lane64(ca, wc.lane), wf = read_lane64(cf, wc.lane), wk = read_lane64(ck, wc.lane);
        if (lane == 0) {
          sh.wv[0][w] = wc.v;
          sh.wi[0][w] = wc.i;
          sh.wa[0][w] = wa;
          sh.wv[1][w] = wf;
          sh.wa[1][w] = wk;
        }
      }
      __syncthreads();
      ++epoch;  // the second exchange's tags (records alternate parity buffers per exchange)
      unsigned long long* rec2 = slots + (size_t(epoch & 1) * (64 * RPL)) * kRecStride;
      if (w == 0) {
        VI a{inf, kSentinel};
        double aa = 0.0, af = 0.0, ak = 0.0;
        {
          VI c{inf, kSentinel};
          double c_a = 0.0, c_f = 0.0, c_k = 0.0;
          if (lane < NW) {
            c = VI{sh.wv[0][lane], sh.wi[0][lane]};
            c_a = sh.wa[0][lane];
            c_f = sh.wv[1][lane];
            c_k = sh.wa[1][lane];
          }
          const VIL r = wave_arg<true, NW>(c);
          a = VI{r.v, r.i};
          aa = read_lane64(c_a, r.lane);
          af = read_lane64(c_f, r.lane);
          ak = read_lane64(c_k, r.lane);
        }
        if (lane < kGranules) {
          uint32_t pay = lo32(a.v);
          pay = lane == 1 ? hi32(a.v) : pay;
          pay = lane == 2 ? a.i : pay;
          pay = lane == 3 ? lo32(aa) : pay;
          pay = lane == 4 ? hi32(aa) : pay;
          pay = lane == 5 ? lo32(af) : pay;
          pay = lane == 6 ? hi32(af) : pay;
          pay = lane == 7 ? a.i : pay;
          pay = lane == 8 ? lo32(ak) : pay;
          pay = lane == 9 ? hi32(ak) : pay;
          if constexpr (XLOCAL)  // same scope rule as the first exchange (memory-model note above)
            __hip_atomic_store(rec2 + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
          else
            __hip_atomic_store(rec2 + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        VI gm{inf, kSentinel};
        double ga = 0.0, gf = 0.0, gk = 0.0;
        bool timed_out = false;
        if (lane < G) {  // lane L: records L, L + 64, ... (as in the first exchange)
          uint32_t v[RPL][kGranules];
          for (int64_t spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int rr = 0; rr < RPL; ++rr) {
              if (RPL == 1 || lane + 64 * rr < G) {
                const unsigned long long* r = rec2 + size_t(lane + 64 * rr) * kRecStride;
#pragma unroll
                for (int k = 0; k < kGranules; ++k) {
                  const unsigned long long x = __hip_atomic_load(r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  v[rr][k] = uint32_t(x);
                  ok &= uint32_t(x >> 32) == epoch;
                }
              }
            }
            if (ok) break;
            if (spins > spin_limit) {
              timed_out = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (!timed_out) {
#pragma unroll
            for (int rr = 0; rr < RPL; ++rr) {
              if (RPL == 1 || lane + 64 * rr < G) {
                const VI c{mk64(v[rr][0], v[rr][1]), v[rr][2]};
                if (rr == 0 || beats<true>(c, gm)) {
                  gm = c;
                  ga = mk64(v[rr][3], v[rr][4]);
                  gf = mk64(v[rr][5], v[rr][6]);
                  gk = mk64(v[rr][8], v[rr][9]);
                }
              }
            }
          }
        }
        const bool any_to2 = __any(timed_out);
        const VIL wgm = wave_arg<true>(gm);
        const double wga = read_lane64(ga, wgm.lane), wgf = read_lane64(gf, wgm.lane), wgk = read_lane64(gk, wgm.lane);
        if (lane == 0) {
          sh.gi[1] = wgm.i;
          sh.ga[1] = wga;
          sh.gv[1] = wgf;
          sh.k12 = wgk;
          if (!any_to2 && wgm.i != kSentinel) rows.choose_one(sh, 1, wgm.i, sh.rslot[0]);  // keep row i_high
          if (any_to2) {
            sh.timeout = 1;
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      __syncthreads();
      if (sh.timeout) {
        stop = -1;
        break;
      }
      il = sh.gi[1];  // exists: the first-order i_low lies above f_ih + 2 tau
      bl_upd = sh.gv[1];
      al = sh.ga[1];
      K12 = sh.k12;
      rows.template fetch_one<NT, E>(sh, 1, il, lo, t, hi_end, kl, K22);
      yh = y[ih];
      yl = y[il];
    } else {
      // One memory round trip: scalars + this slice of rows i_high and i_low.
      yh = y[ih];
      yl = y[il];
      rows.template fetch<NT, E>(sh, ih, il, lo, t, hi_end, kh, kl, K11, K22, K12);
    }
    PSTAMP(5);
    const double ah = sh.ga[0];
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
      stop = SVM_STOP_INFEASIBLE;
      break;
    }
    if (eta <= eps) {
      stop = SVM_STOP_NONPOS_ETA;
      break;
    }
    double al_new = al + double(yl) * (bh - bl_upd) / eta;
    if (al_new > V) al_new = V;
    if (al_new < U) al_new = U;
    const double ah_new = ah + double(s) * (al - al_new);
    const double ch = (ah_new - ah) * double(yh);
    const double cl = (al_new - al) * double(yl);
    // ---- 5. apply: f for the whole slice, alpha for the owners
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      fr[e] += ch * kh[e] + cl * kl[e];  // main3.cpp:274 operation order
      if (i == ih) ar[e] = ah_new;
      if (i == il) ar[e] = al_new;
    }
    PSTAMP(6);
    if (g == 0 && t == 0 && trace && num_iter - 1 < trace_cap) {
      trace[2 * (num_iter - 1)] = ih;
      trace[2 * (num_iter - 1) + 1] = il;
    }
    ++num_iter;
    if (num_iter > max_iter) {
      stop = SVM_STOP_MAX_ITER;
      break;
    }
  }
  // Write the slice back; workgroup 0 publishes the final state (visible at kernel end).
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t i = lo + t + NT * e;
    if (i < hi_end) {
      f[i] = fr[e];
      alpha[i] = ar[e];
    }
  }
  if (STAMP && g == 0 && t == 0)
    for (int k = 0; k < 8; ++k) stamps[k] = sacc[k];
  if (g == 0 && t == 0) {
    st->num_iter = num_iter;
    st->b_high = b_high;
    st->b_low = b_low;
    st->pending = 0;
    st->stop = stop < 0 ? SVM_STOP_RUNNING : stop;
  }
  return epoch;
}


// XCD-local team registration (thread 0 of a workgroup running on XCD `xcc`).  reg[0] counts the
// workgroups that landed on the team's XCD: the first glocal take ranks 0..glocal-1 and wait until
// all have registered, for at most kRegisterTicks.  The outcome is one compare-and-swap on the
// decision word reg[1] (0 forming, 1 go, 2 abandoned), so all participants agree even when the last
// one registers just as another gives up.  Returns the rank, -1 (not a participant) or -2
// (abandoned: *err = 2, nothing touched).
__device__ int xcd_register(unsigned* reg, unsigned* err, int glocal, unsigned long long ticks) {
  const unsigned tk = __hip_atomic_fetch_add(reg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tk >= unsigned(glocal)) return -1;
  unsigned* decision = reg + 1;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned d;
  while ((d = __hip_atomic_load(decision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
    unsigned want = 0u;
    if (__hip_atomic_load(reg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= unsigned(glocal))
      __hip_atomic_compare_exchange_strong(decision, &want, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    else if (__builtin_amdgcn_s_memrealtime() - t_start > ticks)
      __hip_atomic_compare_exchange_strong(decision, &want, 2u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    else
      __builtin_amdgcn_s_sleep(2);
  }
  if (d != 1u) {
    __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return -2;
  }
  return int(tk);
}

__device__ __forceinline__ unsigned xcc_id() {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return xcc & 0xF;
}

// XLOCAL: all participating workgroups run on ONE XCD (XCD 0; the grid is over-provisioned, see
// xcd_register, the rest exit).  Records are then exchanged through that XCD's shared L2 (plain
// stores, L1-bypassing sc1 loads) instead of the device-wide fabric.  If XCD 0 receives fewer than
// glocal workgroups the registration is abandoned before any state is touched (err = 2) and the
// host falls back to the device-wide kernel.
template <int NT, int E, bool STAMP, bool XLOCAL = false, bool WSS2 = false>
__global__ __launch_bounds__(NT) void smo_persistent_kernel(
    const double* __restrict__ K, int64_t ldk, const int32_t* __restrict__ y, double* __restrict__ alpha,
    double* __restrict__ f, int64_t n, int64_t slice, unsigned long long* __restrict__ slots,
    SmoState* __restrict__ st, double C, double eps, double tau, int64_t max_iter, int64_t* __restrict__ trace,
    int64_t trace_cap, unsigned* __restrict__ err, int64_t spin_limit, unsigned long long* __restrict__ stamps,
    int glocal = 0, unsigned long long reg_ticks = kRegisterTicks) {
  __shared__ PersistShared sh;
  int G = gridDim.x, g = blockIdx.x;
  if constexpr (XLOCAL) {
    __shared__ int s_rank;
    if (threadIdx.x == 0) s_rank = xcc_id() == 0 ? xcd_register(err + 2, err, glocal, reg_ticks) : -1;
    __syncthreads();
    if (s_rank < 0) return;  // not a participant (or registration abandoned: nothing touched)
    G = glocal;
    g = s_rank;
  }
  persist_solve<NT, E, STAMP, XLOCAL, ResidentRows, 1, WSS2>(sh, G, g, 0, ResidentRows{K, ldk}, y, alpha, f, n, slice,
                                                             slots, st, C, eps,
                                      tau, max_iter,
                                      trace, trace_cap, err, spin_limit, stamps);
}

// Persistent SMO on the HBM row cache (n beyond the resident Gram; driven by rowcache.hip's
// run_smo_rowcache): device-wide exchange over G co-resident workgroups, CachedRows as the row
// source with its directory (nslots int32 tags + nslots / 2 MRU bytes) in dynamic LDS.
template <int NT, int E, bool INT, bool STAMP, int RPL, bool WSS2 = false>
__global__ __launch_bounds__(NT) void smo_rc_persistent_kernel(
    QRows q, double* __restrict__ cache, int64_t ldc, int64_t nslots, double neg_gamma, const int32_t* __restrict__ y,
    double* __restrict__ alpha, double* __restrict__ f, int64_t n, int64_t slice, unsigned long long* __restrict__ slots,
    SmoState* __restrict__ st, double C, double eps, double tau, int64_t max_iter, int64_t* __restrict__ trace,
    int64_t trace_cap, unsigned* __restrict__ err, int64_t spin_limit, unsigned long long* __restrict__ stamps) {
  __shared__ PersistShared sh;
  extern __shared__ __attribute__((aligned(16))) char rc_dir[];
  int32_t* tags = reinterpret_cast<int32_t*>(rc_dir);
  uint8_t* mru = reinterpret_cast<uint8_t*>(tags + nslots);
  for (int64_t k = threadIdx.x; k < nslots; k += NT) tags[k] = -1;
  for (int64_t k = threadIdx.x; k < nslots / 2; k += NT) mru[k] = 0;
  __syncthreads();
  const CachedRows<INT> rows{q, cache, ldc, tags, mru, nslots / 2, neg_gamma};
  persist_solve<NT, E, STAMP, false, CachedRows<INT>, RPL, WSS2>(sh, int(gridDim.x), int(blockIdx.x), 0, rows, y, alpha, f,
                                                          n, slice, slots, st, C, eps, tau, max_iter, trace, trace_cap,
                                                          err, spin_limit, stamps);
}

// ------------------------------------------------------------------------------------------------
// Batched solves (one-vs-rest: one SMO per class on the same resident Gram).  Every XCD forms its
// own team of glocal workgroups (xcd_register on its own registration words) and runs whole solves
// with the XCD-local exchange; teams pull class indices from one queue, so the eight XCDs work on
// eight classes at once and a team that finishes early takes the next class.  Team rank 0 takes
// the class and posts it in the team's mailbox ((round << 10) | class); the other members poll it.
// A team that cannot form leaves its classes to the others; the host re-runs any class no team
// took (st[k].stop still RUNNING).  ctl layout (u32): team x at [4x .. 4x+3] = {count, decision,
// mailbox, -}, queue at [kMultiQueue], error word at [kMultiErr].
constexpr int kMultiTeams = 8;
constexpr int kMultiQueue = 4 * kMultiTeams, kMultiErr = kMultiQueue + 1, kMultiCtlWords = 64;
constexpr unsigned long long kMailTicks = 10000000ull;  // 100 ms: a team member gives up waiting for a class

template <int NT, int E, bool WSS2 = false>
__global__ __launch_bounds__(NT) void smo_multi_kernel(
    const double* __restrict__ K, int64_t ldk, const int32_t* __restrict__ Y, double* __restrict__ A,
    double* __restrict__ F, int64_t n, int64_t slice, unsigned long long* __restrict__ slots,
    SmoState* __restrict__ st, int nclass, double C, double eps, double tau, int64_t max_iter,
    unsigned* __restrict__ ctl, int64_t spin_limit, int glocal, unsigned long long reg_ticks) {
  __shared__ PersistShared sh;
  __shared__ int s_rank, s_cls;
  const unsigned team = xcc_id();
  unsigned* err = ctl + kMultiErr;
  if (threadIdx.x == 0)
    s_rank = team < unsigned(kMultiTeams) ? xcd_register(ctl + 4 * team, err, glocal, reg_ticks) : -1;
  __syncthreads();
  const int g = s_rank;
  if (g < 0) return;
  unsigned* mail = ctl + 4 * team + 2;
  unsigned long long* tslots = slots + size_t(team) * 2 * kMaxG * kRecStride;
  uint32_t epoch = 0;
  for (unsigned round = 1;; ++round) {
    if (threadIdx.x == 0) {
      int cls = nclass;
      if (g == 0) {
        const unsigned c = __hip_atomic_fetch_add(ctl + kMultiQueue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cls = c < unsigned(nclass) ? int(c) : nclass;
        __hip_atomic_store(mail, (round << 10) | unsigned(cls), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          const unsigned v = __hip_atomic_load(mail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((v >> 10) == round) {
            cls = int(v & 1023u);
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > kMailTicks) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      s_cls = cls;
    }
    __syncthreads();
    const int cls = s_cls;
    if (cls >= nclass) break;
    epoch = persist_solve<NT, E, false, true, ResidentRows, 1, WSS2>(sh, glocal, g, epoch, ResidentRows{K, ldk},
                                                                     Y + int64_t(cls) * n,
                                              A + int64_t(cls) * n,
                                              F + int64_t(cls) * n, n, slice, tslots, st + cls, C, eps, tau, max_iter,
                                              nullptr, 0, err, spin_limit, nullptr);
    if (sh.timeout) break;
  }
}

// Cold start of nclass problems: alpha = 0, f = -y, fresh state.
__global__ void smo_multi_init_kernel(const int32_t* __restrict__ Y, double* __restrict__ A, double* __restrict__ F,
                                      int64_t total, SmoState* st, int nclass) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < total) {
    A[i] = 0.0;
    F[i] = -static_cast<double>(Y[i]);
  }
  if (i < nclass) st[i] = SmoState{0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, SVM_STOP_RUNNING};
}

// ------------------------------------------------------------------------------------------------
// Single-workgroup SMO for small problems (n <= NT * E, e.g. the cascade's merge solves on the
// gathered support vectors).  No cross-workgroup exchange at all: one NT-thread workgroup keeps
// the whole problem in registers and an iteration is
//   local scan -> wave64 two-stage arg-reduction -> per-wave record in LDS (double-buffered by
//   iteration parity) -> ONE __syncthreads -> every wave reduces the NT/64 records itself (identical
//   inputs and instruction sequence -> identical winners in every wave, no second barrier) ->
//   update scalars + one memory round trip for K11/K22/K12 and the two kernel rows -> f update.
// The arithmetic is the persistent kernel's (main3.cpp:235-275 order), so the trajectory is the
// same bit for bit.
struct SingleShared {
  double wv[2][2][16], wa[2][2][16];  // [parity][min|max][wave]
  uint32_t wi[2][2][16];
};

template <int kSingleNT, int E, bool STAMP>
__global__ __launch_bounds__(kSingleNT) void smo_single_kernel(
    const double* __restrict__ K, int64_t ldk, const int32_t* __restrict__ y, double* __restrict__ alpha,
    double* __restrict__ f, int64_t n, SmoState* __restrict__ st, double C, double eps, double tau, int64_t max_iter,
    int64_t* __restrict__ trace, int64_t trace_cap, unsigned long long* __restrict__ stamps) {
  constexpr int NW = kSingleNT / 64;
  __shared__ SingleShared sh;
  unsigned long long sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sprev = 0, rt0 = 0;
  bool stamping = false;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  const double inf = __builtin_inf();
  double fr[E], ar[E];
  int32_t yr[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t i = t + kSingleNT * e;
    const bool ok = i < n;
    fr[e] = ok ? f[i] : 0.0;
    ar[e] = ok ? alpha[i] : 0.0;
    yr[e] = ok ? y[i] : 0;
  }
  int64_t num_iter = st->num_iter;
  double b_high = st->b_high, b_low = st->b_low;
  int32_t stop = SVM_STOP_RUNNING;
  for (uint32_t it = 0;; ++it) {
    const int par = it & 1;
    if (STAMP) {
      const uint32_t epoch = it + 1;
      const bool on = threadIdx.x == 0 && epoch >= kStampFrom && epoch < kStampFrom + kStampCount;
      if (on && !stamping) rt0 = __builtin_amdgcn_s_memrealtime();
      if (!on && stamping) sacc[7] = __builtin_amdgcn_s_memrealtime() - rt0;
      stamping = on;
      if (stamping) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sprev)::"memory");
    }
    VI mn{inf, kSentinel}, mx{-inf, kSentinel};
    double amn = 0.0, amx = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t i = uint32_t(t + kSingleNT * e);
      const double a = ar[e], fi = fr[e];
      const int32_t yi = yr[e];
      const bool in_high = (yi == 1 && a < c_hi) || (yi == -1 && a > c_lo);
      const bool in_low = (yi == 1 && a > c_lo) || (yi == -1 && a < c_hi);
      if (in_high && fi < mn.v) {
        mn = VI{fi, i};
        amn = a;
      }
      if (in_low && fi > mx.v) {
        mx = VI{fi, i};
        amx = a;
      }
    }
    {
      const VIL wmn = wave_arg<true>(mn), wmx = wave_arg<false>(mx);
      const double awmn = read_lane64(amn, wmn.lane), awmx = read_lane64(amx, wmx.lane);
      PSTAMP(0);
      if (lane == 0) {
        sh.wv[par][0][w] = wmn.v;
        sh.wi[par][0][w] = wmn.i;
        sh.wa[par][0][w] = awmn;
        sh.wv[par][1][w] = wmx.v;
        sh.wi[par][1][w] = wmx.i;
        sh.wa[par][1][w] = awmx;
      }
    }
    __syncthreads();
    PSTAMP(1);
    VI ca{inf, kSentinel}, cb{-inf, kSentinel};
    double caa = 0.0, cba = 0.0;
    if (lane < NW) {
      ca = VI{sh.wv[par][0][lane], sh.wi[par][0][lane]};
      cb = VI{sh.wv[par][1][lane], sh.wi[par][1][lane]};
      caa = sh.wa[par][0][lane];
      cba = sh.wa[par][1][lane];
    }
    const VIL ga = wave_arg<true, NW>(ca), gb = wave_arg<false, NW>(cb);
    const double aga = read_lane64(caa, ga.lane), agb = read_lane64(cba, gb.lane);
    const uint32_t uih = ga.i, uil = gb.i;
    if (uih == kSentinel || uil == kSentinel) {
      stop = SVM_STOP_NO_CANDIDATE;
      break;
    }
    PSTAMP(2);
    const int64_t ih = uih, il = uil;
    const double bh = ga.v, bl = gb.v;
    b_high = bh;
    b_low = bl;
    if (bl <= bh + 2.0 * tau) {
      stop = SVM_STOP_CONVERGED;
      break;
    }
    const int32_t yh = y[ih], yl = y[il];
    const double K11 = K[ih * ldk + ih], K22 = K[il * ldk + il], K12 = K[ih * ldk + il];
    double kh[E], kl[E];
    const double* Kh = K + ih * ldk;
    const double* Kl = K + il * ldk;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = t + kSingleNT * e;
      const bool ok = i < n;
      kh[e] = ok ? Kh[i] : 0.0;
      kl[e] = ok ? Kl[i] : 0.0;
    }
    PSTAMP(3);
    const double ah = aga, al = agb;
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
      stop = SVM_STOP_INFEASIBLE;
      break;
    }
    if (eta <= eps) {
      stop = SVM_STOP_NONPOS_ETA;
      break;
    }
    double al_new = al + double(yl) * (bh - bl) / eta;
    if (al_new > V) al_new = V;
    if (al_new < U) al_new = U;
    const double ah_new = ah + double(s) * (al - al_new);
    const double ch = (ah_new - ah) * double(yh);
    const double cl = (al_new - al) * double(yl);
    PSTAMP(4);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = t + kSingleNT * e;
      fr[e] += ch * kh[e] + cl * kl[e];  // main3.cpp:274 operation order
      if (i == ih) ar[e] = ah_new;
      if (i == il) ar[e] = al_new;
    }
    PSTAMP(5);
    if (t == 0 && trace && num_iter - 1 < trace_cap) {
      trace[2 * (num_iter - 1)] = ih;
      trace[2 * (num_iter - 1) + 1] = il;
    }
    ++num_iter;
    if (num_iter > max_iter) {
      stop = SVM_STOP_MAX_ITER;
      break;
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t i = t + kSingleNT * e;
    if (i < n) {
      f[i] = fr[e];
      alpha[i] = ar[e];
    }
  }
  if (STAMP && t == 0)
    for (int q = 0; q < 8; ++q) stamps[q] = sacc[q];
  if (t == 0) {
    st->num_iter = num_iter;
    st->b_high = b_high;
    st->b_low = b_low;
    st->pending = 0;
    st->stop = stop;
  }
}

}  // namespace

namespace {

// XCD-local registration window (SVM355_PSMO_REG_US overrides, microseconds).
unsigned long long register_ticks() {
  if (const char* v = getenv("SVM355_PSMO_REG_US")) return std::max(1ull, strtoull(v, nullptr, 10)) * 100ull;
  return kRegisterTicks;
}

// Dynamic LDS reserved (unused) by the XCD-local launches so that at most one workgroup lands on a
// CU: the team then spreads over the XCD's CUs instead of doubling up, e.g. 2.75 instead of 3.25
// us/iter at n = 24k (SVM355_PSMO_LDS overrides; 0 = none).  1024-thread workgroups need none.
size_t xcd_lds_pad(int NT) {
  if (const char* v = getenv("SVM355_PSMO_LDS")) return size_t(std::max(0, atoi(v)));
  return NT == 1024 ? 0 : size_t(96) << 10;
}

template <class Kern>
void allow_lds(Kern k, size_t bytes) {
  if (bytes > (size_t(64) << 10))
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(bytes));
}

// Launch the persistent solver for a (threads per workgroup NT, elements per thread E) shape.
template <int NT, int E>
int launch_persistent_e(hipStream_t s, int G, const double* K, int64_t ldk, const int32_t* y, double* alpha,
                        double* f, int64_t n, unsigned long long* slots, SmoState* st, double C, double eps,
                        double tau, int64_t max_iter, int64_t* trace, int64_t tcap, unsigned* err, bool xlocal,
                        bool wss2) {
  unsigned long long* stamps = reinterpret_cast<unsigned long long*>(err) + 8;
  const int64_t slice = int64_t(NT) * E;
  if (wss2) {  // opt-in second-order selection (no stamp variant)
    if (xlocal) {
      const size_t lds = xcd_lds_pad(NT);
      allow_lds(smo_persistent_kernel<NT, E, false, true, true>, lds);
      hipLaunchKernelGGL((smo_persistent_kernel<NT, E, false, true, true>), dim3(16 * G), dim3(NT), lds, s, K, ldk, y,
                         alpha, f, n, slice, slots, st, C, eps, tau, max_iter, trace, tcap, err, int64_t(1) << 22,
                         stamps, G, register_ticks());
    } else {
      hipLaunchKernelGGL((smo_persistent_kernel<NT, E, false, false, true>), dim3(G), dim3(NT), 0, s, K, ldk, y, alpha,
                         f, n, slice, slots, st, C, eps, tau, max_iter, trace, tcap, err, int64_t(1) << 24, stamps);
    }
    SVMD_LAUNCH_CHECK();
    return SVM_OK;
  }
  const char* sv = getenv("SVM355_PSMO_STAMP");
  if (xlocal) {
    // Over-provisioned grid: ~2*G workgroups per XCD under round-robin dispatch; G of XCD 0's join.
    const int grid = 16 * G;
    const size_t lds = xcd_lds_pad(NT);
    if (sv && atoi(sv)) {
      allow_lds(smo_persistent_kernel<NT, E, true, true>, lds);
      hipLaunchKernelGGL((smo_persistent_kernel<NT, E, true, true>), dim3(grid), dim3(NT), lds, s, K, ldk, y, alpha,
                         f, n, slice, slots, st, C, eps, tau, max_iter, trace, tcap, err, int64_t(1) << 22, stamps, G,
                         register_ticks());
    } else {
      allow_lds(smo_persistent_kernel<NT, E, false, true>, lds);
      hipLaunchKernelGGL((smo_persistent_kernel<NT, E, false, true>), dim3(grid), dim3(NT), lds, s, K, ldk, y, alpha,
                         f, n, slice, slots, st, C, eps, tau, max_iter, trace, tcap, err, int64_t(1) << 22, stamps, G,
                         register_ticks());
    }
    SVMD_LAUNCH_CHECK();
    return SVM_OK;
  }
  if (sv && atoi(sv))
    hipLaunchKernelGGL((smo_persistent_kernel<NT, E, true>), dim3(G), dim3(NT), 0, s, K, ldk, y, alpha, f, n, slice,
                       slots, st, C, eps, tau, max_iter, trace, tcap, err, int64_t(1) << 24, stamps);
  else
    hipLaunchKernelGGL((smo_persistent_kernel<NT, E, false>), dim3(G), dim3(NT), 0, s, K, ldk, y, alpha, f, n,
                       slice, slots, st, C, eps, tau, max_iter, trace, tcap, err, int64_t(1) << 24, stamps);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

// Grid shape: NT threads per workgroup (SVM355_PSMO_NT, default kDefaultNT), the smallest E in
// {1, 2, 4, 8, 16} (capped per NT) with G = ceil(n / (NT*E)) <= target workgroups (SVM355_PSMO_WG,
// default 64; all co-resident, one sweep pass).
constexpr int kDefaultNT = 512;
constexpr int kXcdMaxG = 32;              // workgroups of the XCD-local solver (one XCD has 32 CUs)
constexpr int64_t kXcdDefaultMax = 65536;  // default n limit of the XCD-local solver (tuned on MI355X)
constexpr int64_t kSingleDefaultMax = 2048;  // auto mode: single workgroup up to this n (tuned on MI355X)
constexpr int kSingleDefaultNT = 512;
int persistent_grid(int64_t n, int* G_out, int* E_out, int* NT_out, int gcap) {
  int target = 64;
  if (const char* v = getenv("SVM355_PSMO_WG")) target = std::max(1, std::min(kMaxG, atoi(v)));
  if (gcap > 0) target = std::min(target, gcap);
  // Measured on MI355X (profiles/r1_smo_launch_shape.txt): the XCD-local solver wants 256-thread
  // workgroups up to ~16k points and 512-thread ones above, one per CU (xcd_lds_pad): 2.45-3.44
  // us/iter from 10k to 60k, 4-17 % below the device-wide exchange.
  int nt = kDefaultNT;
  if (gcap > 0 && n <= 16000) nt = 256;
  if (const char* v = getenv("SVM355_PSMO_NT")) nt = atoi(v);
  if (nt != 256 && nt != 512 && nt != 1024) nt = kDefaultNT;
  const int emax = nt == 256 ? 16 : nt == 512 ? 8 : 4;
  for (int E = 1; E <= emax; E *= 2) {
    const int64_t per_wg = int64_t(nt) * E;
    const int64_t G = (n + per_wg - 1) / per_wg;
    if (G <= target) {
      *G_out = int(std::max<int64_t>(1, G));
      *E_out = E;
      *NT_out = nt;
      return 1;
    }
  }
  return 0;
}

int launch_persistent(hipStream_t s, int NT, int E, int G, const double* K, int64_t ldk, const int32_t* y,
                      double* alpha, double* f, int64_t n, unsigned long long* slots, SmoState* st, double C,
                      double eps, double tau, int64_t max_iter, int64_t* trace, int64_t tcap, unsigned* err,
                      bool xlocal, bool wss2) {
#define SVM_PSMO_CASE(nt, e)                                                                                 \
  if (NT == nt && E == e)                                                                                    \
    return launch_persistent_e<nt, e>(s, G, K, ldk, y, alpha, f, n, slots, st, C, eps, tau, max_iter, trace, \
                                      tcap, err, xlocal, wss2);
  SVM_PSMO_CASE(256, 1) SVM_PSMO_CASE(256, 2) SVM_PSMO_CASE(256, 4) SVM_PSMO_CASE(256, 8) SVM_PSMO_CASE(256, 16)
  SVM_PSMO_CASE(512, 1) SVM_PSMO_CASE(512, 2) SVM_PSMO_CASE(512, 4) SVM_PSMO_CASE(512, 8)
  SVM_PSMO_CASE(1024, 1) SVM_PSMO_CASE(1024, 2) SVM_PSMO_CASE(1024, 4)
#undef SVM_PSMO_CASE
  set_error("persistent SMO: no kernel for NT=%d E=%d", NT, E);
  return SVM_ERR_INTERNAL;
}

int finish_smo(const SmoState& fin, svm_result* r, int64_t* trace, const int64_t* dtrace, int64_t tcap,
               std::chrono::steady_clock::time_point t0) {
  if (!fin.stop) {
    set_error("svmd_smo: solver did not stop within its budget");
    return SVM_ERR_INTERNAL;
  }
  if (tcap) {
    const int64_t nt = std::min<int64_t>(fin.num_iter - 1, tcap);
    if (nt > 0) SVMD_CHECK(hipMemcpy(trace, dtrace, size_t(nt) * 16, hipMemcpyDeviceToHost));
  }
  if (r) {
    r->iterations = fin.num_iter;
    r->b_high = fin.b_high;
    r->b_low = fin.b_low;
    r->b = (fin.b_high + fin.b_low) / 2;
    r->stop_reason = fin.stop;
    r->reserved = 0;
    r->n_sv = -1;  // filled by the caller (needs alpha on the host or a device count)
    r->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return SVM_OK;
}

}  // namespace

namespace {
template <int E, bool INT, bool STAMP, int RPL, bool WSS2 = false>
void launch_rc_e(hipStream_t s, int G, size_t lds, const QRows& q, double* cache, int64_t ldc, int64_t nslots,
                 double neg_gamma, const int32_t* y, double* alpha, double* f, int64_t n, unsigned long long* slots,
                 SmoState* st, const svm_params& p, int64_t* trace, int64_t tcap, unsigned* err) {
  allow_lds(smo_rc_persistent_kernel<512, E, INT, STAMP, RPL, WSS2>, lds);
  hipLaunchKernelGGL((smo_rc_persistent_kernel<512, E, INT, STAMP, RPL, WSS2>), dim3(G), dim3(512), lds, s, q, cache, ldc,
                     nslots, neg_gamma, y, alpha, f, n, int64_t(512) * E, slots, st, p.C, p.eps, p.tau, p.max_iter,
                     trace, tcap, err, int64_t(1) << 24, reinterpret_cast<unsigned long long*>(err) + 8);
}
template <int E, int RPL>
void launch_rc_variant(bool int_rows, bool stamp, hipStream_t s, int G, size_t lds, const QRows& q, double* cache,
                       int64_t ldc, int64_t nslots, double neg_gamma, const int32_t* y, double* alpha, double* f,
                       int64_t n, unsigned long long* slots, SmoState* st, const svm_params& p, int64_t* trace,
                       int64_t tcap, unsigned* err) {
  if (int_rows && p.wss == 2)  // opt-in second-order selection (exact-integer rows)
    launch_rc_e<E, true, false, RPL, true>(s, G, lds, q, cache, ldc, nslots, neg_gamma, y, alpha, f, n, slots, st, p,
                                           trace, tcap, err);
  else if (int_rows && stamp)
    launch_rc_e<E, true, true, RPL>(s, G, lds, q, cache, ldc, nslots, neg_gamma, y, alpha, f, n, slots, st, p, trace,
                                    tcap, err);
  else if (int_rows)
    launch_rc_e<E, true, false, RPL>(s, G, lds, q, cache, ldc, nslots, neg_gamma, y, alpha, f, n, slots, st, p, trace,
                                     tcap, err);
  else
    launch_rc_e<E, false, false, RPL>(s, G, lds, q, cache, ldc, nslots, neg_gamma, y, alpha, f, n, slots, st, p, trace,
                                      tcap, err);
}
constexpr int kRcMaxG = 256;  // records per epoch parity of the row-cache solver's slot array
}  // namespace

// Persistent row-cache solve (see smo_rc_persistent_kernel).  f / alpha hold the initial state (cold
// or warm, set up by the caller); cache: nslots x ldc doubles.  Returns kRcNotApplicable when no
// persistent shape covers n (the caller then replays its select/step graph).
int run_smo_rc_persistent(DeviceCtx* ctx, const QRows& q, bool int_rows, double* cache, int64_t ldc, int64_t nslots,
                          const int32_t* y, double* alpha, double* f, int64_t n, const svm_params& p, svm_result* r,
                          int64_t* trace, int64_t trace_cap) {
  if (const char* m = getenv("SVM355_RC_SMO"); m && !strcmp(m, "graph")) return kRcNotApplicable;
  if (n <= 0 || n >= int64_t(kSentinel)) return kRcNotApplicable;
  if (int_rows && q.kq > 32 * 128) return kRcNotApplicable;  // CachedRows::k12: two k-steps per lane
  if (p.wss == 2 && !int_rows) return kRcNotApplicable;       // second order: exact-integer rows only
  // Shape: up to 8 register-resident points per thread (E = 16 needs more than 256 VGPRs and
  // spills) and one 512-thread workgroup per CU, all co-resident.  Teams of up to 64 workgroups
  // (one record per sweep lane) with E <= 4, then 128 and 256 (two / four records per lane, capped
  // by the CU count) with E <= 8: n <= 256 x 512 x 8 = 1,048,576.  Measured (profiles/
  // r2_rowcache_persistent.txt): at 60k 59 x E=2 beats 118 x E=1 (98 vs 104 ms); at 250k 123 x E=4
  // beats 62 x E=8 (465 vs 572 ms: half the miss fill per workgroup); 256-wide teams lose to 128
  // wherever both fit.  SVM355_RC_MAXG=128|256 starts at a wider team.  Larger n keep the replayed
  // select / step graph.
  int ncu = 0;
  SVMD_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
  int cap0 = 64;
  if (const char* v = getenv("SVM355_RC_MAXG")) cap0 = std::max(64, std::min(kRcMaxG, atoi(v)));
  int E = 0, G = 0;
  for (int cap = cap0; cap <= kRcMaxG && !E; cap *= 2) {
    const int maxg = std::min(cap, ncu);
    for (int e = 1; e <= (cap == 64 ? 4 : 8) && !E; e *= 2)
      if ((n + 512 * e - 1) / (512 * e) <= maxg) E = e;
  }
  if (!E) return kRcNotApplicable;
  G = int((n + 512 * E - 1) / (512 * E));
  const int rpl = G <= 64 ? 1 : G <= 128 ? 2 : 4;
  // Directory in LDS: up to 16384 slots (64 KB of tags + 8 KB of MRU bits) next to PersistShared.
  const int64_t nd = std::min<int64_t>(nslots, 16384) / 2 * 2;
  if (nd < 4) return kRcNotApplicable;
  const size_t lds = (size_t(nd) * 4 + size_t(nd) / 2 + 15) / 16 * 16;
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = ctx->stream;
  const int64_t tcap = trace ? std::max<int64_t>(trace_cap, 0) : 0;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  // records (both epoch parities), error word + phase stamps, exchange-skew stamps (RPL = 1)
  const size_t rec_bytes = size_t(2) * kRcMaxG * kRecStride * 8;
  const size_t off_slots = 0, slot_bytes = rec_bytes + 256 + (size_t(kMaxG) + 1) * kSkewEpochs * 8;
  const size_t off_st = off_slots + al(slot_bytes);
  const size_t off_trace = off_st + al(sizeof(SmoState));
  int rc = ctx->ensure_ws(off_trace + al(size_t(tcap) * 16));
  if (rc) return rc;
  rc = ctx->ensure_pinned(sizeof(SmoState) * 3);
  if (rc) return rc;
  char* ws = static_cast<char*>(ctx->ws);
  auto* slots = reinterpret_cast<unsigned long long*>(ws + off_slots);
  auto* err = reinterpret_cast<unsigned*>(ws + off_slots + rec_bytes);
  auto* st = reinterpret_cast<SmoState*>(ws + off_st);
  int64_t* dtrace = tcap ? reinterpret_cast<int64_t*>(ws + off_trace) : nullptr;
  SmoState* hst = static_cast<SmoState*>(ctx->pinned);
  hst[0] = SmoState{0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, SVM_STOP_RUNNING};
  SVMD_CHECK(hipMemsetAsync(slots, 0, slot_bytes, s));
  SVMD_CHECK(hipMemcpyAsync(st, &hst[0], sizeof(SmoState), hipMemcpyHostToDevice, s));
  const double ng = -p.gamma;
  const char* stv = getenv("SVM355_PSMO_STAMP");
  const bool stamp = stv && atoi(stv);
  if (stamp) {
    const char* fv = getenv("SVM355_PSMO_STAMP_FROM");
    const unsigned long long from = fv ? std::max(1ll, atoll(fv)) : 0ull;
    SVMD_CHECK(hipMemcpyAsync(reinterpret_cast<unsigned long long*>(err) + 16, &from, 8, hipMemcpyHostToDevice, s));
    SVMD_CHECK(hipStreamSynchronize(s));
  }
#define SVM_RC_CASE(e, r)                                                                                           \
  else if (E == e && rpl == r) launch_rc_variant<e, r>(int_rows, stamp, s, G, lds, q, cache, ldc, nd, ng, y, alpha, f, \
                                                       n, slots, st, p, dtrace, tcap, err);
  if (false) {
  }
  SVM_RC_CASE(1, 1) SVM_RC_CASE(2, 1) SVM_RC_CASE(4, 1) SVM_RC_CASE(8, 1)
  SVM_RC_CASE(1, 2) SVM_RC_CASE(2, 2) SVM_RC_CASE(4, 2) SVM_RC_CASE(8, 2)
  SVM_RC_CASE(1, 4) SVM_RC_CASE(2, 4) SVM_RC_CASE(4, 4) SVM_RC_CASE(8, 4)
  else {
    set_error("row-cache SMO: no kernel for E=%d, %d records per lane", E, rpl);
    return SVM_ERR_INTERNAL;
  }
#undef SVM_RC_CASE
  SVMD_LAUNCH_CHECK();
  unsigned herr = 0;
  SVMD_CHECK(hipMemcpyAsync(&hst[2], st, sizeof(SmoState), hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipMemcpyAsync(&herr, err, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  if (herr) {
    set_error("row-cache SMO: persistent solver timed out waiting for a workgroup record (G=%d)", G);
    return SVM_ERR_DEVICE;
  }
  if (stamp && int_rows) {
    unsigned long long hs[8];
    SVMD_CHECK(hipMemcpy(hs, reinterpret_cast<unsigned long long*>(err) + 8, sizeof(hs), hipMemcpyDeviceToHost));
    const double cnt = double(kStampCount);
    fprintf(stderr, "[rc stamps G=%d E=%d RPL=%d] cycles/iter: scan+wavered %.0f | barrier1 %.0f | publish %.0f | sweep %.0f | "
            "globalred+choose+barrier2 %.0f | rows (hit read / miss fill) %.0f | update %.0f | us/iter %.3f\n", G, E, rpl,
            hs[0] / cnt, hs[1] / cnt, hs[2] / cnt, hs[3] / cnt, hs[4] / cnt, hs[5] / cnt, hs[6] / cnt,
            double(hs[7]) / 100.0 / cnt);
  }
  return finish_smo(hst[2], r, trace, dtrace, tcap, t0);
}

int run_smo(DeviceCtx* ctx, const double* K, int64_t ldk, const int32_t* y, int64_t n, double* alpha,
            int32_t warm, const svm_params& p, svm_result* r, int64_t* trace, int64_t trace_cap) {
  if (n <= 0) {
    set_error("svmd_smo: empty problem");
    return SVM_ERR_EMPTY;
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = ctx->stream;
  const int nblk = int(std::min<int64_t>((n + kSelectThreads - 1) / kSelectThreads, 2048));
  if (trace_cap < 0) trace_cap = 0;
  const int64_t tcap = trace ? trace_cap : 0;
  // Workspace layout (256-byte aligned pieces).
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t off_f = 0;
  const size_t off_part = off_f + al(size_t(n) * 8);
  const size_t off_state = off_part + al(size_t(nblk) * sizeof(Partial));
  const size_t off_idx = off_state + al(sizeof(SmoState));
  const size_t off_coef = off_idx + al(size_t(n) * 8);
  const size_t off_cnt = off_coef + al(size_t(n) * 8);
  const size_t off_trace = off_cnt + al(8);
  const size_t off_slots = off_trace + al(size_t(tcap) * 16);
  // records + error word + phase stamps + exchange-skew stamps
  const size_t slot_bytes = size_t(2) * kMaxG * kRecStride * 8 + 256 + (size_t(kMaxG) + 1) * kSkewEpochs * 8;
  const size_t total = off_slots + al(slot_bytes);
  int rc = ctx->ensure_ws(total);
  if (rc) return rc;
  rc = ctx->ensure_pinned(sizeof(SmoState) * 3);
  if (rc) return rc;
  char* ws = static_cast<char*>(ctx->ws);
  double* f = reinterpret_cast<double*>(ws + off_f);
  Partial* part = reinterpret_cast<Partial*>(ws + off_part);
  SmoState* st = reinterpret_cast<SmoState*>(ws + off_state);
  int64_t* idx = reinterpret_cast<int64_t*>(ws + off_idx);
  double* coef = reinterpret_cast<double*>(ws + off_coef);
  int64_t* cnt = reinterpret_cast<int64_t*>(ws + off_cnt);
  int64_t* dtrace = tcap ? reinterpret_cast<int64_t*>(ws + off_trace) : nullptr;

  if (!warm) {
    hipLaunchKernelGGL(smo_init_cold_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, y, alpha, f,
                       n, st);
    SVMD_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(nonzero_compact_kernel, dim3(1), dim3(1024), 0, s, alpha, y, n, idx, coef, cnt, st);
    SVMD_LAUNCH_CHECK();
    hipLaunchKernelGGL(warm_f_kernel, dim3(unsigned((n + 63) / 64)), dim3(64), 0, s, K, ldk, y, idx, coef, cnt, f,
                       n);
    SVMD_LAUNCH_CHECK();
  }

  // ---- persistent single-launch solver (default when the slices fit in registers)
  int G = 0, E = 0, NT = 0;
  const char* mode = getenv("SVM355_SMO");
  // ---- single-workgroup solver for small problems (no cross-workgroup exchange)
  const bool force_single = mode && strcmp(mode, "single") == 0;
  int64_t single_max = kSingleDefaultMax;
  if (const char* v = getenv("SVM355_SMO_SINGLE_MAX")) single_max = atoll(v);
  // Second-order selection (p.wss == 2, opt-in) exists in the persistent solver only.
  const bool wss2 = p.wss == 2;
  if (!wss2 && (force_single || !mode || strcmp(mode, "auto") == 0) && (force_single || n <= single_max) &&
      n <= 8192) {
    int snt = kSingleDefaultNT;
    if (const char* v = getenv("SVM355_SMO_SINGLE_NT")) snt = atoi(v);
    if (snt != 256 && snt != 512 && snt != 1024) snt = kSingleDefaultNT;
    int e = 1;
    while (int64_t(snt) * e < n) e *= 2;
    const char* stv = getenv("SVM355_PSMO_STAMP");
    const bool stamp = stv && atoi(stv);
    auto* sstamps = reinterpret_cast<unsigned long long*>(ws + off_slots);
#define SVM_SINGLE_CASE(nt, ee)                                                                                     \
  else if (snt == nt && e == ee) {                                                                                  \
    if (stamp)                                                                                                      \
      hipLaunchKernelGGL((smo_single_kernel<nt, ee, true>), dim3(1), dim3(nt), 0, s, K, ldk, y, alpha, f, n, st,    \
                         p.C, p.eps, p.tau, p.max_iter, dtrace, tcap, sstamps);                                     \
    else                                                                                                            \
      hipLaunchKernelGGL((smo_single_kernel<nt, ee, false>), dim3(1), dim3(nt), 0, s, K, ldk, y, alpha, f, n, st,   \
                         p.C, p.eps, p.tau, p.max_iter, dtrace, tcap, sstamps);                                     \
  }
    if (false) {
    }
    SVM_SINGLE_CASE(256, 1) SVM_SINGLE_CASE(256, 2) SVM_SINGLE_CASE(256, 4) SVM_SINGLE_CASE(256, 8)
    SVM_SINGLE_CASE(256, 16) SVM_SINGLE_CASE(256, 32)
    SVM_SINGLE_CASE(512, 1) SVM_SINGLE_CASE(512, 2) SVM_SINGLE_CASE(512, 4) SVM_SINGLE_CASE(512, 8) SVM_SINGLE_CASE(512, 16)
    SVM_SINGLE_CASE(1024, 1) SVM_SINGLE_CASE(1024, 2) SVM_SINGLE_CASE(1024, 4) SVM_SINGLE_CASE(1024, 8)
    else {
      set_error("single-workgroup SMO: n = %lld too large for %d threads", (long long)n, snt);
      return SVM_ERR_INTERNAL;
    }
#undef SVM_SINGLE_CASE
    SVMD_LAUNCH_CHECK();
    SmoState* hst = static_cast<SmoState*>(ctx->pinned);
    SVMD_CHECK(hipMemcpyAsync(&hst[2], st, sizeof(SmoState), hipMemcpyDeviceToHost, s));
    SVMD_CHECK(hipStreamSynchronize(s));
    if (stamp) {
      unsigned long long hs[8];
      SVMD_CHECK(hipMemcpy(hs, sstamps, sizeof(hs), hipMemcpyDeviceToHost));
      const double cnt = double(kStampCount);
      fprintf(stderr, "[single stamps NT=%d E=%d] cycles/iter: scan+wavered %.0f | barrier %.0f | blockred %.0f | "
              "loads %.0f | scalar %.0f | update %.0f | us/iter %.3f\n", snt, e, hs[0] / cnt, hs[1] / cnt, hs[2] / cnt,
              hs[3] / cnt, hs[4] / cnt, hs[5] / cnt, double(hs[7]) / 100.0 / cnt);
    }
    return finish_smo(hst[2], r, trace, dtrace, tcap, t0);
  }
  const bool want_persistent = wss2 || !(mode && strcmp(mode, "graph") == 0);
  // XCD-local exchange (all workgroups on one XCD, records through its L2): SVM355_PSMO_XCD=1/0
  // forces it on/off; the default enables it up to kXcdDefaultMax points.
  bool xlocal = n <= kXcdDefaultMax;
  if (const char* v = getenv("SVM355_PSMO_XCD")) xlocal = atoi(v) != 0;
  if (want_persistent && n < int64_t(kSentinel) && persistent_grid(n, &G, &E, &NT, xlocal ? kXcdMaxG : 0)) {
    auto* slots = reinterpret_cast<unsigned long long*>(ws + off_slots);
    auto* err = reinterpret_cast<unsigned*>(ws + off_slots + size_t(2) * kMaxG * kRecStride * 8);
    SmoState* hst = static_cast<SmoState*>(ctx->pinned);
    unsigned herr = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
      SVMD_CHECK(hipMemsetAsync(slots, 0, slot_bytes, s));  // epochs restart at 1 every launch
      const int lrc = launch_persistent(s, NT, E, G, K, ldk, y, alpha, f, n, slots, st, p.C, p.eps, p.tau,
                                        p.max_iter, dtrace, tcap, err, xlocal, wss2);
      if (lrc) return lrc;
      SVMD_CHECK(hipMemcpyAsync(&hst[2], st, sizeof(SmoState), hipMemcpyDeviceToHost, s));
      SVMD_CHECK(hipMemcpyAsync(&herr, err, sizeof(unsigned), hipMemcpyDeviceToHost, s));
      SVMD_CHECK(hipStreamSynchronize(s));
      if (!(xlocal && herr == 2)) break;
      // XCD 0 did not receive enough workgroups: nothing was touched, run the device-wide kernel.
      unsigned reg[2] = {0, 0};
      SVMD_CHECK(hipMemcpy(reg, err + 2, sizeof(reg), hipMemcpyDeviceToHost));
      static std::atomic<int> reported{0};
      if (reported.fetch_add(1) == 0)
        fprintf(stderr, "[svm355] XCD-local SMO: fewer than %d workgroups registered on XCD 0 within %.0f us "
                "(%u landed there in all, grid %d; another XCD-local solve running concurrently?); running the "
                "device-wide solver (reported once)\n", G, double(register_ticks()) / 100.0, reg[0], 16 * G);
      xlocal = false;
      if (!persistent_grid(n, &G, &E, &NT, 0)) break;
      herr = 0;
    }
    if (herr) {
      set_error("svmd_smo: persistent solver timed out waiting for a workgroup record (G=%d)", G);
      return SVM_ERR_DEVICE;
    }
    if (const char* sv = getenv("SVM355_PSMO_STAMP"); sv && atoi(sv)) {
      unsigned long long hs[8];
      SVMD_CHECK(hipMemcpy(hs, reinterpret_cast<unsigned long long*>(err) + 8, sizeof(hs), hipMemcpyDeviceToHost));
      const double cnt = double(kStampCount), mhz = hs[7] ? double(hs[0] + hs[1] + hs[2] + hs[3] + hs[4] + hs[5] + hs[6]) / (double(hs[7]) / 100.0) : 0.0;
      fprintf(stderr, "[psmo stamps NT=%d G=%d E=%d] cycles/iter: scan+wavered %.0f | barrier1 %.0f | publish %.0f | sweep %.0f | "
              "globalred+barrier2 %.0f | loads %.0f | update %.0f | clock %.0f MHz | us/iter %.3f\n", NT, G, E,
              hs[0] / cnt, hs[1] / cnt, hs[2] / cnt, hs[3] / cnt, hs[4] / cnt, hs[5] / cnt, hs[6] / cnt, mhz,
              double(hs[7]) / 100.0 / cnt);
      if (atoi(sv) == 2) {  // exchange skew: spread of the record publications, and WG 0's wait past the last
        std::vector<unsigned long long> sk(size_t(kMaxG + 1) * kSkewEpochs);
        SVMD_CHECK(hipMemcpy(sk.data(), reinterpret_cast<unsigned long long*>(err) + 8 + kSkewBase,
                             sk.size() * 8, hipMemcpyDeviceToHost));
        double spread = 0.0, tail = 0.0;
        std::vector<double> late(size_t(G), 0.0);  // mean lateness of each workgroup behind the first
        int used = 0;
        for (uint32_t e = 0; e < kSkewEpochs; ++e) {
          unsigned long long lo = ~0ull, hi = 0;
          for (int q = 0; q < G; ++q) {
            const unsigned long long v = sk[size_t(q) * kSkewEpochs + e];
            lo = std::min(lo, v);
            hi = std::max(hi, v);
          }
          const unsigned long long done = sk[size_t(kMaxG) * kSkewEpochs + e];
          if (!lo || !done || done < hi) continue;
          ++used;
          spread += double(hi - lo) * 10.0;
          tail += double(done - hi) * 10.0;
          for (int q = 0; q < G; ++q) late[size_t(q)] += double(sk[size_t(q) * kSkewEpochs + e] - lo) * 10.0;
        }
        if (used) {
          fprintf(stderr, "[psmo skew G=%d, %d epochs] publication spread %.0f ns | last publication -> WG0 sweep done %.0f ns\n",
                  G, used, spread / used, tail / used);
          fprintf(stderr, "[psmo skew] mean lateness per workgroup (ns):");
          for (int q = 0; q < G; ++q) fprintf(stderr, " %.0f", late[size_t(q)] / used);
          fprintf(stderr, "\n");
        }
      }
    }
    return finish_smo(hst[2], r, trace, dtrace, tcap, t0);
  }
  if (wss2) {
    set_error("svmd_smo: second-order selection (wss = 2) needs the persistent solver (n = %lld has no shape)",
              (long long)n);
    return SVM_ERR_ARG;
  }

  // Graph of kChunk iterations, cached per context for identical arguments.
  const double C = p.C, eps = p.eps, tau = p.tau;
  const int64_t max_iter = p.max_iter;
  std::vector<uint64_t> key = {uint64_t(uintptr_t(K)), uint64_t(ldk), uint64_t(uintptr_t(y)),
                               uint64_t(n), uint64_t(uintptr_t(alpha)), uint64_t(uintptr_t(ws)),
                               uint64_t(tcap), uint64_t(uintptr_t(s)), uint64_t(nblk)};
  for (double v : {C, eps, tau}) {
    key.push_back(__builtin_bit_cast(uint64_t, v));
  }
  key.push_back(uint64_t(max_iter));
  if (!ctx->smo_exec || ctx->smo_key != key) {
    ctx->release_graph();
    SVMD_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int it = 0; it < kChunk; ++it) {
      hipLaunchKernelGGL(smo_select_kernel, dim3(nblk), dim3(kSelectThreads), 0, s, K, ldk, y, alpha, f, n,
                         st, part, C, eps);
      hipLaunchKernelGGL(smo_step_kernel, dim3(1), dim3(256), 0, s, part, nblk, K, ldk, y, alpha, n, st, C,
                         eps, tau, max_iter, dtrace, tcap);
    }
    hipGraph_t graph;
    SVMD_CHECK(hipStreamEndCapture(s, &graph));
    hipGraphExec_t exec;
    SVMD_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    ctx->smo_exec = exec;
    ctx->smo_graph = graph;
    ctx->smo_key = key;
  }

  // Replay with two chunks in flight; poll the stop flag of the older one.
  SmoState* hst = static_cast<SmoState*>(ctx->pinned);  // [0], [1] poll slots, [2] final
  hst[0].stop = hst[1].stop = 0;
  hipEvent_t ev[2];
  SVMD_CHECK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
  SVMD_CHECK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  const int64_t max_replays = max_iter / kChunk + 4;
  int rc_loop = SVM_OK;
  auto enqueue = [&](int slot) -> int {
    SVMD_CHECK(hipGraphLaunch(ctx->smo_exec, s));
    SVMD_CHECK(hipMemcpyAsync(&hst[slot], st, sizeof(SmoState), hipMemcpyDeviceToHost, s));
    SVMD_CHECK(hipEventRecord(ev[slot], s));
    return SVM_OK;
  };
  rc_loop = enqueue(0);
  for (int64_t rep = 0; rc_loop == SVM_OK; ++rep) {
    if (rep + 1 < max_replays) rc_loop = enqueue(int((rep + 1) & 1));
    if (rc_loop) break;
    hipError_t e = hipEventSynchronize(ev[rep & 1]);
    if (e != hipSuccess) {
      set_error("svmd_smo: %s", hipGetErrorString(e));
      rc_loop = SVM_ERR_DEVICE;
      break;
    }
    if (hst[rep & 1].stop || rep + 1 >= max_replays) break;
  }
  hipError_t e = hipStreamSynchronize(s);
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  if (rc_loop) return rc_loop;
  if (e != hipSuccess) {
    set_error("svmd_smo: %s", hipGetErrorString(e));
    return SVM_ERR_DEVICE;
  }
  SVMD_CHECK(hipMemcpy(&hst[2], st, sizeof(SmoState), hipMemcpyDeviceToHost));
  return finish_smo(hst[2], r, trace, dtrace, tcap, t0);
}

namespace {
template <int NT, int E>
void launch_multi_e(hipStream_t s, int grid, const double* K, int64_t ldk, const int32_t* Y, double* A, double* F,
                    int64_t n, unsigned long long* slots, SmoState* st, int nclass, const svm_params& p, unsigned* ctl,
                    int G) {
  const size_t lds = xcd_lds_pad(NT);
  if (p.wss == 2) {  // opt-in second-order selection: the same persist_solve as the single-class solver
    allow_lds(smo_multi_kernel<NT, E, true>, lds);
    hipLaunchKernelGGL((smo_multi_kernel<NT, E, true>), dim3(grid), dim3(NT), lds, s, K, ldk, Y, A, F, n,
                       int64_t(NT) * E, slots, st, nclass, p.C, p.eps, p.tau, p.max_iter, ctl, int64_t(1) << 22, G,
                       register_ticks());
    return;
  }
  allow_lds(smo_multi_kernel<NT, E>, lds);
  hipLaunchKernelGGL((smo_multi_kernel<NT, E>), dim3(grid), dim3(NT), lds, s, K, ldk, Y, A, F, n, int64_t(NT) * E,
                     slots, st, nclass, p.C, p.eps, p.tau, p.max_iter, ctl, int64_t(1) << 22, G, register_ticks());
}
}  // namespace

int run_smo_multi(DeviceCtx* ctx, const double* K, int64_t ldk, const int32_t* Y, int64_t n, int nclass, double* A,
                  const svm_params& p, svm_result* r, int32_t* batched) {
  if (n <= 0 || nclass <= 0) {
    set_error("svmd_smo_multi: empty problem");
    return SVM_ERR_EMPTY;
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = ctx->stream;
  std::vector<SmoState> fin(static_cast<size_t>(nclass));
  int G = 0, E = 0, NT = 0;
  bool ok = nclass < 1000 && n < int64_t(kSentinel) && persistent_grid(n, &G, &E, &NT, kXcdMaxG);
  ok = ok && ((NT == 256 && E <= 2) || (NT == 512 && E <= 4));
  if (const char* v = getenv("SVM355_SMO_MULTI"); v && atoi(v) == 0) ok = false;
  if (batched) *batched = 0;
  if (ok) {
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t total = size_t(nclass) * size_t(n);
    const size_t off_f = 0;
    const size_t off_st = off_f + al(total * 8);
    const size_t off_slots = off_st + al(size_t(nclass) * sizeof(SmoState));
    const size_t slot_bytes = size_t(kMultiTeams) * 2 * kMaxG * kRecStride * 8;
    const size_t off_ctl = off_slots + al(slot_bytes);
    int rc = ctx->ensure_ws(off_ctl + al(kMultiCtlWords * 4));
    if (rc) return rc;
    char* ws = static_cast<char*>(ctx->ws);
    double* F = reinterpret_cast<double*>(ws + off_f);
    SmoState* st = reinterpret_cast<SmoState*>(ws + off_st);
    auto* slots = reinterpret_cast<unsigned long long*>(ws + off_slots);
    auto* ctl = reinterpret_cast<unsigned*>(ws + off_ctl);
    const int64_t init_n = std::max<int64_t>(int64_t(total), nclass);
    hipLaunchKernelGGL(smo_multi_init_kernel, dim3(unsigned((init_n + 255) / 256)), dim3(256), 0, s, Y, A, F,
                       int64_t(total), st, nclass);
    SVMD_LAUNCH_CHECK();
    SVMD_CHECK(hipMemsetAsync(ws + off_slots, 0, al(slot_bytes) + al(kMultiCtlWords * 4), s));
    // Over-provisioned grid as for the single XCD-local solve: ~2*G workgroups per XCD.
    const int grid = 16 * G;
#define SVM_MULTI_CASE(nt, e) \
  else if (NT == nt && E == e) launch_multi_e<nt, e>(s, grid, K, ldk, Y, A, F, n, slots, st, nclass, p, ctl, G);
    if (false) {
    }
    SVM_MULTI_CASE(256, 1) SVM_MULTI_CASE(256, 2) SVM_MULTI_CASE(512, 1) SVM_MULTI_CASE(512, 2)
    SVM_MULTI_CASE(512, 4)
#undef SVM_MULTI_CASE
    SVMD_LAUNCH_CHECK();
    unsigned herr = 0;
    SVMD_CHECK(hipMemcpyAsync(fin.data(), st, size_t(nclass) * sizeof(SmoState), hipMemcpyDeviceToHost, s));
    SVMD_CHECK(hipMemcpyAsync(&herr, ctl + kMultiErr, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    SVMD_CHECK(hipStreamSynchronize(s));
    if (const char* v = getenv("SVM355_SMO_MULTI_DEBUG"); v && atoi(v)) {
      unsigned hc[kMultiCtlWords];
      SVMD_CHECK(hipMemcpy(hc, ctl, sizeof(hc), hipMemcpyDeviceToHost));
      fprintf(stderr, "[smo_multi G=%d NT=%d E=%d] per XCD landed/decision:", G, NT, E);
      for (int x = 0; x < kMultiTeams; ++x) fprintf(stderr, " %u/%u", hc[4 * x], hc[4 * x + 1]);
      fprintf(stderr, " | queue %u err %u\n", hc[kMultiQueue], hc[kMultiErr]);
    }
    if (herr == 1) {
      set_error("svmd_smo_multi: a team timed out waiting for a workgroup record or its mailbox");
      return SVM_ERR_DEVICE;
    }
    if (batched) *batched = 1;
  }
  // Classes no team solved (batched path off or unavailable, or teams that could not form): one by one.
  for (int k = 0; k < nclass; ++k) {
    if (ok && fin[size_t(k)].stop != SVM_STOP_RUNNING) {
      const int rc = finish_smo(fin[size_t(k)], r ? &r[k] : nullptr, nullptr, nullptr, 0, t0);
      if (rc) return rc;
      continue;
    }
    const int rc = run_smo(ctx, K, ldk, Y + int64_t(k) * n, n, A + int64_t(k) * n, 0, p, r ? &r[k] : nullptr,
                           nullptr, 0);
    if (rc) return rc;
  }
  return SVM_OK;
}

namespace {
// counts[r] = #{i < n : alpha[r*n + i] > tol}; grid (x: row chunks, y: rows).
__global__ __launch_bounds__(256) void count_above_kernel(const double* __restrict__ alpha, int64_t n, double tol,
                                                          unsigned long long* __restrict__ counts) {
  const int64_t r = blockIdx.y;
  const double* a = alpha + r * n;
  unsigned c = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    c += a[i] > tol ? 1u : 0u;
  // wave64 sum, then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(counts + r, (unsigned long long)c);
}
}  // namespace

int count_sv(DeviceCtx* ctx, const double* alpha, int64_t n, int64_t rows, double tol, int64_t* out) {
  if (n <= 0 || rows <= 0) {
    for (int64_t r = 0; r < rows; ++r) out[r] = 0;
    return SVM_OK;
  }
  hipStream_t s = ctx->stream;
  constexpr int64_t kMaxRows = 1024;
  if (rows > kMaxRows) {
    set_error("count_sv: %lld rows (max %lld)", (long long)rows, (long long)kMaxRows);
    return SVM_ERR_ARG;
  }
  if (!ctx->count_d) SVMD_CHECK(hipMalloc(&ctx->count_d, kMaxRows * 8));
  int rc = ctx->ensure_pinned(size_t(kMaxRows) * 8);
  if (rc) return rc;
  SVMD_CHECK(hipMemsetAsync(ctx->count_d, 0, size_t(rows) * 8, s));
  const unsigned bx = unsigned(std::min<int64_t>((n + 255) / 256, 256));
  hipLaunchKernelGGL(count_above_kernel, dim3(bx, unsigned(rows)), dim3(256), 0, s, alpha, n, tol, ctx->count_d);
  SVMD_LAUNCH_CHECK();
  auto* h = static_cast<unsigned long long*>(ctx->pinned);
  SVMD_CHECK(hipMemcpyAsync(h, ctx->count_d, size_t(rows) * 8, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  for (int64_t r = 0; r < rows; ++r) out[r] = int64_t(h[r]);
  return SVM_OK;
}

}  // namespace svm355
