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
#include "persist.h"
#include "qrows.h"

namespace svm355 {
namespace {

constexpr int kSelectThreads = 256;
constexpr int kChunk = 128;  // SMO iterations per graph replay


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
// ascending j per point (the reference's order); the wave-uniform idx / coef loads are read U
// at a time and the U column loads issued before the adds consume them, so each group costs
// one memory round trip instead of a dependent chain per term.  64-thread blocks spread a
// cascade-sized n over many CUs.
// PIPE: the next group's loads are issued before the current group's adds (2 U loads in flight).
template <int U, bool PIPE>
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
  if constexpr (PIPE) {
    double kv[U], c[U];
    if (U <= cnt) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c[u] = coef[u];
        kv[u] = K[idx[u] * ldk + ic];
      }
    }
    for (; k + U <= cnt; k += U) {
      double kn[U], cn[U];
      const bool more = k + 2 * U <= cnt;  // wave-uniform
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cn[u] = coef[k + U + u];
          kn[u] = K[idx[k + U + u] * ldk + ic];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) sum += c[u] * kv[u];
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          c[u] = cn[u];
          kv[u] = kn[u];
        }
      }
    }
  } else {
    for (; k + U <= cnt; k += U) {
      double kv[U], c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c[u] = coef[k + u];
        kv[u] = K[idx[k + u] * ldk + ic];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) sum += c[u] * kv[u];
    }
  }
  for (; k < cnt; ++k) sum += coef[k] * K[idx[k] * ldk + ic];
  if (i < n) f[i] = sum - static_cast<double>(y[i]);
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
    // SVM355_WARM_U = 8 (one group of 8 in flight) | 16 | 32 (two groups in flight, pipelined)
    int wu = 16;
    if (const char* v = getenv("SVM355_WARM_U")) wu = atoi(v);
    const dim3 wg(unsigned((n + 63) / 64));
    if (wu == 8)
      hipLaunchKernelGGL((warm_f_kernel<8, false>), wg, dim3(64), 0, s, K, ldk, y, idx, coef, cnt, f, n);
    else if (wu == 32)
      hipLaunchKernelGGL((warm_f_kernel<32, true>), wg, dim3(64), 0, s, K, ldk, y, idx, coef, cnt, f, n);
    else
      hipLaunchKernelGGL((warm_f_kernel<16, true>), wg, dim3(64), 0, s, K, ldk, y, idx, coef, cnt, f, n);
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

SVMD_TU_WARM(smo)
