// L2/L3 for problems whose n x n Gram does not fit in HBM (n > ~180k on one MI355X): SMO with an
// HBM-resident kernel-row cache filled on demand.
//
// Reference: the reference never stores the Gram; it keeps the last i_high / i_low rows and
// recomputes a row (calc_kernel_matrix, gpu_svm_main3.cu:137-147, :394-411) whenever the pair
// changes.  Here rows live in a 2-way set-associative LRU cache of C slots (C x n doubles, sized
// from the free HBM, held by the device context), and the host is never involved per iteration.
//
// Default solver: smo.hip's persistent row-cache kernel (run_smo_rc_persistent: one launch, the
// directory replicated in every workgroup's LDS, misses filled per workgroup slice from the
// chunk-interleaved quantised rows built here), for n <= 1,048,576.  Beyond its shapes (or with
// SVM355_RC_SMO=graph) one SMO iteration = two kernels of a replayed hipGraph:
//
//   kc_select  f += ch*row(ih) + cl*row(il) for the previous pair — each row read from its cache
//              slot or, on a miss, computed here for every column and stored into the slot (the
//              fill is fused into this grid-wide pass) — then the masked argmin/argmax partials
//              (the smo_select_kernel arithmetic);
//   kc_step    final reduction, stop tests, K12 computed directly, the two-variable update, and
//              the cache directory (2-way sets, LRU clock): slots and miss flags of (ih, il).
//
// Kernel values come from the quantised rows with EXACTLY the arithmetic of the exact-integer
// Gram kernel (igram.hip: int32 group cross terms, group-ordered FP64 flushes, the same dist and
// exp expressions), so the trajectory is bit-identical to the full-Gram solver.  Feature data that
// are not integer-valued use the FP64 expression ||a||^2 + ||b||^2 - 2 a.b instead.
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ctx.h"
#include "qrows.h"

namespace svm355 {
namespace {

constexpr int kNT = 256;
constexpr int kKcChunk = 64;
constexpr int64_t kNone = INT64_MAX;

struct KcState {
  int64_t ih, il;  // pair of the last update
  int64_t sh, sl;  // cache slots holding rows ih / il
  double ch, cl;
  double b_high, b_low;
  int64_t num_iter;
  int64_t clock;
  int32_t pending, stop;
  int32_t miss_h, miss_l;
};

struct KcPartial {
  double vmin;
  int64_t imin;
  double vmax;
  int64_t imax;
};

// Chunk-interleaved copy of the quantised rows (QRows::Qt): thread (c, i) moves 16-byte chunk c of
// row i; consecutive threads write consecutive rows of one chunk.
__global__ void interleave_rows_kernel(const int8_t* __restrict__ Q, int64_t n, int kq, int8_t* __restrict__ Qt) {
  const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t nc = kq / 16;
  if (idx >= n * nc) return;
  const int64_t c = idx / n, i = idx - c * n;
  reinterpret_cast<int4*>(Qt)[c * n + i] = reinterpret_cast<const int4*>(Q + i * int64_t(kq))[c];
}

__global__ void kc_init_cold_kernel(const int32_t* __restrict__ y, double* __restrict__ alpha, double* __restrict__ f,
                                    int64_t n, KcState* st) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) {
    alpha[i] = 0.0;
    f[i] = -static_cast<double>(y[i]);
  }
  if (i == 0) *st = KcState{0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, 0, SVM_STOP_RUNNING, 0, 0};
}

// Warm start: f_i = sum_{alpha_j != 0, ascending j} alpha_j y_j K(j, i) - y_i (mpi_svm_main3.cpp:169-186),
// kernel values computed on the fly (same summation order as smo.hip's warm_f_kernel).
template <bool INT>
__global__ __launch_bounds__(kNT) void kc_warm_f_kernel(QRows q, const int32_t* __restrict__ y,
                                                        const double* __restrict__ alpha,
                                                        const int64_t* __restrict__ idx, int64_t cnt,
                                                        double* __restrict__ f, int64_t n, double neg_gamma,
                                                        KcState* st) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i == 0) *st = KcState{0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, 0, SVM_STOP_RUNNING, 0, 0};
  if (i >= n) return;
  double sum = 0.0;
  for (int64_t k = 0; k < cnt; ++k) {
    const int64_t j = idx[k];
    sum += alpha[j] * double(y[j]) * kval<INT>(q, j, i, neg_gamma);
  }
  f[i] = sum - static_cast<double>(y[i]);
}

template <bool INT>
__global__ __launch_bounds__(kNT) void kc_select_kernel(QRows q, double* __restrict__ cache, int64_t ldc,
                                                        const int32_t* __restrict__ y,
                                                        const double* __restrict__ alpha, double* __restrict__ f,
                                                        int64_t n, const KcState* __restrict__ st,
                                                        KcPartial* __restrict__ part, double C, double eps,
                                                        double neg_gamma) {
  if (st->stop) return;
  const int32_t pending = st->pending;
  const double ch = st->ch, cl = st->cl;
  // Rows of the pending pair: cached, or (miss) computed here for every column and stored into
  // the slot the step kernel assigned — the fill is fused into this pass over n.
  const int32_t mh = pending ? st->miss_h : 0, ml = pending ? st->miss_l : 0;
  const int64_t ih = st->ih, il = st->il;
  double* Kh = cache + st->sh * ldc;
  double* Kl = cache + st->sl * ldc;
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  double hv = __builtin_inf(), lv = -__builtin_inf();
  int64_t hi = kNone, li = kNone;
  const int64_t stride = int64_t(gridDim.x) * kNT;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += stride) {
    double fi = f[i];
    if (pending) {
      double kh, kl;
      if (mh) {
        kh = kval<INT>(q, ih, i, neg_gamma);
        Kh[i] = kh;
      } else {
        kh = Kh[i];
      }
      if (ml) {
        kl = kval<INT>(q, il, i, neg_gamma);
        Kl[i] = kl;
      } else {
        kl = Kl[i];
      }
      fi += ch * kh + cl * kl;  // main3.cpp:274 operation order
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
  __shared__ KcPartial sp[kNT / kWave];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sp[w] = KcPartial{hv, hi, lv, li};
  __syncthreads();
  if (threadIdx.x == 0) {
    KcPartial r = sp[0];
    for (int k = 1; k < kNT / kWave; ++k) {
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

// 2-way set-associative LRU lookup; returns the slot and whether the row must be filled.  `keep` is
// a slot that must not be evicted (the other row of this iteration's pair).
__device__ __forceinline__ int64_t kc_lookup(int64_t row, int64_t nsets, int64_t* tags, int64_t* stamp,
                                             int64_t clock, int64_t keep, int32_t* miss) {
  const int64_t s0 = 2 * (row % nsets), s1 = s0 + 1;
  if (tags[s0] == row) {
    stamp[s0] = clock;
    *miss = 0;
    return s0;
  }
  if (tags[s1] == row) {
    stamp[s1] = clock;
    *miss = 0;
    return s1;
  }
  int64_t v = stamp[s0] <= stamp[s1] ? s0 : s1;
  if (v == keep) v = v == s0 ? s1 : s0;
  tags[v] = row;
  stamp[v] = clock;
  *miss = 1;
  return v;
}

template <bool INT>
__global__ __launch_bounds__(kNT) void kc_step_kernel(const KcPartial* __restrict__ part, int nparts, QRows q,
                                                      const int32_t* __restrict__ y, double* __restrict__ alpha,
                                                      int64_t n, KcState* __restrict__ st, int64_t* __restrict__ tags,
                                                      int64_t* __restrict__ stamp, int64_t nsets, double C,
                                                      double eps, double tau, double neg_gamma, int64_t max_iter,
                                                      int64_t* __restrict__ trace, int64_t trace_cap) {
  if (st->stop) return;
  double hv = __builtin_inf(), lv = -__builtin_inf();
  int64_t hi = kNone, li = kNone;
  for (int k = threadIdx.x; k < nparts; k += blockDim.x) {
    const KcPartial p = part[k];
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
  __shared__ KcPartial sp[kNT / kWave];
  __shared__ int32_t sdot[128];  // exact int32 cross term of each 32-column k-step of (i_high, i_low)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sp[w] = KcPartial{hv, hi, lv, li};
  __syncthreads();
  // Every thread merges the per-wave partials (same inputs, same order -> the same pair everywhere).
  hv = sp[0].vmin;
  hi = sp[0].imin;
  lv = sp[0].vmax;
  li = sp[0].imax;
  for (int k = 1; k < kNT / kWave; ++k) {
    if (better_min(hv, hi, sp[k].vmin, sp[k].imin)) {
      hv = sp[k].vmin;
      hi = sp[k].imin;
    }
    if (better_max(lv, li, sp[k].vmax, sp[k].imax)) {
      lv = sp[k].vmax;
      li = sp[k].imax;
    }
  }
  // K12 of the exact-integer path: one k-step per thread (the integer sums are exact, so the
  // group-ordered FP64 flushes below reproduce kval() bit for bit) instead of one thread walking
  // all kq columns -- that serial dot product was most of this kernel's ~15 us.
  const bool need_k12 = INT && hi < n && li < n && hi != li && !(lv <= hv + 2.0 * tau);  // block-uniform
  if (need_k12) {
    const int nsteps = q.kq / 32;
    if (int(threadIdx.x) < nsteps) {
      const int4* pa = reinterpret_cast<const int4*>(q.Q + hi * int64_t(q.kq)) + 2 * threadIdx.x;
      const int4* pb = reinterpret_cast<const int4*>(q.Q + li * int64_t(q.kq)) + 2 * threadIdx.x;
      const int4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
      int32_t acc = 0;
      acc = __builtin_amdgcn_sdot4(a0.x, b0.x, acc, false);
      acc = __builtin_amdgcn_sdot4(a0.y, b0.y, acc, false);
      acc = __builtin_amdgcn_sdot4(a0.z, b0.z, acc, false);
      acc = __builtin_amdgcn_sdot4(a0.w, b0.w, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.x, b1.x, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.y, b1.y, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.z, b1.z, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.w, b1.w, acc, false);
      sdot[threadIdx.x] = acc;
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  st->miss_h = st->miss_l = 0;
  if (hi >= n || li >= n) {  // main3.cpp:205-209
    st->pending = 0;
    st->stop = SVM_STOP_NO_CANDIDATE;
    return;
  }
  const double bh = hv, bl = lv;
  st->b_high = bh;
  st->b_low = bl;
  if (bl <= bh + 2.0 * tau) {
    st->pending = 0;
    st->stop = SVM_STOP_CONVERGED;
    return;
  }
  const int32_t yh = y[hi], yl = y[li];
  const double K11 = kval<INT>(q, hi, hi, neg_gamma), K22 = kval<INT>(q, li, li, neg_gamma);
  double K12;
  if (need_k12) {  // kval<true>(q, hi, li) from the per-step sums, same operation order
    int32_t acc = 0;
    double x = 0.0;
    for (int st_k = 0; st_k < q.kq / 32; ++st_k) {
      acc += sdot[st_k];
      if (st_k < q.main_step0) {
        const double wg = q.step_w[st_k];
        if (wg != 0.0) {
          x = __builtin_fma(wg, double(acc), x);
          acc = 0;
        }
      }
    }
    const int32_t D0 = q.N0[hi] + q.N0[li] - 2 * acc;
    double dist = q.w0 * double(D0);
    if (q.main_step0 > 0) dist += (q.WN[hi] + q.WN[li]) - 2.0 * x;
    dist = dist > 0.0 ? dist : 0.0;
    K12 = exp(neg_gamma * dist);
  } else {
    K12 = kval<INT>(q, hi, li, neg_gamma);
  }
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
  // Cache directory for the rows the next select needs.
  const int64_t clock = st->clock + 1;
  st->clock = clock;
  int32_t mh = 0, ml = 0;
  const int64_t sh = kc_lookup(hi, nsets, tags, stamp, clock, -1, &mh);
  const int64_t sl = li == hi ? sh : kc_lookup(li, nsets, tags, stamp, clock, sh, &ml);
  st->sh = sh;
  st->sl = sl;
  st->miss_h = mh;
  st->miss_l = ml;
  const int64_t it = st->num_iter;
  if (trace && it - 1 < trace_cap) {
    trace[2 * (it - 1)] = hi;
    trace[2 * (it - 1) + 1] = li;
  }
  st->num_iter = it + 1;
  if (it + 1 > max_iter) st->stop = SVM_STOP_MAX_ITER;
}

}  // namespace

// SMO with the on-demand row cache.  X_d: preprocessed rows (n x ld); P: quantisation plan (P.ok ->
// exact-integer rows, else FP64 rows with sqn_d).  cache_bytes: HBM budget for the row cache.
int run_smo_rowcache(DeviceCtx* ctx, const double* X_d, const double* sqn_d, int64_t n, int64_t ld, int64_t d,
                     const QuantPlan& P, const int32_t* y, double* alpha, int32_t warm, const svm_params& p,
                     svm_result* r, size_t cache_bytes, int64_t* trace, int64_t trace_cap, int32_t* used_int) {
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = ctx->stream;
  const int64_t ldc = (n + 1) / 2 * 2;
  int64_t C = int64_t(cache_bytes / (size_t(ldc) * 8));
  C = std::min<int64_t>(C, 2 * ((n + 1) / 2)) / 2 * 2;
  if (C < 4) {
    set_error("row cache: %zu bytes hold fewer than 4 rows of %lld doubles", cache_bytes, (long long)n);
    return SVM_ERR_OOM;
  }
  const int nblk = int(std::min<int64_t>((n + kNT - 1) / kNT, 2048));
  const int64_t tcap = trace ? std::max<int64_t>(trace_cap, 0) : 0;
  std::vector<void*> bufs;
  auto dalloc = [&](size_t bytes) -> void* {
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(bytes, 256)) != hipSuccess) return nullptr;
    bufs.push_back(q);
    return q;
  };
  auto release = [&]() {
    (void)hipStreamSynchronize(s);
    for (void* b : bufs) (void)hipFree(b);
  };
  QRows q{};
  bool int_ok = false;
  if (P.ok) {
    auto* Q = static_cast<int8_t*>(dalloc(size_t(n) * size_t(P.kq)));
    auto* N0 = static_cast<int32_t*>(dalloc(size_t(n) * 4));
    auto* WN = static_cast<double*>(dalloc(size_t(n) * 8));
    auto* stw = static_cast<double*>(dalloc(P.step_w.size() * 8));
    void* aux = dalloc(quantize_aux_bytes(P));
    if (!Q || !N0 || !WN || !stw || !aux) {
      release();
      set_error("row cache: out of device memory for the quantised rows");
      return SVM_ERR_OOM;
    }
    int rc = quantize_rows(s, X_d, n, ld, P, aux, Q, N0, WN, &int_ok);
    if (rc) {
      release();
      return rc;
    }
    if (hipMemcpyAsync(stw, P.step_w.data(), P.step_w.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess) {
      release();
      set_error("row cache: H2D failed");
      return SVM_ERR_DEVICE;
    }
    q.Q = Q;
    q.N0 = N0;
    q.WN = WN;
    q.step_w = stw;
    q.kq = P.kq;
    q.main_step0 = P.main0 / 32;
    q.w0 = P.w0;
  }
  if (!int_ok) {
    if (!sqn_d) {
      release();
      set_error("row cache: FP64 rows need the squared row norms");
      return SVM_ERR_ARG;
    }
    q.X = X_d;
    q.sqn = sqn_d;
    q.ld = ld;
    q.d = d;
  }
  if (used_int) *used_int = int_ok ? 1 : 0;
  auto* f = static_cast<double*>(dalloc(size_t(n) * 8));
  auto* part = static_cast<KcPartial*>(dalloc(size_t(nblk) * sizeof(KcPartial)));
  auto* st = static_cast<KcState*>(dalloc(sizeof(KcState)));
  auto* tags = static_cast<int64_t*>(dalloc(size_t(C) * 8));
  auto* stamp = static_cast<int64_t*>(dalloc(size_t(C) * 8));
  auto* idx = static_cast<int64_t*>(dalloc(size_t(n) * 8));
  auto* dtrace = tcap ? static_cast<int64_t*>(dalloc(size_t(tcap) * 16)) : nullptr;
  double* cache = ctx->ensure_rc_cache(size_t(C) * size_t(ldc) * 8);  // context-held slab
  if (!f || !part || !st || !tags || !stamp || !idx || !cache || (tcap && !dtrace)) {
    release();
    set_error("row cache: out of device memory (cache of %lld rows x %lld)", (long long)C, (long long)n);
    return SVM_ERR_OOM;
  }
  int rc = ctx->ensure_pinned(sizeof(KcState) * 3);
  if (rc) {
    release();
    return rc;
  }
  const double neg_gamma = -p.gamma;
  // tags = -1 (empty), stamps = 0
  (void)hipMemsetAsync(tags, 0xFF, size_t(C) * 8, s);
  (void)hipMemsetAsync(stamp, 0, size_t(C) * 8, s);
  if (!warm) {
    hipLaunchKernelGGL(kc_init_cold_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, y, alpha, f, n, st);
  } else {
    // ascending list of nonzero alphas (host compaction: the warm set is small and this runs once)
    std::vector<double> ah(static_cast<size_t>(n));
    (void)hipMemcpyAsync(ah.data(), alpha, size_t(n) * 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    std::vector<int64_t> nz;
    for (int64_t i = 0; i < n; ++i)
      if (ah[size_t(i)] != 0.0) nz.push_back(i);
    if (!nz.empty()) (void)hipMemcpyAsync(idx, nz.data(), nz.size() * 8, hipMemcpyHostToDevice, s);
    if (int_ok)
      hipLaunchKernelGGL(kc_warm_f_kernel<true>, dim3(unsigned((n + kNT - 1) / kNT)), dim3(kNT), 0, s, q, y, alpha,
                         idx, int64_t(nz.size()), f, n, neg_gamma, st);
    else
      hipLaunchKernelGGL(kc_warm_f_kernel<false>, dim3(unsigned((n + kNT - 1) / kNT)), dim3(kNT), 0, s, q, y, alpha,
                         idx, int64_t(nz.size()), f, n, neg_gamma, st);
    (void)hipStreamSynchronize(s);
  }
  if (hipGetLastError() != hipSuccess) {
    release();
    set_error("row cache: init launch failed");
    return SVM_ERR_DEVICE;
  }
  // Default: the persistent solver (one launch, register-resident state, directory in LDS), whose
  // misses walk each element's quantised row: give it the coalesced interleaved copy.
  if (int_ok) {
    auto* Qt = static_cast<int8_t*>(dalloc(size_t(n) * size_t(q.kq)));
    if (Qt) {
      const int64_t work = n * (q.kq / 16);
      hipLaunchKernelGGL(interleave_rows_kernel, dim3(unsigned((work + 255) / 256)), dim3(256), 0, s, q.Q, n, q.kq,
                         Qt);
      if (hipGetLastError() == hipSuccess) {
        q.Qt = Qt;
        q.n_rows = n;
      }
    }
  }
  const char* vb = getenv("SVM355_RC_VERBOSE");
  const bool verbose = vb && atoi(vb);
  auto ms_since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  if (verbose) (void)hipStreamSynchronize(s);
  const double t_prep = ms_since(t0);
  rc = run_smo_rc_persistent(ctx, q, int_ok, cache, ldc, C, y, alpha, f, n, p, r, trace, tcap);
  if (rc == kRcNotApplicable && p.wss == 2) {
    release();
    set_error("row cache: second-order selection (wss = 2) needs the persistent row-cache solver (exact-integer "
              "rows, n <= 1,048,576)");
    return SVM_ERR_ARG;
  }
  if (rc != kRcNotApplicable) {
    if (verbose)
      fprintf(stderr, "[rowcache n=%lld] cache %lld slots (%.1f GB, slab %.1f GB) | prep (alloc, quantise, interleave) "
              "%.1f ms | persistent solve %.1f ms, %lld iterations\n", (long long)n, (long long)C,
              double(C) * double(ldc) * 8e-9, double(ctx->rc_cache_bytes) * 1e-9, t_prep, ms_since(t0) - t_prep,
              (long long)(r ? r->iterations : -1));
    release();
    return rc;
  }
  const int64_t nsets = C / 2;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int it = 0; e == hipSuccess && it < kKcChunk; ++it) {
    if (int_ok) {
      hipLaunchKernelGGL(kc_select_kernel<true>, dim3(nblk), dim3(kNT), 0, s, q, cache, ldc, y, alpha, f, n, st,
                         part, p.C, p.eps, neg_gamma);
      hipLaunchKernelGGL(kc_step_kernel<true>, dim3(1), dim3(kNT), 0, s, part, nblk, q, y, alpha, n, st, tags, stamp,
                         nsets, p.C, p.eps, p.tau, neg_gamma, p.max_iter, dtrace, tcap);
    } else {
      hipLaunchKernelGGL(kc_select_kernel<false>, dim3(nblk), dim3(kNT), 0, s, q, cache, ldc, y, alpha, f, n, st,
                         part, p.C, p.eps, neg_gamma);
      hipLaunchKernelGGL(kc_step_kernel<false>, dim3(1), dim3(kNT), 0, s, part, nblk, q, y, alpha, n, st, tags,
                         stamp, nsets, p.C, p.eps, p.tau, neg_gamma, p.max_iter, dtrace, tcap);
    }
  }
  hipError_t e2 = hipStreamEndCapture(s, &graph);
  if (e == hipSuccess) e = e2;
  if (e == hipSuccess) e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    release();
    set_error("row cache: graph capture failed: %s", hipGetErrorString(e));
    return SVM_ERR_DEVICE;
  }
  KcState* hst = static_cast<KcState*>(ctx->pinned);
  const int64_t max_replays = p.max_iter / kKcChunk + 4;
  hipEvent_t ev[2];
  (void)hipEventCreateWithFlags(&ev[0], hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&ev[1], hipEventDisableTiming);
  hst[0].stop = hst[1].stop = 0;
  auto enqueue = [&](int slot) {
    hipError_t er = hipGraphLaunch(exec, s);
    if (er == hipSuccess) er = hipMemcpyAsync(&hst[slot], st, sizeof(KcState), hipMemcpyDeviceToHost, s);
    if (er == hipSuccess) er = hipEventRecord(ev[slot], s);
    return er;
  };
  e = enqueue(0);
  for (int64_t rep = 0; e == hipSuccess; ++rep) {
    if (rep + 1 < max_replays) e = enqueue(int((rep + 1) & 1));
    if (e != hipSuccess) break;
    e = hipEventSynchronize(ev[rep & 1]);
    if (e != hipSuccess || hst[rep & 1].stop || rep + 1 >= max_replays) break;
  }
  hipError_t es = hipStreamSynchronize(s);
  if (e == hipSuccess) e = es;
  KcState fin{};
  if (e == hipSuccess) e = hipMemcpy(&fin, st, sizeof(KcState), hipMemcpyDeviceToHost);
  if (e == hipSuccess && tcap) {
    const int64_t nt = std::min<int64_t>(fin.num_iter - 1, tcap);
    if (nt > 0) e = hipMemcpy(trace, dtrace, size_t(nt) * 16, hipMemcpyDeviceToHost);
  }
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  (void)hipGraphExecDestroy(exec);
  (void)hipGraphDestroy(graph);
  release();
  if (e != hipSuccess) {
    set_error("row cache SMO: %s", hipGetErrorString(e));
    return SVM_ERR_DEVICE;
  }
  if (!fin.stop) {
    set_error("row cache SMO: solver did not stop within its budget");
    return SVM_ERR_INTERNAL;
  }
  if (r) {
    r->iterations = fin.num_iter;
    r->b_high = fin.b_high;
    r->b_low = fin.b_low;
    r->b = (fin.b_high + fin.b_low) / 2;
    r->stop_reason = fin.stop;
    r->reserved = 0;
    r->n_sv = -1;
    r->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return SVM_OK;
}

}  // namespace svm355

SVMD_TU_WARM(rowcache)
