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
#include <chrono>
#include <vector>

#include "ctx.h"

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

// Warm start, step 1: ascending list of j with alpha_j != 0 (single workgroup, ballot compaction).
__global__ __launch_bounds__(1024) void nonzero_compact_kernel(const double* __restrict__ alpha, int64_t n,
                                                               int64_t* __restrict__ idx,
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
    if (nz) idx[off + __popcll(m & ((1ull << lane) - 1ull))] = i;
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
// (mpi_svm_main3.cpp:169-186; column access K[j][i] is coalesced across i).
__global__ __launch_bounds__(256) void warm_f_kernel(const double* __restrict__ K, int64_t ldk,
                                                     const int32_t* __restrict__ y,
                                                     const double* __restrict__ alpha,
                                                     const int64_t* __restrict__ idx,
                                                     const int64_t* __restrict__ count,
                                                     double* __restrict__ f, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t cnt = *count;
  double sum = 0.0;
  for (int64_t k = 0; k < cnt; ++k) {
    const int64_t j = idx[k];
    sum += alpha[j] * double(y[j]) * K[j * ldk + i];
  }
  f[i] = sum - static_cast<double>(y[i]);
}

}  // namespace

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
  const size_t off_cnt = off_idx + al(size_t(n) * 8);
  const size_t off_trace = off_cnt + al(8);
  const size_t total = off_trace + al(size_t(tcap) * 16);
  int rc = ctx->ensure_ws(total);
  if (rc) return rc;
  rc = ctx->ensure_pinned(sizeof(SmoState) * 3);
  if (rc) return rc;
  char* ws = static_cast<char*>(ctx->ws);
  double* f = reinterpret_cast<double*>(ws + off_f);
  Partial* part = reinterpret_cast<Partial*>(ws + off_part);
  SmoState* st = reinterpret_cast<SmoState*>(ws + off_state);
  int64_t* idx = reinterpret_cast<int64_t*>(ws + off_idx);
  int64_t* cnt = reinterpret_cast<int64_t*>(ws + off_cnt);
  int64_t* dtrace = tcap ? reinterpret_cast<int64_t*>(ws + off_trace) : nullptr;

  if (!warm) {
    hipLaunchKernelGGL(smo_init_cold_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, y, alpha, f,
                       n, st);
    SVMD_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(nonzero_compact_kernel, dim3(1), dim3(1024), 0, s, alpha, n, idx, cnt, st);
    SVMD_LAUNCH_CHECK();
    hipLaunchKernelGGL(warm_f_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, K, ldk, y, alpha,
                       idx, cnt, f, n);
    SVMD_LAUNCH_CHECK();
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
  const SmoState fin = hst[2];
  if (!fin.stop) {
    set_error("svmd_smo: solver did not stop within the replay budget");
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

}  // namespace svm355
