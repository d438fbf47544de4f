// Working-set decomposition SMO (decomp.hip): shapes and the host driver, shared by the one-GPU C ABI
// (svmd_train_decomp_u8) and the distributed solve over a cascade group or process rank
// (cascade_dev.hip: svmd_cascade_group_decomp / svmd_cascade_rank_decomp).
#pragma once
#include <cstdint>
#include <functional>
#include <mutex>
#include <vector>

#include "ctx.h"

namespace svm355 {

// Selection shape for n points: NB blocks of `per` points, T candidates per side per block, L = 2 NB T
// gathered candidates (<= 1024), q the working-set capacity.
struct DecompShape {
  bool ok = false;
  int q = 0, T = 0;
  int64_t NB = 0, per = 0, L = 0;
};
DecompShape decomp_shape(int64_t n, int qws, int world);

// All-gather of `bytes` from every GPU into recv (world * bytes, GPU-major), ordered on the solver's
// stream (the distributed solve's one exchange per outer iteration), and optionally the wait for an
// event recorded on that stream (true: waited under the transport's deadline / abort policy; false /
// empty: the solver waits for it itself).
struct DecompAllGather {
  std::function<void(const void* send, int64_t bytes, void* recv)> gather;
  std::function<bool(void* event)> wait;
  explicit operator bool() const { return bool(gather); }
};

// One-GPU rehearsal of P ranks with every rank's device work timed alone (SVM355_CASCADE_SERIAL_SOLVES=1,
// as the cascade rehearsal's solves): the ranks sharing the device take `mu` around each of their two
// device segments per outer iteration -- the selection (before the candidate all-gather) and the rest
// (build, K(W, W), inner solve, f update) -- and time them with events, so the P-GPU critical path is
// sum over outer iterations of max over ranks of each segment (exchanges excluded).
struct DecompSolo {
  std::mutex* mu = nullptr;
  std::vector<double> sel_ms, rest_ms;  // per outer iteration of this rank
};

// How a solve runs beyond its problem: the distributed form (world > 1: this GPU's rank and the
// candidate all-gather), a warm start (alpha holds the start; f = K (alpha y) - y over its nonzero
// entries), and an optional per-outer-iteration trace (tests; one GPU only, one synchronisation per
// outer iteration).
struct DecompOpts {
  int world = 1, rank = 0;
  DecompAllGather allgather;
  bool warm = false;
  svm_decomp_trace* trace = nullptr;
  DecompSolo* solo = nullptr;  // world > 1 rehearsal on one GPU: per-rank solo timing (above)
  double* host_wait_ms = nullptr;  // out: host time blocked in the per-batch waits (all outer iterations)
};

// The rows a solve reads its kernel values from: the exact-integer plan's quantised rows (Q; int8
// MFMA, igram.hip) or the min-max scaled FP64 rows themselves (X, n x ld, ld a multiple of 16, and
// their squared norms nrm; FP64 MFMA, gram_mfma.hip) -- the latter for real-valued data.
struct DecompRows {
  const int8_t* Q = nullptr;
  const int32_t* N0 = nullptr;
  const double* WN = nullptr;
  const double* stw = nullptr;  // the plan's step weights, on the device
  const QuantPlan* P = nullptr;
  const double* X = nullptr;
  const double* nrm = nullptr;
  int64_t ld = 0;
  bool fp64() const { return X != nullptr; }
};

// stats: SVM_DECOMP_STATS int64 (see run_decomp).
constexpr int kDecompStats = SVM_DECOMP_STATS;
int run_decomp(DeviceCtx* ctx, const DecompRows& R, const int32_t* y, double* alpha, int64_t n, const svm_params& p,
               int qws, svm_result* r, int64_t* stats, const DecompOpts& o = {});

// Quantise the device uint8 rows (all n) into the context's grow-only buffer and run the solve.
// *used = false (nothing done) when the rows' statistics do not admit the exact-integer plan.
// prep_ms: the quantisation's host-side time.
int decomp_fit_u8(DeviceCtx* ctx, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h, const double* mx_h,
                  const int32_t* y_d, double* alpha_d, const svm_params& p, int q, svm_result* r, int64_t* stats,
                  bool* used, double* prep_ms, const DecompOpts& o = {});

// The same from min-max scaled FP64 rows on the device (X_d: n x ld), one GPU: quantised into the
// exact-integer plan when the statistics admit one (the uint8 path's integers), else -- real-valued
// data, or SVM355_DECOMP_F64=1 -- solved on the FP64 rows with FP64-MFMA kernel values (*used = false
// only when ld is not a multiple of 16).
int decomp_fit_rows(DeviceCtx* ctx, const double* X_d, int64_t n, int64_t ld, int64_t d, const double* mn_h,
                    const double* mx_h, const int32_t* y_d, double* alpha_d, const svm_params& p, int q, svm_result* r,
                    int64_t* stats, bool* used, double* prep_ms, const DecompOpts& o = {});

}  // namespace svm355
