// Native Cascade SVM driver (one host thread per rank, device solves on the rank's GPU).
//
// Both topologies of the reference, with its round structure, warm starts, ID de-duplication and
// ID-set convergence test:
//   tree  classical Cascade, mpi_svm_main3.cpp:565-828 (power-of-two P; layers step = 1, 2, ..., P)
//   star  modified two-layer Cascade, mpi_svm_main2.cpp:439-769 (any P; gather to rank 0, whose
//         merge keeps its own alphas and resets the workers' to 0, :600-601)
// Same semantics -- and, on the same device solver, the same bits -- as the Python driver
// svm355/parallel/cascade.py; this one needs no Python and drives RCCL directly.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "svm355.h"
#include "transport.h"

namespace svm355 {

struct CascadeConfig {
  bool tree = false;    // false = star (modified two-layer)
  int max_rounds = 50;  // mpi_svm_main3.cpp:544, mpi_svm_main2.cpp:428
  svm_params params{};  // C, gamma, tau, eps, sv_tol, max_iter
  bool log = true;      // rank 0 prints the reference's per-round lines
  // Per-round checkpoint: rank 0 writes <checkpoint_dir>/cascade_state.bin after every
  // round (global SV set with alphas, b, next round); resume = start from that file if present.
  std::string checkpoint_dir;
  bool resume = false;
};

// cascade_state.bin layout (little-endian): char magic[8] = "SVM355C1"; int32 topology (0 star,
// 1 tree); int32 reserved; int64 next_round; double b; int64 d; int64 ld; int64 k; then k records of
// ld + 3 doubles [scaled row (ld, zero padded) | y | alpha | global id].
constexpr char kCheckpointMagic[9] = "SVM355C1";

struct CascadeOutput {
  // Final global SV set (every rank holds it after the final broadcast).
  std::vector<int64_t> ids;
  std::vector<int32_t> y;
  std::vector<double> alpha;
  double* X_d = nullptr;  // nsv x ld scaled rows on the rank's device; the caller frees it (svmd_free)
  double b = 0.0;
  int rounds = 0;
  bool converged = false;
  std::vector<int64_t> sv_history, merged_history;
  std::vector<double> round_ms;
  double train_ms = 0.0;
  std::vector<double> mn, mx;  // global column min / max the rows were scaled with
  int64_t solves = 0, iterations = 0;
};

// Train on this rank's partition: X_host (n_part x d raw rows), labels +-1, global sample ids.
// ctx: this rank's svmd device context.  Throws TransportError / std::runtime_error on failure.
CascadeOutput run_cascade(Transport& t, void* ctx, const double* X_host, const int32_t* y_host,
                          const int64_t* ids_host, int64_t n_part, int64_t d, int64_t n_total,
                          const CascadeConfig& cfg);

}  // namespace svm355
