// svm_cascade — the reference's MPI Cascade programs as ONE native process driving P GPUs:
// --topology star = mpi_svm_main2.cpp (modified two-layer), --topology tree = mpi_svm_main3.cpp
// (classical).
//
//   svm_cascade [--topology star|tree] [--gpus P] [--transport auto|rccl|loopback] [--max-rounds R]
//               [--checkpoint-dir D [--resume]]   (per-round state, cascade.h cascade_state.bin)
//               [--comm-timeout S] [--fail-rank R --fail-round K]   (fault injection)
//               [the svm_gpu options: --dataset | --train/--test | --synthetic N[,M] | --C ... --json F
//                --model-dir D --quiet]
//
// One host thread per rank through svmd_cascade_group_*: rccl = ncclCommInitAll over
// GPUs 0..P-1 (one node, no bootstrap server), every exchange an RCCL collective over xGMI;
// loopback = the ranks share the visible GPUs and exchange through host memory (rehearsals of any P
// on one GPU).  auto = rccl when P GPUs are visible, else loopback.
// Partitioning: contiguous chunks of ceil(N/P) rows with global ids (mpi_svm_main3.cpp:464-518).
// Timing (mpi_svm_main3.cpp:526-773): training = after the data distribution (each rank's H2D of its
// chunk) until convergence; prediction = rank 0 test read, scaling with the training statistics and
// decision over the final SVs with s >= 0 -> +1 (M3 :800).  stdout = the reference's [rank 0] lines.
// A failed rank aborts every communicator (the MPI_Abort of M3 :426, :453) and the exit status is 1.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cli_common.h"
#include "svm355_device.h"

namespace {

void usage(const char* prog) {
  fprintf(stderr,
          "usage: %s [--topology star|tree] [--gpus P] [--transport auto|rccl|loopback] [--max-rounds R]\n"
          "       [--checkpoint-dir D [--resume]] [--comm-timeout S] [--fail-rank R --fail-round K]\n"
          "       [svm_gpu options, see svm_gpu --help]\n",
          prog);
}

std::string list_i(const int64_t* v, int64_t n) {
  std::string s = "[";
  for (int64_t i = 0; i < n; ++i) s += (i ? ", " : "") + std::to_string(v[i]);
  return s + "]";
}

}  // namespace

int main(int argc, char** argv) {
  std::string topology = "star", transport = "auto", checkpoint_dir;
  int P = 1, max_rounds = 50, fail_rank = -1, fail_round = -1;
  double timeout = 600.0;
  bool resume = false;
  std::vector<char*> rest{argv[0]};
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--topology") topology = val();
    else if (a == "--gpus") P = int(cli::parse_int("--gpus", val().c_str()));
    else if (a == "--transport") transport = val();
    else if (a == "--max-rounds") max_rounds = int(cli::parse_int("--max-rounds", val().c_str()));
    else if (a == "--checkpoint-dir") checkpoint_dir = val();
    else if (a == "--resume") resume = true;
    else if (a == "--comm-timeout") timeout = cli::parse_num("--comm-timeout", val().c_str());
    else if (a == "--fail-rank") fail_rank = int(cli::parse_int("--fail-rank", val().c_str()));
    else if (a == "--fail-round") fail_round = int(cli::parse_int("--fail-round", val().c_str()));
    else if (a == "-h" || a == "--help") {
      usage(argv[0]);
      cli::usage(argv[0]);
      return 0;
    } else rest.push_back(argv[i]);
  }
  cli::Options o;
  if (!cli::parse(int(rest.size()), rest.data(), o, 0)) return 2;
  if ((topology != "star" && topology != "tree") || P < 1 || max_rounds < 1 || !(timeout > 0) ||
      (transport != "auto" && transport != "rccl" && transport != "loopback")) {
    usage(argv[0]);
    return 2;
  }
  const bool tree = topology == "tree";
  if (tree && (P & (P - 1))) {  // mpi_svm_main3.cpp:420-428 (MPI_Abort)
    fprintf(stderr, "[rank 0] Error: the classical CascadeSVM needs a power-of-2 number of processes, got %d\n", P);
    return 1;
  }
  cli::Data tr;
  if (!cli::load_split(o, true, tr)) return 1;
  if (tr.n == 0) {
    fprintf(stderr, "Error: No data read from file.\n");
    return 1;
  }
  void* group = svmd_cascade_group_create(P, transport.c_str(), timeout);
  if (!group) {
    fprintf(stderr, "svm_cascade: %s\n", svm_last_error());
    return 1;
  }
  svm_cascade_cfg cfg;
  svm_cascade_default_cfg(&cfg);
  cfg.tree = tree ? 1 : 0;
  cfg.max_rounds = max_rounds;
  cfg.params = o.p;
  cfg.log = 1;
  cfg.resume = resume ? 1 : 0;
  cfg.checkpoint_dir = checkpoint_dir.empty() ? nullptr : checkpoint_dir.c_str();
  cfg.comm_timeout_s = timeout;
  cfg.fail_rank = fail_rank;
  cfg.fail_round = fail_round;
  cfg.solver = o.solver;  // --solver auto (default: per solve) | decomp | smo
  svm_cascade_out* R = svmd_cascade_group_fit(group, tr.X.data(), 0, tr.y.data(), tr.n, tr.d, &cfg);
  if (!R) {
    fprintf(stderr, "[rank 0] error: %s\n", svm_last_error());
    fflush(stdout);
    svmd_cascade_group_destroy(group);
    return 1;
  }

  // ---- prediction scope (rank 0, GPU 0)
  const auto t1 = std::chrono::steady_clock::now();
  cli::Data te;
  if (!cli::load_split(o, false, te)) return 1;
  const int64_t m = te.n, d = tr.d, ld = svmd_padded_dim(d), nsv = R->n_sv;
  long long correct = 0;
  auto ck = [](int rc) {
    if (rc != SVM_OK) {
      fprintf(stderr, "%s\n", svm_last_error());
      exit(1);
    }
  };
  if (m > 0) {
    void* ctx = svmd_create(0);
    if (!ctx) {
      fprintf(stderr, "%s\n", svm_last_error());
      return 1;
    }
    std::vector<void*> bufs;
    auto alloc = [&](int64_t bytes) {
      void* p = svmd_alloc(ctx, std::max<int64_t>(bytes, 8));
      if (!p) {
        fprintf(stderr, "%s\n", svm_last_error());
        exit(1);
      }
      bufs.push_back(p);
      return p;
    };
    auto* Xq = static_cast<double*>(alloc(m * ld * 8));
    auto* nq = static_cast<double*>(alloc(m * 8));
    auto* out = static_cast<double*>(alloc(m * 8));
    auto* mn = static_cast<double*>(alloc(d * 8));
    auto* mx = static_cast<double*>(alloc(d * 8));
    ck(svmd_memcpy_h2d(ctx, mn, R->mn, d * 8));
    ck(svmd_memcpy_h2d(ctx, mx, R->mx, d * 8));
    ck(svmd_upload_rows(ctx, te.X.data(), m, d, Xq, ld));
    ck(svmd_preprocess(ctx, Xq, m, d, ld, mn, mx, nq, 1));
    const int64_t ns = std::max<int64_t>(nsv, 1);
    auto* Xs = static_cast<double*>(alloc(ns * ld * 8));
    auto* nsq = static_cast<double*>(alloc(ns * 8));
    auto* coef = static_cast<double*>(alloc(ns * 8));
    std::vector<double> ch(size_t(ns), 0.0);
    for (int64_t k = 0; k < nsv; ++k) ch[size_t(k)] = R->alpha[k] * R->y[k];
    if (nsv > 0) {
      ck(svmd_upload_rows(ctx, R->sv_rows, nsv, d, Xs, ld));  // already scaled
      ck(svmd_row_norms(ctx, Xs, nsv, d, ld, nsq));
      ck(svmd_memcpy_h2d(ctx, coef, ch.data(), nsv * 8));
    }
    ck(svmd_decision(ctx, nsv ? Xs : nullptr, nsv ? nsq : nullptr, nsv ? coef : nullptr, nsv, ld, Xq, nq, m, ld, ld,
                     o.p.gamma, R->b, out));
    auto* yq = static_cast<int32_t*>(alloc(m * 4));
    ck(svmd_memcpy_h2d(ctx, yq, te.y.data(), m * 4));
    int64_t c = 0;
    ck(svmd_count_correct(ctx, out, yq, m, 1, &c));  // s >= 0 -> +1 (M3 :800), counted on the device
    correct = c;
    for (void* p : bufs) svmd_free(ctx, p);
    svmd_destroy(ctx);
    printf("[rank 0] Test accuracy (final model) = %g (%lld/%lld)\n", double(correct) / double(m), correct,
           (long long)m);
  } else {
    printf("[rank 0] No test data found or test file empty.\n");
  }
  const auto t2 = std::chrono::steady_clock::now();
  const double pred_ms = cli::ms_between(t1, t2);
  printf("[rank 0] Final global SV count = %lld\n", (long long)nsv);
  printf("[rank 0] Cascade finished in %d rounds\n", R->rounds);
  printf("[rank 0] training time = %d ms\n", int(R->train_ms));
  printf("[rank 0] prediction time = %d ms\n", int(pred_ms));
  printf("[rank 0] elapsed time = %d ms\n", int(R->train_ms + pred_ms));
  int64_t r0_solves = 0, r0_iters = 0;
  for (int64_t i = 0; i < R->n_solves; ++i)
    if (R->solves[SVM_CASCADE_SOLVE_COLS * i] == 0.0) {
      ++r0_solves;
      r0_iters += int64_t(R->solves[SVM_CASCADE_SOLVE_COLS * i + 4]);
    }
  if (!o.quiet)
    fprintf(stderr, "[svm_cascade] transport %s, %lld solves on rank 0, %lld SMO iterations on rank 0\n", R->transport,
            (long long)r0_solves, (long long)r0_iters);
  if (!o.model_dir.empty() && svm_model_save(o.model_dir.c_str(), R->ids, R->y, R->alpha, nsv, R->b) != SVM_OK)
    fprintf(stderr, "%s\n", svm_last_error());
  if (!o.json.empty()) {
    FILE* f = fopen(o.json.c_str(), "w");
    if (f) {
      std::string rms = "[";
      for (int64_t i = 0; i < R->n_hist; ++i) {
        char b[32];
        snprintf(b, sizeof(b), "%s%.3f", i ? ", " : "", R->round_ms[i]);
        rms += b;
      }
      rms += "]";
      std::vector<int64_t> sorted_ids(R->ids, R->ids + nsv);
      std::sort(sorted_ids.begin(), sorted_ids.end());
      fprintf(f,
              "{\"program\": \"svm_cascade (%s)\", \"transport\": \"%s\", \"world\": %d, \"n\": %lld, \"rounds\": %d, "
              "\"converged\": %s, \"n_sv\": %lld, \"b\": %.17g, \"train_ms\": %.3f, \"prediction_ms\": %.3f, "
              "\"test_correct\": %lld, \"test_m\": %lld, \"sv_history\": %s, \"merged_history\": %s, \"round_ms\": %s, "
              "\"rank0_solves\": %lld, \"rank0_iterations\": %lld, \"sv_ids\": %s}\n",
              topology.c_str(), R->transport, P, (long long)tr.n, R->rounds, R->converged ? "true" : "false",
              (long long)nsv, R->b, R->train_ms, pred_ms, correct, (long long)m,
              list_i(R->sv_history, R->n_hist).c_str(), list_i(R->merged_history, R->n_merged).c_str(), rms.c_str(),
              (long long)r0_solves, (long long)r0_iters, list_i(sorted_ids.data(), nsv).c_str());
      fclose(f);
    }
  }
  svm_cascade_free(R);
  svmd_cascade_group_destroy(group);
  return 0;
}
