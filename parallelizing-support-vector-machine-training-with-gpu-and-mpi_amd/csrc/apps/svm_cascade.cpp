// svm_cascade — the reference's MPI Cascade programs as ONE native process driving P GPUs:
// --topology star = mpi_svm_main2.cpp (modified two-layer), --topology tree = mpi_svm_main3.cpp
// (classical).
//
//   svm_cascade [--topology star|tree] [--gpus P] [--transport auto|rccl|loopback] [--max-rounds R]
//               [--checkpoint-dir D [--resume]]   (per-round state, cascade.h cascade_state.bin)
//               [the svm_gpu options: --dataset | --train/--test | --synthetic N[,M] | --C ... --json F
//                --model-dir D --quiet]
//
// One host thread per rank.  rccl: ncclCommInitAll over GPUs 0..P-1 (one node, no
// bootstrap server), every exchange an RCCL collective over xGMI.  loopback: the ranks share the
// visible GPUs round-robin and exchange through host memory -- rehearsals of any P on one GPU.
// auto = rccl when P GPUs are visible, else loopback.
// Partitioning: contiguous chunks of ceil(N/P) rows with global ids (mpi_svm_main3.cpp:464-518).
// Timing (mpi_svm_main3.cpp:526-773): training = after the data distribution (each rank's H2D of its
// chunk) until convergence; prediction = rank 0 test read, scaling with the training statistics and
// decision over the final SVs with s >= 0 -> +1 (M3 :800).  stdout = the reference's [rank 0] lines.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../cascade/cascade.h"
#include "cli_common.h"
#include "svm355_device.h"

using namespace svm355;

namespace {

void usage(const char* prog) {
  fprintf(stderr,
          "usage: %s [--topology star|tree] [--gpus P] [--transport auto|rccl|loopback] [--max-rounds R]\n"
          "       [--checkpoint-dir D [--resume]]\n"
          "       [svm_gpu options, see svm_gpu --help]\n",
          prog);
}

}  // namespace

int main(int argc, char** argv) {
  std::string topology = "star", transport = "auto";
  int P = 1, max_rounds = 50;
  std::string checkpoint_dir;
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
    else if (a == "--gpus") P = atoi(val().c_str());
    else if (a == "--transport") transport = val();
    else if (a == "--max-rounds") max_rounds = atoi(val().c_str());
    else if (a == "--checkpoint-dir") checkpoint_dir = val();
    else if (a == "--resume") resume = true;
    else if (a == "-h" || a == "--help") {
      usage(argv[0]);
      cli::usage(argv[0]);
      return 0;
    } else rest.push_back(argv[i]);
  }
  cli::Options o;
  if (!cli::parse(int(rest.size()), rest.data(), o, 0)) return 2;
  if ((topology != "star" && topology != "tree") || P < 1 ||
      (transport != "auto" && transport != "rccl" && transport != "loopback")) {
    usage(argv[0]);
    return 2;
  }
  const bool tree = topology == "tree";
  if (tree && (P & (P - 1))) {  // mpi_svm_main3.cpp:420-428 (MPI_Abort)
    fprintf(stderr, "[rank 0] Error: the classical CascadeSVM needs a power-of-2 number of processes, got %d\n", P);
    return 1;
  }
  int32_t ndev = 0;
  svmd_device_count(&ndev);
  if (ndev < 1) {
    fprintf(stderr, "svm_cascade: no HIP device visible\n");
    return 1;
  }
  if (transport == "auto") transport = P <= ndev ? "rccl" : "loopback";
  if (transport == "rccl" && P > ndev) {
    fprintf(stderr, "svm_cascade: --transport rccl needs one GPU per rank (%d ranks, %d GPUs visible)\n", P, ndev);
    return 1;
  }

  cli::Data tr;
  if (!cli::load_split(o, true, tr)) return 1;
  if (tr.n == 0) {
    fprintf(stderr, "Error: No data read from file.\n");
    return 1;
  }
  const int64_t n = tr.n, d = tr.d;

  std::vector<ncclComm_t> comms;
  if (transport == "rccl") {
    comms.resize(size_t(P));
    std::vector<int> devs(static_cast<size_t>(P));
    std::iota(devs.begin(), devs.end(), 0);
    const ncclResult_t rc = ncclCommInitAll(comms.data(), P, devs.data());
    if (rc != ncclSuccess) {
      fprintf(stderr, "svm_cascade: ncclCommInitAll: %s\n", ncclGetErrorString(rc));
      return 1;
    }
  }
  auto group = std::make_shared<LoopbackGroup>(P);
  CascadeConfig cfg;
  cfg.tree = tree;
  cfg.max_rounds = max_rounds;
  cfg.params = o.p;
  cfg.log = true;
  cfg.checkpoint_dir = checkpoint_dir;
  cfg.resume = resume;

  std::vector<CascadeOutput> outs(static_cast<size_t>(P));
  std::vector<void*> ctxs(size_t(P), nullptr);
  std::vector<int> devs(static_cast<size_t>(P));
  const int64_t chunk = (n + P - 1) / P;
  auto body = [&](int r) {
    const int dev = transport == "rccl" ? r : r % ndev;
    devs[size_t(r)] = dev;
    try {
      if (hipSetDevice(dev) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
      void* ctx = svmd_create(dev);
      if (!ctx) throw std::runtime_error(svm_last_error());
      ctxs[size_t(r)] = ctx;
      std::unique_ptr<Transport> t;
      if (transport == "rccl")
        t.reset(new RcclTransport(comms[size_t(r)], dev));
      else
        t.reset(new LoopbackTransport(group, r, dev));
      const int64_t lo = std::min<int64_t>(n, int64_t(r) * chunk), hi = std::min<int64_t>(n, lo + chunk);
      std::vector<int64_t> ids(static_cast<size_t>(hi - lo));
      std::iota(ids.begin(), ids.end(), lo);
      outs[size_t(r)] = run_cascade(*t, ctx, tr.X.data() + lo * d, tr.y.data() + lo, ids.data(), hi - lo, d, n, cfg);
    } catch (const std::exception& e) {
      // MPI_Abort equivalent: the other ranks may be blocked in a collective, so end the job.
      fprintf(stderr, "[rank %d] error: %s\n", r, e.what());
      fflush(stderr);
      fflush(stdout);
      std::_Exit(1);
    }
  };
  std::vector<std::thread> threads;
  for (int r = 0; r < P; ++r) threads.emplace_back(body, r);
  for (auto& th : threads) th.join();

  // ---- prediction scope (rank 0)
  CascadeOutput& R0 = outs[0];
  void* ctx = ctxs[0];
  hipSetDevice(devs[0]);
  const auto t1 = std::chrono::steady_clock::now();
  cli::Data te;
  if (!cli::load_split(o, false, te)) return 1;
  const int64_t m = te.n, ld = svmd_padded_dim(d), nsv = int64_t(R0.ids.size());
  long long correct = 0;
  auto ck = [](int rc) {
    if (rc != SVM_OK) {
      fprintf(stderr, "%s\n", svm_last_error());
      exit(1);
    }
  };
  if (m > 0) {
    std::vector<void*> bufs;
    auto alloc = [&](int64_t bytes) {
      void* p = svmd_alloc(ctx, bytes);
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
    ck(svmd_memcpy_h2d(ctx, mn, R0.mn.data(), d * 8));
    ck(svmd_memcpy_h2d(ctx, mx, R0.mx.data(), d * 8));
    ck(svmd_upload_rows(ctx, te.X.data(), m, d, Xq, ld));
    ck(svmd_preprocess(ctx, Xq, m, d, ld, mn, mx, nq, 1));
    const int64_t ns = std::max<int64_t>(nsv, 1);
    auto* nsq = static_cast<double*>(alloc(ns * 8));
    auto* coef = static_cast<double*>(alloc(ns * 8));
    std::vector<double> ch(size_t(ns), 0.0);
    for (int64_t k = 0; k < nsv; ++k) ch[size_t(k)] = R0.alpha[size_t(k)] * R0.y[size_t(k)];
    if (nsv > 0) {
      ck(svmd_row_norms(ctx, R0.X_d, nsv, d, ld, nsq));
      ck(svmd_memcpy_h2d(ctx, coef, ch.data(), nsv * 8));
    }
    ck(svmd_decision(ctx, nsv ? R0.X_d : nullptr, nsv ? nsq : nullptr, nsv ? coef : nullptr, nsv, ld, Xq, nq, m, ld,
                     ld, o.p.gamma, R0.b, out));
    // s >= 0 -> +1 (M3 :800), counted on the device
    auto* yq = static_cast<int32_t*>(alloc(m * 4));
    ck(svmd_memcpy_h2d(ctx, yq, te.y.data(), m * 4));
    int64_t c = 0;
    ck(svmd_count_correct(ctx, out, yq, m, 1, &c));
    correct = c;
    for (void* p : bufs) svmd_free(ctx, p);
    printf("[rank 0] Test accuracy (final model) = %g (%lld/%lld)\n", double(correct) / double(m), correct,
           (long long)m);
  } else {
    printf("[rank 0] No test data found or test file empty.\n");
  }
  const auto t2 = std::chrono::steady_clock::now();
  const double pred_ms = cli::ms_between(t1, t2);
  printf("[rank 0] Final global SV count = %lld\n", (long long)nsv);
  printf("[rank 0] Cascade finished in %d rounds\n", R0.rounds);
  printf("[rank 0] training time = %d ms\n", int(R0.train_ms));
  printf("[rank 0] prediction time = %d ms\n", int(pred_ms));
  printf("[rank 0] elapsed time = %d ms\n", int(R0.train_ms + pred_ms));
  if (!o.quiet)
    fprintf(stderr, "[svm_cascade] transport %s, %lld solves on rank 0, %lld SMO iterations on rank 0\n",
            transport.c_str(), (long long)R0.solves, (long long)R0.iterations);
  if (!o.model_dir.empty() &&
      svm_model_save(o.model_dir.c_str(), R0.ids.data(), R0.y.data(), R0.alpha.data(), nsv, R0.b) != SVM_OK)
    fprintf(stderr, "%s\n", svm_last_error());
  if (!o.json.empty()) {
    FILE* f = fopen(o.json.c_str(), "w");
    if (f) {
      auto list_i = [&](const std::vector<int64_t>& v) {
        std::string s = "[";
        for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + std::to_string(v[i]);
        return s + "]";
      };
      std::string rms = "[";
      for (size_t i = 0; i < R0.round_ms.size(); ++i) {
        char b[32];
        snprintf(b, sizeof(b), "%s%.3f", i ? ", " : "", R0.round_ms[i]);
        rms += b;
      }
      rms += "]";
      std::vector<int64_t> sorted_ids = R0.ids;
      std::sort(sorted_ids.begin(), sorted_ids.end());
      fprintf(f,
              "{\"program\": \"svm_cascade (%s)\", \"transport\": \"%s\", \"world\": %d, \"n\": %lld, \"rounds\": %d, "
              "\"converged\": %s, \"n_sv\": %lld, \"b\": %.17g, \"train_ms\": %.3f, \"prediction_ms\": %.3f, "
              "\"test_correct\": %lld, \"test_m\": %lld, \"sv_history\": %s, \"merged_history\": %s, \"round_ms\": %s, "
              "\"rank0_solves\": %lld, \"rank0_iterations\": %lld, \"sv_ids\": %s}\n",
              topology.c_str(), transport.c_str(), P, (long long)n, R0.rounds, R0.converged ? "true" : "false",
              (long long)nsv, R0.b, R0.train_ms, pred_ms, correct, (long long)m, list_i(R0.sv_history).c_str(),
              list_i(R0.merged_history).c_str(), rms.c_str(), (long long)R0.solves, (long long)R0.iterations,
              list_i(sorted_ids).c_str());
      fclose(f);
    }
  }
  for (int r = 0; r < P; ++r) {
    if (outs[size_t(r)].X_d) svmd_free(ctxs[size_t(r)], outs[size_t(r)].X_d);
    if (ctxs[size_t(r)]) svmd_destroy(ctxs[size_t(r)]);
  }
  for (auto c : comms) ncclCommDestroy(c);
  return 0;
}
