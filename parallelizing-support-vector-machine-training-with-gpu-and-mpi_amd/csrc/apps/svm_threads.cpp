// svm_threads: the threaded host code of the library run end to end, for the sanitizer builds
// (python -m svm355.build --sanitize: bin_asan/svm_threads with ASan + UBSan, bin_tsan/svm_threads with
// TSan; tests/test_sanitized.py).  SURVEY §5.2: the reference has no race detection at all; its MPI
// ranks are processes (mpi_svm_main3.cpp:414-845).  Ours are threads wherever a test or a rehearsal
// runs several ranks in one process, so every one of these paths must be race- and UB-free:
//
//   cascade   star P = 2 / 3 / 8, tree P = 2 / 4 / 8 over the strict loopback transport (rank threads
//             exchanging through LoopbackGroup: collectives, rendezvous sends, the deadlock graph);
//   hostcomm  the same driver over HostCommTransport (hostcomm.cpp), its callbacks served by loopback
//             ranks in threads -- the per-process transport's code with threads as the "processes";
//   abort     a rank failing mid-round: every rank leaves its exchange, the token carries the reason;
//   resume    a one-round checkpoint, then a resumed fit equal to the uninterrupted one;
//   decomp    the decomposition oracle with an 8-thread worker team, its distributed form on 8 loopback
//             thread ranks and on 4 hostcomm ranks, and a rank failing mid-solve.
//
// Usage: svm_threads [--n N] [--quick]; exit 0 when every scenario met its expectation (each prints one
// line), 1 otherwise.  Sanitizer reports make the process exit non-zero on their own.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <memory>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "cascade_capi.h"
#include "svm355.h"

using namespace svm355;

namespace {

int g_fail = 0;

void report(const char* what, bool ok, const std::string& detail = "") {
  std::printf("%-44s %s%s%s\n", what, ok ? "ok" : "FAILED", detail.empty() ? "" : "  ", detail.c_str());
  std::fflush(stdout);
  if (!ok) ++g_fail;
}

struct Data {
  int64_t n = 0, d = 784;
  std::vector<double> X;  // raw pixel rows (the cascade scales them itself)
  std::vector<int32_t> y;
};

Data make_data(int64_t n, uint64_t seed) {
  Data D;
  D.n = n;
  D.X.resize(size_t(n * D.d));
  std::vector<int32_t> lab(static_cast<size_t>(n));
  if (svm_synth_mnist(seed, 0, n, D.X.data(), lab.data(), 2) != SVM_OK) std::abort();
  D.y.resize(size_t(n));
  for (int64_t i = 0; i < n; ++i) D.y[size_t(i)] = lab[size_t(i)] == 1 ? 1 : -1;
  return D;
}

svm_cascade_cfg base_cfg(bool tree) {
  svm_cascade_cfg c;
  svm_cascade_default_cfg(&c);
  c.tree = tree ? 1 : 0;
  c.log = 0;
  c.params.n_threads = 1;
  c.comm_timeout_s = 60.0;
  return c;
}

struct Fit {
  bool ok = false;
  std::string err;
  double b = 0.0;
  int rounds = 0;
  std::vector<int64_t> ids;
};

Fit take(svm_cascade_out* o) {
  Fit f;
  if (!o) {
    f.err = svm_last_error();
    return f;
  }
  f.ok = true;
  f.b = o->b;
  f.rounds = o->rounds;
  f.ids.assign(o->ids, o->ids + o->n_sv);
  svm_cascade_free(o);
  return f;
}

// ---- svm_host_comm callbacks served by a loopback rank (ctx = its LoopbackTransport)
LoopbackTransport* T(void* c) { return static_cast<LoopbackTransport*>(c); }
template <class F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (...) {
    return 1;
  }
}
int cb_bcast(void* c, void* buf, int64_t bytes, int32_t root) { return guarded([&] { T(c)->bcast(buf, bytes, root); }); }
int cb_allgather(void* c, const void* s, int64_t bytes, void* r) { return guarded([&] { T(c)->allgather(s, bytes, r); }); }
int cb_allreduce(void* c, double* buf, int64_t n, int32_t op) {
  return guarded([&] { op == 0 ? T(c)->allreduce_min(buf, n) : T(c)->allreduce_max(buf, n); });
}
int cb_gather(void* c, const void* s, int64_t bytes, void* r, int32_t root) {
  return guarded([&] { T(c)->gather(s, bytes, r, root); });
}
int cb_send(void* c, const void* buf, int64_t bytes, int32_t peer) { return guarded([&] { T(c)->send(buf, bytes, peer); }); }
int cb_recv(void* c, void* buf, int64_t bytes, int32_t peer) { return guarded([&] { T(c)->recv(buf, bytes, peer); }); }
int cb_barrier(void* c) { return guarded([&] { T(c)->barrier(); }); }

// P thread "processes", each a HostCommTransport over its loopback rank; fn(rank, comm) per thread.
void hostcomm_ranks(int P, const std::function<void(int, const svm_host_comm&)>& fn) {
  auto token = std::make_shared<AbortToken>();
  auto lg = std::make_shared<LoopbackGroup>(P, WaitPolicy{token, 60.0});
  auto be = make_cpu_backend();
  std::vector<std::unique_ptr<LoopbackTransport>> lt;
  for (int r = 0; r < P; ++r) lt.push_back(std::make_unique<LoopbackTransport>(lg, r, be.get()));
  run_rank_threads(
      P, token,
      [&](int r) {
        svm_host_comm c{lt[size_t(r)].get(), r, P, cb_bcast, cb_allgather, cb_allreduce, cb_gather,
                        cb_send,            cb_recv, cb_barrier};
        fn(r, c);
      },
      [&](int) {});
}

// ---------------------------------------------------------------------------------- scenarios
void cascades(const Data& D, bool quick) {
  const std::vector<std::pair<bool, int>> runs =
      quick ? std::vector<std::pair<bool, int>>{{false, 3}, {true, 4}}
            : std::vector<std::pair<bool, int>>{{false, 2}, {false, 3}, {false, 8}, {true, 2}, {true, 4}, {true, 8}};
  for (auto [tree, P] : runs) {
    const svm_cascade_cfg c = base_cfg(tree);
    const Fit f = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n, D.d, P, &c));
    const std::string name = std::string("cascade loopback ") + (tree ? "tree" : "star") + " P=" + std::to_string(P);
    report(name.c_str(), f.ok && f.rounds >= 1 && !f.ids.empty(), f.ok ? "rounds " + std::to_string(f.rounds) : f.err);

    // the same cascade over HostCommTransport: the per-process transport's code, bit-identical
    std::vector<Fit> hf(static_cast<size_t>(P));
    bool ok = true;
    std::string err;
    try {
      hostcomm_ranks(P, [&](int r, const svm_host_comm& comm) {
        int64_t lo = 0, hi = 0;
        const std::vector<int64_t> ids = partition_ids(D.n, P, r, &lo, &hi);
        hf[size_t(r)] = take(svm_cascade_rank_fit_cpu(&comm, D.X.data() + lo * D.d, D.y.data() + lo, ids.data(),
                                                      hi - lo, D.d, D.n, &c));
        if (!hf[size_t(r)].ok) throw CascadeError(hf[size_t(r)].err);
      });
    } catch (const std::exception& e) {
      ok = false;
      err = e.what();
    }
    const std::string hname = std::string("cascade hostcomm ") + (tree ? "tree" : "star") + " P=" + std::to_string(P);
    report(hname.c_str(), ok && hf[0].ok && hf[0].b == f.b && hf[0].ids == f.ids, err);
  }
}

void abort_mid_round(const Data& D) {
  svm_cascade_cfg c = base_cfg(false);
  c.fail_rank = 2;
  c.fail_round = 1;
  const auto t0 = std::chrono::steady_clock::now();
  const Fit f = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n, D.d, 4, &c));
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  report("cascade abort mid-round (rank 2, round 1)", !f.ok && f.err.find("rank 2") != std::string::npos && s < 50,
         f.err.substr(0, 90));
  c = base_cfg(true);
  c.fail_rank = 1;
  c.fail_round = 1;
  bool ok = false;
  std::string err;
  try {
    hostcomm_ranks(4, [&](int r, const svm_host_comm& comm) {
      int64_t lo = 0, hi = 0;
      const std::vector<int64_t> ids = partition_ids(D.n, 4, r, &lo, &hi);
      const Fit h = take(svm_cascade_rank_fit_cpu(&comm, D.X.data() + lo * D.d, D.y.data() + lo, ids.data(), hi - lo,
                                                  D.d, D.n, &c));
      if (!h.ok) throw CascadeError(h.err);
    });
  } catch (const std::exception& e) {
    err = e.what();
    ok = err.find("injected failure") != std::string::npos;
  }
  report("cascade hostcomm abort mid-round (tree)", ok, err.substr(0, 90));
}

void resume(const Data& D) {
  namespace fs = std::filesystem;
  const fs::path dir = fs::temp_directory_path() / ("svm_threads_ck_" + std::to_string(::getpid()));
  fs::create_directories(dir);
  const std::string ds = dir.string();
  svm_cascade_cfg c = base_cfg(false);
  const Fit full = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n, D.d, 2, &c));
  c.checkpoint_dir = ds.c_str();
  c.max_rounds = 1;
  const Fit part = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n, D.d, 2, &c));
  c.max_rounds = 50;
  c.resume = 1;
  const Fit res = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n, D.d, 2, &c));
  fs::remove_all(dir);
  report("cascade checkpoint + resume (star P=2)", full.ok && part.ok && res.ok && res.b == full.b && res.ids == full.ids,
         res.ok ? "" : res.err);
}

// Degenerate partitions: rows sorted by label, 8 ranks, so every partition holds one class and no rank
// has a support vector (rank 0's gather of the empty sets once read past its id lists), and more ranks
// than rows (empty partitions); a resume on other rows is refused.
void degenerate(const Data& D) {
  Data S;
  S.n = 24;
  S.d = D.d;
  S.X.assign(D.X.begin(), D.X.begin() + S.n * S.d);
  S.y.resize(size_t(S.n));
  for (int64_t i = 0; i < S.n; ++i) S.y[size_t(i)] = i < S.n / 2 ? 1 : -1;
  for (bool tree : {false, true}) {
    const svm_cascade_cfg c = base_cfg(tree);
    const Fit f = take(svm_cascade_fit_cpu(S.X.data(), S.y.data(), S.n, S.d, 8, &c));
    report(tree ? "cascade tree P=8, one class per partition" : "cascade star P=8, one class per partition",
           f.ok && f.ids.empty(), f.ok ? "" : f.err);
    const Fit g = take(svm_cascade_fit_cpu(S.X.data(), S.y.data(), 5, S.d, 8, &c));
    report(tree ? "cascade tree P=8 on 5 rows (empty partitions)" : "cascade star P=8 on 5 rows (empty partitions)",
           g.ok, g.ok ? "" : g.err);
  }
  namespace fs = std::filesystem;
  const fs::path dir = fs::temp_directory_path() / ("svm_threads_fp_" + std::to_string(::getpid()));
  const std::string ds = dir.string();
  svm_cascade_cfg c = base_cfg(false);
  c.checkpoint_dir = ds.c_str();
  c.max_rounds = 1;
  const Fit part = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n, D.d, 2, &c));
  c.max_rounds = 50;
  c.resume = 1;
  const Fit other = take(svm_cascade_fit_cpu(D.X.data(), D.y.data(), D.n - 5, D.d, 2, &c));
  fs::remove_all(dir);
  report("cascade resume on other rows is refused", part.ok && !other.ok &&
                                                       other.err.find("another training set") != std::string::npos,
         other.err.substr(0, 90));
}

void decomp(int64_t n) {
  Data D = make_data(n, 11);
  std::vector<double> mn(size_t(D.d)), mx(size_t(D.d));
  svm_minmax(D.X.data(), D.n, D.d, mn.data(), mx.data());
  svm_scale(D.X.data(), D.n, D.d, mn.data(), mx.data());
  std::vector<double> K(size_t(D.n * D.n));
  svm_rbf_matrix(D.X.data(), D.n, D.X.data(), D.n, D.d, 0.00125, K.data(), 8);
  svm_params p;
  svm_default_params(&p);
  p.n_threads = 8;
  std::vector<double> a1(size_t(D.n)), a8(size_t(D.n)), ah(size_t(D.n));
  svm_result r1{}, r8{};
  int64_t st[SVM_DECOMP_STATS];
  const int rc1 = svm_decomp_train_gram(K.data(), D.n, D.y.data(), D.n, a1.data(), 0, &p, 1024, 0.1, 3, &r1, st, nullptr);
  report("decomp oracle, 8-thread worker team", rc1 == SVM_OK && r1.stop_reason == SVM_STOP_CONVERGED,
         rc1 ? svm_last_error() : "iterations " + std::to_string(r1.iterations));
  p.n_threads = 2;
  const int rc8 = svm_decomp_group_train_gram(8, K.data(), D.n, D.y.data(), D.n, a8.data(), 0, &p, 1024, 0.1, 3, &r8,
                                              st, 60.0);
  report("decomp distributed, 8 loopback thread ranks", rc8 == SVM_OK && a8 == a1 && r8.b == r1.b,
         rc8 ? svm_last_error() : "");
  bool ok = true;
  std::string err;
  try {
    hostcomm_ranks(4, [&](int r, const svm_host_comm& comm) {
      std::vector<double> a(size_t(D.n));
      svm_result rr{};
      if (svm_decomp_rank_train_gram(&comm, K.data(), D.n, D.y.data(), D.n, a.data(), 0, &p, 1024, 0.1, 3, &rr,
                                     nullptr) != SVM_OK)
        throw CascadeError(svm_last_error());
      if (r == 0) ah = a;
      if (a != a1 || rr.b != r1.b) throw CascadeError("rank " + std::to_string(r) + ": differs from the one-rank solve");
    });
  } catch (const std::exception& e) {
    ok = false;
    err = e.what();
  }
  report("decomp distributed, 4 hostcomm ranks", ok && ah == a1, err);
  setenv("SVM355_DECOMP_FAIL_RANK", "3", 1);
  setenv("SVM355_DECOMP_FAIL_OUTER", "2", 1);
  const int rcf = svm_decomp_group_train_gram(4, K.data(), D.n, D.y.data(), D.n, a8.data(), 0, &p, 1024, 0.1, 3, &r8,
                                              st, 60.0);
  const std::string ef = rcf ? svm_last_error() : "";
  unsetenv("SVM355_DECOMP_FAIL_RANK");
  unsetenv("SVM355_DECOMP_FAIL_OUTER");
  report("decomp rank failing mid-solve", rcf != SVM_OK && ef.find("injected failure of rank 3") != std::string::npos,
         ef.substr(0, 90));
}

void exercise() {
  double el = 0.0;
  for (int P : {2, 4, 8}) {
    const int rc = svm_loopback_exercise(P, preflight_script(P, 1 << 16).c_str(), 1, 20.0, &el);
    report(("strict loopback preflight script P=" + std::to_string(P)).c_str(), rc == SVM_OK,
           rc ? svm_last_error() : "");
  }
  const int rc2 = svm_loopback_exercise(2, "r:8<1|r:8<0", 1, 20.0, &el);
  report("strict loopback names a deadlock", rc2 != SVM_OK && std::string(svm_last_error()).find("deadlock") !=
                                                                  std::string::npos,
         std::string(svm_last_error()).substr(0, 90));
}

}  // namespace

int main(int argc, char** argv) {
  int64_t n = 600;
  bool quick = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--n") && i + 1 < argc) n = std::atoll(argv[++i]);
    if (!std::strcmp(argv[i], "--quick")) quick = true;
  }
  const Data D = make_data(n, 7);
  exercise();
  cascades(D, quick);
  abort_mid_round(D);
  resume(D);
  degenerate(D);
  decomp(std::max<int64_t>(n, 600));
  std::printf("%s\n", g_fail ? "SOME SCENARIOS FAILED" : "ALL SCENARIOS OK");
  return g_fail ? 1 : 0;
}
