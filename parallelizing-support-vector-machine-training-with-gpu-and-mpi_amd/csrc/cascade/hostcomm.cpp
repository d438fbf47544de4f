// HostCommTransport: one cascade rank per PROCESS on the CPU oracle backend, exchanging through
// collectives the caller supplies as C callbacks (svm_host_comm, svm355.h) -- in practice a
// torch.distributed gloo group (svm355.parallel.hostcomm).  It is the CPU twin of the per-process
// RCCL rank (svmd_cascade_rank_fit, cascade_dev.hip): the same run_cascade, the same per-process
// bootstrap shape as a torchrun launch of bench.py, so multi-process CPU tests cover that path.
//
// The reference's MPI call sites map onto the callbacks exactly as onto RcclTransport (cascade.h):
// scalar broadcasts / count all-gathers ride on 8-byte bcast / allgather, min/max on allreduce_f64,
// the star gather on gather, the tree pairs on send / recv.  Every callback returns 0 on success;
// anything else (the caller's group timed out, a peer died) becomes a TransportError, and the rank
// leaves run_cascade with an error instead of waiting.
#include <cstring>

#include "../core/internal.h"
#include "cascade_capi.h"

namespace svm355 {
namespace {

class HostCommTransport final : public Transport {
 public:
  explicit HostCommTransport(const svm_host_comm& c) : c_(c) {}
  int rank() const override { return c_.rank; }
  int world() const override { return c_.world; }
  const char* name() const override { return "hostcomm"; }

  int64_t bcast_i64(int64_t v, int root) override {
    ok(c_.bcast(c_.ctx, &v, 8, root), "bcast(i64)");
    return v;
  }
  std::vector<int64_t> allgather_i64(int64_t v) override {
    std::vector<int64_t> out(size_t(c_.world));
    ok(c_.allgather(c_.ctx, &v, 8, out.data()), "allgather(i64)");
    return out;
  }
  void allreduce_min(double* buf, int64_t n) override { ok(c_.allreduce_f64(c_.ctx, buf, n, 0), "allreduce(min)"); }
  void allreduce_max(double* buf, int64_t n) override { ok(c_.allreduce_f64(c_.ctx, buf, n, 1), "allreduce(max)"); }
  void bcast(void* buf, int64_t bytes, int root) override {
    if (bytes > 0) ok(c_.bcast(c_.ctx, buf, bytes, root), "bcast");
  }
  void gather(const void* send, int64_t bytes, void* recv, int root) override {
    if (bytes > 0) ok(c_.gather(c_.ctx, send, bytes, c_.rank == root ? recv : nullptr, root), "gather");
  }
  void send_i64(int64_t v, int peer) override { ok(c_.send(c_.ctx, &v, 8, peer), "send(i64)"); }
  int64_t recv_i64(int peer) override {
    int64_t v = 0;
    ok(c_.recv(c_.ctx, &v, 8, peer), "recv(i64)");
    return v;
  }
  void send(const void* buf, int64_t bytes, int peer) override {
    if (bytes > 0) ok(c_.send(c_.ctx, buf, bytes, peer), "send");
  }
  void recv(void* buf, int64_t bytes, int peer) override {
    if (bytes > 0) ok(c_.recv(c_.ctx, buf, bytes, peer), "recv");
  }
  void barrier() override { ok(c_.barrier(c_.ctx), "barrier"); }

 private:
  static void ok(int rc, const char* what) {
    if (rc != 0) throw TransportError(std::string("hostcomm ") + what + " failed (rc " + std::to_string(rc) + ")");
  }
  svm_host_comm c_;
};

}  // namespace
}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API svm_cascade_out* svm_cascade_rank_fit_cpu(const svm_host_comm* comm, const double* X, const int32_t* y,
                                                  const int64_t* ids, int64_t n_part, int64_t d, int64_t n_total,
                                                  const svm_cascade_cfg* c) {
  if (!comm || comm->world < 1 || comm->rank < 0 || comm->rank >= comm->world || !comm->bcast || !comm->allgather ||
      !comm->allreduce_f64 || !comm->gather || !comm->send || !comm->recv || !comm->barrier || n_part < 0 || d <= 0 ||
      (n_part && (!X || !y || !ids))) {
    set_error("svm_cascade_rank_fit_cpu: bad arguments");
    return nullptr;
  }
  try {
    const CascadeConfig cfg = config_from(c);
    HostCommTransport t(*comm);
    auto be = make_cpu_backend();
    const CascadeOutput o = run_cascade(t, *be, X, false, y, ids, n_part, d, n_total, cfg);
    return build_cascade_out({&o}, *be, comm->world, comm->rank, "hostcomm", "cpu");
  } catch (const std::exception& e) {
    set_error("cascade: %s", e.what());
    return nullptr;
  }
}

}  // extern "C"
