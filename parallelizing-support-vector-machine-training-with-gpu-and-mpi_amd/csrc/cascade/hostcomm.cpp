// HostCommTransport: one rank per PROCESS exchanging through collectives the caller supplies as C
// callbacks (svm_host_comm, svm355.h) -- in practice a torch.distributed gloo group
// (svm355.parallel.hostcomm).  Two uses:
//   * the CPU oracle backend (svm_cascade_rank_fit_cpu, svm_decomp_rank_train_gram): buffers are host
//     memory and go to the callbacks as they are -- the CPU twin of the per-process RCCL rank;
//   * a GPU rank without RCCL (svmd_cascade_rank_create_hostcomm, cascade_dev.hip): buffers are device
//     memory, staged through host vectors with the backend's synchronous copies.  This is how one GPU
//     rehearses the per-process launch of the N-GPU run (torchrun, several processes on one device:
//     RCCL refuses two ranks on one GPU) with the same driver code, so the torchrun path of the
//     distributed decomposition solver and of the cascades runs at world > 1 before any RCCL run does.
//
// The reference's MPI call sites map onto the callbacks exactly as onto RcclTransport (cascade.h):
// scalar broadcasts / count all-gathers ride on 8-byte bcast / allgather, min/max on allreduce_f64,
// the star gather on gather, the tree pairs on send / recv, the decomposition's candidate exchange on
// allgather.  Every callback returns 0 on success; anything else (the caller's group timed out, a peer
// died) becomes a TransportError, and the rank leaves the driver with an error instead of waiting.
#include <cstring>

#include "../core/internal.h"
#include "cascade_capi.h"

namespace svm355 {
namespace {

class HostCommTransport final : public Transport {
 public:
  HostCommTransport(const svm_host_comm& c, Backend* staging) : c_(c), mem_(staging) {}
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
  void allreduce_min(double* buf, int64_t n) override { allreduce(buf, n, 0, "allreduce(min)"); }
  void allreduce_max(double* buf, int64_t n) override { allreduce(buf, n, 1, "allreduce(max)"); }
  void bcast(void* buf, int64_t bytes, int root) override {
    if (bytes <= 0) return;
    if (!mem_) return ok(c_.bcast(c_.ctx, buf, bytes, root), "bcast");
    std::vector<char> h(static_cast<size_t>(bytes));
    if (c_.rank == root) mem_->d2h(h.data(), buf, bytes);
    ok(c_.bcast(c_.ctx, h.data(), bytes, root), "bcast");
    if (c_.rank != root) mem_->h2d(buf, h.data(), bytes);
  }
  void gather(const void* send, int64_t bytes, void* recv, int root) override {
    if (bytes <= 0) return;
    const bool me = c_.rank == root;
    if (!mem_) return ok(c_.gather(c_.ctx, send, bytes, me ? recv : nullptr, root), "gather");
    std::vector<char> s(static_cast<size_t>(bytes)), r(me ? size_t(bytes) * size_t(c_.world) : 0);
    mem_->d2h(s.data(), send, bytes);
    ok(c_.gather(c_.ctx, s.data(), bytes, me ? r.data() : nullptr, root), "gather");
    if (me) mem_->h2d(recv, r.data(), int64_t(r.size()));
  }
  void allgather(const void* send, int64_t bytes, void* recv) override {
    if (bytes <= 0) return;
    if (!mem_) return ok(c_.allgather(c_.ctx, send, bytes, recv), "allgather");
    std::vector<char> s(static_cast<size_t>(bytes)), r(size_t(bytes) * size_t(c_.world));
    mem_->d2h(s.data(), send, bytes);  // synchronous on the rank's stream: ordered after the producer
    ok(c_.allgather(c_.ctx, s.data(), bytes, r.data()), "allgather");
    mem_->h2d(recv, r.data(), int64_t(r.size()));
  }
  void send_i64(int64_t v, int peer) override { ok(c_.send(c_.ctx, &v, 8, peer), "send(i64)"); }
  int64_t recv_i64(int peer) override {
    int64_t v = 0;
    ok(c_.recv(c_.ctx, &v, 8, peer), "recv(i64)");
    return v;
  }
  void send(const void* buf, int64_t bytes, int peer) override {
    if (bytes <= 0) return;
    if (!mem_) return ok(c_.send(c_.ctx, buf, bytes, peer), "send");
    std::vector<char> h(static_cast<size_t>(bytes));
    mem_->d2h(h.data(), buf, bytes);
    ok(c_.send(c_.ctx, h.data(), bytes, peer), "send");
  }
  void recv(void* buf, int64_t bytes, int peer) override {
    if (bytes <= 0) return;
    if (!mem_) return ok(c_.recv(c_.ctx, buf, bytes, peer), "recv");
    std::vector<char> h(static_cast<size_t>(bytes));
    ok(c_.recv(c_.ctx, h.data(), bytes, peer), "recv");
    mem_->h2d(buf, h.data(), bytes);
  }
  void barrier() override { ok(c_.barrier(c_.ctx), "barrier"); }

 private:
  void allreduce(double* buf, int64_t n, int op, const char* what) {
    if (n <= 0) return;
    if (!mem_) return ok(c_.allreduce_f64(c_.ctx, buf, n, op), what);
    std::vector<double> h(static_cast<size_t>(n));
    mem_->d2h(h.data(), buf, n * 8);
    ok(c_.allreduce_f64(c_.ctx, h.data(), n, op), what);
    mem_->h2d(buf, h.data(), n * 8);
  }
  static void ok(int rc, const char* what) {
    if (rc != 0) throw TransportError(std::string("hostcomm ") + what + " failed (rc " + std::to_string(rc) + ")");
  }
  svm_host_comm c_;
  Backend* mem_;  // null: buffers are host memory
};

}  // namespace

bool host_comm_valid(const svm_host_comm* c) {
  return c && c->world >= 1 && c->rank >= 0 && c->rank < c->world && c->bcast && c->allgather && c->allreduce_f64 &&
         c->gather && c->send && c->recv && c->barrier;
}

std::unique_ptr<Transport> make_hostcomm_transport(const svm_host_comm& c, Backend* staging) {
  return std::make_unique<HostCommTransport>(c, staging);
}

}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API svm_cascade_out* svm_cascade_rank_fit_cpu(const svm_host_comm* comm, const double* X, const int32_t* y,
                                                  const int64_t* ids, int64_t n_part, int64_t d, int64_t n_total,
                                                  const svm_cascade_cfg* c) {
  if (!host_comm_valid(comm) || n_part < 0 || d <= 0 || (n_part && (!X || !y || !ids))) {
    set_error("svm_cascade_rank_fit_cpu: bad arguments");
    return nullptr;
  }
  try {
    const CascadeConfig cfg = config_from(c);
    auto t = make_hostcomm_transport(*comm, nullptr);
    auto be = make_cpu_backend();
    const CascadeOutput o = run_cascade(*t, *be, X, false, y, ids, n_part, d, n_total, cfg);
    return build_cascade_out({&o}, *be, comm->world, comm->rank, "hostcomm", "cpu");
  } catch (const std::exception& e) {
    set_error("cascade: %s", e.what());
    return nullptr;
  }
}

}  // extern "C"
