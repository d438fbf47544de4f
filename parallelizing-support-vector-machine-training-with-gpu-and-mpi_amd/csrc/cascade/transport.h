// Rank-to-rank transports of the native Cascade SVM.
//
// The reference's MPI call sites (mpi_svm_main3.cpp / mpi_svm_main2.cpp) re-expressed as the few
// collectives the cascade needs.  Every buffer argument is DEVICE memory of the calling rank's GPU;
// each call returns once its data is complete (the exchanges are a few MB per round and the solves
// between them take milliseconds, so there is nothing to overlap).
//
// | reference call site                                   | Transport method                       |
// |-------------------------------------------------------|----------------------------------------|
// | MPI_Bcast n_features / n_total, SV count, converged   | bcast_i64                              |
// | MPI_Bcast min / max (M3 :534-535)                     | allreduce_min / allreduce_max of the   |
// |                                                       |   local column statistics              |
// | MPI_Bcast X_sv, Y_sv, alpha_sv, ID_sv (M3 :598-601)   | bcast of ONE packed SV buffer          |
// | star MPI_Send/Recv to rank 0 (M2 :578-607, 748-760)   | allgather_i64 (counts) + gather of     |
// |                                                       |   max-count-padded packed buffers      |
// | tree MPI_Send/Recv pairs (M3 :689-716)                | send / recv                            |
//
// RcclTransport: one RCCL communicator per rank (ncclCommInitAll over the node's GPUs, one host
// thread per GPU); ncclBroadcast / ncclAllReduce / ncclAllGather / ncclGather / ncclSend+ncclRecv
// on the rank's own stream, over xGMI.
// LoopbackTransport: P ranks as threads of one process staging every exchange through host memory,
// so any P runs on one GPU (RCCL refuses two ranks on one device) -- the test transport.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace svm355 {

// Thrown by the transports on any runtime / RCCL error (the message names the failing call).
struct TransportError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual int64_t bcast_i64(int64_t v, int root) = 0;
  virtual std::vector<int64_t> allgather_i64(int64_t v) = 0;
  virtual void allreduce_min(double* buf_d, int64_t n) = 0;
  virtual void allreduce_max(double* buf_d, int64_t n) = 0;
  virtual void bcast(void* buf_d, int64_t bytes, int root) = 0;
  // Every rank sends `bytes` from send_d; root receives world * bytes into recv_d (rank order).
  virtual void gather(const void* send_d, int64_t bytes, void* recv_d, int root) = 0;
  virtual void send(const void* buf_d, int64_t bytes, int peer) = 0;
  virtual void recv(void* buf_d, int64_t bytes, int peer) = 0;
  virtual void barrier() = 0;
  virtual const char* name() const = 0;
};

// ---------------------------------------------------------------------------------------- RCCL
class RcclTransport : public Transport {
 public:
  RcclTransport(ncclComm_t comm, int device);  // comm: this rank's communicator; device: its GPU
  ~RcclTransport() override;
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  int64_t bcast_i64(int64_t v, int root) override;
  std::vector<int64_t> allgather_i64(int64_t v) override;
  void allreduce_min(double* buf_d, int64_t n) override;
  void allreduce_max(double* buf_d, int64_t n) override;
  void bcast(void* buf_d, int64_t bytes, int root) override;
  void gather(const void* send_d, int64_t bytes, void* recv_d, int root) override;
  void send(const void* buf_d, int64_t bytes, int peer) override;
  void recv(void* buf_d, int64_t bytes, int peer) override;
  void barrier() override;
  const char* name() const override { return "rccl"; }

 private:
  void sync();
  int64_t* scratch(int64_t n);
  ncclComm_t comm_;
  int device_, rank_ = 0, world_ = 1;
  hipStream_t stream_ = nullptr;
  int64_t* scratch_d_ = nullptr;  // small device staging for the scalar collectives
  int64_t scratch_n_ = 0;
};

// ------------------------------------------------------------------------------------ loopback
class LoopbackGroup {
 public:
  explicit LoopbackGroup(int world)
      : world_(world), slots_(size_t(world)), mail_(size_t(world) * size_t(world)) {}
  int world() const { return world_; }
  void arrive_and_wait();  // reusable (generation-counted) barrier
  std::vector<char>& slot(int r) { return slots_[size_t(r)]; }
  void post(int src, int dst, std::vector<char> msg);
  std::vector<char> take(int src, int dst);

 private:
  int world_;
  std::mutex mu_;
  std::condition_variable cv_;
  int waiting_ = 0;
  uint64_t gen_ = 0;
  std::vector<std::vector<char>> slots_;
  std::mutex mail_mu_;
  std::condition_variable mail_cv_;
  std::vector<std::deque<std::vector<char>>> mail_;  // [src * world + dst]
};

class LoopbackTransport : public Transport {
 public:
  LoopbackTransport(std::shared_ptr<LoopbackGroup> g, int rank, int device)
      : g_(std::move(g)), rank_(rank), device_(device) {}
  int rank() const override { return rank_; }
  int world() const override { return g_->world(); }
  int64_t bcast_i64(int64_t v, int root) override;
  std::vector<int64_t> allgather_i64(int64_t v) override;
  void allreduce_min(double* buf_d, int64_t n) override { allreduce(buf_d, n, true); }
  void allreduce_max(double* buf_d, int64_t n) override { allreduce(buf_d, n, false); }
  void bcast(void* buf_d, int64_t bytes, int root) override;
  void gather(const void* send_d, int64_t bytes, void* recv_d, int root) override;
  void send(const void* buf_d, int64_t bytes, int peer) override;
  void recv(void* buf_d, int64_t bytes, int peer) override;
  void barrier() override { g_->arrive_and_wait(); }
  const char* name() const override { return "loopback"; }

 private:
  void to_host(std::vector<char>& dst, const void* src_d, int64_t bytes);
  void to_device(void* dst_d, const std::vector<char>& src, int64_t bytes);
  void allreduce(double* buf_d, int64_t n, bool is_min);
  std::shared_ptr<LoopbackGroup> g_;
  int rank_, device_;
};

}  // namespace svm355
