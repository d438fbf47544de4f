// Transport implementations (see transport.h).
#include "transport.h"

#include <algorithm>
#include <cstring>

namespace svm355 {
namespace {

#define HIPT(expr)                                                                            \
  do {                                                                                        \
    const hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) throw TransportError(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCLT(expr)                                                                              \
  do {                                                                                           \
    const ncclResult_t r_ = (expr);                                                              \
    if (r_ != ncclSuccess) throw TransportError(std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

}  // namespace

// ---------------------------------------------------------------------------------------- RCCL
RcclTransport::RcclTransport(ncclComm_t comm, int device) : comm_(comm), device_(device) {
  HIPT(hipSetDevice(device_));
  NCCLT(ncclCommUserRank(comm_, &rank_));
  NCCLT(ncclCommCount(comm_, &world_));
  HIPT(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
}

RcclTransport::~RcclTransport() {
  (void)hipSetDevice(device_);
  if (scratch_d_) (void)hipFree(scratch_d_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

int64_t* RcclTransport::scratch(int64_t n) {
  if (n > scratch_n_) {
    if (scratch_d_) HIPT(hipFree(scratch_d_));
    HIPT(hipMalloc(&scratch_d_, size_t(n) * 8));
    scratch_n_ = n;
  }
  return scratch_d_;
}

void RcclTransport::sync() { HIPT(hipStreamSynchronize(stream_)); }

int64_t RcclTransport::bcast_i64(int64_t v, int root) {
  HIPT(hipSetDevice(device_));
  int64_t* s = scratch(1);
  HIPT(hipMemcpyAsync(s, &v, 8, hipMemcpyHostToDevice, stream_));
  NCCLT(ncclBroadcast(s, s, 1, ncclInt64, root, comm_, stream_));
  int64_t out = 0;
  HIPT(hipMemcpyAsync(&out, s, 8, hipMemcpyDeviceToHost, stream_));
  sync();
  return out;
}

std::vector<int64_t> RcclTransport::allgather_i64(int64_t v) {
  HIPT(hipSetDevice(device_));
  int64_t* s = scratch(1 + world_);
  HIPT(hipMemcpyAsync(s, &v, 8, hipMemcpyHostToDevice, stream_));
  NCCLT(ncclAllGather(s, s + 1, 1, ncclInt64, comm_, stream_));
  std::vector<int64_t> out(static_cast<size_t>(world_));
  HIPT(hipMemcpyAsync(out.data(), s + 1, size_t(world_) * 8, hipMemcpyDeviceToHost, stream_));
  sync();
  return out;
}

void RcclTransport::allreduce_min(double* buf_d, int64_t n) {
  HIPT(hipSetDevice(device_));
  NCCLT(ncclAllReduce(buf_d, buf_d, size_t(n), ncclFloat64, ncclMin, comm_, stream_));
  sync();
}

void RcclTransport::allreduce_max(double* buf_d, int64_t n) {
  HIPT(hipSetDevice(device_));
  NCCLT(ncclAllReduce(buf_d, buf_d, size_t(n), ncclFloat64, ncclMax, comm_, stream_));
  sync();
}

void RcclTransport::bcast(void* buf_d, int64_t bytes, int root) {
  if (bytes <= 0) return;
  HIPT(hipSetDevice(device_));
  NCCLT(ncclBroadcast(buf_d, buf_d, size_t(bytes), ncclUint8, root, comm_, stream_));
  sync();
}

void RcclTransport::gather(const void* send_d, int64_t bytes, void* recv_d, int root) {
  if (bytes <= 0) return;
  HIPT(hipSetDevice(device_));
  NCCLT(ncclGather(send_d, recv_d, size_t(bytes), ncclUint8, root, comm_, stream_));
  sync();
}

void RcclTransport::send(const void* buf_d, int64_t bytes, int peer) {
  if (bytes <= 0) return;
  HIPT(hipSetDevice(device_));
  NCCLT(ncclSend(buf_d, size_t(bytes), ncclUint8, peer, comm_, stream_));
  sync();
}

void RcclTransport::recv(void* buf_d, int64_t bytes, int peer) {
  if (bytes <= 0) return;
  HIPT(hipSetDevice(device_));
  NCCLT(ncclRecv(buf_d, size_t(bytes), ncclUint8, peer, comm_, stream_));
  sync();
}

void RcclTransport::barrier() {
  HIPT(hipSetDevice(device_));
  int64_t* s = scratch(1);
  NCCLT(ncclAllReduce(s, s, 1, ncclInt64, ncclSum, comm_, stream_));
  sync();
}

// ------------------------------------------------------------------------------------ loopback
void LoopbackGroup::arrive_and_wait() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t g = gen_;
  if (++waiting_ == world_) {
    waiting_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  cv_.wait(lk, [&] { return gen_ != g; });
}

void LoopbackGroup::post(int src, int dst, std::vector<char> msg) {
  {
    std::lock_guard<std::mutex> lk(mail_mu_);
    mail_[size_t(src) * size_t(world_) + size_t(dst)].push_back(std::move(msg));
  }
  mail_cv_.notify_all();
}

std::vector<char> LoopbackGroup::take(int src, int dst) {
  std::unique_lock<std::mutex> lk(mail_mu_);
  auto& q = mail_[size_t(src) * size_t(world_) + size_t(dst)];
  mail_cv_.wait(lk, [&] { return !q.empty(); });
  std::vector<char> m = std::move(q.front());
  q.pop_front();
  return m;
}

void LoopbackTransport::to_host(std::vector<char>& dst, const void* src_d, int64_t bytes) {
  dst.resize(size_t(std::max<int64_t>(bytes, 0)));
  if (bytes > 0) {
    HIPT(hipSetDevice(device_));
    HIPT(hipMemcpy(dst.data(), src_d, size_t(bytes), hipMemcpyDeviceToHost));
  }
}

void LoopbackTransport::to_device(void* dst_d, const std::vector<char>& src, int64_t bytes) {
  if (bytes > 0) {
    HIPT(hipSetDevice(device_));
    HIPT(hipMemcpy(dst_d, src.data(), size_t(bytes), hipMemcpyHostToDevice));
  }
}

int64_t LoopbackTransport::bcast_i64(int64_t v, int root) {
  auto& mine = g_->slot(rank_);
  mine.resize(8);
  std::memcpy(mine.data(), &v, 8);
  g_->arrive_and_wait();
  int64_t out = 0;
  std::memcpy(&out, g_->slot(root).data(), 8);
  g_->arrive_and_wait();
  return out;
}

std::vector<int64_t> LoopbackTransport::allgather_i64(int64_t v) {
  auto& mine = g_->slot(rank_);
  mine.resize(8);
  std::memcpy(mine.data(), &v, 8);
  g_->arrive_and_wait();
  std::vector<int64_t> out(static_cast<size_t>(world()));
  for (int r = 0; r < world(); ++r) std::memcpy(&out[size_t(r)], g_->slot(r).data(), 8);
  g_->arrive_and_wait();
  return out;
}

void LoopbackTransport::allreduce(double* buf_d, int64_t n, bool is_min) {
  to_host(g_->slot(rank_), buf_d, n * 8);
  g_->arrive_and_wait();
  std::vector<double> acc(static_cast<size_t>(n));
  std::memcpy(acc.data(), g_->slot(0).data(), size_t(n) * 8);
  for (int r = 1; r < world(); ++r) {
    const double* o = reinterpret_cast<const double*>(g_->slot(r).data());
    for (int64_t i = 0; i < n; ++i) acc[size_t(i)] = is_min ? std::min(acc[size_t(i)], o[i]) : std::max(acc[size_t(i)], o[i]);
  }
  g_->arrive_and_wait();  // every rank has read every slot
  if (n > 0) {
    HIPT(hipSetDevice(device_));
    HIPT(hipMemcpy(buf_d, acc.data(), size_t(n) * 8, hipMemcpyHostToDevice));
  }
}

void LoopbackTransport::bcast(void* buf_d, int64_t bytes, int root) {
  if (rank_ == root) to_host(g_->slot(rank_), buf_d, bytes);
  g_->arrive_and_wait();
  if (rank_ != root) to_device(buf_d, g_->slot(root), bytes);
  g_->arrive_and_wait();
}

void LoopbackTransport::gather(const void* send_d, int64_t bytes, void* recv_d, int root) {
  to_host(g_->slot(rank_), send_d, bytes);
  g_->arrive_and_wait();
  if (rank_ == root)
    for (int r = 0; r < world(); ++r) to_device(static_cast<char*>(recv_d) + int64_t(r) * bytes, g_->slot(r), bytes);
  g_->arrive_and_wait();
}

void LoopbackTransport::send(const void* buf_d, int64_t bytes, int peer) {
  std::vector<char> m;
  to_host(m, buf_d, bytes);
  g_->post(rank_, peer, std::move(m));
}

void LoopbackTransport::recv(void* buf_d, int64_t bytes, int peer) {
  std::vector<char> m = g_->take(peer, rank_);
  if (int64_t(m.size()) != std::max<int64_t>(bytes, 0))
    throw TransportError("loopback recv: message size " + std::to_string(m.size()) + " != expected " +
                         std::to_string(bytes));
  to_device(buf_d, m, bytes);
}

}  // namespace svm355
