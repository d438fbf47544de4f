// LoopbackTransport (see cascade.h): P thread-ranks of one process, every exchange staged through
// host memory with the rank backend's own copies.  Every wait honours the group's WaitPolicy, so a
// rank that fails (or never arrives) ends the others' waits instead of hanging them.
#include <chrono>
#include <cstring>

#include "cascade.h"

namespace svm355 {

namespace {
constexpr auto kPoll = std::chrono::milliseconds(20);
}

LoopbackGroup::LoopbackGroup(int world, WaitPolicy wp)
    : world_(world), wp_(std::move(wp)), slots_(size_t(world)), mail_(size_t(world) * size_t(world)) {}

void LoopbackGroup::arrive_and_wait() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t g = gen_;
  if (++waiting_ == world_) {
    waiting_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  while (gen_ == g) {
    cv_.wait_for(lk, kPoll);
    if (gen_ != g) break;
    wp_.check(t0, "loopback collective");
  }
}

void LoopbackGroup::post(int src, int dst, std::vector<char> msg) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    mail_[size_t(src) * size_t(world_) + size_t(dst)].push_back(std::move(msg));
  }
  cv_.notify_all();
}

std::vector<char> LoopbackGroup::take(int src, int dst) {
  std::unique_lock<std::mutex> lk(mu_);
  auto& q = mail_[size_t(src) * size_t(world_) + size_t(dst)];
  const auto t0 = std::chrono::steady_clock::now();
  while (q.empty()) {
    cv_.wait_for(lk, kPoll);
    if (!q.empty()) break;
    wp_.check(t0, "loopback recv");
  }
  std::vector<char> m = std::move(q.front());
  q.pop_front();
  return m;
}

void LoopbackTransport::to_host(std::vector<char>& dst, const void* src, int64_t bytes) {
  dst.resize(size_t(std::max<int64_t>(bytes, 0)));
  if (bytes > 0) mem_->d2h(dst.data(), src, bytes);
}

void LoopbackTransport::to_backend(void* dst, const std::vector<char>& src, int64_t bytes) {
  if (bytes > 0) mem_->h2d(dst, src.data(), bytes);
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

void LoopbackTransport::allreduce(double* buf, int64_t n, bool is_min) {
  to_host(g_->slot(rank_), buf, n * 8);
  g_->arrive_and_wait();
  std::vector<double> acc(static_cast<size_t>(n));
  if (n) std::memcpy(acc.data(), g_->slot(0).data(), size_t(n) * 8);
  for (int r = 1; r < world(); ++r) {
    const double* o = reinterpret_cast<const double*>(g_->slot(r).data());
    for (int64_t i = 0; i < n; ++i)
      acc[size_t(i)] = is_min ? std::min(acc[size_t(i)], o[i]) : std::max(acc[size_t(i)], o[i]);
  }
  g_->arrive_and_wait();  // every rank has read every slot
  if (n > 0) mem_->h2d(buf, acc.data(), n * 8);
}

void LoopbackTransport::bcast(void* buf, int64_t bytes, int root) {
  if (rank_ == root) to_host(g_->slot(rank_), buf, bytes);
  g_->arrive_and_wait();
  if (rank_ != root) to_backend(buf, g_->slot(root), bytes);
  g_->arrive_and_wait();
}

void LoopbackTransport::gather(const void* send, int64_t bytes, void* recv, int root) {
  to_host(g_->slot(rank_), send, bytes);
  g_->arrive_and_wait();
  if (rank_ == root)
    for (int r = 0; r < world(); ++r) to_backend(static_cast<char*>(recv) + int64_t(r) * bytes, g_->slot(r), bytes);
  g_->arrive_and_wait();
}

void LoopbackTransport::send_i64(int64_t v, int peer) {
  std::vector<char> m(8);
  std::memcpy(m.data(), &v, 8);
  g_->post(rank_, peer, std::move(m));
}

int64_t LoopbackTransport::recv_i64(int peer) {
  const std::vector<char> m = g_->take(peer, rank_);
  if (m.size() != 8) throw TransportError("loopback recv_i64: message of " + std::to_string(m.size()) + " bytes");
  int64_t v = 0;
  std::memcpy(&v, m.data(), 8);
  return v;
}

void LoopbackTransport::send(const void* buf, int64_t bytes, int peer) {
  std::vector<char> m;
  to_host(m, buf, bytes);
  g_->post(rank_, peer, std::move(m));
}

void LoopbackTransport::recv(void* buf, int64_t bytes, int peer) {
  const std::vector<char> m = g_->take(peer, rank_);
  if (int64_t(m.size()) != std::max<int64_t>(bytes, 0))
    throw TransportError("loopback recv: message size " + std::to_string(m.size()) + " != expected " +
                         std::to_string(bytes));
  to_backend(buf, m, bytes);
}

}  // namespace svm355
