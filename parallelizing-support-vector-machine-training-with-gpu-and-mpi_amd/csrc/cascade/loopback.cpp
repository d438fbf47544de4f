// LoopbackTransport (see cascade.h): P thread-ranks of one process, every exchange staged through
// host memory with the rank backend's own copies.  Every wait honours the group's WaitPolicy, so a
// rank that fails (or never arrives) ends the others' waits instead of hanging them.
//
// Strict mode (default) holds the call sequence to RCCL's contract: collectives must match in op,
// root and byte count on every rank; a send completes only once the peer's recv has taken it (a
// rendezvous, like ncclSend); and a cycle in the wait-for graph of the blocked ranks is reported as
// a deadlock naming the ranks and their calls, instead of waiting for the deadline.
#include <chrono>
#include <cstring>

#include "cascade.h"

namespace svm355 {

namespace {
constexpr auto kPoll = std::chrono::milliseconds(20);

bool is_collective(int kind) {
  return kind >= LoopbackGroup::kBcastI64 && kind <= LoopbackGroup::kBarrier;
}

bool same_op(const LoopbackGroup::OpDesc& a, const LoopbackGroup::OpDesc& b) {
  return a.kind == b.kind && a.root == b.root && a.bytes == b.bytes;
}

std::string op_text(const LoopbackGroup::OpDesc& o) {
  std::string s = LoopbackGroup::op_name(o.kind);
  s += "(";
  bool sep = false;
  if (o.kind == LoopbackGroup::kSend || o.kind == LoopbackGroup::kRecv) {
    s += (o.kind == LoopbackGroup::kSend ? "to rank " : "from rank ") + std::to_string(o.peer);
    sep = true;
  }
  if (o.root >= 0) {
    s += std::string(sep ? ", " : "") + "root " + std::to_string(o.root);
    sep = true;
  }
  if (o.bytes >= 0) s += std::string(sep ? ", " : "") + std::to_string(o.bytes) + " B";
  return s + ")";
}

// Resets a rank's state to idle when its wait ends by an exception (runs with the group lock held:
// declared after the unique_lock, destroyed before it).
struct IdleOnThrow {
  LoopbackGroup::OpDesc* op;
  bool armed = true;
  ~IdleOnThrow() {
    if (armed) *op = LoopbackGroup::OpDesc{};
  }
};
}  // namespace

const char* LoopbackGroup::op_name(int kind) {
  switch (kind) {
    case kBcastI64: return "bcast_i64";
    case kAllgatherI64: return "allgather_i64";
    case kAllreduceMin: return "allreduce_min";
    case kAllreduceMax: return "allreduce_max";
    case kBcast: return "bcast";
    case kGather: return "gather";
    case kBarrier: return "barrier";
    case kSend: return "send";
    case kRecv: return "recv";
    default: return "idle";
  }
}

LoopbackGroup::LoopbackGroup(int world, WaitPolicy wp, bool strict)
    : world_(world),
      wp_(std::move(wp)),
      strict_(strict),
      slots_(size_t(world)),
      mail_(size_t(world) * size_t(world)),
      sent_(size_t(world) * size_t(world), 0),
      taken_(size_t(world) * size_t(world), 0),
      rejected_(size_t(world) * size_t(world), 0),
      st_(size_t(world)),
      coll_(size_t(world)) {}

// ---- wait-for graph (all under mu_)
bool LoopbackGroup::blocked(int r) const {
  const RankState& s = st_[size_t(r)];
  if (is_collective(s.op.kind)) return gen_ == s.gen;
  if (s.op.kind == kSend) {
    const size_t ch = size_t(r) * size_t(world_) + size_t(s.op.peer);
    return taken_[ch] < s.seq && uint64_t(rejected_[ch]) != s.seq;
  }
  if (s.op.kind == kRecv) return mail_[size_t(s.op.peer) * size_t(world_) + size_t(r)].empty();
  return false;
}

std::vector<int> LoopbackGroup::waits_for(int r) const {
  const RankState& s = st_[size_t(r)];
  std::vector<int> out;
  if (is_collective(s.op.kind)) {
    for (int q = 0; q < world_; ++q) {
      if (q == r) continue;
      const RankState& o = st_[size_t(q)];
      if (!(is_collective(o.op.kind) && o.gen == s.gen)) out.push_back(q);  // has not arrived
    }
  } else if (s.op.kind == kSend || s.op.kind == kRecv) {
    out.push_back(s.op.peer);
  }
  return out;
}

std::string LoopbackGroup::describe(int r) const {
  return "rank " + std::to_string(r) + " in " + op_text(st_[size_t(r)].op);
}

// A cycle of blocked ranks reachable from r through blocked ranks: none of them can move again.
std::string LoopbackGroup::deadlock_cycle(int r) const {
  if (!blocked(r)) return "";
  std::vector<int> color(size_t(world_), 0), parent(size_t(world_), -1);  // 0 new, 1 on stack, 2 done
  std::vector<std::pair<int, size_t>> stack{{r, 0}};
  std::vector<std::vector<int>> edges(static_cast<size_t>(world_));
  edges[size_t(r)] = waits_for(r);
  color[size_t(r)] = 1;
  while (!stack.empty()) {
    auto& [u, next] = stack.back();
    if (next >= edges[size_t(u)].size()) {
      color[size_t(u)] = 2;
      stack.pop_back();
      continue;
    }
    const int v = edges[size_t(u)][next++];
    if (!blocked(v)) continue;
    if (color[size_t(v)] == 1) {  // cycle v -> ... -> u -> v
      std::vector<int> cyc{v};
      for (int x = u; x != v && x >= 0; x = parent[size_t(x)]) cyc.push_back(x);
      std::string msg;
      for (size_t i = cyc.size(); i-- > 0;) {
        if (!msg.empty()) msg += " waits for ";
        msg += describe(cyc[i]);
      }
      return msg + " waits for rank " + std::to_string(cyc.back());
    }
    if (color[size_t(v)] == 0) {
      color[size_t(v)] = 1;
      parent[size_t(v)] = u;
      edges[size_t(v)] = waits_for(v);
      stack.emplace_back(v, 0);
    }
  }
  return "";
}

void LoopbackGroup::wait_until(std::unique_lock<std::mutex>& lk, int rank, const char* what,
                               const std::function<bool()>& done) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!done()) {
    if (strict_ && rank >= 0) {
      const std::string cyc = deadlock_cycle(rank);
      if (!cyc.empty()) throw TransportError(std::string("loopback deadlock: ") + cyc);
    }
    cv_.wait_for(lk, kPoll);
    if (done()) break;
    wp_.check(t0, what);
  }
}

void LoopbackGroup::arrive_and_wait(int rank) {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t g = gen_;
  OpDesc dummy;
  IdleOnThrow guard{rank >= 0 ? &st_[size_t(rank)].op : &dummy};
  if (rank >= 0) {
    if (st_[size_t(rank)].op.kind == kIdle) st_[size_t(rank)].op.kind = kBarrier;
    st_[size_t(rank)].gen = g;
  }
  if (++waiting_ == world_) {
    waiting_ = 0;
    ++gen_;
    cv_.notify_all();
  } else {
    wait_until(lk, rank, "loopback collective", [&] { return gen_ != g; });
  }
  guard.armed = false;
  if (rank >= 0) st_[size_t(rank)].op = OpDesc{};
}

void LoopbackGroup::collective(int rank, const OpDesc& op, const std::function<void()>& between) {
  {
    std::unique_lock<std::mutex> lk(mu_);
    IdleOnThrow guard{&st_[size_t(rank)].op};
    coll_[size_t(rank)] = op;
    st_[size_t(rank)].op = op;
    const uint64_t g = gen_;
    st_[size_t(rank)].gen = g;
    if (++waiting_ == world_) {  // last to arrive: compare every rank's call with rank 0's
      waiting_ = 0;
      mismatch_.clear();
      if (strict_)
        for (int q = 1; q < world_; ++q)
          if (!same_op(coll_[size_t(q)], coll_[0])) {
            mismatch_ = "loopback collective mismatch: rank 0 called " + op_text(coll_[0]) + " but rank " +
                        std::to_string(q) + " called " + op_text(coll_[size_t(q)]);
            break;
          }
      ++gen_;
      cv_.notify_all();
    } else {
      wait_until(lk, rank, "loopback collective", [&] { return gen_ != g; });
    }
    // mismatch_ belongs to this generation until every rank has passed the second barrier (a rank
    // cannot complete the next collective's first barrier before that).
    if (!mismatch_.empty()) throw TransportError(mismatch_);
    guard.armed = false;
  }
  if (between) between();
  {
    std::unique_lock<std::mutex> lk(mu_);
    IdleOnThrow guard{&st_[size_t(rank)].op};
    const uint64_t g = gen_;
    st_[size_t(rank)].gen = g;
    if (++waiting_ == world_) {
      waiting_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      wait_until(lk, rank, "loopback collective", [&] { return gen_ != g; });
    }
    guard.armed = false;
    st_[size_t(rank)].op = OpDesc{};
  }
}

void LoopbackGroup::post(int src, int dst, std::vector<char> msg) {
  const size_t ch = size_t(src) * size_t(world_) + size_t(dst);
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t bytes = int64_t(msg.size());
  const uint64_t seq = ++sent_[ch];
  mail_[ch].push_back(Msg{std::move(msg), seq});
  cv_.notify_all();
  if (!strict_) return;
  IdleOnThrow guard{&st_[size_t(src)].op};
  st_[size_t(src)].op = OpDesc{kSend, -1, bytes, dst};
  st_[size_t(src)].seq = seq;
  wait_until(lk, src, "loopback send", [&] { return taken_[ch] >= seq || uint64_t(rejected_[ch]) == seq; });
  if (uint64_t(rejected_[ch]) == seq)
    throw TransportError("loopback send to rank " + std::to_string(dst) + ": the receiver refused the " +
                         std::to_string(bytes) + "-byte message (size mismatch)");
  guard.armed = false;
  st_[size_t(src)].op = OpDesc{};
}

std::vector<char> LoopbackGroup::take(int src, int dst, int64_t expect) {
  const size_t ch = size_t(src) * size_t(world_) + size_t(dst);
  std::unique_lock<std::mutex> lk(mu_);
  IdleOnThrow guard{&st_[size_t(dst)].op};
  st_[size_t(dst)].op = OpDesc{kRecv, -1, expect, src};
  auto& q = mail_[ch];
  wait_until(lk, dst, "loopback recv", [&] { return !q.empty(); });
  Msg m = std::move(q.front());
  q.pop_front();
  taken_[ch] = m.seq;
  if (expect >= 0 && int64_t(m.data.size()) != expect) {
    rejected_[ch] = int64_t(m.seq);
    cv_.notify_all();
    throw TransportError("loopback recv from rank " + std::to_string(src) + ": message of " +
                         std::to_string(m.data.size()) + " bytes, expected " + std::to_string(expect));
  }
  cv_.notify_all();
  guard.armed = false;
  st_[size_t(dst)].op = OpDesc{};
  return std::move(m.data);
}

// ------------------------------------------------------------------------------ LoopbackTransport
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
  int64_t out = 0;
  g_->collective(rank_, {LoopbackGroup::kBcastI64, root, 8, -1}, [&] { std::memcpy(&out, g_->slot(root).data(), 8); });
  return out;
}

std::vector<int64_t> LoopbackTransport::allgather_i64(int64_t v) {
  auto& mine = g_->slot(rank_);
  mine.resize(8);
  std::memcpy(mine.data(), &v, 8);
  std::vector<int64_t> out(static_cast<size_t>(world()));
  g_->collective(rank_, {LoopbackGroup::kAllgatherI64, -1, 8, -1}, [&] {
    for (int r = 0; r < world(); ++r) std::memcpy(&out[size_t(r)], g_->slot(r).data(), 8);
  });
  return out;
}

void LoopbackTransport::allreduce(double* buf, int64_t n, bool is_min) {
  to_host(g_->slot(rank_), buf, n * 8);
  std::vector<double> acc(static_cast<size_t>(n));
  g_->collective(rank_, {is_min ? LoopbackGroup::kAllreduceMin : LoopbackGroup::kAllreduceMax, -1, n * 8, -1}, [&] {
    if (n) std::memcpy(acc.data(), g_->slot(0).data(), size_t(n) * 8);
    for (int r = 1; r < world(); ++r) {
      const double* o = reinterpret_cast<const double*>(g_->slot(r).data());
      for (int64_t i = 0; i < n; ++i)
        acc[size_t(i)] = is_min ? std::min(acc[size_t(i)], o[i]) : std::max(acc[size_t(i)], o[i]);
    }
  });
  if (n > 0) mem_->h2d(buf, acc.data(), n * 8);
}

void LoopbackTransport::bcast(void* buf, int64_t bytes, int root) {
  if (rank_ == root) to_host(g_->slot(rank_), buf, bytes);
  g_->collective(rank_, {LoopbackGroup::kBcast, root, bytes, -1}, [&] {
    if (rank_ != root) to_backend(buf, g_->slot(root), bytes);
  });
}

void LoopbackTransport::gather(const void* send, int64_t bytes, void* recv, int root) {
  to_host(g_->slot(rank_), send, bytes);
  g_->collective(rank_, {LoopbackGroup::kGather, root, bytes, -1}, [&] {
    if (rank_ == root)
      for (int r = 0; r < world(); ++r) to_backend(static_cast<char*>(recv) + int64_t(r) * bytes, g_->slot(r), bytes);
  });
}

void LoopbackTransport::barrier() { g_->collective(rank_, {LoopbackGroup::kBarrier, -1, -1, -1}, nullptr); }

void LoopbackTransport::send_i64(int64_t v, int peer) {
  std::vector<char> m(8);
  std::memcpy(m.data(), &v, 8);
  g_->post(rank_, peer, std::move(m));
}

int64_t LoopbackTransport::recv_i64(int peer) {
  const std::vector<char> m = g_->take(peer, rank_, 8);
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
  const std::vector<char> m = g_->take(peer, rank_, std::max<int64_t>(bytes, 0));
  to_backend(buf, m, bytes);
}

}  // namespace svm355
