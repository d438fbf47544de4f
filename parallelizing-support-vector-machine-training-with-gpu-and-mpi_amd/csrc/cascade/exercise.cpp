// Transport exerciser: a script of Transport calls per rank, run with rank-dependent payloads whose
// every received byte is checked.  Two uses:
//   * tests: svm_loopback_exercise drives a (strict) LoopbackGroup of CPU-backend ranks through any
//     call sequence -- including deliberately wrong ones, which must fail naming the ranks;
//   * preflight: the device groups / ranks (cascade_dev.hip) run preflight_script(P) -- every op the
//     cascade driver issues, the tree's send / recv pairs per level included -- on the real RCCL
//     communicators right after creating them, before any timed region, with a short deadline.
//
// Script: one op list per rank separated by '|' (a single list = every rank runs it); ops are
// separated by spaces or commas:
//   bi@R  bcast_i64 (root R)          ag     allgather_i64           ba       barrier
//   mn:N  allreduce_min of N doubles  mx:N   allreduce_max of N      bc:B@R   bcast of B bytes
//   ga:B@R gather of B bytes per rank si>P   send_i64 to P           ri<P     recv_i64 from P
//   s:B>P send of B bytes to P        r:B<P  recv of B bytes from P
// Payloads: collective c of a run (c-th collective call of the rank, equal on matched ranks) and
// message k of a channel src -> dst give every rank the same expected values.
#include <chrono>
#include <cstring>
#include <sstream>

#include "../core/internal.h"
#include "cascade_capi.h"

namespace svm355 {

namespace {

struct XOp {
  char kind[3] = {0, 0, 0};  // bi ag mn mx bc ga ba si ri s r
  int64_t n = 0;             // bytes (bc, ga, s, r) or doubles (mn, mx)
  int peer = -1;             // root or peer
  std::string text;
};

std::vector<std::vector<XOp>> parse_script(const std::string& script, int world) {
  std::vector<std::string> lists;
  {
    std::string cur;
    for (char c : script) {
      if (c == '|') {
        lists.push_back(cur);
        cur.clear();
      } else {
        cur += c;
      }
    }
    lists.push_back(cur);
  }
  if (lists.size() != 1 && int(lists.size()) != world)
    throw CascadeError("exercise script: " + std::to_string(lists.size()) + " rank lists for world " +
                       std::to_string(world));
  std::vector<std::vector<XOp>> out(static_cast<size_t>(world));
  for (int r = 0; r < world; ++r) {
    std::string s = lists[lists.size() == 1 ? 0 : size_t(r)];
    for (char& c : s)
      if (c == ',') c = ' ';
    std::istringstream is(s);
    std::string tok;
    while (is >> tok) {
      XOp op;
      op.text = tok;
      auto num = [&](size_t from, size_t to) -> int64_t {
        if (from >= tok.size() || to <= from) throw CascadeError("exercise script: bad op '" + tok + "'");
        return std::stoll(tok.substr(from, to - from));
      };
      const std::string k2 = tok.substr(0, 2);
      if (k2 == "bi") {
        std::memcpy(op.kind, "bi", 2);
        op.peer = int(num(3, tok.size()));
      } else if (k2 == "ag" || k2 == "ba") {
        std::memcpy(op.kind, k2.c_str(), 2);
      } else if (k2 == "mn" || k2 == "mx") {
        std::memcpy(op.kind, k2.c_str(), 2);
        op.n = num(3, tok.size());
      } else if (k2 == "bc" || k2 == "ga") {
        std::memcpy(op.kind, k2.c_str(), 2);
        const size_t at = tok.find('@');
        op.n = num(3, at);
        op.peer = int(num(at + 1, tok.size()));
      } else if (k2 == "si" || k2 == "ri") {
        std::memcpy(op.kind, k2.c_str(), 2);
        op.peer = int(num(3, tok.size()));
      } else if (tok[0] == 's' || tok[0] == 'r') {
        op.kind[0] = tok[0];
        const size_t arrow = tok.find_first_of("<>");
        op.n = num(2, arrow);
        op.peer = int(num(arrow + 1, tok.size()));
      } else {
        throw CascadeError("exercise script: unknown op '" + tok + "'");
      }
      if (op.peer >= world) throw CascadeError("exercise script: rank out of range in '" + tok + "'");
      out[size_t(r)].push_back(op);
    }
  }
  return out;
}

uint8_t pat(int64_t a, int64_t b, int64_t i) {
  const uint64_t x = uint64_t(a) * 0x9E3779B97F4A7C15ull ^ uint64_t(b) * 0xC2B2AE3D27D4EB4Full ^ uint64_t(i);
  return uint8_t((x * 0x2545F4914F6CDD1Dull) >> 56);
}

int64_t chan_value(int src, int dst, int64_t k) { return int64_t(src) * 1000003 + int64_t(dst) * 1009 + k; }

}  // namespace

std::string preflight_script(int P, int64_t bulk_bytes) {
  std::ostringstream s;
  const std::string B = std::to_string(bulk_bytes);
  std::vector<std::string> per(static_cast<size_t>(P));
  for (int r = 0; r < P; ++r) {
    std::ostringstream o;
    o << "bi@0 ag mn:784 mx:784 bc:" << B << "@0 ga:" << B << "@0 ";
    if (P > 1) o << "bi@" << (P - 1) << " ";
    // the classical cascade's pairs per level (mpi_svm_main3.cpp:689-716): a count, then the set
    for (int step = 1; step < P; step *= 2) {
      if (r % (2 * step) == step)
        o << "si>" << r - step << " s:" << B << ">" << r - step << " ";
      else if (r % (2 * step) == 0 && r + step < P)
        o << "ri<" << r + step << " r:" << B << "<" << r + step << " ";
    }
    o << "ba";
    per[size_t(r)] = o.str();
  }
  for (int r = 0; r < P; ++r) s << (r ? "|" : "") << per[size_t(r)];
  return s.str();
}

void exercise_transport(Transport& t, Backend& B, const std::string& script) {
  const int P = t.world(), me = t.rank();
  const auto ops = parse_script(script, P);
  int64_t coll = 0;
  std::vector<int64_t> sent(static_cast<size_t>(P), 0), recvd(static_cast<size_t>(P), 0);
  int64_t cap = 64;
  for (const XOp& op : ops[size_t(me)]) {
    const bool dbl = op.kind[0] == 'm';  // mn / mx: doubles
    cap = std::max<int64_t>(cap, (dbl ? 8 * op.n : op.n * (op.kind[0] == 'g' ? P : 1)) + 64);
  }
  Buf buf(&B);
  buf.ensure(cap);
  std::vector<uint8_t> h(static_cast<size_t>(cap));
  int idx = 0;
  auto fail = [&](const XOp& op, const std::string& why) {
    throw TransportError("exercise rank " + std::to_string(me) + " op " + std::to_string(idx) + " (" + op.text +
                         "): " + why);
  };
  for (const XOp& op : ops[size_t(me)]) {
    const std::string k(op.kind);
    if (k == "bi") {
      const int64_t v = t.bcast_i64(1000 * int64_t(me) + coll, op.peer);
      if (v != 1000 * int64_t(op.peer) + coll) fail(op, "got " + std::to_string(v));
      ++coll;
    } else if (k == "ag") {
      const auto v = t.allgather_i64(1000 * int64_t(me) + coll);
      if (int(v.size()) != P) fail(op, "wrong size");
      for (int r = 0; r < P; ++r)
        if (v[size_t(r)] != 1000 * int64_t(r) + coll) fail(op, "rank " + std::to_string(r) + " entry wrong");
      ++coll;
    } else if (k == "mn" || k == "mx") {
      std::vector<double> v(static_cast<size_t>(op.n));
      for (int64_t i = 0; i < op.n; ++i) v[size_t(i)] = double(((me + i + coll) % P) * 3 + coll);
      if (op.n) B.h2d(buf.get(), v.data(), op.n * 8);
      if (k == "mn")
        t.allreduce_min(buf.as<double>(), op.n);
      else
        t.allreduce_max(buf.as<double>(), op.n);
      if (op.n) B.d2h(v.data(), buf.get(), op.n * 8);
      const double want = k == "mn" ? double(coll) : double(3 * (P - 1) + coll);
      for (int64_t i = 0; i < op.n; ++i)
        if (v[size_t(i)] != want) fail(op, "element " + std::to_string(i) + " = " + std::to_string(v[size_t(i)]));
      ++coll;
    } else if (k == "bc") {
      for (int64_t i = 0; i < op.n; ++i) h[size_t(i)] = me == op.peer ? pat(op.peer, coll, i) : uint8_t(0xA5);
      if (op.n) B.h2d(buf.get(), h.data(), op.n);
      t.bcast(buf.get(), op.n, op.peer);
      if (op.n) B.d2h(h.data(), buf.get(), op.n);
      for (int64_t i = 0; i < op.n; ++i)
        if (h[size_t(i)] != pat(op.peer, coll, i)) fail(op, "byte " + std::to_string(i) + " differs from the root's");
      ++coll;
    } else if (k == "ga") {
      std::vector<uint8_t> mine(static_cast<size_t>(op.n));
      for (int64_t i = 0; i < op.n; ++i) mine[size_t(i)] = pat(me, coll, i);
      Buf snd(&B);
      snd.ensure(std::max<int64_t>(op.n, 8));
      if (op.n) B.h2d(snd.get(), mine.data(), op.n);
      t.gather(snd.get(), op.n, me == op.peer ? buf.get() : nullptr, op.peer);
      if (me == op.peer && op.n) {
        std::vector<uint8_t> all(static_cast<size_t>(op.n * P));
        B.d2h(all.data(), buf.get(), op.n * P);
        for (int r = 0; r < P; ++r)
          for (int64_t i = 0; i < op.n; ++i)
            if (all[size_t(r * op.n + i)] != pat(r, coll, i))
              fail(op, "segment of rank " + std::to_string(r) + " byte " + std::to_string(i) + " wrong");
      }
      ++coll;
    } else if (k == "ba") {
      t.barrier();
      ++coll;
    } else if (k == "si") {
      t.send_i64(chan_value(me, op.peer, sent[size_t(op.peer)]++), op.peer);
    } else if (k == "ri") {
      const int64_t v = t.recv_i64(op.peer);
      if (v != chan_value(op.peer, me, recvd[size_t(op.peer)]++)) fail(op, "got " + std::to_string(v));
    } else if (k == "s") {
      const int64_t kk = sent[size_t(op.peer)]++;
      for (int64_t i = 0; i < op.n; ++i) h[size_t(i)] = pat(chan_value(me, op.peer, kk), 7, i);
      if (op.n) B.h2d(buf.get(), h.data(), op.n);
      t.send(buf.get(), op.n, op.peer);
    } else if (k == "r") {
      const int64_t kk = recvd[size_t(op.peer)]++;
      if (op.n) B.h2d(buf.get(), std::vector<uint8_t>(size_t(op.n), 0x5A).data(), op.n);
      t.recv(buf.get(), op.n, op.peer);
      if (op.n) B.d2h(h.data(), buf.get(), op.n);
      for (int64_t i = 0; i < op.n; ++i)
        if (h[size_t(i)] != pat(chan_value(op.peer, me, kk), 7, i)) fail(op, "byte " + std::to_string(i) + " wrong");
    }
    ++idx;
  }
  B.sync();
}

}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API int svm_loopback_exercise(int32_t world, const char* script, int32_t strict, double timeout_s,
                                  double* elapsed_s) {
  const auto t0 = std::chrono::steady_clock::now();
  auto done = [&](int rc) {
    if (elapsed_s) *elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
  };
  if (world < 1 || !script) {
    set_error("svm_loopback_exercise: bad arguments");
    return done(SVM_ERR_ARG);
  }
  try {
    auto token = std::make_shared<AbortToken>();
    auto group = std::make_shared<LoopbackGroup>(world, WaitPolicy{token, timeout_s > 0 ? timeout_s : 20.0},
                                                 strict != 0);
    std::vector<std::unique_ptr<Backend>> be(static_cast<size_t>(world));
    std::vector<std::unique_ptr<LoopbackTransport>> tr(static_cast<size_t>(world));
    for (int r = 0; r < world; ++r) {
      be[size_t(r)] = make_cpu_backend();
      tr[size_t(r)] = std::make_unique<LoopbackTransport>(group, r, be[size_t(r)].get());
    }
    const std::string s = script;
    run_rank_threads(world, token, [&](int r) { exercise_transport(*tr[size_t(r)], *be[size_t(r)], s); },
                     [&](int r) { tr[size_t(r)]->abort(); });
    return done(SVM_OK);
  } catch (const std::exception& e) {
    set_error("%s", e.what());
    return done(SVM_ERR_DEVICE);
  }
}

SVM_API int svm_preflight_script(int32_t world, int64_t bulk_bytes, char* out, int64_t cap) {
  const std::string s = preflight_script(world, bulk_bytes);
  if (!out || cap < int64_t(s.size()) + 1) return int(s.size()) + 1;
  std::memcpy(out, s.c_str(), s.size() + 1);
  return 0;
}

}  // extern "C"
