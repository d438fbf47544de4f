// Crash evidence (failures reported with a reason, never silently): an opt-in handler for
// SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT that writes, with async-signal-safe calls only, the
// signal, the faulting address, the program counter, a raw backtrace and the process's memory map
// (/proc/self/maps) to a file, then hands the signal to whatever handler was installed before (a
// profiler's, Python's faulthandler) or to the default action.  With the map, every PC of a stack -- also
// those a profiler's own handler prints as "(unknown)" -- resolves to library + offset, which
// llvm-symbolizer / nm turn into a function.  Python: set SVM355_CRASH_MAPS=<path> (svm355._native
// installs it when the core library loads), or call svm_crash_handler_install directly.
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <ucontext.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>

#include "internal.h"

namespace {

constexpr int kSignals[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
constexpr int kNumSignals = sizeof(kSignals) / sizeof(kSignals[0]);
struct sigaction g_prev[kNumSignals];
char g_path[512];
volatile sig_atomic_t g_in_handler = 0;

void put(int fd, const char* s) {
  size_t n = std::strlen(s);
  while (n > 0) {
    const ssize_t w = ::write(fd, s, n);
    if (w <= 0) return;
    s += w;
    n -= size_t(w);
  }
}

void put_hex(int fd, uint64_t v) {
  char buf[19] = "0x";
  for (int i = 0; i < 16; ++i) buf[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
  buf[18] = 0;
  put(fd, buf);
}

void put_dec(int fd, int64_t v) {
  char buf[24];
  int i = 23;
  buf[i] = 0;
  const bool neg = v < 0;
  uint64_t u = neg ? uint64_t(-v) : uint64_t(v);
  do {
    buf[--i] = char('0' + u % 10);
    u /= 10;
  } while (u && i > 1);
  if (neg) buf[--i] = '-';
  put(fd, buf + i);
}

void handler(int sig, siginfo_t* si, void* uc) {
  int idx = 0;
  while (idx < kNumSignals && kSignals[idx] != sig) ++idx;
  if (!g_in_handler) {
    g_in_handler = 1;
    const int fd = ::open(g_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
      put(fd, "=== svm355 crash: signal ");
      put_dec(fd, sig);
      put(fd, " pid ");
      put_dec(fd, ::getpid());
      put(fd, " tid ");
      put_dec(fd, int64_t(::gettid()));
      put(fd, " addr ");
      put_hex(fd, uint64_t(reinterpret_cast<uintptr_t>(si ? si->si_addr : nullptr)));
#if defined(__x86_64__)
      if (uc) {
        put(fd, " pc ");
        put_hex(fd, uint64_t(static_cast<ucontext_t*>(uc)->uc_mcontext.gregs[REG_RIP]));
      }
#endif
      put(fd, "\n--- backtrace\n");
      void* frames[64];
      const int nf = ::backtrace(frames, 64);
      ::backtrace_symbols_fd(frames, nf, fd);
      put(fd, "--- /proc/self/maps\n");
      const int mfd = ::open("/proc/self/maps", O_RDONLY);
      if (mfd >= 0) {
        char buf[4096];
        for (;;) {
          const ssize_t r = ::read(mfd, buf, sizeof(buf));
          if (r <= 0) break;
          ssize_t off = 0;
          while (off < r) {
            const ssize_t w = ::write(fd, buf + off, size_t(r - off));
            if (w <= 0) break;
            off += w;
          }
        }
        ::close(mfd);
      }
      put(fd, "=== end\n");
      ::close(fd);
    }
  }
  // hand over: the previous handler (profiler / faulthandler), else the default action
  if (idx < kNumSignals) {
    const struct sigaction& p = g_prev[idx];
    if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
      p.sa_sigaction(sig, si, uc);
      return;
    }
    if (!(p.sa_flags & SA_SIGINFO) && p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
      p.sa_handler(sig);
      return;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

extern "C" SVM_API int svm_crash_handler_install(const char* path) {
  if (!path || !*path || std::strlen(path) >= sizeof(g_path)) {
    svm355::set_error("svm_crash_handler_install: bad path");
    return SVM_ERR_ARG;
  }
  std::strncpy(g_path, path, sizeof(g_path) - 1);
  void* warm[2];
  (void)::backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the handler
  for (int i = 0; i < kNumSignals; ++i) {
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (::sigaction(kSignals[i], &sa, &g_prev[i]) != 0) {
      svm355::set_error("svm_crash_handler_install: sigaction failed");
      return SVM_ERR_ARG;
    }
  }
  return SVM_OK;
}
