// H2D of the headline's 47 MB of uint8 rows from pageable host memory: one copy vs the copy split over
// 2 / 4 streams, and a hipHostRegister'd buffer (registration timed separately).  Best of 5 each.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  const size_t bytes = size_t(60000) * 784;
  std::vector<unsigned char> h(bytes);
  for (size_t i = 0; i < bytes; ++i) h[i] = (unsigned char)(i * 2654435761u >> 24);
  void* d = nullptr;
  CK(hipMalloc(&d, bytes));
  hipStream_t st[4];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));  // warm
  for (int parts : {1, 2, 4}) {
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now_ms();
      const size_t chunk = (bytes + parts - 1) / parts;
      for (int p = 0; p < parts; ++p) {
        const size_t o = p * chunk, b = std::min(chunk, bytes - o);
        CK(hipMemcpyAsync((char*)d + o, h.data() + o, b, hipMemcpyHostToDevice, st[p]));
      }
      for (int p = 0; p < parts; ++p) CK(hipStreamSynchronize(st[p]));
      best = std::min(best, now_ms() - t0);
    }
    printf("pageable, %d stream(s): %.3f ms (%.1f GB/s)\n", parts, best, bytes / best / 1e6);
  }
  double treg = now_ms();
  CK(hipHostRegister(h.data(), bytes, hipHostRegisterDefault));
  treg = now_ms() - treg;
  for (int parts : {1, 2}) {
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now_ms();
      const size_t chunk = (bytes + parts - 1) / parts;
      for (int p = 0; p < parts; ++p) {
        const size_t o = p * chunk, b = std::min(chunk, bytes - o);
        CK(hipMemcpyAsync((char*)d + o, h.data() + o, b, hipMemcpyHostToDevice, st[p]));
      }
      for (int p = 0; p < parts; ++p) CK(hipStreamSynchronize(st[p]));
      best = std::min(best, now_ms() - t0);
    }
    printf("registered (register %.3f ms), %d stream(s): %.3f ms (%.1f GB/s)\n", treg, parts, best, bytes / best / 1e6);
  }
  double tun = now_ms();
  CK(hipHostUnregister(h.data()));
  printf("unregister %.3f ms\n", now_ms() - tun);
  return 0;
}
