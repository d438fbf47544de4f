// Which XCD each workgroup of a 1 + 8 H grid lands on (HW_REG_XCC_ID), over several launches: checks the
// "blocks b and b + 8 share an XCD" placement the inner solve's L2 prefetch helpers rely on (speed only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void where(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 15;
}

int main() {
  const int G = 1 + 8 * 31;
  int* d;
  if (hipMalloc(&d, G * sizeof(int)) != hipSuccess) return 1;
  std::vector<int> h(G);
  int same_all = 0;
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL(where, dim3(G), dim3(256), 0, 0, d);
    if (hipMemcpy(h.data(), d, G * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int same = 0;
    for (int b = 8; b < G; b += 8) same += h[b] == h[0];
    int hist[8] = {0};
    for (int b = 0; b < G; ++b) hist[h[b] & 7]++;
    printf("launch %2d: block0 on XCD %d, %d/31 helper blocks share it; first 16 blocks:", rep, h[0], same);
    for (int b = 0; b < 16; ++b) printf(" %d", h[b]);
    printf("  | per-XCD counts:");
    for (int x = 0; x < 8; ++x) printf(" %d", hist[x]);
    printf("\n");
    same_all += same == 31;
  }
  printf("launches with all helpers co-located: %d/20\n", same_all);
  (void)hipFree(d);
  return 0;
}
