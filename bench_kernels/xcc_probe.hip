#include <hip/hip_runtime.h>
__global__ void k(unsigned* out) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = x;
}
int main() {
  unsigned* d; hipMalloc(&d, 4096 * 4);
  hipLaunchKernelGGL(k, dim3(512), dim3(256), 0, 0, d);
  unsigned h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int cnt[16] = {0};
  for (int i = 0; i < 512; ++i) cnt[h[i] & 15]++;
  printf("first 16 blocks xcc:"); for (int i = 0; i < 16; ++i) printf(" %u", h[i]); printf("\nper-xcc counts:");
  for (int i = 0; i < 16; ++i) printf(" %d", cnt[i]); printf("\nraw[0]=0x%x\n", h[0]);
  return 0;
}
