// Reads HW_REG_XCC_ID per block to check the block -> XCD placement.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) o[blockIdx.x] = x;
}
int main() {
  unsigned* d; hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, d);
  unsigned h[64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int i = 0; i < 64; i++) printf("%u%c", h[i], i % 16 == 15 ? '\n' : ' ');
  return 0;
}
