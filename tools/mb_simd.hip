// diagnostic: which SIMD each wave of a 512-thread workgroup runs on (HW_ID, gfx9 layout:
// wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh [12], se [15:13])
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(1024) simd_of_wave(unsigned* out) {
  extern __shared__ float big[];
  unsigned id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = id;
  if (threadIdx.x == 0) big[0] = 1.f;
}
int main() {
  unsigned* d; hipMalloc(&d, 4 * 16 * 4);
  for (int nt : {256, 512, 1024}) {
    hipMemset(d, 0xff, 4 * 16 * 4);
    hipFuncSetAttribute((const void*)simd_of_wave, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(simd_of_wave, dim3(4), dim3(nt), 160 * 1024, 0, d);
    unsigned h[64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int b = 0; b < 4; ++b) {
      printf("nt=%d wg=%d simd:", nt, b);
      for (int w = 0; w < nt / 64; ++w) printf(" w%d->s%u(slot%u)", w, (h[b * 16 + w] >> 4) & 3, h[b * 16 + w] & 15);
      printf("\n");
    }
  }
  return 0;
}
