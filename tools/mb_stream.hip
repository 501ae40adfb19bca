// Microbenchmark: per-CU streaming ingest (gfx950).  NWG workgroups (one per CU, 160 KiB
// dynamic LDS each so no two share a CU) of 512 threads each sweep their own contiguous
// region with float4 loads, D loads in flight per lane, in the tv kernels' two access shapes:
//   shape 0: 64-B row segments (16 rows x 64 B per wave-instruction, the tv alpha slice)
//   shape 1: 128-B row segments (8 rows x 128 B, the tv beta slice)
//   shape 2: 1 KiB contiguous per wave-instruction
// Prints GB/s per CU and chip-wide.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
template <int SHAPE, int D>
__global__ void __launch_bounds__(512) mb(const float* __restrict__ a, size_t per_wg_f4, float* out) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const float4* base = reinterpret_cast<const float4*>(a) + (size_t)blockIdx.x * per_wg_f4;
  // one "step" = 64 KiB = 4096 float4: rows of 128 floats (32 float4), 128 rows
  int off;
  if (SHAPE == 0) off = ((l >> 2) * 32) + (w * 4) + (l & 3);          // row l/4, quad 4w + l%4 (+16 rows per v)
  else if (SHAPE == 1) off = ((l >> 3) + 16 * w) * 32 + (l & 7);      // row 16w + l/8, quad l%8 (+8 quads per m)
  else off = w * 64 + l;
  const size_t steps = per_wg_f4 / 4096;
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t s = 0; s < steps; s += D) {
    float4 r[D][8];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        size_t o = (s + d) * 4096 + off;
        if (SHAPE == 0) o += v * 16 * 32;        // +16 rows
        else if (SHAPE == 1) o += (v & 3) * 8 + (v >> 2) * 8 * 32;
        else o += v * 512;
        r[d][v] = base[o];
      }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int v = 0; v < 8; ++v) { acc.x += r[d][v].x; acc.y += r[d][v].y; acc.z += r[d][v].z; acc.w += r[d][v].w; }
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}
template <int SHAPE, int D>
void run(const float* a, float* out, int nwg, size_t per_wg_f4) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(mb<SHAPE, D>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((mb<SHAPE, D>), dim3(nwg), dim3(512), 160 * 1024, 0, a, per_wg_f4, out);
  hipEventRecord(e0);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((mb<SHAPE, D>), dim3(nwg), dim3(512), 160 * 1024, 0, a, per_wg_f4, out);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  const double bytes = (double)nwg * per_wg_f4 * 16;
  printf("shape %d D %d nwg %3d: %.3f ms  %.1f GB/s per CU  %.2f TB/s\n", SHAPE, D, nwg, ms, bytes / ms / 1e6 / nwg, bytes / ms / 1e9);
}
int main() {
  const size_t per_wg_f4 = (size_t)131072000 / 16;  // 131 MB per workgroup (one tv chain)
  const int maxwg = 256;
  float* a; float* out;
  if (hipMalloc(&a, per_wg_f4 * 16 * maxwg) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&out, 64);
  hipMemset(a, 0, per_wg_f4 * 16 * maxwg);
  for (int nwg : {32, 64, 128, 256}) {
    run<0, 2>(a, out, nwg, per_wg_f4); run<0, 4>(a, out, nwg, per_wg_f4);
    run<1, 2>(a, out, nwg, per_wg_f4); run<1, 4>(a, out, nwg, per_wg_f4);
    run<2, 4>(a, out, nwg, per_wg_f4);
  }
  return 0;
}
