// Microbenchmark: the per-step floor of an LDS all-to-all exchange + s_barrier (gfx950).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int V>
__global__ void __launch_bounds__(1024) mb(float* out, unsigned long long* cyc, int iters) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  float x = out[tid];
  lds[tid] = x; lds[tid + 1024] = x;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const int par = it & 1;
    if constexpr (V == 0) {  // barrier only
      asm volatile("s_barrier" ::: "memory");
    } else if constexpr (V == 1) {  // write, wait, barrier
      lds[par * 1024 + tid] = x;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else if constexpr (V == 2) {  // write, wait, barrier, dependent read (b32)
      lds[par * 1024 + tid] = x;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      x = lds[par * 1024 + ((tid * 7 + 5) & 1023)] + 1.0f;
    } else if constexpr (V == 3) {  // ... dependent read b128
      lds[par * 1024 + tid] = x;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const float4 v = *reinterpret_cast<const float4*>(lds + par * 1024 + ((tid * 4) & 1023));
      x = (v.x + v.y) + (v.z + v.w);
    } else if constexpr (V == 4) {  // read-only dependent chain, no barrier (LDS latency)
      x = lds[((int)x & 1023)] + 1.0f;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[tid + 2048] = x;
  if ((tid & 63) == 0) cyc[tid >> 6] = t1 - t0;
}
int main() {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 1 << 12); hipMemset(out, 0, 1 << 20);
  const char* names[] = {"barrier only", "ds_write+wait+barrier", "+ dependent ds_read_b32", "+ dependent ds_read_b128", "ds_read latency chain"};
  int iters = 2000;
  for (int threads : {256, 512, 1024})
    for (int v = 0; v < 5; ++v) {
      for (int rep = 0; rep < 2; ++rep) {
        switch (v) {
          case 0: mb<0><<<1, threads, 16384>>>(out, cyc, iters); break;
          case 1: mb<1><<<1, threads, 16384>>>(out, cyc, iters); break;
          case 2: mb<2><<<1, threads, 16384>>>(out, cyc, iters); break;
          case 3: mb<3><<<1, threads, 16384>>>(out, cyc, iters); break;
          case 4: mb<4><<<1, threads, 16384>>>(out, cyc, iters); break;
        }
        hipDeviceSynchronize();
      }
      unsigned long long h[16]; hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double mx = 0; for (int i = 0; i < threads / 64; ++i) mx = h[i] > mx ? h[i] : mx;
      printf("%4d threads  %-28s %7.1f cycles/iter\n", threads, names[v], mx / iters);
    }
  return 0;
}
