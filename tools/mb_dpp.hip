// Microbenchmark: issue cost of the candidate inner-loop instructions on gfx950
// (8 waves per workgroup = 2 per SIMD, like the recursion kernels).
#include <hip/hip_runtime.h>
#include <stdio.h>
#define REP 256
template <int V>
__global__ void __launch_bounds__(1024) mb(float* out, unsigned long long* cyc, int iters) {
  float x = out[threadIdx.x], m0 = out[threadIdx.x + 1], a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  float m1 = m0 * 1.1f, m2 = m0 * 1.2f, m3 = m0 * 1.3f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < REP / 4; ++r) {
      if constexpr (V == 1) {
        asm volatile("v_fmac_f32_dpp %0, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %1, %4, %6 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %2, %4, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %3, %4, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(m0), "v"(m1), "v"(m2), "v"(m3));
      } else if constexpr (V == 2) {
        asm volatile("v_fmac_f32 %0, %4, %5\n v_fmac_f32 %1, %4, %6\n v_fmac_f32 %2, %4, %7\n v_fmac_f32 %3, %4, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(m0), "v"(m1), "v"(m2), "v"(m3));
      } else if constexpr (V == 3) {
        float t0_, t1_, t2_, t3_;
        asm volatile("v_mov_b32_dpp %0, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                     "v_mov_b32_dpp %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                     "v_mov_b32_dpp %2, %4 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_mov_b32_dpp %3, %4 row_newbcast:4 row_mask:0xf bank_mask:0xf"
                     : "=&v"(t0_), "=&v"(t1_), "=&v"(t2_), "=&v"(t3_) : "v"(x));
        asm volatile("v_fmac_f32 %0, %4, %5\n v_fmac_f32 %1, %6, %7\n v_fmac_f32 %2, %8, %9\n v_fmac_f32 %3, %10, %11"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(t0_), "v"(m0), "v"(t1_), "v"(m1), "v"(t2_), "v"(m2), "v"(t3_), "v"(m3));
      } else if constexpr (V == 4) {
        asm volatile("v_add_f32_dpp %0, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                     "v_add_f32_dpp %1, %4, %6 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                     "v_max3_f32 %2, %2, %0, %1\n"
                     "v_add_f32_dpp %0, %4, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_add_f32_dpp %1, %4, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                     "v_max3_f32 %3, %3, %0, %1"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(m0), "v"(m1), "v"(m2), "v"(m3));
      } else if constexpr (V == 5) {
        asm volatile("v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
      } else if constexpr (V == 6) {  // independent DPP fmac: 8 accumulators
        asm volatile("v_fmac_f32_dpp %0, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %1, %4, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %2, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %3, %4, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %0, %6, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %1, %6, %5 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %2, %6, %5 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f32_dpp %3, %6, %5 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(m0), "v"(m1));
      } else if constexpr (V == 7) {  // pk_fma with pre-broadcast operands
        asm volatile("v_pk_fma_f32 %0, %2, %3, %0\n v_pk_fma_f32 %1, %2, %3, %1"
                     : "+v"(*(double*)&a0), "+v"(*(double*)&a2) : "v"(*(double*)&x), "v"(*(double*)&m0));
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x + 1024] = a0 + a1 + a2 + a3;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}
static void run(int threads) {
  static float* out = nullptr; static unsigned long long* cyc = nullptr;
  if (!out) { hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 1 << 16); hipMemset(out, 0, 1 << 20); }
  int iters = 200;
  const char* names[] = {"", "fmac_dpp(4acc)", "fmac plain", "mov_dpp+fmac", "add_dpp+max3", "permlane16_swap", "fmac_dpp(indep x2)", "pk_fma (2 FMA/instr)"};
  int per[] = {0, REP, REP, 2 * REP, REP * 6 / 4, REP / 2, REP * 2, REP / 2};
  for (int v = 1; v <= 7; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (v) {
        case 1: mb<1><<<1, threads>>>(out, cyc, iters); break;
        case 2: mb<2><<<1, threads>>>(out, cyc, iters); break;
        case 3: mb<3><<<1, threads>>>(out, cyc, iters); break;
        case 4: mb<4><<<1, threads>>>(out, cyc, iters); break;
        case 5: mb<5><<<1, threads>>>(out, cyc, iters); break;
        case 6: mb<6><<<1, threads>>>(out, cyc, iters); break;
        case 7: mb<7><<<1, threads>>>(out, cyc, iters); break;
      }
      hipDeviceSynchronize();
    }
    unsigned long long h[16]; hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    int nw = threads / 64;
    double avg = 0; for (int i = 0; i < nw; ++i) avg += h[i]; avg /= nw;
    printf("%-22s cycles/instr/wave = %.2f  (%d waves, %d per SIMD)\n", names[v], avg / (double)iters / per[v], nw, nw / 4);
  }
}
int main() { run(256); run(512); run(1024); return 0; }
