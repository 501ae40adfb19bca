// hmm355 — torch-CPU's summation order for the HSMM segment sums
// torch.sum(obs_log_probs[t:t+d, s]) (reference hsmm.py:273,285), on the device.
//
// ATen's cascade_sum (aten/src/ATen/native/cpu/SumKernel.cpp, fp32 accumulation) over a
// strided 1-D slice of n elements (oracle/hmm_oracle.c torch_sum_f32 restates it in full and
// tests/test_oracle.py pins it to torch.sum for n = 1..1024):
//   rows of 4 elements feed four lane accumulators; every 16 rows the level-0 accumulators are
//   added into level 1 and cleared (level 1 into level 2 every 256 rows, ...); at the end each
//   lane is ((l0 + l1) + l2) + l3, the n mod 4 tail goes into lane 0, and the result is
//   ((lane0 + lane1) + lane2) + lane3.
// For n <= 1024 (at most 256 rows) that is exactly, per lane k:
//   R_k = the running sum of the lane's elements since the last completed 16-row block
//         (from +0), A_k = fl(A_k + R_k) when a block completes (from +0), lane_k = fl(R_k + A_k)
// (the level-2 step at 256 rows adds +0's only; no accumulator is ever -0).  Every kernel
// that forms a segment sum keeps this (R, A) state; hsmm_fwd_kernel keeps it per register slot.
#pragma once
#include <hip/hip_runtime.h>

namespace hmm355 {

constexpr int kTsumBlockElems = 64;  // 16 rows of 4: one level-0 block

// torch-order sum of x(0) .. x(n-1) (time order), n <= 1024
template <typename Get>
__device__ __forceinline__ float tsum_strided(Get&& x, int n) {
  float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
  const int m = n & ~3;
  int i = 0;
  for (; i < m; i += 4) {
    r0 += x(i);
    r1 += x(i + 1);
    r2 += x(i + 2);
    r3 += x(i + 3);
    if (((i + 4) & (kTsumBlockElems - 1)) == 0) {  // a 16-row block completes
      c0 += r0; c1 += r1; c2 += r2; c3 += r3;
      r0 = r1 = r2 = r3 = 0.f;
    }
  }
  float a = r0 + c0;
  for (; i < n; ++i) a += x(i);
  return ((a + (r1 + c1)) + (r2 + c2)) + (r3 + c3);
}

// the contiguous slice (num_states == 1: stride 1): 8-wide vectors, four of them per row,
// the d mod 32 whole vectors into vector 0, the vectors summed lane-wise, then 0 + the
// d mod 8 tail scalars + the 8 lanes in order (n >= 8; shorter slices take tsum_strided).
// n <= 1024 keeps the same two-level (R, A) form per vector lane (32 lanes, 16-row blocks
// of 512 elements).
template <typename Get>
__device__ __forceinline__ float tsum_contig(Get&& x, int n) {
  if (n < 8) return tsum_strided(x, n);
  float R[32], C[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) R[k] = C[k] = 0.f;
  const int nv = n / 8, nr = nv / 4;
  for (int r = 0; r < nr; ++r) {
#pragma unroll
    for (int k = 0; k < 32; ++k) R[k] += x(32 * r + k);
    if (((r + 1) & 15) == 0) {
#pragma unroll
      for (int k = 0; k < 32; ++k) { C[k] += R[k]; R[k] = 0.f; }
    }
  }
  float L[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) L[k] = R[k] + C[k];
  for (int v = nr * 4; v < nv; ++v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) L[j] += x(8 * v + j);
  }
#pragma unroll
  for (int k = 1; k < 4; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) L[j] += L[8 * k + j];
  }
  float r = 0.f;
  for (int i = nv * 8; i < n; ++i) r += x(i);
#pragma unroll
  for (int j = 0; j < 8; ++j) r += L[j];
  return r;
}

}  // namespace hmm355
