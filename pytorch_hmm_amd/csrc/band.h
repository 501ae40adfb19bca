// hmm355 — exact banded decomposition of the transition table (gfx950).
//
// The reference's matrices are dense N x N tables, but the ones its factories build
// (create_left_to_right_matrix, 'left_to_right_skip', 'circular'; utils.py:43-103) are a
// narrow band on top of a constant floor: log_P = log(P + 1e-8) puts the same value
// log(1e-8) in every structural zero of a row.  With r_i = min_o L[i][o] (the row floor)
// and, for each column o, the smallest window [lo_o, lo_o + W) of rows holding every entry
// L[i][o] != r_i, the recursions decompose EXACTLY:
//
//   Viterbi   max_i fl(d_i + L[i][o]) = max( max_i fl(d_i + r_i),  max_{k<W} fl(d_{lo+k} + L[lo+k][o]) )
//             (for i inside the window fl(d_i + r_i) <= fl(d_i + L[i][o]) because r_i is the row
//              minimum and rounding is monotone, so the first term may include them: the result
//              is the same set maximum, bit for bit, and its first argmax is recoverable —
//              vit_psi_kernel);
//   forward   sum_i y_i A[i][o] = sum_i y_i a_i + sum_{k<W} y_{lo+k} (A[lo+k][o] - a_{lo+k}),
//             a_i = exp(r_i)   (fp32, same tolerance contract as the dense sum);
//   backward  sum_o A[i][o] y_o = a_i sum_o y_o + sum_{k<W} (A[i][lo+k] - a_i) y_{lo+k}  with
//             row windows.
//
// One wide reduction (a wave sum or max) plus W products per state replaces the N-wide
// reduction per state, so a step costs O(N W) instead of O(N^2) and fits ONE wave (no
// workgroup barrier on the chain).  band_prep_kernel measures the structure on the device
// (no host round trip) and the recursion kernels branch on it; any matrix whose window
// exceeds kBandMax takes the dense path unchanged.
#pragma once
#include <stdlib.h>

#include "common.h"

namespace hmm355 {

constexpr int kBandMax = 8;   // widest window handled by the banded chains
constexpr int kBandN = 256;   // max states

struct BandDesc {
  int wc;                      // column-window width (forward / Viterbi); > kBandMax: dense
  int wr;                      // row-window width (backward); > kBandMax: dense
  int wcp, wrp;                // widths rounded up to 2 / 4 / 8 (the kernels' template width)
  float rfl[kBandN];           // row floor r_i = min_o L[i][o]
  float afl[kBandN];           // exp(r_i)
  int clo[kBandN];             // column window start (rows clo_o .. clo_o + wc - 1)
  int rlo[kBandN];             // row window start (columns rlo_i .. rlo_i + wr - 1)
  float cL[kBandN][kBandMax];  // L[clo_o + k][o]
  float cD[kBandN][kBandMax];  // exp(L[clo_o + k][o]) - afl[clo_o + k]
  float rD[kBandN][kBandMax];  // exp(L[i][rlo_i + k]) - afl[i]
};

__device__ __forceinline__ int band_pad(int w) { return w <= 2 ? 2 : (w <= 4 ? 4 : 8); }

// One workgroup of 256 threads.  Thread j handles row j and column j (j < N).
static __global__ void __launch_bounds__(256) band_prep_kernel(const float* __restrict__ L, int N, BandDesc* d) {
  __shared__ float rfl[kBandN];
  __shared__ int wmax[2];
  const int j = threadIdx.x;
  if (j < 2) wmax[j] = 0;
  if (j < N) {
    float m = INFINITY;
    for (int o = 0; o < N; ++o) m = fminf(m, L[(size_t)j * N + o]);
    rfl[j] = m;
  }
  __syncthreads();
  int clo = 0, rlo = 0;
  if (j < N) {
    // column j: rows whose entry differs from their floor
    int lo = N, hi = -1;
    for (int i = 0; i < N; ++i)
      if (L[(size_t)i * N + j] != rfl[i]) { lo = lo < i ? lo : i; hi = i; }
    clo = hi < 0 ? j : lo;
    atomicMax(&wmax[0], hi < 0 ? 1 : hi - lo + 1);
    // row j: columns whose entry differs from the row floor
    lo = N; hi = -1;
    for (int o = 0; o < N; ++o)
      if (L[(size_t)j * N + o] != rfl[j]) { lo = lo < o ? lo : o; hi = o; }
    rlo = hi < 0 ? j : lo;
    atomicMax(&wmax[1], hi < 0 ? 1 : hi - lo + 1);
  }
  __syncthreads();
  const int wc = wmax[0], wr = wmax[1];
  const int wcp = band_pad(wc), wrp = band_pad(wr);
  if (j == 0) { d->wc = wc; d->wr = wr; d->wcp = wcp; d->wrp = wrp; }
  const float rf = j < N ? rfl[j] : 0.f;
  d->rfl[j] = rf;
  d->afl[j] = j < N ? expf(rf) : 0.f;
  if (j < N) {
    // windows of the padded width, clamped to start inside [0, N - width]: entries inside a
    // window but outside the hull hold their true table value (the floor), which the
    // decomposition treats exactly either way; slots past N hold the neutral element
    if (wc <= kBandMax) {
      int lo = clo < N - wcp ? clo : N - wcp;
      lo = lo > 0 ? lo : 0;
      d->clo[j] = lo;
      for (int k = 0; k < kBandMax; ++k) {
        const int i = lo + k;
        const bool in = k < wcp && i < N;
        const float v = in ? L[(size_t)i * N + j] : -INFINITY;
        d->cL[j][k] = v;
        d->cD[j][k] = in ? expf(v) - expf(rfl[i]) : 0.f;
      }
    }
    if (wr <= kBandMax) {
      int lo = rlo < N - wrp ? rlo : N - wrp;
      lo = lo > 0 ? lo : 0;
      d->rlo[j] = lo;
      for (int k = 0; k < kBandMax; ++k) {
        const int o = lo + k;
        const bool in = k < wrp && o < N;
        d->rD[j][k] = in ? expf(L[(size_t)j * N + o]) - expf(rf) : 0.f;
      }
    }
  } else {
    d->clo[j] = 0;
    d->rlo[j] = 0;
    for (int k = 0; k < kBandMax; ++k) { d->cL[j][k] = -INFINITY; d->cD[j][k] = 0.f; d->rD[j][k] = 0.f; }
  }
}

// HMM355_DENSE=1 in the environment disables the banded chains (read per call; parity
// tests compare the two paths on the same inputs).
inline bool use_band() {
  const char* e = getenv("HMM355_DENSE");
  return !(e && e[0] == '1');
}

inline hipError_t launch_band_prep(const float* log_P, int N, BandDesc* d, hipStream_t st) {
  hipLaunchKernelGGL(band_prep_kernel, dim3(1), dim3(256), 0, st, log_P, N, d);
  return hipGetLastError();
}

}  // namespace hmm355
