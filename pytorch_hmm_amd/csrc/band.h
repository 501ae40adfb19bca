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
#include <stddef.h>
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
  // Toeplitz windows: every column's (row's) window is the same offset range around its
  // own index, slot k <-> state o + d0 + k, so the window values are lane shifts of the
  // state vector (DPP, no LDS round trip).  tw = 0 when no such range of width <= 3 exists.
  int tcd0, tcw;               // column windows (forward / Viterbi)
  int trd0, trw;               // row windows (backward)
  int uafl, pad_[3];           // 1: every row has the same floor (afl uniform)
  float tL[kBandN][4];         // L[o + tcd0 + k][o]                (-inf outside [0, N))
  float tD[kBandN][4];         // exp(L[o + tcd0 + k][o]) - afl[.]  (0 outside)
  float tR[kBandN][4];         // exp(L[i][i + trd0 + k]) - afl[i]  (0 outside)
};
// the host reads a plan's chain choice at these offsets (pytorch_hmm_amd/ops.py plan_info)
static_assert(offsetof(BandDesc, wc) == 0 && offsetof(BandDesc, wrp) == 12, "BandDesc header");
static_assert(offsetof(BandDesc, tcd0) == 4 * 7172 && offsetof(BandDesc, uafl) == 4 * 7176, "BandDesc Toeplitz fields");

// max over the 64 lanes, every lane receives it (DPP rows, then permlane swaps)
__device__ __forceinline__ float wave_max_dpp(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x124>(x));
  x = fmaxf(x, dpp_f<0x128>(x));
  return rows_max(x);
}

__device__ __forceinline__ int band_pad(int w) { return w <= 2 ? 2 : (w <= 4 ? 4 : 8); }

// One workgroup of 1024 threads.  Pass 1 (coalesced): wave w reads rows w, w+16, ...;
// the row minimum is the floor r_i; entries != r_i update the row's and their column's
// hull through LDS atomics (only the band's entries do).  Pass 2: thread j < N writes the
// window tables of column j and row j.
constexpr int kPrepThreads = 1024;
static __global__ void __launch_bounds__(kPrepThreads) band_prep_kernel(const float* __restrict__ L, int N,
                                                                        BandDesc* d) {
  __shared__ float rfl[kBandN];
  __shared__ int clo_s[kBandN], chi_s[kBandN], rlo_s[kBandN], rhi_s[kBandN];
  __shared__ int red[6];  // wc, wr, cd0, cd1, rd0, rd1
  __shared__ int dense_s;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  constexpr int NWV = kPrepThreads / 64;
  if (kAbl & 16) return;  // diagnostic builds only (tools/ablate.py)
  for (int j = tid; j < kBandN; j += kPrepThreads) { clo_s[j] = rlo_s[j] = 1 << 20; chi_s[j] = rhi_s[j] = -1; }
  if (tid == 0) { red[0] = red[1] = 0; red[2] = red[4] = 1 << 20; red[3] = red[5] = -(1 << 20); dense_s = 0; }
  __syncthreads();
  // all of this wave's row loads first (rows w, w + 16, ...), then one DPP min per row
  constexpr int RPW = kBandN / NWV;  // rows per wave (<= 16)
  constexpr int KB = kBandN / 64;
  float v[RPW][KB];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int i = w + NWV * rr;
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int o = l + 64 * k;
      v[rr][k] = (i < N && o < N) ? L[(size_t)i * N + o] : INFINITY;
    }
  }
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int i = w + NWV * rr;
    if (i >= N) break;
    float m = v[rr][0];
#pragma unroll
    for (int k = 1; k < KB; ++k) m = fminf(m, v[rr][k]);
    m = -wave_max_dpp(-m);
    if (l == 0) rfl[i] = m;
    // a row with more than kBandMax non-floor entries makes the table dense: record that
    // and skip its hull updates (a dense table would otherwise issue N^2 LDS atomics)
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int o = l + 64 * k;
      cnt += __popcll(__ballot(o < N && v[rr][k] != m));
    }
    if (cnt > kBandMax) {
      if (l == 0) dense_s = 1;
      continue;
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int o = l + 64 * k;
      if (o < N && v[rr][k] != m) {  // a band entry: update its row's and column's hull
        atomicMin(&rlo_s[i], o);
        atomicMax(&rhi_s[i], o);
        atomicMin(&clo_s[o], i);
        atomicMax(&chi_s[o], i);
      }
    }
  }
  __syncthreads();
  if (kAbl & 8) return;
  {
    // window widths and Toeplitz offset ranges: wave reductions, then one LDS atomic per wave
    int wcm = 0, wrm = 0, c0 = 1 << 20, c1 = -(1 << 20), r0 = 1 << 20, r1 = -(1 << 20);
    if (tid < N) {
      const int j = tid;
      if (chi_s[j] >= 0) { wcm = chi_s[j] - clo_s[j] + 1; c0 = clo_s[j] - j; c1 = chi_s[j] - j; } else { wcm = 1; }
      if (rhi_s[j] >= 0) { wrm = rhi_s[j] - rlo_s[j] + 1; r0 = rlo_s[j] - j; r1 = rhi_s[j] - j; } else { wrm = 1; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      wcm = max(wcm, __shfl_xor(wcm, off)); wrm = max(wrm, __shfl_xor(wrm, off));
      c0 = min(c0, __shfl_xor(c0, off)); c1 = max(c1, __shfl_xor(c1, off));
      r0 = min(r0, __shfl_xor(r0, off)); r1 = max(r1, __shfl_xor(r1, off));
    }
    if (l == 0 && tid < N) {
      atomicMax(&red[0], wcm); atomicMax(&red[1], wrm);
      atomicMin(&red[2], c0); atomicMax(&red[3], c1);
      atomicMin(&red[4], r0); atomicMax(&red[5], r1);
    }
  }
  __syncthreads();
  const int wc = dense_s ? kBandN : red[0], wr = dense_s ? kBandN : red[1];
  const int wcp = band_pad(wc), wrp = band_pad(wr);
  int cd0 = red[2], cd1 = red[3], rd0 = red[4], rd1 = red[5];
  if (cd1 < cd0) { cd0 = 0; cd1 = 0; }  // all-floor table: any range fits
  if (rd1 < rd0) { rd0 = 0; rd1 = 0; }
  const int tcw = (cd1 - cd0 + 1 <= 3 && cd0 >= -2 && cd1 <= 2) ? cd1 - cd0 + 1 : 0;
  const int trw = (rd1 - rd0 + 1 <= 3 && rd0 >= -2 && rd1 <= 2) ? rd1 - rd0 + 1 : 0;
  if (tid == 0) {
    d->wc = wc; d->wr = wr; d->wcp = wcp; d->wrp = wrp;
    d->tcd0 = cd0; d->tcw = tcw; d->trd0 = rd0; d->trw = trw;
    int u = 1;
    for (int i = 1; i < N; ++i) u &= rfl[i] == rfl[0];
    d->uafl = u;
  }
  if (tid >= kBandN) return;
  const int j = tid;
  const bool jin = j < N;
  const int jc = jin ? j : 0;
  const float rf = jin ? rfl[j] : 0.f;
  d->rfl[j] = rf;
  d->afl[j] = jin ? expf(rf) : 0.f;
  // every table value below is loaded unconditionally from a clamped index, so the loads
  // issue together (a guarded load per slot serialises one memory latency per slot)
  auto clampi = [&](int x) { return x < 0 ? 0 : (x >= N ? N - 1 : x); };
  // Toeplitz windows: slot k <-> state j + d0 + k
  float tl[4], trv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    tl[k] = L[(size_t)clampi(j + cd0 + k) * N + jc];
    trv[k] = L[(size_t)jc * N + clampi(j + rd0 + k)];
  }
  // general windows of the padded width, clamped to start inside [0, N - width]: entries
  // inside a window but outside the hull hold their true table value (the floor), which the
  // decomposition treats exactly either way; slots past N hold the neutral element
  const int hc = chi_s[jc] >= 0 && jin ? clo_s[jc] : j;
  int clo = hc < N - wcp ? hc : N - wcp;
  clo = clo > 0 ? clo : 0;
  const int hr = rhi_s[jc] >= 0 && jin ? rlo_s[jc] : j;
  int rlo = hr < N - wrp ? hr : N - wrp;
  rlo = rlo > 0 ? rlo : 0;
  float cv[kBandMax], rv[kBandMax];
#pragma unroll
  for (int k = 0; k < kBandMax; ++k) {
    cv[k] = L[(size_t)clampi(clo + k) * N + jc];
    rv[k] = L[(size_t)jc * N + clampi(rlo + k)];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = j + cd0 + k;
    const bool cin = jin && k < tcw && i >= 0 && i < N;
    d->tL[j][k] = cin ? tl[k] : -INFINITY;
    d->tD[j][k] = cin ? expf(tl[k]) - expf(rfl[clampi(i)]) : 0.f;
    const int o = j + rd0 + k;
    const bool rin = jin && k < trw && o >= 0 && o < N;
    d->tR[j][k] = rin ? expf(trv[k]) - expf(rf) : 0.f;
  }
  if (wc <= kBandMax) {
    d->clo[j] = clo;
#pragma unroll
    for (int k = 0; k < kBandMax; ++k) {
      const int i = clo + k;
      const bool in = jin && k < wcp && i < N;
      d->cL[j][k] = in ? cv[k] : -INFINITY;
      d->cD[j][k] = in ? expf(cv[k]) - expf(rfl[clampi(i)]) : 0.f;
    }
  }
  if (wr <= kBandMax) {
    d->rlo[j] = rlo;
#pragma unroll
    for (int k = 0; k < kBandMax; ++k) {
      const bool in = jin && k < wrp && rlo + k < N;
      d->rD[j][k] = in ? expf(rv[k]) - expf(rf) : 0.f;
    }
  }
}

// force_dense (a plan made with HMM355_PLAN_DENSE): both window widths are set beyond kBandMax
// after the measurement, so every recursion of that plan takes the dense chains (parity tests
// compare the two paths on the same inputs; the plan's tables are left as measured).
inline hipError_t launch_band_prep(const float* log_P, int N, BandDesc* d, hipStream_t st, bool force_dense = false) {
  hipLaunchKernelGGL(band_prep_kernel, dim3(1), dim3(kPrepThreads), 0, st, log_P, N, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && force_dense)
    e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d), 0x7fffffff, 2, st);  // wc, wr
  return e;
}

}  // namespace hmm355
