// hmm355 — adjoint (vector-Jacobian product) of forward-backward's OUTPUTS on gfx950.
//
// The reference trains through HMMPyTorch.forward_backward with plain autograd over its
// log-space loops (hmm.py:89-130; HMMLayer training mode returns these posteriors,
// hmm_layer.py:119-121, and the supervised loss is a cross-entropy on them, :159-165).
// For output gradients Gp (posterior), Gf (forward = exp(log alpha)), Gb (backward =
// exp(log beta)) the adjoints of log alpha / log beta obey two linear recursions with
// per-step SOURCE terms, run here as two chains per sequence (pytorch_hmm_amd/autograd.py
// derives them and forms the sources and the final contractions):
//
//   W (adjoint of the forward recursion, in alpha's scaling; runs backward in time)
//       W_{T-1} = S_{T-1};   W_{t-1}[i] = S_{t-1}[i] + F_{t-1} * sum_j A[i][j] E_t[j] W_t[j]
//   Z (adjoint of the backward recursion, in beta's scaling; runs forward in time)
//       Z_0 = R_0;           Z_{t+1}[j] = R_{t+1}[j] + P_{t+1}[j],
//                            P_{t+1}[j] = G_{t+1} * E_{t+1}[j] * sum_i Z_t[i] A[i][j]
//
// with A = exp(log_P), E the chains' staged emissions, F / G the forward chains' step
// normalisers (1/c).  Outputs: W (B,T,N) and the propagated part P (B,T,N) of Z (P_0 = 0):
// Z = R + P is formed by the caller, and dL/d log_obs needs V * P on its own (forming it as
// V * (Z - R) would cancel).
//
// Kernel fb_adjoint<NP>: one workgroup per (sequence, chain), blockIdx.x = 2b + chain.
// NP/32 waves; wave w owns outputs o = 32w + (lane & 31), the two half-waves split the inputs
// (lane >> 5 = input half h, inputs NP/2*h .. +NP/2), the lane's matrix slice lives in VGPRs.
// Per step: the previous product input x (NP floats) is read from LDS by broadcast float4
// reads (each half-wave reads one address), NP/2 FMAs into four accumulators, one
// v_permlane32_swap joins the halves, the new value leaves to HBM (half 0 lanes, 128-B
// segments) and the next product input goes to the other LDS buffer: one s_barrier per
// step.  The per-step source / emission / scale loads are issued PD steps ahead into a
// register ring, so the chain never waits on HBM.
#include "common.h"

namespace hmm355 {

template <int NP>
struct AdjGeo {
  static constexpr int NW = NP / 32;      // waves
  static constexpr int NT = NW * kWave;   // threads
  static constexpr int HALF = NP / 2;     // inputs per lane
  static constexpr int XS = HALF + 4;     // LDS stride of an input half (the two half-wave
                                          // broadcast addresses fall in different banks)
  static constexpr int PD = 8;            // steps of loads in flight
};

struct AdjArgs {
  const float* E;      // (B,T,N) staged emissions
  const float* log_P;  // (N,N)
  const float* srcW;   // (B,T,N) sources S of the W chain
  const float* scW;    // (B,T)    F_t: scale of the step producing W_t (F[T-1] unused)
  const float* srcZ;   // (B,T,N) sources R of the Z chain
  const float* scZ;    // (B,T)    G_t: scale of the step producing Z_t (G[0] unused)
  float* W;            // (B,T,N)
  float* P;            // (B,T,N)
  int B, T, N;
};

template <int NP, int CH>
__device__ __forceinline__ void adj_chain(const AdjArgs& a, int b, float* lds) {
  using G = AdjGeo<NP>;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int o = 32 * w + (l & 31), h = l >> 5;
  const int T = a.T, N = a.N;
  const bool ook = o < N;
  const int oc = ook ? o : 0;
  // matrix slice: CH 0 (W): out i = o, inputs j;  CH 1 (Z): out j = o, inputs i
  float M[G::HALF];
#pragma unroll
  for (int k = 0; k < G::HALF; ++k) {
    const int i = G::HALF * h + k;
    const bool ok = ook && i < N;
    const float v = a.log_P[ok ? (CH == 0 ? (size_t)o * N + i : (size_t)i * N + o) : 0];
    M[k] = ok ? __expf(v) : 0.f;
  }
  const size_t rb = (size_t)b * T;
  // row of step q (q = 0 .. T-1): W runs t = T-1 .. 0, Z runs t = 0 .. T-1
  auto tau = [&](int q) { return CH == 0 ? T - 1 - q : q; };
  const float* src = CH == 0 ? a.srcW : a.srcZ;
  const float* sc = CH == 0 ? a.scW : a.scZ;
  float* out = CH == 0 ? a.W : a.P;
  float rs[G::PD], re[G::PD], rf[G::PD];
  auto load = [&](int q, int p) {
    const int qq = q < T ? q : T - 1;   // clamped: the tail re-loads the last row
    const size_t row = rb + tau(qq);
    rs[p] = src[row * N + oc];
    re[p] = a.E[row * N + oc];
    rf[p] = sc[row];
  };
#pragma unroll
  for (int p = 0; p < G::PD; ++p) load(p, p);

  // step 0: the chain's first value is its source (Z: P_0 = 0)
  float* xb = lds;  // [2][2][XS]
  {
    const float v = rs[0];
    if (h == 0 && ook) out[(rb + tau(0)) * N + o] = CH == 0 ? v : 0.f;
    const float x = CH == 0 ? re[0] * v : v;  // W: the product input is E_t * W_t
    if (h == 0) xb[(o / G::HALF) * G::XS + (o % G::HALF)] = ook ? x : 0.f;
    load(G::PD, 0);
  }
  __syncthreads();
  for (int q0 = 1; q0 < T; q0 += G::PD) {
#pragma unroll
    for (int pp = 0; pp < G::PD; ++pp) {
      const int q = q0 + pp;
      const int p = (1 + pp) % G::PD;  // ring slot of step q (step 0 used slot 0)
      if (q < T) {
        const float* xin = xb + ((q - 1) & 1) * 2 * G::XS + h * G::XS;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
        for (int k = 0; k < G::HALF; k += 4) {
          const float4 x4 = *reinterpret_cast<const float4*>(xin + k);
          a0 = fmaf(M[k], x4.x, a0);
          a1 = fmaf(M[k + 1], x4.y, a1);
          a2 = fmaf(M[k + 2], x4.z, a2);
          a3 = fmaf(M[k + 3], x4.w, a3);
        }
        float s0 = (a0 + a1) + (a2 + a3), s1 = s0;
        permlane32_swap(s0, s1);
        const float tot = s0 + s1;  // the full sum over inputs, in both halves
        float v, x;
        if (CH == 0) {
          v = rs[p] + rf[p] * tot;   // W_t = S_t + F_t * (A (E_{t+1} W_{t+1}))_o
          x = re[p] * v;
          if (h == 0 && ook) out[(rb + tau(q)) * N + o] = v;
        } else {
          const float pr = rf[p] * (re[p] * tot);  // P_t = G_t * E_t * (Z_{t-1} A)_o
          v = rs[p] + pr;                          // Z_t = R_t + P_t
          x = v;
          if (h == 0 && ook) out[(rb + tau(q)) * N + o] = pr;
        }
        if (h == 0) xb[(q & 1) * 2 * G::XS + (o / G::HALF) * G::XS + (o % G::HALF)] = ook ? x : 0.f;
        load(q + G::PD, p);
        __syncthreads();
      }
    }
  }
}

template <int NP>
__global__ void __launch_bounds__(AdjGeo<NP>::NT) fb_adjoint_kernel(AdjArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[2 * 2 * AdjGeo<NP>::XS];
  const int b = blockIdx.x >> 1;
  if (blockIdx.x & 1) adj_chain<NP, 1>(a, b, lds);
  else adj_chain<NP, 0>(a, b, lds);
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API int hmm355_fb_adjoint_f32(const float* E, const float* log_P, const float* src_w, const float* scale_w,
                                     const float* src_z, const float* scale_z, int B, int T, int N, float* W,
                                     float* P, void* stream) {
  if (B < 0 || N < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!E || !log_P || !src_w || !scale_w || !src_z || !scale_z || !W || !P) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40 || B > (1 << 30)) return HMM355_E_SHAPE;
  AdjArgs a{E, log_P, src_w, scale_w, src_z, scale_z, W, P, B, T, N};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int NP = pad_states(N);
  switch (NP) {
    case 64: hipLaunchKernelGGL(fb_adjoint_kernel<64>, dim3(2 * B), dim3(AdjGeo<64>::NT), 0, st, a); break;
    case 128: hipLaunchKernelGGL(fb_adjoint_kernel<128>, dim3(2 * B), dim3(AdjGeo<128>::NT), 0, st, a); break;
    default: hipLaunchKernelGGL(fb_adjoint_kernel<256>, dim3(2 * B), dim3(AdjGeo<256>::NT), 0, st, a); break;
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}
