// hmm355 — diagonal Gaussian-mixture emission scorer on gfx950.
//
// Replaces MixtureGaussianHMMLayer.get_observation_log_probs (reference
// mixture_gaussian.py:157-214, mixture LSE :141-155), whose (B,T,S,C,D) broadcast
// temporary is 10.5 GB fp32 at BASELINE config 3; also serves GaussianHMMLayer
// (hmm_layer.py:270-323) and HSMMLayer (hsmm.py:181-206) with C == 1.
//
// Per frame and component p = (s,c):
//     comp = -0.5 * (sum_d ((x_d - mu_pd) * w_pd)^2 + K_p) + log_w_p,   w = exp(-lv/2)
//     K_p  = sum_d lv_pd + D*log(2*pi)
//     lp[s] = log(clamp(sum_c exp(comp - m), 1e-8)) + m,   m = max_c comp (inf -> 0)
// gmm_prep (one thread per (p,d)) turns (means, log_vars, log_w) into the scales.
// gmm_score: a workgroup owns FT frames x floor(256/C) states.  Each lane owns one
// component: its 2*16*DCH scale/offset values live in VGPRs for the whole tile; the frame
// row is wave-uniform and read by scalar loads, so the inner loop is two v_fma_f32 per
// (frame, component, d) with one SGPR operand and no LDS or vector-memory traffic —
// VALU-FMA-bound (~1.2e5 FMA per frame at S=128, C=4, D=80) as §8(d) of the survey notes.
// Component values go through a 16-frame LDS tile for the LSE over c and leave as rows.
#include "common.h"

namespace hmm355 {

constexpr int kGmmThreads = 256;
constexpr int kGmmFrames = 32;  // frames per workgroup
constexpr int kGmmSub = 16;     // frames per LDS LSE tile

__global__ void gmm_prep_kernel(const float* __restrict__ means, const float* __restrict__ log_vars,
                                const float* __restrict__ log_w, float* __restrict__ prm, float* __restrict__ cst,
                                int P, int D, int DP) {
  const int p = blockIdx.x;
  if (p >= P) return;
  for (int d = threadIdx.x; d < DP; d += blockDim.x) {
    float w = 0.f, mw = 0.f;
    if (d < D) {
      const float lv = log_vars[(size_t)p * D + d];
      w = expf(-0.5f * lv);
      mw = -means[(size_t)p * D + d] * w;
    }
    prm[((size_t)p * 2 + 0) * DP + d] = w;
    prm[((size_t)p * 2 + 1) * DP + d] = mw;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += log_vars[(size_t)p * D + d];
    cst[2 * p + 0] = s + (float)((double)D * 1.8378770664093453);  // D*log(2*pi)
    cst[2 * p + 1] = log_w ? log_w[p] : 0.f;
  }
}

template <int DCH, bool FULL>
__global__ void __launch_bounds__(kGmmThreads) gmm_score_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ prm,
                                                               const float* __restrict__ cst,
                                                               float* __restrict__ out, int nframes, int D,
                                                               int S, int C, int mix_lse) {
  constexpr int DP = 16 * DCH;
  __shared__ float tile[kGmmSub][kGmmThreads];
  const int tid = threadIdx.x;
  const int spb = kGmmThreads / C;  // states per workgroup
  const int s0 = blockIdx.y * spb;
  const int sl = tid / C, c = tid - sl * C;
  const int s = s0 + sl;
  const bool active = sl < spb && s < S;
  const int p = active ? s * C + c : 0;

  float w[DP], mw[DP];
#pragma unroll
  for (int d = 0; d < DP; ++d) {
    w[d] = prm[((size_t)p * 2 + 0) * DP + d];
    mw[d] = prm[((size_t)p * 2 + 1) * DP + d];
  }
  const float kp = cst[2 * p], lw = cst[2 * p + 1];
  const int f_begin = blockIdx.x * kGmmFrames;

  for (int f0 = 0; f0 < kGmmFrames; f0 += kGmmSub) {
    for (int fi = 0; fi < kGmmSub; ++fi) {
      int frame = f_begin + f0 + fi;
      frame = frame < nframes ? frame : nframes - 1;  // uniform clamp (rows past the end are not written)
      const float* xr = x + (size_t)__builtin_amdgcn_readfirstlane(frame) * D;
      float q0 = 0.f, q1 = 0.f;
#pragma unroll
      for (int d = 0; d < DP; d += 2) {
        // FULL (D == 16*DCH): plain indices -> wide s_load_dwordx16; else clamp (w = 0 there)
        const float x0 = xr[FULL ? d : (d < D ? d : D - 1)];
        const float x1 = xr[FULL ? d + 1 : (d + 1 < D ? d + 1 : D - 1)];
        const float z0 = fmaf(x0, w[d], mw[d]);
        const float z1 = fmaf(x1, w[d + 1], mw[d + 1]);
        q0 = fmaf(z0, z0, q0);
        q1 = fmaf(z1, z1, q1);
      }
      tile[fi][tid] = -0.5f * ((q0 + q1) + kp) + lw;
    }
    __syncthreads();
    for (int pair = tid; pair < kGmmSub * spb; pair += kGmmThreads) {
      const int fi = pair / spb, sj = pair - fi * spb;
      const int frame = f_begin + f0 + fi;
      const int ss = s0 + sj;
      if (frame < nframes && ss < S) {
        float r;
        if (!mix_lse) {
          r = tile[fi][sj * C];
        } else {
          float m = -INFINITY;
          for (int cc = 0; cc < C; ++cc) m = fmaxf(m, tile[fi][sj * C + cc]);
          if (isinf(m)) m = 0.f;  // mixture_gaussian.py:144
          float e = 0.f;
          for (int cc = 0; cc < C; ++cc) e += expf(tile[fi][sj * C + cc] - m);
          r = logf(fmaxf(e, 1e-8f)) + m;  // :149-153
        }
        out[(size_t)frame * S + ss] = r;
      }
    }
    __syncthreads();
  }
}

template <int DCH>
static hipError_t launch_gmm(const float* x, const float* prm, const float* cst, float* out, int nframes, int D,
                             int S, int C, int mix_lse, hipStream_t st) {
  const int spb = kGmmThreads / C;
  dim3 grid((nframes + kGmmFrames - 1) / kGmmFrames, (S + spb - 1) / spb);
  if (D == 16 * DCH)
    hipLaunchKernelGGL((gmm_score_kernel<DCH, true>), grid, dim3(kGmmThreads), 0, st, x, prm, cst, out, nframes, D,
                       S, C, mix_lse);
  else
    hipLaunchKernelGGL((gmm_score_kernel<DCH, false>), grid, dim3(kGmmThreads), 0, st, x, prm, cst, out, nframes, D,
                       S, C, mix_lse);
  return hipGetLastError();
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_gmm_workspace_bytes(int D, int S, int C) {
  if (D < 1 || D > 128 || S < 1 || C < 1 || C > 256) return 0;
  const size_t P = (size_t)S * C, DP = (size_t)((D + 15) / 16) * 16;
  return align_up(P * 2 * DP * sizeof(float), 256) + align_up(P * 2 * sizeof(float), 256);
}

HMM355_API int hmm355_gmm_diag_logprob_f32(const float* x, const float* means, const float* log_vars,
                                           const float* log_w, int B, int T, int D, int S, int C, int mix_lse,
                                           float* out, void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || T < 0 || D < 1 || S < 1 || C < 1) return HMM355_E_ARG;
  if (D > 128 || C > 256 || (size_t)S * C > 65536) return HMM355_E_SHAPE;
  if ((size_t)B * T == 0) return HMM355_OK;
  if (!x || !means || !log_vars || !out || !workspace) return HMM355_E_ARG;
  if (!mix_lse && C != 1) return HMM355_E_ARG;
  if (workspace_bytes < hmm355_gmm_workspace_bytes(D, S, C)) return HMM355_E_WORKSPACE;
  const int DCH = (D + 15) / 16, DP = DCH * 16;
  const int P = S * C;
  float* prm = static_cast<float*>(workspace);
  float* cst = reinterpret_cast<float*>(static_cast<char*>(workspace) + align_up((size_t)P * 2 * DP * sizeof(float), 256));
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gmm_prep_kernel, dim3(P), dim3(64), 0, st, means, log_vars, log_w, prm, cst, P, D, DP);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int nframes = B * T;
  switch (DCH) {
    case 1: e = launch_gmm<1>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    case 2: e = launch_gmm<2>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    case 3: e = launch_gmm<3>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    case 4: e = launch_gmm<4>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    case 5: e = launch_gmm<5>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    case 6: e = launch_gmm<6>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    case 7: e = launch_gmm<7>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
    default: e = launch_gmm<8>(x, prm, cst, out, nframes, D, S, C, mix_lse, st); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}
