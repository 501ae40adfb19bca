// hmm355 — forward-backward on gfx950.
//
// Replaces HMMPyTorch.forward_backward (reference hmm.py:66-130): the two per-time-step
// Python loops (hmm.py:95-101 forward, :110-117 backward) and the posterior epilogue
// (:119-128).
//
// Kernel 1, fb_recur<NP>: one workgroup per (sequence, direction): blockIdx.x = 2b + dir,
//   the serial recursion of recur.h.  The recursion runs in the probability domain with
//   per-step normalisation (Rabiner scaling) instead of log-sum-exp: for the reference's
//   log-space update   la_t[j] = LSE_i(la_{t-1}[i] + logP[i,j]) + log_obs_t[j]
//   it keeps u_t = alpha_t / prod(c) with A = exp(logP), e_t = obs_t + 1e-8:
//       u_t[j] = (sum_i u_{t-1}[i] A[i,j]) / c_{t-1} * e_t[j],   c = sum_j u[j]
//   and the running log-scale LA_t = sum log c, so log alpha_t = log u_t + LA_t: one fp32
//   FMA per (i,j) cell instead of add + exp + max + add.  The backward pass is the same with
//   A^T and the emission applied before the product (hmm.py:113-115).
//
// With a banded plan and HMM355_FB_PAIR (N <= 128) both chains and the outputs run in ONE
// workgroup per sequence instead (fbpair.h, fb_pair_kernel): kernels 1 and 2 below are the
// dense-matrix path and the path that keeps the scaled rows for the adjoint (autograd.py).
//
// Kernel 2, fb_posterior<NP>: one wave per (b,t) row, grid-stride, HBM-bound:
//   posterior = (u*v)/sum(u*v) (scale-invariant) and the reference's compute_likelihood value
//   (forward = exp(log u + LA) and backward = exp(log v + LB) are written by kernel 1's flushes)
//   logsumexp_j(log(forward_{T-1}[j] + 1e-8)) (hmm.py:206) for t = T-1.
#include <atomic>

#include "recur.h"
#include "post.h"
#include "fbpair.h"

namespace hmm355 {

// per-NP launchers (fb_kern.h, instantiated in fb_np64/128/256.hip)
template <int NP>
hipError_t launch_fb(const RecArgs& fa, const RecArgs& fb, const PostArgs& pa, bool prep, hipStream_t st, int nfollow);
template <int NP>
hipError_t launch_fb_pair(const PairArgs& pa, int B, hipStream_t st);
// OBS_LOG: the row maxima M_t = max_j lo_t[j] (one wave per (b,t) row, grid-stride); the
// chains stage e_t = exp(lo_t - M_t) and add M_t to the log-scales (recur.h rec_stage /
// rec_flush), so log-emissions far below -87 (Gaussian log-densities at D = 80) do not
// underflow.  A row without a finite maximum gets M = 0 (its emissions stay exp(lo)).
__global__ void __launch_bounds__(256) row_max_kernel(const float* __restrict__ lo, int N, size_t rows,
                                                      float* __restrict__ m) {
  const int l = threadIdx.x & 63;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t row = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; row < rows; row += nw) {
    const float* src = lo + row * N;
    float v = -INFINITY;
    for (int j = l; j < N; j += 64) v = fmaxf(v, src[j]);
    v = wave_max_dpp2(v);
    if (l == 0) m[row] = (v > -INFINITY && v < INFINITY) ? v : 0.f;
  }
}

// Workspace layout (documented in include/hmm355.h for adjoint callers):
//   U (B,T,NP) | V (B,T,NP) | LA (B,T) | LB (B,T) | BandDesc | beta init (B,NP) | its scale (B)
//   | row maxima M (B,T) (OBS_LOG) | CA (B,T) | CB (B,T) (each step's normaliser, recur.h RecArgs::cs)
struct FbWs {
  float *U, *V, *LA, *LB, *binit, *bscale, *rmax, *CA, *CB;
  BandDesc* band;
  int* pub;  // (2B x kPubStride) the chains' published block counts (posterior followers, follow.h)
};
static size_t fb_ws_layout(int B, int T, int N, char* base, FbWs* w) {
  const size_t NP = pad_states(N);
  const size_t rows = (size_t)B * T;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += align_up(bytes, 256); return o; };
  const size_t oU = take(2 * rows * NP * sizeof(float));
  const size_t oL = take(2 * rows * sizeof(float));
  const size_t oD = take(sizeof(BandDesc));
  const size_t oI = take((size_t)B * NP * sizeof(float));
  const size_t oS = take((size_t)B * sizeof(float));
  const size_t oM = take(rows * sizeof(float));
  const size_t oC = take(2 * rows * sizeof(float));
  const size_t oP = take((size_t)2 * B * kPubStride * sizeof(int));
  if (w && base) {
    w->U = reinterpret_cast<float*>(base + oU);
    w->V = w->U + rows * NP;
    w->LA = reinterpret_cast<float*>(base + oL);
    w->LB = w->LA + rows;
    w->band = reinterpret_cast<BandDesc*>(base + oD);
    w->binit = reinterpret_cast<float*>(base + oI);
    w->bscale = reinterpret_cast<float*>(base + oS);
    w->rmax = reinterpret_cast<float*>(base + oM);
    w->CA = reinterpret_cast<float*>(base + oC);
    w->CB = w->CA + rows;
    w->pub = reinterpret_cast<int*>(base + oP);
  }
  return off;
}

// CUs of the current device, queried once per device (a relaxed atomic per slot)
static int fb_device_cus() {
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  int n = cus[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = -1;
    cus[dev].store(n, std::memory_order_relaxed);
  }
  return n > 0 ? n : 0;
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_fb_workspace_bytes(int B, int T, int N) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return 0;
  return fb_ws_layout(B, T, N, nullptr, nullptr);
}

HMM355_API int hmm355_fb_workspace_layout(int B, int T, int N, size_t* offsets) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return HMM355_E_SHAPE;
  if (!offsets) return HMM355_E_ARG;
  FbWs w;
  char* base = reinterpret_cast<char*>((uintptr_t)1 << 20);  // any 256-B aligned base: offsets only
  fb_ws_layout(B, T, N, base, &w);
  const void* piece[10] = {w.U, w.V, w.LA, w.LB, w.band, w.binit, w.bscale, w.rmax, w.CA, w.CB};
  for (int i = 0; i < 10; ++i) offsets[i] = (size_t)(reinterpret_cast<const char*>(piece[i]) - base);
  return HMM355_OK;
}

HMM355_API size_t hmm355_plan_bytes(int N) { return (N >= 1 && N <= 256) ? sizeof(BandDesc) : 0; }

HMM355_API int hmm355_plan_ex_f32(const float* log_P, int N, unsigned flags, void* plan, void* stream) {
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (!log_P || !plan || (flags & ~HMM355_PLAN_DENSE)) return HMM355_E_ARG;
  const hipError_t e = launch_band_prep(log_P, N, static_cast<BandDesc*>(plan), static_cast<hipStream_t>(stream),
                                        (flags & HMM355_PLAN_DENSE) != 0);
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_plan_f32(const float* log_P, int N, void* plan, void* stream) {
  return hmm355_plan_ex_f32(log_P, N, 0u, plan, stream);
}

HMM355_API int hmm355_plan_banded(const void* plan, void* stream) {
  if (!plan) return HMM355_E_ARG;
  int wcr[2];
  hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) e = hipMemcpy(wcr, plan, sizeof(wcr), hipMemcpyDeviceToHost);  // BandDesc wc, wr
  if (e != hipSuccess) return (int)e;
  return (wcr[0] <= kBandMax && wcr[1] <= kBandMax) ? 1 : 0;
}

HMM355_API int hmm355_forward_backward_plan_f32(const float* obs, int obs_mode, const float* log_P,
                                                const float* log_p0, const void* plan, const float* log_beta_T,
                                                int B, int T, int N, unsigned out_mask, float* posterior,
                                                float* forward, float* backward, float* loglik, float* lik_ref,
                                                void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || N < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!obs || !log_P || !log_p0 || !workspace) return HMM355_E_ARG;
  if ((out_mask & HMM355_FB_POSTERIOR) && !posterior) return HMM355_E_ARG;
  if ((out_mask & HMM355_FB_FORWARD) && !forward) return HMM355_E_ARG;
  if ((out_mask & HMM355_FB_BACKWARD) && !backward) return HMM355_E_ARG;
  if (obs_mode != HMM355_OBS_PROB && obs_mode != HMM355_OBS_LOG) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40) return HMM355_E_SHAPE;
  if (workspace_bytes < hmm355_fb_workspace_bytes(B, T, N)) return HMM355_E_WORKSPACE;
  const int NP = pad_states(N);
  FbWs w;
  fb_ws_layout(B, T, N, static_cast<char*>(workspace), &w);
  BandDesc* band = plan ? static_cast<BandDesc*>(const_cast<void*>(plan)) : w.band;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const float* binit = nullptr;
  const float* bscale = nullptr;
  if (log_beta_T) {
    switch (NP) {
      case 64: hipLaunchKernelGGL(beta_init_kernel<64>, dim3(B), dim3(64), 0, st, log_beta_T, N, w.binit, w.bscale); break;
      case 128: hipLaunchKernelGGL(beta_init_kernel<128>, dim3(B), dim3(64), 0, st, log_beta_T, N, w.binit, w.bscale); break;
      default: hipLaunchKernelGGL(beta_init_kernel<256>, dim3(B), dim3(64), 0, st, log_beta_T, N, w.binit, w.bscale); break;
    }
    const hipError_t e0 = hipGetLastError();
    if (e0 != hipSuccess) return (int)e0;
    binit = w.binit;
    bscale = w.bscale;
  }
  const float* rmax = nullptr;
  if (obs_mode == HMM355_OBS_LOG) {
    const size_t rows = (size_t)B * T;
    size_t blocks = (rows + 3) / 4;
    blocks = blocks < 4096 ? blocks : 4096;
    hipLaunchKernelGGL(row_max_kernel, dim3((unsigned)blocks), dim3(256), 0, st, obs, N, rows, w.rmax);
    const hipError_t e1 = hipGetLastError();
    if (e1 != hipSuccess) return (int)e1;
    rmax = w.rmax;
  }
  RecArgs fa{obs, log_P, log_p0, w.U, w.LA, loglik, B, T, N, obs_mode, NP, band, nullptr, nullptr, nullptr, rmax, nullptr};
  RecArgs fb{obs, log_P, log_p0, w.V, w.LB, nullptr, B, T, N, obs_mode, NP, band, binit, bscale, nullptr, rmax, nullptr};
  fa.cs = w.CA;  // each step's normaliser, by time (the adjoint's step factors, autograd.py)
  fb.cs = w.CB;
  hipStream_t st0 = static_cast<hipStream_t>(stream);
  if ((out_mask & HMM355_FB_PAIR) && plan && band && NP <= 128 && !log_beta_T &&
      (size_t)T * NP * sizeof(float) < ((size_t)1 << 31)) {
    // both chains of a sequence in one workgroup, outputs formed inside it (fbpair.h)
    PairArgs pa{fa, fb, posterior, forward, backward, lik_ref, out_mask};
    const hipError_t e = NP == 64 ? launch_fb_pair<64>(pa, B, st0) : launch_fb_pair<128>(pa, B, st0);
    return e == hipSuccess ? HMM355_OK : (int)e;
  }
  // the chains' flushes write forward / backward (exp(log u + LA), exp(log v + LB)) from their
  // LDS rows; the posterior pass then reads U / V and writes the posterior only
  fa.out_exp = (out_mask & HMM355_FB_FORWARD) ? forward : nullptr;
  fb.out_exp = (out_mask & HMM355_FB_BACKWARD) ? backward : nullptr;
  // HMM355_FB_PLAN_BANDED (the caller read hmm355_plan_banded(plan) == 1): the posterior and the
  // reference's likelihood are formed inside the chains' launch (follow.h) -- F follower
  // workgroups per sequence beside the 2B chains (two while 4B fit the chip, else one while 3B
  // do: a follower CU's write-through reads bound its rate)
  int nfollow = 0;
  if ((out_mask & HMM355_FB_PLAN_BANDED) && plan && (out_mask & HMM355_FB_POSTERIOR) && 3 * B <= fb_device_cus() &&
      (size_t)T * NP * 4 < ((size_t)1 << 31)) {
    fa.pub = fb.pub = w.pub;
    fa.lik_ref = lik_ref;
    nfollow = HMM355_FBF > 0 ? HMM355_FBF : (4 * B <= fb_device_cus() ? 2 : 1);
  }
  PostArgs pa{w.U, w.V, w.LA, w.LB, posterior, forward, backward, lik_ref, B, T, N,
              out_mask & (HMM355_FB_POSTERIOR)};
  hipError_t e;
  switch (NP) {
    case 64: e = launch_fb<64>(fa, fb, pa, plan == nullptr, st, nfollow); break;
    case 128: e = launch_fb<128>(fa, fb, pa, plan == nullptr, st, nfollow); break;
    default: e = launch_fb<256>(fa, fb, pa, plan == nullptr, st, nfollow); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_forward_backward_ex_f32(const float* obs, int obs_mode, const float* log_P,
                                              const float* log_p0, const float* log_beta_T, int B, int T, int N,
                                              unsigned out_mask, float* posterior, float* forward, float* backward,
                                              float* loglik, float* lik_ref, void* workspace,
                                              size_t workspace_bytes, void* stream) {
  return hmm355_forward_backward_plan_f32(obs, obs_mode, log_P, log_p0, nullptr, log_beta_T, B, T, N, out_mask,
                                          posterior, forward, backward, loglik, lik_ref, workspace,
                                          workspace_bytes, stream);
}

HMM355_API int hmm355_forward_backward_f32(const float* obs, int obs_mode, const float* log_P,
                                           const float* log_p0, int B, int T, int N, unsigned out_mask,
                                           float* posterior, float* forward, float* backward, float* loglik,
                                           float* lik_ref, void* workspace, size_t workspace_bytes,
                                           void* stream) {
  return hmm355_forward_backward_ex_f32(obs, obs_mode, log_P, log_p0, nullptr, B, T, N, out_mask, posterior, forward,
                                        backward, loglik, lik_ref, workspace, workspace_bytes, stream);
}

