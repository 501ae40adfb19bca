/*
 * hmm355 — MI355X (gfx950) HMM inference core: the C ABI.
 *
 * This is the drop-in boundary for the hot path of crlotwhite/pytorch_hmm.  The reference
 * is pure Python over ATen (no FFI of its own); each entry point below replaces the
 * per-time-step Python loop of one reference routine (file:line into
 * /root/reference/pytorch_hmm) and is what a binding (ctypes, pybind11, or the
 * torch.library custom ops in pytorch_hmm_amd/ops.py) calls.
 *
 * Conventions (all entry points)
 *   - Plain device pointers and sizes; no framework types.  Every buffer is caller-owned
 *     device memory (hipMalloc / torch allocator); the library allocates nothing.
 *   - Dense row-major fp32, (B, T, N) = batch, time, states; states int64 (B, T).
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Launches are
 *     stream-ordered and asynchronous; there is no host synchronisation and no global
 *     mutable state, so calls are re-entrant and may run concurrently on different streams
 *     (and may be captured into a hipGraph).
 *   - Return 0 on success, a negative HMM355_E* code on a rejected argument (nothing is
 *     launched), or a positive hipError_t if a launch failed.  hmm355_strerror() names it.
 *   - Supported sizes: 1 <= N <= 256 states (padded internally to 64/128/256),
 *     T >= 1, B >= 0 (B == 0 is a no-op).
 */
#ifndef HMM355_H
#define HMM355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HMM355_OK 0
#define HMM355_E_ARG (-1)       /* null pointer or negative size                      */
#define HMM355_E_STATES (-2)    /* N outside [1, 256]                                  */
#define HMM355_E_SHAPE (-3)     /* T < 1, or a size product overflows                  */
#define HMM355_E_WORKSPACE (-4) /* workspace smaller than *_workspace_bytes() reports   */
#define HMM355_E_DURATION (-5)  /* HSMM max_duration outside [1, 1024]                  */

/* Emission encodings accepted by the recursions. */
#define HMM355_OBS_PROB 0   /* x is a probability: the kernel uses log(x + 1e-8) / x + 1e-8 (hmm.py:86,152) */
#define HMM355_OBS_LOG 1    /* x is already a log-emission (mixture_gaussian.py:354, hsmm.py:225)           */

/* forward_backward output mask bits */
#define HMM355_FB_POSTERIOR 1u   /* posterior (B,T,N)              hmm.py:120-126 */
#define HMM355_FB_FORWARD 2u     /* forward = exp(log alpha)        hmm.py:127     */
#define HMM355_FB_BACKWARD 4u    /* backward = exp(log beta)        hmm.py:128     */
/* Hint (forward_backward with a plan, no log_beta_T): the plan is banded in both directions
 * (hmm355_plan_banded() returned 1).  Both chains of a sequence then run in one workgroup and
 * form posterior / forward / backward inside it (csrc/fbpair.h): the scaled rows are not
 * written back in full, so the workspace does NOT hold U / V / LA / LB afterwards.  A wrong
 * hint still gives correct results (slower).  N <= 128; ignored otherwise. */
#define HMM355_FB_PAIR 0x100u
/* Hint (forward_backward with a plan): the caller read hmm355_plan_banded(plan) == 1.  The chains
 * then publish their rows as they go and extra workgroups (two per sequence while 4B workgroups
 * fit the device, else one) form the posterior (and the chain forms lik_ref) inside the chains'
 * own launch, instead of a pass after them (csrc/follow.h).  Needs HMM355_FB_POSTERIOR; ignored
 * when the 3B workgroups would not fit the device at once.  Passing it with a plan that is not banded is a caller error: posterior and
 * lik_ref come back NaN. */
#define HMM355_FB_PLAN_BANDED 0x200u

const char* hmm355_strerror(int code);
int hmm355_version(void);

/* ---------------------------------------------------------------------------------
 * Forward-backward.  Replaces HMMPyTorch.forward_backward (hmm.py:66-130) and the
 * likelihood of HMMPyTorch.compute_likelihood (hmm.py:186-211).
 *   obs        (B,T,N) emissions, encoding `obs_mode`
 *   log_P      (N,N) log transition matrix, exactly as the reference holds it
 *              (log(P/rowsum + 1e-8), hmm.py:39-42, or hmm_layer.py:84)
 *   log_p0     (N) log initial distribution (hmm.py:55 / hmm_layer.py:86)
 *   posterior, forward, backward  (B,T,N) outputs, written iff the mask bit is set
 *   loglik     (B) or NULL: log sum_j alpha_{T-1}[j] (the well-defined sequence
 *              log-likelihood the reference's exp() underflow hides)
 *   lik_ref    (B) or NULL: the reference's compute_likelihood value
 *              logsumexp_j(log(exp(log alpha_{T-1}[j]) + 1e-8))  (hmm.py:206)
 *   workspace  >= hmm355_fb_workspace_bytes(B,T,N) bytes of device memory
 * ------------------------------------------------------------------------------ */
size_t hmm355_fb_workspace_bytes(int B, int T, int N);
/* Same as hmm355_forward_backward_f32 with a custom terminal backward vector:
 *   log_beta_T (B,N) or NULL: log beta_{T-1} (NULL = 0, the reference's beta_{T-1} = 1,
 *              hmm.py:105).  With log_beta_T = log(dL/d log alpha_{T-1}) - log alpha_{T-1}
 *              the backward pass is the adjoint of the forward recursion for a loss L of
 *              alpha_{T-1}: dL/d log_obs_t = G * posterior_t with G = sum_j dL/d log alpha_{T-1,j}
 *              (pytorch_hmm_amd/autograd.py; replaces the reference's autograd through
 *              hmm.py:89-101 for compute_likelihood / HMMLayer.compute_loss, hmm_layer.py:144-173).
 * Workspace layout (256-B aligned pieces, in order): U (B,T,NP) scaled alpha rows | V
 * (B,T,NP) scaled beta rows | LA (B,T) | LB (B,T) | BandDesc (hmm355_plan_bytes(N)) |
 * (B,NP) | (B) | (B,T) | CA (B,T) | CB (B,T); alpha_t = U_t exp(LA_t), beta_t = V_t exp(LB_t),
 * NP = N padded to 64/128/256.  CA / CB are the steps' normalisers by time:
 * U_{t+1} = (A^T U_t) e_{t+1} / CA_t  (t <= T-2)  and  V_{t-1} = A (e_t V_t) / CB_t  (t >= 1),
 * A = exp(log_P) -- the chains do not normalise every row to sum 1 (the dense chain applies a
 * scale predicted a step ahead), so an adjoint takes its step factors from CA / CB.  With obs_mode == HMM355_OBS_LOG
 * the chains use the shifted emissions e_t = exp(obs_t - M_t), M_t = max_j obs_t[j] (a row
 * without a finite maximum: M_t = 0), and LA / LB carry the shifts, so log-emissions far
 * below -87 do not underflow; U and V are the rows of that shifted recursion. */
/* Byte offsets of the workspace pieces above, in order U, V, LA, LB, BandDesc, beta init, its
 * scale, row maxima M, CA, CB (offsets[10]), for callers that read U / V / LA / LB / CA / CB back
 * (pytorch_hmm_amd/autograd.py); 0 or an HMM355_E_* code. */
int hmm355_fb_workspace_layout(int B, int T, int N, size_t* offsets);
int hmm355_forward_backward_ex_f32(const float* obs, int obs_mode, const float* log_P,
                                   const float* log_p0, const float* log_beta_T, int B, int T, int N,
                                   unsigned out_mask, float* posterior, float* forward,
                                   float* backward, float* loglik, float* lik_ref, void* workspace,
                                   size_t workspace_bytes, void* stream);
int hmm355_forward_backward_f32(const float* obs, int obs_mode, const float* log_P,
                                const float* log_p0, int B, int T, int N, unsigned out_mask,
                                float* posterior, float* forward, float* backward,
                                float* loglik, float* lik_ref, void* workspace,
                                size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Adjoint of forward-backward's outputs (posterior / forward / backward).  Replaces the
 * reference's autograd through its log-space loops (hmm.py:89-130) when a loss of the
 * posteriors is back-propagated (HMMLayer training mode, hmm_layer.py:119-121; the
 * supervised cross-entropy of compute_loss, :159-165).  Two linear chains per sequence:
 *   W_{T-1} = Sw_{T-1};  W_{t-1}[i] = Sw_{t-1}[i] + Fw_{t-1} * sum_j A[i][j] E_t[j] W_t[j]
 *   Z_0 = Sz_0;          Z_{t+1}[j] = Sz_{t+1}[j] + P_{t+1}[j],
 *                        P_{t+1}[j] = Fz_{t+1} * E_{t+1}[j] * sum_i Z_t[i] A[i][j]
 * with A = exp(log_P).  E, src_w (Sw), src_z (Sz) are (B,T,N); scale_w (Fw), scale_z (Fz)
 * are (B,T) (Fw[T-1] and Fz[0] are not read).  Outputs W (B,T,N) and P (B,T,N), P_0 = 0.
 * pytorch_hmm_amd/autograd.py (ForwardBackwardFn) forms the sources from the output
 * gradients and the stored scaled rows, and the parameter gradients from W and Z.
 * ------------------------------------------------------------------------------ */
int hmm355_fb_adjoint_f32(const float* E, const float* log_P, const float* src_w,
                          const float* scale_w, const float* src_z, const float* scale_z,
                          int B, int T, int N, float* W, float* P, void* stream);

/* ---------------------------------------------------------------------------------
 * Transition plan: the banded decomposition of log_P (csrc/band.h) measured once into
 * caller-owned device memory (hmm355_plan_bytes(N) bytes), for callers whose matrix is fixed
 * across calls (HMMPyTorch computes log_P once in __init__, hmm.py:39-42).  The *_plan_f32
 * entry points use it instead of re-measuring the matrix on every call; plan == NULL
 * behaves exactly as the plain entry points.  A plan is valid for the log_P it was made
 * from; the results are identical with or without it.
 * ------------------------------------------------------------------------------ */
size_t hmm355_plan_bytes(int N);
int hmm355_plan_f32(const float* log_P, int N, void* plan, void* stream);
/* As hmm355_plan_f32 with flags.  HMM355_PLAN_DENSE: the plan selects the dense chains for every
 * recursion whatever the matrix's structure (hmm355_plan_banded then reads 0): the two chain
 * families give the same results, and parity tests run both on one matrix. */
#define HMM355_PLAN_DENSE 0x1u
int hmm355_plan_ex_f32(const float* log_P, int N, unsigned flags, void* plan, void* stream);
/* 1 if the plan selects banded chains for both the forward and the backward recursion (the
 * condition for HMM355_FB_PAIR), 0 if not, < 0 on error.  Synchronous: waits for `stream`
 * and copies a few bytes of the plan to the host (call once per plan, not per step). */
int hmm355_plan_banded(const void* plan, void* stream);
int hmm355_forward_backward_plan_f32(const float* obs, int obs_mode, const float* log_P,
                                     const float* log_p0, const void* plan,
                                     const float* log_beta_T, int B, int T, int N,
                                     unsigned out_mask, float* posterior, float* forward,
                                     float* backward, float* loglik, float* lik_ref,
                                     void* workspace, size_t workspace_bytes, void* stream);
int hmm355_viterbi_plan_f32(const float* obs, int obs_mode, const float* log_P, const float* init,
                            const void* plan, int B, int T, int N, int64_t* states,
                            float* log_delta, float* final_score, void* workspace,
                            size_t workspace_bytes, void* stream);
/* Viterbi with flags.  HMM355_VIT_PLAN_BANDED: the caller read hmm355_plan_banded(plan) == 1 for
 * this plan.  For N > 64 the decode then finishes inside the chain's own launch (csrc/follow.h):
 * one extra workgroup per sequence forms log(x + 1e-8) of the emissions ahead of the chain
 * (OBS_PROB), composes the 64-step chunk maps from the psi rows the chain publishes, and
 * backtraces the path once the chain is done -- one launch instead of four.  Ignored when the 2B
 * workgroups would not fit the device at once or T exceeds what the follower's LDS holds
 * (~32k steps at N <= 128, ~16k at N <= 256).  Passing the flag with a plan that is not banded
 * is a caller error: the states come back as -1 and the final score as NaN. */
#define HMM355_VIT_PLAN_BANDED 0x1u
/* HMM355_VIT_PLAN_DENSE: the caller read hmm355_plan_banded(plan) == 0.  Then, for N <= 128, the
 * argmax pointers of each 64-step chunk are computed while the chain still runs, by workgroups
 * of the chain's own launch on the CUs the chain leaves idle (they follow the rows the chain
 * has flushed; a chunk they did not finish is computed by the pass after the chain, so the
 * result never depends on their timing).  Without the flag the pointers are computed after the
 * chain.  With HMM355_OBS_PROB the emissions' log(x + 1e-8) is formed in one full-tensor pass
 * into the workspace first.  The flag with a banded plan only costs the idle launch. */
#define HMM355_VIT_PLAN_DENSE 0x2u
int hmm355_viterbi_plan_ex_f32(const float* obs, int obs_mode, const float* log_P, const float* init,
                               const void* plan, unsigned flags, int B, int T, int N, int64_t* states,
                               float* log_delta, float* final_score, void* workspace,
                               size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Viterbi.  Replaces HMMPyTorch.viterbi_decode (hmm.py:132-184) and
 * MixtureGaussianHMMLayer._viterbi_decode (mixture_gaussian.py:290-338).
 *   init       (N) additive t=0 vector: log_p0 (hmm.py:159), or -log(S) per state
 *              (mixture_gaussian.py:312; lp + (-c) == lp - c exactly in fp32)
 *   states     (B,T) int64: backtraced path, first index on ties (hmm.py:167,174)
 *   log_delta  (B,T,N) fp32: the trellis the reference returns as `scores`
 *   final_score (B) or NULL: max_j delta_{T-1}[j] (mixture_gaussian.py:327)
 *   workspace  >= hmm355_viterbi_workspace_bytes(B,T,N) bytes
 * Given identical fp32 log-emissions and log_P the result is bit-identical to the
 * reference's (every delta is one fp32 add of an exact max).
 * ------------------------------------------------------------------------------ */
size_t hmm355_viterbi_workspace_bytes(int B, int T, int N);
/* The size for one emission encoding: HMM355_OBS_LOG decodes need no log-emission buffer
 * (B*T*N*4 bytes less); hmm355_viterbi_workspace_bytes is the HMM355_OBS_PROB (larger) size. */
size_t hmm355_viterbi_workspace_bytes_ex(int B, int T, int N, int obs_mode);
int hmm355_viterbi_f32(const float* obs, int obs_mode, const float* log_P, const float* init,
                       int B, int T, int N, int64_t* states, float* log_delta,
                       float* final_score, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ---------------------------------------------------------------------------------
 * Diagonal-covariance Gaussian-mixture emission scorer.  Replaces
 * MixtureGaussianHMMLayer.get_observation_log_probs for covariance_type='diag'
 * (mixture_gaussian.py:157-214, LSE of :141-155) and, with C == 1 and log_w == 0,
 * GaussianHMMLayer._compute_gaussian_log_probs 'diag'/'full' (hmm_layer.py:300-321) and
 * HSMMLayer.get_observation_log_probs (hsmm.py:181-206).
 *   x (B,T,D); means, log_vars (S,C,D); log_w (S,C) = log(clamp(softmax(w),1e-8));
 *   out (B,T,S) = LSE_c[ -0.5*(sum_d (x-mu)^2/exp(lv) + sum_d lv + D*log(2pi)) + log_w ].
 * `mix_lse` selects the reference's mixture LSE (clamped sum, :141-155); with C == 1 pass 0
 * to get the plain component log-density.  Supported: 1 <= D <= 8192, 1 <= C <= 256,
 * 1 <= S*C <= 65536, B*T < 2^31.  workspace >= hmm355_gmm_workspace_bytes(B,T,D,S,C)
 * (per-component scales and an fp64 copy of the frames; written by the call).  The
 * quadratic form is accumulated in fp64 and each score rounded to fp32 once, so the scores
 * are as close to the exact value as the reference's fp32 ones (its Viterbi paths decode
 * identically at BASELINE config 3).
 * ------------------------------------------------------------------------------ */
size_t hmm355_gmm_workspace_bytes(int B, int T, int D, int S, int C);
int hmm355_gmm_diag_logprob_f32(const float* x, const float* means, const float* log_vars,
                                const float* log_w, int B, int T, int D, int S, int C,
                                int mix_lse, float* out, void* workspace,
                                size_t workspace_bytes, void* stream);
/* ---------------------------------------------------------------------------------
 * HSMM segment Viterbi.  Replaces HSMMLayer.viterbi_decode_hsmm / _viterbi_decode_single
 * (hsmm.py:208-354), reproducing its candidate order (s' outer, d' inner, strict >), its
 * fp32 addition order ((prev + logT) + obs_sum) + dur and torch-CPU's summation order for
 * obs_sum, so paths are bit-identical given identical fp32 inputs.
 *   lp (B,T,S) obs log-probs; dur_lp (S,Dmax) = log(p_dur + 1e-8); log_T (S,S)
 *   states (B,T) int64; scores (B) fp32
 *   1 <= S <= 1024 (HMM355_E_STATES beyond), 1 <= Dmax <= 1024 (HMM355_E_DURATION beyond).
 *   obs_sum follows ATen's cascade_sum order (csrc/tsum.h; it changes from 72 frames on).
 *   S = 1: the slice is contiguous and takes torch's vectorised order; the path is all 0.
 *   Frames the walk never reaches (no predecessor path: every score -inf) are written 0,
 *   the reference's torch.zeros initial value.
 *   S <= 64 with Dmax <= 71, or S <= 128 with Dmax <= 63: one workgroup per sequence keeps
 *   every open segment in registers and the tables in LDS (csrc/hsmm.hip); larger sizes take
 *   the general form (csrc/hsmm_wide.hip: M history and segment sums in the workspace,
 *   B*T*S*(Dmax+1) floats).
 * ------------------------------------------------------------------------------ */
size_t hmm355_hsmm_workspace_bytes(int B, int T, int S, int Dmax);
int hmm355_hsmm_viterbi_f32(const float* lp, const float* dur_lp, const float* log_T, int B,
                            int T, int S, int Dmax, int64_t* states, float* scores,
                            void* workspace, size_t workspace_bytes, void* stream);
/* Kernel-form flags of the segment recursions (results are identical in every form; parity
 * tests compare them):
 *   HMM355_FORM_GENERAL      the general form (workspace tables) whatever the size
 *   HMM355_FORM_SERIAL_WALK  HSMM only: the serial backtrace walk instead of the chunked one
 * The _ex workspace queries take the same flags. */
#define HMM355_FORM_GENERAL 0x1u
#define HMM355_FORM_SERIAL_WALK 0x2u
size_t hmm355_hsmm_workspace_bytes_ex(int B, int T, int S, int Dmax, unsigned flags);
int hmm355_hsmm_viterbi_ex_f32(const float* lp, const float* dur_lp, const float* log_T, int B,
                               int T, int S, int Dmax, unsigned flags, int64_t* states,
                               float* scores, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Recursions with one transition matrix per time step (NeuralHMM).  Replace
 * NeuralHMM._forward_algorithm / _backward_algorithm and the posterior epilogue of
 * NeuralHMM.forward (neural.py:391-461) and NeuralHMM.viterbi_decode (neural.py:463-511).
 *   log_obs (B,T,N): log-emissions (the observation network's output, any finite values);
 *   log_A: log transition matrices, element (b,k,i,j) at
 *          log_A[b*a_bstride + k*a_tstride + i*N + j] (strides in elements; pass 0, 0 for one
 *          (N,N) matrix shared by every step: neural.py:383-385).  Forward and Viterbi step t
 *          use matrix k = t-1 (neural.py:419-427, :489-496), backward step t matrix k = t
 *          (neural.py:449-458); matrix T-1 is never read.  Entries must be <= ~88 (exp range);
 *          -inf is allowed.
 *   log_p0 / init (N): log initial probabilities (neural.py:388-389, :478-479).
 * FB outputs as hmm355_forward_backward_f32 (posterior = exp(log_post), forward =
 * exp(log_forward), backward = exp(log_backward), loglik = LSE(log_forward[T-1]), lik_ref =
 * the reference's compute_likelihood LSE(log(forward[T-1] + 1e-8)), neural.py:513-519).
 * Viterbi: states (B,T) int64, log_delta (B,T,N) fp32 (bit-identical to the reference's
 * fp32 sums; first index on ties).  1 <= N <= 256.
 * Workspaces >= hmm355_tv_fb_workspace_bytes / hmm355_tv_viterbi_workspace_bytes(B,T,N).
 * ------------------------------------------------------------------------------ */
size_t hmm355_tv_fb_workspace_bytes(int B, int T, int N);
int hmm355_tv_forward_backward_f32(const float* log_obs, const float* log_A, long long a_bstride,
                                   long long a_tstride, const float* log_p0, int B, int T, int N,
                                   unsigned out_mask, float* posterior, float* forward,
                                   float* backward, float* loglik, float* lik_ref,
                                   void* workspace, size_t workspace_bytes, void* stream);
/* As hmm355_tv_forward_backward_f32 with an optional terminal backward vector log_beta_T
 * (B,N) (NULL = 0, the reference's beta_{T-1}); used by the adjoint (see
 * hmm355_forward_backward_ex_f32).  Workspace layout: U | V (B,T,NP) | LA | LB (B,T) |
 * E (B,T,NP) = exp(log_obs - M) | M (B,T) | CA | CB (B,T) | ..., pieces 256-B aligned,
 * NP = 64/128/256; log alpha = log U + LA, log beta = log V + LB. */
int hmm355_tv_forward_backward_ex_f32(const float* log_obs, const float* log_A, long long a_bstride,
                                      long long a_tstride, const float* log_p0,
                                      const float* log_beta_T, int B, int T, int N,
                                      unsigned out_mask, float* posterior, float* forward,
                                      float* backward, float* loglik, float* lik_ref,
                                      void* workspace, size_t workspace_bytes, void* stream);
/* Adjoint of the time-varying forward-backward outputs (NeuralHMM training through its
 * posteriors, neural.py:355-461): hmm355_fb_adjoint_f32's two chains with matrix k
 * (exp(log_A[b,k]), linking steps k and k+1, strides as above) in place of one log_P.  E, the
 * sources and W / P are (B,T,N) with row stride N; scale_w / scale_z (B,T). */
int hmm355_tv_fb_adjoint_f32(const float* E, const float* log_A, long long a_bstride,
                             long long a_tstride, const float* src_w, const float* scale_w,
                             const float* src_z, const float* scale_z, int B, int T, int N,
                             float* W, float* P, void* stream);
size_t hmm355_tv_viterbi_workspace_bytes(int B, int T, int N);
int hmm355_tv_viterbi_f32(const float* log_obs, const float* log_A, long long a_bstride,
                          long long a_tstride, const float* init, int B, int T, int N,
                          int64_t* states, float* log_delta, void* workspace,
                          size_t workspace_bytes, void* stream);
/* ---------------------------------------------------------------------------------
 * Explicit-duration (semi-Markov) HMM, indexed by segment END time.  Replace
 * SemiMarkovHMM.viterbi_decode (semi_markov.py:455-570), the segment observation score
 * SemiMarkovHMM._compute_segment_observation_logprob (semi_markov.py:411-435) and the
 * segment forward SemiMarkovHMM._unsupervised_forward (semi_markov.py:308-383, whose
 * intended logaddexp recursion this computes; the reference raises TypeError there).
 *
 * hmm355_semimarkov_quad_f32: per-frame Mahalanobis term
 *   quad[b,t,s] = sum_k ((x[b,t,k] - mu[s,k])^2) / var[s,k]   (k ascending, fp32)
 *   x (B,T,Df); means_t, vars_t are (Df,S) (transposed); var = exp(logvar) formed by the
 *   caller with the reference's torch op (semi_markov.py:418).
 * hmm355_semimarkov_viterbi_f32 / _forward_f32: the segment recursions over
 *   quad (B,T,S); seg_const (S) or NULL.  Segment score of frames [st, t] in state s:
 *     seg_const != NULL (gaussian): seg_const[s] - 0.5 * Q   (the reference adds the
 *        constant -0.5*sum(logvar) - 0.5*D*log(2 pi) once per SEGMENT, :420-424)
 *     seg_const == NULL (additive, observation_model='neural'): Q
 *   with Q = quad[st] + quad[st+1] + ... + quad[t] (left to right).
 *   log_init (S) = log(softmax(initial_logits) + 1e-8); log_T (S,S) = log(softmax(
 *   transition_logits) + 1e-8) (self-transitions are excluded by the recursion);
 *   dur_lp (S,Dmax) = DurationModel log-probabilities for d = 1..Dmax.
 * Viterbi outputs: segments right-aligned in (B,T) int64 seg_states / seg_durs, the last
 *   seg_count[b] entries of row b in time order; scores (B) = best final delta.  Candidate
 *   order (s' outer, d' inner, strict >) and fp32 addition order ((prev + logT) then
 *   (best + obs) + dur) are the reference's, so segmentations are bit-identical given
 *   identical fp32 quad/table inputs.
 * Forward outputs: log_prob (B) = LSE over (s,d) of log alpha[T-1]; log_alpha (B,T,S,Dmax)
 *   optional (NULL = not written), -inf where a segment is impossible.
 * 1 <= S <= 1024, 1 <= Dmax <= 1024.  S <= 64 with Dmax <= 63 runs the register form; larger
 * sizes the general form (its workspace holds a (B,T,S,Dmax) fp32 segment-score table:
 * hmm355_semimarkov_workspace_bytes).
 * ------------------------------------------------------------------------------ */
size_t hmm355_semimarkov_workspace_bytes(int B, int T, int S, int Dmax);
int hmm355_semimarkov_quad_f32(const float* x, const float* means_t, const float* vars_t, int B,
                               int T, int Df, int S, float* quad, void* stream);
int hmm355_semimarkov_viterbi_f32(const float* quad, const float* seg_const,
                                  const float* log_init, const float* log_T,
                                  const float* dur_lp, int B, int T, int S, int Dmax,
                                  int64_t* seg_states, int64_t* seg_durs, int* seg_count,
                                  float* scores, void* workspace, size_t workspace_bytes,
                                  void* stream);
int hmm355_semimarkov_forward_f32(const float* quad, const float* seg_const,
                                  const float* log_init, const float* log_T,
                                  const float* dur_lp, int B, int T, int S, int Dmax,
                                  float* log_alpha, float* log_prob, void* workspace,
                                  size_t workspace_bytes, void* stream);
/* The same with kernel-form flags (HMM355_FORM_GENERAL). */
size_t hmm355_semimarkov_workspace_bytes_ex(int B, int T, int S, int Dmax, unsigned flags);
int hmm355_semimarkov_viterbi_ex_f32(const float* quad, const float* seg_const,
                                     const float* log_init, const float* log_T,
                                     const float* dur_lp, int B, int T, int S, int Dmax,
                                     unsigned flags, int64_t* seg_states, int64_t* seg_durs,
                                     int* seg_count, float* scores, void* workspace,
                                     size_t workspace_bytes, void* stream);
int hmm355_semimarkov_forward_ex_f32(const float* quad, const float* seg_const,
                                     const float* log_init, const float* log_T,
                                     const float* dur_lp, int B, int T, int S, int Dmax,
                                     unsigned flags, float* log_alpha, float* log_prob,
                                     void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Streaming decoders of StreamingHMMProcessor, one chunk of B independent streams.
 *   emis (B,T,N): the emission network's log-probabilities; log_T (N,N) =
 *   log(softmax(transition_logits) + 1e-8).  1 <= N <= 256 (log_T LDS-resident up to 128; above
 *   that its rows are read from global memory per step).
 * hmm355_stream_greedy_f32 replaces _greedy_decode (streaming.py:267-320):
 *   s_t = argmax_j (log_T[s_{t-1}][j] + emis[t][j]), first index on ties; the chain starts
 *   from prev_state[b], or, when prev_state[b] < 0 (the stream's first chunk), from
 *   emis[0][j] - log_n with log_n = log(N) in fp32.  states (B,T) int64, scores (B,T) the
 *   chosen step scores (the reference returns exp(scores)).
 * hmm355_stream_beam_f32 replaces _beam_search_decode (streaming.py:322-377):
 *   hyp_score / hyp_last (B,32) and hyp_count (B) (<= 32) hold each stream's hypotheses in
 *   rank order and are updated in place (a stream may carry more hypotheses than the new K,
 *   after its beam width was lowered, streaming.py:459-461); first[b] != 0 applies the empty-path rule of the stream's first
 *   frame (score + emis, no transition).  Each step keeps the K best of the hyp_count * N
 *   expansions by score descending, ties by expansion index h*N + j ascending (Python's
 *   stable sort), score = (score_h + log_T[last_h][j]) + emis[t][j] in fp32.
 *   parent / hstate (B,T,K) int16: new hypothesis r at step t came from hypothesis
 *   parent[t][r] of step t-1 and entered state hstate[t][r].  states (B,T) int64: the best
 *   hypothesis' last T states.  1 <= K <= 32 and live_max (<= 32) bounds every hyp_count[b];
 *   for N > 128, K and live_max <= 16 (else HMM355_E_ARG).
 * ------------------------------------------------------------------------------ */
int hmm355_stream_greedy_f32(const float* emis, const float* log_T, const int* prev_state,
                             float log_n, int B, int T, int N, int64_t* states, float* scores,
                             void* stream);
int hmm355_stream_beam_f32(const float* emis, const float* log_T, int B, int T, int N, int K,
                           int live_max, float* hyp_score, int* hyp_last, int* hyp_count, const int* first,
                           int16_t* parent, int16_t* hstate, int64_t* states, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HMM355_H */
