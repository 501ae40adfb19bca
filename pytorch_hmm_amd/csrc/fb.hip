// hmm355 — forward-backward on gfx950.
//
// Replaces HMMPyTorch.forward_backward (reference hmm.py:66-130): the two per-time-step
// Python loops (hmm.py:95-101 forward, :110-117 backward) and the posterior epilogue
// (:119-128).
//
// Kernel 1, fb_recur<NP>: one workgroup per (sequence, direction): blockIdx.x = 2b + dir.
//   The recursion runs in the probability domain with per-step normalisation (Rabiner
//   scaling) instead of log-sum-exp: for the reference's log-space update
//       la_t[j] = LSE_i(la_{t-1}[i] + logP[i,j]) + log_obs_t[j]
//   the kernel keeps u_t = alpha_t / prod(c) with A = exp(logP), e_t = obs_t + 1e-8:
//       u_t[j] = (sum_i u_{t-1}[i] A[i,j]) / c_{t-1} * e_t[j],   c = sum_j u[j]
//   and the running log-scale LA_t = sum log c, so log alpha_t = log u_t + LA_t.  That is
//   one fp32 FMA per (i,j) cell instead of add + exp + max + add, which is what makes the
//   16384-cell step fit in ~128 VALU cycles on one CU.  The backward pass is the same
//   with A^T and the emission applied before the product (hmm.py:113-115).
//   Layout per step (NP = padded states, NW = NP/16 waves): wave w owns outputs
//   16w..16w+15 (lane c = l&15); the lane's row group r = l>>4 covers inputs
//   i = 64*blk + 16r + n.  A[i][o] lives in VGPRs (16*NP/64 per lane, loaded once); the
//   state vector u_{t-1} is read from LDS once per lane (one ds_read_b32 per 64 inputs) and
//   broadcast across the 16-lane row by DPP row_newbcast folded into v_fmac_f32_dpp, so the
//   inner loop is pure FMA with no LDS traffic.  Row groups are summed with
//   v_permlane16_swap / v_permlane32_swap, the wave's partial of sum_j u_t[j] with DPP.  One
//   s_barrier per step.
//   Emissions are staged 16 steps at a time into an LDS ring, loaded two blocks ahead into
//   registers; outputs go to a 32-row LDS ring and leave as one 16-B store per lane per
//   block, so the loop has no per-step global memory traffic.
//
// Kernel 2, fb_posterior<NP>: one wave per (b,t) row, grid-stride, HBM-bound:
//   posterior = (u*v)/sum(u*v) (scale-invariant), forward = exp(log u + LA),
//   backward = exp(log v + LB), and the reference's compute_likelihood value
//   logsumexp_j(log(forward_{T-1}[j] + 1e-8)) (hmm.py:206) for t = T-1.
#include "common.h"

namespace hmm355 {

template <int NP>
struct FB {
  static constexpr int NW = NP / 16;
  static constexpr int NT = NW * kWave;
  static constexpr int NBLK = NP / 64;
  static constexpr int U = 16;        // steps per staging block
  static constexpr int RING = 2 * U;  // output ring rows
  // LDS layout (floats)
  static constexpr int OFF_EMIS = 0;                      // [2][U][NP]
  static constexpr int OFF_RING = OFF_EMIS + 2 * U * NP;  // [RING][NP]
  static constexpr int OFF_Y = OFF_RING + RING * NP;      // [2][NP]   (backward's y = v*e)
  static constexpr int OFF_PSUM = OFF_Y + 2 * NP;         // [2][NW]
  static constexpr int OFF_LS = OFF_PSUM + 2 * NW;        // [RING]
  static constexpr int LDS_FLOATS = OFF_LS + RING;
};

struct FBArgs {
  const float* obs;
  const float* log_P;
  const float* log_p0;
  float* U;      // (B,T,NP) forward scaled values u_t
  float* V;      // (B,T,NP) backward scaled values v_t
  float* LA;     // (B,T) log-scale of u_t
  float* LB;     // (B,T) log-scale of v_t
  float* loglik; // (B) or null
  int B, T, N, obs_mode;
};

// Load one 16-step emission block for this lane: 4 consecutive states of one step.
template <int NP, bool ALPHA>
__device__ __forceinline__ void fb_load_block(const FBArgs& a, int b, int blk, int w, int l, float (&r)[4]) {
  const int q = blk * 16 + (l >> 2);
  const int tau = ALPHA ? q : a.T - 1 - q;
  const int col = 16 * w + 4 * (l & 3);
  const bool qok = q < a.T;
  const float* src = a.obs + ((size_t)b * a.T + (qok ? tau : 0)) * a.N;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool ok = qok && col + k < a.N;
    const float x = src[ok ? col + k : 0];
    r[k] = ok ? x : 0.f;
  }
}

template <int NP>
__device__ __forceinline__ void fb_store_block(const FBArgs& a, float* lds, int blk, int w, int l,
                                               const float (&r)[4]) {
  using C = FB<NP>;
  const int sq = l >> 2;
  const int col = 16 * w + 4 * (l & 3);
  float e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool ok = col + k < a.N;
    const float x = r[k];
    const float ev = a.obs_mode == HMM355_OBS_LOG ? __expf(x) : x + 1e-8f;
    e[k] = ok ? ev : 0.f;
  }
  float4* dst = reinterpret_cast<float4*>(lds + C::OFF_EMIS + ((blk & 1) * 16 + sq) * NP + col);
  *dst = make_float4(e[0], e[1], e[2], e[3]);
}

// Flush ring rows of staging block `blk` (16 rows) to global U/V and LA/LB.
template <int NP, bool ALPHA>
__device__ __forceinline__ void fb_flush(const FBArgs& a, const float* lds, int b, int blk, int tid) {
  using C = FB<NP>;
  constexpr int PER_ROW = NP / 4;
  const int row = tid / PER_ROW;  // 0..15
  const int c4 = (tid % PER_ROW) * 4;
  const int q = blk * 16 + row;
  if (q < a.T) {
    const int tau = ALPHA ? q : a.T - 1 - q;
    const float4 v = *reinterpret_cast<const float4*>(lds + C::OFF_RING + (q % C::RING) * NP + c4);
    float* dst = (ALPHA ? a.U : a.V) + ((size_t)b * a.T + tau) * NP + c4;
    *reinterpret_cast<float4*>(dst) = v;
    if (c4 == 0) (ALPHA ? a.LA : a.LB)[(size_t)b * a.T + tau] = lds[C::OFF_LS + (q % C::RING)];
  }
}

template <int NP, bool ALPHA>
__device__ __forceinline__ void fb_run(const FBArgs& a, float* lds, int b) {
  using C = FB<NP>;
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int o = 16 * w + c;  // output state of this lane
  const int T = a.T, N = a.N;

  // A = exp(log P) slice in registers.  ALPHA: M[blk][n] = A[i][o]; BETA: A[o][i].
  float M[C::NBLK][16];
#pragma unroll
  for (int blk = 0; blk < C::NBLK; ++blk)
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int i = 64 * blk + 16 * r + n;
      const bool ok = i < N && o < N;
      // unconditional (clamped) load, then select: a load under a per-element branch
      // makes hipcc wait vmcnt(0) per element
      const size_t idx = ok ? (ALPHA ? (size_t)i * N + o : (size_t)o * N + i) : 0;
      const float lp = a.log_P[idx];
      M[blk][n] = __expf(ok ? lp : -INFINITY);
    }

  const int nblocks = (T + 15) / 16;
  float er0[4], er1[4];
  fb_load_block<NP, ALPHA>(a, b, 0, w, l, er0);
  if (nblocks > 1) fb_load_block<NP, ALPHA>(a, b, 1, w, l, er1);
  fb_store_block<NP>(a, lds, 0, w, l, er0);
  lds_barrier();

  // q = 0: alpha_0 = p0 * e_0 (hmm.py:92) ; beta_{T-1} = 1 (hmm.py:107)
  {
    const float e = lds[C::OFF_EMIS + o];
    float st, y;
    if (ALPHA) {
      const float p0 = o < N ? __expf(a.log_p0[o]) : 0.f;
      st = y = p0 * e;
    } else {
      st = o < N ? 1.f : 0.f;
      y = st * e;
    }
    if (r == 0) {
      lds[C::OFF_RING + o] = st;
      if (!ALPHA) lds[C::OFF_Y + o] = y;
    }
    const float ws = row16_sum(y);
    if (l == 0) lds[C::OFF_PSUM + w] = ws;
    if (tid == 0) lds[C::OFF_LS + 0] = 0.f;
  }
  lds_barrier();

  double ls = 0.0;  // running log-scale (thread 0 keeps the authoritative copy)
  auto run_block = [&](int kb, float(&ernext)[4], float(&erfree)[4]) {
    // ---- block begin: stage block kb+1's emissions, prefetch block kb+2, flush kb-1
    if (kb + 1 < nblocks) fb_store_block<NP>(a, lds, kb + 1, w, l, ernext);
    if (kb + 2 < nblocks) fb_load_block<NP, ALPHA>(a, b, kb + 2, w, l, erfree);
    if (kb >= 1) fb_flush<NP, ALPHA>(a, lds, b, kb - 1, tid);

    const int q0 = kb * 16 < 1 ? 1 : kb * 16;
    const int q1 = (kb + 1) * 16 < T ? (kb + 1) * 16 : T;
    for (int q = q0; q < q1; ++q) {
      const int prv = (q - 1) & 1;
      float yv[C::NBLK];
#pragma unroll
      for (int blk = 0; blk < C::NBLK; ++blk)
        yv[blk] = ALPHA ? lds[C::OFF_RING + ((q - 1) % C::RING) * NP + 64 * blk + l]
                        : lds[C::OFF_Y + prv * NP + 64 * blk + l];
      float csum = 0.f;
#pragma unroll
      for (int ww = 0; ww < C::NW; ww += 4) {
        const float4 p = *reinterpret_cast<const float4*>(lds + C::OFF_PSUM + prv * C::NW + ww);
        csum += (p.x + p.y) + (p.z + p.w);
      }
      const float rsc = 1.0f / csum;

      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
      for (int blk = 0; blk < C::NBLK; ++blk) {
        fmac_bcast<0>(a0, yv[blk], M[blk][0]);
        fmac_bcast<1>(a1, yv[blk], M[blk][1]);
        fmac_bcast<2>(a2, yv[blk], M[blk][2]);
        fmac_bcast<3>(a3, yv[blk], M[blk][3]);
        fmac_bcast<4>(a0, yv[blk], M[blk][4]);
        fmac_bcast<5>(a1, yv[blk], M[blk][5]);
        fmac_bcast<6>(a2, yv[blk], M[blk][6]);
        fmac_bcast<7>(a3, yv[blk], M[blk][7]);
        fmac_bcast<8>(a0, yv[blk], M[blk][8]);
        fmac_bcast<9>(a1, yv[blk], M[blk][9]);
        fmac_bcast<10>(a2, yv[blk], M[blk][10]);
        fmac_bcast<11>(a3, yv[blk], M[blk][11]);
        fmac_bcast<12>(a0, yv[blk], M[blk][12]);
        fmac_bcast<13>(a1, yv[blk], M[blk][13]);
        fmac_bcast<14>(a2, yv[blk], M[blk][14]);
        fmac_bcast<15>(a3, yv[blk], M[blk][15]);
      }
      const float z = rows_sum((a0 + a1) + (a2 + a3)) * rsc;
      const float e = lds[C::OFF_EMIS + ((kb & 1) * 16 + (q & 15)) * NP + o];
      const float y = z * e;
      const float st = ALPHA ? y : z;
      if (r == 0) {
        lds[C::OFF_RING + (q % C::RING) * NP + o] = st;
        if (!ALPHA) lds[C::OFF_Y + (q & 1) * NP + o] = y;
      }
      const float ws = row16_sum(y);
      if (l == 0) lds[C::OFF_PSUM + (q & 1) * C::NW + w] = ws;
      if (tid == 0) {
        ls += (double)__logf(csum);
        lds[C::OFF_LS + (q % C::RING)] = (float)ls;
      }
      lds_barrier();
    }
  };
  for (int k = 0; k < nblocks; k += 2) {
    run_block(k, er1, er0);
    if (k + 1 < nblocks) run_block(k + 1, er0, er1);
  }
  // flush the last block (and the one before it if it was never flushed: nblocks == 1)
  fb_flush<NP, ALPHA>(a, lds, b, nblocks - 1, tid);
  if (ALPHA && tid == 0 && a.loglik) {
    float csum = 0.f;
    const int prv = (T - 1) & 1;
    for (int ww = 0; ww < C::NW; ++ww) csum += lds[C::OFF_PSUM + prv * C::NW + ww];
    a.loglik[b] = (float)(ls + (double)__logf(csum));
  }
}

template <int NP>
__global__ void __launch_bounds__(FB<NP>::NT) fb_recur_kernel(FBArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x >> 1;
  if (blockIdx.x & 1)
    fb_run<NP, false>(a, lds, b);
  else
    fb_run<NP, true>(a, lds, b);
}

struct PostArgs {
  const float* U;
  const float* V;
  const float* LA;
  const float* LB;
  float* posterior;
  float* forward;
  float* backward;
  float* lik_ref;
  int B, T, N;
  unsigned mask;
};

template <int NP>
__global__ void __launch_bounds__(256) fb_posterior_kernel(PostArgs a) {
  constexpr int K = NP / 64;
  const int l = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const size_t rows = (size_t)a.B * a.T;
  for (size_t row = wave; row < rows; row += nwaves) {
    float u[K], v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      u[k] = a.U[row * NP + l + 64 * k];
      v[k] = a.V[row * NP + l + 64 * k];
    }
    const float la = a.LA[row], lb = a.LB[row];
    float mu = 0.f, mv = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { mu = fmaxf(mu, u[k]); mv = fmaxf(mv, v[k]); }
    mu = wave_max(mu);
    mv = wave_max(mv);
    const float iu = mu > 0.f ? 1.f / mu : 0.f, iv = mv > 0.f ? 1.f / mv : 0.f;
    float p[K], s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { p[k] = (u[k] * iu) * (v[k] * iv); s += p[k]; }
    s = wave_sum(s);
    const float is = s > 0.f ? 1.f / s : 0.f;
    const bool last = (row % a.T) == (size_t)(a.T - 1);
    float fw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) fw[k] = __expf(__logf(u[k]) + la);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = l + 64 * k;
      if (j < a.N) {
        const size_t off = row * a.N + j;
        if (a.mask & HMM355_FB_POSTERIOR) a.posterior[off] = p[k] * is;
        if (a.mask & HMM355_FB_FORWARD) a.forward[off] = fw[k];
        if (a.mask & HMM355_FB_BACKWARD) a.backward[off] = __expf(__logf(v[k]) + lb);
      }
    }
    if (last && a.lik_ref) {
      // hmm.py:206: logsumexp(log(forward[:, -1] + 1e-8))
      float lv[K], m = -INFINITY;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        lv[k] = (l + 64 * k < a.N) ? __logf(fw[k] + 1e-8f) : -INFINITY;
        m = fmaxf(m, lv[k]);
      }
      m = wave_max(m);
      float e = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) e += (l + 64 * k < a.N) ? __expf(lv[k] - m) : 0.f;
      e = wave_sum(e);
      if (l == 0) a.lik_ref[row / a.T] = m + __logf(e);
    }
  }
}

template <int NP>
static hipError_t launch_fb(const FBArgs& fa, const PostArgs& pa, hipStream_t st) {
  using C = FB<NP>;
  const size_t lds = C::LDS_FLOATS * sizeof(float);
  hipError_t e = allow_lds(fb_recur_kernel<NP>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fb_recur_kernel<NP>, dim3(2 * fa.B), dim3(C::NT), lds, st, fa);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t rows = (size_t)pa.B * pa.T;
  const size_t waves = rows < 8192 ? rows : 8192;
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  hipLaunchKernelGGL(fb_posterior_kernel<NP>, dim3(blocks), dim3(256), 0, st, pa);
  return hipGetLastError();
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_fb_workspace_bytes(int B, int T, int N) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return 0;
  const size_t NP = pad_states(N);
  const size_t rows = (size_t)B * T;
  return align_up(2 * rows * NP * sizeof(float), 256) + align_up(2 * rows * sizeof(float), 256);
}

HMM355_API int hmm355_forward_backward_f32(const float* obs, int obs_mode, const float* log_P,
                                           const float* log_p0, int B, int T, int N, unsigned out_mask,
                                           float* posterior, float* forward, float* backward, float* loglik,
                                           float* lik_ref, void* workspace, size_t workspace_bytes,
                                           void* stream) {
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
  const size_t rows = (size_t)B * T;
  char* ws = static_cast<char*>(workspace);
  float* U = reinterpret_cast<float*>(ws);
  float* V = U + rows * NP;
  float* LA = reinterpret_cast<float*>(ws + align_up(2 * rows * NP * sizeof(float), 256));
  float* LB = LA + rows;
  FBArgs fa{obs, log_P, log_p0, U, V, LA, LB, loglik, B, T, N, obs_mode};
  PostArgs pa{U, V, LA, LB, posterior, forward, backward, lik_ref, B, T, N, out_mask};
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (NP) {
    case 64: e = launch_fb<64>(fa, pa, st); break;
    case 128: e = launch_fb<128>(fa, pa, st); break;
    default: e = launch_fb<256>(fa, pa, st); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}
