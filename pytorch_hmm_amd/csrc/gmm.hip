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
//
// Precision.  The Viterbi path the reference decodes from these scores is decided by
// differences far below one fp32 ulp of a 2000-frame path score, so the scores must sit as
// close to the exact value as the reference's own fp32 ones do: an fp32 sum over D = 80
// terms here (2 fused FMAs per term) flipped 2 states of one sequence at config 3 against
// the reference (tests/test_gpu_fullsize.py), while the exact value rounded once does not.
// The quadratic form is therefore accumulated in fp64 — v_fma_f64 issues at the same rate
// as v_fma_f32 on gfx950 (78.6 TF fp64 vector = non-packed fp32), so the accuracy costs no
// throughput — and the score is rounded to fp32 once at the end.
//
// Layout.  gmm_prep (one thread per (p,d)) writes the scales w and offsets -mu*w in fp64,
// d-major ([d][P]: one coalesced 8-byte load per lane).  gmm_xt converts the frames to fp64
// in tiles [frame tile][d chunk][64 frames][8 dims]: a chunk (4 KiB) is staged in LDS by the
// workgroup and every lane reads a frame's 8 dims as broadcast LDS reads.  gmm_score: a workgroup owns
// 64 frames x floor(nt/C) states (nt = 64..256 threads, sized to S*C), a lane one component.  Per 8-dim chunk the lane holds 16
// fp64 parameters in VGPRs and updates the 64 frames' accumulators (two v_fma_f64 per (frame,
// component, d), no LDS or vector-memory traffic in the inner loop).  The components' LSE
// over c runs through a 16-frame LDS tile; rows leave as fp32.
#include "common.h"

namespace hmm355 {

constexpr int kGmmThreads = 256;
constexpr int kGmmFrames = 64;  // frames per workgroup (accumulators per lane)
constexpr int kGmmDc = 8;       // dims per chunk (one s_load_dwordx16 of fp64 per frame)
constexpr int kGmmSub = 16;     // frames per LDS LSE tile
// feature dimensions: the scorer walks D in 8-dim chunks with no per-D register or LDS state,
// so D is bounded only by the workspace (frames * D * 8 bytes for the fp64 frame tiles)
constexpr int kGmmDMax = 8192;

// one block per component p < PP (PP: P padded to the scorers' component groups; the pad
// components get w = mw = 0 and are never written out)
__global__ void gmm_prep_kernel(const float* __restrict__ means, const float* __restrict__ log_vars,
                                const float* __restrict__ log_w, double* __restrict__ pw,
                                double* __restrict__ pmw, double* __restrict__ cst, int P, int PP, int D,
                                int DP) {
  const int p = blockIdx.x;
  if (p >= PP) return;
  for (int d = threadIdx.x; d < DP; d += blockDim.x) {
    double w = 0.0, mw = 0.0;
    if (d < D && p < P) {
      w = exp(-0.5 * (double)log_vars[(size_t)p * D + d]);
      mw = -(double)means[(size_t)p * D + d] * w;
    }
    pw[(size_t)d * PP + p] = w;
    pmw[(size_t)d * PP + p] = mw;
  }
  if (threadIdx.x == 0 && p < P) {
    double s = 0.0;
    for (int d = 0; d < D; ++d) s += (double)log_vars[(size_t)p * D + d];
    cst[2 * p + 0] = s + (double)D * 1.8378770664093453;  // D*log(2*pi)
    cst[2 * p + 1] = log_w ? (double)log_w[p] : 0.0;
  }
}

// x (nframes, D) fp32 -> xt [tile][chunk][64 frames][8 dims] fp64 (zeros past the ends)
__global__ void __launch_bounds__(256) gmm_xt_kernel(const float* __restrict__ x, double* __restrict__ xt,
                                                     int nframes, int D, int NDC, size_t total) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int k = (int)(i % kGmmDc);
    const size_t r = i / kGmmDc;
    const int f = (int)(r % kGmmFrames);
    const size_t r2 = r / kGmmFrames;
    const int dc = (int)(r2 % NDC);
    const size_t tile = r2 / NDC;
    const size_t frame = tile * kGmmFrames + f;
    const int d = dc * kGmmDc + k;
    xt[i] = (frame < (size_t)nframes && d < D) ? (double)x[frame * D + d] : 0.0;
  }
}

__global__ void __launch_bounds__(kGmmThreads) gmm_score_kernel(const double* __restrict__ xt,
                                                               const double* __restrict__ pw,
                                                               const double* __restrict__ pmw,
                                                               const double* __restrict__ cst,
                                                               float* __restrict__ out, int nframes, int NDC,
                                                               int S, int C, int PP, int mix_lse) {
  __shared__ double tile[kGmmSub][kGmmThreads];
  const int tid = threadIdx.x;
  const int nt = blockDim.x;        // 64..256: sized to S*C by the host (a lane per component)
  const int spb = nt / C;           // states per workgroup
  const int s0 = blockIdx.y * spb;
  const int sl = tid / C, c = tid - sl * C;
  const int s = s0 + sl;
  const bool active = sl < spb && s < S;
  const int P = S * C;
  const int p = active ? s * C + c : 0;
  const size_t ft = blockIdx.x;

  // The frames' 8-dim chunks go through an LDS double buffer (one coalesced 16-B load per
  // lane per chunk, prefetched a chunk ahead) and reach the FMAs as broadcast LDS reads.
  // Taking them as wave-uniform scalar loads instead left one s_load -> s_waitcnt pair per
  // frame in the inner loop: the scalar-load latency per 16 FMAs (619 us at config 3).
  constexpr int CH2 = kGmmFrames * kGmmDc / 2;  // double2 per chunk (256)
  __shared__ double2 xs[2][CH2];
  double q[kGmmFrames];
#pragma unroll
  for (int f = 0; f < kGmmFrames; ++f) q[f] = 0.0;
  const double2* xtile = reinterpret_cast<const double2*>(xt + ft * (size_t)NDC * kGmmFrames * kGmmDc);
  const int nt0 = blockDim.x;
  double2 pre[4];
  auto fetch = [&](int dc) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * nt0;
      pre[j] = i < CH2 ? xtile[(size_t)dc * CH2 + i] : make_double2(0.0, 0.0);
    }
  };
  fetch(0);
  for (int dc = 0; dc < NDC; ++dc) {
    double2* xb = xs[dc & 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * nt0;
      if (i < CH2) xb[i] = pre[j];
    }
    __syncthreads();
    if (dc + 1 < NDC) fetch(dc + 1);
    double w[kGmmDc], mw[kGmmDc];
#pragma unroll
    for (int k = 0; k < kGmmDc; ++k) {
      w[k] = pw[(size_t)(dc * kGmmDc + k) * PP + p];
      mw[k] = pmw[(size_t)(dc * kGmmDc + k) * PP + p];
    }
#pragma unroll
    for (int f = 0; f < kGmmFrames; ++f) {
      double xv[kGmmDc];
#pragma unroll
      for (int k2 = 0; k2 < kGmmDc / 2; ++k2) {
        const double2 v = xb[f * (kGmmDc / 2) + k2];  // same address in every lane: broadcast
        xv[2 * k2] = v.x;
        xv[2 * k2 + 1] = v.y;
      }
#pragma unroll
      for (int k = 0; k < kGmmDc; ++k) {
        const double z = fma(xv[k], w[k], mw[k]);
        q[f] = fma(z, z, q[f]);
      }
    }
  }
  const double kp = cst[2 * p], lw = cst[2 * p + 1];
  const size_t f_begin = ft * kGmmFrames;
#pragma unroll
  for (int f0 = 0; f0 < kGmmFrames; f0 += kGmmSub) {
#pragma unroll
    for (int fi = 0; fi < kGmmSub; ++fi) tile[fi][tid] = -0.5 * (q[f0 + fi] + kp) + lw;
    __syncthreads();
    for (int pair = tid; pair < kGmmSub * spb; pair += nt) {
      const int fi = pair / spb, sj = pair - fi * spb;
      const size_t frame = f_begin + f0 + fi;
      const int ss = s0 + sj;
      if (frame < (size_t)nframes && ss < S) {
        double r;
        if (!mix_lse) {
          r = tile[fi][sj * C];
        } else {
          double m = -INFINITY;
          for (int cc = 0; cc < C; ++cc) m = fmax(m, tile[fi][sj * C + cc]);
          if (isinf(m)) m = 0.0;  // mixture_gaussian.py:144
          float e = 0.f;          // terms <= 1: fp32 sum and log add ~1e-7 absolute to |lp| ~ 1e2
          for (int cc = 0; cc < C; ++cc) e += expf((float)(tile[fi][sj * C + cc] - m));
          r = (double)logf(fmaxf(e, 1e-8f)) + m;  // :149-153
        }
        out[frame * S + ss] = (float)r;
      }
    }
    __syncthreads();
  }
}

// ---- the scorer for C in {1, 2, 4} (every BASELINE layer: C = 4 at config 3, C = 1 for the
// Gaussian and HSMM layers).
//
// gmm_score_kernel above reads one broadcast ds_read_b128 (2 dims of a frame) per 4 fp64 FMAs of
// its one component per lane: 4 LDS cycles per 8 issue cycles per SIMD, so the CU's shared LDS
// (4 SIMDs) is the bound (376 us per call at config 3, 28 TFLOP/s fp64).  Here a
// lane owns 4 components (p = g0 + 4*cl + j) and 16 frames (64 fp64 accumulators): each
// broadcast x read feeds 16 FMAs, and each component's parameters, read once per dim pair from
// LDS, feed 16 frames.  Per dim pair and lane: 8 parameter reads + 16 x reads for 256 FMAs.
// Frame groups (FG): the 64 lanes of a wave are FG groups of 64/FG component lanes, group fg
// taking frames fg*16 .. fg*16+15 of the wave's block (small P: 64 components per wave at FG = 4).
// The NW waves of a workgroup take consecutive frame blocks and share one staged copy of the
// parameters.  The fp32 frames are converted to fp64 while staged (no separate pass).
// Arithmetic per (frame, component): z = fma(x_d, w_d, mw_d), q = fma(z, z, q) for d = 0, 1, ...
// in order, then the LSE over the state's components, exactly as gmm_score_kernel: same bits.
constexpr int kG4Dc = 8;   // dims per staged chunk

template <int FG, int NW, int kG4Nf>  // frame groups per wave, waves, frames per lane
struct G4 {
  static constexpr int CL = 64 / FG;            // component lanes per frame group
  static constexpr int CG = 4 * CL;             // components per workgroup
  static constexpr int FW = FG * kG4Nf;         // frames per wave
  static constexpr int FT = NW * FW;            // frames per workgroup
  static constexpr int NT = NW * 64;
  // x tile row offset (doubles): 16-frame blocks padded by 2 doubles, so the FG groups' broadcast
  // reads (one frame each) fall in different banks
  static constexpr int NF = kG4Nf;
  static constexpr int XROW = kG4Nf * kG4Dc + 2;
  static constexpr int XS = (FT / kG4Nf) * XROW;
  static constexpr int PS = 2 * kG4Dc * 2 * CL;   // double2 per parameter buffer: [array][dim][half][cl]
  static constexpr int PV = (2 * kG4Dc * CG / 2 + NT - 1) / NT;  // double2 staged per thread
  static constexpr int XV = (FT * kG4Dc + NT - 1) / NT;          // floats staged per thread
};

template <int FG, int NW, int kG4Nf, bool REGP = false>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(kG4Nf >= 16 ? 2 : 3))) gmm_score4_kernel(const float* __restrict__ x,
                                                             const double* __restrict__ pw,
                                                             const double* __restrict__ pmw,
                                                             const double* __restrict__ cst,
                                                             float* __restrict__ out, int nframes, int D,
                                                             int NDC, int S, int C, int P, int PP,
                                                             int mix_lse, int T, int t0, int L) {
  using G = G4<FG, NW, kG4Nf>;
  // frame f of this launch is row f + (f / L) (T - L) + t0 of x / out: the time slice
  // [t0, t0 + L) of every sequence (L = T, t0 = 0: every frame in order, no division)
  const bool sliced = L != T;
  auto row_of = [&](size_t f) -> size_t {
    if (!sliced) return f;
    const unsigned q = (unsigned)f / (unsigned)L;  // (frames < 2^31: gmm_run checks)
    return f + (size_t)q * (size_t)(T - L) + (size_t)t0;
  };
  __shared__ double2 ps[2][G::PS];
  __shared__ double xs[2][G::XS];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int fg = l / G::CL, cl = l % G::CL;
  const int g0 = blockIdx.y * G::CG;
  const size_t f0 = (size_t)blockIdx.x * G::FT;
  const int fblk = w * FG + fg;  // this lane's 16-frame block in the tile

  // Parameter buffer element e = ((a*8 + k)*2 + h)*CL + cl holds components g0 + 4cl + 2h, +1
  // of array a at dim k.  REGP (the default): the parameters and the frames (fp32 -> fp64 on
  // the way into LDS) of chunk dc + 1 are loaded into registers when chunk dc starts and stored
  // to the other LDS buffers when its reads end.  Otherwise the parameters go global -> LDS
  // directly (global_load_lds_dwordx4, one wave instruction per 64 consecutive double2), issued
  // when the chunk's reads end: an LDS-DMA in flight makes the compiler wait for it before every
  // LDS read, so it cannot overlap them (4-7 % slower).  __syncthreads publishes both.
  constexpr int PI = G::PS / 64;  // wave instructions per parameter buffer
  auto fetch_params = [&](int dc, int buf) {
    for (int i = w; i < PI; i += NW) {
      const int e = i * 64 + l;
      const int cle = e % G::CL, rest = e / G::CL;
      const int h = rest & 1, k = (rest >> 1) % kG4Dc, a = rest / (2 * kG4Dc);
      const double* src = (a ? pmw : pw) + (size_t)(dc * kG4Dc + k) * PP + g0 + 4 * cle + 2 * h;
      // PP (the padded stride) is a multiple of CG: every pair is in bounds and 16-B aligned
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                       reinterpret_cast<void*>(&ps[buf][i * 64]), 16, 0, 0);
    }
  };
  // (REGP, diagnostic: the parameters through registers, loaded with the frames when a chunk
  // starts and stored to LDS when its reads end -- no LDS-DMA in flight during the reads)
  constexpr int PV = REGP ? (2 * kG4Dc * G::CG / 2 + G::NT - 1) / G::NT : 1;
  double2 pre_p[PV];
  auto fetch_preg = [&](int dc) {
#pragma unroll
    for (int r = 0; r < PV; ++r) {
      const int e = tid + r * G::NT;
      const int cle = e % G::CL, rest = e / G::CL;
      const int h = rest & 1, k = (rest >> 1) % kG4Dc, a = rest / (2 * kG4Dc);
      const double* src = (a ? pmw : pw) + (size_t)(dc * kG4Dc + k) * PP + g0 + 4 * cle + 2 * h;
      pre_p[r] = e < G::PS ? *reinterpret_cast<const double2*>(src) : make_double2(0.0, 0.0);
    }
  };
  auto stage_preg = [&](int buf) {
#pragma unroll
    for (int r = 0; r < PV; ++r) {
      const int e = tid + r * G::NT;
      if (e < G::PS) ps[buf][e] = pre_p[r];
    }
  };
  float pre_x[G::XV];
  auto fetch_x = [&](int dc) {
#pragma unroll
    for (int r = 0; r < G::XV; ++r) {
      const int i = tid + r * G::NT;
      const int f = i / kG4Dc, k = i % kG4Dc;
      const size_t frame = f0 + f;
      const int d = dc * kG4Dc + k;
      pre_x[r] = (i < G::FT * kG4Dc && frame < (size_t)nframes && d < D) ? x[row_of(frame) * D + d] : 0.f;
    }
  };
  auto stage_x = [&](int buf) {
#pragma unroll
    for (int r = 0; r < G::XV; ++r) {
      const int i = tid + r * G::NT;
      if (i < G::FT * kG4Dc) {
        const int f = i / kG4Dc, k = i % kG4Dc;
        xs[buf][(f / kG4Nf) * G::XROW + (f % kG4Nf) * kG4Dc + k] = (double)pre_x[r];
      }
    }
  };

  double q[4][kG4Nf];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int f = 0; f < kG4Nf; ++f) q[j][f] = 0.0;

  if constexpr (REGP) {
    fetch_preg(0);
    stage_preg(0);
  } else {
    fetch_params(0, 0);
  }
  fetch_x(0);
  stage_x(0);
  __syncthreads();
  for (int dc = 0; dc < NDC; ++dc) {
    const int buf = dc & 1;
    // the frames of chunk dc + 1 into registers now; its parameters (LDS-DMA) after this chunk's
    // reads: an LDS-DMA in flight makes the compiler wait for it before every LDS read
    if (dc + 1 < NDC) {
      fetch_x(dc + 1);
      if constexpr (REGP) fetch_preg(dc + 1);
    }
    const double2* pb = ps[buf];
    const double* xb = xs[buf] + fblk * G::XROW;
#pragma unroll 1
    for (int kp = 0; kp < kG4Dc / 2; ++kp) {  // (not unrolled: each pair's 16 parameters stay live alone)
      double wv[2][4], mv[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const double2 a = pb[((0 * kG4Dc + 2 * kp + kk) * 2 + h) * G::CL + cl];
          const double2 b = pb[((1 * kG4Dc + 2 * kp + kk) * 2 + h) * G::CL + cl];
          wv[kk][2 * h] = a.x; wv[kk][2 * h + 1] = a.y;
          mv[kk][2 * h] = b.x; mv[kk][2 * h + 1] = b.y;
        }
      // frame f's two dims read one frame ahead; its 8 z values formed before their squares
      // are accumulated (no FMA waits on the one just issued)
      double2 xn = *reinterpret_cast<const double2*>(xb + 2 * kp);  // broadcast per group
#pragma unroll
      for (int f = 0; f < kG4Nf; ++f) {
        const double2 xv = xn;
        if (f + 1 < kG4Nf) xn = *reinterpret_cast<const double2*>(xb + (f + 1) * kG4Dc + 2 * kp);
        double z[2][4];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 4; ++j) z[kk][j] = fma(kk ? xv.y : xv.x, wv[kk][j], mv[kk][j]);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 4; ++j) q[j][f] = fma(z[kk][j], z[kk][j], q[j][f]);
      }
    }
    if (dc + 1 < NDC) {
      // the other buffers' last readers passed the barrier that ended chunk dc - 1
      if constexpr (REGP) stage_preg(buf ^ 1);
      else fetch_params(dc + 1, buf ^ 1);
      stage_x(buf ^ 1);
      __syncthreads();
    }
  }

  // scores, then the LSE over each state's components (lane-local: C divides 4)
  const size_t fbase = f0 + (size_t)fblk * kG4Nf;
  const int pl = g0 + 4 * cl;  // first component of this lane
  double kp4[4], lw4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = pl + j < P ? pl + j : 0;
    kp4[j] = cst[2 * p];
    lw4[j] = cst[2 * p + 1];
  }
#pragma unroll
  for (int f = 0; f < kG4Nf; ++f) {
    const size_t frame = fbase + f;
    if (frame >= (size_t)nframes) break;
    double v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = -0.5 * (q[j][f] + kp4[j]) + lw4[j];
    for (int j0 = 0; j0 < 4; j0 += C) {
      const int p0 = pl + j0;
      if (p0 >= P) break;
      double r;
      if (!mix_lse) {
        r = v[j0];
      } else {
        double m = -INFINITY;
        for (int cc = 0; cc < C; ++cc) m = fmax(m, v[j0 + cc]);
        if (isinf(m)) m = 0.0;  // mixture_gaussian.py:144
        float e = 0.f;
        for (int cc = 0; cc < C; ++cc) e += expf((float)(v[j0 + cc] - m));
        r = (double)logf(fmaxf(e, 1e-8f)) + m;  // :149-153
      }
      out[row_of(frame) * S + p0 / C] = (float)r;
    }
  }
}

template <int FG, int NW, int NF, bool REGP = false>
static hipError_t launch_g4(const float* x, const double* pw, const double* pmw, const double* cst, float* out,
                            int nframes, int D, int NDC, int S, int C, int P, int PP, int mix_lse, int T, int t0,
                            int L, hipStream_t st) {
  using G = G4<FG, NW, NF>;
  dim3 grid((unsigned)(((size_t)nframes + G::FT - 1) / G::FT), (unsigned)((P + G::CG - 1) / G::CG));
  hipLaunchKernelGGL((gmm_score4_kernel<FG, NW, NF, REGP>), grid, dim3(G::NT), 0, st, x, pw, pmw, cst, out, nframes, D, NDC,
                     S, C, P, PP, mix_lse, T, t0, L);
  return hipGetLastError();
}

struct GmmWs {
  double *pw, *pmw, *cst, *xt;
};
// the v2 scorer (gmm_score4_kernel) serves C in {1, 2, 4}; others take gmm_score_kernel
static bool gmm_v2(int C) { return C == 1 || C == 2 || C == 4; }
// components per v2 workgroup for P components (G4<FG, NW>::CG of the launch below)
static int gmm_v2_group(size_t P) { return P > 128 ? 256 : (P > 64 ? 128 : 64); }
// the configuration index of HMM355_GMM_CFG (diagnostic; -1 = default) and whether the first
// scorer runs (it needs the fp64 frame tiles in the workspace: the size query and the launch
// read the same variable)
static int gmm_cfg() {
#ifdef HMM355_DIAG
  const char* ev = getenv("HMM355_GMM_CFG");  // (diagnostic builds only)
  return ev ? atoi(ev) : -1;
#else
  return -1;
#endif
}
static bool gmm_use_v1(int C) { return !gmm_v2(C) || gmm_cfg() == 0; }
static size_t gmm_ws_layout(int B, int T, int D, int S, int C, char* base, GmmWs* w) {
  const size_t P = (size_t)S * C;
  const size_t CG = gmm_v2_group(P);
  const size_t PP = (P + CG - 1) / CG * CG;  // padded stride of the [d][PP] parameter tables
  const size_t NDC = (D + kGmmDc - 1) / kGmmDc, DP = NDC * kGmmDc;
  const size_t nframes = (size_t)B * T;
  const size_t ntiles = (nframes + kGmmFrames - 1) / kGmmFrames;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += align_up(bytes, 256); return o; };
  const size_t ow = take(PP * DP * sizeof(double));
  const size_t om = take(PP * DP * sizeof(double));
  const size_t oc = take(P * 2 * sizeof(double));
  // fp64 frame tiles: the first scorer only (v2 converts while staging)
  const size_t ox = take(gmm_use_v1(C) ? ntiles * NDC * kGmmFrames * kGmmDc * sizeof(double) : 0);
  if (w && base) {
    w->pw = reinterpret_cast<double*>(base + ow);
    w->pmw = reinterpret_cast<double*>(base + om);
    w->cst = reinterpret_cast<double*>(base + oc);
    w->xt = reinterpret_cast<double*>(base + ox);
  }
  return off;
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_gmm_workspace_bytes(int B, int T, int D, int S, int C) {
  if (B < 0 || T < 0 || D < 1 || D > kGmmDMax || S < 1 || C < 1 || C > 256) return 0;
  return gmm_ws_layout(B, T, D, S, C, nullptr, nullptr);
}

static int gmm_run(const float* x, const float* means, const float* log_vars, const float* log_w, int B, int T,
                   int D, int S, int C, int mix_lse, int t0, int L, float* out, void* workspace,
                   size_t workspace_bytes, void* stream);

HMM355_API int hmm355_gmm_diag_logprob_f32(const float* x, const float* means, const float* log_vars,
                                           const float* log_w, int B, int T, int D, int S, int C, int mix_lse,
                                           float* out, void* workspace, size_t workspace_bytes, void* stream) {
  return gmm_run(x, means, log_vars, log_w, B, T, D, S, C, mix_lse, 0, T, out, workspace, workspace_bytes, stream);
}

static int gmm_run(const float* x, const float* means, const float* log_vars, const float* log_w, int B, int T,
                   int D, int S, int C, int mix_lse, int t0, int L, float* out, void* workspace,
                   size_t workspace_bytes, void* stream) {
  if (B < 0 || T < 0 || D < 1 || S < 1 || C < 1) return HMM355_E_ARG;
  if (D > kGmmDMax || C > 256 || (size_t)S * C > 65536) return HMM355_E_SHAPE;
  if ((size_t)B * T == 0) return HMM355_OK;
  if ((size_t)B * T > ((size_t)1 << 31) - kGmmFrames) return HMM355_E_SHAPE;
  if (!x || !means || !log_vars || !out || !workspace) return HMM355_E_ARG;
  if (!mix_lse && C != 1) return HMM355_E_ARG;
  if (workspace_bytes < hmm355_gmm_workspace_bytes(B, T, D, S, C)) return HMM355_E_WORKSPACE;
  GmmWs w;
  gmm_ws_layout(B, T, D, S, C, static_cast<char*>(workspace), &w);
  const int NDC = (D + kGmmDc - 1) / kGmmDc, DP = NDC * kGmmDc;
  const int P = S * C;
  const int CG = gmm_v2_group(P), PP = (P + CG - 1) / CG * CG;
  const int nframes = B * L;  // (the v1 scorer below runs whole tensors only: L == T, t0 == 0)
  const size_t ntiles = ((size_t)nframes + kGmmFrames - 1) / kGmmFrames;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gmm_prep_kernel, dim3(PP), dim3(64), 0, st, means, log_vars, log_w, w.pw, w.pmw, w.cst, P, PP,
                     D, DP);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int cfg = gmm_cfg();  // diagnostic: 0 = the first scorer, 1.. = v2 shapes
  if (!gmm_use_v1(C)) {
    static_assert(G4<1, 4, 16>::CG == 256 && G4<2, 2, 16>::CG == 128 && G4<4, 2, 16>::CG == 64, "gmm_v2_group");
#define G4L(fg, nw, nf) launch_g4<fg, nw, nf>(x, w.pw, w.pmw, w.cst, out, nframes, D, NDC, S, C, P, PP, mix_lse, T, t0, L, st)
    // shapes from tools/time_gmm.py (profiles/r4h_gmm2.log): config 3 (P = 512) 326 us with
    // 16 frames per lane; P = 64 (configs 2, 5) 57 / 34 us with 4 (the work is small: more waves)
    // (round 4, profiles/r4m_gmm_regp.log: the parameters staged through registers, config 5
    // below and the default, beat the LDS-DMA staging, config 1, by 4-7 %: 311 / 54 / 31 us per
    // call at configs 3 / 2 / 5; identical bits)
#define G4R(fg, nw, nf) launch_g4<fg, nw, nf, true>(x, w.pw, w.pmw, w.cst, out, nframes, D, NDC, S, C, P, PP, mix_lse, T, t0, L, st)
    if (CG == 256) {
      e = cfg == 1 ? G4L(1, 4, 16) : cfg == 2 ? G4L(1, 4, 8) : cfg == 3 ? G4L(1, 2, 16) : cfg == 4 ? G4L(1, 1, 16)
                   : G4R(1, 4, 16);
    } else if (CG == 128) {
      e = cfg == 1 ? G4L(2, 2, 8) : cfg == 2 ? G4L(2, 2, 16) : cfg == 3 ? G4L(2, 1, 8) : G4R(2, 2, 8);
    } else {
      e = cfg == 1 ? G4L(4, 2, 4) : cfg == 2 ? G4L(4, 2, 8) : cfg == 3 ? G4L(4, 1, 4) : cfg == 4 ? G4L(4, 2, 16)
                   : G4R(4, 2, 4);
    }
#undef G4R
#undef G4L
    return e == hipSuccess ? HMM355_OK : (int)e;
  }
  const size_t total = ntiles * NDC * kGmmFrames * kGmmDc;
  size_t blocks = (total + 255) / 256;
  blocks = blocks < 8192 ? blocks : 8192;
  hipLaunchKernelGGL(gmm_xt_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, w.xt, nframes, D, NDC, total);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  // a lane per (state, component): small S*C (GaussianHMMLayer / HSMMLayer, C = 1) gets
  // 64- or 128-thread workgroups instead of 256 threads of which most would idle
  const int nt = P <= 64 ? 64 : (P <= 128 ? 128 : (P <= 192 ? 192 : kGmmThreads));
  const int spb = nt / C;
  dim3 grid((unsigned)ntiles, (S + spb - 1) / spb);
  hipLaunchKernelGGL(gmm_score_kernel, grid, dim3(nt), 0, st, w.xt, w.pw, w.pmw, w.cst, out, nframes, NDC,
                     S, C, PP, mix_lse);
  e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}
