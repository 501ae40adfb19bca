// hmm355 — Viterbi on gfx950.
//
// Replaces HMMPyTorch.viterbi_decode (reference hmm.py:132-184) and
// MixtureGaussianHMMLayer._viterbi_decode (mixture_gaussian.py:290-338).
//
// Kernel 1, vit_fwd<NP> (one workgroup per sequence): the max-plus recursion
//     delta_t[j] = max_i(delta_{t-1}[i] + logP[i,j]) + log_obs_t[j]            (hmm.py:164-168)
//   computing the max only, on the serial-chain skeleton of recur.h (wave w owns input
//   slice 16w..16w+15, delta_{t-1} broadcast by DPP row_newbcast folded into
//   v_add_f32_dpp, two candidates per v_max3_f32: 1.5 VALU per cell; per-wave partial maxima
//   combined through LDS after the step's one barrier).  The max of a set of fp32 values is
//   order-independent and each delta is one fp32 add, so delta is bit-identical to the
//   reference given identical log-emissions.  The emission log(x + 1e-8) is formed in fp32
//   and the log correctly rounded (logcr.h) while the emissions are staged.
//
// Kernel 2, vit_psi<NP> (one workgroup per (sequence, 64-step chunk), ~1000 workgroups):
//   the argmax pointers psi_t[j] = first argmax_i(delta_{t-1}[i] + logP[i,j]) recomputed
//   from the stored trellis — the same fp32 sums, so the same argmax the reference's
//   torch.max(dim=1) returns (first index on ties, hmm.py:167).  Taking the argmax out of
//   the serial loop (4 VALU per cell there) and onto the whole chip is what lets the serial
//   kernel run at the max-only cost.  While the chunk's psi rows are in LDS the kernel also
//   composes them into the chunk map G_c[j] = state at the end of chunk c-1 given state j
//   at the end of chunk c (pointer jumping: 64 dependent LDS lookups per lane).
//   On a banded matrix with NP >= 128 (recur.h kVitFused) the chain kernel's psi waves have
//   already written the psi rows, and this kernel only composes the chunk maps.
//
// Kernel 3, vit_backtrace<NP> (one wave per (sequence, chunk)): argmax of delta_{T-1}
//   (first index, hmm.py:174), the chain of chunk maps from the last chunk down to this one
//   (LDS lookups), then this chunk's 64-step walk (hmm.py:177-178).  The serial depth is
//   T/64 + 64 lookups instead of T dependent gathers.
#include "recur.h"
#include "post.h"

namespace hmm355 {

template <int NP>
__global__ void __launch_bounds__(kVitNT<NP>) vit_fwd_kernel(RecArgs ra) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  rec_dispatch<NP, kVit>(ra, lds, blockIdx.x);
}

// psi rows of one chunk -> HBM, and the chunk map G[j] = state at t_lo - 1 given j at t_hi
template <int NP>
__device__ __forceinline__ void psi_write_rows(const VitArgs& a, uint8_t (*prow)[NP], int b, int chunk, int t_lo,
                                               int t_hi) {
  using C = VF<NP>;
  const int tid = threadIdx.x;
  const int T = a.T, N = a.N;
  const int rows = t_hi - t_lo + 1;
  uint8_t* pdst = a.psi + ((size_t)b * T + t_lo) * NP;
  for (int idx = tid; idx < rows * NP / 16; idx += C::NT) {
    const int row = idx / (NP / 16), c16 = (idx % (NP / 16)) * 16;
    *reinterpret_cast<uint4*>(pdst + (size_t)row * NP + c16) = *reinterpret_cast<const uint4*>(&prow[row][c16]);
  }
  compose_chunk_map<NP>(a, prow, b, chunk, t_lo, t_hi);
}

// Banded psi rows (band.h): psi_t[o] = first argmax_i fl(delta_{t-1,i} + L[i][o]).  With
// g_i = fl(delta_{t-1,i} + r_i), M = max_i g_i and i1 its first index, the maximum is
// v = max(M, window values) and its first index is min({i1 if M == v} U {window i with
// value == v}): an index outside the window has value g_i, and no g_j == M precedes i1;
// i1 itself attains v whenever M == v (inside the window its value is >= g_i1 = M = v).
template <int NP>
__device__ __forceinline__ void psi_band_rows(const VitArgs& a, uint8_t (*prow)[NP], float* rowM, int* rowI,
                                              float* drows, int b, int t_lo, int t_hi) {
  using C = VF<NP>;
  const BandDesc* __restrict__ d = a.band;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int T = a.T, N = a.N, W = d->wcp;
  const int t_first = t_lo > 0 ? t_lo : 1;
  const int rows = t_hi - t_first + 1;
  // the chunk's delta rows t_first-1 .. t_hi-1, coalesced, into LDS (row stride NP)
  const float* dsrc = a.delta + ((size_t)b * T + (t_first - 1)) * N;
  if (N == NP && (reinterpret_cast<uintptr_t>(dsrc) & 15) == 0) {
    // full rows: 16-B loads, no index division
    const float4* s4 = reinterpret_cast<const float4*>(dsrc);
    float4* d4 = reinterpret_cast<float4*>(drows);
    for (int idx = tid; idx < rows * (NP / 4); idx += C::NT) d4[idx] = s4[idx];
  } else {
    for (int idx = tid; idx < rows * N; idx += C::NT) {
      const int r = idx / N, c = idx - r * N;
      drows[r * NP + c] = dsrc[idx];
    }
  }
  __syncthreads();
  float rf[C::NBLK];
#pragma unroll
  for (int blk = 0; blk < C::NBLK; ++blk) rf[blk] = d->rfl[64 * blk + l];
  for (int r = w; r < rows; r += C::NW) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) {
      const int i = 64 * blk + l;
      if (i < N) argmax_combine(bv, bi, drows[r * NP + i] + rf[blk], i);
    }
    wave_argmax_dpp(bv, bi);
    if (l == 0) { rowM[r] = bv; rowI[r] = bi; }
  }
  // each thread keeps one output column o for all rows (NT is a multiple of NP)
  static_assert(C::NT % NP == 0, "psi layout");
  const int o = tid % NP;
  const int lo = d->clo[o];
  float wl[kBandMax];
#pragma unroll
  for (int k = 0; k < kBandMax; ++k) wl[k] = (k < W && lo + k < N) ? d->cL[o][k] : -INFINITY;
  __syncthreads();
  for (int r = tid / NP; r < rows; r += C::NT / NP) {
    int arg = 0;
    if (o < N) {
      const float M = rowM[r];
      float v = M;
      float val[kBandMax];
#pragma unroll
      for (int k = 0; k < kBandMax; ++k) {
        val[k] = (k < W && lo + k < N) ? drows[r * NP + lo + k] + wl[k] : -INFINITY;
        v = fmaxf(v, val[k]);
      }
      arg = M == v ? rowI[r] : 0x7fffffff;
#pragma unroll
      for (int k = 0; k < kBandMax; ++k)
        if (k < W && val[k] == v && lo + k < arg) arg = lo + k;
    }
    prow[t_first + r - t_lo][o] = (uint8_t)arg;
  }
}

template <int NP>
__global__ void __launch_bounds__(VF<NP>::NT) vit_psi_kernel(VitArgs a) {
  using C = VF<NP>;
  static_assert(kPsiChunk == kChunk, "chunk length shared with the fused banded chain");
  __shared__ __attribute__((aligned(16))) uint8_t prow[kChunk][NP];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x;
  if (kVitFused<NP> && a.band && a.band->wc <= kBandMax) {
    // the banded chain's helpers wrote the psi rows (recur.h kVitFused): compose the map only
    if (chunk == 0) return;
    const int t_lo = chunk * kChunk;
    const int t_hi = (t_lo + kChunk < a.T ? t_lo + kChunk : a.T) - 1;
    const uint8_t* psrc = a.psi + ((size_t)b * a.T + t_lo) * NP;
    for (int idx = tid; idx < (t_hi - t_lo + 1) * NP / 16; idx += C::NT)
      *reinterpret_cast<uint4*>(&prow[0][0] + idx * 16) = *reinterpret_cast<const uint4*>(psrc + idx * 16);
    __syncthreads();
    compose_chunk_map<NP>(a, prow, b, chunk, t_lo, t_hi);
    return;
  }
  const int w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int o = 16 * w + c;
  const int T = a.T, N = a.N;
  const int t_lo = chunk * kChunk;
  const int t_hi = (t_lo + kChunk < T ? t_lo + kChunk : T) - 1;

  float M[C::NBLK][16];
#pragma unroll
  for (int blk = 0; blk < C::NBLK; ++blk)
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int i = 64 * blk + 16 * r + n;
      const bool ok = i < N && o < N;
      const float v = a.log_P[ok ? (size_t)i * N + o : 0];
      M[blk][n] = ok ? v : -INFINITY;
    }
  if (t_lo == 0 && tid < NP) prow[0][tid] = 0;  // psi_0 (hmm.py:156 zeros)
  if (a.band && a.band->wc <= kBandMax) {
    __shared__ float rowM[kChunk];
    __shared__ int rowI[kChunk];
    extern __shared__ __attribute__((aligned(16))) float drows[];  // [kChunk][NP] (dynamic)
    psi_band_rows<NP>(a, prow, rowM, rowI, drows, b, t_lo, t_hi);
    __syncthreads();
    psi_write_rows<NP>(a, prow, b, chunk, t_lo, t_hi);
    return;
  }

  const float* dbase = a.delta + (size_t)b * T * N;
  auto load_row = [&](int t, float(&yv)[C::NBLK]) {
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) {
      const int i = 64 * blk + l;
      const bool ok = i < N;
      const float v = dbase[(size_t)(t - 1) * N + (ok ? i : 0)];
      yv[blk] = ok ? v : -INFINITY;
    }
  };
  const int t_first = t_lo > 0 ? t_lo : 1;
  float ycur[C::NBLK], ynext[C::NBLK];
  if (t_first <= t_hi) load_row(t_first, ycur);
  for (int t = t_first; t <= t_hi; ++t) {
    if (t + 1 <= t_hi) load_row(t + 1, ynext);
    // lane-local scan in increasing i (i = 64*blk + 16r + n): strict > keeps the first
    float bv = row_bcast<0>(ycur[0]) + M[0][0];
    int bk = 0;  // local index 16*blk + n
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) {
#define PSI_STEP(n)                                                  \
  if (blk != 0 || n != 0) {                                          \
    const float s = row_bcast<n>(ycur[blk]) + M[blk][n];             \
    const bool gt = s > bv;                                          \
    bv = gt ? s : bv;                                                \
    bk = gt ? 16 * blk + n : bk;                                     \
  }
      PSI_STEP(0) PSI_STEP(1) PSI_STEP(2) PSI_STEP(3) PSI_STEP(4) PSI_STEP(5) PSI_STEP(6) PSI_STEP(7)
      PSI_STEP(8) PSI_STEP(9) PSI_STEP(10) PSI_STEP(11) PSI_STEP(12) PSI_STEP(13) PSI_STEP(14) PSI_STEP(15)
#undef PSI_STEP
    }
    int bi = 64 * (bk >> 4) + 16 * r + (bk & 15);
    // combine the four row groups: (value, index) lexicographic, ties -> smaller index
    {
      float va = bv, vb = bv;
      int ia = bi, ib = bi;
      permlane16_swap(va, vb);
      permlane16_swap_i(ia, ib);
      argmax_combine(va, ia, vb, ib);
      float vc = va, vd = va;
      int ic = ia, id = ia;
      permlane32_swap(vc, vd);
      permlane32_swap_i(ic, id);
      argmax_combine(vc, ic, vd, id);
      bi = ic;
    }
    if (r == 0) prow[t - t_lo][o] = (uint8_t)bi;
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) ycur[blk] = ynext[blk];
  }
  __syncthreads();
  psi_write_rows<NP>(a, prow, b, chunk, t_lo, t_hi);
}

template <int NP>
static hipError_t launch_vit(const VitArgs& va, bool prep, hipStream_t sm) {
  hipError_t e = allow_lds(vit_fwd_kernel<NP>, kExclusiveLds);  // own the CU (recur.h)
  if (e != hipSuccess) return e;
  if (va.band && prep) {
    e = launch_band_prep(va.log_P, va.N, const_cast<BandDesc*>(va.band), sm);
    if (e != hipSuccess) return e;
  }
  RecArgs ra{va.obs, va.log_P, va.init, va.delta, nullptr, nullptr, va.B, va.T, va.N, va.obs_mode, va.N, va.band,
             nullptr, nullptr, va.psi};
  hipLaunchKernelGGL(vit_fwd_kernel<NP>, dim3(va.B), dim3(kVitNT<NP>), kExclusiveLds, sm, ra);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // banded psi stages the chunk's delta rows in LDS (dynamic, kChunk x NP floats)
  const size_t psi_lds = va.band ? (size_t)kChunk * NP * sizeof(float) : 0;
  hipLaunchKernelGGL(vit_psi_kernel<NP>, dim3(va.nchunks, va.B), dim3(VF<NP>::NT), psi_lds, sm, va);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(vit_backtrace_kernel<NP>, dim3(va.nchunks, va.B), dim3(64), 0, sm, va);
  return hipGetLastError();
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_viterbi_workspace_bytes(int B, int T, int N) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return 0;
  const size_t NP = pad_states(N);
  const size_t nc = (T + kChunk - 1) / kChunk;
  return align_up((size_t)B * T * NP, 256) + align_up((size_t)B * nc * NP, 256) + align_up(sizeof(BandDesc), 256);
}

HMM355_API int hmm355_viterbi_plan_f32(const float* obs, int obs_mode, const float* log_P, const float* init,
                                       const void* plan, int B, int T, int N, int64_t* states, float* log_delta,
                                       float* final_score, void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || N < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!obs || !log_P || !init || !states || !log_delta || !workspace) return HMM355_E_ARG;
  if (obs_mode != HMM355_OBS_PROB && obs_mode != HMM355_OBS_LOG) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40 || B > 65535) return HMM355_E_SHAPE;
  if (workspace_bytes < hmm355_viterbi_workspace_bytes(B, T, N)) return HMM355_E_WORKSPACE;
  const int NP = pad_states(N);
  const int nc = (T + kChunk - 1) / kChunk;
  uint8_t* psi = static_cast<uint8_t*>(workspace);
  uint8_t* G = psi + align_up((size_t)B * T * NP, 256);
  uint8_t* bandp = G + align_up((size_t)B * nc * NP, 256);
  BandDesc* band = use_band() ? (plan ? static_cast<BandDesc*>(const_cast<void*>(plan))
                                      : reinterpret_cast<BandDesc*>(bandp))
                               : nullptr;
  // OBS_PROB: the chain's staging takes log(x + 1e-8) itself (logcr.h, ~12 fp64 operations
  // per element on the helper waves), so the emissions are read once and no log_obs tensor
  // round-trips through HBM
  VitArgs va{obs, log_P, init, log_delta, final_score, states, psi, G, B, T, N, obs_mode, nc, band};
  hipStream_t sm = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (NP) {
    case 64: e = launch_vit<64>(va, plan == nullptr, sm); break;
    case 128: e = launch_vit<128>(va, plan == nullptr, sm); break;
    default: e = launch_vit<256>(va, plan == nullptr, sm); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_viterbi_f32(const float* obs, int obs_mode, const float* log_P, const float* init, int B,
                                  int T, int N, int64_t* states, float* log_delta, float* final_score,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  return hmm355_viterbi_plan_f32(obs, obs_mode, log_P, init, nullptr, B, T, N, states, log_delta, final_score,
                                 workspace, workspace_bytes, stream);
}

#if HMM355_STAMP
HMM355_API int hmm355_debug_stamps_vit(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hmm355::g_rec_stamps), sizeof(unsigned long long) * (size_t)n);
}
#endif
