// hmm355 — Viterbi kernels and their per-NP launcher (included by vit_np*.hip, one translation
// unit per padded state count, so the three instantiations compile in parallel).
#pragma once
#include "recur.h"
#include "post.h"
#include "follow.h"

namespace hmm355 {


template <int NP>
__device__ __forceinline__ void vit_psi_follow(const RecArgs& ra, float* lds);

template <int NP>
__global__ void __launch_bounds__(kVitNT<NP>) vit_fwd_kernel(RecArgs ra) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if ((int)blockIdx.x >= ra.B) {
    if (ra.pub) {  // the decode beside a banded chain (HMM355_VIT_PLAN_BANDED, follow.h)
      if constexpr (kVitFused<NP>) {
        const int b = (int)blockIdx.x - ra.B;
        vit_lead<NP>(ra, b);
        vit_decode_follow<NP>(ra, b, lds);
      }
      return;
    }
    if constexpr (NP <= 128) vit_psi_follow<NP>(ra, lds);  // psi followers (HMM355_VIT_PLAN_DENSE)
    return;
  }
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

// ---- dense psi rows (every non-banded matrix: config 3, every trained layer)
// The matrix slice of lane (r, c) of wave w: M[blk][n] = L[i][o], i = 64*blk + 16*r + n,
// o = 16*w + c (-inf outside N x N).
template <int NP>
__device__ __forceinline__ void psi_dense_matrix(const VitArgs& a, float (&M)[VF<NP>::NBLK][16]) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int o = 16 * w + c, N = a.N;
#pragma unroll
  for (int blk = 0; blk < VF<NP>::NBLK; ++blk)
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int i = 64 * blk + 16 * r + n;
      const bool ok = i < N && o < N;
      const float v = a.log_P[ok ? (size_t)i * N + o : 0];
      M[blk][n] = ok ? v : -INFINITY;
    }
}

// Dense rows of one chunk into prow, then to HBM with the chunk map.  Lane (r, c) of wave w
// scans the inputs i = 64*blk + 16*r + n (n = 0..15) of output o = 16*w + c:
// s_i = fl(delta_{t-1,i} + L[i][o]), delta_{t-1,i} broadcast from lane 16r + n of the row (one
// v_add_f32_dpp row_newbcast per candidate).  The first argmax (torch.max, hmm.py:164-168) in
// three exact passes: the maximum m over the lane's candidates and then over the four row
// groups (max is order-free); each lane's smallest i with s_i == m (a reverse equality scan, no
// value carried); the smallest such i over the row groups.  Rows stream through a three-deep
// register ring (loads three steps ahead, no register copies, so no VALU-write -> DPP-read
// padding).  i >= N or o >= N: L = -inf, so s = -inf (and the row value read for such lanes is
// a valid element of the row).
template <int NP>
__device__ __forceinline__ void psi_dense_chunk(const VitArgs& a, uint8_t (*prow)[NP],
                                                const float (&M)[VF<NP>::NBLK][16], int b, int chunk) {
  using C = VF<NP>;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int o = 16 * w + c;
  const int T = a.T, N = a.N;
  const int t_lo = chunk * kChunk;
  const int t_hi = (t_lo + kChunk < T ? t_lo + kChunk : T) - 1;
  if (t_lo == 0 && tid < NP) prow[0][tid] = 0;  // psi_0 (hmm.py:156 zeros)
  const float* dbase = a.delta + (size_t)b * T * N;
  auto load_row = [&](int t, float(&yv)[C::NBLK]) {
    const int tt = t <= t_hi ? t : t_hi;  // (ahead of the chunk end: a valid row, unused)
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) {
      const int i = 64 * blk + l;
      yv[blk] = dbase[(size_t)(tt - 1) * N + (i < N ? i : 0)];
    }
  };
  auto psi_row = [&](int t, const float(&yv)[C::NBLK]) {
    float s[C::NBLK][16];
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) {
#define PSI_ADD(n)                                                                      \
  asm("v_add_f32_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf"         \
      : "=v"(s[blk][n])                                                                 \
      : "v"(yv[blk]), "v"(M[blk][n]));
      PSI_ADD(0) PSI_ADD(1) PSI_ADD(2) PSI_ADD(3) PSI_ADD(4) PSI_ADD(5) PSI_ADD(6) PSI_ADD(7)
      PSI_ADD(8) PSI_ADD(9) PSI_ADD(10) PSI_ADD(11) PSI_ADD(12) PSI_ADD(13) PSI_ADD(14) PSI_ADD(15)
#undef PSI_ADD
    }
    float m = fmaxf(s[0][0], s[0][1]);
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk)
#pragma unroll
      for (int n = (blk == 0 ? 2 : 0); n < 16; n += 2) m = fmaxf(fmaxf(m, s[blk][n]), s[blk][n + 1]);
    m = rows_max(m);
    int bk = 1 << 20;  // local index 16*blk + n of the first candidate equal to m (none: large)
#pragma unroll
    for (int blk = C::NBLK - 1; blk >= 0; --blk)
#pragma unroll
      for (int n = 15; n >= 0; --n) bk = s[blk][n] == m ? 16 * blk + n : bk;
    int bi = 64 * (bk >> 4) + 16 * r + (bk & 15);
    {
      int ia = bi, ib = bi;
      permlane16_swap_i(ia, ib);
      ia = ia < ib ? ia : ib;
      int ic = ia, id = ia;
      permlane32_swap_i(ic, id);
      bi = ic < id ? ic : id;
    }
    if (r == 0) prow[t - t_lo][o] = (uint8_t)bi;
  };
  const int t_first = t_lo > 0 ? t_lo : 1;
  if (t_first <= t_hi) {  // (T = 1: chunk 0 has psi_0 only)
    float y0[C::NBLK], y1[C::NBLK], y2[C::NBLK];
    load_row(t_first, y0);
    load_row(t_first + 1, y1);
    load_row(t_first + 2, y2);
    int t = t_first;
    for (; t + 2 <= t_hi; t += 3) {
      psi_row(t, y0);
      load_row(t + 3, y0);
      psi_row(t + 1, y1);
      load_row(t + 4, y1);
      psi_row(t + 2, y2);
      load_row(t + 5, y2);
    }
    if (t <= t_hi) psi_row(t, y0);
    if (t + 1 <= t_hi) psi_row(t + 1, y1);
  }
  __syncthreads();
  psi_write_rows<NP>(a, prow, b, chunk, t_lo, t_hi);
}

template <int NP>
__global__ void __launch_bounds__(VF<NP>::NT) vit_psi_kernel(VitArgs a) {
  using C = VF<NP>;
  static_assert(kPsiChunk == kChunk, "chunk length shared with the fused banded chain");
  __shared__ __attribute__((aligned(16))) uint8_t prow[kChunk][NP];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x;
  const bool banded = a.band && a.band->wc <= kBandMax;
  if (kVitFused<NP> && banded) {
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
  if (!banded && a.done && a.done[(size_t)b * a.nchunks + chunk]) return;  // a follower did it
  if (banded) {
    const int t_lo = chunk * kChunk;
    const int t_hi = (t_lo + kChunk < a.T ? t_lo + kChunk : a.T) - 1;
    if (t_lo == 0 && tid < NP) prow[0][tid] = 0;  // psi_0 (hmm.py:156 zeros)
    __shared__ float rowM[kChunk];
    __shared__ int rowI[kChunk];
    extern __shared__ __attribute__((aligned(16))) float drows[];  // [kChunk][NP] (dynamic)
    psi_band_rows<NP>(a, prow, rowM, rowI, drows, b, t_lo, t_hi);
    __syncthreads();
    psi_write_rows<NP>(a, prow, b, chunk, t_lo, t_hi);
    return;
  }
  float M[C::NBLK][16];
  psi_dense_matrix<NP>(a, M);
  psi_dense_chunk<NP>(a, prow, M, b, chunk);
}

// ---- psi followers (HMM355_VIT_PLAN_DENSE; RecArgs::prog): workgroups blockIdx >= B of the
// chain's own launch.  Workgroups are dispatched in index order, so the B chain workgroups own
// their CUs before any follower is placed, and a follower waiting for rows can never keep a
// chain from starting.  Each follower takes the tasks (chunk, sequence) chunk-major with a
// stride of the follower count, waits until that sequence's chain has published the blocks
// holding the chunk's rows (rec_rb_helper: once per chunk; acquire at agent scope, then a
// workgroup barrier), computes the chunk's psi rows and map exactly as the pass after the chain does,
// and marks the chunk done.  Waits are bounded by ONE stall budget per launch: the clock
// restarts whenever the awaited sequence's count moves, and a follower that sees no progress
// for kFollowStall ticks of the 100 MHz real-time counter (2 ms: a published 64-step chunk
// takes ~20-30 us) gives up ALL its remaining tasks.  A chain held back behind other work on
// its XCD therefore costs each follower at most 2 ms of polling, never 2 ms per task.  Chunks a
// follower does not finish are left to the pass after the chain, which computes every chunk
// not marked done, so the result never depends on the followers' timing.
constexpr long long kFollowStall = 200000;  // 2 ms

template <int NP>
__device__ __forceinline__ void vit_psi_follow(const RecArgs& ra, float* lds) {
  using C = VF<NP>;
  if (rec_band_code<kVit, NP>(ra) != 0) return;  // banded: the psi pass after the chain
  if (threadIdx.x >= C::NT) return;              // the dense psi layout's waves
  const VitArgs a{ra.obs, ra.mat, ra.init, ra.rows, ra.final_score, ra.states, ra.psi, ra.G,
                  ra.B, ra.T, ra.N, ra.obs_mode, ra.nchunks, ra.band, 0, ra.prog, ra.done};
  uint8_t(*prow)[NP] = reinterpret_cast<uint8_t(*)[NP]>(lds);
  int* ok_slot = reinterpret_cast<int*>(lds + kChunk * NP / 4);
  float M[C::NBLK][16];
  psi_dense_matrix<NP>(a, M);
  const int nf = (int)gridDim.x - a.B;
  const int c_lo = 0, c_hi = a.nchunks;
  const int ntask = a.B * (c_hi - c_lo);
  int last_have = -1;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int task = (int)blockIdx.x - a.B; task < ntask; task += nf) {
    const int chunk = c_lo + task / a.B, b = task % a.B;
    const int t_lo = chunk * kChunk;
    const int t_hi = (t_lo + kChunk < a.T ? t_lo + kChunk : a.T) - 1;
    // rows t_first - 1 .. t_hi - 1 are read: blocks 0 .. (t_hi - 1) / 16 must be out
    const int need = t_hi >= 1 ? ((t_hi - 1) >> 4) + 1 : 0;
    if (threadIdx.x == 0) {
      int ok = 1;
      // relaxed polls (no cache maintenance per poll), one agent-scope acquire once the count
      // is there (it invalidates this XCD's caches: once per task, not per poll)
      for (;;) {
        const int have = __hip_atomic_load(a.prog + (size_t)b * kProgSlots, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        if (have >= need) break;
        const long long now = __builtin_amdgcn_s_memrealtime();
        if (have != last_have) {  // progress (or a new sequence): restart the stall clock
          last_have = have;
          t0 = now;
        } else if (now - t0 > kFollowStall) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(16);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      *ok_slot = ok;
    }
    __syncthreads();
    const int ok = *ok_slot;
    __syncthreads();  // (ok_slot is rewritten by the next task's wait)
    if (!ok) return;  // stalled: every remaining task goes to the pass after the chain
    psi_dense_chunk<NP>(a, prow, M, b, chunk);
    __syncthreads();  // (prow is rewritten by the next task; the rows and map are issued)
    if (threadIdx.x == 0) a.done[(size_t)b * a.nchunks + chunk] = 1;
  }
}

template <int NP>
hipError_t launch_vit(const VitArgs& va, bool prep, hipStream_t sm) {
  hipError_t e = allow_lds(vit_fwd_kernel<NP>, kExclusiveLds);  // own the CU (recur.h)
  if (e != hipSuccess) return e;
  if (va.band && prep) {
    e = launch_band_prep(va.log_P, va.N, const_cast<BandDesc*>(va.band), sm);
    if (e != hipSuccess) return e;
  }
  RecArgs ra{va.obs, va.log_P, va.init, va.delta, nullptr, nullptr, va.B, va.T, va.N, va.obs_mode, va.N, va.band,
             nullptr, nullptr, va.psi};
  ra.G = va.G;
  ra.states = va.states;
  ra.final_score = va.final_score;
  ra.nchunks = va.nchunks;
  if (va.pub) {
    // the decode beside the banded chain (follow.h): B chains + B decode workgroups, nothing after
    ra.pub = va.pub;
    ra.lobuf = va.lobuf;
    ra.lready = va.lready;
    ra.path = va.path;
    ra.token = va.token;
    hipLaunchKernelGGL(vit_fwd_kernel<NP>, dim3(2 * va.B), dim3(kVitNT<NP>), kExclusiveLds, sm, ra);
    return hipGetLastError();
  }
  // psi followers beside a dense chain (NP <= 128: the chain with block-work helpers publishes)
  const int nfollow = (NP <= 128 && va.prog && va.done) ? va.nfollow : 0;
  if (nfollow > 0) {
    e = zero_words(va.prog, (size_t)va.B * kProgSlots * sizeof(int), sm);
    if (e == hipSuccess) e = zero_words(va.done, (size_t)va.B * va.nchunks, sm);
    if (e != hipSuccess) return e;
    ra.prog = va.prog;
    ra.done = va.done;
  }
  hipLaunchKernelGGL(vit_fwd_kernel<NP>, dim3(va.B + nfollow), dim3(kVitNT<NP>), kExclusiveLds, sm, ra);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // banded psi stages the chunk's delta rows in LDS (dynamic, kChunk x NP floats)
  const size_t psi_lds = va.band ? (size_t)kChunk * NP * sizeof(float) : 0;
  VitArgs vp = va;
  if (nfollow == 0) vp.done = nullptr;  // (no followers: every chunk here)
  hipLaunchKernelGGL(vit_psi_kernel<NP>, dim3(va.nchunks, va.B), dim3(VF<NP>::NT), psi_lds, sm, vp);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(vit_backtrace_kernel<NP>, dim3(va.nchunks, va.B), dim3(64), 0, sm, va);
  return hipGetLastError();
}

}  // namespace hmm355
