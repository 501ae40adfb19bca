// hmm355 — streaming decoders on gfx950 (§8(f) row 4).
//
// Replace the per-frame Python loops of StreamingHMMProcessor (reference streaming.py):
//   greedy  _greedy_decode       streaming.py:267-320: s_t = argmax_j fl(logT[s_{t-1}][j] + e_t[j])
//           (first chunk: fl(e_0[j] - log N)), first index on ties (torch.argmax);
//   beam    _beam_search_decode  streaming.py:322-377: every hypothesis h (score, last state)
//           expands to every state j, new score fl(fl(score_h + logT[last_h][j]) + e_t[j])
//           (the stream's very first frame, paths empty: fl(score_h + e_0[j])); the K best
//           survive, ordered by score descending and, on equal scores, by candidate index
//           h*N + j (Python's stable sort, reverse=True, keeps insertion order for ties).
//
// One workgroup per stream, 4 waves: wave 0 runs the recursion; waves 1-3 stage the next
// 64-frame tile of emissions into LDS while wave 0 consumes the current one (one barrier per
// 64 frames), so the chain never waits on HBM.  log T (N x N) is LDS-resident for N <= 128; for
// 128 < N <= 256 (round 5) the two emission tiles take 128 KiB and log T rows are read from
// global memory (L2) per step.  Each step is a wave argmax (greedy) or K rounds of wave argmax
// over the lane-local candidates (beam; K <= 32, K <= 16 when N > 128: the candidates of a lane
// are KM x NJ registers and one 64-bit mask).
// stream_beam_path_kernel walks the stored back-pointers from the best hypothesis (separate
// launch: it reads what the forward kernel wrote).
#include "common.h"

#pragma clang fp contract(off)

namespace hmm355 {

constexpr int kStMaxN = 256;   // states
constexpr int kStLdsN = 128;   // log T in LDS up to this many states
constexpr int kStMaxK = 32;    // beam width (hypothesis slots per stream)
constexpr int kStTile = 64;    // frames per staged tile

// LDS: two emission tiles [2][64][N], then log T [N][N] when N <= kStLdsN
inline size_t st_lds_bytes(int N) {
  return (size_t)2 * kStTile * N * sizeof(float) + (N <= kStLdsN ? (size_t)N * N * sizeof(float) : 0);
}

// stage tile `k` of the stream's emissions (rows [64k, 64k+64) of (T, N)) into buffer k&1;
// run by waves 1..3 (192 threads)
__device__ __forceinline__ void st_stage(float* em, const float* e, int T, int N, int k, int ltid) {
  const int r0 = k * kStTile;
  const int rows = min(kStTile, T - r0);
  if (rows <= 0) return;
  const int n = rows * N;
  float* dst = em + (k & 1) * kStTile * N;
  const float* src = e + (size_t)r0 * N;
  for (int i = ltid; i < n; i += 3 * kWave) dst[i] = src[i];
}

// log T: the LDS copy (N <= kStLdsN) or the global matrix
__device__ __forceinline__ const float* st_logT(float* smem, const float* logT, int N, int tid) {
  if (N > kStLdsN) return logT;
  float* lt = smem + 2 * kStTile * N;
  for (int i = tid; i < N * N; i += 256) lt[i] = logT[i];
  return lt;
}

template <int NJ>
__global__ void __launch_bounds__(256) stream_greedy_kernel(const float* emis, const float* logT, const int* prev,
                                                            float log_n, int T, int N, int64_t* states,
                                                            float* scores) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const float* e = emis + (size_t)b * T * N;
  const float* lt = st_logT(smem, logT, N, tid);
  if (w > 0) st_stage(smem, e, T, N, 0, tid - kWave);
  __syncthreads();
  const int ntiles = (T + kStTile - 1) / kStTile;
  int sp = prev[b];
  for (int k = 0; k < ntiles; ++k) {
    if (w > 0) {
      if (k + 1 < ntiles) st_stage(smem, e, T, N, k + 1, tid - kWave);
    } else {
      const float* et = smem + (k & 1) * kStTile * N;
      const int rows = min(kStTile, T - k * kStTile);
      for (int r = 0; r < rows; ++r) {
        float best = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
          const int j = lane + kWave * jj;
          if (j < N) {
            const float ev = et[r * N + j];
            const float v = sp < 0 ? ev - log_n : lt[sp * N + j] + ev;
            argmax_combine(best, bi, v, j);
          }
        }
        wave_argmax_dpp(best, bi);
        if (lane == 0) {
          const size_t o = (size_t)b * T + k * kStTile + r;
          states[o] = bi;
          scores[o] = best;
        }
        sp = bi;
      }
    }
    __syncthreads();
  }
}

struct BeamArgs {
  const float* emis;    // (B,T,N)
  const float* logT;    // (N,N)
  float* hyp_score;     // (B,kStMaxK) in/out
  int* hyp_last;        // (B,kStMaxK) in/out
  int* hyp_count;       // (B) in/out
  const int* first;     // (B): 1 = the stream's paths are empty (first frame rule)
  int16_t* parent;      // (B,T,K)
  int16_t* hstate;      // (B,T,K)
  int64_t* states;      // (B,T) best path of this chunk
  int T, N, K;
};

template <int NJ, int KM>
__global__ void __launch_bounds__(256) stream_beam_kernel(BeamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int T = a.T, N = a.N, K = a.K;
  const float* e = a.emis + (size_t)b * T * N;
  const float* lt = st_logT(smem, a.logT, N, tid);
  if (w > 0) st_stage(smem, e, T, N, 0, tid - kWave);
  __syncthreads();
  // hypotheses: uniform across the wave (every lane holds all of them)
  float hs[KM];
  int hl[KM];
  int kc = a.hyp_count[b];
#pragma unroll
  for (int h = 0; h < KM; ++h) {
    hs[h] = h < kc ? a.hyp_score[(size_t)b * kStMaxK + h] : -INFINITY;
    hl[h] = h < kc ? a.hyp_last[(size_t)b * kStMaxK + h] : 0;
  }
  bool empty = a.first[b] != 0;
  const int ntiles = (T + kStTile - 1) / kStTile;
  for (int k = 0; k < ntiles; ++k) {
    if (w > 0) {
      if (k + 1 < ntiles) st_stage(smem, e, T, N, k + 1, tid - kWave);
    } else {
      const float* et = smem + (k & 1) * kStTile * N;
      const int rows = min(kStTile, T - k * kStTile);
      for (int r = 0; r < rows; ++r) {
        const int t = k * kStTile + r;
        // lane-local expansions c[h][jj] of hypothesis h into state j = lane + 64 jj;
        // invalid ones (h >= kc, j >= N) are pre-marked as taken
        float c[KM][NJ];
        static_assert(KM * NJ <= 64, "candidate mask");
        uint64_t taken = 0;  // bit h*NJ + jj
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
          const int j = lane + kWave * jj;
          const float ev = j < N ? et[r * N + j] : 0.f;
#pragma unroll
          for (int h = 0; h < KM; ++h) {
            const bool ok = h < kc && j < N;
            const float tr = ok ? lt[hl[h] * N + j] : 0.f;
            c[h][jj] = empty ? hs[h] + ev : (hs[h] + tr) + ev;
            taken |= ok ? 0ull : 1ull << (h * NJ + jj);
          }
        }
        const int kn = min(K, kc * N);
        float ns[KM];
        int nl[KM], np[KM];
#pragma unroll
        for (int rr = 0; rr < KM; ++rr) {
          ns[rr] = -INFINITY; nl[rr] = 0; np[rr] = 0;
          if (rr < kn) {
            // best remaining expansion: score desc, then index h*N + j asc
            float bv = -INFINITY;
            int bi = 0x7fffffff;
#pragma unroll
            for (int h = 0; h < KM; ++h)
#pragma unroll
              for (int jj = 0; jj < NJ; ++jj) {
                const bool live = !((taken >> (h * NJ + jj)) & 1ull);
                const int ci = live ? h * N + lane + kWave * jj : 0x7fffffff;
                argmax_combine(bv, bi, live ? c[h][jj] : -INFINITY, ci);
              }
            wave_argmax_dpp(bv, bi);
            const int wh = bi / N, wj = bi - wh * N;
            ns[rr] = bv; nl[rr] = wj; np[rr] = wh;
#pragma unroll
            for (int h = 0; h < KM; ++h)
#pragma unroll
              for (int jj = 0; jj < NJ; ++jj)
                if (h == wh && lane + kWave * jj == wj) taken |= 1ull << (h * NJ + jj);
          }
        }
        if (lane < kn) {
          const size_t o = ((size_t)b * T + t) * K + lane;
          int lv = 0, pv = 0;
#pragma unroll
          for (int rr = 0; rr < KM; ++rr)
            if (rr == lane) { lv = nl[rr]; pv = np[rr]; }
          a.parent[o] = (int16_t)pv;
          a.hstate[o] = (int16_t)lv;
        }
#pragma unroll
        for (int h = 0; h < KM; ++h) { hs[h] = ns[h]; hl[h] = nl[h]; }
        kc = kn;
        empty = false;
      }
    }
    __syncthreads();
  }
  if (tid == 0) a.hyp_count[b] = kc;
  if (tid < KM && tid < kc) {
    float sv = 0.f; int lv = 0;
#pragma unroll
    for (int h = 0; h < KM; ++h)
      if (h == tid) { sv = hs[h]; lv = hl[h]; }
    a.hyp_score[(size_t)b * kStMaxK + tid] = sv;
    a.hyp_last[(size_t)b * kStMaxK + tid] = lv;
  }
}

// best path of the chunk: hypothesis 0 at the last frame, followed back through the parents
__global__ void __launch_bounds__(64) stream_beam_path_kernel(BeamArgs a) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  int r = 0;
  for (int t = a.T - 1; t >= 0; --t) {
    const size_t o = ((size_t)b * a.T + t) * a.K + r;
    a.states[(size_t)b * a.T + t] = a.hstate[o];
    r = a.parent[o];
  }
}

}  // namespace hmm355

using namespace hmm355;

static hipError_t st_lds(const void* k, int N) {
  return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)st_lds_bytes(N));
}

HMM355_API int hmm355_stream_greedy_f32(const float* emis, const float* log_T, const int* prev_state, float log_n,
                                        int B, int T, int N, int64_t* states, float* scores, void* stream) {
  if (B < 0 || T < 0 || N < 0) return HMM355_E_ARG;
  if (N < 1 || N > kStMaxN) return HMM355_E_STATES;
  if (B == 0 || T == 0) return HMM355_OK;
  if (!emis || !log_T || !prev_state || !states || !scores) return HMM355_E_ARG;
  auto kern = N <= kWave ? stream_greedy_kernel<1> : (N <= 2 * kWave ? stream_greedy_kernel<2> : stream_greedy_kernel<4>);
  hipError_t e = st_lds(reinterpret_cast<const void*>(kern), N);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kern, dim3(B), dim3(256), st_lds_bytes(N), static_cast<hipStream_t>(stream),
                     emis, log_T, prev_state, log_n, T, N, states, scores);
  e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_stream_beam_f32(const float* emis, const float* log_T, int B, int T, int N, int K,
                                      int live_max, float* hyp_score, int* hyp_last, int* hyp_count, const int* first,
                                      int16_t* parent, int16_t* hstate, int64_t* states, void* stream) {
  if (B < 0 || T < 0 || N < 0 || K < 0) return HMM355_E_ARG;
  if (N < 1 || N > kStMaxN) return HMM355_E_STATES;
  if (K < 1 || K > kStMaxK || live_max < 0 || live_max > kStMaxK) return HMM355_E_ARG;
  if (N > 2 * kWave && (K > 16 || live_max > 16)) return HMM355_E_ARG;  // (KM x NJ <= 64 candidates per lane)
  if (B == 0 || T == 0) return HMM355_OK;
  if (!emis || !log_T || !hyp_score || !hyp_last || !hyp_count || !first || !parent || !hstate || !states)
    return HMM355_E_ARG;
  BeamArgs ba{emis, log_T, hyp_score, hyp_last, hyp_count, first, parent, hstate, states, T, N, K};
  hipStream_t st = static_cast<hipStream_t>(stream);
  // hypothesis registers: enough for K and for the live count (which exceeds K after the
  // beam width was lowered)
  const int km = (K <= 8 && live_max <= 8) ? 8 : ((K <= 16 && live_max <= 16) ? 16 : 32);
  const int nj = N <= kWave ? 1 : (N <= 2 * kWave ? 2 : 4);
  void (*kern)(BeamArgs) = nullptr;
  switch (nj * 100 + km) {
    case 108: kern = stream_beam_kernel<1, 8>; break;
    case 116: kern = stream_beam_kernel<1, 16>; break;
    case 132: kern = stream_beam_kernel<1, 32>; break;
    case 208: kern = stream_beam_kernel<2, 8>; break;
    case 216: kern = stream_beam_kernel<2, 16>; break;
    case 232: kern = stream_beam_kernel<2, 32>; break;
    case 408: kern = stream_beam_kernel<4, 8>; break;
    default: kern = stream_beam_kernel<4, 16>; break;
  }
  hipError_t e = st_lds(reinterpret_cast<const void*>(kern), N);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kern, dim3(B), dim3(256), st_lds_bytes(N), st, ba);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(stream_beam_path_kernel, dim3(B), dim3(64), 0, st, ba);
  e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}
