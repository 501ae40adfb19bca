// hmm355 — HSMM segment Viterbi on gfx950 (BASELINE config 5).
//
// Replaces HSMMLayer.viterbi_decode_hsmm / _viterbi_decode_single (reference
// hsmm.py:208-354): a 5-deep Python loop over (t, s, d, s', d') with one 0-d tensor op per
// candidate (~55 h per sequence at S=64, Dmax=40, T=2000 on the reference's CPU path).
//
// Exact reorganisation (same as oracle/hmm_oracle.c:hsmm_viterbi_fast):
//   delta[e][s][d] for the segment [st, e], st = e-d+1, equals
//       st == 0 : fl(obs_sum(0,s,d) + dur[s][d-1])                       (hsmm.py:269-274)
//       st >= 1 : fl(fl(M[st][s] + obs_sum(st,s,d)) + dur[s][d-1])       (hsmm.py:304-314)
//   with M[st][s] = max_{s' != s, d'} fl(delta[st-1][s'][d'] + logT[s'][s]), because
//   g(x) = fl(fl(x + o) + u) is monotone: the literal max over candidates is g(M).  The
//   literal strict-> argmax is the first candidate (s' asc, d' asc) whose g(x) equals g(M):
//   the first candidate attaining M (p1) unless an EARLIER candidate rounds to the same
//   final value — so the kernel stores p1 and xb = max over the candidates before p1, and
//   the backtrace re-resolves exactly (rare) only for segments on the decoded path.
//   obs_sum is torch-CPU's order for a strided slice of length d: four accumulators over
//   whole groups of 4, the tail folded into the first, then ((a0+a1)+a2)+a3.
//
// hsmm_fwd_kernel: one 1024-thread workgroup per sequence (16 lanes = one DPP row per
// state), 3 barriers per start time:
//   A  group-complete updates of the per-(start,state) accumulators F0..F3 (LDS ring);
//   B  the S x Dmax candidate values delta[st-1][s'][d'] and their max over d';
//   C  M[st][s], p1 and xb (row-wide DPP combines).
//   lp rows arrive 64 at a time into a 128-row LDS ring, prefetched a chunk ahead.
// hsmm_backtrace_kernel: one wave per sequence walks the segments (hsmm.py:331-352).
#include "common.h"

namespace hmm355 {

constexpr int kHsS = 64;    // max states
constexpr int kHsR = 64;    // start-time ring (>= Dmax + 1)
constexpr int kHsL = 128;   // lp row ring
constexpr int kHsSub = 16;                 // lanes per state in phases B/C (one DPP row)
constexpr int kHsThreads = kHsS * kHsSub;  // 1024

struct HsArgs {
  const float* lp;      // (B,T,S)
  const float* dur;     // (S,Dm)
  const float* logT;    // (S,S)
  float* Mg;            // (B,T,S)
  uint16_t* P1;         // (B,T,S): s1 | d1 << 8
  float* XB;            // (B,T,S)
  int* fin;             // (B,2): final (s, d)
  float* scores;        // (B)
  int64_t* states;      // (B,T)
  int B, T, S, Dm;
};

struct HsLds {
  float lpr[kHsL][kHsS];
  float Mr[kHsR][kHsS];
  float F[kHsR][kHsS][4];
  float cand[kHsS][kHsR];
  float dmx[kHsS];
  float logT[kHsS][kHsS];
};

__device__ __forceinline__ float quad_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  return fmaxf(v, dpp_f<0x4E>(v));
}
__device__ __forceinline__ int quad_min_i(int v) {
  v = min(v, dpp_i<0xB1>(v));
  return min(v, dpp_i<0x4E>(v));
}

// torch-order obs_sum from the F accumulators of start st0 (length d, elements up to row st0+d-1)
__device__ __forceinline__ float hs_obs_sum(const HsLds& L, int st0, int d, int sp) {
  const float* Fv = L.F[st0 % kHsR][sp];
  const int g = d >> 2, rt = d & 3;
  float a0 = Fv[0];
  for (int i = 0; i < rt; ++i) a0 += L.lpr[(st0 + 4 * g + i) % kHsL][sp];
  float r = 0.f + a0;
  r = r + Fv[1];
  r = r + Fv[2];
  r = r + Fv[3];
  return r;
}

// all-reduce over the 16 lanes of a DPP row (the SUB lanes of one state)
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  return fmaxf(v, dpp_f<0x128>(v));
}
__device__ __forceinline__ int row_min16_i(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x124>(v));
  return min(v, dpp_i<0x128>(v));
}

__global__ void __launch_bounds__(kHsThreads) hsmm_fwd_kernel(HsArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  HsLds& L = *reinterpret_cast<HsLds*>(smem);
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const float* lp = a.lp + (size_t)b * T * S;
  // phases B/C: 16 lanes (one DPP row) per state q; lane `sub` owns d' = sub + 1 + 16j and
  // s' = sub + 16j
  const int q = tid >> 4, sub = tid & 15;
  constexpr int NJ = kHsR / kHsSub;  // 4

  for (int i = tid; i < S * S; i += kHsThreads) L.logT[i / S][i % S] = a.logT[i];
  float du[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int d = sub + 1 + kHsSub * j;
    const bool ok = q < S && d <= Dm;
    const float v = a.dur[ok ? (size_t)q * Dm + d - 1 : 0];
    du[j] = ok ? v : 0.f;
  }
  // phase-A item walk without integer division in the loop
  const int a_k0 = tid / S, a_s0 = tid % S;
  const int a_dk = kHsThreads / S, a_ds = kHsThreads % S;

  constexpr int PER = kHsS * 64 / kHsThreads;  // lp values per thread per 64-row chunk
  auto chunk_load = [&](int c, float (&r)[PER]) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int idx = tid + k * kHsThreads;
      const int row = c * 64 + idx / kHsS, col = idx % kHsS;
      const bool ok = row < T && col < S;
      const float v = lp[ok ? (size_t)row * S + col : 0];
      r[k] = ok ? v : 0.f;
    }
  };
  auto chunk_store = [&](int c, const float (&r)[PER]) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int idx = tid + k * kHsThreads;
      const int row = c * 64 + idx / kHsS, col = idx % kHsS;
      L.lpr[row % kHsL][col] = r[k];
    }
  };
  float rc[PER];
  chunk_load(0, rc);
  chunk_store(0, rc);
  if (T > 64) chunk_load(1, rc);
  __syncthreads();

  // ---- A(st): element row st-1 joins every active start; complete groups fold into F.
  // Runs for st = 1 before the loop and for st + 1 in the same phase as C(st) (they touch
  // disjoint LDS), so a start costs two barriers: A+C | B.
  auto phaseA = [&](int st) {
    const int e = st - 1;
    int k = a_k0, sp = a_s0;
    while (k < Dm) {
      const int st0 = e - k;  // start whose element index k is row e
      if (st0 >= 0) {
        float* Fv = L.F[st0 % kHsR][sp];
        if (k == 0) { Fv[0] = 0.f; Fv[1] = 0.f; Fv[2] = 0.f; Fv[3] = 0.f; }
        if ((k & 3) == 3) {  // group [k-3, k] complete
          Fv[0] += L.lpr[(st0 + k - 3) % kHsL][sp];
          Fv[1] += L.lpr[(st0 + k - 2) % kHsL][sp];
          Fv[2] += L.lpr[(st0 + k - 1) % kHsL][sp];
          Fv[3] += L.lpr[(st0 + k) % kHsL][sp];
        }
      }
      k += a_dk;
      sp += a_ds;
      if (sp >= S) { sp -= S; ++k; }
    }
  };
  phaseA(1);
  __syncthreads();

  for (int st = 1; st <= T; ++st) {
    // ---- B: candidates delta[st-1][s'][d'-1] and their max over d'
    const int dlim = Dm < st ? Dm : st;
    if (q < S) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int d = sub + 1 + kHsSub * j;
        if (d <= Dm) {
          float v = -INFINITY;
          if (d <= dlim) {
            const int st0 = st - d;
            const float o = hs_obs_sum(L, st0, d, q);
            if (st0 == 0) {
              v = o + du[j];
            } else {
              const float m = L.Mr[st0 % kHsR][q];
              v = (m == -INFINITY) ? -INFINITY : (m + o) + du[j];
            }
          }
          L.cand[q][d - 1] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = row_max16(mx);
      if (sub == 0) L.dmx[q] = mx;
    }
    __syncthreads();
    if (st == T) break;  // final candidates are in L.cand
    // ---- C: M[st][s], first candidate attaining it (p1) and xb
    if (q < S) {
      const int s = q;
      float lm = -INFINITY;
      int ls = 0x7fff;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int sp = sub + kHsSub * j;
        if (sp < S) {
          const float dm = L.dmx[sp];
          const float v = (sp == s || dm == -INFINITY) ? -INFINITY : dm + L.logT[sp][s];
          if (v > lm) { lm = v; ls = sp; }
        }
      }
      const float M = row_max16(lm);
      int s1 = row_min16_i(lm == M && M != -INFINITY ? ls : 0x7fff);
      float xb1 = -INFINITY, xb2 = -INFINITY;
      int d1 = 0x7fff;
      if (M != -INFINITY) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int sp = sub + kHsSub * j;
          if (sp < s1) {
            const float dm = L.dmx[sp];
            const float v = (sp == s || dm == -INFINITY) ? -INFINITY : dm + L.logT[sp][s];
            xb1 = fmaxf(xb1, v);
          }
        }
        const float lt = L.logT[s1][s];
        int ld = 0x7fff;
        float cv[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int d = sub + 1 + kHsSub * j;
          const float c = d <= Dm ? L.cand[s1][d - 1] : -INFINITY;
          cv[j] = c == -INFINITY ? -INFINITY : c + lt;
          if (d <= Dm && cv[j] == M && ld == 0x7fff) ld = d;
        }
        d1 = row_min16_i(ld);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int d = sub + 1 + kHsSub * j;
          if (d < d1 && d <= Dm) xb2 = fmaxf(xb2, cv[j]);
        }
      } else {
        s1 = 0;
        d1 = 0;  // literal: psi never written (hsmm.py:313)
      }
      const float xb = row_max16(fmaxf(xb1, xb2));
      if (sub == 0) {
        L.Mr[st % kHsR][s] = M;
        const size_t gi = ((size_t)b * T + st) * S + s;
        a.Mg[gi] = M;
        a.P1[gi] = (uint16_t)(s1 | (d1 << 8));
        a.XB[gi] = xb;
      }
    }
    if ((st + 1) % 64 == 0) {  // chunk c = (st+1)/64 holds row st, which A(st+1) needs
      const int c = (st + 1) >> 6;
      chunk_store(c, rc);
      if ((c + 1) * 64 < T) chunk_load(c + 1, rc);
    }
    phaseA(st + 1);
    __syncthreads();
  }
  // final: best over (s asc, d asc) of delta[T-1][s][d-1], strict > (hsmm.py:319-329):
  // the maximum with the smallest linear index s*Dm + d-1
  {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < S * Dm; i += kHsThreads) {
      const float v = L.cand[i / Dm][i % Dm];
      argmax_combine(bv, bi, v, i);
    }
    wave_argmax(bv, bi);
    __shared__ float fv[kHsThreads / 64];
    __shared__ int fi[kHsThreads / 64];
    if ((tid & 63) == 0) { fv[tid >> 6] = bv; fi[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
      float best = fv[0];
      int besti = fi[0];
      for (int w = 1; w < kHsThreads / 64; ++w) argmax_combine(best, besti, fv[w], fi[w]);
      a.scores[b] = best;
      a.fin[2 * b] = besti / Dm;
      a.fin[2 * b + 1] = besti % Dm + 1;
    }
  }
}

// torch-order sum of lp[t0 .. t0+d-1][s] from global memory (lane 0 only; d <= 63)
__device__ float hs_obs_sum_global(const float* lp, int S, int t0, int d, int s) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  const int m = d & ~3;
  int i = 0;
  for (; i < m; i += 4) {
    a0 += lp[(size_t)(t0 + i) * S + s];
    a1 += lp[(size_t)(t0 + i + 1) * S + s];
    a2 += lp[(size_t)(t0 + i + 2) * S + s];
    a3 += lp[(size_t)(t0 + i + 3) * S + s];
  }
  for (; i < d; ++i) a0 += lp[(size_t)(t0 + i) * S + s];
  float r = 0.f + a0;
  r = r + a1;
  r = r + a2;
  r = r + a3;
  return r;
}

// delta value of the segment (start st0, state s, duration d), as the forward defines it
__device__ float hs_delta(const HsArgs& a, const float* lp, int b, int st0, int s, int d) {
  if (st0 < 0) return -INFINITY;
  const float o = hs_obs_sum_global(lp, a.S, st0, d, s);
  const float u = a.dur[(size_t)s * a.Dm + d - 1];
  if (st0 == 0) return o + u;
  const float m = a.Mg[((size_t)b * a.T + st0) * a.S + s];
  return m == -INFINITY ? -INFINITY : (m + o) + u;
}

__global__ void __launch_bounds__(64) hsmm_backtrace_kernel(HsArgs a) {
  const int b = blockIdx.x, l = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const float* lp = a.lp + (size_t)b * T * S;
  int t = T - 1, cs = a.fin[2 * b], cd = a.fin[2 * b + 1];
  while (t >= 0 && cd > 0) {
    int start = t - cd + 1;
    if (start < 0) start = 0;
    for (int u = start + l; u <= t; u += 64) a.states[(size_t)b * T + u] = cs;
    if (start == 0) break;
    const size_t gi = ((size_t)b * T + start) * S + cs;
    const float M = a.Mg[gi];
    const uint16_t p = a.P1[gi];
    int ns = p & 0xff, nd = p >> 8;
    if (M != -INFINITY) {
      const float xb = a.XB[gi];
      const float o = hs_obs_sum_global(lp, S, start, cd, cs);
      const float u = a.dur[(size_t)cs * Dm + cd - 1];
      const float F = (M + o) + u;
      if (xb != -INFINITY && (xb + o) + u == F) {
        // rare: an earlier candidate rounds to the same total — first one wins (hsmm.py:308)
        const int p1 = ns * Dm + (nd - 1);
        int win = p1;
        for (int base = 0; base < p1; base += 64) {
          const int k = base + l;
          bool hit = false;
          if (k < p1) {
            const int sp = k / Dm, dp = k % Dm + 1;
            if (sp != cs) {
              const float dv = hs_delta(a, lp, b, start - dp, sp, dp);
              if (dv != -INFINITY) {
                const float x = dv + a.logT[(size_t)sp * S + cs];
                hit = ((x + o) + u) == F;
              }
            }
          }
          const unsigned long long mask = __ballot(hit);
          if (mask) { win = base + __ffsll((long long)mask) - 1; break; }
        }
        ns = win / Dm;
        nd = win % Dm + 1;
      }
    }
    t = start - 1;
    cs = ns;
    cd = nd;
  }
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_hsmm_workspace_bytes(int B, int T, int S, int Dmax) {
  if (B < 0 || T < 1 || S < 1 || S > kHsS || Dmax < 1 || Dmax >= kHsR) return 0;
  const size_t n = (size_t)B * T * S;
  return align_up(n * 4, 256) + align_up(n * 2, 256) + align_up(n * 4, 256) + align_up((size_t)B * 8, 256);
}

HMM355_API int hmm355_hsmm_viterbi_f32(const float* lp, const float* dur_lp, const float* log_T, int B, int T,
                                       int S, int Dmax, int64_t* states, float* scores, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  if (B < 0 || S < 0 || Dmax < 0) return HMM355_E_ARG;
  if (S < 1 || S > kHsS) return HMM355_E_STATES;
  if (Dmax < 1 || Dmax >= kHsR) return HMM355_E_DURATION;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!lp || !dur_lp || !log_T || !states || !scores || !workspace) return HMM355_E_ARG;
  if (workspace_bytes < hmm355_hsmm_workspace_bytes(B, T, S, Dmax)) return HMM355_E_WORKSPACE;
  const size_t n = (size_t)B * T * S;
  char* ws = static_cast<char*>(workspace);
  float* Mg = reinterpret_cast<float*>(ws);
  uint16_t* P1 = reinterpret_cast<uint16_t*>(ws + align_up(n * 4, 256));
  float* XB = reinterpret_cast<float*>(ws + align_up(n * 4, 256) + align_up(n * 2, 256));
  int* fin = reinterpret_cast<int*>(ws + align_up(n * 4, 256) + align_up(n * 2, 256) + align_up(n * 4, 256));
  HsArgs ha{lp, dur_lp, log_T, Mg, P1, XB, fin, scores, states, B, T, S, Dmax};
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = allow_lds(hsmm_fwd_kernel, sizeof(HsLds));
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(hsmm_fwd_kernel, dim3(B), dim3(kHsThreads), sizeof(HsLds), st, ha);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(hsmm_backtrace_kernel, dim3(B), dim3(64), 0, st, ha);
  e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}
