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
// hsmm_fwd_kernel: one 1024-thread workgroup per sequence, the segment END time t as the
//   loop index (semimarkov.hip's layout): 16 lanes (one DPP row) per state; lane `sub` owns
//   the start-time slots k = 4*sub + j (mod 64) of its state.  A live segment's torch-order
//   obs_sum state (the four group accumulators, the pending group and the tail sum) and its
//   predecessor score M stay in the slot's registers for the segment's life, so a step reads
//   one lp row, writes delta's per-state maximum Dm for the predecessor phase, and meets at
//   ONE barrier.  Per end time t it stores M[t][s] (the best fl(delta + logT) over
//   predecessors ending at t, for segments starting at t+1), the first s' attaining it, and
//   Dm[t][s].
// hsmm_backtrace_kernel: one wave per sequence walks the segments (hsmm.py:331-352); for each
//   segment it recomputes, bit-identically, the candidate deltas of the winning s' to find
//   the first d' and xb (the best total of the earlier candidates), and re-resolves the rare
//   case where an earlier candidate rounds to the same total.
#include <type_traits>

#include "common.h"

namespace hmm355 {

constexpr int kHsS = 64;    // max states
constexpr int kHsR = 64;    // start-time slots (> Dmax)
constexpr int kHsL = 128;   // lp row ring (two 64-row chunks)
constexpr int kHsSub = 16;                 // lanes per state (one DPP row)
constexpr int kHsThreads = kHsS * kHsSub;  // 1024
constexpr int kHsNJ = 4;                   // slots / predecessor states per lane

struct HsArgs {
  const float* lp;      // (B,T,S)
  const float* dur;     // (S,Dm)
  const float* logT;    // (S,S)
  float* Mg;            // (B,T,S): M[t][s], best predecessor total for segments starting at t+1
  uint8_t* S1;          // (B,T,S): first s' attaining M[t][s]
  float* Dg;            // (B,T,S): Dm[t][s] = max_d delta[t][s][d]
  int* fin;             // (B,2): final (s, d)
  float* scores;        // (B)
  int64_t* states;      // (B,T)
  int B, T, S, Dm;
};

struct HsLds {
  float lpr[kHsL][kHsS];
  float dur[kHsS][kHsR + 1];
  float dmx[2][kHsS];
  int fd[kHsS];
};

// compile-time loop: f(integral_constant<int, J>) for J in [B, E)
template <int J, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (J < E) {
    f(std::integral_constant<int, J>{});
    static_for<J + 1, E>(f);
  }
}

// all-reduce over the 16 lanes of a DPP row (the lanes of one state)
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
  const int s = tid >> 4, sub = tid & 15;
  const bool live = s < S;
  const float* lp = a.lp + (size_t)b * T * S;

  for (int i = tid; i < kHsS * kHsR; i += kHsThreads) {
    const int r = i / kHsR, d = i % kHsR;
    L.dur[r][d] = (r < S && d < Dm) ? a.dur[(size_t)r * Dm + d] : -INFINITY;
  }
  float lt[kHsNJ];  // log T[s'][s] for the lane's predecessor states s' = sub + 16j (-inf: excluded)
#pragma unroll
  for (int j = 0; j < kHsNJ; ++j) {
    const int sp = sub + kHsSub * j;
    const bool ok = live && sp < S && sp != s;
    const float v = a.logT[ok ? (size_t)sp * S + s : 0];
    lt[j] = ok ? v : -INFINITY;
  }

  constexpr int PER = kHsS * 64 / kHsThreads;  // lp values per thread per 64-row chunk
  float rc[PER];
  auto chunk_load = [&](int c) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int idx = tid + k * kHsThreads;
      const int row = c * 64 + idx / kHsS, col = idx % kHsS;
      const bool ok = row < T && col < S;
      const float v = lp[ok ? (size_t)row * S + col : 0];
      rc[k] = ok ? v : 0.f;
    }
  };
  auto chunk_store = [&](int c) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int idx = tid + k * kHsThreads;
      L.lpr[(c * 64 + idx / kHsS) % kHsL][idx % kHsS] = rc[k];
    }
  };
  chunk_load(0);
  chunk_store(0);
  if (T > 64) chunk_load(1);
  __syncthreads();

  // torch-CPU order of sum(lp[st:st+d, s]) (a strided slice): four accumulators over the
  // whole groups of 4, the tail folded into the first, then ((a0+a1)+a2)+a3.  Per slot:
  // G = completed-group sums, Q = the open group's sums (G_i + x_i), A0 = G0 + tail.
  float G[kHsNJ][4], Q[kHsNJ][4], A0[kHsNJ], mp[kHsNJ];
#pragma unroll
  for (int j = 0; j < kHsNJ; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { G[j][i] = 0.f; Q[j][i] = 0.f; }
    A0[j] = 0.f;
    mp[j] = -INFINITY;
  }
  float Mlast = -INFINITY;

  // One end time.  Lane `sub` owns slots k = 4*sub + j, so the new element's position in its
  // segment's group of four, (t - k) & 3 = (U - j) & 3 with U = t & 3, is a compile-time
  // constant of the unrolled copy: each slot runs only its own accumulator update.
  // Branch-free: every LDS read of the step is issued before its first use (a guarded read
  // ends in its own s_waitcnt, which serialised four duration-table round trips per step).
  // Rows s >= S of the tables hold -inf / 0, so the unguarded reads are in range and inert.
  auto end_step = [&](const int t, auto Uc) -> bool {
    constexpr int U = decltype(Uc)::value;
    const float x = L.lpr[t % kHsL][s];
    float v[kHsNJ], du[kHsNJ];
    int dd[kHsNJ];
    float mx = -INFINITY;
    static_for<0, kHsNJ>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      du[j] = L.dur[s][(t - (4 * sub + j)) & (kHsR - 1)];  // dur[s][d - 1], -inf for d > Dm
    });
    static_for<0, kHsNJ>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      const int age = (t - (4 * sub + j)) & (kHsR - 1);
      const int d = age + 1, st = t - age;
      dd[j] = d;
      constexpr int pos = (U - j) & 3;  // == age & 3
      if constexpr (pos == 0) {
        const bool fresh = age == 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) G[j][i] = fresh ? 0.f : G[j][i];
        mp[j] = fresh ? Mlast : mp[j];
        Q[j][0] = G[j][0] + x;
        A0[j] = Q[j][0];
      } else if constexpr (pos == 3) {
        Q[j][3] = G[j][3] + x;
#pragma unroll
        for (int i = 0; i < 4; ++i) G[j][i] = Q[j][i];
        A0[j] = G[j][0];
      } else {
        Q[j][pos] = G[j][pos] + x;
        A0[j] = A0[j] + x;
      }
      float o = 0.f + A0[j];
      o = o + G[j][1];
      o = o + G[j][2];
      o = o + G[j][3];
      const float u = du[j];
      // hsmm.py:269-274 (st == 0: no predecessor) / :304-314; mp == -inf (no predecessor path)
      // gives (mp + o) + u == -inf since o is finite
      const float val = st == 0 ? o + u : (mp[j] + o) + u;
      v[j] = (live && d <= Dm && st >= 0) ? val : -INFINITY;
      mx = fmaxf(mx, v[j]);
    });
    mx = row_max16(mx);
    if (sub == 0) {
      L.dmx[t & 1][s] = mx;  // -inf for the padding states s >= S (read unguarded below)
      if (live) a.Dg[((size_t)b * T + t) * S + s] = mx;
    }
    if (t == T - 1) {
      // best over (s asc, d asc) of delta[T-1][s][d-1], strict > (hsmm.py:319-329)
      int ld = 0x7fff;
#pragma unroll
      for (int j = 0; j < kHsNJ; ++j)
        if (v[j] == mx && dd[j] < ld) ld = dd[j];
      ld = row_min16_i(ld);
      if (live && sub == 0) L.fd[s] = ld;
      __syncthreads();
      if (tid < 64) {
        float bv = tid < S ? L.dmx[t & 1][tid] : -INFINITY;
        int bi = tid < S ? tid : 0x7fffffff;
        wave_argmax(bv, bi);
        if (tid == 0) {
          const bool any = bv != -INFINITY;
          a.scores[b] = bv;
          a.fin[2 * b] = any ? bi : 0;
          a.fin[2 * b + 1] = any ? L.fd[bi] : 1;
        }
      }
      return false;
    }
    step_barrier();
    // M[t][s] = max_{s' != s} fl(Dm[t][s'] + logT[s'][s]) and the first s' attaining it
    {
      float lm = -INFINITY;
      int ls = 0x7fff;
      float dmv[kHsNJ];
#pragma unroll
      for (int j = 0; j < kHsNJ; ++j) dmv[j] = L.dmx[t & 1][sub + kHsSub * j];  // all reads first
#pragma unroll
      for (int j = 0; j < kHsNJ; ++j) {
        const int sp = sub + kHsSub * j;
        // lt == -inf (excluded s') or dm == -inf: the sum is -inf (never +inf: no NaN)
        const float c = dmv[j] + lt[j];
        const bool gt = c > lm;
        lm = gt ? c : lm;
        ls = gt ? sp : ls;
      }
      const float M = row_max16(lm);
      const int s1 = row_min16_i((lm == M && M != -INFINITY) ? ls : 0x7fff);
      Mlast = M;
      if (live && sub == 0) {
        const size_t gi = ((size_t)b * T + t) * S + s;
        a.Mg[gi] = M;
        a.S1[gi] = (uint8_t)(M == -INFINITY ? 0 : s1);
      }
    }
    if ((t + 2) % 64 == 0) {  // rows of chunk c = (t+2)/64 are first read at step t+2
      const int cidx = (t + 2) >> 6;
      chunk_store(cidx);
      if ((cidx + 1) * 64 < T) chunk_load(cidx + 1);
      __syncthreads();
    }
    return true;
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  for (int t = 0; t < T; t += 4) {
    if (!end_step(t, I0{})) break;
    if (!end_step(t + 1, I1{})) break;
    if (!end_step(t + 2, I2{})) break;
    if (!end_step(t + 3, I3{})) break;
  }
}

// torch-order sum of lp[t0 .. t0+d-1][s] from global memory (d <= 63)
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

// delta of the segment (start st0, state s, duration d), exactly as the forward forms it
__device__ float hs_delta(const HsArgs& a, const float* lp, const float* Mb, int st0, int s, int d) {
  if (st0 < 0) return -INFINITY;
  const float o = hs_obs_sum_global(lp, a.S, st0, d, s);
  const float u = a.dur[(size_t)s * a.Dm + d - 1];
  if (st0 == 0) return o + u;
  const float m = Mb[(size_t)(st0 - 1) * a.S + s];
  return m == -INFINITY ? -INFINITY : (m + o) + u;
}

// torch-order sum of the d elements col[d-1-e], e = 0..d-1 (a segment's column in time
// order, staged newest-first in LDS)
__device__ __forceinline__ float hs_obs_sum_lds(const float* col, int d) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  const int m = d & ~3;
  int i = 0;
  for (; i < m; i += 4) {
    a0 += col[d - 1 - i];
    a1 += col[d - 2 - i];
    a2 += col[d - 3 - i];
    a3 += col[d - 4 - i];
  }
  for (; i < d; ++i) a0 += col[d - 1 - i];
  float r = 0.f + a0;
  r = r + a1;
  r = r + a2;
  r = r + a3;
  return r;
}

__global__ void __launch_bounds__(64) hsmm_backtrace_kernel(HsArgs a) {
  __shared__ float pcol[kHsR];  // lp[tau - i][s1], i < Dm: the predecessor's candidate column
  __shared__ float ccol[kHsR];  // lp[t - i][cs], i < cd: the current segment, newest first
  const int b = blockIdx.x, l = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const float* lp = a.lp + (size_t)b * T * S;
  const float* Mb = a.Mg + (size_t)b * T * S;
  const float* Db = a.Dg + (size_t)b * T * S;
  int t = T - 1, cs = a.fin[2 * b], cd = a.fin[2 * b + 1];
  while (t >= 0 && cd > 0) {
    int start = t - cd + 1;
    if (start < 0) start = 0;
    for (int u = start + l; u <= t; u += 64) a.states[(size_t)b * T + u] = cs;
    if (start == 0) break;
    const int tau = start - 1;  // end of the previous segment
    const size_t gi = (size_t)tau * S + cs;
    const float M = Mb[gi];
    int ns = 0, nd = 0;  // literal: psi never written when no predecessor exists (hsmm.py:313)
    if (M != -INFINITY) {
      ns = a.S1[(size_t)b * T * S + gi];
      const float lt = a.logT[(size_t)ns * S + cs];
      const int dlim = Dm < tau + 1 ? Dm : tau + 1;
      // one round trip: both columns, the candidates' predecessor scores, the per-state maxima
      const bool pin = l < dlim;
      const float pv = lp[(size_t)(pin ? tau - l : 0) * S + ns];
      const float cv = lp[(size_t)(l < cd ? t - l : 0) * S + cs];
      const int pst = tau - l;  // candidate d' = l + 1 starts at tau - l
      const float pm = (pin && pst >= 1) ? Mb[(size_t)(pst - 1) * S + ns] : 0.f;
      const float dm = l < ns ? Db[(size_t)tau * S + l] : -INFINITY;
      const float ltl = l < ns ? a.logT[(size_t)l * S + cs] : 0.f;
      if (pin) pcol[l] = pv;
      if (l < cd) ccol[l] = cv;
      __syncthreads();
      // first d' of s1 whose fl(delta + logT) equals M, and the best earlier total (xb)
      float dv = -INFINITY;
      bool hit = false;
      if (pin) {
        const float o = hs_obs_sum_lds(pcol, l + 1);
        const float u = a.dur[(size_t)ns * Dm + l];
        dv = pst == 0 ? o + u : (pm == -INFINITY ? -INFINITY : (pm + o) + u);
        hit = dv != -INFINITY && dv + lt == M;
      }
      const unsigned long long mask = __ballot(hit);
      nd = mask ? __ffsll((long long)mask) : 1;  // lane index + 1 = d'
      float xb = (l + 1 < nd && dv != -INFINITY) ? dv + lt : -INFINITY;
      if (l < ns && l != cs && dm != -INFINITY) xb = fmaxf(xb, dm + ltl);
      xb = wave_max(xb);
      const float o = hs_obs_sum_lds(ccol, cd);
      const float u = a.dur[(size_t)cs * Dm + cd - 1];
      const float F = (M + o) + u;
      if (xb != -INFINITY && (xb + o) + u == F) {
        // rare: an earlier candidate rounds to the same total — the first one wins (hsmm.py:308)
        const int p1 = ns * Dm + (nd - 1);
        int win = p1;
        for (int base = 0; base < p1; base += 64) {
          const int k = base + l;
          bool h2 = false;
          if (k < p1) {
            const int sp = k / Dm, dp = k % Dm + 1;
            if (sp != cs && dp <= tau + 1) {
              const float c2 = hs_delta(a, lp, Mb, tau - dp + 1, sp, dp);
              if (c2 != -INFINITY) h2 = ((c2 + a.logT[(size_t)sp * S + cs]) + o) + u == F;
            }
          }
          const unsigned long long m2 = __ballot(h2);
          if (m2) { win = base + __ffsll((long long)m2) - 1; break; }
        }
        ns = win / Dm;
        nd = win % Dm + 1;
      }
      __syncthreads();  // the columns are restaged for the next segment
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
  return align_up(n * 4, 256) + align_up(n, 256) + align_up(n * 4, 256) + align_up((size_t)B * 8, 256);
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
  uint8_t* S1 = reinterpret_cast<uint8_t*>(ws + align_up(n * 4, 256));
  float* Dg = reinterpret_cast<float*>(ws + align_up(n * 4, 256) + align_up(n, 256));
  int* fin = reinterpret_cast<int*>(ws + align_up(n * 4, 256) + align_up(n, 256) + align_up(n * 4, 256));
  HsArgs ha{lp, dur_lp, log_T, Mg, S1, Dg, fin, scores, states, B, T, S, Dmax};
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
