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
// hsmm_fwd_kernel<SUB, NJ, SMAX>: one workgroup per sequence (SMAX * SUB threads), the segment
//   END time t as the loop index (semimarkov.hip's layout): SUB lanes (a DPP group) per state;
//   lane `sub` owns the start-time slots k = NJ*sub + j (mod R = SUB*NJ) of its state.  A live
//   segment's torch-order obs_sum state (the four group accumulators, the pending group and
//   the tail sum) and its predecessor score M stay in the slot's registers for the segment's
//   life, so a step reads one lp row, writes delta's per-state maximum Dm for the predecessor
//   phase, and meets at ONE barrier.  Per end time t it stores M[t][s] (the best
//   fl(delta + logT) over predecessors ending at t, for segments starting at t+1), the first
//   s' attaining it, and Dm[t][s].  Geometries: (16, 4, 64) for the config-5 class (S <= 64,
//   Dmax <= 63), (8, 8, 64) the same with 8-lane groups, (8, 16, 64) for Dmax <= 127 and
//   (4, 16, 128) for 65 <= S <= 128 with Dmax <= 63.
// hsmm_backtrace_kernel: one wave per sequence walks the segments (hsmm.py:331-352); for each
//   segment it recomputes, bit-identically, the candidate deltas of the winning s' to find
//   the first d' and xb (the best total of the earlier candidates), and re-resolves the rare
//   case where an earlier candidate rounds to the same total.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace hmm355 {

constexpr int kHsL = 128;    // lp row ring (two 64-row chunks)
constexpr int kHsSMax = 128; // states (the largest geometry below)
constexpr int kHsDMax = 127; // durations (slot ring R = 128)

// Kernel geometry: SUB lanes per state (one DPP group), NJ start-time slots per lane, SMAX
// states per workgroup.  R = SUB * NJ slots (a segment's duration is < R), NT threads.
template <int SUB, int NJ, int SMAX>
struct HsG {
  static constexpr int R = SUB * NJ;
  static constexpr int NT = SMAX * SUB;
  static constexpr int NPRED = SMAX / SUB;   // predecessor states per lane
  static constexpr int PER = 64 * SMAX / NT; // lp values per thread per 64-row chunk
  static_assert(NJ % 4 == 0, "slot position (t - k) & 3 must be a compile-time constant");
  static_assert(NT <= 1024, "one workgroup per sequence");
};

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

template <int SMAX, int R>
struct HsLds {
  float lpr[kHsL][SMAX];
  float dur[SMAX][R + 1];
  float dmx[2][SMAX];
  int fd[SMAX];
};

// all-reduce over the SUB lanes of a state group (16: one DPP row; 8: half a row; 4: a quad)
template <int SUB>
__device__ __forceinline__ float grp_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));                       // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp_f<0x4E>(v));                       // quad_perm [2,3,0,1]
  if constexpr (SUB == 8) v = fmaxf(v, dpp_f<0x141>(v));   // row_half_mirror
  if constexpr (SUB == 16) {
    v = fmaxf(v, dpp_f<0x124>(v));                    // row_ror:4
    v = fmaxf(v, dpp_f<0x128>(v));                    // row_ror:8
  }
  return v;
}
template <int SUB>
__device__ __forceinline__ int grp_min_i(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  if constexpr (SUB == 8) v = min(v, dpp_i<0x141>(v));
  if constexpr (SUB == 16) {
    v = min(v, dpp_i<0x124>(v));
    v = min(v, dpp_i<0x128>(v));
  }
  return v;
}

template <int SUB, int NJ, int SMAX>
__global__ void __launch_bounds__((HsG<SUB, NJ, SMAX>::NT)) hsmm_fwd_kernel(HsArgs a) {
  using G = HsG<SUB, NJ, SMAX>;
  constexpr int R = G::R, NT = G::NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  HsLds<SMAX, R>& L = *reinterpret_cast<HsLds<SMAX, R>*>(smem);
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const int s = tid / SUB, sub = tid % SUB;
  const bool live = s < S;
  const float* lp = a.lp + (size_t)b * T * S;

  for (int i = tid; i < SMAX * R; i += NT) {
    const int r = i / R, d = i % R;
    L.dur[r][d] = (r < S && d < Dm) ? a.dur[(size_t)r * Dm + d] : -INFINITY;
  }
  float lt[G::NPRED];  // log T[s'][s] for the lane's predecessor states s' = sub + SUB j (-inf: excluded)
#pragma unroll
  for (int j = 0; j < G::NPRED; ++j) {
    const int sp = sub + SUB * j;
    const bool ok = live && sp < S && sp != s;
    const float v = a.logT[ok ? (size_t)sp * S + s : 0];
    lt[j] = ok ? v : -INFINITY;
  }

  float rc[G::PER];
  auto chunk_load = [&](int c) {
#pragma unroll
    for (int k = 0; k < G::PER; ++k) {
      const int idx = tid + k * NT;
      const int row = c * 64 + idx / SMAX, col = idx % SMAX;
      const bool ok = row < T && col < S;
      const float v = lp[ok ? (size_t)row * S + col : 0];
      rc[k] = ok ? v : 0.f;
    }
  };
  auto chunk_store = [&](int c) {
#pragma unroll
    for (int k = 0; k < G::PER; ++k) {
      const int idx = tid + k * NT;
      L.lpr[(c * 64 + idx / SMAX) % kHsL][idx % SMAX] = rc[k];
    }
  };
  chunk_load(0);
  chunk_store(0);
  if (T > 64) chunk_load(1);
  __syncthreads();

  // torch-CPU order of sum(lp[st:st+d, s]) (a strided slice): four accumulators over the
  // whole groups of 4, the tail folded into the first, then ((a0+a1)+a2)+a3.  Per slot:
  // G = completed-group sums, A0 = G0 + tail.  A group's four elements are the state's last
  // four lp values whatever the slot, so they come from one per-lane ring xr (x at time t in
  // xr[t & 3]) when the group closes: G_i += x_{t-3+i} (the same fp32 adds as accumulating
  // each element into its own accumulator as it arrives).
  float Gs[NJ][4], A0[NJ], mp[NJ], xr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) Gs[j][i] = 0.f;
    A0[j] = 0.f;
    mp[j] = -INFINITY;
  }
  float Mlast = -INFINITY;
  // delta of slot j's segment (duration d, start st) ending now, from its updated registers
  auto slot_val = [&](int j, int d, int st, float u) -> float {
    float o = 0.f + A0[j];
    o = o + Gs[j][1];
    o = o + Gs[j][2];
    o = o + Gs[j][3];
    // hsmm.py:269-274 (st == 0: no predecessor) / :304-314; mp == -inf (no predecessor path)
    // gives (mp + o) + u == -inf since o is finite
    const float val = st == 0 ? o + u : (mp[j] + o) + u;
    return (live && d <= Dm && st >= 0) ? val : -INFINITY;
  };

  // One end time.  Lane `sub` owns slots k = NJ*sub + j, so the new element's position in its
  // segment's group of four, (t - k) & 3 = (U - j) & 3 with U = t & 3 (NJ is a multiple of 4),
  // is a compile-time constant of the unrolled copy: each slot runs only its own accumulator
  // update.  Branch-free: every LDS read of the step is issued before its first use (a guarded
  // read ends in its own s_waitcnt, which serialised the duration-table round trips).  Rows
  // s >= S of the tables hold -inf / 0, so the unguarded reads are in range and inert.
  auto end_step = [&](const int t, auto Uc) -> bool {
    constexpr int U = decltype(Uc)::value;
    const float x = L.lpr[t % kHsL][s];
    xr[U] = x;
    float du[NJ];
    float mx = -INFINITY;
    static_for<0, NJ>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      du[j] = L.dur[s][(t - (NJ * sub + j)) & (R - 1)];  // dur[s][d - 1], -inf for d > Dm
    });
    static_for<0, NJ>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      const int age = (t - (NJ * sub + j)) & (R - 1);
      const int d = age + 1, st = t - age;
      constexpr int pos = (U - j) & 3;  // == age & 3
      if constexpr (pos == 0) {
        const bool fresh = age == 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) Gs[j][i] = fresh ? 0.f : Gs[j][i];
        mp[j] = fresh ? Mlast : mp[j];
        A0[j] = Gs[j][0] + x;
      } else if constexpr (pos == 3) {
#pragma unroll
        for (int i = 0; i < 4; ++i) Gs[j][i] = Gs[j][i] + xr[(U - 3 + i) & 3];
        A0[j] = Gs[j][0];
      } else {
        A0[j] = A0[j] + x;
      }
      mx = fmaxf(mx, slot_val(j, d, st, du[j]));
    });
    mx = grp_max<SUB>(mx);
    if (sub == 0) {
      L.dmx[t & 1][s] = mx;  // -inf for the padding states s >= S (read unguarded below)
      if (live) a.Dg[((size_t)b * T + t) * S + s] = mx;
    }
    if (t == T - 1) {
      // best over (s asc, d asc) of delta[T-1][s][d-1], strict > (hsmm.py:319-329)
      int ld = 0x7fff;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {  // (recomputed here, once, rather than kept live every step)
        const int age = (t - (NJ * sub + j)) & (R - 1);
        const int d = age + 1;
        if (slot_val(j, d, t - age, du[j]) == mx && d < ld) ld = d;
      }
      ld = grp_min_i<SUB>(ld);
      if (live && sub == 0) L.fd[s] = ld;
      __syncthreads();
      if (tid < 64) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < (SMAX + 63) / 64; ++k) {
          const int ss = tid + 64 * k;
          if (ss < S) argmax_combine(bv, bi, L.dmx[t & 1][ss], ss);
        }
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
      float dmv[G::NPRED];
#pragma unroll
      for (int j = 0; j < G::NPRED; ++j) dmv[j] = L.dmx[t & 1][sub + SUB * j];  // all reads first
#pragma unroll
      for (int j = 0; j < G::NPRED; ++j) {
        const int sp = sub + SUB * j;
        // lt == -inf (excluded s') or dm == -inf: the sum is -inf (never +inf: no NaN)
        const float c = dmv[j] + lt[j];
        const bool gt = c > lm;
        lm = gt ? c : lm;
        ls = gt ? sp : ls;
      }
      const float M = grp_max<SUB>(lm);
      const int s1 = grp_min_i<SUB>((lm == M && M != -INFINITY) ? ls : 0x7fff);
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

// torch-order sum of lp[t0 .. t0+d-1][s] from global memory
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

// R >= the longest duration; every lane owns the candidates d' = l + 1 + 64k, k < R/64, and
// the predecessor states s' = l + 64k, k < SMAX/64
template <int R, int SMAX>
__global__ void __launch_bounds__(64) hsmm_backtrace_kernel(HsArgs a) {
  constexpr int K = R / 64;
  constexpr int KS = (SMAX + 63) / 64;
  __shared__ float pcol[R];  // lp[tau - i][s1], i < Dm: the predecessor's candidate column
  __shared__ float ccol[R];  // lp[t - i][cs], i < cd: the current segment, newest first
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
      // one round trip: both columns, the candidates' predecessor scores, the other states'
      // best totals (xb)
      float pm[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = l + 64 * k;
        const bool pin = e < dlim;
        const float pv = lp[(size_t)(pin ? tau - e : 0) * S + ns];
        const int pst = tau - e;  // candidate d' = e + 1 starts at tau - e
        pm[k] = (pin && pst >= 1) ? Mb[(size_t)(pst - 1) * S + ns] : 0.f;
        if (pin) pcol[e] = pv;
        if (e < cd) ccol[e] = lp[(size_t)(t - e) * S + cs];
      }
      // max over s' < ns, s' != cs of fl(Dm[tau][s'] + logT[s'][cs]) (loads in the same round trip)
      float dm[KS], ltl[KS];
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int sp = l + 64 * k;
        const bool ok = sp < ns;
        dm[k] = ok ? Db[(size_t)tau * S + sp] : -INFINITY;
        ltl[k] = ok ? a.logT[(size_t)sp * S + cs] : 0.f;
      }
      __syncthreads();
      float xo = -INFINITY;
#pragma unroll
      for (int k = 0; k < KS; ++k)
        if (l + 64 * k != cs && dm[k] != -INFINITY) xo = fmaxf(xo, dm[k] + ltl[k]);
      // first d' of s1 whose fl(delta + logT) equals M, and the best earlier total (xb)
      float dv[K];
      nd = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = l + 64 * k;
        dv[k] = -INFINITY;
        bool hit = false;
        if (e < dlim) {
          const float o = hs_obs_sum_lds(pcol, e + 1);
          const float u = a.dur[(size_t)ns * Dm + e];
          const int pst = tau - e;
          dv[k] = pst == 0 ? o + u : (pm[k] == -INFINITY ? -INFINITY : (pm[k] + o) + u);
          hit = dv[k] != -INFINITY && dv[k] + lt == M;
        }
        const unsigned long long mask = __ballot(hit);
        if (nd == 0 && mask) nd = 64 * k + __ffsll((long long)mask);  // lane index + 1 = d'
      }
      if (nd == 0) nd = 1;
      float xb = xo;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (l + 64 * k + 1 < nd && dv[k] != -INFINITY) xb = fmaxf(xb, dv[k] + lt);
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

// Geometries (S <= SMAX, Dmax < R): the config-5 class S <= 64, Dmax <= 63 takes the 8-lane
// form unless HMM355_HSMM_SUB=16 asks for the 16-lane one.
// The larger geometries run 512 threads (8 waves) so a lane has 256 VGPRs for its 16 slots.
// (S <= 128 with 64 <= Dmax <= 127 would need 32 slots per lane: beyond the register file;
// rejected.)
enum HsCfg : int { kHs16x4 = 0, kHs8x8s64 = 1, kHs8x16 = 2, kHs4x16 = 3, kHsNone = -1 };
inline int hsmm_cfg(int S, int Dm) {
  if (S < 1 || Dm < 1) return kHsNone;
  if (S <= 64 && Dm < 64) {
    // 8-lane groups, 512 threads: 1.48 vs 1.57 ms for the 16-lane form at config 5
    // (profiles/r3f_c5_sub*.log); HMM355_HSMM_SUB=16 selects the 16-lane form
    const char* e = getenv("HMM355_HSMM_SUB");
    return (e && e[0] == '1' && e[1] == '6') ? kHs16x4 : kHs8x8s64;
  }
  if (S <= 64 && Dm < 128) return kHs8x16;
  if (S <= 128 && Dm < 64) return kHs4x16;
  return kHsNone;
}

template <int SUB, int NJ, int SMAX>
static hipError_t launch_hsmm(const HsArgs& ha, hipStream_t st) {
  using G = HsG<SUB, NJ, SMAX>;
  const size_t lds = sizeof(HsLds<SMAX, G::R>);
  hipError_t e = allow_lds(hsmm_fwd_kernel<SUB, NJ, SMAX>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((hsmm_fwd_kernel<SUB, NJ, SMAX>), dim3(ha.B), dim3(G::NT), lds, st, ha);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((hsmm_backtrace_kernel<G::R, SMAX>), dim3(ha.B), dim3(64), 0, st, ha);
  return hipGetLastError();
}

}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_hsmm_workspace_bytes(int B, int T, int S, int Dmax) {
  if (B < 0 || T < 1 || hsmm_cfg(S, Dmax) == kHsNone) return 0;
  const size_t n = (size_t)B * T * S;
  return align_up(n * 4, 256) + align_up(n, 256) + align_up(n * 4, 256) + align_up((size_t)B * 8, 256);
}

HMM355_API int hmm355_hsmm_viterbi_f32(const float* lp, const float* dur_lp, const float* log_T, int B, int T,
                                       int S, int Dmax, int64_t* states, float* scores, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  if (B < 0 || S < 0 || Dmax < 0) return HMM355_E_ARG;
  if (S < 1 || S > kHsSMax) return HMM355_E_STATES;
  if (Dmax < 1 || Dmax > kHsDMax || hsmm_cfg(S, Dmax) == kHsNone) return HMM355_E_DURATION;  // S > 64: Dmax <= 63
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
  hipError_t e;
  switch (hsmm_cfg(S, Dmax)) {
    case kHs16x4: e = launch_hsmm<16, 4, 64>(ha, st); break;
    case kHs8x8s64: e = launch_hsmm<8, 8, 64>(ha, st); break;
    case kHs8x16: e = launch_hsmm<8, 16, 64>(ha, st); break;
    default: e = launch_hsmm<4, 16, 128>(ha, st); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}
