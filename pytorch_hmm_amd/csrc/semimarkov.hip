// hmm355 — explicit-duration (semi-Markov) HMM: segment Viterbi and segment forward on
// gfx950.  §8(f) row 3.
//
// Replaces SemiMarkovHMM.viterbi_decode (reference semi_markov.py:455-570) and the
// evidently intended SemiMarkovHMM._unsupervised_forward (semi_markov.py:308-383; the
// reference raises TypeError there).  The reference walks
// (t, s, d, s', d') in Python with one tensor op per candidate and recomputes every segment's
// observation score from the raw frames (semi_markov.py:411-435).
//
// Recursion over segment END times t (reference indexing):
//   delta[t][s][d], segment [st, t], st = t-d+1, d <= min(Dmax, t+1)
//     st == 0 : fl(fl(li[s] + o) + u)                                (semi_markov.py:497-507)
//     st >= 1 : M[st-1][s] == -inf ? -inf : fl(fl(M[st-1][s] + o) + u)   (:513-545)
//   o = seg_obs(st..t, s), u = dur[s][d-1], li = log initial probs.
//   M[tau][s] = max_{s' != s, d'} fl(delta[tau][s'][d'] + logT[s'][s])
//             = max_{s' != s} fl(Dm[tau][s'] + logT[s'][s]),  Dm[tau][s'] = max_{d'} delta
//   (fl(x + c) is monotone in x, so hoisting the max over d' is exact).  The literal strict->
//   argmax is the first (s' asc, d' asc) candidate whose rounded total equals M: s' is the
//   first s' whose fl(Dm + logT) equals M (stored per (tau, s)); d' is the first d' of that
//   s' whose fl(delta + logT) equals M — resolved exactly by the backtrace, which recomputes
//   delta[tau][s'][d'] bit-identically from the stored M and the quad table.
//
// Segment observation score (semi_markov.py:420-424):
//   gaussian : o = fl(cseg[s] - fl(0.5 * Q)),  cseg[s] = -0.5*sum(logvar_s) - 0.5*D*log(2 pi)
//              (host, the reference's torch expression), Q = sum over the segment's frames of
//              q[t][s] = sum_k fl(fl(diff*diff) / var[s][k]); the reference adds the constant
//              ONCE per segment, not per frame, and so does this kernel.
//   additive : o = Q with q = per-frame log-probabilities (observation_model='neural').
//   Q is accumulated left to right over the segment's frames (one running sum per
//   (start, state)); torch-CPU's reduction order for the same sums is ISA-dependent
//   (AVX2 vs AVX512 host), so Q and q agree with the reference to ~1 ulp of the sum, and the
//   oracle (oracle/hmm_oracle.c: smk_*) restates this kernel's order bit for bit.
//
// smk_quad_kernel   q (B,T,S), one thread per (frame, state), full-chip.
// smk_fwd_kernel    one 1024-thread workgroup per sequence: 16 lanes (one DPP row) per
//                   state, lane `sub` owns start-time slots k = sub+16j (mod 64, Dmax <= 63)
//                   and, in the predecessor phase, states s' = sub+16j.  A segment's running
//                   sum and predecessor score live in its slot's registers; ONE barrier per end
//                   time, for the only cross-wave value, Dm (double-buffered in LDS).
// smk_backtrace_kernel  one wave per sequence walks the segments back (semi_markov.py:548-568).
#include <stdlib.h>

#include "common.h"

#pragma clang fp contract(off)

namespace hmm355 {

constexpr int kSmS = 64;    // max states
constexpr int kSmR = 64;    // start-time ring (> Dmax)
constexpr int kSmL = 128;   // quad row ring (two 64-row chunks)
constexpr int kSmSub = 16;  // lanes per state
constexpr int kSmThreads = kSmS * kSmSub;  // 1024
constexpr int kSmNJ = 4;    // durations / predecessor states per lane

struct SmArgs {
  const float* q;      // (B,T,S)
  const float* cseg;   // (S) or null (additive mode)
  const float* li;     // (S)
  const float* logT;   // (S,S)
  const float* dur;    // (S,Dm)
  float* Mg;           // (B,T,S)  M (Viterbi) / L (forward): best / LSE predecessor score
  uint8_t* argS;       // (B,T,S)  first s' attaining M (Viterbi)
  int* fin;            // (B,2)    final (s, d)
  float* scores;       // (B)      best final score / total log-probability
  float* alpha;        // (B,T,S,Dm) or null: forward variables (forward mode)
  int64_t* seg_states; // (B,T)    segments, right-aligned (Viterbi)
  int64_t* seg_durs;   // (B,T)
  int* seg_count;      // (B)
  int B, T, S, Dm;
};

struct SmLds {
  float qr[kSmL][kSmS];          // quad rows (two 64-row chunks)
  float dur[kSmS][kSmR + 1];     // duration table, d-1 major per state (+1: bank spread)
  float dmx[2][kSmS];            // Dm / A of the current end time (double-buffered)
};

__device__ __forceinline__ float sm_row_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  return fmaxf(v, dpp_f<0x128>(v));
}
__device__ __forceinline__ int sm_row_min_i(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x124>(v));
  return min(v, dpp_i<0x128>(v));
}

__device__ __forceinline__ float sm_seg_obs(float cs, float Q, bool gaussian) {
  return gaussian ? cs - 0.5f * Q : Q;
}

// ---------------------------------------------------------------- per-frame quad table
// q[f][s] = sum_k fl(fl((x[f][k] - mu[s][k])^2) / var[s][k]), k ascending.  muT/varT are
// (Df, S) so a wave's 64 states read one coalesced row per k.
__global__ void __launch_bounds__(256) smk_quad_kernel(const float* __restrict__ x, const float* __restrict__ muT,
                                                       const float* __restrict__ varT, int F, int Df, int S,
                                                       float* __restrict__ q) {
  const int s = (threadIdx.x & 63) + 64 * blockIdx.y;
  const long long f = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= F || s >= S) return;
  const float* xf = x + f * Df;
  float acc = 0.f;
  for (int k = 0; k < Df; ++k) {
    const float d = xf[k] - muT[(size_t)k * S + s];
    acc = acc + (d * d) / varT[(size_t)k * S + s];
  }
  q[f * S + s] = acc;
}

// ------------------------------------------------------------- segment recursion (fwd)
// Lane (s, sub) owns the start-time slots k = sub + 16j (j < 4) of state s: the segment that
// started at the latest st == k (mod 64).  Its running sum Q(st..t) and its predecessor score
// M[st-1][s] stay in registers for the segment's whole life (d = t - st + 1 <= Dmax < 64, so
// a slot is free again when its start time comes round).  Per end time the only LDS traffic
// is one quad broadcast, one duration-table read and the cross-wave Dm exchange.
template <bool kViterbi>
__global__ void __launch_bounds__(kSmThreads) smk_fwd_kernel(SmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SmLds& L = *reinterpret_cast<SmLds*>(smem);
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const int s = tid >> 4, sub = tid & 15;
  const bool live = s < S;
  const bool gaussian = a.cseg != nullptr;
  const float* q = a.q + (size_t)b * T * S;

  for (int i = tid; i < kSmS * kSmR; i += kSmThreads) {
    const int r = i / kSmR, d = i % kSmR;
    L.dur[r][d] = (r < S && d < Dm) ? a.dur[(size_t)r * Dm + d] : -INFINITY;
  }
  // predecessor phase: lane owns s' = sub + 16j; log T[s'][s] in registers (-inf: excluded)
  float lt[kSmNJ];
#pragma unroll
  for (int j = 0; j < kSmNJ; ++j) {
    const int sp = sub + kSmSub * j;
    const bool ok = live && sp < S && sp != s;
    const float v = a.logT[ok ? (size_t)sp * S + s : 0];
    lt[j] = ok ? v : -INFINITY;
  }
  const float cs = (live && gaussian) ? a.cseg[s] : 0.f;
  const float lis = live ? a.li[s] : 0.f;

  // quad rows stream through a 2-chunk LDS ring, one chunk (64 rows) ahead
  constexpr int PER = kSmS * 64 / kSmThreads;  // 4 values per thread per chunk
  float rc[PER];
  auto chunk_load = [&](int c) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int idx = tid + k * kSmThreads;
      const int row = c * 64 + idx / kSmS, col = idx % kSmS;
      const bool ok = row < T && col < S;
      const float v = q[ok ? (size_t)row * S + col : 0];
      rc[k] = ok ? v : 0.f;
    }
  };
  auto chunk_store = [&](int c) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int idx = tid + k * kSmThreads;
      L.qr[(c * 64 + idx / kSmS) % kSmL][idx % kSmS] = rc[k];
    }
  };
  chunk_load(0);
  chunk_store(0);
  if (T > 64) chunk_load(1);
  __syncthreads();

  float* alpha = a.alpha ? a.alpha + (size_t)b * T * S * Dm : nullptr;
  float acc[kSmNJ], mp[kSmNJ];
#pragma unroll
  for (int j = 0; j < kSmNJ; ++j) { acc[j] = 0.f; mp[j] = -INFINITY; }
  float Mlast = -INFINITY;  // M[t-1][s] (every lane of the row holds it)

  // one end time (returns false after the last); the loop below runs it four times per
  // iteration so the compiler can schedule across consecutive end times
  auto end_step = [&](const int t) -> bool {
    // ---- A: every segment ending at t, for this lane's start slots
    const float qt = live ? L.qr[t % kSmL][s] : 0.f;
    float v[kSmNJ];
    int dd[kSmNJ];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kSmNJ; ++j) {
      const int age = (t - (sub + kSmSub * j)) & (kSmR - 1);
      const int d = age + 1, st = t - age;
      dd[j] = d;
      const bool fresh = age == 0;
      acc[j] = fresh ? qt : acc[j] + qt;
      mp[j] = fresh ? Mlast : mp[j];
      v[j] = -INFINITY;
      if (live && d <= Dm && st >= 0) {
        const float o = sm_seg_obs(cs, acc[j], gaussian);
        const float u = L.dur[s][d - 1];
        if (st == 0) v[j] = (lis + o) + u;
        else v[j] = (mp[j] == -INFINITY) ? -INFINITY : (mp[j] + o) + u;
      }
      mx = fmaxf(mx, v[j]);
    }
    mx = sm_row_max(mx);
    float red = mx;  // Viterbi: Dm[t][s]; forward: A[t][s] = LSE_d
    if constexpr (!kViterbi) {
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < kSmNJ; ++j) se += (v[j] == -INFINITY) ? 0.f : __expf(v[j] - mx);
      se = row16_sum(se);
      red = (mx == -INFINITY) ? -INFINITY : mx + __logf(se);
      if (alpha && live) {
        float* ar = alpha + ((size_t)t * S + s) * Dm;
#pragma unroll
        for (int j = 0; j < kSmNJ; ++j)
          if (dd[j] <= Dm) ar[dd[j] - 1] = v[j];
      }
    }
    if (live && sub == 0) L.dmx[t & 1][s] = red;
    if (t == T - 1) {
      // final: Viterbi — first (s asc, d asc) with the max (semi_markov.py:548-556);
      // forward — LSE over (s, d) (semi_markov.py:373-381)
      __shared__ int fd[kSmS];
      if constexpr (kViterbi) {
        int ld = 0x7fff;
#pragma unroll
        for (int j = 0; j < kSmNJ; ++j)
          if (v[j] == mx && dd[j] < ld) ld = dd[j];
        ld = sm_row_min_i(ld);
        if (live && sub == 0) fd[s] = ld;
      }
      __syncthreads();
      if (tid < 64) {
        float bv = tid < S ? L.dmx[t & 1][tid] : -INFINITY;
        int bi = tid < S ? tid : 0x7fffffff;
        if constexpr (kViterbi) {
          wave_argmax(bv, bi);
          if (tid == 0) {
            a.scores[b] = bv;
            // all -inf: the reference keeps its defaults (state 0, duration 1)
            const bool any = bv != -INFINITY;
            a.fin[2 * b] = any ? bi : 0;
            a.fin[2 * b + 1] = any ? fd[bi] : 1;
          }
        } else {
          const float m = wave_max(bv);
          float e = (tid < S && bv != -INFINITY) ? __expf(bv - m) : 0.f;
          e = wave_sum(e);
          if (tid == 0) a.scores[b] = (m == -INFINITY) ? -INFINITY : m + __logf(e);
        }
      }
      return false;
    }
    step_barrier();
    // ---- C: best (or LSE) predecessor score for segments starting at t+1
    {
      float c[kSmNJ];
      float lm = -INFINITY;
      int ls = 0x7fff;
#pragma unroll
      for (int j = 0; j < kSmNJ; ++j) {
        const int sp = sub + kSmSub * j;
        const float dm = L.dmx[t & 1][sp < S ? sp : 0];
        c[j] = (lt[j] == -INFINITY || dm == -INFINITY) ? -INFINITY : dm + lt[j];
        if (c[j] > lm) { lm = c[j]; ls = sp; }
      }
      const float M = sm_row_max(lm);
      float out = M;
      if constexpr (kViterbi) {
        const int s1 = sm_row_min_i((lm == M && M != -INFINITY) ? ls : 0x7fff);
        if (live && sub == 0) a.argS[((size_t)b * T + t) * S + s] = (uint8_t)(M == -INFINITY ? 0 : s1);
      } else {
        float se = 0.f;
#pragma unroll
        for (int j = 0; j < kSmNJ; ++j) se += (c[j] == -INFINITY) ? 0.f : __expf(c[j] - M);
        se = row16_sum(se);
        out = (M == -INFINITY) ? -INFINITY : M + __logf(se);
      }
      Mlast = out;
      if (live && sub == 0) a.Mg[((size_t)b * T + t) * S + s] = out;
    }
    if ((t + 2) % 64 == 0) {  // rows of chunk c = (t+2)/64 are first read at step t+2
      const int cidx = (t + 2) >> 6;
      chunk_store(cidx);
      if ((cidx + 1) * 64 < T) chunk_load(cidx + 1);
      __syncthreads();
    }
    return true;
  };
  for (int t = 0; t < T; t += 4) {
    if (!end_step(t)) break;
    if (!end_step(t + 1)) break;
    if (!end_step(t + 2)) break;
    if (!end_step(t + 3)) break;
  }
}

__global__ void __launch_bounds__(64) smk_backtrace_kernel(SmArgs a) {
  __shared__ float col[kSmR];  // q[tau - i][s1], i < Dm: the predecessor's candidate column
  const int b = blockIdx.x, l = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const float* q = a.q + (size_t)b * T * S;
  const float* Mb = a.Mg + (size_t)b * T * S;
  int t = T - 1, cs = a.fin[2 * b], cd = a.fin[2 * b + 1];
  int k = 0;
  while (t >= 0) {
    if (l == 0) {
      a.seg_states[(size_t)b * T + (T - 1 - k)] = cs;
      a.seg_durs[(size_t)b * T + (T - 1 - k)] = cd;
    }
    ++k;
    const int tau = t - cd;
    if (tau < 0) break;
    const size_t gi = (size_t)tau * S + cs;
    const float M = Mb[gi];
    int ns = 0, nd = 1;  // the reference's defaults when no predecessor exists
    if (M != -INFINITY) {
      ns = a.argS[(size_t)b * T * S + gi];
      const float lt = a.logT[(size_t)ns * S + cs];
      const int dlim = Dm < tau + 1 ? Dm : tau + 1;
      // one round trip: the candidate column and the candidates' predecessor scores
      const bool pin = l < dlim;
      const int st = tau - l;  // candidate d' = l + 1 starts at tau - l
      const float qv = q[(size_t)(pin ? st : 0) * S + ns];
      const float pm = (pin && st >= 1) ? Mb[(size_t)(st - 1) * S + ns] : 0.f;
      if (pin) col[l] = qv;
      __syncthreads();
      bool hit = false;
      if (pin) {
        // delta[tau][s1][d'] exactly as smk_fwd_kernel forms it: Q left to right from st
        float Q = col[l];
        for (int e = l - 1; e >= 0; --e) Q = Q + col[e];
        const float o = sm_seg_obs(a.cseg ? a.cseg[ns] : 0.f, Q, a.cseg != nullptr);
        const float u = a.dur[(size_t)ns * Dm + l];
        const float dv = st == 0 ? (a.li[ns] + o) + u : (pm == -INFINITY ? -INFINITY : (pm + o) + u);
        hit = dv != -INFINITY && (dv + lt) == M;
      }
      const unsigned long long mask = __ballot(hit);
      nd = mask ? __ffsll((long long)mask) : 1;  // lane index + 1 = d' (always found when M is finite)
      __syncthreads();  // the column is restaged for the next segment
    }
    t = tau;
    cs = ns;
    cd = nd;
  }
  if (l == 0) a.seg_count[b] = k;
}

// ---------------------------------------------------------------- the general form
// For S > 64 or Dmax > 63 (up to S, Dmax <= 1024), where the open segments no longer fit the
// register slots of smk_fwd_kernel: the same recursion and the same fp32 operations in the same
// order, with the segment scores and the predecessor history in the workspace instead of
// registers (the design of hsmm_wide.hip).
//   smk_wide_osum_kernel  o(st, d, s) = seg_obs(Q), Q = q[st] + ... + q[st+d-1] left to right
//                         (the running sum smk_fwd_kernel keeps per slot, so the same bits),
//                         one thread per (sequence, start, state), stored by END time
//                         os[e][d-1][s] so the recursion reads coalesced rows over states.
//   smk_wide_kernel       one 1024-thread workgroup per sequence; per end time t: phase 1,
//                         Dm[t][s'] = max_d delta(t, s', d) (forward: LSE_d, and log alpha),
//                         lanes over s', waves over d, partials through LDS; phase 2,
//                         M[t][s] = max_{s' != s} fl(Dm[t][s'] + logT[s'][s]) (forward: LSE),
//                         1024 / S threads per state (or states in turn).  Viterbi then walks
//                         the segments in the same workgroup: each step's pointer is the first
//                         candidate (s' ascending, d' ascending) whose fl(delta + logT) equals
//                         M (semi_markov.py:513-530's strict >), found by one parallel pass over
//                         the S * Dmax candidates instead of a stored argS.
// Forward LSE sums run in another order than smk_fwd_kernel's (checked against float64, not bit
// for bit); the Viterbi path and scores are bit-identical to the register form and to the
// literal loop (tests/test_gpu_semimarkov.py).
constexpr int kSwS = 1024;
constexpr int kSwD = 1024;
constexpr int kSwNT = 1024;

struct SwArgs {
  const float* q;      // (B,T,S)
  const float* cseg;   // (S) or null
  const float* li;     // (S)
  const float* logT;   // (S,S)
  const float* dur;    // (S,Dm)
  float* Mg;           // (B,T,S) M[tau][s] (forward: L), for segments starting at tau + 1
  float* os;           // (B,T,Dm,S) by end time
  float* scores;       // (B)
  float* alpha;        // (B,T,S,Dm) or null (forward)
  int64_t* seg_states; // (B,T)
  int64_t* seg_durs;   // (B,T)
  int* seg_count;      // (B)
  int B, T, S, Dm;
};

__global__ void __launch_bounds__(256) smk_wide_osum_kernel(SwArgs a) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)a.B * a.T * a.S;
  if (idx >= n) return;
  const int s = (int)(idx % a.S);
  const size_t bt = idx / a.S;
  const int st = (int)(bt % a.T);
  const int b = (int)(bt / a.T);
  const bool gaussian = a.cseg != nullptr;
  const float cs = gaussian ? a.cseg[s] : 0.f;
  const float* col = a.q + ((size_t)b * a.T + st) * a.S + s;
  float* out = a.os + (((size_t)b * a.T + st) * a.Dm) * a.S + s;
  const size_t estep = (size_t)(a.Dm + 1) * a.S;  // (e + 1, d + 1) from (e, d)
  const int dlim = a.Dm < a.T - st ? a.Dm : a.T - st;
  float acc = 0.f;
  for (int d = 1; d <= dlim; ++d) {
    acc = d == 1 ? col[0] : acc + col[(size_t)(d - 1) * a.S];
    out[(size_t)(d - 1) * estep] = sm_seg_obs(cs, acc, gaussian);
  }
}

__device__ __forceinline__ float sw_fresh(const float* p) {  // M rows other waves wrote (L1 bypass)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// delta(end t, state s, duration d) exactly as smk_fwd_kernel forms it
__device__ __forceinline__ float sw_delta(const SwArgs& a, int b, int t, int s, int d) {
  const int st = t - d + 1;
  if (st < 0) return -INFINITY;
  const float o = a.os[(((size_t)b * a.T + t) * a.Dm + (d - 1)) * a.S + s];
  const float u = a.dur[(size_t)s * a.Dm + (d - 1)];
  if (st == 0) return (a.li[s] + o) + u;
  const float m = sw_fresh(a.Mg + ((size_t)b * a.T + (st - 1)) * a.S + s);
  return m == -INFINITY ? -INFINITY : (m + o) + u;
}

// workgroup reductions over kSwNT threads: max of a float; min of an int
__device__ __forceinline__ float wg_max_sw(float v, float* red) {
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
  for (int k = 1; k < kSwNT / 64; ++k) r = fmaxf(r, red[k]);
  return r;
}
__device__ __forceinline__ int wg_min_sw(int v, int* red) {
  for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = red[0];
  for (int k = 1; k < kSwNT / 64; ++k) r = min(r, red[k]);
  return r;
}

// (max, sum of exp(x - max)) pairs: the online log-sum-exp merge
__device__ __forceinline__ void lse_merge(float& m, float& z, float m2, float z2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; z = z2; return; }
  if (m2 > m) { z = z * __expf(m - m2) + z2; m = m2; }
  else z = z + z2 * __expf(m2 - m);
}

template <bool kViterbi>
__global__ void __launch_bounds__(kSwNT) smk_wide_kernel(SwArgs a) {
  __shared__ float dm[kSwS];     // Dm[t][s'] (forward: A[t][s'])
  __shared__ float pm[kSwNT];    // phase-2 partials (max)
  __shared__ float pz[kSwNT];    //                  (forward: sum)
  __shared__ float redf[kSwNT / 64];
  __shared__ int redi[kSwNT / 64];
  extern __shared__ float part[];  // [16][S] phase-1 partial maxima, then [16][S] sums (forward)
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int T = a.T, S = a.S, Dm = a.Dm;
  constexpr int NWv = kSwNT / 64;
  float* Mrow = a.Mg + (size_t)b * T * S;
  float* alpha = a.alpha ? a.alpha + (size_t)b * T * S * Dm : nullptr;
  for (int t = 0; t < T; ++t) {
    // ---- phase 1: lanes over s', waves over d
    for (int s0 = 0; s0 < S; s0 += 64) {
      const int sp = s0 + l;
      if (sp < S) {
        float m = -INFINITY, z = 0.f;
        for (int d = w + 1; d <= Dm; d += NWv) {
          const float v = sw_delta(a, b, t, sp, d);
          if (alpha) alpha[((size_t)t * S + sp) * Dm + d - 1] = v;
          if (kViterbi) m = fmaxf(m, v);
          else lse_merge(m, z, v, 1.f);
        }
        part[w * S + sp] = m;
        if (!kViterbi) part[(NWv + w) * S + sp] = z;
      }
    }
    __syncthreads();
    for (int sp = tid; sp < S; sp += kSwNT) {
      float m = part[sp], z = kViterbi ? 0.f : part[NWv * S + sp];
      for (int k = 1; k < NWv; ++k) {
        if (kViterbi) m = fmaxf(m, part[k * S + sp]);
        else lse_merge(m, z, part[k * S + sp], part[(NWv + k) * S + sp]);
      }
      dm[sp] = kViterbi ? m : (m == -INFINITY ? -INFINITY : m + __logf(z));
    }
    __syncthreads();
    if (t == T - 1) break;
    // ---- phase 2: M[t][s] over s' != s (P threads per state, or states in turn)
    const int P = S <= kSwNT ? kSwNT / S : 1;
    for (int s0 = 0; s0 < S; s0 += kSwNT / P) {
      const int s = s0 + tid / P, pt = tid % P;
      float m = -INFINITY, z = 0.f;
      if (s < S) {
        for (int sp = pt; sp < S; sp += P) {
          const float lt = a.logT[(size_t)sp * S + s];
          const float dv = dm[sp];
          const float c = (sp == s || lt == -INFINITY || dv == -INFINITY) ? -INFINITY : dv + lt;
          if (kViterbi) m = fmaxf(m, c);
          else lse_merge(m, z, c, 1.f);
        }
      }
      pm[tid] = m;
      pz[tid] = z;
      __syncthreads();
      if (s < S && pt == 0) {
        for (int k = 1; k < P; ++k) {
          if (kViterbi) m = fmaxf(m, pm[tid + k]);
          else lse_merge(m, z, pm[tid + k], pz[tid + k]);
        }
        Mrow[(size_t)t * S + s] = kViterbi ? m : (m == -INFINITY ? -INFINITY : m + __logf(z));
      }
      __syncthreads();
    }
    // the M row is read by other waves (sw_fresh, from L2): the stores complete first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // ---- final (dm holds row T-1)
  if constexpr (!kViterbi) {
    float m = -INFINITY, z = 0.f;
    for (int s = tid; s < S; s += kSwNT) lse_merge(m, z, dm[s], 1.f);
    for (int off = 32; off >= 1; off >>= 1) {
      const float m2 = __shfl_xor(m, off), z2 = __shfl_xor(z, off);
      lse_merge(m, z, m2, z2);
    }
    if (l == 0) { pm[w] = m; pz[w] = z; }
    __syncthreads();
    if (tid == 0) {
      for (int k = 1; k < NWv; ++k) lse_merge(m, z, pm[k], pz[k]);
      a.scores[b] = m == -INFINITY ? -INFINITY : m + __logf(z);
    }
    return;
  } else {
    // first (s ascending, d ascending) with the best delta (semi_markov.py:548-556)
    float bv = -INFINITY;
    for (int s = tid; s < S; s += kSwNT) bv = fmaxf(bv, dm[s]);
    const float best = wg_max_sw(bv, redf);
    const int nk = S * Dm;
    int bk = 0x7fffffff;
    if (best != -INFINITY)
      for (int j = tid; j < nk; j += kSwNT) {
        const int s = j % S, d = j / S + 1;
        if (sw_delta(a, b, T - 1, s, d) == best) bk = min(bk, s * Dm + d - 1);
      }
    bk = wg_min_sw(bk, redi);
    int cs = 0, cd = 1;  // every score -inf: the reference's defaults
    if (bk != 0x7fffffff) { cs = bk / Dm; cd = bk % Dm + 1; }
    if (tid == 0) a.scores[b] = best;
    // ---- segment walk (semi_markov.py:558-568), right-aligned output as smk_backtrace_kernel
    int t = T - 1, k = 0;
    while (t >= 0) {
      if (tid == 0) {
        a.seg_states[(size_t)b * T + (T - 1 - k)] = cs;
        a.seg_durs[(size_t)b * T + (T - 1 - k)] = cd;
      }
      ++k;
      const int tau = t - cd;
      if (tau < 0) break;
      const float M = sw_fresh(Mrow + (size_t)tau * S + cs);
      int ns = 0, nd = 1;
      if (M != -INFINITY) {
        const int dlim = Dm < tau + 1 ? Dm : tau + 1;
        int win = 0x7fffffff;
        for (int j = tid; j < S * dlim; j += kSwNT) {
          const int sp = j % S, dp = j / S + 1;
          if (sp == cs) continue;
          const float lt = a.logT[(size_t)sp * S + cs];
          const float dv = sw_delta(a, b, tau, sp, dp);
          if (lt != -INFINITY && dv != -INFINITY && dv + lt == M) win = min(win, sp * Dm + dp - 1);
        }
        win = wg_min_sw(win, redi);
        if (win != 0x7fffffff) { ns = win / Dm; nd = win % Dm + 1; }
      }
      t = tau;
      cs = ns;
      cd = nd;
      __syncthreads();
    }
    if (tid == 0) a.seg_count[b] = k;
  }
}

}  // namespace hmm355

using namespace hmm355;

// the register form holds S <= 64, Dmax <= 63; the general form the rest (HMM355_FORM_GENERAL
// forces it, for tests and comparison)
static bool smk_wide(int S, int Dmax, unsigned flags) {
  return (S > kSmS || Dmax >= kSmR) || (flags & HMM355_FORM_GENERAL);
}

HMM355_API size_t hmm355_semimarkov_workspace_bytes_ex(int B, int T, int S, int Dmax, unsigned flags) {
  if (B < 0 || T < 1 || S < 1 || S > kSwS || Dmax < 1 || Dmax > kSwD) return 0;
  const size_t n = (size_t)B * T * S;
  if (smk_wide(S, Dmax, flags)) return align_up(n * 4, 256) + align_up(n * (size_t)Dmax * 4, 256);
  return align_up(n * 4, 256) + align_up(n * 4, 256) + align_up(n, 256) + align_up((size_t)B * 8, 256);
}

HMM355_API size_t hmm355_semimarkov_workspace_bytes(int B, int T, int S, int Dmax) {
  return hmm355_semimarkov_workspace_bytes_ex(B, T, S, Dmax, 0u);
}

static int smk_check(int B, int T, int S, int Dmax) {
  if (B < 0 || S < 0 || Dmax < 0) return HMM355_E_ARG;
  if (S < 1 || S > kSwS) return HMM355_E_STATES;
  if (Dmax < 1 || Dmax > kSwD) return HMM355_E_DURATION;
  if (T < 1) return HMM355_E_SHAPE;
  return HMM355_OK;
}

HMM355_API int hmm355_semimarkov_quad_f32(const float* x, const float* means_t, const float* vars_t, int B, int T,
                                          int Df, int S, float* quad, void* stream) {
  if (B < 0 || T < 0 || Df < 1) return HMM355_E_ARG;
  if (S < 1 || S > kSwS) return HMM355_E_STATES;
  const long long F = (long long)B * T;
  if (F == 0) return HMM355_OK;
  if (!x || !means_t || !vars_t || !quad) return HMM355_E_ARG;
  hipLaunchKernelGGL(smk_quad_kernel, dim3((unsigned)((F + 3) / 4), (unsigned)((S + 63) / 64)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), x, means_t, vars_t, (int)F, Df, S, quad);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}

static int smk_run(bool viterbi, const float* quad, const float* seg_const, const float* log_init,
                   const float* log_T, const float* dur_lp, int B, int T, int S, int Dmax, int64_t* seg_states,
                   int64_t* seg_durs, int* seg_count, float* alpha, float* scores, unsigned flags,
                   void* workspace, size_t workspace_bytes, void* stream) {
  if (flags & ~HMM355_FORM_GENERAL) return HMM355_E_ARG;
  int rc = smk_check(B, T, S, Dmax);
  if (rc != HMM355_OK) return rc;
  if (B == 0) return HMM355_OK;
  if (!quad || !log_init || !log_T || !dur_lp || !scores || !workspace) return HMM355_E_ARG;
  if (viterbi && (!seg_states || !seg_durs || !seg_count)) return HMM355_E_ARG;
  if (workspace_bytes < hmm355_semimarkov_workspace_bytes_ex(B, T, S, Dmax, flags)) return HMM355_E_WORKSPACE;
  const size_t n = (size_t)B * T * S;
  char* ws = static_cast<char*>(workspace);
  if (smk_wide(S, Dmax, flags)) {
    SwArgs wa{quad, seg_const, log_init, log_T, dur_lp, reinterpret_cast<float*>(ws),
              reinterpret_cast<float*>(ws + align_up(n * 4, 256)), scores, alpha, seg_states, seg_durs, seg_count,
              B, T, S, Dmax};
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(smk_wide_osum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wa);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    const size_t lds = (viterbi ? 1 : 2) * (kSwNT / 64) * (size_t)S * sizeof(float);
    if (viterbi) {
      if ((e = allow_lds(smk_wide_kernel<true>, lds)) != hipSuccess) return (int)e;
      hipLaunchKernelGGL(smk_wide_kernel<true>, dim3(B), dim3(kSwNT), lds, st, wa);
    } else {
      if ((e = allow_lds(smk_wide_kernel<false>, lds)) != hipSuccess) return (int)e;
      hipLaunchKernelGGL(smk_wide_kernel<false>, dim3(B), dim3(kSwNT), lds, st, wa);
    }
    e = hipGetLastError();
    return e == hipSuccess ? HMM355_OK : (int)e;
  }
  float* Mg = reinterpret_cast<float*>(ws);
  uint8_t* argS = reinterpret_cast<uint8_t*>(ws + 2 * align_up(n * 4, 256));
  int* fin = reinterpret_cast<int*>(ws + 2 * align_up(n * 4, 256) + align_up(n, 256));
  SmArgs sa{quad, seg_const, log_init, log_T, dur_lp, Mg, argS, fin, scores, alpha,
            seg_states, seg_durs, seg_count, B, T, S, Dmax};
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (viterbi) {
    e = allow_lds(smk_fwd_kernel<true>, sizeof(SmLds));
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(smk_fwd_kernel<true>, dim3(B), dim3(kSmThreads), sizeof(SmLds), st, sa);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(smk_backtrace_kernel, dim3(B), dim3(64), 0, st, sa);
  } else {
    e = allow_lds(smk_fwd_kernel<false>, sizeof(SmLds));
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(smk_fwd_kernel<false>, dim3(B), dim3(kSmThreads), sizeof(SmLds), st, sa);
  }
  e = hipGetLastError();
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_semimarkov_viterbi_ex_f32(const float* quad, const float* seg_const, const float* log_init,
                                                const float* log_T, const float* dur_lp, int B, int T, int S,
                                                int Dmax, unsigned flags, int64_t* seg_states, int64_t* seg_durs,
                                                int* seg_count, float* scores, void* workspace,
                                                size_t workspace_bytes, void* stream) {
  return smk_run(true, quad, seg_const, log_init, log_T, dur_lp, B, T, S, Dmax, seg_states, seg_durs, seg_count,
                 nullptr, scores, flags, workspace, workspace_bytes, stream);
}

HMM355_API int hmm355_semimarkov_forward_ex_f32(const float* quad, const float* seg_const, const float* log_init,
                                                const float* log_T, const float* dur_lp, int B, int T, int S,
                                                int Dmax, unsigned flags, float* log_alpha, float* log_prob,
                                                void* workspace, size_t workspace_bytes, void* stream) {
  return smk_run(false, quad, seg_const, log_init, log_T, dur_lp, B, T, S, Dmax, nullptr, nullptr, nullptr,
                 log_alpha, log_prob, flags, workspace, workspace_bytes, stream);
}

HMM355_API int hmm355_semimarkov_viterbi_f32(const float* quad, const float* seg_const, const float* log_init,
                                             const float* log_T, const float* dur_lp, int B, int T, int S, int Dmax,
                                             int64_t* seg_states, int64_t* seg_durs, int* seg_count, float* scores,
                                             void* workspace, size_t workspace_bytes, void* stream) {
  return hmm355_semimarkov_viterbi_ex_f32(quad, seg_const, log_init, log_T, dur_lp, B, T, S, Dmax, 0u, seg_states,
                                          seg_durs, seg_count, scores, workspace, workspace_bytes, stream);
}

HMM355_API int hmm355_semimarkov_forward_f32(const float* quad, const float* seg_const, const float* log_init,
                                             const float* log_T, const float* dur_lp, int B, int T, int S, int Dmax,
                                             float* log_alpha, float* log_prob, void* workspace,
                                             size_t workspace_bytes, void* stream) {
  return hmm355_semimarkov_forward_ex_f32(quad, seg_const, log_init, log_T, dur_lp, B, T, S, Dmax, 0u, log_alpha,
                                          log_prob, workspace, workspace_bytes, stream);
}
