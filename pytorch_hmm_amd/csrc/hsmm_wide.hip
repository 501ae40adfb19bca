// hmm355 — HSMM segment Viterbi for sizes beyond the register-slot kernels of hsmm.hip
// (S > 128, Dmax > 127, or S > 64 with Dmax > 63), up to S <= 1024 and Dmax <= 1024.
//
// Same recursion and the same exactness argument as hsmm.hip (reference hsmm.py:245-354; the
// C restatement oracle/hmm_oracle.c hsmm_viterbi_fast, proven equal to the literal 5-deep
// loop in tests/test_oracle.py):
//   M[st][s] = max_{s' != s} fl(dmax_{st-1}[s'] + logT[s'][s]),   dmax_{st-1}[s'] = max_d' delta,
//   delta(end e, s, d) = fl(fl(M[e-d+1][s] + obs_sum(e-d+1, d, s)) + dur[s][d-1])
//                        (start 0: fl(obs_sum + dur)),
// and the reference's first-candidate pointer (s' ascending, d' ascending, strict >) is
// re-resolved exactly where an earlier candidate rounds to the same total.  Instead of
// keeping every open segment in registers, this form keeps the (T, S) history of M in HBM
// and the segment sums obs_sum(t0, d, s) in a (T, S, Dmax) table (hsmm_wide_osum_kernel,
// torch-CPU's 4-accumulator order, O(1) per entry), so its limits are memory, not
// registers.  The pointers are not stored: the backtrace recomputes the candidate set of
// each segment it follows (S * Dmax values, one parallel pass per segment).
//
// Kernels: hsmm_wide_osum_kernel (one thread per (sequence, start, state)), then
// hsmm_wide_kernel (one 1024-thread workgroup per sequence: per start time two parallel
// phases and two barriers, then the segment walk).  Slower than the register-slot kernels
// (it exists for the sizes they cannot hold), but exact.
#include <stdint.h>
#include <stdlib.h>

#include "common.h"
#include "tsum.h"

namespace hmm355 {

constexpr int kHwSMax = 1024;
constexpr int kHwDMax = 1024;
constexpr int kHwNT = 1024;

struct HwArgs {
  const float* lp;    // (B,T,S)
  const float* dur;   // (S,Dm)
  const float* logT;  // (S,S)
  float* Mh;          // (B,T,S) M[st][s]
  float* os;          // (B,T,Dm,S) by END time: os[e][d-1][s] = obs_sum(e-d+1, d, s)
  float* scores;      // (B)
  int64_t* states;    // (B,T)
  int B, T, S, Dm;
  int tlds;           // 1: logT staged in LDS (behind the partial maxima) when it fits
};

// obs_sum(t0, d, s) for d = 1..Dm in torch-CPU's order (tsum.h; oracle torch_sum_f32): four
// strided lane sums over the whole quads with the cascade step every 16 quads (R_k, A_k), the
// tail (d mod 4 frames) into lane 0, then ((l0 + l1) + l2) + l3.  The quads are shared by every
// d, so each entry is O(1).
__global__ void __launch_bounds__(256) hsmm_wide_osum_kernel(HwArgs a) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)a.B * a.T * a.S;
  if (idx >= n) return;
  const int s = (int)(idx % a.S);
  const size_t bt = idx / a.S;
  const int t0 = (int)(bt % a.T);
  const int b = (int)(bt / a.T);
  const float* col = a.lp + ((size_t)b * a.T + t0) * a.S + s;  // frame t0 + i at col[i * S]
  // written by end time e = t0 + d - 1 (lanes over s: coalesced), where the recursion reads it
  float* out = a.os + (((size_t)b * a.T + t0) * a.Dm) * a.S + s;
  const size_t estep = (size_t)(a.Dm + 1) * a.S;  // (e + 1, d + 1) from (e, d)
  const int dlim = a.Dm < a.T - t0 ? a.Dm : a.T - t0;
  float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;  // R_k: lane sums since the last 16-quad block
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;  // A_k: the completed blocks (cascade level 1)
  float l0 = 0.f, l1 = 0.f, l2 = 0.f, l3 = 0.f;  // fl(R_k + A_k)
  for (int d = 1; d <= dlim; ++d) {
    const int m = d & ~3;
    if (m == d) {  // a new whole quad: frames d-4 .. d-1
      q0 += col[(size_t)(d - 4) * a.S];
      q1 += col[(size_t)(d - 3) * a.S];
      q2 += col[(size_t)(d - 2) * a.S];
      q3 += col[(size_t)(d - 1) * a.S];
      if ((d & (kTsumBlockElems - 1)) == 0) {
        c0 += q0; c1 += q1; c2 += q2; c3 += q3;
        q0 = q1 = q2 = q3 = 0.f;
      }
      l0 = q0 + c0; l1 = q1 + c1; l2 = q2 + c2; l3 = q3 + c3;
    }
    float a0 = l0;
    for (int i = m; i < d; ++i) a0 += col[(size_t)i * a.S];
    out[(size_t)(d - 1) * estep] = ((a0 + l1) + l2) + l3;
  }
}

// an L1-bypassing load (agent scope): M rows written earlier by other waves of this workgroup
__device__ __forceinline__ float ld_fresh(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// delta(end e, state s, duration d) from M (oracle DELTA_AT)
__device__ __forceinline__ float hw_delta(const HwArgs& a, int b, int e, int s, int d) {
  const int st = e - d + 1;
  if (st < 0) return -INFINITY;
  const float o = a.os[(((size_t)b * a.T + e) * a.Dm + (d - 1)) * a.S + s];
  const float u = a.dur[(size_t)s * a.Dm + (d - 1)];
  if (st == 0) return o + u;
  const float m = ld_fresh(a.Mh + ((size_t)b * a.T + st) * a.S + s);
  return m == -INFINITY ? -INFINITY : (m + o) + u;
}

// workgroup reductions over kHwNT threads (16 waves): max of a float; min of an int
__device__ __forceinline__ float wg_max(float v, float* red) {
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int k = 1; k < kHwNT / 64; ++k) r = fmaxf(r, red[k]);
  return r;
}
__device__ __forceinline__ int wg_min(int v, int* red) {
  for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  int r = red[0];
  for (int k = 1; k < kHwNT / 64; ++k) r = min(r, red[k]);
  return r;
}

__global__ void __launch_bounds__(kHwNT) hsmm_wide_kernel(HwArgs a) {
  __shared__ float dmax[kHwSMax];
  __shared__ float mpart[kHwNT];
  extern __shared__ float dpart[];  // [16][S] per-wave partial maxima, then logT (a.tlds)
  __shared__ float redf[kHwNT / 64];
  __shared__ int redi[kHwNT / 64];
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int T = a.T, S = a.S, Dm = a.Dm;
  float* Mrow = a.Mh + (size_t)b * T * S;
  // logT is read S * S times per start time: from LDS where it fits beside the partial maxima
  const float* lTs = a.logT;
  if (a.tlds) {
    float* t = dpart + (kHwNT / 64) * S;
    for (int k = tid; k < S * S; k += kHwNT) t[k] = a.logT[k];
    __syncthreads();
    lTs = t;
  }

  // ------------------------------------------------------------------ forward
  for (int st = 1; st < T; ++st) {
    // dmax[s'] = max_d' delta(st-1, s', d'): lanes over s' (coalesced rows of os and M), wave w
    // over d' = w+1, w+17, ...; the 16 waves' partial maxima combined through LDS
    for (int sp0 = 0; sp0 < S; sp0 += 64) {
      const int sp = sp0 + l;
      float m = -INFINITY;
      if (sp < S) {
#pragma unroll 4
        for (int dp = w + 1; dp <= Dm; dp += kHwNT / 64) m = fmaxf(m, hw_delta(a, b, st - 1, sp, dp));
        dpart[w * S + sp] = m;
      }
    }
    __syncthreads();
    for (int sp = tid; sp < S; sp += kHwNT) {
      float m = dpart[sp];
      for (int k = 1; k < kHwNT / 64; ++k) m = fmaxf(m, dpart[k * S + sp]);
      dmax[sp] = m;
    }
    __syncthreads();
    // M[st][s] = max_{s' != s} fl(dmax[s'] + logT[s'][s]) (exact in any order): P = 1024 / S
    // threads per state, each over every P-th s', then the P partial maxima
    const int P = kHwNT / S;
    if (tid < P * S) {
      const int s = tid % S, part = tid / S;
      float M = -INFINITY;
#pragma unroll 4
      for (int sp = part; sp < S; sp += P) {
        const float dm = dmax[sp];
        const float v = dm + lTs[(size_t)sp * S + s];
        M = (sp == s || dm == -INFINITY) ? M : fmaxf(M, v);
      }
      mpart[tid] = M;
    }
    __syncthreads();
    for (int s = tid; s < S; s += kHwNT) {
      float M = mpart[s];
      for (int part = 1; part < P; ++part) M = fmaxf(M, mpart[part * S + s]);
      Mrow[(size_t)st * S + s] = M;
    }
    // the M row is read by other waves (ld_fresh, from L2): the stores complete first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ------------------------------------------------------- final argmax (s, d ascending)
  // candidates enumerated as j = (d-1) * S + s (s fastest: coalesced rows of os and M); the
  // reference's order is k = s * Dm + d - 1 (s ascending, then d), kept for the first index
  const int nk = S * Dm;
  float bv = -INFINITY;
  for (int j = tid; j < nk; j += kHwNT) bv = fmaxf(bv, hw_delta(a, b, T - 1, j % S, j / S + 1));
  const float best = wg_max(bv, redf);
  int bk = 0x7fffffff;
  for (int j = tid; j < nk; j += kHwNT)
    if (hw_delta(a, b, T - 1, j % S, j / S + 1) == best) bk = min(bk, (j % S) * Dm + j / S);
  bk = wg_min(bk, redi);
  if (bk == 0x7fffffff) bk = 0;  // every score -inf: (s, d) = (0, 1) as the reference's init
  if (tid == 0) a.scores[b] = best;

  // --------------------------------------------------- segment walk (oracle hsmm_backtrack)
  int64_t* sts = a.states + (size_t)b * T;
  int t = T - 1, cs = bk / Dm, cd = bk % Dm + 1;
  for (int guard = 0; guard <= T && t >= 0; ++guard) {
    int start = t - cd + 1;
    if (start < 0) start = 0;
    for (int u = start + tid; u <= t; u += kHwNT) sts[u] = cs;
    if (start <= 0) break;
    // the pointer of segment (start, cs, cd): first candidate (s', d') whose total rounds to
    // the winning value F = fl(fl(M + od) + ud)
    const float M = ld_fresh(Mrow + (size_t)start * S + cs);
    int ns = 0, nd = 0;
    if (M != -INFINITY) {
      const float* lT = lTs + cs;
      // the reference's total of candidate k is g(x_k) = fl(fl(x_k + od) + ud), monotone in x_k,
      // and the winner's is F = g(M): the pointer is the first k with g(x_k) == F (the first
      // candidate attaining M, or an earlier one that rounds to the same total), one pass
      const float od = a.os[(((size_t)b * T + (start + cd - 1)) * Dm + (cd - 1)) * S + cs];
      const float ud = a.dur[(size_t)cs * Dm + (cd - 1)];
      const float F = (M + od) + ud;
      int win = 0x7fffffff;
      for (int j = tid; j < nk; j += kHwNT) {
        const int sp = j % S, dp = j / S + 1;
        const float pv = hw_delta(a, b, start - 1, sp, dp);
        const float x = (sp == cs || pv == -INFINITY) ? -INFINITY : pv + lT[(size_t)sp * S];
        if (x != -INFINITY && (x + od) + ud == F) win = min(win, sp * Dm + dp - 1);
      }
      win = wg_min(win, redi);
      if (win == 0x7fffffff) win = 0;  // (unreachable: the candidate attaining M qualifies)
      ns = win / Dm;
      nd = win % Dm + 1;
    }
    if (nd == 0) break;  // (no predecessor: frames below keep 0; the reference's walk would not terminate)
    t = start - 1;
    cs = ns;
    cd = nd;
    __syncthreads();
  }
}

size_t hsmm_wide_workspace_bytes(int B, int T, int S, int Dm) {
  const size_t n = (size_t)B * T * S;
  return align_up(n * 4, 256) + align_up(n * (size_t)Dm * 4, 256);
}

bool hsmm_wide_fits(int S, int Dm) { return S >= 1 && S <= kHwSMax && Dm >= 1 && Dm <= kHwDMax; }

hipError_t launch_hsmm_wide(const float* lp, const float* dur, const float* logT, int B, int T, int S, int Dm,
                            int64_t* states, float* scores, void* workspace, hipStream_t st) {
  const size_t n = (size_t)B * T * S;
  char* ws = static_cast<char*>(workspace);
  const size_t part = sizeof(float) * (kHwNT / 64) * S, tab = sizeof(float) * (size_t)S * S;
  const int tlds = part + tab + 16384 <= 163840 ? 1 : 0;  // (static LDS: dmax, mpart, reductions)
  HwArgs a{lp, dur, logT, reinterpret_cast<float*>(ws), reinterpret_cast<float*>(ws + align_up(n * 4, 256)),
           scores, states, B, T, S, Dm, tlds};
  // frames the walk never reaches keep the reference's torch.zeros value (hsmm.py:332)
  hipError_t e = hipMemsetAsync(states, 0, (size_t)B * T * sizeof(int64_t), st);
  if (e != hipSuccess) return e;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(hsmm_wide_osum_kernel, dim3(blocks), dim3(256), 0, st, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = part + (tlds ? tab : 0);
  e = allow_lds(hsmm_wide_kernel, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(hsmm_wide_kernel, dim3(B), dim3(kHwNT), lds, st, a);
  return hipGetLastError();
}

}  // namespace hmm355
