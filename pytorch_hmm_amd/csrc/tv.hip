// hmm355 — recursions with one transition matrix per time step (NeuralHMM) on gfx950.
//
// Replaces NeuralHMM._forward_algorithm / _backward_algorithm / the posterior epilogue
// (reference neural.py:391-461) and NeuralHMM.viterbi_decode (neural.py:463-511).  The
// reference feeds log_transition_probs of shape (B,T,N,N) from its transition network
// (neural.py:377-381); forward step t uses matrix t-1 (neural.py:419-427), backward step t
// matrix t (:449-458), Viterbi step t matrix t-1 (:489-496).  Without a transition network
// one matrix is expanded over (B,T) (:383-385): strides sb = st = 0 here.
//
// Per (sequence, step) the recursion consumes N^2 fresh matrix entries (64 KiB at N = 128)
// read once from HBM, so this path is bound by the bytes a chain's CU can pull and by the
// N^2 exponentials, not by the serial latency that bounds the time-invariant path.
//
// HBM layout: the caller's matrices, element (b,k,i,j) at lA[b*sb + k*st + i*N + j].
// FB workspace: U | V (B,T,NP) | LA | LB (B,T) | E (B,T,NP) | M | CA | CB (B,T).
//
// tv_fb<NP>: one 512-thread workgroup (8 waves, two per SIMD) per (sequence, direction),
//   owning its CU.  Each wave streams a fixed slice of every step's matrix with PD steps of
//   float4 loads in flight (PD x 64 KiB per CU at N = 128), 128-B row segments per load
//   instruction on the backward slice and 64-B segments on the forward slice:
//   - alpha: wave w holds columns [NP/8 w, +NP/8) of every row; lane (q = l % QW,
//     r = l / QW) the column quad q of rows r + RL k.  u_t[j] = sum_i u_{t-1}[i] exp(lA[i][j])
//     is a lane-local FMA chain and a reduction over the RL row lanes (transposed through
//     v_permlane32/16_swap, then DPP row_ror), so a column never leaves its wave.
//   - beta: wave w holds rows [NP/8 w, +NP/8) of every column; lane (qq = l & 7, r = l >> 3)
//     the quads qq + 8m of rows r + 8k.  v_t[i] = sum_j exp(lA[i][j]) w_{t+1}[j] reduces over
//     the 8 quad lanes of a row (DPP quad_perm / row_half_mirror).
//   The Rabiner normaliser of the previous vector is formed in every wave (each wave reads
//   all of it), so a step has ONE s_barrier: publish the new vector to LDS, barrier, read it.
//   Scales: u_t = (u_{t-1} A_t) * E_t / c_{t-1} with E_t = exp(lo_t - M_t), M_t the row max
//   of the log-emission, so log alpha_t = log u_t + LA_t, LA_t = LA_{t-1} + log c_{t-1} + M_t;
//   beta likewise.  The normalisers go to CA / CB and one wave per sequence scans them
//   (tv_scan) in fp64; the posterior epilogue is post.h's.
// tv_vit<NP>: the alpha layout in max-plus with the first-index argmax kept in the chain
//   (the matrix is read once, so the argmax cannot be recomputed off-chain for free as
//   viterbi.hip does), psi rows to the workspace, then post.h's chunk maps and backtrace.
//   delta_t[j] = fl(max_i fl(delta_{t-1}[i] + lA[i][j]) + lo_t[j]): the reference's sums
//   (neural.py:494-497), so delta and the states are bit-identical to it.
#include "post.h"

namespace hmm355 {

template <int NP>
struct TvGeo {
  static constexpr int NT = 512;           // 8 waves
  // alpha / Viterbi: wave w = (column block cb = w % CB, row part p = w / CB) holds 32 columns
  // of RPP rows; lane (q = l & 7, r = l >> 3) the column quad q of rows p*RPP + r + 8k, k < KA,
  // so every load instruction reads 8 whole 128-B row segments
  static constexpr int CB = NP / 32;
  static constexpr int RH = 8 / CB;        // row parts: partial results the readers combine
  static constexpr int RPP = NP / RH;
  static constexpr int KA = RPP / 8;
  // beta: wave w holds rows [NP/8 w, +NP/8) of every column; lane (qq = l & 7, r = l >> 3)
  static constexpr int SLICE = NP / 8;
  static constexpr int KB = NP / 64;       // rows per lane
  static constexpr int MB = NP / 32;       // column quads per lane
  static constexpr int NV = KA;            // float4 per lane per step (= KB * MB)
  static constexpr int PD = NP == 64 ? 8 : (NP == 128 ? 3 : 1);  // steps in flight
  // alpha / Viterbi LDS per parity: P[RH][NP] partials, I[RH][NP] argmax rows, S[8] wave sums
  static constexpr int BUF = 2 * RH * NP + 8;
  static_assert(KB * MB == KA, "slice shapes");
};

struct TvArgs {
  const float* lo;    // (B,T,N) log emissions
  const float* lA;    // log transition matrices, element (b,k,i,j) at b*sb + k*st + i*N + j
  long long sb, st;   // batch / step strides of lA (elements)
  const float* init;  // (N) log initial probabilities
  const float* E;     // (B,T,NP) exp(lo - M) (FB)
  float* rows;        // U or V (B,T,NP) (FB); delta (B,T,N) (Viterbi)
  float* cs;          // (B,T) normalisers (FB)
  uint8_t* psi;       // (B,T,NP) (Viterbi)
  const float* binit; // beta: terminal vector exp(l - max l) (B,NP) or null (= 1)
  int B, T, N;
};

enum TvKind : int { kTvAlpha = 0, kTvBeta = 1, kTvVit = 2 };

// one step's slice of the matrix, one float4 per entry of dst.  Every lane issues its loads
// unconditionally and uses the values as loaded: an out-of-range entry reads a clamped
// in-range (finite) address, and its contribution vanishes downstream instead of being
// masked here — padded rows meet u = 0 (alpha), padded columns meet w = 0 (beta) or
// delta = -inf (Viterbi), and padded outputs are multiplied by E = 0 / added to lo = -inf.
// Nothing touches a prefetched register before the step that consumes it, and each ring
// slot is reloaded only after its last use, so the loop-carried registers coalesce (no
// copies at the back edge) and the compiler's vmcnt waits stay one ring slot deep.
template <int NP, int KIND, bool VEC>
__device__ __forceinline__ void tv_load(const TvArgs& a, int b, int kmat, float4 (&dst)[TvGeo<NP>::NV]) {
  using G = TvGeo<NP>;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float* base = a.lA + (size_t)b * a.sb + (size_t)kmat * a.st;
  const int N = a.N;
#pragma unroll
  for (int v = 0; v < G::NV; ++v) {
    int i, c0;
    if (KIND == kTvBeta) {
      const int k = v / G::MB, m = v % G::MB;
      i = G::SLICE * w + (l >> 3) + 8 * k;
      c0 = 4 * ((l & 7) + 8 * m);
    } else {
      i = (w / G::CB) * G::RPP + (l >> 3) + 8 * v;
      c0 = 32 * (w % G::CB) + 4 * (l & 7);
    }
    const float* p = base + (size_t)(i < N ? i : N - 1) * N;
    if (VEC) {
      dst[v] = *reinterpret_cast<const float4*>(p + (c0 < N ? c0 : N - 4));
    } else {
      dst[v].x = p[c0 < N ? c0 : N - 1];
      dst[v].y = p[c0 + 1 < N ? c0 + 1 : N - 1];
      dst[v].z = p[c0 + 2 < N ? c0 + 2 : N - 1];
      dst[v].w = p[c0 + 3 < N ? c0 + 3 : N - 1];
    }
  }
}

__device__ __forceinline__ float f4(const float4& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); }

// sum over the whole wave of a value held twice (lanes l and l ^ 8 after the row-lane
// reduction): the pair sum is exact, so the result is the sum over the 32 distinct values
__device__ __forceinline__ float wave_sum_pairs(float x) {
  x += dpp_f<0x128>(x);  // row_ror:8 (the duplicate)
  x += dpp_f<0xB1>(x);
  x += dpp_f<0x4E>(x);
  x += dpp_f<0x124>(x);
  return 0.5f * rows_sum(x);
}

// alpha: the four column partials reduced over the row lanes, transposed: lane keeps column
// cc = 2*bit5 + bit4 of its quad
template <int QW>
__device__ __forceinline__ float rowlanes_transpose_sum(float (&acc)[4]) {
  float a0 = acc[0], a2 = acc[2], a1 = acc[1], a3 = acc[3];
  permlane32_swap(a0, a2);  // lower: (c0 own, c0 partner)  upper: (c2 partner, c2 own)
  permlane32_swap(a1, a3);
  float p0 = a0 + a2, p1 = a1 + a3;
  permlane16_swap(p0, p1);  // even rows: (p0, p0 partner)  odd rows: (p1 partner, p1)
  float z = p0 + p1;
  if (QW <= 2) z += dpp_f<0x4E>(z);
  if (QW <= 4) z += dpp_f<0x124>(z);
  if (QW <= 8) z += dpp_f<0x128>(z);
  return z;
}

template <int QW>
__device__ __forceinline__ void rowlanes_transpose_argmax(float (&bv)[4], int (&bi)[4], float& v, int& i) {
  float a0 = bv[0], a2 = bv[2], a1 = bv[1], a3 = bv[3];
  int i0 = bi[0], i2 = bi[2], i1 = bi[1], i3 = bi[3];
  permlane32_swap(a0, a2);
  permlane32_swap_i(i0, i2);
  permlane32_swap(a1, a3);
  permlane32_swap_i(i1, i3);
  argmax_combine(a0, i0, a2, i2);
  argmax_combine(a1, i1, a3, i3);
  permlane16_swap(a0, a1);
  permlane16_swap_i(i0, i1);
  argmax_combine(a0, i0, a1, i1);
  if (QW <= 2) argmax_combine(a0, i0, dpp_f<0x4E>(a0), dpp_i<0x4E>(i0));
  if (QW <= 4) argmax_combine(a0, i0, dpp_f<0x124>(a0), dpp_i<0x124>(i0));
  if (QW <= 8) argmax_combine(a0, i0, dpp_f<0x128>(a0), dpp_i<0x128>(i0));
  v = a0;
  i = i0;
}

// beta: full sum over the 8 quad lanes of a row (bits 0..2)
__device__ __forceinline__ float quadlanes_sum(float x) {
  x += dpp_f<0xB1>(x);   // xor 1
  x += dpp_f<0x4E>(x);   // xor 2
  x += dpp_f<0x141>(x);  // row_half_mirror: lane k <-> 7-k (pairs the bit-2 halves)
  return x;
}

// beta: the KB row partials reduced over the quad lanes, transposed where KB > 1
template <int KB>
__device__ __forceinline__ float quadlanes_transpose_sum(float (&z)[KB], int l) {
  if constexpr (KB == 1) {
    return quadlanes_sum(z[0]);
  } else if constexpr (KB == 2) {
    const bool hi = l & 4;
    const float keep = hi ? z[1] : z[0], send = hi ? z[0] : z[1];
    float x = keep + dpp_f<0x141>(send);
    x += dpp_f<0xB1>(x);
    x += dpp_f<0x4E>(x);
    return x;
  } else {
    const bool h2 = l & 4, h1 = l & 2;
    float y0, y1;
    {
      const float k0 = h2 ? z[2] : z[0], s0 = h2 ? z[0] : z[2];
      const float k1 = h2 ? z[3] : z[1], s1 = h2 ? z[1] : z[3];
      y0 = k0 + dpp_f<0x141>(s0);
      y1 = k1 + dpp_f<0x141>(s1);
    }
    const float keep = h1 ? y1 : y0, send = h1 ? y0 : y1;
    float x = keep + dpp_f<0x4E>(send);
    x += dpp_f<0xB1>(x);
    return x;
  }
}

template <int NP, int KIND, bool VEC>
__device__ void tv_chain(const TvArgs& a, float* lds, int b) {
  using G = TvGeo<NP>;
  constexpr int PD = G::PD;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int T = a.T, N = a.N;
  constexpr bool COLS = KIND != kTvBeta;   // alpha / Viterbi layout

  // this lane's output index after the reduction, and whether it is the lane that stores it
  int jo;
  bool writer;
  const int part = w / G::CB, r8 = l >> 3;
  if (KIND == kTvBeta) {
    int kk = 0;
    if (G::KB == 2) kk = (l >> 2) & 1;
    if (G::KB == 4) kk = 2 * ((l >> 2) & 1) + ((l >> 1) & 1);
    jo = G::SLICE * w + r8 + 8 * kk;
    writer = G::KB == 1 ? (l & 7) == 0 : (G::KB == 2 ? (l & 3) == 0 : (l & 1) == 0);
  } else {
    const int cc = 2 * (l >> 5) + ((l >> 4) & 1);
    jo = 32 * (w % G::CB) + 4 * (l & 7) + cc;
    writer = (l & 8) == 0;
  }
  // alpha / Viterbi partial vectors are stored so that a lane's KA rows are contiguous
  auto perm = [&](int i) { return (i / G::RPP) * G::RPP + (i % 8) * G::KA + (i % G::RPP) / 8; };
  // lanes that publish the previous row (alpha: U row; Viterbi: delta + psi row): in the
  // column-block-0 waves, quad lane q publishes row k = q of its row lane (KA <= 8) or rows
  // q, q + 8, ... (KA > 8): every row exactly once, one or a few per lane
  const bool rowout = COLS && (w % G::CB) == 0 && (l & 7) < G::KA;
  auto Pbuf = [&](int par) { return lds + par * G::BUF; };                           // [RH][NP]
  auto Ibuf = [&](int par) { return reinterpret_cast<int*>(lds + par * G::BUF + G::RH * NP); };
  auto Sbuf = [&](int par) { return lds + par * G::BUF + 2 * G::RH * NP; };          // [8]
  float* vbuf = lds;  // beta: [2][NP]

  auto kmat_of = [&](int q) { return KIND == kTvBeta ? T - 1 - q : q - 1; };
  auto tout_of = [&](int q) { return KIND == kTvBeta ? T - 1 - q : q; };
  // the per-step scalar input (masked at use): E at the output time (alpha: scales u_t; beta:
  // forms the next product input w_t = v_t E_t) or the raw log-emission (Viterbi)
  auto emis_of = [&](int q) -> float {
    const int t = tout_of(q < T ? q : T - 1);
    if (KIND == kTvVit) return a.lo[((size_t)b * T + t) * N + (jo < N ? jo : N - 1)];
    return a.E[((size_t)b * T + t) * NP + jo];
  };
  // matrix loads for step q (clamped to the last step past the end: issued unconditionally)
  // (sched_barrier pins the loads where they are issued: left alone, the scheduler sinks them
  // to the end of the block, next to their uses in the next iteration, and the step that
  // consumes the slot then waits for nearly every load in flight)
  auto prefetch = [&](int q, float4 (&rw)[G::NV]) {
    __builtin_amdgcn_sched_barrier(0);
    tv_load<NP, KIND, VEC>(a, b, kmat_of(q < T ? q : T - 1), rw);
    __builtin_amdgcn_sched_barrier(0);
  };
  // alpha / Viterbi: this lane's KA rows of the previous vector = combination of the RH partials
  auto read_rows = [&](int par, float (&y)[G::KA]) {
    const float* P = Pbuf(par) + part * G::RPP + r8 * G::KA;
#pragma unroll
    for (int h = 0; h < G::RH; ++h) {
      float x[G::KA];
      if constexpr (G::KA % 4 == 0) {
#pragma unroll
        for (int k4 = 0; k4 < G::KA / 4; ++k4) {
          const float4 v = *reinterpret_cast<const float4*>(P + h * NP + 4 * k4);
          x[4 * k4] = v.x; x[4 * k4 + 1] = v.y; x[4 * k4 + 2] = v.z; x[4 * k4 + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int k2 = 0; k2 < G::KA / 2; ++k2) {
          const float2 v = *reinterpret_cast<const float2*>(P + h * NP + 2 * k2);
          x[2 * k2] = v.x; x[2 * k2 + 1] = v.y;
        }
      }
#pragma unroll
      for (int k = 0; k < G::KA; ++k) y[k] = h == 0 ? x[k] : (KIND == kTvVit ? fmaxf(y[k], x[k]) : y[k] + x[k]);
    }
  };
  // publish row t of the vector in buffer `par` (rowout lanes): alpha the U row (sum of the
  // partials), Viterbi delta (max of the partials) and psi (the index of the first part
  // attaining it: parts hold increasing row ranges, so that is the first index)
  auto publish_row = [&](int par, int t) {
#pragma unroll
    for (int kq = 0; kq < (G::KA + 7) / 8; ++kq) {
      const int k = (l & 7) + 8 * kq;
      if (k < G::KA) {
        const int off = part * G::RPP + r8 * G::KA + k;
        const int i = part * G::RPP + r8 + 8 * k;
        const float* P = Pbuf(par) + off;
        if (KIND == kTvAlpha) {
          float u = P[0];
#pragma unroll
          for (int h = 1; h < G::RH; ++h) u += P[h * NP];
          a.rows[((size_t)b * T + t) * NP + i] = u;
        } else {
          const int* I = Ibuf(par) + off;
          float m = P[0];
          int arg = I[0];
#pragma unroll
          for (int h = 1; h < G::RH; ++h) {
            const float x = P[h * NP];
            arg = x > m ? I[h * NP] : arg;
            m = fmaxf(m, x);
          }
          if (i < N) a.rows[((size_t)b * T + t) * N + i] = m;
          a.psi[((size_t)b * T + t) * NP + i] = (uint8_t)arg;
        }
      }
    }
  };

  float4 raw[PD][G::NV];
  float eR[PD];
  if (T > 1) {
#pragma unroll
    for (int s = 0; s < PD; ++s) {
      prefetch(1 + s, raw[s]);
      eR[s] = emis_of(1 + s);
    }
  }

  // row 0 of the recursion
  {
    float v0;
    const int jj = jo < N ? jo : 0;
    if (KIND == kTvAlpha) v0 = jo < N ? __expf(a.init[jj]) * a.E[(size_t)b * T * NP + jo] : 0.f;
    else if (KIND == kTvBeta) v0 = jo < N ? a.E[((size_t)b * T + T - 1) * NP + jo] * (a.binit ? a.binit[(size_t)b * NP + jo] : 1.f) : 0.f;  // w_{T-1} = E_{T-1} v_{T-1}
    else v0 = jo < N ? a.init[jj] + a.lo[(size_t)b * T * N + jo] : -INFINITY;
    if (COLS) {
      // row part 0 carries the vector, the other parts the identity (0 / -inf)
      const float pv = part == 0 ? v0 : (KIND == kTvAlpha ? 0.f : -INFINITY);
      if (writer) {
        Pbuf(0)[part * NP + perm(jo)] = pv;
        if (KIND == kTvVit) Ibuf(0)[part * NP + perm(jo)] = 0;
      }
      if (KIND == kTvAlpha) {
        const float sw = wave_sum_pairs(pv);
        if (l == 0) Sbuf(0)[w] = sw;
      }
    } else if (writer) {
      vbuf[jo] = v0;
      a.rows[((size_t)b * T + T - 1) * NP + jo] = jo < N ? (a.binit ? a.binit[(size_t)b * NP + jo] : 1.f) : 0.f;
    }
  }
  lds_barrier();

  auto step = [&](int q, float4 (&rw)[G::NV], float& er) {
    const int t = tout_of(q);
    if (KIND == kTvBeta) {
      const float* prev = vbuf + ((q - 1) & 1) * NP;
      float* cur = vbuf + (q & 1) * NP;
      float wv[G::MB][4];
#pragma unroll
      for (int m = 0; m < G::MB; ++m) {
        const float4 x = *reinterpret_cast<const float4*>(prev + 4 * ((l & 7) + 8 * m));
        wv[m][0] = x.x; wv[m][1] = x.y; wv[m][2] = x.z; wv[m][3] = x.w;
      }
      float cs = 0.f;
#pragma unroll
      for (int m = 0; m < G::MB; ++m) cs += (wv[m][0] + wv[m][1]) + (wv[m][2] + wv[m][3]);
      cs = quadlanes_sum(cs);
      float z[G::KB];
#pragma unroll
      for (int k = 0; k < G::KB; ++k) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int m = 0; m < G::MB; ++m) {
          const float4 A = rw[k * G::MB + m];
          s0 = fmaf(__expf(A.x), wv[m][0], s0);
          s1 = fmaf(__expf(A.y), wv[m][1], s1);
          s0 = fmaf(__expf(A.z), wv[m][2], s0);
          s1 = fmaf(__expf(A.w), wv[m][3], s1);
        }
        z[k] = s0 + s1;
      }
      prefetch(q + PD, rw);
      const float zz = quadlanes_transpose_sum<G::KB>(z, l);
      const float v = zz * __builtin_amdgcn_rcpf(cs);
      if (writer) {
        cur[jo] = v * er;
        a.rows[((size_t)b * T + t) * NP + jo] = v;
      }
      if (tid == 0) a.cs[(size_t)b * T + t] = cs;
      er = emis_of(q + PD);
    } else {
      const int pp = (q - 1) & 1, cp = q & 1;
      float y[G::KA];
      read_rows(pp, y);
      if (KIND == kTvAlpha) {
        const float4 s0 = *reinterpret_cast<const float4*>(Sbuf(pp));
        const float4 s1 = *reinterpret_cast<const float4*>(Sbuf(pp) + 4);
        const float cs = ((s0.x + s0.y) + (s0.z + s0.w)) + ((s1.x + s1.y) + (s1.z + s1.w));   // c_{q-1}
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < G::KA; ++k) {
          const float4 A = rw[k];
          acc[0] = fmaf(y[k], __expf(A.x), acc[0]);
          acc[1] = fmaf(y[k], __expf(A.y), acc[1]);
          acc[2] = fmaf(y[k], __expf(A.z), acc[2]);
          acc[3] = fmaf(y[k], __expf(A.w), acc[3]);
        }
        prefetch(q + PD, rw);
        const float z = rowlanes_transpose_sum<8>(acc);
        const float u = z * (er * __builtin_amdgcn_rcpf(cs));
        if (writer) Pbuf(cp)[part * NP + perm(jo)] = u;
        const float sw = wave_sum_pairs(u);
        if (l == 0) Sbuf(cp)[w] = sw;
        if (rowout) publish_row(pp, q - 1);  // u_{q-1} -> the U row of the posterior pass
        if (tid == 0) a.cs[(size_t)b * T + t] = cs;
        er = emis_of(q + PD);
      } else {
        // max-plus with the first index: rows increase with k, strict > keeps the first
        const int i0 = part * G::RPP + r8;
        float bv[4];
        int bi[4];
        {
          const float4 A = rw[0];
          bv[0] = y[0] + A.x; bv[1] = y[0] + A.y; bv[2] = y[0] + A.z; bv[3] = y[0] + A.w;
          bi[0] = bi[1] = bi[2] = bi[3] = i0;
        }
#pragma unroll
        for (int k = 1; k < G::KA; ++k) {
          const float4 A = rw[k];
          const int ii = i0 + 8 * k;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float s = y[k] + f4(A, c);
            bi[c] = s > bv[c] ? ii : bi[c];
            bv[c] = fmaxf(bv[c], s);
          }
        }
        prefetch(q + PD, rw);
        float v;
        int vi;
        rowlanes_transpose_argmax<8>(bv, bi, v, vi);
        // fl(max + lo) per part: rounding is monotone, so the readers' max over parts is the
        // reference's fl(max_i(...) + lo)
        const float d = v + (jo < N ? er : -INFINITY);
        if (writer) {
          Pbuf(cp)[part * NP + perm(jo)] = d;
          Ibuf(cp)[part * NP + perm(jo)] = vi;
        }
        if (rowout) publish_row(pp, q - 1);
        er = emis_of(q + PD);
      }
    }
    lds_barrier();
  };

  // full blocks of PD steps (no exit inside the unrolled body), then the tail
  int q0 = 1;
  for (; q0 + PD <= T; q0 += PD) {
#pragma unroll
    for (int s = 0; s < PD; ++s) step(q0 + s, raw[s], eR[s]);
  }
#pragma unroll
  for (int s = 0; s < PD; ++s)
    if (q0 + s < T) step(q0 + s, raw[s], eR[s]);
  if (COLS) {
    // the last row: combined from its partials
    const int pl = (T - 1) & 1;
    if (rowout) publish_row(pl, T - 1);
    if (KIND == kTvAlpha) {
      // c_{T-1} = sum u_{T-1} (the sequence log-likelihood), kept in slot t = 0 of CA
      if (tid == 0) {
        const float* S = Sbuf(pl);
        a.cs[(size_t)b * T] = ((S[0] + S[1]) + (S[2] + S[3])) + ((S[4] + S[5]) + (S[6] + S[7]));
      }
    }
  }
}

template <int NP, bool VEC>
__global__ void __launch_bounds__(512) tv_fb_kernel(TvArgs fa, TvArgs fb) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x >> 1;
  if (blockIdx.x & 1)
    tv_chain<NP, kTvBeta, VEC>(fb, lds, b);
  else
    tv_chain<NP, kTvAlpha, VEC>(fa, lds, b);
}

template <int NP, bool VEC>
__global__ void __launch_bounds__(512) tv_vit_kernel(TvArgs va) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  tv_chain<NP, kTvVit, VEC>(va, lds, blockIdx.x);
}

// ---------------------------------------------------------------------------------------
// Adjoint of the time-varying forward-backward OUTPUTS (NeuralHMM training through its
// posteriors / forward / backward; reference neural.py:355-461, where autograd runs back
// through the per-step logsumexp loops).  The same two linear chains as csrc/adjoint.hip
// (pytorch_hmm_amd/autograd.py derives them), with the step's own matrix A_k = exp(lA_k)
// (k links steps k and k+1) streamed from HBM exactly as the forward chains stream it:
//   W (beta layout, backward in time):  W_{T-1} = S_{T-1};
//        W_t[i] = S_t[i] + F_t * sum_j A_t[i][j] E_{t+1}[j] W_{t+1}[j]
//   Z (alpha layout, forward in time):  Z_0 = R_0;  Z_t = R_t + P_t,
//        P_t[j] = G_t * E_t[j] * sum_i Z_{t-1}[i] A_{t-1}[i][j]
// Outputs W and P (B,T,N) (P_0 = 0; P kept apart from R so that V * P never cancels).  The
// alpha layout's row parts hold PARTIAL sums (linear in the previous vector), so the P
// partials go to Pbuf and R_t to a row of its own (Rbuf); a reader forms Z = sum P + R, the
// published row is sum P alone.  Per-step loads (source, emission, scale) are issued PD steps
// ahead beside the matrix prefetch.
struct TvAdjArgs {
  const float* lA;
  long long sb, st;
  const float* E;    // (B,T,N) staged emissions exp(lo - M)
  const float* src;  // (B,T,N) S (W chain) / R (Z chain)
  const float* sc;   // (B,T)   F_t (W chain) / G_t (Z chain)
  float* out;        // (B,T,N) W / P
  int B, T, N;
};

template <int NP, int CH, bool VEC>
__device__ void tv_adj_chain(const TvAdjArgs& j, float* lds, int b) {
  using G = TvGeo<NP>;
  constexpr int PD = G::PD;
  constexpr int KIND = CH == 0 ? kTvBeta : kTvAlpha;   // matrix slice layout (tv_load)
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int T = j.T, N = j.N;
  // tv_load reads lA / sb / st / N from a TvArgs
  TvArgs ta{nullptr, j.lA, j.sb, j.st, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, j.B, T, N};
  int jo;
  bool writer;
  const int part = w / G::CB, r8 = l >> 3;
  if (CH == 0) {
    int kk = 0;
    if (G::KB == 2) kk = (l >> 2) & 1;
    if (G::KB == 4) kk = 2 * ((l >> 2) & 1) + ((l >> 1) & 1);
    jo = G::SLICE * w + r8 + 8 * kk;
    writer = G::KB == 1 ? (l & 7) == 0 : (G::KB == 2 ? (l & 3) == 0 : (l & 1) == 0);
  } else {
    const int cc = 2 * (l >> 5) + ((l >> 4) & 1);
    jo = 32 * (w % G::CB) + 4 * (l & 7) + cc;
    writer = (l & 8) == 0;
  }
  const bool jok = jo < N;
  const int jc = jok ? jo : 0;
  auto perm = [&](int i) { return (i / G::RPP) * G::RPP + (i % 8) * G::KA + (i % G::RPP) / 8; };
  const bool rowout = CH == 1 && (w % G::CB) == 0 && (l & 7) < G::KA;
  constexpr int BUFZ = (G::RH + 1) * NP;  // Z chain per parity: P partials [RH][NP] + R [NP]
  auto Pbuf = [&](int par) { return lds + par * BUFZ; };
  auto Rbuf = [&](int par) { return lds + par * BUFZ + G::RH * NP; };
  float* xbuf = lds;  // W chain: [2][NP] product input E W

  const size_t rb = (size_t)b * T;
  auto kmat_of = [&](int q) { return CH == 0 ? T - 1 - q : q - 1; };
  auto tout_of = [&](int q) { return CH == 0 ? T - 1 - q : q; };
  auto prefetch = [&](int q, float4 (&rw)[G::NV]) {
    __builtin_amdgcn_sched_barrier(0);
    tv_load<NP, KIND, VEC>(ta, b, kmat_of(q < T ? q : T - 1), rw);
    __builtin_amdgcn_sched_barrier(0);
  };
  // per-step scalars of this lane's output, loaded PD steps ahead (clamped past the end)
  auto aux = [&](int q, float& s_, float& e_, float& f_) {
    const size_t row = rb + tout_of(q < T ? q : T - 1);
    s_ = j.src[row * N + jc];
    e_ = j.E[row * N + jc];
    f_ = j.sc[row];
  };
  auto read_rows = [&](int par, float (&y)[G::KA]) {
    const float* P = Pbuf(par) + part * G::RPP + r8 * G::KA;
    const float* R = Rbuf(par) + part * G::RPP + r8 * G::KA;
#pragma unroll
    for (int h = 0; h <= G::RH; ++h) {
      const float* src = h < G::RH ? P + h * NP : R;
      float x[G::KA];
      if constexpr (G::KA % 4 == 0) {
#pragma unroll
        for (int k4 = 0; k4 < G::KA / 4; ++k4) {
          const float4 v = *reinterpret_cast<const float4*>(src + 4 * k4);
          x[4 * k4] = v.x; x[4 * k4 + 1] = v.y; x[4 * k4 + 2] = v.z; x[4 * k4 + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int k2 = 0; k2 < G::KA / 2; ++k2) {
          const float2 v = *reinterpret_cast<const float2*>(src + 2 * k2);
          x[2 * k2] = v.x; x[2 * k2 + 1] = v.y;
        }
      }
#pragma unroll
      for (int k = 0; k < G::KA; ++k) y[k] = h == 0 ? x[k] : y[k] + x[k];
    }
  };
  // P row t (the sum of the partials, no R) -> HBM
  auto publish_row = [&](int par, int t) {
#pragma unroll
    for (int kq = 0; kq < (G::KA + 7) / 8; ++kq) {
      const int k = (l & 7) + 8 * kq;
      if (k < G::KA) {
        const int off = part * G::RPP + r8 * G::KA + k;
        const int i = part * G::RPP + r8 + 8 * k;
        const float* P = Pbuf(par) + off;
        float u = P[0];
#pragma unroll
        for (int h = 1; h < G::RH; ++h) u += P[h * NP];
        if (i < N) j.out[(rb + t) * N + i] = u;
      }
    }
  };

  float4 raw[PD][G::NV];
  float rS[PD], rE[PD], rF[PD];
  if (T > 1) {
#pragma unroll
    for (int s = 0; s < PD; ++s) {
      prefetch(1 + s, raw[s]);
      aux(1 + s, rS[s], rE[s], rF[s]);
    }
  }
  // step 0: W_{T-1} = S_{T-1};  Z_0 = R_0 (P_0 = 0)
  {
    float s0, e0, f0;
    aux(0, s0, e0, f0);
    s0 = jok ? s0 : 0.f;
    if (CH == 0) {
      if (writer) {
        xbuf[jo] = jok ? e0 * s0 : 0.f;
        if (jok) j.out[(rb + T - 1) * N + jo] = s0;
      }
    } else if (writer) {
      Pbuf(0)[part * NP + perm(jo)] = 0.f;
      if (part == 0) Rbuf(0)[perm(jo)] = s0;
    }
  }
  lds_barrier();

  auto step = [&](int q, float4 (&rw)[G::NV], float& rs, float& re, float& rf) {
    const int t = tout_of(q);
    if (CH == 0) {
      const float* prev = xbuf + ((q - 1) & 1) * NP;
      float* cur = xbuf + (q & 1) * NP;
      float wv[G::MB][4];
#pragma unroll
      for (int m = 0; m < G::MB; ++m) {
        const float4 x = *reinterpret_cast<const float4*>(prev + 4 * ((l & 7) + 8 * m));
        wv[m][0] = x.x; wv[m][1] = x.y; wv[m][2] = x.z; wv[m][3] = x.w;
      }
      float z[G::KB];
#pragma unroll
      for (int k = 0; k < G::KB; ++k) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int m = 0; m < G::MB; ++m) {
          const float4 A = rw[k * G::MB + m];
          s0 = fmaf(__expf(A.x), wv[m][0], s0);
          s1 = fmaf(__expf(A.y), wv[m][1], s1);
          s0 = fmaf(__expf(A.z), wv[m][2], s0);
          s1 = fmaf(__expf(A.w), wv[m][3], s1);
        }
        z[k] = s0 + s1;
      }
      prefetch(q + PD, rw);
      const float zz = quadlanes_transpose_sum<G::KB>(z, l);
      const float v = (jok ? rs : 0.f) + rf * zz;   // W_t = S_t + F_t (A_t (E W)_{t+1})
      if (writer) {
        cur[jo] = jok ? re * v : 0.f;
        if (jok) j.out[(rb + t) * N + jo] = v;
      }
    } else {
      const int pp = (q - 1) & 1, cp = q & 1;
      float y[G::KA];
      read_rows(pp, y);   // Z_{t-1} = R + sum of the P partials
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < G::KA; ++k) {
        const float4 A = rw[k];
        acc[0] = fmaf(y[k], __expf(A.x), acc[0]);
        acc[1] = fmaf(y[k], __expf(A.y), acc[1]);
        acc[2] = fmaf(y[k], __expf(A.z), acc[2]);
        acc[3] = fmaf(y[k], __expf(A.w), acc[3]);
      }
      prefetch(q + PD, rw);
      const float z = rowlanes_transpose_sum<8>(acc);
      const float pr = rf * ((jok ? re : 0.f) * z);   // this row part's share of P_t
      if (writer) {
        Pbuf(cp)[part * NP + perm(jo)] = pr;
        if (part == 0) Rbuf(cp)[perm(jo)] = jok ? rs : 0.f;
      }
      if (rowout) publish_row(pp, q - 1);
    }
    aux(q + PD, rs, re, rf);
    lds_barrier();
  };
  int q0 = 1;
  for (; q0 + PD <= T; q0 += PD) {
#pragma unroll
    for (int s = 0; s < PD; ++s) step(q0 + s, raw[s], rS[s], rE[s], rF[s]);
  }
#pragma unroll
  for (int s = 0; s < PD; ++s)
    if (q0 + s < T) step(q0 + s, raw[s], rS[s], rE[s], rF[s]);
  if (CH == 1 && rowout) publish_row((T - 1) & 1, T - 1);
}

template <int NP, bool VEC>
__global__ void __launch_bounds__(512) tv_adjoint_kernel(TvAdjArgs aw, TvAdjArgs az) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x >> 1;
  if (blockIdx.x & 1) tv_adj_chain<NP, 1, VEC>(az, lds, b);
  else tv_adj_chain<NP, 0, VEC>(aw, lds, b);
}

// E = exp(lo - M) per (b,t) row (zero-padded to NP), M = the row max (0 for an all -inf row).
// One wave per row, grid-stride.
template <int NP>
__global__ void __launch_bounds__(256) tv_emis_kernel(const float* __restrict__ lo, float* __restrict__ E,
                                                      float* __restrict__ M, size_t rows, int N) {
  constexpr int K = NP / 64;
  const int l = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t row = wave; row < rows; row += nw) {
    float v[K], m = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = l + 64 * k;
      v[k] = j < N ? lo[row * N + j] : -INFINITY;
      m = fmaxf(m, v[k]);
    }
    m = wave_max(m);
    if (m == -INFINITY) m = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) E[row * NP + l + 64 * k] = __expf(v[k] - m);
    if (l == 0) M[row] = m;
  }
}

// LA_t = M_0 + sum_{s=1..t} (log CA_s + M_s)  (block 2b), loglik = LA_{T-1} + log CA_0 (CA_0
// holds sum u_{T-1});  LB_t = bscale + sum_{s=t..T-2} (log CB_s + M_{s+1})  (block 2b+1).
// One wave per (sequence, direction), fp64 running sums.
__global__ void __launch_bounds__(64) tv_scan_kernel(const float* __restrict__ CA, const float* __restrict__ CB,
                                                     const float* __restrict__ M, float* __restrict__ LA,
                                                     float* __restrict__ LB, float* __restrict__ loglik,
                                                     const float* __restrict__ bscale, int T) {
  const int b = blockIdx.x >> 1, l = threadIdx.x;
  const size_t o = (size_t)b * T;
  if ((blockIdx.x & 1) == 0) {
    double base = 0.0;
    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + l;
      double x = 0.0;
      if (t < T) x = t == 0 ? (double)M[o] : (double)__logf(CA[o + t]) + (double)M[o + t];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_up(x, off);
        if (l >= off) x += y;
      }
      if (t < T) LA[o + t] = (float)(base + x);
      base += __shfl(x, 63);
    }
    if (l == 0 && loglik) loglik[b] = (float)(base + (double)__logf(CA[o]));
  } else {
    double base = bscale ? (double)bscale[b] : 0.0;  // LB_{T-1} = log of the terminal vector's scale
    for (int t1 = T; t1 > 0; t1 -= 64) {
      const int t = t1 - 1 - l;  // descending
      double x = 0.0;
      if (t >= 0 && t <= T - 2) x = (double)__logf(CB[o + t]) + (double)M[o + t + 1];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_up(x, off);
        if (l >= off) x += y;
      }
      if (t >= 0) LB[o + t] = (float)(base + x);
      base += __shfl(x, 63);
    }
  }
}

// psi rows of one chunk (written by the chain) -> the chunk map (post.h)
template <int NP>
__global__ void __launch_bounds__(NP) tv_chunkmap_kernel(VitArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t prow[kChunk][NP];
  const int chunk = blockIdx.x, b = blockIdx.y;
  if (chunk == 0) return;
  const int t_lo = chunk * kChunk;
  const int t_hi = (t_lo + kChunk < a.T ? t_lo + kChunk : a.T) - 1;
  const int rows = t_hi - t_lo + 1;
  const uint8_t* src = a.psi + ((size_t)b * a.T + t_lo) * NP;
  for (int idx = threadIdx.x; idx < rows * NP / 16; idx += NP)
    *reinterpret_cast<uint4*>(&prow[0][0] + idx * 16) = *reinterpret_cast<const uint4*>(src + idx * 16);
  __syncthreads();
  compose_chunk_map<NP>(a, prow, b, chunk, t_lo, t_hi);
}

struct TvFbWs {
  float *U, *V, *LA, *LB, *E, *M, *CA, *CB, *binit, *bscale;
};
static size_t tv_fb_ws_layout(int B, int T, int N, char* base, TvFbWs* w) {
  const size_t NP = pad_states(N), rows = (size_t)B * T;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += align_up(bytes, 256); return o; };
  const size_t oU = take(2 * rows * NP * sizeof(float));   // U | V (post.h expects V = U + rows*NP)
  const size_t oL = take(2 * rows * sizeof(float));        // LA | LB
  const size_t oE = take(rows * NP * sizeof(float));
  const size_t oM = take(rows * sizeof(float));
  const size_t oC = take(2 * rows * sizeof(float));        // CA | CB
  const size_t oI = take((size_t)B * NP * sizeof(float));   // terminal vector (adjoint)
  const size_t oS = take((size_t)B * sizeof(float));
  if (w && base) {
    w->U = reinterpret_cast<float*>(base + oU);
    w->V = w->U + rows * NP;
    w->LA = reinterpret_cast<float*>(base + oL);
    w->LB = w->LA + rows;
    w->E = reinterpret_cast<float*>(base + oE);
    w->M = reinterpret_cast<float*>(base + oM);
    w->CA = reinterpret_cast<float*>(base + oC);
    w->CB = w->CA + rows;
    w->binit = reinterpret_cast<float*>(base + oI);
    w->bscale = reinterpret_cast<float*>(base + oS);
  }
  return off;
}

static bool tv_vec_ok(const float* lA, long long sb, long long st, int N) {
  return (N % 4) == 0 && (sb % 4) == 0 && (st % 4) == 0 && (reinterpret_cast<uintptr_t>(lA) & 15) == 0;
}

template <int NP>
static hipError_t launch_tv_fb(const TvArgs& fa, const TvArgs& fb, const PostArgs& pa, const TvFbWs& w,
                               float* loglik, const float* bscale, bool vec, hipStream_t st) {
  const size_t rows = (size_t)fa.B * fa.T;
  {
    const size_t waves = rows < 16384 ? rows : 16384;
    hipLaunchKernelGGL(tv_emis_kernel<NP>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, fa.lo, w.E, w.M,
                       rows, fa.N);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipError_t e;
  if (vec) {
    e = allow_lds(tv_fb_kernel<NP, true>, kExclusiveLds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((tv_fb_kernel<NP, true>), dim3(2 * fa.B), dim3(512), kExclusiveLds, st, fa, fb);
  } else {
    e = allow_lds(tv_fb_kernel<NP, false>, kExclusiveLds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((tv_fb_kernel<NP, false>), dim3(2 * fa.B), dim3(512), kExclusiveLds, st, fa, fb);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tv_scan_kernel, dim3(2 * fa.B), dim3(64), 0, st, w.CA, w.CB, w.M, w.LA, w.LB, loglik, bscale,
                     fa.T);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t waves = rows < 8192 ? rows : 8192;
  hipLaunchKernelGGL(fb_posterior_kernel<NP>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, pa);
  return hipGetLastError();
}

template <int NP>
static hipError_t launch_tv_vit(const TvArgs& ta, const VitArgs& va, bool vec, hipStream_t st) {
  hipError_t e;
  if (vec) {
    e = allow_lds(tv_vit_kernel<NP, true>, kExclusiveLds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((tv_vit_kernel<NP, true>), dim3(ta.B), dim3(512), kExclusiveLds, st, ta);
  } else {
    e = allow_lds(tv_vit_kernel<NP, false>, kExclusiveLds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((tv_vit_kernel<NP, false>), dim3(ta.B), dim3(512), kExclusiveLds, st, ta);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tv_chunkmap_kernel<NP>, dim3(va.nchunks, va.B), dim3(NP), 0, st, va);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(vit_backtrace_kernel<NP>, dim3(va.nchunks, va.B), dim3(64), 0, st, va);
  return hipGetLastError();
}


}  // namespace hmm355

using namespace hmm355;

HMM355_API size_t hmm355_tv_fb_workspace_bytes(int B, int T, int N) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return 0;
  return tv_fb_ws_layout(B, T, N, nullptr, nullptr);
}

HMM355_API int hmm355_tv_forward_backward_ex_f32(const float* log_obs, const float* log_A, long long a_bstride,
                                                 long long a_tstride, const float* log_p0, const float* log_beta_T,
                                                 int B, int T, int N, unsigned out_mask, float* posterior,
                                                 float* forward, float* backward, float* loglik, float* lik_ref,
                                                 void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || N < 0 || a_bstride < 0 || a_tstride < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!log_obs || !log_A || !log_p0 || !workspace) return HMM355_E_ARG;
  if ((out_mask & HMM355_FB_POSTERIOR) && !posterior) return HMM355_E_ARG;
  if ((out_mask & HMM355_FB_FORWARD) && !forward) return HMM355_E_ARG;
  if ((out_mask & HMM355_FB_BACKWARD) && !backward) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40) return HMM355_E_SHAPE;
  if (workspace_bytes < hmm355_tv_fb_workspace_bytes(B, T, N)) return HMM355_E_WORKSPACE;
  const int NP = pad_states(N);
  TvFbWs w;
  tv_fb_ws_layout(B, T, N, static_cast<char*>(workspace), &w);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const float* binit = nullptr;
  const float* bscale = nullptr;
  if (log_beta_T) {  // the same terminal-vector preparation as fb.hip
    switch (NP) {
      case 64: hipLaunchKernelGGL(beta_init_kernel<64>, dim3(B), dim3(64), 0, st, log_beta_T, N, w.binit, w.bscale); break;
      case 128: hipLaunchKernelGGL(beta_init_kernel<128>, dim3(B), dim3(64), 0, st, log_beta_T, N, w.binit, w.bscale); break;
      default: hipLaunchKernelGGL(beta_init_kernel<256>, dim3(B), dim3(64), 0, st, log_beta_T, N, w.binit, w.bscale); break;
    }
    const hipError_t e0 = hipGetLastError();
    if (e0 != hipSuccess) return (int)e0;
    binit = w.binit;
    bscale = w.bscale;
  }
  TvArgs fa{log_obs, log_A, a_bstride, a_tstride, log_p0, w.E, w.U, w.CA, nullptr, nullptr, B, T, N};
  TvArgs fb{log_obs, log_A, a_bstride, a_tstride, log_p0, w.E, w.V, w.CB, nullptr, binit, B, T, N};
  PostArgs pa{w.U, w.V, w.LA, w.LB, posterior, forward, backward, lik_ref, B, T, N, out_mask};
  const bool vec = tv_vec_ok(log_A, a_bstride, a_tstride, N);
  hipError_t e;
  switch (NP) {
    case 64: e = launch_tv_fb<64>(fa, fb, pa, w, loglik, bscale, vec, st); break;
    case 128: e = launch_tv_fb<128>(fa, fb, pa, w, loglik, bscale, vec, st); break;
    default: e = launch_tv_fb<256>(fa, fb, pa, w, loglik, bscale, vec, st); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_tv_forward_backward_f32(const float* log_obs, const float* log_A, long long a_bstride,
                                              long long a_tstride, const float* log_p0, int B, int T, int N,
                                              unsigned out_mask, float* posterior, float* forward,
                                              float* backward, float* loglik, float* lik_ref, void* workspace,
                                              size_t workspace_bytes, void* stream) {
  return hmm355_tv_forward_backward_ex_f32(log_obs, log_A, a_bstride, a_tstride, log_p0, nullptr, B, T, N, out_mask,
                                           posterior, forward, backward, loglik, lik_ref, workspace, workspace_bytes,
                                           stream);
}

HMM355_API size_t hmm355_tv_viterbi_workspace_bytes(int B, int T, int N) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return 0;
  const size_t NP = pad_states(N);
  const size_t nc = (T + kChunk - 1) / kChunk;
  return align_up((size_t)B * T * NP, 256) + align_up((size_t)B * nc * NP, 256);
}

HMM355_API int hmm355_tv_viterbi_f32(const float* log_obs, const float* log_A, long long a_bstride,
                                     long long a_tstride, const float* init, int B, int T, int N, int64_t* states,
                                     float* log_delta, void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || N < 0 || a_bstride < 0 || a_tstride < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!log_obs || !log_A || !init || !states || !log_delta || !workspace) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40 || B > 65535) return HMM355_E_SHAPE;
  if (workspace_bytes < hmm355_tv_viterbi_workspace_bytes(B, T, N)) return HMM355_E_WORKSPACE;
  const int NP = pad_states(N);
  const int nc = (T + kChunk - 1) / kChunk;
  uint8_t* psi = static_cast<uint8_t*>(workspace);
  uint8_t* G = psi + align_up((size_t)B * T * NP, 256);
  TvArgs ta{log_obs, log_A, a_bstride, a_tstride, init, nullptr, log_delta, nullptr, psi, nullptr, B, T, N};
  VitArgs va{log_obs, log_A, init, log_delta, nullptr, states, psi, G, B, T, N, HMM355_OBS_LOG, nc, nullptr};
  const bool vec = tv_vec_ok(log_A, a_bstride, a_tstride, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (NP) {
    case 64: e = launch_tv_vit<64>(ta, va, vec, st); break;
    case 128: e = launch_tv_vit<128>(ta, va, vec, st); break;
    default: e = launch_tv_vit<256>(ta, va, vec, st); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_tv_fb_adjoint_f32(const float* E, const float* log_A, long long a_bstride, long long a_tstride,
                                        const float* src_w, const float* scale_w, const float* src_z,
                                        const float* scale_z, int B, int T, int N, float* W, float* P, void* stream) {
  if (B < 0 || N < 0 || a_bstride < 0 || a_tstride < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!E || !log_A || !src_w || !scale_w || !src_z || !scale_z || !W || !P) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40 || B > (1 << 30)) return HMM355_E_SHAPE;
  TvAdjArgs aw{log_A, a_bstride, a_tstride, E, src_w, scale_w, W, B, T, N};
  TvAdjArgs az{log_A, a_bstride, a_tstride, E, src_z, scale_z, P, B, T, N};
  const bool vec = tv_vec_ok(log_A, a_bstride, a_tstride, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipSuccess;
  auto go = [&](auto kern) {
    e = allow_lds(kern, kExclusiveLds);
    if (e != hipSuccess) return;
    hipLaunchKernelGGL(kern, dim3(2 * B), dim3(512), kExclusiveLds, st, aw, az);
    e = hipGetLastError();
  };
  switch (pad_states(N)) {
    case 64: vec ? go(tv_adjoint_kernel<64, true>) : go(tv_adjoint_kernel<64, false>); break;
    case 128: vec ? go(tv_adjoint_kernel<128, true>) : go(tv_adjoint_kernel<128, false>); break;
    default: vec ? go(tv_adjoint_kernel<256, true>) : go(tv_adjoint_kernel<256, false>); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}
