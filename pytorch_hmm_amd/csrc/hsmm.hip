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
//   final value — so the forward stores only M and Dm, and the backtrace finds p1 and
//   xb = max over the candidates before p1 for the segments on the decoded path and
//   re-resolves exactly there (rare).
//   obs_sum is torch-CPU's order for a strided slice of length d (tsum.h): four accumulators
//   over whole groups of 4 with ATen's cascade step every 16 groups, the tail folded into the
//   first, then ((a0+a1)+a2)+a3.
//
// hsmm_fwd_kernel<SUB, NJ, SMAX>: one workgroup per sequence (SMAX * SUB threads), the segment
//   END time t as the loop index (semimarkov.hip's layout): SUB lanes (a DPP group) per state;
//   lane `sub` owns the start-time slots k = NJ*sub + j (mod R = SUB*NJ) of its state.  A live
//   segment's torch-order obs_sum state (the four group accumulators and the tail sum) and its
//   predecessor score M stay in the slot's registers for the segment's life, so a step reads
//   one lp row, writes delta's per-state maximum Dm for the predecessor phase, and meets at ONE
//   barrier.  Slots j and j + NJ/2 run as one packed-fp32 pair (v_pk_add_f32: the obs_sum and
//   delta adds of two segments per instruction; with NJ/2 a multiple of 4 both halves take the
//   same accumulator update).  The branchy literal conditions are folded into the data: a slot
//   not yet started has M = -inf, the slot starting at time 0 has M = 0 (fl(0 + o) == o), and
//   durations beyond Dmax or padding states read -inf from the duration table.  Per end time t
//   the kernel stores M[t][s] (the best fl(delta + logT) over predecessors ending at t, for
//   segments starting at t+1) and Dm[t][s].  Geometries: (4, 16, 64) for the config-5 class
//   (S <= 64, Dmax <= 63), (8, 8, 64) / (16, 4, 64) the same with 8- and 16-lane groups, (8, 16, 64) for Dmax <= 71 (longer segments take torch's
//   cascade order: hsmm_wide.hip) and (4, 16, 128) for 65 <= S <= 128 with
//   Dmax <= 63.
// hsmm_backtrace_kernel / hsmm_chunk_walk_kernel + hsmm_stitch_kernel: the walk over the
//   segments (hsmm.py:331-352).  For each segment it finds the first predecessor state
//   attaining M from the stored Dm row (the forward's own candidate values), recomputes,
//   bit-identically, that state's candidate deltas to find the first d' and xb (the best
//   total of the earlier candidates), and re-resolves the rare case where an earlier
//   candidate rounds to the same total.  Two dependent global round trips per segment, so
//   from 3 chunks of 64 frames up the walk is cut into chunks walked in parallel and stitched
//   exactly (see hsmm_chunk_walk_kernel).
#include <stdlib.h>

#include <algorithm>

#include <type_traits>

#include "common.h"
#include "tsum.h"

namespace hmm355 {

constexpr int kHsL = 128;    // lp row ring (two 64-row chunks)
constexpr int kHsSMax = 128; // states (the largest geometry below)
constexpr int kHsRegDMax = 71;  // the longest duration the register-slot kernels take (tsum.h)

typedef float hs_f2 __attribute__((ext_vector_type(2)));

// Kernel geometry: SUB lanes per state (one DPP group), NJ start-time slots per lane, SMAX
// states per workgroup.  R = SUB * NJ slots (a segment's duration is < R), NT threads.
template <int SUB, int NJ, int SMAX>
struct HsG {
  static constexpr int R = SUB * NJ;
  static constexpr int NT = SMAX * SUB;
  static constexpr int NPRED = SMAX / SUB;   // predecessor states per lane
  static constexpr int PER = 64 * SMAX / NT; // lp values per thread per 64-row chunk
  static constexpr int NP2 = NJ / 2;         // packed slot pairs (j, j + NJ/2)
  static constexpr int DW = R + NJ + 1;      // duration-pair table row stride
  static_assert(NJ % 4 == 0, "slot position (t - k) & 3 must be a compile-time constant");
  static_assert((R & (R - 1)) == 0, "slot ring is a power of two");
  static_assert(NPRED % 4 == 0, "predecessor scores are read as float4");
  static_assert(NT <= 1024, "one workgroup per sequence");
};

struct HsArgs {
  const float* lp;      // (B,T,S)
  const float* dur;     // (S,Dm)
  const float* logT;    // (S,S)
  float* Mg;            // (B,T,S): M[t][s], best predecessor total for segments starting at t+1
  float* Dg;            // (B,T,S): Dm[t][s] = max_d delta[t][s][d]
  int* fin;             // (B,2): final (s, d)
  float* scores;        // (B)
  int64_t* states;      // (B,T)
  int B, T, S, Dm;
};

template <int SMAX, int DW>
struct HsLds {
  float dmx[2][SMAX];      // Dm[t][s'] at q(s') = (s' % SUB) * NPRED + s' / SUB: a lane's
                           // predecessors are contiguous
  float lpr[kHsL][SMAX];   // lp row ring; after the last step, the final slot values
  hs_f2 dpair[SMAX][DW];   // dpair[s][c] = {dur[s][(c - NJ) mod R], dur[s][(c - NJ - NJ/2) mod R]}
  int fd[SMAX];
};

constexpr int kHsOOB = 0x7FFFFFF0;  // a buffer offset past every record count: the store is dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hs_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

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
  constexpr int R = G::R, NT = G::NT, NP2 = G::NP2, NPRED = G::NPRED, DW = G::DW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  HsLds<SMAX, DW>& L = *reinterpret_cast<HsLds<SMAX, DW>*>(smem);
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = a.T, S = a.S, Dm = a.Dm;
  const int s = tid / SUB, sub = tid % SUB;
  const bool live = s < S;
  const int q = (s % SUB) * NPRED + s / SUB;
  const float* lp = a.lp + (size_t)b * T * S;
  // Dm / M rows: one lane per state stores (buffer offsets past the records drop the rest)
  const __amdgpu_buffer_rsrc_t dg_r = hs_rsrc(a.Dg + (size_t)b * T * S, (unsigned)T * S * 4u);
  const __amdgpu_buffer_rsrc_t mg_r = hs_rsrc(a.Mg + (size_t)b * T * S, (unsigned)T * S * 4u);
  const int st_off = (live && sub == 0) ? s * 4 : kHsOOB;

  auto dur_at = [&](int r, int age) -> float {  // -inf beyond Dmax and for padding states
    return (r < S && age < Dm) ? a.dur[(size_t)r * Dm + age] : -INFINITY;
  };
  for (int i0 = 0; i0 < SMAX * DW; i0 += 8 * NT) {  // 8 entries per thread in flight
    hs_f2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + k * NT + tid, r = i / DW, c = i % DW;
      v[k] = i < SMAX * DW ? hs_f2{dur_at(r, (c - NJ) & (R - 1)), dur_at(r, (c - NJ - NP2) & (R - 1))}
                           : hs_f2{0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + k * NT + tid;
      if (i < SMAX * DW) L.dpair[i / DW][i % DW] = v[k];
    }
  }
  const float u0 = dur_at(s, 0), u1 = dur_at(s, 1);  // duration terms of d = 1, 2
  hs_f2 lt2[NPRED / 2];  // log T[s'][s] for the lane's predecessors s' = sub + SUB j (-inf: excluded)
#pragma unroll
  for (int j = 0; j < NPRED; ++j) {
    const int sp = sub + SUB * j;
    const bool ok = live && sp < S && sp != s;
    const float v = a.logT[ok ? (size_t)sp * S + s : 0];
    lt2[j >> 1][j & 1] = ok ? v : -INFINITY;
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
  // Gs = completed-group sums, A0 = G0 + tail.  A group's four elements are the state's last
  // four lp values whatever the slot, so they come from one per-lane ring xr (x at time t in
  // xr[t & 3]) when the group closes: G_i += x_{t-3+i} (the same fp32 adds as accumulating
  // each element into its own accumulator as it arrives).  (The leading 0 + a0 of torch's
  // sum is an identity here: a0 is never -0, every accumulator starting from +0.)
  // Durations stay below 72 (hsmm_cfg), so torch's cascade step (tsum.h), which first changes
  // the order at 72 frames, never applies here: a 64..71-frame sum is fl(R + A) with R the last
  // row or two, the same value as A + R.
  hs_f2 Gs[NP2][4], A0[NP2], mp[NP2];
#pragma unroll
  for (int p = 0; p < NP2; ++p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) Gs[p][i] = hs_f2{0.f, 0.f};
    A0[p] = hs_f2{0.f, 0.f};
    mp[p] = hs_f2{-INFINITY, -INFINITY};  // not started: delta = -inf
  }
  hs_f2 xr[4] = {};
  float xcur = 0.f, xnext = 0.f;  // lp[t][s], lp[t+1][s]
  float mxc = -INFINITY, mxn = -INFINITY;  // best delta of the segments of age >= 2 at t, t+1
  float v1c = -INFINITY;   // delta of the segment that started at t-1 (d = 2), ending at t
  float vv[NJ];            // phase B's slot values (the final step's selection)
  bool age1 = false;       // this lane owns the slot of age 1 (started at t-1) at phase B's t
  int Af = 0;
  // phase B's LDS operands, read a step ahead into the buffer of t's parity (NJ is even, so
  // the parity is a compile-time constant of every unrolled copy)
  float xq[2] = {0.f, 0.f};
  hs_f2 duq[2][NP2];
  auto prefetch = [&](const int t, auto Bc) {
    constexpr int B2 = decltype(Bc)::value;
    const int A = (t - NJ * sub) & (R - 1);
    xq[B2] = L.lpr[t % kHsL][s];
    const hs_f2* drow = &L.dpair[s][A + NJ];  // {dur[age_p], dur[age_{p+NP2}]} = drow[-p]
#pragma unroll
    for (int p = 0; p < NP2; ++p) duq[B2][p] = drow[-p];
  };

  // Phase B for end time t (U = t % NJ): every segment of age >= 2 ending at t takes lp[t]
  // into its sums; mxn = their best delta.  It does not depend on M[t-1] or M[t-2], so it
  // runs in the shadow of the predecessor phase of t-1: `mid1` (its predecessor scores)
  // and `mid2` (the group reduction, M, Dm[t-1]'s store) run between pairs of slots, fenced
  // so that the in-order issue fills their LDS and DPP latencies with slot work.
  // Lane `sub` owns slots k = NJ*sub + j, so the new element's position in its segment's
  // group of four, (t - k) & 3 = (U - j) & 3, is a compile-time constant of the unrolled
  // copy; the slot of age 0 at t is j = U (iff A == U) and the one of age 1 is j = U - 1 mod NJ.
  auto phase_b = [&](const int t, auto Uc, auto&& mid1, auto&& mid2) {
    constexpr int U = decltype(Uc)::value;
    constexpr int J1 = (U + NJ - 1) % NJ;
    const int A = (t - NJ * sub) & (R - 1);
    const float x = xq[U & 1];
    age1 = ((A - J1) & (R - 1)) == 1;
    {
      // the segment that started at t-1: sums restart from lp[t-1] (its M is set by the
      // predecessor phase of t-1, before its first use at t+1)
      constexpr int p1 = J1 % NP2, h1 = J1 / NP2;
#pragma unroll
      for (int i = 0; i < 4; ++i) Gs[p1][i][h1] = age1 ? 0.f : Gs[p1][i][h1];
      A0[p1][h1] = age1 ? xcur : A0[p1][h1];
    }
    xnext = x;
    const hs_f2 x2 = {x, x};
    xr[U & 3] = x2;
    float mx = -INFINITY;
    static_for<0, NP2>([&](auto Pc) {
      constexpr int p = decltype(Pc)::value;
      if constexpr (p == NP2 / 2) {
        __builtin_amdgcn_sched_barrier(0);
        mid1();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (p == (3 * NP2) / 4) {
        __builtin_amdgcn_sched_barrier(0);
        mid2();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (kAbl & (1 << 21)) {  // ablation: no slot work (timing only)
        vv[p] = vv[p + NP2] = x;
        mx = fmaxf(mx, x);
        return;
      }
      constexpr int pa = (U - p + 4 * NJ) & 3, pb = (U - p - NP2 + 4 * NJ) & 3;
      if constexpr (pa == pb) {
        if constexpr (pa == 0) {
          A0[p] = Gs[p][0] + x2;
        } else if constexpr (pa == 3) {
#pragma unroll
          for (int i = 0; i < 4; ++i) Gs[p][i] = Gs[p][i] + xr[(U + 1 + i) & 3];
        } else {
          A0[p] = A0[p] + x2;
        }
      } else {
        static_for<0, 2>([&](auto Hc) {
          constexpr int h = decltype(Hc)::value;
          constexpr int ps = h ? pb : pa;
          if constexpr (ps == 0) {
            A0[p][h] = Gs[p][0][h] + x;
          } else if constexpr (ps == 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) Gs[p][i][h] = Gs[p][i][h] + xr[(U + 1 + i) & 3][0];
          } else {
            A0[p][h] = A0[p][h] + x;
          }
        });
      }
      hs_f2 a0;
      if constexpr (pa == 3 && pb == 3) {
        a0 = Gs[p][0];  // the group just closed: empty tail
      } else if constexpr (pa != 3 && pb != 3) {
        a0 = A0[p];
      } else {
        a0 = hs_f2{pa == 3 ? Gs[p][0].x : A0[p].x, pb == 3 ? Gs[p][0].y : A0[p].y};
      }
      const hs_f2 o = ((a0 + Gs[p][1]) + Gs[p][2]) + Gs[p][3];
      // hsmm.py:304-314: fl(fl(M + o) + u); mp == -inf (no predecessor path) gives -inf
      hs_f2 v = (mp[p] + o) + duq[U & 1][p];
      if constexpr (p == U % NP2) v[U / NP2] = A == U ? -INFINITY : v[U / NP2];  // age 0
      if constexpr (p == J1 % NP2) v[J1 / NP2] = age1 ? -INFINITY : v[J1 / NP2];  // age 1
      vv[p] = v.x;
      vv[p + NP2] = v.y;
      mx = fmaxf(mx, fmaxf(v.x, v.y));
    });
    mxn = grp_max<SUB>(mx);
    Af = A;
  };

  // The predecessor phase of end time t: M[t-1] (0 at t = 0: the segment starting at 0 is
  // o + u, hsmm.py:269-274), then the segments of age 0 and 1 (their deltas
  // fl(fl(M + o) + dur) are the same in every lane of the group) and Dm[t].
  float M = 0.f, v0 = -INFINITY, dmt = -INFINITY, lm = -INFINITY;
  auto chain1 = [&](const float4 (&dq)[NPRED / 4]) {
    // M[t-1][s] = max_{s' != s} fl(Dm[t-1][s'] + logT[s'][s]) (the first s' attaining it is
    // recovered by the backtrace from the stored Dm row, for the path's segments only)
    lm = -INFINITY;
    if constexpr (kAbl & (1 << 20)) {  // ablation: no predecessor scores (timing only)
      lm = lt2[0][0];
      return;
    }
#pragma unroll
    for (int i = 0; i < NPRED / 4; ++i) {
      // lt == -inf (excluded s') or dm == -inf: the sum is -inf (never +inf: no NaN)
      const hs_f2 c0 = hs_f2{dq[i].x, dq[i].y} + lt2[2 * i];
      const hs_f2 c1 = hs_f2{dq[i].z, dq[i].w} + lt2[2 * i + 1];
      lm = fmaxf(lm, fmaxf(c0.x, c0.y));
      lm = fmaxf(lm, fmaxf(c1.x, c1.y));
    }
  };
  auto chain2 = [&](const int t) {
    M = t > 0 ? grp_max<SUB>(lm) : 0.f;  // (t = 0 read an unwritten row: discarded)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, M), mg_r, t > 0 ? st_off : kHsOOB,
                                          (t - 1) * S * 4, 0);
    v0 = (M + xcur) + u0;
    dmt = fmaxf(fmaxf(mxc, v1c), v0);
    L.dmx[t & 1][q] = dmt;  // every lane of the group: the same value; -inf for padding states
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dmt), dg_r, st_off, t * S * 4, 0);
  };
  auto read_dq = [&](const int t, float4 (&dq)[NPRED / 4]) {
    if constexpr (kAbl & (1 << 20)) return;
    const float4* dp = reinterpret_cast<const float4*>(&L.dmx[(t - 1) & 1][sub * NPRED]);
#pragma unroll
    for (int i = 0; i < NPRED / 4; ++i) dq[i] = dp[i];
  };

  prefetch(0, std::integral_constant<int, 0>{});
  phase_b(0, std::integral_constant<int, 0>{}, [] {}, [] {});
  xcur = xnext;
  mxc = mxn;
  if (T > 1) prefetch(1, std::integral_constant<int, 1>{});
  // End times t < T-1: barrier, the LDS reads (predecessor scores, t+2's operands), phase B
  // of t+1 with the predecessor phase of t between its slot pairs.  One basic block.
  bool go = T > 1;
  for (int t0 = 0; go; t0 += NJ)
    static_for<0, NJ>([&](auto Uc) {
      constexpr int U = decltype(Uc)::value;
      const int t = t0 + U;
      if (!go) return;
      step_barrier();
      float4 dq[NPRED / 4];
      read_dq(t, dq);
      prefetch(t + 2, std::integral_constant<int, U & 1>{});  // in range past T-1: unused
      phase_b(t + 1, std::integral_constant<int, (U + 1) % NJ>{}, [&] { chain1(dq); }, [&] { chain2(t); });
      {
        // the segment that started at t takes M (its slot is j = U, age 1 at t+1)
        constexpr int pf = U % NP2, hf = U / NP2;
        mp[pf][hf] = age1 ? M : mp[pf][hf];
      }
      v1c = (M + (xcur + xnext)) + u1;  // d = 2 at t+1: torch's sum of two elements
      xcur = xnext;
      mxc = mxn;
      if (t + 2 >= T) {
        go = false;
        return;
      }
      if ((t + 3) % 64 == 0) {  // rows of chunk c = (t+3)/64 are first read by the prefetch
        const int cidx = (t + 3) >> 6;  // at t+1, behind the barrier of t+1
        chunk_store(cidx);
        if ((cidx + 1) * 64 < T) chunk_load(cidx + 1);
      }
    });
  // the last end time: its predecessor phase, then the best over (s asc, d asc) of
  // delta[T-1][s][d-1], strict > (hsmm.py:319-329): d = 1 and d = 2 (ages 0 and 1) first
  {
    const int t = T - 1;
    step_barrier();
    float4 dq[NPRED / 4];
    read_dq(t, dq);
    chain1(dq);
    chain2(t);
    int ld = 0x7fff;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int d = ((Af - j) & (R - 1)) + 1;
      if (vv[j] == dmt && d < ld) ld = d;
    }
    if (v1c == dmt) ld = 2;
    if (v0 == dmt) ld = 1;
    ld = grp_min_i<SUB>(ld);
    if (live && sub == 0) L.fd[s] = ld;
    __syncthreads();
    if (tid < 64) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < (SMAX + 63) / 64; ++k) {
        const int ss = tid + 64 * k;
        if (ss < S) argmax_combine(bv, bi, L.dmx[t & 1][(ss % SUB) * NPRED + ss / SUB], ss);
      }
      wave_argmax(bv, bi);
      if (tid == 0) {
        const bool any = bv != -INFINITY;
        a.scores[b] = bv;
        a.fin[2 * b] = any ? bi : 0;
        a.fin[2 * b + 1] = any ? L.fd[bi] : 1;
      }
    }
  }
}

// torch-order sum of the d elements col[d-1-e], e = 0..d-1 (a segment's column in time
// order, staged newest-first in LDS)
__device__ __forceinline__ float hs_obs_sum_lds(const float* col, int d) {
  return tsum_strided([&](int i) { return col[d - 1 - i]; }, d);
}

// The segment walker of the backtrace (hsmm.py:331-352), one wave.  R >= the longest
// duration; every lane owns the candidates d' = l + 1 + 64k, k < R/64, and the predecessor
// states s' = l + 64k, k < SMAX/64.  LDS: dur (S, Dm), logT (S, S), the predecessor's
// candidate column lp[tau - e][s1], e < Dm, and the tie path's columns.
struct HsWalk {
  const float* lp;  // this sequence's (T, S) rows
  const float* Mb;
  const float* Db;
  float* sdur;
  float* slt;
  float* pcol;
  float* rcol;  // tie path: lp[tau - e][s'], (e, s' mod 64)
  float* rmc;   //           M[tau - e - 1][s']
  int T, S, Dm;
};

// torch-order sum of lp[t0 .. t0+d-1][s] by one wave (d <= 128): the column is staged in
// `scratch` with all its loads in flight, then summed from LDS (a loop over global loads
// waits for each group of four in turn)
__device__ float hs_obs_sum_wave(const float* lp, int S, int t0, int d, int s, float* scratch, int l) {
  float v[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = l + 64 * k;
    v[k] = e < d ? lp[(size_t)(t0 + d - 1 - e) * S + s] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (l + 64 * k < d) scratch[l + 64 * k] = v[k];
  __syncthreads();
  const float r = hs_obs_sum_lds(scratch, d);
  __syncthreads();
  return r;
}

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline size_t hsmm_walk_lds(int S, int Dm, int R) {
  return (size_t)(S * Dm + S * S + R + 2 * 64 * Dm) * sizeof(float);
}

// global -> LDS copy by one wave, 16 loads per lane in flight (a plain strided loop waits
// for each load before the next: one round trip per 64 values)
// (indices past n are clamped to n - 1, which rewrites that entry with its own value: no
// branch per load or store)
__device__ __forceinline__ void hs_copy_lds(float* dst, const float* src, int n, int l) {
  for (int i0 = 0; i0 < n; i0 += 64 * 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = i0 + 64 * k + l;
      v[k] = src[i < n ? i : n - 1];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = i0 + 64 * k + l;
      dst[i < n ? i : n - 1] = v[k];
    }
  }
}

// tables into LDS (the caller's barrier publishes them); copy = false: the pointers only (the
// stitch copies the tables when it first has to walk itself, hs_walk_tables)
template <int R>
__device__ HsWalk hs_walk_init(const HsArgs& a, char* bsm, int b, int l, bool copy = true) {
  HsWalk w;
  w.T = a.T;
  w.S = a.S;
  w.Dm = a.Dm;
  const size_t off = (size_t)b * a.T * a.S;
  w.lp = a.lp + off;
  w.Mb = a.Mg + off;
  w.Db = a.Dg + off;
  w.sdur = reinterpret_cast<float*>(bsm);
  w.slt = w.sdur + a.S * a.Dm;
  w.pcol = w.slt + a.S * a.S;
  w.rcol = w.pcol + R;
  w.rmc = w.rcol + 64 * a.Dm;
  if (copy) {
    hs_copy_lds(w.sdur, a.dur, a.S * a.Dm, l);
    hs_copy_lds(w.slt, a.logT, a.S * a.S, l);
  }
  return w;
}
__device__ __forceinline__ void hs_walk_tables(const HsArgs& a, const HsWalk& w, int l) {
  hs_copy_lds(w.sdur, a.dur, a.S * a.Dm, l);
  hs_copy_lds(w.slt, a.logT, a.S * a.S, l);
}

#ifdef HMM355_HSMM_STAMP
// diagnostic: walker cycles per phase summed over every segment of every chunk walk
__device__ unsigned long long g_hs_stamp[8];
// (accumulated in registers, one atomic per phase when the walk returns: an atomic per phase
// and segment would put its completion on the next load's wait)
struct HsStampAcc {
  long long a[7] = {0, 0, 0, 0, 0, 0, 0};
  bool on;
  int l;
  __device__ ~HsStampAcc() {
    if (on && l == 0)
      for (int k = 0; k < 7; ++k) atomicAdd(&g_hs_stamp[k], (unsigned long long)a[k]);
  }
};
#define HS_STAMP(k) do { const long long _n = clock64(); st_acc.a[k] += _n - st_t; st_t = _n; } while (0)
#else
#define HS_STAMP(k) do { } while (0)
#endif

// Walks from the segment (end t, state cs, duration cd, obs_sum o) towards t = 0, calling
// emit(t, cs, cd, o, start) for every segment in walk order (the first one included); stops
// when emit returns true, or after the first segment that ends below `stop`, starts at 0, or
// has no predecessor.
template <int R, int SMAX, typename Emit>
__device__ void hs_walk(const HsWalk& w, int l, int t, int cs, int cd, float o, int stop, Emit&& emit) {
  constexpr int K = R / 64;
  constexpr int KS = (SMAX + 63) / 64;
  const int S = w.S, Dm = w.Dm;
  const float* lp = w.lp;
  const float* Mb = w.Mb;
  const float* Db = w.Db;
  float* sdur = w.sdur;
  float* slt = w.slt;
  float* pcol = w.pcol;
  float* rcol = w.rcol;
  float* rmc = w.rmc;
#ifdef HMM355_HSMM_STAMP
  HsStampAcc st_acc;
  st_acc.on = stop >= 0;  // chunk walks (and the stitch's own walks)
  st_acc.l = l;
  long long st_t = clock64();
#endif
  while (t >= 0 && cd > 0) {
    int start = t - cd + 1;
    if (start < 0) start = 0;
    if (emit(t, cs, cd, o, start)) return;
    if (start == 0 || t < stop) return;
    HS_STAMP(0);
#ifdef HMM355_HSMM_STAMP
    st_acc.a[6] += 1;
#endif
    const int tau = start - 1;  // end of the previous segment
    // round trip 1: M and the Dm row at tau
    const float M = Mb[(size_t)tau * S + cs];
    float dm[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int sp = l + 64 * k;
      dm[k] = sp < S ? Db[(size_t)tau * S + sp] : -INFINITY;
    }
    int ns = 0, nd = 0;  // literal: psi never written when no predecessor exists (hsmm.py:313)
    float on = 0.f;
    if (M != -INFINITY) {
      // the first s' != cs attaining M: the forward's own candidate values fl(Dm + logT)
      float cv[KS];
      ns = -1;
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int sp = l + 64 * k;
        cv[k] = (sp < S && sp != cs) ? dm[k] + slt[sp * S + cs] : -INFINITY;
        const unsigned long long mask = __ballot(cv[k] == M);
        if (ns < 0 && mask) ns = 64 * k + __ffsll((long long)mask) - 1;
      }
      if (ns < 0) ns = 0;  // unreachable: M is the maximum of these candidates
      HS_STAMP(1);
      const float lt = slt[ns * S + cs];
      float xo = -INFINITY;  // best total of the states before ns
#pragma unroll
      for (int k = 0; k < KS; ++k)
        if (l + 64 * k < ns) xo = fmaxf(xo, cv[k]);
      // round trip 2: ns's candidate column and its candidates' predecessor scores
      const int dlim = Dm < tau + 1 ? Dm : tau + 1;
      float pm[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = l + 64 * k;
        const bool pin = e < dlim;
        const float pv = lp[(size_t)(pin ? tau - e : 0) * S + ns];
        const int pst = tau - e;  // candidate d' = e + 1 starts at tau - e
        pm[k] = (pin && pst >= 1) ? Mb[(size_t)(pst - 1) * S + ns] : 0.f;
        if (pin) pcol[e] = pv;
      }
      __syncthreads();
      HS_STAMP(2);
      // first d' of ns whose fl(delta + logT) equals M, and the best earlier total (xb)
      float dv[K], ov[K];
      nd = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = l + 64 * k;
        dv[k] = -INFINITY;
        ov[k] = 0.f;
        bool hit = false;
        if (e < dlim) {
          ov[k] = hs_obs_sum_lds(pcol, e + 1);
          const float u = sdur[ns * Dm + e];
          const int pst = tau - e;
          dv[k] = pst == 0 ? ov[k] + u : (pm[k] == -INFINITY ? -INFINITY : (pm[k] + ov[k]) + u);
          hit = dv[k] != -INFINITY && dv[k] + lt == M;
        }
        const unsigned long long mask = __ballot(hit);
        if (nd == 0 && mask) nd = 64 * k + __ffsll((long long)mask);  // lane index + 1 = d'
      }
      if (nd == 0) nd = 1;
      HS_STAMP(3);
      float xb = xo;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (l + 64 * k + 1 < nd && dv[k] != -INFINITY) xb = fmaxf(xb, dv[k] + lt);
      xb = wave_max_dpp2(xb);  // (DPP + permlane: no ds_bpermute round trips on the walk)
      // the next segment's obs_sum is candidate nd's
      {
        float ok = ov[0];
#pragma unroll
        for (int k = 1; k < K; ++k) ok = (nd - 1) >> 6 == k ? ov[k] : ok;
        on = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ok), (nd - 1) & 63));
      }
      const float u = sdur[cs * Dm + cd - 1];
      const float F = (M + o) + u;
      if (xb != -INFINITY && (xb + o) + u == F) {
        // rare: an earlier candidate rounds to the same total — the first one wins
        // (hsmm.py:308).  Lane l takes the predecessor state s' = l + 64k: both columns
        // (lp and M, d' <= dlim) are staged for 64 states at once, each lane walks its own
        // d' ascending, and the lowest state with a hit wins.
        int win = ns * Dm + (nd - 1);  // p1 when no earlier candidate hits
        for (int k = 0; 64 * k <= ns; ++k) {
          const int sp = l + 64 * k;
          const bool in = sp < S;
          for (int e0 = 0; e0 < dlim; e0 += 16) {  // 16 loads of each column in flight
            float cv2[16], mv2[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const int e = e0 + j;
              const bool ok = in && e < dlim;
              cv2[j] = ok ? lp[(size_t)(tau - e) * S + sp] : 0.f;
              mv2[j] = (ok && tau - e >= 1) ? Mb[(size_t)(tau - e - 1) * S + sp] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              if (e0 + j < dlim) {
                rcol[(e0 + j) * 64 + l] = cv2[j];
                rmc[(e0 + j) * 64 + l] = mv2[j];
              }
            }
          }
          __syncthreads();
          int first = 0;
          if (in && sp <= ns && sp != cs) {
            const int lim = sp == ns ? nd - 1 : dlim;
            const float ltc = slt[sp * S + cs];
            for (int dp = 1; dp <= lim; ++dp) {
              // delta of (s', d'), exactly as the forward forms it: torch-order sum of the
              // d' elements rcol[e][l], e = d'-1 .. 0 (time order)
              const float oc = tsum_strided([&](int i) { return rcol[(dp - 1 - i) * 64 + l]; }, dp);
              const float uc = sdur[sp * Dm + dp - 1];
              const float mc = rmc[(dp - 1) * 64 + l];
              const float dlt = tau - dp + 1 == 0 ? oc + uc : (mc == -INFINITY ? -INFINITY : (mc + oc) + uc);
              if (dlt != -INFINITY && ((dlt + ltc) + o) + u == F) {
                first = dp;
                break;
              }
            }
          }
          const unsigned long long m2 = __ballot(first > 0);
          if (m2) {
            const int ln = __ffsll((long long)m2) - 1;
            win = (ln + 64 * k) * Dm + __shfl(first, ln) - 1;
            break;
          }
          __syncthreads();  // the columns are restaged for the next 64 states
        }
        ns = win / Dm;
        nd = win % Dm + 1;
        on = hs_obs_sum_wave(lp, S, tau - nd + 1, nd, ns, pcol, l);
      }
      __syncthreads();  // the column is restaged for the next segment
      HS_STAMP(4);
    }
    t = start - 1;
    cs = ns;
    cd = nd;
    o = on;
  }
}

__device__ __forceinline__ void hs_write_states(int64_t* st, int start, int t, int cs, int l) {
  for (int u = start + l; u <= t; u += 64) st[u] = cs;
}

// the serial backtrace: one wave walks the whole sequence from the final segment
template <int R, int SMAX>
__global__ void __launch_bounds__(64) hsmm_backtrace_kernel(HsArgs a) {
  extern __shared__ __attribute__((aligned(16))) char bsm[];
  const int b = blockIdx.x, l = threadIdx.x;
  const HsWalk w = hs_walk_init<R>(a, bsm, b, l);
  const int T = a.T, cs = a.fin[2 * b], cd = a.fin[2 * b + 1];
  const float o = hs_obs_sum_wave(w.lp, a.S, T - cd, cd, cs, w.pcol, l);
  int64_t* st = a.states + (size_t)b * T;
  hs_walk<R, SMAX>(w, l, T - 1, cs, cd, o, -1, [&](int t, int s, int, float, int start) {
    hs_write_states(st, start, t, s, l);
    return false;
  });
}

// ---- chunked backtrace: the walk is one dependent chain of segments (≈ 1-2 µs each), so
// it is cut into time chunks of kHsChunk frames walked in parallel and stitched exactly.
// hsmm_chunk_walk_kernel: chunk c's wave walks from a guessed segment 128 frames above
//   the chunk (the best state ending there, d = 1; the true final segment for the top
//   chunks) down to the first segment ending below c * kHsChunk, recording every segment.
//   Walks from different segments merge quickly (the backpointers coalesce).
// hsmm_stitch_kernel: one wave per sequence runs the chunks top-down with the true segment
//   entering each chunk: found in the chunk's record, the record from there IS the true
//   path (the walk is a deterministic function of the segment, its tie resolution included);
//   not found (the guessed walk had not merged yet), the true walk continues serially until
//   it meets the record or leaves the chunk.  Either way the result is the serial walk's, bit
//   for bit.  (Warm-up 64 / 128 / 192 frames: the same within 1 % at config 5,
//   profiles/r3u_warm.log.)
constexpr int kHsChunk = 64;
constexpr int kHsWarmMax = 256;
inline int hsmm_warm() {  // frames walked above a chunk before it
#ifdef HMM355_DIAG
  const char* e = getenv("HMM355_HSMM_WARM");  // (diagnostic builds only)
  const int w = e ? atoi(e) : 128;
  return w < 0 ? 0 : (w > kHsWarmMax ? kHsWarmMax : w);
#else
  return 128;
#endif
}
constexpr int kHsCap = kHsChunk + kHsWarmMax + 2;  // segments per record (each >= 1 frame)
struct HsChunks {
  int4* rec;  // (B, C, kHsCap): {end, state, duration, obs_sum bits}
  int* cnt;   // (B, C)
  int C;
  int warm;
  int stage;  // chunks whose first 64 records the stitch stages in LDS (the top ones)
};

template <int R, int SMAX>
__global__ void __launch_bounds__(64) hsmm_chunk_walk_kernel(HsArgs a, HsChunks c) {
  extern __shared__ __attribute__((aligned(16))) char bsm[];
  const int ch = blockIdx.x, b = blockIdx.y, l = threadIdx.x;
  const int T = a.T, S = a.S;
  const HsWalk w = hs_walk_init<R>(a, bsm, b, l);
  const int t0 = min(T - 1, (ch + 1) * kHsChunk + c.warm - 1);
  int cs, cd;
  if (t0 == T - 1) {
    cs = a.fin[2 * b];
    cd = a.fin[2 * b + 1];
  } else {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < (SMAX + 63) / 64; ++k) {
      const int sp = l + 64 * k;
      if (sp < S) argmax_combine(bv, bi, w.Db[(size_t)t0 * S + sp], sp);
    }
    wave_argmax_dpp(bv, bi);
    cs = bi < S ? bi : 0;
    cd = 1;
  }
  const float o = hs_obs_sum_wave(w.lp, S, t0 - cd + 1, cd, cs, w.pcol, l);
  // the record is kept in LDS during the walk (a global store per segment would put its
  // completion on the walk's next load) and written out at the end
  int4* lrec = reinterpret_cast<int4*>(bsm + align16(hsmm_walk_lds(S, a.Dm, R)));
  int n = 0;
  hs_walk<R, SMAX>(w, l, t0, cs, cd, o, ch * kHsChunk, [&](int t, int s, int d, float ob, int) {
    if (l == 0 && n < kHsCap) lrec[n] = make_int4(t, s, d, __float_as_int(ob));
    ++n;
    return false;
  });
  n = n < kHsCap ? n : kHsCap;
  __syncthreads();
  int4* rec = c.rec + ((size_t)b * c.C + ch) * kHsCap;
  for (int j = l; j < n; j += 64) rec[j] = lrec[j];
  if (l == 0) c.cnt[(size_t)b * c.C + ch] = n;
}


template <int R, int SMAX>
__global__ void __launch_bounds__(64) hsmm_stitch_kernel(HsArgs a, HsChunks c) {
  extern __shared__ __attribute__((aligned(16))) char bsm[];
  const int b = blockIdx.x, l = threadIdx.x;
  const int T = a.T;
  // the walker's tables are copied only if the stitch has to walk itself (records usually merge)
#ifdef HMM355_HSMM_STAMP
  const long long st0 = clock64();
#endif
  const HsWalk w = hs_walk_init<R>(a, bsm, b, l, false);
  bool tables = false;
  // after the walker's tables: the first 64 records of the top kHsStage chunks, their counts
  int4* srec = reinterpret_cast<int4*>(bsm + align16(hsmm_walk_lds(a.S, a.Dm, R)));
  int* scnt = reinterpret_cast<int*>(srec + c.stage * 64);
  const int4* recb = c.rec + (size_t)b * c.C * kHsCap;
  const int* cntb = c.cnt + (size_t)b * c.C;
  const int c0 = c.C - c.stage;  // staged: chunks c0 .. C-1
  // independent loads (entries past a record's count are read but never used), 16 chunks' entries
  // in flight at a time: a plain loop waits for each load before its LDS store, one round trip per
  // chunk (round 4: 32 serial round trips at config 5, most of the stitch's 68 us)
  for (int ch0 = c0; ch0 < c.C; ch0 += 16) {
    int4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      v[k] = ch0 + k < c.C ? recb[(size_t)(ch0 + k) * kHsCap + l] : make_int4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (ch0 + k < c.C) srec[(ch0 + k - c0) * 64 + l] = v[k];
  }
  for (int k = l; k < c.stage; k += 64) scnt[k] = cntb[c0 + k];
  int t = T - 1, cs = a.fin[2 * b], cd = a.fin[2 * b + 1];
  float o = hs_obs_sum_wave(w.lp, a.S, T - cd, cd, cs, w.pcol, l);
  int64_t* st = a.states + (size_t)b * T;
#ifdef HMM355_HSMM_STAMP
  if (l == 0) atomicAdd(&g_hs_stamp[7], (unsigned long long)(clock64() - st0));
#endif
  // Records come from LDS (staged, n <= 64) or from global memory, never both in one loop:
  // a load that may come from either makes the compiler wait for every outstanding global
  // operation at the join, the state stores included.
  auto from_lds = [&](int ch) { return [&, ch](int j) { return srec[(ch - c0) * 64 + j]; }; };
  auto from_glb = [&](int ch) { return [&, ch](int j) { return recb[(size_t)ch * kHsCap + j]; }; };
  bool done = false;
  int serial = 0;  // segments the stitch walked itself (diagnostic count, after the chunk counts)
  // the true segment (t, cs, cd) in chunk ch's record (n entries): its index, or -1
  auto find = [&](auto&& rd, int n) -> int {
    for (int base = 0; base < n; base += 64) {
      const int4 e = base + l < n ? rd(base + l) : make_int4(-1, -1, -1, 0);
      const unsigned long long m = __ballot(e.x == t && e.y == cs && e.z == cd);
      if (m) return base + __ffsll((long long)m) - 1;
    }
    return -1;
  };
  // the record from index j on is the true path: write it down to the next chunk's entry
  auto follow = [&](auto&& rd, int j, int n, int lo) {
    for (;; ++j) {
      if (j >= n) {  // the walk ended (no predecessor): nothing below is written
        done = true;
        return;
      }
      const int4 e = rd(j);  // the same address in every lane: a broadcast
      if (e.x < lo) {  // enters the next chunk down
        t = e.x;
        cs = e.y;
        cd = e.z;
        o = __int_as_float(e.w);
        return;
      }
      const int start = e.x - e.z + 1 < 0 ? 0 : e.x - e.z + 1;
      hs_write_states(st, start, e.x, e.y, l);
      if (start == 0) {
        done = true;
        return;
      }
    }
  };
  for (int ch = c.C - 1; ch >= 0 && !done; --ch) {
    const int lo = ch * kHsChunk;
    const bool lds = ch >= c0 && scnt[ch - c0] <= 64;
    const int n = ch >= c0 ? scnt[ch - c0] : cntb[ch];
    int at = lds ? find(from_lds(ch), n) : find(from_glb(ch), n);
    if (at < 0) {
      // not merged: walk serially from the true segment until it meets the record's first
      // 64 segments (then the record is the true path from there) or leaves the chunk
      bool below = false;
      const int4 e0 = l < n ? (lds ? srec[(ch - c0) * 64 + l] : recb[(size_t)ch * kHsCap + l])
                            : make_int4(-1, -1, -1, 0);
      if (!tables) {  // (uniform: `at` comes from a ballot)
        hs_walk_tables(a, w, l);
        __syncthreads();  // every lane reads entries other lanes wrote
        tables = true;
      }
      hs_walk<R, SMAX>(w, l, t, cs, cd, o, lo, [&](int et, int es, int ed, float eo, int start) {
        ++serial;
        if (et < lo) {
          t = et;
          cs = es;
          cd = ed;
          o = eo;
          below = true;
          return true;
        }
        const unsigned long long m = __ballot(e0.x == et && e0.y == es && e0.z == ed);
        if (m) {
          at = __ffsll((long long)m) - 1;
          return true;
        }
        hs_write_states(st, start, et, es, l);
        return false;
      });
      if (at < 0 && !below) done = true;
    }
    if (at >= 0) {
      if (lds)
        follow(from_lds(ch), at, n, lo);
      else
        follow(from_glb(ch), at, n, lo);
    }
  }
  if (l == 0) c.cnt[(size_t)a.B * c.C + b] = serial;
#ifdef HMM355_HSMM_STAMP
  if (l == 0) atomicAdd(&g_hs_stamp[5], (unsigned long long)(clock64() - st0));
#endif
}

// Geometries (S <= SMAX, Dmax < R).  The config-5 class S <= 64, Dmax <= 63 takes the
// 4-lane form (256 threads: one wave per SIMD, 16 slots per lane; 0.81 ms at config 5 vs 0.83
// for 8 lanes and 1.00 for 16, profiles/r3q_c5_sub*.log: those two geometries were removed in
// round 6).  The larger geometries run 512 threads (8 waves) so a lane has 256 VGPRs for its
// 16 slots.  (S <= 128 with 64 <= Dmax <= 127 would need 32 slots per lane: beyond the register
// file; rejected.)
enum HsCfg : int { kHs8x16 = 2, kHs4x16 = 3, kHs4x16s64 = 4, kHsNone = -1 };
inline int hsmm_cfg(int S, int Dm) {
  if (S < 1 || Dm < 1) return kHsNone;
  if (S <= 64 && Dm < 64) return kHs4x16s64;
  // Dm <= 71: from 72 frames on torch's cascade step changes the segment-sum order (tsum.h);
  // its extra per-slot accumulators do not fit this geometry's registers (measured: 189 VGPRs
  // spilled), so longer durations take the general form (hsmm_wide.hip), which has it
  if (S <= 64 && Dm <= kHsRegDMax) return kHs8x16;
  if (S <= 128 && Dm < 64) return kHs4x16;
  return kHsNone;
}

inline int hsmm_chunks(int T) { return (T + kHsChunk - 1) / kHsChunk; }
// the chunked backtrace from 3 chunks up (HMM355_FORM_SERIAL_WALK: always the serial walk)
inline bool hsmm_use_chunks(int T, unsigned flags) {
  return hsmm_chunks(T) >= 3 && !(flags & HMM355_FORM_SERIAL_WALK);
}

template <int SUB, int NJ, int SMAX>
static hipError_t launch_hsmm(const HsArgs& ha, const HsChunks& hc, unsigned flags, hipStream_t st) {
  using G = HsG<SUB, NJ, SMAX>;
  const size_t lds = sizeof(HsLds<SMAX, G::DW>);
  hipError_t e = allow_lds(hsmm_fwd_kernel<SUB, NJ, SMAX>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((hsmm_fwd_kernel<SUB, NJ, SMAX>), dim3(ha.B), dim3(G::NT), lds, st, ha);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if constexpr (kAbl & (1 << 22)) return hipSuccess;  // ablation: forward only (timing)
  const size_t blds = hsmm_walk_lds(ha.S, ha.Dm, G::R);
  if (hsmm_use_chunks(ha.T, flags)) {
    const size_t wlds = align16(blds) + kHsCap * sizeof(int4);
    if ((e = allow_lds(hsmm_chunk_walk_kernel<G::R, SMAX>, wlds)) != hipSuccess) return e;
    HsChunks hs = hc;
    const long room = 163840 - (long)align16(blds) - 16;
    hs.stage = (int)std::min<long>(hc.C, std::max<long>(0, room / (long)(64 * sizeof(int4) + sizeof(int))));
    const size_t slds = align16(blds) + hs.stage * 64 * sizeof(int4) + hs.stage * sizeof(int);
    if ((e = allow_lds(hsmm_stitch_kernel<G::R, SMAX>, slds)) != hipSuccess) return e;
    hipLaunchKernelGGL((hsmm_chunk_walk_kernel<G::R, SMAX>), dim3(hc.C, ha.B), dim3(64), wlds, st, ha, hc);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((hsmm_stitch_kernel<G::R, SMAX>), dim3(ha.B), dim3(64), slds, st, ha, hs);
    return hipGetLastError();
  }
  e = allow_lds(hsmm_backtrace_kernel<G::R, SMAX>, blds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((hsmm_backtrace_kernel<G::R, SMAX>), dim3(ha.B), dim3(64), blds, st, ha);
  return hipGetLastError();
}

// One state (S = 1): the reference skips every s' == s candidate, so only the segment that
// starts at 0 and ends at T-1 can score: delta = fl(sum(lp[0:T]) + dur[T-1]) when T <= Dmax,
// else -inf (hsmm.py:266-329).  obs_log_probs[b] is (T, 1), so that slice is CONTIGUOUS and
// torch.sum takes its vectorised order (tsum.h tsum_contig).  The path is all zeros (the
// reference's torch.zeros states; with a -inf score its walk does not terminate when T > 1).
__global__ void __launch_bounds__(64) hsmm_single_state_kernel(HsArgs a) {
  const int b = blockIdx.x, l = threadIdx.x, T = a.T;
  int64_t* st = a.states + (size_t)b * T;
  for (int u = l; u < T; u += 64) st[u] = 0;
  if (l == 0) {
    const float* x = a.lp + (size_t)b * T;
    a.scores[b] = T <= a.Dm ? tsum_contig([&](int i) { return x[i]; }, T) + a.dur[T - 1] : -INFINITY;
  }
}

// hsmm_wide.hip: the general form for sizes the register-slot geometries cannot hold
size_t hsmm_wide_workspace_bytes(int B, int T, int S, int Dm);
bool hsmm_wide_fits(int S, int Dm);
hipError_t launch_hsmm_wide(const float* lp, const float* dur, const float* logT, int B, int T, int S, int Dm,
                            int64_t* states, float* scores, void* workspace, hipStream_t st);
// HMM355_FORM_GENERAL takes the general form for every size (tests / comparison)
inline bool hsmm_wide(int S, int Dm, unsigned flags) {
  return hsmm_wide_fits(S, Dm) && (hsmm_cfg(S, Dm) == kHsNone || (flags & HMM355_FORM_GENERAL));
}

}  // namespace hmm355

using namespace hmm355;

#ifdef HMM355_HSMM_STAMP
// diagnostic export: read and clear the walker phase counters (8 values)
HMM355_API int hmm355_diag_hsmm_stamp(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hs_stamp), 8 * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_hs_stamp), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
#endif

HMM355_API size_t hmm355_hsmm_workspace_bytes_ex(int B, int T, int S, int Dmax, unsigned flags) {
  if (B < 0 || T < 1) return 0;
  if (hsmm_wide(S, Dmax, flags)) return hsmm_wide_workspace_bytes(B, T, S, Dmax);
  if (hsmm_cfg(S, Dmax) == kHsNone) return 0;
  const size_t n = (size_t)B * T * S, nc = (size_t)B * hsmm_chunks(T);
  return 2 * align_up(n * 4, 256) + align_up((size_t)B * 8, 256) + align_up(nc * kHsCap * sizeof(int4), 256) +
         align_up((nc + B) * 4, 256);
}

HMM355_API size_t hmm355_hsmm_workspace_bytes(int B, int T, int S, int Dmax) {
  return hmm355_hsmm_workspace_bytes_ex(B, T, S, Dmax, 0u);
}

HMM355_API int hmm355_hsmm_viterbi_ex_f32(const float* lp, const float* dur_lp, const float* log_T, int B, int T,
                                          int S, int Dmax, unsigned flags, int64_t* states, float* scores,
                                          void* workspace, size_t workspace_bytes, void* stream) {
  if (flags & ~(HMM355_FORM_GENERAL | HMM355_FORM_SERIAL_WALK)) return HMM355_E_ARG;
  if (B < 0 || S < 0 || Dmax < 0) return HMM355_E_ARG;
  if (S < 1 || S > 1024) return HMM355_E_STATES;
  if (Dmax < 1 || Dmax > 1024) return HMM355_E_DURATION;
  if (T < 1) return HMM355_E_SHAPE;
  if (B == 0) return HMM355_OK;
  if (!lp || !dur_lp || !log_T || !states || !scores || !workspace) return HMM355_E_ARG;
  if ((size_t)B * T * S * Dmax > ((size_t)1 << 40)) return HMM355_E_SHAPE;
  if (workspace_bytes < hmm355_hsmm_workspace_bytes_ex(B, T, S, Dmax, flags)) return HMM355_E_WORKSPACE;
  if (hsmm_wide(S, Dmax, flags) && S > 1) {
    const hipError_t e = launch_hsmm_wide(lp, dur_lp, log_T, B, T, S, Dmax, states, scores, workspace,
                                          static_cast<hipStream_t>(stream));
    return e == hipSuccess ? HMM355_OK : (int)e;
  }
  const size_t n = (size_t)B * T * S;
  char* ws = static_cast<char*>(workspace);
  float* Mg = reinterpret_cast<float*>(ws);
  float* Dg = reinterpret_cast<float*>(ws + align_up(n * 4, 256));
  int* fin = reinterpret_cast<int*>(ws + 2 * align_up(n * 4, 256));
  const size_t nc = (size_t)B * hsmm_chunks(T);
  int4* rec = reinterpret_cast<int4*>(ws + 2 * align_up(n * 4, 256) + align_up((size_t)B * 8, 256));
  int* cnt = reinterpret_cast<int*>(reinterpret_cast<char*>(rec) + align_up(nc * kHsCap * sizeof(int4), 256));
  HsArgs ha{lp, dur_lp, log_T, Mg, Dg, fin, scores, states, B, T, S, Dmax};
  HsChunks hc{rec, cnt, hsmm_chunks(T), hsmm_warm(), 0};
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (S == 1) {
    hipLaunchKernelGGL(hsmm_single_state_kernel, dim3(B), dim3(64), 0, st, ha);
    e = hipGetLastError();
    return e == hipSuccess ? HMM355_OK : (int)e;
  }
  // frames the walk never reaches (a segment without a predecessor path ends it) keep the
  // reference's torch.zeros initial value (hsmm.py:332)
  if ((e = hipMemsetAsync(states, 0, (size_t)B * T * sizeof(int64_t), st)) != hipSuccess) return (int)e;
  switch (hsmm_cfg(S, Dmax)) {
    case kHs4x16s64: e = launch_hsmm<4, 16, 64>(ha, hc, flags, st); break;
    case kHs8x16: e = launch_hsmm<8, 16, 64>(ha, hc, flags, st); break;
    default: e = launch_hsmm<4, 16, 128>(ha, hc, flags, st); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_hsmm_viterbi_f32(const float* lp, const float* dur_lp, const float* log_T, int B, int T,
                                       int S, int Dmax, int64_t* states, float* scores, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  return hmm355_hsmm_viterbi_ex_f32(lp, dur_lp, log_T, B, T, S, Dmax, 0u, states, scores, workspace,
                                    workspace_bytes, stream);
}
