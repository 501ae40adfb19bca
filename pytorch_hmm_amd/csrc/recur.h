// hmm355 — the serial recursion shared by forward-backward and Viterbi (gfx950).
//
// One workgroup runs one chain (a sequence's forward pass, backward pass, or Viterbi
// max-plus pass) over T steps.  The chain is latency-bound (T dependent steps of an
// NP x NP reduction), so the layout minimises the per-step critical path and the LDS
// instruction count:
//
//   * NW = NP/16 waves; wave w owns outputs o = 16w + c (c = lane & 15); the lane's row
//     r = lane >> 4 owns the inputs i = 64*blk + 16r + n.  Its matrix slice lives in VGPRs.
//   * The previous vector is held one value per lane (input 64*blk + lane), so DPP
//     row_newbcast folded into v_fmac_f32_dpp / v_add_f32_dpp feeds every product from a
//     register: the inner loop has no LDS traffic.
//   * The four row groups' partial results for each output are halved in-register by one
//     v_permlane32_swap (rows {0,2} and {1,3}); lanes 0..31 write the two halves as a
//     float2 per output (conflict-free ds_write_b32).  After the step's single s_barrier
//     every lane reads each of its inputs' float2 with one conflict-free ds_read_b64 (the
//     LDS cycles per step, not only the latency, bound the exchange: 8 waves x NBLK x 2).
//   * Forward-backward runs in the probability domain with Rabiner scaling: the scale of
//     step q is 1/c_{q-1} (c = sum of the previous vector, a DPP wave sum beside the FMAs)
//     and is folded, with the emission, into the partials before they are written.
//     Viterbi adds the log-emission to each partial max (fl(max + lo) == max(fl(x + lo)),
//     so the result is still the bit-exact delta).  log-scales accumulate at flush time.
//   * Emissions are staged 16 steps at a time through a 3-slot LDS ring (global loads issued
//     two blocks ahead); finished rows sit in a 64-row LDS ring and leave as 16-B stores once
//     per 16 steps.  The loop body issues no per-step global memory operation.
//   * The workgroup requests all 160 KiB of LDS so it owns its CU (no co-resident
//     workgroup of a concurrent kernel steals issue slots from the chain).
#pragma once
#include "band.h"
#include "common.h"
#include "logcr.h"

namespace hmm355 {

enum RecKind : int { kFbAlpha = 0, kFbBeta = 1, kVit = 2 };

// diagnostic builds (HMM355_STAMP=1): per wave [gather, compute, write-wait, barrier, steps,
// total cycles, memtime, memrealtime] summed over the steps (tools/stamps.py)
constexpr int kStampWaves = 512 * 16;
static __device__ unsigned long long g_rec_stamps[kStamp ? kStampWaves * 8 : 1];

template <int NP>
struct RC {
  static constexpr int NW = NP / 16;     // waves
  static constexpr int NT = NW * kWave;  // threads
  static constexpr int NBLK = NP / 64;   // 64-input blocks per lane
  static constexpr int RING = 64;        // stored-row ring
  static constexpr int OFF_PART = 0;                       // [2][NP][2] half-wave partials
  static constexpr int OFF_EMIS = OFF_PART + 2 * NP * 2;   // [3][16][NP]
  static constexpr int OFF_RING = OFF_EMIS + 3 * 16 * NP;  // [RING][NP]
  static constexpr int OFF_SC = OFF_RING + RING * NP;      // [RING][64] normalisers c_rho (entry 0;
                                                           // the banded chain writes all 64 lanes)
  static constexpr int OFF_M = OFF_SC + RING * 64;        // [128] OBS_LOG FB: staged row maxima (0 else)
  static constexpr int MRING = 128;                        // rows kb-3 .. kb+1 live at once
  static constexpr int OFF_LOGT = OFF_M + MRING;           // [256] doubles: Viterbi log table (logcr.h)
  static constexpr int LDS_FLOATS = OFF_LOGT + 512;
  static_assert(LDS_FLOATS * 4 <= kExclusiveLds, "LDS layout too large");
  // fused-psi Viterbi (kVitFused; the chain kernel owns all 160 KiB): the psi rows of the last
  // 64 steps (bytes [64][NP]), written by the psi waves, copied to HBM by the staging helpers
  static constexpr int PSR = 64;
  static constexpr int OFF_PSR = LDS_FLOATS;
  static_assert((OFF_PSR + PSR * NP / 4) * 4 <= kExclusiveLds, "fused Viterbi LDS layout too large");
};

// threads of a launch that may run the register-blocked dense chain (rec_run_rb, NP <= 128):
// its NW chain waves plus NH block-work helper waves (rec_rb_helper)
template <int NP>
struct kRbHelpers {
  static constexpr int NH = NP <= 128 ? RC<NP>::NW / 2 : 0;
  static constexpr int NT = RC<NP>::NT + NH * kWave;
  static_assert(NH <= 8, "kProgSlots");
};
// the forward-backward chain kernel's threads: the dense chain's helpers included (the banded
// chains use the first RC<NP>::NT and the rest end at once, rec_dispatch)
template <int NP>
constexpr int kFbNT = kRbHelpers<NP>::NT;

// Sum over all 64 lanes with DPP only (row sums, then row_bcast:15 / row_bcast:31), read
// from lane 63: wave-uniform.
__device__ __forceinline__ float wave_sum_bcast(float x) {
  x = row16_sum(x);
  // row_bcast:15 / :31 folded into the add; rows outside the mask keep x (one instruction each)
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(x));
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(x));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

// Max over all 64 lanes with DPP only, read from lane 63: wave-uniform.
__device__ __forceinline__ float wave_max_bcast(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x124>(x));
  x = fmaxf(x, dpp_f<0x128>(x));
  asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(x));
  asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(x));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

// v_writelane_b32: lane LANE of dst takes the (wave-uniform) value v; the lane is an inline
// constant (no s_mov: a single wave issues one instruction per issue cycle whatever its type).
template <int LANE>
__device__ __forceinline__ void writelane_c(float& dst, float v) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(dst) : "s"(v), "i"(LANE));
}

// ---- one-instruction shifted window terms (DPP on src0; a lane whose DPP source falls off
// the 64-lane wave is disabled and keeps the destination's previous value)
#define HMM355_DPP_OP(name, op, ctrl)                                                         \
  __device__ __forceinline__ void name(float& dst, float src, float w) {                      \
    asm("s_nop 1\n\t" op " %0, %1, %2 " ctrl " row_mask:0xf bank_mask:0xf" : "+v"(dst) : "v"(src), "v"(w)); \
  }
HMM355_DPP_OP(dpp_add_shr1, "v_add_f32_dpp", "wave_shr:1")    // dst = src[l-1] + w  (lane 0 keeps)
HMM355_DPP_OP(dpp_add_shl1, "v_add_f32_dpp", "wave_shl:1")    // dst = src[l+1] + w  (lane 63 keeps)
HMM355_DPP_OP(dpp_add_ror1, "v_add_f32_dpp", "wave_ror:1")    // dst = src[l-1 mod 64] + w
HMM355_DPP_OP(dpp_add_rol1, "v_add_f32_dpp", "wave_rol:1")    // dst = src[l+1 mod 64] + w
HMM355_DPP_OP(dpp_mul_shr1, "v_mul_f32_dpp", "wave_shr:1")
HMM355_DPP_OP(dpp_mul_shl1, "v_mul_f32_dpp", "wave_shl:1")
HMM355_DPP_OP(dpp_mul_ror1, "v_mul_f32_dpp", "wave_ror:1")
HMM355_DPP_OP(dpp_mul_rol1, "v_mul_f32_dpp", "wave_rol:1")
HMM355_DPP_OP(dpp_fmac_shr1, "v_fmac_f32_dpp", "wave_shr:1")  // dst += src[l-1] * w (lane 0 keeps)
HMM355_DPP_OP(dpp_fmac_shl1, "v_fmac_f32_dpp", "wave_shl:1")  // dst += src[l+1] * w (lane 63 keeps)
#undef HMM355_DPP_OP

// dst = dst (op) src[perm(lane)] as ONE VALU instruction, for the in-row reductions of the
// register-blocked dense chain (hipcc emits a separate v_mov_b32_dpp plus a zeroed "old"
// operand for each of these)
#define HMM355_DPP_RED(name, op, ctrl)                                                        \
  __device__ __forceinline__ void name(float& dst, float src) {                               \
    asm("s_nop 1\n\t" op " %0, %1, %0 " ctrl " row_mask:0xf bank_mask:0xf" : "+v"(dst) : "v"(src)); \
  }
HMM355_DPP_RED(red_add_mirror, "v_add_f32_dpp", "row_mirror")
HMM355_DPP_RED(red_add_hmirror, "v_add_f32_dpp", "row_half_mirror")
HMM355_DPP_RED(red_add_q3210, "v_add_f32_dpp", "quad_perm:[3,2,1,0]")
HMM355_DPP_RED(red_add_q1032, "v_add_f32_dpp", "quad_perm:[1,0,3,2]")
HMM355_DPP_RED(red_max_mirror, "v_max_f32_dpp", "row_mirror")
HMM355_DPP_RED(red_max_hmirror, "v_max_f32_dpp", "row_half_mirror")
HMM355_DPP_RED(red_max_q3210, "v_max_f32_dpp", "quad_perm:[3,2,1,0]")
HMM355_DPP_RED(red_max_q1032, "v_max_f32_dpp", "quad_perm:[1,0,3,2]")
#undef HMM355_DPP_RED

// The reduce-scatter of the four output partials of rec_run_rb over the 16 lanes of a row
// (mirror, half mirror, two quad permutations: slot 0 of every lane of quad x ends with output
// 4g + x), written as one block with only the wait states the DPP-read hazard needs (a DPP
// source written by one of the two previous VALU instructions: 2 wait states).  The separate
// helpers above pad every DPP op with "s_nop 1"; here the forward-backward form interleaves the
// all-reduce of the scale c with the outputs' tree, so most reads are two instructions away
// from their writes (tools/mb_dense.hip: 297 -> 279 ns per FB step).  Same operations in the same
// order as the helpers: identical bits.
__device__ __forceinline__ void red4_add_with_c(float& s0, float& s1, float s2, float s3, float& c) {
  asm("s_nop 1\n\t"
      "v_add_f32_dpp %2, %2, %2 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %0, %3, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %4, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_add_f32_dpp %0, %1, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 quad_perm:[3,2,1,0] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[3,2,1,0] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "+v"(s0), "+v"(s1), "+v"(c)
      : "v"(s3), "v"(s2));
}
__device__ __forceinline__ void red4_max(float& s0, float& s1, float s2, float s3) {
  asm("s_nop 1\n\t"
      "v_max_f32_dpp %0, %2, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %1, %3, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_f32_dpp %0, %1, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[3,2,1,0] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "+v"(s0), "+v"(s1)
      : "v"(s3), "v"(s2));
}

// Window term of slot offset DD in {-1, +1} for state vector v (state 64*blk + lane), weights
// w: Viterbi -> t = v(s + DD) + w (neutral -inf past the ends); FB -> acc += v(s + DD) * w.
template <int NB, bool FB, int DD>
__device__ __forceinline__ void win_term1(const float (&v)[NB], const float (&w)[NB], float (&acc)[NB]) {
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    const bool edge = DD < 0 ? blk == 0 : blk == NB - 1;  // no neighbouring block
    if (FB) {
      if (edge) {
        if (DD < 0) dpp_fmac_shr1(acc[blk], v[blk], w[blk]);
        else dpp_fmac_shl1(acc[blk], v[blk], w[blk]);
      } else {
        float t;
        if (DD < 0) { dpp_mul_ror1(t, v[blk - 1], w[blk]); dpp_mul_shr1(t, v[blk], w[blk]); }
        else { dpp_mul_rol1(t, v[blk + 1], w[blk]); dpp_mul_shl1(t, v[blk], w[blk]); }
        acc[blk] += t;
      }
    } else {
      float t = -INFINITY;
      if (!edge) {
        if (DD < 0) dpp_add_ror1(t, v[blk - 1], w[blk]);
        else dpp_add_rol1(t, v[blk + 1], w[blk]);
      }
      if (DD < 0) dpp_add_shr1(t, v[blk], w[blk]);
      else dpp_add_shl1(t, v[blk], w[blk]);
      acc[blk] = fmaxf(acc[blk], t);
    }
  }
}

// Whole-vector lane shifts of a state vector held as v[blk] = state 64*blk + lane (DPP
// wave_shr:1 / wave_shl:1; the lane that falls off a 64-block takes the neighbouring block's
// edge value through wave_ror:1 / wave_rol:1 passed as the DPP "old" operand).
// out(s) = v(s - 1) (shr) or v(s + 1) (shl); states outside [0, NB*64) read `edge`.
template <int NB>
__device__ __forceinline__ void vec_shr1(const float (&v)[NB], float (&out)[NB], float edge) {
#pragma unroll
  for (int blk = NB - 1; blk >= 0; --blk) {
    const int carry = blk > 0 ? __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[blk - 1]), 0x13C, 0xF, 0xF, false)
                              : __builtin_bit_cast(int, edge);
    out[blk] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(carry, __builtin_bit_cast(int, v[blk]), 0x138, 0xF, 0xF, false));
  }
}
template <int NB>
__device__ __forceinline__ void vec_shl1(const float (&v)[NB], float (&out)[NB], float edge) {
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    const int carry = blk < NB - 1 ? __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[blk + 1]), 0x134, 0xF, 0xF, false)
                                   : __builtin_bit_cast(int, edge);
    out[blk] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(carry, __builtin_bit_cast(int, v[blk]), 0x130, 0xF, 0xF, false));
  }
}
// window slots k = 0..TW-1 <-> states s + TD0 + k, from registers
template <int NB, int TD0, int TW>
__device__ __forceinline__ void vec_window(const float (&v)[NB], float (&win)[NB][TW > 0 ? TW : 1], float edge) {
  float neg[3][NB], pos[3][NB];
  // negative offsets: successive right shifts; positive: successive left shifts
  if constexpr (TD0 < 0) {
    vec_shr1<NB>(v, neg[0], edge);
    if constexpr (TD0 < -1) vec_shr1<NB>(neg[0], neg[1], edge);
    if constexpr (TD0 < -2) vec_shr1<NB>(neg[1], neg[2], edge);
  }
  if constexpr (TD0 + TW - 1 > 0) {
    vec_shl1<NB>(v, pos[0], edge);
    if constexpr (TD0 + TW - 1 > 1) vec_shl1<NB>(pos[0], pos[1], edge);
    if constexpr (TD0 + TW - 1 > 2) vec_shl1<NB>(pos[1], pos[2], edge);
  }
#pragma unroll
  for (int k = 0; k < TW; ++k) {
    const int dd = TD0 + k;
#pragma unroll
    for (int blk = 0; blk < NB; ++blk)
      win[blk][k] = dd == 0 ? v[blk] : (dd < 0 ? neg[-dd - 1][blk] : pos[dd - 1][blk]);
  }
}

struct RecArgs {
  const float* obs;   // (B,T,N) emissions
  const float* mat;   // (N,N) log transition matrix
  const float* init;  // (N) log_p0 (FB alpha, Viterbi) / unused (FB beta)
  float* rows;        // stored rows: FB -> (B,T,NP) scaled alpha/beta; Viterbi -> (B,T,N) delta
  float* ls;          // (B,T) log-scales (FB) or null
  float* loglik;      // (B) sequence log-likelihood (FB alpha) or null
  int B, T, N, obs_mode, row_stride;
  const BandDesc* band;  // banded decomposition (band.h) or null: dense chain
  const float* binit;    // backward only: (B,NP) terminal vector (max-normalised) or null = ones
  const float* bscale;   // backward only: (B) log-scale of binit
  uint8_t* psi;          // Viterbi, fused banded chain only: (B,T,NP) argmax pointers (kVitFused)
  const float* rmax;     // FB with OBS_LOG: (B,T) row maxima M_t (e_t = exp(lo_t - M_t)), else null
  float* out_exp;        // FB: (B,T,N) forward (alpha) / backward (beta) output written at flush, or null
  // Viterbi with psi followers (dense chains, vit_kern.h): chunk maps, path, final score
  uint8_t* G;            // (B, nchunks, NP) chunk maps
  int64_t* states;       // (B,T) decoded path
  float* final_score;    // (B) max of the last trellis row, or null
  int nchunks;
  // Viterbi, dense chain with psi followers (HMM355_VIT_PLAN_DENSE, vit_kern.h): the helpers
  // publish the blocks they have flushed in prog[b * kProgSlots + h]; the follower workgroups
  // (blockIdx >= B) mark the chunks they finished in done[b * nchunks + c]
  int* prog;
  uint8_t* done;
  // FB: (B,T) the normaliser of each step, by time (alpha: cs[t] = c with u_{t+1} = A^T u_t e_{t+1} / c;
  // beta: cs[t] = c with v_{t-1} = A (e_t v_t) / c), written beside LS for the adjoint
  // (autograd.py), or null
  float* cs;
  // Banded chains with followers (follow.h): the helpers' row flushes (FB: U / V rows) and psi
  // row copies (fused Viterbi) are write-through (sc1) stores, and one lane publishes how many
  // 16-step blocks of them are complete in pub[b * 2 + direction] (FB) / pub[b] (Viterbi):
  // blocks [0, pub) done while the chain runs, nblocks + 1 once everything (rows, psi, the last
  // trellis row) is stored.  Null: no publishing.
  int* pub;
  // Viterbi with OBS_PROB emissions and log leaders (follow.h vit_lead): lobuf (B,T,N) holds
  // log(x + 1e-8) of 16-step blocks [4, lready[b]) of sequence b, written by the leaders; the
  // staging helpers load a block from there when it is ready (checked two blocks ahead), else
  // the raw emissions, and take the log themselves
  const float* lobuf;
  const int* lready;
  float* lik_ref;        // FB alpha with publishing: (B) the reference's compute_likelihood value
  uint8_t* path;         // Viterbi decode follower: (B, nchunks, NP, 64) chunk paths (follow.h)
  unsigned token;        // the published counts' call token (common.h poll_count / publish_count)
};
constexpr int kProgSlots = 8;  // >= kRbHelpers<NP>::NH

// The banded Viterbi chain computes the argmax pointers psi itself (helper waves on the idle
// SIMDs, from the delta rows still in its LDS ring), so the psi pass only composes the
// 64-step chunk maps from them.  Enabled where the helpers have the issue slots: NP >= 128.
constexpr int kPsiChunk = 64;
template <int NP>
constexpr bool kVitFused = RC<NP>::NW >= 6;
// threads of the Viterbi chain kernel: the fused banded chain runs 16 waves (rec_band: two
// staging helpers and two psi waves on each of SIMDs 1..3); the dense chains use the first
// RC<NP>::NW waves and the rest exit at once
template <int NP>
constexpr int kVitNT = kVitFused<NP> ? (1024 > kRbHelpers<NP>::NT ? 1024 : kRbHelpers<NP>::NT)
                                     : kRbHelpers<NP>::NT;

template <int KIND>
__device__ __forceinline__ int rec_tau(int q, int T) {
  return KIND == kFbBeta ? T - 1 - q : q;
}

// the log table of logcr.h; each wave that stages Viterbi emissions copies it into LDS itself
// (identical values from every copier, so no barrier: a wave's own LDS writes precede its reads)
__device__ const double g_logcr_tab[256] = {HMM355_LOGCR_TABLE};
template <int NP>
__device__ __forceinline__ void rec_logt_fill(float* lds, int l) {
  double* t = reinterpret_cast<double*>(lds + RC<NP>::OFF_LOGT);
#pragma unroll
  for (int k = 0; k < 4; ++k) t[l + 64 * k] = g_logcr_tab[l + 64 * k];
}

// ---- emission staging: lane l of wave w holds 4 consecutive states of one step
// r[0..3]: the emissions; r[4]: the step's row maximum M_t (FB with OBS_LOG; the load reads an
// address of the same row otherwise, so the staging stays branch-free, and is not used)
// Viterbi: r[4] is the block's emission form, 1 = log-emissions (OBS_LOG, or rows the log
// leaders converted: `obs` = RecArgs::lobuf), 0 = probabilities (the staging takes the log);
// vmode < 0: from a.obs_mode.
// SC1 (the fused Viterbi chain, whose rows may come from the log leaders in this launch,
// follow.h): every load is an sc1 load (L1 bypassed: no stale line of a row another workgroup
// wrote), from a buffer resource over the sequence's rows of `obs`.
template <int NP, int KIND, bool FULL = false, bool SC1 = false>
__device__ __forceinline__ void rec_load(const RecArgs& a, int b, int blk, int w, int l, float (&r)[5],
                                         const float* obs = nullptr, float vmode = -1.f) {
  const int q = blk * 16 + (l >> 2);
  const int col = 16 * w + 4 * (l & 3);
  const bool qok = q < a.T;
  const int tq = qok ? rec_tau<KIND>(q, a.T) : 0;
  const size_t bt = (size_t)b * a.T + tq;
  const float* src = (obs ? obs : a.obs) + bt * a.N;
  if constexpr (KIND != kVit) {
    const float* mp = a.rmax ? a.rmax + bt : src;  // a pointer select, not a branch
    r[4] = *mp;
  } else {
    r[4] = vmode >= 0.f ? vmode : (a.obs_mode == HMM355_OBS_LOG ? 1.f : 0.f);
  }
  if constexpr (SC1) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc((obs ? obs : a.obs) + (size_t)b * a.T * a.N, (size_t)a.T * a.N * 4);
    const int off = (tq * a.N + col) * 4;
    if constexpr (FULL) {
      const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kAuxSc1));
      r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = qok && col + k < a.N;
        r[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? off + 4 * k : 0, 0, kAuxSc1));
      }
    }
    return;
  }
  if constexpr (FULL) {  // full 16-B aligned rows (the caller checked): one 16-B load
    const float4 v = *reinterpret_cast<const float4*>(src + col);
    r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    return;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool ok = qok && col + k < a.N;
    r[k] = src[ok ? col + k : 0];  // no select: the wait lands at the first (masked) use
  }
}

// PERBLK (the fused Viterbi chain with log leaders): the emission form is r[4] of the block's
// registers (rec_load); otherwise a.obs_mode
template <int NP, int KIND, bool PERBLK = false>
__device__ __forceinline__ void rec_stage(const RecArgs& a, float* lds, int blk, int w, int l, const float (&r)[5]) {
  using C = RC<NP>;
  const int sq = l >> 2;
  const int col = 16 * w + 4 * (l & 3);
  const bool qok = blk * 16 + sq < a.T;
  // one uniform branch on the emission mode per call, selects inside: per-element branches
  // bloat the helpers' unrolled code (three block copies x HV virtual waves) and end in
  // waitcnt joins
  float e[4];
  // (Viterbi: the form travels with the block's registers, r[4]; uniform across the wave)
  const bool lg = (KIND == kVit && PERBLK) ? __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, r[4])) != 0
                                          : a.obs_mode == HMM355_OBS_LOG;
  if (lg) {
    // FB: e = exp(lo - M_t) with the row maximum M_t (log-emissions of -100 .. -400 would
    // underflow exp); M_t is carried into the log-scales by rec_flush
    const float m = KIND == kVit ? 0.f : (a.rmax ? r[4] : 0.f);
    if (KIND != kVit && w == 0 && (l & 3) == 0) lds[C::OFF_M + ((blk * 16 + sq) & (C::MRING - 1))] = m;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = qok && col + k < a.N;
      e[k] = KIND == kVit ? (ok ? r[k] : -INFINITY) : (ok ? __expf(r[k] - m) : 0.f);
    }
  } else {
    // Viterbi: log(x + 1e-8) correctly rounded (logcr.h; the fp32 sum as hmm.py:152 forms it)
    const double* lt = reinterpret_cast<const double*>(lds + C::OFF_LOGT);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = qok && col + k < a.N;
      // (diagnostic ablation bit 1 << 22: no log, timing only)
      const float lv = (kAbl & (1 << 22)) ? r[k] + 1e-8f : logcr_fast(r[k] + 1e-8f, lt);
      e[k] = KIND == kVit ? (ok ? lv : -INFINITY) : (ok ? r[k] + 1e-8f : 0.f);
    }
  }
  *reinterpret_cast<float4*>(lds + C::OFF_EMIS + ((blk % 3) * 16 + sq) * NP + col) = make_float4(e[0], e[1], e[2], e[3]);
}

// ---- the Rabiner log-scales of the 16 rows of staging block `blk` (FB):
// LS_rho = LS_{rho-1} + log c_{rho-1}, a 16-lane inclusive scan with the running base in
// double.  Every flushing wave computes it (so each knows its rows' log-scales for the exp
// outputs and keeps its own `base`); the one with write_ls stores LA / LB.  Lane j < 16
// returns LS of row 16*blk + j.
template <int NP, int KIND>
__device__ __forceinline__ float rec_ls_scan(const RecArgs& a, const float* lds, int b, int blk, double& base,
                                             bool write_ls) {
  using C = RC<NP>;
  if constexpr (KIND == kVit) return 0.f;
  const int lane = threadIdx.x & 63, j = lane & 15;
  const int rho = blk * 16 + j;
  const float c = lds[C::OFF_SC + 64 * ((rho - 1) & (C::RING - 1))];  // unconditional (see rec_flush)
  const bool live = lane < 16 && rho >= 1 && rho < a.T;
  float x = live ? __logf(c) : 0.f;
  // the step's normaliser by time for the adjoint (alpha: time rho - 1; beta: time T - rho)
  if (write_ls && a.cs && live)
    a.cs[(size_t)b * a.T + (KIND == kFbBeta ? a.T - rho : rho - 1)] = c;
  if (a.obs_mode == HMM355_OBS_LOG) {
    // shifted emissions: alpha row rho used M_{tau(rho)}, beta row rho used M_{tau(rho)+1}
    // (the row staged as rho - 1); beta row 0 (the terminal vector) none
    const int src = KIND == kFbBeta ? rho - 1 : rho;
    const float m = lds[C::OFF_M + (src & (C::MRING - 1))];
    x += (lane < 16 && src >= 0 && rho < a.T) ? m : 0.f;
  }
  x += dpp_f<0x111>(x);  // row_shr:1
  x += dpp_f<0x112>(x);  // row_shr:2
  x += dpp_f<0x114>(x);  // row_shr:4
  x += dpp_f<0x118>(x);  // row_shr:8
  const float lsv = (float)(base + (double)x);
  if (write_ls && lane < 16 && rho < a.T) a.ls[(size_t)b * a.T + rec_tau<KIND>(rho, a.T)] = lsv;
  base += (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 15));
  return lsv;
}

// ---- flush the 16 stored rows of staging block `blk`; FB with a.out_exp also writes the
// reference's output row exp(log x + LS) (forward = exp(log alpha) for alpha, backward for
// beta, hmm.py:127-128) from the same LDS row, so the posterior pass only forms the posterior.
// lsv: rec_ls_scan's vector (LS of row j in lane j).  A row whose log-scale is below -110 is
// exactly 0 (x <= N <= 256 < e^6 and e^-104 is below the smallest fp32 denormal), as the
// reference's exp underflows: no transcendentals for it.
// (WHAT: 1 the stored rows, 2 the exp outputs, 3 both)
template <int NP, int KIND, int WHAT = 3>
__device__ __forceinline__ void rec_flush(const RecArgs& a, const float* lds, int b, int blk, int tid, float lsv) {
  using C = RC<NP>;
  const int q_base = blk * 16;
  if (a.row_stride == NP) {
    constexpr int PER_ROW = NP / 4;
    const int row = tid / PER_ROW, c4 = (tid % PER_ROW) * 4;
    const int q = q_base + row;
    // the LDS read is unconditional (only the store is guarded): a read under the guard
    // ends in an s_waitcnt vmcnt(0) join that drains the helper's emission prefetches
    const float4 v = *reinterpret_cast<const float4*>(lds + C::OFF_RING + (q & (C::RING - 1)) * NP + c4);
    const size_t tr = (size_t)b * a.T + rec_tau<KIND>(q, a.T);
    if ((WHAT & 1) && q < a.T) {
      if (a.pub && !(kFAbl & 4)) {
        // followers read these rows in this launch: write-through (sc1) 16-B stores (follow.h)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            a.rows + (size_t)b * a.T * NP, (short)0, (int)((size_t)a.T * NP * 4), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs,
                                               (rec_tau<KIND>(q, a.T) * NP + c4) * 4, 0, kAuxSc1);
      } else {
        *reinterpret_cast<float4*>(a.rows + tr * NP + c4) = v;
      }
    }
    if constexpr (KIND != kVit && (WHAT & 2)) {
      if (a.out_exp) {
        const float ls = __shfl(lsv, row);
        const bool live = ls >= -110.f;
        float ov[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) ov[k] = live ? __expf(__logf(ov[k]) + ls) : 0.f;
        if (q < a.T) {
          if (a.N == NP) {
            *reinterpret_cast<float4*>(a.out_exp + tr * NP + c4) = make_float4(ov[0], ov[1], ov[2], ov[3]);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (c4 + k < a.N) a.out_exp[tr * a.N + c4 + k] = ov[k];
          }
        }
      }
    }
  } else {
    for (int idx = tid; idx < 16 * a.N; idx += C::NT) {
      const int row = idx / a.N, col = idx - row * a.N;
      const int q = q_base + row;
      float* dst = a.rows + ((size_t)b * a.T + rec_tau<KIND>(q, a.T)) * a.row_stride + col;
      const float v = lds[C::OFF_RING + (q & (C::RING - 1)) * NP + col];
      if ((WHAT & 1) && q < a.T) {
        if (a.pub && !(kFAbl & 4)) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (sc1)
        else *dst = v;
      }
    }
  }
}

template <int NP, int KIND>
__device__ __forceinline__ void rec_run(const RecArgs& a, float* lds, int b) {
  using C = RC<NP>;
  constexpr bool FB = KIND != kVit;
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int o = 16 * w + c;  // output of this lane
  const int T = a.T, N = a.N;

  // matrix slice: M[blk][n] = Mat[i][o] (alpha/Viterbi) or Mat[o][i] (beta), i = 64blk+16r+n
  float M[C::NBLK][16];
#pragma unroll
  for (int blk = 0; blk < C::NBLK; ++blk)
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int i = 64 * blk + 16 * r + n;
      const bool ok = i < N && o < N;
      const size_t idx = ok ? (KIND == kFbBeta ? (size_t)o * N + i : (size_t)i * N + o) : 0;
      const float v = a.mat[idx];
      M[blk][n] = FB ? __expf(ok ? v : -INFINITY) : (ok ? v : -INFINITY);
    }

  const int nblocks = (T + 15) / 16;
  float er0[5], er1[5];
  if (KIND == kVit) rec_logt_fill<NP>(lds, l);
  rec_load<NP, KIND>(a, b, 0, w, l, er0);
  rec_stage<NP, KIND>(a, lds, 0, w, l, er0);
  if (nblocks > 1) rec_load<NP, KIND>(a, b, 1, w, l, er1);
  lds_barrier();

  auto emis = [&](int rho, int idx) { return lds[C::OFF_EMIS + (((rho >> 4) % 3) * 16 + (rho & 15)) * NP + idx]; };
  // row 0 partials: the whole value in group 0, the identity in groups 1..3
  {
    float v0;
    const int oo = o < N ? o : 0;
    if (KIND == kFbAlpha) v0 = o < N ? __expf(a.init[oo]) * emis(0, o) : 0.f;  // alpha_0 = p0 * e_0
    else if (KIND == kFbBeta) v0 = o < N ? (a.binit ? a.binit[(size_t)b * NP + o] : 1.f) : 0.f;  // beta_{T-1}
    else v0 = o < N ? a.init[oo] + emis(0, o) : -INFINITY;                      // delta_0 = init + lo_0
    const float ident = FB ? 0.f : -INFINITY;
    if (r < 2) lds[C::OFF_PART + o * 2 + r] = r == 0 ? v0 : ident;
  }
  lds_barrier();

  double base = (KIND == kFbBeta && a.bscale) ? (double)a.bscale[b] : 0.0;
  unsigned long long st_acc[4] = {0, 0, 0, 0}, st_prev = 0, st_t0 = 0, st_steps = 0;
  long long rt0 = 0;
  if (kStamp) { st_t0 = stamp(); st_prev = st_t0; rt0 = __builtin_amdgcn_s_memrealtime(); }
  auto mark = [&](int k) {
    if (kStamp) { const unsigned long long t = stamp(); st_acc[k] += t - st_prev; st_prev = t; }
  };
  // sum (FB) / max (Viterbi) of the four row-group partials of input 64*blk + lane
  auto gather = [&](int prv, float (&y)[C::NBLK]) {
#pragma unroll
    for (int blk = 0; blk < C::NBLK; ++blk) {
      // one conflict-free ds_read_b64 per block (2 LDS cycles per wave)
      const float2 pp = *reinterpret_cast<const float2*>(lds + C::OFF_PART + (prv * NP + 64 * blk + l) * 2);
      y[blk] = FB ? pp.x + pp.y : fmaxf(pp.x, pp.y);
    }
  };
  // wave 0 keeps the finished row rho (alpha: u, beta: v, Viterbi: delta)
  auto keep_row = [&](int rho, const float (&y)[C::NBLK]) {
    if (w == 0) {
#pragma unroll
      for (int blk = 0; blk < C::NBLK; ++blk) lds[C::OFF_RING + (rho & (C::RING - 1)) * NP + 64 * blk + l] = y[blk];
    }
  };

  auto run_block = [&](int kb, float(&ernext)[5], float(&erfree)[5]) {
    if (!(kAbl & 4)) {
      // straight-line staging and loads (the tail stages a padding block and re-loads the
      // last one), as in the banded helpers: exact waitcnt counts
      rec_stage<NP, KIND>(a, lds, kb + 1, w, l, ernext);
      rec_load<NP, KIND>(a, b, kb + 2 < nblocks ? kb + 2 : nblocks - 1, w, l, erfree);
      if (kb >= 2) rec_flush<NP, KIND>(a, lds, b, kb - 2, tid, rec_ls_scan<NP, KIND>(a, lds, b, kb - 2, base, w == C::NW - 1));
    }
    const int q0 = kb * 16 < 1 ? 1 : kb * 16;
    const int q1 = (kb + 1) * 16 < T ? (kb + 1) * 16 : T;
    for (int q = q0; q < q1; ++q) {
      const int prv = (q - 1) & 1, cur = q & 1;
      // the step's emissions are read beside the partials, off the dependent chain
      float eo = 0.f, ey[C::NBLK];
      if (KIND == kFbBeta) {
#pragma unroll
        for (int blk = 0; blk < C::NBLK; ++blk) ey[blk] = emis(q - 1, 64 * blk + l);
      } else {
        eo = emis(q, o);
      }
      float y[C::NBLK];
      if (kStamp) mark(3);
      gather(prv, y);
      if (kStamp) { keep(y[0]); mark(0); }
      keep_row(q - 1, y);
      if (KIND == kFbBeta) {  // beta's product input is y = v * e (hmm.py:113-115)
#pragma unroll
        for (int blk = 0; blk < C::NBLK; ++blk) y[blk] *= ey[blk];
      }
      float part;
      if (FB) {
        // 32 (NP=128) v_fmac_f32_dpp into four accumulators, with the DPP wave sum of the
        // product input (c_{q-1}, the Rabiner normaliser) interleaved stage by stage: issue is
        // in order within a wave, so a sum issued as one block would add its full dependent
        // latency to the step.  sched_barrier pins the interleave.
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        float cx = y[0];
#pragma unroll
        for (int blk = 1; blk < C::NBLK; ++blk) cx += y[blk];
        float cs = 0.f;
        constexpr int G = 4 * C::NBLK;  // groups of 4 fmacs
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int blk = g >> 2, n0 = 4 * (g & 3);
          if (kAbl & 2) {
            if ((g & 3) == 0) a0 += y[blk];
          } else {
            switch (n0) {
              case 0:  fmac_bcast<0>(a0, y[blk], M[blk][0]);   fmac_bcast<1>(a1, y[blk], M[blk][1]);
                       fmac_bcast<2>(a2, y[blk], M[blk][2]);   fmac_bcast<3>(a3, y[blk], M[blk][3]);   break;
              case 4:  fmac_bcast<4>(a0, y[blk], M[blk][4]);   fmac_bcast<5>(a1, y[blk], M[blk][5]);
                       fmac_bcast<6>(a2, y[blk], M[blk][6]);   fmac_bcast<7>(a3, y[blk], M[blk][7]);   break;
              case 8:  fmac_bcast<8>(a0, y[blk], M[blk][8]);   fmac_bcast<9>(a1, y[blk], M[blk][9]);
                       fmac_bcast<10>(a2, y[blk], M[blk][10]); fmac_bcast<11>(a3, y[blk], M[blk][11]); break;
              default: fmac_bcast<12>(a0, y[blk], M[blk][12]); fmac_bcast<13>(a1, y[blk], M[blk][13]);
                       fmac_bcast<14>(a2, y[blk], M[blk][14]); fmac_bcast<15>(a3, y[blk], M[blk][15]); break;
            }
          }
          // wave-sum stages spread over the groups (all eight done by the last group)
#pragma unroll
          for (int st = (g * 8) / G; st < ((g + 1) * 8) / G; ++st) {
            switch (st) {
              case 0: cx += dpp_f<0xB1>(cx); break;   // quad_perm [1,0,3,2]
              case 1: cx += dpp_f<0x4E>(cx); break;   // quad_perm [2,3,0,1]
              case 2: cx += dpp_f<0x124>(cx); break;  // row_ror:4
              case 3: cx += dpp_f<0x128>(cx); break;  // row_ror:8
              case 4:
                cx += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, cx), 0x142, 0xA, 0xF, false));
                break;                                // row_bcast:15
              case 5:
                cx += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, cx), 0x143, 0xC, 0xF, false));
                break;                                // row_bcast:31
              case 6: cs = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cx), 63)); break;
              default: break;
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        const float scale = __builtin_amdgcn_rcpf(cs);
        if (tid == 0) lds[C::OFF_SC + 64 * ((q - 1) & (C::RING - 1))] = cs;
        float h0 = (a0 + a1) + (a2 + a3), h1 = h0;
        permlane32_swap(h0, h1);  // rows {0,2} / {1,3} summed: lanes 0..31 hold both halves
        const float acc = h0 + h1;
        // alpha: u_q = z * e_q / c_{q-1};  beta: v_q = z / c_{q-1}
        part = KIND == kFbAlpha ? acc * (scale * eo) : acc * scale;
      } else {
        float m0 = -INFINITY, m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY;
#pragma unroll
        for (int blk = 0; blk < C::NBLK; ++blk) {
          if (kAbl & 2) { m0 = fmaxf(m0, y[blk]); continue; }
          m0 = fmaxf(m0, fmaxf(row_bcast<0>(y[blk]) + M[blk][0], row_bcast<1>(y[blk]) + M[blk][1]));
          m1 = fmaxf(m1, fmaxf(row_bcast<2>(y[blk]) + M[blk][2], row_bcast<3>(y[blk]) + M[blk][3]));
          m2 = fmaxf(m2, fmaxf(row_bcast<4>(y[blk]) + M[blk][4], row_bcast<5>(y[blk]) + M[blk][5]));
          m3 = fmaxf(m3, fmaxf(row_bcast<6>(y[blk]) + M[blk][6], row_bcast<7>(y[blk]) + M[blk][7]));
          m0 = fmaxf(m0, fmaxf(row_bcast<8>(y[blk]) + M[blk][8], row_bcast<9>(y[blk]) + M[blk][9]));
          m1 = fmaxf(m1, fmaxf(row_bcast<10>(y[blk]) + M[blk][10], row_bcast<11>(y[blk]) + M[blk][11]));
          m2 = fmaxf(m2, fmaxf(row_bcast<12>(y[blk]) + M[blk][12], row_bcast<13>(y[blk]) + M[blk][13]));
          m3 = fmaxf(m3, fmaxf(row_bcast<14>(y[blk]) + M[blk][14], row_bcast<15>(y[blk]) + M[blk][15]));
        }
        float h0 = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3)), h1 = h0;
        permlane32_swap(h0, h1);
        // delta_q = max(...) + lo_q: adding lo to each partial max is exact (monotone)
        part = fmaxf(h0, h1) + eo;
      }
      if (kStamp) { keep(part); mark(1); }
      if (l < 32) lds[C::OFF_PART + (cur * NP + o) * 2 + r] = part;
      if (kStamp) { mark(2); ++st_steps; }
      step_barrier();
    }
  };
  for (int k = 0; k < nblocks; k += 2) {
    run_block(k, er1, er0);
    if (k + 1 < nblocks) run_block(k + 1, er0, er1);
  }
  if (kStamp && (tid & 63) == 0) {
    const unsigned long long t1 = stamp();
    const long long rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o8 = g_rec_stamps + ((size_t)(blockIdx.x * C::NW + w) % kStampWaves) * 8;
    o8[0] = st_acc[0]; o8[1] = st_acc[1]; o8[2] = st_acc[2]; o8[3] = st_acc[3];
    o8[4] = st_steps; o8[5] = t1 - st_t0; o8[6] = t1 - st_t0; o8[7] = (unsigned long long)(rt1 - rt0);
  }
  // final row T-1 (its partials were written by the last step, or are the init for T == 1)
  float y[C::NBLK];
  gather((T - 1) & 1, y);
  keep_row(T - 1, y);
  if (KIND == kFbAlpha && a.loglik && w == C::NW - 1) {
    float ys = y[0];
#pragma unroll
    for (int blk = 1; blk < C::NBLK; ++blk) ys += y[blk];
    const float cs = wave_sum_bcast(ys);
    if (l == 0) lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))] = cs;  // c_{T-1} (loglik only)
  }
  lds_barrier();
  if (nblocks >= 2)
    rec_flush<NP, KIND>(a, lds, b, nblocks - 2, tid, rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 2, base, w == C::NW - 1));
  rec_flush<NP, KIND>(a, lds, b, nblocks - 1, tid, rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 1, base, w == C::NW - 1));
  if (KIND == kFbAlpha && a.loglik && tid == C::NT - 64) {
    // loglik = LS_{T-1} + log c_{T-1}; `base` (wave NW-1) now holds LS_{T-1}
    a.loglik[b] = (float)(base + (double)__logf(lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))]));
  }
}

// ---------------------------------------------------------------------------------------
// Dense chain, register-operand form (NP <= 128; round 2).  Same lane layout as rec_run
// (wave w owns outputs 16w + c, the lane's row r owns inputs 64*blk + 16r + n), but the
// previous vector is not broadcast by DPP: every lane reads its row's 16 inputs per block
// from LDS (4 ds_read_b128 at one address per 16-lane row: broadcasts, conflict-free) and
// the products run as packed fp32 (v_pk_fma_f32, two inputs per instruction; Viterbi
// v_pk_add_f32 + v_max3).  rec_run's v_fmac_f32_dpp issues at half rate, so its compute
// phase was ~680 cycles per step on the slower wave of each SIMD (tools/stamps.py); here
// the same 16K products are 16 packed ops per wave.  The four row groups are summed in
// registers (permlane32 + permlane16 swaps), so each step writes ONE value per output
// (lanes 0..15): Y[2][NP] holds the rows, and for beta P[2][NP] its product input v * e.
template <int NP, int KIND>
__device__ __forceinline__ void rec_run_bc(const RecArgs& a, float* lds, int b) {
  using C = RC<NP>;
  static_assert(NP <= 128, "register-operand dense chain: NP <= 128");
  constexpr bool FB = KIND != kVit;
  constexpr int NBK = C::NBLK;
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int o = 16 * w + c;  // output of this lane
  const int T = a.T, N = a.N;
  float* Y = lds + C::OFF_PART;            // [2][NP] rows (alpha u, beta v, Viterbi delta)
  float* Pv = lds + C::OFF_PART + 2 * NP;  // [2][NP] beta: product input v * e

  // matrix slice as pairs: M2[blk][m] = (Mat[i][o], Mat[i+1][o]) (beta: Mat[o][i]),
  // i = 64 blk + 16 r + 2 m
  f2 M2[NBK][8];
#pragma unroll
  for (int blk = 0; blk < NBK; ++blk)
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int i = 64 * blk + 16 * r + n;
      const bool ok = i < N && o < N;
      const size_t idx = ok ? (KIND == kFbBeta ? (size_t)o * N + i : (size_t)i * N + o) : 0;
      const float v = a.mat[idx];
      M2[blk][n >> 1][n & 1] = FB ? __expf(ok ? v : -INFINITY) : (ok ? v : -INFINITY);
    }

  const int nblocks = (T + 15) / 16;
  float er0[5], er1[5];
  if (KIND == kVit) rec_logt_fill<NP>(lds, l);
  rec_load<NP, KIND>(a, b, 0, w, l, er0);
  rec_stage<NP, KIND>(a, lds, 0, w, l, er0);
  if (nblocks > 1) rec_load<NP, KIND>(a, b, 1, w, l, er1);
  lds_barrier();

  auto emis = [&](int rho, int idx) { return lds[C::OFF_EMIS + (((rho >> 4) % 3) * 16 + (rho & 15)) * NP + idx]; };
  {
    float v0;
    const int oo = o < N ? o : 0;
    if (KIND == kFbAlpha) v0 = o < N ? __expf(a.init[oo]) * emis(0, o) : 0.f;  // alpha_0 = p0 * e_0
    else if (KIND == kFbBeta) v0 = o < N ? (a.binit ? a.binit[(size_t)b * NP + o] : 1.f) : 0.f;  // beta_{T-1}
    else v0 = o < N ? a.init[oo] + emis(0, o) : -INFINITY;                      // delta_0 = init + lo_0
    if (l < 16) {
      Y[o] = v0;
      if (KIND == kFbBeta) Pv[o] = v0 * emis(0, o);
    }
  }
  lds_barrier();

  double base = (KIND == kFbBeta && a.bscale) ? (double)a.bscale[b] : 0.0;
  unsigned long long st_acc[4] = {0, 0, 0, 0}, st_prev = 0, st_t0 = 0, st_steps = 0;
  long long rt0 = 0;
  if (kStamp) { st_t0 = stamp(); st_prev = st_t0; rt0 = __builtin_amdgcn_s_memrealtime(); }
  auto mark = [&](int k) {
    if (kStamp) { const unsigned long long t = stamp(); st_acc[k] += t - st_prev; st_prev = t; }
  };
  auto keep_row = [&](int rho, const float (&y)[NBK]) {
    if (w == 0) {
#pragma unroll
      for (int blk = 0; blk < NBK; ++blk) lds[C::OFF_RING + (rho & (C::RING - 1)) * NP + 64 * blk + l] = y[blk];
    }
  };

  auto run_block = [&](int kb, float(&ernext)[5], float(&erfree)[5]) {
    rec_stage<NP, KIND>(a, lds, kb + 1, w, l, ernext);
    rec_load<NP, KIND>(a, b, kb + 2 < nblocks ? kb + 2 : nblocks - 1, w, l, erfree);
    if (kb >= 2) rec_flush<NP, KIND>(a, lds, b, kb - 2, tid, rec_ls_scan<NP, KIND>(a, lds, b, kb - 2, base, w == C::NW - 1));
    const int q0 = kb * 16 < 1 ? 1 : kb * 16;
    const int q1 = (kb + 1) * 16 < T ? (kb + 1) * 16 : T;
    for (int q = q0; q < q1; ++q) {
      const int prv = (q - 1) & 1, cur = q & 1;
      const float eo = emis(q, o);  // alpha / Viterbi: emission of output o; beta: of v_q -> P
      if (kStamp) mark(3);
      const float* src = (KIND == kFbBeta ? Pv : Y) + prv * NP;
      f2 yin[NBK][8];
      float yown[NBK], cx = 0.f;
#pragma unroll
      for (int blk = 0; blk < NBK; ++blk) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float4 v4 = *reinterpret_cast<const float4*>(src + 64 * blk + 16 * r + 4 * k);
          yin[blk][2 * k] = f2{v4.x, v4.y};
          yin[blk][2 * k + 1] = f2{v4.z, v4.w};
        }
        yown[blk] = Y[prv * NP + 64 * blk + l];
        if (FB) cx += src[64 * blk + l];  // the normaliser's input (beta: sum of v * e)
      }
      if (kStamp) { keep(yown[0]); mark(0); }
      keep_row(q - 1, yown);
      float h;
      float cs = 0.f;
      if (FB) {
        f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
#pragma unroll
        for (int blk = 0; blk < NBK; ++blk)
#pragma unroll
          for (int m = 0; m < 8; m += 2) {
            acc0 = __builtin_elementwise_fma(yin[blk][m], M2[blk][m], acc0);
            acc1 = __builtin_elementwise_fma(yin[blk][m + 1], M2[blk][m + 1], acc1);
          }
        cs = wave_sum_bcast(cx);  // c_{q-1}, beside the products
        h = (acc0.x + acc0.y) + (acc1.x + acc1.y);
      } else {
        float m0 = -INFINITY, m1 = -INFINITY;
#pragma unroll
        for (int blk = 0; blk < NBK; ++blk)
#pragma unroll
          for (int m = 0; m < 8; m += 2) {
            const f2 t0 = yin[blk][m] + M2[blk][m];
            const f2 t1 = yin[blk][m + 1] + M2[blk][m + 1];
            m0 = fmaxf(m0, fmaxf(t0.x, t0.y));
            m1 = fmaxf(m1, fmaxf(t1.x, t1.y));
          }
        h = fmaxf(m0, m1);
      }
      // the four row groups: rows {0,2} / {1,3} (permlane32), then {0,1} (permlane16)
      float h1 = h;
      permlane32_swap(h, h1);
      h = FB ? h + h1 : fmaxf(h, h1);
      float h2 = h;
      permlane16_swap(h, h2);
      h = FB ? h + h2 : fmaxf(h, h2);
      float val, pval = 0.f;
      if (FB) {
        const float scale = __builtin_amdgcn_rcpf(cs);
        if (tid == 0) lds[C::OFF_SC + 64 * ((q - 1) & (C::RING - 1))] = cs;
        val = KIND == kFbAlpha ? h * (scale * eo) : h * scale;  // alpha: u_q = z e_q / c;  beta: v_q = z / c
        if (KIND == kFbBeta) pval = val * eo;
      } else {
        val = h + eo;  // delta_q = max(...) + lo_q (exact: monotone)
      }
      if (kStamp) { keep(val); mark(1); }
      if (l < 16) {
        Y[cur * NP + o] = val;
        if (KIND == kFbBeta) Pv[cur * NP + o] = pval;
      }
      if (kStamp) { mark(2); ++st_steps; }
      step_barrier();
    }
  };
  for (int k = 0; k < nblocks; k += 2) {
    run_block(k, er1, er0);
    if (k + 1 < nblocks) run_block(k + 1, er0, er1);
  }
  if (kStamp && (tid & 63) == 0) {
    const unsigned long long t1 = stamp();
    const long long rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o8 = g_rec_stamps + ((size_t)(blockIdx.x * C::NW + w) % kStampWaves) * 8;
    o8[0] = st_acc[0]; o8[1] = st_acc[1]; o8[2] = st_acc[2]; o8[3] = st_acc[3];
    o8[4] = st_steps; o8[5] = t1 - st_t0; o8[6] = t1 - st_t0; o8[7] = (unsigned long long)(rt1 - rt0);
  }
  float y[NBK];
#pragma unroll
  for (int blk = 0; blk < NBK; ++blk) y[blk] = Y[((T - 1) & 1) * NP + 64 * blk + l];
  keep_row(T - 1, y);
  if (KIND == kFbAlpha && a.loglik && w == C::NW - 1) {
    float ys = y[0];
#pragma unroll
    for (int blk = 1; blk < NBK; ++blk) ys += y[blk];
    const float cs = wave_sum_bcast(ys);
    if (l == 0) lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))] = cs;  // c_{T-1} (loglik only)
  }
  lds_barrier();
  if (nblocks >= 2)
    rec_flush<NP, KIND>(a, lds, b, nblocks - 2, tid, rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 2, base, w == C::NW - 1));
  rec_flush<NP, KIND>(a, lds, b, nblocks - 1, tid, rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 1, base, w == C::NW - 1));
  if (KIND == kFbAlpha && a.loglik && tid == C::NT - 64) {
    a.loglik[b] = (float)(base + (double)__logf(lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))]));
  }
}

// ---------------------------------------------------------------------------------------
// Dense chain helpers (round 4).  The per-16-step block work of the register-blocked chain --
// the next block's emission staging (exp / log), the global loads two blocks ahead, the log-scale
// scan and the flush of the rows two blocks back (rows + the exp(log x + LS) output) -- costs the
// chain waves ~55 ns per step when they do it themselves between two steps
// (tools/mb_dense.hip: 229 -> 285 ns per FB step, 267 -> 325 Viterbi, prefetched), since every
// wave waits at the next barrier for the slowest.  kRbHelpers<NP>::NH extra waves (launched
// beside the NW chain waves) do it instead, one item per step, each item small enough to finish
// inside the step they share a barrier with:
//   item 0, 1    stage block kb + 1, column slices 2h, 2h + 1 (from registers loaded a block ago)
//   item 2, 3    load block kb + 2 (clamped), the same slices
//   item 4       the log-scale scan of block kb - 2 (every helper keeps its own running base;
//                the last one writes LS)
//   item 5, 6    flush block kb - 2, rows 0..7 and 8..15
//   (Viterbi with psi followers: item 0 also publishes the blocks flushed a block earlier,
//   once per chunk)
// Barriers: the helpers pass exactly the chain's barriers (two before the loop, one per step,
// one after), so the s_barrier counts of all waves agree.  The last two blocks are flushed by
// the helpers after the loop, and the FB log-likelihood (which needs the running base) is
// written by the last helper.
// items per block.  (An eighth, empty item per block measured 58 ns per step slower on the
// dense FB chain, 828 -> 944 us per op, profiles/r4k_ops.log: the publish rides on item 0.)
template <int KIND>
constexpr int kRbItems = 7;


template <int NP, int KIND>
__device__ __forceinline__ void rec_rb_helper(const RecArgs& a, float* lds, int b) {
  using C = RC<NP>;
  constexpr int NH = kRbHelpers<NP>::NH;
  const int tid = threadIdx.x;
  const int h = (tid >> 6) - C::NW, l = tid & 63, th = tid - C::NT;
  const int T = a.T;
  const int kb0 = 0;
  const int nblocks = (T + 15) / 16;
  // register sets: [set = block & 1][slice 0/1][5]
  float er[2][2][5];
  if (KIND == kVit) rec_logt_fill<NP>(lds, l);
  if (nblocks > kb0 + 1) {
    rec_load<NP, KIND>(a, b, kb0 + 1, 2 * h, l, er[1][0]);
    rec_load<NP, KIND>(a, b, kb0 + 1, 2 * h + 1, l, er[1][1]);
  }
  lds_barrier();  // (the chain's: block 0 staged)
  lds_barrier();  // (the chain's: row 0 written)
  double base = (KIND == kFbBeta && a.bscale) ? (double)a.bscale[b] : 0.0;
  float lsv = 0.f;
  // psi followers (Viterbi, vit_kern.h): the count of flushed blocks, published once per 64-step
  // chunk.  Every helper waits for its own flush stores (a workgroup-scope release: vmcnt(0), no
  // cache maintenance) before the step barrier; one lane of helper 0 then, after the barrier,
  // makes them visible to the other XCDs (an agent-scope release: this XCD's L2 written back)
  // and stores the count.  Agent-scope releases are L2-wide: per block and helper they slowed
  // the whole chip (Viterbi op 0.77 -> 1.79 ms), so there is one per chunk and sequence.
  const bool follow = KIND == kVit && a.prog;
  auto flushed = [&]() {
    if (follow) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  };
  auto publish = [&](int blocks) {
    if (follow && h == 0 && l == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store(a.prog + (size_t)b * kProgSlots, blocks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // item it of block kb; `set` = kb & 1 as a template-free pair of branches over er[0] / er[1]
  auto item = [&](int kb, int it, float(&cur)[2][5], float(&nxt)[2][5]) {
    // cur: block kb + 1's rows (loaded a block ago); nxt: block kb + 2's (loaded now)
    switch (it) {
      case 0:
        if (kb + 1 < nblocks) rec_stage<NP, KIND>(a, lds, kb + 1, 2 * h, l, cur[0]);
        // (Viterbi with psi followers) blocks 0 .. kb - 3 were flushed in block kb - 1, before
        // the barriers since: publish them once per chunk
        if (kb >= kb0 + 3 && ((kb - 2) & 3) == 0) publish(kb - 2);
        break;
      case 1: if (kb + 1 < nblocks) rec_stage<NP, KIND>(a, lds, kb + 1, 2 * h + 1, l, cur[1]); break;
      case 2: rec_load<NP, KIND>(a, b, kb + 2 < nblocks ? kb + 2 : nblocks - 1, 2 * h, l, nxt[0]); break;
      case 3: rec_load<NP, KIND>(a, b, kb + 2 < nblocks ? kb + 2 : nblocks - 1, 2 * h + 1, l, nxt[1]); break;
      case 4: if (kb >= kb0 + 2) lsv = rec_ls_scan<NP, KIND>(a, lds, b, kb - 2, base, h == NH - 1); break;
      case 5: if (kb >= kb0 + 2) rec_flush<NP, KIND>(a, lds, b, kb - 2, th, lsv); break;
      case 6:
        if (kb >= kb0 + 2) {
          rec_flush<NP, KIND>(a, lds, b, kb - 2, th + NH * kWave, lsv);
          flushed();
        }
        break;
      default: break;
    }
  };
  const int qend = nblocks * 16 < T ? nblocks * 16 : T;
  auto run_block = [&](int kb, float(&cur)[2][5], float(&nxt)[2][5]) {
    const int q0 = kb * 16 < 1 ? 1 : kb * 16;
    const int q1 = (kb + 1) * 16 < qend ? (kb + 1) * 16 : qend;
    int it = 0;
    for (int q = q0; q < q1; ++q, ++it) {
      if (it < kRbItems<KIND>) item(kb, it, cur, nxt);
      step_barrier();
    }
    for (; it < kRbItems<KIND>; ++it) item(kb, it, cur, nxt);  // (a short last block)
  };
  // block kb stages block kb + 1 from set (kb + 1) & 1 and loads block kb + 2 into set kb & 1
  for (int k = kb0; k < nblocks; k += 2) {
    run_block(k, er[1], er[0]);
    if (k + 1 < nblocks) run_block(k + 1, er[0], er[1]);
  }
  lds_barrier();  // (the chain's: the last rows and c_{T-1} written)
  static_assert(2 * NH * kWave == C::NT, "two flush passes cover the block");
  if (nblocks >= kb0 + 2) {
    lsv = rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 2, base, h == NH - 1);
    rec_flush<NP, KIND>(a, lds, b, nblocks - 2, th, lsv);
    rec_flush<NP, KIND>(a, lds, b, nblocks - 2, th + NH * kWave, lsv);
  }
  lsv = rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 1, base, h == NH - 1);
  rec_flush<NP, KIND>(a, lds, b, nblocks - 1, th, lsv);
  rec_flush<NP, KIND>(a, lds, b, nblocks - 1, th + NH * kWave, lsv);
  if (follow) {
    flushed();
    __syncthreads();  // (the chain waves have ended: the helpers alone)
    publish(nblocks);
  }
  if (KIND == kFbAlpha && a.loglik && h == NH - 1 && l == 0) {
    a.loglik[b] = (float)(base + (double)__logf(lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))]));
  }
}

// ---------------------------------------------------------------------------------------
// Dense chain, register-blocked form (round 3; every NP).  rec_run_bc gives each lane ONE
// output and 16 inputs per 64-block, so every step moves NP * NP * 4 bytes out of LDS
// (64 KiB at NP = 128: 64 ds_read_b128 = 256 LDS-array cycles, the largest term of its
// ~830-cycle step).  Here each lane owns FOUR outputs and NP/16 inputs, so the same products
// need a quarter of the LDS traffic (2 ds_read_b128 per lane at NP = 128):
//   * wave w, row r (lane >> 4) owns output group g = 4w + r, i.e. outputs 4g .. 4g+3; lane
//     c (lane & 15) of the row owns inputs 64m + 4c .. 64m + 4c + 3 (m < NP/64), read as one
//     float4 per block (the four rows of a wave read the same addresses: broadcasts; the 16
//     lanes of each ds_read_b128 lane group read 16 distinct 16-B slots: conflict-free);
//   * the 4 x NP/16 products per lane run as packed fp32 (v_pk_fma_f32 over input pairs;
//     Viterbi v_pk_add_f32 + v_max3_f32) into four per-output accumulators;
//   * the 16 lanes of a row are reduced by a reduce-scatter of DPP adds / maxes with no
//     selects: register slot k of lane c holds output k ^ (c >> 2) (the matrix slice is loaded
//     in that order), so row_mirror (c <-> 15 - c) pairs slots {0,1} with the partner's {3,2},
//     row_half_mirror (c <-> c ^ 7) slot 0 with the partner's slot 1, and two quad_perms finish:
//     5 DPP operations, after which quad c >> 2 holds output 4g + (c >> 2);
//   * lane (c & 3) == 0 of each quad writes it straight into the row ring (the ring row q is
//     both the exchange buffer the next step reads and the row that is flushed), so a step is
//     2 reads, ~25 (FB) / ~37 (Viterbi) VALU operations, 1 write and one s_barrier.
// Forward-backward keeps Rabiner scaling: c_{q-1} = sum of the step's input vector, formed
// by each row from its 16 lanes' partial sums (4 more DPP adds beside the products, the same
// bits in every row).  Beta's product input v * e sits in Pv[2][NP] (OFF_PART).
template <int NP, int KIND>
__device__ __forceinline__ void rec_run_rb(const RecArgs& a, float* lds, int b) {
  using C = RC<NP>;
  constexpr bool FB = KIND != kVit;
  constexpr int NM = NP / 64;  // float4 input blocks per lane
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x;
  if (tid >= C::NT) {  // the block-work helpers (kRbHelpers)
    rec_rb_helper<NP, KIND>(a, lds, b);
    return;
  }
  // the chain waves issue first: a helper takes the SIMD only while they wait (LDS, barrier)
  // (one priority for all chain waves: the younger half one level above the older half,
  // MI355X_MICROARCH.md "Two waves per SIMD" item 4, measured the same, round 5)
  __builtin_amdgcn_s_setprio(2);
  const int w = tid >> 6, l = tid & 63, r = l >> 4, c = l & 15;
  const int g = 4 * w + r;      // output group
  const int x = c >> 2;         // register slot k holds output 4g + (k ^ x)
  const int o = 4 * g + x;      // the output this lane's quad finishes
  const int T = a.T, N = a.N;
  float* ring = lds + C::OFF_RING;
  float* Pv = lds + C::OFF_PART;  // [2][NP] beta: product input v * e

  // matrix slice: Mk[k][m][p] = (Mat[i][ok], Mat[i+1][ok]) for inputs i = 64m + 4c + 2p,
  // output ok = 4g + (k ^ x); beta takes Mat[ok][i]; FB stores exp(log P)
  f2 Mk[4][NM][2];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 64 * m + 4 * c + e, ok = 4 * g + (k ^ x);
        const bool in = i < N && ok < N;
        const size_t idx = in ? (KIND == kFbBeta ? (size_t)ok * N + i : (size_t)i * N + ok) : 0;
        const float v = a.mat[idx];
        Mk[k][m][e >> 1][e & 1] = FB ? __expf(in ? v : -INFINITY) : (in ? v : -INFINITY);
      }

  const int qend = T;
  const int nblocks = (qend + 15) / 16;
  {
    float er0[5];
    if (KIND == kVit) rec_logt_fill<NP>(lds, l);
    rec_load<NP, KIND>(a, b, 0, w, l, er0);
    rec_stage<NP, KIND>(a, lds, 0, w, l, er0);
  }
  lds_barrier();  // (block 1 on: the helpers stage)

  auto emis = [&](int rho, int idx) { return lds[C::OFF_EMIS + (((rho >> 4) % 3) * 16 + (rho & 15)) * NP + idx]; };
  const bool writer = (c & 3) == 0;
  {
    float v0;
    const int oo = o < N ? o : 0;
    if (KIND == kFbAlpha) v0 = o < N ? __expf(a.init[oo]) * emis(0, o) : 0.f;  // alpha_0 = p0 * e_0
    else if (KIND == kFbBeta) v0 = o < N ? (a.binit ? a.binit[(size_t)b * NP + o] : 1.f) : 0.f;  // beta_{T-1}
    else v0 = o < N ? a.init[oo] + emis(0, o) : -INFINITY;                      // delta_0 = init + lo_0
    if (writer) {
      ring[o] = v0;
      if (KIND == kFbBeta) Pv[o] = v0 * emis(0, o);
    }
  }
  lds_barrier();

  unsigned long long st_acc[4] = {0, 0, 0, 0}, st_prev = 0, st_t0 = 0, st_steps = 0;
  long long rt0 = 0;
  if (kStamp) { st_t0 = stamp(); st_prev = st_t0; rt0 = __builtin_amdgcn_s_memrealtime(); }
  auto mark = [&](int k) {
    if (kStamp) { const unsigned long long t = stamp(); st_acc[k] += t - st_prev; st_prev = t; }
  };

  // one step q of the chain (ring row q from row q - 1)
  auto stepq = [&](int q) {
    if (kStamp) mark(3);
    const float* src = KIND == kFbBeta ? Pv + ((q - 1) & 1) * NP : ring + ((q - 1) & (C::RING - 1)) * NP;
    // alpha / Viterbi: emission of output o; beta: of v_q -> P.  Read first and pinned below:
    // used only by the writer lanes, it would otherwise sink behind the reduction into their
    // branch and put an LDS round trip on the chain
    float eo = emis(q, o);
    f2 yin[NM][2];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const float4 v4 = *reinterpret_cast<const float4*>(src + 64 * m + 4 * c);
      yin[m][0] = f2{v4.x, v4.y};
      yin[m][1] = f2{v4.z, v4.w};
    }
    keep(eo);
    if (kStamp) { keep(yin[0][0]); mark(0); }
    float s0, s1, s2, s3;
    float cs = 0.f;
    if (FB) {
      f2 acc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = f2{0.f, 0.f};
      f2 ysum = f2{0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] = __builtin_elementwise_fma(yin[m][p], Mk[k][m][p], acc[k]);
          ysum += yin[m][p];
        }
      // c_{q-1}: the row's 16 lanes hold all NP inputs; an all-reduce of their sums (every
      // lane, every row and every wave ends with the same bits), interleaved with the outputs'
      // reduction (issue is in order within a wave)
      float cx = ysum.x + ysum.y;
      s0 = acc[0].x + acc[0].y; s1 = acc[1].x + acc[1].y;
      s2 = acc[2].x + acc[2].y; s3 = acc[3].x + acc[3].y;
      red4_add_with_c(s0, s1, s2, s3, cx);
      cs = cx;
    } else {
      // the four packed sums of one input pair first, then their max3 folds: no max waits on
      // the packed add just issued (tools/mb_dense.hip: 329 -> 291 ns per step), and the first
      // pair initialises the maxima (no max against -inf)
      float mx[4];
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          f2 t[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) t[k] = yin[m][p] + Mk[k][m][p];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            mx[k] = (m == 0 && p == 0) ? fmaxf(t[k].x, t[k].y) : fmaxf(fmaxf(mx[k], t[k].x), t[k].y);
        }
      s0 = mx[0]; s1 = mx[1]; s2 = mx[2]; s3 = mx[3];
      red4_max(s0, s1, s2, s3);
    }
    if (kStamp) { keep(s0); mark(1); }
    float val, pval = 0.f;
    if (FB) {
      const float scale = __builtin_amdgcn_rcpf(cs);
      // (every lane holds the same c: wave 0 writes it, a wave-uniform branch)
      if (w == 0) lds[C::OFF_SC + 64 * ((q - 1) & (C::RING - 1))] = cs;
      val = KIND == kFbAlpha ? s0 * (scale * eo) : s0 * scale;  // alpha: u_q = z e_q / c;  beta: v_q = z / c
      if (KIND == kFbBeta) pval = val * eo;
    } else {
      val = s0 + eo;  // delta_q = max(...) + lo_q (exact: monotone)
    }
    // The four lanes of a quad hold the same bits (the last two reduction levels are
    // all-reduces of commutative pairs), so all of them store: no divergent writer branch
    // (tools/mb_dense.hip: 291 -> 268 ns per Viterbi step, 255 -> 229 ns FB)
    ring[(q & (C::RING - 1)) * NP + o] = val;
    if (KIND == kFbBeta) Pv[(q & 1) * NP + o] = pval;
    if (kStamp) { mark(2); ++st_steps; }
    step_barrier();
  };
  auto run_block = [&](int kb) {
    const int q0 = kb * 16 < 1 ? 1 : kb * 16;
    const int q1 = (kb + 1) * 16 < qend ? (kb + 1) * 16 : qend;
    if (q0 == kb * 16 && q1 == q0 + 16) {
      // a whole 16-step block, unrolled: the ring / staging indices of every step are the
      // block's plus a constant, so no per-step scalar index arithmetic (round 5: the rolled
      // loop spent ~20 SALU instructions per step on them; the dense FB op 714 -> 646 us,
      // Viterbi 788 -> 764 us alone at B=32, T=2000, N=128, tools/ab.py, profiles/r5j_ab.log)
#pragma unroll
      for (int i = 0; i < 16; ++i) stepq(kb * 16 + i);
    } else {
      for (int q = q0; q < q1; ++q) stepq(q);
    }
  };
  for (int k = 0; k < nblocks; ++k) run_block(k);
  if (kStamp && (tid & 63) == 0) {
    const unsigned long long t1 = stamp();
    const long long rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o8 = g_rec_stamps + ((size_t)(blockIdx.x * C::NW + w) % kStampWaves) * 8;
    o8[0] = st_acc[0]; o8[1] = st_acc[1]; o8[2] = st_acc[2]; o8[3] = st_acc[3];
    o8[4] = st_steps; o8[5] = t1 - st_t0; o8[6] = t1 - st_t0; o8[7] = (unsigned long long)(rt1 - rt0);
  }
  if (KIND == kFbAlpha && a.loglik && w == C::NW - 1) {
    float ys = 0.f;
#pragma unroll
    for (int m = 0; m < NM; ++m) ys += ring[((T - 1) & (C::RING - 1)) * NP + 64 * m + l];
    const float cs = wave_sum_bcast(ys);
    if (l == 0) lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))] = cs;  // c_{T-1} (loglik only)
  }
  lds_barrier();  // the last blocks' flush and the log-likelihood: the helpers
}

// The banded chain wave (wave 0 of rec_band; waves 0 and 1 of the forward-backward pair
// kernel, fbpair.h): the whole recursion of one sequence in one wave, one lds_barrier per
// 16-step block and one after the last row, matching the helpers' barriers.  `lds` is the
// chain's own RC<NP> layout.
template <int NP, int KIND, int WP, int TD0 = 0, int TW = 0>
__device__ __forceinline__ void band_chain(const RecArgs& a, float* lds, int b, const BandDesc* __restrict__ d) {
  using C = RC<NP>;
  constexpr int NB = C::NBLK;
  constexpr bool FB = KIND != kVit;
  constexpr bool FUSE = KIND == kVit && kVitFused<NP>;
  const int l = threadIdx.x & 63;
  const int T = a.T, N = a.N;
  const int nblocks = (T + 15) / 16;
  // ------------------------------------------------------------------ chain wave
  // Lane l holds the consecutive states s = NB*l + j (j < NB): a window offset of +-1 is
  // then another register of the same lane or ONE DPP lane shift (zero-filled at the wave
  // edge, where the window weight is the neutral element), folded by the compiler into the
  // add / fma that consumes it.  A wave issues one instruction per ~4 cycles, so the step is
  // written for instruction count: 16-step blocks fully unrolled (no scalar address math),
  // the emission read one step ahead, the block's normalisers collected by v_writelane and
  // stored once per block.
  constexpr int WW = TW > 0 ? TW : WP;  // window slots per state
  int lo[NB];
  float wv[NB][WW], fl[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int s = NB * l + j;
    lo[j] = KIND == kFbBeta ? d->rlo[s] : d->clo[s];
#pragma unroll
    for (int k = 0; k < WW; ++k) {
      if (TW > 0)
        wv[j][k] = KIND == kVit ? d->tL[s][k] : (KIND == kFbAlpha ? d->tD[s][k] : d->tR[s][k]);
      else
        wv[j][k] = KIND == kVit ? d->cL[s][k] : (KIND == kFbAlpha ? d->cD[s][k] : d->rD[s][k]);
    }
    fl[j] = KIND == kVit ? d->rfl[s] : d->afl[s];
  }
  const bool uafl = d->uafl != 0;  // one floor for every row: weighted sum = afl0 * plain sum
  const float afl0 = d->afl[0];
  auto erow = [&](int rho) { return lds + C::OFF_EMIS + (((rho >> 4) % 3) * 16 + (rho & 15)) * NP + NB * l; };
  auto ld = [&](const float* p, float(&v)[NB]) {
    if constexpr (NB == 1) v[0] = p[0];
    else if constexpr (NB == 2) { const float2 t = *reinterpret_cast<const float2*>(p); v[0] = t.x; v[1] = t.y; }
    else { const float4 t = *reinterpret_cast<const float4*>(p); v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w; }
  };
  auto st = [&](float* p, const float(&v)[NB]) {
    if constexpr (NB == 1) p[0] = v[0];
    else if constexpr (NB == 2) *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    else *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  };
  float y[NB];
  {
    float e0[NB];
    ld(erow(0), e0);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int s = NB * l + j;
      const int ss = s < N ? s : 0;
      if (KIND == kFbAlpha) y[j] = s < N ? __expf(a.init[ss]) * e0[j] : 0.f;
      else if (KIND == kFbBeta) y[j] = s < N ? (a.binit ? a.binit[(size_t)b * NP + s] : 1.f) : 0.f;
      else y[j] = s < N ? a.init[ss] + e0[j] : -INFINITY;
    }
  }
  float* ybuf = lds + C::OFF_PART;  // beta's LDS window source [2][NP] (LDS-window mode)
  constexpr int EL = KIND == kFbBeta ? 1 : 0;
  float en[NB];  // the next step's emission (alpha / Viterbi e_q, beta e_{q-1})
  float gprev = -INFINITY;  // (diagnostic bit 1 << 24)

  // the value of state s + dd (s = NB*l + j) from register vector v
  auto at = [&](const float(&v)[NB], int j, int dd) -> float {
    const int t = j + dd + 4 * NB;
    const int qq = t / NB - 4, jj = t % NB;
    const int x = __builtin_bit_cast(int, v[jj]);
    if (qq == 0) return v[jj];
    if (qq == -1) return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x138, 0xF, 0xF, true));
    if (qq == 1) return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x130, 0xF, 0xF, true));
    if (qq == -2) {
      const int t1 = __builtin_amdgcn_update_dpp(0, x, 0x138, 0xF, 0xF, true);
      return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, t1, 0x138, 0xF, 0xF, true));
    }
    const int t1 = __builtin_amdgcn_update_dpp(0, x, 0x130, 0xF, 0xF, true);
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, t1, 0x130, 0xF, 0xF, true));
  };

  // UA: uniform floor (alpha), a compile-time branch: a runtime one splits every unrolled
  // step into basic blocks whose joins wait for all outstanding LDS reads
  // Per-step LDS addresses come from per-block bases (row / emission slots of step jj are
  // base + jj * NP: immediate offsets), and the step's normaliser c (FB) / floor maximum M
  // (fused Viterbi psi) goes into lane jj of `blk` by v_writelane, stored once per block
  // (lanes < 16, after the last step): no per-step address arithmetic or scalar-to-vector
  // moves on the chain.
  auto step = [&](int q, int jj, bool last_in_block, auto UA, float* row, const float* enext, float& blk,
                  auto wlane) {
    st(row + NB * l, y);  // row q-1: flushed by the helpers, window source in LDS mode
    float eo[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) eo[j] = en[j];
    if (!last_in_block) ld(enext, en);
    float acc[NB], src[NB];
    float cs = 0.f, scale = 1.f;
    if (KIND == kFbBeta) {  // the product input is y = v * e_{q-1} (hmm.py:113-115)
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j) { src[j] = y[j] * eo[j]; t = j == 0 ? src[j] : t + src[j]; }
      if (TW == 0) st(ybuf + ((q - 1) & 1) * NP + NB * l, src);
      cs = (kAbl & (1 << 23)) ? __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t))) : wave_sum_bcast(t);  // (diag 1 << 23: no reduction)
      // the floor term fl_j * c is folded into the end: y_j = fl_j + (window sum) / c, one fma
      // after the reduction instead of a multiply before the window fmas and one after
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = 0.f;
    } else if (KIND == kFbAlpha) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j) { src[j] = y[j]; t = j == 0 ? y[j] : t + y[j]; }
      cs = (kAbl & (1 << 23)) ? __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t))) : wave_sum_bcast(t);  // (diag 1 << 23: no reduction)
      float sw;
      if constexpr (decltype(UA)::value) {
        sw = 0.f;  // uniform floor: folded into the end as for beta, y = (afl0 + wsum / c) e
      } else {
        float tw = 0.f;
#pragma unroll
        for (int j = 0; j < NB; ++j) tw = fmaf(y[j], fl[j], tw);
        sw = wave_sum_bcast(tw);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = sw;
    } else {
      float g = -INFINITY;
#pragma unroll
      for (int j = 0; j < NB; ++j) { src[j] = y[j]; g = fmaxf(g, y[j] + fl[j]); }
      // (diagnostic timing bits, wrong results: 1 << 23 no reduction, 1 << 24 the reduction of
      // the previous step's values, off the step's dependency chain)
      float M;
      if constexpr (kAbl & (1 << 23)) {
        M = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, g)));
      } else if constexpr (kAbl & (1 << 24)) {
        M = wave_max_bcast(gprev);
        gprev = g;
      } else {
        M = wave_max_bcast(g);
      }
      // fused psi: M_q = max_i fl(delta_{q-1,i} + r_i) is also psi row q's floor maximum
      if constexpr (FUSE) wlane(blk, M);
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = M;
    }
    if (FB) {
      scale = __builtin_amdgcn_rcpf(cs);
      wlane(blk, cs);  // c_{q-1}
    }
    if constexpr (TW > 0) {
#pragma unroll
      for (int k = 0; k < TW; ++k)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const float v = at(src, j, TD0 + k);
          acc[j] = FB ? fmaf(v, wv[j][k], acc[j]) : fmaxf(acc[j], v + wv[j][k]);
        }
    } else {
      const float* wsrc = KIND == kFbBeta ? ybuf + ((q - 1) & 1) * NP : row;
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int k = 0; k < WW; ++k) {
          const float v = wsrc[lo[j] + k];
          acc[j] = FB ? fmaf(v, wv[j][k], acc[j]) : fmaxf(acc[j], v + wv[j][k]);
        }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      // padded states: the staged emission is 0 (FB) / -inf (Viterbi) and the floors 0
      if (KIND == kFbAlpha) {
        if constexpr (decltype(UA)::value) y[j] = fmaf(acc[j], scale, afl0) * eo[j];
        else y[j] = acc[j] * (scale * eo[j]);
      } else if (KIND == kFbBeta) {
        y[j] = fmaf(acc[j], scale, fl[j]);
      } else {
        y[j] = acc[j] + eo[j];
      }
    }
  };

  // (diagnostic builds: cycles at the block barriers, the whole chain, and its real time)
  unsigned long long st_bar = 0, st_t0 = 0;
  long long rt0 = 0;
  if (kStamp) { st_t0 = stamp(); rt0 = __builtin_amdgcn_s_memrealtime(); }
  auto run_blocks = [&](auto UA) {
    for (int kb = 0; kb < nblocks; ++kb) {
      const int q0 = kb * 16 < 1 ? 1 : kb * 16;
      const int q1 = (kb + 1) * 16 < T ? (kb + 1) * 16 : T;
      if (q0 < q1) ld(erow(q0 - EL), en);
      // step jj of this block writes row 16kb + jj - 1: slot (16kb & 63) + jj - 1 for jj >= 1
      // (no wrap inside a block), slot (16kb - 1) & 63 for jj = 0; it loads the emission row
      // of step 16kb + jj + 1 - EL, slot (kb % 3) * 16 + jj + 1 - EL of the staging ring
      float* rbase = lds + C::OFF_RING + ((16 * kb) & (C::RING - 1)) * NP;
      float* rwrap = lds + C::OFF_RING + ((16 * kb - 1) & (C::RING - 1)) * NP;
      const float* ebase = lds + C::OFF_EMIS + ((kb % 3) * 16 + 1 - EL) * NP + NB * l;
      float blk = 0.f;
      if (q0 == kb * 16 && q1 == kb * 16 + 16) {
        static_for<0, 16>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          step(kb * 16 + jj, jj, jj == 15, UA, jj == 0 ? rwrap : rbase + (jj - 1) * NP, ebase + jj * NP, blk,
               [](float& d, float v) { writelane_c<jj>(d, v); });
        });
        // the block's normalisers / floor maxima: lane jj -> row 16kb + jj - 1 (entry 0 of its
        // 64-float slot, where rec_ls_scan / the psi waves / fbpair's scan read it)
        if constexpr (FB || FUSE) {
          if (l < 16) lds[C::OFF_SC + 64 * ((16 * kb + l - 1) & (C::RING - 1))] = blk;
        }
      } else {
        // first and last (partial) blocks: one store per step, as it is computed
        for (int q = q0; q < q1; ++q) {
          const int jj = q - kb * 16;
          float* sc = lds + C::OFF_SC + 64 * ((q - 1) & (C::RING - 1));
          step(q, jj, q + 1 == q1, UA, jj == 0 ? rwrap : rbase + (jj - 1) * NP, ebase + jj * NP, blk,
               [sc](float&, float v) { *sc = v; });
        }
      }
      unsigned long long sb = 0;
      if (kStamp) sb = stamp();
      if (!(kAbl & 16384)) lds_barrier();  // B_{kb+1}: block kb+1 staged by the helpers, rows of block kb-1 written
      if (kStamp) st_bar += stamp() - sb;
    }
  };
  if constexpr (KIND == kFbAlpha) {
    if (uafl) run_blocks(std::true_type{});
    else run_blocks(std::false_type{});
  } else {
    run_blocks(std::false_type{});
  }
  if (kStamp && l == 0) {
    const unsigned long long t1 = stamp();
    const long long rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o8 = g_rec_stamps + ((size_t)blockIdx.x * 16 % kStampWaves) * 8;
    o8[0] = (unsigned long long)rt0; o8[1] = (unsigned long long)rt1; o8[3] = st_bar;
    o8[4] = T; o8[5] = t1 - st_t0; o8[6] = t1 - st_t0; o8[7] = (unsigned long long)(rt1 - rt0);
  }
  float* row = lds + C::OFF_RING + ((T - 1) & (C::RING - 1)) * NP;
  st(row + NB * l, y);
  if (KIND == kFbAlpha && a.loglik) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < NB; ++j) t += y[j];
    const float cs = wave_sum_bcast(t);
    if (l == 0) lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))] = cs;
  }
  lds_barrier();
}

// ---------------------------------------------------------------------------------------
// Banded chain (band.h).  Wave 0 runs the whole recursion; lane l owns states
// s = 64*blk + l.  Per step: the previous row goes to the LDS ring (it is both the window
// source and the row that is flushed), one DPP wave reduction (sum / weighted sum / max)
// runs beside the W window reads, then W fma / add+max per state.  No s_barrier inside the
// 16-step block: LDS accesses of one wave complete in order.  Waves 1..NW-1 are helpers:
// during block kb they stage the emissions of block kb+1 (log / +1e-8 transform included),
// issue the global loads of block kb+3 and flush the rows and log-scales of block kb-2, so
// the chain wave issues no global memory operation and no transcendental of the staging.
// All waves meet at one s_barrier per 16 steps.
template <int NP, int KIND, int WP, int TD0 = 0, int TW = 0>
__device__ __forceinline__ void rec_band(const RecArgs& a, float* lds, int b, const BandDesc* __restrict__ d) {
  using C = RC<NP>;
  constexpr int NB = C::NBLK;
  // Waves 1..3 are the helpers (forward-backward); waves 4.. exit at once, so the chain wave
  // is alone on its SIMD (a workgroup's waves are spread over the 4 SIMDs).  Ended waves do
  // not take part in s_barrier.
  // The Viterbi staging also takes the emission log (logcr.h), so it runs on a fourth helper,
  // wave 4, beside the chain on SIMD 0: measured alone, 3 helpers 259 us, 4 helpers 238 us,
  // the separate log pass 248 us (B=32, T=2000, N=128); 3 of the 8 virtual waves on wave 4
  // and 5 on waves 1..3 was slower (262 us).
  // Round 3, fused-psi Viterbi (kVitFused, NP >= 128): the workgroup has 16 waves (kVitWideNT).
  // With the chain's step down to ~95 ns its helpers had become the limit (one process,
  // B=32 T=2000 N=128: Viterbi op 242 us; without the emission log 209, without the psi rows
  // 195, neither 189; tools/ablate.py, profiles/r3g_ablate.log), so SIMDs 1..3 each carry
  // TWO staging helpers (waves 1,2,3 and 9,10,11) and TWO psi waves (5,6,7 and 13,14,15), and
  // nothing shares the chain's SIMD: waves 4, 8, 12 (w = 0 mod 4, the chain's SIMD) exit.
  // Round 6, forward-backward (FBW): every wave of the launch off the chain's SIMD stages
  // (waves 1,2,3, 5,6,7, 9,10,11 of kFbNT<128>: one virtual staging wave each).  With three
  // helpers of three virtual waves, helper 1's block work took ~3.4 k cycles, the chain's 16
  // steps ~3.2 k, and the chains waited 18 (beta) / 28 (alpha) cycles a step at the block
  // barrier (tools/band_stamps.py).
  constexpr bool FUSE = KIND == kVit && kVitFused<NP>;
  constexpr bool WIDE = FUSE;
  constexpr bool FBW = KIND != kVit;
  constexpr int NWB = kFbNT<NP> / kWave;  // (FBW) the launch's waves
  constexpr int NH = WIDE ? 6 : FBW ? (NWB / 4) * 3 + (NWB % 4 > 1 ? NWB % 4 - 1 : 0)
                                    : ((KIND == kVit && C::NW >= 8) ? 4 : 3);  // (NP = 64: a 4-wave workgroup)
  constexpr int HV = (C::NW + NH - 1) / NH;  // virtual staging waves per helper
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  // role of wave w: staging helper index hi (0 .. NH-1), psi wave index, or neither (exit)
  const int grp = (w >> 3) * 3 + (w & 3) - 1;  // WIDE: waves 1,2,3 / 5,6,7 -> 0,1,2; 9,.. / 13,.. -> 3,4,5
  const bool stager = WIDE ? ((w & 4) == 0 && (w & 3) != 0) : FBW ? (w & 3) != 0 : (w > 0 && w <= NH);
  const bool psiw = WIDE && (w & 4) != 0 && (w & 3) != 0;
  const int hi = WIDE ? grp : FBW ? (w >> 2) * 3 + (w & 3) - 1 : w - 1;
  auto vw_of = [&](int h) -> int { return hi + h * NH; };  // virtual staging wave h of this helper
  constexpr bool FB = KIND != kVit;
  if (w != 0 && !stager && !psiw) return;  // ended waves take no part in s_barrier
  const int T = a.T, N = a.N;
  const int nblocks = (T + 15) / 16;
  double base = (KIND == kFbBeta && a.bscale) ? (double)a.bscale[b] : 0.0;

  // prologue: the helpers stage block 0 and load blocks 1 and 2
  // three register sets: the loads of block kb+3 are issued during block kb, so each has two
  // blocks (~3 us) to land before it is staged
  float er0[HV][5], er1[HV][5], er2[HV][5];
  if (stager) {
    if (KIND == kVit) rec_logt_fill<NP>(lds, l);
#pragma unroll
    for (int h = 0; h < HV; ++h) {
      const int vw = vw_of(h);
      if (vw < C::NW) {
        float er[5];
        rec_load<NP, KIND>(a, b, 0, vw, l, er);
        rec_stage<NP, KIND, FUSE>(a, lds, 0, vw, l, er);
        if (nblocks > 1) rec_load<NP, KIND>(a, b, 1, vw, l, er1[h]);
        if (nblocks > 2) rec_load<NP, KIND>(a, b, 2, vw, l, er2[h]);
      }
    }
  }
  lds_barrier();

  if (w == 0) {
    band_chain<NP, KIND, WP, TD0, TW>(a, lds, b, d);
    return;
  }
  // ---------------------------------------------------------------- helper waves
  // Fused psi (vit_psi_kernel's banded rule, psi_band_rows in viterbi.hip), on the
  // psi-only waves 5..7 and 13..15 (SIMDs 1..3, so neither the chain nor the staging helpers
  // lose issue slots).  With g_i = fl(delta_{t-1,i} + r_i) and M = max g (the chain's own floor
  // term, left in LDS), i1 = first index with g_i == M is a ballot + s_ff1, and psi_t[o] is the
  // first index attaining max(M, window values), i1 when M attains it.  The window is the
  // chain's: Toeplitz offsets TD0.. (TW > 0) or the column windows clo_o .. clo_o + WP.
  // Lane l owns outputs o = NB*l + j.  Rows r == grp (mod 6) of the block; a wave's rows are
  // computed without branches so their latencies overlap.  The rows go to the LDS ring OFF_PSR
  // (the last 64 steps); the staging helpers copy each block of them to HBM (psi_copy).
    constexpr int PWN = TW > 0 ? TW : WP;  // window slots per output
    [[maybe_unused]] float prf[NB];
    [[maybe_unused]] int plo[NB];
    [[maybe_unused]] float pcl[NB][PWN];
    if constexpr (FUSE) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int o = NB * l + j;
        prf[j] = o < N ? d->rfl[o] : -INFINITY;  // -inf: padded states never attain M
        plo[j] = TW > 0 ? o + TD0 : d->clo[o];
#pragma unroll
        for (int kk = 0; kk < PWN; ++kk) {
          const int i = plo[j] + kk;
          pcl[j][kk] = (i >= 0 && i < N && o < N) ? (TW > 0 ? d->tL[o][kk] : d->cL[o][kk]) : -INFINITY;
        }
      }
      // resolve the table loads here, once: left pending, the waitcnt pass would re-wait for
      // them inside the loop with a vmcnt that also drains in-flight memory operations
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        keep(prf[j]);
        keep(plo[j]);
#pragma unroll
        for (int kk = 0; kk < PWN; ++kk) keep(pcl[j][kk]);
      }
    }
    auto psi_rows = [&](int bk) {
      if constexpr (FUSE) {
        if (bk < 0 || (kAbl & 128)) return;
        constexpr int NPW = WIDE ? 6 : 3, PR = (16 + NPW - 1) / NPW;
        const int hw = grp;
#pragma unroll
        for (int m = 0; m < PR; ++m) {
          const int r = hw + NPW * m;
          int t = 16 * bk + (r < 16 ? r : 15);
          t = t < T ? t : T - 1;
          const int rho = (t - 1) & (C::RING - 1);
          const float* drow = lds + C::OFF_RING + rho * NP;
          // no guards around the LDS reads (out-of-range slots carry -inf in prf / pcl): a
          // read under a guard ends in an s_waitcnt vmcnt(0) join
          float yv[NB], xw[NB][PWN];
          if constexpr (NB == 2) {
            const float2 v2 = *reinterpret_cast<const float2*>(drow + NB * l);
            yv[0] = v2.x; yv[1] = v2.y;
          } else {
            const float4 v4 = *reinterpret_cast<const float4*>(drow + NB * l);
            yv[0] = v4.x; yv[1] = v4.y; yv[2] = v4.z; yv[3] = v4.w;
          }
          const float M = lds[C::OFF_SC + 64 * rho];  // the chain's floor maximum of row rho (broadcast read)
#pragma unroll
          for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int kk = 0; kk < PWN; ++kk) {
              const int i = plo[j] + kk;
              xw[j][kk] = drow[i < 0 ? 0 : (i < NP ? i : NP - 1)];
            }
          int i1 = 0x7fffffff;
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const float g = yv[j] + prf[j];
            const unsigned long long hit = __ballot(g == M);
            const int c = NB * (__ffsll((long long)hit) - 1) + j;
            i1 = (hit && c < i1) ? c : i1;
          }
          unsigned pk = 0;
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            float v = M, val[PWN];
#pragma unroll
            for (int kk = 0; kk < PWN; ++kk) {
              val[kk] = xw[j][kk] + pcl[j][kk];  // -inf outside [0, N)
              v = fmaxf(v, val[kk]);
            }
            int arg = M == v ? i1 : 0x7fffffff;
#pragma unroll
            for (int kk = 0; kk < PWN; ++kk)
              if (val[kk] == v && plo[j] + kk < arg) arg = plo[j] + kk;
            arg = (NB * l + j < N && t > 0) ? arg : 0;  // psi_0 = 0 (hmm.py:156 zeros)
            pk |= (unsigned)arg << (8 * j);
          }
          if (r < 16 && 16 * bk + r < T) {
            // the LDS ring of the last 64 rows; the staging helpers copy whole blocks of it to
            // HBM with 16-B stores (psi_copy)
            uint8_t* ldst = reinterpret_cast<uint8_t*>(lds + C::OFF_PSR) + (t & (C::PSR - 1)) * NP + NB * l;
            if constexpr (NB == 2) *reinterpret_cast<uint16_t*>(ldst) = (uint16_t)pk;
            else *reinterpret_cast<uint32_t*>(ldst) = pk;
          }
        }
      }
    };
    // Publishing (a.pub, follow.h): the flushes of the rows (FB: U / V, Viterbi: delta) and the
    // copies of the psi rows are write-through stores, and a wave's vector-memory counter retires
    // in issue order, so the compiler's wait for a register set's loads at its staging also
    // retires every store issued before those loads.  The loads of block k + 4 are issued in
    // block_work(k + 1), after block_work(k)'s flush of block k - 2 and psi copy of block k - 3, and
    // they are staged (waited for) in block_work(k + 3): after the barrier that ends it those
    // stores are complete in every helper, and in block_work(k + 4) one lane publishes the count.
    // (The stores are never waited for sooner: a write-through store retires late, and a helper
    // stalled on it stalls the chain at the next barrier.)
    const bool pubon = a.pub != nullptr;
    int* const pubp = pubon ? a.pub + (FB ? 2 * b + (KIND == kFbBeta) : b) * kPubStride : nullptr;
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t psi_rs =
        FUSE ? make_rsrc(a.psi + (size_t)b * T * NP, (size_t)T * NP) : make_rsrc(a.obs, 0);
    // copy the 16 psi rows of block bk from the LDS ring to HBM, one 16-B sc1 store per lane
    // (the last helpers' lanes: 16 * NP / 16 of them)
    [[maybe_unused]] auto psi_copy = [&](int bk) {
      if constexpr (FUSE) {
        constexpr int PER = NP / 16;  // 16-B pieces per row
        const int hidx = (NH - 1 - hi) * 64 + l;
        const int r = hidx / PER, pc = hidx % PER;
        const int t = 16 * bk + r;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint8_t*>(lds + C::OFF_PSR) +
                                                            (t & (C::PSR - 1)) * NP + 16 * pc);
        if (bk >= 0 && hidx < 16 * PER && t < T)
          __builtin_amdgcn_raw_buffer_store_b128(v, psi_rs, t * NP + 16 * pc, 0, (kFAbl & 4) ? 0 : kAuxSc1);
      }
    };
    // Straight-line block work (no branch around the staging or the loads: the tail stages
    // a block past the end as padding and re-loads the last block), so the waitcnt pass
    // keeps exact counts and never drains the in-flight prefetches or the flush stores.
    // Viterbi with log leaders: `lp` holds the leaders' count as polled three blocks ago (read
    // here, where the staging's wait has already retired that poll, so it never stalls the
    // helper), and takes this block's poll.
    // (diagnostic builds: a helper's cycles of block work and at the barrier)
    unsigned long long hs_work = 0, hs_wait = 0;
    auto block_work = [&](int kb, float(&ernext)[HV][5], float(&erfree)[HV][5], int& lp, auto FULLC) {
      asm volatile("" ::: "memory");  // (block_work(kb - 1)'s stores stay ahead of this block's loads)
      unsigned long long hs0 = 0;
      if (kStamp) hs0 = stamp();
      const int kload = kb + 3 < nblocks ? kb + 3 : nblocks - 1;
      // the block's log-scales once per helper (its own base); helper 1 writes LA / LB
      float lsv = 0.f;
      if (!(kAbl & 32) && kb >= 2) lsv = rec_ls_scan<NP, KIND>(a, lds, b, kb - 2, base, w == 1);
      // Viterbi: the block's source -- the leaders' log rows when they are ready, else the raw
      // emissions (the staging takes the log)
      const bool fromlog = KIND == kVit && a.lobuf && kload >= 4 && lp >= kload + 1;
      const float* src = fromlog ? a.lobuf : a.obs;
      const float vmode = (fromlog || a.obs_mode == HMM355_OBS_LOG) ? 1.f : 0.f;
#pragma unroll
      for (int h = 0; h < HV; ++h) {
        const int vw = vw_of(h);
        if (vw < C::NW && !(kAbl & 32768)) {
          if (!(kAbl & 64)) {
            rec_stage<NP, KIND, FUSE>(a, lds, kb + 1, vw, l, ernext[h]);
            rec_load<NP, KIND, decltype(FULLC)::value, FUSE>(a, b, kload, vw, l, erfree[h], src, vmode);
          }
          if (!(kAbl & 32) && kb >= 2) rec_flush<NP, KIND>(a, lds, b, kb - 2, l + 64 * vw, lsv);
        }
      }
      psi_copy(kb - 3);
      if (KIND == kVit && a.lready) lp = poll_count(a.lready + b * kPubStride, a.token, nblocks);
      // every fourth block (Viterbi: whole 64-step chunks of psi rows), after this block's loads
      // (so the stores it signals are never waited for sooner than three blocks on)
      if (pubon && !(kFAbl & 1) && hi == 0 && l == 0) {
        const int cnt = FB ? kb - 5 : kb - 6;
        if (cnt > 0 && (cnt & 3) == 0) publish_count(pubp, cnt, a.token);
      }
      unsigned long long hs1 = 0;
      if (kStamp) { hs1 = stamp(); hs_work += hs1 - hs0; }
      if (!(kAbl & 16384)) lds_barrier();
      if (kStamp) hs_wait += stamp() - hs1;
    };
    if constexpr (FUSE) {
      if (psiw) {  // psi-only waves: one compact loop, same barrier count as the helpers
        for (int kb = 0; kb < nblocks; ++kb) {
          psi_rows(kb - 2);
          if (!(kAbl & 16384)) lds_barrier();
        }
        lds_barrier();  // the chain's last row
        psi_rows(nblocks - 2);
        psi_rows(nblocks - 1);
        lds_barrier();  // the last psi rows are in the ring (the helpers copy them)
        return;
      }
    }
    int lp0 = 0, lp1 = 0, lp2 = 0;  // the leaders' polls (block kb's is read at kb + 3)
    auto helper_loop = [&](auto FULLC) {
      for (int kb = 0; kb < nblocks; kb += 3) {
        block_work(kb, er1, er0, lp0, FULLC);
        if (kb + 1 < nblocks) block_work(kb + 1, er2, er1, lp1, FULLC);
        if (kb + 2 < nblocks) block_work(kb + 2, er0, er2, lp2, FULLC);
      }
    };
    if (a.N == NP && (reinterpret_cast<uintptr_t>(a.obs) & 15) == 0 &&
        (!a.lobuf || (reinterpret_cast<uintptr_t>(a.lobuf) & 15) == 0))
      helper_loop(std::true_type{});
    else
      helper_loop(std::false_type{});
    if (kStamp && l == 0 && stager) {
      unsigned long long* o8 = g_rec_stamps + (((size_t)blockIdx.x * 16 + w) % kStampWaves) * 8;
      o8[0] = hs_work; o8[1] = hs_wait; o8[4] = (unsigned long long)nblocks;
    }
    lds_barrier();  // the chain's last row and c_{T-1}
    if (FB && pubon && nblocks > 6) {
      // the loop's flushes (blocks < nblocks - 2) retired: published now, so the followers form
      // those rows while the last two blocks are flushed (the final count comes after them)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // (the chain wave has ended: the helpers alone)
      if (hi == 0 && l == 0) publish_count(pubp, nblocks - 2, a.token);
    }
    const float lsv2 = nblocks >= 2 ? rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 2, base, w == 1) : 0.f;
    const float lsv1 = rec_ls_scan<NP, KIND>(a, lds, b, nblocks - 1, base, w == 1);
    if (FB && pubon) {
      // the last two blocks' rows first, then completion published, then their exp outputs
      // (the followers read only the rows)
#pragma unroll
      for (int h = 0; h < HV; ++h) {
        const int vw = vw_of(h);
        if (vw < C::NW) {
          if (nblocks >= 2) rec_flush<NP, KIND, 1>(a, lds, b, nblocks - 2, l + 64 * vw, lsv2);
          rec_flush<NP, KIND, 1>(a, lds, b, nblocks - 1, l + 64 * vw, lsv1);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // (the chain wave has ended: the helpers alone)
      if (hi == 0 && l == 0) publish_count(pubp, nblocks + 1, a.token);
      if (kStamp && hi == 0 && l == 0) g_rec_stamps[((size_t)blockIdx.x * 16 % kStampWaves) * 8 + 2] = __builtin_amdgcn_s_memrealtime();
    }
#pragma unroll
    for (int h = 0; h < HV; ++h) {
      const int vw = vw_of(h);
      if (vw < C::NW) {
        if (FB && pubon) {
          if (nblocks >= 2) rec_flush<NP, KIND, 2>(a, lds, b, nblocks - 2, l + 64 * vw, lsv2);
          rec_flush<NP, KIND, 2>(a, lds, b, nblocks - 1, l + 64 * vw, lsv1);
        } else {
          if (nblocks >= 2) rec_flush<NP, KIND>(a, lds, b, nblocks - 2, l + 64 * vw, lsv2);
          rec_flush<NP, KIND>(a, lds, b, nblocks - 1, l + 64 * vw, lsv1);
        }
        if (KIND == kFbAlpha && a.loglik && vw == C::NW - 1 && l == 0)
          a.loglik[b] = (float)(base + (double)__logf(lds[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))]));
      }
    }
    if constexpr (KIND == kFbAlpha) {
      // the reference's compute_likelihood, logsumexp_j log(forward_{T-1}[j] + 1e-8)
      // (hmm.py:206), from the last row in LDS and its log-scale: post.h's arithmetic
      if (a.lik_ref && hi == 0) {
        const float ls = __shfl(lsv1, (T - 1) & 15);
        const float* u = lds + C::OFF_RING + ((T - 1) & (C::RING - 1)) * NP;
        float lv[NB], m = -INFINITY;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          const int j = l + 64 * k;
          lv[k] = j < N ? __logf(__expf(__logf(u[j]) + ls) + 1e-8f) : -INFINITY;
          m = fmaxf(m, lv[k]);
        }
        m = wave_max(m);
        float e = 0.f;
#pragma unroll
        for (int k = 0; k < NB; ++k) e += (l + 64 * k < N) ? __expf(lv[k] - m) : 0.f;
        e = wave_sum(e);
        if (l == 0) a.lik_ref[b] = m + __logf(e);
      }
    }
    if constexpr (FUSE) {
      // the psi rows of the last three blocks (the loop copied up to block nblocks - 4)
      psi_copy(nblocks - 3);
      lds_barrier();  // the psi waves' last rows
      psi_copy(nblocks - 2);
      psi_copy(nblocks - 1);
    }
    if (!FB && pubon) {
      // everything stored: every helper's stores retired, then one lane publishes completion
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // (the chain and psi waves have ended: the helpers alone)
      if (hi == 0 && l == 0) publish_count(pubp, nblocks + 1, a.token);
      if (kStamp && hi == 0 && l == 0) g_rec_stamps[((size_t)blockIdx.x * 16 % kStampWaves) * 8 + 2] = __builtin_amdgcn_s_memrealtime();
    }
}

// Which chain serves a recursion (band.h): Toeplitz register windows when the window is a
// fixed offset range instantiated below (code 16*TW + TD0 + 2), else banded with LDS windows
// of the padded width (2/4/8), else the dense chain (0).
template <int KIND, int NP>
__device__ __forceinline__ int rec_band_code(const RecArgs& a) {
  if (!a.band) return 0;
  const BandDesc* d = a.band;
  const int W = KIND == kFbBeta ? d->wr : d->wc;
  if (W > kBandMax) return 0;
  const int tw = KIND == kFbBeta ? d->trw : d->tcw;
  const int td0 = KIND == kFbBeta ? d->trd0 : d->tcd0;
  if (NP <= 128 && tw > 0) {
    const int code = 16 * tw + td0 + 2;
    switch (code) {
      case 16 * 1 + 0 + 2: case 16 * 2 - 1 + 2: case 16 * 2 + 0 + 2:
      case 16 * 3 - 2 + 2: case 16 * 3 - 1 + 2: case 16 * 3 + 0 + 2: return code;
      default: break;
    }
  }
  return KIND == kFbBeta ? d->wrp : d->wcp;
}

template <int NP, int KIND>
__device__ __forceinline__ void rec_dispatch(const RecArgs& a, float* lds, int b) {
  const int code = rec_band_code<KIND, NP>(a);
  // the banded chains are written for RC<NP>::NT threads (the fused Viterbi form for 1024)
  constexpr int kBandNT = (KIND == kVit && kVitFused<NP>) ? 1024 : (KIND != kVit ? kFbNT<NP> : RC<NP>::NT);
  if (code != 0 && threadIdx.x >= kBandNT) return;
  switch (code) {
    case 2: rec_band<NP, KIND, 2>(a, lds, b, a.band); break;
    case 4: rec_band<NP, KIND, 4>(a, lds, b, a.band); break;
    case 8: rec_band<NP, KIND, 8>(a, lds, b, a.band); break;
    case 16 * 1 + 0 + 2: rec_band<NP, KIND, 2, 0, 1>(a, lds, b, a.band); break;
    case 16 * 2 - 1 + 2: rec_band<NP, KIND, 2, -1, 2>(a, lds, b, a.band); break;
    case 16 * 2 + 0 + 2: rec_band<NP, KIND, 2, 0, 2>(a, lds, b, a.band); break;
    case 16 * 3 - 2 + 2: rec_band<NP, KIND, 2, -2, 3>(a, lds, b, a.band); break;
    case 16 * 3 - 1 + 2: rec_band<NP, KIND, 2, -1, 3>(a, lds, b, a.band); break;
    case 16 * 3 + 0 + 2: rec_band<NP, KIND, 2, 0, 3>(a, lds, b, a.band); break;
    default:
      // (diagnostic ablation bits: 1 << 25 the round-2 register-operand chain (NP <= 128),
      // 1 << 24 the DPP-broadcast chain)
      // (NP = 256 keeps the DPP-broadcast chain: 16 waves leave 128 VGPRs a lane, too few for
      // the register-blocked slices)
      if constexpr (NP <= 128 && !(kAbl & (3 << 24))) {
        if (threadIdx.x >= kRbHelpers<NP>::NT) return;  // (waves beyond the chain and its helpers)
        rec_run_rb<NP, KIND>(a, lds, b);
      } else {
        if (threadIdx.x >= RC<NP>::NT) return;
        if constexpr (NP <= 128 && !(kAbl & (1 << 24))) rec_run_bc<NP, KIND>(a, lds, b);
        else rec_run<NP, KIND>(a, lds, b);
      }
      break;
  }
}

}  // namespace hmm355
