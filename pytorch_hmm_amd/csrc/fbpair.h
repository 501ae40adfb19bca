// hmm355 — forward-backward with both chains of a sequence in ONE workgroup, and the
// posterior formed inside it (banded matrices; reference hmm.py:89-130).
//
// fb_recur_kernel + fb_posterior_kernel write the scaled alpha and beta rows U, V of every
// time step to HBM and read them back (2 x 33 MB each way at B=32, T=2000, N=128).  Here one
// workgroup per sequence runs the alpha chain on wave 0 (SIMD 0) and the beta chain on wave
// 1 (SIMD 1), each in its own half of the CU's LDS (the RC<NP> layout of recur.h).  The two
// chains advance one 16-step block per barrier in lockstep, so time t is reached by alpha
// in block t/16 and by beta in block (T-1-t)/16.  Helper waves 2..15 stage both chains'
// emissions and, for every finished row, write forward = exp(log u + LA) / backward =
// exp(log v + LB) straight from the LDS ring.  The posterior of time t needs both rows:
//   - the chain that reaches t FIRST stores its scaled row to HBM (half the rows of each);
//   - the chain that reaches t SECOND reads that row back and writes the posterior;
//   - when both flush t in the same block interval (the middle of the sequence) both rows
//     are still in the LDS rings and nothing goes through HBM.
// Row t of either chain is always handled by helper wave 2 + (t mod 14), so the HBM row is
// written and read back by the same wave (program order: no cross-wave fence).  The reads
// are issued two block intervals ahead.  Scratch traffic drops from
// 4 x 33 MB to 2 x 33 MB and the separate posterior pass (a 26 us launch) disappears.
//
// Stores and the scratch reads use raw buffer operations: a lane or row that must not write
// gets an out-of-range offset (stores dropped, loads return 0), so the helpers' code stays
// straight-line.
//
// Host side (fb.hip): used when the caller sets HMM355_FB_PAIR (the plan is banded in both
// directions, hmm355_plan_banded) and N <= 128.  If the device nevertheless finds a dense
// chain (a wrong hint) the workgroup runs the two dense chains one after the other and the
// posterior rows itself: correct, only slower.
#pragma once
#include "recur.h"
#include "post.h"

namespace hmm355 {

template <int NP>
struct PairL {
  static constexpr int OFF_B = (RC<NP>::LDS_FLOATS + 63) / 64 * 64;  // the beta chain's RC layout
  static constexpr int LDS_FLOATS = 2 * OFF_B;
  static_assert(LDS_FLOATS * 4 <= (int)kExclusiveLds, "pair LDS layout too large");
  static constexpr int NT = 1024;  // 16 waves: 2 chains + 14 helpers (4 waves per SIMD, <= 128 VGPRs)
};

struct PairArgs {
  RecArgs fa, fb;  // alpha / beta chains (rows: U / V scratch with stride NP; ls: LA / LB)
  float* posterior;
  float* forward;
  float* backward;
  float* lik_ref;
  unsigned mask;
};

// the type the b64 buffer builtins take and return (a GCC vector: an ext_vector_type(2) here
// converts element-wise from a splat and loses the second dword)
typedef unsigned int u32x2_t __attribute__((__vector_size__(2 * sizeof(unsigned int))));
constexpr int kBufOOB = 0x7FFFFFF0;  // a byte offset past every num_records: store dropped, load 0
constexpr int kBufNT = (kAbl & (1 << 30)) ? 0 : 2;  // gfx950 cache policy: non-temporal (diag 1 << 30: default)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <int K, int AUX>
__device__ __forceinline__ void buf_store(__amdgpu_buffer_rsrc_t r, int off, const float (&v)[K]) {
  if constexpr (K == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[0]), r, off, 0, AUX);
  } else {
    const float2 f = make_float2(v[0], v[1]);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, f), r, off, 0, AUX);
  }
}
template <int K>
__device__ __forceinline__ void buf_load(__amdgpu_buffer_rsrc_t r, int off, float (&v)[K]) {
  if constexpr (K == 1) {
    v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
  } else {
    const float2 f = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    v[0] = f.x;
    v[1] = f.y;
  }
}

template <int NP, int KIND>
__device__ __forceinline__ void band_chain_dispatch(const RecArgs& a, float* lds, int b, int code) {
  switch (code) {
    case 2: band_chain<NP, KIND, 2>(a, lds, b, a.band); break;
    case 4: band_chain<NP, KIND, 4>(a, lds, b, a.band); break;
    case 8: band_chain<NP, KIND, 8>(a, lds, b, a.band); break;
    case 16 * 1 + 0 + 2: band_chain<NP, KIND, 2, 0, 1>(a, lds, b, a.band); break;
    case 16 * 2 - 1 + 2: band_chain<NP, KIND, 2, -1, 2>(a, lds, b, a.band); break;
    case 16 * 2 + 0 + 2: band_chain<NP, KIND, 2, 0, 2>(a, lds, b, a.band); break;
    case 16 * 3 - 2 + 2: band_chain<NP, KIND, 2, -2, 3>(a, lds, b, a.band); break;
    case 16 * 3 - 1 + 2: band_chain<NP, KIND, 2, -1, 3>(a, lds, b, a.band); break;
    default: band_chain<NP, KIND, 2, 0, 3>(a, lds, b, a.band); break;  // 16 * 3 + 0 + 2
  }
}

// Wrong-hint fallback: the dense chains one after the other (rec_run_rb writes U/LA and V/LB),
// then the posterior rows of this sequence, one wave per row.
template <int NP>
__device__ __forceinline__ void fb_pair_dense(const PairArgs& p, float* lds, int b) {
  constexpr int K = NP / 64;
  // rec_run_rb's NW chain waves and NH block-work helpers (ended waves skip barriers)
  constexpr int NWD = kRbHelpers<NP>::NT / kWave;
  static_assert(kRbHelpers<NP>::NT <= PairL<NP>::NT, "the pair launch holds the dense chain's helpers");
  if ((int)(threadIdx.x >> 6) >= NWD) return;
  rec_run_rb<NP, kFbAlpha>(p.fa, lds, b);
  __syncthreads();
  rec_run_rb<NP, kFbBeta>(p.fb, lds, b);
  __syncthreads();
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int T = p.fa.T, N = p.fa.N;
  for (int t = w; t < T; t += NWD) {
    const size_t row = (size_t)b * T + t;
    float u[K], v[K], mu = 0.f, mv = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      u[k] = p.fa.rows[row * NP + K * l + k];
      v[k] = p.fb.rows[row * NP + K * l + k];
      mu = fmaxf(mu, u[k]);
      mv = fmaxf(mv, v[k]);
    }
    mu = wave_max(mu);
    mv = wave_max(mv);
    const float iu = mu > 0.f ? 1.f / mu : 0.f, iv = mv > 0.f ? 1.f / mv : 0.f;
    float pp[K], s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { pp[k] = (u[k] * iu) * (v[k] * iv); s += pp[k]; }
    s = wave_sum(s);
    const float is = s > 0.f ? 1.f / s : 0.f;
    const float la = p.fa.ls[row], lb = p.fb.ls[row];
    float lv = -INFINITY, lm;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = K * l + k;
      const float fw = __expf(__logf(u[k]) + la);
      if (j < N) {
        if (p.mask & HMM355_FB_POSTERIOR) p.posterior[row * N + j] = pp[k] * is;
        if (p.mask & HMM355_FB_FORWARD) p.forward[row * N + j] = fw;
        if (p.mask & HMM355_FB_BACKWARD) p.backward[row * N + j] = __expf(__logf(v[k]) + lb);
        lv = fmaxf(lv, __logf(fw + 1e-8f));
      }
    }
    if (t == T - 1 && p.lik_ref) {  // hmm.py:206
      lm = wave_max(lv);
      float e = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (K * l + k < N) e += __expf(__logf(__expf(__logf(u[k]) + la) + 1e-8f) - lm);
      e = wave_sum(e);
      if (l == 0) p.lik_ref[b] = lm + __logf(e);
    }
  }
}

template <int NP>
__global__ void __launch_bounds__(PairL<NP>::NT) fb_pair_kernel(PairArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using C = RC<NP>;
  using PL = PairL<NP>;
  constexpr int K = NP / 64;   // states per lane in a row task (contiguous: K*l .. K*l+K-1)
  constexpr int NW = C::NW;    // staging units per chain
  // Helpers are waves 2..15; each stages up to HV of the 2*NW staging units and owns the rows
  // of the times t with t % 14 == w - 2 in both chains.  The row work is latency-bound per
  // wave (a read, a wave sum, stores), so it is spread over as many waves as the CU holds
  // (measured: 4 task waves 0.46 ms, 6 waves 0.38 ms per B=32, T=2000 call).
  constexpr int NH = PL::NT / 64 - 2;          // 14 helpers
  constexpr int RQ = (16 + NH - 1) / NH;       // rows per chain per block per helper
  constexpr int HV = (2 * NW + NH - 1) / NH;   // staging units per helper
  const int b = blockIdx.x;
  const int ca = rec_band_code<kFbAlpha, NP>(p.fa), cb = rec_band_code<kFbBeta, NP>(p.fb);
  if (ca == 0 || cb == 0) {
    fb_pair_dense<NP>(p, lds, b);
    return;
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  float* la = lds;
  float* lb = lds + PL::OFF_B;
  const int T = p.fa.T, N = p.fa.N;
  const int nblocks = (T + 15) / 16;

  // staging unit h of this helper: u = (w - 2) + NH h -> (chain u / NW, virtual wave u % NW)
  auto unit = [&](int h, int& chain, int& vw) __attribute__((always_inline)) {
    const int u = (w - 2) + NH * h;
    chain = u >= NW ? 1 : 0;
    vw = (w >= 2 && u < 2 * NW) ? u - chain * NW : NW;
  };
  float er0[HV][5], er1[HV][5], er2[HV][5];
  if (w >= 2) {
#pragma unroll
    for (int h = 0; h < HV; ++h) {
      int ch, vw;
      unit(h, ch, vw);
      if (vw < NW) {
        float er[5];
        if (ch) {
          rec_load<NP, kFbBeta>(p.fb, b, 0, vw, l, er);
          rec_stage<NP, kFbBeta>(p.fb, lb, 0, vw, l, er);
          if (nblocks > 1) rec_load<NP, kFbBeta>(p.fb, b, 1, vw, l, er1[h]);
          if (nblocks > 2) rec_load<NP, kFbBeta>(p.fb, b, 2, vw, l, er2[h]);
        } else {
          rec_load<NP, kFbAlpha>(p.fa, b, 0, vw, l, er);
          rec_stage<NP, kFbAlpha>(p.fa, la, 0, vw, l, er);
          if (nblocks > 1) rec_load<NP, kFbAlpha>(p.fa, b, 1, vw, l, er1[h]);
          if (nblocks > 2) rec_load<NP, kFbAlpha>(p.fa, b, 2, vw, l, er2[h]);
        }
      }
    }
  }
  lds_barrier();

  if (w == 0) { band_chain_dispatch<NP, kFbAlpha>(p.fa, la, b, ca); return; }
  if (w == 1) { band_chain_dispatch<NP, kFbBeta>(p.fb, lb, b, cb); return; }

  // ------------------------------------------------------------------------ helpers
  const int hi = w - 2;  // row tasks: helper hi owns the times t with t % NH == hi (both chains)
  const bool tasks = !(kAbl & (1 << 26));  // (diagnostic bit 1 << 26: no row tasks, timing only)
  const size_t sb = (size_t)b * T;
  const unsigned slab_np = (unsigned)((size_t)T * NP * 4), slab_n = (unsigned)((size_t)T * N * 4);
  const __amdgpu_buffer_rsrc_t rU = buf_rsrc(p.fa.rows + sb * NP, slab_np);
  const __amdgpu_buffer_rsrc_t rV = buf_rsrc(p.fb.rows + sb * NP, slab_np);
  const unsigned m = p.mask;
  const __amdgpu_buffer_rsrc_t rP = buf_rsrc((m & HMM355_FB_POSTERIOR) ? p.posterior + sb * N : p.fa.rows, (m & HMM355_FB_POSTERIOR) ? slab_n : 0u);
  const __amdgpu_buffer_rsrc_t rF = buf_rsrc((m & HMM355_FB_FORWARD) ? p.forward + sb * N : p.fa.rows, (m & HMM355_FB_FORWARD) ? slab_n : 0u);
  const __amdgpu_buffer_rsrc_t rB = buf_rsrc((m & HMM355_FB_BACKWARD) ? p.backward + sb * N : p.fa.rows, (m & HMM355_FB_BACKWARD) ? slab_n : 0u);
  const bool full = N == NP;
  double baseA = 0.0, baseB = 0.0;
  // first row of block k (in the chain's step order) this helper owns: alpha step rho is
  // time rho, beta step rho is time T-1-rho
  auto j0A = [&](int k) __attribute__((always_inline)) { return (((hi - 16 * k) % NH) + NH) % NH; };
  auto j0B = [&](int k) __attribute__((always_inline)) { return ((((T - 1 - hi) - 16 * k) % NH) + NH) % NH; };
  auto fi = [&](int rho) __attribute__((always_inline)) { const int k = (rho >> 4) + 2; return k < nblocks ? k : nblocks; };  // flush interval of a step

  // Rabiner log-scales of the 16 rows of block k of chain X (rec_flush's scan): lane j < 16
  auto scan = [&](int X, int k) __attribute__((always_inline)) -> float {
    const float* lx = X ? lb : la;
    const int j = l & 15, rho = 16 * k + j;
    const float c = lx[C::OFF_SC + 64 * ((rho - 1) & (C::RING - 1))];
    float x = (l < 16 && rho >= 1 && rho < T) ? __logf(c) : 0.f;
    if (p.fa.obs_mode == HMM355_OBS_LOG) {
      const int src = X ? rho - 1 : rho;
      const float mm = lx[C::OFF_M + (src & (C::MRING - 1))];
      x += (l < 16 && src >= 0 && rho < T) ? mm : 0.f;
    }
    x += dpp_f<0x111>(x);
    x += dpp_f<0x112>(x);
    x += dpp_f<0x114>(x);
    x += dpp_f<0x118>(x);
    return x;
  };
  // scratch reads of the other chain's rows for the rows of block k this helper will
  // flush SECOND (other rows: an out-of-range offset, no traffic)
  // Scratch reads of the other chain's rows for the rows of block k this helper will flush
  // SECOND, at least two intervals after the other chain (closer pairs are both still in the
  // LDS rings).  Issued two intervals ahead, right after this interval's row stores (the rows
  // they read were stored in this interval at the latest, by this wave): so the wait that
  // uses them only waits for stores two intervals old.  Other rows: out-of-range, no traffic.
  auto prefetch = [&](int k, float (&pa)[RQ][K], float (&pb)[RQ][K]) __attribute__((always_inline)) {
    const int ja = j0A(k), jb = j0B(k);
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int ra = 16 * k + ja + NH * q;  // alpha step = time
      const bool sa = ja + NH * q < 16 && ra < T && fi(ra) - fi(T - 1 - ra) >= 2;
      buf_load<K>(rV, sa ? (ra * NP + K * l) * 4 : kBufOOB, pa[q]);
      const int rb = 16 * k + jb + NH * q;  // beta step; time T-1-rb
      const int tb = T - 1 - rb;
      const bool sbb = jb + NH * q < 16 && rb < T && fi(rb) - fi(tb) >= 2;
      buf_load<K>(rU, sbb ? (tb * NP + K * l) * 4 : kBufOOB, pb[q]);
    }
  };
  // The RQ rows of block k of chain X this helper owns, as one straight-line batch (their
  // LDS reads, transcendentals and wave sums overlap): own output exp(log x + LS); the row
  // to scratch when X reaches the time two or more intervals FIRST; the posterior when X
  // reaches it SECOND (the other row from `pf`, or from the other LDS ring when the intervals
  // are adjacent) or in the same interval as the other chain (alpha writes it).  Rows / lanes that must not write get an
  // out-of-range offset.  Posterior = x*y / sum(x*y): u <= N and v <= 1 (row-stochastic A,
  // scaled rows), and with e >= 1e-8 (OBS_PROB) or max e = 1 (OBS_LOG) some product stays far
  // from underflow, so no max-normalisation pass is needed.
  auto chain_tasks = [&](auto XC, int k, float xs, double base, const float (&pf)[RQ][K], auto EPI) __attribute__((always_inline)) {
    constexpr int X = decltype(XC)::value;
    const float* lx = X ? lb : la;
    const float* ly = X ? la : lb;
    const int j0 = X ? j0B(k) : j0A(k);
    const __amdgpu_buffer_rsrc_t rO = X ? rB : rF;
    const __amdgpu_buffer_rsrc_t rS = X ? rV : rU;
    float x[RQ][K], y[RQ][K], o[RQ][K], pp[RQ][K], ps[RQ];
    int soff[RQ], ooff[RQ], poff[RQ];
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int rho = 16 * k + j0 + NH * q, rhoY = T - 1 - rho;
      const int t = X ? rhoY : rho;
      const bool valid = j0 + NH * q < 16 && rho < T;
      const int fx = fi(rho), fy = fi(rhoY);
      // the other chain's row is still in its LDS ring when the flush intervals are <= 1
      // apart (a row of block k stays readable in intervals k+2 and k+3)
      const bool near = fx - fy <= 1 && fy - fx <= 1;
      soff[q] = (valid && fy - fx >= 2) ? (t * NP + K * l) * 4 : kBufOOB;
      ooff[q] = valid ? (t * N + K * l) * 4 : kBufOOB;
      poff[q] = (valid && (fx > fy || (fx == fy && X == 0))) ? (t * N + K * l) * 4 : kBufOOB;
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        x[q][kk] = lx[C::OFF_RING + (rho & (C::RING - 1)) * NP + K * l + kk];
        const float yv = ly[C::OFF_RING + (rhoY & (C::RING - 1)) * NP + K * l + kk];
        y[q][kk] = near ? yv : pf[q][kk];
      }
    }
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const float LS = (float)(base + (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xs), (j0 + NH * q) & 15)));
      float sq = 0.f;
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        pp[q][kk] = x[q][kk] * y[q][kk];
        sq += pp[q][kk];
      }
      // exp(log x + LS) (the two-kernel path's bits); a row whose log-scale is below -110 is
      // exactly 0 (x <= N = 128 < e^5, and e^-105 is below the smallest fp32 denormal), as
      // the reference's exp(log alpha) underflows: a uniform branch skips the transcendentals
      if (LS >= -110.f) {
#pragma unroll
        for (int kk = 0; kk < K; ++kk) o[q][kk] = __expf(__logf(x[q][kk]) + LS);
      } else {
#pragma unroll
        for (int kk = 0; kk < K; ++kk) o[q][kk] = 0.f;
      }
      ps[q] = row16_sum(sq);
    }
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      if (kAbl & (1 << 29)) continue;  // (diag: no output / scratch stores)
      buf_store<K, 0>(rS, soff[q], x[q]);
      if (full) {
        buf_store<K, kBufNT>(rO, ooff[q], o[q]);
      } else {
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          const float ok[1] = {o[q][kk]};
          buf_store<1, kBufNT>(rO, K * l + kk < N ? ooff[q] + 4 * kk : kBufOOB, ok);
        }
      }
    }
    // the four row sums: row_bcast stages interleaved, then lane 63
#pragma unroll
    for (int q = 0; q < RQ; ++q) asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(ps[q]));
#pragma unroll
    for (int q = 0; q < RQ; ++q) asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(ps[q]));
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const float sw = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ps[q]), 63));
      const float is = sw > 0.f ? __builtin_amdgcn_rcpf(sw) : 0.f;
#pragma unroll
      for (int kk = 0; kk < K; ++kk) pp[q][kk] *= (kAbl & (1 << 25)) ? 1.f : is;
      if (kAbl & ((1 << 28) | (1 << 29))) continue;  // (diag: no posterior stores)
      if (full) {
        buf_store<K, kBufNT>(rP, poff[q], pp[q]);
      } else {
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          const float pk[1] = {pp[q][kk]};
          buf_store<1, kBufNT>(rP, K * l + kk < N ? poff[q] + 4 * kk : kBufOOB, pk);
        }
      }
    }
    if constexpr (decltype(EPI)::value && X == 0) {
#pragma unroll
      for (int q = 0; q < RQ; ++q) {
        if (j0 + NH * q < 16 && 16 * k + j0 + NH * q == T - 1) {
          const float LS = (float)(base + (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xs), (j0 + NH * q) & 15)));
          // loglik = LS_{T-1} + log c_{T-1} (the chain left c_{T-1} = sum u_{T-1} in its ring)
          if (p.fa.loglik && l == 0) p.fa.loglik[b] = LS + __logf(la[C::OFF_SC + 64 * ((T - 1) & (C::RING - 1))]);
          if (p.lik_ref) {  // hmm.py:206: logsumexp_j log(forward_{T-1}[j] + 1e-8)
            float lv[K], mm = -INFINITY;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) {
              lv[kk] = K * l + kk < N ? __logf(o[q][kk] + 1e-8f) : -INFINITY;
              mm = fmaxf(mm, lv[kk]);
            }
            mm = wave_max(mm);
            float e = 0.f;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) e += K * l + kk < N ? __expf(lv[kk] - mm) : 0.f;
            e = wave_sum(e);
            if (l == 0) p.lik_ref[b] = mm + __logf(e);
          }
        }
      }
    }
  };
  auto block_tasks = [&](int k, const float (&pa)[RQ][K], const float (&pb)[RQ][K], auto EPI) __attribute__((always_inline)) {
    const float xa = scan(0, k), xb = scan(1, k);
    const double ba = baseA, bb = baseB;
    baseA += (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xa), 15));
    baseB += (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xb), 15));
    chain_tasks(std::integral_constant<int, 0>{}, k, xa, ba, pa, EPI);
    chain_tasks(std::integral_constant<int, 1>{}, k, xb, bb, pb, EPI);
  };

  // scratch rows read two intervals ahead: parity kb & 1 (the loop is unrolled 6 ways so
  // both the emission register sets and these are compile-time)
  float pfa0[RQ][K], pfb0[RQ][K], pfa1[RQ][K], pfb1[RQ][K];
#pragma unroll
  for (int q = 0; q < RQ; ++q)
#pragma unroll
    for (int k = 0; k < K; ++k) pfa0[q][k] = pfb0[q][k] = pfa1[q][k] = pfb1[q][k] = 0.f;
  // Straight-line block work (the tail stages a padding block and re-loads the last one), as
  // in rec_band: row tasks of block kb-2, the reads for block kb, then the staging.
  auto block_work = [&](int kb, float (&ernext)[HV][5], float (&erfree)[HV][5], float (&pa)[RQ][K], float (&pb)[RQ][K],
                        auto FULLC) __attribute__((always_inline)) {
    if (tasks && kb >= 2) block_tasks(kb - 2, pa, pb, std::false_type{});
    if (tasks) prefetch(kb, pa, pb);
    const int kload = kb + 3 < nblocks ? kb + 3 : nblocks - 1;
#pragma unroll
    for (int h = 0; h < HV; ++h) {
      int ch, vw;
      unit(h, ch, vw);
      if (vw < NW) {
        if (ch) {
          rec_stage<NP, kFbBeta>(p.fb, lb, kb + 1, vw, l, ernext[h]);
          rec_load<NP, kFbBeta, decltype(FULLC)::value>(p.fb, b, kload, vw, l, erfree[h]);
        } else {
          rec_stage<NP, kFbAlpha>(p.fa, la, kb + 1, vw, l, ernext[h]);
          rec_load<NP, kFbAlpha, decltype(FULLC)::value>(p.fa, b, kload, vw, l, erfree[h]);
        }
      }
    }
    lds_barrier();
  };
  // (every lambda is always_inline: block_work has six call sites, and an out-of-line copy
  // takes the register arrays by reference, through scratch)
  auto helper_loop = [&](auto FULLC) __attribute__((always_inline)) {
    for (int kb = 0; kb < nblocks; kb += 6) {
      block_work(kb, er1, er0, pfa0, pfb0, FULLC);
      if (kb + 1 < nblocks) block_work(kb + 1, er2, er1, pfa1, pfb1, FULLC);
      if (kb + 2 < nblocks) block_work(kb + 2, er0, er2, pfa0, pfb0, FULLC);
      if (kb + 3 < nblocks) block_work(kb + 3, er1, er0, pfa1, pfb1, FULLC);
      if (kb + 4 < nblocks) block_work(kb + 4, er2, er1, pfa0, pfb0, FULLC);
      if (kb + 5 < nblocks) block_work(kb + 5, er0, er2, pfa1, pfb1, FULLC);
    }
  };
  if (N == NP && (reinterpret_cast<uintptr_t>(p.fa.obs) & 15) == 0) helper_loop(std::true_type{});
  else helper_loop(std::false_type{});
  lds_barrier();  // the chains' last rows and c_{T-1}
  if (!tasks) return;
  // the last two blocks of each chain (their rows are flushed here, after both chains ended;
  // their scratch reads were issued in intervals nblocks-2 and nblocks-1)
  const bool odd = (nblocks & 1) != 0;  // block nblocks-1 used parity (nblocks-1) & 1
  float qa[RQ][K], qb[RQ][K];
  if (nblocks >= 2) {
#pragma unroll
    for (int q = 0; q < RQ; ++q)
#pragma unroll
      for (int k = 0; k < K; ++k) {
        qa[q][k] = odd ? pfa1[q][k] : pfa0[q][k];
        qb[q][k] = odd ? pfb1[q][k] : pfb0[q][k];
      }
    block_tasks(nblocks - 2, qa, qb, std::true_type{});
  }
#pragma unroll
  for (int q = 0; q < RQ; ++q)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      qa[q][k] = odd ? pfa0[q][k] : pfa1[q][k];
      qb[q][k] = odd ? pfb0[q][k] : pfb1[q][k];
    }
  block_tasks(nblocks - 1, qa, qb, std::true_type{});
}

}  // namespace hmm355
