// hmm355 — work beside the banded chains, inside the chains' own launch (gfx950).
//
// At B = 32 the north-star chains own 32 (Viterbi) and 64 (forward-backward) of the 256 CUs,
// and until round 5 every full-chip pass ran in series with them: the Viterbi emission log
// before the chain (15.8 us), the psi chunk maps (14.1 us) and the backtrace (8.1 us) after it,
// the posterior pass (19.5 us) after the FB chains, plus a launch gap each.  Here they run as
// extra workgroups of the chain launch, one per sequence, on the CUs the chains leave idle:
//
//   vit_lead           (Viterbi, OBS_PROB) log(x + 1e-8) of the sequence's 16-step blocks 4..,
//                      in time order into RecArgs::lobuf, publishing the count lready[b]; the
//                      chain's staging helpers load a block from there once it is counted
//                      (recur.h rec_band, checked two blocks ahead) and take the log of the raw
//                      block themselves otherwise, so the chain never waits for the leader.
//   vit_decode_follow  (Viterbi) composes the 64-step chunk maps G_c[j] = state at the chunk's
//                      first step - 1 given state j at its last (post.h compose_chunk_map's
//                      map) from the psi rows the chain's helpers publish, storing each chunk's
//                      path for every end state on the way; once the chain is complete, the
//                      backtrace (hmm.py:174-178) is the first argmax of the last trellis row,
//                      the walk over the maps, and a gather of every chunk's path at its end
//                      state, all in this workgroup.
//   fb_post_follow     (forward-backward) the posterior (hmm.py:119-126) of every row t as soon
//                      as both chains have published it: rows from the middle outwards, two per
//                      chain step in the second half.
//
// Hand-off (common.h; MI355X_MICROARCH.md inter-workgroup visibility, the table's first row):
// the chains' helpers store rows and psi bytes write-through (sc1), retire them before a
// workgroup barrier, and one lane stores the block count (relaxed, agent scope); a follower
// polls the count with one lane (relaxed sc1 loads, s_sleep between polls), joins a workgroup
// barrier, and reads the rows with sc1 loads only.
//
// Progress: a follower waits only for chains of its own launch with lower workgroup indices
// (dispatched first, never waiting for a follower), and the chains never wait for a leader, so
// every wait ends.  A follower that sees no progress for kFollowGiveUp (0.2 s, far beyond any
// chain step) marks its outputs invalid (NaN posteriors / states -1) instead of hanging.
#pragma once
#include "recur.h"
#include "post.h"

namespace hmm355 {

constexpr long long kFollowGiveUp = 20000000;  // 0.2 s of the 100 MHz real-time counter

// (diagnostic builds: real-time stamp k of this workgroup, tools/band_stamps.py)
__device__ __forceinline__ void fstamp(int k) {
  if (kStamp && threadIdx.x == 0)
    g_rec_stamps[((size_t)blockIdx.x * 16 % kStampWaves) * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

// One lane polls *p until it reaches `need` or the count stops moving for kFollowGiveUp;
// the value seen goes to *slot (LDS), -1 on give-up.  The caller's workgroup barrier follows.
__device__ __forceinline__ void follow_poll(const int* p, int need, int* slot, unsigned token, int cap) {
  int have = poll_count(p, token, cap), last = have;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  while (have < need) {
    __builtin_amdgcn_s_sleep(20);
    have = poll_count(p, token, cap);
    const long long now = __builtin_amdgcn_s_memrealtime();
    if (have != last) {
      last = have;
      t0 = now;
    } else if (now - t0 > kFollowGiveUp) {
      have = -1;
      break;
    }
  }
  *slot = have;
}

// ------------------------------------------------------------------------ log leaders
// Blocks [4, nblocks) of sequence b, 8 blocks per round: load (plain: the raw emissions are
// not written in this launch), log(x + 1e-8) correctly rounded (logcr.h, the chain staging's
// arithmetic bit for bit), write-through stores, retire, barrier, publish.
template <int NP>
__device__ __forceinline__ void vit_lead(const RecArgs& a, int b) {
  const int T = a.T, N = a.N, nblocks = (T + 15) / 16;
  if (!a.lobuf || nblocks <= 4 || (kFAbl & (2 | 8))) return;
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t off = (size_t)b * T * N;
  const float* src = a.obs + off;
  float* dst = const_cast<float*>(a.lobuf) + off;
  int* cnt = const_cast<int*>(a.lready) + b * kPubStride;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(dst, (size_t)T * N * 4);
  const bool vec = (N & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  constexpr int kRound = 8;  // blocks per round
  for (int k0 = 4; k0 < nblocks; k0 += kRound) {
    const int k1 = k0 + kRound < nblocks ? k0 + kRound : nblocks;
    const int e0 = 16 * k0 * N, e1 = (16 * k1 < T ? 16 * k1 : T) * N;  // element range (< 2^31)
    if (vec) {
      // four 16-B loads in flight per lane, then the logs and the stores
      for (int i0 = e0 / 4 + tid; i0 < e1 / 4; i0 += 4 * nt) {
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = i0 + k * nt;
          v[k] = reinterpret_cast<const float4*>(src)[i < e1 / 4 ? i : i0];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = i0 + k * nt;
          const float4 o = make_float4(logcr_fast(v[k].x + 1e-8f, g_logcr_tab), logcr_fast(v[k].y + 1e-8f, g_logcr_tab),
                                       logcr_fast(v[k].z + 1e-8f, g_logcr_tab), logcr_fast(v[k].w + 1e-8f, g_logcr_tab));
          if (i < e1 / 4) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), rs, i * 16, 0, kAuxSc1);
        }
      }
    } else {
      for (int i = e0 + tid; i < e1; i += nt)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, logcr_fast(src[i] + 1e-8f, g_logcr_tab)), rs,
                                              i * 4, 0, kAuxSc1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) publish_count(cnt, k1, a.token);
  }
}

// ------------------------------------------------------------- Viterbi decode follower
// LDS: chunk maps [nc][NP] | staging of up to G chunks' psi rows [G][64][NP] | chunk end
// states [nc] | control words.  The host admits the follower path only while it fits
// (vit_follow_lds_bytes <= kExclusiveLds).
// chunks composed at once: NP lanes each, 1024 threads, at most 8 (64 KiB of staged rows)
__host__ __device__ constexpr int follow_g(int NP) { return 1024 / NP < 8 ? 1024 / NP : 8; }
inline size_t vit_follow_lds_bytes(int T, int NP) {
  const size_t nc = (T + kChunk - 1) / kChunk;
  return align_up(nc * NP, 16) + (size_t)follow_g(NP) * kChunk * NP + align_up(nc, 4) * 4 + 64;
}

template <int NP>
__device__ __forceinline__ void vit_decode_follow(const RecArgs& a, int b, float* ldsf) {
  const int T = a.T, N = a.N, nblocks = (T + 15) / 16, nc = (T + kChunk - 1) / kChunk;
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, nw = blockDim.x >> 6;
  uint8_t* lds = reinterpret_cast<uint8_t*>(ldsf);
  uint8_t* gm = lds;                                             // [nc][NP]
  uint8_t* stg = gm + align_up((size_t)nc * NP, 16);             // [G][64][NP]
  int* send = reinterpret_cast<int*>(stg + (size_t)follow_g(NP) * kChunk * NP);  // [nc]
  int* ctl = send + align_up((size_t)nc, 4);                     // control words
  int64_t* sb = a.states + (size_t)b * T;
  auto invalid = [&]() {  // the chain never published (a dense plan passed as banded, or stalled)
    for (int t = tid; t < T; t += blockDim.x) sb[t] = -1;
    if (tid == 0 && a.final_score) a.final_score[b] = __builtin_bit_cast(float, 0x7fc00000u);
  };
  fstamp(0);
  if (kFAbl & 2) return;
  if (rec_band_code<kVit, NP>(a) == 0) {
    invalid();
    return;
  }
  const int* pubp = a.pub + b * kPubStride;
  const __amdgpu_buffer_rsrc_t psi_rs = make_rsrc(a.psi + (size_t)b * T * NP, (size_t)T * NP);
  constexpr int G = follow_g(NP);
  int have = 0;   // psi blocks published (nblocks + 1: everything)
  int next = 0;   // the next chunk to compose (chunk 0 for its paths; its map is unused)
  auto wait_for = [&](int need) -> bool {
    if (tid == 0) follow_poll(pubp, need, ctl, a.token, nblocks + 1);
    __syncthreads();
    const int v = ctl[0];
    __syncthreads();
    if (v < 0) return false;
    have = v;
    return true;
  };
  // compose chunks [next, c_end) in groups of G: group member g (NP lanes) takes chunk next + g.
  // Lane j walks the chunk's psi rows down from state j at its last step: the state it reaches
  // at each step is byte k of the chunk's path for end state j (the state at t_lo + k), stored
  // (64 bytes) to the workspace, and the state before the chunk is the map entry G_c[j].  The
  // backtrace is then one map walk and a gather of each chunk's path at its end state.
  uint8_t* const pbase = a.path + (size_t)b * nc * NP * kChunk;
  auto compose = [&](int c_end) {
    while (next < c_end) {
      const int cnt = c_end - next < G ? c_end - next : G;
      // stage the chunks' psi rows (sc1 16-B loads)
      const int per = kChunk * NP / 16;  // 16-B pieces per chunk
      for (int idx = tid; idx < cnt * per; idx += blockDim.x) {
        const int g = idx / per, pc = idx - g * per;
        const int t = (next + g) * kChunk + pc / (NP / 16);
        const u32x4_t v = t < T ? __builtin_amdgcn_raw_buffer_load_b128(psi_rs, (t * NP) + 16 * (pc % (NP / 16)), 0, kAuxSc1)
                                : u32x4_t{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4_t*>(stg + (size_t)g * kChunk * NP + 16 * pc) = v;
      }
      __syncthreads();
      const int g = tid / NP, j = tid % NP;
      if (g < cnt) {
        const int c = next + g;
        const int t_lo = c * kChunk, t_hi = (t_lo + kChunk < T ? t_lo + kChunk : T) - 1;
        const int len = t_hi - t_lo;  // the chunk's last step, relative (< 63: the short last chunk)
        const uint8_t* pr = stg + (size_t)g * kChunk * NP;
        int st = j < N ? j : 0;
        unsigned acc[kChunk / 4];
        static_for<0, kChunk>([&](auto KK) {
          constexpr int k = kChunk - 1 - decltype(KK)::value;
          // st = the state at t_lo + min(k, len); beyond len: the end state (never read)
          if constexpr ((k & 3) == 3) acc[k >> 2] = (unsigned)st << 24;
          else acc[k >> 2] |= (unsigned)st << (8 * (k & 3));
          if constexpr (k >= 1) {
            const int nx = pr[k * NP + st];  // (unconditional read, inside the staged chunk)
            st = k <= len ? nx : st;
          }
        });
        gm[(size_t)c * NP + j] = pr[st];
        uint8_t* dst = pbase + ((size_t)c * NP + j) * kChunk;
#pragma unroll
        for (int q = 0; q < kChunk / 16; ++q)
          *reinterpret_cast<u32x4_t*>(dst + 16 * q) = u32x4_t{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
      }
      next += cnt;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the paths stored before the barrier)
      __syncthreads();
    }
  };
  // while the chain runs: every chunk whose four psi blocks are published
  while (next < nc) {
    const int need = 4 * (next + 1) < nblocks ? 4 * (next + 1) : nblocks;
    if (have < need && !wait_for(need)) {
      invalid();
      return;
    }
    int c_end = have > nblocks ? nc : have / 4;  // chunks with all rows published
    if (c_end > nc) c_end = nc;
    if (c_end <= next) c_end = next + 1;  // (the last, short chunk once have == nblocks)
    compose(c_end);
  }
  // the whole trellis and every psi row stored
  if (have <= nblocks && !wait_for(nblocks + 1)) {
    invalid();
    return;
  }
  fstamp(1);
  // s_{T-1} = first argmax of delta_{T-1} (hmm.py:174); the maps from the last chunk down
  if (w == 0) {
    const float* dl = a.rows + ((size_t)b * T + T - 1) * a.row_stride;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < NP / 64; ++k) {
      const int j = l + 64 * k;
      const float v = __hip_atomic_load(dl + (j < N ? j : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (j < N) argmax_combine(bv, bi, v, j);
    }
    wave_argmax_dpp(bv, bi);
    if (l == 0 && a.final_score) a.final_score[b] = bv;
    int s = bi < N ? bi : 0;
    if (l == 0) send[nc - 1] = s;
    for (int c = nc - 1; c >= 1; --c) {
      s = gm[(size_t)c * NP + s];
      if (l == 0) send[c - 1] = s;
    }
  }
  __syncthreads();
  fstamp(2);
  // every state: chunk c's path at its end state send[c], one dword (4 steps) per thread
  const __amdgpu_buffer_rsrc_t path_rs = make_rsrc(pbase, (size_t)nc * NP * kChunk);
  for (int idx = tid; idx < nc * (kChunk / 4); idx += blockDim.x) {
    const int c = idx / (kChunk / 4), q = idx % (kChunk / 4);
    const int t0 = c * kChunk + 4 * q;
    if (t0 < T) {
      const unsigned word = __builtin_amdgcn_raw_buffer_load_b32(path_rs, (c * NP + send[c]) * kChunk + 4 * q, 0, kAuxSc1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (t0 + i < T) sb[t0 + i] = (int64_t)((word >> (8 * i)) & 0xffu);
    }
  }
  if (kStamp) {
    __syncthreads();
    fstamp(3);
  }
}

// ---------------------------------------------------------- forward-backward posterior
// Row t's posterior needs alpha row t (published by the alpha chain after step t) and beta row
// t (by the beta chain after step T-1-t): the ready rows are [T - rows_beta, rows_alpha).  The
// done rows are always one interval [plo, phi); each round takes the new rows at both ends,
// R rows per wave, with fb_posterior_kernel's arithmetic (post.h) bit for bit.
template <int NP>
__device__ __forceinline__ void fb_post_follow(const RecArgs& fa, const RecArgs& fb, float* posterior, int b, float* ldsf) {
  // (b: the follower's index among the F * B followers, split below)
  const int T = fa.T, N = fa.N, nblocks = (T + 15) / 16;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, nw = blockDim.x >> 6;
  int* ctl = reinterpret_cast<int*>(ldsf);
  constexpr int K = NP / 64;
  // F followers per sequence (the launch's grid: 2B chains + F*B followers); follower f forms
  // the rows t with t % F == f (a follower's CU moves ~50 GB/s of write-through rows: DESIGN §5)
  const int F = ((int)gridDim.x - 2 * fa.B) / fa.B, f = b / fa.B;
  b -= f * fa.B;
  auto first_own = [&](int x) { return x + ((f - x % F) % F + F) % F; };
  float* pbase = posterior + (size_t)b * T * N;
  auto invalid = [&]() {
    for (size_t i = tid; i < (size_t)T * N; i += blockDim.x) pbase[i] = __builtin_bit_cast(float, 0x7fc00000u);
    if (tid == 0 && fa.lik_ref) fa.lik_ref[b] = __builtin_bit_cast(float, 0x7fc00000u);
  };
  fstamp(0);
  if (kFAbl & 2) return;
  if (rec_band_code<kFbAlpha, NP>(fa) == 0 || rec_band_code<kFbBeta, NP>(fb) == 0) {
    invalid();  // (the dense chains publish nothing: a plan passed as banded that is not)
    return;
  }
  const int* pa = fa.pub + 2 * b * kPubStride;
  const int* pb_ = pa + kPubStride;
  const __amdgpu_buffer_rsrc_t rU = make_rsrc(fa.rows + (size_t)b * T * NP, (size_t)T * NP * 4);
  const __amdgpu_buffer_rsrc_t rV = make_rsrc(fb.rows + (size_t)b * T * NP, (size_t)T * NP * 4);
  const bool vec = N == NP && (reinterpret_cast<uintptr_t>(posterior) % (4 * K)) == 0;
  auto rows_of = [&](int c) { return c > nblocks ? T : (16 * c < T ? 16 * c : T); };
  // up to R rows per wave per pass, all 2R loads issued before the first row's arithmetic: the
  // second half of the chains hands over two rows per step (a 4-block publish: 128 rows), and
  // a row's write-through source is a far cache's round trip away -- one exposed round trip per
  // pass, not per row
  constexpr int R = HMM355_FBR;
  auto rows = [&](const int (&t)[R], int nv) {
    float u[R][K], v[R][K];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int tr = r < nv ? t[r] : t[0];
      if constexpr (K == 1) {
        u[r][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rU, (tr * NP + l) * 4, 0, kAuxSc1));
        v[r][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rV, (tr * NP + l) * 4, 0, kAuxSc1));
      } else if constexpr (K == 2) {
        const float2 x = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rU, (tr * NP + 2 * l) * 4, 0, kAuxSc1));
        const float2 y = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rV, (tr * NP + 2 * l) * 4, 0, kAuxSc1));
        u[r][0] = x.x; u[r][1] = x.y; v[r][0] = y.x; v[r][1] = y.y;
      } else {
        const float4 x = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rU, (tr * NP + 4 * l) * 4, 0, kAuxSc1));
        const float4 y = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rV, (tr * NP + 4 * l) * 4, 0, kAuxSc1));
        u[r][0] = x.x; u[r][1] = x.y; u[r][2] = x.z; u[r][3] = x.w;
        v[r][0] = y.x; v[r][1] = y.y; v[r][2] = y.z; v[r][3] = y.w;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r >= nv) break;
      const int t_ = t[r];
      // post.h fb_posterior_kernel: max-normalised product, normalised by its sum
      float mu = 0.f, mv = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) { mu = fmaxf(mu, u[r][k]); mv = fmaxf(mv, v[r][k]); }
      mu = wave_max_dpp2(mu);
      mv = wave_max_dpp2(mv);
      const float iu = mu > 0.f ? 1.f / mu : 0.f, iv = mv > 0.f ? 1.f / mv : 0.f;
      float p[K], sum = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) { p[k] = (u[r][k] * iu) * (v[r][k] * iv); sum += p[k]; }
      sum = wave_sum_dpp(sum);
      const float is = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) p[k] *= is;
      if (vec) {
        float* dst = pbase + (size_t)t_ * N + K * l;
        if constexpr (K == 1) dst[0] = p[0];
        else if constexpr (K == 2) *reinterpret_cast<float2*>(dst) = make_float2(p[0], p[1]);
        else *reinterpret_cast<float4*>(dst) = make_float4(p[0], p[1], p[2], p[3]);
      } else {
        // (not vec: lane l holds states K*l .. K*l + K - 1 all the same)
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (K * l + k < N) pbase[(size_t)t_ * N + K * l + k] = p[k];
      }
    }
  };
  int plo = -1, phi = -1;  // done rows [plo, phi); empty while plo < 0
  int ca = 0, cb = 0;
  while (plo != 0 || phi != T) {
    // wait for rows beyond the done interval (one lane polls both chains)
    if (tid == 0) {
      int ok = 1;
      long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const int na = poll_count(pa, fa.token, nblocks + 1), nb = poll_count(pb_, fa.token, nblocks + 1);
        const int lo = T - rows_of(nb), hi = rows_of(na);
        const bool more = lo < hi && (plo < 0 || lo < plo || hi > phi);
        if (more) { ca = na; cb = nb; break; }
        if (na != ca || nb != cb) { ca = na; cb = nb; t0 = __builtin_amdgcn_s_memrealtime(); }
        else if (__builtin_amdgcn_s_memrealtime() - t0 > kFollowGiveUp) { ok = 0; break; }
        __builtin_amdgcn_s_sleep(20);
      }
      ctl[0] = ok; ctl[1] = ca; ctl[2] = cb;
    }
    __syncthreads();
    const int ok = ctl[0];
    ca = ctl[1];
    cb = ctl[2];
    __syncthreads();
    if (!ok) {
      invalid();
      return;
    }
    if (kStamp && ca > nblocks && cb > nblocks) fstamp(1);
    const int lo = T - rows_of(cb), hi = rows_of(ca);
    // new rows: [lo, plo) and [phi, hi) (all of [lo, hi) the first time); this follower's are
    // those with t % F == f
    const int a0 = first_own(lo), a1 = plo < 0 ? hi : plo;
    const int b0 = first_own(plo < 0 ? hi : phi), b1 = hi;
    const int na = a1 > a0 ? (a1 - a0 + F - 1) / F : 0;
    const int nn = na + (b1 > b0 ? (b1 - b0 + F - 1) / F : 0);
    // R consecutive (own) rows per wave
    for (int i0 = w * R; i0 < nn; i0 += nw * R) {
      int t[R];
#pragma unroll
      for (int r = 0; r < R; ++r) t[r] = i0 + r < na ? a0 + F * (i0 + r) : b0 + F * (i0 + r - na);
      rows(t, nn - i0 < R ? nn - i0 : R);
    }
    plo = lo;
    phi = hi;
  }
  if (kStamp) {
    __syncthreads();
    fstamp(2);
  }
}

}  // namespace hmm355
