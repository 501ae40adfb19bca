// hmm355 — epilogues shared by the time-invariant (fb.hip, viterbi.hip) and time-varying
// (tv.hip) recursions: the forward-backward posterior pass and the Viterbi chunk maps +
// backtrace.  Both consume the row layouts the recursions leave in the workspace.
#pragma once
#include <type_traits>
#include "common.h"
#include "band.h"

namespace hmm355 {

struct PostArgs {
  const float* U;
  const float* V;
  const float* LA;
  const float* LB;
  float* posterior;
  float* forward;
  float* backward;
  float* lik_ref;
  int B, T, N;
  unsigned mask;
};

constexpr int kPostWaves = 32768;  // waves of the posterior pass (grid-stride; 8192 measured 2.4 us slower than 16384)

template <int NP>
__global__ void __launch_bounds__(256) fb_posterior_kernel(PostArgs a) {
  // One wave per row, grid-stride, the next row's loads issued before this row's math (one
  // row in flight behind the stores).  When N == NP every lane owns K consecutive states:
  // one 8/16-byte load per array and one 8/16-byte store per output row.
  constexpr int K = NP / 64;
  using VecK = typename std::conditional<K == 1, float, typename std::conditional<K == 2, float2, float4>::type>::type;
  const int l = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const size_t rows = (size_t)a.B * a.T;
  const bool vec = a.N == NP && (reinterpret_cast<uintptr_t>(a.posterior) | reinterpret_cast<uintptr_t>(a.forward) |
                                 reinterpret_cast<uintptr_t>(a.backward)) % sizeof(VecK) == 0;
  // element k of this lane: state j(k) (contiguous when vec, else strided by 64)
  auto jof = [&](int k) { return vec ? K * l + k : l + 64 * k; };
  auto load = [&](size_t row, float (&u)[K], float (&v)[K], float& la, float& lb) {
    if (vec) {
      const VecK tu = reinterpret_cast<const VecK*>(a.U + row * NP)[l];
      const VecK tv = reinterpret_cast<const VecK*>(a.V + row * NP)[l];
      __builtin_memcpy(u, &tu, sizeof(tu));
      __builtin_memcpy(v, &tv, sizeof(tv));
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        u[k] = a.U[row * NP + l + 64 * k];
        v[k] = a.V[row * NP + l + 64 * k];
      }
    }
    la = a.LA[row];
    lb = a.LB[row];
  };
  float u[K], v[K], la = 0.f, lb = 0.f;
  size_t row = wave;
  if (row < rows) load(row, u, v, la, lb);
  for (; row < rows; row += nwaves) {
    float un[K], vn[K], lan = 0.f, lbn = 0.f;
    if (row + nwaves < rows) load(row + nwaves, un, vn, lan, lbn);
    float mu = 0.f, mv = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { mu = fmaxf(mu, u[k]); mv = fmaxf(mv, v[k]); }
    mu = wave_max_dpp2(mu);
    mv = wave_max_dpp2(mv);
    const float iu = mu > 0.f ? 1.f / mu : 0.f, iv = mv > 0.f ? 1.f / mv : 0.f;
    float p[K], s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { p[k] = (u[k] * iu) * (v[k] * iv); s += p[k]; }
    s = wave_sum_dpp(s);
    const float is = s > 0.f ? 1.f / s : 0.f;
    const bool last = (row % a.T) == (size_t)(a.T - 1);
    // forward / backward only where they are stored (fb.hip's chains write them at flush
    // time) or the reference's likelihood needs the last forward row: the transcendentals
    // are most of this pass's issue otherwise
    float fw[K], bw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      p[k] *= is;
      fw[k] = 0.f;
      bw[k] = 0.f;
    }
    if ((a.mask & HMM355_FB_FORWARD) || (last && a.lik_ref)) {
#pragma unroll
      for (int k = 0; k < K; ++k) fw[k] = __expf(__logf(u[k]) + la);
    }
    if (a.mask & HMM355_FB_BACKWARD) {
#pragma unroll
      for (int k = 0; k < K; ++k) bw[k] = __expf(__logf(v[k]) + lb);
    }
    if (vec) {
      VecK t;
      const size_t off = row * NP;
      // outputs are not re-read here: non-temporal stores (kAbl bit 1 << 18 for plain ones)
      auto put = [&](float* dst, const float (&x)[K]) {
        __builtin_memcpy(&t, x, sizeof(t));
        VecK* pd = reinterpret_cast<VecK*>(dst + off) + l;
        if constexpr (kAbl & (1 << 18)) {
          *pd = t;
        } else {
          typedef float nvec __attribute__((ext_vector_type(K)));
          nvec tv;
          __builtin_memcpy(&tv, &t, sizeof(t));
          __builtin_nontemporal_store(tv, reinterpret_cast<nvec*>(pd));
        }
      };
      if (a.mask & HMM355_FB_POSTERIOR) put(a.posterior, p);
      if (a.mask & HMM355_FB_FORWARD) put(a.forward, fw);
      if (a.mask & HMM355_FB_BACKWARD) put(a.backward, bw);
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int j = l + 64 * k;
        if (j < a.N) {
          const size_t off = row * a.N + j;
          if (a.mask & HMM355_FB_POSTERIOR) a.posterior[off] = p[k];
          if (a.mask & HMM355_FB_FORWARD) a.forward[off] = fw[k];
          if (a.mask & HMM355_FB_BACKWARD) a.backward[off] = bw[k];
        }
      }
    }
    if (last && a.lik_ref) {
      // hmm.py:206: logsumexp(log(forward[:, -1] + 1e-8))
      float lv[K], m = -INFINITY;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        lv[k] = (jof(k) < a.N) ? __logf(fw[k] + 1e-8f) : -INFINITY;
        m = fmaxf(m, lv[k]);
      }
      m = wave_max(m);
      float e = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) e += (jof(k) < a.N) ? __expf(lv[k] - m) : 0.f;
      e = wave_sum(e);
      if (l == 0) a.lik_ref[row / a.T] = m + __logf(e);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) { u[k] = un[k]; v[k] = vn[k]; }
    la = lan;
    lb = lbn;
  }
}

constexpr int kChunk = 64;  // psi / backtrace chunk length (time steps)

template <int NP>
struct VF {
  static constexpr int NW = NP / 16;
  static constexpr int NT = NW * kWave;
  static constexpr int NBLK = NP / 64;
  static constexpr int RING = 32;
  static constexpr int OFF_EMIS = 0;                       // [2][16][NP]
  static constexpr int OFF_RING = OFF_EMIS + 2 * 16 * NP;  // [RING][NP]
  static constexpr int LDS_FLOATS = OFF_RING + RING * NP;
};

struct VitArgs {
  const float* obs;
  const float* log_P;
  const float* init;
  float* delta;          // (B,T,N) output trellis
  float* final_score;    // (B) or null
  int64_t* states;       // (B,T)
  uint8_t* psi;          // (B,T,NP) workspace
  uint8_t* G;            // (B,nchunks,NP) workspace
  int B, T, N, obs_mode, nchunks;
  const BandDesc* band;  // banded decomposition (band.h) or null
  // psi followers (HMM355_VIT_PLAN_DENSE): workgroups beside the chain, their progress and
  // finished-chunk words (RecArgs::prog / done), zeroed before each launch
  int nfollow;
  int* prog;
  uint8_t* done;
  // the decode beside a banded chain (HMM355_VIT_PLAN_BANDED, follow.h): published psi blocks
  // (B), and with OBS_PROB the log leaders' rows and counts (RecArgs::lobuf / lready)
  int* pub;
  const float* lobuf;
  const int* lready;
  uint8_t* path;  // (B, nchunks, NP, 64) the decode follower's chunk paths (follow.h)
  unsigned token;  // the counts' call token (common.h)
};

// chunk map: G[j] = state at t_lo - 1 given state j at t_hi (psi rows of the chunk in LDS)
template <int NP>
__device__ __forceinline__ void compose_chunk_map(const VitArgs& a, const uint8_t (*prow)[NP], int b, int chunk,
                                                  int t_lo, int t_hi) {
  const int tid = threadIdx.x;
  if (chunk > 0 && tid < NP) {
    int s = tid < a.N ? tid : 0;
    for (int t = t_hi; t > t_lo; --t) s = prow[t - t_lo][s];
    a.G[((size_t)b * a.nchunks + chunk) * NP + tid] = prow[0][s];
  }
}

// ----------------------------------------------------------------------- backtrace
template <int NP>
__global__ void __launch_bounds__(64) vit_backtrace_kernel(VitArgs a) {
  constexpr int K = NP / 64;
  constexpr int GB = 64;  // chunk maps staged per LDS batch
  __shared__ __attribute__((aligned(16))) uint8_t gs[GB][NP];
  __shared__ __attribute__((aligned(16))) uint8_t ps[kChunk][NP];
  __shared__ int st[kChunk];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int l = threadIdx.x;
  const int T = a.T, N = a.N, nc = a.nchunks;

  // s_{T-1} = argmax delta_{T-1} (first index; hmm.py:174)
  const float* dl = a.delta + ((size_t)b * T + T - 1) * N;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int j = l + 64 * k;
    const bool ok = j < N;
    const float v = dl[ok ? j : 0];
    if (ok) argmax_combine(bv, bi, v, j);
  }
  wave_argmax(bv, bi);
  if (chunk == 0 && l == 0 && a.final_score) a.final_score[b] = bv;
  int s = bi;

  // walk the chunk maps from the last chunk down to chunk+1
  for (int hi = nc - 1; hi > chunk; hi -= GB) {
    const int lo = hi - GB + 1 > chunk + 1 ? hi - GB + 1 : chunk + 1;
    const int cnt = hi - lo + 1;
    const uint8_t* gsrc = a.G + ((size_t)b * nc + lo) * NP;
    for (int idx = l; idx < cnt * NP / 16; idx += 64)
      *reinterpret_cast<uint4*>(&gs[0][0] + idx * 16) = *reinterpret_cast<const uint4*>(gsrc + idx * 16);
    __syncthreads();
    for (int cc = hi; cc >= lo; --cc) s = gs[cc - lo][s];
    __syncthreads();
  }
  // this chunk's psi rows, then the walk
  const int t_lo = chunk * kChunk;
  const int t_hi = (t_lo + kChunk < T ? t_lo + kChunk : T) - 1;
  const int rows = t_hi - t_lo + 1;
  const uint8_t* psrc = a.psi + ((size_t)b * T + t_lo) * NP;
  for (int idx = l; idx < rows * NP / 16; idx += 64)
    *reinterpret_cast<uint4*>(&ps[0][0] + idx * 16) = *reinterpret_cast<const uint4*>(psrc + idx * 16);
  __syncthreads();
  if (l == 0) {
    st[t_hi - t_lo] = s;
    for (int t = t_hi; t > t_lo; --t) {
      s = ps[t - t_lo][s];
      st[t - 1 - t_lo] = s;
    }
  }
  __syncthreads();
  for (int i = l; i < rows; i += 64) a.states[(size_t)b * T + t_lo + i] = st[i];
}

// terminal backward vector from its logarithm: binit = exp(l - max l) (padded states 0),
// bscale = max l.  One wave per sequence.
template <int NP>
__global__ void __launch_bounds__(64) beta_init_kernel(const float* __restrict__ lbt, int N, float* binit, float* bscale) {
  const int b = blockIdx.x, l = threadIdx.x;
  constexpr int K = NP / 64;
  float v[K], m = -INFINITY;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int j = l + 64 * k;
    v[k] = j < N ? lbt[(size_t)b * N + j] : -INFINITY;
    m = fmaxf(m, v[k]);
  }
  m = wave_max(m);
  if (m == -INFINITY) m = 0.f;  // an all-zero terminal vector: every adjoint is 0
#pragma unroll
  for (int k = 0; k < K; ++k) binit[(size_t)b * NP + l + 64 * k] = (l + 64 * k < N) ? __expf(v[k] - m) : 0.f;
  if (l == 0) bscale[b] = m;
}

}  // namespace hmm355
