// hmm355 — Viterbi on gfx950.
//
// Replaces HMMPyTorch.viterbi_decode (reference hmm.py:132-184) and
// MixtureGaussianHMMLayer._viterbi_decode (mixture_gaussian.py:290-338).
//
// Kernel 1, vit_fwd<NP> (one workgroup per sequence): the max-plus recursion
//     delta_t[j] = max_i(delta_{t-1}[i] + logP[i,j]) + log_obs_t[j]            (hmm.py:164-168)
//   computing the max only, on the serial-chain skeleton of recur.h (wave w owns input
//   slice 16w..16w+15, delta_{t-1} broadcast by DPP row_newbcast folded into
//   v_add_f32_dpp, two candidates per v_max3_f32: 1.5 VALU per cell; per-wave partial maxima
//   combined through LDS after the step's one barrier).  The max of a set of fp32 values is
//   order-independent and each delta is one fp32 add, so delta is bit-identical to the
//   reference given identical log-emissions.  The emission log(x + 1e-8) is formed in fp32
//   and the log correctly rounded (logcr.h) while the emissions are staged.
//
// Kernel 2, vit_psi<NP> (one workgroup per (sequence, 64-step chunk), ~1000 workgroups):
//   the argmax pointers psi_t[j] = first argmax_i(delta_{t-1}[i] + logP[i,j]) recomputed
//   from the stored trellis — the same fp32 sums, so the same argmax the reference's
//   torch.max(dim=1) returns (first index on ties, hmm.py:167).  Taking the argmax out of
//   the serial loop (4 VALU per cell there) and onto the whole chip is what lets the serial
//   kernel run at the max-only cost.  While the chunk's psi rows are in LDS the kernel also
//   composes them into the chunk map G_c[j] = state at the end of chunk c-1 given state j
//   at the end of chunk c (pointer jumping: 64 dependent LDS lookups per lane).
//   On a banded matrix with NP >= 128 (recur.h kVitFused) the chain kernel's psi waves have
//   already written the psi rows, and this kernel only composes the chunk maps.
//
// Kernel 3, vit_backtrace<NP> (one wave per (sequence, chunk)): argmax of delta_{T-1}
//   (first index, hmm.py:174), the chain of chunk maps from the last chunk down to this one
//   (LDS lookups), then this chunk's 64-step walk (hmm.py:177-178).  The serial depth is
//   T/64 + 64 lookups instead of T dependent gathers.
#include <atomic>

#include "recur.h"
#include "post.h"
#include "follow.h"

namespace hmm355 {

// per-NP launcher (vit_kern.h, instantiated in vit_np64/128/256.hip)
template <int NP>
hipError_t launch_vit(const VitArgs& va, bool prep, hipStream_t sm);

}  // namespace hmm355

using namespace hmm355;

// OBS_PROB emissions: log(x + 1e-8) correctly rounded (logcr.h, the fp32 sum as hmm.py:152
// forms it) in one full-chip pass before the chain, which then stages them as OBS_LOG.  In the
// chain's staging the log cost ~60 ns per dense step (vit_fwd 725 us OBS_PROB vs 603 us
// OBS_LOG at B=32, T=2000, N=128, profiles/r5h_*), and on the banded chain, where one helper
// wave staged 2048 logs per 16-step block, it bounded the chain (vit_fwd 202 -> 163 us, the
// Viterbi op 229 -> 213 us, NS 269 -> 288 M frames/s, profiles/r5y*): this pass moves 2 x 33 MB
// instead.
__global__ void __launch_bounds__(256) vit_log_obs_kernel(const float* __restrict__ x, float* __restrict__ lo,
                                                          size_t n, int vec) {
  const size_t n4 = vec ? n / 4 : 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<float4*>(lo)[i] = make_float4(logcr_fast(v.x + 1e-8f, g_logcr_tab), logcr_fast(v.y + 1e-8f, g_logcr_tab),
                                                   logcr_fast(v.z + 1e-8f, g_logcr_tab), logcr_fast(v.w + 1e-8f, g_logcr_tab));
  }
  for (size_t i = 4 * n4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    lo[i] = logcr_fast(x[i] + 1e-8f, g_logcr_tab);
}

// the log-emission buffer: OBS_PROB decodes only (the log pass / log leaders write it)
static size_t vit_lobuf_bytes(int B, int T, int N, int obs_mode) {
  return obs_mode == HMM355_OBS_PROB ? align_up((size_t)B * T * N * sizeof(float), 256) : 0;
}

HMM355_API size_t hmm355_viterbi_workspace_bytes_ex(int B, int T, int N, int obs_mode) {
  if (B < 0 || T < 1 || N < 1 || N > 256) return 0;
  if (obs_mode != HMM355_OBS_PROB && obs_mode != HMM355_OBS_LOG) return 0;
  const size_t NP = pad_states(N);
  const size_t nc = (T + kChunk - 1) / kChunk;
  // psi rows, chunk maps, the plan-less band descriptor, the log-emissions (OBS_PROB), the
  // decode follower's chunk paths (follow.h), the psi followers' progress and done words, the
  // banded followers' counts (last)
  return align_up((size_t)B * T * NP, 256) + align_up((size_t)B * nc * NP, 256) + align_up(sizeof(BandDesc), 256) +
         vit_lobuf_bytes(B, T, N, obs_mode) + align_up((size_t)B * nc * kChunk * NP, 256) +
         align_up((size_t)B * kProgSlots * sizeof(int), 256) +
         align_up((size_t)B * nc, 256) + (size_t)2 * B * kPubStride * sizeof(int);
}

// (every encoding: the OBS_PROB size, the larger)
HMM355_API size_t hmm355_viterbi_workspace_bytes(int B, int T, int N) {
  return hmm355_viterbi_workspace_bytes_ex(B, T, N, HMM355_OBS_PROB);
}

// CUs of the current device, queried once per device (a relaxed atomic per slot: concurrent
// first calls may both query, and store the same value).  The psi followers take the CUs the
// chain leaves, at most one workgroup per CU (the launch owns a CU's LDS).
static constexpr int kFollowPerSeq = 2;

static int device_cus() {
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  int n = cus[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = -1;
    cus[dev].store(n, std::memory_order_relaxed);
  }
  return n > 0 ? n : 0;
}

// The decode beside a banded chain (HMM355_VIT_PLAN_BANDED, follow.h): the fused-psi chain
// (NP >= 128), one extra workgroup per sequence, and room for both on the chip with CUs to spare
// for a concurrent forward-backward (2B <= CUs / 2); the follower's chunk maps must fit its LDS and
// every per-sequence byte offset an int.
static bool vit_follow_ok(unsigned flags, const void* plan, int B, int T, int N) {
  const int NP = pad_states(N);
  return (flags & HMM355_VIT_PLAN_BANDED) && plan && NP >= 128 && 4 * B <= device_cus() &&
         vit_follow_lds_bytes(T, NP) <= kExclusiveLds && (size_t)T * NP * 4 < ((size_t)1 << 31) &&
         (size_t)T * N * 4 < ((size_t)1 << 31);
}

static int viterbi_run(const float* obs, int obs_mode, const float* log_P, const float* init, const void* plan,
                       unsigned flags, int B, int T, int N, int64_t* states, float* log_delta, float* final_score,
                       void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || N < 0) return HMM355_E_ARG;
  if (N < 1 || N > 256) return HMM355_E_STATES;
  if (T < 1) return HMM355_E_SHAPE;
  if (flags & ~(HMM355_VIT_PLAN_BANDED | HMM355_VIT_PLAN_DENSE)) return HMM355_E_ARG;
  if (B == 0) return HMM355_OK;
  if (!obs || !log_P || !init || !states || !log_delta || !workspace) return HMM355_E_ARG;
  if (obs_mode != HMM355_OBS_PROB && obs_mode != HMM355_OBS_LOG) return HMM355_E_ARG;
  if ((size_t)B * T > (size_t)1 << 40 || B > 65535) return HMM355_E_SHAPE;
  if ((size_t)T * N * sizeof(float) >= ((size_t)1 << 31)) return HMM355_E_SHAPE;  // (per-sequence buffer loads)
  if (workspace_bytes < hmm355_viterbi_workspace_bytes_ex(B, T, N, obs_mode)) return HMM355_E_WORKSPACE;
  const int NP = pad_states(N);
  const int nc = (T + kChunk - 1) / kChunk;
  uint8_t* psi = static_cast<uint8_t*>(workspace);
  uint8_t* G = psi + align_up((size_t)B * T * NP, 256);
  uint8_t* bandp = G + align_up((size_t)B * nc * NP, 256);
  float* lobuf = reinterpret_cast<float*>(bandp + align_up(sizeof(BandDesc), 256));
  uint8_t* path = reinterpret_cast<uint8_t*>(lobuf) + vit_lobuf_bytes(B, T, N, obs_mode);
  int* prog = reinterpret_cast<int*>(path + align_up((size_t)B * nc * kChunk * NP, 256));
  uint8_t* done = reinterpret_cast<uint8_t*>(prog) + align_up((size_t)B * kProgSlots * sizeof(int), 256);
  int* counts = reinterpret_cast<int*>(done + align_up((size_t)B * nc, 256));  // (2B x kPubStride) follow.h
  BandDesc* band = plan ? static_cast<BandDesc*>(const_cast<void*>(plan)) : reinterpret_cast<BandDesc*>(bandp);
  VitArgs va{obs, log_P, init, log_delta, final_score, states, psi, G, B, T, N, obs_mode, nc, band};
  hipStream_t sm = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (vit_follow_ok(flags, plan, B, T, N)) {
    // one launch: the chains, and per sequence a workgroup that first forms log(x + 1e-8) of
    // the sequence's emissions ahead of its chain (OBS_PROB) and then composes the chunk maps and
    // backtraces the path (follow.h).  The counts, one per 128-B line, zeroed first: [0, B) the
    // published psi blocks, [B, 2B) the leaders' blocks.
    if ((e = prepare_counts(counts, (size_t)2 * B * kPubStride * sizeof(int), sm, &va.token)) != hipSuccess) return (int)e;
    va.pub = counts;
    va.path = path;
    if (obs_mode == HMM355_OBS_PROB) {
      va.lobuf = lobuf;
      va.lready = counts + (size_t)B * kPubStride;
    }
    va.nfollow = B;
    switch (NP) {
      case 128: e = launch_vit<128>(va, false, sm); break;
      default: e = launch_vit<256>(va, false, sm); break;
    }
    return e == hipSuccess ? HMM355_OK : (int)e;
  }
  // psi followers: the caller's word that the plan is dense, N <= 128, and CUs beside the chain.
  // A chain publishes a 64-step chunk every ~17 us (dense step ~270 ns) and a follower takes
  // ~25-30 us per chunk, so two followers per sequence keep up; more would only hold CUs (each
  // owns one: the launch asks for the CU's whole LDS) that a concurrent op on another stream
  // could use.  With nfollow = 2B follower f serves sequence f mod B, every other chunk.
  if ((flags & HMM355_VIT_PLAN_DENSE) && plan && NP <= 128) {
    const long room = (long)device_cus() - B;
    const long tasks = (long)B * nc;
    long nf = room < tasks ? room : tasks;
    if (nf > (long)kFollowPerSeq * B) nf = (long)kFollowPerSeq * B;
    va.nfollow = (int)(nf > 0 ? nf : 0);
    va.prog = prog;
    va.done = done;
  }
  // OBS_PROB emissions otherwise: the full-chip log pass before the chain (vit_log_obs_kernel)
  if (obs_mode == HMM355_OBS_PROB) {
    const size_t n = (size_t)B * T * N;
    size_t blocks = (n / 4 + 255) / 256;
    blocks = blocks < 8192 ? (blocks > 0 ? blocks : 1) : 8192;
    const int vec = (reinterpret_cast<uintptr_t>(obs) & 15) == 0;  // (lobuf is 256-B aligned)
    hipLaunchKernelGGL(vit_log_obs_kernel, dim3((unsigned)blocks), dim3(256), 0, sm, obs, lobuf, n, vec);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    va.obs = lobuf;
    va.obs_mode = HMM355_OBS_LOG;
  }
  switch (NP) {
    case 64: e = launch_vit<64>(va, plan == nullptr, sm); break;
    case 128: e = launch_vit<128>(va, plan == nullptr, sm); break;
    default: e = launch_vit<256>(va, plan == nullptr, sm); break;
  }
  return e == hipSuccess ? HMM355_OK : (int)e;
}

HMM355_API int hmm355_viterbi_plan_ex_f32(const float* obs, int obs_mode, const float* log_P, const float* init,
                                          const void* plan, unsigned flags, int B, int T, int N, int64_t* states,
                                          float* log_delta, float* final_score, void* workspace,
                                          size_t workspace_bytes, void* stream) {
  return viterbi_run(obs, obs_mode, log_P, init, plan, flags, B, T, N, states, log_delta, final_score, workspace,
                     workspace_bytes, stream);
}

HMM355_API int hmm355_viterbi_plan_f32(const float* obs, int obs_mode, const float* log_P, const float* init,
                                       const void* plan, int B, int T, int N, int64_t* states, float* log_delta,
                                       float* final_score, void* workspace, size_t workspace_bytes, void* stream) {
  return hmm355_viterbi_plan_ex_f32(obs, obs_mode, log_P, init, plan, 0u, B, T, N, states, log_delta, final_score,
                                    workspace, workspace_bytes, stream);
}

HMM355_API int hmm355_viterbi_f32(const float* obs, int obs_mode, const float* log_P, const float* init, int B,
                                  int T, int N, int64_t* states, float* log_delta, float* final_score,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  return hmm355_viterbi_plan_f32(obs, obs_mode, log_P, init, nullptr, B, T, N, states, log_delta, final_score,
                                 workspace, workspace_bytes, stream);
}

