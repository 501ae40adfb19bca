// hmm355 — shared device helpers for the gfx950 (CDNA4) kernels.
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/hmm355.h"

#define HMM355_API extern "C" __attribute__((visibility("default")))

// Ablation knobs for diagnostic builds only (tools/ablate.py); 0 in the product build.
#ifndef HMM355_ABL
#define HMM355_ABL 0
#endif

#ifndef HMM355_STAMP
#define HMM355_STAMP 0
#endif

// Ablation knobs of the work beside the chains (csrc/follow.h), diagnostic builds only: 1 no
// per-block publishing (completion only), 2 followers return at once (timing only), 4 plain
// instead of write-through row / psi stores (timing only), 8 no log leaders.
#ifndef HMM355_FBR
#define HMM355_FBR 4  // posterior rows per follower wave per pass (follow.h)
#endif
#ifndef HMM355_FBF
#define HMM355_FBF 0  // diagnostic builds: posterior followers per sequence (0: the host's choice)
#endif
#ifndef HMM355_FABL
#define HMM355_FABL 0
#endif

namespace hmm355 {

constexpr int kWave = 64;
constexpr bool kStamp = HMM355_STAMP;

// In-kernel cycle stamp (diagnostic builds only, cdna guide §7): s_memtime with its
// lgkmcnt wait in ONE asm statement, fenced by sched_barrier on both sides.
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
template <typename T>
__device__ __forceinline__ void keep(T& v) { asm volatile("" : "+v"(v)); }
constexpr int kAbl = HMM355_ABL;
constexpr int kFAbl = HMM355_FABL;

// compile-time loop: f(integral_constant<int, J>) for J in [B, E)
template <int J, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (J < E) {
    f(std::integral_constant<int, J>{});
    static_for<J + 1, E>(f);
  }
}

// ---- DPP: row_newbcast:N — every lane of a 16-lane row receives lane N of that row. ----
template <int N>
__device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + N, 0xF, 0xF, false));
}

// acc += row_bcast<N>(v) * m as ONE instruction (v_fmac_f32_dpp).  hipcc does not fold the
// DPP mov into v_fmac, so it is written out; the hazard recognizer still pads around it.
template <int N>
__device__ __forceinline__ void fmac_bcast(float& acc, float v, float m) {
  asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(v), "v"(m), "n"(N));
}

// ---- cross-lane sums / maxima without LDS ----
// v_permlane16_swap / v_permlane32_swap written out: hipcc 7.2's
// __builtin_amdgcn_permlane{16,32}_swap reads the same register for both halves of the
// returned pair (miscompile observed at -O0 and -O3), so the pair is kept in two named
// VGPRs here.  "s_nop 1" covers the VALU-write -> permlane-read hazard inside the asm.
__device__ __forceinline__ void permlane16_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void permlane32_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void permlane16_swap_i(int& a, int& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void permlane32_swap_i(int& a, int& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}

// sum over the four 16-lane rows of a wave (lanes c, c+16, c+32, c+48), result in every lane
__device__ __forceinline__ float rows_sum(float x) {
  float a = x, b = x;
  permlane16_swap(a, b);   // a = rows [0,0,2,2], b = rows [1,1,3,3]
  float y = a + b;
  float c = y, d = y;
  permlane32_swap(c, d);   // c = halves [0,0], d = halves [1,1]
  return c + d;
}

__device__ __forceinline__ float rows_max(float x) {
  float a = x, b = x;
  permlane16_swap(a, b);
  float y = fmaxf(a, b);
  float c = y, d = y;
  permlane32_swap(c, d);
  return fmaxf(c, d);
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float,
                            __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// sum over the 16 lanes of a row (all lanes of the row get the row sum)
__device__ __forceinline__ float row16_sum(float x) {
  x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_f<0x124>(x);  // row_ror:4
  x += dpp_f<0x128>(x);  // row_ror:8
  return x;
}

// (value, index) argmax combine: larger value wins; equal values -> smaller index
__device__ __forceinline__ void argmax_combine(float& v, int& i, float v2, int i2) {
  // bitwise, not short-circuit: || / && here compile to exec-mask branches
  const bool take = (v2 > v) | ((v2 == v) & (i2 < i));
  v = take ? v2 : v;
  i = take ? i2 : i;
}

// full-wave (value, index) argmax via ds_bpermute-free shuffles (used off the hot loop)
__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    float v2 = __shfl_xor(v, off);
    int i2 = __shfl_xor(i, off);
    argmax_combine(v, i, v2, i2);
  }
}

// full-wave (value, index) argmax on DPP + permlane swaps (no LDS round trips): the four
// in-row levels by quad_perm / row_ror, then the two cross-row levels by permlane16/32 swaps.
// Every lane ends with the wave's (max value, smallest index attaining it).
__device__ __forceinline__ void wave_argmax_dpp(float& v, int& i) {
  argmax_combine(v, i, dpp_f<0xB1>(v), dpp_i<0xB1>(i));
  argmax_combine(v, i, dpp_f<0x4E>(v), dpp_i<0x4E>(i));
  argmax_combine(v, i, dpp_f<0x124>(v), dpp_i<0x124>(i));
  argmax_combine(v, i, dpp_f<0x128>(v), dpp_i<0x128>(i));
  float a = v, b = v;
  int ia = i, ib = i;
  permlane16_swap(a, b);
  permlane16_swap_i(ia, ib);
  argmax_combine(a, ia, b, ib);
  float c = a, d = a;
  int ic = ia, id = ia;
  permlane32_swap(c, d);
  permlane32_swap_i(ic, id);
  argmax_combine(c, ic, d, id);
  v = c;
  i = ic;
}

// all-lane wave sum / max on DPP + permlane swaps (no LDS round trips)
__device__ __forceinline__ float wave_sum_dpp(float x) { return rows_sum(row16_sum(x)); }
__device__ __forceinline__ float wave_max_dpp2(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x124>(x));
  x = fmaxf(x, dpp_f<0x128>(x));
  return rows_max(x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}

// Correctly rounded fp32 log(x + 1e-8f): the sum is formed in fp32 exactly as the
// reference does (hmm.py:86), the log in fp64 then rounded once.  torch-CPU's logf agrees
// with the correctly rounded value on all but ~2.5e-5 of softmax-distributed inputs.
__device__ __forceinline__ float log_obs_cr(float x) {
  float s = x + 1e-8f;
  return (float)log((double)s);
}

// LDS barrier: waits for this wave's LDS ops, then s_barrier.  Global stores stay in flight
// (no vmcnt(0) per step); the "memory" clobber keeps the compiler from moving LDS accesses
// across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// the per-time-step barrier of the recursions (ablation bit 1 drops it: timing only)
__device__ __forceinline__ void step_barrier() {
  if constexpr (kAbl & 1)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else
    lds_barrier();
}

// Allow a kernel more than the default 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU).
template <typename K>
inline hipError_t allow_lds(K kernel, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                             static_cast<int>(bytes));
}

constexpr size_t kExclusiveLds = 160 * 1024;  // a workgroup that owns its CU

// ---- hand-offs between workgroups of one launch (MI355X_MICROARCH.md, inter-workgroup
// visibility; cdna_hip_programming.md Guideline 16, R1): payload stored write-through (sc1),
// every storing wave's stores complete before a workgroup barrier, then ONE lane stores the
// count (relaxed, agent scope: an sc1 store); the consumer polls the count relaxed and loads the
// payload with sc1 loads only (no L1 copy can be stale), so neither side needs a fence.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
constexpr int kAuxSc1 = 16;  // buffer instruction cache-policy bits: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// published counts sit one per 128-B line (no two counters share a line: a chain's store and
// another chain's follower polls never meet on one)
constexpr int kPubStride = 32;
// A count is one 8-byte word {call token, count ^ mix(token)}, stored and polled whole (8-B
// granules are untorn).  An eager call takes a fresh nonzero token (count_token()), so the
// words a previous call or any other use of the workspace left behind read as 0 -- no reset
// launch before the chains; a stale word passes only if its high half equals the token AND its
// low half decodes to a count <= cap.  Token 0 (calls captured into a HIP graph, whose replays
// share one token) keeps the reset kernel below before every launch.
__device__ __host__ __forceinline__ unsigned count_mix(unsigned token) { return token * 2654435761u; }
__device__ __forceinline__ int poll_count(const int* p, unsigned token, int cap) {
  const unsigned long long v =
      __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned c = (unsigned)v ^ count_mix(token);
  return ((unsigned)(v >> 32) == token && c <= (unsigned)cap) ? (int)c : 0;
}
__device__ __forceinline__ void publish_count(int* p, int v, unsigned token) {
  const unsigned long long w = ((unsigned long long)token << 32) | ((unsigned)v ^ count_mix(token));
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a fresh nonzero token per eager call (process-wide, wraps past 0)
inline unsigned next_count_token() {
  static std::atomic<unsigned> g_token{0x5bd1e995u};
  unsigned t;
  do t = g_token.fetch_add(0x9e3779b9u, std::memory_order_relaxed) + 0x9e3779b9u; while (t == 0u);
  return t;
}
// true while `st` is being captured into a graph (its replays would share one token)
inline bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Zeroes n 4-byte words (the followers' counters under token 0) as a kernel node: a
// hipMemsetAsync captured into a HIP graph was measured not to order against the chain launch
// that follows it in replay (the followers then saw the previous replay's final counts;
// tools/diag_graph.py)
static __global__ void zero_words_kernel(unsigned* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0u;
}
inline hipError_t zero_words(void* p, size_t bytes, hipStream_t st) {
  const int n = (int)((bytes + 3) / 4);
  const int blocks = n < 256 * 64 ? (n + 255) / 256 : 64;
  hipLaunchKernelGGL(zero_words_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, static_cast<unsigned*>(p), n);
  return hipGetLastError();
}
// the counts before a publishing launch: a fresh token for an eager call, else token 0 and
// the reset kernel
inline hipError_t prepare_counts(void* p, size_t bytes, hipStream_t st, unsigned* token) {
  if (!stream_capturing(st)) {
    *token = next_count_token();
    return hipSuccess;
  }
  *token = 0u;
  return zero_words(p, bytes, st);
}

inline int pad_states(int N) { return N <= 64 ? 64 : (N <= 128 ? 128 : 256); }

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace hmm355
