// hmm355 — forward-backward kernels and their per-NP launchers (included by fb_np*.hip, one
// translation unit per padded state count, so the three instantiations compile in parallel).
#pragma once
#include "recur.h"
#include "post.h"
#include "fbpair.h"
#include "follow.h"

namespace hmm355 {


// blockIdx.x = 2b + direction: the chains; with publishing chains (fa.pub) blockIdx.x = 2B + b
// is sequence b's posterior follower (follow.h)
template <int NP>
__global__ void __launch_bounds__(kFbNT<NP>) fb_recur_kernel(RecArgs fa, RecArgs fb, float* posterior) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if ((int)blockIdx.x >= 2 * fa.B) {
    fb_post_follow<NP>(fa, fb, posterior, (int)blockIdx.x - 2 * fa.B, lds);
    return;
  }
  const int b = blockIdx.x >> 1;
  if (blockIdx.x & 1) {
    if (!(kAbl & (1 << 20))) rec_dispatch<NP, kFbBeta>(fb, lds, b);  // diagnostic: alpha only
  } else {
    if (!(kAbl & (1 << 21))) rec_dispatch<NP, kFbAlpha>(fa, lds, b);  // diagnostic: beta only
  }
}

template <int NP>
hipError_t launch_fb(const RecArgs& fa, const RecArgs& fb, const PostArgs& pa, bool prep, hipStream_t st, int nfollow) {
  hipError_t e = allow_lds(fb_recur_kernel<NP>, kExclusiveLds);  // own the CU (recur.h)
  if (e != hipSuccess) return e;
  if (fa.band && prep) {
    e = launch_band_prep(fa.mat, fa.N, const_cast<BandDesc*>(fa.band), st);
    if (e != hipSuccess) return e;
  }
  if (fa.pub) {
    // posterior followers beside the banded chains (follow.h): 2B chains + F*B followers (F from
    // the host: fb.hip), no pass after
    unsigned token = 0;
    e = prepare_counts(fa.pub, (size_t)2 * fa.B * kPubStride * sizeof(int), st, &token);
    if (e != hipSuccess) return e;
    RecArgs ta = fa, tb = fb;
    ta.token = tb.token = token;
    hipLaunchKernelGGL(fb_recur_kernel<NP>, dim3((2 + nfollow) * fa.B), dim3(kFbNT<NP>), kExclusiveLds, st, ta, tb,
                       pa.posterior);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(fb_recur_kernel<NP>, dim3(2 * fa.B), dim3(kFbNT<NP>), kExclusiveLds, st, fa, fb, pa.posterior);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t rows = (size_t)pa.B * pa.T;
  const size_t waves = rows < (size_t)kPostWaves ? rows : (size_t)kPostWaves;
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  hipLaunchKernelGGL(fb_posterior_kernel<NP>, dim3(blocks), dim3(256), 0, st, pa);
  return hipGetLastError();
}


// both chains of a sequence in one workgroup (fbpair.h), NP <= 128
template <int NP>
hipError_t launch_fb_pair(const PairArgs& pa, int B, hipStream_t st) {
  hipError_t e = allow_lds(fb_pair_kernel<NP>, PairL<NP>::LDS_FLOATS * sizeof(float));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fb_pair_kernel<NP>, dim3(B), dim3(PairL<NP>::NT), PairL<NP>::LDS_FLOATS * sizeof(float), st, pa);
  return hipGetLastError();
}

}  // namespace hmm355
