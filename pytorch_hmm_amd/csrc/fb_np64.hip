// hmm355 — forward-backward kernels for NP = 64 (fb_kern.h; one translation unit per NP).
#include "fb_kern.h"

namespace hmm355 {
template hipError_t launch_fb<64>(const RecArgs& fa, const RecArgs& fb, const PostArgs& pa, bool prep,
                                   hipStream_t st, int nfollow);
template hipError_t launch_fb_pair<64>(const PairArgs& pa, int B, hipStream_t st);
}  // namespace hmm355
