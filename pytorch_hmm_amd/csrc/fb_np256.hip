// hmm355 — forward-backward kernels for NP = 256 (fb_kern.h; one translation unit per NP).
#include "fb_kern.h"

namespace hmm355 {
template hipError_t launch_fb<256>(const RecArgs& fa, const RecArgs& fb, const PostArgs& pa, bool prep,
                                   hipStream_t st, int nfollow);
}  // namespace hmm355
