// hmm355 — forward-backward kernels for NP = 128 (fb_kern.h; one translation unit per NP).
#include "fb_kern.h"

namespace hmm355 {
template hipError_t launch_fb<128>(const RecArgs& fa, const RecArgs& fb, const PostArgs& pa, bool prep,
                                   hipStream_t st, int nfollow);
template hipError_t launch_fb_pair<128>(const PairArgs& pa, int B, hipStream_t st);
}  // namespace hmm355

// diagnostic builds: the stamps live in this translation unit's code object (recur.h)
#if HMM355_STAMP
HMM355_API int hmm355_debug_stamps_fb(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hmm355::g_rec_stamps), sizeof(unsigned long long) * (size_t)n);
}
#endif
