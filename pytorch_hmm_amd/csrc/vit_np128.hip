// hmm355 — Viterbi kernels for NP = 128 (vit_kern.h; one translation unit per NP).
#include "vit_kern.h"

namespace hmm355 {
template hipError_t launch_vit<128>(const VitArgs& va, bool prep, hipStream_t sm);
}  // namespace hmm355

// diagnostic builds: the stamps live in this translation unit's code object (recur.h)
#if HMM355_STAMP
HMM355_API int hmm355_debug_stamps_vit(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hmm355::g_rec_stamps), sizeof(unsigned long long) * (size_t)n);
}
#endif
