// hmm355 — Viterbi kernels for NP = 256 (vit_kern.h; one translation unit per NP).
#include "vit_kern.h"

namespace hmm355 {
template hipError_t launch_vit<256>(const VitArgs& va, bool prep, hipStream_t sm);
}  // namespace hmm355
