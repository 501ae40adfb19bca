// hmm355 — C ABI housekeeping (error strings, version).
#include "common.h"

HMM355_API int hmm355_version(void) { return 1; }

HMM355_API const char* hmm355_strerror(int code) {
  switch (code) {
    case HMM355_OK: return "ok";
    case HMM355_E_ARG: return "invalid argument (null pointer, negative size or unknown mode)";
    case HMM355_E_STATES: return "number of states outside the op's range (HMM recursions [1, 256], HSMM [1, 1024])";
    case HMM355_E_SHAPE: return "invalid shape (T < 1 or size overflow)";
    case HMM355_E_WORKSPACE: return "workspace too small";
    case HMM355_E_DURATION: return "HSMM max_duration outside [1, 1024]";
    default: break;
  }
  if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
  return "unknown hmm355 error";
}
