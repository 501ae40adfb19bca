// Exhaustive check of csrc/logcr.h (TEST INFRASTRUCTURE): for every fp32 bit pattern s in
// [lo_bits, hi_bits) (default: all 2^32), logcr_fast(s) must equal (float)logl((long double)s), the log
// correctly rounded to fp32 (x87 64-bit significand, rounded once more: wrong only within
// 2^-64 relative of a midpoint).  Also counts where it differs from (float)log((double)s), the
// value the chains used before (common.h log_obs_cr), whose double rounding is off on a few
// inputs.  NaN matches any NaN.  Prints up to 20 mismatching inputs ("bad 0x...") and "mismatches N olddiff D
// checked M"; the exit status is 0 (tests/test_logcr.py judges the list).
// Build: g++ -O2 -fopenmp -ffp-contract=off (tests/test_logcr.py).
#include <stdio.h>
#include <stdlib.h>
#include "../pytorch_hmm_amd/csrc/logcr.h"

static const double kTab[256] = {HMM355_LOGCR_TABLE};

int main(int argc, char** argv) {
  const uint64_t lo = argc > 1 ? strtoull(argv[1], 0, 0) : 0;
  const uint64_t hi = argc > 2 ? strtoull(argv[2], 0, 0) : 0x100000000ull;
  long long bad = 0, olddiff = 0;
  const long long n = (long long)hi - (long long)lo;
#pragma omp parallel for reduction(+ : bad, olddiff) schedule(static, 1 << 16)
  for (long long k = 0; k < n; ++k) {
    const uint32_t b = (uint32_t)(lo + (uint64_t)k);
    float s;
    memcpy(&s, &b, 4);
    const float ref = (float)logl((long double)s);
    const float old = (float)log((double)s);
    const float got = hmm355::logcr_fast(s, kTab);
    const bool nan_ok = isnan(ref) && isnan(got), nan_old = isnan(old) && isnan(got);
    if (!nan_old && memcmp(&old, &got, 4) != 0) ++olddiff;
    if (!nan_ok && memcmp(&ref, &got, 4) != 0) {
      ++bad;
      if (bad <= 20) {
#pragma omp critical
        printf("bad 0x%08x s=%a ref=%a got=%a old=%a\n", b, s, ref, got, old);
      }
    }
  }
  printf("mismatches %lld olddiff %lld checked %lld\n", bad, olddiff, n);
  return 0;
}
