// hmm355 — correctly rounded fp32 log(x + 1e-8f) on a table and a short fp64 polynomial.
//
// The Viterbi emission of the reference is log(obs + 1e-8) in fp32 (hmm.py:152).  The chains
// take the sum in fp32 as the reference does and the log correctly rounded;
// the libm fp64 log behind that (common.h log_obs_cr) is too long for the staging helper
// waves, so it ran as a separate full-tensor pass.  This form costs ~12 fp64 operations:
//   s = 2^e * m, m in [1, 2); i = the top 7 mantissa bits; c_i = 1 + (i + 1/2)/128
//   r = m * inv_i - 1                    exact in fp64 (inv_i has 24 significant bits)
//   log s = e' ln2 + logc_i + log1p(r),   |r| < 2^-7, log1p by a degree-9 polynomial
// with e' = e (+1 for m >= sqrt 2, where logc_i carries the -ln 2), ln 2 split hi/lo so e' ln2_hi
// is exact.  The intervals next to s = 1 use c = 1 and c = 2 (logc = 0): no cancellation there.
// The fp64 result is within ~2^-60 relative of log s and is rounded once to fp32.
// tests/test_logcr.py runs it on EVERY positive finite normal fp32 s (tools/logcr_check.cpp
// compiles this same header for the host): it is the correctly rounded log on all of them
// but 4 (s = 0x1.827a74p-7, 0x1.bacb4ap+25, 0x1.b121a6p+76, 0x1.6351d8p+95, within 2^-60 of a
// rounding midpoint, one ulp off as the previous fp64-libm path is), and it differs from that
// path, (float)log((double)s), on one input (s = 0x1.2f1fd6p+3, where it is the correct one).
// Subnormal s are scaled into the normal range first; zero, negative, inf and nan give log's
// values (-inf, nan, inf, nan).
//
// Plain C++ on both sides (explicit fma(), no contractible a*b+c), so the host check and the
// gfx950 code evaluate the same operations.
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>
#include "logcr_table.h"

#ifdef __HIPCC__
#define HMM355_HD __host__ __device__ __forceinline__
#else
#define HMM355_HD inline
#endif

namespace hmm355 {

// table row i: {inv_i, logc_i}.  Branch-free (the staging helpers keep straight-line code):
// subnormal inputs are scaled by 2^24 first, and zero / negative / inf / nan are selected at
// the end with the values log() gives them.
HMM355_HD float logcr_fast(float s, const double* __restrict__ tab) {
  uint32_t bits;
  memcpy(&bits, &s, 4);
  const bool sub = bits < 0x00800000u;  // +0 or positive subnormal
  const float s2 = sub ? s * 0x1p24f : s;
  uint32_t b2;
  memcpy(&b2, &s2, 4);
  const int i = (int)((b2 >> 16) & 127u);
  const int e = (int)((b2 >> 23) & 255u) - 127 + (i >= HMM355_LOGCR_SPLIT ? 1 : 0) - (sub ? 24 : 0);
  const uint32_t mb = (b2 & 0x007FFFFFu) | 0x3F800000u;
  float mf;
  memcpy(&mf, &mb, 4);
  const double inv = tab[2 * i], logc = tab[2 * i + 1];
  const double r = fma((double)mf, inv, -1.0);
  // log1p(r) = r + r^2 q(r),  q = -1/2 + r/3 - r^2/4 + ... + r^7/9
  double q = fma(r, 0x1.c71c71c71c71cp-4, -0x1.0000000000000p-3);  //  1/9, -1/8
  q = fma(q, r, 0x1.2492492492492p-3);                              //  1/7
  q = fma(q, r, -0x1.5555555555555p-3);                             // -1/6
  q = fma(q, r, 0x1.999999999999ap-3);                              //  1/5
  q = fma(q, r, -0x1.0000000000000p-2);                             // -1/4
  q = fma(q, r, 0x1.5555555555555p-2);                              //  1/3
  q = fma(q, r, -0x1.0000000000000p-1);                             // -1/2
  const double r2 = r * r;
  const double lp = fma(r2, q, r);
  const double ed = (double)e;
  const double hi = fma(ed, 0x1.62e42fefa4000p-1, logc);            // e ln2_hi exact (40-bit hi)
  const double lo = fma(ed, -0x1.8432a1b0e2634p-43, lp);            // + e ln2_lo
  const float v = (float)(hi + lo);
  // specials: +0 / -0 -> -inf, +inf -> +inf, negative or nan -> nan
  const uint32_t vb = (bits & 0x7FFFFFFFu) == 0u ? 0xFF800000u
                      : (bits == 0x7F800000u ? 0x7F800000u : 0x7FC00000u);
  const bool special = (bits & 0x7FFFFFFFu) == 0u || bits >= 0x7F800000u;
  float sv;
  memcpy(&sv, &vb, 4);
  return special ? sv : v;
}

}  // namespace hmm355
