/*
 * TEST INFRASTRUCTURE ONLY — plain-C parity oracle for the HMM hot path.
 * Never linked into the product (pytorch_hmm_amd); loaded by tests/ and bench.py's
 * cpu_baseline leg through ctypes (oracle/lib/liboracle.so, built by oracle/Makefile).
 *
 * Restates, from the reference's published behaviour (crlotwhite/pytorch_hmm):
 *   viterbi_f32         hmm.py:154-184 and mixture_gaussian.py:306-338 — max-plus recursion,
 *                       first-index argmax on ties (torch.max / torch.argmax semantics).
 *                       Bit-exact given identical fp32 log-emissions: every delta is one
 *                       fp32 add of an exact max, independent of reduction order.
 *   fb_f64              hmm.py:89-130 in float64 (tolerance reference, not bit-exact).
 *   gmm_diag_f64        mixture_gaussian.py:157-214 in float64 (tolerance reference).
 *   hsmm_viterbi_literal hsmm.py:245-354, the literal 5-deep loop, incl. torch's CPU order
 *                       for sum(obs_log_probs[t:t+d, s]): ATen's cascade_sum restated
 *                       (torch_sum_f32 below; equal to torch.sum for every d = 1..1024).
 *   tv_viterbi_f32      neural.py:463-511 — Viterbi with one transition matrix per step
 *                       (log_A (B,T,N,N); step t uses matrix t-1), exact as viterbi_f32.
 *   tv_fb_f64           neural.py:391-461 in float64 (forward step t uses matrix t-1,
 *                       backward step t matrix t; tolerance reference).
 *   hsmm_viterbi_fast   the same recursion reorganised (max over d' hoisted out of the
 *                       candidate loop, exact tie re-resolution per d) — bit-identical to
 *                       the literal form; cross-checked in tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <stddef.h>
#include <string.h>

/* ---------------------------------------------------------------- Viterbi (exact) */
void viterbi_f32(const float* log_obs, const float* log_P, const float* init, int B, int T,
                 int N, int64_t* states, float* delta, uint8_t* psi_opt) {
    uint8_t* psi = psi_opt ? psi_opt : (uint8_t*)malloc((size_t)T * N);
    for (int b = 0; b < B; ++b) {
        const float* lo = log_obs + (size_t)b * T * N;
        float* dl = delta + (size_t)b * T * N;
        uint8_t* ps = psi_opt ? psi + (size_t)b * T * N : psi;
        for (int j = 0; j < N; ++j) { dl[j] = init[j] + lo[j]; ps[j] = 0; }
        for (int t = 1; t < T; ++t) {
            const float* dp = dl + (size_t)(t - 1) * N;
            for (int j = 0; j < N; ++j) {
                float best = dp[0] + log_P[j];
                int bi = 0;
                for (int i = 1; i < N; ++i) {
                    float s = dp[i] + log_P[(size_t)i * N + j];
                    if (s > best) { best = s; bi = i; }
                }
                dl[(size_t)t * N + j] = best + lo[(size_t)t * N + j];
                ps[(size_t)t * N + j] = (uint8_t)bi;   /* N <= 256 */
            }
        }
        const float* dlast = dl + (size_t)(T - 1) * N;
        int s = 0;
        for (int j = 1; j < N; ++j) if (dlast[j] > dlast[s]) s = j;
        int64_t* st = states + (size_t)b * T;
        st[T - 1] = s;
        for (int t = T - 2; t >= 0; --t) { s = ps[(size_t)(t + 1) * N + s]; st[t] = s; }
    }
    if (!psi_opt) free(psi);
}

/* ------------------------------------------------------- forward-backward (float64) */
static double lse(const double* v, int n) {
    double m = -INFINITY;
    for (int i = 0; i < n; ++i) if (v[i] > m) m = v[i];
    if (!isfinite(m)) return m;
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += exp(v[i] - m);
    return m + log(s);
}

/* log_alpha/log_beta/posterior are (B,T,N) float64; loglik (B) = LSE(alpha_{T-1}). */
void fb_f64(const float* log_obs, const float* log_P, const float* log_p0, int B, int T, int N,
            double* log_alpha, double* log_beta, double* posterior, double* loglik) {
    double* tmp = (double*)malloc(sizeof(double) * N);
    for (int b = 0; b < B; ++b) {
        const float* lo = log_obs + (size_t)b * T * N;
        double* la = log_alpha + (size_t)b * T * N;
        double* lb = log_beta + (size_t)b * T * N;
        for (int j = 0; j < N; ++j) la[j] = (double)log_p0[j] + lo[j];
        for (int t = 1; t < T; ++t)
            for (int j = 0; j < N; ++j) {
                for (int i = 0; i < N; ++i) tmp[i] = la[(size_t)(t - 1) * N + i] + log_P[(size_t)i * N + j];
                la[(size_t)t * N + j] = lse(tmp, N) + lo[(size_t)t * N + j];
            }
        for (int j = 0; j < N; ++j) lb[(size_t)(T - 1) * N + j] = 0.0;
        for (int t = T - 2; t >= 0; --t)
            for (int i = 0; i < N; ++i) {
                for (int j = 0; j < N; ++j)
                    tmp[j] = (double)log_P[(size_t)i * N + j] + lo[(size_t)(t + 1) * N + j] + lb[(size_t)(t + 1) * N + j];
                lb[(size_t)t * N + i] = lse(tmp, N);
            }
        for (int t = 0; t < T; ++t) {
            double* pr = posterior + ((size_t)b * T + t) * N;
            for (int j = 0; j < N; ++j) tmp[j] = la[(size_t)t * N + j] + lb[(size_t)t * N + j];
            double z = lse(tmp, N);
            for (int j = 0; j < N; ++j) pr[j] = exp(tmp[j] - z);
        }
        loglik[b] = lse(la + (size_t)(T - 1) * N, N);
    }
    free(tmp);
}

/* ------------------------------------------- time-varying transitions (NeuralHMM) */
/* log_A element (b,k,i,j) at log_A[b*sb + k*st + i*N + j] (sb = st = 0: one matrix). */
void tv_viterbi_f32(const float* log_obs, const float* log_A, long long sb, long long st,
                    const float* init, int B, int T, int N, int64_t* states, float* delta) {
    uint8_t* ps = (uint8_t*)malloc((size_t)T * N);
    for (int b = 0; b < B; ++b) {
        const float* lo = log_obs + (size_t)b * T * N;
        float* dl = delta + (size_t)b * T * N;
        for (int j = 0; j < N; ++j) { dl[j] = init[j] + lo[j]; ps[j] = 0; }
        for (int t = 1; t < T; ++t) {
            const float* A = log_A + (size_t)b * sb + (size_t)(t - 1) * st;
            const float* dp = dl + (size_t)(t - 1) * N;
            for (int j = 0; j < N; ++j) {
                float best = dp[0] + A[j];
                int bi = 0;
                for (int i = 1; i < N; ++i) {
                    float s = dp[i] + A[(size_t)i * N + j];
                    if (s > best) { best = s; bi = i; }
                }
                dl[(size_t)t * N + j] = best + lo[(size_t)t * N + j];
                ps[(size_t)t * N + j] = (uint8_t)bi;
            }
        }
        const float* dlast = dl + (size_t)(T - 1) * N;
        int s = 0;
        for (int j = 1; j < N; ++j) if (dlast[j] > dlast[s]) s = j;
        int64_t* so = states + (size_t)b * T;
        so[T - 1] = s;
        for (int t = T - 2; t >= 0; --t) { s = ps[(size_t)(t + 1) * N + s]; so[t] = s; }
    }
    free(ps);
}

void tv_fb_f64(const float* log_obs, const float* log_A, long long sb, long long st,
               const float* log_p0, int B, int T, int N, double* log_alpha, double* log_beta,
               double* posterior, double* loglik) {
    double* tmp = (double*)malloc(sizeof(double) * N);
    for (int b = 0; b < B; ++b) {
        const float* lo = log_obs + (size_t)b * T * N;
        double* la = log_alpha + (size_t)b * T * N;
        double* lb = log_beta + (size_t)b * T * N;
        for (int j = 0; j < N; ++j) la[j] = (double)log_p0[j] + lo[j];
        for (int t = 1; t < T; ++t) {
            const float* A = log_A + (size_t)b * sb + (size_t)(t - 1) * st;
            for (int j = 0; j < N; ++j) {
                for (int i = 0; i < N; ++i) tmp[i] = la[(size_t)(t - 1) * N + i] + A[(size_t)i * N + j];
                la[(size_t)t * N + j] = lse(tmp, N) + lo[(size_t)t * N + j];
            }
        }
        for (int j = 0; j < N; ++j) lb[(size_t)(T - 1) * N + j] = 0.0;
        for (int t = T - 2; t >= 0; --t) {
            const float* A = log_A + (size_t)b * sb + (size_t)t * st;
            for (int i = 0; i < N; ++i) {
                for (int j = 0; j < N; ++j)
                    tmp[j] = (double)A[(size_t)i * N + j] + lo[(size_t)(t + 1) * N + j] + lb[(size_t)(t + 1) * N + j];
                lb[(size_t)t * N + i] = lse(tmp, N);
            }
        }
        for (int t = 0; t < T; ++t) {
            double* pr = posterior + ((size_t)b * T + t) * N;
            for (int j = 0; j < N; ++j) tmp[j] = la[(size_t)t * N + j] + lb[(size_t)t * N + j];
            double z = lse(tmp, N);
            for (int j = 0; j < N; ++j) pr[j] = exp(tmp[j] - z);
        }
        loglik[b] = lse(la + (size_t)(T - 1) * N, N);
    }
    free(tmp);
}

/* ------------------------------------------------ diagonal GMM emission (float64) */
void gmm_diag_f64(const float* x, const float* means, const float* log_vars, const float* log_w,
                  int B, int T, int D, int S, int C, double* out) {
    const double l2pi = log(2.0 * M_PI);
    double* comp = (double*)malloc(sizeof(double) * C);
    for (size_t f = 0; f < (size_t)B * T; ++f) {
        const float* xf = x + f * D;
        for (int s = 0; s < S; ++s) {
            for (int c = 0; c < C; ++c) {
                const float* mu = means + ((size_t)s * C + c) * D;
                const float* lv = log_vars + ((size_t)s * C + c) * D;
                double q = 0.0, slv = 0.0;
                for (int d = 0; d < D; ++d) {
                    double df = (double)xf[d] - mu[d];
                    q += df * df / exp((double)lv[d]);
                    slv += lv[d];
                }
                comp[c] = -0.5 * (q + slv + D * l2pi) + log_w[(size_t)s * C + c];
            }
            double m = -INFINITY;
            for (int c = 0; c < C; ++c) if (comp[c] > m) m = comp[c];
            if (isinf(m)) m = 0.0;
            double sum = 0.0;
            for (int c = 0; c < C; ++c) sum += exp(comp[c] - m);
            if (sum < 1e-8) sum = 1e-8;
            out[f * S + s] = log(sum) + m;
        }
    }
    free(comp);
}

/* ----------------------------------------------------------------- HSMM (exact) */
/* torch 2.10 CPU order for torch.sum over a 1-D fp32 slice (the reference's
 * torch.sum(obs_log_probs[t:t+d, s]), hsmm.py:273,285).  ATen's cascade_sum
 * (aten/src/ATen/native/cpu/SumKernel.cpp, accumulating in fp32), restated:
 *   multi_row_sum: `lanes` independent accumulators over `nrow` rows, with 4 cascade levels:
 *     after every 2^lp rows level 0 is added into level 1 and cleared, level j into j+1
 *     while the row count is a multiple of 2^(j*lp) (lp = max(4, ceil_log2(nrow) / 4)),
 *     and at the end acc0 = ((acc0 + acc1) + acc2) + acc3;
 *   strided slice (stride != 1): row_sum = multi_row_sum over rows of 4 (lanes 0..3), the
 *     d mod 4 tail into lane 0, then ((l0 + l1) + l2) + l3;
 *   contiguous slice (stride 1, d >= 8: the 8-wide Vectorized<float> of the kernel torch
 *     dispatches on both AVX2 and AVX512 hosts): row_sum over 8-wide vectors (lanes 0..31 =
 *     4 vectors), tail vectors into vector 0, vectors summed lane-wise, then
 *     r = 0, the d mod 8 tail scalars, then the 8 lanes in order.
 * Checked against torch.sum for d = 1..1024 (and longer) at strides 1, 5, 64, 150
 * (tests/test_oracle.py::test_tsum_matches_torch_sum). */
static int ceil_log2_i64(int64_t x) {
    if (x <= 2) return 1;
    int r = 0;
    for (uint64_t v = (uint64_t)(x - 1); v; v >>= 1) ++r;
    return r;
}
static void multi_row_sum(const float* x, ptrdiff_t stride, int64_t nrow, int lanes, float* out) {
    float acc[4][32];
    memset(acc, 0, sizeof(acc));
    int lp = ceil_log2_i64(nrow) / 4;
    if (lp < 4) lp = 4;
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    int64_t i = 0;
    while (i + step <= nrow) {
        for (int64_t j = 0; j < step; ++j, ++i)
            for (int k = 0; k < lanes; ++k) acc[0][k] += x[(i * lanes + k) * stride];
        for (int j = 1; j < 4; ++j) {
            for (int k = 0; k < lanes; ++k) {
                acc[j][k] += acc[j - 1][k];
                acc[j - 1][k] = 0.f;
            }
            if (i & (mask << (j * lp))) break;
        }
    }
    for (; i < nrow; ++i)
        for (int k = 0; k < lanes; ++k) acc[0][k] += x[(i * lanes + k) * stride];
    for (int j = 1; j < 4; ++j)
        for (int k = 0; k < lanes; ++k) acc[0][k] += acc[j][k];
    for (int k = 0; k < lanes; ++k) out[k] = acc[0][k];
}
float torch_sum_f32(const float* x, ptrdiff_t stride, int64_t n) {
    if (stride != 1 || n < 8) {
        float ps[4];
        const int64_t nr = n / 4;
        multi_row_sum(x, stride, nr, 4, ps);
        for (int64_t i = nr * 4; i < n; ++i) ps[0] += x[i * stride];
        return ((ps[0] + ps[1]) + ps[2]) + ps[3];
    }
    const int64_t nv = n / 8, nr = nv / 4;
    float ps[32];
    multi_row_sum(x, 1, nr, 32, ps);
    for (int64_t v = nr * 4; v < nv; ++v)
        for (int j = 0; j < 8; ++j) ps[j] += x[v * 8 + j];
    for (int k = 1; k < 4; ++k)
        for (int j = 0; j < 8; ++j) ps[j] += ps[k * 8 + j];
    float r = 0.f;
    for (int64_t i = nv * 8; i < n; ++i) r += x[i];
    for (int j = 0; j < 8; ++j) r += ps[j];
    return r;
}
static float tsum(const float* lp, int S, int t0, int d, int s) {
    return torch_sum_f32(lp + (size_t)t0 * S + s, S, d);
}

static void hsmm_backtrack(int T, int S, int Dm, const int16_t* psi_s, const int16_t* psi_d,
                           int fs, int fd, int64_t* states) {
    int t = T - 1, cs = fs, cd = fd;
    while (t >= 0) {
        int start = t - cd + 1;
        if (start < 0) start = 0;
        for (int u = start; u <= t; ++u) states[u] = cs;
        if (start > 0) {
            int di = ((cd - 1) % Dm + Dm) % Dm;            /* python negative index wrap */
            size_t k = ((size_t)t * S + cs) * Dm + di;
            int ns = psi_s[k], nd = psi_d[k];
            t = start - 1; cs = ns; cd = nd;
        } else {
            break;
        }
    }
}

/* Literal hsmm.py:245-354 for one sequence.  lp (T,S); dur (S,Dm); logT (S,S). */
void hsmm_viterbi_literal(const float* lp, const float* dur, const float* logT, int T, int S,
                          int Dm, int64_t* states, float* score) {
    size_t n = (size_t)T * S * Dm;
    float* delta = (float*)malloc(n * sizeof(float));
    int16_t* psi_s = (int16_t*)calloc(n, sizeof(int16_t));
    int16_t* psi_d = (int16_t*)calloc(n, sizeof(int16_t));
    for (size_t k = 0; k < n; ++k) delta[k] = -INFINITY;
#define DL(e, s, d) delta[((size_t)(e) * S + (s)) * Dm + (d)]
    int dl0 = Dm < T ? Dm : T;
    for (int s = 0; s < S; ++s)
        for (int d = 1; d <= dl0; ++d) DL(d - 1, s, d - 1) = tsum(lp, S, 0, d, s) + dur[(size_t)s * Dm + d - 1];
    for (int t = 1; t < T; ++t)
        for (int s = 0; s < S; ++s) {
            int dlim = Dm < T - t ? Dm : T - t;
            for (int d = 1; d <= dlim; ++d) {
                int end = t + d - 1;
                float os = tsum(lp, S, t, d, s), du = dur[(size_t)s * Dm + d - 1];
                float best = -INFINITY;
                int bs = 0, bd = 1;
                for (int ps = 0; ps < S; ++ps) {
                    if (ps == s) continue;
                    for (int pd = 1; pd <= Dm; ++pd) {
                        int pst = t - 1 - pd + 1;
                        if (pst < 0) continue;
                        float prev = DL(t - 1, ps, pd - 1);
                        if (prev == -INFINITY) continue;
                        float tot = ((prev + logT[(size_t)ps * S + s]) + os) + du;
                        if (tot > best) { best = tot; bs = ps; bd = pd; }
                    }
                }
                if (best != -INFINITY) {
                    size_t k = ((size_t)end * S + s) * Dm + d - 1;
                    delta[k] = best; psi_s[k] = (int16_t)bs; psi_d[k] = (int16_t)bd;
                }
            }
        }
    float best = -INFINITY;
    int fs = 0, fd = 1;
    for (int s = 0; s < S; ++s)
        for (int d = 1; d <= Dm; ++d) {
            float sc = DL(T - 1, s, d - 1);
            if (sc > best) { best = sc; fs = s; fd = d; }
        }
#undef DL
    hsmm_backtrack(T, S, Dm, psi_s, psi_d, fs, fd, states);
    *score = best;
    free(delta); free(psi_s); free(psi_d);
}

/* Exact fast form.  M[st][s] = max_{s'!=s,d'} fl(delta[st-1][s'][d'-1] + logT[s'][s]);
 * delta[st+d-1][s][d-1] = fl(fl(M + obs_sum(st,s,d)) + dur[s][d-1]) (st = 0: fl(obs_sum + dur)).
 * g_d(x) = fl(fl(x + o_d) + u_d) is monotone, so the literal max over candidates equals
 * g_d(M); the literal first-argmax is the first candidate (s' asc, d' asc) whose
 * g_d(x) == g_d(M): the first candidate attaining M unless an EARLIER candidate rounds
 * to the same final value, which is checked exactly (rare path). */
void hsmm_viterbi_fast(const float* lp, const float* dur, const float* logT, int T, int S,
                       int Dm, int64_t* states, float* score) {
    size_t n = (size_t)T * S * Dm;
    float* Mst = (float*)malloc(sizeof(float) * (size_t)T * S);
    int16_t* psi_s = (int16_t*)calloc(n, sizeof(int16_t));
    int16_t* psi_d = (int16_t*)calloc(n, sizeof(int16_t));
    float* prevd = (float*)malloc(sizeof(float) * (size_t)S * Dm);   /* delta[st-1][s'][d'-1] */
    float* x = (float*)malloc(sizeof(float) * (size_t)S * Dm);
    float* dmax = (float*)malloc(sizeof(float) * S);
    /* delta value at end e, state s, duration d (start e-d+1) from M */
#define DELTA_AT(e, s, d) ({ int _st = (e) - (d) + 1; float _r;                                  \
        if (_st < 0) _r = -INFINITY;                                                             \
        else { float _o = tsum(lp, S, _st, (d), (s)); float _u = dur[(size_t)(s) * Dm + (d) - 1]; \
               if (_st == 0) _r = _o + _u;                                                       \
               else { float _m = Mst[(size_t)_st * S + (s)];                                     \
                      _r = (_m == -INFINITY) ? -INFINITY : (_m + _o) + _u; } }                   \
        _r; })
    for (int st = 1; st < T; ++st) {
        for (int sp = 0; sp < S; ++sp) {
            float mx = -INFINITY;
            for (int dp = 1; dp <= Dm; ++dp) {
                float v = DELTA_AT(st - 1, sp, dp);
                prevd[(size_t)sp * Dm + dp - 1] = v;
                if (v > mx) mx = v;
            }
            dmax[sp] = mx;
        }
        int dlim = Dm < T - st ? Dm : T - st;
        for (int s = 0; s < S; ++s) {
            float M = -INFINITY;
            for (int sp = 0; sp < S; ++sp) {
                if (sp == s || dmax[sp] == -INFINITY) continue;
                float v = dmax[sp] + logT[(size_t)sp * S + s];
                if (v > M) M = v;
            }
            Mst[(size_t)st * S + s] = M;
            if (M == -INFINITY) continue;               /* literal: delta/psi never written */
            /* candidate values and the first candidate attaining M */
            int p1 = -1;
            float xb = -INFINITY;                       /* max over candidates before p1 */
            for (int sp = 0; sp < S; ++sp)
                for (int dp = 1; dp <= Dm; ++dp) {
                    int k = sp * Dm + dp - 1;
                    float pv = prevd[k];
                    float v = (sp == s || pv == -INFINITY) ? -INFINITY : pv + logT[(size_t)sp * S + s];
                    x[k] = v;
                    if (p1 < 0) {
                        if (v == M) p1 = k;
                        else if (v > xb) xb = v;
                    }
                }
            for (int d = 1; d <= dlim; ++d) {
                float od = tsum(lp, S, st, d, s), ud = dur[(size_t)s * Dm + d - 1];
                float F = (M + od) + ud;
                int win = p1;
                if (xb != -INFINITY && ((xb + od) + ud) == F) {   /* rare: earlier tie */
                    for (int k = 0; k < p1; ++k)
                        if (x[k] != -INFINITY && ((x[k] + od) + ud) == F) { win = k; break; }
                }
                size_t e = (size_t)(st + d - 1);
                psi_s[(e * S + s) * Dm + d - 1] = (int16_t)(win / Dm);
                psi_d[(e * S + s) * Dm + d - 1] = (int16_t)(win % Dm + 1);
            }
        }
    }
    float best = -INFINITY;
    int fs = 0, fd = 1;
    for (int s = 0; s < S; ++s)
        for (int d = 1; d <= Dm; ++d) {
            float sc = DELTA_AT(T - 1, s, d);
            if (sc > best) { best = sc; fs = s; fd = d; }
        }
#undef DELTA_AT
    hsmm_backtrack(T, S, Dm, psi_s, psi_d, fs, fd, states);
    *score = best;
    free(Mst); free(psi_s); free(psi_d); free(prevd); free(x); free(dmax);
}

/* ------------------------------------------------ explicit-duration (semi-Markov) HMM
 * SemiMarkovHMM (semi_markov.py:195-633), segments indexed by END time.
 *   smk_quad_f32            per-frame q[t][s] = sum_k ((x - mu)^2) / var, k ascending
 *                           (semi_markov.py:422-424 per frame; the reference's torch-CPU sum
 *                           order over k is ISA-dependent).
 *   smk_viterbi_literal     semi_markov.py:455-570 as written: init (:495-507), the
 *                           (t, s, d, s', d') loop with strict > (:513-545), the final
 *                           (s, d) search (:548-556) and the backtrack (:558-568).  Segment
 *                           score o = cs[s] - 0.5*Q (gaussian, constant once per segment,
 *                           :416-424) or Q (cs == NULL: additive per-frame scores), with
 *                           Q = q[st] + q[st+1] + ... + q[t] left to right.
 *   smk_forward_f64         the segment forward the reference means at :308-383 (logaddexp
 *                           over the same candidates; it raises TypeError as written), in
 *                           float64 as a tolerance reference.
 */
void smk_quad_f32(const float* x, const float* mu, const float* var, int T, int D, int S, float* q) {
    for (int t = 0; t < T; ++t)
        for (int s = 0; s < S; ++s) {
            float acc = 0.f;
            for (int k = 0; k < D; ++k) {
                float d = x[(size_t)t * D + k] - mu[(size_t)s * D + k];
                acc = acc + (d * d) / var[(size_t)s * D + k];
            }
            q[(size_t)t * S + s] = acc;
        }
}

static float smk_obs(const float* q, const float* cs, int S, int st, int t, int s) {
    float Q = q[(size_t)st * S + s];
    for (int k = st + 1; k <= t; ++k) Q = Q + q[(size_t)k * S + s];
    return cs ? cs[s] - 0.5f * Q : Q;
}

/* seg_s / seg_d receive the segments in time order; returns the segment count. */
int smk_viterbi_literal(const float* q, const float* cs, const float* li, const float* logT,
                        const float* dur, int T, int S, int Dm, int64_t* seg_s, int64_t* seg_d,
                        float* score) {
    size_t n = (size_t)T * S * Dm;
    float* delta = (float*)malloc(sizeof(float) * n);
    int* psi_s = (int*)calloc(n, sizeof(int));
    int* psi_d = (int*)malloc(sizeof(int) * n);
    for (size_t i = 0; i < n; ++i) { delta[i] = -INFINITY; psi_d[i] = 1; }
#define DL(t, s, d) delta[((size_t)(t) * S + (s)) * Dm + (d) - 1]
    for (int s = 0; s < S; ++s)
        for (int d = 1; d <= (Dm < T ? Dm : T); ++d)
            DL(d - 1, s, d) = (li[s] + smk_obs(q, cs, S, 0, d - 1, s)) + dur[(size_t)s * Dm + d - 1];
    for (int t = 0; t < T; ++t)
        for (int s = 0; s < S; ++s)
            for (int d = 1; d <= (Dm < t + 1 ? Dm : t + 1); ++d) {
                if (t - d < 0) continue;
                float best = -INFINITY;
                int bs = 0, bd = 1;
                int pdl = Dm < t - d + 1 ? Dm : t - d + 1;
                for (int sp = 0; sp < S; ++sp) {
                    if (sp == s) continue;
                    for (int dp = 1; dp <= pdl; ++dp) {
                        float tot = DL(t - d, sp, dp) + logT[(size_t)sp * S + s];
                        if (tot > best) { best = tot; bs = sp; bd = dp; }
                    }
                }
                if (best > -INFINITY) {
                    DL(t, s, d) = (best + smk_obs(q, cs, S, t - d + 1, t, s)) + dur[(size_t)s * Dm + d - 1];
                    psi_s[((size_t)t * S + s) * Dm + d - 1] = bs;
                    psi_d[((size_t)t * S + s) * Dm + d - 1] = bd;
                }
            }
    float bf = -INFINITY;
    int fs = 0, fd = 1;
    for (int s = 0; s < S; ++s)
        for (int d = 1; d <= (Dm < T ? Dm : T); ++d)
            if (DL(T - 1, s, d) > bf) { bf = DL(T - 1, s, d); fs = s; fd = d; }
    *score = bf;
    int cnt = 0, ct = T - 1, cs_ = fs, cd = fd;
    int64_t* rs = (int64_t*)malloc(sizeof(int64_t) * T);
    int64_t* rd = (int64_t*)malloc(sizeof(int64_t) * T);
    while (ct >= 0) {
        rs[cnt] = cs_; rd[cnt] = cd; ++cnt;
        if (ct - cd >= 0) {
            size_t i = ((size_t)ct * S + cs_) * Dm + cd - 1;
            int ns = psi_s[i], nd = psi_d[i];
            ct -= cd; cs_ = ns; cd = nd;
        } else break;
    }
    for (int k = 0; k < cnt; ++k) { seg_s[k] = rs[cnt - 1 - k]; seg_d[k] = rd[cnt - 1 - k]; }
#undef DL
    free(rs); free(rd); free(delta); free(psi_s); free(psi_d);
    return cnt;
}

static double lse_acc(double a, double b) {
    if (a == -INFINITY) return b;
    if (b == -INFINITY) return a;
    double m = a > b ? a : b;
    return m + log(exp(a - m) + exp(b - m));
}

/* log_alpha (T,S,Dm) float64; returns log P(o) */
double smk_forward_f64(const float* q, const float* cs, const float* li, const float* logT,
                       const float* dur, int T, int S, int Dm, double* la) {
    size_t n = (size_t)T * S * Dm;
    for (size_t i = 0; i < n; ++i) la[i] = -INFINITY;
#define LA(t, s, d) la[((size_t)(t) * S + (s)) * Dm + (d) - 1]
    for (int t = 0; t < T; ++t)
        for (int s = 0; s < S; ++s)
            for (int d = 1; d <= (Dm < t + 1 ? Dm : t + 1); ++d) {
                int st = t - d + 1;
                double Q = q[(size_t)st * S + s];
                for (int k = st + 1; k <= t; ++k) Q += q[(size_t)k * S + s];
                double o = cs ? (double)cs[s] - 0.5 * Q : Q;
                double u = dur[(size_t)s * Dm + d - 1];
                if (st == 0) { LA(t, s, d) = (double)li[s] + o + u; continue; }
                double acc = -INFINITY;
                int pdl = Dm < st ? Dm : st;
                for (int sp = 0; sp < S; ++sp) {
                    if (sp == s) continue;
                    for (int dp = 1; dp <= pdl; ++dp)
                        acc = lse_acc(acc, LA(st - 1, sp, dp) + (double)logT[(size_t)sp * S + s]);
                }
                if (acc > -INFINITY) LA(t, s, d) = acc + o + u;
            }
    double tot = -INFINITY;
    for (int s = 0; s < S; ++s)
        for (int d = 1; d <= (Dm < T ? Dm : T); ++d) tot = lse_acc(tot, LA(T - 1, s, d));
#undef LA
    return tot;
}

/* ------------------------------------------------------------- streaming decoders
 *   stream_greedy_f32  StreamingHMMProcessor._greedy_decode (streaming.py:267-320):
 *                      s_t = first argmax_j (logT[s_{t-1}][j] + e_t[j]); prev < 0 starts
 *                      from e_0[j] - log_n (:295-298).
 *   stream_beam_f32    _beam_search_decode (streaming.py:322-377) as written: expand every
 *                      hypothesis to every state in (h, j) order, sort by score descending
 *                      keeping insertion order for ties (Python's stable sort), keep K.
 *                      hs/hl hold the hypotheses (in/out, *kc of them); paths are tracked
 *                      as (parent, state) per step, like the kernel's outputs.
 */
void stream_greedy_f32(const float* e, const float* logT, int prev, float log_n, int T, int N,
                       int64_t* states, float* scores) {
    int sp = prev;
    for (int t = 0; t < T; ++t) {
        float best = 0.f;
        int bi = -1;
        for (int j = 0; j < N; ++j) {
            float v = sp < 0 ? e[(size_t)t * N + j] - log_n : logT[(size_t)sp * N + j] + e[(size_t)t * N + j];
            if (bi < 0 || v > best) { best = v; bi = j; }
        }
        states[t] = bi; scores[t] = best; sp = bi;
    }
}

typedef struct { float v; int idx; } smk_cand_t;
static int cand_cmp(const void* a, const void* b) {
    const smk_cand_t* x = (const smk_cand_t*)a;
    const smk_cand_t* y = (const smk_cand_t*)b;
    if (x->v > y->v) return -1;
    if (x->v < y->v) return 1;
    return (x->idx > y->idx) - (x->idx < y->idx);
}

void stream_beam_f32(const float* e, const float* logT, int T, int N, int K, float* hs, int* hl,
                     int* kc_io, int first, int16_t* parent, int16_t* hstate) {
    int kc = *kc_io;
    smk_cand_t* c = (smk_cand_t*)malloc(sizeof(smk_cand_t) * (size_t)(kc > K ? kc : K) * N);
    float* ns = (float*)malloc(sizeof(float) * K);
    int* nl = (int*)malloc(sizeof(int) * K);
    for (int t = 0; t < T; ++t) {
        int n = 0;
        for (int h = 0; h < kc; ++h)
            for (int j = 0; j < N; ++j) {
                float v = first ? hs[h] + e[(size_t)t * N + j]
                                : (hs[h] + logT[(size_t)hl[h] * N + j]) + e[(size_t)t * N + j];
                c[n].v = v; c[n].idx = h * N + j; ++n;
            }
        qsort(c, n, sizeof(smk_cand_t), cand_cmp);
        int kn = n < K ? n : K;
        for (int r = 0; r < kn; ++r) {
            ns[r] = c[r].v; nl[r] = c[r].idx % N;
            parent[(size_t)t * K + r] = (int16_t)(c[r].idx / N);
            hstate[(size_t)t * K + r] = (int16_t)nl[r];
        }
        for (int r = 0; r < kn; ++r) { hs[r] = ns[r]; hl[r] = nl[r]; }
        kc = kn;
        first = 0;
    }
    *kc_io = kc;
    free(c); free(ns); free(nl);
}
