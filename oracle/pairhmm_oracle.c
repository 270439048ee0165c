/*
 * PairHMM CPU oracle — TEST INFRASTRUCTURE ONLY (see pairhmm_oracle.h).
 *
 * Scalar restatement of the reference PairHMM, written from the semantics in
 * SURVEY.md Appendix A. Every function cites the reference file:line it
 * follows (paths relative to src/haplotypecaller/pairhmm/).
 *
 * Build: plain C, -O2 -ffp-contract=off (no FMA: the reference is compiled
 * -O3 -mavx -mavx2 without -mfma, CMakeLists.txt:5, so every mul/add rounds).
 */
#include "pairhmm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <xmmintrin.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAX_QUAL 254                                   /* Context.h:6 */
#define JAC_TOL 8.0                                    /* Context.h:7 */
#define JAC_STEP 0.0001                                /* Context.h:8 */
#define JAC_SIZE 80001   /* (int)(JAC_TOL / JAC_STEP) + 1, Context.h:10 */
#define MM_SIZE (((MAX_QUAL + 1) * (MAX_QUAL + 2)) >> 1)   /* Context.h:23 */

static float  ph2pr_f[128];
static double ph2pr_d[128];
static float  jac_f[JAC_SIZE];
static double jac_d[JAC_SIZE];
static float  mm_f[MM_SIZE];
static double mm_d[MM_SIZE];
static float  init_f, log10_init_f;
static double init_d, log10_init_d;
static int    ready;

/* ContextBase::approximateLog10SumLog10 in NUMBER precision, Context.h:112-135.
 * The reference's `std::isinf(x) == -1` test compares a C++ bool with -1 and is
 * therefore never true; it is omitted (inputs here are always finite). */
static float approx_sum_f(float small, float big)
{
    if (small > big) { float t = big; big = small; small = t; }
    float diff = big - small;
    if (diff >= (float)JAC_TOL) return big;
    float v = diff * (float)(1.0 / JAC_STEP);
    int ind = (v > 0.0f) ? (int)(v + 0.5f) : (int)(v - 0.5f);   /* fastRound, :108-110 */
    return big + jac_f[ind];
}

static double approx_sum_d(double small, double big)
{
    if (small > big) { double t = big; big = small; small = t; }
    double diff = big - small;
    if (diff >= JAC_TOL) return big;
    double v = diff * (1.0 / JAC_STEP);
    int ind = (v > 0.0) ? (int)(v + 0.5) : (int)(v - 0.5);
    return big + jac_d[ind];
}

void hco_init(void)
{
    if (ready) return;
    /* initializeJacobianLogTable, Context.h:87-92 */
    for (int k = 0; k < JAC_SIZE; ++k) {
        double v = log10(1.0 + pow(10.0, -((double)k) * JAC_STEP));
        jac_f[k] = (float)v;
        jac_d[k] = v;
    }
    /* initializeMatchToMatchProb, Context.h:95-106: the log-sum runs in NUMBER
     * precision, the rest in double, the result is rounded to NUMBER. */
    const double inv_ln10 = 1.0 / log(10);
    for (int i = 0, off = 0; i <= MAX_QUAL; off += ++i) {
        for (int j = 0; j <= i; ++j) {
            double sf = (double)approx_sum_f((float)(-0.1 * i), (float)(-0.1 * j));
            double sd = approx_sum_d(-0.1 * i, -0.1 * j);
            double lf = log1p(-fmin(1.0, pow(10, sf))) * inv_ln10;
            double ld = log1p(-fmin(1.0, pow(10, sd))) * inv_ln10;
            mm_f[off + j] = (float)pow(10, lf);
            mm_d[off + j] = pow(10, ld);
        }
    }
    /* Context<double>/<float> ctors, Context.h:150-156 / :190-196 */
    for (int x = 0; x < 128; ++x) {
        ph2pr_d[x] = pow(10.0, -((double)x) / 10.0);
        ph2pr_f[x] = powf(10.f, -((float)x) / 10.f);
    }
    init_d = ldexp(1.0, 1020);
    log10_init_d = log10(init_d);
    init_f = ldexpf(1.f, 120);
    log10_init_f = log10f(init_f);
    ready = 1;
}

int hco_lut_sizes(int* n_ph2pr, int* n_mm, int* n_jac)
{
    if (n_ph2pr) *n_ph2pr = 128;
    if (n_mm) *n_mm = MM_SIZE;
    if (n_jac) *n_jac = JAC_SIZE;
    return 0;
}

void hco_get_luts(float* pf, double* pd, float* mf, double* md, float* jf, double* jd)
{
    hco_init();
    if (pf) memcpy(pf, ph2pr_f, sizeof ph2pr_f);
    if (pd) memcpy(pd, ph2pr_d, sizeof ph2pr_d);
    if (mf) memcpy(mf, mm_f, sizeof mm_f);
    if (md) memcpy(md, mm_d, sizeof mm_d);
    if (jf) memcpy(jf, jac_f, sizeof jac_f);
    if (jd) memcpy(jd, jac_d, sizeof jac_d);
}

/* ConvertChar, pairhmm_common.h:26-44: A0 C1 T2 G3 N4, every other byte -> 0.
 * (Byte 255 indexes one past the reference's 255-entry table; defined as 0.) */
static inline int conv(uint8_t b)
{
    switch (b) {
    case 'C': return 1;
    case 'T': return 2;
    case 'G': return 3;
    case 'N': return 4;
    default:  return 0;
    }
}

/* set_mm_prob, Context.h:168-179 / :208-219 (quals are < 128 <= MAX_QUAL). */
static inline int mm_index(int a, int b)
{
    int lo = a < b ? a : b, hi = a < b ? b : a;
    return ((hi * (hi + 1)) >> 1) + lo;
}

/* Scalar forward recurrence; order of every operation as computeMXY
 * (avx-pairhmm-template.h:183-198); row constants as initializeVectors (:83-128)
 * and stripeINITIALIZATION (:136-177); final sums as :308-343. */
#define DEFINE_FULL_PROB(NAME, T, PH2PR, MMT, INITC)                                   \
static T NAME##_impl(int R, int H, const uint8_t* rs, const uint8_t* q,               \
                     const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,      \
                     const uint8_t* hap, T* buf)                                       \
{                                                                                      \
    T *Mp = buf, *Xp = buf + (H + 1), *Yp = buf + 2 * (H + 1);                         \
    T *Mc = buf + 3 * (H + 1), *Xc = buf + 4 * (H + 1), *Yc = buf + 5 * (H + 1);       \
    const T init_Y = INITC / (T)H;                                                     \
    for (int j = 0; j <= H; ++j) { Mp[j] = 0; Xp[j] = 0; Yp[j] = init_Y; }             \
    for (int i = 1; i <= R; ++i) {                                                     \
        const int I = ins[i - 1] & 127, D = del[i - 1] & 127;                          \
        const int C = gcp[i - 1] & 127, Q = q[i - 1] & 127;                            \
        const T mm = MMT[mm_index(I, D)];                                              \
        const T gapm = (T)1 - PH2PR[C];                                                \
        const T mx = PH2PR[I], xx = PH2PR[C], my = PH2PR[D], yy = PH2PR[C];            \
        const T distm = PH2PR[Q];                                                      \
        const T pm = (T)1 - distm, px = distm / (T)3;                                  \
        const int rc = conv(rs[i - 1]);                                                \
        Mc[0] = 0; Xc[0] = 0; Yc[0] = 0;                                               \
        for (int j = 1; j <= H; ++j) {                                                 \
            const int hc = conv(hap[j - 1]);                                           \
            const T prior = (rc == hc || rc == 4 || hc == 4) ? pm : px;                \
            Mc[j] = ((Mp[j - 1] * mm + Xp[j - 1] * gapm) + Yp[j - 1] * gapm) * prior;  \
            Xc[j] = Mp[j] * mx + Xp[j] * xx;                                           \
            Yc[j] = Mc[j - 1] * my + Yc[j - 1] * yy;                                   \
        }                                                                              \
        T* t;                                                                          \
        t = Mp; Mp = Mc; Mc = t;                                                       \
        t = Xp; Xp = Xc; Xc = t;                                                       \
        t = Yp; Yp = Yc; Yc = t;                                                       \
    }                                                                                  \
    T sumM = 0, sumX = 0;                                                              \
    for (int j = 1; j <= H; ++j) sumM = sumM + Mp[j];                                  \
    for (int j = 1; j <= H; ++j) sumX = sumX + Xp[j];                                  \
    return sumM + sumX;                                                                \
}

DEFINE_FULL_PROB(full_f32, float, ph2pr_f, mm_f, init_f)
DEFINE_FULL_PROB(full_f64, double, ph2pr_d, mm_d, init_d)

/* MXCSR FTZ on for the duration of the computation (intel_pairhmm.hpp:101-105). */
static unsigned ftz_on(void)
{
    unsigned old = _mm_getcsr();
    _mm_setcsr(old | 0x8000);
    return old;
}

float hco_full_prob_f32(int R, int H, const uint8_t* rs, const uint8_t* q,
                        const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                        const uint8_t* hap)
{
    hco_init();
    if (R <= 0 || H <= 0) return 0.0f;
    float* buf = (float*)malloc(sizeof(float) * 6 * (size_t)(H + 1));
    unsigned old = ftz_on();
    float r = full_f32_impl(R, H, rs, q, ins, del, gcp, hap, buf);
    _mm_setcsr(old);
    free(buf);
    return r;
}

double hco_full_prob_f64(int R, int H, const uint8_t* rs, const uint8_t* q,
                         const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                         const uint8_t* hap)
{
    hco_init();
    if (R <= 0 || H <= 0) return 0.0;
    double* buf = (double*)malloc(sizeof(double) * 6 * (size_t)(H + 1));
    unsigned old = ftz_on();
    double r = full_f64_impl(R, H, rs, q, ins, del, gcp, hap, buf);
    _mm_setcsr(old);
    free(buf);
    return r;
}

/* intel_pairhmm.hpp:137-143 (MIN_ACCEPTED = 1e-28f, pairhmm_common.h:16). */
double hco_finish(float f, double d)
{
    hco_init();
    if (f < 1e-28f) return log10(d) - log10_init_d;
    return (double)(log10f(f) - log10_init_f);
}

long hco_pairs(long n, const int64_t* read_off, const int32_t* R,
               const int64_t* hap_off, const int32_t* H,
               const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
               const uint8_t* del, const uint8_t* gcp, const uint8_t* hap,
               float* raw_f32, double* raw_f64, uint8_t* rescued, double* loglik,
               int nthreads)
{
    hco_init();
    int maxH = 1;
    for (long p = 0; p < n; ++p) if (H[p] > maxH) maxH = H[p];
    long nres = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+ : nres)
#endif
    {
        unsigned old = ftz_on();
        double* bd = (double*)malloc(sizeof(double) * 6 * (size_t)(maxH + 1));
        float* bf = (float*)malloc(sizeof(float) * 6 * (size_t)(maxH + 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (long p = 0; p < n; ++p) {
            const int64_t ro = read_off[p], ho = hap_off[p];
            float f = 0.0f;
            double d = 0.0;
            int resc = 0;
            if (R[p] > 0 && H[p] > 0) {
                f = full_f32_impl(R[p], H[p], rs + ro, q + ro, ins + ro, del + ro, gcp + ro, hap + ho, bf);
                if (f < 1e-28f) {
                    d = full_f64_impl(R[p], H[p], rs + ro, q + ro, ins + ro, del + ro, gcp + ro, hap + ho, bd);
                    resc = 1;
                }
            }
            nres += resc;
            if (raw_f32) raw_f32[p] = f;
            if (raw_f64) raw_f64[p] = d;
            if (rescued) rescued[p] = (uint8_t)resc;
            if (loglik) loglik[p] = resc ? (log10(d) - log10_init_d)
                                         : (double)(log10f(f) - log10_init_f);
        }
        free(bd);
        free(bf);
        _mm_setcsr(old);
    }
    (void)nthreads;
    return nres;
}

/* IntelPairHMM::normalize_likelihoods_and_filter_poorly_modeled_reads,
 * intel_pairhmm.hpp:24-46 (constants :19-23). */
int hco_normalize(int nReads, int nHaps, const int32_t* read_len, double* L, uint8_t* keep)
{
    int kept = 0;
    for (int r = 0; r < nReads; ++r) {
        double* row = L + (size_t)r * nHaps;
        double best = row[0];
        for (int h = 1; h < nHaps; ++h) if (best < row[h]) best = row[h];
        double cap = best + -4.5;
        for (int h = 0; h < nHaps; ++h) if (row[h] < cap) row[h] = cap;
        double thr = fmin(2.0, ceil((double)read_len[r] * 0.02)) * -4.0;
        keep[r] = !(best < thr);
        kept += keep[r];
    }
    return kept;
}
