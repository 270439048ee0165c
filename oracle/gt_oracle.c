/*
 * Genotyper numeric-core CPU oracle — TEST INFRASTRUCTURE ONLY (see gt_oracle.h).
 * Paths are relative to the reference's src/haplotypecaller/.
 */
#include "gt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>

#define MAX_TOLERANCE 8.0          /* JacobianLogTable::MAX_TOLERANCE, utils/math_utils.hpp:19 */
#define TABLE_STEP 0.0001          /* :24 */
#define TABLE_LEN 80001            /* MAX_TOLERANCE / TABLE_STEP + 1, :28 */

/* cache[k] = log10(1 + 10^(-TABLE_STEP * k)), utils/math_utils.hpp:27-31. g++
 * evaluates that initializer at compile time with correctly rounded pow/log10
 * (glibc's run-time results differ by 1 ulp on some entries), so the table is
 * generated the same way by tools/gen_jacobian.py (oracle/Makefile). */
#include "_gen/math_jacobian.inc"
static double g_jac[TABLE_LEN];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void jac_init(void)
{
    for (int k = 0; k < TABLE_LEN; ++k) {
        union { unsigned long long u; double d; } v;
        v.u = kMathJacobianBits[k];
        g_jac[k] = v.d;
    }
}

/* MathUtils::approximate_log10_sum_log10, utils/math_utils.hpp:11-16 */
double hco_approx_log10_sum_log10(double a, double b)
{
    pthread_once(&g_once, jac_init);
    if (a > b) {
        const double t = a;
        a = b;
        b = t;
    }
    const double diff = b - a;
    /* JacobianLogTable::get: cache[std::round(difference * INV_STEP)], :21-22 */
    return b + (diff < MAX_TOLERANCE ? g_jac[(size_t)round(diff * (1.0 / TABLE_STEP))] : 0.0);
}

void hco_gt_site(const double* L, int n_haps, const int32_t* keep, int n_keep, const int32_t* hap_allele,
                 int n_alleles, double* gl, int32_t* gt_index, int32_t* gq)
{
    hco_gt_site_with(L, n_haps, keep, n_keep, hap_allele, n_alleles, gl, gt_index, gq, hco_approx_log10_sum_log10);
}

void hco_gt_site_with(const double* L, int n_haps, const int32_t* keep, int n_keep, const int32_t* hap_allele,
                      int n_alleles, double* gl, int32_t* gt_index, int32_t* gq, double (*approx)(double, double))
{
    const double log10_2 = log10(2.0);   /* std::log10(2), genotyper.hpp:280,321 */
    double* al = (double*)malloc(sizeof(double) * (size_t)(n_keep > 0 ? n_keep : 1) * (size_t)n_alleles);
    /* marginal_likelihoods (:245-264): max over the haplotypes of each allele,
     * from std::numeric_limits<double>::lowest(), strict > in haplotype order */
    for (int r = 0; r < n_keep; ++r) {
        for (int a = 0; a < n_alleles; ++a) al[(size_t)r * n_alleles + a] = -DBL_MAX;
        const double* row = L + (size_t)keep[r] * (size_t)n_haps;
        for (int h = 0; h < n_haps; ++h) {
            double* slot = &al[(size_t)r * n_alleles + hap_allele[h]];
            if (row[h] > *slot) *slot = row[h];
        }
    }
    /* calculate_read_likelihoods_by_genotype_index (:294-311) + get_genotype_likelihoods (:313-322):
     * genotypes (a1 <= a2) in a1-major order; per read a1 == a2 ? al + log10(2) :
     * approximate_log10_sum_log10(al[a1], al[a2]); std::accumulate from 0.0, minus n_keep * log10(2) */
    int g = 0;
    for (int a1 = 0; a1 < n_alleles; ++a1) {
        for (int a2 = a1; a2 < n_alleles; ++a2, ++g) {
            double acc = 0.0;
            for (int r = 0; r < n_keep; ++r) {
                const double* x = &al[(size_t)r * n_alleles];
                acc += a1 == a2 ? x[a1] + log10_2 : approx(x[a1], x[a2]);
            }
            gl[g] = acc - (double)n_keep * log10_2;
        }
    }
    free(al);
    /* get_genotype_quality_and_max_genotype_index (:324-355) */
    double mx, second;
    int idx;
    if (gl[0] > gl[1]) {
        second = gl[1];
        mx = gl[0];
        idx = 0;
    } else {
        second = gl[0];
        mx = gl[1];
        idx = 1;
    }
    for (int i = 2; i < g; ++i) {
        if (gl[i] >= mx) {
            second = mx;
            mx = gl[i];
            idx = i;
        } else if (gl[i] > second) {
            second = gl[i];
        }
    }
    /* static_cast<std::size_t>(std::round(...)), capped at MAX_GENOTYPE_QUALITY (99).
     * The cast is undefined for NaN (all genotypes -inf) and for values >= 2^64
     * (second = -inf); this follows what g++'s x86-64 conversion sequence yields
     * there: NaN -> 2^63 (capped to 99), >= 2^64 -> 0. */
    const double q = round(-10.0 * (second - mx));
    *gt_index = idx;
    *gq = isnan(q) ? 99 : q >= 18446744073709551616.0 ? 0 : q > 99.0 ? 99 : (int32_t)q;
}
