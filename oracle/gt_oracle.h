/*
 * Genotyper numeric-core CPU oracle — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the per-site likelihood arithmetic of
 * avis9ditiu/gatk-haplotypecaller-cpp17 (src/haplotypecaller/):
 *   Genetyper::marginal_likelihoods              genotyper/genotyper.hpp:245-264
 *   Genetyper::calculate_read_likelihoods_by_genotype_index / get_genotype_likelihoods
 *                                                genotyper/genotyper.hpp:276-328
 *   Genetyper::get_genotype_quality_and_max_genotype_index  :330-365
 *   MathUtils::approximate_log10_sum_log10       utils/math_utils.hpp:11-33
 * Only tests/ and bench.py load it; the product library never links it.
 *
 * Pinning: approximate_log10_sum_log10 and its Jacobian table are checked
 * against the reference's own math_utils.hpp compiled in place
 * (oracle/_ref/libref_math.so, tests/golden/gt_golden.npz). genotyper.hpp
 * itself includes sam.hpp (Boost) and cannot be compiled here, so the loops
 * above are a restatement (their fixtures are regression pins, not reference
 * outputs).
 */
#ifndef HC_GT_ORACLE_H
#define HC_GT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

double hco_approx_log10_sum_log10(double a, double b);

/* One site: L read-major (rows of n_haps), the kept reads, the haplotype ->
 * allele map (haplotype_mapper) and the allele count (2..7). Writes the
 * n_alleles*(n_alleles+1)/2 genotype log10 likelihoods, the index of the best
 * genotype and its quality (capped at 99). */
void hco_gt_site(const double* L, int n_haps, const int32_t* keep, int n_keep, const int32_t* hap_allele,
                 int n_alleles, double* gl, int32_t* gt_index, int32_t* gq);
/* The same with the approximate_log10_sum_log10 implementation passed in (e.g.
 * the reference's own, compiled in oracle/_ref/libref_math.so). */
void hco_gt_site_with(const double* L, int n_haps, const int32_t* keep, int n_keep, const int32_t* hap_allele,
                      int n_alleles, double* gl, int32_t* gt_index, int32_t* gq, double (*approx)(double, double));

#ifdef __cplusplus
}
#endif
#endif
