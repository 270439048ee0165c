/*
 * hc_gt.h — C ABI of the MI355X genotyper numeric core (in libhcpairhmm.so).
 *
 * Drop-in for the per-site likelihood arithmetic of
 * avis9ditiu/gatk-haplotypecaller-cpp17's Genetyper::assign_genotype_likelihoods
 * (src/haplotypecaller/genotyper/genotyper.hpp:369-399), for many sites at once:
 *
 *   marginalize / marginal_likelihoods            :245-274  allele likelihood of a read =
 *                                                            max over the haplotypes of the allele
 *   calculate_genotype_likelihoods                :276-328  per genotype (a1 <= a2), sum over reads
 *                                                            of log10(2)+L[a] or
 *                                                            MathUtils::approximate_log10_sum_log10
 *                                                            (utils/math_utils.hpp:11-33), minus
 *                                                            n_reads * log10(2)
 *   get_genotype_quality_and_max_genotype_index   :330-365  best genotype and its quality (<= 99)
 *
 * The caller keeps the event bookkeeping (set_events_for_haplotypes,
 * get_compatible_alleles, get_allele_mapper, get_read_indices_to_keep) and
 * passes, per site, the region's read-major likelihood matrix (the return value
 * of compute_likelihoods), the kept read indices, the haplotype -> allele map
 * (haplotype_mapper) and the allele count. Sites that share a matrix (one
 * region) share its upload. Results are bit-identical to the reference
 * arithmetic (sequential sums in read order, the Jacobian table as g++ folds it).
 *
 * Status codes are the HC_PHMM_* codes of hc_pairhmm.h; message via
 * hc_phmm_last_error(). No CPU fallback: without a gfx950 device the call fails.
 */
#ifndef HC_GT_H
#define HC_GT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HC_GT_MAX_ALLELES 7   /* Genetyper::MAX_ALLELE_COUNT (genotyper.hpp:19) */
#define HC_GT_MAX_GENOTYPES 28

typedef struct hc_gt_site {
    const double* L;              /* n_reads x n_haps, read-major (row r at L + r*n_haps) */
    int32_t n_reads;
    int32_t n_haps;
    const int32_t* keep;          /* n_keep read indices (< n_reads), in the reference's order */
    int32_t n_keep;
    const int32_t* hap_allele;    /* n_haps allele indices (< n_alleles) */
    int32_t n_alleles;            /* 2 .. HC_GT_MAX_ALLELES */
    double* genotype_likelihoods; /* out: n_alleles*(n_alleles+1)/2, genotype order a1 <= a2, a1-major */
    int32_t* genotype_index;      /* out: argmax (ties: the later index, :344-349) */
    int32_t* genotype_quality;    /* out: round(-10*(second - best)), capped at 99 */
} hc_gt_site;

int hc_gt_genotype_sites(const hc_gt_site* sites, int32_t n_sites);

#ifdef __cplusplus
}
#endif
#endif /* HC_GT_H */
