/*
 * PairHMM CPU oracle — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C scalar restatement of the reference PairHMM path
 * (avis9ditiu/gatk-haplotypecaller-cpp17, src/haplotypecaller/pairhmm/).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as a checker / CPU baseline. The product path
 * (libhcpairhmm.so) never links or calls it.
 *
 * Parity is pinned: tests/golden/ fixtures were produced by the reference's
 * own AVX kernel (oracle/_ref, compiled from /root/reference sources by
 * oracle/Makefile) and this restatement must match them bit for bit.
 */
#ifndef HC_PAIRHMM_ORACLE_H
#define HC_PAIRHMM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Build LUTs (idempotent). Mirrors Context<float>/Context<double> ctors,
 * Context.h:142-175 (double) / :182-220 (float) and ContextBase :86-135. */
void hco_init(void);

/* LUT accessors for fixture checks. mm tables hold (254+1)(254+2)/2 entries. */
int  hco_lut_sizes(int* n_ph2pr, int* n_mm, int* n_jac);
void hco_get_luts(float* ph2pr_f, double* ph2pr_d, float* mm_f, double* mm_d,
                  float* jac_f, double* jac_d);

/* One pair, raw scaled probability (Σ_j M[R][j] + Σ_j X[R][j]).
 * Follows compute_full_prob_avx{s,d}, avx-pairhmm-template.h:210-346.
 * rs/hap are raw base bytes; q/i/d/c raw quality bytes (used & 127).
 * Runs with MXCSR FTZ on, as intel_pairhmm.hpp:105 does. */
float  hco_full_prob_f32(int R, int H, const uint8_t* rs, const uint8_t* q,
                         const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                         const uint8_t* hap);
double hco_full_prob_f64(int R, int H, const uint8_t* rs, const uint8_t* q,
                         const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                         const uint8_t* hap);

/* Batch of independent pairs with the fp32 -> fp64 rescue and log10 finish of
 * intel_pairhmm.hpp:131-146. Pair p uses read rows read_off[p] .. +R[p]-1 of the
 * concatenated read arrays and hap bytes hap_off[p] .. +H[p]-1. Any output
 * pointer may be NULL. Returns number of rescued pairs. */
long hco_pairs(long n, const int64_t* read_off, const int32_t* R,
               const int64_t* hap_off, const int32_t* H,
               const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
               const uint8_t* del, const uint8_t* gcp, const uint8_t* hap,
               float* raw_f32, double* raw_f64, uint8_t* rescued, double* loglik,
               int nthreads);

/* log10 finish of one pair (intel_pairhmm.hpp:137-143). */
double hco_finish(float raw_f32, double raw_f64);

/* normalize_likelihoods_and_filter_poorly_modeled_reads, intel_pairhmm.hpp:24-46.
 * L is nReads x nHaps read-major, modified in place (cap applied to every row).
 * keep[r] = 1 when read r survives. Returns the number of kept reads. */
int hco_normalize(int nReads, int nHaps, const int32_t* read_len, double* L, uint8_t* keep);

#ifdef __cplusplus
}
#endif
#endif
