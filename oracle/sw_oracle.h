/*
 * Smith-Waterman CPU oracle — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C scalar restatement of the reference's haplotype-to-reference
 * aligner (avis9ditiu/gatk-haplotypecaller-cpp17, src/haplotypecaller/
 * smithwaterman/): smithWatermanBackTrack (native/PairWiseSW.h:41-238),
 * getCIGAR (:240-415) and runSWOnePairBT (:418-447), plus the all-match
 * shortcut of IntelSWAligner::align (intel_smithwaterman.hpp:29-58).
 * Only tests/ and bench.py load it; libhcpairhmm.so never links or calls it.
 *
 * Parity is pinned: tests/golden/sw_golden.npz holds the reference aligner's
 * own outputs (oracle/_ref/libref_sw.so, compiled from /root/reference by
 * oracle/Makefile) and this restatement must reproduce every offset and CIGAR.
 */
#ifndef HC_SW_ORACLE_H
#define HC_SW_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* runSWOnePairBT: align seq2 (alt, columns) against seq1 (ref, rows) with the
 * given scores and overhang strategy (9 SOFTCLIP, 10 INDEL, 11 LEADING_INDEL,
 * 12 IGNORE; smithwaterman_common.h:26-29). Writes the NUL-terminated CIGAR to
 * cigar[cap] and the best end-point score to *score (may be NULL). Returns
 * the alignment offset, or INT32_MIN if the CIGAR does not fit in cap. */
int hco_sw_align(int match, int mismatch, int open, int extend,
                 const uint8_t* seq1, int len1, const uint8_t* seq2, int len2,
                 int overhang, char* cigar, int cap, int* score);

/* IntelSWAligner::is_all_match (intel_smithwaterman.hpp:47-58): equal lengths
 * and at most MINIMAL_MISMATCH_TO_TOLERANCE (2) differing bytes. */
int hco_sw_is_all_match(const uint8_t* ref, int ref_len, const uint8_t* alt, int alt_len);

/* Many pairs (flat pools), OpenMP: IntelSWAligner::align semantics when
 * shortcut != 0 (all-match pairs -> offset 0, "<len>M"), runSWOnePairBT on
 * every pair otherwise. CIGAR k at cigars + k*stride. Returns 0, or -1 when a
 * CIGAR does not fit. */
int hco_sw_batch(long n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                 const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts,
                 int match, int mismatch, int open, int extend, int overhang, int shortcut,
                 int32_t* offsets, char* cigars, int stride, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
