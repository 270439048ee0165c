/*
 * hc_sw.h — C ABI of the MI355X Smith-Waterman aligner (in libhcpairhmm.so).
 *
 * Drop-in for the haplotype-to-reference aligner of
 * avis9ditiu/gatk-haplotypecaller-cpp17 (paths relative to src/haplotypecaller/):
 *
 *   hc_sw_align_flat     replaces IntelSWAligner::align
 *                        (smithwaterman/intel_smithwaterman.hpp:29-44) over a
 *                        list of (ref, alt) pairs — the loop of
 *                        assembler/graph_wrapper.hpp:232-240 in one device pass:
 *                        all-match shortcut (:36-37,47-58) when `shortcut` != 0,
 *                        then runSWOnePairBT_avx2 (native/PairWiseSW.h:418-447)
 *   hc_sw_batch_*        the same split into plan (H2D) and execute (device only)
 *
 * seq1 is the reference window (rows), seq2 the haplotype (columns), exactly as
 * runSWOnePairBT_avx2(match, mismatch, open, extend, seq1, seq2, len1, len2,
 * overhangStrategy, ...) takes them. Bases are compared as raw bytes. Results
 * are identical to the reference: the alignment offset and the CIGAR string
 * ("%d%c" runs of M I D S, PairWiseSW.h:388-413), including its end-point
 * tie-breaks (:201-226) and traceback order (:254-366).
 *
 * Lengths: 1 <= len1 <= HC_SW_MAX_LEN1 and 1 <= len2 <= HC_SW_MAX_LEN2 — the
 * reference's own limits (MAX_SEQ_LEN = 1024, native/smithwaterman_common.h:47;
 * a 1024-base seq1 writes E[-1] there). The reference throws on empty input
 * (intel_smithwaterman.hpp:33-34); here that is HC_SW_EINVAL.
 *
 * Pointers are borrowed for the duration of a call. Calls are synchronous and
 * serialised. Status codes are the HC_PHMM_* codes of hc_pairhmm.h; the message
 * of the calling thread's last error is hc_phmm_last_error(). No CPU fallback:
 * without a gfx950 device every call fails with HC_SW_ENODEV.
 */
#ifndef HC_SW_H
#define HC_SW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HC_SW_OK 0
#define HC_SW_EINVAL (-1)
#define HC_SW_ENODEV (-2)
#define HC_SW_EHIP (-3)
#define HC_SW_ENOMEM (-4)
#define HC_SW_ERANGE (-5)   /* a CIGAR does not fit in the caller's stride */

#define HC_SW_MAX_LEN1 1023
#define HC_SW_MAX_LEN2 1024

/* Overhang strategies (native/smithwaterman_common.h:26-29). */
#define HC_SW_SOFTCLIP 9
#define HC_SW_INDEL 10
#define HC_SW_LEADING_INDEL 11
#define HC_SW_IGNORE 12

/* IntelSWAligner::SWParameters (intel_smithwaterman.hpp:12-24). */
typedef struct hc_sw_params {
    int32_t match, mismatch, open, extend;
} hc_sw_params;

typedef struct hc_sw_stats {
    int64_t n_pairs;
    int64_t n_shortcut;   /* pairs answered by the all-match shortcut  */
    int64_t cells;        /* sum of len1*len2 over the DP pairs        */
    double dp_ms;         /* DP kernel, HIP events, mean over n_runs   */
    double trace_ms;      /* traceback kernel, mean over n_runs        */
    double run_ms;        /* whole device pass, mean over n_runs       */
    int64_t n_runs;
} hc_sw_stats;

typedef struct hc_sw_batch hc_sw_batch;

/* Select the device (-1: current) — shared with hc_phmm_init. */
int hc_sw_init(int device);

/* IntelSWAligner::align over n pairs. Pair k aligns seq2 = alts[alt_off[k] ..
 * +alt_len[k]) against seq1 = refs[ref_off[k] .. +ref_len[k]). Writes
 * offsets[k] and the NUL-terminated CIGAR of pair k at cigars + k*stride.
 * overhang is one of HC_SW_SOFTCLIP..HC_SW_IGNORE (IntelSWAligner::align uses
 * SOFTCLIP); shortcut != 0 applies the all-match shortcut first. */
int hc_sw_align_flat(int64_t n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                     const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts,
                     hc_sw_params params, int32_t overhang, int32_t shortcut,
                     int32_t* offsets, char* cigars, int32_t stride);

/* Plan / execute split (device-resident batches, bench). */
int hc_sw_batch_create(int64_t n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                       const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts,
                       hc_sw_params params, int32_t overhang, int32_t shortcut, hc_sw_batch** out);
int hc_sw_batch_run(hc_sw_batch* b, void* stream /* hipStream_t, NULL = library stream */);
int hc_sw_batch_results(hc_sw_batch* b, int32_t* offsets, char* cigars, int32_t stride,
                        int32_t* scores /* optional: best end-point score, 0 for shortcut pairs */);
int hc_sw_batch_stats(hc_sw_batch* b, hc_sw_stats* st);
int hc_sw_batch_destroy(hc_sw_batch* b);

#ifdef __cplusplus
}
#endif
#endif /* HC_SW_H */
