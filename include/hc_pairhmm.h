/*
 * hc_pairhmm.h — C ABI of the MI355X PairHMM engine (libhcpairhmm.so).
 *
 * Drop-in for the PairHMM hot path of avis9ditiu/gatk-haplotypecaller-cpp17
 * (paths below are relative to the reference's src/haplotypecaller/):
 *
 *   hc_phmm_compute_likelihoods  replaces IntelPairHMM::compute_likelihoods
 *                                (pairhmm/intel_pairhmm.hpp:48-56), including the
 *                                normalize/filter step (:24-46)
 *   hc_phmm_cross                replaces computeLikelihoodsNative
 *                                (pairhmm/intel_pairhmm.hpp:115-152): every read x
 *                                every hap, fp32 kernel + fp64 rescue + log10
 *   hc_phmm_pairs_flat           the same per-pair computation over an explicit
 *                                list of independent (read, hap) pairs
 *   hc_phmm_batch_*              the same split into plan (pack + H2D) and execute
 *                                (device only) for device-resident batches
 *   hc_phmm_submit_* / _collect  asynchronous form of the calls above: host
 *                                planning of the next batch overlaps the device
 *                                pass of the previous one (the driver's window
 *                                loop, haplotypecaller.hpp:138-152, keeps
 *                                assembling while the GPU works)
 *   hc_phmm_init_devices         one process, several GPUs: every call is split
 *                                by cells over the configured devices, each with
 *                                its own stream (the in-call parallelism the
 *                                reference has as an OpenMP loop,
 *                                intel_pairhmm.hpp:128-130)
 *   hc_phmm_read / hc_phmm_hap   field-for-field the accelerator hook structs
 *                                shacc_pairhmm::Read / ::Haplotype
 *                                (pairhmm/native/shacc_pairhmm.h:12-24)
 *
 * Value semantics are the reference's: bases are raw bytes (A C T G N, any other
 * byte counts as A, N matches everything); q/i/d/c are raw quality bytes used
 * `& 127` (no -33), exactly as compute_full_prob_avx{s,d} reads them
 * (pairhmm/native/avx-pairhmm-template.h:110-125). Results are bit-identical to
 * the reference kernel: raw fp32 sum, fp64 rescue when raw < 1e-28f, glibc
 * log10f/log10 finish (intel_pairhmm.hpp:131-146).
 *
 * Every pointer is borrowed for the duration of the call (for hc_phmm_submit_*:
 * inputs until submit returns, outputs until hc_phmm_collect returns); nothing
 * else is retained. Calls are thread-safe, except that one hc_phmm_batch or
 * hc_phmm_job handle must not be used by two threads at once (different
 * handles may be used concurrently). All entry points return 0 on success
 * or a negative HC_PHMM_E* code; the message of the calling thread's last
 * error is available from hc_phmm_last_error(). There is no CPU fallback:
 * without a usable MI355X the calls fail with HC_PHMM_ENODEV, and a device
 * pass that could not complete (a kernel reports it in the part's device
 * error word) fails with HC_PHMM_EHIP. The contents of a failed call's
 * output arrays are then unspecified (some pairs may already have been
 * written): a caller must not use them.
 */
#ifndef HC_PAIRHMM_H
#define HC_PAIRHMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HC_PHMM_OK 0
#define HC_PHMM_EINVAL (-1)   /* bad argument (null pointer, length <= 0, too long) */
#define HC_PHMM_ENODEV (-2)   /* no usable gfx950 device / not initialised        */
#define HC_PHMM_EHIP (-3)     /* HIP runtime error                                  */
#define HC_PHMM_ENOMEM (-4)   /* host or device allocation failed                   */

#define HC_PHMM_MAX_HAP_LEN 262144   /* longer haps: anti-diagonal kernel with its stripe ring in HBM */
#define HC_PHMM_MAX_READ_LEN 65536

/* shacc_pairhmm::Read (shacc_pairhmm.h:12-19): same fields, same order. */
typedef struct hc_phmm_read {
    int32_t length;
    const char* bases;
    const char* q;   /* base qualities, raw SAM bytes */
    const char* i;   /* insertion gap-open qualities  */
    const char* d;   /* deletion gap-open qualities   */
    const char* c;   /* gap-continuation qualities    */
} hc_phmm_read;

/* shacc_pairhmm::Haplotype (shacc_pairhmm.h:21-24). */
typedef struct hc_phmm_hap {
    int32_t length;
    const char* bases;
} hc_phmm_hap;

typedef struct hc_phmm_stats {
    int64_t n_pairs;
    int64_t cells;          /* sum over pairs of R*H                      */
    int64_t n_rescued;      /* pairs recomputed in fp64                   */
    double kernel_ms_f32;   /* fp32 kernel(s), HIP events, mean over n_runs  */
    double kernel_ms_f64;   /* fp64 rescue kernel, mean over n_runs          */
    double run_ms;          /* whole device pass, mean over n_runs           */
    int64_t n_launch_waves; /* waves launched by the fp32 pass               */
    int64_t n_runs;         /* runs since the previous stats() call          */
    int64_t n_lane_pairs;   /* pairs on the lane kernels: segmented or one lane per pair (rest: anti-diagonal) */
    int64_t n_seg_waves;    /* column-segmented waves: a pair over nb lanes of BC columns */
    int64_t n_devices;      /* device slots the batch is split over                  */
    double pack_ms;         /* device packing of a new batch (rows + hap tables),
                               done once at create; max over devices               */
    int64_t upload_bytes;   /* host -> device bytes of the batch's inputs            */
} hc_phmm_stats;

/* hc_phmm_init / hc_phmm_init_devices flags. */
#define HC_PHMM_FLAG_F64 1u   /* initNative(use_double = true), intel_pairhmm.hpp:71,81,135:
                                 result_float = 0 for every pair, so every pair is computed
                                 in fp64 only: raw_f32 = 0, rescued = 1, raw_f64 = the fp64
                                 sum, loglik = log10(raw_f64) - log10(2^1020) */
#define HC_PHMM_FLAG_KEEP_MODE 2u /* hc_phmm_init only: select / initialise the device and leave the
                                     process's default mode as it is (callers that pass their mode
                                     per call, e.g. hc::MI355XPairHMM through *_ex) */

/* Select the device (HIP ordinal; -1 = current) and build the device LUTs
 * (intel_pairhmm.hpp:77-113 initNative). flags: 0, HC_PHMM_FLAG_F64 and/or
 * HC_PHMM_FLAG_KEEP_MODE; other bits are HC_PHMM_EINVAL. The mode of the
 * latest successful init (HC_PHMM_FLAG_F64 or not, unless KEEP_MODE) is the
 * default of every later call and batch until the next init or
 * hc_phmm_shutdown (which resets it to 0); each call or batch fixes its mode
 * when it is made (hc_phmm_batch_create, submit), so a later init does not
 * change work already submitted. The *_ex calls take their mode explicitly
 * (the reference's use_double is per IntelPairHMM instance,
 * intel_pairhmm.hpp:58,81). Calling it again is a no-op for the same device
 * or for -1 (apart from the mode); naming a different device than the engine
 * runs on is HC_PHMM_EINVAL (hc_phmm_shutdown first). */
int hc_phmm_init(uint32_t flags, int device);
/* Several device slots in one process: devices[k] is a HIP ordinal (-1 =
 * current); devices == NULL or n == 0 means every visible device. An ordinal
 * may repeat (two streams on one GPU). Every later call splits its pairs by
 * cells over the slots, one stream each; results are identical to one device. */
int hc_phmm_init_devices(uint32_t flags, const int32_t* devices, int32_t n);
int hc_phmm_device_count(void);   /* configured device slots (0: not initialised) */
int hc_phmm_shutdown(void);       /* releases every engine (PairHMM, SW, genotyper) */
const char* hc_phmm_last_error(void);
int hc_phmm_version(void);   /* major*10000 + minor*100 + patch */
/* Which sources this binary was built from (no reference equivalent): a static
 * string "kernel=<16 hex> lib=<16 hex> git=<HEAD>[-dirty]" — the device-kernel
 * source hash, the hash of every library source and build flag
 * (tools/kernel_src_hash.py), and the git HEAD at build time. Callers compare
 * the hashes with their source tree to refuse a stale binary. */
const char* hc_phmm_build_id(void);

/* All reads x all haps. out is n_reads*n_haps doubles, read-major
 * (out[r*n_haps + h]), log10 likelihoods before normalisation.
 * n_reads == 0 or n_haps == 0 is a no-op. */
int hc_phmm_cross(const hc_phmm_read* reads, int32_t n_reads,
                  const hc_phmm_hap* haps, int32_t n_haps, double* out);
/* The same with this call's mode: mode = 0 or HC_PHMM_FLAG_F64 (other bits:
 * HC_PHMM_EINVAL), independent of the process default set by hc_phmm_init. */
int hc_phmm_cross_ex(const hc_phmm_read* reads, int32_t n_reads,
                     const hc_phmm_hap* haps, int32_t n_haps, double* out, uint32_t mode);

/* Many active regions in one device pass (cross-region batching, SURVEY §8(f)
 * row 2): region k is the cross product reads x haps of regions[k], written
 * read-major to regions[k].out exactly as hc_phmm_cross would. All regions'
 * pairs are packed, length-binned and launched together, so a caller that
 * queues regions fills the GPU even though one region (<= 415 reads x <= 128
 * haps in the reference, haplotypecaller.hpp:83-107) does not. */
typedef struct hc_phmm_region {
    const hc_phmm_read* reads;
    int32_t n_reads;
    const hc_phmm_hap* haps;
    int32_t n_haps;
    double* out;   /* n_reads * n_haps, read-major */
} hc_phmm_region;
int hc_phmm_cross_regions(const hc_phmm_region* regions, int32_t n_regions);

/* hc_phmm_cross followed by normalize_likelihoods_and_filter_poorly_modeled_reads
 * (intel_pairhmm.hpp:24-46). out is n_reads*n_haps read-major with the cap
 * applied to every row; keep[r] = 1 for reads that survive the filter, and
 * *n_kept is their count. The caller erases rows/reads with keep[r] == 0. */
int hc_phmm_compute_likelihoods(const hc_phmm_read* reads, int32_t n_reads,
                                const hc_phmm_hap* haps, int32_t n_haps,
                                double* out, uint8_t* keep, int32_t* n_kept);
/* The same with this call's mode (as hc_phmm_cross_ex). */
int hc_phmm_compute_likelihoods_ex(const hc_phmm_read* reads, int32_t n_reads,
                                   const hc_phmm_hap* haps, int32_t n_haps,
                                   double* out, uint8_t* keep, int32_t* n_kept, uint32_t mode);

/* Independent pairs over flat byte pools: pair p uses rs/q/ins/del/gcp rows
 * [read_off[p], read_off[p]+R[p]) and hap bytes [hap_off[p], hap_off[p]+H[p]).
 * Outputs (any may be NULL): loglik[p], raw_f32[p], raw_f64[p] (0 unless
 * rescued), rescued[p]. */
int hc_phmm_pairs_flat(int64_t n, const int64_t* read_off, const int32_t* R,
                       const int64_t* hap_off, const int32_t* H,
                       const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                       const uint8_t* del, const uint8_t* gcp, const uint8_t* hap,
                       double* loglik, float* raw_f32, double* raw_f64, uint8_t* rescued);

/* Plan / execute split for device-resident batches (bench, multi-GPU shards). */
typedef struct hc_phmm_batch hc_phmm_batch;
int hc_phmm_batch_create(int64_t n, const int64_t* read_off, const int32_t* R,
                         const int64_t* hap_off, const int32_t* H,
                         const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap,
                         hc_phmm_batch** out);
/* Enqueue the whole device pass (fp32 kernel, rescue list, fp64 kernel) on
 * `stream` (a hipStream_t; NULL = the library's stream). Asynchronous. */
int hc_phmm_batch_run(hc_phmm_batch* b, void* stream);
/* Wait for the last run, copy results back and apply the log10 finish. */
int hc_phmm_batch_results(hc_phmm_batch* b, double* loglik, float* raw_f32,
                          double* raw_f64, uint8_t* rescued);
/* Counters and device timings averaged over every run since the previous
 * stats() call (the event log is reset by this call). */
int hc_phmm_batch_stats(hc_phmm_batch* b, hc_phmm_stats* st);
/* Device pointers of the per-pair results of the last run (in caller pair order):
 * raw_f32 (float[n]), raw_f64 (double[n]), rescued flags (uint8[n]). */
int hc_phmm_batch_device_results(hc_phmm_batch* b, void** raw_f32, void** raw_f64,
                                 void** rescued);
/* Make later runs write their per-pair results into caller-owned device buffers
 * (e.g. torch tensors, for an RCCL gather without a copy): raw_f32 float[n],
 * raw_f64 double[n], rescued uint8[n], all on the engine's device. NULL keeps
 * the library's own buffer for that output. */
int hc_phmm_batch_bind_outputs(hc_phmm_batch* b, void* raw_f32, void* raw_f64, void* rescued);
int hc_phmm_batch_destroy(hc_phmm_batch* b);

/* Asynchronous calls. submit plans the batch on the host, stages it, enqueues
 * H2D + device pass + D2H on the device stream(s) and returns; the inputs may
 * be released as soon as submit returns. collect waits for the device, applies
 * the log10 finish into the outputs named at submit and frees the job. Jobs may
 * be collected in any order; several may be in flight (each holds its own
 * device and pinned workspace until collected). */
typedef struct hc_phmm_job hc_phmm_job;
int hc_phmm_submit_pairs(int64_t n, const int64_t* read_off, const int32_t* R,
                         const int64_t* hap_off, const int32_t* H,
                         const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap,
                         double* loglik, float* raw_f32, double* raw_f64, uint8_t* rescued,
                         hc_phmm_job** job);
int hc_phmm_submit_regions(const hc_phmm_region* regions, int32_t n_regions, hc_phmm_job** job);
int hc_phmm_job_ready(hc_phmm_job* job);   /* 1: device work done, 0: not yet, < 0: error */
int hc_phmm_collect(hc_phmm_job* job);

/* LUTs the engine uses (for parity tests against the reference's Context<>):
 * ph2pr_f/d[128], mm_f/d[n_mm] with n_mm = 255*256/2 = 32640. */
int hc_phmm_get_luts(float* ph2pr_f, double* ph2pr_d, float* mm_f, double* mm_d);

#ifdef __cplusplus
}
#endif
#endif /* HC_PAIRHMM_H */
