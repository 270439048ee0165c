// Driver around the REFERENCE PairHMM kernel — TEST INFRASTRUCTURE ONLY.
//
// Compiled by oracle/Makefile directly against the reference headers where
// they lie (/root/reference/src/haplotypecaller/pairhmm/native/avx-pairhmm.h);
// no reference source is copied into this repository. The output goes to
// oracle/_ref/ (git-ignored) and is used to (1) generate the golden fixtures in
// tests/golden/ and (2) time the reference CPU kernel as bench.py's
// cpu_baseline ("kind": "reference").
//
// The flags in the Makefile are the reference's own (-O3 -mavx -mavx2,
// CMakeLists.txt:5) plus -fopenmp for the multi-core baseline. The driver
// restates only the 10-line rescue/log10 loop of intel_pairhmm.hpp:131-146,
// because intel_pairhmm.hpp itself pulls Boost headers that are absent here.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <xmmintrin.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "avx-pairhmm.h"

namespace {
Context<float>& ctxf() { static Context<float> c; return c; }
Context<double>& ctxd() { static Context<double> c; return c; }

void ensure_init()
{
    static bool done = false;
    if (done) return;
    ctxf();
    ctxd();
    ConvertChar::init();
    done = true;
}

testcase make_tc(int R, int H, const uint8_t* rs, const uint8_t* q, const uint8_t* i,
                 const uint8_t* d, const uint8_t* c, const uint8_t* hap)
{
    testcase tc;
    tc.rslen = R;
    tc.haplen = H;
    tc.q = reinterpret_cast<const char*>(q);
    tc.i = reinterpret_cast<const char*>(i);
    tc.d = reinterpret_cast<const char*>(d);
    tc.c = reinterpret_cast<const char*>(c);
    tc.hap = reinterpret_cast<const char*>(hap);
    tc.rs = reinterpret_cast<const char*>(rs);
    return tc;
}
} // namespace

extern "C" {

int ref_lut_sizes(int* n_ph2pr, int* n_mm, int* n_jac)
{
    *n_ph2pr = 128;
    *n_mm = ((MAX_QUAL + 1) * (MAX_QUAL + 2)) >> 1;
    *n_jac = JACOBIAN_LOG_TABLE_SIZE;
    return 0;
}

void ref_get_luts(float* pf, double* pd, float* mf, double* md, float* jf, double* jd)
{
    ensure_init();
    int np, nm, nj;
    ref_lut_sizes(&np, &nm, &nj);
    std::memcpy(pf, ContextBase<float>::ph2pr, sizeof(float) * np);
    std::memcpy(pd, ContextBase<double>::ph2pr, sizeof(double) * np);
    std::memcpy(mf, ContextBase<float>::matchToMatchProb, sizeof(float) * nm);
    std::memcpy(md, ContextBase<double>::matchToMatchProb, sizeof(double) * nm);
    std::memcpy(jf, ContextBase<float>::jacobianLogTable, sizeof(float) * nj);
    std::memcpy(jd, ContextBase<double>::jacobianLogTable, sizeof(double) * nj);
}

float ref_full_prob_f32(int R, int H, const uint8_t* rs, const uint8_t* q, const uint8_t* i,
                        const uint8_t* d, const uint8_t* c, const uint8_t* hap)
{
    ensure_init();
    testcase tc = make_tc(R, H, rs, q, i, d, c, hap);
    unsigned old = _mm_getcsr();
    _MM_SET_FLUSH_ZERO_MODE(_MM_FLUSH_ZERO_ON);
    float r = compute_full_prob_avxs<float>(&tc);
    _mm_setcsr(old);
    return r;
}

double ref_full_prob_f64(int R, int H, const uint8_t* rs, const uint8_t* q, const uint8_t* i,
                         const uint8_t* d, const uint8_t* c, const uint8_t* hap)
{
    ensure_init();
    testcase tc = make_tc(R, H, rs, q, i, d, c, hap);
    unsigned old = _mm_getcsr();
    _MM_SET_FLUSH_ZERO_MODE(_MM_FLUSH_ZERO_ON);
    double r = compute_full_prob_avxd<double>(&tc);
    _mm_setcsr(old);
    return r;
}

// The per-pair loop of IntelPairHMM::computeLikelihoodsNative
// (intel_pairhmm.hpp:128-147) over independent pairs, OpenMP dynamic schedule.
long ref_pairs(long n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
               const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
               const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, float* raw_f32,
               double* raw_f64, uint8_t* rescued, double* loglik, int nthreads)
{
    ensure_init();
    long nres = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+ : nres)
#endif
    {
        unsigned old = _mm_getcsr();
        _MM_SET_FLUSH_ZERO_MODE(_MM_FLUSH_ZERO_ON);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (long p = 0; p < n; ++p) {
            const int64_t ro = read_off[p], ho = hap_off[p];
            testcase tc = make_tc(R[p], H[p], rs + ro, q + ro, ins + ro, del + ro, gcp + ro, hap + ho);
            float f = compute_full_prob_avxs<float>(&tc);
            double dd = 0.0, L;
            int resc = 0;
            if (f < MIN_ACCEPTED) {
                dd = compute_full_prob_avxd<double>(&tc);
                L = std::log10(dd) - ctxd().LOG10_INITIAL_CONSTANT;
                resc = 1;
            } else {
                L = (double)(log10f(f) - ctxf().LOG10_INITIAL_CONSTANT);
            }
            nres += resc;
            if (raw_f32) raw_f32[p] = f;
            if (raw_f64) raw_f64[p] = dd;
            if (rescued) rescued[p] = (uint8_t)resc;
            if (loglik) loglik[p] = L;
        }
        _mm_setcsr(old);
    }
    (void)nthreads;
    return nres;
}

} // extern "C"
