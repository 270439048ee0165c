// Genotyper numeric core on gfx950: one wave per variant site.
//
// Reference: src/haplotypecaller/genotyper/genotyper.hpp — marginal_likelihoods
// (:245-264), calculate_read_likelihoods_by_genotype_index / get_genotype_likelihoods
// (:294-322), get_genotype_quality_and_max_genotype_index (:324-355); and
// MathUtils::approximate_log10_sum_log10 (utils/math_utils.hpp:11-33).
//
// Phase 1: lanes over the site's kept reads, each lane takes its read's row of
//          the region's likelihood matrix and keeps the per-allele maximum in
//          registers (strict >, haplotype order, from -DBL_MAX) -> HBM scratch.
// Phase 2: lane g < #genotypes sums its genotype's per-read term in read order
//          (std::accumulate is sequential; so is this) — the Jacobian table
//          lookups hit the L2-resident 640 KB table.
// Phase 3: the wave's first lane picks the best genotype and its quality from
//          the lanes' sums (shuffles), with the reference's comparisons.
// The work is tiny and latency-bound; batching every site of every region into
// one launch is what makes it pay.
#include "gt_kernels.hpp"

#include <cfloat>
#include <cmath>

namespace hcgt {
namespace {

__device__ __forceinline__ double approx_sum(double a, double b, const double* jac, double inv_step)
{
    if (a > b) {
        const double t = a;
        a = b;
        b = t;
    }
    const double diff = b - a;
    return b + (diff < 8.0 ? jac[size_t(round(diff * inv_step))] : 0.0);
}

__global__ __launch_bounds__(256) void gt_sites_kernel(GtArgs a)
{
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= a.n) return;
    const GtSite S = a.sites[s];
    const int nh = __builtin_amdgcn_readfirstlane(S.n_haps);
    const int nk = __builtin_amdgcn_readfirstlane(S.n_keep);
    const int A = __builtin_amdgcn_readfirstlane(S.n_alleles);
    const double* L = a.L + S.L_off;
    const int32_t* keep = a.keep + S.keep_off;
    const int32_t* amap = a.amap + S.map_off;
    double* al = a.al + S.al_off;

    for (int r = lane; r < nk; r += 64) {
        const double* row = L + int64_t(keep[r]) * nh;
        double m[kMaxAlleles];
#pragma unroll
        for (int k = 0; k < kMaxAlleles; ++k) m[k] = -DBL_MAX;
        for (int h = 0; h < nh; ++h) {
            const double x = row[h];
            const int al_h = amap[h];
#pragma unroll
            for (int k = 0; k < kMaxAlleles; ++k)
                if (al_h == k && x > m[k]) m[k] = x;
        }
#pragma unroll
        for (int k = 0; k < kMaxAlleles; ++k)
            if (k < A) al[int64_t(r) * A + k] = m[k];
    }
    __threadfence_block();   // this wave's scratch stores are visible to its other lanes

    const int G = A * (A + 1) / 2;
    double gl = 0.0;
    if (lane < G) {
        int a1 = 0, rem = lane;
        while (rem >= A - a1) {
            rem -= A - a1;
            ++a1;
        }
        const int a2 = a1 + rem;
        double acc = 0.0;
        for (int r = 0; r < nk; ++r) {
            const double x1 = al[int64_t(r) * A + a1];
            acc += a1 == a2 ? x1 + a.log10_2 : approx_sum(x1, al[int64_t(r) * A + a2], a.jac, a.inv_step);
        }
        gl = acc - double(nk) * a.log10_2;
        a.gl[S.out_off + lane] = gl;
    }
    // get_genotype_quality_and_max_genotype_index, on every lane with the same values.
    const double g0 = __shfl(gl, 0), g1 = __shfl(gl, 1);
    double mx, second;
    int idx;
    if (g0 > g1) {
        second = g1;
        mx = g0;
        idx = 0;
    } else {
        second = g0;
        mx = g1;
        idx = 1;
    }
    for (int i = 2; i < G; ++i) {
        const double gi = __shfl(gl, i);
        if (gi >= mx) {
            second = mx;
            mx = gi;
            idx = i;
        } else if (gi > second) {
            second = gi;
        }
    }
    if (lane == 0) {
        // static_cast<size_t>(round(...)) capped at 99; NaN and >= 2^64 as the
        // reference's g++ x86-64 build converts them (see oracle/gt_oracle.c).
        const double q = round(-10.0 * (second - mx));
        a.gi[s] = idx;
        a.gq[s] = isnan(q) ? 99 : q >= 18446744073709551616.0 ? 0 : q > 99.0 ? 99 : int(q);
    }
}

}  // namespace

hipError_t launch_sites(const GtArgs& a, hipStream_t s)
{
    if (a.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gt_sites_kernel, dim3((a.n + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcgt
