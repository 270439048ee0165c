// Genotyper numeric-core device layout (gt_kernels.hip / gt_engine.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hcgt {

constexpr int kMaxAlleles = 7;            // Genetyper::MAX_ALLELE_COUNT (genotyper.hpp:19)
constexpr int kJacobianLen = 80001;       // MathUtils table (utils/math_utils.hpp:24-31)

struct GtSite {
    int64_t L_off;    // first double of the site's matrix in L[]
    int64_t al_off;   // allele-likelihood scratch (n_keep x n_alleles doubles)
    int32_t n_haps;
    int32_t keep_off, n_keep;
    int32_t map_off;
    int32_t n_alleles;
    int32_t out_off;  // first genotype likelihood in gl[]
};

struct GtArgs {
    const GtSite* sites;
    int n;
    const double* L;
    const int32_t* keep;
    const int32_t* amap;
    const double* jac;
    double inv_step;   // 1.0 / TABLE_STEP as the reference computes it
    double log10_2;    // std::log10(2)
    double* al;
    double* gl;
    int32_t* gi;
    int32_t* gq;
};

hipError_t launch_sites(const GtArgs& a, hipStream_t s);

}  // namespace hcgt
