// Micro-benchmark: pure-register throughput of the lane kernel's cell update
// (lane_kernel.hip `cell`) for P = 1 (scalar) and P = 2 (packed v_pk_*), no
// memory traffic: the rows of one column block recomputed in a loop. Tells
// whether packed f32 can beat scalar on the real dependency structure.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize \
//         -I../../gatk-haplotypecaller-cpp17_amd/csrc cell_rate.hip -o cell_rate
#include "../../gatk-haplotypecaller-cpp17_amd/csrc/lane_kernel.hip"

#include <cstdio>

namespace hcphmm {
namespace {

template <int P, int BC, int OCC>
__global__ __launch_bounds__(256, OCC) void cell_bench(float* out, const float* __restrict__ kc, int rows, uint32_t seed)
{
    using V = typename VT<P>::type;
    V T[BC], X[BC];
    const float b = 1.f + (threadIdx.x & 7) * 1e-3f;
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        T[j] = splat<V>(b);
        X[j] = splat<V>(0.f);
    }
    RowConst<P> k;
    // distinct, opaque constants (loaded) so the compiler cannot share products
    const int q = threadIdx.x & 7;
    k.pm = splat<V>(kc[q]); k.px = splat<V>(kc[8 + q]); k.my = splat<V>(kc[16 + q]); k.yy = splat<V>(kc[24 + q]);
    k.mm = splat<V>(kc[32 + q]); k.g = splat<V>(kc[40 + q]); k.mx = splat<V>(kc[48 + q]); k.xx = splat<V>(kc[56 + q]);
    uint32_t w = seed ^ (threadIdx.x * 0x9e3779b9u);
    V sumM = splat<V>(0.f), sumX = splat<V>(0.f);
    const int lim[P] = {};
    for (int i = 0; i < rows; ++i) {
        uint32_t mw[P][2];
        int pmi[P], pxi[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            mw[p][0] = w + p;
            mw[p][1] = w ^ (p + 1);
            pmi[p] = __float_as_int(comp(k.pm, p));
            pxi[p] = __float_as_int(comp(k.px, p));
        }
        w = w * 1664525u + 1013904223u;
        V Ml = splat<V>(0.f), Yl = splat<V>(0.f);
        const V M0 = T[0] * prior_vec<P, 0>(mw, pmi, pxi);
        cell<P, BC, 0, BC, false>(T, X, M0, Ml, Yl, mw, pmi, pxi, k, lim, sumM, sumX);
        // keep values bounded without extra per-cell work: renormalise column 0
        T[0] = T[0] * k.mm;
    }
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < BC; ++j)
#pragma unroll
        for (int p = 0; p < P; ++p) acc += comp(T[j], p) + comp(X[j], p);
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int P, int BC, int OCC>
double run(float* out, const float* kc, int blocks, int rows)
{
    hipEvent_t a, e;
    hipEventCreate(&a);
    hipEventCreate(&e);
    cell_bench<P, BC, OCC><<<blocks, 256>>>(out, kc, rows, 1u);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) cell_bench<P, BC, OCC><<<blocks, 256>>>(out, kc, rows, 7u + r);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, a, e);
    const double cells = double(blocks) * 256 * P * BC * rows * reps;
    return cells / (ms * 1e-3);
}

}  // namespace
}  // namespace hcphmm

int main()
{
    using namespace hcphmm;
    float* out;
    const int rows = 2048;
    hipMalloc(&out, sizeof(float) * 256 * 64 * 256);
    float hk[64];
    const float base[8] = {0.9f, 0.03f, 1.1e-4f, 0.1f, 0.99f, 0.89f, 1.3e-4f, 0.11f};
    for (int c = 0; c < 8; ++c)
        for (int q = 0; q < 8; ++q) hk[c * 8 + q] = base[c] * (1.f + q * 1e-3f);
    float* kc;
    hipMalloc(&kc, sizeof(hk));
    hipMemcpy(kc, hk, sizeof(hk), hipMemcpyHostToDevice);
    for (int blocks_per_cu : {2, 3, 4, 8}) {
        const int blocks = 256 * blocks_per_cu;
        printf("{\"blocks_per_cu\": %d, \"P1_BC64_occ3\": %.1f, \"P1_BC64_occ2\": %.1f, \"P2_BC32_occ2\": %.1f, "
               "\"P2_BC16_occ4\": %.1f, \"P1_BC32_occ4\": %.1f, \"unit\": \"GCUPS\"}\n",
               blocks_per_cu, run<1, 64, 3>(out, kc, blocks, rows) / 1e9, run<1, 64, 2>(out, kc, blocks, rows) / 1e9,
               run<2, 32, 2>(out, kc, blocks, rows) / 1e9, run<2, 16, 4>(out, kc, blocks, rows) / 1e9,
               run<1, 32, 4>(out, kc, blocks, rows) / 1e9);
    }
    return 0;
}
