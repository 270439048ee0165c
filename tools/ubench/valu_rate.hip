// Micro-benchmark: issue rate of the VALU forms the PairHMM cell update can use
// on gfx950 (v_mul_f32, v_add_f32, v_pk_mul_f32, v_pk_add_f32, v_mov_b32_dpp,
// v_cndmask_b32). Sets the peak the roofline in bench.py is priced against.
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float c)
{
    float a0 = threadIdx.x * 1e-3f + 1.f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
    f2 cc = {c, c};
    int i0 = threadIdx.x, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (MODE == 0) {   // 8 x v_mul_f32
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a0) : "v"(c)); asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a1) : "v"(c));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a2) : "v"(c)); asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a3) : "v"(c));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a4) : "v"(c)); asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a5) : "v"(c));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a6) : "v"(c)); asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a7) : "v"(c));
            } else if constexpr (MODE == 1) {   // 8 x v_pk_mul_f32 (16 lane-ops each lane)
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p0) : "v"(cc)); asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p1) : "v"(cc));
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p2) : "v"(cc)); asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p3) : "v"(cc));
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p0) : "v"(cc)); asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p1) : "v"(cc));
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p2) : "v"(cc)); asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p3) : "v"(cc));
            } else if constexpr (MODE == 2) {   // 8 x v_pk_add_f32
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p0) : "v"(cc)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p1) : "v"(cc));
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p2) : "v"(cc)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p3) : "v"(cc));
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p0) : "v"(cc)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p1) : "v"(cc));
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p2) : "v"(cc)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p3) : "v"(cc));
            } else if constexpr (MODE == 3) {   // 8 x v_mov_b32_dpp row_shr:1
                asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i0)); asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i1));
                asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i2)); asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i3));
                asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i0)); asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i1));
                asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i2)); asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(i3));
            } else if constexpr (MODE == 4) {   // 8 x v_mul_f32 with a DPP source (fused shift)
                asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a0) : "v"(c)); asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a1) : "v"(c));
                asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a2) : "v"(c)); asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a3) : "v"(c));
                asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a4) : "v"(c)); asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a5) : "v"(c));
                asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a6) : "v"(c)); asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a7) : "v"(c));
            } else {   // 8 x v_cndmask_b32 on vcc
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a0) : "v"(c)); asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a1) : "v"(c));
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a2) : "v"(c)); asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a3) : "v"(c));
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a4) : "v"(c)); asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a5) : "v"(c));
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a6) : "v"(c)); asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a7) : "v"(c));
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y +
                                          p2.x + p2.y + p3.x + p3.y + i0 + i1 + i2 + i3;
}

template <int MODE>
double run(float* out, int blocks)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<MODE><<<blocks, 256>>>(out, 1.0000001f);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k<MODE><<<blocks, 256>>>(out, 1.0000001f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double wave_instr = double(blocks) * 4 * ITERS * 32 * 5;   // waves x instructions
    return wave_instr / (ms * 1e-3);   // wave-instructions per second
}

int main()
{
    int blocks = 256 * 8;   // 8 blocks of 4 waves per CU = 8 waves / SIMD
    float* out;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    const char* names[] = {"v_mul_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_mov_b32_dpp", "v_mul_f32_dpp", "v_cndmask_b32"};
    double r[6] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks), run<4>(out, blocks), run<5>(out, blocks)};
    for (int m = 0; m < 6; ++m) {
        // lane-ops/s: packed forms do 2 per lane
        const double lanes = r[m] * 64 * ((m == 1 || m == 2) ? 2 : 1);
        printf("{\"instr\": \"%s\", \"wave_instr_per_s\": %.4g, \"lane_ops_T_per_s\": %.2f, \"cycles_per_wave_instr_per_SIMD_at_2.4GHz\": %.2f}\n",
               names[m], r[m], lanes / 1e12, (256 * 4 * 2.4e9) / r[m]);
    }
    return 0;
}
