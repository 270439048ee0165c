// Micro-benchmark: issue rate of the VALU forms the Smith-Waterman step
// (int32 add/sub/max/alignbit, DPP moves), the PairHMM cell (fp32 mul/add and
// the prior select: bfe/bitop3/and/xor/cndmask) and its fp64 rescue (f64
// mul/add) can use on gfx950. 16 independent chains per lane, 8 waves per
// SIMD, so the result is the issue rate, not the latency. gfx950 issues some
// forms (f32 add/mul, u32 add) twice as fast as others (max, alignbit, f64,
// DPP): the kernels' instruction choice and the rooflines follow from this.
//   hipcc --offload-arch=gfx950 -O3 op_rate.hip -o op_rate && ./op_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 2048;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

// One benchmark: name + an asm body applied to a[i] (int) with operand c / cf / d[i].
#define OPS(F)                                                                    \
    F(0, "v_add_u32", "v_add_u32 %0, %0, %1")                                     \
    F(1, "v_sub_u32", "v_sub_u32 %0, %0, %1")                                     \
    F(2, "v_max_i32", "v_max_i32 %0, %0, %1")                                     \
    F(3, "v_min_u32", "v_min_u32 %0, %0, %1")                                     \
    F(4, "v_max3_i32", "v_max3_i32 %0, %0, %1, %1")                               \
    F(5, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %1, 31")                       \
    F(6, "v_and_b32", "v_and_b32 %0, %0, %1")                                     \
    F(7, "v_xor_b32", "v_xor_b32 %0, %0, %1")                                     \
    F(8, "v_or_b32", "v_or_b32 %0, %0, %1")                                       \
    F(9, "v_lshlrev_b32", "v_lshlrev_b32 %0, 1, %0")                              \
    F(10, "v_ashrrev_i32", "v_ashrrev_i32 %0, 31, %0")                            \
    F(11, "v_bfe_i32", "v_bfe_i32 %0, %1, %0, 1")                                 \
    F(12, "v_bitop3_b32", "v_bitop3_b32 %0, %0, %1, %1 bitop3:0xe4")             \
    F(13, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %1")                                \
    F(14, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 1, %1")                         \
    F(15, "v_lshl_add_u32", "v_lshl_add_u32 %0, %0, 1, %1")                       \
    F(16, "v_add3_u32", "v_add3_u32 %0, %0, %1, %1")                              \
    F(17, "v_perm_b32", "v_perm_b32 %0, %0, %1, %1")                              \
    F(18, "v_cndmask_b32(vcc)", "v_cndmask_b32 %0, %0, %1, vcc")                  \
    F(19, "v_mov_b32", "v_mov_b32 %0, %1")                                        \
    F(20, "v_mov_b32_dpp wave_shr:1", "v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf") \
    F(21, "v_add_u32_dpp wave_shr:1", "v_add_u32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf") \
    F(22, "v_mov_b32_dpp row_shr:1", "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf") \
    F(23, "v_add_u32_sdwa", "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1") \
    F(24, "v_add_f32", "v_add_f32 %0, %0, %1")                                    \
    F(25, "v_mul_f32", "v_mul_f32 %0, %0, %1")                                    \
    F(26, "v_max_f32", "v_max_f32 %0, %0, %1")                                    \
    F(27, "v_cmp_gt_i32(vcc)", "v_cmp_gt_i32 vcc, %0, %1")                        \
    F(28, "v_sub_co_u32", "v_sub_co_u32 %0, vcc, %0, %1")                         \
    F(29, "v_addc_co_u32", "v_addc_co_u32 %0, vcc, %0, %0, vcc")                  \
    F(30, "v_mul_f32_dpp wave_shr:1", "v_mul_f32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf") \
    F(31, "v_med3_i32", "v_med3_i32 %0, %0, %1, %1")                             \
    F(32, "v_cndmask_b32(vcc,no-clobber)", "v_cndmask_b32 %0, %0, %1, vcc")       \
    F(33, "v_cndmask_b32_e64(sgpr)", "v_cndmask_b32_e64 %0, %0, %1, s[20:21]")    \
    F(34, "v_cmp_eq_u32+v_cndmask_b32(2)", "v_cmp_eq_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc") \
    F(35, "v_add_u32_e64", "v_add_u32_e64 %0, %0, %1")                            \
    F(36, "v_lshrrev_b32", "v_lshrrev_b32 %0, 1, %0")                             \
    F(37, "v_add_u32(sgpr)", "v_add_u32 %0, s20, %0")                             \
    F(38, "v_sub_i32(vop3)", "v_sub_i32 %0, %0, %1")                                    \
    F(39, "v_not_b32", "v_not_b32 %0, %0")                                        \
    F(40, "v_sub_u32+v_ashrrev+v_and(3)", "v_sub_u32 %0, %0, %1\n v_ashrrev_i32 %0, 31, %0\n v_and_b32 %0, %0, %1") \
    F(41, "v_lshlrev_b32(vgpr-shift)", "v_lshlrev_b32 %0, %1, %0")                \
    F(42, "v_subrev_u32", "v_subrev_u32 %0, %0, %1")                              \
    F(43, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %1")                        \
    F(44, "v_mul_u32_u24", "v_mul_u32_u24 %0, %0, %1")                            \
    F(45, "v_and_b32_sdwa sext(BYTE_1)", "v_and_b32_sdwa %0, %1, sext(%0) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1") \
    F(46, "prior select v_bfe_i32+v_bitop3_b32(2)", "v_bfe_i32 %0, %1, %0, 1\n v_bitop3_b32 %0, %0, %1, %1 bitop3:0xe4") \
    F(47, "prior select v_and_b32_sdwa+v_xor_b32(2)", "v_and_b32_sdwa %0, %1, sext(%0) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_xor_b32 %0, %0, %1")

constexpr int NOPS = 48;

template <int MODE>
__global__ __launch_bounds__(256) void k(int* out, int c)
{
    int a[16];
    for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 7 + i;
    asm volatile("v_cmp_gt_u32 vcc, 32, %0\n s_mov_b64 s[20:21], vcc" ::"v"(int(threadIdx.x)) : "vcc", "s20", "s21");
    for (int it = 0; it < ITERS; ++it) {
#define CASE(ID, NAME, ASM)                                                 \
    if constexpr (MODE == ID) {                                             \
        _Pragma("unroll") for (int i = 0; i < 16; ++i)                      \
            { if constexpr (ID == 27 || ID == 28 || ID == 29 || ID == 34 || ID == 18) asm volatile(ASM : "+v"(a[i]) : "v"(c) : "vcc"); \
              else asm volatile(ASM : "+v"(a[i]) : "v"(c)); }                \
    }
        OPS(CASE)
#undef CASE
    }
    int s = 0;
    for (int i = 0; i < 16; ++i) s += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
__global__ __launch_bounds__(256) void kd(int* out, int mode)
{
    double d[16];
    for (int i = 0; i < 16; ++i) d[i] = 1.0 + threadIdx.x * 1e-3 + i;
    const double cd = 1.0000001;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (MODE == 0) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(cd));
            else asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(cd));
        }
    }
    int s = 0;
    for (int i = 0; i < 16; ++i) s += int(d[i]);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

static int g_per = 1;
template <typename K>
double run(K kern, int* out, int blocks)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) kern<<<blocks, 256>>>(out, 3);
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; ++r) kern<<<blocks, 256>>>(out, 3);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double wave_instr = double(blocks) * 4 * ITERS * 16 * 10 * g_per;
    return wave_instr / (ms * 1e-3);
}

static void report(const char* name, double r)
{
    printf("{\"instr\": \"%s\", \"wave_instr_per_s\": %.4g, \"lane_ops_T_per_s\": %.2f, "
           "\"cycles_per_wave_instr_per_SIMD_at_2.4GHz\": %.2f}\n",
           name, r, r * 64 / 1e12, (256 * 4 * 2.4e9) / r);
}

template <int M>
void all(int* out, int blocks)
{
    if constexpr (M < NOPS) {
        static const char* names[NOPS] = {
#define NAME(ID, NAME, ASM) NAME,
            OPS(NAME)
#undef NAME
        };
        g_per = (M == 34 || M == 46 || M == 47) ? 2 : (M == 40) ? 3 : 1;
        report(names[M], run(k<M>, out, blocks));
        g_per = 1;
        all<M + 1>(out, blocks);
    }
}

int main()
{
    const int blocks = 256 * 8;   // 8 blocks of 4 waves per CU = 8 waves / SIMD
    int* out;
    (void)hipMalloc(&out, sizeof(int) * blocks * 256);
    all<0>(out, blocks);
    report("v_mul_f64", run(kd<0>, out, blocks));
    report("v_add_f64", run(kd<1>, out, blocks));
    return 0;
}
