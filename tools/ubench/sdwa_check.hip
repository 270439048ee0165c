// Semantics check of the SDWA byte-sign-extended AND on gfx950 (the fp32
// prior select of seg_common.hpp prior_sel): v_and_b32_sdwa d, sext(w.BYTE_j)
// must equal d & (int32)(int8)(w >> 8j) for every input.
//   hipcc --offload-arch=gfx950 -O3 sdwa_check.hip -o sdwa_check && ./sdwa_check
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

template <int J>
__device__ __forceinline__ uint32_t and_sext(uint32_t d, uint32_t w)
{
    uint32_t r;
    if constexpr (J == 0)
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(d), "v"(w));
    else if constexpr (J == 1)
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(d), "v"(w));
    else if constexpr (J == 2)
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(d), "v"(w));
    else
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(d), "v"(w));
    return r;
}

__global__ void k(uint32_t* o, const uint32_t* d, const uint32_t* w, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    o[4 * t + 0] = and_sext<0>(d[t], w[t]);
    o[4 * t + 1] = and_sext<1>(d[t], w[t]);
    o[4 * t + 2] = and_sext<2>(d[t], w[t]);
    o[4 * t + 3] = and_sext<3>(d[t], w[t]);
}

int main()
{
    const int n = 1 << 20;
    std::mt19937 g(7);
    std::vector<uint32_t> d(n), w(n), o(4 * size_t(n));
    for (int i = 0; i < n; ++i) {
        d[i] = g();
        w[i] = g();
    }
    uint32_t *dd, *dw, *dout;
    (void)hipMalloc(&dd, 4 * size_t(n));
    (void)hipMalloc(&dw, 4 * size_t(n));
    (void)hipMalloc(&dout, 16 * size_t(n));
    (void)hipMemcpy(dd, d.data(), 4 * size_t(n), hipMemcpyHostToDevice);
    (void)hipMemcpy(dw, w.data(), 4 * size_t(n), hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dout, dd, dw, n);
    (void)hipMemcpy(o.data(), dout, 16 * size_t(n), hipMemcpyDeviceToHost);
    long bad = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 4; ++j) {
            const uint32_t m = uint32_t(int32_t(int8_t(uint8_t(w[i] >> (8 * j)))));
            bad += o[4 * size_t(i) + j] != (d[i] & m);
        }
    printf("{\"check\": \"v_and_b32_sdwa sext(BYTE_j)\", \"cases\": %d, \"mismatches\": %ld}\n", 4 * n, bad);
    return bad != 0;
}
