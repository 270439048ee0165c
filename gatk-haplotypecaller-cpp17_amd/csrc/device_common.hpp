// Device helpers shared by the PairHMM kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hcphmm {

// Fields of a packed read row (kernels.hpp pack_row).
__device__ __forceinline__ int row_q(uint32_t w) { return w & 127; }
__device__ __forceinline__ int row_i(uint32_t w) { return (w >> 7) & 127; }
__device__ __forceinline__ int row_d(uint32_t w) { return (w >> 14) & 127; }
__device__ __forceinline__ int row_c(uint32_t w) { return (w >> 21) & 127; }
__device__ __forceinline__ int row_rc(uint32_t w) { return (w >> 28) & 7; }

// set_mm_prob index (Context.h:168-179): triangular table over (min, max).
__device__ __forceinline__ int mm_idx(int a, int b)
{
    const int lo = min(a, b), hi = max(a, b);
    return ((hi * (hi + 1)) >> 1) + lo;
}

}  // namespace hcphmm
