// PairHMM forward kernels for gfx950 (MI355X).
//
// Semantics: compute_full_prob_avx{s,d} of the reference
// (pairhmm/native/avx-pairhmm-template.h:210-346), bit-exact: IEEE mul/add
// in the reference's operation order, no FMA (built -ffp-contract=off),
// denormal results flushed (built -fgpu-flush-denormals-to-zero for f32 and
// -fdenormal-fp-math=preserve-sign for f64, the MXCSR FTZ of
// intel_pairhmm.hpp:105).
//
// Mapping ("anti-diagonal, W lanes per pair"): a group of W lanes owns one
// (read, hap) pair; lane l holds row i = s*W + l + 1 of stripe s and at step t
// computes column j = t - l, so a group sweeps one anti-diagonal per step.
// The recurrence is carried in a two-value form: after computing cell (i, j)
//   T  = (M*mm' + X*gapm') + Y*gapm'   (row i+1's transition constants)
//   XN = M*mx' + X*xx'                 (= X[i+1][j])
// so row i+1 needs only T[i][j-1] (diagonal) and XN (vertical) from the lane
// above: two DPP lane shifts per step (row_shr:1 inside 16-lane rows, or
// wave_shr:1 / row_bcast:15 for wider groups), instead of the reference's
// three shifted vectors (M, X, Y_t_1: avx-vector-shift.h:3-30). The values are
// the same IEEE operations in the same order, only evaluated one step earlier.
// The last lane of a stripe hands T/XN of its row to lane 0 of the next stripe
// through an LDS ring indexed by column (the reference's shiftOutM/X buffers,
// avx-pairhmm-template.h:224,287-291). The match prior comes from 32-column
// bit windows of the hap match table (precompute_masks, :3-35), one select per
// cell.
#include "device_common.hpp"
#include "kernels.hpp"
#include "luts.hpp"

namespace hcphmm {
namespace {

template <typename T> struct Pair2 { T t, xn; };

// Lane shift by one inside each W-lane group: lane l gets lane l-1's `src`,
// lane 0 of the group gets `old` (the stripe carry-in).
template <int W>
__device__ __forceinline__ int shr1_i(int src, int old)
{
    if constexpr (W == 16) {
        return __builtin_amdgcn_update_dpp(old, src, 0x111, 0xf, 0xf, false);   // row_shr:1
    } else if constexpr (W == 32) {
        // rows 1 and 3 first take lane 15/47 of the row before (row_bcast:15),
        // then row_shr:1 fills lanes 1..15 of every row.
        const int b = __builtin_amdgcn_update_dpp(old, src, 0x142, 0xa, 0xf, false);
        return __builtin_amdgcn_update_dpp(b, src, 0x111, 0xf, 0xf, false);
    } else {
        return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);   // wave_shr:1
    }
}

template <int W>
__device__ __forceinline__ float shr1(float src, float old)
{
    return __int_as_float(shr1_i<W>(__float_as_int(src), __float_as_int(old)));
}

template <int W>
__device__ __forceinline__ double shr1(double src, double old)
{
    const long long s = __double_as_longlong(src), o = __double_as_longlong(old);
    const int lo = shr1_i<W>(int(s & 0xffffffffll), int(o & 0xffffffffll));
    const int hi = shr1_i<W>(int(s >> 32), int(o >> 32));
    return __longlong_as_double((long long)((unsigned long long)(unsigned)hi << 32 | (unsigned)lo));
}

// Prior of the column whose match bit is bit B (MSB first) of the lane's 32-bit
// window: v_bfe_i32 (bit -> 0 / -1) + one bit-select (v_bitop3 / v_cndmask).
template <int B>
__device__ __forceinline__ float take_prior(uint32_t win, float pm, float px)
{
    int t;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(t) : "v"(win), "i"(B));
    return __int_as_float((t & __float_as_int(pm)) | (~t & __float_as_int(px)));
}
template <int B>
__device__ __forceinline__ double take_prior(uint32_t win, double pm, double px)
{
    return int(win << (31 - B)) < 0 ? pm : px;
}

template <typename T> __device__ __forceinline__ T initial_constant();
template <> __device__ __forceinline__ float initial_constant<float>() { return 0x1p120f; }
template <> __device__ __forceinline__ double initial_constant<double>() { return 0x1p1020; }

// One anti-diagonal step (column t - l for lane l). S = step index inside the
// 32-step window (compile time), so the prior bit is a constant.
template <typename T, int W, bool SUM, int S>
__device__ __forceinline__ void diag_step(Pair2<T>* __restrict__ wp, const Pair2<T>& rv, uint32_t win, int l,
                                          int lim, int t, T pm, T px, T my, T yy, T mm1, T g1, T mx1,
                                          T xx1, T& Ml, T& Yl, T& shT2, T& shT1, T& shX, T& sumM, T& sumX)
{
    const T prior = take_prior<31 - S>(win, pm, px);
    const T M = shT2 * prior;
    const T X = shX;
    const T Y = Ml * my + Yl * yy;
    const T Tn = (M * mm1 + X * g1) + Y * g1;
    const T XN = M * mx1 + X * xx1;
    shT2 = shT1;
    shT1 = shr1<W>(Tn, rv.t);
    shX = shr1<W>(XN, rv.xn);
    if (l == W - 1) *wp = Pair2<T>{Tn, XN};   // column t-W+1 (+W offset)
    Ml = M;
    Yl = Y;
    if constexpr (SUM) {
        const bool c = t <= lim;   // lane holds row R and column t-l <= H
        sumM = sumM + (c ? M : T(0));
        sumX = sumX + (c ? X : T(0));
    }
}

// Eight steps starting at step t0 + U. Returns false when the stripe ended first.
template <typename T, int W, bool SUM, int U>
__device__ __forceinline__ bool sub_block(Pair2<T>* __restrict__ ring, int t0, int nsteps, uint32_t win, int l,
                                          int lim, T pm, T px, T my, T yy, T mm1, T g1, T mx1, T xx1,
                                          T& Ml, T& Yl, T& shT2, T& shT1, T& shX, T& sumM, T& sumX)
{
    if (t0 + U > nsteps) return false;
    Pair2<T>* rp = ring + (t0 + U);
    // Carry-ins of lane 0 for the next 8 columns, read in one batch: they were
    // written a whole stripe ago and are overwritten only W steps from now.
    Pair2<T> rv[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) rv[v] = rp[v + W + 1];
    const int t = t0 + U;
#define HC_STEP(v) diag_step<T, W, SUM, U + v>(rp + v + 1, rv[v], win, l, lim, t + v, pm, px, my, yy, mm1, \
                                              g1, mx1, xx1, Ml, Yl, shT2, shT1, shX, sumM, sumX)
    HC_STEP(0); HC_STEP(1); HC_STEP(2); HC_STEP(3); HC_STEP(4); HC_STEP(5); HC_STEP(6); HC_STEP(7);
#undef HC_STEP
    return true;
}

template <typename T, int W, bool SUM>
__device__ __forceinline__ void run_stripe(
    Pair2<T>* __restrict__ ring, const uint32_t* __restrict__ hw, int nwpad, int rc, int l,
    int nsteps, int H, bool last, T pm, T px, T my, T yy, T mm1, T g1, T mx1, T xx1,
    T& sumM, T& sumX)
{
    T Ml = T(0), Yl = T(0);
    const Pair2<T> r0 = ring[W + 0], r1 = ring[W + 1];
    T shT2 = (l == 0) ? r0.t : T(0);   // T of row above at column j-1 (diagonal)
    T shT1 = (l == 0) ? r1.t : T(0);   // ... one step younger
    T shX = (l == 0) ? r1.xn : T(0);   // X of this row at column j (from row above)
    const int lim = last ? H + l : -1;
    for (int t0 = 1; t0 <= nsteps; t0 += 32) {
        // 32-column match window starting at this lane's column j0 = t0 - l.
        const int k = t0 - 1 - l;
        const int wi = k >> 5, sh = k & 31;
        const int a0 = min(wi + kHapLead, nwpad), a1 = min(wi + kHapLead + 1, nwpad);
        const uint32_t hiw = hw[a0 * 5 + rc], low = hw[a1 * 5 + rc];
        const uint32_t win = sh ? ((hiw << sh) | (low >> (32 - sh))) : hiw;
        if (!sub_block<T, W, SUM, 0>(ring, t0, nsteps, win, l, lim, pm, px, my, yy, mm1, g1, mx1, xx1,
                                     Ml, Yl, shT2, shT1, shX, sumM, sumX)) break;
        if (!sub_block<T, W, SUM, 8>(ring, t0, nsteps, win, l, lim, pm, px, my, yy, mm1, g1, mx1, xx1,
                                     Ml, Yl, shT2, shT1, shX, sumM, sumX)) break;
        if (!sub_block<T, W, SUM, 16>(ring, t0, nsteps, win, l, lim, pm, px, my, yy, mm1, g1, mx1, xx1,
                                      Ml, Yl, shT2, shT1, shX, sumM, sumX)) break;
        if (!sub_block<T, W, SUM, 24>(ring, t0, nsteps, win, l, lim, pm, px, my, yy, mm1, g1, mx1, xx1,
                                      Ml, Yl, shT2, shT1, shX, sumM, sumX)) break;
    }
}

// GRING: the ring in global memory (a.ring_global, this workgroup's slice),
// for haps too long for the LDS; a wave reads back only what it wrote itself,
// in program order.
template <typename T, int W, bool GRING>
__global__ __launch_bounds__(64) void phmm_diag_kernel(DiagArgs a)
{
    constexpr int G = 64 / W;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int g = lane / W, l = lane % W;
    const T* __restrict__ lut = static_cast<const T*>(a.lut);
    const T* __restrict__ ph2pr = lut + kOffPh2pr;
    Pair2<T>* ring = GRING ? static_cast<Pair2<T>*>(a.ring_global) + (size_t(blockIdx.x) * G + g) * size_t(a.ring_len)
                           : reinterpret_cast<Pair2<T>*>(smem) + g * a.ring_len;
    const int n = a.n_slots_dev ? *a.n_slots_dev : a.n_slots;
    if (a.count_reset && blockIdx.x == 0 && threadIdx.x == 0) *a.count_reset = 0;

    for (int wv = blockIdx.x; wv * G < n; wv += gridDim.x) {
        const int slot = wv * G + g;
        const bool active = slot < n;
        const int pid = a.order[active ? slot : wv * G];
        const PairDesc pd = a.pairs[pid];
        const int R = pd.y, H = pd.w;
        const int Sg = (R + W - 1) / W;
        int Hmax = H, S = Sg;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            Hmax = max(Hmax, __builtin_amdgcn_readlane(H, k * W));
            S = max(S, __builtin_amdgcn_readlane(Sg, k * W));
        }
        const uint32_t* __restrict__ rrow = a.rows + pd.x;
        const uint32_t* __restrict__ hw = a.hapw + pd.z;
        const int nwpad = (H + 31) / 32 + kHapLead;   // index of the trailing zero row

        // Row 0 (avx-pairhmm-template.h:86-92, 164-169): M = X = 0, Y = INITIAL/H.
        {
            const uint32_t w1 = rrow[0];
            const T mm1 = lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
            const T g1 = lut[kOffGapm + row_c(w1)];
            const T mx1 = ph2pr[row_i(w1)], xx1 = ph2pr[row_c(w1)];
            const T initY = initial_constant<T>() / T(H);
            const T T0 = (T(0) * mm1 + T(0) * g1) + initY * g1;
            const T X0 = T(0) * mx1 + T(0) * xx1;
            for (int j = l; j < a.ring_len; j += W) ring[j] = Pair2<T>{T0, X0};
        }
        __syncthreads();

        T sumM = T(0), sumX = T(0);
        const int nsteps = Hmax + W - 1;
        for (int s = 0; s < S; ++s) {
            const int i = s * W + l + 1;
            const uint32_t wc = rrow[min(i, R) - 1];
            const uint32_t wn = rrow[min(i + 1, R) - 1];
            const T my = ph2pr[row_d(wc)], yy = ph2pr[row_c(wc)];
            const T pm = lut[kOffPm + row_q(wc)], px = lut[kOffPx + row_q(wc)];
            const T mm1 = lut[kOffMM + mm_idx(row_i(wn), row_d(wn))];
            const T g1 = lut[kOffGapm + row_c(wn)];
            const T mx1 = ph2pr[row_i(wn)], xx1 = ph2pr[row_c(wn)];
            const int rc = row_rc(wc);
            const bool last = (i == R);
            bool any_last = false;
#pragma unroll
            for (int k = 0; k < G; ++k) any_last |= (__builtin_amdgcn_readlane(Sg, k * W) == s + 1);
            if (any_last)
                run_stripe<T, W, true>(ring, hw, nwpad, rc, l, nsteps, H, last, pm, px, my, yy,
                                       mm1, g1, mx1, xx1, sumM, sumX);
            else
                run_stripe<T, W, false>(ring, hw, nwpad, rc, l, nsteps, H, last, pm, px, my, yy,
                                        mm1, g1, mx1, xx1, sumM, sumX);
        }
        // Result: Σ_j M[R][j] + Σ_j X[R][j] (avx-pairhmm-template.h:341-343).
        if (active && l == (R - 1) % W) {
            const T raw = sumM + sumX;
            static_cast<T*>(a.raw_out)[pid] = raw;
            if constexpr (sizeof(T) == 4) {
                const bool resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
                a.rescue_flag[pid] = resc;
                a.raw64_zero[pid] = 0.0;
                if (resc) {
                    const int pos = atomicAdd(a.rescue_count, 1);
                    a.rescue_list[pos] = pid;
                    a.rescue_rh[pos] = pack_rh(R, H);
                }
            }
        }
        __syncthreads();   // ring reuse by the next pair group of this wave
    }
}

template <typename T>
hipError_t launch_diag(int W, const DiagArgs& a, int grid, hipStream_t s)
{
    const size_t lds = diag_lds_bytes(W, a.ring_len, sizeof(T) == 8);
    if (a.ring_global) {
        grid = grid < kDiagRingBlocks ? grid : kDiagRingBlocks;
        switch (W) {
        case 16: hipLaunchKernelGGL((phmm_diag_kernel<T, 16, true>), dim3(grid), dim3(64), 0, s, a); break;
        case 32: hipLaunchKernelGGL((phmm_diag_kernel<T, 32, true>), dim3(grid), dim3(64), 0, s, a); break;
        case 64: hipLaunchKernelGGL((phmm_diag_kernel<T, 64, true>), dim3(grid), dim3(64), 0, s, a); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (lds > kDiagLdsMax) return hipErrorInvalidValue;
    switch (W) {
    case 16: hipLaunchKernelGGL((phmm_diag_kernel<T, 16, false>), dim3(grid), dim3(64), lds, s, a); break;
    case 32: hipLaunchKernelGGL((phmm_diag_kernel<T, 32, false>), dim3(grid), dim3(64), lds, s, a); break;
    case 64: hipLaunchKernelGGL((phmm_diag_kernel<T, 64, false>), dim3(grid), dim3(64), lds, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

size_t diag_lds_bytes(int W, int ring_len, bool f64)
{
    return size_t(64 / W) * size_t(ring_len) * (f64 ? 16 : 8);
}

hipError_t launch_diag_f32(int W, const DiagArgs& a, int grid, hipStream_t s)
{
    return launch_diag<float>(W, a, grid, s);
}

hipError_t launch_diag_f64(int W, const DiagArgs& a, int grid, hipStream_t s)
{
    return launch_diag<double>(W, a, grid, s);
}

hipError_t configure_kernels()
{
    const int lim = 160 * 1024;
    hipError_t e = hipSuccess;
#define HC_SET(T, W)                                                                        \
    if (e == hipSuccess)                                                                    \
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&phmm_diag_kernel<T, W, false>), \
                                hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    HC_SET(float, 16) HC_SET(float, 32) HC_SET(float, 64)
    HC_SET(double, 16) HC_SET(double, 32) HC_SET(double, 64)
#undef HC_SET
    return e;
}

}  // namespace hcphmm
