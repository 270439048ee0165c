// Lane-per-pair PairHMM kernel for large batches (gfx950, fp32 pass).
//
// Same semantics as the anti-diagonal kernel (kernels.hip) and the reference's
// compute_full_prob_avxs (avx-pairhmm-template.h:210-346), bit for bit, but the
// parallelism is across pairs instead of inside one: each lane owns one
// (read, hap) pair and walks its DP matrix row by row over register-resident
// blocks of up to 64 columns. A wave holds 64 pairs binned by (column blocks,
// R), so its lanes run the same trip counts. Nothing crosses lanes: no DPP
// shifts, no fill/drain of anti-diagonals, no LDS — 12 mul/add + 2 select ops
// per cell.
//
// Per column j of the block the lane keeps two values between rows
//   T[j] = (M*mm + X*gapm) + Y*gapm of the previous row (row i's constants),
//          i.e. the diagonal term of M[i][j+1] before the prior
//   X[j] = X[i][j], computed one row early as M[i-1][j]*mx + X[i-1][j]*xx
// and the horizontal Y recurrence runs along the row. Between column blocks
// the lane hands {T of the block's last column, Y of the next block's first
// column} per row through a global carry buffer (coalesced: [row][lane]).
#include <type_traits>

#include "device_common.hpp"
#include "kernels.hpp"
#include "luts.hpp"

namespace hcphmm {
namespace {

struct RowConst {
    float pm, px;        // prior: 1 - ph2pr[q], ph2pr[q] / 3          (this row)
    float my, yy;        // Y transitions: ph2pr[d], ph2pr[c]           (this row)
    float mm, g, mx, xx; // transitions into the NEXT row: mm, 1 - ph2pr[c], ph2pr[i], ph2pr[c]
    int rc;              // read base code of this row
};

__device__ __forceinline__ void row_const(const float* __restrict__ lut, uint32_t wc, uint32_t wn,
                                          RowConst& k)
{
    const float* __restrict__ ph2pr = lut + kOffPh2pr;
    k.pm = lut[kOffPm + row_q(wc)];
    k.px = lut[kOffPx + row_q(wc)];
    k.my = ph2pr[row_d(wc)];
    k.yy = ph2pr[row_c(wc)];
    k.mm = lut[kOffMM + mm_idx(row_i(wn), row_d(wn))];
    k.g = lut[kOffGapm + row_c(wn)];
    k.mx = ph2pr[row_i(wn)];
    k.xx = ph2pr[row_c(wn)];
    k.rc = row_rc(wc);
}

// Match-bit words of this row's read code for the block's 64 columns.
__device__ __forceinline__ void select_mask(const uint32_t (&m)[10], int rc, uint32_t& lo, uint32_t& hi)
{
    lo = m[0];
    hi = m[1];
#pragma unroll
    for (int c = 1; c < 5; ++c) {
        lo = (rc == c) ? m[2 * c] : lo;
        hi = (rc == c) ? m[2 * c + 1] : hi;
    }
}

// Prior of column bit `B` (MSB-first) of the row's match word: 2 VALU ops,
// v_bfe_i32 (bit -> 0 / -1) and v_bfi_b32 (select pm / px bits). The asm keeps
// the compiler from turning it into and + cmp + cndmask (3 ops + s_nop).
template <int B>
__device__ __forceinline__ float prior_of(uint32_t w, int pmi, int pxi)
{
    int t;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(t) : "v"(w), "i"(B));
    return __int_as_float((t & pmi) | (~t & pxi));
}

struct RowIO {
    float Tdiag;   // in: T of the previous row at column c0 (block-local column -1)
    float Yfirst;  // in: Y of this row at the block's first column
    float Tout;    // out: T of this row at the block's last column
    float Yout;    // out: Y of this row at the column after the block
};

// Column J of one row of one block; recursion unrolls the row at compile time.
template <int J, int NC, bool SUM>
__device__ __forceinline__ void cell(float (&T)[kLaneBlock], float (&X)[kLaneBlock], float& Tdiag,
                                     float& Ml, float& Yl, uint32_t mlo, uint32_t mhi, int pmi, int pxi,
                                     const RowConst& k, int lim, float& sumM, float& sumX)
{
    if constexpr (J < NC) {
        const float prior = prior_of<31 - (J & 31)>(J < 32 ? mlo : mhi, pmi, pxi);
        const float M = Tdiag * prior;
        Tdiag = T[J];
        const float Xc = X[J];
        const float Y = (J == 0) ? Yl : (Ml * k.my + Yl * k.yy);
        T[J] = (M * k.mm + Xc * k.g) + Y * k.g;
        X[J] = M * k.mx + Xc * k.xx;
        if constexpr (SUM) {
            const bool c = J < lim;   // column c0+J+1 <= H on the lane's last row
            sumM = sumM + (c ? M : 0.f);
            sumX = sumX + (c ? Xc : 0.f);
        }
        Ml = M;
        Yl = Y;
        cell<J + 1, NC, SUM>(T, X, Tdiag, Ml, Yl, mlo, mhi, pmi, pxi, k, lim, sumM, sumX);
    }
}

// One row of one column block (columns c0+1 .. c0+NC).
template <int NC, bool SUM>
__device__ __forceinline__ void block_row(float (&T)[kLaneBlock], float (&X)[kLaneBlock], RowIO& io,
                                          uint32_t mlo, uint32_t mhi, const RowConst& k, int lim,
                                          float& sumM, float& sumX)
{
    float Tdiag = io.Tdiag, Ml = 0.f, Yl = io.Yfirst;
    cell<0, NC, SUM>(T, X, Tdiag, Ml, Yl, mlo, mhi, __float_as_int(k.pm), __float_as_int(k.px), k, lim,
                     sumM, sumX);
    io.Tout = T[NC - 1];
    io.Yout = Ml * k.my + Yl * k.yy;
}

template <int NC>
__device__ __forceinline__ void run_block(const LaneArgs& a, const LaneWave& wv, int lane, int b, int nb,
                                          const uint32_t* __restrict__ rrow, const uint32_t* __restrict__ hw,
                                          int R, int H, float T0, float& sumM, float& sumX)
{
    const int c0 = b * kLaneBlock;
    // Match words of all 5 read codes for this block (rows of 5 words, MSB first).
    const int nwpad = (H + 31) / 32 + kHapLead;
    const int w0 = min(c0 / 32 + kHapLead, nwpad), w1 = min(c0 / 32 + kHapLead + 1, nwpad);
    uint32_t m[10];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        m[2 * c] = hw[w0 * 5 + c];
        m[2 * c + 1] = hw[w1 * 5 + c];
    }
    float T[kLaneBlock], X[kLaneBlock];
#pragma unroll
    for (int j = 0; j < kLaneBlock; ++j) {
        T[j] = T0;    // row 0: (0*mm + 0*gapm) + (INITIAL/H)*gapm, every column
        X[j] = 0.f;   // X[1][j] = 0*mx + 0*xx
    }
    float2* __restrict__ carry = a.carry + size_t(wv.carry_row) * 64 + lane;
    const bool has_in = b > 0, has_out = b + 1 < nb;
    // Row 1's diagonal at column c0-1 is row 0's T (c0 = 0: column 0 of row 0, same value).
    float Tdiag = T0;
    uint32_t wc = rrow[0];
    uint32_t wn = rrow[min(2, R) - 1];
    float2 cin = has_in ? carry[64] : make_float2(0.f, 0.f);
    // Rows before any lane's last row run without the sum; from wv.rmin on, the
    // lanes whose row == R accumulate Σ M[R][j] and Σ X[R][j] (j ascending).
    auto row = [&](int i, auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        RowConst k;
        row_const(a.lut, wc, wn, k);
        const uint32_t wnn = rrow[min(i + 2, R) - 1];
        const float2 cnext = (has_in && i < wv.rmax) ? carry[size_t(i + 1) * 64] : make_float2(0.f, 0.f);
        uint32_t mlo, mhi;
        select_mask(m, k.rc, mlo, mhi);
        RowIO io;
        io.Tdiag = Tdiag;
        io.Yfirst = cin.y;   // block 0: Y[i][1] = 0*my + 0*yy = 0
        const int lim = (SUM && i == R) ? H - c0 : 0;
        block_row<NC, SUM>(T, X, io, mlo, mhi, k, lim, sumM, sumX);
        if (has_out) carry[size_t(i) * 64] = make_float2(io.Tout, io.Yout);
        // next row's diagonal at column c0: this row's T there (block 0: column 0 -> 0)
        Tdiag = has_in ? cin.x : 0.f;
        cin = cnext;
        wc = wn;
        wn = wnn;
    };
    int i = 1;
    for (; i < wv.rmin; ++i) row(i, std::false_type{});
    for (; i <= wv.rmax; ++i) row(i, std::true_type{});
}

__global__ __launch_bounds__(256) void phmm_lane_kernel(LaneArgs a)
{
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= a.n_waves) return;
    const int lane = threadIdx.x & 63;
    // Wave metadata is wave-uniform: pin it to SGPRs so loops and the tail switch
    // are scalar branches.
    LaneWave wv;
    {
        const LaneWave w = a.waves[wid];
        wv.slot0 = __builtin_amdgcn_readfirstlane(w.slot0);
        wv.rmax = __builtin_amdgcn_readfirstlane(w.rmax);
        wv.rmin = __builtin_amdgcn_readfirstlane(w.rmin);
        wv.ncols = __builtin_amdgcn_readfirstlane(w.ncols);
        const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(w.carry_row & 0xffffffffll));
        const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(w.carry_row >> 32));
        wv.carry_row = (long long)(((unsigned long long)hi << 32) | lo);
    }
    const int slot = wv.slot0 + lane;
    const bool active = slot < a.n_slots;
    const int pid = a.order[active ? slot : wv.slot0];
    const PairDesc pd = a.pairs[pid];
    const int R = pd.y, H = pd.w;
    const uint32_t* __restrict__ rrow = a.rows + pd.x;
    const uint32_t* __restrict__ hw = a.hapw + pd.z;

    float T0;
    {
        const uint32_t w1 = rrow[0];
        const float mm1 = a.lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
        const float g1 = a.lut[kOffGapm + row_c(w1)];
        const float initY = 0x1p120f / float(H);
        T0 = (0.f * mm1 + 0.f * g1) + initY * g1;
    }
    float sumM = 0.f, sumX = 0.f;
    const int nb = (wv.ncols + kLaneBlock - 1) / kLaneBlock;
    const int tail = wv.ncols - (nb - 1) * kLaneBlock;   // 16, 32, 48 or 64
    for (int b = 0; b + 1 < nb; ++b)
        run_block<64>(a, wv, lane, b, nb, rrow, hw, R, H, T0, sumM, sumX);
    switch (tail) {
    case 16: run_block<16>(a, wv, lane, nb - 1, nb, rrow, hw, R, H, T0, sumM, sumX); break;
    case 32: run_block<32>(a, wv, lane, nb - 1, nb, rrow, hw, R, H, T0, sumM, sumX); break;
    case 48: run_block<48>(a, wv, lane, nb - 1, nb, rrow, hw, R, H, T0, sumM, sumX); break;
    default: run_block<64>(a, wv, lane, nb - 1, nb, rrow, hw, R, H, T0, sumM, sumX); break;
    }
    if (active) {
        const float raw = sumM + sumX;
        a.raw_out[pid] = raw;
        const bool resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
        a.rescue_flag[pid] = resc;
        if (resc) a.rescue_list[atomicAdd(a.rescue_count, 1)] = pid;
    }
}

}  // namespace

hipError_t launch_lane_f32(const LaneArgs& a, hipStream_t s)
{
    if (a.n_waves <= 0) return hipSuccess;
    const int grid = (a.n_waves + 3) / 4;
    hipLaunchKernelGGL(phmm_lane_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
