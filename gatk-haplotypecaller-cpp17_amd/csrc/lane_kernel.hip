// Lane-parallel PairHMM kernels for gfx950: the recurrence runs along rows of
// register-resident column blocks, one lane per block.
//
// Same semantics as the anti-diagonal kernel (kernels.hip) and the reference's
// compute_full_prob_avx{s,d} (avx-pairhmm-template.h:210-346), bit for bit.
// Per column j of a block the lane keeps two values between rows
//   T[j] = (M*mm + X*gapm) + Y*gapm of the previous row (row i's constants),
//          i.e. the diagonal term of M[i][j+1] before the prior
//   X[j] = X[i][j], computed one row early as M[i-1][j]*mx + X[i-1][j]*xx
// and the horizontal Y recurrence runs along the row: the reference's
// operations in the reference's order, evaluated one row earlier.
//
// Three kernels:
//   phmm_seg_kernel   (fp32)  column-segmented waves planned on the host: a pair
//                             over ceil(H/BC) consecutive lanes, one row of skew
//                             per lane, values handed right by DPP (run_seg);
//   phmm_seg64_kernel (fp64)  the rescue pass in the same form, planned on the
//                             device from the rescue list (rescue_plan_kernel);
//   phmm_lane_kernel  (fp32)  one lane per pair, blocks chained through a
//                             global carry buffer (haps too long to segment).
#include <type_traits>

#include "device_common.hpp"
#include "kernels.hpp"
#include "luts.hpp"

namespace hcphmm {
namespace {

template <typename T> __device__ __forceinline__ T initial_value();
template <> __device__ __forceinline__ float initial_value<float>() { return 0x1p120f; }    // Context.h:149
template <> __device__ __forceinline__ double initial_value<double>() { return 0x1p1020; }  // Context.h:109

template <typename T>
struct RowConst {
    T pm, px;        // prior: 1 - ph2pr[q], ph2pr[q] / 3          (this row)
    T my, yy;        // Y transitions: ph2pr[d], ph2pr[c]           (this row)
    T mm, g, mx, xx; // transitions into the NEXT row: mm, 1 - ph2pr[c], ph2pr[i], ph2pr[c]
    int rc;          // read base code of this row
};

// initializeVectors / stripeINITIALIZATION (avx-pairhmm-template.h:83-177):
// wc = this row's packed word, wn = the next row's.
template <typename T>
__device__ __forceinline__ void row_const(const T* __restrict__ lut, uint32_t wc, uint32_t wn, RowConst<T>& k)
{
    const T* __restrict__ ph2pr = lut + kOffPh2pr;
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

// Prior of column bit `B` (MSB-first) of a match word: v_bfe_i32 (bit -> 0 /
// -1) and one bit-select per 32-bit half (v_bitop3). The asm keeps the
// compiler from turning it into and + cmp + cndmask.
template <int B>
__device__ __forceinline__ float prior_of(uint32_t w, float pm, float px)
{
    int t;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(t) : "v"(w), "i"(B));
    return __int_as_float((t & __float_as_int(pm)) | (~t & __float_as_int(px)));
}
template <int B>
__device__ __forceinline__ double prior_of(uint32_t w, double pm, double px)
{
    int t;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(t) : "v"(w), "i"(B));
    const long long a = __double_as_longlong(pm), b = __double_as_longlong(px);
    const unsigned lo = unsigned((t & int(a)) | (~t & int(b)));
    const unsigned hi = unsigned((t & int(a >> 32)) | (~t & int(b >> 32)));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Column J of one row of one block; recursion unrolls the row at compile time.
// M enters as M[i][c0+J+1] (= T_old[J-1] * prior). Before T[J] is overwritten,
// its old value (the next column's diagonal) is consumed into the next M, so
// the new T[J] can take the old one's register: no copies between rows.
// mw0/mw1: the row's match words for block columns 1-32 / 33-64.
// EQ: mx == my bitwise (insertion and deletion gap qualities equal on every
// row: the reference's SAMRecord passes 'I' for both, sam.hpp:30-32), so the
// product M*mx that feeds X[J] is also the M*my term of the next column's Y:
// one multiply fewer per cell, the same rounded values. Ml then carries that
// product instead of M.
template <typename T, int BC, int J, int NC, bool SUM, bool EQ>
__device__ __forceinline__ void cell(T (&Tt)[BC], T (&X)[BC], T M, T& Ml, T& Yl, uint32_t mw0, uint32_t mw1,
                                     T pm, T px, const RowConst<T>& k, int lim, T& sumM, T& sumX)
{
    if constexpr (J < NC) {
        T Mn = M;
        if constexpr (J + 1 < NC)
            Mn = Tt[J] * prior_of<31 - ((J + 1) & 31)>(((J + 1) >> 5) ? mw1 : mw0, pm, px);
        const T Xc = X[J];
        T Y;
        if constexpr (EQ) {
            const T Mx = M * k.mx;
            Y = (J == 0) ? Yl : (Ml + Yl * k.yy);
            Tt[J] = (M * k.mm + Xc * k.g) + Y * k.g;
            X[J] = Mx + Xc * k.xx;
            Ml = Mx;
        } else {
            Y = (J == 0) ? Yl : (Ml * k.my + Yl * k.yy);
            Tt[J] = (M * k.mm + Xc * k.g) + Y * k.g;
            X[J] = M * k.mx + Xc * k.xx;
            Ml = M;
        }
        if constexpr (SUM) {
            const bool c = J < lim;   // column c0+J+1 <= H on the pair's last row
            sumM = sumM + (c ? M : T(0));
            sumX = sumX + (c ? Xc : T(0));
        }
        Yl = Y;
        cell<T, BC, J + 1, NC, SUM, EQ>(Tt, X, Mn, Ml, Yl, mw0, mw1, pm, px, k, lim, sumM, sumX);
    }
}

// Y entering the column after the last one of a row segment: Ml*my + Yl*yy
// (EQ: Ml already holds M*mx = M*my).
template <bool EQ, typename T>
__device__ __forceinline__ T y_next(T Ml, T Yl, T my, T yy)
{
    if constexpr (EQ)
        return Ml + Yl * yy;
    else
        return Ml * my + Yl * yy;
}

struct LaneCtx {
    const uint32_t* rrow;   // the read's packed rows
    const uint32_t* hw;     // the hap's match table
    int R, H;
};

// Row-0 diagonal T0 = (0*mm + 0*gapm) + (INITIAL/H)*gapm with row 1's
// constants (avx-pairhmm-template.h:160-166: Y[0][j] = INITIAL / H).
template <typename T>
__device__ __forceinline__ T row0_t(const T* __restrict__ lut, uint32_t w1, int H)
{
    const T mm1 = lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
    const T g1 = lut[kOffGapm + row_c(w1)];
    const T initY = initial_value<T>() / T(H);
    return (T(0) * mm1 + T(0) * g1) + initY * g1;
}

__device__ __forceinline__ LaneCtx pair_ctx(const PairDesc* pairs, const uint32_t* rows, const uint32_t* hapw,
                                            int pid)
{
    const PairDesc pd = pairs[pid];
    return LaneCtx{rows + pd.x, hapw + pd.z, pd.y, pd.w};
}

// Constant-gap tag of a read: bit 31 of its first row word (pack_reads_kernel).
// EQ additionally needs insertion == deletion gap quality.
__device__ __forceinline__ bool read_cg(uint32_t w1) { return (w1 >> 31) != 0; }
__device__ __forceinline__ bool read_eq(uint32_t w1) { return read_cg(w1) && row_i(w1) == row_d(w1); }

// ---------------------------------------------------------------------------
// One lane per pair, column blocks of BC chained through the carry buffer.

// One register block of columns c0+1 .. c0+NC for all rows of the wave.
// CG: every pair of the wave has constant gap qualities, so the six
// transition constants are per-lane registers and a row only needs its prior
// (pm, px from q) and match word; those are fetched one row ahead.
// mt: this wave's LDS match table [5 read codes][64 lanes] of 2 words.
template <int BC, int NC, bool CG, bool EQ>
__device__ __forceinline__ void run_block(const LaneArgs& a, const LaneWave& wv, int lane, int b, int nb,
                                          const LaneCtx& cx, float T0, float& sumM, float& sumX,
                                          uint2* __restrict__ mt)
{
    const int c0 = b * BC;
    {   // match words of all 5 read codes for this block (MSB first) into LDS
        const int nwpad = (cx.H + 31) / 32 + kHapLead;
        const int w0 = min(c0 / 32 + kHapLead, nwpad), w1 = min(c0 / 32 + kHapLead + 1, nwpad);
#pragma unroll
        for (int c = 0; c < 5; ++c)
            mt[c * 64 + lane] = make_uint2(cx.hw[w0 * 5 + c], (BC > 32) ? cx.hw[w1 * 5 + c] : 0u);
    }
    float T[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        T[j] = T0;   // row 0: (0*mm + 0*gapm) + (INITIAL/H)*gapm, every column
        X[j] = 0.f;  // X[1][j] = 0*mx + 0*xx
    }
    float2* __restrict__ carry = a.carry + size_t(wv.carry_row) * 64 + lane;
    const bool has_in = b > 0, has_out = b + 1 < nb;
    // Row 1's diagonal at column c0 is row 0's T (c0 = 0: column 0 of row 0, same value).
    float Tdiag = T0;
    uint32_t wc = cx.rrow[0], wn = cx.rrow[min(2, cx.R) - 1];
    const float2 zero = make_float2(0.f, 0.f);
    float2 cin = has_in ? carry[64] : zero;   // {T, Y} of the block to the left, row 1
    RowConst<float> k;
    row_const<float>(a.lut, wc, wn, k);   // CG: the transition constants of every row
    uint2 mrow = mt[k.rc * 64 + lane];
    // Rows before any pair's last row run without the sum; from wv.rmin on, the
    // pairs whose row == R accumulate Σ M[R][j] and Σ X[R][j] (j ascending).
    auto row = [&](int i, auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        if constexpr (!CG) {
            row_const<float>(a.lut, wc, wn, k);
            mrow = mt[k.rc * 64 + lane];
        }
        const uint32_t wnn = cx.rrow[min(i + 2, cx.R) - 1];
        const float2 cnext = (has_in && i < wv.rmax) ? carry[size_t(i + 1) * 64] : zero;
        float pm_n = 0.f, px_n = 0.f;
        uint2 m_n = mrow;
        if constexpr (CG) {   // next row's prior constants and match words, a row ahead
            pm_n = a.lut[kOffPm + row_q(wn)];
            px_n = a.lut[kOffPx + row_q(wn)];
            m_n = mt[row_rc(wn) * 64 + lane];
        }
        const int lim = (SUM && i == cx.R) ? cx.H - c0 : 0;
        float Ml = 0.f, Yl = cin.y;   // block 0: Y[i][1] = 0*my + 0*yy = 0
        const float M0 = Tdiag * prior_of<31>(mrow.x, k.pm, k.px);
        cell<float, BC, 0, NC, SUM, EQ>(T, X, M0, Ml, Yl, mrow.x, mrow.y, k.pm, k.px, k, lim, sumM, sumX);
        if (has_out) carry[size_t(i) * 64] = make_float2(T[NC - 1], y_next<EQ>(Ml, Yl, k.my, k.yy));
        // next row's diagonal at column c0: this row's T there (block 0: column 0 -> 0)
        Tdiag = has_in ? cin.x : 0.f;
        cin = cnext;
        if constexpr (CG) {
            k.pm = pm_n;
            k.px = px_n;
            mrow = m_n;
        }
        wc = wn;
        wn = wnn;
    };
    int i = 1;
    for (; i < wv.rmin; ++i) row(i, std::false_type{});
    for (; i <= wv.rmax; ++i) row(i, std::true_type{});
}

template <int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_pairs(const LaneArgs& a, const LaneWave& wv, int lane, const LaneCtx& cx,
                                          float T0, float& sumM, float& sumX, uint2* __restrict__ mt)
{
    const int nb = (wv.ncols + BC - 1) / BC;
    const int tail = wv.ncols - (nb - 1) * BC;   // multiple of 16, <= BC
    for (int b = 0; b + 1 < nb; ++b) run_block<BC, BC, CG, EQ>(a, wv, lane, b, nb, cx, T0, sumM, sumX, mt);
    if (tail == 16) run_block<BC, 16, CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
    else if (BC >= 32 && tail == 32) run_block<BC, (BC >= 32 ? 32 : 16), CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
    else if (BC >= 64 && tail == 48) run_block<BC, (BC >= 64 ? 48 : 16), CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
    else run_block<BC, BC, CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
}

// ---------------------------------------------------------------------------
// Column-segmented waves.

__device__ __forceinline__ float from_left(float v)
{
    // DPP wave_shr:1: lane l receives lane l-1's v (lane 0 receives 0).
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ double from_left(double v)
{
    const long long x = __double_as_longlong(v);
    const unsigned lo = unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x138, 0xf, 0xf, false));
    const unsigned hi = unsigned(__builtin_amdgcn_update_dpp(0, int(x >> 32), 0x138, 0xf, 0xf, false));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Step bounds of a column-segmented wave (wave-uniform).
struct SegSteps {
    int rmax;     // rows swept by every lane
    int rmin;     // first step that may need the row sums
    int nsteps;   // max over the wave's pairs of R + nb - 1
};

// A pair's nb column blocks of BC columns sit on nb consecutive lanes (a
// "group"), lane s of the group owning columns s*BC+1 .. s*BC+BC on every row,
// and lane s sweeps row i = k - s in step k — a one-row skew per block — so the
// pair finishes in R + nb - 1 steps, with no carry buffer. Each step lane s
// takes from lane s-1 (DPP wave_shr:1; ignored on a group's first lane):
//   - the Y entering its first column on row i (lane s-1's row i, last step),
//   - the right-edge T of row i-1, its first diagonal (two steps back: held
//     one step in a register),
//   - on row R, the running sums ΣM, ΣX, so the final sums are accumulated
//     column by column left to right exactly as the reference does.
// Lanes outside 1 <= i <= rmax (pipeline fill / drain) are masked off; columns
// past H compute values that only flow right and are never summed.
// Rows of read words a lane keeps in flight (loaded PD steps before use). A
// lone step of a narrow block is too short to cover a global load, so narrow
// blocks prefetch deeper; the step loop is unrolled by PD so every word lands
// in its own register and is not touched (no wait) until its step.
#ifndef HC_SEG_DEEP
#define HC_SEG_DEEP 1   // 0: one-step prefetch everywhere, prior tables read from global memory (A/B builds)
#endif
template <typename T, int BC>
constexpr int seg_prefetch()
{
    if (!HC_SEG_DEEP) return 1;
    return sizeof(T) == 8 ? (BC >= 16 ? 1 : 2) : (BC >= 32 ? 1 : (BC >= 16 ? 2 : 4));
}

// Call f(integral_constant<P>) for P = 0 .. N-1 (compile-time phases).
template <int P, int N, typename F>
__device__ __forceinline__ void for_phases(F&& f)
{
    if constexpr (P < N) {
        f(std::integral_constant<int, P>{});
        for_phases<P + 1, N>(f);
    }
}

template <typename T, int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_seg(const T* __restrict__ lut, const T* __restrict__ slut, const SegSteps& st,
                                        int lane, int s, const LaneCtx& cx, T T0, T& sumM, T& sumX,
                                        uint2* __restrict__ mt)
{
    constexpr int PD = seg_prefetch<T, BC>();
    const int c0 = s * BC;
    const int R = cx.R;
    {   // this lane's BC-column window of the match table, fixed for the sweep:
        // columns c0+1 .. c0+BC start at bit 31-r of table row c0/32+lead
        const int nwpad = (cx.H + 31) / 32 + kHapLead;   // the trailing zero row
        const int w0 = c0 / 32 + kHapLead, r = c0 & 31;
        const int i0 = min(w0, nwpad), i1 = min(w0 + 1, nwpad), i2 = min(w0 + 2, nwpad);
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const uint64_t x01 = (uint64_t(cx.hw[i0 * 5 + c]) << 32) | cx.hw[i1 * 5 + c];
            const uint64_t x12 = (uint64_t(cx.hw[i1 * 5 + c]) << 32) | cx.hw[i2 * 5 + c];
            mt[c * 64 + lane] = make_uint2(uint32_t((x01 << r) >> 32), uint32_t((x12 << r) >> 32));
        }
    }
    T Tt[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        Tt[j] = T0;   // row 0
        X[j] = T(0);
    }
    // wq[P]: the word of row i+1 (clamped to 1..R) at the steps of phase
    // P = (k-1) mod PD, for every lane at every step; the loads are issued
    // unconditionally so that each path has the same outstanding loads and
    // the wait for a word is the one PD steps after its load.
    uint32_t wc = cx.rrow[0];
    uint32_t wq[PD];
#pragma unroll
    for (int P = 0; P < PD; ++P) wq[P] = cx.rrow[min(max(P + 2 - s, 1), R) - 1];
    RowConst<T> k;
    row_const<T>(lut, wc, cx.rrow[min(2, R) - 1], k);
    uint2 mrow = mt[k.rc * 64 + lane];
    T y_out = T(0), t_out = T(0);   // handed to lane s+1: Y past column c0+BC, T[BC-1] of the last row
    T t_hold = T(0);                // lane s-1's right-edge T of the previous row
    const int lim0 = cx.H - c0;     // columns of this block inside the hap (<= 0: none)
    auto step = [&](int kk, auto sum_tag, auto ph_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        constexpr int P = decltype(ph_tag)::value;
        const int i = kk - s;
        const uint32_t wn = wq[P];   // row i+1, loaded PD steps ago
        T pm_n = T(0), px_n = T(0);
        uint2 m_n = mrow;
        int ridx = min(max(i + PD + 1, 1), R) - 1;   // the word needed PD steps from now
        if constexpr (CG) {   // next row's prior constants (LDS) and match words
            const int qo = row_q(wn), mo = row_rc(wn) * 64 + lane;
            // Order the load after the last use of wn, so the word can land in
            // wn's register (no register move, hence no wait, at the loop back edge).
            asm volatile("" : "+v"(ridx) : "v"(qo), "v"(mo));
            const T* __restrict__ pl = HC_SEG_DEEP ? slut : lut;
            pm_n = pl[kOffPm + qo];
            px_n = pl[kOffPx + qo];
            m_n = mt[mo];
        } else {
            asm volatile("" : "+v"(ridx) : "v"(wn));
        }
        wq[P] = cx.rrow[ridx];
        const T y_in = from_left(y_out);
        const T t_in = from_left(t_out);
        T sM_in = T(0), sX_in = T(0);
        if constexpr (SUM) {
            sM_in = from_left(sumM);
            sX_in = from_left(sumX);
        }
        // Row 1's diagonal is row 0's T at every column; below that, lane
        // s-1's right edge (column 0 for block 0: T[i][0] = 0 for i >= 1).
        const T Tdiag = i == 1 ? T0 : (s ? t_hold : T(0));
        const T Yl0 = s ? y_in : T(0);   // block 0: Y[i][1] = 0*my + 0*yy = 0
        t_hold = t_in;
        if (unsigned(i - 1) < unsigned(st.rmax)) {
            if constexpr (!CG) {
                row_const<T>(lut, wc, wn, k);
                mrow = mt[k.rc * 64 + lane];
            }
            const bool last = SUM && i == R;
            const int lim = last ? lim0 : 0;
            if (last) {
                sumM = s ? sM_in : T(0);
                sumX = s ? sX_in : T(0);
            }
            T Ml = T(0), Yl = Yl0;
            const T M0 = Tdiag * prior_of<31>(mrow.x, k.pm, k.px);
            cell<T, BC, 0, BC, SUM, EQ>(Tt, X, M0, Ml, Yl, mrow.x, mrow.y, k.pm, k.px, k, lim, sumM, sumX);
            y_out = y_next<EQ>(Ml, Yl, k.my, k.yy);
            t_out = Tt[BC - 1];
            if constexpr (CG) {
                k.pm = pm_n;
                k.px = px_n;
                mrow = m_n;
            }
        }
        wc = wn;
    };
    // Everything the prologue loaded is in registers before the sweep: the
    // wait-count pass then sees only the sweep's own prefetches in flight and
    // waits on each word exactly PD steps after its load (s_waitcnt vmcnt(0)).
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // Groups of PD steps (phases 0..PD-1); the sum variant from the group that
    // holds step rmin on (extra steps past nsteps find every lane inactive).
    int kk = 1;
    for (; kk + PD - 1 < st.rmin; kk += PD)
        for_phases<0, PD>([&](auto ph) { step(kk + decltype(ph)::value, std::false_type{}, ph); });
    for (; kk <= st.nsteps; kk += PD)
        for_phases<0, PD>([&](auto ph) { step(kk + decltype(ph)::value, std::true_type{}, ph); });
}

// Two compiled paths per width: EQ (the reference's constant 'I'/'I'/'+' gap
// qualities) and the generic per-row path (any gap qualities).
template <typename T, int BC>
__device__ __forceinline__ void run_seg_bc(const T* __restrict__ lut, const T* __restrict__ slut, const SegSteps& st,
                                           int lane, int s, const LaneCtx& cx, T T0, T& sumM, T& sumX,
                                           uint2* __restrict__ mt, bool wave_eq)
{
    if (wave_eq)
        run_seg<T, BC, true, true>(lut, slut, st, lane, s, cx, T0, sumM, sumX, mt);
    else
        run_seg<T, BC, false, false>(lut, slut, st, lane, s, cx, T0, sumM, sumX, mt);
}

// The prior tables [ph2pr | pm | px | gapm] (luts.hpp) in LDS: the per-row
// prior lookups of the segmented kernels read them there.
constexpr int kSlutLen = kOffMM;
template <typename T>
__device__ __forceinline__ void load_slut(T* __restrict__ slut, const T* __restrict__ lut)
{
    for (int t = threadIdx.x; t < kSlutLen; t += blockDim.x) slut[t] = lut[t];
    __syncthreads();
}

// Block widths of fp32 column-segmented waves (LaneWave.ncols of a seg wave).
#define HC_SEG_WIDTHS(X) \
    X(8) X(10) X(12) X(14) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

// Wave metadata is wave-uniform: pin it to SGPRs so loops and switches are
// scalar branches.
__device__ __forceinline__ LaneWave load_wave(const LaneWave* waves, int wid)
{
    LaneWave wv;
    const LaneWave w = waves[wid];
    wv.slot0 = __builtin_amdgcn_readfirstlane(w.slot0);
    wv.rmax = __builtin_amdgcn_readfirstlane(w.rmax);
    wv.rmin = __builtin_amdgcn_readfirstlane(w.rmin);
    wv.ncols = __builtin_amdgcn_readfirstlane(w.ncols);
    wv.npairs = __builtin_amdgcn_readfirstlane(w.npairs);
    wv.nsteps = __builtin_amdgcn_readfirstlane(w.nsteps);
    const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(w.carry_row & 0xffffffffll));
    const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(w.carry_row >> 32));
    wv.carry_row = (long long)(((unsigned long long)hi << 32) | lo);
    return wv;
}

// fp32 pass result of one pair: raw sum, rescue decision (intel_pairhmm.hpp:
// 133-139), the pair's raw f64 slot zeroed (the rescue pass fills rescued ones).
__device__ __forceinline__ void emit(const LaneArgs& a, int pid, float raw)
{
    a.raw_out[pid] = raw;
    const bool resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
    a.rescue_flag[pid] = resc;
    a.raw64_zero[pid] = 0.0;
    if (resc) a.rescue_list[atomicAdd(a.rescue_count, 1)] = pid;
}

// One lane per pair, column blocks of BC with the carry buffer between blocks.
template <int BC, int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_lane_kernel(LaneArgs a)
{
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= a.n_waves) return;
    const int lane = threadIdx.x & 63;
    const LaneWave wv = load_wave(a.waves, wid);
    const int slot = wv.slot0 + lane;
    const bool active = slot < a.n_slots;
    const int pid = a.order[active ? slot : wv.slot0];
    const LaneCtx cx = pair_ctx(a.pairs, a.rows, a.hapw, pid);
    const uint32_t w1 = cx.rrow[0];
    const float T0 = row0_t<float>(a.lut, w1, cx.H);
    const bool wave_cg = __builtin_amdgcn_ballot_w64(!read_cg(w1)) == 0;
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!read_eq(w1)) == 0;
    float sumM = 0.f, sumX = 0.f;
    __shared__ uint2 mtab[4][5 * 64];
    uint2* mt = mtab[threadIdx.x >> 6];
    if (wave_eq)
        run_pairs<BC, true, true>(a, wv, lane, cx, T0, sumM, sumX, mt);
    else if (wave_cg)
        run_pairs<BC, true, false>(a, wv, lane, cx, T0, sumM, sumX, mt);
    else
        run_pairs<BC, false, false>(a, wv, lane, cx, T0, sumM, sumX, mt);
    if (active) emit(a, pid, sumM + sumX);
}

// The fp64 rescue (intel_pairhmm.hpp:137-139) of the pairs this wave's fp32
// pass flagged (`todo`: their owner lanes). A wave with at most two, each with
// H <= kInWaveRescueMaxH, recomputes them itself while the rest of the pass
// runs — one pair at a time over the whole wave (8 columns per lane, the
// same run_seg in double) — so a batch with a few rescues (S2: ~2e-5 of
// the pairs) needs no separate latency-bound pass after the fp32 kernel. The
// others are appended to the rescue list for that pass.
__device__ __forceinline__ void rescue_in_wave(const LaneArgs& a, uint64_t todo, int pid, int lane,
                                            uint2* __restrict__ mt)
{
    const bool few = a.inker_count != nullptr && __popcll(todo) <= 2;
    while (todo) {
        const int l = __builtin_ctzll(todo);
        todo &= todo - 1;
        const int rp = __builtin_amdgcn_readlane(pid, l);
        const PairDesc pd = a.pairs[rp];
        const int R = __builtin_amdgcn_readfirstlane(pd.y), H = __builtin_amdgcn_readfirstlane(pd.w);
        bool here = few && H <= kInWaveRescueMaxH;
        if (here) {
            int c = 0;
            if (lane == 0) c = atomicAdd(a.inker_count, 1);
            here = __builtin_amdgcn_readfirstlane(c) < a.inker_limit;
        }
        if (!here) {
            if (lane == l) a.rescue_list[atomicAdd(a.rescue_count, 1)] = rp;
            continue;
        }
        const LaneCtx cx{a.rows + __builtin_amdgcn_readfirstlane(pd.x), a.hapw + __builtin_amdgcn_readfirstlane(pd.z),
                         R, H};
        const int nb = (H + 7) / 8;
        const SegSteps st{R, R, R + nb - 1};
        const uint32_t w1 = cx.rrow[0];
        const double T0 = row0_t<double>(a.lut64, w1, H);
        const bool eq = read_eq(w1);
        double sM = 0.0, sX = 0.0;
        run_seg_bc<double, 8>(a.lut64, a.lut64, st, lane, lane, cx, T0, sM, sX, mt, eq);
        if (lane == nb - 1) a.raw64_zero[rp] = sM + sX;
        __builtin_amdgcn_wave_barrier();   // the next pair rewrites mt
    }
}

// Column-segmented fp32 waves (host-planned). The wave's npairs pairs are the
// slots slot0 .. slot0+npairs-1; pair g takes nb_g = ceil(H_g / BC) consecutive
// lanes in slot order. Lanes past the last group idle (s = 0, no output).
template <int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_seg_kernel(LaneArgs a)
{
    __shared__ float slut[kSlutLen];
    load_slut(slut, a.lut);
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= a.n_waves) return;
    const int lane = threadIdx.x & 63;
    const LaneWave wv = load_wave(a.waves, wid);
    const int bc = wv.ncols;
    __shared__ uint2 mtab[4][5 * 64];
    uint2* mt = mtab[threadIdx.x >> 6];
    // Lane -> (group, block): group g's lanes start at the prefix sum of nb.
    int* gmap = reinterpret_cast<int*>(mt);   // 128 ints, used before the match table
    int nb_g = 0;
    if (lane < wv.npairs) nb_g = (a.pairs[a.order[wv.slot0 + lane]].w + bc - 1) / bc;
    int start = nb_g;   // inclusive scan of nb over lanes (Hillis-Steele through LDS)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        gmap[lane] = start;
        __builtin_amdgcn_wave_barrier();
        const int v = lane >= d ? gmap[lane - d] : 0;
        __builtin_amdgcn_wave_barrier();
        start += v;
    }
    start -= nb_g;
    gmap[lane] = -1;
    __builtin_amdgcn_wave_barrier();
    if (lane < wv.npairs)
        for (int t = 0; t < nb_g; ++t) {
            gmap[start + t] = lane;
            gmap[64 + start + t] = t;
        }
    __builtin_amdgcn_wave_barrier();
    const int g = gmap[lane];
    int s = gmap[64 + lane];
    __builtin_amdgcn_wave_barrier();
    const int pid = a.order[wv.slot0 + (g >= 0 ? g : 0)];
    const LaneCtx cx = pair_ctx(a.pairs, a.rows, a.hapw, pid);
    const bool owner = g >= 0 && s == (cx.H + bc - 1) / bc - 1;
    if (g < 0) s = 0;
    const uint32_t w1 = cx.rrow[0];
    const float T0 = row0_t<float>(a.lut, w1, cx.H);
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!read_eq(w1)) == 0;
    const SegSteps st{wv.rmax, wv.rmin, wv.nsteps};
    float sumM = 0.f, sumX = 0.f;
    switch (bc) {
#define HC_SEG_CASE(W) \
    case W: run_seg_bc<float, W>(a.lut, slut, st, lane, s, cx, T0, sumM, sumX, mt, wave_eq); break;
        HC_SEG_WIDTHS(HC_SEG_CASE)
#undef HC_SEG_CASE
    default: break;
    }
    // fp32 result and rescue decision (intel_pairhmm.hpp:133-139).
    bool resc = false;
    if (owner) {
        const float raw = sumM + sumX;
        resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
        a.raw_out[pid] = raw;
        a.rescue_flag[pid] = resc;
        if (!resc) a.raw64_zero[pid] = 0.0;
    }
    const uint64_t todo = __builtin_amdgcn_ballot_w64(resc);
    if (todo) rescue_in_wave(a, todo, pid, lane, mt);
}

// ---------------------------------------------------------------------------
// fp64 rescue pass (intel_pairhmm.hpp:137-139) in column-segmented form.
//
// The rescue list is built on the device by the fp32 pass, so the waves are
// planned on the device too: rescue_plan_kernel picks the block width bc[0]
// for the pass (32 columns, narrower when the list is too short to give every
// SIMD two waves: short lists are latency-bound), puts every pair in class k =
// ceil(log2(ceil(H/bc))) — a slot of 2^k lanes, 64/2^k pairs per wave — with
// bc = bc[0], or bc[1] = 32 if that needs more than 64 lanes, and scatters the
// list into class order (order inside a class is arbitrary; each pair's result
// is independent of it). Pairs needing more than 64 lanes at 32 columns go to
// the anti-diagonal fp64 kernel through `big`.

__device__ __forceinline__ int ceil_log2(int nb) { return nb <= 1 ? 0 : 32 - __clz(nb - 1); }

__device__ __forceinline__ int rescue_class(int H, int bc0)
{
    const int nb0 = (H + bc0 - 1) / bc0;
    if (nb0 <= 64) return ceil_log2(nb0);
    const int nb1 = (H + 31) / 32;
    if (nb1 <= 64) return 7 + ceil_log2(nb1);
    return 14;
}

__global__ __launch_bounds__(1024) void rescue_plan_kernel(Seg64Args a)
{
    constexpr int NC = kSeg64Classes;
    __shared__ int cnt[NC], fill[NC];
    __shared__ unsigned long long lanes_sh;
    const int n = *a.count;
    const int t = threadIdx.x;
    if (t < NC) cnt[t] = 0;
    if (t == 0) {
        lanes_sh = 0;
        *a.count_reset = 0;
        *a.inker_reset = 0;
    }
    __syncthreads();
    // Width: 32 unless the lanes at width 32 give fewer than min_lanes
    // (2 waves per SIMD), then 16, then 8.
    unsigned long long mine = 0;
    for (int i = t; i < n; i += blockDim.x) mine += (a.pairs[a.list[i]].w + 31) / 32;
    atomicAdd(&lanes_sh, mine);
    __syncthreads();
    const long long l32 = (long long)lanes_sh;
    const int bc0 = l32 >= a.min_lanes ? 32 : (2 * l32 >= a.min_lanes ? 16 : 8);
    for (int i = t; i < n; i += blockDim.x) atomicAdd(&cnt[rescue_class(a.pairs[a.list[i]].w, bc0)], 1);
    __syncthreads();
    if (t == 0) {
        Seg64Plan p;
        p.bc[0] = bc0;
        p.bc[1] = 32;
        int off = 0, wb = 0;
        for (int c = 0; c < NC; ++c) {
            p.n_class[c] = cnt[c];
            p.off_class[c] = off;
            fill[c] = off;
            off += cnt[c];
            p.wave_base[c] = wb;
            if (c < NC - 1) {
                const int per = 64 >> (c % 7);
                wb += (cnt[c] + per - 1) / per;
            }
        }
        *a.plan = p;
        *a.big_count = cnt[NC - 1];
    }
    __syncthreads();
    for (int i = t; i < n; i += blockDim.x) {
        const int pid = a.list[i];
        const int c = rescue_class(a.pairs[pid].w, bc0);
        const int pos = atomicAdd(&fill[c], 1);
        if (c < NC - 1)
            a.sorted[pos] = pid;
        else
            a.big[pos - (n - cnt[NC - 1])] = pid;
    }
}

// Wave-uniform max / min of a per-lane int (once per wave).
__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_min(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_seg64_kernel(Seg64Args a)
{
    __shared__ uint2 mtab[4][5 * 64];
    __shared__ double slut[kSlutLen];
    load_slut(slut, a.lut);
    uint2* mt = mtab[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    const Seg64Plan* __restrict__ p = a.plan;
    const int total = __builtin_amdgcn_readfirstlane(p->wave_base[kSeg64Classes - 1]);
    for (int w = blockIdx.x * 4 + (threadIdx.x >> 6); w < total; w += gridDim.x * 4) {
        int c = 0;
        while (c < kSeg64Classes - 2 && __builtin_amdgcn_readfirstlane(p->wave_base[c + 1]) <= w) ++c;
        const int k = c % 7;
        const int bc = __builtin_amdgcn_readfirstlane(p->bc[c / 7]);
        const int nk = __builtin_amdgcn_readfirstlane(p->n_class[c]);
        const int ok = __builtin_amdgcn_readfirstlane(p->off_class[c]);
        const int wk = w - __builtin_amdgcn_readfirstlane(p->wave_base[c]);
        const int e = wk * (64 >> k) + (lane >> k);
        const bool valid = e < nk;
        int s = lane & ((1 << k) - 1);
        const int pid = a.sorted[ok + (valid ? e : wk * (64 >> k))];
        const LaneCtx cx = pair_ctx(a.pairs, a.rows, a.hapw, pid);
        const int nb = (cx.H + bc - 1) / bc;
        const bool owner = valid && s == nb - 1;
        if (!valid) s = 0;
        const SegSteps st{wave_max(valid ? cx.R : 0), wave_min(valid ? cx.R : INT32_MAX),
                          wave_max(valid ? cx.R + nb - 1 : 0)};
        const uint32_t w1 = cx.rrow[0];
        const double T0 = row0_t<double>(a.lut, w1, cx.H);
        const bool wave_eq = __builtin_amdgcn_ballot_w64(!read_eq(w1)) == 0;
        double sumM = 0.0, sumX = 0.0;
        switch (bc) {
        case 8: run_seg_bc<double, 8>(a.lut, slut, st, lane, s, cx, T0, sumM, sumX, mt, wave_eq); break;
        case 16: run_seg_bc<double, 16>(a.lut, slut, st, lane, s, cx, T0, sumM, sumX, mt, wave_eq); break;
        default: run_seg_bc<double, 32>(a.lut, slut, st, lane, s, cx, T0, sumM, sumX, mt, wave_eq); break;
        }
        if (owner) a.raw_out[pid] = sumM + sumX;
        __builtin_amdgcn_wave_barrier();   // the next wave's match table reuses mt
    }
}

}  // namespace

// One-lane kernel variants: {pairs per lane, block columns, waves per SIMD}.
// Block widths are multiples of 32 (a block starts on a match-word boundary).
#ifndef HC_SEG_OCC
#define HC_SEG_OCC 3
#endif
constexpr int kSegOcc = HC_SEG_OCC;   // waves per SIMD of the fp32 column-segmented kernel
constexpr int kSeg64Occ = 2;   // fp64: 2 VGPRs per value
static const LaneVariant kVariants[] = {
    {1, 64, 3}, {1, 64, 2}, {1, 32, 4},
};
constexpr int kNumVariants = int(sizeof(kVariants) / sizeof(kVariants[0]));

const LaneVariant& lane_variant(int id)
{
    return kVariants[(id >= 0 && id < kNumVariants) ? id : 0];
}

hipError_t launch_lane_f32(int id, const LaneArgs& a, hipStream_t s)
{
    if (a.n_waves <= 0) return hipSuccess;
    const int grid = (a.n_waves + 3) / 4;
    const dim3 g(grid), blk(256);
    switch ((id >= 0 && id < kNumVariants) ? id : 0) {
    case 1: hipLaunchKernelGGL((phmm_lane_kernel<64, 2>), g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL((phmm_lane_kernel<32, 4>), g, blk, 0, s, a); break;
    default: hipLaunchKernelGGL((phmm_lane_kernel<64, 3>), g, blk, 0, s, a); break;
    }
    return hipGetLastError();
}

bool seg_width_ok(int bc)
{
    switch (bc) {
#define HC_SEG_OK(W) case W:
        HC_SEG_WIDTHS(HC_SEG_OK)
#undef HC_SEG_OK
        return true;
    default: return false;
    }
}

int seg_width_ceil(int bc)
{
    for (int w = bc < kSegMinBC ? kSegMinBC : bc; w <= kSegMaxBC; ++w)
        if (seg_width_ok(w)) return w;
    return -1;
}

hipError_t launch_lane_seg_f32(const LaneArgs& a, hipStream_t s)
{
    if (a.n_waves <= 0) return hipSuccess;
    const int grid = (a.n_waves + 3) / 4;
    hipLaunchKernelGGL((phmm_seg_kernel<kSegOcc>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_rescue_seg64(const Seg64Args& a, int grid, hipStream_t s)
{
    hipLaunchKernelGGL(rescue_plan_kernel, dim3(1), dim3(1024), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((phmm_seg64_kernel<kSeg64Occ>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
