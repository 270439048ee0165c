// Lane-per-pair PairHMM kernel for large batches (gfx950, fp32 pass).
//
// Same semantics as the anti-diagonal kernel (kernels.hip) and the reference's
// compute_full_prob_avxs (avx-pairhmm-template.h:210-346), bit for bit, but the
// parallelism is across pairs instead of inside one: each lane owns P pairs
// (P = 1, or P = 2 held in the .x/.y halves of float2 registers so that every
// mul/add is one packed v_pk_mul_f32 / v_pk_add_f32 for two cells) and walks
// their DP matrices row by row over register-resident column blocks
// (64 columns for P = 1, 32 for P = 2: the same 128 state VGPRs). A wave holds
// 64*P pairs binned by (column blocks, R), so its lanes run the same trip
// counts. Nothing crosses lanes: no DPP shifts, no anti-diagonal fill/drain,
// no LDS — 12 mul/add + 2 select ops per cell.
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

typedef float f2 __attribute__((ext_vector_type(2)));

template <int P> struct VT;
template <> struct VT<1> { using type = float; };
template <> struct VT<2> { using type = f2; };

__device__ __forceinline__ float comp(float v, int) { return v; }
__device__ __forceinline__ float comp(f2 v, int p) { return p ? v.y : v.x; }
__device__ __forceinline__ void set_comp(float& v, int, float s) { v = s; }
__device__ __forceinline__ void set_comp(f2& v, int p, float s)
{
    if (p) v.y = s; else v.x = s;
}
template <typename V> __device__ __forceinline__ V splat(float s) { return V(s); }


template <int P>
struct RowConst {
    using V = typename VT<P>::type;
    V pm, px;        // prior: 1 - ph2pr[q], ph2pr[q] / 3          (this row)
    V my, yy;        // Y transitions: ph2pr[d], ph2pr[c]           (this row)
    V mm, g, mx, xx; // transitions into the NEXT row: mm, 1 - ph2pr[c], ph2pr[i], ph2pr[c]
    int rc[P];       // read base code of this row
};

template <int P>
__device__ __forceinline__ void row_const(const float* __restrict__ lut, const uint32_t (&wc)[P],
                                          const uint32_t (&wn)[P], RowConst<P>& k)
{
    const float* __restrict__ ph2pr = lut + kOffPh2pr;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        set_comp(k.pm, p, lut[kOffPm + row_q(wc[p])]);
        set_comp(k.px, p, lut[kOffPx + row_q(wc[p])]);
        set_comp(k.my, p, ph2pr[row_d(wc[p])]);
        set_comp(k.yy, p, ph2pr[row_c(wc[p])]);
        set_comp(k.mm, p, lut[kOffMM + mm_idx(row_i(wn[p]), row_d(wn[p]))]);
        set_comp(k.g, p, lut[kOffGapm + row_c(wn[p])]);
        set_comp(k.mx, p, ph2pr[row_i(wn[p])]);
        set_comp(k.xx, p, ph2pr[row_c(wn[p])]);
        k.rc[p] = row_rc(wc[p]);
    }
}

// Prior of column bit `B` (MSB-first) of a match word: 2 VALU ops, v_bfe_i32
// (bit -> 0 / -1) and v_bitop3/v_bfi (select pm / px bits). The asm keeps the
// compiler from turning it into and + cmp + cndmask (3 ops + s_nop).
template <int B>
__device__ __forceinline__ float prior_of(uint32_t w, int pmi, int pxi)
{
    int t;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(t) : "v"(w), "i"(B));
    return __int_as_float((t & pmi) | (~t & pxi));
}

template <int P, int J>
__device__ __forceinline__ typename VT<P>::type prior_vec(const uint32_t (&mw)[P][2], const int (&pmi)[P],
                                                       const int (&pxi)[P])
{
    typename VT<P>::type prior;
#pragma unroll
    for (int p = 0; p < P; ++p) set_comp(prior, p, prior_of<31 - (J & 31)>(mw[p][J >> 5], pmi[p], pxi[p]));
    return prior;
}

// Column J of one row of one block; recursion unrolls the row at compile time.
// M enters as M[i][c0+J+1] (= T_old[J-1] * prior). Before T[J] is overwritten,
// its old value (the next column's diagonal) is consumed into the next M, so
// the new T[J] can take the old one's register: no copies between rows.
// mw[p][w]: match words of pair p for this row (w = 0, 1 for 64 columns).
// EQ: mx == my bitwise (insertion and deletion gap qualities equal on every
// row: the reference's SAMRecord passes 'I' for both, sam.hpp:30-32), so the
// product M*mx that feeds X[J] is also the M*my term of the next column's Y:
// one multiply fewer per cell, the same rounded values. Ml then carries that
// product instead of M.
template <int P, int BC, int J, int NC, bool SUM, bool EQ>
__device__ __forceinline__ void cell(typename VT<P>::type (&T)[BC], typename VT<P>::type (&X)[BC],
                                     typename VT<P>::type M, typename VT<P>::type& Ml,
                                     typename VT<P>::type& Yl, const uint32_t (&mw)[P][2],
                                     const int (&pmi)[P], const int (&pxi)[P], const RowConst<P>& k,
                                     const int (&lim)[P], typename VT<P>::type& sumM,
                                     typename VT<P>::type& sumX)
{
    using V = typename VT<P>::type;
    if constexpr (J < NC) {
        V Mn = M;
        if constexpr (J + 1 < NC) Mn = T[J] * prior_vec<P, J + 1>(mw, pmi, pxi);
        const V Xc = X[J];
        V Y, Mx;
        if constexpr (EQ) {
            Mx = M * k.mx;
            Y = (J == 0) ? Yl : (Ml + Yl * k.yy);
        } else {
            Y = (J == 0) ? Yl : (Ml * k.my + Yl * k.yy);
        }
        T[J] = (M * k.mm + Xc * k.g) + Y * k.g;
        if constexpr (EQ)
            X[J] = Mx + Xc * k.xx;
        else
            X[J] = M * k.mx + Xc * k.xx;
        if constexpr (SUM) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const bool c = J < lim[p];   // column c0+J+1 <= H on the pair's last row
                set_comp(sumM, p, comp(sumM, p) + (c ? comp(M, p) : 0.f));
                set_comp(sumX, p, comp(sumX, p) + (c ? comp(Xc, p) : 0.f));
            }
        }
        if constexpr (EQ)
            Ml = Mx;
        else
            Ml = M;
        Yl = Y;
        cell<P, BC, J + 1, NC, SUM, EQ>(T, X, Mn, Ml, Yl, mw, pmi, pxi, k, lim, sumM, sumX);
    }
}

// Y entering the column after the last one of a row segment: Ml*my + Yl*yy
// (EQ: Ml already holds M*mx = M*my).
template <bool EQ, typename V>
__device__ __forceinline__ V y_next(V Ml, V Yl, V my, V yy)
{
    if constexpr (EQ)
        return Ml + Yl * yy;
    else
        return Ml * my + Yl * yy;
}

template <int P>
struct Carry {
    typename VT<P>::type t, y;
};

template <int P>
struct LaneCtx {
    const uint32_t* rrow[P];
    const uint32_t* hw[P];
    int R[P], H[P];
};

// One register block of columns c0+1 .. c0+NC for all rows of the wave.
// CG: every pair of the wave has constant gap qualities (i, d, c identical on
// all rows — what the reference's SAMRecord always supplies, sam.hpp:30-32), so
// the six transition constants are per-lane registers and a row only needs its
// prior (pm, px from q) and match word; those are fetched one row ahead.
// mt: this wave's LDS match table [P][5 read codes][64 lanes] of 2 words.
template <int P, int BC, int NC, bool CG, bool EQ>
__device__ __forceinline__ void run_block(const LaneArgs& a, const LaneWave& wv, int lane, int b, int nb,
                                          const LaneCtx<P>& cx, typename VT<P>::type T0,
                                          typename VT<P>::type& sumM, typename VT<P>::type& sumX,
                                          uint2* __restrict__ mt)
{
    using V = typename VT<P>::type;
    const int c0 = b * BC;
    // Match words of all 5 read codes for this block (rows of 5 words, MSB first)
    // into LDS; each lane later reads only its own entries.
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int nwpad = (cx.H[p] + 31) / 32 + kHapLead;
        const int w0 = min(c0 / 32 + kHapLead, nwpad), w1 = min(c0 / 32 + kHapLead + 1, nwpad);
#pragma unroll
        for (int c = 0; c < 5; ++c)
            mt[(p * 5 + c) * 64 + lane] = make_uint2(cx.hw[p][w0 * 5 + c], (BC > 32) ? cx.hw[p][w1 * 5 + c] : 0u);
    }
    V T[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        T[j] = T0;           // row 0: (0*mm + 0*gapm) + (INITIAL/H)*gapm, every column
        X[j] = splat<V>(0.f);   // X[1][j] = 0*mx + 0*xx
    }
    Carry<P>* __restrict__ carry = reinterpret_cast<Carry<P>*>(a.carry) + size_t(wv.carry_row) * 64 + lane;
    const bool has_in = b > 0, has_out = b + 1 < nb;
    // Row 1's diagonal at column c0 is row 0's T (c0 = 0: column 0 of row 0, same value).
    V Tdiag = T0;
    uint32_t wc[P], wn[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        wc[p] = cx.rrow[p][0];
        wn[p] = cx.rrow[p][min(2, cx.R[p]) - 1];
    }
    const Carry<P> zero{splat<V>(0.f), splat<V>(0.f)};
    Carry<P> cin = has_in ? carry[64] : zero;
    RowConst<P> k;
    row_const<P>(a.lut, wc, wn, k);   // CG: the transition constants of every row
    uint2 mrow[P];                    // this row's match words
#pragma unroll
    for (int p = 0; p < P; ++p) mrow[p] = mt[(p * 5 + k.rc[p]) * 64 + lane];
    // Rows before any pair's last row run without the sum; from wv.rmin on, the
    // pairs whose row == R accumulate Σ M[R][j] and Σ X[R][j] (j ascending).
    auto row = [&](int i, auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        if constexpr (!CG) {
            row_const<P>(a.lut, wc, wn, k);
#pragma unroll
            for (int p = 0; p < P; ++p) mrow[p] = mt[(p * 5 + k.rc[p]) * 64 + lane];
        }
        uint32_t wnn[P];
#pragma unroll
        for (int p = 0; p < P; ++p) wnn[p] = cx.rrow[p][min(i + 2, cx.R[p]) - 1];
        const Carry<P> cnext = (has_in && i < wv.rmax) ? carry[size_t(i + 1) * 64] : zero;
        // CG: next row's prior constants and match words, issued a row ahead.
        V pm_n, px_n;
        uint2 m_n[P];
        if constexpr (CG) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                set_comp(pm_n, p, a.lut[kOffPm + row_q(wn[p])]);
                set_comp(px_n, p, a.lut[kOffPx + row_q(wn[p])]);
                m_n[p] = mt[(p * 5 + row_rc(wn[p])) * 64 + lane];
            }
        }
        uint32_t mw[P][2];
        int pmi[P], pxi[P], lim[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            mw[p][0] = mrow[p].x;
            mw[p][1] = mrow[p].y;
            pmi[p] = __float_as_int(comp(k.pm, p));
            pxi[p] = __float_as_int(comp(k.px, p));
            lim[p] = (SUM && i == cx.R[p]) ? cx.H[p] - c0 : 0;
        }
        V Ml = splat<V>(0.f), Yl = cin.y;   // block 0: Y[i][1] = 0*my + 0*yy = 0
        const V M0 = Tdiag * prior_vec<P, 0>(mw, pmi, pxi);
        cell<P, BC, 0, NC, SUM, EQ>(T, X, M0, Ml, Yl, mw, pmi, pxi, k, lim, sumM, sumX);
        if (has_out) carry[size_t(i) * 64] = Carry<P>{T[NC - 1], y_next<EQ>(Ml, Yl, k.my, k.yy)};
        // next row's diagonal at column c0: this row's T there (block 0: column 0 -> 0)
        Tdiag = has_in ? cin.t : splat<V>(0.f);
        cin = cnext;
        if constexpr (CG) {
            k.pm = pm_n;
            k.px = px_n;
#pragma unroll
            for (int p = 0; p < P; ++p) mrow[p] = m_n[p];
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
            wc[p] = wn[p];
            wn[p] = wnn[p];
        }
    };
    int i = 1;
    for (; i < wv.rmin; ++i) row(i, std::false_type{});
    for (; i <= wv.rmax; ++i) row(i, std::true_type{});
}

template <int P, int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_pairs(const LaneArgs& a, const LaneWave& wv, int lane, const LaneCtx<P>& cx,
                                          typename VT<P>::type T0, typename VT<P>::type& sumM,
                                          typename VT<P>::type& sumX, uint2* __restrict__ mt)
{
    const int nb = (wv.ncols + BC - 1) / BC;
    const int tail = wv.ncols - (nb - 1) * BC;   // multiple of 16, <= BC
    for (int b = 0; b + 1 < nb; ++b) run_block<P, BC, BC, CG, EQ>(a, wv, lane, b, nb, cx, T0, sumM, sumX, mt);
    if (tail == 16) run_block<P, BC, 16, CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
    else if (BC >= 32 && tail == 32) run_block<P, BC, (BC >= 32 ? 32 : 16), CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
    else if (BC >= 64 && tail == 48) run_block<P, BC, (BC >= 64 ? 48 : 16), CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
    else run_block<P, BC, BC, CG, EQ>(a, wv, lane, nb - 1, nb, cx, T0, sumM, sumX, mt);
}

__device__ __forceinline__ float from_left(float v)
{
    // DPP wave_shr:1: lane l receives lane l-1's v (lane 0 receives 0).
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}

// Column-segmented wave: a pair's nb column blocks of BC columns sit on nb
// consecutive lanes (a "group"), lane s of the group owning columns
// s*BC+1 .. s*BC+BC on every row, and lane s sweeps row i = k - s in step k —
// a one-row skew per block — so the pair finishes in R + nb - 1 steps, with no
// carry buffer. Groups of different nb share a wave (the host packs the 64
// lanes); BC is per wave (all its pairs have nb*BC >= H). Each step lane s
// takes from lane s-1 (DPP wave_shr:1; ignored on a group's first lane):
//   - the Y entering its first column on row i (lane s-1's row i, last step),
//   - the right-edge T of row i-1, its first diagonal (two steps back: held
//     one step in a register),
//   - on row R, the running sums ΣM, ΣX, so the final sums are accumulated
//     column by column left to right exactly as the reference does.
// Lanes outside 1 <= i <= rmax (pipeline fill / drain) are masked off; columns
// past H compute values that only flow right and are never summed.
template <int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_seg(const LaneArgs& a, const LaneWave& wv, int lane, int s,
                                        const LaneCtx<1>& cx, float T0, float& sumM, float& sumX,
                                        uint2* __restrict__ mt)
{
    const int c0 = s * BC;
    const int R = cx.R[0];
    {   // this lane's BC-column window of the match table, fixed for the sweep:
        // columns c0+1 .. c0+BC start at bit 31-r of table row c0/32+lead
        const int nwpad = (cx.H[0] + 31) / 32 + kHapLead;   // the trailing zero row
        const int w0 = c0 / 32 + kHapLead, r = c0 & 31;
        const int i0 = min(w0, nwpad), i1 = min(w0 + 1, nwpad), i2 = min(w0 + 2, nwpad);
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const uint64_t x01 = (uint64_t(cx.hw[0][i0 * 5 + c]) << 32) | cx.hw[0][i1 * 5 + c];
            const uint64_t x12 = (uint64_t(cx.hw[0][i1 * 5 + c]) << 32) | cx.hw[0][i2 * 5 + c];
            mt[c * 64 + lane] = make_uint2(uint32_t((x01 << r) >> 32), uint32_t((x12 << r) >> 32));
        }
    }
    float T[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        T[j] = T0;   // row 0
        X[j] = 0.f;
    }
    uint32_t wc[1] = {cx.rrow[0][0]}, wn[1] = {cx.rrow[0][min(2, R) - 1]};
    RowConst<1> k;
    row_const<1>(a.lut, wc, wn, k);
    uint2 mrow = mt[k.rc[0] * 64 + lane];
    float y_out = 0.f, t_out = 0.f;   // handed to lane s+1: Y past column c0+BC, T[BC-1] of the last row
    float t_hold = 0.f;               // lane s-1's right-edge T of the previous row
    const int lim0 = cx.H[0] - c0;    // columns of this block inside the hap (<= 0: none)
    auto step = [&](int kk, auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        const int i = kk - s;
        const float y_in = from_left(y_out);
        const float t_in = from_left(t_out);
        float sM_in = 0.f, sX_in = 0.f;
        if constexpr (SUM) {
            sM_in = from_left(sumM);
            sX_in = from_left(sumX);
        }
        // Row 1's diagonal is row 0's T at every column; below that, lane
        // s-1's right edge (column 0 for block 0: T[i][0] = 0 for i >= 1).
        const float Tdiag = i == 1 ? T0 : (s ? t_hold : 0.f);
        const float Yl0 = s ? y_in : 0.f;   // block 0: Y[i][1] = 0*my + 0*yy = 0
        t_hold = t_in;
        if (unsigned(i - 1) < unsigned(wv.rmax)) {
            if constexpr (!CG) {
                row_const<1>(a.lut, wc, wn, k);
                mrow = mt[k.rc[0] * 64 + lane];
            }
            const uint32_t wnn = cx.rrow[0][min(i + 2, R) - 1];
            float pm_n = 0.f, px_n = 0.f;
            uint2 m_n = mrow;
            if constexpr (CG) {
                pm_n = a.lut[kOffPm + row_q(wn[0])];
                px_n = a.lut[kOffPx + row_q(wn[0])];
                m_n = mt[row_rc(wn[0]) * 64 + lane];
            }
            const uint32_t mw[1][2] = {{mrow.x, mrow.y}};
            const int pmi[1] = {__float_as_int(k.pm)}, pxi[1] = {__float_as_int(k.px)};
            const bool last = SUM && i == R;
            const int lim[1] = {last ? lim0 : 0};
            if (last) {
                sumM = s ? sM_in : 0.f;
                sumX = s ? sX_in : 0.f;
            }
            float Ml = 0.f, Yl = Yl0;
            const float M0 = Tdiag * prior_vec<1, 0>(mw, pmi, pxi);
            cell<1, BC, 0, BC, SUM, EQ>(T, X, M0, Ml, Yl, mw, pmi, pxi, k, lim, sumM, sumX);
            y_out = y_next<EQ>(Ml, Yl, k.my, k.yy);
            t_out = T[BC - 1];
            if constexpr (CG) {
                k.pm = pm_n;
                k.px = px_n;
                mrow = m_n;
            }
            wc[0] = wn[0];
            wn[0] = wnn;
        }
    };
    int kk = 1;
    for (; kk < wv.rmin; ++kk) step(kk, std::false_type{});
    for (; kk <= wv.nsteps; ++kk) step(kk, std::true_type{});
}

// Block widths of column-segmented waves (LaneWave.ncols of a segmented wave).
#define HC_SEG_WIDTHS(X) \
    X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

template <int BC>
__device__ __forceinline__ void run_seg_bc(const LaneArgs& a, const LaneWave& wv, int lane, int s,
                                           const LaneCtx<1>& cx, float T0, float& sumM, float& sumX,
                                           uint2* __restrict__ mt, bool wave_cg, bool wave_eq)
{
    // Two compiled paths per width: EQ (the reference's constant 'I'/'I'/'+'
    // gap qualities) and the generic per-row path (any gap qualities).
    (void)wave_cg;
    if (wave_eq)
        run_seg<BC, true, true>(a, wv, lane, s, cx, T0, sumM, sumX, mt);
    else
        run_seg<BC, false, false>(a, wv, lane, s, cx, T0, sumM, sumX, mt);
}

// Per-lane pair context and the row-0 diagonal T0 = (0*mm + 0*gapm) + (INITIAL/H)*gapm
// (avx-pairhmm-template.h:160-166 with row 1's constants).
__device__ __forceinline__ void load_pair(const LaneArgs& a, int pid, LaneCtx<1>& cx, int p, float& t0)
{
    const PairDesc pd = a.pairs[pid];
    cx.R[p] = pd.y;
    cx.H[p] = pd.w;
    cx.rrow[p] = a.rows + pd.x;
    cx.hw[p] = a.hapw + pd.z;
    const uint32_t w1 = cx.rrow[p][0];
    const float mm1 = a.lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
    const float g1 = a.lut[kOffGapm + row_c(w1)];
    const float initY = 0x1p120f / float(pd.w);
    t0 = (0.f * mm1 + 0.f * g1) + initY * g1;
}

// Wave metadata is wave-uniform: pin it to SGPRs so loops and switches are
// scalar branches.
__device__ __forceinline__ LaneWave load_wave(const LaneArgs& a, int wid)
{
    LaneWave wv;
    const LaneWave w = a.waves[wid];
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

__device__ __forceinline__ void emit(const LaneArgs& a, int pid, float raw)
{
    a.raw_out[pid] = raw;
    const bool resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
    a.rescue_flag[pid] = resc;
    a.raw64_zero[pid] = 0.0;
    if (resc) a.rescue_list[atomicAdd(a.rescue_count, 1)] = pid;
}

// Constant-gap tag of a read: bit 31 of its first row word (mark_cg_kernel).
// EQ additionally needs insertion == deletion gap quality.
__device__ __forceinline__ bool read_cg(uint32_t w1) { return (w1 >> 31) != 0; }
__device__ __forceinline__ bool read_eq(uint32_t w1) { return read_cg(w1) && row_i(w1) == row_d(w1); }

// One lane per pair (P pairs per lane), column blocks of BC with the carry
// buffer between blocks.
template <int P, int BC, int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_lane_kernel(LaneArgs a)
{
    using V = typename VT<P>::type;
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= a.n_waves) return;
    const int lane = threadIdx.x & 63;
    const LaneWave wv = load_wave(a, wid);
    LaneCtx<P> cx;
    int pid[P];
    bool active[P];
    V T0;
    bool cg = true, eq = true;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int slot = wv.slot0 + lane * P + p;
        active[p] = slot < a.n_slots;
        pid[p] = a.order[active[p] ? slot : wv.slot0];
        const PairDesc pd = a.pairs[pid[p]];
        cx.R[p] = pd.y;
        cx.H[p] = pd.w;
        cx.rrow[p] = a.rows + pd.x;
        cx.hw[p] = a.hapw + pd.z;
        const uint32_t w1 = cx.rrow[p][0];
        const float mm1 = a.lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
        const float g1 = a.lut[kOffGapm + row_c(w1)];
        const float initY = 0x1p120f / float(pd.w);
        set_comp(T0, p, (0.f * mm1 + 0.f * g1) + initY * g1);
        cg &= read_cg(w1);
        eq &= read_eq(w1);
    }
    const bool wave_cg = __builtin_amdgcn_ballot_w64(!cg) == 0;
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!eq) == 0;
    V sumM = splat<V>(0.f), sumX = splat<V>(0.f);
    __shared__ uint2 mtab[4][P * 5 * 64];
    uint2* mt = mtab[threadIdx.x >> 6];
    if (wave_eq)
        run_pairs<P, BC, true, true>(a, wv, lane, cx, T0, sumM, sumX, mt);
    else if (wave_cg)
        run_pairs<P, BC, true, false>(a, wv, lane, cx, T0, sumM, sumX, mt);
    else
        run_pairs<P, BC, false, false>(a, wv, lane, cx, T0, sumM, sumX, mt);
#pragma unroll
    for (int p = 0; p < P; ++p)
        if (active[p]) emit(a, pid[p], comp(sumM, p) + comp(sumX, p));
}

// Column-segmented waves (run_seg). The wave's npairs pairs are the slots
// slot0 .. slot0+npairs-1; pair g takes nb_g = ceil(H_g / BC) consecutive lanes
// in slot order. Lanes past the last group idle (s = 0, no output).
template <int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_seg_kernel(LaneArgs a)
{
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= a.n_waves) return;
    const int lane = threadIdx.x & 63;
    const LaneWave wv = load_wave(a, wid);
    const int bc = wv.ncols;
    __shared__ uint2 mtab[4][5 * 64];
    uint2* mt = mtab[threadIdx.x >> 6];
    // Lane -> (group, block): group g's lanes start at the prefix sum of nb.
    int* gmap = reinterpret_cast<int*>(mt);   // 64 ints, reused before the match table
    int pid_g = 0, nb_g = 0;
    if (lane < wv.npairs) {
        pid_g = a.order[wv.slot0 + lane];
        nb_g = (a.pairs[pid_g].w + bc - 1) / bc;
    }
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
    int pid = a.order[wv.slot0 + (g >= 0 ? g : 0)];
    bool owner = false;
    if (g >= 0)
        owner = s == (a.pairs[pid].w + bc - 1) / bc - 1;
    else
        s = 0;
    LaneCtx<1> cx;
    float T0;
    load_pair(a, pid, cx, 0, T0);
    const uint32_t w1 = cx.rrow[0][0];
    const bool wave_cg = __builtin_amdgcn_ballot_w64(!read_cg(w1)) == 0;
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!read_eq(w1)) == 0;
    float sumM = 0.f, sumX = 0.f;
    switch (bc) {
#define HC_SEG_CASE(W) \
    case W: run_seg_bc<W>(a, wv, lane, s, cx, T0, sumM, sumX, mt, wave_cg, wave_eq); break;
        HC_SEG_WIDTHS(HC_SEG_CASE)
#undef HC_SEG_CASE
    default: break;
    }
    if (owner) emit(a, pid, sumM + sumX);
}

}  // namespace

// Lane kernel variants: {pairs per lane, block columns, waves per SIMD}.
// Block widths are multiples of 32 (a block starts on a match-word boundary).
// Measured on S2 (ms per fp32 pass): v0 11.5, v1 12.8, v2 15.6, v3 17.7.
constexpr int kSegOcc = 3;   // waves per SIMD of the column-segmented kernel
static const LaneVariant kVariants[] = {
    {1, 64, 3}, {1, 64, 2}, {1, 32, 4}, {2, 32, 2},
};

const LaneVariant& lane_variant(int id)
{
    const int n = int(sizeof(kVariants) / sizeof(kVariants[0]));
    return kVariants[(id >= 0 && id < n) ? id : 0];
}

hipError_t launch_lane_f32(int id, const LaneArgs& a, hipStream_t s)
{
    if (a.n_waves <= 0) return hipSuccess;
    const int grid = (a.n_waves + 3) / 4;
    const dim3 g(grid), blk(256);
    switch ((id >= 0 && id < 4) ? id : 0) {
    case 1: hipLaunchKernelGGL((phmm_lane_kernel<1, 64, 2>), g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL((phmm_lane_kernel<1, 32, 4>), g, blk, 0, s, a); break;
    case 3: hipLaunchKernelGGL((phmm_lane_kernel<2, 32, 2>), g, blk, 0, s, a); break;
    default: hipLaunchKernelGGL((phmm_lane_kernel<1, 64, 3>), g, blk, 0, s, a); break;
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

hipError_t launch_lane_seg_f32(const LaneArgs& a, hipStream_t s)
{
    if (a.n_waves <= 0) return hipSuccess;
    const int grid = (a.n_waves + 3) / 4;
    hipLaunchKernelGGL((phmm_seg_kernel<kSegOcc>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
