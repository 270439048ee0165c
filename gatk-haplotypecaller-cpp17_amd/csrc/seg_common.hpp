// Device building blocks shared by the column-segmented PairHMM kernels
// (lane_kernel.hip: phmm_seg_kernel, phmm_seg64_kernel, the one-lane kernel):
// the cell update in the reference's operation order, the per-row constants,
// DPP hand-offs, prefetch depth.
// Same semantics as compute_full_prob_avx{s,d} (avx-pairhmm-template.h:210-346).
#pragma once
#include <type_traits>

#include "device_common.hpp"
#include "kernels.hpp"
#include "luts.hpp"

namespace hcphmm {
namespace seg {

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
// MASK (the one-lane kernel, whose blocks start at column 1): only columns
// J < lim enter the sums (lim = columns of the block inside the hap on the
// pair's last row, else 0).
template <typename T, int BC, int J, int NC, bool SUM, bool EQ, bool MASK = false>
__device__ __forceinline__ void cell(T (&Tt)[BC], T (&X)[BC], T M, T& Ml, T& Yl, uint32_t mw0, uint32_t mw1,
                                     T pm, T px, const RowConst<T>& k, int lim, T& sumM, T& sumX)
{
    if constexpr (J < NC) {
        T Mn = M;
        if constexpr (J + 1 < NC)
            Mn = Tt[J] * prior_of<31 - ((J + 1) & 31)>(((J + 1) >> 5) ? mw1 : mw0, pm, px);
        const T Xc = X[J];
        if constexpr (SUM && !MASK) {
            // The row sums first: they read M and the old X[J] before X[J] is
            // rewritten (after it, the old value needed a copy per column).
            // Every column of a block is a hap column or a zero padding column
            // (run_seg), so the row's sums need no column mask; rows other than
            // the pair's last accumulate values that run_seg discards.
            sumM = sumM + M;
            sumX = sumX + Xc;
        }
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
        if constexpr (SUM && MASK) {
            const bool c = J < lim;   // column c0+J+1 <= H on the pair's last row
            sumM = sumM + (c ? M : T(0));
            sumX = sumX + (c ? Xc : T(0));
        }
        Yl = Y;
        cell<T, BC, J + 1, NC, SUM, EQ, MASK>(Tt, X, Mn, Ml, Yl, mw0, mw1, pm, px, k, lim, sumM, sumX);
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

// A lane's pair: its read rows and hap match table as 32-bit offsets from the
// part's uniform bases (one VGPR each per lane and SGPR bases, so the loads
// take the global_load SGPR-base + VGPR-offset form and no 64-bit address
// stays live per lane: they spilled).
struct LaneCtx {
    const uint32_t* rbase;  // rows - kRowPadBefore (uniform)
    uint32_t rbyte;         // byte offset of the read's first row word from rbase
    const uint32_t* hbase;  // the part's hap tables (uniform)
    uint32_t hbyte;         // byte offset of the hap's match table from hbase
    int R, H;
};

// Row word idx of the lane's read (idx may be negative, down to
// -kRowPadBefore: prefetches before a read's first row).
__device__ __forceinline__ uint32_t row_word(const LaneCtx& cx, int idx)
{
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cx.rbase) +
                                             (cx.rbyte + unsigned(idx) * 4u));
}
// Word idx of the lane's hap match table.
__device__ __forceinline__ uint32_t hap_word(const LaneCtx& cx, int idx)
{
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cx.hbase) +
                                             (cx.hbyte + unsigned(idx) * 4u));
}

// Row-0 diagonal T0 = (0*mm + 0*gapm) + (INITIAL/H)*gapm with row 1's
// constants (avx-pairhmm-template.h:160-166: Y[0][j] = INITIAL / H).
template <typename T>
__device__ __forceinline__ T row0_t(const T* __restrict__ lut, uint32_t w1, int H)
{
    const T mm1 = lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
    // Opaque offset: otherwise the address lut + 4 * row_c is shared with row
    // 1's ph2pr[row_c] load in the step loop's set-up, and that 64-bit address,
    // live across the wave's whole prologue, is spilled to scratch.
    unsigned go = unsigned(kOffGapm + row_c(w1)) * unsigned(sizeof(T));
    asm volatile("" : "+v"(go));
    const T g1 = *reinterpret_cast<const T*>(reinterpret_cast<const char*>(lut) + go);
    const T initY = initial_value<T>() / T(H);
    return (T(0) * mm1 + T(0) * g1) + initY * g1;
}

__device__ __forceinline__ LaneCtx desc_ctx(const PairDesc pd, const uint32_t* rows, const uint32_t* hapw)
{
    return LaneCtx{rows - kRowPadBefore, unsigned(pd.x + kRowPadBefore) * 4u, hapw, unsigned(pd.z) * 4u, pd.y, pd.w};
}
__device__ __forceinline__ LaneCtx pair_ctx(const PairDesc* pairs, const uint32_t* rows, const uint32_t* hapw,
                                            int pid)
{
    return desc_ctx(pairs[pid], rows, hapw);
}

// Constant-gap tag of a read: bit 31 of its first row word (pack_reads_kernel).
// EQ additionally needs insertion == deletion gap quality.
__device__ __forceinline__ bool read_cg(uint32_t w1) { return (w1 >> 31) != 0; }
__device__ __forceinline__ bool read_eq(uint32_t w1) { return read_cg(w1) && row_i(w1) == row_d(w1); }

__device__ __forceinline__ float from_left(float v)
{
    // DPP wave_shr:1: lane l receives lane l-1's v; lane 0 receives 0 by
    // bound_ctrl (no zeroed destination to materialise first).
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ double from_left(double v)
{
    const long long x = __double_as_longlong(v);
    const unsigned lo = unsigned(__builtin_amdgcn_mov_dpp(int(x), 0x138, 0xf, 0xf, true));
    const unsigned hi = unsigned(__builtin_amdgcn_mov_dpp(int(x >> 32), 0x138, 0xf, 0xf, true));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// v & mask bitwise (mask all ones or zero, in a VGPR): one full-rate v_and per
// 32 bits. (Written as C the compiler proves the mask boolean and selects with
// v_cndmask on an SGPR lane mask instead, a half-rate form.)
__device__ __forceinline__ uint32_t and_v(uint32_t a, uint32_t m)
{
    uint32_t r;
    asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(m));
    return r;
}
// AND: the v_and form (the mask lives in a VGPR: one register more, so only
// where the block's registers leave room — the widest fp32 blocks spill with it).
template <bool AND>
__device__ __forceinline__ float masked(float v, uint32_t m)
{
    return __uint_as_float(AND ? and_v(__float_as_uint(v), m) : (__float_as_uint(v) & m));
}
template <bool AND>
__device__ __forceinline__ double masked(double v, uint32_t m)
{
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    if (!AND) return __longlong_as_double((long long)(x & ((unsigned long long)m << 32 | m)));
    return __longlong_as_double(
        (long long)(((unsigned long long)and_v(uint32_t(x >> 32), m) << 32) | and_v(uint32_t(x), m)));
}


// Step bounds of a column-segmented wave (wave-uniform).
struct SegSteps {
    int rmax;     // max R of the wave's pairs
    int rmin;     // first step that may need the row sums
    int nsteps;   // max over the wave's pairs of R + nb - 1
    int prio = 0; // issue priority: 0 off, 1 by remaining steps, 2 by age (set_prio)
    unsigned long long t0 = 0;   // the wave's start (s_memrealtime), for prio 2
};

// VALU issue between the waves of a SIMD is arbitrated by priority, then age
// (MI355X_MICROARCH.md, two waves per SIMD): the oldest wave runs ahead and
// the last waves of a pass, the youngest, are left to finish alone at half
// the issue rate. With prio on, a wave raises its priority with the steps it
// has left (longest remaining first), so co-resident waves tend to finish
// together. s_setprio takes an immediate: four uniform branches.
__device__ __forceinline__ void set_prio_by_remaining(int rem)
{
    if (rem > 192) __builtin_amdgcn_s_setprio(3);
    else if (rem > 96) __builtin_amdgcn_s_setprio(2);
    else if (rem > 32) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
// In a pass whose waves are fetched from a counter, a hardware wave keeps its
// slot for the whole launch, so between the two waves of a SIMD the older
// always wins a tie: with chains of four, one wave per SIMD took 3.2 ms while
// the other slot ran four 0.78 ms chains (tools/chain_probe.py, DESIGN.md
// §16.2), and neither the remaining-steps bands nor bands by progress undid
// it (a fresh wave on the older slot ties or outranks the starved one). There
// the priority rises with the time since the wave's start instead (quanta of
// ~100 us): the wave that started first goes first, as if each wave were a
// fresh hardware wave dispatched in order.
__device__ __forceinline__ void set_prio_by_age(unsigned long long t0)
{
    const unsigned long long q = (__builtin_amdgcn_s_memrealtime() - t0) / 10000;   // 100 MHz ticks
    if (q >= 3) __builtin_amdgcn_s_setprio(3);
    else if (q == 2) __builtin_amdgcn_s_setprio(2);
    else if (q == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
// prio mode: 1 by remaining steps, 2 by the wave's age (SegSteps::prio).
__device__ __forceinline__ void set_prio(int mode, int kk, int nsteps, unsigned long long t0)
{
    if (mode == 2) set_prio_by_age(t0);
    else set_prio_by_remaining(nsteps - kk);
}

// Rows of read words a lane keeps in flight (loaded PD steps before use). A
// lone step of a narrow block is too short to cover a global load, so narrow
// blocks prefetch deeper; the step loop is unrolled by PD so every word lands
// in its own register and is not touched (no wait) until its step. fp32
// blocks of 32-64 columns take two steps too (round 3: S2 fp32 pass 8.884 ->
// 8.815 ms, a 125k-pair shard -1.5 %, S1w at 1M pairs +0.8 %; three steps no
// better: profiles/r03_prefetch_depth_ab.jsonl).
template <typename T, int BC>
constexpr int seg_prefetch()
{
    return sizeof(T) == 8 ? (BC >= 16 ? 1 : 2) : (BC >= 16 ? 2 : 4);
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

// The prior tables [ph2pr | pm | px | gapm] (luts.hpp) in LDS: the per-row
// prior lookups of the segmented kernels read them there.
constexpr int kSlutLen = kOffMM;
template <typename T>
__device__ __forceinline__ void load_slut(T* __restrict__ slut, const T* __restrict__ lut)
{
    for (int t = threadIdx.x; t < kSlutLen; t += blockDim.x) slut[t] = lut[t];
    __syncthreads();
}

// Block widths of fp32 column-segmented waves (LaneWave.ncols of a seg wave):
// 8..64 in steps of 2 (steps of 4 measured the same kernel time at a worse
// column rounding; odd widths model only 0.6 % better).
#define HC_SEG_WIDTHS(X)                                                                                       \
    X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) X(26) X(28) X(30) X(32) X(34) X(36) X(38) X(40) X(42) \
    X(44) X(46) X(48) X(50) X(52) X(54) X(56) X(58) X(60) X(62) X(64)

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
// A lane computes rows 1 .. R of its pair (pipeline fill / drain and a
// shorter pair's steps past its R are masked off).
// Block 0 starts `pad` = nb*BC - H columns left of column 1: those padding
// columns hold exact zeros (row 0's T is 0 left of column 0, so their M, X, Y
// and T stay 0 on every row, and column 0's T is T0 on row 0 and 0 below, as
// the reference's boundary), so the pair's last block ends exactly at column
// H and the last row's sums add only hap columns and leading +0.0 terms —
// the reference's sums, with no per-column mask.
// A lane's match window: columns c0+1 .. c0+64 of the hap's match table
// (rows of 32 bits, MSB first, kHapLead zero rows before), for each of the 5
// read codes, into its LDS slots mt[code * 64 + lane].
__device__ __forceinline__ void fill_window(uint2* __restrict__ mt, int lane, const LaneCtx& cx, int c0)
{
    const int H = cx.H;
    const int nwpad = (H + 31) / 32 + kHapLead;   // the trailing zero row
    const int w0 = (c0 >> 5) + kHapLead, r = c0 & 31;   // c0 >= -63 (block 0's padding): floor division
    const int i0 = min(w0, nwpad), i1 = min(w0 + 1, nwpad), i2 = min(w0 + 2, nwpad);
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const uint32_t h0 = hap_word(cx, i0 * 5 + c), h1 = hap_word(cx, i1 * 5 + c), h2 = hap_word(cx, i2 * 5 + c);
        const uint64_t x01 = (uint64_t(h0) << 32) | h1;
        const uint64_t x12 = (uint64_t(h1) << 32) | h2;
        mt[c * 64 + lane] = make_uint2(uint32_t((x01 << r) >> 32), uint32_t((x12 << r) >> 32));
    }
}

template <typename T, int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_seg(const T* __restrict__ lut, const T* __restrict__ slut, const SegSteps& st,
                                        int lane, int s, const LaneCtx& cx, T T0, T& sumM, T& sumX,
                                        uint2* __restrict__ mt)
{
    constexpr int PD = seg_prefetch<T, BC>();
    const int pad = ((cx.H + BC - 1) / BC) * BC - cx.H;   // zero columns left of column 1 (block 0)
    const int c0 = s * BC - pad;                          // this block: columns c0+1 .. c0+BC
    const int R = cx.R;
    fill_window(mt, lane, cx, c0);
    T Tt[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        Tt[j] = c0 + j + 1 >= 0 ? T0 : T(0);   // row 0: T0 from column 0 on, 0 on the padding left of it
        X[j] = T(0);
    }
    // wq[P]: the word of row i+1 (clamped to 1..R) at the steps of phase
    // P = (k-1) mod PD, for every lane at every step; the loads are issued
    // unconditionally so that each path has the same outstanding loads and
    // the wait for a word is the one PD steps after its load.
    uint32_t wc = row_word(cx, 0);
    uint32_t wq[PD];
#pragma unroll
    for (int P = 0; P < PD; ++P) wq[P] = row_word(cx, min(max(P + 2 - s, 1), R) - 1);
    RowConst<T> k;
    row_const<T>(lut, wc, row_word(cx, min(2, R) - 1), k);
    uint2 mrow = mt[k.rc * 64 + lane];
    // A pair's last block (and any lane past it) hands zeros to the lane on its
    // right, so a group's first lane needs no select: it receives Y = 0 entering
    // column 1 and T = 0 (column 0 below row 0) from its left neighbour, and
    // T0 (row 0's diagonal) from its own initial t_hold on row 1. Inside a
    // group, lane s-1's initial t_out is T0: lane s's row-1 diagonal.
    const uint32_t keep = (s + 1) * BC < cx.H ? 0xffffffffu : 0u;
    constexpr bool AND = BC * int(sizeof(T)) <= 128;   // masked's v_and form: fp32 up to 32 columns, fp64 16
    T y_out = T(0);                      // handed to lane s+1: Y past column c0+BC,
    T t_out = masked<AND>(T0, keep);     //   T[BC-1] of the last row
    T t_hold = c0 >= 0 ? T0 : T(0);      // lane s-1's right-edge T of the previous row (row 0: column c0's)
    // Running row sums (sumM, sumX): every lane adds its columns on every
    // sum-variant step and restarts from its left neighbour's at its last row
    // R; a lane stops at row R (rows past a pair's R feed nothing), so after
    // the sweep the pair's last block holds the pair's sums.
    auto step = [&](int kk, auto sum_tag, auto ph_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        constexpr int P = decltype(ph_tag)::value;
        const int i = kk - s;
        const uint32_t wn = wq[P];   // row i+1, loaded PD steps ago
        T pm_n = T(0), px_n = T(0);
        uint2 m_n = mrow;
        // The word needed PD steps from now (row i + PD + 1). Not clamped to
        // the read: outside rows 1..R it feeds only rows no result depends on,
        // and the packed rows carry slack on both sides (engine.cpp o_rows).
        int ridx = i + PD;
        if constexpr (CG) {   // next row's prior constants (LDS) and match words
            const int qo = row_q(wn), mo = row_rc(wn) * 64 + lane;
            // Order the load after the last use of wn, so the word can land in
            // wn's register (no register move, hence no wait, at the loop back edge).
            asm volatile("" : "+v"(ridx) : "v"(qo), "v"(mo));
            pm_n = slut[kOffPm + qo];
            px_n = slut[kOffPx + qo];
            m_n = mt[mo];
        } else {
            asm volatile("" : "+v"(ridx) : "v"(wn));
        }
        wq[P] = row_word(cx, ridx);
        const T y_in = from_left(y_out);
        const T t_in = from_left(t_out);
        T sM_in = T(0), sX_in = T(0);
        if constexpr (SUM) {
            sM_in = from_left(sumM);
            sX_in = from_left(sumX);
        }
        // Row 1's diagonal is row 0's T at every column; below that, lane
        // s-1's right edge (column 0 for block 0: T[i][0] = 0 for i >= 1,
        // handed as 0 by the left neighbour, see keep).
        const T Tdiag = t_hold;
        const T Yl0 = y_in;   // block 0: Y[i][1] = 0*my + 0*yy = 0 (likewise)
        t_hold = t_in;
        if (unsigned(i - 1) < unsigned(R)) {   // this lane's rows 1 .. R of its pair
            if constexpr (!CG) {
                row_const<T>(lut, wc, wn, k);
                mrow = mt[k.rc * 64 + lane];
            }
            if (SUM && i == R) {
                sumM = s ? sM_in : T(0);
                sumX = s ? sX_in : T(0);
            }
            T Ml = T(0), Yl = Yl0;
            const T M0 = Tdiag * prior_of<31>(mrow.x, k.pm, k.px);
            cell<T, BC, 0, BC, SUM, EQ>(Tt, X, M0, Ml, Yl, mrow.x, mrow.y, k.pm, k.px, k, 0, sumM, sumX);
            y_out = masked<AND>(y_next<EQ>(Ml, Yl, k.my, k.yy), keep);
            t_out = masked<AND>(Tt[BC - 1], keep);
        }
        if constexpr (CG) {
            // Unconditional (no register moves for a conditional update): a
            // lane before its row 1 takes row i + 1's constants too, and at
            // i = 0 those are row 1's, what it needs on its first row.
            k.pm = pm_n;
            k.px = px_n;
            mrow = m_n;
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
    int pk = st.prio ? 1 : INT32_MAX;   // next step at which the priority is updated (every 16 steps)
    for (; kk + PD - 1 < st.rmin; kk += PD) {
        if (kk >= pk) {
            set_prio(st.prio, kk, st.nsteps, st.t0);
            pk += 16;
        }
        for_phases<0, PD>([&](auto ph) { step(kk + decltype(ph)::value, std::false_type{}, ph); });
    }
    for (; kk <= st.nsteps; kk += PD) {
        if (kk >= pk) {
            set_prio(st.prio, kk, st.nsteps, st.t0);
            pk += 16;
        }
        for_phases<0, PD>([&](auto ph) { step(kk + decltype(ph)::value, std::true_type{}, ph); });
    }
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

// The fp64 rescue (intel_pairhmm.hpp:137-139) of the pairs this wave's fp32
// pass flagged (`todo`: their owner lanes). A wave with at most two, each with
// H <= kInWaveRescueMaxH, recomputes them itself while the rest of the pass
// runs — one pair at a time over the whole wave (8 columns per lane, the
// same run_seg in double) — so a batch with a few rescues (S2: ~2e-5 of
// the pairs) needs no separate latency-bound pass after the fp32 kernel. The
// others are appended to the rescue list for that pass.
// fp64 recompute of pair rp (slot rs) by the whole wave: 64 lanes of 8
// columns, raw f64 sum to the slot's record or raw64_zero[rp].
__device__ __forceinline__ void rescue_one(const LaneArgs& a, const PairDesc pd, int rp, int rs, int lane,
                                           uint2* __restrict__ mt)
{
    const int R = __builtin_amdgcn_readfirstlane(pd.y), H = __builtin_amdgcn_readfirstlane(pd.w);
    const int rx = __builtin_amdgcn_readfirstlane(pd.x);
    const LaneCtx cx{a.rows - kRowPadBefore, unsigned(rx + kRowPadBefore) * 4u, a.hapw,
                     unsigned(__builtin_amdgcn_readfirstlane(pd.z)) * 4u, R, H};
    constexpr int bc = seg64_width(0);
    const int nb = (H + bc - 1) / bc;
    const SegSteps st{R, R, R + nb - 1, 0};
    const uint32_t w1 = row_word(cx, 0);
    const double T0 = row0_t<double>(a.lut64, w1, H);
    const bool eq = read_eq(w1);
    double sM = 0.0, sX = 0.0;
    run_seg_bc<double, bc>(a.lut64, a.lut64, st, lane, lane, cx, T0, sM, sX, mt, eq);
    if (lane == nb - 1) {
        const double r = sM + sX;
        if (a.rec) {   // record of slot rs: state and raw f64 (after the owner's store: same wave, program order)
            const unsigned long long b = (unsigned long long)__double_as_longlong(r);
            uint4* q = a.rec + rs;
            q->y = kRecInWave;
            *reinterpret_cast<uint2*>(&q->z) = make_uint2(unsigned(b), unsigned(b >> 32));
        } else {
            a.raw64_zero[rp] = r;
        }
    }
    __builtin_amdgcn_wave_barrier();   // the next pair rewrites mt
}

// Rescue pair rp (slot rs, hap length H) in this wave if it qualifies and the
// run's in-wave budget allows (wave-uniform), else append it to the fp64
// launch's list (lane `owner_lane`).
__device__ __forceinline__ void rescue_or_defer(const LaneArgs& a, bool few, int rp, int rs, int H, int R, int lane,
                                                int owner_lane, uint2* __restrict__ mt)
{
    bool here = few && H <= kInWaveRescueMaxH;
    if (here) {
        int c = 0;
        if (lane == 0) c = atomicAdd(a.inker_count, 1);
        here = __builtin_amdgcn_readfirstlane(c) < a.inker_limit;
    }
    if (here)
        rescue_one(a, a.sdesc[rs], rp, rs, lane, mt);   // sdesc[rs] = pairs[rp]
    else if (lane == owner_lane) {
        const int pos = atomicAdd(a.rescue_count, 1);
        a.rescue_list[pos] = rp;
        a.rescue_rh[pos] = pack_rh(R, H);
    }
}

__device__ __forceinline__ void rescue_in_wave(const LaneArgs& a, uint64_t todo, int pid, int slot, int H, int R,
                                               int lane, uint2* __restrict__ mt)
{
    // (No fp64 launch after this pass: every one, the list would go unread.)
    const bool few = a.inker_count != nullptr && (a.solo_counters != nullptr || __popcll(todo) <= 2);
    // The owners' result records are complete before a rescue rewrites part
    // of one (the same address from another lane of this wave).
    if (a.rec) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    while (todo) {
        const int l = __builtin_ctzll(todo);
        todo &= todo - 1;
        rescue_or_defer(a, few, __builtin_amdgcn_readlane(pid, l), __builtin_amdgcn_readlane(slot, l),
                        __builtin_amdgcn_readlane(H, l), __builtin_amdgcn_readlane(R, l), lane, l, mt);
    }
}

}  // namespace seg
}  // namespace hcphmm
