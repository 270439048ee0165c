// Smith-Waterman (Gotoh, int32) with backtrack on gfx950.
//
// Reference: src/haplotypecaller/smithwaterman/native/PairWiseSW.h — the AVX2
// anti-diagonal sweep smithWatermanBackTrack (:41-238, cell update MAIN_CODE
// :4-38), the end-point scan (:201-226) and getCIGAR (:240-415).
//
// sw_dp_kernel: one wave per pair. The 64 lanes own 64 consecutive rows of
// seq1 (a stripe) and sweep the seq2 columns with a one-row skew: at step t
// lane k computes cell (64s + k + 1, t - k + 1). The upper neighbour's H and F
// arrive from lane k-1 by DPP wave_shr:1 — the reference's _vector_shift moves
// become one v_mov_dpp each — and lane 0 takes them from an LDS row buffer that
// holds the previous stripe's last row (written in place by the stripe's lanes,
// the last writer of each column being lane 63). The alt base travels the same
// way. Each lane packs its cells' 4-bit backtrack codes (op | INSERT_EXT |
// DELETE_EXT) into one 32-bit word per 8 steps and stores it coalesced (a wave
// writes 256 contiguous bytes). After the last stripe the wave picks the end
// point among the last-row (LDS row buffer) and last-column (LDS) candidates
// with the reference's tie-breaks, in the reference's anti-diagonal order.
//
// Fast path (the default when the host proves the cutoff inert): the same
// cells and bits from fewer VALU issue slots. gfx950 issues v_add/v_sub at
// full rate but v_max, DPP moves, v_alignbit, compares and any VALU op with an
// SGPR operand at half rate (tools/ubench/op_rate.hip), so a lane keeps
// E + extend, F + extend and H(i-1, j-1) + open (the previous step's vertical
// open score), hands the lane below H + open rather than H (the vertical open
// score arrives ready by DPP, the diagonal needs no add of its own), and keeps
// the gap scores in VGPRs: 9 full-rate + 11 half-rate instructions per cell
// (the first form: 11 + 11 plus 5 SGPR-operand adds). The match/mismatch
// choice is a compare of the haplotype byte with the lane's seq1 byte. (An
// int16 LDS substitution profile per distinct seq1 byte and a spiral layout
// running lanes on into the next stripe were measured slower on W2 / W3 —
// DESIGN.md §8.2 — and removed in round 6: their code paths held the kernel's
// registers at 90 VGPRs, 79 without.)
//
// sw_trace_kernel: one wave per pair walks the backtrack from the end point
// (getCIGAR's state machine), 64 cells per step along the current direction,
// and writes run-length CIGAR elements.
#include "sw_kernels.hpp"

#include <algorithm>
#include <climits>

namespace hcsw {
namespace {

__device__ __forceinline__ int shr1(int old, int v)
{
    // DPP wave_shr:1: lane k receives lane k-1's v; lane 0 keeps `old`.
    return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false);
}

// LDS ordering between the lanes of one wave (a pair is one wave; several
// pairs may share a workgroup, so no workgroup barrier): the LDS executes a
// wave's operations in order, the fences keep the compiler from moving them.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_max(int v)
{
    for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ int wave_sum(int v)
{
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// H(x, 0) and H(0, x) for x >= 1 (PairWiseSW.h:188-197); H(0, 0) = 0 (:80).
__device__ __forceinline__ int boundary(int overhang, int open, int extend, int x)
{
    return (x > 0 && (overhang == 10 || overhang == 11)) ? open + (x - 1) * extend : 0;
}

struct Lane {
    int h;      // H(i, j) of this lane's last cell (= H(i, j-1) for the next one)
    int e;      // E(i, j)
    int f;      // F(i, j)
    int diag;   // H(i-1, j-1) for the next cell
    uint32_t acc;
};

struct Scores {
    int match, mismatch, open, extend;
};

// Group modes: which lanes are outside their columns [0, n2) somewhere in the group.
enum { kBulk = 0, kFill = 1, kDrain = 2, kBoth = 3 };

// One cell of MAIN_CODE (PairWiseSW.h:4-38) per lane. The backtrack nibble is
// (MSB first) [eo > ee][fo > fe][en > hn0][fn > hn1]: "open beats extend"
// horizontally / vertically (the reference stores their negation as
// INSERT_EXT / DELETE_EXT) and "E wins" / "F wins" (INSERT / DELETE).
//   FAST: the host proved every H stays above MATRIX_MIN_CUTOFF (so the
//         cutoff max is the identity) and no difference below overflows, so
//         each bit is the sign of a difference, shifted in by v_alignbit.
//   MODE: lanes not yet at column 0 hold H = H(i,0) and E = LOW (fill); lanes
//         past column n2 hold H = H(i,n2) for the end-point scan (drain).
//         A lane's F and its values past its end feed only lanes in the same
//         state, so nothing else needs holding.
//   LASTW: last, partial stripe: lanes past seq1's end leave the row buffer alone.
template <int MODE, bool LASTW, bool FAST>
__device__ __forceinline__ void step(Lane& L, int t, int lane, int n2, int rb, bool row_ok, int uh, int uf,
                                     int ab, const Scores& sc, int* rowH, int* rowF)
{
    const int up_h = shr1(uh, L.h);   // H(i-1, j)
    const int up_f = shr1(uf, L.f);   // F(i-1, j)
    const int eo = L.h + sc.open, ee = L.e + sc.extend;
    const int en = max(eo, ee);
    const int fo = up_h + sc.open, fe = up_f + sc.extend;
    const int fn = max(fe, fo);
    int hn0 = L.diag + (ab == rb ? sc.match : sc.mismatch);
    if (!FAST) hn0 = max(kMinCutoff, hn0);
    const int hn1 = max(hn0, en);
    const int hn = max(hn1, fn);
    if (FAST) {
        L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(ee - eo), 31);
        L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(fe - fo), 31);
        L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(hn0 - en), 31);
        L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(hn1 - fn), 31);
    } else {
        const uint32_t b = (eo > ee ? 8u : 0u) | (fo > fe ? 4u : 0u) | (en > hn0 ? 2u : 0u) | (fn > hn1 ? 1u : 0u);
        L.acc = (L.acc << 4) | b;
    }
    L.diag = up_h;
    L.f = fn;
    if (MODE == kBulk) {
        L.h = hn;
        L.e = en;
    } else if (MODE == kFill) {
        const bool act = t >= lane;
        L.h = act ? hn : L.h;
        L.e = act ? en : L.e;
    } else if (MODE == kDrain) {
        L.h = (t - lane < n2) ? hn : L.h;
        L.e = en;
    } else {
        const bool act = unsigned(t - lane) < unsigned(n2);
        L.h = act ? hn : L.h;
        L.e = act ? en : L.e;
    }
    if (!LASTW || row_ok) {
        rowH[64 + t - lane] = L.h;
        rowF[64 + t - lane] = L.f;
    }
}

template <int MODE, bool LASTW, bool FAST>
__device__ __forceinline__ void group(Lane& L, int t0, int lane, int n2, int rb, bool row_ok, const Scores& sc,
                                      int* rowH, int* rowF, const uint8_t* altB)
{
    // Lane 0's upper neighbours for the 8 steps (uniform addresses, 16-B reads)
    // and every lane's haplotype base (column t - lane; altB has 64 leading pads).
    const int4 h0 = *reinterpret_cast<const int4*>(rowH + 64 + t0);
    const int4 h1 = *reinterpret_cast<const int4*>(rowH + 68 + t0);
    const int4 f0 = *reinterpret_cast<const int4*>(rowF + 64 + t0);
    const int4 f1 = *reinterpret_cast<const int4*>(rowF + 68 + t0);
    const int uh[kGroup] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    const int uf[kGroup] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
    int ab[kGroup];
#pragma unroll
    for (int k = 0; k < kGroup; ++k) ab[k] = altB[64 + t0 + k - lane];
#pragma unroll
    for (int k = 0; k < kGroup; ++k)
        step<MODE, LASTW, FAST>(L, t0 + k, lane, n2, rb, row_ok, uh[k], uf[k], ab[k], sc, rowH, rowF);
}

template <bool LASTW, bool FAST>
__device__ __forceinline__ void stripe(Lane& L, int lane, int n2, int rb, bool row_ok, int T, uint32_t* btw,
                                       const Scores& sc, int* rowH, int* rowF, const uint8_t* altB)
{
    for (int t0 = 0; t0 < T; t0 += kGroup) {
        const bool fill = t0 < kStripe, drain = t0 + kGroup > n2;
        if (!fill && !drain)
            group<kBulk, LASTW, FAST>(L, t0, lane, n2, rb, row_ok, sc, rowH, rowF, altB);
        else if (fill && drain)
            group<kBoth, LASTW, FAST>(L, t0, lane, n2, rb, row_ok, sc, rowH, rowF, altB);
        else if (fill)
            group<kFill, LASTW, FAST>(L, t0, lane, n2, rb, row_ok, sc, rowH, rowF, altB);
        else
            group<kDrain, LASTW, FAST>(L, t0, lane, n2, rb, row_ok, sc, rowH, rowF, altB);
        btw[(t0 / kGroup) * kStripe + lane] = L.acc;
    }
}

// ---- fast compare path --------------------------------------------------
struct PLane {
    int h;    // H(i, j-1): this lane's last cell
    int ex;   // E(i, j-1) + extend
    int fx;   // F(i, j-1) + extend (read by the lane below by DPP)
    int dg;   // H(i-1, j-1) + open: the previous step's vertical open score
    uint32_t acc;
};

// One cell of MAIN_CODE (PairWiseSW.h:4-38) per lane, FAST semantics (see
// step): hn0 = H(i-1,j-1) + score = dg + (score - open).
template <int MODE, bool LASTW>
__device__ __forceinline__ void pstep(PLane& L, int t, int lane, int n2, bool row_ok, int ho, int fxo, int sc,
                                      int open, int extend, int* rowHo, int* rowF)
{
    const int eo = L.h + open;        // open_score_h: H(i, j-1) + open
    const int fo = shr1(ho, eo);      // open_score_v: H(i-1, j) + open (lane 0: row buffer)
    const int fe = shr1(fxo, L.fx);   // ext_score_v:  F(i-1, j) + extend
    const int fn = max(fe, fo);
    const int en = max(eo, L.ex);
    const int hn0 = L.dg + sc;
    const int hn1 = max(hn0, en);
    const int hn = max(hn1, fn);
    L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(L.ex - eo), 31);
    L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(fe - fo), 31);
    L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(hn0 - en), 31);
    L.acc = __builtin_amdgcn_alignbit(L.acc, uint32_t(hn1 - fn), 31);
    L.dg = fo;
    L.fx = fn + extend;
    const int exn = en + extend;
    if (MODE == kBulk) {
        L.h = hn;
        L.ex = exn;
    } else if (MODE == kFill) {
        const bool act = t >= lane;
        L.h = act ? hn : L.h;
        L.ex = act ? exn : L.ex;
    } else if (MODE == kDrain) {
        L.h = (t - lane < n2) ? hn : L.h;
        L.ex = exn;
    } else {
        const bool act = unsigned(t - lane) < unsigned(n2);
        L.h = act ? hn : L.h;
        L.ex = act ? exn : L.ex;
    }
    // H(i, j-1) + open for column j - 1 = t - lane, F(i, j) + extend for column
    // j: the last writer of each slot is the stripe's last row.
    if (!LASTW || row_ok) {
        rowHo[63 + t - lane] = eo;
        rowF[64 + t - lane] = L.fx;
    }
}

struct PGroupIn {
    int ho[kGroup];    // lane 0's H(64s, j) + open
    int fxo[kGroup];   // lane 0's F(64s, j) + extend
    int sc[kGroup];    // score(j) - open for this lane's row
};

// A lane's score(j) - open: a compare of the haplotype byte with its seq1 byte.
struct Scorer {
    const uint8_t* arow;   // arow[t] = haplotype byte of the column computed at step t
    int rb;                // this lane's seq1 byte (-1: no row)
    int mp, mmp;           // match - open, mismatch - open (VGPRs)
};

typedef const volatile __attribute__((address_space(3))) int LdsInt;
typedef const volatile __attribute__((address_space(3))) uint8_t LdsU8;

// Separate 32-bit loads (volatile: not merged into 64/128-bit tuples, whose
// elements the register allocator will not reuse as the DPP destinations) and
// one ds_read_u8 per score (no SDWA extract, which issues at half rate).
__device__ __forceinline__ void pload(PGroupIn& g, int t0, LdsInt* rowHo, LdsInt* rowF, const Scorer& sr)
{
#pragma unroll
    for (int k = 0; k < kGroup; ++k) {
        g.ho[k] = rowHo[64 + t0 + k];
        g.fxo[k] = rowF[64 + t0 + k];
        const int ab = ((LdsU8*)sr.arow)[t0 + k];
        g.sc[k] = ab == sr.rb ? sr.mp : sr.mmp;
    }
}

// A uniform value in a VGPR: a VALU operand read from an SGPR halves the issue
// rate of v_add_u32 on gfx950 (tools/ubench/op_rate.hip).
__device__ __forceinline__ int in_vgpr(int x)
{
    int v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}

template <int MODE, bool LASTW>
__device__ __forceinline__ void pgroup(PLane& L, int t0, int lane, int n2, bool row_ok, int open, int extend,
                                       int* rowHo, int* rowF, const Scorer& sr)
{
    PGroupIn g;
    pload(g, t0, (LdsInt*)rowHo, (LdsInt*)rowF, sr);
#pragma unroll
    for (int k = 0; k < kGroup; ++k)
        pstep<MODE, LASTW>(L, t0 + k, lane, n2, row_ok, g.ho[k], g.fxo[k], g.sc[k], open, extend, rowHo, rowF);
}

template <bool LASTW>
__device__ __forceinline__ void pstripe(PLane& L, int lane, int n2, bool row_ok, int T, uint32_t* btw, int open,
                                        int extend, int* rowHo, int* rowF, const Scorer& sr)
{
    for (int t0 = 0; t0 < T; t0 += kGroup) {
        const bool fill = t0 < kStripe, drain = t0 + kGroup > n2;
        if (!fill && !drain)
            pgroup<kBulk, LASTW>(L, t0, lane, n2, row_ok, open, extend, rowHo, rowF, sr);
        else if (fill && drain)
            pgroup<kBoth, LASTW>(L, t0, lane, n2, row_ok, open, extend, rowHo, rowF, sr);
        else if (fill)
            pgroup<kFill, LASTW>(L, t0, lane, n2, row_ok, open, extend, rowHo, rowF, sr);
        else
            pgroup<kDrain, LASTW>(L, t0, lane, n2, row_ok, open, extend, rowHo, rowF, sr);
        btw[(t0 / kGroup) * kStripe + lane] = L.acc;
    }
}

template <bool FAST, int WPG>
__global__ __launch_bounds__(64 * WPG) void sw_dp_kernel(SwDpArgs a)
{
    extern __shared__ int4 lds4[];
    const int wave = WPG > 1 ? int(threadIdx.x >> 6) : 0;
    const int lane = threadIdx.x & 63;
    const int idx = int(blockIdx.x) * WPG + wave;
    if (idx >= a.n) return;
    int* lds = reinterpret_cast<int*>(lds4) + size_t(wave) * (a.lds_wave_bytes / sizeof(int));
    const int p = a.order[idx];
    const SwPair P = a.pairs[p];
    const int n1 = __builtin_amdgcn_readfirstlane(P.n1);
    const int n2 = __builtin_amdgcn_readfirstlane(P.n2);
    const uint8_t* s1 = a.refs + P.ref_off;
    const uint8_t* s2 = a.alts + P.alt_off;

    // IntelSWAligner::is_all_match (intel_smithwaterman.hpp:47-58).
    if (a.shortcut && n1 == n2) {
        int mm = 0;
        for (int x = lane; x < n1; x += 64) mm += s1[x] != s2[x];
        if (wave_sum(mm) <= 2) {
            if (lane == 0) a.res[p] = SwResult{0, 0, 0, 1};
            return;
        }
    }

    const int slots = row_slots(a.n2max);
    int* rowH = lds;
    int* rowF = rowH + slots;
    uint8_t* altB = reinterpret_cast<uint8_t*>(rowF + fslots(a.n1max, a.n2max));   // 64 pads, columns, pads
    // H(i, n2) of every row goes to this pair's CIGAR-element scratch in HBM
    // (the trace kernel reuses it later); after the last stripe it is copied
    // into rowF, free by then, for the end-point scan.
    int* colG = reinterpret_cast<int*>(a.elems + P.el_off);
    const int open = a.open, extend = a.extend, ovh = a.overhang;
    const Scores sc{a.match, a.mismatch, open, extend};
    const int T = stripe_steps(n2);
    const int nstripes = (n1 + kStripe - 1) / kStripe;
    uint32_t* bt = a.bt + P.bt_off;
    const int nw = T / kGroup;
    int hofs = 0;   // the row buffer holds H + hofs

    if (FAST) {
        hofs = open;
        // Row 0 in this path's form: H(0, j) + open, F(0, j) + extend.
        for (int j = lane; j < kStripe + T + 2 * kGroup; j += 64) {
            rowH[j] = (j >= 64 ? boundary(ovh, open, extend, j - 63) : 0) + open;
            rowF[j] = kLow + extend;
        }
        for (int c = lane; c < kStripe + T + kGroup; c += 64)
            altB[c] = (c >= kStripe && c < kStripe + n2) ? s2[c - kStripe] : 0;
        wave_sync();
        const int open_v = in_vgpr(open), extend_v = in_vgpr(extend);
        Scorer sr;
        sr.mp = in_vgpr(a.match - open);
        sr.mmp = in_vgpr(a.mismatch - open);
        for (int s = 0; s < nstripes; ++s) {
            const int i = s * kStripe + lane + 1;
            const bool row_ok = i <= n1;
            PLane L;
            L.h = boundary(ovh, open, extend, i);   // H(i, 0)
            L.ex = kLow + extend;                    // E(i, 0) + extend (:199)
            L.fx = kLow + extend;
            L.dg = rowH[63];                         // lane 0: H(64s, 0) + open
            L.acc = 0;
            uint32_t* btw = bt + int64_t(s) * nw * kStripe;
            const bool lastw = s == nstripes - 1 && (n1 % kStripe) != 0;
            // A partial last stripe of r rows is done after n2 + r - 1 steps
            // (lane r - 1 leaves column n2), not n2 + 63: its unwritten
            // backtrack words lie past every cell the trace reads.
            const int Ts = lastw ? std::min(T, (n2 + (n1 - s * kStripe) + kGroup - 1) & ~(kGroup - 1)) : T;
            sr.rb = row_ok ? int(s1[i - 1]) : -1;   // never equals a byte
            sr.arow = altB + 64 - lane;
            if (lastw)
                pstripe<true>(L, lane, n2, row_ok, Ts, btw, open_v, extend_v, rowH, rowF, sr);
            else
                pstripe<false>(L, lane, n2, row_ok, T, btw, open_v, extend_v, rowH, rowF, sr);
            if (row_ok) colG[i] = L.h;   // H(i, n2): frozen since the lane left column n2
            wave_sync();
        }
    } else {
    // Row 0: H(0, j) = boundary, F(0, j) = LOW (PairWiseSW.h:72-75,198).
    for (int j = lane; j < kStripe + T; j += 64) {
        rowH[j] = j >= 64 ? boundary(ovh, open, extend, j - 63) : 0;
        rowF[j] = kLow;
    }
    for (int c = lane; c < kStripe + T + kGroup; c += 64) altB[c] = (c >= kStripe && c < kStripe + n2) ? s2[c - kStripe] : 0;
    wave_sync();

    for (int s = 0; s < nstripes; ++s) {
        const int i = s * kStripe + lane + 1;
        const bool row_ok = i <= n1;
        Lane L;
        L.h = boundary(ovh, open, extend, i);   // H(i, 0)
        L.e = kLow;                              // E(i, 0) (:199)
        L.f = kLow;
        L.diag = boundary(ovh, open, extend, s * kStripe);   // lane 0: H(64s, 0)
        L.acc = 0;
        const int rb = row_ok ? int(s1[i - 1]) : -1;   // never equals a byte
        uint32_t* btw = bt + int64_t(s) * nw * kStripe;
        if (s == nstripes - 1 && (n1 % kStripe) != 0)
            stripe<true, FAST>(L, lane, n2, rb, row_ok, T, btw, sc, rowH, rowF, altB);
        else
            stripe<false, FAST>(L, lane, n2, rb, row_ok, T, btw, sc, rowH, rowF, altB);
        if (row_ok) colG[i] = L.h;   // H(i, n2): frozen since the lane left column n2
        wave_sync();
    }
    }

    __threadfence_block();   // this wave's colG stores complete before its lanes read them back
    int* colC = rowF;
    for (int x = lane + 1; x <= n1; x += 64) colC[x] = colG[x];
    wave_sync();

    // End point (PairWiseSW.h:201-226): candidates in anti-diagonal order d =
    // 1..n1+n2, the last-row cell (n1, d-n1) before the last-column cell
    // (d-n2, n2); the last row counts only for SOFTCLIP / IGNORE. Every
    // candidate with the best score is then replayed in that order through the
    // reference's replacement rules.
    const bool use_row = ovh == 9 || ovh == 12;
    const int D = n1 + n2;
    int mx = INT_MIN;
    for (int d0 = 1; d0 <= D; d0 += 32) {
        const int d = d0 + (lane >> 1);
        const bool col = lane & 1;
        const bool ok = col ? (d > n2 && d <= D) : (use_row && d > n1 && d <= D);
        if (ok) mx = max(mx, col ? colC[d - n2] : rowH[63 + d - n1] - hofs);
    }
    const int best = wave_max(mx);
    int bi = 0, bj = 0;
    bool have = false;
    for (int d0 = 1; d0 <= D; d0 += 32) {
        const int d = d0 + (lane >> 1);
        const bool col = lane & 1;
        const bool ok = col ? (d > n2 && d <= D) : (use_row && d > n1 && d <= D);
        const bool tie = ok && (col ? colC[d - n2] : rowH[63 + d - n1] - hofs) == best;
        uint64_t m = __builtin_amdgcn_ballot_w64(tie);
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const int dd = d0 + (l >> 1);
            if (l & 1) {
                const int ci = dd - n2;
                if (!have || bj == n2 || abs(ci - n2) <= abs(bi - bj)) { bi = ci; bj = n2; have = true; }
            } else {
                const int cj = dd - n1;
                if (!have || abs(n1 - cj) < abs(bi - bj)) { bi = n1; bj = cj; have = true; }
            }
        }
    }
    if (lane == 0) a.res[p] = SwResult{best, bi, bj, 0};
}

// 4-bit backtrack code of cell (i, j), 1-based (layout of sw_dp_kernel:
// [stripe][word][lane]).
__device__ __forceinline__ int bt_nibble(const uint32_t* bt, int nw, int i, int j)
{
    const int k = (i - 1) & (kStripe - 1), s = (i - 1) / kStripe;
    const int t = j - 1 + k;
    const uint32_t w = bt[(int64_t(s) * nw + (t >> 3)) * kStripe + k];
    return (w >> ((7 - (t & 7)) * 4)) & 15;
}

// getCIGAR (PairWiseSW.h:240-415), one wave per pair. The walk is the
// reference's state machine; the wave fetches the next 64 cells along the
// direction the state implies (diagonal while matching, along the row in an
// insertion, along the column in a deletion), finds with one ballot where the
// direction changes, takes the whole run at once and applies the one cell that
// changes it. Equal neighbours are merged on the fly (the reference merges them
// afterwards, :368-386: same result). Elements are written CIGAR-end first,
// to the pair's scratch and (the first kSlotElems, 16 bits each) to its slot.
__global__ __launch_bounds__(256) void sw_trace_kernel(SwTraceArgs a)
{
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= a.n) return;
    const SwPair P = a.pairs[p];
    const SwResult r = a.res[p];
    uint32_t* el = a.elems + P.el_off;
    const int n1 = __builtin_amdgcn_readfirstlane(P.n1), n2 = __builtin_amdgcn_readfirstlane(P.n2);
    if (__builtin_amdgcn_readfirstlane(r.shortcut)) {
        if (lane == 0) {
            a.slots[int64_t(p) * kSlotElems] = uint16_t((n1 << 4) | kOpM);
            a.n_elems[p] = 1;
            a.offsets[p] = 0;
        }
        return;
    }
    const uint32_t* bt = a.bt + P.bt_off;
    const int nw = stripe_steps(n2) / kGroup;
    const int ovh = a.overhang;
    int i = __builtin_amdgcn_readfirstlane(r.max_i), j = __builtin_amdgcn_readfirstlane(r.max_j);
    if (ovh == 10) {
        i = n1;
        j = n2;
    } else if (ovh == 11) {
        j = n2;
    }
    int cnt = 0, cop = -1, len = 0;   // uniform; lane 0 stores
    auto push = [&](int nop, int nlen) {
        if (nop == cop) {
            len += nlen;
        } else {
            if (cop >= 0 && lane == 0) el[cnt] = (uint32_t(len) << 4) | uint32_t(cop);
            cnt += cop >= 0;
            cop = nop;
            len = nlen;
        }
    };
    if (j < n2) push(kOpS, n2 - j);
    int state = 0;
    while (i > 0 && j > 0) {
        const int di = state == 4 ? 0 : lane, dj = state == 8 ? 0 : lane;
        const int ci = i - di, cj = j - dj;
        const bool valid = ci > 0 && cj > 0;
        const int b = valid ? bt_nibble(bt, nw, ci, cj) : 0;
        // nibble [eo > ee][fo > fe][E wins][F wins] (see step): the reference's
        // code is op | INSERT_EXT(4) | DELETE_EXT(8), the EXT bits being "not open".
        const int op = (b & 1) ? kOpD : (b & 2) ? kOpI : kOpM;
        const bool ins_ext = !(b & 8), del_ext = !(b & 4);
        if (state == 0) {
            const uint64_t brk = __builtin_amdgcn_ballot_w64(!(valid && op == kOpM));
            const int k = brk ? __builtin_ctzll(brk) : 64;
            if (k > 0) push(kOpM, k);
            i -= k;
            j -= k;
            if (k < 64 && i > 0 && j > 0) {   // cell k: an insertion or deletion opens
                const int bk = __builtin_amdgcn_readlane(b, k);
                if (bk & 1) {
                    --i;
                    push(kOpD, 1);
                    state = (bk & 4) ? 0 : 8;
                } else {
                    --j;
                    push(kOpI, 1);
                    state = (bk & 8) ? 0 : 4;
                }
            }
        } else {
            // In an insertion (deletion) every cell is consumed along the row
            // (column); the run goes on while the consumed cell's EXT bit is set.
            const bool go = valid && (state == 4 ? ins_ext : del_ext);
            const uint64_t brk = __builtin_amdgcn_ballot_w64(!go);
            const int k = brk ? __builtin_ctzll(brk) : 64;
            const bool kv = k < 64 && ((state == 4 ? j - k : i - k) > 0);
            const int take = k + (kv ? 1 : 0);   // cell k is consumed too, and ends the run
            push(state == 4 ? kOpI : kOpD, take);
            if (state == 4) j -= take;
            else i -= take;
            if (k < 64) state = 0;
        }
    }
    int offset;
    if (ovh == 9) {
        if (j > 0) push(kOpS, j);
        offset = i;
    } else if (ovh == 12) {
        if (j > 0) len += j;   // the last element repeated over the overhang (:345-352)
        offset = i - j;
    } else {
        if (i > 0) push(kOpD, i);
        else if (j > 0) push(kOpI, j);
        offset = 0;
    }
    if (cop >= 0) {
        if (lane == 0) el[cnt] = (uint32_t(len) << 4) | uint32_t(cop);
        ++cnt;
    }
    __threadfence_block();   // lane 0's element stores are visible to the other lanes
    if (lane < kSlotElems && lane < cnt) a.slots[int64_t(p) * kSlotElems + lane] = uint16_t(el[lane]);
    if (lane == 0) {
        a.n_elems[p] = cnt;
        a.offsets[p] = offset;
    }
}

}  // namespace

size_t dp_lds_bytes(int n1max, int n2max)
{
    // [rowH | rowF | altB]
    const size_t rows = sizeof(int) * (size_t(row_slots(n2max)) + size_t(fslots(n1max, n2max)));
    return rows + size_t(alt_slots(n2max));
}

hipError_t launch_dp(const SwDpArgs& a, int n1max, hipStream_t s)
{
    if (a.n <= 0) return hipSuccess;
    SwDpArgs b = a;
    b.lds_wave_bytes = int((dp_lds_bytes(n1max, a.n2max) + 15) & ~size_t(15));
    const int wpg = a.wpg == 4 ? 4 : a.wpg == 2 ? 2 : 1;
    const size_t lds = size_t(b.lds_wave_bytes) * wpg;
    const dim3 grid((a.n + wpg - 1) / wpg), block(64 * wpg);
    if (a.fast) {
        if (wpg == 4) hipLaunchKernelGGL((sw_dp_kernel<true, 4>), grid, block, lds, s, b);
        else if (wpg == 2) hipLaunchKernelGGL((sw_dp_kernel<true, 2>), grid, block, lds, s, b);
        else hipLaunchKernelGGL((sw_dp_kernel<true, 1>), grid, block, lds, s, b);
    } else {
        if (wpg == 4) hipLaunchKernelGGL((sw_dp_kernel<false, 4>), grid, block, lds, s, b);
        else if (wpg == 2) hipLaunchKernelGGL((sw_dp_kernel<false, 2>), grid, block, lds, s, b);
        else hipLaunchKernelGGL((sw_dp_kernel<false, 1>), grid, block, lds, s, b);
    }
    return hipGetLastError();
}

hipError_t launch_trace(const SwTraceArgs& a, hipStream_t s)
{
    if (a.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(sw_trace_kernel, dim3((a.n + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcsw
