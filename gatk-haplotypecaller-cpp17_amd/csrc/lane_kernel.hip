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
//   phmm_seg_kernel   (fp32)  column-segmented waves (planned on the host or, for
//                             flat calls, on the device): a pair
//                             over ceil(H/BC) consecutive lanes, one row of skew
//                             per lane, values handed right by DPP (run_seg);
//   phmm_seg64_kernel (fp64)  the rescue pass in the same form, planned on the
//                             device from the rescue list (rescue_plan_kernel);
//   phmm_lane_kernel  (fp32)  one lane per pair, blocks chained through a
//                             global carry buffer (haps too long to segment).
#include <algorithm>
#include <type_traits>

#include "seg_common.hpp"

namespace hcphmm {
namespace {
using namespace seg;

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
            mt[c * 64 + lane] = make_uint2(hap_word(cx, w0 * 5 + c), (BC > 32) ? hap_word(cx, w1 * 5 + c) : 0u);
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
    uint32_t wc = row_word(cx, 0), wn = row_word(cx, min(2, cx.R) - 1);
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
        const uint32_t wnn = row_word(cx, min(i + 2, cx.R) - 1);
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
        cell<float, BC, 0, NC, SUM, EQ, true>(T, X, M0, Ml, Yl, mrow.x, mrow.y, k.pm, k.px, k, lim, sumM, sumX);
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
__device__ __forceinline__ void emit(const LaneArgs& a, int pid, float raw, int R, int H)
{
    a.raw_out[pid] = raw;
    const bool resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
    a.rescue_flag[pid] = resc;
    a.raw64_zero[pid] = 0.0;
    if (resc) {
        const int pos = atomicAdd(a.rescue_count, 1);
        a.rescue_list[pos] = pid;
        a.rescue_rh[pos] = pack_rh(R, H);
    }
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
    const uint32_t w1 = row_word(cx, 0);
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
    if (active) emit(a, pid, sumM + sumX, cx.R, cx.H);
}

// Column-segmented fp32 waves (host-planned). The wave's npairs pairs are the
// slots slot0 .. slot0+npairs-1; pair g takes nb_g = ceil(H_g / BC) consecutive
// lanes in slot order. Lanes past the last group idle (s = 0, no output).
// Seg waves per workgroup (HC_SEG_WPB, A/B builds: EXTRA_DEV_FLAGS=-DHC_SEG_WPB=n).
// A workgroup is dispatched when a CU has room for all its waves, so with 4
// the slot a finished wave frees can wait for its workgroup's others (a 125k
// pass spent 18 % of its SIMD time at 2 resident waves). One wave per
// workgroup (each wave has its own LDS tables): S2 8.64 -> 8.59 ms, S1 and
// the shard sizes unchanged (profiles/r04_wpb_ab.txt).
#ifndef HC_SEG_WPB
#define HC_SEG_WPB 1
#endif
constexpr int kSegWPB = HC_SEG_WPB;
// ---------------------------------------------------------------------------
// fp64 rescue pass (intel_pairhmm.hpp:137-139) in column-segmented form.
//
// The rescue list is built on the device by the fp32 pass, so the waves are
// planned on the device too: rescue_plan_kernel picks the pass's block width
// bound bc0 (32 columns, narrower when the list is too short to give every
// SIMD two waves: short lists are latency-bound), gives every pair a slot of
// 2^k lanes with k = ceil(log2(ceil(H/bc0))) (64 lanes if that needs more),
// and then the narrowest fp64 width covering the hap on those 2^k lanes, so a
// pair's slot has no idle lanes (a 1 100-column hap: 64 lanes of 20 columns,
// not 35 lanes of 32 in a 64-lane slot). The list is scattered into class
// order, classes with the longest waves first (order inside a class is
// arbitrary; each pair's result is independent of it). Pairs needing more
// than 64 lanes of 32 columns go to the anti-diagonal fp64 kernel through `big`.

__device__ __forceinline__ int ceil_log2(int nb) { return nb <= 1 ? 0 : 32 - __clz(nb - 1); }

__device__ __forceinline__ int rescue_class(int H, int bc0)
{
    const int nb0 = (H + bc0 - 1) / bc0;
    const int k = nb0 <= 64 ? ceil_log2(nb0) : 6;
    const int need = (H + (1 << k) - 1) >> k;   // columns per lane on 2^k lanes (<= bc0 when nb0 <= 64)
    if (need > seg64_width(kSeg64Widths - 1)) return kSeg64Classes - 1;
    const int wi = need <= 8 ? 0 : (need - 8 + 3) / 4;
    return kChainClasses + (6 - k) * kSeg64Widths + (kSeg64Widths - 1 - wi);
}
// Class c's lanes per pair (log2) and block width; the chain classes are
// 64-lane classes (their pairs one after the other, not side by side).
__device__ __forceinline__ int class_k(int c)
{
    return c < kChainClasses ? 6 : 6 - (c - kChainClasses) / kSeg64Widths;
}
__device__ __forceinline__ int class_bc(int c)
{
    return seg64_width(kSeg64Widths - 1 - (c < kChainClasses ? c : c - kChainClasses) % kSeg64Widths);
}

// Wave order of the pass. With at most two waves per SIMD (fp64 occupancy)
// every wave is resident at once and the pass lasts as long as its busiest
// SIMD: position p and p + n_simd share a SIMD (workgroups of four waves, the
// first n_simd positions filling one slot per SIMD), so the heaviest waves go
// first, in descending cost, and the rest after them in ascending cost — the
// heaviest wave shares its SIMD with the lightest. With more, waves are
// fetched from a counter in descending cost (greedy longest-first). Wave
// cost: (rows + skew) steps x (14 ops per column + ~40 per step), sorted by a
// counting sort over 256 cost buckets (order inside a bucket is arbitrary).
constexpr int kMaxSortWaves = 8192;
constexpr int kPlanThreads = 256;   // the planning workgroup (a phmm_seg64_kernel workgroup)
constexpr int kPlanPhases = 6;      // (diagnostics) the planner's phase stamps
constexpr int kPlanCopies = 16;     // PlanLds counter copies

struct PlanLds {
    int cnt[kSeg64Classes], wbase[kSeg64Classes], off[kSeg64Classes];
    // Class counts at the pass's bc0 and the scatter's cursors, in
    // kPlanCopies copies by lane (lane & 15), so a class's LDS atomics from
    // one wave hit 16 addresses, not one.
    int cntx[kPlanCopies][kSeg64Classes];
    int fillx[kPlanCopies][kSeg64Classes];
    int chain;
    alignas(16) int hist[256];
    unsigned long long lanes;
    unsigned cmax;
    unsigned long long phase[kPlanPhases];
    unsigned cost[kMaxSortWaves];
};

// The planner is one workgroup walking the list: each thread takes
// kPlanBatch entries at a time, their pair ids and their R and H (written
// beside the list by the fp32 pass: coalesced loads; gathering them from the
// pair descriptors, 37 000 scattered lines for S4-20k from one CU, took its
// count and scatter walks 34 and 40 us). f(pid, R, H) per listed pair.
constexpr int kPlanBatch = 16;
template <bool PID = true, typename F>
__device__ __forceinline__ void plan_walk(const Seg64Args& a, int n, F&& f)
{
    for (int b = threadIdx.x; b < n; b += kPlanBatch * kPlanThreads) {
        int pid[kPlanBatch];
        int2 rh[kPlanBatch];
#pragma unroll
        for (int k = 0; k < kPlanBatch; ++k) {
            const int i = b + k * kPlanThreads;
            pid[k] = i < n ? (PID ? a.list[i] : 0) : -1;
        }
#pragma unroll
        for (int k = 0; k < kPlanBatch; ++k) {   // R and H beside the list (coalesced)
            const int i = b + k * kPlanThreads;
            const unsigned v = i < n ? unsigned(a.list_rh[i]) : 0u;
            rh[k] = make_int2(int(v >> 16), int(v & 0xffffu));
        }
#pragma unroll
        for (int k = 0; k < kPlanBatch; ++k)
            if (pid[k] >= 0) f(pid[k], rh[k].x, rh[k].y);
    }
}

// Modelled costs of waves [0, W) into L.cost (and their maximum into L.cmax):
// steps x (14 ops per column + ~40 per step), steps = max R + skew (pairs side
// by side) or sum of R + skew (a chain). L.cost[w] holds wave w's max / sum of
// R on entry (aggregated in LDS by the scatter: no loads here).
__device__ __forceinline__ void wave_costs(PlanLds& L, int W)
{
    constexpr int NC = kSeg64Classes;
    unsigned cm = 0;
    for (int w = threadIdx.x; w < W; w += kPlanThreads) {
        int lo = 0, hi = NC - 1;   // wave w's class: the last whose first wave is <= w
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (L.wbase[mid] <= w) lo = mid;
            else hi = mid;
        }
        const int steps = int(L.cost[w]) + (1 << class_k(lo)) - 1;
        const unsigned cost = unsigned(steps) * unsigned(class_bc(lo) * 14 + 40);
        L.cost[w] = cost;
        cm = max(cm, cost);
    }
    if (cm) atomicMax(&L.cmax, cm);
}

// (diagnostics) phase stamp i of the planner, after a barrier
__device__ __forceinline__ void plan_stamp(const Seg64Args& a, PlanLds& L, int i)
{
    if (a.timeline && threadIdx.x == 0) L.phase[i] = __builtin_amdgcn_s_memrealtime();
}

// Exclusive prefix sum over the 64 lanes of a wave (and the total).
__device__ __forceinline__ int wave_excl_scan(int v, int& total)
{
    const int lane = __lane_id();
    int inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(inc, d, 64);
        if (lane >= d) inc += u;
    }
    total = __shfl(inc, 63, 64);
    return inc - v;
}

// The fp64 pass's plan over the n > 0 listed pairs, by one workgroup of the
// fp64 launch (the first to arrive; the others wait for its flag): the width
// bound bc0 (32 unless the lanes at width 32 give fewer than min_lanes, 2
// waves per SIMD, then 16, then 8), the classes (and in passes of many waves
// the chains), the list scattered into class order (`sorted`; the last class
// into `big`), and the dispatch order.
// Its time is on the pass's critical path (every other workgroup waits) and
// it is load latency, so the list is walked twice only: once counting the
// classes at all three candidate bc0 together (with the lanes that choose
// bc0), once scattering (and aggregating each wave's R in LDS); the class
// table is one wave's scans. (Three walks, a serial class table and the
// costs' dependent descriptor loads: 55 us from the fp32 pass's last wave to
// the first fp64 wave on S4, 91 us on S4-20k, profiles/r06_timeline_*.)
__device__ __forceinline__ void plan_rescue(const Seg64Args& a, int n, PlanLds& L)
{
    constexpr int NC = kSeg64Classes;
    static_assert(NC <= 64, "the class table is one wave");
    const int t = threadIdx.x;
    for (int q = t; q < kPlanCopies * NC; q += kPlanThreads) (&L.cntx[0][0])[q] = 0;
    const int cp = t & (kPlanCopies - 1);   // this thread's counter copy
    if (t == 0) {
        L.lanes = 0;
        L.cmax = 1;
        *a.next_wave = 0;
    }
    __syncthreads();
    // The lanes at width 32 (which choose bc0), then the class counts at that
    // bc0: the LDS atomics are the walks' cost (one lane-op a cycle per CU:
    // counting all three candidate bc0 in one walk took S4-20k's 52 us), the
    // loads beside them are coalesced (list_rh).
    unsigned long long mine = 0;
    plan_walk<false>(a, n, [&](int, int, int H) { mine += (H + 31) / 32; });
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mine += __shfl_xor(mine, d, 64);
    if (__lane_id() == 0 && mine) atomicAdd(&L.lanes, mine);
    __syncthreads();
    const long long l32 = (long long)L.lanes;
    const int b3 = l32 >= a.min_lanes ? 0 : (2 * l32 >= a.min_lanes ? 1 : 2);
    const int bc0 = 32 >> b3;
    plan_walk<false>(a, n, [&](int, int, int H) { atomicAdd(&L.cntx[cp][rescue_class(H, bc0)], 1); });
    __syncthreads();
    plan_stamp(a, L, 0);
    if (t < 64) {   // the class table: lane c holds class c
        const int c = t;
        const int S = a.n_simd;
        const bool real = c >= kChainClasses && c < NC;
        int n0 = 0;
        if (real) {   // the copies' counts, and each copy's first place in the class (the scatter's cursors)
            for (int k = 0; k < kPlanCopies; ++k) {
                L.fillx[k][c] = n0;
                n0 += L.cntx[k][c];
            }
        } else if (c < NC) {
            for (int k = 0; k < kPlanCopies; ++k) L.fillx[k][c] = 0;
        }
        const int per0 = 64 >> class_k(min(c, NC - 1));
        int w_all, n64;
        (void)wave_excl_scan(real && c < NC - 1 ? (n0 + per0 - 1) / per0 : 0, w_all);
        const bool is64 = c >= kChainClasses && c < kChainClasses + kSeg64Widths;   // 64-lane classes
        (void)wave_excl_scan(is64 ? n0 : 0, n64);
        // Chains only in passes of many waves (fetched greedily), and only the
        // 64-lane pairs past chain_tail rounds of single waves (two per SIMD),
        // so the greedy order still ends on short waves; spread over the
        // widths by their share.
        const int L_ch = (a.wave_order && a.chain > 1 && w_all > 2 * S) ? a.chain : 1;
        const long long chained = L_ch > 1 ? max(0LL, (long long)n64 - (long long)a.chain_tail * 2 * S) : 0;
        const int cc = is64 && chained > 0 ? int((long long)n0 * chained / n64) / L_ch * L_ch : 0;
        const int cc_chain = __shfl(cc, c + kChainClasses < 64 ? c + kChainClasses : c, 64);   // chain class c's pairs
        const int nc = c < kChainClasses ? cc_chain : n0 - cc;
        const int per = c < kChainClasses ? L_ch : per0;
        int tot_n, tot_w;
        const int off = wave_excl_scan(c < NC ? nc : 0, tot_n);
        const int wb = wave_excl_scan(c < NC - 1 ? (nc + per - 1) / per : 0, tot_w);
        if (c < NC) {
            Seg64Plan* __restrict__ p = a.plan;
            L.cnt[c] = nc;
            L.off[c] = off;
            L.wbase[c] = wb;
            p->n_class[c] = nc;
            p->off_class[c] = off;
            p->wave_base[c] = wb;
            if (c == NC - 1) *a.big_count = nc;
        }
        if (c == 0) {
            L.chain = L_ch;
            a.plan->bc0 = bc0;
            a.plan->chain = L_ch;
            a.plan->dynamic = a.wave_order != nullptr && w_all > 2 * S;
        }
    }
    __syncthreads();
    const int W = L.wbase[NC - 1];   // segmented waves
    const bool sort = W > 1 && a.wave_order && W <= kMaxSortWaves;
    if (sort) {   // the waves' R aggregates (max, or sum for a chain), filled by the scatter
        for (int w = t; w < W; w += kPlanThreads) L.cost[w] = 0;
        __syncthreads();
    }
    plan_stamp(a, L, 1);
    plan_walk(a, n, [&](int pid, int R, int H) {
        const int c = rescue_class(H, bc0);
        const int q = atomicAdd(&L.fillx[cp][c], 1);   // this pair's place in its class
        if (c == NC - 1) {
            a.big[q] = pid;
            return;
        }
        // A 64-lane class's first pairs go to its chain class.
        const bool c64 = c < kChainClasses + kSeg64Widths;
        const int ch = c - kChainClasses;
        const int nch = c64 ? L.cnt[ch] : 0;
        const bool chained = q < nch;
        const int cls = chained ? ch : c, idx = chained ? q : q - nch;
        a.sorted[L.off[cls] + idx] = pid;
        if (sort) {
            const int w = L.wbase[cls] + (chained ? idx / L.chain : idx >> (6 - class_k(cls)));
            if (chained)
                atomicAdd(&L.cost[w], unsigned(R));
            else
                atomicMax(&L.cost[w], unsigned(R));
        }
    });
    __syncthreads();
    plan_stamp(a, L, 2);
    if (W <= 1 || !a.wave_order) return;
    if (W > kMaxSortWaves) {   // classes longest first, fetched in that order
        for (int w = t; w < W; w += kPlanThreads) a.wave_order[w] = w;
        return;
    }
    // Costs, then a counting sort by cost descending over 256 buckets.
    wave_costs(L, W);
    L.hist[t] = 0;
    __syncthreads();
    plan_stamp(a, L, 3);
    const unsigned cmax = L.cmax;
    auto bucket = [&](unsigned c) { return 255 - int((unsigned long long)c * 255 / cmax); };   // 0: costliest
    for (int w = t; w < W; w += kPlanThreads) atomicAdd(&L.hist[bucket(L.cost[w])], 1);
    __syncthreads();
    if (t < 64) {   // exclusive prefix over the buckets: one wave, 4 buckets a lane
        const int4 h = reinterpret_cast<const int4*>(L.hist)[t];
        int tot;
        const int ex = wave_excl_scan(h.x + h.y + h.z + h.w, tot);
        reinterpret_cast<int4*>(L.hist)[t] = make_int4(ex, ex + h.x, ex + h.x + h.y, ex + h.x + h.y + h.z);
    }
    __syncthreads();
    plan_stamp(a, L, 4);
    const int S = a.n_simd;
    for (int w = t; w < W; w += kPlanThreads) {
        const int r = atomicAdd(&L.hist[bucket(L.cost[w])], 1);   // rank in descending cost
        // At most two waves per SIMD (positions p and p + S share one): the
        // heaviest S waves first, then the rest paired heaviest with lightest.
        // (The 2S - W heaviest alone on a SIMD first measured slower: S4's fp64
        // pass 0.490 vs 0.441 ms; class order without the sort 0.488.)
        const int pos = (W > S && W <= 2 * S && r >= S) ? S + (W - 1 - r) : r;
        a.wave_order[pos] = w;
    }
}

// One column-segmented wave (wid) of the fp32 pass.
__device__ __forceinline__ void seg_wave(const LaneArgs& a, int wid, const float* __restrict__ slut)
{
    // Lane id and the wave's LDS tables in forms the compiler can recompute
    // (mbcnt) or keep in SGPRs (wave-uniform): values live across the step
    // loop that it would otherwise spill at every wave's start.
    const int lane = __lane_id();
    const unsigned long long t_start = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
    const LaneWave wv = load_wave(a.waves, wid);
    const int bc = wv.ncols;
    __shared__ uint2 mtab[kSegWPB][5 * 64];
    uint2* mt = mtab[__builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6))];
    // Lane -> (group, block): group g's lanes start at the prefix sum of nb.
    int* gmap = reinterpret_cast<int*>(mt);   // 128 ints, used before the match table
    int nb_g = 0;
    if (lane < wv.npairs) nb_g = (a.sdesc[wv.slot0 + lane].w + bc - 1) / bc;
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
    const int slot = wv.slot0 + (g >= 0 ? g : 0);
    const LaneCtx cx = desc_ctx(a.sdesc[slot], a.rows, a.hapw);   // slot-ordered: no order -> pairs indirection
    const int pid = a.order[slot];   // needed only to write results by pair id
    const bool owner = g >= 0 && s == (cx.H + bc - 1) / bc - 1;
    if (g < 0) s = 0;
    const uint32_t w1 = row_word(cx, 0);
    const float T0 = row0_t<float>(a.lut, w1, cx.H);
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!read_eq(w1)) == 0;
    const SegSteps st{wv.rmax, wv.rmin, wv.nsteps, a.prio};
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
        if (a.rec) {
            // The wave's pairs own consecutive slots: one 16-byte record each,
            // contiguous over the wave (3 partial lines per pair by pair id
            // before: 0.2 GB of writes per S2 launch for 13 MB of results).
            // A rescue in this wave rewrites the state and raw f64 after this.
            a.rec[slot] = make_uint4(__float_as_uint(raw), resc ? kRecListed : kRecPlain, 0u, 0u);
        } else {
            a.raw_out[pid] = raw;
            a.rescue_flag[pid] = resc;
            if (!resc) a.raw64_zero[pid] = 0.0;
        }
    }
    const uint64_t todo = __builtin_amdgcn_ballot_w64(resc);
    if (todo) rescue_in_wave(a, todo, pid, slot, cx.H, cx.R, lane, mt);
    if (a.timeline && lane == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        a.timeline[3 * size_t(wid)] = t_start;
        a.timeline[3 * size_t(wid) + 1] = t_end;
        // HW_ID (CU / SIMD / SE) in the low word, XCC_ID (hwreg 20) above it
        a.timeline[3 * size_t(wid) + 2] = (unsigned long long)unsigned(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))) |
                                          ((unsigned long long)unsigned(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11))) << 32);
    }
}

template <int OCC>
__global__ __launch_bounds__(64 * kSegWPB, OCC) void phmm_seg_kernel(LaneArgs a)
{
    // Each wave fills its own copy of the prior tables: no workgroup barrier
    // between the kernel's start and a wave's first loads, so the fill
    // overlaps the wave's descriptor loads (small batches are one round of
    // waves: every wave's start-up latency is on the pass's critical path).
    __shared__ float sluts[kSegWPB][kSlutLen];
    const int n_waves = a.n_waves_dev ? __builtin_amdgcn_readfirstlane(*a.n_waves_dev) : a.n_waves;
    const int wib = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
    const int wid = blockIdx.x * kSegWPB + wib;
    if (a.solo_counters && blockIdx.x == 0 && threadIdx.x == 0) {
        // No fp64 launch follows: the other parity's counters for the next run
        // (its last run's kernels are complete: stream order).
        int* c = a.solo_counters;
        const int o = a.solo_other;
        c[o] = 0;                 // rescue list length
        c[2 + o] = 0;             // in-wave rescues
        c[kPlanTicket + o] = 0;
        c[kPlanReady + o] = 0;
    }
    if (wid >= n_waves) return;   // wave-uniform (device-planned parts launch an upper bound)
    float* slut = sluts[wib];
    for (int t = __lane_id(); t < kSlutLen; t += 64) slut[t] = a.lut[t];
    __builtin_amdgcn_wave_barrier();
    seg_wave(a, wid, slut);
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

// Diagnostics (Seg64Args::timeline): wave w's record.
__device__ __forceinline__ void wave_record(const Seg64Args& a, int w, unsigned long long t_start, int pid)
{
    a.timeline[3 * size_t(w)] = t_start;
    a.timeline[3 * size_t(w) + 1] = __builtin_amdgcn_s_memrealtime();
    a.timeline[3 * size_t(w) + 2] =
        (unsigned long long)unsigned(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))) |
        ((unsigned long long)unsigned(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11))) << 32) |
        ((unsigned long long)unsigned(pid) << 40);
}

// Wave wk of a class of 2^k-lane slots (entries [ok, ok + nk) of `sorted`):
// its pairs side by side, 64 >> k of them, each over 2^k lanes of bc columns
// (seg_common.hpp run_seg). Returns the lane's pair id.
__device__ __forceinline__ int slot_wave(const Seg64Args& a, const double* __restrict__ slut, uint2* __restrict__ mt,
                                         int lane, int k, int bc, int ok, int nk, int wk, int pmode)
{
    const int e = wk * (64 >> k) + (lane >> k);
    const bool valid = e < nk;
    int s = lane & ((1 << k) - 1);
    const int pid = a.sorted[ok + (valid ? e : wk * (64 >> k))];
    const LaneCtx cx = pair_ctx(a.pairs, a.rows, a.hapw, pid);
    const int nb = (cx.H + bc - 1) / bc;
    const bool owner = valid && s == nb - 1;
    if (!valid) s = 0;
    const SegSteps st{wave_max(valid ? cx.R : 0), wave_min(valid ? cx.R : INT32_MAX),
                      wave_max(valid ? cx.R + nb - 1 : 0), pmode, __builtin_amdgcn_s_memrealtime()};
    const uint32_t w1 = row_word(cx, 0);
    const double T0 = row0_t<double>(a.lut, w1, cx.H);
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!read_eq(w1)) == 0;
    double sumM = 0.0, sumX = 0.0;
    switch (bc) {
#define HC_SEG64_CASE(WI) \
    case seg64_width(WI): run_seg_bc<double, seg64_width(WI)>(a.lut, slut, st, lane, s, cx, T0, sumM, sumX, mt, wave_eq); break;
        HC_SEG64_CASE(0) HC_SEG64_CASE(1) HC_SEG64_CASE(2) HC_SEG64_CASE(3) HC_SEG64_CASE(4) HC_SEG64_CASE(5)
        HC_SEG64_CASE(6)
#undef HC_SEG64_CASE
    default: break;
    }
    if (owner) a.raw_out[pid] = sumM + sumX;
    return pid;
}

// A chain's pairs (wave-uniform, in LDS): descriptor fields, the first row
// word (the constant-gap check) and row 0's diagonal T0.
struct ChainEnt {
    int pid, R, H, nb;
    unsigned rb, hb, w1, pad_;
    double T0;
};
constexpr int kMtSlot = 5 * 64;   // one pair's match windows (uint2 per lane and read code)

// A chain wave: np <= kMaxChain pairs of one 64-lane class (entries e0 ..
// e0 + np - 1 of `sorted`) streamed through the same lanes one after the
// other. Lane s sweeps global row g = k - s of the rows of pair 0, then pair
// 1, ... (run_seg's column-segmented recurrence, EQ path): on reaching row 1
// of the next pair it hands its owner's sums out, resets its block to that
// pair's row 0 (T0 from column 0 on, X = 0) and takes its diagonal T0 and its
// match window, so the pipeline fill and drain of 63 steps is paid once per
// chain, not once per pair (S4-20k: R ~ 200 rows + 63 skew steps per pair).
// The hand-offs need no change: lane s-1 is one row ahead in the same global
// row order. The next row's word comes from the next pair's rows once past
// the current pair's R (the prefetch base switches a row early). Every pair
// must be an EQ read with the same gap constants (the reference's constant
// 'I'/'I'/'+'): else returns false and the caller runs the pairs one by one.
template <int BC>
__device__ __forceinline__ bool chain_run(const Seg64Args& a, const double* __restrict__ slut, uint2* __restrict__ mt,
                                          ChainEnt* __restrict__ ce, int lane, int e0, int np, int pmode)
{
    using T = double;
    constexpr bool AND = BC * int(sizeof(T)) <= 128;
    if (lane < np) {
        const int pid = a.sorted[e0 + lane];
        const LaneCtx cx = pair_ctx(a.pairs, a.rows, a.hapw, pid);
        const uint32_t w1 = row_word(cx, 0);
        ChainEnt e;
        e.pid = pid;
        e.R = cx.R;
        e.H = cx.H;
        e.nb = (cx.H + BC - 1) / BC;
        e.rb = cx.rbyte;
        e.hb = cx.hbyte;
        e.w1 = w1;
        e.pad_ = 0;
        e.T0 = row0_t<T>(a.lut, w1, cx.H);
        ce[lane] = e;
    }
    // (one wave: its LDS operations are in order; the fences keep the compiler's too)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t wa = ce[0].w1;
    bool ok = read_eq(wa);
    for (int q = 1; q < np; ++q) {
        const uint32_t w = ce[q].w1;
        ok = ok && read_eq(w) && row_i(w) == row_i(wa) && row_c(w) == row_c(wa);
    }
    if (!__builtin_amdgcn_readfirstlane(ok ? 1 : 0)) return false;
    for (int q = 0; q < np; ++q) {
        const ChainEnt e = ce[q];
        const LaneCtx cx{a.rows - kRowPadBefore, e.rb, a.hapw, e.hb, e.R, e.H};
        fill_window(mt + q * kMtSlot, lane, cx, lane * BC - (e.nb * BC - e.H));
    }
    const ChainEnt ea = ce[0];
    const LaneCtx cx0{a.rows - kRowPadBefore, ea.rb, a.hapw, ea.hb, ea.R, ea.H};
    const char* rbase = reinterpret_cast<const char*>(a.rows - kRowPadBefore);
    int q = 0, G = 0, Rc = ea.R;
    unsigned rbc = ea.rb;
    unsigned rbn = np > 1 ? ce[1].rb - unsigned(Rc) * 4u : rbc;   // word widx >= Rc: the next pair's widx - Rc
    T Tt[BC], X[BC];
    const int c0a = lane * BC - (ea.nb * BC - ea.H);
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        Tt[j] = c0a + j + 1 >= 0 ? ea.T0 : T(0);
        X[j] = T(0);
    }
    uint32_t wq = row_word(cx0, min(max(2 - lane, 1), Rc) - 1);   // the word of row i + 1 (PD = 1)
    // The gap constants are the chain's (checked above): wave-uniform, so
    // scalar loads and SGPRs (the per-lane form of run_seg spills here).
    RowConst<T> k;
    row_const<T>(a.lut, __builtin_amdgcn_readfirstlane(row_word(cx0, 0)),
                 __builtin_amdgcn_readfirstlane(row_word(cx0, min(2, Rc) - 1)), k);
    uint2 mrow = mt[k.rc * 64 + lane];
    uint32_t keep = (lane + 1) * BC < ea.H ? 0xffffffffu : 0u;
    T y_out = T(0);
    T t_out = masked<AND>(ea.T0, keep);
    T t_hold = c0a >= 0 ? ea.T0 : T(0);
    T sumM = T(0), sumX = T(0);
    auto step = [&](int kk, auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        int i = kk - lane - G;   // this lane's row of its current pair
        if (i > Rc && q + 1 < np) {   // row 1 of the next pair (once per pair and lane)
            if (lane == ce[q].nb - 1) a.raw_out[ce[q].pid] = sumM + sumX;   // the finished pair's owner
            G += Rc;
            i -= Rc;
            ++q;
            const ChainEnt e = ce[q];
            Rc = e.R;
            rbc = e.rb;
            rbn = q + 1 < np ? ce[q + 1].rb - unsigned(Rc) * 4u : rbc;
            const int c0 = lane * BC - (e.nb * BC - e.H);
            keep = (lane + 1) * BC < e.H ? 0xffffffffu : 0u;
            const T T0 = e.T0;
#pragma unroll
            for (int j = 0; j < BC; ++j) {
                Tt[j] = T0;
                X[j] = T(0);
            }
            if (c0 < -1) {   // block 0's padding columns: 0 left of column 0
#pragma unroll
                for (int j = 0; j < BC; ++j)
                    if (c0 + j + 1 < 0) Tt[j] = T(0);
            }
            t_hold = c0 >= 0 ? T0 : T(0);
        }
        const uint32_t wn = wq;   // row i + 1
        const int qn = (i >= Rc && q + 1 < np) ? q + 1 : q;   // the pair of row i + 1
        const int qo = row_q(wn), mo = row_rc(wn) * 64 + lane + qn * kMtSlot;
        int widx = i + 1;   // the word of row i + 2
        asm volatile("" : "+v"(widx) : "v"(qo), "v"(mo));
        const T pm_n = slut[kOffPm + qo];
        const T px_n = slut[kOffPx + qo];
        const uint2 m_n = mt[mo];
        wq = *reinterpret_cast<const uint32_t*>(rbase + ((widx < Rc ? rbc : rbn) + unsigned(widx) * 4u));
        const T y_in = from_left(y_out);
        const T t_in = from_left(t_out);
        T sM_in = T(0), sX_in = T(0);
        if constexpr (SUM) {
            sM_in = from_left(sumM);
            sX_in = from_left(sumX);
        }
        const T Tdiag = t_hold;
        t_hold = t_in;
        if (unsigned(i - 1) < unsigned(Rc)) {
            if (SUM && i == Rc) {
                sumM = lane ? sM_in : T(0);
                sumX = lane ? sX_in : T(0);
            }
            T Ml = T(0), Yl = y_in;
            const T M0 = Tdiag * prior_of<31>(mrow.x, k.pm, k.px);
            cell<T, BC, 0, BC, SUM, true>(Tt, X, M0, Ml, Yl, mrow.x, mrow.y, k.pm, k.px, k, 0, sumM, sumX);
            y_out = masked<AND>(y_next<true>(Ml, Yl, k.my, k.yy), keep);
            t_out = masked<AND>(Tt[BC - 1], keep);
        }
        k.pm = pm_n;
        k.px = px_n;
        mrow = m_n;
    };
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // The chain's steps (for the issue priority): its rows and the last skew.
    int nsteps = 0;
    for (int qq = 0, g = 0; qq < np; ++qq) {
        const int Rq = __builtin_amdgcn_readfirstlane(ce[qq].R), nbq = __builtin_amdgcn_readfirstlane(ce[qq].nb);
        g += Rq;
        nsteps = max(nsteps, g + nbq - 1);
    }
    // Row sums only in each pair's window of last rows (lane s: step G + R + s);
    // the issue priority by remaining steps as the single waves set it.
    int kk = 1, we = 0, Gq = 0;
    int pk = pmode ? 1 : INT32_MAX;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    auto prio = [&]() {
        if (kk >= pk) {
            set_prio(pmode, kk, nsteps, t0);
            pk += 16;
        }
    };
    for (int qq = 0; qq < np; ++qq) {
        const int Rq = __builtin_amdgcn_readfirstlane(ce[qq].R), nbq = __builtin_amdgcn_readfirstlane(ce[qq].nb);
        const int ws = Gq + Rq;
        we = max(we, ws + nbq - 1);
        for (; kk < ws; ++kk) {
            prio();
            step(kk, std::false_type{});
        }
        for (; kk <= we; ++kk) {
            prio();
            step(kk, std::true_type{});
        }
        Gq += Rq;
    }
    if (lane == ce[q].nb - 1) a.raw_out[ce[q].pid] = sumM + sumX;
    return true;
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_seg64_kernel(Seg64Args a)
{
    // The planner's scratch, then (its plan published) the waves' match windows.
    __shared__ union alignas(16) {
        PlanLds plan;
        uint2 mt[4][kMaxChain * kMtSlot];
    } lds_u;
    __shared__ double slut[kSlutLen];
    __shared__ ChainEnt chain_lds[4][kMaxChain];
    __shared__ int role;
    PlanLds& plan_lds = lds_u.plan;
    const int t = threadIdx.x;
    // The fp32 pass's rescue list is complete (stream order). Its plan is
    // made here, not by a launch of its own: an empty list (most runs) needs
    // none, and otherwise the first workgroup to arrive plans while the others
    // gather the seg records, then wait for its flag (they never wait on a
    // workgroup that is not running: the planner is the first one running).
    const int n = __builtin_amdgcn_readfirstlane(*a.count);
    if (blockIdx.x == 0 && t == 0) {   // the other run parity's counters, zeroed for the next run
        *a.count_reset = 0;
        *a.inker_reset = 0;
        *a.ticket_reset = 0;
        *a.ready_reset = 0;
        if (n == 0) *a.big_count = 0;   // the wide fp64 kernel's list (the plan writes it otherwise)
    }
    if (t == 0) role = n > 0 ? atomicAdd(a.ticket, 1) : 1;
    __syncthreads();
    const bool planner = role == 0;
    if (planner) {
        const unsigned long long t_plan0 = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
        plan_rescue(a, n, plan_lds);
        __syncthreads();
        plan_stamp(a, plan_lds, 5);
        unsigned long long ph[kPlanPhases] = {};
        if (t == 0 && a.timeline)   // (read before the waves reuse the LDS)
            for (int i = 0; i < kPlanPhases; ++i) ph[i] = plan_lds.phase[i];
        // Publish (MI355X_MICROARCH.md, inter-workgroup visibility): every
        // storing wave drains its stores, then one lane releases and flags.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.timeline) {   // (diagnostics) the plan's span and phases
                a.timeline[3 * size_t(a.n_pairs)] = t_plan0;
                a.timeline[3 * size_t(a.n_pairs) + 1] = __builtin_amdgcn_s_memrealtime();
                a.timeline[3 * size_t(a.n_pairs) + 2] = (unsigned long long)n;
                for (int i = 0; i < kPlanPhases; ++i) a.timeline[3 * size_t(a.n_pairs + 1) + i] = ph[i];
            }
        }
    }
    if (a.rec) {
        // The fp32 pass's seg results, slot records -> per-pair outputs (pair
        // order: coalesced stores; the record reads are gathers). A pair the
        // rescue below recomputes (state kRecListed) gets its raw f64 there.
        for (int q = blockIdx.x * 256 + threadIdx.x; q < a.n_pairs; q += gridDim.x * 256) {
            const int s = a.slot_of[q];
            if (s < 0) continue;   // computed by a one-lane / anti-diagonal kernel: in place already
            const uint4 r = a.rec[s];
            a.raw32[q] = __uint_as_float(r.x);
            a.flag[q] = r.y != kRecPlain;
            if (r.y != kRecListed)
                a.raw_out[q] = __longlong_as_double((long long)(((unsigned long long)r.w << 32) | r.z));
        }
    }
    if (n == 0) return;   // most runs: nothing to rescue
    if (!planner) {
        if (t == 0) {
            int ok = 0;
            const int limit = a.force_plan_timeout ? 0 : (1 << 24);
            for (int it = 0; it < limit; ++it) {   // bounded: a wave never waits forever
                if (__hip_atomic_load(a.ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    ok = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // (Not expected.) No plan: this workgroup's share of the rescue is
            // not done, so the run must not return results: the error word
            // makes the host fail the call with HC_PHMM_EHIP (verdict round 4).
            if (!ok) __hip_atomic_fetch_or(a.err, kErrPlanWait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            role = ok ? 1 : -1;
        }
        __syncthreads();
        if (role < 0) return;   // never read a stale plan
    }
    const Seg64Plan* __restrict__ p = a.plan;
    const int total = __builtin_amdgcn_readfirstlane(p->wave_base[kSeg64Classes - 1]);
    if (int(blockIdx.x) * 4 >= total) return;   // workgroup-uniform: a short list costs no LDS fill
    load_slut(slut, a.lut);
    uint2* mt = lds_u.mt[threadIdx.x >> 6];
    ChainEnt* ce = chain_lds[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    // Lane l holds the first wave of class l + 1: a wave's class is the number
    // of class starts at or below it (wave_base is non-decreasing).
    static_assert(kSeg64Classes <= 65, "one ballot covers the classes");
    const int next_base = lane < kSeg64Classes - 1 ? p->wave_base[lane + 1] : INT32_MAX;
    const bool dyn = __builtin_amdgcn_readfirstlane(p->dynamic) != 0;
    const int chain = __builtin_amdgcn_readfirstlane(p->chain);
    const int pmode = a.prio ? (dyn ? 2 : 1) : 0;   // issue priority mode (seg_common.hpp set_prio)
    for (int pos = blockIdx.x * 4 + (threadIdx.x >> 6);;) {
        if (dyn) {   // greedy: the next wave in descending cost
            int v = 0;
            if (lane == 0) v = atomicAdd(a.next_wave, 1);
            pos = __builtin_amdgcn_readfirstlane(v);
        }
        if (pos >= total) break;
        const unsigned long long t_start = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
        const int w = (total > 1 && a.wave_order) ? __builtin_amdgcn_readfirstlane(a.wave_order[pos]) : pos;
        const int c = __popcll(__builtin_amdgcn_ballot_w64(next_base <= w));
        const int bc = class_bc(c);
        const int nk = __builtin_amdgcn_readfirstlane(p->n_class[c]);
        const int ok = __builtin_amdgcn_readfirstlane(p->off_class[c]);
        const int wk = w - __builtin_amdgcn_readfirstlane(p->wave_base[c]);
        int pid;
        // A chain of 64-lane pairs; with chains on, the single 64-lane pairs
        // run as chains of one: the pass's 64-lane waves then run one step
        // loop per width, not two (the instruction cache holds fewer loops;
        // S4-20k's first round of chain waves beside single waves ran ~2.5x
        // slower per step than either alone).
        if (c < kChainClasses || (chain > 1 && class_k(c) == 6)) {
            const int per = c < kChainClasses ? chain : 1;
            const int e0 = ok + wk * per, np = min(per, nk - wk * per);
            bool done = false;
            switch (bc) {   // (64-lane pairs at bc0 = 32: 17-32 columns per lane)
            case 20: done = chain_run<20>(a, slut, mt, ce, lane, e0, np, pmode); break;
            case 24: done = chain_run<24>(a, slut, mt, ce, lane, e0, np, pmode); break;
            case 28: done = chain_run<28>(a, slut, mt, ce, lane, e0, np, pmode); break;
            case 32: done = chain_run<32>(a, slut, mt, ce, lane, e0, np, pmode); break;
            default: break;
            }
            if (!done)   // not one gap-constant set: the pairs one at a time
                for (int qq = 0; qq < np; ++qq) {
                    __builtin_amdgcn_wave_barrier();
                    (void)slot_wave(a, slut, mt, lane, 6, bc, e0 + qq, 1, 0, pmode);
                }
            pid = a.sorted[e0];
        } else {
            pid = slot_wave(a, slut, mt, lane, class_k(c), bc, ok, nk, wk, pmode);
        }
        if (a.timeline && lane == 0) wave_record(a, w, t_start, pid);   // (diagnostics)
        __builtin_amdgcn_wave_barrier();   // the next wave's match table reuses mt
        if (!dyn) pos += gridDim.x * 4;
    }
}

__global__ __launch_bounds__(256) void all_f64_list_kernel(int n, float* __restrict__ raw32,
                                                          uint8_t* __restrict__ flag, int* __restrict__ list,
                                                          int* __restrict__ count, const PairDesc* __restrict__ pairs,
                                                          int* __restrict__ list_rh)
{
    for (int p = blockIdx.x * 256 + threadIdx.x; p < n; p += gridDim.x * 256) {
        raw32[p] = 0.f;   // result_float = 0.0f (intel_pairhmm.hpp:135)
        flag[p] = 1;      // 0 < MIN_ACCEPTED: the double kernel for every pair
        list[p] = p;
        list_rh[p] = pack_rh(pairs[p].y, pairs[p].w);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *count = n;
}

}  // namespace

// One-lane kernel variants: {pairs per lane, block columns, waves per SIMD}.
// Block widths are multiples of 32 (a block starts on a match-word boundary).
// Waves per SIMD of the fp32 column-segmented kernel (168 VGPRs; a 128-VGPR
// build at 4 waves per SIMD needs narrower blocks and measured 1-3 % slower,
// profiles/r02_occ3_vs_occ4_caps.jsonl).
constexpr int kSegOcc = 3;
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
    const int grid = (a.n_waves + kSegWPB - 1) / kSegWPB;
    hipLaunchKernelGGL((phmm_seg_kernel<kSegOcc>), dim3(grid), dim3(64 * kSegWPB), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_all_f64_list(int n, float* raw32, uint8_t* flag, int* list, int* count, const PairDesc* pairs,
                               int* list_rh, hipStream_t s)
{
    const int grid = n <= 0 ? 1 : std::min((n + 255) / 256, 1024);
    hipLaunchKernelGGL(all_f64_list_kernel, dim3(grid), dim3(256), 0, s, n, raw32, flag, list, count, pairs, list_rh);
    return hipGetLastError();
}

hipError_t launch_rescue_seg64(const Seg64Args& a, int grid, hipStream_t s)
{
    hipLaunchKernelGGL((phmm_seg64_kernel<kSeg64Occ>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
