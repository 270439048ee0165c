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

// Column-segmented fp32 waves (host-planned). The wave's npairs pairs are the
// slots slot0 .. slot0+npairs-1; pair g takes nb_g = ceil(H_g / BC) consecutive
// lanes in slot order. Lanes past the last group idle (s = 0, no output).
// Seg waves per workgroup: 1, 2 and 4 time the same (profiles/
// r02_seg_waves_per_workgroup_ab.txt); 4 shares the LDS prior table.
constexpr int kSegWPB = 4;
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
// not 35 lanes of 32 in a 64-lane slot). Lists long enough for several rounds
// of waves chain the pairs of the 32- and 64-lane slots (kernels.hpp
// Seg64Plan::chain): their R + 2^k - 1 steps per pair were up to a third
// pipeline skew. The list is scattered into class order, classes with the
// longest waves first (order inside a class is arbitrary; each pair's result
// is independent of it). Pairs needing more than 64 lanes of 32 columns go to
// the anti-diagonal fp64 kernel through `big`.

__device__ __forceinline__ int ceil_log2(int nb) { return nb <= 1 ? 0 : 32 - __clz(nb - 1); }
__device__ __forceinline__ int seg64_wi(int need) { return need <= 8 ? 0 : (need - 8 + 3) / 4; }
// Unchained classes follow the chained ones; class c of either kind has
// width seg64_width(kSeg64Widths - 1 - c % kSeg64Widths).
__device__ __forceinline__ int plain_class(int k, int wi)
{
    return kSeg64ChainClasses + (6 - k) * kSeg64Widths + (kSeg64Widths - 1 - wi);
}
__device__ __forceinline__ int class_k(int c)
{
    return 6 - (c < kSeg64ChainClasses ? c : c - kSeg64ChainClasses) / kSeg64Widths;
}
__device__ __forceinline__ int class_bc(int c) { return seg64_width(kSeg64Widths - 1 - c % kSeg64Widths); }

// The pair's unchained class; *elig: it may join a chain (a 32- or 64-lane
// slot and a read longer than the slot, so a lane group never works on more
// than two pairs at once: run_chain's two table buffers).
__device__ __forceinline__ int rescue_class(int H, int R, int bc0, bool* elig)
{
    *elig = false;
    if (H > kSeg64MaxH) return kSeg64Classes - 1;
    const int nb0 = (H + bc0 - 1) / bc0;
    const int k = nb0 <= 64 ? ceil_log2(nb0) : 6;
    const int need = (H + (1 << k) - 1) >> k;   // <= bc0 when nb0 <= 64
    *elig = k >= 5 && R > (1 << k) && need > 16;   // chained widths: 20 .. 32 (run_chain cases)
    return plain_class(k, seg64_wi(need));
}

// Wave order of the pass. With at most two waves per SIMD (fp64 occupancy)
// every wave is resident at once and the pass lasts as long as its busiest
// SIMD: position p and p + n_simd share a SIMD (workgroups of four waves, the
// first n_simd positions filling one slot per SIMD), so the heaviest waves go
// first, in descending cost, and the rest after them in ascending cost — the
// heaviest wave shares its SIMD with the lightest. With more, waves are
// fetched from a counter in descending cost (greedy longest-first). Wave
// cost: (rows + skew) steps x (14 ops per column + ~40 per step).
constexpr int kMaxSortWaves = 8192;
// Chaining. A list chains when its chain-eligible pairs fill the resident
// wave slots (two per SIMD, S = 2 x SIMDs) kChainMinRounds times over. Each
// eligible class then keeps its share of kChainTailRounds x S pairs unchained,
// and the rest form chains long enough for at most S chained waves: the
// chained waves are fetched first (the longest), one per slot, and the
// single-pair waves after them even out the slots (greedy longest-first), so
// no slot waits on a last, partial round of long waves. Below two pairs per
// chain the list stays unchained.
constexpr int kChainMinRounds = 3;   // (the tail: Seg64Args::chain_tail rounds, default 2)

__global__ __launch_bounds__(1024) void rescue_plan_kernel(Seg64Args a)
{
    constexpr int NC = kSeg64Classes;
    __shared__ int cnt[NC], fill[NC], wbase[NC], elig_cnt[kSeg64ChainClasses], take[kSeg64ChainClasses];
    __shared__ int clen[kSeg64ChainClasses];
    __shared__ unsigned long long elig_rows[kSeg64ChainClasses];
    __shared__ unsigned long long lanes_sh;
    __shared__ unsigned long long key[kMaxSortWaves];
    const int n = *a.count;
    const int t = threadIdx.x;
    if (t == 0) {
        *a.count_reset = 0;
        *a.inker_reset = 0;
        *a.next_wave = 0;
    }
    if (n == 0) {   // most runs: an empty plan (the fp64 kernel reads only the wave total)
        if (t == 0) {
            a.plan->wave_base[NC - 1] = 0;
            *a.big_count = 0;
        }
        return;
    }
    if (t < NC) cnt[t] = 0;
    if (t < kSeg64ChainClasses) {
        elig_cnt[t] = 0;
        take[t] = 0;
        clen[t] = 0;
        elig_rows[t] = 0;
    }
    if (t == 0) lanes_sh = 0;
    __syncthreads();
    // Width bound: 32 unless the lanes at width 32 give fewer than min_lanes
    // (2 waves per SIMD), then 16, then 8.
    unsigned long long mine = 0;
    for (int i = t; i < n; i += blockDim.x) mine += (a.pairs[a.list[i]].w + 31) / 32;
    if (mine) atomicAdd(&lanes_sh, mine);
    __syncthreads();
    const long long l32 = (long long)lanes_sh;
    // (A forced chain length forces width 32 too, so short test lists chain.)
    const int bc0 = l32 >= a.min_lanes || a.chain_force > 0 ? 32 : (2 * l32 >= a.min_lanes ? 16 : 8);
    for (int i = t; i < n; i += blockDim.x) {
        const PairDesc pd = a.pairs[a.list[i]];
        bool e;
        const int c = rescue_class(pd.w, pd.y, bc0, &e);
        atomicAdd(&cnt[c], 1);
        if (e) {
            atomicAdd(&elig_cnt[c - kSeg64ChainClasses], 1);
            atomicAdd(&elig_rows[c - kSeg64ChainClasses], (unsigned long long)pd.y);
        }
    }
    __syncthreads();
    if (t == 0) {
        const long long S = 2LL * a.n_simd;   // resident wave slots
        long long nel = 0, lanes = 0;         // eligible pairs; their lanes (unit: 64 = one wave)
        for (int c = 0; c < kSeg64ChainClasses; ++c) {
            nel += elig_cnt[c];
            lanes += (long long)elig_cnt[c] << class_k(c);
        }
        if (a.chain_force >= 0) {   // tests / A/B: every eligible pair chained, one length
            for (int c = 0; c < kSeg64ChainClasses; ++c) {
                take[c] = elig_cnt[c];
                clen[c] = a.chain_force;
            }
        } else if (bc0 == 32 && lanes >= kChainMinRounds * S * 64) {
            // Chain lengths per class for waves of equal modelled cost (mean
            // rows x (14 x width + 40) per pair; the G groups of a wave run in
            // parallel), sized so the chained waves number about S.
            const long long tail = min(nel, a.chain_tail * S);
            double total = 0.0;
            for (int c = 0; c < kSeg64ChainClasses; ++c) {
                if (!elig_cnt[c]) continue;
                take[c] = elig_cnt[c] - int((elig_cnt[c] * tail + nel - 1) / nel);
                const double rbar = double(elig_rows[c]) / elig_cnt[c];
                total += double(take[c]) * rbar * (14 * class_bc(c) + 40) / (64 >> class_k(c));
            }
            const double C = total / double(S);   // cost of one chained wave
            for (int c = 0; c < kSeg64ChainClasses; ++c) {
                if (!take[c]) continue;
                const double rbar = double(elig_rows[c]) / elig_cnt[c];
                // rounded up: at most S chained waves, each slot holds one
                clen[c] = min(kSeg64ChainMax, int(ceil(C / (rbar * (14 * class_bc(c) + 40)))));
            }
        }
        int chain = 0;
        for (int c = 0; c < kSeg64ChainClasses; ++c) {
            if (clen[c] < 2) clen[c] = 0;
            const int e = clen[c] ? take[c] : 0;
            take[c] = e;
            cnt[c] = e;
            cnt[c + kSeg64ChainClasses] -= e;
            chain = max(chain, clen[c]);
        }
        Seg64Plan* __restrict__ p = a.plan;   // written in place (a local copy would live in registers)
        p->bc0 = bc0;
        p->chain = chain;
        for (int c = 0; c < kSeg64ChainClasses; ++c) p->chain_len[c] = clen[c];
        int off = 0, wb = 0;
        for (int c = 0; c < NC; ++c) {
            p->n_class[c] = cnt[c];
            p->off_class[c] = off;
            fill[c] = off;
            off += cnt[c];
            p->wave_base[c] = wb;
            wbase[c] = wb;
            if (c < NC - 1 && cnt[c] > 0) {   // (chained classes are empty when chain = 0)
                const int per = (64 >> class_k(c)) * (c < kSeg64ChainClasses ? clen[c] : 1);
                wb += (cnt[c] + per - 1) / per;
            }
        }
        p->dynamic = a.wave_order != nullptr && wb > 2 * a.n_simd;
        *a.big_count = cnt[NC - 1];
    }
    __syncthreads();
    for (int i = t; i < n; i += blockDim.x) {
        const int pid = a.list[i];
        const PairDesc pd = a.pairs[pid];
        bool e;
        int c = rescue_class(pd.w, pd.y, bc0, &e);
        if (e && atomicSub(&take[c - kSeg64ChainClasses], 1) > 0) c -= kSeg64ChainClasses;
        const int pos = atomicAdd(&fill[c], 1);
        if (c < NC - 1)
            a.sorted[pos] = pid;
        else
            a.big[pos - (n - cnt[NC - 1])] = pid;
    }
    __syncthreads();
    const int W = wbase[NC - 1];   // segmented waves
    if (W <= 1 || !a.wave_order) return;
    if (W > kMaxSortWaves) {   // classes longest first, fetched in that order
        for (int w = t; w < W; w += blockDim.x) a.wave_order[w] = w;
        return;
    }
    // Cost of every wave, then a bitonic sort (descending) in LDS.
    int N = 1;
    while (N < W) N <<= 1;
    for (int w = t; w < N; w += blockDim.x) {
        unsigned long long k = 0;
        if (w < W) {
            int c = 0;
            while (c + 1 < NC - 1 && wbase[c + 1] <= w) ++c;
            const int kk = class_k(c), G = 64 >> kk;
            const bool ch = c < kSeg64ChainClasses;
            const int per = G * (ch ? clen[c] : 1);
            const int off = fill[c] - cnt[c];   // the class's first entry (fill ran past it)
            const int e0 = off + (w - wbase[c]) * per;
            const int e1 = min(off + cnt[c], e0 + per);
            int rows = 0;   // longest read (unchained) / a group's chain rows at the class mean (chained)
            if (ch)
                rows = int(elig_rows[c] * (unsigned long long)(e1 - e0) / (unsigned long long)(elig_cnt[c] * G));
            else
                for (int e = e0; e < e1; ++e) rows = max(rows, a.pairs[a.sorted[e]].y);
            const unsigned cost = unsigned(rows + (1 << kk) - 1) * unsigned(class_bc(c) * 14 + 40);
            k = ((unsigned long long)cost << 32) | unsigned(w);
        }
        key[w] = k;
    }
    __syncthreads();
    for (int size = 2; size <= N; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < N / 2; i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool desc = (lo & size) == 0;
                const unsigned long long x = key[lo], y = key[hi];
                if ((x < y) == desc) {
                    key[lo] = y;
                    key[hi] = x;
                }
            }
            __syncthreads();
        }
    const int S = a.n_simd;
    for (int p = t; p < W; p += blockDim.x) {
        // two waves per SIMD at most: positions S.. pair the heaviest with the lightest
        const int r = (W <= 2 * S && p >= S) ? S + (W - 1 - p) : p;
        a.wave_order[p] = int(key[r] & 0xffffffffu);
    }
}

// One column-segmented wave (wid) of the fp32 pass.
__device__ __forceinline__ void seg_wave(const LaneArgs& a, int wid, const float* __restrict__ slut)
{
    const int lane = threadIdx.x & 63;
    const unsigned long long t_start = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
    const LaneWave wv = load_wave(a.waves, wid);
    const int bc = wv.ncols;
    __shared__ uint2 mtab[kSegWPB][5 * 64];
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
    if (a.timeline && lane == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        a.timeline[3 * size_t(wid)] = t_start;
        a.timeline[3 * size_t(wid) + 1] = t_end;
        a.timeline[3 * size_t(wid) + 2] = unsigned(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));
    }
}


template <int OCC>
__global__ __launch_bounds__(64 * kSegWPB, OCC) void phmm_seg_kernel(LaneArgs a)
{
    __shared__ float slut[kSlutLen];
    // Device-planned parts launch an upper bound of waves: surplus workgroups
    // leave before the LDS fill (workgroup-uniform).
    const int n_waves = a.n_waves_dev ? __builtin_amdgcn_readfirstlane(*a.n_waves_dev) : a.n_waves;
    if (int(blockIdx.x) * kSegWPB >= n_waves) return;
    load_slut(slut, a.lut);
    const int wid = blockIdx.x * kSegWPB + (threadIdx.x >> 6);
    if (wid < n_waves) seg_wave(a, wid, slut);
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

// ---------------------------------------------------------------------------
// Chained fp64 waves (Seg64Plan::chain). A wave of a chained class holds
// G = 64 / L lane groups of L = 2^k lanes; group g runs its chain of up to
// `chain` pairs back to back. Lane s of a group sweeps the concatenated rows
// of its chain one step behind lane s - 1, so every DPP hand-off of run_seg
// (Y entering the block, the right-edge T of the row above, the row-R sums)
// comes from the same pair's same row, and a lane that has finished a pair's
// row R starts the next pair's row 1 on its next step: its registers are
// reset to row 0 (T0, 0), its row-1 diagonal is T0, and the pipeline skew is
// paid once per chain. The group's pair descriptors live in LDS, the hap
// match tables in two LDS buffers (pair j in buffer j & 1): once the group's
// last lane has started pair j (R > L: every lane then works on pair j),
// the group copies pair j + 1's table into the free buffer.
struct ChainPair {
    int rows, R, H, pid, tbl, w1;   // packed rows offset, lengths, pair id, table offset, row-1 word
    double T0, mm;                  // row-0 diagonal; mm of the read's (constant) gap qualities
};
static_assert(sizeof(ChainPair) == 40, "ChainPair: ten LDS words");
constexpr int kChainInfoWords = 2 * kSeg64ChainMax * 10;   // two groups (k = 5)
// Table buffers of a wave: G x 2 x (L + 3) rows of 5 words (k = 5: 700, k = 6: 670).
constexpr int kChainTableWords = 2 * 2 * (32 + 3) * 5;
constexpr int kSeg64WaveWords = 1024;   // per wave: the chain LDS, or run_seg's match window
static_assert(kChainInfoWords + kChainTableWords <= kSeg64WaveWords && 5 * 64 * 2 <= kSeg64WaveWords,
              "seg64 per-wave LDS");

// Match word of columns c0+1 .. c0+32 (MSB first) for read code rc from an
// LDS table (rows of 5 words): v_alignbit of rows wa and wa + 1 (see run_chain).
__device__ __forceinline__ uint32_t chain_match(const uint32_t* __restrict__ tb, int wa, int sh, int rc)
{
    return __builtin_amdgcn_alignbit(tb[wa * 5 + rc], tb[(wa + 1) * 5 + rc], sh);
}

// The group's L lanes copy a pair's match table (hap_table_words(H)) to LDS.
__device__ __forceinline__ void chain_table(uint32_t* __restrict__ tb, const uint32_t* __restrict__ hapw,
                                            const ChainPair& p, int s, int L)
{
    const int nw = ((p.H + 31) / 32 + kHapPadWords) * 5;
    for (int j = s; j < nw; j += L) tb[j] = hapw[p.tbl + j];
}

// Transition constants of a read with constant gap qualities (row_const with
// wc = wn = its row-1 word; mm precomputed in its ChainPair).
__device__ __forceinline__ void chain_consts(const double* __restrict__ slut, uint32_t w1, double mm,
                                             RowConst<double>& k)
{
    k.my = slut[kOffPh2pr + row_d(w1)];
    k.yy = slut[kOffPh2pr + row_c(w1)];
    k.mm = mm;
    k.g = slut[kOffGapm + row_c(w1)];
    k.mx = slut[kOffPh2pr + row_i(w1)];
    k.xx = k.yy;
}

template <int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_chain(const Seg64Args& a, const double* __restrict__ slut, int s, int L,
                                          const ChainPair* __restrict__ ci, int np, uint32_t* __restrict__ tb,
                                          int tbw, int nsteps)
{
    using T = double;
    static_assert(seg_prefetch<T, BC>() == 1, "chained waves prefetch one row ahead");
    const int c0 = s * BC;
    // Window rows: columns c0+1 .. start at bit r of row c0/32 + kHapLead;
    // r = 0 takes the row before with a shift of 0 (v_alignbit shifts mod 32).
    const int r = c0 & 31;
    const int wa = c0 / 32 + kHapLead - (r == 0 ? 1 : 0), sh = (32 - r) & 31;
    // Every lane runs the cell update on every step, inside or outside its
    // rows: a lane's registers go back to row 0 when it starts a pair (the
    // first one included), so steps before its first row and after its
    // chain's last row compute values nothing reads, and the register blocks
    // are never written under a divergent branch (which would keep a second
    // copy of them live). Pair "-1" (R = 0) precedes the chain.
    int cur = -1, start = 0, R = 0, rows = 0, pid = 0;
    int nrows = np > 0 ? ci[0].rows : 0;   // rows of the pair after the current one
    uint32_t keep = 0u;
    int lim0 = 0;
    bool owner = false;
    T Tt[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        Tt[j] = T(0);
        X[j] = T(0);
    }
    // Row words: lane 0 starts on row 1 at step 1 (its prior and match word
    // now, row 2 prefetched); lane s >= 1 fetches row 1 on its way there.
    const uint32_t w1 = np > 0 ? uint32_t(ci[0].w1) : 0u;
    uint32_t wc = w1;
    uint32_t wq = a.rows[nrows + (s == 0 ? 1 : 0)];
    RowConst<T> k;
    if constexpr (CG) {
        chain_consts(slut, w1, np > 0 ? ci[0].mm : T(0), k);
        k.pm = slut[kOffPm + row_q(w1)];
        k.px = slut[kOffPx + row_q(w1)];
        k.rc = row_rc(w1);
    } else {
        row_const<T>(a.lut, w1, wq, k);
    }
    uint32_t mrow = chain_match(tb, wa, sh, row_rc(w1));
    T y_out = T(0), t_out = T(0), t_hold = T(0);
    T sumM = T(0), sumX = T(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // Steps where some lane is on its pair's last row run the sums; between
    // them, the plain step (two loops, as run_seg's two phases).
    auto step = [&](int kk, auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        int i = kk - s - start;
        const bool sw = i > R && cur + 1 < np;   // the chain's next pair, row 1
        if (__builtin_amdgcn_ballot_w64(sw)) {
            T T0n = T(0);
            if (sw) {   // small per-lane state only
                start += R;
                ++cur;
                const ChainPair& p = ci[cur];
                R = p.R;
                rows = p.rows;
                pid = p.pid;
                T0n = p.T0;
                nrows = cur + 1 < np ? ci[cur + 1].rows : rows + R;
                keep = (s + 1) * BC < p.H ? 0xffffffffu : 0u;
                lim0 = p.H - c0;
                owner = s == (p.H + BC - 1) / BC - 1;
                i = 1;
            }
            // The register blocks back to row 0 (T0, 0): selects in uniform
            // control flow. Row 1's diagonal is T0; its pm, px and match word
            // came through the row prefetch last step.
#pragma unroll
            for (int j = 0; j < BC; ++j) {
                Tt[j] = sw ? T0n : Tt[j];
                X[j] = sw ? T(0) : X[j];
            }
            t_hold = sw ? T0n : t_hold;
            if constexpr (CG) {
                RowConst<T> kn = k;
                const ChainPair& p = ci[max(cur, 0)];
                chain_consts(slut, uint32_t(p.w1), p.mm, kn);
                k.my = sw ? kn.my : k.my;
                k.yy = sw ? kn.yy : k.yy;
                k.mm = sw ? kn.mm : k.mm;
                k.g = sw ? kn.g : k.g;
                k.mx = sw ? kn.mx : k.mx;
                k.xx = sw ? kn.xx : k.xx;
            }
        }
        // The group's last lane has started pair cur: the table of pair cur + 1
        // replaces pair cur - 1's (group-uniform; one load round trip per pair).
        if (cur >= 1 && kk == start + L && cur + 1 < np) {
            chain_table(tb + ((cur + 1) & 1) * tbw, a.hapw, ci[cur + 1], s, L);
            __builtin_amdgcn_wave_barrier();
        }
        const uint32_t wn = wq;   // row i + 1 (after row R: the next pair's row 1)
        T pm_n = T(0), px_n = T(0);
        uint32_t m_n = mrow;
        // Row i + 2 of the concatenated rows (the packed rows carry slack
        // around each read: words outside a read are read and ignored).
        const int rn = i + 2;
        int off = rn <= R ? rows + rn - 1 : nrows + rn - R - 1;
        const uint32_t* __restrict__ tnext = tb + ((cur + (i + 1 > R ? 1 : 0)) & 1) * tbw;
        if constexpr (CG) {
            const int qo = row_q(wn);
            m_n = chain_match(tnext, wa, sh, row_rc(wn));
            asm volatile("" : "+v"(off) : "v"(qo), "v"(m_n));
            pm_n = slut[kOffPm + qo];
            px_n = slut[kOffPx + qo];
        } else {
            asm volatile("" : "+v"(off) : "v"(wn));
        }
        wq = a.rows[off];
        const T y_in = from_left(y_out);
        const T t_in = from_left(t_out);
        T sM_in = T(0), sX_in = T(0);
        if constexpr (SUM) {
            sM_in = from_left(sumM);
            sX_in = from_left(sumX);
        }
        const T Tdiag = t_hold;
        t_hold = t_in;
        if constexpr (!CG) {
            row_const<T>(a.lut, wc, wn, k);
            mrow = chain_match(tb + (cur & 1) * tbw, wa, sh, k.rc);
        }
        const bool last = SUM && i == R && cur >= 0;
        const int lim = last ? lim0 : 0;
        if (last) {
            sumM = s ? sM_in : T(0);
            sumX = s ? sX_in : T(0);
        }
        T Ml = T(0), Yl = y_in;
        const T M0 = Tdiag * prior_of<31>(mrow, k.pm, k.px);
        cell<T, BC, 0, BC, SUM, EQ>(Tt, X, M0, Ml, Yl, mrow, 0u, k.pm, k.px, k, lim, sumM, sumX);
        y_out = masked(y_next<EQ>(Ml, Yl, k.my, k.yy), keep);
        t_out = masked(Tt[BC - 1], keep);
        if (last && owner) a.raw_out[pid] = sumM + sumX;
        if constexpr (CG) {
            k.pm = pm_n;
            k.px = px_n;
            mrow = m_n;
        }
        wc = wn;
    };
    for (int kk = 1; kk <= nsteps;) {
        // this lane's next last-row step
        int nl = INT32_MAX;
        if (cur >= 0 && kk <= start + R + s)
            nl = start + R + s;
        else if (cur + 1 < np)
            nl = start + R + ci[cur + 1].R + s;
        const int stop = min(wave_min(nl), nsteps + 1);
        for (; kk < stop; ++kk) step(kk, std::false_type{});
        if (kk <= nsteps) step(kk++, std::true_type{});
    }
}

// One chained wave: class c, its wk-th wave (entries off + wk * G * chain ..).
__device__ __forceinline__ void chain_wave(const Seg64Args& a, const double* __restrict__ slut, int lane, int c,
                                           int wk, int nk, int ok, int chain, uint32_t* __restrict__ wl)
{
    const int kk = class_k(c), L = 1 << kk, G = 64 >> kk;
    const int bc = class_bc(c);
    const int per = G * chain;
    const int ne = min(per, nk - wk * per);
    ChainPair* info = reinterpret_cast<ChainPair*>(wl);
    uint32_t* tables = wl + kChainInfoWords;
    bool eq = true;
    if (lane < ne) {
        const int pid = a.sorted[ok + wk * per + lane];
        const PairDesc pd = a.pairs[pid];
        const uint32_t w1 = a.rows[pd.x];
        ChainPair q;
        q.rows = pd.x;
        q.R = pd.y;
        q.H = pd.w;
        q.pid = pid;
        q.tbl = pd.z;
        q.w1 = int(w1);
        q.T0 = row0_t<double>(a.lut, w1, pd.w);
        q.mm = a.lut[kOffMM + mm_idx(row_i(w1), row_d(w1))];
        info[lane] = q;
        eq = read_eq(w1);
    }
    const bool wave_eq = __builtin_amdgcn_ballot_w64(!eq) == 0;
    __builtin_amdgcn_wave_barrier();
    const int g = lane >> kk, s = lane & (L - 1);
    const int np = max(0, min(chain, ne - g * chain));
    const ChainPair* ci = info + g * chain;
    const int tbw = (L + 3) * 5;
    uint32_t* tb = tables + g * 2 * tbw;
    int rows_total = 0;
    for (int j = 0; j < np; ++j) rows_total += ci[j].R;
    if (np > 0) chain_table(tb, a.hapw, ci[0], s, L);
    if (np > 1) chain_table(tb + tbw, a.hapw, ci[1], s, L);
    __builtin_amdgcn_wave_barrier();
    const int nsteps = wave_max(np > 0 ? rows_total + s : 0);
    switch (bc) {
#define HC_CHAIN_CASE(W)                                                                  \
    case W:                                                                               \
        if (wave_eq)                                                                      \
            run_chain<W, true, true>(a, slut, s, L, ci, np, tb, tbw, nsteps);             \
        else                                                                              \
            run_chain<W, false, false>(a, slut, s, L, ci, np, tb, tbw, nsteps);           \
        break;
        HC_CHAIN_CASE(20) HC_CHAIN_CASE(24) HC_CHAIN_CASE(28) HC_CHAIN_CASE(32)
#undef HC_CHAIN_CASE
    default: break;   // narrower widths never reach a chained class (bc0 = 32, 2^k >= 32 lanes)
    }
    __builtin_amdgcn_wave_barrier();   // the next wave rewrites the LDS
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_seg64_kernel(Seg64Args a)
{
    __shared__ double wlds[4][kSeg64WaveWords / 2];
    __shared__ double slut[kSlutLen];
    const Seg64Plan* __restrict__ p = a.plan;
    const int total = __builtin_amdgcn_readfirstlane(p->wave_base[kSeg64Classes - 1]);
    if (int(blockIdx.x) * 4 >= total) return;   // workgroup-uniform: an empty or short list costs no LDS fill
    load_slut(slut, a.lut);
    uint32_t* wl = reinterpret_cast<uint32_t*>(wlds[threadIdx.x >> 6]);
    uint2* mt = reinterpret_cast<uint2*>(wl);
    const int lane = threadIdx.x & 63;
    // Lane l holds the first wave of class l + 1: a wave's class is the number
    // of class starts at or below it (wave_base is non-decreasing).
    static_assert(kSeg64Classes - 1 <= 64, "one ballot covers the class starts");
    const int next_base = lane < kSeg64Classes - 1 ? p->wave_base[lane + 1] : INT32_MAX;
    const bool dyn = __builtin_amdgcn_readfirstlane(p->dynamic) != 0;
    for (int pos = blockIdx.x * 4 + (threadIdx.x >> 6);;) {
        if (dyn) {   // greedy: the next wave in descending cost
            int v = 0;
            if (lane == 0) v = atomicAdd(a.next_wave, 1);
            pos = __builtin_amdgcn_readfirstlane(v);
        }
        if (pos >= total) break;
        const int w = (total > 1 && a.wave_order) ? __builtin_amdgcn_readfirstlane(a.wave_order[pos]) : pos;
        const int c = __popcll(__builtin_amdgcn_ballot_w64(next_base <= w));
        const int nk = __builtin_amdgcn_readfirstlane(p->n_class[c]);
        const int ok = __builtin_amdgcn_readfirstlane(p->off_class[c]);
        const int wk = w - __builtin_amdgcn_readfirstlane(p->wave_base[c]);
        if (c < kSeg64ChainClasses) {
            chain_wave(a, slut, lane, c, wk, nk, ok, __builtin_amdgcn_readfirstlane(p->chain_len[c]), wl);
            if (!dyn) pos += gridDim.x * 4;
            continue;
        }
        const int k = class_k(c);
        const int bc = class_bc(c);
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
#define HC_SEG64_CASE(WI) \
    case seg64_width(WI): run_seg_bc<double, seg64_width(WI)>(a.lut, slut, st, lane, s, cx, T0, sumM, sumX, mt, wave_eq); break;
            HC_SEG64_CASE(0) HC_SEG64_CASE(1) HC_SEG64_CASE(2) HC_SEG64_CASE(3) HC_SEG64_CASE(4) HC_SEG64_CASE(5)
            HC_SEG64_CASE(6)
#undef HC_SEG64_CASE
        default: break;
        }
        if (owner) a.raw_out[pid] = sumM + sumX;
        __builtin_amdgcn_wave_barrier();   // the next wave's match table reuses mt
        if (!dyn) pos += gridDim.x * 4;
    }
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

hipError_t launch_rescue_seg64(const Seg64Args& a, int grid, hipStream_t s)
{
    hipLaunchKernelGGL(rescue_plan_kernel, dim3(1), dim3(1024), 0, s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((phmm_seg64_kernel<kSeg64Occ>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
