// Chained column-segmented PairHMM waves (fp32) for gfx950.
//
// The column-segmented wave of lane_kernel.hip (phmm_seg_kernel) puts a pair's
// nb column blocks on nb consecutive lanes with one row of skew per block, so a
// pair of R rows takes R + nb - 1 steps: nb - 1 steps of pipeline fill and
// drain per pair (about 3 % of the lane-steps on the S2 mix). Here a group of
// nb lanes runs a queue of pairs (rounds) back to back: lane s finishes the
// last row of its pair at step C_t + s and starts row 1 of the next pair at
// step C_t + s + 1, while lane s + 1 still finishes the previous pair (every
// hand-off lane s+1 reads from lane s belongs to the row lane s+1 is on). The
// fill / drain is paid once per wave. The pairs of a round have nearly equal R
// (planned on the host by R), so the row-sum steps of a round (the last rows,
// summed left to right as the reference does) stay a short window.
//
// Same semantics as compute_full_prob_avxs (avx-pairhmm-template.h:210-346)
// bit for bit: the same cell update (seg_common.hpp `cell`), row order and
// sums as the unchained kernel.
#include "seg_common.hpp"

namespace hcphmm {
namespace {
using namespace seg;

template <int BC, bool CG, bool EQ>
__device__ __forceinline__ void run_chain(const LaneArgs& a, const float* __restrict__ slut, int G, int T, int nb,
                                          int lane, int g, int s, const int* __restrict__ pids,
                                          const uint32_t* __restrict__ rounds, uint2* __restrict__ mt,
                                          int* __restrict__ rslot)
{
    constexpr int PD = seg_prefetch<float, BC>();
    constexpr int kNever = 1 << 29;
    const float* __restrict__ lut = a.lut;
    const int c0 = s * BC;
    const bool owner = s == nb - 1;
    float Tt[BC], X[BC];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
        Tt[j] = 0.f;
        X[j] = 0.f;
    }
    // The lane's pair: i = its row (<= 0 before its first pair, -kNever when
    // done), switching to the next round's pair once i passes the round's Rmax.
    int t_l = -1, i = g < G ? -s : -kNever, Rr = g < G ? 0 : kNever, Rg = 1, pid = 0, lim0 = 0;
    const uint32_t* __restrict__ rrow = a.rows;
    float T0 = 0.f;
    uint32_t wc = 0, wq[PD];
#pragma unroll
    for (int P = 0; P < PD; ++P) wq[P] = 0;
    RowConst<float> k{};
    uint2 mrow = make_uint2(0u, 0u);
    float y_out = 0.f, t_out = 0.f, t_hold = 0.f, sumM = 0.f, sumX = 0.f;
    auto step = [&](int kk, auto sum_tag, auto ph_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        constexpr int P = decltype(ph_tag)::value;
        ++i;
        if (i > Rr) {   // next round's pair (lanes of a group switch on consecutive steps)
            ++t_l;
            const int np = t_l < T ? pids[t_l * G + g] : -1;
            if (np >= 0) {
                pid = np;
                const PairDesc pd = a.pairs[np];
                rrow = a.rows + pd.x;
                Rg = pd.y;
                lim0 = pd.w - c0;
                Rr = int(rounds[t_l] & 0xffffu);
                i = 1;
                fill_window(mt, lane, a.hapw + pd.z, pd.w, c0);
                const uint32_t w1 = rrow[0];
                T0 = row0_t<float>(lut, w1, pd.w);
#pragma unroll
                for (int j = 0; j < BC; ++j) {
                    Tt[j] = T0;   // row 0
                    X[j] = 0.f;
                }
                row_const<float>(lut, w1, rrow[min(2, Rg) - 1], k);
                mrow = mt[k.rc * 64 + lane];
                wc = w1;
#pragma unroll
                for (int d = 0; d < PD; ++d) wq[(P + d) % PD] = rrow[min(2 + d, Rg) - 1];
                // Nothing of the switch left in flight: the wait counts of the
                // sweep stay those of the straight path.
                __builtin_amdgcn_s_waitcnt(0x0F70);
            } else {
                i = -kNever;
                Rr = kNever;
            }
        }
        const uint32_t wn = wq[P];   // row i+1, loaded PD steps ago
        float pm_n = 0.f, px_n = 0.f;
        uint2 m_n = mrow;
        int ridx = min(max(i + PD + 1, 1), Rg) - 1;   // the word needed PD steps from now
        if constexpr (CG) {
            const int qo = row_q(wn), mo = row_rc(wn) * 64 + lane;
            asm volatile("" : "+v"(ridx) : "v"(qo), "v"(mo));   // load after the last use of wn (run_seg)
            pm_n = slut[kOffPm + qo];
            px_n = slut[kOffPx + qo];
            m_n = mt[mo];
        } else {
            asm volatile("" : "+v"(ridx) : "v"(wn));
        }
        wq[P] = rrow[ridx];
        const float y_in = from_left(y_out);
        const float t_in = from_left(t_out);
        float sM_in = 0.f, sX_in = 0.f;
        if constexpr (SUM) {
            sM_in = from_left(sumM);
            sX_in = from_left(sumX);
        }
        const float Tdiag = i == 1 ? T0 : (s ? t_hold : 0.f);
        const float Yl0 = s ? y_in : 0.f;
        t_hold = t_in;
        if (i >= 1) {
            if constexpr (!CG) {
                row_const<float>(lut, wc, wn, k);
                mrow = mt[k.rc * 64 + lane];
            }
            const bool last = SUM && i == Rg;
            const int lim = last ? lim0 : 0;
            if (last) {
                sumM = s ? sM_in : 0.f;
                sumX = s ? sX_in : 0.f;
            }
            float Ml = 0.f, Yl = Yl0;
            const float M0 = Tdiag * prior_of<31>(mrow.x, k.pm, k.px);
            cell<float, BC, 0, BC, SUM, EQ>(Tt, X, M0, Ml, Yl, mrow.x, mrow.y, k.pm, k.px, k, lim, sumM, sumX);
            y_out = y_next<EQ>(Ml, Yl, k.my, k.yy);
            t_out = Tt[BC - 1];
            if constexpr (CG) {
                k.pm = pm_n;
                k.px = px_n;
                mrow = m_n;
            }
            if (SUM && last && owner) {   // fp32 result and rescue decision (intel_pairhmm.hpp:133-139)
                const float raw = sumM + sumX;
                const bool resc = raw < 1e-28f;   // MIN_ACCEPTED, pairhmm_common.h:16
                a.raw_out[pid] = raw;
                a.rescue_flag[pid] = resc;
                if (!resc) {
                    a.raw64_zero[pid] = 0.0;
                } else {
                    const int slot = a.inker_count ? atomicAdd(&rslot[0], 1) : kChainRescueSlots;
                    if (slot < kChainRescueSlots)
                        rslot[1 + slot] = pid;
                    else
                        a.rescue_list[atomicAdd(a.rescue_count, 1)] = pid;
                }
            }
        }
        wc = wn;
    };
    __builtin_amdgcn_s_waitcnt(0x0F70);
    int kk = 1, C = 0;
    for (int t = 0; t < T; ++t) {
        const uint32_t ri = __builtin_amdgcn_readfirstlane(rounds[t]);
        const int rmax = int(ri & 0xffffu), rmin = int(ri >> 16);
        const int start = C + rmin, end = C + rmax + nb - 1;
        for (; kk + PD - 1 < start; kk += PD)
            for_phases<0, PD>([&](auto ph) { step(kk + decltype(ph)::value, std::false_type{}, ph); });
        for (; kk <= end; kk += PD)
            for_phases<0, PD>([&](auto ph) { step(kk + decltype(ph)::value, std::true_type{}, ph); });
        C += rmax;
    }
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void phmm_chain_kernel(LaneArgs a)
{
    __shared__ float slut[kSlutLen];
    load_slut(slut, a.lut);
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= a.n_waves) return;
    const int wl = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ uint2 mtab[4][5 * 64];
    __shared__ int pidtab[4][kChainMaxEntries];
    __shared__ uint32_t rtab[4][kChainMaxRounds];
    __shared__ int rslot[4][kChainRescueSlots + 1];
    const ChainWave w = a.cwaves[wid];
    const int pid0 = __builtin_amdgcn_readfirstlane(w.pid0), r0 = __builtin_amdgcn_readfirstlane(w.r0);
    const int shape = __builtin_amdgcn_readfirstlane(w.shape);
    const int bc = shape & 0xff, nb = (shape >> 8) & 0xff, G = (shape >> 16) & 0xff, T = (shape >> 24) & 0x7f;
    const bool eq = shape < 0;
    for (int e = lane; e < T * G; e += 64) pidtab[wl][e] = a.cpids[pid0 + e];
    for (int t = lane; t < T; t += 64) rtab[wl][t] = a.crounds[r0 + t];
    if (lane == 0) rslot[wl][0] = 0;
    __builtin_amdgcn_wave_barrier();
    // lane -> (group, block): exact floor(lane / nb) for lane < 64
    const int g = (lane * ((65536 + nb - 1) / nb)) >> 16;
    const int s = lane - g * nb;
    uint2* mt = mtab[wl];
    switch (bc) {
#define HC_CHAIN_CASE(W)                                                                                   \
    case W:                                                                                                \
        if (eq)                                                                                            \
            run_chain<W, true, true>(a, slut, G, T, nb, lane, g, s, pidtab[wl], rtab[wl], mt, rslot[wl]);  \
        else                                                                                               \
            run_chain<W, false, false>(a, slut, G, T, nb, lane, g, s, pidtab[wl], rtab[wl], mt, rslot[wl]); \
        break;
        HC_SEG_WIDTHS(HC_CHAIN_CASE)
#undef HC_CHAIN_CASE
    default: break;
    }
    __builtin_amdgcn_wave_barrier();
    const int nr = __builtin_amdgcn_readfirstlane(rslot[wl][0]);
    if (nr > 0) {   // the fp64 rescue of the flagged pairs kept in the slots (seg_common.hpp)
        const bool few = a.inker_count != nullptr && nr <= 2;
        for (int j = 0; j < min(nr, kChainRescueSlots); ++j)
            rescue_or_defer(a, few, __builtin_amdgcn_readfirstlane(rslot[wl][1 + j]), lane, 0, mt);
    }
}

}  // namespace

#ifndef HC_SEG_OCC
#define HC_SEG_OCC 3
#endif

hipError_t launch_chain_f32(const LaneArgs& a, hipStream_t s)
{
    if (a.n_waves <= 0) return hipSuccess;
    hipLaunchKernelGGL((phmm_chain_kernel<HC_SEG_OCC>), dim3((a.n_waves + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
