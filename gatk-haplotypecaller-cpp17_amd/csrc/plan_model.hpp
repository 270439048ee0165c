// The planners' cost model of the column-segmented fp32 kernel (shared by the
// host planner, planner.cpp, and the device-planned flat path, flat_plan.cpp).
//
// A pair of hap length H runs on nb lanes of BC columns (BC one of the
// compiled widths, kSegMinBC..kSegMaxBC in steps of 2); a wave costs about
// 13 instructions per column plus ~26 per step over R + nb - 1 steps. The pass
// takes one width cap; each hap then has two candidates, nb0 = ceil(H / cap)
// lanes or one more, each at the narrowest width that covers H.
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>

#include "kernels.hpp"

namespace hcphmm {
namespace eng {

constexpr int kNCaps = 7;
constexpr int kCaps[kNCaps] = {64, 48, 32, 24, 16, 12, 8};

// A hap's two segmented-wave candidates: nb0 = ceil(H / cap) lanes or one more,
// each with the narrowest compiled width covering H.
struct Cand {
    uint8_t bc[2], nb[2];
};
static_assert(sizeof(Cand) == sizeof(uint32_t), "Cand packs into a word");

// seg_width_ceil as a table (the planners call it per hap and cap).
inline const std::array<int8_t, kSegMaxBC + 1>& width_ceil_table()
{
    static const std::array<int8_t, kSegMaxBC + 1> t = [] {
        std::array<int8_t, kSegMaxBC + 1> x{};
        for (int w = 0; w <= kSegMaxBC; ++w) x[size_t(w)] = int8_t(seg_width_ceil(w));
        return x;
    }();
    return t;
}

inline Cand cand_of(int H, int cap)
{
    const auto& wc = width_ceil_table();
    const int nb0 = std::min(64, (H + cap - 1) / cap);
    Cand c{};
    for (int q = 0; q < 2; ++q) {
        const int nb = std::min(nb0 + q, 64);
        const int bc = wc[size_t(std::min(kSegMaxBC, (H + nb - 1) / nb))];
        c.bc[q] = uint8_t(bc);
        c.nb[q] = uint8_t((H + bc - 1) / bc);
    }
    return c;
}

// Modelled wave instructions of nb lanes of bc columns over R rows: 13 per
// column + 26 per step, R + nb - 1 steps, times the lane-waste weight.
inline float seg_cost(int nb, int bc, int R, const float* waste)
{
    return float(int64_t(nb) * (13 * bc + 26) * (R + nb - 1)) * waste[nb];
}

// Lane-waste weights: half the waste of a wave of such pairs alone
// (floor(64 / nb) groups; uniform batches pack like that, mixed ones fill the
// gaps with others), the full waste (planners that pack one lane count per
// wave), and with few waves the wave's own time (per lane).
inline const float* waste_half()
{
    static const std::array<float, 65> f = [] {
        std::array<float, 65> x{};
        for (int nb = 1; nb <= 64; ++nb) x[size_t(nb)] = std::sqrt(64.f / float((64 / nb) * nb));
        return x;
    }();
    return f.data();
}
inline const float* waste_full()
{
    static const std::array<float, 65> f = [] {
        std::array<float, 65> x{};
        for (int nb = 1; nb <= 64; ++nb) x[size_t(nb)] = 64.f / float((64 / nb) * nb);
        return x;
    }();
    return f.data();
}
inline const float* waste_per_lane()
{
    static const std::array<float, 65> f = [] {
        std::array<float, 65> x{};
        for (int nb = 1; nb <= 64; ++nb) x[size_t(nb)] = 1.f / float(nb);
        return x;
    }();
    return f.data();
}

// Accumulate one hap (weight m = the pairs it stands for) into the per-cap
// lane and work totals of the cap model (ravg: the batch's mean read length).
inline void cap_sample(int H, double ravg, int64_t m, int64_t* lanes, double* work)
{
    const auto& wc = width_ceil_table();
    for (int q = 0; q < kNCaps; ++q) {
        const int nbq = std::min(64, (H + kCaps[q] - 1) / kCaps[q]);
        const int bc = wc[size_t(std::min(kSegMaxBC, (H + nbq - 1) / nbq))];
        const int nb = (H + bc - 1) / bc;
        lanes[q] += m * nb;
        work[q] += double(m) * nb * (ravg + nb - 1) * (13.0 * bc + 30.0);
    }
}

// The pass's width cap: the one minimising a modelled pass time. Up to two
// rounds of resident waves (3 per SIMD) the SIMD with the most waves sets the
// time, its last round issuing at half rate if it holds one wave (n waves:
// 3 floor(n/3) + {0, 2, 2}); more rounds: waves start as slots free up, so
// the pass time follows the total work (a ceil() there once picked cap 48 for
// a 415 x 128 region: 1.05 ms vs 0.94 at cap 64). few_waves: the pass gives
// each SIMD at most ~3 waves (latency-bound: prefer more lanes).
struct CapChoice {
    int cap = kSegMaxBC;
    bool few_waves = false;
};
inline CapChoice choose_cap(const int64_t* lanes, const double* work, int n_cu)
{
    CapChoice r;
    if (lanes[0] <= 0) return r;
    const double simds = 4.0 * n_cu;
    double best = 0;
    for (int c = 0; c < kNCaps; ++c) {
        const double waves = double(lanes[c]) / 60.0;   // ~60 of 64 lanes filled
        const double per_simd = waves / simds;
        double rounds = per_simd;
        if (per_simd <= 6.0) {
            const int n = std::max(1, int(std::ceil(per_simd - 1e-9)));
            rounds = 3.0 * (n / 3) + (n % 3 ? 2.0 : 0.0);
        }
        const double est = rounds * work[c] / 60.0 / waves;
        if (c == 0 || est < best * 0.98) {
            best = est;
            r.cap = kCaps[c];
            r.few_waves = waves <= 3.0 * simds;
        }
    }
    return r;
}

}  // namespace eng
}  // namespace hcphmm
