// Host LUT construction; see luts.hpp for the definitions and reference cites.
// Compiled with -ffp-contract=off: every table entry is a chain of separately
// rounded IEEE operations, as in the reference build (no -mfma).
#include "luts.hpp"

#include <cmath>
#include <mutex>

namespace hcphmm {
namespace {

constexpr double kJacStep = 0.0001;        // Context.h:8
constexpr double kJacTolerance = 8.0;      // Context.h:7
constexpr int kJacEntries = 80001;         // (int)(8.0 / 0.0001) + 1

// log10(10^a + 10^b) by table, in precision N (ContextBase::approximateLog10SumLog10).
template <typename N>
N log10_sum(const std::vector<N>& jac, N a, N b)
{
    N lo = a, hi = b;
    if (lo > hi) std::swap(lo, hi);
    const N diff = hi - lo;
    if (diff >= static_cast<N>(kJacTolerance)) return hi;
    const N scaled = diff * static_cast<N>(1.0 / kJacStep);
    const int k = scaled > N(0) ? static_cast<int>(scaled + N(0.5)) : static_cast<int>(scaled - N(0.5));
    return hi + jac[k];
}

template <typename N>
void fill_mm(std::vector<N>& mm)
{
    std::vector<N> jac(kJacEntries);
    for (int k = 0; k < kJacEntries; ++k)
        jac[k] = static_cast<N>(std::log10(1.0 + std::pow(10.0, -static_cast<double>(k) * kJacStep)));
    const double inv_ln10 = 1.0 / std::log(10.0);
    mm.assign(kMMEntries, N(0));
    for (int hi = 0; hi <= kMaxQual; ++hi) {
        const int row = (hi * (hi + 1)) >> 1;
        for (int lo = 0; lo <= hi; ++lo) {
            const double s = static_cast<double>(
                log10_sum<N>(jac, static_cast<N>(-0.1 * hi), static_cast<N>(-0.1 * lo)));
            const double l = std::log1p(-std::fmin(1.0, std::pow(10.0, s))) * inv_ln10;
            mm[row + lo] = static_cast<N>(std::pow(10.0, l));
        }
    }
}

template <typename N>
void device_table(const N* ph2pr, const std::vector<N>& mm, std::vector<N>& out)
{
    out.assign(kTableLen, N(0));
    for (int x = 0; x < kQuals; ++x) {
        const N p = ph2pr[x];
        out[kOffPh2pr + x] = p;
        out[kOffPm + x] = N(1) - p;
        out[kOffPx + x] = p / N(3);
        out[kOffGapm + x] = N(1) - p;
    }
    for (int k = 0; k < kMMSmall; ++k) out[kOffMM + k] = mm[k];
}

Luts* build()
{
    auto* L = new Luts();
    for (int x = 0; x < kQuals; ++x) {
        L->ph2pr_f[x] = std::pow(10.f, -static_cast<float>(x) / 10.f);
        L->ph2pr_d[x] = std::pow(10.0, -static_cast<double>(x) / 10.0);
    }
    fill_mm<float>(L->mm_f);
    fill_mm<double>(L->mm_d);
    L->init_f = std::ldexp(1.f, 120);
    L->log10_init_f = std::log10(L->init_f);
    L->init_d = std::ldexp(1.0, 1020);
    L->log10_init_d = std::log10(L->init_d);
    device_table<float>(L->ph2pr_f, L->mm_f, L->dev_f);
    device_table<double>(L->ph2pr_d, L->mm_d, L->dev_d);
    return L;
}

}  // namespace

const Luts& luts()
{
    static std::once_flag once;
    static Luts* L = nullptr;
    std::call_once(once, [] { L = build(); });
    return *L;
}

}  // namespace hcphmm
