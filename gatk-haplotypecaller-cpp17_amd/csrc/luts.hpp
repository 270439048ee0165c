// Host-side Phred / transition tables of the PairHMM engine.
//
// Same values as the reference's Context<float>/Context<double>
// (pairhmm/native/Context.h:13-175), rebuilt here in their own code:
//   ph2pr[x]   = 10^(-x/10), x < 128         (powf in float, pow in double)
//   jac[k]     = log10(1 + 10^(-k*1e-4))     k <= 80000, rounded to NUMBER
//   mm(i, j)   = 1 - 10^(log10sum(-i/10, -j/10)), the log-sum evaluated in
//                NUMBER precision with the Jacobian table, the rest in double
//   INITIAL    = 2^120 (f32) / 2^1020 (f64), LOG10_INITIAL = log10(INITIAL)
// Parity with the reference tables is a test (tests/test_luts.py) against the
// golden LUT dump taken from the reference build.
#pragma once
#include <cstdint>
#include <vector>

namespace hcphmm {

constexpr int kMaxQual = 254;                                   // Context.h:6
constexpr int kMMEntries = ((kMaxQual + 1) * (kMaxQual + 2)) / 2; // 32640
constexpr int kQuals = 128;                                     // quality bytes are & 127
constexpr int kMMSmall = kQuals * (kQuals + 1) / 2;             // 8256: hi < 128

// Device table layout (per precision), contiguous:
//   [ph2pr 128][pm 128][px 128][gapm 128][mm 8256]
// pm[q] = 1 - ph2pr[q], px[q] = ph2pr[q] / 3, gapm[c] = 1 - ph2pr[c], all
// evaluated in NUMBER precision exactly as stripeINITIALIZATION
// (avx-pairhmm-template.h:152-158) and initializeVectors (:115).
constexpr int kOffPh2pr = 0;
constexpr int kOffPm = 128;
constexpr int kOffPx = 256;
constexpr int kOffGapm = 384;
constexpr int kOffMM = 512;
constexpr int kTableLen = kOffMM + kMMSmall;

struct Luts {
    float ph2pr_f[kQuals];
    double ph2pr_d[kQuals];
    std::vector<float> mm_f;    // kMMEntries
    std::vector<double> mm_d;   // kMMEntries
    float init_f, log10_init_f;
    double init_d, log10_init_d;
    std::vector<float> dev_f;   // kTableLen
    std::vector<double> dev_d;  // kTableLen
};

// Built once (thread-safe).
const Luts& luts();

inline int mm_index(int a, int b)
{
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    return ((hi * (hi + 1)) >> 1) + lo;
}

}  // namespace hcphmm
