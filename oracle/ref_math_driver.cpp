// Driver around the REFERENCE MathUtils (utils/math_utils.hpp) — TEST INFRASTRUCTURE ONLY.
// Compiled by oracle/Makefile against the reference header where it lies
// (header-only, <array>/<cmath>); nothing is copied into this repository.
#include "math_utils.hpp"

extern "C" double ref_approx_log10_sum_log10(double a, double b)
{
    return hc::MathUtils::approximate_log10_sum_log10(a, b);
}
