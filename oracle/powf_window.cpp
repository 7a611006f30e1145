// powf_window.cpp -- test infrastructure for the fast exact paths of the
// device powf (cfd-simulations_amd/csrc/libm_powf.hpp: powf_sq, powf_sqrt).
//
// 1. Measures, over EVERY float input, how far glibc powf's double result
//    (before its final rounding to float; libm_powf.hpp's powf_log2 +
//    powf_exp2, which restate glibc 2.35's e_powf.c) lies from the exact value:
//    y = 2 over all 2^32 floats (the exact square is exact in double), y = 0.5
//    over all 2^31 non-negative floats (against the correctly rounded double
//    sqrt, itself within 2^-29 float ulp of the exact root).  The unit is 2^-29
//    of the result's float ulp: the bits below the float's last place in a
//    double.  Prints the maxima and the windows (1.05x + 4) to compile in.
// 2. Checks powf_sq(x) == libm powf(x, 2.0f) and powf_sqrt(x) == libm
//    powf(x, 0.5f) bit for bit for every float x (NaNs: both NaN), with the
//    windows libm_powf.hpp compiles in (or -DCFD_POWF_SQ_WIN=..
//    -DCFD_POWF_SQRT_WIN=..), and reports how often the fast path is left.
//
//   g++ -O2 -fopenmp -ffp-contract=off -fno-builtin -DCFD_LIBM_HOST \
//       [-DCFD_POWF_SQ_WIN=W2 -DCFD_POWF_SQRT_WIN=W5] powf_window.cpp -o powf_window
//   ./powf_window measure   |   ./powf_window verify
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../cfd-simulations_amd/csrc/libm_powf.hpp"

using namespace cfd::libm;

// |e - exact| in units of 2^-29 of exact's float ulp (exact > 0, float-normal)
static double err_units(double e, double exact) {
    int k;
    std::frexp(exact, &k);  // exact in [2^(k-1), 2^k): float ulp 2^(k-24)
    return std::fabs(std::ldexp(e - exact, 29 - (k - 24)));
}

static int measure() {
    double max2 = 0, max5 = 0;
    uint32_t arg2 = 0, arg5 = 0;
#pragma omp parallel
    {
        double m2 = 0, m5 = 0;
        uint32_t a2 = 0, a5 = 0;
#pragma omp for schedule(dynamic, 65536)
        for (int64_t b = 0x00800000; b < 0x7f800000; ++b) {  // positive normal floats
            const uint32_t ix = (uint32_t)b;
            const float x = asf32u(ix);
            // y = 2: the sign of x does not matter (2 is an even integer)
            const double sq = (double)x * (double)x;
            if (sq >= 0x1p-126 && sq < 0x1p127) {
                const double ylogx = 2.0 * powf_log2(ix);
                const double e = powf_exp2(ylogx, 0);
                const double u = err_units(e, sq);
                if (u > m2) { m2 = u; a2 = ix; }
            }
            const double rt = std::sqrt((double)x);
            const double e5 = powf_exp2(0.5 * powf_log2(ix), 0);
            const double u5 = err_units(e5, rt);
            if (u5 > m5) { m5 = u5; a5 = ix; }
        }
#pragma omp critical
        {
            if (m2 > max2) { max2 = m2; arg2 = a2; }
            if (m5 > max5) { max5 = m5; arg5 = a5; }
        }
    }
    // subnormal x normalise inside powf; their squares underflow (slow path),
    // their roots are handled by the x > 0 test plus the window like any other
    printf("y=2:   max |e - x*x|     = %.1f units (2^-29 ulp) at x=%a\n", max2, (double)asf32u(arg2));
    printf("y=0.5: max |e - sqrt(x)| = %.1f units (2^-29 ulp) at x=%a (+1 for the double sqrt's rounding)\n",
           max5, (double)asf32u(arg5));
    printf("windows (max x 1.05 + 4): -DCFD_POWF_SQ_WIN=%uu -DCFD_POWF_SQRT_WIN=%uu\n",
           (uint32_t)std::ceil(1.05 * max2) + 4, (uint32_t)std::ceil(1.05 * (max5 + 1)) + 4);
    return 0;
}

static int verify() {
    long long bad2 = 0, bad5 = 0, slow2 = 0, slow5 = 0, nonneg = 0;
#pragma omp parallel for schedule(dynamic, 65536) reduction(+ : bad2, bad5, slow2, slow5, nonneg)
    for (int64_t b = 0; b <= 0xffffffffLL; ++b) {
        const uint32_t ix = (uint32_t)b;
        const float x = asf32u(ix);
        const float w2 = ::powf(x, 2.0f), g2 = powf_sq(x);
        if (!(asu32f(w2) == asu32f(g2) || (std::isnan(w2) && std::isnan(g2)))) {
            if (bad2 < 5) printf("  y=2 x=%a libm=%a fast=%a\n", (double)x, (double)w2, (double)g2);
            ++bad2;
        }
        float tmp;
        if (!powf_sq_fast(x, tmp)) ++slow2;
        const float w5 = ::powf(x, 0.5f), g5 = powf_sqrt(x);
        if (!(asu32f(w5) == asu32f(g5) || (std::isnan(w5) && std::isnan(g5)))) {
            if (bad5 < 5) printf("  y=0.5 x=%a libm=%a fast=%a\n", (double)x, (double)w5, (double)g5);
            ++bad5;
        }
        if (!(ix >> 31)) {
            ++nonneg;
            if (!powf_sqrt_fast(x, tmp)) ++slow5;
        }
    }
    printf("windows: sq %u, sqrt %u (units of 2^-29 float ulp)\n", kPowfSqWin, kPowfSqrtWin);
    printf("y=2:   %lld of 2^32 floats differ from libm; slow path on %lld (%.4f%%)\n", bad2, slow2,
           100.0 * slow2 / 4294967296.0);
    printf("y=0.5: %lld of 2^32 floats differ from libm; slow path on %lld of %lld non-negative (%.4f%%)\n", bad5,
           slow5, nonneg, 100.0 * slow5 / nonneg);
    return (bad2 || bad5) ? 1 : 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "measure")) return measure();
    return verify();
}
