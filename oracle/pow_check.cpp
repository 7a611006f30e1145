// pow_check.cpp -- test infrastructure: compares the device restatement of
// glibc's double pow (cfd-simulations_amd/csrc/libm_pow.hpp, compiled here for
// the host) with this host's libm pow, bit for bit, on random and edge-case
// inputs at the exponents the reference uses (2 and 0.5: v5.py:155's
// (u**2 + v**2)**0.5 in float64).  Prints the number of mismatches per
// exponent and exits 1 if any.
//   g++ -O2 -ffp-contract=off -mfma -DCFD_LIBM_HOST -I.. pow_check.cpp -o pow_check
//   ./pow_check [n_random]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../cfd-simulations_amd/csrc/libm_pow.hpp"

static uint64_t bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
static double from(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    volatile double (*libm_pow)(double, double) = nullptr;
    (void)libm_pow;
    std::mt19937_64 rng(12345);
    std::vector<double> xs = {0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 1e-310, -1e-310, 4.9e-324, 1e300, -1e300, 1e-300,
                              INFINITY, -INFINITY, 1.7976931348623157e308, 2.2250738585072014e-308};
    for (long i = 0; i < n; ++i) {
        const uint64_t r = rng();
        switch (i % 4) {
            case 0: xs.push_back(from(r & 0x7fffffffffffffffULL)); break;  // any positive pattern
            case 1: xs.push_back(from(r)); break;                           // any pattern
            case 2: xs.push_back(std::ldexp((double)(r >> 11) * 0x1p-53, (int)(r % 40) - 20)); break;  // O(1)
            default: xs.push_back(-std::ldexp((double)(r >> 11) * 0x1p-53, (int)(r % 12) - 6)); break;
        }
    }
    int bad_total = 0;
    for (double y : {2.0, 0.5}) {
        long bad = 0, differ_from_naive = 0;
        for (double x : xs) {
            const double want = std::pow(x, y);
            const double got = cfd::libm::pow(x, y);
            const bool same = bits(want) == bits(got) || (std::isnan(want) && std::isnan(got));
            if (!same) {
                if (bad < 5) printf("  y=%g x=%a libm=%a port=%a\n", y, x, want, got);
                ++bad;
            }
            const double naive = y == 2.0 ? x * x : std::sqrt(x);
            if (!std::isnan(want) && bits(naive) != bits(want)) ++differ_from_naive;
        }
        printf("y=%g: %ld inputs, %ld mismatches vs libm (libm differs from the correctly rounded form on %ld)\n", y,
               (long)xs.size(), bad, differ_from_naive);
        bad_total += bad != 0;
    }
    return bad_total ? 1 : 0;
}
