// Host check of grape_cis::cis_fast (robustgrape_amd/csrc/grape_cis.hpp, the phase-covariant walks'
// e^{i t}) against x87 long double sinl / cosl: prints the largest absolute error in units of 2^-52 over
// 4 million arguments in four ranges, and the values at exact points.
#include "grape_cis.hpp"

#include <cmath>
#include <cstdio>
#include <random>

int main() {
    std::mt19937_64 g(1);
    double worst_s = 0, worst_c = 0;
    auto err = [](long double ref, double got) { return (double)(fabsl((long double)got - ref) / 2.220446049250313e-16L); };
    auto k = [](int i) { return grape_cis::kCisCoef[i]; };
    const double span[4] = {7.0, 100.0, 1.0e5, 1.0e-3};
    for (int it = 0; it < 4000000; ++it) {
        const double t = std::uniform_real_distribution<double>(-span[it % 4], span[it % 4])(g);
        double s, c;
        grape_cis::cis_fast(t, s, c, k);
        worst_s = std::fmax(worst_s, err(sinl((long double)t), s));
        worst_c = std::fmax(worst_c, err(cosl((long double)t), c));
    }
    double s0, c0, s1, c1;
    grape_cis::cis_fast(0.0, s0, c0, k);
    grape_cis::cis_fast(-0.0, s1, c1, k);
    printf("sin_err %.4f\ncos_err %.4f\nsin0 %.17g\ncos0 %.17g\nsinm0_sign %d\n", worst_s, worst_c, s0, c0, (int)std::signbit(s1));
    return 0;
}
