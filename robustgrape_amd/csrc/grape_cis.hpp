// grape_cis.hpp -- e^{i t} for the phase-covariant walks' per-step phases (round 6).
//
// The walks take p_k = e^{i a x_k} once per (step, lane) (grape_walk.hpp GAUGE): with the library
// sincos that was ~120 VALU instructions per step of the merged gradient walk's ~650 -- the
// library reduces every argument with the Payne-Hanek path ready (v_trig_preop) and evaluates both
// kernels behind selects.  Here: Cody-Waite reduction by pi/2 in three FMA steps (|t| <= kCisFast,
// so |k| < 2^17 and the two 33-bit pieces of pi/2 reduce exactly), then fdlibm's __kernel_sin / __kernel_cos polynomials on |r| <= pi/4
// (< 1 ulp each) and the quadrant by selects.  Larger |t| (never reached by the reference's laser
// phases, |a x| ~ 2 pi) take the library sincos in a divergent branch.  Checked against x87 long
// double sinl / cosl on the host (tests/test_cis_cpu.py): max error 1 ulp of 1.
#pragma once

#include <hip/hip_runtime.h>

namespace grape_cis {

constexpr double kCisFast = 1.0e5;  // |t| above this: the library sincos
constexpr double kTwoOverPi = 6.36619772367581382433e-01;
// pi/2 = kPio2Hi + kPio2Mid + kPio2Lo: hi and mid have 33 significant bits (fdlibm pio2_1, pio2_2),
// so the first two reduction steps are exact for |k| < 2^20; lo (fdlibm pio2_2t) the rounded remainder
constexpr double kPio2Hi = 1.57079632673412561417e+00;
constexpr double kPio2Mid = 6.07710050630396597660e-11;
constexpr double kPio2Lo = 2.02226624879595063154e-21;
// fdlibm k_sin.c / k_cos.c
constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;

// The constants of cis_fast by index: reduction, then sin, then cos coefficients
enum : int { kTwoPi_ = 0, kHi_, kMid_, kLo_, S1_, S2_, S3_, S4_, S5_, S6_, C1_, C2_, C3_, C4_, C5_, C6_, kCisN };
constexpr double kCisCoef[kCisN] = {kTwoOverPi, kPio2Hi, kPio2Mid, kPio2Lo, S1, S2, S3, S4, S5, S6,
                                    C1, C2, C3, C4, C5, C6};

// sin and cos of t, |t| <= kCisFast.  k(i) returns constant i of kCisCoef: on the host the array itself
// (tests/test_cis_cpu.py); on the device a scalar load from a __constant__ copy (grape_walk.hpp
// gauge_cis), so that every Horner step is one v_fma_f64 with an SGPR operand instead of a
// v_fmac_f64 behind two v_mov_b32 of a literal (the walks are built without MachineLICM, so literals
// were re-materialised every step)
template <class K>
__host__ __device__ __forceinline__ void cis_fast(double t, double &s, double &c, K k) {
    const double kf = rint(t * k(kTwoPi_));
    double r = fma(-kf, k(kHi_), t);
    r = fma(-kf, k(kMid_), r);
    r = fma(-kf, k(kLo_), r);
    const double z = r * r;
    // sin r = r + r^3 (S1 + z (S2 + ... + z S6))
    const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, k(S6_), k(S5_)), k(S4_)), k(S3_)), k(S2_)), k(S1_));
    const double sr = fma(z * r, ps, r);
    // cos r = w + ((1 - w) - z / 2 + z^2 (C1 + ... + z C6)), w = 1 - z / 2 (fdlibm's compensated form)
    const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, k(C6_), k(C5_)), k(C4_)), k(C3_)), k(C2_)), k(C1_));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + (z * z) * pc);
    const int q = (int)kf & 3;  // quadrant (two's complement: & 3 is k mod 4 for negative k too)
    const double a = (q & 1) ? cr : sr, b = (q & 1) ? sr : cr;
    s = (q & 2) ? -a : a;
    c = ((q + 1) & 2) ? -b : b;
}

}  // namespace grape_cis
