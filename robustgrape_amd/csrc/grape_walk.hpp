// grape_walk.hpp -- chunk walks: the sector pipeline without HBM intermediates (round 3).
//
// For sector classes of D <= kWalkMaxD levels without error sources (the Rydberg sectors of
// 4 and 2 levels), ONE LANE OWNS ONE (sub-evaluation b', chunk c) and walks the chunk's
// steps twice:
//
//   k_walk_fwd   E_k = exp(A_k) and the chunk chain Q <- E_k Q, in registers; writes only
//                the chunk total T_c (k_scan then scans the totals: B.Tc).
//                                                     UnitaryCalculations.jl:45-47,99
//   k_walk_grad  X = M'_c = Carry_c M Carry_c^dag (formed in the lane) and per step
//                  E_k again, Y_k = X E_k^dag, and for every gradient parameter u the
//                  eps-variant E'_k contracted on the spot,
//                  F_dx[u,k] = Re tr(Y_k (E'_k - E_k)/eps)    (FidelityCalculations.jl:56-76),
//                  then X <- E_k Y_k.
//
// Algebra (grape_kernels.hpp): F_dx[u,k] = Re tr(C_{k-1} M C_k^dag dE_{k,u}) with
// C_k = E_k C_{k-1}, so with X_{k-1} = C_{k-1} M C_{k-1}^dag (= M'_c at a chunk start) the
// gradient kernel of step k is Y_k = X_{k-1} E_k^dag and X_k = E_k X_{k-1} E_k^dag = E_k Y_k.
// The nominal propagator is recomputed in the second walk instead of being stored: at 4
// levels one exponential costs ~1.2 k FMAs per lane, storing and re-reading it 512 B of HBM
// traffic, and the round-2 pipeline moved 1.08 MB of E / Q intermediates per evaluation.
//
// Arithmetic.  A = -i dt H is skew-Hermitian (grape_plan_create checks that H0's terms are
// Hermitian), A^2 Hermitian and A^3 skew-Hermitian, so each is kept COMPRESSED: its diagonal
// (the imaginary / real parts) and strict upper triangle -- 16 instead of 32 doubles at D = 4,
// and every product with a diagonal entry is 2 FMAs instead of 4.  The exponential is the
// row-group kernels' solve-free Taylor evaluation (Paterson-Stockmeyer in A^3; degree 12, 9 or 6
// by the |re|+|im| column bound of A shifted by the midpoint of its diagonal, sm_regime), column
// by column: column i of exp(A) needs
// only column i of A, A^2 and the running vector, so no full matrix is materialised for it.
// Above the Taylor-12 range (exact 1-norm > 0.25) the lane takes Taylor 30 of A / 2^s with
// |A / 2^s|_1 <= 3.2 and squares s times (Higham's scaling and squaring; kWalkThetaHi) -- where
// the row-group path parks the item for Julia's Pade 7 / 9 / 13, with the same measured accuracy.  Both are
// exp(A) to a few ulps (T0); the FD differences keep the reference's (E' - E) / eps form,
// element by element, before the contraction.
//
// Registers (D = 4): X 64 VGPRs across the walk, the A / A^2 / A^3 set 96, one vector of
// temporaries; in k_walk_grad E lives in the lane's private LDS slot (17 complex, padded so
// that the 16-B reads of 16 lanes hit 64 distinct banks).  The walks are compiled in their own
// translation unit (grape_walk_inst.hip) without MachineLICM: hoisting the trig / log
// polynomial constants of the inlined ocml calls out of the step loop pinned ~50 VGPRs and
// spilled the walk state (k_walk_grad<2>: 128 VGPRs + 18 spilled -> 98, none spilled).
#pragma once
#include "grape_cis.hpp"
#include "grape_kernels.hpp"
#include "grape_walk_api.hpp"

namespace grape {

constexpr int kWalkBlock = kWalkBlockA;
// 1/k! as literals (the column kernels index them with compile-time constants)
__device__ __forceinline__ constexpr double inv_fact(int k) {
    return k == 0 ? 1.0 : k == 1 ? 1.0 : k == 2 ? 0.5 : k == 3 ? 1.0 / 6 : k == 4 ? 1.0 / 24 : k == 5 ? 1.0 / 120
         : k == 6 ? 1.0 / 720 : k == 7 ? 1.0 / 5040 : k == 8 ? 1.0 / 40320 : k == 9 ? 1.0 / 362880
         : k == 10 ? 1.0 / 3628800 : k == 11 ? 1.0 / 39916800 : 1.0 / 479001600;
}

// ---------------------------------------------------------------------------
// compressed (skew-)Hermitian matrices
// ---------------------------------------------------------------------------
template <int D>
struct SM {
    static constexpr int NU = D * (D - 1) / 2;
    double d[D];  // diagonal: imaginary parts (skew-Hermitian) or real parts (Hermitian)
    cd u[NU];     // strict upper triangle, row by row
};
__host__ __device__ constexpr int uix(int D, int j, int k) { return j * D - j * (j + 1) / 2 + (k - j - 1); }

// element (j, k) (compile-time indices after unrolling)
template <int D, bool HERM>
__device__ __forceinline__ cd sm_el(const SM<D> &M, int j, int k) {
    if (j == k) return HERM ? cmake(M.d[j], 0.0) : cmake(0.0, M.d[j]);
    if (j < k) return M.u[uix(D, j, k)];
    const cd t = M.u[uix(D, k, j)];
    return HERM ? cmake(t.re, -t.im) : cmake(-t.re, t.im);
}
// c += M[j][k] v: 2 FMAs for a diagonal entry, 4 otherwise
template <int D, bool HERM>
__device__ __forceinline__ void sm_mac(cd &c, const SM<D> &M, int j, int k, cd v) {
    if (j == k) {
        const double s = M.d[j];
        if (HERM) {
            c.re = fma(s, v.re, c.re);
            c.im = fma(s, v.im, c.im);
        } else {
            c.re = fma(-s, v.im, c.re);
            c.im = fma(s, v.re, c.im);
        }
    } else {
        cmac(c, sm_el<D, HERM>(M, j, k), v);
    }
}
template <int D, bool HERM>
__device__ __forceinline__ void sm_matvec(const SM<D> &M, const cd (&v)[D], cd (&out)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        cd c = czero();
#pragma unroll
        for (int k = 0; k < D; ++k) sm_mac<D, HERM>(c, M, j, k, v[k]);
        out[j] = c;
    }
}

// A^2 (Hermitian) and A^3 = A A^2 (skew-Hermitian) of a skew-Hermitian A
template <int D>
__device__ __forceinline__ void sm_cube(const SM<D> &A, SM<D> &A2, SM<D> &A3) {
#pragma unroll
    for (int j = 0; j < D; ++j) {  // (A^2)_jj = -sum_m |A_jm|^2
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < D; ++m) {
            if (m == j) {
                s = fma(A.d[j], A.d[j], s);
            } else {
                const cd a = sm_el<D, false>(A, j, m);
                s = fma(a.re, a.re, s);
                s = fma(a.im, a.im, s);
            }
        }
        A2.d[j] = -s;
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int k = j + 1; k < D; ++k) {
            cd c = czero();
#pragma unroll
            for (int m = 0; m < D; ++m) sm_mac<D, false>(c, A, j, m, sm_el<D, false>(A, m, k));
            A2.u[uix(D, j, k)] = c;
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {  // Im (A^3)_jj
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < D; ++m) {
            const cd b = sm_el<D, true>(A2, m, j);
            if (m == j) {
                s = fma(A.d[j], b.re, s);
            } else {
                const cd a = sm_el<D, false>(A, j, m);
                s = fma(a.re, b.im, s);
                s = fma(a.im, b.re, s);
            }
        }
        A3.d[j] = s;
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int k = j + 1; k < D; ++k) {
            cd c = czero();
#pragma unroll
            for (int m = 0; m < D; ++m) sm_mac<D, false>(c, A, j, m, sm_el<D, true>(A2, m, k));
            A3.u[uix(D, j, k)] = c;
        }
    }
}

// The high-norm regime (|A - i mu I|_1 > 0.25, where Julia's exp! takes Pade 7 / 9 / 13): Taylor 30
// (Paterson-Stockmeyer in A^3, kWalkNstHi = 9 Horner steps) of A / 2^s with s = max(0,
// ceil(log2(|A|_1 / kWalkThetaHi))) and s squarings.  The remainder at 3.2 is 3.2^31 / 31! = 6e-19;
// the measured errors of E, (E' - E) / eps and the eps2 mixed stencil against an extended-precision
// reference equal Julia's Pade 13 at every |A|_1 from 0.3 to 80 (scripts/probes/highnorm_study.py,
// DESIGN.md 4.2), where the round-3 Taylor 12 at 0.25 (s = ceil(log2 4|A|_1): 4 more squarings) was up
// to 10x worse.  Coefficients by index from constant memory (the Horner loop is not unrolled: a rare
// path, kept out of the common path's registers and code).
constexpr double kWalkThetaHi = 3.2;
constexpr int kWalkNstHi = 9;
__host__ __device__ constexpr double inv_fact_r(int k) { return k <= 1 ? 1.0 : inv_fact_r(k - 1) / k; }
static __constant__ double kWalkInvFact[3 * kWalkNstHi + 4] = {
    inv_fact_r(0),  inv_fact_r(1),  inv_fact_r(2),  inv_fact_r(3),  inv_fact_r(4),  inv_fact_r(5),  inv_fact_r(6),
    inv_fact_r(7),  inv_fact_r(8),  inv_fact_r(9),  inv_fact_r(10), inv_fact_r(11), inv_fact_r(12), inv_fact_r(13),
    inv_fact_r(14), inv_fact_r(15), inv_fact_r(16), inv_fact_r(17), inv_fact_r(18), inv_fact_r(19), inv_fact_r(20),
    inv_fact_r(21), inv_fact_r(22), inv_fact_r(23), inv_fact_r(24), inv_fact_r(25), inv_fact_r(26), inv_fact_r(27),
    inv_fact_r(28), inv_fact_r(29), inv_fact_r(30)};

// The top coefficients of a Paterson-Stockmeyer evaluation in A^3 with nst Horner steps
// (degree 3 nst + 3: nst = 1, 2, 3 -> Taylor 6, 9, 12)
__device__ __forceinline__ double ps_top(int nst, int m) {
    return nst == 1 ? inv_fact(3 + m) : nst == 2 ? inv_fact(6 + m) : inv_fact(9 + m);
}

// x = column i of the Taylor polynomial, Paterson-Stockmeyer in A^3 (grape_device.hpp
// expm_taylor): degree 3 nst + 3 (12, 9 or 6).  B_j = c_3j I + c_3j+1 A + c_3j+2 A^2.
template <int D>
__device__ __forceinline__ void sm_taylor_col(int nst, int i, const SM<D> &A, const SM<D> &A2, const SM<D> &A3,
                                              cd (&x)[D]) {
    {
        const double k0 = ps_top(nst, 0), k1 = ps_top(nst, 1), k2 = ps_top(nst, 2), k3 = ps_top(nst, 3);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x[j] = caxpy(k1, sm_el<D, false>(A, j, i), caxpy(k2, sm_el<D, true>(A2, j, i), cscale(k3, sm_el<D, false>(A3, j, i))));
            if (j == i) x[j].re += k0;
        }
    }
#pragma unroll
    for (int st = 2; st >= 0; --st) {
        if (st == 0 || st < nst) {  // (the last step unconditionally: no branch around it)
            cd t[D];
            sm_matvec<D, false>(A3, x, t);
            const double k0 = inv_fact(3 * st), k1 = inv_fact(3 * st + 1), k2 = inv_fact(3 * st + 2);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                x[j] = caxpy(k1, sm_el<D, false>(A, j, i), caxpy(k2, sm_el<D, true>(A2, j, i), t[j]));
                if (j == i) x[j].re += k0;
            }
        }
    }
    pin<D>(x);  // the column is final here: nothing of the next one is scheduled into it
}

// column i of the high-norm regime's Taylor 30 (a2: column i of A^2, from A2 or regenerated)
template <int D, bool KEEP_A2>
__device__ __forceinline__ void sm_taylor_col_hi(int i, const SM<D> &A, const SM<D> &A2, const SM<D> &A3, cd (&x)[D]) {
    cd a2[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        if constexpr (KEEP_A2) {
            a2[j] = sm_el<D, true>(A2, j, i);
        } else {
            cd c = czero();
#pragma unroll
            for (int k = 0; k < D; ++k) sm_mac<D, false>(c, A, j, k, sm_el<D, false>(A, k, i));
            a2[j] = c;
        }
    }
    constexpr int N = kWalkNstHi;
    {
        const double k0 = kWalkInvFact[3 * N], k1 = kWalkInvFact[3 * N + 1], k2 = kWalkInvFact[3 * N + 2],
                     k3 = kWalkInvFact[3 * N + 3];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x[j] = caxpy(k1, sm_el<D, false>(A, j, i), caxpy(k2, a2[j], cscale(k3, sm_el<D, false>(A3, j, i))));
            if (j == i) x[j].re += k0;
        }
    }
#pragma unroll 1
    for (int st = N - 1; st >= 0; --st) {
        cd t[D];
        sm_matvec<D, false>(A3, x, t);
        const double k0 = kWalkInvFact[3 * st], k1 = kWalkInvFact[3 * st + 1], k2 = kWalkInvFact[3 * st + 2];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x[j] = caxpy(k1, sm_el<D, false>(A, j, i), caxpy(k2, a2[j], t[j]));
            if (j == i) x[j].re += k0;
        }
    }
    pin<D>(x);
}

// Degree choice (grape_device.hpp expm_prologue_fast, per lane): 0 = diagonal (isdiag), 3 =
// Taylor 6, 4 = Taylor 9, 5 = Taylor 12, 13 = Taylor 30 of A / 2^s (A scaled here) and s squarings.
//
// Diagonal shift (GRAPE_WALK_SHIFT): the walks exponentiate A - i mu I, i.e. they compute
// E~ = e^{-i mu} exp(A), with mu (`choose`) the midpoint of the diagonal's imaginary parts, which
// minimises the largest diagonal modulus -- the Rydberg 4-level sector (diagonal 0, 0, 0, B = 10)
// drops from |A|_1 ~ 0.17 to ~ 0.09 and takes Taylor 9 (two Horner steps per column instead of
// three).  The phase e^{i mu} is never multiplied in per step: every eps-variant of a step is
// shifted by the nominal propagator's mu (choose = false), so E' - E = e^{i mu} (E~' - E~) and the
// phase cancels in every sandwich the walks form (Y = X E^dag, X E^dag (E' - E), E X E^dag,
// E^dag dX); only the chunk totals take e^{i sum mu} (walk_phase).  The thresholds bound the
// Taylor remainder sum_{k > m} |A|^k / k! by ~3e-17 (0.015 at m = 6, 0.1 at m = 9; 2.4e-18 at
// 0.25, m = 12).  A diagonal A (kind 0) keeps mu = 0 when choosing, and so does an A whose shifted
// norm still exceeds 0.25 (the high-norm regime: no Horner step to save, more FD noise).
#ifndef GRAPE_WALK_SHIFT
#define GRAPE_WALK_SHIFT 1
#endif
template <int D, bool SHIFT>
__device__ __forceinline__ int sm_regime(SM<D> &A, int &s, double &mu, bool choose) {
    s = 0;
    bool off = false;
#pragma unroll
    for (int t = 0; t < SM<D>::NU; ++t) off = off || A.u[t].re != 0.0 || A.u[t].im != 0.0;
    if (choose) {
        mu = 0.0;
#if GRAPE_WALK_SHIFT
        if (SHIFT && off) {
            double lo = A.d[0], hi = A.d[0];
#pragma unroll
            for (int j = 1; j < D; ++j) {
                lo = fmin(lo, A.d[j]);
                hi = fmax(hi, A.d[j]);
            }
            mu = 0.5 * (lo + hi);
            // Only where the shifted A stays in the Taylor 6 / 9 / 12 regime: above that the shift
            // saves no Horner step and its rounding raises the eps / eps2 stencils' noise (the
            // shifted Taylor 30 at |A|_1 = 2.6 ... 84 measured 3-10x Julia's error on F_dx and
            // F_d2err_dx against an extended-precision exponential, unshifted ~1x:
            // scripts/probes/shift_noise_study.py).
            double nsh = 0.0;
#pragma unroll
            for (int c = 0; c < D; ++c) {
                double ub = fabs(A.d[c] - mu);
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    if (j == c) continue;
                    const cd a = sm_el<D, false>(A, j, c);
                    ub += fabs(a.re) + fabs(a.im);
                }
                nsh = fmax(nsh, ub);
            }
            if (!(nsh <= 0.25)) mu = 0.0;
        }
#endif
    }
    if (!off) return 0;  // (walk_expm shifts the diagonal itself)
    if (SHIFT) {
#pragma unroll
        for (int j = 0; j < D; ++j) A.d[j] -= mu;  // exact for mu = 0
    }
    double nub = 0.0;
#pragma unroll
    for (int c = 0; c < D; ++c) {
        double ub = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const cd a = sm_el<D, false>(A, j, c);
            ub += fabs(a.re) + fabs(a.im);
        }
        nub = c == 0 ? ub : fmax(nub, ub);
    }
    if (nub <= 0.015) return 3;
    if (GRAPE_WALK_SHIFT && SHIFT && nub <= 0.1) return 4;
    if (nub <= 0.25) return 5;
    double nA = 0.0;  // Julia's opnorm(A, 1)
#pragma unroll
    for (int c = 0; c < D; ++c) {
        double cs = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const cd a = sm_el<D, false>(A, j, c);
            cs += sqrt(a.re * a.re + a.im * a.im);
        }
        nA = c == 0 ? cs : fmax(nA, cs);
    }
    if (nA <= 0.015) return 3;
    if (GRAPE_WALK_SHIFT && SHIFT && nA <= 0.1) return 4;
    if (nA <= 0.25) return 5;
    if (!(nA <= 1e300)) return 5;  // NaN / Inf: propagates through the polynomial
    s = nA <= kWalkThetaHi ? 0 : (int)ceil(log2(nA / kWalkThetaHi));  // |A / 2^s|_1 <= 3.2 (Taylor 30)
    const double f = ldexp(1.0, -s);  // exact
#pragma unroll
    for (int j = 0; j < D; ++j) A.d[j] *= f;
#pragma unroll
    for (int t = 0; t < SM<D>::NU; ++t) A.u[t] = cscale(f, A.u[t]);
    return 13;
}

// x = column i of the same polynomial without a stored A^2: column i of A^2 is A (A e_i), one
// matrix-vector product per column (+56 FMAs at D = 4) for 32 fewer live registers.
template <int D>
__device__ __forceinline__ void sm_taylor_col_na2(int nst, int i, const SM<D> &A, const SM<D> &A3, cd (&x)[D]) {
    cd a2[D];  // column i of A is read from A itself (no copy)
#pragma unroll
    for (int j = 0; j < D; ++j) {
        cd c = czero();
#pragma unroll
        for (int k = 0; k < D; ++k) sm_mac<D, false>(c, A, j, k, sm_el<D, false>(A, k, i));
        a2[j] = c;
    }
    {
        const double k0 = ps_top(nst, 0), k1 = ps_top(nst, 1), k2 = ps_top(nst, 2), k3 = ps_top(nst, 3);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x[j] = caxpy(k1, sm_el<D, false>(A, j, i), caxpy(k2, a2[j], cscale(k3, sm_el<D, false>(A3, j, i))));
            if (j == i) x[j].re += k0;
        }
    }
#pragma unroll
    for (int st = 2; st >= 0; --st) {
        if (st == 0 || st < nst) {  // (the last step unconditionally: no branch around it)
            cd t[D];
            sm_matvec<D, false>(A3, x, t);
            const double k0 = inv_fact(3 * st), k1 = inv_fact(3 * st + 1), k2 = inv_fact(3 * st + 2);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                x[j] = caxpy(k1, sm_el<D, false>(A, j, i), caxpy(k2, a2[j], t[j]));
                if (j == i) x[j].re += k0;
            }
        }
    }
    pin<D>(x);
}

// exp(A), column by column into sink(i, column i).  The squaring path (kind 13, rare) parks
// the scaled approximant in the lane's global scratch slot `scr` (two D x D column-major
// tiles) and squares it there element by element, so that it adds no live registers to the
// common path.  FENCE: pin every column and keep the scheduler from overlapping them (register
// discipline at D = 4; at D <= 3 the columns and sectors may interleave for ILP).  KEEP_A2:
// keep A^2 through the column loop (else regenerate its columns, sm_taylor_col_na2).
// mu: the diagonal shift (sm_regime): chosen here and returned (choose), or the nominal's (an
// eps-variant); the columns are those of E~ = exp(A - i mu I).
template <int D, bool FENCE, bool KEEP_A2, bool SHIFT, class Sink>
__device__ __forceinline__ void walk_expm(SM<D> &A, cd *scr, double &mu, bool choose, Sink &&sink) {
    int s = 0;
    const int kind = sm_regime<D, SHIFT>(A, s, mu, choose);
    if (kind == 0) {  // isdiag(A): exp of the diagonal (Julia's fast path)
#pragma unroll
        for (int i = 0; i < D; ++i) {
            cd x[D];
            const double a = A.d[i] - mu;  // (exact for mu = 0)
            const double sn = sin(a), cn = cos(a);  // exp(0) (cos, sin), as the row-group path
#pragma unroll
            for (int j = 0; j < D; ++j) x[j] = (j == i) ? cmake(cn, sn) : czero();
            if (FENCE) pin<D>(x);
            sink(i, x);
        }
        return;
    }
    SM<D> A2, A3;
    sm_cube<D>(A, A2, A3);
    auto col = [&](int nst, int i, cd (&x)[D]) {
        if constexpr (KEEP_A2) sm_taylor_col<D>(nst, i, A, A2, A3, x);
        else sm_taylor_col_na2<D>(nst, i, A, A3, x);
    };
    if (kind != 13) {
        const int nst = kind == 3 ? 1 : kind == 4 ? 2 : 3;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            cd x[D];
            col(nst, i, x);
            sink(i, x);
            if (FENCE) __builtin_amdgcn_sched_barrier(0);
        }
        return;
    }
    cd *T = scr, *R = scr + D * D;
#pragma unroll
    for (int i = 0; i < D; ++i) {  // (unrolled: register arrays are only ever indexed by constants)
        cd x[D];
        sm_taylor_col_hi<D, KEEP_A2>(i, A, A2, A3, x);
#pragma unroll
        for (int j = 0; j < D; ++j) T[i * D + j] = x[j];
    }
#pragma unroll 1
    for (int r = 0; r < s; ++r) {  // T <- T T, column-major tiles
        __threadfence_block();
#pragma unroll 1
        for (int i = 0; i < D; ++i) {
#pragma unroll 1
            for (int j = 0; j < D; ++j) {
                cd c = czero();
#pragma unroll
                for (int m = 0; m < D; ++m) cmac(c, T[m * D + j], T[i * D + m]);
                R[i * D + j] = c;
            }
        }
        cd *t = T;
        T = R;
        R = t;
    }
    __threadfence_block();
#pragma unroll
    for (int i = 0; i < D; ++i) {
        cd x[D];
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = T[i * D + j];
        if (FENCE) pin<D>(x);
        sink(i, x);
    }
}

// Problem data every lane reads at the same address (term tables, the sector's operators) is
// read through the constant address space: scalar loads into SGPRs from the scalar cache, off
// the vector-memory counter (through a flat pointer the compiler cannot rule out that the
// kernel's own stores alias them and issues per-lane vector loads, a dependent chain of them per
// term -- the round-3 first cut spent 74 % of k_walk_fwd<2>'s wave cycles waiting on it).
template <class T>
using cptr = const __attribute__((address_space(4))) T *;
template <class T>
__device__ __forceinline__ cptr<T> as_constant(const T *p) {
    return (cptr<T>)(p);
}
// field-wise copies out of the constant address space (a reference cannot bind across spaces)
__device__ __forceinline__ cd cload(cptr<cd> p, size_t i) { return cmake(p[i].re, p[i].im); }
__device__ __forceinline__ Term tload(cptr<Term> p, int i) {
    Term t;
    t.op = p[i].op;
    t.var = p[i].var;
    t.index = p[i].index;
    t.func = p[i].func;
    t.a = p[i].a;
    t.b = p[i].b;
    t.sre = p[i].sre;
    t.sim = p[i].sim;
    return t;
}
__device__ __forceinline__ Pert pload(cptr<VSpec> p, int i) {
    Pert q;
    q.var = p[i].pert.var;
    q.index = p[i].pert.index;
    q.delta = p[i].pert.delta;
    return q;
}

// The step's controls x[:, k] (np <= 2) and x_add (na <= 2) in registers:
// the next step's controls are loaded one step ahead, so the build never waits on memory.
struct WalkX {  // named registers (an array picked by index would be demoted to scratch)
    double k0, k1;  // x[:, k]  (np <= kWalkMaxNpA = 2)
    double a0, a1;  // x_add    (na <= 2)
    __device__ __forceinline__ double xk(int i) const { return i == 0 ? k0 : k1; }
    __device__ __forceinline__ double xa(int i) const { return i == 0 ? a0 : a1; }
};
struct X2 {
    double v0, v1;
};
// Unconditional loads (the second one clamped into the vector): a load under a branch leaves the
// compiler without a static count of the outstanding vector-memory operations, and it then waits
// with vmcnt(0) -- for every store of the step too -- before the prefetched value is used.
// xs: the transposed controls (B.xT) at this lane's evaluation, consecutive values `stride` apart
__device__ __forceinline__ X2 walk_load_x(int n, const double *xs, int stride) {  // n (uniform) <= 2 values
    X2 r;
    const double a = xs[0], b = xs[n > 1 ? stride : 0];
    r.v0 = n > 0 ? a : 0.0;
    r.v1 = n > 1 ? b : 0.0;
    return r;
}
__device__ __forceinline__ void walk_set_xk(WalkX &X, const X2 &r) {
    X.k0 = r.v0;
    X.k1 = r.v1;
}
__device__ __forceinline__ void walk_set_xa(WalkX &X, const X2 &r) {
    X.a0 = r.v0;
    X.a1 = r.v1;
}

// term_coef (grape_kernels.hpp) with the variable read from registers
__device__ __forceinline__ cd walk_coef(const Term &t, int nt1, const WalkX &X, const Pert &pp, TrigCache &tc) {
    double v = 1.0;
    if (t.var == VAR_X) v = X.xk(t.index);
    else if (t.var == VAR_XADD) v = X.xa(t.index);
    else if (t.var == VAR_TSTEP) v = (double)nt1;
    if (t.var == pp.var && t.index == pp.index) v = v + pp.delta;
    const double arg = t.a * v + t.b;  // built with -ffp-contract=off: no fusion, like Julia
    double fr = 1.0, fi = 0.0;
    if (t.func == FN_LINEAR) fr = arg;
    else if (t.func == FN_COS || t.func == FN_SIN || t.func == FN_CIS) {
        tc.at(arg);
        if (t.func == FN_COS) fr = tc.c;
        else if (t.func == FN_SIN) fr = tc.s;
        else {
            fr = tc.c;
            fi = tc.s;
        }
    }
    return cmul(cmake(t.sre, t.sim), cmake(fr, fi));
}

// A_w += g H_w-term for the NS sectors of this lane (compressed; diagonal as the imaginary part
// of the same complex MAC)
template <int D, int NS>
__device__ __forceinline__ void walk_add_term(const DevProblem &P, cptr<cd> ops, int op_index, cd g, SM<D> (&A)[NS]) {
#pragma unroll
    for (int w = 0; w < NS; ++w) {
        const cptr<cd> op = ops + (size_t)w * P.sec_ops + (size_t)op_index * D * D;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const cd o = cload(op, j * D + j);
            A[w].d[j] = fma(g.im, o.re, fma(g.re, o.im, A[w].d[j]));
#pragma unroll
            for (int k = j + 1; k < D; ++k) cmac(A[w].u[uix(D, j, k)], g, cload(op, j * D + k));
        }
    }
}

// A_w = -i dt H_w(x_k perturbed by pp) for the NS sectors w of this lane, compressed: the
// builder of ItemBuilder with each sector's row-major operators, term by term in order (the same
// cmac operand roles).  The term coefficients (the trig of the controls) are computed once for all
// NS sectors.  err >= 0 adds errval Herror_err (perturbed by pp too) after H0's terms, as
// ItemBuilder<D, true> does (UnitaryCalculations.jl:67-68, 71-72, 77-78).
template <int D, int NS>
__device__ __forceinline__ void walk_build(const DevProblem &P, cptr<cd> ops, const WalkX &X, int nt1, const Pert &pp,
                                           SM<D> (&A)[NS], int err = -1, double errval = 0.0) {
#pragma unroll
    for (int w = 0; w < NS; ++w) {
#pragma unroll
        for (int j = 0; j < D; ++j) A[w].d[j] = 0.0;
#pragma unroll
        for (int t = 0; t < SM<D>::NU; ++t) A[w].u[t] = czero();
    }
    TrigCache tc;
    const cptr<Term> terms = as_constant(P.h0);
#pragma unroll 1
    for (int t = 0; t < P.n_h0; ++t) {
        const Term tm = tload(terms, t);
        const cd c = walk_coef(tm, nt1, X, pp, tc);
        walk_add_term<D, NS>(P, ops, tm.op, cmake(P.dt * c.im, -(P.dt * c.re)), A);  // -i dt c
    }
    if (err >= 0) {  // (wave-uniform)
        const cptr<int> off = as_constant(P.err_off);
        const int o0 = off[err], o1 = off[err + 1];
        const cptr<Term> et = as_constant(P.err);
#pragma unroll 1
        for (int t = o0; t < o1; ++t) {
            const Term tm = tload(et, t);
            const cd c = cscale(errval, walk_coef(tm, nt1, X, pp, tc));
            walk_add_term<D, NS>(P, ops, tm.op, cmake(P.dt * c.im, -(P.dt * c.re)), A);
        }
    }
}

// A lane's D x D matrix: registers, or (D = 4, where registers run out) its private LDS slot,
// row-major, 17 complex apart so that the 16-B accesses of 16 lanes hit 64 distinct banks.
template <int D, bool LDS>
struct MStore;
template <int D>
struct MStore<D, false> {
    cd e[D][D];
    __device__ __forceinline__ cd at(int j, int k) const { return e[j][k]; }
    __device__ __forceinline__ void set(int j, int k, cd v) { e[j][k] = v; }
    __device__ __forceinline__ const MStore &opaque() const { return *this; }
};
using lds_cd = __attribute__((address_space(3))) cd;  // typed LDS pointer: ds_read / ds_write, never flat
template <int D>
struct MStore<D, true> {
    static constexpr int kStride = D * D + 1;
    lds_cd *p;
    __device__ __forceinline__ cd at(int j, int k) const { return cmake(p[j * D + k].re, p[j * D + k].im); }
    __device__ __forceinline__ void set(int j, int k, cd v) {
        p[j * D + k].re = v.re;
        p[j * D + k].im = v.im;
    }
    __device__ __forceinline__ static lds_cd *slot(cd *lds_base) {  // this lane's slot
        return (lds_cd *)(lds_base) + threadIdx.x * kStride;
    }
    // a copy whose address the compiler cannot see through: its loads stay where they are
    // written (no hoisting of 64 VGPRs of LDS reads out of a loop or across an exponential)
    __device__ __forceinline__ MStore opaque() const {
        MStore o{p};
        asm volatile("" : "+v"(o.p));
        return o;
    }
};

// Launch geometry: one lane per (chunk c, evaluation be) -- the evaluation fastest, so that a
// wave's per-step reads of the transposed controls (B.xT) and stores of its F_dx terms (B.sec_part,
// evaluation-fastest) are contiguous -- and group of NS sectors (w0 = NS * blockIdx.y);
// sub-evaluation of sector w: be * nsec + w.  Lanes past the end (ok = false) run the walk on
// clamped indices and store nothing, so that every loop in the walks has a wave-uniform trip
// count (scalar loads of the term tables).
struct WalkLane {
    int w0, be, c, nbe;  // nbe: evaluations of the launch (the stride of B.xT and B.sec_part)
    long slot;           // the lane's scratch slot (NS consecutive pairs of D x D tiles)
    bool ok;
};
// The workgroup's place in the class's launch grid: the hardware block, or (pair kernels, two
// sector classes in one launch for latency-bound calls) a block of one class's part of the grid.
struct VBlock {
    int x, y, gx;  // blockIdx.x, blockIdx.y, gridDim.x of the class's own grid
};
__device__ __forceinline__ VBlock hw_block() { return VBlock{(int)blockIdx.x, (int)blockIdx.y, (int)gridDim.x}; }
template <int NS>
__device__ __forceinline__ WalkLane walk_lane(const DevProblem &P, const DevBatch &B, const VBlock &vb) {
    WalkLane L;
    const int ns = P.nsec > 1 ? P.nsec : 1;
    L.nbe = B.nb / ns;
    const long per = (long)L.nbe * P.nchunks;
    const long g = (long)vb.x * kWalkBlock + threadIdx.x;
    L.w0 = vb.y * NS;
    L.ok = g < per;
    const long gg = L.ok ? g : 0;
    L.c = (int)(gg / L.nbe);
    L.be = (int)(gg - (long)L.c * L.nbe);
    // own scratch slot for every lane, past-the-end ones included (they walk lane 0's inputs)
    const long per_pad = (per + kWalkBlock - 1) / kWalkBlock * kWalkBlock;
    L.slot = (long)vb.y * per_pad + g;
    return L;
}

#ifndef GRAPE_WALK_G4_KEEP_A2_GRAD  // k_walk_grad<4>: keep A'^2 of the eps-variant (0: regenerate its columns)
#define GRAPE_WALK_G4_KEEP_A2_GRAD 1
#endif
#ifndef GRAPE_WALK_IMG4_KEEP_A2  // k_walk_img<4>: keep each variant's A^2 (0: regenerate its columns)
#define GRAPE_WALK_IMG4_KEEP_A2 1
#endif
#ifndef GRAPE_WALK_F4_WAVES  // k_walk_fwd<4>: waves per SIMD
#define GRAPE_WALK_F4_WAVES 2
#endif
#ifndef GRAPE_WALK_F4_FENCE  // k_walk_fwd<4>: fence the exponential's columns
#define GRAPE_WALK_F4_FENCE 1
#endif
#ifndef GRAPE_WALK_G4_KEEP_A2_NOM
#define GRAPE_WALK_G4_KEEP_A2_NOM 1
#endif
#ifndef GRAPE_WALK_G4_WAVES
#define GRAPE_WALK_G4_WAVES 1
#endif
#ifndef GRAPE_WALK_G4S_WAVES  // k_walk_grad<4> with stored propagators
#define GRAPE_WALK_G4S_WAVES 1
#endif
#ifndef GRAPE_WALK_G4_XLDS  // k_walk_grad<4>: 1 = X / Y in the LDS slot and E in registers, 0 = the reverse
#define GRAPE_WALK_G4_XLDS 1
#endif
#ifndef GRAPE_WALK_I21_WAVES  // k_walk_img occupancy: one 2-level sector per lane ...
#define GRAPE_WALK_I21_WAVES 3
#endif
#ifndef GRAPE_WALK_I22_WAVES  // ... or two
#define GRAPE_WALK_I22_WAVES 2
#endif
#ifndef GRAPE_WALK_IMG2_NS1  // the 2-level image walks (error sources) with one sector per lane
#define GRAPE_WALK_IMG2_NS1 0
#endif
#ifndef GRAPE_WALK_FDX_IN_ERR  // F_dx traces in k_walk_err_grad (k_walk_img_sum: W chunk sums only)
#define GRAPE_WALK_FDX_IN_ERR 1
#endif
// ... and those sums in the 2-level image walk itself (LDS accumulators; needs GRAPE_WALK_IMG2_NS1).
// Off: measured slower, C3 580 k -> 569-570 k evals/s (k_walk_img +1.55 ms, k_walk_img_sum -1.0 ms
// per bench step, A/B in one GPU call)
#ifndef GRAPE_WALK_IMG_WSUM
#define GRAPE_WALK_IMG_WSUM 0
#endif
constexpr int kWsumMaxE = 4;
// k_walk_grad with several sectors per lane (the 2-level classes without error sources) writes ONE
// F_dx part per lane row -- its sectors' terms summed in sector order -- so k_sec_reduce reads
// nsec / NS parts for that class (grape_walk_api.hpp walk_parts)
#ifndef GRAPE_WALK_PRESUM
#define GRAPE_WALK_PRESUM 1
#endif
constexpr bool kWalkPresum = GRAPE_WALK_PRESUM;
  // error sources whose W chunk sums the 2-level image walk accumulates
#ifndef GRAPE_WALK_IMG_LDS
#define GRAPE_WALK_IMG_LDS 1
#endif
#ifndef GRAPE_WALK_SHIFT_MIN_D  // the diagonal shift for classes of >= this many levels
#define GRAPE_WALK_SHIFT_MIN_D 3
#endif
#ifndef GRAPE_WALK_F3_WAVES  // k_walk_fwd<3>: waves per SIMD
#define GRAPE_WALK_F3_WAVES 2
#endif
#ifndef GRAPE_WALK_G3_WAVES  // k_walk_grad<3, 1> (recomputed propagators)
#define GRAPE_WALK_G3_WAVES 2
#endif
#ifndef GRAPE_WALK_F22_WAVES  // k_walk_fwd<2, 2>: waves per SIMD
#define GRAPE_WALK_F22_WAVES 3
#endif
#ifndef GRAPE_WALK_G22_WAVES  // k_walk_grad<2, 2>
#define GRAPE_WALK_G22_WAVES 3
#endif
#ifndef GRAPE_WALK_G3S_WAVES  // k_walk_grad<3, 1> with stored propagators
#define GRAPE_WALK_G3S_WAVES 1
#endif
#ifndef GRAPE_WALK_GAUGE2_WAVES
#define GRAPE_WALK_GAUGE2_WAVES 4
#endif
#ifndef GRAPE_WALK_GAUGE3_WAVES
#define GRAPE_WALK_GAUGE3_WAVES 3
#endif
#ifndef GRAPE_WALK_GAUGE4_WAVES
#define GRAPE_WALK_GAUGE4_WAVES 2
#endif
template <int D, int NS>
struct WalkCfg {
    static constexpr bool FENCE = D >= 4;        // per-column scheduling fences (register discipline)
    static constexpr bool E_LDS_FWD = false;     // k_walk_fwd keeps E in registers
    static constexpr bool X_LDS = D >= 4 && NS == 1 && GRAPE_WALK_G4_XLDS;  // k_walk_grad: X / Y in LDS
    static constexpr bool E_LDS_GRAD = D >= 4 && NS == 1 && !GRAPE_WALK_G4_XLDS;  // ... or E in LDS
    // k_walk_grad<4> keeps A'^2 too (round 3: 2.28-2.32 -> 2.20 ms per C2 pass; the stored-propagator
    // kernel has the registers at one wave per SIMD); the image walk regenerates its columns
    static constexpr bool KEEP_A2_GRAD = D < 4 || GRAPE_WALK_G4_KEEP_A2_GRAD;
    static constexpr bool KEEP_A2_IMG = D < 4 || GRAPE_WALK_IMG4_KEEP_A2;
    static constexpr bool KEEP_A2_NOM = D < 4 || GRAPE_WALK_G4_KEEP_A2_NOM;
    static constexpr int WAVES_FWD = D <= 2 ? (NS == 1 ? 4 : NS == 2 ? GRAPE_WALK_F22_WAVES : 3)
                                   : D == 3 ? GRAPE_WALK_F3_WAVES : GRAPE_WALK_F4_WAVES;
    static constexpr bool FENCE_FWD = D >= 4 && GRAPE_WALK_F4_FENCE;
    static constexpr int WAVES_GRAD = D <= 2 ? (NS == 1 ? 4 : NS == 2 ? GRAPE_WALK_G22_WAVES : 2)
                                    : D == 3 ? (NS == 1 ? GRAPE_WALK_G3_WAVES : 1) : GRAPE_WALK_G4_WAVES;
    static constexpr int WAVES_GRAD_STORED = D <= 2 ? (NS == 1 ? 3 : 2) : D == 3 ? GRAPE_WALK_G3S_WAVES : GRAPE_WALK_G4S_WAVES;
    static constexpr int WAVES_IMG = D <= 2 ? (NS == 1 ? GRAPE_WALK_I21_WAVES : GRAPE_WALK_I22_WAVES) : 1;  // k_walk_img
    static constexpr bool IMG_LDS = D >= 4 && GRAPE_WALK_IMG_LDS;      // k_walk_img: eps2 propagators in LDS
    // k_walk_img sums W_e over the chunk in LDS (kWalkBlock x kWsumMaxE x D^2 entries: 64 KB at D = 2)
    // and k_walk_img_sum is not launched (ne <= kWsumMaxE)
    static constexpr bool IMG_WSUM = D == 2 && NS == 1 && GRAPE_WALK_IMG_WSUM && GRAPE_WALK_FDX_IN_ERR;
    // the diagonal shift + Taylor 9 (sm_regime) for the 4-level class only: it pays where the
    // Taylor-12 columns dominate; the smaller classes (Taylor 6 at C2) measured slower with its
    // bookkeeping (k_walk_fwd<2,2> 0.295 -> 0.34 ms per pass) and keep the unshifted walk bitwise
    static constexpr bool SHIFT = D >= GRAPE_WALK_SHIFT_MIN_D;
    // phase-covariant classes (GAUGE): E~, E and the walk state only -- no exponential per step
    static constexpr int WAVES_GAUGE = D <= 2 ? (NS >= 3 ? 2 : GRAPE_WALK_GAUGE2_WAVES)
                                              : D == 3 ? GRAPE_WALK_GAUGE3_WAVES : GRAPE_WALK_GAUGE4_WAVES;
};

// The chunk's phase: sum of the steps' diagonal shifts (sm_regime), TwoSum-compensated; the chunk
// total is e^{i phi} Q~ with Q~ the product of the shifted propagators.
struct WalkPhase {
    double hi = 0.0, lo = 0.0;
    __device__ __forceinline__ void add(double m) {  // (adding 0 is exact: steps past N_t)
        const double t = hi + m, bp = t - hi;
        lo += (hi - (t - bp)) + (m - bp);
        hi = t;
    }
};
template <int D>
__device__ __forceinline__ void walk_phase(const WalkPhase &ph, cd (&Q)[D][D]) {
    const double phi = ph.hi + ph.lo;
    if (phi == 0.0) return;  // (no shift: Q~ is the total)
    double sn, cn;
    sincos(phi, &sn, &cn);
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int i = 0; i < D; ++i) Q[j][i] = cmul(cmake(cn, sn), Q[j][i]);
    }
}
// Stored propagators (B.Ew): per (step, sector) the D*D elements of E~ and, as element D*D, the
// shift mu (real part), each element one coalesced row over the launch's lanes.
template <int D>
constexpr int kEwStride = D * D + 1;

// ---------------------------------------------------------------------------
// Phase-covariant classes (P.gauge, round 5): E_k = D_k E~ D_k^dag
// ---------------------------------------------------------------------------
// A control that enters H only as a phase -- the laser phase phi of the Rydberg models
// (RydbergTools.jl:31-130: e^{-i phi} Omega / 2 on every |1> -> |r> coupling) -- obeys
// H(x) = D(a x) H(0) D(a x)^dag, D(t) = diag(e^{i t N_j}) with integer charges N_j (the Rydberg
// excitation number).  The engine checks this per sector at plan creation (find_gauge: every entry
// of every sector block is e^{i a x (N_j - N_k)} times its value at x = 0).  Then
//   E_k = exp(-i dt H(x_k)) = D_k E~ D_k^dag,   E~ = exp(-i dt H(0))    (exactly, for any x_k)
// and the eps-variant of the step is E'_k = D'_k E~ D'_k^dag with D'_k = D_k diag(e^{i phi N_j}),
// phi = a ((x_k + eps) - x_k).  So a lane computes ONE exponential (E~, at its start) instead of
// one per step and variant; per step it forms E_k from E~ and the D phases of its levels, and
//   (E'_k - E_k)_rj = E_rj (rho_r + conj(rho_j) + rho_r conj(rho_j)),   1 + rho_j = e^{i phi N_j},
// with rho computed without cancellation (gauge_rho), so the reference's forward difference
// (UnitaryCalculations.jl:48-56) is formed from the exact perturbed propagator: same quantity, less
// rounding noise than two separate exponentials.  The charges are wave-uniform (one sector per
// workgroup row: scalar loads), so the per-level powers below are scalar-uniform loops.
template <int D>
struct GaugeN {
    int n[D];
};
template <int D>
constexpr int kGaugePairs = D > 1 ? D * (D - 1) / 2 : 1;  // level pairs j < k of a sector
__host__ __device__ constexpr int gauge_pair(int D, int j, int k) {  // j < k, row-major pair order
    return j * D - j * (j + 1) / 2 + (k - j - 1);
}
template <int D>
__device__ __forceinline__ GaugeN<D> gauge_charges(const DevProblem &P, int w) {
    const cptr<int> g = as_constant(P.gauge_n) + (size_t)w * D;
    GaugeN<D> r;
#pragma unroll
    for (int j = 0; j < D; ++j) r.n[j] = g[j];
    return r;
}
// z^n for a small wave-uniform n >= 0 (n - 1 complex products; exact 1 for n = 0)
__device__ __forceinline__ cd gauge_pow(cd z, int n) {
    cd r = cmake(1.0, 0.0);
    if (n > 0) r = z;
#pragma unroll 1
    for (int m = 1; m < n; ++m) r = cmul(r, z);
    return r;
}
// p = e^{i t}: the per-step phase base of the phase-covariant walks (grape_cis.hpp: Cody-Waite reduction
// and fdlibm kernels, <= 0.67 ulp; the library sincos above |t| = 1e5).  Every gauge kernel (forward,
// gradient, image walk, eval1) takes its phases here, so the walks of one evaluation agree bit for bit.
#ifndef GRAPE_GAUGE_FAST_CIS  // 0: the library sincos (A/B)
#define GRAPE_GAUGE_FAST_CIS 1
#endif
// the constants of grape_cis::cis_fast as opaque SGPR pairs: an empty asm hides the literal from the
// instruction selector, so each Horner step is one v_fma_f64 with a scalar operand (not a v_fmac_f64 on
// a VGPR copy of the literal, two v_mov_b32 per constant and step: the walks are built without
// MachineLICM, so nothing is hoisted).  Not volatile: the asm stays free to move and to merge.
struct CisConst {
    __device__ __forceinline__ double operator()(int i) const {
        double v = grape_cis::kCisCoef[i];
        asm("" : "+s"(v));
        return v;
    }
};
__device__ __forceinline__ cd gauge_cis(double t) {
    double s, c;
#if GRAPE_GAUGE_FAST_CIS
    if (fabs(t) <= grape_cis::kCisFast) grape_cis::cis_fast(t, s, c, CisConst());
    else sincos(t, &s, &c);
#else
    sincos(t, &s, &c);
#endif
    return cmake(c, s);
}
// e^{i phi} - 1 without cancellation: (-2 sin^2(phi / 2), sin phi); Taylor for the FD-sized
// phases (|phi| <= 0.05: truncation below 1e-22 relative), the library otherwise
// (round 5: Horner in t^2 with the reciprocal factorials as constants -- the quotient form spent
// 8 double divisions per step, ~7 % of the merged gradient walk's VALU instructions)
__device__ __forceinline__ double sin_small(double t) {  // sin t, |t| <= 0.05: Taylor to t^9
    const double t2 = t * t;
    return t * fma(t2, fma(t2, fma(t2, fma(t2, 1.0 / 362880.0, -1.0 / 5040.0), 1.0 / 120.0), -1.0 / 6.0), 1.0);
}
__device__ __forceinline__ cd cis_m1(double phi) {
    if (fabs(phi) <= 0.05) {
        const double sh = sin_small(0.5 * phi);
        return cmake(-2.0 * sh * sh, sin_small(phi));
    }
    const double sh = sin(0.5 * phi);
    return cmake(-2.0 * sh * sh, sin(phi));
}
// rho = (1 + q)^n - 1 by rho <- rho + q + q rho (no cancellation), n wave-uniform
__device__ __forceinline__ cd gauge_rho(cd q, int n) {
    cd r = czero();
#pragma unroll 1
    for (int m = 0; m < n; ++m) r = cadd(cadd(r, q), cmul(q, r));
    return r;
}
// the difference weights f_rj = (1 + rho_r)(1 + conj(rho_j)) - 1 = rho_r + conj(rho_j) + rho_r conj(rho_j)
// (no cancellation) of (E' - E)_rj = E_rj f_rj, formed once per pair r < j: f_jr = conj(f_rj) bit for bit
// (the same roundings, conjugated)
template <int D>
__device__ __forceinline__ void gauge_fd_weights(const cd (&rho)[D], cd (&f)[kGaugePairs<D>]) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
#pragma unroll
        for (int j = r + 1; j < D; ++j) {
            const cd rj = cconj(rho[j]);
            f[gauge_pair(D, r, j)] = cadd(cadd(rho[r], rj), cmul(rho[r], rj));
        }
    }
}
// GRAPE_GAUGE_FD_DN (default): the weights straight from the charge differences, f_rj = e^{i phi (N_r - N_j)} - 1 =
// rho(N_r - N_j) (conjugated for N_r < N_j; rho(1) = q exactly), no per-level rho -- the same quantity,
// other roundings (<= a few ulp of f)
#ifndef GRAPE_GAUGE_FD_DN  // (default: C2 43.7-44.0 -> 45.3-45.4 M evals/s, A/B in one GPU call)
#define GRAPE_GAUGE_FD_DN 1
#endif
template <int D>
__device__ __forceinline__ void gauge_fd_weights_dn(cd q, const GaugeN<D> &g, cd (&f)[kGaugePairs<D>]) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
#pragma unroll
        for (int j = r + 1; j < D; ++j) {
            const int dn = g.n[r] - g.n[j], m = dn < 0 ? -dn : dn;
            cd z = q;
#pragma unroll 1
            for (int i = 1; i < m; ++i) z = cadd(cadd(z, q), cmul(q, z));
            f[gauge_pair(D, r, j)] = m == 0 ? czero() : cmake(z.re, dn < 0 ? -z.im : z.im);
        }
    }
}
template <int D>
__device__ __forceinline__ cd gauge_fd_weight(const cd (&f)[kGaugePairs<D>], int r, int j) {
    return r < j ? f[gauge_pair(D, r, j)] : cconj(f[gauge_pair(D, j, r)]);
}
// E~ = exp(-i dt H_w(0)) of the workgroup's NE sectors (the nominal build at x = 0; no diagonal shift,
// so E~ carries its own phase), into every lane's Et.  Every lane of a workgroup walks the same
// sectors (walk_lane: w0 = NS * blockIdx.y), so lane w < NE computes sector w's exponential into LDS
// once for the whole workgroup -- the same code, hence the same bits, in the forward and the
// gradient walk.  (Every lane of the workgroup reaches the barrier: the pair kernels give each
// workgroup to one class.)
template <int D, int NE>
__device__ __forceinline__ void gauge_base(const DevProblem &P, cptr<cd> ops, cd *scr, cd (&Et)[NE][D][D]) {
    __shared__ cd gE[NE * D * D];
    if ((int)threadIdx.x < NE) {
        const int w = threadIdx.x;
        WalkX X0;
        X0.k0 = X0.k1 = X0.a0 = X0.a1 = 0.0;
        Pert none;
        none.var = -1;
        none.index = 0;
        none.delta = 0.0;
        SM<D> A[1];
        walk_build<D, 1>(P, ops + (size_t)w * P.sec_ops, X0, 1, none, A);
        double mu0 = 0.0;
        walk_expm<D, false, true, false>(A[0], scr, mu0, true, [&](int i, const cd (&x)[D]) {
#pragma unroll
            for (int j = 0; j < D; ++j) gE[(w * D + j) * D + i] = x[j];
        });
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NE; ++w) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int i = 0; i < D; ++i) Et[w][j][i] = gE[(w * D + j) * D + i];
        }
    }
}
// gauge_base without the register copy: E~ of the workgroup's NE sectors stays in LDS, row-major
// [w][D][D] (the merged walks read it at every step: 52 VGPRs fewer at DA = 3)
template <int D, int NE>
__device__ __forceinline__ const cd *gauge_base_lds(const DevProblem &P, cptr<cd> ops, cd *scr) {
    __shared__ cd gE[NE * D * D];
    if ((int)threadIdx.x < NE) {
        const int w = threadIdx.x;
        WalkX X0;
        X0.k0 = X0.k1 = X0.a0 = X0.a1 = 0.0;
        Pert none;
        none.var = -1;
        none.index = 0;
        none.delta = 0.0;
        SM<D> A[1];
        walk_build<D, 1>(P, ops + (size_t)w * P.sec_ops, X0, 1, none, A);
        double mu0 = 0.0;
        walk_expm<D, false, true, false>(A[0], scr, mu0, true, [&](int i, const cd (&x)[D]) {
#pragma unroll
            for (int j = 0; j < D; ++j) gE[(w * D + j) * D + i] = x[j];
        });
    }
    __syncthreads();
    return gE;
}
// The pair phases e_jk = e^{i theta (N_j - N_k)}, j < k (gauge_pair order), of one
// sector from p = e^{i theta}: p^|N_j - N_k| (|N_j - N_k| - 1 products, exactly 1 for equal charges),
// conjugated when N_j < N_k.  Round 5: E_jk = E~_jk e_jk and e_kj = conj(e_jk) take one complex
// product per off-diagonal element where d_j E~_jk conj(d_k) from the level phases took two.
template <int D>
__device__ __forceinline__ void gauge_phases(cd p, const GaugeN<D> &g, cd (&e)[kGaugePairs<D>]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int k = j + 1; k < D; ++k) {
            const int dn = g.n[j] - g.n[k];
            const cd z = gauge_pow(p, dn < 0 ? -dn : dn);
            e[gauge_pair(D, j, k)] = cmake(z.re, dn < 0 ? -z.im : z.im);
        }
    }
}
// d_j M_jk conj(d_k) = M_jk e_jk (e_jj = 1: the diagonal unchanged)
template <int D>
__device__ __forceinline__ cd gauge_sandwich(const cd (&e)[kGaugePairs<D>], int j, int k, cd m) {
    return j == k ? m : j < k ? cmul(m, e[gauge_pair(D, j, k)]) : cmul(m, cconj(e[gauge_pair(D, k, j)]));
}
// E_k = D_k E~ D_k^dag; the diagonal is E~'s own
template <int D, class Store>
__device__ __forceinline__ void gauge_prop(const cd (&Et)[D][D], const cd (&e)[kGaugePairs<D>], Store &E) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int k = 0; k < D; ++k) E.set(j, k, gauge_sandwich<D>(e, j, k, Et[j][k]));
    }
}

// Ladder charges N_j = j (DevProblem::gauge_ladder, round 6): the pair phases e_jk = conj(p^{k-j}) and the
// difference weights f_rj = conj(rho(j - r)) (r < j) from compile-time charge differences -- the products
// of gauge_phases / gauge_fd_weights_dn in the same order (same bits), without their scalar loops over
// runtime charge differences
template <int D>
__device__ __forceinline__ void ladder_powers(cd z, cd (&pw)[D]) {  // pw[m] = z^m (gauge_pow's product order)
    pw[0] = cmake(1.0, 0.0);
#pragma unroll
    for (int m = 1; m < D; ++m) pw[m] = m == 1 ? z : cmul(pw[m - 1], z);
}
template <int D>
__device__ __forceinline__ void ladder_rho(cd q, cd (&rh)[D]) {  // rho(m) = (1 + q)^m - 1 (gauge_fd_weights_dn)
    rh[0] = czero();
#pragma unroll
    for (int m = 1; m < D; ++m) rh[m] = m == 1 ? q : cadd(cadd(rh[m - 1], q), cmul(q, rh[m - 1]));
}
template <int D>
__device__ __forceinline__ void gauge_phases_ladder(cd p, cd (&e)[kGaugePairs<D>]) {
    cd pw[D];
    ladder_powers<D>(p, pw);
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int k = j + 1; k < D; ++k) e[gauge_pair(D, j, k)] = cconj(pw[k - j]);
    }
}

// STORE: also hand the propagators to the gradient walk (B.Ew; P.walk_store_e)
// TWIN (P.twin, NS = 2): the lane's two sectors have identical operator blocks (e.g. the Rydberg
// sectors {01, 0r} and {10, r0} at equal Rabi frequencies and detunings): their propagators, chains
// and chunk totals are identical, so one exponential and one chain per step serve both.
// GAUGE: a phase-covariant class (P.gauge): E_k = D_k E~ D_k^dag from the lane's one exponential E~
template <int D, int NS, bool STORE, bool TWIN = false, bool GAUGE = false>
__device__ __forceinline__ void walk_fwd_body(const DevProblem &P, const DevBatch &B, const VBlock vb) {
    using C = WalkCfg<D, NS>;
    static_assert(!TWIN || (NS == 2 && !STORE), "twin sectors: two per lane, recomputed propagators");
    static_assert(!(GAUGE && STORE), "gauge classes form E_k from E~: nothing to store");
    constexpr int NE = TWIN ? 1 : NS;  // distinct propagators / chains per lane
    constexpr int TS = D * D;
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const double *xt = B.xT + (size_t)L.be * (kWalkXRow ? P.nx : 1);  // x[q] of this evaluation at xt[q * xs]
    const int xs = kWalkXRow ? 1 : L.nbe;
    const cptr<cd> ops = as_constant(P.ops) + (size_t)L.w0 * P.sec_ops;
    cd *scr = B.wscr + (size_t)L.slot * NS * 2 * TS;
    Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    const size_t lanes = (size_t)vb.gx * kWalkBlock, lane = (size_t)vb.x * kWalkBlock + threadIdx.x;
    MStore<D, C::E_LDS_FWD> E;
    if constexpr (C::E_LDS_FWD) {
        __shared__ cd lds[kWalkBlock * MStore<D, true>::kStride];
        E.p = MStore<D, true>::slot(lds);
    }
    WalkX X;
    walk_set_xa(X, walk_load_x(P.na, xt + (size_t)P.np * P.Nt * xs, xs));  // x_add
    const int k0 = L.c * P.L;
    X2 xn = walk_load_x(P.np, xt + (size_t)min(k0, P.Nt - 1) * P.np * xs, xs);
    cd Q[NE][D][D];
    WalkPhase ph[NE];
#pragma unroll
    for (int w = 0; w < NE; ++w) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int i = 0; i < D; ++i) Q[w][j][i] = cmake(i == j ? 1.0 : 0.0, 0.0);
        }
    }
    cd Et[GAUGE ? NE : 1][D][D];  // GAUGE: E~ of the lane's sectors
    GaugeN<D> gn[GAUGE ? NE : 1];
    if constexpr (GAUGE) {
        gauge_base<D, NE>(P, ops, scr, Et);
#pragma unroll
        for (int w = 0; w < NE; ++w) gn[w] = gauge_charges<D>(P, L.w0 + w);
    }
    constexpr bool SHIFT = C::SHIFT && !GAUGE;
#pragma unroll 1
    for (int jj = 0; jj < P.L; ++jj) {  // uniform trip count; steps past N_t leave Q alone
        const int k = min(k0 + jj, P.Nt - 1);
        const bool act = k0 + jj < P.Nt;
        walk_set_xk(X, xn);
        xn = walk_load_x(P.np, xt + (size_t)min(k + 1, P.Nt - 1) * P.np * xs, xs);  // next step's controls
        SM<D> A[GAUGE ? 1 : NE];
        cd p1 = czero();
        if constexpr (GAUGE) {
            p1 = gauge_cis(P.gauge_a * X.k0);  // e^{i a x_k}
        } else {
            walk_build<D, NE>(P, ops, X, k + 1, none, A);
        }
#pragma unroll
        for (int w = 0; w < NE; ++w) {
            double mu = 0.0;
            if constexpr (GAUGE) {
                cd dph[kGaugePairs<D>];
                gauge_phases<D>(p1, gn[w], dph);
                gauge_prop<D>(Et[w], dph, E);
            } else {
                walk_expm<D, C::FENCE_FWD, true, C::SHIFT>(A[w], scr + (size_t)w * 2 * TS, mu, true, [&](int i, const cd (&x)[D]) {
#pragma unroll
                    for (int j = 0; j < D; ++j) E.set(j, i, x[j]);
                });
            }
            if constexpr (SHIFT) ph[w].add(act ? mu : 0.0);
            if constexpr (STORE) {  // the gradient walk's copy: lane-minor, one coalesced 1-KB store per element
                cd *ew = B.Ew + ((((size_t)vb.y * P.L + jj) * NS + w) * kEwStride<D>) * lanes + lane;
#pragma unroll
                for (int j = 0; j < D; ++j) {
#pragma unroll
                    for (int i = 0; i < D; ++i) ew[(size_t)(j * D + i) * lanes] = E.at(j, i);
                }
                ew[(size_t)TS * lanes] = cmake(mu, 0.0);
            }
#pragma unroll
            for (int i = 0; i < D; ++i) {  // column i of E_k Q (in place: it reads only column i)
                cd q[D], t[D];
#pragma unroll
                for (int m = 0; m < D; ++m) q[m] = Q[w][m][i];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    cd c = czero();
#pragma unroll
                    for (int m = 0; m < D; ++m) cmac(c, q[m], E.at(j, m));
                    t[j] = c;
                }
#pragma unroll
                for (int j = 0; j < D; ++j)
                    Q[w][j][i] = cmake(act ? t[j].re : Q[w][j][i].re, act ? t[j].im : Q[w][j][i].im);
            }
        }
    }
    if (L.ok) {
        if constexpr (SHIFT) {
#pragma unroll
            for (int w = 0; w < NE; ++w) walk_phase<D>(ph[w], Q[w]);
        }
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            const int we = TWIN ? 0 : w;
            cd *dst = B.Tc + (((size_t)L.be * ns + L.w0 + w) * P.nchunks + L.c) * TS;  // row-major chunk total
#pragma unroll
            for (int j = 0; j < D; ++j) {
#pragma unroll
                for (int i = 0; i < D; ++i) dst[j * D + i] = Q[we][j][i];
            }
        }
    }
}

template <int D, int NS, bool STORE, bool TWIN = false, bool GAUGE = false>
__global__ __launch_bounds__(kWalkBlock, (GAUGE ? WalkCfg<D, NS>::WAVES_GAUGE : WalkCfg<D, NS>::WAVES_FWD))
void k_walk_fwd(DevProblem P, DevBatch B) {
    walk_fwd_body<D, NS, STORE, TWIN, GAUGE>(P, B, hw_block());
}

// STORED: the nominal propagators come from the forward walk's copy (B.Ew, prefetched one step
// ahead) instead of being recomputed -- one exponential of the three per step saved for 512 B of
// HBM traffic per step and sector.
// NVG: the number of gradient parameters when known at compile time (1: C1 / C2 / C4), else 0
// (a runtime loop) -- a static count of the F_dx stores per step keeps the prefetch waits exact.
// TWIN: one nominal and one eps-variant exponential per step serve both sectors of the lane (their
// X, Y and contractions stay per sector: M differs between them in general)
// GAUGE: a phase-covariant class (P.gauge; NVG == 1): E_k from E~ and the level phases, and the
// eps-variant's difference E' - E = E o f with f_rj = rho_r + conj(rho_j) + rho_r conj(rho_j)
template <int D, int NS, bool STORED, int NVG, bool TWIN = false, bool GAUGE = false>
__device__ __forceinline__ void walk_grad_body(const DevProblem &P, const DevBatch &B, const VBlock vb) {
    using C = WalkCfg<D, NS>;
    static_assert(!TWIN || (NS == 2 && !STORED), "twin sectors: two per lane, recomputed propagators");
    static_assert(!GAUGE || (!STORED && NVG == 1), "gauge classes: recomputed propagators, one control");
    constexpr int NE = TWIN ? 1 : NS;     // distinct propagators per lane
    constexpr int NSH = TWIN ? NS : 1;    // sectors sharing each of them
    constexpr int TS = D * D;
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const double *xt = B.xT + (size_t)L.be * (kWalkXRow ? P.nx : 1);  // x[q] of this evaluation at xt[q * xs]
    const int xs = kWalkXRow ? 1 : L.nbe;
    const cptr<cd> ops = as_constant(P.ops) + (size_t)L.w0 * P.sec_ops;
    cd *scr = B.wscr + (size_t)L.slot * NS * 2 * TS;
    Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    // X_{k-1} = C_{k-1} M C_{k-1}^dag of every sector (M'_c at the chunk start); Y_k in place
    constexpr bool XL = C::X_LDS && !STORED, EL = C::E_LDS_GRAD && !STORED;
    MStore<D, XL> X[NS];
    MStore<D, EL> E[NE];
    if constexpr (XL || EL) {
        static_assert(NS == 1 && !(XL && EL), "one LDS slot per lane");
        __shared__ cd lds[kWalkBlock * MStore<D, true>::kStride];
        if constexpr (XL) X[0].p = MStore<D, true>::slot(lds);
        else E[0].p = MStore<D, true>::slot(lds);
    }
    const size_t lanes = (size_t)vb.gx * kWalkBlock, lane = (size_t)vb.x * kWalkBlock + threadIdx.x;
    auto ew = [&](int jj, int w) { return B.Ew + ((((size_t)vb.y * P.L + jj) * NS + w) * kEwStride<D>) * lanes + lane; };
    cd En[STORED ? NS : 1][D][D];  // the next step's stored propagators (STORED)
    double mun[NS], mu[NE];        // ... and their shifts; this step's shifts
    if constexpr (STORED) {
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            const cd *src = ew(0, w);
#pragma unroll
            for (int j = 0; j < D; ++j) {
#pragma unroll
                for (int i = 0; i < D; ++i) En[w][j][i] = src[(size_t)(j * D + i) * lanes];
            }
            mun[w] = src[(size_t)TS * lanes].re;
        }
    }
    // X = M'_c = Carry_c M_ww Carry_c^dagger from the carry and the head's sector block (k_sec_mc's
    // arithmetic, element by element: the same values, and one launch less per sector class)
#pragma unroll
    for (int w = 0; w < NS; ++w) {
        const size_t bw = (size_t)L.be * ns + L.w0 + w;
        const cd *Cr = B.Carry + (bw * P.nchunks + L.c) * TS, *Mw = B.Msec + bw * TS;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            cd r[D];  // column j of M_ww Carry^dagger
#pragma unroll
            for (int a = 0; a < D; ++a) {
                cd v = czero();
#pragma unroll
                for (int e = 0; e < D; ++e) v = cadd(v, cmul(Mw[a * D + e], cconj(Cr[j * D + e])));
                r[a] = v;
            }
#pragma unroll
            for (int i = 0; i < D; ++i) {
                cd acc = czero();
#pragma unroll
                for (int a = 0; a < D; ++a) acc = cadd(acc, cmul(Cr[i * D + a], r[a]));
                X[w].set(i, j, acc);
            }
        }
    }
    WalkX XV;
    walk_set_xa(XV, walk_load_x(P.na, xt + (size_t)P.np * P.Nt * xs, xs));
    const int k0 = L.c * P.L;
    X2 xn = walk_load_x(P.np, xt + (size_t)min(k0, P.Nt - 1) * P.np * xs, xs);
    const cptr<VSpec> vs = as_constant(P.vs);
    cd Et[GAUGE ? NE : 1][D][D];  // GAUGE: E~ of the lane's sectors (the forward walk's bits)
    GaugeN<D> gn[GAUGE ? NE : 1];
    cd fwp[GAUGE ? NE : 1][kGaugePairs<D>];  // GAUGE: this step's difference weights (gauge_fd_weights)
    if constexpr (GAUGE) {
        gauge_base<D, NE>(P, ops, scr, Et);
#pragma unroll
        for (int w = 0; w < NE; ++w) gn[w] = gauge_charges<D>(P, L.w0 + w);
    }
#pragma unroll 1
    for (int jj = 0; jj < P.L; ++jj) {  // uniform trip count; steps past N_t store nothing
        const int k = min(k0 + jj, P.Nt - 1);
        const bool act = L.ok && k0 + jj < P.Nt;
        walk_set_xk(XV, xn);
        xn = walk_load_x(P.np, xt + (size_t)min(k + 1, P.Nt - 1) * P.np * xs, xs);  // next step's controls
        if constexpr (GAUGE) {
            const double xk = XV.k0, xe = xk + P.eps;  // the reference's perturbed control (Pert delta = eps)
            const cd p1 = gauge_cis(P.gauge_a * xk), q = cis_m1(P.gauge_a * (xe - xk));  // (xe - xk: exact)
#pragma unroll
            for (int w = 0; w < NE; ++w) {
                cd dph[kGaugePairs<D>];
                gauge_phases<D>(p1, gn[w], dph);
                gauge_prop<D>(Et[w], dph, E[w]);
                mu[w] = 0.0;
#if GRAPE_GAUGE_FD_DN
                gauge_fd_weights_dn<D>(q, gn[w], fwp[w]);
#else
                cd rho[D];  // e^{i phi N_j} - 1
#pragma unroll
                for (int j = 0; j < D; ++j) rho[j] = gauge_rho(q, gn[w].n[j]);
                gauge_fd_weights<D>(rho, fwp[w]);
#endif
            }
        } else if constexpr (STORED) {  // this step's propagators; the next step's loads go out now
#pragma unroll
            for (int w = 0; w < NS; ++w) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
#pragma unroll
                    for (int i = 0; i < D; ++i) E[w].set(j, i, En[w][j][i]);
                }
                mu[w] = mun[w];
            }
            const int jn = jj + 1 < P.L ? jj + 1 : jj;
#pragma unroll
            for (int w = 0; w < NS; ++w) {
                const cd *src = ew(jn, w);
#pragma unroll
                for (int j = 0; j < D; ++j) {
#pragma unroll
                    for (int i = 0; i < D; ++i) En[w][j][i] = src[(size_t)(j * D + i) * lanes];
                }
                mun[w] = src[(size_t)TS * lanes].re;
            }
        } else {
            SM<D> A[NE];
            walk_build<D, NE>(P, ops, XV, k + 1, none, A);
#pragma unroll
            for (int w = 0; w < NE; ++w)
                walk_expm<D, C::FENCE, C::KEEP_A2_NOM, C::SHIFT>(A[w], scr + (size_t)w * 2 * TS, mu[w], true, [&](int i, const cd (&x)[D]) {
#pragma unroll
                    for (int j = 0; j < D; ++j) E[w].set(j, i, x[j]);
                });
        }
        // Y = X E^dag, in place row by row (row r of Y reads row r of X only)
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            const int we = TWIN ? 0 : w;
#pragma unroll
            for (int r = 0; r < D; ++r) {
                cd xr[D], y[D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[j] = X[w].at(r, j);
#pragma unroll
                for (int cc = 0; cc < D; ++cc) {
                    cd s = czero();
#pragma unroll
                    for (int j = 0; j < D; ++j) cmac(s, xr[j], cconj(E[we].at(cc, j)));
                    y[cc] = s;
                }
#pragma unroll
                for (int cc = 0; cc < D; ++cc) X[w].set(r, cc, y[cc]);
            }
        }
        if constexpr (GAUGE) {  // F_dx[k] = Re tr(Y (E' - E)) / eps with (E' - E)_rj = E_rj f_rj (f_jj = 0)
            double tot = 0.0;
#pragma unroll
            for (int we = 0; we < NE; ++we) {
                double s[NSH];
#pragma unroll
                for (int t = 0; t < NSH; ++t) s[t] = 0.0;
                const auto &Ej = E[we].opaque();
                const auto &fw = fwp[we];
#pragma unroll
                for (int r = 0; r < D; ++r) {
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        if (r == j) continue;
                        const cd de = cscale(P.inv_eps, cmul(Ej.at(r, j), gauge_fd_weight<D>(fw, r, j)));
#pragma unroll
                        for (int t = 0; t < NSH; ++t) {
                            const cd y = X[we * NSH + t].opaque().at(j, r);
                            s[t] = fma(y.re, de.re, s[t]);
                            s[t] = fma(-y.im, de.im, s[t]);
                        }
                    }
                }
#pragma unroll
                for (int t = 0; t < NSH; ++t) {
                    const int w = we * NSH + t;
                    if constexpr (kWalkPresum && NS > 1) {
                        tot += s[t];
                    } else {
                        double *dst = act ? B.sec_part + ((((size_t)(L.w0 + w) * P.Nt) + k) * P.nvg) * L.nbe + L.be
                                          : reinterpret_cast<double *>(B.sink);
                        *dst = s[t];
                    }
                }
            }
            if constexpr (kWalkPresum && NS > 1) {
                double *dst = act ? B.sec_part + ((((size_t)(L.w0 / NS) * P.Nt) + k) * P.nvg) * L.nbe + L.be
                                  : reinterpret_cast<double *>(B.sink);
                *dst = tot;
            }
        }
        // eps-variants: F_dx[u, k] = Re tr(Y (E' - E)) / eps, column j of E' against row j of Y
#pragma unroll 1
        for (int u = 0; u < (GAUGE ? 0 : NVG > 0 ? NVG : P.nvg); ++u) {
            SM<D> Ap[NE];
            walk_build<D, NE>(P, ops, XV, k + 1, pload(vs, P.off_dx + u), Ap);
            double tot = 0.0;  // (kWalkPresum: the lane's sectors summed, in sector order)
#pragma unroll
            for (int we = 0; we < NE; ++we) {
                double s[NSH];
#pragma unroll
                for (int t = 0; t < NSH; ++t) s[t] = 0.0;
                walk_expm<D, C::FENCE, C::KEEP_A2_GRAD, C::SHIFT>(Ap[we], scr + (size_t)we * 2 * TS, mu[we], false, [&](int j, const cd (&x)[D]) {
                    if constexpr (NSH == 1) {
                        const auto &Yj = X[we].opaque();  // row j of Y and column j of E read here, after
                        const auto &Ej = E[we].opaque();  // column j of E'
#pragma unroll
                        for (int r = 0; r < D; ++r) {
                            const cd de = cscale(P.inv_eps, csub(x[r], Ej.at(r, j)));  // (1/eps) (E' - E)
                            const cd y = Yj.at(j, r);
                            s[0] = fma(y.re, de.re, s[0]);
                            s[0] = fma(-y.im, de.im, s[0]);
                        }
                    } else {  // twins: one difference column, contracted with each sector's row j of Y
                        const auto &Ej = E[we].opaque();
                        cd de[D];
#pragma unroll
                        for (int r = 0; r < D; ++r) de[r] = cscale(P.inv_eps, csub(x[r], Ej.at(r, j)));
#pragma unroll
                        for (int t = 0; t < NSH; ++t) {
                            const auto &Yj = X[we * NSH + t].opaque();
#pragma unroll
                            for (int r = 0; r < D; ++r) {
                                const cd y = Yj.at(j, r);
                                s[t] = fma(y.re, de[r].re, s[t]);
                                s[t] = fma(-y.im, de[r].im, s[t]);
                            }
                        }
                    }
                });
#pragma unroll
                for (int t = 0; t < NSH; ++t) {
                    const int w = we * NSH + t;
                    if constexpr (kWalkPresum && NS > 1) {
                        tot += s[t];
                    } else {
                        // unconditional store (inactive lanes write the sink): exact vmcnt accounting
                        double *dst = act ? B.sec_part + ((((size_t)(L.w0 + w) * P.Nt) + k) * P.nvg + u) * L.nbe + L.be
                                          : reinterpret_cast<double *>(B.sink);
                        *dst = s[t];
                    }
                }
            }
            if constexpr (kWalkPresum && NS > 1) {  // one part per lane row: index w0 / NS
                double *dst = act ? B.sec_part + ((((size_t)(L.w0 / NS) * P.Nt) + k) * P.nvg + u) * L.nbe + L.be
                                  : reinterpret_cast<double *>(B.sink);
                *dst = tot;
            }
        }
        // X <- E Y, in place column by column
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            const int we = TWIN ? 0 : w;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                cd y[D], t[D];
#pragma unroll
                for (int m = 0; m < D; ++m) y[m] = X[w].at(m, i);
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    cd c = czero();
#pragma unroll
                    for (int m = 0; m < D; ++m) cmac(c, E[we].at(j, m), y[m]);
                    t[j] = c;
                }
#pragma unroll
                for (int j = 0; j < D; ++j) X[w].set(j, i, t[j]);
            }
        }
    }
}

template <int D, int NS, bool STORED, int NVG, bool TWIN = false, bool GAUGE = false>
__global__ __launch_bounds__(kWalkBlock, (GAUGE ? WalkCfg<D, NS>::WAVES_GAUGE
                                                : STORED ? WalkCfg<D, NS>::WAVES_GRAD_STORED : WalkCfg<D, NS>::WAVES_GRAD))
void k_walk_grad(DevProblem P, DevBatch B) {
    walk_grad_body<D, NS, STORED, NVG, TWIN, GAUGE>(P, B, hw_block());
}

// Pair kernels (latency-bound calls): two sector classes' walks in ONE launch -- the first
// n0 = gx0 * gy0 workgroups walk class 0 (D0, NS0; STORE0: its stored propagators), the rest class 1
// -- so a single evaluation's classes run side by side instead of one launch after the other
// (graph branches do not run concurrently on this runtime: scripts/probes/graph_branch_probe.hip).
// The registers are the larger class's; at these sizes the grid is a few workgroups.
// GA: both classes phase-covariant (P.gauge; then class 0 stores nothing)
template <int D0, int NS0, bool ST0, int D1, int NS1, bool TW1 = false, bool GA = false>
__global__ __launch_bounds__(kWalkBlock, 1) void k_walk_fwd_pair(DevProblem P0, DevBatch B0, DevProblem P1, DevBatch B1,
                                                                 int gx0, int gy0, int gx1) {
    const int id = blockIdx.x, n0 = gx0 * gy0;
    if (id < n0) walk_fwd_body<D0, NS0, ST0 && !GA, false, GA>(P0, B0, VBlock{id % gx0, id / gx0, gx0});
    else walk_fwd_body<D1, NS1, false, TW1, GA>(P1, B1, VBlock{(id - n0) % gx1, (id - n0) / gx1, gx1});
}
template <int D0, int NS0, bool ST0, int D1, int NS1, bool TW1 = false, bool GA = false>
__global__ __launch_bounds__(kWalkBlock, 1) void k_walk_grad_pair(DevProblem P0, DevBatch B0, DevProblem P1, DevBatch B1,
                                                                  int gx0, int gy0, int gx1) {
    const int id = blockIdx.x, n0 = gx0 * gy0;
    if (id < n0) walk_grad_body<D0, NS0, ST0 && !GA, 1, false, GA>(P0, B0, VBlock{id % gx0, id / gx0, gx0});
    else walk_grad_body<D1, NS1, false, 1, TW1, GA>(P1, B1, VBlock{(id - n0) % gx1, (id - n0) / gx1, gx1});
}

// ---------------------------------------------------------------------------
// Merged phase-covariant walks (round 5): BOTH sector classes of the Rydberg layout in one lane
// ---------------------------------------------------------------------------
// The C2 walks are VALU-issue bound (≈ 84 % of SIMD cycles issue VALU instructions in every one of
// the four walk kernels, profiles/r05/final_c2 instruction mix), and the two classes' lanes of one
// (evaluation, chunk) repeat the same per-step work: the load of x_k, e^{i a x_k}, e^{i phi} - 1,
// the loop.  A merged lane walks class A (one sector of DA levels) and class B (two 2-level
// sectors, twins or not) over the same chunk, sharing that work, and its gradient walk writes ONE
// F_dx part, (0 + part_A) + part_B in the plan's class order -- the value k_sec_reduce would have
// formed from the two parts -- so the reduction reads one part.  Per class the operations are the
// gauge walks' own (walk_fwd_body / walk_grad_body with GAUGE): at equal chunking the results are
// those of the per-class kernels bit for bit.  Both classes take class A's chunking (the engine
// sets class B's L and nchunks to class A's).
#ifndef GRAPE_WALK_MERGED_WAVES  // waves per SIMD of the merged gradient walk (222 VGPRs with E~ in registers)
#define GRAPE_WALK_MERGED_WAVES 2
#endif
// E~ of the merged walks (round 6, GRAPE_WALK_FWD_ET_SMEM / GRAPE_WALK_GRAD_ET_SMEM): from the plan's
// global copy (DevProblem::gauge_Et) through scalar loads -- E~ is launch-uniform, so each entry is an SGPR
// operand of the complex product that forms E_k -- re-issued every step (the pointer is made opaque per
// step, so the loads are not hoisted into 13 complex registers held across the walk).  The forward walk
// then fits in 120 VGPRs (four waves per SIMD: fwd 0.161 -> 0.145 ms per C2 pass); the gradient walk would
// fit in 160 (three waves) but measured slower there (0.308 -> 0.322 ms: the per-step scalar loads sit on
// its critical path), so it keeps E~ from LDS in registers at two waves (A/B in one GPU call,
// profiles/r06/ab_smem).  0: E~ in LDS (gauge_base_lds).
#ifndef GRAPE_WALK_FWD_ET_SMEM
#define GRAPE_WALK_FWD_ET_SMEM 1
#endif
#ifndef GRAPE_WALK_GRAD_ET_SMEM
#define GRAPE_WALK_GRAD_ET_SMEM 0
#endif
template <int D, bool SMEM>
__device__ __forceinline__ void gauge_prop_lds(const cd *Et, const cd (&e)[kGaugePairs<D>],
                                               MStore<D, false> &E) {  // gauge_prop, E~ in LDS or (SMEM) global
    if constexpr (SMEM) {
        cptr<cd> g = as_constant(Et);
        asm volatile("" : "+s"(g));
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int k = 0; k < D; ++k) E.set(j, k, gauge_sandwich<D>(e, j, k, cload(g, j * D + k)));
        }
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int k = 0; k < D; ++k) E.set(j, k, gauge_sandwich<D>(e, j, k, Et[j * D + k]));
        }
    }
}
// E~ = exp(-i dt H_w(0)) of sectors w < nsec of a class into out [nsec][D][D] row-major: gauge_base_lds's
// code (the nominal build at x = 0, the walks' exponential, unshifted), one lane per sector
template <int D>
__global__ __launch_bounds__(64) void k_gauge_base_fill(DevProblem P, cd *scr, cd *out, int nsec) {
    const int w = threadIdx.x;
    if (w >= nsec) return;
    WalkX X0;
    X0.k0 = X0.k1 = X0.a0 = X0.a1 = 0.0;
    Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    SM<D> A[1];
    walk_build<D, 1>(P, as_constant(P.ops) + (size_t)w * P.sec_ops, X0, 1, none, A);
    double mu0 = 0.0;
    walk_expm<D, false, true, false>(A[0], scr + (size_t)w * 2 * D * D, mu0, true, [&](int i, const cd (&x)[D]) {
#pragma unroll
        for (int j = 0; j < D; ++j) out[(w * D + j) * D + i] = x[j];
    });
}
template <int D, int NE, bool LAD>
__device__ __forceinline__ void merged_step_fwd(const cd *Et, const GaugeN<D> (&gn)[NE], cd p1, cd (&Q)[NE][D][D]) {
#pragma unroll
    for (int w = 0; w < NE; ++w) {
        cd dph[kGaugePairs<D>];
        if constexpr (LAD) gauge_phases_ladder<D>(p1, dph);
        else gauge_phases<D>(p1, gn[w], dph);
        MStore<D, false> E;
        gauge_prop_lds<D, GRAPE_WALK_FWD_ET_SMEM>(Et + w * D * D, dph, E);
#pragma unroll
        for (int i = 0; i < D; ++i) {  // column i of E_k Q (the forward walk's order)
            cd q[D], t[D];
#pragma unroll
            for (int m = 0; m < D; ++m) q[m] = Q[w][m][i];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                cd c = czero();
#pragma unroll
                for (int m = 0; m < D; ++m) cmac(c, q[m], E.at(j, m));
                t[j] = c;
            }
#pragma unroll
            for (int j = 0; j < D; ++j) Q[w][j][i] = t[j];
        }
    }
}
#ifndef GRAPE_WALK_FWD_M_UNROLL  // the merged forward walk's main loop unrolled (loop-carried register moves)
#define GRAPE_WALK_FWD_M_UNROLL 2  // (2: no loop-carried register moves, 2 waves/SIMD: fwd 0.183 -> 0.179 ms per C2 pass)
#endif
constexpr int kFwdMUnroll = GRAPE_WALK_FWD_M_UNROLL;
#ifndef GRAPE_WALK_FWD_M_WAVES  // the merged forward walk (120 VGPRs with E~ in SGPRs: four waves fit)
#define GRAPE_WALK_FWD_M_WAVES 4
#endif
template <int DA, bool TWB, bool LAD>
__global__ __launch_bounds__(kWalkBlock, GRAPE_WALK_FWD_M_WAVES) void k_walk_fwd_m(DevProblem PA, DevBatch BA,
                                                                                  DevProblem PB, DevBatch BB) {
    constexpr int NEB = TWB ? 1 : 2;
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<1>(PA, BA, vb);  // (class A: one sector; its chunking is both classes')
    const double *xt = BA.xT + (size_t)L.be * (kWalkXRow ? PA.nx : 1);
    const int xs = kWalkXRow ? 1 : L.nbe;
    const cd *EtA = GRAPE_WALK_FWD_ET_SMEM
                        ? PA.gauge_Et
                        : gauge_base_lds<DA, 1>(PA, as_constant(PA.ops), BA.wscr + (size_t)L.slot * 2 * DA * DA);
    const cd *EtB = GRAPE_WALK_FWD_ET_SMEM
                        ? PB.gauge_Et
                        : gauge_base_lds<2, NEB>(PB, as_constant(PB.ops), BB.wscr + (size_t)L.slot * 2 * 2 * 4);
    GaugeN<DA> gA[1];
    GaugeN<2> gB[NEB];
    gA[0] = gauge_charges<DA>(PA, 0);
#pragma unroll
    for (int w = 0; w < NEB; ++w) gB[w] = gauge_charges<2>(PB, w);
    cd QA[1][DA][DA], QB[NEB][2][2];
#pragma unroll
    for (int j = 0; j < DA; ++j) {
#pragma unroll
        for (int i = 0; i < DA; ++i) QA[0][j][i] = cmake(i == j ? 1.0 : 0.0, 0.0);
    }
#pragma unroll
    for (int w = 0; w < NEB; ++w) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int i = 0; i < 2; ++i) QB[w][j][i] = cmake(i == j ? 1.0 : 0.0, 0.0);
        }
    }
    const int k0 = L.c * PA.L;
    X2 xn = walk_load_x(1, xt + (size_t)min(k0, PA.Nt - 1) * xs, xs);
    auto step = [&](int jj) {
        const int k = min(k0 + jj, PA.Nt - 1);
        const double xk = xn.v0;
        xn = walk_load_x(1, xt + (size_t)min(k + 1, PA.Nt - 1) * xs, xs);  // next step's control
        const cd p1 = gauge_cis(PA.gauge_a * xk);  // e^{i a x_k}, both classes (the engine checks one a)
        merged_step_fwd<DA, 1, LAD>(EtA, gA, p1, QA);
        merged_step_fwd<2, NEB, LAD>(EtB, gB, p1, QB);
    };
    // steps past N_t leave Q alone: only the last chunk has them, so the first n_last steps of every
    // chunk run unpredicated and the rest only in the other chunks' lanes (a branch, not selects)
    const int nlast = PA.Nt - (PA.nchunks - 1) * PA.L;
    // unrolled by hand (two steps per trip, then the odd one): the phases' constants pass through an
    // inline asm (gauge_cis), which LLVM treats as convergent and will not runtime-unroll
    static_assert(kFwdMUnroll == 1 || kFwdMUnroll == 2, "GRAPE_WALK_FWD_M_UNROLL: 1 or 2");
    int j2 = 0;
    if constexpr (kFwdMUnroll == 2) {
#pragma unroll 1
        for (; j2 + 1 < nlast; j2 += 2) {
            step(j2);
            step(j2 + 1);
        }
    }
#pragma unroll 1
    for (; j2 < nlast; ++j2) step(j2);
#pragma unroll 1
    for (int jj = nlast; jj < PA.L; ++jj) {
        if (L.c != PA.nchunks - 1) step(jj);
    }
    if (L.ok) {  // chunk totals lane-minor (k_scan_seq's coalesced reads): [c][element][evaluation]
        const size_t nbe = (size_t)L.nbe;
        cd *da = BA.Tc + (size_t)L.c * DA * DA * nbe + L.be;
#pragma unroll
        for (int j = 0; j < DA; ++j) {
#pragma unroll
            for (int i = 0; i < DA; ++i) da[(size_t)(j * DA + i) * nbe] = QA[0][j][i];
        }
#pragma unroll
        for (int w = 0; w < NEB; ++w) {  // (twins: one chain)
            cd *db = BB.Tc + ((size_t)w * PB.nchunks + L.c) * 4 * nbe + L.be;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int i = 0; i < 2; ++i) db[(size_t)(j * 2 + i) * nbe] = QB[w][j][i];
            }
        }
    }
}
// The merged path's scan: one lane per evaluation walks its chunk totals in order,
// Carry_0 = I, Carry_{c+1} = T_c Carry_c, U = T_{n-1} Carry_{n-1} -- 2 x (n - 1) small products per
// lane where k_scan_pair spends a wave per sub-evaluation on a Hillis-Steele scan, and every read and
// carry write coalesced (lane-minor [c][element][evaluation]); U row-major per sub-evaluation, as
// the sector head reads it.  (The association of the chain differs from k_scan's: rounding only.)
// Round 5: both classes' chains advance in one loop over the chunks (class B has class A's chunk
// count on merged passes), each with its next chunk total in flight while the current product runs,
// in one-wave workgroups (32 768 evaluations: 2 waves on every CU): 0.064 -> 0.057 ms per C2 pass.
// The pass moves ~26 tiles per (evaluation, chunk) through HBM, so the scan runs near the HBM rate;
// three column lanes per evaluation (more waves, same bytes) measured 0.059 ms.
template <int D>
struct SeqChain {
    const cd *T;
    cd *Carry;
    cd P[D][D], tn[D][D];
    __device__ __forceinline__ void init(const cd *T_, cd *Carry_, size_t nbe, size_t be) {
        T = T_ + be;
        Carry = Carry_ + be;
#pragma unroll
        for (int e = 0; e < D * D; ++e) {
            P[e / D][e % D] = cmake(e / D == e % D ? 1.0 : 0.0, 0.0);
            tn[e / D][e % D] = T[(size_t)e * nbe];
        }
    }
    __device__ __forceinline__ void step(int c, int nch, size_t nbe) {
        cd *dc = Carry + (size_t)c * D * D * nbe;
        const cd *tc = T + (size_t)min(c + 1, nch - 1) * D * D * nbe;
        cd t[D][D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int i = 0; i < D; ++i) {
                dc[(size_t)(j * D + i) * nbe] = P[j][i];
                t[j][i] = tn[j][i];
                tn[j][i] = tc[(size_t)(j * D + i) * nbe];
            }
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {  // P <- T_c P, column by column
            cd q[D];
#pragma unroll
            for (int m = 0; m < D; ++m) q[m] = P[m][i];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                cd acc = czero();
#pragma unroll
                for (int m = 0; m < D; ++m) cmac(acc, t[j][m], q[m]);
                P[j][i] = acc;
            }
        }
    }
};
constexpr int kSeqBlock = 64;
template <int DA, bool TWB>
__global__ __launch_bounds__(kSeqBlock) void k_scan_seq(DevProblem PA, DevBatch BA, DevProblem PB, DevBatch BB, int nb) {
    constexpr int NEB = TWB ? 1 : 2;
    const size_t be = (size_t)blockIdx.x * kSeqBlock + threadIdx.x;
    if (be >= (size_t)nb) return;
    const size_t nbe = (size_t)nb;
    const int nch = PA.nchunks;  // (== PB.nchunks: the engine gives class B class A's chunking)
    SeqChain<DA> ca;
    SeqChain<2> cb[NEB];
    ca.init(BA.Tc, BA.Carry, nbe, be);
#pragma unroll
    for (int w = 0; w < NEB; ++w)
        cb[w].init(BB.Tc + (size_t)w * PB.nchunks * 4 * nbe, BB.Carry + (size_t)w * PB.nchunks * 4 * nbe, nbe, be);
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
        ca.step(c, nch, nbe);
#pragma unroll
        for (int w = 0; w < NEB; ++w) cb[w].step(c, nch, nbe);
    }
    cd *ua = BA.Ub + be * DA * DA;
#pragma unroll
    for (int j = 0; j < DA; ++j) {
#pragma unroll
        for (int i = 0; i < DA; ++i) ua[j * DA + i] = ca.P[j][i];
    }
#pragma unroll
    for (int w = 0; w < NEB; ++w) {
#pragma unroll
        for (int ws = 0; ws < (TWB ? 2 : 1); ++ws) {  // (twins: both sectors' U)
            cd *ub = BB.Ub + (be * 2 + w + ws) * 4;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int i = 0; i < 2; ++i) ub[j * 2 + i] = cb[w].P[j][i];
            }
        }
    }
}
// X = Carry_c M_ww Carry_c^dag of sector w (walk_grad_body's arithmetic)
template <int D>
__device__ __forceinline__ void merged_xinit(const cd *Cr, const cd *Mw, cd (&X)[D][D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        cd r[D];
#pragma unroll
        for (int a = 0; a < D; ++a) {
            cd v = czero();
#pragma unroll
            for (int e = 0; e < D; ++e) v = cadd(v, cmul(Mw[a * D + e], cconj(Cr[j * D + e])));
            r[a] = v;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            cd acc = czero();
#pragma unroll
            for (int a = 0; a < D; ++a) acc = cadd(acc, cmul(Cr[i * D + a], r[a]));
            X[i][j] = acc;
        }
    }
}
// one gradient step of NSEC sectors over NE propagators (NSH = NSEC / NE sectors share one):
// Y = X E^dag, the contraction, X <- E Y; returns the sectors' terms summed in sector order
// (kWalkPresum: (0 + s_0) + s_1 ...; one sector: s_0)
#ifndef GRAPE_WALK_LADDER_CONTR  // ladder classes: the contraction grouped by charge difference (below)
#define GRAPE_WALK_LADDER_CONTR 1
#endif
template <int D, int NE, int NSEC, bool LAD>
__device__ __forceinline__ double merged_step_grad(const cd *Et, const GaugeN<D> (&gn)[NE], cd p1, cd q,
                                                   double inv_eps, cd (&X)[NSEC][D][D]) {
    constexpr int NSH = NSEC / NE;
    MStore<D, false> E[NE];
    cd rho[NE][D];
#pragma unroll
    for (int w = 0; w < NE; ++w) {
        cd dph[kGaugePairs<D>];
        if constexpr (LAD) gauge_phases_ladder<D>(p1, dph);
        else gauge_phases<D>(p1, gn[w], dph);
        gauge_prop_lds<D, GRAPE_WALK_GRAD_ET_SMEM>(Et + w * D * D, dph, E[w]);
#if !GRAPE_GAUGE_FD_DN
#pragma unroll
        for (int j = 0; j < D; ++j) rho[w][j] = gauge_rho(q, gn[w].n[j]);
#endif
    }
#pragma unroll
    for (int w = 0; w < NSEC; ++w) {  // Y = X E^dag, row by row
        const int we = w / NSH;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            cd xr[D], y[D];
#pragma unroll
            for (int j = 0; j < D; ++j) xr[j] = X[w][r][j];
#pragma unroll
            for (int cc = 0; cc < D; ++cc) {
                cd s = czero();
#pragma unroll
                for (int j = 0; j < D; ++j) cmac(s, xr[j], cconj(E[we].at(cc, j)));
                y[cc] = s;
            }
#pragma unroll
            for (int cc = 0; cc < D; ++cc) X[w][r][cc] = y[cc];
        }
    }
    double tot = 0.0, one = 0.0;
    if constexpr (LAD && GRAPE_WALK_LADDER_CONTR) {
        // Ladder charges: f_rj = rho(r - j) for r > j and conj(rho(j - r)) for r < j, so with
        // T_m = sum_{r - j = m} Y_jr E_rj + conj(sum_{r - j = -m} Y_jr E_rj) (m = 1 .. D-1)
        //   sum_{r != j} Re(Y_jr E_rj f_rj) = sum_m Re(rho(m) T_m):
        // one complex MAC per off-diagonal entry and one product per charge difference, where the
        // per-entry form spends E_rj f_rj / eps and a real MAC pair on every entry (same quantity,
        // other roundings)
        cd rh[D];
        ladder_rho<D>(q, rh);
#pragma unroll
        for (int we = 0; we < NE; ++we) {
#pragma unroll
            for (int t = 0; t < NSH; ++t) {
                double tre[D], tim[D];
#pragma unroll
                for (int m = 0; m < D; ++m) tre[m] = tim[m] = 0.0;
#pragma unroll
                for (int r = 0; r < D; ++r) {
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        if (r == j) continue;
                        const int m = r > j ? r - j : j - r;
                        const cd y = X[we * NSH + t][j][r], e = E[we].at(r, j);
                        tre[m] = fma(y.re, e.re, tre[m]);
                        tre[m] = fma(-y.im, e.im, tre[m]);
                        if (r > j) {
                            tim[m] = fma(y.re, e.im, tim[m]);
                            tim[m] = fma(y.im, e.re, tim[m]);
                        } else {
                            tim[m] = fma(-y.re, e.im, tim[m]);
                            tim[m] = fma(-y.im, e.re, tim[m]);
                        }
                    }
                }
                double c = 0.0;
#pragma unroll
                for (int m = 1; m < D; ++m) {
                    c = fma(rh[m].re, tre[m], c);
                    c = fma(-rh[m].im, tim[m], c);
                }
                const double sv = c * inv_eps;
                tot += sv;
                one = sv;
            }
        }
    } else {
#pragma unroll
    for (int we = 0; we < NE; ++we) {
        double s[NSH];
#pragma unroll
        for (int t = 0; t < NSH; ++t) s[t] = 0.0;
        cd fw[kGaugePairs<D>];
#if GRAPE_GAUGE_FD_DN
        gauge_fd_weights_dn<D>(q, gn[we], fw);
#else
        gauge_fd_weights<D>(rho[we], fw);
#endif
#pragma unroll
        for (int r = 0; r < D; ++r) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                if (r == j) continue;
                const cd de = cscale(inv_eps, cmul(E[we].at(r, j), gauge_fd_weight<D>(fw, r, j)));
#pragma unroll
                for (int t = 0; t < NSH; ++t) {
                    const cd y = X[we * NSH + t][j][r];
                    s[t] = fma(y.re, de.re, s[t]);
                    s[t] = fma(-y.im, de.im, s[t]);
                }
            }
        }
#pragma unroll
        for (int t = 0; t < NSH; ++t) {
            tot += s[t];
            one = s[t];
        }
    }
    }
#pragma unroll
    for (int w = 0; w < NSEC; ++w) {  // X <- E Y, column by column
        const int we = w / NSH;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            cd y[D], t[D];
#pragma unroll
            for (int m = 0; m < D; ++m) y[m] = X[w][m][i];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                cd c = czero();
#pragma unroll
                for (int m = 0; m < D; ++m) cmac(c, E[we].at(j, m), y[m]);
                t[j] = c;
            }
#pragma unroll
            for (int j = 0; j < D; ++j) X[w][j][i] = t[j];
        }
    }
    return (kWalkPresum && NSEC > 1) ? tot : one;
}
#ifndef GRAPE_WALK_TWIN_SUM  // merged gradient walk, twin class B: one summed state for both sectors
#define GRAPE_WALK_TWIN_SUM 1
#endif
#ifndef GRAPE_WALK_MERGED_FDX  // the merged gradient walk writes F_dx itself (1) or a part for k_sec_reduce (0)
#define GRAPE_WALK_MERGED_FDX 1
#endif
constexpr int kFdxTile = 16;  // steps per F_dx tile flush
template <int DA, bool TWB, bool LAD>
__global__ __launch_bounds__(kWalkBlock, GRAPE_WALK_MERGED_WAVES) void k_walk_grad_m(DevProblem PA, DevBatch BA,
                                                                                   DevProblem PB, DevBatch BB, int a_first) {
    constexpr int NEB = TWB ? 1 : 2;
    __shared__ double ftile[kWalkBlock][kFdxTile + 1];  // (GRAPE_WALK_MERGED_FDX; +1: conflict-free rows)
    __shared__ int2 frow[kWalkBlock];                   // each row's evaluation and first step
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<1>(PA, BA, vb);
    const double *xt = BA.xT + (size_t)L.be * (kWalkXRow ? PA.nx : 1);
    const int xs = kWalkXRow ? 1 : L.nbe;
    if constexpr (GRAPE_WALK_MERGED_FDX) frow[threadIdx.x] = make_int2(L.ok ? L.be : -1, L.c * PA.L);
    // Twin class B (one propagator for both sectors): X_w <- E X_w E^dag is linear and the lane sums
    // the sectors' terms, so ONE state X = Carry (M_00 + M_11) Carry^dag carries both (GRAPE_WALK_TWIN_SUM:
    // half of class B's products; the sectors' sum formed once instead of per step -- rounding only)
    constexpr int NXB = (TWB && GRAPE_WALK_TWIN_SUM) ? 1 : 2;
    cd XA[1][DA][DA], XB[NXB][2][2];
    {  // carries lane-minor (k_scan_seq), the head's M blocks row-major per sub-evaluation
        const size_t nbe = (size_t)L.nbe, be = (size_t)L.be;
        cd Cr[DA * DA];
        const cd *ca = BA.Carry + (size_t)L.c * DA * DA * nbe + be;
#pragma unroll
        for (int e = 0; e < DA * DA; ++e) Cr[e] = ca[(size_t)e * nbe];
        merged_xinit<DA>(Cr, BA.Msec + be * DA * DA, XA[0]);
#pragma unroll
        for (int w = 0; w < NXB; ++w) {
            cd Cb[4], Mb[4];
            const cd *cb = BB.Carry + ((size_t)(TWB ? 0 : w) * PB.nchunks + L.c) * 4 * nbe + be;
            const cd *mb = BB.Msec + (be * 2 + w) * 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                Cb[e] = cb[(size_t)e * nbe];
                Mb[e] = NXB == 1 ? cadd(mb[e], mb[4 + e]) : mb[e];
            }
            merged_xinit<2>(Cb, Mb, XB[w]);
        }
    }
    const cd *EtA = GRAPE_WALK_GRAD_ET_SMEM
                        ? PA.gauge_Et
                        : gauge_base_lds<DA, 1>(PA, as_constant(PA.ops), BA.wscr + (size_t)L.slot * 2 * DA * DA);
    const cd *EtB = GRAPE_WALK_GRAD_ET_SMEM
                        ? PB.gauge_Et
                        : gauge_base_lds<2, NEB>(PB, as_constant(PB.ops), BB.wscr + (size_t)L.slot * 2 * 2 * 4);
    GaugeN<DA> gA[1];
    GaugeN<2> gB[NEB];
    gA[0] = gauge_charges<DA>(PA, 0);
#pragma unroll
    for (int w = 0; w < NEB; ++w) gB[w] = gauge_charges<2>(PB, w);
    const int k0 = L.c * PA.L;
    X2 xn = walk_load_x(1, xt + (size_t)min(k0, PA.Nt - 1) * xs, xs);
    auto step = [&](int jj) {  // one step of both classes: the F_dx value, in the plan's class order
        const int k = min(k0 + jj, PA.Nt - 1);
        const double xk = xn.v0, xe = xk + PA.eps;  // the reference's perturbed control
        xn = walk_load_x(1, xt + (size_t)min(k + 1, PA.Nt - 1) * xs, xs);  // next step's control
        const cd p1 = gauge_cis(PA.gauge_a * xk), q = cis_m1(PA.gauge_a * (xe - xk));  // (xe - xk: exact)
        const double sa = merged_step_grad<DA, 1, 1, LAD>(EtA, gA, p1, q, PA.inv_eps, XA);
        const double sb = merged_step_grad<2, NEB, NXB, LAD>(EtB, gB, p1, q, PB.inv_eps, XB);
        double v = 0.0;  // k_sec_reduce's sum of the classes' parts, in the plan's class order
        v += a_first ? sa : sb;
        v += a_first ? sb : sa;
        return v;
    };
    if constexpr (GRAPE_WALK_MERGED_FDX) {
        // F_dx straight to its [evaluation][n_x] row through a workgroup tile of kFdxTile steps: the
        // lanes of a workgroup hold consecutive evaluations, so a flush writes 16 lanes' kFdxTile-long
        // row pieces per instruction (no part array, no k_sec_reduce).  Uniform trip counts: every
        // lane reaches the barriers; steps past N_t are walked and not stored.
#pragma unroll 1
        for (int j0 = 0; j0 < PA.L; j0 += kFdxTile) {
            const int nj = min(kFdxTile, PA.L - j0);
#pragma unroll 1  // (unrolled by 2: the same instructions per step)
            for (int t = 0; t < nj; ++t) ftile[threadIdx.x][t] = step(j0 + t);
            __syncthreads();
            const int j = threadIdx.x % kFdxTile;
#pragma unroll 1
            for (int row = threadIdx.x / kFdxTile; row < kWalkBlock; row += kWalkBlock / kFdxTile) {
                const int br = frow[row].x, kk = frow[row].y + j0 + j;  // (br < 0: past the last lane)
                if (j < nj && br >= 0 && kk < PA.Nt) BA.Fdx[(size_t)br * PA.nx + kk] = ftile[row][j];
            }
            __syncthreads();
        }
    } else {
#pragma unroll 1
        for (int jj = 0; jj < PA.L; ++jj) {
            const int k = min(k0 + jj, PA.Nt - 1);
            const bool act = L.ok && k0 + jj < PA.Nt;
            const double v = step(jj);
            double *dst = act ? BA.sec_part + (size_t)k * L.nbe + L.be : reinterpret_cast<double *>(BA.sink);
            *dst = v;
        }
    }
}

// ---------------------------------------------------------------------------
// Error sources: the image walk (k_walk_img, stage 0) and its F_dx traces (k_img_fdx, stage 1)
// ---------------------------------------------------------------------------
// With error sources the error kernels (grape_errpath.hpp: k_err_scan, k_err_grad) consume, per
// step, the local-frame images Y(dX) = Q_k^dag dX Q_{k-1} of every finite difference dX:
//   Z1_u = Y((E(x_u + eps) - E) / eps),  W_e = Y((E(err_e eps) - E) / eps),
//   Z2_{e,u} = Y((E(x_u + eps2, err_e eps2) + E - E(err_e eps2) - E(x_u + eps2)) / eps2^2)
// (UnitaryCalculations.jl:48-95).  Round 2 stored every variant propagator of the step (k_expm:
// 15 at C3) and Q_k (k_scan), and read them back (k_err_local): 2.95 MB of E per evaluation
// written and re-read.  The image walk forms the images in the lane that walks the chunk:
// per step the nominal E_k, then every variant's exponential column by column, its difference
// column dX e_i and at once column i of Z = E_k^dag dX, then
//   Y = Q_k^dag dX Q_{k-1} = Q_{k-1}^dag Z Q_{k-1}      (Q_k = E_k Q_{k-1}, unitary)
// column by column into its Zl slot, and finally Q <- E_k Q.  Only the images (9 tiles per step
// at C3) and the chunk totals T_c (k_scan's input, as k_walk_fwd) reach HBM.  The eps2
// propagators E(x_u + eps2) and E(err_e eps2) that the mixed stencil needs stay in registers:
// the walk serves any number nvg of gradient parameters per step (controls, and x_add when H0 or
// Herror read it); round 3 served nvg == 1 only.
struct VArg {
    Pert p;
    int err;
    double errval;
};
__device__ __forceinline__ VArg vload(cptr<VSpec> p, int i) {
    VArg a;
    a.p.var = p[i].pert.var;
    a.p.index = p[i].pert.index;
    a.p.delta = p[i].pert.delta;
    a.err = p[i].err;
    a.errval = p[i].errval;
    return a;
}

// The images of the walk path (B.Zl), lane-minor like the stored propagators (B.Ew): element el of
// image slot of sector w (of the lane's NS) at step jj of the lane's chunk, lanes = the image walk's
// launch width (gx * kWalkBlock lanes: one per (chunk, evaluation), evaluation fastest).  A wave's
// store or load of one element is 64 consecutive complex values (1 KB).
template <int D, int NS>
__device__ __forceinline__ size_t img_index(const DevProblem &P, int vy, int jj, int w, int slot, int el, size_t lanes,
                                            size_t lane) {
    return (((((size_t)vy * P.L + jj) * NS + w) * P.nz + slot) * (D * D) + el) * lanes + lane;
}
// the image walk's launch width for nbe evaluations (walk_lane: per = nbe * nchunks lanes, padded)
__device__ __forceinline__ size_t img_lanes(const DevProblem &P, int nbe) {
    return ((size_t)nbe * P.nchunks + kWalkBlock - 1) / kWalkBlock * kWalkBlock;
}

enum { IMG_DIFF = 0, IMG_MIX = 1, IMG_KEEP_D2 = 2, IMG_KEEP_E2 = 3 };
template <int K>
struct ImgKind {
    static constexpr int value = K;
};

template <int D, int NS>
__global__ __launch_bounds__(kWalkBlock, (WalkCfg<D, NS>::WAVES_IMG)) void k_walk_img(DevProblem P, DevBatch B) {
    using C = WalkCfg<D, NS>;
    constexpr int TS = D * D;
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const size_t lanes = (size_t)vb.gx * kWalkBlock, lane = (size_t)vb.x * kWalkBlock + threadIdx.x;
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const double *xt = B.xT + (size_t)L.be * (kWalkXRow ? P.nx : 1);  // x[q] of this evaluation at xt[q * xs]
    const int xs = kWalkXRow ? 1 : L.nbe;
    const cptr<cd> ops = as_constant(P.ops) + (size_t)L.w0 * P.sec_ops;
    const cptr<VSpec> vs = as_constant(P.vs);
    cd *scr = B.wscr + (size_t)L.slot * NS * 2 * TS;
    Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    WalkX X;
    walk_set_xa(X, walk_load_x(P.na, xt + (size_t)P.np * P.Nt * xs, xs));  // x_add
    const int k0 = L.c * P.L;
    X2 xn = walk_load_x(P.np, xt + (size_t)min(k0, P.Nt - 1) * P.np * xs, xs);
    // Q_{k-1} (chunk-local), E_k, and the step's eps2 propagators E(x + eps2), E(err_e eps2) (the
    // latter two in the lane's LDS slots at D = 4, where the registers run out)
    cd Q[NS][D][D], E[NS][D][D];
    WalkPhase ph[NS];
    double mu[NS];  // this step's diagonal shifts (every variant takes the nominal's)
    constexpr bool EL = C::IMG_LDS;
    MStore<D, EL> Ed2[NS], Ee2[NS];
    // W chunk sums in LDS (IMG_WSUM): entry (e, t) of this lane at wacc[(e * TS + t) * kWalkBlock]
    const bool ws = C::IMG_WSUM && P.ne <= kWsumMaxE;
    cd *wacc = nullptr;
    if constexpr (C::IMG_WSUM) {
        __shared__ cd lds_w[kWalkBlock * kWsumMaxE * TS];
        wacc = lds_w + threadIdx.x;
#pragma unroll
        for (int t = 0; t < kWsumMaxE * TS; ++t) wacc[t * kWalkBlock] = czero();
    }
    if constexpr (EL) {
        static_assert(NS == 1, "one pair of LDS slots per lane");
        __shared__ cd lds_d2[kWalkBlock * MStore<D, true>::kStride], lds_e2[kWalkBlock * MStore<D, true>::kStride];
        Ed2[0].p = MStore<D, true>::slot(lds_d2);
        Ee2[0].p = MStore<D, true>::slot(lds_e2);
    }
#pragma unroll
    for (int w = 0; w < NS; ++w) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int i = 0; i < D; ++i) Q[w][j][i] = cmake(i == j ? 1.0 : 0.0, 0.0);
        }
    }
#pragma unroll 1
    for (int jj = 0; jj < P.L; ++jj) {  // uniform trip count; steps past N_t store into the sink
        const int k = min(k0 + jj, P.Nt - 1);
        const bool act = L.ok && k0 + jj < P.Nt;
        walk_set_xk(X, xn);
        xn = walk_load_x(P.np, xt + (size_t)min(k + 1, P.Nt - 1) * P.np * xs, xs);  // next step's controls
        {
            SM<D> A[NS];
            walk_build<D, NS>(P, ops, X, k + 1, none, A);
#pragma unroll
            for (int w = 0; w < NS; ++w) {
                walk_expm<D, C::FENCE, true, C::SHIFT>(A[w], scr + (size_t)w * 2 * TS, mu[w], true, [&](int i, const cd (&x)[D]) {
#pragma unroll
                    for (int j = 0; j < D; ++j) E[w][j][i] = x[j];
                });
                if constexpr (C::SHIFT) ph[w].add(act ? mu[w] : 0.0);
            }
        }
        // one variant: its exponential, and (IMG_DIFF / IMG_MIX) the image of its difference to slot
        auto variant = [&](auto kind, int v, int slot) {
            constexpr int KIND = decltype(kind)::value;
            const VArg va = vload(vs, v);
            SM<D> A[NS];
            walk_build<D, NS>(P, ops, X, k + 1, va.p, A, va.err, va.errval);
#pragma unroll
            for (int w = 0; w < NS; ++w) {
                if constexpr (KIND == IMG_KEEP_D2 || KIND == IMG_KEEP_E2) {
                    walk_expm<D, C::FENCE, C::KEEP_A2_IMG, C::SHIFT>(A[w], scr + (size_t)w * 2 * TS, mu[w], false, [&](int i, const cd (&x)[D]) {
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            if constexpr (KIND == IMG_KEEP_D2) Ed2[w].set(j, i, x[j]);
                            else Ee2[w].set(j, i, x[j]);
                        }
                    });
                } else {
                    cd Z[D][D];  // E_k^dag dX, column by column as the variant's columns come out
                    walk_expm<D, C::FENCE, C::KEEP_A2_IMG, C::SHIFT>(A[w], scr + (size_t)w * 2 * TS, mu[w], false, [&](int i, const cd (&x)[D]) {
                        cd dx[D];
                        const auto &e2 = Ee2[w].opaque();  // (LDS reads issued here, not hoisted)
                        const auto &d2 = Ed2[w].opaque();
#pragma unroll
                        for (int r = 0; r < D; ++r) {
                            if constexpr (KIND == IMG_DIFF) dx[r] = cscale(P.inv_eps, csub(x[r], E[w][r][i]));  // (E' - E) / eps
                            else  // (E(u + eps2, err eps2) + E - E(err eps2) - E(u + eps2)) / eps2^2, left to right
                                dx[r] = cscale(P.inv_eps2sq, csub(csub(cadd(x[r], E[w][r][i]), e2.at(r, i)), d2.at(r, i)));
                        }
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            cd c = czero();
#pragma unroll
                            for (int r = 0; r < D; ++r) cmac(c, cconj(E[w][r][j]), dx[r]);
                            Z[j][i] = c;
                        }
                    });
                    // Y = Q^dag Z Q column by column: t = Z q_c, y = Q^dag t, lane-minor (img_index): each
                    // store one coalesced 1-KB row per wave (steps past N_t fill the padding rows)
                    cd *dst = B.Zl + img_index<D, NS>(P, vb.y, jj, w, slot, 0, lanes, lane);
#pragma unroll
                    for (int cc = 0; cc < D; ++cc) {
                        cd t[D];
#pragma unroll
                        for (int m = 0; m < D; ++m) {
                            cd c = czero();
#pragma unroll
                            for (int n = 0; n < D; ++n) cmac(c, Z[m][n], Q[w][n][cc]);
                            t[m] = c;
                        }
#pragma unroll
                        for (int r = 0; r < D; ++r) {
                            cd c = czero();
#pragma unroll
                            for (int m = 0; m < D; ++m) cmac(c, cconj(Q[w][m][r]), t[m]);
                            dst[(size_t)(r * D + cc) * lanes] = c;
                            if constexpr (C::IMG_WSUM && KIND == IMG_DIFF) {  // W_e: the chunk sum, in step order
                                if (ws && act && slot >= P.nvg) {
                                    cd &a = wacc[((slot - P.nvg) * TS + r * D + cc) * kWalkBlock];
                                    a = cadd(a, c);
                                }
                            }
                        }
                    }
                }
            }
        };
        // the variant table of grape_plan_create, for nvg gradient parameters u (controls, then x_add
        // when H0 / Herror read it).  The mixed stencil of (u, e) needs E(x_u + eps2) and E(err_e eps2)
        // at once: one of each is kept, so E(err_e eps2) is recomputed for every u > 0 (nvg = 1, C3:
        // exactly round 3's sequence, each exponential once)
#pragma unroll 1
        for (int u = 0; u < P.nvg; ++u) variant(ImgKind<IMG_DIFF>{}, P.off_dx + u, u);  // Z1_u
#pragma unroll 1
        for (int u = 0; u < P.nvg; ++u) {
            variant(ImgKind<IMG_KEEP_D2>{}, P.off_dx2 + u, 0);  // E(x_u + eps2)
#pragma unroll 1
            for (int e = 0; e < P.ne; ++e) {
                const int ve = P.off_err + e * P.err_stride;
                if (u == 0) variant(ImgKind<IMG_DIFF>{}, ve, P.nvg + e);                 // W_e
                variant(ImgKind<IMG_KEEP_E2>{}, ve + 1, 0);                              // E(err_e eps2)
                variant(ImgKind<IMG_MIX>{}, ve + 2 + u, P.nvg + P.ne + e * P.nvg + u);  // Z2_{e,u}
            }
        }
#pragma unroll
        for (int w = 0; w < NS; ++w) {
#pragma unroll
            for (int i = 0; i < D; ++i) {  // column i of E_k Q (in place: it reads only column i)
                cd q[D], t[D];
#pragma unroll
                for (int m = 0; m < D; ++m) q[m] = Q[w][m][i];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    cd c = czero();
#pragma unroll
                    for (int m = 0; m < D; ++m) cmac(c, q[m], E[w][j][m]);
                    t[j] = c;
                }
#pragma unroll
                for (int j = 0; j < D; ++j)
                    Q[w][j][i] = cmake(act ? t[j].re : Q[w][j][i].re, act ? t[j].im : Q[w][j][i].im);
            }
        }
    }
    if constexpr (C::IMG_WSUM) {
        if (ws && L.ok) {  // B.Wc [sub-evaluation][ne][nchunks][D][D] (k_walk_img_sum's layout and sums)
            const size_t sub = (size_t)L.be * ns + L.w0;
#pragma unroll 1
            for (int e = 0; e < P.ne; ++e) {
                cd *dst = B.Wc + ((sub * P.ne + e) * P.nchunks + L.c) * TS;
#pragma unroll
                for (int t = 0; t < TS; ++t) dst[t] = wacc[(e * TS + t) * kWalkBlock];
            }
        }
    }
    if (L.ok) {
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            if constexpr (C::SHIFT) walk_phase<D>(ph[w], Q[w]);
            cd *dst = B.Tc + (((size_t)L.be * ns + L.w0 + w) * P.nchunks + L.c) * TS;  // row-major chunk total
#pragma unroll
            for (int j = 0; j < D; ++j) {
#pragma unroll
                for (int i = 0; i < D; ++i) dst[j * D + i] = Q[w][j][i];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The image walk of a phase-covariant class (P.gauge with error sources, nvg = 1; round 5)
// ---------------------------------------------------------------------------
// With H0 and every Herror_e covariant under the same D(a x) (find_gauge: the C3 Rabi and detuning
// errors of the Rydberg models are), every variant propagator of a step is a phase sandwich of an
// x-independent matrix: E_k = D E0 D^dag, E(err_e eps) = D E_e1 D^dag, E(x + eps2, err_e eps2) =
// D'' E_e2 D''^dag ... with E0 = exp(A0), E_e1 = exp(A0 + eps A_e0), E_e2 = exp(A0 + eps2 A_e0) (A at
// x = 0).  So the images' kernels Z = E_k^dag dX (UnitaryCalculations.jl:48-95) are
//   Z1   = D (E0^dag (E0 o f1)) D^dag / eps                           f1 from (x + eps) - x
//   W_e  = D (E0^dag (E_e1 - E0) / eps) D^dag = D K_e D^dag           x-independent K_e
//   Z2_e = D (E0^dag ((E_e2 - E0) o f2)) D^dag / eps2^2                f2 from (x + eps2) - x
// with (M o f)_rj = M_rj (rho_r + conj(rho_j) + rho_r conj(rho_j)) as in the gradient walk: the
// mixed stencil's four-term difference becomes one product without cancellation.  The workgroup
// (all lanes one sector group: blockIdx.y) computes E0, K_e and E_e2 - E0 once into LDS (1 + 2 ne
// exponentials per sector, the first lanes in parallel); per step a lane forms D from its control's
// phase, Z1 and Z2_e with one product each, and every image Y = Q^dag Z Q with two, instead of
// 3 + 3 ne exponentials per step.  Images, chunk totals and their layouts are k_walk_img's.

template <int D, int NS>
__device__ __forceinline__ cd *img_gauge_base(cd *g, int w, int b) {  // matrix b of sector w, row-major
    return g + ((size_t)w * (1 + 2 * kGaugeMaxE) + b) * D * D;
}
template <int D, int NS>
constexpr int img_gauge_waves() { return D >= 4 ? 1 : D == 3 ? 2 : NS == 1 ? 3 : 2; }
template <int D, int NS>
__global__ __launch_bounds__(kWalkBlock, (img_gauge_waves<D, NS>())) void k_walk_img_gauge(DevProblem P, DevBatch B) {
    constexpr int TS = D * D;
    constexpr int NBM = 1 + 2 * kGaugeMaxE;
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const size_t lanes = (size_t)vb.gx * kWalkBlock, lane = (size_t)vb.x * kWalkBlock + threadIdx.x;
    const int ns = P.nsec > 1 ? P.nsec : 1, NE = P.ne;
    const double *xt = B.xT + (size_t)L.be * (kWalkXRow ? P.nx : 1);
    const int xs = kWalkXRow ? 1 : L.nbe;
    __shared__ cd gbase[NS * NBM * TS];
    // --- the workgroup's x-independent bases: lane t < NS (1 + 2 NE) computes matrix (w, b) ---
    {
        const int t = threadIdx.x, nb = 1 + 2 * NE;
        if (t < NS * nb) {
            const int w = t / nb, b = t % nb;
            const int e = b == 0 ? -1 : b <= NE ? b - 1 : b - 1 - NE;
            const double ev = b == 0 ? 0.0 : b <= NE ? P.eps : P.eps2;
            WalkX X0;
            X0.k0 = X0.k1 = X0.a0 = X0.a1 = 0.0;
            Pert none;
            none.var = -1;
            none.index = 0;
            none.delta = 0.0;
            SM<D> A[1];
            walk_build<D, 1>(P, as_constant(P.ops) + (size_t)(L.w0 + w) * P.sec_ops, X0, 1, none, A, e, ev);
            double mu0 = 0.0;
            cd *dst = img_gauge_base<D, NS>(gbase, w, b);
            walk_expm<D, false, true, false>(A[0], B.wscr + (size_t)L.slot * NS * 2 * TS, mu0, true,
                                             [&](int i, const cd (&x)[D]) {
#pragma unroll
                                                 for (int j = 0; j < D; ++j) dst[j * D + i] = x[j];
                                             });
        }
        __syncthreads();
        // K_e = E0^dag (E_e1 - E0) / eps and M_e = E_e2 - E0, in place (lane (w, e) owns both)
        cd K[TS], Mm[TS];
        const bool own = t < NS * NE;
        const int w = own ? t / NE : 0, e = own ? t % NE : 0;
        if (own) {
            const cd *E0 = img_gauge_base<D, NS>(gbase, w, 0), *E1 = img_gauge_base<D, NS>(gbase, w, 1 + e),
                     *E2 = img_gauge_base<D, NS>(gbase, w, 1 + NE + e);
#pragma unroll
            for (int r = 0; r < D; ++r) {
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    cd acc = czero();
#pragma unroll
                    for (int m = 0; m < D; ++m) cmac(acc, cconj(E0[m * D + r]), csub(E1[m * D + c], E0[m * D + c]));
                    K[r * D + c] = cscale(P.inv_eps, acc);
                    Mm[r * D + c] = csub(E2[r * D + c], E0[r * D + c]);
                }
            }
        }
        __syncthreads();
        if (own) {
            cd *K1 = img_gauge_base<D, NS>(gbase, w, 1 + e), *M2 = img_gauge_base<D, NS>(gbase, w, 1 + NE + e);
#pragma unroll
            for (int q = 0; q < TS; ++q) {
                K1[q] = K[q];
                M2[q] = Mm[q];
            }
        }
        __syncthreads();
    }
    GaugeN<D> gn[NS];
#pragma unroll
    for (int w = 0; w < NS; ++w) gn[w] = gauge_charges<D>(P, L.w0 + w);
    const int k0 = L.c * P.L;
    X2 xn = walk_load_x(1, xt + (size_t)min(k0, P.Nt - 1) * xs, xs);
    cd Q[NS][D][D];
#pragma unroll
    for (int w = 0; w < NS; ++w) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
#pragma unroll
            for (int i = 0; i < D; ++i) Q[w][j][i] = cmake(i == j ? 1.0 : 0.0, 0.0);
        }
    }
#pragma unroll 1
    for (int jj = 0; jj < P.L; ++jj) {  // uniform trip count; steps past N_t store into the padding rows
        const int k = min(k0 + jj, P.Nt - 1);
        const bool act = L.ok && k0 + jj < P.Nt;
        const double xk = xn.v0;
        xn = walk_load_x(1, xt + (size_t)min(k + 1, P.Nt - 1) * xs, xs);  // next step's control
        const cd p1 = gauge_cis(P.gauge_a * xk);
        const cd q1 = cis_m1(P.gauge_a * ((xk + P.eps) - xk)), q2 = cis_m1(P.gauge_a * ((xk + P.eps2) - xk));
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            cd d[kGaugePairs<D>], f1[kGaugePairs<D>], f2[kGaugePairs<D>];
            gauge_phases<D>(p1, gn[w], d);
#if GRAPE_GAUGE_FD_DN
            gauge_fd_weights_dn<D>(q1, gn[w], f1);
            gauge_fd_weights_dn<D>(q2, gn[w], f2);
#else
            {
                cd r1[D], r2[D];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    r1[j] = gauge_rho(q1, gn[w].n[j]);
                    r2[j] = gauge_rho(q2, gn[w].n[j]);
                }
                gauge_fd_weights<D>(r1, f1);
                gauge_fd_weights<D>(r2, f2);
            }
#endif
            const cd *E0 = img_gauge_base<D, NS>(gbase, w, 0);
            // image of slot: Y = Q^dag (D Zt D^dag) Q, Zt given row-major (scaled by `sc`)
            auto emit = [&](const cd (&Zt)[D][D], int slot, double sc) {
                cd Z[D][D];
#pragma unroll
                for (int r = 0; r < D; ++r) {
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        Z[r][c] = cscale(sc, gauge_sandwich<D>(d, r, c, Zt[r][c]));
                }
                cd *dst = B.Zl + img_index<D, NS>(P, vb.y, jj, w, slot, 0, lanes, lane);
#pragma unroll
                for (int cc = 0; cc < D; ++cc) {
                    cd tt[D];
#pragma unroll
                    for (int m = 0; m < D; ++m) {
                        cd c = czero();
#pragma unroll
                        for (int n = 0; n < D; ++n) cmac(c, Z[m][n], Q[w][n][cc]);
                        tt[m] = c;
                    }
#pragma unroll
                    for (int r = 0; r < D; ++r) {
                        cd c = czero();
#pragma unroll
                        for (int m = 0; m < D; ++m) cmac(c, cconj(Q[w][m][r]), tt[m]);
                        dst[(size_t)(r * D + cc) * lanes] = c;
                    }
                }
            };
            // E0^dag (M o f) for M = E0 (Z1) or E_e2 - E0 (Z2_e)
            auto kernel_f = [&](const cd *M, const cd (&fw)[kGaugePairs<D>], cd (&Zt)[D][D]) {
                cd Mf[D][D];
#pragma unroll
                for (int r = 0; r < D; ++r) {
#pragma unroll
                    for (int c = 0; c < D; ++c) Mf[r][c] = r == c ? czero() : cmul(M[r * D + c], gauge_fd_weight<D>(fw, r, c));
                }
#pragma unroll
                for (int r = 0; r < D; ++r) {
#pragma unroll
                    for (int c = 0; c < D; ++c) {
                        cd acc = czero();
#pragma unroll
                        for (int m = 0; m < D; ++m) cmac(acc, cconj(E0[m * D + r]), Mf[m][c]);
                        Zt[r][c] = acc;
                    }
                }
            };
            {  // Z1 (slot 0)
                cd Zt[D][D];
                kernel_f(E0, f1, Zt);
                emit(Zt, 0, P.inv_eps);
            }
#pragma unroll 1
            for (int e = 0; e < NE; ++e) {  // W_e (slot 1 + e) and Z2_e (slot 1 + NE + e)
                cd Zt[D][D];
                const cd *Ke = img_gauge_base<D, NS>(gbase, w, 1 + e);
#pragma unroll
                for (int r = 0; r < D; ++r) {
#pragma unroll
                    for (int c = 0; c < D; ++c) Zt[r][c] = Ke[r * D + c];
                }
                emit(Zt, 1 + e, 1.0);
                kernel_f(img_gauge_base<D, NS>(gbase, w, 1 + NE + e), f2, Zt);
                emit(Zt, 1 + NE + e, P.inv_eps2sq);
            }
            // Q <- E_k Q with E_k = D E0 D^dag (column by column, in place)
            cd E[D][D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
#pragma unroll
                for (int m = 0; m < D; ++m) E[j][m] = gauge_sandwich<D>(d, j, m, E0[j * D + m]);
            }
#pragma unroll
            for (int i = 0; i < D; ++i) {
                cd qq[D], t[D];
#pragma unroll
                for (int m = 0; m < D; ++m) qq[m] = Q[w][m][i];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    cd c = czero();
#pragma unroll
                    for (int m = 0; m < D; ++m) cmac(c, qq[m], E[j][m]);
                    t[j] = c;
                }
#pragma unroll
                for (int j = 0; j < D; ++j)
                    Q[w][j][i] = cmake(act ? t[j].re : Q[w][j][i].re, act ? t[j].im : Q[w][j][i].im);
            }
        }
    }
    if (L.ok) {
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            cd *dst = B.Tc + (((size_t)L.be * ns + L.w0 + w) * P.nchunks + L.c) * TS;
#pragma unroll
            for (int j = 0; j < D; ++j) {
#pragma unroll
                for (int i = 0; i < D; ++i) dst[j * D + i] = Q[w][j][i];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The image walk's back end (error sources, walk path): walks over the lane-minor images
// ---------------------------------------------------------------------------
// Stage 1, k_walk_img_sum: one lane per (chunk c, evaluation) as the image walk, its NS sectors:
//   F_dx[u, k] (sector part) = Re tr(M'_c Z1_u)          (FidelityCalculations.jl:56-76)
// written lane-major (B.sec_part, [nsec][Nt][nvg][nbe], as k_walk_grad), and the chunk sums of the
// error images sum_{k in c} W_{e,k} to B.Wc ([sub-evaluation][ne][nchunks][D][D], row-major tiles:
// Phase A of k_err_scan, UnitaryCalculations.jl:112).  One read of Z1 and of every W per step.
// GRAPE_WALK_FDX_IN_ERR (default): the F_dx traces are taken by k_walk_err_grad's e = 0 lanes, which
// read Z1 anyway, so this kernel reads only the W images (C3: 5 -> 4 of the 9 tiles per step), and
// not at all for the 2-level classes whose image walk sums W itself (WalkCfg::IMG_WSUM).
#ifndef GRAPE_WALK_IMGSUM_UNROLL
#define GRAPE_WALK_IMGSUM_UNROLL 1
#endif
template <int D, int NS>
__global__ __launch_bounds__(kWalkBlock, 2) void k_walk_img_sum(DevProblem P, DevBatch B) {
    constexpr int TS = D * D;
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const size_t lanes = (size_t)vb.gx * kWalkBlock, lane = (size_t)vb.x * kWalkBlock + threadIdx.x;
    const int k0 = L.c * P.L;
#pragma unroll
    for (int w = 0; w < NS; ++w) {
        const size_t sub = (size_t)L.be * ns + L.w0 + w;
#if !GRAPE_WALK_FDX_IN_ERR
        cd Mt[TS];  // M'_c, row-major
        const cd *Mc = B.Mc + (sub * P.nchunks + L.c) * TS;
#pragma unroll
        for (int t = 0; t < TS; ++t) Mt[t] = Mc[t];
#pragma unroll 1
        for (int u = 0; u < P.nvg; ++u) {
#pragma unroll 1
            for (int jj = 0; jj < P.L; ++jj) {
                const int k = k0 + jj;
                const cd *Z = B.Zl + img_index<D, NS>(P, vb.y, jj, w, u, 0, lanes, lane);
                double s = 0.0;  // sum_ij Re(Z1[i][j] M'[j][i]) in k_img_fdx's (round 3) order
#pragma unroll
                for (int i = 0; i < D; ++i) {
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const cd z = Z[(size_t)(i * D + j) * lanes], m = Mt[j * D + i];
                        s += z.re * m.re - z.im * m.im;
                    }
                }
                double *dst = (L.ok && k < P.Nt)
                                  ? B.sec_part + ((((size_t)(L.w0 + w) * P.Nt) + k) * P.nvg + u) * L.nbe + L.be
                                  : reinterpret_cast<double *>(B.sink);
                *dst = s;
            }
        }
#endif
#pragma unroll 1
        for (int e = 0; e < P.ne; ++e) {
            cd acc[TS];
#pragma unroll
            for (int t = 0; t < TS; ++t) acc[t] = czero();
            // GRAPE_WALK_IMGSUM_UNROLL steps per iteration, loads unconditional (the step index
            // clamped), so their reads are in flight together; the sums stay in step order
            constexpr int UN = GRAPE_WALK_IMGSUM_UNROLL;
#pragma unroll 1
            for (int j0 = 0; j0 < P.L; j0 += UN) {
                cd v[UN][TS];
#pragma unroll
                for (int du = 0; du < UN; ++du) {
                    const int jj = min(j0 + du, P.L - 1);
                    const cd *Wk = B.Zl + img_index<D, NS>(P, vb.y, jj, w, P.nvg + e, 0, lanes, lane);
#pragma unroll
                    for (int t = 0; t < TS; ++t) v[du][t] = Wk[(size_t)t * lanes];
                }
#pragma unroll
                for (int du = 0; du < UN; ++du) {
                    const bool act = j0 + du < P.L && k0 + j0 + du < P.Nt;  // (uniform within a chunk's lanes)
#pragma unroll
                    for (int t = 0; t < TS; ++t) acc[t] = act ? cadd(acc[t], v[du][t]) : acc[t];
                }
            }
            if (L.ok) {
                cd *dst = B.Wc + ((sub * P.ne + e) * P.nchunks + L.c) * TS;
#pragma unroll
                for (int t = 0; t < TS; ++t) dst[t] = acc[t];
            }
        }
    }
}

// Stage 2, k_walk_err_grad: one lane per (chunk c, evaluation, error e), e fastest (the ne lanes of
// an evaluation share one wave, so its Z1 rows are fetched once), its NS sectors.  The B_k
// recurrence of k_err_grad (grape_errpath.hpp) in the lane's registers:
//   B = T_c M' - M' T_c + M' Ttot at the chunk start, then per step
//   Lambda = B - M' W_k,  F_d2err_dx[u, k] (sector part) = Re tr(Lambda Z1_{k,u}) + Re tr(M' Z2_{k,e,u}),
//   B <- Lambda + W_k M'                                 (UnitaryCalculations.jl:112-139,
//                                                         FidelityCalculations.jl:85-113)
// with M' = M'_{c,e}, T_c, Ttot from k_err_scan / k_sec_mc_err (B.Me), the images lane-minor.  The
// terms go lane-major to B.sec_part_err ([nsec][ne][Nt][nvg][nbe]).
template <int D>
__device__ __forceinline__ void walk_mm(const cd (&A)[D * D], const cd (&Bm)[D * D], cd (&C)[D * D]) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            cd c = czero();
#pragma unroll
            for (int m = 0; m < D; ++m) cmac(c, A[i * D + m], Bm[m * D + j]);
            C[i * D + j] = c;
        }
    }
}
template <int D, int NS>
__global__ __launch_bounds__(kWalkBlock, (D >= 4 ? 1 : 2)) void k_walk_err_grad(DevProblem P, DevBatch B) {
    constexpr int TS = D * D;
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const int nbe = B.nb / ns;
    const long per = (long)nbe * P.nchunks;
    const long gtot = (long)blockIdx.x * kWalkBlock + threadIdx.x;
    const int e = (int)(gtot % P.ne);
    const long g = gtot / P.ne;  // the image walk's lane
    const bool ok = g < per;
    const long gg = ok ? g : 0;
    const int c = (int)(gg / nbe), be = (int)(gg - (long)c * nbe);
    const size_t lanes = img_lanes(P, nbe), lane = (size_t)gg;
    const int vy = blockIdx.y, w0 = vy * NS;
    const int k0 = c * P.L;
#pragma unroll
    for (int w = 0; w < NS; ++w) {
        const size_t sub = (size_t)be * ns + w0 + w;
        const cd *Mo = B.Me + ((sub * P.ne + e) * P.nchunks + c) * 3 * TS;  // M', T_c, Ttot
        cd Mp[TS], Bk[TS], T1[TS], T2[TS];
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            Mp[t] = Mo[t];
            T1[t] = Mo[TS + t];
        }
        walk_mm<D>(T1, Mp, Bk);  // T_c M'
        walk_mm<D>(Mp, T1, T2);  // M' T_c
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            Bk[t] = csub(Bk[t], T2[t]);
            T1[t] = Mo[2 * TS + t];
        }
        walk_mm<D>(Mp, T1, T2);  // M' Ttot
#pragma unroll
        for (int t = 0; t < TS; ++t) Bk[t] = cadd(Bk[t], T2[t]);
        const int w_slot = P.nvg + e, z2_slot = P.nvg + P.ne + e * P.nvg;
#if GRAPE_WALK_FDX_IN_ERR
        cd Mc[TS];  // M'_c (F_dx; every e-lane of an evaluation loads the same rows, the e = 0 lane stores)
        {
            const cd *Mcp = B.Mc + (sub * P.nchunks + c) * TS;
#pragma unroll
            for (int t = 0; t < TS; ++t) Mc[t] = Mcp[t];
        }
#endif
#pragma unroll 1
        for (int jj = 0; jj < P.L; ++jj) {
            const int k = k0 + jj;
            const bool act = ok && k < P.Nt;
            cd Wk[TS];
            const cd *Wp = B.Zl + img_index<D, NS>(P, vy, jj, w, w_slot, 0, lanes, lane);
#pragma unroll
            for (int t = 0; t < TS; ++t) Wk[t] = Wp[(size_t)t * lanes];
#pragma unroll
            for (int t = 0; t < TS; ++t) {  // Lambda_k = B - M' W, in place (no product temporary)
                cd c = czero();
#pragma unroll
                for (int m = 0; m < D; ++m) cmac(c, Mp[(t / D) * D + m], Wk[m * D + t % D]);
                Bk[t] = csub(Bk[t], c);
            }
#pragma unroll 1
            for (int u = 0; u < P.nvg; ++u) {
                const cd *z1 = B.Zl + img_index<D, NS>(P, vy, jj, w, u, 0, lanes, lane);
                const cd *z2 = B.Zl + img_index<D, NS>(P, vy, jj, w, z2_slot + u, 0, lanes, lane);
                double s = 0.0;  // sum_i sum_j Lambda[i][j] Z1[j][i] + M'[i][j] Z2[j][i]
                double sdx = 0.0;  // F_dx: sum_i sum_j M'_c[i][j] Z1[j][i] (from the same Z1 loads)
#pragma unroll
                for (int i = 0; i < D; ++i) {
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const cd a = z1[(size_t)(j * D + i) * lanes], bz = z2[(size_t)(j * D + i) * lanes];
                        s += Bk[i * D + j].re * a.re - Bk[i * D + j].im * a.im;
                        s += Mp[i * D + j].re * bz.re - Mp[i * D + j].im * bz.im;
#if GRAPE_WALK_FDX_IN_ERR
                        sdx += Mc[i * D + j].re * a.re - Mc[i * D + j].im * a.im;
#endif
                    }
                }
#if GRAPE_WALK_FDX_IN_ERR
                if (e == 0) {  // F_dx[u, k] (sector part) = Re tr(M'_c Z1_u)
                    double *dx = act ? B.sec_part + ((((size_t)(w0 + w) * P.Nt) + k) * P.nvg + u) * nbe + be
                                     : reinterpret_cast<double *>(B.sink);
                    *dx = sdx;
                }
#else
                (void)sdx;
#endif
                double *dst = act ? B.sec_part_err +
                                        (((((size_t)(w0 + w) * P.ne + e) * P.Nt + k) * P.nvg + u) * nbe + be)
                                  : reinterpret_cast<double *>(B.sink);
                *dst = s;
            }
#pragma unroll
            for (int t = 0; t < TS; ++t) {  // B_{k+1} = Lambda_k + W_k M', in place
                cd c = czero();
#pragma unroll
                for (int m = 0; m < D; ++m) cmac(c, Wk[(t / D) * D + m], Mp[m * D + t % D]);
                Bk[t] = cadd(Bk[t], c);
            }
        }
    }
}


// ---------------------------------------------------------------------------
// Phase-covariant classes with error sources, without images (round 6, GRAPE_WALK_ERR_LAB)
// ---------------------------------------------------------------------------
// The image walk (k_walk_img_gauge) writes 1 + 2 ne local-frame images Y(Z) = Q_{k-1}^dag Z Q_{k-1} per
// step and sector -- 9 tiles at C3's 4-level class, ~10 GB per pass of 8 192 evaluations -- for
// k_walk_img_sum and k_walk_err_grad to read back.  But every use of an image is a trace against a
// chunk-local matrix A, Re tr(A Y(Z)) = Re tr(Abar Z) with Abar = Q_{k-1} A Q_{k-1}^dag, and the chunk-local
// states of the back end obey recurrences whose lab-frame forms close over E_k and the step's differences
// alone.  So both ends carry transported states and no image is formed or stored:
//
// stage 0, k_walk_wsum_lab -- one lane per (chunk, evaluation, error e):
//     R <- (E R + dW_e) E^dag
//   R = Q (sum_{j<k} W_j) Q^dag and dW_e = (E(err_e eps) - E) / eps = E w_e; at the chunk end R = T_c W_c T_c^dag,
//   the chunk sum of the W images (UnitaryCalculations.jl:111-112) in the lab frame, which k_err_scan maps
//   with Carry_{c+1} = T_c Carry_c; lanes e = ne walk Q <- E Q for the chunk total T_c.
// stage 2, k_walk_err_lab -- one lane per (chunk, evaluation, error e); the lanes of e = ne take F_dx:
//   X = M'_{c,e}, L = B_c = T_c M' - M' T_c + M' Ttot (k_walk_err_grad's chunk start), then per step
//     Y = X E^dag,  L <- L - Y dW  (= Lambda_k),  G = L E^dag,
//     F_d2err_dx[k] (sector part) = Re tr(G dX1) + Re tr(Y dX2_e)
//     L <- E G + dW Y  (B_{k+1} = Lambda_k + W_k M'),  X <- E Y
//   with dX1 = (E' - E) / eps and dX2_e the mixed stencil's numerator over eps2^2 (UnitaryCalculations.jl
//   :48-95): with z = E^dag dX, Re tr(Lambda z1) = Re tr(G dX1), Re tr(X z2) = Re tr(Y dX2), and
//   E w E^dag = dW E^dag gives the L update.  F_dx lanes: X = M'_c, Re tr(Y dX1), X <- E Y
//   (FidelityCalculations.jl:56-76, the gauge gradient walk's step).
//
// Gauge frame.  E_k = D_k E~ D_k^dag (D_k = diag(e^{i a x_k N_j})), dW_e = D_k N_e D_k^dag with
// N_e = (E~_e1 - E~) / eps, dX1 = D_k (E~ o f1) D_k^dag / eps and dX2_e = D_k (M_e o f2) D_k^dag / eps2^2 with
// M_e = E~_e2 - E~ (E~_e1 = exp(A0 + eps A_e0), E~_e2 = exp(A0 + eps2 A_e0), A at x = 0; f1, f2 the
// difference weights of the image walk).  So the states are carried as S~ = D_k^dag S D_k: every product
// then has an x-independent, workgroup-uniform factor (E~ or N_e: LDS broadcasts, no per-lane propagator),
// the traces take E~ o f1 and M_e o f2, and moving to the next step's frame is an element-wise phase,
// S~ <- Om S~ Om^dag with Om = D_{k+1}^dag D_k (pair phases of e^{i a (x_k - x_{k+1})}).  The forward lane
// carries Q^ = D_{k+1}^dag Q (Q^ <- Om E~ Q^) or R~, and the chunk end maps back with D_next.
// Six D x D products per step and error (k_walk_err_grad: two, plus 9 image reads; the image walk: two
// per image), the live state three matrices (two waves per SIMD at D = 4).
#ifndef GRAPE_WALK_WSUM_LAB_WAVES
#define GRAPE_WALK_WSUM_LAB_WAVES 2
#endif
#ifndef GRAPE_WALK_ERR_LAB_WAVES
#define GRAPE_WALK_ERR_LAB_WAVES 2
#endif
#ifndef GRAPE_WALK_ERR_LAB4_WAVES  // k_walk_err_lab<4>: four 4 x 4 complex matrices live (256 VGPRs) at the peak
#define GRAPE_WALK_ERR_LAB4_WAVES 2
#endif
template <int D>
constexpr int err_lab_waves() { return D >= 4 ? GRAPE_WALK_ERR_LAB4_WAVES : GRAPE_WALK_ERR_LAB_WAVES; }
// the base table: lanes t < nsec (1 + 2 ne) compute exp(A0), exp(A0 + eps A_e0), exp(A0 + eps2 A_e0)
// (k_walk_img_gauge's builds and exponential), then N_e and M_e in place
template <int D>
__global__ __launch_bounds__(kLabBaseMaxLanes) void k_gauge_err_base_fill(DevProblem P, cd *scr, cd *out, int nsec) {
    constexpr int TS = D * D;
    const int nb = 1 + 2 * P.ne, t = threadIdx.x;
    if (t < nsec * nb) {
        const int w = t / nb, b = t % nb;
        const int e = b == 0 ? -1 : b <= P.ne ? b - 1 : b - 1 - P.ne;
        const double ev = b == 0 ? 0.0 : b <= P.ne ? P.eps : P.eps2;
        WalkX X0;
        X0.k0 = X0.k1 = X0.a0 = X0.a1 = 0.0;
        Pert none;
        none.var = -1;
        none.index = 0;
        none.delta = 0.0;
        SM<D> A[1];
        walk_build<D, 1>(P, as_constant(P.ops) + (size_t)w * P.sec_ops, X0, 1, none, A, e, ev);
        double mu0 = 0.0;
        cd *dst = out + (size_t)t * TS;
        walk_expm<D, false, true, false>(A[0], scr + (size_t)t * 2 * TS, mu0, true, [&](int i, const cd (&x)[D]) {
#pragma unroll
            for (int j = 0; j < D; ++j) dst[j * D + i] = x[j];
        });
    }
    __syncthreads();
    for (int q = t; q < nsec * P.ne * TS; q += blockDim.x) {
        const int w = q / (P.ne * TS), r = q % (P.ne * TS), e = r / TS, el = r % TS;
        const cd e0 = out[(size_t)w * nb * TS + el];
        cd *n = out + ((size_t)w * nb + 1 + e) * TS + el, *m = out + ((size_t)w * nb + 1 + P.ne + e) * TS + el;
        *n = cscale(P.inv_eps, csub(*n, e0));
        *m = csub(*m, e0);
    }
}
// The base table through scalar loads: every operand is uniform over a workgroup (sector group blockIdx.y,
// error e = blockIdx.z), so each entry is an SGPR operand of the FMAs -- no VGPRs, no LDS instructions.  A
// uniform matrix is consumed one row at a time: row r + 1's loads are issued with row r's FMAs and a
// scheduling barrier closes each row, so at most two rows (32 SGPRs at D = 4) are live.  Without the
// barriers the scheduler interleaves the rows of a product and the loaded rows spill to VGPR lanes
// (~700 v_writelane / v_readlane per step at D = 4: 39 % of the VALU instructions were not FP64); LDS
// copies instead cost 190+ VGPRs of preloaded operands.
#ifndef GRAPE_WALK_LAB_SEG
#define GRAPE_WALK_LAB_SEG 1
#endif
struct LabBase {
    cptr<cd> g;  // the class's table
    int nb, ne, e;
    template <int D>
    __device__ __forceinline__ cptr<cd> mat(int w, int m) const {  // sector w; m: 0 E~, 1 N_e, 2 M_e
        const int b = m == 0 ? 0 : m == 1 ? 1 + e : 1 + ne + e;
        return g + ((size_t)w * nb + b) * (D * D);
    }
};
__device__ __forceinline__ LabBase lab_base(const DevProblem &P, int e) {
    LabBase b;
    b.nb = 1 + 2 * P.ne;
    b.ne = P.ne;
    b.e = e < P.ne ? e : 0;  // (F_dx lanes: E~ only)
    b.g = as_constant(P.gauge_Et);
    return b;
}
// the table pointer made opaque once per step: the row addresses are formed in the step (a few scalar adds)
// instead of being hoisted out of the loop as loop-invariant 64-bit SGPR values
__device__ __forceinline__ LabBase lab_step(LabBase b) {
    asm volatile("" : "+s"(b.g));
    return b;
}
__device__ __forceinline__ void lab_seg() {
#if GRAPE_WALK_LAB_SEG
    __builtin_amdgcn_sched_barrier(0);
#endif
}
// row r of U through an opaque pointer tied to `dep` (an empty asm with a register input): neither the asm nor
// the loads can move above the instruction that produced dep
// the row's results pinned where the row ends (an empty asm that reads and rewrites them): instruction
// selection otherwise sinks a row's FMAs towards their later uses, past the barrier, and the row's SGPRs
// stay live (spilled to VGPR lanes) until then
__device__ __forceinline__ void lab_pin(cd &v) { asm volatile("" : "+v"(v.re), "+v"(v.im)); }
template <int D>
__device__ __forceinline__ void lab_row(cptr<cd> U, int r, double dep, cd (&v)[D]) {
    cptr<cd> p = U;  // (the row offset is the loads' immediate: no per-row address to hoist out of the walk)
    asm volatile("" : "+s"(p) : "v"(dep));
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = cload(p, r * D + j);
}
// Row-wise consumption of a uniform matrix U: d_r = body(r, row r of U) (a result of the row), row r + 1 loaded
// after row r - 1's result exists and consumed after a scheduling barrier: two rows live at most
#ifndef GRAPE_WALK_LAB_PREFETCH  // row r + 1's loads issued with row r's FMAs
#define GRAPE_WALK_LAB_PREFETCH 1
#endif
template <int D, class Body>
__device__ __forceinline__ void lab_rows(cptr<cd> U, double dep0, Body &&body) {
    cd cur[D], nxt[D];
    lab_row<D>(U, 0, dep0, cur);
    double dprev = dep0;
#pragma unroll
    for (int r = 0; r < D; ++r) {
        if (GRAPE_WALK_LAB_PREFETCH && r + 1 < D) lab_row<D>(U, r + 1, dprev, nxt);
        const double d = body(r, cur);
        lab_seg();
        if (r + 1 < D) {
            if (!GRAPE_WALK_LAB_PREFETCH) lab_row<D>(U, r + 1, d, nxt);
#pragma unroll
            for (int j = 0; j < D; ++j) cur[j] = nxt[j];
        }
        dprev = d;
    }
}
// C (+)= A U^dag, U uniform: row c of U gives column c of C
template <int D, bool ACC>
__device__ __forceinline__ void lab_mul_udag(const cd (&A)[D][D], cptr<cd> U, cd (&C)[D][D]) {
    lab_rows<D>(U, A[0][0].re, [&](int c, const cd (&u)[D]) {
#pragma unroll
        for (int m = 0; m < D; ++m) {
            const cd uc = cconj(u[m]);
#pragma unroll
            for (int r = 0; r < D; ++r) {
                if (!ACC && m == 0) C[r][c] = cmulf(A[r][m], uc);
                else cmac(C[r][c], A[r][m], uc);
            }
        }
#pragma unroll
        for (int r = 0; r < D; ++r) lab_pin(C[r][c]);
        return C[D - 1][c].re;
    });
}
// C (+)= U A, U uniform: row r of U gives row r of C
template <int D, bool ACC>
__device__ __forceinline__ void lab_umul(cptr<cd> U, const cd (&A)[D][D], cd (&C)[D][D]) {
    lab_rows<D>(U, A[D - 1][D - 1].re, [&](int r, const cd (&u)[D]) {
#pragma unroll
        for (int m = 0; m < D; ++m) {
#pragma unroll
            for (int c = 0; c < D; ++c) {
                if (!ACC && m == 0) C[r][c] = cmulf(u[m], A[m][c]);
                else cmac(C[r][c], u[m], A[m][c]);
            }
        }
#pragma unroll
        for (int c = 0; c < D; ++c) lab_pin(C[r][c]);
        return C[r][D - 1].re;
    });
}
// C -= A U, U uniform: row m of U updates every entry of C
template <int D>
__device__ __forceinline__ void lab_sub_mul_u(const cd (&A)[D][D], cptr<cd> U, cd (&C)[D][D]) {
    lab_rows<D>(U, A[D - 1][D - 1].re, [&](int m, const cd (&u)[D]) {
#pragma unroll
        for (int c = 0; c < D; ++c) {
#pragma unroll
            for (int r = 0; r < D; ++r) cmac(C[r][c], cmake(-A[r][m].re, -A[r][m].im), u[c]);
        }
#pragma unroll
        for (int c = 0; c < D; ++c) {
#pragma unroll
            for (int r = 0; r < D; ++r) lab_pin(C[r][c]);
        }
        return C[D - 1][D - 1].re;
    });
}
// C += U element-wise, U uniform
template <int D>
__device__ __forceinline__ void lab_add_u(cptr<cd> U, cd (&C)[D][D]) {
    lab_rows<D>(U, C[D - 1][D - 1].re, [&](int r, const cd (&u)[D]) {
#pragma unroll
        for (int c = 0; c < D; ++c) {
            C[r][c] = cadd(C[r][c], u[c]);
            lab_pin(C[r][c]);
        }
        return C[r][D - 1].re;
    });
}
// S <- Om S Om^dag: S_ij e_ij with the pair phases e of Om (e_ji = conj(e_ij), the diagonal unchanged)
template <int D>
__device__ __forceinline__ void lab_rotate(const cd (&e)[kGaugePairs<D>], cd (&S)[D][D]) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (i != j) S[i][j] = cmulf(S[i][j], i < j ? e[gauge_pair(D, i, j)] : cconj(e[gauge_pair(D, j, i)]));
        }
    }
}
// sum_{r != j} Re(Y_jr (U o f)_rj): the trace of Y against a uniform matrix with the difference weights
template <int D>
__device__ __forceinline__ double lab_trace_f(const cd (&Y)[D][D], cptr<cd> U, const cd (&f)[kGaugePairs<D>]) {
    double s = 0.0;
    lab_rows<D>(U, Y[D - 1][D - 1].re, [&](int r, const cd (&u)[D]) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (r == j) continue;
            const cd d = cmulf(u[j], gauge_fd_weight<D>(f, r, j));
            s = fma(Y[j][r].re, d.re, s);
            s = fma(-Y[j][r].im, d.im, s);
        }
        asm volatile("" : "+v"(s));
        return s;
    });
    return s;
}

// stage 0: lanes of blockIdx.z = e < ne carry R~ only and write R at the chunk end in the lab frame,
// R = T_c (sum_k W_k) T_c^dag (k_err_scan's Phase A' then takes Carry_{c+1} = T_c Carry_c in place of Carry_c:
// Carry_{c+1}^dag R Carry_{c+1} = Carry_c^dag (sum W) Carry_c); the lanes of blockIdx.z = ne walk Q^ for T_c
template <int D, int NS>
__global__ __launch_bounds__(kWalkBlock, GRAPE_WALK_WSUM_LAB_WAVES) void k_walk_wsum_lab(DevProblem P, DevBatch B) {
    constexpr int TS = D * D;
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const int ns = P.nsec > 1 ? P.nsec : 1, e = blockIdx.z;
    const bool tc = e == P.ne;  // (workgroup-uniform)
    const double *xt = B.xT + (size_t)L.be * (kWalkXRow ? P.nx : 1);
    const int xs = kWalkXRow ? 1 : L.nbe;
    const LabBase lb = lab_base(P, e);
    GaugeN<D> gn[NS];
#pragma unroll
    for (int w = 0; w < NS; ++w) gn[w] = gauge_charges<D>(P, L.w0 + w);
    const int k0 = L.c * P.L;
    double xk = walk_load_x(1, xt + (size_t)min(k0, P.Nt - 1) * xs, xs).v0;
    // Q^ = D_{k0}^dag (Q = I at the chunk start), R~ = 0
    cd S[NS][D][D];
    {
        const cd pc = cconj(gauge_cis(P.gauge_a * xk));
#pragma unroll
        for (int w = 0; w < NS; ++w) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const cd dj = tc ? gauge_pow(pc, gn[w].n[j]) : czero();
#pragma unroll
                for (int i = 0; i < D; ++i) S[w][j][i] = i == j ? dj : czero();
            }
        }
    }
    double xnext = xk;
    auto step = [&](int jj) {
        const int k = min(k0 + jj, P.Nt - 1);
        xnext = walk_load_x(1, xt + (size_t)min(k + 1, P.Nt - 1) * xs, xs).v0;
        const cd om = gauge_cis(P.gauge_a * xk - P.gauge_a * xnext);  // Om = D_{k+1}^dag D_k
        xk = xnext;
        const LabBase lbs = lab_step(lb);
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            cd T[D][D];
            if (tc) {
                lab_umul<D, false>(lbs.mat<D>(L.w0 + w, 0), S[w], T);  // T = E~ Q^, Q^ <- Om T (rows: om^{N_j})
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const cd dl = gauge_pow(om, gn[w].n[j]);
#pragma unroll
                    for (int i = 0; i < D; ++i) S[w][j][i] = cmulf(dl, T[j][i]);
                }
            } else {
                lab_umul<D, false>(lbs.mat<D>(L.w0 + w, 0), S[w], T);  // T = E~ R~ + N_e
                lab_add_u<D>(lbs.mat<D>(L.w0 + w, 1), T);
                lab_mul_udag<D, false>(T, lbs.mat<D>(L.w0 + w, 0), S[w]);  // R~ = T E~^dag
                cd ep[kGaugePairs<D>];
                gauge_phases<D>(om, gn[w], ep);
                lab_rotate<D>(ep, S[w]);
            }
        }
    };
    // steps past N_t leave the state alone: only the last chunk has them
    const int nlast = P.Nt - (P.nchunks - 1) * P.L;
    int j = 0;
#pragma unroll 1
    for (; j < nlast; ++j) step(j);
#pragma unroll 1
    for (; j < P.L; ++j) {
        if (L.c != P.nchunks - 1) step(j);
    }
    if (!L.ok) return;
    const cd pn = gauge_cis(P.gauge_a * xnext);  // D_next: the frame of the last rotation
#pragma unroll
    for (int w = 0; w < NS; ++w) {
        const size_t sub = (size_t)L.be * ns + L.w0 + w;
        if (tc) {  // T_c = D_next Q^ (k_walk_img_gauge's layout)
            cd *dst = B.Tc + (sub * P.nchunks + L.c) * TS;
#pragma unroll
            for (int r = 0; r < D; ++r) {
                const cd dr = gauge_pow(pn, gn[w].n[r]);
#pragma unroll
                for (int c = 0; c < D; ++c) dst[r * D + c] = cmul(dr, S[w][r][c]);
            }
        } else {  // R = D_next R~ D_next^dag, row-major
            cd ep[kGaugePairs<D>];
            gauge_phases<D>(pn, gn[w], ep);
            lab_rotate<D>(ep, S[w]);
            cd *dw = B.Wc + ((sub * P.ne + e) * P.nchunks + L.c) * TS;
#pragma unroll
            for (int r = 0; r < D; ++r) {
#pragma unroll
                for (int c = 0; c < D; ++c) dw[r * D + c] = S[w][r][c];
            }
        }
    }
}

template <int D, int NS>
__global__ __launch_bounds__(kWalkBlock, err_lab_waves<D>()) void k_walk_err_lab(DevProblem P, DevBatch B) {
    constexpr int TS = D * D;
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<NS>(P, B, vb);
    const int ns = P.nsec > 1 ? P.nsec : 1, e = blockIdx.z;
    const bool fdx = e == P.ne;  // (workgroup-uniform)
    const double *xt = B.xT + (size_t)L.be * (kWalkXRow ? P.nx : 1);
    const int xs = kWalkXRow ? 1 : L.nbe;
    const LabBase lb = lab_base(P, e);
    GaugeN<D> gn[NS];
#pragma unroll
    for (int w = 0; w < NS; ++w) gn[w] = gauge_charges<D>(P, L.w0 + w);
    const int k0 = L.c * P.L;
    double xk = walk_load_x(1, xt + (size_t)min(k0, P.Nt - 1) * xs, xs).v0;
    cd X[NS][D][D], Lm[NS][D][D];
#pragma unroll
    for (int w = 0; w < NS; ++w) {
        const size_t sub = (size_t)L.be * ns + L.w0 + w;
        // M'_c = Carry_c M Carry_c^dag of the head's block, formed here (k_sec_mc / k_sec_mc_err's arithmetic:
        // merged_xinit) instead of by two launches that store it for this kernel to read
        const cd *Cr = B.Carry + (sub * P.nchunks + L.c) * TS;
        if (fdx) {  // F_dx[k] (sector part) = Re tr(M'_c Z1_k): X = M'_c
            merged_xinit<D>(Cr, B.Msec + sub * TS, X[w]);
        } else {  // X = M'_{c,e}, L = T_c M' - M' T_c + M' Ttot (k_walk_err_grad's B)
            const cd *Mo = B.Me + ((sub * P.ne + e) * P.nchunks + L.c) * 3 * TS;  // (M'), T_c, Ttot
            cd Mp[TS], T1[TS], Bk[TS], T2[TS];
            {
                cd Xm[D][D];
                merged_xinit<D>(Cr, B.MsecE + (sub * P.ne + e) * TS, Xm);
#pragma unroll
                for (int t = 0; t < TS; ++t) Mp[t] = Xm[t / D][t % D];
            }
#pragma unroll
            for (int t = 0; t < TS; ++t) T1[t] = Mo[TS + t];
            walk_mm<D>(T1, Mp, Bk);  // T_c M'
            walk_mm<D>(Mp, T1, T2);  // M' T_c
#pragma unroll
            for (int t = 0; t < TS; ++t) {
                Bk[t] = csub(Bk[t], T2[t]);
                T1[t] = Mo[2 * TS + t];
            }
            walk_mm<D>(Mp, T1, T2);  // M' Ttot
#pragma unroll
            for (int t = 0; t < TS; ++t) {
                Lm[w][t / D][t % D] = cadd(Bk[t], T2[t]);
                X[w][t / D][t % D] = Mp[t];
            }
        }
    }
    {  // into the first step's frame: S~ = D_{k0}^dag S D_{k0}
        const cd pc = cconj(gauge_cis(P.gauge_a * xk));
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            cd ep[kGaugePairs<D>];
            gauge_phases<D>(pc, gn[w], ep);
            lab_rotate<D>(ep, X[w]);
            if (!fdx) lab_rotate<D>(ep, Lm[w]);
        }
    }
    if (fdx) {
#pragma unroll 1
        for (int jj = 0; jj < P.L; ++jj) {
            const int k = min(k0 + jj, P.Nt - 1);
            const bool act = L.ok && k0 + jj < P.Nt;
            const double xn = walk_load_x(1, xt + (size_t)min(k + 1, P.Nt - 1) * xs, xs).v0;
            const cd q1 = cis_m1(P.gauge_a * ((xk + P.eps) - xk));
            const cd om = gauge_cis(P.gauge_a * xk - P.gauge_a * xn);
            xk = xn;
            const LabBase lbs = lab_step(lb);
#pragma unroll
            for (int w = 0; w < NS; ++w) {
                cd f1[kGaugePairs<D>], Y[D][D];
                gauge_fd_weights_dn<D>(q1, gn[w], f1);
                lab_mul_udag<D, false>(X[w], lbs.mat<D>(L.w0 + w, 0), Y);  // Y~ = X~ E~^dag
                const double s = lab_trace_f<D>(Y, lbs.mat<D>(L.w0 + w, 0), f1);
                lab_umul<D, false>(lbs.mat<D>(L.w0 + w, 0), Y, X[w]);  // X~ = E~ Y~
                cd ep[kGaugePairs<D>];
                gauge_phases<D>(om, gn[w], ep);
                lab_rotate<D>(ep, X[w]);
                double *dst = act ? B.sec_part + ((((size_t)(L.w0 + w) * P.Nt) + k) * P.nvg) * L.nbe + L.be
                                  : reinterpret_cast<double *>(B.sink);
                *dst = s * P.inv_eps;
            }
        }
        return;
    }
#pragma unroll 1
    for (int jj = 0; jj < P.L; ++jj) {
        const int k = min(k0 + jj, P.Nt - 1);
        const bool act = L.ok && k0 + jj < P.Nt;
        const double xn = walk_load_x(1, xt + (size_t)min(k + 1, P.Nt - 1) * xs, xs).v0;
        const cd q1 = cis_m1(P.gauge_a * ((xk + P.eps) - xk)), q2 = cis_m1(P.gauge_a * ((xk + P.eps2) - xk));
        const cd om = gauge_cis(P.gauge_a * xk - P.gauge_a * xn);
        xk = xn;
        const LabBase lbs = lab_step(lb);
#pragma unroll
        for (int w = 0; w < NS; ++w) {
            cd Y[D][D], G[D][D];
            lab_mul_udag<D, false>(X[w], lbs.mat<D>(L.w0 + w, 0), Y);  // Y~ = X~ E~^dag
            double s2, s1;
            {
                cd f2[kGaugePairs<D>];
                gauge_fd_weights_dn<D>(q2, gn[w], f2);
                s2 = lab_trace_f<D>(Y, lbs.mat<D>(L.w0 + w, 2), f2);  // Re tr(Y~ (M_e o f2))
            }
            lab_sub_mul_u<D>(Y, lbs.mat<D>(L.w0 + w, 1), Lm[w]);        // L~ <- L~ - Y~ N_e (Lambda)
            lab_mul_udag<D, false>(Lm[w], lbs.mat<D>(L.w0 + w, 0), G);  // G~ = L~ E~^dag
            {
                cd f1[kGaugePairs<D>];
                gauge_fd_weights_dn<D>(q1, gn[w], f1);
                s1 = lab_trace_f<D>(G, lbs.mat<D>(L.w0 + w, 0), f1);  // Re tr(G~ (E~ o f1))
            }
            lab_umul<D, false>(lbs.mat<D>(L.w0 + w, 0), G, Lm[w]);  // L~ = E~ G~ + N_e Y~
            lab_umul<D, true>(lbs.mat<D>(L.w0 + w, 1), Y, Lm[w]);
            lab_umul<D, false>(lbs.mat<D>(L.w0 + w, 0), Y, X[w]);  // X~ = E~ Y~
            cd ep[kGaugePairs<D>];
            gauge_phases<D>(om, gn[w], ep);  // into the next step's frame
            lab_rotate<D>(ep, X[w]);
            lab_rotate<D>(ep, Lm[w]);
            double *dst = act ? B.sec_part_err +
                                    (((((size_t)(L.w0 + w) * P.ne + e) * P.Nt + k) * P.nvg) * L.nbe + L.be)
                              : reinterpret_cast<double *>(B.sink);
            *dst = s1 * P.inv_eps + s2 * P.inv_eps2sq;
        }
    }
}


// ---------------------------------------------------------------------------
// The merged gradient walk in the gauge frame (round 6, GRAPE_WALK_GRAD_TILDE)
// ---------------------------------------------------------------------------
// k_walk_grad_m carries X_k = C M C^dag per class and forms E_k = D_k E~ D_k^dag in registers each step.
// Here the state is X~ = D_k^dag X D_k (k_walk_err_lab's frame): per step
//   Y~ = X~ E~^dag,  F_dx part = Re tr(Y~ (E~ o f)) / eps,  X~ <- Om (E~ Y~) Om^dag   (Om = D_{k+1}^dag D_k)
// -- the same quantities (traces are frame-invariant), E~ a workgroup-uniform SGPR operand read row by row
// (lab_rows), so E_k's registers and its formation go and the lane fits three waves per SIMD; the rotation
// costs what E_k's formation did.  Ladder classes only (the merged walks' classes); output as k_walk_grad_m.
// Measured slower and off: 168 VGPRs, three waves per SIMD, no scratch, parity-green (the gauge / walk /
// parity suites on it), but 0.343 against 0.309-0.316 ms per C2 pass (A/B twice in one GPU call): the
// row-wise uniform operands cost the products their cross-row ILP, which the third wave does not win back
#ifndef GRAPE_WALK_GRAD_TILDE
#define GRAPE_WALK_GRAD_TILDE 0
#endif
#ifndef GRAPE_WALK_GRAD_TILDE_WAVES
#define GRAPE_WALK_GRAD_TILDE_WAVES 3
#endif
// sum_{r != j} Re(Y_jr (U o f)_rj) for ladder charges: f_rj = rho(r - j) (conj for r < j), grouped by charge
// difference (merged_step_grad's contraction) with U uniform
template <int D>
__device__ __forceinline__ double lab_trace_ladder(const cd (&Y)[D][D], cptr<cd> U, const cd (&rh)[D]) {
    double tre[D], tim[D];
#pragma unroll
    for (int m = 0; m < D; ++m) tre[m] = tim[m] = 0.0;
    lab_rows<D>(U, Y[D - 1][D - 1].re, [&](int r, const cd (&u)[D]) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (r == j) continue;
            const int m = r > j ? r - j : j - r;
            const cd y = Y[j][r], e = u[j];
            tre[m] = fma(y.re, e.re, tre[m]);
            tre[m] = fma(-y.im, e.im, tre[m]);
            if (r > j) {
                tim[m] = fma(y.re, e.im, tim[m]);
                tim[m] = fma(y.im, e.re, tim[m]);
            } else {
                tim[m] = fma(-y.re, e.im, tim[m]);
                tim[m] = fma(-y.im, e.re, tim[m]);
            }
        }
#pragma unroll
        for (int m = 1; m < D; ++m) asm volatile("" : "+v"(tre[m]), "+v"(tim[m]));
        return tre[D - 1];
    });
    double c = 0.0;
#pragma unroll
    for (int m = 1; m < D; ++m) {
        c = fma(rh[m].re, tre[m], c);
        c = fma(-rh[m].im, tim[m], c);
    }
    return c;
}
template <int D>
__device__ __forceinline__ double tilde_step(cptr<cd> Et, const cd (&om_e)[kGaugePairs<D>], const cd (&rh)[D],
                                             cd (&X)[D][D]) {
    cd Y[D][D];
    lab_mul_udag<D, false>(X, Et, Y);            // Y~ = X~ E~^dag
    const double s = lab_trace_ladder<D>(Y, Et, rh);
    lab_umul<D, false>(Et, Y, X);                // X~ = E~ Y~
    lab_rotate<D>(om_e, X);                      // into the next step's frame
    return s;
}
template <int DA, bool TWB>
__global__ __launch_bounds__(kWalkBlock, GRAPE_WALK_GRAD_TILDE_WAVES) void k_walk_grad_mt(DevProblem PA, DevBatch BA,
                                                                                       DevProblem PB, DevBatch BB, int a_first) {
    constexpr int NXB = (TWB && GRAPE_WALK_TWIN_SUM) ? 1 : 2;
    __shared__ double ftile[kWalkBlock][kFdxTile + 1];
    __shared__ int2 frow[kWalkBlock];
    const VBlock vb = hw_block();
    const WalkLane L = walk_lane<1>(PA, BA, vb);
    const double *xt = BA.xT + (size_t)L.be * (kWalkXRow ? PA.nx : 1);
    const int xs = kWalkXRow ? 1 : L.nbe;
    frow[threadIdx.x] = make_int2(L.ok ? L.be : -1, L.c * PA.L);
    cd XA[DA][DA], XB[NXB][2][2];
    {
        const size_t nbe = (size_t)L.nbe, be = (size_t)L.be;
        cd Cr[DA * DA];
        const cd *ca = BA.Carry + (size_t)L.c * DA * DA * nbe + be;
#pragma unroll
        for (int e = 0; e < DA * DA; ++e) Cr[e] = ca[(size_t)e * nbe];
        merged_xinit<DA>(Cr, BA.Msec + be * DA * DA, XA);
#pragma unroll
        for (int w = 0; w < NXB; ++w) {
            cd Cb[4], Mb[4];
            const cd *cb = BB.Carry + ((size_t)(TWB ? 0 : w) * PB.nchunks + L.c) * 4 * nbe + be;
            const cd *mb = BB.Msec + (be * 2 + w) * 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                Cb[e] = cb[(size_t)e * nbe];
                Mb[e] = NXB == 1 ? cadd(mb[e], mb[4 + e]) : mb[e];
            }
            merged_xinit<2>(Cb, Mb, XB[w]);
        }
    }
    const int k0 = L.c * PA.L;
    double xk = walk_load_x(1, xt + (size_t)min(k0, PA.Nt - 1) * xs, xs).v0;
    {  // into the first step's frame: X~ = D_{k0}^dag X D_{k0}
        const cd pc = cconj(gauge_cis(PA.gauge_a * xk));
        cd ea[kGaugePairs<DA>], eb[kGaugePairs<2>];
        gauge_phases_ladder<DA>(pc, ea);
        gauge_phases_ladder<2>(pc, eb);
        lab_rotate<DA>(ea, XA);
#pragma unroll
        for (int w = 0; w < NXB; ++w) lab_rotate<2>(eb, XB[w]);
    }
    const cptr<cd> gA0 = as_constant(PA.gauge_Et), gB0 = as_constant(PB.gauge_Et);
    auto step = [&](int jj) {
        const int k = min(k0 + jj, PA.Nt - 1);
        const double xn = walk_load_x(1, xt + (size_t)min(k + 1, PA.Nt - 1) * xs, xs).v0;
        const double xe = xk + PA.eps;  // the reference's perturbed control
        const cd q = cis_m1(PA.gauge_a * (xe - xk)), om = gauge_cis(PA.gauge_a * xk - PA.gauge_a * xn);
        xk = xn;
        cptr<cd> gA = gA0, gB = gB0;  // (opaque per step: the row addresses stay in the step)
        asm volatile("" : "+s"(gA), "+s"(gB));
        cd rh[DA];
        ladder_rho<DA>(q, rh);
        cd ea[kGaugePairs<DA>], eb[kGaugePairs<2>];
        gauge_phases_ladder<DA>(om, ea);
        gauge_phases_ladder<2>(om, eb);
        cd rb[2];
        rb[0] = rh[0];
        rb[1] = rh[1];
        const double sa = tilde_step<DA>(gA, ea, rh, XA) * PA.inv_eps;
        double sb = 0.0;
#pragma unroll
        for (int w = 0; w < NXB; ++w) sb += tilde_step<2>(gB + (TWB ? 0 : w) * 4, eb, rb, XB[w]) * PB.inv_eps;
        double v = 0.0;  // k_sec_reduce's sum of the classes' parts, in the plan's class order
        v += a_first ? sa : sb;
        v += a_first ? sb : sa;
        return v;
    };
#pragma unroll 1
    for (int j0 = 0; j0 < PA.L; j0 += kFdxTile) {
        const int nj = min(kFdxTile, PA.L - j0);
#pragma unroll 1
        for (int t = 0; t < nj; ++t) ftile[threadIdx.x][t] = step(j0 + t);
        __syncthreads();
        const int j = threadIdx.x % kFdxTile;
#pragma unroll 1
        for (int row = threadIdx.x / kFdxTile; row < kWalkBlock; row += kWalkBlock / kFdxTile) {
            const int br = frow[row].x, kk = frow[row].y + j0 + j;
            if (j < nj && br >= 0 && kk < PA.Nt) BA.Fdx[(size_t)br * PA.nx + kk] = ftile[row][j];
        }
        __syncthreads();
    }
}

}  // namespace grape
