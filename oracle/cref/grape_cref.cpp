// grape_cref.cpp -- reference-faithful C++ restatement of RobustGRAPE.jl's hot path.
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY: built into oracle/build/libgrape_cref.so,
// loaded by tests/ and by bench.py's cpu_baseline leg, never by robustgrape_amd/.
//
// It performs the SAME work as the Julia reference, op for op, so that timing it
// stands in for timing the reference (Julia is absent from this image):
//   * calculate_unitary_and_derivatives   src/UnitaryCalculations.jl:20-155
//       - one exp per closure call site per step, including the eps2
//         exponentials that only the mixed stencils consume (:53-54, :61-62),
//         which are dead work when there are no error sources;
//       - cum_evo_inv = inv(cum_evo) by LU (getrf + getri) every step (:47);
//       - C_k^-1 * dE * C_{k-1} as two products per derivative (:52,60,69,79,91);
//       - cumsum / reverse cumsum and the assembly loops (:102-152).
//   * calculate_fidelity_and_derivatives  src/FidelityCalculations.jl:19-119
//       - every product chain of the trace expressions evaluated left to right
//         as dense matrix products, tr_mod(A) = tr(P0*A) as a product + trace.
//   * Julia LinearAlgebra.exp! (isdiag, zgebal 'B', Pade 3/5/7/9/13 by 1-norm,
//     gesv with partial pivoting, squaring, undo balancing) and inv (getrf/getri).
// Hamiltonians come from the operator-basis descriptor (include/grape.h), built
// afresh at every closure call site, like the closures are called.
// Matrices are column-major like Julia.
#include <cmath>
#include <cstring>
#include <vector>

#include "grape.h"

namespace {

struct cx {
    double re, im;
};
inline cx operator+(cx a, cx b) { return {a.re + b.re, a.im + b.im}; }
inline cx operator-(cx a, cx b) { return {a.re - b.re, a.im - b.im}; }
inline cx operator*(cx a, cx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
inline cx operator*(double s, cx a) { return {s * a.re, s * a.im}; }
inline cx conj(cx a) { return {a.re, -a.im}; }
inline double cabs1(cx a) { return std::fabs(a.re) + std::fabs(a.im); }
inline double cabs(cx a) { return std::hypot(a.re, a.im); }
inline cx cdiv(cx a, cx b) {  // Smith (gfortran)
    if (std::fabs(b.re) >= std::fabs(b.im)) {
        const double r = b.im / b.re, den = b.re + b.im * r;
        return {(a.re + a.im * r) / den, (a.im - a.re * r) / den};
    }
    const double r = b.re / b.im, den = b.im + b.re * r;
    return {(a.re * r + a.im) / den, (a.im * r - a.re) / den};
}

struct Mat {
    int n = 0;
    std::vector<cx> a;
    Mat() = default;
    explicit Mat(int n_) : n(n_), a((size_t)n_ * n_, cx{0, 0}) {}
    cx &operator()(int i, int j) { return a[i + (size_t)j * n]; }
    cx operator()(int i, int j) const { return a[i + (size_t)j * n]; }
    static Mat eye(int n) {
        Mat m(n);
        for (int i = 0; i < n; ++i) m(i, i) = {1, 0};
        return m;
    }
};

Mat operator*(const Mat &A, const Mat &B) {  // zgemm-style column sweep
    const int n = A.n;
    Mat C(n);
    for (int j = 0; j < n; ++j)
        for (int k = 0; k < n; ++k) {
            const cx b = B(k, j);
            for (int i = 0; i < n; ++i) C(i, j) = C(i, j) + A(i, k) * b;
        }
    return C;
}
Mat operator+(const Mat &A, const Mat &B) {
    Mat C(A.n);
    for (size_t i = 0; i < C.a.size(); ++i) C.a[i] = A.a[i] + B.a[i];
    return C;
}
Mat operator-(const Mat &A, const Mat &B) {
    Mat C(A.n);
    for (size_t i = 0; i < C.a.size(); ++i) C.a[i] = A.a[i] - B.a[i];
    return C;
}
Mat operator*(double s, const Mat &A) {
    Mat C(A.n);
    for (size_t i = 0; i < C.a.size(); ++i) C.a[i] = s * A.a[i];
    return C;
}
Mat operator*(cx s, const Mat &A) {
    Mat C(A.n);
    for (size_t i = 0; i < C.a.size(); ++i) C.a[i] = s * A.a[i];
    return C;
}
Mat adj(const Mat &A) {
    Mat C(A.n);
    for (int i = 0; i < A.n; ++i)
        for (int j = 0; j < A.n; ++j) C(i, j) = conj(A(j, i));
    return C;
}
cx trace(const Mat &A) {
    cx t{0, 0};
    for (int i = 0; i < A.n; ++i) t = t + A(i, i);
    return t;
}

// ---------------------------------------------------------------- LAPACK-like
// getrf with partial pivoting (izamax on |re|+|im|), in place; ipiv 0-based.
bool getrf(Mat &A, std::vector<int> &ipiv) {
    const int n = A.n;
    ipiv.assign(n, 0);
    bool ok = true;
    for (int j = 0; j < n; ++j) {
        int p = j;
        double best = cabs1(A(j, j));
        for (int i = j + 1; i < n; ++i)
            if (cabs1(A(i, j)) > best) {
                best = cabs1(A(i, j));
                p = i;
            }
        ipiv[j] = p;
        if (best == 0.0) {
            ok = false;
            continue;
        }
        if (p != j)
            for (int c = 0; c < n; ++c) std::swap(A(j, c), A(p, c));
        const cx r = cdiv({1, 0}, A(j, j));
        for (int i = j + 1; i < n; ++i) A(i, j) = A(i, j) * r;
        for (int c = j + 1; c < n; ++c) {
            const cx t = {-A(j, c).re, -A(j, c).im};
            for (int i = j + 1; i < n; ++i) A(i, c) = A(i, c) + A(i, j) * t;
        }
    }
    return ok;
}
// getrs: solve A X = B given the factorisation
void getrs(const Mat &LU, const std::vector<int> &ipiv, Mat &B) {
    const int n = LU.n;
    for (int j = 0; j < n; ++j)
        if (ipiv[j] != j)
            for (int c = 0; c < n; ++c) std::swap(B(j, c), B(ipiv[j], c));
    for (int c = 0; c < n; ++c) {
        for (int k = 0; k < n; ++k) {
            const cx bk = B(k, c);
            for (int i = k + 1; i < n; ++i) B(i, c) = B(i, c) - bk * LU(i, k);
        }
        for (int k = n - 1; k >= 0; --k) {
            B(k, c) = cdiv(B(k, c), LU(k, k));
            const cx bk = B(k, c);
            for (int i = 0; i < k; ++i) B(i, c) = B(i, c) - bk * LU(i, k);
        }
    }
}
thread_local bool g_singular = false;
Mat gesv(Mat A, Mat B) {
    std::vector<int> ipiv;
    if (!getrf(A, ipiv)) g_singular = true;
    getrs(A, ipiv, B);
    return B;
}
// Julia inv: getrf + getri (here: solve A X = I with the factorisation)
Mat inv(Mat A) {
    std::vector<int> ipiv;
    if (!getrf(A, ipiv)) g_singular = true;
    Mat X = Mat::eye(A.n);
    getrs(A, ipiv, X);
    return X;
}

// zgebal 'B' (LAPACK 3.10 algorithm)
void gebal(Mat &A, int &ilo, int &ihi, std::vector<double> &scale) {
    const int n = A.n;
    scale.assign(n, 1.0);
    int k = 1, l = n;
    auto swap = [&](int j, int m) {
        scale[m - 1] = j;
        if (j != m) {
            for (int r = 0; r < l; ++r) std::swap(A(r, j - 1), A(r, m - 1));
            for (int c = k - 1; c < n; ++c) std::swap(A(j - 1, c), A(m - 1, c));
        }
    };
    bool done = false;
    while (!done) {
        bool found = false;
        for (int j = l; j >= 1 && !found; --j) {
            bool zero = true;
            for (int i = 1; i <= l && zero; ++i)
                if (i != j && (A(j - 1, i - 1).re != 0 || A(j - 1, i - 1).im != 0)) zero = false;
            if (zero) {
                swap(j, l);
                found = true;
            }
        }
        if (!found) break;
        if (l == 1) {
            ilo = k;
            ihi = l;
            return;
        }
        --l;
    }
    while (true) {
        bool found = false;
        for (int j = k; j <= l && !found; ++j) {
            bool zero = true;
            for (int i = k; i <= l && zero; ++i)
                if (i != j && (A(i - 1, j - 1).re != 0 || A(i - 1, j - 1).im != 0)) zero = false;
            if (zero) {
                swap(j, k);
                found = true;
            }
        }
        if (!found) break;
        ++k;
    }
    for (int i = k; i <= l; ++i) scale[i - 1] = 1.0;
    const double sfmin1 = 2.2250738585072014e-308 / 2.220446049250313e-16, sfmax1 = 1.0 / sfmin1;
    const double sfmin2 = sfmin1 * 2.0, sfmax2 = 1.0 / sfmin2;
    bool noconv = true;
    while (noconv) {
        noconv = false;
        for (int i = k; i <= l; ++i) {
            double c = 0, r = 0, ca = 0, ra = 0;
            for (int q = k; q <= l; ++q) {
                c = std::hypot(c, cabs(A(q - 1, i - 1)));
                r = std::hypot(r, cabs(A(i - 1, q - 1)));
            }
            for (int q = 1; q <= l; ++q) ca = std::fmax(ca, cabs(A(q - 1, i - 1)));
            for (int q = k; q <= n; ++q) ra = std::fmax(ra, cabs(A(i - 1, q - 1)));
            if (c == 0.0 || r == 0.0) continue;
            double g = r / 2.0, f = 1.0, s = c + r;
            while (!(c >= g || std::fmax(f, std::fmax(c, ca)) >= sfmax2 || std::fmin(r, std::fmin(g, ra)) <= sfmin2)) {
                f *= 2; c *= 2; ca *= 2; r /= 2; g /= 2; ra /= 2;
            }
            g = c / 2.0;
            while (!(g < r || std::fmax(r, ra) >= sfmax2 ||
                     std::fmin(std::fmin(f, c), std::fmin(g, ca)) <= sfmin2)) {
                f /= 2; c /= 2; g /= 2; ca /= 2; r *= 2; ra *= 2;
            }
            if ((c + r) >= 0.95 * s) continue;
            if (f < 1.0 && scale[i - 1] < 1.0 && f * scale[i - 1] <= sfmin1) continue;
            if (f > 1.0 && scale[i - 1] > 1.0 && scale[i - 1] >= sfmax1 / f) continue;
            const double gi = 1.0 / f;
            scale[i - 1] *= f;
            noconv = true;
            for (int q = k; q <= n; ++q) A(i - 1, q - 1) = gi * A(i - 1, q - 1);
            for (int q = 1; q <= l; ++q) A(q - 1, i - 1) = f * A(q - 1, i - 1);
        }
    }
    ilo = k;
    ihi = l;
}

const double P3[] = {120.0, 60.0, 12.0, 1.0};
const double P5[] = {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0};
const double P7[] = {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0};
const double P9[] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                     2162160.0, 110880.0, 3960.0, 90.0, 1.0};
const double P13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                      1187353796428800.0, 129060195264000.0, 10559470521600.0,
                      670442572800.0, 33522128640.0, 1323241920.0,
                      40840800.0, 960960.0, 16380.0, 182.0, 1.0};
thread_local long g_exp_calls = 0;

Mat julia_exp(Mat A) {
    ++g_exp_calls;
    const int n = A.n;
    bool diag = true;
    for (int j = 0; j < n && diag; ++j)
        for (int i = 0; i < n; ++i)
            if (i != j && (A(i, j).re != 0 || A(i, j).im != 0)) {
                diag = false;
                break;
            }
    if (diag) {
        Mat E(n);
        for (int i = 0; i < n; ++i) {
            const double e = std::exp(A(i, i).re);
            E(i, i) = {e * std::cos(A(i, i).im), e * std::sin(A(i, i).im)};
        }
        return E;
    }
    int ilo, ihi;
    std::vector<double> scale;
    gebal(A, ilo, ihi, scale);
    double nA = 0;
    for (int j = 0; j < n; ++j) {
        double s = 0;
        for (int i = 0; i < n; ++i) s += cabs(A(i, j));
        nA = std::fmax(nA, s);
    }
    const Mat I = Mat::eye(n);
    Mat X;
    if (nA <= 2.1) {
        const double *C;
        int len;
        if (nA > 0.95) { C = P9; len = 10; }
        else if (nA > 0.25) { C = P7; len = 8; }
        else if (nA > 0.015) { C = P5; len = 6; }
        else { C = P3; len = 4; }
        const Mat A2 = A * A;
        Mat P = I;
        Mat U = C[1] * P;
        Mat V = C[0] * P;
        for (int kk = 1; kk < len / 2; ++kk) {
            P = P * A2;
            U = U + C[2 * kk + 1] * P;
            V = V + C[2 * kk] * P;
        }
        U = A * U;
        X = gesv(V - U, V + U);
    } else {
        const double s = std::log2(nA / 5.4);
        int si = 0;
        if (s > 0) {
            si = (int)std::ceil(s);
            A = (1.0 / std::ldexp(1.0, si)) * A;
        }
        const double *c = P13;
        const Mat A2 = A * A, A4 = A2 * A2, A6 = A2 * A4;
        const Mat U = A * (A6 * (c[13] * A6 + c[11] * A4 + c[9] * A2) + c[7] * A6 + c[5] * A4 + c[3] * A2 + c[1] * I);
        const Mat V = A6 * (c[12] * A6 + c[10] * A4 + c[8] * A2) + c[6] * A6 + c[4] * A4 + c[2] * A2 + c[0] * I;
        X = gesv(V - U, V + U);
        for (int t = 0; t < si; ++t) X = X * X;
    }
    for (int j = ilo; j <= ihi; ++j) {
        const double scj = scale[j - 1];
        for (int i = 0; i < n; ++i) X(j - 1, i) = scj * X(j - 1, i);
        for (int i = 0; i < n; ++i) X(i, j - 1) = cdiv(X(i, j - 1), {scj, 0.0});
    }
    auto rcswap = [&](int i, int j) {
        for (int r = 0; r < n; ++r) std::swap(X(r, i - 1), X(r, j - 1));
        for (int c = 0; c < n; ++c) std::swap(X(i - 1, c), X(j - 1, c));
    };
    if (ilo > 1)
        for (int j = ilo - 1; j >= 1; --j) rcswap(j, (int)scale[j - 1]);
    if (ihi < n)
        for (int j = ihi + 1; j <= n; ++j) rcswap(j, (int)scale[j - 1]);
    return X;
}

// ---------------------------------------------------------------- closures
struct Problem {
    const grape_desc *d;
    int n, Nt, np, na, ne;
    std::vector<Mat> ops;
};

cx coef(const grape_term &t, int nt1, const double *xk, const double *xadd) {
    double v = 1.0;
    if (t.var == 1) v = xk[t.index];
    else if (t.var == 2) v = xadd[t.index];
    else if (t.var == 3) v = nt1;
    const double arg = t.a * v + t.b;
    double fr = 1, fi = 0;
    if (t.func == 1) fr = arg;
    else if (t.func == 2) fr = std::cos(arg);
    else if (t.func == 3) fr = std::sin(arg);
    else if (t.func == 4) { fr = std::cos(arg); fi = std::sin(arg); }
    return cx{t.scale_re, t.scale_im} * cx{fr, fi};
}
Mat eval_terms(const Problem &p, const grape_term *t, int nterm, int nt1, const double *xk, const double *xadd) {
    Mat H(p.n);
    for (int q = 0; q < nterm; ++q) H = H + coef(t[q], nt1, xk, xadd) * p.ops[t[q].op];
    return H;
}
Mat H0(const Problem &p, int nt1, const double *xk, const double *xadd) {
    return eval_terms(p, p.d->h0_terms, p.d->n_h0_terms, nt1, xk, xadd);
}
Mat Herr(const Problem &p, int e, int nt1, const double *xk, const double *xadd, double err) {
    const int o0 = p.d->err_term_offsets[e], o1 = p.d->err_term_offsets[e + 1];
    return err * eval_terms(p, p.d->err_terms + o0, o1 - o0, nt1, xk, xadd);
}
Mat target(const Problem &p, const double *xadd) {
    return eval_terms(p, p.d->target_terms, p.d->n_target_terms, 1, nullptr, xadd);
}

struct UnitaryOut {
    Mat U;
    std::vector<Mat> U_dx;          // [k*np + p]
    std::vector<Mat> U_dx_add;      // [q]
    std::vector<Mat> U_derr;        // [e]
    std::vector<Mat> U_derr_dx;     // [(e*Nt + k)*np + p]
    std::vector<Mat> U_derr_dx_add; // [e*na + q]
};

// src/UnitaryCalculations.jl:20-155
UnitaryOut unitary_and_derivatives(const Problem &p, const double *x) {
    const int n = p.n, Nt = p.Nt, np = p.np, na = p.na, ne = p.ne;
    const double eps = p.d->eps, eps2 = p.d->eps2;
    const double dt = p.d->t0 / Nt;
    const cx mdt = {0.0, -dt};  // -im*dt
    const double *xadd = x + (size_t)np * Nt;
    std::vector<double> xadd_copy(xadd, xadd + na), xm(np);
    auto E = [&](const Mat &H) { return julia_exp(mdt * H); };
    Mat cum = Mat::eye(n), old = cum;
    std::vector<Mat> iU_dx((size_t)np * Nt, Mat(n)), iU_dx_add((size_t)na * Nt, Mat(n)),
        iU_derr((size_t)ne * Nt, Mat(n)), iU_derr_dx((size_t)np * ne * Nt, Mat(n)),
        iU_derr_dx_add((size_t)na * ne * Nt, Mat(n));
    std::vector<Mat> derr_arr(ne, Mat(n)), dx_arr(np, Mat(n)), dxa_arr(na, Mat(n));
    const double ie = 1.0 / eps, ie2 = 1.0 / (eps2 * eps2);
    for (int k = 0; k < Nt; ++k) {
        const int nt1 = k + 1;
        const double *xk = x + (size_t)k * np;
        const Mat Ek = E(H0(p, nt1, xk, xadd));
        cum = Ek * cum;
        const Mat cinv = inv(cum);
        for (int q = 0; q < np; ++q) xm[q] = xk[q];
        for (int q = 0; q < np; ++q) {
            xm[q] += eps;
            const Mat Ed = E(H0(p, nt1, xm.data(), xadd));
            iU_dx[(size_t)k * np + q] = cinv * (ie * (Ed - Ek)) * old;
            xm[q] = xk[q] + eps2;
            dx_arr[q] = E(H0(p, nt1, xm.data(), xadd));
            xm[q] = xk[q];
        }
        for (int q = 0; q < na; ++q) {
            xadd_copy[q] += eps;
            const Mat Ed = E(H0(p, nt1, xk, xadd_copy.data()));
            iU_dx_add[(size_t)k * na + q] = cinv * (ie * (Ed - Ek)) * old;
            xadd_copy[q] = xadd[q] + eps2;
            dxa_arr[q] = E(H0(p, nt1, xk, xadd_copy.data()));
            xadd_copy[q] = xadd[q];
        }
        for (int e = 0; e < ne; ++e) {
            const Mat Ee = E(Herr(p, e, nt1, xk, xadd, eps) + H0(p, nt1, xk, xadd));
            iU_derr[(size_t)k * ne + e] = cinv * (ie * (Ee - Ek)) * old;
            derr_arr[e] = E(Herr(p, e, nt1, xk, xadd, eps2) + H0(p, nt1, xk, xadd));
            for (int q = 0; q < np; ++q) {
                xm[q] += eps2;
                const Mat Em = E(Herr(p, e, nt1, xm.data(), xadd, eps2) + H0(p, nt1, xm.data(), xadd));
                iU_derr_dx[((size_t)k * ne + e) * np + q] =
                    cinv * (ie2 * (Em + Ek - derr_arr[e] - dx_arr[q])) * old;
                xm[q] = xk[q];
            }
            for (int q = 0; q < na; ++q) {
                xadd_copy[q] += eps2;
                const Mat Em =
                    E(Herr(p, e, nt1, xk, xadd_copy.data(), eps2) + H0(p, nt1, xk, xadd_copy.data()));
                iU_derr_dx_add[((size_t)k * ne + e) * na + q] =
                    cinv * (ie2 * (Em + Ek - derr_arr[e] - dxa_arr[q])) * old;
                xadd_copy[q] = xadd[q];
            }
        }
        old = cum;
    }
    UnitaryOut o;
    o.U = cum;
    o.U_dx.resize((size_t)np * Nt);
    for (int k = 0; k < Nt; ++k)
        for (int q = 0; q < np; ++q) o.U_dx[(size_t)k * np + q] = cum * iU_dx[(size_t)k * np + q];
    o.U_dx_add.assign(na, Mat(n));
    for (int q = 0; q < na; ++q) {
        Mat s(n);
        for (int k = 0; k < Nt; ++k) s = s + iU_dx_add[(size_t)k * na + q];
        o.U_dx_add[q] = cum * s;
    }
    o.U_derr.assign(ne, Mat(n));
    o.U_derr_dx.assign((size_t)ne * Nt * np, Mat(n));
    o.U_derr_dx_add.assign((size_t)ne * na, Mat(n));
    for (int e = 0; e < ne; ++e) {
        std::vector<Mat> cs(Nt, Mat(n)), rcs(Nt, Mat(n));
        Mat acc(n);
        for (int k = 0; k < Nt; ++k) {
            acc = acc + iU_derr[(size_t)k * ne + e];
            cs[k] = acc;
        }
        acc = Mat(n);
        for (int k = Nt - 1; k >= 0; --k) {
            acc = acc + iU_derr[(size_t)k * ne + e];
            rcs[k] = acc;
        }
        Mat s(n);
        for (int k = 0; k < Nt; ++k) s = s + iU_derr[(size_t)k * ne + e];
        o.U_derr[e] = cum * s;
        auto &Y = o.U_derr_dx;
        for (int k = 1; k < Nt; ++k)
            for (int q = 0; q < np; ++q) {
                Mat &y = Y[((size_t)e * Nt + k) * np + q];
                y = y + iU_dx[(size_t)k * np + q] * cs[k - 1];
            }
        for (int k = 0; k < Nt - 1; ++k)
            for (int q = 0; q < np; ++q) {
                Mat &y = Y[((size_t)e * Nt + k) * np + q];
                y = y + rcs[k + 1] * iU_dx[(size_t)k * np + q];
            }
        for (int k = 0; k < Nt; ++k)
            for (int q = 0; q < np; ++q) {
                Mat &y = Y[((size_t)e * Nt + k) * np + q];
                y = y + iU_derr_dx[((size_t)k * ne + e) * np + q];
                y = cum * y;
            }
        for (int q = 0; q < na; ++q) {
            Mat a2(n);
            for (int k = 1; k < Nt; ++k) a2 = a2 + iU_dx_add[(size_t)k * na + q] * cs[k - 1];
            for (int k = 0; k < Nt - 1; ++k) a2 = a2 + rcs[k + 1] * iU_dx_add[(size_t)k * na + q];
            for (int k = 0; k < Nt; ++k) a2 = a2 + iU_derr_dx_add[((size_t)k * ne + e) * na + q];
            o.U_derr_dx_add[(size_t)e * na + q] = cum * a2;
        }
    }
    return o;
}

Mat load_col_major(const double *src, int n) {
    Mat m(n);
    for (int i = 0; i < n * n; ++i) m.a[i] = {src[2 * i], src[2 * i + 1]};
    return m;
}
void store_col_major(const Mat &m, double *dst) {
    for (size_t i = 0; i < m.a.size(); ++i) {
        dst[2 * i] = m.a[i].re;
        dst[2 * i + 1] = m.a[i].im;
    }
}

Problem make_problem(const grape_desc *d) {
    Problem p;
    p.d = d;
    p.n = d->ndim;
    p.Nt = d->ntimes;
    p.np = d->nparam;
    p.na = d->nadd;
    p.ne = d->nerr;
    for (int o = 0; o < d->n_ops; ++o) p.ops.push_back(load_col_major(d->ops + (size_t)2 * o * p.n * p.n, p.n));
    return p;
}

}  // namespace

extern "C" {

long grape_cref_exp_calls(void) { return g_exp_calls; }

int grape_cref_expm(int n, const double *A, double *E) {
    const Mat X = julia_exp(load_col_major(A, n));
    store_col_major(X, E);
    return 0;
}

// src/FidelityCalculations.jl:19-119 (outputs as grape_fidelity_grad for ONE eval)
int grape_cref_fidelity_grad(const grape_desc *d, const double *x, double *F_out, double *F_dx_out,
                             double *F_d2err_out, double *F_d2err_dx_out) {
    g_singular = false;
    const Problem p = make_problem(d);
    const int n = p.n, Nt = p.Nt, np = p.np, na = p.na, ne = p.ne;
    const int nx = np * Nt + na;
    const UnitaryOut u = unitary_and_derivatives(p, x);
    const double *xadd = x + (size_t)np * Nt;
    const Mat U0 = target(p, xadd);
    std::vector<Mat> U0d(na, Mat(n));
    std::vector<double> xac(xadd, xadd + na);
    for (int q = 0; q < na; ++q) {
        xac[q] += d->eps;
        U0d[q] = (1.0 / d->eps) * (target(p, xac.data()) - U0);
        xac[q] = xadd[q];
    }
    Mat P0(n), P(n);
    double D = 0;
    for (int i = 0; i < n; ++i) {
        P0(i, i) = {d->projector_diag[i], 0};
        P(i, i) = {d->projector_diag[i] != 0 ? 1.0 : 0.0, 0};
        D += d->projector_diag[i];
    }
    auto trm = [&](const Mat &A) { return trace(P0 * A); };
    const double DD = D * (D + 1);
    const Mat &U = u.U;
    const Mat U0a = adj(U0), Ua = adj(U);
    *F_out = (trm(P * U0a * U * P * Ua * U0).re + std::pow(cabs(trm(P * U0a * U)), 2)) / DD;
    const cx tc = conj(trm(P * U0a * U));
    for (int k = 0; k < Nt; ++k)
        for (int q = 0; q < np; ++q) {
            const Mat &Ud = u.U_dx[(size_t)k * np + q];
            F_dx_out[(size_t)k * np + q] =
                (trm(P * U0a * Ud * P * Ua * U0 + P * U0a * U * P * adj(Ud) * U0).re +
                 2 * (tc * trm(P * U0a * Ud)).re) / DD;
        }
    for (int q = 0; q < na; ++q) {
        const Mat &Ud = u.U_dx_add[q];
        const Mat &U0q = U0d[q];
        F_dx_out[(size_t)np * Nt + q] =
            (trm(P * U0a * Ud * P * Ua * U0 + P * U0a * U * P * adj(Ud) * U0 + P * adj(U0q) * U * P * Ua * U0 +
                 P * U0a * U * P * Ua * U0q).re +
             2 * (tc * trm(P * U0a * Ud + P * adj(U0q) * U)).re) / DD;
    }
    for (int e = 0; e < ne; ++e) {
        const Mat &Ue = u.U_derr[e];
        const Mat Uea = adj(Ue);
        F_d2err_out[e] = 2 * (trm(P * U0a * Ue * P * Uea * U0 - P * Uea * Ue).re +
                              std::pow(cabs(trm(P * U0a * Ue)), 2) - D * trm(P * Uea * Ue).re) / DD;
        const cx te = conj(trm(P * U0a * Ue));
        double *col = F_d2err_dx_out + (size_t)e * nx;
        for (int k = 0; k < Nt; ++k)
            for (int q = 0; q < np; ++q) {
                const Mat &Y = u.U_derr_dx[((size_t)e * Nt + k) * np + q];
                const Mat Ya = adj(Y);
                col[(size_t)k * np + q] =
                    2 * (trm(P * U0a * Y * P * Uea * U0 + P * U0a * Ue * P * Ya * U0 - P * Ya * Ue - P * Uea * Y).re +
                         2 * (te * trm(P * U0a * Y)).re - D * trm(P * Ya * Ue + P * Uea * Y).re) / DD;
            }
        for (int q = 0; q < na; ++q) {
            const Mat &Y = u.U_derr_dx_add[(size_t)e * na + q];
            const Mat Ya = adj(Y);
            const Mat &U0q = U0d[q];
            col[(size_t)np * Nt + q] =
                2 * (trm(P * adj(U0q) * Ue * P * Uea * U0 + P * U0a * Y * P * Uea * U0 + P * U0a * Ue * P * Ya * U0 +
                         P * U0a * Ue * P * Uea * U0q - P * Ya * Ue - P * Uea * Y).re +
                     2 * (te * trm(P * adj(U0q) * Ue + P * U0a * Y)).re - D * trm(P * Ya * Ue + P * Uea * Y).re) /
                DD;
        }
    }
    return g_singular ? GRAPE_ERR_SINGULAR : GRAPE_OK;
}

// SURVEY.md 8d C4 CPU baseline: nb independent evaluations (restarts) spread over
// nthreads OpenMP threads (the reference itself is single-threaded; this is the
// "all host cores" form of the port).  Per-eval outputs as grape_cref_fidelity_grad,
// eval b's arrays at b * (n_x | ne | ne * n_x).  Returns the first nonzero status.
int grape_cref_fidelity_grad_batch(const grape_desc *d, int nb, int nthreads, const double *x, double *F,
                                   double *F_dx, double *F_d2err, double *F_d2err_dx) {
    const int nx = d->nparam * d->ntimes + d->nadd, ne = d->nerr;
    int status = GRAPE_OK;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int b = 0; b < nb; ++b) {
        const int rc = grape_cref_fidelity_grad(d, x + (size_t)b * nx, F + b, F_dx + (size_t)b * nx,
                                                ne ? F_d2err + (size_t)b * ne : nullptr,
                                                ne ? F_d2err_dx + (size_t)b * ne * nx : nullptr);
        if (rc) {
#pragma omp critical
            if (!status) status = rc;
        }
    }
    return status;
}

// src/UnitaryCalculations.jl:154 outputs, column-major, reference shapes
int grape_cref_unitary_derivs(const grape_desc *d, const double *x, double *U, double *U_dx, double *U_dx_add,
                              double *U_derr, double *U_derr_dx, double *U_derr_dx_add) {
    g_singular = false;
    const Problem p = make_problem(d);
    const UnitaryOut u = unitary_and_derivatives(p, x);
    const size_t T = (size_t)2 * p.n * p.n;
    if (U) store_col_major(u.U, U);
    for (int k = 0; k < p.Nt; ++k)
        for (int q = 0; q < p.np; ++q)
            if (U_dx) store_col_major(u.U_dx[(size_t)k * p.np + q], U_dx + T * ((size_t)k * p.np + q));
    for (int q = 0; q < p.na; ++q)
        if (U_dx_add) store_col_major(u.U_dx_add[q], U_dx_add + T * q);
    for (int e = 0; e < p.ne; ++e) {
        if (U_derr) store_col_major(u.U_derr[e], U_derr + T * e);
        for (int k = 0; k < p.Nt; ++k)
            for (int q = 0; q < p.np; ++q)
                if (U_derr_dx)
                    store_col_major(u.U_derr_dx[((size_t)e * p.Nt + k) * p.np + q],
                                    U_derr_dx + T * (((size_t)e * p.Nt + k) * p.np + q));
        for (int q = 0; q < p.na; ++q)
            if (U_derr_dx_add) store_col_major(u.U_derr_dx_add[(size_t)e * p.na + q], U_derr_dx_add + T * ((size_t)e * p.na + q));
    }
    return g_singular ? GRAPE_ERR_SINGULAR : GRAPE_OK;
}

}  // extern "C"
