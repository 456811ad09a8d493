// grape_device.hpp -- CDNA4 (gfx950) device building blocks of the GRAPE engine.
//
// Execution model ("row groups"): a 64-lane wave is split into GPW = 64/D
// groups of D lanes; each group owns ONE d x d complex FP64 matrix at a time,
// lane i of the group holding row i in VGPRs (D complex = 4*D VGPRs per
// matrix).  A product C = A.B keeps the left operand's row in registers and
// broadcasts the right operand from the group's LDS tile (all D lanes of a
// group read the same 16-B element -> one ds_read_b128 per complex MAC, groups
// land on disjoint banks because a tile is D*D*16 B = 4 (mod 64) dwords apart).
//
// The matrix exponential runs in COLUMN form: lane i holds column i of A (the
// same code computes exp(A)^T-rows = exp(A)-columns; the Pade polynomial
// products commute, so only their rounding order changes).  Column ownership
// makes the 1-norm, the dominance test and the whole LU solve local to a lane
// except for one multiplier broadcast per elimination step: ~4x fewer LDS
// stores than a row-distributed solve, and LDS (stores cost 13 cycles per
// ds_write_b128) is what bounds this kernel family on gfx950.
// FP64 throughout: eps = 1e-8 finite differences forbid lower precision.
//
// Numerics follow the reference's third-party kernels (Julia LinearAlgebra
// exp!, LAPACK zgetrf/zgetrs as called by gesv!):
//   * Pade degree by 1-norm thresholds 0.015/0.25/0.95/2.1 (m = 3/5/7/9),
//     else m = 13 with s = ceil(log2(|A|_1/5.4)) squarings;
//   * Julia's accumulation order for U and V;
//   * gesv: partial pivoting with izamax's |re|+|im| (first max wins), the
//     multiplier formed as a_ij * (1/pivot) (zgetf2's zscal by the reciprocal),
//     forward substitution in pivot order, back substitution dividing by the
//     diagonal (ztrsm), complex division by Smith's method (gfortran).
// Balancing (zgebal 'B') is not applied on the device: for the skew-Hermitian
// generators A = -i dt H of a Hermitian H it is a permutation only (scaling is
// the identity because row and column norms coincide), which changes nothing
// but the summation order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace grape {

struct cd {
    double re, im;
};

__device__ __forceinline__ cd cmake(double r, double i) { cd z; z.re = r; z.im = i; return z; }
__device__ __forceinline__ cd czero() { return cmake(0.0, 0.0); }
__device__ __forceinline__ cd cadd(cd a, cd b) { return cmake(a.re + b.re, a.im + b.im); }
__device__ __forceinline__ cd csub(cd a, cd b) { return cmake(a.re - b.re, a.im - b.im); }
__device__ __forceinline__ cd cconj(cd a) { return cmake(a.re, -a.im); }
__device__ __forceinline__ cd cscale(double s, cd a) { return cmake(s * a.re, s * a.im); }
// plain (unfused) complex product, as Julia's *(::Complex, ::Complex)
__device__ __forceinline__ cd cmul(cd a, cd b) {
    return cmake(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
// fused forms: s*x + y (2 FMAs) and a*b with 2 MULs + 2 FMAs
__device__ __forceinline__ cd caxpy(double s, cd x, cd y) { return cmake(fma(s, x.re, y.re), fma(s, x.im, y.im)); }
__device__ __forceinline__ cd cmulf(cd a, cd b) {
    return cmake(fma(a.re, b.re, -(a.im * b.im)), fma(a.re, b.im, a.im * b.re));
}
// c += a*b with four FMAs (the BLAS-kernel form)
__device__ __forceinline__ void cmac(cd &c, cd a, cd b) {
    c.re = fma(a.re, b.re, c.re);
    c.re = fma(-a.im, b.im, c.re);
    c.im = fma(a.re, b.im, c.im);
    c.im = fma(a.im, b.re, c.im);
}
// Smith's complex division a/b (gfortran's complex division, used by LAPACK)
__device__ __forceinline__ cd cdiv(cd a, cd b) {
    if (fabs(b.re) >= fabs(b.im)) {
        const double r = b.im / b.re, den = b.re + b.im * r;
        return cmake((a.re + a.im * r) / den, (a.im - a.re * r) / den);
    }
    const double r = b.re / b.im, den = b.im + b.re * r;
    return cmake((a.re * r + a.im) / den, (a.im * r - a.re) / den);
}

// ---------------------------------------------------------------------------
// Group geometry
// ---------------------------------------------------------------------------
template <int D>
struct Geo {
    static constexpr int GPW = 64 / D;          // groups per wave
    static constexpr int TILE = D * D;          // complex elements per matrix tile
    static constexpr int AUX = 2 * D + 1;       // complex scratch per group (pivot row + reciprocal / reductions)
    static constexpr int GROUP_CD = TILE + AUX; // LDS complex elements per group
    // groups that only need the tile and a group reduction (D doubles): the solve-free
    // exponential kernels -- a smaller LDS footprint lets more one-wave workgroups share a CU
    static constexpr int LEAN_CD = TILE + (D + 1) / 2;
};

// Per-lane view of its group.
template <int D>
struct Group {
    int i;          // row owned by this lane (0..D-1)
    int g;          // group index within the wave
    bool lane_ok;   // lane belongs to a group (lane < GPW*D)
    cd *tile;       // LDS D*D tile (row-major)
    cd *aux;        // LDS 2*D scratch
    __device__ __forceinline__ double *auxd() { return reinterpret_cast<double *>(aux); }
};

template <int D>
__device__ __forceinline__ Group<D> make_group(cd *wave_lds, int lane, int stride = Geo<D>::GROUP_CD) {
    Group<D> G;
    G.lane_ok = lane < Geo<D>::GPW * D;
    G.g = G.lane_ok ? lane / D : Geo<D>::GPW - 1;
    G.i = G.lane_ok ? lane % D : 0;
    G.tile = wave_lds + G.g * stride;
    G.aux = G.tile + Geo<D>::TILE;
    return G;
}

// All group synchronisation goes through the workgroup barrier; kernels that
// use row groups launch 64-thread (one-wave) workgroups or keep every wave on
// the same barrier sequence.
__device__ __forceinline__ void gsync() { __syncthreads(); }
// Wave-local synchronisation for phases in which each group touches only its own tile: the
// LDS accesses of one wave complete in order, so a fence at wavefront scope is all a group
// needs between publishing its tile and reading it back -- no workgroup barrier.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int D>
__device__ __forceinline__ void tile_store_row(Group<D> &G, const cd (&r)[D], bool wr) {
    if (wr) {
#pragma unroll
        for (int j = 0; j < D; ++j) G.tile[G.i * D + j] = r[j];
    }
}

// Materialise a register row here: the empty asm "redefines" every element,
// so the compiler can neither sink the producing FMAs past this point nor keep
// the operands they consumed alive.  Without it, fully unrolled straight-line
// code gets its product chains interleaved with later stages (the LU solve)
// and register use quadruples (measured 412 -> 146 VGPRs at d = 9).
template <int D>
__device__ __forceinline__ void pin(cd (&r)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) asm volatile("" : "+v"(r[j].re), "+v"(r[j].im));
}

// c = a . B with R broadcast reads in flight: the read of element e + R is issued in step e,
// and a scheduling barrier per step keeps the compiler from sinking it to its use (the
// default schedule keeps one read ahead).  Measured on the exp kernels (d = 9, 16 384
// evaluations per pass): k_expm 24.8 -> 24.4 ms with R = 3, k_expm_grad 38.6 -> 38.1 ms and
// the error-variant k_expm 27.4 -> 26.5 ms with R = 2; deeper rings spill in k_expm_grad.
template <int D, bool TRANS, bool CONJ, int R>
__device__ __forceinline__ void mm_tile_ring(const cd (&a)[D], const cd *B, cd (&c)[D]) {
    auto ld = [&](int e) {
        const int k = e / D, j = e % D;
        cd b = TRANS ? B[j * D + k] : B[k * D + j];
        if (CONJ) b.im = -b.im;
        return b;
    };
    cd buf[R];
#pragma unroll
    for (int j = 0; j < D; ++j) c[j] = czero();
#pragma unroll
    for (int r = 0; r < R; ++r) buf[r] = ld(r);
#pragma unroll
    for (int e = 0; e < D * D; ++e) {
        const cd b = buf[e % R];
        if (e + R < D * D) buf[e % R] = ld(e + R);
        cmac(c[e % D], a[e / D], b);
        __builtin_amdgcn_sched_barrier(0);
    }
    pin<D>(c);
}
// c = a . B  (a: this lane's row, B: tile in LDS, row-major)
template <int D, bool TRANS = false, bool CONJ = false>
__device__ __forceinline__ void mm_tile(const cd (&a)[D], const cd *B, cd (&c)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) c[j] = czero();
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const cd ak = a[k];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            cd b = TRANS ? B[j * D + k] : B[k * D + j];
            if (CONJ) b.im = -b.im;
            cmac(c[j], ak, b);
        }
    }
    pin<D>(c);
}
// the product with a read ring of depth R (0: mm_tile's default schedule)
template <int D, int R, bool TRANS = false, bool CONJ = false>
__device__ __forceinline__ void mm_tile_r(const cd (&a)[D], const cd *B, cd (&c)[D]) {
    if constexpr (R > 0) mm_tile_ring<D, TRANS, CONJ, R>(a, B, c);
    else mm_tile<D, TRANS, CONJ>(a, B, c);
}

// The same product with row k+1 of B read while row k is consumed: D LDS
// reads in flight behind D complex MACs instead of one or two.  For the
// latency-bound scan kernels (two waves per SIMD, registers to spare); the
// exp kernels keep mm_tile, whose registers are spoken for.
template <int D, bool TRANS = false, bool CONJ = false>
__device__ __forceinline__ void mm_tile_pf(const cd (&a)[D], const cd *B, cd (&c)[D]) {
    auto ld = [&](int k, int j) {
        cd b = TRANS ? B[j * D + k] : B[k * D + j];
        if (CONJ) b.im = -b.im;
        return b;
    };
    cd cur[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        c[j] = czero();
        cur[j] = ld(0, j);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        cd nxt[D];
        if (k + 1 < D) {
#pragma unroll
            for (int j = 0; j < D; ++j) nxt[j] = ld(k + 1, j);
        }
        const cd ak = a[k];
#pragma unroll
        for (int j = 0; j < D; ++j) cmac(c[j], ak, cur[j]);
        if (k + 1 < D) {
#pragma unroll
            for (int j = 0; j < D; ++j) cur[j] = nxt[j];
        }
    }
    pin<D>(c);
}

// Group-wide sum / max of one double per lane (all lanes receive the result).
template <int D>
__device__ __forceinline__ double group_sum(Group<D> &G, double v, bool wr) {
    double *s = G.auxd();
    if (wr) s[G.i] = v;
    gsync();
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < D; ++r) t += s[r];
    gsync();
    return t;
}
template <int D>
__device__ __forceinline__ double group_max(Group<D> &G, double v, bool wr) {
    double *s = G.auxd();
    if (wr) s[G.i] = v;
    gsync();
    double t = s[0];
#pragma unroll
    for (int r = 1; r < D; ++r) t = fmax(t, s[r]);
    gsync();
    return t;
}

// Group-wide "any" through the wave ballot (no LDS traffic).  A lane outside
// every group (lane 63 when D does not divide 64) sees the last group's answer.
template <int D>
__device__ __forceinline__ bool group_any(const Group<D> &G, bool pred) {
    const unsigned long long m = __ballot(pred ? 1 : 0);
    const unsigned long long gm = ((1ull << D) - 1ull) << (G.g * D);
    return (m & gm) != 0ull;
}

// Lane i holds column i of a matrix -> lane i holds row i (and vice versa).
template <int D>
__device__ __forceinline__ void transpose_group(Group<D> &G, cd (&v)[D], bool wr) {
    if (wr) {
#pragma unroll
        for (int r = 0; r < D; ++r) G.tile[r * D + G.i] = v[r];
    }
    gsync();
#pragma unroll
    for (int c = 0; c < D; ++c) v[c] = G.tile[G.i * D + c];
    gsync();
}

// ---------------------------------------------------------------------------
// Pade tables (Julia LinearAlgebra.exp!)
// ---------------------------------------------------------------------------
__constant__ const double kPade3[4] = {120.0, 60.0, 12.0, 1.0};
__constant__ const double kPade5[6] = {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0};
__constant__ const double kPade7[8] = {17297280.0, 8648640.0, 1995840.0, 277200.0,
                                       25200.0, 1512.0, 56.0, 1.0};
__constant__ const double kPade9[10] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0,
                                        30270240.0, 2162160.0, 110880.0, 3960.0, 90.0, 1.0};
__constant__ const double kPade13[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                                         1187353796428800.0, 129060195264000.0, 10559470521600.0,
                                         670442572800.0, 33522128640.0, 1323241920.0,
                                         40840800.0, 960960.0, 16380.0, 182.0, 1.0};

// Degree choice of exp! for a 1-norm: returns m, writes s (squarings).
__device__ __forceinline__ int pade_degree(double nA, int &s) {
    s = 0;
    if (nA <= 2.1) {
        if (nA > 0.95) return 9;
        if (nA > 0.25) return 7;
        if (nA > 0.015) return 5;
        return 3;
    }
    const double l = log2(nA / 5.4);
    if (l > 0.0) s = (int)ceil(l);
    return 13;
}

// ---------------------------------------------------------------------------
// gesv(Y, X): solve Y Z = X in place (Z returned in x), LAPACK semantics
// (zgetrf partial pivoting + zgetrs).  General path with row interchanges.
// On return lane i holds row `pos` of the solution (pos returned).
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ int gesv_rows_pivot(Group<D> &G, cd (&y)[D], cd (&x)[D], bool wr, int &singular) {
    int pos = G.i;  // physical row position of the row this lane holds
    double *red = G.auxd();
    cd *prow = G.tile;  // pivot row broadcast: y part [0,D), x part [D,2D)
#pragma unroll
    for (int j = 0; j < D; ++j) {
        __builtin_amdgcn_sched_barrier(0);
        // izamax over positions j..D-1 with |re|+|im|; first (smallest position) max wins
        const double v = (pos >= j) ? (fabs(y[j].re) + fabs(y[j].im)) : -1.0;
        if (wr) {
            red[2 * G.i] = v;
            red[2 * G.i + 1] = (double)pos;
        }
        gsync();
        double best = -1.0;
        int bpos = D;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const double vr = red[2 * r];
            const int pr = (int)red[2 * r + 1];
            if (vr > best || (vr == best && pr < bpos)) {
                best = vr;
                bpos = pr;
            }
        }
        gsync();
        if (pos == bpos) pos = j;
        else if (pos == j) pos = bpos;
        if (best == 0.0) singular = 1;
        if (pos == j && wr) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) {
                prow[jj] = y[jj];
                prow[D + jj] = x[jj];
            }
        }
        gsync();
        if (pos > j && best != 0.0) {
            const cd piv = prow[j];
            const cd rp = cdiv(cmake(1.0, 0.0), piv);
            const cd l = cmul(y[j], rp);
            y[j] = l;
#pragma unroll
            for (int jj = j + 1; jj < D; ++jj) {
                const cd u = prow[jj];
                y[jj] = cadd(y[jj], cmul(l, cmake(-u.re, -u.im)));
            }
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = csub(x[jj], cmul(prow[D + jj], l));
        }
        gsync();
    }
    // back substitution (ztrsm, upper, non-unit)
#pragma unroll
    for (int k = D - 1; k >= 0; --k) {
        __builtin_amdgcn_sched_barrier(0);
        if (pos == k) {
            const cd piv = y[k];
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = cdiv(x[jj], piv);
            if (wr) {
#pragma unroll
                for (int jj = 0; jj < D; ++jj) prow[jj] = x[jj];
            }
        }
        gsync();
        if (pos < k) {
            const cd u = y[k];
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = csub(x[jj], cmul(prow[jj], u));
        }
        gsync();
    }
    return pos;
}

// Interchange-free elimination, used when partial pivoting provably never
// swaps rows.  Sufficient condition (checked by gesv_cols): every column of
// Y is diagonally dominant with margin r = 3/2 > sqrt(2),
//     |y_jj| >= r * sum_{i != j} |y_ij|.
// Margin-r column dominance is inherited by every Schur complement (the
// excess |a_jj| - r*sum|a_ij| cannot decrease under one elimination step when
// the pivot column is itself margin-r dominant), so at every step the
// diagonal modulus exceeds sqrt(2) times any sub-diagonal modulus, and since
// |z| <= |re z| + |im z| <= sqrt(2)|z|, izamax's |re|+|im| metric picks the
// diagonal too: the pivoted algorithm would perform this same elimination.
// Pade denominators for |A|_1 <= 0.25 (m <= 5) have margin ~7.
//
// Arithmetic (rounding-level differences from zgetrf/zgetrs, all within T0):
//   fused complex multiply-adds (4 FMAs), the pivot reciprocal as
//   conj(p)/|p|^2 (zgetf2 scales the column by it), back substitution
//   multiplying by the reciprocal diagonal instead of dividing (ztrsm).
__device__ __forceinline__ cd crecip(cd z) {
    const double s = 1.0 / fma(z.re, z.re, z.im * z.im);
    return cmake(z.re * s, -z.im * s);
}
// c -= a*b (fused)
__device__ __forceinline__ void cmsub(cd &c, cd a, cd b) {
    c.re = fma(-a.re, b.re, c.re);
    c.re = fma(a.im, b.im, c.re);
    c.im = fma(-a.re, b.im, c.im);
    c.im = fma(-a.im, b.re, c.im);
}

// Column-distributed Y Z = X (lane i: column i of Y and of X; returns column i
// of Z in x).  Step p: the pivot lane publishes the multipliers l_q = y_qp/y_pp
// (q > p); every lane applies them to rows q > p of its Y and X columns (the
// forward substitution rides along).  Lanes left of p only touch L entries no
// one reads again, so no lane masking is needed.  Then every lane publishes
// its U column once (reciprocal on the diagonal) and back-substitutes its own
// X column without further synchronisation.
template <int D>
__device__ __forceinline__ void gesv_cols_nopivot(Group<D> &G, cd (&y)[D], cd (&x)[D], bool wr) {
    // (all loops have constant bounds so that full unrolling leaves no
    // dynamically indexed register array behind)
    const int i = G.i;
#pragma unroll
    for (int p = 0; p < D - 1; ++p) {
        cd *l = G.aux + (p & 1) * D;  // alternating broadcast buffers: one barrier per step
        if (i == p && wr) {
            const cd r = crecip(y[p]);
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (q > p) l[q] = cmulf(y[q], r);
        }
        gsync();
#pragma unroll
        for (int q = 0; q < D; ++q) {
            if (q > p) {
                const cd lq = l[q];
                cmsub(y[q], lq, y[p]);
                cmsub(x[q], lq, x[p]);
            }
        }
        pin<D>(y);
        pin<D>(x);
    }
    cd dg = czero();
#pragma unroll
    for (int q = 0; q < D; ++q)
        if (q == i) dg = y[q];
    const cd rd = crecip(dg);
    if (wr) {
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const bool d = q == i;  // (value selects: an lvalue ?: would force y onto the stack)
            G.tile[i * D + q] = cmake(d ? rd.re : y[q].re, d ? rd.im : y[q].im);
        }
    }
    gsync();
#pragma unroll
    for (int k = D - 1; k >= 0; --k) {
        x[k] = cmulf(x[k], G.tile[k * D + k]);
#pragma unroll
        for (int q = 0; q < D; ++q)
            if (q < k) cmsub(x[q], G.tile[k * D + q], x[k]);
    }
    gsync();
}

// Put row `pos` of a distributed matrix back on lane `pos` (via the tile).
template <int D>
__device__ __forceinline__ void regather_rows(Group<D> &G, cd (&x)[D], int pos, bool wr) {
    if (wr) {
#pragma unroll
        for (int j = 0; j < D; ++j) G.tile[pos * D + j] = x[j];
    }
    gsync();
#pragma unroll
    for (int j = 0; j < D; ++j) x[j] = G.tile[G.i * D + j];
    gsync();
}

// Solve Y Z = X, column-distributed in and out.
template <int D>
__device__ __forceinline__ void gesv_cols(Group<D> &G, cd (&y)[D], cd (&x)[D], bool wr, int &singular) {
    const int i = G.i;
    // sufficient, sqrt-free form of the margin test (own column, no communication):
    // |y_ii| >= max(|re|,|im|) and |y_qi| <= |re|+|im| (looser by at most 2x;
    // Pade denominators pass by ~3.5x)
    double off = 0.0, dgm = 0.0;
#pragma unroll
    for (int q = 0; q < D; ++q) {
        const double m1 = fabs(y[q].re) + fabs(y[q].im);
        const double mx = fmax(fabs(y[q].re), fabs(y[q].im));
        off += (q == i) ? 0.0 : m1;
        dgm = (q == i) ? mx : dgm;
    }
    const bool dominant = dgm >= 1.5 * off && dgm > 0.0;  // false on NaN
    if (!group_any(G, wr && !dominant)) {
        gesv_cols_nopivot<D>(G, y, x, wr);
    } else {  // general path: partial pivoting on the row-distributed system
        transpose_group<D>(G, y, wr);
        transpose_group<D>(G, x, wr);
        const int pos = gesv_rows_pivot<D>(G, y, x, wr, singular);
        regather_rows<D>(G, x, pos, wr);
        transpose_group<D>(G, x, wr);
    }
}

// ---------------------------------------------------------------------------
// expm of the group's matrix (column form: a = this lane's COLUMN of A, x
// returns this lane's column of exp(A)).
//
// expm_prologue: Julia's isdiag fast path and the 1-norm -> (m, s) choice.
// expm_low:      m in {3, 5} with at most three row-matrices live in VGPRs
//                (A2, A4 and an accumulator); the row of A is REBUILT by the
//                caller-supplied `reload` for the final U = A*U' product
//                instead of being kept alive -- A is cheap to rebuild from
//                the operator basis, registers are not.
// expm_high:     m in {7, 9, 13} (+ squarings), generous registers; runs in a
//                separate kernel so its pressure does not cap the main one.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ int expm_prologue(Group<D> &G, const cd (&a)[D], cd (&x)[D], bool wr, int &s_out) {
    const int i = G.i;
    bool off = false;
    double cs = 0.0;  // this column's 1-norm (Julia: sum of abs over rows, in order)
#pragma unroll
    for (int j = 0; j < D; ++j) {
        if (j != i && (a[j].re != 0.0 || a[j].im != 0.0)) off = true;
        cs += sqrt(a[j].re * a[j].re + a[j].im * a[j].im);
    }
    s_out = 0;
    if (!group_any(G, wr && off)) {  // isdiag(A): exp of the diagonal
        cd aii = czero();
#pragma unroll
        for (int j = 0; j < D; ++j)
            if (j == i) aii = a[j];
        const double e = exp(aii.re);
        const double sn = sin(aii.im), cn = cos(aii.im);
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = (j == i) ? cmake(e * cn, e * sn) : czero();
        return 0;
    }
    const double nA = group_max(G, cs, wr);  // opnorm(A, 1)
    return pade_degree(nA, s_out);
}

// Final stage shared by every degree: X = V + U, Y = V - U, gesv(Y, X).
// GENERAL = false skips the dominance test: for m <= 5 the degree choice
// guarantees a finite |A|_1 <= 0.25 (NaN/Inf norms select m = 13), and then
// |y_jj| >= c0 - sum_k c_k |A|^k >= 6.5 * sum_{i != j} |y_ij| (Pade-5
// coefficients), far beyond the sqrt(2) margin partial pivoting needs, so the
// interchange-free elimination IS what zgetrf would do.
template <int D, bool GENERAL>
__device__ __forceinline__ void pade_finish(Group<D> &G, const cd (&v)[D], const cd (&u)[D], cd (&x)[D],
                                            bool wr, int &singular) {
    cd y[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        x[j] = cadd(v[j], u[j]);
        y[j] = csub(v[j], u[j]);
    }
    if (GENERAL) gesv_cols<D>(G, y, x, wr, singular);
    else gesv_cols_nopivot<D>(G, y, x, wr);
}

// ---------------------------------------------------------------------------
// Low-norm regime (Julia's Pade 3 / 5, |A|_1 <= 0.25) without a linear solve.
//
// Julia's exp! evaluates r_m(A) = q_m(A)^-1 p_m(A), whose backward error is below
// u = 2^-53 in this regime (Higham's theta_3 = 0.015, theta_5 = 0.25).  The device
// evaluates the Taylor polynomial of the same accuracy instead: degree 12 for
// |A|_1 <= 0.25 (remainder |A|^13/13! <= 2.4e-18) and degree 6 for |A|_1 <= 0.015
// (<= 3.4e-17).  Both approximants agree with exp(A) -- and with each other -- to a
// few u, inside the T0 tier (1e-13), and both are smooth in A, so the eps-differences
// of the reference keep their u/eps rounding floor.  What the change buys on gfx950:
// no elimination (its per-pivot broadcasts are one-lane VALU work and LDS round
// trips), two tile images in all (A, then A^3) and no rebuild of A.  Products:
// degree 12: A^2, A^3 + 3 Horner steps = 5 (Pade 5: 3 + the LU solve); degree 6: 3.
// Measured (C2, 16 384 evaluations per pass): k_expm_grad 41.5 -> 37.7 ms, C2
// 748k -> 810k evals/s; C3 67.7k -> 76.1k (a Horner-in-A^2 variant with 6 products was
// slower than Pade in k_expm_grad: 47.5 ms).  -DGRAPE_LOW_PADE=1 restores Pade 3 / 5.
// ---------------------------------------------------------------------------
__constant__ const double kInvFact[13] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120, 1.0 / 720,
                                          1.0 / 5040, 1.0 / 40320, 1.0 / 362880, 1.0 / 3628800,
                                          1.0 / 39916800, 1.0 / 479001600};

// Degree choice without square roots: the column sums of |re| + |im| bound the 1-norm
// from above (|z| <= |re| + |im|), so a group whose bound is <= 0.25 is in the low regime
// for sure; only groups above it take the exact norm (Julia's opnorm(A, 1)) and the
// Pade degree of exp!.  Returns 0 (isdiag fast path, x = exp(A) done), 3 (Taylor 6),
// 5 (Taylor 12) or the exact Pade degree > 5 (s_out squarings).
template <int D>
__device__ __forceinline__ int expm_prologue_fast(Group<D> &G, const cd (&a)[D], cd (&x)[D], bool wr, int &s_out) {
    const int i = G.i;
    bool off = false;
    double ub = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        if (j != i && (a[j].re != 0.0 || a[j].im != 0.0)) off = true;
        ub += fabs(a[j].re) + fabs(a[j].im);
    }
    s_out = 0;
    if (!group_any(G, wr && off)) {  // isdiag(A): exp of the diagonal
        cd aii = czero();
#pragma unroll
        for (int j = 0; j < D; ++j)
            if (j == i) aii = a[j];
        const double e = exp(aii.re);
        const double sn = sin(aii.im), cn = cos(aii.im);
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = (j == i) ? cmake(e * cn, e * sn) : czero();
        return 0;
    }
    const double nub = group_max(G, ub, wr);
    if (nub <= 0.015) return 3;
    if (nub <= 0.25) return 5;
    return expm_prologue<D>(G, a, x, wr, s_out);  // exact 1-norm (Julia's degree choice)
}

// Paterson-Stockmeyer with blocks of three: T = B0 + A^3 (B1 + A^3 (B2 + A^3 B3)),
// B_j = c_3j I + c_3j+1 A + c_3j+2 A^2 (B3 also + c12 A^3); degree 6: B0 + A^3 (B1 + c6 A^3).
// Products: A^2, A^3, then 3 (degree 12) or 1 (degree 6) Horner steps with A^3 in the tile.
template <int D, int RING = 0>
__device__ __forceinline__ void expm_taylor(Group<D> &G, int m, const cd (&a)[D], cd (&x)[D], bool wr) {
    const int i = G.i;
    const bool small = m == 3;
    cd a2[D], p[D];
    tile_store_row(G, a, wr);
    gsync();
    mm_tile_r<D, RING>(a, G.tile, a2);  // A^2
    mm_tile_r<D, RING>(a2, G.tile, p);  // A^3
    {
        const int b = small ? 3 : 9;  // top block: c_b I + c_b+1 A + c_b+2 A^2 + c_b+3 A^3
        const double k0 = kInvFact[b], k1 = kInvFact[b + 1], k2 = kInvFact[b + 2], k3 = kInvFact[b + 3];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x[j] = caxpy(k1, a[j], caxpy(k2, a2[j], cscale(k3, p[j])));
            if (j == i) x[j].re += k0;
        }
    }
    gsync();
    tile_store_row(G, p, wr);  // the tile holds A^3 from here on
    gsync();
#pragma unroll
    for (int st = 2; st >= 0; --st) {
        if (st == 0 || !small) {  // group-uniform
            mm_tile_r<D, RING>(x, G.tile, p);
            const double k0 = kInvFact[3 * st], k1 = kInvFact[3 * st + 1], k2 = kInvFact[3 * st + 2];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                x[j] = caxpy(k1, a[j], caxpy(k2, a2[j], p[j]));
                if (j == i) x[j].re += k0;
            }
        }
    }
    gsync();
}

template <int D, class Reload>
__device__ __forceinline__ void expm_low(Group<D> &G, int m, cd (&a)[D], cd (&x)[D], bool wr, int &singular,
                                         Reload reload) {
    const int i = G.i;
    const double *C = (m == 3) ? kPade3 : kPade5;
    cd p[D], q[D];
    // A2 = A*A
    tile_store_row(G, a, wr);
    gsync();
    mm_tile<D>(a, G.tile, p);
    gsync();
    if (m == 5) {
        // A4 = P*A2 with P = I*A2 = A2 (Julia's first loop product is exact)
        tile_store_row(G, p, wr);
        gsync();
        mm_tile<D>(p, G.tile, q);
        gsync();
    }
    // U' = (C1 I + C3 A2) [+ C5 A4],  V = (C0 I + C2 A2) [+ C4 A4]   (Julia's order)
#pragma unroll
    for (int j = 0; j < D; ++j) {  // (fused: rounding-level differences from Julia's order)
        const double du = (j == i) ? C[1] : 0.0, dv = (j == i) ? C[0] : 0.0;
        cd u = cmake(fma(C[3], p[j].re, du), C[3] * p[j].im);
        cd v = cmake(fma(C[2], p[j].re, dv), C[2] * p[j].im);
        if (m == 5) {
            u = caxpy(C[5], q[j], u);
            v = caxpy(C[4], q[j], v);
        }
        p[j] = u;
        q[j] = v;
    }
    // U = A*U'
    tile_store_row(G, p, wr);
    gsync();
    reload(a);
    mm_tile<D>(a, G.tile, p);
    gsync();
    pade_finish<D, false>(G, q, p, x, wr, singular);
}

template <int D>
__device__ __forceinline__ void expm_high(Group<D> &G, int m, int s, cd (&a)[D], cd (&x)[D], bool wr, int &singular) {
    const int i = G.i;
    if (m <= 9) {
        const double *C = m == 3 ? kPade3 : m == 5 ? kPade5 : m == 7 ? kPade7 : kPade9;
        const int half = (m + 1) / 2;
        cd p[D], u[D], v[D], t[D];
        tile_store_row(G, a, wr); gsync(); mm_tile<D>(a, G.tile, p); gsync();
        tile_store_row(G, p, wr); gsync();  // A2 stays in the tile for P *= A2
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const double du = (j == i) ? C[1] : 0.0, dv = (j == i) ? C[0] : 0.0;
            u[j] = cmake(du + C[3] * p[j].re, 0.0 + C[3] * p[j].im);
            v[j] = cmake(dv + C[2] * p[j].re, 0.0 + C[2] * p[j].im);
        }
        for (int kk = 2; kk < half; ++kk) {
            mm_tile<D>(p, G.tile, t);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                p[j] = t[j];
                u[j] = cadd(u[j], cscale(C[2 * kk + 1], p[j]));
                v[j] = cadd(v[j], cscale(C[2 * kk], p[j]));
            }
        }
        gsync();
        tile_store_row(G, u, wr); gsync(); mm_tile<D>(a, G.tile, t); gsync();
        pade_finish<D, true>(G, v, t, x, wr, singular);
        return;
    }
    // m = 13: A /= 2^s, Pade 13, s squarings
    if (s > 0) {
        const double f = ldexp(1.0, s);
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = cmake(a[j].re / f, a[j].im / f);
    }
    const double *C = kPade13;
    cd a2[D], a4[D], a6[D], w[D], u[D], v[D];
    tile_store_row(G, a, wr); gsync(); mm_tile<D>(a, G.tile, a2); gsync();
    tile_store_row(G, a2, wr); gsync(); mm_tile<D>(a2, G.tile, a4); gsync();
    tile_store_row(G, a4, wr); gsync(); mm_tile<D>(a2, G.tile, a6); gsync();
#pragma unroll
    for (int j = 0; j < D; ++j)
        w[j] = cadd(cadd(cscale(C[12], a6[j]), cscale(C[10], a4[j])), cscale(C[8], a2[j]));
    tile_store_row(G, w, wr); gsync(); mm_tile<D>(a6, G.tile, v); gsync();
#pragma unroll
    for (int j = 0; j < D; ++j) {
        v[j] = cadd(cadd(cadd(v[j], cscale(C[6], a6[j])), cscale(C[4], a4[j])), cscale(C[2], a2[j]));
        if (j == i) v[j] = cadd(v[j], cmake(C[0], 0.0));
        w[j] = cadd(cadd(cscale(C[13], a6[j]), cscale(C[11], a4[j])), cscale(C[9], a2[j]));
    }
    tile_store_row(G, w, wr); gsync(); mm_tile<D>(a6, G.tile, u); gsync();
#pragma unroll
    for (int j = 0; j < D; ++j) {
        u[j] = cadd(cadd(cadd(u[j], cscale(C[7], a6[j])), cscale(C[5], a4[j])), cscale(C[3], a2[j]));
        if (j == i) u[j] = cadd(u[j], cmake(C[1], 0.0));
    }
    tile_store_row(G, u, wr); gsync(); mm_tile<D>(a, G.tile, w); gsync();
    pade_finish<D, true>(G, v, w, x, wr, singular);
    for (int r = 0; r < s; ++r) {
        tile_store_row(G, x, wr); gsync(); mm_tile<D>(x, G.tile, w); gsync();
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = w[j];
    }
}

}  // namespace grape
