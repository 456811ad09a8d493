// grape_lane.hpp -- lane-matrix kernels for small d (selected for d <= 3: the Rydberg S = 2
// sector class; grape_launch.hpp kLaneMaxD has the measurement that keeps d = 4 on row groups).
//
// The row-group engine (grape_device.hpp) spreads one matrix over D lanes and moves every
// product operand through LDS behind a workgroup barrier.  At D = 4 / 2 a whole complex
// matrix is 64 / 16 VGPRs, so here ONE LANE OWNS ONE ITEM: the generator, the exponential and
// the gradient contraction live in registers, with no LDS, no barrier and no group
// reduction -- 64 independent items per wave, each a stream of FMAs.
//
//   k_expm_lane       = k_expm<D, false>  (nominal propagators, no error sources)
//   k_expm_grad_lane  = k_expm_grad<D>    (eps-variant exp + contraction, no error sources)
//
// The arithmetic is the row-group kernels' operation for operation: the same Taylor /
// Paterson-Stockmeyer evaluation (expm_taylor), every product element accumulated over the
// inner index in ascending order with the same cmac operand roles (mm_tile_r), the same
// contraction (grad_kernel_col / grad_store) and the same lane-ordered sum (group_sum) -- so
// results are bit-identical to the row-group path (tests/test_gpu_lane.py compares both).
// Items with Pade degree > 5 are parked in the row-group slot layout (column c of A at
// slot + c*D) for k_expm_high / k_grad_high, exactly as park<D> does.
// References: UnitaryCalculations.jl:45,51 (propagators), FidelityCalculations.jl:56-76
// (gradient); the exponential is Julia's exp! (see grape_device.hpp).
#pragma once
#include "grape_kernels.hpp"

namespace grape {

#if !(defined(GRAPE_LOW_PADE) && GRAPE_LOW_PADE)
#define GRAPE_HAVE_LANE 1

// out = X . v for one column v; element j sums k = 0..D-1 in order with cmac(c, v[k], X[j][k]) --
// the operand roles of mm_tile_r(column v, tile = X^T) in the column-form exponential.
template <int D>
__device__ __forceinline__ void lane_matvec(const cd (&X)[D][D], const cd (&v)[D], cd (&out)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        cd c = czero();
#pragma unroll
        for (int k = 0; k < D; ++k) cmac(c, v[k], X[j][k]);
        out[j] = c;
    }
}

// Materialise a register matrix (grape_device.hpp pin): keeps the straight-line product chains
// from being interleaved across stages, which would multiply the live registers.
template <int D>
__device__ __forceinline__ void lane_pin(cd (&M)[D][D]) {
#pragma unroll
    for (int r = 0; r < D; ++r) pin<D>(M[r]);
    __builtin_amdgcn_sched_barrier(0);
}

// A = -i dt H of one item (column c from the builder's column-c call).
template <int D>
__device__ __forceinline__ void lane_build(ItemBuilder<D, false> &rb, cd (&A)[D][D]) {
#pragma unroll
    for (int c = 0; c < D; ++c) {
        cd col[D];
        rb.i = c;
        rb(col);
#pragma unroll
        for (int j = 0; j < D; ++j) A[j][c] = col[j];
        pin<D>(col);
        __builtin_amdgcn_sched_barrier(0);  // one column's operator loads at a time
    }
}

// expm_prologue_fast for a whole matrix: 0 (isdiag, X = exp(A) done), 3 / 5 (Taylor 6 / 12)
// or the exact Pade degree > 5 with s squarings.
template <int D>
__device__ __forceinline__ int lane_prologue(const cd (&A)[D][D], cd (&X)[D][D], int &s) {
    bool off = false;
    double nub = 0.0;
#pragma unroll
    for (int c = 0; c < D; ++c) {
        double ub = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (j != c && (A[j][c].re != 0.0 || A[j][c].im != 0.0)) off = true;
            ub += fabs(A[j][c].re) + fabs(A[j][c].im);
        }
        nub = c == 0 ? ub : fmax(nub, ub);
    }
    s = 0;
    if (!off) {
#pragma unroll
        for (int c = 0; c < D; ++c) {
            const double e = exp(A[c][c].re);
            const double sn = sin(A[c][c].im), cn = cos(A[c][c].im);
#pragma unroll
            for (int j = 0; j < D; ++j) X[j][c] = (j == c) ? cmake(e * cn, e * sn) : czero();
        }
        return 0;
    }
    if (nub <= 0.015) return 3;
    if (nub <= 0.25) return 5;
    double nA = 0.0;  // Julia's opnorm(A, 1): column sums of |a| in row order, max over columns
#pragma unroll
    for (int c = 0; c < D; ++c) {
        double cs = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) cs += sqrt(A[j][c].re * A[j][c].re + A[j][c].im * A[j][c].im);
        nA = c == 0 ? cs : fmax(nA, cs);
    }
    return pade_degree(nA, s);
}

// expm_taylor column by column.  A complex D x D matrix is 4*D*D VGPRs (64 at D = 4), so the
// whole-matrix form (A, A^2, A^3, X live) would not fit a lane's budget.  Every column of the
// evaluation reads only the same column of A^2 and of the running polynomial, so the lane keeps
// A and A^3 and regenerates column i of A^2 (one mat-vec) when it works on column i:
//   A^3 e_i = A (A (A e_i)),   X e_i <- A^3 (X e_i) + c_0 e_i + c_1 A e_i + c_2 A^2 e_i.
template <int D>
__device__ __forceinline__ void lane_col(const cd (&A)[D][D], int i, cd (&v)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = A[j][i];
}
template <int D>
__device__ __forceinline__ void lane_cube(const cd (&A)[D][D], cd (&A3)[D][D]) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
        cd a[D], a2[D], a3[D];
        lane_col<D>(A, i, a);
        lane_matvec<D>(A, a, a2);   // A^2 e_i
        lane_matvec<D>(A, a2, a3);  // A^3 e_i = A . A^2 e_i  (the row-group A . A2)
#pragma unroll
        for (int j = 0; j < D; ++j) A3[j][i] = a3[j];
        __builtin_amdgcn_sched_barrier(0);
    }
}
// column i of the Taylor polynomial (degree 12 for m = 5, degree 6 for m = 3)
template <int D>
__device__ __forceinline__ void lane_taylor_col(int m, int i, const cd (&A)[D][D], const cd (&A3)[D][D],
                                                cd (&x)[D]) {
    const bool small = m == 3;
    cd a[D], a2[D], t[D];
    lane_col<D>(A, i, a);
    lane_matvec<D>(A, a, a2);
    {
        const int b = small ? 3 : 9;  // top block: c_b I + c_b+1 A + c_b+2 A^2 + c_b+3 A^3
        const double k0 = kInvFact[b], k1 = kInvFact[b + 1], k2 = kInvFact[b + 2], k3 = kInvFact[b + 3];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x[j] = caxpy(k1, a[j], caxpy(k2, a2[j], cscale(k3, A3[j][i])));
            if (j == i) x[j].re += k0;
        }
    }
#pragma unroll
    for (int st = 2; st >= 0; --st) {
        if (st == 0 || !small) {
            lane_matvec<D>(A3, x, t);
            const double k0 = kInvFact[3 * st], k1 = kInvFact[3 * st + 1], k2 = kInvFact[3 * st + 2];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                x[j] = caxpy(k1, a[j], caxpy(k2, a2[j], t[j]));
                if (j == i) x[j].re += k0;
            }
        }
    }
    pin<D>(x);
    __builtin_amdgcn_sched_barrier(0);
}

// park<D>'s slot layout: column c of A at slot + c*D.
template <int D>
__device__ __forceinline__ void lane_park(cd *slot, const cd (&A)[D][D], long gid, int *list, int *count) {
#pragma unroll
    for (int c = 0; c < D; ++c) {
#pragma unroll
        for (int j = 0; j < D; ++j) slot[c * D + j] = A[j][c];
    }
    list[atomicAdd(count, 1)] = (int)gid;
}

template <int D>
__device__ __forceinline__ void lane_load(const cd *src, cd (&M)[D][D]) {  // row-major
#pragma unroll
    for (int r = 0; r < D; ++r) {
#pragma unroll
        for (int c = 0; c < D; ++c) M[r][c] = src[r * D + c];
    }
}

constexpr int kLaneBlock = 256;
#ifndef GRAPE_LANE_WAVES
#define GRAPE_LANE_WAVES 2  // waves per SIMD (register budget 512 / 2 = 256 VGPRs)
#endif
constexpr int kLaneWaves = GRAPE_LANE_WAVES;
constexpr int kLaneGradBlock = 128;  // k_expm_grad_lane: 128 lanes x (D*D + 1) x 16 B of LDS per block
template <int D>
constexpr size_t lane_grad_lds() { return (size_t)kLaneGradBlock * (D * D + 1) * sizeof(cd); }

// Nominal propagators (ne = 0): one item (b, k, v) per lane, E row-major.
template <int D>
__global__ __launch_bounds__(kLaneBlock, kLaneWaves) void k_expm_lane(DevProblem P, DevBatch B) {
    const long nitems = (long)B.nb * P.Nt * P.nv;
    const long gid = (long)blockIdx.x * kLaneBlock + threadIdx.x;
    if (gid >= nitems) return;
    int v, k, b;
    split_item(gid, nitems, P.nv, P.Nt, b, k, v);
    const int ns = P.nsec > 1 ? P.nsec : 1, bx = b / ns;
    const double *xb = B.x + (size_t)bx * P.nx;
    ItemBuilder<D, false> rb(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, 0, k + 1, P.vs[v], true,
                             b - bx * ns);
    cd A[D][D], X[D][D];
    lane_build<D>(rb, A);
    int s = 0;
    const int m = lane_prologue<D>(A, X, s);
    cd *out = B.E + (size_t)gid * D * D;
    if (m > 5) {
        lane_park<D>(out, A, gid, B.overflow, B.overflow_count);
        return;
    }
    if (m == 3 || m == 5) {
        cd A3[D][D];
        lane_cube<D>(A, A3);
#pragma unroll
        for (int i = 0; i < D; ++i) {  // column i straight to E (row-major)
            cd x[D];
            lane_taylor_col<D>(m, i, A, A3, x);
#pragma unroll
            for (int j = 0; j < D; ++j) out[j * D + i] = x[j];
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < D; ++r) {
#pragma unroll
        for (int c = 0; c < D; ++c) out[r * D + c] = X[r][c];
    }
}

// eps-variant exponential + contraction (ne = 0): one item (b, k, u) per lane.
//   Y = Q_{k-1} M'_c Q_k^dag (Q_{k-1} = I at a chunk start), F_dx term = Re sum_ij Y_ij dE_ji.
template <int D>
__global__ __launch_bounds__(kLaneGradBlock, kLaneWaves) void k_expm_grad_lane(DevProblem P, DevBatch B) {
    constexpr int TILE = D * D;
    const int nvg = P.np + (P.xadd_dep ? P.na : 0);
    const long nitems = (long)B.nb * P.Nt * nvg;
    const long gid = (long)blockIdx.x * kLaneGradBlock + threadIdx.x;
    if (gid >= nitems) return;
    int u, k, b;
    split_item(gid, nitems, nvg, P.Nt, b, k, u);
    const int ns = P.nsec > 1 ? P.nsec : 1, bx = b / ns;
    const double *xb = B.x + (size_t)bx * P.nx;
    ItemBuilder<D, false> rb(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, 0, k + 1, P.vs[P.off_dx + u],
                             true, b - bx * ns);
    cd A[D][D], X[D][D];
    lane_build<D>(rb, A);
    int s = 0;
    const int m = lane_prologue<D>(A, X, s);
    if (m > 5) {
        lane_park<D>(B.ovf2_slots + (size_t)gid * TILE, A, gid, B.ovf2, B.ovf2_count);
        return;
    }
    // E' parks in this lane's LDS slot (column-major, padded: lanes 16 B apart in the bank map),
    // so the exponential (A, A^3 live) and the contraction (M'_c live) never hold it in VGPRs.
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *Xs = reinterpret_cast<cd *>(smem_raw) + (size_t)threadIdx.x * (TILE + 1);
    if (m == 3 || m == 5) {
        cd A3[D][D];
        lane_cube<D>(A, A3);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            cd x[D];
            lane_taylor_col<D>(m, i, A, A3, x);
#pragma unroll
            for (int j = 0; j < D; ++j) Xs[i * D + j] = x[j];
        }
    } else {
#pragma unroll
        for (int i = 0; i < D; ++i) {
#pragma unroll
            for (int j = 0; j < D; ++j) Xs[i * D + j] = X[j][i];
        }
    }
    // contraction (grad_kernel_col's operand roles, lane-ordered sum of grad_store)
    const int c = k / P.L, j0 = k - c * P.L;
    __builtin_amdgcn_sched_barrier(0);  // operand loads after the exponential (registers)
    const cd *Qk = B.Q + ((size_t)b * P.Nt + k) * TILE;
    const cd *E0 = B.E + ((size_t)b * P.Nt + k) * P.nv * TILE;
    const cd *Mcp = B.Mc + ((size_t)b * P.nchunks + c) * TILE;
    cd Mp[D][D];
    lane_load<D>(Mcp, Mp);
    double sum = 0.0;
#pragma unroll 1
    for (int i = 0; i < D; ++i) {  // row i of Y = lane i of the row group (a rolled loop: one
        const cd *Qr = Qk, *Er = E0;  // row's temporaries live at a time)
        cd t[D];
        if (j0 > 0) {
            cd qm[D];
#pragma unroll
            for (int q = 0; q < D; ++q) qm[q] = Qr[(size_t)i * D + q - TILE];  // row i of Q_{k-1}
#pragma unroll
            for (int j = 0; j < D; ++j) {
                cd acc = czero();
#pragma unroll
                for (int q = 0; q < D; ++q) cmac(acc, qm[q], Mp[q][j]);
                t[j] = acc;
            }
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) t[j] = Mcp[i * D + j];  // (row i from memory: no dynamic index into VGPRs)
        }
        double si = 0.0;  // column i of E' and E against row i of Y
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            cd y = czero();  // Y[i][jj] = t . conj(row jj of Q_k)
#pragma unroll
            for (int q = 0; q < D; ++q) cmac(y, t[q], cconj(Qr[jj * D + q]));
            const cd de = cscale(P.inv_eps, csub(Xs[i * D + jj], Er[jj * D + i]));
            si += y.re * de.re - y.im * de.im;
        }
        sum += si;
        __builtin_amdgcn_sched_barrier(0);
    }
    if (B.sec_part) B.sec_part[((size_t)b * P.Nt + k) * nvg + u] = sum;
    else if (u < P.np) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + u] = sum;
    else B.part_add[((size_t)b * P.Nt + k) * P.na + (u - P.np)] = sum;
}

#else
#define GRAPE_HAVE_LANE 0
#endif

}  // namespace grape
