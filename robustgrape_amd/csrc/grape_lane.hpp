// grape_lane.hpp -- lane-matrix kernels for small d (selected for d <= 3: the Rydberg S = 2
// sector class; grape_launch.hpp kLaneMaxD has the measurement that keeps d = 4 on row groups).
//
// The row-group engine (grape_device.hpp) spreads one matrix over D lanes and moves every
// product operand through LDS behind a workgroup barrier.  At D = 4 / 2 a whole complex
// matrix is 64 / 16 VGPRs, so here ONE LANE OWNS ONE PROPAGATOR: the generator and the
// exponential live in registers, with no LDS, no barrier and no group reduction -- 64
// independent items per wave, each a stream of FMAs.
//
//   k_expm_lane<D, ERR> = k_expm<D, ERR>  (the propagators of every stored variant)
//
// The arithmetic is the row-group kernel's operation for operation: the same Taylor /
// Paterson-Stockmeyer evaluation (expm_taylor), every product element accumulated over the
// inner index in ascending order with the same cmac operand roles (mm_tile_r) -- so E is
// bit-identical to the row-group path (tests/test_gpu_lane.py compares both).  Items with Pade
// degree > 5 are parked in the row-group slot layout (column c of A at slot + c*D) for
// k_expm_high, exactly as park<D> does.
// Measured and dropped: the same treatment for k_expm_grad (eps-variant exp + contraction in
// one lane, E' parked in LDS): bit-identical but slower -- S = 2: 1.69 vs 1.55 ms per pass
// (the contraction's per-lane operand loads are 16-B pieces of different items' tiles), S = 4:
// 5.07 vs 2.90 ms (2 waves/SIMD).
// References: UnitaryCalculations.jl:45 (propagators); the exponential is Julia's exp! (see
// grape_device.hpp).
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

// A = -i dt H of one item (column c from the builder's column-c call).
template <int D, bool ERR>
__device__ __forceinline__ void lane_build(ItemBuilder<D, ERR> &rb, cd (&A)[D][D]) {
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

#ifndef GRAPE_LANE_BLOCK
#define GRAPE_LANE_BLOCK 256
#endif
constexpr int kLaneBlock = GRAPE_LANE_BLOCK;
#ifndef GRAPE_LANE_WAVES
#define GRAPE_LANE_WAVES 2  // waves per SIMD (register budget 512 / 2 = 256 VGPRs)
#endif
constexpr int kLaneWaves = GRAPE_LANE_WAVES;

// Propagators of every stored variant: one item (b, k, v) per lane, E row-major.  ERR selects
// the builder with error terms (every variant of the error-source pipeline), as k_expm<D, ERR>.
template <int D, bool ERR>
__global__ __launch_bounds__(kLaneBlock, kLaneWaves) void k_expm_lane(DevProblem P, DevBatch B) {
    const long nitems = (long)B.nb * P.Nt * P.nv;
    const long gid = (long)blockIdx.x * kLaneBlock + threadIdx.x;
    if (gid >= nitems) return;
    int v, k, b;
    split_item(gid, nitems, P.nv, P.Nt, b, k, v);
    const int ns = P.nsec > 1 ? P.nsec : 1, bx = b / ns;
    const double *xb = B.x + (size_t)bx * P.nx;
    ItemBuilder<D, ERR> rb(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, 0, k + 1, P.vs[v], true,
                           b - bx * ns);
    cd A[D][D], X[D][D];
    lane_build<D, ERR>(rb, A);
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

// Sectors without error sources (one stored variant): one lane per (sub-evaluation b, chunk c)
// walks the chunk's steps, computes E_k (k_expm_lane's arithmetic) and extends the chunk chain
// Q_k = E_k Q_{k-1} (Q = E at the chunk start) in registers -- exactly k_scan's Phase A, element
// (j, i) summed over k in order with cmac(c, Q[k][i], E[j][k]) -- writing E_k and Q_k.  k_scan
// then starts at the chunk totals (B.chains_done) and never streams E for the chains.  A step
// parked for k_expm_high (Pade degree > 5) poisons the rest of its chunk's chain with NaN, and
// k_scan rechains that chunk from E after k_expm_high has filled it in.
// Measured and dropped: the same walk at d = 4 with E re-read through the cache and the chain in
// the lane's LDS slot (A, A^3, E and Q do not fit a lane's registers together): bitwise equal
// but 7.32 ms per pass against 1.95 + 1.86 ms for k_expm<4> + k_scan<4> (2 waves/SIMD, spills).
// Also measured and dropped: nontemporal 16-B stores for E and Q (9.48 vs 1.77-1.91 ms), and
// tighter launch bounds (4 waves/SIMD: 128 VGPRs with spills).
template <int D>
__global__ __launch_bounds__(kLaneBlock, kLaneWaves) void k_expm_chain_lane(DevProblem P, DevBatch B) {
    constexpr int TILE = D * D;
    const long nitems = (long)B.nb * P.nchunks;
    const long gid = (long)blockIdx.x * kLaneBlock + threadIdx.x;
    if (gid >= nitems) return;
    const int b = (int)(gid / P.nchunks), c = (int)(gid - (long)b * P.nchunks);
    const int ns = P.nsec > 1 ? P.nsec : 1, bx = b / ns;
    const double *xb = B.x + (size_t)bx * P.nx;
    cd Q[D][D];
    const int k0 = c * P.L, k1 = min(k0 + P.L, P.Nt);
    for (int k = k0; k < k1; ++k) {
        int sec = b - bx * ns;
        asm volatile("" : "+v"(sec));  // per-step opaque: the operator loads stay inside the step (no LICM)
        ItemBuilder<D, false> rb(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, 0, k + 1, P.vs[0], true,
                                 sec);
        cd A[D][D], X[D][D];
        lane_build<D, false>(rb, A);
        int s = 0;
        const int m = lane_prologue<D>(A, X, s);
        const long item = (long)b * P.Nt + k;  // nv = 1
        cd *out = B.E + (size_t)item * TILE;
        if (m > 5) {
            lane_park<D>(out, A, item, B.overflow, B.overflow_count);
            const double nan = __builtin_nan("");
#pragma unroll
            for (int r = 0; r < D; ++r) {
#pragma unroll
                for (int cc = 0; cc < D; ++cc) X[r][cc] = cmake(nan, nan);
            }
        } else {
            if (m == 3 || m == 5) {
                cd A3[D][D];
                lane_cube<D>(A, A3);
#pragma unroll
                for (int i = 0; i < D; ++i) {
                    cd x[D];
                    lane_taylor_col<D>(m, i, A, A3, x);
#pragma unroll
                    for (int j = 0; j < D; ++j) X[j][i] = x[j];
                }
            }
#pragma unroll
            for (int r = 0; r < D; ++r) {
#pragma unroll
                for (int cc = 0; cc < D; ++cc) out[r * D + cc] = X[r][cc];
            }
        }
        if (k == k0) {
#pragma unroll
            for (int r = 0; r < D; ++r) {
#pragma unroll
                for (int cc = 0; cc < D; ++cc) Q[r][cc] = X[r][cc];
            }
        } else {
#pragma unroll
            for (int i = 0; i < D; ++i) {  // column i of E_k . Q
                cd q[D], t[D];
#pragma unroll
                for (int r = 0; r < D; ++r) q[r] = Q[r][i];
                lane_matvec<D>(X, q, t);
#pragma unroll
                for (int r = 0; r < D; ++r) Q[r][i] = t[r];
            }
        }
        cd *dq = B.Q + (size_t)item * TILE;
#pragma unroll
        for (int r = 0; r < D; ++r) {
#pragma unroll
            for (int cc = 0; cc < D; ++cc) dq[r * D + cc] = Q[r][cc];
        }
    }
}

#else
#define GRAPE_HAVE_LANE 0
#endif

}  // namespace grape
