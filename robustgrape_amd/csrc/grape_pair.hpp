// grape_pair.hpp -- column-PAIR groups for the small-d exponential (register
// blocking against the LDS bandwidth bound).
//
// In the row-group engine (grape_device.hpp) a lane owns ONE column and every
// complex MAC of a product consumes one 16-B LDS broadcast: per CU the LDS
// delivers 128 B/clk = 8 operands/clk while the SIMDs could retire 16 complex
// MACs/clk, so products cap at half of FP64 peak.  Here a lane owns TWO
// columns (2i, 2i+1) of its group's matrix: each LDS read feeds two MACs and a
// wave holds floor(64 / ceil(d/2)) matrices (12 at d = 9, against 7), so the
// LDS traffic per matrix product drops by ~40 %, at twice the registers per
// lane-matrix (two waves per SIMD instead of three).
//
// Same numerics as expm_low (Julia exp!'s Pade 3/5, interchange-free column
// elimination under the proven dominance margin); items with m > 5 are parked
// for k_expm_high exactly like k_expm.  The last lane of an odd-d group
// carries a duplicate of column d-1 in its second slot, which is never stored.
#pragma once
#include "grape_kernels.hpp"

namespace grape {

template <int D>
struct Geo2 {
    static constexpr int L = (D + 1) / 2;           // lanes per group
    static constexpr int GPW = 64 / L;              // groups per wave
    static constexpr int TILE = D * D;
    static constexpr int AUX = 2 * D + 4;           // multipliers (double-buffered) + reductions
    static constexpr int GROUP_CD = TILE + AUX;
};

template <int D>
struct Group2 {
    int i;         // lane in the group: owns columns c0 = 2i, c1 = min(2i + 1, D - 1)
    int g;         // group in the wave
    bool lane_ok;  // lane belongs to a group
    bool has1;     // 2i + 1 < D (the second column is real)
    int c0, c1;
    cd *tile;
    cd *aux;
    __device__ __forceinline__ double *auxd() { return reinterpret_cast<double *>(aux); }
};

template <int D>
__device__ __forceinline__ Group2<D> make_group2(cd *wave_lds, int lane) {
    constexpr int L = Geo2<D>::L, GPW = Geo2<D>::GPW;
    Group2<D> G;
    G.lane_ok = lane < GPW * L;
    G.g = G.lane_ok ? lane / L : GPW - 1;
    G.i = G.lane_ok ? lane % L : 0;
    G.c0 = 2 * G.i;
    G.has1 = 2 * G.i + 1 < D;
    G.c1 = G.has1 ? 2 * G.i + 1 : D - 1;
    G.tile = wave_lds + G.g * Geo2<D>::GROUP_CD;
    G.aux = G.tile + Geo2<D>::TILE;
    return G;
}

template <int D>
__device__ __forceinline__ void tile_store2(Group2<D> &G, const cd (&v0)[D], const cd (&v1)[D], bool wr) {
    if (wr) {
#pragma unroll
        for (int j = 0; j < D; ++j) G.tile[G.c0 * D + j] = v0[j];
        if (G.has1) {
#pragma unroll
            for (int j = 0; j < D; ++j) G.tile[G.c1 * D + j] = v1[j];
        }
    }
}

// c_s = a_s . B for both slots: one LDS read of B[k][j] feeds two complex MACs
template <int D>
__device__ __forceinline__ void mm2(const cd (&a0)[D], const cd (&a1)[D], const cd *B, cd (&c0)[D], cd (&c1)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        c0[j] = czero();
        c1[j] = czero();
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const cd x0 = a0[k], x1 = a1[k];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const cd b = B[k * D + j];
            cmac(c0[j], x0, b);
            cmac(c1[j], x1, b);
        }
    }
    pin<D>(c0);
    pin<D>(c1);
}

template <int D>
__device__ __forceinline__ double group_max2(Group2<D> &G, double v, bool wr) {
    double *s = G.auxd() + 2 * (2 * D);  // past the multiplier buffers
    if (wr) s[G.i] = v;
    gsync();
    double t = s[0];
#pragma unroll
    for (int r = 1; r < Geo2<D>::L; ++r) t = fmax(t, s[r]);
    gsync();
    return t;
}

template <int D>
__device__ __forceinline__ bool group_any2(const Group2<D> &G, bool pred) {
    constexpr int L = Geo2<D>::L;
    const unsigned long long m = __ballot(pred ? 1 : 0);
    const unsigned long long gm = ((1ull << L) - 1ull) << (G.g * L);
    return (m & gm) != 0ull;
}

// isdiag fast path and the 1-norm -> (m, s) choice (expm_prologue for pairs)
template <int D>
__device__ __forceinline__ int expm_prologue2(Group2<D> &G, const cd (&a0)[D], const cd (&a1)[D], cd (&x0)[D],
                                              cd (&x1)[D], bool wr, int &s_out) {
    bool off = false;
    double cs0 = 0.0, cs1 = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        if (j != G.c0 && (a0[j].re != 0.0 || a0[j].im != 0.0)) off = true;
        if (G.has1 && j != G.c1 && (a1[j].re != 0.0 || a1[j].im != 0.0)) off = true;
        cs0 += sqrt(a0[j].re * a0[j].re + a0[j].im * a0[j].im);
        cs1 += sqrt(a1[j].re * a1[j].re + a1[j].im * a1[j].im);
    }
    s_out = 0;
    if (!group_any2(G, wr && off)) {  // isdiag(A): exp of the diagonal
        cd d0 = czero(), d1 = czero();
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (j == G.c0) d0 = a0[j];
            if (j == G.c1) d1 = a1[j];
        }
        const double e0 = exp(d0.re), e1 = exp(d1.re);
        const cd z0 = cmake(e0 * cos(d0.im), e0 * sin(d0.im)), z1 = cmake(e1 * cos(d1.im), e1 * sin(d1.im));
#pragma unroll
        for (int j = 0; j < D; ++j) {
            x0[j] = (j == G.c0) ? z0 : czero();
            x1[j] = (j == G.c1) ? z1 : czero();
        }
        return 0;
    }
    const double nA = group_max2(G, fmax(cs0, G.has1 ? cs1 : 0.0), wr);  // opnorm(A, 1)
    return pade_degree(nA, s_out);
}

// Y Z = X without interchanges (columns of Y and X distributed two per lane;
// see gesv_cols_nopivot for the algorithm and the dominance argument)
template <int D>
__device__ __forceinline__ void gesv_pairs_nopivot(Group2<D> &G, cd (&y0)[D], cd (&y1)[D], cd (&x0)[D],
                                                   cd (&x1)[D], bool wr) {
#pragma unroll
    for (int p = 0; p < D - 1; ++p) {
        cd *l = G.aux + (p & 1) * D;
        if (G.i == (p >> 1) && wr) {  // owner of column p publishes the multipliers
            const bool s1 = p & 1;
            cd piv = czero();
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (q == p) piv = s1 ? y1[q] : y0[q];
            const cd r = crecip(piv);
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (q > p) l[q] = cmulf(s1 ? y1[q] : y0[q], r);
        }
        gsync();
#pragma unroll
        for (int q = 0; q < D; ++q) {
            if (q > p) {
                const cd lq = l[q];
                cmsub(y0[q], lq, y0[p]);
                cmsub(y1[q], lq, y1[p]);
                cmsub(x0[q], lq, x0[p]);
                cmsub(x1[q], lq, x1[p]);
            }
        }
        pin<D>(y0);
        pin<D>(y1);
        pin<D>(x0);
        pin<D>(x1);
    }
    // publish U columns (reciprocal on the diagonal), then back-substitute both X columns
    cd dg0 = czero(), dg1 = czero();
#pragma unroll
    for (int q = 0; q < D; ++q) {
        if (q == G.c0) dg0 = y0[q];
        if (q == G.c1) dg1 = y1[q];
    }
    const cd rd0 = crecip(dg0), rd1 = crecip(dg1);
    if (wr) {
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const bool d = q == G.c0;
            G.tile[G.c0 * D + q] = cmake(d ? rd0.re : y0[q].re, d ? rd0.im : y0[q].im);
        }
        if (G.has1) {
#pragma unroll
            for (int q = 0; q < D; ++q) {
                const bool d = q == G.c1;
                G.tile[G.c1 * D + q] = cmake(d ? rd1.re : y1[q].re, d ? rd1.im : y1[q].im);
            }
        }
    }
    gsync();
#pragma unroll
    for (int k = D - 1; k >= 0; --k) {
        const cd ukk = G.tile[k * D + k];
        x0[k] = cmulf(x0[k], ukk);
        x1[k] = cmulf(x1[k], ukk);
#pragma unroll
        for (int q = 0; q < D; ++q)
            if (q < k) {
                const cd u = G.tile[k * D + q];
                cmsub(x0[q], u, x0[k]);
                cmsub(x1[q], u, x1[k]);
            }
    }
    gsync();
}

// Pade 3/5 for a column pair (expm_low's stages); reload(c, a) rebuilds column c of A
template <int D, class Reload>
__device__ __forceinline__ void expm_low2(Group2<D> &G, int m, cd (&a0)[D], cd (&a1)[D], cd (&x0)[D], cd (&x1)[D],
                                          bool wr, Reload reload) {
    const double *C = (m == 3) ? kPade3 : kPade5;
    cd p0[D], p1[D], q0[D], q1[D];
    tile_store2(G, a0, a1, wr);  // A2 = A*A
    gsync();
    mm2<D>(a0, a1, G.tile, p0, p1);
    gsync();
    if (m == 5) {  // A4 = A2*A2
        tile_store2(G, p0, p1, wr);
        gsync();
        mm2<D>(p0, p1, G.tile, q0, q1);
        gsync();
    }
    // U' = (C1 I + C3 A2) [+ C5 A4],  V = (C0 I + C2 A2) [+ C4 A4]
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const double du0 = (j == G.c0) ? C[1] : 0.0, dv0 = (j == G.c0) ? C[0] : 0.0;
        const double du1 = (j == G.c1) ? C[1] : 0.0, dv1 = (j == G.c1) ? C[0] : 0.0;
        cd u0 = cmake(fma(C[3], p0[j].re, du0), C[3] * p0[j].im);
        cd v0 = cmake(fma(C[2], p0[j].re, dv0), C[2] * p0[j].im);
        cd u1 = cmake(fma(C[3], p1[j].re, du1), C[3] * p1[j].im);
        cd v1 = cmake(fma(C[2], p1[j].re, dv1), C[2] * p1[j].im);
        if (m == 5) {
            u0 = caxpy(C[5], q0[j], u0);
            v0 = caxpy(C[4], q0[j], v0);
            u1 = caxpy(C[5], q1[j], u1);
            v1 = caxpy(C[4], q1[j], v1);
        }
        p0[j] = u0;
        q0[j] = v0;
        p1[j] = u1;
        q1[j] = v1;
    }
    // U = A*U' (U' commutes with A: the tile holds U', the registers A's columns)
    tile_store2(G, p0, p1, wr);
    gsync();
    reload(G.c0, a0);
    reload(G.c1, a1);
    mm2<D>(a0, a1, G.tile, p0, p1);
    gsync();
    // X = V + U, Y = V - U, solve Y Z = X
#pragma unroll
    for (int j = 0; j < D; ++j) {
        x0[j] = cadd(q0[j], p0[j]);
        x1[j] = cadd(q1[j], p1[j]);
        const cd y0 = csub(q0[j], p0[j]), y1 = csub(q1[j], p1[j]);
        q0[j] = y0;
        q1[j] = y1;
    }
    gesv_pairs_nopivot<D>(G, q0, q1, x0, x1, wr);
}

// Nominal propagators without error sources (the k_expm<D, false> work) in pair form.
template <int D>
__global__ __launch_bounds__(64, 2) void k_expm2(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group2<D> G = make_group2<D>(lds, threadIdx.x);
    const long nitems = (long)B.nb * P.Nt * P.nv;
    const long gid = (long)blockIdx.x * Geo2<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    const int v = (int)(gidc % P.nv);
    const int k = (int)((gidc / P.nv) % P.Nt);
    const int b = (int)(gidc / ((long)P.nv * P.Nt));
    const double *xb = B.x + (size_t)b * P.nx;
    ItemBuilder<D, false> rebuild(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, G.c0, k + 1, P.vs[v], valid);
    auto reload = [&](int col, cd (&a)[D]) {
        rebuild.i = col;
        rebuild(a);
    };
    cd a0[D], a1[D], x0[D], x1[D];
    reload(G.c0, a0);
    reload(G.c1, a1);
    int s = 0;
    const int m = expm_prologue2<D>(G, a0, a1, x0, x1, valid, s);
    cd *base = B.E + (size_t)gidc * D * D;
    if (m > 5) {  // group-uniform: A (columns) to the slot, exp'd by k_expm_high
        if (valid) {
#pragma unroll
            for (int j = 0; j < D; ++j) base[G.c0 * D + j] = a0[j];
            if (G.has1) {
#pragma unroll
                for (int j = 0; j < D; ++j) base[G.c1 * D + j] = a1[j];
            }
            if (G.i == 0) B.overflow[atomicAdd(B.overflow_count, 1)] = (int)gid;
        }
        return;
    }
    if (m == 3 || m == 5) expm_low2<D>(G, m, a0, a1, x0, x1, valid, reload);
    if (valid) {  // E row-major: column c at stride D
#pragma unroll
        for (int j = 0; j < D; ++j) base[j * D + G.c0] = x0[j];
        if (G.has1) {
#pragma unroll
            for (int j = 0; j < D; ++j) base[j * D + G.c1] = x1[j];
        }
    }
}

}  // namespace grape
