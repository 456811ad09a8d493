// grape_errpath.hpp -- error sources: sensitivities F_d2err and their gradients.
//
// Reference: src/UnitaryCalculations.jl:66-98 (error / mixed propagators),
// :111-151 (cumsum, reverse cumsum, U_derr, U_derr_dx), and
// src/FidelityCalculations.jl:78-113 (F_d2err, F_d2err_dx).
//
// Interaction-picture algebra (C_k = Q_k Carry_c for step k of chunk c,
// C_k^-1 = C_k^dagger):
//   V^err_k = C_k^dag dE^err_k C_{k-1} = Carry_c^dag W_k Carry_c,  W_k = Q_k^dag dE^err_k Q_{k-1}
//   U_derr  = U * Tot,  Tot = sum_k V^err_k                        (UnitaryCalculations.jl:122-123)
//   F_d2err_dx[p,k] = Re tr(G_e U_derr_dx[p,k]),  M_e = G_e U,
//     G_e = 4[P Ue^dag U0 W U0^dag + conj(tau_e) W U0^dag - (1+D) W Ue^dag]/(D(D+1))
//   and with Z1 = Q_k^dag dE^dx Q_{k-1}, Z2 = Q_k^dag dE^mix Q_{k-1},
//     M' = Carry M_e Carry^dag, A_k = Carry S_{k-1} Carry^dag, Ttot = Carry Tot Carry^dag:
//   F_d2err_dx[p,k,e] = Re[ tr(A_k (M' Z1)) + tr((Ttot - A_k - W_k)(Z1 M')) + tr(M' Z2) ]
//   (S_{k-1} = cumsum up to k-1 and R_{k+1} = Tot - S_{k-1} - V_k: :112-113, :124-139).
//
// k_err_scan  one workgroup per (b, e): chunk totals of W, carry transform,
//             additive scan over chunks, U_derr, F_d2err, M_e, per-chunk M', T, Ttot.
// k_err_grad  one row group per (b, chunk, e): walks the chunk's steps, 8 products/step
//             per gradient parameter (controls; x_add too when H0 / Herror read it,
//             U_derr_dx_add being the sum over k of the same per-step terms, :140-151).
#pragma once
#include "grape_kernels.hpp"

namespace grape {

// E-variant row (E_v - E_0) * s  (the reference's (1/eps) * (E' - E))
template <int D>
__device__ __forceinline__ void delta_row(const cd *Ek, int v, int i, double s, cd (&out)[D]) {
    const cd *e0 = Ek + i * D;
    const cd *ev = Ek + (size_t)v * D * D + i * D;
#pragma unroll
    for (int j = 0; j < D; ++j) out[j] = cscale(s, csub(ev[j], e0[j]));
}

// Local-frame transform Z = Q_k^dag X Q_{k-1} (Q_{k-1} = I at a chunk start).
// x: this lane's row of X (destroyed); z: row of Z.  Uses the group tile.
template <int D>
__device__ __forceinline__ void local_frame(Group<D> &G, const cd *Qk, bool first, cd (&x)[D], cd (&z)[D],
                                            bool wr) {
    const int i = G.i;
    tile_store_row(G, x, wr);
    gsync();
    cd l[D];
#pragma unroll
    for (int r = 0; r < D; ++r) l[r] = cconj(Qk[r * D + i]);  // column i of Q_k, conjugated
    mm_tile<D>(l, G.tile, z);
    gsync();
    if (!first) {
        if (wr) {
#pragma unroll
            for (int j = 0; j < D; ++j) G.tile[i * D + j] = Qk[i * D + j - D * D];  // Q_{k-1}
        }
        gsync();
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = z[j];
        mm_tile<D>(x, G.tile, z);
        gsync();
    }
}

// sum_j a[j] * X[j][i] for the tile X (trace helper: tr(A X) = sum_i row_i(A) . col_i(X))
template <int D>
__device__ __forceinline__ cd row_dot_col(const cd (&a)[D], const cd *X, int i) {
    cd s = czero();
#pragma unroll
    for (int j = 0; j < D; ++j) s = cadd(s, cmul(a[j], X[j * D + i]));
    return s;
}

template <int D, int W>
__global__ __launch_bounds__(64 * W) void k_err_scan(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int GPW = Geo<D>::GPW, GCD = Geo<D>::GROUP_CD, TILE = Geo<D>::TILE;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    Group<D> G = make_group<D>(lds + wave * GPW * GCD, lane);
    cd *S1 = lds + W * GPW * GCD, *S2 = S1 + TILE, *S3 = S2 + TILE, *S4 = S3 + TILE;
    const int c = wave * GPW + G.g;
    const int i = G.i;
    const int b = blockIdx.x / P.ne, e = blockIdx.x % P.ne;
    const bool gvalid = G.lane_ok && c < P.nchunks;
    auto tile_of = [&](int cc) -> cd * { return lds + (cc / GPW) * GPW * GCD + (cc % GPW) * GCD; };
    const cd *Eb = B.E + (size_t)b * P.Nt * P.nv * TILE;
    const cd *Qb = B.Q + (size_t)b * P.Nt * TILE;
    const int v_err = P.off_err + e * P.err_stride;

    // Phase A: chunk total of W_k = Q_k^dag dE^err_k Q_{k-1}
    cd acc[D], x[D], w[D];
#pragma unroll
    for (int j = 0; j < D; ++j) acc[j] = czero();
    for (int j = 0; j < P.L; ++j) {
        const int k = c * P.L + j;
        const bool act = gvalid && k < P.Nt;
        const int kc = act ? k : 0;
        delta_row<D>(Eb + (size_t)kc * P.nv * TILE, v_err, i, P.inv_eps, x);
        local_frame<D>(G, Qb + (size_t)kc * TILE, j == 0, x, w, act);
        if (act) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) acc[jj] = cadd(acc[jj], w[jj]);
        }
    }
    // Phase A': Vc_c = Carry_c^dag (sum W) Carry_c  -> own tile
    const cd *Cr = B.Carry + ((size_t)b * P.nchunks + (gvalid ? c : 0)) * TILE;
    tile_store_row(G, acc, gvalid);
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) x[r] = cconj(Cr[r * D + i]);
    mm_tile<D>(x, G.tile, w);
    gsync();
    if (gvalid) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) G.tile[i * D + jj] = Cr[i * D + jj];
    }
    gsync();
    mm_tile<D>(w, G.tile, acc);
    gsync();
    tile_store_row(G, acc, gvalid);
    gsync();
    // Phase B: inclusive additive scan over chunks: X_c = sum_{c' <= c} Vc_c'
    for (int o = 1; o < P.nchunks; o <<= 1) {
        const bool doit = gvalid && c >= o;
        if (doit) {
            const cd *src = tile_of(c - o);
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = cadd(G.tile[i * D + jj], src[i * D + jj]);
        }
        gsync();
        if (doit) tile_store_row(G, x, true);
        gsync();
    }
    // Phase C (group 0): Ue = U Tot, F_d2err, M_e = G_e U, target x_add part
    const bool f0 = (c == 0) && G.lane_ok;
    const cd *Tot = tile_of(P.nchunks - 1);
    const cd *Ub = B.Ub + (size_t)b * TILE;
    const double *xb = B.x + (size_t)b * P.nx;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    Pert none;
    none.var = -1; none.index = 0; none.delta = 0.0;
    cd ue[D], ke[D];
#pragma unroll
    for (int jj = 0; jj < D; ++jj) x[jj] = Ub[i * D + jj];
    mm_tile<D>(x, Tot, ue);  // Ue row i
    target_row<D>(P, B, b, 0, i, xb, xadd, none, w);  // U0 row i
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            S1[i * D + jj] = w[jj];
            S2[i * D + jj] = ue[jj];
            S3[i * D + jj] = x[jj];
        }
    }
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) w[r] = cconj(S1[r * D + i]);
    mm_tile<D>(w, S2, ke);   // Ke = U0^dag Ue
    mm_tile<D>(w, S3, acc);  // K  = U0^dag U
    const double wi = P.W[i], pi_ = wi != 0.0 ? 1.0 : 0.0;
    double a1 = 0.0, a2 = 0.0;
    cd keii = czero();
#pragma unroll
    for (int jj = 0; jj < D; ++jj) {
        const double pj = P.W[jj] != 0.0 ? 1.0 : 0.0;
        a1 += pj * (ke[jj].re * ke[jj].re + ke[jj].im * ke[jj].im);
        const cd u = S2[jj * D + i];
        a2 += u.re * u.re + u.im * u.im;
        if (jj == i) keii = ke[jj];
    }
    const double s_a1 = group_sum(G, wi * a1, f0);
    const double s_a2 = group_sum(G, wi * a2, f0);
    const double te_re = group_sum(G, wi * keii.re, f0);
    const double te_im = group_sum(G, wi * keii.im, f0);
    // F_d2err = 2[ sum W_i P_j |Ke_ij|^2 - (1+D) sum_i W_i (Ue^dag Ue)_ii + |te|^2 ] / (D(D+1))
    const double fd2 = 2.0 * (s_a1 - (1.0 + P.Dtr) * s_a2 + te_re * te_re + te_im * te_im) / P.DD;
    // Ue^dag U (row i): left conj(Ue col i), right U (S3)
#pragma unroll
    for (int r = 0; r < D; ++r) w[r] = cconj(S2[r * D + i]);
    cd ueu[D];
    mm_tile<D>(w, S3, ueu);
    gsync();
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            S1[i * D + jj] = ke[jj];
            S3[i * D + jj] = acc[jj];  // K
        }
    }
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) w[r] = cscale(P.W[r], cconj(S1[r * D + i]));
    mm_tile<D>(w, S3, x);  // Ke^dag W K
    {
        const double sc = 4.0 / P.DD;
        const cd ctau = cmake(te_re, -te_im);
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            cd m = cadd(cscale(pi_, x[jj]), cmul(ctau, cscale(wi, acc[jj])));
            m = csub(m, cscale((1.0 + P.Dtr) * wi, ueu[jj]));
            w[jj] = cscale(sc, m);
        }
    }
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) S4[i * D + jj] = w[jj];
    }
    gsync();
    // target part of F_d2err_dx_add (FidelityCalculations.jl:100-112, the U0_dx_add terms):
    // 2[2 Re sum W P Kde conj(Ke) + 2 Re(conj(te) tr(W Kde))]/DD.  When H0 / Herror read x_add
    // the U_derr_dx_add terms are per-step sums added by k_err_grad + k_reduce_add.
    for (int qd = 0; qd < P.na; ++qd) {
        Pert pq;
        pq.var = VAR_XADD; pq.index = qd; pq.delta = P.eps;
        target_row<D>(P, B, b, 1 + qd, i, xb, xadd, pq, x);
        target_row<D>(P, B, b, 0, i, xb, xadd, none, ueu);
        if (f0) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) S1[i * D + jj] = cscale(P.inv_eps, csub(x[jj], ueu[jj]));
        }
        gsync();
#pragma unroll
        for (int r = 0; r < D; ++r) x[r] = cconj(S1[r * D + i]);
        mm_tile<D>(x, S2, ueu);  // Kde = U0d^dag Ue
        double pr = 0.0;
        cd kdii = czero();
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            const double pj = P.W[jj] != 0.0 ? 1.0 : 0.0;
            pr += pj * (ueu[jj].re * ke[jj].re + ueu[jj].im * ke[jj].im);
            if (jj == i) kdii = ueu[jj];
        }
        const double s1 = group_sum(G, wi * pr, f0);
        const double tr_re = group_sum(G, wi * kdii.re, f0);
        const double tr_im = group_sum(G, wi * kdii.im, f0);
        const double val = 2.0 * (2.0 * s1 + 2.0 * (te_re * tr_re + te_im * tr_im)) / P.DD;
        if (f0 && i == 0) B.Fd2dx[((size_t)b * P.ne + e) * P.nx + (size_t)P.np * P.Nt + qd] = val;
        gsync();
    }
    if (f0 && i == 0) B.Fd2[(size_t)b * P.ne + e] = fd2;
    // Phase D: per chunk M' = Carry M_e Carry^dag, T = Carry Sc Carry^dag, Ttot = Carry Tot Carry^dag
    cd sc[D], tot[D], cr[D];
#pragma unroll
    for (int jj = 0; jj < D; ++jj) {
        sc[jj] = (c > 0 && gvalid) ? tile_of(c - 1)[i * D + jj] : czero();
        tot[jj] = Tot[i * D + jj];
        cr[jj] = Cr[i * D + jj];
    }
    gsync();
    tile_store_row(G, cr, gvalid);  // own tile <- Carry_c
    gsync();
    cd *Mo = B.Me + (((size_t)b * P.ne + e) * P.nchunks + (gvalid ? c : 0)) * 3 * TILE;
    mm_tile<D>(cr, S4, x);
    mm_tile<D, true, true>(x, G.tile, w);  // M'
    if (gvalid) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) Mo[i * D + jj] = w[jj];
    }
    // T and Ttot: (X Carry^dag) to global scratch, then Carry * that
    for (int which = 0; which < 2; ++which) {
        cd *dst = Mo + (1 + which) * TILE;
        mm_tile<D, true, true>(which == 0 ? sc : tot, G.tile, x);
        if (gvalid) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) dst[i * D + jj] = x[jj];
        }
        __threadfence_block();
        gsync();
        mm_tile<D>(cr, dst, w);
        gsync();
        if (gvalid) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) dst[i * D + jj] = w[jj];
        }
    }
}

#ifndef GRAPE_ERRGRAD_WAVES
#define GRAPE_ERRGRAD_WAVES 2  // 2 waves/SIMD (308 B/lane of spills) beat 1 (336 registers): 2.51 -> 2.23 ms, C3 B=256
#endif
template <int D>
__global__ __launch_bounds__(64, GRAPE_ERRGRAD_WAVES) void k_err_grad(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int TILE = Geo<D>::TILE;
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const long nitems = (long)B.nb * P.nchunks * P.ne;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gc = valid ? gid : 0;
    const int e = (int)(gc % P.ne);
    const int c = (int)((gc / P.ne) % P.nchunks);
    const int b = (int)(gc / ((long)P.ne * P.nchunks));
    const int i = G.i;
    const cd *Eb = B.E + (size_t)b * P.Nt * P.nv * TILE;
    const cd *Qb = B.Q + (size_t)b * P.Nt * TILE;
    const cd *Mo = B.Me + (((size_t)b * P.ne + e) * P.nchunks + c) * 3 * TILE;
    const cd *Mp = Mo, *Tc = Mo + TILE, *Tt = Mo + 2 * TILE;
    const int v_err = P.off_err + e * P.err_stride, v_err2 = v_err + 1;
    double *out = B.Fd2dx + ((size_t)b * P.ne + e) * P.nx;
    const int nvg = P.np + (P.xadd_dep ? P.na : 0);
    cd A[D], Wk[D], z1[D], x[D], t[D];
#pragma unroll
    for (int jj = 0; jj < D; ++jj) A[jj] = Tc[i * D + jj];
    for (int j = 0; j < P.L; ++j) {
        const int k = c * P.L + j;
        const bool act = valid && k < P.Nt;
        const int kc = act ? k : 0;
        const cd *Ek = Eb + (size_t)kc * P.nv * TILE;
        const cd *Qk = Qb + (size_t)kc * TILE;
        delta_row<D>(Ek, v_err, i, P.inv_eps, x);
        local_frame<D>(G, Qk, j == 0, x, Wk, act);  // W_k
        for (int p = 0; p < nvg; ++p) {  // controls, then x_add (xadd_dep): variants off_dx + p
            delta_row<D>(Ek, P.off_dx + p, i, P.inv_eps, x);
            local_frame<D>(G, Qk, j == 0, x, z1, act);  // Z1 = Q^dag dE^dx Q
            // S1 = tr(A (M' Z1))
            tile_store_row(G, z1, act);
            gsync();
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = Mp[i * D + jj];
            mm_tile<D>(x, G.tile, t);  // (M' Z1) row i
            gsync();
            tile_store_row(G, t, act);
            gsync();
            cd s = row_dot_col<D>(A, G.tile, i);
            gsync();
            // S2 = tr((Ttot - A - W)(Z1 M'))
            if (act) {
#pragma unroll
                for (int jj = 0; jj < D; ++jj) G.tile[i * D + jj] = Mp[i * D + jj];
            }
            gsync();
            mm_tile<D>(z1, G.tile, t);  // (Z1 M') row i
            gsync();
            tile_store_row(G, t, act);
            gsync();
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = csub(csub(Tt[i * D + jj], A[jj]), Wk[jj]);
            s = cadd(s, row_dot_col<D>(x, G.tile, i));
            gsync();
            // S3 = tr(M' Z2), dE^mix = (E_mix + E - E_err2 - E_dx2) / eps2^2  (UnitaryCalculations.jl:79-83)
            {
                const cd *e0 = Ek + i * D;
                const cd *em = Ek + (size_t)(v_err + 2 + p) * TILE + i * D;
                const cd *ee2 = Ek + (size_t)v_err2 * TILE + i * D;
                const cd *ed2 = Ek + (size_t)(P.off_dx2 + p) * TILE + i * D;
#pragma unroll
                for (int jj = 0; jj < D; ++jj)
                    x[jj] = cscale(P.inv_eps2sq, csub(csub(cadd(em[jj], e0[jj]), ee2[jj]), ed2[jj]));
            }
            local_frame<D>(G, Qk, j == 0, x, t, act);  // Z2
            tile_store_row(G, t, act);
            gsync();
#pragma unroll
            for (int jj = 0; jj < D; ++jj) x[jj] = Mp[i * D + jj];
            s = cadd(s, row_dot_col<D>(x, G.tile, i));
            gsync();
            const double tot = group_sum(G, s.re, act);
            if (act && i == 0) {
                if (p < P.np) out[(size_t)k * P.np + p] = tot;
                else B.part_err_add[(((size_t)b * P.ne + e) * P.Nt + k) * P.na + (p - P.np)] = tot;
            }
        }
        if (act) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) A[jj] = cadd(A[jj], Wk[jj]);
        }
    }
}

}  // namespace grape
