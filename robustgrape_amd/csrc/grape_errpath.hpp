// grape_errpath.hpp -- error sources: sensitivities F_d2err and their gradients.
//
// Reference: src/UnitaryCalculations.jl:66-98 (error / mixed propagators),
// :111-151 (cumsum, reverse cumsum, U_derr, U_derr_dx), and
// src/FidelityCalculations.jl:78-113 (F_d2err, F_d2err_dx).
//
// Interaction-picture algebra (C_k = Q_k Carry_c for step k of chunk c,
// C_k^-1 = C_k^dagger), for one evaluation and error e:
//   local frame of step k:  Y(dX) = Q_k^dag dX Q_{k-1}   (Q_{k-1} = I at a chunk start)
//   W_k = Y(dE^err_k),  Z1_{k,u} = Y(dE^dx_u),  Z2_{k,u} = Y(dE^mix_{u})  (UnitaryCalculations.jl:48-95)
//   V^err_k = Carry_c^dag W_k Carry_c;  U_derr = U * Tot,  Tot = sum_k V^err_k       (:122-123)
//   F_d2err_dx[u,k] = Re tr(G_e U_derr_dx[u,k]),  M_e = G_e U,                  (FidelityCalculations.jl:85-113)
//     G_e = 4[P Ue^dag U0 W U0^dag + conj(tau_e) W U0^dag - (1+D) W Ue^dag]/(D(D+1))
//   with M' = Carry M_e Carry^dag, A_k = Carry S_{k-1} Carry^dag (S = cumsum, :112; R_{k+1} =
//   Tot - S_{k-1} - V_k, :113) and Ttot = Carry Tot Carry^dag, the reference's
//   U (V^dx S_{k-1} + R_{k+1} V^dx + V^mix) contracted with G_e (:124-139) is
//     Re[ tr(A_k M' Z1) + tr((Ttot - A_k - W_k) Z1 M') + tr(M' Z2) ]
//   = Re[ tr(Lambda_k Z1) + tr(M' Z2) ],  Lambda_k = [A_k, M'] + M' Ttot - M' W_k.
//   The running state B_k = [A_k, M'] + M' Ttot obeys B_{k+1} = B_k + W_k M' - M' W_k
//   (A_{k+1} = A_k + W_k), so a step costs two products per error.  The same Z1 gives the
//   fidelity gradient F_dx[u,k] = Re tr(M'_c Z1_{k,u}) (FidelityCalculations.jl:56-76).
//
// k_err_local one row group per (b, k): every local-frame image Z1_u, W_e, Z2_{e,u} of
//             step k (2 products each, Q_k / Q_{k-1} staged once), stored to Zl; F_dx.
// k_err_scan  one workgroup per (b, e): chunk totals of W, carry transform,
//             additive scan over chunks, U_derr, F_d2err, M_e, per-chunk M', T, Ttot.
// k_err_grad  one row group per (b, chunk, e): walks the chunk's steps carrying B_k,
//             two products per step (M' W_k, W_k M') and the traces per gradient
//             parameter (controls; x_add too when H0 / Herror read it, U_derr_dx_add
//             being the sum over k of the same per-step terms, :140-151).
#pragma once
#include "grape_kernels.hpp"

namespace grape {

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
    // Phase A: chunk total of the stored W_k = Q_k^dag dE^err_k Q_{k-1} (k_err_local)
    cd acc[D], x[D], w[D];
#pragma unroll
    for (int j = 0; j < D; ++j) acc[j] = czero();
    const int w_slot = P.nvg + e;
    if (B.Wc) {  // the walk path's chunk sums (k_walk_img_sum, same summation order)
        if (gvalid) {
            const cd *Ws = B.Wc + (((size_t)b * P.ne + e) * P.nchunks + c) * TILE + i * D;
#pragma unroll
            for (int jj = 0; jj < D; ++jj) acc[jj] = Ws[jj];
        }
    } else {
        for (int j = 0; j < P.L; ++j) {
            const int k = c * P.L + j;
            if (gvalid && k < P.Nt) {
                const cd *Wk = B.Zl + ((size_t)(b * P.Nt + k) * P.nz + w_slot) * TILE + i * D;
#pragma unroll
                for (int jj = 0; jj < D; ++jj) acc[jj] = cadd(acc[jj], Wk[jj]);
            }
        }
    }
    // Phase A': Vc_c = Carry_c^dag (sum W) Carry_c  -> own tile.  The lab-frame walks (P.gauge_lab,
    // grape_walk.hpp k_walk_wsum_lab) hand over R = T_c (sum W) T_c^dag: Vc_c = Carry_{c+1}^dag R Carry_{c+1}
    // (Carry_{c+1} = T_c Carry_c; past the last chunk, U)
    const int cc = gvalid ? c : 0;
    const cd *Cr = B.Carry + ((size_t)b * P.nchunks + cc) * TILE;
    const cd *Ca = (P.gauge_lab && B.Wc) ? (cc + 1 < P.nchunks ? Cr + TILE : B.Ub + (size_t)b * TILE) : Cr;
    tile_store_row(G, acc, gvalid);
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) x[r] = cconj(Ca[r * D + i]);
    mm_tile<D>(x, G.tile, w);
    gsync();
    if (gvalid) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) G.tile[i * D + jj] = Ca[i * D + jj];
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
    const cd *Tot = tile_of(P.nchunks - 1);
    if (P.sectors) {  // the sector error head forms F_d2err and M_e from the assembled U and Tot
        if (c == P.nchunks - 1 && G.lane_ok) {
            cd *dt = B.TotS + ((size_t)b * P.ne + e) * TILE + i * D;
#pragma unroll
            for (int jj = 0; jj < D; ++jj) dt[jj] = Tot[i * D + jj];
        }
    } else {
    // Phase C (group 0): Ue = U Tot, F_d2err, M_e = G_e U, target x_add part
    const bool f0 = (c == 0) && G.lane_ok;
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
    }  // Phase C
    // Phase D: per chunk M' = Carry M_e Carry^dag (sectors: k_sec_mc_err, after the head),
    // T = Carry Sc Carry^dag, Ttot = Carry Tot Carry^dag
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
    if (!P.sectors) {
        mm_tile<D>(cr, S4, x);
        mm_tile<D, true, true>(x, G.tile, w);  // M'
        if (gvalid) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) Mo[i * D + jj] = w[jj];
        }
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

// LDS of the error-path row-group kernels: per group its tile + aux, then one more tile
template <int D>
__device__ __forceinline__ cd *second_tile(cd *lds, const Group<D> &G) {
    return lds + Geo<D>::GPW * Geo<D>::GROUP_CD + G.g * Geo<D>::TILE;
}

// k_err_local: one row group per (b, k).  Lane i holds column i of each difference dX
// (coalesced loads of the row-major E tiles) and produces row i of Q_k^dag dX Q_{k-1}:
//   row i of Q_k^dag X = conj(column i of Q_k) . X   (X staged in the group tile)
//   then . Q_{k-1}                                   (Q_{k-1} staged once in the second tile)
// (A column-form variant with coalesced Zl stores measured 11 % slower.)
template <int D>
__global__ __launch_bounds__(64, 2) void k_err_local(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int TILE = Geo<D>::TILE;
    Group<D> G = make_group<D>(lds, threadIdx.x);
    cd *Qp = second_tile<D>(lds, G);
    const long nitems = (long)B.nb * P.Nt;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    int k, b, unused;
    split_item(gidc, nitems, P.Nt, 1, b, unused, k);
    const int c = k / P.L;
    const bool first = k == c * P.L;  // chunk start: Q_{k-1} = I
    const int i = G.i;
    const cd *Qk = B.Q + ((size_t)b * P.Nt + k) * TILE;
    const cd *Ek = B.E + (((size_t)b * P.Nt + k) * P.nv) * TILE;
    cd *Zk = B.Zl + (((size_t)b * P.Nt + k) * P.nz) * TILE;
    if (valid && !first) {
#pragma unroll
        for (int m = 0; m < D; ++m) Qp[m * D + i] = Qk[m * D + i - TILE];
    }
    cd qc[D], e0[D], x[D], y[D];
#pragma unroll
    for (int m = 0; m < D; ++m) {
        qc[m] = cconj(Qk[m * D + i]);
        e0[m] = Ek[m * D + i];
    }
    // y <- row i of Q_k^dag X Q_{k-1} for the column x of X (x destroyed), stored to slot
    auto frame = [&](int slot) {
        if (valid) {
#pragma unroll
            for (int m = 0; m < D; ++m) G.tile[m * D + i] = x[m];
        }
        gsync();
        mm_tile<D>(qc, G.tile, y);
        gsync();
        if (!first) {
#pragma unroll
            for (int j = 0; j < D; ++j) x[j] = y[j];
            mm_tile<D>(x, Qp, y);
        }
        if (valid) {
            cd *dst = Zk + (size_t)slot * TILE + i * D;
#pragma unroll
            for (int j = 0; j < D; ++j) dst[j] = y[j];
        }
    };
    // gradient parameters: Z1_u = Y((E_u - E_0) / eps) and F_dx[u,k] = Re tr(M'_c Z1_u)
    const cd *Mc = B.Mc + ((size_t)b * P.nchunks + c) * TILE;
    for (int u = 0; u < P.nvg; ++u) {
        const cd *Ev = Ek + (size_t)(P.off_dx + u) * TILE;
#pragma unroll
        for (int m = 0; m < D; ++m) x[m] = cscale(P.inv_eps, csub(Ev[m * D + i], e0[m]));  // (1/eps)(E' - E)
        frame(u);
        double s = 0.0;  // sum_j Z1[i][j] M'[j][i]
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const cd mm = Mc[j * D + i];
            s += y[j].re * mm.re - y[j].im * mm.im;
        }
        s = group_sum(G, s, valid);
        if (valid && i == 0) {
            if (B.sec_part) B.sec_part[((size_t)b * P.Nt + k) * P.nvg + u] = s;  // sector term (k_sec_reduce)
            else if (u < P.np) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + u] = s;
            else B.part_add[((size_t)b * P.Nt + k) * P.na + (u - P.np)] = s;
        }
    }
    for (int e = 0; e < P.ne; ++e) {
        const int v_err = P.off_err + e * P.err_stride;
        const cd *Ee = Ek + (size_t)v_err * TILE;
#pragma unroll
        for (int m = 0; m < D; ++m) x[m] = cscale(P.inv_eps, csub(Ee[m * D + i], e0[m]));
        frame(P.nvg + e);  // W_e
        for (int u = 0; u < P.nvg; ++u) {
            // dE^mix = (E(u + eps2, err eps2) + E - E(err eps2) - E(u + eps2)) / eps2^2  (:79-83, :91-94)
            const cd *em = Ek + (size_t)(v_err + 2 + u) * TILE, *ee2 = Ek + (size_t)(v_err + 1) * TILE;
            const cd *ed2 = Ek + (size_t)(P.off_dx2 + u) * TILE;
#pragma unroll
            for (int m = 0; m < D; ++m)
                x[m] = cscale(P.inv_eps2sq, csub(csub(cadd(em[m * D + i], e0[m]), ee2[m * D + i]), ed2[m * D + i]));
            frame(P.nvg + P.ne + e * P.nvg + u);  // Z2_{e,u}
        }
    }
}

// k_err_grad: one row group per (b, chunk, e), lane i holding row i of B_k.
template <int D>
__global__ __launch_bounds__(64, 2) void k_err_grad(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int TILE = Geo<D>::TILE;
    Group<D> G = make_group<D>(lds, threadIdx.x);
    cd *Mt = second_tile<D>(lds, G);  // M' (constant over the chunk)
    const long nitems = (long)B.nb * P.nchunks * P.ne;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gc = valid ? gid : 0;
    int e, c, b;
    split_item(gc, nitems, P.ne, P.nchunks, b, c, e);
    const int i = G.i;
    const cd *Mo = B.Me + (((size_t)b * P.ne + e) * P.nchunks + c) * 3 * TILE;  // M', Tc, Ttot
    double *out = B.Fd2dx + ((size_t)b * P.ne + e) * P.nx;
    cd mrow[D], bp[D], w[D], t[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        mrow[j] = Mo[i * D + j];
        w[j] = Mo[TILE + i * D + j];  // Tc = A at the chunk start
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < D; ++j) Mt[i * D + j] = mrow[j];
    }
    tile_store_row(G, w, valid);
    gsync();
    // B = Tc M' - M' Tc + M' Ttot
    mm_tile<D>(w, Mt, bp);
    mm_tile<D>(mrow, G.tile, t);
#pragma unroll
    for (int j = 0; j < D; ++j) {
        bp[j] = csub(bp[j], t[j]);
        w[j] = Mo[2 * TILE + i * D + j];
    }
    gsync();
    tile_store_row(G, w, valid);
    gsync();
    mm_tile<D>(mrow, G.tile, t);
#pragma unroll
    for (int j = 0; j < D; ++j) bp[j] = cadd(bp[j], t[j]);
    gsync();
    const int w_slot = P.nvg + e, z2_slot = P.nvg + P.ne + e * P.nvg;
    for (int jstep = 0; jstep < P.L; ++jstep) {
        const int k = c * P.L + jstep;
        const bool act = valid && k < P.Nt;
        const int kc = act ? k : 0;
        const cd *Zk = B.Zl + ((size_t)b * P.Nt + kc) * P.nz * TILE;
#pragma unroll
        for (int j = 0; j < D; ++j) w[j] = Zk[(size_t)w_slot * TILE + i * D + j];  // row i of W_k
        tile_store_row(G, w, valid);
        gsync();
        mm_tile<D>(mrow, G.tile, t);  // M' W
#pragma unroll
        for (int j = 0; j < D; ++j) bp[j] = csub(bp[j], t[j]);  // Lambda_k
        for (int u = 0; u < P.nvg; ++u) {
            const cd *z1 = Zk + (size_t)u * TILE + i, *z2 = Zk + (size_t)(z2_slot + u) * TILE + i;
            double s = 0.0;  // sum_j Lambda[i][j] Z1[j][i] + M'[i][j] Z2[j][i]
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const cd a = z1[j * D], bz = z2[j * D];
                s += bp[j].re * a.re - bp[j].im * a.im;
                s += mrow[j].re * bz.re - mrow[j].im * bz.im;
            }
            s = group_sum(G, s, valid);
            if (act && i == 0) {
                if (B.sec_part_err) B.sec_part_err[(((size_t)b * P.ne + e) * P.Nt + k) * P.nvg + u] = s;
                else if (u < P.np) out[(size_t)k * P.np + u] = s;
                else B.part_err_add[(((size_t)b * P.ne + e) * P.Nt + k) * P.na + (u - P.np)] = s;
            }
        }
        mm_tile<D>(w, Mt, t);  // W M'
#pragma unroll
        for (int j = 0; j < D; ++j) bp[j] = cadd(bp[j], t[j]);  // B_{k+1} = Lambda_k + W_k M'
        gsync();
    }
}

}  // namespace grape
