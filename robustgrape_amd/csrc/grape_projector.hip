// grape_projector.hip -- fidelity and error-sensitivity heads for a GENERAL projector.
//
// The reference accepts any matrix as FidelityRobustGRAPEProblem.projector
// (src/FidelityCalculations.jl:47-51):
//     P0 = projector,  tr_mod(X) = tr(P0 X),  P = P0 with every nonzero entry set to 1,
//     D = Re tr(P0),   F = [Re tr_mod(P K P K^dag) + |tr_mod(P K)|^2] / (D(D+1)),  K = U0^dag U.
// The engines' hot kernels specialise to a real diagonal P0 (every test, example and
// RydbergTools problem of the reference): tr_mod(P X) = sum_i w_i X_ii.  For any other P0
// the plan sets DevProblem::gen_proj and these heads run right after the scans, over the
// matrices the scans leave in HBM (U, the chunk carries, the error totals), and OVERWRITE
// the diagonal-specialised results: F, the gradient kernel M = G U (and its per-chunk
// images M'_c), the target part of F_dx_add, and with error sources F_d2err, M_e (and
// M'_{c,e}) and the target part of F_d2err_dx_add.  Everything downstream (the gradient
// contractions) is linear in M / M_e and is unchanged.
//
// With A = P0 P and B = P (both d x d), the reference's expressions are
//   F       = [Re tr(A K B K^dag) + |tau|^2] / DD,  tau = tr(A K)                       (:54)
//   dF      = Re tr(G dU),  M = G U = [(B K^dag A + B^dag K^dag A^dag) K + 2 conj(tau) A K] / DD
//                                                                           (:58-63, linear in U_dx)
//   F_dx_add target part = [Re tr(A Kd B K^dag) + Re tr(A K B Kd^dag) + 2 Re(conj(tau) tr(A Kd))] / DD,
//             Kd = U0d^dag U, U0d = (U0(x_add + eps e_q) - U0) / eps                    (:34-40, 67-76)
//   F_d2err = 2 [Re tr(A Ke B Ke^dag) - (1 + D) Re tr(A Ue^dag Ue) + |tau_e|^2] / DD,
//             Ue = U_derr = U Tot, Ke = U0^dag Ue, tau_e = tr(A Ke)                      (:79-83)
//   M_e     = 2 [(B Ke^dag A + B^dag Ke^dag A^dag) K + 2 conj(tau_e) A K
//                - (1 + D)(A + A^dag) Ue^dag U] / DD                               (:85-97, linear in U_derr_dx)
//   F_d2err_dx_add target part = 2 [Re tr(A Kde B Ke^dag) + Re tr(A Ke B Kde^dag)
//                                   + 2 Re(conj(tau_e) tr(A Kde))] / DD, Kde = U0d^dag Ue   (:100-112)
// (for A = diag(w), B = diag(w != 0) these are the hot kernels' formulas).
//
// These heads run once per evaluation (per error source), not per time step: plain
// thread-per-element products over row-major d x d scratch matrices in HBM (L2-resident),
// one 256-thread workgroup per evaluation, any d <= 64.
#include "grape_projector_api.hpp"

namespace grape_proj {

namespace {

using grape::cd;
constexpr int BLOCK = 256;

__device__ __forceinline__ cd p_add(cd a, cd b) { return cd{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cd p_sub(cd a, cd b) { return cd{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cd p_scale(double s, cd a) { return cd{s * a.re, s * a.im}; }
__device__ __forceinline__ cd p_mul(cd a, cd b) { return cd{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ cd p_conj(cd a) { return cd{a.re, -a.im}; }

// op(X)(i, l): X row-major, op = N (X) or H (X^dagger)
template <bool H>
__device__ __forceinline__ cd el(const cd *X, int D, int i, int l) {
    return H ? p_conj(X[(size_t)l * D + i]) : X[(size_t)i * D + l];
}

// C = op(A) op(B); C must not alias A or B.  Ends with a workgroup barrier.
template <bool HA, bool HB>
__device__ void bmm(cd *C, const cd *A, const cd *B, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const int i = t / D, j = t % D;
        cd s{0.0, 0.0};
        for (int l = 0; l < D; ++l) s = p_add(s, p_mul(el<HA>(A, D, i, l), el<HB>(B, D, l, j)));
        C[t] = s;
    }
    __syncthreads();
}

// workgroup sums (every thread receives the result); NT = threads of the workgroup
template <int NT = BLOCK>
__device__ double bsum(double v, double *red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}
// tr(X) (complex)
template <int NT = BLOCK>
__device__ cd btrace(const cd *X, int D, double *red) {
    double re = 0.0, im = 0.0;
    for (int i = threadIdx.x; i < D; i += blockDim.x) {
        re += X[(size_t)i * D + i].re;
        im += X[(size_t)i * D + i].im;
    }
    return cd{bsum<NT>(re, red), bsum<NT>(im, red)};
}
// Re tr(X Y^dagger) = Re sum_ij X_ij conj(Y_ij)
template <int NT = BLOCK>
__device__ double bdot(const cd *X, const cd *Y, int D, double *red) {
    double s = 0.0;
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) s += X[t].re * Y[t].re + X[t].im * Y[t].im;
    return bsum<NT>(s, red);
}
// Re tr(X Y) = Re sum_ij X_ij Y_ji
__device__ double btrprod(const cd *X, const cd *Y, int D, double *red) {
    double s = 0.0;
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const int i = t / D, j = t % D;
        const cd a = X[t], b = Y[(size_t)j * D + i];
        s += a.re * b.re - a.im * b.im;
    }
    return bsum(s, red);
}

// dense-engine register-file image (grape_engine.hip to_dense_image): element (row, col)
__device__ __forceinline__ size_t img_off(int row, int col) {
    const int w = col >> 4, t = row >> 4, r = (row & 15) >> 2, l = ((row & 3) << 4) | (col & 15);
    return (size_t)((w * 4 + t) * 4 + r) * 64 + l;
}
// source matrix: row-major d x d (small engine) or a padded 64 x 64 image (dense engine)
__device__ void load_mat(cd *dst, const void *src, int D, bool image) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        if (image) {
            const double *img = static_cast<const double *>(src);
            const size_t o = img_off(t / D, t % D);
            dst[t] = cd{img[o], img[4096 + o]};
        } else {
            dst[t] = static_cast<const cd *>(src)[t];
        }
    }
    __syncthreads();
}
__device__ void store_image(double *img, const cd *src, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const size_t o = img_off(t / D, t % D);
        img[o] = src[t].re;
        img[4096 + o] = src[t].im;
    }
    __syncthreads();
}

// U0(x_add [+ eps e_q]) row-major: from the target terms over the row-major operator basis,
// or (closure fallback) from the host-evaluated table (column-major, slot 0 / 1 + q)
__device__ void build_target(const grape::DevProblem &P, const cd *U0tab, int b, const double *xb, int slot,
                             cd *dst) {
    const int D = P.D;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    grape::Pert pp;
    pp.var = slot > 0 ? grape::VAR_XADD : -1;
    pp.index = slot > 0 ? slot - 1 : 0;
    pp.delta = slot > 0 ? P.eps : 0.0;
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const int i = t / D, j = t % D;
        if (U0tab) {
            dst[t] = U0tab[((size_t)b * (1 + P.na) + slot) * D * D + i + (size_t)j * D];
            continue;
        }
        cd h{0.0, 0.0};
        for (int q = 0; q < P.n_tgt; ++q) {
            const grape::Term tm = P.tgt[q];
            h = p_add(h, p_mul(grape::term_coef(tm, 1, xb, xadd, pp), P.ops[(size_t)tm.op * D * D + t]));
        }
        dst[t] = h;
    }
    __syncthreads();
}

// dst = Carry src Carry^dagger (tmp: scratch)
__device__ void conjugate_by(cd *dst, const cd *Carry, const cd *src, cd *tmp, int D) {
    bmm<false, false>(tmp, Carry, src, D);
    bmm<false, true>(dst, tmp, Carry, D);
}

enum { S_U, S_U0, S_K, S_X, S_Y, S_T1, S_T2, S_T3, S_M, S_UE, S_KE, S_XE, S_YE, S_TOT, S_C, kSlots };
static_assert(kSlots <= kScratchSlots, "projector scratch");

// F, M and the target part of F_dx_add for evaluation b = blockIdx.x
__global__ __launch_bounds__(BLOCK) void k_proj_fid(Heads H) {
    __shared__ double red[BLOCK];
    const grape::DevProblem &P = H.P;
    const int D = P.D, b = blockIdx.x;
    const size_t T = (size_t)D * D;
    cd *s = H.scr + (size_t)b * kScratchSlots * T;
    cd *U = s + S_U * T, *U0 = s + S_U0 * T, *K = s + S_K * T, *X = s + S_X * T, *Y = s + S_Y * T;
    cd *T1 = s + S_T1 * T, *T2 = s + S_T2 * T, *T3 = s + S_T3 * T, *M = s + S_M * T, *C = s + S_C * T;
    const cd *A = P.PA, *Bm = P.PB;
    const double *xb = H.x + (size_t)b * P.nx;
    if (H.dense) load_mat(U, H.Ub_img + (size_t)b * kImg, D, true);
    else load_mat(U, H.Ub + (size_t)b * T, D, false);
    build_target(P, H.U0tab, b, xb, 0, U0);
    bmm<true, false>(K, U0, U, D);   // K = U0^dag U
    bmm<false, false>(X, A, K, D);   // A K
    const cd tau = btrace(X, D, red);
    bmm<false, false>(Y, X, Bm, D);  // A K B
    const double Fv = (bdot(Y, K, D, red) + tau.re * tau.re + tau.im * tau.im) / P.DD;
    // M = [B (K^dag A K) + B^dag ((A K)^dag K) + 2 conj(tau) A K] / DD
    bmm<true, false>(T1, K, X, D);
    bmm<false, false>(M, Bm, T1, D);
    bmm<true, false>(T1, X, K, D);
    bmm<true, false>(T2, Bm, T1, D);
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) {
        const cd ct = p_mul(cd{tau.re, -tau.im}, X[t]);
        M[t] = p_scale(1.0 / P.DD, p_add(p_add(M[t], T2[t]), p_scale(2.0, ct)));
    }
    __syncthreads();
    for (int q = 0; q < P.na; ++q) {  // target part of F_dx_add
        build_target(P, H.U0tab, b, xb, 1 + q, T1);
        for (int t = threadIdx.x; t < (int)T; t += blockDim.x) T1[t] = p_scale(P.inv_eps, p_sub(T1[t], U0[t]));
        __syncthreads();
        bmm<true, false>(T2, T1, U, D);   // Kd
        bmm<false, false>(T1, A, T2, D);  // A Kd
        const cd trd = btrace(T1, D, red);
        bmm<false, false>(T3, T1, Bm, D);  // A Kd B
        const double sa = bdot(T3, K, D, red), sb = bdot(Y, T2, D, red);
        const double val = (sa + sb + 2.0 * (tau.re * trd.re + tau.im * trd.im)) / P.DD;
        if (threadIdx.x == 0) {
            if (P.xadd_dep && H.tgt_part) H.tgt_part[(size_t)b * P.na + q] = val;
            else H.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + q] = val;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) H.F[b] = Fv;
    if (H.dense) {  // k_dmc forms the per-chunk images from M
        store_image(H.M_img + (size_t)b * kImg, M, D);
        return;
    }
    for (int c = 0; c < P.nchunks; ++c) {  // M'_c = Carry_c M Carry_c^dagger
        load_mat(C, H.Carry + ((size_t)b * P.nchunks + c) * T, D, false);
        conjugate_by(T1, C, M, T2, D);
        cd *dst = H.Mc + ((size_t)b * P.nchunks + c) * T;
        for (int t = threadIdx.x; t < (int)T; t += blockDim.x) dst[t] = T1[t];
        __syncthreads();
    }
}

// F_d2err, M_e and the target part of F_d2err_dx_add for (b, e) = (blockIdx.x / ne, blockIdx.x % ne)
__global__ __launch_bounds__(BLOCK) void k_proj_err(Heads H) {
    __shared__ double red[BLOCK];
    const grape::DevProblem &P = H.P;
    const int D = P.D, ne = P.ne, b = blockIdx.x / ne, e = blockIdx.x % ne;
    const size_t T = (size_t)D * D, be = (size_t)b * ne + e;
    cd *s = H.scr + be * kScratchSlots * T;
    cd *U = s + S_U * T, *U0 = s + S_U0 * T, *K = s + S_K * T, *X = s + S_X * T;
    cd *T1 = s + S_T1 * T, *T2 = s + S_T2 * T, *T3 = s + S_T3 * T, *M = s + S_M * T, *C = s + S_C * T;
    cd *Ue = s + S_UE * T, *Ke = s + S_KE * T, *Xe = s + S_XE * T, *Ye = s + S_YE * T, *Tot = s + S_TOT * T;
    const cd *A = P.PA, *Bm = P.PB;
    const double *xb = H.x + (size_t)b * P.nx;
    if (H.dense) {
        load_mat(U, H.Ub_img + (size_t)b * kImg, D, true);
        load_mat(Tot, H.Tot_img + be * kImg, D, true);
    } else {
        load_mat(U, H.Ub + (size_t)b * T, D, false);
        // chunk 0 of k_err_scan's [M', T_c, Ttot_c] triple: Carry_0 = I, so Ttot_0 = Tot
        load_mat(Tot, H.Me + (be * P.nchunks) * 3 * T + 2 * T, D, false);
    }
    build_target(P, H.U0tab, b, xb, 0, U0);
    bmm<false, false>(Ue, U, Tot, D);  // U_derr = U Tot                (UnitaryCalculations.jl:122-123)
    bmm<true, false>(Ke, U0, Ue, D);
    bmm<true, false>(K, U0, U, D);
    bmm<false, false>(Xe, A, Ke, D);
    const cd te = btrace(Xe, D, red);
    bmm<false, false>(Ye, Xe, Bm, D);
    const double t1 = bdot(Ye, Ke, D, red);
    bmm<true, false>(T1, Ue, Ue, D);
    const double t2 = btrprod(A, T1, D, red);  // Re tr(A Ue^dag Ue)
    const double fd2 = 2.0 * (t1 - (1.0 + P.Dtr) * t2 + te.re * te.re + te.im * te.im) / P.DD;
    // M_e = 2 [B Ke^dag (A K) + B^dag (A Ke)^dag K + 2 conj(te) A K - (1 + D)(A + A^dag) Ue^dag U] / DD
    bmm<false, false>(X, A, K, D);
    bmm<true, false>(T1, Ke, X, D);
    bmm<false, false>(M, Bm, T1, D);
    bmm<true, false>(T1, Xe, K, D);
    bmm<true, false>(T2, Bm, T1, D);
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) {
        M[t] = p_add(p_add(M[t], T2[t]), p_scale(2.0, p_mul(cd{te.re, -te.im}, X[t])));
        const int i = t / D, j = t % D;
        T2[t] = p_add(A[t], p_conj(A[(size_t)j * D + i]));  // A + A^dagger
    }
    __syncthreads();
    bmm<true, false>(T1, Ue, U, D);
    bmm<false, false>(T3, T2, T1, D);
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x)
        M[t] = p_scale(2.0 / P.DD, p_sub(M[t], p_scale(1.0 + P.Dtr, T3[t])));
    __syncthreads();
    for (int q = 0; q < P.na; ++q) {  // target part of F_d2err_dx_add
        build_target(P, H.U0tab, b, xb, 1 + q, T1);
        for (int t = threadIdx.x; t < (int)T; t += blockDim.x) T1[t] = p_scale(P.inv_eps, p_sub(T1[t], U0[t]));
        __syncthreads();
        bmm<true, false>(T2, T1, Ue, D);  // Kde
        bmm<false, false>(T1, A, T2, D);
        const cd trd = btrace(T1, D, red);
        bmm<false, false>(T3, T1, Bm, D);
        const double sa = bdot(T3, Ke, D, red), sb = bdot(Ye, T2, D, red);
        const double val = 2.0 * (sa + sb + 2.0 * (te.re * trd.re + te.im * trd.im)) / P.DD;
        if (threadIdx.x == 0) H.Fd2dx[be * P.nx + (size_t)P.np * P.Nt + q] = val;
        __syncthreads();
    }
    if (threadIdx.x == 0) H.Fd2[be] = fd2;
    if (H.dense) {  // k_dmce forms M'_{c,e} and the chunk-start states from M_e
        store_image(H.Me_img + be * kImg, M, D);
        return;
    }
    for (int c = 0; c < P.nchunks; ++c) {  // M'_{c,e} = Carry_c M_e Carry_c^dagger
        load_mat(C, H.Carry + ((size_t)b * P.nchunks + c) * T, D, false);
        conjugate_by(T1, C, M, T2, D);
        cd *dst = H.Me + ((be * P.nchunks) + c) * 3 * T;
        for (int t = threadIdx.x; t < (int)T; t += blockDim.x) dst[t] = T1[t];
        __syncthreads();
    }
}

// Sector head, evaluation b = blockIdx.x (grape_projector_api.hpp SectorHead).  d <= 12: one
// wave per evaluation, every d x d intermediate in LDS (9 slots).
constexpr int SEC_BLOCK = 64;
enum { H_U, H_U0, H_K, H_X, H_Y, H_T1, H_T2, H_T3, H_M, kHeadSlots };
__global__ __launch_bounds__(SEC_BLOCK) void k_sec_head(SectorHead H) {
    __shared__ double red[SEC_BLOCK];
    extern __shared__ __attribute__((aligned(16))) unsigned char sec_smem[];
    const grape::DevProblem &P = H.P;
    const int D = P.D, b = blockIdx.x;
    const size_t T = (size_t)D * D;
    cd *s = reinterpret_cast<cd *>(sec_smem);
    cd *U = s + H_U * T, *U0 = s + H_U0 * T, *K = s + H_K * T, *X = s + H_X * T, *Y = s + H_Y * T;
    cd *T1 = s + H_T1 * T, *T2 = s + H_T2 * T, *T3 = s + H_T3 * T, *M = s + H_M * T;
    const cd *A = P.PA, *Bm = P.PB;
    const double *xb = H.x + (size_t)b * P.nx;
    // U = direct sum of the sector propagators and of the identity on the levels no operator
    // touches (exact zeros across sectors, as in the dense product)
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) U[t] = cd{0.0, 0.0};
    __syncthreads();
    for (int cl = 0; cl < H.ncls; ++cl) {
        const int S = H.S[cl], SS = S * S, ns = H.nsec[cl];
        for (int t = threadIdx.x; t < ns * SS; t += blockDim.x) {
            const int w = t / SS, r = (t % SS) / S, c = t % S;
            const int gi = H.sidx[cl][w * S + r], gj = H.sidx[cl][w * S + c];
            if (gi >= 0 && gj >= 0) U[(size_t)gi * D + gj] = H.Ub[cl][((size_t)b * ns + w) * SS + r * S + c];
        }
    }
    for (int t = threadIdx.x; t < H.nfixed; t += blockDim.x) {
        const int g = H.fixed[t];
        U[(size_t)g * D + g] = cd{1.0, 0.0};
    }
    __syncthreads();
    build_target(P, nullptr, b, xb, 0, U0);
    bmm<true, false>(K, U0, U, D);   // K = U0^dag U
    bmm<false, false>(X, A, K, D);   // A K
    const cd tau = btrace<SEC_BLOCK>(X, D, red);
    bmm<false, false>(Y, X, Bm, D);  // A K B
    const double Fv = (bdot<SEC_BLOCK>(Y, K, D, red) + tau.re * tau.re + tau.im * tau.im) / P.DD;
    bmm<true, false>(T1, K, X, D);
    bmm<false, false>(M, Bm, T1, D);
    bmm<true, false>(T1, X, K, D);
    bmm<true, false>(T2, Bm, T1, D);
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) {
        const cd ct = p_mul(cd{tau.re, -tau.im}, X[t]);
        M[t] = p_scale(1.0 / P.DD, p_add(p_add(M[t], T2[t]), p_scale(2.0, ct)));
    }
    __syncthreads();
    for (int q = 0; q < P.na; ++q) {  // target part of F_dx_add
        build_target(P, nullptr, b, xb, 1 + q, T1);
        for (int t = threadIdx.x; t < (int)T; t += blockDim.x) T1[t] = p_scale(P.inv_eps, p_sub(T1[t], U0[t]));
        __syncthreads();
        bmm<true, false>(T2, T1, U, D);   // Kd
        bmm<false, false>(T1, A, T2, D);  // A Kd
        const cd trd = btrace<SEC_BLOCK>(T1, D, red);
        bmm<false, false>(T3, T1, Bm, D);  // A Kd B
        const double sa = bdot<SEC_BLOCK>(T3, K, D, red), sb = bdot<SEC_BLOCK>(Y, T2, D, red);
        const double val = (sa + sb + 2.0 * (tau.re * trd.re + tau.im * trd.im)) / P.DD;
        if (threadIdx.x == 0) {
            if (P.xadd_dep && H.tgt_part) H.tgt_part[(size_t)b * P.na + q] = val;
            else H.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + q] = val;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) H.F[b] = Fv;
    // the sector blocks M_ww: the only part of M the block-diagonal contractions see
    for (int cl = 0; cl < H.ncls; ++cl) {
        const int S = H.S[cl], SS = S * S, ns = H.nsec[cl];
        for (int t = threadIdx.x; t < ns * SS; t += blockDim.x) {
            const int w = t / SS, r = (t % SS) / S, c = t % S;
            const int gi = H.sidx[cl][w * S + r], gj = H.sidx[cl][w * S + c];
            H.Msec[cl][(size_t)b * ns * SS + t] = (gi >= 0 && gj >= 0) ? M[(size_t)gi * D + gj] : cd{0.0, 0.0};
        }
    }
}

// Sector error head, (b, e) = (blockIdx.x / ne, blockIdx.x % ne): k_proj_err's formulas over
// U and Tot assembled from the sector blocks (Tot is zero on the untouched levels).
enum { E_U, E_U0, E_K, E_X, E_T1, E_T2, E_T3, E_M, E_UE, E_KE, E_XE, E_YE, E_TOT, kErrHeadSlots };
__global__ __launch_bounds__(SEC_BLOCK) void k_sec_err_head(SectorHead H) {
    __shared__ double red[SEC_BLOCK];
    extern __shared__ __attribute__((aligned(16))) unsigned char sec_smem[];
    const grape::DevProblem &P = H.P;
    const int D = P.D, ne = P.ne, b = blockIdx.x / ne, e = blockIdx.x % ne;
    const size_t T = (size_t)D * D, be = (size_t)b * ne + e;
    cd *s = reinterpret_cast<cd *>(sec_smem);
    cd *U = s + E_U * T, *U0 = s + E_U0 * T, *K = s + E_K * T, *X = s + E_X * T;
    cd *T1 = s + E_T1 * T, *T2 = s + E_T2 * T, *T3 = s + E_T3 * T, *M = s + E_M * T;
    cd *Ue = s + E_UE * T, *Ke = s + E_KE * T, *Xe = s + E_XE * T, *Ye = s + E_YE * T, *Tot = s + E_TOT * T;
    const cd *A = P.PA, *Bm = P.PB;
    const double *xb = H.x + (size_t)b * P.nx;
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) U[t] = Tot[t] = cd{0.0, 0.0};
    __syncthreads();
    for (int cl = 0; cl < H.ncls; ++cl) {
        const int S = H.S[cl], SS = S * S, ns = H.nsec[cl];
        for (int t = threadIdx.x; t < ns * SS; t += blockDim.x) {
            const int w = t / SS, r = (t % SS) / S, c = t % S;
            const int gi = H.sidx[cl][w * S + r], gj = H.sidx[cl][w * S + c];
            if (gi < 0 || gj < 0) continue;
            const size_t bw = (size_t)b * ns + w;
            U[(size_t)gi * D + gj] = H.Ub[cl][bw * SS + r * S + c];
            Tot[(size_t)gi * D + gj] = H.TotS[cl][(bw * ne + e) * SS + r * S + c];
        }
    }
    for (int t = threadIdx.x; t < H.nfixed; t += blockDim.x) {
        const int g = H.fixed[t];
        U[(size_t)g * D + g] = cd{1.0, 0.0};
    }
    __syncthreads();
    build_target(P, nullptr, b, xb, 0, U0);
    bmm<false, false>(Ue, U, Tot, D);  // U_derr = U Tot                (UnitaryCalculations.jl:122-123)
    bmm<true, false>(Ke, U0, Ue, D);
    bmm<true, false>(K, U0, U, D);
    bmm<false, false>(Xe, A, Ke, D);
    const cd te = btrace<SEC_BLOCK>(Xe, D, red);
    bmm<false, false>(Ye, Xe, Bm, D);
    const double t1 = bdot<SEC_BLOCK>(Ye, Ke, D, red);
    bmm<true, false>(T1, Ue, Ue, D);
    double tr = 0.0;  // Re tr(A Ue^dag Ue)
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) {
        const int i = t / D, j = t % D;
        const cd a = A[t], bb = T1[(size_t)j * D + i];
        tr += a.re * bb.re - a.im * bb.im;
    }
    const double t2 = bsum<SEC_BLOCK>(tr, red);
    const double fd2 = 2.0 * (t1 - (1.0 + P.Dtr) * t2 + te.re * te.re + te.im * te.im) / P.DD;
    bmm<false, false>(X, A, K, D);
    bmm<true, false>(T1, Ke, X, D);
    bmm<false, false>(M, Bm, T1, D);
    bmm<true, false>(T1, Xe, K, D);
    bmm<true, false>(T2, Bm, T1, D);
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x) {
        M[t] = p_add(p_add(M[t], T2[t]), p_scale(2.0, p_mul(cd{te.re, -te.im}, X[t])));
        const int i = t / D, j = t % D;
        T2[t] = p_add(A[t], p_conj(A[(size_t)j * D + i]));  // A + A^dagger
    }
    __syncthreads();
    bmm<true, false>(T1, Ue, U, D);
    bmm<false, false>(T3, T2, T1, D);
    for (int t = threadIdx.x; t < (int)T; t += blockDim.x)
        M[t] = p_scale(2.0 / P.DD, p_sub(M[t], p_scale(1.0 + P.Dtr, T3[t])));
    __syncthreads();
    for (int q = 0; q < P.na; ++q) {  // target part of F_d2err_dx_add
        build_target(P, nullptr, b, xb, 1 + q, T1);
        for (int t = threadIdx.x; t < (int)T; t += blockDim.x) T1[t] = p_scale(P.inv_eps, p_sub(T1[t], U0[t]));
        __syncthreads();
        bmm<true, false>(T2, T1, Ue, D);  // Kde
        bmm<false, false>(T1, A, T2, D);
        const cd trd = btrace<SEC_BLOCK>(T1, D, red);
        bmm<false, false>(T3, T1, Bm, D);
        const double sa = bdot<SEC_BLOCK>(T3, Ke, D, red), sb = bdot<SEC_BLOCK>(Ye, T2, D, red);
        const double val = 2.0 * (sa + sb + 2.0 * (te.re * trd.re + te.im * trd.im)) / P.DD;
        if (threadIdx.x == 0) H.Fd2dx[be * P.nx + (size_t)P.np * P.Nt + q] = val;
        __syncthreads();
    }
    if (threadIdx.x == 0) H.Fd2[be] = fd2;
    for (int cl = 0; cl < H.ncls; ++cl) {  // the sector blocks of M_e
        const int S = H.S[cl], SS = S * S, ns = H.nsec[cl];
        for (int t = threadIdx.x; t < ns * SS; t += blockDim.x) {
            const int w = t / SS, r = (t % SS) / S, c = t % S;
            const int gi = H.sidx[cl][w * S + r], gj = H.sidx[cl][w * S + c];
            H.MsecE[cl][(((size_t)b * ns + w) * ne + e) * SS + r * S + c] =
                (gi >= 0 && gj >= 0) ? M[(size_t)gi * D + gj] : cd{0.0, 0.0};
        }
    }
}

}  // namespace


// ---------------------------------------------------------------------------
// Diagonal projector and diagonal target (H.diag: the Rydberg CZ problems).  Every matrix of the
// head is then block-diagonal with the sectors, and k_sec_head's products reduce to sums over
// the sector blocks of U, one THREAD per evaluation (k_sec_head: one wave per evaluation, ten
// LDS-staged d x d products; 0.41 ms of a 4.6-ms C2 pass):
//   K = U0^dag U: K_ij = conj(u0_i) U_ij,   tau = sum_i w_i K_ii,
//   F = [sum_ij w_i p_j |K_ij|^2 + |tau|^2] / DD                      (FidelityCalculations.jl:54)
//   M_ij = 2 [p_i (K^dag W K)_ij + conj(tau) w_i K_ij] / DD   (i, j in one sector; k_sec_head's
//          B (K^dag A K) + B^dag ((A K)^dag K) + 2 conj(tau) A K with A = diag(w), B = diag(p))
//   target part of F_dx_add (:34-40, 67-76), d = (u0(x_add + eps e_q) - u0) / eps:
//   [2 sum_ij w_i p_j Re(conj(d_i) U_ij conj(K_ij)) + 2 Re(conj(tau) sum_i w_i conj(d_i) U_ii)] / DD
// The untouched levels g contribute U_gg = 1.  Sector classes of at most kDiagMaxS levels.
constexpr int kDiagBlock = 64, kDiagMaxS = 4;
// u[i] = diagonal of the target at x_add (perturbed by pp), i < D, in this thread's LDS row
__device__ void target_diag(const grape::DevProblem &P, const double *xb, const grape::Pert &pp, cd *u) {
    const double *xadd = xb + (size_t)P.np * P.Nt;
    for (int i = 0; i < P.D; ++i) u[i] = cd{0.0, 0.0};
    for (int q = 0; q < P.n_tgt; ++q) {
        const grape::Term tm = P.tgt[q];
        const cd c = grape::term_coef(tm, 1, xb, xadd, pp);
        const cd *op = P.ops + (size_t)tm.op * P.D * P.D;
        for (int i = 0; i < P.D; ++i) u[i] = p_add(u[i], p_mul(c, op[(size_t)i * P.D + i]));
    }
}
__device__ __forceinline__ double pdiag(const grape::DevProblem &P, int g) { return P.W[g] != 0.0 ? 1.0 : 0.0; }

// Row-parallel form (latency).  One thread per evaluation spent 25-30 us on a one-evaluation call:
// ~3 k dependent FP64 operations and ~100 dependent LDS / global loads in a single lane.  Now a
// GROUP of G lanes serves one evaluation (G = the sector rows sum_c nsec_c S_c rounded up to a
// power of two: 8 at C2), lane r one row of one sector block; the row sums of F, tau and the
// F_dx_add terms meet in a shuffle tree (fixed order: deterministic), and each lane writes its
// row of M_ww.  The workgroup first copies every table it reads and its evaluations' U blocks and
// x_add values into LDS in one coalesced pass.  Per element the operations are diag_blocks's of
// round 3's first cut (the same K, M and target entries); only the order of the sums over rows
// changed.
__host__ __device__ inline int diag_rows(const SectorHead &H) {
    int n = 0;
    for (int cl = 0; cl < H.ncls; ++cl) n += H.nsec[cl] * H.S[cl];
    return n;
}
__host__ __device__ inline int diag_group(const SectorHead &H) {
    int g = 1;
    while (g < diag_rows(H)) g <<= 1;
    return g;
}
struct DiagLayout {
    size_t terms, tdiag, W, sidx[2], fixed, xa, Ub[2], u, cq, total;
    int G, EB;  // lanes per evaluation, evaluations per workgroup
};
__host__ __device__ inline DiagLayout diag_layout(const SectorHead &H) {
    DiagLayout L{};
    L.G = diag_group(H);
    L.EB = kDiagBlock / L.G;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 15) / 16 * 16;
        return at;
    };
    const grape::DevProblem &P = H.P;
    L.terms = take((size_t)P.n_tgt * sizeof(grape::Term));
    L.tdiag = take((size_t)P.n_tgt * P.D * sizeof(cd));
    L.W = take((size_t)P.D * sizeof(double));
    for (int cl = 0; cl < 2; ++cl) L.sidx[cl] = take(cl < H.ncls ? (size_t)H.nsec[cl] * H.S[cl] * sizeof(int) : 0);
    L.fixed = take((size_t)H.nfixed * sizeof(int));
    L.xa = take((size_t)L.EB * P.na * sizeof(double));
    for (int cl = 0; cl < 2; ++cl)
        L.Ub[cl] = take(cl < H.ncls ? (size_t)L.EB * H.nsec[cl] * H.S[cl] * H.S[cl] * sizeof(cd) : 0);
    L.u = take((size_t)L.EB * 2 * P.D * sizeof(cd));
    L.cq = take((size_t)L.EB * P.n_tgt * sizeof(cd));
    L.total = o;
    return L;
}
struct DiagStage {  // the workgroup's LDS copies
    const grape::Term *terms;  // [n_tgt]
    const cd *tdiag;           // [n_tgt][D]: the diagonal of each target operator
    const double *W;           // [D]
    const int *sidx0, *sidx1;  // [nsec][S] of each class
    const int *fixed;          // [nfixed]
    const cd *Ub0, *Ub1;       // [EB * nsec][S][S] of each class (this workgroup's evaluations)
    // (named fields, picked by value: an array indexed by the class would live in scratch)
    __device__ __forceinline__ const int *sidx(int cl) const { return cl == 0 ? sidx0 : sidx1; }
    __device__ __forceinline__ const cd *Ub(int cl) const { return cl == 0 ? Ub0 : Ub1; }
};
// entry i of the target's diagonal from the term coefficients cq (target_diag's operations)
__device__ __forceinline__ cd target_entry(const grape::DevProblem &P, const DiagStage &St, const cd *cq, int i) {
    cd u{0.0, 0.0};
    for (int q = 0; q < P.n_tgt; ++q) u = p_add(u, p_mul(cq[q], St.tdiag[(size_t)q * P.D + i]));
    return u;
}
// group sum over G lanes (fixed tree)
__device__ __forceinline__ double group_add(double v, int G) {
    for (int o = G >> 1; o >= 1; o >>= 1) v += __shfl_xor(v, o, G);
    return v;
}

// Row r of sector block w of class cl (S levels) of the thread's evaluation (el in the workgroup):
// pass 0: F's row sum and tau's term; pass 1: row r of M_ww; pass 2: the F_dx_add row terms against d
template <int S>
__device__ __forceinline__ void diag_row(const SectorHead &H, const DiagStage &St, int cl, int w, int r, int el, size_t b, int pass,
                         const cd *u0, const cd *d, cd tau, double &fsum, cd &acc) {
    const grape::DevProblem &P = H.P;
    const int ns = H.nsec[cl];
    const double sc = 2.0 / P.DD;
    auto pd = [&](int g) { return St.W[g] != 0.0 ? 1.0 : 0.0; };
    const cd *Ub = St.Ub(cl) + ((size_t)el * ns + w) * S * S;
    int g[S];
#pragma unroll
    for (int k = 0; k < S; ++k) g[k] = St.sidx(cl)[w * S + k];
    const int gr = St.sidx(cl)[w * S + r];
    // K_kc = conj(u0_{g_k}) U_kc (zero on padding slots)
    auto Kel = [&](int k, int gk, int c, int gc) -> cd {
        return (gk >= 0 && gc >= 0) ? p_mul(p_conj(u0[gk >= 0 ? gk : 0]), Ub[k * S + c]) : cd{0.0, 0.0};
    };
    if (pass == 0) {
        if (gr < 0) return;
        const double wr = St.W[gr];
#pragma unroll
        for (int c = 0; c < S; ++c) {
            if (g[c] < 0) continue;
            const cd K = Kel(r, gr, c, g[c]);
            fsum += wr * pd(g[c]) * (K.re * K.re + K.im * K.im);
        }
        acc = p_add(acc, p_scale(wr, Kel(r, gr, r, gr)));
    } else if (pass == 1) {
        cd *dst = H.Msec[cl] + (b * ns + w) * S * S + (size_t)r * S;
        cd Kr[S];  // column r of K
#pragma unroll
        for (int k = 0; k < S; ++k) Kr[k] = Kel(k, g[k], r, gr);
#pragma unroll
        for (int c = 0; c < S; ++c) {
            cd m{0.0, 0.0};
            if (gr >= 0 && g[c] >= 0) {
                cd s{0.0, 0.0};
#pragma unroll
                for (int k = 0; k < S; ++k)
                    if (g[k] >= 0) s = p_add(s, p_scale(St.W[g[k]], p_mul(p_conj(Kr[k]), Kel(k, g[k], c, g[c]))));
                m = p_scale(sc, p_add(p_scale(pd(gr), s), p_scale(St.W[gr], p_mul(cd{tau.re, -tau.im}, Kel(r, gr, c, g[c])))));
            }
            dst[c] = m;
        }
    } else {
        if (gr < 0) return;
        const double wr = St.W[gr];
        const cd dr = p_conj(d[gr]);
#pragma unroll
        for (int c = 0; c < S; ++c) {
            if (g[c] < 0) continue;
            const cd kd = p_mul(dr, Ub[r * S + c]);  // Kd_rc
            const cd K = Kel(r, gr, c, g[c]);
            fsum += wr * pd(g[c]) * (kd.re * K.re + kd.im * K.im);
        }
        acc = p_add(acc, p_scale(wr, p_mul(dr, Ub[r * S + r])));
    }
}
__device__ __forceinline__ void diag_row_any(const SectorHead &H, const DiagStage &St, int row, int el, size_t b, int pass,
                             const cd *u0, const cd *d, cd tau, double &fsum, cd &acc) {
    int cl = 0;
    if (row >= H.nsec[0] * H.S[0]) {
        row -= H.nsec[0] * H.S[0];
        cl = 1;
        if (cl >= H.ncls || row >= H.nsec[1] * H.S[1]) return;  // padding lane of the group
    }
    const int S = H.S[cl], w = row / S, r = row - w * S;
    switch (S) {
    case 2: diag_row<2>(H, St, cl, w, r, el, b, pass, u0, d, tau, fsum, acc); break;
    case 3: diag_row<3>(H, St, cl, w, r, el, b, pass, u0, d, tau, fsum, acc); break;
    default: diag_row<4>(H, St, cl, w, r, el, b, pass, u0, d, tau, fsum, acc); break;
    }
}

__global__ __launch_bounds__(kDiagBlock) void k_sec_head_diag(SectorHead H, int nb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char diag_smem[];
    const grape::DevProblem &P = H.P;
    const DiagLayout Lo = diag_layout(H);
    const int G = Lo.G, EB = Lo.EB;
    const int t = threadIdx.x, el = t / G, row = t - el * G;
    const int b0 = blockIdx.x * EB, nloc = min(EB, nb - b0);
    // stage (every thread of the workgroup; coalesced where the source is contiguous)
    {
        grape::Term *terms = reinterpret_cast<grape::Term *>(diag_smem + Lo.terms);
        cd *tdiag = reinterpret_cast<cd *>(diag_smem + Lo.tdiag);
        const int nti = P.n_tgt * (int)(sizeof(grape::Term) / sizeof(int));
        for (int i = t; i < nti; i += kDiagBlock)
            reinterpret_cast<int *>(terms)[i] = reinterpret_cast<const int *>(P.tgt)[i];
        for (int i = t; i < P.n_tgt * P.D; i += kDiagBlock) {
            const int q = i / P.D, j = i - q * P.D;
            tdiag[i] = P.ops[((size_t)P.tgt[q].op * P.D + j) * P.D + j];
        }
        double *W = reinterpret_cast<double *>(diag_smem + Lo.W);
        for (int i = t; i < P.D; i += kDiagBlock) W[i] = P.W[i];
        for (int cl = 0; cl < H.ncls; ++cl) {
            // (offsets picked by value: a layout array indexed by the class would live in scratch)
            int *sx = reinterpret_cast<int *>(diag_smem + (cl == 0 ? Lo.sidx[0] : Lo.sidx[1]));
            for (int i = t; i < H.nsec[cl] * H.S[cl]; i += kDiagBlock) sx[i] = H.sidx[cl][i];
            const size_t SS = (size_t)H.S[cl] * H.S[cl], n = (size_t)nloc * H.nsec[cl] * SS;
            const cd *src = H.Ub[cl] + (size_t)b0 * H.nsec[cl] * SS;
            cd *ub = reinterpret_cast<cd *>(diag_smem + (cl == 0 ? Lo.Ub[0] : Lo.Ub[1]));
            for (size_t i = t; i < n; i += kDiagBlock) ub[i] = src[i];
        }
        int *fx = reinterpret_cast<int *>(diag_smem + Lo.fixed);
        for (int i = t; i < H.nfixed; i += kDiagBlock) fx[i] = H.fixed[i];
        double *xa = reinterpret_cast<double *>(diag_smem + Lo.xa);
        for (int i = t; i < nloc * P.na; i += kDiagBlock) {
            const int l = i / P.na, q = i - l * P.na;
            xa[i] = H.x[(size_t)(b0 + l) * P.nx + (size_t)P.np * P.Nt + q];
        }
    }
    __syncthreads();
    DiagStage St;
    St.terms = reinterpret_cast<const grape::Term *>(diag_smem + Lo.terms);
    St.tdiag = reinterpret_cast<const cd *>(diag_smem + Lo.tdiag);
    St.W = reinterpret_cast<const double *>(diag_smem + Lo.W);
    St.fixed = reinterpret_cast<const int *>(diag_smem + Lo.fixed);
    St.sidx0 = reinterpret_cast<const int *>(diag_smem + Lo.sidx[0]);
    St.sidx1 = reinterpret_cast<const int *>(diag_smem + Lo.sidx[1]);
    St.Ub0 = reinterpret_cast<const cd *>(diag_smem + Lo.Ub[0]);
    St.Ub1 = reinterpret_cast<const cd *>(diag_smem + Lo.Ub[1]);
    const bool ok = el < nloc;  // group-uniform
    const size_t b = (size_t)b0 + (ok ? el : 0);
    cd *u0 = reinterpret_cast<cd *>(diag_smem + Lo.u) + (size_t)el * 2 * P.D, *d = u0 + P.D;
    const double *xb = H.x + b * P.nx;
    const double *xadd = reinterpret_cast<const double *>(diag_smem + Lo.xa) + (size_t)(ok ? el : 0) * P.na;
    grape::Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    // the target's term coefficients (one lane per term), then its diagonal (one lane per entry)
    cd *cq = reinterpret_cast<cd *>(diag_smem + Lo.cq) + (size_t)el * P.n_tgt;
    if (ok)
        for (int q = row; q < P.n_tgt; q += G) cq[q] = grape::term_coef(St.terms[q], 1, xb, xadd, none);
    __syncthreads();
    if (ok)
        for (int i = row; i < P.D; i += G) u0[i] = target_entry(P, St, cq, i);
    __syncthreads();
    double fsum = 0.0;
    cd tau{0.0, 0.0};
    if (ok) diag_row_any(H, St, row, el, b, 0, u0, d, tau, fsum, tau);
    fsum = group_add(fsum, G);
    tau.re = group_add(tau.re, G);
    tau.im = group_add(tau.im, G);
    for (int q = 0; q < H.nfixed; ++q) {  // U_gg = 1: K_gg = conj(u0_g)
        const int g = St.fixed[q];
        const cd k = p_conj(u0[g]);
        fsum += St.W[g] * (St.W[g] != 0.0 ? 1.0 : 0.0) * (k.re * k.re + k.im * k.im);
        tau = p_add(tau, p_scale(St.W[g], k));
    }
    if (ok && row == 0) H.F[b] = (fsum + tau.re * tau.re + tau.im * tau.im) / P.DD;
    double unused = 0.0;
    cd unused_c{0.0, 0.0};
    if (ok) diag_row_any(H, St, row, el, b, 1, u0, d, tau, unused, unused_c);
    for (int q = 0; q < P.na; ++q) {  // target part of F_dx_add
        grape::Pert pq;
        pq.var = grape::VAR_XADD;
        pq.index = q;
        pq.delta = P.eps;
        __syncthreads();  // every lane is done with the previous d and cq
        if (ok)
            for (int k = row; k < P.n_tgt; k += G) cq[k] = grape::term_coef(St.terms[k], 1, xb, xadd, pq);
        __syncthreads();
        if (ok)
            for (int i = row; i < P.D; i += G) d[i] = p_scale(P.inv_eps, p_sub(target_entry(P, St, cq, i), u0[i]));
        __syncthreads();
        double sa = 0.0;
        cd trd{0.0, 0.0};
        if (ok) diag_row_any(H, St, row, el, b, 2, u0, d, tau, sa, trd);
        sa = group_add(sa, G);
        trd.re = group_add(trd.re, G);
        trd.im = group_add(trd.im, G);
        for (int r = 0; r < H.nfixed; ++r) {
            const int g = St.fixed[r];
            const cd kd = p_conj(d[g]), k = p_conj(u0[g]);
            sa += St.W[g] * (St.W[g] != 0.0 ? 1.0 : 0.0) * (kd.re * k.re + kd.im * k.im);
            trd = p_add(trd, p_scale(St.W[g], kd));
        }
        const double val = (2.0 * sa + 2.0 * (tau.re * trd.re + tau.im * trd.im)) / P.DD;
        if (ok && row == 0) {
            if (P.xadd_dep && H.tgt_part) H.tgt_part[b * P.na + q] = val;
            else H.Fdx[b * P.nx + (size_t)P.np * P.Nt + q] = val;
        }
    }
}

// The error head in the same diagonal form, one thread per (evaluation, error source): with
// Ue = U Tot (block-diagonal, zero on the untouched levels), Ke = U0^dag Ue and K = U0^dag U,
// k_sec_err_head's products reduce to (A = diag(w), B = diag(p); FidelityCalculations.jl:78-113)
//   te = sum_i w_i Ke_ii,  t1 = sum_ij w_i p_j |Ke_ij|^2,  t2 = sum_i w_i (Ue^dag Ue)_ii,
//   F_d2err = 2 [t1 - (1 + D) t2 + |te|^2] / DD,
//   M_e,ij = (2/DD) [2 p_i (Ke^dag W K)_ij + 2 conj(te) w_i K_ij - 2 (1 + D) w_i (Ue^dag U)_ij],
//   target part of F_d2err_dx_add: 2 [2 sum_ij w_i p_j Re(conj(d_i) Ue_ij conj(Ke_ij))
//                                     + 2 Re(conj(te) sum_i w_i conj(d_i) Ue_ii)] / DD.
// pass 0: te, t1, t2; pass 1: the blocks of M_e; pass 2: the F_d2err_dx_add sums against d.
template <int S>
__device__ void diag_err_blocks(const SectorHead &H, int cl, int b, int e, int pass, const cd *u0, const cd *d, cd te,
                                double &t1, double &t2, cd &acc) {
    const grape::DevProblem &P = H.P;
    const int ns = H.nsec[cl], ne = P.ne;
    const double sc = 2.0 / P.DD;
    for (int w = 0; w < ns; ++w) {
        const size_t bw = (size_t)b * ns + w;
        const cd *Ub = H.Ub[cl] + bw * S * S, *Tb = H.TotS[cl] + (bw * ne + e) * S * S;
        int g[S];
#pragma unroll
        for (int r = 0; r < S; ++r) g[r] = H.sidx[cl][w * S + r];
        cd Ue[S][S];
#pragma unroll
        for (int r = 0; r < S; ++r) {
#pragma unroll
            for (int c = 0; c < S; ++c) {
                cd v{0.0, 0.0};
#pragma unroll
                for (int m = 0; m < S; ++m) v = p_add(v, p_mul(Ub[r * S + m], Tb[m * S + c]));
                Ue[r][c] = (g[r] >= 0 && g[c] >= 0) ? v : cd{0.0, 0.0};
            }
        }
        auto cu0 = [&](int r) { return p_conj(u0[g[r] >= 0 ? g[r] : 0]); };
        if (pass == 0) {
#pragma unroll
            for (int r = 0; r < S; ++r) {
                if (g[r] < 0) continue;
                const double wr = P.W[g[r]];
                double col = 0.0;  // (Ue^dag Ue)_rr
#pragma unroll
                for (int c = 0; c < S; ++c) {
                    if (g[c] < 0) continue;
                    const cd ke = p_mul(cu0(r), Ue[r][c]);
                    t1 += wr * pdiag(P, g[c]) * (ke.re * ke.re + ke.im * ke.im);
                    col += Ue[c][r].re * Ue[c][r].re + Ue[c][r].im * Ue[c][r].im;
                }
                t2 += wr * col;
                acc = p_add(acc, p_scale(wr, p_mul(cu0(r), Ue[r][r])));
            }
        } else if (pass == 1) {
            cd *dst = H.MsecE[cl] + (bw * ne + e) * S * S;
#pragma unroll
            for (int r = 0; r < S; ++r) {
#pragma unroll
                for (int c = 0; c < S; ++c) {
                    cd m{0.0, 0.0};
                    if (g[r] >= 0 && g[c] >= 0) {
                        cd kwk{0.0, 0.0}, uu{0.0, 0.0};  // (Ke^dag W K)_rc, (Ue^dag U)_rc
#pragma unroll
                        for (int k = 0; k < S; ++k) {
                            if (g[k] < 0) continue;
                            const cd kk = p_mul(cu0(k), Ub[k * S + c]), ke = p_mul(cu0(k), Ue[k][r]);
                            kwk = p_add(kwk, p_scale(P.W[g[k]], p_mul(p_conj(ke), kk)));
                            uu = p_add(uu, p_mul(p_conj(Ue[k][r]), Ub[k * S + c]));
                        }
                        const double wr = P.W[g[r]];
                        const cd krc = p_mul(cu0(r), Ub[r * S + c]);
                        m = p_add(p_scale(2.0 * pdiag(P, g[r]), kwk), p_scale(2.0 * wr, p_mul(cd{te.re, -te.im}, krc)));
                        m = p_scale(sc, p_sub(m, p_scale(2.0 * (1.0 + P.Dtr) * wr, uu)));
                    }
                    dst[r * S + c] = m;
                }
            }
        } else {
#pragma unroll
            for (int r = 0; r < S; ++r) {
                if (g[r] < 0) continue;
                const double wr = P.W[g[r]];
                const cd dr = p_conj(d[g[r]]);
#pragma unroll
                for (int c = 0; c < S; ++c) {
                    if (g[c] < 0) continue;
                    const cd kde = p_mul(dr, Ue[r][c]), ke = p_mul(cu0(r), Ue[r][c]);
                    t1 += wr * pdiag(P, g[c]) * (kde.re * ke.re + kde.im * ke.im);
                }
                acc = p_add(acc, p_scale(wr, p_mul(dr, Ue[r][r])));
            }
        }
    }
}
__device__ void diag_err_class(const SectorHead &H, int cl, int b, int e, int pass, const cd *u0, const cd *d, cd te,
                               double &t1, double &t2, cd &acc) {
    switch (H.S[cl]) {
    case 2: diag_err_blocks<2>(H, cl, b, e, pass, u0, d, te, t1, t2, acc); break;
    case 3: diag_err_blocks<3>(H, cl, b, e, pass, u0, d, te, t1, t2, acc); break;
    default: diag_err_blocks<4>(H, cl, b, e, pass, u0, d, te, t1, t2, acc); break;
    }
}

__global__ __launch_bounds__(kDiagBlock) void k_sec_err_head_diag(SectorHead H, int nb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char diag_smem[];
    const grape::DevProblem &P = H.P;
    const int be = blockIdx.x * kDiagBlock + threadIdx.x;
    if (be >= nb * P.ne) return;
    const int b = be / P.ne, e = be - b * P.ne;
    cd *u0 = reinterpret_cast<cd *>(diag_smem) + (size_t)threadIdx.x * 2 * P.D, *d = u0 + P.D;
    const double *xb = H.x + (size_t)b * P.nx;
    grape::Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    target_diag(P, xb, none, u0);
    double t1 = 0.0, t2 = 0.0;
    cd te{0.0, 0.0};
    for (int cl = 0; cl < H.ncls; ++cl) diag_err_class(H, cl, b, e, 0, u0, d, te, t1, t2, te);
    H.Fd2[be] = 2.0 * (t1 - (1.0 + P.Dtr) * t2 + te.re * te.re + te.im * te.im) / P.DD;
    double u1 = 0.0, u2 = 0.0;
    cd uc{0.0, 0.0};
    for (int cl = 0; cl < H.ncls; ++cl) diag_err_class(H, cl, b, e, 1, u0, d, te, u1, u2, uc);
    for (int q = 0; q < P.na; ++q) {  // target part of F_d2err_dx_add
        grape::Pert pq;
        pq.var = grape::VAR_XADD;
        pq.index = q;
        pq.delta = P.eps;
        target_diag(P, xb, pq, d);
        for (int i = 0; i < P.D; ++i) d[i] = p_scale(P.inv_eps, p_sub(d[i], u0[i]));
        double sa = 0.0, unused = 0.0;
        cd trd{0.0, 0.0};
        for (int cl = 0; cl < H.ncls; ++cl) diag_err_class(H, cl, b, e, 2, u0, d, te, sa, unused, trd);
        H.Fd2dx[(size_t)be * P.nx + (size_t)P.np * P.Nt + q] = 2.0 * (2.0 * sa + 2.0 * (te.re * trd.re + te.im * trd.im)) / P.DD;
    }
}

// Row-parallel form of k_sec_err_head_diag (round 6, latency): one group of G lanes per (evaluation, error
// source), lane = row r of one sector block, as k_sec_head_diag.  Pass 0 forms row r of Ue = U Tot and its
// terms of te, t1, t2 (t2 regrouped by rows: sum_rc w_c |Ue_rc|^2), a shuffle tree sums them; row r of Ue
// goes to LDS, and pass 1 writes row r of M_e from the block's columns; pass 2 the F_d2err_dx_add row terms.
// Lane 0 of the group forms the target's diagonal (target_diag).  The per-element operations are
// diag_err_blocks's; only the order of the sums over rows changed.  One C3 evaluation: 36.9 us in one lane.
#ifndef GRAPE_ERR_HEAD_ROWS
#define GRAPE_ERR_HEAD_ROWS 1
#endif
template <int S>
__device__ void err_row(const SectorHead &H, int cl, int w, int r, size_t b, int e, int pass, const cd *u0, const cd *d,
                        cd te, cd *ue, double &t1, double &t2, cd &acc) {
    const grape::DevProblem &P = H.P;
    const int ns = H.nsec[cl], ne = P.ne;
    const double sc = 2.0 / P.DD;
    const size_t bw = b * ns + w;
    const cd *Ub = H.Ub[cl] + bw * S * S;
    int g[S];
#pragma unroll
    for (int k = 0; k < S; ++k) g[k] = H.sidx[cl][w * S + k];
    const int gr = g[r];
    auto cu0 = [&](int k) { return p_conj(u0[g[k] >= 0 ? g[k] : 0]); };
    if (pass == 0) {
        const cd *Tb = H.TotS[cl] + (bw * ne + e) * S * S;
        cd Ur[S];
#pragma unroll
        for (int c = 0; c < S; ++c) {
            cd v{0.0, 0.0};
#pragma unroll
            for (int m = 0; m < S; ++m) v = p_add(v, p_mul(Ub[r * S + m], Tb[m * S + c]));
            Ur[c] = (gr >= 0 && g[c] >= 0) ? v : cd{0.0, 0.0};
            ue[r * S + c] = Ur[c];
        }
        if (gr < 0) return;
        const double wr = P.W[gr];
#pragma unroll
        for (int c = 0; c < S; ++c) {
            if (g[c] < 0) continue;
            const cd ke = p_mul(cu0(r), Ur[c]);
            t1 += wr * pdiag(P, g[c]) * (ke.re * ke.re + ke.im * ke.im);
            t2 += P.W[g[c]] * (Ur[c].re * Ur[c].re + Ur[c].im * Ur[c].im);
        }
        acc = p_add(acc, p_scale(wr, p_mul(cu0(r), Ur[r])));
    } else if (pass == 1) {
        cd *dst = H.MsecE[cl] + (bw * ne + e) * S * S + (size_t)r * S;
#pragma unroll
        for (int c = 0; c < S; ++c) {
            cd m{0.0, 0.0};
            if (gr >= 0 && g[c] >= 0) {
                cd kwk{0.0, 0.0}, uu{0.0, 0.0};  // (Ke^dag W K)_rc, (Ue^dag U)_rc
#pragma unroll
                for (int k = 0; k < S; ++k) {
                    if (g[k] < 0) continue;
                    const cd kk = p_mul(cu0(k), Ub[k * S + c]), ke = p_mul(cu0(k), ue[k * S + r]);
                    kwk = p_add(kwk, p_scale(P.W[g[k]], p_mul(p_conj(ke), kk)));
                    uu = p_add(uu, p_mul(p_conj(ue[k * S + r]), Ub[k * S + c]));
                }
                const double wr = P.W[gr];
                const cd krc = p_mul(cu0(r), Ub[r * S + c]);
                m = p_add(p_scale(2.0 * pdiag(P, gr), kwk), p_scale(2.0 * wr, p_mul(cd{te.re, -te.im}, krc)));
                m = p_scale(sc, p_sub(m, p_scale(2.0 * (1.0 + P.Dtr) * wr, uu)));
            }
            dst[c] = m;
        }
    } else {
        if (gr < 0) return;
        const double wr = P.W[gr];
        const cd dr = p_conj(d[gr]);
#pragma unroll
        for (int c = 0; c < S; ++c) {
            if (g[c] < 0) continue;
            const cd kde = p_mul(dr, ue[r * S + c]), ke = p_mul(cu0(r), ue[r * S + c]);
            t1 += wr * pdiag(P, g[c]) * (kde.re * ke.re + kde.im * ke.im);
        }
        acc = p_add(acc, p_scale(wr, p_mul(dr, ue[r * S + r])));
    }
}
__device__ __forceinline__ void err_row_any(const SectorHead &H, int row, size_t b, int e, int pass, const cd *u0,
                                            const cd *d, cd te, cd *ue_grp, double &t1, double &t2, cd &acc) {
    int cl = 0;
    cd *ue = ue_grp;
    if (row >= H.nsec[0] * H.S[0]) {
        row -= H.nsec[0] * H.S[0];
        ue += (size_t)H.nsec[0] * H.S[0] * H.S[0];
        cl = 1;
        if (cl >= H.ncls || row >= H.nsec[1] * H.S[1]) return;  // padding lane of the group
    }
    const int S = H.S[cl], w = row / S, r = row - w * S;
    ue += (size_t)w * S * S;
    switch (S) {
    case 2: err_row<2>(H, cl, w, r, b, e, pass, u0, d, te, ue, t1, t2, acc); break;
    case 3: err_row<3>(H, cl, w, r, b, e, pass, u0, d, te, ue, t1, t2, acc); break;
    default: err_row<4>(H, cl, w, r, b, e, pass, u0, d, te, ue, t1, t2, acc); break;
    }
}
__host__ __device__ inline size_t err_rows_group_cd(const SectorHead &H) {  // per group: u0, d, the Ue blocks
    size_t n = 2 * (size_t)H.P.D;
    for (int cl = 0; cl < H.ncls; ++cl) n += (size_t)H.nsec[cl] * H.S[cl] * H.S[cl];
    return n;
}
__global__ __launch_bounds__(kDiagBlock) void k_sec_err_head_rows(SectorHead H, int nb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char diag_smem[];
    const grape::DevProblem &P = H.P;
    const int G = diag_group(H), EB = kDiagBlock / G;
    const int t = threadIdx.x, el = t / G, row = t - el * G;
    const int be = blockIdx.x * EB + el;
    const bool ok = be < nb * P.ne;  // (group-uniform; every lane reaches every barrier)
    const int bb = ok ? be : 0, b = bb / P.ne, e = bb - b * P.ne;
    cd *u0 = reinterpret_cast<cd *>(diag_smem) + (size_t)el * err_rows_group_cd(H), *d = u0 + P.D, *ue = d + P.D;
    const double *xb = H.x + (size_t)b * P.nx;
    grape::Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    if (ok && row == 0) target_diag(P, xb, none, u0);
    __syncthreads();
    double t1 = 0.0, t2 = 0.0;
    cd te{0.0, 0.0};
    if (ok) err_row_any(H, row, b, e, 0, u0, d, te, ue, t1, t2, te);
    t1 = group_add(t1, G);
    t2 = group_add(t2, G);
    te.re = group_add(te.re, G);
    te.im = group_add(te.im, G);
    if (ok && row == 0) H.Fd2[be] = 2.0 * (t1 - (1.0 + P.Dtr) * t2 + te.re * te.re + te.im * te.im) / P.DD;
    __syncthreads();  // the group's Ue rows
    double u1 = 0.0, u2 = 0.0;
    cd uc{0.0, 0.0};
    if (ok) err_row_any(H, row, b, e, 1, u0, d, te, ue, u1, u2, uc);
    for (int q = 0; q < P.na; ++q) {  // target part of F_d2err_dx_add
        grape::Pert pq;
        pq.var = grape::VAR_XADD;
        pq.index = q;
        pq.delta = P.eps;
        __syncthreads();
        if (ok && row == 0) {
            target_diag(P, xb, pq, d);
            for (int i = 0; i < P.D; ++i) d[i] = p_scale(P.inv_eps, p_sub(d[i], u0[i]));
        }
        __syncthreads();
        double sa = 0.0, unused = 0.0;
        cd trd{0.0, 0.0};
        if (ok) err_row_any(H, row, b, e, 2, u0, d, te, ue, sa, unused, trd);
        sa = group_add(sa, G);
        trd.re = group_add(trd.re, G);
        trd.im = group_add(trd.im, G);
        if (ok && row == 0)
            H.Fd2dx[(size_t)be * P.nx + (size_t)P.np * P.Nt + q] = 2.0 * (2.0 * sa + 2.0 * (te.re * trd.re + te.im * trd.im)) / P.DD;
    }
}

hipError_t launch_sector_err_head(const SectorHead &H, int nb, hipStream_t st) {
    if (H.P.ne == 0) return hipSuccess;
    if (H.diag && GRAPE_ERR_HEAD_ROWS && diag_group(H) <= kDiagBlock) {
        const int G = diag_group(H), EB = kDiagBlock / G, n = nb * H.P.ne;
        const size_t lds = (size_t)EB * err_rows_group_cd(H) * sizeof(cd);
        hipLaunchKernelGGL(k_sec_err_head_rows, dim3((unsigned)((n + EB - 1) / EB)), dim3(kDiagBlock), lds, st, H, nb);
        return hipGetLastError();
    }
    if (H.diag) {
        const int n = nb * H.P.ne;
        const size_t lds = (size_t)kDiagBlock * 2 * H.P.D * sizeof(cd);
        hipLaunchKernelGGL(k_sec_err_head_diag, dim3((unsigned)((n + kDiagBlock - 1) / kDiagBlock)), dim3(kDiagBlock),
                           lds, st, H, nb);
        return hipGetLastError();
    }
    const size_t lds = (size_t)kErrHeadSlots * H.P.D * H.P.D * sizeof(cd);
    hipLaunchKernelGGL(k_sec_err_head, dim3((unsigned)(nb * H.P.ne)), dim3(SEC_BLOCK), lds, st, H);
    return hipGetLastError();
}

hipError_t launch_sector_head(const SectorHead &H, int nb, hipStream_t st) {
    if (H.diag) {
        const DiagLayout L = diag_layout(H);  // G lanes per evaluation (G <= 16: d <= 12, sectors of <= 4 levels)
        hipLaunchKernelGGL(k_sec_head_diag, dim3((unsigned)((nb + L.EB - 1) / L.EB)), dim3(kDiagBlock), L.total, st, H,
                           nb);
        return hipGetLastError();
    }
    const size_t lds = (size_t)kHeadSlots * H.P.D * H.P.D * sizeof(cd);
    hipLaunchKernelGGL(k_sec_head, dim3((unsigned)nb), dim3(SEC_BLOCK), lds, st, H);
    return hipGetLastError();
}

hipError_t launch_fid_head(const Heads &H, int nb, hipStream_t st) {
    hipLaunchKernelGGL(k_proj_fid, dim3((unsigned)nb), dim3(BLOCK), 0, st, H);
    return hipGetLastError();
}

hipError_t launch_err_head(const Heads &H, int nb, hipStream_t st) {
    if (H.P.ne == 0) return hipSuccess;
    hipLaunchKernelGGL(k_proj_err, dim3((unsigned)(nb * H.P.ne)), dim3(BLOCK), 0, st, H);
    return hipGetLastError();
}

}  // namespace grape_proj
