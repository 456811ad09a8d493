// grape_dense.hip -- the dense engine's kernels (13 <= d <= 64, padded to 64):
//
//   k_dexp    one workgroup per (eval b, step k): A_k = -i dt H(x_b,k) from the
//             operator basis, E_k = exp(A_k) on MFMA.      UnitaryCalculations.jl:45
//   k_dscan   one workgroup per (b, chunk c): chunk-local prefix products
//             Q_k = E_k Q_{k-1} (Q = E at a chunk start).  UnitaryCalculations.jl:46-47
//   k_dcarry  one workgroup per b: carries Carry_c = Q_{end(c-1)} Carry_{c-1},
//             U = C_Nt, fidelity F, gradient kernel M = G U and the target
//             derivative part of F_dx_add.              FidelityCalculations.jl:32-54,67-76
//   k_dmc     one workgroup per (b, c): M'_c = Carry_c M Carry_c^dagger
//   k_dgrad   one workgroup per (b, k): Z_k = Y_k^T = conj(Q_k) (Q_{k-1} M'_c)^T,
//             then for every control p the eps-variant exponential E' and
//             F_dx[p,k] = Re sum(Z_k o (E' - E_k)/eps).   UnitaryCalculations.jl:48-52,
//                                                        FidelityCalculations.jl:56-65
// With error sources (the algebra of grape_errpath.hpp on 64 x 64 images):
//   k_dexp       every propagator variant of every step (nominal, eps / eps2 controls,
//                error eps / eps2, mixed)                 UnitaryCalculations.jl:45-83
//   k_dlocal     one workgroup per (b, k, slot): the local-frame image Q_k^dag dX Q_{k-1}
//                of one difference dX (Z1_u, W_e, Z2_{e,u}), stored transposed; F_dx
//   k_dwsum      one workgroup per (b, e, c): Carry_c^dag (sum over chunk c of W) Carry_c
//   k_derr_scan  one workgroup per (b, e): prefix over chunks, U_derr, F_d2err, M_e = G_e U,
//                target part of F_d2err_dx_add            FidelityCalculations.jl:78-113
//   k_dmce       one workgroup per (b, e, c): M' = Carry M_e Carry^dag, B at the chunk start
//   k_derr_grad  one workgroup per (b, c, e): walks the chunk carrying B_k, two products per
//                step; F_d2err_dx                         UnitaryCalculations.jl:124-139
// (algebra: grape_kernels.hpp and grape_errpath.hpp headers; layouts and numerics:
// grape_dense.hpp).
#include "grape_dense.hpp"
#include "grape_dense_api.hpp"

namespace grape_dense {

namespace {

constexpr grape::Pert kNoPert = {-1, 0, 0.0};

// A = -i dt (sum_t c_t OP_t) for step k of eval b, one variable perturbed
__device__ __forceinline__ void build_generator(const DenseProblem &DP, const double *xb, int k, const grape::Pert &pp,
                                                HM &A, const Lane &ln) {
    const grape::DevProblem &P = DP.P;
    const double *xk = xb + (size_t)k * P.np;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    hm_zero(A);
    for (int t = 0; t < P.n_h0; ++t) {
        const Term tm = P.h0[t];
        const cd c = grape::term_coef(tm, k + 1, xk, xadd, pp);
        const cd g = grape::cmake(P.dt * c.im, -(P.dt * c.re));  // -i dt c
        hm_cmac_img(A, g, DP.opimg + (size_t)tm.op * IMG, ln);
    }
}

// A = -i dt (H0 + errval Herror_e) of propagator variant v (grape::VSpec) for step k of eval b
// (UnitaryCalculations.jl:45-90: the perturbed variable in both, H0's terms first)
__device__ __forceinline__ void build_variant(const DenseProblem &DP, const double *xb, int k, const grape::VSpec &vs,
                                              HM &A, const Lane &ln) {
    const grape::DevProblem &P = DP.P;
    const double *xk = xb + (size_t)k * P.np;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    hm_zero(A);
    for (int t = 0; t < P.n_h0; ++t) {
        const Term tm = P.h0[t];
        const cd c = grape::term_coef(tm, k + 1, xk, xadd, vs.pert);
        hm_cmac_img(A, grape::cmake(P.dt * c.im, -(P.dt * c.re)), DP.opimg + (size_t)tm.op * IMG, ln);
    }
    if (vs.err >= 0) {
        for (int t = P.err_off[vs.err]; t < P.err_off[vs.err + 1]; ++t) {
            const Term tm = P.err[t];
            const cd c = grape::cscale(vs.errval, grape::term_coef(tm, k + 1, xk, xadd, vs.pert));
            hm_cmac_img(A, grape::cmake(P.dt * c.im, -(P.dt * c.re)), DP.opimg + (size_t)tm.op * IMG, ln);
        }
    }
}

// M += c X (images in registers), elementwise
__device__ __forceinline__ void hm_acc(HM &M, double c, const HM &X) { hm_axpy(M, c, X); }
__device__ __forceinline__ void hm_sub(HM &M, const HM &X) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        M.re[i] -= X.re[i];
        M.im[i] -= X.im[i];
    }
}
__device__ __forceinline__ void hm_add(HM &M, const HM &X) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        M.re[i] += X.re[i];
        M.im[i] += X.im[i];
    }
}
// Re sum_ij A_ij B_ij over the workgroup (the trace of A B^T)
__device__ __forceinline__ double hm_dot_re(const HM &A, const HM &Bm) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc += A.re[i][r] * Bm.re[i][r] - A.im[i][r] * Bm.im[i][r];
    return acc;
}

// U0(x_add (+ eps e_q)) from the target terms
__device__ __forceinline__ void build_target(const DenseProblem &DP, const double *xb, const grape::Pert &pp, HM &T,
                                             const Lane &ln) {
    const grape::DevProblem &P = DP.P;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    hm_zero(T);
    for (int t = 0; t < P.n_tgt; ++t) {
        const Term tm = P.tgt[t];
        const cd c = grape::term_coef(tm, 1, xadd, xadd, pp);
        hm_cmac_img(T, c, DP.opimg + (size_t)tm.op * IMG, ln);
    }
}

__device__ __forceinline__ void note_m(int *mstats, int m) {
    if (mstats && threadIdx.x == 0) atomicAdd(mstats + m_index(m), 1);
}

__global__ __launch_bounds__(NTHREADS, 1) void k_dexp(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const long item = blockIdx.x;  // (b, k, v), v fastest; E[b][k][v]
    const int v = (int)(item % P.nv), k = (int)((item / P.nv) % P.Nt), b = (int)(item / ((long)P.nv * P.Nt));
    HM X;
    const double *xb = B.x + (size_t)b * P.nx;
    bool singular = false;
    const grape::VSpec vs = P.vs[v];
    const int m = wg_expm([&](HM &A) { build_variant(DP, xb, k, vs, A, ln); }, X, lds, ln, singular);
    img_store(B.E + (size_t)item * IMG, X, ln);
    if (singular) atomicOr(B.status, 1);
    note_m(B.mstats, m);
}

__global__ __launch_bounds__(NTHREADS, 1) void k_dexp_raw(const double *Ain, double *Eout, int *status, int *mstats) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    HM X;
    const double *src = Ain + (size_t)blockIdx.x * IMG;
    bool singular = false;
    const int m = wg_expm([&](HM &A) { img_load(src, A, ln); }, X, lds, ln, singular);
    img_store(Eout + (size_t)blockIdx.x * IMG, X, ln);
    if (singular) atomicOr(status, 1);
    note_m(mstats, m);
}

// chunk-local prefix products Q_k = E_k Q_{k-1}
__global__ __launch_bounds__(NTHREADS, 1) void k_dscan(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const int b = blockIdx.x / DP.Nc, c = blockIdx.x % DP.Nc;
    const int k0 = c * DP.Lc, k1 = min(k0 + DP.Lc, P.Nt);
    if (k0 >= k1) return;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    const size_t base = (size_t)b * P.Nt;
    HM Qm, Ek;
    const size_t nv = P.nv;  // nominal propagator: variant 0 of each step
    img_load(B.E + (base + k0) * nv * IMG, Qm, ln);
    img_store(B.Q + (base + k0) * IMG, Qm, ln);
    for (int k = k0 + 1; k < k1; ++k) {
        img_load(B.E + (base + k) * nv * IMG, Ek, ln);
        __syncthreads();  // previous product done reading
        sm_store(S0, Ek, ln);
        sm_store(S1, Qm, ln);
        __syncthreads();
        hm_zero(Qm);
        mm<false, false, false, false>(S0, S1, Qm, ln);
        img_store(B.Q + (base + k) * IMG, Qm, ln);
    }
}

// carries, U, F, M = G U, target part of F_dx_add
__global__ __launch_bounds__(NTHREADS, 1) void k_dcarry(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const int b = blockIdx.x;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    const size_t qbase = (size_t)b * P.Nt;
    HM U, T;
    hm_identity(U, ln, 1.0);
    img_store(B.Carry + ((size_t)b * DP.Nc) * IMG, U, ln);
    for (int c = 1; c <= DP.Nc; ++c) {
        const int kend = min(c * DP.Lc, P.Nt) - 1;  // last step of chunk c-1
        img_load(B.Q + (qbase + kend) * IMG, T, ln);
        __syncthreads();
        sm_store(S0, T, ln);
        sm_store(S1, U, ln);
        __syncthreads();
        hm_zero(U);
        mm<false, false, false, false>(S0, S1, U, ln);
        if (c < DP.Nc) img_store(B.Carry + ((size_t)b * DP.Nc + c) * IMG, U, ln);
    }
    // U = C_Nt.  K = U0^dag U, tau = tr(W K)                 FidelityCalculations.jl:47-54
    if (B.Ub) img_store(B.Ub + (size_t)b * IMG, U, ln);
    const double *xb = B.x + (size_t)b * P.nx;
    HM U0, K;
    build_target(DP, xb, kNoPert, U0, ln);
    __syncthreads();
    sm_store(S0, U0, ln);
    sm_store(S1, U, ln);
    __syncthreads();
    hm_zero(K);
    mm<true, true, false, false>(S0, S1, K, ln);
    const int col = ln.col();
    const double pcol = DP.W[col] != 0.0 ? 1.0 : 0.0;
    double part = 0.0, tre = 0.0, tim = 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = ln.row(i, r);
            const double wr = DP.W[row];
            const double kr = K.re[i][r], ki = K.im[i][r];
            part += wr * (pcol * (kr * kr + ki * ki));
            if (row == col) {
                tre += wr * kr;
                tim += wr * ki;
            }
        }
    const double sum_part = wg_sum(part, lds, ln);
    const double tau_re = wg_sum(tre, lds, ln);
    const double tau_im = wg_sum(tim, lds, ln);
    const double Fv = (sum_part + tau_re * tau_re + tau_im * tau_im) / P.DD;
    // M = (2/DD) (P K^dag W K + conj(tau) W K) with T = K^dag (W K)
    HM WK = K;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double wr = DP.W[ln.row(i, r)];
            WK.re[i][r] *= wr;
            WK.im[i][r] *= wr;
        }
    __syncthreads();
    sm_store(S0, K, ln);
    sm_store(S1, WK, ln);
    __syncthreads();
    hm_zero(T);
    mm<true, true, false, false>(S0, S1, T, ln);
    const double sc = 2.0 / P.DD;
    HM Mm;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double prow = DP.W[ln.row(i, r)] != 0.0 ? 1.0 : 0.0;
            const double a = prow * T.re[i][r], bb = prow * T.im[i][r];
            const double wr = WK.re[i][r], wi = WK.im[i][r];
            const double cr = tau_re * wr + tau_im * wi, ci = tau_re * wi - tau_im * wr;  // conj(tau) WK
            Mm.re[i][r] = sc * (a + cr);
            Mm.im[i][r] = sc * (bb + ci);
        }
    img_store(B.M + (size_t)b * IMG, Mm, ln);
    // target derivative part of F_dx_add (FidelityCalculations.jl:34-40, 67-76)
    for (int q = 0; q < P.na; ++q) {
        grape::Pert pq;
        pq.var = grape::VAR_XADD;
        pq.index = q;
        pq.delta = P.eps;
        HM U0e, Kd;
        build_target(DP, xb, pq, U0e, ln);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            U0e.re[i] = (U0e.re[i] - U0.re[i]) * P.inv_eps;
            U0e.im[i] = (U0e.im[i] - U0.im[i]) * P.inv_eps;
        }
        __syncthreads();
        sm_store(S0, U0e, ln);
        sm_store(S1, U, ln);
        __syncthreads();
        hm_zero(Kd);
        mm<true, true, false, false>(S0, S1, Kd, ln);
        double pr = 0.0, dre = 0.0, dim = 0.0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = ln.row(i, r);
                const double wr = DP.W[row];
                pr += wr * (pcol * (Kd.re[i][r] * K.re[i][r] + Kd.im[i][r] * K.im[i][r]));
                if (row == col) {
                    dre += wr * Kd.re[i][r];
                    dim += wr * Kd.im[i][r];
                }
            }
        const double s1 = wg_sum(pr, lds, ln);
        const double tr_re = wg_sum(dre, lds, ln);
        const double tr_im = wg_sum(dim, lds, ln);
        if (threadIdx.x == 0)
            B.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + q] =
                (2.0 * s1 + 2.0 * (tau_re * tr_re + tau_im * tr_im)) / P.DD;
    }
    if (threadIdx.x == 0) B.F[b] = Fv;
}

// M'_c = Carry_c M Carry_c^dagger
__global__ __launch_bounds__(NTHREADS, 1) void k_dmc(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const int b = blockIdx.x / DP.Nc, c = blockIdx.x % DP.Nc;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    HM X, T;
    img_load(B.Carry + ((size_t)b * DP.Nc + c) * IMG, X, ln);
    sm_store(S0, X, ln);
    img_load(B.M + (size_t)b * IMG, X, ln);
    sm_store(S1, X, ln);
    __syncthreads();
    hm_zero(T);
    mm<false, false, false, false>(S0, S1, T, ln);  // Carry M
    __syncthreads();
    sm_store(S1, T, ln);
    __syncthreads();
    hm_zero(X);
    mm<false, false, true, true>(S1, S0, X, ln);  // (Carry M) Carry^dagger
    img_store(B.Mc + ((size_t)b * DP.Nc + c) * IMG, X, ln);
}

// F_dx[p, k] for every control p of step k, and (H0 reading x_add, DP.nva > 0) step k's term of
// F_dx_add[q] = Re tr(M'_c Y((E(x_add + eps e_q) - E) / eps)) to B.Fadd (UnitaryCalculations.jl:57-64:
// the x_add variant of every step, FidelityCalculations.jl:67-76: summed with the target's part)
__global__ __launch_bounds__(NTHREADS, 1) void k_dgrad(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const long item = blockIdx.x;
    const int b = (int)(item / P.Nt), k = (int)(item % P.Nt);
    const int c = k / DP.Lc, j0 = k - c * DP.Lc;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    const size_t qbase = (size_t)b * P.Nt;
    HM T, Z;
    img_load(B.Mc + ((size_t)b * DP.Nc + c) * IMG, T, ln);
    if (j0 > 0) {
        img_load(B.Q + (qbase + k - 1) * IMG, Z, ln);
        sm_store(S0, Z, ln);
        sm_store(S1, T, ln);
        __syncthreads();
        hm_zero(T);
        mm<false, false, false, false>(S0, S1, T, ln);  // Q_{k-1} M'_c
        __syncthreads();
    }
    img_load(B.Q + (qbase + k) * IMG, Z, ln);
    sm_store(S0, Z, ln);
    sm_store(S1, T, ln);
    __syncthreads();
    hm_zero(Z);
    mm<false, true, true, false>(S0, S1, Z, ln);  // Z = Y^T = conj(Q_k) (Q_{k-1} M'_c)^T
    // Z is parked in HBM (one coalesced 64-KB image) while the exponentials run:
    // kept live it costs 32 VGPRs through wg_expm and spills far more than 64 KB
    double *zimg = B.Z + (size_t)item * IMG;
    img_store(zimg, Z, ln);
    const double *xb = B.x + (size_t)b * P.nx;
    for (int p = 0; p < P.np + DP.nva; ++p) {
        grape::Pert pp;
        pp.var = p < P.np ? grape::VAR_X : grape::VAR_XADD;
        pp.index = p < P.np ? p : p - P.np;
        pp.delta = P.eps;
        HM A, X;
        bool singular = false;
        wg_expm([&](HM &G) { build_generator(DP, xb, k, pp, G, ln); }, X, lds, ln, singular);
        if (singular) atomicOr(B.status, 1);
        img_load(B.E + (qbase + k) * IMG, A, ln);
        img_load(zimg, Z, ln);  // written by this same lane above
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double dr = (X.re[i][r] - A.re[i][r]) * P.inv_eps;
                const double di = (X.im[i][r] - A.im[i][r]) * P.inv_eps;
                acc += Z.re[i][r] * dr - Z.im[i][r] * di;
            }
        const double s = wg_sum(acc, lds, ln);
        if (threadIdx.x == 0) {
            if (p < P.np) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + p] = s;
            else B.Fadd[(size_t)item * DP.nva + (p - P.np)] = s;
        }
    }
}

// F_dx_add[q] += sum_k Fadd[k][q] (after k_dcarry wrote the target's part), one workgroup per (b, q),
// fixed summation order
__global__ __launch_bounds__(256) void k_dadd(DenseProblem DP, DenseBatch B) {
    const grape::DevProblem &P = DP.P;
    const int b = blockIdx.x / DP.nva, q = blockIdx.x % DP.nva;
    __shared__ double red[256];
    double s = 0.0;
    for (int k = threadIdx.x; k < P.Nt; k += 256) s += B.Fadd[((size_t)b * P.Nt + k) * DP.nva + q];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) B.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + q] += red[0];
}

// F_d2err_dx_add[q, e] += sum_k Fd2add[e][k][q] (after k_derr_scan / the error head wrote the target's
// part), one workgroup per (b, e, q), fixed summation order
__global__ __launch_bounds__(256) void k_dadd_err(DenseProblem DP, DenseBatch B) {
    const grape::DevProblem &P = DP.P;
    const int q = blockIdx.x % DP.nva, be = blockIdx.x / DP.nva;
    __shared__ double red[256];
    double s = 0.0;
    for (int k = threadIdx.x; k < P.Nt; k += 256) s += B.Fd2add[((size_t)be * P.Nt + k) * DP.nva + q];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) B.Fd2dx[(size_t)be * P.nx + (size_t)P.np * P.Nt + q] += red[0];
}

// ---------------------------------------------------------------------------
// error sources
// ---------------------------------------------------------------------------
// local-frame image Y = Q_k^dag dX Q_{k-1} of one difference, stored as Y^T (slot s of step k), over the
// G = P.nvg gradient parameters of a step (np controls, then -- H0 / Herror reading x_add -- the x_add ones):
//   s < G: Z1_u = Y((E_dx_u - E)/eps), and F_dx[u, k] = Re tr(M'_c Z1_u) = Re sum M'_c o Z1_u^T (a control's
//          entry of F_dx, or step k's term of F_dx_add[u - np], summed by k_dadd);
//   G <= s < G + ne: W_e = Y((E_err_e - E)/eps);  then Z2_{e,u} = Y(mixed stencil, :79-95)
__global__ __launch_bounds__(NTHREADS, 1) void k_dlocal(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const long item = blockIdx.x;  // (b, k, s), s fastest
    const int s = (int)(item % DP.nz), k = (int)((item / DP.nz) % P.Nt), b = (int)(item / ((long)DP.nz * P.Nt));
    const int c = k / DP.Lc;
    const bool first = k == c * DP.Lc;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    const size_t nv = P.nv, step = (size_t)b * P.Nt + k;
    const double *Ek = B.E + step * nv * IMG;
    const int G = P.nvg;
    HM X, T;
    {
        img_load(Ek, T, ln);  // E_k (nominal)
        if (s < G + P.ne) {
            const int v = s < G ? P.off_dx + s : P.off_err + (s - G) * P.err_stride;  // (dxa follows dx)
            img_load(Ek + (size_t)v * IMG, X, ln);
            hm_sub(X, T);
            hm_scale(X, P.inv_eps);  // (1/eps) (E' - E)
        } else {
            const int r = s - G - P.ne, e = r / G, u = r % G;
            const int v_err = P.off_err + e * P.err_stride;
            img_load(Ek + (size_t)(v_err + 2 + u) * IMG, X, ln);
            hm_add(X, T);
            img_load(Ek + (size_t)(v_err + 1) * IMG, T, ln);
            hm_sub(X, T);
            img_load(Ek + (size_t)(P.off_dx2 + u) * IMG, T, ln);
            hm_sub(X, T);
            hm_scale(X, P.inv_eps2sq);  // ((E_mix + E) - E_err2 - E_dx2) / eps2^2
        }
    }
    img_load(B.Q + step * IMG, T, ln);
    sm_store(S0, T, ln);
    sm_store(S1, X, ln);
    __syncthreads();
    hm_zero(X);
    mm<true, true, false, false>(S0, S1, X, ln);  // Q_k^dag dX
    __syncthreads();
    if (first) hm_identity(T, ln, 1.0);
    else img_load(B.Q + (step - 1) * IMG, T, ln);
    sm_store(S0, T, ln);
    sm_store(S1, X, ln);
    __syncthreads();
    hm_zero(T);
    mm<true, false, true, false>(S0, S1, T, ln);  // Q_{k-1}^T (Q_k^dag dX)^T = Y^T
    img_store(B.Zl + (step * DP.nz + s) * IMG, T, ln);
    if (s < G) {
        img_load(B.Mc + ((size_t)b * DP.Nc + c) * IMG, X, ln);
        const double tr = wg_sum(hm_dot_re(X, T), lds, ln);
        if (threadIdx.x == 0) {
            if (s < P.np) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + s] = tr;
            else B.Fadd[step * DP.nva + (s - P.np)] = tr;
        }
    }
}

// Vc_c = Carry_c^dag (sum_{k in chunk c} W_k) Carry_c for (b, e, c)
__global__ __launch_bounds__(NTHREADS, 1) void k_dwsum(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const int c = blockIdx.x % DP.Nc, e = (blockIdx.x / DP.Nc) % P.ne, b = blockIdx.x / (DP.Nc * P.ne);
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    HM acc, T;
    hm_zero(acc);
    const int k0 = c * DP.Lc, k1 = min(k0 + DP.Lc, P.Nt);
    for (int k = k0; k < k1; ++k) {
        img_load(B.Zl + (((size_t)b * P.Nt + k) * DP.nz + P.nvg + e) * IMG, T, ln);  // W_k^T
        hm_add(acc, T);
    }
    img_load(B.Carry + ((size_t)b * DP.Nc + c) * IMG, T, ln);
    sm_store(S0, T, ln);
    sm_store(S1, acc, ln);
    __syncthreads();
    hm_zero(T);
    mm<true, true, true, false>(S0, S1, T, ln);  // Carry^dag (sum W)   [S1 holds (sum W)^T]
    __syncthreads();
    sm_store(S1, T, ln);
    __syncthreads();
    hm_zero(acc);
    mm<false, false, false, false>(S1, S0, acc, ln);  // (.) Carry
    img_store(B.Vc + (((size_t)b * P.ne + e) * DP.Nc + c) * IMG, acc, ln);
}

// prefix over chunks, Tot, U_derr = U Tot, F_d2err, M_e = G_e U, target part of F_d2err_dx_add
__global__ __launch_bounds__(NTHREADS, 1) void k_derr_scan(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const int e = blockIdx.x % P.ne, b = blockIdx.x / P.ne;
    const size_t be = (size_t)b * P.ne + e;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    HM run, T;
    hm_zero(run);
    for (int c = 0; c < DP.Nc; ++c) {  // exclusive prefix S_{c-1} (in the global frame)
        img_store(B.Sx + (be * DP.Nc + c) * IMG, run, ln);
        img_load(B.Vc + (be * DP.Nc + c) * IMG, T, ln);
        hm_add(run, T);
    }
    img_store(B.Tot + be * IMG, run, ln);
    const double *xb = B.x + (size_t)b * P.nx;
    HM U, Ue, Ke;
    img_load(B.Ub + (size_t)b * IMG, U, ln);
    sm_store(S0, U, ln);
    sm_store(S1, run, ln);
    __syncthreads();
    hm_zero(Ue);
    mm<false, false, false, false>(S0, S1, Ue, ln);  // U_derr = U Tot          (:122-123)
    HM U0;
    build_target(DP, xb, kNoPert, U0, ln);
    __syncthreads();
    sm_store(S0, U0, ln);
    sm_store(S1, Ue, ln);
    __syncthreads();
    hm_zero(Ke);
    mm<true, true, false, false>(S0, S1, Ke, ln);  // Ke = U0^dag Ue
    const int col = ln.col();
    const double wcol = DP.W[col], pcol = wcol != 0.0 ? 1.0 : 0.0;
    double a1 = 0.0, a2 = 0.0, tre = 0.0, tim = 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = ln.row(i, r);
            const double wr = DP.W[row];
            a1 += wr * (pcol * (Ke.re[i][r] * Ke.re[i][r] + Ke.im[i][r] * Ke.im[i][r]));
            a2 += wcol * (Ue.re[i][r] * Ue.re[i][r] + Ue.im[i][r] * Ue.im[i][r]);  // W_j (Ue^dag Ue)_jj
            if (row == col) {
                tre += wr * Ke.re[i][r];
                tim += wr * Ke.im[i][r];
            }
        }
    const double s_a1 = wg_sum(a1, lds, ln), s_a2 = wg_sum(a2, lds, ln);
    const double te_re = wg_sum(tre, lds, ln), te_im = wg_sum(tim, lds, ln);
    // F_d2err = 2[sum W_i P_j |Ke_ij|^2 - (1+D) sum W (Ue^dag Ue)_ii + |te|^2] / (D(D+1))   (:79-83)
    const double fd2 = 2.0 * (s_a1 - (1.0 + P.Dtr) * s_a2 + te_re * te_re + te_im * te_im) / P.DD;
    // target part of F_d2err_dx_add (FidelityCalculations.jl:100-112, the U0_dx_add terms)
    for (int q = 0; q < P.na; ++q) {
        grape::Pert pq;
        pq.var = grape::VAR_XADD;
        pq.index = q;
        pq.delta = P.eps;
        HM U0e;
        build_target(DP, xb, pq, U0e, ln);
        hm_sub(U0e, U0);
        hm_scale(U0e, P.inv_eps);
        __syncthreads();
        sm_store(S0, U0e, ln);
        __syncthreads();
        hm_zero(T);
        mm<true, true, false, false>(S0, S1, T, ln);  // Kde = U0d^dag Ue (S1 still holds Ue)
        double pr = 0.0, dre = 0.0, dim = 0.0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = ln.row(i, r);
                const double wr = DP.W[row];
                pr += wr * (pcol * (T.re[i][r] * Ke.re[i][r] + T.im[i][r] * Ke.im[i][r]));
                if (row == col) {
                    dre += wr * T.re[i][r];
                    dim += wr * T.im[i][r];
                }
            }
        const double s1 = wg_sum(pr, lds, ln), tr_re = wg_sum(dre, lds, ln), tr_im = wg_sum(dim, lds, ln);
        if (threadIdx.x == 0)
            B.Fd2dx[be * P.nx + (size_t)P.np * P.Nt + q] = 2.0 * (2.0 * s1 + 2.0 * (te_re * tr_re + te_im * tr_im)) / P.DD;
    }
    if (threadIdx.x == 0) B.Fd2[be] = fd2;
    // M_e = (4/DD) [P Ke^dag W K + conj(te) W K - (1+D) W Ue^dag U],  K = U0^dag U
    HM K;
    __syncthreads();
    sm_store(S0, U0, ln);
    sm_store(S1, U, ln);
    __syncthreads();
    hm_zero(K);
    mm<true, true, false, false>(S0, S1, K, ln);  // K = U0^dag U
    __syncthreads();
    sm_store(S0, Ue, ln);  // S1 still holds U
    __syncthreads();
    hm_zero(T);
    mm<true, true, false, false>(S0, S1, T, ln);  // Ue^dag U
    HM WK = K;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double wr = DP.W[ln.row(i, r)];
            WK.re[i][r] *= wr;
            WK.im[i][r] *= wr;
        }
    __syncthreads();
    sm_store(S0, Ke, ln);
    sm_store(S1, WK, ln);
    __syncthreads();
    hm_zero(U0);
    mm<true, true, false, false>(S0, S1, U0, ln);  // Ke^dag (W K)
    const double sc = 4.0 / P.DD;
    HM Mm;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = ln.row(i, r);
            const double wr = DP.W[row], prow = wr != 0.0 ? 1.0 : 0.0;
            const double wkr = WK.re[i][r], wki = WK.im[i][r];
            const double cr = te_re * wkr + te_im * wki, ci = te_re * wki - te_im * wkr;  // conj(te) W K
            const double ur = (1.0 + P.Dtr) * wr * T.re[i][r], ui = (1.0 + P.Dtr) * wr * T.im[i][r];
            Mm.re[i][r] = sc * (prow * U0.re[i][r] + cr - ur);
            Mm.im[i][r] = sc * (prow * U0.im[i][r] + ci - ui);
        }
    img_store(B.Me + be * IMG, Mm, ln);
}

// per (b, e, c): M' = Carry M_e Carry^dag and B at the chunk start, [T_c, M'] + M' Ttot with
// T_c = Carry S_{c-1} Carry^dag, Ttot = Carry Tot Carry^dag
__global__ __launch_bounds__(NTHREADS, 1) void k_dmce(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const int c = blockIdx.x % DP.Nc, e = (blockIdx.x / DP.Nc) % P.ne, b = blockIdx.x / (DP.Nc * P.ne);
    const size_t be = (size_t)b * P.ne + e, bec = be * DP.Nc + c;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    HM X, Mp, Tc, Tt;
    img_load(B.Carry + ((size_t)b * DP.Nc + c) * IMG, X, ln);
    sm_store(S0, X, ln);  // S0 = Carry through the three conjugations
    auto conj_by_carry = [&](const double *img, HM &out) {
        img_load(img, X, ln);
        __syncthreads();
        sm_store(S1, X, ln);
        __syncthreads();
        hm_zero(X);
        mm<false, false, false, false>(S0, S1, X, ln);  // Carry Y
        __syncthreads();
        sm_store(S1, X, ln);
        __syncthreads();
        hm_zero(out);
        mm<false, false, true, true>(S1, S0, out, ln);  // (Carry Y) Carry^dag
    };
    conj_by_carry(B.Me + be * IMG, Mp);
    img_store(B.Mp + bec * IMG, Mp, ln);
    conj_by_carry(B.Sx + bec * IMG, Tc);
    conj_by_carry(B.Tot + be * IMG, Tt);
    __syncthreads();
    sm_store(S0, Tc, ln);
    sm_store(S1, Mp, ln);
    __syncthreads();
    HM Bp;
    hm_zero(Bp);
    mm<false, false, false, false>(S0, S1, Bp, ln);  // Tc M'
    hm_zero(X);
    mm<false, false, false, false>(S1, S0, X, ln);  // M' Tc
    hm_sub(Bp, X);
    __syncthreads();
    sm_store(S0, Tt, ln);
    __syncthreads();
    mm<false, false, false, false>(S1, S0, Bp, ln);  // += M' Ttot
    img_store(B.B0 + bec * IMG, Bp, ln);
}

// F_d2err_dx[u, k, e] = Re[tr(Lambda_k Z1_u) + tr(M' Z2_{e,u})], Lambda_k = B_k - M' W_k,
// B_{k+1} = Lambda_k + W_k M'   (grape_errpath.hpp header)
__global__ __launch_bounds__(NTHREADS, 1) void k_derr_grad(DenseProblem DP, DenseBatch B) {
    extern __shared__ double lds[];
    const Lane ln = make_lane();
    const grape::DevProblem &P = DP.P;
    const int e = blockIdx.x % P.ne, c = (blockIdx.x / P.ne) % DP.Nc, b = blockIdx.x / (P.ne * DP.Nc);
    const size_t be = (size_t)b * P.ne + e, bec = be * DP.Nc + c;
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    HM Bp, Mr, L, T;
    img_load(B.B0 + bec * IMG, Bp, ln);
    img_load(B.Mp + bec * IMG, Mr, ln);
    sm_store(S1, Mr, ln);  // M' for the whole chunk
    double *out = B.Fd2dx + be * P.nx;
    const int k0 = c * DP.Lc, k1 = min(k0 + DP.Lc, P.Nt), G = P.nvg;
    for (int k = k0; k < k1; ++k) {
        const double *Zk = B.Zl + ((size_t)b * P.Nt + k) * DP.nz * IMG;
        img_load(Zk + (size_t)(G + e) * IMG, T, ln);  // W_k^T
        __syncthreads();
        sm_store(S0, T, ln);
        __syncthreads();
        hm_zero(L);
        mm<false, false, true, false>(S1, S0, L, ln);  // M' W
        hm_scale(L, -1.0);
        hm_add(L, Bp);  // Lambda = B - M' W
        for (int u = 0; u < G; ++u) {
            img_load(Zk + (size_t)u * IMG, T, ln);  // Z1_u^T
            double acc = hm_dot_re(L, T);
            img_load(Zk + (size_t)(G + P.ne + e * G + u) * IMG, T, ln);  // Z2_{e,u}^T
            acc += hm_dot_re(Mr, T);
            const double tr = wg_sum(acc, lds, ln);
            if (threadIdx.x == 0) {
                if (u < P.np) out[(size_t)k * P.np + u] = tr;
                else B.Fd2add[(be * P.Nt + k) * DP.nva + (u - P.np)] = tr;  // step k's x_add term (k_dadd_err)
            }
        }
        hm_zero(Bp);
        mm<true, false, false, false>(S0, S1, Bp, ln);  // W M'
        hm_add(Bp, L);
    }
}

constexpr size_t kLds = (size_t)LDS_TOTAL * sizeof(double);

}  // namespace

hipError_t set_lds_limits() {
    const void *fs[] = {reinterpret_cast<const void *>(&k_dexp),      reinterpret_cast<const void *>(&k_dexp_raw),
                        reinterpret_cast<const void *>(&k_dscan),     reinterpret_cast<const void *>(&k_dcarry),
                        reinterpret_cast<const void *>(&k_dmc),       reinterpret_cast<const void *>(&k_dgrad),
                        reinterpret_cast<const void *>(&k_dlocal),    reinterpret_cast<const void *>(&k_dwsum),
                        reinterpret_cast<const void *>(&k_derr_scan), reinterpret_cast<const void *>(&k_dmce),
                        reinterpret_cast<const void *>(&k_derr_grad)};
    for (const void *f : fs) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// the general-projector heads' view of a dense batch (grape_projector_api.hpp)
static grape_proj::Heads dense_heads(const DenseProblem &P, const DenseBatch &B) {
    grape_proj::Heads H{};
    H.P = P.P;
    H.dense = 1;
    H.x = B.x;
    H.Ub_img = B.Ub;
    H.Tot_img = B.Tot;
    H.M_img = B.M;
    H.Me_img = B.Me;
    H.F = B.F;
    H.Fdx = B.Fdx;
    H.Fd2 = B.Fd2;
    H.Fd2dx = B.Fd2dx;
    H.scr = B.gp_scr;
    return H;
}

// padded register-file image -> row-major d x d tile, one workgroup per matrix
__global__ __launch_bounds__(256) void k_img_rows(const double *img, grape::cd *rows, int D) {
    const double *src = img + (size_t)blockIdx.x * IMG;
    grape::cd *dst = rows + (size_t)blockIdx.x * D * D;
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const int row = t / D, col = t % D;
        const int w = col >> 4, tr = row >> 4, r = (row & 15) >> 2, l = ((row & 3) << 4) | (col & 15);
        const size_t o = (size_t)((w * 4 + tr) * 4 + r) * 64 + l;
        dst[t] = grape::cmake(src[o], src[IMG / 2 + o]);
    }
}

hipError_t launch_variant_table(const DenseProblem &P, const DenseBatch &B, grape::cd *rows, hipStream_t st) {
    const unsigned n = (unsigned)((long)B.nb * P.P.Nt * P.P.nv);
    hipLaunchKernelGGL(k_dexp, dim3(n), dim3(NTHREADS), kLds, st, P, B);
    hipLaunchKernelGGL(k_img_rows, dim3(n), dim3(256), 0, st, B.E, rows, P.P.D);
    return hipGetLastError();
}

hipError_t launch_pipeline(const DenseProblem &P, const DenseBatch &B, hipStream_t st, const grape_host::KMark &mark) {
    const unsigned nsteps = (unsigned)((long)B.nb * P.P.Nt);
    const unsigned nchunks = (unsigned)((long)B.nb * P.Nc);
    mark(GRAPE_KERNEL_DEXP, 0);
    hipLaunchKernelGGL(k_dexp, dim3(nsteps * (unsigned)P.P.nv), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DEXP, 1);
    mark(GRAPE_KERNEL_DSCAN, 0);
    hipLaunchKernelGGL(k_dscan, dim3(nchunks), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DSCAN, 1);
    mark(GRAPE_KERNEL_DCARRY, 0);
    hipLaunchKernelGGL(k_dcarry, dim3((unsigned)B.nb), dim3(NTHREADS), kLds, st, P, B);
    if (P.P.gen_proj) {  // general projector: F, M (and F_dx_add's target part) in general form
        const hipError_t e = grape_proj::launch_fid_head(dense_heads(P, B), B.nb, st);
        if (e != hipSuccess) return e;
    }
    mark(GRAPE_KERNEL_DCARRY, 1);
    mark(GRAPE_KERNEL_DMC, 0);
    hipLaunchKernelGGL(k_dmc, dim3(nchunks), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DMC, 1);
    if (P.P.ne == 0) {
        mark(GRAPE_KERNEL_DGRAD, 0);
        hipLaunchKernelGGL(k_dgrad, dim3(nsteps), dim3(NTHREADS), kLds, st, P, B);
        if (P.nva > 0) hipLaunchKernelGGL(k_dadd, dim3((unsigned)(B.nb * P.nva)), dim3(256), 0, st, P, B);
        mark(GRAPE_KERNEL_DGRAD, 1);
        return hipGetLastError();
    }
    const unsigned nerr_chunks = nchunks * (unsigned)P.P.ne;
    mark(GRAPE_KERNEL_GRAD, 0);
    hipLaunchKernelGGL(k_dlocal, dim3(nsteps * (unsigned)P.nz), dim3(NTHREADS), kLds, st, P, B);
    if (P.nva > 0) hipLaunchKernelGGL(k_dadd, dim3((unsigned)(B.nb * P.nva)), dim3(256), 0, st, P, B);
    mark(GRAPE_KERNEL_GRAD, 1);
    mark(GRAPE_KERNEL_ERR_SCAN, 0);
    hipLaunchKernelGGL(k_dwsum, dim3(nerr_chunks), dim3(NTHREADS), kLds, st, P, B);
    hipLaunchKernelGGL(k_derr_scan, dim3((unsigned)B.nb * P.P.ne), dim3(NTHREADS), kLds, st, P, B);
    if (P.P.gen_proj) {
        const hipError_t e = grape_proj::launch_err_head(dense_heads(P, B), B.nb, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_dmce, dim3(nerr_chunks), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_ERR_SCAN, 1);
    mark(GRAPE_KERNEL_ERR_GRAD, 0);
    hipLaunchKernelGGL(k_derr_grad, dim3(nerr_chunks), dim3(NTHREADS), kLds, st, P, B);
    if (P.nva > 0)
        hipLaunchKernelGGL(k_dadd_err, dim3((unsigned)(B.nb * P.P.ne * P.nva)), dim3(256), 0, st, P, B);
    mark(GRAPE_KERNEL_ERR_GRAD, 1);
    return hipGetLastError();
}

// padded image <-> column-major d x d complex (the C ABI's layout), one workgroup per matrix
__global__ __launch_bounds__(256) void k_img_cols(const double *img, grape::cd *cols, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const int col = t / D, row = t % D;
        const int w = col >> 4, tr = row >> 4, r = (row & 15) >> 2, l = ((row & 3) << 4) | (col & 15);
        const size_t o = (size_t)((w * 4 + tr) * 4 + r) * 64 + l;
        cols[t] = grape::cmake(img[o], img[IMG / 2 + o]);
    }
}
__global__ __launch_bounds__(256) void k_cols_img(const grape::cd *cols, double *img, int D) {
    for (int o = threadIdx.x; o < 64 * 64; o += blockDim.x) {
        const int l = o & 63, r = (o >> 6) & 3, t = (o >> 8) & 3, w = o >> 10;
        const int row = 16 * t + (l >> 4) + 4 * r, col = 16 * w + (l & 15);
        const bool in = row < D && col < D;
        const grape::cd v = in ? cols[(size_t)row + (size_t)col * D] : grape::cmake(0.0, 0.0);
        img[o] = v.re;
        img[IMG / 2 + o] = v.im;
    }
}

hipError_t launch_slice_forward(const DenseProblem &P, const DenseBatch &B, grape::cd *Ucols, hipStream_t st) {
    if (B.nb != 1 || !B.Ub) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_dexp, dim3((unsigned)P.P.Nt * (unsigned)P.P.nv), dim3(NTHREADS), kLds, st, P, B);
    hipLaunchKernelGGL(k_dscan, dim3((unsigned)P.Nc), dim3(NTHREADS), kLds, st, P, B);
    hipLaunchKernelGGL(k_dcarry, dim3(1), dim3(NTHREADS), kLds, st, P, B);  // carries and U (F, M unused)
    hipLaunchKernelGGL(k_img_cols, dim3(1), dim3(256), 0, st, B.Ub, Ucols, P.P.D);
    return hipGetLastError();
}

hipError_t launch_slice_gradient(const DenseProblem &P, const DenseBatch &B, const grape::cd *Mcols, hipStream_t st) {
    if (B.nb != 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_cols_img, dim3(1), dim3(256), 0, st, Mcols, B.M, P.P.D);
    hipLaunchKernelGGL(k_dmc, dim3((unsigned)P.Nc), dim3(NTHREADS), kLds, st, P, B);
    hipLaunchKernelGGL(k_dgrad, dim3((unsigned)P.P.Nt), dim3(NTHREADS), kLds, st, P, B);
    return hipGetLastError();
}

// A = -i dt H of host-tabulated H (closure fallback, column-major d x d), zero-padded images
__global__ __launch_bounds__(256) void k_tab_images(const grape::cd *H, double *img, int D, double dt) {
    const grape::cd *src = H + (size_t)blockIdx.x * D * D;
    double *dst = img + (size_t)blockIdx.x * IMG;
    for (int o = threadIdx.x; o < 64 * 64; o += blockDim.x) {
        const int l = o & 63, r = (o >> 6) & 3, t = (o >> 8) & 3, w = o >> 10;
        const int row = 16 * t + (l >> 4) + 4 * r, col = 16 * w + (l & 15);
        const bool in = row < D && col < D;
        const grape::cd h = in ? src[(size_t)row + (size_t)col * D] : grape::cmake(0.0, 0.0);
        dst[o] = dt * h.im;             // -i dt (re + i im) = dt im - i dt re
        dst[IMG / 2 + o] = -(dt * h.re);
    }
}

hipError_t launch_table_variants(const grape::cd *H, int D, int n, double dt, double *Aimg, double *Eimg,
                                 grape::cd *rows, int *status, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tab_images, dim3((unsigned)n), dim3(256), 0, st, H, Aimg, D, dt);
    hipLaunchKernelGGL(k_dexp_raw, dim3((unsigned)n), dim3(NTHREADS), kLds, st, Aimg, Eimg, status, nullptr);
    hipLaunchKernelGGL(k_img_rows, dim3((unsigned)n), dim3(256), 0, st, Eimg, rows, D);
    return hipGetLastError();
}

hipError_t launch_expm_raw(const double *A, double *E, int n, int *status, int *mstats, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dexp_raw, dim3((unsigned)n), dim3(NTHREADS), kLds, st, A, E, status, mstats);
    return hipGetLastError();
}

}  // namespace grape_dense
