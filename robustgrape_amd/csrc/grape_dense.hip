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
// (algebra: grape_kernels.hpp header; layouts and numerics: grape_dense.hpp).
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
    const long item = blockIdx.x;
    const int b = (int)(item / P.Nt), k = (int)(item % P.Nt);
    HM X;
    const double *xb = B.x + (size_t)b * P.nx;
    bool singular = false;
    const int m = wg_expm([&](HM &A) { build_generator(DP, xb, k, kNoPert, A, ln); }, X, lds, ln, singular);
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
    img_load(B.E + (base + k0) * IMG, Qm, ln);
    img_store(B.Q + (base + k0) * IMG, Qm, ln);
    for (int k = k0 + 1; k < k1; ++k) {
        img_load(B.E + (base + k) * IMG, Ek, ln);
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

// F_dx[p, k] for every control p of step k
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
    for (int p = 0; p < P.np; ++p) {
        grape::Pert pp;
        pp.var = grape::VAR_X;
        pp.index = p;
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
        if (threadIdx.x == 0) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + p] = s;
    }
}

constexpr size_t kLds = (size_t)LDS_TOTAL * sizeof(double);

}  // namespace

hipError_t set_lds_limits() {
    const void *fs[] = {reinterpret_cast<const void *>(&k_dexp), reinterpret_cast<const void *>(&k_dexp_raw),
                        reinterpret_cast<const void *>(&k_dscan), reinterpret_cast<const void *>(&k_dcarry),
                        reinterpret_cast<const void *>(&k_dmc), reinterpret_cast<const void *>(&k_dgrad)};
    for (const void *f : fs) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pipeline(const DenseProblem &P, const DenseBatch &B, hipStream_t st, const grape_host::KMark &mark) {
    const unsigned nsteps = (unsigned)((long)B.nb * P.P.Nt);
    const unsigned nchunks = (unsigned)((long)B.nb * P.Nc);
    mark(GRAPE_KERNEL_DEXP, 0);
    hipLaunchKernelGGL(k_dexp, dim3(nsteps), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DEXP, 1);
    mark(GRAPE_KERNEL_DSCAN, 0);
    hipLaunchKernelGGL(k_dscan, dim3(nchunks), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DSCAN, 1);
    mark(GRAPE_KERNEL_DCARRY, 0);
    hipLaunchKernelGGL(k_dcarry, dim3((unsigned)B.nb), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DCARRY, 1);
    mark(GRAPE_KERNEL_DMC, 0);
    hipLaunchKernelGGL(k_dmc, dim3(nchunks), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DMC, 1);
    mark(GRAPE_KERNEL_DGRAD, 0);
    hipLaunchKernelGGL(k_dgrad, dim3(nsteps), dim3(NTHREADS), kLds, st, P, B);
    mark(GRAPE_KERNEL_DGRAD, 1);
    return hipGetLastError();
}

hipError_t launch_expm_raw(const double *A, double *E, int n, int *status, int *mstats, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dexp_raw, dim3((unsigned)n), dim3(NTHREADS), kLds, st, A, E, status, mstats);
    return hipGetLastError();
}

}  // namespace grape_dense
