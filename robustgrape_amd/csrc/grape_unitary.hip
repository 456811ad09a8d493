// grape_unitary.hip -- materialised unitary derivatives for ONE control vector,
// the output of calculate_unitary_and_derivatives (src/UnitaryCalculations.jl:20-155)
// through the C ABI (grape_unitary_derivs).
//
// The propagator table E[k][v] (every finite-difference variant of every step,
// the closure call sites :45-90) comes from the small engine's k_expm (d <= 12) or
// the dense engine's k_dexp, converted from its register-file images (12 < d <= 64).  Then:
//   k_u_chain     C_k = E_k C_{k-1}                                    (:46)
//   k_u_vmats     V_{k,s} = C_k^dagger (stencil_s of E[k][.]) C_{k-1}   (:51-52,59-60,67-68,77-83,89-95)
//                 (C_k^{-1} = C_k^dagger: C_k is unitary; the reference's LU inverse
//                  differs at the 1e-15 level)
//   k_u_cumsum    S_{k,e} = sum_{j<=k} V^err_{j,e}                      (:112)
//   k_u_assemble  U_dx[p,k] = U V^dx_{k,p};  U_derr_dx[p,k,e] =
//                 U (V^dx_{k,p} S_{k-1,e} + R_{k+1,e} V^dx_{k,p} + V^mix_{k,p,e}),
//                 R_{k+1,e} = S_{N-1,e} - S_{k,e}                       (:114-118, :124-139)
//   k_u_reduce    U_dx_add, U_derr, U_derr_dx_add (sums over k)         (:119-123, :140-151)
// Outputs are written straight into the reference's column-major layouts.
//
// This path is write-bound (U_dx is d^2 np N_t complex numbers) and runs once per
// call, not inside an optimiser loop, so its kernels are plain thread-per-element
// ones over d x d tiles: staged in LDS for d <= kMaxD (one workgroup per item), and
// for the dense engine's 12 < d <= 64 in global scratch (kTiles tiles per workgroup,
// kResident workgroups striding over the items, the operands L2-resident).
#include "grape_unitary_api.hpp"

namespace grape_unitary {

namespace {

constexpr int BLOCK = 256;  // >= d^2 for d <= 12 (kMaxD)

__device__ __forceinline__ cd u_add(cd a, cd b) { return cd{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cd u_sub(cd a, cd b) { return cd{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cd u_scale(double s, cd a) { return cd{s * a.re, s * a.im}; }
__device__ __forceinline__ cd u_mul(cd a, cd b) { return cd{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ cd u_mulc(cd a, cd b) {  // conj(a) b
    return cd{a.re * b.re + a.im * b.im, a.re * b.im - a.im * b.re};
}

// element (i, j) of A B, A and B row-major D x D
__device__ __forceinline__ cd mm_el(const cd *A, const cd *B, int D, int i, int j) {
    cd s{0.0, 0.0};
    for (int l = 0; l < D; ++l) s = u_add(s, u_mul(A[i * D + l], B[l * D + j]));
    return s;
}
// element (i, j) of A^dagger B
__device__ __forceinline__ cd mmh_el(const cd *A, const cd *B, int D, int i, int j) {
    cd s{0.0, 0.0};
    for (int l = 0; l < D; ++l) s = u_add(s, u_mulc(A[l * D + i], B[l * D + j]));
    return s;
}

__device__ __forceinline__ void load_tile(cd *dst, const cd *src, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) dst[t] = src[t];
}
__device__ __forceinline__ void identity_tile(cd *dst, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) dst[t] = cd{(t / D == t % D) ? 1.0 : 0.0, 0.0};
}
__device__ __forceinline__ void zero_tile(cd *dst, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) dst[t] = cd{0.0, 0.0};
}

// the workgroup's kTiles tiles: LDS for d <= kMaxD, its slice of the global scratch above
__device__ __forceinline__ cd *tiles(cd *lds, cd *gscr, int D) {
    return D <= kMaxD ? lds : gscr + (size_t)blockIdx.x * kTiles * D * D;
}
// barrier that also orders the workgroup's global-scratch tile traffic
__device__ __forceinline__ void tsync() {
    __threadfence_block();
    __syncthreads();
}

// C_k = E_k C_{k-1}: one workgroup walks the chain (the only serial dependency, :46)
__global__ __launch_bounds__(BLOCK) void k_u_chain(UProblem P, const cd *E, cd *C) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D;
    cd *sE = tiles(lds, P.gscr, D), *sC = sE + DD, *sT = sC + DD;
    identity_tile(sC, D);
    for (int k = 0; k < P.Nt; ++k) {
        load_tile(sE, E + ((size_t)k * P.nv) * DD, D);
        tsync();
        for (int t = threadIdx.x; t < DD; t += blockDim.x) sT[t] = mm_el(sE, sC, D, t / D, t % D);
        tsync();
        for (int t = threadIdx.x; t < DD; t += blockDim.x) {
            sC[t] = sT[t];
            C[(size_t)k * DD + t] = sT[t];
        }
    }
}

// the stencil of slot s at step k (difference of stored variants, reference order)
__device__ __forceinline__ cd stencil(const UProblem &P, const cd *Ek, int s, int t) {
    const int DD = P.D * P.D;
    const cd e0 = Ek[t];
    if (s < P.np + P.na)  // dx_p / dxa_q: inv_eps * (E' - E)
        return u_scale(P.inv_eps, u_sub(Ek[(size_t)(1 + s) * DD + t], e0));
    s -= P.np + P.na;
    if (s < P.ne)  // err_e
        return u_scale(P.inv_eps, u_sub(Ek[(size_t)P.v_err(s) * DD + t], e0));
    s -= P.ne;
    // mixed: (E(x + eps2, err eps2) + E - E(err eps2) - E(x + eps2)) / eps2^2
    const int nq = P.np + P.na, e = s / nq, q = s % nq;
    const cd a = Ek[(size_t)P.v_mix(e, q) * DD + t];
    const cd b = Ek[(size_t)P.v_err2(e) * DD + t];
    const cd c = Ek[(size_t)P.v_x2(q) * DD + t];
    return u_scale(P.inv_eps2sq, u_sub(u_sub(u_add(a, e0), b), c));
}

// V_{k,s} = C_k^dagger stencil C_{k-1}, items (k, s)
__global__ __launch_bounds__(BLOCK) void k_u_vmats(UProblem P, const cd *E, const cd *C, cd *V) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sCk = tiles(lds, P.gscr, D), *sCp = sCk + DD, *sX = sCp + DD, *sT = sX + DD;
    for (long item = blockIdx.x; item < (long)P.Nt * P.nslots; item += gridDim.x) {
        const int k = (int)(item / P.nslots), s = (int)(item % P.nslots);
        load_tile(sCk, C + (size_t)k * DD, D);
        if (k > 0) load_tile(sCp, C + (size_t)(k - 1) * DD, D);
        else identity_tile(sCp, D);
        const cd *Ek = E + (size_t)k * P.nv * DD;
        for (int t = t0; t < DD; t += blockDim.x) sX[t] = stencil(P, Ek, s, t);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) sT[t] = mm_el(sX, sCp, D, t / D, t % D);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) V[((size_t)k * P.nslots + s) * DD + t] = mmh_el(sCk, sT, D, t / D, t % D);
        tsync();
    }
}

// S_{k,e} = sum_{j<=k} V^err_{j,e}  (one thread per (e, element), sequential in k)
__global__ void k_u_cumsum(UProblem P, const cd *V, cd *S) {
    const int DD = P.D * P.D;
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= P.ne * DD) return;
    const int e = id / DD, t = id % DD;
    const int s = P.np + P.na + e;
    cd acc{0.0, 0.0};
    for (int k = 0; k < P.Nt; ++k) {
        acc = u_add(acc, V[((size_t)k * P.nslots + s) * DD + t]);
        S[((size_t)k * P.ne + e) * DD + t] = acc;
    }
}

// column-major (reference) offset of element (i, j) of matrix number `m` (complex units)
__device__ __forceinline__ size_t cm(int D, size_t m, int i, int j) { return m * D * D + (size_t)i + (size_t)j * D; }

// U_dx (d,d,np,Nt) and U_derr_dx (d,d,np,Nt,ne): items (k, p, e|-1)
__global__ __launch_bounds__(BLOCK) void k_u_assemble(UProblem P, const cd *C, const cd *V, const cd *S, cd *Udx,
                                                      cd *Uedx) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sU = tiles(lds, P.gscr, D), *sA = sU + DD, *sB = sA + DD, *sX = sB + DD;
    const int per_k = P.np * (1 + P.ne);
    load_tile(sU, C + (size_t)(P.Nt - 1) * DD, D);
    for (long item = blockIdx.x; item < (long)P.Nt * per_k; item += gridDim.x) {
        const int k = (int)(item / per_k), r = (int)(item % per_k), p = r % P.np, e = r / P.np - 1;
        load_tile(sA, V + ((size_t)k * P.nslots + p) * DD, D);  // V^dx_{k,p}
        if (e < 0) {
            tsync();
            for (int t = t0; t < DD; t += blockDim.x)
                Udx[cm(D, (size_t)k * P.np + p, t / D, t % D)] = mm_el(sU, sA, D, t / D, t % D);
            tsync();
            continue;
        }
        // X = V^dx S_{k-1,e} + R_{k+1,e} V^dx + V^mix_{k,p,e}
        if (k > 0) load_tile(sB, S + ((size_t)(k - 1) * P.ne + e) * DD, D);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) sX[t] = k > 0 ? mm_el(sA, sB, D, t / D, t % D) : cd{0.0, 0.0};
        tsync();
        if (k < P.Nt - 1) {  // R_{k+1,e} = S_{N-1,e} - S_{k,e}
            const cd *Stot = S + ((size_t)(P.Nt - 1) * P.ne + e) * DD, *Sk = S + ((size_t)k * P.ne + e) * DD;
            for (int q = t0; q < DD; q += blockDim.x) sB[q] = u_sub(Stot[q], Sk[q]);
        }
        tsync();
        const int smix = P.np + P.na + P.ne + e * (P.np + P.na) + p;
        for (int t = t0; t < DD; t += blockDim.x) {
            cd x = sX[t];
            if (k < P.Nt - 1) x = u_add(x, mm_el(sB, sA, D, t / D, t % D));
            sX[t] = u_add(x, V[((size_t)k * P.nslots + smix) * DD + t]);
        }
        tsync();
        for (int t = t0; t < DD; t += blockDim.x)
            Uedx[cm(D, ((size_t)e * P.Nt + k) * P.np + p, t / D, t % D)] = mm_el(sU, sX, D, t / D, t % D);
        tsync();
    }
}

// U_dx_add (d,d,na), U_derr (d,d,ne), U_derr_dx_add (d,d,na,ne): one item per output matrix
__global__ __launch_bounds__(BLOCK) void k_u_reduce(UProblem P, const cd *C, const cd *V, const cd *S, cd *Udxa,
                                                    cd *Ue, cd *Uedxa) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sU = tiles(lds, P.gscr, D), *sA = sU + DD, *sB = sA + DD, *sX = sB + DD;
    load_tile(sU, C + (size_t)(P.Nt - 1) * DD, D);
    const int nred = P.na + P.ne + P.na * P.ne;
    for (int item = blockIdx.x; item < nred; item += gridDim.x) {
        int m = item;
        zero_tile(sX, D);  // the accumulator of this output
        cd *out;
        size_t oidx;
        if (m < P.na) {  // U_dx_add[q] = U sum_k V^dxa_{k,q}
            const int s = P.np + m;
            for (int t = t0; t < DD; t += blockDim.x) {
                cd acc{0.0, 0.0};
                for (int k = 0; k < P.Nt; ++k) acc = u_add(acc, V[((size_t)k * P.nslots + s) * DD + t]);
                sX[t] = acc;
            }
            out = Udxa;
            oidx = m;
        } else if ((m -= P.na) < P.ne) {  // U_derr[e] = U S_{N-1,e}
            for (int t = t0; t < DD; t += blockDim.x) sX[t] = S[((size_t)(P.Nt - 1) * P.ne + m) * DD + t];
            out = Ue;
            oidx = m;
        } else {  // U_derr_dx_add[q, e]
            m -= P.ne;
            const int q = m % P.na, e = m / P.na, sq = P.np + q;
            const int smix = P.np + P.na + P.ne + e * (P.np + P.na) + P.np + q;
            const cd *Stot = S + ((size_t)(P.Nt - 1) * P.ne + e) * DD;
            for (int k = 0; k < P.Nt; ++k) {
                tsync();
                load_tile(sA, V + ((size_t)k * P.nslots + sq) * DD, D);
                if (k > 0) load_tile(sB, S + ((size_t)(k - 1) * P.ne + e) * DD, D);
                tsync();
                if (k > 0)
                    for (int t = t0; t < DD; t += blockDim.x) sX[t] = u_add(sX[t], mm_el(sA, sB, D, t / D, t % D));
                tsync();
                if (k < P.Nt - 1) {
                    const cd *Sk = S + ((size_t)k * P.ne + e) * DD;
                    for (int w = t0; w < DD; w += blockDim.x) sB[w] = u_sub(Stot[w], Sk[w]);
                }
                tsync();
                if (k < P.Nt - 1)
                    for (int t = t0; t < DD; t += blockDim.x) sX[t] = u_add(sX[t], mm_el(sB, sA, D, t / D, t % D));
            }
            for (int t = t0; t < DD; t += blockDim.x) {
                cd acc = sX[t];
                for (int k = 0; k < P.Nt; ++k) acc = u_add(acc, V[((size_t)k * P.nslots + smix) * DD + t]);
                sX[t] = acc;
            }
            out = Uedxa;
            oidx = (size_t)e * P.na + q;
        }
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) out[cm(D, oidx, t / D, t % D)] = mm_el(sU, sX, D, t / D, t % D);
        tsync();
    }
}

// O_{k,e} = C_{k-1}^dagger (Herror_e / eps) C_{k-1}: items (k, e)
__global__ __launch_bounds__(BLOCK) void k_u_interaction(grape::DevProblem P, const double *x, const cd *C, cd *O,
                                                         cd *gscr) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sC = tiles(lds, gscr, D), *sH = sC + DD, *sT = sH + DD;
    for (long item = blockIdx.x; item < (long)P.Nt * P.ne; item += gridDim.x) {
        const int k = (int)(item % P.Nt), e = (int)(item / P.Nt);
        if (k > 0) load_tile(sC, C + (size_t)(k - 1) * DD, D);
        else identity_tile(sC, D);
        const double *xk = x + (size_t)k * P.np, *xadd = x + (size_t)P.np * P.Nt;
        grape::Pert none;
        none.var = -1;
        none.index = 0;
        none.delta = 0.0;
        for (int t = t0; t < DD; t += blockDim.x) {  // Herror_e(k, x_k, x_add, eps) = eps sum_t c_t OP_t, then / eps
            cd h{0.0, 0.0};
            for (int q = P.err_off[e]; q < P.err_off[e + 1]; ++q) {
                const grape::Term tm = P.err[q];
                h = u_add(h, u_mul(grape::term_coef(tm, k + 1, xk, xadd, none), P.ops[(size_t)tm.op * DD + t]));
            }
            sH[t] = u_scale(1.0 / P.eps, u_scale(P.eps, h));
        }
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) sT[t] = mm_el(sH, sC, D, t / D, t % D);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) O[cm(D, (size_t)e * P.Nt + k, t / D, t % D)] = mmh_el(sC, sT, D, t / D, t % D);
        tsync();
    }
}

// closure fallback: O_{k,e} = C_{k-1}^dagger Oerr_{k,e} C_{k-1}, Oerr host-evaluated (column-major)
__global__ __launch_bounds__(BLOCK) void k_u_interaction_table(grape::DevProblem P, const cd *Oerr, const cd *C,
                                                               cd *O, cd *gscr) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sC = tiles(lds, gscr, D), *sH = sC + DD, *sT = sH + DD;
    for (long item = blockIdx.x; item < (long)P.Nt * P.ne; item += gridDim.x) {
        const int k = (int)(item % P.Nt), e = (int)(item / P.Nt);
        if (k > 0) load_tile(sC, C + (size_t)(k - 1) * DD, D);
        else identity_tile(sC, D);
        for (int t = t0; t < DD; t += blockDim.x) sH[t] = Oerr[cm(D, (size_t)k * P.ne + e, t / D, t % D)];
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) sT[t] = mm_el(sH, sC, D, t / D, t % D);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) O[cm(D, (size_t)e * P.Nt + k, t / D, t % D)] = mmh_el(sC, sT, D, t / D, t % D);
        tsync();
    }
}

// expectation values: one thread per error source walks the time steps
__global__ void k_u_expect(grape::DevProblem P, const cd *O, double *ev) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.ne) return;
    const int D = P.D;
    cd acc{0.0, 0.0};
    for (int k = 0; k < P.Nt; ++k) {
        if (P.gen_proj) {  // tr(P0 O) = sum_ij P0_ij O_ji for a general projector
            for (int i = 0; i < D; ++i)
                for (int j = 0; j < D; ++j)
                    acc = u_add(acc, u_mul(P.P0g[i * D + j], O[cm(D, (size_t)e * P.Nt + k, j, i)]));
        } else {
            for (int i = 0; i < D; ++i) acc = u_add(acc, u_scale(P.W[i], O[cm(D, (size_t)e * P.Nt + k, i, i)]));
        }
        ev[(size_t)e * P.Nt + k] = P.dt * acc.re / P.Dtr;
    }
}

// one workgroup per item for d <= kMaxD (LDS tiles), kResident striding workgroups above
inline unsigned grid_for(int D, long items) {
    const long g = D <= kMaxD ? items : (items < kResident ? items : kResident);
    return (unsigned)(g > 0 ? g : 1);
}

}  // namespace

hipError_t launch_chain(const UProblem &P, const cd *E, cd *C, hipStream_t st) {
    hipLaunchKernelGGL(k_u_chain, dim3(1), dim3(BLOCK), 0, st, P, E, C);
    return hipGetLastError();
}

hipError_t launch_interaction(const grape::DevProblem &P, const double *x, const cd *C, cd *O, cd *gscr,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_u_interaction, dim3(grid_for(P.D, (long)P.Nt * P.ne)), dim3(BLOCK), 0, st, P, x, C, O, gscr);
    return hipGetLastError();
}

hipError_t launch_interaction_table(const grape::DevProblem &P, const cd *Oerr, const cd *C, cd *O, cd *gscr,
                                    hipStream_t st) {
    hipLaunchKernelGGL(k_u_interaction_table, dim3(grid_for(P.D, (long)P.Nt * P.ne)), dim3(BLOCK), 0, st, P, Oerr, C,
                       O, gscr);
    return hipGetLastError();
}

hipError_t launch_expectation(const grape::DevProblem &P, const cd *O, double *ev, hipStream_t st) {
    hipLaunchKernelGGL(k_u_expect, dim3((P.ne + 63) / 64), dim3(64), 0, st, P, O, ev);
    return hipGetLastError();
}

hipError_t launch_assembly(const UProblem &P, const UBuffers &B, hipStream_t st) {
    const int DD = P.D * P.D;
    hipLaunchKernelGGL(k_u_chain, dim3(1), dim3(BLOCK), 0, st, P, B.E, B.C);
    hipLaunchKernelGGL(k_u_vmats, dim3(grid_for(P.D, (long)P.Nt * P.nslots)), dim3(BLOCK), 0, st, P, B.E, B.C, B.V);
    if (P.ne > 0)
        hipLaunchKernelGGL(k_u_cumsum, dim3((P.ne * DD + 63) / 64), dim3(64), 0, st, P, B.V, B.S);
    hipLaunchKernelGGL(k_u_assemble, dim3(grid_for(P.D, (long)P.Nt * P.np * (1 + P.ne))), dim3(BLOCK), 0, st, P, B.C,
                       B.V, B.S, B.Udx, B.Uedx);
    const int nred = P.na + P.ne + P.na * P.ne;
    if (nred > 0)
        hipLaunchKernelGGL(k_u_reduce, dim3(grid_for(P.D, nred)), dim3(BLOCK), 0, st, P, B.C, B.V, B.S, B.Udxa, B.Ue,
                           B.Uedxa);
    return hipGetLastError();
}

}  // namespace grape_unitary
