// grape_unitary.hip -- materialised unitary derivatives for ONE control vector,
// the output of calculate_unitary_and_derivatives (src/UnitaryCalculations.jl:20-155)
// through the C ABI (grape_unitary_derivs).
//
// The propagator table E[k][v] (every finite-difference variant of every step,
// the closure call sites :45-90) comes from the small engine's k_expm (d <= 12) or
// the dense engine's k_dexp, converted from its register-file images (12 < d <= 64).  Then:
//   k_u_chain     C_k = E_k C_{k-1}                                    (:46)
//   k_u_vmats     V_{k,s} = C_k^-1 (stencil_s of E[k][.]) C_{k-1}     (:51-52,59-60,67-68,77-83,89-95)
//                 (Hermitian H0: C_k^-1 = C_k^dagger, C_k is unitary -- the reference's LU
//                  inverse differs at the 1e-15 level; general H0, e.g. a -i Gamma/2 decay term:
//                  k_u_inverse forms C_k^-1 by Gauss-Jordan with partial pivoting, :47)
//   k_u_cumsum    S_{k,e} = sum_{j<=k} V^err_{j,e}                      (:112)
//   k_u_assemble  U_dx[p,k] = U V^dx_{k,p};  U_derr_dx[p,k,e] =
//                 U (V^dx_{k,p} S_{k-1,e} + R_{k+1,e} V^dx_{k,p} + V^mix_{k,p,e}),
//                 R_{k+1,e} = S_{N-1,e} - S_{k,e}                       (:114-118, :124-139)
//   k_u_reduce    U_dx_add, U_derr, U_derr_dx_add (sums over k)         (:119-123, :140-151)
// Outputs are written straight into the reference's column-major layouts.
// General H0 also serves the fidelity path from these tensors (k_u_fid_head, k_u_fid_contract:
// FidelityCalculations.jl:19-119 as linear functionals of U_dx / U_derr_dx).
//
// This path is write-bound (U_dx is d^2 np N_t complex numbers) and runs once per
// call, not inside an optimiser loop, so its kernels are plain thread-per-element
// ones over d x d tiles: staged in LDS for d <= kMaxD (one workgroup per item), and
// for the dense engine's 12 < d <= 64 in global scratch (kTiles tiles per workgroup,
// kResident workgroups striding over the items, the operands L2-resident).
#include "grape_unitary_api.hpp"

#include <algorithm>

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

// Ci_k = C_k^-1 (UnitaryCalculations.jl:47, inv(cum_evo) for a general H0): Gauss-Jordan on
// [C_k | I] with partial pivoting (izamax: largest |re| + |im|, first maximum wins), items k.
// A zero pivot (singular chain) sets status bit 1 (Julia's inv throws SingularException).
__global__ __launch_bounds__(BLOCK) void k_u_inverse(UProblem P, const cd *C, cd *Ci, int *status) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    __shared__ cd fac[64];
    __shared__ int piv;
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sA = tiles(lds, P.gscr, D), *sI = sA + DD;
    for (long k = blockIdx.x; k < P.Nt; k += gridDim.x) {
        load_tile(sA, C + (size_t)k * DD, D);
        identity_tile(sI, D);
        tsync();
        bool singular = false;
        for (int c = 0; c < D; ++c) {
            if (t0 == 0) {
                int best = c;
                double bv = -1.0;
                for (int r = c; r < D; ++r) {
                    const double v = fabs(sA[r * D + c].re) + fabs(sA[r * D + c].im);
                    if (v > bv) {
                        bv = v;
                        best = r;
                    }
                }
                piv = bv > 0.0 ? best : -1;
            }
            tsync();
            const int pr = piv;
            if (pr < 0) {
                singular = true;
                break;
            }
            if (pr != c)
                for (int t = t0; t < 2 * D; t += blockDim.x) {
                    cd *M = t < D ? sA : sI;
                    const int j = t < D ? t : t - D;
                    const cd a = M[c * D + j];
                    M[c * D + j] = M[pr * D + j];
                    M[pr * D + j] = a;
                }
            tsync();
            const cd pv = sA[c * D + c];
            const double den = pv.re * pv.re + pv.im * pv.im;
            const cd rp{pv.re / den, -pv.im / den};
            tsync();
            for (int t = t0; t < 2 * D; t += blockDim.x) {  // pivot row * (1 / pivot)
                cd *M = t < D ? sA : sI;
                const int j = t < D ? t : t - D;
                M[c * D + j] = u_mul(M[c * D + j], rp);
            }
            for (int i = t0; i < D; i += blockDim.x) fac[i] = i == c ? cd{0.0, 0.0} : sA[i * D + c];
            tsync();
            for (int t = t0; t < 2 * DD; t += blockDim.x) {  // eliminate column c from every other row
                cd *M = t < DD ? sA : sI;
                const int e = t < DD ? t : t - DD, i = e / D, j = e % D;
                if (i != c) M[e] = u_sub(M[e], u_mul(fac[i], M[c * D + j]));
            }
            tsync();
        }
        if (singular) {
            if (t0 == 0) atomicOr(status, 2);
            for (int t = t0; t < DD; t += blockDim.x) Ci[(size_t)k * DD + t] = cd{0.0, 0.0};
        } else {
            for (int t = t0; t < DD; t += blockDim.x) Ci[(size_t)k * DD + t] = sI[t];
        }
        tsync();
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

// V_{k,s} = C_k^-1 stencil C_{k-1}, items (k, s); C_k^-1 = C_k^dagger unless Ci is given
__global__ __launch_bounds__(BLOCK) void k_u_vmats(UProblem P, const cd *E, const cd *C, const cd *Ci, cd *V) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sCk = tiles(lds, P.gscr, D), *sCp = sCk + DD, *sX = sCp + DD, *sT = sX + DD;
    for (long item = blockIdx.x; item < (long)P.Nt * P.nslots; item += gridDim.x) {
        const int k = (int)(item / P.nslots), s = (int)(item % P.nslots);
        load_tile(sCk, (Ci ? Ci : C) + (size_t)k * DD, D);
        if (k > 0) load_tile(sCp, C + (size_t)(k - 1) * DD, D);
        else identity_tile(sCp, D);
        const cd *Ek = E + (size_t)k * P.nv * DD;
        for (int t = t0; t < DD; t += blockDim.x) sX[t] = stencil(P, Ek, s, t);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) sT[t] = mm_el(sX, sCp, D, t / D, t % D);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x)
            V[((size_t)k * P.nslots + s) * DD + t] = Ci ? mm_el(sCk, sT, D, t / D, t % D) : mmh_el(sCk, sT, D, t / D, t % D);
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

// O_{k,e} = C_{k-1}^-1 (Herror_e / eps) C_{k-1}: items (k, e); C^-1 = C^dagger unless Ci is given
__global__ __launch_bounds__(BLOCK) void k_u_interaction(grape::DevProblem P, const double *x, const cd *C,
                                                         const cd *Ci, cd *O, cd *gscr) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sC = tiles(lds, gscr, D), *sH = sC + DD, *sT = sH + DD, *sCi = sT + DD;
    for (long item = blockIdx.x; item < (long)P.Nt * P.ne; item += gridDim.x) {
        const int k = (int)(item % P.Nt), e = (int)(item / P.Nt);
        if (k > 0) load_tile(sC, C + (size_t)(k - 1) * DD, D);
        else identity_tile(sC, D);
        if (Ci) {
            if (k > 0) load_tile(sCi, Ci + (size_t)(k - 1) * DD, D);
            else identity_tile(sCi, D);
        }
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
        for (int t = t0; t < DD; t += blockDim.x)
            O[cm(D, (size_t)e * P.Nt + k, t / D, t % D)] = Ci ? mm_el(sCi, sT, D, t / D, t % D) : mmh_el(sC, sT, D, t / D, t % D);
        tsync();
    }
}

// closure fallback: O_{k,e} = C_{k-1}^-1 Oerr_{k,e} C_{k-1}, Oerr host-evaluated (column-major)
__global__ __launch_bounds__(BLOCK) void k_u_interaction_table(grape::DevProblem P, const cd *Oerr, const cd *C,
                                                               const cd *Ci, cd *O, cd *gscr) {
    __shared__ cd lds[kTiles * kMaxD * kMaxD];
    const int D = P.D, DD = D * D, t0 = threadIdx.x;
    cd *sC = tiles(lds, gscr, D), *sH = sC + DD, *sT = sH + DD, *sCi = sT + DD;
    for (long item = blockIdx.x; item < (long)P.Nt * P.ne; item += gridDim.x) {
        const int k = (int)(item % P.Nt), e = (int)(item / P.Nt);
        if (k > 0) load_tile(sC, C + (size_t)(k - 1) * DD, D);
        else identity_tile(sC, D);
        if (Ci) {
            if (k > 0) load_tile(sCi, Ci + (size_t)(k - 1) * DD, D);
            else identity_tile(sCi, D);
        }
        for (int t = t0; t < DD; t += blockDim.x) sH[t] = Oerr[cm(D, (size_t)k * P.ne + e, t / D, t % D)];
        tsync();
        for (int t = t0; t < DD; t += blockDim.x) sT[t] = mm_el(sH, sC, D, t / D, t % D);
        tsync();
        for (int t = t0; t < DD; t += blockDim.x)
            O[cm(D, (size_t)e * P.Nt + k, t / D, t % D)] = Ci ? mm_el(sCi, sT, D, t / D, t % D) : mmh_el(sC, sT, D, t / D, t % D);
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

// ---------------------------------------------------------------------------
// General H0: the fidelity path from the materialised derivatives (FidelityCalculations.jl:19-119)
// ---------------------------------------------------------------------------
// Every F_dx / F_d2err_dx entry of the reference is a real-linear functional of one U_dx /
// U_derr_dx matrix X (its trace expressions are sums of tr(A X B), tr(A X^dagger B) and
// conj(tau) tr(A X)), so it is Re tr(X G) with one matrix G per error source (and one for the
// controls), formed once per evaluation by k_u_fid_head:
//   K = U0^dag U, tau = tr(PA K), F = [Re tr(PA K PB K^dag) + |tau|^2] / DD,
//   G = [(PB K^dag PA + PB^dag K^dag PA^dag + 2 conj(tau) PA) U0^dag] / DD          (:56-64)
//   Ke = U0^dag Ue, s = tr(PA Ke),
//   F_d2err = 2 [Re tr(PA Ke PB Ke^dag) + |s|^2 - (1 + D) Re tr(PA Ue^dag Ue)] / DD     (:79-85)
//   G_e = 2 [(PB Ke^dag PA + PB^dag Ke^dag PA^dag + 2 conj(s) PA) U0^dag
//            - (1 + D)(PA^dag + PA) Ue^dag] / DD                                     (:87-97)
// with PA = P0 P, PB = P (P0 with its nonzeros set to 1), DD = D (D + 1); the x_add entries
// add the target-derivative terms (:66-76, :99-113) directly.  k_u_fid_contract then forms
// Re tr(X G) = Re sum_t X[t] G[t] for every (k, p, e) (X column-major, G row-major: the same
// flat index).
namespace fid {

__device__ __forceinline__ double ctr_re(cd a, cd b) { return a.re * b.re - a.im * b.im; }

// C = op(A) op(B) on D x D row-major LDS tiles (op: 0 plain, 1 dagger), block-wide
__device__ void mm(cd *C, const cd *A, int ha, const cd *B, int hb, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
        const int i = t / D, j = t % D;
        cd s{0.0, 0.0};
        for (int l = 0; l < D; ++l) {
            const cd a = ha ? cd{A[l * D + i].re, -A[l * D + i].im} : A[i * D + l];
            const cd b = hb ? cd{B[j * D + l].re, -B[j * D + l].im} : B[l * D + j];
            s = u_add(s, u_mul(a, b));
        }
        C[t] = s;
    }
    tsync();
}

// block sum of one complex value per thread (red: blockDim.x scratch)
__device__ cd bsum(cd v, cd *red) {
    red[threadIdx.x] = v;
    tsync();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = u_add(red[threadIdx.x], red[threadIdx.x + w]);
        tsync();
    }
    const cd r = red[0];
    tsync();
    return r;
}
// tr(A B) = sum_ij A_ij B_ji
__device__ cd trace_ab(const cd *A, const cd *B, int D, cd *red) {
    cd s{0.0, 0.0};
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) s = u_add(s, u_mul(A[t], B[(t % D) * D + t / D]));
    return bsum(s, red);
}
// sum_ij A_ij conj(B_ij) = tr(A B^dagger)
__device__ cd trace_abh(const cd *A, const cd *B, int D, cd *red) {
    cd s{0.0, 0.0};
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) s = u_add(s, u_mul(A[t], cd{B[t].re, -B[t].im}));
    return bsum(s, red);
}
// column-major global matrix -> row-major LDS tile
__device__ void load_cm(cd *dst, const cd *src, int D) {
    for (int t = threadIdx.x; t < D * D; t += blockDim.x) dst[t] = src[(t / D) + (t % D) * D];
    tsync();
}
// U0(x_add [+ eps e_q]) of this evaluation: operator-basis target terms, or the host table (slot)
__device__ void target(cd *dst, const FidArgs &A, int slot) {
    const grape::DevProblem &P = A.P;
    const int D = P.D, DD = D * D;
    if (A.U0tab) {
        load_cm(dst, A.U0tab + (size_t)slot * DD, D);
        return;
    }
    grape::Pert pp;
    pp.var = slot > 0 ? grape::VAR_XADD : -1;
    pp.index = slot > 0 ? slot - 1 : 0;
    pp.delta = slot > 0 ? P.eps : 0.0;
    const double *xadd = A.x + (size_t)P.np * P.Nt;
    for (int t = threadIdx.x; t < DD; t += blockDim.x) {
        cd h{0.0, 0.0};
        for (int q = 0; q < P.n_tgt; ++q) {
            const grape::Term tm = P.tgt[q];
            h = u_add(h, u_mul(grape::term_coef(tm, 1, A.x, xadd, pp), P.ops[(size_t)tm.op * DD + t]));
        }
        dst[t] = h;
    }
    tsync();
}

}  // namespace fid

__global__ __launch_bounds__(BLOCK) void k_u_fid_head(FidArgs A) {
    __shared__ cd lds_sm[kFidTiles * kMaxD * kMaxD];
    __shared__ cd red[BLOCK];
    const grape::DevProblem &P = A.P;
    const int D = P.D, DD = D * D, np = P.np, na = P.na, ne = P.ne, Nt = P.Nt, nx = P.nx;
    const int MT = D <= kMaxD ? kMaxD * kMaxD : DD;
    cd *sm = D <= kMaxD ? lds_sm : A.scr;  // d > kMaxD: kFidTiles tiles of global scratch
    const double Dn = P.DD, Dtr = P.Dtr;
    cd *U = sm, *U0 = sm + MT, *PA = sm + 2 * MT, *PB = sm + 3 * MT, *K = sm + 4 * MT, *R = sm + 5 * MT,
       *T1 = sm + 6 * MT, *T2 = sm + 7 * MT, *T3 = sm + 8 * MT, *Ue = sm + 9 * MT, *Ke = sm + 10 * MT,
       *Re_ = sm + 11 * MT, *U0d = sm + 12 * MT, *Kd = sm + 13 * MT;
    for (int t = threadIdx.x; t < DD; t += blockDim.x) {
        U[t] = A.U[t];
        PA[t] = P.PA[t];
        PB[t] = P.PB[t];
    }
    tsync();
    fid::target(U0, A, 0);
    fid::mm(K, U0, 1, U, 0, D);    // K = U0^dag U
    const cd tau = fid::trace_ab(PA, K, D, red);
    fid::mm(T1, K, 0, PB, 0, D);   // K PB
    fid::mm(R, PA, 0, T1, 0, D);   // R = PA K PB
    const double F1 = fid::trace_abh(R, K, D, red).re;
    if (threadIdx.x == 0) A.F[0] = (F1 + tau.re * tau.re + tau.im * tau.im) / Dn;
    // G = (PB K^dag PA + PB^dag K^dag PA^dag + 2 conj(tau) PA) U0^dag / DD
    fid::mm(T1, K, 1, PA, 0, D);
    fid::mm(T2, PB, 0, T1, 0, D);
    fid::mm(T1, K, 1, PA, 1, D);
    fid::mm(T3, PB, 1, T1, 0, D);
    for (int t = threadIdx.x; t < DD; t += blockDim.x)
        T1[t] = u_add(u_add(T2[t], T3[t]), u_mul(cd{2.0 * tau.re, -2.0 * tau.im}, PA[t]));
    tsync();
    fid::mm(T2, T1, 0, U0, 1, D);
    for (int t = threadIdx.x; t < DD; t += blockDim.x) A.G[t] = u_scale(1.0 / Dn, T2[t]);
    tsync();
    // x_add: F_dx_add[q] = Re tr(U_dx_add[q] G) + target-derivative terms (:66-76)
    for (int q = 0; q < na; ++q) {
        fid::target(U0d, A, 1 + q);
        for (int t = threadIdx.x; t < DD; t += blockDim.x) U0d[t] = u_scale(P.inv_eps, u_sub(U0d[t], U0[t]));
        tsync();
        fid::mm(Kd, U0d, 1, U, 0, D);  // Kd = U0d^dag U
        fid::mm(T1, Kd, 0, PB, 0, D);
        fid::mm(T3, PA, 0, T1, 0, D);  // PA Kd PB
        const double a = fid::trace_abh(T3, K, D, red).re + fid::trace_abh(R, Kd, D, red).re;
        const cd tk = fid::trace_ab(PA, Kd, D, red);
        cd lin{0.0, 0.0};
        const cd *X = A.Udxa + (size_t)q * DD;
        for (int t = threadIdx.x; t < DD; t += blockDim.x) lin.re += fid::ctr_re(X[t], T2[t]) / Dn;  // T2 = DD G
        lin = fid::bsum(lin, red);
        if (threadIdx.x == 0)
            A.Fdx[(size_t)np * Nt + q] = lin.re + (a + 2.0 * (tau.re * tk.re + tau.im * tk.im)) / Dn;
    }
    for (int e = 0; e < ne; ++e) {
        fid::load_cm(Ue, A.Ue + (size_t)e * DD, D);
        fid::mm(Ke, U0, 1, Ue, 0, D);  // Ke = U0^dag Ue
        const cd sg = fid::trace_ab(PA, Ke, D, red);
        fid::mm(T1, Ke, 0, PB, 0, D);
        fid::mm(Re_, PA, 0, T1, 0, D);  // PA Ke PB
        const double f1 = fid::trace_abh(Re_, Ke, D, red).re;
        fid::mm(T1, Ue, 1, Ue, 0, D);
        const double f2 = fid::trace_ab(PA, T1, D, red).re;
        if (threadIdx.x == 0) A.Fd2[e] = 2.0 * (f1 + sg.re * sg.re + sg.im * sg.im - (1.0 + Dtr) * f2) / Dn;
        // G_e
        fid::mm(T1, Ke, 1, PA, 0, D);
        fid::mm(T2, PB, 0, T1, 0, D);
        fid::mm(T1, Ke, 1, PA, 1, D);
        fid::mm(T3, PB, 1, T1, 0, D);
        for (int t = threadIdx.x; t < DD; t += blockDim.x)
            T1[t] = u_add(u_add(T2[t], T3[t]), u_mul(cd{2.0 * sg.re, -2.0 * sg.im}, PA[t]));
        tsync();
        fid::mm(T2, T1, 0, U0, 1, D);
        for (int t = threadIdx.x; t < DD; t += blockDim.x) {  // (PA^dag + PA)
            const int i = t / D, j = t % D;
            T1[t] = u_add(cd{PA[j * D + i].re, -PA[j * D + i].im}, PA[t]);
        }
        tsync();
        fid::mm(T3, T1, 0, Ue, 1, D);
        cd *Ge = A.G + (size_t)(1 + e) * DD;
        for (int t = threadIdx.x; t < DD; t += blockDim.x) {
            T2[t] = u_scale(2.0 / Dn, u_sub(T2[t], u_scale(1.0 + Dtr, T3[t])));  // kept for the x_add entries
            Ge[t] = T2[t];
        }
        tsync();
        // F_d2err_dx_add[q, e] = Re tr(U_derr_dx_add[q, e] G_e) + target-derivative terms (:99-113)
        for (int q = 0; q < na; ++q) {
            fid::target(U0d, A, 1 + q);
            for (int t = threadIdx.x; t < DD; t += blockDim.x) U0d[t] = u_scale(P.inv_eps, u_sub(U0d[t], U0[t]));
            tsync();
            fid::mm(Kd, U0d, 1, Ue, 0, D);  // Ked = U0d^dag Ue
            fid::mm(T1, Kd, 0, PB, 0, D);
            fid::mm(T3, PA, 0, T1, 0, D);   // PA Ked PB
            const double a = fid::trace_abh(T3, Ke, D, red).re + fid::trace_abh(Re_, Kd, D, red).re;
            const cd tk = fid::trace_ab(PA, Kd, D, red);
            cd lin{0.0, 0.0};
            const cd *X = A.Uedxa + ((size_t)e * na + q) * DD;
            for (int t = threadIdx.x; t < DD; t += blockDim.x) lin.re += fid::ctr_re(X[t], T2[t]);
            lin = fid::bsum(lin, red);
            if (threadIdx.x == 0)
                A.Fd2dx[(size_t)e * nx + (size_t)np * Nt + q] =
                    lin.re + 2.0 * (a + 2.0 * (sg.re * tk.re + sg.im * tk.im)) / Dn;
        }
    }
}

// Re tr(X G) for every (k, p) and (k, p, e): one wave per item
__global__ __launch_bounds__(BLOCK) void k_u_fid_contract(FidArgs A) {
    const grape::DevProblem &P = A.P;
    const int DD = P.D * P.D, np = P.np, Nt = P.Nt;
    const int lane = threadIdx.x & 63;
    const long items = (long)Nt * np * (1 + P.ne);
    for (long item = (long)blockIdx.x * (BLOCK / 64) + threadIdx.x / 64; item < items;
         item += (long)gridDim.x * (BLOCK / 64)) {
        const int e = (int)(item / ((long)Nt * np)) - 1;
        const long m = item % ((long)Nt * np);  // k * np + p
        const cd *X = e < 0 ? A.Udx + (size_t)m * DD : A.Uedx + ((size_t)e * Nt * np + m) * DD;
        const cd *G = A.G + (size_t)(1 + e) * DD;
        double s = 0.0;
        for (int t = lane; t < DD; t += 64) s += fid::ctr_re(X[t], G[t]);
        for (int w = 32; w > 0; w >>= 1) s += __shfl_xor(s, w, 64);
        if (lane == 0) {
            if (e < 0) A.Fdx[m] = s;
            else A.Fd2dx[(size_t)e * P.nx + m] = s;
        }
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

hipError_t launch_inverse(const UProblem &P, const cd *C, cd *Ci, int *status, hipStream_t st) {
    if (P.D > kMaxD && !P.gscr) return hipErrorInvalidValue;  // d > kMaxD: the tiles live in P.gscr
    hipLaunchKernelGGL(k_u_inverse, dim3(grid_for(P.D, P.Nt)), dim3(BLOCK), 0, st, P, C, Ci, status);
    return hipGetLastError();
}

hipError_t launch_interaction(const grape::DevProblem &P, const double *x, const cd *C, const cd *Ci, cd *O,
                              cd *gscr, hipStream_t st) {
    hipLaunchKernelGGL(k_u_interaction, dim3(grid_for(P.D, (long)P.Nt * P.ne)), dim3(BLOCK), 0, st, P, x, C, Ci, O,
                       gscr);
    return hipGetLastError();
}

hipError_t launch_interaction_table(const grape::DevProblem &P, const cd *Oerr, const cd *C, const cd *Ci, cd *O,
                                    cd *gscr, hipStream_t st) {
    hipLaunchKernelGGL(k_u_interaction_table, dim3(grid_for(P.D, (long)P.Nt * P.ne)), dim3(BLOCK), 0, st, P, Oerr, C,
                       Ci, O, gscr);
    return hipGetLastError();
}

hipError_t launch_expectation(const grape::DevProblem &P, const cd *O, double *ev, hipStream_t st) {
    hipLaunchKernelGGL(k_u_expect, dim3((P.ne + 63) / 64), dim3(64), 0, st, P, O, ev);
    return hipGetLastError();
}

hipError_t launch_fidelity(const FidArgs &A, hipStream_t st) {
    if (A.P.D > kMaxD && !A.scr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_u_fid_head, dim3(1), dim3(BLOCK), 0, st, A);
    const long items = (long)A.P.Nt * A.P.np * (1 + A.P.ne);
    const long per = BLOCK / 64;
    hipLaunchKernelGGL(k_u_fid_contract, dim3((unsigned)std::min<long>((items + per - 1) / per, 4096)), dim3(BLOCK), 0,
                       st, A);
    return hipGetLastError();
}

hipError_t launch_assembly(const UProblem &P, const UBuffers &B, hipStream_t st) {
    const int DD = P.D * P.D;
    hipLaunchKernelGGL(k_u_chain, dim3(1), dim3(BLOCK), 0, st, P, B.E, B.C);
    if (B.Ci) {
        if (const hipError_t e = launch_inverse(P, B.C, B.Ci, B.status, st)) return e;
    }
    hipLaunchKernelGGL(k_u_vmats, dim3(grid_for(P.D, (long)P.Nt * P.nslots)), dim3(BLOCK), 0, st, P, B.E, B.C, B.Ci,
                       B.V);
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
