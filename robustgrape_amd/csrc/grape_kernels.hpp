// grape_kernels.hpp -- the hot-path kernels (small-d row-group engine).
//
//   k_expm    one row group per (eval b, step k, variant v): builds
//             A = -i dt H(x_b,k perturbed by v) from the operator basis and
//             computes E = exp(A) (Pade m <= 9 in registers); m = 13 items are
//             parked for k_expm13.                      UnitaryCalculations.jl:45,51,59
//   k_expm13  m = 13 scaling-and-squaring for parked items.
//   k_scan    one workgroup per eval: chunked prefix product of the nominal
//             propagators (local chains + Hillis-Steele over chunk totals),
//             fidelity F, the gradient kernel M = G U and the per-chunk
//             M'_c = Carry_c M Carry_c^dagger.         UnitaryCalculations.jl:46-47,99
//                                                        FidelityCalculations.jl:32-54
//   k_grad    one row group per (b, k): Z_k = (C_{k-1} M C_k^dagger)^T and
//             F_dx[p,k] = Re sum(Z_k o dE_{k,p}).     FidelityCalculations.jl:56-76
//   k_reduce_add  sum over k of the x_add contributions (only when H0 depends on x_add).
//
// Gradient algebra (verified against the reference formulas at rounding level):
//   F_dx[p,k] = Re tr(G U_dx[p,k]),  G = 2(P K^dag + conj(tau) I) W U0^dag / (D(D+1)),
//   K = U0^dag U, tau = tr(W K), U_dx[p,k] = U C_k^-1 dE C_{k-1} (UnitaryCalculations.jl:52,116)
//   => F_dx[p,k] = Re tr(C_{k-1} M C_k^dag dE_{k,p}), M = G U, with C_k^-1 = C_k^dag
//      (C_k is unitary; the reference's LU inverse differs at the 1e-15 level).
#pragma once
#include "grape_device.hpp"

namespace grape {

struct Term {  // layout-identical to grape_term (include/grape.h)
    int32_t op, var, index, func;
    double a, b, sre, sim;
};

enum { VAR_ONE = 0, VAR_X = 1, VAR_XADD = 2, VAR_TSTEP = 3 };
enum { FN_ONE = 0, FN_LINEAR = 1, FN_COS = 2, FN_SIN = 3, FN_CIS = 4 };

struct Pert {
    int var;      // -1: none
    int index;
    double delta;
};

// One propagator variant of a time step: the closure call sites of
// UnitaryCalculations.jl:45-90 (perturb one variable by delta; optionally add
// the error Hamiltonian e with strength errval).
struct VSpec {
    Pert pert;
    int err;        // -1: none
    double errval;
};

// Everything a kernel needs to know about the problem (passed by value).
struct DevProblem {
    int D, Nt, np, na, ne, nx;
    int nv;              // propagator variants per step (nominal + FD variants)
    int n_h0, n_tgt;
    int xadd_dep;        // H0 depends on x_add -> x_add FD variants exist
    int L, nchunks;      // scan chunking
    // variant layout (see grape_engine.hip: build_variants)
    int off_dx, off_dxa, off_dx2, off_err, err_stride;
    double dt, eps, eps2, inv_eps, inv_eps2sq, DD, Dtr;
    const cd *ops;       // [n_ops][D][D] row-major
    const Term *h0;
    const Term *tgt;
    const Term *err;     // error-source terms
    const int *err_off;  // [ne+1]
    const VSpec *vs;     // [nv]
    const double *W;     // projector diagonal (weights)
};

struct DevBatch {
    int nb;                 // evaluations in this launch
    const double *x;        // [nb][nx]
    cd *E;                  // [nb][Nt][nv][D][D]
    cd *Q;                  // [nb][Nt][D][D]
    cd *Mc;                 // [nb][nchunks][D][D]
    double *F;              // [nb]
    double *Fdx;            // [nb][nx]
    double *part_add;       // [nb][Nt][na]   (xadd_dep only)
    double *tgt_part;       // [nb][na]
    cd *Carry;              // [nb][nchunks][D][D]  C_{cL-1} (identity for c = 0)
    cd *Ub;                 // [nb][D][D]           U = C_Nt
    cd *Me;                 // [nb][ne][nchunks][3][D][D]  M'_{c,e}, T_c, Ttot_c (error path)
    double *Fd2;            // [nb][ne]
    double *Fd2dx;          // [nb][ne][nx]
    int *overflow;          // parked m=13 item ids
    int *overflow_count;
    int *status;            // bit 0: singular Pade denominator
};

__device__ __forceinline__ cd term_coef(const Term &t, int nt1, const double *xk, const double *xadd,
                                        const Pert &pp) {
    double v = 1.0;
    if (t.var == VAR_X) v = xk[t.index];
    else if (t.var == VAR_XADD) v = xadd[t.index];
    else if (t.var == VAR_TSTEP) v = (double)nt1;
    if (t.var == pp.var && t.index == pp.index) v = v + pp.delta;
    const double arg = t.a * v + t.b;  // built with -ffp-contract=off: no fusion, like Julia
    double fr = 1.0, fi = 0.0;
    if (t.func == FN_LINEAR) fr = arg;
    else if (t.func == FN_COS) fr = cos(arg);
    else if (t.func == FN_SIN) fr = sin(arg);
    else if (t.func == FN_CIS) {
        fr = cos(arg);
        fi = sin(arg);
    }
    return cmul(cmake(t.sre, t.sim), cmake(fr, fi));
}

template <int D>
__device__ __forceinline__ void build_row(const cd *ops, const Term *terms, int n, int i, int nt1,
                                          const double *xk, const double *xadd, const Pert &pp, cd (&h)[D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) h[j] = czero();
    for (int t = 0; t < n; ++t) {
        const Term tm = terms[t];
        const cd c = term_coef(tm, nt1, xk, xadd, pp);
        const cd *op = ops + (size_t)tm.op * D * D + i * D;
#pragma unroll
        for (int j = 0; j < D; ++j) h[j] = cadd(h[j], cmul(c, op[j]));
    }
}

// ---------------------------------------------------------------------------
// k_expm: all propagator variants of the batch
// ---------------------------------------------------------------------------
template <int D, bool ERR>
struct ItemBuilder {  // rebuilds this lane's row of A = -i dt H for one (b, k, v) item
    const DevProblem *P;
    const double *xk, *xadd;
    int i, nt1;
    VSpec vs;
    bool valid;
    __device__ __forceinline__ void operator()(cd (&a)[D]) const {
        cd h[D];
        build_row<D>(P->ops, P->h0, P->n_h0, i, nt1, xk, xadd, vs.pert, h);
        if (ERR && vs.err >= 0) {  // exp(-i dt (Herror(.., err) + H0(..)))   UnitaryCalculations.jl:67-68
            cd he[D];
            const int o0 = P->err_off[vs.err], o1 = P->err_off[vs.err + 1];
            build_row<D>(P->ops, P->err + o0, o1 - o0, i, nt1, xk, xadd, vs.pert, he);
#pragma unroll
            for (int j = 0; j < D; ++j) h[j] = cadd(cscale(vs.errval, he[j]), h[j]);
        }
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = valid ? cmake(P->dt * h[j].im, -P->dt * h[j].re) : czero();
    }
};

// Parks an item whose Pade degree is > 5: A goes to its output slot, the id to the list.
template <int D>
__device__ __forceinline__ void park(Group<D> &G, cd *slot_row, const cd (&a)[D], long gid, int *list, int *count) {
#pragma unroll
    for (int j = 0; j < D; ++j) slot_row[j] = a[j];
    if (G.i == 0) list[atomicAdd(count, 1)] = (int)gid;
}

// ERR = false for problems without error sources (keeps the error-term
// builder, and its registers, out of the common kernel).
template <int D, bool ERR>
__global__ __launch_bounds__(64, (D <= 9 ? 3 : 2)) void k_expm(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const long nitems = (long)B.nb * P.Nt * P.nv;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    const int v = (int)(gidc % P.nv);
    const int k = (int)((gidc / P.nv) % P.Nt);
    const int b = (int)(gidc / ((long)P.nv * P.Nt));
    const double *xb = B.x + (size_t)b * P.nx;
    ItemBuilder<D, ERR> rebuild{&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, G.i, k + 1, P.vs[v], valid};
    cd a[D], x[D];
    rebuild(a);
    int singular = 0, s = 0;
    const int m = expm_prologue<D>(G, a, x, valid, s);
    cd *out = B.E + (size_t)gidc * D * D + G.i * D;
    if (m == 3 || m == 5) expm_low<D>(G, m, a, x, valid, singular, rebuild);
    if (valid) {
        if (m > 5) {
            park<D>(G, out, a, gid, B.overflow, B.overflow_count);
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) out[j] = x[j];
        }
        if (singular) atomicOr(B.status, 1);
    }
}

// Items parked by k_expm / k_expm_raw (slots hold A, overwritten with exp(A)).
template <int D>
__global__ __launch_bounds__(64) void k_expm_high(cd *slots, const int *list, const int *count, int *status) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const int n = *count;
    for (int base = blockIdx.x * Geo<D>::GPW; base < n; base += gridDim.x * Geo<D>::GPW) {
        const int idx = base + G.g;
        const bool valid = G.lane_ok && idx < n;
        cd *slot = slots + (size_t)(valid ? list[idx] : 0) * D * D + G.i * D;
        cd a[D], x[D];
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = valid ? slot[j] : czero();
        int singular = 0, s = 0;
        const int m = expm_prologue<D>(G, a, x, valid, s);
        if (m > 0) expm_high<D>(G, m, s, a, x, valid, singular);
        gsync();
        if (valid) {
#pragma unroll
            for (int j = 0; j < D; ++j) slot[j] = x[j];
            if (singular) atomicOr(status, 1);
        }
    }
}

// Standalone batched expm of column-major matrices (grape_expm_batch); writes
// row-major tiles that k_transpose_tiles turns back into column-major.
template <int D>
__global__ __launch_bounds__(64) void k_expm_raw(const cd *A, cd *E, int n, int *overflow, int *overflow_count,
                                                 int *status, int *mstats) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const int gid = blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < n;
    const cd *src = A + (size_t)(valid ? gid : 0) * D * D;
    auto reload = [&](cd (&a)[D]) {
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = valid ? src[G.i + j * D] : czero();
    };
    cd a[D], x[D];
    reload(a);
    int singular = 0, s = 0;
    const int m = expm_prologue<D>(G, a, x, valid, s);
    if (m == 3 || m == 5) expm_low<D>(G, m, a, x, valid, singular, reload);
    cd *out = E + (size_t)(valid ? gid : 0) * D * D + G.i * D;
    if (valid) {
        if (m > 5) {
            park<D>(G, out, a, gid, overflow, overflow_count);
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) out[j] = x[j];
        }
        if (G.i == 0) {
            const int slot = m <= 3 ? 0 : m == 5 ? 1 : m == 7 ? 2 : m == 9 ? 3 : 4;
            atomicAdd(mstats + slot, 1);
        }
        if (singular) atomicOr(status, 1);
    }
}

template <int D>
__global__ void k_transpose_tiles(const cd *in, cd *out, int n) {  // row-major -> column-major
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)n * D * D) return;
    const long m = t / (D * D);
    const int r = (int)(t % (D * D)) / D, c = (int)(t % (D * D)) % D;
    out[m * D * D + r + c * D] = in[m * D * D + r * D + c];
}

// ---------------------------------------------------------------------------
// k_scan: one workgroup (W waves) per evaluation
// ---------------------------------------------------------------------------
template <int D, int W>
__global__ __launch_bounds__(64 * W) void k_scan(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int GPW = Geo<D>::GPW, GCD = Geo<D>::GROUP_CD, TILE = Geo<D>::TILE;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    Group<D> G = make_group<D>(lds + wave * GPW * GCD, lane);
    cd *S1 = lds + W * GPW * GCD, *S2 = S1 + TILE, *S3 = S2 + TILE;
    const int c = wave * GPW + G.g;  // chunk owned by this group
    const int i = G.i;
    const int b = blockIdx.x;
    const bool gvalid = G.lane_ok && c < P.nchunks;
    auto tile_of = [&](int cc) -> cd * {
        return lds + (cc / GPW) * GPW * GCD + (cc % GPW) * GCD;
    };
    const cd *Eb = B.E + (size_t)b * P.Nt * P.nv * TILE;
    cd *Qb = B.Q + (size_t)b * P.Nt * TILE;

    // Phase A: local inclusive chain Q_k = E_k ... E_{cL}
    cd q[D], e[D], t[D];
    const int k0 = c * P.L;
    for (int j = 0; j < P.L; ++j) {
        const int k = k0 + j;
        const bool act = gvalid && k < P.Nt;
        if (act) {
            const cd *src = Eb + ((size_t)k * P.nv) * TILE + i * D;
#pragma unroll
            for (int jj = 0; jj < D; ++jj) e[jj] = src[jj];
        } else {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) e[jj] = czero();
        }
        if (j == 0) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) q[jj] = e[jj];
        } else {
            mm_tile<D>(e, G.tile, q);
        }
        gsync();
        if (act) {
            tile_store_row(G, q, true);
            cd *dst = Qb + (size_t)k * TILE + i * D;
#pragma unroll
            for (int jj = 0; jj < D; ++jj) dst[jj] = q[jj];
        }
        gsync();
    }
    // Phase B: inclusive scan of the chunk totals, P_c = T_c ... T_0 (Hillis-Steele)
    for (int o = 1; o < P.nchunks; o <<= 1) {
        const bool doit = gvalid && c >= o;
        if (doit) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) q[jj] = G.tile[i * D + jj];
            mm_tile<D>(q, tile_of(c - o), t);
        }
        gsync();
        if (doit) tile_store_row(G, t, true);
        gsync();
    }
    // Phase C: fidelity and M = G U on group 0 (everyone keeps the barrier sequence)
    const bool f0 = (c == 0) && G.lane_ok;
    const cd *Ut = tile_of(P.nchunks - 1);
    const double *xb = B.x + (size_t)b * P.nx;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    Pert none;
    none.var = -1; none.index = 0; none.delta = 0.0;
    cd l[D], kk[D];
    build_row<D>(P.ops, P.tgt, P.n_tgt, i, 1, xb, xadd, none, l);  // U0 row i
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) S1[i * D + jj] = l[jj];
    }
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) l[r] = cconj(S1[r * D + i]);
    mm_tile<D>(l, Ut, kk);  // K = U0^dag U, row i
    const double wi = P.W[i];
    double part = 0.0;
    cd kii = czero();
#pragma unroll
    for (int jj = 0; jj < D; ++jj) {
        const double pj = P.W[jj] != 0.0 ? 1.0 : 0.0;
        part += pj * (kk[jj].re * kk[jj].re + kk[jj].im * kk[jj].im);
        if (jj == i) kii = kk[jj];
    }
    const double sum_part = group_sum(G, wi * part, f0);
    const double tau_re = group_sum(G, wi * kii.re, f0);
    const double tau_im = group_sum(G, wi * kii.im, f0);
    // F = [Re tr(W K P K^dag) + |tau|^2] / (D(D+1))          (FidelityCalculations.jl:54)
    const double Fv = (sum_part + tau_re * tau_re + tau_im * tau_im) / P.DD;
    // M = G U = 2 (P K^dag W K + conj(tau) W K) / (D(D+1))
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) S2[i * D + jj] = kk[jj];
    }
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) l[r] = cscale(P.W[r], cconj(S2[r * D + i]));
    mm_tile<D>(l, S2, t);
    {
        const double pi_ = wi != 0.0 ? 1.0 : 0.0;
        const double sc = 2.0 / P.DD;
#pragma unroll
        for (int jj = 0; jj < D; ++jj)
            l[jj] = cscale(sc, cadd(cscale(pi_, t[jj]), cmul(cmake(tau_re, -tau_im), cscale(wi, kk[jj]))));
    }
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) S3[i * D + jj] = l[jj];
    }
    gsync();
    // target derivative part of F_dx_add (FidelityCalculations.jl:34-40, 67-76)
    for (int qd = 0; qd < P.na; ++qd) {
        Pert pq;
        pq.var = VAR_XADD; pq.index = qd; pq.delta = P.eps;
        build_row<D>(P.ops, P.tgt, P.n_tgt, i, 1, xb, xadd, pq, l);
        build_row<D>(P.ops, P.tgt, P.n_tgt, i, 1, xb, xadd, none, t);
        if (f0) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) S1[i * D + jj] = cscale(P.inv_eps, csub(l[jj], t[jj]));
        }
        gsync();
#pragma unroll
        for (int r = 0; r < D; ++r) l[r] = cconj(S1[r * D + i]);
        mm_tile<D>(l, Ut, t);  // Kd = U0d^dag U
        double pr = 0.0;
        cd kdii = czero();
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            const double pj = P.W[jj] != 0.0 ? 1.0 : 0.0;
            pr += pj * (t[jj].re * kk[jj].re + t[jj].im * kk[jj].im);
            if (jj == i) kdii = t[jj];
        }
        const double s1 = group_sum(G, wi * pr, f0);
        const double tr_re = group_sum(G, wi * kdii.re, f0);
        const double tr_im = group_sum(G, wi * kdii.im, f0);
        const double val = (2.0 * s1 + 2.0 * (tau_re * tr_re + tau_im * tr_im)) / P.DD;
        if (f0 && i == 0) {
            if (P.xadd_dep) B.tgt_part[(size_t)b * P.na + qd] = val;
            else B.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + qd] = val;
        }
    }
    if (f0 && i == 0) B.F[b] = Fv;
    if (f0 && B.Ub) {  // U for the error path
        cd *du = B.Ub + (size_t)b * TILE + i * D;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) du[jj] = Ut[i * D + jj];
    }
    // Phase D: M'_c = Carry_c M Carry_c^dag, Carry_c = P_{c-1} (identity for c = 0)
    if (gvalid && B.Carry) {  // carries for the error path (identity for chunk 0)
        cd *dc = B.Carry + ((size_t)b * P.nchunks + c) * TILE + i * D;
        const cd *Cr = c > 0 ? tile_of(c - 1) : nullptr;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) dc[jj] = Cr ? Cr[i * D + jj] : cmake(jj == i ? 1.0 : 0.0, 0.0);
    }
    if (gvalid) {
        cd mc[D];
        if (c == 0) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) mc[jj] = S3[i * D + jj];
        } else {
            const cd *Cr = tile_of(c - 1);
#pragma unroll
            for (int jj = 0; jj < D; ++jj) q[jj] = Cr[i * D + jj];
            mm_tile<D>(q, S3, t);
            mm_tile<D, true, true>(t, Cr, mc);
        }
        cd *dst = B.Mc + ((size_t)b * P.nchunks + c) * TILE + i * D;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) dst[jj] = mc[jj];
    }
}

// ---------------------------------------------------------------------------
// k_grad: one row group per (b, k)
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64, (D <= 9 ? 4 : 2)) void k_grad(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int TILE = Geo<D>::TILE;
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const long nitems = (long)B.nb * P.Nt;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    const int k = (int)(gidc % P.Nt), b = (int)(gidc / P.Nt);
    const int c = k / P.L, j0 = k - c * P.L;
    const int i = G.i;
    const cd *Qk = B.Q + ((size_t)b * P.Nt + k) * TILE;
    const cd *Mc = B.Mc + ((size_t)b * P.nchunks + c) * TILE;
    cd ql[D], t[D], z[D];
#pragma unroll
    for (int jj = 0; jj < D; ++jj) ql[jj] = cconj(Qk[i * D + jj]);
    if (valid) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) G.tile[i * D + jj] = Mc[i * D + jj];
    }
    gsync();
    mm_tile<D, true>(ql, G.tile, t);  // conj(Q_k) . M'^T
    gsync();
    if (j0 > 0) {
        if (valid) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) G.tile[i * D + jj] = Qk[i * D + jj - TILE];
        }
        gsync();
        mm_tile<D, true>(t, G.tile, z);  // . Q_{k-1}^T
        gsync();
    } else {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) z[jj] = t[jj];
    }
    const cd *E0 = B.E + (((size_t)b * P.Nt + k) * P.nv) * TILE + i * D;
    cd e0[D];
#pragma unroll
    for (int jj = 0; jj < D; ++jj) e0[jj] = E0[jj];
    const int nvg = P.np + (P.xadd_dep ? P.na : 0);  // dx then dxa variants are contiguous
    for (int vi = 0; vi < nvg; ++vi) {
        const int v = P.off_dx + vi;
        const cd *Ev = E0 + (size_t)v * TILE;
        double s = 0.0;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
            const cd de = cscale(P.inv_eps, csub(Ev[jj], e0[jj]));
            s += z[jj].re * de.re - z[jj].im * de.im;
        }
        s = group_sum(G, s, valid);
        if (valid && i == 0) {
            if (vi < P.np) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + vi] = s;
            else B.part_add[((size_t)b * P.Nt + k) * P.na + (vi - P.np)] = s;
        }
    }
}

// F_dx_add = target part + sum_k per-step contributions (xadd_dep only)
__global__ void k_reduce_add(DevProblem P, DevBatch B) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B.nb * P.na) return;
    const int b = t / P.na, q = t % P.na;
    double s = 0.0;
    for (int k = 0; k < P.Nt; ++k) s += B.part_add[((size_t)b * P.Nt + k) * P.na + q];
    B.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + q] = B.tgt_part[(size_t)b * P.na + q] + s;
}

}  // namespace grape
