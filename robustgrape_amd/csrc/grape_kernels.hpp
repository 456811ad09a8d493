// grape_kernels.hpp -- the hot-path kernels (small-d row-group engine).
//
//   k_expm       one row group per (eval b, step k, variant v): builds column i
//                of A = -i dt H(x_b,k perturbed by v) from the operator basis and
//                computes E = exp(A) in column form (Pade m <= 5 here; m > 5 items
//                are parked for k_expm_high).   UnitaryCalculations.jl:45,51,59-90
//                Without error sources only the nominal v = 0 is launched.
//   k_expm_high  Pade 7/9/13 (+ squarings) for parked items.
//   k_scan       one workgroup per eval: chunked prefix product of the nominal
//                propagators (local chains + Hillis-Steele over chunk totals),
//                fidelity F, the gradient kernel M = G U and the per-chunk
//                M'_c = Carry_c M Carry_c^dagger.   UnitaryCalculations.jl:46-47,99
//                                                   FidelityCalculations.jl:32-54
//   k_expm_grad  (no error sources) one row group per (b, k, eps-variant u): exp of
//                the variant and, in place, F_dx[u,k] = Re sum(Z_k o dE) with
//                Z_k = (C_{k-1} M C_k^dagger)^T.   FidelityCalculations.jl:56-76
//   k_grad_high  the same for its parked (Pade m > 5) items.
//   k_grad       (error-source pipeline) one row group per (b, k): Z_k and the
//                traces against every stored variant.
//   k_reduce_add sum over k of the x_add contributions (only when H0 depends on x_add).
//   (d <= 3: k_expm is replaced by the lane-matrix k_expm_lane and, for sector problems without
//   error sources, k_expm + k_scan Phase A by k_expm_chain_lane -- grape_lane.hpp)
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
    int scan_waves;      // waves per k_scan / k_err_scan workgroup (4 or 8)
    // variant layout (see grape_engine.hip: build_variants)
    int off_dx, off_dxa, off_dx2, off_err, err_stride;
    int nvg, nz;         // gradient parameters (np + x_add when xadd_dep); local-frame slots per step (error path)
    double dt, eps, eps2, inv_eps, inv_eps2sq, DD, Dtr;
    const cd *ops;       // [n_ops][D][D] row-major
    const cd *opsT;      // [n_ops][D][D] column-major (column builds for the exp kernels)
    const Term *h0;
    const Term *tgt;
    const Term *err;     // error-source terms
    const int *err_off;  // [ne+1]
    const VSpec *vs;     // [nv]
    const double *W;     // projector diagonal (weights)
    // general (non-diagonal or complex) projector P0: the diagonal-specialised results are
    // overwritten by the heads of grape_projector.hip (FidelityCalculations.jl:47-51)
    int gen_proj;
    const cd *PA;        // P0 P  (row-major), P = P0 with nonzeros set to 1
    const cd *PB;        // P     (row-major)
    const cd *P0g;       // P0    (row-major; expectation values)
    // Sectors (grape_engine.hip find_sectors): when every operator H0 uses is block-diagonal in
    // a common permutation, one evaluation is run as nsec independent D x D sector problems
    // (sub-evaluation b' = b * nsec + w reads x of b and the operators of sector w at
    // ops / opsT + w * sec_ops); k_scan stops after the chunk carries, the sector head
    // (grape_projector.hip) forms F and the blocks of M from the assembled U, and k_sec_mc the
    // per-chunk images M'_c.  sectors = 0: whole matrices (nsec = 1).
    int sectors;         // 1: this is the sector problem (k_scan stops after the carries)
    int nsec;
    size_t sec_ops;
    int walk;            // sector class served by the chunk walks (grape_walk.hpp: k_walk_fwd / k_walk_grad)
    int walk_store_e;    // ... k_walk_fwd stores the nominal propagators for k_walk_grad (B.Ew) instead of
                         //     k_walk_grad recomputing them
    int twin;            // ... two sectors with identical operator blocks (grape_walk.hpp TWIN): one
                         //     exponential per step serves both
    int opts;            // grape_desc.reserved[1]: GRAPE_OPT_* (fixed at plan creation)
    // Phase-covariant walk class (grape_walk.hpp GAUGE, round 5): every sector w of the class obeys
    // H_w(x) = D(a x) H_w(0) D(a x)^dag with D(t) = diag(e^{i t N_j}) for the one control x (np = 1,
    // H0 free of x_add and of the step index), so E_k = D_k E~ D_k^dag with E~ = exp(-i dt H_w(0))
    // and the eps-variant is E' = D'_k E~ D'_k^dag: one exponential per lane instead of one per step
    // and variant.  gauge_n: [nsec][D] the integer charges N_j >= 0 (engine: find_gauge).
    int gauge;
    double gauge_a;
    const int *gauge_n;
    // (round 6) every sector of the class has the ladder charges N_j = j (the Rydberg sectors in the
    // engine's level order: {11, S, rr} and {01, 0r}): the merged walks then take the pair phases and
    // difference weights from compile-time charge differences (grape_walk.hpp kLadder), same values
    int gauge_ladder;
    // (round 6) E~ of every sector of the class, [nsec][D][D] row-major, computed once at plan creation by
    // the walks' own exponential (grape_walk.hpp k_gauge_base_fill: the same bits as gauge_base_lds) for
    // the merged walks, which read it through scalar loads (SGPR operands) instead of LDS copies
    // With error sources (gauge_lab, round 6): the lab-frame error walks (grape_walk.hpp k_walk_wsum_lab /
    // k_walk_err_lab, no images) and gauge_Et = [nsec][1 + 2 ne][D][D]: E~, N_e = (E~_e1 - E~) / eps,
    // M_e = E~_e2 - E~ (k_gauge_err_base_fill)
    const cd *gauge_Et;
    int gauge_lab;
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
    cd *Wc;                 // walk path with error sources: [nb][ne][nchunks][D][D] chunk sums of W (k_walk_img_sum)
    cd *Zl;                 // [nb][Nt][nz][D][D]  local-frame differences (error path, k_err_local):
                            //   Z1_u (nvg) | W_e (ne) | Z2_{e,u} (ne x nvg), row-major
    double *Fd2;            // [nb][ne]
    double *Fd2dx;          // [nb][ne][nx]
    double *part_err_add;   // [nb][ne][Nt][na]  per-step x_add terms of F_d2err_dx (xadd_dep only)
    int *overflow;          // parked (Pade m > 5) item ids of k_expm
    int *overflow_count;
    int *ovf2;              // parked item ids of k_expm_grad
    int *ovf2_count;
    cd *ovf2_slots;         // [nb][Nt][nvg][D][D]  A of parked k_expm_grad items
    int *status;            // bit 0: singular Pade denominator
    cd *sink;               // [D][D] write-only target of inactive lanes' unconditional stores
    // closure fallback (grape_fidelity_grad_tables): host-evaluated closures, per evaluation
    const cd *Htab;         // [nb][Nt][nv][D][D] column-major H at every closure call site (else null)
    const cd *U0tab;        // [nb][1 + na][D][D] column-major target at x_add, x_add + eps e_q (else null)
    cd *gp_scr;             // general projector: head scratch (grape_projector_api.hpp)
    double *sec_part;       // sectors: [nb][Nt][nvg] per-sector F_dx terms (k_sec_reduce sums them), else null;
                            // chunk walks: [nsec][Nt][nvg][nb / nsec], the evaluation fastest (coalesced)
    const double *xT;       // chunk walks: the controls transposed, [nx][nb / nsec] (coalesced lane reads)
    const cd *Msec;         // sectors: [nb][D][D] the sector blocks of M = G U (the sector head)
    // sectors with error sources
    double *sec_part_err;   // [nb][ne][Nt][nvg] per-sector F_d2err_dx terms (k_sec_reduce_err sums them)
    cd *TotS;               // [nb][ne][D][D] the sector blocks of Tot = sum_k V^err_k (k_err_scan)
    const cd *MsecE;        // [nb][ne][D][D] the sector blocks of M_e = G_e U (the sector error head)
    int chains_done;        // k_scan: Phase A's chunk chains Q_k are already in Q (k_expm_chain_lane);
                            //   a chunk whose total holds a NaN (a parked step) is rechained from E
    // chunk walks (grape_walk.hpp): k_scan starts from the chunk totals in Tc when it is set
    cd *Tc;                 // [nb][nchunks][D][D] row-major chunk totals T_c (k_walk_fwd), else null
    cd *wscr;               // [nsec][nb / nsec][nchunks][2][D][D] per-lane scratch of the squaring path
    cd *Ew;                 // walk_store_e: [nsec/NS][L][NS][D*D + 1][lanes] shifted E~_k and its shift, lane-minor
};

// Trig of the last argument seen by one builder: the operator bases pair cos(arg) and sin(arg)
// terms of one control (rydberg.py _drive_terms), so one sincos serves both (ocml's sin, cos and
// sincos share one argument reduction and kernel: same values).
struct TrigCache {
    double arg = __builtin_nan("");
    double s = 0.0, c = 0.0;
    __device__ __forceinline__ void at(double a) {
        if (!(a == arg)) {  // NaN never matches: recomputed
            sincos(a, &s, &c);
            arg = a;
        }
    }
};

__device__ __forceinline__ cd term_coef(const Term &t, int nt1, const double *xk, const double *xadd,
                                        const Pert &pp, TrigCache &tc) {
    double v = 1.0;
    if (t.var == VAR_X) v = xk[t.index];
    else if (t.var == VAR_XADD) v = xadd[t.index];
    else if (t.var == VAR_TSTEP) v = (double)nt1;
    if (t.var == pp.var && t.index == pp.index) v = v + pp.delta;
    const double arg = t.a * v + t.b;  // built with -ffp-contract=off: no fusion, like Julia
    double fr = 1.0, fi = 0.0;
    if (t.func == FN_LINEAR) fr = arg;
    else if (t.func == FN_COS || t.func == FN_SIN || t.func == FN_CIS) {
        tc.at(arg);
        if (t.func == FN_COS) fr = tc.c;
        else if (t.func == FN_SIN) fr = tc.s;
        else {
            fr = tc.c;
            fi = tc.s;
        }
    }
    return cmul(cmake(t.sre, t.sim), cmake(fr, fi));
}

__device__ __forceinline__ cd term_coef(const Term &t, int nt1, const double *xk, const double *xadd,
                                        const Pert &pp) {  // one term on its own (same trig as the cached form)
    TrigCache tc;
    return term_coef(t, nt1, xk, xadd, pp, tc);
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

// Row i of the target U0(x_add [+ eps e_q]) of evaluation b: from the operator
// basis, or from the host-evaluated table in closure mode (slot 0: x_add, 1 + q: x_add + eps e_q)
template <int D>
__device__ __forceinline__ void target_row(const DevProblem &P, const DevBatch &B, int b, int slot, int i,
                                           const double *xb, const double *xadd, const Pert &pp, cd (&h)[D]) {
    if (B.U0tab) {
        const cd *U = B.U0tab + ((size_t)b * (1 + P.na) + slot) * D * D + i;
#pragma unroll
        for (int j = 0; j < D; ++j) h[j] = U[(size_t)j * D];
        return;
    }
    build_row<D>(P.ops, P.tgt, P.n_tgt, i, 1, xb, xadd, pp, h);
}

// ---------------------------------------------------------------------------
// k_expm: all propagator variants of the batch
// ---------------------------------------------------------------------------
// Rebuilds this lane's COLUMN of A = -i dt H for one (b, k, v) item.  The scalar
// coefficients (the trig of the controls) are evaluated once and cached in
// registers (up to kCachedTerms per operator set); the row is then a short
// sum of cached coefficient x operator-row products, cheap enough to redo
// instead of keeping A live through the Pade evaluation.
constexpr int kCachedTerms = 6;

// Low-norm regime (m in {3, 5}): the solve-free Taylor evaluation (grape_device.hpp,
// default) or, built with -DGRAPE_LOW_PADE=1, Julia's Pade 3 / 5 with the LU solve.
#if defined(GRAPE_LOW_PADE) && GRAPE_LOW_PADE
#define EXPM_LOW(m_, ring_) expm_low<D>(G, (m_), a, x, valid, singular, rebuild)
#define EXPM_GROUP_CD(D_) ::grape::Geo<D_>::GROUP_CD
#else
#define EXPM_LOW(m_, ring_) expm_taylor<D, (ring_)>(G, (m_), a, x, valid)
#define EXPM_GROUP_CD(D_) ::grape::Geo<D_>::LEAN_CD
#endif
#ifndef GRAPE_EXPM_GRAD_WAVES
#define GRAPE_EXPM_GRAD_WAVES 3
#endif

template <int D, bool ERR>
struct ItemBuilder {
    const DevProblem *P;
    const cd *opsT;  // this item's sector of the column-major basis
    const double *xk, *xadd;
    int i, nt1;
    VSpec vs;
    bool valid;
    cd c0[kCachedTerms], ce[kCachedTerms];  // coefficients pre-scaled by -i dt (and errval)
    int o0, ne_t;

    // -i dt c
    __device__ __forceinline__ cd gen(cd c) const { return cmake(P->dt * c.im, -(P->dt * c.re)); }

    __device__ __forceinline__ ItemBuilder(const DevProblem *P_, const double *xk_, const double *xadd_, int i_,
                                           int nt1_, const VSpec &vs_, bool valid_, int sector = 0)
        : P(P_), opsT(P_->opsT + (size_t)sector * P_->sec_ops), xk(xk_), xadd(xadd_), i(i_), nt1(nt1_), vs(vs_),
          valid(valid_), o0(0), ne_t(0) {
        TrigCache tc;
#pragma unroll
        for (int t = 0; t < kCachedTerms; ++t)
            c0[t] = (t < P->n_h0) ? gen(term_coef(P->h0[t], nt1, xk, xadd, vs.pert, tc)) : czero();
        if (ERR && vs.err >= 0) {
            o0 = P->err_off[vs.err];
            ne_t = P->err_off[vs.err + 1] - o0;
#pragma unroll
            for (int t = 0; t < kCachedTerms; ++t)
                ce[t] = (t < ne_t) ? gen(cscale(vs.errval, term_coef(P->err[o0 + t], nt1, xk, xadd, vs.pert, tc)))
                                   : czero();
        }
    }

    __device__ __forceinline__ void accumulate(const Term *terms, int n, const cd (&cache)[kCachedTerms], double sc,
                                               cd (&h)[D]) const {
#pragma unroll
        for (int t = 0; t < kCachedTerms; ++t) {
            if (t < n) {
                const cd *op = opsT + (size_t)terms[t].op * D * D + i * D;
#pragma unroll
                for (int j = 0; j < D; ++j) cmac(h[j], cache[t], op[j]);
            }
        }
        for (int t = kCachedTerms; t < n; ++t) {  // rare: more terms than cached
            const cd c = gen(cscale(sc, term_coef(terms[t], nt1, xk, xadd, vs.pert)));
            const cd *op = opsT + (size_t)terms[t].op * D * D + i * D;
#pragma unroll
            for (int j = 0; j < D; ++j) cmac(h[j], c, op[j]);
        }
    }

    // column i of A = -i dt (H0 [+ errval Herror]): sum of cached coefficient x operator-column
    // MACs (fused: rounding-level differences from Julia's -1im*dt*H, within T0)
    __device__ __forceinline__ void operator()(cd (&a)[D]) const {
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = czero();
        accumulate(P->h0, P->n_h0, c0, 1.0, a);
        if (ERR && vs.err >= 0) accumulate(P->err + o0, ne_t, ce, vs.errval, a);  // UnitaryCalculations.jl:67-68
        if (!valid) {
#pragma unroll
            for (int j = 0; j < D; ++j) a[j] = czero();
        }
    }
};

// Item index -> (outer, mid, inner) for inner extent n1 and mid extent n2: 32-bit unsigned
// divisions (a few instructions) whenever the launch's items fit in 32 bits -- a uniform branch --
// instead of the 64-bit division sequence.
__device__ __forceinline__ void split_item(long g, long nitems, int n1, int n2, int &outer, int &mid, int &inner) {
    if (nitems <= 0xffffffffL) {
        const unsigned u = (unsigned)g, t = u / (unsigned)n1;
        inner = (int)(u - t * (unsigned)n1);
        outer = (int)(t / (unsigned)n2);
        mid = (int)(t - (unsigned)outer * (unsigned)n2);
    } else {
        inner = (int)(g % n1);
        mid = (int)((g / n1) % n2);
        outer = (int)(g / ((long)n1 * n2));
    }
}

// Parks an item whose Pade degree is > 5: A (column i at slot + i*D) goes to
// its output slot, the id to the list.
template <int D>
__device__ __forceinline__ void park(Group<D> &G, cd *slot_row, const cd (&a)[D], long gid, int *list, int *count) {
#pragma unroll
    for (int j = 0; j < D; ++j) slot_row[j] = a[j];
    if (G.i == 0) list[atomicAdd(count, 1)] = (int)gid;
}

// ERR = false for problems without error sources (keeps the error-term
// builder, and its registers, out of the common kernel).
#ifndef GRAPE_EXPM_WAVES_D9
#define GRAPE_EXPM_WAVES_D9 3   // waves per SIMD requested for d <= 9 (register budget 512/w)
#endif
template <int D, bool ERR>
__global__ __launch_bounds__(64, (D <= 9 ? GRAPE_EXPM_WAVES_D9 : 2)) void k_expm(DevProblem P, DevBatch B) {
    constexpr int RING = ERR ? 2 : 3;  // LDS read ring of the products (mm_tile_ring)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group<D> G = make_group<D>(lds, threadIdx.x, EXPM_GROUP_CD(D));
    const long nitems = (long)B.nb * P.Nt * P.nv;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    int v, k, b;
    split_item(gidc, nitems, P.nv, P.Nt, b, k, v);
    const int ns = P.nsec > 1 ? P.nsec : 1, bx = b / ns;  // sectors: evaluation bx, sector b - bx * ns
    const double *xb = B.x + (size_t)bx * P.nx;
    const ItemBuilder<D, ERR> rebuild(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, G.i, k + 1, P.vs[v],
                                      valid, b - bx * ns);
    cd a[D], x[D];
    rebuild(a);
    int singular = 0, s = 0;
    const int m = expm_prologue_fast<D>(G, a, x, valid, s);
    cd *out = B.E + (size_t)gidc * D * D + G.i * D;
    if (m > 5) {  // group-uniform: A (columns) to the slot, exp'd by k_expm_high
        if (valid) park<D>(G, out, a, gid, B.overflow, B.overflow_count);
        return;
    }
    if (m == 3 || m == 5) EXPM_LOW(m, RING);
    if (valid) {  // E row-major: column i at stride D (coalesced across the group)
        cd *col = B.E + (size_t)gidc * D * D + G.i;
#pragma unroll
        for (int j = 0; j < D; ++j) col[j * D] = x[j];
        if (singular) atomicOr(B.status, 1);
    }
}

// Closure mode: column i of A = -i dt H for item gid from the host-evaluated table
// (element-wise (-i dt) * h, exactly the reference's -im*dt*H before exp).
template <int D>
struct TableBuilder {
    const cd *H;  // this item's H, column-major
    int i;
    double dt;
    bool valid;
    __device__ __forceinline__ void operator()(cd (&a)[D]) const {
        const cd *col = H + i * D;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const cd h = col[j];
            a[j] = valid ? cmake(dt * h.im, -(dt * h.re)) : czero();
        }
    }
};

// k_expm for closure mode: every variant of every step from the H table
template <int D>
__global__ __launch_bounds__(64, (D <= 9 ? GRAPE_EXPM_WAVES_D9 : 2)) void k_expm_table(DevProblem P, DevBatch B) {
    constexpr int RING = 3;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group<D> G = make_group<D>(lds, threadIdx.x, EXPM_GROUP_CD(D));
    const long nitems = (long)B.nb * P.Nt * P.nv;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    TableBuilder<D> rebuild{B.Htab + (size_t)gidc * D * D, G.i, P.dt, valid};
    cd a[D], x[D];
    rebuild(a);
    int singular = 0, s = 0;
    const int m = expm_prologue_fast<D>(G, a, x, valid, s);
    cd *out = B.E + (size_t)gidc * D * D + G.i * D;
    if (m > 5) {
        if (valid) park<D>(G, out, a, gid, B.overflow, B.overflow_count);
        return;
    }
    if (m == 3 || m == 5) EXPM_LOW(m, RING);
    if (valid) {
        cd *col = B.E + (size_t)gidc * D * D + G.i;
#pragma unroll
        for (int j = 0; j < D; ++j) col[j * D] = x[j];
        if (singular) atomicOr(B.status, 1);
    }
}

// Items parked by k_expm / k_expm_raw (slots hold A column-major, overwritten
// with exp(A): row-major for the pipeline, column-major for grape_expm_batch).
template <int D>
__global__ __launch_bounds__(64) void k_expm_high(cd *slots, const int *list, const int *count, int *status,
                                                  int rows_out) {
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
        gsync();  // every lane has read its A column before any result lands in the slot
        if (valid) {
            cd *dst = rows_out ? slot - G.i * D + G.i : slot;  // row-major / column-major result
            const int stride = rows_out ? D : 1;
#pragma unroll
            for (int j = 0; j < D; ++j) dst[j * stride] = x[j];
            if (singular) atomicOr(status, 1);
        }
    }
}

// Standalone batched expm of column-major matrices (grape_expm_batch): lane i
// loads column i and stores column i of the result (column-major in and out).
template <int D>
__global__ __launch_bounds__(64) void k_expm_raw(const cd *A, cd *E, int n, int *overflow, int *overflow_count,
                                                 int *status, int *mstats) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const int gid = blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < n;
    const cd *src = A + (size_t)(valid ? gid : 0) * D * D + G.i * D;
    auto reload = [&](cd (&a)[D]) {
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = valid ? src[j] : czero();
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

// ---------------------------------------------------------------------------
// k_scan: one workgroup (W waves) per evaluation
//
// Column form: lane j of a group holds column j of its chunk's running
// product, so that every global access is coalesced (lane j touches the
// pieces m*D + j of a row-major tile: D lanes cover 16*D contiguous bytes per
// instruction) -- the local chain is a dependent load -> product -> store
// sequence, and its per-step latency is what bounds this kernel.  Chunk
// totals live in the groups' LDS tiles COLUMN-major (tile[j*D + i] = S[i][j]).
// ---------------------------------------------------------------------------
template <int D, int W>
__device__ __forceinline__ void scan_body(const DevProblem &P, const DevBatch &B, const int b) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int GPW = Geo<D>::GPW, GCD = Geo<D>::GROUP_CD, TILE = Geo<D>::TILE;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    Group<D> G = make_group<D>(lds + wave * GPW * GCD, lane);
    cd *S1 = lds + W * GPW * GCD, *S2 = S1 + TILE, *S3 = S2 + TILE;
    const int c = wave * GPW + G.g;  // chunk owned by this group
    const int i = G.i;
    const bool gvalid = G.lane_ok && c < P.nchunks;
    auto tile_of = [&](int cc) -> cd * {
        return lds + (cc / GPW) * GPW * GCD + (cc % GPW) * GCD;
    };
    const cd *Eb = B.E + (size_t)b * P.Nt * P.nv * TILE;
    cd *Qb = B.Q + (size_t)b * P.Nt * TILE;

    // Phase A: local inclusive chain Q_k = E_k ... E_{cL}; lane i owns column i
    cd q[D], e[D], t[D];
    const int k0 = c * P.L;
    // Column i of E_k (coalesced).  The load is unconditional (k clamped into range):
    // a guarded load compiles to exec-masked branches around the loads, after which
    // the compiler can no longer count outstanding vector-memory ops and waits with
    // vmcnt(0) -- i.e. for the prefetch just issued and the previous step's Q stores.
    // Out-of-range steps only feed products whose results are discarded (act below).
    auto load_e = [&](int k, cd (&dst)[D]) {
        const int kk = k < P.Nt ? k : P.Nt - 1;
        const cd *src = Eb + ((size_t)kk * P.nv) * TILE + i;
#pragma unroll
        for (int m = 0; m < D; ++m) dst[m] = src[m * D];
    };
    bool redo = true;
    if (B.Tc) {  // chunk walks: the totals are given (column i of T_c, row-major storage)
        const cd *src = B.Tc + ((size_t)b * P.nchunks + (gvalid ? c : 0)) * TILE + i;
#pragma unroll
        for (int m = 0; m < D; ++m) q[m] = src[m * D];
        redo = false;
    } else if (B.chains_done) {  // the chunk total is the chain's last stored step
        const int kend = min(k0 + P.L, P.Nt) - 1;
        const cd *src = Qb + (size_t)(gvalid ? kend : 0) * TILE + i;
        bool bad = false;
#pragma unroll
        for (int m = 0; m < D; ++m) {
            q[m] = src[m * D];
            bad = bad || q[m].re != q[m].re || q[m].im != q[m].im;
        }
        redo = group_any(G, gvalid && bad);  // group-uniform
    }
    if (redo) load_e(k0, e);
    for (int j = 0; redo && j < P.L; ++j) {
        const int k = k0 + j;
        const bool act = gvalid && k < P.Nt;
        cd en[D];
        load_e(k + 1, en);  // prefetch the next step's propagator column behind this product
        if (j == 0) {
#pragma unroll
            for (int m = 0; m < D; ++m) q[m] = e[m];
        } else {
            tile_store_row(G, e, gvalid);  // E_k column-major in the tile (lanes outside a group must not write)
            wsync();  // the chains are independent: no workgroup barrier inside Phase A (k_scan 19.0 -> 18.7 ms)
            mm_tile_pf<D>(q, G.tile, t);  // E_k . q
            wsync();
            if (act) {  // past N_t (last chunk's tail) the total stays put
#pragma unroll
                for (int m = 0; m < D; ++m) q[m] = t[m];
            }
        }
        {  // Q row-major: column i at stride D (coalesced).  Unconditional store (inactive
           // lanes write the sink tile): a store under a branch makes the loop's vmcnt
           // accounting path-dependent and the compiler then waits for everything
           // (vmcnt(0)) -- the stores included -- before the next step's prefetch is used.
            cd *dst = act ? Qb + (size_t)k * TILE + i : B.sink + i;
#pragma unroll
            for (int m = 0; m < D; ++m) dst[m * D] = q[m];
        }
#pragma unroll
        for (int m = 0; m < D; ++m) e[m] = en[m];
    }
    tile_store_row(G, q, gvalid);  // chunk total T_c, column-major
    gsync();
    // Phase B: inclusive scan of the chunk totals, P_c = T_c ... T_0 (Hillis-Steele):
    // column i of S_c . S_{c-o} = S_c . (column i of S_{c-o})
    for (int o = 1; o < P.nchunks; o <<= 1) {
        const bool doit = gvalid && c >= o;
        if (doit) {
            const cd *src = tile_of(c - o) + i * D;
#pragma unroll
            for (int m = 0; m < D; ++m) q[m] = src[m];
            mm_tile_pf<D>(q, G.tile, t);
        }
        gsync();
        if (doit) tile_store_row(G, t, true);
        gsync();
    }
    if (P.sectors) {  // sectors: U and the carries only; the sector head and k_sec_mc do F, M, M'_c
        if (c == P.nchunks - 1 && G.lane_ok) {
            const cd *Ut = tile_of(c);
            cd *du = B.Ub + (size_t)b * TILE + i * D;
#pragma unroll
            for (int jj = 0; jj < D; ++jj) du[jj] = Ut[jj * D + i];
        }
        if (gvalid) {
            cd *dc = B.Carry + ((size_t)b * P.nchunks + c) * TILE + i * D;
            const cd *Cr = c > 0 ? tile_of(c - 1) : nullptr;
#pragma unroll
            for (int jj = 0; jj < D; ++jj) dc[jj] = Cr ? Cr[jj * D + i] : cmake(jj == i ? 1.0 : 0.0, 0.0);
        }
        return;
    }
    // Phase C: fidelity and M = G U on group 0 (everyone keeps the barrier sequence)
    const bool f0 = (c == 0) && G.lane_ok;
    const cd *Ut = tile_of(P.nchunks - 1);  // U column-major
    const double *xb = B.x + (size_t)b * P.nx;
    const double *xadd = xb + (size_t)P.np * P.Nt;
    Pert none;
    none.var = -1; none.index = 0; none.delta = 0.0;
    cd l[D], kk[D];
    target_row<D>(P, B, b, 0, i, xb, xadd, none, l);  // U0 row i
    if (f0) {
#pragma unroll
        for (int jj = 0; jj < D; ++jj) S1[i * D + jj] = l[jj];
    }
    gsync();
#pragma unroll
    for (int r = 0; r < D; ++r) l[r] = cconj(S1[r * D + i]);
    mm_tile_pf<D, true>(l, Ut, kk);  // K = U0^dag U, row i
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
    mm_tile_pf<D>(l, S2, t);
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
        target_row<D>(P, B, b, 1 + qd, i, xb, xadd, pq, l);
        target_row<D>(P, B, b, 0, i, xb, xadd, none, t);
        if (f0) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) S1[i * D + jj] = cscale(P.inv_eps, csub(l[jj], t[jj]));
        }
        gsync();
#pragma unroll
        for (int r = 0; r < D; ++r) l[r] = cconj(S1[r * D + i]);
        mm_tile_pf<D, true>(l, Ut, t);  // Kd = U0d^dag U
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
        for (int jj = 0; jj < D; ++jj) du[jj] = Ut[jj * D + i];
    }
    // Phase D: M'_c = Carry_c M Carry_c^dag, Carry_c = P_{c-1} (identity for c = 0)
    if (gvalid && B.Carry) {  // carries for the error path (identity for chunk 0)
        cd *dc = B.Carry + ((size_t)b * P.nchunks + c) * TILE + i * D;
        const cd *Cr = c > 0 ? tile_of(c - 1) : nullptr;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) dc[jj] = Cr ? Cr[jj * D + i] : cmake(jj == i ? 1.0 : 0.0, 0.0);
    }
    if (gvalid) {
        cd mc[D];
        if (c == 0) {
#pragma unroll
            for (int jj = 0; jj < D; ++jj) mc[jj] = S3[i * D + jj];
        } else {
            const cd *Cr = tile_of(c - 1);  // column-major
#pragma unroll
            for (int jj = 0; jj < D; ++jj) q[jj] = Cr[jj * D + i];
            mm_tile_pf<D>(q, S3, t);
            mm_tile_pf<D, false, true>(t, Cr, mc);
        }
        cd *dst = B.Mc + ((size_t)b * P.nchunks + c) * TILE + i * D;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) dst[jj] = mc[jj];
    }
}
template <int D, int W>
__global__ __launch_bounds__(64 * W) void k_scan(DevProblem P, DevBatch B) {
    scan_body<D, W>(P, B, blockIdx.x);
}
// Two sector classes' scans in one launch (latency-bound calls): workgroups [0, B0.nb) scan class 0,
// the rest class 1 (dynamic LDS: the larger of the two)
template <int D0, int D1, int W>
__global__ __launch_bounds__(64 * W) void k_scan_pair(DevProblem P0, DevBatch B0, DevProblem P1, DevBatch B1) {
    if ((int)blockIdx.x < B0.nb) scan_body<D0, W>(P0, B0, blockIdx.x);
    else scan_body<D1, W>(P1, B1, blockIdx.x - B0.nb);
}

// ---------------------------------------------------------------------------
// Gradient contraction.  Row i of Z_k = Y_k^T with Y_k = C_{k-1} M C_k^dag
// = Q_{k-1} M'_c Q_k^dag:  Z_k = conj(Q_k) M'^T Q_{k-1}^T  (Q_{k-1} = I at a
// chunk start), so that F_dx[p,k] = Re tr(Y_k dE) = Re sum_ij Z_ij dE_ij.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ void grad_kernel_row(Group<D> &G, const DevProblem &P, const DevBatch &B, int b, int k,
                                                bool valid, cd (&z)[D]) {
    constexpr int TILE = Geo<D>::TILE;
    const int c = k / P.L, j0 = k - c * P.L;
    const int i = G.i;
    const cd *Qk = B.Q + ((size_t)b * P.Nt + k) * TILE;
    const cd *Mc = B.Mc + ((size_t)b * P.nchunks + c) * TILE;
    cd ql[D], t[D];
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
}

// Column j of Z_k for lane j (the fused kernels keep E' in columns):
//   column j of Z = conj(Q_k) M'^T (row j of Q_{k-1})^T,
// with M' and Q_k staged through the group tile by coalesced cooperative loads.
template <int D>
__device__ __forceinline__ void tile_load(Group<D> &G, const cd *src, bool valid) {  // row-major copy
    if (valid) {
#pragma unroll
        for (int m = 0; m < D; ++m) G.tile[m * D + G.i] = src[m * D + G.i];
    }
}
template <int D, int RING = 0>
__device__ __forceinline__ void grad_kernel_col(Group<D> &G, const DevProblem &P, const DevBatch &B, int b, int k,
                                                bool valid, cd (&z)[D], cd (&e0)[D]) {
    constexpr int TILE = Geo<D>::TILE;
    const int c = k / P.L, j0 = k - c * P.L;
    const int i = G.i;
    const cd *Qk = B.Q + ((size_t)b * P.Nt + k) * TILE;
    const cd *Mc = B.Mc + ((size_t)b * P.nchunks + c) * TILE;
    cd r[D], t[D];
    if (j0 > 0) {
#pragma unroll
        for (int m = 0; m < D; ++m) r[m] = Qk[i * D + m - TILE];  // row i of Q_{k-1}
    }
    tile_load<D>(G, Mc, valid);
    gsync();
    if (j0 > 0) {
        mm_tile_r<D, RING>(r, G.tile, t);  // M'^T r
    } else {
#pragma unroll
        for (int m = 0; m < D; ++m) t[m] = G.tile[i * D + m];  // row i of M'
    }
    gsync();
    tile_load<D>(G, Qk, valid);
    gsync();
    mm_tile_r<D, RING, true, true>(t, G.tile, z);  // conj(Q_k) t
    gsync();
    const cd *E0 = B.E + (((size_t)b * P.Nt + k) * P.nv) * TILE + i;
#pragma unroll
    for (int m = 0; m < D; ++m) e0[m] = E0[m * D];
}

// Group-summed Re sum_j z_j * (ev_j - e0_j) * inv_eps, written to F_dx (control
// variant u < np) or to the per-step x_add partial (u >= np).
template <int D>
__device__ __forceinline__ void grad_store(Group<D> &G, const DevProblem &P, const DevBatch &B, int b, int k, int u,
                                           const cd (&z)[D], const cd (&ev)[D], const cd (&e0)[D], bool valid) {
    double s = 0.0;
#pragma unroll
    for (int jj = 0; jj < D; ++jj) {
        const cd de = cscale(P.inv_eps, csub(ev[jj], e0[jj]));  // (1/eps) * (E' - E)
        s += z[jj].re * de.re - z[jj].im * de.im;
    }
    s = group_sum(G, s, valid);
    if (valid && G.i == 0) {
        if (B.sec_part) B.sec_part[((size_t)b * P.Nt + k) * P.nvg + u] = s;  // sector term, summed by k_sec_reduce
        else if (u < P.np) B.Fdx[(size_t)b * P.nx + (size_t)k * P.np + u] = s;
        else B.part_add[((size_t)b * P.Nt + k) * P.na + (u - P.np)] = s;
    }
}

// k_grad: one row group per (b, k), variants read back from E (error-source pipeline)
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
    cd z[D];
    grad_kernel_row<D>(G, P, B, b, k, valid, z);
    const cd *E0 = B.E + (((size_t)b * P.Nt + k) * P.nv) * TILE + G.i * D;
    cd e0[D];
#pragma unroll
    for (int jj = 0; jj < D; ++jj) e0[jj] = E0[jj];
    const int nvg = P.np + (P.xadd_dep ? P.na : 0);  // dx then dxa variants are contiguous
    for (int u = 0; u < nvg; ++u) {
        const cd *Ev = E0 + (size_t)(P.off_dx + u) * TILE;
        cd ev[D];
#pragma unroll
        for (int jj = 0; jj < D; ++jj) ev[jj] = Ev[jj];
        grad_store<D>(G, P, B, b, k, u, z, ev, e0, valid);
    }
}

// k_expm_grad (no error sources): one row group per (b, k, eps-variant u):
// the variant's propagator E' = exp(-i dt H(x + eps e_u)) is computed and
// contracted on the spot -- it never goes to memory.  Pade m > 5 items are
// parked (A to a slot) for k_grad_high.
template <int D>
__global__ __launch_bounds__(64, (D <= 9 ? GRAPE_EXPM_GRAD_WAVES : 2)) void k_expm_grad(DevProblem P, DevBatch B) {
    constexpr int RING = 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int TILE = Geo<D>::TILE;
    Group<D> G = make_group<D>(lds, threadIdx.x, EXPM_GROUP_CD(D));
    const int nvg = P.np + (P.xadd_dep ? P.na : 0);
    const long nitems = (long)B.nb * P.Nt * nvg;
    const long gid = (long)blockIdx.x * Geo<D>::GPW + G.g;
    const bool valid = G.lane_ok && gid < nitems;
    const long gidc = valid ? gid : 0;
    int u, k, b;
    split_item(gidc, nitems, nvg, P.Nt, b, k, u);
    const int ns = P.nsec > 1 ? P.nsec : 1, bx = b / ns;
    const double *xb = B.x + (size_t)bx * P.nx;
    const ItemBuilder<D, false> rebuild(&P, xb + (size_t)k * P.np, xb + (size_t)P.np * P.Nt, G.i, k + 1,
                                        P.vs[P.off_dx + u], valid, b - bx * ns);
    cd a[D], x[D];
    rebuild(a);
    int singular = 0, s = 0;
    const int m = expm_prologue_fast<D>(G, a, x, valid, s);
    if (m == 3 || m == 5) EXPM_LOW(m, RING);
    if (m > 5) {
        if (valid) park<D>(G, B.ovf2_slots + (size_t)gidc * TILE + G.i * D, a, gid, B.ovf2, B.ovf2_count);
        return;  // group-uniform: the whole group parks
    }
    if (valid && singular) atomicOr(B.status, 1);
    cd z[D], e0[D];
    grad_kernel_col<D, RING>(G, P, B, b, k, valid, z, e0);  // e0: column i of E_k
    grad_store<D>(G, P, B, b, k, u, z, x, e0, valid);
}

// Parked k_expm_grad items: Pade m = 7/9/13, then the same contraction.
template <int D>
__global__ __launch_bounds__(64) void k_grad_high(DevProblem P, DevBatch B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cd *lds = reinterpret_cast<cd *>(smem_raw);
    constexpr int TILE = Geo<D>::TILE;
    Group<D> G = make_group<D>(lds, threadIdx.x);
    const int nvg = P.np + (P.xadd_dep ? P.na : 0);
    const int n = *B.ovf2_count;
    for (int base = blockIdx.x * Geo<D>::GPW; base < n; base += gridDim.x * Geo<D>::GPW) {
        const int idx = base + G.g;
        const bool valid = G.lane_ok && idx < n;
        const long gid = valid ? B.ovf2[idx] : 0;
        const int u = (int)(gid % nvg);
        const int k = (int)((gid / nvg) % P.Nt);
        const int b = (int)(gid / ((long)nvg * P.Nt));
        const cd *slot = B.ovf2_slots + (size_t)gid * TILE + G.i * D;
        cd a[D], x[D];
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = valid ? slot[j] : czero();
        int singular = 0, s = 0;
        const int m = expm_prologue<D>(G, a, x, valid, s);
        if (m > 0) expm_high<D>(G, m, s, a, x, valid, singular);
        gsync();
        if (valid && singular) atomicOr(B.status, 1);
        cd z[D], e0[D];
        grad_kernel_col<D>(G, P, B, b, k, valid, z, e0);
        grad_store<D>(G, P, B, b, k, u, z, x, e0, valid);
    }
}

// (xadd_dep only) F_dx_add = target part + sum_k per-step contributions
// (FidelityCalculations.jl:67-76 over U_dx_add = U sum_k V^dxa_k, UnitaryCalculations.jl:119-121);
// with error sources also F_d2err_dx_add[q, e] += sum_k per-step terms (k_err_grad) on top of
// the target part k_err_scan wrote (:99-113 over U_derr_dx_add, UnitaryCalculations.jl:140-151).
// Threads t < nb*na: F_dx_add; the next nb*ne*na: F_d2err_dx_add.
template <int D>
__global__ void k_reduce_add(DevProblem P, DevBatch B) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < B.nb * P.na) {
        const int b = t / P.na, q = t % P.na;
        double s = 0.0;
        for (int k = 0; k < P.Nt; ++k) s += B.part_add[((size_t)b * P.Nt + k) * P.na + q];
        B.Fdx[(size_t)b * P.nx + (size_t)P.np * P.Nt + q] = B.tgt_part[(size_t)b * P.na + q] + s;
        return;
    }
    t -= B.nb * P.na;
    if (P.ne == 0 || t >= B.nb * P.ne * P.na) return;
    const int q = t % P.na, be = t / P.na;  // be = b * ne + e
    const double *src = B.part_err_add + (size_t)be * P.Nt * P.na + q;
    double s = 0.0;
    for (int k = 0; k < P.Nt; ++k) s += src[(size_t)k * P.na];
    B.Fd2dx[(size_t)be * P.nx + (size_t)P.np * P.Nt + q] += s;
}

// Sectors: M'_{c,w} = Carry_{c,w} M_ww Carry_{c,w}^dagger, one thread per element (i, j) of one
// (sub-evaluation, chunk): sum_a C[i][a] sum_e M_ww[a][e] conj(C[j][e]); consecutive threads
// store consecutive elements.
template <int D>
__global__ void k_sec_mc(DevProblem P, DevBatch B) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B.nb * P.nchunks * D * D) return;
    const int j = (int)(t % D), i = (int)((t / D) % D);
    const long bc = t / (D * D);  // b' * nchunks + c
    const int b = (int)(bc / P.nchunks);
    const cd *C = B.Carry + (size_t)bc * D * D;
    const cd *Mw = B.Msec + (size_t)b * D * D;
    cd ci[D], cj[D];
#pragma unroll
    for (int e = 0; e < D; ++e) {
        ci[e] = C[i * D + e];
        cj[e] = cconj(C[j * D + e]);
    }
    cd acc = czero();
#pragma unroll
    for (int a = 0; a < D; ++a) {
        cd r = czero();  // (M_ww Carry^dagger)[a][j]
#pragma unroll
        for (int e = 0; e < D; ++e) r = cadd(r, cmul(Mw[a * D + e], cj[e]));
        acc = cadd(acc, cmul(ci[a], r));
    }
    B.Mc[(size_t)t] = acc;
}

// Sectors with error sources: M'_{c,e} = Carry_c M_e,ww Carry_c^dagger into slot 0 of the error
// path's per-chunk triple (k_err_scan wrote T_c and Ttot_c), one thread per element.
template <int D>
__global__ void k_sec_mc_err(DevProblem P, DevBatch B) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B.nb * P.ne * P.nchunks * D * D) return;
    const int j = (int)(t % D), i = (int)((t / D) % D);
    const long bec = t / (D * D);  // (b' * ne + e) * nchunks + c
    const int c = (int)(bec % P.nchunks);
    const long be = bec / P.nchunks;
    const int b = (int)(be / P.ne);
    const cd *C = B.Carry + ((size_t)b * P.nchunks + c) * D * D;
    const cd *Mw = B.MsecE + (size_t)be * D * D;
    cd ci[D], cj[D];
#pragma unroll
    for (int e = 0; e < D; ++e) {
        ci[e] = C[i * D + e];
        cj[e] = cconj(C[j * D + e]);
    }
    cd acc = czero();
#pragma unroll
    for (int a = 0; a < D; ++a) {
        cd r = czero();
#pragma unroll
        for (int e = 0; e < D; ++e) r = cadd(r, cmul(Mw[a * D + e], cj[e]));
        acc = cadd(acc, cmul(ci[a], r));
    }
    B.Me[(size_t)bec * 3 * D * D + i * D + j] = acc;
}

// Sectors: F_dx[b][k, u] (or the per-step x_add term) = sum over the evaluation's sectors of
// both classes, in sector order (deterministic).  A class's terms are laid out per evaluation
// ([nb][nsec][Nt][nvg]) or, from the chunk walks, evaluation-fastest ([nsec][Nt][nvg][nb]);
// one workgroup transposes a 32 x 32 tile of (evaluation, k * nvg + u) through LDS so that both
// the walk layout's reads and the F_dx rows' writes are coalesced.
struct SecParts {
    const double *part[2];      // per sector class, layout by lane_major
    const double *part_err[2];  // per sector class (error sources), layout by lane_major_err
    int nsec[2];                // 0 for an absent class
    int lane_major[2];          // 1: [nsec][Nt][nvg][nb] (chunk walks), else [nb][nsec][Nt][nvg]
    int lane_major_err[2];      // 1: [nsec][ne][Nt][nvg][nb] (k_walk_err_grad), else [nb][nsec][ne][Nt][nvg]
};
constexpr int kRedTile = 32;
template <int D>
__global__ __launch_bounds__(256) void k_sec_reduce(DevProblem P, double *Fdx, double *part_add, SecParts S, int nb) {
    __shared__ double tile[kRedTile][kRedTile + 1];
    const long per = (long)P.Nt * P.nvg;
    const int b0 = blockIdx.x * kRedTile;
    const long r0 = (long)blockIdx.y * kRedTile;
    const int tx = threadIdx.x % kRedTile, ty = threadIdx.x / kRedTile;
    for (int i = ty; i < kRedTile; i += 256 / kRedTile) {  // reads: the evaluation fastest
        const int b = b0 + tx;
        const long r = r0 + i;
        double s = 0.0;
        if (b < nb && r < per)
            for (int c = 0; c < 2; ++c)
                for (int w = 0; w < S.nsec[c]; ++w)
                    s += S.lane_major[c] ? S.part[c][((size_t)w * per + r) * nb + b]
                                         : S.part[c][((size_t)b * S.nsec[c] + w) * per + r];
        tile[i][tx] = s;
    }
    __syncthreads();
    for (int i = ty; i < kRedTile; i += 256 / kRedTile) {  // writes: k * nvg + u fastest
        const int b = b0 + i;
        const long r = r0 + tx;
        if (b >= nb || r >= per) continue;
        const int k = (int)(r / P.nvg), u = (int)(r - (long)k * P.nvg);
        const double s = tile[tx][i];
        if (u < P.np) Fdx[(size_t)b * P.nx + (size_t)k * P.np + u] = s;
        else part_add[((size_t)b * P.Nt + k) * P.na + (u - P.np)] = s;
    }
}

// The same for F_d2err_dx (or its per-step x_add term): rows q = e * Nt * nvg + (k * nvg + u) of every
// evaluation, through the same LDS transpose (reads evaluation-fastest, writes q-fastest).
template <int D>
__global__ __launch_bounds__(256) void k_sec_reduce_err(DevProblem P, double *Fd2dx, double *part_err_add, SecParts S,
                                                        int nb) {
    __shared__ double tile[kRedTile][kRedTile + 1];
    const long per = (long)P.Nt * P.nvg, rows = per * P.ne;
    const int b0 = blockIdx.x * kRedTile;
    const long q0 = (long)blockIdx.y * kRedTile;
    const int tx = threadIdx.x % kRedTile, ty = threadIdx.x / kRedTile;
    for (int i = ty; i < kRedTile; i += 256 / kRedTile) {
        const int b = b0 + tx;
        const long q = q0 + i;
        double s = 0.0;
        if (b < nb && q < rows) {
            const int e = (int)(q / per);
            const long r = q - (long)e * per;
            for (int c = 0; c < 2; ++c)
                for (int w = 0; w < S.nsec[c]; ++w)
                    s += S.lane_major_err[c] ? S.part_err[c][(((size_t)w * P.ne + e) * per + r) * nb + b]
                                             : S.part_err[c][(((size_t)b * S.nsec[c] + w) * P.ne + e) * per + r];
        }
        tile[i][tx] = s;
    }
    __syncthreads();
    for (int i = ty; i < kRedTile; i += 256 / kRedTile) {
        const int b = b0 + i;
        const long q = q0 + tx;
        if (b >= nb || q >= rows) continue;
        const int e = (int)(q / per);
        const long r = q - (long)e * per;
        const int k = (int)(r / P.nvg), u = (int)(r - (long)k * P.nvg);
        const size_t be = (size_t)b * P.ne + e;
        const double s = tile[tx][i];
        if (u < P.np) Fd2dx[be * P.nx + (size_t)k * P.np + u] = s;
        else part_err_add[(be * P.Nt + k) * P.na + (u - P.np)] = s;
    }
}

}  // namespace grape
