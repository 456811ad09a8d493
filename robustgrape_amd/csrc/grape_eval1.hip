// grape_eval1.hip -- latency-bound calls: ONE WORKGROUP PER EVALUATION (round 5).
//
// A single C2 evaluation through the pair path is five dependent launches (walk fwd, scan, sector
// head, walk grad, reduce) plus two staging copies: 52 us of kernel time for ~0.8 MFLOP, most of
// it launch ramps and global round trips (profiles/r05/single).  For the Rydberg sector layout
// with phase-covariant classes (grape_walk.hpp GAUGE) the whole evaluation fits one CU, so one
// workgroup runs it end to end, every intermediate in LDS:
//
//   x          the evaluation's controls, HBM (or mapped host memory) -> LDS, once
//   phase A    lane c of class A (one 3- or 4-level sector) and lane c of class B (two 2-level
//              sectors) build E_k = D_k E~ D_k^dag for the L steps of chunk c and their product
//              T_c (UnitaryCalculations.jl:45-47, 99); the head wave forms the target's diagonal
//              u0 and its x_add forward differences meanwhile (FidelityCalculations.jl:34-40)
//   phase B    inclusive Hillis-Steele scan of the chunk totals in LDS: S_c = T_c ... T_0
//   phase C    the head wave: F and the sector blocks of M = G U from U = S_last
//              (FidelityCalculations.jl:47-76, the diagonal head of grape_projector.hip)
//   phase D    lane c: X = S_{c-1} M S_{c-1}^dag, then per step Y = X E_k^dag,
//              F_dx[k] = Re tr(Y (E'_k - E_k)) / eps with E' - E = E o f from the level phases,
//              X <- E_k Y (grape_walk.hpp walk_grad_body's GAUGE step)
//   phase E    F_dx[k] = class 0's part + class 1's part, coalesced stores
//
// Same quantities and the same per-step arithmetic as the chunk walks; the chain products are
// associated differently (a scan over 256 chunks instead of the pair path's walk + scan
// geometry), so results agree with the pair path to rounding, not bit for bit.
#include <bitset>
#include <mutex>

#include "grape_eval1_api.hpp"
#include "grape_walk.hpp"

namespace grape_eval1 {
using namespace grape;

// E~ of sectors [0, nsec) of one class into out [nsec][D][D] (row-major): gauge_base's lane code
template <int D>
__global__ __launch_bounds__(64) void k_gauge_tilde(DevProblem P, cd *out, cd *scr, int nsec) {
    const int w = threadIdx.x;
    if (w >= nsec) return;
    WalkX X0;
    X0.k0 = X0.k1 = X0.a0 = X0.a1 = 0.0;
    Pert none;
    none.var = -1;
    none.index = 0;
    none.delta = 0.0;
    SM<D> A[1];
    walk_build<D, 1>(P, as_constant(P.ops) + (size_t)w * P.sec_ops, X0, 1, none, A);
    double mu0 = 0.0;
    walk_expm<D, false, true, false>(A[0], scr + (size_t)w * 2 * D * D, mu0, true, [&](int i, const cd (&x)[D]) {
#pragma unroll
        for (int j = 0; j < D; ++j) out[((size_t)w * D + j) * D + i] = x[j];
    });
}

struct Lay {
    size_t SA, SB, Wt, MA, MB, u0, dq, xs, ph, pA, pB, out, cq, tab, Et, gn, sidx, W, fixed, terms, tdiag, tab_bytes,
        total;
};
__host__ __device__ inline Lay layout(int DA, int neB, int nch, int Nt, int nx, int D, int na, int nfixed, int ntgt) {
    Lay L{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 15) / 16 * 16;
        return at;
    };
    L.SA = take((size_t)nch * DA * DA * sizeof(cd));
    L.SB = take((size_t)neB * nch * 4 * sizeof(cd));
    L.Wt = take((size_t)(kLanes / 64) * (DA * DA + 2 * 4) * sizeof(cd));  // wave totals of the scan
    L.MA = take((size_t)DA * DA * sizeof(cd));
    L.MB = take(2 * 4 * sizeof(cd));
    L.u0 = take((size_t)D * sizeof(cd));
    L.dq = take((size_t)na * D * sizeof(cd));
    L.xs = take((size_t)nx * sizeof(double));
    L.ph = take((size_t)Nt * sizeof(cd));  // e^{i a x_k} of every step (phase 0b)
    L.pA = take((size_t)Nt * sizeof(double));
    L.pB = take((size_t)Nt * sizeof(double));
    L.out = take((size_t)(1 + na) * sizeof(double));  // F and the x_add entries of F_dx (stored in phase E)
    // the target terms' coefficients at x_add, x_add + eps e_q; then the head's K blocks and weights
    L.cq = take((size_t)(1 + na) * ntgt * sizeof(cd) + 27 * sizeof(cd) + 9 * sizeof(double));
    // the plan's tables, one contiguous region: a byte copy of the plan's table blob (tab_build)
    L.tab = o;
    L.Et = take((size_t)(DA * DA + neB * 4) * sizeof(cd));  // E~ of class A, then class B
    L.gn = take((size_t)(DA + 2 * 2) * sizeof(int));        // charges: class A's sector, B's two
    L.sidx = take((size_t)(DA + 2 * 2) * sizeof(int));      // sector slots: plan class 0, then 1
    L.W = take((size_t)D * sizeof(double));
    L.fixed = take((size_t)(nfixed > 0 ? nfixed : 1) * sizeof(int));
    L.terms = take((size_t)ntgt * sizeof(Term));       // the target's terms ...
    L.tdiag = take((size_t)ntgt * D * sizeof(cd));     // ... and the diagonals of their operators
    L.tab_bytes = o - L.tab;
    L.total = o;
    return L;
}

template <int D>
__device__ __forceinline__ void m_load(const cd *s, cd (&M)[D][D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int i = 0; i < D; ++i) M[j][i] = s[j * D + i];
    }
}
template <int D>
__device__ __forceinline__ void m_store(cd *s, const cd (&M)[D][D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int i = 0; i < D; ++i) s[j * D + i] = M[j][i];
    }
}
template <int D>
__device__ __forceinline__ void m_ident(cd (&M)[D][D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int i = 0; i < D; ++i) M[j][i] = cmake(i == j ? 1.0 : 0.0, 0.0);
    }
}
// R <- A R (column by column, the forward walk's chain order)
template <int D>
__device__ __forceinline__ void m_lmul(const cd (&A)[D][D], cd (&R)[D][D]) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
        cd q[D];
#pragma unroll
        for (int m = 0; m < D; ++m) q[m] = R[m][i];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            cd c = czero();
#pragma unroll
            for (int m = 0; m < D; ++m) cmac(c, q[m], A[j][m]);
            R[j][i] = c;
        }
    }
}
// R <- R B (row by row)
template <int D>
__device__ __forceinline__ void m_rmul(cd (&R)[D][D], const cd (&B)[D][D]) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        cd r[D];
#pragma unroll
        for (int m = 0; m < D; ++m) r[m] = R[j][m];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            cd c = czero();
#pragma unroll
            for (int m = 0; m < D; ++m) cmac(c, r[m], B[m][i]);
            R[j][i] = c;
        }
    }
}
// E_k = D_k E~ D_k^dag from p1 = e^{i a x_k} (gauge_prop's arithmetic)
template <int D>
__device__ __forceinline__ void step_prop(const cd (&Et)[D][D], const GaugeN<D> &gn, cd p1, cd (&E)[D][D]) {
    cd dph[kGaugePairs<D>];
    gauge_phases<D>(p1, gn, dph);
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int k = 0; k < D; ++k) E[j][k] = gauge_sandwich<D>(dph, j, k, Et[j][k]);
    }
}
template <int D>
__device__ __forceinline__ GaugeN<D> charges(const int *g) {
    GaugeN<D> r;
#pragma unroll
    for (int j = 0; j < D; ++j) r.n[j] = g[j];
    return r;
}

// phase A: the chunk total T_c of each of the lane's NE chains (E~ and the charges from LDS)
template <int D, int NE>
__device__ __forceinline__ void lane_total(const cd *EtL, const int *gnL, const cd *ph, int c, int L, int Nt,
                                           cd (&R)[NE][D][D]) {
    cd Et[NE][D][D];
    GaugeN<D> gn[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        m_load<D>(EtL + (size_t)e * D * D, Et[e]);
        gn[e] = charges<D>(gnL + e * D);
        m_ident<D>(R[e]);
    }
    const int k0 = c * L, k1 = min(k0 + L, Nt);
#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        const cd p1 = ph[k];  // e^{i a x_k} (phase 0b)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            cd E[D][D];
            step_prop<D>(Et[e], gn[e], p1, E);
            if (k == k0) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
#pragma unroll
                    for (int i = 0; i < D; ++i) R[e][j][i] = E[j][i];
                }
            } else {
                m_lmul<D>(E, R[e]);
            }
        }
    }
}

// phase B, inside a wave: inclusive scan over its 64 lanes, R_l <- R_l R_{l-o} (o = 1 .. 32)
template <int D, int NE>
__device__ __forceinline__ void wave_scan(cd (&R)[NE][D][D], int lane) {
#pragma unroll 1
    for (int o = 1; o < 64; o <<= 1) {
        cd Rm[NE][D][D];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
#pragma unroll
                for (int i = 0; i < D; ++i) {
                    Rm[e][j][i].re = __shfl_up(R[e][j][i].re, (unsigned)o, 64);
                    Rm[e][j][i].im = __shfl_up(R[e][j][i].im, (unsigned)o, 64);
                }
            }
        }
        if (lane >= o) {
#pragma unroll
            for (int e = 0; e < NE; ++e) m_rmul<D>(R[e], Rm[e]);
        }
    }
}
// ... then across the class's waves: R <- R (T_{w-1} ... T_0) with T_v wave v's total (LDS)
template <int D, int NE>
__device__ __forceinline__ void wave_carry(cd (&R)[NE][D][D], const cd *Wt, int w, int stride) {
    if (w == 0) return;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        cd C[D][D];
        m_load<D>(Wt + (size_t)(w - 1) * stride + e * D * D, C);
#pragma unroll 1
        for (int v = w - 2; v >= 0; --v) {
            cd T[D][D];
            m_load<D>(Wt + (size_t)v * stride + e * D * D, T);
            m_rmul<D>(C, T);
        }
        m_rmul<D>(R[e], C);
    }
}

// phase D: X = S_{c-1} M_w S_{c-1}^dag for every sector w of the lane (NSEC sectors over NE chains),
// then the chunk's steps (walk_grad_body's GAUGE step, presummed over the lane's sectors)
template <int D, int NE, int NSEC>
__device__ __forceinline__ void lane_grad(const DevProblem &Pc, const cd *EtL, const int *gnL, const cd *S, const cd *Mb,
                                          const double *xs, const cd *ph, int c, int L, int Nt, int nch, double *part) {
    constexpr int NSH = NSEC / NE;  // sectors per chain (twins: 2)
    cd Et[NE][D][D];
    GaugeN<D> gn[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        m_load<D>(EtL + (size_t)e * D * D, Et[e]);
        gn[e] = charges<D>(gnL + e * D);
    }
    cd X[NSEC][D][D];
#pragma unroll
    for (int w = 0; w < NSEC; ++w) {
        const int e = w / NSH;
        cd Cr[D][D], Mw[D][D];
        if (c > 0) m_load<D>(S + ((size_t)e * nch + c - 1) * D * D, Cr);
        else m_ident<D>(Cr);
        m_load<D>(Mb + (size_t)w * D * D, Mw);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            cd r[D];  // column j of M_w Carry^dag
#pragma unroll
            for (int a = 0; a < D; ++a) {
                cd v = czero();
#pragma unroll
                for (int q = 0; q < D; ++q) cmac(v, Mw[a][q], cconj(Cr[j][q]));
                r[a] = v;
            }
#pragma unroll
            for (int i = 0; i < D; ++i) {
                cd acc = czero();
#pragma unroll
                for (int a = 0; a < D; ++a) cmac(acc, Cr[i][a], r[a]);
                X[w][i][j] = acc;
            }
        }
    }
    const int k0 = c * L, k1 = min(k0 + L, Nt);
#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        const double xk = xs[k], xe = xk + Pc.eps;  // the reference's perturbed control
        const cd q = cis_m1(Pc.gauge_a * (xe - xk));
        const cd p1 = ph[k];
        cd E[NE][D][D], fwp[NE][kGaugePairs<D>];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            step_prop<D>(Et[e], gn[e], p1, E[e]);
#if GRAPE_GAUGE_FD_DN
            gauge_fd_weights_dn<D>(q, gn[e], fwp[e]);
#else
            cd rho[D];
#pragma unroll
            for (int j = 0; j < D; ++j) rho[j] = gauge_rho(q, gn[e].n[j]);
            gauge_fd_weights<D>(rho, fwp[e]);
#endif
        }
#pragma unroll
        for (int w = 0; w < NSEC; ++w) {  // Y = X E^dag, row by row
            const int e = w / NSH;
#pragma unroll
            for (int r = 0; r < D; ++r) {
                cd xr[D], y[D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[j] = X[w][r][j];
#pragma unroll
                for (int cc = 0; cc < D; ++cc) {
                    cd s = czero();
#pragma unroll
                    for (int j = 0; j < D; ++j) cmac(s, xr[j], cconj(E[e][cc][j]));
                    y[cc] = s;
                }
#pragma unroll
                for (int cc = 0; cc < D; ++cc) X[w][r][cc] = y[cc];
            }
        }
        double tot = 0.0, s[NSEC];
#pragma unroll
        for (int w = 0; w < NSEC; ++w) s[w] = 0.0;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const auto &fw = fwp[e];
#pragma unroll
            for (int r = 0; r < D; ++r) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    if (r == j) continue;
                    const cd de = cscale(Pc.inv_eps, cmul(E[e][r][j], gauge_fd_weight<D>(fw, r, j)));
#pragma unroll
                    for (int t = 0; t < NSH; ++t) {
                        const cd y = X[e * NSH + t][j][r];
                        s[e * NSH + t] = fma(y.re, de.re, s[e * NSH + t]);
                        s[e * NSH + t] = fma(-y.im, de.im, s[e * NSH + t]);
                    }
                }
            }
        }
#pragma unroll
        for (int w = 0; w < NSEC; ++w) tot += s[w];
        part[k] = NSEC > 1 ? tot : s[0];
        if (k + 1 == k1) break;  // (the last step's X <- E Y is not needed)
#pragma unroll
        for (int w = 0; w < NSEC; ++w) {  // X <- E Y, column by column
            const int e = w / NSH;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                cd y[D], t[D];
#pragma unroll
                for (int m = 0; m < D; ++m) y[m] = X[w][m][i];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    cd cc = czero();
#pragma unroll
                    for (int m = 0; m < D; ++m) cmac(cc, E[e][j][m], y[m]);
                    t[j] = cc;
                }
#pragma unroll
                for (int j = 0; j < D; ++j) X[w][j][i] = t[j];
            }
        }
    }
}

__device__ __forceinline__ double gadd(double v, int G) {
    for (int o = G >> 1; o >= 1; o >>= 1) v += __shfl_xor(v, o, G);
    return v;
}

template <int DA, bool TW>
__global__ __launch_bounds__(kBlock) void k_eval1(Args A) {
    constexpr int NEB = TW ? 1 : 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char e1_smem[];
    const DevProblem &P = A.H.P;
    const grape_proj::SectorHead &H = A.H;
    const Lay Lo = layout(DA, NEB, A.nch, P.Nt, P.nx, P.D, P.na, H.nfixed, P.n_tgt);
    cd *SA = reinterpret_cast<cd *>(e1_smem + Lo.SA), *SB = reinterpret_cast<cd *>(e1_smem + Lo.SB);
    cd *Wt = reinterpret_cast<cd *>(e1_smem + Lo.Wt);
    cd *MA = reinterpret_cast<cd *>(e1_smem + Lo.MA), *MB = reinterpret_cast<cd *>(e1_smem + Lo.MB);
    cd *u0 = reinterpret_cast<cd *>(e1_smem + Lo.u0), *dq = reinterpret_cast<cd *>(e1_smem + Lo.dq);
    double *xs = reinterpret_cast<double *>(e1_smem + Lo.xs);
    cd *ph = reinterpret_cast<cd *>(e1_smem + Lo.ph);
    double *pA = reinterpret_cast<double *>(e1_smem + Lo.pA), *pB = reinterpret_cast<double *>(e1_smem + Lo.pB);
    cd *EtL = reinterpret_cast<cd *>(e1_smem + Lo.Et);
    int *gnL = reinterpret_cast<int *>(e1_smem + Lo.gn), *sxL = reinterpret_cast<int *>(e1_smem + Lo.sidx);
    double *WL = reinterpret_cast<double *>(e1_smem + Lo.W);
    int *fxL = reinterpret_cast<int *>(e1_smem + Lo.fixed);
    double *outL = reinterpret_cast<double *>(e1_smem + Lo.out);
    Term *tmL = reinterpret_cast<Term *>(e1_smem + Lo.terms);
    cd *tdL = reinterpret_cast<cd *>(e1_smem + Lo.tdiag);
    cd *cqL = reinterpret_cast<cd *>(e1_smem + Lo.cq);
    const int t = threadIdx.x, b = blockIdx.x;
    // (trace: clocks along thread 0's path -- a class-A lane -- at the phase boundaries)
    const bool tr = A.trace && b == 0 && t == 0;
    long long tc[10];
    if (tr) {
        tc[0] = clock64();
        A.trace[14] = wall_clock64();
    }
    const int role = t / kLanes;  // 0: class A lanes, 1: class B lanes, 2: the head wave (wave-uniform)
    const int c = t - role * kLanes;
    // phase 0: the controls and the plan's table blob (one coalesced 16-B copy) into LDS
    const double *xb = A.x + (size_t)b * P.nx;
    for (int i = t; i < P.nx; i += kBlock) xs[i] = xb[i];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.tab);
        uint4 *dst = reinterpret_cast<uint4 *>(e1_smem + Lo.tab);
        for (int i = t; i < (int)(Lo.tab_bytes / 16); i += kBlock) dst[i] = src[i];
    }
    __syncthreads();
    // phase 0b: the level phases' base e^{i a x_k} of every step, once (both classes share a), in
    // parallel over the workgroup instead of twice per step on each class's critical path
    for (int k = t; k < P.Nt; k += kBlock) {
        ph[k] = gauge_cis(A.PA.gauge_a * xs[k]);
    }
    __syncthreads();
    if (tr) tc[1] = clock64();
    const bool act = role < 2 && c < A.nch;
    const bool wact = role < 2 && (c & ~63) < A.nch;  // the lane's wave holds a chunk (wave-uniform)
    const double *xadd = xs + (size_t)P.np * P.Nt;
    const int lane = c & 63, wv = c >> 6;
    // phases A and B (class lanes): chunk totals, then their inclusive scan -- inside each wave by
    // shuffles, then across the class's waves through LDS
    cd RA[1][DA][DA], RB[NEB][2][2];
    if (role == 0) {
        if (wact) {
            lane_total<DA, 1>(EtL, gnL, ph, c, A.L, P.Nt, RA);
            if (tr) tc[2] = clock64();
            wave_scan<DA, 1>(RA, lane);
            if (tr) tc[3] = clock64();
            if (lane == 63) m_store<DA>(Wt + (size_t)wv * (DA * DA + 8), RA[0]);
        }
    } else if (role == 1) {
        if (wact) {
            lane_total<2, NEB>(EtL + DA * DA, gnL + DA, ph, c, A.L, P.Nt, RB);
            wave_scan<2, NEB>(RB, lane);
            if (A.trace && b == 0 && c == 0) A.trace[22] = clock64();  // (class B's phase A + scan done)
            if (lane == 63) {
#pragma unroll
                for (int e = 0; e < NEB; ++e) m_store<2>(Wt + (size_t)wv * (DA * DA + 8) + DA * DA + e * 4, RB[e]);
            }
        }
    } else {  // the head wave: the target's diagonal at x_add and its x_add forward differences --
              // one lane per (term, variant) coefficient (the trig in parallel), then one per level
        const int ncq = (1 + P.na) * P.n_tgt;
        if (c < ncq) {
            const int v = c / P.n_tgt, q = c - v * P.n_tgt;
            Pert pp;
            pp.var = v == 0 ? -1 : (int)VAR_XADD;
            pp.index = v == 0 ? 0 : v - 1;
            pp.delta = v == 0 ? 0.0 : P.eps;
            cqL[c] = term_coef(tmL[q], 1, xs, xadd, pp);
        }
        // (LDS is in order within a wave: the fences keep the compiler from hoisting the reads)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (c < P.D) {
            const int i = c;
            auto entry = [&](int v) {  // target_entry's sum, in term order
                cd u = czero();
                for (int q = 0; q < P.n_tgt; ++q) u = cadd(u, cmul(cqL[v * P.n_tgt + q], tdL[(size_t)q * P.D + i]));
                return u;
            };
            const cd u = entry(0);
            u0[i] = u;
            for (int q = 0; q < P.na; ++q) dq[(size_t)q * P.D + i] = cscale(P.inv_eps, csub(entry(1 + q), u));
        }
        if (A.trace && b == 0 && c == 0) A.trace[21] = clock64();  // (the head wave's phase A done)
    }
    __syncthreads();
    if (tr) tc[4] = clock64();
    if (role == 0) {
        if (act) {
            wave_carry<DA, 1>(RA, Wt, wv, DA * DA + 8);
            m_store<DA>(SA + (size_t)c * DA * DA, RA[0]);
        }
    } else if (role == 1) {
        if (act) {
            wave_carry<2, NEB>(RB, Wt + DA * DA, wv, DA * DA + 8);
#pragma unroll
            for (int e = 0; e < NEB; ++e) m_store<2>(SB + ((size_t)e * A.nch + c) * 4, RB[e]);
        }
    }
    __syncthreads();
    if (tr) tc[5] = clock64();
    // phase C: the head wave, one lane per element (r, c) of each sector block (blocks padded to 3 x 3:
    // 27 lanes) -- K_rc = conj(u0_{g_r}) U_rc and its terms of F, tau and the F_dx_add sums, a
    // shuffle reduction over the wave, then M_rc from the K columns in LDS (diag_row's quantities,
    // FidelityCalculations.jl:47-76)
    if (role == 2) {
        const bool trh = A.trace && b == 0 && c == 0;  // (trace: the head wave's own steps, [16..20])
        long long th[5];
        if (trh) th[0] = clock64();
        const int S0 = H.S[0], S1 = H.S[1];
        const int n0 = S0 == 2 ? 2 : 1, nsec = n0 + (S1 == 2 ? 2 : 1);
        const int l = c / 9, e = c - 9 * l, r = e / 3, col = e - 3 * (e / 3);
        const int cl = l < n0 ? 0 : 1, w = l < n0 ? l : l - n0, S = cl == 0 ? S0 : S1;
        const bool isA = (cl == 0) == (A.a_first != 0);
        const bool valid = l < nsec && r < S && col < S;
        const int *sx = (cl == 0 ? sxL : sxL + S0 * H.nsec[0]) + w * S;
        // U = S_last of each class (the 2-level twins share one chain)
        const cd *Ub = isA ? SA + (size_t)(A.nch - 1) * DA * DA
                           : SB + ((size_t)(TW ? 0 : w) * A.nch + A.nch - 1) * 4;
        const int gr = valid ? sx[r] : -1, gc = valid ? sx[col] : -1;
        const bool live = gr >= 0 && gc >= 0;
        const cd U = live ? Ub[r * S + col] : czero();
        const cd u0r = u0[gr >= 0 ? gr : 0];
        const double wr = gr >= 0 ? WL[gr] : 0.0, pc = (gc >= 0 && WL[gc] != 0.0) ? 1.0 : 0.0;
        const cd K = live ? cmul(cconj(u0r), U) : czero();
        cd *kb = cqL + (size_t)(1 + P.na) * P.n_tgt;  // K of every block, [l][r][c] (LDS)
        double *wb = reinterpret_cast<double *>(kb + 27);  // W at each block's slots, [l][r]
        if (c < 27) kb[c] = K;
        if (c < 27 && col == 0) wb[l * 3 + r] = wr;
        double fsum = wr * pc * (K.re * K.re + K.im * K.im);
        cd tau = (r == col) ? cscale(wr, K) : czero();
        double sa[kMaxNa];
        cd trd[kMaxNa];
#pragma unroll
        for (int q = 0; q < kMaxNa; ++q) {
            sa[q] = 0.0;
            trd[q] = czero();
            if (q < P.na && gr >= 0) {
                const cd dr = cconj(dq[(size_t)q * P.D + gr]);
                const cd kd = cmul(dr, U);
                sa[q] = wr * pc * (kd.re * K.re + kd.im * K.im);
                if (r == col) trd[q] = cscale(wr, kd);
            }
        }
        if (trh) th[1] = clock64();
        fsum = gadd(fsum, 32);
        tau = cmake(gadd(tau.re, 32), gadd(tau.im, 32));
        for (int q = 0; q < H.nfixed; ++q) {  // U_gg = 1: K_gg = conj(u0_g)
            const int g = fxL[q];
            const cd k = cconj(u0[g]);
            fsum += WL[g] * (WL[g] != 0.0 ? 1.0 : 0.0) * (k.re * k.re + k.im * k.im);
            tau = cadd(tau, cscale(WL[g], k));
        }
        if (c == 0) outL[0] = (fsum + tau.re * tau.re + tau.im * tau.im) / P.DD;
        if (trh) th[2] = clock64();
        // (LDS is in order within a wave: the fences keep the compiler from hoisting the reads)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid) {  // M_rc = (2/DD) [p_r sum_k W_k conj(K_kr) K_kc + W_r conj(tau) K_rc]
            const cd *kl = kb + l * 9;
            cd sm = czero();
#pragma unroll
            for (int k = 0; k < 3; ++k) sm = cadd(sm, cscale(wb[l * 3 + k], cmul(cconj(kl[k * 3 + r]), kl[k * 3 + col])));
            const double pr = wr != 0.0 ? 1.0 : 0.0;
            const cd m = live ? cscale(2.0 / P.DD, cadd(cscale(pr, sm), cscale(wr, cmul(cconj(tau), K)))) : czero();
            (isA ? MA : MB + (size_t)w * 4)[r * S + col] = m;
        }
        if (trh) th[3] = clock64();
#pragma unroll
        for (int q = 0; q < kMaxNa; ++q) {
            if (q >= P.na) break;
            double s_ = gadd(sa[q], 32);
            cd t_ = cmake(gadd(trd[q].re, 32), gadd(trd[q].im, 32));
            const cd *d = dq + (size_t)q * P.D;
            for (int rr = 0; rr < H.nfixed; ++rr) {
                const int g = fxL[rr];
                const cd kd = cconj(d[g]), k = cconj(u0[g]);
                s_ += WL[g] * (WL[g] != 0.0 ? 1.0 : 0.0) * (kd.re * k.re + kd.im * k.im);
                t_ = cadd(t_, cscale(WL[g], kd));
            }
            if (c == 0) outL[1 + q] = (2.0 * s_ + 2.0 * (tau.re * t_.re + tau.im * t_.im)) / P.DD;
        }
        if (trh) {
            th[4] = clock64();
            for (int i = 0; i < 5; ++i) A.trace[16 + i] = th[i];
        }
    }
    __syncthreads();
    if (tr) tc[6] = clock64();
    // phase D
    if (role == 0) {
        if (act) lane_grad<DA, 1, 1>(A.PA, EtL, gnL, SA, MA, xs, ph, c, A.L, P.Nt, A.nch, pA);
        if (tr) tc[7] = clock64();
    } else if (role == 1) {
        if (act) lane_grad<2, NEB, 2>(A.PB, EtL + DA * DA, gnL + DA, SB, MB, xs, ph, c, A.L, P.Nt, A.nch, pB);
    }
    __syncthreads();
    if (tr) tc[8] = clock64();
    // phase E: F_dx = class 0's part + class 1's part (k_sec_reduce's order), F and the x_add entries
    // (every global -- possibly host-mapped -- store of the kernel is here: no barrier waits on one)
    double *dst = A.Fdx + (size_t)b * P.nx;
    for (int k = t; k < P.Nt; k += kBlock) {
        double v = 0.0;
        v += A.a_first ? pA[k] : pB[k];
        v += A.a_first ? pB[k] : pA[k];
        dst[k] = v;
    }
    if (t >= kBlock - 64 && t - (kBlock - 64) <= P.na) {
        const int q = t - (kBlock - 64);
        if (q == 0) A.F[b] = outL[0];
        else dst[(size_t)P.np * P.Nt + q - 1] = outL[q];
    }
    if (tr) {
        tc[9] = clock64();
        for (int i = 0; i < 10; ++i) A.trace[i] = tc[i];
        A.trace[15] = wall_clock64();
    }
}

// The plan's table blob (once per plan): k_eval1's LDS tables region, byte for byte -- E~ of both
// classes, their charges, the sector slots, W, the fixed levels, the target's terms and the
// diagonals of their operators -- gathered from wherever the plan keeps them.
template <int DA, bool TW>
__global__ __launch_bounds__(64) void k_tab_build(Args A, unsigned char *blob) {
    constexpr int NEB = TW ? 1 : 2;
    const DevProblem &P = A.H.P;
    const grape_proj::SectorHead &H = A.H;
    const Lay Lo = layout(DA, NEB, 1, P.Nt, P.nx, P.D, P.na, H.nfixed, P.n_tgt);
    auto at = [&](size_t off) { return blob + (off - Lo.tab); };
    cd *EtL = reinterpret_cast<cd *>(at(Lo.Et));
    int *gnL = reinterpret_cast<int *>(at(Lo.gn)), *sxL = reinterpret_cast<int *>(at(Lo.sidx));
    double *WL = reinterpret_cast<double *>(at(Lo.W));
    int *fxL = reinterpret_cast<int *>(at(Lo.fixed));
    Term *tmL = reinterpret_cast<Term *>(at(Lo.terms));
    cd *tdL = reinterpret_cast<cd *>(at(Lo.tdiag));
    const int c = threadIdx.x;
    const int nEA = DA * DA, nE = nEA + NEB * 4;
    for (int i = c; i < nE; i += 64) EtL[i] = i < nEA ? A.EtA[i] : A.EtB[i - nEA];
    for (int i = c; i < DA + 4; i += 64) gnL[i] = i < DA ? A.PA.gauge_n[i] : A.PB.gauge_n[i - DA];
    const int n0 = H.S[0] * H.nsec[0];
    for (int i = c; i < n0 + H.S[1] * H.nsec[1]; i += 64) sxL[i] = i < n0 ? H.sidx[0][i] : H.sidx[1][i - n0];
    for (int i = c; i < P.D; i += 64) WL[i] = P.W[i];
    for (int i = c; i < H.nfixed; i += 64) fxL[i] = H.fixed[i];
    for (int i = c; i < P.n_tgt; i += 64) tmL[i] = P.tgt[i];
    for (int i = c; i < P.n_tgt * P.D; i += 64) {
        const int q = i / P.D, j = i - q * P.D;
        tdL[i] = P.ops[((size_t)P.tgt[q].op * P.D + j) * P.D + j];
    }
}

size_t tab_bytes(const DevProblem &PA, const DevProblem &PB, const grape_proj::SectorHead &H) {
    const DevProblem &P = H.P;
    return layout(PA.D, PB.twin ? 1 : 2, 1, P.Nt, P.nx, P.D, P.na, H.nfixed, P.n_tgt).tab_bytes;
}
hipError_t tab_build(const Args &A, unsigned char *blob, hipStream_t st) {
    if (A.PA.D != 3) return hipErrorInvalidValue;
    if (A.PB.twin) hipLaunchKernelGGL((k_tab_build<3, true>), dim3(1), dim3(64), 0, st, A, blob);
    else hipLaunchKernelGGL((k_tab_build<3, false>), dim3(1), dim3(64), 0, st, A, blob);
    return hipGetLastError();
}

bool eligible(const DevProblem &PA, const DevProblem &PB, const grape_proj::SectorHead &H) {
    const DevProblem &P = H.P;
    const int neB = PB.twin ? 1 : 2;
    // (class A of 3 levels: the symmetry-adapted sectors.  The 4-level permutation sectors spill at
    // this workgroup's 168-VGPR budget and keep the pair kernels.)
    const bool shape = PA.D == 3 && PA.nsec == 1 && PB.D == 2 && PB.nsec == 2 && H.ncls == 2;
    const bool gauge = PA.gauge && PB.gauge && PA.walk && PB.walk && PA.gauge_a == PB.gauge_a;
    const bool path = P.ne == 0 && P.np == 1 && P.nvg == 1 && !P.xadd_dep && P.na <= kMaxNa && H.diag &&
                      P.Nt >= 1 && P.Nt <= kMaxNt && P.gen_proj == 0;
    if (!(shape && gauge && path)) return false;
    const int L = (P.Nt + kLanes - 1) / kLanes, nch = (P.Nt + L - 1) / L;
    return layout(PA.D, neB, nch, P.Nt, P.nx, P.D, P.na, H.nfixed, P.n_tgt).total <= 160 * 1024;
}

hipError_t prepare(const DevProblem &PA, const DevProblem &PB, cd *EtA, cd *EtB, cd *scr, hipStream_t st) {
    if (PA.D != 3) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_gauge_tilde<3>, dim3(1), dim3(64), 0, st, PA, EtA, scr, 1);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gauge_tilde<2>, dim3(1), dim3(64), 0, st, PB, EtB, scr, PB.twin ? 1 : 2);
    return hipGetLastError();
}

template <int DA, bool TW>
static hipError_t go(const Args &A, int nb, size_t lds, hipStream_t st) {
    // 160 KB of dynamic LDS: the attribute is per device, so it is raised once per (instantiation,
    // device) -- under a lock, as plans may be created and called from several threads
    static std::mutex mu;
    static std::bitset<256> raised;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (dev < 0 || dev >= (int)raised.size() || !raised.test((size_t)dev)) {
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_eval1<DA, TW>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            if (dev >= 0 && dev < (int)raised.size()) raised.set((size_t)dev);
        }
    }
    hipLaunchKernelGGL((k_eval1<DA, TW>), dim3((unsigned)nb), dim3(kBlock), lds, st, A);
    return hipGetLastError();
}

hipError_t launch(Args A, int nb, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    const DevProblem &P = A.H.P;
    A.L = (P.Nt + kLanes - 1) / kLanes;
    A.nch = (P.Nt + A.L - 1) / A.L;
    const bool tw = A.PB.twin != 0;
    const size_t lds = layout(A.PA.D, tw ? 1 : 2, A.nch, P.Nt, P.nx, P.D, P.na, A.H.nfixed, P.n_tgt).total;
    if (A.PA.D != 3) return hipErrorInvalidValue;
    return tw ? go<3, true>(A, nb, lds, st) : go<3, false>(A, nb, lds, st);
}

}  // namespace grape_eval1
