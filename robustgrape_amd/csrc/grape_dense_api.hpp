// grape_dense_api.hpp -- what the C ABI (grape_engine.hip) sees of the dense
// engine (grape_dense.hip): the problem / batch descriptors and the launchers.
#pragma once
#include <hip/hip_runtime.h>

#include "grape_launch.hpp"

namespace grape_dense {

// Scalars and term tables are shared with the small-d engine (DevProblem:
// ops/opsT/vs unused here); the operator basis is stored as padded 64 x 64
// register-file images (grape_dense.hpp).
struct DenseProblem {
    grape::DevProblem P;  // with error sources: P.nv variants per step, P.vs / off_* as the small engine
    const double *opimg;  // [n_ops][IMG]
    const double *W;      // [64] projector diagonal, zero-padded
    int Lc, Nc;           // chunk length / count of the prefix-product scan
    int nz;               // error path: local-frame slots per step, np (Z1) + ne (W) + ne np (Z2)
    int nva;              // x_add gradient variants per step: na when H0 / Herror read x_add, else 0
};

struct DenseBatch {
    int nb;
    const double *x;  // [nb][nx]
    double *E;        // [nb][Nt][IMG]   nominal propagators
    double *Q;        // [nb][Nt][IMG]   chunk-local prefix products
    double *Carry;    // [nb][Nc][IMG]   C_{cL-1} (identity for c = 0)
    double *M;        // [nb][IMG]       gradient kernel M = G U
    double *Mc;       // [nb][Nc][IMG]   Carry_c M Carry_c^dagger
    double *Z;        // [nb][Nt][IMG]   k_dgrad's Z_k, parked in HBM across the eps-variant exps
    double *F;        // [nb]
    double *Fdx;      // [nb][nx]
    double *Fadd;     // [nb][Nt][nva]   H0 reads x_add: step k's term of F_dx_add[q] (k_dgrad; k_dadd sums)
    int *status;      // bit 0: singular Pade denominator
    int *mstats;      // optional [5]: Pade degree histogram (m = 3, 5, 7, 9, 13)
    // error path (P.ne > 0; the algebra of grape_errpath.hpp on 64 x 64 images):
    double *Ub;       // [nb][IMG]           U = C_Nt
    double *Zl;       // [nb][Nt][nz][IMG]   Z1_u^T | W_e | Z2_{e,u}^T (local frame of step k)
    double *Vc;       // [nb][ne][Nc][IMG]   Carry_c^dag (sum_chunk W) Carry_c
    double *Sx;       // [nb][ne][Nc][IMG]   exclusive prefix of Vc over chunks
    double *Tot;      // [nb][ne][IMG]       sum_k V^err_k
    double *Me;       // [nb][ne][IMG]       M_e = G_e U
    double *Mp;       // [nb][ne][Nc][IMG]   M'_{c,e} = Carry M_e Carry^dag
    double *B0;       // [nb][ne][Nc][IMG]   B at the chunk start: [T_c, M'] + M' Ttot
    double *Fd2;      // [nb][ne]
    double *Fd2dx;    // [nb][ne][nx]
    double *Fd2add;   // [nb][ne][Nt][nva]  H0 / Herror read x_add: step k's term of F_d2err_dx_add[q] (k_derr_grad;
                      //                    k_dadd_err sums them onto the target's part)
    grape::cd *gp_scr;  // general projector: head scratch (grape_projector_api.hpp)
};

constexpr int kImgDoubles = 2 * 64 * 64;

// Pipeline of one batch (k_dexp, k_dscan, k_dcarry, k_dmc, k_dgrad) on `st`.
hipError_t launch_pipeline(const DenseProblem &P, const DenseBatch &B, hipStream_t st,
                           const grape_host::KMark &mark);
// n exponentials of padded images (grape_expm_batch for 12 < d <= 64).
hipError_t launch_expm_raw(const double *A, double *E, int n, int *status, int *mstats, hipStream_t st);
hipError_t set_lds_limits();
// Every variant P.vs[0..P.nv) of every step of ONE evaluation (B.nb = 1): k_dexp into the
// images B.E, then converted to row-major d x d tiles rows[Nt][nv][D][D] (the table the
// materialised-derivative kernels of grape_unitary.hip read).
hipError_t launch_variant_table(const DenseProblem &P, const DenseBatch &B, grape::cd *rows, hipStream_t st);
// Time sharding: one evaluation (B.nb = 1) of a slice plan.  Forward: the slice's
// propagators, chunk prefixes and carries (kept in B) and its total U_slice into Ucols (column-major
// d x d).  Gradient: M' (column-major) replaces the plan's M = G U, then k_dmc / k_dgrad give the
// slice's F_dx entries (B.Fdx).  Uses B.Ub.
hipError_t launch_slice_forward(const DenseProblem &P, const DenseBatch &B, grape::cd *Ucols, hipStream_t st);
hipError_t launch_slice_gradient(const DenseProblem &P, const DenseBatch &B, const grape::cd *Mcols, hipStream_t st);
// Closure fallback above GRAPE_MAX_SMALL_DIM: n host-tabulated H (column-major d x d) -> exp(-i dt H)
// as row-major d x d tiles (`rows`), through the padded images Aimg / Eimg (n images each); the
// no-interchange solve needs a Hermitian H (checked on the host, robustgrape_amd/engine.py)
hipError_t launch_table_variants(const grape::cd *H, int D, int n, double dt, double *Aimg, double *Eimg,
                                 grape::cd *rows, int *status, hipStream_t st);

}  // namespace grape_dense
