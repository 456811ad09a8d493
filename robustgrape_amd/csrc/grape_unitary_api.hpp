// grape_unitary_api.hpp -- what the C ABI sees of grape_unitary.hip (materialised
// unitary derivatives, grape_unitary_derivs).
#pragma once
#include <hip/hip_runtime.h>

#include "grape_kernels.hpp"

namespace grape_unitary {

using grape::cd;

constexpr int kMaxD = 12;      // GRAPE_MAX_SMALL_DIM: d x d tiles staged in LDS up to here
constexpr int kTiles = 4;      // tiles per workgroup
constexpr int kFidTiles = 14;  // the general-H0 fidelity head's tiles
constexpr int kResident = 256; // d > kMaxD: workgroups of the grid-stride launches, each with
                               // kTiles d x d tiles of global scratch (scratch_elems)
inline size_t scratch_elems(int D) { return D > kMaxD ? (size_t)kResident * kTiles * D * D : 0; }

// Propagator variants of one step, E[k][v] (built by the engine's k_expm):
//   0 nominal | 1 + q, q < np + na: x_q + eps (controls, then x_add)
//   ne > 0:  off_x2 + q: x_q + eps2 | per error e (stride 2 + np + na), from off_err:
//            err eps, err eps2, then x_q + eps2 with err eps2
// Slots of V (per step): dx_p (np) | dxa_q (na) | err_e (ne) | mix_{e,q} (ne x (np + na)).
struct UProblem {
    int D, Nt, np, na, ne, nv, nslots;
    int off_x2, off_err;
    double inv_eps, inv_eps2sq;
    cd *gscr;  // d > kMaxD: tile scratch (scratch_elems(D) complex), else unused
    __host__ __device__ int v_x2(int q) const { return off_x2 + q; }
    __host__ __device__ int v_err(int e) const { return off_err + e * (2 + np + na); }
    __host__ __device__ int v_err2(int e) const { return v_err(e) + 1; }
    __host__ __device__ int v_mix(int e, int q) const { return v_err(e) + 2 + q; }
};

struct UBuffers {
    const cd *E;  // [Nt][nv][D][D] row-major
    cd *C;        // [Nt][D][D]     C_k
    cd *Ci;       // [Nt][D][D]     C_k^-1 (general H0; null: C_k^dagger, Hermitian H0)
    int *status;  // bit 1: a singular C_k (general H0)
    cd *V;        // [Nt][nslots][D][D]
    cd *S;        // [Nt][ne][D][D] cumulative sums of V^err
    cd *Udx, *Uedx, *Udxa, *Ue, *Uedxa;  // outputs, reference column-major layouts
};

hipError_t launch_assembly(const UProblem &P, const UBuffers &B, hipStream_t st);
// Ci_k = C_k^-1 by Gauss-Jordan with partial pivoting (general H0, UnitaryCalculations.jl:47);
// status bit 1 on a singular C_k
hipError_t launch_inverse(const UProblem &P, const cd *C, cd *Ci, int *status, hipStream_t st);
// C_k = E_k C_{k-1} for the nominal table E[k][0] (P.nv variants per step)
hipError_t launch_chain(const UProblem &P, const cd *E, cd *C, hipStream_t st);
// O[:, :, k, e] = C_{k-1}^-1 (Herror_e(k, eps) / eps) C_{k-1}, column-major (d, d, Nt, ne)
// (UnitaryCalculations.jl:180-204; C^-1 = Ci when given, else C^dagger); x is the plan's device
// copy of the control vector
hipError_t launch_interaction(const grape::DevProblem &P, const double *x, const cd *C, const cd *Ci, cd *O,
                              cd *gscr, hipStream_t st);
// The same from host-evaluated closures (closure fallback): Oerr [Nt][ne][D][D] column-major
// holds (1/eps) Herror_e(k, x_k, x_add, eps) as the reference forms it
hipError_t launch_interaction_table(const grape::DevProblem &P, const cd *Oerr, const cd *C, const cd *Ci, cd *O,
                                    cd *gscr, hipStream_t st);
// General H0 (non-Hermitian, e.g. a -i Gamma/2 decay term): F, F_dx, F_d2err, F_d2err_dx of ONE
// evaluation from its materialised derivatives (launch_assembly's outputs, reference layouts),
// FidelityCalculations.jl:19-119.  P.PA / P.PB: the projector's P0 P and P (row-major; for a
// diagonal projector diag(w), diag(w != 0)).
struct FidArgs {
    grape::DevProblem P;
    const double *x;     // [nx] this evaluation's controls (operator-basis target terms)
    const cd *U0tab;     // [1 + na][D][D] column-major host target table (closures), else null
    const cd *U;         // [D][D] row-major C_Nt
    const cd *Udx, *Udxa, *Ue, *Uedx, *Uedxa;  // launch_assembly outputs
    cd *G;               // [1 + ne][D][D] scratch: the functionals of the controls and of each error
    cd *scr;             // d > kMaxD: kFidTiles D x D tiles of global scratch for the head (else unused)
    double *F, *Fdx, *Fd2, *Fd2dx;  // this evaluation's outputs ([1], [nx], [ne], [ne][nx])
};
hipError_t launch_fidelity(const FidArgs &A, hipStream_t st);
// ev[k + Nt e] = Re(dt tr(P0 sum_{j<=k} O_j,e) / D)   (FidelityCalculations.jl:368-390)
hipError_t launch_expectation(const grape::DevProblem &P, const cd *O, double *ev, hipStream_t st);

}  // namespace grape_unitary
