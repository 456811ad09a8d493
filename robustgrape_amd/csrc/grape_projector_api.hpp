// grape_projector_api.hpp -- general-projector heads (grape_projector.hip) as seen by the
// engines' launch sequences: what they read (U, carries, error totals) and what they
// overwrite (F, M / M'_c, F_d2err, M_e / M'_{c,e}, the target parts of the x_add gradients).
#pragma once
#include <hip/hip_runtime.h>

#include "grape_kernels.hpp"

namespace grape_proj {

constexpr int kScratchSlots = 16;             // d x d scratch matrices per workgroup
constexpr size_t kImg = 2 * 64 * 64;          // doubles per dense-engine image (grape_dense_api.hpp)

struct Heads {
    grape::DevProblem P;    // P.gen_proj, P.PA = P0 P, P.PB = P (row-major)
    int dense;              // 1: U / Tot / M / M_e are dense-engine images
    const double *x;        // [nb][nx]
    const grape::cd *U0tab; // closure fallback target table (else null)
    // small engine, row-major tiles
    const grape::cd *Ub;    // [nb][D][D]
    const grape::cd *Carry; // [nb][nchunks][D][D]
    grape::cd *Mc;          // [nb][nchunks][D][D]          (overwritten)
    grape::cd *Me;          // [nb][ne][nchunks][3][D][D]  M' slots overwritten; Ttot_0 = Tot read
    // dense engine images
    const double *Ub_img, *Tot_img;
    double *M_img, *Me_img;  // (overwritten)
    double *F, *Fdx, *tgt_part, *Fd2, *Fd2dx;
    grape::cd *scr;          // [nb * max(ne, 1)][kScratchSlots][D][D]
};

// one workgroup per evaluation: F, M (small engine: M'_c of every chunk), F_dx_add target part
hipError_t launch_fid_head(const Heads &H, int nb, hipStream_t st);
// one workgroup per (evaluation, error source): F_d2err, M_e (small engine: M'_{c,e}),
// F_d2err_dx_add target part
hipError_t launch_err_head(const Heads &H, int nb, hipStream_t st);

// Sectors (DevProblem::sectors): the fidelity head of a block-diagonal problem.  The sector
// pipeline leaves U_w of every sector (S x S, row-major); this head assembles U (d x d; the
// identity on levels no operator touches), forms F, M = G U and the target part of F_dx_add
// exactly as k_proj_fid does (with A = P0 P, B = P, any projector), and stores the sector
// blocks M_ww; k_sec_mc then forms the per-chunk images M'_{c,w} = Carry M_ww Carry^dagger
// that the sector k_expm_grad contracts.
struct SectorHead {
    grape::DevProblem P;      // the FULL d-dimensional problem (target terms, operators, PA / PB), d <= 12
    int ncls;                 // sector classes (1 or 2), each of nsec[c] sectors of S[c] slots
    int S[2], nsec[2];
    const int *sidx[2];       // [nsec][S]: level of each sector slot (-1: padding)
    const grape::cd *Ub[2];   // [nb * nsec][S][S]
    grape::cd *Msec[2];       // [nb * nsec][S][S]  (written)
    const int *fixed;         // levels no operator touches (identity in U, zero in Tot)
    int nfixed;
    const double *x;          // [nb][nx]
    double *F, *Fdx, *tgt_part;
    // error sources: the sector blocks of Tot (k_err_scan) in, F_d2err, the target part of
    // F_d2err_dx_add and the sector blocks of M_e out
    const grape::cd *TotS[2]; // [nb * nsec][ne][S][S]
    grape::cd *MsecE[2];      // [nb * nsec][ne][S][S]  (written)
    double *Fd2, *Fd2dx;
    int diag;                 // diagonal projector and target, sector classes of <= 4 levels: the
                              // fidelity head runs one thread per evaluation on the sector blocks
};
constexpr int kSectorLds = 2048;  // complex elements of LDS for the sector blocks M_ww (nsec * S * S)
hipError_t launch_sector_head(const SectorHead &H, int nb, hipStream_t st);
// one wave per (evaluation, error source): F_d2err, M_e blocks, F_d2err_dx_add target part
hipError_t launch_sector_err_head(const SectorHead &H, int nb, hipStream_t st);

// the small engine's view (grape_launch.hpp)
inline Heads small_heads(const grape::DevProblem &P, const grape::DevBatch &B) {
    Heads H{};
    H.P = P;
    H.dense = 0;
    H.x = B.x;
    H.U0tab = B.U0tab;
    H.Ub = B.Ub;
    H.Carry = B.Carry;
    H.Mc = B.Mc;
    H.Me = B.Me;
    H.F = B.F;
    H.Fdx = B.Fdx;
    H.tgt_part = B.tgt_part;
    H.Fd2 = B.Fd2;
    H.Fd2dx = B.Fd2dx;
    H.scr = B.gp_scr;
    return H;
}

}  // namespace grape_proj
