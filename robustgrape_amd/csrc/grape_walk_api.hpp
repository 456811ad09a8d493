// grape_walk_api.hpp -- host launchers of the chunk walks (grape_walk.hpp), compiled in their own
// translation unit (grape_walk_inst.hip, built without MachineLICM; see grape_walk.hpp).
#pragma once
#include <hip/hip_runtime.h>

namespace grape {
struct DevProblem;
struct DevBatch;
constexpr int kWalkMaxD = 4;  // sector classes of at most this many levels take the walks
constexpr int kWalkMaxNpA = 2;  // ... with at most this many controls per step and x_add entries
constexpr int kGaugeMaxE = 8;  // error sources of a phase-covariant image walk (grape_walk.hpp k_walk_img_gauge)
constexpr int kWalkBlockA = 128;  // lanes per workgroup (grape_walk.hpp kWalkBlock)
// walk classes of at least this many levels hand the forward walk's propagators to the gradient walk
// (B.Ew) instead of recomputing them (the engine's P.walk_store_e and the launchers agree on it)
#ifndef GRAPE_WALK_STORE_MIN_D
#define GRAPE_WALK_STORE_MIN_D 4
#endif
constexpr int kWalkStoreMinD = GRAPE_WALK_STORE_MIN_D;
// GRAPE_WALK_XROW: the walks read the controls row-major from x itself (B.xT = x, stride 1 per value,
// nx per evaluation) instead of a transposed copy, and the engine skips k_transpose_x.  Each lane
// streams its own row: 8 steps per 64-B line, reused from the vector cache.  Round 4 (per-class
// walks) measured it neutral; with the merged walks it wins: C2 36.8 -> 38.4 M evals/s (fwd 0.269 ->
// 0.222, grad 0.470 -> 0.481 ms per pass, no transpose; profiles/r05/ab_xrow)
#ifndef GRAPE_WALK_XROW
#define GRAPE_WALK_XROW 1
#endif
constexpr bool kWalkXRow = GRAPE_WALK_XROW;
// error sources on a phase-covariant class (round 6): the lab-frame walks k_walk_wsum_lab / k_walk_err_lab
// (grape_walk.hpp; the engine's P.gauge_lab), no images.  0: the image walk and its back end (A/B)
#ifndef GRAPE_WALK_ERR_LAB
#define GRAPE_WALK_ERR_LAB 1
#endif
constexpr int kLabBaseMaxLanes = 256;  // k_gauge_err_base_fill: one lane per (sector, base matrix)
}  // namespace grape

namespace grape_walk {
// one lane per (sector, evaluation, chunk) of the class: stage 0 = k_walk_fwd (chunk totals to
// B.Tc), stage 1 = k_walk_grad (per-sector F_dx terms to B.sec_part, evaluation-fastest).  With
// error sources (P.ne > 0, nvg == 1): stage 0 = k_walk_img (chunk totals and the lane-minor
// local-frame images to B.Zl), stage 1 = k_walk_img_sum (per-sector F_dx terms to B.sec_part,
// lane-major, and the chunk sums of W to B.Wc), stage 2 = k_walk_err_grad (per-sector F_d2err_dx
// terms to B.sec_part_err, lane-major).  Phase-covariant classes with error sources (P.gauge_lab): stage 0 =
// k_walk_wsum_lab (chunk totals and the chunk sums of W to B.Wc), stage 1 = nothing, stage 2 =
// k_walk_err_lab (F_dx and F_d2err_dx terms, lane-major), no images
template <int D>
hipError_t launch(int stage, const grape::DevProblem &P, const grape::DevBatch &B, hipStream_t st);
// Latency-bound calls of the Rydberg layout -- class 0: one 4-level sector (permutation sectors) or
// one 3-level sector (symmetry-adapted), class 1: two 2-level sectors, no error sources, one gradient
// parameter -- run both classes' walks
// of a stage in ONE launch (k_walk_fwd_pair / k_walk_grad_pair).  pair_ok tells whether the layout
// fits; launch_pair(stage, ...) then replaces launch<4>(stage, class 0) + launch<2>(stage, class 1).
bool pair_ok(const grape::DevProblem &P0, const grape::DevProblem &P1);
hipError_t launch_pair(int stage, const grape::DevProblem &P0, const grape::DevBatch &B0, const grape::DevProblem &P1,
                       const grape::DevBatch &B1, hipStream_t st);
// Throughput passes of the same layout with phase-covariant classes at equal chunking: ONE lane walks
// both classes of an (evaluation, chunk) (k_walk_fwd_m / k_walk_grad_m); the gradient stage writes
// one F_dx part, class 0's + class 1's (a_first: class A is the plan's class 0), into class A's
// sec_part.  Stage 0: k_walk_fwd_m (chunk totals, lane-minor), stage 2: k_scan_seq (carries and U
// from them), stage 1: k_walk_grad_m.  merged_ok tells whether the classes fit.
bool merged_ok(const grape::DevProblem &PA, const grape::DevProblem &PB);
// 1: the merged gradient walk writes F_dx rows itself (no k_sec_reduce for such passes)
bool merged_writes_fdx();
// E~ of the class's nsec sectors into out [nsec][D][D] (DevProblem::gauge_Et; scr: 2 D^2 complex per sector)
hipError_t fill_gauge_base(const grape::DevProblem &P, int nsec, grape::cd *scr, grape::cd *out, hipStream_t st);
// the lab-frame error walks' base table [nsec][1 + 2 ne][D][D] (DevProblem::gauge_Et with gauge_lab; scr: 2 D^2
// complex per base matrix)
hipError_t fill_gauge_err_base(const grape::DevProblem &P, int nsec, grape::cd *scr, grape::cd *out, hipStream_t st);
hipError_t launch_merged(int stage, const grape::DevProblem &PA, const grape::DevBatch &BA, const grape::DevProblem &PB,
                         const grape::DevBatch &BB, int a_first, hipStream_t st);
// F_dx parts the class's gradient stage writes per evaluation: its sectors, or (k_walk_grad with several
// sectors per lane, no error sources) one pre-summed part per lane row (grape_walk.hpp kWalkPresum)
int grad_parts(const grape::DevProblem &P);
// the walks' controls: x [nb][nx] -> xT [nx][nb] (B.xT), once per launch for every walk class
hipError_t transpose_x(const double *x, double *xT, int nb, int nx, hipStream_t st);
}  // namespace grape_walk
