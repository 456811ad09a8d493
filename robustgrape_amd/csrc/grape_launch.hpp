// grape_launch.hpp -- host-side launch sequences of the small-d engine, one
// instantiation per compile-time dimension D.  Each D is compiled in its own
// translation unit (grape_inst.hip with -DGRAPE_INST_DIM=D) so the build runs
// in parallel; grape_engine.hip only sees the declarations (extern template).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "grape.h"
#include "grape_errpath.hpp"
#include "grape_lane.hpp"
#include "grape_walk_api.hpp"
#include "grape_projector_api.hpp"

namespace grape_host {

using grape::cd;
using grape::DevBatch;
using grape::DevProblem;

// Scan workgroups: one per evaluation, W waves of row groups.  W = 8 (52 chunks
// of L = 10 steps at d = 9, N_t = 512) has the shortest chains; W = 4 halves
// the LDS and registers per block so two evaluations share a CU, which wins
// once there are more evaluations than CUs (plan-time choice, see kScanWide).
// Sector problems with many sub-evaluations per CU take W = 1: fewer chunks mean
// fewer carries and per-chunk images to stream (C2 2.69 -> 2.80 M evals/s).
constexpr int kScanWide = 8, kScanNarrow = 4, kScanTiny = 1;
// Latency-bound calls (fewer sub-evaluations than CUs: single evaluations, C4's 32 restarts per
// GPU, the optimiser's tail rounds) of the chunk-walk classes (<= kWalkMaxD levels, no error
// sources) take 16-wave scans: twice the chunks of kScanWide, so each walk lane steps half as far
// (L = 2 at 4 levels, L = 1 at 2 levels for N_t = 512).
constexpr int kScanLatency = 16;

// Lane-matrix exponentials (grape_lane.hpp k_expm_lane) for d <= kLaneMaxD (operator-basis
// builders; closure tables keep k_expm_table); GRAPE_OPT_NO_LANE selects the row-group k_expm (A/B and
// the bit-identity test).  Measured per instantiation (C2 sectors, 32 768 evaluations per pass,
// rocprof, one box, profiles/r02/lane): S = 2 k_expm 1.057 -> 0.957 ms; S = 4 1.99 -> 2.26 ms (a
// 4 x 4 complex matrix per lane is 64 VGPRs: 2 waves/SIMD), so d = 4 keeps the row groups.
constexpr int kLaneMaxD = 3;
// Sector stage 0 without error sources: propagators and chunk chains per lane up to kChainMaxD
// (k_expm_chain_lane; a d = 4 variant measured 7.32 vs 3.81 ms and was dropped, grape_lane.hpp);
// GRAPE_OPT_NO_CHAIN keeps k_expm + k_scan.  (Both are the fallbacks of the chunk walks,
// grape_walk.hpp, which serve these classes by default.)
constexpr int kChainMaxD = kLaneMaxD;
template <int D>
bool use_chain(const DevProblem &P, const DevBatch &B) {
    return GRAPE_HAVE_LANE && D <= kChainMaxD && B.Htab == nullptr && !(P.opts & (GRAPE_OPT_NO_LANE | GRAPE_OPT_NO_CHAIN));
}
template <int D>
bool use_lane(const DevProblem &P, const DevBatch &B) {
    return GRAPE_HAVE_LANE && D <= kLaneMaxD && B.Htab == nullptr && !(P.opts & GRAPE_OPT_NO_LANE);
}
template <int D, bool ERR>
void launch_expm_lane(const DevProblem &P, const DevBatch &B, hipStream_t st) {
#if GRAPE_HAVE_LANE
    if constexpr (D <= kLaneMaxD) {
        const long n = (long)B.nb * P.Nt * P.nv;
        hipLaunchKernelGGL((grape::k_expm_lane<D, ERR>),
                           dim3((unsigned)((n + grape::kLaneBlock - 1) / grape::kLaneBlock)), dim3(grape::kLaneBlock), 0,
                           st, P, B);
    }
#endif
}
template <int D>
size_t expm_lds() { return (size_t)grape::Geo<D>::GPW * grape::Geo<D>::GROUP_CD * sizeof(cd); }
template <int D>  // k_expm / k_expm_grad / k_expm_table (grape_kernels.hpp EXPM_GROUP_CD)
size_t expm_lean_lds() { return (size_t)grape::Geo<D>::GPW * EXPM_GROUP_CD(D) * sizeof(cd); }
template <int D>
size_t errpath_lds() {  // per group: tile + aux, then a second tile (k_err_local, k_err_grad)
    return (size_t)grape::Geo<D>::GPW * (grape::Geo<D>::GROUP_CD + grape::Geo<D>::TILE) * sizeof(cd);
}
template <int D>
size_t errscan_lds(int W) {
    return ((size_t)W * grape::Geo<D>::GPW * grape::Geo<D>::GROUP_CD + 4 * grape::Geo<D>::TILE) * sizeof(cd);
}
template <int D>
size_t scan_lds(int W) {
    return ((size_t)W * grape::Geo<D>::GPW * grape::Geo<D>::GROUP_CD + 3 * grape::Geo<D>::TILE) * sizeof(cd);
}

// k_scan / k_err_scan at the plan's width (P.scan_waves: 1, 4 or 8 waves per workgroup)
template <int D>
void launch_scan(const DevProblem &P, const DevBatch &B, hipStream_t st) {
    if constexpr (D <= grape::kWalkMaxD) {
        if (P.scan_waves == kScanLatency) {
            hipLaunchKernelGGL((grape::k_scan<D, kScanLatency>), dim3(B.nb), dim3(64 * kScanLatency),
                               scan_lds<D>(kScanLatency), st, P, B);
            return;
        }
    }
    if (P.scan_waves == kScanTiny)
        hipLaunchKernelGGL((grape::k_scan<D, kScanTiny>), dim3(B.nb), dim3(64 * kScanTiny), scan_lds<D>(kScanTiny), st,
                           P, B);
    else if (P.scan_waves == kScanNarrow)
        hipLaunchKernelGGL((grape::k_scan<D, kScanNarrow>), dim3(B.nb), dim3(64 * kScanNarrow),
                           scan_lds<D>(kScanNarrow), st, P, B);
    else
        hipLaunchKernelGGL((grape::k_scan<D, kScanWide>), dim3(B.nb), dim3(64 * kScanWide), scan_lds<D>(kScanWide), st,
                           P, B);
}
// the scans of two walk classes in one launch (D0 = 4 or 3, D1 = 2: the Rydberg layout), both at
// width W: the latency scans (16 waves), and the throughput passes' one-wave scans, where the two
// classes' short, under-filled scans then run side by side instead of one after the other
template <int D0, int D1, int W = kScanLatency>
hipError_t launch_scan_pair(const DevProblem &P0, const DevBatch &B0, const DevProblem &P1, const DevBatch &B1,
                            hipStream_t st) {
    const size_t lds = std::max(scan_lds<D0>(W), scan_lds<D1>(W));
    static unsigned long long limit_set = 0;  // per device (idempotent: a race only repeats the call)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev >= 64) return hipErrorInvalidDevice;
    if (!((limit_set >> dev) & 1ull)) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&grape::k_scan_pair<D0, D1, W>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        limit_set |= 1ull << dev;
    }
    hipLaunchKernelGGL((grape::k_scan_pair<D0, D1, W>), dim3((unsigned)(B0.nb + B1.nb)), dim3(64 * W), lds, st, P0,
                       B0, P1, B1);
    return hipGetLastError();
}
template <int D>
void launch_err_scan(const DevProblem &P, const DevBatch &B, hipStream_t st) {
    if constexpr (D <= grape::kWalkMaxD) {
        if (P.scan_waves == kScanLatency) {  // (the lab-frame error walks' latency-bound calls)
            hipLaunchKernelGGL((grape::k_err_scan<D, kScanLatency>), dim3(B.nb * P.ne), dim3(64 * kScanLatency),
                               errscan_lds<D>(kScanLatency), st, P, B);
            return;
        }
    }
    if (P.scan_waves == kScanTiny)
        hipLaunchKernelGGL((grape::k_err_scan<D, kScanTiny>), dim3(B.nb * P.ne), dim3(64 * kScanTiny),
                           errscan_lds<D>(kScanTiny), st, P, B);
    else if (P.scan_waves == kScanNarrow)
        hipLaunchKernelGGL((grape::k_err_scan<D, kScanNarrow>), dim3(B.nb * P.ne), dim3(64 * kScanNarrow),
                           errscan_lds<D>(kScanNarrow), st, P, B);
    else
        hipLaunchKernelGGL((grape::k_err_scan<D, kScanWide>), dim3(B.nb * P.ne), dim3(64 * kScanWide),
                           errscan_lds<D>(kScanWide), st, P, B);
}

// ---------------------------------------------------------------------------
// dispatch helpers over the compile-time dimension
// ---------------------------------------------------------------------------
// Optional per-kernel event marks (profiling mode): fn(ctx, kernel, 0|1) around each launch.
struct KMark {
    void *ctx = nullptr;
    void (*fn)(void *, int, int) = nullptr;
    void operator()(int k, int phase) const {
        if (fn) fn(ctx, k, phase);
    }
};

template <int D>
hipError_t launch_pipeline(const DevProblem &P, const DevBatch &B, hipStream_t st, const KMark &mark) {
    constexpr int GPW = grape::Geo<D>::GPW;
    const long nexp = (long)B.nb * P.Nt * P.nv;
    // closure mode (grape_fidelity_grad_tables): every variant comes from the host H table
    const bool table = B.Htab != nullptr;
    const bool fused = P.ne == 0 && !table;  // eps-variants exp'd and contracted in k_expm_grad
    mark(GRAPE_KERNEL_EXPM, 0);
    if (table)
        hipLaunchKernelGGL(grape::k_expm_table<D>, dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
    else if (use_lane<D>(P, B))
        fused ? launch_expm_lane<D, false>(P, B, st) : launch_expm_lane<D, true>(P, B, st);
    else if (!fused)
        hipLaunchKernelGGL((grape::k_expm<D, true>), dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
    else
        hipLaunchKernelGGL((grape::k_expm<D, false>), dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
    mark(GRAPE_KERNEL_EXPM, 1);
    mark(GRAPE_KERNEL_EXPM_HIGH, 0);
    hipLaunchKernelGGL(grape::k_expm_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, B.E, B.overflow,
                       B.overflow_count, B.status, 1);
    mark(GRAPE_KERNEL_EXPM_HIGH, 1);
    mark(GRAPE_KERNEL_SCAN, 0);
    launch_scan<D>(P, B, st);
    if (P.gen_proj) {  // general projector: F, M'_c (and F_dx_add's target part) redone in general form
        const hipError_t e = grape_proj::launch_fid_head(grape_proj::small_heads(P, B), B.nb, st);
        if (e != hipSuccess) return e;
    }
    mark(GRAPE_KERNEL_SCAN, 1);
    if (fused) {
        const int nvg = P.np + (P.xadd_dep ? P.na : 0);
        const long ng = (long)B.nb * P.Nt * nvg;
        mark(GRAPE_KERNEL_EXPM_GRAD, 0);
        hipLaunchKernelGGL(grape::k_expm_grad<D>, dim3((unsigned)((ng + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
        mark(GRAPE_KERNEL_EXPM_GRAD, 1);
        mark(GRAPE_KERNEL_GRAD_HIGH, 0);
        hipLaunchKernelGGL(grape::k_grad_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, P, B);
        mark(GRAPE_KERNEL_GRAD_HIGH, 1);
    } else if (P.ne == 0) {
        const long ng = (long)B.nb * P.Nt;
        mark(GRAPE_KERNEL_GRAD, 0);
        hipLaunchKernelGGL(grape::k_grad<D>, dim3((unsigned)((ng + GPW - 1) / GPW)), dim3(64), expm_lds<D>(), st,
                           P, B);
        mark(GRAPE_KERNEL_GRAD, 1);
    } else {  // error sources: local-frame images of every difference (and F_dx) per step
        const long ng = (long)B.nb * P.Nt;
        mark(GRAPE_KERNEL_GRAD, 0);
        hipLaunchKernelGGL(grape::k_err_local<D>, dim3((unsigned)((ng + GPW - 1) / GPW)), dim3(64), errpath_lds<D>(),
                           st, P, B);
        mark(GRAPE_KERNEL_GRAD, 1);
    }
    if (P.ne > 0) {
        mark(GRAPE_KERNEL_ERR_SCAN, 0);
        launch_err_scan<D>(P, B, st);
        if (P.gen_proj) {
            const hipError_t e = grape_proj::launch_err_head(grape_proj::small_heads(P, B), B.nb, st);
            if (e != hipSuccess) return e;
        }
        mark(GRAPE_KERNEL_ERR_SCAN, 1);
        const long ne_items = (long)B.nb * P.nchunks * P.ne;
        mark(GRAPE_KERNEL_ERR_GRAD, 0);
        hipLaunchKernelGGL(grape::k_err_grad<D>, dim3((unsigned)((ne_items + GPW - 1) / GPW)), dim3(64),
                           errpath_lds<D>(), st, P, B);
        mark(GRAPE_KERNEL_ERR_GRAD, 1);
    }
    if (P.xadd_dep && P.na > 0) {
        mark(GRAPE_KERNEL_REDUCE, 0);
        const int nred = B.nb * P.na * (1 + P.ne);
        hipLaunchKernelGGL(grape::k_reduce_add<D>, dim3((nred + 255) / 256), dim3(256), 0, st, P, B);
        mark(GRAPE_KERNEL_REDUCE, 1);
    }
    return hipGetLastError();
}

// Sectors (P.sectors, D = the sector size of one class, B.nb = evaluations x nsec).  Stage 0:
// nominal sector propagators (every variant with error sources) -> sector scans (U_w,
// carries).  Then (grape_engine.hip) the sector head over every class (F, the blocks of M,
// target part).  Stage 1: per-chunk images M'_c (k_sec_mc), then without error sources the
// eps-variant sector exps contracted in place, with error sources the local-frame images (and
// F_dx terms) and the sector error scans (Tot blocks, T_c, Ttot_c).  Then the sector error
// head (F_d2err, the blocks of M_e).  Stage 2 (error sources): M'_{c,e} (k_sec_mc_err) and
// the F_d2err_dx walks.  Finally launch_sector_reduce sums the sector terms.
template <int D>
hipError_t launch_sector_stage(int stage, const DevProblem &P, const DevBatch &B, hipStream_t st,
                               const KMark &mark) {
    constexpr int GPW = grape::Geo<D>::GPW;
    if constexpr (D >= 2 && D <= grape::kWalkMaxD) {
        if (P.walk) {  // chunk walks (grape_walk.hpp): no E / Q intermediates
            if (stage == 0) {
                mark(GRAPE_KERNEL_WALK_FWD, 0);
                const hipError_t e = grape_walk::launch<D>(0, P, B, st);
                mark(GRAPE_KERNEL_WALK_FWD, 1);
                if (e != hipSuccess) return e;
                mark(GRAPE_KERNEL_SCAN, 0);
                launch_scan<D>(P, B, st);
                mark(GRAPE_KERNEL_SCAN, 1);
                return hipGetLastError();
            }
            if (stage == 1) {
                if (P.ne > 0 && !P.gauge_lab) {  // k_walk_img_sum reads M'_c (k_walk_grad / k_walk_err_lab form it in the lane)
                    mark(GRAPE_KERNEL_REDUCE, 0);
                    const long nmc = (long)B.nb * P.nchunks * D * D;
                    hipLaunchKernelGGL(grape::k_sec_mc<D>, dim3((unsigned)((nmc + 255) / 256)), dim3(256), 0, st, P, B);
                    mark(GRAPE_KERNEL_REDUCE, 1);
                }
                const int kid = P.ne > 0 ? GRAPE_KERNEL_GRAD : GRAPE_KERNEL_WALK_GRAD;  // k_walk_img_sum / k_walk_grad
                mark(kid, 0);
                const hipError_t e = grape_walk::launch<D>(1, P, B, st);
                mark(kid, 1);
                if (e != hipSuccess) return e;
                if (P.ne > 0) {  // the error scans start from the chunk sums of W (B.Wc)
                    mark(GRAPE_KERNEL_ERR_SCAN, 0);
                    launch_err_scan<D>(P, B, st);
                    mark(GRAPE_KERNEL_ERR_SCAN, 1);
                }
                return hipGetLastError();
            }
            if (P.ne == 0) return hipErrorInvalidValue;  // no stage 2 without error sources
            // stage 2 with error sources: M'_{c,e}, then the F_d2err_dx walks over the lane-minor images
            mark(GRAPE_KERNEL_ERR_GRAD, 0);
            const long nmce = (long)B.nb * P.ne * P.nchunks * D * D;
            if (!P.gauge_lab)  // (k_walk_err_lab forms M'_{c,e} in the lane)
                hipLaunchKernelGGL(grape::k_sec_mc_err<D>, dim3((unsigned)((nmce + 255) / 256)), dim3(256), 0, st, P, B);
            const hipError_t e = grape_walk::launch<D>(2, P, B, st);
            mark(GRAPE_KERNEL_ERR_GRAD, 1);
            return e != hipSuccess ? e : hipGetLastError();
        }
    }
    if (stage == 0) {
        const long nexp = (long)B.nb * P.Nt * P.nv;
#if GRAPE_HAVE_LANE
        if constexpr (D <= kChainMaxD) {
            if (use_chain<D>(P, B) && P.ne == 0 && P.nv == 1) {  // propagators + chunk chains per lane
                mark(GRAPE_KERNEL_EXPM, 0);
                const long n = (long)B.nb * P.nchunks;
                hipLaunchKernelGGL(grape::k_expm_chain_lane<D>,
                                   dim3((unsigned)((n + grape::kLaneBlock - 1) / grape::kLaneBlock)),
                                   dim3(grape::kLaneBlock), 0, st, P, B);
                mark(GRAPE_KERNEL_EXPM, 1);
                mark(GRAPE_KERNEL_EXPM_HIGH, 0);
                hipLaunchKernelGGL(grape::k_expm_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, B.E, B.overflow,
                                   B.overflow_count, B.status, 1);
                mark(GRAPE_KERNEL_EXPM_HIGH, 1);
                mark(GRAPE_KERNEL_SCAN, 0);
                DevBatch Bc = B;
                Bc.chains_done = 1;
                launch_scan<D>(P, Bc, st);
                mark(GRAPE_KERNEL_SCAN, 1);
                return hipGetLastError();
            }
        }
#endif
        mark(GRAPE_KERNEL_EXPM, 0);
        if (use_lane<D>(P, B))
            P.ne > 0 ? launch_expm_lane<D, true>(P, B, st) : launch_expm_lane<D, false>(P, B, st);
        else if (P.ne > 0)
            hipLaunchKernelGGL((grape::k_expm<D, true>), dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                               expm_lean_lds<D>(), st, P, B);
        else
            hipLaunchKernelGGL((grape::k_expm<D, false>), dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                               expm_lean_lds<D>(), st, P, B);
        mark(GRAPE_KERNEL_EXPM, 1);
        mark(GRAPE_KERNEL_EXPM_HIGH, 0);
        hipLaunchKernelGGL(grape::k_expm_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, B.E, B.overflow,
                           B.overflow_count, B.status, 1);
        mark(GRAPE_KERNEL_EXPM_HIGH, 1);
        mark(GRAPE_KERNEL_SCAN, 0);
        launch_scan<D>(P, B, st);
        mark(GRAPE_KERNEL_SCAN, 1);
        return hipGetLastError();
    }
    if (stage == 1) {
        mark(GRAPE_KERNEL_REDUCE, 0);
        const long nmc = (long)B.nb * P.nchunks * D * D;
        hipLaunchKernelGGL(grape::k_sec_mc<D>, dim3((unsigned)((nmc + 255) / 256)), dim3(256), 0, st, P, B);
        mark(GRAPE_KERNEL_REDUCE, 1);
        if (P.ne > 0) {
            const long ng = (long)B.nb * P.Nt;
            mark(GRAPE_KERNEL_GRAD, 0);
            hipLaunchKernelGGL(grape::k_err_local<D>, dim3((unsigned)((ng + GPW - 1) / GPW)), dim3(64),
                               errpath_lds<D>(), st, P, B);
            mark(GRAPE_KERNEL_GRAD, 1);
            mark(GRAPE_KERNEL_ERR_SCAN, 0);
            launch_err_scan<D>(P, B, st);
            mark(GRAPE_KERNEL_ERR_SCAN, 1);
            return hipGetLastError();
        }
        const long ng = (long)B.nb * P.Nt * P.nvg;
        mark(GRAPE_KERNEL_EXPM_GRAD, 0);
        hipLaunchKernelGGL(grape::k_expm_grad<D>, dim3((unsigned)((ng + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
        mark(GRAPE_KERNEL_EXPM_GRAD, 1);
        mark(GRAPE_KERNEL_GRAD_HIGH, 0);
        hipLaunchKernelGGL(grape::k_grad_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, P, B);
        mark(GRAPE_KERNEL_GRAD_HIGH, 1);
        return hipGetLastError();
    }
    // stage 2 (error sources)
    mark(GRAPE_KERNEL_ERR_GRAD, 0);
    const long nmce = (long)B.nb * P.ne * P.nchunks * D * D;
    hipLaunchKernelGGL(grape::k_sec_mc_err<D>, dim3((unsigned)((nmce + 255) / 256)), dim3(256), 0, st, P, B);
    const long ne_items = (long)B.nb * P.nchunks * P.ne;
    hipLaunchKernelGGL(grape::k_err_grad<D>, dim3((unsigned)((ne_items + GPW - 1) / GPW)), dim3(64),
                       errpath_lds<D>(), st, P, B);
    mark(GRAPE_KERNEL_ERR_GRAD, 1);
    return hipGetLastError();
}

// The sum over sectors (and, xadd_dep, over steps) of one launch of nev evaluations.
template <int D>
hipError_t launch_sector_reduce(const DevProblem &P, const DevBatch &B, const grape::SecParts &S, int nev,
                                hipStream_t st, const KMark &mark) {
    mark(GRAPE_KERNEL_REDUCE, 0);
    const long per = (long)P.Nt * P.nvg;
    hipLaunchKernelGGL(grape::k_sec_reduce<D>,
                       dim3((unsigned)((nev + grape::kRedTile - 1) / grape::kRedTile),
                            (unsigned)((per + grape::kRedTile - 1) / grape::kRedTile)),
                       dim3(256), 0, st, P, B.Fdx, B.part_add, S, nev);
    if (P.ne > 0)
        hipLaunchKernelGGL(grape::k_sec_reduce_err<D>,
                           dim3((unsigned)((nev + grape::kRedTile - 1) / grape::kRedTile),
                                (unsigned)((per * P.ne + grape::kRedTile - 1) / grape::kRedTile)),
                           dim3(256), 0, st, P, B.Fd2dx, B.part_err_add, S, nev);
    if (P.xadd_dep && P.na > 0) {
        DevBatch Be = B;  // the x_add sums run over evaluations, not sub-evaluations
        Be.nb = nev;
        const int nr = nev * P.na * (1 + P.ne);
        hipLaunchKernelGGL(grape::k_reduce_add<D>, dim3((nr + 255) / 256), dim3(256), 0, st, P, Be);
    }
    mark(GRAPE_KERNEL_REDUCE, 1);
    return hipGetLastError();
}

template <int D>
hipError_t launch_expm_raw(const cd *A, cd *E, int n, int *ovf, int *ovf_count, int *status, int *mstats,
                           hipStream_t st) {
    constexpr int GPW = grape::Geo<D>::GPW;
    hipLaunchKernelGGL(grape::k_expm_raw<D>, dim3((n + GPW - 1) / GPW), dim3(64), expm_lds<D>(), st, A, E, n, ovf,
                       ovf_count, status, mstats);
    hipLaunchKernelGGL(grape::k_expm_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, E, ovf, ovf_count, status, 0);
    return hipGetLastError();
}

// Every variant of every step of ONE launch's evaluations stored in B.E (P.nv, P.vs
// as given): grape_unitary_derivs' propagator table.  ERR selects the builder with
// error terms.
template <int D>
hipError_t launch_expm_variants(const DevProblem &P, const DevBatch &B, hipStream_t st) {
    constexpr int GPW = grape::Geo<D>::GPW;
    const long nexp = (long)B.nb * P.Nt * P.nv;
    if (P.ne > 0)
        hipLaunchKernelGGL((grape::k_expm<D, true>), dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
    else
        hipLaunchKernelGGL((grape::k_expm<D, false>), dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64),
                           expm_lean_lds<D>(), st, P, B);
    hipLaunchKernelGGL(grape::k_expm_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, B.E, B.overflow,
                       B.overflow_count, B.status, 1);
    return hipGetLastError();
}

// Closure mode: every variant of every step of ONE launch's evaluations from the host H
// table B.Htab ([nb][Nt][P.nv][D][D] column-major) into B.E (row-major).
template <int D>
hipError_t launch_expm_table(const DevProblem &P, const DevBatch &B, hipStream_t st) {
    constexpr int GPW = grape::Geo<D>::GPW;
    const long nexp = (long)B.nb * P.Nt * P.nv;
    hipLaunchKernelGGL(grape::k_expm_table<D>, dim3((unsigned)((nexp + GPW - 1) / GPW)), dim3(64), expm_lean_lds<D>(), st,
                       P, B);
    hipLaunchKernelGGL(grape::k_expm_high<D>, dim3(64), dim3(64), expm_lds<D>(), st, B.E, B.overflow,
                       B.overflow_count, B.status, 1);
    return hipGetLastError();
}

template <int D, int W>
hipError_t set_lds_limits_w() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&grape::k_scan<D, W>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)scan_lds<D>(W));
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(&grape::k_err_scan<D, W>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)errscan_lds<D>(W));
}
template <int D>
hipError_t set_lds_limits() {
    hipError_t e = set_lds_limits_w<D, kScanWide>();
    if constexpr (D <= grape::kWalkMaxD) {
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(&grape::k_scan<D, kScanLatency>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)scan_lds<D>(kScanLatency));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(&grape::k_err_scan<D, kScanLatency>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)errscan_lds<D>(kScanLatency));
    }
    if (e == hipSuccess) e = set_lds_limits_w<D, kScanNarrow>();
    return e != hipSuccess ? e : set_lds_limits_w<D, kScanTiny>();
}


#define GRAPE_DIMS(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
// (the scan pair is instantiated in the D = 4 translation unit)
#define GRAPE_DECLARE_SCAN_PAIR(EXT)                                                                       \
    EXT template hipError_t launch_scan_pair<4, 2>(const DevProblem &, const DevBatch &, const DevProblem &, \
                                                    const DevBatch &, hipStream_t);

#define GRAPE_DECLARE_DIM(d, EXT)                                                                          \
    EXT template hipError_t launch_pipeline<d>(const DevProblem &, const DevBatch &, hipStream_t, const KMark &); \
    EXT template hipError_t launch_sector_stage<d>(int, const DevProblem &, const DevBatch &, hipStream_t,     \
                                                   const KMark &);                                            \
    EXT template hipError_t launch_sector_reduce<d>(const DevProblem &, const DevBatch &, const grape::SecParts &, \
                                                    int, hipStream_t, const KMark &);                         \
    EXT template hipError_t launch_expm_raw<d>(const cd *, cd *, int, int *, int *, int *, int *, hipStream_t);  \
    EXT template hipError_t set_lds_limits<d>();                                                          \
    EXT template hipError_t launch_expm_variants<d>(const DevProblem &, const DevBatch &, hipStream_t);     \
    EXT template hipError_t launch_expm_table<d>(const DevProblem &, const DevBatch &, hipStream_t);

}  // namespace grape_host
