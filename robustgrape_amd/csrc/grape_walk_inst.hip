// grape_walk_inst.hip -- the chunk-walk kernels (grape_walk.hpp) for D = 2 .. kWalkMaxD and their
// launchers; built with -mllvm -disable-machine-licm (robustgrape_amd/build.py).
#include <type_traits>

#include "grape_walk.hpp"
#include "grape_walk_api.hpp"

namespace grape_walk {

template <int D, int NS>
void launch_ns(int stage, const grape::DevProblem &P, const grape::DevBatch &B, hipStream_t st) {
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const long lanes = (long)(B.nb / ns) * P.nchunks;
    const dim3 grid((unsigned)((lanes + grape::kWalkBlock - 1) / grape::kWalkBlock), (unsigned)(ns / NS));
    const dim3 blk(grape::kWalkBlock);
    if (P.ne > 0 && P.gauge_lab) {  // phase-covariant class with error sources: the lab-frame walks
        if (stage == 0) {  // chunk sums of W per error (blockIdx.z < ne) and chunk totals (blockIdx.z = ne)
            hipLaunchKernelGGL((grape::k_walk_wsum_lab<D, NS>), dim3(grid.x, grid.y, (unsigned)P.ne + 1), blk, 0, st, P, B);
        } else if (stage == 2) {  // F_d2err_dx per error (blockIdx.z < ne) and F_dx (blockIdx.z = ne)
            hipLaunchKernelGGL((grape::k_walk_err_lab<D, NS>), dim3(grid.x, grid.y, (unsigned)P.ne + 1), blk, 0, st, P, B);
        }
        return;
    }
    if (P.ne > 0) {  // error sources: the image walk, then its back end (grape_walk.hpp)
        if (stage == 0) {
            if (P.gauge) hipLaunchKernelGGL((grape::k_walk_img_gauge<D, NS>), grid, blk, 0, st, P, B);
            else hipLaunchKernelGGL((grape::k_walk_img<D, NS>), grid, blk, 0, st, P, B);
        } else if (stage == 1) {  // F_dx traces of Z1 and the chunk sums of W (k_err_scan's Phase A)
            // (the 2-level image walk summed W itself: WalkCfg::IMG_WSUM)
            if (!(grape::WalkCfg<D, NS>::IMG_WSUM && P.ne <= grape::kWsumMaxE))
                hipLaunchKernelGGL((grape::k_walk_img_sum<D, NS>), grid, blk, 0, st, P, B);
        } else {  // the F_d2err_dx walks, one lane per (chunk, evaluation, error)
            const dim3 grid_e((unsigned)((lanes * P.ne + grape::kWalkBlock - 1) / grape::kWalkBlock), (unsigned)(ns / NS));
            hipLaunchKernelGGL((grape::k_walk_err_grad<D, NS>), grid_e, blk, 0, st, P, B);
        }
        return;
    }
    if (P.gauge) {  // phase-covariant class: E_k = D_k E~ D_k^dag, one exponential per lane (grape_walk.hpp)
        if constexpr (NS == 2) {
            if (P.twin) {
                if (stage == 0) hipLaunchKernelGGL((grape::k_walk_fwd<D, NS, false, true, true>), grid, blk, 0, st, P, B);
                else hipLaunchKernelGGL((grape::k_walk_grad<D, NS, false, 1, true, true>), grid, blk, 0, st, P, B);
                return;
            }
        }
        if (stage == 0) hipLaunchKernelGGL((grape::k_walk_fwd<D, NS, false, false, true>), grid, blk, 0, st, P, B);
        else hipLaunchKernelGGL((grape::k_walk_grad<D, NS, false, 1, false, true>), grid, blk, 0, st, P, B);
        return;
    }
    if constexpr (NS == 2) {  // twin sectors (P.twin): one exponential per step for both
        if (P.twin) {
            if (stage == 0) hipLaunchKernelGGL((grape::k_walk_fwd<D, NS, false, true>), grid, blk, 0, st, P, B);
            else if (P.nvg == 1) hipLaunchKernelGGL((grape::k_walk_grad<D, NS, false, 1, true>), grid, blk, 0, st, P, B);
            else hipLaunchKernelGGL((grape::k_walk_grad<D, NS, false, 0, true>), grid, blk, 0, st, P, B);
            return;
        }
    }
    // stored propagators: classes of >= kWalkStoreMinD levels (engine: P.walk_store_e)
    constexpr bool CAN_STORE = D >= grape::kWalkStoreMinD;
    const bool store = CAN_STORE && P.walk_store_e;
    if (stage == 0) {
        if (store) hipLaunchKernelGGL((grape::k_walk_fwd<D, NS, CAN_STORE>), grid, blk, 0, st, P, B);
        else hipLaunchKernelGGL((grape::k_walk_fwd<D, NS, false>), grid, blk, 0, st, P, B);
        return;
    }
    if (store) {
        if (P.nvg == 1) hipLaunchKernelGGL((grape::k_walk_grad<D, NS, CAN_STORE, 1>), grid, blk, 0, st, P, B);
        else hipLaunchKernelGGL((grape::k_walk_grad<D, NS, CAN_STORE, 0>), grid, blk, 0, st, P, B);
    } else {
        if (P.nvg == 1) hipLaunchKernelGGL((grape::k_walk_grad<D, NS, false, 1>), grid, blk, 0, st, P, B);
        else hipLaunchKernelGGL((grape::k_walk_grad<D, NS, false, 0>), grid, blk, 0, st, P, B);
    }
}

// sectors per lane: all of the class's sectors (<= 3) for D <= 3 -- one set of control trig for
// all of them and independent chains to interleave -- one sector per lane at D = 4 (registers)
template <int D>
hipError_t launch(int stage, const grape::DevProblem &P, const grape::DevBatch &B, hipStream_t st) {
    const int ns = P.nsec > 1 ? P.nsec : 1;
    if ((long)(B.nb / ns) * P.nchunks <= 0) return hipSuccess;
    if constexpr (D == 2) {  // (the Rydberg two-level classes; a three-level class takes one sector per lane)
        if (GRAPE_WALK_IMG2_NS1 && P.ne > 0) {
            launch_ns<D, 1>(stage, P, B, st);
            return hipGetLastError();
        }
        if (ns == 2) {
            launch_ns<D, 2>(stage, P, B, st);
            return hipGetLastError();
        }
        if (ns == 3) {
            launch_ns<D, 3>(stage, P, B, st);
            return hipGetLastError();
        }
    }
    launch_ns<D, 1>(stage, P, B, st);
    return hipGetLastError();
}

int grad_parts(const grape::DevProblem &P) {
    const int ns = P.nsec > 1 ? P.nsec : 1;
    if (!grape::kWalkPresum || P.ne > 0 || P.D != 2) return ns;
    if (ns == 2 || ns == 3) return 1;  // launch<2>: both (all three) sectors in one lane
    return ns;
}

// class 0: one sector of 4 levels with stored propagators (permutation sectors of the Rydberg model)
// or of 3 levels (its symmetry-adapted sectors, grape_symmetry.hpp); class 1: two 2-level sectors
// (phase-covariant: both classes gauge, class 0 storing nothing)
bool pair_ok(const grape::DevProblem &P0, const grape::DevProblem &P1) {
    const bool c0 = (P0.D == 4 || P0.D == 3) &&
                    (P0.walk_store_e != 0) == (!P0.gauge && P0.D >= grape::kWalkStoreMinD);
    return P0.walk && P1.walk && P0.ne == 0 && P0.nvg == 1 && c0 && P0.nsec == 1 && P1.D == 2 && P1.nsec == 2 &&
           P1.nvg == 1 && !P1.walk_store_e && (P0.gauge != 0) == (P1.gauge != 0);
}
hipError_t launch_pair(int stage, const grape::DevProblem &P0, const grape::DevBatch &B0, const grape::DevProblem &P1,
                       const grape::DevBatch &B1, hipStream_t st) {
    if (!pair_ok(P0, P1)) return hipErrorInvalidValue;
    auto gx = [](const grape::DevProblem &P, const grape::DevBatch &B) {
        const int ns = P.nsec > 1 ? P.nsec : 1;
        const long lanes = (long)(B.nb / ns) * P.nchunks;
        return (int)((lanes + grape::kWalkBlock - 1) / grape::kWalkBlock);
    };
    const int gx0 = gx(P0, B0), gy0 = 1, gx1 = gx(P1, B1);  // class 0: one sector per lane; class 1: both per lane
    const dim3 grid((unsigned)(gx0 * gy0 + gx1)), blk(grape::kWalkBlock);
    auto go = [&](auto d0, auto tw, auto ga) {
        constexpr int D0 = decltype(d0)::value;
        constexpr bool TW = decltype(tw)::value, GA = decltype(ga)::value;
        if (stage == 0)
            hipLaunchKernelGGL((grape::k_walk_fwd_pair<D0, 1, (D0 >= grape::kWalkStoreMinD), 2, 2, TW, GA>), grid, blk, 0,
                               st, P0, B0, P1, B1, gx0, gy0, gx1);
        else
            hipLaunchKernelGGL((grape::k_walk_grad_pair<D0, 1, (D0 >= grape::kWalkStoreMinD), 2, 2, TW, GA>), grid, blk, 0,
                               st, P0, B0, P1, B1, gx0, gy0, gx1);
    };
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using T = std::true_type;
    using F = std::false_type;
    auto go2 = [&](auto ga) {
        if (P0.D == 4) P1.twin ? go(I4{}, T{}, ga) : go(I4{}, F{}, ga);
        else P1.twin ? go(I3{}, T{}, ga) : go(I3{}, F{}, ga);
    };
    if (P0.gauge) go2(T{});
    else go2(F{});
    return hipGetLastError();
}

bool merged_ok(const grape::DevProblem &PA, const grape::DevProblem &PB) {
    // (class A of 3 levels: at 4 levels the merged gradient lane spills at 2 waves per SIMD).  The merged
    // gradient walk writes F_dx itself and k_sec_reduce is skipped on merged passes, which is only right
    // when there are no x_add variants (H0 free of x_add: one gradient parameter per step) -- required
    // here, not left to pair_ok / gauge detection
    return pair_ok(PA, PB) && PA.D == 3 && PA.gauge && PB.gauge && PA.gauge_a == PB.gauge_a && PA.L == PB.L &&
           PA.nchunks == PB.nchunks && PA.np == 1 && PA.na <= 1 && !PA.xadd_dep && !PB.xadd_dep &&
           PA.nvg == 1 && PB.nvg == 1 && PA.ne == 0 && PB.ne == 0;
}
bool merged_writes_fdx() { return GRAPE_WALK_MERGED_FDX != 0; }
hipError_t fill_gauge_base(const grape::DevProblem &P, int nsec, grape::cd *scr, grape::cd *out, hipStream_t st) {
    if (nsec < 1 || nsec > 64) return hipErrorInvalidValue;
    switch (P.D) {
        case 2: hipLaunchKernelGGL(grape::k_gauge_base_fill<2>, dim3(1), dim3(64), 0, st, P, scr, out, nsec); break;
        case 3: hipLaunchKernelGGL(grape::k_gauge_base_fill<3>, dim3(1), dim3(64), 0, st, P, scr, out, nsec); break;
        case 4: hipLaunchKernelGGL(grape::k_gauge_base_fill<4>, dim3(1), dim3(64), 0, st, P, scr, out, nsec); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t fill_gauge_err_base(const grape::DevProblem &P, int nsec, grape::cd *scr, grape::cd *out, hipStream_t st) {
    if (nsec < 1 || P.ne < 1 || nsec * (1 + 2 * P.ne) > grape::kLabBaseMaxLanes) return hipErrorInvalidValue;
    const dim3 g(1), b(grape::kLabBaseMaxLanes);
    switch (P.D) {
        case 2: hipLaunchKernelGGL(grape::k_gauge_err_base_fill<2>, g, b, 0, st, P, scr, out, nsec); break;
        case 3: hipLaunchKernelGGL(grape::k_gauge_err_base_fill<3>, g, b, 0, st, P, scr, out, nsec); break;
        case 4: hipLaunchKernelGGL(grape::k_gauge_err_base_fill<4>, g, b, 0, st, P, scr, out, nsec); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_merged(int stage, const grape::DevProblem &PA, const grape::DevBatch &BA, const grape::DevProblem &PB,
                         const grape::DevBatch &BB, int a_first, hipStream_t st) {
    if (!merged_ok(PA, PB)) return hipErrorInvalidValue;
    const long lanes = (long)BA.nb * PA.nchunks;  // (class A: one sector, BA.nb evaluations)
    const dim3 grid((unsigned)((lanes + grape::kWalkBlock - 1) / grape::kWalkBlock)), blk(grape::kWalkBlock);
    auto go = [&](auto da, auto tw, auto lad) {
        constexpr int DA = decltype(da)::value;
        constexpr bool TW = decltype(tw)::value;
        constexpr bool LAD = decltype(lad)::value;
        if (stage == 0) {
            hipLaunchKernelGGL((grape::k_walk_fwd_m<DA, TW, LAD>), grid, blk, 0, st, PA, BA, PB, BB);
        } else if (stage == 2) {  // the chunk-total scan (one lane per evaluation)
            hipLaunchKernelGGL((grape::k_scan_seq<DA, TW>), dim3((unsigned)((BA.nb + grape::kSeqBlock - 1) / grape::kSeqBlock)), dim3(grape::kSeqBlock), 0, st, PA,
                               BA, PB, BB, BA.nb);
        } else if (GRAPE_WALK_GRAD_TILDE && LAD) {  // the gauge-frame gradient walk (ladder classes)
            hipLaunchKernelGGL((grape::k_walk_grad_mt<DA, TW>), grid, blk, 0, st, PA, BA, PB, BB, a_first);
        } else {
            hipLaunchKernelGGL((grape::k_walk_grad_m<DA, TW, LAD>), grid, blk, 0, st, PA, BA, PB, BB, a_first);
        }
    };
    using I3 = std::integral_constant<int, 3>;
    // ladder charges in both classes (DevProblem::gauge_ladder): compile-time charge differences
    const bool lad = PA.gauge_ladder && PB.gauge_ladder;
    if (PB.twin)
        lad ? go(I3{}, std::true_type{}, std::true_type{}) : go(I3{}, std::true_type{}, std::false_type{});
    else
        lad ? go(I3{}, std::false_type{}, std::true_type{}) : go(I3{}, std::false_type{}, std::false_type{});
    return hipGetLastError();
}

// x [nb][nx] -> xT [nx][nb] through a 32 x 32 LDS tile (both sides coalesced)
__global__ __launch_bounds__(256) void k_transpose_x(const double *x, double *xT, int nb, int nx) {
    __shared__ double t[32][33];
    const int b0 = blockIdx.x * 32, q0 = blockIdx.y * 32, tx = threadIdx.x % 32, ty = threadIdx.x / 32;
    for (int i = ty; i < 32; i += 8) {
        const int b = b0 + i, q = q0 + tx;
        if (b < nb && q < nx) t[i][tx] = x[(size_t)b * nx + q];
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) {
        const int q = q0 + i, b = b0 + tx;
        if (b < nb && q < nx) xT[(size_t)q * nb + b] = t[tx][i];
    }
}

hipError_t transpose_x(const double *x, double *xT, int nb, int nx, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_transpose_x, dim3((unsigned)((nb + 31) / 32), (unsigned)((nx + 31) / 32)), dim3(256), 0, st, x,
                       xT, nb, nx);
    return hipGetLastError();
}

template hipError_t launch<2>(int, const grape::DevProblem &, const grape::DevBatch &, hipStream_t);
template hipError_t launch<3>(int, const grape::DevProblem &, const grape::DevBatch &, hipStream_t);
template hipError_t launch<4>(int, const grape::DevProblem &, const grape::DevBatch &, hipStream_t);

}  // namespace grape_walk
