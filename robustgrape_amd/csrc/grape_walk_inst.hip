// grape_walk_inst.hip -- the chunk-walk kernels (grape_walk.hpp) for D = 2 .. kWalkMaxD and their
// launchers; built with -mllvm -disable-machine-licm (robustgrape_amd/build.py).
#include "grape_walk.hpp"
#include "grape_walk_api.hpp"

namespace grape_walk {

template <int D>
hipError_t launch(int stage, const grape::DevProblem &P, const grape::DevBatch &B, hipStream_t st) {
    const int ns = P.nsec > 1 ? P.nsec : 1;
    const long lanes = (long)(B.nb / ns) * P.nchunks;
    if (lanes <= 0) return hipSuccess;
    const dim3 grid((unsigned)((lanes + grape::kWalkBlock - 1) / grape::kWalkBlock), (unsigned)ns);
    if (stage == 0)
        hipLaunchKernelGGL(grape::k_walk_fwd<D>, grid, dim3(grape::kWalkBlock), 0, st, P, B);
    else
        hipLaunchKernelGGL(grape::k_walk_grad<D>, grid, dim3(grape::kWalkBlock), 0, st, P, B);
    return hipGetLastError();
}

template hipError_t launch<2>(int, const grape::DevProblem &, const grape::DevBatch &, hipStream_t);
template hipError_t launch<3>(int, const grape::DevProblem &, const grape::DevBatch &, hipStream_t);
template hipError_t launch<4>(int, const grape::DevProblem &, const grape::DevBatch &, hipStream_t);

}  // namespace grape_walk
