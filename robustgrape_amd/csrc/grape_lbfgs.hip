// grape_lbfgs.hip -- the L-BFGS two-loop recursion of the batched restart optimiser
// (robustgrape_amd/optimize.py, lbfgs_batched) as one launch per iteration.
//
// The optimiser replaces Optim.jl's LBFGS driving calculate_fidelity_and_derivatives
// (src/FidelityCalculations.jl:199-217).  All restarts advance together; their
// histories are ring buffers S, Y [m][R][n] and rho [m][R].  In torch the recursion
// is ~160 small launches per iteration (2 m gathers, dots and axpys); here one
// workgroup per restart walks its own history: the q vector lives in the output
// row D[r] (each thread owns the same elements in every pass, so only the dot
// products need the workgroup barrier).  HBM-bound: reads 2 m n doubles of
// history twice per restart.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "grape.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxHistory = 64;

// Sum over the workgroup; every thread gets the result.
__device__ __forceinline__ double block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();  // red[] free (previous reduction consumed)
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    return s;
}

// D[r] = -H_r g[r]: H_r the L-BFGS inverse-Hessian estimate of restart r from its
// newest hist[r] pairs (ring buffer, newest at head[r] - 1), scaled by gamma[r].
__global__ __launch_bounds__(kThreads) void k_lbfgs_dir(int R, int n, int m, const double *__restrict__ S,
                                                        const double *__restrict__ Y,
                                                        const double *__restrict__ rho,
                                                        const int64_t *__restrict__ head,
                                                        const int64_t *__restrict__ hist,
                                                        const double *__restrict__ gamma,
                                                        const double *__restrict__ g, double *__restrict__ D) {
    __shared__ double red[kThreads / 64];
    __shared__ double alpha[kMaxHistory];
    const int r = blockIdx.x;  // grid == R
    const size_t row = (size_t)r * n;
    double *q = D + row;
    for (int i = threadIdx.x; i < n; i += kThreads) q[i] = -g[row + i];
    const int h = (int)hist[r], hd = (int)head[r];
    for (int j = 0; j < h; ++j) {  // newest first
        const int slot = ((hd - 1 - j) % m + m) % m;
        const double *s = S + ((size_t)slot * R) * n + row, *y = Y + ((size_t)slot * R) * n + row;
        double part = 0.0;
        for (int i = threadIdx.x; i < n; i += kThreads) part += s[i] * q[i];
        const double a = rho[(size_t)slot * R + r] * block_sum(part, red);
        if (threadIdx.x == 0) alpha[j] = a;
        for (int i = threadIdx.x; i < n; i += kThreads) q[i] -= a * y[i];
    }
    const double gm = gamma[r];
    for (int i = threadIdx.x; i < n; i += kThreads) q[i] *= gm;
    __syncthreads();  // alpha[] visible
    for (int j = h - 1; j >= 0; --j) {  // oldest first
        const int slot = ((hd - 1 - j) % m + m) % m;
        const double *s = S + ((size_t)slot * R) * n + row, *y = Y + ((size_t)slot * R) * n + row;
        double part = 0.0;
        for (int i = threadIdx.x; i < n; i += kThreads) part += y[i] * q[i];
        const double c = alpha[j] - rho[(size_t)slot * R + r] * block_sum(part, red);
        for (int i = threadIdx.x; i < n; i += kThreads) q[i] += c * s[i];
    }
}

}  // namespace

extern "C" int grape_lbfgs_direction(int R, int n, int m, const double *S, const double *Y, const double *rho,
                                     const int64_t *head, const int64_t *hist, const double *gamma,
                                     const double *g, double *D, void *stream) {
    if (R < 0 || n < 1 || m < 1 || m > kMaxHistory) return GRAPE_ERR_INVALID;
    if (R == 0) return GRAPE_OK;
    if (!S || !Y || !rho || !head || !hist || !gamma || !g || !D) return GRAPE_ERR_INVALID;
    hipLaunchKernelGGL(k_lbfgs_dir, dim3(R), dim3(kThreads), 0, static_cast<hipStream_t>(stream), R, n, m, S, Y,
                       rho, head, hist, gamma, g, D);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}
