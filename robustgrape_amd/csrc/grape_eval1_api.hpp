// grape_eval1_api.hpp -- host side of the one-workgroup-per-evaluation kernel (grape_eval1.hip)
// for latency-bound calls of the Rydberg sector layout.
#pragma once
#include <hip/hip_runtime.h>

#include "grape_kernels.hpp"
#include "grape_projector_api.hpp"

namespace grape_eval1 {
constexpr int kLanes = 256;                // chunks per sector class (lanes of the class's waves)
constexpr int kBlock = 2 * kLanes + 64;    // both classes' lanes + the head wave
constexpr int kMaxNt = 2048, kMaxNa = 4;   // steps and x_add entries it serves (LDS budget)

struct Args {
    grape::DevProblem PA;         // class A: one 3-level sector (phase-covariant)
    grape::DevProblem PB;         // class B: two 2-level sectors (phase-covariant; twins or not)
    grape_proj::SectorHead H;     // the full problem's target, weights, sector slots, fixed levels
    const grape::cd *EtA, *EtB;   // E~ = exp(-i dt H_w(0)) of A's sector and B's sector(s), row-major
    const double *x;              // [nb][nx]  (device memory or mapped pinned host memory)
    double *F, *Fdx;              // [nb], [nb][nx]
    int L, nch;                   // steps per chunk, chunks (<= kLanes)
    int a_first;                  // 1: class A is the plan's class 0 (F_dx sums class 0, then class 1)
    long long *trace;             // optional: workgroup 0's phase clocks [0..9], wall clocks [14], [15]
    const unsigned char *tab;     // the plan's table blob (tab_build), 16-B aligned
};

// Which plans it serves: both classes phase-covariant chunk walks of the pair layout
// (grape_walk_api.hpp pair_ok), one control per step, no error sources, x_add outside H, the
// diagonal head, at most kMaxNt steps and kMaxNa x_add entries.
bool eligible(const grape::DevProblem &PA, const grape::DevProblem &PB, const grape_proj::SectorHead &H);
// E~ of class A's sector and class B's (one sector when twins), once per plan (k_gauge_tilde: the
// walks' own gauge_base arithmetic, hence their bits); scr: 2 * 4 * 16 complex of scratch
hipError_t prepare(const grape::DevProblem &PA, const grape::DevProblem &PB, grape::cd *EtA, grape::cd *EtB,
                   grape::cd *scr, hipStream_t st);
// the plan's table blob (E~, charges, sector slots, W, fixed levels, target terms and diagonals):
// its size, and its one-time build from the plan's device tables (after prepare)
size_t tab_bytes(const grape::DevProblem &PA, const grape::DevProblem &PB, const grape_proj::SectorHead &H);
hipError_t tab_build(const Args &A, unsigned char *blob, hipStream_t st);
// one workgroup per evaluation of the batch: F and F_dx (controls and x_add) of nb evaluations
hipError_t launch(Args A, int nb, hipStream_t st);
}  // namespace grape_eval1
