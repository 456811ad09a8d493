// Probe: what crashed round 3's captured fork/join?  Round 3 forked the second
// sector class onto an auxiliary stream INSIDE graph capture (event record on the capturing stream,
// wait on the aux stream, work on aux, event record on aux, wait on the main stream), then kept the
// SAME two event objects for the eager (non-graph) fork of larger calls, and destroyed the captured
// hipGraph_t right after instantiation; replays "crashed the runtime intermittently".  This probe
// replays that pattern and its variants in one process each (mode argument) and reports the first
// HIP error or the iteration count reached:
//   shared    : capture fork/join with events E1/E2, then alternate graph replays and eager fork/join
//               with the SAME E1/E2 (round 3's design)
//   separate  : the same, the eager fork/join uses its own events E3/E4 (capture events only in capture)
//   capture   : graph replays only (captured fork/join, no eager use of any event)
//   eager     : eager fork/join only (no capture)
//   nocapfork : the graph captures one stream (no events), the eager path forks with E1/E2 (round 4)
//   cache     : the engine's life cycle: graphs captured lazily per "batch size" (10 sizes cycling
//               through a cache of 8 execs, the oldest destroyed and re-captured), each capture
//               forking with E1/E2 after eager fork/joins that used the same E1/E2, one
//               synchronize per call as grape_fidelity_grad does
// Kernels are one wave each writing a counter slot in range: no memory fault is possible.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void bump(int *c, int slot) {
    if (threadIdx.x == 0) atomicAdd(c + slot, 1);
}

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            printf("FAIL at iteration %d: %s -> %s\n", it, #x, hipGetErrorString(e_));              \
            fflush(stdout);                                                                          \
            return 2;                                                                                \
        }                                                                                            \
    } while (0)

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "shared";
    const int iters = argc > 2 ? atoi(argv[2]) : 20000;
    int it = -1;
    int *c;
    CK(hipMalloc(&c, 64 * sizeof(int)));
    CK(hipMemset(c, 0, 64 * sizeof(int)));
    hipStream_t st, aux;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    hipEvent_t e1, e2, e3, e4;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e3, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e4, hipEventDisableTiming));
    const bool cap_fork = strcmp(mode, "nocapfork") != 0;
    const bool use_graph = strcmp(mode, "eager") != 0;
    const bool use_eager = strcmp(mode, "capture") != 0;
    hipEvent_t f1 = strcmp(mode, "separate") == 0 ? e3 : e1, f2 = strcmp(mode, "separate") == 0 ? e4 : e2;
    if (strcmp(mode, "cache") == 0) {
        constexpr int kCache = 8, kSizes = 10;
        int sz[kCache];
        hipGraphExec_t cx[kCache];
        int n = 0;
        long long expect[3] = {0, 0, 0};
        for (it = 0; it < iters; ++it) {
            const int size = it % kSizes;
            hipGraphExec_t g = nullptr;
            for (int j = 0; j < n; ++j)
                if (sz[j] == size) g = cx[j];
            if (!g) {
                hipGraph_t gr;
                CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
                hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 0);
                CK(hipEventRecord(e1, st));
                CK(hipStreamWaitEvent(aux, e1, 0));
                hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, aux, c, 1);
                CK(hipEventRecord(e2, aux));
                CK(hipStreamWaitEvent(st, e2, 0));
                hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 2);
                CK(hipStreamEndCapture(st, &gr));
                CK(hipGraphInstantiate(&g, gr, nullptr, nullptr, 0));
                CK(hipGraphDestroy(gr));
                if (n == kCache) {  // evict the oldest, as the engine's graph cache does
                    CK(hipGraphExecDestroy(cx[0]));
                    for (int j = 1; j < n; ++j) {
                        cx[j - 1] = cx[j];
                        sz[j - 1] = sz[j];
                    }
                    --n;
                }
                cx[n] = g;
                sz[n++] = size;
            }
            CK(hipGraphLaunch(g, st));
            for (int k = 0; k < 3; ++k) ++expect[k];
            CK(hipStreamSynchronize(st));
            if (it % 3 == 1) {  // an eager large call with the same events
                hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 0);
                CK(hipEventRecord(e1, st));
                CK(hipStreamWaitEvent(aux, e1, 0));
                hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, aux, c, 1);
                CK(hipEventRecord(e2, aux));
                CK(hipStreamWaitEvent(st, e2, 0));
                hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 2);
                for (int k = 0; k < 3; ++k) ++expect[k];
                CK(hipStreamSynchronize(st));
            }
        }
        CK(hipStreamSynchronize(aux));
        int h[3];
        CK(hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost));
        const bool ok = h[0] == (int)expect[0] && h[1] == (int)expect[1] && h[2] == (int)expect[2];
        printf("mode %-9s iterations %d counters %d %d %d expected %lld %lld %lld %s\n", mode, it, h[0], h[1], h[2],
               expect[0], expect[1], expect[2], ok ? "OK" : "MISMATCH");
        for (int j = 0; j < n; ++j) (void)hipGraphExecDestroy(cx[j]);
        return ok ? 0 : 3;
    }
    hipGraphExec_t ex = nullptr;
    if (use_graph) {  // capture: main kernel, fork, aux kernel, join, main kernel
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 0);
        if (cap_fork) {
            CK(hipEventRecord(e1, st));
            CK(hipStreamWaitEvent(aux, e1, 0));
            hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, aux, c, 1);
            CK(hipEventRecord(e2, aux));
            CK(hipStreamWaitEvent(st, e2, 0));
        } else {
            hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 1);
        }
        hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 2);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));  // as round 3: the exec is independent of g
    }
    long long expect[3] = {0, 0, 0};
    for (it = 0; it < iters; ++it) {
        if (use_graph) {
            CK(hipGraphLaunch(ex, st));
            for (int k = 0; k < 3; ++k) ++expect[k];
        }
        if (use_eager && (it % 3 == 1)) {  // an eager "large call" between replays
            hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 0);
            CK(hipEventRecord(f1, st));
            CK(hipStreamWaitEvent(aux, f1, 0));
            hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, aux, c, 1);
            CK(hipEventRecord(f2, aux));
            CK(hipStreamWaitEvent(st, f2, 0));
            hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st, c, 2);
            for (int k = 0; k < 3; ++k) ++expect[k];
        }
        if (it % 64 == 63) CK(hipStreamSynchronize(st));
    }
    CK(hipStreamSynchronize(st));
    CK(hipStreamSynchronize(aux));
    int h[3];
    CK(hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost));
    const bool ok = h[0] == (int)expect[0] && h[1] == (int)expect[1] && h[2] == (int)expect[2];
    printf("mode %-9s iterations %d counters %d %d %d expected %lld %lld %lld %s\n", mode, it, h[0], h[1], h[2], expect[0],
           expect[1], expect[2], ok ? "OK" : "MISMATCH");
    if (ex) (void)hipGraphExecDestroy(ex);
    return ok ? 0 : 3;
}
