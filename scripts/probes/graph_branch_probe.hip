// Probe: do parallel branches of a HIP graph run concurrently on this runtime?  Two kernels that
// each busy-wait ~T us (s_memrealtime, 100 MHz) as (a) one stream-captured chain, (b) two child
// graphs on parallel branches of a manually built graph.  Prints the replay time of each.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(long long ticks, int *out) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));                    \
            return 1;                                                                \
        }                                                                            \
    } while (0)

static double replay_us(hipGraphExec_t ex, hipStream_t st, int n) {
    (void)hipGraphLaunch(ex, st);
    (void)hipStreamSynchronize(st);
    auto t = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
        (void)hipGraphLaunch(ex, st);
        (void)hipStreamSynchronize(st);
    }
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / n;
}

int main() {
    int *d;
    CK(hipMalloc(&d, 1024 * sizeof(int)));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const long long ticks = 5000;  // 50 us at 100 MHz
    // (a) serial chain by capture
    hipGraph_t ga;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, ticks, d);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, ticks, d + 1);
    CK(hipStreamEndCapture(st, &ga));
    hipGraphExec_t ea;
    CK(hipGraphInstantiate(&ea, ga, nullptr, nullptr, 0));
    // (b) two child graphs on parallel branches
    hipGraph_t c1, c2, gb;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, ticks, d + 2);
    CK(hipStreamEndCapture(st, &c1));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, ticks, d + 3);
    CK(hipStreamEndCapture(st, &c2));
    CK(hipGraphCreate(&gb, 0));
    hipGraphNode_t n1, n2;
    CK(hipGraphAddChildGraphNode(&n1, gb, nullptr, 0, c1));
    CK(hipGraphAddChildGraphNode(&n2, gb, nullptr, 0, c2));
    hipGraphExec_t eb;
    CK(hipGraphInstantiate(&eb, gb, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep)
        printf("serial chain %.1f us, parallel child graphs %.1f us\n", replay_us(ea, st, 200), replay_us(eb, st, 200));
    CK(hipGraphExecDestroy(ea));
    CK(hipGraphExecDestroy(eb));
    CK(hipGraphDestroy(ga));
    CK(hipGraphDestroy(gb));
    CK(hipGraphDestroy(c1));
    CK(hipGraphDestroy(c2));
    CK(hipStreamDestroy(st));
    CK(hipFree(d));
    printf("probe done\n");
    return 0;
}
