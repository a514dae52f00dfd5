// Probe: does a hipGraph run two independent kernel nodes at once on gfx950?
// Two one-workgroup kernels that each spin for ~20 us (s_memrealtime, 100 MHz):
// launched as a graph with no edge between them, as a graph with an edge, and
// on two streams (joined after every pair, and free).  If the no-edge graph takes ~20 us per replay the runtime
// overlaps the branches (a frame graph could keep k_prep beside the previous
// render); ~40 us means it serialises them.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void k_spin(unsigned long long ticks, int* out)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

using Clock = std::chrono::steady_clock;

int main()
{
    int* d;
    CK(hipMalloc(&d, 1024));
    unsigned long long ticks = 2000;          // 20 us at 100 MHz
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipGraphExec_t ex[2];
    for (int edge = 0; edge < 2; ++edge) {
        hipGraph_t g;
        CK(hipGraphCreate(&g, 0));
        void* args[] = {&ticks, &d};
        hipKernelNodeParams kp = {};
        kp.func = reinterpret_cast<void*>(k_spin);
        kp.gridDim = dim3(1);
        kp.blockDim = dim3(64);
        kp.kernelParams = args;
        hipGraphNode_t a, b;
        CK(hipGraphAddKernelNode(&a, g, nullptr, 0, &kp));
        CK(hipGraphAddKernelNode(&b, g, edge ? &a : nullptr, edge ? 1 : 0, &kp));
        CK(hipGraphInstantiate(&ex[edge], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    const int n = 200;
    const char* names[] = {"graph, no edge", "graph, edge", "two streams", "two streams, free"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            const auto t0 = Clock::now();
            for (int i = 0; i < n; ++i) {
                if (mode < 2) {
                    CK(hipGraphLaunch(ex[mode], s0));
                } else if (mode == 3) {               // no joins: each stream runs its own chain
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s0, ticks, d);
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, d);
                } else {
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s0, ticks, d);
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, d);
                    // keep the pairs in step, as a graph replay is
                    hipEvent_t ev;
                    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                    CK(hipEventRecord(ev, s1));
                    CK(hipStreamWaitEvent(s0, ev, 0));
                    CK(hipEventRecord(ev, s0));
                    CK(hipStreamWaitEvent(s1, ev, 0));
                    CK(hipEventDestroy(ev));
                }
            }
            CK(hipDeviceSynchronize());
            const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / n;
            std::printf("%-16s %.1f us per pair (one kernel: 20 us)\n", names[mode], us);
        }
    }
    return 0;
}
