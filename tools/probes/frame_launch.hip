// Probe: host cost per frame of the render path's launch pattern against a
// hipGraph replay of the same two kernels.  Kernels are empty (one workgroup),
// so the rate is the host's.  A: per frame, the set-reuse wait, k_prep on the
// prep stream with a stop event, an event query + stream wait, the render with
// a stop event (xrt_abi.hip prepare_frame / launch_frame).  B: one graph per
// buffer set (k_prep node -> render node), hipGraphLaunch on stream k % 2.
// C: both kernels plain on stream k % 2 (stream order is the dependency), no
// events.  D: A without the events on the launches (plain launches, an event
// record without timing after each).  E: A with one stream for the renders.
// Prints microseconds per frame.
#include <hip/hip_ext.h>
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

struct Big {
    float f[72];
};

__global__ void k_prep_like(int* p, Big b) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = (int)b.f[3]; }
__global__ void k_render_like(int* p, Big b) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[1] = (int)b.f[5]; }

using Clock = std::chrono::steady_clock;

int main()
{
    constexpr int kSets = 4;
    hipStream_t st[2], prep;
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&prep, hipStreamNonBlocking));
    hipEvent_t ready[kSets], done[kSets];
    for (int i = 0; i < kSets; ++i) {
        CK(hipEventCreate(&ready[i]));
        CK(hipEventCreate(&done[i]));
    }
    int* d;
    CK(hipMalloc(&d, 64 * kSets));
    Big b = {};
    // graphs, one per set
    hipGraphExec_t exec[kSets];
    for (int i = 0; i < kSets; ++i) {
        hipGraph_t g;
        CK(hipGraphCreate(&g, 0));
        int* p = d + 16 * i;
        void* args[] = {&p, &b};
        hipKernelNodeParams kp = {};
        kp.blockDim = dim3(64);
        kp.gridDim = dim3(1);
        kp.kernelParams = args;
        kp.func = reinterpret_cast<void*>(k_prep_like);
        hipGraphNode_t a, r;
        CK(hipGraphAddKernelNode(&a, g, nullptr, 0, &kp));
        kp.func = reinterpret_cast<void*>(k_render_like);
        CK(hipGraphAddKernelNode(&r, g, &a, 1, &kp));
        CK(hipGraphInstantiate(&exec[i], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    const int n = 4000;
    hipEvent_t rdy_nt[kSets], done_nt[kSets];
    for (int i = 0; i < kSets; ++i) {
        CK(hipEventCreateWithFlags(&rdy_nt[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&done_nt[i], hipEventDisableTiming));
    }
    const char* names[] = {"A: launches + events", "B: graph per set", "C: plain, stream order", "D: plain + records",
                           "E: A, one render stream"};
    for (int mode = 0; mode < 5; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            const auto t0 = Clock::now();
            for (int k = 0; k < n; ++k) {
                const int s = k % kSets;
                hipStream_t q = st[k % 2];
                int* p = d + 16 * s;
                if (mode == 4) q = st[0];
                if (mode == 0 || mode == 4) {
                    if (k >= kSets) CK(hipEventSynchronize(done[s]));
                    hipExtLaunchKernelGGL(k_prep_like, dim3(1), dim3(64), 0, prep, nullptr, ready[s], 0u, p, b);
                    const hipError_t e = hipEventQuery(ready[s]);
                    if (e == hipErrorNotReady) CK(hipStreamWaitEvent(q, ready[s], 0));
                    hipExtLaunchKernelGGL(k_render_like, dim3(1), dim3(64), 0, q, nullptr, done[s], 0u, p, b);
                } else if (mode == 1) {
                    CK(hipGraphLaunch(exec[s], q));
                } else if (mode == 2) {
                    hipLaunchKernelGGL(k_prep_like, dim3(1), dim3(64), 0, q, p, b);
                    hipLaunchKernelGGL(k_render_like, dim3(1), dim3(64), 0, q, p, b);
                } else {
                    if (k >= kSets) CK(hipEventSynchronize(done_nt[s]));
                    hipLaunchKernelGGL(k_prep_like, dim3(1), dim3(64), 0, prep, p, b);
                    CK(hipEventRecord(rdy_nt[s], prep));
                    CK(hipStreamWaitEvent(q, rdy_nt[s], 0));
                    hipLaunchKernelGGL(k_render_like, dim3(1), dim3(64), 0, q, p, b);
                    CK(hipEventRecord(done_nt[s], q));
                }
            }
            const auto t1 = Clock::now();
            CK(hipDeviceSynchronize());
            const auto t2 = Clock::now();
            std::printf("%-28s enqueue %.2f us/frame, to completion %.2f us/frame\n",
                        names[mode],
                        std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                        std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
        }
    }
    return 0;
}
