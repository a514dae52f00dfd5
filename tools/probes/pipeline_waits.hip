// Probe: the frame pipeline's cross-queue waits (xrt_abi.hip prepare_frame /
// launch_frame) with spin kernels standing in for k_prep (on a prep stream) and
// the render (on stream k % 2).  One workgroup each, so the GPU is never full:
// any time above the ideal is the waits' own serialisation.
//   A: k_prep with a stop event (hipExtLaunchKernelGGL), the render's stream
//      waits for it (hipStreamWaitEvent), the render with a stop event; the host
//      waits for the set's render four frames back (as the product does).
//   B: as A, without the render's wait for k_prep (not a valid pipeline: the
//      ideal overlap).
//   C: as A, with hipEventRecord instead of stop events on the launches.
//   D: as A, with k_prep launched two frames ahead of its render (the product's
//      prepared-ahead frames) and the wait skipped when the event has already
//      completed (hipEventQuery), as launch_frame does.
// Prints microseconds per frame; a render spins 20 us, a k_prep 10 us, so two
// renders in flight and one k_prep at a time give 10 us per frame at best.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t err_ = (x);                                                             \
        if (err_ != hipSuccess) {                                                          \
            std::printf("%s: %s\n", #x, hipGetErrorString(err_));                          \
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

int main(int argc, char**)
{
    constexpr int kSets = 4;
    int* d;
    CK(hipMalloc(&d, 1024));
    unsigned long long t_prep = 1000, t_render = 2000;           // 10 us, 20 us; argv: 25 us, 42 us
    if (argc > 1) { t_prep = 2500; t_render = 4200; }
    hipStream_t prep, st[2];
    CK(hipStreamCreateWithFlags(&prep, hipStreamNonBlocking));
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ready[kSets], done[kSets];
    for (int i = 0; i < kSets; ++i) {
        CK(hipEventCreate(&ready[i]));
        CK(hipEventCreate(&done[i]));
    }
    const int n = 400;
    const char* names[] = {"A: back-to-back", "B: no render wait (ideal)", "C: A with event records",
                           "D: prepared 2 ahead + query"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            bool valid[kSets] = {};
            const auto t0 = Clock::now();
            if (mode == 3)                            // frames 0 and 1 prepared ahead
                for (int j = 0; j < 2; ++j)
                    hipExtLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, prep, nullptr, ready[j], 0u, t_prep, d);
            for (int k = 0; k < n; ++k) {
                const int s = k % kSets;
                hipStream_t q = st[k % 2];
                if (mode == 3) {
                    const hipError_t e = hipEventQuery(ready[s]);
                    if (e == hipErrorNotReady) CK(hipStreamWaitEvent(q, ready[s], 0));
                    hipExtLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, q, nullptr, done[s], 0u, t_render, d);
                    valid[s] = true;
                    const int a = (k + 2) % kSets;    // frame k + 2's set: its render of frame k - 2
                    if (valid[a]) CK(hipEventSynchronize(done[a]));
                    hipExtLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, prep, nullptr, ready[a], 0u, t_prep, d);
                    continue;
                }
                if (valid[s]) CK(hipEventSynchronize(done[s]));
                if (mode == 2) {
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, prep, t_prep, d);
                    CK(hipEventRecord(ready[s], prep));
                } else {
                    hipExtLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, prep, nullptr, ready[s], 0u, t_prep, d);
                }
                if (mode != 1) CK(hipStreamWaitEvent(q, ready[s], 0));
                if (mode == 2) {
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, q, t_render, d);
                    CK(hipEventRecord(done[s], q));
                } else {
                    hipExtLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, q, nullptr, done[s], 0u, t_render, d);
                }
                valid[s] = true;
            }
            CK(hipDeviceSynchronize());
            const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / n;
            std::printf("%-28s %.1f us per frame\n", names[mode], us);
        }
    }
    return 0;
}
