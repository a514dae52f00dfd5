// Probe: host CPU cost of one kernel launch on gfx950 under the launch forms
// the render path uses (plain, hipExtLaunchKernel with a stop event, with a
// start/stop pair, plain + hipEventRecord), with a small and a large kernarg
// block.  Prints microseconds of host time per launch (the GPU work is empty).
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
    float f[80];
};

__global__ void k_small(int* p) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1; }
__global__ void k_big(int* p, Big b) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = (int)b.f[3]; }

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1, ed;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&ed, hipEventDisableTiming));
    int* d;
    CK(hipMalloc(&d, 64));
    Big b = {};
    const int n = 2000;
    const char* names[] = {"plain small", "plain big", "ext stop-event big", "ext start+stop big",
                           "plain big + hipEventRecord(timing)", "plain big + hipEventRecord(no timing)"};
    for (int mode = 0; mode < 6; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            double acc = 0.0;
            for (int i = 0; i < n; ++i) {
                auto t = std::chrono::steady_clock::now();
                switch (mode) {
                case 0: hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d); break;
                case 1: hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, d, b); break;
                case 2: hipExtLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, nullptr, e1, 0, d, b); break;
                case 3: hipExtLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, e0, e1, 0, d, b); break;
                case 4:
                    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, d, b);
                    CK(hipEventRecord(e1, s));
                    break;
                default:
                    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, d, b);
                    CK(hipEventRecord(ed, s));
                    break;
                }
                acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
                if ((i & 7) == 7) CK(hipStreamSynchronize(s));   // a shallow queue, as the render path keeps
            }
            CK(hipStreamSynchronize(s));
            if (rep) std::printf("%-40s %.2f us of host time per launch call\n", names[mode], acc * 1e6 / n);
        }
    }
    return 0;
}
