// Probe: how long after a kernel ends does the host see it?  A 20 us spin
// kernel with a stop event (as k_prep's prep_done), then the host waits for
// the event by hipEventSynchronize, by spinning on hipEventQuery, or by
// hipStreamSynchronize.  Prints the mean launch-to-return time per method
// (the kernel itself is 20 us).
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

__global__ void k_spin(unsigned long long ticks)
{
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {}
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreate(&ev));
    const int n = 100;
    const char* names[] = {"hipEventSynchronize", "spin on hipEventQuery", "hipStreamSynchronize",
                           "empty kernel + hipEventSynchronize"};
    for (int mode = 0; mode < 4; ++mode) {
        double acc = 0.0;
        for (int i = 0; i < n + 20; ++i) {
            auto t = std::chrono::steady_clock::now();
            hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, nullptr, ev, 0, mode == 3 ? 0ull : 2000ull);
            if (mode == 1) {
                hipError_t e;
                const auto t_spin = std::chrono::steady_clock::now();
                while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
                    if (std::chrono::steady_clock::now() - t_spin > std::chrono::seconds(1)) {
                        std::printf("hipEventQuery never ready\n");
                        std::fflush(stdout);
                        CK(hipEventSynchronize(ev));
                        break;
                    }
                }
            } else if (mode == 2) {
                CK(hipStreamSynchronize(s));
            } else {
                CK(hipEventSynchronize(ev));
            }
            if (i >= 20) acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        }
        std::printf("%-36s %.2f us launch-to-return (kernel %s)\n", names[mode], acc * 1e6 / n,
                    mode == 3 ? "empty" : "20 us");
        std::fflush(stdout);
    }
    return 0;
}
