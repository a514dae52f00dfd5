// Probe: how long after a kernel ends does the host see it?  A 20 us spin
// kernel with a stop event (as k_prep's prep_done), then the host waits for
// the event by hipEventSynchronize, by spinning on hipEventQuery, or by
// hipStreamSynchronize.  Prints the mean launch-to-return time per method
// (the kernel itself is 20 us).  Modes 4-5: the kernel's last act is a
// system-scope release store of a sequence number into host-mapped memory
// (after an agent-scope fence in mode 5, as a producer of device data would
// need), and the host spins on that word instead of on the event.
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

__global__ void k_spin(unsigned long long ticks, unsigned* flag, unsigned seq, int fence)
{
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {}
    if (flag && threadIdx.x == 0) {
        if (fence) __threadfence();
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreate(&ev));
    const int n = 100;
    unsigned* flag = nullptr;
    CK(hipHostMalloc((void**)&flag, sizeof(unsigned), hipHostMallocCoherent));
    *flag = 0u;
    unsigned seq = 0u;
    const char* names[] = {"hipEventSynchronize", "spin on hipEventQuery", "hipStreamSynchronize",
                           "empty kernel + hipEventSynchronize", "spin on a host-mapped flag",
                           "fence + spin on a host-mapped flag"};
    for (int mode = 0; mode < 6; ++mode) {
        double acc = 0.0;
        for (int i = 0; i < n + 20; ++i) {
            auto t = std::chrono::steady_clock::now();
            const bool fl = mode >= 4;
            ++seq;
            hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, nullptr, ev, 0, mode == 3 ? 0ull : 2000ull,
                                  fl ? flag : nullptr, seq, mode == 5 ? 1 : 0);
            if (fl) {
                volatile unsigned* vf = flag;
                const auto t_spin = std::chrono::steady_clock::now();
                while (*vf != seq) {
                    if (std::chrono::steady_clock::now() - t_spin > std::chrono::seconds(1)) {
                        std::printf("flag never written\n");
                        std::fflush(stdout);
                        break;
                    }
                }
                if (i >= 20) acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
                CK(hipEventSynchronize(ev));
                continue;
            }
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
