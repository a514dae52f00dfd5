// Probe: a long kernel on stream s waits (hipStreamWaitEvent) for a short one
// on stream s2 each frame, the frame pipeline of xrt_abi.hip.  How do
// dispatch-attached start/stop events (hipExtLaunchKernelGGL) time the long
// kernel against its true span (in-kernel wall_clock64 stamps), with and
// without a marker between the wait and the launch, and what does each
// variant cost per frame?
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_spin(unsigned long long* stamps, unsigned long long ticks, int slot)
{
    unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {}
    if (threadIdx.x == 0) {
        atomicMin(&stamps[2 * slot], t0);
        atomicMax(&stamps[2 * slot + 1], wall_clock64());
    }
}

int main()
{
    const int iters = 200, sets = 4;
    unsigned long long* st;
    const int slots = 2 * iters + 8;
    CK(hipMalloc(&st, slots * 2 * sizeof(unsigned long long)));
    std::vector<unsigned long long> h(slots * 2);
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi));
    hipEvent_t ready[sets], done[sets], t0[iters], t1[iters], mark, a, b;
    for (int i = 0; i < sets; ++i) { CK(hipEventCreate(&ready[i])); CK(hipEventCreate(&done[i])); }
    for (int i = 0; i < iters; ++i) { CK(hipEventCreate(&t0[i])); CK(hipEventCreate(&t1[i])); }
    CK(hipEventCreate(&mark));
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[] = {"wait + ext start/stop", "wait + marker + ext start/stop", "no wait, ext start/stop",
                           "wait, record t0 before wait", "wait + ext stop only",
                           "one stream: short, long any-order", "one stream: short, long any-order stop only",
                           "long only, ext start/stop"};
    for (unsigned long long long_ticks : {400ull, 4000ull, 140000ull}) {      // 4 us, 40 us, 1.4 ms
        for (int mode = 0; mode < 8; ++mode) {
            for (int i = 0; i < slots; ++i) { h[2 * i] = ~0ull; h[2 * i + 1] = 0; }
            CK(hipMemcpy(st, h.data(), h.size() * 8, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, s));
            for (int it = 0; it < iters; ++it) {
                const int k = it % sets;
                if (it >= sets) CK(hipEventSynchronize(done[k]));          // the set's last render
                if (mode == 5 || mode == 6) {
                    // the short one (the next frame's preparation) first, then this frame's long
                    // one without the barrier bit: it dispatches beside the short one
                    hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, nullptr, nullptr, 0, st, 1500ull,
                                          2 * it + 1);
                    hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, mode == 5 ? t0[it] : nullptr, t1[it],
                                          hipExtAnyOrderLaunch, st, long_ticks, 2 * it);
                    CK(hipEventRecord(done[k], s));
                    continue;
                }
                if (mode == 7) {
                    hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, t0[it], t1[it], 0, st, long_ticks, 2 * it);
                    CK(hipEventRecord(done[k], s));
                    continue;
                }
                hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s2, nullptr, ready[k], 0, st, 1500ull,
                                      2 * it + 1);
                if (mode == 3) CK(hipEventRecord(t0[it], s));
                if (mode != 2) CK(hipStreamWaitEvent(s, ready[k], 0));
                if (mode == 1) CK(hipEventRecord(mark, s));
                hipEvent_t e0 = (mode == 3 || mode == 4) ? nullptr : t0[it];
                hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, e0, t1[it], 0, st, long_ticks, 2 * it);
                CK(hipEventRecord(done[k], s));
            }
            CK(hipEventRecord(b, s));
            CK(hipDeviceSynchronize());
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            double ev = 0, tru = 0, gap = 0;
            int n = 0;
            for (int it = 10; it < iters; ++it) {
                const unsigned long long ls = h[2 * (2 * it)], le = h[2 * (2 * it) + 1];
                const unsigned long long pe = h[2 * (2 * (it - 1)) + 1];
                float evms = 0;
                if (mode != 4 && mode != 6) CK(hipEventElapsedTime(&evms, t0[it], t1[it]));
                else CK(hipEventElapsedTime(&evms, t1[it - 1], t1[it]));
                ev += evms * 1000.0;
                tru += (double)(le - ls) / 100.0;
                gap += (double)(ls - pe) / 100.0;
                ++n;
            }
            printf("long %6.0f us  %-32s per-frame %8.2f us  event %8.2f us  true span %8.2f us  gap %6.2f us\n",
                   long_ticks / 100.0, names[mode], ms * 1000.0 / iters, ev / n, tru / n, gap / n);
        }
    }
    return 0;
}
