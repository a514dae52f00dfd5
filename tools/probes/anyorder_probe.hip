// Probe: does hipExtAnyOrderLaunch let a small kernel overlap the previous
// full-chip kernel on the same stream on gfx950, and what does the per-frame
// cost of [long, short] look like under three orderings?
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_spin(unsigned long long* stamps, unsigned long long ticks, int slot) {
  unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {}
  if (threadIdx.x == 0) {
    atomicMin(&stamps[2 * slot], t0);
    atomicMax(&stamps[2 * slot + 1], wall_clock64());
  }
}

int main(int argc, char** argv) {
  int iters = 200;
  unsigned long long* st;
  int slots = 2 * iters + 8;
  CK(hipMalloc(&st, slots * 2 * sizeof(unsigned long long)));
  std::vector<unsigned long long> h(slots * 2);
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int lo, hi; CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi));
  hipEvent_t ev[2], done[2], a, b;
  unsigned evflags = hipEventDisableTiming;
  if (argc > 1 && argv[1][0] == 'd') evflags |= hipEventReleaseToDevice;
  if (argc > 1 && argv[1][0] == 'n') evflags |= hipEventDisableSystemFence;
  printf("event flags 0x%x\n", evflags);
  for (int i = 0; i < 2; ++i) { CK(hipEventCreateWithFlags(&ev[i], evflags)); CK(hipEventCreateWithFlags(&done[i], evflags)); }
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipEvent_t tev[4], tdone[4];
  for (int i = 0; i < 4; ++i) { CK(hipEventCreate(&tev[i])); CK(hipEventCreate(&tdone[i])); }
  const unsigned long long long_ticks = 5000, short_ticks = 500;  // 50 us, 5 us at 100 MHz
  const char* names[] = {"same-stream barrier", "same-stream anyorder", "prep-stream+event", "long only", "short only", "long+record", "long+wait(s2 short)", "long ext stop-event", "prep-stream ext events", "ext, no done wait", "ext, 4 sets, wait even", "host-synced prep, K=4", "host-synced, short prep"};
  for (int mode = 0; mode < 13; ++mode) {
    for (int i = 0; i < slots; ++i) { h[2 * i] = ~0ull; h[2 * i + 1] = 0; }
    CK(hipMemcpy(st, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, s));
    for (int it = 0; it < iters; ++it) {
      if (mode == 0 || mode == 1 || mode == 4) {
        if (mode != 4)
          hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, nullptr, nullptr, mode == 1 ? hipExtAnyOrderLaunch : 0, st, short_ticks, 2 * it + 1);
        else
          hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, nullptr, nullptr, 0, st, short_ticks, 2 * it + 1);
        if (mode != 4)
          hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, nullptr, nullptr, 0, st, long_ticks, 2 * it);
      } else if (mode == 2) {
        int k = it & 1;
        if (it >= 2) CK(hipStreamWaitEvent(s2, done[k], 0));
        hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s2, st, short_ticks, 2 * it + 1);
        CK(hipEventRecord(ev[k], s2));
        CK(hipStreamWaitEvent(s, ev[k], 0));
        hipLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, st, long_ticks, 2 * it);
        CK(hipEventRecord(done[k], s));
      } else if (mode == 7) {
        hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, nullptr, tdone[it & 1], 0, st, long_ticks, 2 * it);
      } else if (mode == 8) {
        int k = it & 1;
        if (it >= 2) CK(hipStreamWaitEvent(s2, tdone[k], 0));
        hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s2, nullptr, tev[k], 0, st, short_ticks, 2 * it + 1);
        CK(hipStreamWaitEvent(s, tev[k], 0));
        hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, nullptr, tdone[k], 0, st, long_ticks, 2 * it);
      } else if (mode == 9) {
        int k = it & 1;
        hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s2, nullptr, tev[k], 0, st, short_ticks, 2 * it + 1);
        CK(hipStreamWaitEvent(s, tev[k], 0));
        hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, nullptr, nullptr, 0, st, long_ticks, 2 * it);
      } else if (mode == 10) {
        int k = it & 3;
        // done events only on even frames; prep(it) waits the newest even frame <= it-2 (covers it-4)
        if (it >= 2) { int j = (it - 2) & ~1; CK(hipStreamWaitEvent(s2, tdone[j & 3], 0)); }
        hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s2, nullptr, tev[k], 0, st, short_ticks, 2 * it + 1);
        CK(hipStreamWaitEvent(s, tev[k], 0));
        hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, nullptr, (it & 1) ? nullptr : tdone[k], 0, st, long_ticks, 2 * it);
      } else if (mode == 11 || mode == 12) {
        int k = it & 3;
        if (it >= 4) CK(hipEventSynchronize(tdone[k]));      // render(it-4) complete
        hipExtLaunchKernelGGL(k_spin, dim3(mode == 11 ? 2048 : 64), dim3(256), 0, s2, nullptr, tev[k], 0, st,
                              mode == 11 ? 2000ull : short_ticks, 2 * it + 1);
        CK(hipEventSynchronize(tev[k]));                     // preparation complete
        hipExtLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, nullptr, tdone[k], 0, st, long_ticks, 2 * it);
      } else if (mode == 5) {
        hipLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, st, long_ticks, 2 * it);
        CK(hipEventRecord(done[it & 1], s));
      } else if (mode == 6) {
        hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s2, st, short_ticks, 2 * it + 1);
        CK(hipEventRecord(ev[it & 1], s2));
        CK(hipStreamWaitEvent(s, ev[it & 1], 0));
        hipLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, st, long_ticks, 2 * it);
      } else {
        hipLaunchKernelGGL(k_spin, dim3(8192), dim3(256), 0, s, st, long_ticks, 2 * it);
      }
    }
    CK(hipEventRecord(b, s));
    CK(hipStreamSynchronize(s));
    CK(hipDeviceSynchronize());
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    // overlap of short(it) with long(it-1), and gap long(it-1).end -> long(it).start (us)
    double gap = 0, ovl = 0, llen = 0; int n = 0;
    for (int it = 10; it < iters; ++it) {
      unsigned long long le_prev = h[2 * (2 * (it - 1)) + 1], ls = h[2 * (2 * it)], le = h[2 * (2 * it) + 1];
      unsigned long long ss = h[2 * (2 * it + 1)];
      if (mode == 4) { ls = ss; le = h[2 * (2 * it + 1) + 1]; le_prev = h[2 * (2 * (it - 1) + 1) + 1]; }
      gap += (double)(ls - le_prev) / 100.0;
      llen += (double)(le - ls) / 100.0;
      if (mode <= 2 || mode >= 6) ovl += ((double)le_prev - (double)ss) / 100.0;
      ++n;
    }
    printf("%-22s per-iter %.2f us  gap long->long %.2f us  long len %.2f us  short.start before prev long.end %.2f us\n",
           names[mode], ms * 1000.0 / iters, gap / n, llen / n, ovl / n);
  }
  return 0;
}
