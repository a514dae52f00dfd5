// Probe: ways to bring a rendered frame's three planes (image f32, L-buffer
// f32, u8: 9 B per pixel) from HBM into caller-owned host memory, as the
// host-buffer entry xrt_render_rows must.  Per method, the mean over reps of
// the wall time to land every byte in the destination, for a destination that
// is fresh (mmap'd, never touched: the first frame into a new Image / numpy
// array) and one already touched (a caller that renders into the same buffer
// again).  Usage: d2h_probe [pixels] (default 2048^2).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count() * 1e3; }

static char* fresh(size_t n)
{
    void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) std::exit(2);
    return (char*)p;
}

static void par_copy(char* dst, const char* src, size_t n, int threads)
{
    if (threads <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const size_t b = std::min(n, t * per), e = std::min(n, b + per);
        th.emplace_back([=] { std::memcpy(dst + b, src + b, e - b); });
    }
    for (auto& x : th) x.join();
}

int main(int argc, char** argv)
{
    const size_t px = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2048ull * 2048ull;
    const size_t sizes[3] = {4 * px, 4 * px, px};
    const size_t total = 9 * px;
    const int reps = 4;
    std::printf("planes: %.1f MB in all\n", total / 1e6);
    auto t = Clock::now();
    CK(hipFree(nullptr));
    std::printf("runtime init %.2f ms\n", ms_since(t));
    char* d[3];
    for (int k = 0; k < 3; ++k) {
        t = Clock::now();
        CK(hipMalloc(&d[k], sizes[k]));
        std::printf("hipMalloc plane %d (%.1f MB): %.3f ms\n", k, sizes[k] / 1e6, ms_since(t));
        CK(hipMemset(d[k], 0x3f, sizes[k]));
    }
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    // page-fault cost alone: touch fresh memory
    {
        double acc = 0;
        for (int r = 0; r < reps; ++r) {
            char* h = fresh(total);
            t = Clock::now();
            std::memset(h, 1, total);
            acc += ms_since(t);
            munmap(h, total);
        }
        std::printf("%-58s %8.3f ms\n", "first touch of fresh memory (memset)", acc / reps);
    }
    auto run = [&](const char* name, auto&& fn) {
        for (int touched = 0; touched < 2; ++touched) {
            double acc = 0;
            for (int r = 0; r < reps + 1; ++r) {
                char* h[3];
                for (int k = 0; k < 3; ++k) {
                    h[k] = fresh(sizes[k]);
                    if (touched) std::memset(h[k], 1, sizes[k]);
                }
                t = Clock::now();
                fn(h);
                const double ms = ms_since(t);
                if (r) acc += ms;
                for (int k = 0; k < 3; ++k) munmap(h[k], sizes[k]);
            }
            std::printf("%-50s %-7s %8.3f ms  (%.1f GB/s)\n", name, touched ? "touched" : "fresh", acc / reps,
                        total / (acc / reps) / 1e6);
            std::fflush(stdout);
        }
    };
    run("pageable hipMemcpy x3", [&](char** h) {
        for (int k = 0; k < 3; ++k) CK(hipMemcpy(h[k], d[k], sizes[k], hipMemcpyDeviceToHost));
    });
    run("pageable hipMemcpyAsync x3 + sync", [&](char** h) {
        for (int k = 0; k < 3; ++k) CK(hipMemcpyAsync(h[k], d[k], sizes[k], hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    });
    run("hipHostRegister + DMA + unregister", [&](char** h) {
        for (int k = 0; k < 3; ++k) CK(hipHostRegister(h[k], sizes[k], hipHostRegisterDefault));
        for (int k = 0; k < 3; ++k) CK(hipMemcpyAsync(h[k], d[k], sizes[k], hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        for (int k = 0; k < 3; ++k) CK(hipHostUnregister(h[k]));
    });
    // pinned destination (upper bound: no host copy)
    {
        char* pin[3];
        t = Clock::now();
        for (int k = 0; k < 3; ++k) CK(hipHostMalloc((void**)&pin[k], sizes[k], hipHostMallocDefault));
        std::printf("hipHostMalloc of the three planes: %.3f ms\n", ms_since(t));
        double acc = 0;
        for (int r = 0; r < reps + 1; ++r) {
            t = Clock::now();
            for (int k = 0; k < 3; ++k) CK(hipMemcpyAsync(pin[k], d[k], sizes[k], hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            if (r) acc += ms_since(t);
        }
        std::printf("%-50s %-7s %8.3f ms  (%.1f GB/s)\n", "DMA into pinned planes", "-", acc / reps,
                    total / (acc / reps) / 1e6);
        for (int k = 0; k < 3; ++k) CK(hipHostFree(pin[k]));
    }
    // a ring of pinned chunks: DMA chunk i+1 while the host copies chunk i out
    for (size_t chunk : {(size_t)1 << 21, (size_t)1 << 22, (size_t)1 << 23}) {
        for (int threads : {1, 4, 8}) {
            const int nring = 3;
            char* ring[nring];
            hipEvent_t ev[nring];
            t = Clock::now();
            for (int i = 0; i < nring; ++i) {
                CK(hipHostMalloc((void**)&ring[i], chunk, hipHostMallocDefault));
                CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
            }
            const double alloc_ms = ms_since(t);
            char name[96];
            std::snprintf(name, sizeof name, "ring %d x %zu MB, %d copy threads (alloc %.2f ms)", nring, chunk >> 20,
                          threads, alloc_ms);
            run(name, [&](char** h) {
                struct Piece {
                    int k;
                    size_t off, n;
                };
                std::vector<Piece> pcs;
                for (int k = 0; k < 3; ++k)
                    for (size_t o = 0; o < sizes[k]; o += chunk) pcs.push_back({k, o, std::min(chunk, sizes[k] - o)});
                size_t issued = 0;
                for (size_t i = 0; i < pcs.size(); ++i) {
                    while (issued < pcs.size() && issued < i + nring) {
                        const Piece& p = pcs[issued];
                        CK(hipMemcpyAsync(ring[issued % nring], d[p.k] + p.off, p.n, hipMemcpyDeviceToHost, s));
                        CK(hipEventRecord(ev[issued % nring], s));
                        ++issued;
                    }
                    CK(hipEventSynchronize(ev[i % nring]));
                    par_copy(h[pcs[i].k] + pcs[i].off, ring[i % nring], pcs[i].n, threads);
                }
            });
            for (int i = 0; i < nring; ++i) {
                CK(hipHostFree(ring[i]));
                CK(hipEventDestroy(ev[i]));
            }
        }
    }
    return 0;
}
