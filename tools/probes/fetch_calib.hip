// Probe: FETCH_SIZE / WRITE_SIZE calibration for the render's own access
// patterns (MI355X_MICROARCH.md, HBM section: gfx950 reports half the bytes of
// a wide coalesced streaming read; other widths are uncalibrated).  Each
// kernel touches a known byte count once, over buffers far larger than the
// 256 MiB Infinity Cache, so the counters can be divided by it:
//   stream16  lane L reads 16 B at 16*L (the guide's calibrated pattern)
//   entry64   lane L reads its 64-B element as 4 x 16 B (the render's
//             region-list entries, k_render_binned's footprint loads)
//   dma64     lane L DMAs its 64-B element into LDS, 4 x 16 B
//             (stage_survivor_records)
//   gather64  entry64 through a scrambled index (records read through ids)
//   tile_store 8x8-pixel tiles of an f32 plane and a u8 plane, one pixel per
//             lane (the render's output stores)
// Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib   (then WRITE_SIZE)
#include <hip/hip_runtime.h>

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

constexpr size_t kBytes = (size_t)1 << 30;          // 1 GiB per read pattern
constexpr size_t kElems64 = kBytes / 64;

__global__ __launch_bounds__(256) void stream16(const float4* __restrict__ in, float* __restrict__ sink)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const float4 v = in[i];
    const float s = v.x + v.y + v.z + v.w;
    if (s == 12345.0f) sink[i & 1023] = s;          // never true: keeps the load
}

__global__ __launch_bounds__(256) void entry64(const float4* __restrict__ in, float* __restrict__ sink)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const float4* e = in + 4 * i;
    const float4 a = e[0], b = e[1], c = e[2], d = e[3];
    const float s = a.x + b.y + c.z + d.w;
    if (s == 12345.0f) sink[i & 1023] = s;
}

__device__ __forceinline__ uint32_t scramble(uint32_t i, uint32_t n)
{
    // a bijection on [0, n) for n a power of two: odd multiplier, xor-shift
    i = (i * 2654435761u) & (n - 1u);
    i ^= i >> 7;
    return (i * 2246822519u) & (n - 1u);
}

__global__ __launch_bounds__(256) void gather64(const float4* __restrict__ in, float* __restrict__ sink)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const float4* e = in + 4 * (size_t)scramble(i, (uint32_t)kElems64);
    const float4 a = e[0], b = e[1], c = e[2], d = e[3];
    const float s = a.x + b.y + c.z + d.w;
    if (s == 12345.0f) sink[i & 1023u] = s;
}

__global__ __launch_bounds__(64) void dma64(const float4* __restrict__ in, float* __restrict__ sink)
{
    __shared__ float4 q[4][64];
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    const float4* src = in + 4 * i;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        __builtin_amdgcn_global_load_lds((const void*)(src + k), (__attribute__((address_space(3))) void*)&q[k][0], 16,
                                         0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float s = q[0][threadIdx.x].x + q[3][threadIdx.x].w;
    if (s == 12345.0f) sink[i & 1023] = s;
}

// one 8x8 tile per wave, tiles row-major over a W x H frame
__global__ __launch_bounds__(64) void tile_store(float* __restrict__ img, uint8_t* __restrict__ u8, uint32_t W)
{
    const uint32_t tiles_x = W / 8u;
    const uint32_t tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const uint32_t col = tx * 8u + (threadIdx.x & 7u), row = ty * 8u + (threadIdx.x >> 3);
    const size_t o = (size_t)row * W + col;
    img[o] = (float)o;
    u8[o] = (uint8_t)o;
}

int main()
{
    float4* in = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&in, kBytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(in, 0, kBytes));
    const uint32_t W = 16384;                       // 16384^2 pixels: 1 GiB f32 + 256 MiB u8
    float* img = nullptr;
    uint8_t* u8 = nullptr;
    CK(hipMalloc(&img, (size_t)W * W * 4));
    CK(hipMalloc(&u8, (size_t)W * W));
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        stream16<<<kBytes / 16 / 256, 256>>>(in, sink);
        entry64<<<kElems64 / 256, 256>>>(in, sink);
        gather64<<<kElems64 / 256, 256>>>(in, sink);
        dma64<<<kElems64 / 64, 64>>>(in, sink);
        tile_store<<<(W / 8) * (W / 8), 64>>>(img, u8, W);
        CK(hipDeviceSynchronize());
    }
    std::printf("bytes read per read kernel: %zu (%.1f MiB); tile_store writes %zu f32 + %zu u8 bytes (%.1f MiB)\n",
                kBytes, kBytes / 1048576.0, (size_t)W * W * 4, (size_t)W * W, (size_t)W * W * 5 / 1048576.0);
    CK(hipFree(in));
    CK(hipFree(sink));
    CK(hipFree(img));
    CK(hipFree(u8));
    return 0;
}
