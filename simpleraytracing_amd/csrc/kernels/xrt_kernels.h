// xrt_kernels.h -- HIP kernels of the X-ray render path for gfx950 (CDNA4).
//
// Kernels
//   k_prep           one thread per triangle: TriRec (ray-independent part of
//                    Ray::intersect for the shared origin) and the cull planes
//                    (the conservative screen-space footprint, SoA float4).
//   k_render_brute   renderLoop as written: one ray per lane, one 8x8 ray tile
//                    per wavefront, every ray tests every triangle; triangle
//                    records are wave-uniform scalar loads.
//   k_render_tiled   one 32x32 pixel region per workgroup (4 waves, 4 tiles of
//                    8x8 each).  Phase 1: all 256 lanes sweep the whole mesh's
//                    footprint boxes (coalesced 16-B loads) and compact the
//                    region's candidates into an LDS list.  Phase 2: per 8x8
//                    tile, one lane per candidate evaluates the three relaxed
//                    edge functions, a wave ballot keeps the survivors, and
//                    every survivor runs the exact Moller-Trumbore test for all
//                    64 rays.  Output is bit-identical to k_render_brute.
//   Rays whose register hit list overflows are recomputed exactly by their
//   own wave before the tile's stores (wave_overflow_distance).
//   k_probe_*        device probes of the exact device code paths (tests).
#pragma once

#include "xrt_device.h"


namespace XRT_KERNEL_NS {

// Binning control block, cleared with the region counters before every binned
// frame's k_prep; read back by xrt_read_stats (list sizing).
struct BinState {
    unsigned int max_count;     // largest region count of the frame (list sizing)
    unsigned int global_count;  // triangles in the global list
    unsigned int overflow;      // some region count exceeded the list capacity
    unsigned int cursor;        // a device-sized frame's pool cursor (k_size_lists)
    unsigned int pairs;         // a device-sized frame's appended pairs (BinBuffers::pairs)
    unsigned int tile_slots;    // a device-planned frame's tile regions (k_size_lists; BinBuffers::dev_plan)
    unsigned int fill_slots;    //                          and its empty ones
    unsigned int pad;
};

// Host-computed bounds for the cull derivation (DESIGN.md "Tile cull").
struct CullParams {
    double dmax;      // upper bound of |D| (unnormalised ray direction) over the image
    double mag;       // upper bound of the magnitudes summed while forming D
    double width, height;
    int dir_grid;     // every nonzero component of every ray direction of the image is a
                      // multiple of 2^dir_grid (DESIGN.md "Tile cull", step 0)
    int pad;
    // The camera in f64, formed on the host exactly as compute_footprint would
    // (detector - origin, up, right, spacing and the centring offsets): kernel
    // arguments stay in SGPRs, where converting the floats in the kernel held
    // 24 VGPRs of uniform values through the edge loop.
    double cvec[3], up[3], rt[3];
    double ps, cv, cu;
};

// Grid exponent of a float: x is a multiple of 2^grid_exp(x), the weight of
// its lowest set bit.  Zero lies on every grid (kNoGrid).
constexpr int kNoGrid = 1000;
__host__ __device__ __forceinline__ int grid_exp(float x)
{
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    if ((u & 0x7FFFFFFFu) == 0u) return kNoGrid;
    const int e = (int)((u >> 23) & 0xFFu);
    const uint32_t m = (u & 0x7FFFFFu) | (e ? 0x800000u : 0u);
    return (e ? e - 150 : -149) + __builtin_ctz(m);
}

// Per-workgroup (BINNED: per-wave) statistics, written with plain stores, one
// record each, and summed on the host by xrt_read_stats: same-address global
// atomics from every wave serialise in L2, and a reduction kernel would sit
// on every frame's critical path.
struct BlockStats {
    unsigned int rays, hit_rays, odd_rays, overflow_rays, hits, tile_tests, candidates, max_hits;
};
static_assert(sizeof(BlockStats) == 32, "BlockStats must be 32 bytes");

struct Outputs {
    float* image;
    float* lbuffer;
    uint8_t* image_u8;
    BlockStats* block_stats;   // one per workgroup (BINNED: per wave) of the render grid
    // Timing records (timed regions, every kTimingStride-th frame; else null):
    // beside each statistics record its wave's (workgroup's) s_memrealtime
    // start and end, low 32 bits of the 100 MHz counter.  The host takes the
    // kernel's span, last end - first start, from them (xrt_timing_end).
    uint2* wave_times;
    // The frame's parameters in device memory (written by k_prep), read by
    // make_ray through this constant-address-space pointer: scalar loads where
    // a tile first needs its rays, instead of camera kernel arguments held in
    // SGPRs for the whole kernel.
    const __attribute__((address_space(4))) RenderParams* frame;
    PixelOffsets off;          // the frame's pixel-offset tables (k_prep)
    // L-buffer value of a ray that hits nothing: +inf (the reference's
    // z_buffer), or a transit code for strips gathered as L-buffers only
    // (kMissTransit, expanded on the receiving device by k_expand).
    float miss_l;
    float mu;                  // kModelSigned: mesh 0's attenuation coefficient (fork :800)
    // Transit layouts (BINNED with a fill plan only; lbuffer is the message):
    // kLayoutPacked -- pixel (row, col) of the region in launch slot s goes to
    // s * 1024 + its row-major offset in the region's 32x32 block; the plan's
    // filled regions store nothing.  kLayoutHits -- tile t of slot s (index i =
    // s * 16 + t, i < hit_tiles) stores the 64-bit mask of its hit rays at
    // words [2i, 2i + 2) and their L values, in lane order, at words
    // 2 * hit_tiles + hit_off[i] ..; hit_off comes from the geometry's hit plan
    // (xrt_plan_hit_layout).
    uint32_t packed;
    uint32_t hit_tiles;
    const uint32_t* hit_off;
};
// (the hit layout has its own instantiation of the binned render, kHits: its
// stores in the ordinary render cost 10-35% of the kernel's time)
constexpr uint32_t kLayoutRowMajor = 0u, kLayoutPacked = 1u, kLayoutHits = 2u;

// A wave-uniform table entry read through the constant address space (a scalar load).
__device__ __forceinline__ const __attribute__((address_space(4))) uint32_t* as_const_u32(const uint32_t* p)
{
    return (const __attribute__((address_space(4))) uint32_t*)p;
}

// The hit layout's element of a tile: its index (low 32 bits) and its plan's
// first hit word (high 32 bits; hit_off, a scalar load issued when the tile
// starts rather than where its values are stored).
__device__ __forceinline__ size_t hit_element(const Outputs& out, uint32_t index)
{
    return (size_t)index | ((size_t)as_const_u32(out.hit_off)[index] << 32);
}

// The hit layout's per-tile stores (kLayoutHits): the mask by lane 0, a hit
// lane's L value at its rank among the tile's hits.  `hit`: the lane's ray hit
// mesh 0 at least once; `e`: hit_element's.  Every lane of the wave calls it.
// Values past the plan's count for the tile (hit_off[i + 1] - hit_off[i]; the
// plan has tiles + 1 offsets) are not stored: a tile can never write into the
// next tile's values.  Its mask still says how many hits it had, so the
// receiver (k_unpack_hits) flags the disagreement.
__device__ __forceinline__ void store_hit_tile(const Outputs& out, size_t e, bool hit, float lval)
{
    const unsigned long long m = __ballot(hit);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t* msg = reinterpret_cast<uint32_t*>(out.lbuffer);
    if (lane == 0u) reinterpret_cast<uint2*>(msg)[(uint32_t)e] = make_uint2((uint32_t)m, (uint32_t)(m >> 32));
    if (hit) {
        const uint32_t first = (uint32_t)(e >> 32);
        const uint32_t planned = as_const_u32(out.hit_off)[(uint32_t)e + 1u] - first;
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (rank < planned) out.lbuffer[2u * (size_t)out.hit_tiles + first + rank] = lval;
    }
}

// A signalling NaN no render produces (path lengths are >= 0, +inf, or x86's
// default NaN): marks "no hit" in L-buffer strips in transit, where +inf
// would be ambiguous (a ray with t = +inf hits also has L = +inf, but its
// image value is 0, not 80).
constexpr uint32_t kMissTransit = 0x7F800001u;

// A pixel inside the image for the offset tables (lanes of a partial tile
// outside it compute a ray nobody stores).
__device__ __forceinline__ void make_tile_ray(const RenderParams& p, const Outputs& out, uint32_t row,
                                              uint32_t col, float& dx, float& dy, float& dz)
{
    make_ray(*out.frame, out.off, min(row, p.height - 1u), min(col, p.width - 1u), dx, dy, dz);
}

// With the once-normalised direction too (the signed model's sign test).
__device__ __forceinline__ void make_tile_ray(const RenderParams& p, const Outputs& out, uint32_t row,
                                              uint32_t col, float& dx, float& dy, float& dz, float& sx,
                                              float& sy, float& sz)
{
    const uint32_t r = min(row, p.height - 1u), c = min(col, p.width - 1u);
    make_ray_from(*out.frame, out.off.v[r], out.off.u[c], dx, dy, dz, sx, sy, sz);
}

// Running counters of one wave: ballot counts (wave-uniform), per-lane hit sum
// and maximum (reduced across the wave once, in store_block_stats).
struct WaveStats {
    uint32_t rays, hit_rays, odd_rays, overflow_rays;
    uint32_t lane_hits, lane_max;   // per lane
    uint32_t tile_tests;
};

constexpr double kEps = 0x1p-24;

// Wave-uniform values the compiler cannot prove uniform (a wave's index in its
// workgroup, a count loaded through a plain pointer): moved to an SGPR, so the
// loops they bound are scalar-controlled and what derives from them is scalar.
__device__ __forceinline__ uint32_t wave_uniform(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint32_t wave_in_block() { return wave_uniform(threadIdx.x >> 6); }

__device__ __forceinline__ void cross_d(const double a[3], const double b[3], double o[3])
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ double dot_d(const double a[3], const double b[3])
{
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

__device__ __forceinline__ double l1_d(const double a[3])
{
    return fabs(a[0]) + fabs(a[1]) + fabs(a[2]);
}

// ---------------------------------------------------------------------------
// Per-ray epilogue shared by the render kernels: statistics, the exact fix-up
// of overflowed rays, L-buffer, shade, LUT, stores.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_stats(WaveStats& ws, bool active, uint32_t n, bool odd,
                                           bool overflow)
{
    ws.rays += (uint32_t)__popcll(__ballot(active));
    ws.hit_rays += (uint32_t)__popcll(__ballot(active && n > 0));
    ws.odd_rays += (uint32_t)__popcll(__ballot(active && odd));
    ws.overflow_rays += (uint32_t)__popcll(__ballot(active && overflow));
    const uint32_t h = active ? n : 0u;
    ws.lane_hits += h;
    ws.lane_max = ws.lane_max > h ? ws.lane_max : h;
}

// Start of a wave (workgroup) for its timing record: the 100 MHz
// s_memrealtime counter (one scalar load; awaited with the first others).
__device__ __forceinline__ uint64_t block_start_stamp() { return __builtin_amdgcn_s_memrealtime(); }

// The timing record of a statistics record: (start, end), low 32 bits.
__device__ __forceinline__ void store_times(uint2* times, uint32_t index, uint64_t t_start)
{
    if (times) times[index] = make_uint2((uint32_t)t_start, (uint32_t)__builtin_amdgcn_s_memrealtime());
}

// Combines the block's wave counters through LDS and stores one BlockStats
// (and its timing record).  Must be reached by every thread of the block.
__device__ __forceinline__ void store_block_stats(const WaveStats& ws, uint32_t candidates,
                                                  BlockStats* out, uint2* times, uint64_t t_start)
{
    __shared__ WaveStats s_ws[4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t hits = ws.lane_hits, mx = ws.lane_max;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        hits += __shfl_xor(hits, off);
        const uint32_t o = __shfl_xor(mx, off);
        mx = mx > o ? mx : o;
    }
    if (lane == 0) {
        s_ws[wave] = ws;
        s_ws[wave].lane_hits = hits;
        s_ws[wave].lane_max = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        BlockStats b = {};
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            b.rays += s_ws[w].rays;
            b.hit_rays += s_ws[w].hit_rays;
            b.odd_rays += s_ws[w].odd_rays;
            b.overflow_rays += s_ws[w].overflow_rays;
            b.hits += s_ws[w].lane_hits;
            b.tile_tests += s_ws[w].tile_tests;
            b.max_hits = b.max_hits > s_ws[w].lane_max ? b.max_hits : s_ws[w].lane_max;
        }
        b.candidates = candidates;
        out[blockIdx.y * gridDim.x + blockIdx.x] = b;
        store_times(times, blockIdx.y * gridDim.x + blockIdx.x, t_start);
    }
}

// Wave-wide sum / max of a u32 with DPP row shifts and row broadcasts (six
// VALU ops, the total lands in lane 63) instead of six ds_bpermute rounds.
// row_shr:n (0x110 + n) reads lane i-n of the same 16-lane row (0 past the
// row start: bound_ctrl); row_bcast:15 (0x142) adds lane 15 of rows 0 / 2 to
// rows 1 / 3; row_bcast:31 (0x143) adds lane 31 to rows 2 and 3.
// m with bit b (its lowest set bit) cleared: one s_bitset0_b64 instead of the
// three SALU ops of m & (m - 1).
__device__ __forceinline__ void clear_lane_bit(unsigned long long& m, uint32_t b)
{
    asm("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(b));
}

template <bool kMax>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t x)
{
    auto op = [](uint32_t a, uint32_t b) { return kMax ? (a > b ? a : b) : a + b; };
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// Sum of a and maximum of b over the wave, the two DPP chains interleaved (each
// step's DPP read of the other chain's last write fills the hazard gap).
__device__ __forceinline__ void wave_reduce_sum_max(uint32_t a, uint32_t b, uint32_t& sum, uint32_t& mx)
{
#define XRT_DPP_STEP(ctrl, rmask, bc)                                                                     \
    a += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, ctrl, rmask, 0xf, bc);                         \
    {                                                                                                     \
        const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, ctrl, rmask, 0xf, bc);        \
        b = b > o ? b : o;                                                                                \
    }
    XRT_DPP_STEP(0x111, 0xf, true)
    XRT_DPP_STEP(0x112, 0xf, true)
    XRT_DPP_STEP(0x114, 0xf, true)
    XRT_DPP_STEP(0x118, 0xf, true)
    XRT_DPP_STEP(0x142, 0xa, false)
    XRT_DPP_STEP(0x143, 0xc, false)
#undef XRT_DPP_STEP
    sum = (uint32_t)__builtin_amdgcn_readlane((int)a, 63);
    mx = (uint32_t)__builtin_amdgcn_readlane((int)b, 63);
}

// One wave's statistics as one BlockStats record (no LDS, no barrier): the
// lane sums are reduced across the wave and lane 0 stores the record (and its
// timing record, `copies` of it from index on).
__device__ __forceinline__ void store_wave_stats(const WaveStats& ws, uint32_t candidates,
                                                 BlockStats* out, uint32_t index, uint2* times,
                                                 uint64_t t_start, uint32_t copies = 1)
{
    uint32_t hits, mx;
    wave_reduce_sum_max(ws.lane_hits, ws.lane_max, hits, mx);
    if ((threadIdx.x & 63u) == 0u) {
        BlockStats b;
        b.rays = ws.rays;
        b.hit_rays = ws.hit_rays;
        b.odd_rays = ws.odd_rays;
        b.overflow_rays = ws.overflow_rays;
        b.hits = hits;
        b.tile_tests = ws.tile_tests;
        b.candidates = candidates;
        b.max_hits = mx;
        out[index] = b;
        if (times) {
            const uint2 t = make_uint2((uint32_t)t_start, (uint32_t)__builtin_amdgcn_s_memrealtime());
            for (uint32_t k = 0; k < copies; ++k) times[index + k] = t;
        }
    }
}

// ---------------------------------------------------------------------------
// Exact distance of a ray whose hit count exceeded the register list
// (n > capacity), computed by the whole wave: lane k tests candidates k,
// k + 64, ... and keeps its accepted distances in a sorted register list of
// kFixupSlots; the 64 x kFixupSlots lists are bitonic-sorted across the wave
// (element e = slot * 64 + lane) and the pairs summed in ascending order,
// sequentially, as main.cxx:703-708 does.  A ray with more hits than one lane
// can hold streams its sorted sequence instead: repeated wave-wide scans for
// the next larger distance and its multiplicity.  The candidates are the
// ones the render tested before its tile cull (the cull is conservative, so
// the hit set is the same).  Ray and result are wave-uniform; rare path.
// ---------------------------------------------------------------------------
constexpr int kFixupSlots = 8;

__device__ __forceinline__ bool fixup_hit(const TriRec* __restrict__ recs, uint32_t j, float dx,
                                          float dy, float dz, float& t)
{
    const TriRec r = recs[j];
    return mt_intersect(dx, dy, dz, r.e1x, r.e1y, r.e1z, r.e2x, r.e2y, r.e2z, r.tvx, r.tvy, r.tvz,
                        r.qvx, r.qvy, r.qvz, r.tnum, t) &&
           accept_t(t);
}

// Compare-exchange of the slot pairs (r, r | S) (element distance 64 S) of
// one bitonic stage; ascending where (r & size_slots) == 0.
template <uint32_t S>
__device__ __forceinline__ void bitonic_slots(float (&v)[kFixupSlots], uint32_t size_slots)
{
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kFixupSlots; ++r) {
        if (r & S) continue;
        const float a = v[r], b = v[r | S];
        const bool asc = (r & size_slots) == 0u;
        v[r] = asc ? fminf(a, b) : fmaxf(a, b);
        v[r | S] = asc ? fmaxf(a, b) : fminf(a, b);
    }
}

template <typename Fetch>
__device__ float wave_overflow_distance(const TriRec* __restrict__ recs, uint32_t n_cand, Fetch fetch,
                                        float dx, float dy, float dz)
{
    const uint32_t lane = threadIdx.x & 63u;
    float v[kFixupSlots];
#pragma unroll
    for (int r = 0; r < kFixupSlots; ++r) v[r] = __builtin_inff();
    uint32_t cnt = 0;
    for (uint32_t base = 0; base < n_cand; base += 64u) {
        const uint32_t k = base + lane;
        float t = 0.0f;
        const bool hit = k < n_cand && fixup_hit(recs, fetch(k), dx, dy, dz, t);
        if (hit) {                                    // sorted insert (drops the largest past 8)
            float prev = v[0];
            v[0] = fminf(prev, t);
#pragma unroll
            for (int r = 1; r < kFixupSlots; ++r) {
                const float cur = v[r];
                v[r] = __builtin_amdgcn_fmed3f(prev, cur, t);
                prev = cur;
            }
            ++cnt;
        }
    }
    uint32_t total = cnt, most = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        total += __shfl_xor(total, off);
        const uint32_t o = __shfl_xor(most, off);
        most = most > o ? most : o;
    }
    total = (uint32_t)__builtin_amdgcn_readfirstlane((int)total);   // uniform: the loops below
    most = (uint32_t)__builtin_amdgcn_readfirstlane((int)most);     // index lanes with it
    if (total & 1u) return 0.0f;                      // odd count: main.cxx:709-713
    float distance = 0.0f;
    if (most <= (uint32_t)kFixupSlots) {
        constexpr uint32_t N = 64u * kFixupSlots;
        // rolled loops: unrolled, this rare path is most of the render's code
        // (and its instruction cache footprint)
#pragma nounroll
        for (uint32_t size = 2; size <= N; size <<= 1) {
#pragma nounroll
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                if (stride >= 64u) {
                    const uint32_t ss = size >> 6;
                    if (stride == 64u) bitonic_slots<1>(v, ss);
                    else if (stride == 128u) bitonic_slots<2>(v, ss);
                    else bitonic_slots<4>(v, ss);
                } else {
                    const bool lower = (lane & stride) == 0u;
#pragma unroll
                    for (uint32_t r = 0; r < (uint32_t)kFixupSlots; ++r) {
                        const float o = __shfl_xor(v[r], (int)stride);
                        const bool asc = size < 64u ? (lane & size) == 0u : (r & (size >> 6)) == 0u;
                        v[r] = (lower == asc) ? fminf(v[r], o) : fmaxf(v[r], o);
                    }
                }
            }
        }
        // pair differences on the even lanes, then the sequential f32 sum
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kFixupSlots; ++r) {
            const float d = __shfl_xor(v[r], 1) - v[r];
#pragma nounroll
            for (uint32_t l = 0; l < 64u && r * 64u + l + 1u < total; l += 2u)
                distance += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), (int)l));
        }
        return distance;
    }
    // Streamed: the sorted sequence by repeated scans (value, multiplicity).
    uint32_t pos = 0;
    float prev = -__builtin_inff(), pending = 0.0f;
    while (pos < total) {
        float cur = __builtin_inff();
        uint32_t mult = 0;
        for (uint32_t base = 0; base < n_cand; base += 64u) {
            const uint32_t k = base + lane;
            float t = 0.0f;
            if (k < n_cand && fixup_hit(recs, fetch(k), dx, dy, dz, t) && t > prev) {
                if (t < cur) { cur = t; mult = 1; }
                else if (t == cur) ++mult;
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float oc = __shfl_xor(cur, off);
            const uint32_t om = __shfl_xor(mult, off);
            if (oc < cur) { cur = oc; mult = om; }
            else if (oc == cur) mult += om;
        }
        if (mult == 0) break;                         // cannot happen; keeps the loop bounded
        for (uint32_t q = 0; q < mult && pos < total; ++q, ++pos) {
            if ((pos & 1u) == 0) pending = cur;
            else distance += cur - pending;
        }
        prev = cur;
    }
    return distance;
}

// ---------------------------------------------------------------------------
// The fix-up over the tile's survivors.  A tile's overflowed rays hit only
// candidates that passed its tile cull, and there are few of those (a tile
// with overflowed rays on the 1.12 M-triangle mesh has ~100 survivors of
// thousands of candidates).  collect_survivors makes one pass over the
// candidates and keeps the survivors' candidate indices, 64 per slot
// (survivor s in slot s / 64 of lane s % 64); each overflowed ray then tests
// at most kSurvSlots records per lane, keeps its hits sorted in registers, and
// the wave takes them in ascending order, one wave minimum per hit, summing
// the pairs as main.cxx:703-708 does.  More than 64 * kSurvSlots survivors:
// the whole-candidate path above.
// ---------------------------------------------------------------------------
constexpr uint32_t kSurvSlots = 4;

// A cull functor answers "does candidate k pass the tile cull of the render
// that called finish_ray"; NoCull (the brute-force render, which has none)
// takes the whole-candidate fix-up, and so does an EntryCull (k_render_binned)
// of a region rendered from the whole mesh.
struct NoCull {
    __device__ bool operator()(uint32_t) const { return true; }
};

struct EntryCull;
__device__ __forceinline__ bool cull_enabled(const NoCull&) { return false; }
template <typename Cull>
__device__ __forceinline__ bool cull_enabled(const Cull& c)
{
    if constexpr (std::is_same<Cull, EntryCull>::value) return c.enabled;
    else return true;
}

// Position of the r-th (from 0) set bit of m; r < popcount(m).
__device__ __forceinline__ uint32_t nth_set_bit(unsigned long long m, uint32_t r)
{
    uint32_t pos = 0, w = (uint32_t)m, c = (uint32_t)__popc(w);
    if (r >= c) { r -= c; w = (uint32_t)(m >> 32); pos = 32u; }
    c = (uint32_t)__popc(w & 0xFFFFu);
    if (r >= c) { r -= c; w >>= 16; pos += 16u; }
    c = (uint32_t)__popc(w & 0xFFu);
    if (r >= c) { r -= c; w >>= 8; pos += 8u; }
    c = (uint32_t)__popc(w & 0xFu);
    if (r >= c) { r -= c; w >>= 4; pos += 4u; }
    c = (uint32_t)__popc(w & 0x3u);
    if (r >= c) { r -= c; w >>= 2; pos += 2u; }
    return pos + (r >= (w & 1u) ? 1u : 0u);
}

// false (wave-uniform) when the tile has more than 64 * kSurvSlots survivors.
template <typename Cull>
__device__ __forceinline__ bool collect_survivors(uint32_t n_cand, Cull cull, uint32_t (&surv)[kSurvSlots],
                                                  uint32_t& n_surv)
{
    const uint32_t lane = threadIdx.x & 63u;
    n_surv = 0;
    for (uint32_t base = 0; base < n_cand; base += 64u) {
        const uint32_t k = base + lane;
        const unsigned long long m = __ballot(k < n_cand && cull(k));
        const uint32_t c = (uint32_t)__popcll(m);
        if (n_surv + c > 64u * kSurvSlots) return false;
        // this batch's survivors take positions [n_surv, n_surv + c); lane keeps p = lane (mod 64)
        const uint32_t r = (lane - n_surv) & 63u;
        if (r < c) {
            const uint32_t slot = (n_surv + r) >> 6, kk = base + nth_set_bit(m, r);
#pragma unroll
            for (uint32_t i = 0; i < kSurvSlots; ++i)
                if (slot == i) surv[i] = kk;
        }
        n_surv += c;
    }
    return true;
}

// Minimum over the wave of t >= 0 (ordered like its bits): the maximum of the
// complemented bits, so DPP's zero fill is the identity.
__device__ __forceinline__ float wave_min_pos(float t)
{
    return __uint_as_float(~wave_reduce_u32<true>(~__float_as_uint(t)));
}

template <typename Fetch>
__device__ float wave_survivor_distance(const TriRec* __restrict__ recs, const uint32_t (&surv)[kSurvSlots],
                                        uint32_t n_surv, Fetch fetch, float dx, float dy, float dz)
{
    const uint32_t lane = threadIdx.x & 63u;
    float v[kSurvSlots];
#pragma unroll
    for (uint32_t i = 0; i < kSurvSlots; ++i) v[i] = __builtin_inff();
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSurvSlots; ++i) {
        if (i * 64u >= n_surv) break;                 // wave-uniform
        float t = 0.0f;
        if (i * 64u + lane < n_surv && fixup_hit(recs, fetch(surv[i]), dx, dy, dz, t)) {
            float prev = v[0];                        // sorted insert (a lane holds <= kSurvSlots)
            v[0] = fminf(prev, t);
#pragma unroll
            for (uint32_t r = 1; r < kSurvSlots; ++r) {
                const float cur = v[r];
                v[r] = __builtin_amdgcn_fmed3f(prev, cur, t);
                prev = cur;
            }
            ++cnt;
        }
    }
    const uint32_t total = wave_reduce_u32<false>(cnt);
    if (total & 1u) return 0.0f;                      // odd count: main.cxx:709-713
    float distance = 0.0f, pending = 0.0f;
    for (uint32_t pos = 0; pos < total; ++pos) {
        // the next hit in ascending order: popped from the first lane that holds it
        // (+inf hits are the largest and equal: whichever lane pops, the value is right)
        const float mn = wave_min_pos(v[0]);
        if (lane == (uint32_t)__builtin_ctzll(__ballot(v[0] == mn))) {
#pragma unroll
            for (uint32_t r = 0; r + 1 < kSurvSlots; ++r) v[r] = v[r + 1];
            v[kSurvSlots - 1] = __builtin_inff();
        }
        if (pos & 1u) distance += mn - pending;
        else pending = mn;
    }
    return distance;
}

// The exact distances of the wave's overflowed rays (lanes of om; whole wave):
// each lane of om gets its ray's.
template <typename Fetch, typename Cull>
__device__ __forceinline__ float overflow_fixup(unsigned long long om, const TriRec* __restrict__ recs,
                                                uint32_t n_cand, Fetch fetch, Cull cull, float dx, float dy,
                                                float dz)
{
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t surv[kSurvSlots] = {}, n_surv = 0;
    const bool few = cull_enabled(cull) && collect_survivors(n_cand, cull, surv, n_surv);
    float mine = 0.0f;
    // one loop per path: surv is not live in the whole-candidate one
    auto each = [&](auto dist) {
        do {
            const uint32_t L = (uint32_t)__builtin_ctzll(om);
            om &= om - 1ull;
            const float d = dist(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(dx), (int)L)),
                                 __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dy), (int)L)),
                                 __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dz), (int)L)));
            if (lane == L) mine = d;
        } while (om);
    };
    if (few)
        each([&](float rx, float ry, float rz) { return wave_survivor_distance(recs, surv, n_surv, fetch, rx, ry, rz); });
    else
        each([&](float rx, float ry, float rz) { return wave_overflow_distance(recs, n_cand, fetch, rx, ry, rz); });
    return mine;
}

// Must be reached by the whole wave (the overflow fix-up is wave-wide).
// (dx, dy, dz) is this lane's ray; n_cand / fetch the candidates the render
// tested (fetch(k) = triangle of the k-th), cull(k) their tile cull.  kHits:
// the hit layout (o is the tile's hit_element).
template <bool kHits = false, typename Fetch, typename Cull = NoCull>
__device__ __forceinline__ void finish_ray(const RenderParams& p, const Outputs& out, bool active,
                                           size_t o, const HitList& hl,
                                           WaveStats& ws, const TriRec* __restrict__ recs, float dx,
                                           float dy, float dz, uint32_t n_cand, Fetch fetch,
                                           Cull cull = Cull())
{
    const uint32_t lane = threadIdx.x & 63u;
    bool overflow = hl.n > p.hit_capacity;
    bool odd = (hl.n & 1u) != 0u;
    wave_stats(ws, active, hl.n, odd, overflow);
    // main.cxx:700-718
    float distance = 0.0f;
    float lval = out.miss_l;
    if (hl.n > 0) {
        if (!odd) distance = hl.path_length();
        lval = distance;
    }
    const unsigned long long om = __ballot(active && overflow);
    if (__builtin_expect(om != 0ull, 0)) {            // wave-uniform, rare
        const float d = overflow_fixup(om, recs, n_cand, fetch, cull, dx, dy, dz);
        if ((om >> lane) & 1ull) {                    // n > capacity >= 1: the ray hit
            distance = d;
            lval = d;
        }
    }
    if (distance != distance) {                       // inf - inf: x86's default NaN (xrt_device.h)
        distance = xrt_f32_from_bits(kX86DefaultNaN);
        lval = distance;
    }
    if constexpr (kHits) {
        store_hit_tile(out, o, active && hl.n > 0u, lval);
        return;
    }
    if (!active) return;
    // distance 0 (a miss or an odd count) shades to 80 * expf(-0) = 80 -> 255;
    // the wave skips expf and the LUT when none of its rays needs them.
    float photon = 80.0f;
    uint8_t u8 = 255u;
    if (__ballot(distance != 0.0f)) {
        photon = shade(distance);
        u8 = lut_u8(photon);
    }
    if (out.image) out.image[o] = photon;
    if (out.lbuffer) out.lbuffer[o] = lval;
    if (out.image_u8) out.image_u8[o] = u8;
}

// The signed model's exact sum for a ray with more hits than its list holds,
// by the whole wave: the hits in triangle order by repeated scans for the
// next larger triangle id (ids are distinct), each term added in turn.  Ray
// (both directions) and result are wave-uniform; rare path.
template <typename Fetch>
__device__ float wave_signed_overflow_distance(const TriRec* __restrict__ recs, uint32_t n_cand, Fetch fetch,
                                               float dx, float dy, float dz, float sx, float sy, float sz)
{
    const uint32_t lane = threadIdx.x & 63u;
    float distance = 0.0f;
    uint32_t prev = 0;
    bool first = true;
    for (;;) {
        uint32_t best = 0xFFFFFFFFu;
        for (uint32_t base = 0; base < n_cand; base += 64u) {
            const uint32_t k = base + lane;
            if (k >= n_cand) continue;
            const uint32_t j = fetch(k);
            float t;
            if ((first || j > prev) && j < best && fixup_hit(recs, j, dx, dy, dz, t)) best = j;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)best, off);
            best = o < best ? o : best;
        }
        best = wave_uniform(best);
        if (best == 0xFFFFFFFFu) break;
        float t = 0.0f;
        fixup_hit(recs, best, dx, dy, dz, t);
        const TriRec& r = recs[best];
        distance += (float)hit_sign(sx, sy, sz, r.pad0, r.pad1, r.pad2) * t;
        prev = best;
        first = false;
    }
    return distance;
}

// The same over the tile's survivors (collect_survivors): each lane tests at
// most kSurvSlots records and keeps (triangle id, term); the wave takes the
// terms by ascending id, one wave minimum per hit.
template <typename Fetch>
__device__ float wave_signed_survivor_distance(const TriRec* __restrict__ recs,
                                               const uint32_t (&surv)[kSurvSlots], uint32_t n_surv, Fetch fetch,
                                               float dx, float dy, float dz, float sx, float sy, float sz)
{
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t id[kSurvSlots];
    float term[kSurvSlots];
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSurvSlots; ++i) {
        id[i] = 0xFFFFFFFFu;
        term[i] = 0.0f;
        if (i * 64u >= n_surv) continue;              // wave-uniform
        if (i * 64u + lane < n_surv) {
            const uint32_t j = fetch(surv[i]);
            float t = 0.0f;
            if (fixup_hit(recs, j, dx, dy, dz, t)) {
                const TriRec& r = recs[j];
                id[i] = j;
                term[i] = (float)hit_sign(sx, sy, sz, r.pad0, r.pad1, r.pad2) * t;
                ++cnt;
            }
        }
    }
    const uint32_t total = wave_reduce_u32<false>(cnt);
    float distance = 0.0f;
    for (uint32_t q = 0; q < total; ++q) {
        uint32_t mine = id[0];
#pragma unroll
        for (uint32_t i = 1; i < kSurvSlots; ++i) mine = id[i] < mine ? id[i] : mine;
        const uint32_t best = ~wave_reduce_u32<true>(~mine);          // ids are distinct
        const uint32_t owner = (uint32_t)__builtin_ctzll(__ballot(mine == best));
        float v = 0.0f;
#pragma unroll
        for (uint32_t i = 0; i < kSurvSlots; ++i) {
            if (id[i] == best) {
                v = term[i];
                id[i] = 0xFFFFFFFFu;
            }
        }
        distance += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)owner));
    }
    return distance;
}

// finish_ray of the signed model: the fork's L-buffer value (-1 flags) into
// out.lbuffer (image and u8 come from the hole fill, k_hole_fill).  The odd
// counter counts flagged rays.
template <typename Fetch, typename Cull = NoCull>
__device__ __forceinline__ void finish_ray_signed(const RenderParams& p, const Outputs& out, bool active,
                                                  uint32_t row, uint32_t col, const SignedHits& hl,
                                                  WaveStats& ws, const TriRec* __restrict__ recs, float dx,
                                                  float dy, float dz, float sx, float sy, float sz,
                                                  uint32_t n_cand, Fetch fetch, Cull cull = Cull())
{
    const uint32_t lane = threadIdx.x & 63u;
    const bool overflow = hl.n > p.hit_capacity;
    const bool flagged = hl.sign_sum != 0;
    wave_stats(ws, active, hl.n, flagged, overflow);
    float distance = hl.distance();
    unsigned long long om = __ballot(active && overflow && !flagged);
    if (om) {                                         // wave-uniform, rare
        uint32_t surv[kSurvSlots] = {}, n_surv = 0;
        const bool few = cull_enabled(cull) && collect_survivors(n_cand, cull, surv, n_surv);
        auto each = [&](auto dist) {                  // one loop per path, as in finish_ray
            do {
                const uint32_t L = (uint32_t)__builtin_ctzll(om);
                om &= om - 1ull;
                auto at = [L](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)L)); };
                const float d = dist(at(dx), at(dy), at(dz), at(sx), at(sy), at(sz));
                if (lane == L) distance = d;
            } while (om);
        };
        if (few)
            each([&](float rx, float ry, float rz, float qx, float qy, float qz) {
                return wave_signed_survivor_distance(recs, surv, n_surv, fetch, rx, ry, rz, qx, qy, qz);
            });
        else
            each([&](float rx, float ry, float rz, float qx, float qy, float qz) {
                return wave_signed_overflow_distance(recs, n_cand, fetch, rx, ry, rz, qx, qy, qz);
            });
    }
    if (!active || !out.lbuffer) return;
    float lval = 80.0f;                               // no term: 80 * exp(-0.0)
    if (__ballot(distance != 0.0f || flagged)) lval = signed_lbuffer(distance, hl.sign_sum, out.mu);
    out.lbuffer[(size_t)(row - p.row_begin) * p.width + col] = lval;
}

// Loads one triangle record with a wave-uniform index (scalar loads).
__device__ __forceinline__ void test_record(const TriRec* __restrict__ recs, uint32_t j, float dx,
                                            float dy, float dz, HitList& hl)
{
    const float4* q = reinterpret_cast<const float4*>(recs + j);
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
    float t;
    const bool hit =
        mt_intersect(dx, dy, dz, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, t) &&
        accept_t(t);
    if (__ballot(hit)) hl.push_if(hit, t);   // wave-uniform: most tests miss on every lane
}

// ---------------------------------------------------------------------------
// k_render_brute: block = 256 lanes = 2x2 waves, each wave one 8x8 ray tile.
// ---------------------------------------------------------------------------
// The signed model's test: the term's sign from the record's unit normal.
__device__ __forceinline__ void test_record(const TriRec* __restrict__ recs, uint32_t j, float dx,
                                            float dy, float dz, float sx, float sy, float sz, SignedHits& hl)
{
    const float4* q = reinterpret_cast<const float4*>(recs + j);
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
    float t;
    const bool hit =
        mt_intersect(dx, dy, dz, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, t) &&
        accept_t(t);
    if (__ballot(hit)) hl.push_if(hit, t, j, hit_sign(sx, sy, sz, d.y, d.z, d.w));
}

template <bool kSigned>
__global__ __launch_bounds__(256) void k_render_brute(const TriRec* __restrict__ recs,
                                                      RenderParams p, Outputs out)
{
    const uint64_t t_start = block_start_stamp();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_in_block();
    const uint32_t col = (blockIdx.x * 2u + (wave & 1u)) * 8u + (lane & 7u);
    const uint32_t row = p.row_begin + (blockIdx.y * 2u + (wave >> 1)) * 8u + (lane >> 3);
    const bool active = col < p.width && row < p.row_end;

    float dx, dy, dz, sx, sy, sz;
    make_tile_ray(p, out, row, col, dx, dy, dz, sx, sy, sz);
    typename std::conditional<kSigned, SignedHits, HitList>::type hl;
    hl.init();
    const uint32_t T = p.num_triangles;
    for (uint32_t j = 0; j < T; ++j) {
        if constexpr (kSigned) test_record(recs, j, dx, dy, dz, sx, sy, sz, hl);
        else test_record(recs, j, dx, dy, dz, hl);
    }
    WaveStats ws = {};
    ws.tile_tests = T;
    auto fetch = [](uint32_t k) { return k; };
    if constexpr (kSigned)
        finish_ray_signed(p, out, active, row, col, hl, ws, recs, dx, dy, dz, sx, sy, sz, T, fetch);
    else
        finish_ray(p, out, active, (size_t)(row - p.row_begin) * p.width + col, hl, ws, recs, dx, dy, dz, T, fetch);
    store_block_stats(ws, 0u, out.block_stats, out.wave_times, t_start);
}

// ---------------------------------------------------------------------------
// Tile cull (k_render_tiled, k_render_binned)
// ---------------------------------------------------------------------------
constexpr uint32_t kRegion = 32;        // pixels per region side (one workgroup)
constexpr uint32_t kPackBlock = kRegion * kRegion;   // floats per region in packed transit
constexpr uint32_t kListCap = 2048;     // LDS candidate list capacity (tiled)
#ifndef XRT_GLOBAL_REGIONS
#define XRT_GLOBAL_REGIONS 4096
#endif
#ifndef XRT_GLOBAL_REGIONS_UNBOUNDED
#define XRT_GLOBAL_REGIONS_UNBOUNDED 65536
#endif
constexpr uint32_t kGlobalRegionsUnbounded = XRT_GLOBAL_REGIONS_UNBOUNDED;
constexpr uint32_t kGlobalRegions = XRT_GLOBAL_REGIONS;   // footprints over more regions go to the global list

// Relaxed edge functions are stored as (a, b, c_t) with c_t = c + kTileHalf *
// (|a| + |b|) rounded up (compute_footprint): the edge's maximum over an 8x8
// tile's pixel-centre square [xc +- 3.5] x [yc +- 3.5] is a*xc + b*yc + c_t --
// two FMAs per edge for the render's per-candidate tile test.  Over a 32x32
// region's square (+- 15.5) it is 12 more half-widths.  (Conservative: c_t is
// not below the exact value, and the margin in c covers the f32 evaluation,
// DESIGN.md "Tile cull", step 5.)
constexpr float kTileHalf = 3.5f;
__device__ __forceinline__ float edge_tile(float4 e, float xc, float yc)
{
    return __builtin_fmaf(e.x, xc, __builtin_fmaf(e.y, yc, e.z));
}
__device__ __forceinline__ float edge_region(float4 e, float xc, float yc)
{
    return __builtin_fmaf(e.x, xc, __builtin_fmaf(e.y, yc, e.z)) + (15.5f - kTileHalf) * (fabsf(e.x) + fabsf(e.y));
}

// Footprint box (xmin, xmax, ymin, ymax) against the pixel-centre rectangle
// [x0, x1] x [y0, y1]; an unbounded or NaN box overlaps.
__device__ __forceinline__ bool box_overlaps(float4 bb, float x0, float x1, float y0, float y1)
{
    return !((bb.y < x0) | (bb.x > x1) | (bb.w < y0) | (bb.z > y1));
}

// All three edges evaluated, combined with `&` (not `&&`): a short-circuit
// lets the compiler sink each edge's load behind the previous edge's compare,
// three dependent memory round trips per candidate chunk instead of one.
// (xc, yc): the centre of an 8x8 tile.
__device__ __forceinline__ bool edges_pass_tile(float4 e0, float4 e1, float4 e2, float xc, float yc)
{
    return (edge_tile(e0, xc, yc) >= 0.0f) & (edge_tile(e1, xc, yc) >= 0.0f) & (edge_tile(e2, xc, yc) >= 0.0f);
}
// (xc, yc): the centre of a 32x32 region.
__device__ __forceinline__ bool edges_pass_region(float4 e0, float4 e1, float4 e2, float xc, float yc)
{
    return (edge_region(e0, xc, yc) >= 0.0f) & (edge_region(e1, xc, yc) >= 0.0f) &
           (edge_region(e2, xc, yc) >= 0.0f);
}

// Phase 2, shared by the tiled and binned kernels.
//
// The region's candidates (fetch(k) = triangle of the k-th candidate) are
// staged into LDS in chunks of kStage: their three relaxed edge functions and
// their Moller-Trumbore record, structure-of-arrays, loaded by all 256 lanes
// in one parallel round trip.  Each wave then renders its four 8x8 tiles from
// LDS only: one lane per staged candidate tests the tile rectangle against
// the relaxed edges, a ballot keeps the survivors, and each survivor's record
// is read with a wave-uniform (broadcast) LDS read and tested exactly for all
// 64 rays.  A region with more than kStage candidates re-stages per chunk
// (every wave reaches every barrier: the loop trip counts are block-uniform).
constexpr uint32_t kStage = 128;

struct StageLDS {
    float4 e0[kStage], e1[kStage], e2[kStage];
    float4 r0[kStage], r1[kStage], r2[kStage];
    float tnum[kStage];
};

template <typename Fetch>
__device__ __forceinline__ void stage_candidates(StageLDS& st, const TriRec* __restrict__ recs,
                                                 const float4* __restrict__ culls, uint32_t T,
                                                 uint32_t first, uint32_t count, Fetch fetch)
{
    for (uint32_t k = threadIdx.x; k < count; k += blockDim.x) {
        const uint32_t j = fetch(first + k);
        const float4* q = reinterpret_cast<const float4*>(recs + j);
        float4 e0 = culls[(size_t)T + j], e1 = culls[2 * (size_t)T + j], e2 = culls[3 * (size_t)T + j];
        float4 r0 = q[0], r1 = q[1], r2 = q[2];
        float tn = recs[j].tnum;
        st.e0[k] = e0; st.e1[k] = e1; st.e2[k] = e2;
        st.r0[k] = r0; st.r1[k] = r1; st.r2[k] = r2;
        st.tnum[k] = tn;
    }
}

__device__ __forceinline__ float test_lds(const StageLDS& st, uint32_t k, float dx, float dy,
                                          float dz, bool& hit)
{
    const float4 a = st.r0[k], b = st.r1[k], c = st.r2[k];
    return mt_exact(dx, dy, dz, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w,
                    st.tnum[k], hit);
}

// Survivors are tested two at a time (independent dependency chains for the
// scheduler to interleave), then pushed in ascending staged order.  The hit
// set, and so the sorted list, does not depend on the pairing.
__device__ __forceinline__ uint32_t test_staged(const StageLDS& st, uint32_t count, float xc,
                                                float yc, float dx, float dy, float dz, HitList& hl)
{
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t tests = 0;
    for (uint32_t base = 0; base < count; base += 64u) {
        const uint32_t k = base + lane;
        const bool pass = k < count && edges_pass_tile(st.e0[k], st.e1[k], st.e2[k], xc, yc);
        unsigned long long m = __ballot(pass);
        tests += (uint32_t)__popcll(m);
        while (m) {
            const uint32_t k0 = base + (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            bool h0, h1 = false;
            const float t0 = test_lds(st, k0, dx, dy, dz, h0);
            float t1 = 0.0f;
            if (m) {                                          // wave-uniform
                const uint32_t k1 = base + (uint32_t)__builtin_ctzll(m);
                m &= m - 1ull;
                t1 = test_lds(st, k1, dx, dy, dz, h1);
            }
            hl.push_if(h0, t0);
            hl.push_if(h1, t1);
        }
    }
    return tests;
}

template <typename Fetch>
__device__ __forceinline__ void render_region_tiles(const RenderParams& p, const Outputs& out,
                                                    const TriRec* __restrict__ recs,
                                                    const float4* __restrict__ culls,
                                                    uint32_t rx0, uint32_t ry0, uint32_t n_cand,
                                                    Fetch fetch, WaveStats& ws, StageLDS& st)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_in_block();
    const uint32_t T = p.num_triangles;
    const bool once = n_cand <= kStage;
    if (once) {
        stage_candidates(st, recs, culls, T, 0u, n_cand, fetch);
        __syncthreads();
    }
    for (uint32_t tile = wave; tile < 16u; tile += 4u) {
        const uint32_t tx0 = rx0 + (tile & 3u) * 8u;
        const uint32_t ty0 = ry0 + (tile >> 2) * 8u;
        const bool tile_live = tx0 < p.width && ty0 < p.row_end;   // wave-uniform
        const uint32_t col = tx0 + (lane & 7u);
        const uint32_t row = ty0 + (lane >> 3);
        const bool active = tile_live && col < p.width && row < p.row_end;
        const float xc = (float)tx0 + 3.5f, yc = (float)ty0 + 3.5f;

        float dx = 0.0f, dy = 0.0f, dz = 0.0f;
        if (tile_live) make_tile_ray(p, out, row, col, dx, dy, dz);
        else dx = 1.0f;
        HitList hl;
        hl.init();
        uint32_t tests = 0;
        if (once) {
            if (tile_live) tests = test_staged(st, n_cand, xc, yc, dx, dy, dz, hl);
        } else {
            for (uint32_t first = 0; first < n_cand; first += kStage) {
                const uint32_t count = min(kStage, n_cand - first);
                __syncthreads();
                stage_candidates(st, recs, culls, T, first, count, fetch);
                __syncthreads();
                if (tile_live) tests += test_staged(st, count, xc, yc, dx, dy, dz, hl);
            }
        }
        if (tile_live) {
            ws.tile_tests += tests;
            auto cull = [=](uint32_t k) {
                const uint32_t j = fetch(k);
                return edges_pass_tile(culls[(size_t)T + j], culls[2 * (size_t)T + j], culls[3 * (size_t)T + j],
                                       xc, yc);
            };
            finish_ray(p, out, active, (size_t)(row - p.row_begin) * p.width + col, hl, ws, recs, dx, dy, dz,
                       n_cand, fetch, cull);
        }
    }
}

// k_render_tiled: one 32x32 region per workgroup.  Phase 1: the 256 lanes
// sweep the footprint boxes of the whole mesh (every region sees every
// triangle) and compact the region's candidates into an LDS list.
__global__ __launch_bounds__(256) void k_render_tiled(const TriRec* __restrict__ recs,
                                                      const float4* __restrict__ culls,
                                                      RenderParams p, Outputs out)
{
    __shared__ uint32_t s_list[kListCap];
    __shared__ uint32_t s_count;
    __shared__ StageLDS st;
    const uint64_t t_start = block_start_stamp();

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t T = p.num_triangles;
    const uint32_t rx0 = blockIdx.x * kRegion;
    const uint32_t ry0 = p.row_begin + blockIdx.y * kRegion;
    const uint32_t rx1 = min(rx0 + kRegion, p.width) - 1u;       // inclusive
    const uint32_t ry1 = min(ry0 + kRegion, p.row_end) - 1u;

    if (tid == 0) s_count = 0;
    __syncthreads();

    // Chunks of 1024 boxes (4 independent 16-B loads per lane in flight); every
    // workgroup starts at a different chunk so concurrent reads spread over
    // the L2 channels.
    const float fx0 = (float)rx0, fx1 = (float)rx1, fy0 = (float)ry0, fy1 = (float)ry1;
    const uint32_t nchunks = (T + 1023u) / 1024u;
    uint32_t chunk =
        nchunks ? (uint32_t)(((uint64_t)(blockIdx.y * gridDim.x + blockIdx.x) * 2654435761u) % nchunks) : 0u;
    for (uint32_t c = 0; c < nchunks; ++c, chunk = (chunk + 1u == nchunks) ? 0u : chunk + 1u) {
        const uint32_t base = chunk * 1024u + tid;
        float4 bb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint32_t j = base + 256u * u;
            bb[u] = j < T ? culls[j] : make_float4(1.0f, -1.0f, 1.0f, -1.0f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint32_t j = base + 256u * u;
            bool pass = j < T && !(bb[u].y < fx0 || bb[u].x > fx1 || bb[u].w < fy0 || bb[u].z > fy1);
            unsigned long long m = __ballot(pass);
            if (m) {
                uint32_t cnt = (uint32_t)__popcll(m);
                uint32_t wbase = 0;
                if (lane == 0) wbase = atomicAdd(&s_count, cnt);
                wbase = __shfl(wbase, 0);
                if (pass) {
                    uint32_t idx = wbase + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                    if (idx < kListCap) s_list[idx] = j;
                }
            }
        }
    }
    __syncthreads();
    const uint32_t n_cand = wave_uniform(s_count);
    WaveStats ws = {};
    if (n_cand <= kListCap)
        render_region_tiles(p, out, recs, culls, rx0, ry0, n_cand,
                            [&](uint32_t k) { return s_list[k]; }, ws, st);
    else   // list overflow: every triangle is a candidate (still exact)
        render_region_tiles(p, out, recs, culls, rx0, ry0, T, [](uint32_t k) { return k; }, ws, st);
    store_block_stats(ws, n_cand, out.block_stats, out.wave_times, t_start);
}

// Conservative footprint of one triangle (DESIGN.md "Tile cull").
struct Footprint {
    float4 bbox, e0, e1, e2;
};

// Box of the loosened triangle when it is unbounded (its inward normals do not
// positively span the plane, e.g. a sliver seen edge-on): the bounding box of
// {A_k x + B_k y + C_k >= 0, k < 3} inside the image rectangle [-1, W] x
// [-1, H] in pixel-centre coordinates.  That set is a convex polygon whose
// vertices are intersections of two of its seven boundary lines; candidate
// vertices are accepted with a generous tolerance (so the box can only grow).
// Leaves `box` unchanged (unbounded: never culled by the box) if none is found.
// One of three doubles by a uniform index, as bit masks (a select chain the
// optimiser would turn into an indexed table in scratch memory).
__device__ __forceinline__ double pick3(uint32_t k, double x0, double x1, double x2)
{
    const uint64_t m0 = 0ull - (uint64_t)(k == 0u), m1 = 0ull - (uint64_t)(k == 1u), m2 = 0ull - (uint64_t)(k == 2u);
    return __longlong_as_double((long long)(((uint64_t)__double_as_longlong(x0) & m0) |
                                            ((uint64_t)__double_as_longlong(x1) & m1) |
                                            ((uint64_t)__double_as_longlong(x2) & m2)));
}

struct ClipEdges {
    double a0, a1, a2, b0, b1, b2, c0, c1, c2;
};

// Line k of the seven: k < 3 the edge (A_k x + B_k y + C_k >= 0), then the
// image rectangle's x >= -1, x <= W, y >= -1, y <= H.
__device__ __forceinline__ void clip_line(uint32_t k, const ClipEdges& e, double W, double H, double& la,
                                          double& lb, double& lc)
{
    if (k < 3u) {
        la = pick3(k, e.a0, e.a1, e.a2);
        lb = pick3(k, e.b0, e.b1, e.b2);
        lc = pick3(k, e.c0, e.c1, e.c2);
    } else {
        la = k == 3u ? 1.0 : k == 4u ? -1.0 : 0.0;
        lb = k < 5u ? 0.0 : k == 5u ? 1.0 : -1.0;
        lc = k == 3u ? 1.0 : k == 4u ? W : k == 5u ? 1.0 : H;
    }
}

// The 21 pairs are walked in a rolled loop (lines selected, not indexed): this
// rare path (unbounded footprints) fully unrolled set the kernel's register
// footprint (112 VGPRs; 72 without it).
__device__ __forceinline__ void clipped_box(const double A[3], const double B[3], const double C[3], double W,
                                            double H, float4& box)
{
    const ClipEdges e = {A[0], A[1], A[2], B[0], B[1], B[2], C[0], C[1], C[2]};
    double xmin = __builtin_inf(), xmax = -__builtin_inf();
    double ymin = __builtin_inf(), ymax = -__builtin_inf();
    bool any = false;
#pragma unroll 1
    for (uint32_t pr = 0; pr < 21u; ++pr) {
        // pair (a, b), a < b: (0,1) (0,2) ... (0,6) (1,2) ... (5,6)
        uint32_t a = 0, rest = pr;
        while (rest >= 6u - a) { rest -= 6u - a; ++a; }
        const uint32_t b = a + 1u + rest;
        double la, lb_, lc, ma, mb, mc;
        clip_line(a, e, W, H, la, lb_, lc);
        clip_line(b, e, W, H, ma, mb, mc);
        const double det = la * mb - ma * lb_;
        const double scale = (fabs(la) + fabs(lb_)) * (fabs(ma) + fabs(mb));
        if (!(fabs(det) > 1e-9 * scale)) continue;           // parallel (or NaN)
        const double x = (lb_ * mc - mb * lc) / det;
        const double y = (ma * lc - la * mc) / det;
        bool ok = isfinite(x) && isfinite(y);
#pragma unroll
        for (uint32_t k = 0; k < 7u; ++k) {
            double qa, qb, qc;
            clip_line(k, e, W, H, qa, qb, qc);
            const double v = qa * x + qb * y + qc;
            const double tol = 1e-6 * (fabs(qa * x) + fabs(qb * y) + fabs(qc)) + 1e-6;
            ok = ok && v >= -tol;
        }
        if (ok) {
            xmin = fmin(xmin, x); xmax = fmax(xmax, x);
            ymin = fmin(ymin, y); ymax = fmax(ymax, y);
            any = true;
        }
    }
    if (!any) return;
    const double sx = 0.01 + 1e-4 * (fabs(xmin) + fabs(xmax));
    const double sy = 0.01 + 1e-4 * (fabs(ymin) + fabs(ymax));
    box = make_float4((float)(xmin - sx), (float)(xmax + sx), (float)(ymin - sy), (float)(ymax + sy));
}

__device__ Footprint compute_footprint(const TriRec& r, const RenderParams& p, const CullParams& cp)
{
    const float kInf = __builtin_inff();
    Footprint c;
    c.bbox = make_float4(-kInf, kInf, -kInf, kInf);   // never cull
    c.e0 = make_float4(0.0f, 0.0f, kInf, 0.0f);
    c.e1 = c.e0;
    c.e2 = c.e0;
    c.e2.w = kInf;     // the regions the footprint reaches: unknown (bin_rect)

    bool finite = isfinite(r.tnum) && isfinite(r.qvx) && isfinite(r.qvy) && isfinite(r.qvz);
    if (finite && r.tnum == 0.0f) {
        // t = 0 * inv_det is never > 1e-7: the triangle never contributes.
        c.bbox = make_float4(kInf, -kInf, kInf, -kInf);
        c.e0 = make_float4(0.0f, 0.0f, -kInf, 0.0f);
        return c;
    }
    double E1[3] = {r.e1x, r.e1y, r.e1z};
    double E2[3] = {r.e2x, r.e2y, r.e2z};
    double TV[3] = {r.tvx, r.tvy, r.tvz};
    double l1e1 = l1_d(E1), l1e2 = l1_d(E2), l1tv = l1_d(TV);
    bool sane = finite && l1e1 > 0x1p-60 && l1e1 < 0x1p60 && l1e2 > 0x1p-60 && l1e2 < 0x1p60 &&
                l1tv > 0x1p-60 && l1tv < 0x1p60;
    if (!sane) {
        return c;
    }
    // Step 0: 1/det must stay finite.  Where a nonzero |det_f| falls to
    // 2^-128, (float)(1.0 / det) overflows and Ray.cxx records t = +inf
    // "hits" (u = 0 * inf = NaN passes its tests) for rays nowhere near the
    // triangle, which no footprint bounds.  det_f = e1 . RN(d x e2) is a
    // rounded sum of products of multiples of 2^g1, 2^gd and 2^g2 (a rounded
    // sum or product of multiples of 2^k is a multiple of 2^k), so a nonzero
    // one is >= 2^(g1 + gd + g2).  Triangles this cannot bound above 2^-128
    // (geometry at the 1e-20 scale) are never culled.  (Denormal
    // intermediates elsewhere add absolute errors of 2^-150, far below the
    // bounds B_k >= 2^-139 that the l1 ranges above guarantee.)
    {
        auto gmin3 = [](float x, float y, float z) { return min(grid_exp(x), min(grid_exp(y), grid_exp(z))); };
        const int g1 = gmin3(r.e1x, r.e1y, r.e1z), g2 = gmin3(r.e2x, r.e2y, r.e2z);
        if (g1 + cp.dir_grid + g2 < -127) return c;
    }
    double s = r.tnum > 0.0f ? 1.0 : -1.0;

    double N[3][3];
    cross_d(E2, TV, N[1]);     // a   = d . (edge2 x tvec)
    cross_d(TV, E1, N[2]);     // b   = d . (tvec x edge1)
    double Nd[3];
    cross_d(E2, E1, Nd);       // det = d . (edge2 x edge1)
    for (int k = 0; k < 3; ++k) N[0][k] = Nd[k] - N[1][k] - N[2][k];

    double Ba = 32.0 * kEps * l1tv * l1e2;
    double Bb = 32.0 * kEps * l1tv * l1e1;
    double Bd = 32.0 * kEps * l1e1 * l1e2;
    double Bx = 16.0 * kEps * l1e1 * l1e2;
    double B[3] = {Bd + Ba + Bb + Bx, Ba + Bx, Bb + Bx};

    const double* Cv = cp.cvec;
    const double* Up = cp.up;
    const double* Rt = cp.rt;
    const double ps = cp.ps, cv = cp.cv, cu = cp.cu;

    float ea[3], eb[3], ec[3];
    double c_edge[3] = {0.0, 0.0, 0.0};   // the constants before the tile half-width (the box below)
    bool constant_edge = false;
    for (int k = 0; k < 3; ++k) {
        double upn = dot_d(Up, N[k]);
        double rtn = dot_d(Rt, N[k]);
        double alpha = dot_d(Cv, N[k]) + cv * upn + cu * rtn;
        double beta = ps * upn;    // per image row
        double gamma = ps * rtn;   // per image column
        double l1n = l1_d(N[k]);
        double M = 4.0 * ((B[k] + 12.0 * kEps * l1n) * cp.dmax + 8.0 * kEps * cp.mag * l1n);
        // The edge is scaled by 1 / |(beta, gamma)|.  Any positive scale keeps
        // the inequality; the unit length only makes the margins below pixel
        // distances, so an approximate one serves: v_rsq_f32 (relative error
        // ~1e-7) where beta^2 + gamma^2 is in f32's normal range, instead of an
        // f64 sqrt and three f64 divisions per edge.
        const double nn = beta * beta + gamma * gamma;
        double nrm, inv_nrm;
        if (nn > 0x1p-120 && nn < 0x1p120) {
            inv_nrm = (double)__builtin_amdgcn_rsqf((float)nn);
            nrm = 1.0 / inv_nrm;
        } else {
            nrm = sqrt(nn);
            inv_nrm = 1.0 / nrm;
        }
        if (!(nrm > 1e-30 * (fabs(alpha) + M + 1e-300))) {
            // Edge function constant over the image plane.
            if (s * alpha + M < 0.0) {
                c.bbox = make_float4(kInf, -kInf, kInf, -kInf);
                c.e0 = make_float4(0.0f, 0.0f, -kInf, 0.0f);
                c.e1 = c.e2 = make_float4(0.0f, 0.0f, kInf, kInf);
                return c;
            }
            ea[k] = 0.0f;
            eb[k] = 0.0f;
            ec[k] = kInf;
            constant_edge = true;
            continue;
        }
        double a = s * gamma * inv_nrm;
        double b = s * beta * inv_nrm;
        double cc = (s * alpha + M) * inv_nrm;
        cc += 0.05 + 64.0 * kEps * (cp.width + cp.height + fabs(cc));
        ea[k] = (float)a;
        eb[k] = (float)b;
        c_edge[k] = (double)(float)cc;
        // stored with an 8x8 tile's half-width folded in (edge_tile), rounded up
        ec[k] = __double2float_ru(cc + (double)kTileHalf * (fabs((double)ea[k]) + fabs((double)eb[k])));
    }
    c.e0 = make_float4(ea[0], eb[0], ec[0], 0.0f);
    c.e1 = make_float4(ea[1], eb[1], ec[1], 0.0f);
    c.e2 = make_float4(ea[2], eb[2], ec[2], kInf);

    if (!constant_edge) {
        // Loosened triangle {a_k x + b_k y + c_k >= 0}: bounded iff the inward
        // normals positively span the plane (cross products share a sign).
        double A[3] = {ea[0], ea[1], ea[2]}, Bq[3] = {eb[0], eb[1], eb[2]}, Cq[3] = {c_edge[0], c_edge[1], c_edge[2]};
        double x01 = A[0] * Bq[1] - A[1] * Bq[0];
        double x12 = A[1] * Bq[2] - A[2] * Bq[1];
        double x20 = A[2] * Bq[0] - A[0] * Bq[2];
        const double tiny = 1e-9;
        bool pos = x01 > tiny && x12 > tiny && x20 > tiny;
        bool neg = x01 < -tiny && x12 < -tiny && x20 < -tiny;
        if (pos || neg) {
            double vx[3], vy[3];
            const int pi[3] = {0, 1, 2}, pj[3] = {1, 2, 0};
            const double cr[3] = {x01, x12, x20};
            for (int q = 0; q < 3; ++q) {     // (the box's margins cover the reciprocal's rounding)
                int ii = pi[q], jj = pj[q];
                const double inv_cr = 1.0 / cr[q];
                vx[q] = (-Cq[ii] * Bq[jj] + Cq[jj] * Bq[ii]) * inv_cr;
                vy[q] = (-A[ii] * Cq[jj] + A[jj] * Cq[ii]) * inv_cr;
            }
            double xmin = fmin(vx[0], fmin(vx[1], vx[2])), xmax = fmax(vx[0], fmax(vx[1], vx[2]));
            double ymin = fmin(vy[0], fmin(vy[1], vy[2])), ymax = fmax(vy[0], fmax(vy[1], vy[2]));
            double sx = 0.01 + 1e-4 * (fabs(xmin) + fabs(xmax));
            double sy = 0.01 + 1e-4 * (fabs(ymin) + fabs(ymax));
            if (isfinite(xmin) && isfinite(xmax) && isfinite(ymin) && isfinite(ymax)) {
                c.bbox = make_float4((float)(xmin - sx), (float)(xmax + sx), (float)(ymin - sy),
                                     (float)(ymax + sy));
                // Regions the loosened triangle can touch, by its size rather than
                // its box (a sliver's box is far larger): area / 32^2 + perimeter / 32
                // + the corners' cells (bin_rect's global-list choice).  Only its part
                // inside the image rectangle [-1, W] x [-1, H] can touch a region, and
                // that convex part has neither more area nor more perimeter than
                // either set: an edge-on sliver whose loosened triangle runs far past
                // the image (1.12 M-triangle frame at 8192^2: 44 of them) is walked
                // over its box's cells, not put on every region's list.
                const double iw = cp.width + 2.0, ih = cp.height + 2.0;
                const double area = fmin(0.5 * fabs((vx[1] - vx[0]) * (vy[2] - vy[0]) - (vx[2] - vx[0]) * (vy[1] - vy[0])),
                                         iw * ih);
                double perim = 0.0;         // (a size estimate: f32 square roots serve)
                for (int q = 0; q < 3; ++q)
                    perim += (double)__builtin_amdgcn_sqrtf(
                        (float)((vx[pj[q]] - vx[q]) * (vx[pj[q]] - vx[q]) + (vy[pj[q]] - vy[q]) * (vy[pj[q]] - vy[q])));
                perim = fmin(perim, 2.0 * (iw + ih));
                c.e2.w = (float)(area / (kRegion * kRegion) + 2.0 * perim / kRegion + 8.0);
            }
        } else {
            clipped_box(A, Bq, Cq, cp.width, cp.height, c.bbox);
        }
    }
    return c;
}

// ---------------------------------------------------------------------------
// Binning (XRT_KERNEL_BINNED), inside k_prep: each triangle's conservative
// footprint is assigned to the 32x32 regions it may touch, straight into
// fixed-capacity region lists -- slot = atomic increment of the region's
// count (line-padded counters, all of a lane's atomics in flight together),
// entry = (triangle, 16-bit mask of the region's 8x8 tiles its relaxed edges
// pass).  No scan and no second pass, so the whole preparation is one kernel.
// The capacity per region is sized from the largest count of the last frame
// of the same geometry (xrt_context::BinKey); a region past it renders from
// the whole mesh (exact, slower).  Footprints over more than kGlobalRegions
// regions go to a global list every region reads.
// ---------------------------------------------------------------------------
// Region counters touched by atomics are padded to one 128-B L2 line each:
// atomics on one line serialise, and neighbouring regions are hot together.
constexpr uint32_t kCounterStride = 32;
#ifndef XRT_BIN_BATCH
#define XRT_BIN_BATCH 4
#endif
#ifndef XRT_BIN_QUEUE
#define XRT_BIN_QUEUE 256
#endif
constexpr uint32_t kBinBatch = XRT_BIN_BATCH;  // queued pairs per lane per commit round (their atomics in flight together)
constexpr uint32_t kBinSmall = 64;           // region rectangles up to this many cells are flattened over the wave
constexpr uint32_t kBinQueue = XRT_BIN_QUEUE;  // passing (region, triangle) pairs queued per wave before a commit
// Launch slots of a k_prep wave's regions cached in LDS (0: off): when the
// union of the wave's region rectangles has at most this many cells, the
// wave DMAs their region -> slot entries into LDS before its cell tests, so
// the commit reads LDS instead of a dependent global load.
#ifndef XRT_PREP_RANK_LDS
#define XRT_PREP_RANK_LDS 0
#endif
constexpr uint32_t kRankCache = XRT_PREP_RANK_LDS;
static_assert(kRankCache % 64u == 0u, "whole DMA rounds");
// k_prep's commit through buffer instructions (range-checked, no per-lane
// branches around the memory ops; 0: plain guarded loads and atomics)
#ifndef XRT_PREP_BUFFER_OPS
#define XRT_PREP_BUFFER_OPS 1
#endif
// Per-wave aggregation of the commit's count atomics (0: off): when the union
// of the wave's region rectangles has at most kAggCells cells, the wave's pairs
// first count per cell in LDS (each pair's offset in its cell from an LDS
// atomic), then ONE global atomic per cell with pairs returns the cell's base
// -- a wave's triangles are mesh-adjacent, so its pairs share few regions.
#ifndef XRT_PREP_AGG
#define XRT_PREP_AGG 1
#endif
constexpr uint32_t kAggCells = 256;
static_assert(!(XRT_PREP_AGG && XRT_PREP_RANK_LDS), "one cell-indexed queue layout at a time");
static_assert(!XRT_PREP_AGG || XRT_PREP_BUFFER_OPS, "the aggregated commit uses the buffer-op tables");
// raw buffer atomic OR (no clang builtin for it; the LLVM intrinsic, whose
// no-return form is selected when the result is unused)
__device__ int buffer_atomic_or_i32(int v, __amdgpu_buffer_rsrc_t r, int off, int soff, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.atomic.or.i32");
constexpr int kBufferWord3 = 0x00020000;          // raw buffer resource, gfx9 family (32-bit elements)
constexpr uint32_t kBufferOut = 0x80000000u;      // an offset past every buffer: no-op access

// Counters and lists are indexed by launch slot, not by region: the render
// wave of slot s loads its count and list without first looking up which
// region it renders (order[s], loaded alongside); k_prep maps region -> slot
// through rank.
// Region-list entry: the triangle's conservative footprint, copied into every
// region list it joins, so a render wave's tile test reads a candidate with
// one coalesced 64-B load per lane and no indirection.  The record of a
// candidate that survives the tile test is read through its id (e0.w) straight
// into LDS by DMA (k_render_binned): only survivors' records move, and the
// lists k_prep writes and the render reads are half what an inlined record
// would make them (the 1.12 M-triangle frame bins 6.2 M entries).
struct alignas(16) RegionEntry {
    float4 e0;   // relaxed edge 0 (a, b, c); w = triangle id (bits)
    float4 e1;   // relaxed edge 1
    float4 e2;   // relaxed edge 2
    float4 bb;   // footprint box (xmin, xmax, ymin, ymax)
};
static_assert(sizeof(RegionEntry) == 64, "RegionEntry must be 64 bytes");
constexpr uint32_t kEntryQuads = sizeof(RegionEntry) / sizeof(float4);

// Read-only data of a launch (written by the host or an earlier kernel) read
// through the constant address space: scalar loads, issued together.
template <typename T>
using const_ptr = const __attribute__((address_space(4))) T*;
template <typename T>
__device__ __forceinline__ const_ptr<T> as_const(const T* p)
{
    return (const_ptr<T>)p;
}

// One launch slot's static description (host-built per region grid / frame
// geometry): its list is list[base .. base + cap), it renders region
// (x, y) = (xy & 0xFFFF, xy >> 16).  A tile wave reads it with ONE
// s_load_dwordx4 beside its count -- no dependent reads before its DMA.
struct SlotDesc {
    uint32_t base, cap, xy;
    // Tile plan: bit t = tile t of the region had a survivor in the frame the
    // plan was taken from (k_tile_plan; 0xFFFF = every tile live).  The cull of
    // a frame geometry is deterministic -- the same footprints join the same
    // region lists and pass the same tiles -- so a tile without a survivor in
    // one frame has none in any frame of that geometry, and the render stores
    // its misses without reading its region's list (BinBuffers::tile_plan).
    uint32_t live;
};
static_assert(sizeof(SlotDesc) == 16, "SlotDesc must be 16 bytes");

struct BinBuffers {
    uint32_t* counts;        // [n_regions * kCounterStride] by slot; cleared before every binned frame
    RegionEntry* list;       // the slots' lists (SlotDesc::base / cap)
    RegionEntry* global_list;   // [T] entries of the footprints over > kGlobalRegions regions
    const SlotDesc* desc;    // [n_regions] slot -> list and region, in the render's launch order
    const uint32_t* rank;    // [n_regions] region -> slot (desc's inverse)
    uint32_t regions_x, regions_y;
    uint32_t* clear;         // the other half's counters (its BinState line precedes them), cleared by k_prep
    uint32_t clear_regions;  // counters to clear there
    // Slots [0, tile_slots) render as tiles (16 waves a region); the rest are
    // the fill plan's empty regions (one workgroup each).  = regions: no plan.
    uint32_t tile_slots;
    // Slots [0, split_slots) (the heaviest regions of the plan's order) render
    // each tile with two waves, each testing half of the tile's survivors, the
    // halves' hit lists merged (k_render_binned); 0: none.
    uint32_t split_slots;
    // k_prep's flags (host-mapped memory, read by the host before it launches
    // the render): [0] = 1 when it bins a pair past tile_slots (the fill plan)
    // or a triangle into the global list, [1] = 1 when a region's count passes
    // its list's capacity.  Null: nothing to check.
    uint32_t* plan_miss;
    // 1: this frame's geometry is the one its layout's tile plan was taken for
    // (SlotDesc::live may skip tiles); 0: every tile renders.
    uint32_t tile_plan;
    // Device-sized frames (a moving camera): the count-only pass also appends
    // every pair as (slot, its index in the slot's list, triangle) to `pairs`
    // (BinState::pairs counts them, at most pairs_cap); k_scatter_pairs writes
    // the entries once k_size_lists has placed the lists.  Null: no pairs.
    uint4* pairs;
    uint32_t pairs_cap;
    // 1: the render's tile regions number BinState::tile_slots (a device fill
    // plan, k_size_lists: the slots with candidates first, then one fill
    // workgroup per empty region); its grid covers every region as tiles and
    // the workgroups past the plan's tiles and fills leave at once.
    uint32_t dev_plan;
    // 1: k_prep ORs each pair's box tile mask (span_tile_mask) into its slot's
    // counter line, and the render stores the misses of a tile outside its
    // slot's mask without reading the list (exact: no candidate's box meets
    // it).  0: neither (xrt_context::box_masks).
    uint32_t box_masks;
};

constexpr uint32_t kEmpty = 0xFFFFFFFFu;

// A render wave's first reads: its slot's count (k_prep's atomics) and its
// SlotDesc, issued back to back as scalar loads and awaited once.  One asm
// statement, so the compiler cannot put the count load behind a branch that
// consumes the description (two serial round trips).  slot is wave-uniform.
// The counter line of a slot: [0] its pair count, [1] its box tile mask (the
// OR over its pairs of box_tile_mask), both from k_prep's atomics.
__device__ __forceinline__ void load_slot(const BinBuffers& bins, uint32_t slot, uint32_t& count, uint32_t& mask,
                                          uint32_t& base, uint32_t& cap, uint32_t& xy, uint32_t& live)
{
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t* count_addr = bins.counts + (size_t)slot * kCounterStride;
    const SlotDesc* desc_addr = bins.desc + slot;
    u32x4 d;
    u32x2 c;
    asm volatile("s_load_dwordx2 %0, %2, 0x0\n\t"
                 "s_load_dwordx4 %1, %3, 0x0\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(c), "=&s"(d)
                 : "s"(count_addr), "s"(desc_addr)
                 : "memory");
    count = c.x;
    mask = c.y;
    base = d.x;
    cap = d.y;
    xy = d.z;
    live = d.w;
}

#ifndef XRT_TILE_MASK
#define XRT_TILE_MASK 1   // k_prep ORs each pair's box tile mask into its slot; the render skips tiles outside it
#endif
// The 8x8 tiles a footprint box meets by box_overlaps' test, as a span of
// strip tile columns and rows (tile column j: pixels 8j .. 8j + 7; tile row i:
// strip rows 8i .. 8i + 7): column j meets [xmin, xmax] iff j runs from
// ceil((xmin - 7) / 8) to floor(xmax / 8).  Rounded to nearest, the
// subtractions cannot cross a multiple of 8 (every integer here is a float),
// so the computed span never lies inside the exact one; NaN bounds give the
// widest span.  Packed (first + 4) | (last + 4) << 16 per axis, clamped to
// [-4, 32000] first.
__device__ __forceinline__ uint2 box_tile_span(float4 bb, uint32_t row_begin)
{
    const float rb = (float)row_begin;
    auto first = [](float v) { return (uint32_t)(fminf(fmaxf(ceilf(v * 0.125f), -4.0f), 32000.0f) + 4.0f); };
    auto last = [](float v) { return (uint32_t)(fmaxf(fminf(floorf(v * 0.125f), 32000.0f), -4.0f) + 4.0f); };
    return make_uint2(first(bb.x - 7.0f) | last(bb.y) << 16, first(bb.z - (rb + 7.0f)) | last(bb.w - rb) << 16);
}

// The tiles of region (rx, ry) in a box_tile_span: bit 4i + j for the
// region's tile row i, column j (render_tile's numbering).
__device__ __forceinline__ uint32_t span_tile_mask(uint2 span, uint32_t rx, uint32_t ry)
{
    const int dx = (int)(rx * 4u) + 4, dy = (int)(ry * 4u) + 4;
    const int j0 = min(max((int)(span.x & 0xFFFFu) - dx, 0), 4), j1 = min(max((int)(span.x >> 16) + 1 - dx, 0), 4);
    const int i0 = min(max((int)(span.y & 0xFFFFu) - dy, 0), 4), i1 = min(max((int)(span.y >> 16) + 1 - dy, 0), 4);
    const uint32_t cols = j1 > j0 ? (1u << j1) - (1u << j0) : 0u;
    const uint32_t rows = i1 > i0 ? (1u << (4 * i1)) - (1u << (4 * i0)) : 0u;
    return rows & (cols * 0x1111u);
}

#ifndef XRT_BIN_TIGHT
#define XRT_BIN_TIGHT 1   // the region rectangle of a footprint box: exactly the regions the box meets
#endif
// Region rectangle [x0,x1] x [y0,y1] (strip-relative region indices) that a
// footprint box may touch; false when it touches none.
__device__ __forceinline__ bool footprint_regions(float4 bb, const RenderParams& p,
                                                  const BinBuffers& bins, uint32_t& x0,
                                                  uint32_t& x1, uint32_t& y0, uint32_t& y1)
{
    if (!(bb.x <= bb.y) || !(bb.z <= bb.w)) return false;           // empty or NaN
    const float rows = (float)(p.row_end - p.row_begin);
    float xmin = fmaxf(bb.x, -64.0f), xmax = fminf(bb.y, (float)p.width + 64.0f);
    float ymin = fmaxf(bb.z - (float)p.row_begin, -64.0f), ymax = fminf(bb.w - (float)p.row_begin, rows + 64.0f);
    if (xmax < 0.0f || ymax < 0.0f || xmin > (float)p.width || ymin > rows) return false;
    // Region r covers columns [32r, 32r + 31] and meets the box (box_overlaps'
    // test) iff 32r + 31 >= xmin and 32r <= xmax: r from ceil((xmin - 31) / 32)
    // to floor(xmax / 32).  (Rounded to nearest, the subtractions cannot cross an
    // integer -- every integer here is a float -- so the computed first region is
    // never past the exact one.)  Round 1-5 took floor for the first one too: one
    // region column and row more than the box meets for nearly every footprint.
#if XRT_BIN_TIGHT
    int ix0 = (int)ceilf((xmin - 31.0f) * (1.0f / 32.0f));
    int iy0 = (int)ceilf((ymin - 31.0f) * (1.0f / 32.0f));
#else
    int ix0 = (int)floorf((xmin - 31.0f) * (1.0f / 32.0f));
    int iy0 = (int)floorf((ymin - 31.0f) * (1.0f / 32.0f));
#endif
    int ix1 = (int)floorf(xmax * (1.0f / 32.0f));
    int iy1 = (int)floorf(ymax * (1.0f / 32.0f));
    ix0 = max(ix0, 0);
    iy0 = max(iy0, 0);
    ix1 = min(ix1, (int)bins.regions_x - 1);
    iy1 = min(iy1, (int)bins.regions_y - 1);
    if (ix0 > ix1 || iy0 > iy1) return false;
    x0 = (uint32_t)ix0; x1 = (uint32_t)ix1; y0 = (uint32_t)iy0; y1 = (uint32_t)iy1;
    return true;
}

// Region rectangle of a footprint; false when the triangle is in no region
// list (no region, or in the global list -- `global` tells which).
__device__ __forceinline__ bool bin_rect(float4 bb, float reach, const RenderParams& p, const BinBuffers& bins,
                                         uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1,
                                         bool& global)
{
    global = false;
    if (!footprint_regions(bb, p, bins, x0, x1, y0, y1)) return false;
    // Past kGlobalRegions regions a footprint goes to the global list (every
    // region's candidate) -- unless the loosened triangle itself reaches few
    // regions (`reach`, compute_footprint: a sliver, whose box is much larger
    // than it), which are found by walking its box, up to
    // kGlobalRegionsUnbounded cells.  In the global list a sliver would leave
    // no region empty (no fill plan) and cost every region a staged candidate.
    const uint64_t cells = (uint64_t)(x1 - x0 + 1) * (y1 - y0 + 1);
    if (cells > kGlobalRegions && (cells > kGlobalRegionsUnbounded || !(reach <= (float)kGlobalRegions))) {
        global = true;
        return false;
    }
    return true;
}


// ---------------------------------------------------------------------------
// k_prep: one thread per triangle -- TriRec (Ray.cxx:86-122's ray-independent
// terms), cull planes and (binned) the triangle's region list entries.
// ---------------------------------------------------------------------------
// k_prep runs beside the previous frame's render: single-wave workgroups fit
// the holes that retiring render waves leave (a 4-wave one needs a free slot
// on all four SIMDs of a CU at once).
#ifndef XRT_PREP_PRIO
#define XRT_PREP_PRIO 0   // k_prep's wave priority (s_setprio; 0: the render's)
#endif
#ifndef XRT_PREP_LATE_STORES
#define XRT_PREP_LATE_STORES 1   // k_prep's global stores after its binning (1) or before it (0)
#endif
constexpr uint32_t kPrepThreads = XRT_PREP_THREADS;
constexpr uint32_t kPrepWaves = kPrepThreads / 64u;
#ifndef XRT_PREP_TRIS
#define XRT_PREP_TRIS 32
#endif
constexpr uint32_t kPrepTris = XRT_PREP_TRIS;     // triangles per k_prep wave (1..64) of small meshes
static_assert(kPrepTris >= 1u && kPrepTris <= 64u, "kPrepTris");
// Meshes of at least kPrepBigMesh triangles prepare 64 per wave: half the
// waves, each binning twice the pairs (1.12 M triangles at 8192^2: k_prep
// 922 -> 760 us beside the render, step 1,064 -> 1,056 us; 1024^2 dragon
// frames lose 1.6 us with 64, so small meshes keep kPrepTris).
constexpr uint32_t kPrepBigMesh = 1u << 18;
__host__ __device__ constexpr uint32_t prep_tris_for(uint64_t T) { return T >= kPrepBigMesh ? 64u : kPrepTris; }

__global__ __launch_bounds__(kPrepThreads) void k_prep(const float* __restrict__ tris, uint32_t T,
                                              RenderParams p, CullParams cp,
                                              TriRec* __restrict__ recs,
                                              float4* __restrict__ culls, BinBuffers bins,
                                              BinState* __restrict__ bs,
                                              RenderParams* __restrict__ frame_out,
                                              float* __restrict__ offsets_out,
                                              uint4* __restrict__ prep_times)
{
    // Diagnostics (xrt_debug_prep_times; null otherwise): per wave 8
    // s_memrealtime stamps -- [0] start, [1] triangle loaded and its record
    // formed, [2] footprint, [3] the binning's LDS staging and scan, [4] the
    // union of the wave's rectangles, [5] small rectangles' cells tested,
    // [6] large rectangles' cells tested (binning phase 1), [7] end.
    uint32_t ts[8] = {};
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if (prep_times) ts[k] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    auto stamp_end = [&]() __attribute__((always_inline)) {
        stamp(7);
        if (prep_times && (threadIdx.x & 63u) == 0u) {
            uint4* o = prep_times + 2 * (blockIdx.x * kPrepWaves + (threadIdx.x >> 6));
            o[0] = make_uint4(ts[0], ts[1], ts[2], ts[3]);
            o[1] = make_uint4(ts[4], ts[5], ts[6], ts[7]);
        }
    };
    // The preparation shares the CUs with earlier frames' renders (prep
    // stream) at the default wave priority: frames are prepared ahead of their
    // renders, and a raised priority only took issue slots from the render
    // (1024^2 step 29.0 -> 27.6 us without it).
    // i: the thread's index over the grid (pixel-offset tables, counter
    // clears); tri: its triangle -- p.prep_tris per wave (fewer than 64 spreads
    // the binning's cells and commits of a frame over more waves).
#if XRT_PREP_PRIO
    __builtin_amdgcn_s_setprio(XRT_PREP_PRIO);
#endif
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t tri_lane = threadIdx.x & 63u;
    const uint32_t tri = (blockIdx.x * kPrepWaves + (threadIdx.x >> 6)) * p.prep_tris + tri_lane;
    const bool valid = tri_lane < p.prep_tris && tri < T;
    // (the one wave that writes the frame's parameters does so at once: kept to
    // the end they would live in scratch)
    if (i == 0 && frame_out) *frame_out = p;       // the render's make_ray reads it (Outputs::frame)
    Footprint fp;
    TriRec r = {};
    if (valid) {
        const float* P = tris + 9ull * tri;
        float p1x = P[0], p1y = P[1], p1z = P[2];
        float p2x = P[3], p2y = P[4], p2z = P[5];
        float p3x = P[6], p3y = P[7], p3z = P[8];
        // Exactly the reference's f32 operations (Ray.cxx:86-87, 102, 112, 122).
        r.e1x = p2x - p1x; r.e1y = p2y - p1y; r.e1z = p2z - p1z;
        r.e2x = p3x - p1x; r.e2y = p3y - p1y; r.e2z = p3z - p1z;
        r.tvx = p.ox - p1x; r.tvy = p.oy - p1y; r.tvz = p.oz - p1z;
        r.qvx = r.tvy * r.e1z - r.tvz * r.e1y;
        r.qvy = r.tvz * r.e1x - r.tvx * r.e1z;
        r.qvz = r.tvx * r.e1y - r.tvy * r.e1x;
        r.tnum = (r.e2x * r.qvx + r.e2y * r.qvy) + r.e2z * r.qvz;
        r.pad0 = r.pad1 = r.pad2 = 0.0f;
        if (p.model == kModelSigned) {             // Triangle::computeNormal, Triangle.inl:170-178
            const float nx = r.e1y * r.e2z - r.e1z * r.e2y;
            const float ny = r.e1z * r.e2x - r.e1x * r.e2z;
            const float nz = r.e1x * r.e2y - r.e1y * r.e2x;
            const float len = sqrtf((nx * nx + ny * ny) + nz * nz);
            r.pad0 = nx / len;
            r.pad1 = ny / len;
            r.pad2 = nz / len;
        }
        stamp(1);
        if (culls) {
            fp = compute_footprint(r, p, cp);
            fp.e0.w = __uint_as_float(tri);          // the region entries carry the id (make_entry's layout)
        }
    }
    // The wave's global stores -- records, cull planes, the frame's pixel
    // offsets, the other counter half's clears -- are issued at its
    // END, after the binning: on gfx9 a store holds the vector-memory counter
    // until it is acknowledged, and the binning's first wait for a load (its
    // commit's slot loads, a loop's conservative wait) would otherwise wait
    // for every one of them (2048^2: ~1-2 us per wave beside the render).
    auto store_outputs = [&]() __attribute__((always_inline)) {
        if (offsets_out) {                         // v_off of every row, then u_off of every column
            if (i < p.height) offsets_out[i] = pixel_offset(p.spacing, i, p.height);
            else if (i - p.height < p.width) offsets_out[i] = pixel_offset(p.spacing, i - p.height, p.width);
        }
        if (valid) {
            recs[tri] = r;
            if (culls) {
                culls[tri] = fp.bbox;
                culls[(size_t)T + tri] = make_float4(fp.e0.x, fp.e0.y, fp.e0.z, 0.0f);
                culls[2 * (size_t)T + tri] = fp.e1;
                culls[3 * (size_t)T + tri] = fp.e2;
            }
        }
        if (bins.counts && bins.clear) {           // the other half, for the set's next frame
            if (i < bins.clear_regions)            // count and tile mask
                *reinterpret_cast<uint2*>(bins.clear + (size_t)i * kCounterStride) = make_uint2(0u, 0u);
            if (i < sizeof(BinState) / sizeof(uint32_t)) (bins.clear - kCounterStride)[i] = 0u;
        }
    };
#if !XRT_PREP_LATE_STORES
    store_outputs();                               // (A/B: the stores before the binning)
#endif
    stamp(2);
    if (!bins.counts) {                            // kernel-uniform
#if XRT_PREP_LATE_STORES
        store_outputs();
#endif
        stamp_end();
        return;
    }

    // Binning, per wave, in two phases.  (1) Test: every cell of the wave's
    // 64 region rectangles against its triangle's relaxed edges -- VALU and
    // LDS only; the cells of rectangles up to kBinSmall cells are flattened
    // over the wave (inclusive scan of the counts, a binary search per cell),
    // larger rectangles are walked by the whole wave one after the other --
    // and the passing (region, triangle) pairs appended to a wave-local queue.
    // (2) Commit: the queue dealt kBinBatch pairs per lane per round, each
    // round's launch slots, count atomics and entry stores in flight together.
    // A full queue is committed early.
    __shared__ float4 s_fp[kPrepWaves][kEntryQuads][64];   // the lane's region entry (footprint, e0.w = id)
    __shared__ uint2 s_rect[kPrepWaves][64];       // (x0 | x1 << 16, y0 | y1 << 16)
    __shared__ uint32_t s_cum[kPrepWaves][64];     // inclusive prefix of the small cell counts
    __shared__ uint32_t s_qreg[kPrepWaves][kBinQueue];   // passing pairs: region
    __shared__ uint8_t s_qown[kPrepWaves][kBinQueue];    //                owner lane
#if XRT_TILE_MASK
    __shared__ uint16_t s_qmask[kPrepWaves][kBinQueue];  //                box tile mask
    __shared__ uint2 s_tspan[kPrepWaves][64];      // the lane's box_tile_span
#endif
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x0 = 0, x1 = 0, y0 = 0, y1 = 0;
    bool global = false;
    const bool has = valid && bin_rect(fp.bbox, fp.e2.w, p, bins, x0, x1, y0, y1, global);
    if (valid && global) {                         // footprint over > kGlobalRegions regions
        if (bins.plan_miss) *bins.plan_miss = 1u;  // the plan assumed an empty global list
        RegionEntry* e = bins.global_list + atomicAdd(&bs->global_count, 1u);
        e->e0 = fp.e0;
        e->e1 = fp.e1;
        e->e2 = fp.e2;
        e->bb = fp.bbox;
    }
    const uint32_t cells = has ? (x1 - x0 + 1u) * (y1 - y0 + 1u) : 0u;
    const bool big = cells > kBinSmall;
    uint32_t cum = big ? 0u : cells;
#pragma unroll
    for (uint32_t off = 1; off < 64u; off <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)cum, off);
        if (lane >= off) cum += o;
    }
    const uint32_t total = wave_uniform((uint32_t)__builtin_amdgcn_readlane((int)cum, 63));
    s_fp[wave][0][lane] = fp.e0;
    s_fp[wave][1][lane] = fp.e1;
    s_fp[wave][2][lane] = fp.e2;
    s_fp[wave][3][lane] = fp.bbox;
    s_rect[wave][lane] = make_uint2(x0 | (x1 << 16), y0 | (y1 << 16));
#if XRT_TILE_MASK
    const bool masks = bins.box_masks != 0u;       // kernel-uniform
    if (masks) s_tspan[wave][lane] = box_tile_span(fp.bbox, p.row_begin);
#endif
    s_cum[wave][lane] = cum;
    // The slots of the union of the wave's rectangles (mesh-adjacent triangles
    // bin to neighbouring regions), DMAed into LDS under phase 1 when few.
    bool cached = false;
    uint32_t ux0 = 0, uy0 = 0, uw = 0;
#if XRT_PREP_RANK_LDS
    __shared__ uint32_t s_rank[kPrepWaves][kRankCache];
    if (__ballot(has) != 0ull) {
        ux0 = ~wave_reduce_u32<true>(has ? ~x0 : 0u);
        uy0 = ~wave_reduce_u32<true>(has ? ~y0 : 0u);
        const uint32_t ux1 = wave_reduce_u32<true>(has ? x1 : 0u);
        const uint32_t uy1 = wave_reduce_u32<true>(has ? y1 : 0u);
        uw = ux1 - ux0 + 1u;
        const uint32_t ucells = uw * (uy1 - uy0 + 1u);
        cached = ucells <= kRankCache;
        if (cached) {
            for (uint32_t c0 = 0; c0 < ucells; c0 += 64u) {
                const uint32_t c = c0 + lane;
                if (c < ucells)
                    __builtin_amdgcn_global_load_lds((const void*)(bins.rank + (uy0 + c / uw) * bins.regions_x + ux0 +
                                                                   c % uw),
                                                     (__attribute__((address_space(3))) void*)&s_rank[wave][c0], 4, 0,
                                                     0);
            }
        }
    }
#endif
    bool rank_waited = false;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    stamp(3);

#if XRT_PREP_AGG
    // the union of the wave's rectangles (wave-uniform)
    uint32_t ax0 = 0, ay0 = 0, aw = 0, acells = 0;
    if (__ballot(has) != 0ull) {
        ax0 = ~wave_reduce_u32<true>(has ? ~x0 : 0u);
        ay0 = ~wave_reduce_u32<true>(has ? ~y0 : 0u);
        const uint32_t ax1 = wave_reduce_u32<true>(has ? x1 : 0u);
        const uint32_t ay1 = wave_reduce_u32<true>(has ? y1 : 0u);
        aw = ax1 - ax0 + 1u;
        acells = aw * (ay1 - ay0 + 1u);
    }
    const bool agg = acells <= kAggCells;
    __shared__ uint32_t s_acnt[kPrepWaves][kAggCells];   // per cell: its pairs' count, then its base slot
    __shared__ uint32_t s_alb[kPrepWaves][kAggCells];    //           its list's base
    __shared__ uint32_t s_alc[kPrepWaves][kAggCells];    //           its list's capacity
    __shared__ uint8_t s_qoff[kPrepWaves][kBinQueue];    // per queued pair: its offset in its cell
    cached = agg;                                  // the queue holds cell indices (enqueue)
    ux0 = ax0;
    uy0 = ay0;
    uw = aw;
#endif
    // No lists (the sizing pass of a new geometry, DESIGN.md "List sizing"):
    // the pairs are counted, nothing is stored, nothing can overflow.
    stamp(4);
    const uint32_t count_only = wave_uniform(bins.list == nullptr ? 1u : 0u);
#if XRT_PREP_BUFFER_OPS
    // the commit's tables as buffers (range-checked: kBufferOut is past all of them)
    const uint32_t n_regions = bins.regions_x * bins.regions_y;
    const __amdgpu_buffer_rsrc_t r_rank =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(bins.rank), 0, (int)(n_regions * 4u), kBufferWord3);
    const __amdgpu_buffer_rsrc_t r_cnt =
        __builtin_amdgcn_make_buffer_rsrc(bins.counts, 0, (int)(n_regions * kCounterStride * 4u), kBufferWord3);
    const __amdgpu_buffer_rsrc_t r_desc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<SlotDesc*>(bins.desc), 0, (int)(n_regions * (uint32_t)sizeof(SlotDesc)), kBufferWord3);
#endif
    const uint32_t tri_base = (blockIdx.x * kPrepWaves + wave) * p.prep_tris;   // the triangle of lane 0
    uint32_t my_max = 0;                           // 1 + the largest slot this lane took
    bool over = false;                             // a slot past its list's capacity
    uint32_t queued = 0;                           // wave-uniform queue length
#if XRT_PREP_AGG
    // Device sizing (BinBuffers::pairs), aggregated commit: every queued pair
    // as (slot, its index in the slot's list, triangle) -- s_alb[c] holds the
    // cell's slot, s_acnt[c] its base index, s_qoff the pair's offset in its
    // cell -- appended to the frame's pair buffer, one atomic per wave.
    auto append_pairs = [&](bool) __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t at = 0;
        if (lane == 0u) at = atomicAdd(&bs->pairs, queued);
        at = (uint32_t)__builtin_amdgcn_readfirstlane((int)at);
        for (uint32_t q = lane; q < queued; q += 64u) {
            const uint32_t c = s_qreg[wave][q];
            if (at + q < bins.pairs_cap)
                bins.pairs[at + q] = make_uint4(s_alb[wave][c], s_acnt[wave][c] + s_qoff[wave][q],
                                                tri_base + s_qown[wave][q], 0u);
        }
    };
#endif
    auto commit = [&]() __attribute__((always_inline)) {
#if XRT_PREP_AGG
        if (agg) {
            // (a) per-cell counts in LDS; each pair's offset in its cell
            // (and per cell the OR of its pairs' tile masks, in s_alc until (b) reads it)
            for (uint32_t c = lane; c < acells; c += 64u) s_acnt[wave][c] = 0u;
#if XRT_TILE_MASK
            if (masks)
                for (uint32_t c = lane; c < acells; c += 64u) s_alc[wave][c] = 0u;
#endif
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t q = lane; q < queued; q += 64u) {
                s_qoff[wave][q] = (uint8_t)atomicAdd(&s_acnt[wave][s_qreg[wave][q]], 1u);
#if XRT_TILE_MASK
                if (masks) atomicOr(&s_alc[wave][s_qreg[wave][q]], (uint32_t)s_qmask[wave][q]);
#endif
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // (b) one count atomic per cell with pairs: every cell's slot loads,
            // then every atomic and list description, in flight together
            constexpr uint32_t kAggRounds = kAggCells / 64u;
            uint32_t cn[kAggRounds], cs[kAggRounds], cb[kAggRounds], clb[kAggRounds], clc[kAggRounds];
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k) {
                const uint32_t c = k * 64u + lane;
                cn[k] = c < acells ? s_acnt[wave][c] : 0u;
                const uint32_t region = (ay0 + c / max(aw, 1u)) * bins.regions_x + ax0 + c % max(aw, 1u);
                cs[k] = __builtin_amdgcn_raw_buffer_load_b32(r_rank, cn[k] ? region * 4u : kBufferOut, 0, 0);
            }
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k) cs[k] = cn[k] ? cs[k] : kEmpty;
#if XRT_TILE_MASK
            uint32_t cm[kAggRounds];               // the cells' tile masks
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k) cm[k] = masks ? s_alc[wave][k * 64u + lane] : 0u;
#endif
            bool planned_empty = false;            // pairs for a region the fill plan fills
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k) planned_empty |= cs[k] != kEmpty && cs[k] >= bins.tile_slots;
            if (__builtin_expect(bins.plan_miss != nullptr && __ballot(planned_empty) != 0ull, 0) && lane == 0)
                *bins.plan_miss = 1u;
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k)
                cb[k] = (uint32_t)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(
                    (int)cn[k], r_cnt, cs[k] != kEmpty ? cs[k] * (kCounterStride * 4u) : kBufferOut, 0, 0);
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k) {
                const auto bc = __builtin_amdgcn_raw_buffer_load_b64(
                    r_desc, cs[k] != kEmpty && count_only == 0u ? cs[k] * (uint32_t)sizeof(SlotDesc) : kBufferOut, 0,
                    0);
                clb[k] = bc[0];
                clc[k] = bc[1];
            }
#if XRT_TILE_MASK
            // the masks' atomics last (no return value; issued after the loads and
            // atomics whose results the wave waits for, they do not delay them)
            if (masks) {
#pragma unroll
                for (uint32_t k = 0; k < kAggRounds; ++k)
                    buffer_atomic_or_i32((int)cm[k], r_cnt,
                                         cs[k] != kEmpty ? cs[k] * (kCounterStride * 4u) + 4u : kBufferOut, 0, 0);
            }
#endif
            if (count_only) {                       // the sizing pass: counts only
                if (bins.pairs) {                   // (device sizing: and the pairs)
#pragma unroll
                    for (uint32_t k = 0; k < kAggRounds; ++k) {
                        const uint32_t c = k * 64u + lane;
                        if (cs[k] != kEmpty) {
                            s_acnt[wave][c] = cb[k];
                            s_alb[wave][c] = cs[k];
                        }
                    }
                    append_pairs(true);
                }
                __builtin_amdgcn_wave_barrier();
                queued = 0;
                return;
            }
#pragma unroll
            for (uint32_t k = 0; k < kAggRounds; ++k) {
                const uint32_t c = k * 64u + lane;
                if (cs[k] == kEmpty) continue;
                my_max = max(my_max, cb[k] + cn[k]);
                if (cb[k] + cn[k] > clc[k]) over = true;
                s_acnt[wave][c] = cb[k];
                s_alb[wave][c] = clb[k];
                s_alc[wave][c] = clc[k];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // (c) the entries
            for (uint32_t q = lane; q < queued; q += 64u) {
                const uint32_t c = s_qreg[wave][q];
                const uint32_t idx = s_acnt[wave][c] + s_qoff[wave][q];
                if (idx < s_alc[wave][c]) {
                    float4* e = reinterpret_cast<float4*>(bins.list + (size_t)s_alb[wave][c] + idx);
                    const uint32_t own = s_qown[wave][q];
#pragma unroll
                    for (uint32_t w = 0; w < kEntryQuads; ++w) e[w] = s_fp[wave][w][own];
                }
            }
            __builtin_amdgcn_wave_barrier();      // the queue is refilled after every lane read it
            queued = 0;
            return;
        }
#endif
#if XRT_PREP_RANK_LDS
        if (cached && !rank_waited) {              // the slots' DMA has landed (issued before phase 1)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            rank_waited = true;
        }
#endif
        for (uint32_t base = 0; base < queued; base += 64u * kBinBatch) {
            uint32_t reg[kBinBatch], own[kBinBatch], slot[kBinBatch];
#if XRT_PREP_BUFFER_OPS
            // Buffer loads and atomics with an out-of-range offset for the lanes
            // without a pair (a load returns 0, an atomic does nothing): no
            // exec-masked branch around each memory op, so the round's four
            // slot loads issue back to back, then its four count atomics and four
            // list descriptions -- two memory round trips a round.  (The guarded
            // form compiled to a wait after every load and every atomic: eight.)
            bool val[kBinBatch];
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) {
                const uint32_t q = base + b * 64u + lane;
                val[b] = q < queued;
                const uint32_t qq = q < kBinQueue ? q : kBinQueue - 1u;   // in the array; ignored unless val
                reg[b] = s_qreg[wave][qq];
                own[b] = s_qown[wave][qq];
            }
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) {
#if XRT_PREP_RANK_LDS
                if (cached) reg[b] = val[b] ? s_rank[wave][reg[b]] : kEmpty;
                else
#endif
                reg[b] = __builtin_amdgcn_raw_buffer_load_b32(r_rank, val[b] ? reg[b] * 4u : kBufferOut, 0, 0);
            }
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) reg[b] = val[b] ? reg[b] : kEmpty;
#else
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) {
                const uint32_t q = base + b * 64u + lane;
                reg[b] = kEmpty;
                own[b] = 0u;
                if (q < queued) {
#if XRT_PREP_RANK_LDS
                    reg[b] = cached ? s_rank[wave][s_qreg[wave][q]] : bins.rank[s_qreg[wave][q]];
#else
                    reg[b] = bins.rank[s_qreg[wave][q]];
#endif
                    own[b] = s_qown[wave][q];
                }
            }
#endif
            bool planned_empty = false;            // a pair for a region the fill plan fills
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) planned_empty |= reg[b] != kEmpty && reg[b] >= bins.tile_slots;
            if (__builtin_expect(bins.plan_miss != nullptr && __ballot(planned_empty) != 0ull, 0) && lane == 0)
                *bins.plan_miss = 1u;
            uint32_t lbase[kBinBatch], lcap[kBinBatch];
#if XRT_PREP_BUFFER_OPS
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b)
                slot[b] = (uint32_t)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(
                    1, r_cnt, reg[b] != kEmpty ? reg[b] * (kCounterStride * 4u) : kBufferOut, 0, 0);
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) {
                const auto bc = __builtin_amdgcn_raw_buffer_load_b64(
                    r_desc, reg[b] != kEmpty && count_only == 0u ? reg[b] * (uint32_t)sizeof(SlotDesc) : kBufferOut, 0, 0);
                lbase[b] = bc[0];
                lcap[b] = bc[1];
            }
#if XRT_TILE_MASK
            if (masks) {
#pragma unroll
                for (uint32_t b = 0; b < kBinBatch; ++b) {   // the pairs' tile masks, last (no return value)
                    const uint32_t q = base + b * 64u + lane;
                    buffer_atomic_or_i32((int)s_qmask[wave][q < kBinQueue ? q : 0u], r_cnt,
                                         reg[b] != kEmpty ? reg[b] * (kCounterStride * 4u) + 4u : kBufferOut, 0, 0);
                }
            }
#endif
#else
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) {
                slot[b] = reg[b] != kEmpty ? atomicAdd(&bins.counts[(size_t)reg[b] * kCounterStride], 1u) : 0u;
#if XRT_TILE_MASK
                if (masks && reg[b] != kEmpty)
                    atomicOr(&bins.counts[(size_t)reg[b] * kCounterStride + 1u],
                             (uint32_t)s_qmask[wave][min(base + b * 64u + lane, kBinQueue - 1u)]);
#endif
                const uint2 bc = reg[b] != kEmpty && count_only == 0u
                                     ? *reinterpret_cast<const uint2*>(bins.desc + reg[b]) : make_uint2(0u, 0u);
                lbase[b] = bc.x;
                lcap[b] = bc.y;
            }
#endif
            if (count_only) {                      // the sizing pass: counts only
                if (bins.pairs) {                  // (device sizing: and the pairs)
#pragma unroll
                    for (uint32_t b = 0; b < kBinBatch; ++b) {
                        const unsigned long long vm = __ballot(reg[b] != kEmpty);
                        uint32_t at = 0;
                        if (lane == 0u && vm) at = atomicAdd(&bs->pairs, (uint32_t)__popcll(vm));
                        at = (uint32_t)__builtin_amdgcn_readfirstlane((int)at);
                        if (reg[b] != kEmpty) {
                            const uint32_t q = at + __builtin_amdgcn_mbcnt_hi((uint32_t)(vm >> 32),
                                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)vm, 0u));
                            if (q < bins.pairs_cap)
                                bins.pairs[q] = make_uint4(reg[b], slot[b], tri_base + own[b], 0u);
                        }
                    }
                }
                continue;
            }
#pragma unroll
            for (uint32_t b = 0; b < kBinBatch; ++b) {
                if (reg[b] == kEmpty) continue;
                my_max = max(my_max, slot[b] + 1u);
                if (slot[b] >= lcap[b]) over = true;
                else {
                    float4* e = reinterpret_cast<float4*>(bins.list + (size_t)lbase[b] + slot[b]);
#pragma unroll
                    for (uint32_t w = 0; w < kEntryQuads; ++w) e[w] = s_fp[wave][w][own[b]];
                }
            }
        }
        __builtin_amdgcn_wave_barrier();          // the queue is refilled after every lane read it
        queued = 0;
    };
    // append the passing cells of one round (pass, region rx/ry, owner) to the queue
    auto enqueue = [&](bool pass, uint32_t rx, uint32_t ry, uint32_t owner) {
        const unsigned long long m = __ballot(pass);
        if (!m) return;
        if (queued + 64u > kBinQueue) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            commit();
        }
        if (pass) {
            const uint32_t q = queued + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            // the cached slot's index, or the region
            s_qreg[wave][q] = cached ? (ry - uy0) * uw + (rx - ux0) : ry * bins.regions_x + rx;
            s_qown[wave][q] = (uint8_t)owner;
#if XRT_TILE_MASK
            if (masks) s_qmask[wave][q] = (uint16_t)span_tile_mask(s_tspan[wave][owner], rx, ry);
#endif
        }
        queued += (uint32_t)__popcll(m);
    };
    auto cell_pass = [&](uint32_t owner, uint32_t rx, uint32_t ry) {
        const float xc = (float)(rx * kRegion) + 15.5f;
        const float yc = (float)(p.row_begin + ry * kRegion) + 15.5f;
        return edges_pass_region(s_fp[wave][0][owner], s_fp[wave][1][owner], s_fp[wave][2][owner], xc, yc);
    };
    // (1a) small rectangles, flattened over the wave
    for (uint32_t base = 0; base < total; base += 64u) {
        const uint32_t c = base + lane;
        bool pass = false;
        uint32_t rx = 0, ry = 0, lo = 0;
        if (c < total) {
            uint32_t hi = 63u;                        // the first lane whose prefix exceeds c
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_cum[wave][mid] > c) hi = mid; else lo = mid + 1u;
            }
            const uint2 rc = s_rect[wave][lo];
            const uint32_t bx0 = rc.x & 0xFFFFu, bw = (rc.x >> 16) - bx0 + 1u, by0 = rc.y & 0xFFFFu;
            const uint32_t k = c - (lo ? s_cum[wave][lo - 1u] : 0u);
            rx = bx0 + k % bw;
            ry = by0 + k / bw;
            pass = cell_pass(lo, rx, ry);
        }
        enqueue(pass, rx, ry, lo);
    }
    stamp(5);
    // (1b) large rectangles, one at a time over the whole wave
    unsigned long long mbig = __ballot(big);
    while (mbig) {                                 // wave-uniform
        const uint32_t owner = (uint32_t)__builtin_ctzll(mbig);
        mbig &= mbig - 1ull;
        const uint2 rc = s_rect[wave][owner];
        const uint32_t bx0 = rc.x & 0xFFFFu, bw = (rc.x >> 16) - bx0 + 1u, by0 = rc.y & 0xFFFFu;
        const uint32_t n = wave_uniform(bw * ((rc.y >> 16) - by0 + 1u));
        for (uint32_t base = 0; base < n; base += 64u) {
            const uint32_t k = base + lane;
            const uint32_t rx = bx0 + k % bw, ry = by0 + k / bw;
            enqueue(k < n && cell_pass(owner, rx, ry), rx, ry, owner);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    stamp(6);
    commit();                                      // (2)
    // A region count past the list capacity: the render of that region falls
    // back to the whole mesh, and the host grows the lists for the next frame
    // (xrt_read_stats / the sizing read).  No global atomic otherwise.
    my_max = wave_reduce_u32<true>(my_max);
    if (__ballot(over) && lane == 0) {
        atomicMax(&bs->max_count, my_max);
        atomicOr(&bs->overflow, 1u);
        if (bins.plan_miss) bins.plan_miss[1] = 1u;  // the host re-sizes for the next frame
    }
#if XRT_PREP_LATE_STORES
    store_outputs();
#endif
    stamp_end();
}

// ---------------------------------------------------------------------------
// k_size_lists: the list sizing of a moving camera's frame on the device
// (DESIGN.md "Moving camera"), after k_prep's count-only pass (which appended
// its pairs) and before k_scatter_pairs -- no host round trip.  Each slot of
// the launch layout `fixed` (its order and regions) gets room for exactly the
// pairs the count pass counted, carved from the set's pool by one atomic per
// wave (BinState::cursor; the lists need not follow the slot order); the
// counters stay (the render reads them).  A slot past the pool gets what is
// left (its overflow makes the render take that region from the whole mesh,
// exactly, and flags the frame: the host grows the pool for later frames).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_size_lists(uint32_t* __restrict__ counts, const SlotDesc* __restrict__ fixed,
                                                   SlotDesc* __restrict__ out, uint32_t n_slots, uint32_t pool,
                                                   BinState* __restrict__ bs, SlotDesc* __restrict__ plan_desc,
                                                   uint32_t* __restrict__ plan_counts)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = s < n_slots ? counts[(size_t)s * kCounterStride] : 0u;
    // The device fill plan (BinBuffers::dev_plan; plan_desc null: none): the
    // render's layout lists the slots with candidates first (tiles), then the
    // empty ones (one fill workgroup each) -- empty only when the global list
    // is empty too.  Counts (and box tile masks) follow into that order.
    uint32_t pos = 0;
    if (plan_desc) {
        const bool empty = c == 0u && as_const(bs)->global_count == 0u;
        const unsigned long long m_tile = __ballot(s < n_slots && !empty), m_fill = __ballot(s < n_slots && empty);
        uint32_t t0 = 0, f0 = 0;
        if (lane == 0u) {
            if (m_tile) t0 = atomicAdd(&bs->tile_slots, (uint32_t)__popcll(m_tile));
            if (m_fill) f0 = atomicAdd(&bs->fill_slots, (uint32_t)__popcll(m_fill));
        }
        t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)t0);
        f0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)f0);
        const unsigned long long mine = empty ? m_fill : m_tile;
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
        pos = empty ? n_slots - 1u - (f0 + r) : t0 + r;
    }
    uint32_t incl = c;
#pragma unroll
    for (uint32_t off = 1; off < 64u; off <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)incl, off);
        if (lane >= off) incl += o;
    }
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    uint32_t base0 = 0;
    if (lane == 0u && total) base0 = atomicAdd(&bs->cursor, total);
    base0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)base0);
    // More pairs than the pair buffer holds (its capacity is the pool's): the
    // lost pairs may belong to any slot, so no list is known complete -- every
    // region with a pair renders from the whole mesh (exact) and the frame is
    // flagged (k_scatter_pairs).
    const bool lost = as_const(bs)->pairs > pool;
    if (s < n_slots) {
        const uint32_t base = base0 + incl - c;
        const uint32_t cap = lost || base >= pool ? 0u : min(c, pool - base);
        const SlotDesc d = SlotDesc{min(base, pool), cap, fixed[s].xy, 0xFFFFu};
        out[s] = d;
        if (plan_desc) {
            plan_desc[pos] = d;
            *reinterpret_cast<uint2*>(plan_counts + (size_t)pos * kCounterStride) =
                make_uint2(c, counts[(size_t)s * kCounterStride + 1u]);
        }
    }
}

// k_scatter_pairs: the entries of a device-sized frame (after k_size_lists):
// pair i = (slot, index in the slot's list, triangle) from k_prep's count pass
// becomes the triangle's region entry -- its footprint from the frame's cull
// planes, e0.w = its id -- at list[base(slot) + index].  A pair past its list's
// capacity (the pool ran out) is dropped and flagged: that region's count
// exceeds its capacity, so the render takes it from the whole mesh (exact).
__global__ __launch_bounds__(256) void k_scatter_pairs(const uint4* __restrict__ pairs, const BinState* __restrict__ bs,
                                                      uint32_t pairs_cap, const SlotDesc* __restrict__ desc,
                                                      const float4* __restrict__ culls, uint32_t T,
                                                      RegionEntry* __restrict__ list, uint32_t* __restrict__ flag)
{
    const uint32_t total = as_const(bs)->pairs;
    const uint32_t n = min(total, pairs_cap);
    if (blockIdx.x == 0u && threadIdx.x == 0u && total > pairs_cap && flag) flag[1] = 1u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint4 pr = pairs[i];
        const SlotDesc d = desc[pr.x];
        if (pr.y >= d.cap) {
            if (flag) flag[1] = 1u;
            continue;
        }
        float4 e0 = culls[(size_t)T + pr.z];
        e0.w = __uint_as_float(pr.z);
        float4* e = reinterpret_cast<float4*>(list + (size_t)d.base + pr.y);
        e[0] = e0;
        e[1] = culls[2 * (size_t)T + pr.z];
        e[2] = culls[3 * (size_t)T + pr.z];
        e[3] = culls[pr.z];
    }
}

// ---------------------------------------------------------------------------
// k_render_binned: the render over the binned region lists.
//
// A workgroup of kTileWaves waves renders kTileWaves of a region's 8x8 tiles,
// one tile per wave, and every wave works on its own (render_tile): the
// region's candidates -- its list entries followed by the global list's,
// 64-B footprints -- are read by the wave into registers, one per lane per
// round, and only the survivors of the tile test move their triangle records
// (into the wave's LDS stage, by DMA).  Round 3 staged every candidate's
// footprint and record (128 B) through a workgroup-shared stage: every wave
// of a workgroup waited at two barriers per round for the slowest, and a tile
// without survivors still paid the records' DMA.  Rays are generated when the
// first survivor appears (pixel offsets from the frame's tables); a tile
// without survivors stores the miss constants.
// ---------------------------------------------------------------------------
constexpr uint32_t kTileWaves = XRT_TILE_WAVES;         // tile waves per workgroup
constexpr uint32_t kWavesPerRegion = 16u;               // one 8x8 tile per wave
// Candidates a tile wave culls per round: kRoundSlots per lane, their
// footprints loaded together; the survivors of each 64 then have their
// records staged in the wave's own LDS (64 B each) and tested.
constexpr uint32_t kBinStage = XRT_STAGE;
constexpr uint32_t kRoundSlots = kBinStage / 64u;
static_assert(kBinStage % 64u == 0u && kRoundSlots >= 1u && kRoundSlots <= 4u, "64 to 256 candidates per round");
static_assert(16u % kTileWaves == 0u, "a workgroup's waves render tiles of one region");

// One tile wave's staged records: q[0..3][L] = the TriRec of lane L's
// candidate, written by that lane's DMA when the candidate survived the tile
// test, read back as a broadcast by the survivor loop.  Private to the wave:
// no workgroup barrier anywhere in the render.
struct RecStage {
    float4 q[4][64];
};
// LDS of one render workgroup (k_prep's residency cap is derived from it, xrt_abi.hip)
constexpr uint32_t kRenderLdsPerWave = sizeof(RecStage);

// The survivors of one round slot into st: each survivor lane (`pass`) DMAs
// its candidate's record (`id`) to q[*][lane].  Wave-private, so a vmcnt
// wait makes them readable.
__device__ __forceinline__ void stage_survivor_records(RecStage& st, const TriRec* __restrict__ recs, bool pass,
                                                       uint32_t id)
{
    if (pass) {
        const float4* src = reinterpret_cast<const float4*>(recs + id);
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q)
            __builtin_amdgcn_global_load_lds((const void*)(src + q),
                                             (__attribute__((address_space(3))) void*)&st.q[q][0], 16, 0, 0);
    }
}

#ifndef XRT_PUSH_BALLOT
#define XRT_PUSH_BALLOT 1
#endif
// TriRec: e1 (a0.xyz), e2 (a0.w, a1.xy), tvec (a1.zw, a2.x), qvec (a2.yzw), tnum (q[3].x)
__device__ __forceinline__ void test_rec(float4 a0, float4 a1, float4 a2, float tnum, float dx, float dy, float dz,
                                         HitList& hl)
{
    float det, u, v;
    mt_numerators(dx, dy, dz, a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w, a2.x, a2.y, a2.z, a2.w,
                  det, u, v);
    // the short reciprocal on every survivor, the IEEE division only behind one
    // rarely taken wave-uniform branch (straight-line common path)
    float inv = rcp_newton(det);
    if (__builtin_expect(__ballot(!rcp_newton_exact_for(det)) != 0ull, 0)) inv = inv_det_of(det);
    bool h;
    const float t = mt_finish_inv(det, inv, u, v, tnum, h);
#if XRT_PUSH_BALLOT
    // a survivor of the conservative tile cull often hits none of the tile's
    // rays: its insert (kMaxHits v_med3) skipped behind one wave-uniform branch
    if (__ballot(h)) hl.push_if(h, t);
#else
    hl.push_if(h, t);
#endif
}

__device__ __forceinline__ void test_staged_one(const RecStage& st, uint32_t k, float dx, float dy, float dz,
                                                HitList& hl)
{
    test_rec(st.q[0][k], st.q[1][k], st.q[2][k], st.q[3][k].x, dx, dy, dz, hl);
}


// The signed model's: the term's sign from the record's unit normal (pad0..2),
// `id` the candidate's triangle id (wave-uniform).
__device__ __forceinline__ void test_staged_one(const RecStage& st, uint32_t k, uint32_t id, float dx, float dy,
                                                float dz, float sx, float sy, float sz, SignedHits& hl)
{
    const float4 a0 = st.q[0][k], a1 = st.q[1][k], a2 = st.q[2][k], a3 = st.q[3][k];
    float det, u, v;
    mt_numerators(dx, dy, dz, a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w, a2.x, a2.y, a2.z, a2.w,
                  det, u, v);
    bool h;
    const float t = mt_finish(det, u, v, a3.x, h);
    if (__ballot(h)) hl.push_if(h, t, id, hit_sign(sx, sy, sz, a3.y, a3.z, a3.w));
}

// The tile test of candidate k, from its list entry (the overflow fix-up's
// survivors; a region rendered from the whole mesh takes the whole-candidate
// fix-up).  The tile rectangle is recomputed from its corner here rather than
// kept live from the loop.
struct EntryCull {
    const RegionEntry* __restrict__ local;
    const RegionEntry* __restrict__ glob;
    uint32_t n_local, tx0, ty0;
    bool enabled;
    __device__ bool operator()(uint32_t k) const
    {
        uint32_t x = tx0, y = ty0;
        asm volatile("" : "+s"(x), "+s"(y));
        const float fx0 = (float)x, fy0 = (float)y;
        const RegionEntry& e = k < n_local ? local[k] : glob[k - n_local];
        return edges_pass_tile(e.e0, e.e1, e.e2, fx0 + 3.5f, fy0 + 3.5f) &
               box_overlaps(e.bb, fx0, fx0 + 7.0f, fy0, fy0 + 7.0f);
    }
};

// One wave's 8x8 tile `tile` of the region in launch slot `slot`: the body of
// k_render_binned.  The wave works alone: per round, each lane loads one
// candidate's footprint (its region-list entry, 64 B, or the whole mesh's cull
// planes) into registers and tests the tile rectangle against it, a ballot
// keeps the survivors, each survivor lane DMAs its candidate's record into the
// wave's LDS stage, and each survivor is tested exactly for the tile's 64
// rays from a broadcast LDS read.  A tile whose candidates all fail never
// touches a record; no wave waits for another.  The statistics accumulate in
// ws, and `cand` gets the region's candidate count.
// Split tiles (BinBuffers::split_slots): the two waves of a tile cull the same
// candidates (same ballots, so both see the same rounds with survivors and
// both generate the rays) and test alternate survivors -- half 1 the survivors
// in odd lanes, half 0 the even ones.  Half 1 then publishes its sorted hit
// list, its hit count and its test count in its own LDS stage; after one
// workgroup barrier half 0 inserts them into its own list (the union of two
// sorted lists is the ray's sorted hit set when the counts fit the list, and
// a count past it takes the exact fix-up as any overflowed ray does) and
// finishes the tile alone.  kSplitNone: an ordinary tile.
constexpr uint32_t kSplitNone = 0u, kSplitHalf0 = 1u, kSplitHalf1 = 2u;
constexpr bool kCanSplit = kTileWaves % 2u == 0u;   // a tile's two waves share a workgroup
static_assert(kMaxHits <= 12, "a half's hit list fits three float4 of its stage");

__device__ __forceinline__ void publish_half(RecStage& st, const HitList& hl, uint32_t tests)
{
    const uint32_t lane = threadIdx.x & 63u;
    float v[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) v[k] = k < kMaxHits ? hl.h[k < kMaxHits ? k : 0] : __builtin_inff();
    st.q[0][lane] = make_float4(v[0], v[1], v[2], v[3]);
    st.q[1][lane] = make_float4(v[4], v[5], v[6], v[7]);
    st.q[2][lane] = make_float4(v[8], v[9], v[10], v[11]);
    st.q[3][lane] = make_float4(__uint_as_float(hl.n), __uint_as_float(tests), 0.0f, 0.0f);
}

__device__ __forceinline__ void merge_half(const RecStage& other, HitList& hl, uint32_t& tests)
{
    const uint32_t lane = threadIdx.x & 63u;
    const float4 a = other.q[0][lane], b = other.q[1][lane], c = other.q[2][lane], d = other.q[3][lane];
    const float v[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    const uint32_t n1 = __float_as_uint(d.x), n0 = hl.n;
#pragma unroll
    for (int k = 0; k < kMaxHits; ++k) hl.push_if((uint32_t)k < n1, v[k]);
    hl.n = n0 + n1;                                // past the list: the overflow fix-up recomputes the ray
    tests += wave_uniform(__float_as_uint(d.y));
}

template <bool kSigned, bool kHits>
__device__ __forceinline__ void render_tile(RecStage& st, const TriRec* __restrict__ recs,
                                            const float4* __restrict__ culls, const RenderParams& p,
                                            const Outputs& out, const BinBuffers& bins, uint32_t n_glob,
                                            uint32_t slot, uint32_t tile, WaveStats& ws, uint32_t& cand,
                                            uint32_t split = kSplitNone, const RecStage* partner = nullptr)
{
    const uint32_t lane = threadIdx.x & 63u;
    // the slot's count (k_prep) and description (host): two scalar loads in flight together
    uint32_t n_local, box_mask, d_base, d_cap, d_xy, d_live;
    load_slot(bins, slot, n_local, box_mask, d_base, d_cap, d_xy, d_live);
    const uint32_t reg_x = d_xy & 0xFFFFu, reg_y = d_xy >> 16;
    const RegionEntry* __restrict__ local = bins.list + d_base;
    const RegionEntry* __restrict__ glob = bins.global_list;
    const uint32_t T = p.num_triangles;
    const bool whole = n_local > d_cap;   // the list overflowed: whole mesh (exact, slower)
    const uint32_t n_cand = whole ? T : n_local + n_glob;
    cand = n_cand;

    const uint32_t tx0 = reg_x * kRegion + (tile & 3u) * 8u;
    const uint32_t ty0 = p.row_begin + reg_y * kRegion + (tile >> 2) * 8u;
    const bool tile_live = tx0 < p.width && ty0 < p.row_end;       // wave-uniform
    const uint32_t col = tx0 + (lane & 7u);
    const uint32_t row = ty0 + (lane >> 3);
    const bool active = col < p.width && row < p.row_end;
    const float xc = (float)tx0 + 3.5f, yc = (float)ty0 + 3.5f;
    const float fx0 = (float)tx0, fx1 = (float)tx0 + 7.0f, fy0 = (float)ty0, fy1 = (float)ty0 + 7.0f;
    // the lane's output element: row-major in the strip, or in its slot's packed
    // block; the hit layout's hit_element
    constexpr bool hits = kHits;
    const size_t o = hits ? hit_element(out, slot * kWavesPerRegion + tile)
                   : out.packed ? (size_t)slot * kPackBlock + ((tile >> 2) * 8u + (lane >> 3)) * kRegion +
                                      (tile & 3u) * 8u + (lane & 7u)
                                : (size_t)(row - p.row_begin) * p.width + col;
    if (!tile_live) {
        if (hits && split != kSplitHalf1) store_hit_tile(out, o, false, 0.0f);
        if (split != kSplitNone) __syncthreads();  // the pair's one barrier (workgroup-uniform count)
        return;
    }
    // a tile the geometry's tile plan found without survivors: its misses,
    // without reading the region's list (exact: SlotDesc::live)
    // A tile no candidate's footprint box meets (the region's box tile mask,
    // k_prep's OR over its pairs; the global list's entries are not in it):
    // no candidate can pass its tile test -- its misses, the same way.  Both
    // halves of a split tile skip alike.
    const bool planned_dead = (!kSigned && bins.tile_plan && split == kSplitNone && !((d_live >> tile) & 1u))
#if XRT_TILE_MASK
                              || (bins.box_masks && n_glob == 0u && !((box_mask >> tile) & 1u))
#endif
        ;

    float dx = 1.0f, dy = 0.0f, dz = 0.0f;
    float sx = 1.0f, sy = 0.0f, sz = 0.0f;         // kSigned: the once-normalised direction
    bool have_ray = false;                         // wave-uniform
    // the tile's pixel offsets, loaded beside the first footprints: a tile with
    // survivors generates its rays without another memory round trip
    const float pre_v = out.off.v[min(row, p.height - 1u)];
    const float pre_u = out.off.u[min(col, p.width - 1u)];
    typename std::conditional<kSigned, SignedHits, HitList>::type hl;
    hl.init();
    uint32_t tests = 0;
    for (uint32_t base = 0; base < (planned_dead ? 0u : n_cand); base += kBinStage) {
        // the round's footprints, kRoundSlots per lane, all loads in flight together
        float4 f[kRoundSlots][4];
        uint32_t id[kRoundSlots];
#pragma unroll
        for (uint32_t r = 0; r < kRoundSlots; ++r) {
            const uint32_t k = base + r * 64u + lane;
            id[r] = k;
            f[r][0] = f[r][1] = f[r][2] = make_float4(0.0f, 0.0f, -1.0f, 0.0f);   // fails the edges
            f[r][3] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (k < n_cand) {
                if (whole) {                       // SoA cull planes: box, then edges 0..2
                    f[r][0] = culls[(size_t)T + k];
                    f[r][1] = culls[2 * (size_t)T + k];
                    f[r][2] = culls[3 * (size_t)T + k];
                    f[r][3] = culls[k];
                } else {
                    const float4* e = reinterpret_cast<const float4*>(k < n_local ? local + k : glob + (k - n_local));
                    f[r][0] = e[0];
                    f[r][1] = e[1];
                    f[r][2] = e[2];
                    f[r][3] = e[3];
                }
            }
        }
        // the tile test of every slot first (the footprints' registers die here)
        unsigned long long m[kRoundSlots];
#pragma unroll
        for (uint32_t r = 0; r < kRoundSlots; ++r) {
            const bool pass = edges_pass_tile(f[r][0], f[r][1], f[r][2], xc, yc) &
                              box_overlaps(f[r][3], fx0, fx1, fy0, fy1);
            if (!whole) id[r] = __float_as_uint(f[r][0].w);
            m[r] = __ballot(pass);
        }
#pragma unroll
        for (uint32_t r = 0; r < kRoundSlots; ++r) {
            if (!m[r]) continue;
            // a split tile's half takes every other lane's survivor
            unsigned long long mm = split == kSplitNone ? m[r]
                                  : m[r] & (split == kSplitHalf0 ? 0x5555555555555555ull : 0xAAAAAAAAAAAAAAAAull);
            // the survivors' records into the wave's stage (DMA, no registers)
            if (mm) stage_survivor_records(st, recs, (mm >> lane) & 1ull, id[r]);
            if (!have_ray) {                       // under the records' DMA
                make_ray_from(*out.frame, pre_v, pre_u, dx, dy, dz, sx, sy, sz);
                have_ray = true;
            }
            if (!mm) continue;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's records have landed
            tests += (uint32_t)__popcll(mm);
            while (mm) {
                const uint32_t b = (uint32_t)__builtin_ctzll(mm);
                clear_lane_bit(mm, b);
                if constexpr (kSigned)
                    test_staged_one(st, b, (uint32_t)__builtin_amdgcn_readlane((int)id[r], (int)b), dx, dy, dz, sx,
                                    sy, sz, hl);
                else
                    test_staged_one(st, b, dx, dy, dz, hl);
            }
        }
    }
    if constexpr (!kSigned) {
        if (split != kSplitNone) {
            if (split == kSplitHalf1) publish_half(st, hl, tests);
            __syncthreads();                       // the pair's one barrier
            if (split == kSplitHalf1) return;      // half 0 finishes the tile
            if (have_ray) merge_half(*partner, hl, tests);
        }
    }
    ws.tile_tests += tests;
    if (have_ray) {
        const uint32_t nl = whole ? 0u : n_local;
        auto fetch = [=](uint32_t k) {
            return whole ? k : __float_as_uint((k < nl ? local[k] : glob[k - nl]).e0.w);
        };
        const EntryCull cull{local, glob, nl, tx0, ty0, !whole};
        if constexpr (kSigned)
            finish_ray_signed(p, out, active, row, col, hl, ws, recs, dx, dy, dz, sx, sy, sz, n_cand, fetch, cull);
        else
            finish_ray<kHits>(p, out, active, o, hl, ws, recs, dx, dy, dz, n_cand, fetch, cull);
    } else if (kSigned) {   // no survivor: L stays 80 (fork :314; :808 with distance 0)
        ws.rays += (uint32_t)__popcll(__ballot(active));
        if (active && out.lbuffer) out.lbuffer[(size_t)(row - p.row_begin) * p.width + col] = 80.0f;
    } else {   // no survivor: every ray of the tile misses (main.cxx:700-718 with no hit)
        ws.rays += (uint32_t)__popcll(__ballot(active));
        if (hits) store_hit_tile(out, o, false, 0.0f);
        else if (active) {
            if (out.image) out.image[o] = 80.0f;
            if (out.lbuffer) out.lbuffer[o] = out.miss_l;
            if (out.image_u8) out.image_u8[o] = 255u;
        }
    }
}

// The misses of a planned-empty region: wave w stores rows [w * kRows, ...)
// of it, 64 / kRegion rows per store (128-B row segments); ws.rays counts them.
__device__ __forceinline__ void fill_region_rows(const RenderParams& p, const Outputs& out,
                                                 const BinBuffers& bins, uint32_t slot, uint32_t wave,
                                                 WaveStats& ws)
{
    const uint32_t xy = as_const(bins.desc)[slot].xy;
    const uint32_t reg_x = xy & 0xFFFFu, reg_y = xy >> 16;
    constexpr uint32_t kRows = kRegion / kTileWaves;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t col = reg_x * kRegion + (lane % kRegion);
    const uint32_t r0 = p.row_begin + reg_y * kRegion + wave * kRows;
    uint32_t n = 0;
#pragma unroll
    for (uint32_t i = 0; i < kRows; i += 64u / kRegion) {
        const uint32_t row = r0 + i + lane / kRegion;
        if (col < p.width && row < p.row_end) {
            ++n;
            const size_t o = (size_t)(row - p.row_begin) * p.width + col;
            if (!out.packed) {
                if (out.image) out.image[o] = 80.0f;
                if (out.lbuffer) out.lbuffer[o] = out.miss_l;
                if (out.image_u8) out.image_u8[o] = 255u;
            }
        }
    }
    ws.rays = wave_reduce_u32<false>(n);
}

// Binned render: kTileWaves waves per workgroup (one 32x8 row of a region's
// tiles), regions in the launch order of bins.order; each wave stores its own
// statistics record.  8 waves per SIMD: the tile waves are latency-bound, and
// occupancy is what hides it.
//
// Fill plan (bins.tile_slots < regions): the slots past tile_slots hold the
// regions the geometry's sizing frame counted empty (no list entry, no global
// list); each gets ONE workgroup -- wave w stores the misses of the region's
// rows [w * 32 / kTileWaves, ...) -- instead of 16 / kTileWaves tile
// workgroups.  The counts are a function of the geometry, and the host only
// launches a plan that this frame's k_prep confirmed (no pair binned past
// tile_slots, an empty global list: BinBuffers::plan_miss); otherwise every
// region renders as tiles.  The signed model always renders tiles.
template <bool kSigned, bool kHits>
__device__ __forceinline__ void render_binned(RecStage* st, const TriRec* __restrict__ recs,
                                              const float4* __restrict__ culls, const RenderParams& p,
                                              const Outputs& out, const BinBuffers& bins,
                                              const BinState* __restrict__ bs)
{
    static_assert(kWavesPerRegion >= kTileWaves && kWavesPerRegion % kTileWaves == 0,
                  "a workgroup's waves render tiles of one region");
    constexpr uint32_t kBlocksPerRegion = kWavesPerRegion / kTileWaves;
    const uint64_t t_start = block_start_stamp();
    // a device-planned frame (BinBuffers::dev_plan, a moving camera): its tile
    // regions' number from k_size_lists
    const uint32_t tile_slots = !kSigned && !kHits && bins.dev_plan ? as_const(bs)->tile_slots : bins.tile_slots;
    const uint32_t tile_blocks = tile_slots * kBlocksPerRegion;
    const uint32_t split_slots = kSigned || !kCanSplit ? 0u : bins.split_slots;
    const uint32_t tile_end = tile_blocks + split_slots * kBlocksPerRegion;   // the tile regions' workgroups
    const uint32_t wave = wave_in_block();
    const uint32_t n_glob = as_const(bs)->global_count;
    WaveStats ws = {};
    uint32_t cand = 0;
    if (!kSigned && blockIdx.x >= tile_end) {      // a planned-empty region (workgroup-uniform)
        const uint32_t slot = tile_slots + (blockIdx.x - tile_end);
        if (!kHits && bins.dev_plan && slot >= bins.regions_x * bins.regions_y) return;   // past the device plan
        // statistics records: kBlocksPerRegion per wave, after the tile waves' (16 per region)
        const uint32_t rec0 =
            tile_blocks * kTileWaves + ((blockIdx.x - tile_end) * kTileWaves + wave) * kBlocksPerRegion;
        fill_region_rows(p, out, bins, slot, wave, ws);    // (packed layout: counts only)
        store_wave_stats(ws, 0u, out.block_stats, rec0, out.wave_times, t_start, kBlocksPerRegion);
        if ((threadIdx.x & 63u) == 0u) {
#pragma unroll
            for (uint32_t k = 1; k < kBlocksPerRegion; ++k) out.block_stats[rec0 + k] = BlockStats{};
        }
        return;
    }
    // Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8).  Within
    // each run of 8 regions, give XCD x all workgroups of region x, so a region's
    // candidate list and triangle records are cached by one L2 instead of four.
    // A bijection on full runs of a segment's workgroups (the split regions',
    // then the other tile regions'); a segment's tail keeps the identity.
    auto xcd_remap = [](uint32_t b, uint32_t n_blocks, uint32_t per_region) {
        const uint32_t run = 8u * per_region;                        // one region per XCD per run
        if (b < (n_blocks / run) * run) {
            const uint32_t within = b % run;
            b = (b - within) + (within & 7u) * per_region + (within >> 3);
        }
        return b;
    };
    // Split regions first (BinBuffers::split_slots, heaviest first): two waves
    // per tile, 2 * kBlocksPerRegion workgroups a region; then the other tile
    // regions, one wave per tile.  One render_tile call site for both: inlined
    // twice, the render's code outgrew the instruction cache.
    const uint32_t split_blocks = split_slots * 2u * kBlocksPerRegion;
    uint32_t slot, tile, split = kSplitNone;
    const RecStage* partner = nullptr;
    if (!kSigned && blockIdx.x < split_blocks) {                     // workgroup-uniform
        const uint32_t blk = xcd_remap(blockIdx.x, split_blocks, 2u * kBlocksPerRegion);
        const uint32_t g = blk * kTileWaves + wave;                  // wave of the split segment
        slot = g / (2u * kWavesPerRegion);
        tile = (g / 2u) % kWavesPerRegion;
        split = (g & 1u) ? kSplitHalf1 : kSplitHalf0;
        partner = &st[kCanSplit ? wave ^ 1u : wave];
    } else {
        const uint32_t blk = split_blocks + xcd_remap(blockIdx.x - split_blocks, tile_blocks - split_blocks / 2u,
                                                      kBlocksPerRegion);
        const uint32_t g = (blk - split_blocks / 2u) * kTileWaves + wave; // wave of the grid (16 per region)
        slot = g / kWavesPerRegion;                  // workgroup-uniform
        tile = g % kWavesPerRegion;
    }
    render_tile<kSigned, kHits>(st[wave], recs, culls, p, out, bins, n_glob, slot, tile, ws, cand, split, partner);
    // one record per tile (a split tile's by half 0); candidates are counted
    // once per region (by the wave holding tile 0)
    if (split != kSplitHalf1)
        store_wave_stats(ws, tile == 0u ? cand : 0u, out.block_stats, slot * kWavesPerRegion + tile,
                         out.wave_times, t_start);
}

template <bool kSigned>
__global__ __launch_bounds__(64 * kTileWaves) __attribute__((amdgpu_waves_per_eu(kSigned ? 5 : XRT_RENDER_WAVES, 8))) void k_render_binned(
    const TriRec* __restrict__ recs, const float4* __restrict__ culls, RenderParams p, Outputs out,
    BinBuffers bins, const BinState* __restrict__ bs)
{
    __shared__ RecStage st[kTileWaves];            // one private stage per wave
    render_binned<kSigned, false>(st, recs, culls, p, out, bins, bs);
}

// The same render writing the hit layout (Outputs::packed == kLayoutHits).
__global__ __launch_bounds__(64 * kTileWaves) __attribute__((amdgpu_waves_per_eu(XRT_RENDER_WAVES, 8))) void k_render_binned_hits(
    const TriRec* __restrict__ recs, const float4* __restrict__ culls, RenderParams p, Outputs out,
    BinBuffers bins, const BinState* __restrict__ bs)
{
    __shared__ RecStage st[kTileWaves];
    render_binned<false, true>(st, recs, culls, p, out, bins, bs);
}

// ---------------------------------------------------------------------------
// k_tile_plan: a geometry's tile plan (SlotDesc::live) from the statistics
// records of one of its binned renders -- bit t of slot s = tile t tested a
// survivor (record s * 16 + t).  Slots [first, end): the tile regions past the
// split ones (a split tile's two waves keep one record, every split tile
// stays live).  Renders in flight may read `live` while it is written: either
// value is exact for the geometry.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tile_plan(const BlockStats* __restrict__ recs, SlotDesc* __restrict__ desc,
                                                  uint32_t first, uint32_t end)
{
    const uint32_t s = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= end) return;
    uint32_t live = 0;
#pragma unroll
    for (uint32_t t = 0; t < kWavesPerRegion; ++t)
        live |= (recs[(size_t)s * kWavesPerRegion + t].tile_tests != 0u ? 1u : 0u) << t;
    desc[s].live = live;
}

// ---------------------------------------------------------------------------
// k_band_model: the balanced split's model from a binned strip render's own
// records (xrt_render_rows_multi, DESIGN.md "Multi-GPU") -- per 32-row band of
// the strip (its region row, SlotDesc::xy >> 16) the wave time of its regions'
// waves (timing records, 100 MHz ticks), the hit rays and the number of its
// tile regions (slots below tile_slots: the regions that travel); span[0] /
// span[1] = the first wave start / the last wave end.  One thread per slot (its
// 16 records); `bands` and `span` are cleared by the caller (span[0] to ~0).
// ---------------------------------------------------------------------------
struct BandModel {
    uint32_t ticks, hits, tiles, pad;
};
__global__ __launch_bounds__(256) void k_band_model(const BlockStats* __restrict__ recs,
                                                   const uint2* __restrict__ times,
                                                   const SlotDesc* __restrict__ desc, uint32_t n_slots,
                                                   uint32_t tile_slots, BandModel* __restrict__ bands,
                                                   uint32_t* __restrict__ span)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
    if (s < n_slots) {
        uint32_t ticks = 0, hits = 0;
        for (uint32_t t = 0; t < kWavesPerRegion; ++t) {
            const uint2 tt = times[(size_t)s * kWavesPerRegion + t];
            ticks += tt.y - tt.x;
            lo = min(lo, tt.x);
            hi = max(hi, tt.y);
            hits += recs[(size_t)s * kWavesPerRegion + t].hit_rays;
        }
        BandModel* b = bands + (desc[s].xy >> 16);
        atomicAdd(&b->ticks, ticks);
        if (s < tile_slots) {
            atomicAdd(&b->hits, hits);
            atomicAdd(&b->tiles, 1u);
        }
    }
    lo = ~wave_reduce_u32<true>(~lo);
    hi = wave_reduce_u32<true>(hi);
    if ((threadIdx.x & 63u) == 0u && hi != 0u) {
        atomicMin(&span[0], lo);
        atomicMax(&span[1], hi);
    }
}

// ---------------------------------------------------------------------------
// k_reduce_stats: a render's statistics records (one per tile wave / workgroup)
// and their timing records summed on the device for xrt_read_stats, so the
// host reads one 80-B record instead of copying every record back (1.2 MB at
// 2048^2, 32 MB at 8192^2).  Blocks stride over the records and leave their
// partial sums in `partial`; the last block to finish (a device-scope counter,
// reset by that block) adds them and the set's BinState into `out`.  The
// kernel span is the latest end minus the earliest start, as 32-bit tick
// differences from the first record's start (records_span_ms on the host).
// ---------------------------------------------------------------------------
struct StatsSum {
    unsigned long long rays, hit_rays, odd_rays, overflow_rays, hits, tile_tests, candidates;
    unsigned int max_hits;
    int span_lo, span_hi;          // ticks relative to the first record's start
    unsigned int global_count, overflow;
    unsigned int pad;
};
static_assert(sizeof(StatsSum) == 80, "StatsSum layout");
constexpr uint32_t kReduceThreads = 256;
constexpr uint32_t kReduceMaxBlocks = 256;

__global__ __launch_bounds__(kReduceThreads) void k_reduce_stats(const BlockStats* __restrict__ recs,
                                                               const uint2* __restrict__ times, uint32_t n,
                                                               const BinState* __restrict__ bs,
                                                               StatsSum* __restrict__ partial,
                                                               unsigned int* __restrict__ done, StatsSum* __restrict__ out)
{
    __shared__ StatsSum s_part[kReduceThreads / 64];
    __shared__ bool s_last;
    StatsSum a = {};
    a.span_lo = 0x7FFFFFFF;
    a.span_hi = -0x7FFFFFFF - 1;
    const uint32_t ref = times && n ? times[0].x : 0u;
    for (uint32_t i = blockIdx.x * kReduceThreads + threadIdx.x; i < n; i += gridDim.x * kReduceThreads) {
        const BlockStats b = recs[i];
        a.rays += b.rays;
        a.hit_rays += b.hit_rays;
        a.odd_rays += b.odd_rays;
        a.overflow_rays += b.overflow_rays;
        a.hits += b.hits;
        a.tile_tests += b.tile_tests;
        a.candidates += b.candidates;
        a.max_hits = max(a.max_hits, b.max_hits);
        if (times) {
            const uint2 t = times[i];
            a.span_lo = min(a.span_lo, (int)(t.x - ref));
            a.span_hi = max(a.span_hi, (int)(t.y - ref));
        }
    }
    auto combine = [](StatsSum& x, const StatsSum& y) {
        x.rays += y.rays;
        x.hit_rays += y.hit_rays;
        x.odd_rays += y.odd_rays;
        x.overflow_rays += y.overflow_rays;
        x.hits += y.hits;
        x.tile_tests += y.tile_tests;
        x.candidates += y.candidates;
        x.max_hits = max(x.max_hits, y.max_hits);
        x.span_lo = min(x.span_lo, y.span_lo);
        x.span_hi = max(x.span_hi, y.span_hi);
    };
    // wave, then block
    for (int off = 32; off > 0; off >>= 1) {
        StatsSum o;
        o.rays = __shfl_xor(a.rays, off);
        o.hit_rays = __shfl_xor(a.hit_rays, off);
        o.odd_rays = __shfl_xor(a.odd_rays, off);
        o.overflow_rays = __shfl_xor(a.overflow_rays, off);
        o.hits = __shfl_xor(a.hits, off);
        o.tile_tests = __shfl_xor(a.tile_tests, off);
        o.candidates = __shfl_xor(a.candidates, off);
        o.max_hits = __shfl_xor(a.max_hits, off);
        o.span_lo = __shfl_xor(a.span_lo, off);
        o.span_hi = __shfl_xor(a.span_hi, off);
        combine(a, o);
    }
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (lane == 0) s_part[wave] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < kReduceThreads / 64; ++w) combine(a, s_part[w]);
        partial[blockIdx.x] = a;
        __threadfence();
        s_last = atomicAdd(done, 1u) == gridDim.x - 1u;
    }
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    __threadfence();
    StatsSum t = partial[0];
    for (uint32_t b = 1; b < gridDim.x; ++b) combine(t, partial[b]);
    t.global_count = bs ? bs->global_count : 0u;
    t.overflow = bs ? bs->overflow : 0u;
    t.pad = 0u;
    *out = t;
    __threadfence();
    *done = 0u;                                    // for the next reduction
}

// ---------------------------------------------------------------------------
// k_hole_fill: the L-buffer fork's "error correction" pass
// (main-pthreads-lbuffer.cxx:327-404) over a whole frame's L-buffer: a pixel
// flagged -1 takes the mean of the first unflagged non-zero value within 4
// steps in each of four directions (+-1 along the row-major index, running on
// into the next / previous row, and +-1 row; unsigned 32-bit index arithmetic
// as written, a walk ends past the buffer -- the fork also reads one element
// past it, taken as the end); no value gives 0.0f / 0.  Others keep their
// value.  Reads lbuffer only, so the pass does not cascade.  NaN results
// carry x86's bits: the mean of values with a NaN (the render's 0x7FC00000)
// keeps that NaN; 0.0f / 0 is the default NaN 0xFFC00000.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hole_fill(const float* __restrict__ lbuffer, float* __restrict__ image,
                                                   uint8_t* __restrict__ image_u8, uint32_t width, uint32_t height)
{
    const uint64_t size = (uint64_t)width * height;
    const uint64_t pixel = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pixel >= size) return;
    const uint32_t row = (uint32_t)(pixel / width), col = (uint32_t)(pixel % width);
    float photon = lbuffer[pixel];
    if (photon == -1.0f) {
        float sum = 0.0f;
        uint32_t count = 0;
        for (int dir = 0; dir < 4; ++dir) {
            float value = 0.0f;
            for (uint32_t i = 1; i <= 4u; ++i) {
                const uint32_t idx = dir == 0 ? row * width + (col + i)
                                   : dir == 1 ? (row - i) * width + col
                                   : dir == 2 ? row * width + (col - i)
                                              : (row + i) * width + col;
                if ((uint64_t)idx >= size) break;
                const float l = lbuffer[idx];
                if (l != -1.0f) {
                    value = l;
                    break;
                }
            }
            if (value != 0.0f) {                   // :353 (NaN != 0 is kept)
                sum += value;
                ++count;
            }
        }
        photon = sum / (float)count;
        if (photon != photon) photon = xrt_f32_from_bits(count ? kX86SignedNaN : kX86DefaultNaN);
    }
    if (image) image[pixel] = photon;
    if (image_u8) image_u8[pixel] = lut_u8(photon);
}

// ---------------------------------------------------------------------------
// Region-packed strips in transit (multi-GPU gathers, DESIGN.md "Multi-GPU"):
// the regions a strip's fill plan filled hold nothing but misses, so only the
// others travel -- region r's 32x32 block of L values at packed[map[r] * 1024]
// (rows of the block row-major; past the strip or the image width the block
// holds kMissTransit).  map[r] = kEmpty for a filled region.  One workgroup of
// 256 threads per region, 4 pixels per thread.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack_regions(const float* __restrict__ lbuffer, float* __restrict__ packed,
                                                      const uint32_t* __restrict__ map, uint32_t width,
                                                      uint32_t rows, uint32_t regions_x)
{
    const uint32_t r = blockIdx.x;
    const uint32_t slot = map[r];
    if (slot == kEmpty) return;
    const uint32_t row = (r / regions_x) * kRegion + threadIdx.x / 8u;
    const uint32_t col = (r % regions_x) * kRegion + 4u * (threadIdx.x % 8u);
    float v[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        v[k] = row < rows && col + k < width ? lbuffer[(size_t)row * width + col + k] : __uint_as_float(kMissTransit);
    *reinterpret_cast<float4*>(packed + (size_t)slot * kPackBlock + 4u * threadIdx.x) = make_float4(v[0], v[1], v[2], v[3]);
}

// One block of the receiving side: 4 pixels of a 32x32 block (thread t: row
// t / 8, columns 4 (t % 8) ..) from `v` into the planes at frame row `row`.
__device__ __forceinline__ void unpack_pixels(float4 v, uint32_t row, uint32_t col, uint32_t width,
                                              float* __restrict__ lbuffer, float* __restrict__ image,
                                              uint8_t* __restrict__ image_u8)
{
    const float l[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        if (col + k >= width) break;
        const bool miss = __float_as_uint(l[k]) == kMissTransit;
        const float img = miss ? 80.0f : shade(l[k]);
        const size_t o = (size_t)row * width + col + k;
        if (image) image[o] = img;
        if (image_u8) image_u8[o] = miss ? (uint8_t)255u : lut_u8(img);
        if (lbuffer) lbuffer[o] = miss ? __builtin_inff() : l[k];
    }
}

// Many strips' packed regions in one launch (the gather's root): block b is
// described by desc[b] = (first frame row, rows of it in its strip, first
// column, packed block index or kEmpty for a filled region).
__global__ __launch_bounds__(256) void k_unpack_blocks(const float* __restrict__ packed,
                                                       const uint4* __restrict__ desc,
                                                       float* __restrict__ lbuffer, float* __restrict__ image,
                                                       uint8_t* __restrict__ image_u8, uint32_t width)
{
    const uint4 d = desc[blockIdx.x];
    const uint32_t r = threadIdx.x / 8u;
    if (r >= d.y) return;
    float4 v = make_float4(__uint_as_float(kMissTransit), __uint_as_float(kMissTransit),
                           __uint_as_float(kMissTransit), __uint_as_float(kMissTransit));
    if (d.w != kEmpty) v = *reinterpret_cast<const float4*>(packed + (size_t)d.w * kPackBlock + 4u * threadIdx.x);
    unpack_pixels(v, d.x + r, d.z + 4u * (threadIdx.x % 8u), width, lbuffer, image, image_u8);
}

// Many strips' hit-layout messages in one launch (Outputs::packed ==
// kLayoutHits): block b is a region described by desc[b] as k_unpack_blocks'
// (its last word: the index of the region's first tile descriptor, or kEmpty),
// tile t of it by tdesc[desc[b].w + t] = (word of its 64-bit hit mask in msg,
// word of its first hit value, the hit count its plan expects, 0).  A mask
// whose count differs from the plan's sets *bad (the message is not this
// geometry's), and hits past the plan's count read as misses: the reads stay
// inside the plan's words.
__global__ __launch_bounds__(256) void k_unpack_hits(const uint32_t* __restrict__ msg, const uint4* __restrict__ desc,
                                                     const uint4* __restrict__ tdesc, float* __restrict__ lbuffer,
                                                     float* __restrict__ image, uint8_t* __restrict__ image_u8,
                                                     uint32_t width, uint32_t* __restrict__ bad)
{
    const uint4 d = desc[blockIdx.x];
    const uint32_t r = threadIdx.x / 8u;
    if (r >= d.y) return;
    const uint32_t c4 = 4u * (threadIdx.x % 8u);
    float l[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) l[k] = __uint_as_float(kMissTransit);
    if (d.w != kEmpty) {
        const uint4 td = tdesc[(size_t)d.w + (r / 8u) * 4u + c4 / 8u];
        const uint2 mw = *reinterpret_cast<const uint2*>(msg + td.x);
        const unsigned long long m = (unsigned long long)mw.x | ((unsigned long long)mw.y << 32);
        if ((r & 7u) == 0u && (c4 & 7u) == 0u && (uint32_t)__popcll(m) != td.z && bad) atomicOr(bad, 1u);
        const uint32_t bit0 = (r & 7u) * 8u + (c4 & 7u);
        uint32_t rank = (uint32_t)__popcll(m & ((1ull << bit0) - 1ull));
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            if ((m >> (bit0 + k)) & 1ull) {
                if (rank < td.z) l[k] = __uint_as_float(msg[td.y + rank]);
                ++rank;
            }
        }
    }
    unpack_pixels(make_float4(l[0], l[1], l[2], l[3]), d.x + r, d.z + c4, width, lbuffer, image, image_u8);
}

// The receiving side: a packed strip into the frame's three planes (k_expand's
// values: misses -- kMissTransit, or a filled region -- give image 80, u8 255,
// L +inf; hits the shade of L and its LUT).
__global__ __launch_bounds__(256) void k_unpack_regions(const float* __restrict__ packed,
                                                        const uint32_t* __restrict__ map,
                                                        float* __restrict__ lbuffer, float* __restrict__ image,
                                                        uint8_t* __restrict__ image_u8, uint32_t width,
                                                        uint32_t rows, uint32_t regions_x)
{
    const uint32_t r = blockIdx.x;
    const uint32_t slot = map[r];
    const uint32_t row = (r / regions_x) * kRegion + threadIdx.x / 8u;
    const uint32_t col = (r % regions_x) * kRegion + 4u * (threadIdx.x % 8u);
    if (row >= rows) return;
    float4 v = make_float4(__uint_as_float(kMissTransit), __uint_as_float(kMissTransit),
                           __uint_as_float(kMissTransit), __uint_as_float(kMissTransit));
    if (slot != kEmpty) v = *reinterpret_cast<const float4*>(packed + (size_t)slot * kPackBlock + 4u * threadIdx.x);
    unpack_pixels(v, row, col, width, lbuffer, image, image_u8);
}

// ---------------------------------------------------------------------------
// k_expand: a gathered strip's L-buffer (misses as kMissTransit) into the
// frame's three planes -- image = 80 and u8 = 255 for misses, else the shade
// of the path length and its LUT, exactly as finish_ray computes them (for a
// hit the image is shade(L): L is the path length, 0 for an odd count) -- and
// the miss code back to +inf.  Four pixels per thread.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_expand(float* __restrict__ lbuffer, float* __restrict__ image,
                                                uint8_t* __restrict__ image_u8, uint64_t n)
{
    const uint64_t i0 = 4ull * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (i0 >= n) return;
    float l[4], img[4];
    uint8_t u8[4];
    bool miss[4];
    const bool full = i0 + 4u <= n && (reinterpret_cast<uintptr_t>(lbuffer + i0) & 15u) == 0u;
    if (full) {
        const float4 v = *reinterpret_cast<const float4*>(lbuffer + i0);
        l[0] = v.x; l[1] = v.y; l[2] = v.z; l[3] = v.w;
    } else {
        for (int k = 0; k < 4; ++k) l[k] = i0 + k < n ? lbuffer[i0 + k] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        miss[k] = __float_as_uint(l[k]) == kMissTransit;
        img[k] = miss[k] ? 80.0f : shade(l[k]);
        u8[k] = miss[k] ? (uint8_t)255u : lut_u8(img[k]);
    }
    if (full) {
        if (image) *reinterpret_cast<float4*>(image + i0) = make_float4(img[0], img[1], img[2], img[3]);
        if (image_u8 && (reinterpret_cast<uintptr_t>(image_u8 + i0) & 3u) == 0u)
            *reinterpret_cast<uint32_t*>(image_u8 + i0) =
                (uint32_t)u8[0] | ((uint32_t)u8[1] << 8) | ((uint32_t)u8[2] << 16) | ((uint32_t)u8[3] << 24);
        else if (image_u8)
            for (int k = 0; k < 4; ++k) image_u8[i0 + k] = u8[k];
        if (miss[0] | miss[1] | miss[2] | miss[3]) {
            const float inf = __builtin_inff();
            *reinterpret_cast<float4*>(lbuffer + i0) = make_float4(miss[0] ? inf : l[0], miss[1] ? inf : l[1],
                                                                   miss[2] ? inf : l[2], miss[3] ? inf : l[3]);
        }
    } else {
        for (int k = 0; k < 4; ++k) {
            if (i0 + k >= n) break;
            if (image) image[i0 + k] = img[k];
            if (image_u8) image_u8[i0 + k] = u8[k];
            if (miss[k]) lbuffer[i0 + k] = __builtin_inff();
        }
    }
}

// ---------------------------------------------------------------------------
// Probes
// ---------------------------------------------------------------------------
__global__ void k_probe_intersect(const float* __restrict__ rays, const float* __restrict__ tris,
                                  uint64_t n, uint8_t* __restrict__ hit, float* __restrict__ tout)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* R = rays + 6 * i;
    const float* P = tris + 9 * i;
    // The ray origin and the Ray ctor's re-normalisation (Ray.inl:80-84).
    float ox = R[0], oy = R[1], oz = R[2];
    float X = R[3], Y = R[4], Z = R[5];
    float len = sqrtf((X * X + Y * Y) + Z * Z);
    float dx = 0.0f, dy = 0.0f, dz = 0.0f;
    if (len != 0.0f) {
        dx = X / len;
        dy = Y / len;
        dz = Z / len;
    }
    float e1x = P[3] - P[0], e1y = P[4] - P[1], e1z = P[5] - P[2];
    float e2x = P[6] - P[0], e2y = P[7] - P[1], e2z = P[8] - P[2];
    float tvx = ox - P[0], tvy = oy - P[1], tvz = oz - P[2];
    float qvx = tvy * e1z - tvz * e1y;
    float qvy = tvz * e1x - tvx * e1z;
    float qvz = tvx * e1y - tvy * e1x;
    float tnum = (e2x * qvx + e2y * qvy) + e2z * qvz;
    float t = 0.0f;
    bool h = mt_intersect(dx, dy, dz, e1x, e1y, e1z, e2x, e2y, e2z, tvx, tvy, tvz, qvx, qvy, qvz,
                          tnum, t);
    hit[i] = h ? 1 : 0;
    tout[i] = h ? t : 0.0f;
}

__global__ void k_probe_math(int op, const float* __restrict__ in, float* __restrict__ outp,
                             uint64_t n)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[i];
    float y;
    switch (op) {
    case 0: y = xrt_expf(x); break;
    case 1: y = sqrtf(x); break;
    case 2: y = inv_det_of(x); break;
    case 4: y = rcp_newton_exact_for(x) ? rcp_newton(x) : inv_det_of(x); break;   // inv_det_fast per lane
    case 5: y = signed_lbuffer(x, 0, 0.1037f); break;   // the fork's 80 * exp(-(mu * (d * 0.1)))
    default: y = (float)lut_u8(x); break;
    }
    outp[i] = y;
}

}  // namespace XRT_KERNEL_NS
