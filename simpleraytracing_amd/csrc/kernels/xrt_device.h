// xrt_device.h -- device-side arithmetic of the X-ray render path (gfx950).
//
// Every function here reproduces the reference's f32/f64 rounding sequence
// exactly, so the GPU image is bit-identical to src/main.cxx's.  The numerical
// contract (DESIGN.md "Numerical contract"):
//   * no FMA contraction on the f32 path (built with -ffp-contract=off, and the
//     pragma below); the only fused ops are the explicit fma() calls of
//     glibc's expf, which are part of that function's definition;
//   * f32 sqrt is correctly rounded (HIP's default
//     -fhip-fp32-correctly-rounded-divide-sqrt); src/Ray.cxx:99's
//     (float)(1.0/(double)det) is the correctly rounded f32 1.0f/det for
//     every det (inv_det_of);
//   * f32 denormals are preserved (no -fgpu-flush-denormals-to-zero).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

// Variant builds (tools/build_variants.sh) get their own kernel namespace so
// several can be loaded side by side without kernel-name collisions.
#ifndef XRT_KERNEL_NS
#define XRT_KERNEL_NS xrt
#endif

// Compile-time variants for A/B timing (tools/build_variants.sh, tools/ab.py);
// the defaults are the measured-faster choices.
#ifndef XRT_MED3
#define XRT_MED3 1        // med3 insertion (else the compare-exchange chain)
#endif
#ifndef XRT_PAIR
#define XRT_PAIR 1        // culled kernels test survivors two at a time
#endif
#ifndef XRT_WAVES_PER_EU
#define XRT_WAVES_PER_EU 0   // >0: occupancy hint for the culled render kernels
#endif
#ifndef XRT_XCD_REMAP
#define XRT_XCD_REMAP 1  // binned render: >0 = regions per XCD per run of 8 XCDs, all of a region on one XCD (A/B: render 55.1 -> 53.8 us); 0 off
#endif
#ifndef XRT_TILE_WAVES
#define XRT_TILE_WAVES 4  // binned render: tile waves per workgroup
#endif
#ifndef XRT_PREP_SETPRIO
#define XRT_PREP_SETPRIO 1   // preparation kernels raise their wave priority (s_setprio 3)
#endif
#ifndef XRT_DEFAULT_ORDER
#define XRT_DEFAULT_ORDER 1    // binned render launch order: 0 raster, 1 centre first
#endif
#ifndef XRT_PRE_REJECT
#define XRT_PRE_REJECT 0     // culled tests: wave-wide division-free reject before the exact test (A/B: slower, off)
#endif
#ifndef XRT_FAST_RCP
#define XRT_FAST_RCP 2    // culled tests' 1/det: 0 IEEE division; 1 rcp + Newton per test (slower);
                          // 2 rcp + Newton with one range check per survivor pair (fastest)
#endif
#ifndef XRT_STAGED_PAIRS
#define XRT_STAGED_PAIRS 0   // binned render: survivors tested two at a time (A/B: spills at 8 waves/SIMD, slower)
#endif
#ifndef XRT_RENDER_WAVES
#define XRT_RENDER_WAVES 8   // binned render: minimum waves per SIMD (8 = 64 VGPRs)
#endif
#ifndef XRT_STAGE
#define XRT_STAGE 128     // binned render: candidates staged in LDS per round (16 KB)
#endif
#ifndef XRT_PREP_THREADS
#define XRT_PREP_THREADS 64  // k_prep workgroup size (64: single-wave groups fill the render's holes)
#endif
#ifndef XRT_ABLATION
#define XRT_ABLATION 0    // diagnostics: honour RenderParams::ablate ($XRT_ABLATE)
#endif
#ifndef XRT_STAMPS
#define XRT_STAMPS 0      // diagnostics: per-workgroup start/end/hw-id in BlockStats
#endif
#if XRT_WAVES_PER_EU > 0
#define XRT_CULLED_ATTR __attribute__((amdgpu_waves_per_eu(XRT_WAVES_PER_EU, 8)))
#else
#define XRT_CULLED_ATTR
#endif

namespace XRT_KERNEL_NS {

// Per-render triangle record: the ray-independent part of Ray::intersect
// (src/Ray.cxx:86-122) for the shared ray origin.  64 bytes, read
// wave-uniformly (one s_load_dwordx16 per triangle).
struct alignas(16) TriRec {
    float e1x, e1y, e1z;    // edge1 = P2 - P1                 Ray.cxx:86
    float e2x, e2y, e2z;    // edge2 = P3 - P1                 Ray.cxx:87
    float tvx, tvy, tvz;    // tvec  = origin - P1             Ray.cxx:102
    float qvx, qvy, qvz;    // qvec  = tvec x edge1            Ray.cxx:112
    float tnum;             // edge2 . qvec  (t * det)          Ray.cxx:122
    float pad0, pad1, pad2;
};
static_assert(sizeof(TriRec) == 64, "TriRec must be 64 bytes");

// Conservative screen-space footprint of a triangle (DESIGN.md "Tile cull"),
// stored structure-of-arrays as four float4 planes of length T:
//   plane 0  bbox  = (xmin, xmax, ymin, ymax) in pixel-centre coordinates
//   plane 1..3 edge k = (a, b, c, 0):  a*col + b*row + c >= 0 holds at every
//   pixel whose ray the reference's Ray::intersect can report as a hit with
//   t > 1e-7.
constexpr int kCullPlanes = 4;

// Camera + strip parameters, passed by value.
struct RenderParams {
    float ox, oy, oz;       // RayTracerInfo::origin
    float cx, cy, cz;       // RayTracerInfo::detector_position
    float ux, uy, uz;       // RayTracerInfo::up
    float rx, ry, rz;       // RayTracerInfo::right
    float spacing;          // pixel_spacing, main.cxx:639-641
    uint32_t width, height; // full image
    uint32_t row_begin, row_end;
    uint32_t num_triangles;
    uint32_t hit_capacity;  // <= XRT_MAX_HITS
    uint32_t ablate;        // diagnostics only ($XRT_ABLATE bits, kAblate*); 0 in production
};

// Ablation bits (timing studies; outputs are wrong when any is set).  Only
// XRT_ABLATION builds (tools/gpu_ablate.sh) read them: the production kernels
// carry neither the field nor its branches.
constexpr uint32_t kAblateCandidates = 1;   // phase 2 sees no candidates
constexpr uint32_t kAblateSweep = 2;        // tiled: no phase-1 footprint sweep
constexpr uint32_t kAblateRayGen = 4;       // constant ray direction
constexpr uint32_t kAblateStores = 8;       // no output stores
constexpr uint32_t kAblateShade = 16;       // no expf / LUT
constexpr uint32_t kAblateExact = 32;       // culled kernels: no Moller-Trumbore for survivors
constexpr uint32_t kAblatePush = 64;        // culled kernels: exact test but no hit-list insert

__device__ __forceinline__ uint32_t ablation(const RenderParams& p)
{
#if XRT_ABLATION
    return p.ablate;
#else
    (void)p;
    return 0u;
#endif
}

// Register hit list per ray.  Each slot costs every exact test one
// v_med3_f32; a ray with more hits is recomputed exactly by its wave
// (finish_ray's fix-up, tens of microseconds for that wave).  dragon.ply rays
// have at most 12 hits (2048^2: 102 rays above 8): 12 slots render it 3 %
// faster than 16 with no fix-up; 8 slots would send those 102 rays through
// it and run 5x slower (DESIGN.md "Hit list").
#ifndef XRT_MAX_HITS
#define XRT_MAX_HITS 12
#endif
constexpr int kMaxHits = XRT_MAX_HITS;

// ---------------------------------------------------------------------------
// Ray generation: src/main.cxx:652-661 and the Ray ctor, include/Ray.inl:74-85.
// ---------------------------------------------------------------------------
// :655-656  float * (0.5 + unsigned - unsigned / 2.0) in double, narrowed once.
// A function of one pixel index: k_prep tabulates it per frame (pixel_offsets)
// for the render kernels.
__host__ __device__ __forceinline__ float pixel_offset(float spacing, uint32_t i, uint32_t n)
{
    return (float)((double)spacing * ((0.5 + (double)i) - (double)n / 2.0));
}

// The frame's pixel offsets: v_off of every image row, then u_off of every
// column (H + W floats, written by k_prep next to the frame's RenderParams).
struct PixelOffsets {
    const float* __restrict__ v;   // [height]
    const float* __restrict__ u;   // [width]
};

// P: RenderParams in any address space (kernel argument or constant memory).
template <typename P>
__device__ __forceinline__ void make_ray(const P& p, uint32_t row, uint32_t col,
                                         float& dx, float& dy, float& dz);

template <typename P>
__device__ __forceinline__ void make_ray_from(const P& p, float v_off, float u_off, float& dx,
                                              float& dy, float& dz);

template <typename P>
__device__ __forceinline__ void make_ray(const P& p, uint32_t row, uint32_t col,
                                         float& dx, float& dy, float& dz)
{
    make_ray_from(p, pixel_offset(p.spacing, row, p.height), pixel_offset(p.spacing, col, p.width), dx,
                  dy, dz);
}

// The same ray with the offsets read from the frame's tables.
template <typename P>
__device__ __forceinline__ void make_ray(const P& p, const PixelOffsets& off, uint32_t row,
                                         uint32_t col, float& dx, float& dy, float& dz)
{
    make_ray_from(p, off.v[row], off.u[col], dx, dy, dz);
}

template <typename P>
__device__ __forceinline__ void make_ray_from(const P& p, float v_off, float u_off, float& dx,
                                              float& dy, float& dz)
{
    // :659  detector + up*v + right*u - origin  (Vec3 ops left to right, f32)
    float X = ((p.cx + p.ux * v_off) + p.rx * u_off) - p.ox;
    float Y = ((p.cy + p.uy * v_off) + p.ry * u_off) - p.oy;
    float Z = ((p.cz + p.uz * v_off) + p.rz * u_off) - p.oz;
    // :660  Vec3::normalise (Vec3.inl:469-476)
    float len = sqrtf((X * X + Y * Y) + Z * Z);
    X = X / len;
    Y = Y / len;
    Z = Z / len;
    // Ray ctor normalises again; a zero length keeps the default (0,0,0).
    float len2 = sqrtf((X * X + Y * Y) + Z * Z);
    if (len2 != 0.0f) {
        dx = X / len2;
        dy = Y / len2;
        dz = Z / len2;
    } else {
        dx = 0.0f;
        dy = 0.0f;
        dz = 0.0f;
    }
}

// ---------------------------------------------------------------------------
// Ray::intersect, src/Ray.cxx:72-124, with the ray-independent terms taken
// from the TriRec.  A conservative pre-test rejects only when the reference's
// `u < 0 || u > 1` test (Ray.cxx:106) provably rejects, so the f64 division
// runs only for candidates (DESIGN.md "Early reject").
// ---------------------------------------------------------------------------
// Ray.cxx:99 computes (float)(1.0 / (double)det).  For every f32 det that is
// the correctly rounded f32 quotient 1.0f / det: 1/det is never within 2^-49
// (relative) of an f32 rounding midpoint, so the f64 rounding cannot move it
// across one.  Checked on all 2^32 inputs (tools/check_fp_identities.c,
// tests/test_abi.py); the f32 division sequence is about half the f64 one.
__host__ __device__ __forceinline__ float inv_det_of(float det) { return 1.0f / det; }

// v_rcp_f32 (within 1 ulp) and one FMA Newton step give the correctly rounded
// 1.0f / d for every d with biased exponent in [1, 252], i.e. 2^-126 <= |d| <
// 2^126: checked on all 2^32 inputs on the GPU (tools/probes/rcp_probe.hip,
// profiles/r01_rcp_exhaustive.txt; the XRT_PROBE_RCP_FAST sweep of
// tests/test_gpu_parity.py).  Three VALU ops instead of the ten of the IEEE
// division sequence (div_scale / rcp / 4 fma / div_fmas / div_fixup).
__device__ __forceinline__ float rcp_newton(float d)
{
    const float r = __builtin_amdgcn_rcpf(d);
    return __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
}
__device__ __forceinline__ bool rcp_newton_exact_for(float d)
{
    const float a = fabsf(d);
    return a >= 0x1p-126f && a < 0x1p126f;       // false for NaN
}
// The culled tests' 1/det: the short sequence, unless some lane of the wave
// has a det outside its range (zero, denormal, |det| >= 2^126, inf, NaN) --
// that wave takes the IEEE division on every lane.  Equal to inv_det_of(det)
// on every lane either way.
__device__ __forceinline__ float inv_det_fast(float det)
{
    if (__builtin_expect(__ballot(!rcp_newton_exact_for(det)) != 0ull, 0)) return inv_det_of(det);
    return rcp_newton(det);
}

// Branch-free Ray::intersect for the culled kernels, whose survivors almost
// always have a hitting lane (so the early reject would not skip the wave's
// division): the same comparisons as mt_intersect, combined with no control
// flow so two tests can be interleaved.  `hit` includes accept_t.
__device__ __forceinline__ float mt_exact(float dx, float dy, float dz, float e1x, float e1y,
                                         float e1z, float e2x, float e2y, float e2z, float tvx,
                                         float tvy, float tvz, float qvx, float qvy, float qvz,
                                         float tnum, bool& hit);

__device__ __forceinline__ bool mt_intersect(float dx, float dy, float dz,
                                             float e1x, float e1y, float e1z,
                                             float e2x, float e2y, float e2z,
                                             float tvx, float tvy, float tvz,
                                             float qvx, float qvy, float qvz,
                                             float tnum, float& t)
{
    // pvec = direction x edge2               Ray.cxx:90 (Vec3.inl:321-329)
    float px = dy * e2z - dz * e2y;
    float py = dz * e2x - dx * e2z;
    float pz = dx * e2y - dy * e2x;
    // det = edge1 . pvec                     Ray.cxx:93
    float det = (e1x * px + e1y * py) + e1z * pz;
    // tvec . pvec (u * det)                  Ray.cxx:105
    float a = (tvx * px + tvy * py) + tvz * pz;

    // Early reject.  With D = |det|, A = a*sign(det): u = RN(A * RN(1/D)).
    //   A < -2^-20 D       =>  u <= -2^-20 (1 - 2^-21) < 0        (reference rejects)
    //   A > RN(D (1+2^-20)) =>  u >= RN(1 + 2^-22 - tiny) > 1      (reference rejects)
    // NaNs fail both compares and fall through to the exact test; det == +-0
    // with a != 0 rejects here, as the reference does at Ray.cxx:94.
    float D = fabsf(det);
    float A = __int_as_float(__float_as_int(a) ^ (__float_as_int(det) & 0x80000000));
    if (A < D * -0x1p-20f || A > D * 0x1.00001p0f) return false;

    if (det == 0.0f) return false;                        // Ray.cxx:94 (fpclassify FP_ZERO)
    float inv_det = inv_det_of(det);                      // Ray.cxx:99
    float u = a * inv_det;                                // Ray.cxx:105
    if (u < 0.0f || u > 1.0f) return false;               // Ray.cxx:106
    float v = ((dx * qvx + dy * qvy) + dz * qvz) * inv_det;   // Ray.cxx:115
    if (v < 0.0f || u + v > 1.0f) return false;           // Ray.cxx:116
    t = tnum * inv_det;                                   // Ray.cxx:122
    return true;
}

// main.cxx:687: (double)t > 0.0000001.  For f32 t that is t > 0x1.ad7f28p-24f,
// the largest float not above 1e-7 (all 2^32 inputs: tools/check_fp_identities.c).
__host__ __device__ __forceinline__ bool accept_t(float t) { return t > 0x1.ad7f28p-24f; }

// The division-free part of Ray::intersect: det (Ray.cxx:93) and the
// numerators of u (:105, tvec . pvec) and v (:115, dir . qvec), with the
// reference's operation order.
__device__ __forceinline__ void mt_numerators(float dx, float dy, float dz, float e1x, float e1y,
                                              float e1z, float e2x, float e2y, float e2z,
                                              float tvx, float tvy, float tvz, float qvx,
                                              float qvy, float qvz, float& det, float& a, float& b)
{
    const float px = dy * e2z - dz * e2y;                 // Ray.cxx:90
    const float py = dz * e2x - dx * e2z;
    const float pz = dx * e2y - dy * e2x;
    det = (e1x * px + e1y * py) + e1z * pz;               // Ray.cxx:93
    a = (tvx * px + tvy * py) + tvz * pz;                 // Ray.cxx:105 (u * det)
    b = (dx * qvx + dy * qvy) + dz * qvz;                 // Ray.cxx:115 (v * det)
}

// False only when the reference provably rejects (no division needed): with
// D = |det| and A, B, T the numerators of u, v, t carrying det's sign,
//   det == +-0                        Ray.cxx:94
//   A < -2^-20 D or A > (1+2^-20) D   u < 0 or u > 1   (mt_intersect's bounds)
//   B < -2^-20 D                      v < 0            (same argument as for u)
//   A + B > (1+2^-18) D, D normal     u + v > 1: u and v each lose at most 2 ulps
//                                     to their two roundings, the f32 sum one (for
//                                     denormal det, 1/det may overflow and u = 0 * inf
//                                     is NaN, which the reference lets through)
//   T <= 0                            t <= 0 (t = tnum * RN(1/det), same sign)
// NaNs fail every compare and are kept.  Used wave-wide: a triangle that
// every lane rejects skips the division and the hit-list insertion.
__host__ __device__ __forceinline__ float xrt_flip_sign(float x, uint32_t sgn)
{
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    u ^= sgn;
    __builtin_memcpy(&x, &u, 4);
    return x;
}

__host__ __device__ __forceinline__ bool mt_may_hit(float det, float a, float b, float tnum)
{
    uint32_t bits;
    __builtin_memcpy(&bits, &det, 4);
    const uint32_t sgn = bits & 0x80000000u;
    const float D = fabsf(det);
    const float A = xrt_flip_sign(a, sgn);
    const float B = xrt_flip_sign(b, sgn);
    const float T = xrt_flip_sign(tnum, sgn);
    const float lo = D * -0x1p-20f;
    return !(det == 0.0f || A < lo || A > D * 0x1.00001p0f || B < lo ||
             (D >= 0x1p-126f && A + B > D * 0x1.00004p0f) || T <= 0.0f);
}

// The rest of Ray::intersect from mt_numerators' values; `hit` includes accept_t.
__host__ __device__ __forceinline__ float mt_finish_inv(float det, float inv_det, float a, float b,
                                                       float tnum, bool& hit)
{
    const float u = a * inv_det;                          // Ray.cxx:105
    const float v = b * inv_det;                          // Ray.cxx:115
    const float t = tnum * inv_det;                       // Ray.cxx:122
    hit = det != 0.0f && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) && accept_t(t);
    return t;
}

__host__ __device__ __forceinline__ float mt_finish(float det, float a, float b, float tnum, bool& hit)
{
    return mt_finish_inv(det, inv_det_of(det), a, b, tnum, hit);   // Ray.cxx:99
}

__device__ __forceinline__ float mt_exact(float dx, float dy, float dz, float e1x, float e1y,
                                         float e1z, float e2x, float e2y, float e2z, float tvx,
                                         float tvy, float tvz, float qvx, float qvy, float qvz,
                                         float tnum, bool& hit)
{
    float det, a, b;
    mt_numerators(dx, dy, dz, e1x, e1y, e1z, e2x, e2y, e2z, tvx, tvy, tvz, qvx, qvy, qvz, det, a, b);
    return mt_finish_inv(det, XRT_FAST_RCP == 1 ? inv_det_fast(det) : inv_det_of(det), a, b, tnum, hit);   // Ray.cxx:99
}

// ---------------------------------------------------------------------------
// Per-ray sorted hit list in registers (static indices only).  Replaces the
// per-pixel std::vector + std::sort of main.cxx:666-704.
// ---------------------------------------------------------------------------
struct HitList {
    float h[kMaxHits];
    uint32_t n;

    __device__ __forceinline__ void init()
    {
#pragma unroll
        for (int k = 0; k < kMaxHits; ++k) h[k] = __builtin_inff();
        n = 0;
    }

    // Keeps h ascending with +inf sentinels.  With h sorted, inserting x gives
    // h'[k] = max(h[k-1], min(h[k], x)) = med3(h[k-1], h[k], x) (old values):
    // one independent v_med3_f32 per slot instead of a compare-exchange chain.
    // A miss inserts +inf, which leaves h unchanged.  hit == false or x > 0.
    __device__ __forceinline__ void push_if(bool hit, float t)
    {
#if !XRT_MED3
        if (hit) {
#pragma unroll
            for (int k = 0; k < kMaxHits; ++k) {
                const float cur = h[k];
                const bool lt = t < cur;
                h[k] = lt ? t : cur;
                t = lt ? cur : t;
            }
            ++n;
        }
        return;
#endif
        const float x = hit ? t : __builtin_inff();
        float prev = h[0];
        h[0] = fminf(prev, x);
#pragma unroll
        for (int k = 1; k < kMaxHits; ++k) {
            const float cur = h[k];
            h[k] = __builtin_amdgcn_fmed3f(prev, cur, x);
            prev = cur;
        }
        n += hit ? 1u : 0u;
    }

    __device__ __forceinline__ void push(float t) { push_if(true, t); }

    // main.cxx:703-708: pairwise sum of the sorted list, sequential f32.
    __device__ __forceinline__ float path_length() const
    {
        float distance = 0.0f;
#pragma unroll
        for (int k = 0; k < kMaxHits / 2; ++k)
            if (2u * k + 1u < n) distance += h[2 * k + 1] - h[2 * k];
        return distance;
    }
};

// ---------------------------------------------------------------------------
// glibc 2.35 expf (sysdeps/ieee754/flt-32/e_expf.c with e_exp2f_data.c,
// EXP2F_TABLE_BITS = 5), as x86-64 glibc dispatches it on FMA hardware
// (e_expf-fma.c: the compiler fuses InvLn2N*x into both uses and the
// polynomial).  This is the function std::exp(float) binds to in
// src/main.cxx:739.  Bit-identical to the system libm on all 2^32 inputs
// (tools/gen_expf_table.py; tests/test_abi.py::test_host_expf_restatement_matches_libm on
// the host build, tests/test_gpu_parity.py::test_probe_expf_matches_libm on the device).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ double xrt_u64_as_double(uint64_t u)
{
    double d;
    __builtin_memcpy(&d, &u, 8);
    return d;
}

__host__ __device__ __forceinline__ uint64_t xrt_double_as_u64(double d)
{
    uint64_t u;
    __builtin_memcpy(&u, &d, 8);
    return u;
}

__host__ __device__ __forceinline__ uint64_t xrt_exp2f_tab(uint32_t i)
{
    // tab[i] = asuint64(RN(2^(i/32))) - (i << 47)
    constexpr uint64_t tab[32] = {
        0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL,
        0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL,
        0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL,
        0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL,
        0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL,
        0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL,
        0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL,
        0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL,
    };
    return tab[i & 31];
}

__host__ __device__ __forceinline__ float xrt_expf(float x)
{
    constexpr double kInvLn2N = 0x1.71547652b82fep+0 * 32;
    constexpr double kShift = 0x1.8p+52;
    constexpr double kC0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32;
    constexpr double kC1 = 0x1.ebfce50fac4f3p-3 / 32 / 32;
    constexpr double kC2 = 0x1.62e42ff0c52d6p-1 / 32;

    uint32_t ix;
    __builtin_memcpy(&ix, &x, 4);
    uint32_t abstop = (ix >> 20) & 0x7ff;
    if (abstop >= 0x42b) {                  // |x| >= 88 or NaN
        if (ix == 0xff800000u) return 0.0f; // -inf
        if (abstop >= 0x7f8) return x + x;  // +inf or NaN
        if (x > 0x1.62e42ep6f) return __builtin_inff();   // overflow
        if (x < -0x1.9fe368p6f) return 0.0f;              // underflow
    }
    double xd = (double)x;
    double kd = __builtin_fma(kInvLn2N, xd, kShift);
    uint64_t ki = xrt_double_as_u64(kd);
    kd -= kShift;
    double r = __builtin_fma(kInvLn2N, xd, -kd);
    uint64_t t = xrt_exp2f_tab((uint32_t)(ki % 32)) + (ki << 47);
    double s = xrt_u64_as_double(t);
    double z = __builtin_fma(kC0, r, kC1);
    double r2 = r * r;
    double y = __builtin_fma(kC2, r, 1.0);
    y = __builtin_fma(z, r2, y);
    y = y * s;
    return (float)y;
}

__host__ __device__ __forceinline__ float xrt_f32_from_bits(uint32_t u)
{
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// NaN path lengths.  The only NaN the reference's pair sum can produce is
// inf - inf (two t = +inf "hits", which Ray.cxx records when 1/det overflows,
// DESIGN.md "Tile cull" step 0); x86 SSE returns its default NaN for it
// (0xFFC00000) and every later add propagates that operand.  The device's NaN
// encodings differ, so the kernels store the x86 bits explicitly.
constexpr uint32_t kX86DefaultNaN = 0xFFC00000u;
// shade() of that NaN on x86: (double) and * 0.1 keep it, the negation in
// -(0.3971f * cm) flips its sign, expf(x) returns x + x and 80 * x keeps it.
constexpr uint32_t kX86ShadeNaN = 0x7FC00000u;

// Beer-Lambert shade, main.cxx:725 and :739.
__host__ __device__ __forceinline__ float shade(float distance)
{
    if (distance != distance) return xrt_f32_from_bits(kX86ShadeNaN);
    float cm = (float)((double)distance * 0.1);
    return 80.000f * xrt_expf(-(0.3971f * cm));
}

// 8-bit image: Image::applyLUT's per-pixel formula (include/Image.inl:195-211)
// with vmin = 0, vmax = 80; NaN (undefined in the reference) maps to 0.
__host__ __device__ __forceinline__ uint8_t lut_u8(float v)
{
    const float vmin = 0.0f, vmax = 80.0f;
    if (v < vmin) return 0;
    if (v > vmax) return 255;
    if (v != v) return 0;
    // 255.0 * v / 80.0 == v * 3.1875 exactly: 255*v is exact in f64 and the
    // quotient 51*v/16 has at most 30 significant bits, so the correctly
    // rounded division returns it unchanged (checked for every f32 in
    // [0, 80]: tools/check_fp_identities.c).
    return (uint8_t)__builtin_round((double)(v - vmin) * 3.1875);
}

}  // namespace XRT_KERNEL_NS
