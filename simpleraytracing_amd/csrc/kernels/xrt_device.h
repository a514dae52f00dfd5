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

// Tuning constants (overridable with -D for A/B builds, tools/build_variants.sh);
// the defaults are the measured-faster choices.
#ifndef XRT_TILE_WAVES
#define XRT_TILE_WAVES 2  // binned render: tile waves per workgroup (2: 2048^2 step -4 %, 1.12M-tri -5 % vs 4)
#endif
#ifndef XRT_RENDER_WAVES
#define XRT_RENDER_WAVES 8   // binned render: minimum waves per SIMD (8 = 64 VGPRs)
#endif
#ifndef XRT_STAGE
#define XRT_STAGE 64      // binned render: candidates a tile wave culls per round -- one footprint per lane, read into registers (64..256); only survivors' records go to the wave's 4-KB LDS stage
#endif
#ifndef XRT_PREP_THREADS
#define XRT_PREP_THREADS 64  // k_prep workgroup size (64: single-wave groups fill the render's holes)
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
    uint32_t prep_tris;     // triangles per k_prep wave (prep_tris_for)
    uint32_t model;         // kModelAttenuation (main.cxx) or kModelSigned (the L-buffer fork)
};

// What a render computes per ray.
constexpr uint32_t kModelAttenuation = 0;   // renderLoop, src/main.cxx:626-743
constexpr uint32_t kModelSigned = 1;        // renderLoopCallBack, src/main-pthreads-lbuffer.cxx:733-813

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
                                              float& dy, float& dz, float& sx, float& sy, float& sz);

template <typename P>
__device__ __forceinline__ void make_ray_from(const P& p, float v_off, float u_off, float& dx,
                                              float& dy, float& dz)
{
    float sx, sy, sz;
    make_ray_from(p, v_off, u_off, dx, dy, dz, sx, sy, sz);
}

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

// Also returns the direction after the first normalisation (sx, sy, sz): the
// L-buffer fork takes sign(direction . normal) with it, not with the Ray's
// twice-normalised copy (main-pthreads-lbuffer.cxx:761-762, :791).
template <typename P>
__device__ __forceinline__ void make_ray_from(const P& p, float v_off, float u_off, float& dx,
                                              float& dy, float& dz, float& sx, float& sy, float& sz)
{
    // :659  detector + up*v + right*u - origin  (Vec3 ops left to right, f32)
    float X = ((p.cx + p.ux * v_off) + p.rx * u_off) - p.ox;
    float Y = ((p.cy + p.uy * v_off) + p.ry * u_off) - p.oy;
    float Z = ((p.cz + p.uz * v_off) + p.rz * u_off) - p.oz;
    // :660  Vec3::normalise (Vec3.inl:469-476)
    const float len = sqrtf((X * X + Y * Y) + Z * Z);
    X = X / len;
    Y = Y / len;
    Z = Z / len;
    sx = X;
    sy = Y;
    sz = Z;
    // Ray ctor normalises again; a zero length keeps the default (0,0,0).
    const float len2 = sqrtf((X * X + Y * Y) + Z * Z);
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
    // Ray.cxx:106 and :116 with two compares: !(u < 0) && !(v < 0) is
    // !(min(u, v) < 0), and !(u > 1) && !(u + v > 1) is !(max(u, u + v) > 1),
    // because IEEE minNum / maxNum return the other operand when one is a
    // (quiet) NaN -- and a NaN passes the reference's tests -- and a NaN only
    // when both are.
    // (bitwise &: evaluated without branches)
    hit = (det != 0.0f) & !(fminf(u, v) < 0.0f) & !(fmaxf(u, u + v) > 1.0f) & accept_t(t);
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
    return mt_finish_inv(det, inv_det_of(det), a, b, tnum, hit);   // Ray.cxx:99
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
        const float x = hit ? t : __builtin_inff();
        // top slot first: each slot's new value is its last reader's, so the
        // list is updated in place
#pragma unroll
        for (int k = kMaxHits - 1; k >= 1; --k) h[k] = __builtin_amdgcn_fmed3f(h[k - 1], h[k], x);
        // min(h[0], x): the values are never NaN, so one plain v_min_f32 (the
        // compiler's fminnum adds a canonicalising v_max of the loop-carried h[0])
        asm("v_min_f32 %0, %1, %2" : "=v"(h[0]) : "v"(h[0]), "v"(x));
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
// Signed hit list of the L-buffer fork (main-pthreads-lbuffer.cxx:778-795):
// the per-hit terms sign(direction . normal) * t kept in triangle order --
// the f32 sum runs in that order -- and the sum of the signs.  Slots hold
// (triangle id, term) ascending by id, 0xFFFFFFFF past the end; n and
// sign_sum count every hit, so a ray with more hits than slots knows it and
// its flag is exact (finish_ray_signed recomputes the sum).
// ---------------------------------------------------------------------------
struct SignedHits {
    uint32_t id[kMaxHits];
    float v[kMaxHits];
    uint32_t n;
    int sign_sum;

    __device__ __forceinline__ void init()
    {
#pragma unroll
        for (int k = 0; k < kMaxHits; ++k) {
            id[k] = 0xFFFFFFFFu;
            v[k] = 0.0f;
        }
        n = 0;
        sign_sum = 0;
    }

    // :791-793  sign = signum(direction . normal), distance += sign * t
    __device__ __forceinline__ void push_if(bool hit, float t, uint32_t tid, int sign)
    {
        if (!hit) return;
        ++n;
        sign_sum += sign;
        uint32_t cid = tid;
        float cv = (float)sign * t;
#pragma unroll
        for (int k = 0; k < kMaxHits; ++k) {   // sorted insert by id (ids are distinct)
            const bool lt = cid < id[k];
            const uint32_t oid = id[k];
            const float ov = v[k];
            id[k] = lt ? cid : oid;
            v[k] = lt ? cv : ov;
            cid = lt ? oid : cid;
            cv = lt ? ov : cv;
        }
    }

    // :778, :792: 0.0f plus the terms in triangle order, sequential f32
    __device__ __forceinline__ float distance() const
    {
        float d = 0.0f;
#pragma unroll
        for (int k = 0; k < kMaxHits; ++k)
            if ((uint32_t)k < n) d += v[k];
        return d;
    }
};

// signum(direction . normal) of the fork (:729-731, :791), Vec3::dotProduct's order.
__host__ __device__ __forceinline__ int hit_sign(float sx, float sy, float sz, float nx, float ny, float nz)
{
    const float dp = (sx * nx + sy * ny) + sz * nz;
    return (int)(0.0f < dp) - (int)(dp < 0.0f);
}

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
    // the special cases as selects over the main path's value (which is
    // computed, and discarded, for them too): no divergent branches
    float out = (float)y;
    if (abstop >= 0x42b) {
        out = x < -0x1.9fe368p6f ? 0.0f : out;                   // underflow
        out = x > 0x1.62e42ep6f ? __builtin_inff() : out;        // overflow
        out = abstop >= 0x7f8 ? x + x : out;                     // +inf or NaN
        out = ix == 0xff800000u ? 0.0f : out;                    // -inf
    }
    return out;
}

// ---------------------------------------------------------------------------
// glibc 2.35 exp (sysdeps/ieee754/dbl-64/e_exp.c with exp_data.c,
// EXP_TABLE_BITS = 7, EXP_POLY_ORDER = 5) as x86-64 glibc dispatches it on FMA
// hardware (e_exp-fma.c: the compiler fuses kd = InvLn2N*x + Shift, the two
// steps of r, the polynomial's multiply-adds and scale + scale*tmp, except in
// the special case's k < 0 branch -- found by the exhaustive check).  The
// function std::exp(double) binds to in src/main-pthreads-lbuffer.cxx:808.
// Table: tools/gen_exp_table.py (equal to the one inside the system libm);
// the function: tests/test_abi.py::test_host_exp_restatement_matches_libm
// (every exponent the signed L-buffer can produce) and the device probe.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t xrt_exp_tab(uint32_t i)
{
    constexpr uint64_t tab[256] = {
        0x0000000000000000ULL, 0x3ff0000000000000ULL, 0x3c9b3b4f1a88bf6eULL, 0x3feff63da9fb3335ULL,
        0xbc7160139cd8dc5dULL, 0x3fefec9a3e778061ULL, 0xbc905e7a108766d1ULL, 0x3fefe315e86e7f85ULL,
        0x3c8cd2523567f613ULL, 0x3fefd9b0d3158574ULL, 0xbc8bce8023f98efaULL, 0x3fefd06b29ddf6deULL,
        0x3c60f74e61e6c861ULL, 0x3fefc74518759bc8ULL, 0x3c90a3e45b33d399ULL, 0x3fefbe3ecac6f383ULL,
        0x3c979aa65d837b6dULL, 0x3fefb5586cf9890fULL, 0x3c8eb51a92fdeffcULL, 0x3fefac922b7247f7ULL,
        0x3c3ebe3d702f9cd1ULL, 0x3fefa3ec32d3d1a2ULL, 0xbc6a033489906e0bULL, 0x3fef9b66affed31bULL,
        0xbc9556522a2fbd0eULL, 0x3fef9301d0125b51ULL, 0xbc5080ef8c4eea55ULL, 0x3fef8abdc06c31ccULL,
        0xbc91c923b9d5f416ULL, 0x3fef829aaea92de0ULL, 0x3c80d3e3e95c55afULL, 0x3fef7a98c8a58e51ULL,
        0xbc801b15eaa59348ULL, 0x3fef72b83c7d517bULL, 0xbc8f1ff055de323dULL, 0x3fef6af9388c8deaULL,
        0x3c8b898c3f1353bfULL, 0x3fef635beb6fcb75ULL, 0xbc96d99c7611eb26ULL, 0x3fef5be084045cd4ULL,
        0x3c9aecf73e3a2f60ULL, 0x3fef54873168b9aaULL, 0xbc8fe782cb86389dULL, 0x3fef4d5022fcd91dULL,
        0x3c8a6f4144a6c38dULL, 0x3fef463b88628cd6ULL, 0x3c807a05b0e4047dULL, 0x3fef3f49917ddc96ULL,
        0x3c968efde3a8a894ULL, 0x3fef387a6e756238ULL, 0x3c875e18f274487dULL, 0x3fef31ce4fb2a63fULL,
        0x3c80472b981fe7f2ULL, 0x3fef2b4565e27cddULL, 0xbc96b87b3f71085eULL, 0x3fef24dfe1f56381ULL,
        0x3c82f7e16d09ab31ULL, 0x3fef1e9df51fdee1ULL, 0xbc3d219b1a6fbffaULL, 0x3fef187fd0dad990ULL,
        0x3c8b3782720c0ab4ULL, 0x3fef1285a6e4030bULL, 0x3c6e149289cecb8fULL, 0x3fef0cafa93e2f56ULL,
        0x3c834d754db0abb6ULL, 0x3fef06fe0a31b715ULL, 0x3c864201e2ac744cULL, 0x3fef0170fc4cd831ULL,
        0x3c8fdd395dd3f84aULL, 0x3feefc08b26416ffULL, 0xbc86a3803b8e5b04ULL, 0x3feef6c55f929ff1ULL,
        0xbc924aedcc4b5068ULL, 0x3feef1a7373aa9cbULL, 0xbc9907f81b512d8eULL, 0x3feeecae6d05d866ULL,
        0xbc71d1e83e9436d2ULL, 0x3feee7db34e59ff7ULL, 0xbc991919b3ce1b15ULL, 0x3feee32dc313a8e5ULL,
        0x3c859f48a72a4c6dULL, 0x3feedea64c123422ULL, 0xbc9312607a28698aULL, 0x3feeda4504ac801cULL,
        0xbc58a78f4817895bULL, 0x3feed60a21f72e2aULL, 0xbc7c2c9b67499a1bULL, 0x3feed1f5d950a897ULL,
        0x3c4363ed60c2ac11ULL, 0x3feece086061892dULL, 0x3c9666093b0664efULL, 0x3feeca41ed1d0057ULL,
        0x3c6ecce1daa10379ULL, 0x3feec6a2b5c13cd0ULL, 0x3c93ff8e3f0f1230ULL, 0x3feec32af0d7d3deULL,
        0x3c7690cebb7aafb0ULL, 0x3feebfdad5362a27ULL, 0x3c931dbdeb54e077ULL, 0x3feebcb299fddd0dULL,
        0xbc8f94340071a38eULL, 0x3feeb9b2769d2ca7ULL, 0xbc87deccdc93a349ULL, 0x3feeb6daa2cf6642ULL,
        0xbc78dec6bd0f385fULL, 0x3feeb42b569d4f82ULL, 0xbc861246ec7b5cf6ULL, 0x3feeb1a4ca5d920fULL,
        0x3c93350518fdd78eULL, 0x3feeaf4736b527daULL, 0x3c7b98b72f8a9b05ULL, 0x3feead12d497c7fdULL,
        0x3c9063e1e21c5409ULL, 0x3feeab07dd485429ULL, 0x3c34c7855019c6eaULL, 0x3feea9268a5946b7ULL,
        0x3c9432e62b64c035ULL, 0x3feea76f15ad2148ULL, 0xbc8ce44a6199769fULL, 0x3feea5e1b976dc09ULL,
        0xbc8c33c53bef4da8ULL, 0x3feea47eb03a5585ULL, 0xbc845378892be9aeULL, 0x3feea34634ccc320ULL,
        0xbc93cedd78565858ULL, 0x3feea23882552225ULL, 0x3c5710aa807e1964ULL, 0x3feea155d44ca973ULL,
        0xbc93b3efbf5e2228ULL, 0x3feea09e667f3bcdULL, 0xbc6a12ad8734b982ULL, 0x3feea012750bdabfULL,
        0xbc6367efb86da9eeULL, 0x3fee9fb23c651a2fULL, 0xbc80dc3d54e08851ULL, 0x3fee9f7df9519484ULL,
        0xbc781f647e5a3ecfULL, 0x3fee9f75e8ec5f74ULL, 0xbc86ee4ac08b7db0ULL, 0x3fee9f9a48a58174ULL,
        0xbc8619321e55e68aULL, 0x3fee9feb564267c9ULL, 0x3c909ccb5e09d4d3ULL, 0x3feea0694fde5d3fULL,
        0xbc7b32dcb94da51dULL, 0x3feea11473eb0187ULL, 0x3c94ecfd5467c06bULL, 0x3feea1ed0130c132ULL,
        0x3c65ebe1abd66c55ULL, 0x3feea2f336cf4e62ULL, 0xbc88a1c52fb3cf42ULL, 0x3feea427543e1a12ULL,
        0xbc9369b6f13b3734ULL, 0x3feea589994cce13ULL, 0xbc805e843a19ff1eULL, 0x3feea71a4623c7adULL,
        0xbc94d450d872576eULL, 0x3feea8d99b4492edULL, 0x3c90ad675b0e8a00ULL, 0x3feeaac7d98a6699ULL,
        0x3c8db72fc1f0eab4ULL, 0x3feeace5422aa0dbULL, 0xbc65b6609cc5e7ffULL, 0x3feeaf3216b5448cULL,
        0x3c7bf68359f35f44ULL, 0x3feeb1ae99157736ULL, 0xbc93091fa71e3d83ULL, 0x3feeb45b0b91ffc6ULL,
        0xbc5da9b88b6c1e29ULL, 0x3feeb737b0cdc5e5ULL, 0xbc6c23f97c90b959ULL, 0x3feeba44cbc8520fULL,
        0xbc92434322f4f9aaULL, 0x3feebd829fde4e50ULL, 0xbc85ca6cd7668e4bULL, 0x3feec0f170ca07baULL,
        0x3c71affc2b91ce27ULL, 0x3feec49182a3f090ULL, 0x3c6dd235e10a73bbULL, 0x3feec86319e32323ULL,
        0xbc87c50422622263ULL, 0x3feecc667b5de565ULL, 0x3c8b1c86e3e231d5ULL, 0x3feed09bec4a2d33ULL,
        0xbc91bbd1d3bcbb15ULL, 0x3feed503b23e255dULL, 0x3c90cc319cee31d2ULL, 0x3feed99e1330b358ULL,
        0x3c8469846e735ab3ULL, 0x3feede6b5579fdbfULL, 0xbc82dfcd978e9db4ULL, 0x3feee36bbfd3f37aULL,
        0x3c8c1a7792cb3387ULL, 0x3feee89f995ad3adULL, 0xbc907b8f4ad1d9faULL, 0x3feeee07298db666ULL,
        0xbc55c3d956dcaebaULL, 0x3feef3a2b84f15fbULL, 0xbc90a40e3da6f640ULL, 0x3feef9728de5593aULL,
        0xbc68d6f438ad9334ULL, 0x3feeff76f2fb5e47ULL, 0xbc91eee26b588a35ULL, 0x3fef05b030a1064aULL,
        0x3c74ffd70a5fddcdULL, 0x3fef0c1e904bc1d2ULL, 0xbc91bdfbfa9298acULL, 0x3fef12c25bd71e09ULL,
        0x3c736eae30af0cb3ULL, 0x3fef199bdd85529cULL, 0x3c8ee3325c9ffd94ULL, 0x3fef20ab5fffd07aULL,
        0x3c84e08fd10959acULL, 0x3fef27f12e57d14bULL, 0x3c63cdaf384e1a67ULL, 0x3fef2f6d9406e7b5ULL,
        0x3c676b2c6c921968ULL, 0x3fef3720dcef9069ULL, 0xbc808a1883ccb5d2ULL, 0x3fef3f0b555dc3faULL,
        0xbc8fad5d3ffffa6fULL, 0x3fef472d4a07897cULL, 0xbc900dae3875a949ULL, 0x3fef4f87080d89f2ULL,
        0x3c74a385a63d07a7ULL, 0x3fef5818dcfba487ULL, 0xbc82919e2040220fULL, 0x3fef60e316c98398ULL,
        0x3c8e5a50d5c192acULL, 0x3fef69e603db3285ULL, 0x3c843a59ac016b4bULL, 0x3fef7321f301b460ULL,
        0xbc82d52107b43e1fULL, 0x3fef7c97337b9b5fULL, 0xbc892ab93b470dc9ULL, 0x3fef864614f5a129ULL,
        0x3c74b604603a88d3ULL, 0x3fef902ee78b3ff6ULL, 0x3c83c5ec519d7271ULL, 0x3fef9a51fbc74c83ULL,
        0xbc8ff7128fd391f0ULL, 0x3fefa4afa2a490daULL, 0xbc8dae98e223747dULL, 0x3fefaf482d8e67f1ULL,
        0x3c8ec3bc41aa2008ULL, 0x3fefba1bee615a27ULL, 0x3c842b94c3a9eb32ULL, 0x3fefc52b376bba97ULL,
        0x3c8a64a931d185eeULL, 0x3fefd0765b6e4540ULL, 0xbc8e37bae43be3edULL, 0x3fefdbfdad9cbe14ULL,
        0x3c77893b4d91cd9dULL, 0x3fefe7c1819e90d8ULL, 0x3c5305c14160cc89ULL, 0x3feff3c22b8f71f1ULL,
    };
    return tab[i & 255u];
}

__host__ __device__ __forceinline__ double xrt_exp_special(double tmp, uint64_t sbits, uint64_t ki)
{
    if ((ki & 0x80000000u) == 0) {              // k > 0: the scale's exponent may have overflowed
        sbits -= 1009ull << 52;
        const double scale = xrt_u64_as_double(sbits);
        return 0x1p1009 * __builtin_fma(scale, tmp, scale);
    }
    sbits += 1022ull << 52;                     // k < 0: subnormal range
    const double scale = xrt_u64_as_double(sbits);
    double y = scale + scale * tmp;
    if (y < 1.0) {
        double lo = scale - y + scale * tmp;
        const double hi = 1.0 + y;
        lo = 1.0 - hi + y + lo;
        y = (hi + lo) - 1.0;
        if (y == 0.0) y = 0.0;                  // no -0.0
    }
    return 0x1p-1022 * y;
}

__host__ __device__ __forceinline__ double xrt_exp(double x)
{
    constexpr double kInvLn2N = 0x1.71547652b82fep0 * 128;
    constexpr double kNegLn2hiN = -0x1.62e42fefa0000p-8;
    constexpr double kNegLn2loN = -0x1.cf79abc9e3b3ap-47;
    constexpr double kShift = 0x1.8p52;
    constexpr double kC2 = 0x1.ffffffffffdbdp-2;
    constexpr double kC3 = 0x1.555555555543cp-3;
    constexpr double kC4 = 0x1.55555cf172b91p-5;
    constexpr double kC5 = 0x1.1111167a4d017p-7;

    const uint64_t ix = xrt_double_as_u64(x);
    uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
    if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {   // |x| < 2^-54, |x| >= 512, inf or NaN
        if (abstop - 0x3c9u >= 0x80000000u) return 1.0 + x;
        if (abstop >= 0x409u) {                 // |x| >= 1024
            if (ix == 0xfff0000000000000ull) return 0.0;
            if (abstop >= 0x7ffu) return 1.0 + x;
            return (ix >> 63) ? 0.0 : __builtin_inf();
        }
        abstop = 0;                             // large |x|: the special case below
    }
    double kd = __builtin_fma(kInvLn2N, x, kShift);
    const uint64_t ki = xrt_double_as_u64(kd);
    kd -= kShift;
    const double r = __builtin_fma(kd, kNegLn2loN, __builtin_fma(kd, kNegLn2hiN, x));
    const uint32_t idx = 2u * (uint32_t)(ki & 127u);
    const uint64_t top = ki << 45;
    const double tail = xrt_u64_as_double(xrt_exp_tab(idx));
    const uint64_t sbits = xrt_exp_tab(idx + 1u) + top;
    const double r2 = r * r;
    const double tmp = __builtin_fma(r2 * r2, __builtin_fma(r, kC5, kC4),
                                     __builtin_fma(r2, __builtin_fma(r, kC3, kC2), tail + r));
    if (abstop == 0) return xrt_exp_special(tmp, sbits, ki);
    const double scale = xrt_u64_as_double(sbits);
    return __builtin_fma(scale, tmp, scale);
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

// The fork's L-buffer update for mesh 0 (main-pthreads-lbuffer.cxx:805-808):
// L = 80 (its initial value, :314) times exp(-(mu * (distance * 0.1))) in f64,
// rounded to f32; -1 when the signs do not cancel.  A NaN distance (x86's
// default NaN from inf - inf or 0 * inf) gives 0x7FC00000 there: the f64
// negation flips its sign before exp returns it.
constexpr uint32_t kX86SignedNaN = 0x7FC00000u;
__host__ __device__ __forceinline__ float signed_lbuffer(float distance, int sign_sum, float mu)
{
    if (sign_sum != 0) return -1.0f;
    if (distance != distance) return xrt_f32_from_bits(kX86SignedNaN);
    return (float)((double)80.000f * xrt_exp(-((double)mu * ((double)distance * 0.1))));
}

// 8-bit image: Image::applyLUT's per-pixel formula (include/Image.inl:195-211)
// with vmin = 0, vmax = 80; NaN (undefined in the reference) maps to 0.
__host__ __device__ __forceinline__ uint8_t lut_u8(float v)
{
    const float vmin = 0.0f, vmax = 80.0f;
    // 255.0 * v / 80.0 == v * 3.1875 exactly (below); for x = v * 3.1875 >= 0
    // (at most 30 significant bits, < 256) x + 0.5 is exact, so round-half-
    // away-from-zero is floor(x + 0.5).  Selects instead of branches; the
    // product is computed, and discarded, for out-of-range v and NaN.
    const uint32_t r = (uint32_t)__builtin_floor((double)v * 3.1875 + 0.5);
    return v > vmax ? (uint8_t)255u : v >= vmin ? (uint8_t)r : (uint8_t)0u;
}

}  // namespace XRT_KERNEL_NS
