/*
 * xrt_debug.h -- test hooks, device probes and diagnostics of libxrt.so.
 *
 * Not part of the drop-in boundary (include/xrt.h): the parity tests, the
 * benchmark's measurement tools and the CPU test suite use these to reach
 * the exact device code paths (Ray::intersect, expf, the LUT, k_prep), to
 * force the rare exact paths (hit-list overflow, list overflow, fill-plan
 * fallback) and to read the pipeline's counters and timing records.
 */
#ifndef XRT_DEBUG_H
#define XRT_DEBUG_H

#include "xrt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* --- device probes of the exact device code paths ----------------------- */

/*
 * Runs the kernel's Ray::intersect (src/Ray.cxx:72-124) on the device:
 * rays[6*i] = origin xyz, unit direction xyz; triangles[9*i] = p1, p2, p3.
 * hit[i] = 0/1, t[i] = distance (0 when no hit).  Host buffers.
 */
int xrt_probe_intersect(xrt_context* ctx, const float* rays, const float* triangles,
                        uint64_t n, uint8_t* hit, float* t);

typedef enum xrt_probe_op {
    XRT_PROBE_EXPF = 0,     /* std::exp(float) == glibc expf                     */
    XRT_PROBE_SQRTF = 1,    /* std::sqrt(float), correctly rounded               */
    XRT_PROBE_RCP = 2,      /* (float)(1.0 / (double)x), src/Ray.cxx:99           */
    XRT_PROBE_LUT_U8 = 3,   /* 8-bit LUT of a photon value (out[i] = (float)u8)  */
    XRT_PROBE_RCP_FAST = 4, /* the culled tests' 1/det (rcp + Newton where exact) */
    XRT_PROBE_SIGNED_L = 5  /* (float)(80.0 * exp(-(0.1037f * (d * 0.1)))): the signed
                               model's L for distance d (glibc exp in f64)          */
} xrt_probe_op;

/* Evaluates one scalar device function elementwise.  Host buffers. */
int xrt_probe_math(xrt_context* ctx, int op, const float* in, float* out, uint64_t n);

/*
 * Runs the per-render triangle preparation (k_prep) of the uploaded mesh for
 * `camera` and copies its outputs to the host: records[16*i] = edge1, edge2,
 * tvec, qvec, t*det, pad (the ray-independent terms of Ray::intersect,
 * src/Ray.cxx:86-122) and footprint[16*i] = bbox (xmin, xmax, ymin, ymax) and
 * the three relaxed edge functions (a, b, c, 0) of the tile cull.  Either
 * output may be NULL.
 */
int xrt_probe_prep(xrt_context* ctx, const xrt_camera* camera, float* records, float* footprint);

/*
 * Host-side evaluation of the device expf restatement (the same source,
 * compiled for the host): lets CPU-only tests check it against libm.
 */
void xrt_host_expf_batch(const float* in, float* out, uint64_t n);

/*
 * The same for the signed model: the device glibc exp restatement, and its L
 * update (float)(80.0 * exp(-(mu * (distance * 0.1)))) (-1 for a non-zero
 * sign sum; sign_sum may be NULL for all zero).
 */
void xrt_host_exp_batch(const double* in, double* out, uint64_t n);
void xrt_host_signed_lbuffer_batch(const float* distance, const int32_t* sign_sum, float mu, float* out,
                                   uint64_t n);

/*
 * Test hook: caps the per-ray register hit list at `capacity` (1..12) so the
 * exact overflow path runs.  0 restores the default (12).
 */
int xrt_set_hit_capacity(xrt_context* ctx, uint32_t capacity);

/*
 * Test hook: caps the BINNED kernel's region-list capacity at `entries` so the
 * whole-mesh fallback runs.  0 restores automatic sizing.
 */
int xrt_set_bin_capacity(xrt_context* ctx, uint64_t entries);

/*
 * The BINNED kernel's fill plan (DESIGN.md "Fill plan"): regions whose lists
 * the geometry's sizing frame counted empty render as one miss-filling
 * workgroup each instead of 16 tile waves.  mode 1 (default) on, 0 off;
 * test hook 2 plans every region as empty, so every workgroup takes the
 * exact fallback of a region that is not.  The next frame re-sizes (after a
 * camera change under the same image size and strip the context keeps its
 * lists and plan instead: DESIGN.md "Moving camera").
 */
int xrt_set_fill_plan(xrt_context* ctx, int mode);

/* Diagnostics: regions the last enqueued BINNED frame rendered through the fill plan. */
int xrt_debug_fill_regions(xrt_context* ctx, uint32_t* regions);

/*
 * Diagnostics: BINNED frames by geometry path since the context was created --
 * counters[0] frames whose lists were sized synchronously (a new frame
 * geometry), [1] frames rendered over lists sized for another camera of the
 * same region grid (a moving camera), [2] frames k_prep flagged for a fill-plan
 * miss, [3] frames k_prep flagged for a list overflow.
 */
int xrt_debug_geometry_counters(xrt_context* ctx, uint64_t counters[4]);

/*
 * Diagnostics: counters[0] = host-buffer frames (xrt_render_rows) of a geometry
 * seen for the first time that were sized on the device (the count pass, one
 * 32-byte read-back of its pair
 * total, the lists carved and filled by k_size_lists / k_scatter_pairs; no
 * host plan, no second k_prep; XRT_DEVICE_FIRST=0 turns it off), [1] = those
 * whose pool was too small for the pair total, grown and counted again, [2] /
 * [3] = the last such frame's pair total and the pool its count pass had.
 */
int xrt_debug_first_frames(xrt_context* ctx, uint64_t counters[4]);

/*
 * Diagnostics: the frame pipeline since the context was created --
 * counters[0] frames rendered from a preparation made ahead of their call
 * (xrt_render_rows_device repeating its frame geometry), [1] preparations made
 * ahead and dropped (the next call's geometry or settings differed), [2]
 * renders launched with their preparation already complete (no wait), [3]
 * renders launched after the host read k_prep's check (sizing / validation).
 */
int xrt_debug_pipeline_counters(xrt_context* ctx, uint64_t counters[4]);

/*
 * Diagnostics: copies the last render's statistics records (32 bytes each, one
 * per workgroup -- per tile wave for BINNED: u32 rays, hit rays, odd rays,
 * overflow rays, hits, wave-level triangle tests, candidates, max hits)
 * into `dst`, at most `capacity` bytes; `*n_records` receives the number of
 * records.
 */
int xrt_debug_block_records(xrt_context* ctx, void* dst, uint64_t capacity, uint64_t* n_records);

/*
 * Diagnostics: the timing records of the render `frames_back` frames before
 * the last (0 = the last; up to XRT_FRAME_SETS - 1 = 3; after a timed region too), one per statistics
 * record (u32 s_memrealtime start, u32 end; 100 MHz, low 32 bits), into `dst`,
 * at most `capacity` records; `*n_records` receives their number.
 */
int xrt_debug_wave_times(xrt_context* ctx, uint32_t frames_back, uint32_t* dst, uint64_t capacity,
                         uint64_t* n_records);


/*
 * Test hook (host code, no device): for each i, the culled render's
 * division-free reject mt_may_hit(det, a, b, tnum) and the exact remainder of
 * Ray::intersect from the same numerators (hit with t > 1e-7, and t).
 */
void xrt_host_mt_check(const float* det, const float* a, const float* b, const float* tnum, uint64_t n,
                       uint8_t* may_hit, uint8_t* hit, float* t);

/*
 * Diagnostics: host time of the last xrt_render_rows call (host buffers), ms:
 * ms[0] device planes (allocated once per size), [1] enqueue (preparation,
 * list sizing of a new geometry, launch), [2] wait for the render, [3] D2H of
 * the planes (DMA into the context's pinned ring, overlapped with its copy
 * threads moving the pieces into the caller's pages), [4] copy threads (a
 * count), [5] MB copied, [6] statistics, [7] total; within them [8] the time
 * in hipMalloc, [9] a new frame geometry's list sizing, [10] synchronisations
 * before a launch layout's upload (only when frames in flight may read it) --
 * [13] of which the prep stream's, [14] the buffer sets' render events',
 * [15] the last stream's --, [11] host waits for the preparation (k_prep),
 * [12] kernel launches.
 */
int xrt_debug_host_call_ms(xrt_context* ctx, double ms[16]);

/*
 * Diagnostics: [0] binned frames rendered with a tile plan (tiles that had no
 * survivor in an earlier frame of the same geometry store their misses without
 * reading the region's list), [1] tile plans taken.
 * The plan is OFF by default (it reuses an earlier frame's cull results, so
 * it only helps a loop of identical frames); XRT_TILE_PLAN=1 in the
 * environment at xrt_create, or xrt_debug_set_tile_plan, turns it on.
 */
int xrt_debug_tile_plan(xrt_context* ctx, uint64_t counters[2]);

/*
 * Host code (no device): the cull's direction grid of `camera` (DESIGN.md
 * section 5, step 0) as the library computes it -- grids[0], a bisection per
 * axis -- and by a scan of every row or column, grids[1].  Equal for every
 * camera (the test's claim).
 */
int xrt_debug_direction_grid(const xrt_camera* camera, int grids[2]);

/* Turns the tile plan on (1) or off (0) for later frames. */
int xrt_debug_set_tile_plan(xrt_context* ctx, int on);

/*
 * Diagnostics: k_prep's per-wave timestamps.  enable 1 / 0 turns the records
 * on / off for later launches (-1 leaves it); *n_waves = the waves of the last
 * recorded launch; with dst, waits for the context's work and copies up to
 * `capacity` records of 8 u32 (s_memrealtime, 100 MHz, low 32 bits): the
 * wave's start, its triangle's record formed, its footprint, the binning's LDS
 * staging and scan, the union of its rectangles, small then large rectangles'
 * cells tested, its end.
 */
int xrt_debug_prep_times(xrt_context* ctx, int enable, uint32_t* dst, uint64_t capacity, uint64_t* n_waves);

/*
 * Diagnostics: the phases of the last xrt_destroy, ms: [0] waiting for the
 * context's own work, [1] device frees, [2] pinned host frees, [3] streams and
 * events destroyed.
 */
int xrt_debug_destroy_ms(double ms[4]);

/*
 * Diagnostics of a multi context's transit (xrt_multi_set_transit): [0]
 * frames whose strips travelled in the hit layout, [1] frames that travelled
 * packed, [2] bytes the last frame sent into device 0, [3] 1 when a received
 * hit mask disagreed with its sender's plan (waits for the last gather).
 */
int xrt_multi_transit_stats(xrt_multi* m, uint64_t out[4]);

/*
 * Diagnostics of a multi context's balanced split (xrt_multi_set_split): [0]
 * balanced plans made (each from the strips' own records of an earlier
 * frame -- no extra render), [1] frames split equally because no such model
 * existed yet (the first frame), [2] link probes run (at most one per gather
 * path), [3] strip models collected (one per new camera).
 */
int xrt_multi_plan_stats(xrt_multi* m, uint64_t out[4]);

/*
 * Test hook: the expected hit count of the first tile of the first sender's
 * hit plan plus one, so the next hit frame's receive disagrees with its plan
 * (the mismatch path: the frame's call fails, the plans are made again).
 */
int xrt_multi_debug_corrupt_hit_plan(xrt_multi* m);

#ifdef __cplusplus
}
#endif

#endif /* XRT_DEBUG_H */
