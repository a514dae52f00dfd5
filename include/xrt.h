/*
 * xrt.h -- C ABI of the MI355X-native X-ray attenuation render path.
 *
 * This is the drop-in boundary for the reference's per-pixel render loop
 * (Brandagot/SimpleRayTracing):
 *
 *   void renderLoop(Image&, const vector<TriangleMesh>&, RayTracerInfo&)
 *       declared src/main.cxx:159-161, defined src/main.cxx:626-743,
 *       called   src/main.cxx:237
 *   void* renderLoopCallBack(void*)   (pixel-range twin)
 *       src/main-pthreads-redo.cxx:660-771, PThreadData :184-213
 *
 * src/main-cuda.cxx (0 bytes) marks where the reference expected a GPU
 * driver; this ABI fills that slot.  The C++ host library in
 * simpleraytracing_amd/csrc/host keeps the reference's renderLoop signature and
 * calls these entry points; INTEGRATION.md shows the binding a maintainer adds.
 *
 * Conventions
 *   - Plain C types only.  Every function returns an xrt_status (0 = OK);
 *     xrt_last_error() gives the message.  Nothing throws across the ABI
 *     (the reference throws std::runtime_error / std::out_of_range, which the
 *     C++ host re-raises: main() exits 1 with "ERROR: ...", main.cxx:243-247).
 *   - Image buffers are row-major, index (row - row_begin) * width + col, as
 *     Image::setPixel (include/Image.inl:139-160) with a strip offset.
 *   - One context per device; a context is not thread-safe (the reference's
 *     threads write disjoint pixels of one Image, main-pthreads-redo.cxx:332).
 *
 * Output semantics (bit-exact with the reference):
 *   image    f32  photonOut = 80 * expf(-(0.3971 * (float)(L * 0.1)))   main.cxx:725,739
 *   lbuffer  f32  L = sum of sorted pair differences of the ray's hit
 *                 distances (main.cxx:700-718); 0 for an odd hit count;
 *                 +inf for a ray that hits nothing (z_buffer init, :646)
 *   image_u8 u8   round(255 * image / 80), clamped -- Image::applyLUT's
 *                 per-pixel formula (include/Image.inl:195-211), vmin 0, vmax 80
 */
#ifndef XRT_H
#define XRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XRT_ABI_VERSION 5

typedef enum xrt_status {
    XRT_OK = 0,
    XRT_ERR_ARGUMENT = 1,   /* bad pointer / size / row range (Image::setPixel's out_of_range) */
    XRT_ERR_DEVICE = 2,     /* HIP runtime failure */
    XRT_ERR_NO_MESH = 3,    /* render before xrt_upload_mesh */
    XRT_ERR_OVERFLOW = 4,   /* internal capacity exceeded */
    XRT_ERR_IO = 5,         /* file could not be read / written */
    XRT_ERR_FORMAT = 6      /* malformed input file */
} xrt_status;

/* Kernel selection. */
typedef enum xrt_kernel {
    XRT_KERNEL_AUTO = 0,    /* TILED, or BINNED when T x regions > 2e7 */
    XRT_KERNEL_BRUTE = 1,   /* every ray tests every triangle (renderLoop as written) */
    XRT_KERNEL_TILED = 2,   /* every 32x32 region sweeps every triangle's conservative
                               footprint; per 8x8 ray tile the survivors of a relaxed
                               edge-function test get the exact Moller-Trumbore test */
    XRT_KERNEL_BINNED = 3   /* as TILED, but footprints are binned to regions once per
                               frame (atomic slots in fixed-capacity region lists)
                               instead of swept per region */
} xrt_kernel;

/*
 * Camera: RayTracerInfo (src/main.cxx:111-121, built by initialiseRayTracing
 * :566-622) plus the pixel spacing computed in renderLoop's prologue
 * (:634-641) and the image size.
 */
typedef struct xrt_camera {
    float origin[3];        /* point source              RayTracerInfo::origin            */
    float detector[3];      /* detector centre           RayTracerInfo::detector_position */
    float up[3];            /* detector "v" axis         RayTracerInfo::up                */
    float right[3];         /* detector "u" axis         RayTracerInfo::right             */
    float pixel_spacing;    /* 2 * max(range_z / W, range_y / H)  main.cxx:639-641         */
    uint32_t width;         /* Image::getWidth()                                           */
    uint32_t height;        /* Image::getHeight()                                          */
} xrt_camera;

/* Per-render counters (the reference prints one line per odd ray, main.cxx:710). */
typedef struct xrt_stats {
    uint64_t rays;          /* rays rendered */
    uint64_t hit_rays;      /* rays with >= 1 hit on mesh 0 */
    uint64_t odd_rays;      /* rays with an odd hit count ("Only one intersect on this ray") */
    uint64_t overflow_rays; /* rays whose hit list exceeded the register list (resolved exactly) */
    uint64_t hits;          /* total recorded intersections */
    uint32_t max_hits;      /* largest per-ray hit count */
    uint32_t kernel;        /* xrt_kernel actually used */
    double kernel_ms;       /* the last render kernel's span (its waves' s_memrealtime records) */
    uint64_t candidates;    /* TILED: triangles kept by the region footprint test, summed over regions */
    uint64_t tile_tests;    /* triangle tests issued per 8x8 wave tile (64 ray-triangle tests each) */
    uint64_t global_triangles; /* BINNED: footprints too large for the region lists (every region's candidates) */
} xrt_stats;

typedef struct xrt_context xrt_context;

/* --- lifetime ----------------------------------------------------------- */

/* Creates a context on HIP device `device`. */
int xrt_create(int device, xrt_context** out);
void xrt_destroy(xrt_context* ctx);
/* Last error message of `ctx` (or of the last failed xrt_create when ctx is NULL). */
const char* xrt_last_error(const xrt_context* ctx);
int xrt_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int xrt_device_count(void);

/* --- mesh ---------------------------------------------------------------- */

/*
 * Uploads mesh 0 as a triangle soup: triangles[9*i .. 9*i+8] = p1, p2, p3 of
 * TriangleMesh::getTriangle(i) (include/TriangleMesh.inl:208, Triangle.h:125-127).
 * Only mesh 0 contributes to the image (the mesh filter at main.cxx:687), so the
 * host uploads meshes[0] only.  Replaces any previous mesh; num_triangles may be 0.
 */
int xrt_upload_mesh(xrt_context* ctx, const float* triangles, uint64_t num_triangles);

/* --- camera (host-side arithmetic, no device needed) ---------------------- */

/*
 * Bounding box of a triangle soup: TriangleMesh::computeBoundingBox
 * (src/TriangleMesh.cxx:192-228) / getBBox (src/main.cxx:538-563).
 */
int xrt_mesh_bbox(const float* triangles, uint64_t num_triangles, float lower[3], float upper[3]);

/*
 * Bounding box of a scene of several meshes: getBBox over each mesh's
 * computeBoundingBox (src/main.cxx:538-563).  tris holds the meshes' soups one
 * after another; mesh_triangles[m] is mesh m's triangle count.  The camera
 * comes from the box of every mesh (main.cxx:634), while only mesh 0 is
 * uploaded -- the only mesh whose hits count (main.cxx:687).
 */
int xrt_scene_bbox(const float* tris, const uint64_t* mesh_triangles, uint32_t num_meshes, float lower[3],
                   float upper[3]);

/*
 * Camera from the scene bounding box: initialiseRayTracing (main.cxx:566-622)
 * and renderLoop's pixel spacing (main.cxx:634-641), f32/f64 rounding as written.
 */
int xrt_camera_from_bbox(const float lower[3], const float upper[3], uint32_t width,
                         uint32_t height, xrt_camera* out);

/* --- render --------------------------------------------------------------- */

int xrt_set_kernel(xrt_context* ctx, int kernel);

/*
 * Renders image rows [row_begin, row_end) of camera->width x camera->height.
 * HOST buffers (any may be NULL), each (row_end-row_begin)*width elements.
 * Synchronous.  renderLoop == xrt_render_rows(ctx, cam, 0, H, image, ...).
 */
int xrt_render_rows(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin,
                    uint32_t row_end, float* image, float* lbuffer, uint8_t* image_u8,
                    xrt_stats* stats);

/*
 * Same with DEVICE buffers on HIP stream `stream` (hipStream_t, NULL = default
 * stream).  Asynchronous: returns once the render is enqueued.  The frame's
 * preparation (k_prep) runs on the context's own prep stream, beside earlier
 * renders; the render waits for it on the device.  The host waits only when
 * the frame geometry is new (its region lists are sized from a synchronous
 * count, and the first frame over them is checked), when the frame reuses
 * lists sized for another camera (k_prep's check decides its launch), and
 * when four frames are already in flight (for the oldest).  When a call
 * repeats the previous call's frame geometry (mesh, camera, rows) and
 * settings, the preparations of the next two frames of that geometry are
 * enqueued at once; a later call that matches takes one (rendered with no
 * wait), any other call drops them.  Renders enqueued on different streams
 * (each into its own buffers) may run at once: every frame's lists, records
 * and statistics live in its own buffer set.  Call xrt_read_stats() (which
 * synchronises the last frame's stream) for counters and kernel time.
 */
int xrt_render_rows_device(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin,
                           uint32_t row_end, float* d_image, float* d_lbuffer,
                           uint8_t* d_image_u8, void* stream);

/*
 * Counters and kernel time of the last render.  Enqueues a small reduction
 * kernel (k_reduce_stats) on that render's stream and waits for it: call it
 * after a sequence of frames, not between frames in flight.
 */
int xrt_read_stats(xrt_context* ctx, xrt_stats* stats);

/*
 * Many frames of one geometry (camera, rows) in one call -- a series of
 * projections of a fixed set-up, or a throughput run.  Frame k (k = 0 ..
 * n_frames-1) renders into plane set s = k % n_sets -- d_image[s],
 * d_lbuffer[s], d_u8[s] (device pointers; a NULL array or entry skips that
 * plane) -- on stream streams[s] (hipStream_t; a NULL array or entry is the
 * default stream).  Each frame is prepared and rendered as by one
 * xrt_render_rows_device call (its own k_prep, prepared ahead beside earlier
 * renders; nothing is reused between frames), with the host side of all
 * n_frames frames done in one pass: no per-frame crossing of the boundary,
 * which at 1024^2 costs about as much host time as the GPU's frame.
 * Asynchronous, like xrt_render_rows_device.  Replaces the caller's loop
 * around renderLoop (src/main.cxx:237) for a batch of frames.
 */
int xrt_render_frames_device(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin, uint32_t row_end,
                             uint32_t n_frames, uint32_t n_sets, float* const* d_image, float* const* d_lbuffer,
                             uint8_t* const* d_u8, void* const* streams);

/*
 * The host-buffer form: n_frames frames rendered back to back into the
 * context's device planes, then the last frame's planes copied into the host
 * buffers (any may be NULL) as xrt_render_rows does.  *ms_per_frame (may be
 * NULL) = host wall time from the first frame's enqueue to the last frame's
 * completion, / n_frames.  Synchronous.
 */
int xrt_render_frames(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin, uint32_t row_end,
                      uint32_t n_frames, float* image, float* lbuffer, uint8_t* image_u8, xrt_stats* stats,
                      double* ms_per_frame);

/*
 * Kernel timing over a region of many renders without host synchronisation.
 * A begin while a region is open ends that region first (its results are
 * dropped).  The record space is sized from the context's last frame, and
 * from the region's first frame when that is larger.
 * Every render's waves store their s_memrealtime start and end beside their
 * statistics records (xrt_stats::kernel_ms is the last frame's span: last end -
 * first start).  After xrt_timing_begin, every render keeps its records apart
 * (up to 2^27 records, 1 GiB, per region); xrt_timing_end synchronises the
 * device and returns the summed spans of those renders and their number.  Every 16th render of the region also
 * carries a HIP start/stop event pair on its dispatch: xrt_timing_events
 * returns their summed durations and number (a cross-check; a start event
 * costs its frame a few microseconds).
 */
int xrt_timing_begin(xrt_context* ctx);
int xrt_timing_end(xrt_context* ctx, double* total_ms, uint64_t* launches);
int xrt_timing_events(xrt_context* ctx, double* total_ms, uint64_t* launches);

/* --- strips in transit ---------------------------------------------------- */

/*
 * The L-buffer alone determines a pixel's image and 8-bit values (image =
 * shade(L) for a hit, 80 for a miss), except that a miss and a ray with a t =
 * +inf "hit" both have L = +inf.  Strips gathered to another device travel as
 * L-buffers with misses written as XRT_MISS_TRANSIT (a signalling NaN no render
 * produces): 4 bytes per pixel instead of 9.
 */
#define XRT_MISS_TRANSIT 0x7F800001u

/* L-buffer bits of a miss for later renders: 0 (+inf, the default) or XRT_MISS_TRANSIT. */
int xrt_set_miss_code(xrt_context* ctx, uint32_t bits);

/*
 * Expands num_pixels of a received L-buffer (misses as XRT_MISS_TRANSIT) in
 * place: d_image / d_u8 (either may be NULL) get the pixels' image and 8-bit
 * values and the miss codes become +inf -- bit-identical to a direct render.
 * Asynchronous on `stream` (device buffers).
 */
int xrt_expand_rows_device(xrt_context* ctx, uint64_t num_pixels, float* d_lbuffer, float* d_image,
                           uint8_t* d_image_u8, void* stream);

/* --- the signed multi-material L-buffer (the L-buffer fork) --------------- */

/*
 * What renders compute per ray:
 *   XRT_MODEL_ATTENUATION  renderLoop, src/main.cxx:626-743 (the default):
 *                          image, L-buffer and 8-bit planes as above.
 *   XRT_MODEL_SIGNED       renderLoopCallBack of src/main-pthreads-lbuffer.cxx
 *                          (:733-813): per ray, distance = the sum of
 *                          sign(direction . normal) * t over the mesh-0 hits
 *                          in triangle order (f32), L = 80 * exp(-(mu *
 *                          (distance * 0.1))) in f64 (glibc exp), or -1 when
 *                          the signs do not cancel (:805-806).  Renders write
 *                          the L-buffer plane only (image and u8 must be NULL);
 *                          xrt_hole_fill makes the image.  Kernels: BRUTE or
 *                          BINNED (AUTO picks BINNED).
 * mu: mesh 0's attenuation coefficient, 0.1037f in the fork (soft tissue,
 * :800).  Other meshes add no hits (the mesh-0 filter, :788), so their
 * coefficient (0.3971f, :802) multiplies L by exp(-0.0) = 1.
 */
#define XRT_MODEL_ATTENUATION 0
#define XRT_MODEL_SIGNED 1
int xrt_set_model(xrt_context* ctx, int model, float mu);

/*
 * The fork's hole fill (main-pthreads-lbuffer.cxx:327-404) over a whole
 * width x height L-buffer: pixels flagged -1 become the mean of the first
 * unflagged non-zero value within 4 steps in each of four directions; others
 * keep their value.  Writes image (f32) and/or image_u8 (the LUT of
 * image_u8's plane above).  Host buffers, synchronous; _device: device
 * buffers, asynchronous on `stream`.
 */
int xrt_hole_fill(xrt_context* ctx, uint32_t width, uint32_t height, const float* lbuffer, float* image,
                  uint8_t* image_u8);
int xrt_hole_fill_device(xrt_context* ctx, uint32_t width, uint32_t height, const float* d_lbuffer,
                         float* d_image, uint8_t* d_image_u8, void* stream);

/*
 * The fork end to end on the whole frame (XRT_MODEL_SIGNED): render, hole
 * fill; host buffers (any may be NULL): image = the fork's output image,
 * lbuffer = its L_buffer (-1 flags), image_u8 = the image's LUT.  stats.odd_rays
 * counts the flagged rays.
 */
int xrt_render_signed(xrt_context* ctx, const xrt_camera* camera, float* image, float* lbuffer,
                      uint8_t* image_u8, xrt_stats* stats);

/* --- multi-GPU: row strips + RCCL root gather (one process) --------------- */

/*
 * The image split into contiguous row strips over several devices, as the
 * reference's parallel drivers split the pixel index space
 * (src/main-pthreads-rows.cxx:311-334, src/main-mpi.cxx:262-290; see
 * xrt_multi_set_split for the two rules).  Strip g renders on devices[g]; the
 * strips' planes are gathered into device 0's frame with grouped ncclSend /
 * ncclRecv over xGMI -- the analogue of the MPI root gather of
 * src/main-mpi.cxx:855-881 -- on one communicator per device
 * (ncclCommInitAll).  A device listed more than once (rehearsing the strip
 * logic on fewer GPUs) gathers with device copies instead.
 */
typedef struct xrt_multi xrt_multi;

int xrt_multi_create(const int* devices, int num_devices, xrt_multi** out);
void xrt_multi_destroy(xrt_multi* m);
const char* xrt_multi_last_error(const xrt_multi* m);
int xrt_multi_num_devices(const xrt_multi* m);
/* The mesh, replicated on every device (xrt_upload_mesh). */
int xrt_multi_upload_mesh(xrt_multi* m, const float* triangles, uint64_t num_triangles);
int xrt_multi_set_kernel(xrt_multi* m, int kernel);

/*
 * Renders the whole camera->height x width frame as strips and gathers it into
 * HOST buffers (any may be NULL).  Synchronous.  `stats` sums the devices'.
 * renderLoop over n GPUs == xrt_render_rows_multi(m, cam, image, ...).
 */
int xrt_render_rows_multi(xrt_multi* m, const xrt_camera* camera, float* image, float* lbuffer,
                          uint8_t* image_u8, xrt_stats* stats);

/*
 * The same into device-0 DEVICE buffers (full-frame planes; NULL planes are
 * neither rendered nor gathered), ordered on device 0's HIP stream `stream`.
 * Asynchronous: the next frame's strips render while this frame's gather is
 * in flight (double-buffered strip planes).
 */
int xrt_render_rows_multi_device(xrt_multi* m, const xrt_camera* camera, float* d_image,
                                 float* d_lbuffer, uint8_t* d_image_u8, void* stream);

/*
 * The per-ray model of every device (xrt_set_model).  With XRT_MODEL_SIGNED the
 * gathered planes are the fork's: lbuffer = its L_buffer, image / image_u8 =
 * the hole-filled image (device 0 fills the assembled frame).
 */
int xrt_multi_set_model(xrt_multi* m, int model, float mu);

/* Waits for the last frame's gathers; the devices' statistics, summed. */
int xrt_multi_read_stats(xrt_multi* m, xrt_stats* stats);

/*
 * How the strips reach device 0.  XRT_GATHER_AUTO (the default): RCCL when
 * every listed device is distinct, device copies when one is listed twice.
 * XRT_GATHER_RCCL on a list that names ONE device n times (a one-GPU
 * rehearsal) gathers through a one-rank RCCL communicator on that device --
 * grouped ncclSend / ncclRecv from the rank to itself, the same calls and
 * stream order as the distinct-device gather.  XRT_GATHER_COPY forces copies.
 * A list that mixes repeated and distinct devices gathers with copies.
 */
#define XRT_GATHER_AUTO 0
#define XRT_GATHER_COPY 1
#define XRT_GATHER_RCCL 2
int xrt_multi_set_gather(xrt_multi* m, int mode);

/*
 * What a sender's strip sends to device 0 (attenuation model).
 * XRT_TRANSIT_HITS (the default): once a strip geometry repeats (the same
 * camera, rows, mesh and kernel as the sender's previous frame), per 8x8 tile
 * of the regions its fill plan leaves a 64-bit hit mask and the hit rays' L
 * values, rendered straight into that layout (xrt_set_transit_hits; the plan
 * is made once per geometry, synchronously); a frame of a new geometry sends
 * the packed layout.  XRT_TRANSIT_PACKED: always the 32x32 blocks of the
 * regions the fill plan leaves (xrt_set_transit_layout's layout).  A received
 * hit mask that disagrees with its sender's plan fails the call that sees it
 * (xrt_render_rows_multi: that frame; the device entry: its next call) with
 * XRT_ERR_DEVICE and drops the hit plans (the next frames travel packed, then
 * plan again).
 */
#define XRT_TRANSIT_PACKED 0
#define XRT_TRANSIT_HITS 1
int xrt_multi_set_transit(xrt_multi* m, int mode);

/*
 * How the rows are split over the devices.
 *   XRT_SPLIT_EQUAL     rows_per = H / n, the remainder going to the first
 *                       strips, strip g = device g in frame order -- the
 *                       reference's row rule (src/main-pthreads-rows.cxx:311-334).
 *   XRT_SPLIT_BALANCED  (the default) the gather bounds a multi-GPU frame: a
 *                       sender's rows cost their transfer over ONE link into
 *                       device 0, device 0's rows only their render.  Device 0
 *                       renders ONE run of 32-row bands anywhere in the frame,
 *                       devices 1 .. n-1 the bands above it, then below it, in
 *                       frame order, so that max(device 0's render + unpack,
 *                       each sender's max(render, bytes / link)) is least
 *                       (xrt_balanced_bounds).  The model comes from the
 *                       strips' own renders of an earlier frame -- per band the
 *                       wave time of its regions (timing records, summed on each
 *                       device behind its render of a new camera) and its
 *                       transit bytes -- never from an extra render; the first
 *                       frame of a multi context has no model and splits
 *                       equally.  Link rate: link_bytes_per_us when > 0, else
 *                       measured once per context and gather path (every sender
 *                       sends 4 MB to device 0 at once through the context's
 *                       gather) when a balanced plan is first made.  A camera
 *                       keeps its plan; a new camera plans from the latest
 *                       complete model without waiting.  The signed model, and
 *                       frames with fewer bands than devices, split equally.
 * Every split is exact: the gathered frame equals one device's frame.
 */
#define XRT_SPLIT_EQUAL 0
#define XRT_SPLIT_BALANCED 1
int xrt_multi_set_split(xrt_multi* m, int mode, double link_bytes_per_us);

/*
 * The strips of `camera`'s frame (planned now from the latest strip model when
 * the camera is new; the equal split, info zeros, before any frame):
 * bounds[2g], bounds[2g+1] = [begin, end) rows of device g's strip (2n
 * entries).  info (may be NULL): [0] the link rate the plan used (bytes per
 * microsecond), [1] the modelled frame's render span (us), [2] the step the
 * plan predicts (us); zeros for an equal split.
 */
int xrt_multi_plan(xrt_multi* m, const xrt_camera* camera, uint32_t* bounds, double* info);

/*
 * The balanced split as host arithmetic (no device): band_cost[b] = render time
 * of band b (us), band_bytes[b] = the bytes band b's strip sends to device 0,
 * n devices, link rate in bytes per microsecond, `band_rows` rows per band
 * (the last band may be shorter: rows are clamped to `height`), unpack_us =
 * device 0's per-frame unpack.  bounds: 2n entries as xrt_multi_plan's;
 * *step_us (may be NULL) = the step the split implies.  XRT_ERR_ARGUMENT when
 * there are fewer bands than devices.
 */
int xrt_balanced_bounds(const double* band_cost, const double* band_bytes, uint32_t n_bands, uint32_t n,
                        double link_bytes_per_us, uint32_t height, uint32_t band_rows, double unpack_us,
                        uint32_t* bounds, double* step_us);

/* --- region-packed transit (multi-GPU gathers) ---------------------------- */

/*
 * Region-packed strips for multi-GPU gathers (DESIGN.md "Multi-GPU").  A strip
 * rendered as an L-buffer with misses coded XRT_MISS_TRANSIT travels as the
 * 32x32 blocks of the regions its fill plan did NOT fill (the filled ones hold
 * only misses): 1024 floats per packed region.
 *
 * xrt_plan_region_map: map[r] for the n_regions = ceil(width/32) x
 * ceil(rows/32) regions of the strip (row-major) -- the packed index of
 * region r, or 0xFFFFFFFF for a region the last enqueued frame filled;
 * *n_packed = packed regions.  Without a plan in that frame every region is
 * packed (map[r] = r).  The map belongs to the strip's geometry: a receiver
 * needs the sender's map once, not per frame.
 * xrt_pack_regions_device: d_lbuffer (the strip, rows x width) -> d_packed
 * (n_packed x 1024 floats, 16-B aligned) on `stream`.
 * xrt_unpack_regions_device: d_packed -> the strip's three planes (any may be
 * NULL), with xrt_expand_rows_device's values.
 */
int xrt_plan_region_map(xrt_context* ctx, uint32_t width, uint32_t rows, uint32_t* map, uint64_t n_regions,
                        uint32_t* n_packed);
int xrt_pack_regions_device(xrt_context* ctx, uint32_t width, uint32_t rows, const uint32_t* d_map,
                            const float* d_lbuffer, float* d_packed, void* stream);
int xrt_unpack_regions_device(xrt_context* ctx, uint32_t width, uint32_t rows, const uint32_t* d_map,
                              const float* d_packed, float* d_lbuffer, float* d_image, uint8_t* d_u8, void* stream);
/*
 * Renders of this context write the L-buffer in the packed layout directly
 * (no xrt_pack_regions_device pass): region r of the strip to block map[r] of
 * d_lbuffer, nothing for the regions the fill plan fills.  For BINNED
 * attenuation renders of the L-buffer only (image and u8 NULL), typically with
 * XRT_MISS_TRANSIT; `packed_floats` is the L-buffer's capacity in floats.  A
 * frame whose fill plan does not hold (or does not fit) is not rendered and
 * returns XRT_ERR_OVERFLOW.  0 restores the row-major layout.
 */
int xrt_set_transit_layout(xrt_context* ctx, uint64_t packed_floats);

/*
 * Many strips' packed regions in one launch: d_desc holds 4 u32 per block --
 * first frame row, rows of the block inside its strip (<= 32), first column,
 * packed block index in d_packed (0xFFFFFFFF: a filled region, all misses).
 * The planes are whole frames (row-major, `width` columns).  16-B aligned.
 */
int xrt_unpack_blocks_device(xrt_context* ctx, uint32_t width, uint64_t n_blocks, const uint32_t* d_desc,
                             const float* d_packed, float* d_lbuffer, float* d_image, uint8_t* d_u8, void* stream);

/* --- hit transit (multi-GPU gathers) ------------------------------------- */

/*
 * Hit-only strips: a strip's message holds, per tile of its fill plan (8x8
 * pixels; tile t of tile slot s is tile i = 16 s + t), a 64-bit mask of the
 * tile's rays that hit mesh 0 (bit 8 y + x for pixel (x, y) of the tile) at
 * 32-bit words [2i, 2i + 2), then the hit rays' L values -- tile by tile, in
 * bit order -- from word 2 n_tiles.  A miss is an unset bit (its L is +inf,
 * image 80, u8 255); the filled regions send nothing.  The per-tile hit counts
 * are a function of the strip's geometry, like the fill plan.
 *
 * xrt_plan_hit_layout: the hit plan of the last frame's geometry, from that
 * frame's records (it must be a BINNED render of that geometry over its fill
 * plan: typically the geometry's first frame, row-major).  *n_tiles = 16 x
 * the plan's tile slots, *words = the message's words (2 n_tiles + hits);
 * tile_hits (nullable, `capacity` entries) receives each tile's hit count.
 * Synchronous.  The tiles' order is xrt_plan_region_map's: tile slot s is
 * packed region s.
 * xrt_set_transit_hits: renders of this context write the hit layout into
 * d_lbuffer (capacity_words >= *words + 64), instead of the packed
 * (xrt_set_transit_layout) or row-major layout; 0 turns it off.  For BINNED
 * attenuation renders of the L-buffer only; a frame of another geometry than
 * the plan's, or whose fill plan does not hold, is not rendered and returns
 * XRT_ERR_OVERFLOW.
 * xrt_unpack_hits_device: many strips' messages in one launch on the receiver
 * -- d_desc as xrt_unpack_blocks_device's, its last word the index in d_tdesc
 * of the region's first tile descriptor (or 0xFFFFFFFF: a filled region);
 * d_tdesc holds 4 u32 per tile: the word of its mask in d_msg, the word of its
 * first hit value, its planned hit count, 0.  A mask whose count is not the
 * planned one sets *d_bad (nullable) to 1.  d_desc, d_tdesc 16-B aligned;
 * d_msg 8-B aligned.
 */
int xrt_plan_hit_layout(xrt_context* ctx, uint32_t* tile_hits, uint64_t capacity, uint64_t* n_tiles,
                        uint64_t* words);
int xrt_set_transit_hits(xrt_context* ctx, uint64_t capacity_words);
int xrt_unpack_hits_device(xrt_context* ctx, uint32_t width, uint64_t n_blocks, const uint32_t* d_desc,
                           const uint32_t* d_tdesc, const uint32_t* d_msg, float* d_lbuffer, float* d_image,
                           uint8_t* d_u8, uint32_t* d_bad, void* stream);

/*
 * Test hooks, device probes and diagnostics: include/xrt_debug.h (not part of
 * the drop-in surface).
 */

#ifdef __cplusplus
}
#endif

#endif /* XRT_H */
