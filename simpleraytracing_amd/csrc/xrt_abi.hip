// xrt_abi.hip -- the C ABI of include/xrt.h: device/context management,
// launches and the host-side camera arithmetic.  Built into libxrt.so by
// simpleraytracing_amd/csrc/Makefile (hipcc --offload-arch=gfx950).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "xrt_debug.h"
#include "kernels/xrt_kernels.h"

using namespace XRT_KERNEL_NS;

// Region lists: the first frame of a geometry (xrt_context::BinKey) bins into
// lists of kInitialRegionCap entries per region, reads every region's count
// back once, and re-bins into compact lists sized from them (the counts of
// every later frame of the geometry are the same): the sum of the counts plus
// 1/8 + 4 per region, instead of the largest count times the regions.
constexpr uint32_t kInitialRegionCap = 256;
// Timed regions (xrt_timing_begin/end) keep the timing records of every
// frame (Outputs::wave_times: each wave's s_memrealtime start and end), up to
// kTimingRecords of them (8 B each) per region, and put a HIP start/stop event
// pair on the render dispatch of every kEventStride-th frame, a cross-check of
// the in-kernel spans (a start event costs the frame a few microseconds).
// xrt_timing_begin allocates the region's record space (one chunk: room for
// kTimingFrames frames of the context's last frame size, at most
// kTimingRecords = 1 GB, 128 frames of 8192^2) and its events up front: an allocation inside the region
// stalls the host for long enough that the GPU idles, and an idle GPU drops
// its clocks and takes ~30 ms of load to ramp them back (DESIGN.md
// "Measurement").  Frames past the record space are not sampled.
constexpr size_t kTimingRecords = (size_t)1 << 27;
constexpr size_t kTimingFrames = 256;
// After a timed region a context keeps one chunk of at most this many bytes
// for the next region; larger ones are freed (xrt_timing_end).
constexpr size_t kKeptTimingBytes = (size_t)64 << 20;
constexpr uint64_t kEventStride = 16;
constexpr size_t kTimingEvents = 256;          // start/stop pairs created by xrt_timing_begin
// s_memrealtime ticks per millisecond (100 MHz on gfx950)
constexpr double kTicksPerMs = 1e5;
// Buffer sets in rotation: frame N's preparation reuses the set of frame
// N - kFrameSets, whose render the host has seen complete by then.
#ifndef XRT_FRAME_SETS
#define XRT_FRAME_SETS 4
#endif
constexpr int kFrameSets = XRT_FRAME_SETS;
#ifndef XRT_DEV_SIZE_ON_PREP
// Where a device-sized frame's k_size_lists / k_scatter_pairs run: 0 on the
// render's stream (behind that stream's previous render), 1 on the prep stream
// (behind the count pass: the prep chain grows), 2 on the device's host stream
// after the count pass's event (idle in a device-pointer pipeline; no extra
// queue): 2048^2 moving frames 47.0 / 57.5 / 41.1 us (profiles/r06ac, r06ae).
#define XRT_DEV_SIZE_ON_PREP 2
#endif
// LDS a k_prep workgroup holds (its own + dynamic padding): the CU's LDS left
// beside a render at full occupancy (XRT_RENDER_WAVES waves per SIMD, each
// with its record stage), split over kPrepPerCu workgroups, so no more of
// them share a CU with the render (round 3: three beside the render, 1.12
// M-triangle frame 1,224 -> 1,143 us, 4096^2 -1.5 %, 2048^2 equal; one or two
// per CU starve the preparation, DESIGN.md "Pipelining").  LDS is allocated
// in 512-B granules.
#ifndef XRT_PREP_PER_CU
#define XRT_PREP_PER_CU 3
#endif
constexpr size_t kLdsPerCu = 160 * 1024;
constexpr size_t kLdsGranule = 512;
constexpr size_t kRenderLdsPerCu = (size_t)XRT_RENDER_WAVES * 4 * kRenderLdsPerWave;
static_assert(kRenderLdsPerCu < kLdsPerCu, "the render's stages fit a CU at full occupancy");
constexpr size_t kPrepLds = (kLdsPerCu - kRenderLdsPerCu) / XRT_PREP_PER_CU / kLdsGranule * kLdsGranule;
// Split tiles (DESIGN.md "Split tiles"): in a frame whose tile waves are at
// most kSplitFillFactor x the GPU's wave slots (its span is its heaviest tiles'),
// the regions with at least kSplitHeavyFrac of the heaviest region's candidates
// (and at least kSplitFloor) render each tile with two waves.  Larger frames
// split nothing (their heavy regions start first and others cover the tail).
// XRT_SPLIT_MIN=n instead splits every region of at least n candidates in any
// frame (0: never).
constexpr double kSplitFillFactor = 2.0;
constexpr double kSplitHeavyFrac = 0.6;
constexpr uint32_t kSplitFloor = 64;
constexpr uint32_t kSplitAuto = 0xFFFFFFFFu;
// A camera that stays put this many frames over lists sized for another
// camera is sized for itself.
constexpr uint32_t kStillFrames = 2;
// Frames prepared ahead of their call when a device-pointer render repeats
// its geometry (xrt_context::ahead); with kFrameSets sets, two renders can be
// in flight beside them.
#ifndef XRT_AHEAD_FRAMES
#define XRT_AHEAD_FRAMES 2
#endif
constexpr size_t kAheadFrames = XRT_AHEAD_FRAMES;
static_assert(kAheadFrames + 2 <= (size_t)kFrameSets, "sets for the renders in flight and the frames ahead");


// Everything one frame's preparation writes and its render reads or writes.
// kFrameSets sets rotate, so frame N+1's preparation (k_prep, binning) runs on
// the context's prep stream while frame N renders on the caller's stream.
// Ordering is kept by the host, not by cross-queue waits on the device
// (each costs the render queue several microseconds per frame, DESIGN.md
// "Pipelining"): the host waits for the preparation's completion event before
// it launches the render, and for the completion event of the render that
// last used the set before it prepares into the set again.
constexpr uint32_t kDirtyAll = 0xFFFFFFFFu;
constexpr int kHostCallFields = 16;    // xrt_debug_host_call_ms
constexpr int kAccFields = 8;          // running sums behind host_call_ms[8..15]
// D2H of the host-buffer entry points (xrt_render_rows, ...): the planes are
// DMAed in pieces of at most kStageChunk into a pinned staging ring of
// kStageSlots pieces (allocated with the context), and the context's copy
// threads move each piece into the caller's pages while the DMA of the next
// pieces runs.  A pageable hipMemcpy stages through one thread at 12.7 GB/s
// into fresh pages (tools/probes/d2h_probe.hip); the DMA into pinned memory
// runs at ~54 GB/s and the page faults of fresh caller pages are taken by
// several threads at once.  Pieces end at 2-MB boundaries of the caller's
// buffer (a transparent huge page is faulted in by one thread: 512-KB parts of
// one page on several threads measured 3.7-4.9 ms for 37.7 MB of fresh pages
// against 1.5-1.8 ms).  XRT_D2H_THREADS overrides the thread count (0:
// pageable hipMemcpy).
constexpr size_t kStageChunk = (size_t)2 << 20;
constexpr size_t kStageSlots = 16;
constexpr int kD2HThreads = 8;
// Pinned scratch of the list sizing (the count read-back) and of the launch
// layouts' uploads, allocated with the context and grown on demand: pageable
// copies there stage or pin the caller-side memory inside the HIP call, and a
// fresh context's first sizing right after a long frame loop once waited
// 10-22 ms in them (DESIGN.md "Measurement").
constexpr size_t kSizingScratch = (size_t)1 << 20;

struct FrameSet {
    TriRec* recs = nullptr;        // per-render records
    size_t recs_cap = 0;
    float4* cull = nullptr;        // per-render cull planes (4 x T float4)
    size_t cull_cap = 0;
    RenderParams* frame = nullptr;       // the frame's parameters (k_prep writes, make_ray reads)
    float* offsets = nullptr;            // the frame's pixel offsets, rows then columns (k_prep)
    size_t offsets_cap = 0;
    BlockStats* block_stats = nullptr;   // the render's per-workgroup / per-wave records
    size_t block_stats_cap = 0;
    uint2* times = nullptr;              // their timing records (Outputs::wave_times), frames not sampled
    size_t times_cap = 0;
    // where the set's last render stored its timing records: `times`, or a
    // timed region's chunk (copied back into `times` by xrt_timing_end)
    const uint2* last_times = nullptr;
    uint32_t rendered_blocks = 0;        // records of the set's last render (n_blocks of its frame)
    uint32_t n_blocks = 0;         // records of the set's last render
    bool binned = false;           // the set's last frame was binned (BinState valid)

    // binning (XRT_KERNEL_BINNED)
    // Two halves (parities), each [BinState line | line-padded region counts].
    // A frame counts into one half while its k_prep clears the other, which
    // the set's previous frame used (its render is complete: the host waited
    // for it before reusing the set) -- no memset on the per-frame path.
    uint32_t* bin_counts = nullptr;
    size_t bin_counts_cap = 0;         // words, both halves
    size_t bin_half_words = 0;         // words per half
    uint32_t half = 0;                 // half of the set's last frame
    // Per half: the counters past dirty[h] are zero, and so is its BinState
    // when dirty[h] == 0; kDirtyAll = unknown (fresh allocation).
    uint32_t dirty[2] = {kDirtyAll, kDirtyAll};
    BinState* last_state = nullptr;    // BinState of the set's last binned frame
    RegionEntry* bin_list = nullptr;   // regions x capacity footprint entries
    size_t bin_list_cap = 0;
    RegionEntry* global_list = nullptr;
    size_t global_list_cap = 0;

    // Completion events ride on the kernel dispatches themselves
    // (hipExtLaunchKernel stop events): no separate event packets.
    SlotDesc* dyn_desc = nullptr;      // a device-sized frame's launch layout (k_size_lists)
    size_t dyn_desc_cap = 0;
    uint4* pairs = nullptr;            // its (slot, index, triangle) pairs (k_prep's count pass)
    size_t pairs_cap = 0;
    SlotDesc* plan_desc = nullptr;     // its render layout under the device fill plan (tiles first, then fills)
    size_t plan_desc_cap = 0;
    uint32_t* plan_counts = nullptr;   // and its counter lines in that order
    size_t plan_counts_cap = 0;
    bool lazy_flags = false;           // plan_flag armed for a frame launched without reading it
    hipEvent_t ready = nullptr;        // k_prep complete (prep stream)
    hipEvent_t done = nullptr;         // render end (a stop event on the render's dispatch)
    hipEvent_t done_ev = nullptr;      // the event that marks the set's last render complete
    bool done_valid = false;
    // k_prep's flags (BinBuffers::plan_miss): [0] the fill plan did not hold,
    // [1] a list overflowed.  Host-mapped, cleared by the host before k_prep,
    // read after the host has waited for k_prep's completion.
    volatile uint32_t* plan_flag = nullptr;
};

using HostClock = std::chrono::steady_clock;

// A fixed set of host threads that run the pieces of one job at a time
// (start: tasks 0 .. count-1 claimed in order; wait: until every piece ran).
class CopyPool {
public:
    explicit CopyPool(int n)
    {
        for (int i = 0; i < n; ++i) threads_.emplace_back([this] { loop(); });
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    int size() const { return (int)threads_.size(); }
    void start(size_t count, std::function<void(size_t)> task)
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            task_ = std::move(task);
            count_ = count;
            next_.store(0);
            active_ = threads_.size();
            ++gen_;
        }
        cv_.notify_all();
    }
    void wait()
    {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return active_ == 0; });
    }

private:
    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const size_t count = count_;
            lk.unlock();
            for (size_t i; (i = next_.fetch_add(1)) < count;) task_(i);
            lk.lock();
            if (--active_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::function<void(size_t)> task_;
    size_t count_ = 0, active_ = 0;
    std::atomic<size_t> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// A launch layout of a region grid: launch slot -> region and list
// (SlotDesc, device), region -> slot (k_prep's binning), and the host copy of
// slot -> region (row-major over the strip).
struct SlotLayout {
    SlotDesc* d_desc = nullptr;
    size_t desc_cap = 0;
    uint32_t* d_rank = nullptr;
    size_t rank_cap = 0;
    std::vector<uint32_t> slot_region;
    uint32_t rx = 0, ry = 0, cap = 0;  // the fixed-capacity layout's key
};

// A frame between its preparation (enqueued) and its render launch.  Split so
// that a multi-device render can enqueue every device's preparation before it
// waits for any (xrt_render_rows_multi).
struct PendingFrame {
    FrameSet* fs = nullptr;
    // the frame renders the current geometry (bin_key) over its compact
    // layout and fill plan: its records can give the tile plan
    bool plan_source = false;
    bool hit_plan_ok = false;          // hit layout: the context's hit plan is this frame's geometry's
    hipStream_t stream = nullptr;
    hipEvent_t prep_done = nullptr;    // k_prep complete (prep stream)
    // The host waits for prep_done and reads k_prep's check before the launch
    // (a sizing frame, a frame with the check armed); otherwise the render's
    // queue waits for prep_done on the device and the host runs ahead.
    bool host_wait = false;
    bool ahead = false;                // prepared ahead of its call (xrt_context::ahead)
    int kernel = XRT_KERNEL_AUTO;
    bool binned = false;
    uint32_t rows = 0, rx = 0, ry = 0;
    dim3 grid;
    RenderParams p;
    Outputs out;
    BinBuffers bins = {};
    BinState* bin_ctl = nullptr;
    // A device-sized frame (a moving camera): k_size_lists and k_scatter_pairs
    // run on the render's stream ahead of the render (the prep stream holds
    // only the count passes, so the next frame's k_prep is not queued behind them).
    struct DevSize {
        bool on = false;
        uint32_t n_slots = 0, pool = 0;
        const SlotDesc* fixed = nullptr;
        uint32_t* flag = nullptr;
        uint32_t* counts = nullptr;        // the count pass's counter lines (the base layout's order)
        SlotDesc* plan_desc = nullptr;     // the device fill plan's layout (null: none)
        uint32_t* plan_counts = nullptr;
    } dev_size;
    HostClock::time_point t_call;
};

struct xrt_context {
    int device = 0;
    std::string error;

    float* d_tris = nullptr;       // raw triangle soup, 9 f32 per triangle
    uint64_t num_tris = 0;
    size_t tris_cap = 0;

    FrameSet sets[kFrameSets];
    int next_set = 0;
    FrameSet* last_set = nullptr;      // set of the last enqueued frame
    hipStream_t prep_stream = nullptr;    // the device's, shared with its other contexts (acquire_streams)
    bool owns_streams = false;         // holds a reference to them
    size_t prep_lds = 0;               // dynamic LDS of a k_prep launch (kPrepLds in all)

    // Launch layouts of the region grid (SlotLayout): the fixed-capacity one
    // the first frame of a geometry bins into (centre-first order), and the
    // compact one sized from its counts (the fill plan's order when there is
    // a plan).
    SlotLayout fixed;
    SlotLayout compact_layout;
    uint64_t slot_pool = 0;            // entries of the compact lists
    uint64_t motion_pool = 0;          // entries of a device-sized (moving camera) frame's lists
    uint64_t motion_pool_forced = 0;   // test hook XRT_MOTION_POOL: that many entries, never grown
    bool device_fill = true;           // moving frames render over the device fill plan (XRT_DEVICE_FILL=0: off)
    bool device_first = true;          // a geometry's first frame sized on the device (XRT_DEVICE_FIRST=0: off)
    bool dev_geometry = false;         // bin_key's only frame was sized on the device (no compact lists)
    // Box tile masks (BinBuffers::box_masks; XRT_BOX_MASKS): 0 (default)
    // never, 1 in the host-sized frames of meshes under kPrepBigMesh
    // triangles, 2 in every binned frame.  Exact either way; measured a wash
    // (DESIGN.md "Box tile masks"): the renders' dispatches shrink, k_prep's
    // grow by about as much, and the step does not move beyond box-to-box noise.
    int box_masks = 0;
    bool compact = false;              // compact_layout is valid for bin_key
    size_t bin_force_cap = 0;          // test hook (xrt_set_bin_capacity)
    // Fill plan of the current geometry (bin_key): the compact layout's
    // slots [plan_tile_slots, regions) are the regions its sizing frame
    // counted empty, one workgroup each (DESIGN.md "Fill plan").  fill_plan:
    // 1 on (xrt_set_fill_plan 0 turns it off); 2 plans EVERY region as empty
    // (tests of the exact fallback).
    int fill_plan = 1;
    uint32_t plan_tile_slots = 0;
    // the plan's heaviest regions render each tile with two waves (BinBuffers::
    // split_slots): the leading tile slots whose candidate count is at least
    // split_min (XRT_SPLIT_MIN; 0 = never)
    uint32_t plan_split_slots = 0;
    uint32_t split_min = kSplitAuto;   // kSplitAuto: the rule above
    uint32_t wave_slots = 0;           // the device's CUs x 32 (render waves resident at full occupancy)
    bool plan_valid = false;
    // Tile plan (SlotDesc::live): 0 = the compact layout's tiles all live (as
    // uploaded), 1 = k_tile_plan ran after a render of the current geometry
    // (bin_key) with its fill plan.  Off by default: it reuses an earlier
    // frame's cull results, so it helps only a loop of identical frames
    // (XRT_TILE_PLAN=1 or xrt_debug_set_tile_plan turn it on).
    bool tile_plan_enabled = false;
    // xrt_debug_prep_times: k_prep's per-wave timestamps of the last launch
    bool prep_times_on = false;
    uint4* d_prep_times = nullptr;
    size_t prep_times_cap = 0, prep_times_n = 0;
    int tile_plan_state = 0;
    uint64_t hp_tile_plan_frames = 0, hp_tile_plans = 0;
    uint32_t last_fill_regions = 0;    // regions the last enqueued frame filled (diagnostics)
    uint64_t packed_cap = 0;           // xrt_set_transit_layout: the packed L-buffer's floats (0: row-major)

    // staging for the host-pointer entry point
    float* d_image = nullptr;
    float* d_lbuffer = nullptr;
    uint8_t* d_u8 = nullptr;
    size_t stage_cap = 0;
    // The host-buffer entry points run on this context-owned non-blocking
    // stream (never the null stream, whose legacy semantics order it against
    // every blocking stream of the device), and copy back through the pinned
    // ring h_stage (kStageSlots x kStageChunk) with the copy threads of `pool`.
    hipStream_t host_stream = nullptr;
    uint8_t* h_stage = nullptr;
    hipEvent_t stage_ev[kStageSlots] = {};
    uint8_t* h_sizing = nullptr;       // pinned scratch of the sizing path (kSizingScratch, grown on demand)
    size_t h_sizing_cap = 0;
    hipEvent_t sizing_ev = nullptr;    // the last upload from h_sizing (prep stream)
    bool sizing_busy = false;
    hipEvent_t host_render_done = nullptr;
    std::unique_ptr<CopyPool> pool;
    // the preparation stream holds work that reads a launch layout (k_prep)
    // since it was last synchronised (upload_layout needs it idle)
    bool prep_reads_layout = false;
    // XRT_SIZING_PROFILE=1: a new geometry's preparation step by step, each
    // step synchronised and timed on the host (stderr) -- diagnostics only
    int sizing_profile = 0;
    HostClock::time_point prof_t{};

    hipEvent_t ev_begin = nullptr, ev_end = nullptr;
    // xrt_read_stats: the last render's records summed on the device
    // (k_reduce_stats) into one record, read through pinned memory
    StatsSum* d_stats_partial = nullptr;   // [kReduceMaxBlocks]
    unsigned int* d_stats_done = nullptr;  // the last-block counter (reset by that block)
    StatsSum* d_stats_out = nullptr;
    StatsSum* h_stats = nullptr;           // pinned
    // host time of the last host-buffer call (xrt_render_rows), ms:
    // [0] device planes, [1] enqueue (preparation, sizing, launch), [2] wait for
    // the render, [3] D2H of the planes (DMA into the pinned ring overlapped with
    // the copy threads), [4] copy threads, [5] MB copied, [6] statistics,
    // [7] total; within them: [8] every hipMalloc of the call, [9] a new
    // geometry's list sizing (count read-back, layout upload), [10] the
    // synchronisations before a launch layout's upload -- [13] of them the prep
    // stream's, [14] the sets' render events', [15] the last stream's --,
    // [11] host waits for k_prep, [12] kernel launches (k_prep and render)
    double host_call_ms[kHostCallFields] = {};
    double acc_ms[kAccFields] = {};                  // running sums of [8..15]
    // region timing (xrt_timing_begin/end)
    bool timing = false;
    std::vector<hipEvent_t> tev;      // pairs: [2i] start, [2i+1] stop of a sampled render dispatch
    size_t tev_used = 0;
    uint64_t timed_frames = 0;        // frames enqueued since xrt_timing_begin
    size_t timed_records = 0;         // their timing records kept
    size_t timing_space = 0;          // records the region's chunk holds (xrt_timing_begin)
    // the sampled frames' timing records: chunks of device memory (a chunk is
    // never moved while kernels may write it), and where each frame's are
    struct TimesChunk {
        uint2* p;
        size_t cap, used;
    };
    std::vector<TimesChunk> tchunks;
    struct TimesSample {              // a frame's records: where they are (chunks never move) and how many
        const uint2* p;
        size_t n;
    };
    std::vector<TimesSample> tsamples;
    double event_ms = 0.0;            // the last timed region's HIP-event samples
    uint64_t event_launches = 0;
    hipStream_t last_stream = nullptr;
    bool pending = false;
    int kernel = XRT_KERNEL_AUTO;
    uint64_t mesh_gen = 0;             // bumped by every upload
    // Binned list sizing: the region lists are sized by a synchronous count
    // whenever the frame geometry changes (mesh, camera, strip); later frames
    // of the same geometry reuse the size without a host round trip.
    struct BinKey {
        xrt_camera cam;
        uint32_t row_begin, row_end;
        uint64_t T, gen;
        // field by field (the struct has padding; the camera's floats by bits)
        bool same(const BinKey& o) const
        {
            return std::memcmp(&cam, &o.cam, sizeof cam) == 0 && row_begin == o.row_begin &&
                   row_end == o.row_end && T == o.T && gen == o.gen;
        }
        // the same region grid and mesh: only the camera's pose differs
        bool same_layout(const BinKey& o) const
        {
            return cam.width == o.cam.width && cam.height == o.cam.height && row_begin == o.row_begin &&
                   row_end == o.row_end && T == o.T && gen == o.gen;
        }
    } bin_key = {};
    static_assert(sizeof(xrt_camera) == 15 * 4, "xrt_camera has no padding (compared bytewise)");
    bool bin_key_valid = false;
    // The last frame rendered over lists sized for another camera (DESIGN.md
    // "Moving camera"): a sizing then plans for motion (roomier lists, no
    // fill plan).
    bool moving = false;
    bool reuse_cameras = true;         // false for xrt_render_rows_multi's contexts
    BinKey last_key = {};              // the last frame's geometry
    // Hit transit (xrt_set_transit_hits): the message buffer's capacity in
    // 32-bit words (0: off), and the hit plan of geometry hit_key
    // (xrt_plan_hit_layout): per tile of its fill plan the exclusive scan of
    // the tiles' hit counts, n_tiles + 1 entries on the device.
    uint64_t hits_cap = 0;
    bool hit_valid = false;
    BinKey hit_key = {};
    uint32_t hit_tiles = 0;
    uint64_t hit_words = 0;
    uint32_t* d_hit_off = nullptr;
    size_t hit_off_cap = 0;
    uint32_t still_frames = 0;         // frames in a row on one camera over reused lists
    // Prepare-ahead (DESIGN.md "Pipelining"): when a device-pointer render
    // repeats the previous call's frame geometry, the preparations of the next
    // kAheadFrames frames of that geometry are enqueued at once on the prep
    // stream; a later call whose geometry and settings match takes the oldest
    // (its k_prep then ran beside earlier renders and is complete: the render
    // is launched with no wait at all).  Any mismatch drops them (their k_prep
    // runs, on the prep stream, before any newer one).  state_gen counts the
    // setting changes a prepared frame depends on.
    struct AheadFrame {
        PendingFrame pf;
        BinKey key;
        uint64_t state_gen;
        uint32_t outs;                 // which output planes (image 1, L-buffer 2, u8 4)
    };
    std::deque<AheadFrame> ahead;
    uint64_t state_gen = 0;
    BinKey call_key = {};              // the last device-pointer call's geometry
    uint64_t call_state_gen = ~0ull;
    uint64_t hp_ahead_used = 0, hp_ahead_dropped = 0, hp_launch_nowait = 0, hp_host_waits = 0;
    uint64_t hp_dev_first = 0, hp_dev_first_recounts = 0;   // first frames sized on the device; pools regrown
    uint64_t dev_first_pairs = 0, dev_first_pool = 0;       // the last one's pair total and first pool
    uint32_t miss_code = 0;            // L-buffer bits of a miss (0: +inf; xrt_set_miss_code)
    uint32_t model = kModelAttenuation;   // xrt_set_model
    float mu = 0.1037f;                // kModelSigned: mesh 0's attenuation coefficient
    xrt_camera cull_cam = {};          // camera of the cached cull parameters
    CullParams cull = {};
    bool cull_valid = false;
    int last_kernel = XRT_KERNEL_BINNED;
    uint32_t hit_capacity = kMaxHits;
    // XRT_HOST_PROFILE=1: host time per enqueue, split by wait (printed at destroy)
    bool host_profile = false;
    double hp_total = 0, hp_done = 0, hp_prep = 0, hp_lprep = 0, hp_lrender = 0, hp_gap = 0;
    uint64_t hp_calls = 0;
    uint64_t hp_sizings = 0, hp_reused = 0, hp_plan_miss = 0, hp_overflow = 0;   // frames by geometry path
    HostClock::time_point hp_last_end{};
};

inline double seconds_since(HostClock::time_point t)
{
    return std::chrono::duration<double>(HostClock::now() - t).count();
}

// XRT_SIZING_PROFILE: synchronise the prep stream and print the time since the
// last mark (the step's enqueue + execution).
void prof_mark(xrt_context* ctx, const char* what)
{
    if (!ctx->sizing_profile) return;
    const auto t_enq = HostClock::now();
    // XRT_SIZING_PROFILE=2: host time per step only, no synchronisation
    const hipError_t e = ctx->sizing_profile == 2 ? hipSuccess : hipStreamSynchronize(ctx->prep_stream);
    const auto now = HostClock::now();
    std::fprintf(stderr, "xrt sizing profile: %-34s %9.3f ms (of which sync %8.3f ms)%s\n", what,
                 std::chrono::duration<double, std::milli>(now - ctx->prof_t).count(),
                 std::chrono::duration<double, std::milli>(now - t_enq).count(), e == hipSuccess ? "" : " ERROR");
    ctx->prof_t = HostClock::now();
}

// No static object of libxrt has a destructor: process exit runs the shared
// libraries' finalizers (__cxa_finalize) in an order libxrt does not control,
// the HIP runtime's among them, and contexts a caller leaks (RayTracer.cpp's
// per-device slots) are reclaimed by the process's end, not torn down.  The
// error strings of a failed create are heap objects that are never freed.
static std::string& g_create_error = *new std::string();
// xrt_destroy's phases, ms (xrt_debug_destroy_ms): [0] waiting for the
// context's work, [1] device frees, [2] pinned host frees, [3] streams and events
static double g_destroy_ms[4] = {};

// The prep and host streams are shared by every context of one device in the
// process (reference-counted; the last context's destroy destroys them).  A
// process gets GPU_MAX_HW_QUEUES hardware queues (4 by default) and HIP shares
// one between streams past that: a second context with streams of its own
// beside a caller's two render streams put its prep stream on a render
// stream's queue, where a frame's k_prep waits for the render queued before it
// and the next render for that k_prep -- preparation and render serialised
// (2048^2: 32 -> 58 us a still frame, 51 -> 69 us a moving one; DESIGN.md
// "Moving camera").  Shared, contexts add no queue: their k_preps serialise on
// the device's prep stream, which they would on one queue anyway.
struct DeviceStreams {
    hipStream_t prep = nullptr, host = nullptr;
    int refs = 0;
};
static std::mutex& g_streams_mu = *new std::mutex();
static std::vector<DeviceStreams>& g_streams = *new std::vector<DeviceStreams>();

bool acquire_streams(int device, hipStream_t& prep, hipStream_t& host)
{
    std::lock_guard<std::mutex> lock(g_streams_mu);
    if ((size_t)device >= g_streams.size()) g_streams.resize((size_t)device + 1);
    DeviceStreams& d = g_streams[(size_t)device];
    if (d.refs == 0) {
        if (hipStreamCreateWithFlags(&d.prep, hipStreamNonBlocking) != hipSuccess) return false;
        if (hipStreamCreateWithFlags(&d.host, hipStreamNonBlocking) != hipSuccess) {
            (void)hipStreamDestroy(d.prep);
            d.prep = nullptr;
            return false;
        }
    }
    ++d.refs;
    prep = d.prep;
    host = d.host;
    return true;
}

void release_streams(int device)
{
    std::lock_guard<std::mutex> lock(g_streams_mu);
    DeviceStreams& d = g_streams[(size_t)device];
    if (--d.refs == 0) {
        (void)hipStreamDestroy(d.prep);
        (void)hipStreamDestroy(d.host);
        d.prep = d.host = nullptr;
    }
}

// AUTO switches from TILED to BINNED past this many footprint-box tests
// (T x regions) per frame (DESIGN.md "Kernels").
constexpr uint64_t kAutoSweep = 20000000ull;

namespace {

int fail(xrt_context* ctx, int code, const std::string& msg)
{
    if (ctx) ctx->error = msg;
    else g_create_error = msg;
    return code;
}

#define XRT_HIP(ctx, expr)                                                                    \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return fail((ctx), XRT_ERR_DEVICE,                                                \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                   \
    } while (0)

template <typename T>
int ensure(xrt_context* ctx, T*& ptr, size_t& cap, size_t need_elems)
{
    if (need_elems <= cap && ptr) return XRT_OK;
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
    size_t n = std::max<size_t>(need_elems, 1);
    const auto t = HostClock::now();
    XRT_HIP(ctx, hipMalloc(&ptr, n * sizeof(T)));
    if (ctx) ctx->acc_ms[0] += std::chrono::duration<double, std::milli>(HostClock::now() - t).count();
    cap = n;
    return XRT_OK;
}

// The pinned sizing scratch, at least `bytes`, once no upload from it is still
// in flight (its last upload's event, long complete as a rule).
int sizing_scratch(xrt_context* ctx, size_t bytes, uint8_t*& out)
{
    if (ctx->sizing_busy) {
        XRT_HIP(ctx, hipEventSynchronize(ctx->sizing_ev));
        ctx->sizing_busy = false;
    }
    if (ctx->h_sizing_cap < bytes) {
        if (ctx->h_sizing) (void)hipHostFree(ctx->h_sizing);
        ctx->h_sizing = nullptr;
        ctx->h_sizing_cap = 0;
        XRT_HIP(ctx, hipHostMalloc((void**)&ctx->h_sizing, bytes, hipHostMallocDefault));
        ctx->h_sizing_cap = bytes;
    }
    out = ctx->h_sizing;
    return XRT_OK;
}

// Waits for this context's own work: its preparations (prep stream), every
// render still marked in flight (the sets' completion events) and the last
// enqueue's stream (a statistics reduction behind the render).  Not the whole
// device: other contexts' and the caller's unrelated work are not this
// context's to wait for (a device-wide synchronise measured 21 ms once, in a
// process whose device was otherwise idle).
int sync_context(xrt_context* ctx)
{
    auto t = HostClock::now();
    auto lap = [&](int k) {
        const auto now = HostClock::now();
        ctx->acc_ms[k] += std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    };
    XRT_HIP(ctx, hipStreamSynchronize(ctx->prep_stream));
    ctx->prep_reads_layout = false;
    lap(5);
    for (FrameSet& fs : ctx->sets)
        if (fs.done_valid) XRT_HIP(ctx, hipEventSynchronize(fs.done_ev));
    lap(6);
    if (ctx->pending) XRT_HIP(ctx, hipStreamSynchronize(ctx->last_stream));
    lap(7);
    return XRT_OK;
}

// True when a render or preparation of this context may still read its launch
// layouts (upload_layout must not overwrite them under it).
bool layouts_in_use(const xrt_context* ctx)
{
    if (ctx->prep_reads_layout || ctx->pending) return true;
    for (const FrameSet& fs : ctx->sets)
        if (fs.done_valid) return true;
    return false;
}

// The reference's stdmin / stdmax semantics (std::min(a,b) = b<a ? b : a).
inline float stdmin(float a, float b) { return (b < a) ? b : a; }
inline float stdmax(float a, float b) { return (a < b) ? b : a; }

inline void cross3(const float a[3], const float b[3], float o[3])
{
    float x = a[1] * b[2] - a[2] * b[1];
    float y = a[2] * b[0] - a[0] * b[2];
    float z = a[0] * b[1] - a[1] * b[0];
    o[0] = x;
    o[1] = y;
    o[2] = z;
}

inline float length3(const float a[3]) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }

inline void normalise3(float a[3])
{
    float len = length3(a);
    a[0] /= len;
    a[1] /= len;
    a[2] /= len;
}

RenderParams make_params(const xrt_camera& c, uint32_t row_begin, uint32_t row_end, uint64_t T,
                         uint32_t capacity)
{
    RenderParams p;
    p.ox = c.origin[0]; p.oy = c.origin[1]; p.oz = c.origin[2];
    p.cx = c.detector[0]; p.cy = c.detector[1]; p.cz = c.detector[2];
    p.ux = c.up[0]; p.uy = c.up[1]; p.uz = c.up[2];
    p.rx = c.right[0]; p.ry = c.right[1]; p.rz = c.right[2];
    p.spacing = c.pixel_spacing;
    p.width = c.width;
    p.height = c.height;
    p.row_begin = row_begin;
    p.row_end = row_end;
    p.num_triangles = (uint32_t)T;
    p.hit_capacity = capacity;
    p.prep_tris = prep_tris_for(T);
    return p;
}

// Grid exponent shared by every float of magnitude >= m > 0 (their ulps are
// at least 2^(floor(log2 m) - 23); 2^-149 at worst).
inline int grid_floor(double m)
{
    if (!(m > 0.0) || !std::isfinite(m)) return -149;
    return std::max(std::ilogb(m) - 23, -149);
}

// The f32 pixel offset of make_ray (main.cxx:655-656).
inline float pixel_offset(float spacing, uint32_t i, uint32_t n)
{
    return (float)((double)spacing * ((0.5 + (double)i) - (double)n / 2.0));
}

// Smallest nonzero |X_k| over the image, X_k = ((detector_k + up_k v) +
// right_k u) - origin_k in f32 as make_ray forms it (main.cxx:659): exact over
// the rows (right_k == 0) or the columns (up_k == 0) it varies with.  When it
// varies with both, a grid bound: X_k is a rounded sum of multiples of the
// grids of its terms, every nonzero offset being >= spacing / 2.  0 when X_k
// is 0 at every pixel.
// Smallest nonzero |x(i)| over i < n of a monotone sequence (non-decreasing or
// non-increasing; NaN-free): the last element below 0 and the first above 0,
// found by bisection -- O(log n) instead of a scan.
template <typename F>
double min_nonzero_monotone(uint32_t n, F x)
{
    double best = std::numeric_limits<double>::infinity();
    if (n == 0) return best;
    const bool up = x(0) <= x(n - 1);
    // first index whose value is past 0 in the sequence's direction (n if none)
    auto first = [&](auto past) {
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (past(x(mid))) hi = mid; else lo = mid + 1;
        }
        return lo;
    };
    // up: the first x > 0, and the last x < 0 (one before the first x >= 0)
    const uint32_t i_pos = up ? first([](float v) { return v > 0.0f; }) : first([](float v) { return v <= 0.0f; });
    const uint32_t i_neg = up ? first([](float v) { return v >= 0.0f; }) : first([](float v) { return v < 0.0f; });
    if (up) {
        if (i_pos < n) best = std::min(best, (double)std::fabs(x(i_pos)));
        if (i_neg > 0) best = std::min(best, (double)std::fabs(x(i_neg - 1)));
    } else {                                           // positives first, then zeros, then negatives
        if (i_pos > 0) best = std::min(best, (double)std::fabs(x(i_pos - 1)));
        if (i_neg < n) best = std::min(best, (double)std::fabs(x(i_neg)));
    }
    return best;
}

double min_nonzero_x(const xrt_camera& c, int k, bool scan = false)
{
    const float cu = c.up[k], cr = c.right[k], cc = c.detector[k], co = c.origin[k];
    auto x_of = [&](float v, float u) { return ((cc + cu * v) + cr * u) - co; };
    const uint32_t kMaxScan = 1u << 20;
    double best = std::numeric_limits<double>::infinity();
    auto take = [&](float x) {
        if (x != 0.0f) best = std::min(best, (double)std::fabs(x));
    };
    // Along one axis x is monotone in the pixel index (pixel_offset and each
    // rounded f32 operation are monotone), so its smallest nonzero magnitude is
    // next to its sign change: a bisection per camera instead of a scan of
    // every row or column (xrt_debug_direction_grid compares the two).
    const bool finite = std::isfinite(cu) && std::isfinite(cr) && std::isfinite(cc) && std::isfinite(co) &&
                        std::isfinite(c.pixel_spacing);
    if (cr == 0.0f && c.height <= kMaxScan) {
        const float u0 = pixel_offset(c.pixel_spacing, 0, c.width);
        auto xr = [&](uint32_t row) { return x_of(pixel_offset(c.pixel_spacing, row, c.height), u0); };
        if (!scan && finite) best = min_nonzero_monotone(c.height, xr);
        else for (uint32_t row = 0; row < c.height; ++row) take(xr(row));
    } else if (cu == 0.0f && c.width <= kMaxScan) {
        const float v0 = pixel_offset(c.pixel_spacing, 0, c.height);
        auto xc = [&](uint32_t col) { return x_of(v0, pixel_offset(c.pixel_spacing, col, c.width)); };
        if (!scan && finite) best = min_nonzero_monotone(c.width, xc);
        else for (uint32_t col = 0; col < c.width; ++col) take(xc(col));
    } else {
        const double ps = std::fabs((double)c.pixel_spacing);
        const int goff = ps > 0.0 ? grid_floor(0.5 * ps * (1.0 - 0x1p-23)) : kNoGrid;
        int gx = std::min(grid_exp(cc), grid_exp(co));
        if (cu != 0.0f && goff != kNoGrid) gx = std::min(gx, std::max(grid_exp(cu) + goff, -149));
        if (cr != 0.0f && goff != kNoGrid) gx = std::min(gx, std::max(grid_exp(cr) + goff, -149));
        if (gx != kNoGrid) best = std::ldexp(1.0, gx);
    }
    return std::isfinite(best) ? best : 0.0;
}

// A grid 2^g such that every nonzero component of every ray direction of the
// image (make_ray: main.cxx:652-661 and Ray.inl:80-84) is a multiple of it:
// the two normalisations divide X_k by |X| <= dmax and by ~1, so a nonzero
// component is >= min|X_k| / (1.001 dmax), a float whose ulp is the grid.
int direction_grid(const xrt_camera& c, double dmax, bool scan = false)
{
    int g = kNoGrid;
    for (int k = 0; k < 3; ++k) {
        const double xmin = min_nonzero_x(c, k, scan);
        if (xmin > 0.0) g = std::min(g, grid_floor(xmin / (1.001 * dmax)));
    }
    return g;
}

// Bounds used by the cull derivation (DESIGN.md "Tile cull"): over every pixel
// of the image, |D| <= dmax and the terms summed into D are <= mag.
CullParams make_cull_params(const xrt_camera& c)
{
    double ps = std::fabs((double)c.pixel_spacing);
    double vmax = ps * ((double)c.height / 2.0 + 1.0);
    double umax = ps * ((double)c.width / 2.0 + 1.0);
    double d2 = 0.0, mag = 0.0;
    for (int k = 0; k < 3; ++k) {
        double cterm = std::fabs((double)c.detector[k] - (double)c.origin[k]);
        double spread = std::fabs((double)c.up[k]) * vmax + std::fabs((double)c.right[k]) * umax;
        d2 += (cterm + spread) * (cterm + spread);
        mag = std::max(mag, std::fabs((double)c.detector[k]) + spread + std::fabs((double)c.origin[k]));
    }
    CullParams cp;
    cp.dmax = std::sqrt(d2) * (1.0 + 1e-6);
    cp.mag = mag;
    cp.width = c.width;
    cp.height = c.height;
    cp.dir_grid = direction_grid(c, cp.dmax);
    cp.pad = 0;
    for (int k = 0; k < 3; ++k) {
        cp.cvec[k] = (double)c.detector[k] - (double)c.origin[k];
        cp.up[k] = c.up[k];
        cp.rt[k] = c.right[k];
    }
    cp.ps = c.pixel_spacing;
    cp.cv = cp.ps * (0.5 - cp.height / 2.0);
    cp.cu = cp.ps * (0.5 - cp.width / 2.0);
    return cp;
}

int check_camera(xrt_context* ctx, const xrt_camera* cam, uint32_t row_begin, uint32_t row_end)
{
    if (!cam) return fail(ctx, XRT_ERR_ARGUMENT, "camera is NULL");
    if (cam->width == 0 || cam->height == 0)
        return fail(ctx, XRT_ERR_ARGUMENT, "image size must be non-zero");
    if (row_begin > row_end || row_end > cam->height)
        return fail(ctx, XRT_ERR_ARGUMENT,
                    "row range [" + std::to_string(row_begin) + ", " + std::to_string(row_end) +
                        ") outside image height " + std::to_string(cam->height));
    if ((uint64_t)cam->width * cam->height > (1ull << 32) - 1)
        return fail(ctx, XRT_ERR_ARGUMENT, "image larger than 2^32-1 pixels");
    return XRT_OK;
}

// k_prep: one thread per triangle, and at least one per image row and column
// (the pixel-offset tables).
int launch_prep(xrt_context* ctx, FrameSet& fs, const RenderParams& p, const CullParams& cp, bool culled,
                const BinBuffers& bins, BinState* bin_ctl, hipStream_t stream, hipEvent_t done)
{
    const uint64_t T = ctx->num_tris;
    // p.prep_tris triangles per wave; every thread covers a pixel-offset entry / counter
    const uint64_t threads = std::max<uint64_t>((uint64_t)p.height + p.width, bins.clear ? bins.clear_regions : 0u);
    const uint64_t per_block = (uint64_t)kPrepWaves * p.prep_tris;
    const uint64_t blocks = std::max<uint64_t>((T + per_block - 1) / per_block,
                                               (threads + kPrepThreads - 1) / kPrepThreads);
    uint4* ptimes = nullptr;                       // xrt_debug_prep_times
    if (ctx->prep_times_on) {
        int rc = ensure(ctx, ctx->d_prep_times, ctx->prep_times_cap, 2 * (size_t)blocks * kPrepWaves);
        if (rc) return rc;
        ptimes = ctx->d_prep_times;
        ctx->prep_times_n = (size_t)blocks * kPrepWaves;
    }
    const auto t_launch = HostClock::now();
    hipExtLaunchKernelGGL(k_prep, dim3((unsigned)blocks), dim3(kPrepThreads),
                          ctx->prep_lds, stream, nullptr, done, 0u,
                          ctx->d_tris, (uint32_t)T, p, cp, fs.recs, culled ? fs.cull : nullptr, bins, bin_ctl,
                          fs.frame, fs.offsets, ptimes);
    XRT_HIP(ctx, hipGetLastError());
    if (bins.counts) ctx->prep_reads_layout = true;
    ctx->acc_ms[4] += std::chrono::duration<double, std::milli>(HostClock::now() - t_launch).count();
    if (ctx->host_profile) ctx->hp_lprep += seconds_since(t_launch);
    return XRT_OK;
}

// Region buffers of a binned frame.  The frame counts into one half of the
// set's counters (FrameSet::bin_counts); k_prep clears the other half.  A half
// is cleared here, on the prep stream, only when it is not known clean for
// this many regions (the first frames, a larger region grid, a re-run).  The
// caller sets the launch layout (bins.desc / bins.rank).
int bin_buffers(xrt_context* ctx, FrameSet& fs, uint32_t n_regions, uint64_t list_entries, BinBuffers& bins,
                BinState*& ctl, hipStream_t stream, bool& cleared, bool rerun = false)
{
    cleared = false;
    const uint64_t T = ctx->num_tris;
    static_assert(sizeof(BinState) <= kCounterStride * sizeof(uint32_t), "BinState fits its line");
    int rc;
    // per half: control block padded to a line, then one line-padded counter per region
    const size_t half_words = kCounterStride + (size_t)kCounterStride * n_regions;
    if (!fs.bin_counts || fs.bin_half_words < half_words) {
        if ((rc = ensure(ctx, fs.bin_counts, fs.bin_counts_cap, 2 * half_words))) return rc;
        fs.bin_half_words = half_words;
        fs.dirty[0] = fs.dirty[1] = kDirtyAll;
    }
    if ((rc = ensure(ctx, fs.bin_list, fs.bin_list_cap, (size_t)list_entries))) return rc;
    if ((rc = ensure(ctx, fs.global_list, fs.global_list_cap, T))) return rc;
    const uint32_t q = rerun ? fs.half : fs.half ^ 1u;     // a re-run recounts into the same half
    uint32_t* mine = fs.bin_counts + (size_t)q * fs.bin_half_words;
    uint32_t* other = fs.bin_counts + (size_t)(q ^ 1u) * fs.bin_half_words;
    if (rerun || fs.dirty[q] != 0u) {
        XRT_HIP(ctx, hipMemsetAsync(mine, 0, half_words * sizeof(uint32_t), stream));
        cleared = true;                                     // k_prep must not overtake it
    }
    fs.half = q;
    fs.dirty[q] = n_regions;                                // this frame counts into it
    // k_prep clears the other half: its control block and its dirty counters
    const uint32_t alloc_regions = (uint32_t)((fs.bin_half_words - kCounterStride) / kCounterStride);
    bins.clear = other + kCounterStride;
    bins.clear_regions = fs.dirty[q ^ 1u] == kDirtyAll ? alloc_regions : fs.dirty[q ^ 1u];
    fs.dirty[q ^ 1u] = 0u;
    ctl = reinterpret_cast<BinState*>(mine);
    fs.last_state = ctl;
    bins.counts = mine + kCounterStride;
    bins.list = fs.bin_list;
    bins.global_list = fs.global_list;
    return XRT_OK;
}

// The base launch order of a region grid: centre first (regions by the
// distance of their centre from the image centre), so the dense middle of a
// centred object does not start last and set the tail.
std::vector<uint32_t> centre_first_order(uint32_t rx, uint32_t ry)
{
    // by squared distance from the grid's centre, ties in region order: keys
    // (4 x the squared distance, exact in integers) beside the indices, sorted
    // once (a comparator recomputing the distances took 0.37 ms at 64 x 64)
    const size_t n = (size_t)rx * ry;
    std::vector<std::pair<uint64_t, uint32_t>> key(n);
    for (uint32_t y = 0; y < ry; ++y)
        for (uint32_t x = 0; x < rx; ++x) {
            const int64_t dx = 2 * (int64_t)x - ((int64_t)rx - 1), dy = 2 * (int64_t)y - ((int64_t)ry - 1);
            const size_t r = (size_t)y * rx + x;
            key[r] = {(uint64_t)(dx * dx + dy * dy), (uint32_t)r};
        }
    std::sort(key.begin(), key.end());
    std::vector<uint32_t> order(n);
    for (size_t k = 0; k < n; ++k) order[k] = key[k].second;
    return order;
}

// Uploads a launch layout: slot s renders region slot_region[s] from
// list[base[s] .. base[s] + cap[s]).  Frames in flight may read the previous
// one, so the device is synchronised first.
int upload_layout(xrt_context* ctx, SlotLayout& L, uint32_t rx, uint32_t ry, std::vector<uint32_t> slot_region,
                  const std::vector<uint32_t>& base, const std::vector<uint32_t>& cap)
{
    const size_t n = slot_region.size();
    std::vector<SlotDesc> desc(n);
    std::vector<uint32_t> rank(n);
    for (size_t s = 0; s < n; ++s) {
        const uint32_t r = slot_region[s];
        desc[s] = SlotDesc{base[s], cap[s], (r % rx) | ((r / rx) << 16), 0xFFFFu};   // every tile live
        rank[r] = (uint32_t)s;
    }
    // Frames in flight may read the old layout: wait for them, but only when
    // there are any (a fresh context's first frame waits for nothing).
    int rc;
    if (layouts_in_use(ctx)) {
        const auto t_sync = HostClock::now();
        if ((rc = sync_context(ctx))) return rc;
        ctx->acc_ms[2] += std::chrono::duration<double, std::milli>(HostClock::now() - t_sync).count();
    }
    if ((rc = ensure(ctx, L.d_desc, L.desc_cap, n))) return rc;
    if ((rc = ensure(ctx, L.d_rank, L.rank_cap, n))) return rc;
    // from the pinned scratch, on the prep stream, in order before the k_prep
    // that reads them
    uint8_t* h = nullptr;
    if ((rc = sizing_scratch(ctx, n * (sizeof(SlotDesc) + sizeof(uint32_t)), h))) return rc;
    std::memcpy(h, desc.data(), n * sizeof(SlotDesc));
    std::memcpy(h + n * sizeof(SlotDesc), rank.data(), n * sizeof(uint32_t));
    XRT_HIP(ctx, hipMemcpyAsync(L.d_desc, h, n * sizeof(SlotDesc), hipMemcpyHostToDevice, ctx->prep_stream));
    XRT_HIP(ctx, hipMemcpyAsync(L.d_rank, h + n * sizeof(SlotDesc), n * sizeof(uint32_t), hipMemcpyHostToDevice,
                                ctx->prep_stream));
    XRT_HIP(ctx, hipEventRecord(ctx->sizing_ev, ctx->prep_stream));
    ctx->sizing_busy = true;
    L.slot_region = std::move(slot_region);
    L.rx = rx;
    L.ry = ry;
    return XRT_OK;
}

// The fixed-capacity layout (centre-first order, `cap` entries per slot) of a
// region grid: the first frame of a geometry bins into it.
int fixed_layout(xrt_context* ctx, uint32_t rx, uint32_t ry, uint32_t cap, BinBuffers& bins)
{
    SlotLayout& L = ctx->fixed;
    if (L.rx != rx || L.ry != ry || L.cap != cap || !L.d_desc) {
        const size_t n = (size_t)rx * ry;
        std::vector<uint32_t> base(n), caps(n, cap);
        for (size_t s = 0; s < n; ++s) base[s] = (uint32_t)(s * cap);
        int rc = upload_layout(ctx, L, rx, ry, centre_first_order(rx, ry), base, caps);
        if (rc) return rc;
        L.cap = cap;
    }
    bins.desc = L.d_desc;
    bins.rank = L.d_rank;
    return XRT_OK;
}

// The current geometry's compact layout (its fill plan's order when there is
// a plan, DESIGN.md "Fill plan").  The signed model keeps the plan's order (the
// compact lists are sized by its slots) but renders every region as tiles.
void use_compact(xrt_context* ctx, uint32_t n_regions, BinBuffers& bins, bool fill)
{
    bins.desc = ctx->compact_layout.d_desc;
    bins.rank = ctx->compact_layout.d_rank;
    bins.tile_slots = fill && ctx->plan_valid ? ctx->plan_tile_slots : n_regions;
    bins.split_slots = fill && ctx->plan_valid && kCanSplit ? ctx->plan_split_slots : 0u;
}

// Arms the k_prep check of a frame whose region lists or fill plan k_prep's
// binning has not yet been seen to match: the first frame over a new plan
// (`validate`) and frames over lists sized for another camera (`reused`).
// The binning of a frame geometry (mesh, camera, strip) is deterministic --
// the same footprints join the same regions, only the order of a list's
// entries varies with the atomics -- so later frames of a validated geometry
// cannot miss it and are launched without the host reading the check
// (DESIGN.md "Pipelining").
void arm_plan_check(FrameSet& fs, uint32_t n_regions, BinBuffers& bins, bool reused, bool validate)
{
    bins.plan_miss = nullptr;
    if (fs.plan_flag && ((validate && bins.tile_slots < n_regions) || reused)) {
        fs.plan_flag[0] = 0u;
        fs.plan_flag[1] = 0u;
        bins.plan_miss = const_cast<uint32_t*>(fs.plan_flag);
    }
}

int prepare_frame(xrt_context* ctx, const xrt_camera* cam, uint32_t row_begin, uint32_t row_end,
                  float* d_image, float* d_lbuffer, uint8_t* d_u8, hipStream_t stream, PendingFrame& pf,
                  int set_index = -1)
{
    int rc = check_camera(ctx, cam, row_begin, row_end);
    if (rc) return rc;
    if (!ctx->d_tris && ctx->num_tris) return fail(ctx, XRT_ERR_NO_MESH, "no mesh uploaded");
    if (ctx->num_tris > 0xFFFFFFFFull) return fail(ctx, XRT_ERR_ARGUMENT, "too many triangles");
    XRT_HIP(ctx, hipSetDevice(ctx->device));

    const uint64_t T = ctx->num_tris;
    const uint32_t rows = row_end - row_begin;
    const uint32_t rx = (cam->width + kRegion - 1) / kRegion, ry = (rows + kRegion - 1) / kRegion;
    // AUTO: the per-region footprint sweep of TILED costs T x regions box
    // tests; past kAutoSweep of them binning once per frame is cheaper.
    const uint64_t sweep = T * (uint64_t)rx * ry;
    const bool signed_model = ctx->model == kModelSigned;
    int kernel = ctx->kernel != XRT_KERNEL_AUTO ? ctx->kernel
                 : signed_model || sweep > kAutoSweep ? XRT_KERNEL_BINNED
                                                      : XRT_KERNEL_TILED;
    if (signed_model) {
        if (kernel == XRT_KERNEL_TILED)
            return fail(ctx, XRT_ERR_ARGUMENT, "the signed model renders with the BRUTE or BINNED kernel");
        if (d_image || d_u8)
            return fail(ctx, XRT_ERR_ARGUMENT,
                        "the signed model writes the L-buffer only (the image is xrt_hole_fill's)");
    }
    // k_prep packs a footprint's region rectangle in 16-bit fields: grids past
    // 65535 regions a side render TILED (exact, slower) -- BRUTE for the signed model.
    const bool binned = kernel == XRT_KERNEL_BINNED && rows > 0 && T > 0 && rx <= 0xFFFFu && ry <= 0xFFFFu;
    if (signed_model && !binned) kernel = XRT_KERNEL_BRUTE;
    const bool culled = kernel != XRT_KERNEL_BRUTE;

    // This frame's buffer set.  The render that last used it (kFrameSets
    // frames ago) must be complete before the set is prepared again.
    FrameSet& fs = ctx->sets[set_index < 0 ? ctx->next_set : set_index];
    // The preparation runs on the context's prep stream, beside the previous
    // frame's render; the host waits for its completion before it launches
    // the render (DESIGN.md "Pipelining": no cross-queue event on the render
    // queue).  The fill plan needs the attenuation model (the signed render
    // fills nothing).
    hipStream_t ps = ctx->prep_stream;
    const bool fill_ok = !signed_model;
    const auto t_call = HostClock::now();
    if (fs.done_valid) {
        const auto t = HostClock::now();
        XRT_HIP(ctx, hipEventSynchronize(fs.done_ev));
        fs.done_valid = false;
        if (ctx->host_profile) ctx->hp_done += seconds_since(t);
    }
    if (fs.lazy_flags) {
        // the set's last frame was device-sized and launched without reading
        // k_prep's flags; its render is complete: a list past the pool there
        // (that region rendered from the whole mesh, exactly) grows the pool
        fs.lazy_flags = false;
        if (fs.plan_flag && fs.plan_flag[1] != 0u) {
            ++ctx->hp_overflow;
            ctx->motion_pool = std::min<uint64_t>(2 * ctx->motion_pool + 65536u, 0xFFFFFFFFull);
        }
    }
    if ((rc = ensure(ctx, fs.recs, fs.recs_cap, T))) return rc;
    if (culled && (rc = ensure(ctx, fs.cull, fs.cull_cap, (size_t)T * kCullPlanes))) return rc;
    if ((rc = ensure(ctx, fs.offsets, fs.offsets_cap, (size_t)cam->height + cam->width))) return rc;

    RenderParams p = make_params(*cam, row_begin, row_end, T, ctx->hit_capacity);
    p.model = ctx->model;
    if (!ctx->cull_valid || std::memcmp(&ctx->cull_cam, cam, sizeof *cam) != 0) {
        ctx->cull = make_cull_params(*cam);      // a scan over the rows / columns: once per camera
        ctx->cull_cam = *cam;
        ctx->cull_valid = true;
    }
    const CullParams cp = ctx->cull;
    Outputs out;
    out.image = d_image;
    out.lbuffer = d_lbuffer;
    out.image_u8 = d_u8;
    out.frame = (const __attribute__((address_space(4))) RenderParams*)fs.frame;
    out.off.v = fs.offsets;
    out.off.u = fs.offsets + cam->height;
    const uint32_t miss_bits = ctx->miss_code ? ctx->miss_code : 0x7F800000u;   // +inf
    std::memcpy(&out.miss_l, &miss_bits, sizeof miss_bits);
    out.mu = ctx->mu;
    out.packed = 0u;
    out.wave_times = nullptr;          // launch_frame
    out.hit_tiles = 0u;
    out.hit_off = nullptr;
    if (ctx->packed_cap || ctx->hits_cap) {        // xrt_set_transit_layout / _hits
        if (!binned || signed_model || d_image || d_u8)
            return fail(ctx, XRT_ERR_ARGUMENT,
                        "the transit layouts are for BINNED attenuation renders of the L-buffer only");
        out.packed = ctx->hits_cap ? kLayoutHits : kLayoutPacked;
        out.hit_tiles = ctx->hit_tiles;
        out.hit_off = ctx->d_hit_off;
    }
    const uint32_t n_regions = rows ? rx * ry : 0u;
    BinBuffers bins = {};
    BinState* bin_ctl = nullptr;
    xrt_context::BinKey key = {};                  // the frame geometry of the region lists
    key.cam = *cam;
    key.row_begin = row_begin;
    key.row_end = row_end;
    key.T = T;
    key.gen = ctx->mesh_gen;
    // A new camera over the same region grid (a projection sweep) reuses the
    // lists sized for an earlier camera instead of the synchronous sizing
    // (DESIGN.md "Moving camera"), without a fill plan: k_prep flags a region
    // count past its list's capacity, that region renders from the whole mesh
    // (exact) and the next frame re-sizes.  A camera that then stays put for
    // kStillFrames frames is sized for itself (tight lists and a fill plan).
    // Contexts of xrt_render_rows_multi size every camera (reuse_cameras).
    ctx->still_frames = key.same(ctx->last_key) ? ctx->still_frames + 1u : 0u;
    ctx->last_key = key;
    bool reuse = false;
    if (binned && rows > 0 && fill_ok && ctx->bin_key_valid && (ctx->compact || ctx->dev_geometry) &&
        !ctx->bin_force_cap && !ctx->packed_cap && !ctx->hits_cap) {
        if (ctx->reuse_cameras && !key.same(ctx->bin_key) && key.same_layout(ctx->bin_key) &&
            ctx->still_frames < kStillFrames) {
            reuse = true;
            ctx->moving = true;
            ++ctx->hp_reused;
        } else if (ctx->moving && ctx->still_frames >= kStillFrames) {
            ctx->moving = false;           // the camera stopped: sized for it below
            ctx->bin_key_valid = false;
        }
    }
    if (!key.same_layout(ctx->bin_key)) ctx->moving = false;
    // (a geometry whose only frame was sized on the device has no compact
    // lists: the same camera again is sized on the host)
    const bool new_geometry = binned && rows > 0 && !reuse &&
                              (!ctx->bin_key_valid || !key.same(ctx->bin_key) || ctx->dev_geometry);
    if (new_geometry) ctx->compact = false;
    const uint32_t fixed_cap = ctx->bin_force_cap ? (uint32_t)std::min<size_t>(kInitialRegionCap, ctx->bin_force_cap)
                                                  : kInitialRegionCap;
    // A frame geometry seen for the first time -- a context's first frame, the
    // reference's whole workload -- is sized on the device as a moving camera's
    // frame is (below; one 32-byte read-back for the pool, no host plan and no
    // second k_prep); the same geometry again is sized on the host (compact
    // lists, fill plan, heaviest regions first) for the frames that follow.
    // Host-buffer calls only (xrt_render_rows: the drop-in renderLoop's one
    // frame into an Image): device-pointer callers -- pipelines, and strips
    // whose transit plans (xrt_plan_region_map, xrt_plan_hit_layout) describe
    // the host-sized layout of the frame before -- keep the host sizing.
    const bool dev_first = new_geometry && !ctx->bin_force_cap && ctx->device_first && ctx->still_frames == 0u &&
                           fill_ok && !ctx->packed_cap && !ctx->hits_cap && ctx->reuse_cameras &&
                           stream == ctx->host_stream;
    const bool device_sized = reuse || dev_first;
    if (new_geometry) ctx->dev_geometry = false;
    if (dev_first) {                               // later cameras over its region grid take the moving path
        ctx->dev_geometry = true;
        ctx->bin_key = key;
        ctx->bin_key_valid = true;
    }
    // A new geometry's first k_prep only counts its pairs (no lists): the
    // compact lists are sized from the counts and k_prep runs again into them.
    const bool sizing = new_geometry && !ctx->bin_force_cap && !dev_first;
    if ((sizing || dev_first) && ctx->sizing_profile) {
        ctx->prof_t = t_call;
        prof_mark(ctx, "set wait + buffers");
    }
    if (binned) {
        bins.regions_x = rx;
        bins.regions_y = ry;
    }
    if (binned && !device_sized) {
        const bool compact = ctx->compact && !ctx->bin_force_cap;
        bool cleared = false;
        const uint64_t entries = compact ? ctx->slot_pool : sizing ? 0u : (uint64_t)n_regions * fixed_cap;
        if ((rc = bin_buffers(ctx, fs, n_regions, entries, bins, bin_ctl, ps, cleared))) return rc;
        if (sizing) prof_mark(ctx, "bin buffers (counter memset)");
        if (sizing) bins.list = nullptr;
        bins.tile_slots = n_regions;
        if (compact) use_compact(ctx, n_regions, bins, fill_ok && !reuse);
        else if ((rc = fixed_layout(ctx, rx, ry, fixed_cap, bins))) return rc;
        bins.tile_plan = compact && fill_ok && !reuse && !sizing && ctx->plan_valid && ctx->tile_plan_enabled &&
                         ctx->tile_plan_state == 1 ? 1u : 0u;
        bins.box_masks = ctx->box_masks == 2 || (ctx->box_masks == 1 && ctx->num_tris < kPrepBigMesh) ? 1u : 0u;
        if (sizing) prof_mark(ctx, "fixed layout upload");
        // the fill plan's test hook (every region planned empty) is checked every frame
        arm_plan_check(fs, n_regions, bins, false, ctx->fill_plan == 2);
    }

    hipEvent_t prep_done = fs.ready;
    if (device_sized) {
        // A moving camera (DESIGN.md "Moving camera"): its lists sized on the
        // device, no host round trip -- k_prep counts its pairs per slot of the
        // region grid's base layout (centre first), k_size_lists carves each
        // slot's list from the set's pool, k_prep bins into them.  Every region
        // renders as tiles (no fill plan: the host never sees the counts).
        // k_prep's flags are read when the set is next used (lazy_flags).
        // (a geometry's first frame: room for ~6 pairs a triangle, checked below)
        const uint64_t first_guess = dev_first ? 6u * (uint64_t)T + 2u * n_regions : 0u;
        ctx->motion_pool = ctx->motion_pool_forced
                               ? ctx->motion_pool_forced
                               : std::max<uint64_t>(std::max<uint64_t>(ctx->motion_pool, first_guess),
                                                    std::max<uint64_t>(2 * ctx->slot_pool, 65536u));
        bool cleared = false;
        if ((rc = bin_buffers(ctx, fs, n_regions, ctx->motion_pool, bins, bin_ctl, ps, cleared))) return rc;
        if (dev_first) prof_mark(ctx, "device first: bin buffers");
        if ((rc = fixed_layout(ctx, rx, ry, fixed_cap, bins))) return rc;
        if (dev_first) prof_mark(ctx, "device first: fixed layout");
        if ((rc = ensure(ctx, fs.dyn_desc, fs.dyn_desc_cap, n_regions))) return rc;
        if ((rc = ensure(ctx, fs.pairs, fs.pairs_cap, ctx->motion_pool))) return rc;
        // the device fill plan (not for the transit layouts, whose tiles follow a host plan)
        const bool dev_plan = ctx->device_fill && ctx->fill_plan != 0 && out.packed == 0u;
        if (dev_plan && ((rc = ensure(ctx, fs.plan_desc, fs.plan_desc_cap, n_regions)) ||
                         (rc = ensure(ctx, fs.plan_counts, fs.plan_counts_cap, (size_t)n_regions * kCounterStride))))
            return rc;
        uint32_t pool = (uint32_t)std::min<uint64_t>(ctx->motion_pool, 0xFFFFFFFFull);
        bins.tile_slots = n_regions;
        bins.split_slots = 0u;
        bins.tile_plan = 0u;
        bins.plan_miss = nullptr;
        bins.box_masks = ctx->box_masks == 2 ? 1u : 0u;
        RegionEntry* list = bins.list;
        bins.list = nullptr;                           // the count-only pass, appending its pairs
        bins.pairs = fs.pairs;
        bins.pairs_cap = pool;
        if ((rc = launch_prep(ctx, fs, p, cp, culled, bins, bin_ctl, ps, prep_done))) return rc;
        if (dev_first) prof_mark(ctx, "device first: count pass (buffers before it)");
        if (dev_first) {
            // A first frame has no earlier pose to size its pool from: the count
            // pass's pair total (32 bytes read back) checks it, and a pool too
            // small grows and counts again -- never the whole-mesh fallback.
            ++ctx->hp_dev_first;
            uint8_t* hs = nullptr;
            if ((rc = sizing_scratch(ctx, sizeof(BinState), hs))) return rc;
            XRT_HIP(ctx, hipMemcpyAsync(hs, bin_ctl, sizeof(BinState), hipMemcpyDeviceToHost, ps));
            XRT_HIP(ctx, hipStreamSynchronize(ps));
            BinState st;
            std::memcpy(&st, hs, sizeof st);
            prof_mark(ctx, "device first: pair total read back");
            ctx->dev_first_pairs = st.pairs;
            ctx->dev_first_pool = pool;
            if (st.pairs > pool && !ctx->motion_pool_forced) {
                ++ctx->hp_dev_first_recounts;
                ctx->motion_pool = std::min<uint64_t>((uint64_t)st.pairs + st.pairs / 4u + 65536u, 0xFFFFFFFFull);
                pool = (uint32_t)ctx->motion_pool;
                if ((rc = bin_buffers(ctx, fs, n_regions, ctx->motion_pool, bins, bin_ctl, ps, cleared, true)))
                    return rc;                     // (clears this frame's counters)
                if ((rc = fixed_layout(ctx, rx, ry, fixed_cap, bins))) return rc;
                if ((rc = ensure(ctx, fs.pairs, fs.pairs_cap, ctx->motion_pool))) return rc;
                list = bins.list;
                bins.list = nullptr;
                bins.pairs = fs.pairs;
                bins.pairs_cap = pool;
                if ((rc = launch_prep(ctx, fs, p, cp, culled, bins, bin_ctl, ps, prep_done))) return rc;
            }
        }
        uint32_t* const flag = fs.plan_flag ? const_cast<uint32_t*>(fs.plan_flag) : nullptr;
        if (flag) {                                    // [1]: a list past the pool, read lazily
            flag[0] = 0u;
            flag[1] = 0u;
            fs.lazy_flags = true;
        }
        // k_size_lists and k_scatter_pairs: launch_frame, on the render's stream
        pf.dev_size.on = true;
        pf.dev_size.n_slots = n_regions;
        pf.dev_size.pool = pool;
        pf.dev_size.fixed = bins.desc;
        pf.dev_size.flag = flag;
        pf.dev_size.counts = bins.counts;
        pf.dev_size.plan_desc = dev_plan ? fs.plan_desc : nullptr;
        pf.dev_size.plan_counts = dev_plan ? fs.plan_counts : nullptr;
        bins.list = list;
        bins.desc = dev_plan ? fs.plan_desc : fs.dyn_desc;
        if (dev_plan) {                                // the render reads the plan's order
            bins.counts = fs.plan_counts;
            bins.dev_plan = 1u;
        }
        bins.pairs = nullptr;
        bins.clear = nullptr;
#if XRT_DEV_SIZE_ON_PREP
        // k_size_lists and k_scatter_pairs behind the count pass on the prep
        // stream (on a render stream they queue behind that stream's previous
        // render), the preparation's event after them
        {
            // (2: on the device's host stream -- idle in a device-pointer
            // pipeline, no extra queue -- after the count pass's event)
            const hipStream_t ss = XRT_DEV_SIZE_ON_PREP == 2 ? ctx->host_stream : ps;
            if (ss != ps) XRT_HIP(ctx, hipStreamWaitEvent(ss, prep_done, 0));
            const PendingFrame::DevSize& d = pf.dev_size;
            hipLaunchKernelGGL(k_size_lists, dim3((d.n_slots + 255) / 256), dim3(256), 0, ss, d.counts, d.fixed,
                               fs.dyn_desc, d.n_slots, d.pool, bin_ctl, d.plan_desc, d.plan_counts);
            XRT_HIP(ctx, hipGetLastError());
            const uint32_t scatter_blocks = (uint32_t)std::min<uint64_t>((d.pool + 255u) / 256u, 2048u);
            hipLaunchKernelGGL(k_scatter_pairs, dim3(scatter_blocks), dim3(256), 0, ss, (const uint4*)fs.pairs,
                               (const BinState*)bin_ctl, d.pool, (const SlotDesc*)fs.dyn_desc,
                               (const float4*)fs.cull, (uint32_t)ctx->num_tris, bins.list, d.flag);
            XRT_HIP(ctx, hipGetLastError());
            XRT_HIP(ctx, hipEventRecord(prep_done, ss));
            pf.dev_size.on = false;
        }
#endif
    }
    if (rows > 0 && !device_sized && (rc = launch_prep(ctx, fs, p, cp, culled, bins, bin_ctl, ps, prep_done)))
        return rc;
    if (sizing) {
        // Size the compact region lists once per frame geometry (mesh, camera,
        // strip): a synchronous read of every region's count (the count-only
        // pass above), slot offsets from them, and a re-run of k_prep into the
        // compact lists.
        ++ctx->hp_sizings;
        prof_mark(ctx, "k_prep count pass");
        const auto t_sizing = HostClock::now();
        // every region's count (line-padded) and the BinState, into the pinned scratch
        const size_t cbytes = (size_t)n_regions * kCounterStride * sizeof(uint32_t);
        uint8_t* hs = nullptr;
        if ((rc = sizing_scratch(ctx, cbytes + sizeof(BinState), hs))) return rc;
        XRT_HIP(ctx, hipMemcpyAsync(hs, bins.counts, cbytes, hipMemcpyDeviceToHost, ps));
        prof_mark(ctx, "count read-back: counts enqueued");
        XRT_HIP(ctx, hipMemcpyAsync(hs + cbytes, bin_ctl, sizeof(BinState), hipMemcpyDeviceToHost, ps));
        prof_mark(ctx, "count read-back: state enqueued");
        XRT_HIP(ctx, hipStreamSynchronize(ps));
        prof_mark(ctx, "count read-back");
        const uint32_t* counts = reinterpret_cast<const uint32_t*>(hs);
        BinState st;
        std::memcpy(&st, hs + cbytes, sizeof st);
        const std::vector<uint32_t>& fixed_region = ctx->fixed.slot_region;   // the counts' slots
        std::vector<uint32_t> count_of(n_regions);     // by region
        for (uint32_t s = 0; s < n_regions; ++s) count_of[fixed_region[s]] = counts[(size_t)s * kCounterStride];
        // The fill plan (not for a moving camera, whose next pose would miss it):
        // the regions this frame counted empty (with an empty global list) go to
        // the end of the launch order, one workgroup each; the tile regions by
        // candidate count, heaviest first (their long tiles start first instead
        // of setting the tail: render 2048^2 -6 %, 1024^2 -10 %).
        std::vector<uint32_t> slot_region = fixed_region;
        uint32_t tile_slots = n_regions, split_slots = 0;
        const int plan = ctx->fill_plan;
        if (plan != 0 && st.global_count == 0u && !ctx->moving) {
            std::vector<uint32_t> full, empty;
            for (uint32_t r : fixed_region) (count_of[r] != 0u && plan != 2 ? full : empty).push_back(r);
            std::stable_sort(full.begin(), full.end(), [&](uint32_t a, uint32_t b) { return count_of[a] > count_of[b]; });
            tile_slots = (uint32_t)full.size();
            // the heaviest regions (the first slots): two waves per tile
            uint32_t split_min = ctx->split_min;
            if (split_min == kSplitAuto) {
                const bool small = (double)tile_slots * kWavesPerRegion <= kSplitFillFactor * ctx->wave_slots;
                const uint32_t heaviest = tile_slots ? count_of[full[0]] : 0u;
                split_min = small ? std::max<uint32_t>(kSplitFloor, (uint32_t)std::ceil(kSplitHeavyFrac * heaviest))
                                  : 0u;
            }
            while (split_min && split_slots < tile_slots && count_of[full[split_slots]] >= split_min)
                ++split_slots;
            full.insert(full.end(), empty.begin(), empty.end());
            slot_region.swap(full);
        }
        std::vector<uint32_t> base(n_regions), cap(n_regions);
        uint64_t run = 0;
        for (uint32_t s = 0; s < n_regions; ++s) {
            const uint64_t c = count_of[slot_region[s]];
            // a moving camera: room for the counts of the next poses (2c + 64)
            const uint64_t room = ctx->moving ? 2u * c + 64u : c + c / 8u + 4u;
            base[s] = (uint32_t)run;
            cap[s] = (uint32_t)std::min<uint64_t>(room, 0xFFFFFFFFull);
            run += room;
        }
        if (run > 0xFFFFFFFFull) return fail(ctx, XRT_ERR_OVERFLOW, "region lists exceed 2^32 entries");
        prof_mark(ctx, "plan (host)");
        if ((rc = upload_layout(ctx, ctx->compact_layout, rx, ry, std::move(slot_region), base, cap))) return rc;
        ctx->tile_plan_state = 0;                  // the new layout's tiles are all live
        prof_mark(ctx, "compact layout upload");
        ctx->acc_ms[1] += std::chrono::duration<double, std::milli>(HostClock::now() - t_sizing).count();
        ctx->plan_tile_slots = tile_slots;
        ctx->plan_split_slots = split_slots;
        ctx->plan_valid = tile_slots < n_regions;
        ctx->slot_pool = run;
        ctx->compact = true;
        ctx->bin_key = key;
        ctx->bin_key_valid = true;
        bool cleared = false;
        if ((rc = bin_buffers(ctx, fs, n_regions, run, bins, bin_ctl, ps, cleared, true))) return rc;   // clears
        bins.tile_slots = n_regions;
        use_compact(ctx, n_regions, bins, fill_ok);
        arm_plan_check(fs, n_regions, bins, false, true);
        prof_mark(ctx, "counter memset (re-run)");
        if ((rc = launch_prep(ctx, fs, p, cp, culled, bins, bin_ctl, ps, prep_done))) return rc;
        prof_mark(ctx, "k_prep into the compact lists");
    }
    // BINNED: one 8x8 tile per render wave, kTileWaves waves per workgroup, and
    // one workgroup per region of the fill plan
    const dim3 grid = kernel == XRT_KERNEL_BRUTE ? dim3((cam->width + 15) / 16, (rows + 15) / 16)
                    : binned ? dim3(kWavesPerRegion / kTileWaves * (bins.tile_slots + bins.split_slots) +
                                    (n_regions - bins.tile_slots))
                             : dim3(rx, ry);
    // stats records: one per workgroup; BINNED one per tile wave, 16 per fill region
    const uint32_t n_blocks = !rows ? 0u : binned ? kWavesPerRegion * n_regions : grid.x * grid.y;
    if ((rc = ensure(ctx, fs.block_stats, fs.block_stats_cap, n_blocks))) return rc;
    if ((rc = ensure(ctx, fs.times, fs.times_cap, n_blocks))) return rc;
    fs.n_blocks = n_blocks;
    fs.binned = binned;
    out.block_stats = fs.block_stats;
    pf.fs = &fs;
    pf.plan_source = binned && fill_ok && !reuse && ctx->compact && ctx->plan_valid && !ctx->bin_force_cap &&
                     bins.desc == ctx->compact_layout.d_desc && bins.tile_slots == ctx->plan_tile_slots;
    pf.hit_plan_ok = ctx->hit_valid && key.same(ctx->hit_key);
    pf.stream = stream;
    pf.prep_done = rows > 0 ? prep_done : nullptr;
    pf.host_wait = bins.plan_miss != nullptr && !device_sized;
    pf.kernel = kernel;
    pf.binned = binned;
    pf.rows = rows;
    pf.rx = rx;
    pf.ry = ry;
    pf.grid = grid;
    pf.p = p;
    pf.out = out;
    pf.bins = bins;
    pf.bin_ctl = bin_ctl;
    pf.t_call = t_call;
    return XRT_OK;
}

// Room for n timing records of a sampled frame in the timed region's chunks
// (a new chunk, never a moved one, when the last is full).
int timing_slot(xrt_context* ctx, size_t n, uint2*& slot)
{
    if (ctx->tchunks.empty() || ctx->tchunks.back().cap - ctx->tchunks.back().used < n) {
        size_t want = std::max<size_t>(n * 64, (size_t)1 << 16);
        // chunks of earlier regions are reused before new ones are allocated
        size_t k = 0;
        while (k < ctx->tchunks.size() && !(ctx->tchunks[k].used == 0 && ctx->tchunks[k].cap >= n)) ++k;
        if (k < ctx->tchunks.size() && k + 1 < ctx->tchunks.size()) {
            // an unused chunk to the end (the samples hold device pointers, not indices)
            std::swap(ctx->tchunks[k], ctx->tchunks.back());
        } else if (k == ctx->tchunks.size()) {
            xrt_context::TimesChunk c = {nullptr, want, 0};
            XRT_HIP(ctx, hipMalloc(&c.p, want * sizeof(uint2)));
            ctx->tchunks.push_back(c);
        }
    }
    xrt_context::TimesChunk& c = ctx->tchunks.back();
    ctx->tsamples.push_back({c.p + c.used, n});
    slot = c.p + c.used;
    c.used += n;
    return XRT_OK;
}

// A frame's kernel span from its waves' timing records: the last end minus
// the first start, in ms (32-bit tick differences: spans below 21 s).
double records_span_ms(const std::vector<uint2>& t)
{
    if (t.empty()) return 0.0;
    const uint32_t ref = t[0].x;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (const uint2& r : t) {
        lo = std::min<int64_t>(lo, (int32_t)(r.x - ref));
        hi = std::max<int64_t>(hi, (int32_t)(r.y - ref));
    }
    return hi > lo ? (double)(hi - lo) / kTicksPerMs : 0.0;
}

int launch_frame(xrt_context* ctx, PendingFrame& pf)
{
    FrameSet& fs = *pf.fs;
    hipStream_t stream = pf.stream;
    const int kernel = pf.kernel;
    const bool binned = pf.binned;
    const uint32_t rows = pf.rows, rx = pf.rx, ry = pf.ry;
    const RenderParams& p = pf.p;
    BinState* bin_ctl = pf.bin_ctl;
    const auto t_call = pf.t_call;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    // The render runs once its preparation is complete: the caller's queue
    // waits for it on the device (a barrier packet, ~2.4 us per frame), or --
    // when the host must read k_prep's check to choose the grid -- the host
    // waits for it before the launch.
    if (pf.prep_done && pf.host_wait) {
        const auto t = HostClock::now();
        XRT_HIP(ctx, hipEventSynchronize(pf.prep_done));
        ctx->acc_ms[3] += std::chrono::duration<double, std::milli>(HostClock::now() - t).count();
        ++ctx->hp_host_waits;
        if (ctx->host_profile) ctx->hp_prep += seconds_since(t);
    } else if (pf.prep_done) {
        // a preparation already complete needs no wait packet (a frame prepared
        // ahead usually is); hipErrorNotReady otherwise
        const hipError_t q = hipEventQuery(pf.prep_done);
        if (q == hipSuccess) ++ctx->hp_launch_nowait;
        else if (q == hipErrorNotReady) XRT_HIP(ctx, hipStreamWaitEvent(stream, pf.prep_done, 0));
        else XRT_HIP(ctx, q);
    }
    if (pf.dev_size.on) {                          // a device-sized frame's lists (prepare_frame)
        const PendingFrame::DevSize& d = pf.dev_size;
        hipLaunchKernelGGL(k_size_lists, dim3((d.n_slots + 255) / 256), dim3(256), 0, stream, d.counts, d.fixed,
                           fs.dyn_desc, d.n_slots, d.pool, bin_ctl, d.plan_desc, d.plan_counts);
        XRT_HIP(ctx, hipGetLastError());
        const uint32_t scatter_blocks = (uint32_t)std::min<uint64_t>((d.pool + 255u) / 256u, 2048u);
        hipLaunchKernelGGL(k_scatter_pairs, dim3(scatter_blocks), dim3(256), 0, stream, (const uint4*)fs.pairs,
                           (const BinState*)bin_ctl, d.pool, (const SlotDesc*)fs.dyn_desc, (const float4*)fs.cull,
                           (uint32_t)ctx->num_tris, pf.bins.list, d.flag);
        XRT_HIP(ctx, hipGetLastError());
    }
    dim3 grid = pf.grid;
    BinBuffers bins = pf.bins;
    bool missed = false;
    if (binned && bins.plan_miss && pf.host_wait && (fs.plan_flag[0] | fs.plan_flag[1]) != 0u) {
        missed = true;
        // k_prep binned a pair into a region the plan fills, into the global
        // list or past a list's capacity: this frame renders every region as
        // tiles (an overflowed region from the whole mesh -- exact, slower), and
        // the next frame re-sizes its lists.
        ++(fs.plan_flag[1] != 0u ? ctx->hp_overflow : ctx->hp_plan_miss);
        bins.tile_slots = rx * ry;
        bins.tile_plan = 0u;
        pf.plan_source = false;
        // an overflowed list renders its region from the whole mesh: as ordinary
        // tiles (split tiles only ever merge list-rendered halves)
        if (fs.plan_flag[1] != 0u) bins.split_slots = 0u;
        grid = dim3(kWavesPerRegion / kTileWaves * (bins.tile_slots + bins.split_slots));
        ctx->bin_key_valid = false;
    }
    ctx->last_fill_regions = binned ? rx * ry - bins.tile_slots : 0u;
    if (pf.out.packed == kLayoutPacked && rows > 0 &&
        (bins.tile_slots >= rx * ry || (uint64_t)bins.tile_slots * kPackBlock > ctx->packed_cap))
        return fail(ctx, XRT_ERR_OVERFLOW, "the packed layout needs this frame's fill plan (and room for its "
                                        "unfilled regions): the frame was not rendered");
    // the hit layout: the plan's tiles are exactly this frame's tile regions',
    // and the message has room for the plan's words plus one tile's hits (a
    // tile with more hits than its plan stays inside the buffer)
    if (pf.out.packed == kLayoutHits && rows > 0 &&
        (!pf.hit_plan_ok || missed || (uint64_t)bins.tile_slots * kWavesPerRegion != pf.out.hit_tiles ||
         ctx->hit_words + kWavesPerRegion * 4u > ctx->hits_cap))
        return fail(ctx, XRT_ERR_OVERFLOW, "the hit layout needs this geometry's hit plan (xrt_plan_hit_layout), "
                                        "its fill plan and room for its words: the frame was not rendered");

    // Every render dispatch carries the set's stop event (the host needs it
    // to reuse the set).  Its waves store their timing records beside their
    // statistics (the span of the set's last frame: xrt_read_stats); in a
    // timed region every frame keeps them apart (the mean span over the
    // region's frames: xrt_timing_end) and every kEventStride-th
    // dispatch also carries a start event (xrt_timing_events).
    Outputs out = pf.out;
    out.wave_times = fs.times;
    hipEvent_t t0 = nullptr, t1 = fs.done;
    const uint64_t frame_in_region = ctx->timing ? ctx->timed_frames++ : 0;
    if (ctx->timing && rows > 0 && frame_in_region == 0 &&
        ctx->timing_space < std::min(kTimingRecords, kTimingFrames * (size_t)fs.n_blocks)) {
        // the region's first frame is larger than the space xrt_timing_begin
        // sized from the context's previous frame (or there was none): room for
        // kTimingFrames of these, before any record of the region is kept
        const size_t space = std::min(kTimingRecords, kTimingFrames * (size_t)fs.n_blocks);
        XRT_HIP(ctx, hipStreamSynchronize(stream));
        for (auto& c : ctx->tchunks) (void)hipFree(c.p);
        ctx->tchunks.clear();
        xrt_context::TimesChunk c = {nullptr, space, 0};
        XRT_HIP(ctx, hipMalloc(&c.p, space * sizeof(uint2)));
        ctx->tchunks.push_back(c);
        ctx->timing_space = space;
    }
    if (ctx->timing && rows > 0 && ctx->timed_records + fs.n_blocks <= ctx->timing_space) {
        ctx->timed_records += fs.n_blocks;
        uint2* slot = nullptr;
        int rc = timing_slot(ctx, fs.n_blocks, slot);
        if (rc) return rc;
        out.wave_times = slot;
    }
    fs.last_times = out.wave_times;
    fs.rendered_blocks = fs.n_blocks;
    if (ctx->timing && rows > 0 && frame_in_region % kEventStride == 0) {
        if (ctx->tev_used + 2 > ctx->tev.size()) {
            for (int k = 0; k < 64; ++k) {
                hipEvent_t e;
                XRT_HIP(ctx, hipEventCreate(&e));
                ctx->tev.push_back(e);
            }
        }
        t0 = ctx->tev[ctx->tev_used];
        t1 = ctx->tev[ctx->tev_used + 1];
        ctx->tev_used += 2;
    }
    if (rows > 0) {
        const bool sgn = p.model == kModelSigned;
        const auto t_launch = HostClock::now();
        if (kernel == XRT_KERNEL_BRUTE)
            hipExtLaunchKernelGGL(sgn ? k_render_brute<true> : k_render_brute<false>, grid, dim3(256), 0, stream,
                                  t0, t1, 0, fs.recs, p, out);
        else if (kernel == XRT_KERNEL_TILED || !binned)
            hipExtLaunchKernelGGL(k_render_tiled, dim3(rx, ry), dim3(256), 0, stream, t0, t1, 0,
                                  fs.recs, fs.cull, p, out);
        else
            hipExtLaunchKernelGGL(sgn ? k_render_binned<true>
                                      : out.packed == kLayoutHits ? k_render_binned_hits : k_render_binned<false>, grid, dim3(64 * kTileWaves),
                                  0, stream, t0, t1, 0, fs.recs, fs.cull, p, out, bins, (const BinState*)bin_ctl);
        XRT_HIP(ctx, hipGetLastError());
        ctx->acc_ms[4] += std::chrono::duration<double, std::milli>(HostClock::now() - t_launch).count();
        if (ctx->host_profile) ctx->hp_lrender += seconds_since(t_launch);
        fs.done_ev = t1;
        fs.done_valid = true;
        if (binned && bins.tile_plan) ++ctx->hp_tile_plan_frames;
        // The geometry's tile plan from this render's records, once (behind
        // the render on its stream; frames in flight read either value, both
        // exact for the geometry).
        if (binned && !sgn && pf.plan_source && ctx->tile_plan_enabled && ctx->tile_plan_state == 0 &&
            bins.tile_slots > bins.split_slots) {
            const uint32_t n = bins.tile_slots - bins.split_slots;
            hipLaunchKernelGGL(k_tile_plan, dim3((n + 255) / 256), dim3(256), 0, stream, fs.block_stats,
                               ctx->compact_layout.d_desc, bins.split_slots, bins.tile_slots);
            XRT_HIP(ctx, hipGetLastError());
            // the set's completion event covers k_tile_plan too: the set's
            // statistics records and the layout's descriptions are not
            // rewritten while it reads / writes them
            XRT_HIP(ctx, hipEventRecord(fs.done, stream));
            fs.done_ev = fs.done;
            ctx->tile_plan_state = 1;
            ++ctx->hp_tile_plans;
        }
    }
    if (ctx->host_profile) {
        ctx->hp_total += seconds_since(t_call);
        if (ctx->hp_calls) ctx->hp_gap += std::chrono::duration<double>(t_call - ctx->hp_last_end).count();
        ctx->hp_last_end = HostClock::now();
        ++ctx->hp_calls;
    }
    ctx->last_set = &fs;
    ctx->next_set = (int)((&fs - ctx->sets) + 1) % kFrameSets;
    ctx->last_stream = stream;
    ctx->pending = true;
    ctx->last_kernel = kernel;
    return XRT_OK;
}

xrt_context::BinKey geometry_key(const xrt_context* ctx, const xrt_camera* cam, uint32_t row_begin,
                                 uint32_t row_end)
{
    xrt_context::BinKey key = {};
    key.cam = *cam;
    key.row_begin = row_begin;
    key.row_end = row_end;
    key.T = ctx->num_tris;
    key.gen = ctx->mesh_gen;
    return key;
}

// One frame: its preparation (or the one prepared ahead for it) and its
// render; `ahead` (the pipelined device-pointer entry) prepares the next
// frames of a repeated geometry ahead of their calls (xrt_context::ahead).
int enqueue_render(xrt_context* ctx, const xrt_camera* cam, uint32_t row_begin, uint32_t row_end,
                   float* d_image, float* d_lbuffer, uint8_t* d_u8, hipStream_t stream, bool ahead = false)
{
    int rc = check_camera(ctx, cam, row_begin, row_end);
    if (rc) return rc;
    const xrt_context::BinKey key = geometry_key(ctx, cam, row_begin, row_end);
    const uint32_t outs = (d_image ? 1u : 0u) | (d_lbuffer ? 2u : 0u) | (d_u8 ? 4u : 0u);
    PendingFrame pf;
    bool taken = false;
    if (!ctx->ahead.empty()) {
        xrt_context::AheadFrame& a = ctx->ahead.front();
        if (ahead && a.key.same(key) && a.state_gen == ctx->state_gen && a.outs == outs) {
            pf = a.pf;
            ctx->ahead.pop_front();
            pf.stream = stream;
            pf.out.image = d_image;
            pf.out.lbuffer = d_lbuffer;
            pf.out.image_u8 = d_u8;
            pf.t_call = HostClock::now();
            taken = true;
            ++ctx->hp_ahead_used;
        } else {                       // their k_prep runs before any newer one (prep stream)
            ctx->hp_ahead_dropped += ctx->ahead.size();
            ctx->ahead.clear();
        }
    }
    if (!taken && (rc = prepare_frame(ctx, cam, row_begin, row_end, d_image, d_lbuffer, d_u8, stream, pf)))
        return rc;
    const bool repeated = ahead && key.same(ctx->call_key) && ctx->call_state_gen == ctx->state_gen;
    ctx->call_key = key;
    ctx->call_state_gen = ahead ? ctx->state_gen : ~0ull;
    if ((rc = launch_frame(ctx, pf))) return rc;
    // the next frames of a repeated geometry, prepared now (a steady frame:
    // no sizing, no check to read on the host)
    if (repeated && !pf.host_wait && pf.rows > 0) {
        while (ctx->ahead.size() < kAheadFrames) {
            xrt_context::AheadFrame a;
            a.key = key;
            a.state_gen = ctx->state_gen;
            a.outs = outs;
            const int set = (int)((ctx->next_set + ctx->ahead.size()) % kFrameSets);
            if ((rc = prepare_frame(ctx, cam, row_begin, row_end, d_image, d_lbuffer, d_u8, stream, a.pf, set))) {
                ctx->ahead.clear();
                return rc;
            }
            a.pf.ahead = true;
            ctx->ahead.push_back(a);
        }
    }
    return XRT_OK;
}

// One plane's device -> host copy of a host-buffer call.
struct D2HCopy {
    void* dst;
    const void* src;
    size_t bytes;
};

// Copies `copies` (device -> the caller's host pages) behind the work already
// on `stream`: kStageChunk pieces DMAed in order into the pinned ring on the
// stream, each moved into the caller's pages by a copy thread once its DMA is
// complete; a ring slot is reused once its previous piece has been moved.
// Without copy threads (XRT_D2H_THREADS=0): pageable copies + synchronise.
int d2h_copy(xrt_context* ctx, hipStream_t stream, const std::vector<D2HCopy>& copies)
{
    struct Piece {
        uint8_t* dst;
        const uint8_t* src;
        size_t bytes;
    };
    std::vector<Piece> pieces;                         // at most kStageChunk, ending at 2-MB boundaries of dst
    for (const D2HCopy& c : copies) {
        size_t o = 0;
        while (o < c.bytes) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(c.dst) + o;
            const size_t len = std::min(kStageChunk - (size_t)(a % kStageChunk), c.bytes - o);
            pieces.push_back({(uint8_t*)c.dst + o, (const uint8_t*)c.src + o, len});
            o += len;
        }
    }
    if (pieces.empty()) return XRT_OK;
    if (!ctx->pool) {
        for (const D2HCopy& c : copies)
            if (c.bytes) XRT_HIP(ctx, hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost, stream));
        XRT_HIP(ctx, hipStreamSynchronize(stream));
        return XRT_OK;
    }
    const size_t n = pieces.size();
    std::atomic<size_t> enqueued{0};                   // pieces whose DMA (and event) is enqueued
    std::unique_ptr<std::atomic<uint8_t>[]> moved(new std::atomic<uint8_t>[n]);
    for (size_t i = 0; i < n; ++i) moved[i].store(0);
    std::atomic<int> failed{0};
    ctx->pool->start(n, [&](size_t i) {
        while (enqueued.load(std::memory_order_acquire) <= i) {
            if (failed.load()) {
                moved[i].store(1, std::memory_order_release);
                return;
            }
            std::this_thread::yield();
        }
        if (hipEventSynchronize(ctx->stage_ev[i % kStageSlots]) != hipSuccess)
            failed.store(1);
        else
            std::memcpy(pieces[i].dst, ctx->h_stage + (i % kStageSlots) * kStageChunk, pieces[i].bytes);
        moved[i].store(1, std::memory_order_release);
    });
    hipError_t err = hipSuccess;
    for (size_t i = 0; i < n; ++i) {
        if (i >= kStageSlots)                          // the slot's previous piece has been moved
            while (!moved[i - kStageSlots].load(std::memory_order_acquire)) std::this_thread::yield();
        uint8_t* slot = ctx->h_stage + (i % kStageSlots) * kStageChunk;
        err = hipMemcpyAsync(slot, pieces[i].src, pieces[i].bytes, hipMemcpyDeviceToHost, stream);
        if (err == hipSuccess) err = hipEventRecord(ctx->stage_ev[i % kStageSlots], stream);
        if (err != hipSuccess) {
            failed.store(1);
            break;
        }
        enqueued.store(i + 1, std::memory_order_release);
    }
    ctx->pool->wait();
    if (err != hipSuccess) return fail(ctx, XRT_ERR_DEVICE, std::string("D2H copy: ") + hipGetErrorString(err));
    if (failed.load()) return fail(ctx, XRT_ERR_DEVICE, "D2H copy: a staged piece failed");
    return XRT_OK;
}

}  // namespace

extern "C" {

int xrt_debug_destroy_ms(double ms[4])
{
    if (!ms) return XRT_ERR_ARGUMENT;
    std::copy(g_destroy_ms, g_destroy_ms + 4, ms);
    return XRT_OK;
}

int xrt_abi_version(void) { return XRT_ABI_VERSION; }

int xrt_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// XRT_SEGV_TRACE=1 (diagnostics): a fatal signal prints every frame of the
// faulting thread with the shared library it lies in (dladdr), then the
// signal is raised again with its default action.
namespace {
void fatal_signal_trace(int sig, siginfo_t* si, void*)
{
    void* frames[64];
    const int n = backtrace(frames, 64);
    char line[512];
    int k = std::snprintf(line, sizeof line, "xrt: signal %d (fault address %p), pid %d, %d frames:\n", sig,
                          si ? si->si_addr : nullptr, (int)getpid(), n);
    (void)!write(2, line, (size_t)std::max(k, 0));
    for (int i = 0; i < n; ++i) {
        Dl_info d = {};
        if (dladdr(frames[i], &d) && d.dli_fname)
            k = std::snprintf(line, sizeof line, "  #%-2d %p %s + %#lx (%s)\n", i, frames[i], d.dli_fname,
                              (unsigned long)((uintptr_t)frames[i] - (uintptr_t)d.dli_fbase),
                              d.dli_sname ? d.dli_sname : "?");
        else
            k = std::snprintf(line, sizeof line, "  #%-2d %p (no library)\n", i, frames[i]);
        (void)!write(2, line, (size_t)std::max(k, 0));
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

void install_fatal_signal_trace()
{
    static std::once_flag once;
    std::call_once(once, [] {
        const char* v = std::getenv("XRT_SEGV_TRACE");
        if (!v || std::atoi(v) == 0) return;
        struct sigaction sa = {};
        sa.sa_sigaction = fatal_signal_trace;
        sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
        sigemptyset(&sa.sa_mask);
        for (int sig : {SIGSEGV, SIGBUS, SIGABRT, SIGILL, SIGFPE}) sigaction(sig, &sa, nullptr);
    });
}
}  // namespace

int xrt_create(int device, xrt_context** out)
{
    install_fatal_signal_trace();
    if (!out) return fail(nullptr, XRT_ERR_ARGUMENT, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(nullptr, XRT_ERR_DEVICE,
                    std::string("no HIP device available: ") + hipGetErrorString(e));
    if (device < 0 || device >= n)
        return fail(nullptr, XRT_ERR_ARGUMENT, "device index out of range");
    if ((e = hipSetDevice(device)) != hipSuccess)
        return fail(nullptr, XRT_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
    xrt_context* ctx = new xrt_context();
    ctx->device = device;
    const char* hp = std::getenv("XRT_HOST_PROFILE");
    ctx->host_profile = hp && std::atoi(hp) != 0;
    if (const char* tp = std::getenv("XRT_TILE_PLAN")) ctx->tile_plan_enabled = std::atoi(tp) != 0;
    const char* sp = std::getenv("XRT_SIZING_PROFILE");
    ctx->sizing_profile = sp ? std::atoi(sp) : 0;
    if (const char* sm = std::getenv("XRT_SPLIT_MIN")) ctx->split_min = (uint32_t)std::strtoul(sm, nullptr, 10);
    if (const char* mp = std::getenv("XRT_MOTION_POOL")) ctx->motion_pool_forced = std::strtoull(mp, nullptr, 10);
    if (const char* bm = std::getenv("XRT_BOX_MASKS")) ctx->box_masks = std::atoi(bm);
    if (const char* df = std::getenv("XRT_DEVICE_FILL")) ctx->device_fill = std::atoi(df) != 0;
    if (const char* dq = std::getenv("XRT_DEVICE_FIRST")) ctx->device_first = std::atoi(dq) != 0;
    int n_cu = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu <= 0)
        n_cu = 256;
    ctx->wave_slots = (uint32_t)n_cu * 32u;
    // The prep stream at the default queue priority: frames are prepared ahead
    // of their renders (the highest and the lowest priority measured the same).
    bool ok = hipEventCreate(&ctx->ev_begin) == hipSuccess && hipEventCreate(&ctx->ev_end) == hipSuccess;
    ok = ok && acquire_streams(device, ctx->prep_stream, ctx->host_stream);
    ctx->owns_streams = ok;
    hipFuncAttributes prep_attr = {};
    ok = ok && hipFuncGetAttributes(&prep_attr, reinterpret_cast<const void*>(k_prep)) == hipSuccess;
    // k_prep's own LDS must fit the cap (else more than XRT_PREP_PER_CU would not fit beside the render)
    ok = ok && prep_attr.sharedSizeBytes <= kPrepLds;
    ctx->prep_lds = ok ? kPrepLds - prep_attr.sharedSizeBytes : 0;
    ok = ok && hipMalloc(&ctx->d_stats_partial, kReduceMaxBlocks * sizeof(StatsSum)) == hipSuccess &&
         hipMalloc(&ctx->d_stats_done, sizeof(unsigned int)) == hipSuccess &&
         hipMemset(ctx->d_stats_done, 0, sizeof(unsigned int)) == hipSuccess &&
         hipMalloc(&ctx->d_stats_out, sizeof(StatsSum)) == hipSuccess &&
         hipHostMalloc((void**)&ctx->h_stats, sizeof(StatsSum), hipHostMallocDefault) == hipSuccess;
    for (FrameSet& fs : ctx->sets)     // dispatch-attached events need timing enabled
        ok = ok && hipMalloc(&fs.frame, sizeof(RenderParams)) == hipSuccess &&
             hipEventCreate(&fs.ready) == hipSuccess &&
             hipEventCreate(&fs.done) == hipSuccess &&
             hipHostMalloc((void**)&fs.plan_flag, 2 * sizeof(uint32_t), hipHostMallocCoherent) == hipSuccess;
    // the host-buffer entry points' stream, pinned D2H ring and copy threads
    int threads = kD2HThreads;
    if (const char* th = std::getenv("XRT_D2H_THREADS")) threads = std::max(0, std::atoi(th));
    ok = ok && hipEventCreateWithFlags(&ctx->host_render_done, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&ctx->sizing_ev, hipEventDisableTiming) == hipSuccess &&
         hipHostMalloc((void**)&ctx->h_sizing, kSizingScratch, hipHostMallocDefault) == hipSuccess;
    if (ok) ctx->h_sizing_cap = kSizingScratch;
    if (ok && threads > 0) {
        ok = hipHostMalloc((void**)&ctx->h_stage, kStageSlots * kStageChunk, hipHostMallocDefault) == hipSuccess;
        for (hipEvent_t& e : ctx->stage_ev)
            ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
        if (ok) ctx->pool.reset(new CopyPool(threads));
    }
    if (!ok) {
        xrt_destroy(ctx);
        return fail(nullptr, XRT_ERR_DEVICE, "device allocation failed");
    }
    *out = ctx;
    return XRT_OK;
}

void xrt_destroy(xrt_context* ctx)
{
    if (!ctx) return;
    if (ctx->host_profile && ctx->hp_calls)
        std::fprintf(stderr, "xrt host profile: %llu enqueues, per call %.1f us (waiting: set reuse %.1f us, "
                     "preparation %.1f us; launching: k_prep %.1f us, render %.1f us; between calls %.1f us)\n",
                     (unsigned long long)ctx->hp_calls, ctx->hp_total / ctx->hp_calls * 1e6,
                     ctx->hp_done / ctx->hp_calls * 1e6, ctx->hp_prep / ctx->hp_calls * 1e6,
                     ctx->hp_lprep / ctx->hp_calls * 1e6, ctx->hp_lrender / ctx->hp_calls * 1e6,
                     ctx->hp_gap / ctx->hp_calls * 1e6);
    if (ctx->host_profile && ctx->hp_calls)
        std::fprintf(stderr, "xrt geometry: %llu sizings, %llu camera reuses; frames flagged by k_prep: %llu plan "
                     "misses, %llu list overflows; prepared ahead: %llu used, %llu dropped; renders launched "
                     "without a wait: %llu\n", (unsigned long long)ctx->hp_sizings,
                     (unsigned long long)ctx->hp_reused, (unsigned long long)ctx->hp_plan_miss,
                     (unsigned long long)ctx->hp_overflow, (unsigned long long)ctx->hp_ahead_used,
                     (unsigned long long)ctx->hp_ahead_dropped, (unsigned long long)ctx->hp_launch_nowait);
    (void)hipSetDevice(ctx->device);
    auto t = HostClock::now();
    auto lap = [&](int k) {
        const auto now = HostClock::now();
        g_destroy_ms[k] = std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    };
    (void)sync_context(ctx);
    if (ctx->host_stream) (void)hipStreamSynchronize(ctx->host_stream);
    lap(0);
    ctx->pool.reset();
    (void)hipFree(ctx->d_tris);
    for (FrameSet& fs : ctx->sets) {
        (void)hipFree(fs.recs);
        (void)hipFree(fs.cull);
        (void)hipFree(fs.block_stats);
        (void)hipFree(fs.frame);
        if (fs.plan_flag) (void)hipHostFree((void*)fs.plan_flag);
        (void)hipFree(fs.offsets);
        (void)hipFree(fs.bin_counts);
        (void)hipFree(fs.bin_list);
        (void)hipFree(fs.global_list);
        (void)hipFree(fs.times);
        (void)hipFree(fs.dyn_desc);
        (void)hipFree(fs.pairs);
        (void)hipFree(fs.plan_desc);
        (void)hipFree(fs.plan_counts);
        for (hipEvent_t e : {fs.ready, fs.done})
            if (e) (void)hipEventDestroy(e);
    }
    for (SlotLayout* L : {&ctx->fixed, &ctx->compact_layout}) {
        (void)hipFree(L->d_desc);
        (void)hipFree(L->d_rank);
    }
    (void)hipFree(ctx->d_image);
    (void)hipFree(ctx->d_lbuffer);
    (void)hipFree(ctx->d_u8);
    (void)hipFree(ctx->d_stats_partial);
    (void)hipFree(ctx->d_stats_done);
    (void)hipFree(ctx->d_stats_out);
    (void)hipFree(ctx->d_hit_off);
    (void)hipFree(ctx->d_prep_times);
    for (auto& c : ctx->tchunks) (void)hipFree(c.p);
    lap(1);
    if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->h_sizing) (void)hipHostFree(ctx->h_sizing);
    lap(2);
    if (ctx->owns_streams) release_streams(ctx->device);     // the device's shared streams
    for (hipEvent_t e : ctx->tev) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->stage_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->host_render_done) (void)hipEventDestroy(ctx->host_render_done);
    if (ctx->sizing_ev) (void)hipEventDestroy(ctx->sizing_ev);
    if (ctx->ev_begin) (void)hipEventDestroy(ctx->ev_begin);
    if (ctx->ev_end) (void)hipEventDestroy(ctx->ev_end);
    lap(3);
    delete ctx;
}

const char* xrt_last_error(const xrt_context* ctx)
{
    return ctx ? ctx->error.c_str() : g_create_error.c_str();
}

int xrt_upload_mesh(xrt_context* ctx, const float* triangles, uint64_t num_triangles)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (num_triangles && !triangles) return fail(ctx, XRT_ERR_ARGUMENT, "triangles is NULL");
    if (num_triangles > 0xFFFFFFFFull) return fail(ctx, XRT_ERR_ARGUMENT, "too many triangles");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    int rc = sync_context(ctx);                   // frames in flight read the mesh (prep stream)
    if (rc) return rc;
    rc = ensure(ctx, ctx->d_tris, ctx->tris_cap, 9 * num_triangles);
    if (rc) return rc;
    if (num_triangles)
        XRT_HIP(ctx, hipMemcpy(ctx->d_tris, triangles, 9 * num_triangles * sizeof(float),
                               hipMemcpyHostToDevice));
    ctx->num_tris = num_triangles;
    ++ctx->mesh_gen;
    ++ctx->state_gen;
    return XRT_OK;
}

int xrt_mesh_bbox(const float* tris, uint64_t n, float lower[3], float upper[3])
{
    if ((n && !tris) || !lower || !upper) return XRT_ERR_ARGUMENT;
    const float inf = std::numeric_limits<float>::infinity();
    for (int k = 0; k < 3; ++k) {
        lower[k] = inf;
        upper[k] = -inf;
    }
    // TriangleMesh::computeBoundingBox, src/TriangleMesh.cxx:200-227 (p1, p2, p3 in turn)
    for (uint64_t i = 0; i < n; ++i)
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) {
                float x = tris[9 * i + 3 * v + k];
                lower[k] = stdmin(lower[k], x);
                upper[k] = stdmax(upper[k], x);
            }
    return XRT_OK;
}

int xrt_scene_bbox(const float* tris, const uint64_t* mesh_triangles, uint32_t num_meshes, float lower[3],
                   float upper[3])
{
    if ((num_meshes && !mesh_triangles) || !lower || !upper) return XRT_ERR_ARGUMENT;
    const float inf = std::numeric_limits<float>::infinity();
    for (int k = 0; k < 3; ++k) {
        lower[k] = inf;
        upper[k] = -inf;
    }
    // getBBox, src/main.cxx:545-562: the corners of each mesh's box in turn
    uint64_t first = 0;
    for (uint32_t m = 0; m < num_meshes; ++m) {
        float lo[3], hi[3];
        const uint64_t n = mesh_triangles[m];
        if (n && !tris) return XRT_ERR_ARGUMENT;
        xrt_mesh_bbox(n ? tris + 9 * first : nullptr, n, lo, hi);
        for (int k = 0; k < 3; ++k) {
            lower[k] = stdmin(lower[k], lo[k]);
            upper[k] = stdmax(upper[k], hi[k]);
        }
        first += n;
    }
    return XRT_OK;
}

int xrt_camera_from_bbox(const float lower[3], const float upper[3], uint32_t width,
                         uint32_t height, xrt_camera* out)
{
    if (!lower || !upper || !out || !width || !height) return XRT_ERR_ARGUMENT;
    // initialiseRayTracing, src/main.cxx:575-604
    float range[3] = {upper[0] - lower[0], upper[1] - lower[1], upper[2] - lower[2]};
    float centre[3];
    for (int k = 0; k < 3; ++k) centre[k] = lower[k] + (float)((double)range[k] / 2.0);
    float diagonal = length3(range);
    float up[3] = {0.0f, 0.0f, -1.0f};
    float origin[3] = {centre[0] - diagonal * 1, centre[1] - 0.0f, centre[2] - 0.0f};
    float xoff = (float)((double)diagonal * 0.6);
    float detector[3] = {centre[0] + xoff, centre[1] + 0.0f, centre[2] + 0.0f};
    float direction[3] = {detector[0] - origin[0], detector[1] - origin[1], detector[2] - origin[2]};
    normalise3(direction);
    normalise3(direction);
    float right[3];
    cross3(direction, up, right);
    // renderLoop prologue, src/main.cxx:637-641
    float res1 = range[2] / (float)width;
    float res2 = range[1] / (float)height;
    float spacing = 2 * stdmax(res1, res2);
    std::memcpy(out->origin, origin, sizeof origin);
    std::memcpy(out->detector, detector, sizeof detector);
    std::memcpy(out->up, up, sizeof up);
    std::memcpy(out->right, right, sizeof right);
    out->pixel_spacing = spacing;
    out->width = width;
    out->height = height;
    return XRT_OK;
}

int xrt_set_kernel(xrt_context* ctx, int kernel)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (kernel < XRT_KERNEL_AUTO || kernel > XRT_KERNEL_BINNED)
        return fail(ctx, XRT_ERR_ARGUMENT, "unknown kernel");
    ctx->kernel = kernel;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_set_model(xrt_context* ctx, int model, float mu)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (model != XRT_MODEL_ATTENUATION && model != XRT_MODEL_SIGNED)
        return fail(ctx, XRT_ERR_ARGUMENT, "unknown model");
    ctx->model = (uint32_t)model;
    ctx->mu = mu;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_hole_fill_device(xrt_context* ctx, uint32_t width, uint32_t height, const float* d_lbuffer,
                         float* d_image, uint8_t* d_u8, void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    const uint64_t n = (uint64_t)width * height;
    if (n > 0xFFFFFFFFull) return fail(ctx, XRT_ERR_ARGUMENT, "image larger than 2^32-1 pixels");
    if (!n) return XRT_OK;
    if (!d_lbuffer) return fail(ctx, XRT_ERR_ARGUMENT, "L-buffer is NULL");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_hole_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_lbuffer, d_image, d_u8, width, height);
    XRT_HIP(ctx, hipGetLastError());
    return XRT_OK;
}

int xrt_hole_fill(xrt_context* ctx, uint32_t width, uint32_t height, const float* lbuffer, float* image,
                  uint8_t* image_u8)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    const size_t n = (size_t)width * height;
    if (!n) return XRT_OK;
    if (!lbuffer) return fail(ctx, XRT_ERR_ARGUMENT, "L-buffer is NULL");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    int rc;
    size_t cap_f = ctx->stage_cap, cap_l = ctx->stage_cap, cap_u = ctx->stage_cap;
    if ((rc = ensure(ctx, ctx->d_image, cap_f, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_lbuffer, cap_l, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_u8, cap_u, n))) return rc;
    ctx->stage_cap = std::min(cap_f, std::min(cap_l, cap_u));
    XRT_HIP(ctx, hipMemcpyAsync(ctx->d_lbuffer, lbuffer, n * sizeof(float), hipMemcpyHostToDevice, ctx->host_stream));
    if ((rc = xrt_hole_fill_device(ctx, width, height, ctx->d_lbuffer, image ? ctx->d_image : nullptr,
                                   image_u8 ? ctx->d_u8 : nullptr, ctx->host_stream)))
        return rc;
    std::vector<D2HCopy> copies;
    if (image) copies.push_back({image, ctx->d_image, n * sizeof(float)});
    if (image_u8) copies.push_back({image_u8, ctx->d_u8, n});
    return d2h_copy(ctx, ctx->host_stream, copies);
}

int xrt_render_signed(xrt_context* ctx, const xrt_camera* camera, float* image, float* lbuffer,
                      uint8_t* image_u8, xrt_stats* stats)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (ctx->model != kModelSigned) return fail(ctx, XRT_ERR_ARGUMENT, "xrt_render_signed needs XRT_MODEL_SIGNED");
    int rc = check_camera(ctx, camera, 0, camera ? camera->height : 0);
    if (rc) return rc;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)camera->width * camera->height;
    size_t cap_f = ctx->stage_cap, cap_l = ctx->stage_cap, cap_u = ctx->stage_cap;
    if ((rc = ensure(ctx, ctx->d_image, cap_f, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_lbuffer, cap_l, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_u8, cap_u, n))) return rc;
    ctx->stage_cap = std::min(cap_f, std::min(cap_l, cap_u));
    if ((rc = enqueue_render(ctx, camera, 0, camera->height, nullptr, ctx->d_lbuffer, nullptr, ctx->host_stream)))
        return rc;
    if ((rc = xrt_hole_fill_device(ctx, camera->width, camera->height, ctx->d_lbuffer,
                                   image ? ctx->d_image : nullptr, image_u8 ? ctx->d_u8 : nullptr,
                                   ctx->host_stream)))
        return rc;
    std::vector<D2HCopy> copies;
    if (n) {
        if (image) copies.push_back({image, ctx->d_image, n * sizeof(float)});
        if (lbuffer) copies.push_back({lbuffer, ctx->d_lbuffer, n * sizeof(float)});
        if (image_u8) copies.push_back({image_u8, ctx->d_u8, n});
    }
    if ((rc = d2h_copy(ctx, ctx->host_stream, copies))) return rc;
    xrt_stats local;
    return xrt_read_stats(ctx, stats ? stats : &local);
}

int xrt_set_miss_code(xrt_context* ctx, uint32_t bits)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (bits && bits != kMissTransit) return fail(ctx, XRT_ERR_ARGUMENT, "miss code must be 0 or XRT_MISS_TRANSIT");
    ctx->miss_code = bits;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_expand_rows_device(xrt_context* ctx, uint64_t num_pixels, float* d_lbuffer, float* d_image,
                           uint8_t* d_u8, void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (num_pixels && !d_lbuffer) return fail(ctx, XRT_ERR_ARGUMENT, "lbuffer is NULL");
    if (!num_pixels) return XRT_OK;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    const uint64_t threads = (num_pixels + 3) / 4;
    hipLaunchKernelGGL(k_expand, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_lbuffer, d_image, d_u8, num_pixels);
    XRT_HIP(ctx, hipGetLastError());
    return XRT_OK;
}

int xrt_set_hit_capacity(xrt_context* ctx, uint32_t capacity)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (capacity > (uint32_t)kMaxHits)
        return fail(ctx, XRT_ERR_ARGUMENT, "capacity > " + std::to_string(kMaxHits));
    ctx->hit_capacity = capacity ? capacity : (uint32_t)kMaxHits;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_set_bin_capacity(xrt_context* ctx, uint64_t entries)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    ctx->bin_force_cap = (size_t)entries;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_plan_region_map(xrt_context* ctx, uint32_t width, uint32_t rows, uint32_t* map, uint64_t n_regions,
                        uint32_t* n_packed)
{
    if (!ctx || !map || !n_packed) return fail(ctx, XRT_ERR_ARGUMENT, "NULL argument");
    const uint32_t rx = (width + kRegion - 1) / kRegion, ry = (rows + kRegion - 1) / kRegion;
    if (n_regions != (uint64_t)rx * ry)
        return fail(ctx, XRT_ERR_ARGUMENT, "map must hold ceil(width/32) x ceil(rows/32) regions");
    const SlotLayout& L = ctx->compact_layout;
    const bool layout = L.rx == rx && L.ry == ry && L.slot_region.size() == n_regions;
    const bool planned = ctx->last_fill_regions > 0 && ctx->plan_valid && layout;
    // no region of the geometry is empty: every region travels, in slot order
    // (the order of the hit layout's tiles)
    const bool whole = !ctx->plan_valid && ctx->last_fill_regions == 0 && layout && ctx->compact &&
                       ctx->bin_key_valid && ctx->last_key.same(ctx->bin_key);
    if (!planned && !whole) {                       // every region travels
        for (uint64_t r = 0; r < n_regions; ++r) map[r] = (uint32_t)r;
        *n_packed = (uint32_t)n_regions;
        return XRT_OK;
    }
    for (uint64_t s = 0; s < n_regions; ++s)
        map[L.slot_region[s]] = s < ctx->plan_tile_slots ? (uint32_t)s : kEmpty;
    *n_packed = ctx->plan_tile_slots;
    return XRT_OK;
}

int xrt_pack_regions_device(xrt_context* ctx, uint32_t width, uint32_t rows, const uint32_t* d_map,
                            const float* d_lbuffer, float* d_packed, void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    const uint32_t rx = (width + kRegion - 1) / kRegion, ry = (rows + kRegion - 1) / kRegion;
    if (!rx || !ry) return XRT_OK;
    if (!d_map || !d_lbuffer || !d_packed) return fail(ctx, XRT_ERR_ARGUMENT, "NULL buffer");
    if (reinterpret_cast<uintptr_t>(d_packed) & 15u) return fail(ctx, XRT_ERR_ARGUMENT, "packed buffer not 16-B aligned");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_pack_regions, dim3(rx * ry), dim3(256), 0, (hipStream_t)stream, d_lbuffer, d_packed, d_map,
                       width, rows, rx);
    XRT_HIP(ctx, hipGetLastError());
    return XRT_OK;
}

int xrt_unpack_regions_device(xrt_context* ctx, uint32_t width, uint32_t rows, const uint32_t* d_map,
                              const float* d_packed, float* d_lbuffer, float* d_image, uint8_t* d_u8, void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    const uint32_t rx = (width + kRegion - 1) / kRegion, ry = (rows + kRegion - 1) / kRegion;
    if (!rx || !ry) return XRT_OK;
    if (!d_map || !d_packed) return fail(ctx, XRT_ERR_ARGUMENT, "NULL buffer");
    if (reinterpret_cast<uintptr_t>(d_packed) & 15u) return fail(ctx, XRT_ERR_ARGUMENT, "packed buffer not 16-B aligned");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_unpack_regions, dim3(rx * ry), dim3(256), 0, (hipStream_t)stream, d_packed, d_map,
                       d_lbuffer, d_image, d_u8, width, rows, rx);
    XRT_HIP(ctx, hipGetLastError());
    return XRT_OK;
}

int xrt_unpack_blocks_device(xrt_context* ctx, uint32_t width, uint64_t n_blocks, const uint32_t* d_desc,
                             const float* d_packed, float* d_lbuffer, float* d_image, uint8_t* d_u8, void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (!n_blocks) return XRT_OK;
    if (!d_desc || !d_packed) return fail(ctx, XRT_ERR_ARGUMENT, "NULL buffer");
    if (n_blocks > 0x7FFFFFFFull) return fail(ctx, XRT_ERR_ARGUMENT, "too many blocks");
    if ((reinterpret_cast<uintptr_t>(d_packed) | reinterpret_cast<uintptr_t>(d_desc)) & 15u)
        return fail(ctx, XRT_ERR_ARGUMENT, "packed buffer or descriptors not 16-B aligned");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_unpack_blocks, dim3((unsigned)n_blocks), dim3(256), 0, (hipStream_t)stream, d_packed,
                       reinterpret_cast<const uint4*>(d_desc), d_lbuffer, d_image, d_u8, width);
    XRT_HIP(ctx, hipGetLastError());
    return XRT_OK;
}

int xrt_set_transit_layout(xrt_context* ctx, uint64_t packed_floats)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    ctx->packed_cap = packed_floats;
    if (packed_floats) ctx->hits_cap = 0;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_set_transit_hits(xrt_context* ctx, uint64_t capacity_words)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    ctx->hits_cap = capacity_words;
    if (capacity_words) ctx->packed_cap = 0;
    ++ctx->state_gen;
    return XRT_OK;
}

int xrt_plan_hit_layout(xrt_context* ctx, uint32_t* tile_hits, uint64_t capacity, uint64_t* n_tiles,
                        uint64_t* words)
{
    if (!ctx || !n_tiles || !words) return fail(ctx, XRT_ERR_ARGUMENT, "NULL argument");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    int rc = sync_context(ctx);
    if (rc) return rc;
    const FrameSet* fs = ctx->last_set;
    // the last frame rendered the lists' geometry over its fill plan (or, with
    // no empty region, every region in slot order): its records s * 16 + t
    // (s < the plan's tile slots) are the plan's tiles
    const bool fill_frame = ctx->plan_valid && ctx->last_fill_regions > 0;
    const bool whole_frame = !ctx->plan_valid && ctx->last_fill_regions == 0;
    if (!fs || !fs->binned || !ctx->bin_key_valid || !ctx->compact || !(fill_frame || whole_frame) ||
        !ctx->last_key.same(ctx->bin_key) || (uint64_t)ctx->plan_tile_slots * kWavesPerRegion > fs->rendered_blocks)
        return fail(ctx, XRT_ERR_ARGUMENT, "the hit plan needs a BINNED frame rendered over its geometry's fill "
                                           "plan just before");
    const uint32_t tiles = ctx->plan_tile_slots * kWavesPerRegion;
    std::vector<BlockStats> rec(tiles);
    if (tiles) XRT_HIP(ctx, hipMemcpy(rec.data(), fs->block_stats, tiles * sizeof(BlockStats), hipMemcpyDeviceToHost));
    std::vector<uint32_t> off(tiles + 1u);
    uint64_t run = 0;
    for (uint32_t i = 0; i < tiles; ++i) {
        off[i] = (uint32_t)run;
        run += rec[i].hit_rays;
        if (tile_hits && i < capacity) tile_hits[i] = rec[i].hit_rays;
    }
    if (run + 2ull * tiles > 0xFFFFFFFFull) return fail(ctx, XRT_ERR_OVERFLOW, "hit message exceeds 2^32 words");
    off[tiles] = (uint32_t)run;
    if ((rc = ensure(ctx, ctx->d_hit_off, ctx->hit_off_cap, (size_t)tiles + 1u))) return rc;
    XRT_HIP(ctx, hipMemcpy(ctx->d_hit_off, off.data(), off.size() * 4u, hipMemcpyHostToDevice));
    ctx->hit_key = ctx->bin_key;
    ctx->hit_tiles = tiles;
    ctx->hit_words = 2ull * tiles + run;
    ctx->hit_valid = true;
    ++ctx->state_gen;                   // frames prepared ahead carry the old plan
    *n_tiles = tiles;
    *words = ctx->hit_words;
    return XRT_OK;
}

int xrt_unpack_hits_device(xrt_context* ctx, uint32_t width, uint64_t n_blocks, const uint32_t* d_desc,
                           const uint32_t* d_tdesc, const uint32_t* d_msg, float* d_lbuffer, float* d_image,
                           uint8_t* d_u8, uint32_t* d_bad, void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (!n_blocks) return XRT_OK;
    if (!d_desc || !d_tdesc || !d_msg) return fail(ctx, XRT_ERR_ARGUMENT, "NULL buffer");
    if (n_blocks > 0x7FFFFFFFull) return fail(ctx, XRT_ERR_ARGUMENT, "too many blocks");
    if (((reinterpret_cast<uintptr_t>(d_desc) | reinterpret_cast<uintptr_t>(d_tdesc)) & 15u) ||
        (reinterpret_cast<uintptr_t>(d_msg) & 7u))
        return fail(ctx, XRT_ERR_ARGUMENT, "descriptors not 16-B aligned or message not 8-B aligned");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_unpack_hits, dim3((unsigned)n_blocks), dim3(256), 0, (hipStream_t)stream, d_msg,
                       reinterpret_cast<const uint4*>(d_desc), reinterpret_cast<const uint4*>(d_tdesc), d_lbuffer,
                       d_image, d_u8, width, d_bad);
    XRT_HIP(ctx, hipGetLastError());
    return XRT_OK;
}

int xrt_debug_fill_regions(xrt_context* ctx, uint32_t* regions)
{
    if (!ctx || !regions) return XRT_ERR_ARGUMENT;
    *regions = ctx->last_fill_regions;
    return XRT_OK;
}

int xrt_debug_geometry_counters(xrt_context* ctx, uint64_t counters[4])
{
    if (!ctx || !counters) return XRT_ERR_ARGUMENT;
    counters[0] = ctx->hp_sizings;
    counters[1] = ctx->hp_reused;
    counters[2] = ctx->hp_plan_miss;
    counters[3] = ctx->hp_overflow;
    return XRT_OK;
}

int xrt_debug_first_frames(xrt_context* ctx, uint64_t counters[4])
{
    if (!ctx || !counters) return XRT_ERR_ARGUMENT;
    counters[0] = ctx->hp_dev_first;
    counters[1] = ctx->hp_dev_first_recounts;
    counters[2] = ctx->dev_first_pairs;
    counters[3] = ctx->dev_first_pool;
    return XRT_OK;
}

int xrt_debug_host_call_ms(xrt_context* ctx, double ms[16])
{
    if (!ctx || !ms) return XRT_ERR_ARGUMENT;
    std::copy(ctx->host_call_ms, ctx->host_call_ms + kHostCallFields, ms);
    return XRT_OK;
}

int xrt_debug_prep_times(xrt_context* ctx, int enable, uint32_t* dst, uint64_t capacity, uint64_t* n_waves)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (enable >= 0) ctx->prep_times_on = enable != 0;
    if (n_waves) *n_waves = ctx->prep_times_n;
    if (!dst || !ctx->d_prep_times || !ctx->prep_times_n) return XRT_OK;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    int rc = sync_context(ctx);
    if (rc) return rc;
    const size_t n = std::min<size_t>(capacity, ctx->prep_times_n);
    XRT_HIP(ctx, hipMemcpy(dst, ctx->d_prep_times, n * 2 * sizeof(uint4), hipMemcpyDeviceToHost));
    return XRT_OK;
}

int xrt_debug_direction_grid(const xrt_camera* camera, int grids[2])
{
    if (!camera || !grids) return XRT_ERR_ARGUMENT;
    const CullParams cp = make_cull_params(*camera);
    grids[0] = cp.dir_grid;
    grids[1] = direction_grid(*camera, cp.dmax, true);
    return XRT_OK;
}

int xrt_debug_set_tile_plan(xrt_context* ctx, int on)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (ctx->tile_plan_enabled != (on != 0)) ++ctx->state_gen;   // frames prepared ahead are dropped
    ctx->tile_plan_enabled = on != 0;
    return XRT_OK;
}

int xrt_debug_tile_plan(xrt_context* ctx, uint64_t counters[2])
{
    if (!ctx || !counters) return XRT_ERR_ARGUMENT;
    counters[0] = ctx->hp_tile_plan_frames;
    counters[1] = ctx->hp_tile_plans;
    return XRT_OK;
}

int xrt_debug_pipeline_counters(xrt_context* ctx, uint64_t counters[4])
{
    if (!ctx || !counters) return XRT_ERR_ARGUMENT;
    counters[0] = ctx->hp_ahead_used;
    counters[1] = ctx->hp_ahead_dropped;
    counters[2] = ctx->hp_launch_nowait;
    counters[3] = ctx->hp_host_waits;
    return XRT_OK;
}

int xrt_set_fill_plan(xrt_context* ctx, int mode)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (mode < 0 || mode > 2) return fail(ctx, XRT_ERR_ARGUMENT, "fill plan mode must be 0, 1 or 2");
    ctx->fill_plan = mode;
    ctx->bin_key_valid = false;         // the next frame re-sizes and re-plans
    ctx->plan_valid = false;
    ++ctx->state_gen;                   // frames prepared ahead are stale
    return XRT_OK;
}

int xrt_debug_block_records(xrt_context* ctx, void* dst, uint64_t capacity, uint64_t* n_records)
{
    if (!ctx || !n_records) return XRT_ERR_ARGUMENT;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    if (ctx->pending) {
        XRT_HIP(ctx, hipStreamSynchronize(ctx->last_stream));
        ctx->pending = false;
    }
    const FrameSet* fs = ctx->last_set;
    *n_records = fs ? fs->rendered_blocks : 0u;
    const size_t bytes = std::min<size_t>((size_t)capacity, (size_t)*n_records * sizeof(BlockStats));
    if (bytes && dst) XRT_HIP(ctx, hipMemcpy(dst, fs->block_stats, bytes, hipMemcpyDeviceToHost));
    return XRT_OK;
}

int xrt_debug_wave_times(xrt_context* ctx, uint32_t frames_back, uint32_t* dst, uint64_t capacity,
                         uint64_t* n_records)
{
    if (!ctx || !n_records) return XRT_ERR_ARGUMENT;
    if (frames_back >= (uint32_t)kFrameSets)
        return fail(ctx, XRT_ERR_ARGUMENT, "frames_back must be < " + std::to_string(kFrameSets));
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    int rc = sync_context(ctx);
    if (rc) return rc;
    const FrameSet* fs = ctx->last_set
                             ? &ctx->sets[((ctx->last_set - ctx->sets) + kFrameSets - (int)frames_back) % kFrameSets]
                             : nullptr;
    // the set's last RENDER's count (a frame prepared ahead into the set since has its own)
    *n_records = fs && fs->last_times ? fs->rendered_blocks : 0u;
    const size_t n = std::min<size_t>((size_t)capacity, (size_t)*n_records);
    if (n && dst) XRT_HIP(ctx, hipMemcpy(dst, fs->last_times, n * sizeof(uint2), hipMemcpyDeviceToHost));
    return XRT_OK;
}

int xrt_render_rows_device(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin,
                           uint32_t row_end, float* d_image, float* d_lbuffer, uint8_t* d_u8,
                           void* stream)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    return enqueue_render(ctx, camera, row_begin, row_end, d_image, d_lbuffer, d_u8,
                          (hipStream_t)stream, true);
}

int xrt_render_frames_device(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin, uint32_t row_end,
                             uint32_t n_frames, uint32_t n_sets, float* const* d_image, float* const* d_lbuffer,
                             uint8_t* const* d_u8, void* const* streams)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (n_frames && !n_sets) return fail(ctx, XRT_ERR_ARGUMENT, "n_sets must be >= 1");
    for (uint32_t k = 0; k < n_frames; ++k) {
        const uint32_t s = k % n_sets;
        int rc = enqueue_render(ctx, camera, row_begin, row_end, d_image ? d_image[s] : nullptr,
                                d_lbuffer ? d_lbuffer[s] : nullptr, d_u8 ? d_u8[s] : nullptr,
                                streams ? (hipStream_t)streams[s] : nullptr, true);
        if (rc) return rc;
    }
    return XRT_OK;
}

int xrt_render_frames(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin, uint32_t row_end,
                      uint32_t n_frames, float* image, float* lbuffer, uint8_t* image_u8, xrt_stats* stats,
                      double* ms_per_frame)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    int rc = check_camera(ctx, camera, row_begin, row_end);
    if (rc) return rc;
    if (!n_frames) return fail(ctx, XRT_ERR_ARGUMENT, "n_frames must be >= 1");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)(row_end - row_begin) * camera->width;
    size_t cap_f = ctx->stage_cap, cap_l = ctx->stage_cap, cap_u = ctx->stage_cap;
    if ((rc = ensure(ctx, ctx->d_image, cap_f, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_lbuffer, cap_l, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_u8, cap_u, n))) return rc;
    ctx->stage_cap = std::min(cap_f, std::min(cap_l, cap_u));
    float* di = image ? ctx->d_image : nullptr;
    float* dl = lbuffer ? ctx->d_lbuffer : nullptr;
    uint8_t* du = image_u8 ? ctx->d_u8 : nullptr;
    void* st = ctx->host_stream;
    const auto t0 = HostClock::now();
    if ((rc = xrt_render_frames_device(ctx, camera, row_begin, row_end, n_frames, 1, &di, &dl, &du, &st))) return rc;
    XRT_HIP(ctx, hipStreamSynchronize(ctx->host_stream));
    if (ms_per_frame)
        *ms_per_frame = std::chrono::duration<double, std::milli>(HostClock::now() - t0).count() / n_frames;
    std::vector<D2HCopy> copies;
    if (n) {
        if (image) copies.push_back({image, ctx->d_image, n * sizeof(float)});
        if (lbuffer) copies.push_back({lbuffer, ctx->d_lbuffer, n * sizeof(float)});
        if (image_u8) copies.push_back({image_u8, ctx->d_u8, n});
    }
    if ((rc = d2h_copy(ctx, ctx->host_stream, copies))) return rc;
    xrt_stats local;
    return xrt_read_stats(ctx, stats ? stats : &local);
}

int xrt_read_stats(xrt_context* ctx, xrt_stats* stats)
{
    if (!ctx || !stats) return XRT_ERR_ARGUMENT;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(stats, 0, sizeof *stats);
    stats->kernel = (uint32_t)ctx->last_kernel;
    const FrameSet* fs = ctx->last_set;
    if (!fs || !fs->rendered_blocks) {
        if (ctx->pending) XRT_HIP(ctx, hipStreamSynchronize(ctx->last_stream));
        ctx->pending = false;
        return XRT_OK;
    }
    // The last render's records (and where its timing records went, and its
    // BinState) summed on the device behind the render, on its stream: one
    // record comes back instead of every wave's.
    const uint32_t n = fs->rendered_blocks;
    const hipStream_t s = ctx->last_stream;
    const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>(kReduceMaxBlocks, (n + 4 * kReduceThreads - 1) /
                                                                                          (4 * kReduceThreads)));
    hipLaunchKernelGGL(k_reduce_stats, dim3(blocks), dim3(kReduceThreads), 0, s, fs->block_stats, fs->last_times, n,
                       fs->binned ? (const BinState*)fs->last_state : nullptr, ctx->d_stats_partial, ctx->d_stats_done,
                       ctx->d_stats_out);
    XRT_HIP(ctx, hipGetLastError());
    XRT_HIP(ctx, hipMemcpyAsync(ctx->h_stats, ctx->d_stats_out, sizeof(StatsSum), hipMemcpyDeviceToHost, s));
    XRT_HIP(ctx, hipStreamSynchronize(s));
    ctx->pending = false;
    const StatsSum& t = *ctx->h_stats;
    stats->rays = t.rays;
    stats->hit_rays = t.hit_rays;
    stats->odd_rays = t.odd_rays;
    stats->overflow_rays = t.overflow_rays;
    stats->hits = t.hits;
    stats->tile_tests = t.tile_tests;
    stats->candidates = t.candidates;
    stats->max_hits = t.max_hits;
    stats->kernel_ms = fs->last_times && t.span_hi > t.span_lo ? (double)(t.span_hi - t.span_lo) / kTicksPerMs : 0.0;
    stats->global_triangles = fs->binned ? t.global_count : 0u;
    if (fs->binned && t.overflow && !ctx->bin_force_cap) {   // the next frame re-sizes its lists
        ctx->bin_key_valid = false;
        ++ctx->state_gen;
    }
    return XRT_OK;
}

int xrt_timing_begin(xrt_context* ctx)
{
    if (!ctx) return XRT_ERR_ARGUMENT;
    if (ctx->timing) {                 // a region still open: end it (its results are dropped)
        double ms = 0.0;
        uint64_t n = 0;
        if (int rc = xrt_timing_end(ctx, &ms, &n)) return rc;
    }
    // Frames in flight may mark their completion with events of the previous
    // timed region, which this one re-records: wait for them first.
    for (FrameSet& fs : ctx->sets) {
        if (fs.done_valid) XRT_HIP(ctx, hipEventSynchronize(fs.done_ev));
        fs.done_valid = false;
    }
    // the region's record space and events, before the region
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    const size_t last_blocks = ctx->last_set ? ctx->last_set->n_blocks : 0u;
    const size_t space = std::min(kTimingRecords, std::max<size_t>((size_t)1 << 20, kTimingFrames * last_blocks));
    bool have = false;
    for (auto& c : ctx->tchunks) have = have || c.cap >= space;
    if (!have) {
        for (auto& c : ctx->tchunks) (void)hipFree(c.p);
        ctx->tchunks.clear();
        xrt_context::TimesChunk c = {nullptr, space, 0};
        XRT_HIP(ctx, hipMalloc(&c.p, space * sizeof(uint2)));
        ctx->tchunks.push_back(c);
    }
    ctx->timing_space = space;
    while (ctx->tev.size() < kTimingEvents) {
        hipEvent_t e;
        XRT_HIP(ctx, hipEventCreate(&e));
        ctx->tev.push_back(e);
    }
    ctx->timing = true;
    ctx->tev_used = 0;
    ctx->timed_frames = 0;
    ctx->timed_records = 0;
    for (auto& c : ctx->tchunks) c.used = 0;
    ctx->tsamples.clear();
    return XRT_OK;
}

int xrt_timing_end(xrt_context* ctx, double* total_ms, uint64_t* launches)
{
    if (!ctx || !total_ms || !launches) return XRT_ERR_ARGUMENT;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    double ev = 0.0;
    for (size_t i = 0; i + 1 < ctx->tev_used; i += 2) {
        XRT_HIP(ctx, hipEventSynchronize(ctx->tev[i + 1]));
        float ms = 0.0f;
        XRT_HIP(ctx, hipEventElapsedTime(&ms, ctx->tev[i], ctx->tev[i + 1]));
        ev += ms;
    }
    ctx->event_ms = ev;
    ctx->event_launches = ctx->tev_used / 2;
    if (int rc = sync_context(ctx)) return rc;     // the sampled frames' records are written
    double sum = 0.0;
    std::vector<uint2> t;
    for (const auto& smp : ctx->tsamples) {
        t.resize(smp.n);
        XRT_HIP(ctx, hipMemcpy(t.data(), smp.p, smp.n * sizeof(uint2), hipMemcpyDeviceToHost));
        sum += records_span_ms(t);
    }
    *total_ms = sum;
    *launches = ctx->tsamples.size();
    ctx->tsamples.clear();
    ctx->timing = false;
    ctx->tev_used = 0;
    // Each set's last records back into its own buffer (xrt_read_stats and
    // xrt_debug_wave_times read them there), then the chunks go: a context
    // keeps at most one small chunk (kKeptTimingBytes) for its next region.
    for (FrameSet& fs : ctx->sets) {
        if (fs.last_times && fs.last_times != fs.times && fs.times && fs.rendered_blocks <= fs.times_cap)
            XRT_HIP(ctx, hipMemcpy(fs.times, fs.last_times, fs.rendered_blocks * sizeof(uint2),
                                   hipMemcpyDeviceToDevice));
        if (fs.last_times) fs.last_times = fs.times;
    }
    size_t keep = ctx->tchunks.size();
    for (size_t k = 0; k < ctx->tchunks.size(); ++k)
        if (ctx->tchunks[k].cap * sizeof(uint2) <= kKeptTimingBytes &&
            (keep == ctx->tchunks.size() || ctx->tchunks[k].cap > ctx->tchunks[keep].cap))
            keep = k;
    for (size_t k = 0; k < ctx->tchunks.size(); ++k)
        if (k != keep) (void)hipFree(ctx->tchunks[k].p);
    if (keep < ctx->tchunks.size()) {
        xrt_context::TimesChunk c = ctx->tchunks[keep];
        c.used = 0;
        ctx->tchunks.assign(1, c);
    } else {
        ctx->tchunks.clear();
    }
    return XRT_OK;
}

int xrt_timing_events(xrt_context* ctx, double* total_ms, uint64_t* launches)
{
    if (!ctx || !total_ms || !launches) return XRT_ERR_ARGUMENT;
    *total_ms = ctx->event_ms;
    *launches = ctx->event_launches;
    return XRT_OK;
}

int xrt_render_rows(xrt_context* ctx, const xrt_camera* camera, uint32_t row_begin,
                    uint32_t row_end, float* image, float* lbuffer, uint8_t* image_u8,
                    xrt_stats* stats)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    int rc = check_camera(ctx, camera, row_begin, row_end);
    if (rc) return rc;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    double* hc = ctx->host_call_ms;
    const auto t0 = HostClock::now();
    auto lap = [&](int k, HostClock::time_point& t) {
        const auto now = HostClock::now();
        hc[k] = std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    };
    auto t = t0;
    std::fill(hc, hc + kHostCallFields, 0.0);
    double acc0[kAccFields];
    std::copy(ctx->acc_ms, ctx->acc_ms + kAccFields, acc0);
    const size_t n = (size_t)(row_end - row_begin) * camera->width;
    size_t cap_f = ctx->stage_cap, cap_l = ctx->stage_cap, cap_u = ctx->stage_cap;
    if ((rc = ensure(ctx, ctx->d_image, cap_f, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_lbuffer, cap_l, n))) return rc;
    if ((rc = ensure(ctx, ctx->d_u8, cap_u, n))) return rc;
    ctx->stage_cap = std::min(cap_f, std::min(cap_l, cap_u));
    lap(0, t);
    // the context's own non-blocking stream (not the null stream)
    rc = enqueue_render(ctx, camera, row_begin, row_end, image ? ctx->d_image : nullptr,
                        lbuffer ? ctx->d_lbuffer : nullptr, image_u8 ? ctx->d_u8 : nullptr, ctx->host_stream);
    if (rc) return rc;
    XRT_HIP(ctx, hipEventRecord(ctx->host_render_done, ctx->host_stream));
    lap(1, t);
    XRT_HIP(ctx, hipEventSynchronize(ctx->host_render_done));
    lap(2, t);
    std::vector<D2HCopy> copies;
    if (n) {
        if (image) copies.push_back({image, ctx->d_image, n * sizeof(float)});
        if (lbuffer) copies.push_back({lbuffer, ctx->d_lbuffer, n * sizeof(float)});
        if (image_u8) copies.push_back({image_u8, ctx->d_u8, n});
    }
    if ((rc = d2h_copy(ctx, ctx->host_stream, copies))) return rc;
    lap(3, t);
    double bytes = 0.0;
    for (const D2HCopy& c : copies) bytes += (double)c.bytes;
    hc[4] = ctx->pool ? (double)ctx->pool->size() : 0.0;
    hc[5] = bytes / 1e6;
    xrt_stats local;
    rc = xrt_read_stats(ctx, stats ? stats : &local);
    lap(6, t);
    hc[7] = std::chrono::duration<double, std::milli>(t - t0).count();
    for (int k = 0; k < kAccFields; ++k) hc[8 + k] = ctx->acc_ms[k] - acc0[k];
    return rc;
}

int xrt_probe_intersect(xrt_context* ctx, const float* rays, const float* tris, uint64_t n,
                        uint8_t* hit, float* t)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (n == 0) return XRT_OK;
    if (!rays || !tris || !hit || !t) return fail(ctx, XRT_ERR_ARGUMENT, "NULL buffer");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    float *dr = nullptr, *dt = nullptr, *dout = nullptr;
    uint8_t* dh = nullptr;
    int rc = XRT_OK;
    if (hipMalloc(&dr, n * 6 * sizeof(float)) != hipSuccess ||
        hipMalloc(&dt, n * 9 * sizeof(float)) != hipSuccess ||
        hipMalloc(&dout, n * sizeof(float)) != hipSuccess || hipMalloc(&dh, n) != hipSuccess) {
        rc = fail(ctx, XRT_ERR_DEVICE, "probe allocation failed");
    } else if (hipMemcpy(dr, rays, n * 6 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
               hipMemcpy(dt, tris, n * 9 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        rc = fail(ctx, XRT_ERR_DEVICE, "probe upload failed");
    } else {
        hipLaunchKernelGGL(k_probe_intersect, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dr,
                           dt, n, dh, dout);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpy(hit, dh, n, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(t, dout, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(ctx, XRT_ERR_DEVICE, "probe kernel failed");
    }
    (void)hipFree(dr);
    (void)hipFree(dt);
    (void)hipFree(dout);
    (void)hipFree(dh);
    return rc;
}

int xrt_probe_math(xrt_context* ctx, int op, const float* in, float* outp, uint64_t n)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    if (op < XRT_PROBE_EXPF || op > XRT_PROBE_SIGNED_L) return fail(ctx, XRT_ERR_ARGUMENT, "bad op");
    if (n == 0) return XRT_OK;
    if (!in || !outp) return fail(ctx, XRT_ERR_ARGUMENT, "NULL buffer");
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    float *di = nullptr, *dout = nullptr;
    int rc = XRT_OK;
    if (hipMalloc(&di, n * sizeof(float)) != hipSuccess ||
        hipMalloc(&dout, n * sizeof(float)) != hipSuccess) {
        rc = fail(ctx, XRT_ERR_DEVICE, "probe allocation failed");
    } else if (hipMemcpy(di, in, n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        rc = fail(ctx, XRT_ERR_DEVICE, "probe upload failed");
    } else {
        hipLaunchKernelGGL(k_probe_math, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, op, di,
                           dout, n);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpy(outp, dout, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(ctx, XRT_ERR_DEVICE, "probe kernel failed");
    }
    (void)hipFree(di);
    (void)hipFree(dout);
    return rc;
}

int xrt_probe_prep(xrt_context* ctx, const xrt_camera* camera, float* records, float* footprint)
{
    if (!ctx) return fail(nullptr, XRT_ERR_ARGUMENT, "context is NULL");
    int rc = check_camera(ctx, camera, 0, camera ? camera->height : 0);
    if (rc) return rc;
    XRT_HIP(ctx, hipSetDevice(ctx->device));
    const uint64_t T = ctx->num_tris;
    if (!T) return XRT_OK;
    if ((rc = sync_context(ctx))) return rc;      // no frame in flight uses the set
    FrameSet& fs = ctx->sets[ctx->next_set];
    if ((rc = ensure(ctx, fs.recs, fs.recs_cap, T))) return rc;
    if ((rc = ensure(ctx, fs.cull, fs.cull_cap, (size_t)T * kCullPlanes))) return rc;
    RenderParams p = make_params(*camera, 0, camera->height, T, ctx->hit_capacity);
    p.model = ctx->model;
    CullParams cp = make_cull_params(*camera);
    BinBuffers nobins = {};
    hipLaunchKernelGGL(k_prep, dim3((unsigned)((T + kPrepWaves * p.prep_tris - 1) / (kPrepWaves * p.prep_tris))),
                       dim3(kPrepThreads), 0, 0, ctx->d_tris,
                       (uint32_t)T, p, cp, fs.recs, fs.cull, nobins, nullptr, nullptr, nullptr, nullptr);
    XRT_HIP(ctx, hipGetLastError());
    if (records)
        XRT_HIP(ctx, hipMemcpy(records, fs.recs, T * sizeof(TriRec), hipMemcpyDeviceToHost));
    if (footprint) {
        // planes [bbox | e0 | e1 | e2] of T float4 -> per triangle 16 floats
        std::vector<float4> planes((size_t)T * kCullPlanes);
        XRT_HIP(ctx, hipMemcpy(planes.data(), fs.cull, planes.size() * sizeof(float4),
                               hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < T; ++i)
            for (int k = 0; k < kCullPlanes; ++k)
                std::memcpy(footprint + 16 * i + 4 * k, &planes[(size_t)k * T + i], sizeof(float4));
    }
    return XRT_OK;
}

// Host evaluation of the device expf restatement (same source, host-compiled);
// lets the CPU test suite check it exhaustively against libm without a GPU.
// Host evaluation of the culled tests' division-free reject (mt_may_hit) and
// of the exact remainder (mt_finish), same source: the CPU suite checks that
// the reject never drops a hit.
void xrt_host_mt_check(const float* det, const float* a, const float* b, const float* tnum, uint64_t n,
                       uint8_t* may_hit, uint8_t* hit, float* t)
{
    for (uint64_t i = 0; i < n; ++i) {
        bool h = false;
        t[i] = mt_finish(det[i], a[i], b[i], tnum[i], h);
        hit[i] = h ? 1 : 0;
        may_hit[i] = mt_may_hit(det[i], a[i], b[i], tnum[i]) ? 1 : 0;
    }
}

void xrt_host_expf_batch(const float* in, float* outp, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) outp[i] = xrt_expf(in[i]);
}

void xrt_host_exp_batch(const double* in, double* outp, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) outp[i] = xrt_exp(in[i]);
}

void xrt_host_signed_lbuffer_batch(const float* distance, const int32_t* sign_sum, float mu, float* outp,
                                   uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) outp[i] = signed_lbuffer(distance[i], sign_sum ? sign_sum[i] : 0, mu);
}

}  // extern "C"

#include "xrt_multi.inc"
