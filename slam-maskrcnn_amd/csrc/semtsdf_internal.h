// Internal interface between the C-ABI host layer (semtsdf_api.cpp) and the gfx950
// kernels (semtsdf_kernels.hip).  Plain-old-data argument blocks, passed by value as
// kernel arguments so that pose, intrinsics and volume geometry land in SGPRs.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace semtsdf {

constexpr int kMaxObjects = 32;
constexpr int kMaxDetections = 256;  // detections per frame accepted by semtsdf_masks_to_labels
constexpr int kRcpTable = 1024;  // RN(1/n) table of the running means (w + 1 <= kRcpTable)
constexpr int kZAlign = 32;      // stored z planes per x,y column: a multiple of the unit z-extent
#ifndef SEMTSDF_BRICK_DIST_CAP
#define SEMTSDF_BRICK_DIST_CAP 16
#endif
constexpr int kBrickDistCap = SEMTSDF_BRICK_DIST_CAP;  // brick distance map: radius of the largest skip box (bricks)
constexpr int kListSegs = 64;    // segments (and counters) of the live-unit list
constexpr unsigned kPreWaves = 65534;  // k_integrate reads entries 2w+1 (+4) ahead for waves w < kPreWaves
constexpr int kListCountStride = 64;  // counters 256 B apart (separate memory channels)
#ifndef SEMTSDF_DYN_SUB
#define SEMTSDF_DYN_SUB 8
#endif
constexpr unsigned kDynSub = SEMTSDF_DYN_SUB;           // integrate dynamic counters per XCD (power of two)
constexpr int kDynCounters = 8 * SEMTSDF_DYN_SUB;       // after the list counts (zeroed by the prepass)
// words of list_count: the segment counts, the dynamic counters, then the compact lists' (base, total)
constexpr int kListTotalsWord = (3 * kListSegs + kDynCounters) * kListCountStride;
constexpr int kListCountWords = kListTotalsWord + 8;
constexpr int kLists = 3;             // live-unit lists: general, free (projected), full free (no projection)

// Geometry of the locally stored part of the volume.
struct VolGeom {
    int dimx, dimy, dimz;      // global dims
    int lz;                    // local z planes (chunks * (chunk + halo))
    int zs;                    // row stride in voxels: lz rounded up to a multiple of kZAlign
    int shard, nshards, chunk, halo;
    float start[3];            // vol_start
    float end[3];              // vol_end
    float voxel[3];
    float mu;
    uint64_t nvox;             // dimx * nuy * nuz * 256: stored voxels of the tiled layout (padding included)
    uint32_t nuy, nuz;         // 8-row y groups and 32-plane z groups (one 256-voxel tile each)
    uint32_t tx, ty;           // tile-index strides of x (nuy * nuz * 256) and of y / 8 (nuz * 256)
    int nbx, nby, nbz;         // 8^3 bricks of the local storage (empty-space map)
    int nsx, nsy, nsz;         // 64^3 super-bricks (8^3 bricks each)
    float rvox[3];             // RN(1 / voxel) per axis (exact divisions by the voxel size)
};

// Tiled layout of every per-voxel array: the 1 x 8 x 32 (x, y, z) block of an integrate
// unit is 256 consecutive voxels, ordered (z/4, y, z%4).  The 4 z-neighbours of a lane are
// one 16-B vector and 8 y-rows of 4 planes fill one 128-B line, so the ends of a column's
// updated run and thin bands of gated voxels touch few lines (z-rows of 32 voxels would
// cost a whole line per row), and a trilinear sample's 8 corners span ~2 lines, not 4.
// Indices are 32-bit (the host rejects volumes of 2^32 stored voxels or more; a histogram
// plane offset k * nvox is added in 64 bits by the caller).  tx = nuy * nuz * 256 and
// ty = nuz * 256 < 2^24 (checked at create), so the y term is a full-rate 24-bit product.
__device__ inline uint32_t tile_xterm(const VolGeom& g, int x) { return (uint32_t)x * g.tx; }
__device__ inline uint32_t tile_yterm(const VolGeom& g, int y) {
    return __umul24((uint32_t)(y >> 3), g.ty) + (uint32_t)(y & 7) * 4u;
}
__device__ inline uint32_t tile_zterm(int zl) { return (uint32_t)(zl >> 5) * 256u + (uint32_t)((zl >> 2) & 7) * 32u + (uint32_t)(zl & 3); }
__device__ inline uint32_t tile_index(const VolGeom& g, int x, int y, int zl) {
    return tile_xterm(g, x) + tile_yterm(g, y) + tile_zterm(zl);
}

// Device buffers of one volume.
struct VolBufs {
    float* sdf;
    int32_t* wt;
    void* color;       // u8x4 or i32x4 per voxel (3 channels + pad)
    uint32_t* hist;    // bin-major [32][nvox]
    uint32_t* hmask;   // [nvox] bit k set when hist[k][v] > 0 (kept by the integrate; samplers
                       // interpolate only the bins set at one of their 8 corners)
    int32_t* cls;      // vote mode
    int32_t* cls_cnt;  // vote mode
    float* bmin;       // per 8^3 brick: min sdf over its voxels and the +1 border (ray skipping)
    float* bplain;     // per 8^3 brick: min sdf over its own voxels
    float* sbmin;      // per 64^3 super-brick (8^3 bricks): min of bmin over its bricks
    uint8_t* bdist;    // per 8^3 brick: L-inf distance in bricks to the nearest non-skippable
                       // brick (0: not skippable), capped at kBrickDistCap
    uint64_t* boct;    // per 8^3 brick, byte o: the same distance within octant o only (bit a of o
                       // set: negative along axis a), so a ray heading into octant o may step
                       // through the box reaching that many bricks ahead of it (bdist = the min)
    uint64_t* botmp;   // scratch of the distance passes
    uint32_t* bdirty;  // per quad of 4 z-consecutive 8^3 bricks ((bx, by, bz/4), z fastest): bit j set when
                       // a voxel of brick 4q + j crossed the skip threshold since the last map update
    uint32_t* dlist;   // [1 + quads]: count, then the quads whose dirty word is nonzero
    uint8_t* sflag;    // per 128-B sdf line (32 voxels): s >= 1 = every sdf is 1.0f and every weight
                       // < 2^23 (k_integrate skips the sdf traffic of such lines), and s - 1 increments
                       // of every weight of the line are pending (lazy weights); 0 = unknown
};

// Per-frame images of the integrate: depth in metres and rgb+label per pixel (row-major,
// W x H), and per 8- and 32-pixel tile the max raw depth (bits 0-15) and 0xFFFF - the min
// nonzero raw depth (bits 16-31; 0 when the tile has no nonzero pixel), used by the unit
// culler (dead units, and free units whose touched voxels all have f == 1).
struct DepthPyramid {
    uint2* px;      // pixel records {bits of depth / depth_scale (IEEE, tsdf.cu:49),
                    //                r | g << 8 | b << 16 | label << 24}: one 8-B gather per voxel,
                    // in 4 x 4-pixel tiles of one 128-B line each, a tile column-major (rec_index):
                    // the voxels of a unit project onto a compact patch of the image, which then
                    // spans few lines.  The record image has one more column (u = W) and row (v = H)
                    // than the frame, always zero (depth 0): off-image coordinates clamp onto them
    uint2* l0;  // [ceil(H/8)][ceil(W/8)]  {max | (0xFFFF - min nonzero) << 16, 1 if a pixel has depth 0}
    uint2* l1;  // [ceil(H/32)][ceil(W/32)]
    int w0, h0, w1, h1;
    unsigned rs;    // records per band of 4 rows: 4 * (W + 1 rounded up to a multiple of 4)
};

// Record of pixel (u, v), 0 <= u <= W, 0 <= v <= H: bands of 4 rows, in a band the 4 records of
// a column consecutive, so a 128-B line holds the 4 x 4 pixels u = 4a..4a+3, v = 4b..4b+3.
__device__ inline unsigned rec_index(const DepthPyramid& p, unsigned u, unsigned v) {
    return __umul24(v >> 2, p.rs) + ((u << 2) | (v & 3u));
}

// What the integrate reads only on its rare paths (a voxel crossing the marches' skip threshold,
// an id without a histogram bin), in device memory (one per volume, filled at create): loaded in
// those paths only, so the kernel does not hold them in scalar registers through its loop.
struct IntegrateRare {
    uint32_t* bdirty;                // VolBufs::bdirty, dlist (nullptr: no empty-space maps)
    uint32_t* dlist;
    int nby, nbz;                    // VolGeom::nby, nbz
    unsigned long long* counters;    // IntegrateArgs::counters
};

struct IntegrateArgs {
    VolGeom g;
    VolBufs b;
    float E[12];     // rows 0..2 of extrinsic2init
    float K[9];      // rows 0..2, cols 0..2 of the intrinsic
    float M[9];      // RN(K E[0:3,0:3]) (products summed in double): screen map s = M p + m
    float m[3];      // RN(K E[0:3,3])
    float cullC[16]; // cull only (conservative, not the contract): rows sx, sy, sz, qz as affine
                     // functions (cx, cy, cz, c0) of the global voxel index (x, y, gz)
    float ftol;      // 0.5 - B 2^-21, B = 2^ceil(log2(max(W, H) + 2)): exactness window of the pixel floor
    float skip_thr;  // the marches' skip threshold (skip_threshold): a voxel crossing it dirties its brick
    const float* rcp_table;        // [kRcpTable] RN(1/n), n = 1.. (volume constant)
    int width, height;
    float depth_scale;
    float gate;
    uint32_t flags;
    int cull;
    int debug;       // timing probes (SEMTSDF_DEBUG_INTEGRATE): 1 cull only, 2 skip, 3 classify only, ...
    const uint16_t* depth;
    const uint8_t* rgb;
    const uint8_t* mask;    // semantic
    const int32_t* cls;     // vote
    DepthPyramid pyr;
    unsigned long long* counters;  // [0] touched, [1] gated, [2] bad-label flag, [3] live units, [4] free units
                                   // (projected and full), [5] full free units
    int pinhole;                   // K rows are (fx 0 cx; 0 fy cy; 0 0 1)
    float rmu;                     // RN(1/mu), for the exact division by mu (k_integrate)
    int fastdiv;                   // mu in [2^-20, 2^20]: divisions by mu/(w+1) via RN reciprocals
    unsigned* unit_list;           // live units: three lists (general, free, full free) of kListSegs segments (k_cull_units)
    unsigned* list_count;          // [3][kListSegs * kListCountStride] entries per segment, then the dynamic
                                   // counters, then the compact lists' (base, total) pairs (k_compact_lists)
    unsigned* units;               // the three lists back to back (k_compact_lists), each followed by a ~0u pad
                                   // counters of the 8 XCDs (all zeroed by the frame prepass)
    int free_ok;                   // free units allowed: gated colour with gate <= 1 (f == 1 updates sdf/weight only)
    int color_wide;                // colour stored as int32 x 4 (else u8 x 4; see semtsdf_vol::color_wide)
    unsigned long long* wtrace;    // instrumentation (build with SEMTSDF_WAVE_TRACE=1, run with
                                   // SEMTSDF_WAVE_TRACE=<file>): per wave kWaveTraceWords timestamps
    unsigned wtrace_slots;         // waves wtrace holds (waves past it are not traced)
    const uint8_t* lut;            // deferred relabel of an association decision (256 bytes, device): the
                                   // pixel records carry the frame's raw labels; nullptr: none
    uint8_t* relabel_mask;         // the frame's mask, relabelled in place through lut by the kernel (nullable)
    const IntegrateRare* rare;     // rare-path fields (device memory)
    unsigned* first_tab;           // XCD split: entries of each wave's first group of its first list, two per
                                   // wave slot, written by k_compact_lists for first_nwaves persistent waves
    unsigned first_nwaves;         // integrate_pre_waves(): the integrate reads the table only at this grid
};
constexpr int kWaveTraceWords = 8;

// Association accumulators (fixed point, scale 2^28, deterministic).
constexpr double kFixScale = 268435456.0;  // 2^28
struct AssocTables {
    long long t1[kMaxObjects][kMaxObjects];   // sum over mask==m pixels of log(max(p_j/n, eps))
    long long t3[kMaxObjects][kMaxObjects];   // sum over box_n & mask==m of log(max(1-p_n/n, eps))
    long long t2[kMaxObjects];                // sum over box_n of log(max(1-p_n/n, eps))
    unsigned int c1[kMaxObjects];             // pixels with mask == m
    unsigned int c2[kMaxObjects];             // pixels with box_n
    unsigned int c3[kMaxObjects][kMaxObjects];// pixels with box_n & mask == m
    unsigned int first_px[256];               // first pixel index of each label (UINT_MAX none)
    unsigned int max_label;                   // max(mask)
    unsigned int pos_max;                     // largest positive t1 term (p > n_obs), 2^-28 fixed point,
                                              // saturating; >= 1 whenever any term was positive (0: none)
};
static_assert(sizeof(AssocTables) % 8 == 0, "AssocTables is cleared as 8-B words");

// Decision output written by the decide kernel.
struct AssocDecision {
    int max_obj_now;
    int num_objs_before;
    int num_objs_after;
    int bad_label;
    int assigned_prev[kMaxObjects];
    float assigned_prob[kMaxObjects];
    unsigned char lut[256];
    unsigned exact_rows;    // bit i: row i decided from its exact f32 pixel-order sums
    unsigned exact_missing; // bit i: row i needed them but no pixel data was given (decided from
                            // the fixed-point sums; the sharded protocol then exchanges pixels)
    unsigned reject_rows;   // bit i: the certificate shows every candidate of row i at or below
                            // 3 * prior whatever the f32 rounding (rejected without the exact path)
};

// Per-pixel association data of the last march (the exact path of the decision): for pixel k
// the bins present at its hit and its box bins (p > box_thresh), and the trilinear counts of
// the present bins, bin-major (other entries are stale: readers test the present bit).
struct AssocPixels {
    uint2* bits;   // [npx] {present, box}
    float* p;      // [kMaxObjects][npx]
};

// Scratch of the exact path: the flagged rows' f32 pixel-order sums and the decide
// kernel's last-workgroup counter (left at 0).
struct AssocExact {
    float A[kMaxObjects][kMaxObjects];
    unsigned counter;
    unsigned frames;        // decisions that took the exact path (instrumentation)
    unsigned rows;          // rows decided from exact sums, summed over frames
    unsigned pos_max;       // largest AssocTables::pos_max any decision saw (instrumentation)
};

struct DecideArgs {
    AssocTables* T;
    AssocDecision* D;
    AssocExact* X;
    int* num_objs_dev;
    float eps;              // prior_mrcnn_err_rate
    float n_obs;
    const uint8_t* mask;    // the frame's raw labels (the rows of the sums)
    AssocPixels px;         // bits == nullptr: no pixel data (exact_missing)
    int npx;
    int force_exact;        // debug/tests: every present row takes the exact path
    int id_policy;          // 0: new ids num_objs++ as tsdf.cu:379-383 (ids >= 32 get no histogram bin);
                            // 1 (SEMTSDF_F_ID_SATURATE): new ids >= 32 become 0 (background)
    int certify_only;       // write the rows needing the exact path to D->exact_missing, decide nothing
    const unsigned* tile_cost;  // tile_n > 0: an extra workgroup orders the fused march's tiles by cost
    unsigned* tile_perm;
    int tile_n;
};

struct MarchCamera {
    float Kinv[9];   // 3x3 part of the inverse intrinsic
    float Rt[9];     // R^T of extrinsic2init (association) or identity (render)
    float o[3];      // ray origin
    // render: s2w rows 0..2 (4 cols); association uses Kinv/Rt
    float s2w[12];
    int use_s2w;
};

struct AssocArgs {
    VolGeom g;
    VolBufs b;
    MarchCamera cam;
    int width, height;
    float n_obs;
    float eps;          // prior_mrcnn_err_rate
    float box_thresh;
    const uint8_t* mask;
    AssocTables* tables;
    float* probs_out;       // optional debug [H*W*32]
    uint8_t* box_out;       // optional debug [H*W*32]
    AssocPixels px;         // per-pixel data for the decision's exact path (bits == nullptr: none)
    int debug;              // timing probes (SEMTSDF_DEBUG_ASSOC): 1 no accumulation, 2 no march
    // k_march_fused launch order (heaviest tiles of the previous frame first): the kernel
    // writes each tile's duration to tile_cost[tile] and takes block b's tile from tile_perm[b]
    // (nullptr: identity); the next decision computes the next order (DecideArgs::tile_*)
    unsigned* tile_cost;
    const unsigned* tile_perm;
};

struct RenderArgs {
    VolGeom g;
    VolBufs b;
    MarchCamera cam;
    int width, height;
    int mode;
    int color_i32;
    const uint8_t* palette;  // [32*3] RGB, written BGR
    uint8_t* out_bgr;
    float* out_t;
    unsigned* ray_stats;     // instrumentation (SEMTSDF_RAY_STATS): per pixel iterations, lookups,
                             // evaluations, skipped samples; per wave start/end ticks after them
    int row0, row1;          // instrumentation (SEMTSDF_RENDER_ROWS): only 16-px tile rows [row0, row1)
};

// Z-sharded raycast protocol (k_shard_* in semtsdf_kernels.hip): per-pixel march state.
struct ShardRayState {
    int* k;      // global coarse event index, -1 = miss
    float* fk;   // sample value at the coarse event
    int* j;      // fine hit index (0 = hit in the coarse phase)
    float* fj;   // sample value at the fine hit
    float* fp;   // sample value before the hit
    float* t;    // refined hit t, -1 = miss
};

constexpr int kAssocPartialLen = 3 * kMaxObjects * kMaxObjects + 3 * kMaxObjects;  // int64 words

struct ShardRayArgs {
    VolGeom g;
    VolBufs b;
    MarchCamera cam;
    int width, height;
    int kind;                 // 0 label render, 1 colour render, 2 association
    int step;                 // 0..2 (k_shard_ray_step)
    const int2* gathered;     // [nrec][npx] records of the previous step ({value, key} each)
    int nrec;                 // records per pixel in gathered: nshards (all-gather) or 1 (all-reduce MIN)
    int2* send;               // [npx] this shard's records
    ShardRayState st;
    int color_i32;
    const uint8_t* palette;
    uint8_t* out_bgr;
    float* out_t;
    const uint8_t* mask;
    float n_obs, eps, box_thresh;
    long long* partial;       // [kAssocPartialLen]
};

// ---- launchers (semtsdf_kernels.hip) ----
hipError_t launch_shard_ray_step(const ShardRayArgs& a, hipStream_t s);
hipError_t launch_shard_render_final(const ShardRayArgs& a, hipStream_t s);
hipError_t launch_shard_render_finish(const ShardRayArgs& a, hipStream_t s);
hipError_t launch_shard_assoc_partial(const ShardRayArgs& a, hipStream_t s);
hipError_t launch_shard_assoc_pixels(const ShardRayArgs& a, int32_t* out, hipStream_t s);
hipError_t launch_tables_from_partial(const long long* reduced, AssocTables* t, hipStream_t s);
hipError_t launch_copy_f4(const void* src, void* dst, size_t n16, hipStream_t s);
hipError_t launch_min_i64(long long* dst, const long long* src, size_t n, hipStream_t s);
// detector masks [npx][n] (bytes) -> u8 labels (dmask.py:34-59); scratch of mask_scratch_bytes()
hipError_t launch_masks_to_labels(const uint8_t* masks, int npx, int n, int min_area, void* scratch, uint8_t* out,
                                  hipStream_t s);
size_t mask_scratch_bytes();
size_t mask_scratch_kept_offset();
// global_passes: the octant maps by k_brick_dilate + k_brick_oct_axis, else by the LDS line
// passes (k_brick_oct_lds); both give the same maps.
hipError_t launch_brick_min(const VolGeom& g, const VolBufs& b, bool all, hipStream_t s, bool global_passes = false);
hipError_t launch_fill_volume(const VolGeom& g, const VolBufs& b, uint32_t flags, hipStream_t s);
hipError_t launch_flush_lazy(const VolGeom& g, const VolBufs& b, hipStream_t s);  // lazy weights -> weights
hipError_t launch_depth_pyramid(const uint16_t* depth, const uint8_t* rgb, uint8_t* mask, int w, int h,
                                float scale, const DepthPyramid& p, unsigned* list_count, hipStream_t s,
                                const uint8_t* lut = nullptr);  // lut: relabel the mask in place (k_relabel folded in)
hipError_t launch_vox_chunk(const void* src, void* dst, bool to_ref, const VolGeom& g, uint64_t v0, uint64_t nv,
                            hipStream_t s);
hipError_t launch_color_widen(const uint8_t* narrow, int32_t* wide, uint64_t nvox, hipStream_t s);  // u8x4 -> i32x4
hipError_t launch_color_chunk(const void* src, void* dst, bool to_ref, bool ref_i32, bool dev_i32, const VolGeom& g,
                              uint64_t v0, uint64_t nv, hipStream_t s);
hipError_t launch_integrate(const IntegrateArgs& a, hipStream_t s, hipEvent_t e0 = nullptr,
                            hipEvent_t e1 = nullptr);  // e0/e1: kernel start/end events (timing)
uint64_t unit_count(const VolGeom& g);
uint64_t unit_list_capacity(const VolGeom& g);
int unit_grid_fits(int dimx, int dimy, int local_z);  // list entries (pack_unit) hold the unit grid
hipError_t launch_cull(const IntegrateArgs& a, hipStream_t s);       // per-unit cull flags
hipError_t launch_compact_lists(const IntegrateArgs& a, hipStream_t s);  // segments -> a.units
unsigned integrate_pre_waves();  // persistent waves of the bench-mode integrate (first-group table size)
hipError_t launch_tables_init(AssocTables* t, hipStream_t s);  // zero sums, first_px = UINT_MAX
hipError_t launch_mask_stats(const uint8_t* mask, int npx, AssocTables* t, hipStream_t s);
hipError_t launch_assoc_march(const AssocArgs& a, hipStream_t s);
hipError_t launch_assoc_decide(const DecideArgs& a, hipStream_t s);
// reference filter_overlaps input (probs [npx][32] f32, box [npx][32] u8, tsdf.cu:304) -> the
// tables and per-pixel data the march would leave (mask statistics included)
hipError_t launch_assoc_from_probs(const float* probs, const uint8_t* box, const uint8_t* mask, int npx, float n_obs,
                                   float eps, AssocTables* t, AssocPixels px, hipStream_t s);
// the association's f32 log / exp (semtsdf_libm.h) over n values (fn 0: logf, 1: expf)
hipError_t launch_libm_eval(int fn, const float* x, float* y, size_t n, hipStream_t s);
hipError_t launch_first_frame_objs(const AssocTables* t, int* num_objs_dev, hipStream_t s);
hipError_t launch_relabel(uint8_t* mask, int npx, const AssocDecision* d, hipStream_t s);
hipError_t launch_relabel_records(uint8_t* mask, int w, int h, const DepthPyramid& p, const AssocDecision* d, hipStream_t s);
hipError_t launch_render(const RenderArgs& a, hipStream_t s);
// Work of the frame folded into the fused march's launch (blocks before the march tiles): nms
// blocks of mask statistics (k_mask_stats) and npy = pyr.w1 * pyr.h1 prepass tiles
// (k_depth_pyramid, raw labels); nms = npy = 0: none.
struct FramePre {
    const uint8_t* mask;
    int npx;
    AssocTables* T;
    int nms;
    const uint16_t* depth;
    const uint8_t* rgb;
    uint8_t* pmask;
    int w, h;
    float scale;
    int vec;
    DepthPyramid pyr;
    unsigned* list_count;
    int npy;
};
hipError_t launch_march_fused(const AssocArgs& aa, const RenderArgs& ra, const FramePre& pre, hipStream_t s);
int depth_pyramid_vec(const uint16_t* depth, const uint8_t* rgb, const uint8_t* mask, int w, const DepthPyramid& p);
hipError_t launch_copy_host(const void* src, void* dst, size_t n16, hipStream_t s);
// chunk [v0, v0+nv) of the bin-major histogram <-> voxel-major [nv][32] staging buffer
hipError_t launch_hist_chunk_to_vm(const uint32_t* bm, uint32_t* vm, const VolGeom& g, uint64_t v0, uint64_t nv,
                                   hipStream_t s);
hipError_t launch_hist_chunk_to_bm(const uint32_t* vm, uint32_t* bm, const VolGeom& g, uint64_t v0, uint64_t nv,
                                   hipStream_t s);
hipError_t launch_hist_mask(const VolGeom& g, const VolBufs& b, hipStream_t s);  // hmask from hist
struct SurfacePoint {  // one exported surface voxel (semtsdf_surface_point)
    uint32_t x, y, z;  // global voxel index
    float sdf;
    uint32_t rgbl;     // r | g << 8 | b << 16 | label << 24
};
hipError_t launch_export_surface(const VolGeom& g, const VolBufs& b, float sdf_max, int min_w, int color_wide,
                                 int semantic, SurfacePoint* out, uint64_t cap, unsigned long long* count, hipStream_t s);

}  // namespace semtsdf
