/*
 * semtsdf.h — C ABI of the MI355X-native semantic TSDF engine (libsemtsdf.so).
 *
 * This is the drop-in boundary for the fusion hot path of qq456cvb/SLAM-MaskRCNN:
 *   - the C++ class `TSDF` of src/SfM_CUDA (tsdf.cuh:7-67, tsdf.cu:137-540) and the
 *     `Viewer` raycast (viewer.cu:17-179), and
 *   - the pybind11 extension `tsdf_cuda.tsdf_update` of src/TSDF_Python
 *     (tsdf.cpp:11-33, module tsdf.cpp:35-37).
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and returns an
 * `int` status (SEMTSDF_OK == 0).  On failure `semtsdf_last_error()` returns a
 * thread-local message.  Host pointers are borrowed for the duration of the call; the
 * library owns all device memory it allocates.  `stream` arguments are `hipStream_t`
 * passed as `void*` (NULL = the handle's own stream).
 *
 * Volume layout at this boundary (TSDF_Python tsdf.py:48-52, SfM tsdf.cu:55): flat
 *   x-major, z fastest, idx = x*Dy*Dz + y*Dz + z.  sdf f32, weight i32, colour u8x3 (SfM)
 *   or i32x3 (TSDF_Python), histogram 32 x u32 per voxel.  The device storage is private:
 *   1x8x32 tiles of 256 voxels, histogram bin-major;
 *   semtsdf_download()/semtsdf_upload() convert to and from the reference layouts.
 */
#ifndef SEMTSDF_H
#define SEMTSDF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEMTSDF_ABI_VERSION 12
#define SEMTSDF_MAX_OBJECTS 32 /* tsdf.cuh:4 */

/* ---- status codes ------------------------------------------------------------ */
#define SEMTSDF_OK 0
#define SEMTSDF_ERR_INVALID (-1)     /* bad argument, shape or parameter */
#define SEMTSDF_ERR_HIP (-2)         /* a HIP runtime call failed (message has the HIP error) */
#define SEMTSDF_ERR_OOM (-3)         /* device allocation failed */
#define SEMTSDF_ERR_LABEL (-4)       /* a mask label >= SEMTSDF_MAX_OBJECTS (tsdf.cu:61 UB in the reference) */
#define SEMTSDF_ERR_STATE (-5)       /* call out of order (e.g. raycast on a sharded handle) */
#define SEMTSDF_ERR_COMM (-6)        /* collective failure */
#define SEMTSDF_ERR_UNSUPPORTED (-7) /* feature not available for this handle/mode */
#define SEMTSDF_NEED_PIXELS 1        /* semtsdf_shard_assoc_apply: the decision needs the per-pixel
                                        data of every shard (semtsdf_shard_assoc_pixels) */

/* ---- volume flags -------------------------------------------------------------- */
#define SEMTSDF_F_SEMANTIC 0x1u   /* 32-bin per-voxel instance histogram (SfM tsdf.cu:61) */
#define SEMTSDF_F_GATE_COLOR 0x2u /* colour+histogram only when f < gate (SfM tsdf.cu:57) */
#define SEMTSDF_F_COLOR_I32 0x4u  /* colour int32x3 (TSDF_Python tsdf.py:50) instead of u8x3 */
#define SEMTSDF_F_VOTE 0x8u       /* label vote tsdf_cls/tsdf_cls_cnt (TSDF_Python/tsdf.cu:48-57) */
#define SEMTSDF_F_NO_CULL 0x10u   /* disable brick frustum/depth culling (debug; same results) */
/* Instance ids past the histogram (a deviation, opt-in).  The reference hands every unmatched
 * label the id num_objs++ (tsdf.cu:379-383) without a bound, and its integrate then counts an
 * id >= 32 in the bins of the next voxel (tsdf.cu:61, out of bounds).  By default the engine
 * keeps the reference's ids (the u8 mask holds them modulo 256, as mask_ptr[i] = num_objs does),
 * drops the histogram votes of ids >= 32 (counted in semtsdf_state::label_votes_dropped) and
 * reports SEMTSDF_ERR_LABEL from the synchronous calls of the frame that minted one; the handle
 * stays usable.  With SEMTSDF_F_ID_SATURATE an unmatched label that would get an id >= 32 is
 * relabelled 0 (background) instead, num_objs stops at 32 and no error is reported. */
#define SEMTSDF_F_ID_SATURATE 0x20u

/* ---- placement modes (a1) ---------------------------------------------- */
#define SEMTSDF_PLACE_SFM 0    /* SfM tsdf.cu:173-199: f32, depth->u8 saturates, mean in metres */
#define SEMTSDF_PLACE_PYTHON 1 /* TSDF_Python tsdf.py:32-47: f64, depth->u8 wraps mod 256 */

/* ---- raycast render modes (a8) ------------------------------------------------------ */
#define SEMTSDF_RENDER_LABEL 0 /* argmax instance -> palette BGR (viewer.cu:71-79) */
#define SEMTSDF_RENDER_COLOR 1 /* trilinear colour at the hit (tsdf_render.frag:125-131) */

typedef struct semtsdf_params {
    int32_t dim[3];          /* global volume dims (Dx, Dy, Dz); reference: 256^3 (tsdf.cuh:52) */
    float vol_start[3];      /* world position of voxel (0,0,0) (tsdf.cu:195) */
    float vol_end[3];        /* world position of voxel (D-1) (tsdf.cu:196) */
    float voxel[3];          /* (vol_end - vol_start)/(D-1) (tsdf.cu:197) */
    float mu;                /* truncation, 5*voxel.x (tsdf.cu:199) */
    float K[16];             /* row-major 4x4 intrinsic (tsdf.cu:143-146) */
    float Kinv[16];          /* its inverse (tsdf.cu:147) */
    int32_t width, height;   /* frame size (640x480) */
    float depth_scale;       /* raw depth units per metre: 5000 (tsdf.cu:49) */
    float gate;              /* colour/histogram gate on f: 0.99 (tsdf.cu:57) */
    float box_thresh;        /* association box-mask threshold: 0.3 (tsdf.cu:128) */
    float prior_mrcnn_err_rate; /* Configuration::prior_mrcnn_err_rate = 0.05 (configuration.h:8);
                                   must lie in [2^-10, 1) */
    float duplicate_thresh;  /* Configuration::duplicate_thresh = 0.5 (configuration.h:9; unused upstream) */
    uint32_t flags;          /* SEMTSDF_F_* */
    /* Z-slab sharding.  The global z axis is cut into chunks of z_chunk
     * planes, dealt round by round in boustrophedon order: with n = z_nshards, chunk c of
     * round r = c / n, position k = c % n, is owned by shard k (r even) or n - 1 - k (r odd).
     * z_nshards == 1 -> whole volume
     * (z_chunk is then ignored).  Sharded handles store one extra halo plane per chunk. */
    int32_t z_shard, z_nshards, z_chunk;
} semtsdf_params;

typedef struct semtsdf_vol semtsdf_vol; /* opaque volume handle */

typedef struct semtsdf_state {
    uint32_t n_obs;          /* integrated frames used by association (tsdf.cuh:46) */
    int32_t num_objs;        /* next global instance id (tsdf.cuh:61) */
    int32_t local_dim[3];    /* stored dims on this device (z includes halo planes) */
    uint64_t local_voxels;   /* local_dim product */
    uint64_t device_bytes;   /* bytes of device memory owned by the handle */
    uint64_t label_votes_dropped; /* histogram votes of ids >= 32 dropped by the integrate since the
                                     last reset: the id policy without SEMTSDF_F_ID_SATURATE (with
                                     the flag no such id is minted and this stays 0) */
} semtsdf_state;

/* Per-frame association result (filter_overlaps tsdf.cu:304-416). */
typedef struct semtsdf_assoc_stats {
    int32_t max_obj_now;                /* max(mask)+1 of the incoming mask */
    int32_t num_objs;                   /* after relabel */
    int32_t assigned_prev[SEMTSDF_MAX_OBJECTS]; /* current label i -> previous id, or -1 */
    float assigned_prob[SEMTSDF_MAX_OBJECTS];   /* exp(A/C) of the accepted match */
    uint8_t lut[256];                   /* old label -> new label applied to the mask */
    uint32_t exact_rows;                /* bit i: current label i was decided from its exact f32
                                           pixel-order sums (the rows the fixed-point certificate
                                           could not decide) */
    uint32_t reject_rows;               /* bit i: the certificate proved every candidate of label i
                                           at or below 3 * prior for every f32 rounding of its sums:
                                           rejected (a new id) without the exact path */
} semtsdf_assoc_stats;

/* Accumulated kernel timings (HIP events on the launch stream). */
typedef struct semtsdf_timing {
    double integrate_ms;  /* sum over integrate kernel launches */
    double assoc_ms;      /* sum over association (march+accumulate+decide+relabel) */
    double render_ms;     /* sum over raycast render launches */
    uint64_t n_integrate, n_assoc, n_render;
    uint64_t touched;     /* voxels updated (count mode only) */
    uint64_t gated;       /* voxels whose colour/histogram were updated (count mode only) */
    uint64_t bricks;      /* integrate units that survived the frustum/depth cull (count mode only) */
    double prep_ms;       /* sum over the per-frame depth-pyramid + brick-cull passes */
    uint64_t n_prep;
    uint64_t free_units;  /* of those, units whose touched voxels all have f == 1 (count mode only) */
    uint64_t full_units;  /* of those, free units whose every voxel is touched (no projection; count mode only) */
    uint64_t lazy_voxels; /* touched voxels of steady lines whose +1 weight went to the line's pending count
                             instead of a weight store (count mode only) */
    uint64_t assoc_exact_frames; /* association decisions that took the exact f32 path (always counted) */
    uint64_t assoc_exact_rows;   /* rows decided on it, summed over those decisions */
    uint64_t touched_lines;      /* 128-B lines of the sdf array (8 y x 4 z voxels of a tile) holding a
                                    touched voxel: the line-granular floor of the state traffic (count mode only) */
    double assoc_pos_max;        /* largest positive association term log(p / n_obs) any decision saw
                                    (p > n_obs; 0: none); from log 32 on every row takes the exact path */
} semtsdf_timing;

/* ---- library ------------------------------------------------------------------------ */
const char* semtsdf_last_error(void);
int semtsdf_abi_version(void);
/* SHA-256 (hex) of the sources, hipcc flags and compiler version the library was built from
 * (__graft_entry__.build_key): the key PMC traffic records are stamped with. */
const char* semtsdf_build_key(void);
int semtsdf_device_count(int* out);
int semtsdf_set_device(int device);
int semtsdf_stream_create(void** out_stream);
int semtsdf_stream_destroy(void* stream);
int semtsdf_stream_sync(void* stream);
int semtsdf_dev_malloc(void** out, size_t bytes);
int semtsdf_dev_free(void* ptr);
/* kind: 1 = host->device, 2 = device->host, 3 = device->device (async on stream);
 * 4 = a copy kernel on stream reading a device-accessible source (pinned host memory),
 *     16-B aligned pointers and size: does not block the calling thread */
int semtsdf_memcpy(void* dst, const void* src, size_t bytes, int kind, void* stream);

/* ---- parameters / placement (a1) --------------------------------------------------- */
/* Fill defaults: K from (fx, fy, cx, cy) as tsdf.cu:137-147, constants of §a10, cubic dim. */
int semtsdf_params_default(semtsdf_params* p, int dim, const float intrinsics[4], int width, int height);
/* Place the volume from the first frame's depth (tsdf.cu:173-199 / tsdf.py:32-47).
 * mean_depth is in metres for SEMTSDF_PLACE_SFM and in raw depth units for
 * SEMTSDF_PLACE_PYTHON (tsdf.py:38-40). Writes vol_start, vol_end, voxel, mu. */
int semtsdf_place_from_frame(semtsdf_params* p, const uint16_t* depth, double mean_depth, int mode);

/* ---- volume lifecycle ------------------------------------------------------------- */
int semtsdf_create(const semtsdf_params* p, int device, semtsdf_vol** out);
int semtsdf_destroy(semtsdf_vol* v);
int semtsdf_get_params(const semtsdf_vol* v, semtsdf_params* out);
int semtsdf_get_state(const semtsdf_vol* v, semtsdf_state* out);
int semtsdf_set_state(semtsdf_vol* v, uint32_t n_obs, int32_t num_objs);
void* semtsdf_get_stream(const semtsdf_vol* v);
/* sdf := mu (metres, tsdf.cu:243-244), weight/colour/histogram := 0, n_obs = num_objs = 0. */
int semtsdf_reset(semtsdf_vol* v, void* stream);

/* ---- integrate (a4) ------------------------------------------------------------------
 * One frame into the volume: E = extrinsic * init_extrinsic_inv (row-major 4x4 f32,
 * tsdf.cu:217).  depth u16 [H*W], rgb u8 [H*W*3], mask u8 [H*W] (may be NULL unless
 * SEMANTIC).  In a SEMANTIC volume every integrated frame is an observation, as every
 * integrated frame of the reference advances n_obs_ (tsdf.cu:218-220): the first one (n_obs ==
 * 0) sets num_objs = max(mask) + 1 (tsdf.cu:463-468), and each one advances n_obs by 1, so
 * semtsdf_associate + semtsdf_integrate leave the state semtsdf_parse_frame leaves (ABI 12; up
 * to ABI 11 only parse_frame advanced n_obs).  Mask labels >= 32: without
 * SEMTSDF_F_ID_SATURATE their histogram votes are dropped and counted and the host-pointer
 * call reports SEMTSDF_ERR_LABEL after applying the frame in full; with it they are refused
 * (SEMTSDF_ERR_LABEL, nothing applied). */
int semtsdf_integrate(semtsdf_vol* v, const uint16_t* depth, const uint8_t* rgb,
                      const uint8_t* mask, const float E[16], void* stream);
/* Same with device pointers (inputs already resident in HBM). */
int semtsdf_integrate_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d,
                          const uint8_t* mask_d, const float E[16], void* stream);
/* As semtsdf_integrate_dev, with the frame prepass (pixel records, depth pyramid, unit
 * cull) on the volume's own prep stream, ordered only after inputs_ready (a hipEvent_t
 * marking the inputs complete; NULL: the inputs are already complete) and after the
 * integrate two frames back -- not after the earlier work of `stream` -- so it overlaps the
 * previous frame's integrate.  The integrate itself is ordered on `stream` as usual.  The
 * inputs must stay unchanged until this frame's integrate has run. */
int semtsdf_integrate_dev_async(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d,
                                const uint8_t* mask_d, const float E[16], void* inputs_ready, void* stream);
/* Label-vote mode input (TSDF_Python/tsdf.cu:48-57): cls is int32 [H*W]. */
int semtsdf_integrate_vote_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d,
                               const int32_t* cls_d, const float E[16], void* stream);

/* ---- association (a5 + a6) -----------------------------------------------------------
 * Raycast the volume from the current camera (back_proj_kernel tsdf.cu:72-135), fuse the
 * 32x32 log-likelihood accumulation on device, decide assignments (tsdf.cu:337-389) and
 * relabel the mask in place.  Requires n_obs > 0 (tsdf.cu:426).  Host-pointer variant
 * copies the mask in and the relabelled mask back out; stats may be NULL. */
int semtsdf_associate(semtsdf_vol* v, uint8_t* mask_inout, const float E[16],
                      semtsdf_assoc_stats* stats, void* stream);
int semtsdf_associate_dev(semtsdf_vol* v, uint8_t* mask_d, const float E[16],
                          semtsdf_assoc_stats* stats_host_or_null, void* stream);
/* Debug/parity: per-pixel probs [H*W*32] f32 and box_mask [H*W*32] u8 exactly as the
 * reference back_proj_kernel leaves them (zeros where no hit).  Host outputs. */
int semtsdf_assoc_probs(semtsdf_vol* v, const float E[16], float* probs, uint8_t* box_mask, void* stream);
/* TSDF::filter_overlaps (tsdf.cu:304-416) on given inputs: probs_d f32 [H*W][32], box_d u8
 * [H*W][32] (nonzero = set), mask_d u8 [H*W] relabelled in place; n_obs, num_objs and the
 * knobs of the handle (n_obs > 0).  The decision the association march feeds, on the
 * reference's own function boundary (device pointers; async unless stats is given). */
int semtsdf_filter_overlaps_dev(semtsdf_vol* v, const float* probs_d, const uint8_t* box_d, uint8_t* mask_d,
                                semtsdf_assoc_stats* stats_host_or_null, void* stream);
/* The association's f32 logf (fn 0) / expf (fn 1) on the device over n values (device
 * pointers): the host C library's results bit for bit (semtsdf_libm.h), for verification;
 * fn 2: the device's own logf, which the march's fixed-point sums use (within the
 * certificate's slack of the host's). */
int semtsdf_libm_eval(int fn, const float* x_d, float* y_d, size_t n, void* stream);

/* ---- per-frame driver (a7: TSDF::parse_frame/launch_kernel tsdf.cu:171-228,418-504) ----
 * Integrated-frame count n_obs: if n_obs > 0 associate (relabels mask), else
 * num_objs = max(mask)+1; then integrate; n_obs++.  Placement is the caller's job
 * (semtsdf_place_from_frame + semtsdf_create). */
int semtsdf_parse_frame(semtsdf_vol* v, const uint16_t* depth, const uint8_t* rgb,
                        uint8_t* mask_inout, const float E[16], semtsdf_assoc_stats* stats, void* stream);
int semtsdf_parse_frame_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d,
                            uint8_t* mask_d, const float E[16], void* stream);
/* parse_frame_dev whose integrate (the frame's only write of the volume) first waits for
 * `integrate_after_event` (a hipEvent_t, or NULL), e.g. the end of the previous frame's live
 * render on another stream; the association, which only reads the volume, may overlap it. */
int semtsdf_parse_frame_dev_after(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d,
                                  uint8_t* mask_d, const float E[16], void* integrate_after_event, void* stream);
/* parse_frame_dev plus one live view (semtsdf_raycast_dev arguments) of the volume as it
 * stands BEFORE this frame -- the view Viewer::show_tsdf shows after the previous frame
 * (kernel.cpp:96-107) -- rendered in the same launch as this frame's association march: both
 * read that state and both are bound by their slowest rays, so each fills the other's tail.
 * Without an association (first frame, non-semantic volume) the view is rendered first, alone.
 * out_bgr_d / out_t_d are written by the time the frame's work on `stream` completes. */
int semtsdf_parse_frame_view_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d,
                                 uint8_t* mask_d, const float E[16], const float s2w[16], const float c[3],
                                 int mode, uint8_t* out_bgr_d, float* out_t_d, void* stream);

/* ---- raycast render (a8: Viewer::show_tsdf viewer.cu:137-179) -------------------------
 * Orbit camera helper: s2w = rot(angle, dist) * Kinv, c = ((dist+0.5) sin, 0, (dist+0.5)(1-cos)). */
int semtsdf_orbit_camera(const float Kinv[16], float angle, float dist, float s2w[16], float c[3]);
/* out_bgr u8 [H*W*3] (host) black where nothing is hit; out_t f32 [H*W] (host, optional)
 * refined hit distance or -1. */
int semtsdf_raycast(semtsdf_vol* v, const float s2w[16], const float c[3], int mode,
                    uint8_t* out_bgr, float* out_t, void* stream);
int semtsdf_raycast_dev(semtsdf_vol* v, const float s2w[16], const float c[3], int mode,
                        uint8_t* out_bgr_d, float* out_t_d, void* stream);

/* ---- Z-sharded raycast (replaces the single-GPU back_proj_kernel
 * tsdf.cu:72-135 and show_tsdf_kernel viewer.cu:17-86 when the volume is split across GPUs)
 * Every shard of a group runs the same call sequence.  Between calls the host exchanges
 * the per-pixel `send` records (record_bytes each) of all shards into `gathered` (device
 * memory) as `exchange` says (SEMTSDF_EXCHANGE_*):
 *   begin(kind, cam, c, exchange, &rec, &nsteps)
 *   for s in 0..nsteps-1:  step(s, s ? gathered : NULL, send);  all-gather send -> gathered
 *   kind RENDER_*:  render_finish(gathered, out_bgr, out_t)   -- all-gathered composite
 *   kind RAY_ASSOC: assoc_partial(gathered, mask, partial);    all-reduce(SUM) partial;
 *                   assoc_apply(reduced, mask, stats)         -- decide + relabel
 * The result is bit-identical to the single-volume raycast / association. */
#define SEMTSDF_RAY_ASSOC 2
#define SEMTSDF_ASSOC_PARTIAL_LEN 3168 /* int64 words: 32x32 t1, t3; 32 t2, c1, c2; 32x32 c3
                                         (the unused c1[0] word: the largest positive term) */
/* exchange between protocol steps: every shard's records concatenated in shard order
 * (all-gather; gathered = z_nshards * record_bytes), or their element-wise minimum as
 * little-endian int64 (all-reduce MIN; gathered = record_bytes), 1/z_nshards of the bytes. */
#define SEMTSDF_EXCHANGE_ALLGATHER 0
#define SEMTSDF_EXCHANGE_MIN 1
int semtsdf_shard_ray_begin(semtsdf_vol* v, int kind, const float cam[16], const float c[3], int exchange,
                            size_t* record_bytes, int* nsteps);
int semtsdf_shard_ray_step(semtsdf_vol* v, int step, const void* gathered_d, void* send_d, void* stream);
int semtsdf_shard_render_finish(semtsdf_vol* v, const void* gathered_d, uint8_t* out_bgr_d, float* out_t_d,
                                void* stream);
int semtsdf_shard_assoc_partial(semtsdf_vol* v, const void* gathered_d, const uint8_t* mask_d,
                                int64_t* partial_d, void* stream);
int semtsdf_shard_assoc_apply(semtsdf_vol* v, const int64_t* reduced_d, uint8_t* mask_d,
                              semtsdf_assoc_stats* stats, void* stream);
/* When assoc_apply returns SEMTSDF_NEED_PIXELS (some labels are too close to call from the
 * reduced fixed-point sums; nothing was decided or relabelled):
 *   assoc_pixels(gathered, px): this shard's per-pixel association data, zeros for pixels it
 *       does not own; all-reduce(SUM, int32) px over the group;
 *   assoc_apply_exact(reduced, px_reduced, mask, stats): decide + relabel.
 * px: SEMTSDF_ASSOC_PIXEL_WORDS int32 words per pixel (device memory). */
#define SEMTSDF_ASSOC_PIXEL_WORDS 34
int semtsdf_shard_assoc_pixels(semtsdf_vol* v, const void* gathered_d, int32_t* px_d, void* stream);
int semtsdf_shard_assoc_apply_exact(semtsdf_vol* v, const int64_t* reduced_d, const int32_t* px_d, uint8_t* mask_d,
                                    semtsdf_assoc_stats* stats, void* stream);
/* dst[i] = min(dst[i], src[i]) over n int64 (device, async on stream): the exchange
 * SEMTSDF_EXCHANGE_MIN for shards driven from one process. */
int semtsdf_min_i64(int64_t* dst_d, const int64_t* src_d, size_t n, void* stream);
/* parse_frame for a sharded handle: the host runs the association protocol above (when
 * n_obs > 0), then integrate_dev (which advances n_obs and sets the first frame's object count).
 * note_integrated did that up to ABI 11; it is kept as a no-op that checks its handle. */
int semtsdf_shard_note_integrated(semtsdf_vol* v, const uint8_t* mask_d, void* stream);

/* ---- mask producer contract --------------------------------------
 * Detector output -> the u8 instance-label mask the fusion consumes, as Mask_RCNN/dmask.py's
 * mask_detect (dmask.py:47-59, without the optional depth filter that mask_process.py does
 * not use): detection i is kept when its area > min_area (filter_tiny_objects, 2000 in the
 * reference), a pixel belongs to the smallest kept detection containing it (preserve_small_objs;
 * equal areas: the lower index), labelled 1 + its index among the kept ones.
 * masks_d: bytes [height][width][n] (nonzero = inside; the detector's masks[H, W, N]),
 * labels_d: u8 [height * width]; 0 <= n <= 256; device pointers, async on stream.
 * n_kept (optional, host) receives the number of kept detections (synchronises). */
int semtsdf_masks_to_labels(const uint8_t* masks_d, int width, int height, int n, int min_area,
                            uint8_t* labels_d, int* n_kept, void* stream);

/* Achievable HBM bandwidth on `device` (GB/s, read + write bytes) of a float4 device copy
 * of `bytes` bytes, best of `reps` runs: the practical ceiling beside the 8 TB/s spec peak. */
int semtsdf_copy_bandwidth(int device, size_t bytes, int reps, double* gbs);

/* ---- state transfer (parity, checkpoint/resume) ------------------------------------------
 * Reference layouts, local storage (for an unsharded handle: the whole volume).  Any
 * pointer may be NULL.  color is u8 [N*3] or i32 [N*3] per SEMTSDF_F_COLOR_I32; hist is
 * voxel-major u32 [N*32] (tsdf.cu:249); cls/cls_cnt i32 [N] (vote mode). */
int semtsdf_download(semtsdf_vol* v, float* sdf, int32_t* wt, void* color, uint32_t* hist,
                     int32_t* cls, int32_t* cls_cnt);
/* The x-planes [x0, x1) only, same layouts (arrays sized (x1-x0) * Dy * local Dz [* 3 | * 32]):
 * checks of volumes too large to download whole (a 1024^3 histogram is 128 GiB). */
int semtsdf_download_slab(semtsdf_vol* v, int x0, int x1, float* sdf, int32_t* wt, void* color,
                          uint32_t* hist, int32_t* cls, int32_t* cls_cnt);
int semtsdf_upload(semtsdf_vol* v, const float* sdf, const int32_t* wt, const void* color,
                   const uint32_t* hist, const int32_t* cls, const int32_t* cls_cnt);

/* ---- surface export (no reference counterpart) -------------------------
 * Every stored voxel of this handle (a shard: its owned planes) with weight >= min_weight and
 * |sdf| < sdf_max (sdf in the volume's normalised units, f = diff / mu), in the reference's flat
 * order (x-major, z fastest; global indices), with its colour (int32 colours clamped to [0, 255])
 * and instance label (the argmax of its histogram, first maximum; 0 without a count).  out may
 * be NULL (count only); otherwise it receives min(count, capacity) points.  Synchronises. */
typedef struct semtsdf_surface_point {
    uint32_t x, y, z; /* voxel index; position = vol_start + index * voxel (tsdf.cu:30) */
    float sdf;
    uint8_t r, g, b, label;
} semtsdf_surface_point;
int semtsdf_export_surface(semtsdf_vol* v, float sdf_max, int32_t min_weight, semtsdf_surface_point* out,
                           uint64_t capacity, uint64_t* count);

/* ---- empty-space maps (tests) ------------------------------------------------------------
 * The octant distance map of the current volume state, one word per 8^3 brick (x-major, z
 * fastest): byte o = the octant-o distance in bricks (0: the brick is not skippable).  count =
 * the number of bricks (0: the handle has no octant maps); out may be NULL.  Synchronises. */
int semtsdf_map_words(semtsdf_vol* v, uint64_t* out, uint64_t capacity, uint64_t* count);

/* ---- measurement ------------------------------------------------------------------------ */
/* enable bit0: record HIP events around kernels; bit1: count touched/gated voxels; bit2: every
 * association row takes the exact f32 path (tests and its cost measurement); bit3: the octant
 * maps by the other of their two implementations (global-memory passes, the default, or LDS
 * line passes; tests: same maps); bit4: parse_frame_view_dev folds the frame's mask statistics
 * and depth pyramid into its march launch (SEMTSDF_FRAME_FOLD; tests: same results). */
int semtsdf_set_instrumentation(semtsdf_vol* v, int enable);
int semtsdf_get_timing(semtsdf_vol* v, semtsdf_timing* out); /* synchronises the stream */
int semtsdf_reset_timing(semtsdf_vol* v);

/* ---- drop-in for tsdf_cuda.tsdf_update (TSDF_Python/tsdf.cpp:11-33, exact argument order) --
 * Host arrays updated in place: tsdf_diff f32[D^3], tsdf_color i32[D^3*3], tsdf_wt i32[D^3],
 * tsdf_cls i32[D^3], tsdf_cls_cnt i32[D^3]; vol_start f32[3]; intrinsic f32[16];
 * depth u16[H*W]; color u8[H*W*3]; cls i32[H*W]; extrinsic2init f32[16]. */
int semtsdf_tsdf_update(float* tsdf_diff, int32_t* tsdf_color, int32_t* tsdf_wt, int32_t* tsdf_cls,
                        int32_t* tsdf_cls_cnt, int vol_dim, const float* vol_start, float voxel,
                        float miu, const float* intrinsic, const uint16_t* depth, const uint8_t* color,
                        const int32_t* cls, const float* extrinsic2init, int width, int height);

#ifdef __cplusplus
}
#endif
#endif /* SEMTSDF_H */
