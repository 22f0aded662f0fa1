// Internal interface between the C-ABI host layer (semtsdf_api.cpp) and the gfx950
// kernels (semtsdf_kernels.hip).  Plain-old-data argument blocks, passed by value as
// kernel arguments so that pose, intrinsics and volume geometry land in SGPRs.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace semtsdf {

constexpr int kMaxObjects = 32;

// Geometry of the locally stored part of the volume.
struct VolGeom {
    int dimx, dimy, dimz;      // global dims
    int lz;                    // local z planes (chunks * (chunk + halo))
    int shard, nshards, chunk, halo;
    float start[3];            // vol_start
    float end[3];              // vol_end
    float voxel[3];
    float mu;
    uint64_t nvox;             // dimx * dimy * lz (local voxels)
};

// Device buffers of one volume.
struct VolBufs {
    float* sdf;
    int32_t* wt;
    void* color;       // u8x3 or i32x3, AoS
    uint32_t* hist;    // bin-major [32][nvox]
    int32_t* cls;      // vote mode
    int32_t* cls_cnt;  // vote mode
};

// Per-frame depth pyramid used by the brick culler: max raw depth over tiles of
// 8, 32 and 128 pixels.
struct DepthPyramid {
    uint16_t* l0;  // [ceil(H/8)][ceil(W/8)]
    uint16_t* l1;  // [ceil(H/32)][ceil(W/32)]
    uint32_t* l2;  // [ceil(H/128)][ceil(W/128)] (u32 for atomicMax)
    int w0, h0, w1, h1, w2, h2;
};

struct IntegrateArgs {
    VolGeom g;
    VolBufs b;
    float E[12];     // rows 0..2 of extrinsic2init
    float K[9];      // rows 0..2, cols 0..2 of the intrinsic
    int width, height;
    float depth_scale;
    float gate;
    uint32_t flags;
    int cull;
    const uint16_t* depth;
    const uint8_t* rgb;
    const uint8_t* mask;    // semantic
    const int32_t* cls;     // vote
    DepthPyramid pyr;
    unsigned long long* counters;  // [0] touched, [1] gated, [2] bad-label flag
};

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
    unsigned int pad;
};

// Decision output written by the single-workgroup decide kernel.
struct AssocDecision {
    int max_obj_now;
    int num_objs_before;
    int num_objs_after;
    int bad_label;
    int assigned_prev[kMaxObjects];
    float assigned_prob[kMaxObjects];
    unsigned char lut[256];
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
};

// ---- launchers (semtsdf_kernels.hip) ----
hipError_t launch_fill_volume(const VolGeom& g, const VolBufs& b, uint32_t flags, hipStream_t s);
hipError_t launch_depth_pyramid(const uint16_t* depth, int w, int h, const DepthPyramid& p, hipStream_t s);
hipError_t launch_integrate(const IntegrateArgs& a, hipStream_t s);
hipError_t launch_mask_stats(const uint8_t* mask, int npx, AssocTables* t, hipStream_t s);
hipError_t launch_assoc_march(const AssocArgs& a, hipStream_t s);
hipError_t launch_assoc_decide(const AssocTables* t, AssocDecision* d, int num_objs, float eps,
                               int* num_objs_dev, hipStream_t s);
hipError_t launch_first_frame_objs(const AssocTables* t, int* num_objs_dev, hipStream_t s);
hipError_t launch_relabel(uint8_t* mask, int npx, const AssocDecision* d, hipStream_t s);
hipError_t launch_render(const RenderArgs& a, hipStream_t s);
// chunk [v0, v0+nv) of the bin-major histogram <-> voxel-major [nv][32] staging buffer
hipError_t launch_hist_chunk_to_vm(const uint32_t* bm, uint32_t* vm, uint64_t nvox, uint64_t v0, uint64_t nv,
                                   hipStream_t s);
hipError_t launch_hist_chunk_to_bm(const uint32_t* vm, uint32_t* bm, uint64_t nvox, uint64_t v0, uint64_t nv,
                                   hipStream_t s);

}  // namespace semtsdf
