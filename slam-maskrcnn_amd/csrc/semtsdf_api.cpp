// C-ABI host layer of libsemtsdf.so (include/semtsdf.h).
//
// Replaces the host side of the reference fusion engine:
//   TSDF::TSDF / parse_frame / init_cuda_vars / launch_kernel  src/SfM_CUDA/tsdf.cu:137-280,418-504
//   Viewer::show_tsdf                                          src/SfM_CUDA/viewer.cu:137-179
//   tsdf_cuda.tsdf_update (pybind11)                           src/TSDF_Python/tsdf.cpp:11-33, tsdf.cu:61-125
// Differences by design: every HIP call is checked and reported through an int status and
// a thread-local message (the reference checks only cudaGetLastError and throws
// std::string); all device work is stream-ordered and asynchronous; association runs on
// the device (no 49 MB probs/box_mask D2H, tsdf.cu:457-458); 64-bit voxel indexing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/semtsdf.h"
#include "semtsdf_internal.h"

using namespace semtsdf;

#ifndef SEMTSDF_EVENT_FLAGS_DEFAULT
#define SEMTSDF_EVENT_FLAGS_DEFAULT 2  // order_event_flags(): 0 system-scope release, 1 device-scope release, 2 no system fence
#endif
#ifndef SEMTSDF_FRAME_FOLD_DEFAULT
#define SEMTSDF_FRAME_FOLD_DEFAULT 0  // env SEMTSDF_FRAME_FOLD=0/1 overrides (A/B)
#endif
#ifndef SEMTSDF_MARCH_LPT_DEFAULT
#define SEMTSDF_MARCH_LPT_DEFAULT 1  // env SEMTSDF_MARCH_LPT=0/1 overrides (A/B)
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPC(expr)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail(e_ == hipErrorOutOfMemory ? SEMTSDF_ERR_OOM : SEMTSDF_ERR_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                          \
    } while (0)

// Palette of viewer.cu:93-126 (RGB triplets; written as BGR, viewer.cu:272).
const uint8_t kPalette[kMaxObjects * 3] = {
    230, 25,  75,  60,  180, 75,  255, 225, 25,  0,   130, 200, 245, 130, 48,  145, 30,  180,
    70,  240, 240, 240, 50,  230, 210, 245, 60,  250, 190, 190, 0,   128, 128, 230, 190, 255,
    170, 110, 40,  255, 250, 200, 128, 0,   0,   170, 255, 195, 230, 25,  75,  60,  180, 75,
    255, 225, 25,  0,   130, 200, 245, 130, 48,  145, 30,  180, 70,  240, 240, 240, 50,  230,
    210, 245, 60,  250, 190, 190, 0,   128, 128, 230, 190, 255, 170, 110, 40,  255, 250, 200,
    128, 0,   0,   170, 255, 195};

constexpr int kCounters = 8;  // device counters of a volume (IntegrateArgs::counters)
#ifndef SEMTSDF_FRAME_SETS
#define SEMTSDF_FRAME_SETS 2
#endif
constexpr int kFrameSets = SEMTSDF_FRAME_SETS;  // per-frame prepass output sets used in turn

struct EventPair {
    hipEvent_t a, b;
};

}  // namespace

struct semtsdf_vol {
    semtsdf_params p{};
    VolGeom g{};
    VolBufs b{};
    int device = 0;
    hipStream_t stream = nullptr;
    size_t device_bytes = 0;
    // per-frame staging (host-pointer API)
    uint16_t* depth_d = nullptr;
    uint8_t* rgb_d = nullptr;
    uint8_t* mask_d = nullptr;
    int32_t* cls_d = nullptr;
    // Per-frame prepass outputs (pixel records + depth pyramid, live-unit lists), two sets
    // used in turn: the prepass of frame k+1 may run on prep_stream while the integrate of
    // frame k still reads the other set (semtsdf_integrate_dev_async).
    struct FrameSet {
        DepthPyramid pyr{};
        unsigned* unit_list = nullptr;   // live units of the frame (cull pass)
        unsigned* list_count = nullptr;  // [kLists][kListSegs * kListCountStride] (general, free, full free)
        unsigned* units = nullptr;       // the lists compacted back to back (k_compact_lists)
        unsigned* first_tab = nullptr;   // inside units: each persistent wave's first group (XCD split)
        hipEvent_t prep_done = nullptr;  // the set's prepass finished (prep_stream)
        hipEvent_t set_free = nullptr;   // the integrate reading the set finished (recorded once async is in use)
        bool free_recorded = false;
        hipStream_t reader = nullptr;    // stream of the last integrate that read the set
    } fs[kFrameSets];
    int next_set = 0;
    hipStream_t prep_stream = nullptr;   // created on the first asynchronous integrate
    hipEvent_t in_ev = nullptr;          // parse_frame: the caller's work before the frame (inputs ready)
    bool async_used = false;
    // association state
    AssocTables* tables_d = nullptr;
    AssocDecision* decision_d = nullptr;
    AssocExact* exact_d = nullptr;  // the decision's exact path: flagged rows' f32 sums, counter
    AssocPixels px{};               // per-pixel data of the last association march (exact path)
    bool assoc_ray_done = false;    // sharded: the last ray protocol was an association (its records stand)
    int* num_objs_d = nullptr;
    float* probs_d = nullptr;     // debug only (allocated lazily)
    uint8_t* box_d = nullptr;
    uint8_t* palette_d = nullptr;
    uint8_t* render_d = nullptr;
    float* render_t_d = nullptr;
    unsigned long long* counters_d = nullptr;
    IntegrateRare* rare_d = nullptr;  // the integrate's rare-path fields (IntegrateArgs::rare)
    float* rcp_table_d = nullptr;    // RN(1/n), n = 1..kRcpTable
    AssocDecision* decision_h = nullptr;  // pinned
    // Z-sharded raycast protocol (allocated on first use)
    void* ray_state_d = nullptr;   // ShardRayState arrays, 6 x npx x 4 B
    MarchCamera ray_cam{};
    int ray_kind = -1;
    int ray_nrec = 1;              // records per pixel of the exchange (nshards: all-gather; 1: all-reduce MIN)
    int ray_next = 0;              // next expected step
    uint32_t n_obs = 0;
    bool bmin_dirty = false;       // integrated since the last map update: update marked bricks
    bool bmin_stale = true;        // reset/upload: rebuild the whole map
    hipEvent_t bmin_ev = nullptr;  // marks the last map update on map_stream (recorded when needed)
    bool bmin_ev_set = false;      // bmin_ev covers the last map update
    hipStream_t map_stream = nullptr;
    bool map_set = false;          // a map update has run (on map_stream)
    bool multi_stream = false;     // the volume has been used from more than one stream
    // Colour storage of a COLOR_I32 volume (the NumPy rule's int32 colours): u8 x 4 while every
    // value fits a byte -- the running means of byte inputs never leave [0, 255] -- and int32 x 4
    // once an upload brings values outside that range.  Integrate, render and the transfers
    // follow the storage; the int32 boundary is unchanged.
    bool color_wide = false;
    int64_t wmax_bound = 0;        // upper bound of every weight (uploads, +1 per integrate): byte storage
                                   // is left before a colour mean could take the int32 wrap (w >= 2^23)
    const uint8_t* pending_lut = nullptr;  // relabel table the next integrate's prepass applies
    unsigned long long* wtrace_d = nullptr;  // instrumentation: per-wave trace slots (kWtSlots, allocated once)
    // launch order of the fused view + association march (AssocArgs::tile_*): per-tile durations
    // of the last launch and the order the decision computed from them for tile_n tiles
    unsigned* tile_cost_d = nullptr;
    unsigned* tile_perm_d = nullptr;
    int tile_cap = 0, tile_n = 0;
    bool tables_clean = false;     // tables_d holds the cleared state (left by k_assoc_decide)
    unsigned long long votes_dropped_seen = 0;  // counters[2] at the last check_bad_label
    // instrumentation
    int instr = 0;
    std::vector<EventPair> ev_integrate, ev_assoc, ev_render, ev_prep;
    double t_integrate = 0, t_assoc = 0, t_render = 0, t_prep = 0;
    uint64_t n_integrate = 0, n_assoc = 0, n_render = 0, n_prep = 0;
};

namespace {

// Flags of the events that order this device's own streams (prepass, map update, frame sets):
// no timing and, by default, a device-scope release (the consumers are kernels of the same
// device, never the host).  SEMTSDF_EVENT_FLAGS=0 selects the default system-scope release.
unsigned order_event_flags() {
    static const char* e = getenv("SEMTSDF_EVENT_FLAGS");
    static const int mode = e ? atoi(e) : SEMTSDF_EVENT_FLAGS_DEFAULT;
    return hipEventDisableTiming | (mode == 1 ? hipEventReleaseToDevice : 0u) | (mode == 2 ? hipEventDisableSystemFence : 0u);
}

size_t npx(const semtsdf_vol* v) { return (size_t)v->p.width * (size_t)v->p.height; }

hipStream_t pick(const semtsdf_vol* v, void* s) { return s ? (hipStream_t)s : v->stream; }

int dev_alloc(semtsdf_vol* v, void** p, size_t bytes) {
    if (bytes == 0) { *p = nullptr; return SEMTSDF_OK; }
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? SEMTSDF_ERR_OOM : SEMTSDF_ERR_HIP, "hipMalloc(%zu): %s", bytes,
                    hipGetErrorString(e));
    v->device_bytes += bytes;
    return SEMTSDF_OK;
}

void free_all(semtsdf_vol* v) {
    void* ptrs[] = {v->b.sdf, v->b.wt, v->b.bmin, v->b.bplain, v->b.sbmin, v->b.bdist, v->b.boct, v->b.botmp, v->b.bdirty, v->b.dlist, v->b.sflag, v->b.color, v->b.hist, v->b.hmask, v->b.cls, v->b.cls_cnt, v->depth_d, v->rgb_d,
                    v->mask_d, v->cls_d, v->tables_d, v->decision_d,
                    v->num_objs_d, v->probs_d, v->box_d, v->palette_d, v->render_d, v->render_t_d,
                    v->counters_d, v->ray_state_d, v->rcp_table_d, v->wtrace_d, v->exact_d, v->px.bits, v->px.p, v->tile_cost_d, v->tile_perm_d, v->rare_d};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    for (auto& f : v->fs)
        for (void* q : {(void*)f.pyr.px, (void*)f.pyr.l0, (void*)f.pyr.l1, (void*)f.unit_list, (void*)f.list_count,
                        (void*)f.units})
            if (q) (void)hipFree(q);
    if (v->decision_h) (void)hipHostFree(v->decision_h);
    for (auto* vec : {&v->ev_integrate, &v->ev_assoc, &v->ev_render, &v->ev_prep})
        for (auto& e : *vec) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
    if (v->bmin_ev) (void)hipEventDestroy(v->bmin_ev);
    for (auto& f : v->fs) {
        if (f.prep_done) (void)hipEventDestroy(f.prep_done);
        if (f.set_free) (void)hipEventDestroy(f.set_free);
    }
    if (v->prep_stream) (void)hipStreamDestroy(v->prep_stream);
    if (v->in_ev) (void)hipEventDestroy(v->in_ev);
    if (v->stream) (void)hipStreamDestroy(v->stream);
}

int local_planes(const semtsdf_params* p, int* chunk, int* halo);
int after_bmin(semtsdf_vol* v, hipStream_t s);

int check_params(const semtsdf_params* p) {
    if (!p) return fail(SEMTSDF_ERR_INVALID, "params is NULL");
    for (int i = 0; i < 3; ++i) {
        if (p->dim[i] < 2 || p->dim[i] > 65535)
            return fail(SEMTSDF_ERR_INVALID, "dim[%d]=%d out of range [2, 65535]", i, p->dim[i]);
        if (!(p->voxel[i] > 0.0f) || !std::isfinite(p->voxel[i]))
            return fail(SEMTSDF_ERR_INVALID, "voxel[%d]=%g must be > 0 (place the volume first)", i, p->voxel[i]);
    }
    {  // 32-bit voxel indices of the tiled layout (tile_index): stored voxels < 2^32, tx < 2^32
        const uint64_t ny = ((uint64_t)p->dim[1] + 7) / 8 * 8, nz = ((uint64_t)p->dim[2] + 2 * kZAlign) / kZAlign * kZAlign;
        if ((uint64_t)p->dim[0] * ny * nz >= (1ull << 32) || ny * nz >= (1ull << 32) || nz * 32 >= (1ull << 24))
            return fail(SEMTSDF_ERR_INVALID, "volume %d x %d x %d too large (2^32 stored voxels or more)", p->dim[0],
                        p->dim[1], p->dim[2]);
    }
    if (!(p->mu > 0.0f)) return fail(SEMTSDF_ERR_INVALID, "mu=%g must be > 0", p->mu);
    if (p->width <= 0 || p->height <= 0 || p->width > 65535 || p->height > 65535 || (int64_t)p->width * p->height > (1 << 28))
        return fail(SEMTSDF_ERR_INVALID, "bad frame size %dx%d", p->width, p->height);
    if (!(p->depth_scale > 0.0f)) return fail(SEMTSDF_ERR_INVALID, "depth_scale must be > 0");
    // the association's log terms log(max(p / n, prior)) (tsdf.cu:318,329) stay finite and <= 0 for
    // p <= n, and its f32 rule is evaluated (certificate or exact sums) for a prior
    // in this range; the reference's value is 0.05 (configuration.h:8)
    if (!(p->prior_mrcnn_err_rate >= 0x1p-10f && p->prior_mrcnn_err_rate < 1.0f))
        return fail(SEMTSDF_ERR_INVALID, "prior_mrcnn_err_rate=%g outside [2^-10, 1)", (double)p->prior_mrcnn_err_rate);
    if ((p->flags & SEMTSDF_F_VOTE) && (p->flags & SEMTSDF_F_SEMANTIC))
        return fail(SEMTSDF_ERR_INVALID, "SEMANTIC and VOTE are exclusive");
    for (int i = 0; i < 3; ++i)
        if (!(p->voxel[i] >= 0x1p-20f && p->voxel[i] <= 0x1p20f))
            return fail(SEMTSDF_ERR_INVALID, "voxel size %g outside [2^-20, 2^20]", (double)p->voxel[i]);
    if (p->z_nshards < 1 || p->z_shard < 0 || p->z_shard >= p->z_nshards)
        return fail(SEMTSDF_ERR_INVALID, "bad shard %d of %d", p->z_shard, p->z_nshards);
    if (p->z_nshards > 1 && (p->z_chunk < 1 || p->z_chunk > p->dim[2]))
        return fail(SEMTSDF_ERR_INVALID, "bad z_chunk %d", p->z_chunk);
    {  // integrate list entries pack a unit's coordinates into 12 + 10 + 10 bits (pack_unit)
        int chunk, halo;
        const int lz = local_planes(p, &chunk, &halo);
        if (!unit_grid_fits(p->dim[0], p->dim[1], lz))
            return fail(SEMTSDF_ERR_INVALID, "volume %d x %d x %d (%d local planes) outside the unit grid limits "
                        "of the list entries (default units: x <= 4096, y <= 8192, local z <= 16384)", p->dim[0],
                        p->dim[1], p->dim[2], lz);
    }
    return SEMTSDF_OK;
}

// local z planes owned by a shard
int local_planes(const semtsdf_params* p, int* chunk, int* halo) {
    if (p->z_nshards == 1) { *chunk = p->dim[2]; *halo = 0; return p->dim[2]; }
    *chunk = p->z_chunk;
    *halo = 1;
    const int nchunks = (p->dim[2] + p->z_chunk - 1) / p->z_chunk;
    int mine = 0;
    // one chunk per round (boustrophedon order, chunk_pos in semtsdf_kernels.hip); the last
    // round may lack this shard's position
    const int n = p->z_nshards;
    for (int r = 0; r * n < nchunks; ++r)
#ifdef SEMTSDF_DEAL_RR
        if (r * n + p->z_shard < nchunks) ++mine;
#else
        if (r * n + ((r & 1) ? n - 1 - p->z_shard : p->z_shard) < nchunks) ++mine;
#endif
    return mine * (p->z_chunk + 1);
}

void fill_E(float dst[12], const float E[16]) {
    for (int i = 0; i < 12; ++i) dst[i] = E[i];
}

void timing_begin(semtsdf_vol* v, std::vector<EventPair>& vec, hipStream_t s, EventPair* ep) {
    ep->a = ep->b = nullptr;
    if (!(v->instr & 1)) return;
    if (hipEventCreate(&ep->a) != hipSuccess || hipEventCreate(&ep->b) != hipSuccess) return;
    (void)hipEventRecord(ep->a, s);
    (void)vec;
}

void timing_end(semtsdf_vol* v, std::vector<EventPair>& vec, hipStream_t s, EventPair* ep) {
    if (!(v->instr & 1) || !ep->a) return;
    (void)hipEventRecord(ep->b, s);
    vec.push_back(*ep);
}

// Screen map of the integrate contract: s = M p + m with M = RN(K E3),
// m = RN(K t), each entry a left-to-right sum of three double products rounded once to
// f32 (oracle_integrate restates it); ftol is the exactness window of the reciprocal pixel
// floor in k_integrate.
void screen_map(IntegrateArgs& a) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            const double acc = (double)a.K[i * 3 + 0] * (double)a.E[0 * 4 + j] +
                               (double)a.K[i * 3 + 1] * (double)a.E[1 * 4 + j] +
                               (double)a.K[i * 3 + 2] * (double)a.E[2 * 4 + j];
            a.M[i * 3 + j] = (float)acc;
        }
        const double acc = (double)a.K[i * 3 + 0] * (double)a.E[3] + (double)a.K[i * 3 + 1] * (double)a.E[7] +
                           (double)a.K[i * 3 + 2] * (double)a.E[11];
        a.m[i] = (float)acc;
    }
    // cull map: s(x, y, gz) = K (E3 (start + voxel * (x, y, gz)) + t), in double, rounded once
    double KE[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            if (i == 3) {
                KE[i][j] = (double)a.E[2 * 4 + j];  // qz = E row 2
                continue;
            }
            KE[i][j] = (double)a.K[i * 3 + 0] * (double)a.E[0 * 4 + j] + (double)a.K[i * 3 + 1] * (double)a.E[1 * 4 + j] +
                       (double)a.K[i * 3 + 2] * (double)a.E[2 * 4 + j];
        }
    for (int i = 0; i < 4; ++i) {
        double c0 = KE[i][3];
        for (int j = 0; j < 3; ++j) {
            a.cullC[i * 4 + j] = (float)(KE[i][j] * (double)a.g.voxel[j]);
            c0 += KE[i][j] * (double)a.g.start[j];
        }
        a.cullC[i * 4 + 3] = (float)c0;
    }
    int b = 1;
    while (b < (a.width > a.height ? a.width : a.height) + 2) b <<= 1;
    a.ftol = 0.5f - ldexpf((float)b, -21);
}

// A COLOR_I32 volume leaves byte colour storage for int32 x 4 (values converted on the device).
int widen_color(semtsdf_vol* v, hipStream_t s) {
    if (v->color_wide) return SEMTSDF_OK;
    void* wide = nullptr;
    if (int rc = dev_alloc(v, &wide, v->g.nvox * 16)) return rc;
    HIPC(launch_color_widen(static_cast<const uint8_t*>(v->b.color), static_cast<int32_t*>(wide), v->g.nvox, s));
    HIPC(hipStreamSynchronize(s));
    HIPC(hipFree(v->b.color));
    v->device_bytes -= v->g.nvox * 4;
    v->b.color = wide;
    v->color_wide = true;
    return SEMTSDF_OK;
}


int ensure_prep_stream(semtsdf_vol* v) {
    if (v->prep_stream) return SEMTSDF_OK;
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    HIPC(hipStreamCreateWithPriority(&v->prep_stream, hipStreamNonBlocking, hi));
    for (auto& f : v->fs) {
        HIPC(hipEventCreateWithFlags(&f.prep_done, order_event_flags()));
        HIPC(hipEventCreateWithFlags(&f.set_free, order_event_flags()));
    }
    return SEMTSDF_OK;
}

// async: the frame prepass runs on the volume's prep stream, ordered after inputs_ready (when
// given) and after the integrate that last read its frame set -- not after the earlier work
// of stream s -- so it may overlap the previous frame's integrate.
// inputs_on_s: inputs_ready was recorded on s at the start of the caller's frame.  When s is the
// handle's own stream and the set's last reader ran on it too, inputs_ready follows that reader
// and the prepass needs no frame-set event; on any other stream (a caller's, whose lifetime the
// handle does not control) the set's event is recorded after every integrate and waited for.
// pre_done: the frame's depth pyramid is already in the next frame set (computed in the fused
// march's launch, raw labels): only the cull runs, on s.
int integrate_impl(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, const uint8_t* mask_d,
                   const int32_t* cls_d, const float E[16], hipStream_t s, bool async = false,
                   hipEvent_t inputs_ready = nullptr, bool inputs_on_s = false, bool pre_done = false) {
    if (!E) return fail(SEMTSDF_ERR_INVALID, "E is NULL");
    if (!depth_d || !rgb_d) return fail(SEMTSDF_ERR_INVALID, "depth/rgb is NULL");
    if ((v->p.flags & SEMTSDF_F_SEMANTIC) && !mask_d) return fail(SEMTSDF_ERR_INVALID, "semantic volume needs a mask");
    if ((v->p.flags & SEMTSDF_F_VOTE) && !cls_d) return fail(SEMTSDF_ERR_INVALID, "vote volume needs cls");
    // byte colour storage holds the integer means exactly until a weight could reach 2^23,
    // where the int32 arithmetic of the reference wraps (then the means need int32 storage);
    // before the kernel arguments are built, which copy the buffer pointers
    if ((v->p.flags & SEMTSDF_F_COLOR_I32) && !v->color_wide && v->wmax_bound + 1 >= (1ll << 23)) {
        if (int rc = widen_color(v, s)) return rc;
    }
    IntegrateArgs a{};
    a.g = v->g;
    a.b = v->b;
    fill_E(a.E, E);
    const float* K = v->p.K;
    a.K[0] = K[0]; a.K[1] = K[1]; a.K[2] = K[2];
    a.K[3] = K[4]; a.K[4] = K[5]; a.K[5] = K[6];
    a.K[6] = K[8]; a.K[7] = K[9]; a.K[8] = K[10];
    a.width = v->p.width;
    a.height = v->p.height;
    a.depth_scale = v->p.depth_scale;
    a.gate = v->p.gate;
    a.flags = v->p.flags | ((v->instr & 2) ? 0x80000000u : 0u);
    a.color_wide = v->color_wide ? 1 : 0;
    a.cull = (v->p.flags & SEMTSDF_F_NO_CULL) ? 0 : 1;
    {
        static const char* dbg = getenv("SEMTSDF_DEBUG_INTEGRATE");  // timing probes only
        a.debug = dbg ? atoi(dbg) : 0;
    }
    a.depth = depth_d;
    a.rgb = rgb_d;
    a.mask = mask_d;
    a.cls = cls_d;
    const int fset = v->next_set;
    semtsdf_vol::FrameSet& F = v->fs[fset];
    a.pyr = F.pyr;
    a.counters = v->counters_d;
    a.rare = v->rare_d;
    a.unit_list = F.unit_list;
    a.list_count = F.list_count;
    a.units = F.units;
    a.first_tab = F.first_tab;
    a.first_nwaves = integrate_pre_waves();
    a.rcp_table = v->rcp_table_d;
    screen_map(a);
    a.pinhole = (a.K[1] == 0.0f && a.K[3] == 0.0f && a.K[6] == 0.0f && a.K[7] == 0.0f && a.K[8] == 1.0f) ? 1 : 0;
    a.rmu = 1.0f / v->g.mu;  // IEEE: the correctly rounded reciprocal
    a.skip_thr = v->g.voxel[0] / 2.0f * (1.0f + 0x1p-16f);  // = skip_threshold (device), same IEEE ops
    a.fastdiv = (v->g.mu >= 0x1p-20f && v->g.mu <= 0x1p20f && a.debug != 8) ? 1 : 0;
    // free units (f == 1 everywhere they are touched) change only sdf and weight when the
    // colour/histogram gate rejects f == 1 (tsdf.cu:57): SfM gated modes with gate <= 1
    a.free_ok = ((v->p.flags & SEMTSDF_F_GATE_COLOR) && !(v->p.flags & SEMTSDF_F_VOTE) && !(a.gate > 1.0f) &&
                 a.fastdiv && a.debug != 9)
                    ? 1
                    : 0;
    if (a.debug == 2) return SEMTSDF_OK;
    // a deferred relabel of this frame's association is applied by the prepass (in place):
    // that prepass follows the association on s
    // asynchronous with a pending relabel: the prepass writes the frame's raw labels beside
    // the association, and the relabel of the mask and of the records' label bytes follows
    // the decision on s (k_relabel_records)
    // the pending table stays set until the launch consuming it is queued: an error before
    // that leaves it for relabel_unconsumed (the decision already advanced num_objs)
    const uint8_t* lut = mask_d ? v->pending_lut : nullptr;
    const bool relabel_after = (async || pre_done) && lut;
    if (async)
        if (int rc = ensure_prep_stream(v)) return rc;
    hipStream_t ps = s;
    const bool own_order = inputs_ready && inputs_on_s && s == v->stream && (!F.reader || F.reader == v->stream);
    if (async) {
        ps = v->prep_stream;
        v->async_used = true;
        if (inputs_ready) HIPC(hipStreamWaitEvent(ps, inputs_ready, 0));
        if (!own_order) {
            if (!F.free_recorded) {
                // the set's event was skipped after its last integrate (which then ran on the handle's
                // own stream): everything queued there; or the first asynchronous frame: all of s
                HIPC(hipEventRecord(F.set_free, F.reader == v->stream ? v->stream : s));
                F.free_recorded = true;
            }
            HIPC(hipStreamWaitEvent(ps, F.set_free, 0));
        }
    }
    v->next_set = (v->next_set + 1) % kFrameSets;
    EventPair epp;
    timing_begin(v, v->ev_prep, ps, &epp);
    if (!pre_done)
        HIPC(launch_depth_pyramid(depth_d, rgb_d, const_cast<uint8_t*>(mask_d), v->p.width, v->p.height,
                                  v->p.depth_scale, F.pyr, F.list_count, ps, relabel_after ? nullptr : lut));
    if (lut && !relabel_after) v->pending_lut = nullptr;  // consumed by the prepass
    HIPC(launch_cull(a, ps));
    HIPC(launch_compact_lists(a, ps));
    timing_end(v, v->ev_prep, ps, &epp);
    v->n_prep++;
    if (async) {
        HIPC(hipEventRecord(F.prep_done, ps));
        HIPC(hipStreamWaitEvent(s, F.prep_done, 0));
    }
    // the relabel of a frame whose prepass ran beside its association: by the integrate
    // itself (records mapped as they are read, the mask at the kernel's end; one launch and the
    // stream gap in front of it fewer) or, with SEMTSDF_RELABEL_KERNEL=1, by k_relabel_records
    static const bool relabel_kernel = getenv("SEMTSDF_RELABEL_KERNEL") && atoi(getenv("SEMTSDF_RELABEL_KERNEL"));
    if (relabel_after && relabel_kernel) {
        HIPC(launch_relabel_records(const_cast<uint8_t*>(mask_d), v->p.width, v->p.height, F.pyr, v->decision_d, s));
        v->pending_lut = nullptr;
    } else if (relabel_after) {
        a.lut = &v->decision_d->lut[0];
        a.relabel_mask = const_cast<uint8_t*>(mask_d);
    }
    // the volume's writer: after the last empty-space map update
    if (int rc = after_bmin(v, s)) return rc;
    v->wmax_bound += 1;
    // timing: the integrate kernel's own start/end (events recorded by its dispatch, the
    // duration rocprofv3 reports for the same kernel)
    EventPair ep{nullptr, nullptr};
    if ((v->instr & 1) && (hipEventCreate(&ep.a) != hipSuccess || hipEventCreate(&ep.b) != hipSuccess))
        ep.a = ep.b = nullptr;
    // instrumentation (a SEMTSDF_WAVE_TRACE=1 build): SEMTSDF_WAVE_TRACE=<file> appends the
    // per-wave phase timestamps of the first 32 integrates (kWaveTraceWords u64 per wave slot)
    static const char* wt_path = getenv("SEMTSDF_WAVE_TRACE");
    static int wt_calls = 0;
    constexpr size_t kWtSlots = 65536;  // waves past it are not traced (the kernel checks wtrace_slots)
    const bool wt = wt_path && wt_calls < 32;
    if (wt) {
        ++wt_calls;
        if (!v->wtrace_d) HIPC(hipMalloc((void**)&v->wtrace_d, kWtSlots * kWaveTraceWords * 8));
        a.wtrace = v->wtrace_d;
        a.wtrace_slots = (unsigned)kWtSlots;
        HIPC(hipMemsetAsync(a.wtrace, 0, kWtSlots * kWaveTraceWords * 8, s));
    }
    HIPC(launch_integrate(a, s, ep.a, ep.b));
    if (a.lut) v->pending_lut = nullptr;  // consumed by the integrate
    if (wt) {
        std::vector<unsigned long long> h(kWtSlots * kWaveTraceWords);
        HIPC(hipMemcpyAsync(h.data(), a.wtrace, h.size() * 8, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        if (FILE* f = fopen(wt_path, "ab")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
    if (ep.a) v->ev_integrate.push_back(ep);
    F.reader = s;
    if (v->async_used && async && own_order) {
        F.free_recorded = false;  // a later prepass ordered otherwise records its event then
    } else if (v->async_used || s != v->stream) {
        // a later asynchronous prepass into this set waits for this integrate; recorded on a caller's
        // stream before the first asynchronous frame too, so that frame's prepass (on the prep stream)
        // waits for the stream that read the set, not for its own caller stream
        if (!F.set_free)
            if (int rc = ensure_prep_stream(v)) return rc;  // the sets' events
        HIPC(hipEventRecord(F.set_free, s));
        F.free_recorded = true;
    }
    v->bmin_dirty = true;
    v->n_integrate++;
    return SEMTSDF_OK;
}

MarchCamera assoc_camera(const semtsdf_vol* v, const float E[16]) {
    MarchCamera c{};
    const float* Ki = v->p.Kinv;
    c.Kinv[0] = Ki[0]; c.Kinv[1] = Ki[1]; c.Kinv[2] = Ki[2];
    c.Kinv[3] = Ki[4]; c.Kinv[4] = Ki[5]; c.Kinv[5] = Ki[6];
    c.Kinv[6] = Ki[8]; c.Kinv[7] = Ki[9]; c.Kinv[8] = Ki[10];
    // Rt = E(0:3,0:3)^T, o = -Rt * t (tsdf.cu:432-435); the product is accumulated in
    // double and rounded once, like cv::gemm on CV_32F.
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) c.Rt[i * 3 + j] = E[j * 4 + i];
    for (int i = 0; i < 3; ++i) {
        const double acc = (double)c.Rt[i * 3 + 0] * (double)E[3] + (double)c.Rt[i * 3 + 1] * (double)E[7] +
                           (double)c.Rt[i * 3 + 2] * (double)E[11];
        c.o[i] = -(float)acc;
    }
    c.use_s2w = 0;
    return c;
}

// Orders stream s after the last empty-space map update.  On the stream that ran it nothing
// is needed; the event is recorded on that stream only once another stream shows up (then
// eagerly after every update), so single-stream use carries no event barriers.
int order_after_map(semtsdf_vol* v, hipStream_t s) {
    if (!v->map_set || v->map_stream == s) return SEMTSDF_OK;
    v->multi_stream = true;
    if (!v->bmin_ev_set) {
        if (!v->bmin_ev) HIPC(hipEventCreateWithFlags(&v->bmin_ev, order_event_flags()));
        HIPC(hipEventRecord(v->bmin_ev, v->map_stream));  // everything queued there so far
        v->bmin_ev_set = true;
    }
    HIPC(hipStreamWaitEvent(s, v->bmin_ev, 0));
    return SEMTSDF_OK;
}

// Rebuild the empty-space map after the volume changed (integrate, upload, reset).  The
// update runs on the stream of the first march that needs it; marches on other streams (a
// render overlapping the next frame's association) and the next writer of the volume are
// ordered after it (order_after_map).
int ensure_bmin(semtsdf_vol* v, hipStream_t s) {
    if (int rc = order_after_map(v, s)) return rc;
    if (!v->bmin_dirty && !v->bmin_stale) return SEMTSDF_OK;
    // stale (reset/upload): every brick; dirty (integrate): the bricks the cull marked
    // the octant maps by the global-memory passes (default) or the LDS line passes (same maps,
    // measured no faster: profiles/r04/ab_map_passes_pipeline.txt); env SEMTSDF_MAP_GLOBAL=0/1
    // chooses, instrumentation bit 3 takes the other one (tests)
    static const char* mg = getenv("SEMTSDF_MAP_GLOBAL");
    static const bool global_default = mg ? atoi(mg) != 0 : true;
    HIPC(launch_brick_min(v->g, v->b, v->bmin_stale, s, global_default != ((v->instr & 8) != 0)));
    v->map_stream = s;
    v->map_set = true;
    v->bmin_ev_set = false;
    // on a stream other than the volume's own, record now: that stream may be gone (a
    // caller's temporary render stream) by the time another stream needs the ordering
    if (v->multi_stream || s != v->stream) {
        if (!v->bmin_ev) HIPC(hipEventCreateWithFlags(&v->bmin_ev, order_event_flags()));
        HIPC(hipEventRecord(v->bmin_ev, s));
        v->bmin_ev_set = true;
    }
    v->bmin_dirty = false;
    v->bmin_stale = false;
    return SEMTSDF_OK;
}

// A writer of the volume (integrate, upload, reset) orders itself after the last map update.
int after_bmin(semtsdf_vol* v, hipStream_t s) { return order_after_map(v, s); }

// The association tables in their cleared state before a frame's statistics: one init
// launch unless the last decide left them cleared.
int tables_ready(semtsdf_vol* v, hipStream_t s) {
    if (!v->tables_clean) HIPC(launch_tables_init(v->tables_d, s));
    v->tables_clean = false;  // the caller's kernels fill them next
    return SEMTSDF_OK;
}

// Arguments of the decision (k_assoc_decide) on the frame's raw mask; px.bits == nullptr: no
// per-pixel data (rows needing the exact path are reported in exact_missing).
DecideArgs decide_args(semtsdf_vol* v, const uint8_t* mask_d, AssocPixels px, bool certify_only = false) {
    DecideArgs d{};
    d.T = v->tables_d;
    d.D = v->decision_d;
    d.X = v->exact_d;
    d.num_objs_dev = v->num_objs_d;
    d.eps = v->p.prior_mrcnn_err_rate;
    d.n_obs = (float)v->n_obs;
    d.mask = mask_d;
    d.px = px;
    d.npx = (int)npx(v);
    d.force_exact = (v->instr & 4) ? 1 : 0;
    d.id_policy = (v->p.flags & SEMTSDF_F_ID_SATURATE) ? 1 : 0;
    d.certify_only = certify_only ? 1 : 0;
    return d;
}

// defer_relabel: the caller integrates this mask next; the relabel is left to that
// integrate's prepass (v->pending_lut), saving a launch.
// view (optional): a render of the same volume state launched together with the march
// (k_march_fused); its arguments were validated by the caller.
// pre_depth/pre_rgb (with a view): the frame's mask statistics and its prepass tiles (depth
// pyramid into the next frame set, raw labels) run as the first blocks of the fused launch; the
// caller's integrate then skips the pyramid (integrate_impl pre_done).
int associate_impl(semtsdf_vol* v, uint8_t* mask_d, const float E[16], hipStream_t s, bool want_decision,
                   bool defer_relabel = false, const RenderArgs* view = nullptr, const uint16_t* pre_depth = nullptr,
                   const uint8_t* pre_rgb = nullptr) {
    if (v->p.z_nshards != 1) return fail(SEMTSDF_ERR_UNSUPPORTED, "association on a Z-sharded handle is not supported yet");
    if (!(v->p.flags & SEMTSDF_F_SEMANTIC)) return fail(SEMTSDF_ERR_STATE, "association needs a SEMANTIC volume");
    if (v->n_obs == 0) return fail(SEMTSDF_ERR_STATE, "association needs n_obs > 0 (tsdf.cu:426)");
    EventPair ep;
    timing_begin(v, v->ev_assoc, s, &ep);
    if (int rc = ensure_bmin(v, s)) return rc;
    if (int rc = tables_ready(v, s)) return rc;
    const bool fold = view && pre_depth && pre_rgb;
    if (!fold) HIPC(launch_mask_stats(mask_d, (int)npx(v), v->tables_d, s));
    AssocArgs a{};
    a.g = v->g;
    a.b = v->b;
    a.cam = assoc_camera(v, E);
    a.width = v->p.width;
    a.height = v->p.height;
    a.n_obs = (float)v->n_obs;
    a.eps = v->p.prior_mrcnn_err_rate;
    a.box_thresh = v->p.box_thresh;
    a.mask = mask_d;
    a.tables = v->tables_d;
    a.px = v->px;
    {
        static const char* dbg = getenv("SEMTSDF_DEBUG_ASSOC");  // timing probes only
        a.debug = dbg ? atoi(dbg) : 0;
    }
    int order_n = 0;  // the decision orders the fused march's next launch (largest tiles first)
    if (view) {
        RenderArgs r = *view;
        r.b = v->b;  // the map buffers as ensure_bmin left them
        static const char* lpt = getenv("SEMTSDF_MARCH_LPT");
        if (lpt ? atoi(lpt) != 0 : SEMTSDF_MARCH_LPT_DEFAULT) {
            const int n = ((a.width + 15) / 16) * ((a.height + 15) / 16) + ((r.width + 15) / 16) * ((r.height + 15) / 16);
            if (n <= 8192 && n > v->tile_cap) {  // tile_order sorts up to 8192 tiles (256 x kTileOrderPer)
                for (unsigned** q : {&v->tile_cost_d, &v->tile_perm_d})
                    if (*q) { (void)hipFree(*q); v->device_bytes -= (size_t)v->tile_cap * sizeof(unsigned); *q = nullptr; }
                v->tile_cap = 0;
                v->tile_n = 0;
                if (int rc = dev_alloc(v, (void**)&v->tile_cost_d, (size_t)n * sizeof(unsigned))) return rc;
                if (int rc = dev_alloc(v, (void**)&v->tile_perm_d, (size_t)n * sizeof(unsigned))) return rc;
                v->tile_cap = n;
            }
            if (n <= 8192) {
                a.tile_cost = v->tile_cost_d;
                a.tile_perm = v->tile_n == n ? v->tile_perm_d : nullptr;  // sizes changed: identity
                order_n = n;
            }
        }
        FramePre pre{};
        if (fold) {
            const DepthPyramid& pyr = v->fs[v->next_set].pyr;  // the set the caller's integrate uses next
            pre.mask = mask_d;
            pre.npx = (int)npx(v);
            pre.T = v->tables_d;
            pre.nms = std::min(64, (pre.npx + 255) / 256);
            pre.depth = pre_depth;
            pre.rgb = pre_rgb;
            pre.pmask = mask_d;
            pre.w = v->p.width;
            pre.h = v->p.height;
            pre.scale = v->p.depth_scale;
            pre.vec = depth_pyramid_vec(pre_depth, pre_rgb, mask_d, v->p.width, pyr);
            pre.pyr = pyr;
            pre.list_count = v->fs[v->next_set].list_count;
            pre.npy = pyr.w1 * pyr.h1;
        }
        HIPC(launch_march_fused(a, r, pre, s));
        v->n_render++;
    } else {
        HIPC(launch_assoc_march(a, s));
    }
    {
        DecideArgs d = decide_args(v, mask_d, v->px);
        if (order_n) {
            d.tile_cost = v->tile_cost_d;
            d.tile_perm = v->tile_perm_d;
            d.tile_n = order_n;
            v->tile_n = order_n;
        }
        HIPC(launch_assoc_decide(d, s));
    }
    v->tables_clean = true;  // the decide kernel clears them
    if (defer_relabel)
        v->pending_lut = &v->decision_d->lut[0];
    else
        HIPC(launch_relabel(mask_d, (int)npx(v), v->decision_d, s));
    timing_end(v, v->ev_assoc, s, &ep);
    v->n_assoc++;
    if (want_decision) HIPC(hipMemcpyAsync(v->decision_h, v->decision_d, sizeof(AssocDecision), hipMemcpyDeviceToHost, s));
    return SEMTSDF_OK;
}

void decision_to_stats(const AssocDecision& d, semtsdf_assoc_stats* st) {
    st->max_obj_now = d.max_obj_now;
    st->num_objs = d.num_objs_after;
    st->exact_rows = d.exact_rows;
    st->reject_rows = d.reject_rows;
    for (int i = 0; i < kMaxObjects; ++i) {
        st->assigned_prev[i] = d.assigned_prev[i];
        st->assigned_prob[i] = d.assigned_prob[i];
    }
    memcpy(st->lut, d.lut, 256);
}

int validate_mask_host(const semtsdf_vol* v, const uint8_t* mask) {
    const size_t n = npx(v);
    for (size_t i = 0; i < n; ++i)
        if (mask[i] >= kMaxObjects)
            return fail(SEMTSDF_ERR_LABEL, "mask label %d at pixel %zu >= %d (tsdf.cu:61 would overflow)", mask[i], i,
                        kMaxObjects);
    return SEMTSDF_OK;
}

// The integrate counts the histogram votes it drops for ids >= 32 (counters[2], cumulative until
// a reset): a synchronous frame that added some reports SEMTSDF_ERR_LABEL, after the frame has
// been applied in full (the handle stays usable).
int check_bad_label(semtsdf_vol* v, hipStream_t s) {
    unsigned long long c[3];
    HIPC(hipMemcpyAsync(c, v->counters_d, sizeof(c), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (c[2] != v->votes_dropped_seen) {
        const unsigned long long d = c[2] - v->votes_dropped_seen;
        v->votes_dropped_seen = c[2];
        return fail(SEMTSDF_ERR_LABEL, "%llu histogram votes of ids >= %d dropped (tsdf.cu:61 would write past the "
                    "voxel's bins; SEMTSDF_F_ID_SATURATE avoids such ids)", d, kMaxObjects);
    }
    return SEMTSDF_OK;
}

}  // namespace

namespace {
// Contiguous runs of the flat x-major D^3 array whose voxels have a coordinate >= d8.
template <class F>
void for_tail_runs(int D, int d8, F&& f) {
    const size_t D2 = (size_t)D * D;
    for (int x = 0; x < D; ++x) {
        if (x >= d8) { f((size_t)x * D2, D2); continue; }
        for (int y = 0; y < D; ++y) {
            const size_t row = (size_t)x * D2 + (size_t)y * D;
            if (y >= d8) f(row, (size_t)D);
            else if (D > d8) f(row + d8, (size_t)(D - d8));
        }
    }
}
template <class T>
void tail_save(const T* a, int comps, int D, int d8, std::vector<T>& buf) {
    buf.clear();
    for_tail_runs(D, d8, [&](size_t off, size_t n) { buf.insert(buf.end(), a + off * comps, a + (off + n) * comps); });
}
template <class T>
void tail_restore(T* a, int comps, int D, int d8, const std::vector<T>& buf) {
    size_t k = 0;
    for_tail_runs(D, d8, [&](size_t off, size_t n) {
        std::copy(buf.begin() + k, buf.begin() + k + n * comps, a + off * comps);
        k += n * comps;
    });
}
}  // namespace

// =====================================================================================
extern "C" {

const char* semtsdf_last_error(void) { return g_err.c_str(); }
int semtsdf_abi_version(void) { return SEMTSDF_ABI_VERSION; }
#ifndef SEMTSDF_BUILD_KEY
#define SEMTSDF_BUILD_KEY "unknown"
#endif
const char* semtsdf_build_key(void) { return SEMTSDF_BUILD_KEY; }

int semtsdf_device_count(int* out) {
    if (!out) return fail(SEMTSDF_ERR_INVALID, "out is NULL");
    HIPC(hipGetDeviceCount(out));
    return SEMTSDF_OK;
}

int semtsdf_set_device(int device) {
    HIPC(hipSetDevice(device));
    return SEMTSDF_OK;
}

int semtsdf_stream_create(void** out) {
    if (!out) return fail(SEMTSDF_ERR_INVALID, "out is NULL");
    hipStream_t s;
    HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = (void*)s;
    return SEMTSDF_OK;
}

int semtsdf_stream_destroy(void* s) {
    if (s) HIPC(hipStreamDestroy((hipStream_t)s));
    return SEMTSDF_OK;
}

int semtsdf_stream_sync(void* s) {
    HIPC(hipStreamSynchronize((hipStream_t)s));
    return SEMTSDF_OK;
}

int semtsdf_dev_malloc(void** out, size_t bytes) {
    if (!out) return fail(SEMTSDF_ERR_INVALID, "out is NULL");
    HIPC(hipMalloc(out, bytes));
    return SEMTSDF_OK;
}

int semtsdf_dev_free(void* p) {
    if (p) HIPC(hipFree(p));
    return SEMTSDF_OK;
}

int semtsdf_memcpy(void* dst, const void* src, size_t bytes, int kind, void* stream) {
    hipMemcpyKind k;
    switch (kind) {
        case 1: k = hipMemcpyHostToDevice; break;
        case 2: k = hipMemcpyDeviceToHost; break;
        case 3: k = hipMemcpyDeviceToDevice; break;
        case 4: {  // a copy kernel: the source is read by the GPU (pinned host memory over the bus)
            if (((uintptr_t)dst | (uintptr_t)src | bytes) & 15u)
                return fail(SEMTSDF_ERR_INVALID, "kernel copy needs 16-B aligned pointers and size");
            // both ends must be GPU-addressable (device memory, or host memory pinned/registered
            // with the runtime): a kernel touching pageable memory would fault on the device.
            // The kernel gets each end's device address, which for hipHostRegister'd memory
            // need not equal the host address.
            void* dev[2] = {nullptr, nullptr};
            const void* ends[2] = {dst, src};
            for (int e = 0; e < 2; ++e) {
                hipPointerAttribute_t at{};
                if (hipPointerGetAttributes(&at, ends[e]) != hipSuccess || !at.devicePointer) {
                    (void)hipGetLastError();
                    return fail(SEMTSDF_ERR_INVALID, "kernel copy: %p is not device-accessible memory", ends[e]);
                }
                dev[e] = at.devicePointer;
                if (((uintptr_t)dev[e]) & 15u)
                    return fail(SEMTSDF_ERR_INVALID, "kernel copy: device address of %p is not 16-B aligned", ends[e]);
            }
            HIPC(launch_copy_host(dev[1], dev[0], bytes / 16, (hipStream_t)stream));
            return SEMTSDF_OK;
        }
        default: return fail(SEMTSDF_ERR_INVALID, "bad memcpy kind %d", kind);
    }
    HIPC(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream));
    return SEMTSDF_OK;
}

int semtsdf_params_default(semtsdf_params* p, int dim, const float intr[4], int width, int height) {
    if (!p || !intr) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    memset(p, 0, sizeof(*p));
    p->dim[0] = p->dim[1] = p->dim[2] = dim;
    const float fx = intr[0], fy = intr[1], cx = intr[2], cy = intr[3];
    // K as tsdf.cu:143-146 (4x4, row-major)
    p->K[0] = fx; p->K[2] = cx; p->K[5] = fy; p->K[6] = cy; p->K[10] = 1.0f; p->K[15] = 1.0f;
    // K^-1, computed exactly in double and rounded once
    p->Kinv[0] = (float)(1.0 / (double)fx);
    p->Kinv[2] = (float)(-(double)cx / (double)fx);
    p->Kinv[5] = (float)(1.0 / (double)fy);
    p->Kinv[6] = (float)(-(double)cy / (double)fy);
    p->Kinv[10] = 1.0f;
    p->Kinv[15] = 1.0f;
    p->width = width;
    p->height = height;
    p->depth_scale = 5000.0f;
    p->gate = 0.99f;
    p->box_thresh = 0.3f;
    p->prior_mrcnn_err_rate = 0.05f;
    p->duplicate_thresh = 0.5f;
    p->flags = SEMTSDF_F_SEMANTIC | SEMTSDF_F_GATE_COLOR;
    p->z_shard = 0;
    p->z_nshards = 1;
    p->z_chunk = dim;
    return SEMTSDF_OK;
}

int semtsdf_place_from_frame(semtsdf_params* p, const uint16_t* depth, double mean_depth, int mode) {
    if (!p || !depth) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    const int W = p->width, H = p->height;
    if (W <= 0 || H <= 0) return fail(SEMTSDF_ERR_INVALID, "bad frame size");
    // boundingRect(findNonZero(depth -> u8)) : SfM saturates (tsdf.cu:180), Python wraps (tsdf.py:35)
    int x0 = W, y0 = H, x1 = -1, y1 = -1;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint16_t d = depth[(size_t)y * W + x];
            const bool nz = (mode == SEMTSDF_PLACE_PYTHON) ? ((d & 0xFF) != 0) : (d != 0);
            if (nz) {
                x0 = std::min(x0, x); x1 = std::max(x1, x);
                y0 = std::min(y0, y); y1 = std::max(y1, y);
            }
        }
    if (x1 < 0) return fail(SEMTSDF_ERR_INVALID, "depth frame has no valid pixel");
    const int rx = x0, ry = y0, rw = x1 - x0 + 1, rh = y1 - y0 + 1;
    const float* Ki = p->Kinv;
    if (mode == SEMTSDF_PLACE_PYTHON) {
        // tsdf.py:36-47, float64 throughout from the f32 K^-1 entries
        const double md = mean_depth / 5000.0;
        double tl[3], br[3];
        const double tv[3] = {(double)rx, (double)ry, 1.0}, bv[3] = {(double)(rx + rw), (double)(ry + rh), 1.0};
        for (int i = 0; i < 3; ++i) {
            tl[i] = ((double)Ki[i * 4 + 0] * tv[0] + (double)Ki[i * 4 + 1] * tv[1]) + (double)Ki[i * 4 + 2] * tv[2];
            br[i] = ((double)Ki[i * 4 + 0] * bv[0] + (double)Ki[i * 4 + 1] * bv[1]) + (double)Ki[i * 4 + 2] * bv[2];
            tl[i] *= md;
            br[i] *= md;
        }
        const double dx = tl[0] - br[0], dy = tl[1] - br[1];
        const double half = std::sqrt(dx * dx + dy * dy) / 2.0;
        double vox[3];
        for (int i = 0; i < 3; ++i) {
            const double c = (tl[i] + br[i]) / 2.0;
            const double s = c - half, e = c + half;
            p->vol_start[i] = (float)s;
            p->vol_end[i] = (float)e;
            vox[i] = (e - s) / (double)(p->dim[i] - 1);
            p->voxel[i] = (float)vox[i];
        }
        p->mu = (float)(5.0 * vox[0]);  // tsdf.py:47, rounded to f32 for the kernel argument
    } else {
        // tsdf.cu:185-199, f32 cv::Mat arithmetic (gemm accumulates in double)
        const float md = (float)mean_depth;
        float tl[4], br[4];
        const float tv[4] = {(float)rx, (float)ry, 1.0f, 1.0f};
        const float bv[4] = {(float)(rx + rw), (float)(ry + rh), 1.0f, 1.0f};
        for (int i = 0; i < 4; ++i) {
            double at = 0, ab = 0;
            for (int k = 0; k < 4; ++k) {
                at += (double)Ki[i * 4 + k] * (double)tv[k];
                ab += (double)Ki[i * 4 + k] * (double)bv[k];
            }
            tl[i] = (float)((double)(float)at * (double)md);
            br[i] = (float)((double)(float)ab * (double)md);
        }
        const float dx = tl[0] - br[0], dy = tl[1] - br[1];
        const float half = (float)(std::sqrt(std::pow((double)dx, 2) + std::pow((double)dy, 2)) / 2.0);
        for (int i = 0; i < 3; ++i) {
            const float c = (tl[i] + br[i]) * 0.5f;
            p->vol_start[i] = c - half;
            p->vol_end[i] = c + half;
            p->voxel[i] = (p->vol_end[i] - p->vol_start[i]) / (float)(p->dim[i] - 1);
        }
        p->mu = 5.0f * p->voxel[0];
    }
    return SEMTSDF_OK;
}

int semtsdf_create(const semtsdf_params* p, int device, semtsdf_vol** out) {
    if (!out) return fail(SEMTSDF_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int rc = check_params(p);
    if (rc) return rc;
    HIPC(hipSetDevice(device));
    semtsdf_vol* v = new semtsdf_vol();
    v->p = *p;
    v->device = device;
    int chunk, halo;
    const int lz = local_planes(p, &chunk, &halo);
    VolGeom& g = v->g;
    g.dimx = p->dim[0]; g.dimy = p->dim[1]; g.dimz = p->dim[2];
    g.lz = lz;
    g.zs = (lz + kZAlign - 1) & ~(kZAlign - 1);  // whole tiles of 32 planes (tile_index)
    g.shard = p->z_shard; g.nshards = p->z_nshards; g.chunk = chunk; g.halo = halo;
    for (int i = 0; i < 3; ++i) { g.start[i] = p->vol_start[i]; g.end[i] = p->vol_end[i]; g.voxel[i] = p->voxel[i]; }
    g.mu = p->mu;
    g.nuy = (uint32_t)(g.dimy + 7) / 8;
    g.nuz = (uint32_t)g.zs / 32;
    g.nvox = (uint64_t)g.dimx * g.nuy * g.nuz * 256u;  // tiled layout (tile_index)
    g.ty = g.nuz * 256u;
    g.tx = g.nuy * g.ty;
    g.nbx = (g.dimx + 7) / 8; g.nby = (g.dimy + 7) / 8; g.nbz = (g.lz + 7) / 8;
    g.nsx = (g.nbx + 7) / 8; g.nsy = (g.nby + 7) / 8; g.nsz = (g.nbz + 7) / 8;
    for (int i = 0; i < 3; ++i) g.rvox[i] = 1.0f / g.voxel[i];  // IEEE: correctly rounded
    const size_t n = g.nvox;
    const size_t px = (size_t)p->width * p->height;
    auto bail = [&](int code) { free_all(v); delete v; return code; };
    // the fusion stream takes the device's greatest priority: the per-frame kernels are the
    // latency-critical consumer of a frame, the detector feeding it is throughput work
    int prio_least = 0, prio_greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
    if (hipStreamCreateWithPriority(&v->stream, hipStreamNonBlocking, prio_greatest) != hipSuccess)
        return bail(fail(SEMTSDF_ERR_HIP, "hipStreamCreate failed"));
    const bool ci32 = p->flags & SEMTSDF_F_COLOR_I32;
    if ((rc = dev_alloc(v, (void**)&v->b.sdf, n * 4))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.wt, n * 4))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.sflag, n / 32 + 1))) return bail(rc);
    const size_t nbricks = (size_t)g.nbx * g.nby * g.nbz;
    if ((rc = dev_alloc(v, (void**)&v->b.bmin, nbricks * 4))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.bplain, nbricks * 4))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.sbmin, (size_t)g.nsx * g.nsy * g.nsz * 4))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.bdist, nbricks))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.boct, nbricks * 8))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.botmp, nbricks * 8))) return bail(rc);
    const size_t nquads = (size_t)g.nbx * g.nby * (size_t)((g.nbz + 3) / 4);
    if ((rc = dev_alloc(v, (void**)&v->b.bdirty, nquads * 4))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->b.dlist, (nquads + 1) * 4))) return bail(rc);
    if (nquads && (hipMemset(v->b.bdirty, 0, nquads * 4) != hipSuccess || hipMemset(v->b.dlist, 0, 4) != hipSuccess))
        return bail(fail(SEMTSDF_ERR_HIP, "memset failed"));
    (void)ci32;  // COLOR_I32 volumes start with byte storage (color_wide)
    if ((rc = dev_alloc(v, &v->b.color, g.nvox * 4))) return bail(rc);
    if (p->flags & SEMTSDF_F_SEMANTIC)
    {
        if ((rc = dev_alloc(v, (void**)&v->b.hist, g.nvox * kMaxObjects * 4))) return bail(rc);
        if ((rc = dev_alloc(v, (void**)&v->b.hmask, n * 4))) return bail(rc);
    }
    if (p->flags & SEMTSDF_F_VOTE) {
        if ((rc = dev_alloc(v, (void**)&v->b.cls, n * 4))) return bail(rc);
        if ((rc = dev_alloc(v, (void**)&v->b.cls_cnt, n * 4))) return bail(rc);
        if ((rc = dev_alloc(v, (void**)&v->cls_d, px * 4))) return bail(rc);
    }
    if ((rc = dev_alloc(v, (void**)&v->depth_d, px * 2))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->rgb_d, px * 3))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->mask_d, px))) return bail(rc);
    for (auto& f : v->fs) {
        DepthPyramid& pyr = f.pyr;
        pyr.w0 = (p->width + 7) / 8; pyr.h0 = (p->height + 7) / 8;
        pyr.w1 = (p->width + 31) / 32; pyr.h1 = (p->height + 31) / 32;
        pyr.rs = 4u * (unsigned)((p->width + 1 + 3) / 4 * 4);
        // the zero column u = W and row v = H (and the padding of the last band) stay zero
        const size_t nrec = (size_t)pyr.rs * (size_t)((p->height + 1 + 3) / 4);
        if ((rc = dev_alloc(v, (void**)&pyr.px, nrec * 8))) return bail(rc);
        if (hipMemset(pyr.px, 0, nrec * 8) != hipSuccess) return bail(fail(SEMTSDF_ERR_HIP, "memset failed"));
        if ((rc = dev_alloc(v, (void**)&pyr.l0, (size_t)pyr.w1 * 4 * pyr.h1 * 4 * sizeof(uint2)))) return bail(rc);
        if ((rc = dev_alloc(v, (void**)&pyr.l1, (size_t)pyr.w1 * pyr.h1 * sizeof(uint2)))) return bail(rc);
        if ((rc = dev_alloc(v, (void**)&f.unit_list, unit_list_capacity(g) * sizeof(unsigned)))) return bail(rc);
        // + the integrate's dynamic counters (per XCD and workgroup slot), kListCountStride words apart
        if ((rc = dev_alloc(v, (void**)&f.list_count, kListCountWords * sizeof(unsigned)))) return bail(rc);
        // every unit in at most one list, + one pad per list, bases rounded up to even; at least two
        // entries per persistent wave (k_integrate reads a wave's first free group unconditionally)
        const uint64_t nunits = std::max<uint64_t>(unit_count(g) + 2 * kLists + 2, 2u * (uint64_t)kPreWaves + 6u);
        // + the first-group table of the XCD split (two entries per wave slot, k_compact_lists)
        if ((rc = dev_alloc(v, (void**)&f.units, (nunits + 2u * (uint64_t)kPreWaves) * sizeof(unsigned)))) return bail(rc);
        f.first_tab = f.units + nunits;
    }
    if ((rc = dev_alloc(v, (void**)&v->rcp_table_d, kRcpTable * sizeof(float)))) return bail(rc);
    {
        float t[kRcpTable];
        for (int i = 0; i < kRcpTable; ++i) t[i] = 1.0f / (float)(i + 1);  // IEEE: correctly rounded
        if (hipMemcpy(v->rcp_table_d, t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(SEMTSDF_ERR_HIP, "rcp table upload failed"));
    }
    if ((rc = dev_alloc(v, (void**)&v->tables_d, sizeof(AssocTables)))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->decision_d, sizeof(AssocDecision)))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->exact_d, sizeof(AssocExact)))) return bail(rc);
    if (hipMemset(v->exact_d, 0, sizeof(AssocExact)) != hipSuccess) return bail(fail(SEMTSDF_ERR_HIP, "memset failed"));
    if ((p->flags & SEMTSDF_F_SEMANTIC) && p->z_nshards == 1) {  // the association's per-pixel data
        if ((rc = dev_alloc(v, (void**)&v->px.bits, npx(v) * sizeof(uint2)))) return bail(rc);
        if ((rc = dev_alloc(v, (void**)&v->px.p, npx(v) * kMaxObjects * sizeof(float)))) return bail(rc);
    }
    if ((rc = dev_alloc(v, (void**)&v->num_objs_d, 16))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->counters_d, kCounters * sizeof(unsigned long long)))) return bail(rc);
    if ((rc = dev_alloc(v, (void**)&v->rare_d, sizeof(IntegrateRare)))) return bail(rc);
    {
        const IntegrateRare r{v->b.bdirty, v->b.dlist, g.nby, g.nbz, v->counters_d};
        if (hipMemcpy(v->rare_d, &r, sizeof(r), hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(SEMTSDF_ERR_HIP, "upload of the integrate's rare-path fields failed"));
    }
    if ((rc = dev_alloc(v, (void**)&v->palette_d, sizeof(kPalette)))) return bail(rc);
    if (hipHostMalloc((void**)&v->decision_h, sizeof(AssocDecision), 0) != hipSuccess)
        return bail(fail(SEMTSDF_ERR_HIP, "hipHostMalloc failed"));
    if (hipMemcpy(v->palette_d, kPalette, sizeof(kPalette), hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(SEMTSDF_ERR_HIP, "palette upload failed"));
    if ((rc = semtsdf_reset(v, nullptr))) return bail(rc);
    if (hipStreamSynchronize(v->stream) != hipSuccess) return bail(fail(SEMTSDF_ERR_HIP, "sync failed"));
    *out = v;
    return SEMTSDF_OK;
}

int semtsdf_destroy(semtsdf_vol* v) {
    if (!v) return SEMTSDF_OK;
    (void)hipSetDevice(v->device);
    (void)hipStreamSynchronize(v->stream);
    free_all(v);
    delete v;
    return SEMTSDF_OK;
}

int semtsdf_get_params(const semtsdf_vol* v, semtsdf_params* out) {
    if (!v || !out) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    *out = v->p;
    return SEMTSDF_OK;
}

int semtsdf_get_state(const semtsdf_vol* v, semtsdf_state* out) {
    if (!v || !out) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    int n = 0;
    unsigned long long dropped = 0;
    HIPC(hipMemcpyAsync(&n, v->num_objs_d, sizeof(int), hipMemcpyDeviceToHost, v->stream));
    HIPC(hipMemcpyAsync(&dropped, v->counters_d + 2, sizeof(dropped), hipMemcpyDeviceToHost, v->stream));
    HIPC(hipStreamSynchronize(v->stream));
    out->n_obs = v->n_obs;
    out->num_objs = n;
    out->local_dim[0] = v->g.dimx;
    out->local_dim[1] = v->g.dimy;
    out->local_dim[2] = v->g.lz;
    out->local_voxels = (uint64_t)v->g.dimx * v->g.dimy * v->g.lz;
    out->device_bytes = v->device_bytes;
    out->label_votes_dropped = dropped;
    return SEMTSDF_OK;
}

int semtsdf_set_state(semtsdf_vol* v, uint32_t n_obs, int32_t num_objs) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    v->n_obs = n_obs;
    HIPC(hipMemcpyAsync(v->num_objs_d, &num_objs, sizeof(int), hipMemcpyHostToDevice, v->stream));
    HIPC(hipStreamSynchronize(v->stream));
    return SEMTSDF_OK;
}

void* semtsdf_get_stream(const semtsdf_vol* v) { return v ? (void*)v->stream : nullptr; }

int semtsdf_reset(semtsdf_vol* v, void* stream) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    const size_t n = v->g.nvox;
    if (int rc = after_bmin(v, s)) return rc;
    HIPC(launch_fill_volume(v->g, v->b, v->p.flags, s));
    HIPC(hipMemsetAsync(v->b.wt, 0, n * 4, s));
    HIPC(hipMemsetAsync(v->b.sflag, 0, n / 32 + 1, s));  // steady flags: unknown
    HIPC(hipMemsetAsync(v->b.color, 0, v->g.nvox * 4 * (v->color_wide ? 4 : 1), s));
    if (v->b.hist) HIPC(hipMemsetAsync(v->b.hist, 0, v->g.nvox * kMaxObjects * 4, s));
    if (v->b.hmask) HIPC(hipMemsetAsync(v->b.hmask, 0, n * 4, s));
    if (v->b.cls) HIPC(hipMemsetAsync(v->b.cls, 0, n * 4, s));
    if (v->b.cls_cnt) HIPC(hipMemsetAsync(v->b.cls_cnt, 0, n * 4, s));
    HIPC(hipMemsetAsync(v->num_objs_d, 0, 16, s));
    HIPC(hipMemsetAsync(v->counters_d, 0, kCounters * sizeof(unsigned long long), s));
    v->votes_dropped_seen = 0;
    v->n_obs = 0;
    v->wmax_bound = 0;
    v->bmin_stale = true;
    return SEMTSDF_OK;
}

// The observation count of a semantic volume follows its integrated frames, as in the
// reference, where every integrated frame advances n_obs_ (tsdf.cu:218-220) and the first one
// sets num_objs = max(mask) + 1 (tsdf.cu:463-468): the split calls (associate, then integrate)
// leave the state TSDF::parse_frame leaves, and an association never sees histogram counts
// above n_obs that the reference could not produce (r06).  Before the frame's
// integrate: the first frame's object count.
static int observe_before(semtsdf_vol* v, const uint8_t* mask_d, hipStream_t s) {
    if (!(v->p.flags & SEMTSDF_F_SEMANTIC) || v->n_obs > 0) return SEMTSDF_OK;
    if (!mask_d) return fail(SEMTSDF_ERR_INVALID, "semantic volume needs a mask");
    if (int rc = tables_ready(v, s)) return rc;
    HIPC(launch_mask_stats(mask_d, (int)npx(v), v->tables_d, s));
    HIPC(launch_first_frame_objs(v->tables_d, v->num_objs_d, s));
    return SEMTSDF_OK;
}
// ... and after it (only when it was enqueued: a failed integrate leaves n_obs alone)
static void observe_after(semtsdf_vol* v) {
    if (v->p.flags & SEMTSDF_F_SEMANTIC) v->n_obs++;
}

int semtsdf_integrate(semtsdf_vol* v, const uint16_t* depth, const uint8_t* rgb, const uint8_t* mask,
                      const float E[16], void* stream) {
    if (!v || !depth || !rgb) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    const size_t n = npx(v);
    const bool sem = v->p.flags & SEMTSDF_F_SEMANTIC;
    bool past_bins = false;  // a label >= 32 in the mask
    if (sem) {
        if (!mask) return fail(SEMTSDF_ERR_INVALID, "semantic volume needs a mask");
        // id policy 0: ids >= 32 (an association's fresh ids past the histogram, semtsdf_associate)
        // are integrated with their votes dropped and counted, and the frame reports ERR_LABEL
        // once applied in full, as semtsdf_parse_frame does; with SEMTSDF_F_ID_SATURATE no
        // association mints them, so such a label is a bad input
        if (v->p.flags & SEMTSDF_F_ID_SATURATE) {
            if (int rc = validate_mask_host(v, mask)) return rc;
        } else {
            past_bins = validate_mask_host(v, mask) != SEMTSDF_OK;
        }
    }
    HIPC(hipMemcpyAsync(v->depth_d, depth, n * 2, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(v->rgb_d, rgb, n * 3, hipMemcpyHostToDevice, s));
    if (sem) HIPC(hipMemcpyAsync(v->mask_d, mask, n, hipMemcpyHostToDevice, s));
    if (int rc = observe_before(v, sem ? v->mask_d : nullptr, s)) return rc;
    int rc = integrate_impl(v, v->depth_d, v->rgb_d, sem ? v->mask_d : nullptr, nullptr, E, s);
    if (rc) return rc;
    observe_after(v);
    HIPC(hipStreamSynchronize(s));  // host buffers are borrowed for the call only
    if (!sem) return SEMTSDF_OK;
    const int rc_votes = check_bad_label(v, s);  // takes note of the votes this frame dropped
    if (past_bins)
        return fail(SEMTSDF_ERR_LABEL, "mask labels >= %d have no histogram bin: their votes were dropped, the "
                    "frame was applied (SEMTSDF_F_ID_SATURATE keeps ids below %d)", kMaxObjects, kMaxObjects);
    return rc_votes;
}

int semtsdf_integrate_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, const uint8_t* mask_d,
                          const float E[16], void* stream) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    if (int rc = observe_before(v, mask_d, s)) return rc;
    if (int rc = integrate_impl(v, depth_d, rgb_d, mask_d, nullptr, E, s)) return rc;
    observe_after(v);
    return SEMTSDF_OK;
}

int semtsdf_integrate_dev_async(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, const uint8_t* mask_d,
                                const float E[16], void* inputs_ready, void* stream) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    if (int rc = observe_before(v, mask_d, s)) return rc;
    if (int rc = integrate_impl(v, depth_d, rgb_d, mask_d, nullptr, E, s, true, (hipEvent_t)inputs_ready)) return rc;
    observe_after(v);
    return SEMTSDF_OK;
}

int semtsdf_integrate_vote_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, const int32_t* cls_d,
                               const float E[16], void* stream) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    if (!(v->p.flags & SEMTSDF_F_VOTE)) return fail(SEMTSDF_ERR_STATE, "volume is not in VOTE mode");
    return integrate_impl(v, depth_d, rgb_d, nullptr, cls_d, E, pick(v, stream));
}

int semtsdf_associate(semtsdf_vol* v, uint8_t* mask_inout, const float E[16], semtsdf_assoc_stats* stats,
                      void* stream) {
    if (!v || !mask_inout || !E) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    int rc = validate_mask_host(v, mask_inout);
    if (rc) return rc;
    hipStream_t s = pick(v, stream);
    HIPC(hipMemcpyAsync(v->mask_d, mask_inout, npx(v), hipMemcpyHostToDevice, s));
    rc = associate_impl(v, v->mask_d, E, s, true);
    if (rc) return rc;
    HIPC(hipMemcpyAsync(mask_inout, v->mask_d, npx(v), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (stats) decision_to_stats(*v->decision_h, stats);
    if (v->decision_h->bad_label)
        return fail(SEMTSDF_ERR_LABEL, "association produced %d objects (> %d)", v->decision_h->num_objs_after,
                    kMaxObjects);
    return SEMTSDF_OK;
}

int semtsdf_associate_dev(semtsdf_vol* v, uint8_t* mask_d, const float E[16], semtsdf_assoc_stats* stats,
                          void* stream) {
    if (!v || !mask_d || !E) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    hipStream_t s = pick(v, stream);
    int rc = associate_impl(v, mask_d, E, s, stats != nullptr);
    if (rc) return rc;
    if (stats) {
        HIPC(hipStreamSynchronize(s));
        decision_to_stats(*v->decision_h, stats);
    }
    return SEMTSDF_OK;
}

int semtsdf_filter_overlaps_dev(semtsdf_vol* v, const float* probs_d, const uint8_t* box_d, uint8_t* mask_d,
                                semtsdf_assoc_stats* stats, void* stream) {
    if (!v || !probs_d || !box_d || !mask_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (!(v->p.flags & SEMTSDF_F_SEMANTIC) || !v->px.bits)
        return fail(SEMTSDF_ERR_STATE, "filter_overlaps needs an unsharded SEMANTIC volume");
    if (v->n_obs == 0) return fail(SEMTSDF_ERR_STATE, "filter_overlaps needs n_obs > 0 (tsdf.cu:317 divides by it)");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    if (int rc = tables_ready(v, s)) return rc;
    HIPC(launch_mask_stats(mask_d, (int)npx(v), v->tables_d, s));
    HIPC(launch_assoc_from_probs(probs_d, box_d, mask_d, (int)npx(v), (float)v->n_obs, v->p.prior_mrcnn_err_rate,
                                 v->tables_d, v->px, s));
    HIPC(launch_assoc_decide(decide_args(v, mask_d, v->px), s));
    v->tables_clean = true;
    HIPC(launch_relabel(mask_d, (int)npx(v), v->decision_d, s));
    if (stats) {
        HIPC(hipMemcpyAsync(v->decision_h, v->decision_d, sizeof(AssocDecision), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        decision_to_stats(*v->decision_h, stats);
    }
    return SEMTSDF_OK;
}

int semtsdf_libm_eval(int fn, const float* x_d, float* y_d, size_t n, void* stream) {
    if (fn < 0 || fn > 2) return fail(SEMTSDF_ERR_INVALID, "fn must be 0 (logf), 1 (expf) or 2 (device logf)");
    if (n && (!x_d || !y_d)) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(launch_libm_eval(fn, x_d, y_d, n, (hipStream_t)stream));
    return SEMTSDF_OK;
}

int semtsdf_assoc_probs(semtsdf_vol* v, const float E[16], float* probs, uint8_t* box_mask, void* stream) {
    if (!v || !E || !probs || !box_mask) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (v->p.z_nshards != 1) return fail(SEMTSDF_ERR_UNSUPPORTED, "sharded handle");
    if (!(v->p.flags & SEMTSDF_F_SEMANTIC)) return fail(SEMTSDF_ERR_STATE, "needs a SEMANTIC volume");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    const size_t n = npx(v) * kMaxObjects;
    if (!v->probs_d) {
        int rc = dev_alloc(v, (void**)&v->probs_d, n * 4);
        if (rc) return rc;
        rc = dev_alloc(v, (void**)&v->box_d, n);
        if (rc) return rc;
    }
    // tables scratch is reused; the mask is all-zero so no log terms are needed
    HIPC(hipMemsetAsync(v->mask_d, 0, npx(v), s));
    HIPC(hipMemsetAsync(v->tables_d, 0, sizeof(AssocTables), s));
    v->tables_clean = false;
    AssocArgs a{};
    a.g = v->g;
    a.b = v->b;
    a.cam = assoc_camera(v, E);
    a.width = v->p.width;
    a.height = v->p.height;
    a.n_obs = (float)(v->n_obs ? v->n_obs : 1);
    a.eps = v->p.prior_mrcnn_err_rate;
    a.box_thresh = v->p.box_thresh;
    a.mask = v->mask_d;
    a.tables = v->tables_d;
    a.probs_out = v->probs_d;
    a.box_out = v->box_d;
    if (int rc = ensure_bmin(v, s)) return rc;
    HIPC(launch_assoc_march(a, s));
    HIPC(hipMemcpyAsync(probs, v->probs_d, n * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(box_mask, v->box_d, n, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return SEMTSDF_OK;
}

// An integrate that failed before its prepass leaves the association's deferred relabel
// unapplied: apply it here, so the mask matches the object count the decide kernel already
// advanced (the state an immediate relabel would have left), then report the error.
static int relabel_unconsumed(semtsdf_vol* v, uint8_t* mask_d, hipStream_t s, int rc) {
    if (v->pending_lut) {
        v->pending_lut = nullptr;
        (void)launch_relabel(mask_d, (int)npx(v), v->decision_d, s);
    }
    return rc;
}

int semtsdf_parse_frame(semtsdf_vol* v, const uint16_t* depth, const uint8_t* rgb, uint8_t* mask_inout,
                        const float E[16], semtsdf_assoc_stats* stats, void* stream) {
    if (!v || !depth || !rgb || !E) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    const size_t n = npx(v);
    const bool sem = v->p.flags & SEMTSDF_F_SEMANTIC;
    if (sem) {
        if (!mask_inout) return fail(SEMTSDF_ERR_INVALID, "semantic volume needs a mask");
        int rc = validate_mask_host(v, mask_inout);
        if (rc) return rc;
    }
    HIPC(hipMemcpyAsync(v->depth_d, depth, n * 2, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(v->rgb_d, rgb, n * 3, hipMemcpyHostToDevice, s));
    if (sem) {
        HIPC(hipMemcpyAsync(v->mask_d, mask_inout, n, hipMemcpyHostToDevice, s));
        if (v->n_obs > 0) {
            int rc = associate_impl(v, v->mask_d, E, s, true, true);
            if (rc) return rc;
        } else {
            if (int rc = tables_ready(v, s)) return rc;
            HIPC(launch_mask_stats(v->mask_d, (int)n, v->tables_d, s));
            HIPC(launch_first_frame_objs(v->tables_d, v->num_objs_d, s));
        }
    }
    int rc = integrate_impl(v, v->depth_d, v->rgb_d, sem ? v->mask_d : nullptr, nullptr, E, s);
    if (rc) return relabel_unconsumed(v, v->mask_d, s, rc);
    v->n_obs++;
    if (sem) HIPC(hipMemcpyAsync(mask_inout, v->mask_d, n, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    int rc_label = SEMTSDF_OK;  // reported after the frame is applied in full (the handle stays usable)
    if (sem && v->n_obs > 1) {
        if (stats) decision_to_stats(*v->decision_h, stats);
        if (v->decision_h->bad_label)
            rc_label = fail(SEMTSDF_ERR_LABEL, "association produced %d objects (> %d): ids >= %d have no "
                            "histogram bin (SEMTSDF_F_ID_SATURATE avoids them)", v->decision_h->num_objs_after,
                            kMaxObjects, kMaxObjects);
    } else if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (int i = 0; i < kMaxObjects; ++i) stats->assigned_prev[i] = -1;
        for (int i = 0; i < 256; ++i) stats->lut[i] = (uint8_t)i;
        int no = 0;
        HIPC(hipMemcpy(&no, v->num_objs_d, sizeof(int), hipMemcpyDeviceToHost));
        stats->num_objs = no;
        stats->max_obj_now = no;
    }
    if (sem) {
        const int rc_votes = check_bad_label(v, s);  // also takes note of this frame's dropped votes
        return rc_label ? rc_label : rc_votes;
    }
    return SEMTSDF_OK;
}

int semtsdf_parse_frame_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, uint8_t* mask_d,
                            const float E[16], void* stream) {
    return semtsdf_parse_frame_dev_after(v, depth_d, rgb_d, mask_d, E, nullptr, stream);
}

#ifndef SEMTSDF_OVERLAP_PREP
#define SEMTSDF_OVERLAP_PREP 1  // parse_frame_dev paths: the frame prepass on the prep stream beside the march
#endif
static int launch_view(semtsdf_vol* v, const RenderArgs& view, hipStream_t s);
static int render_args(semtsdf_vol* v, const float s2w[16], const float c[3], int mode, uint8_t* out_bgr_d,
                       float* out_t_d, RenderArgs& a);

// view (optional): a render of the volume state before this frame, launched with this
// frame's association march when there is one (else on its own, first).
static int parse_frame_dev_impl(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, uint8_t* mask_d,
                                const float E[16], void* integrate_after_event, hipStream_t s,
                                const RenderArgs* view) {
    const bool sem = v->p.flags & SEMTSDF_F_SEMANTIC;
    if (sem && !mask_d) return fail(SEMTSDF_ERR_INVALID, "semantic volume needs a mask");
    const bool fused = view && sem && v->n_obs > 0;
    if (view && !fused)
        if (int rc = launch_view(v, *view, s)) return rc;
    // with an association, the frame's prepass (depth pyramid, cull) runs on the prep stream
    // beside the march (it reads only the frame's inputs), from the work queued so far on s
    // (the mask statistics stay on s: on the prep stream they slowed the fused view + march
    // launch, 2.45 -> 2.20 k frames/s same-box, profiles/r03/s2/ab_pipeline_mask_stats.txt)
    // fused view with the frame's mask statistics and depth pyramid folded into the march's
    // launch (SEMTSDF_FRAME_FOLD): everything on s, no prep-stream events
    static const char* ff_env = getenv("SEMTSDF_FRAME_FOLD");
    static const bool ff_on = ff_env ? atoi(ff_env) != 0 : SEMTSDF_FRAME_FOLD_DEFAULT;
    const bool fold = (ff_on || (v->instr & 16)) && fused && !integrate_after_event;
    const bool overlap_prep = !fold && SEMTSDF_OVERLAP_PREP && sem && v->n_obs > 0 && !integrate_after_event;
    if (overlap_prep) {
        if (!v->in_ev) HIPC(hipEventCreateWithFlags(&v->in_ev, order_event_flags()));
        HIPC(hipEventRecord(v->in_ev, s));
    }
    if (sem) {
        if (v->n_obs > 0) {
            int rc = associate_impl(v, mask_d, E, s, false, true, fused ? view : nullptr, fold ? depth_d : nullptr,
                                    fold ? rgb_d : nullptr);
            if (rc) return rc;
        } else {
            if (int rc = tables_ready(v, s)) return rc;
            HIPC(launch_mask_stats(mask_d, (int)npx(v), v->tables_d, s));
            HIPC(launch_first_frame_objs(v->tables_d, v->num_objs_d, s));
        }
    }
    // the integrate is the frame's only write of the volume: readers of the previous state on
    // other streams (a live render) finish first; the association above, a read, may overlap them
    if (integrate_after_event) HIPC(hipStreamWaitEvent(s, (hipEvent_t)integrate_after_event, 0));
    int rc = integrate_impl(v, depth_d, rgb_d, sem ? mask_d : nullptr, nullptr, E, s, overlap_prep,
                            overlap_prep ? v->in_ev : nullptr, overlap_prep, fold);
    if (rc) return relabel_unconsumed(v, mask_d, s, rc);
    v->n_obs++;
    // the next frame's association (and a live view) march this state: refresh the
    // empty-space map now, on this stream, so a view on another stream ordered after this
    // call and the next association on this stream both find it current
    if (sem) return ensure_bmin(v, s);
    return SEMTSDF_OK;
}

int semtsdf_parse_frame_dev_after(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, uint8_t* mask_d,
                                  const float E[16], void* integrate_after_event, void* stream) {
    if (!v || !E || !depth_d || !rgb_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    return parse_frame_dev_impl(v, depth_d, rgb_d, mask_d, E, integrate_after_event, pick(v, stream), nullptr);
}

int semtsdf_parse_frame_view_dev(semtsdf_vol* v, const uint16_t* depth_d, const uint8_t* rgb_d, uint8_t* mask_d,
                                 const float E[16], const float s2w[16], const float c[3], int mode,
                                 uint8_t* out_bgr_d, float* out_t_d, void* stream) {
    if (!v || !E || !depth_d || !rgb_d || !s2w || !c || !out_bgr_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    RenderArgs view;
    if (int rc = render_args(v, s2w, c, mode, out_bgr_d, out_t_d, view)) return rc;
    return parse_frame_dev_impl(v, depth_d, rgb_d, mask_d, E, nullptr, pick(v, stream), &view);
}

// ---- Z-sharded raycast protocol ------------------------------------------------------
static ShardRayArgs shard_args(semtsdf_vol* v) {
    ShardRayArgs a{};
    a.g = v->g;
    a.b = v->b;
    a.cam = v->ray_cam;
    a.width = v->p.width;
    a.height = v->p.height;
    a.kind = v->ray_kind;
    a.nrec = v->ray_nrec;
    const size_t n = npx(v);
    char* base = (char*)v->ray_state_d;
    a.st.k = (int*)(base);
    a.st.fk = (float*)(base + 4 * n);
    a.st.j = (int*)(base + 8 * n);
    a.st.fj = (float*)(base + 12 * n);
    a.st.fp = (float*)(base + 16 * n);
    a.st.t = (float*)(base + 20 * n);
    a.color_i32 = v->color_wide ? 1 : 0;
    a.palette = v->palette_d;
    a.n_obs = (float)v->n_obs;
    a.eps = v->p.prior_mrcnn_err_rate;
    a.box_thresh = v->p.box_thresh;
    return a;
}

int semtsdf_shard_ray_begin(semtsdf_vol* v, int kind, const float cam[16], const float c[3], int exchange,
                            size_t* record_bytes, int* nsteps) {
    if (!v || !cam) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (exchange != SEMTSDF_EXCHANGE_ALLGATHER && exchange != SEMTSDF_EXCHANGE_MIN)
        return fail(SEMTSDF_ERR_INVALID, "bad exchange %d", exchange);
    if (kind != SEMTSDF_RENDER_LABEL && kind != SEMTSDF_RENDER_COLOR && kind != SEMTSDF_RAY_ASSOC)
        return fail(SEMTSDF_ERR_INVALID, "bad ray kind %d", kind);
    if (kind != SEMTSDF_RAY_ASSOC && !c) return fail(SEMTSDF_ERR_INVALID, "render needs the camera centre");
    if ((kind == SEMTSDF_RENDER_LABEL || kind == SEMTSDF_RAY_ASSOC) && !(v->p.flags & SEMTSDF_F_SEMANTIC))
        return fail(SEMTSDF_ERR_STATE, "label render / association needs a SEMANTIC volume");
    if (kind == SEMTSDF_RAY_ASSOC && v->n_obs == 0)
        return fail(SEMTSDF_ERR_STATE, "association needs n_obs > 0 (tsdf.cu:426)");
    HIPC(hipSetDevice(v->device));
    if (!v->ray_state_d) {
        int rc = dev_alloc(v, &v->ray_state_d, 24 * npx(v));
        if (rc) return rc;
    }
    if (kind == SEMTSDF_RAY_ASSOC) {
        v->ray_cam = assoc_camera(v, cam);
    } else {
        MarchCamera m{};
        for (int i = 0; i < 12; ++i) m.s2w[i] = cam[i];
        m.o[0] = c[0]; m.o[1] = c[1]; m.o[2] = c[2];
        m.use_s2w = 1;
        v->ray_cam = m;
    }
    if (int rc = ensure_bmin(v, v->stream)) return rc;
    HIPC(hipStreamSynchronize(v->stream));  // the protocol's steps may run on another stream
    v->ray_kind = kind;
    v->assoc_ray_done = false;
    v->ray_nrec = exchange == SEMTSDF_EXCHANGE_MIN ? 1 : v->p.z_nshards;
    v->ray_next = 0;
    if (record_bytes) *record_bytes = 8 * npx(v);
    if (nsteps) *nsteps = kind == SEMTSDF_RAY_ASSOC ? 3 : 4;
    return SEMTSDF_OK;
}

int semtsdf_shard_ray_step(semtsdf_vol* v, int step, const void* gathered_d, void* send_d, void* stream) {
    if (!v || !send_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (v->ray_kind < 0) return fail(SEMTSDF_ERR_STATE, "shard_ray_begin was not called");
    const int nsteps = v->ray_kind == SEMTSDF_RAY_ASSOC ? 3 : 4;
    if (step != v->ray_next || step >= nsteps)
        return fail(SEMTSDF_ERR_STATE, "ray step %d out of order (expected %d of %d)", step, v->ray_next, nsteps);
    if (step > 0 && !gathered_d) return fail(SEMTSDF_ERR_INVALID, "step %d needs the gathered records", step);
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    ShardRayArgs a = shard_args(v);
    a.step = step;
    a.gathered = (const int2*)gathered_d;
    a.send = (int2*)send_d;
    EventPair ep;
    timing_begin(v, v->ray_kind == SEMTSDF_RAY_ASSOC ? v->ev_assoc : v->ev_render, s, &ep);
    if (step < 3) HIPC(launch_shard_ray_step(a, s));
    else HIPC(launch_shard_render_final(a, s));
    timing_end(v, v->ray_kind == SEMTSDF_RAY_ASSOC ? v->ev_assoc : v->ev_render, s, &ep);
    v->ray_next = step + 1;
    return SEMTSDF_OK;
}

int semtsdf_shard_render_finish(semtsdf_vol* v, const void* gathered_d, uint8_t* out_bgr_d, float* out_t_d,
                                void* stream) {
    if (!v || !gathered_d || !out_bgr_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (v->ray_kind != SEMTSDF_RENDER_LABEL && v->ray_kind != SEMTSDF_RENDER_COLOR)
        return fail(SEMTSDF_ERR_STATE, "no render in progress");
    if (v->ray_next != 4) return fail(SEMTSDF_ERR_STATE, "render_finish before step 3");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    ShardRayArgs a = shard_args(v);
    a.gathered = (const int2*)gathered_d;
    a.out_bgr = out_bgr_d;
    a.out_t = out_t_d;
    HIPC(launch_shard_render_finish(a, s));
    v->ray_kind = -1;
    v->n_render++;
    return SEMTSDF_OK;
}

int semtsdf_shard_assoc_partial(semtsdf_vol* v, const void* gathered_d, const uint8_t* mask_d, int64_t* partial_d,
                                void* stream) {
    if (!v || !gathered_d || !mask_d || !partial_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (v->ray_kind != SEMTSDF_RAY_ASSOC || v->ray_next != 3)
        return fail(SEMTSDF_ERR_STATE, "assoc_partial needs the three association steps first");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    ShardRayArgs a = shard_args(v);
    a.gathered = (const int2*)gathered_d;
    a.mask = mask_d;
    a.partial = (long long*)partial_d;
    EventPair ep;
    timing_begin(v, v->ev_assoc, s, &ep);
    HIPC(hipMemsetAsync(partial_d, 0, sizeof(int64_t) * SEMTSDF_ASSOC_PARTIAL_LEN, s));
    HIPC(launch_shard_assoc_partial(a, s));
    timing_end(v, v->ev_assoc, s, &ep);
    v->ray_kind = -1;
    v->assoc_ray_done = true;
    return SEMTSDF_OK;
}

int semtsdf_shard_assoc_pixels(semtsdf_vol* v, const void* gathered_d, int32_t* px_d, void* stream) {
    if (!v || !gathered_d || !px_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (!v->assoc_ray_done) return fail(SEMTSDF_ERR_STATE, "assoc_pixels needs a completed association protocol");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    ShardRayArgs a = shard_args(v);
    a.kind = SEMTSDF_RAY_ASSOC;  // the protocol's kind (assoc_partial has closed it)
    a.gathered = (const int2*)gathered_d;
    HIPC(launch_shard_assoc_pixels(a, px_d, s));
    return SEMTSDF_OK;
}

int semtsdf_shard_assoc_apply_exact(semtsdf_vol* v, const int64_t* reduced_d, const int32_t* px_d, uint8_t* mask_d,
                                    semtsdf_assoc_stats* stats, void* stream) {
    if (!v || !reduced_d || !px_d || !mask_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    EventPair ep;
    timing_begin(v, v->ev_assoc, s, &ep);
    if (int rc = tables_ready(v, s)) return rc;
    HIPC(launch_mask_stats(mask_d, (int)npx(v), v->tables_d, s));
    HIPC(launch_tables_from_partial((const long long*)reduced_d, v->tables_d, s));
    AssocPixels px;
    px.bits = reinterpret_cast<uint2*>(const_cast<int32_t*>(px_d));
    px.p = reinterpret_cast<float*>(const_cast<int32_t*>(px_d) + 2 * npx(v));
    HIPC(launch_assoc_decide(decide_args(v, mask_d, px), s));
    v->tables_clean = true;
    HIPC(launch_relabel(mask_d, (int)npx(v), v->decision_d, s));
    timing_end(v, v->ev_assoc, s, &ep);
    v->n_assoc++;
    if (stats) {
        HIPC(hipMemcpyAsync(v->decision_h, v->decision_d, sizeof(AssocDecision), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        decision_to_stats(*v->decision_h, stats);
    }
    return SEMTSDF_OK;
}

int semtsdf_shard_assoc_apply(semtsdf_vol* v, const int64_t* reduced_d, uint8_t* mask_d, semtsdf_assoc_stats* stats,
                              void* stream) {
    if (!v || !reduced_d || !mask_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    EventPair ep;
    timing_begin(v, v->ev_assoc, s, &ep);
    if (int rc = tables_ready(v, s)) return rc;
    HIPC(launch_mask_stats(mask_d, (int)npx(v), v->tables_d, s));
    HIPC(launch_tables_from_partial((const long long*)reduced_d, v->tables_d, s));
    // the certificate first: rows it cannot decide from the reduced sums need every pixel's
    // data, which the shards hold in parts (semtsdf_shard_assoc_pixels)
    HIPC(launch_assoc_decide(decide_args(v, mask_d, AssocPixels{}, true), s));
    unsigned missing = 0;
    HIPC(hipMemcpyAsync(&missing, &v->decision_d->exact_missing, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (missing) {
        timing_end(v, v->ev_assoc, s, &ep);
        return SEMTSDF_NEED_PIXELS;  // the tables stay filled for semtsdf_shard_assoc_apply_exact
    }
    HIPC(launch_assoc_decide(decide_args(v, mask_d, AssocPixels{}), s));
    v->tables_clean = true;  // the decide kernel clears them
    HIPC(launch_relabel(mask_d, (int)npx(v), v->decision_d, s));
    timing_end(v, v->ev_assoc, s, &ep);
    v->n_assoc++;
    if (stats) {
        HIPC(hipMemcpyAsync(v->decision_h, v->decision_d, sizeof(AssocDecision), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        decision_to_stats(*v->decision_h, stats);
    }
    return SEMTSDF_OK;
}

// ABI <= 11 advanced n_obs here after a sharded integrate; the integrate entry points do it
// themselves since ABI 12 (observe_before/after), so this call only checks its handle.
int semtsdf_shard_note_integrated(semtsdf_vol* v, const uint8_t* mask_d, void* stream) {
    (void)mask_d;
    (void)stream;
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    return SEMTSDF_OK;
}

int semtsdf_masks_to_labels(const uint8_t* masks_d, int width, int height, int n, int min_area, uint8_t* labels_d,
                            int* n_kept, void* stream) {
    if (!masks_d && n > 0) return fail(SEMTSDF_ERR_INVALID, "masks is NULL");
    if (!labels_d) return fail(SEMTSDF_ERR_INVALID, "labels is NULL");
    if (width <= 0 || height <= 0 || (int64_t)width * height > (1 << 28)) return fail(SEMTSDF_ERR_INVALID, "bad size");
    if (n < 0 || n > kMaxDetections) return fail(SEMTSDF_ERR_INVALID, "n=%d detections outside [0, %d]", n, kMaxDetections);
    hipStream_t s = (hipStream_t)stream;
    void* scratch = nullptr;
    HIPC(hipMallocAsync(&scratch, mask_scratch_bytes(), s));
    hipError_t e = launch_masks_to_labels(masks_d, width * height, n, min_area, scratch, labels_d, s);
    if (e == hipSuccess && n_kept) {
        unsigned k = 0;
        e = hipMemcpyAsync(&k, (char*)scratch + mask_scratch_kept_offset(), sizeof(unsigned), hipMemcpyDeviceToHost,
                           s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        *n_kept = (int)k;
    }
    const hipError_t ef = hipFreeAsync(scratch, s);
    if (e != hipSuccess) return fail(SEMTSDF_ERR_HIP, "masks_to_labels: %s", hipGetErrorString(e));
    HIPC(ef);
    return SEMTSDF_OK;
}

int semtsdf_min_i64(int64_t* dst_d, const int64_t* src_d, size_t n, void* stream) {
    if (!dst_d || !src_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(launch_min_i64((long long*)dst_d, (const long long*)src_d, n, (hipStream_t)stream));
    return SEMTSDF_OK;
}

int semtsdf_copy_bandwidth(int device, size_t bytes, int reps, double* gbs) {
    if (!gbs || bytes < 16 || reps < 1) return fail(SEMTSDF_ERR_INVALID, "bad argument");
    HIPC(hipSetDevice(device));
    bytes &= ~(size_t)15;
    void *a = nullptr, *b = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = SEMTSDF_OK;
    float best = 1e30f;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess || hipMemsetAsync(a, 0, bytes, s) != hipSuccess) {
        rc = fail(SEMTSDF_ERR_HIP, "copy_bandwidth setup failed");
    } else {
        for (int r = 0; r <= reps && rc == SEMTSDF_OK; ++r) {
            float ms = 0.0f;
            if (hipEventRecord(e0, s) != hipSuccess || launch_copy_f4(a, b, bytes / 16, s) != hipSuccess ||
                hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
                rc = fail(SEMTSDF_ERR_HIP, "copy_bandwidth run failed");
            else if (r > 0 && ms < best)  // run 0 is a warm-up
                best = ms;
        }
    }
    if (rc == SEMTSDF_OK) *gbs = 2.0 * (double)bytes / ((double)best * 1e-3) / 1e9;
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    return rc;
}

int semtsdf_orbit_camera(const float Kinv[16], float angle, float dist, float s2w[16], float c[3]) {
    if (!Kinv || !s2w || !c) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    // viewer.cu:140-146
    const float ca = cosf(angle), sa = sinf(angle);
    const float rot[16] = {ca, 0, -sa, dist * sa, 0, 1, 0, 0, sa, 0, ca, dist - dist * ca, 0, 0, 0, 1};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double acc = 0;
            for (int k = 0; k < 4; ++k) acc += (double)rot[i * 4 + k] * (double)Kinv[k * 4 + j];
            s2w[i * 4 + j] = (float)acc;
        }
    const float r = dist + 0.5f;
    c[0] = r * sa;
    c[1] = 0.0f;
    c[2] = r - r * ca;
    return SEMTSDF_OK;
}

static int render_args(semtsdf_vol* v, const float s2w[16], const float c[3], int mode, uint8_t* out_bgr_d,
                       float* out_t_d, RenderArgs& a) {
    if (v->p.z_nshards != 1) return fail(SEMTSDF_ERR_UNSUPPORTED, "raycast on a Z-sharded handle is not supported yet");
    if (mode == SEMTSDF_RENDER_LABEL && !(v->p.flags & SEMTSDF_F_SEMANTIC))
        return fail(SEMTSDF_ERR_STATE, "label render needs a SEMANTIC volume");
    if (mode != SEMTSDF_RENDER_LABEL && mode != SEMTSDF_RENDER_COLOR) return fail(SEMTSDF_ERR_INVALID, "bad render mode %d", mode);
    a = RenderArgs{};
    a.g = v->g;
    a.b = v->b;
    for (int i = 0; i < 12; ++i) a.cam.s2w[i] = s2w[i];
    a.cam.o[0] = c[0]; a.cam.o[1] = c[1]; a.cam.o[2] = c[2];
    a.cam.use_s2w = 1;
    a.width = v->p.width;
    a.height = v->p.height;
    a.mode = mode;
    a.color_i32 = v->color_wide ? 1 : 0;
    a.palette = v->palette_d;
    a.out_bgr = out_bgr_d;
    a.out_t = out_t_d;
    return SEMTSDF_OK;
}

static int raycast_impl(semtsdf_vol* v, const float s2w[16], const float c[3], int mode, uint8_t* out_bgr_d,
                        float* out_t_d, hipStream_t s) {
    RenderArgs a;
    if (int rc = render_args(v, s2w, c, mode, out_bgr_d, out_t_d, a)) return rc;
    EventPair ep;
    if (int rc = ensure_bmin(v, s)) return rc;
    a.b = v->b;
    // instrumentation: SEMTSDF_RAY_STATS=<file> appends per-pixel march counters and
    // per-wave timestamps of every render
    static const char* rs_path = getenv("SEMTSDF_RAY_STATS");
    const size_t rs_words = npx(v) * 4 + ((npx(v) + 63) / 64 + 64) * 4;
    if (rs_path) HIPC(hipMalloc((void**)&a.ray_stats, rs_words * 4));
    if (rs_path) HIPC(hipMemsetAsync(a.ray_stats, 0, rs_words * 4, s));
    static const char* rows = getenv("SEMTSDF_RENDER_ROWS");  // instrumentation: "r0,r1"
    if (rows && sscanf(rows, "%d,%d", &a.row0, &a.row1) != 2) a.row0 = a.row1 = 0;
    timing_begin(v, v->ev_render, s, &ep);
    HIPC(launch_render(a, s));
    timing_end(v, v->ev_render, s, &ep);
    if (rs_path) {
        std::vector<unsigned> h(rs_words);
        HIPC(hipMemcpyAsync(h.data(), a.ray_stats, rs_words * 4, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        HIPC(hipFree(a.ray_stats));
        if (FILE* f = fopen(rs_path, "ab")) {
            fwrite(h.data(), 4, h.size(), f);
            fclose(f);
        }
    }
    v->n_render++;
    return SEMTSDF_OK;
}

static int launch_view(semtsdf_vol* v, const RenderArgs& view, hipStream_t s) {
    if (int rc = ensure_bmin(v, s)) return rc;
    RenderArgs a = view;
    a.b = v->b;
    HIPC(launch_render(a, s));
    v->n_render++;
    return SEMTSDF_OK;
}

int semtsdf_raycast(semtsdf_vol* v, const float s2w[16], const float c[3], int mode, uint8_t* out_bgr, float* out_t,
                    void* stream) {
    if (!v || !s2w || !c || !out_bgr) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = pick(v, stream);
    const size_t n = npx(v);
    if (!v->render_d) {
        int rc = dev_alloc(v, (void**)&v->render_d, n * 3);
        if (rc) return rc;
        rc = dev_alloc(v, (void**)&v->render_t_d, n * 4);
        if (rc) return rc;
    }
    int rc = raycast_impl(v, s2w, c, mode, v->render_d, v->render_t_d, s);
    if (rc) return rc;
    HIPC(hipMemcpyAsync(out_bgr, v->render_d, n * 3, hipMemcpyDeviceToHost, s));
    if (out_t) HIPC(hipMemcpyAsync(out_t, v->render_t_d, n * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return SEMTSDF_OK;
}

int semtsdf_raycast_dev(semtsdf_vol* v, const float s2w[16], const float c[3], int mode, uint8_t* out_bgr_d,
                        float* out_t_d, void* stream) {
    if (!v || !s2w || !c || !out_bgr_d) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    return raycast_impl(v, s2w, c, mode, out_bgr_d, out_t_d, pick(v, stream));
}

// A 4-byte per-voxel array between the reference layout (rows of lz planes, dense) and the
// tiled device storage, chunked through a device staging buffer.
// Voxels of the reference layout (rows of lz planes) held by the handle.
static uint64_t nref(const semtsdf_vol* v) { return (uint64_t)v->g.dimx * v->g.dimy * v->g.lz; }

// Voxels [vb, ve) of the reference layout (host[0] is voxel vb).
static int vox_xfer(semtsdf_vol* v, void* host, void* dev, bool to_host, const char* what, hipStream_t s, uint64_t vb,
                    uint64_t ve) {
    if (ve <= vb) return SEMTSDF_OK;
    const uint64_t chunk = std::min<uint64_t>(ve - vb, 1ull << 26);  // <= 256 MiB staging
    void* stage = nullptr;
    HIPC(hipMalloc(&stage, chunk * 4));
    for (uint64_t v0 = vb; v0 < ve; v0 += chunk) {
        const uint64_t nv = std::min<uint64_t>(chunk, ve - v0);
        char* h = static_cast<char*>(host) + (v0 - vb) * 4;
        hipError_t e;
        if (to_host) {
            e = launch_vox_chunk(dev, stage, true, v->g, v0, nv, s);
            if (e == hipSuccess) e = hipMemcpyAsync(h, stage, nv * 4, hipMemcpyDeviceToHost, s);
        } else {
            e = hipMemcpyAsync(stage, h, nv * 4, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = launch_vox_chunk(stage, dev, false, v->g, v0, nv, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            (void)hipFree(stage);
            return fail(SEMTSDF_ERR_HIP, "%s transfer: %s", what, hipGetErrorString(e));
        }
    }
    HIPC(hipFree(stage));
    return SEMTSDF_OK;
}

// colour between the padded device layout and the reference [N][3] layout, chunked
static int color_xfer(semtsdf_vol* v, void* host, bool to_host, hipStream_t s, uint64_t vb, uint64_t ve) {
    const bool i32 = v->p.flags & SEMTSDF_F_COLOR_I32;  // the boundary's element type
    const size_t es = i32 ? 4 : 1;
    if (ve <= vb) return SEMTSDF_OK;
    const uint64_t chunk = std::min<uint64_t>(ve - vb, 1ull << 24);
    void* stage = nullptr;
    HIPC(hipMalloc(&stage, chunk * 3 * es));
    for (uint64_t v0 = vb; v0 < ve; v0 += chunk) {
        const uint64_t nv = std::min<uint64_t>(chunk, ve - v0);
        char* h = static_cast<char*>(host) + (v0 - vb) * 3 * es;
        hipError_t e;
        if (to_host) {
            e = launch_color_chunk(v->b.color, stage, true, i32, v->color_wide, v->g, v0, nv, s);
            if (e == hipSuccess) e = hipMemcpyAsync(h, stage, nv * 3 * es, hipMemcpyDeviceToHost, s);
        } else {
            e = hipMemcpyAsync(stage, h, nv * 3 * es, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = launch_color_chunk(stage, v->b.color, false, i32, v->color_wide, v->g, v0, nv, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            (void)hipFree(stage);
            return fail(SEMTSDF_ERR_HIP, "colour transfer: %s", hipGetErrorString(e));
        }
    }
    HIPC(hipFree(stage));
    return SEMTSDF_OK;
}

int semtsdf_download_slab(semtsdf_vol* v, int x0, int x1, float* sdf, int32_t* wt, void* color, uint32_t* hist,
                          int32_t* cls, int32_t* cls_cnt) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    if (x0 < 0 || x1 > v->g.dimx || x0 > x1) return fail(SEMTSDF_ERR_INVALID, "bad x range [%d, %d)", x0, x1);
    HIPC(hipSetDevice(v->device));
    hipStream_t s = v->stream;
    const uint64_t plane = (uint64_t)v->g.dimy * v->g.lz;  // reference layout: x-major, z fastest
    const uint64_t vb = (uint64_t)x0 * plane, ve = (uint64_t)x1 * plane;
    int rc;
    if (sdf && (rc = vox_xfer(v, sdf, v->b.sdf, true, "sdf", s, vb, ve))) return rc;
    if (wt) HIPC(launch_flush_lazy(v->g, v->b, s));  // pending increments of steady lines into the weights
    if (wt && (rc = vox_xfer(v, wt, v->b.wt, true, "weight", s, vb, ve))) return rc;
    if (color) {
        rc = color_xfer(v, color, true, s, vb, ve);
        if (rc) return rc;
    }
    if (cls) {
        if (!(v->p.flags & SEMTSDF_F_VOTE)) return fail(SEMTSDF_ERR_STATE, "not a VOTE volume");
        if ((rc = vox_xfer(v, cls, v->b.cls, true, "cls", s, vb, ve))) return rc;
    }
    if (cls_cnt) {
        if (!(v->p.flags & SEMTSDF_F_VOTE)) return fail(SEMTSDF_ERR_STATE, "not a VOTE volume");
        if ((rc = vox_xfer(v, cls_cnt, v->b.cls_cnt, true, "cls_cnt", s, vb, ve))) return rc;
    }
    if (hist) {
        if (!(v->p.flags & SEMTSDF_F_SEMANTIC)) return fail(SEMTSDF_ERR_STATE, "not a SEMANTIC volume");
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(ve - vb, 1ull << 22));  // <= 512 MiB staging
        uint32_t* stage = nullptr;
        HIPC(hipMalloc(&stage, chunk * kMaxObjects * 4));
        for (uint64_t v0 = vb; v0 < ve; v0 += chunk) {
            const uint64_t nv = std::min<uint64_t>(chunk, ve - v0);
            hipError_t e = launch_hist_chunk_to_vm(v->b.hist, stage, v->g, v0, nv, s);
            if (e == hipSuccess)
                e = hipMemcpyAsync(hist + (v0 - vb) * kMaxObjects, stage, nv * kMaxObjects * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                (void)hipFree(stage);
                return fail(SEMTSDF_ERR_HIP, "histogram download: %s", hipGetErrorString(e));
            }
        }
        HIPC(hipFree(stage));
    }
    HIPC(hipStreamSynchronize(s));
    return SEMTSDF_OK;
}

int semtsdf_download(semtsdf_vol* v, float* sdf, int32_t* wt, void* color, uint32_t* hist, int32_t* cls,
                     int32_t* cls_cnt) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    return semtsdf_download_slab(v, 0, v->g.dimx, sdf, wt, color, hist, cls, cls_cnt);
}

int semtsdf_upload(semtsdf_vol* v, const float* sdf, const int32_t* wt, const void* color, const uint32_t* hist,
                   const int32_t* cls, const int32_t* cls_cnt) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = v->stream;
    int rc;
    if ((rc = after_bmin(v, s))) return rc;
    // derived maps first: a transfer that fails half-way must not leave steady flags or an
    // empty-space map that describe the old contents (0 = unknown is always safe)
    v->bmin_stale = true;
    // the weights a flag byte's pending increments apply to stay: fold them in before the
    // flags are dropped (an upload of the weights replaces them, pending counts included)
    if (sdf && !wt) HIPC(launch_flush_lazy(v->g, v->b, s));
    if (sdf || wt) HIPC(hipMemsetAsync(v->b.sflag, 0, v->g.nvox / 32 + 1, s));  // steady flags: unknown
    if (sdf && (rc = vox_xfer(v, const_cast<float*>(sdf), v->b.sdf, false, "sdf", s, 0, nref(v)))) return rc;
    if (wt && (rc = vox_xfer(v, const_cast<int32_t*>(wt), v->b.wt, false, "weight", s, 0, nref(v)))) return rc;
    if (wt) {
        int64_t m = 0;
        for (uint64_t i = 0, n = nref(v); i < n; ++i) m = std::max<int64_t>(m, wt[i]);
        v->wmax_bound = m;
    }
    if (color) {
        if ((v->p.flags & SEMTSDF_F_COLOR_I32) && !v->color_wide) {
            // int32 colours outside [0, 255] need the wide storage (a one-way switch)
            const int32_t* c = static_cast<const int32_t*>(color);
            const uint64_t nc = nref(v) * 3;
            bool fits = true;
            for (uint64_t i = 0; i < nc && fits; ++i) fits = (uint32_t)c[i] <= 255u;
            if (!fits && (rc = widen_color(v, s))) return rc;
        }
        rc = color_xfer(v, const_cast<void*>(color), false, s, 0, nref(v));
        if (rc) return rc;
    }
    if (cls) {
        if (!(v->p.flags & SEMTSDF_F_VOTE)) return fail(SEMTSDF_ERR_STATE, "not a VOTE volume");
        if ((rc = vox_xfer(v, const_cast<int32_t*>(cls), v->b.cls, false, "cls", s, 0, nref(v)))) return rc;
    }
    if (cls_cnt) {
        if (!(v->p.flags & SEMTSDF_F_VOTE)) return fail(SEMTSDF_ERR_STATE, "not a VOTE volume");
        if ((rc = vox_xfer(v, const_cast<int32_t*>(cls_cnt), v->b.cls_cnt, false, "cls_cnt", s, 0, nref(v)))) return rc;
    }
    if (hist) {
        if (!(v->p.flags & SEMTSDF_F_SEMANTIC)) return fail(SEMTSDF_ERR_STATE, "not a SEMANTIC volume");
        // bin mask "every bin may be present" until it is rebuilt from the new histogram
        HIPC(hipMemsetAsync(v->b.hmask, 0xFF, v->g.nvox * 4, s));
        const uint64_t n = (uint64_t)v->g.dimx * v->g.dimy * v->g.lz;
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(n, 1ull << 22));
        uint32_t* stage = nullptr;
        HIPC(hipMalloc(&stage, chunk * kMaxObjects * 4));
        for (uint64_t v0 = 0; v0 < n; v0 += chunk) {
            const uint64_t nv = std::min<uint64_t>(chunk, n - v0);
            hipError_t e =
                hipMemcpyAsync(stage, hist + v0 * kMaxObjects, nv * kMaxObjects * 4, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = launch_hist_chunk_to_bm(stage, v->b.hist, v->g, v0, nv, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                (void)hipFree(stage);
                return fail(SEMTSDF_ERR_HIP, "histogram upload: %s", hipGetErrorString(e));
            }
        }
        HIPC(hipFree(stage));
        HIPC(launch_hist_mask(v->g, v->b, s));
    }
    v->bmin_stale = true;
    HIPC(hipStreamSynchronize(s));
    return SEMTSDF_OK;
}

int semtsdf_map_words(semtsdf_vol* v, uint64_t* out, uint64_t capacity, uint64_t* count) {
    if (!v || !count) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = v->stream;
    const bool dist = v->b.bdist && v->b.boct && v->b.botmp;
    *count = dist ? (uint64_t)v->g.nbx * v->g.nby * v->g.nbz : 0u;
    if (!dist) return SEMTSDF_OK;
    if (int rc = ensure_bmin(v, s)) return rc;  // the maps of the current state
    const uint64_t n = std::min<uint64_t>(capacity, *count);
    if (out && n) HIPC(hipMemcpyAsync(out, v->b.boct, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return SEMTSDF_OK;
}

int semtsdf_export_surface(semtsdf_vol* v, float sdf_max, int32_t min_weight, semtsdf_surface_point* out,
                           uint64_t capacity, uint64_t* count) {
    static_assert(sizeof(semtsdf_surface_point) == sizeof(SurfacePoint), "surface point layout");
    if (!v || !count) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (!(sdf_max > 0.0f)) return fail(SEMTSDF_ERR_INVALID, "sdf_max must be > 0");
    HIPC(hipSetDevice(v->device));
    hipStream_t s = v->stream;
    if (int rc = after_bmin(v, s)) return rc;
    HIPC(launch_flush_lazy(v->g, v->b, s));  // pending weight increments (lazy-weight builds)
    unsigned long long* cnt_d = nullptr;
    HIPC(hipMalloc((void**)&cnt_d, sizeof(unsigned long long)));
    SurfacePoint* pts_d = nullptr;
    auto cleanup = [&]() {
        if (cnt_d) (void)hipFree(cnt_d);
        if (pts_d) (void)hipFree(pts_d);
    };
    auto run = [&](SurfacePoint* o, uint64_t cap, unsigned long long* n) -> hipError_t {
        hipError_t e = hipMemsetAsync(cnt_d, 0, sizeof(unsigned long long), s);
        if (e == hipSuccess) e = launch_export_surface(v->g, v->b, sdf_max, min_weight, v->color_wide ? 1 : 0,
                                                       (v->p.flags & SEMTSDF_F_SEMANTIC) ? 1 : 0, o, cap, cnt_d, s);
        if (e == hipSuccess) e = hipMemcpyAsync(n, cnt_d, sizeof(*n), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    };
    unsigned long long n = 0;
    hipError_t e = run(nullptr, 0, &n);
    if (e != hipSuccess) { cleanup(); return fail(SEMTSDF_ERR_HIP, "surface count: %s", hipGetErrorString(e)); }
    *count = n;
    if (!out || n == 0 || capacity == 0) { cleanup(); return SEMTSDF_OK; }
    e = hipMalloc((void**)&pts_d, n * sizeof(SurfacePoint));
    if (e != hipSuccess) { cleanup(); return fail(SEMTSDF_ERR_OOM, "surface export: %s", hipGetErrorString(e)); }
    unsigned long long n2 = 0;
    e = run(pts_d, n, &n2);
    std::vector<SurfacePoint> h(n);
    if (e == hipSuccess) e = hipMemcpy(h.data(), pts_d, n * sizeof(SurfacePoint), hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) return fail(SEMTSDF_ERR_HIP, "surface export: %s", hipGetErrorString(e));
    if (n2 != n) return fail(SEMTSDF_ERR_STATE, "surface export: count changed (%llu, %llu)", n, n2);
    // the reference's flat order (x-major, z fastest)
    std::sort(h.begin(), h.end(), [](const SurfacePoint& a, const SurfacePoint& b) {
        return a.x != b.x ? a.x < b.x : a.y != b.y ? a.y < b.y : a.z < b.z;
    });
    const uint64_t m = n < capacity ? n : capacity;
    memcpy(out, h.data(), m * sizeof(SurfacePoint));
    return SEMTSDF_OK;
}

int semtsdf_set_instrumentation(semtsdf_vol* v, int enable) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    v->instr = enable;
    return SEMTSDF_OK;
}

static double drain(std::vector<EventPair>& vec) {
    double t = 0;
    for (auto& e : vec) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) t += ms;
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    vec.clear();
    return t;
}

int semtsdf_get_timing(semtsdf_vol* v, semtsdf_timing* out) {
    if (!v || !out) return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    HIPC(hipSetDevice(v->device));
    HIPC(hipStreamSynchronize(v->stream));
    HIPC(hipDeviceSynchronize());
    v->t_integrate += drain(v->ev_integrate);
    v->t_assoc += drain(v->ev_assoc);
    v->t_render += drain(v->ev_render);
    v->t_prep += drain(v->ev_prep);
    unsigned long long c[kCounters] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPC(hipMemcpy(c, v->counters_d, sizeof(c), hipMemcpyDeviceToHost));
    out->integrate_ms = v->t_integrate;
    out->assoc_ms = v->t_assoc;
    out->render_ms = v->t_render;
    out->n_integrate = v->n_integrate;
    out->n_assoc = v->n_assoc;
    out->n_render = v->n_render;
    out->touched = c[0];
    out->gated = c[1];
    out->bricks = c[3];
    out->free_units = c[4];
    out->full_units = c[5];
    out->lazy_voxels = c[6];
    out->touched_lines = c[7];
    unsigned xr[3] = {0, 0, 0};  // AssocExact::frames, rows, pos_max
    HIPC(hipMemcpy(xr, &v->exact_d->frames, sizeof(xr), hipMemcpyDeviceToHost));
    out->assoc_exact_frames = xr[0];
    out->assoc_exact_rows = xr[1];
    out->assoc_pos_max = xr[2] / kFixScale;
    out->prep_ms = v->t_prep;
    out->n_prep = v->n_prep;
    return SEMTSDF_OK;
}

int semtsdf_reset_timing(semtsdf_vol* v) {
    if (!v) return fail(SEMTSDF_ERR_INVALID, "NULL handle");
    HIPC(hipSetDevice(v->device));
    HIPC(hipDeviceSynchronize());
    drain(v->ev_integrate);
    drain(v->ev_assoc);
    drain(v->ev_render);
    drain(v->ev_prep);
    v->t_integrate = v->t_assoc = v->t_render = v->t_prep = 0;
    v->n_integrate = v->n_assoc = v->n_render = v->n_prep = 0;
    HIPC(hipMemset(v->counters_d, 0, 2 * sizeof(unsigned long long)));
    HIPC(hipMemset(v->counters_d + 3, 0, (kCounters - 3) * sizeof(unsigned long long)));
    HIPC(hipMemset(&v->exact_d->frames, 0, 3 * sizeof(unsigned)));
    return SEMTSDF_OK;
}

// Drop-in for tsdf_cuda.tsdf_update: whole-volume in, kernel, whole-volume out, like the
// reference (TSDF_Python/tsdf.cu:78-112), but with a device volume cached across calls
// (recreated, and re-validated by semtsdf_create, whenever an argument that shapes it
// changes: vol_dim, vol_start, voxel, miu, intrinsic, frame size or the current device).
// The reference launches (vol_dim/8)^3 blocks of 8^3 threads with no bounds check
// (TSDF_Python/tsdf.cu:90), so voxels with a coordinate >= 8*(vol_dim/8) are never updated;
// they are kept unchanged here as well.
int semtsdf_tsdf_update(float* tsdf_diff, int32_t* tsdf_color, int32_t* tsdf_wt, int32_t* tsdf_cls,
                        int32_t* tsdf_cls_cnt, int vol_dim, const float* vol_start, float voxel, float miu,
                        const float* intrinsic, const uint16_t* depth, const uint8_t* color, const int32_t* cls,
                        const float* extrinsic2init, int width, int height) {
    if (!tsdf_diff || !tsdf_color || !tsdf_wt || !tsdf_cls || !tsdf_cls_cnt || !vol_start || !intrinsic || !depth ||
        !color || !cls || !extrinsic2init)
        return fail(SEMTSDF_ERR_INVALID, "NULL argument");
    if (vol_dim < 2) return fail(SEMTSDF_ERR_INVALID, "vol_dim=%d", vol_dim);
    const int d8 = vol_dim / 8 * 8;  // (vol_dim/8)^3 blocks of 8^3 voxels
    if (d8 == 0) return SEMTSDF_OK;  // the reference launches no block
    static std::mutex mu_cache;
    static semtsdf_vol* cache = nullptr;
    std::lock_guard<std::mutex> lock(mu_cache);
    int device = 0;
    HIPC(hipGetDevice(&device));
    semtsdf_params p{};
    const float intr[4] = {intrinsic[0], intrinsic[5], intrinsic[2], intrinsic[6]};
    int rc = semtsdf_params_default(&p, vol_dim, intr, width, height);
    if (rc) return rc;
    for (int i = 0; i < 16; ++i) p.K[i] = intrinsic[i];
    for (int i = 0; i < 3; ++i) {
        p.vol_start[i] = vol_start[i];
        p.voxel[i] = voxel;  // TSDF_Python passes the scalar voxel[0] (tsdf.py:63)
        p.vol_end[i] = vol_start[i] + voxel * (float)(vol_dim - 1);
    }
    p.mu = miu;
    p.flags = SEMTSDF_F_VOTE | SEMTSDF_F_COLOR_I32;
    if (cache && (memcmp(&cache->p, &p, sizeof(p)) != 0 || cache->device != device)) {
        semtsdf_destroy(cache);
        cache = nullptr;
    }
    if (!cache) {
        rc = semtsdf_create(&p, device, &cache);  // check_params validates the new arguments
        if (rc) return rc;
    }
    semtsdf_vol* v = cache;
    std::vector<float> t_sdf;
    std::vector<int32_t> t_col, t_wt, t_cls, t_cnt;
    if (d8 < vol_dim) {
        tail_save(tsdf_diff, 1, vol_dim, d8, t_sdf);
        tail_save(tsdf_color, 3, vol_dim, d8, t_col);
        tail_save(tsdf_wt, 1, vol_dim, d8, t_wt);
        tail_save(tsdf_cls, 1, vol_dim, d8, t_cls);
        tail_save(tsdf_cls_cnt, 1, vol_dim, d8, t_cnt);
    }
    rc = semtsdf_upload(v, tsdf_diff, tsdf_wt, tsdf_color, nullptr, tsdf_cls, tsdf_cls_cnt);
    if (rc) return rc;
    const size_t n = npx(v);
    hipStream_t s = v->stream;
    HIPC(hipMemcpyAsync(v->depth_d, depth, n * 2, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(v->rgb_d, color, n * 3, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(v->cls_d, cls, n * 4, hipMemcpyHostToDevice, s));
    rc = integrate_impl(v, v->depth_d, v->rgb_d, nullptr, v->cls_d, extrinsic2init, s);
    if (rc) return rc;
    rc = semtsdf_download(v, tsdf_diff, tsdf_wt, tsdf_color, nullptr, tsdf_cls, tsdf_cls_cnt);
    if (rc) return rc;
    if (d8 < vol_dim) {
        tail_restore(tsdf_diff, 1, vol_dim, d8, t_sdf);
        tail_restore(tsdf_color, 3, vol_dim, d8, t_col);
        tail_restore(tsdf_wt, 1, vol_dim, d8, t_wt);
        tail_restore(tsdf_cls, 1, vol_dim, d8, t_cls);
        tail_restore(tsdf_cls_cnt, 1, vol_dim, d8, t_cnt);
    }
    return SEMTSDF_OK;
}

}  // extern "C"
