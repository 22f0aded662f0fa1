// Greedy non-maximum suppression for the Mask R-CNN producer (include/semtsdf_det.h): the rule of
// tf.image.non_max_suppression as the reference's ProposalLayer (Mask_RCNN/mrcnn/model.py:314-323) and
// refine_detections_graph (model.py:736-750) call it, restated by mrcnn/utils.py:116-150.
//
// Two kernels.  k_nms_mask: one workgroup per (row block, column block) of 64 x 64 boxes, column
// blocks at or right of the row block only; lane r owns box i = 64 bi + r and writes one 64-bit word,
// bit c set when box 64 bj + c comes after i and overlaps it with IoU > threshold.  k_nms_sweep: one
// workgroup walks the row blocks in order.  Inside a block, wave 0 decides its 64 boxes serially from
// the block's diagonal words (a register per lane, broadcast by readlane: no memory round trip per box);
// then the 256 threads OR the kept rows' words right of the block into the LDS removed-bitmap (every
// load independent, one LDS atomic per word and wave).  Stops when max_out boxes are kept.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/semtsdf_det.h"

namespace semtsdf_det {

constexpr int kB = 64;  // boxes per block (one bit per box of a 64-bit word)

__device__ __forceinline__ float iou(float ay1, float ax1, float ay2, float ax2, float aarea, float by1, float bx1,
                                     float by2, float bx2, float barea) {
    // mrcnn/utils.py:58-76 compute_iou, in f32: intersection of the clipped extents, union of the areas
    const float y1 = fmaxf(ay1, by1), y2 = fminf(ay2, by2), x1 = fmaxf(ax1, bx1), x2 = fminf(ax2, bx2);
    const float inter = fmaxf(x2 - x1, 0.0f) * fmaxf(y2 - y1, 0.0f);
    const float uni = aarea + barea - inter;
    return inter / uni;
}

__global__ __launch_bounds__(64) void k_nms_mask(const float4* __restrict__ boxes, int n, float thr, int ncol,
                                                 unsigned long long* __restrict__ mask) {
    const int bi = (int)blockIdx.y, bj = (int)blockIdx.x;
    if (bj < bi) return;  // the sweep reads only the words at or right of a row's own block
    __shared__ float4 cb[kB];
    __shared__ float ca[kB];
    const int t = (int)threadIdx.x;
    const int j0 = bj * kB;
    if (j0 + t < n) {
        const float4 b = boxes[j0 + t];
        cb[t] = b;
        ca[t] = (b.z - b.x) * (b.w - b.y);
    }
    __syncthreads();
    const int i = bi * kB + t;
    if (i >= n) return;
    const float4 a = boxes[i];
    const float aa = (a.z - a.x) * (a.w - a.y);
    const int nc = min(kB, n - j0);
    unsigned long long w = 0;
    for (int c = 0; c < nc; ++c) {
        const int j = j0 + c;
        if (j <= i) continue;
        const float4 b = cb[c];
        if (iou(a.x, a.y, a.z, a.w, aa, b.x, b.y, b.z, b.w, ca[c]) > thr) w |= 1ull << c;
    }
    mask[(size_t)i * ncol + bj] = w;
}

__global__ __launch_bounds__(256) void k_nms_sweep(const unsigned long long* __restrict__ mask, int n, int ncol,
                                                   int max_out, int* __restrict__ keep, int* __restrict__ count) {
    __shared__ unsigned long long removed[SEMTSDF_DET_MAX_BOXES / kB];
    __shared__ unsigned long long s_kept;
    __shared__ int s_count;
    const int t = (int)threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int w = t; w < ncol; w += 256) removed[w] = 0ull;
    if (t == 0) s_count = 0;
    __syncthreads();
    for (int b = 0; b < ncol; ++b) {
        const int i0 = b * kB, nb = min(kB, n - i0);
        if (wv == 0) {
            // the block's diagonal words, one per lane, and the serial decision over its boxes
            const unsigned long long diag = lane < nb ? mask[(size_t)(i0 + lane) * ncol + b] : 0ull;
            unsigned long long cur = removed[b], kept = 0;
            int cnt = s_count;
            for (int r = 0; r < nb && cnt < max_out; ++r) {
                const unsigned long long dr =
                    ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)diag, r)) |
                    ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(diag >> 32), r) << 32);
                if (!((cur >> r) & 1ull)) {
                    kept |= 1ull << r;
                    if (lane == 0) keep[cnt] = i0 + r;
                    ++cnt;
                    cur |= dr;
                }
            }
            if (lane == 0) {
                s_kept = kept;
                s_count = cnt;
            }
        }
        __syncthreads();
        const unsigned long long kept = s_kept;
        if (s_count >= max_out) break;
        // the kept rows' words right of the block: wave q takes the kept rows q, q + 4, ... (by rank),
        // lane l the words b + 1 + l + 64 k
        unsigned long long acc[SEMTSDF_DET_MAX_BOXES / kB / 64];
#pragma unroll
        for (int k = 0; k < SEMTSDF_DET_MAX_BOXES / kB / 64; ++k) acc[k] = 0ull;
        unsigned long long km = kept;
        int rank = 0;
        while (km) {
            const int r = __builtin_ctzll(km);
            km &= km - 1ull;
            if ((rank++ & 3) != wv) continue;
            const unsigned long long* row = mask + (size_t)(i0 + r) * ncol;
#pragma unroll
            for (int k = 0; k < SEMTSDF_DET_MAX_BOXES / kB / 64; ++k) {
                const int w = b + 1 + lane + 64 * k;
                if (w < ncol) acc[k] |= row[w];
            }
        }
#pragma unroll
        for (int k = 0; k < SEMTSDF_DET_MAX_BOXES / kB / 64; ++k) {
            const int w = b + 1 + lane + 64 * k;
            if (w < ncol && acc[k]) atomicOr(&removed[w], acc[k]);
        }
        __syncthreads();
    }
    const int cnt = s_count;
    for (int k = cnt + t; k < max_out; k += 256) keep[k] = -1;
    if (t == 0) *count = cnt;
}


// PyramidROIAlign (model.py:374-452) over the four pyramid levels P2..P5 [C][H][W] (NCHW, batch 1): the
// output element (roi r, channel c, py, px) samples roi r's own level (lvl[r], 2..5) at the
// crop_and_resize position y = y1 (H - 1) + py ((y2 - y1) (H - 1) / (pool - 1)) (same for x, the
// same f32 operations as the PyTorch formulation), bilinearly in f32, 0 outside [0, H - 1] x [0, W - 1]
// (extrapolation_value).  One thread per output element, px fastest (neighbouring threads read
// neighbouring x of one channel row); only the roi's level is read, where a static-shape PyTorch
// graph samples all four.
struct Levels {
    const void* f[4];
    int H[4], W[4];
};

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }
template <>
__device__ __forceinline__ float to_f<__hip_bfloat16>(__hip_bfloat16 v) { return __bfloat162float(v); }
template <typename T>
__device__ __forceinline__ T from_f(float v);
template <>
__device__ __forceinline__ __half from_f<__half>(float v) { return __float2half(v); }
template <>
__device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

template <typename T>
__global__ __launch_bounds__(256) void k_roi_align(Levels L, int C, const float* __restrict__ rois,
                                                   const int32_t* __restrict__ lvl, int n, int pool,
                                                   T* __restrict__ out) {
    const long long total = (long long)n * C * pool * pool;
    for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total;
         o += (long long)gridDim.x * blockDim.x) {
        const int px = (int)(o % pool), py = (int)((o / pool) % pool);
        const long long rc = o / ((long long)pool * pool);
        const int c = (int)(rc % C), r = (int)(rc / C);
        const int l = min(max(lvl[r], 2), 5) - 2;
        const int H = L.H[l], W = L.W[l];
        const float y1 = rois[4 * r], x1 = rois[4 * r + 1], y2 = rois[4 * r + 2], x2 = rois[4 * r + 3];
        const float hm = (float)(H - 1), wm = (float)(W - 1), pm = (float)(pool - 1);
        const float y = y1 * hm + (float)py * (((y2 - y1) * hm) / pm);
        const float x = x1 * wm + (float)px * (((x2 - x1) * wm) / pm);
        float v = 0.0f;
        if (y >= 0.0f && y <= hm && x >= 0.0f && x <= wm) {
            const T* f = reinterpret_cast<const T*>(L.f[l]) + (size_t)c * H * W;
            const int y0 = (int)floorf(y), x0 = (int)floorf(x);
            const int yb = min(y0 + 1, H - 1), xb = min(x0 + 1, W - 1);
            const float fy = y - (float)y0, fx = x - (float)x0;
            const float v00 = to_f(f[(size_t)y0 * W + x0]), v01 = to_f(f[(size_t)y0 * W + xb]);
            const float v10 = to_f(f[(size_t)yb * W + x0]), v11 = to_f(f[(size_t)yb * W + xb]);
            const float top = v00 * (1.0f - fx) + v01 * fx, bot = v10 * (1.0f - fx) + v11 * fx;
            v = top * (1.0f - fy) + bot * fy;
        }
        out[o] = from_f<T>(v);
    }
}
}  // namespace semtsdf_det

using namespace semtsdf_det;

extern "C" {

int semtsdf_det_abi_version(void) { return SEMTSDF_DET_ABI_VERSION; }

size_t semtsdf_det_nms_workspace(int n) {
    if (n <= 0) return 8;
    const size_t ncol = (size_t)(n + kB - 1) / kB;
    return (size_t)n * ncol * sizeof(unsigned long long);
}

int semtsdf_det_nms(const float* boxes, int n, float iou_threshold, int max_out, int32_t* keep, int32_t* count,
                    void* work, void* stream) {
    if (n < 0 || n > SEMTSDF_DET_MAX_BOXES || max_out < 0 || !keep || !count || (n > 0 && (!boxes || !work)))
        return SEMTSDF_DET_ERR_INVALID;
    if (((uintptr_t)boxes & 15u) != 0) return SEMTSDF_DET_ERR_INVALID;  // float4 rows
    hipStream_t s = (hipStream_t)stream;
    const int ncol = (n + kB - 1) / kB;
    if (n > 0) {
        hipLaunchKernelGGL(k_nms_mask, dim3(ncol, ncol), dim3(kB), 0, s, reinterpret_cast<const float4*>(boxes), n,
                           iou_threshold, ncol, reinterpret_cast<unsigned long long*>(work));
        if (hipGetLastError() != hipSuccess) return SEMTSDF_DET_ERR_HIP;
    }
    hipLaunchKernelGGL(k_nms_sweep, dim3(1), dim3(256), 0, s, reinterpret_cast<const unsigned long long*>(work), n,
                       ncol, max_out, keep, count);
    return hipGetLastError() == hipSuccess ? 0 : SEMTSDF_DET_ERR_HIP;
}

int semtsdf_det_roi_align(const void* const feats[4], const int H[4], const int W[4], int C, const float* rois,
                          const int32_t* lvl, int n, int pool, int dtype, void* out, void* stream) {
    if (!feats || !H || !W || C <= 0 || n < 0 || pool < 2 || (dtype != 0 && dtype != 1) || (n > 0 && (!rois || !lvl || !out)))
        return SEMTSDF_DET_ERR_INVALID;
    Levels L;
    for (int k = 0; k < 4; ++k) {
        if (!feats[k] || H[k] < 2 || W[k] < 2) return SEMTSDF_DET_ERR_INVALID;
        L.f[k] = feats[k];
        L.H[k] = H[k];
        L.W[k] = W[k];
    }
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const long long total = (long long)n * C * pool * pool;
    const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 8192);
    if (dtype == 0)
        hipLaunchKernelGGL(k_roi_align<__half>, dim3(grid), dim3(256), 0, s, L, C, rois, lvl, n, pool,
                           reinterpret_cast<__half*>(out));
    else
        hipLaunchKernelGGL(k_roi_align<__hip_bfloat16>, dim3(grid), dim3(256), 0, s, L, C, rois, lvl, n, pool,
                           reinterpret_cast<__hip_bfloat16*>(out));
    return hipGetLastError() == hipSuccess ? 0 : SEMTSDF_DET_ERR_HIP;
}

}  // extern "C"
