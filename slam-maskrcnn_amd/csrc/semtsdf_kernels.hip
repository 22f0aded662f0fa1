// gfx950 (CDNA4) kernels of the semantic TSDF engine.
//
// Reference semantics (restated, not ported):
//   integrate  — src/SfM_CUDA/tsdf.cu:18-70 (design A, histogram) and
//                src/TSDF_Python/tsdf.cu:10-58 (design B, label vote)
//   association raycast — src/SfM_CUDA/tsdf.cu:72-135 + utils.cu:93-170
//   association accumulation/decision — src/SfM_CUDA/tsdf.cu:304-416
//   render raycast — src/SfM_CUDA/viewer.cu:17-86
//
// Floating-point contract (shared with oracle/semtsdf_oracle.c, which is an independent
// CPU restatement): the whole file is compiled with -ffp-contract=off, every fused
// multiply-add below is written out as fmaf(), divisions are IEEE correctly rounded
// (hipcc default), so the f32 results are reproducible bit for bit on the host.
//   p      = fmaf(idx, voxel, start)                            (tsdf.cu:30)
//   dot3   = fmaf(a2,b2, fmaf(a1,b1, a0*b0))                    (helper_math dot)
//   dot4h  = dot3 + a3                                           (w = 1)
//   mix    = fmaf(t, b, (1-t)*a)                                 (utils.cu:94-96)
//   normalize(v) = v * (1/sqrtf(dot3(v,v)))
//
// Memory layout: every per-voxel array in 1x8x32 (x, y, z) tiles of 256
// consecutive voxels, ordered (z/4, y, z%4) inside the tile (tile_index); the histogram is
// bin-major ([32][voxels]) so lanes that see the same instance label update contiguous words.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <limits.h>
#include <stddef.h>
#include <stdlib.h>
#include "semtsdf_internal.h"
#include "semtsdf_libm.h"

#ifndef SEMTSDF_LAZY_WEIGHT
#define SEMTSDF_LAZY_WEIGHT 0  // lazy weights (k_integrate): measured slower, off by default
#endif

namespace semtsdf {

// ------------------------------------------------------------------------------------
// scalar helpers
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int f2i_rd(float x) {
    // __float2int_rd semantics: floor, saturate, NaN -> 0
    const float f = floorf(x);
    if (!(f == f)) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int)f;
}

__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return fmaf(a2, b2, fmaf(a1, b1, a0 * b0));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));  // packed f32 pairs (v_pk_* on gfx950)

// floor and convert in one VALU operation (v_cvt_flr_i32_f32); callers use it only where
// the operand is finite and far inside the int range
__device__ __forceinline__ int cvt_flr(float x) {
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ float mixf(float a, float b, float t) {
    return fmaf(t, b, (1.0f - t) * a);
}

// RN(a / b) from y = RN(1/b): q0 = RN(a y) is within 1 ulp of a/b, the remainder
// r = a - q0 b is exact (fma), and RN(q0 + r y) = RN(a/b) (Markstein's theorem).  The
// remainder stays a normal number for |a| >= 2^-60 and b in [2^-20, 2^20] (checked
// exhaustively on the host for the mu range, tests/test_oracle_props.py); smaller |a|
// takes the IEEE division, zero keeps its sign.
__device__ __forceinline__ float div_by_rcp(float a, float b, float y) {
    const float q0 = a * y;
    const float r = fmaf(-q0, b, a);
    return fmaf(r, y, q0);
}

// (p - start) / voxel, correctly rounded: reciprocal form (div_by_rcp) with the IEEE
// division for operands too small for it (voxel sizes outside [2^-20, 2^20] are rejected
// at create time).
__device__ __forceinline__ float vox_coord(float p, float start, float voxel, float rvox) {
    const float a = p - start;
    float q = div_by_rcp(a, voxel, rvox);
    // tiny |a| takes the IEEE quotient; the wave-uniform branch keeps the compiler from
    // if-converting the division into every sample (it is rare: a sample within 2^-60 of
    // the volume origin)
    const bool tiny = !(fabsf(a) >= 0x1p-60f);
    if (__builtin_expect(__ballot(tiny) != 0ull, 0)) {
        if (tiny) q = a / voxel;
    }
    return q;
}

// Chunks are dealt to the shards round by round, in boustrophedon order: round r holds chunks
// r n .. r n + n - 1, and shard s owns position s of even rounds and n - 1 - s of odd ones, so
// a work density that drifts along z evens out over pairs of rounds.  Local chunk r of a
// shard is its chunk of round r (only the last round may lack it).
__host__ __device__ __forceinline__ int chunk_pos(int round, int shard, int n) {
#ifdef SEMTSDF_DEAL_RR
    (void)round; (void)n;
    return shard;
#else
    return (round & 1) ? n - 1 - shard : shard;
#endif
}
__host__ __device__ __forceinline__ int chunk_owner(int c, int n) {
    const int r = c / n;
    return chunk_pos(r, c - r * n, n);  // the position map is its own inverse
}

__device__ __forceinline__ int local_to_global_z(const VolGeom& g, int l) {
    if (g.nshards == 1) return l;
    const int per = g.chunk + g.halo;
    const int c = l / per;
    const int w = l - c * per;
    return (c * g.nshards + chunk_pos(c, g.shard, g.nshards)) * g.chunk + w;
}

// Local plane of a global plane owned by this shard (inverse of local_to_global_z).
__device__ __forceinline__ int global_to_local_z(const VolGeom& g, int z) {
    const int c = z / g.chunk;
    return (c / g.nshards) * (g.chunk + g.halo) + (z - c * g.chunk);
}

// Shard owning the trilinear sample at world z `pz` (its base plane, clamped as the
// sampler clamps it).
__device__ __forceinline__ int sample_owner(const VolGeom& g, float pz) {
    const float iz = vox_coord(pz, g.start[2], g.voxel[2], g.rvox[2]);
    const int zc = min(max(f2i_rd(iz), 0), g.dimz - 1);
    return chunk_owner(zc / g.chunk, g.nshards);
}

// Project one voxel (reference tsdf.cu:30-44).  Returns camera-space z in *qz and the
// pixel in *px/*py.
__device__ __forceinline__ void project_voxel(const float* __restrict__ E, const float* __restrict__ K,
                                              float px, float py, float pz,
                                              float* qz_out, int* ix, int* iy) {
    const float qx = dot3(E[0], E[1], E[2], px, py, pz) + E[3];
    const float qy = dot3(E[4], E[5], E[6], px, py, pz) + E[7];
    const float qz = dot3(E[8], E[9], E[10], px, py, pz) + E[11];
    const float sx = dot3(K[0], K[1], K[2], qx, qy, qz);
    const float sy = dot3(K[3], K[4], K[5], qx, qy, qz);
    const float sz = dot3(K[6], K[7], K[8], qx, qy, qz);
    *qz_out = qz;
    *ix = f2i_rd(sx / sz);
    *iy = f2i_rd(sy / sz);
}

// ------------------------------------------------------------------------------------
// volume fill: sdf := mu (tsdf.cu:243-244).  Zeros are hipMemsetAsync'd by the host.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fill_f32(float* __restrict__ p, uint64_t n, float v) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 4 <= n) {
            *reinterpret_cast<float4*>(p + i) = make_float4(v, v, v, v);
        } else {
            for (uint64_t k = i; k < n; ++k) p[k] = v;
        }
    }
}

// Achievable-bandwidth probe (semtsdf_copy_bandwidth, the bench's hbm_copy_gbs).
typedef float f32x4 __attribute__((ext_vector_type(4)));
// One float4 per thread and one pass over the grid (n/256 workgroups): the shape that
// reaches the achievable copy rate (6.2 TB/s on MI355X, tools/copybench.hip; persistent
// grid-stride loops stay at 4.2-5.3 TB/s whatever their unroll, grid or cache policy).
__global__ __launch_bounds__(256) void k_copy_f4(const f32x4* __restrict__ a, f32x4* __restrict__ b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

hipError_t launch_copy_f4(const void* src, void* dst, size_t n16, hipStream_t s) {
    size_t blocks = (n16 + 255) / 256;
    if (blocks > 0x7FFFFFFFu) blocks = 0x7FFFFFFFu;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_copy_f4, dim3((unsigned)blocks), dim3(256), 0, s, (const f32x4*)src, (f32x4*)dst, n16);
    return hipGetLastError();
}

// Copy from device-accessible host memory (pinned) by a kernel on a few CUs: the runtime's DMA
// copy from pinned memory measured as blocking the calling thread for the whole transfer while
// the volume's kernels run (tools/host_overhead.py), which stalls a host loop feeding frames.
hipError_t launch_copy_host(const void* src, void* dst, size_t n16, hipStream_t s) {
    if (n16 == 0) return hipSuccess;
    size_t blocks = (n16 + 255) / 256;
    if (blocks > 64) blocks = 64;
    hipLaunchKernelGGL(k_copy_f4, dim3((unsigned)blocks), dim3(256), 0, s, (const f32x4*)src, (f32x4*)dst, n16);
    return hipGetLastError();
}

// dst[i] = min(dst[i], src[i]) over int64: the in-process stand-in of an all-reduce MIN
// (shards driven from one process, semtsdf_min_i64)
__global__ __launch_bounds__(256) void k_min_i64(long long* __restrict__ dst, const long long* __restrict__ src, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = min(dst[i], src[i]);
}

hipError_t launch_min_i64(long long* dst, const long long* src, size_t n, hipStream_t s) {
    size_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_min_i64, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, n);
    return hipGetLastError();
}

// Empty-space map, in two passes.  k_brick_plain: one wave per 8^3 brick (lane = one of
// its 64 (x, y) rows, two float4 loads) writes the min of sdf over the brick's own voxels;
// with all == 0 only bricks the integrate marked dirty are recomputed (a voxel of theirs
// crossed the skip threshold, the only change that can flip the map; the stale minima of
// the other bricks stay on their side of it).  k_brick_dilate: bmin[b] = min of the
// plain map over b + {0,1}^3, which covers [8b, 8b + 8] per axis: every voxel a trilinear
// sample based in brick b reads.
// One wave per 4 z-consecutive bricks (a quad): lane = one (x, y) row of 32 voxels = one
// whole 128-B line (a row of a single brick is only 32 B of a line).  `want` bit j: recompute
// brick 4q + j.
__device__ __forceinline__ void brick_quad_min(const VolGeom& g, const float* __restrict__ sdf,
                                               float* __restrict__ plain, unsigned q, unsigned want) {
    const unsigned nbq = (unsigned)(g.nbz + 3) / 4;
    const int lane = threadIdx.x & 63;
    const int bq = q % nbq, by = (q / nbq) % g.nby, bx = q / (nbq * g.nby);
    const unsigned br0 = ((unsigned)bx * g.nby + (unsigned)by) * g.nbz + (unsigned)bq * 4;
    const int nbr = min(4, g.nbz - bq * 4);
    const int x = bx * 8 + (lane >> 3), y = by * 8 + (lane & 7), z0 = bq * 32;
    float m[4] = {3.0e38f, 3.0e38f, 3.0e38f, 3.0e38f};
    if (x < g.dimx && y < g.dimy) {
        // the row's 32 planes are the tile's 8 z-quads, 32 floats apart (8 y-lanes = one line)
        const float* p = sdf + tile_index(g, x, y, z0);
        if (z0 + 32 <= g.lz) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 a = *reinterpret_cast<const float4*>(p + 64 * j);
                const float4 c = *reinterpret_cast<const float4*>(p + 64 * j + 32);
                m[j] = fminf(fminf(fminf(a.x, a.y), fminf(a.z, a.w)), fminf(fminf(c.x, c.y), fminf(c.z, c.w)));
            }
        } else {
            for (int k = 0; k < g.lz - z0; ++k) {
                const float v = p[tile_zterm(k)];
#pragma unroll
                for (int j = 0; j < 4; ++j) m[j] = (k >> 3) == j ? fminf(m[j], v) : m[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        for (int off = 32; off > 0; off >>= 1) m[j] = fminf(m[j], __shfl_xor(m[j], off, 64));
    if (lane < nbr && ((want >> lane) & 1u)) {
        const float mj = lane == 0 ? m[0] : lane == 1 ? m[1] : lane == 2 ? m[2] : m[3];
        plain[br0 + lane] = mj;
    }
}

// all: every quad (one wave each).  Else the quads on the dirty list (dlist[0] entries from
// dlist[1]; the integrate appends a quad when its dirty word turns nonzero), grid-strided.
// Both clear the dirty words; k_brick_dilate, next on the stream, resets the list.
__global__ __launch_bounds__(256) void k_brick_plain(VolGeom g, const float* __restrict__ sdf, float* __restrict__ plain,
                                                     uint32_t* __restrict__ dirty, const uint32_t* __restrict__ dlist,
                                                     int all) {
    const unsigned nbq = (unsigned)(g.nbz + 3) / 4;
    const unsigned nq = (unsigned)g.nbx * g.nby * nbq;
    const unsigned w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (all) {
        if (w0 >= nq) return;
        brick_quad_min(g, sdf, plain, w0, 0xFu);
        if ((threadIdx.x & 63) == 0) dirty[w0] = 0u;
        return;
    }
    const unsigned n = dlist[0];
    for (unsigned i = w0; i < n; i += gridDim.x * 4) {
        const unsigned q = dlist[1 + i];
        const unsigned want = dirty[q];
        brick_quad_min(g, sdf, plain, q, want);
        if ((threadIdx.x & 63) == 0) dirty[q] = 0u;
    }
}

__device__ __forceinline__ float skip_threshold(const VolGeom& g);

#ifndef SEMTSDF_BRICK_DIST
#define SEMTSDF_BRICK_DIST 1
#endif
#ifndef SEMTSDF_BRICK_OCT
#define SEMTSDF_BRICK_OCT 1  // unsharded marches use the octant boxes of their direction
#endif

__global__ __launch_bounds__(256) void k_brick_dilate(VolGeom g, const float* __restrict__ plain, float* __restrict__ bmin,
                                                      uint64_t* __restrict__ d0, uint32_t* __restrict__ dlist) {
    const unsigned nb = (unsigned)g.nbx * g.nby * g.nbz;
    const unsigned br = blockIdx.x * blockDim.x + threadIdx.x;
    if (br == 0) dlist[0] = 0u;  // k_brick_plain has consumed the dirty list
    if (br >= nb) return;
    const int bz = br % g.nbz, by = (br / g.nbz) % g.nby, bx = br / (g.nbz * g.nby);
    float m = 3.0e38f;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                const int xx = bx + i, yy = by + j, zz = bz + k;
                if (xx < g.nbx && yy < g.nby && zz < g.nbz) m = fminf(m, plain[((unsigned)xx * g.nby + yy) * g.nbz + zz]);
            }
    bmin[br] = m;
    if (d0) d0[br] = m >= skip_threshold(g) ? (uint64_t)kBrickDistCap * 0x0101010101010101ull : 0ull;
}

// Octant brick distance maps, one axis per pass: for octant o (bit a set: negative along axis
// a) out_o[b] = min over 0 <= k < cap of max(k, in_o[b + s k e]), s the octant's sign on this
// axis (neighbours inside the volume).  Three passes (x, y, z) from d0 (0 = not skippable, cap
// = skippable, in every byte) give, per octant, the L-inf distance to the nearest non-skippable
// brick of that octant, capped: the box of the d bricks from b on along each of the octant's
// directions is skippable.  The last pass also writes the symmetric distance (the min over
// the octants: every brick lies in some octant of b) for the sharded march.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));  // v_pk_*_u16 operands

// Octant bytes of a map word in four packed registers of two u16 lanes: R[0] = octants (0, 2),
// R[1] = (1, 3) from the low dword, R[2] = (4, 6), R[3] = (5, 7) from the high dword.  For a
// pass along AXIS, octant o takes its neighbour word from wn (negative side) when bit AXIS of
// o is set, else from wp.
template <int AXIS>
__device__ __forceinline__ void oct_unpack(uint64_t wp, uint64_t wn, u16x2 R[4]) {
    const uint32_t pl = (uint32_t)wp, ph = (uint32_t)(wp >> 32), nl = (uint32_t)wn, nh = (uint32_t)(wn >> 32);
    uint32_t r0, r1, r2, r3;
    if (AXIS == 0) {  // odd octants negative
        r0 = pl & 0x00FF00FFu; r1 = (nl >> 8) & 0x00FF00FFu;
        r2 = ph & 0x00FF00FFu; r3 = (nh >> 8) & 0x00FF00FFu;
    } else if (AXIS == 1) {  // octants 2, 3, 6, 7 negative: the high lane of every register
        r0 = (pl & 0x000000FFu) | (nl & 0x00FF0000u); r1 = ((pl >> 8) & 0x000000FFu) | ((nl >> 8) & 0x00FF0000u);
        r2 = (ph & 0x000000FFu) | (nh & 0x00FF0000u); r3 = ((ph >> 8) & 0x000000FFu) | ((nh >> 8) & 0x00FF0000u);
    } else {  // octants 4..7 negative: the high dword
        r0 = pl & 0x00FF00FFu; r1 = (pl >> 8) & 0x00FF00FFu;
        r2 = nh & 0x00FF00FFu; r3 = (nh >> 8) & 0x00FF00FFu;
    }
    R[0] = __builtin_bit_cast(u16x2, r0); R[1] = __builtin_bit_cast(u16x2, r1);
    R[2] = __builtin_bit_cast(u16x2, r2); R[3] = __builtin_bit_cast(u16x2, r3);
}

// One axis pass of the octant distance maps (see above), the 8 octants as packed u16 lanes
// (v_pk_max_u16 / v_pk_min_u16: 2 octants per operation).
template <int AXIS>
__global__ __launch_bounds__(256) void k_brick_oct_axis(VolGeom g, const uint64_t* __restrict__ in,
                                                        uint64_t* __restrict__ out, uint8_t* __restrict__ sym) {
    const unsigned nb = (unsigned)g.nbx * g.nby * g.nbz;
    const unsigned br = blockIdx.x * blockDim.x + threadIdx.x;
    if (br >= nb) return;
    const int bz = br % g.nbz, by = (br / g.nbz) % g.nby, bx = br / (g.nbz * g.nby);
    const int pos = AXIS == 0 ? bx : AXIS == 1 ? by : bz;
    const int n = AXIS == 0 ? g.nbx : AXIS == 1 ? g.nby : g.nbz;
    const int stride = AXIS == 0 ? g.nby * g.nbz : AXIS == 1 ? g.nbz : 1;
    const uint64_t v = in[br];
    u16x2 d[4];
    oct_unpack<0>(v, v, d);  // the brick's own word (both sides the same): plain unpack
    auto hmax = [](const u16x2* x) {
        const u16x2 m = __builtin_elementwise_max(__builtin_elementwise_max(x[0], x[1]),
                                                  __builtin_elementwise_max(x[2], x[3]));
        return (int)max(m.x, m.y);
    };
    int dmax = hmax(d);
    // neighbours in chunks of 4 (loads in flight together; a k >= every d[o] changes nothing,
    // so the chunk may run past dmax)
    for (int k0 = 1; k0 < kBrickDistCap && k0 < dmax; k0 += 4) {
        uint64_t wp[4], wn[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = k0 + i;
            wp[i] = (k < kBrickDistCap && pos + k < n) ? in[(int)br + k * stride] : ~0ull;   // octants positive on axis
            wn[i] = (k < kBrickDistCap && pos - k >= 0) ? in[(int)br - k * stride] : ~0ull;  // octants negative on axis
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u16x2 w[4];
            oct_unpack<AXIS>(wp[i], wn[i], w);
            const u16x2 kk = {(unsigned short)(k0 + i), (unsigned short)(k0 + i)};
#pragma unroll
            for (int j = 0; j < 4; ++j) d[j] = __builtin_elementwise_min(d[j], __builtin_elementwise_max(w[j], kk));
        }
        dmax = hmax(d);
    }
    // repack: byte o of the word = octant o
    const uint32_t lo = (uint32_t)d[0].x | ((uint32_t)d[1].x << 8) | ((uint32_t)d[0].y << 16) | ((uint32_t)d[1].y << 24);
    const uint32_t hi = (uint32_t)d[2].x | ((uint32_t)d[3].x << 8) | ((uint32_t)d[2].y << 16) | ((uint32_t)d[3].y << 24);
    out[br] = (uint64_t)lo | ((uint64_t)hi << 32);
    if (sym) {
        const u16x2 m = __builtin_elementwise_min(__builtin_elementwise_min(d[0], d[1]),
                                                  __builtin_elementwise_min(d[2], d[3]));
        sym[br] = (uint8_t)min(min((int)m.x, (int)m.y), kBrickDistCap);
    }
}

// The octant maps through LDS, one launch per axis, with the dilation folded in.  A workgroup
// holds L whole lines of n bricks along the pass's axis (lines adjacent in memory, so loads and
// stores coalesce); the neighbour scans then read LDS instead of re-reading the map.  The
// dilation k_brick_dilate applies before the passes (min over b + {0,1}^3, here per octant byte:
// skippable iff every brick of the 2x2x2 box is) is separable into a min with the +1 neighbour
// along each axis, and each of those commutes with the passes along the other axes (a min over
// a shift along one axis, a min-max over another: max distributes over min), so the pass along
// axis A first takes the min with the +1 neighbour along A and then scans: the three passes give
// exactly the maps of k_brick_dilate + k_brick_oct_axis x3.  The first pass reads the plain map
// (FIRST: skippable = plain >= thr); bmin (the float dilated map, read only by volumes without
// octant maps) is not kept on this path.  Dynamic LDS: 2 n L words.
template <int AXIS, bool FIRST>
__global__ __launch_bounds__(256) void k_brick_oct_lds(VolGeom g, const void* __restrict__ in_, uint64_t* __restrict__ out,
                                                       uint8_t* __restrict__ sym, uint32_t* __restrict__ dlist, int L) {
    extern __shared__ uint64_t s_map[];  // raw [n][L], then dilated [n][L]
    const int n = AXIS == 0 ? g.nbx : AXIS == 1 ? g.nby : g.nbz;
    const unsigned S = AXIS == 0 ? (unsigned)g.nby * g.nbz : AXIS == 1 ? (unsigned)g.nbz : 1u;
    const unsigned nlines = AXIS == 0 ? (unsigned)g.nby * g.nbz : AXIS == 1 ? (unsigned)g.nbx * g.nbz : (unsigned)g.nbx * g.nby;
    const unsigned q0 = blockIdx.x * (unsigned)L;
    const int ne = n * L;
    uint64_t* raw = s_map;
    uint64_t* dil = s_map + ne;
    if (FIRST && dlist && blockIdx.x == 0 && threadIdx.x == 0) dlist[0] = 0u;  // k_brick_plain consumed the dirty list
    auto base = [&](unsigned q) -> unsigned {  // first brick of line q
        if (AXIS == 0) return q;                                                // (by, bz)
        if (AXIS == 1) return (q / (unsigned)g.nbz) * (unsigned)g.nby * g.nbz + q % (unsigned)g.nbz;  // (bx, bz)
        return q * (unsigned)g.nbz;                                             // (bx, by)
    };
    // element e <-> (k along the line, l = line): along z the lines are contiguous (k fastest),
    // else adjacent lines are adjacent in memory (l fastest)
    auto split = [&](int e, int& k, int& l) {
        if (AXIS == 2) { k = e % n; l = e / n; } else { k = e / L; l = e - (e / L) * L; }
    };
    const float thr = skip_threshold(g);
    for (int e = (int)threadIdx.x; e < ne; e += 256) {
        int k, l;
        split(e, k, l);
        const unsigned q = q0 + (unsigned)l;
        uint64_t w = 0ull;
        if (q < nlines) {
            const unsigned br = base(q) + (unsigned)k * S;
            if (FIRST) w = reinterpret_cast<const float*>(in_)[br] >= thr ? (uint64_t)kBrickDistCap * 0x0101010101010101ull : 0ull;
            else w = reinterpret_cast<const uint64_t*>(in_)[br];
        }
        raw[k * L + l] = w;
    }
    __syncthreads();
    for (int e = (int)threadIdx.x; e < ne; e += 256) {  // the +1 neighbour along the axis (inside the volume)
        int k, l;
        split(e, k, l);
        uint64_t w = raw[k * L + l];
        if (k + 1 < n) {
            u16x2 a[4], b[4];
            oct_unpack<0>(w, w, a);
            const uint64_t v = raw[(k + 1) * L + l];
            oct_unpack<0>(v, v, b);
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = __builtin_elementwise_min(a[j], b[j]);
            const uint32_t lo = (uint32_t)a[0].x | ((uint32_t)a[1].x << 8) | ((uint32_t)a[0].y << 16) | ((uint32_t)a[1].y << 24);
            const uint32_t hi = (uint32_t)a[2].x | ((uint32_t)a[3].x << 8) | ((uint32_t)a[2].y << 16) | ((uint32_t)a[3].y << 24);
            w = (uint64_t)lo | ((uint64_t)hi << 32);
        }
        dil[k * L + l] = w;
    }
    __syncthreads();
    auto hmax = [](const u16x2* x) {
        const u16x2 m = __builtin_elementwise_max(__builtin_elementwise_max(x[0], x[1]), __builtin_elementwise_max(x[2], x[3]));
        return (int)max(m.x, m.y);
    };
    for (int e = (int)threadIdx.x; e < ne; e += 256) {
        int k, l;
        split(e, k, l);
        const unsigned q = q0 + (unsigned)l;
        const uint64_t v = dil[k * L + l];
        u16x2 d[4];
        oct_unpack<0>(v, v, d);
        int dmax = hmax(d);
        for (int k0 = 1; k0 < kBrickDistCap && k0 < dmax; k0 += 4) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int kk = k0 + i;
                const uint64_t wp = (kk < kBrickDistCap && k + kk < n) ? dil[(k + kk) * L + l] : ~0ull;
                const uint64_t wn = (kk < kBrickDistCap && k - kk >= 0) ? dil[(k - kk) * L + l] : ~0ull;
                u16x2 w[4];
                oct_unpack<AXIS>(wp, wn, w);
                const u16x2 kv = {(unsigned short)kk, (unsigned short)kk};
#pragma unroll
                for (int j = 0; j < 4; ++j) d[j] = __builtin_elementwise_min(d[j], __builtin_elementwise_max(w[j], kv));
            }
            dmax = hmax(d);
        }
        if (q < nlines) {
            const unsigned br = base(q) + (unsigned)k * S;
            const uint32_t lo = (uint32_t)d[0].x | ((uint32_t)d[1].x << 8) | ((uint32_t)d[0].y << 16) | ((uint32_t)d[1].y << 24);
            const uint32_t hi = (uint32_t)d[2].x | ((uint32_t)d[3].x << 8) | ((uint32_t)d[2].y << 16) | ((uint32_t)d[3].y << 24);
            out[br] = (uint64_t)lo | ((uint64_t)hi << 32);
            if (sym) {
                const u16x2 m = __builtin_elementwise_min(__builtin_elementwise_min(d[0], d[1]), __builtin_elementwise_min(d[2], d[3]));
                sym[br] = (uint8_t)min(min((int)m.x, (int)m.y), kBrickDistCap);
            }
        }
    }
}

// Super-brick level: sbmin[s] = min of bmin over the (up to) 8^3 bricks of super-brick s,
// so it bounds every trilinear sample based in its 64^3 voxels.  One wave per super-brick.
__global__ __launch_bounds__(256) void k_brick_super(VolGeom g, const float* __restrict__ bmin, float* __restrict__ sbmin) {
    const unsigned ns = (unsigned)g.nsx * g.nsy * g.nsz;
    const unsigned sb = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (sb >= ns) return;
    const int lane = threadIdx.x & 63;
    const int sz = sb % g.nsz, sy = (sb / g.nsz) % g.nsy, sx = sb / (g.nsz * g.nsy);
    float m = 3.0e38f;
    const int bx = sx * 8 + (lane >> 3), by = sy * 8 + (lane & 7);  // lane = one (x, y) brick column
    if (bx < g.nbx && by < g.nby)
        for (int k = 0; k < 8 && sz * 8 + k < g.nbz; ++k)
            m = fminf(m, bmin[((unsigned)bx * g.nby + (unsigned)by) * g.nbz + (unsigned)(sz * 8 + k)]);
    for (int off = 32; off > 0; off >>= 1) m = fminf(m, __shfl_xor(m, off, 64));
    if (lane == 0) sbmin[sb] = m;
}

// Lines per workgroup of k_brick_oct_lds for lines of n bricks (0: too long, global passes).
static int oct_lds_lines(int n) { return n > 1024 ? 0 : n >= 512 ? 1 : 512 / n; }

hipError_t launch_brick_min(const VolGeom& g, const VolBufs& b, bool all, hipStream_t s, bool global_passes) {
    const unsigned nb = (unsigned)g.nbx * g.nby * g.nbz;
    if (nb == 0) return hipSuccess;
    const unsigned nq = (unsigned)g.nbx * g.nby * (unsigned)((g.nbz + 3) / 4);
    const unsigned nw = all ? nq : (nq < 4096u ? nq : 4096u);  // waves (list mode: grid-strided)
    hipLaunchKernelGGL(k_brick_plain, dim3((nw + 3) / 4), dim3(256), 0, s, g, b.sdf, b.bplain, b.bdirty, b.dlist,
                       all ? 1 : 0);
    const bool dist = SEMTSDF_BRICK_DIST && b.bdist && b.boct && b.botmp;
    const int Lx = oct_lds_lines(g.nbx), Ly = oct_lds_lines(g.nby), Lz = oct_lds_lines(g.nbz);
    if (dist && !global_passes && Lx && Ly && Lz) {  // plain -> x -> boct -> y -> botmp -> z -> boct (+ bdist)
        const unsigned lx = (unsigned)g.nby * g.nbz, ly = (unsigned)g.nbx * g.nbz, lz = (unsigned)g.nbx * g.nby;
        hipLaunchKernelGGL((k_brick_oct_lds<0, true>), dim3((lx + Lx - 1) / Lx), dim3(256), 2 * g.nbx * Lx * 8, s, g,
                           (const void*)b.bplain, b.boct, (uint8_t*)nullptr, b.dlist, Lx);
        hipLaunchKernelGGL((k_brick_oct_lds<1, false>), dim3((ly + Ly - 1) / Ly), dim3(256), 2 * g.nby * Ly * 8, s, g,
                           (const void*)b.boct, b.botmp, (uint8_t*)nullptr, (uint32_t*)nullptr, Ly);
        hipLaunchKernelGGL((k_brick_oct_lds<2, false>), dim3((lz + Lz - 1) / Lz), dim3(256), 2 * g.nbz * Lz * 8, s, g,
                           (const void*)b.botmp, b.boct, b.bdist, (uint32_t*)nullptr, Lz);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_brick_dilate, dim3((nb + 255) / 256), dim3(256), 0, s, g, b.bplain, b.bmin,
                       dist ? b.botmp : nullptr, b.dlist);
    if (dist) {  // d0 in botmp -> x -> boct -> y -> botmp -> z -> boct (+ bdist)
        hipLaunchKernelGGL(k_brick_oct_axis<0>, dim3((nb + 255) / 256), dim3(256), 0, s, g, b.botmp, b.boct, nullptr);
        hipLaunchKernelGGL(k_brick_oct_axis<1>, dim3((nb + 255) / 256), dim3(256), 0, s, g, b.boct, b.botmp, nullptr);
        hipLaunchKernelGGL(k_brick_oct_axis<2>, dim3((nb + 255) / 256), dim3(256), 0, s, g, b.botmp, b.boct, b.bdist);
    } else {
        const unsigned ns = (unsigned)g.nsx * g.nsy * g.nsz;
        if (b.sbmin && ns) hipLaunchKernelGGL(k_brick_super, dim3((ns + 3) / 4), dim3(256), 0, s, g, b.bmin, b.sbmin);
    }
    return hipGetLastError();
}

// Folds the pending weight increments of steady lines into the weights (k_integrate's lazy
// weights): one lane per voxel, the 32 voxels of a line in one half-wave, which reads the flag
// byte before its first lane resets it (loads of one wave-instruction precede its stores).
__global__ __launch_bounds__(256) void k_flush_lazy(int32_t* __restrict__ wt, uint8_t* __restrict__ sflag, uint64_t nvox) {
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < nvox; v += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned f = sflag[v >> 5];
        if (f > 1u) {
            wt[v] += (int)f - 1;
            if ((v & 31u) == 0u) sflag[v >> 5] = 1u;
        }
    }
}

hipError_t launch_flush_lazy(const VolGeom& g, const VolBufs& b, hipStream_t s) {
    if (!SEMTSDF_LAZY_WEIGHT) return hipSuccess;  // no pending counts exist in this build
    const uint64_t n = g.nvox;
    if (n == 0) return hipSuccess;  // a shard that owns no chunk
    const unsigned grid = (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
    hipLaunchKernelGGL(k_flush_lazy, dim3(grid), dim3(256), 0, s, b.wt, b.sflag, n);
    return hipGetLastError();
}

hipError_t launch_fill_volume(const VolGeom& g, const VolBufs& b, uint32_t flags, hipStream_t s) {
    (void)flags;
    const uint64_t n = g.nvox;
    uint64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_fill_f32, dim3((unsigned)blocks), dim3(256), 0, s, b.sdf, n, g.mu);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// frame prepass: depth in metres, rgb+label packed per pixel, and max raw depth over 8- and
// 32-pixel tiles for unit culling.  One workgroup per 32x32 pixel tile; lane = (row,
// 4 columns), loaded as one 8-B depth vector, one 4-B mask word and three 4-B rgb words
// when the rows are 4-pixel aligned (vec), else pixel by pixel.
// ------------------------------------------------------------------------------------
// lut (optional): the association's relabel table (k_relabel folded in): labels are mapped
// through it and the relabelled mask is written back in place.
// One 32x32-pixel tile (tx, ty) of the prepass, a whole workgroup (k_depth_pyramid, and the
// prepass blocks of k_march_fused).
__device__ __forceinline__ void pyramid_tile(const uint16_t* __restrict__ depth, const uint8_t* __restrict__ rgb,
                                             uint8_t* mask, int w, int h, float scale, int vec, const DepthPyramid& p,
                                             unsigned* list_count, const uint8_t* __restrict__ lut, int tx, int ty) {
    const int t = threadIdx.x;
    __shared__ uint32_t s_lut[64];
    if (lut) {  // uniform
        if (t < 64) s_lut[t] = reinterpret_cast<const uint32_t*>(lut)[t];
        __syncthreads();
    }
    auto relab = [&](unsigned m) { return (s_lut[m >> 2] >> (8 * (m & 3))) & 0xFFu; };
    if (list_count && tx == 0 && ty == 0 && t < kLists * kListSegs)  // this frame's lists (general, free, full)
        list_count[(t & (kListSegs - 1)) * kListCountStride + (t >> 6) * kListSegs * kListCountStride] = 0u;
    if (list_count && tx == 0 && ty == 0 && t < kDynCounters)  // the integrate's dynamic counters
        list_count[(kLists * kListSegs + t) * kListCountStride] = 0u;
    const int r = t >> 3;          // row in tile
    const int c4 = (t & 7) * 4;    // first column in tile
    const int yy = ty * 32 + r;
    const int x0 = tx * 32 + c4;
    // m: max raw depth; n: 0xFFFF - min nonzero raw depth (0: no nonzero pixel); both reduce by
    // max; z: 1 when a pixel of the lane has depth 0 (reduces by max too)
    unsigned m = 0, n = 0, z = 0;
    if (yy < h && x0 < w) {
        const size_t px0 = (size_t)yy * w + x0;
        if (vec && x0 + 3 < w) {
            const ushort4 d4 = *reinterpret_cast<const ushort4*>(depth + px0);
            const unsigned d[4] = {d4.x, d4.y, d4.z, d4.w};
            m = max(max(d[0], d[1]), max(d[2], d[3]));
#pragma unroll
            for (int k = 0; k < 4; ++k) n = max(n, d[k] ? 0xFFFFu - d[k] : 0u);
            z = (d[0] == 0u) | (d[1] == 0u) | (d[2] == 0u) | (d[3] == 0u);
            uint4 o = make_uint4(0, 0, 0, 0);
            if (rgb) {
                const uint32_t* c = reinterpret_cast<const uint32_t*>(rgb + px0 * 3);
                const uint32_t c0 = c[0], c1 = c[1], c2 = c[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
                uint32_t lab = mask ? *reinterpret_cast<const uint32_t*>(mask + px0) : 0u;
                if (lut && mask) {
                    lab = relab(lab & 0xFFu) | (relab((lab >> 8) & 0xFFu) << 8) | (relab((lab >> 16) & 0xFFu) << 16) |
                          (relab(lab >> 24) << 24);
                    *reinterpret_cast<uint32_t*>(mask + px0) = lab;
                }
                o.x = (c0 & 0xFFFFFFu) | ((lab & 0xFFu) << 24);
                o.y = (c0 >> 24) | ((c1 & 0xFFFFu) << 8) | (((lab >> 8) & 0xFFu) << 24);
                o.z = (c1 >> 16) | ((c2 & 0xFFu) << 16) | (((lab >> 16) & 0xFFu) << 24);
                o.w = (c2 >> 8) | ((lab >> 24) << 24);
            }
            // depth[img] / 5000.f (tsdf.cu:49), once per pixel; x0 % 4 == 0: one row of a tile,
            // records 4 apart (a tile is column-major)
            uint2* dst = p.px + rec_index(p, (unsigned)x0, (unsigned)yy);
            dst[0] = make_uint2(__float_as_uint((float)d[0] / scale), o.x);
            dst[4] = make_uint2(__float_as_uint((float)d[1] / scale), o.y);
            dst[8] = make_uint2(__float_as_uint((float)d[2] / scale), o.z);
            dst[12] = make_uint2(__float_as_uint((float)d[3] / scale), o.w);
        } else {
            for (int k = 0; k < 4 && x0 + k < w; ++k) {
                const size_t px = px0 + k;
                const unsigned d = depth[px];
                m = max(m, d);
                n = max(n, d ? 0xFFFFu - d : 0u);
                z |= d == 0u ? 1u : 0u;
                unsigned c = 0;
                if (rgb) {
                    unsigned lab = mask ? (unsigned)mask[px] : 0u;
                    if (lut && mask) {
                        lab = relab(lab);
                        mask[px] = (uint8_t)lab;
                    }
                    c = (unsigned)rgb[px * 3] | ((unsigned)rgb[px * 3 + 1] << 8) | ((unsigned)rgb[px * 3 + 2] << 16) |
                        (lab << 24);
                }
                p.px[rec_index(p, (unsigned)(x0 + k), (unsigned)yy)] = make_uint2(__float_as_uint((float)d / scale), c);
            }
        }
    }
    // wave w holds rows 8w..8w+7: the level-0 tiles (w, 0..3), each the lanes with
    // (t & 7) >> 1 == bcol; reduce over lane bits 0, 3, 4, 5 in registers
#pragma unroll
    for (int b : {1, 8, 16, 32}) {
        m = max(m, (unsigned)__shfl_xor((int)m, b));
        n = max(n, (unsigned)__shfl_xor((int)n, b));
        z = max(z, (unsigned)__shfl_xor((int)z, b));
    }
    const int wv = t >> 6, ln = t & 63;
    if (ln < 8 && (ln & 1) == 0) {
        const int gx0 = tx * 4 + (ln >> 1), gy0 = ty * 4 + wv;
        if (gx0 < p.w0 && gy0 < p.h0) p.l0[gy0 * p.w0 + gx0] = make_uint2(m | (n << 16), z);
    }
#pragma unroll
    for (int b : {2, 4}) {
        m = max(m, (unsigned)__shfl_xor((int)m, b));
        n = max(n, (unsigned)__shfl_xor((int)n, b));
        z = max(z, (unsigned)__shfl_xor((int)z, b));
    }
    __shared__ unsigned s_w[4], s_n[4], s_z[4];
    if (ln == 0) { s_w[wv] = m; s_n[wv] = n; s_z[wv] = z; }
    __syncthreads();
    if (t == 0)
        p.l1[ty * p.w1 + tx] = make_uint2(max(max(s_w[0], s_w[1]), max(s_w[2], s_w[3])) |
                                              (max(max(s_n[0], s_n[1]), max(s_n[2], s_n[3])) << 16),
                                          max(max(s_z[0], s_z[1]), max(s_z[2], s_z[3])));
}

__global__ __launch_bounds__(256) void k_depth_pyramid(const uint16_t* __restrict__ depth, const uint8_t* __restrict__ rgb,
                                                       uint8_t* mask, int w, int h, float scale,
                                                       int vec, DepthPyramid p, unsigned* list_count,
                                                       const uint8_t* __restrict__ lut) {
    pyramid_tile(depth, rgb, mask, w, h, scale, vec, p, list_count, lut, (int)blockIdx.x, (int)blockIdx.y);
}

// Whether the prepass may use its vector path (4-pixel rows aligned).
int depth_pyramid_vec(const uint16_t* depth, const uint8_t* rgb, const uint8_t* mask, int w, const DepthPyramid& p) {
    return (w % 4 == 0) && ((uintptr_t)depth % 8 == 0) && (!rgb || (uintptr_t)rgb % 4 == 0) &&
           (!mask || (uintptr_t)mask % 4 == 0);
}

hipError_t launch_depth_pyramid(const uint16_t* depth, const uint8_t* rgb, uint8_t* mask, int w, int h,
                                float scale, const DepthPyramid& p, unsigned* list_count, hipStream_t s,
                                const uint8_t* lut) {
    const bool vec = depth_pyramid_vec(depth, rgb, mask, w, p);
    hipLaunchKernelGGL(k_depth_pyramid, dim3(p.w1, p.h1), dim3(256), 0, s, depth, rgb, mask, w, h, scale,
                       vec ? 1 : 0, p, list_count, lut);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// integrate
// ------------------------------------------------------------------------------------
// ---- work decomposition ------------------------------------------------------------
// Cull unit = UX(x) x UY(y) x UZ(z) voxels, tested once per frame by one lane of the cull
// pass against the frustum and the depth pyramid.  A wavefront integrates kSlots units at
// a time: lane = (slot, y, zq) owns planes 4zq..4zq+3 of row (x, y) of its slot's unit, so
// every state access is one 16-byte vector per lane and the 8 y-lanes of one z-quad cover
// one 128-B line of the tiled layout.  Half tiles (1 x 8 x 16, two per wave) visit 16 %
// fewer voxels than whole tiles (the cull is near exact at unit resolution: 23.5 M against
// 28.0 M visited voxels per 512^3 frame) and measured 14 % faster; quarter tiles visit 5 %
// fewer again but the cull of 4x as many units costs more than that saves.
#ifndef SEMTSDF_UNIT_X
#define SEMTSDF_UNIT_X 1
#define SEMTSDF_UNIT_Y 8
#define SEMTSDF_UNIT_Z 16
#endif
constexpr int UX = SEMTSDF_UNIT_X, UY = SEMTSDF_UNIT_Y, UZ = SEMTSDF_UNIT_Z;
// Timing probes of the integrate (SEMTSDF_DEBUG_INTEGRATE=n at run time) exist only in a
// build with -DSEMTSDF_INTEGRATE_PROBES=1: the production kernel carries no probe branches.
#ifndef SEMTSDF_INTEGRATE_PROBES
#define SEMTSDF_INTEGRATE_PROBES 0
#endif
constexpr bool kProbes = SEMTSDF_INTEGRATE_PROBES != 0;
constexpr int LZQ = UZ / 4;                 // lanes along z
constexpr int kUnitLanes = UX * UY * UZ / 4;  // lanes of one unit (4 z-voxels each)
constexpr int kSlots = 64 / kUnitLanes;     // units per wave
static_assert(kUnitLanes * kSlots == 64 && UZ % 4 == 0, "a wave is kSlots units of 4 z-voxels per lane");
static_assert(kZAlign % UZ == 0, "the stored z extent is whole tiles");
__device__ __forceinline__ int lane_zq(int lane) { return lane % LZQ; }
__device__ __forceinline__ int lane_y(int lane) { return (lane / LZQ) % UY; }
__device__ __forceinline__ int lane_x(int lane) { return (lane / (LZQ * UY)) % UX; }
__device__ __forceinline__ int lane_slot(int lane) { return lane / kUnitLanes; }

// floor(a / b) with the IEEE quotient, through v_rcp when the result is provably the same:
// |a*rcp(b) - RN(a/b)| < |q| 2^-20, so a q farther than |q| 2^-19 from an integer floors the
// same way; everything else (near-integers, zeros, NaN/Inf, tiny or huge operands) takes
// the correctly rounded division.
__device__ __forceinline__ int floor_div(float a, float b) {
    const float q = a * __builtin_amdgcn_rcpf(b);
    const float fq = floorf(q);
    const float fr = q - fq;
    const float tol = fabsf(q) * 0x1p-19f;
    if (fr > tol && fr < 1.0f - tol && fabsf(b) > 1.0e-30f && fabsf(q) < 8.0e6f) return (int)fq;
    return f2i_rd(a / b);
}


// (c*w + x) / (w+1) for 0 <= c, x <= 255 via the float reciprocal plus one exact integer
// correction (quotient <= 255, so the float estimate is within one of it); integer
// division (truncating, as the reference's int arithmetic) above w = 65535, where the
// numerator would leave the exact f32 range, and for negative (uploaded) colours.
__device__ __forceinline__ int avg_div(int num, int den) {
    if (num < 0 || den > 65536) return num / den;  // the reference's truncating int quotient
    int q = (int)((float)num * __builtin_amdgcn_rcpf((float)den));
    if ((q + 1) * den <= num) ++q;
    else if (q * den > num) --q;
    return q;
}

// Screen position of camera point q.  With a pinhole K (k1 = k3 = k6 = k7 = 0, k8 = 1) the
// general dot products reduce exactly (fma(0, a, c) == c up to the sign of a zero, which
// cannot change the floored pixel), saving 5 of 9 operations.
__device__ __forceinline__ void screen(const IntegrateArgs& a, float qx, float qy, float qz, float* sx, float* sy,
                                       float* sz) {
    if (a.pinhole) {
        *sx = fmaf(a.K[2], qz, a.K[0] * qx);
        *sy = fmaf(a.K[5], qz, a.K[4] * qy);
        *sz = qz;
    } else {
        *sx = dot3(a.K[0], a.K[1], a.K[2], qx, qy, qz);
        *sy = dot3(a.K[3], a.K[4], a.K[5], qx, qy, qz);
        *sz = dot3(a.K[6], a.K[7], a.K[8], qx, qy, qz);
    }
}

// Conservative unit test: returns 1 when no voxel of the unit can pass the projection /
// depth tests of tsdf.cu:46-50 (dead), 2 when every voxel that passes them has f == 1
// (free: tsdf.cu:46-56 with diff >= mu), else 0; culling never changes results.
__device__ int unit_cull(const IntegrateArgs& a, int x0, int y0, int lz0) {
    const VolGeom& g = a.g;
    const int x1 = min(x0 + UX - 1, g.dimx - 1);
    const int y1 = min(y0 + UY - 1, g.dimy - 1);
    const int gz0 = local_to_global_z(g, lz0);
    if (gz0 >= g.dimz) return 1;  // only halo/padding planes beyond the volume
    const int gz1 = min(local_to_global_z(g, min(lz0 + UZ - 1, g.lz - 1)), g.dimz - 1);
    float umin = 3.0e38f, umax = -3.0e38f, vmin = 3.0e38f, vmax = -3.0e38f;
    float zmin = 3.0e38f, zmax = -3.0e38f, wmin = 3.0e38f, wmax = -3.0e38f;
    // Corners through the affine cull map (host-rounded, ~1e-4 px from the contract's screen
    // position, far inside the 1-px guard band); a unit one voxel thick in x has 4 distinct
    // corners, which share their x part.
    constexpr int kCorners = UX == 1 ? 4 : 8;
    const float* C = a.cullC;
    float bx[4][2];  // row r at x0 / x1
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        bx[r][0] = fmaf((float)x0, C[r * 4 + 0], C[r * 4 + 3]);
        bx[r][1] = UX == 1 ? bx[r][0] : fmaf((float)x1, C[r * 4 + 0], C[r * 4 + 3]);
    }
#pragma unroll
    for (int cc = 0; cc < kCorners; ++cc) {
        const int c = UX == 1 ? cc << 1 : cc;  // bit 0 selects x1 == x0 when UX == 1
        const float fy = (float)((c & 2) ? y1 : y0), fz = (float)((c & 4) ? gz1 : gz0);
        float v4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v4[r] = fmaf(fz, C[r * 4 + 2], fmaf(fy, C[r * 4 + 1], bx[r][c & 1]));
        const float sx = v4[0], sy = v4[1], sz = v4[2], qz = v4[3];
        // conservative test: the reciprocal's ~1e-4 px error is far inside the 1-px guard band
        const float rz = __builtin_amdgcn_rcpf(sz);
        const float u = sx * rz, v = sy * rz;
        umin = fminf(umin, u); umax = fmaxf(umax, u);
        vmin = fminf(vmin, v); vmax = fmaxf(vmax, v);
        zmin = fminf(zmin, qz); zmax = fmaxf(zmax, qz);
        wmin = fminf(wmin, sz); wmax = fmaxf(wmax, sz);
    }
    // The image of a box under a perspective map is the hull of its corner images only
    // when the projective depth sz keeps one sign over the box.
    const float zeps = 1.0e-3f;
    if (!(wmin > zeps) && !(wmax < -zeps)) return 0;
    if (!(umin == umin) || !(vmin == vmin) || !(umax == umax) || !(vmax == vmax)) return 0;
    const float W = (float)a.width, H = (float)a.height;
    // 1-pixel guard band around the projected hull
    if (umax + 1.0f < 0.0f || umin - 1.0f > W || vmax + 1.0f < 0.0f || vmin - 1.0f > H) return 1;
    const int u0 = (int)fmaxf(floorf(umin) - 1.0f, 0.0f);
    const int u1 = (int)fminf(floorf(umax) + 1.0f, W - 1.0f);
    const int v0 = (int)fmaxf(floorf(vmin) - 1.0f, 0.0f);
    const int v1 = (int)fminf(floorf(vmax) + 1.0f, H - 1.0f);
    if (u0 > u1 || v0 > v1) return 1;
    // max depth (and min nonzero depth) over the footprint, on the finest pyramid level
    // covering it with <= 4x4 tiles: the 16 loads are issued together (predicated), one round trip
    unsigned m = 0, nz = 0;  // nz: 0xFFFF - min nonzero raw depth (0: none)
    unsigned zf = 0;         // a pixel of the covering tiles has depth 0
    const bool fit0 = ((u1 >> 3) - (u0 >> 3)) < 4 && ((v1 >> 3) - (v0 >> 3)) < 4;
    const bool fit1 = ((u1 >> 5) - (u0 >> 5)) < 4 && ((v1 >> 5) - (v0 >> 5)) < 4;
    if (!fit0 && ((u1 >> 3) - (u0 >> 3) + 1) * ((v1 >> 3) - (v0 >> 3) + 1) <= 16) {  // thin footprints
        for (int ty = v0 >> 3; ty <= (v1 >> 3); ++ty)
            for (int tx = u0 >> 3; tx <= (u1 >> 3); ++tx) {
                const uint2 w = a.pyr.l0[ty * a.pyr.w0 + tx];
                m = max(m, w.x & 0xFFFFu);
                nz = max(nz, w.x >> 16);
                zf |= w.y;
            }
    } else if (fit0 || fit1) {
        const int sh = fit0 ? 3 : 5;
        const uint2* lv = fit0 ? a.pyr.l0 : a.pyr.l1;
        const int wl = fit0 ? a.pyr.w0 : a.pyr.w1;
        const int tx0 = u0 >> sh, ty0 = v0 >> sh, nx = (u1 >> sh) - tx0, ny = (v1 >> sh) - ty0;
        uint2 t[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const bool ok = (j & 3) <= nx && (j >> 2) <= ny;
            t[j] = lv[ok ? (ty0 + (j >> 2)) * wl + tx0 + (j & 3) : 0];
            t[j].x = ok ? t[j].x : 0u;
            t[j].y = ok ? t[j].y : 0u;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            m = max(m, t[j].x & 0xFFFFu);
            nz = max(nz, t[j].x >> 16);
            zf |= t[j].y;
        }
    } else if (((u1 >> 5) - (u0 >> 5) + 1) * ((v1 >> 5) - (v0 >> 5) + 1) <= 64) {
        for (int ty = v0 >> 5; ty <= (v1 >> 5); ++ty)
            for (int tx = u0 >> 5; tx <= (u1 >> 5); ++tx) {
                const uint2 w = a.pyr.l1[ty * a.pyr.w1 + tx];
                m = max(m, w.x & 0xFFFFu);
                nz = max(nz, w.x >> 16);
                zf |= w.y;
            }
    } else {
        return 0;  // footprint wider than 256x256 px (units at the near plane): keep
    }
    if (m == 0) return 1;  // every pixel of the footprint has depth 0
    const float dmax = (float)m / a.depth_scale;
    const float margin = 1.0e-3f + 1.0e-4f * fmaxf(fabsf(zmax), fabsf(zmin));
    // every voxel has qz >= zmin, so diff <= dmax - zmin; rejected when that is <= -mu
    if (dmax - zmin < -g.mu - margin) return 1;
    // free unit: every pixel it can touch has depth >= dmin (the zeros leave their voxels
    // untouched), and every voxel has qz <= zmax, so a touched voxel has diff >= mu, i.e.
    // f == 1 exactly; with the gate at or below 1 such a voxel updates only its sdf and weight
    if (a.free_ok && nz != 0) {
        const float dmin = (float)(0xFFFFu - nz) / a.depth_scale;
        if (dmin - zmax > g.mu + margin) {
            // full free unit: besides, every voxel is stored and inside the volume, projects
            // into the image (hull 1 px inside it: the cull map's ~1e-4 px error cannot move a
            // pixel out) and its pixel has depth != 0 (no zero in the covering tiles), so every
            // voxel is touched with f == 1: the integrate needs no projection
            const bool inside = x0 + UX <= g.dimx && y0 + UY <= g.dimy && lz0 + UZ <= g.lz &&
                                local_to_global_z(g, lz0 + UZ - 1) < g.dimz;
            if (inside && zf == 0u && umin >= 1.0f && vmin >= 1.0f && umax <= W - 2.0f && vmax <= H - 2.0f)
                return 3;
            return 2;
        }
    }
    return 0;
}

struct UnitGrid {
    unsigned nux, nuy, nuz, n;
};

// A live-list entry is the unit's coordinates packed into one word (x | uy << 12 | uz << 22),
// so the integrate decodes it with bit-field extracts instead of divisions by the runtime
// unit counts; the host rejects volumes whose unit grid does not fit (check_params).
constexpr int kEntryXBits = 12, kEntryYBits = 10, kEntryZBits = 10;
static_assert(kEntryXBits + kEntryYBits + kEntryZBits == 32, "one word per entry");
// Host side of that guard, from the same unit shape and field widths as the kernels.
int unit_grid_fits(int dimx, int dimy, int local_z) {
    const long long ux = ((long long)dimx + UX - 1) / UX, uy = ((long long)dimy + UY - 1) / UY,
                    uz = ((long long)local_z + UZ - 1) / UZ;
    return ux <= (1ll << kEntryXBits) && uy <= (1ll << kEntryYBits) && uz <= (1ll << kEntryZBits);
}
__device__ __forceinline__ unsigned pack_unit(unsigned ux, unsigned uy, unsigned uz) {
    return ux | (uy << kEntryXBits) | (uz << (kEntryXBits + kEntryYBits));
}

__host__ __device__ inline UnitGrid unit_grid(const VolGeom& g) {
    UnitGrid u;
    u.nux = (unsigned)(g.dimx + UX - 1) / UX;
    u.nuy = (unsigned)(g.dimy + UY - 1) / UY;
    u.nuz = (unsigned)(g.lz + UZ - 1) / UZ;
    u.n = u.nux * u.nuy * u.nuz;
    return u;
}

// Live-unit list: kListSegs segments, segment c filled by the cull workgroups b with
// b % kListSegs == c (one counter per segment, 256 B apart, keeps the same-address atomics
// per counter to 1/64 of the workgroups).  Capacity of a segment: all units of its
// workgroups.
__host__ __device__ inline unsigned list_seg_cap(const UnitGrid& ug) {
    const unsigned groups = (ug.nux + 255u) / 256u * ug.nuy * ug.nuz;  // k_cull_units workgroups
    return (groups + kListSegs - 1u) / kListSegs * 256u;
}

// Cull pass: one lane per unit (x fastest).  The units that may hold a touched voxel are
// appended to the workgroup's segment of one of two live-unit lists: list 0 (general) and
// list 1 (free units, unit_cull == 2), each kListSegs segments of seg_cap entries with its
// own counters (their order is irrelevant: units are independent).
__global__ __launch_bounds__(256) void k_cull_units(IntegrateArgs a, UnitGrid ug, unsigned seg_cap) {
    __shared__ unsigned s_cnt[kLists][4];
    __shared__ unsigned s_base[kLists];
    // grid (x runs of 256 units, uy, uz): no integer division by the runtime unit counts
    const unsigned ux = blockIdx.x * blockDim.x + threadIdx.x, uy = blockIdx.y, uz = blockIdx.z;
    const unsigned bid = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    const bool inside = ux < ug.nux;
    const unsigned u = pack_unit(ux, uy, uz);
    int c = 1;  // dead
    if (inside) c = a.cull ? unit_cull(a, (int)ux * UX, (int)uy * UY, (int)uz * UZ) : 0;
    const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
    // list of class c: 0 general (c == 0), 1 free (c == 2), 2 full free (c == 3)
    const unsigned long long bal0 = __ballot(c == 0), bal1 = __ballot(c == 2), bal2 = __ballot(c == 3);
    if (lane == 0) {
        s_cnt[0][wv] = (unsigned)__popcll(bal0);
        s_cnt[1][wv] = (unsigned)__popcll(bal1);
        s_cnt[2][wv] = (unsigned)__popcll(bal2);
    }
    __syncthreads();
    const unsigned seg = bid % (unsigned)kListSegs;
    if (threadIdx.x < kLists) {
        const unsigned l = threadIdx.x;
        const unsigned tot = s_cnt[l][0] + s_cnt[l][1] + s_cnt[l][2] + s_cnt[l][3];
        s_base[l] = tot ? atomicAdd(a.list_count + (l * kListSegs + seg) * kListCountStride, tot) : 0u;
    }
    __syncthreads();
    if (c != 1) {
        const unsigned l = c == 2 ? 1u : c == 3 ? 2u : 0u;
        unsigned off = s_base[l] + (unsigned)__popcll((l == 1 ? bal1 : l == 2 ? bal2 : bal0) & ((1ull << lane) - 1ull));
        for (int w = 0; w < wv; ++w) off += s_cnt[l][w];
        a.unit_list[(size_t)l * kListSegs * seg_cap + seg * seg_cap + off] = u;
    }
}

hipError_t launch_cull(const IntegrateArgs& a, hipStream_t s) {
    const UnitGrid ug = unit_grid(a.g);
    if (ug.n == 0) return hipSuccess;  // a shard that owns no chunk
    hipLaunchKernelGGL(k_cull_units, dim3((ug.nux + 255) / 256, ug.nuy, ug.nuz), dim3(256), 0, s, a, ug,
                       list_seg_cap(ug));
    return hipGetLastError();
}

#ifndef SEMTSDF_TAIL_CULL_PROBE
#define SEMTSDF_TAIL_CULL_PROBE 0  // instrumentation build: a whole-grid unit cull in the integrate's tail
#endif
#ifndef SEMTSDF_XCD_SPLIT
#define SEMTSDF_XCD_SPLIT 1  // each XCD's waves take a contiguous eighth of every list (list_view)
#endif
// The cull's segments compacted into one array: list l at an even base (so a group's two entries are
// one 8-byte scalar load), followed by a ~0u pad (the second entry of a list's last group when
// its count is odd), bases and totals after the dynamic counters of list_count.  One wave per
// (segment, list): lane j holds the count of segment j of every list; the wave's segment offset
// is the exclusive prefix of its list's counts.  Runs on the prep stream after the cull, so the
// integrate reads its first group's entries without the counts' prefix (one dependent load less
// at its start) and decodes no segment per entry.
__global__ __launch_bounds__(256) void k_compact_lists(unsigned* __restrict__ list_count,
                                                       const unsigned* __restrict__ seg_list, unsigned seg_cap,
                                                       unsigned* __restrict__ units, unsigned* __restrict__ first_tab,
                                                       unsigned nwaves, unsigned first_list) {
    __shared__ unsigned s_incl[64];
    // every wave of the workgroup computes the (tiny) prefix itself; all 256 lanes copy
    const unsigned lane = threadIdx.x & 63u, seg = blockIdx.x, l = blockIdx.y;
    unsigned c[kLists], tot[kLists];
#pragma unroll
    for (int k = 0; k < kLists; ++k) {
        c[k] = list_count[((unsigned)k * kListSegs + lane) * kListCountStride];
        tot[k] = c[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) tot[k] += (unsigned)__shfl_xor((int)tot[k], off, 64);
    }
    // the free list first (k_integrate reads a wave's first free group before the totals), then
    // the full free list, then the general one
    unsigned base[kLists];
    base[1] = 0u;
    base[2] = (tot[1] + 2u) & ~1u;
    base[0] = (base[2] + tot[2] + 2u) & ~1u;
    // this list's counts, exclusive prefix over the segments
    unsigned cl = c[0];
#pragma unroll
    for (int k = 1; k < kLists; ++k) cl = l == (unsigned)k ? c[k] : cl;
    unsigned incl = cl;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned o = (unsigned)__shfl_up((int)incl, off, 64);
        if ((int)lane >= off) incl += o;
    }
    const unsigned n = (unsigned)__shfl((int)cl, (int)seg, 64), off0 = (unsigned)__shfl((int)(incl - cl), (int)seg, 64);
    unsigned bl = base[0];
#pragma unroll
    for (int k = 1; k < kLists; ++k) bl = l == (unsigned)k ? base[k] : bl;
    const unsigned* src = seg_list + ((size_t)l * kListSegs + seg) * seg_cap;
    unsigned* dst = units + bl + off0;
    // four loads in flight per lane before their stores (the copy is latency-bound otherwise)
    for (unsigned i0 = threadIdx.x; i0 < n; i0 += 4u * 256u) {
        unsigned e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = i0 + 256u * k < n ? src[i0 + 256u * k] : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + 256u * k < n) dst[i0 + 256u * k] = e[k];
    }
    if (SEMTSDF_XCD_SPLIT && l == first_list && nwaves) {
        // the first-group table of the XCD split (k_integrate, list_view): wave slot w (workgroup w / 4,
        // XCD xi = workgroup % 8, index wx among the XCD's waves) starts at group lo(xi) + wx of the list;
        // its two entries are read here from the cull's segments (the compacted array is being written
        // by the other workgroups), the segment found by a binary search over the inclusive prefix
        if (threadIdx.x < 64u) s_incl[threadIdx.x] = incl;
        __syncthreads();
        const unsigned w = seg * 256u + threadIdx.x;
        const unsigned tl = tot[0] * (l == 0u) + tot[1] * (l == 1u) + tot[2] * (l == 2u);
        const unsigned ng = (tl + 1u) / 2u, nwx = nwaves / 8u;
        const unsigned blk = w >> 2, xi = blk & 7u, wx = (blk >> 3) * 4u + (w & 3u);
        const unsigned g = ng * xi / 8u + wx;
        if (w < nwaves && w < kPreWaves && wx < nwx && g < ng * (xi + 1u) / 8u) {
            unsigned ev[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const unsigned idx = 2u * g + (unsigned)k;
                unsigned j = 0;  // first segment whose inclusive prefix exceeds idx
#pragma unroll
                for (unsigned step = 32u; step; step >>= 1)
                    if (s_incl[j + step - 1u] <= idx) j += step;
                const unsigned before = j ? s_incl[j - 1u] : 0u;
                ev[k] = idx < tl ? seg_list[((size_t)l * kListSegs + j) * seg_cap + (idx - before)] : ~0u;
            }
            first_tab[2u * w] = ev[0];
            first_tab[2u * w + 1u] = ev[1];
        }
    }
    if (seg == 0u && l == 0u && threadIdx.x < (unsigned)kLists) {
        unsigned b = base[0], t = tot[0];
#pragma unroll
        for (int k = 1; k < kLists; ++k) {
            b = lane == (unsigned)k ? base[k] : b;
            t = lane == (unsigned)k ? tot[k] : t;
        }
        units[b + t] = ~0u;  // the pad
        unsigned* tw = list_count + kListTotalsWord;  // read only by later launches
        tw[2 * lane] = b;
        tw[2 * lane + 1] = t;
    }
}

hipError_t launch_compact_lists(const IntegrateArgs& a, hipStream_t s) {
    const UnitGrid ug = unit_grid(a.g);
    if (ug.n == 0) {  // a shard that owns no chunk: empty lists
        return hipMemsetAsync(a.list_count + kListTotalsWord, 0, 8 * sizeof(unsigned), s);
    }
    // the first-group table for the list the integrate starts with: free units in the gated modes
    const unsigned first_list = ((a.flags & 0x2u) && !(a.flags & 0x8u)) ? 1u : 0u;
    hipLaunchKernelGGL(k_compact_lists, dim3(kListSegs, kLists), dim3(256), 0, s, a.list_count, a.unit_list,
                       list_seg_cap(ug), a.units, a.first_tab, a.first_nwaves, first_list);
    return hipGetLastError();
}

uint64_t unit_count(const VolGeom& g) { return unit_grid(g).n; }
uint64_t unit_list_capacity(const VolGeom& g) { return (uint64_t)list_seg_cap(unit_grid(g)) * kListSegs * kLists; }

// Exact floor of the colour running mean (c*w + x) / (w + 1) for 0 <= c, x <= 255 and
// w + 1 <= kRcpTable, from r = RN(1/(w+1)): floor(RN(num*r + 2^-12)) equals the integer
// quotient (the product is within 2.3e-5 of num/(w+1), whose fraction is 0 or in
// [1/(w+1), 1 - 1/(w+1)]; checked exhaustively, tests/test_oracle_props.py).
__device__ __forceinline__ unsigned avg_u8(unsigned c, unsigned x, unsigned w, float r) {
    const unsigned num = __umul24(c, w) + x;  // exact while w < 2^24 (this path needs w < kRcpTable)
    return (unsigned)fmaf((float)num, r, 0x1p-12f);
}

// ---- the integrate of one unit in stages ---------------------------------------------------
// kSlots units (UX x UY x UZ voxels each) share a wavefront: lane = (slot, y, zq) owns
// planes 4zq..4zq+3 of row (x, y) of its unit, one 16-byte vector per state access.  Stages:
//   project  — screen position, exact pixel, gather of the pixel records (depth, rgb, label)
//   classify — tsdf.cu:46-52 tests
//   load     — state of the touched lanes (sdf, weight; colour and histogram words of the
//              gated voxels)
//   compute  — tsdf.cu:56-68 running means
//   store
// The wave software-pipelines its units in the order
//   project(k+1)  compute(k)  classify(k+1)  store(k)  load(k+1)
// so the state loads of unit k are in flight under the projection of k+1 and the pixel
// gathers of k+1 under the compute of k.  s_waitcnt vmcnt counts memory operations in
// issue order, and the compiler can only count the ones it knows were issued: every load
// is therefore unconditional (lanes with nothing to load read one dummy line), stores come
// after the waits of the iteration, and every wait names the oldest group in flight.  The
// histogram increment is a plain load/store of the 4 words of a lane (one lane owns a
// voxel within a frame); a lane whose gated voxels carry different labels (object borders)
// takes no-return atomics.
struct UnitPos {
    int x, uy, uz;  // per slot of the wave (wave-uniform with one unit per wave)
    bool ok = true; // false: the slot has no unit this iteration (end of the list)
};

__device__ __forceinline__ UnitPos unit_pos(const UnitGrid& ug, unsigned u) {
    (void)ug;  // list entries are packed unit coordinates (pack_unit): bit-field extracts only
    UnitPos p;
    p.x = (int)(u & ((1u << kEntryXBits) - 1u));
    p.uy = (int)((u >> kEntryXBits) & ((1u << kEntryYBits) - 1u));
    p.uz = (int)(u >> (kEntryXBits + kEntryYBits));
    return p;
}


// First voxel of the unit in the tiled layout (a unit is one tile).
__device__ __forceinline__ uint64_t unit_tile(const VolGeom& g, const UnitPos& up) {
    static_assert(UX == 1 && UY == 8 && (UZ == 32 || UZ == 16 || UZ == 8), "a unit is a whole tile or a part of one");
    const uint32_t z0 = (uint32_t)(up.uz * UZ);  // first plane: a multiple of UZ within its tile
    return tile_xterm(g, up.x) + __umul24((uint32_t)up.uy, g.ty) + (z0 >> 5) * 256u + ((z0 >> 2) & 7u) * 32u;
}

#ifndef SEMTSDF_STEADY
#define SEMTSDF_STEADY 1  // skip the sdf traffic of steady lines (Ld::skip)
#endif

// Lazy weights of steady lines.  A steady line (every sdf exactly 1.0f) whose 32 voxels are
// all touched with f == 1 changes only its weights, each by +1, when the colour/histogram
// gate rejects f == 1 (free_ok modes): the increment is kept as a per-line pending count in
// the line's flag byte instead of a read-modify-write of the 128-B weight line (and the sdf
// line is skipped as a steady line anyway).  Flag byte s: 0 = not steady; s >= 1 = steady with
// s - 1 pending increments of every weight of the line.  Any other update of the line adds
// the pending count first (stage_compute), and k_flush_lazy folds the counts into the weights
// before they are read out (download, upload, checkpoint).
#ifndef SEMTSDF_CHAIN
#define SEMTSDF_CHAIN 1  // a wave's last unit of a list overlaps the first unit of its next list
#endif
#ifndef SEMTSDF_WAVE_TRACE
#define SEMTSDF_WAVE_TRACE 0  // instrumentation build only: per-wave phase timestamps (IntegrateArgs::wtrace)
#endif
constexpr unsigned kFlagMax = 255u;  // s - 1 <= 254 pending increments

struct Proj {
    float qz[4];
    uint2 rec[4];  // gathered pixel record {metres bits, rgbl}
    int img[4];    // record index (rec_index); off-image: a record of the zero column / row
    int lin[4];    // vote mode: the pixel's row-major index, W*H off-image or on an invalid plane
    unsigned sflag;  // steady flag of the lane's sdf line (below)
    unsigned vmask;  // bit k: plane l0 + k is a voxel of the volume (others are never touched)
    uint32_t ub;     // tiled index of the lane's unit's first voxel (unit_tile), carried to load and store
};

struct Cls {
    float fv[4];
    unsigned tmask, gmask;
    uint32_t pix[4];   // rgbl of the voxels' pixels
    unsigned hmode;    // 1: the gated voxels share label hlab < 32 (one 16-B histogram RMW); 2: atomics
    unsigned hlab;
    int img[4];        // vote mode
    unsigned sflag;    // steady flag of the lane's sdf line
    uint32_t ub;       // Proj::ub
};

// What stage_store needs of a classification: masks, histogram mode/label and the 4 labels.
struct StoreMeta {
    unsigned meta;  // tmask | gmask << 4 | hmode << 8 | hlab << 16
    unsigned labs;  // label of voxel k in bits 8k..8k+7
};

__device__ __forceinline__ StoreMeta store_meta(const Cls& C) {
    StoreMeta m;
    m.meta = C.tmask | (C.gmask << 4) | (C.hmode << 8) | (C.hlab << 16);
    m.labs = (C.pix[0] >> 24) | ((C.pix[1] >> 24) << 8) | ((C.pix[2] >> 24) << 16) | ((C.pix[3] >> 24) << 24);
    return m;
}

struct Ld {
    bool skip;  // steady line: s4 not loaded, every value is 1.0f
    bool lazy;  // steady line, all 32 voxels touched with f == 1: only the flag byte changes
    float4 s4;
    int4 w4;
    uint4 c8;
    int4 c32[4];
    uint4 h4;
    int4 vc4, vn4;
    int vin[4];
};

struct Out {
    float4 s4;
    int4 w4;
    bool skip;       // the line's sdf was neither loaded nor changes (steady line)
    bool lazy;       // the line's weights take one more pending increment (flag byte + 1)
    unsigned oflag;  // the line's steady flag before this update
    bool cross;      // a voxel's sdf crossed the skip threshold (its brick's map entry may flip)
    uint32_t ub;     // Proj::ub of the unit
    uint4 c8;
    int4 c32[4];
    uint4 h4;
    int4 vc4, vn4;
};

// Screen position s = M p + m (DESIGN.md §4 contract; per-row bases then one fma per
// coordinate per voxel), the exact pixel through the reciprocal, and the record gather.
template <bool SHARD, bool PIN, bool FREE, bool FULL, bool LIN>
__device__ __forceinline__ void stage_project(const IntegrateArgs& a, const UnitPos& up, int lane, Proj& P) {
    const VolGeom& g = a.g;
    P.ub = (uint32_t)unit_tile(g, up);
    if (FULL) {  // full free unit (unit_cull == 3): every voxel touched with f == 1, nothing to project
        P.sflag = SEMTSDF_STEADY ? (unsigned)a.b.sflag[(P.ub + (unsigned)lane_zq(lane) * 32u +
                                                        (unsigned)lane_y(lane) * 4u) >> 5]
                                 : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) P.rec[k] = make_uint2(1u, 0u);  // "depth != 0"
        P.vmask = up.ok ? 0xFu : 0u;  // every voxel of a real unit
        return;
    }
    const int npx = a.width * a.height;
    const int x = up.x * UX + lane_x(lane);
    const int y = up.uy * UY + lane_y(lane);
    const int l0 = up.uz * UZ + lane_zq(lane) * 4;
    const bool row_ok = up.ok & (x < g.dimx) & (y < g.dimy) & (l0 < g.lz);
    const float px = fmaf((float)x, g.voxel[0], g.start[0]);
    const float py = fmaf((float)y, g.voxel[1], g.start[1]);
    const float bsx = fmaf(a.M[1], py, fmaf(a.M[0], px, a.m[0]));
    const float bsy = fmaf(a.M[4], py, fmaf(a.M[3], px, a.m[1]));
    const float bsz = fmaf(a.M[7], py, fmaf(a.M[6], px, a.m[2]));
    const float bqz = PIN ? bsz : fmaf(a.E[9], py, fmaf(a.E[8], px, a.E[11]));
    // (sx, sy) pairs in packed f32 (v_pk_fma / v_pk_mul / v_pk_add: each lane of a packed op is
    // the scalar IEEE operation, so the values are those of the scalar contract)
    const f32x2 bsxy = {bsx, bsy}, Mxy = {a.M[2], a.M[5]};
    // (float)(l0 + k) == fl0 + k (integers far below 2^24): one add per plane; the empty asm
    // keeps the compiler from turning it back into an integer add and a conversion
    float fl0 = (float)l0;
    asm volatile("" : "+v"(fl0));
    // the lane's valid planes (bit k: plane l0 + k exists in this shard's storage and, sharded,
    // in the volume): voxels outside it project like the others but are never touched
    // (stage_classify masks them), so the projection carries no per-voxel validity selects
    unsigned vmask;
    int cblk = 0, w0 = 0;
    const int per = g.chunk + g.halo;
    if (SHARD) {  // the chunk block of l0 once per lane; l0 + k lies in that block or the next
        cblk = l0 / per;
        w0 = l0 - cblk * per;
        vmask = 0u;
    } else {
        // planes l0 .. lz - 1 of the lane (l0 < lz + 16: the shift stays below 20); a listed unit has
        // x < dimx, so only its y rows and its slot can be invalid
        vmask = (up.ok & (y < g.dimy)) ? (0xFu >> (4 - min(g.lz - l0, 4))) : 0u;
    }
    // floor(sx/sz), floor(sy/sz) through the reciprocal: |qu - RN(sx/sz)| <= 2^-22 |qu|, so for
    // |qu| < B (host: B = 2^ceil(log2(max(W, H) + 2))) a fraction farther than B 2^-21 from 0
    // and 1, i.e. |fract - 1/2| < ftol, floors like the IEEE quotient; |qu| >= B is off-image
    // either way.  Per voxel the NaN-propagating maximum (v_maximum) of |fract - 1/2| of both
    // coordinates: a near-integer, a huge quotient (fract 0) or NaN/Inf (fract NaN) takes the
    // exact IEEE division below (per voxel: a wave runs the division of plane k only when one of
    // its lanes needs it).
    float mk[4];
    unsigned uu[4], vv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float pzk;
        if (SHARD) {
            int gz;
            if (per >= 4) {  // 4 consecutive planes span at most two blocks
                const bool nxt = w0 + k >= per;
                const int cb = cblk + (nxt ? 1 : 0);
                gz = (cb * g.nshards + chunk_pos(cb, g.shard, g.nshards)) * g.chunk + (w0 + k - (nxt ? per : 0));
            } else {
                gz = local_to_global_z(g, l0 + k);
            }
            vmask |= ((row_ok & (l0 + k < g.lz) & (gz < g.dimz)) ? 1u : 0u) << k;
            pzk = (float)gz;
        } else {
            pzk = fl0 + (float)k;
        }
        const float pz = fmaf(pzk, g.voxel[2], g.start[2]);
        const f32x2 sxy = __builtin_elementwise_fma(Mxy, (f32x2){pz, pz}, bsxy);
        const float sz = fmaf(a.M[8], pz, bsz);
        P.qz[k] = PIN ? sz : fmaf(a.E[10], pz, bqz);
        const float r = __builtin_amdgcn_rcpf(sz);
        const f32x2 q = sxy * r;
        const f32x2 e = (f32x2){__builtin_amdgcn_fractf(q.x), __builtin_amdgcn_fractf(q.y)} - 0.5f;
        mk[k] = __builtin_elementwise_maximum(fabsf(e.x), fabsf(e.y));
        // off-image pixels (either side) clamp onto the record image's zero column u = W / zero
        // row v = H (unsigned min: negative coordinates are huge)
        uu[k] = min((unsigned)cvt_flr(q.x), (unsigned)a.width);
        vv[k] = min((unsigned)cvt_flr(q.y), (unsigned)a.height);
    }
    const float worst = __builtin_elementwise_maximum(__builtin_elementwise_maximum(mk[0], mk[1]),
                                                      __builtin_elementwise_maximum(mk[2], mk[3]));
    if (!(worst < a.ftol)) {  // rare: exact IEEE quotients (the screen position is recomputed)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (mk[k] < a.ftol) continue;
            const int gz = SHARD ? local_to_global_z(g, l0 + k) : l0 + k;
            const float pz = fmaf((float)gz, g.voxel[2], g.start[2]);
            const float sx = fmaf(a.M[2], pz, bsx), sy = fmaf(a.M[5], pz, bsy), sz = fmaf(a.M[8], pz, bsz);
            uu[k] = min((unsigned)f2i_rd(sx / sz), (unsigned)a.width);
            vv[k] = min((unsigned)f2i_rd(sy / sz), (unsigned)a.height);
        }
    }
    P.vmask = vmask;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        P.img[k] = (int)rec_index(a.pyr, uu[k], vv[k]);
        if (LIN) P.lin[k] = (uu[k] < (unsigned)a.width && vv[k] < (unsigned)a.height && ((vmask >> k) & 1u))
                                ? (int)__umul24(vv[k], (unsigned)a.width) + (int)uu[k]
                                : npx;
    }
    // steady flag of the lane's sdf line (one byte per 128-B line, unconditional)
    P.sflag = SEMTSDF_STEADY ? (unsigned)a.b.sflag[(P.ub + (unsigned)lane_zq(lane) * 32u +
                                                    (unsigned)lane_y(lane) * 4u) >> 5]
                             : 0u;
    // unconditional gathers (an off-image voxel reads a zero record: depth 0); a free unit needs
    // only the depth word (touched <=> depth != 0, f == 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (FREE)
            P.rec[k] = make_uint2(
                reinterpret_cast<const unsigned*>(a.pyr.px)[(kProbes && a.debug == 21) ? 0u : 2u * (unsigned)P.img[k]],
                0u);
        else
            P.rec[k] = a.pyr.px[(kProbes && a.debug == 21) ? 0u : (unsigned)P.img[k]];  // 21: probe, one address
#if SEMTSDF_PROBE_GATHER2
        {  // timing probe: a second gather per voxel (no effect on results)
            const uint2 extra = a.pyr.px[(unsigned)P.img[k] ^ 1u];
            P.rec[k].y += (extra.x == 0x7fc00001u) ? 1u : 0u;
        }
#endif
    }
}

// The deferred relabel of a frame whose prepass ran beside its association (IntegrateArgs::lut):
// label byte of a pixel record -> the decision's new label, from the 256-byte table held one
// dword per lane (lutv, lane l = labels 4l..4l+3; every lane of the wave active).
__device__ __forceinline__ uint32_t relabel_rec(uint32_t rec, unsigned lutv) {
    const unsigned raw = rec >> 24;
    const unsigned w = (unsigned)__shfl((int)lutv, (int)(raw >> 2), 64);
    return (rec & 0x00FFFFFFu) | (((w >> (8u * (raw & 3u))) & 0xFFu) << 24);
}

// Count mode: the 128-B sdf lines of the wave's units holding a touched voxel (a line = the 8
// y-lanes of one slot and z-quad, lanes zq + LZQ y + kUnitLanes slot), on lane 0.
__device__ __forceinline__ unsigned count_lines(unsigned tmask) {
    static_assert(UX == 1 && LZQ * UY == kUnitLanes, "line folding assumes lane = zq + LZQ y + kUnitLanes slot");
    unsigned long long b = __ballot(tmask != 0u);
#pragma unroll
    for (int sft = kUnitLanes / 2; sft >= LZQ; sft >>= 1) b |= b >> sft;
    unsigned long long m = 0;
#pragma unroll
    for (int sl = 0; sl < 64 / kUnitLanes; ++sl) m |= ((1ull << LZQ) - 1ull) << (sl * kUnitLanes);
    return (threadIdx.x & 63) == 0 ? (unsigned)__popcll(b & m) : 0u;
}

template <bool SEM, bool GATE, bool VOTE, bool COUNT, bool FREE>
__device__ __forceinline__ void stage_classify(const IntegrateArgs& a, const Proj& P, Cls& C, bool count,
                                               unsigned& n_touch, unsigned& n_gate, unsigned& n_lines,
                                               unsigned lutv) {
    const VolGeom& g = a.g;
    if (FREE) {  // free unit (unit_cull == 2): a voxel with depth is touched with f == 1, never gated
        unsigned tm = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tm |= (P.rec[k].x != 0u ? 1u : 0u) << k;
            C.fv[k] = 1.0f;
            C.pix[k] = 0u;
        }
        tm &= P.vmask;
        C.sflag = P.sflag;
        C.ub = P.ub;
        if (kProbes && (a.debug == 3 || a.debug == 21)) tm = 0u;  // probe: no state traffic
        C.tmask = tm;
        C.gmask = 0u;
        C.hlab = 0xFFu;
        C.hmode = 0u;
        if (COUNT && count) {
            n_touch += __popc(tm);
            n_lines += count_lines(tm);  // touched lines (lane 0)
        }
        return;
    }
    unsigned tmask = 0;
    float dm[4];
    float dmin = 1.0f;  // min |dc| of the lane (NaN-propagating): tiny differences take the IEEE division
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float d = __uint_as_float(P.rec[k].x);
        dm[k] = d;
        const float diff = d - P.qz[k];
        const bool t = (d != 0.0f) & (diff > -g.mu);
        const float dc = fminf(diff, g.mu);
        C.fv[k] = div_by_rcp(dc, g.mu, a.rmu);
        dmin = __builtin_elementwise_minimum(dmin, fabsf(dc));
        tmask |= (t ? 1u : 0u) << k;
        C.pix[k] = P.rec[k].y;
        if (VOTE) C.img[k] = P.lin[k];
    }
    tmask &= P.vmask;
    if (SEM && a.lut) {  // uniform: records of a deferred relabel carry raw labels
#pragma unroll
        for (int k = 0; k < 4; ++k) C.pix[k] = relabel_rec(C.pix[k], lutv);
    }
    C.sflag = P.sflag;
    C.ub = P.ub;
    if (!(dmin >= 0x1p-60f) || !a.fastdiv) {  // rare: tiny differences, or mu outside the reciprocal range
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float dc = fminf(dm[k] - P.qz[k], g.mu);
            if (!a.fastdiv || !(fabsf(dc) >= 0x1p-60f)) C.fv[k] = dc == 0.0f ? dc : dc / g.mu;
        }
    }
    // gated: touched and f < gate (tsdf.cu:57): the gate bits in a VGPR, then one AND
    unsigned gbits = 0xFu;
    if (GATE) {
        gbits = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) gbits |= (C.fv[k] < a.gate ? 1u : 0u) << k;
    }
    unsigned gmask = tmask & gbits;
    if (COUNT && count) {
        n_touch += __popc(tmask);
        n_gate += __popc(gmask);
        n_lines += count_lines(tmask);  // touched lines (lane 0)
    }
    if (kProbes && (a.debug == 3 || a.debug == 21)) tmask = gmask = 0;  // probe: classification only, no state traffic
    if (kProbes && a.debug == 4) gmask = 0;          // timing probe: no colour/histogram traffic
    C.tmask = tmask;
    C.gmask = gmask;
    // histogram mode of the lane: the label of its first gated voxel, shared by all of them?
    C.hlab = 0xFFu;
    C.hmode = 0u;
    if (SEM && gmask && !(kProbes && a.debug == 6)) {  // ~2/3 of the units have no gated lane: skipped
        unsigned lab = 0xFFu, same = 1u;
#pragma unroll
        for (int k = 3; k >= 0; --k) lab = ((gmask >> k) & 1u) ? (C.pix[k] >> 24) : lab;
#pragma unroll
        for (int k = 0; k < 4; ++k) same &= (((gmask >> k) & 1u) == 0u) | ((C.pix[k] >> 24) == lab);
        C.hlab = lab;
        C.hmode = (same && lab < (unsigned)kMaxObjects) ? 1u : 2u;
    }
}

#ifndef SEMTSDF_FULLROW
#define SEMTSDF_FULLROW 0
#endif
// State traffic per lane (SEMTSDF_FULLROW 0): a lane loads and stores its 16-B vectors only
// when it updates (sdf/weight: a touched voxel; colour: a gated one); a 128-B line of a
// per-voxel array is the 8 lanes of one z-quad (lane % 8).  The line's steady flag is then
// decided from the lanes that loaded their values plus what the old flag says of the others:
// an untouched lane of a steady line still holds sdf 1.0f and a weight < 2^23; of a line not
// known steady, nothing (it stays 0, "unknown").  (r03's per-lane build decided the flag from
// every lane's values, the dummy line's included, and flagged unsteady lines steady:
// profiles/r03/s2/gputest_full_row_0_failure.txt.)  SEMTSDF_FULLROW 1: whole-line traffic
// (all 8 lanes load and store when any of them updates; every line written back fully dirty).
static_assert(!SEMTSDF_LAZY_WEIGHT || SEMTSDF_FULLROW, "lazy weights need whole-line state traffic");
constexpr uint64_t line_lanes() {  // lanes of one line of slot 0, z-quad 0: zq + LZQ y
    uint64_t m = 0;
    for (int y = 0; y < UY; ++y) m |= 1ull << (LZQ * y);
    return m;
}
constexpr uint64_t kLineLanes = line_lanes();

__device__ __forceinline__ bool tile_line_any(bool p) {
    static_assert(UY == 8 && UX == 1, "lane = zq + LZQ y + kUnitLanes slot");
    if (!SEMTSDF_FULLROW) return p;
    const uint64_t b = __ballot(p);
    const int lane = (int)__lane_id();
    return ((b >> (lane % LZQ + lane_slot(lane) * kUnitLanes)) & kLineLanes) != 0ull;
}

// true when p holds on all 8 lanes of the lane's line (inactive lanes count as true)
__device__ __forceinline__ bool tile_line_all(bool p) {
    const uint64_t b = __ballot(!p);
    const int lane = (int)__lane_id();
    return ((b >> (lane % LZQ + lane_slot(lane) * kUnitLanes)) & kLineLanes) == 0ull;
}

#ifndef SEMTSDF_NT_LOAD
#define SEMTSDF_NT_LOAD 0  // nt loads measured 3-5 % slower once the pipeline was chained (r03, same box)
#endif
#ifndef SEMTSDF_NT_STORE
#define SEMTSDF_NT_STORE 0  // default-policy state stores: r06 A/B 73.7 -> 72.2 us (C3), 19.1 -> 18.9 us (C2) over six rounds (profiles/r06/ab/r06_store_policy.txt); nt until r05
#endif
#ifndef SEMTSDF_NT_HIST
#define SEMTSDF_NT_HIST 0  // histogram lines are partial (one bin plane per lane): default policy
#endif
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// 16-B state accesses (sdf, weight, colour, histogram), optionally non-temporal
template <class T, bool NT = SEMTSDF_NT_LOAD>
__device__ __forceinline__ T ld_state(const void* p) {
    static_assert(sizeof(T) == 16, "16-byte vectors");
    if (NT) {
        const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        T t;
        __builtin_memcpy(&t, &r, 16);
        return t;
    }
    return *reinterpret_cast<const T*>(p);
}
template <class T, bool NT = SEMTSDF_NT_STORE>
__device__ __forceinline__ void st_state(void* p, const T& v) {
    static_assert(sizeof(T) == 16, "16-byte vectors");
    if (NT) {
        u32x4 r;
        __builtin_memcpy(&r, &v, 16);
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4*>(p));
        return;
    }
    *reinterpret_cast<T*>(p) = v;
}

#ifndef SEMTSDF_DUMMY0
#define SEMTSDF_DUMMY0 1  // the dummy address of a lane with nothing to load: 1 the array's start, 0 its unit's first line
#endif
// Unconditional loads: a lane with nothing to load reads the dummy line (one 16-B vector
// shared by all such lanes), so the issue count is the same on every path.
template <bool SEM, bool CI32, bool VOTE, bool FREE>
__device__ __forceinline__ void stage_load(const IntegrateArgs& a, const UnitPos& up, unsigned coff, const Cls& C,
                                           Ld& L) {
    const VolGeom& g = a.g;
    // wave-uniform unit bases (scalar) + the lane's 32-bit element offset; a lane with
    // nothing to load reads the unit's first vector instead (same line for all of them)
    (void)up;
    const uint32_t ub = C.ub;
    const uint32_t v = ub + coff;
    // a lane with nothing to load reads the array's first vector (offset 0): one base pointer
    // per array, the offset selected in 32 bits
    const uint4* dummy = reinterpret_cast<const uint4*>(a.b.sdf);
    const bool t = tile_line_any(C.tmask != 0u), gt = tile_line_any(C.gmask != 0u);
    const unsigned lt = t ? coff : 0u, lg = gt ? coff : 0u;
    // Steady line: every sdf of the line is exactly 1.0f with weight < 2^23 (flag) and every
    // touched voxel of it has f == 1.0f, so (1 w + 1) / (w + 1) == 1 exactly (w + 1 < 2^24 in
    // both the reciprocal and the IEEE path): the line's sdf is neither read nor written.
    bool fone = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) fone &= (((C.tmask >> k) & 1u) == 0u) | (C.fv[k] == 1.0f);
    // (whole-line traffic: the whole line skips together; per-lane: each lane for itself)
    const bool skip = SEMTSDF_STEADY && (SEMTSDF_FULLROW ? tile_line_all((C.sflag != 0u) & fone) : ((C.sflag != 0u) & fone));
    // lazy: steady, every voxel of the line touched (f == 1), pending count below the cap
    const bool lazy = SEMTSDF_STEADY && SEMTSDF_LAZY_WEIGHT && !VOTE && a.free_ok &&
                      tile_line_all((C.sflag != 0u) & (C.sflag < kFlagMax) & fone & (C.tmask == 15u));
    L.skip = skip;
    L.lazy = lazy;
    if (SEMTSDF_DUMMY0) {
        // a lane with nothing to load reads the array's first vector, like a steady line: the line
        // stays in L2, where the unit's first line (the other choice) is an extra line fetched
        // whenever that line itself has no update
        L.s4 = ld_state<float4>(a.b.sdf + ((skip | !t) ? 0u : v));
        L.w4 = ld_state<int4>(a.b.wt + ((lazy | !t) ? 0u : v));
    } else {
        L.s4 = ld_state<float4>(a.b.sdf + (skip ? 0u : ub + lt));
        L.w4 = ld_state<int4>(a.b.wt + (lazy ? 0u : ub + lt));
    }
    if (FREE) return;  // sdf and weight only
    if (CI32) {
#pragma unroll
        for (int k = 0; k < 4; ++k) L.c32[k] = reinterpret_cast<const int4*>(a.b.color)[(uint64_t)ub + lg + (gt ? k : 0)];
    } else if (SEMTSDF_DUMMY0) {
        L.c8 = ld_state<uint4>(reinterpret_cast<const uint32_t*>(a.b.color) + (gt ? v : 0u));
    } else {
        L.c8 = ld_state<uint4>(reinterpret_cast<const uint32_t*>(a.b.color) + ub + lg);
    }
    if (SEM)
        L.h4 = ld_state<uint4, SEMTSDF_NT_HIST>(a.b.hist + (C.hmode == 1u ? (uint64_t)C.hlab * g.nvox + v : 0ull));
    if (VOTE) {
        L.vc4 = *(t ? reinterpret_cast<const int4*>(a.b.cls + v) : reinterpret_cast<const int4*>(dummy));
        L.vn4 = *(t ? reinterpret_cast<const int4*>(a.b.cls_cnt + v) : reinterpret_cast<const int4*>(dummy));
#pragma unroll
        for (int k = 0; k < 4; ++k) L.vin[k] = a.cls[C.img[k] < a.width * a.height ? C.img[k] : 0];
    }
}

template <bool SEM, bool GATE, bool CI32, bool VOTE, bool FREE>
__device__ __forceinline__ void stage_compute(const IntegrateArgs& a, const float* __restrict__ s_rcp, const Cls& C,
                                              const Ld& L, Out& O) {
    const unsigned tmask = C.tmask, gmask = C.gmask;
    // ---- running mean (tsdf.cu:56, 68) through RN(1/(w+1)) from the LDS table
    const float so[4] = {L.skip ? 1.0f : L.s4.x, L.skip ? 1.0f : L.s4.y, L.skip ? 1.0f : L.s4.z,
                         L.skip ? 1.0f : L.s4.w};
    O.skip = L.skip;
    O.lazy = L.lazy;
    O.oflag = C.sflag;
    O.ub = C.ub;
    // the stored weights plus the line's pending increments (0 unless the line is steady)
    const int pend = (SEMTSDF_STEADY && SEMTSDF_LAZY_WEIGHT && C.sflag) ? (int)C.sflag - 1 : 0;
    const int wo[4] = {L.w4.x + pend, L.w4.y + pend, L.w4.z + pend, L.w4.w + pend};
    float sn[4];
    int wn[4];
    // the reciprocal path's range over the lane's 4 voxels (touched or not: a running maximum of the
    // weights, a NaN-propagating minimum of |num|) instead of a per-voxel condition; the rare
    // exact path below decides per voxel
    unsigned wmax = 0u;
    float nmin = 1.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int tk = (int)(tmask << (31 - k)) >> 31;  // touched: all ones (v_bfe_i32), else 0
        const float num = fmaf(so[k], (float)wo[k], C.fv[k]);
        const float rw = s_rcp[min((unsigned)wo[k], (unsigned)kRcpTable - 1u)];
        const float upd = div_by_rcp(num, (float)wo[k] + 1.0f, rw);
        wmax = max(wmax, (unsigned)wo[k]);
        nmin = __builtin_elementwise_minimum(nmin, fabsf(num));
        // select by the touched mask as bits (v_bfi_b32): no per-voxel lane-mask compare
        sn[k] = __uint_as_float((__float_as_uint(upd) & (unsigned)tk) | (__float_as_uint(so[k]) & ~(unsigned)tk));
        wn[k] = wo[k] - tk;
    }
    if (!((wmax < (unsigned)kRcpTable) & (nmin >= 0x1p-60f)) || !a.fastdiv) {  // rare: weights past the table, tiny numerators
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float num = fmaf(so[k], (float)wo[k], C.fv[k]);
            const bool slow = !(((unsigned)wo[k] < (unsigned)kRcpTable) & (fabsf(num) >= 0x1p-60f)) || !a.fastdiv;
            if (!((tmask >> k) & 1u) || !slow) continue;
            sn[k] = num / (float)(wo[k] + 1);
        }
    }
    O.s4 = make_float4(sn[0], sn[1], sn[2], sn[3]);
    O.w4 = make_int4(wn[0], wn[1], wn[2], wn[3]);
    // a voxel crossed the threshold when so - thr and sn - thr differ in sign (each difference is
    // exact or keeps its sign; neither is -0): the sign bit of their XOR, ORed over the lane
    unsigned xs = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) xs |= __float_as_uint(so[k] - a.skip_thr) ^ __float_as_uint(sn[k] - a.skip_thr);
    O.cross = (int)xs < 0;
    if (FREE) return;  // no colour, histogram or vote state
    if (CI32) {  // tsdf.cu:57-62 on i32 colour; unchanged voxels of a stored row pass through
        // (element-wise selects: a select of whole int4 values is lowered through scratch)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int4 o = L.c32[k];
            const bool gk = (gmask >> k) & 1u;
            const int wi = wo[k], dw = wo[k] + 1;
            const int r0 = C.pix[k] & 0xFF, r1 = (C.pix[k] >> 8) & 0xFF, r2 = (C.pix[k] >> 16) & 0xFF;
            int4 n;
            n.x = gk ? avg_div(o.x * wi + r0, dw) : o.x;
            n.y = gk ? avg_div(o.y * wi + r1, dw) : o.y;
            n.z = gk ? avg_div(o.z * wi + r2, dw) : o.z;
            n.w = o.w;
            O.c32[k] = n;
        }
    } else {
        O.c8 = L.c8;
    }
    if (gmask) {  // tsdf.cu:57-62
        if (CI32) {
        } else {
            const unsigned co[4] = {L.c8.x, L.c8.y, L.c8.z, L.c8.w};
            unsigned cw[4];
            unsigned cslow = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool gk = (gmask >> k) & 1u;
                const unsigned wi = (unsigned)wo[k], o = co[k], px = C.pix[k];
                const float rw = s_rcp[min(wi, (unsigned)kRcpTable - 1u)];
                const unsigned n0 = avg_u8(o & 0xFFu, px & 0xFFu, wi, rw);
                const unsigned n1 = avg_u8((o >> 8) & 0xFFu, (px >> 8) & 0xFFu, wi, rw);
                const unsigned n2 = avg_u8((o >> 16) & 0xFFu, (px >> 16) & 0xFFu, wi, rw);
                cw[k] = gk ? (n0 | (n1 << 8) | (n2 << 16)) : o;
                cslow |= ((gk & (wi >= (unsigned)kRcpTable)) ? 1u : 0u) << k;
            }
            if (cslow) {  // rare: weights past the reciprocal table, exact integer quotient
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!(cslow & (1u << k))) continue;
                    const unsigned wi = (unsigned)wo[k], o = co[k], px = C.pix[k];
                    // int arithmetic of tsdf.cu:59 (c * w wraps past 2^31 at w > 8.4 M, as on the
                    // reference's hardware), truncating signed quotient, then the u8 store
                    const int dw = (int)(wi + 1u);
                    const unsigned n0 = (unsigned)((int)((o & 0xFFu) * wi + (px & 0xFFu)) / dw);
                    const unsigned n1 = (unsigned)((int)(((o >> 8) & 0xFFu) * wi + ((px >> 8) & 0xFFu)) / dw);
                    const unsigned n2 = (unsigned)((int)(((o >> 16) & 0xFFu) * wi + ((px >> 16) & 0xFFu)) / dw);
                    cw[k] = (n0 & 0xFFu) | ((n1 & 0xFFu) << 8) | ((n2 & 0xFFu) << 16);
                }
            }
            O.c8 = make_uint4(cw[0], cw[1], cw[2], cw[3]);
        }
        if (SEM) {  // tsdf.cu:61: +1 in the bin of the pixel's label
            O.h4 = make_uint4(L.h4.x + (gmask & 1u), L.h4.y + ((gmask >> 1) & 1u), L.h4.z + ((gmask >> 2) & 1u),
                              L.h4.w + ((gmask >> 3) & 1u));
        }
    }
    if (VOTE) {  // TSDF_Python/tsdf.cu:48-57
        int vc[4] = {L.vc4.x, L.vc4.y, L.vc4.z, L.vc4.w}, vn[4] = {L.vn4.x, L.vn4.y, L.vn4.z, L.vn4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!((tmask >> k) & 1u)) continue;
            if (vn[k] == 0) {
                vc[k] = L.vin[k];
                vn[k] = 1;
            } else if (vc[k] == L.vin[k]) {
                vn[k] += 1;
            } else {
                vn[k] -= 1;
            }
        }
        O.vc4 = make_int4(vc[0], vc[1], vc[2], vc[3]);
        O.vn4 = make_int4(vn[0], vn[1], vn[2], vn[3]);
    }
}

// Read-modify-writes of a voxel's own words (its histogram bins and bin mask) as no-return atomics
// at workgroup scope: within a launch one lane owns the voxel (units are disjoint), so no other
// lane -- on this XCD or another -- touches the word, and the kernel boundary's L2 write-back makes
// the result visible as for a store.  A device-scope atomic would be performed at memory (the
// XCDs' L2s are not coherent), hundreds of cycles longer in vmcnt, which the software pipeline's
// ordered waits then sit behind.  (Words shared by lanes, e.g. the bricks' dirty bits, keep device
// scope.)
__device__ __forceinline__ void voxel_or(uint32_t* p, uint32_t v) {
    (void)__hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void voxel_add(uint32_t* p, uint32_t v) {
    (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool SEM, bool CI32, bool VOTE, bool FREE, bool COUNT>
__device__ __forceinline__ void stage_store(const IntegrateArgs& a, const UnitPos& up, unsigned coff,
                                            const StoreMeta& M, const Out& O, unsigned& n_lazy) {
    const VolGeom& g = a.g;
    const unsigned tmask = M.meta & 15u, gmask = (M.meta >> 4) & 15u, hmode = (M.meta >> 8) & 3u,
                   hlab = M.meta >> 16;
    const bool trow = tile_line_any(tmask != 0u), grow = tile_line_any(gmask != 0u);
    // the lines with an update stay active together (the flag below is a ballot over a line)
    const bool line = SEMTSDF_FULLROW ? trow : ((__ballot(tmask != 0u) >> ((int)__lane_id() % LZQ +
                                                 lane_slot((int)__lane_id()) * kUnitLanes)) & kLineLanes) != 0ull;
    if (!line) return;
    const uint64_t v = O.ub + coff;
    {
        // a brick of the empty-space map changes only where a voxel crossed the threshold:
        // z-brick j of the unit holds the lanes of z-quads 2j, 2j+1 (lane = zq + 8 y)
        const uint64_t cb = __ballot(O.cross);
        // the struct through the constant address space (scalar loads, lgkmcnt) and its buffers as
        // global pointers: a pointer loaded from memory is generic, and the FLAT atomics and store
        // it would take count in vmcnt as another kind of event, after which the compiler waits
        // for every vector-memory operation at the top of the next group (vmcnt(0) in place of
        // vmcnt(5): the project stage's gathers no longer overlap the compute stage)
        const __attribute__((address_space(4))) IntegrateRare* R =
            (const __attribute__((address_space(4))) IntegrateRare*)a.rare;
        if (cb && R->bdirty) {  // rare: most updates keep their side of the threshold
            // lane j of a slot marks z-brick j of its unit (z-quads 2j, 2j+1)
            const int lane = (int)__lane_id(), j = lane % kUnitLanes;
            const int bz = (up.uz * UZ >> 3) + j;
            const uint64_t pj = ((kLineLanes << (2 * (j & 3))) | (kLineLanes << (2 * (j & 3) + 1)))
                                << (lane_slot(lane) * kUnitLanes);
            if (j < UZ / 8 && (cb & pj) && bz < R->nbz) {
                // the quad's dirty word; the lane that turns it nonzero lists the quad
                const unsigned nbq = (unsigned)(R->nbz + 3) >> 2;
                const unsigned q = __umul24(__umul24((unsigned)(up.x * UX >> 3), (unsigned)R->nby) +
                                                (unsigned)(up.uy * UY >> 3), nbq) + ((unsigned)bz >> 2);
                __attribute__((address_space(1))) uint32_t* bd = (__attribute__((address_space(1))) uint32_t*)R->bdirty;
                __attribute__((address_space(1))) uint32_t* dl = (__attribute__((address_space(1))) uint32_t*)R->dlist;
                if (__hip_atomic_fetch_or(bd + q, 1u << (bz & 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
                    dl[1 + __hip_atomic_fetch_add(dl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)] = q;
            }
        }
    }
    if (COUNT && O.lazy) n_lazy += 4u;
    if (!(kProbes && a.debug == 10) && !O.lazy && trow) {  // 10: timing probe, loads but no sdf/weight stores
        if (!O.skip) st_state(a.b.sdf + v, O.s4);
        st_state(a.b.wt + v, O.w4);
    }
    if (SEMTSDF_STEADY) {  // the line's flag byte after this update (one lane per line writes)
        // every sdf exactly 1.0f (bits: AND and OR of the four both equal 1.0f's) and every weight < 2^23
        const unsigned s_and = __float_as_uint(O.s4.x) & __float_as_uint(O.s4.y) & __float_as_uint(O.s4.z) &
                               __float_as_uint(O.s4.w);
        const unsigned s_or = __float_as_uint(O.s4.x) | __float_as_uint(O.s4.y) | __float_as_uint(O.s4.z) |
                              __float_as_uint(O.s4.w);
        const int wmx = max(max(O.w4.x, O.w4.y), max(O.w4.z, O.w4.w));
        const bool vals = (s_and == 0x3f800000u) & (s_or == 0x3f800000u) & (wmx < (1 << 23));
        // a lane that did not load its values (per-lane traffic) keeps what the old flag says
        const bool one = trow ? vals : (O.oflag != 0u);
        // a lazy line counts one more pending increment; any other update stored the weights
        // with the pending count folded in: steady (1) or not (0)
        const unsigned nb = O.lazy ? O.oflag + 1u : (tile_line_all(one) ? 1u : 0u);
        if (lane_y((int)__lane_id()) == 0 && nb != O.oflag) a.b.sflag[v >> 5] = (uint8_t)nb;
    }
    if (!FREE && grow) {
        if (CI32) {
#pragma unroll
            for (int k = 0; k < 4; ++k) reinterpret_cast<int4*>(a.b.color)[v + k] = O.c32[k];
        } else {
            st_state(reinterpret_cast<uint32_t*>(a.b.color) + v, O.c8);
        }
        if (SEM && gmask) {
            if (hmode == 1u) {
                st_state<uint4, SEMTSDF_NT_HIST>(a.b.hist + (uint64_t)hlab * g.nvox + v, O.h4);
                // a count that just became 1 sets the bin's bit in the voxel's bin mask (rare
                // once the surface has been seen: the common path neither reads nor writes it)
                const unsigned hk[4] = {O.h4.x, O.h4.y, O.h4.z, O.h4.w};
                unsigned nb = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) nb |= (((((gmask >> k) & 1u) != 0u) & (hk[k] == 1u)) ? 1u : 0u) << k;
                if (nb) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if ((nb >> k) & 1u) voxel_or(a.b.hmask + v + k, 1u << hlab);
                }
            }
            if (hmode == 2u) {  // rare: labels differ inside the lane, or a label >= 32
                unsigned bad = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const unsigned lab = (M.labs >> (8 * k)) & 0xFFu;
                    const bool gk = (gmask >> k) & 1u;
                    if (gk && lab < (unsigned)kMaxObjects) {
                        voxel_add(a.b.hist + (uint64_t)lab * g.nvox + v + k, 1u);
                        voxel_or(a.b.hmask + v + k, 1u << lab);
                    }
                    bad += (gk && lab >= (unsigned)kMaxObjects) ? 1u : 0u;
                }
                // an id without a histogram bin (tsdf.cu:61 writes past the voxel's 32 bins): the
                // vote is dropped and counted
                if (bad) {
                    const __attribute__((address_space(4))) IntegrateRare* R4 =
                        (const __attribute__((address_space(4))) IntegrateRare*)a.rare;
                    __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned long long*)R4->counters + 2,
                                           (unsigned long long)bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    if (!FREE && VOTE && tmask) {
        *reinterpret_cast<int4*>(a.b.cls + v) = O.vc4;
        *reinterpret_cast<int4*>(a.b.cls_cnt + v) = O.vn4;
    }
}

// One list of the frame as one persistent wave sees it: wave w takes the groups w', w' +
// nwaves, ... with w' = (w - rot) mod nwaves (rot continues the round-robin of the lists
// before it, so the waves with an extra group alternate), a group being kSlots consecutive
// entries, one unit per slot, of the list's compact array (k_compact_lists).
struct ListView {
    const unsigned* list;      // the list's first entry
    unsigned total, ngroups;   // wave-uniform; ngroups: end of the wave's range of groups
    unsigned cnt;              // groups in the wave's range (XCD split: its XCD's range)
    unsigned i;                // the wave's current group
};

// List l of the frame (base and total written by k_compact_lists; scalar loads).  XCD split
// (nsp == 8): the list's groups are cut into 8 contiguous ranges, range x taken by the waves of
// XCD x (workgroups b with b % 8 == x; the dispatcher deals workgroups to the XCDs round-robin),
// round-robin among them (wave index wave within the XCD, nwaves of them): a range is a compact
// region of the volume (the cull's segments are y-bands), so each XCD's L2 holds the pixel records
// and steady flags of its own region instead of every XCD fetching all of them.  ngroups is then
// the range's end and cnt its length.
__device__ __forceinline__ ListView list_view(const unsigned* units, const unsigned* list_count, int l, unsigned wave,
                                              unsigned nwaves, unsigned rot, unsigned xi = 0u, unsigned nsp = 1u) {
    const __attribute__((address_space(4))) unsigned* tw =
        (const __attribute__((address_space(4))) unsigned*)(list_count + kListTotalsWord);
    ListView v;
    v.list = units + tw[2 * l];
    v.total = tw[2 * l + 1];
    const unsigned ng = (v.total + kSlots - 1) / kSlots;
    const unsigned lo = nsp == 1u ? 0u : ng * xi / nsp;  // ng < 2^28 (list entries pack 32-bit unit ids)
    v.ngroups = nsp == 1u ? ng : ng * (xi + 1u) / nsp;
    v.cnt = v.ngroups - lo;
    v.i = lo + (wave + nwaves - rot % nwaves) % nwaves;
    return v;
}

// The entries of group grp < ngroups: one 8-byte scalar load (constant address space: it never
// waits behind the wave's vector memory operations); an odd list's last group reads the list's
// ~0u pad as its second entry.
static_assert(kSlots == 2, "two entries per group (one 8-byte load, one pad per list)");
__device__ __forceinline__ void group_entries(const ListView& v, unsigned grp, unsigned seg_cap, unsigned* e) {
    (void)seg_cap;
    const __attribute__((address_space(4))) unsigned* l4 = (const __attribute__((address_space(4))) unsigned*)v.list;
    e[0] = l4[2u * grp];
    e[1] = l4[2u * grp + 1u];
}

// The lane's unit of a group (the group's first entry exists).
__device__ __forceinline__ UnitPos lane_pos(const UnitGrid& ug, const unsigned* e) {
    const int slot = lane_slot(threadIdx.x & 63);
    UnitPos p = unit_pos(ug, e[0]);
#pragma unroll
    for (int k = 1; k < kSlots; ++k) {
        const bool have = e[k] != ~0u;
        const UnitPos q = unit_pos(ug, have ? e[k] : e[0]);
        if (slot == k) {
            p = q;
            p.ok = have;
        }
    }
    return p;
}

// Per-lane counts of the count mode (touched and gated voxels, touched lines on lane 0, lazy voxels).
struct Counts {
    unsigned touch, gate, lines, lazy;
};

// Pipeline state carried from one list into the next: the unit whose project, classify and
// load stages were issued (primed) but not yet computed and stored.
struct Pipe {
    UnitPos cur;
    Proj P;
    Cls C;
    Ld L;
    Out O;
    bool primed = false;
    unsigned lutv = 0;  // deferred relabel table, one dword per lane (IntegrateArgs::lut)
    unsigned groups = 0;  // priority rotation: SEMTSDF_PRIO_EVERY x the workgroup's dispatch round + groups done
};

// Unit-kind of a list: 0 general, 1 free (projected), 2 full free (no projection).
template <int KIND>
struct KindOf {
    static constexpr bool FREE = KIND != 0, FULL = KIND == 2;
};

// The project / classify / load stages of the wave's first group of list v (v.i < v.ngroups).
template <bool SEM, bool GATE, bool CI32, bool VOTE, bool COUNT, bool SHARD, bool PIN, int KIND>
__device__ __forceinline__ void list_prime(const IntegrateArgs& a, const UnitGrid& ug, unsigned seg_cap,
                                           const ListView& v, Pipe& S, Counts& n, const unsigned* pre = nullptr) {
    constexpr bool FREE = KindOf<KIND>::FREE, FULL = KindOf<KIND>::FULL;
    const int lane = threadIdx.x & 63;
    const unsigned coff = (unsigned)lane_zq(lane) * 32u + (unsigned)lane_y(lane) * 4u;
    unsigned e[kSlots];
    if (pre) {  // loaded ahead (the free list's first group, k_integrate)
        e[0] = pre[0];
        e[1] = pre[1];
    } else {
        group_entries(v, v.i, seg_cap, e);
    }
    S.cur = lane_pos(ug, e);
    stage_project<SHARD, PIN, FREE, FULL, VOTE>(a, S.cur, lane, S.P);
    stage_classify<SEM, GATE, VOTE, COUNT, FREE>(a, S.P, S.C, true, n.touch, n.gate, n.lines, S.lutv);
    stage_load<SEM, CI32, VOTE, FREE>(a, S.cur, coff, S.C, S.L);
    S.primed = true;
}

// Issue priority rotation of the persistent waves.  The 4 waves sharing a SIMD (one from each of
// the CU's 4 workgroups) are arbitrated by priority, then age: at equal priority the oldest wave
// issues first, and with equal static shares the waves end in age order, the youngest ≈ 40 %
// after the oldest (per-wave trace, profiles/r04/wave_trace_age.txt), the SIMD running its
// tail with fewer and fewer waves.  Each wave rotates its priority every group, offset by its
// workgroup's dispatch round (blockIdx / CUs: blocks are dealt to the CUs in rounds), so at
// any time the 4 waves of a SIMD hold distinct priorities and each holds the top one a
// quarter of the time.
#ifndef SEMTSDF_PRIO_ROTATE
#define SEMTSDF_PRIO_ROTATE 1
#endif
#ifndef SEMTSDF_PRIO_EVERY
#define SEMTSDF_PRIO_EVERY 4  // groups per priority step (a power of two); 1 rotated every group (r04)
#endif
static_assert((SEMTSDF_PRIO_EVERY & (SEMTSDF_PRIO_EVERY - 1)) == 0, "a power of two");
#ifndef SEMTSDF_PROBE_SALU
#define SEMTSDF_PROBE_SALU 0  // instrumentation builds: extra scalar ALU ops per group (issue probe)
#endif
#ifndef SEMTSDF_PROBE_VALU
#define SEMTSDF_PROBE_VALU 0  // instrumentation builds: extra vector ALU ops per group (issue probe)
#endif
__device__ __forceinline__ void rotate_prio(unsigned p) {
    if (!SEMTSDF_PRIO_ROTATE) return;
    switch (p & 3u) {  // s_setprio takes an immediate
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}
__device__ __forceinline__ unsigned dispatch_round() {
    return __builtin_amdgcn_readfirstlane((blockIdx.x * 4u) / gridDim.x);
}

// One list (kind KIND) by one persistent wave, software-pipelined.  The wave's last unit of
// the list is computed and stored under the project / classify / load of its first unit of
// the next list (kind NKIND, `nx`; NKIND < 0: none), which then starts primed: the pipeline
// does not drain and refill between the lists.
template <bool SEM, bool GATE, bool CI32, bool VOTE, bool COUNT, bool SHARD, bool PIN, int KIND, int NKIND>
__device__ __forceinline__ void integrate_list(const IntegrateArgs& a, const UnitGrid& ug, unsigned seg_cap,
                                               const float* __restrict__ s_rcp, ListView& v, const ListView* nx,
                                               unsigned nwaves, Pipe& S, Counts& n) {
    constexpr bool FREE = KindOf<KIND>::FREE, FULL = KindOf<KIND>::FULL;
    constexpr bool NFREE = KindOf<(NKIND < 0 ? 0 : NKIND)>::FREE, NFULL = KindOf<(NKIND < 0 ? 0 : NKIND)>::FULL;
    const int lane = threadIdx.x & 63;
    // the lane's offset from the unit origin (a volume has < 2^31 stored voxels per x-plane pair)
    const unsigned coff = (unsigned)lane_zq(lane) * 32u + (unsigned)lane_y(lane) * 4u;
    // no group of this list for the wave: the next list primes itself (a primed pipeline
    // always holds a unit of the first list, in order, that has a group for the wave)
    if (v.i >= v.ngroups) return;
    if (!S.primed) list_prime<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, KIND>(a, ug, seg_cap, v, S, n);
    unsigned en[kSlots];
    if (v.i + nwaves < v.ngroups) group_entries(v, v.i + nwaves, seg_cap, en);
    const bool chain = NKIND >= 0 && SEMTSDF_CHAIN && nx->i < nx->ngroups;
    unsigned eb[kSlots];
    if (NKIND >= 0 && SEMTSDF_CHAIN && chain) group_entries(*nx, nx->i, seg_cap, eb);
    while (v.i + nwaves < v.ngroups) {
        const UnitPos nxt = lane_pos(ug, en);
        if (v.i + 2u * nwaves < v.ngroups) group_entries(v, v.i + 2u * nwaves, seg_cap, en);
        stage_project<SHARD, PIN, FREE, FULL, VOTE>(a, nxt, lane, S.P);
        stage_compute<SEM, GATE, CI32, VOTE, FREE>(a, s_rcp, S.C, S.L, S.O);
        const StoreMeta Mc = store_meta(S.C);
        stage_classify<SEM, GATE, VOTE, COUNT, FREE>(a, S.P, S.C, true, n.touch, n.gate, n.lines, S.lutv);
        stage_store<SEM, CI32, VOTE, FREE, COUNT>(a, S.cur, coff, Mc, S.O, n.lazy);
        stage_load<SEM, CI32, VOTE, FREE>(a, nxt, coff, S.C, S.L);
        S.cur = nxt;
        v.i += nwaves;
        // the wave's group counter (no division by nwaves in the loop): a priority step every
        // SEMTSDF_PRIO_EVERY groups
        ++S.groups;
        if (SEMTSDF_PRIO_EVERY == 1 || (S.groups & (SEMTSDF_PRIO_EVERY - 1u)) == 0u)
            rotate_prio(S.groups / SEMTSDF_PRIO_EVERY);
#if SEMTSDF_PROBE_SALU || SEMTSDF_PROBE_VALU
        {  // issue probes (instrumentation builds only): N extra scalar / vector ALU ops per group
            unsigned su = S.groups, vu = threadIdx.x;
#pragma unroll
            for (int q = 0; q < SEMTSDF_PROBE_SALU; ++q) asm volatile("s_mov_b32 %0, %0" : "+s"(su));
#pragma unroll
            for (int q = 0; q < SEMTSDF_PROBE_VALU; ++q) asm volatile("v_add_u32 %0, %0, 1" : "+v"(vu));
            if (su == 0xFFFFFFFFu && vu == 0xFFFFFFFFu) S.lutv ^= 1u;  // keeps the probes live
        }
#endif
    }
    // the wave's last unit of this list
    if (NKIND >= 0 && SEMTSDF_CHAIN && chain) {
        const UnitPos nxt = lane_pos(ug, eb);
        stage_project<SHARD, PIN, NFREE, NFULL, VOTE>(a, nxt, lane, S.P);
        stage_compute<SEM, GATE, CI32, VOTE, FREE>(a, s_rcp, S.C, S.L, S.O);
        const StoreMeta Mc = store_meta(S.C);
        stage_classify<SEM, GATE, VOTE, COUNT, NFREE>(a, S.P, S.C, true, n.touch, n.gate, n.lines, S.lutv);
        stage_store<SEM, CI32, VOTE, FREE, COUNT>(a, S.cur, coff, Mc, S.O, n.lazy);
        stage_load<SEM, CI32, VOTE, NFREE>(a, nxt, coff, S.C, S.L);
        S.cur = nxt;
        S.primed = true;
    } else {
        stage_compute<SEM, GATE, CI32, VOTE, FREE>(a, s_rcp, S.C, S.L, S.O);
        stage_store<SEM, CI32, VOTE, FREE, COUNT>(a, S.cur, coff, store_meta(S.C), S.O, n.lazy);
        S.primed = false;
    }
    v.i += nwaves;
}

// The last list (general units) with its groups past the first round handed out at run time,
// software-pipelined like integrate_list.  The wave's first group is its static one (v.i <
// nwaves, primed by the chain from the list before); groups nwaves .. ngroups - 1 are cut into
// one slice per XCD and handed out through the XCD's own counter (zeroed by the frame's prepass),
// so waves that finished their earlier lists early take more of them and the waves end together.
// The counter of XCD x is only touched by waves running on XCD x (the XCC_ID register), so its
// atomics are workgroup-scope: performed in that XCD's L2.  Every lane of the wave executes the
// atomic (lane 0 adds 1, the others 0: no divergent branch, so the compiler counts the atomic
// among the wave's vector-memory operations in order), and the ticket of the group after next
// is claimed at the end of an iteration and read after the next compute stage, which waits for
// the state loads issued before it anyway: the claim's round trip hides under the pipeline.
#ifndef SEMTSDF_DYN_LAST
#define SEMTSDF_DYN_LAST 0
#endif
template <bool SEM, bool GATE, bool CI32, bool VOTE, bool COUNT, bool SHARD, bool PIN>
__device__ __forceinline__ void integrate_list_dyn(const IntegrateArgs& a, const UnitGrid& ug, unsigned seg_cap,
                                                   const float* __restrict__ s_rcp, ListView& v, unsigned nwaves,
                                                   unsigned* xcd_counters, Pipe& S, Counts& n) {
    const int lane = threadIdx.x & 63;
    const unsigned coff = (unsigned)lane_zq(lane) * 32u + (unsigned)lane_y(lane) * 4u;
    if (v.i >= v.ngroups) return;  // then ngroups <= nwaves: no dynamic group either
    if (!S.primed) list_prime<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 0>(a, ug, seg_cap, v, S, n);
    // HW_REG_XCC_ID (hwreg 20), bits 3:0: the XCD this wave runs on
    const unsigned xcc = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11))) & 7u;
    // one slice per (XCD, workgroup slot): a single counter per XCD saturates (same-address L2
    // atomics serialise), so the waves of an XCD share kDynSub counters
    const unsigned sub = (blockIdx.x >> 3) & (kDynSub - 1u), sl = xcc * kDynSub + sub, ns = 8u * kDynSub;
    const unsigned D = v.ngroups - min(v.ngroups, nwaves);
    const unsigned lo = nwaves + D * sl / ns, cnt = nwaves + D * (sl + 1u) / ns - lo;
    unsigned* ctr = xcd_counters + sl * kListCountStride;
    auto claim = [&]() -> unsigned {
        unsigned r = 0u;
        if (lane == 0) r = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return r;
    };
    unsigned en[kSlots];
    unsigned t = cnt ? (unsigned)__builtin_amdgcn_readlane((int)claim(), 0) : 0u;
    bool have = t < cnt;
    if (have) group_entries(v, lo + t, seg_cap, en);
    // claimed unconditionally (a claim past the slice only moves its counter further): a
    // conditional one merges with the loop's previous value, and that copy waits for the atomic
    unsigned pend = claim();
    while (have) {
        const UnitPos nxt = lane_pos(ug, en);
        stage_project<SHARD, PIN, false, false, VOTE>(a, nxt, lane, S.P);
        stage_compute<SEM, GATE, CI32, VOTE, false>(a, s_rcp, S.C, S.L, S.O);
        const unsigned t2 = (unsigned)__builtin_amdgcn_readlane((int)pend, 0);
        const bool have2 = t2 < cnt;
        if (have2) group_entries(v, lo + t2, seg_cap, en);
        const StoreMeta Mc = store_meta(S.C);
        stage_classify<SEM, GATE, VOTE, COUNT, false>(a, S.P, S.C, true, n.touch, n.gate, n.lines, S.lutv);
        stage_store<SEM, CI32, VOTE, false, COUNT>(a, S.cur, coff, Mc, S.O, n.lazy);
        stage_load<SEM, CI32, VOTE, false>(a, nxt, coff, S.C, S.L);
        pend = claim();
        S.cur = nxt;
        have = have2;
        ++S.groups;
        if (SEMTSDF_PRIO_EVERY == 1 || (S.groups & (SEMTSDF_PRIO_EVERY - 1u)) == 0u)
            rotate_prio(S.groups / SEMTSDF_PRIO_EVERY);
    }
    stage_compute<SEM, GATE, CI32, VOTE, false>(a, s_rcp, S.C, S.L, S.O);
    stage_store<SEM, CI32, VOTE, false, COUNT>(a, S.cur, coff, store_meta(S.C), S.O, n.lazy);
    S.primed = false;
    v.i = v.ngroups;
}

// The dynamic tail of the last list: groups first .. first + ntail - 1, cut into one slice per
// XCD, handed out one at a time through the XCD's own counter (zeroed by the frame's prepass),
// each group integrated without the software pipeline (its latency is hidden across the waves
// instead).  The static round-robin shares end unevenly (per CU by up to ~15 % of the kernel:
// profiles/r05/wave_trace_*.txt); waves that finish theirs early take the tail, so the waves end
// together.  The counter of XCD x is only touched by waves running on XCD x (the XCC_ID register),
// so its atomics are workgroup-scope: performed in that XCD's L2 (agent-scope atomics go to memory
// and serialise at ~20 ns each, 2x slower kernels).  Ticket in lane 0 (the compiler waits for all
// of the wave's memory operations before using it: nothing else is in flight here).
#ifndef SEMTSDF_TAIL_PCT
#define SEMTSDF_TAIL_PCT 0  // percent of the last list's groups handed out dynamically (measured slower at 10-35 %: 0)
#endif
template <bool SEM, bool GATE, bool CI32, bool VOTE, bool COUNT, bool SHARD, bool PIN>
__device__ __forceinline__ void integrate_tail(const IntegrateArgs& a, const UnitGrid& ug, unsigned seg_cap,
                                               const float* __restrict__ s_rcp, const ListView& v, unsigned first,
                                               unsigned ntail, unsigned* counters, Pipe& S, Counts& n) {
    const int lane = threadIdx.x & 63;
    const unsigned coff = (unsigned)lane_zq(lane) * 32u + (unsigned)lane_y(lane) * 4u;
    // HW_REG_XCC_ID (hwreg 20), bits 3:0: the XCD this wave runs on
    const unsigned xcc = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11))) & 7u;
    const unsigned lo = first + ntail * xcc / 8u, hi = first + ntail * (xcc + 1u) / 8u;
    unsigned* counter = counters + xcc * kListCountStride;
    for (;;) {
        unsigned t = 0u;
        if (lane == 0) t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
        if (t >= hi - lo) break;
        unsigned e[kSlots];
        group_entries(v, lo + t, seg_cap, e);
        S.cur = lane_pos(ug, e);
        stage_project<SHARD, PIN, false, false, VOTE>(a, S.cur, lane, S.P);
        stage_classify<SEM, GATE, VOTE, COUNT, false>(a, S.P, S.C, true, n.touch, n.gate, n.lines, S.lutv);
        stage_load<SEM, CI32, VOTE, false>(a, S.cur, coff, S.C, S.L);
        stage_compute<SEM, GATE, CI32, VOTE, false>(a, s_rcp, S.C, S.L, S.O);
        stage_store<SEM, CI32, VOTE, false, COUNT>(a, S.cur, coff, store_meta(S.C), S.O, n.lazy);
    }
}

// Persistent wavefronts over the three live-unit lists of the frame: the full free units, the
// free units (both sdf/weight only, when the mode allows them), then the general units, the
// pipeline chained from each list into the next.  A static round-robin share: dynamic
// schedules (per-XCD device atomics, a whole-CU workgroup sharing an LDS queue) evened the
// waves' end times but ran slower.
static_assert(!SEMTSDF_XCD_SPLIT || (!SEMTSDF_DYN_LAST && !SEMTSDF_TAIL_PCT),
              "the dynamic schedules hand out the whole list (no XCD ranges)");
#ifndef SEMTSDF_INTEGRATE_WPE
#define SEMTSDF_INTEGRATE_WPE 4  // waves per SIMD the register allocation targets (5 spills; measured equal)
#endif
template <bool SEM, bool GATE, bool CI32, bool VOTE, bool COUNT, bool SHARD, bool PIN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VOTE ? 3 : SEMTSDF_INTEGRATE_WPE))) void k_integrate(
    IntegrateArgs a, UnitGrid ug, unsigned seg_cap) {
    __shared__ float s_rcp[kRcpTable];
    // instrumentation: per-wave wall-clock marks (entry, table loaded, after each list) and
    // the wave's group counts per list
    unsigned long long tr[5] = {0, 0, 0, 0, 0};
    unsigned long long trn = 0;
    const unsigned nwaves = gridDim.x * (blockDim.x >> 6);
#ifndef SEMTSDF_WAVE_PERM
#define SEMTSDF_WAVE_PERM 0
#endif
    // the wave's slot in the round-robin of the lists; SEMTSDF_WAVE_PERM=1: the 4 waves of a
    // workgroup take slots nwaves/4 apart, so consecutive (adjacent) groups go to different CUs
    const unsigned wave = __builtin_amdgcn_readfirstlane(
        SEMTSDF_WAVE_PERM ? (threadIdx.x >> 6) * gridDim.x + blockIdx.x : blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    auto groups_of = [&](unsigned n, unsigned rot_) -> unsigned long long {
        const unsigned ng = (n + kSlots - 1) / kSlots, i0 = (wave + nwaves - rot_ % nwaves) % nwaves;
        return i0 < ng ? (ng - 1u - i0) / nwaves + 1u : 0u;
    };
    if (SEMTSDF_WAVE_TRACE) tr[0] = wall_clock64();
    // the reciprocal table is first read by a compute stage: the wave primes its first group
    // (gathers and state loads in flight) before the workgroup's barrier
    for (int i = (int)threadIdx.x; i < kRcpTable; i += (int)blockDim.x) s_rcp[i] = a.rcp_table[i];
    const int lane = threadIdx.x & 63;
    Counts n{};
    unsigned nlive = 0;
    Pipe S;
    S.groups = dispatch_round() * SEMTSDF_PRIO_EVERY;
    if (SEM && a.lut) S.lutv = reinterpret_cast<const uint32_t*>(a.lut)[lane];
    const unsigned* cnt = a.list_count;
    unsigned* tail_counter = a.list_count + kLists * kListSegs * kListCountStride;  // zeroed by the prepass
    const unsigned* lst = a.units;
    unsigned n0;
    unsigned rot0 = 0;
    // XCD split (list_view): the wave's XCD xi and its index wx among the XCD's nwx waves
    const bool split = SEMTSDF_XCD_SPLIT && (gridDim.x & 7u) == 0u;
    const unsigned nsp = split ? 8u : 1u, xi = split ? blockIdx.x & 7u : 0u;
    const unsigned wx = split ? __builtin_amdgcn_readfirstlane((blockIdx.x >> 3) * (blockDim.x >> 6) + (threadIdx.x >> 6))
                              : wave;
    const unsigned nwx = nwaves / nsp;
    if (GATE && !VOTE) {  // free units exist only in gated modes (free_ok): full free, free, general
        // the free list lies at the start of the compact array and its groups start at the wave's
        // own index: the wave's first free group is read before the lists' totals have arrived
        // (one dependent load less at the start of the kernel; most waves prime a free group)
        const __attribute__((address_space(4))) unsigned* u4 = (const __attribute__((address_space(4))) unsigned*)lst;
        // (the array holds at least 2 x 65536 entries, semtsdf_api.cpp: waves past kPreWaves read their
        // first group the ordinary way)
        // XCD split: the wave's first free group from the table k_compact_lists wrote for this grid
        const bool tab = split && a.first_nwaves == nwaves;
        const unsigned wq = min(wave, kPreWaves - 1u);
        const __attribute__((address_space(4))) unsigned* t4 =
            tab ? (const __attribute__((address_space(4))) unsigned*)a.first_tab : u4;
        const unsigned pre1[2] = {t4[2u * wq], t4[2u * wq + 1u]};
        ListView vf = list_view(lst, cnt, 2, wx, nwx, 0u, xi, nsp);
        ListView v1 = list_view(lst, cnt, 1, wx, nwx, 0u, xi, nsp);
        rot0 = (vf.cnt + v1.cnt) % nwx;
        ListView v0 = list_view(lst, cnt, 0, wx, nwx, rot0, xi, nsp);
        const unsigned tail0 = SEMTSDF_TAIL_PCT ? v0.ngroups * SEMTSDF_TAIL_PCT / 100u : 0u;
        v0.ngroups -= tail0;  // the static share: groups 0 .. ngroups - tail0 - 1
        if (vf.i < vf.ngroups)
            list_prime<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 2>(a, ug, seg_cap, vf, S, n);
        else if (v1.i < v1.ngroups)
            list_prime<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 1>(a, ug, seg_cap, v1, S, n,
                                                                   (!split || tab) && wq == wave ? pre1 : nullptr);
        else if (v0.i < v0.ngroups)
            list_prime<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 0>(a, ug, seg_cap, v0, S, n);
        __syncthreads();
        if (SEMTSDF_WAVE_TRACE) tr[1] = tr[2] = tr[3] = wall_clock64();
        integrate_list<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 2, 1>(a, ug, seg_cap, s_rcp, vf, &v1, nwx, S, n);
        if (SEMTSDF_WAVE_TRACE) tr[2] = wall_clock64();
        integrate_list<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 1, 0>(a, ug, seg_cap, s_rcp, v1, &v0, nwx, S, n);
        if (SEMTSDF_WAVE_TRACE) {
            tr[3] = wall_clock64();
            trn = groups_of(vf.total, 0u) | (groups_of(v1.total, 0u) << 20);
        }
        if (SEMTSDF_DYN_LAST)
            integrate_list_dyn<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>(a, ug, seg_cap, s_rcp, v0, nwaves, tail_counter, S, n);
        else
            integrate_list<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 0, -1>(a, ug, seg_cap, s_rcp, v0, nullptr, nwx, S, n);
        if (tail0) integrate_tail<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>(a, ug, seg_cap, s_rcp, v0, v0.ngroups, tail0,
                                                                           tail_counter, S, n);
        n0 = v0.total;
        if (COUNT && blockIdx.x == 0 && threadIdx.x == 0) {
            atomicAdd(a.counters + 4, (unsigned long long)(v1.total + vf.total));
            atomicAdd(a.counters + 5, (unsigned long long)vf.total);
        }
        if (COUNT) nlive += v1.total + vf.total;
    } else {
        // no free units in these modes: the free and full-free lists are empty and the general list
        // starts at entry 4 of the compact array (k_compact_lists), so the wave's first group is
        // read before the totals arrive (used when the base is indeed 4)
        const __attribute__((address_space(4))) unsigned* u4 = (const __attribute__((address_space(4))) unsigned*)lst;
        const bool tab = split && a.first_nwaves == nwaves;
        const unsigned wq = min(wave, kPreWaves - 1u);
        const __attribute__((address_space(4))) unsigned* t4 =
            tab ? (const __attribute__((address_space(4))) unsigned*)a.first_tab - 4 : u4;
        const unsigned pre0[2] = {t4[4u + 2u * wq], t4[5u + 2u * wq]};
        ListView v0 = list_view(lst, cnt, 0, wx, nwx, 0u, xi, nsp);
        const unsigned tail0 = SEMTSDF_TAIL_PCT ? v0.ngroups * SEMTSDF_TAIL_PCT / 100u : 0u;
        v0.ngroups -= tail0;
        if (v0.i < v0.ngroups)
            list_prime<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 0>(a, ug, seg_cap, v0, S, n,
                                                                   (tab || (!split && v0.list == lst + 4)) && wq == wave ? pre0
                                                                                                                : nullptr);
        __syncthreads();
        if (SEMTSDF_WAVE_TRACE) tr[1] = tr[2] = tr[3] = wall_clock64();
        if (SEMTSDF_DYN_LAST)
            integrate_list_dyn<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>(a, ug, seg_cap, s_rcp, v0, nwaves, tail_counter, S, n);
        else
            integrate_list<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN, 0, -1>(a, ug, seg_cap, s_rcp, v0, nullptr, nwx, S, n);
        if (tail0) integrate_tail<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>(a, ug, seg_cap, s_rcp, v0, v0.ngroups, tail0,
                                                                           tail_counter, S, n);
        n0 = v0.total;
    }
#if SEMTSDF_TAIL_CULL_PROBE
    {  // timing probe (instrumentation builds only): a unit cull of the whole grid as tail work,
       // tasks of 64 units claimed through the XCD's own counter (zeroed by the prepass); results discarded
        const unsigned xcc = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11))) & 7u;
        unsigned* ctr = tail_counter + xcc * kListCountStride;
        const unsigned ntask = (ug.n + 63u) / 64u;
        const unsigned nmine = ntask > xcc ? (ntask - xcc + 7u) / 8u : 0u;
        unsigned acc = 0;
        for (;;) {
            unsigned t = 0;
            if (lane == 0) t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
            if (t >= nmine) break;
            const unsigned u = (t * 8u + xcc) * 64u + (unsigned)lane;
            if (u < ug.n) {
                const unsigned ux = u % ug.nux, r = u / ug.nux, uy = r % ug.nuy, uz = r / ug.nuy;
                acc += (unsigned)unit_cull(a, (int)ux * UX, (int)uy * UY, (int)uz * UZ);
            }
        }
        if (acc == 0xFFFFFFFFu) a.counters[7] = acc;  // keeps the work live
    }
#endif
    if (SEM && a.lut && a.relabel_mask) {  // the frame's mask through the same table, in place
        const unsigned npx = (unsigned)(a.width * a.height);
        const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
        uint32_t* m4 = reinterpret_cast<uint32_t*>(a.relabel_mask);
        const bool al = ((uintptr_t)a.relabel_mask & 3u) == 0u;
        const unsigned n4 = al ? npx >> 2 : 0u;
        for (unsigned base = 0; base < n4; base += nth) {  // uniform trip count: every lane shuffles
            const unsigned i = base + gid;
            const uint32_t v = i < n4 ? m4[i] : 0u;
            uint32_t o = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) o |= (relabel_rec(v << (24 - 8 * k), S.lutv) >> 24) << (8 * k);
            if (i < n4) m4[i] = o;
        }
        for (unsigned base = n4 * 4; base < npx; base += nth) {  // unaligned mask or the tail bytes
            const unsigned i = base + gid;
            const uint32_t v = i < npx ? (uint32_t)a.relabel_mask[i] : 0u;
            const uint32_t o = relabel_rec(v << 24, S.lutv) >> 24;
            if (i < npx) a.relabel_mask[i] = (uint8_t)o;
        }
    }
    if (SEMTSDF_WAVE_TRACE && a.wtrace && wave < a.wtrace_slots) {
        tr[4] = wall_clock64();
        trn |= groups_of(n0, rot0) << 40;
        if (lane < 8) {
            const unsigned long long hw = (unsigned long long)__smid() | ((unsigned long long)blockIdx.x << 32);
            // word 7: HW_ID (wave id bits 3:0, SIMD bits 5:4, CU bits 11:8, ...) for per-SIMD analyses
            const unsigned hwid = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
            const unsigned long long v = lane < 5 ? tr[lane < 5 ? lane : 0] : lane == 5 ? hw : lane == 6 ? trn : (unsigned long long)hwid;
            a.wtrace[(size_t)wave * kWaveTraceWords + lane] = v;
        }
    }
    if (COUNT) {
        nlive += n0;
        unsigned long long t = n.touch, gg = n.gate, lz = n.lazy, tl = n.lines;
        for (int off = 32; off > 0; off >>= 1) {
            t += __shfl_xor(t, off, 64);
            gg += __shfl_xor(gg, off, 64);
            lz += __shfl_xor(lz, off, 64);
            tl += __shfl_xor(tl, off, 64);
        }
        if (lane == 0) {
            if (t) atomicAdd(a.counters + 0, t);
            if (gg) atomicAdd(a.counters + 1, gg);
            if (lz) atomicAdd(a.counters + 6, lz);
            if (tl) atomicAdd(a.counters + 7, tl);
        }
        // live units of both lists
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.counters + 3, (unsigned long long)nlive);
    }
}

// Persistent grid sized to exactly the resident capacity (blocks/CU from the occupancy
// query x CUs): an oversubscribed persistent grid leaves a tail of late blocks.
static unsigned resident_grid_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
    return (unsigned)cus;
}

template <typename K>
static unsigned resident_grid(K kernel, int block = 256) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess || per < 1) per = 1;
    return (unsigned)(cus * per);
}

template <bool SEM, bool GATE, bool CI32, bool VOTE, bool COUNT, bool SHARD, bool PIN>
static hipError_t launch_integrate_k(const IntegrateArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const UnitGrid ug = unit_grid(a.g);
    if (ug.n == 0) return hipSuccess;
    // persistent grid of the resident capacity; the waves share the list evenly, so a grid
    // past residency (the occupancy query can over-report, MI355X_MICROARCH.md) only adds
    // late waves with the same share
    constexpr int block = 256;
    static const unsigned grid0 = resident_grid(k_integrate<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>, block);
    const unsigned ncu = resident_grid_cus();
    unsigned grid = grid0;
    if (kProbes && a.debug >= 100) grid = grid0 * (unsigned)(a.debug - 100) / 8u;  // probe: fraction of residency
    static const char* gpc = getenv("SEMTSDF_GRID_PER_CU");              // probe: blocks per CU
    if (gpc && atoi(gpc) > 0) grid = ncu * (unsigned)atoi(gpc);
    if (e0) {  // timing: events recorded by the dispatch itself (kernel start / end)
        hipExtLaunchKernelGGL((k_integrate<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>), dim3(grid), dim3(block), 0, s, e0,
                              e1, 0, a, ug, list_seg_cap(ug));
    } else {
        hipLaunchKernelGGL((k_integrate<SEM, GATE, CI32, VOTE, COUNT, SHARD, PIN>), dim3(grid), dim3(block), 0, s, a, ug,
                           list_seg_cap(ug));
    }
    return hipGetLastError();
}

template <bool SEM, bool GATE, bool CI32, bool VOTE>
static hipError_t launch_integrate_t(const IntegrateArgs& a, bool count, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const bool shard = a.g.nshards > 1, pin = a.pinhole != 0;
    if (count) {  // measurement pass: pinhole only is not assumed
        if (shard) return launch_integrate_k<SEM, GATE, CI32, VOTE, true, true, false>(a, s, e0, e1);
        return launch_integrate_k<SEM, GATE, CI32, VOTE, true, false, false>(a, s, e0, e1);
    }
    if (shard) {
        if (pin) return launch_integrate_k<SEM, GATE, CI32, VOTE, false, true, true>(a, s, e0, e1);
        return launch_integrate_k<SEM, GATE, CI32, VOTE, false, true, false>(a, s, e0, e1);
    }
    if (pin) return launch_integrate_k<SEM, GATE, CI32, VOTE, false, false, true>(a, s, e0, e1);
    return launch_integrate_k<SEM, GATE, CI32, VOTE, false, false, false>(a, s, e0, e1);
}

unsigned integrate_pre_waves() {
    // the SfM semantic instantiation (the others run at the same occupancy; where one does not, its
    // waves read their first group the ordinary way: k_integrate compares first_nwaves with its grid)
    static const unsigned w = 4u * resident_grid(k_integrate<true, true, false, false, false, false, true>, 256);
    return w;
}

hipError_t launch_integrate(const IntegrateArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const bool count = a.counters != nullptr && (a.flags & 0x80000000u);
    // ci32: the colour STORAGE is int32 x 4 (a COLOR_I32 volume holding values outside [0, 255]);
    // a COLOR_I32 volume whose colours fit a byte stores them as u8 x 4 and integrates them
    // with the same integer quotient (semtsdf_api.cpp: color_wide)
    const bool sem = a.flags & 0x1u, gate = a.flags & 0x2u, ci32 = a.color_wide != 0, vote = a.flags & 0x8u;
    // Instantiated mode combinations: SfM semantic (u8 colour, gated), TSDF+colour (NumPy
    // rule: i32 colour, ungated), TSDF_Python vote, plus their neighbours.
    if (vote) {
        if (ci32) return launch_integrate_t<false, false, true, true>(a, count, s, e0, e1);
        return launch_integrate_t<false, false, false, true>(a, count, s, e0, e1);
    }
    if (sem) {
        if (gate) {
            if (ci32) return launch_integrate_t<true, true, true, false>(a, count, s, e0, e1);
            return launch_integrate_t<true, true, false, false>(a, count, s, e0, e1);
        }
        if (ci32) return launch_integrate_t<true, false, true, false>(a, count, s, e0, e1);
        return launch_integrate_t<true, false, false, false>(a, count, s, e0, e1);
    }
    if (gate) {
        if (ci32) return launch_integrate_t<false, true, true, false>(a, count, s, e0, e1);
        return launch_integrate_t<false, true, false, false>(a, count, s, e0, e1);
    }
    if (ci32) return launch_integrate_t<false, false, true, false>(a, count, s, e0, e1);
    return launch_integrate_t<false, false, false, false>(a, count, s, e0, e1);
}

// ------------------------------------------------------------------------------------
// trilinear samplers (utils.cu:99-170), clamped to the volume (the reference reads out of
// range at the far faces; the clamp defines that case).
// ------------------------------------------------------------------------------------
struct Tri {
    uint32_t i000;            // tiled index of the base corner (stored voxels < 2^32)
    uint32_t dx, dy;          // offsets to x+1 / y+1 (0 when clamped)
    uint32_t dz;
    float fx, fy, fz;
};

// Base voxel (clamped) of the trilinear sample at p, its local plane and the fractions.
struct TriCoord {
    int xc, yc, zc, zl;   // clamped base voxel; zl = local plane of zc
    int dxv, dyv, dzv;    // 1, or 0 where the +1 neighbour is clamped
    float fx, fy, fz;
};

// SH = false: an unsharded volume (local z == global z) known at compile time (the
// single-volume marches), so the sharded plane mapping is not compiled in.
template <bool SH = true>
__device__ __forceinline__ TriCoord tri_coord(const VolGeom& g, float px, float py, float pz) {
    const float ix = vox_coord(px, g.start[0], g.voxel[0], g.rvox[0]);
    const float iy = vox_coord(py, g.start[1], g.voxel[1], g.rvox[1]);
    const float iz = vox_coord(pz, g.start[2], g.voxel[2], g.rvox[2]);
    // floor and clamp in the float domain: a sample lies within a few voxels of the volume
    // box, so floor(i) is an integer far inside the int range and (float)f2i_rd(i) ==
    // floorf(i); clamp(x, 0, dim - 1) and clamp(x + 1, 0, dim - 1) - clamp(x, 0, dim - 1)
    // (1 strictly inside [0, dim - 1), else 0) are the same integers as the int forms
    const float flx = floorf(ix), fly = floorf(iy), flz = floorf(iz);
    const float hx = (float)(g.dimx - 1), hy = (float)(g.dimy - 1), hz = (float)(g.dimz - 1);
    TriCoord c;
    c.fx = ix - flx;
    c.fy = iy - fly;
    c.fz = iz - flz;
    c.xc = (int)fminf(fmaxf(flx, 0.0f), hx);
    c.yc = (int)fminf(fmaxf(fly, 0.0f), hy);
    c.zc = (int)fminf(fmaxf(flz, 0.0f), hz);
    c.dxv = ((flx >= 0.0f) & (flx < hx)) ? 1 : 0;
    c.dyv = ((fly >= 0.0f) & (fly < hy)) ? 1 : 0;
    c.dzv = ((flz >= 0.0f) & (flz < hz)) ? 1 : 0;
    // global plane -> local plane of this shard (the caller only samples planes it owns;
    // zc + 1 is then the chunk's next plane or its halo plane)
    c.zl = (!SH || g.nshards == 1) ? c.zc : global_to_local_z(g, c.zc);
    return c;
}

// Corner indices in the tiled layout: the index is a sum of per-axis terms, so the
// offsets to the +1 neighbours are differences of those terms.
__device__ __forceinline__ Tri tri_from(const VolGeom& g, const TriCoord& c) {
    Tri t;
    const uint32_t y0 = tile_yterm(g, c.yc), z0 = tile_zterm(c.zl);
    t.i000 = tile_xterm(g, c.xc) + y0 + z0;
    t.dx = c.dxv ? g.tx : 0u;
    t.dy = tile_yterm(g, c.yc + c.dyv) - y0;
    t.dz = tile_zterm(c.zl + c.dzv) - z0;
    t.fx = c.fx; t.fy = c.fy; t.fz = c.fz;
    return t;
}

template <bool SH = true>
__device__ __forceinline__ Tri tri_setup(const VolGeom& g, float px, float py, float pz) {
    return tri_from(g, tri_coord<SH>(g, px, py, pz));
}

// Empty-space map: brick of 8^3 local voxels holding the sample's 8 corners.
__device__ __forceinline__ int brick_of(const VolGeom& g, const TriCoord& c) {
    return (int)__umul24(__umul24((unsigned)(c.xc >> 3), (unsigned)g.nby) + (unsigned)(c.yc >> 3), (unsigned)g.nbz) +
           (c.zl >> 3);
}

template <typename T>
__device__ __forceinline__ float tri_eval(const T* __restrict__ p, const Tri& t) {
    // d[i*4+j*2+k] = vol[x+i][y+j][z+k]
    const T* q = p + t.i000;
    const float d0 = (float)q[0], d1 = (float)q[t.dz];
    const float d2 = (float)q[t.dy], d3 = (float)q[t.dy + t.dz];
    const float d4 = (float)q[t.dx], d5 = (float)q[t.dx + t.dz];
    const float d6 = (float)q[t.dx + t.dy], d7 = (float)q[t.dx + t.dy + t.dz];
    const float low = mixf(mixf(d0, d4, t.fx), mixf(d2, d6, t.fx), t.fy);
    const float high = mixf(mixf(d1, d5, t.fx), mixf(d3, d7, t.fx), t.fy);
    return mixf(low, high, t.fz);
}

// Histogram bins that are nonzero at one of the 8 corners of a trilinear sample; every
// other bin interpolates to exactly 0 (mixes of zeros), so samplers evaluate only these.
__device__ __forceinline__ unsigned tri_bins(const uint32_t* __restrict__ hm, const Tri& t) {
    const uint32_t* q = hm + t.i000;
    return q[0] | q[t.dz] | q[t.dy] | q[t.dy + t.dz] | q[t.dx] | q[t.dx + t.dz] | q[t.dx + t.dy] |
           q[t.dx + t.dy + t.dz];
}

// The 32 trilinear histogram values at a sample (utils.cu:144-170).
// Returns the bins that may be nonzero (the others are 0 in p).
__device__ __forceinline__ unsigned tri_hist(const VolGeom& g, const VolBufs& b, const Tri& tr, float* p) {
    const unsigned bins = tri_bins(b.hmask, tr);
#pragma unroll
    for (int k = 0; k < kMaxObjects; ++k) p[k] = ((bins >> k) & 1u) ? tri_eval(b.hist + (uint64_t)k * g.nvox, tr) : 0.0f;
    return bins;
}

template <bool SH = true>
__device__ __forceinline__ float sample_sdf(const VolGeom& g, const float* sdf, float px, float py, float pz) {
    return tri_eval(sdf, tri_setup<SH>(g, px, py, pz));
}

// Slab test of the march (tsdf.cu:90-100): returns false when the ray misses the volume,
// else the first sample position and the (exclusive) end of the march.
__device__ __forceinline__ bool ray_bounds(const VolGeom& g, float ox, float oy, float oz, float dx, float dy,
                                           float dz, float* t0, float* t1) {
    const float idx_ = 1.0f / dx, idy = 1.0f / dy, idz = 1.0f / dz;
    const float tbx = idx_ * (g.start[0] - ox), tby = idy * (g.start[1] - oy), tbz = idz * (g.start[2] - oz);
    const float ttx = idx_ * (g.end[0] - ox), tty = idy * (g.end[1] - oy), ttz = idz * (g.end[2] - oz);
    float tnear = fmaxf(fmaxf(fminf(ttx, tbx), fminf(tty, tby)), fminf(ttz, tbz));
    tnear = fmaxf(tnear, 0.01f);
    float tfar = fminf(fminf(fmaxf(ttx, tbx), fmaxf(tty, tby)), fmaxf(ttz, tbz));
    tfar = fminf(tfar, 100.0f);
    if (tnear > tfar) return false;
    *t0 = tnear + 1e-6f;
    *t1 = tfar - 1e-6f;
    return true;
}

// Skip threshold: a trilinear sample whose 8 corners are all >= m is >= m (1 - 2^-21) in
// f32 (three levels of mix), so corners >= thr = (voxel/2)(1 + 2^-16) guarantee a sample
// >= voxel/2: no event of the march (no hit, no step switch).  Skipped samples are not
// evaluated; t still advances by the same additions, so the result is unchanged.
__device__ __forceinline__ float skip_threshold(const VolGeom& g) { return g.voxel[0] / 2.0f * (1.0f + 0x1p-16f); }

// Sample evaluator with the brick map: returns false (and no value) when the sample's
// brick is known to hold only values >= thr.  Caches the last brick looked up.
struct SkipCursor {
    int brick = -1;      // brick of the last lookup, or -2 - s while super-brick s is skipped
    bool skip = false;
    int sb = -1;         // super-brick of the last lookup
    bool sskip = false;
    float lo[3], hi[3];  // approximate voxel-coordinate box surely inside the skippable (super-)brick
};

// Approximate voxel coordinates of a ray point (|error| ~1e-4 voxel; only used to prove
// that a sample lies well inside a brick already known to be skippable).
struct RayVox {
    float k[3], c[3], rk[3];  // rk = 1 / k (the exit parameter is approximate anyway)
};

__device__ __forceinline__ RayVox ray_vox(const VolGeom& g, float ox, float oy, float oz, float dx, float dy,
                                          float dz) {
    RayVox r;
    r.k[0] = dx * g.rvox[0]; r.k[1] = dy * g.rvox[1]; r.k[2] = dz * g.rvox[2];
    r.c[0] = (ox - g.start[0]) * g.rvox[0];
    r.c[1] = (oy - g.start[1]) * g.rvox[1];
    r.c[2] = (oz - g.start[2]) * g.rvox[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) r.rk[i] = 1.0f / r.k[i];
    return r;
}

// Ray parameter where the ray leaves the cursor's box (computed with the same approximate
// voxel coordinates; samples before it are inside the box, which is itself a margin inside
// the skippable brick).
__device__ __forceinline__ float skip_box_exit(const SkipCursor& cur, const RayVox& rv) {
    float te = 3.0e38f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float k = rv.k[i];
        const float bound = k > 0.0f ? cur.hi[i] : cur.lo[i];
        const float ti = (bound - rv.c[i]) * rv.rk[i];  // k == 0: +-inf or NaN, ignored below
        te = (k != 0.0f && ti < te) ? ti : te;
    }
    return te * (1.0f - 0x1p-16f);
}

// t += step repeated while t < tend, as the march's single additions would do it, in O(1)
// per binade of t: inside a binade [2^e, 2^(e+1)) every t is a multiple of its ulp, so
// RN(t + step) = t + d with the same d = RN_ulp(step) for every t there (unless step is an
// exact tie between two multiples of the ulp, which takes single steps), and t + n d is
// exact while it stays below 2^(e+1).  The addition that crosses into the next binade is
// done singly.  On return t >= tend (or t is unchanged when it already was) and t_prev is
// the value before the last addition.
__device__ __forceinline__ void skip_steps(float& t, float& t_prev, float step, float tend) {
    while (t < tend) {
        const float t1 = t + step;
        if (!(t1 < tend)) {  // one more sample ends the run
            t_prev = t;
            t = t1;
            break;
        }
        const int eb = __float_as_int(t) & 0x7F800000;
        const float ulp = __int_as_float(eb - (23 << 23)), top = __int_as_float(eb + (1 << 23));
        const float d = t1 - t;  // exact (t1 within a factor 2 of t)
        const float lim = fminf(tend, top);
        int n = 0;
        if (fabsf(step - d) * 2.0f != ulp && t1 < top) {
            n = (int)((lim - t) * __builtin_amdgcn_rcpf(d));  // estimate, fixed up exactly below
            n = max(n, 1);
            while (n > 1 && !(t + (float)n * d < lim)) --n;
            while (t + (float)(n + 1) * d < lim) ++n;
        }
        if (n <= 1) {  // a tie, or the next addition leaves the binade: single step
            t_prev = t;
            t = t1;
            continue;
        }
        t_prev = t + (float)(n - 1) * d;
        t = t + (float)n * d;
    }
}

__device__ __forceinline__ bool in_skip_box(const SkipCursor& cur, const RayVox& rv, float t) {
    const float ax = fmaf(t, rv.k[0], rv.c[0]), ay = fmaf(t, rv.k[1], rv.c[1]), az = fmaf(t, rv.k[2], rv.c[2]);
    return (ax > cur.lo[0]) & (ax < cur.hi[0]) & (ay > cur.lo[1]) & (ay < cur.hi[1]) & (az > cur.lo[2]) &
           (az < cur.hi[2]);
}

// Evaluates the sample at p unless the brick map proves it >= voxel/2 (returns false).
// Caches the last brick looked up and, with `box`, the conservative voxel-coordinate box
// of a skippable brick for in_skip_box.
__device__ __forceinline__ void skip_box(const VolGeom& g, SkipCursor& cur, int x0, int y0, int z0, int n, bool lx,
                                         bool hx, bool ly, bool hy, bool lz, bool hz) {
    // (super-)brick bounds in voxel coordinates, shrunk by a margin far above the
    // approximation error of RayVox; the outer faces of the volume extend to infinity
    // (samples there clamp into the edge brick)
    const float m = 0.01f;
    cur.lo[0] = lx ? -1e30f : (float)x0 + m;
    cur.hi[0] = hx ? 1e30f : (float)(x0 + n) - m;
    cur.lo[1] = ly ? -1e30f : (float)y0 + m;
    cur.hi[1] = hy ? 1e30f : (float)(y0 + n) - m;
    cur.lo[2] = lz ? -1e30f : (float)z0 + m;
    cur.hi[2] = hz ? 1e30f : (float)(z0 + n) - m;
}

// OCT: the volume has its octant distance maps (a single volume's marches, known on the
// host), so the other map modes are not compiled in.
template <bool SH = true, bool OCT = false>
__device__ __forceinline__ bool sample_or_skip(const VolGeom& g, const VolBufs& b, float thr, SkipCursor& cur,
                                               float px, float py, float pz, float* f, bool box = false,
                                               int oct = -1) {
    const TriCoord c = tri_coord<SH>(g, px, py, pz);
    if (OCT || (SEMTSDF_BRICK_DIST && box && b.bdist)) {
        // the brick's distance r to the nearest non-skippable brick of the ray's octant: the
        // r^3 bricks from it on towards the ray's direction are skippable, one box for the
        // march to step through (without an octant: the (2r-1)^3 bricks around it)
        const int br = brick_of(g, c);
        if (br != cur.brick) {
            cur.brick = br;
            const int r = (OCT || oct >= 0) ? (int)reinterpret_cast<const uint8_t*>(b.boct)[(size_t)br * 8 + oct]
                                            : b.bdist[br];
            cur.skip = r > 0;
            if (cur.skip) {
                const int bx = c.xc >> 3, by = c.yc >> 3, bz = c.zl >> 3;
                const int nx = oct < 0 || (oct & 1), ny = oct < 0 || (oct & 2), nz = oct < 0 || (oct & 4);
                const int px_ = oct < 0 || !(oct & 1), py_ = oct < 0 || !(oct & 2), pz_ = oct < 0 || !(oct & 4);
                const int x0 = bx - (nx ? r - 1 : 0), y0 = by - (ny ? r - 1 : 0), z0 = bz - (nz ? r - 1 : 0);
                const int x1 = bx + (px_ ? r : 1), y1 = by + (py_ ? r : 1), z1 = bz + (pz_ ? r : 1);  // exclusive
                const float m = 0.01f;
                cur.lo[0] = x0 <= 0 ? -1e30f : (float)(x0 * 8) + m;
                cur.hi[0] = x1 >= g.nbx ? 1e30f : (float)(x1 * 8) - m;
                cur.lo[1] = y0 <= 0 ? -1e30f : (float)(y0 * 8) + m;
                cur.hi[1] = y1 >= g.nby ? 1e30f : (float)(y1 * 8) - m;
                cur.lo[2] = z0 <= 0 ? -1e30f : (float)(z0 * 8) + m;
                cur.hi[2] = z1 >= g.nbz ? 1e30f : (float)(z1 * 8) - m;
            }
        }
        if (cur.skip) return false;
        *f = tri_eval(b.sdf, tri_from(g, c));
        return true;
    }
    if (b.bmin) {
        if (box && b.sbmin) {  // super-brick level first: one lookup per 64^3 voxels of free space
            const int sx = c.xc >> 6, sy = c.yc >> 6, sz = c.zl >> 6;
            const int sb = (int)__umul24(__umul24((unsigned)sx, (unsigned)g.nsy) + (unsigned)sy, (unsigned)g.nsz) + sz;
            if (sb != cur.sb) {
                cur.sb = sb;
                cur.sskip = b.sbmin[sb] >= thr;
            }
            if (cur.sskip) {
                if (cur.brick != -2 - sb) {
                    cur.brick = -2 - sb;
                    cur.skip = true;
                    skip_box(g, cur, sx * 64, sy * 64, sz * 64, 64, sx == 0, sx == g.nsx - 1, sy == 0, sy == g.nsy - 1,
                             sz == 0, sz == g.nsz - 1);
                }
                return false;
            }
        }
        const int br = brick_of(g, c);
        if (br != cur.brick) {
            cur.brick = br;
            cur.skip = b.bmin[br] >= thr;
            if (cur.skip && box) {
                const int bx = c.xc >> 3, by = c.yc >> 3, bz = c.zl >> 3;
                skip_box(g, cur, bx * 8, by * 8, bz * 8, 8, bx == 0, bx == g.nbx - 1, by == 0, by == g.nby - 1,
                         bz == 0, bz == g.nbz - 1);
            }
        }
        if (cur.skip) return false;
    }
    *f = tri_eval(b.sdf, tri_from(g, c));
    return true;
}

// The shared ray march of back_proj_kernel (tsdf.cu:90-124) and show_tsdf_kernel
// (viewer.cu:223-257).  Returns true on a hit and the refined t.
struct MarchStats {
    unsigned iters = 0, lookups = 0, evals = 0, skipped = 0;
};

#ifndef SEMTSDF_MARCH_SPEC
#define SEMTSDF_MARCH_SPEC 5
#endif
constexpr int kMarchSpec = SEMTSDF_MARCH_SPEC;  // speculative samples per evaluated sample
#ifndef SEMTSDF_MARCH_PRIO
#define SEMTSDF_MARCH_PRIO 0u  // iterations after which a marching wave's priority rises (0: off; 8-20 measured 0.5-1.5 % slower, profiles/r04/ab_march_priority.txt)
#endif

template <bool OCT>
__device__ bool march_ray(const VolGeom& g, const VolBufs& b, float ox, float oy, float oz, float dx, float dy,
                          float dz, float* t_hit, MarchStats* st = nullptr) {
    float t, tfar;
    if (!ray_bounds(g, ox, oy, oz, dx, dy, dz, &t, &tfar)) return false;
    const float vx = g.voxel[0];
    const float thr = skip_threshold(g);
    SkipCursor cur;
    const RayVox rv = ray_vox(g, ox, oy, oz, dx, dy, dz);
    const bool box = OCT || b.bmin != nullptr;  // single-volume marches only (the host rejects sharded handles)
    const int oct = OCT || (SEMTSDF_BRICK_OCT && b.boct) ? (dx < 0.0f ? 1 : 0) | (dy < 0.0f ? 2 : 0) | (dz < 0.0f ? 4 : 0)
                                                         : -1;
    float f_t = 1.0f, f_tt = 0.0f;
    bool prev_skipped = false;  // f_t not evaluated: re-evaluate it at t_prev if needed
    float t_prev = t;
    {
        float f;
        if (sample_or_skip<false, OCT>(g, b, thr, cur, fmaf(t, dx, ox), fmaf(t, dy, oy), fmaf(t, dz, oz), &f, box, oct)) {
            if (!(f > 0.0f)) return false;
            f_t = f;
        } else {
            prev_skipped = true;
        }
    }
    float step = vx;
    // One memory access (a brick lookup or a sample) per iteration; in between, each lane
    // runs through the samples of its current skippable brick with arithmetic only, so the
    // lanes of a wave do not wait for each other's memory round trips sample by sample.
    unsigned iters = 0;
    while (t < tfar) {
        if (st) st->iters++;
        // a wave still marching after many iterations holds the kernel's tail: raise its
        // issue priority (age arbitration would otherwise favour the older, shorter waves)
        if (SEMTSDF_MARCH_PRIO) {
            const unsigned wi = __builtin_amdgcn_readfirstlane(++iters);
            if (wi == SEMTSDF_MARCH_PRIO) __builtin_amdgcn_s_setprio(1);
            else if (wi == 2u * SEMTSDF_MARCH_PRIO) __builtin_amdgcn_s_setprio(2);
            else if (wi == 4u * SEMTSDF_MARCH_PRIO) __builtin_amdgcn_s_setprio(3);
        }
        if (box && cur.skip && in_skip_box(cur, rv, t)) {
            // the same additions as sample-by-sample stepping (the hit position depends on
            // them), tested against the box's exit parameter, then exactly near the exit
            const float tend = fminf(tfar, skip_box_exit(cur, rv));
            skip_steps(t, t_prev, step, tend);
            while (t < tfar && in_skip_box(cur, rv, t)) {
                t_prev = t;
                t += step;
                if (st) st->skipped++;
            }
            prev_skipped = true;  // those samples are >= voxel/2: no hit, no step switch
            f_tt = 1.0f;
            if (!(t < tfar)) break;
        }
        float f;
        const int brick_before = cur.brick;
        const bool evaluated =
            sample_or_skip<false, OCT>(g, b, thr, cur, fmaf(t, dx, ox), fmaf(t, dy, oy), fmaf(t, dz, oz), &f, box, oct);
        if (st) {
            st->lookups += cur.brick != brick_before;
            st->evals += evaluated;
        }
        if (!evaluated) {
            prev_skipped = true;
            t_prev = t;
            f_tt = 1.0f;
            t += step;
            continue;
        }
        f_tt = f;
        if (f_tt < 0.0f) break;
        f_t = f_tt;
        prev_skipped = false;
        if (f_tt < vx / 2.0f && step != vx / 4.0f) {  // sticky quarter step (switches once)
            step = vx / 4.0f;
            t += step;
            continue;
        }
        t += step;
        if (kMarchSpec > 0) {
            // An evaluated sample means the ray is near a surface: evaluate the next
            // kMarchSpec samples of the same step in one round trip (no map lookups: a sample
            // the map would skip evaluates to >= voxel/2, which is no event either), then
            // run the march logic over them in order; a step switch or a hit ends the batch.
            float fs[kMarchSpec > 0 ? kMarchSpec : 1];
            float tn = t;
#pragma unroll
            for (int j = 0; j < kMarchSpec; ++j) {
                fs[j] = sample_sdf<false>(g, b.sdf, fmaf(tn, dx, ox), fmaf(tn, dy, oy), fmaf(tn, dz, oz));
                tn += step;
            }
            if (st) st->evals += kMarchSpec;
            bool hit = false;
#pragma unroll
            for (int j = 0; j < kMarchSpec; ++j) {
                if (!(t < tfar)) break;
                f_tt = fs[j];
                if (f_tt < 0.0f) {
                    hit = true;
                    break;
                }
                f_t = f_tt;
                if (f_tt < vx / 2.0f && step != vx / 4.0f) {  // the step switches: the rest is stale
                    step = vx / 4.0f;
                    t += step;
                    break;
                }
                t += step;
            }
            if (hit) break;
        }
    }
    if (!(f_tt < 0.0f)) return false;
    if (prev_skipped) f_t = sample_sdf<false>(g, b.sdf, fmaf(t_prev, dx, ox), fmaf(t_prev, dy, oy), fmaf(t_prev, dz, oz));
    t += step * f_tt / (f_t - f_tt);
    *t_hit = t;
    return true;
}

__device__ __forceinline__ void ray_assoc(const MarchCamera& c, int x, int y, float* ox, float* oy, float* oz,
                                          float* dx, float* dy, float* dz) {
    const float fx = (float)x, fy = (float)y;
    const float tx = dot3(c.Kinv[0], c.Kinv[1], c.Kinv[2], fx, fy, 1.0f);
    const float ty = dot3(c.Kinv[3], c.Kinv[4], c.Kinv[5], fx, fy, 1.0f);
    const float tz = dot3(c.Kinv[6], c.Kinv[7], c.Kinv[8], fx, fy, 1.0f);
    const float rx = dot3(c.Rt[0], c.Rt[1], c.Rt[2], tx, ty, tz);
    const float ry = dot3(c.Rt[3], c.Rt[4], c.Rt[5], tx, ty, tz);
    const float rz = dot3(c.Rt[6], c.Rt[7], c.Rt[8], tx, ty, tz);
    const float inv = 1.0f / sqrtf(dot3(rx, ry, rz, rx, ry, rz));
    *dx = rx * inv; *dy = ry * inv; *dz = rz * inv;
    *ox = c.o[0]; *oy = c.o[1]; *oz = c.o[2];
}

__device__ __forceinline__ void ray_render(const MarchCamera& c, int x, int y, float* ox, float* oy, float* oz,
                                           float* dx, float* dy, float* dz) {
    const float fx = (float)x, fy = (float)y;
    const float tx = dot3(c.s2w[0], c.s2w[1], c.s2w[2], fx, fy, 1.0f) + c.s2w[3];
    const float ty = dot3(c.s2w[4], c.s2w[5], c.s2w[6], fx, fy, 1.0f) + c.s2w[7];
    const float tz = dot3(c.s2w[8], c.s2w[9], c.s2w[10], fx, fy, 1.0f) + c.s2w[11];
    const float rx = tx - c.o[0], ry = ty - c.o[1], rz = tz - c.o[2];
    const float inv = 1.0f / sqrtf(dot3(rx, ry, rz, rx, ry, rz));
    *dx = rx * inv; *dy = ry * inv; *dz = rz * inv;
    *ox = c.o[0]; *oy = c.o[1]; *oz = c.o[2];
}

// ------------------------------------------------------------------------------------
// mask statistics: max label and first pixel of every label (for the relabel order of
// tsdf.cu:371-389 and num_objs of tsdf.cu:463-468)
// ------------------------------------------------------------------------------------
// Block `blk` of `nblk` of the frame's mask statistics (k_mask_stats, and the mask-statistics
// blocks of k_march_fused).
__device__ __forceinline__ void mask_stats_block(const uint8_t* __restrict__ mask, int npx, AssocTables* t, int blk,
                                                 int nblk) {
    __shared__ unsigned s_first[256];
    __shared__ unsigned s_max;
    for (int k = threadIdx.x; k < 256; k += 256) s_first[k] = 0xFFFFFFFFu;
    if (threadIdx.x == 0) s_max = 0;
    __syncthreads();
    unsigned mx = 0;
    for (int i = blk * 256 + (int)threadIdx.x; i < npx; i += nblk * 256) {
        const unsigned m = mask[i];
        mx = max(mx, m);
        if (m) atomicMin(&s_first[m], (unsigned)i);
    }
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, off, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(&s_max, mx);
    __syncthreads();
    for (int k = threadIdx.x; k < 256; k += 256)
        if (s_first[k] != 0xFFFFFFFFu) atomicMin(&t->first_px[k], s_first[k]);
    if (threadIdx.x == 0) atomicMax(&t->max_label, s_max);
}

// Association tables before a frame: sums and counts 0, first_px UINT_MAX (one launch in
// place of two fills).
__global__ __launch_bounds__(256) void k_tables_init(AssocTables* t) {
    uint2* w = reinterpret_cast<uint2*>(t);
    for (unsigned i = threadIdx.x; i < sizeof(AssocTables) / 8; i += 256) w[i] = make_uint2(0u, 0u);
    __syncthreads();
    t->first_px[threadIdx.x] = 0xFFFFFFFFu;
}

hipError_t launch_tables_init(AssocTables* t, hipStream_t s) {
    hipLaunchKernelGGL(k_tables_init, dim3(1), dim3(256), 0, s, t);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_mask_stats(const uint8_t* __restrict__ mask, int npx, AssocTables* t) {
    mask_stats_block(mask, npx, t, (int)blockIdx.x, (int)gridDim.x);
}

hipError_t launch_mask_stats(const uint8_t* mask, int npx, AssocTables* t, hipStream_t s) {
    int blocks = (npx + 255) / 256;
    if (blocks > 256) blocks = 256;
    hipLaunchKernelGGL(k_mask_stats, dim3(blocks), dim3(256), 0, s, mask, npx, t);
    return hipGetLastError();
}

__global__ void k_first_frame_objs(const AssocTables* t, int* num_objs) {
    if (threadIdx.x == 0) *num_objs = (int)t->max_label + 1;
}

hipError_t launch_first_frame_objs(const AssocTables* t, int* num_objs_dev, hipStream_t s) {
    hipLaunchKernelGGL(k_first_frame_objs, dim3(1), dim3(64), 0, s, t, num_objs_dev);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// association: ray march + trilinear histogram + fused 32x32 log-likelihood accumulation
// (back_proj_kernel tsdf.cu:72-135 feeding filter_overlaps tsdf.cu:312-334).
//   A[m][j] = T1[m][j] + T2[j] - T3[m][j],  C[m][j] = C1[m] + C2[j] - C3[m][j]
// is the same sum as the reference's per-pixel loops; terms are accumulated in 2^-28
// fixed point with integer atomics, so the totals do not depend on execution order.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ long long to_fix(float L) {
    return (long long)rint((double)L * kFixScale);
}

// A positive t1 term (p / n_obs > 1: a trilinear count rounded above n_obs, or uploaded / given
// probabilities above it) as AssocTables::pos_max records it: its fixed-point value, at least 1,
// saturating at 2^32 - 1.  The decision's certificate widens its bounds by the positive terms
// (prob_interval) and sends every row to the exact path when they leave the validated range.
__device__ __forceinline__ unsigned pos_fix(float L) {
    return (unsigned)min(max(to_fix(L), 1ll), 0xFFFFFFFFll);
}

// Workgroup-local (LDS) copy of the accumulated sums of AssocTables.
struct AssocLds {
    long long t1[kMaxObjects][kMaxObjects];
    long long t3[kMaxObjects][kMaxObjects];
    long long t2[kMaxObjects];
    unsigned c1[kMaxObjects];
    unsigned c2[kMaxObjects];
    unsigned c3[kMaxObjects][kMaxObjects];
    unsigned pos;  // max positive t1 term of the workgroup (pos_fix), 0: none
};

__device__ __forceinline__ void assoc_lds_clear(AssocLds& s) {
    if (threadIdx.x == 0) s.pos = 0u;
    for (int k = threadIdx.x; k < kMaxObjects * kMaxObjects; k += blockDim.x) {
        (&s.t1[0][0])[k] = 0;
        (&s.t3[0][0])[k] = 0;
        (&s.c3[0][0])[k] = 0;
    }
    if (threadIdx.x < kMaxObjects) { s.t2[threadIdx.x] = 0; s.c1[threadIdx.x] = 0; s.c2[threadIdx.x] = 0; }
}

// One pixel's terms of filter_overlaps (tsdf.cu:312-334): p = trilinear histogram at the
// hit (zeros without a hit), m = the pixel's current label.
__device__ __forceinline__ void assoc_accumulate(AssocLds& s, const float* p, unsigned m, float n_obs, float eps,
                                                 float box_thresh) {
    if (m > 0 && m < (unsigned)kMaxObjects) {
        atomicAdd(&s.c1[m], 1u);
#pragma unroll
        for (int j = 1; j < kMaxObjects; ++j) {
            const float L = logf(fmaxf(p[j] / n_obs, eps));
            atomicAdd(reinterpret_cast<unsigned long long*>(&s.t1[m][j]), (unsigned long long)to_fix(L));
            if (L > 0.0f) atomicMax(&s.pos, pos_fix(L));  // rare: p > n_obs
        }
    }
#pragma unroll
    for (int n = 1; n < kMaxObjects; ++n) {
        if (p[n] > box_thresh) {
            const float L = logf(fmaxf(1.0f - p[n] / n_obs, eps));
            const unsigned long long f = (unsigned long long)to_fix(L);
            atomicAdd(reinterpret_cast<unsigned long long*>(&s.t2[n]), f);
            atomicAdd(&s.c2[n], 1u);
            if (m > 0 && m < (unsigned)kMaxObjects) {
                atomicAdd(reinterpret_cast<unsigned long long*>(&s.t3[m][n]), f);
                atomicAdd(&s.c3[m][n], 1u);
            }
        }
    }
}

// The same sums with the bins the sampler found empty folded in: a bin with p[j] == 0 adds
// F0 = to_fix(logf(eps)) to t1[m][j] (p/n_obs = 0 < eps), so every pixel of label m adds F0
// to the whole row and the per-pixel work is the few present bins (their to_fix(L) - F0).
// The row baseline c1[m] * F0 is added when the workgroup flushes its tables; the integer
// sums are identical.  Requires box_thresh >= 0 (an empty bin is never in the box).
// px (optional): the pixel's data for the decision's exact path (AssocPixels), written in the
// same loop: present bins (p != 0) and their counts, box bins (p > box_thresh >= 0 needs p != 0).
__device__ __forceinline__ void assoc_accumulate_sparse(AssocLds& s, const float* p, unsigned bins, unsigned m,
                                                        float n_obs, float eps, float box_thresh, long long F0,
                                                        const AssocPixels& px, int npx, int k) {
    const bool lab = m > 0 && m < (unsigned)kMaxObjects;
    if (lab) atomicAdd(&s.c1[m], 1u);
    unsigned box = 0u;  // bins becomes the present bins (p != 0) as the loop goes
    bins &= ~1u;
#pragma unroll
    for (int j = 1; j < kMaxObjects; ++j) {
        if (!((bins >> j) & 1u)) continue;
        if (p[j] == 0.0f) {
            bins &= ~(1u << j);
            continue;
        }
        if (px.bits) px.p[(size_t)j * npx + k] = p[j];
        if (lab) {
            const float L1 = logf(fmaxf(p[j] / n_obs, eps));
            const long long d = to_fix(L1) - F0;
            if (d) atomicAdd(reinterpret_cast<unsigned long long*>(&s.t1[m][j]), (unsigned long long)d);
            if (L1 > 0.0f) atomicMax(&s.pos, pos_fix(L1));  // rare: p > n_obs
        }
        if (p[j] > box_thresh) {
            const float L = logf(fmaxf(1.0f - p[j] / n_obs, eps));
            const unsigned long long f = (unsigned long long)to_fix(L);
            atomicAdd(reinterpret_cast<unsigned long long*>(&s.t2[j]), f);
            atomicAdd(&s.c2[j], 1u);
            box |= 1u << j;
            if (lab) {
                atomicAdd(reinterpret_cast<unsigned long long*>(&s.t3[m][j]), f);
                atomicAdd(&s.c3[m][j], 1u);
            }
        }
    }
    if (px.bits) px.bits[k] = make_uint2(bins, box);
}

// The pixel's data for the decision's exact path (AssocPixels): present and box bins, and the
// counts of the present bins.  bins: the bins that may be nonzero (tri_hist).
__device__ __forceinline__ void assoc_pixel_out(const AssocPixels& px, int npx, int k, const float* p, unsigned bins,
                                                float box_thresh) {
    unsigned pres = 0, box = 0;
#pragma unroll
    for (int j = 1; j < kMaxObjects; ++j) {
        if (((bins >> j) & 1u) && p[j] != 0.0f) {
            pres |= 1u << j;
            px.p[(size_t)j * npx + k] = p[j];
        }
        if (p[j] > box_thresh) box |= 1u << j;
    }
    px.bits[k] = make_uint2(pres, box);
}

#ifndef SEMTSDF_MARCH_WPE
#define SEMTSDF_MARCH_WPE 1  // no occupancy request (register-limited: 3 waves per SIMD)
#endif

// The single-volume marches take the octant-map specialisation when the volume has the maps.
inline bool oct_maps(const VolBufs& b) {
    return SEMTSDF_BRICK_DIST && SEMTSDF_BRICK_OCT && b.bmin && b.bdist && b.boct;
}

// One 16x16-pixel tile (bx, by) of the association march, a whole workgroup.
template <bool OCT>
__device__ __forceinline__ void assoc_tile(const AssocArgs& a, AssocLds& s, int bx, int by) {
    const int tid = threadIdx.x;
    assoc_lds_clear(s);
    __syncthreads();
    const bool sparse = a.box_thresh >= 0.0f && !a.probs_out;  // see assoc_accumulate_sparse
    const long long F0 = to_fix(logf(fmaxf(0.0f, a.eps)));      // an empty bin's term

    const int x = bx * 16 + (tid & 15);
    const int y = by * 16 + (tid >> 4);
    if (x < a.width && y < a.height) {
        float ox, oy, oz, dx, dy, dz, t;
        ray_assoc(a.cam, x, y, &ox, &oy, &oz, &dx, &dy, &dz);
        float p[kMaxObjects];
#pragma unroll
        for (int k = 0; k < kMaxObjects; ++k) p[k] = 0.0f;
        unsigned bins = 0;
        if (a.debug != 2 && march_ray<OCT>(a.g, a.b, ox, oy, oz, dx, dy, dz, &t)) {
            const Tri tr = tri_setup<false>(a.g, fmaf(t, dx, ox), fmaf(t, dy, oy), fmaf(t, dz, oz));
            bins = tri_hist(a.g, a.b, tr, p);
        }
        const int px = y * a.width + x;
        if (a.px.bits && !sparse) assoc_pixel_out(a.px, a.width * a.height, px, p, bins, a.box_thresh);
        if (a.probs_out) {
#pragma unroll
            for (int k = 0; k < kMaxObjects; ++k) {
                a.probs_out[(size_t)px * kMaxObjects + k] = p[k];
                a.box_out[(size_t)px * kMaxObjects + k] = p[k] > a.box_thresh ? 1 : 0;
            }
        }
        if (a.debug != 1) {
            if (sparse)
                assoc_accumulate_sparse(s, p, bins, a.mask[px], a.n_obs, a.eps, a.box_thresh, F0, a.px,
                                        a.width * a.height, px);
            else
                assoc_accumulate(s, p, a.mask[px], a.n_obs, a.eps, a.box_thresh);
        }
    }
    __syncthreads();
    AssocTables* T = a.tables;
    for (int k = tid; k < kMaxObjects * kMaxObjects; k += 256) {
        const int m = k / kMaxObjects, j = k % kMaxObjects;
        const long long v1 = (&s.t1[0][0])[k] + ((sparse && m >= 1 && j >= 1) ? (long long)s.c1[m] * F0 : 0ll);
        if (v1) atomicAdd(reinterpret_cast<unsigned long long*>(&T->t1[0][0]) + k, (unsigned long long)v1);
        const long long v3 = (&s.t3[0][0])[k];
        if (v3) atomicAdd(reinterpret_cast<unsigned long long*>(&T->t3[0][0]) + k, (unsigned long long)v3);
        const unsigned c3 = (&s.c3[0][0])[k];
        if (c3) atomicAdd(&T->c3[0][0] + k, c3);
    }
    if (tid < kMaxObjects) {
        if (s.t2[tid]) atomicAdd(reinterpret_cast<unsigned long long*>(&T->t2[tid]), (unsigned long long)s.t2[tid]);
        if (s.c1[tid]) atomicAdd(&T->c1[tid], s.c1[tid]);
        if (s.c2[tid]) atomicAdd(&T->c2[tid], s.c2[tid]);
    }
    if (tid == 0 && s.pos) atomicMax(&T->pos_max, s.pos);
}

template <bool OCT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEMTSDF_MARCH_WPE))) void k_assoc_march(AssocArgs a) {
    __shared__ AssocLds s;
    assoc_tile<OCT>(a, s, (int)blockIdx.x, (int)blockIdx.y);
}

hipError_t launch_assoc_march(const AssocArgs& a, hipStream_t s) {
    const dim3 grid((a.width + 15) / 16, (a.height + 15) / 16);
    if (oct_maps(a.b))
        hipLaunchKernelGGL(k_assoc_march<true>, grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_assoc_march<false>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Decision (tsdf.cu:337-389) with the reference's f32 arithmetic by construction.
//
// The reference sums its f32 log terms in pixel order (tsdf.cu:312-334), divides by the
// count and takes expf (tsdf.cu:343); the decision compares those f32 values with strict
// '>' (argmax, first maximum wins; acceptance against 3 * prior) and strict '<' (the greedy
// keep-the-best per previous id).  The march's fixed-point sums S_fix are exact sums of the
// same f32 terms up to 2^-29 per term, so every f32 value the reference forms lies in an
// interval around them:
//   |A_f32 - S| <= gamma |S|,  gamma = (n-1) u / (1 - (n-1) u),  u = 2^-24   (recursive
//   summation of n same-sign terms: every partial sum is at most |A_f32|), |S - S_fix| <= n 2^-29,
//   q = RN(A_f32 / n) within 2^-24 relative, expf within 0.502 ulp (< 2^-23 relative).
// A row whose argmax, acceptance and greedy outcome are the same for every value in those
// intervals is decided from the fixed-point sums; every other row ("flagged") is decided from
// its exact f32 sums, recomputed from the per-pixel data in reference pixel order
// (exact_row_sum: the sequential f32 additions evaluated as integer prefix sums per binade of
// the running sum, bit-identical to the sequential loop) and the glibc expf restatement.
//
// One launch of 32 workgroups: each certifies the whole table (the same computation in
// every workgroup), workgroup j >= 1 computes column j of the flagged rows, and the last
// workgroup to finish (device-scope counter) decides, relabels the tables for the next frame
// and resets the counter.  Unmatched labels get new ids in the order of their first pixel
// (tsdf.cu:378-387) by ranking first_px.
// ------------------------------------------------------------------------------------
constexpr int kScanPer = 8;                    // pixels per lane of one scan chunk
constexpr int kScanChunk = 256 * kScanPer;     // pixels per chunk (one workgroup)

struct ScanLds {
    long long wsum[4];
    int wmin[4];
    int first;
    long long before;
    float xv;
};

// workgroup exclusive scan of one int64 per lane (4 waves); returns the lane's exclusive
// prefix and the total in *tot
__device__ __forceinline__ long long wg_exscan(long long v, ScanLds& L, long long* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    long long inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long o = __shfl_up(inc, off, 64);
        if (lane >= off) inc += o;
    }
    if (lane == 63) L.wsum[w] = inc;
    __syncthreads();
    long long base = 0, all = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < w) base += L.wsum[k];
        all += L.wsum[k];
    }
    __syncthreads();
    *tot = all;
    return base + inc - v;
}

__device__ __forceinline__ int wg_min(int v, ScanLds& L) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    if (lane == 0) L.wmin[w] = v;
    __syncthreads();
    const int r = min(min(L.wmin[0], L.wmin[1]), min(L.wmin[2], L.wmin[3]));
    __syncthreads();
    return r;
}

// One chunk of the reference's sequential f32 additions s <- RN(s + x) (tsdf.cu:318,329) for one
// row: x[e] are the chunk's terms of this lane (pixel base + 8 tid + e, 0 = no term).  While s
// stays in one binade [2^e, 2^(e+1)) (all terms <= 0, |s| grows), its grid is the multiples of
// u = 2^(e-23) and RN(s + x) = s + round_u(x) exactly, so the chunk's steps are an integer prefix
// sum of round_u(x) / u (a workgroup scan).  A step that would reach the next binade, a tie (x an
// odd multiple of u/2, where the parity of s decides), a positive term, s == 0 or a subnormal s
// is taken as the f32 addition itself, and the chunk resumes after it with the new binade.
// Returns the new s (workgroup-uniform).
__device__ float scan_chunk(float s, const float* x, ScanLds& L) {
    const int tid = threadIdx.x;
    int pos = 0;  // chunk elements before pos are done
    for (;;) {
        const unsigned sb = glibc::f2u(s);
        if (s == 0.0f || (sb >> 31) == 0u || ((sb >> 23) & 0xFFu) == 0u) {
            // s == 0 (the first nonzero term is the sum), s > 0 or subnormal (not reached by
            // same-sign terms of the association): one addition at a time
            int f = kScanChunk;
#pragma unroll
            for (int e = 0; e < kScanPer; ++e) {
                const int idx = tid * kScanPer + e;
                if (idx >= pos && x[e] != 0.0f && idx < f) f = idx;
            }
            f = wg_min(f, L);
            if (f == kScanChunk) return s;
            if (f >= tid * kScanPer && f < (tid + 1) * kScanPer) {
#pragma unroll
                for (int e = 0; e < kScanPer; ++e)
                    if (tid * kScanPer + e == f) L.xv = x[e];
            }
            __syncthreads();
            s = s + L.xv;
            __syncthreads();
            pos = f + 1;
            continue;
        }
        const int uexp = (int)((sb >> 23) & 0xFFu) - 150;             // u = 2^uexp
        const long long S0 = (long long)((sb & 0x7FFFFFu) | 0x800000u);  // |s| / u
        long long r[kScanPer];
        bool viol[kScanPer];
        long long lsum = 0;
#pragma unroll
        for (int e = 0; e < kScanPer; ++e) {
            const int idx = tid * kScanPer + e;
            r[e] = 0;
            viol[e] = false;
            if (idx >= pos && x[e] != 0.0f) {
                if (x[e] > 0.0f) {
                    viol[e] = true;
                } else {
                    const double v = ldexp(-(double)x[e], -uexp);  // |x| / u, exact
                    if (v >= 0x1p25) {
                        r[e] = 1ll << 25;
                        viol[e] = true;
                    } else {
                        const double fl = floor(v), fr = v - fl;
                        r[e] = (long long)fl + (fr > 0.5 ? 1 : 0);
                        viol[e] = fr == 0.5;
                    }
                }
            }
            lsum += r[e];
        }
        long long tot;
        const long long ex = wg_exscan(lsum, L, &tot);
        int f = kScanChunk;
        long long run = ex;
#pragma unroll
        for (int e = 0; e < kScanPer; ++e) {
            const int idx = tid * kScanPer + e;
            run += r[e];
            if ((viol[e] || S0 + run >= (1ll << 24)) && idx >= pos && idx < f) f = idx;
        }
        f = wg_min(f, L);
        if (f == kScanChunk)  // the rest of the chunk stays in this binade
            return -(float)ldexp((double)(S0 + tot), uexp);
        if (f >= tid * kScanPer && f < (tid + 1) * kScanPer) {
            long long before = ex;
#pragma unroll
            for (int e = 0; e < kScanPer; ++e) {
                if (tid * kScanPer + e == f) L.xv = x[e];
                if (tid * kScanPer + e < f) before += r[e];
            }
            L.before = before;
        }
        __syncthreads();
        s = -(float)ldexp((double)(S0 + L.before), uexp);  // exact: the steps before f
        s = s + L.xv;                                        // step f as the f32 addition
        __syncthreads();
        pos = f + 1;
        if (pos >= kScanChunk) return s;
    }
}

// The reference's A[i][j] (tsdf.cu:312-334) of every flagged current label i (rows) for previous
// id j: the f32 sum, in pixel order, of logf(max(p/n, eps)) over pixels labelled i and
// logf(max(1 - p/n, eps)) over the other pixels whose box bit j is set (every pixel adds at most
// one term to an entry).  One pass over the pixels serves all rows: a chunk's per-pixel data
// (label, bits, count of bin j) is loaded once, one chunk ahead of its use, and each row scans
// the chunk with its own running sum (s_rows, LDS).
__device__ void exact_rows_sum(unsigned rows, int j, const DecideArgs& a, float c0, ScanLds& L, float* s_rows) {
    const int tid = threadIdx.x;
    const float* pj = a.px.p + (size_t)j * a.npx;
    if (tid < kMaxObjects) s_rows[tid] = 0.0f;
    __syncthreads();
    unsigned m_n[kScanPer];
    uint2 b_n[kScanPer];
    float p_n[kScanPer];
    auto load = [&](int base) {
#pragma unroll
        for (int e = 0; e < kScanPer; ++e) {
            const int k = base + tid * kScanPer + e;
            const bool in = k < a.npx;
            m_n[e] = in ? a.mask[k] : 0u;
            b_n[e] = in ? a.px.bits[k] : make_uint2(0u, 0u);
            p_n[e] = in ? pj[k] : 0.0f;  // stale unless the bin is present: masked below
        }
    };
    load(0);
    for (int base = 0; base < a.npx; base += kScanChunk) {
        unsigned m[kScanPer];
        float t1[kScanPer], t2[kScanPer];
        bool box[kScanPer];
#pragma unroll
        for (int e = 0; e < kScanPer; ++e) {
            m[e] = m_n[e];
            const bool pres = (b_n[e].x >> j) & 1u;
            box[e] = (b_n[e].y >> j) & 1u;
            const float p = pres ? p_n[e] : 0.0f;
            // t1 for the pixel's own label (a flagged row), t2 for every other row (box bit j)
            t1[e] = (m[e] < (unsigned)kMaxObjects && ((rows >> m[e]) & 1u))
                        ? (p == 0.0f ? c0 : glibc::logf(fmaxf(p / a.n_obs, a.eps)))
                        : 0.0f;
            t2[e] = box[e] ? glibc::logf(fmaxf(1.0f - p / a.n_obs, a.eps)) : 0.0f;
        }
        if (base + kScanChunk < a.npx) load(base + kScanChunk);  // the next chunk, in flight meanwhile
        for (unsigned rr = rows; rr; rr &= rr - 1u) {
            const unsigned i = (unsigned)(__ffs((int)rr) - 1);
            float x[kScanPer];
            bool any = false;
#pragma unroll
            for (int e = 0; e < kScanPer; ++e) {
                x[e] = m[e] == i ? t1[e] : t2[e];
                any |= x[e] != 0.0f;
            }
            if (!__syncthreads_or(any)) continue;
            const float s = scan_chunk(s_rows[i], x, L);
            __syncthreads();  // every lane has read s_rows[i]
            if (tid == 0) s_rows[i] = s;
            __syncthreads();
        }
    }
}

// Certified interval [lo, hi] of the reference's f32 exp(A/C) from the fixed-point sums, and
// the point estimate mid (see above).  A fixed = the 2^-28 fixed-point sum, n = count.  Each
// fixed-point term differs from the reference's glibc logf term by at most kTermSlack: half a
// unit of 2^-28 plus the device logf's distance to glibc's (<= 2 ulp over [0.05, 32],
// tests/test_gpu_assoc_exact.py; 4 ulp at |t| < 4 = 2^-20 allowed).  That needs every term in
// (-4, 4): the certificate is used only for eps >= 0.05 and terms below log 32 (kPosCap; the
// decide kernel sends every row to the exact path otherwise).
// P (>= 0): an upper bound of every positive term.  Recursive f32 summation of n terms errs by
// at most gamma * sum |x_i| = gamma (|S| + 2 sum of the positive terms) <= gamma (|S| + 2 n P);
// with P == 0 (every term <= 0) that is the same-sign bound gamma |S|.
constexpr double kTermSlack = 0x1p-29 + 0x1p-20;
constexpr unsigned kPosCap = 930326397u;  // to_fix(log 32) = 3.4657 * 2^28: terms must stay below it
__device__ __forceinline__ void prob_interval(long long A, long long n, double P, double* lo, double* hi,
                                              double* mid) {
    if (n <= 0) { *lo = *hi = *mid = 0.0; return; }
    const double dn = (double)n;
    const double S = (double)A / kFixScale;
    *mid = exp(S / dn);
    const double g = (dn - 1.0) * 0x1p-24;
    if (g >= 0.5) { *lo = 0.0; *hi = 2.0; return; }  // no certificate: the exact path decides
    const double gam = g / (1.0 - g) * (1.0 + 0x1p-40);
    // the exact sum of the reference's f32 terms lies in [slo, shi] (it is <= n P)
    const double slo = S - dn * kTermSlack * (1.0 + 0x1p-40);
    const double shi = fmin(S + dn * kTermSlack * (1.0 + 0x1p-40), dn * P);
    // its f32 pixel-order sum, then q = RN(A / n) within 2^-24 relative, then expf within 0.502 ulp
    const double alo = slo - gam * (fabs(slo) + 2.0 * dn * P);
    const double ahi = shi + gam * (fabs(shi) + 2.0 * dn * P);
    const double q0 = alo / dn, q1 = ahi / dn;
    const double qlo = q0 - fabs(q0) * (0x1p-24 + 0x1p-40) - 0x1p-60;
    const double qhi = q1 + fabs(q1) * (0x1p-24 + 0x1p-40) + 0x1p-60;
    *lo = exp(qlo) * (1.0 - 0x1p-23 - 0x1p-40);
    *hi = exp(qhi) * (1.0 + 0x1p-23 + 0x1p-40);
}

struct DecideLds {
    double lo[kMaxObjects][kMaxObjects], hi[kMaxObjects][kMaxObjects], mid[kMaxObjects][kMaxObjects];
    unsigned cand[kMaxObjects];   // flagged rows: the ids that can be their argmax
    int win[kMaxObjects];         // certain rows: the argmax (-1: none / rejected)
    unsigned flagged;
    unsigned reject;              // rows whose every candidate is certainly <= 3 * prior
    int last;
    double prob[kMaxObjects][kMaxObjects];  // final: exact f32 (flagged rows) or the point estimate
    int bestj[kMaxObjects];
    double bestp[kMaxObjects];
    int map_i[kMaxObjects];
    double map_p[kMaxObjects];
    int rev[256];
    unsigned first[256];
    int newcount;
    ScanLds scan;
    float srow[kMaxObjects];  // exact path: the running f32 sum of each flagged row
    unsigned thist[64];       // tile order: bucket counts, then bucket cursors
    unsigned tmax;
    unsigned fresh_first[256];  // first pixels of the present, unmatched labels (newcount of them)
};

// The fused march's next launch order from this frame's tile durations: 64 linear cost buckets,
// heaviest first (LPT), a counting sort in one workgroup.  Order within a bucket is arbitrary;
// the order never changes results (the association's sums are integer, the render per pixel).
constexpr int kTileOrderPer = 32;  // tiles per thread of tile_order: launch orders of up to 8192 tiles
__device__ void tile_order(const unsigned* __restrict__ cost, unsigned* __restrict__ perm, int n, unsigned* thist,
                           unsigned* tmax) {
    const int tid = threadIdx.x;
    if (tid < 64) thist[tid] = 0u;
    if (tid == 0) *tmax = 0u;
    unsigned c[kTileOrderPer];
#pragma unroll
    for (int j = 0; j < kTileOrderPer; ++j) {  // every load in flight together
        const int i = tid + 256 * j;
        c[j] = i < n ? cost[i] : 0u;
    }
    unsigned mx = 0;
#pragma unroll
    for (int j = 0; j < kTileOrderPer; ++j) mx = max(mx, c[j]);
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, off, 64));
    __syncthreads();  // the counters' initialisation
    if ((tid & 63) == 0) atomicMax(tmax, mx);
    __syncthreads();
    const unsigned long long den = (unsigned long long)*tmax + 1ull;
    unsigned bk[kTileOrderPer];
#pragma unroll
    for (int j = 0; j < kTileOrderPer; ++j) {
        bk[j] = 63u - (unsigned)(((unsigned long long)c[j] * 64ull) / den);
        if (tid + 256 * j < n) atomicAdd(&thist[bk[j]], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        unsigned run = 0;
        for (int k = 0; k < 64; ++k) {
            const unsigned v = thist[k];
            thist[k] = run;
            run += v;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kTileOrderPer; ++j)
        if (tid + 256 * j < n) perm[atomicAdd(&thist[bk[j]], 1u)] = (unsigned)(tid + 256 * j);
}

__global__ __launch_bounds__(256) void k_assoc_decide(DecideArgs a) {
    __shared__ DecideLds L;
    AssocTables* T = a.T;
    const int tid = threadIdx.x;
    // an extra last workgroup orders the next fused march's tiles, beside the decision
    const unsigned nwork = gridDim.x - (a.tile_n > 0 ? 1u : 0u);
    if (blockIdx.x >= nwork) {
        tile_order(a.tile_cost, a.tile_perm, a.tile_n, L.thist, &L.tmax);
        return;
    }
    // every table word this workgroup reads, loads in flight together (the rows past max_now
    // hold zeros), and what the last arriver reads besides
    static_assert(kMaxObjects * kMaxObjects == 4 * 256, "four table entries per thread");
    const unsigned maxl = T->max_label;
    const unsigned first_pre = T->first_px[tid];
    const int num_pre = *a.num_objs_dev;
    long long Av[4], Cv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int k = tid + 256 * m, i = k / kMaxObjects, j = k % kMaxObjects;
        Av[m] = T->t1[i][j] + T->t2[j] - T->t3[i][j];
        Cv[m] = (long long)T->c1[i] + (long long)T->c2[j] - (long long)T->c3[i][j];
    }
    const unsigned posm = T->pos_max;
    const int max_now = min((int)maxl + 1, kMaxObjects);
    const float thr_f = 3.0f * a.eps;  // tsdf.cu:349, a float product
    const double thr = (double)thr_f;
    // the certificate's assumptions (prob_interval): every term within (-4, 4), the range the
    // device logf was checked over; outside it (eps below 0.05, probabilities 32 x n_obs or
    // more) every present row takes the exact path
    const bool cert_ok = a.eps >= 0.05f && a.eps < 1.0f && posm < kPosCap;
    const double P = posm ? ((double)posm + 0.5) / kFixScale + kTermSlack : 0.0;
    // ---- certificate (every workgroup) ----
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int k = tid + 256 * m, i = k / kMaxObjects, j = k % kMaxObjects;
        double lo = 0.0, hi = 0.0, mid = 0.0;
        if (i >= 1 && j >= 1 && i < max_now) prob_interval(Av[m], Cv[m], P, &lo, &hi, &mid);
        L.lo[i][j] = lo;
        L.hi[i][j] = hi;
        L.mid[i][j] = mid;
    }
    if (tid == 0) {
        L.flagged = 0u;
        L.reject = 0u;
    }
    __syncthreads();
    if (tid < kMaxObjects) {
        const int i = tid;
        unsigned cand = 0u;
        int win = -1;
        bool flag = false, rej = false;
        if (i >= 1 && i < max_now) {
            // point-estimate argmax (first maximum) and the best lower bound
            double mp = 0.0, maxlo = 0.0, maxhi = 0.0;
            int w = -1;
            for (int j = 1; j < kMaxObjects; ++j) {
                if (L.mid[i][j] > mp) { mp = L.mid[i][j]; w = j; }
                maxlo = fmax(maxlo, L.lo[i][j]);
                maxhi = fmax(maxhi, L.hi[i][j]);
            }
            bool certain = true;
            if (w < 0) {
                certain = maxhi == 0.0;  // every count zero: no candidate (prob 0 everywhere)
            } else {
                for (int j = 1; j < kMaxObjects; ++j)
                    if (j != w && !(L.hi[i][j] < L.lo[i][w])) certain = false;
            }
            if (!(maxhi > thr)) {
                win = -1;  // every candidate is rejected whatever the argmax
                rej = true;
            } else if (certain && w >= 0 && L.lo[i][w] > thr) {
                win = w;
                cand = 1u << w;
            } else {
                flag = true;
                for (int j = 1; j < kMaxObjects; ++j)
                    if (L.hi[i][j] >= maxlo && L.hi[i][j] > thr) cand |= 1u << j;
            }
        }
        L.cand[i] = cand;
        L.win[i] = win;
        if (flag) atomicOr(&L.flagged, 1u << i);
        if (rej) atomicOr(&L.reject, 1u << i);
    }
    __syncthreads();
    if (tid >= 1 && tid < kMaxObjects) {  // greedy per previous id j: potential winners
        const int j = tid;
        const unsigned F0 = L.flagged;
        double bar = 0.0;
        for (int i = 1; i < max_now; ++i)
            if (!((F0 >> i) & 1u) && L.win[i] == j) bar = fmax(bar, L.lo[i][j]);
        unsigned W = 0u;
        for (int i = 1; i < max_now; ++i)
            if (((L.cand[i] >> j) & 1u) && L.hi[i][j] >= bar) W |= 1u << i;
        if (__popc(W) >= 2) atomicOr(&L.flagged, W);
    }
    __syncthreads();
    const unsigned present = (max_now >= 32 ? 0xFFFFFFFFu : ((1u << max_now) - 1u)) & ~1u;
    unsigned F = L.flagged;
    if (a.force_exact || !cert_ok) F = present;
    const unsigned R = F == present ? 0u : L.reject & ~F;  // rows certainly rejected (not recomputed)
    if (a.certify_only) {  // one workgroup: report, leave tables and counts as they are
        if (tid == 0) {
            a.D->exact_missing = F;
            a.D->exact_rows = 0u;
            a.D->reject_rows = R;
        }
        return;
    }
    const bool have_px = a.px.bits != nullptr;
    // F is the same in every workgroup (the same certificate of the same tables): without a
    // flagged row nothing is handed over but the tickets, so the hand-off needs no fences (an
    // agent-scope release writes back the XCD's L2, an acquire invalidates it)
    const bool exact = F != 0u && have_px;
    // ---- exact sums: column j = blockIdx.x of every flagged row, one pass over the pixels ----
    if (F && have_px && blockIdx.x >= 1) {
        const int j = (int)blockIdx.x;
        const float c0 = glibc::logf(fmaxf(0.0f, a.eps));
        const unsigned rows = F & present;
        exact_rows_sum(rows, j, a, c0, L.scan, L.srow);
        // write-through (sc1) stores: the deciding workgroup may sit on another XCD
        if (tid < kMaxObjects && ((rows >> tid) & 1u))
            __hip_atomic_store(&a.X->A[tid][j], L.srow[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- the last workgroup decides (in-launch hand-off: every storing wave drains its stores,
    // one release + counter ticket per workgroup, one acquire in the last arriver) ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        if (exact) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // self-resetting ticket: the nwork-th increment wraps the counter back to 0 (the decides
        // of one handle never overlap: they share its tables)
        const unsigned ticket = atomicInc(&a.X->counter, nwork - 1u);
        L.last = ticket == nwork - 1u;
    }
    __syncthreads();
    if (!L.last) return;
    if (tid == 0 && exact) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    AssocDecision* D = a.D;
    const unsigned Fx = have_px ? F : 0u;
    for (int k = tid; k < kMaxObjects * kMaxObjects; k += 256) {
        const int i = k / kMaxObjects, j = k % kMaxObjects;
        double prob = L.mid[i][j];
        if (i >= 1 && j >= 1 && i < max_now && ((Fx >> i) & 1u)) {
            const long long C = (long long)T->c1[i] + (long long)T->c2[j] - (long long)T->c3[i][j];
            const float A = __hip_atomic_load(&a.X->A[i][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            prob = C == 0 ? 0.0 : (double)glibc::expf(A / (float)C);  // tsdf.cu:343 in f32
        }
        L.prob[i][j] = prob;
    }
    L.rev[tid] = -1;
    L.first[tid] = first_pre;
    if (tid == 0) L.newcount = 0;
    __syncthreads();
    if (tid < kMaxObjects) {
        int max_j = -1;
        double max_p = 0.0;
        if (tid >= 1 && tid < max_now)
            for (int j = 1; j < kMaxObjects; ++j)
                if (L.prob[tid][j] > max_p) { max_j = j; max_p = L.prob[tid][j]; }
        L.bestj[tid] = max_j;
        L.bestp[tid] = max_p;
    }
    __syncthreads();
    if (tid < kMaxObjects) {
        int mi = -1;
        double mp = 0.0;
        for (int i = 1; i < max_now; ++i)
            if (L.bestj[i] == tid && L.bestp[i] > thr && (mi < 0 || mp < L.bestp[i])) { mi = i; mp = L.bestp[i]; }
        L.map_i[tid] = mi;
        L.map_p[tid] = mp;
        D->assigned_prev[tid] = -1;
        D->assigned_prob[tid] = 0.0f;
    }
    __syncthreads();
    if (tid < kMaxObjects && L.map_i[tid] >= 0) {
        L.rev[L.map_i[tid]] = tid;
        D->assigned_prev[L.map_i[tid]] = tid;
        D->assigned_prob[L.map_i[tid]] = (float)L.map_p[tid];
    }
    __syncthreads();
    const int num = num_pre;
    // lanes 1..255: a present, unmatched label gets num + (rank of its first pixel among those
    // labels; first pixels are distinct), from a compact list of the fresh labels' first pixels
    const bool fresh = tid >= 1 && L.rev[tid] < 0 && L.first[tid] != 0xFFFFFFFFu;
    if (fresh) L.fresh_first[atomicAdd(&L.newcount, 1)] = L.first[tid];
    __syncthreads();
    int lut = tid;
    if (tid >= 1 && L.rev[tid] >= 0) {
        lut = L.rev[tid];
    } else if (fresh) {
        const unsigned mine = L.first[tid];
        int rank = 0;
        for (int u = 0; u < L.newcount; ++u) rank += L.fresh_first[u] < mine ? 1 : 0;
        lut = num + rank;
        // id policy 1 (a deviation, SEMTSDF_F_ID_SATURATE): an id without a histogram bin is not
        // minted, the label becomes background
        if (a.id_policy == 1 && lut >= kMaxObjects) lut = 0;
    }
    // policy 0: the reference's ids (tsdf.cu:379-383), stored in the u8 mask modulo 256 as its
    // mask_ptr[i] = num_objs does; ids >= 32 have no histogram bin (the integrate drops their
    // votes, counting them: semtsdf_state::label_votes_dropped)
    D->lut[tid] = (unsigned char)lut;
    __syncthreads();
    if (tid == 0) {
        const int mx = (int)T->max_label + 1;
        const int after = a.id_policy == 1 ? max(num, min(num + L.newcount, kMaxObjects)) : num + L.newcount;
        D->max_obj_now = mx;
        D->num_objs_before = num;
        D->num_objs_after = after;
        // only a frame that mints an id past the histogram (or brings a raw label past it) is
        // flagged: later frames of a volume beyond 32 objects mint none of their own
        D->bad_label = ((L.newcount > 0 && after > kMaxObjects) || mx > kMaxObjects) ? 1 : 0;
        D->exact_rows = Fx;
        D->exact_missing = have_px ? 0u : F;
        D->reject_rows = R;
        *a.num_objs_dev = after;
        if (posm > a.X->pos_max) a.X->pos_max = posm;
        if (Fx) {
            a.X->frames += 1u;
            a.X->rows += (unsigned)__popc(Fx);
        }
    }
    // every read of T is above (the last barrier orders them): clear it for the next frame
    uint2* w = reinterpret_cast<uint2*>(T);
    for (unsigned i = tid; i < sizeof(AssocTables) / 8; i += 256) w[i] = make_uint2(0u, 0u);
    __syncthreads();
    T->first_px[tid] = 0xFFFFFFFFu;
}

hipError_t launch_assoc_decide(const DecideArgs& a, hipStream_t s) {
    // workgroup j >= 1 computes column j of the exact sums: one workgroup when there is no
    // per-pixel data to compute them from
    const unsigned grid = ((a.certify_only || !a.px.bits) ? 1u : (unsigned)kMaxObjects) + (a.tile_n > 0 ? 1u : 0u);
    hipLaunchKernelGGL(k_assoc_decide, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

// filter_overlaps from the reference's own inputs (tsdf.cu:304: probs [npx][32], box_mask
// [npx][32]): the tables and per-pixel data the association march leaves, for a decision on
// given probabilities (parity tests of the decision; the reference's function boundary).
// The mask statistics are those of k_mask_stats (first pixel of every label, max label).
__global__ __launch_bounds__(256) void k_assoc_from_probs(const float* __restrict__ probs,
                                                          const uint8_t* __restrict__ box, const uint8_t* __restrict__ mask,
                                                          int npx, float n_obs, float eps, AssocTables* t, AssocPixels px) {
    __shared__ AssocLds s;
    assoc_lds_clear(s);
    __syncthreads();
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k < npx) {
        float p[kMaxObjects];
        unsigned bx = 0, pres = 0;
#pragma unroll
        for (int j = 0; j < kMaxObjects; ++j) {
            p[j] = probs[(size_t)k * kMaxObjects + j];
            if (box[(size_t)k * kMaxObjects + j]) bx |= 1u << j;
            if (j >= 1 && p[j] != 0.0f) {
                pres |= 1u << j;
                px.p[(size_t)j * npx + k] = p[j];
            }
        }
        px.bits[k] = make_uint2(pres, bx & ~1u);
        const unsigned m = mask[k];
        if (m > 0 && m < (unsigned)kMaxObjects) {
            atomicAdd(&s.c1[m], 1u);
#pragma unroll
            for (int j = 1; j < kMaxObjects; ++j) {
                const float L = glibc::logf(fmaxf(p[j] / n_obs, eps));
                atomicAdd(reinterpret_cast<unsigned long long*>(&s.t1[m][j]), (unsigned long long)to_fix(L));
                if (L > 0.0f) atomicMax(&s.pos, pos_fix(L));  // probabilities above n_obs
            }
        }
#pragma unroll
        for (int n = 1; n < kMaxObjects; ++n) {
            if (!((bx >> n) & 1u)) continue;
            const unsigned long long f = (unsigned long long)to_fix(glibc::logf(fmaxf(1.0f - p[n] / n_obs, eps)));
            atomicAdd(reinterpret_cast<unsigned long long*>(&s.t2[n]), f);
            atomicAdd(&s.c2[n], 1u);
            if (m > 0 && m < (unsigned)kMaxObjects) {
                atomicAdd(reinterpret_cast<unsigned long long*>(&s.t3[m][n]), f);
                atomicAdd(&s.c3[m][n], 1u);
            }
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kMaxObjects * kMaxObjects; q += 256) {
        const long long v1 = (&s.t1[0][0])[q];
        if (v1) atomicAdd(reinterpret_cast<unsigned long long*>(&t->t1[0][0]) + q, (unsigned long long)v1);
        const long long v3 = (&s.t3[0][0])[q];
        if (v3) atomicAdd(reinterpret_cast<unsigned long long*>(&t->t3[0][0]) + q, (unsigned long long)v3);
        const unsigned c3 = (&s.c3[0][0])[q];
        if (c3) atomicAdd(&t->c3[0][0] + q, c3);
    }
    if (threadIdx.x < kMaxObjects) {
        const int q = threadIdx.x;
        if (s.t2[q]) atomicAdd(reinterpret_cast<unsigned long long*>(&t->t2[q]), (unsigned long long)s.t2[q]);
        if (s.c1[q]) atomicAdd(&t->c1[q], s.c1[q]);
        if (s.c2[q]) atomicAdd(&t->c2[q], s.c2[q]);
    }
    if (threadIdx.x == 0 && s.pos) atomicMax(&t->pos_max, s.pos);
}

hipError_t launch_assoc_from_probs(const float* probs, const uint8_t* box, const uint8_t* mask, int npx, float n_obs,
                                   float eps, AssocTables* t, AssocPixels px, hipStream_t s) {
    if (npx <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_assoc_from_probs, dim3((npx + 255) / 256), dim3(256), 0, s, probs, box, mask, npx, n_obs, eps,
                       t, px);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_libm_eval(int fn, const float* __restrict__ x, float* __restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        y[i] = fn == 0 ? glibc::logf(x[i]) : fn == 1 ? glibc::expf(x[i]) : logf(x[i]);  // 2: the march's logf
}

hipError_t launch_libm_eval(int fn, const float* x, float* y, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t b = (n + 255) / 256;
    hipLaunchKernelGGL(k_libm_eval, dim3((unsigned)(b < 65536 ? b : 65536)), dim3(256), 0, s, fn, x, y, n);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_relabel(uint8_t* __restrict__ mask, int npx, const AssocDecision* __restrict__ d) {
    __shared__ unsigned char s_lut[256];
    s_lut[threadIdx.x] = d->lut[threadIdx.x];
    __syncthreads();
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npx; i += gridDim.x * blockDim.x) mask[i] = s_lut[mask[i]];
}

hipError_t launch_relabel(uint8_t* mask, int npx, const AssocDecision* d, hipStream_t s) {
    int blocks = (npx + 255) / 256;
    if (blocks > 512) blocks = 512;
    hipLaunchKernelGGL(k_relabel, dim3(blocks), dim3(256), 0, s, mask, npx, d);
    return hipGetLastError();
}

// The relabel of a frame whose prepass ran beside its association march (raw labels in the
// pixel records): the mask in place and the label byte of each pixel record.  One image row
// per blockIdx.y; four pixels per lane when the rows are 4-byte aligned (one tile row of
// records).
__global__ __launch_bounds__(256) void k_relabel_records(uint8_t* __restrict__ mask, int w, int h, DepthPyramid p,
                                                         const AssocDecision* __restrict__ d) {
    __shared__ unsigned char s_lut[256];
    s_lut[threadIdx.x] = d->lut[threadIdx.x];
    __syncthreads();
    const bool vec = ((uintptr_t)mask & 3u) == 0 && (w & 3) == 0;
    for (int y = blockIdx.y; y < h; y += gridDim.y) {
        uint8_t* row = mask + (size_t)y * w;
        if (vec) {
            for (int x4 = blockIdx.x * blockDim.x + threadIdx.x; x4 < (w >> 2); x4 += gridDim.x * blockDim.x) {
                const unsigned m4 = reinterpret_cast<const unsigned*>(row)[x4];
                unsigned o4 = 0;
                uint2* r = p.px + rec_index(p, (unsigned)(4 * x4), (unsigned)y);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const unsigned m = s_lut[(m4 >> (8 * j)) & 0xFFu];
                    o4 |= m << (8 * j);
                    r[4 * j].y = (r[4 * j].y & 0x00FFFFFFu) | (m << 24);  // a tile is column-major
                }
                reinterpret_cast<unsigned*>(row)[x4] = o4;
            }
        } else {
            for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < w; x += gridDim.x * blockDim.x) {
                const unsigned m = s_lut[row[x]];
                row[x] = (uint8_t)m;
                uint2& r = p.px[rec_index(p, (unsigned)x, (unsigned)y)];
                r.y = (r.y & 0x00FFFFFFu) | (m << 24);
            }
        }
    }
}

hipError_t launch_relabel_records(uint8_t* mask, int w, int h, const DepthPyramid& p, const AssocDecision* d,
                                  hipStream_t s) {
    const int bx = ((w + 3) / 4 + 255) / 256;
    const int by = h < 512 ? (h > 0 ? h : 1) : 512;
    hipLaunchKernelGGL(k_relabel_records, dim3(bx, by), dim3(256), 0, s, mask, w, h, p, d);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// render raycast (show_tsdf_kernel viewer.cu:17-86; colour mode tsdf_render.frag:125-131)
// ------------------------------------------------------------------------------------
// Shade one hit (viewer.cu:66-84 label mode; tsdf_render.frag:125-131 colour mode).
__device__ __forceinline__ void shade_hit(const VolGeom& g, const VolBufs& vb, const Tri& tr, int mode, int color_i32,
                                          const uint8_t* __restrict__ palette, uint8_t* b, uint8_t* gch, uint8_t* r) {
    if (mode == 0) {
        float max_cnt = 0.0f;
        int obj = 0;
        unsigned bins = tri_bins(vb.hmask, tr);  // bins outside the mask are 0: never a strict max
        while (bins) {
            const int k = __ffs((int)bins) - 1;
            bins &= bins - 1u;
            const float c = tri_eval(vb.hist + (uint64_t)k * g.nvox, tr);
            if (c > max_cnt) { max_cnt = c; obj = k; }
        }
        if (obj > 0) {
            *b = palette[obj * 3 + 2];
            *gch = palette[obj * 3 + 1];
            *r = palette[obj * 3 + 0];
        }
    } else {
        float cc[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            // colour is stored padded to 4 channels: [v*4 + ch]
            const uint64_t i000 = (uint64_t)tr.i000 * 4 + ch;
            const uint64_t sx = (uint64_t)tr.dx * 4, sy = (uint64_t)tr.dy * 4, sz = (uint64_t)tr.dz * 4;
            float d[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint64_t off = ((k & 4) ? sx : 0) + ((k & 2) ? sy : 0) + ((k & 1) ? sz : 0);
                d[k] = color_i32 ? (float)reinterpret_cast<const int32_t*>(vb.color)[i000 + off]
                                 : (float)reinterpret_cast<const uint8_t*>(vb.color)[i000 + off];
            }
            const float low = mixf(mixf(d[0], d[4], tr.fx), mixf(d[2], d[6], tr.fx), tr.fy);
            const float high = mixf(mixf(d[1], d[5], tr.fx), mixf(d[3], d[7], tr.fx), tr.fy);
            cc[ch] = mixf(low, high, tr.fz);
        }
        *b = (uint8_t)(int)cc[0];
        *gch = (uint8_t)(int)cc[1];
        *r = (uint8_t)(int)cc[2];
    }
}

// STATS: instrumentation build of the kernel (a run-time select of the stats pointer would
// keep MarchStats in scratch memory)
// One 16x16-pixel tile (bx, by) of a render, a whole workgroup.
template <bool STATS, bool OCT>
__device__ __forceinline__ void render_tile(const RenderArgs& a, int bx, int by) {
    const int x = bx * 16 + (threadIdx.x & 15);
    const int y = by * 16 + (threadIdx.x >> 4);
    if (x >= a.width || y >= a.height) return;
    if (STATS && a.row1 > 0 && (by < a.row0 || by >= a.row1)) return;
    const int px = y * a.width + x;
    float ox, oy, oz, dx, dy, dz, t;
    ray_render(a.cam, x, y, &ox, &oy, &oz, &dx, &dy, &dz);
    uint8_t b = 0, gch = 0, r = 0;
    float th = -1.0f;
    MarchStats ms;
    const uint64_t t_start = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    if (march_ray<OCT>(a.g, a.b, ox, oy, oz, dx, dy, dz, &t, STATS ? &ms : nullptr)) {
        th = t;
        const Tri tr = tri_setup<false>(a.g, fmaf(t, dx, ox), fmaf(t, dy, oy), fmaf(t, dz, oz));
        shade_hit(a.g, a.b, tr, a.mode, a.color_i32, a.palette, &b, &gch, &r);
    }
    a.out_bgr[(size_t)px * 3 + 0] = b;
    a.out_bgr[(size_t)px * 3 + 1] = gch;
    a.out_bgr[(size_t)px * 3 + 2] = r;
    if (a.out_t) a.out_t[px] = th;
    if (STATS) {  // instrumentation
        unsigned* q = a.ray_stats + (size_t)px * 4;
        q[0] = ms.iters; q[1] = ms.lookups; q[2] = ms.evals; q[3] = ms.skipped;
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const size_t npx = (size_t)a.width * a.height;
        const unsigned wave = (unsigned)(by * ((a.width + 15) / 16) + bx) * 4 + (threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0) {
            unsigned long long* w = reinterpret_cast<unsigned long long*>(a.ray_stats + npx * 4) + wave * 2;
            w[0] = t_start;
            w[1] = t_end;
        }
    }
}

template <bool STATS, bool OCT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEMTSDF_MARCH_WPE))) void k_render(RenderArgs a) {
    render_tile<STATS, OCT>(a, (int)blockIdx.x, (int)blockIdx.y);
}

// A render of the volume and the association march of the next frame in one launch: both
// read the same volume state (the association of frame k + 1 marches the state the live
// view of frame k shows), and both are bound by their slowest rays, so one grid lets the
// tiles of each fill the other's tail.  Workgroup b: tiles alternate (association, render)
// while both have tiles left, then the rest of the larger one.
template <bool OCT>
#ifndef SEMTSDF_FUSED_WPE
#define SEMTSDF_FUSED_WPE 4  // 4 waves per SIMD: at most 128 VGPRs (the association's per-pixel output put it at 131)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEMTSDF_FUSED_WPE))) void k_march_fused(
    AssocArgs aa, RenderArgs ra, FramePre pre, int na, int nr) {
    __shared__ AssocLds s;
    // the frame's mask statistics and prepass tiles first (FramePre: they read only the frame's
    // inputs; the marches read the volume)
    const int npre = pre.nms + pre.npy;
    if ((int)blockIdx.x < npre) {
        const int pb = (int)blockIdx.x;
        if (pb < pre.nms) {
            mask_stats_block(pre.mask, pre.npx, pre.T, pb, pre.nms);
        } else {
            const int q = pb - pre.nms;
            pyramid_tile(pre.depth, pre.rgb, pre.pmask, pre.w, pre.h, pre.scale, pre.vec, pre.pyr, pre.list_count,
                         nullptr, q % pre.pyr.w1, q / pre.pyr.w1);
        }
        return;
    }
    const unsigned bt = blockIdx.x - (unsigned)npre;
    // launch order: block b takes tile perm[b] (the previous frame's heaviest first)
    const int b = aa.tile_perm ? (int)__builtin_amdgcn_readfirstlane(aa.tile_perm[bt]) : (int)bt;
    const int m = min(na, nr);
    const uint64_t t0 = aa.tile_cost ? __builtin_amdgcn_s_memrealtime() : 0;
    bool assoc;
    int t;
    if (b < 2 * m) {
        assoc = (b & 1) == 0;
        t = b >> 1;
    } else {
        assoc = na > nr;
        t = b - m;
    }
    if (assoc) {
        const int tx = (aa.width + 15) / 16;
        assoc_tile<OCT>(aa, s, t % tx, t / tx);
    } else {
        const int tx = (ra.width + 15) / 16;
        render_tile<false, OCT>(ra, t % tx, t / tx);
    }
    if (aa.tile_cost) {  // the tile's duration (100 MHz ticks), all its waves done
        __syncthreads();
        if (threadIdx.x == 0) aa.tile_cost[b] = (unsigned)min(__builtin_amdgcn_s_memrealtime() - t0, (uint64_t)0xFFFFFFFFu);
    }
}

hipError_t launch_march_fused(const AssocArgs& aa, const RenderArgs& ra, const FramePre& pre, hipStream_t s) {
    const int na = ((aa.width + 15) / 16) * ((aa.height + 15) / 16);
    const int nr = ((ra.width + 15) / 16) * ((ra.height + 15) / 16);
    const int grid = pre.nms + pre.npy + na + nr;
    if (oct_maps(aa.b))
        hipLaunchKernelGGL(k_march_fused<true>, dim3(grid), dim3(256), 0, s, aa, ra, pre, na, nr);
    else
        hipLaunchKernelGGL(k_march_fused<false>, dim3(grid), dim3(256), 0, s, aa, ra, pre, na, nr);
    return hipGetLastError();
}

hipError_t launch_render(const RenderArgs& a, hipStream_t s) {
    const dim3 grid((a.width + 15) / 16, (a.height + 15) / 16);
    if (a.ray_stats)
        hipLaunchKernelGGL((k_render<true, false>), grid, dim3(256), 0, s, a);
    else
        if (oct_maps(a.b))
            hipLaunchKernelGGL((k_render<false, true>), grid, dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((k_render<false, false>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Z-sharded raycast.  The march of march_ray is sequential along the ray
// (sticky quarter step, refinement from the previous sample), so it is split into steps
// that every rank of the group runs on its own planes, with an all-gather of one 8-byte
// record per pixel between steps (host side: semtsdf/shard.py):
//   step 0  coarse march (step = voxel.x): first owned sample with f < voxel.x/2, or -1
//           when the first sample rejects the ray;
//   step 1  min over ranks = the global coarse event k.  f_k < 0: the owner of sample
//           k-1 sends f_{k-1}.  Otherwise the quarter-step march continues from t_k and
//           each rank sends its first owned sample with f < 0;
//   step 2  min over ranks = the fine hit j; for j >= 2 the owner of sample j-1 sends it;
//   final   t_hit = t_s + step * f / (f_prev - f) as in march_ray; the owner of the hit
//           point shades it (render) or accumulates its association terms (assoc).
// Sample positions are replayed with the same float additions as march_ray, a sample is
// evaluated only by the shard owning its base plane (which also holds plane + 1), and
// every value is computed with the same arithmetic as the single volume, so the
// composite is bit-identical to the single-volume raycast.
// ------------------------------------------------------------------------------------
// A per-pixel record is 8 bytes {value (low word), key (high word)}: as a little-endian
// int64 it orders by the signed key first, so the exchange between steps can be an
// all-gather of every shard's records (n = nshards; the minimum is taken here) or an
// all-reduce MIN over int64 (n = 1), which moves 1/nshards of the bytes.  Keys are unique
// per pixel except -1 and INT_MAX, whose values agree on every shard.
__device__ __forceinline__ int2 mk_rec(int key, int val) { return make_int2(val, key); }
__device__ __forceinline__ int rkey(int2 r) { return r.y; }
__device__ __forceinline__ int rval(int2 r) { return r.x; }

__device__ __forceinline__ int2 gather_min(const int2* __restrict__ g, int n, int npx, int px) {
    int2 best = mk_rec(INT_MAX, 0);
    for (int r = 0; r < n; ++r) {
        const int2 v = g[(size_t)r * npx + px];
        if (rkey(v) < rkey(best)) best = v;
    }
    return best;
}

// t += step repeated n times (t > 0), in O(1) per binade of t: the closed form of skip_steps
// (inside a binade every RN(t + step) adds the same d, so m additions are t + m d while the
// result stays in the binade; ties and binade crossings are single additions).
__device__ __forceinline__ float advance_n(float t, float step, int n) {
    while (n > 0) {
        const float t1 = t + step;
        const int eb = __float_as_int(t) & 0x7F800000;
        const float ulp = __int_as_float(eb - (23 << 23)), top = __int_as_float(eb + (1 << 23));
        const float d = t1 - t;  // exact (t1 within a factor 2 of t)
        int m = 0;
        if (fabsf(step - d) * 2.0f != ulp && t1 < top) {
            m = min(max((int)((top - t) * __builtin_amdgcn_rcpf(d)), 1), n);  // estimate, fixed up below
            while (m > 1 && !(t + (float)m * d < top)) --m;
        }
        if (m <= 1) {
            t = t1;
            --n;
            continue;
        }
        t = t + (float)m * d;
        n -= m;
    }
    return t;
}

// skip_steps counting its additions in n (t stops at the first value >= tend)
__device__ __forceinline__ void skip_steps_n(float& t, float step, float tend, int& n) {
    while (t < tend) {
        const float t1 = t + step;
        if (!(t1 < tend)) {
            t = t1;
            ++n;
            break;
        }
        const int eb = __float_as_int(t) & 0x7F800000;
        const float ulp = __int_as_float(eb - (23 << 23)), top = __int_as_float(eb + (1 << 23));
        const float d = t1 - t;
        const float lim = fminf(tend, top);
        int m = 0;
        if (fabsf(step - d) * 2.0f != ulp && t1 < top) {
            m = max((int)((lim - t) * __builtin_amdgcn_rcpf(d)), 1);
            while (m > 1 && !(t + (float)m * d < lim)) --m;
            while (t + (float)(m + 1) * d < lim) ++m;
        }
        if (m <= 1) {
            t = t1;
            ++n;
            continue;
        }
        t = t + (float)m * d;
        n += m;
    }
}

__device__ __forceinline__ float replay_t(float t, int ncoarse, int nfine, float vx) {
    return advance_n(advance_n(t, vx, ncoarse), vx / 4.0f, nfine);
}

struct RayGeo {
    float ox, oy, oz, dx, dy, dz, t0, t1;
    bool in;
};

__device__ __forceinline__ RayGeo shard_ray(const ShardRayArgs& a, int x, int y) {
    RayGeo r;
    if (a.kind == 2) ray_assoc(a.cam, x, y, &r.ox, &r.oy, &r.oz, &r.dx, &r.dy, &r.dz);
    else ray_render(a.cam, x, y, &r.ox, &r.oy, &r.oz, &r.dx, &r.dy, &r.dz);
    r.in = ray_bounds(a.g, r.ox, r.oy, r.oz, r.dx, r.dy, r.dz, &r.t0, &r.t1);
    return r;
}

__device__ __forceinline__ bool owns_at(const ShardRayArgs& a, const RayGeo& r, float t) {
    return sample_owner(a.g, fmaf(t, r.dz, r.oz)) == a.g.shard;
}

__device__ __forceinline__ float sample_at(const ShardRayArgs& a, const RayGeo& r, float t) {
    return sample_sdf(a.g, a.b.sdf, fmaf(t, r.dx, r.ox), fmaf(t, r.dy, r.oy), fmaf(t, r.dz, r.oz));
}

// false when the brick map proves the sample >= voxel/2 (see march_ray).  A skippable brick
// also leaves a box in the cursor, in global voxel coordinates: its distance box ((2r-1)^3
// bricks of the local distance map, or the brick alone without one) clipped in z to the
// sample's chunk block and, inside it, to the base planes w < chunk (their +1 plane is stored:
// the halo at most; local bricks across a block boundary are not global neighbours).  Every
// sample inside the box is >= voxel/2 whoever owns it, so the march steps through it with
// exact additions.
__device__ __forceinline__ bool sample_at_skip(const ShardRayArgs& a, const RayGeo& r, float t, float thr,
                                               SkipCursor& cur, float* f) {
    const VolGeom& g = a.g;
    const TriCoord c = tri_coord(g, fmaf(t, r.dx, r.ox), fmaf(t, r.dy, r.oy), fmaf(t, r.dz, r.oz));
    if (a.b.bmin) {
        const int br = brick_of(g, c);
        if (br != cur.brick) {
            cur.brick = br;
            int rad = 0;
            const int oct = SEMTSDF_BRICK_DIST && SEMTSDF_BRICK_OCT && a.b.boct
                                ? (r.dx < 0.0f ? 1 : 0) | (r.dy < 0.0f ? 2 : 0) | (r.dz < 0.0f ? 4 : 0)
                                : -1;
            if (SEMTSDF_BRICK_DIST && a.b.bdist) {
                rad = oct >= 0 ? (int)reinterpret_cast<const uint8_t*>(a.b.boct)[(size_t)br * 8 + oct] : a.b.bdist[br];
                cur.skip = rad > 0;
            } else {
                cur.skip = a.b.bmin[br] >= thr;
                rad = cur.skip ? 1 : 0;
            }
            cur.lo[0] = 1e30f;  // no box unless set below
            cur.hi[0] = -1e30f;
            if (cur.skip) {
                const int bx = c.xc >> 3, by = c.yc >> 3, bz = c.zl >> 3;
                const int per = g.nshards > 1 ? g.chunk + g.halo : g.lz;  // local planes per chunk block
                const int blk0 = g.nshards > 1 ? c.zl / per * per : 0;   // first local plane of the block
                const int own = g.nshards > 1 ? g.chunk : g.lz;          // base planes w < own in the block
                // the box: rad bricks along each axis on the ray's side (both sides without an
                // octant map or with the brick alone)
                const bool sym = oct < 0;
                const int nx = sym || (oct & 1) ? rad - 1 : 0, px_ = sym || !(oct & 1) ? rad : 1;
                const int ny = sym || (oct & 2) ? rad - 1 : 0, py_ = sym || !(oct & 2) ? rad : 1;
                const int nz = sym || (oct & 4) ? rad - 1 : 0, pz_ = sym || !(oct & 4) ? rad : 1;
                const int lz0 = max((bz - nz) * 8, blk0), lz1 = min((bz + pz_) * 8, blk0 + own);  // local, excl.
                if (lz0 < lz1) {
                    const int gz0 = local_to_global_z(g, blk0) + (lz0 - blk0);
                    const int gz1 = gz0 + (lz1 - lz0);
                    const int x0 = bx - nx, y0 = by - ny, x1 = bx + px_, y1 = by + py_;
                    const float m = 0.01f;
                    cur.lo[0] = x0 <= 0 ? -1e30f : (float)(x0 * 8) + m;
                    cur.hi[0] = x1 >= g.nbx ? 1e30f : (float)(x1 * 8) - m;
                    cur.lo[1] = y0 <= 0 ? -1e30f : (float)(y0 * 8) + m;
                    cur.hi[1] = y1 >= g.nby ? 1e30f : (float)(y1 * 8) - m;
                    cur.lo[2] = gz0 <= 0 ? -1e30f : (float)gz0 + m;
                    cur.hi[2] = gz1 >= g.dimz ? 1e30f : (float)gz1 - m;
                }
            }
        }
        if (cur.skip) return false;
    }
    *f = tri_eval(a.b.sdf, tri_from(g, c));
    return true;
}

// Ray parameter a little before the ray's samples enter the next chunk this shard owns
// (along the direction of travel), or false when none lies ahead.  Approximate (half a
// voxel early): the caller jumps there with exact additions and tests ownership sample by
// sample from then on.
__device__ __forceinline__ bool next_owned_t(const ShardRayArgs& a, const RayGeo& r, float t, float* tend) {
    const VolGeom& g = a.g;
    if (r.dz == 0.0f) return false;
    const float iz = ((fmaf(t, r.dz, r.oz)) - g.start[2]) * g.rvox[2];
    const int zc = min(max((int)floorf(fminf(fmaxf(iz, -1.0f), (float)g.dimz)), 0), g.dimz - 1);
    const int c = zc / g.chunk, n = g.nshards, nch = (g.dimz + g.chunk - 1) / g.chunk;
    const int rc = c / n, k = c - rc * n;
    float zb;  // voxel coordinate of the boundary the samples cross into the owned chunk
    if (r.dz > 0.0f) {  // the first owned chunk at or after c
        const int pr = chunk_pos(rc, g.shard, n);
        const int cn = pr >= k ? rc * n + pr : (rc + 1) * n + chunk_pos(rc + 1, g.shard, n);
        if (cn <= c || cn >= nch) return false;
        zb = (float)(cn * g.chunk);
    } else {  // the last owned chunk at or before c
        const int pr = chunk_pos(rc, g.shard, n);
        const int cp = pr <= k ? rc * n + pr : (rc > 0 ? (rc - 1) * n + chunk_pos(rc - 1, g.shard, n) : -1);
        if (cp >= c || cp < 0) return false;
        zb = (float)((cp + 1) * g.chunk);
    }
    const float tb = (fmaf(zb, g.voxel[2], g.start[2]) - r.oz) / r.dz;
    *tend = tb - 0.5f * g.voxel[2] / fabsf(r.dz);
    return true;
}

__global__ __launch_bounds__(256) void k_shard_ray_step(ShardRayArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.width || y >= a.height) return;
    const int npx = a.width * a.height;
    const int px = y * a.width + x;
    const RayGeo r = shard_ray(a, x, y);
    const float vx = a.g.voxel[0];
    int2 rec = mk_rec(INT_MAX, 0);
    if (a.step == 0) {
        if (!r.in) {
            rec = mk_rec(-1, 0);
        } else {
            float t = r.t0;
            bool dead = false;
            const float thr = skip_threshold(a.g);
            SkipCursor cur;
            const RayVox rv = ray_vox(a.g, r.ox, r.oy, r.oz, r.dx, r.dy, r.dz);
            float f0;
            if (owns_at(a, r, t) && sample_at_skip(a, r, t, thr, cur, &f0)) {
                if (!(f0 > 0.0f)) { rec = mk_rec(-1, 0); dead = true; }
            }
            if (!dead) {
                if (!(t < r.t1)) {
                    rec = mk_rec(-1, 0);
                } else {
                    // the samples of the owned chunks only: runs of foreign samples are jumped
                    // with exact additions (sample k is still t0 + vx added k times)
                    int k = 0;
                    while (t < r.t1) {
                        if (cur.skip && in_skip_box(cur, rv, t)) {  // a skippable brick: no event inside
                            skip_steps_n(t, vx, fminf(r.t1, skip_box_exit(cur, rv)), k);
                            while (t < r.t1 && in_skip_box(cur, rv, t)) {
                                t += vx;
                                ++k;
                            }
                            continue;
                        }
                        if (owns_at(a, r, t)) {
                            float f;
                            if (sample_at_skip(a, r, t, thr, cur, &f) && f < vx / 2.0f) {
                                rec = mk_rec(k, __float_as_int(f));
                                break;
                            }
                            t += vx;
                            ++k;
                            continue;
                        }
                        float tend;
                        if (!next_owned_t(a, r, t, &tend)) break;
                        tend = fminf(tend, r.t1);
                        if (t < tend) {
                            skip_steps_n(t, vx, tend, k);
                        } else {
                            t += vx;
                            ++k;
                        }
                    }
                }
            }
        }
    } else if (a.step == 1) {
        const int2 c = gather_min(a.gathered, a.nrec, npx, px);
        if (rkey(c) < 0 || rkey(c) == INT_MAX) {
            a.st.k[px] = -1;
        } else {
            const int k = rkey(c);
            const float fk = __int_as_float(rval(c));
            a.st.k[px] = k;
            a.st.fk[px] = fk;
            if (fk < 0.0f) {
                a.st.j[px] = 0;
                const float t = replay_t(r.t0, k - 1, 0, vx);
                if (owns_at(a, r, t)) rec = mk_rec(0, __float_as_int(sample_at(a, r, t)));
            } else {
                float t = replay_t(r.t0, k, 0, vx);
                const float q = vx / 4.0f;
                const float thr = skip_threshold(a.g);
                SkipCursor cur;
                const RayVox rv = ray_vox(a.g, r.ox, r.oy, r.oz, r.dx, r.dy, r.dz);
                int j = 1;  // sample j of the quarter-step march is t_k + q added j times
                t += q;
                while (t < r.t1) {
                    if (cur.skip && in_skip_box(cur, rv, t)) {
                        skip_steps_n(t, q, fminf(r.t1, skip_box_exit(cur, rv)), j);
                        while (t < r.t1 && in_skip_box(cur, rv, t)) {
                            t += q;
                            ++j;
                        }
                        continue;
                    }
                    if (owns_at(a, r, t)) {
                        float f;
                        if (sample_at_skip(a, r, t, thr, cur, &f) && f < 0.0f) {
                            rec = mk_rec(j, __float_as_int(f));
                            break;
                        }
                        t += q;
                        ++j;
                        continue;
                    }
                    float tend;
                    if (!next_owned_t(a, r, t, &tend)) break;
                    tend = fminf(tend, r.t1);
                    if (t < tend) {
                        skip_steps_n(t, q, tend, j);
                    } else {
                        t += q;
                        ++j;
                    }
                }
            }
        }
    } else {  // step 2
        const int k = a.st.k[px];
        if (k >= 0) {
            const int2 c = gather_min(a.gathered, a.nrec, npx, px);
            if (a.st.fk[px] < 0.0f) {
                a.st.fp[px] = __int_as_float(rval(c));
            } else if (rkey(c) == INT_MAX) {
                a.st.k[px] = -1;  // the quarter-step march ran out: miss
            } else {
                const int j = rkey(c);
                a.st.j[px] = j;
                a.st.fj[px] = __int_as_float(rval(c));
                if (j == 1) {
                    a.st.fp[px] = a.st.fk[px];
                } else {
                    const float t = replay_t(r.t0, k, j - 1, vx);
                    if (owns_at(a, r, t)) rec = mk_rec(0, __float_as_int(sample_at(a, r, t)));
                }
            }
        }
    }
    a.send[px] = rec;
}

// Resolve the hit after step 2's gather: returns false on a miss, else t_hit.
__device__ __forceinline__ bool shard_resolve(const ShardRayArgs& a, const RayGeo& r, int px, int npx, float* t_hit) {
    const int k = a.st.k[px];
    if (k < 0) return false;
    const float vx = a.g.voxel[0];
    float ts, step, f, fp;
    if (a.st.fk[px] < 0.0f) {
        ts = replay_t(r.t0, k, 0, vx);
        step = vx;
        f = a.st.fk[px];
        fp = a.st.fp[px];
    } else {
        const int j = a.st.j[px];
        if (j >= 2) a.st.fp[px] = __int_as_float(rval(gather_min(a.gathered, a.nrec, npx, px)));
        ts = replay_t(r.t0, k, j, vx);
        step = vx / 4.0f;
        f = a.st.fj[px];
        fp = a.st.fp[px];
    }
    *t_hit = ts + step * f / (fp - f);
    return true;
}

__global__ __launch_bounds__(256) void k_shard_render_final(ShardRayArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.width || y >= a.height) return;
    const int npx = a.width * a.height;
    const int px = y * a.width + x;
    const RayGeo r = shard_ray(a, x, y);
    float t;
    int2 rec = mk_rec(INT_MAX, 0);
    if (shard_resolve(a, r, px, npx, &t)) {
        a.st.t[px] = t;
        const float hx = fmaf(t, r.dx, r.ox), hy = fmaf(t, r.dy, r.oy), hz = fmaf(t, r.dz, r.oz);
        if (sample_owner(a.g, hz) == a.g.shard) {
            uint8_t b = 0, gch = 0, rr = 0;
            shade_hit(a.g, a.b, tri_setup(a.g, hx, hy, hz), a.kind, a.color_i32, a.palette, &b, &gch, &rr);
            rec = mk_rec(0, (int)((unsigned)b | ((unsigned)gch << 8) | ((unsigned)rr << 16)));
        }
    } else {
        a.st.t[px] = -1.0f;
        if (a.g.shard == 0) rec = mk_rec(0, 0);
    }
    a.send[px] = rec;
}

__global__ __launch_bounds__(256) void k_shard_render_finish(ShardRayArgs a) {
    const int npx = a.width * a.height;
    for (int px = blockIdx.x * blockDim.x + threadIdx.x; px < npx; px += gridDim.x * blockDim.x) {
        const unsigned v = (unsigned)rval(gather_min(a.gathered, a.nrec, npx, px));
        a.out_bgr[(size_t)px * 3 + 0] = (uint8_t)(v & 0xFF);
        a.out_bgr[(size_t)px * 3 + 1] = (uint8_t)((v >> 8) & 0xFF);
        a.out_bgr[(size_t)px * 3 + 2] = (uint8_t)((v >> 16) & 0xFF);
        if (a.out_t) a.out_t[px] = a.st.t[px];
    }
}

__global__ __launch_bounds__(256) void k_shard_assoc_partial(ShardRayArgs a) {
    __shared__ AssocLds s;
    assoc_lds_clear(s);
    __syncthreads();
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x < a.width && y < a.height) {
        const int npx = a.width * a.height;
        const int px = y * a.width + x;
        const RayGeo r = shard_ray(a, x, y);
        float t;
        float p[kMaxObjects];
#pragma unroll
        for (int k = 0; k < kMaxObjects; ++k) p[k] = 0.0f;
        bool mine;
        if (shard_resolve(a, r, px, npx, &t)) {
            const float hx = fmaf(t, r.dx, r.ox), hy = fmaf(t, r.dy, r.oy), hz = fmaf(t, r.dz, r.oz);
            mine = sample_owner(a.g, hz) == a.g.shard;
            if (mine) {
                tri_hist(a.g, a.b, tri_setup(a.g, hx, hy, hz), p);
            }
        } else {
            mine = a.g.shard == 0;  // pixels without a hit contribute once, from shard 0
        }
        if (mine) assoc_accumulate(s, p, a.mask[px], a.n_obs, a.eps, a.box_thresh);
    }
    __syncthreads();
    // partial layout: t1[32][32], t3[32][32], t2[32], c1[32], c2[32], c3[32][32] (int64); the
    // unused c1[0] word (label 0 has no row) carries the rank's largest positive t1 term
    // (pos_fix): the group's SUM of it bounds the largest term of the group from above
    unsigned long long* P = reinterpret_cast<unsigned long long*>(a.partial);
    if (threadIdx.x == 0 && s.pos) atomicMax(P + 2 * kMaxObjects * kMaxObjects + kMaxObjects, (unsigned long long)s.pos);
    const int NN = kMaxObjects * kMaxObjects;
    for (int k = threadIdx.x; k < NN; k += 256) {
        const long long v1 = (&s.t1[0][0])[k];
        if (v1) atomicAdd(P + k, (unsigned long long)v1);
        const long long v3 = (&s.t3[0][0])[k];
        if (v3) atomicAdd(P + NN + k, (unsigned long long)v3);
        const unsigned c3 = (&s.c3[0][0])[k];
        if (c3) atomicAdd(P + 2 * NN + 3 * kMaxObjects + k, (unsigned long long)c3);
    }
    if (threadIdx.x < kMaxObjects) {
        const int i = threadIdx.x;
        if (s.t2[i]) atomicAdd(P + 2 * NN + i, (unsigned long long)s.t2[i]);
        if (s.c1[i]) atomicAdd(P + 2 * NN + kMaxObjects + i, (unsigned long long)s.c1[i]);
        if (s.c2[i]) atomicAdd(P + 2 * NN + 2 * kMaxObjects + i, (unsigned long long)s.c2[i]);
    }
}

// The shard's part of the association's per-pixel data (AssocPixels layout in one buffer:
// uint2 bits [npx], then f32 p [32][npx]) for the decision's exact path: the owner of a pixel's
// hit writes its bits and its 32 counts, every other shard zeros (pixels without a hit: shard
// 0), so an int32 SUM over the shards is the single volume's data.
__global__ __launch_bounds__(256) void k_shard_assoc_pixels(ShardRayArgs a, int32_t* __restrict__ out) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.width || y >= a.height) return;
    const int npx = a.width * a.height;
    const int px = y * a.width + x;
    const RayGeo r = shard_ray(a, x, y);
    float t;
    float p[kMaxObjects];
#pragma unroll
    for (int k = 0; k < kMaxObjects; ++k) p[k] = 0.0f;
    bool mine;
    unsigned bins = 0;
    if (shard_resolve(a, r, px, npx, &t)) {
        const float hx = fmaf(t, r.dx, r.ox), hy = fmaf(t, r.dy, r.oy), hz = fmaf(t, r.dz, r.oz);
        mine = sample_owner(a.g, hz) == a.g.shard;
        if (mine) bins = tri_hist(a.g, a.b, tri_setup(a.g, hx, hy, hz), p);
    } else {
        mine = a.g.shard == 0;
    }
    unsigned pres = 0, box = 0;
#pragma unroll
    for (int j = 1; j < kMaxObjects; ++j) {
        if (((bins >> j) & 1u) && p[j] != 0.0f) pres |= 1u << j;
        if (p[j] > a.box_thresh) box |= 1u << j;
    }
    uint2* bits = reinterpret_cast<uint2*>(out);
    float* pp = reinterpret_cast<float*>(out + 2 * (size_t)npx);
    bits[px] = mine ? make_uint2(pres, box) : make_uint2(0u, 0u);
#pragma unroll
    for (int j = 0; j < kMaxObjects; ++j) pp[(size_t)j * npx + px] = mine ? p[j] : 0.0f;
}

hipError_t launch_shard_assoc_pixels(const ShardRayArgs& a, int32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_shard_assoc_pixels, dim3((a.width + 15) / 16, (a.height + 15) / 16), dim3(256), 0, s, a, out);
    return hipGetLastError();
}

__global__ void k_tables_from_partial(const long long* __restrict__ P, AssocTables* T) {
    const int NN = kMaxObjects * kMaxObjects;
    for (int k = threadIdx.x; k < NN; k += blockDim.x) {
        (&T->t1[0][0])[k] = P[k];
        (&T->t3[0][0])[k] = P[NN + k];
        (&T->c3[0][0])[k] = (unsigned)P[2 * NN + 3 * kMaxObjects + k];
    }
    if (threadIdx.x < kMaxObjects) {
        const int i = threadIdx.x;
        T->t2[i] = P[2 * NN + i];
        T->c1[i] = i ? (unsigned)P[2 * NN + kMaxObjects + i] : 0u;
        T->c2[i] = (unsigned)P[2 * NN + 2 * kMaxObjects + i];
    }
    if (threadIdx.x == 0) T->pos_max = (unsigned)min(P[2 * NN + kMaxObjects], 0xFFFFFFFFll);
}

static dim3 tile_grid(int w, int h) { return dim3((w + 15) / 16, (h + 15) / 16); }

hipError_t launch_shard_ray_step(const ShardRayArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_shard_ray_step, tile_grid(a.width, a.height), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_shard_render_final(const ShardRayArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_shard_render_final, tile_grid(a.width, a.height), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_shard_render_finish(const ShardRayArgs& a, hipStream_t s) {
    const int npx = a.width * a.height;
    int blocks = (npx + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_shard_render_finish, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_shard_assoc_partial(const ShardRayArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_shard_assoc_partial, tile_grid(a.width, a.height), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tables_from_partial(const long long* reduced, AssocTables* t, hipStream_t s) {
    hipLaunchKernelGGL(k_tables_from_partial, dim3(1), dim3(256), 0, s, reduced, t);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// histogram layout conversion (bin-major device <-> voxel-major reference export)
// ------------------------------------------------------------------------------------
// Bin mask of every stored voxel from the bin-major histogram (after an upload).
// Reference voxel v = (x * dimy + y) * lz + z (rows of lz planes) -> its tiled index.
__device__ __forceinline__ uint64_t tile_of_ref(const VolGeom& g, uint64_t v) {
    const uint64_t row = v / (uint64_t)g.lz;
    const int z = (int)(v - row * (uint64_t)g.lz);
    const int x = (int)(row / (uint64_t)g.dimy), y = (int)(row - (uint64_t)x * g.dimy);
    return tile_index(g, x, y, z);
}

__global__ __launch_bounds__(256) void k_hist_mask(VolGeom g, const uint32_t* __restrict__ hist,
                                                   uint32_t* __restrict__ hmask) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < g.nvox; v += (uint64_t)gridDim.x * blockDim.x) {
        unsigned m = 0;
        for (int k = 0; k < kMaxObjects; ++k) m |= (hist[(uint64_t)k * g.nvox + v] != 0u ? 1u : 0u) << k;
        hmask[v] = m;
    }
}

hipError_t launch_hist_mask(const VolGeom& g, const VolBufs& b, hipStream_t s) {
    if (!b.hist || !b.hmask || g.nvox == 0) return hipSuccess;
    uint64_t blocks = (g.nvox + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_hist_mask, dim3((unsigned)blocks), dim3(256), 0, s, g, b.hist, b.hmask);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_hist_to_vm(VolGeom g, const uint32_t* __restrict__ bm, uint32_t* __restrict__ vm,
                                                    uint64_t v0, uint64_t nv) {
    // vm is a chunk [nv][32] of logical voxels v0 .. v0+nv (rows of lz planes)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv * kMaxObjects;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = v0 + i / kMaxObjects, k = i % kMaxObjects;
        vm[i] = bm[k * g.nvox + tile_of_ref(g, v)];
    }
}

__global__ __launch_bounds__(256) void k_hist_to_bm(VolGeom g, const uint32_t* __restrict__ vm, uint32_t* __restrict__ bm,
                                                    uint64_t v0, uint64_t nv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv * kMaxObjects;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = i / nv, v = v0 + i % nv;
        bm[k * g.nvox + tile_of_ref(g, v)] = vm[(v - v0) * kMaxObjects + k];
    }
}

hipError_t launch_hist_chunk_to_vm(const uint32_t* bm, uint32_t* vm, const VolGeom& g, uint64_t v0, uint64_t nv,
                                   hipStream_t s) {
    uint64_t blocks = (nv * kMaxObjects + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_hist_to_vm, dim3((unsigned)blocks), dim3(256), 0, s, g, bm, vm, v0, nv);
    return hipGetLastError();
}

hipError_t launch_hist_chunk_to_bm(const uint32_t* vm, uint32_t* bm, const VolGeom& g, uint64_t v0, uint64_t nv,
                                   hipStream_t s) {
    uint64_t blocks = (nv * kMaxObjects + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_hist_to_bm, dim3((unsigned)blocks), dim3(256), 0, s, g, vm, bm, v0, nv);
    return hipGetLastError();
}

// 4-byte per-voxel arrays (sdf, weight, vote label/count): tiled device <-> reference rows
__global__ __launch_bounds__(256) void k_vox_to_ref(VolGeom g, const uint32_t* __restrict__ dev, uint32_t* __restrict__ ref,
                                                    uint64_t v0, uint64_t nv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * blockDim.x)
        ref[i] = dev[tile_of_ref(g, v0 + i)];
}

__global__ __launch_bounds__(256) void k_vox_from_ref(VolGeom g, const uint32_t* __restrict__ ref, uint32_t* __restrict__ dev,
                                                      uint64_t v0, uint64_t nv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * blockDim.x)
        dev[tile_of_ref(g, v0 + i)] = ref[i];
}

hipError_t launch_vox_chunk(const void* src, void* dst, bool to_ref, const VolGeom& g, uint64_t v0, uint64_t nv,
                            hipStream_t s) {
    uint64_t blocks = (nv + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    if (blocks == 0) return hipSuccess;
    if (to_ref)
        hipLaunchKernelGGL(k_vox_to_ref, dim3((unsigned)blocks), dim3(256), 0, s, g, (const uint32_t*)src, (uint32_t*)dst, v0, nv);
    else
        hipLaunchKernelGGL(k_vox_from_ref, dim3((unsigned)blocks), dim3(256), 0, s, g, (const uint32_t*)src, (uint32_t*)dst, v0, nv);
    return hipGetLastError();
}

// colour: device storage is padded to 4 channels (u8x4 / i32x4), the reference layout has 3
// TD: device storage element, TR: reference-layout element (int32 boundary of a COLOR_I32
// volume stored as bytes: values in [0, 255], checked by the host before an upload)
template <typename TD, typename TR>
__global__ __launch_bounds__(256) void k_color_to_ref(VolGeom g, const TD* __restrict__ dev, TR* __restrict__ ref,
                                                      uint64_t v0, uint64_t nv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv * 3; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = v0 + i / 3, c = i % 3;
        ref[i] = (TR)dev[tile_of_ref(g, v) * 4 + c];
    }
}

template <typename TD, typename TR>
__global__ __launch_bounds__(256) void k_color_from_ref(VolGeom g, const TR* __restrict__ ref, TD* __restrict__ dev,
                                                        uint64_t v0, uint64_t nv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv * 3; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = v0 + i / 3, c = i % 3;
        dev[tile_of_ref(g, v) * 4 + c] = (TD)ref[i];
    }
}

__global__ __launch_bounds__(256) void k_color_widen(const uint32_t* __restrict__ narrow, int4* __restrict__ wide,
                                                     uint64_t nvox) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvox; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = narrow[v];
        wide[v] = make_int4((int)(c & 0xFFu), (int)((c >> 8) & 0xFFu), (int)((c >> 16) & 0xFFu), 0);
    }
}

hipError_t launch_color_widen(const uint8_t* narrow, int32_t* wide, uint64_t nvox, hipStream_t s) {
    if (nvox == 0) return hipSuccess;
    uint64_t blocks = (nvox + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_color_widen, dim3((unsigned)blocks), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(narrow),
                       reinterpret_cast<int4*>(wide), nvox);
    return hipGetLastError();
}

template <typename TD, typename TR>
static void color_chunk_t(const void* src, void* dst, bool to_ref, const VolGeom& g, uint64_t v0, uint64_t nv,
                          dim3 gr, hipStream_t s) {
    if (to_ref)
        hipLaunchKernelGGL((k_color_to_ref<TD, TR>), gr, dim3(256), 0, s, g, (const TD*)src, (TR*)dst, v0, nv);
    else
        hipLaunchKernelGGL((k_color_from_ref<TD, TR>), gr, dim3(256), 0, s, g, (const TR*)src, (TD*)dst, v0, nv);
}

hipError_t launch_color_chunk(const void* src, void* dst, bool to_ref, bool ref_i32, bool dev_i32, const VolGeom& g,
                              uint64_t v0, uint64_t nv, hipStream_t s) {
    uint64_t blocks = (nv * 3 + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    const dim3 gr((unsigned)blocks);
    if (dev_i32)
        color_chunk_t<int32_t, int32_t>(src, dst, to_ref, g, v0, nv, gr, s);
    else if (ref_i32)
        color_chunk_t<uint8_t, int32_t>(src, dst, to_ref, g, v0, nv, gr, s);
    else
        color_chunk_t<uint8_t, uint8_t>(src, dst, to_ref, g, v0, nv, gr, s);
    return hipGetLastError();
}


// ------------------------------------------------------------------------------------
// Mask R-CNN detections -> instance-label mask (the fusion's mask input contract,
// Mask_RCNN/dmask.py:34-59 mask_detect without its optional depth filter):
//   filter_tiny_objects (dmask.py:34-45): keep detection i when its area > min_area;
//   preserve_small_objs (dmask.py:21-32): over the kept detections sorted by area, each
//     smaller one removes its pixels from every larger one, i.e. a pixel belongs to the
//     smallest kept detection containing it (equal areas: the lower detection index, the
//     stable order; NumPy's argsort leaves ties in an implementation-defined order);
//   cls[masks[:, :, i]] = i + 1 (dmask.py:56-58), i = index among the kept detections.
// Three passes over the detector's [H][W][N] byte masks: areas (wave ballots, LDS then
// global sums), the per-detection keep/rank/label decision (one workgroup), and labels.
// ------------------------------------------------------------------------------------
struct MaskScratch {
    unsigned area[kMaxDetections];
    unsigned short rank[kMaxDetections];  // order among the kept detections by (area, index); 0xFFFF dropped
    unsigned char label[kMaxDetections];  // 1 + index among the kept detections
    unsigned n_kept;
};

__global__ __launch_bounds__(256) void k_mask_areas(const uint8_t* __restrict__ masks, int npx, int n,
                                                     MaskScratch* __restrict__ sc) {
    __shared__ unsigned s_area[kMaxDetections];
    for (int i = threadIdx.x; i < n; i += blockDim.x) s_area[i] = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int base = blockIdx.x * blockDim.x; base < npx; base += gridDim.x * blockDim.x) {
        const int p = base + (int)threadIdx.x;
        const uint8_t* row = masks + (size_t)p * n;
        for (int i = 0; i < n; ++i) {
            const bool on = p < npx && row[i] != 0;
            const unsigned c = (unsigned)__popcll(__ballot(on));
            if (lane == 0 && c) atomicAdd(&s_area[i], c);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (s_area[i]) atomicAdd(&sc->area[i], s_area[i]);
}

__global__ __launch_bounds__(256) void k_mask_decide(MaskScratch* __restrict__ sc, int n, int min_area) {
    const int i = threadIdx.x;
    __shared__ unsigned s_area[kMaxDetections];
    __shared__ unsigned char s_keep[kMaxDetections];
    if (i < n) {
        s_area[i] = sc->area[i];
        s_keep[i] = (long long)sc->area[i] > (long long)min_area ? 1 : 0;
    }
    __syncthreads();
    if (i < n) {
        unsigned rank = 0, before = 0;
        for (int j = 0; j < n; ++j) {
            if (!s_keep[j]) continue;
            rank += (s_area[j] < s_area[i] || (s_area[j] == s_area[i] && j < i)) ? 1u : 0u;
            before += j < i ? 1u : 0u;
        }
        sc->rank[i] = s_keep[i] ? (unsigned short)rank : (unsigned short)0xFFFF;
        sc->label[i] = (unsigned char)(before + 1);  // uint8 label (dmask.py:56), wraps as the reference's
    }
    if (i == 0) {
        unsigned k = 0;
        for (int j = 0; j < n; ++j) k += s_keep[j];
        sc->n_kept = k;
    }
}

__global__ __launch_bounds__(256) void k_mask_labels(const uint8_t* __restrict__ masks, int npx, int n,
                                                      const MaskScratch* __restrict__ sc, uint8_t* __restrict__ out) {
    __shared__ unsigned short s_rank[kMaxDetections];
    __shared__ unsigned char s_label[kMaxDetections];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        s_rank[i] = sc->rank[i];
        s_label[i] = sc->label[i];
    }
    __syncthreads();
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < npx; p += gridDim.x * blockDim.x) {
        const uint8_t* row = masks + (size_t)p * n;
        unsigned best = 0xFFFFu;
        unsigned char lab = 0;
        for (int i = 0; i < n; ++i) {
            const unsigned r = row[i] ? s_rank[i] : 0xFFFFu;
            if (r < best) {
                best = r;
                lab = s_label[i];
            }
        }
        out[p] = lab;
    }
}

hipError_t launch_masks_to_labels(const uint8_t* masks, int npx, int n, int min_area, void* scratch, uint8_t* out,
                                  hipStream_t s) {
    MaskScratch* sc = (MaskScratch*)scratch;
    hipError_t e = hipMemsetAsync(sc, 0, sizeof(MaskScratch), s);
    if (e != hipSuccess) return e;
    int blocks = (npx + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    if (n > 0) hipLaunchKernelGGL(k_mask_areas, dim3(blocks), dim3(256), 0, s, masks, npx, n, sc);
    hipLaunchKernelGGL(k_mask_decide, dim3(1), dim3(kMaxDetections), 0, s, sc, n, min_area);
    hipLaunchKernelGGL(k_mask_labels, dim3(blocks), dim3(256), 0, s, masks, npx, n, (const MaskScratch*)sc, out);
    return hipGetLastError();
}

size_t mask_scratch_bytes() { return sizeof(MaskScratch); }
size_t mask_scratch_kept_offset() { return offsetof(MaskScratch, n_kept); }



// ------------------------------------------------------------------------------------
// Surface export (optional in the reference: the volume layout of
// src/TSDF_Python/tsdf.py:48-52): every stored, owned voxel with weight >= min_w and |sdf| <
// sdf_max, with its colour and instance label (the argmax of its histogram, first maximum,
// as the label render's viewer.cu:66-79 rule applied to the voxel itself; 0 when empty).
// Unordered appends (the host sorts by the reference index); a counting pass when out is null.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_export_surface(VolGeom g, VolBufs b, float sdf_max, int min_w, int color_wide,
                                                        int semantic, SurfacePoint* __restrict__ out, uint64_t cap,
                                                        unsigned long long* __restrict__ count) {
    const uint64_t n = (uint64_t)g.dimx * (uint64_t)g.dimy * (uint64_t)g.lz;
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = v / (uint64_t)g.lz;
        const int l = (int)(v - row * (uint64_t)g.lz);
        const int x = (int)(row / (uint64_t)g.dimy), y = (int)(row - (uint64_t)x * g.dimy);
        if (g.nshards > 1 && (l % (g.chunk + g.halo)) >= g.chunk) continue;  // halo plane: its owner exports it
        const int gz = local_to_global_z(g, l);
        if (gz >= g.dimz) continue;
        const uint32_t t = tile_index(g, x, y, l);
        const int w = b.wt[t];
        const float s = b.sdf[t];
        if (w < min_w || !(fabsf(s) < sdf_max)) continue;
        unsigned r, gg, bb;
        if (color_wide) {
            const int4 c = reinterpret_cast<const int4*>(b.color)[t];
            r = (unsigned)min(max(c.x, 0), 255); gg = (unsigned)min(max(c.y, 0), 255); bb = (unsigned)min(max(c.z, 0), 255);
        } else {
            const unsigned c = reinterpret_cast<const uint32_t*>(b.color)[t];
            r = c & 0xFFu; gg = (c >> 8) & 0xFFu; bb = (c >> 16) & 0xFFu;
        }
        unsigned lab = 0, best = 0;
        if (semantic) {
            unsigned bins = b.hmask[t];
            while (bins) {
                const int k = __ffs((int)bins) - 1;
                bins &= bins - 1u;
                const unsigned c = b.hist[(uint64_t)k * g.nvox + t];
                if (c > best) { best = c; lab = (unsigned)k; }
            }
        }
        const unsigned long long i = atomicAdd(count, 1ull);
        if (out && i < cap) {
            SurfacePoint p;
            p.x = (uint32_t)x; p.y = (uint32_t)y; p.z = (uint32_t)gz;
            p.sdf = s;
            p.rgbl = r | (gg << 8) | (bb << 16) | (lab << 24);
            out[i] = p;
        }
    }
}

hipError_t launch_export_surface(const VolGeom& g, const VolBufs& b, float sdf_max, int min_w, int color_wide,
                                 int semantic, SurfacePoint* out, uint64_t cap, unsigned long long* count, hipStream_t s) {
    const uint64_t n = (uint64_t)g.dimx * g.dimy * g.lz;
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_export_surface, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, g, b, sdf_max,
                       min_w, color_wide, semantic, out, cap, count);
    return hipGetLastError();
}

}  // namespace semtsdf
