// Calibration microbenchmark (not part of the product): access patterns of k_integrate with a
// known byte count, so that rocprofv3's FETCH_SIZE / WRITE_SIZE can be read as bytes for each
// pattern (MI355X_MICROARCH.md §HBM: FETCH_SIZE is validated only for 16-B/lane streaming reads).
// Every kernel is a separate dispatch with its own name; tools/calib_summary.py joins the PMC
// rows with the known bytes this program prints.
//
//   k_read16        16-B/lane streaming read of 512 MiB                    known read 512 MiB
//   k_read8         8-B/lane streaming read of 512 MiB                     known read 512 MiB
//   k_read4         4-B/lane streaming read of 512 MiB                     known read 512 MiB
//   k_rmw16         the integrate's state RMW: 512-B half-tile units of sdf + weight, 16 B per
//                   lane, default-policy loads, non-temporal stores (SEMTSDF_NT_LOAD 0 / _STORE 1),
//                   two units per wave-iteration, over a live set in the cull's x-run order
//                                                                           known read = write = units x 1 KiB
//   k_gather8_lines one 8-B load per distinct 128-B line of a 512 MiB array, lines in a scrambled
//                   order (each line once)                                  4 M lines: 256 MiB at 64 B, 512 MiB at 128 B
//   k_gather8_rec   the integrate's pixel-record gathers: 4 x 8-B loads per lane from a 2.4 MB
//                   record image (640x480 + zero row/column) per unit of the same live set
//                   (unique bytes 2.46 MB; each XCD's L2 misses at most that once)
//   k_rmw16_tile    k_rmw16 with sdf and weight interleaved per 1-KiB tile (layout probe, timing)
//   k_rmw16_unit    k_rmw16 with sdf and weight interleaved per 512-B unit (layout probe, timing)
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench_calib.hip -o build/membench_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                   \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int D = 512;
constexpr size_t NVOX = (size_t)D * D * D;
constexpr int NUY = D / 8, NUZ = D / 16;  // units of 1 x 8 x 16 voxels = 128 voxels = 512 B
constexpr int W = 640, H = 480;
constexpr size_t NREC = (size_t)(W + 1) * (H + 1);

__host__ __device__ inline size_t unit_base(unsigned u) {
    const unsigned x = u & 4095u, uy = (u >> 12) & 1023u, uz = u >> 22;
    return ((size_t)x * NUY * NUZ + (size_t)uy * NUZ + uz) * 128u;
}

__global__ __launch_bounds__(256) void k_read16(const f4* __restrict__ a, float* __restrict__ out, size_t n4) {
    f4 s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256u) s += a[i];
    if (s.x + s.y + s.z + s.w == 1234.5f) out[0] = s.x;
}
__global__ __launch_bounds__(256) void k_read8(const f2* __restrict__ a, float* __restrict__ out, size_t n2) {
    f2 s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256u) s += a[i];
    if (s.x + s.y == 1234.5f) out[0] = s.x;
}
__global__ __launch_bounds__(256) void k_read4(const float* __restrict__ a, float* __restrict__ out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) s += a[i];
    if (s == 1234.5f) out[0] = s;
}

// sdf / weight element offsets of voxel v of a unit under three layouts
template <int L>
__device__ inline size_t off_sdf(size_t v) {
    if (L == 0) return v;
    if (L == 1) return v + (v & ~(size_t)255);  // per 1-KiB tile: sdf tile, then weight tile
    return v + (v & ~(size_t)127);              // per 512-B unit
}
template <int L>
__device__ inline size_t off_wt(size_t v) {
    if (L == 0) return v;
    if (L == 1) return v + (v & ~(size_t)255) + 256;
    return v + (v & ~(size_t)127) + 128;
}

template <int L>
__device__ inline void rmw_body(float* __restrict__ sdf, int* __restrict__ wt, const unsigned* __restrict__ list,
                                unsigned n) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const unsigned nw = gridDim.x * 4u;
    for (unsigned g = wave; 2u * g < n; g += nw) {
        const unsigned i = 2u * g + (lane >> 5);
        if (i >= n) continue;
        const size_t v = unit_base(list[i]) + (lane & 31u) * 4u;
        f4 s = *reinterpret_cast<const f4*>(sdf + off_sdf<L>(v));
        i4 w = *reinterpret_cast<const i4*>(wt + off_wt<L>(v));
        s += 1.f;
        w += 1;
        __builtin_nontemporal_store(s, reinterpret_cast<f4*>(sdf + off_sdf<L>(v)));
        __builtin_nontemporal_store(w, reinterpret_cast<i4*>(wt + off_wt<L>(v)));
    }
}
__global__ __launch_bounds__(256) void k_rmw16(float* sdf, int* wt, const unsigned* list, unsigned n) {
    rmw_body<0>(sdf, wt, list, n);
}
__global__ __launch_bounds__(256) void k_rmw16_tile(float* sdf, int* wt, const unsigned* list, unsigned n) {
    rmw_body<1>(sdf, reinterpret_cast<int*>(sdf), list, n);
}
__global__ __launch_bounds__(256) void k_rmw16_unit(float* sdf, int* wt, const unsigned* list, unsigned n) {
    rmw_body<2>(sdf, reinterpret_cast<int*>(sdf), list, n);
}

// one 8-B load per 128-B line, line index scrambled by an odd multiplier (a bijection mod 2^k)
__global__ __launch_bounds__(256) void k_gather8_lines(const uint2* __restrict__ a, unsigned* __restrict__ out,
                                                        unsigned nlines_log2) {
    const unsigned nl = 1u << nlines_log2;
    unsigned acc = 0;
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < nl; i += gridDim.x * 256u) {
        const unsigned l = (i * 2654435761u) & (nl - 1u);
        const uint2 r = a[(size_t)l * 16u + (i & 15u)];
        acc += r.x ^ r.y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// pixel-record gathers of the integrate: per unit, each lane 4 records around a projected pixel
// (a smooth function of the unit and lane, like a camera's screen map)
__global__ __launch_bounds__(256) void k_gather8_rec(const uint2* __restrict__ rec, const unsigned* __restrict__ list,
                                                      unsigned n, unsigned* __restrict__ out) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const unsigned nw = gridDim.x * 4u;
    unsigned acc = 0;
    for (unsigned g = wave; 2u * g < n; g += nw) {
        const unsigned i = 2u * g + (lane >> 5);
        if (i >= n) continue;
        const unsigned u = list[i];
        const unsigned x = u & 4095u, uy = (u >> 12) & 1023u, uz = u >> 22;
        const unsigned y = uy * 8u + ((lane >> 2) & 7u);
        const float z = 1.0f + 0.01f * (float)(uz * 16u + (lane & 3u) * 4u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float zk = z + 0.01f * (float)k;
            const unsigned px = min((unsigned)(320.0f + ((float)x - 256.0f) * 1.2f / zk), (unsigned)W);
            const unsigned py = min((unsigned)(240.0f + ((float)y - 256.0f) * 1.2f / zk), (unsigned)H);
            const uint2 r = rec[(size_t)py * (W + 1) + px];
            acc += r.x ^ r.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

static unsigned pack(unsigned x, unsigned uy, unsigned uz) { return x | (uy << 12) | (uz << 22); }

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    float *sdf, *wt, *out;
    uint2* rec;
    CK(hipMalloc(&sdf, NVOX * 4 * 2));  // room for the interleaved layouts
    CK(hipMalloc(&wt, NVOX * 4));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&rec, NREC * 8));
    CK(hipMemset(sdf, 0, NVOX * 8));
    CK(hipMemset(wt, 0, NVOX * 4));
    CK(hipMemset(rec, 1, NREC * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned> box;  // about a 512^3 frame's live units, in the cull's x-run order
    for (unsigned uz = 4; uz < 12; ++uz)
        for (unsigned uy = 8; uy < 56; ++uy)
            for (unsigned x = 64; x < 448; ++x) box.push_back(pack(x, uy, uz));
    unsigned* dl;
    CK(hipMalloc(&dl, box.size() * 4));
    CK(hipMemcpy(dl, box.data(), box.size() * 4, hipMemcpyHostToDevice));
    const unsigned nu = (unsigned)box.size();
    const double unit_rw = (double)nu * 1024.0;  // sdf + weight bytes read (= written)
    const size_t half = NVOX * 4;                // 512 MiB
    auto timeit = [&](const char* name, double kr, double kw, auto launch) {
        float best = 1e9f, ms;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        printf("{\"kernel\": \"%s\", \"known_read\": %.0f, \"known_write\": %.0f, \"us\": %.2f, \"gbs\": %.1f}\n", name, kr,
               kw, best * 1e3, (kr + kw) / best / 1e6);
        fflush(stdout);
    };
    const int G = 4096;
    timeit("k_read16", (double)half, 0, [&] { hipLaunchKernelGGL(k_read16, dim3(G), dim3(256), 0, 0, (const f4*)sdf, out, half / 16); });
    timeit("k_read8", (double)half, 0, [&] { hipLaunchKernelGGL(k_read8, dim3(G), dim3(256), 0, 0, (const f2*)sdf, out, half / 8); });
    timeit("k_read4", (double)half, 0, [&] { hipLaunchKernelGGL(k_read4, dim3(G), dim3(256), 0, 0, (const float*)sdf, out, half / 4); });
    timeit("k_rmw16", unit_rw, unit_rw, [&] { hipLaunchKernelGGL(k_rmw16, dim3(2048), dim3(256), 0, 0, sdf, (int*)wt, dl, nu); });
    timeit("k_rmw16_tile", unit_rw, unit_rw, [&] { hipLaunchKernelGGL(k_rmw16_tile, dim3(2048), dim3(256), 0, 0, sdf, (int*)wt, dl, nu); });
    timeit("k_rmw16_unit", unit_rw, unit_rw, [&] { hipLaunchKernelGGL(k_rmw16_unit, dim3(2048), dim3(256), 0, 0, sdf, (int*)wt, dl, nu); });
    // 2^22 lines of 128 B = 512 MiB; known_read printed at 128 B per line (the summary also gives the 64-B reading)
    timeit("k_gather8_lines", (double)(1u << 22) * 128.0, 0,
           [&] { hipLaunchKernelGGL(k_gather8_lines, dim3(G), dim3(256), 0, 0, (const uint2*)sdf, (unsigned*)out, 22u); });
    timeit("k_gather8_rec", (double)NREC * 8.0, 0,
           [&] { hipLaunchKernelGGL(k_gather8_rec, dim3(2048), dim3(256), 0, 0, (const uint2*)rec, dl, nu, (unsigned*)out); });
    CK(hipDeviceSynchronize());
    return 0;
}
