// Microbenchmark (not part of the product): read-modify-write of the integrate's 512-B
// half-tile units (sdf f32 + weight i32, 16 B per lane, two units per wave-iteration, like
// k_integrate) over a live set of units, in three list orders:
//   xrun    x fastest (the cull grid's order today: consecutive units 1 MiB apart at 512^3)
//   zrun    z fastest (consecutive units adjacent in memory)
//   random  shuffled
// Reports GB/s of (sdf + weight) r+w bytes.  Build: hipcc --offload-arch=gfx950 -O3 tools/membench_units.hip -o tools/membench_units
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
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
constexpr int D = 512;
constexpr int NUX = D, NUY = D / 8, NUZ = D / 16;  // units of 1 x 8 x 16 voxels = 128 voxels = 512 B

// unit (x, uy, uz) -> first float of its 512-B chunk in the tiled layout (x slowest, then y tile, then z)
__host__ __device__ inline size_t unit_base(unsigned u) {
    const unsigned x = u & 4095u, uy = (u >> 12) & 1023u, uz = u >> 22;
    return ((size_t)x * NUY * NUZ + (size_t)uy * NUZ + uz) * 128u;
}

__global__ __launch_bounds__(256) void k_rmw(float* __restrict__ sdf, int* __restrict__ wt, const unsigned* __restrict__ list,
                                             unsigned n) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const unsigned nw = gridDim.x * 4u;
    for (unsigned g = wave; 2u * g < n; g += nw) {
        const unsigned i = 2u * g + (lane >> 5);
        if (i >= n) continue;
        const size_t v = unit_base(list[i]) + (lane & 31u) * 4u;
        f4 s = __builtin_nontemporal_load(reinterpret_cast<f4*>(sdf + v));
        i4 w = __builtin_nontemporal_load(reinterpret_cast<i4*>(wt + v));
        s += 1.f;
        w += 1;
        __builtin_nontemporal_store(s, reinterpret_cast<f4*>(sdf + v));
        __builtin_nontemporal_store(w, reinterpret_cast<i4*>(wt + v));
    }
}

static unsigned pack(unsigned x, unsigned uy, unsigned uz) { return x | (uy << 12) | (uz << 22); }

int main() {
    const size_t N = (size_t)D * D * D;
    float* sdf;
    int* wt;
    CK(hipMalloc(&sdf, N * 4));
    CK(hipMalloc(&wt, N * 4));
    CK(hipMemset(sdf, 0, N * 4));
    CK(hipMemset(wt, 0, N * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // the live set: a box of units (about the 512^3 frame's 180 k live units)
    std::vector<unsigned> box;
    for (unsigned uz = 4; uz < 12; ++uz)
        for (unsigned uy = 8; uy < 56; ++uy)
            for (unsigned x = 64; x < 448; ++x) box.push_back(pack(x, uy, uz));
    const double bytes = (double)box.size() * 512.0 * 4.0;  // sdf + weight, read + write
    for (int order = 0; order < 3; ++order) {
        std::vector<unsigned> list = box;  // xrun: x fastest as built
        if (order == 1) std::sort(list.begin(), list.end(), [](unsigned a, unsigned b) { return unit_base(a) < unit_base(b); });
        if (order == 2) std::shuffle(list.begin(), list.end(), std::mt19937(1));
        unsigned* dl;
        CK(hipMalloc(&dl, list.size() * 4));
        CK(hipMemcpy(dl, list.data(), list.size() * 4, hipMemcpyHostToDevice));
        for (int grid : {1024, 2048, 4096}) {
            float best = 1e9f, ms;
            for (int r = 0; r < 6; ++r) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_rmw, dim3(grid), dim3(256), 0, 0, sdf, wt, dl, (unsigned)list.size());
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            printf("order %-6s grid %4d: %zu units %.1f MB  %.1f us  %.0f GB/s\n",
                   order == 0 ? "xrun" : order == 1 ? "zrun" : "random", grid, list.size(), bytes / 1e6, best * 1e3,
                   bytes / best / 1e6);
        }
        CK(hipFree(dl));
    }
    return 0;
}
