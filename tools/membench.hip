// Microbenchmark of the volume read-modify-write access patterns (not part of the product).
// hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int D = 512;

__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// brick RMW, 4 B per lane: lanes (z: tid&31, y: tid>>5), brick 8x8x32, x loop of 8
__global__ void k_rmw_b4(float* sdf, int* wt, const unsigned* list, unsigned n) {
    for (unsigned it = blockIdx.x; it < n; it += gridDim.x) {
        const unsigned b = list[it];
        const int bx = b % (D / 8), by = (b / (D / 8)) % (D / 8), bz = b / ((D / 8) * (D / 8));
        const int z = bz * 32 + (threadIdx.x & 31), y = by * 8 + (threadIdx.x >> 5);
        float s[8]; int w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const size_t v = ((size_t)(bx * 8 + i) * D + y) * D + z;
            s[i] = sdf[v]; w[i] = wt[v];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const size_t v = ((size_t)(bx * 8 + i) * D + y) * D + z;
            sdf[v] = s[i] * 0.5f + 1.0f; wt[v] = w[i] + 1;
        }
    }
}

// brick RMW, 16 B per lane: lanes (zq: tid&7 -> z = 4 zq, y: (tid>>3)&7, x: tid>>6), brick 8x8x32, x loop of 2
__global__ void k_rmw_b16(float* sdf, int* wt, const unsigned* list, unsigned n) {
    for (unsigned it = blockIdx.x; it < n; it += gridDim.x) {
        const unsigned b = list[it];
        const int bx = b % (D / 8), by = (b / (D / 8)) % (D / 8), bz = b / ((D / 8) * (D / 8));
        const int z = bz * 32 + (threadIdx.x & 7) * 4, y = by * 8 + ((threadIdx.x >> 3) & 7);
        const int xl = threadIdx.x >> 6;
        float4 s[2]; int4 w[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const size_t v = ((size_t)(bx * 8 + xl + 4 * i) * D + y) * D + z;
            s[i] = *(float4*)(sdf + v); w[i] = *(int4*)(wt + v);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const size_t v = ((size_t)(bx * 8 + xl + 4 * i) * D + y) * D + z;
            s[i].x += 1.f; s[i].y += 1.f; s[i].z += 1.f; s[i].w += 1.f;
            w[i].x += 1; w[i].y += 1; w[i].z += 1; w[i].w += 1;
            *(float4*)(sdf + v) = s[i]; *(int4*)(wt + v) = w[i];
        }
    }
}

// long-z RMW: brick 2x2x256, 16 B per lane, each wave one row of 256 z
__global__ void k_rmw_row(float* sdf, int* wt, const unsigned* list, unsigned n) {
    for (unsigned it = blockIdx.x; it < n; it += gridDim.x) {
        const unsigned b = list[it];  // brick id over (D/2, D/2, D/256)
        const int bx = b % (D / 2), by = (b / (D / 2)) % (D / 2), bz = b / ((D / 2) * (D / 2));
        const int wv = threadIdx.x >> 6;
        const int x = bx * 2 + (wv & 1), y = by * 2 + (wv >> 1);
        const int z = bz * 256 + (threadIdx.x & 63) * 4;
        const size_t v = ((size_t)x * D + y) * D + z;
        float4 s = *(float4*)(sdf + v); int4 w = *(int4*)(wt + v);
        s.x += 1.f; s.y += 1.f; s.z += 1.f; s.w += 1.f;
        w.x += 1; w.y += 1; w.z += 1; w.w += 1;
        *(float4*)(sdf + v) = s; *(int4*)(wt + v) = w;
    }
}

int main() {
    const size_t N = (size_t)D * D * D;
    float* sdf; int* wt; float4* c0; float4* c1;
    CK(hipMalloc(&sdf, N * 4)); CK(hipMalloc(&wt, N * 4));
    CK(hipMemset(sdf, 0, N * 4)); CK(hipMemset(wt, 0, N * 4));
    const size_t NC = (size_t)1 << 28;  // 1 GiB copy
    CK(hipMalloc(&c0, NC)); CK(hipMalloc(&c1, NC)); CK(hipMemset(c0, 0, NC));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms;
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0)); hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, c0, c1, NC / 16); CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("copy 1 GiB: %.3f ms  %.0f GB/s (r+w)\n", ms, 2.0 * NC / ms / 1e6);
    // brick lists: a contiguous z-slab region with fraction f of bricks (like the live set ~22%)
    for (int variant = 0; variant < 3; ++variant) {
        std::vector<unsigned> list;
        const int nbx = variant == 2 ? D / 2 : D / 8, nby = nbx, nbz = variant == 2 ? D / 256 : D / 32;
        for (int bz = 0; bz < nbz; ++bz) for (int by = 0; by < nby; ++by) for (int bx = 0; bx < nbx; ++bx)
            list.push_back(bx + nbx * (by + nby * bz));
        std::mt19937 rng(1);
        std::shuffle(list.begin(), list.end(), rng);
        list.resize(list.size() / 4);  // 25 % of the volume, random bricks
        unsigned* dl; CK(hipMalloc(&dl, list.size() * 4));
        CK(hipMemcpy(dl, list.data(), list.size() * 4, hipMemcpyHostToDevice));
        const double bytes = (double)list.size() * (variant == 2 ? 1024 : 2048) * 16.0;  // r+w sdf+wt
        for (int grid : {1024, 2048, 4096}) {
            float best = 1e9;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0));
                if (variant == 0) hipLaunchKernelGGL(k_rmw_b4, dim3(grid), dim3(256), 0, 0, sdf, wt, dl, (unsigned)list.size());
                if (variant == 1) hipLaunchKernelGGL(k_rmw_b16, dim3(grid), dim3(256), 0, 0, sdf, wt, dl, (unsigned)list.size());
                if (variant == 2) hipLaunchKernelGGL(k_rmw_row, dim3(grid), dim3(256), 0, 0, sdf, wt, dl, (unsigned)list.size());
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            printf("variant %d (%s) grid %d: %zu bricks %.1f MB %.3f ms %.0f GB/s\n", variant,
                   variant == 0 ? "8x8x32 4B/lane" : variant == 1 ? "8x8x32 16B/lane" : "2x2x256 16B/lane", grid,
                   list.size(), bytes / 1e6, best, bytes / best / 1e6);
        }
        CK(hipFree(dl));
    }
    return 0;
}
