// Copy-bandwidth variants (tools only, not the product): which float4 copy shape reaches
// the achievable HBM rate on this box.  hipcc --offload-arch=gfx950 -O3 tools/copybench.hip -o tools/copybench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_stride(const f32x4* __restrict__ a, f32x4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        f32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = NTL ? __builtin_nontemporal_load(a + i + k * stride) : a[i + k * stride];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (NTS) __builtin_nontemporal_store(v[k], b + i + k * stride);
            else b[i + k * stride] = v[k];
        }
    }
    for (; i < n; i += stride) b[i] = a[i];
}

// each block copies contiguous tiles of 256*U float4 (one tile per iteration)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_tile(const f32x4* __restrict__ a, f32x4* __restrict__ b, size_t n) {
    const size_t tile = 256 * U;
    for (size_t t0 = (size_t)blockIdx.x * tile; t0 < n; t0 += (size_t)gridDim.x * tile) {
        f32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const size_t i = t0 + k * 256 + threadIdx.x;
            v[k] = i < n ? (NT ? __builtin_nontemporal_load(a + i) : a[i]) : f32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const size_t i = t0 + k * 256 + threadIdx.x;
            if (i < n) { if (NT) __builtin_nontemporal_store(v[k], b + i); else b[i] = v[k]; }
        }
    }
}

__global__ __launch_bounds__(256) void k_read(const f32x4* __restrict__ a, float* out, size_t n) {
    f32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;
}

template <class F>
static double timeit(F f, double bytes) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(e0)); f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
    }
    return bytes / (best * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? (size_t)atoll(argv[1]) : (1ull << 30));
    const size_t n = bytes / 16;
    f32x4 *a, *b; float* o;
    CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&o, 4));
    CK(hipMemset(a, 1, bytes)); CK(hipMemset(b, 0, bytes));
    int cus = 256; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double cb = 2.0 * bytes;
    printf("bytes %zu cus %d\n", bytes, cus);
    for (int bpc : {4, 8, 16, 32}) {
        const unsigned g = cus * bpc;
        printf("stride U4 NT/NT  bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_stride<4, true, true><<<g, 256>>>(a, b, n); }, cb));
        printf("stride U4 pl/pl  bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_stride<4, false, false><<<g, 256>>>(a, b, n); }, cb));
        printf("stride U4 NT/pl  bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_stride<4, true, false><<<g, 256>>>(a, b, n); }, cb));
        printf("stride U1 pl/pl  bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_stride<1, false, false><<<g, 256>>>(a, b, n); }, cb));
        printf("tile   U4 pl     bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_tile<4, false><<<g, 256>>>(a, b, n); }, cb));
        printf("tile   U4 NT     bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_tile<4, true><<<g, 256>>>(a, b, n); }, cb));
        printf("tile   U8 pl     bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_tile<8, false><<<g, 256>>>(a, b, n); }, cb));
        printf("read             bpc %2d %7.0f GB/s\n", bpc, timeit([&] { k_read<<<g, 256>>>(a, o, n); }, (double)bytes));
    }
    const unsigned gall = (unsigned)((n + 255) / 256);
    printf("one-shot pl      %7.0f GB/s\n", timeit([&] { k_stride<1, false, false><<<gall, 256>>>(a, b, n); }, cb));
    return 0;
}
