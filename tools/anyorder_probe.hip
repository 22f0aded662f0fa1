// Probe (not part of the product): does hipExtLaunchKernel's hipExtAnyOrderLaunch flag let a kernel
// start before the previous kernel of the same stream has finished on this device?  A spin kernel on
// 8 workgroups (most CUs idle) is followed on the same stream by a marker kernel, launched with flags 0
// and 1; each records s_memrealtime (100 MHz) at its start / end.
// Build: hipcc --offload-arch=gfx950 -O3 tools/anyorder_probe.hip -o build/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                       \
    do {                                                            \
        hipError_t e = (x);                                         \
        if (e != hipSuccess) {                                      \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                \
        }                                                           \
    } while (0)

__global__ void k_spin(unsigned long long* t, unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        t[0] = t0;
        t[1] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ void k_mark(unsigned long long* t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t[2] = __builtin_amdgcn_s_memrealtime();
}

int main() {
    unsigned long long* t;
    CK(hipMalloc(&t, 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int flags = 0; flags <= 1; ++flags) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemsetAsync(t, 0, 64, s));
            hipLaunchKernelGGL(k_spin, dim3(8), dim3(64), 0, s, t, 20000ull);  // 200 us
            void* args[] = {&t};
            CK(hipExtLaunchKernel((const void*)k_mark, dim3(1), dim3(64), args, 0, s, nullptr, nullptr, flags));
            CK(hipStreamSynchronize(s));
            unsigned long long h[3];
            CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
            const double spin_us = (double)(h[1] - h[0]) / 100.0, mark_us = ((double)h[2] - (double)h[1]) / 100.0;
            printf("flags %d: spin %.1f us, marker start %+.1f us after the spin's end (%s)\n", flags, spin_us, mark_us,
                   mark_us < 0 ? "overlapped" : "ordered");
        }
    }
    return 0;
}
