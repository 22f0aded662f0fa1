// Gap between back-to-back kernels on one stream against the dirty data the first leaves in
// L2: each launch spins ~40 us, then stores `mb` MB (plain, nontemporal, or none); the last
// wave's end and the next launch's first wave start are taken with wall_clock64 on the device
// (atomicMax / atomicMin per launch), so the gap is the time the GPU spends between them.
// hipcc --offload-arch=gfx950 -O2 tools/flush_gap.hip -o build/flush_gap && build/flush_gap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void work(unsigned long long ticks, float4* buf, size_t n4, unsigned long long* t,
                                            int launch) {
    const unsigned long long t0 = wall_clock64();
    const int x = blockIdx.x & 7;  // the XCD (round-robin dispatch): clocks compared within one XCD
    if (threadIdx.x == 0) atomicMin(&t[16 * launch + 2 * x], t0);
    while (wall_clock64() - t0 < ticks) {
    }
    const size_t nth = (size_t)gridDim.x * blockDim.x;
    const float4 v = make_float4((float)launch, 1.f, 2.f, 3.f);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += nth) {
        if (MODE == 1) buf[i] = v;
        if (MODE == 2) __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(&buf[i]));
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&t[16 * launch + 2 * x + 1], wall_clock64());
}

int main() {
    int wclk = 100000;
    CK(hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int N = 40;
    unsigned long long* t;
    CK(hipMalloc(&t, 16 * N * 8));
    float4* buf;
    const size_t maxb = 256ull << 20;
    CK(hipMalloc(&buf, maxb));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned long long ticks = (unsigned long long)(40.0 * wclk / 1000.0);
    const char* mn[] = {"no stores", "plain stores", "nontemporal stores"};
    for (int mode = 0; mode < 3; ++mode) {
        for (size_t mb : {0, 4, 16, 64, 128}) {
            if (mode == 0 && mb) continue;
            if (mode && !mb) continue;
            std::vector<unsigned long long> h(16 * N);
            for (int i = 0; i < 8 * N; ++i) { h[2 * i] = ~0ull; h[2 * i + 1] = 0; }
            CK(hipMemcpy(t, h.data(), h.size() * 8, hipMemcpyHostToDevice));
            const size_t n4 = (mb << 20) / 16;
            for (int i = 0; i < N; ++i) {
                if (mode == 0) hipLaunchKernelGGL(work<0>, dim3(cus * 4), dim3(256), 0, s, ticks, buf, n4, t, i);
                if (mode == 1) hipLaunchKernelGGL(work<1>, dim3(cus * 4), dim3(256), 0, s, ticks, buf, n4, t, i);
                if (mode == 2) hipLaunchKernelGGL(work<2>, dim3(cus * 4), dim3(256), 0, s, ticks, buf, n4, t, i);
            }
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> gaps;
            for (int i = 5; i < N; ++i) {  // the XCD that ended last sees the smallest gap
                long long g = -1;
                for (int x = 0; x < 8; ++x) {
                    const long long d = (long long)h[16 * i + 2 * x] - (long long)h[16 * (i - 1) + 2 * x + 1];
                    if (g < 0 || d < g) g = d;
                }
                gaps.push_back((double)g * 1000.0 / wclk);
            }
            std::sort(gaps.begin(), gaps.end());
            printf("%-20s %4zu MB: gap last-wave-end -> next first-wave-start median %6.2f us (p10 %6.2f, p90 %6.2f)\n",
                   mn[mode], mb, gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[9 * gaps.size() / 10]);
        }
    }
    return 0;
}
