// Per-step cost of the stream structure around a persistent kernel (the bench's C3 step):
// back-to-back persistent launches on one stream, with an event recorded after each, and with
// a second stream whose small kernel each launch waits for (the prepass beside the previous
// integrate).  Prints the mean interval per step minus the kernel's own spin time.
// hipcc --offload-arch=gfx950 -O2 tools/packet_gap.hip -o build/packet_gap && build/packet_gap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void spin(unsigned long long ticks, unsigned* sink) {
    const unsigned long long t0 = wall_clock64();
    unsigned n = 0;
    while (wall_clock64() - t0 < ticks) ++n;
    if (n == 0xFFFFFFFFu) sink[threadIdx.x] = n;  // keeps the loop
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int wclk = 100000;  // wall_clock64 rate in kHz
    CK(hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0));
    const int cus = prop.multiProcessorCount;
    unsigned* sink;
    CK(hipMalloc(&sink, 4096));
    hipStream_t s, ps;
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&ps, hipStreamNonBlocking, hi));
    const int N = 200;
    hipEvent_t ev[8], fe[8], t0, t1;
    for (int i = 0; i < 8; ++i) {
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&fe[i], hipEventDisableTiming));
    }
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const double us_big = 60.0, us_small = 8.0;
    const unsigned long long tb = (unsigned long long)(us_big * wclk / 1000.0);
    const unsigned long long ts = (unsigned long long)(us_small * wclk / 1000.0);
    const char* names[] = {"back-to-back", "+ event record after each",
                           "+ prep kernel waited for, prep after launch i-2 (bench step)",
                           "+ prep kernel waited for, prep waits nothing", "as the bench step, two prep kernels",
                           "as the bench step, prep after launch i-3", "prep after launch i-2, not waited for",
                           "host-ordered sets: record every 4th, host waits for launch i-8",
                           "as the bench step, stream wait/write-value (signal memory) in place of events"};
    uint32_t *flag_s = nullptr, *flag_p = nullptr;
    CK(hipExtMallocWithFlags((void**)&flag_s, 8, hipMallocSignalMemory));
    CK(hipExtMallocWithFlags((void**)&flag_p, 8, hipMallocSignalMemory));
    for (int mode = 0; mode < 9; ++mode) {
        if (mode == 8) {
            CK(hipMemset(flag_s, 0, 4));
            CK(hipMemset(flag_p, 0, 4));
            CK(hipDeviceSynchronize());
        }
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, s));
            for (int i = 0; i < N; ++i) {
                if (mode == 8) {  // values are 1-based launch counts; the prep waits for launch i-2
                    const unsigned base = rep * N;
                    if (i >= 2) CK(hipStreamWaitValue32(ps, flag_s, base + (unsigned)(i - 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
                    hipLaunchKernelGGL(spin, dim3(cus / 4), dim3(256), 0, ps, ts, sink);
                    CK(hipStreamWriteValue32(ps, flag_p, base + (unsigned)i + 1u, 0));
                    CK(hipStreamWaitValue32(s, flag_p, base + (unsigned)i + 1u, hipStreamWaitValueGte, 0xFFFFFFFFu));
                    hipLaunchKernelGGL(spin, dim3(cus * 4), dim3(256), 0, s, tb, sink);
                    CK(hipStreamWriteValue32(s, flag_s, base + (unsigned)i + 1u, 0));
                    continue;
                }
                if (mode >= 2) {
                    const int lag = mode == 5 ? 3 : 2;
                    if (mode == 7) {
                        if (i >= 8 && (i & 3) == 0) CK(hipEventSynchronize(ev[(i - 8) & 7]));
                    } else if (mode != 3 && i >= lag) {
                        CK(hipStreamWaitEvent(ps, ev[(i - lag) % 4], 0));
                    }
                    if (mode == 4) hipLaunchKernelGGL(spin, dim3(cus), dim3(256), 0, ps, ts / 2, sink);
                    hipLaunchKernelGGL(spin, dim3(cus / 4), dim3(256), 0, ps, ts, sink);
                    CK(hipEventRecord(fe[i % 8], ps));
                    if (mode != 6) CK(hipStreamWaitEvent(s, fe[i % 8], 0));
                }
                hipLaunchKernelGGL(spin, dim3(cus * 4), dim3(256), 0, s, tb, sink);
                if (mode == 7) {
                    if ((i & 3) == 0) CK(hipEventRecord(ev[i & 7], s));
                } else if (mode != 0 && mode != 3) {
                    CK(hipEventRecord(ev[i % 4], s));
                }
            }
            CK(hipEventRecord(t1, s));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            if (rep == 1) printf("%-48s %7.2f us per step, %6.2f us beyond the kernel's spin\n", names[mode],
                                 ms * 1000.0 / N, ms * 1000.0 / N - us_big);
        }
    }
    return 0;
}
