// Stream-bubble microbenchmark: the device-clock gap between the end of a
// kernel and the start of the next one that depends on it, for the ways the
// engine orders launches (same stream, an event recorded between, a
// cross-stream event wait, an event attached to the launch itself via
// hipExtLaunchKernelGGL, stream wait/write-value). Everything is enqueued
// behind a spinning kernel first, so the gaps are GPU-side only.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/evgap.hip -o /tmp/evgap && /tmp/evgap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_hold(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
// ts[0] = min start, ts[1] = max end over blocks (100 MHz wall clock)
__global__ __launch_bounds__(256) void k_work(unsigned long long* ts, float* sink, int iters) {
    const unsigned long long t0 = wall_clock64();
    float x = threadIdx.x * 1e-3f;
    for (int i = 0; i < iters; ++i) x = x * 0.999f + 1e-4f;
    sink[blockIdx.x * 256 + threadIdx.x] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMin(ts, t0);
        atomicMax(ts + 1, wall_clock64());
    }
}

int main() {
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const int blocks = 2048, reps = 25, pairs = 8;
    float* sink;
    unsigned long long* ts;
    uint32_t* flag;
    CK(hipMalloc(&sink, sizeof(float) * blocks * 256));
    CK(hipMalloc(&ts, sizeof(unsigned long long) * 4 * pairs));
    CK(hipMalloc(&flag, 64));
    hipEvent_t ev[pairs][4];
    const unsigned fl[4] = {hipEventDisableTiming | hipEventReleaseToDevice, hipEventDefault,
                            hipEventDisableTiming, hipEventReleaseToDevice};
    for (auto& p : ev)
        for (int f = 0; f < 4; ++f) CK(hipEventCreateWithFlags(&p[f], fl[f]));
    const char* names[] = {
        "same stream, nothing between",
        "same stream, event (DisableTiming|ReleaseToDevice)",
        "same stream, event (default)",
        "same stream, event (DisableTiming)",
        "cross stream, event (DisableTiming|ReleaseToDevice)",
        "cross stream, event (default)",
        "cross stream, stop event of hipExtLaunchKernelGGL (default)",
        "same stream, stop event of hipExtLaunchKernelGGL (default)",
        "cross stream, write/wait value",
    };
    const int nsc = sizeof(names) / sizeof(names[0]);
    std::vector<unsigned long long> init(4 * pairs);
    for (int i = 0; i < pairs; ++i) { init[4 * i] = init[4 * i + 2] = ~0ull; init[4 * i + 1] = init[4 * i + 3] = 0; }
    for (int sc = 0; sc < nsc; ++sc) {
        std::vector<double> gaps;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemcpy(ts, init.data(), init.size() * 8, hipMemcpyHostToDevice));
            CK(hipMemset(flag, 0, 64));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, s1, 50000ull);     // 500 us
            if (sc >= 4) hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, s2, 1000ull);
            for (int p = 0; p < pairs; ++p) {
                unsigned long long* a = ts + 4 * p;
                const bool cross = sc >= 4 && sc != 7;
                hipStream_t sb = cross ? s2 : s1;
                if (sc == 6 || sc == 7)
                    hipExtLaunchKernelGGL(k_work, dim3(blocks), dim3(256), 0, s1, nullptr, ev[p][1], 0, a, sink, 2000);
                else
                    hipLaunchKernelGGL(k_work, dim3(blocks), dim3(256), 0, s1, a, sink, 2000);
                if (sc >= 1 && sc <= 3) CK(hipEventRecord(ev[p][sc == 1 ? 0 : sc == 2 ? 1 : 2], s1));
                if (sc == 4 || sc == 5) {
                    hipEvent_t e = ev[p][sc == 4 ? 0 : 1];
                    CK(hipEventRecord(e, s1));
                    CK(hipStreamWaitEvent(s2, e, 0));
                }
                if (sc == 6) CK(hipStreamWaitEvent(s2, ev[p][1], 0));
                if (sc == 8) {
                    CK(hipStreamWriteValue32(s1, flag, p + 1, 0));
                    CK(hipStreamWaitValue32(s2, flag, p + 1, hipStreamWaitValueGte, 0xffffffffu));
                }
                hipLaunchKernelGGL(k_work, dim3(blocks), dim3(256), 0, sb, a + 2, sink, 2000);
                if (cross) {   // the next pair's first kernel starts after this one
                    CK(hipEventRecord(ev[p][3], s2));
                    CK(hipStreamWaitEvent(s1, ev[p][3], 0));
                }
            }
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(4 * pairs);
            CK(hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost));
            for (int p = 1; p < pairs; ++p) gaps.push_back((double)(h[4 * p + 2] - h[4 * p + 1]) / 100.0);
        }
        std::sort(gaps.begin(), gaps.end());
        printf("%-62s gap median %6.2f us  p10 %6.2f  p90 %6.2f\n", names[sc], gaps[gaps.size() / 2],
               gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10]);
    }
    // duration of one k_work for scale
    return 0;
}
