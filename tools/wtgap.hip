// Kernel-boundary cost behind a store-heavy kernel, plain (write-back: the L2
// keeps the dirty lines, the boundary's release writes them back) vs sc1
// (write-through) 16-byte stores, and the streaming rate of both.
//   hipcc --offload-arch=gfx950 -O2 tools/wtgap.hip -o /tmp/wtgap && /tmp/wtgap
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_wt(uint4* p, uint4 v) {
    const v4u d = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(d) : "memory");
}
__global__ void k_hold(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
// each block writes `per` contiguous bytes (the stage kernel's chunk pattern)
template <bool WT>
__global__ __launch_bounds__(256) void k_fill(uint4* out, uint64_t per16, unsigned long long* ts) {
    const unsigned long long t0 = wall_clock64();
    uint4* o = out + (uint64_t)blockIdx.x * per16;
    const uint4 v = make_uint4(blockIdx.x, threadIdx.x, 1, 2);
    for (uint64_t i = threadIdx.x; i < per16; i += 256) {
        if (WT) st16_wt(o + i, v);
        else o[i] = v;
    }
    if (ts) {
        __syncthreads();
        if (threadIdx.x == 0) { atomicMin(ts, t0); atomicMax(ts + 1, wall_clock64()); }
    }
}
__global__ void k_tiny(unsigned long long* ts) {
    if (threadIdx.x == 0) { atomicMin(ts + 2, wall_clock64()); atomicMax(ts + 3, wall_clock64()); }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t big = 2ull << 30;
    uint4* buf;
    unsigned long long* ts;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&ts, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // streaming rate: 512 blocks x 4 MB (2 GB)
    for (int wt = 0; wt < 2; ++wt) {
        const uint64_t per16 = (big / 512) / 16;
        std::vector<float> ms;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(e0, s));
            if (wt) hipLaunchKernelGGL(k_fill<true>, dim3(512), dim3(256), 0, s, buf, per16, nullptr);
            else hipLaunchKernelGGL(k_fill<false>, dim3(512), dim3(256), 0, s, buf, per16, nullptr);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%s stores: 2 GiB in %.3f ms = %.2f TB/s\n", wt ? "sc1 (write-through)" : "plain", ms[2],
               big / (ms[2] * 1e-3) / 1e12);
    }
    // boundary: k_fill of B bytes then a dependent tiny kernel, behind a hold
    for (size_t mb : {1, 4, 16, 32, 64}) {
        for (int wt = 0; wt < 2; ++wt) {
            std::vector<double> gaps;
            for (int r = 0; r < 15; ++r) {
                unsigned long long init[4] = {~0ull, 0, ~0ull, 0};
                CK(hipMemcpy(ts, init, 32, hipMemcpyHostToDevice));
                CK(hipDeviceSynchronize());
                hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, s, 20000ull);
                const uint64_t per16 = (mb << 20) / 512 / 16;
                if (wt) hipLaunchKernelGGL(k_fill<true>, dim3(512), dim3(256), 0, s, buf, per16, ts);
                else hipLaunchKernelGGL(k_fill<false>, dim3(512), dim3(256), 0, s, buf, per16, ts);
                hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, ts);
                CK(hipDeviceSynchronize());
                unsigned long long h[4];
                CK(hipMemcpy(h, ts, 32, hipMemcpyDeviceToHost));
                gaps.push_back((double)(h[2] - h[1]) / 100.0);
            }
            std::sort(gaps.begin(), gaps.end());
            printf("boundary after %3zu MB of %s stores: gap median %5.2f us (p10 %5.2f, p90 %5.2f)\n", mb,
                   wt ? "sc1  " : "plain", gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10]);
        }
    }
    return 0;
}
