// Probe: does a hipGraph captured across two streams replay correctly, and do
// hipEventRecord calls captured on the origin stream time its kernels on replay?
//   hipcc --offload-arch=gfx950 -O2 tools/probes/graphtest.hip -o tools/probes/graphtest && ./tools/probes/graphtest
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_fill(float* p, int n, float v, const float* g) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v + (g ? g[0] : 0.f) + (float)(i & 7);
}
__global__ void k_spin(float* p, int n, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = p[i];
    for (int k = 0; k < iters; ++k) x = x * 0.999f + 0.001f;
    p[i] = x;
}

int main() {
    const int n = 1 << 22;
    float *a, *b, *g, *hg;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&g, 4));
    CK(hipHostMalloc(&hg, 4 * 64, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t fork, join, t0, t1;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeRelaxed));
    CK(hipEventRecord(fork, s1));
    CK(hipStreamWaitEvent(s2, fork, 0));
    hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, s1, a, n, 1.f, g);
    CK(hipEventRecord(t0, s1));
    hipLaunchKernelGGL(k_spin, dim3(n / 256), dim3(256), 0, s1, a, n, 2000);
    CK(hipEventRecord(t1, s1));
    hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, s2, b, n, 2.f, nullptr);
    hipLaunchKernelGGL(k_spin, dim3(n / 256), dim3(256), 0, s2, b, n, 1000);
    CK(hipEventRecord(join, s2));
    CK(hipStreamWaitEvent(s1, join, 0));
    CK(hipStreamEndCapture(s1, &graph));
    size_t nn = 0;
    CK(hipGraphGetNodes(graph, nullptr, &nn));
    printf("captured nodes: %zu\n", nn);
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (int it = 0; it < 5; ++it) {
        hg[it] = 100.f * it;
        CK(hipMemcpyAsync(g, hg + it, 4, hipMemcpyHostToDevice, s1));
        auto h0 = std::chrono::steady_clock::now();
        CK(hipGraphLaunch(exec, s1));
        auto h1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(s1));
        float ms = -1;
        hipError_t e = hipEventElapsedTime(&ms, t0, t1);
        float av;
        CK(hipMemcpy(&av, a, 4, hipMemcpyDeviceToHost));
        printf("launch %d: host %.1f us, event elapsed %s %.4f ms, a[0] %.3f\n", it,
               std::chrono::duration<double, std::micro>(h1 - h0).count(), hipGetErrorString(e), ms, av);
    }
    // the same with external event-record nodes (hipEventRecordExternal)
    {
        hipGraph_t gx;
        hipGraphExec_t xx;
        CK(hipStreamBeginCapture(s1, hipStreamCaptureModeRelaxed));
        hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, s1, a, n, 1.f, g);
        CK(hipEventRecordWithFlags(t0, s1, hipEventRecordExternal));
        hipLaunchKernelGGL(k_spin, dim3(n / 256), dim3(256), 0, s1, a, n, 2000);
        CK(hipEventRecordWithFlags(t1, s1, hipEventRecordExternal));
        CK(hipStreamEndCapture(s1, &gx));
        size_t nx = 0;
        CK(hipGraphGetNodes(gx, nullptr, &nx));
        printf("external-record graph nodes: %zu\n", nx);
        CK(hipGraphInstantiate(&xx, gx, nullptr, nullptr, 0));
        for (int it = 0; it < 3; ++it) {
            CK(hipGraphLaunch(xx, s1));
            CK(hipStreamSynchronize(s1));
            float ms = -1;
            hipError_t e = hipEventElapsedTime(&ms, t0, t1);
            printf("external launch %d: elapsed %s %.4f ms\n", it, hipGetErrorString(e), ms);
        }
    }
    // 40-kernel, 3-stream workload: eager enqueue vs graph replay (host + wall)
    {
        hipStream_t s3;
        CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
        hipEvent_t ev[64];
        for (auto& evx : ev) CK(hipEventCreateWithFlags(&evx, hipEventDisableTiming));
        const int m = 1 << 16;
        auto enqueue = [&]() {
            int k = 0;
            CK(hipEventRecord(ev[k], s1)); CK(hipStreamWaitEvent(s2, ev[k++], 0));
            CK(hipEventRecord(ev[k], s1)); CK(hipStreamWaitEvent(s3, ev[k++], 0));
            for (int i = 0; i < 40; ++i) {
                hipStream_t s = i % 3 == 0 ? s1 : i % 3 == 1 ? s2 : s3;
                hipLaunchKernelGGL(k_spin, dim3(m / 256), dim3(256), 0, s, (i % 3 == 0 ? a : b) + (i % 3) * m, m, 50);
            }
            CK(hipEventRecord(ev[k], s2)); CK(hipStreamWaitEvent(s1, ev[k++], 0));
            CK(hipEventRecord(ev[k], s3)); CK(hipStreamWaitEvent(s1, ev[k++], 0));
            return 0;
        };
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            auto h0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 20; ++it) if (enqueue()) return 1;
            auto h1 = std::chrono::steady_clock::now();
            CK(hipStreamSynchronize(s1));
            auto h2 = std::chrono::steady_clock::now();
            printf("eager x20: host %.1f us/iter, wall %.1f us/iter\n",
                   std::chrono::duration<double, std::micro>(h1 - h0).count() / 20,
                   std::chrono::duration<double, std::micro>(h2 - h0).count() / 20);
        }
        hipGraph_t g2;
        hipGraphExec_t x2;
        CK(hipStreamBeginCapture(s1, hipStreamCaptureModeRelaxed));
        if (enqueue()) return 1;
        CK(hipStreamEndCapture(s1, &g2));
        CK(hipGraphInstantiate(&x2, g2, nullptr, nullptr, 0));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            auto h0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 20; ++it) CK(hipGraphLaunch(x2, s1));
            auto h1 = std::chrono::steady_clock::now();
            CK(hipStreamSynchronize(s1));
            auto h2 = std::chrono::steady_clock::now();
            printf("graph x20: host %.1f us/iter, wall %.1f us/iter\n",
                   std::chrono::duration<double, std::micro>(h1 - h0).count() / 20,
                   std::chrono::duration<double, std::micro>(h2 - h0).count() / 20);
        }
    }
    // eager reference timing
    CK(hipEventRecord(t0, s1));
    hipLaunchKernelGGL(k_spin, dim3(n / 256), dim3(256), 0, s1, a, n, 2000);
    CK(hipEventRecord(t1, s1));
    CK(hipStreamSynchronize(s1));
    float ms;
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("eager k_spin: %.4f ms\n", ms);
    return 0;
}
