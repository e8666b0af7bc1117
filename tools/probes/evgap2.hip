// Where does the 7 us same-stream launch boundary come from? Device-clock gap
// between the last block end of a kernel and the first block start of the next
// one on the same stream (everything queued behind a spinning kernel, so the
// gaps are GPU-side only), for predecessors that differ in one thing each:
//   - trivial: 256 blocks, no stores;
//   - dirty B MiB: the predecessor writes B MiB with plain / nt / sc1 16-B stores
//     (sc1: write-through, the line leaves the XCD's L2 at once);
//   - big kernel argument: the successor takes a 3.5 KiB by-value argument
//     (k_stage_multi's StageMulti is of that size);
//   - timestamps: min start from s_memrealtime (100 MHz) per block.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/evgap2.hip -o /tmp/evgap2 && /tmp/evgap2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
struct Big { unsigned w[896]; };   // 3.5 KiB

__global__ void k_hold(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
__device__ __forceinline__ void stamp(unsigned long long* ts, unsigned long long t0) {
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMin(ts, t0);
        atomicMax(ts + 1, __builtin_amdgcn_s_memrealtime());
    }
}
// mode 0: no stores, 1: plain, 2: nt, 3: sc1 (write-through); n16 16-B stores per block
__global__ __launch_bounds__(256) void k_prod(unsigned long long* ts, v4u* out, unsigned n16, int mode) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    v4u* p = out + (size_t)blockIdx.x * n16;
    const v4u v = {blockIdx.x, threadIdx.x, 1u, 2u};
    for (unsigned i = threadIdx.x; i < n16 && mode; i += 256) {
        if (mode == 1) p[i] = v;
        else if (mode == 2) __builtin_nontemporal_store(v, p + i);
        else asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + i), "v"(v) : "memory");
    }
    stamp(ts, t0);
}
__global__ __launch_bounds__(256) void k_cons(unsigned long long* ts, const Big b) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (b.w[threadIdx.x & 7] == 12345u) ts[2] = 0;    // keep the argument alive
    stamp(ts, t0);
}
__global__ __launch_bounds__(256) void k_cons_small(unsigned long long* ts, unsigned x) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (x == 12345u) ts[2] = 0;
    stamp(ts, t0);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int blocks = 1024, reps = 20, pairs = 6;
    const size_t maxb = 64ull << 20;
    v4u* out;
    unsigned long long* ts;
    CK(hipMalloc(&out, maxb));
    CK(hipMalloc(&ts, sizeof(unsigned long long) * 8 * pairs));
    Big big;
    for (auto& w : big.w) w = 7;
    struct Sc { const char* name; int mode; unsigned mib; bool bigarg; };
    const Sc sc[] = {
        {"trivial predecessor (no stores), small arg", 0, 0, false},
        {"trivial predecessor, 3.5 KiB by-value arg", 0, 0, true},
        {"2 MiB plain stores", 1, 2, false},
        {"16 MiB plain stores", 1, 16, false},
        {"64 MiB plain stores", 1, 64, false},
        {"16 MiB nt stores", 2, 16, false},
        {"64 MiB nt stores", 2, 64, false},
        {"16 MiB sc1 stores", 3, 16, false},
        {"64 MiB sc1 stores", 3, 64, false},
    };
    std::vector<unsigned long long> init(8 * pairs);
    for (int i = 0; i < pairs; ++i)
        for (int k = 0; k < 8; k += 4) { init[8 * i + k] = ~0ull; init[8 * i + k + 1] = 0; init[8 * i + k + 2] = 0; init[8 * i + k + 3] = 0; }
    for (const Sc& c : sc) {
        std::vector<double> gaps, durs;
        const unsigned n16 = (unsigned)(((size_t)c.mib << 20) / 16 / blocks);
        for (int r = 0; r < reps; ++r) {
            CK(hipMemcpy(ts, init.data(), init.size() * 8, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, s, 30000ull);     // 300 us
            for (int p = 0; p < pairs; ++p) {
                unsigned long long* a = ts + 8 * p;
                hipLaunchKernelGGL(k_prod, dim3(blocks), dim3(256), 0, s, a, out, n16, c.mode);
                if (c.bigarg) hipLaunchKernelGGL(k_cons, dim3(256), dim3(256), 0, s, a + 4, big);
                else hipLaunchKernelGGL(k_cons_small, dim3(256), dim3(256), 0, s, a + 4, 1u);
            }
            CK(hipStreamSynchronize(s));
            std::vector<unsigned long long> h(8 * pairs);
            CK(hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost));
            for (int p = 1; p < pairs; ++p) {
                gaps.push_back((double)((long long)h[8 * p + 4] - (long long)h[8 * p + 1]) / 100.0);
                durs.push_back((double)(h[8 * p + 1] - h[8 * p]) / 100.0);
            }
        }
        std::sort(gaps.begin(), gaps.end());
        std::sort(durs.begin(), durs.end());
        printf("%-46s gap median %6.2f us  p10 %6.2f  p90 %6.2f   (producer %7.2f us)\n", c.name,
               gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10], durs[durs.size() / 2]);
    }
    return 0;
}
