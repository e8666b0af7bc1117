// Which 16-B store pattern reaches the hipMemset rate (6.35 TB/s) on gfx950?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// A: chunk per block, U stores in flight per lane per iteration (lane-interleaved)
template <int U, bool NT>
__global__ __launch_bounds__(256) void chunkU(u4* p, size_t chunk, size_t n) {
  size_t b0 = (size_t)blockIdx.x * chunk;
  for (size_t i = threadIdx.x; i < chunk; i += 256 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t j = i + u * 256;
      if (j < chunk && b0 + j < n) {
        u4 v = {(unsigned)j, 1u, 2u, 3u};
        if (NT) __builtin_nontemporal_store(v, p + b0 + j); else p[b0 + j] = v;
      }
    }
  }
}
// B: each lane writes 4 consecutive u4 (64 B) -> wave covers 4 KiB per group
__global__ __launch_bounds__(256) void chunk64B(u4* p, size_t chunk, size_t n) {
  size_t b0 = (size_t)blockIdx.x * chunk;
  for (size_t i = threadIdx.x * 4; i < chunk; i += 1024) {
#pragma unroll
    for (int u = 0; u < 4; ++u) if (b0 + i + u < n) p[b0 + i + u] = u4{(unsigned)i, 1u, 2u, 3u};
  }
}
// C: persistent grid-stride over 1 KiB-per-wave units, grid = k * 256 blocks
__global__ __launch_bounds__(256) void persist(u4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = u4{(unsigned)i, 1u, 2u, 3u};
}
template <class F> double timeit(F f, size_t bytes) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return 5.0 * bytes / (ms * 1e-3) / 1e9;
}
int main() {
  size_t bytes = 4ull << 30, n = bytes / 16; u4* p; CK(hipMalloc(&p, bytes));
  size_t ch = 24064; unsigned g = (unsigned)((n + ch - 1) / ch);
  printf("chunk U=1      %.1f\n", timeit([&]{ hipLaunchKernelGGL((chunkU<1,false>), dim3(g), dim3(256), 0, 0, p, ch, n); }, bytes));
  printf("chunk U=2      %.1f\n", timeit([&]{ hipLaunchKernelGGL((chunkU<2,false>), dim3(g), dim3(256), 0, 0, p, ch, n); }, bytes));
  printf("chunk U=4      %.1f\n", timeit([&]{ hipLaunchKernelGGL((chunkU<4,false>), dim3(g), dim3(256), 0, 0, p, ch, n); }, bytes));
  printf("chunk U=4 NT   %.1f\n", timeit([&]{ hipLaunchKernelGGL((chunkU<4,true>), dim3(g), dim3(256), 0, 0, p, ch, n); }, bytes));
  printf("chunk 64B/lane %.1f\n", timeit([&]{ hipLaunchKernelGGL(chunk64B, dim3(g), dim3(256), 0, 0, p, ch, n); }, bytes));
  for (unsigned k : {1u, 2u, 4u, 8u, 16u})
    printf("persist %4u blk %.1f\n", 256 * k, timeit([&]{ hipLaunchKernelGGL(persist, dim3(256 * k), dim3(256), 0, 0, p, n); }, bytes));
  printf("hipMemset      %.1f\n", timeit([&]{ CK(hipMemsetAsync(p, 0, bytes)); }, bytes));
  printf("hipMemsetD32   %.1f\n", timeit([&]{ CK(hipMemsetD32Async((hipDeviceptr_t)p, 0x1234567, bytes / 4, 0)); }, bytes));
  return 0;
}
