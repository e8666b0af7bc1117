// Measured HBM ceilings on this MI355X for the engine's access shapes:
//   store16   : 16 B/lane contiguous stores (the k_stage / scan output shape)
//   copy16    : 16 B/lane load + store
//   store_cells: 32 B cells written as 2 x 16 B half-cells by 2 lanes (= k_stage)
// Usage: membw [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void store16(uint4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((unsigned)i, 1, 2, 3);
}
__global__ void copy16(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}
// contiguous chunks per block, like k_stage: block b writes [b*chunk, (b+1)*chunk)
__global__ void store_chunks(uint4* p, size_t chunk, size_t n) {
  size_t b0 = (size_t)blockIdx.x * chunk;
  for (size_t i = threadIdx.x; i < chunk && b0 + i < n; i += blockDim.x) p[b0 + i] = make_uint4((unsigned)i, 7, 8, 9);
}
int main(int argc, char** argv) {
  double gib = argc > 1 ? atof(argv[1]) : 4.0;
  size_t bytes = (size_t)(gib * (1ull << 30)), n = bytes / 16;
  uint4 *a, *b;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes)); CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms;
  int grids[] = {1024, 2048, 4096, 8192};
  for (int g : grids) {
    hipLaunchKernelGGL(store16, dim3(g), dim3(256), 0, 0, a, n);
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(store16, dim3(g), dim3(256), 0, 0, a, n);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("store16 grid=%d: %.1f GB/s\n", g, 5.0 * bytes / (ms * 1e-3) / 1e9);
  }
  for (int g : grids) {
    hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, 0, a, b, n);
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, 0, a, b, n);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy16 grid=%d: %.1f GB/s (read+write)\n", g, 5.0 * 2 * bytes / (ms * 1e-3) / 1e9);
  }
  size_t chunks[] = {24064 / 2, 24064, 96256};  // half-cells per k_stage block (C=47, E=256) ...
  for (size_t ch : chunks) {
    unsigned g = (unsigned)((n + ch - 1) / ch);
    hipLaunchKernelGGL(store_chunks, dim3(g), dim3(256), 0, 0, a, ch, n);
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(store_chunks, dim3(g), dim3(256), 0, 0, a, ch, n);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("store_chunks chunk=%zu x16B blocks=%u: %.1f GB/s\n", ch, g, 5.0 * bytes / (ms * 1e-3) / 1e9);
  }
  CK(hipMemset(a, 0, bytes));
  CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) CK(hipMemsetAsync(a, r, bytes));
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("hipMemset: %.1f GB/s\n", 5.0 * bytes / (ms * 1e-3) / 1e9);
  return 0;
}
