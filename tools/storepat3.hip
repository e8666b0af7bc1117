// Sweep-front store pattern at the stage kernel's group geometry: persistent
// grids, block b writes chunks b, b+G, ...; chunk sizes around one 4-element
// group of check_mat_diff (4 x 47 cells x 32 B = 6016 B), aligned / misaligned,
// 256- and 512-thread blocks.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
template <int BS>
__global__ __launch_bounds__(BS) void own_chunks(u4* p, size_t chunk, size_t nchunks, size_t n) {
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    size_t b0 = c * chunk;
    for (size_t i = threadIdx.x; i < chunk && b0 + i < n; i += BS) p[b0 + i] = u4{(unsigned)i, 1u, 2u, 3u};
  }
}
template <class F> double timeit(F f, size_t bytes) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return 5.0 * bytes / (ms * 1e-3) / 1e9;
}
int main() {
  size_t bytes = 2ull << 30, n = bytes / 16; u4* base; CK(hipMalloc(&base, bytes + 4096));
  for (size_t mis : {0ul, 2ul})
    for (size_t ch : {128ul, 256ul, 376ul, 512ul, 752ul})
      for (unsigned g : {256u, 512u}) {
        u4* p = base + mis;
        size_t nc = (n + ch - 1) / ch;
        double b256 = timeit([&]{ hipLaunchKernelGGL(own_chunks<256>, dim3(g), dim3(256), 0, 0, p, ch, nc, n); }, bytes);
        double b512 = timeit([&]{ hipLaunchKernelGGL(own_chunks<512>, dim3(g), dim3(512), 0, 0, p, ch, nc, n); }, bytes);
        printf("misalign=%zuB chunk=%5zu B grid=%u: 256thr %.1f  512thr %.1f GB/s\n", mis * 16, ch * 16, g, b256, b512);
      }
  return 0;
}
