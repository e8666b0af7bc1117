// Persistent 256-block grids: own chunks vs interleaved sweep front.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
// block b writes chunks b, b+G, b+2G, ... each `chunk` u4 long, linearly
__global__ __launch_bounds__(256) void own_chunks(u4* p, size_t chunk, size_t nchunks, size_t n) {
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    size_t b0 = c * chunk;
    for (size_t i = threadIdx.x; i < chunk && b0 + i < n; i += 256) p[b0 + i] = u4{(unsigned)i, 1u, 2u, 3u};
  }
}
template <class F> double timeit(F f, size_t bytes) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return 5.0 * bytes / (ms * 1e-3) / 1e9;
}
int main() {
  size_t bytes = 4ull << 30, n = bytes / 16; u4* p; CK(hipMalloc(&p, bytes));
  for (size_t ch : {256ul, 1536ul, 6016ul, 24064ul, 96256ul})
    for (unsigned g : {256u, 512u, 768u}) {
      size_t nc = (n + ch - 1) / ch;
      printf("own_chunks chunk=%6zu (%7zu B) grid=%u: %.1f\n", ch, ch * 16, g,
             timeit([&]{ hipLaunchKernelGGL(own_chunks, dim3(g), dim3(256), 0, 0, p, ch, nc, n); }, bytes));
    }
  return 0;
}
