// Store-front microbenchmark: how does the write rate depend on the number of
// concurrently open write streams (chunk size x resident blocks)?
//   A. grid-stride 16 B/lane stores (narrow front; the reference ceiling)
//   B. non-persistent chunked grid: block b writes [b*chunk, (b+1)*chunk),
//      occupancy forced with dynamic LDS (1, 2, 4, 8 blocks per CU)
//   C. persistent round-robin: block b writes chunks b, b+G, ... (front = G*chunk)
//   D. like B, each block also writes a second chunk of chunk/4 bytes in a
//      second region (the stage kernel's advice + lookup shape)
// Usage: storepat4 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void gstride(uint4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((unsigned)i, 1, 2, 3);
}
__global__ __launch_bounds__(256) void chunked(uint4* p, size_t chunk, size_t n) {
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 1023) lds[0] = 1;  // never true; keeps the LDS allocation
  const size_t b0 = (size_t)blockIdx.x * chunk;
  for (size_t i = threadIdx.x; i < chunk && b0 + i < n; i += 256) p[b0 + i] = make_uint4((unsigned)i, 7, 8, 9);
}
__global__ __launch_bounds__(256) void chunked2(uint4* p, uint4* q, size_t chunk, size_t n) {
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 1023) lds[0] = 1;
  const size_t b0 = (size_t)blockIdx.x * chunk;
  for (size_t i = threadIdx.x; i < chunk && b0 + i < n; i += 256) p[b0 + i] = make_uint4((unsigned)i, 7, 8, 9);
  const size_t c2 = chunk / 4, b1 = (size_t)blockIdx.x * c2;
  for (size_t i = threadIdx.x; i < c2 && b1 + i < n / 4; i += 256) q[b1 + i] = make_uint4((unsigned)i, 7, 8, 9);
}
__global__ __launch_bounds__(256) void roundrobin(uint4* p, size_t chunk, size_t nchunks, size_t n) {
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const size_t b0 = c * chunk;
    for (size_t i = threadIdx.x; i < chunk && b0 + i < n; i += 256) p[b0 + i] = make_uint4((unsigned)i, 1, 2, 3);
  }
}
template <class F> double gbs(F f, size_t bytes) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return 5.0 * bytes / (ms * 1e-3) / 1e9;
}
int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;
  const size_t bytes = (size_t)(gib * (1ull << 30)), n = bytes / 16;
  uint4 *a, *b;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes / 4 + 4096));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes / 4));
  for (int g : {1024, 2048, 8192})
    printf("A gstride grid=%d: %.0f GB/s\n", g, gbs([&] { hipLaunchKernelGGL(gstride, dim3(g), dim3(256), 0, 0, a, n); }, bytes));
  const size_t chunksK[] = {4, 16, 64, 256, 1024};   // KiB
  for (int occ : {1, 2, 4, 8}) {
    const unsigned lds = 160 * 1024 / occ - 1024;
    for (size_t ck : chunksK) {
      const size_t ch = ck * 1024 / 16;
      const unsigned g = (unsigned)((n + ch - 1) / ch);
      printf("B chunked occ=%d chunk=%4zu KiB: %.0f GB/s\n", occ, ck,
             gbs([&] { hipLaunchKernelGGL(chunked, dim3(g), dim3(256), lds, 0, a, ch, n); }, bytes));
    }
  }
  for (int occ : {2, 8}) {
    const unsigned lds = 160 * 1024 / occ - 1024;
    for (size_t ck : chunksK) {
      const size_t ch = ck * 1024 / 16;
      const unsigned g = (unsigned)((n + ch - 1) / ch);
      printf("D chunked2 occ=%d chunk=%4zu KiB (+1/4 second region): %.0f GB/s\n", occ, ck,
             gbs([&] { hipLaunchKernelGGL(chunked2, dim3(g), dim3(256), lds, 0, a, b, ch, n); }, bytes + bytes / 4));
    }
  }
  for (unsigned g : {256u, 512u, 1024u, 2048u})
    for (size_t ck : {4ul, 16ul, 64ul}) {
      const size_t ch = ck * 1024 / 16, nc = (n + ch - 1) / ch;
      printf("C roundrobin grid=%u chunk=%zu KiB: %.0f GB/s\n", g, ck,
             gbs([&] { hipLaunchKernelGGL(roundrobin, dim3(g), dim3(256), 0, 0, a, ch, nc, n); }, bytes));
    }
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  return 0;
}
