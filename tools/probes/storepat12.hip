// Round 6: does the chunk-per-block store pattern's rate depend on where the
// region lies in memory? (tools/r6/realloc.py: the same witness in one process
// takes 1.77-2.03 ms depending on where its cell streams were allocated.)
// G blocks, two per CU (63 KiB of dynamic LDS each, as k_stage_multi's
// 256-element blocks), block b writes chunk map(b) of Q 4 KiB windows, one
// window per iteration in 16 B lane stores (k_stage's phase B pattern), at byte
// offset off of one large allocation; off runs over 0, 2, ..., 126 MiB.
// map: 0 identity, 1 chunk (b * 37) mod G, 2 XCD-contiguous (b mod 8) G/8 + b/8.
// Usage: storepat12 [Q=122] [G=4096]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void chunks(uint4* __restrict__ p, uint32_t Q, uint32_t G, int map) {
  extern __shared__ uint4 lds[];
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  if (t == 0) lds[0] = make_uint4(b, 0, 0, 0);
  uint32_t c = b;
  if (map == 1) c = (uint32_t)(((uint64_t)b * 37u) % G);
  else if (map == 2) c = (b & 7u) * (G >> 3) + (b >> 3);
  uint4* o = p + (size_t)c * Q * 256;
  for (uint32_t i = 0; i < Q; ++i) o[(size_t)i * 256 + t] = make_uint4(i, c, t, b);
}

int main(int argc, char** argv) {
  const uint32_t Q = argc > 1 ? atoi(argv[1]) : 122, G = argc > 2 ? atoi(argv[2]) : 4096;
  const size_t region = (size_t)G * Q * 4096, slack = (size_t)128 << 20;
  uint4* p;
  CK(hipMalloc(&p, region + slack));
  CK(hipFuncSetAttribute((const void*)chunks, hipFuncAttributeMaxDynamicSharedMemorySize, 63 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](size_t off, int map) {
    uint4* q = p + off / 16;
    hipLaunchKernelGGL(chunks, dim3(G), dim3(256), 63 * 1024, 0, q, Q, G, map);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(chunks, dim3(G), dim3(256), 63 * 1024, 0, q, Q, G, map);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return region * 5 / (ms * 1e-3) / 1e12;
  };
  {
    CK(hipMemset(p, 0, region));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) CK(hipMemsetAsync(p, r, region));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("memset %.2f TB/s (region %.2f GB, Q %u, G %u)\n", region * 5 / (ms * 1e-3) / 1e12, region / 1e9, Q, G);
  }
  printf("off_MiB  identity  x37  xcd\n");
  double lo[3] = {1e9, 1e9, 1e9}, hi[3] = {0, 0, 0}, sum[3] = {0, 0, 0};
  int n = 0;
  for (size_t off = 0; off < slack; off += (size_t)2 << 20) {
    double r[3];
    for (int m = 0; m < 3; ++m) {
      r[m] = run(off, m);
      lo[m] = r[m] < lo[m] ? r[m] : lo[m];
      hi[m] = r[m] > hi[m] ? r[m] : hi[m];
      sum[m] += r[m];
    }
    ++n;
    printf("%6zu  %6.2f  %6.2f  %6.2f\n", off >> 20, r[0], r[1], r[2]);
  }
  for (int m = 0; m < 3; ++m) printf("map %d: min %.2f max %.2f mean %.2f TB/s\n", m, lo[m], hi[m], sum[m] / n);
  return 0;
}
