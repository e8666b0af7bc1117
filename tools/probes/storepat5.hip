// Small-chunk store shapes (follow-up of storepat4): non-persistent grids whose
// blocks each write one small contiguous chunk, with and without a phase-A
// like prologue (a dependent global load of E input values into LDS + barrier
// before the stores), optionally with a second region (lookup-like, 1/4 size).
// Every configuration is measured twice (noise check).
// Usage: storepat5 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// chunk in 16-B units; E input words loaded first when PRO
template <bool PRO, bool TWO>
__global__ __launch_bounds__(256) void chunk_k(uint4* __restrict__ p, uint4* __restrict__ q,
                                               const uint4* __restrict__ in, uint32_t chunk,
                                               uint32_t E, size_t n) {
  extern __shared__ uint4 lds[];
  uint4 x = make_uint4(1, 2, 3, 4);
  if (PRO) {
    if (threadIdx.x < E) lds[threadIdx.x] = in[(size_t)blockIdx.x * E + threadIdx.x];
    __syncthreads();
    x = lds[threadIdx.x % E];
  }
  const size_t b0 = (size_t)blockIdx.x * chunk;
  for (uint32_t i = threadIdx.x; i < chunk; i += 256)
    if (b0 + i < n) p[b0 + i] = make_uint4(x.x + i, x.y, x.z, x.w);
  if (TWO) {
    const uint32_t c2 = chunk / 4;
    const size_t b1 = (size_t)blockIdx.x * c2;
    for (uint32_t i = threadIdx.x; i < c2; i += 256)
      if (b1 + i < n / 4) q[b1 + i] = make_uint4(x.x, i, x.z, x.w);
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
  uint4 *a, *b, *in;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes / 4 + 4096)); const size_t nin = n / 2 + 256;  // max block*E over the chunks below is n/2
  CK(hipMalloc(&in, nin * 16));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes / 4)); CK(hipMemset(in, 1, nin * 16));
  for (int rep = 0; rep < 2; ++rep)
    for (int pro = 0; pro < 2; ++pro)
      for (int two = 0; two < 2; ++two)
        for (int occ : {4, 8, 16})
          for (uint32_t ck : {2u, 4u, 8u, 16u, 32u}) {
            const uint32_t ch = ck * 1024 / 16, E = ch < 64 ? ch : 64;
            const unsigned g = (unsigned)((n + ch - 1) / ch);
            const unsigned lds = 160 * 1024 / occ - 512;
            if ((size_t)g * E > nin || E > 256 || (size_t)ch * 16 + 0 > (size_t)-1) { printf("bad shape\n"); return 1; }
            const size_t tot = bytes + (two ? bytes / 4 : 0);
            double r = gbs([&] {
              if (pro && two) hipLaunchKernelGGL((chunk_k<true, true>), dim3(g), dim3(256), lds, 0, a, b, in, ch, E, n);
              else if (pro) hipLaunchKernelGGL((chunk_k<true, false>), dim3(g), dim3(256), lds, 0, a, b, in, ch, E, n);
              else if (two) hipLaunchKernelGGL((chunk_k<false, true>), dim3(g), dim3(256), lds, 0, a, b, in, ch, E, n);
              else hipLaunchKernelGGL((chunk_k<false, false>), dim3(g), dim3(256), lds, 0, a, b, in, ch, E, n);
            }, tot);
            printf("rep%d pro=%d two=%d occ=%2d chunk=%2u KiB: %.0f GB/s\n", rep, pro, two, occ, ck, r);
          }
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  return 0;
}
