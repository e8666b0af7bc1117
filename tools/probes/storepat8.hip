// Persistent store streamers (round 5): what write rate does a persistent grid
// reach when every block loops over tiles of W bytes, by how the tiles are
// handed out?
//   mode 0 "front":   static grid-stride, tile t = b + i*G (the chip's write
//                     front is G*W contiguous bytes)
//   mode 1 "dequeue": tiles taken in order from one atomic counter (the next
//                     tile's index fetched while the current one is stored)
//   mode 2 "streams": block b owns [b*n/G, (b+1)*n/G) (one long stream per
//                     block; the front is G streams n/G apart, like k_stage's
//                     per-block 256-element chunks)
// PRO: per tile, a dependent load of 64 values into LDS (issued one tile
// ahead) and a barrier before the stores, like a stage kernel's phase A.
// Usage: storepat8 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int MODE, bool PRO>
__global__ __launch_bounds__(512) void pers(uint4* __restrict__ p, const uint4* __restrict__ in,
                                            uint32_t* ctr, uint32_t tw, uint32_t ntiles, size_t n) {
  extern __shared__ uint4 lds[];
  __shared__ uint32_t sNext;
  const uint32_t G = gridDim.x, b = blockIdx.x, T = blockDim.x;
  uint32_t t, tEnd = ntiles, i = 0;
  if (MODE == 2) {
    t = (uint32_t)((uint64_t)ntiles * b / G);
    tEnd = (uint32_t)((uint64_t)ntiles * (b + 1) / G);
  } else if (MODE == 1) {
    if (threadIdx.x == 0) sNext = atomicAdd(ctr, 1u);
    __syncthreads();
    t = sNext;
  } else {
    t = b;
  }
  uint4 pre = make_uint4(0, 0, 0, 0);
  if (PRO && t < tEnd && threadIdx.x < 64) pre = in[(size_t)t * 64 + threadIdx.x];
  while (t < tEnd) {
    uint32_t tn;
    if (MODE == 1) {
      __syncthreads();
      if (threadIdx.x == 0) sNext = atomicAdd(ctr, 1u);
    }
    uint4 x = make_uint4(t, 2, 3, 4);
    if (PRO) {
      if (threadIdx.x < 64) lds[(i & 1) * 64 + threadIdx.x] = pre;
      __syncthreads();
      x = lds[(i & 1) * 64 + (threadIdx.x & 63)];
    }
    if (MODE == 1) {
      if (!PRO) __syncthreads();
      tn = sNext;
    } else if (MODE == 2) {
      tn = t + 1;
    } else {
      tn = t + G;
    }
    if (PRO && tn < tEnd && threadIdx.x < 64) pre = in[(size_t)tn * 64 + threadIdx.x];
    const size_t b0 = (size_t)t * tw;
    for (uint32_t k = threadIdx.x; k < tw; k += T)
      if (b0 + k < n) p[b0 + k] = make_uint4(x.x + k, x.y, x.z, x.w);
    t = tn;
    ++i;
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
template <int MODE, bool PRO>
void run(uint4* a, const uint4* in, uint32_t* ctr, size_t n, size_t nin, const char* name) {
  for (uint32_t kib : {4u, 16u, 32u, 64u, 128u, 480u})
    for (int occ : {1, 2, 4})
      for (int waves : {4, 8}) {
        if (occ * waves > 32) continue;
        const uint32_t tw = kib * 1024 / 16;
        const uint32_t ntiles = (uint32_t)((n + tw - 1) / tw);
        if ((size_t)ntiles * 64 > nin) { printf("bad shape\n"); exit(1); }
        const unsigned G = 256 * occ, lds = 160 * 1024 / occ - 1024;
        const double r = gbs([&] {
          if (MODE == 1) CK(hipMemsetAsync(ctr, 0, 4, 0));
          hipLaunchKernelGGL((pers<MODE, PRO>), dim3(G), dim3(64 * waves), lds, 0, a, in, ctr, tw, ntiles, n);
        }, n * 16);
        printf("%-8s pro=%d tile %3u KiB occ %d waves %d: %.0f GB/s\n", name, (int)PRO, kib, occ, waves, r);
      }
}
int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const size_t bytes = (size_t)(gib * (1ull << 30)), n = bytes / 16;
  const size_t nin = (n / 256 + 1) * 64;     // 64 inputs per tile of >= 4 KiB
  uint4 *a, *in;
  uint32_t* ctr;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&in, nin * 16)); CK(hipMalloc(&ctr, 64));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(in, 1, nin * 16));
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  run<0, false>(a, in, ctr, n, nin, "front");
  run<0, true>(a, in, ctr, n, nin, "front");
  run<1, true>(a, in, ctr, n, nin, "dequeue");
  run<2, false>(a, in, ctr, n, nin, "streams");
  run<2, true>(a, in, ctr, n, nin, "streams");
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  return 0;
}
