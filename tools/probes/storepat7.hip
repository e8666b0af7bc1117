// Small-window stores from small blocks, with a phase-A-like prologue (one
// dependent global load per element into LDS + barrier, then the stores):
// how many bytes must a CU keep in flight, and in what block shape, to reach
// the narrow-front rates of storepat5 (4 KiB windows, ~7 TB/s without the
// prologue)? Block sizes 64 / 128 / 256 threads, windows 2-16 KiB, occupancy
// limited with dynamic LDS.
// Usage: storepat7 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// window = ch 16-B units per block; E inputs loaded first (E <= blockDim)
template <int BS>
__global__ __launch_bounds__(BS) void win_k(uint4* __restrict__ p, const uint4* __restrict__ in,
                                            uint32_t ch, uint32_t E, size_t n) {
  extern __shared__ uint4 lds[];
  if (threadIdx.x < E) lds[threadIdx.x] = in[(size_t)blockIdx.x * E + threadIdx.x];
  __syncthreads();
  const uint4 x = lds[threadIdx.x % E];
  const size_t b0 = (size_t)blockIdx.x * ch;
  for (uint32_t i = threadIdx.x; i < ch; i += BS)
    if (b0 + i < n) p[b0 + i] = make_uint4(x.x + i, x.y, x.z, x.w);
}
template <class F> double gbs(F f, size_t bytes) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return 5.0 * bytes / (ms * 1e-3) / 1e9;
}
template <int BS> void sweep(uint4* a, const uint4* in, size_t n, size_t nin) {
  for (uint32_t ck : {2u, 4u, 8u, 16u})
    for (int occ : {8, 16, 32}) {
      if (occ * BS / 64 > 32) continue;                  // 32 waves per CU at most
      const uint32_t ch = ck * 1024 / 16, E = 4;
      const unsigned g = (unsigned)((n + ch - 1) / ch);
      if ((size_t)g * E > nin) { printf("bad shape\n"); exit(1); }
      const unsigned lds = 160 * 1024 / occ - 256;
      const double r = gbs([&] { hipLaunchKernelGGL(win_k<BS>, dim3(g), dim3(BS), lds, 0, a, in, ch, E, n); }, n * 16);
      printf("block %3d window %2u KiB occ %2d blocks/CU: %.0f GB/s\n", BS, ck, occ, r);
    }
}
int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;
  const size_t bytes = (size_t)(gib * (1ull << 30)), n = bytes / 16;
  const size_t nin = n / 32 + 64;   // E = 4 inputs per window of >= 2 KiB (128 units)
  uint4 *a, *in;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&in, nin * 16));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(in, 1, nin * 16));
  sweep<64>(a, in, n, nin);
  sweep<128>(a, in, n, nin);
  sweep<256>(a, in, n, nin);
  return 0;
}
