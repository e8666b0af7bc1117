// Store patterns with k_stage's load-then-store structure (round 5): every
// block first loads its inputs (lw 16-byte words per window it will write, from
// an input array the size of the element values a stage would precompute) into
// LDS, waits for them, then writes its windows (4 KiB each, the whole block per
// window). Two layouts of the same bytes:
//   chunk: block b writes windows [b Q, b Q + Q) (one contiguous chunk: k_stage)
//   inter: block j of a super-chunk of SB blocks writes windows j, j + SB, ...
//          (4 KiB windows interleaved: storepat9's fast pattern)
// Q windows per block; blocks per CU set through the dynamic LDS size.
// Usage: storepat10 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <bool INTER>
__global__ __launch_bounds__(256) void ls(uint4* __restrict__ p, const uint4* __restrict__ in, uint32_t Q, uint32_t SB,
                                          uint32_t lw, size_t n, size_t nin) {
  extern __shared__ uint4 lds[];
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  // loads: lw words per window, Q windows, from the input slice of this block
  const uint32_t nl = lw * Q;
  const size_t i0 = ((size_t)b * nl) % (nin - nl);
  for (uint32_t k = t; k < nl; k += 256) lds[k] = in[i0 + k];
  __syncthreads();
  const uint4 x = lds[t % nl];
  size_t w0;
  for (uint32_t i = 0; i < Q; ++i) {
    if (INTER) {
      const uint32_t sc = b / SB, j = b - sc * SB;
      w0 = (size_t)sc * SB * Q + j + (size_t)i * SB;
    } else {
      w0 = (size_t)b * Q + i;
    }
    const size_t k = w0 * 256 + t;
    if (k < n) p[k] = make_uint4(x.x + (uint32_t)k, x.y, x.z, x.w);
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
  const double gib = argc > 1 ? atof(argv[1]) : 1.6;
  const size_t bytes = (size_t)(gib * (1ull << 30)), n = bytes / 16;
  const size_t nin = (256ull << 20) / 16;                        // 256 MB of inputs
  uint4 *a, *in;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&in, nin * 16));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(in, 1, nin * 16));
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  for (uint32_t lw : {0u, 48u})
    for (uint32_t Q : {8u, 16u, 32u})
      for (int occ : {2, 4, 8, 12})
        for (int inter = 0; inter < 2; ++inter) {
          const uint32_t SB = 8;
          const uint32_t G = (uint32_t)(n / (256ull * Q)) / SB * SB;
          const unsigned lds = 160 * 1024 / occ - 1024;
          if (lw * Q * 16 > lds) continue;
          const double r = gbs([&] {
            if (inter) hipLaunchKernelGGL(ls<true>, dim3(G), dim3(256), lds, 0, a, in, Q, SB, lw ? lw : 1, n, nin);
            else hipLaunchKernelGGL(ls<false>, dim3(G), dim3(256), lds, 0, a, in, Q, SB, lw ? lw : 1, n, nin);
          }, (size_t)G * Q * 4096);
          printf("loads %2u w/win Q %2u occ %2d %s: %.0f GB/s\n", lw, Q, occ, inter ? "inter" : "chunk", r);
        }
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  return 0;
}
