// storepat10 at the load ratio of a precomputed-values window streamer (round 6,
// VERDICT r05 #3): every block writes Q 4 KiB windows and first needs lw 16-byte
// words per window (lw = 4 .. 24: 1.6-9.4 % of the bytes it stores; a stage
// element's 64-192 B of values per ~1.9 KB of cells is 3-10 %).
//   upfront: all Q * lw words into LDS, one barrier, then the Q windows
//            (storepat10's structure, k_stage's);
//   pipe:    the words of window i + 1 are loaded (into registers) before
//            window i is stored, then parked in the other LDS buffer: one
//            barrier per window, the load latency under the stores.
// Layouts of the same windows: chunk (block b writes windows b Q .. b Q + Q - 1)
// and inter (block j of a super-chunk of SB = 8 blocks writes windows
// j, j + SB, ...: storepat9's fast pattern). Blocks per CU through the dynamic
// LDS size. memset before and after, in the same process.
// Usage: storepat11 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ size_t win_of(bool inter, uint32_t b, uint32_t i, uint32_t Q, uint32_t SB) {
  if (inter) {
    const uint32_t sc = b / SB, j = b - sc * SB;
    return (size_t)sc * SB * Q + j + (size_t)i * SB;
  }
  return (size_t)b * Q + i;
}

template <bool INTER, bool PIPE>
__global__ __launch_bounds__(256) void ls(uint4* __restrict__ p, const uint4* __restrict__ in, uint32_t Q,
                                          uint32_t SB, uint32_t lw, size_t n, size_t nin) {
  extern __shared__ uint4 lds[];
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  const uint32_t nl = lw * Q;
  const size_t i0 = ((size_t)b * nl) % (nin - nl);
  if (!PIPE) {
    for (uint32_t k = t; k < nl; k += 256) lds[k] = in[i0 + k];
    __syncthreads();
    for (uint32_t i = 0; i < Q; ++i) {
      const uint4 x = lds[i * lw + t % lw];
      const size_t k = win_of(INTER, b, i, Q, SB) * 256 + t;
      if (k < n) p[k] = make_uint4(x.x + (uint32_t)k, x.y, x.z, x.w);
    }
    return;
  }
  uint4 nx = make_uint4(0, 0, 0, 0);
  if (t < lw) lds[t] = in[i0 + t];
  __syncthreads();
  for (uint32_t i = 0; i < Q; ++i) {
    if (t < lw && i + 1 < Q) nx = in[i0 + (size_t)(i + 1) * lw + t];     // window i + 1, in flight
    const uint4 x = lds[(i & 1) * lw + t % lw];
    const size_t k = win_of(INTER, b, i, Q, SB) * 256 + t;
    if (k < n) p[k] = make_uint4(x.x + (uint32_t)k, x.y, x.z, x.w);
    if (t < lw && i + 1 < Q) lds[((i + 1) & 1) * lw + t] = nx;
    __syncthreads();
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
  for (uint32_t lw : {0u, 4u, 8u, 12u, 16u, 24u})
    for (int pipe = 0; pipe < (lw ? 2 : 1); ++pipe)
      for (uint32_t Q : {8u, 16u, 32u})
        for (int occ : {2, 4, 8})
          for (int inter = 0; inter < 2; ++inter) {
            const uint32_t SB = 8;
            const uint32_t G = (uint32_t)(n / (256ull * Q)) / SB * SB;
            const unsigned lds = 160 * 1024 / occ - 1024;
            const uint32_t l = lw ? lw : 1;
            if ((pipe ? 2 * l : l * Q) * 16 > lds) continue;
            const double r = gbs([&] {
              if (pipe) {
                if (inter) hipLaunchKernelGGL((ls<true, true>), dim3(G), dim3(256), lds, 0, a, in, Q, SB, l, n, nin);
                else hipLaunchKernelGGL((ls<false, true>), dim3(G), dim3(256), lds, 0, a, in, Q, SB, l, n, nin);
              } else {
                if (inter) hipLaunchKernelGGL((ls<true, false>), dim3(G), dim3(256), lds, 0, a, in, Q, SB, l, n, nin);
                else hipLaunchKernelGGL((ls<false, false>), dim3(G), dim3(256), lds, 0, a, in, Q, SB, l, n, nin);
              }
            }, (size_t)G * Q * 4096);
            printf("loads %2u w/win (%4.1f %%) %-7s Q %2u occ %d %s: %.0f GB/s\n", lw, 100.0 * lw * 16 / 4096,
                   pipe ? "pipe" : "upfront", Q, occ, inter ? "inter" : "chunk", r);
          }
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  return 0;
}
