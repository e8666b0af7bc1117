// Persistent round-robin windows with a software-pipelined prologue: grid G
// blocks of 256 threads, block b writes 4 KiB windows b, b+G, b+2G, ...; before
// each window a dependent load (D iterations ahead: D = 0 waits for it, D >= 1
// prefetches into registers) feeds the stored values. Does a one-block-per-CU
// persistent kernel keep storepat4's 6.4 TB/s (grid 256, 4 KiB windows) once
// each window has an input to wait for?
// Usage: storepat8 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int D>
__global__ __launch_bounds__(256) void rr_k(uint4* __restrict__ p, const uint4* __restrict__ in,
                                            uint32_t nwin, uint32_t wpb /* windows per block */) {
  __shared__ uint4 lds[2][64];
  uint4 pre[D > 0 ? D : 1];
  const uint32_t t = threadIdx.x;
  auto win = [&](uint32_t k) { return blockIdx.x + k * gridDim.x; };
  // the per-window input: 16 x 16 B (256 B) read by the first lanes
#pragma unroll
  for (int k = 0; k < D; ++k)
    if (t < 16 && win(k) < nwin) pre[k] = in[(size_t)win(k) * 16 + t];
  for (uint32_t k = 0; k < wpb; ++k) {
    const uint32_t w = win(k);
    if (w >= nwin) break;
    const int slot = k & 1;
    if (t < 16) {
      uint4 x;
      if (D == 0) {
        x = in[(size_t)w * 16 + t];
      } else {
        x = pre[0];
#pragma unroll
        for (int j = 0; j + 1 < D; ++j) pre[j] = pre[j + 1];
        if (win(k + D) < nwin) pre[D - 1] = in[(size_t)win(k + D) * 16 + t];
      }
      lds[slot][t] = x;
    }
    __syncthreads();
    const uint4 v = lds[slot][t & 15];
    p[(size_t)w * 256 + t] = make_uint4(v.x + t, v.y, v.z, v.w);
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
  const size_t bytes = (size_t)(gib * (1ull << 30));
  const uint32_t nwin = (uint32_t)(bytes / 4096);
  uint4 *a, *in;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&in, (size_t)nwin * 256));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(in, 1, (size_t)nwin * 256));
  for (uint32_t G : {256u, 512u, 1024u}) {
    const uint32_t wpb = (nwin + G - 1) / G;
    printf("G=%4u D=0: %.0f GB/s\n", G, gbs([&] { hipLaunchKernelGGL(rr_k<0>, dim3(G), dim3(256), 0, 0, a, in, nwin, wpb); }, bytes));
    printf("G=%4u D=2: %.0f GB/s\n", G, gbs([&] { hipLaunchKernelGGL(rr_k<2>, dim3(G), dim3(256), 0, 0, a, in, nwin, wpb); }, bytes));
    printf("G=%4u D=4: %.0f GB/s\n", G, gbs([&] { hipLaunchKernelGGL(rr_k<4>, dim3(G), dim3(256), 0, 0, a, in, nwin, wpb); }, bytes));
    printf("G=%4u D=8: %.0f GB/s\n", G, gbs([&] { hipLaunchKernelGGL(rr_k<8>, dim3(G), dim3(256), 0, 0, a, in, nwin, wpb); }, bytes));
  }
  return 0;
}
