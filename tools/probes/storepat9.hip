// Chunked store streamers (round 5): the write rate of a NON-persistent grid
// shaped like k_stage's phase B -- block b writes its own contiguous chunk of
// `chunk` bytes in blockDim*16-byte windows (one 16-byte store per lane per
// window) -- by chunk size, blocks per CU (set through the dynamic LDS size)
// and the window a block starts at:
//   rot 0: every block starts at its chunk's first window (k_stage);
//   rot 1: block b starts at window (b * 37) mod nwin and wraps around, so the
//          blocks in flight write addresses spread over their chunks instead of
//          all sitting at the same offset of a chunk-sized stride.
//   rot 2: super-chunks of SB blocks interleave their windows: block j of a
//          super-chunk writes windows j, j + SB, j + 2 SB, ... of the
//          super-chunk's SB * nwin windows, so the blocks in flight form
//          compact fronts of SB adjacent windows (SB = 8 .. 256).
//   groups: k_stage's phase B over interleaved element groups -- block j of a
//          super-chunk of SB blocks owns Q groups of gb 16-byte words (group
//          j + i SB, i < Q) and its lanes stream the concatenation of its
//          groups (lane t: words t, t + 256, ...), with the whole pattern
//          shifted by `off` words (a stage whose first cell is not 128-byte
//          aligned: then every group boundary splits a line between blocks).
//   xcd:   chunks as k_stage, block b writing chunk (b mod 8) G/8 + b / 8, so
//          the blocks of one XCD (dispatched round-robin over the 8 XCDs)
//          write adjacent chunks; wpw: each wave streams its own windows
//          (window 4 i + wave) instead of the block sharing one.
// spin: a per-block delay (s_sleep loop of `spin` iterations) before the
// stores, standing in for phase A.
// Usage: storepat9 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int ROT>
__global__ __launch_bounds__(256) void chunks(uint4* __restrict__ p, uint32_t cw, uint32_t spin, size_t n,
                                              uint32_t SB) {
  extern __shared__ uint4 lds[];
  const uint32_t T = blockDim.x, nwin = cw / T;
  const size_t c0 = (size_t)blockIdx.x * cw;
  for (uint32_t s = 0; s < spin; ++s) __builtin_amdgcn_s_sleep(2);
  if (spin) {
    lds[threadIdx.x] = make_uint4(threadIdx.x, 0, 0, 0);
    __syncthreads();
  }
  if (ROT == 2) {
    const uint32_t sc = blockIdx.x / SB, j = blockIdx.x - sc * SB;
    const size_t s0 = (size_t)sc * SB * cw;
    for (uint32_t i = 0; i < nwin; ++i) {
      const size_t k = s0 + (size_t)(j + i * SB) * T + threadIdx.x;
      if (k < n) p[k] = make_uint4((uint32_t)k, 2, 3, 4);
    }
    return;
  }
  const uint32_t w0 = ROT ? (blockIdx.x * 37u) % nwin : 0u;
  for (uint32_t i = 0; i < nwin; ++i) {
    uint32_t w = w0 + i;
    if (w >= nwin) w -= nwin;
    const size_t k = c0 + (size_t)w * T + threadIdx.x;
    if (k < n) p[k] = make_uint4((uint32_t)k, 2, 3, 4);
  }
}
__global__ __launch_bounds__(256) void groups(uint4* __restrict__ p, uint32_t gb, uint32_t Q, uint32_t SB,
                                              uint32_t off, size_t n) {
  const uint32_t sc = blockIdx.x / SB, j = blockIdx.x - sc * SB;
  const size_t g0 = (size_t)sc * SB * Q + j;
  uint32_t q = 0, r = threadIdx.x;
  while (r >= gb) { r -= gb; ++q; }
  const uint32_t dq = 256 / gb, dr = 256 - dq * gb;
  for (uint32_t hc = threadIdx.x; hc < Q * gb; hc += 256) {
    const size_t k = off + (g0 + (size_t)q * SB) * gb + r;
    if (k < n) p[k] = make_uint4((uint32_t)k, 2, 3, 4);
    q += dq; r += dr;
    if (r >= gb) { r -= gb; ++q; }
  }
}
template <bool XCD, bool WPW>
__global__ __launch_bounds__(256) void chunks2(uint4* __restrict__ p, uint32_t cw, size_t n) {
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t c = XCD ? (b % 8) * (G / 8) + b / 8 : b;
  const size_t c0 = (size_t)c * cw;
  const uint32_t nwin = cw / 256, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (WPW) {
    for (uint32_t i = 0; i < nwin; i += 4)
      for (uint32_t q = 0; q < 4; ++q) {
        const size_t k = c0 + (size_t)(i + wave) * 256 + q * 64 + lane;
        if (i + wave < nwin && k < n) p[k] = make_uint4((uint32_t)k, 2, 3, 4);
      }
  } else {
    for (uint32_t i = 0; i < nwin; ++i) {
      const size_t k = c0 + (size_t)i * 256 + threadIdx.x;
      if (k < n) p[k] = make_uint4((uint32_t)k, 2, 3, 4);
    }
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
  uint4* a;
  CK(hipMalloc(&a, bytes)); CK(hipMemset(a, 0, bytes));
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  for (int rep = 0; rep < 2; ++rep)
    for (uint32_t kib : {32u, 136u, 480u})
      for (int mode = 0; mode < 4; ++mode) {
        const uint32_t cw = kib * 1024 / 16;
        const uint32_t G = (uint32_t)(n / cw) / 8 * 8;
        const double r = gbs([&] {
          if (mode == 0) hipLaunchKernelGGL((chunks2<false, false>), dim3(G), dim3(256), 0, 0, a, cw, n);
          if (mode == 1) hipLaunchKernelGGL((chunks2<true, false>), dim3(G), dim3(256), 0, 0, a, cw, n);
          if (mode == 2) hipLaunchKernelGGL((chunks2<false, true>), dim3(G), dim3(256), 0, 0, a, cw, n);
          if (mode == 3) hipLaunchKernelGGL((chunks2<true, true>), dim3(G), dim3(256), 0, 0, a, cw, n);
        }, (size_t)G * cw * 16);
        printf("chunk %3u KiB xcd %d wpw %d: %.0f GB/s\n", kib, mode & 1, mode >> 1, r);
      }
  printf("memset: %.0f GB/s\n", gbs([&] { CK(hipMemsetAsync(a, 3, bytes)); }, bytes));
  return 0;
}
