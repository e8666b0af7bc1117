// Interleaved-element store shape for the stage kernel: a non-persistent grid
// where each consecutive group of R blocks jointly covers R*E consecutive
// elements of S bytes; block r of a group writes elements r, r+R, ..., so the
// blocks resident together write inside a window of about R*S bytes instead of
// R*E*S. A prologue (one dependent global load per element into LDS +
// barrier) models phase A. Compared with the contiguous-chunk shape
// (block b writes elements [b*E, (b+1)*E)).
// Usage: storepat6 [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// S16 = element size in 16-B units; ne = total elements
template <bool INTERLEAVE>
__global__ __launch_bounds__(256) void elems_k(uint4* __restrict__ p, const uint4* __restrict__ in,
                                               uint32_t S16, uint32_t E, uint32_t R, uint32_t ne) {
  __shared__ uint4 lds[256];
  const uint32_t grp = blockIdx.x / R, r = blockIdx.x - grp * R;
  const uint32_t base = grp * R * E;
  auto elem = [&](uint32_t k) -> uint32_t { return INTERLEAVE ? base + r + k * R : blockIdx.x * E + k; };
  if (threadIdx.x < E) {
    const uint32_t e = elem(threadIdx.x);
    lds[threadIdx.x] = e < ne ? in[e] : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  const uint32_t tot = E * S16;
  for (uint32_t h = threadIdx.x; h < tot; h += 256) {
    const uint32_t k = h / S16, s = h - k * S16;
    const uint32_t e = elem(k);
    if (e < ne) {
      const uint4 x = lds[k];
      p[(size_t)e * S16 + s] = make_uint4(x.x + s, x.y, x.z, x.w);
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
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;
  const size_t bytes = (size_t)(gib * (1ull << 30));
  uint4 *a, *in;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 0, bytes));
  const uint32_t maxne = (uint32_t)(bytes / 128);  // S >= 128 B below
  CK(hipMalloc(&in, (size_t)maxne * 16));
  CK(hipMemset(in, 1, (size_t)maxne * 16));
  for (int rep = 0; rep < 2; ++rep)
    for (uint32_t S : {128u, 1504u, 1888u})
      for (uint32_t E : {16u, 64u, 256u}) {
        const uint32_t S16 = S / 16, ne = (uint32_t)(bytes / S);
        if (ne > maxne || E > 256) { printf("bad shape\n"); return 1; }
        {
          const uint32_t g = (ne + E - 1) / E;
          const double r = gbs([&] { hipLaunchKernelGGL((elems_k<false>), dim3(g), dim3(256), 0, 0, a, in, S16, E, 1u, ne); }, (size_t)ne * S);
          printf("rep%d S=%4u E=%3u contiguous        : %.0f GB/s\n", rep, S, E, r);
        }
        for (uint32_t R : {256u, 1024u, 4096u}) {
          const uint32_t per = R * E, ngrp = (ne + per - 1) / per, g = ngrp * R;
          const double r = gbs([&] { hipLaunchKernelGGL((elems_k<true>), dim3(g), dim3(256), 0, 0, a, in, S16, E, R, ne); }, (size_t)ne * S);
          printf("rep%d S=%4u E=%3u interleave R=%4u: %.0f GB/s\n", rep, S, E, R, r);
        }
      }
  return 0;
}
