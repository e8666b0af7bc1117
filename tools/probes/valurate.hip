// VALU issue rates of the integer instructions the field arithmetic is built
// from (gfx950): 8 independent dependency chains per lane, full occupancy,
// reported as wave-instructions per CU per clock (1.0 = one wave64 op per
// cycle per CU, i.e. every SIMD issuing every 4 cycles).
// Usage: valurate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int ITERS = 256;
#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ __launch_bounds__(256) void k_mad64(uint32_t* out, uint32_t s) {
  uint64_t a[8]; uint32_t b = threadIdx.x | 1, c = s;
#define INIT(i) a[i] = threadIdx.x + i;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) { uint64_t cy; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a[i]), "=s"(cy) : "v"(b), "v"(c)); }
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
#define SUM(i) x ^= (uint32_t)a[i] ^ (uint32_t)(a[i] >> 32);
  REP8(SUM)
  if (x == 0x12345678u) out[0] = x;
}
__global__ __launch_bounds__(256) void k_mullo(uint32_t* out, uint32_t s) {
  uint32_t a[8]; uint32_t b = threadIdx.x | 1;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
#define SUM32(i) x ^= a[i];
  REP8(SUM32)
  if (x == 0x12345678u + s) out[0] = x;
}
__global__ __launch_bounds__(256) void k_mulhi(uint32_t* out, uint32_t s) {
  uint32_t a[8]; uint32_t b = threadIdx.x | 1;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
  REP8(SUM32)
  if (x == 0x12345678u + s) out[0] = x;
}
__global__ __launch_bounds__(256) void k_lshladd64(uint32_t* out, uint32_t s) {
  uint64_t a[8]; uint64_t b = threadIdx.x | 1;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(b));
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
  REP8(SUM)
  if (x == 0x12345678u + s) out[0] = x;
}
__global__ __launch_bounds__(256) void k_addco(uint32_t* out, uint32_t s) {
  uint32_t a[8]; uint32_t b = threadIdx.x | 1;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) { uint64_t cy; asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(a[i]), "=s"(cy) : "v"(b)); }
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
  REP8(SUM32)
  if (x == 0x12345678u + s) out[0] = x;
}
__global__ __launch_bounds__(256) void k_addu32(uint32_t* out, uint32_t s) {
  uint32_t a[8]; uint32_t b = threadIdx.x | 1;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
  REP8(SUM32)
  if (x == 0x12345678u + s) out[0] = x;
}
__global__ __launch_bounds__(256) void k_alignbit(uint32_t* out, uint32_t s) {
  uint32_t a[8]; uint32_t b = threadIdx.x | 1;
  REP8(INIT)
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
    REP8(OP)
#undef OP
  }
  uint32_t x = 0;
  REP8(SUM32)
  if (x == 0x12345678u + s) out[0] = x;
}

template <class K> void run(const char* name, K k, uint32_t* out, int ncu, double ghz) {
  const int grid = ncu * 8;   // 8 blocks x 4 waves = 32 waves per CU
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 3u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 3u);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double winst = 10.0 * grid * 4 * ITERS * 8;           // wave-instructions
  const double per_cu_clk = winst / ncu / (ms * 1e-3 * ghz * 1e9);
  printf("%-14s %.3f wave-inst/CU/clk (%.2f ms)\n", name, per_cu_clk, ms);
}
int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const double ghz = p.clockRate / 1e6;
  printf("CUs %d, clock %.2f GHz\n", p.multiProcessorCount, ghz);
  uint32_t* out; CK(hipMalloc(&out, 64));
  run("v_add_u32", k_addu32, out, p.multiProcessorCount, ghz);
  run("v_add_co_u32", k_addco, out, p.multiProcessorCount, ghz);
  run("v_alignbit", k_alignbit, out, p.multiProcessorCount, ghz);
  run("v_lshl_add_u64", k_lshladd64, out, p.multiProcessorCount, ghz);
  run("v_mul_lo_u32", k_mullo, out, p.multiProcessorCount, ghz);
  run("v_mul_hi_u32", k_mulhi, out, p.multiProcessorCount, ghz);
  run("v_mad_u64_u32", k_mad64, out, p.multiProcessorCount, ghz);
  return 0;
}
