// Standalone timing of the CRT GEMM kernels (round 6): the per-unit
// k_gemm_crt_multi against the persistent k_gemm_crt_pers and the 256 x 128
// tile k_gemm_crt_wide (non-symmetric jobs only), on random balanced
// residue planes shaped like the
// 1024^2 P=63 witness (m.v^T: 19 moduli; u.u^T and v.v^T symmetric: 18), alone
// and as the step's three-job batch. Every variant's residue bytes are compared
// with the shipped kernel's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gemmprobe.hip -o tools/probes/gemmprobe
//   tools/probes/gemmprobe [n=1024] [reps=20]
#include "../../halo2_svd041_amd/csrc/kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

using namespace svdw;

// A stand-in for k_stage beside the GEMM: 256-thread blocks holding 63 KiB of
// LDS (two per CU, as k_stage_multi's 256-element blocks), each writing one
// contiguous 64 KiB chunk in 16-byte lane stores after five LDS word reads per
// store (phase B's descriptor + source words).
__global__ __launch_bounds__(256) void k_standin(uint4* __restrict__ out, size_t n16) {
    extern __shared__ uint32_t L[];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 63 * 256; i += 256) L[i] = i * 2654435761u;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * 4096;
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t k = (r * 256 + t) * 5;
        uint4 v = make_uint4(L[k % 16128], L[(k + 1) % 16128], L[(k + 2) % 16128], L[(k + 3) % 16128]);
        v.x ^= L[(k + 4) % 16128];
        const size_t o = base + r * 256 + t;
        if (o < n16) out[o] = v;
    }
}

// (round 6 also measured LDS-DMA staging with 2-4 chunk buffers and the
// per-unit kernel with the old fp32-quotient epilogue: profiles/r06_ab/r6c)
static constexpr int NV = 3;
static const char* vname[NV] = {"per-unit", "persistent", "wide"};
static bool has_sym(const CrtBatch& b) {
    for (uint32_t j = 0; j < b.njobs; ++j)
        if (b.job[j].sym) return true;
    return false;
}
static void launch_variant(int v, dim3 g, hipStream_t st, const CrtBatch& b) {
    if (v == 0) {
        hipLaunchKernelGGL(k_gemm_crt_multi, g, dim3(256), 0, st, b);
    } else if (v == 1) {
        hipLaunchKernelGGL(k_gemm_crt_pers, dim3(std::min<uint32_t>(g.x, 8 * kCrtPersPerXcd)), dim3(256), 0, st, b);
    } else {
        uint32_t w = 0;
        for (uint32_t j = 0; j < b.njobs; ++j) w += kCrtMaxMod * ((b.job[j].tiles_a + 1) / 2 * b.job[j].tiles_m);
        hipLaunchKernelGGL(k_gemm_crt_wide, dim3((w + 7) / 8 * 8), dim3(256), 0, st, b);
    }
}

__global__ void k_nmod(const unsigned* W, uint32_t lk, int* out) { *out = crt_nmod(W[0], W[1], lk); }

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 20;
    const bool quick = argc > 3 && !strcmp(argv[3], "quick");     // one round, no stand-in (PMC runs)
    const uint32_t kpad = (n + 255) / 256 * 256, rp = (n + 127) / 128 * 128;
    uint32_t lk = 0;
    while ((1u << lk) < n) ++lk;
    const size_t plane = (size_t)rp * kpad, pbytes = (size_t)kCrtMaxResidues * plane;
    uint8_t *A, *B;
    CK(hipMalloc(&A, pbytes));
    CK(hipMalloc(&B, pbytes));
    {
        std::vector<uint8_t> h(pbytes);
        uint64_t s = 88172645463325252ull;
        for (size_t i = 0; i < pbytes; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            h[i] = (uint8_t)(s >> 24);
        }
        CK(hipMemcpy(A, h.data(), pbytes, hipMemcpyHostToDevice));
        for (size_t i = 0; i < pbytes; ++i) h[i] = (uint8_t)(h[i] * 29u + 7u);
        CK(hipMemcpy(B, h.data(), pbytes, hipMemcpyHostToDevice));
    }
    // bit-length words: m (70 bits), v (64), u (64) as at 1024^2 P=63
    unsigned hW[3] = {70, 64, 64}, *W;
    CK(hipMalloc(&W, sizeof hW));
    CK(hipMemcpy(W, hW, sizeof hW, hipMemcpyHostToDevice));
    int *dn, nm[2];
    CK(hipMalloc(&dn, 2 * sizeof(int)));
    hipLaunchKernelGGL(k_nmod, dim3(1), dim3(64), 0, 0, W, lk, dn);
    hipLaunchKernelGGL(k_nmod, dim3(1), dim3(64), 0, 0, W + 1, lk, dn + 1);
    CK(hipMemcpy(nm, dn, sizeof nm, hipMemcpyDeviceToHost));
    printf("n %u: moduli m.v^T %d, sym %d\n", n, nm[0], nm[1]);
    const size_t rbytes = crt_scratch_bytes(n, n);
    auto job = [&](CrtJob& q, bool sym, const unsigned* wa, const unsigned* wb, uint8_t* R) {
        memset(&q, 0, sizeof q);
        q.Ar = A; q.Br = sym ? A : B; q.R = R; q.out = nullptr;
        q.bits_a = wa; q.bits_b = wb; q.ors = n; q.ocs = 1;
        q.astride = rp; q.bstride = rp; q.kpad = kpad; q.N = n; q.M = n; q.lk = lk; q.sym = sym;
    };
    struct Case { const char* name; int njobs; bool sym[3]; int wa[3], wb[3]; double ops; };
    const double nnn = (double)n * n * n;
    const uint32_t nt = (n + 127) / 128;
    const double symfrac = (double)(nt * (nt + 1) / 2) / (nt * nt);
    Case cases[] = {
        {"m.v^T", 1, {false}, {0}, {1}, 2 * nnn * nm[0]},
        {"u.u^T", 1, {true}, {1}, {1}, 2 * nnn * nm[1] * symfrac},
        {"batch3", 3, {false, true, true}, {0, 1, 1}, {1, 1, 1},
         2 * nnn * (nm[0] + 2 * nm[1] * symfrac)},
    };
    std::vector<uint8_t*> Rs;
    for (int v = 0; v < NV; ++v) {
        uint8_t* R;
        CK(hipMalloc(&R, 3 * rbytes));
        CK(hipMemset(R, 0, 3 * rbytes));
        Rs.push_back(R);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Case& cs : cases) {
        double best[NV] = {1e9, 1e9, 1e9};
        bool skip[NV] = {false, false, false};
        for (int round = 0; round < (quick ? 1 : 3); ++round)
            for (int v = 0; v < NV; ++v) {
                CrtBatch b;
                memset(&b, 0, sizeof b);
                b.njobs = cs.njobs;
                for (int j = 0; j < cs.njobs; ++j)
                    job(b.job[j], cs.sym[j], W + cs.wa[j], W + cs.wb[j], Rs[v] + j * rbytes);
                uint32_t units, cblocks;
                CK(prep_crt_batch(b, units, cblocks));
                if (v == 2 && has_sym(b)) {
                    skip[v] = true;
                    continue;
                }
                const dim3 g((units + 7) / 8 * 8);
                auto launch = [&] { launch_variant(v, g, 0, b); };
                for (int w = 0; w < 3; ++w) launch();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                for (uint32_t r = 0; r < reps; ++r) launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / reps;
                if (us < best[v]) best[v] = us;
            }
        // residue bytes of every variant against the shipped kernel (all jobs' scratch)
        std::vector<uint8_t> r0(3 * rbytes), r1(3 * rbytes);
        CK(hipMemcpy(r0.data(), Rs[0], 3 * rbytes, hipMemcpyDeviceToHost));
        for (int v = 0; v < NV; ++v) {
            if (skip[v]) continue;
            size_t diff = 0;
            if (v) {
                CK(hipMemcpy(r1.data(), Rs[v], 3 * rbytes, hipMemcpyDeviceToHost));
                for (size_t i = 0; i < 3 * rbytes; ++i) diff += r0[i] != r1[i];
            }
            printf("%-7s %-13s %8.2f us  %6.3f Pop/s (%4.1f %% of 5.03)  residue bytes differing: %zu\n",
                   cs.name, vname[v], best[v], cs.ops / (best[v] * 1e-6) / 1e15,
                   100.0 * cs.ops / (best[v] * 1e-6) / 5.03e15, diff);
        }
        // per-block timeline of one launch per variant (svdw_debug_trace's clocks,
        // 100 MHz): prologue (start -> first chunk staged), K loop, epilogue
        if (!quick) {
            const size_t nb = 16384;
            unsigned long long* tr;
            CK(hipMalloc(&tr, nb * 5 * 8));
            std::vector<unsigned long long> h(nb * 5);
            for (int v = 0; v < NV; ++v) {
                CrtBatch b;
                memset(&b, 0, sizeof b);
                b.njobs = cs.njobs;
                for (int j = 0; j < cs.njobs; ++j)
                    job(b.job[j], cs.sym[j], W + cs.wa[j], W + cs.wb[j], Rs[v] + j * rbytes);
                uint32_t units, cblocks;
                CK(prep_crt_batch(b, units, cblocks));
                const dim3 g((units + 7) / 8 * 8);
                if (g.x > nb || (v == 2 && has_sym(b))) continue;
                CK(hipMemset(tr, 0, nb * 5 * 8));
                CK(set_debug_trace(tr));
                launch_variant(v, g, 0, b);
                CK(hipDeviceSynchronize());
                CK(set_debug_trace(nullptr));
                CK(hipMemcpy(h.data(), tr, nb * 5 * 8, hipMemcpyDeviceToHost));
                unsigned long long lo = ~0ull, hi = 0;
                double sp = 0, sl = 0, se = 0;
                size_t cnt = 0;
                for (size_t k = 0; k < g.x; ++k) {
                    const unsigned long long* r = &h[5 * k];
                    if (!r[0]) continue;
                    ++cnt;
                    lo = r[0] < lo ? r[0] : lo;
                    hi = r[3] > hi ? r[3] : hi;
                    sp += (double)(r[1] - r[0]);
                    sl += (double)(r[2] - r[1]);
                    se += (double)(r[3] - r[2]);
                }
                if (cnt)
                    printf("%-7s %-13s timeline: %zu blocks, span %.1f us; per block: prologue %.2f us, "
                           "K loop %.2f us, epilogue %.2f us\n", cs.name, vname[v], cnt, (hi - lo) / 100.0,
                           sp / cnt / 100.0, sl / cnt / 100.0, se / cnt / 100.0);
            }
            CK(hipFree(tr));
        }
        for (int v = 0; v < NV; ++v) CK(hipMemset(Rs[v], 0, 3 * rbytes));
    }
    if (quick) return 0;
    // beside the stand-in store stream: the stand-in alone, then with each
    // variant's three-job batch launched on a second stream just after it
    {
        const size_t sbytes = (size_t)2 << 30, n16 = sbytes / 16;
        uint4* so;
        CK(hipMalloc(&so, sbytes));
        hipStream_t sa, sb;
        CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
        hipEvent_t a0, a1, b0, b1;
        CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1)); CK(hipEventCreate(&b0)); CK(hipEventCreate(&b1));
        const uint32_t sgrid = (uint32_t)(n16 / 4096);
        CK(hipFuncSetAttribute((const void*)k_standin, hipFuncAttributeMaxDynamicSharedMemorySize, 63 * 1024));
        const Case& cs = cases[2];
        for (int round = 0; round < 3; ++round)
            for (int v = -1; v < 2; ++v) {
                CrtBatch b;
                memset(&b, 0, sizeof b);
                b.njobs = cs.njobs;
                for (int j = 0; j < cs.njobs; ++j)
                    job(b.job[j], cs.sym[j], W + cs.wa[j], W + cs.wb[j], Rs[v < 0 ? 0 : v] + j * rbytes);
                uint32_t units, cblocks;
                CK(prep_crt_batch(b, units, cblocks));
                const dim3 g((units + 7) / 8 * 8);
                float sms = 0, gms = 0;
                for (int rep = 0; rep < 4; ++rep) {
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(a0, sa));
                    hipLaunchKernelGGL(k_standin, dim3(sgrid), dim3(256), 63 * 1024, sa, so, n16);
                    CK(hipEventRecord(a1, sa));
                    if (v >= 0) {
                        CK(hipEventRecord(b0, sb));
                        launch_variant(v, g, sb, b);
                        CK(hipEventRecord(b1, sb));
                    }
                    CK(hipDeviceSynchronize());
                    float x;
                    CK(hipEventElapsedTime(&x, a0, a1));
                    if (rep) sms += x / 3;
                    if (v >= 0) {
                        CK(hipEventElapsedTime(&x, b0, b1));
                        if (rep) gms += x / 3;
                    }
                }
                printf("beside stand-in (2 GiB, 2 blocks/CU x 63 KiB): %-13s stand-in %8.1f us (%5.0f GB/s)  gemm batch3 %8.1f us\n",
                       v < 0 ? "none" : vname[v], sms * 1e3, sbytes / (sms * 1e-3) / 1e9, gms * 1e3);
            }
    }
    return 0;
}
