// Standalone timing of the CRT GEMM kernels (round 6): the shipped
// register-staged k_gemm_crt_multi against the LDS-DMA variants
// k_gemm_crt_dma<NBUF>, on random balanced residue planes shaped like the
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

__global__ void k_nmod(const unsigned* W, uint32_t lk, int* out) { *out = crt_nmod(W[0], W[1], lk); }

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 20;
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
    for (int v = 0; v < 4; ++v) {
        uint8_t* R;
        CK(hipMalloc(&R, 3 * rbytes));
        CK(hipMemset(R, 0, 3 * rbytes));
        Rs.push_back(R);
    }
    const char* vname[4] = {"shipped(reg)", "dma2", "dma3", "dma4"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Case& cs : cases) {
        double best[4] = {1e9, 1e9, 1e9, 1e9};
        for (int round = 0; round < 3; ++round)
            for (int v = 0; v < 4; ++v) {
                CrtBatch b;
                memset(&b, 0, sizeof b);
                b.njobs = cs.njobs;
                for (int j = 0; j < cs.njobs; ++j)
                    job(b.job[j], cs.sym[j], W + cs.wa[j], W + cs.wb[j], Rs[v] + j * rbytes);
                uint32_t units, cblocks;
                CK(prep_crt_batch(b, units, cblocks));
                const dim3 g((units + 7) / 8 * 8);
                auto launch = [&] {
                    if (v == 0) hipLaunchKernelGGL(k_gemm_crt_multi, g, dim3(256), 0, 0, b);
                    else if (v == 1) hipLaunchKernelGGL(k_gemm_crt_dma<2>, g, dim3(256), 0, 0, b);
                    else if (v == 2) hipLaunchKernelGGL(k_gemm_crt_dma<3>, g, dim3(256), 0, 0, b);
                    else hipLaunchKernelGGL(k_gemm_crt_dma<4>, g, dim3(256), 0, 0, b);
                };
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
        for (int v = 0; v < 4; ++v) {
            size_t diff = 0;
            if (v) {
                CK(hipMemcpy(r1.data(), Rs[v], 3 * rbytes, hipMemcpyDeviceToHost));
                for (size_t i = 0; i < 3 * rbytes; ++i) diff += r0[i] != r1[i];
            }
            printf("%-7s %-13s %8.2f us  %6.3f Pop/s (%4.1f %% of 5.03)  residue bytes differing: %zu\n",
                   cs.name, vname[v], best[v], cs.ops / (best[v] * 1e-6) / 1e15,
                   100.0 * cs.ops / (best[v] * 1e-6) / 5.03e15, diff);
        }
        for (int v = 0; v < 4; ++v) CK(hipMemset(Rs[v], 0, 3 * rbytes));
    }
    return 0;
}
