// Standalone timing of the verify_mul row scans (k_matvec_scan_dpp, round 6):
// one launch of J jobs x 1024 rows x 1024 terms (row operand |a| < 2^64 as
// cells, na = 2 as in the 1024^2 P=63 witness), the shipped kernel against
// timing diagnostics of the same body (k_scan_diag, a copy of it here: DIAG 1
// without the cell stores, 2 without the loads; their cells are wrong). Bytes
// written per launch: rows x (3L + 1) x 32.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/scanprobe.hip -o tools/probes/scanprobe
//   tools/probes/scanprobe [jobs=3] [reps=10]
#include "../../halo2_svd041_amd/csrc/kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

namespace svdw {
template <int T, int NA, int DIAG>
__global__ __launch_bounds__(256) void k_scan_diag(const ScanBatch B) {
    static_assert(256 % T == 0, "T divides the block");
    constexpr uint32_t TPR = 256 / T;                     // threads staged per round
    // a staging thread's 3T cells, padded by 16 B: a lane stride of 6T + 1
    // (odd) 16 B units keeps each b128 store pass on distinct bank groups
    constexpr uint32_t RS = 6 * T + 1;
    __shared__ __attribute__((aligned(16))) uint4 stage[TPR * RS];
    __shared__ U9 wtot[4], wpre[4];
    __shared__ Fr carry_s;
    ScanJob J = B.job[0];
#pragma unroll
    for (int q = 1; q < kMaxScanJobs; ++q)
        if ((uint32_t)q < B.njobs && blockIdx.x >= B.job[q].blk0) J = B.job[q];
    const DView& A = J.A;
    const uint32_t L = J.L;
    const int na = batch_na<NA>(B);
    const Fr* __restrict__ wc = J.wc;
    const Fr* __restrict__ wm = tab_slot(J.tab, J.tl, na);
    const Fr* __restrict__ wn = wm + J.tl;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t lb = blockIdx.x - J.blk0;
    const uint32_t rb = (J.blk0 & 7) ? lb : scan_row(lb, J.rows), r = J.r_begin + rb;
    Fr* rowout = J.out + (uint64_t)rb * (3ull * L + 1);
    const Fr zero = fr_zero();
    Fr eqy = zero;                                        // is_equal's y, loaded ahead
    if (tid == 0) {
        st_fr(rowout, zero);
        carry_s = zero;
        if (J.eq_out) eqy = ld_fr(J.eq_y + (uint64_t)r * J.eq_ys);
    }
    for (uint32_t c0 = 0; c0 < L; c0 += 256 * T) {
        const uint32_t j0 = c0 + tid * T;
        // every load of the chunk issued together (the row operand, both table
        // entries, the vector's canonical cell): one memory round trip per
        // chunk instead of three dependent ones, which beside a saturating cell
        // stream cost microseconds each
        Fr a[T], w[T], tm[T], tn[T], s[T];
#pragma unroll
        for (int i = 0; i < T; ++i) {
            const uint32_t j = j0 + i;
            const bool in = j < L;
            if constexpr (DIAG == 2) {                    // no loads: register values
                a[i] = fr_from_u64(j * 2654435761ull + r);
                w[i] = fr_from_u64(j + 7);
                tm[i] = fr_from_u64(j + 11);
                tn[i] = fr_from_u64(j + 13);
                continue;
            }
            a[i] = in ? view_load(A, zero, r, j) : zero;
            w[i] = in ? ld_fr(wc + j) : zero;
            tm[i] = in ? ld_fr(wm + j) : zero;
            tn[i] = in && na < 8 ? ld_fr(wn + j) : zero;
        }
#pragma unroll
        for (int i = 0; i < T; ++i) s[i] = j0 + i < L ? scan_prod_pre<NA>(na, a[i], tm[i], tn[i]) : zero;
        // local inclusive sums (< T p), the wave scan and the prefixes stay
        // unreduced (exact, < 2^265); each output is reduced once
        U9 loc[T];
        loc[0] = u9_from(s[0]);
#pragma unroll
        for (int i = 1; i < T; ++i) loc[i] = u9_add(loc[i - 1], u9_from(s[i]));
        const U9 tot = wave_scan_u9(loc[T - 1]);
        if (lane == 63) wtot[wave] = tot;
        __syncthreads();
        if (tid == 0) {                                   // wave prefixes and the running carry
            U9 acc = u9_from(carry_s);
#pragma unroll
            for (int w2 = 0; w2 < 4; ++w2) {
                wpre[w2] = acc;
                acc = u9_add(acc, wtot[w2]);
            }
            carry_s = reduce9(acc.w);
        }
        __syncthreads();
        const U9 pre = u9_add(u9_sub(tot, loc[T - 1]), wpre[wave]);
#pragma unroll
        for (int q = 0; q < T; ++q) {
            const uint32_t t0 = c0 + q * 256;                 // first term of this round
            if (t0 >= L) break;
            if (tid / TPR == (uint32_t)q) {
#pragma unroll
                for (int i = 0; i < T; ++i) {
                    const Fr si = reduce9(u9_add(loc[i], pre).w);
                    uint4* st3 = stage + (tid % TPR) * RS + i * 6;
                    st3[0] = make_uint4(a[i].w[0], a[i].w[1], a[i].w[2], a[i].w[3]);
                    st3[1] = make_uint4(a[i].w[4], a[i].w[5], a[i].w[6], a[i].w[7]);
                    st3[2] = make_uint4(w[i].w[0], w[i].w[1], w[i].w[2], w[i].w[3]);
                    st3[3] = make_uint4(w[i].w[4], w[i].w[5], w[i].w[6], w[i].w[7]);
                    st3[4] = make_uint4(si.w[0], si.w[1], si.w[2], si.w[3]);
                    st3[5] = make_uint4(si.w[4], si.w[5], si.w[6], si.w[7]);
                }
            }
            __syncthreads();
            const uint32_t ncell = 3 * min(256u, L - t0);
            uint4* o = reinterpret_cast<uint4*>(rowout + 1 + 3ull * t0);
            if constexpr (DIAG != 1)                       // 1: no cell stores
                for (uint32_t hc = tid; hc < 2 * ncell; hc += 256) o[hc] = stage[hc + hc / (6 * T)];
            __syncthreads();
        }
    }
    // row-end epilogues on the row total carry_s (written before the last barrier)
    if (J.pc && tid < 1 + kTabSlots) {
        const Fr v = carry_s;
        if (tid == 0) {
            st_fr(J.pc + r, v);
        } else {
            const uint32_t sl = tid - 1;
            const Fr x = mont_mul(v, B.f.f[sl]);
            Fr* base = J.ptab + 2ull * sl * J.plen;
            st_fr(base + r, x);
            if (sl < kTabSlots - 1) st_fr(base + J.plen + r, fr_neg(x));
        }
    }
    if (J.eq_out) {
        if (tid == 0) {
            const Fr x = carry_s, y = eqy;
            const Fr d = fr_sub(x, y), one = fr_from_u64(1);
            const bool z = fr_is_zero(d);
            const Fr zf = z ? one : zero;
            Fr inv = one;
            if (!z) inv = fr_inv(d);
            const Fr cell[12] = {d, y, one, x, zf, d, inv, one, zero, d, zf, zero};
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                stage[2 * k] = make_uint4(cell[k].w[0], cell[k].w[1], cell[k].w[2], cell[k].w[3]);
                stage[2 * k + 1] = make_uint4(cell[k].w[4], cell[k].w[5], cell[k].w[6], cell[k].w[7]);
            }
        }
        __syncthreads();
        if (tid < 24) reinterpret_cast<uint4*>(J.eq_out + 12ull * r)[tid] = stage[tid];
    }
}


// Wave-local variant (round 6): one block barrier per chunk (the wave totals)
// instead of six; the prefix carry stays unreduced (U9, < 2^268 for L <= 8192)
// so every wave derives it from the totals; each wave stages and stores its
// own 3 * 64T cells (two half-wave rounds through its own LDS slice, ordered by
// the wave's in-order LDS queue: no barrier).
template <int T, int NA, int DIAG>
__global__ __launch_bounds__(256, 4) void k_scan_wv(const ScanBatch B) {
    constexpr uint32_t WT = 64 * T;                       // terms per wave and chunk
    constexpr uint32_t RS = 6 * T + 1;                    // uint4 per staged lane (odd stride)
    __shared__ __attribute__((aligned(16))) uint4 stage[4][32 * RS];
    __shared__ U9 wtot[2][4];
    ScanJob J = B.job[0];
#pragma unroll
    for (int q = 1; q < kMaxScanJobs; ++q)
        if ((uint32_t)q < B.njobs && blockIdx.x >= B.job[q].blk0) J = B.job[q];
    const DView& A = J.A;
    const uint32_t L = J.L;
    const int na = batch_na<NA>(B);
    const Fr* __restrict__ wc = J.wc;
    const Fr* __restrict__ wm = tab_slot(J.tab, J.tl, na);
    const Fr* __restrict__ wn = wm + J.tl;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t lb = blockIdx.x - J.blk0;
    const uint32_t rb = (J.blk0 & 7) ? lb : scan_row(lb, J.rows), r = J.r_begin + rb;
    Fr* rowout = J.out + (uint64_t)rb * (3ull * L + 1);
    const Fr zero = fr_zero();
    Fr eqy = zero;
    if (tid == 0) {
        st_fr(rowout, zero);
        if (J.eq_out) eqy = ld_fr(J.eq_y + (uint64_t)r * J.eq_ys);
    }
    U9 carry = u9_from(zero);
    uint32_t par = 0;
    uint4* my = stage[wave];
    for (uint32_t c0 = 0; c0 < L; c0 += 256 * T, par ^= 1) {
        const uint32_t j0 = c0 + tid * T;
        Fr a[T], w[T], tm[T], tn[T], s[T];
#pragma unroll
        for (int i = 0; i < T; ++i) {
            const uint32_t j = j0 + i;
            const bool in = j < L;
            a[i] = in ? view_load(A, zero, r, j) : zero;
            w[i] = in ? ld_fr(wc + j) : zero;
            tm[i] = in ? ld_fr(wm + j) : zero;
            tn[i] = in && na < 8 ? ld_fr(wn + j) : zero;
        }
#pragma unroll
        for (int i = 0; i < T; ++i) s[i] = j0 + i < L ? scan_prod_pre<NA>(na, a[i], tm[i], tn[i]) : zero;
        U9 loc[T];
        loc[0] = u9_from(s[0]);
#pragma unroll
        for (int i = 1; i < T; ++i) loc[i] = u9_add(loc[i - 1], u9_from(s[i]));
        const U9 tot = wave_scan_u9(loc[T - 1]);
        if (lane == 63) wtot[par][wave] = tot;
        __syncthreads();                                  // the one block barrier of the chunk
        // (the carry and the wave's prefix are uniform: scalar registers)
        U9 pre = carry;
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2) {
            U9 t = wtot[par][w2];
#pragma unroll
            for (int k = 0; k < 9; ++k) t.w[k] = __builtin_amdgcn_readfirstlane(t.w[k]);
            if ((uint32_t)w2 < wave) pre = u9_add(pre, t);
            carry = u9_add(carry, t);
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            pre.w[k] = __builtin_amdgcn_readfirstlane(pre.w[k]);
            carry.w[k] = __builtin_amdgcn_readfirstlane(carry.w[k]);
        }
        pre = u9_add(u9_sub(tot, loc[T - 1]), pre);
        // this wave's terms [c0 + wave WT, + WT): two half-wave rounds
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t tb = c0 + wave * WT + h * 32 * T;   // first term of the round
            if (tb >= L) break;
            if ((lane >> 5) == (uint32_t)h) {
#pragma unroll
                for (int i = 0; i < T; ++i) {
                    const Fr si = reduce9(u9_add(loc[i], pre).w);
                    uint4* st3 = my + (lane & 31) * RS + i * 6;
                    st3[0] = make_uint4(a[i].w[0], a[i].w[1], a[i].w[2], a[i].w[3]);
                    st3[1] = make_uint4(a[i].w[4], a[i].w[5], a[i].w[6], a[i].w[7]);
                    st3[2] = make_uint4(w[i].w[0], w[i].w[1], w[i].w[2], w[i].w[3]);
                    st3[3] = make_uint4(w[i].w[4], w[i].w[5], w[i].w[6], w[i].w[7]);
                    st3[4] = make_uint4(si.w[0], si.w[1], si.w[2], si.w[3]);
                    st3[5] = make_uint4(si.w[4], si.w[5], si.w[6], si.w[7]);
                }
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t nt = min(32u * T, L - tb), nh = 6 * nt;      // 16 B halves of the round
            uint4* o = reinterpret_cast<uint4*>(rowout + 1 + 3ull * tb);
            if constexpr (DIAG != 1)
                for (uint32_t hc = lane; hc < nh; hc += 64) o[hc] = my[hc + hc / (6 * T)];
            __builtin_amdgcn_wave_barrier();
        }
    }
    // row-end epilogues on the row total
    if (J.pc && tid < 1 + kTabSlots) {
        const Fr v = reduce9(carry.w);
        if (tid == 0) {
            st_fr(J.pc + r, v);
        } else {
            const uint32_t sl = tid - 1;
            const Fr x = mont_mul(v, B.f.f[sl]);
            Fr* base = J.ptab + 2ull * sl * J.plen;
            st_fr(base + r, x);
            if (sl < kTabSlots - 1) st_fr(base + J.plen + r, fr_neg(x));
        }
    }
    if (J.eq_out) {
        __syncthreads();                                  // (stage is reused below)
        uint4* es = stage[0];
        if (tid == 0) {
            const Fr x = reduce9(carry.w), y = eqy;
            const Fr d = fr_sub(x, y), one = fr_from_u64(1);
            const bool z = fr_is_zero(d);
            const Fr zf = z ? one : zero;
            Fr inv = one;
            if (!z) inv = fr_inv(d);
            const Fr cell[12] = {d, y, one, x, zf, d, inv, one, zero, d, zf, zero};
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                es[2 * k] = make_uint4(cell[k].w[0], cell[k].w[1], cell[k].w[2], cell[k].w[3]);
                es[2 * k + 1] = make_uint4(cell[k].w[4], cell[k].w[5], cell[k].w[6], cell[k].w[7]);
            }
        }
        __syncthreads();
        if (tid < 24) reinterpret_cast<uint4*>(J.eq_out + 12ull * r)[tid] = es[tid];
    }
}
// BS threads per block (one chunk per 1024-term row at BS = 512: every load
// of the row issued before any store)
template <int T, int NA, int BS>
__global__ __launch_bounds__(BS) void k_scan_bs(const ScanBatch B) {
    static_assert(BS % T == 0, "T divides the block");
    constexpr uint32_t TPR = BS / T;                     // threads staged per round
    // a staging thread's 3T cells, padded by 16 B: a lane stride of 6T + 1
    // (odd) 16 B units keeps each b128 store pass on distinct bank groups
    constexpr uint32_t RS = 6 * T + 1;
    __shared__ __attribute__((aligned(16))) uint4 stage[TPR * RS];
    __shared__ U9 wtot[BS / 64], wpre[BS / 64];
    __shared__ Fr carry_s;
    ScanJob J = B.job[0];
#pragma unroll
    for (int q = 1; q < kMaxScanJobs; ++q)
        if ((uint32_t)q < B.njobs && blockIdx.x >= B.job[q].blk0) J = B.job[q];
    const DView& A = J.A;
    const uint32_t L = J.L;
    const int na = batch_na<NA>(B);
    const Fr* __restrict__ wc = J.wc;
    const Fr* __restrict__ wm = tab_slot(J.tab, J.tl, na);
    const Fr* __restrict__ wn = wm + J.tl;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t lb = blockIdx.x - J.blk0;
    const uint32_t rb = (J.blk0 & 7) ? lb : scan_row(lb, J.rows), r = J.r_begin + rb;
    Fr* rowout = J.out + (uint64_t)rb * (3ull * L + 1);
    const Fr zero = fr_zero();
    Fr eqy = zero;                                        // is_equal's y, loaded ahead
    if (tid == 0) {
        st_fr(rowout, zero);
        carry_s = zero;
        if (J.eq_out) eqy = ld_fr(J.eq_y + (uint64_t)r * J.eq_ys);
    }
    for (uint32_t c0 = 0; c0 < L; c0 += BS * T) {
        const uint32_t j0 = c0 + tid * T;
        // every load of the chunk issued together (the row operand, both table
        // entries, the vector's canonical cell): one memory round trip per
        // chunk instead of three dependent ones, which beside a saturating cell
        // stream cost microseconds each
        Fr a[T], w[T], tm[T], tn[T], s[T];
#pragma unroll
        for (int i = 0; i < T; ++i) {
            const uint32_t j = j0 + i;
            const bool in = j < L;
            a[i] = in ? view_load(A, zero, r, j) : zero;
            w[i] = in ? ld_fr(wc + j) : zero;
            tm[i] = in ? ld_fr(wm + j) : zero;
            tn[i] = in && na < 8 ? ld_fr(wn + j) : zero;
        }
#pragma unroll
        for (int i = 0; i < T; ++i) s[i] = j0 + i < L ? scan_prod_pre<NA>(na, a[i], tm[i], tn[i]) : zero;
        // local inclusive sums (< T p), the wave scan and the prefixes stay
        // unreduced (exact, < 2^265); each output is reduced once
        U9 loc[T];
        loc[0] = u9_from(s[0]);
#pragma unroll
        for (int i = 1; i < T; ++i) loc[i] = u9_add(loc[i - 1], u9_from(s[i]));
        const U9 tot = wave_scan_u9(loc[T - 1]);
        if (lane == 63) wtot[wave] = tot;
        __syncthreads();
        if (tid == 0) {                                   // wave prefixes and the running carry
            U9 acc = u9_from(carry_s);
#pragma unroll
            for (int w2 = 0; w2 < BS / 64; ++w2) {
                wpre[w2] = acc;
                acc = u9_add(acc, wtot[w2]);
            }
            carry_s = reduce9(acc.w);
        }
        __syncthreads();
        const U9 pre = u9_add(u9_sub(tot, loc[T - 1]), wpre[wave]);
#pragma unroll
        for (int q = 0; q < T; ++q) {
            const uint32_t t0 = c0 + q * BS;                 // first term of this round
            if (t0 >= L) break;
            if (tid / TPR == (uint32_t)q) {
#pragma unroll
                for (int i = 0; i < T; ++i) {
                    const Fr si = reduce9(u9_add(loc[i], pre).w);
                    uint4* st3 = stage + (tid % TPR) * RS + i * 6;
                    st3[0] = make_uint4(a[i].w[0], a[i].w[1], a[i].w[2], a[i].w[3]);
                    st3[1] = make_uint4(a[i].w[4], a[i].w[5], a[i].w[6], a[i].w[7]);
                    st3[2] = make_uint4(w[i].w[0], w[i].w[1], w[i].w[2], w[i].w[3]);
                    st3[3] = make_uint4(w[i].w[4], w[i].w[5], w[i].w[6], w[i].w[7]);
                    st3[4] = make_uint4(si.w[0], si.w[1], si.w[2], si.w[3]);
                    st3[5] = make_uint4(si.w[4], si.w[5], si.w[6], si.w[7]);
                }
            }
            __syncthreads();
            const uint32_t ncell = 3 * min((uint32_t)BS, L - t0);
            uint4* o = reinterpret_cast<uint4*>(rowout + 1 + 3ull * t0);
                for (uint32_t hc = tid; hc < 2 * ncell; hc += BS) o[hc] = stage[hc + hc / (6 * T)];
            __syncthreads();
        }
    }
    // row-end epilogues on the row total carry_s (written before the last barrier)
    if (J.pc && tid < 1 + kTabSlots) {
        const Fr v = carry_s;
        if (tid == 0) {
            st_fr(J.pc + r, v);
        } else {
            const uint32_t sl = tid - 1;
            const Fr x = mont_mul(v, B.f.f[sl]);
            Fr* base = J.ptab + 2ull * sl * J.plen;
            st_fr(base + r, x);
            if (sl < kTabSlots - 1) st_fr(base + J.plen + r, fr_neg(x));
        }
    }
    if (J.eq_out) {
        if (tid == 0) {
            const Fr x = carry_s, y = eqy;
            const Fr d = fr_sub(x, y), one = fr_from_u64(1);
            const bool z = fr_is_zero(d);
            const Fr zf = z ? one : zero;
            Fr inv = one;
            if (!z) inv = fr_inv(d);
            const Fr cell[12] = {d, y, one, x, zf, d, inv, one, zero, d, zf, zero};
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                stage[2 * k] = make_uint4(cell[k].w[0], cell[k].w[1], cell[k].w[2], cell[k].w[3]);
                stage[2 * k + 1] = make_uint4(cell[k].w[4], cell[k].w[5], cell[k].w[6], cell[k].w[7]);
            }
        }
        __syncthreads();
        if (tid < 24) reinterpret_cast<uint4*>(J.eq_out + 12ull * r)[tid] = stage[tid];
    }
}
}  // namespace svdw
using namespace svdw;

static void rnd_fr(std::vector<uint32_t>& v, size_t n, uint64_t seed, int words) {
    v.assign(n * 8, 0u);
    uint64_t s = seed;
    for (size_t i = 0; i < n; ++i)
        for (int w = 0; w < words; ++w) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            v[i * 8 + w] = (uint32_t)(s >> 16);
        }
    if (words == 8)
        for (size_t i = 0; i < n; ++i) v[i * 8 + 7] &= 0x0fffffffu;     // < 2^252 < p
}

int main(int argc, char** argv) {
    const uint32_t J = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint32_t N = 1024, L = 1024;
    std::vector<uint32_t> h;
    Fr *A, *wc, *tab, *out;
    CK(hipMalloc(&A, (size_t)N * L * 32));
    rnd_fr(h, (size_t)N * L, 11, 2);                  // |a| < 2^64
    CK(hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&wc, (size_t)L * 32));
    rnd_fr(h, L, 12, 8);
    CK(hipMemcpy(wc, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&tab, tab_len(L) * 32));
    rnd_fr(h, tab_len(L), 13, 8);
    CK(hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const size_t cells = (size_t)J * N * (3 * L + 1);
    CK(hipMalloc(&out, cells * 32));
    ScanBatch b;
    memset(&b, 0, sizeof b);
    b.njobs = J;
    for (uint32_t q = 0; q < J; ++q) {
        ScanJob& j = b.job[q];
        j.A.ptr = A; j.A.rs = L; j.A.cs = 1; j.A.rows = N; j.A.cols = L; j.A.mode = VIEW_STRIDED;
        j.wc = wc; j.tab = tab; j.tl = L; j.out = out + (size_t)q * N * (3 * L + 1);
        j.L = L; j.rows = N; j.blk0 = q * N; j.r_begin = 0;
        j.spec = NaSpec{-2, -1, 64, 0};
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    constexpr int NV = 7;
    const char* name[NV] = {"shipped", "no-stores", "no-loads", "launcher", "wave-local", "wl-nostores",
                            "512-thread"};
    double best[NV] = {1e9, 1e9, 1e9, 1e9, 1e9, 1e9, 1e9};
    std::vector<uint32_t> ref;
    for (int round = 0; round < 3; ++round)
        for (int v = 0; v < NV; ++v) {
            auto go = [&] {
                const dim3 g(J * N), blk(256);
                if (v == 0) hipLaunchKernelGGL((k_scan_diag<2, 0, 0>), g, blk, 0, 0, b);
                else if (v == 1) hipLaunchKernelGGL((k_scan_diag<2, 0, 1>), g, blk, 0, 0, b);
                else if (v == 2) hipLaunchKernelGGL((k_scan_diag<2, 0, 2>), g, blk, 0, 0, b);
                else if (v == 3) CK(launch_scan_batch(b, 0, 0));
                else if (v == 4) hipLaunchKernelGGL((k_scan_wv<2, 0, 0>), g, blk, 0, 0, b);
                else if (v == 5) hipLaunchKernelGGL((k_scan_wv<2, 0, 1>), g, blk, 0, 0, b);
                else hipLaunchKernelGGL((k_scan_bs<2, 0, 512>), g, dim3(512), 0, 0, b);
            };
            if (round == 0 && (v == 0 || v == 4 || v == 6)) {       // cells of the real variants must agree
                CK(hipMemset(out, 0, cells * 32));
                go();
                CK(hipDeviceSynchronize());
                std::vector<uint32_t> got(cells * 8);
                CK(hipMemcpy(got.data(), out, cells * 32, hipMemcpyDeviceToHost));
                if (v == 0) ref.swap(got);
                else {
                    size_t bad = 0;
                    for (size_t i = 0; i < got.size(); ++i) bad += got[i] != ref[i];
                    printf("%s cells differing words vs shipped: %zu of %zu\n", name[v], bad, got.size());
                }
            }
            for (int w = 0; w < 2; ++w) go();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (uint32_t r = 0; r < reps; ++r) go();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best[v] = std::min(best[v], (double)ms * 1e3 / reps);
        }
    for (int v = 0; v < NV; ++v)
        printf("scan %u jobs x %u rows x %u terms  %-10s %8.1f us  %6.0f GB/s of cells\n", J, N, L, name[v], best[v],
               cells * 32.0 / (best[v] * 1e-6) / 1e9);
    return 0;
}
