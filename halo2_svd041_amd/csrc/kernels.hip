// gfx950 (CDNA4) kernels of the SVD-verify witness engine.
//
//  k_quantize      ZkMatrix::new / ZkVector::new cells   (src/matrix/mod.rs:29-40, 230-252)
//  k_stage         every gadget block of check_svd_phase0 / verify_mul except
//                  the GEMM and the inner-product rows: one cell program per
//                  stage (prog.hpp), HBM-write bound, 16 B/lane coalesced stores
//  k_to_digits +   honest_prover_mat_mul / field_mat_mul (src/matrix/mod.rs:510-568)
//  k_gemm_dot4     as an exact signed-integer GEMM on v_dot4c_i32_i8 over
//                  balanced base-256 digit planes, one reduction mod p per output
//  k_gemm_mont     generic Montgomery fallback (operands not small integers)
//  k_matvec_scan   field_mat_vec_mul rows (src/matrix/mod.rs:574-599): every
//                  prefix sum of the row inner product is a cell -> block Fr scan
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <type_traits>
#include <string.h>

#include "kernels.hpp"
#include "crt_tables.hpp"

namespace svdw {

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ Fr ld_fr(const Fr* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    Fr r;
    r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w;
    r.w[4] = b.x; r.w[5] = b.y; r.w[6] = b.z; r.w[7] = b.w;
    return r;
}
__device__ __forceinline__ void st_fr(Fr* p, const Fr& v) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
    q[1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
}
// ZkMatrix::new's quantization of one f64 (quantize_body's arithmetic):
// x_q = round_half_away(|x| 2^P) as u128 (saturating, NaN -> 0), sign(x) < 0
// (incl. -0.0) -> p - x_q.
__device__ __forceinline__ Fr quantize_fr(double x, double scale) {
    const bool neg = signbit(x) && !isnan(x);
    const double s = round(fabs(x) * scale);
    Fr q = fr_zero();
    if (s >= 340282366920938463463374607431768211456.0) {
        q.w[0] = q.w[1] = q.w[2] = q.w[3] = 0xffffffffu;
    } else if (s > 0.0) {
        const uint64_t bits = __double_as_longlong(s);
        const int e = (int)((bits >> 52) & 0x7ff) - 1075;
        const uint64_t mant = (bits & 0xfffffffffffffull) | (1ull << 52);
        const unsigned __int128 v = e >= 0 ? ((unsigned __int128)mant << e) : (unsigned __int128)(mant >> -e);
        q.w[0] = (uint32_t)v; q.w[1] = (uint32_t)(v >> 32);
        q.w[2] = (uint32_t)(v >> 64); q.w[3] = (uint32_t)(v >> 96);
    }
    return neg ? fr_sub(fr_zero(), q) : q;
}
__device__ __forceinline__ double f64_scale(const DView& v) { return ldexp(1.0, (int)v._r0); }
// X(i, j) of a view; `pad` is the value outside the view (K[v.pad_k]).
__device__ __forceinline__ Fr view_load(const DView v, const Fr pad, uint32_t i, uint32_t j) {
    if (v.mode == VIEW_DIAG) return (i == j) ? ld_fr(v.ptr) : pad;
    if (v.mode == VIEW_F64) {
        if (i < v.rows && j < v.cols)
            return quantize_fr(reinterpret_cast<const double*>(v.ptr)[(int64_t)i * v.rs + (int64_t)j * v.cs],
                               f64_scale(v));
        return pad;
    }
    if (i < v.rows && j < v.cols) return ld_fr(v.ptr + (int64_t)i * v.rs + (int64_t)j * v.cs);
    return pad;
}
__device__ __forceinline__ uint32_t signed_bits(const Fr& x) {
    // bit length of |x| where x is read as the signed representative in (-p/2, p/2]
    Fr half = fr_p();
    // (p-1)/2
    uint32_t c = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
        uint32_t nw = (half.w[i] >> 1) | c;
        c = half.w[i] << 31;
        half.w[i] = nw;
    }
    Fr t;
    bool neg = sub256(t, half, x) != 0;   // x > (p-1)/2
    Fr mag = neg ? fr_sub(fr_zero(), x) : x;
    uint32_t bits = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i)
        if (bits == 0 && mag.w[i]) bits = 32 * i + 32 - __clz(mag.w[i]);
    return bits;
}

// --------------------------------------------------------------- quantize
// x_q = round_half_away(|x| * 2^P) as u128 (saturating, NaN -> 0);
// sign(x) < 0 (incl. -0.0) -> p - x_q.   [zk_fixed_point_chip quantization,
// SURVEY.md Appendix C.1]
// Fold of the block maxima inside the quantize launch (BitFold), fence-free:
// each block publishes its maximum with an agent-scope atomic exchange and
// arrives on its group's counter (group = blk & 7) only once the exchange has
// returned (the register use below makes the arrival wait for it); the last
// arrival of a group arrives on the global counter, the last of those sees
// every maximum with agent-scope loads. An agent-scope release fence instead
// writes back the whole L2 (the block's cells) per block: 670 us instead of 19.
// Hardware assumption (gfx950, several XCDs with their own L2): agent-scope
// atomics are performed at the device coherence point, not in an XCD's L2, so
// a maximum exchanged before the arrival is what the last block's agent-scope
// load returns; the last arrival's counter update is an acquire besides.
// Called after the block's stores are issued, so its latency overlaps them.
__device__ __forceinline__ void bits_fold(const BitFold& f, uint32_t blk, uint32_t bmax) {
    __shared__ uint32_t last, red[4][4];
    if (threadIdx.x == 0) {
        const uint32_t g = blk & 7, gsize = (f.nblk - g + 7) / 8;
        const uint32_t old = __hip_atomic_exchange(f.bm + blk, bmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(old) : "memory");
        bool lst = __hip_atomic_fetch_add(f.cnt + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1;
        if (lst) {
            __hip_atomic_store(f.cnt + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t ng = min(f.nblk, 8u);
            // acquire on the last arrival only (a cache invalidate, no write-back)
            lst = __hip_atomic_fetch_add(f.cnt, 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
        }
        last = lst;
    }
    __syncthreads();
    if (!last) return;
    uint32_t x[3] = {0u, 0u, 0u};
    for (uint32_t k0 = threadIdx.x; k0 < f.nblk; k0 += 8 * blockDim.x) {
        uint32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t k = k0 + q * blockDim.x;
            v[q] = k < f.nblk ? __hip_atomic_load(f.bm + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t k = k0 + q * blockDim.x;
#pragma unroll
            for (int s = 0; s < 3; ++s)
                if (k >= f.b[s] && k < f.b[s + 1]) x[s] = max(x[s], v[q]);
        }
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x[s] = max(x[s], (uint32_t)__shfl_xor((int)x[s], off));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][s] = x[s];
    }
    __syncthreads();
    if (threadIdx.x < f.nred) {
        const uint32_t s = threadIdx.x;
        f.wout[s] = max(max(red[0][s], red[1][s]), max(red[2][s], red[3][s]));
    }
    if (threadIdx.x == 0) __hip_atomic_store(f.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// bit length of |x_q| over a block's values (for the GEMM modulus count):
// thread max -> wave max -> block max (LDS)
template <int PT>
__device__ __forceinline__ uint32_t block_bits(const double (&xv)[PT], double scale) {
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const double s = round(fabs(xv[k]) * scale);
        if (s >= 340282366920938463463374607431768211456.0) bits = 128;
        else if (s >= 1.0) bits = max(bits, (uint32_t)ilogb(s) + 1);
    }
    __shared__ uint32_t wmax[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) bits = max(bits, (uint32_t)__shfl_xor((int)bits, off));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = bits;
    __syncthreads();
    return max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
}
// PT * 256 values per block, PT per thread (value blk * PT * 256 + k * 256 +
// tid: each store instruction coalesced), all loads issued first.
template <int PT>
__device__ __forceinline__ void quantize_body(const double* __restrict__ in, uint64_t n,
                                              Fr* __restrict__ out, double scale,
                                              unsigned* __restrict__ blockmax, uint32_t blk,
                                              QuantKeep keep = QuantKeep{0, 0, 0, 0, 0},
                                              const BitFold fold = BitFold{}, uint32_t gblk = 0) {
    const uint64_t i0 = (uint64_t)blk * (PT * 256) + threadIdx.x;
    uint32_t bmax = 0;
    double xv[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const uint64_t i = i0 + 256ull * k;
        xv[k] = i < n ? in[i] : 0.0;
    }
    if (blockmax) {
        bmax = block_bits<PT>(xv, scale);
        if (!(fold.wout && gblk < fold.nblk) && threadIdx.x == 0) blockmax[blk] = bmax;
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const uint64_t i = i0 + 256ull * k;
        if (i >= n) continue;
        if (keep.cols) {                                  // partial store (row-sharded rank)
            const uint32_t r = (uint32_t)(i / keep.cols), cc = (uint32_t)(i - (uint64_t)r * keep.cols);
            if (!((r >= keep.rlo && r < keep.rhi) || (cc >= keep.clo && cc < keep.chi))) continue;
        }
        st_fr(out + i, quantize_fr(xv[k], scale));    // (L2 joins the two halves of a line)
    }
    if (blockmax && fold.wout && gblk < fold.nblk) bits_fold(fold, gblk, bmax);
}
__global__ __launch_bounds__(256) void k_quantize(const double* __restrict__ in, uint64_t n,
                                                  Fr* __restrict__ out, double scale,
                                                  unsigned* __restrict__ blockmax) {
    quantize_body<kQuantPerBlock / 256>(in, n, out, scale, blockmax, blockIdx.x);
}
// m, u, v, d in one launch (their ZkMatrix::new calls are back to back,
// examples/svd_example.rs:138-144): one ramp-up / tail instead of four.
template <int PT>
__global__ __launch_bounds__(256) void k_quantize_multi(const QuantSegs q, double scale) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 1; k < kMaxQuantSegs; ++k) s += (uint32_t)k < q.nseg && blockIdx.x >= q.blk0[k];
    const double* in = q.in[0];
    Fr* out = q.out[0];
    unsigned* bm = q.blockmax[0];
    uint64_t n = q.n[0];
    uint32_t b0 = q.blk0[0];
    QuantKeep keep = q.keep[0];
#pragma unroll
    for (int k = 1; k < kMaxQuantSegs; ++k)      // selects, not a dynamic index into the argument
        if (s == (uint32_t)k) {
            in = q.in[k]; out = q.out[k]; bm = q.blockmax[k]; n = q.n[k]; b0 = q.blk0[k]; keep = q.keep[k];
        }
    quantize_body<PT>(in, n, out, scale, bm, blockIdx.x - b0, keep, q.fold, blockIdx.x);
}
hipError_t launch_quantize_multi(const QuantSegs& q, int p, hipStream_t st) {
    if (!q.nseg || q.nseg > (uint32_t)kMaxQuantSegs || !q.blk0[q.nseg]) return hipErrorInvalidValue;
    const uint32_t pb = q.per_block ? q.per_block : kQuantPerBlock;
    if (pb == kQuantPerBlockSmall)
        hipLaunchKernelGGL(k_quantize_multi<kQuantPerBlockSmall / 256>, dim3(q.blk0[q.nseg]), dim3(256), 0, st, q,
                           (double)(1ull << p));
    else if (pb == kQuantPerBlock)
        hipLaunchKernelGGL(k_quantize_multi<kQuantPerBlock / 256>, dim3(q.blk0[q.nseg]), dim3(256), 0, st, q,
                           (double)(1ull << p));
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_quantize(const double* in, uint64_t n, Fr* out, int p, unsigned* blockmax,
                           hipStream_t st) {
    if (!n) return hipSuccess;
    double scale = (double)(1ull << p);
    hipLaunchKernelGGL(k_quantize, dim3((unsigned)((n + kQuantPerBlock - 1) / kQuantPerBlock)), dim3(256), 0, st, in, n, out,
                       scale, blockmax);
    return hipGetLastError();
}
// block s: out[s] = max(blockmax[seg.begin[s] .. seg.begin[s + 1]))
__global__ __launch_bounds__(256) void k_bits_reduce(const unsigned* __restrict__ blockmax,
                                                     const BitSegs seg, unsigned* __restrict__ out) {
    __shared__ uint32_t wmax[4];
    const uint32_t s = blockIdx.x;
    uint32_t b = 0;
    for (uint32_t i = seg.begin[s] + threadIdx.x; i < seg.begin[s + 1]; i += 256) b = max(b, blockmax[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, off));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) out[s] = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
}
// Timing aid ("hold_us"): one wave spinning ~us microseconds on the device clock
// (s_memrealtime, 100 MHz) so the host finishes enqueueing before the step runs.
__global__ void k_hold(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
hipError_t launch_hold(uint32_t us, hipStream_t st) {
    hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, st, (uint64_t)us * 100u);
    return hipGetLastError();
}
hipError_t launch_bits_reduce(const unsigned* blockmax, const BitSegs& seg, uint32_t nseg,
                              unsigned* out, hipStream_t st) {
    if (!nseg || nseg >= (uint32_t)kMaxBitSegs) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bits_reduce, dim3(nseg), dim3(256), 0, st, blockmax, seg, out);
    return hipGetLastError();
}

// x mod p for a 9-word x < 2^270
__device__ __forceinline__ Fr reduce9(const uint32_t (&x)[9]) {
    const double two32 = 4294967296.0;
    // 1 / (p / 2^192): quotient estimate within 2 of floor(x / p) (x < 2^270)
    constexpr double inv_pd = 1.0 / (((double)0x30644e72u * 4294967296.0 + (double)0xe131a029u) +
                                     (double)0xb85045b6u / 4294967296.0);
    const double xd = ((double)x[8] * two32 + (double)x[7]) * two32 + (double)x[6];
    const double qd = floor(xd * inv_pd) - 1.0;
    const uint32_t q = qd > 0.0 ? (uint32_t)qd : 0u;
    Fr r;
    uint32_t carry = 0, br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t pr = (uint64_t)q * p_word(i) + carry;   // v_mad_u64_u32
        carry = (uint32_t)(pr >> 32);
        r.w[i] = subb32(x[i], (uint32_t)pr, br);
    }
    // x - q p < 3p < 2^256: the ninth word is gone; two conditional subtractions
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        Fr t;
        const uint32_t b = sub_p(t, r);
#pragma unroll
        for (int i = 0; i < 8; ++i) r.w[i] = b ? r.w[i] : t.w[i];
    }
    return r;
}

// ----------------------------------------------------------- stage kernel
// Phase A: one thread per element (kStageElems = 256 = block size) runs the
// stage's micro-ops, leaving the element's values V[0..nv) (8 words each) in
// LDS. Phase B: the block's E*C advice cells (then E*L lookup cells) are
// produced half a cell (16 B) per lane in stream order, so every wave store
// is 1 KiB contiguous: cell = (V[src] >> lo) & (2^nbits - 1).
constexpr int VW = 8;    // LDS words per value

__device__ __forceinline__ void lds_put(uint32_t* s, const Fr& v) {
    uint4* q = reinterpret_cast<uint4*>(s);
    q[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
    q[1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
}
__device__ __forceinline__ Fr lds_get(const uint32_t* s) {
    const uint4* q = reinterpret_cast<const uint4*>(s);
    uint4 a = q[0], b = q[1];
    Fr r;
    r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w;
    r.w[4] = b.x; r.w[5] = b.y; r.w[6] = b.z; r.w[7] = b.w;
    return r;
}

// Output words [4h, 4h+4) of (S >> lo) & mask(nbits), S = 8 LDS words at s;
// words past the top read as 0 (reads are clamped in-bounds, then masked).
__device__ __forceinline__ uint4 extract_half(const uint32_t* s, uint32_t lo, uint32_t nbits,
                                              uint32_t h) {
    const uint32_t q = (lo >> 5) + 4 * h, r = lo & 31;
    uint32_t x[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t w = q + i;
        const uint32_t v = s[w < 8 ? w : 7];
        x[i] = w < 8 ? v : 0u;
    }
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbit(x[i + 1], x[i], r);
    if (nbits) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int keep = (int)nbits - 32 * (4 * (int)h + i);
            const uint32_t m = keep >= 32 ? 0xffffffffu : (keep <= 0 ? 0u : ((1u << keep) - 1u));
            o[i] &= m;
        }
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// LDS carve (bytes, all 16-aligned): consts | element values | slot ops | micro-ops | views

// x / d for x * d < 2^32 via one 32-bit mul_hi (magic = ceil(2^32 / d), d >= 2).
__device__ __forceinline__ uint32_t fastdiv(uint32_t x, uint32_t d, uint32_t magic) {
    return d == 1 ? x : __umulhi(x, magic);
}

// Phase B: per-(slot, half) descriptors and masks prepared once per block
// (half_desc, prog.hpp), so a half-cell costs one descriptor + one mask LDS
// read, five word reads, four alignbit and four and (no per-cell decoding,
// clamping or mask arithmetic). The (element, slot) of the lane's next cell is
// tracked incrementally (the cell index advances by blockDim / 2 per step).
// ALIGN: the block's iterations cover whole (blockDim * 16 B)-aligned address
// windows (the first one partially), so every wave store is one aligned 1 KiB.
// Half-cells [.., hc_end) of the windows from the one holding hc_begin on (hc_begin
// is this lane's first half-cell: lane tid's half-cells are hc_begin + k * blockDim).
__device__ __forceinline__ void stream_cells_run(uint4* __restrict__ out, uint32_t hc_begin, uint32_t hc_end,
                                                 const uint32_t* __restrict__ sHD,
                                                 const uint4* __restrict__ sHM, uint32_t C, uint32_t magic,
                                                 const uint32_t* smem, uint32_t vbase0, uint32_t nv) {
    const uint32_t h = threadIdx.x & 1, step = blockDim.x >> 1;
    const uint32_t dq = step / C, dr = step - dq * C, ev = stage_elem_words(nv);
    uint32_t c = hc_begin >> 1;
    uint32_t el = fastdiv(c, C, magic), slot = c - el * C;
    uint32_t vbase = vbase0 + el * ev;                    // LDS word of this element's values
    for (uint32_t hc = hc_begin; hc < hc_end; hc += blockDim.x) {
        const uint32_t k = 2 * slot + h;
        const uint32_t d = sHD[k];
        const uint4 m = sHM[k];
        const uint32_t wo = ((d & kHalfElem) ? vbase : 0u) + (d & 0xffffu);
        const uint32_t r = (d >> 16) & 31u;
        const uint32_t* x = smem + wo;
        const uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3], x4 = x[4];
        const uint4 v = make_uint4(__builtin_amdgcn_alignbit(x1, x0, r) & m.x,
                                   __builtin_amdgcn_alignbit(x2, x1, r) & m.y,
                                   __builtin_amdgcn_alignbit(x3, x2, r) & m.z,
                                   __builtin_amdgcn_alignbit(x4, x3, r) & m.w);
        out[hc] = v;
        slot += dr;
        vbase += dq * ev;
        if (slot >= C) {
            slot -= C;
            vbase += ev;
        }
    }
}
// rot: the block starts at window rot mod (its window count) and wraps around
// ("stage_rot"), so that blocks started together do not all write the same
// window offset of their chunks at the same time.
template <bool ALIGN>
__device__ __forceinline__ void stream_cells_desc(uint4* __restrict__ out, uint32_t total,
                                                  const uint32_t* __restrict__ sHD,
                                                  const uint4* __restrict__ sHM, uint32_t C,
                                                  uint32_t magic, const uint32_t* smem,
                                                  uint32_t vbase0, uint32_t nv, uint32_t rot = 0) {
    const uint32_t B = blockDim.x, tid = threadIdx.x;
    const uint32_t mis = ALIGN ? (uint32_t)(reinterpret_cast<uintptr_t>(out) >> 4) & (B - 1) : 0u;
    // lane tid's half-cells: tid - mis + k B (k >= 0, >= 0); window k holds
    // [k B - mis, (k + 1) B - mis)
    const uint32_t first = tid >= mis ? tid - mis : tid + B - mis;
    const uint32_t nw = (total + mis + B - 1) / B;
    const uint32_t r = nw > 1 ? rot % nw : 0u;
    if (!r) {
        stream_cells_run(out, first, total, sHD, sHM, C, magic, smem, vbase0, nv);
        return;
    }
    const uint32_t cut = r * B - mis;                     // first half-cell of window r
    stream_cells_run(out, cut + tid, total, sHD, sHM, C, magic, smem, vbase0, nv);
    stream_cells_run(out, first, cut, sHD, sHM, C, magic, smem, vbase0, nv);
}

// Descriptor and masks of half h of a slot (see half_desc).
__device__ __forceinline__ void make_half(const SlotOp op, uint32_t h, uint32_t* d, uint4* m) {
    const uint32_t lo = op.lo;
    uint32_t nb = op.nbits ? op.nbits : 256u;
    nb = min(nb, 256u - lo);
    const bool elem = op.src < KSRC;
    const uint32_t base = (elem ? op.src : op.src - KSRC) * VW;
    *d = half_desc(base + (lo >> 5) + 4 * h, lo & 31u, elem);
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int keep = (int)nb - 32 * (4 * (int)h + i);
        w[i] = keep >= 32 ? 0xffffffffu : (keep <= 0 ? 0u : ((1u << keep) - 1u));
    }
    *m = make_uint4(w[0], w[1], w[2], w[3]);
}

// a * b mod p for canonical a, b. Fast path when both signed representatives
// (x or x - p) are below 2^128 in magnitude -- quantized cells always are (the
// u128 saturation of ZkMatrix::new), e.g. mat_times_diag_mat's u_ij * d_j:
// an exact 4 x 4-word product (< 2^256 < 6p), a quotient-estimate reduction and
// a conditional negation instead of two full Montgomery products.
__device__ __forceinline__ Fr fr_mul_any(const Fr& a, const Fr& b) {
    Fr na, nb;
    sub256(na, fr_p(), a);                              // p - a
    sub256(nb, fr_p(), b);
    const bool sa = a.w[7] != 0, sb = b.w[7] != 0;     // top word set: the negative side
    uint32_t ma[4], mb[4], hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ma[i] = sa ? na.w[i] : a.w[i];
        mb[i] = sb ? nb.w[i] : b.w[i];
    }
#pragma unroll
    for (int i = 4; i < 8; ++i) hi |= (sa ? na.w[i] : a.w[i]) | (sb ? nb.w[i] : b.w[i]);
    if (__any(hi != 0)) {                               // some lane out of range: generic
        if (hi) return fr_mul(a, b);
    }
    uint32_t t[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) t[i + j] = mac32(ma[i], mb[j], t[i + j], c);
        t[i + 4] = c;
    }
    const Fr r = reduce9(t);                            // < 2^256 -> mod p
    return (sa != sb) ? fr_neg(r) : r;
}

// Phase A for one element: run the stage's micro-ops, values into myV (LDS).
__device__ __forceinline__ void element_program(const StageArgs& a, uint32_t e, uint32_t* myV,
                                                const uint32_t* sK, const MicroOp* sMo,
                                                const DView* sVw, const Fr& pf0, bool in0,
                                                const Fr& pf1, bool in1) {
    const uint32_t i = e / a.cols, j = e - (e / a.cols) * a.cols;
    for (uint32_t m = 0; m < a.nmo; ++m) {
        const MicroOp op = sMo[m];
        uint32_t* dst = myV + op.dst * VW;
        switch (op.op) {
            case MO_LOAD: {
                if (op.a == 0 && in0) {
                    lds_put(dst, pf0);
                } else if (op.a == 1 && in1) {
                    lds_put(dst, pf1);
                } else {
                    const DView vw = sVw[op.a];
                    if (vw.mode == VIEW_DIAGK)
                        lds_put(dst, lds_get(sK + (i == j ? vw.diag_k : vw.pad_k) * VW));
                    else
                        lds_put(dst, view_load(vw, lds_get(sK + vw.pad_k * VW), i, j));
                }
                break;
            }
            case MO_ADDK:
                lds_put(dst, fr_add(lds_get(myV + op.a * VW), lds_get(sK + op.b * VW)));
                break;
            case MO_SUB:
                lds_put(dst, fr_sub(lds_get(myV + op.a * VW), lds_get(myV + op.b * VW)));
                break;
            case MO_MUL:
                lds_put(dst, fr_mul_any(lds_get(myV + op.a * VW), lds_get(myV + op.b * VW)));
                break;
            case MO_LIMBSHL: {
                const Fr sv = lds_get(myV + op.a * VW);
                // 64-bit window at bit p0 (p0 < 256), masked to p1 bits, << b
                const uint32_t lo = op.p0, q = lo >> 5, r = lo & 31;
                uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    w0 = (t == (int)q) ? sv.w[t] : w0;
                    w1 = (t == (int)q + 1) ? sv.w[t] : w1;
                    w2 = (t == (int)q + 2) ? sv.w[t] : w2;
                }
                const uint64_t w01 = (uint64_t)w0 | ((uint64_t)w1 << 32);
                uint64_t x = r ? ((w01 >> r) | ((uint64_t)w2 << (64 - r))) : w01;
                if (op.p1 < 64) x &= (1ull << op.p1) - 1;
                const uint32_t sh = op.b;
                const uint64_t lo64 = sh < 64 ? (x << sh) : 0;
                const uint64_t hi64 = sh == 0 ? 0 : (sh < 64 ? (x >> (64 - sh)) : (x << (sh - 64)));
                Fr v = fr_zero();
                v.w[0] = (uint32_t)lo64; v.w[1] = (uint32_t)(lo64 >> 32);
                v.w[2] = (uint32_t)hi64; v.w[3] = (uint32_t)(hi64 >> 32);
                lds_put(dst, v);
                break;
            }
            case MO_FDBL: {
                Fr v = lds_get(myV + op.a * VW);
                for (uint32_t t = 0; t < op.b; ++t) v = fr_add(v, v);
                lds_put(dst, v);
                break;
            }
            case MO_ISZERO: {
                const Fr v = lds_get(myV + op.a * VW);
                const bool z = fr_is_zero(v);
                // the exponentiation only where some lane needs it (honest
                // is_equal rows are all zero): a select would always run it
                Fr inv = fr_from_u64(1);
                if (__any(!z)) {
                    // word by word: `inv = z ? inv : t` on whole structs compiled
                    // to a select between two stack copies (scratch, 80 B / lane)
                    const Fr t = fr_inv(v);
#pragma unroll
                    for (int w = 0; w < 8; ++w) inv.w[w] = z ? inv.w[w] : t.w[w];
                }
                lds_put(dst, fr_from_u64(z ? 1 : 0));
                lds_put(dst + VW, inv);
                break;
            }
            case MO_POWK: {
                const uint64_t x = (uint64_t)e + op.p0;       // square-and-multiply over its bits only
                lds_put(dst, fr_pow_u64(lds_get(sK + op.a * VW), x, x ? 64 - __clzll(x) : 1));
                break;
            }
            case MO_ISQRT: {
                // bit by bit from 2^127 down: keep the bit when (y | b)^2 <= v
                const Fr v = lds_get(myV + op.a * VW);
                uint32_t y[4] = {0u, 0u, 0u, 0u};
                for (int bit = 127; bit >= 0; --bit) {
                    uint32_t c[4] = {y[0], y[1], y[2], y[3]};
                    c[bit >> 5] |= 1u << (bit & 31);
                    uint32_t sq[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        uint64_t carry = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const uint64_t t = (uint64_t)c[i] * c[j] + sq[i + j] + carry;
                            sq[i + j] = (uint32_t)t;
                            carry = t >> 32;
                        }
                        sq[i + 4] = (uint32_t)carry;
                    }
                    bool le = true;                     // sq <= v (lexicographic from the top word)
                    bool decided = false;
#pragma unroll
                    for (int w = 7; w >= 0; --w) {
                        if (!decided && sq[w] != v.w[w]) { le = sq[w] < v.w[w]; decided = true; }
                    }
                    if (le) { y[0] = c[0]; y[1] = c[1]; y[2] = c[2]; y[3] = c[3]; }
                }
                Fr r = fr_zero();
                r.w[0] = y[0]; r.w[1] = y[1]; r.w[2] = y[2]; r.w[3] = y[3];
                lds_put(dst, r);
                break;
            }
            case MO_SHR: {
                const uint32_t* s = myV + op.a * VW;    // words straight from LDS
                const uint32_t q = op.p0 >> 5, r = op.p0 & 31;
                Fr v;
#pragma unroll
                for (uint32_t t = 0; t < 8; ++t) {
                    const uint32_t lo = t + q < 8 ? s[t + q] : 0u;
                    const uint32_t hi = t + q + 1 < 8 ? s[t + q + 1] : 0u;
                    v.w[t] = r ? (lo >> r) | (hi << (32 - r)) : lo;
                }
                lds_put(dst, v);
                break;
            }
            default:
                break;
        }
    }
    }

// LDS carve of a stage block (the same for every block of a program):
// constants | element values | slot ops | micro-ops | views | half descriptors.
struct StageLds {
    uint32_t* sK;
    uint32_t* sV;
    SlotOp* sAdv;
    SlotOp* sLk;
    MicroOp* sMo;
    DView* sVw;
    uint4* sHM;
    uint32_t* sHD;
};
__device__ __forceinline__ StageLds stage_lds(const StageArgs& a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    StageLds L;
    L.sK = smem;
    L.sV = L.sK + kMaxK * VW;
    const uint32_t E = a.E ? a.E : kStageElems;
    L.sAdv = reinterpret_cast<SlotOp*>(L.sV + E * stage_elem_words(a.nv));
    L.sLk = L.sAdv + kMaxAdv;
    L.sMo = reinterpret_cast<MicroOp*>(L.sLk + kMaxLk);
    L.sVw = reinterpret_cast<DView*>(L.sMo + kMaxMicro);
    // (stage_lds_bytes counts 48 B per view, >= sizeof(DView) + the alignment slack)
    static_assert(sizeof(DView) <= 40, "DView grew: recheck stage_lds_bytes");
    // (word offsets from smem, not integer casts: a cast pointer would lose its
    // LDS address space and every table read would become a flat load)
    const uint32_t hm_off = ((uint32_t)(reinterpret_cast<uint32_t*>(L.sVw + kMaxViews) - smem) + 3u) & ~3u;
    L.sHM = reinterpret_cast<uint4*>(smem + hm_off);
    L.sHD = reinterpret_cast<uint32_t*>(L.sHM + 2 * (a.C + a.L));
    return L;
}
// A block's tables: constants, slot ops, micro-ops, views and the per (slot,
// half) descriptors and masks (no barrier).
__device__ __forceinline__ void stage_setup(const StageArgs& a, const StageLds& L,
                                            const MicroOp* __restrict__ mo, const SlotOp* __restrict__ adv,
                                            const SlotOp* __restrict__ lk, const Fr* __restrict__ K) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < a.nk; k += blockDim.x) lds_put(L.sK + k * VW, K[k]);
    for (uint32_t k = tid; k < a.C; k += blockDim.x) L.sAdv[k] = adv[k];
    for (uint32_t k = tid; k < a.L; k += blockDim.x) L.sLk[k] = lk[k];
    for (uint32_t k = tid; k < a.nmo; k += blockDim.x) L.sMo[k] = mo[k];
    if (tid < kMaxViews) L.sVw[tid] = a.view[tid];
    for (uint32_t k = tid; k < 2 * (a.C + a.L); k += blockDim.x) {
        const uint32_t sl = k >> 1;
        make_half(sl < a.C ? adv[sl] : lk[sl - a.C], k & 1, L.sHD + k, L.sHM + k);
    }
}
// This thread's in-bounds strided view loads of block blk's element.
struct Prefetch {
    Fr v0, v1;
    bool in0, in1;
};
__device__ __forceinline__ Prefetch stage_loads(const StageArgs& a, uint32_t blk) {
    const uint32_t E = a.E ? a.E : kStageElems;
    const uint32_t e0 = a.e_begin + blk * E;
    const uint32_t ne = min(E, a.e_end - e0), e = e0 + threadIdx.x;
    Prefetch f{fr_zero(), fr_zero(), false, false};
    if (threadIdx.x < ne) {
        const uint32_t pi = e / a.cols, pj = e - pi * a.cols;
        const DView& v0 = a.view[0];
        if (v0.ptr && v0.mode == VIEW_STRIDED && pi < v0.rows && pj < v0.cols) {
            f.v0 = ld_fr(v0.ptr + (int64_t)pi * v0.rs + (int64_t)pj * v0.cs);
            f.in0 = true;
        } else if (v0.ptr && v0.mode == VIEW_F64 && pi < v0.rows && pj < v0.cols) {
            f.v0 = quantize_fr(reinterpret_cast<const double*>(v0.ptr)[(int64_t)pi * v0.rs + (int64_t)pj * v0.cs],
                               f64_scale(v0));
            f.in0 = true;
        }
        const DView& v1 = a.view[1];
        if (v1.ptr && v1.mode == VIEW_STRIDED && pi < v1.rows && pj < v1.cols) {
            f.v1 = ld_fr(v1.ptr + (int64_t)pi * v1.rs + (int64_t)pj * v1.cs);
            f.in1 = true;
        } else if (v1.ptr && v1.mode == VIEW_F64 && pi < v1.rows && pj < v1.cols) {
            f.v1 = quantize_fr(reinterpret_cast<const double*>(v1.ptr)[(int64_t)pi * v1.rs + (int64_t)pj * v1.cs],
                               f64_scale(v1));
            f.in1 = true;
        }
    }
    return f;
}
// Phase A and phase B of block blk (tables set up; one barrier in between).
__device__ __forceinline__ void stage_chunk(const StageArgs& a, const StageLds& L, uint32_t blk,
                                            const Prefetch& f) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t nv = a.nv, tid = threadIdx.x;
    const uint32_t E = a.E ? a.E : kStageElems;
    const uint32_t e0 = a.e_begin + blk * E;
    const uint32_t ne = min(E, a.e_end - e0), e = e0 + tid;
    // ---- phase A: per-element micro-ops (constants / ops / views read from LDS:
    // dynamic indexing into the by-value kernel argument would go to scratch)
    if (tid < ne)
        element_program(a, e, L.sV + tid * stage_elem_words(nv), L.sK, L.sMo, L.sVw, f.v0, f.in0, f.v1, f.in1);
    __syncthreads();

    // ---- phase B: advice cells, then lookup cells
    uint4* outA = reinterpret_cast<uint4*>(a.out_adv + (uint64_t)e0 * a.C);
    uint4* outL = a.L ? reinterpret_cast<uint4*>(a.out_lk + (uint64_t)e0 * a.L) : nullptr;
    const uint32_t vb0 = (uint32_t)(L.sV - smem);
    const uint32_t rot = (a.flags & STAGE_ROT) ? blk * 37u : 0u;
    stream_cells_desc<true>(outA, 2 * ne * a.C, L.sHD, L.sHM, a.C, a.cdiv_magic, smem, vb0, nv, rot);
    if (a.L)
        stream_cells_desc<true>(outL, 2 * ne * a.L, L.sHD + 2 * a.C, L.sHM + 2 * a.C, a.L, a.ldiv_magic, smem,
                                vb0, nv, rot);
}

// One block of a stage: `a` supplies the scalar fields and the views (StageArgs
// up to `mo`), the tables come from mo / adv / lk / K (the by-value kernel
// argument of k_stage, or a record of a k_stage_multi batch); blk is the
// block's index within the stage. The view loads are issued before the table
// set-up so their latency overlaps it.
__device__ __forceinline__ void stage_block(const StageArgs& a, const MicroOp* __restrict__ mo,
                                            const SlotOp* __restrict__ adv,
                                            const SlotOp* __restrict__ lk, const Fr* __restrict__ K,
                                            uint32_t blk) {
    const StageLds L = stage_lds(a);
    const Prefetch f = stage_loads(a, blk);
    stage_setup(a, L, mo, adv, lk, K);
    __syncthreads();
    stage_chunk(a, L, blk, f);
}

__global__ __launch_bounds__(256) void k_stage(const StageArgs a) {
    stage_block(a, a.mo, a.adv, a.lk, a.K, blockIdx.x);
}

// the program of batch block g (m.blk0 ascending)
__device__ __forceinline__ uint32_t multi_prog(const StageMulti& m, uint32_t g) {
    uint32_t p = 0;
    for (uint32_t k = 1; k < m.nprog; ++k) p += g >= m.blk0[k];
    return p;
}
struct Rec {
    const StageArgs* a;
    const MicroOp* mo;
    const SlotOp* adv;
    const SlotOp* lk;
    const Fr* K;
};
__device__ __forceinline__ Rec multi_rec(const StageMulti& m, uint32_t p) {
    const uint8_t* r = m.data + m.off[p];
    Rec q;
    q.a = reinterpret_cast<const StageArgs*>(r);                     // fields up to `mo` only
    q.mo = reinterpret_cast<const MicroOp*>(r + kRecHead);
    q.adv = reinterpret_cast<const SlotOp*>(q.mo + q.a->nmo);
    q.lk = q.adv + q.a->C;
    q.K = reinterpret_cast<const Fr*>(q.lk + q.a->L);
    return q;
}

// Several independent stages in one launch (k_stage_multi): block b runs block
// b - blk0[p] of program p, whose compact record (stage_record, prog.hpp) is at
// data + off[p] -- so the small stages of a witness (single cells, d checks,
// gamma powers, is_equal rows, ...) and the phase-0 stages that read only the
// loaded matrices share one launch (one tail, one dispatch).
__global__ __launch_bounds__(256) void k_stage_multi(const StageMulti m) {
    const uint32_t p = multi_prog(m, blockIdx.x);
    const Rec q = multi_rec(m, p);
    stage_block(*q.a, q.mo, q.adv, q.lk, q.K, blockIdx.x - m.blk0[p]);
}
// Profiled stage launches (set_launch_events): the kernel's own dispatch
// records the profiler's events (hipExtLaunchKernelGGL: start on the first
// launch of the scope, stop re-recorded by every launch, so the last one's end
// counts) instead of event records between the launches, which cost a few us
// of stream time each.
static thread_local hipEvent_t tl_ev0 = nullptr, tl_ev1 = nullptr;
static thread_local bool tl_used = false;
void set_launch_events(hipEvent_t e0, hipEvent_t e1) {
    tl_ev0 = e0;
    tl_ev1 = e1;
    tl_used = false;
}
bool launch_events_used() {
    const bool u = tl_used;
    tl_ev0 = tl_ev1 = nullptr;
    tl_used = false;
    return u;
}
template <class K, class... Args>
static void launch_ev(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, Args... args) {
    if (!tl_ev1) {
        hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
        return;
    }
    hipExtLaunchKernelGGL(kernel, grid, block, lds, st, tl_used ? nullptr : tl_ev0, tl_ev1, 0, args...);
    tl_used = true;
}
hipError_t launch_stage(const StageArgs& a, hipStream_t st) {
    if (a.e_end <= a.e_begin) return hipSuccess;
    const uint32_t n = a.e_end - a.e_begin;
    const uint32_t E = a.E ? a.E : kStageElems;
    if (E > kStageElems) return hipErrorInvalidValue;
    const uint32_t lds = stage_lds_bytes(a.nv ? a.nv : 1, E, a.C + a.L);
    const uint32_t grid = (n + E - 1) / E;
    launch_ev(k_stage, dim3(grid), dim3(256), lds, st, a);
    return hipGetLastError();
}
bool stage_multi_fits(const StageArgs& a) {
    return stage_record_bytes(a.nmo, a.C, a.L, a.nk) <= kMultiBytes && (a.E ? a.E : kStageElems) <= kStageElems;
}
hipError_t launch_stage_multi(const StageArgs* const* progs, int n, hipStream_t st) {
    StageMulti m;
    uint32_t used = 0, blocks = 0, lds = 0;
    m.nprog = 0;
    const StageArgs* single = nullptr;
    // launch what is packed (a single program as a plain k_stage launch)
    auto flush = [&]() -> hipError_t {
        hipError_t e = hipSuccess;
        if (m.nprog == 1) {
            e = launch_stage(*single, st);
        } else if (m.nprog > 1) {
            m.blk0[m.nprog] = blocks;
            launch_ev(k_stage_multi, dim3(blocks), dim3(256), lds, st, m);
            e = hipGetLastError();
        }
        m.nprog = 0;
        used = blocks = lds = 0;
        return e;
    };
    for (int i = 0; i < n; ++i) {
        const StageArgs& a = *progs[i];
        if (a.e_end <= a.e_begin) continue;
        const uint32_t E = a.E ? a.E : kStageElems;
        if (E > kStageElems) return hipErrorInvalidValue;
        const uint32_t rb = stage_record_bytes(a.nmo, a.C, a.L, a.nk);
        if (rb > kMultiBytes) return hipErrorInvalidValue;
        if (m.nprog == (uint32_t)kMaxMulti || used + rb > kMultiBytes) {
            const hipError_t e = flush();
            if (e != hipSuccess) return e;
        }
        uint8_t* r = m.data + used;
        memcpy(r, &a, kRecHead);
        uint8_t* q = r + kRecHead;
        memcpy(q, a.mo, 8 * a.nmo);
        q += 8 * a.nmo;
        memcpy(q, a.adv, 4 * a.C);
        q += 4 * a.C;
        memcpy(q, a.lk, 4 * a.L);
        q += 4 * a.L;
        memcpy(q, a.K, 32 * a.nk);
        m.off[m.nprog] = used;
        m.blk0[m.nprog] = blocks;
        ++m.nprog;
        if (m.nprog == 1) single = &a;
        used += rb;
        blocks += (a.e_end - a.e_begin + E - 1) / E;
        lds = lds > stage_lds_bytes(a.nv ? a.nv : 1, E, a.C + a.L) ? lds : stage_lds_bytes(a.nv ? a.nv : 1, E, a.C + a.L);
    }
    return flush();
}

// ----------------------------------------------------------------- maxbits
__global__ __launch_bounds__(256) void k_maxbits(const DView v, uint32_t rows, uint32_t cols,
                                                 unsigned* out) {
    uint64_t n = (uint64_t)rows * cols;
    uint32_t best = 0;
    Fr zero = fr_zero();
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t i = (uint32_t)(e / cols), j = (uint32_t)(e % cols);
        Fr x = view_load(v, zero, i, j);
        best = max(best, signed_bits(x));
    }
    __shared__ uint32_t wmax[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, off));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
}

hipError_t launch_maxbits(const DView& v, uint32_t rows, uint32_t cols, unsigned* out,
                          hipStream_t st) {
    uint64_t n = (uint64_t)rows * cols;
    if (!n) return hipSuccess;
    unsigned blocks = (unsigned)((n + 255) / 256 < kMaxBitBlocks ? (n + 255) / 256 : kMaxBitBlocks);
    hipLaunchKernelGGL(k_maxbits, dim3(blocks), dim3(256), 0, st, v, rows, cols, out);
    return hipGetLastError();
}

// ---------------------------------------------------------- digit planes
// Balanced base-256 digits d_l in [-128, 127]: x = sum_l d_l 256^l.
__global__ __launch_bounds__(256) void k_to_digits(const DView x, uint32_t rows, uint32_t kdim,
                                                   int D, uint32_t rows_pad, uint32_t kg_pad,
                                                   uint32_t* __restrict__ out) {
    uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (uint64_t)rows_pad * kg_pad) return;
    uint32_t row = (uint32_t)(idx / kg_pad), kg = (uint32_t)(idx % kg_pad);
    uint32_t words[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    Fr zero = fr_zero();
    Fr half = fr_p();
    {
        uint32_t c = 0;
#pragma unroll
        for (int i = 7; i >= 0; --i) {
            uint32_t nw = (half.w[i] >> 1) | c;
            c = half.w[i] << 31;
            half.w[i] = nw;
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t k = kg * 4 + t;
        if (row >= rows || k >= kdim) continue;
        Fr v = view_load(x, zero, row, k);
        Fr tmp;
        bool neg = sub256(tmp, half, v) != 0;
        Fr mag = neg ? fr_sub(fr_zero(), v) : v;
        // signed 128-bit value (host guarantees |x| fits D digits, D <= 9)
        __int128 s = (__int128)(((unsigned __int128)mag.w[3] << 96) | ((unsigned __int128)mag.w[2] << 64) |
                                ((unsigned __int128)mag.w[1] << 32) | mag.w[0]);
        if (neg) s = -s;
#pragma unroll
        for (int l = 0; l < 9; ++l) {
            if (l < D) {
                int dg = (int)(uint32_t)(s & 0xff);
                if (dg >= 128) dg -= 256;
                s = (s - dg) >> 8;
                words[l] |= ((uint32_t)dg & 0xffu) << (8 * t);
            }
        }
    }
    uint32_t* o = out + idx * D;
#pragma unroll
    for (int l = 0; l < 9; ++l)
        if (l < D) o[l] = words[l];
}

hipError_t launch_to_digits(const DView& x, uint32_t rows, uint32_t kdim, int D, uint32_t rows_pad,
                            uint32_t kg_pad, uint32_t* out, hipStream_t st) {
    uint64_t n = (uint64_t)rows_pad * kg_pad;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_to_digits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, rows,
                       kdim, D, rows_pad, kg_pad, out);
    return hipGetLastError();
}

// ------------------------------------------------------------- dot4 GEMM
// Block = 256 threads = 16 x 16, each 2 x 2 outputs -> 32 x 32 tile.
// K advances 8 digit-groups (32 k) per LDS stage. acc[.][.][d] is the
// i32 sum of digit products with la + lb = d; |acc| < 9 * 2^14 * K < 2^31
// for K <= 8192 (host-checked).
constexpr int GT = 32;   // tile edge
constexpr int GKC = 8;   // digit groups per K stage

template <int DA, int DB>
__device__ __forceinline__ Fr combine_diagonals(const int (&acc)[DA + DB - 1]) {
    int64_t col[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < DA + DB - 1; ++d) {
        const int sh = 8 * d;
        col[sh >> 5] += (int64_t)acc[d] * ((int64_t)1 << (sh & 31));
    }
    uint32_t w[7];
    int64_t carry = 0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        int64_t t = col[q] + carry;
        w[q] = (uint32_t)t;
        carry = t >> 32;
    }
    return fr_from_signed_words<7>(w);
}

template <int DA, int DB, bool SYM>
__global__ __launch_bounds__(256) void k_gemm_dot4(const uint32_t* __restrict__ Ad,
                                                   const uint32_t* __restrict__ Bd, uint32_t N,
                                                   uint32_t M, uint32_t KG, Fr* __restrict__ out,
                                                   int64_t ors, int64_t ocs, uint32_t tiles_m) {
    __shared__ uint32_t As[GKC][DA][GT];
    __shared__ uint32_t Bs[GKC][DB][GT];
    uint32_t bi, bj;
    if (SYM) {
        // blockIdx -> (bi, bj) with bi <= bj over a tiles_m x tiles_m triangle
        uint32_t b = blockIdx.x, r = 0, rowlen = tiles_m;
        while (b >= rowlen) { b -= rowlen; ++r; --rowlen; }
        bi = r; bj = r + b;
    } else {
        bi = blockIdx.x / tiles_m;
        bj = blockIdx.x % tiles_m;
    }
    const uint32_t tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    const uint32_t i0 = bi * GT, j0 = bj * GT;
    int acc[2][2][DA + DB - 1];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int d = 0; d < DA + DB - 1; ++d) acc[r][c][d] = 0;

    const uint32_t lrow = tid >> 3, lg = tid & 7;
    for (uint32_t kg0 = 0; kg0 < KG; kg0 += GKC) {
        {
            const uint32_t* src = Ad + ((uint64_t)(i0 + lrow) * KG + kg0 + lg) * DA;
#pragma unroll
            for (int l = 0; l < DA; ++l) As[lg][l][lrow] = src[l];
            const uint32_t* srcb = Bd + ((uint64_t)(j0 + lrow) * KG + kg0 + lg) * DB;
#pragma unroll
            for (int l = 0; l < DB; ++l) Bs[lg][l][lrow] = srcb[l];
        }
        __syncthreads();
#pragma unroll 2
        for (int g = 0; g < GKC; ++g) {
            int a0[DA], a1[DA], b0[DB], b1[DB];
#pragma unroll
            for (int l = 0; l < DA; ++l) {
                uint2 v = *reinterpret_cast<const uint2*>(&As[g][l][2 * ty]);
                a0[l] = (int)v.x; a1[l] = (int)v.y;
            }
#pragma unroll
            for (int l = 0; l < DB; ++l) {
                uint2 v = *reinterpret_cast<const uint2*>(&Bs[g][l][2 * tx]);
                b0[l] = (int)v.x; b1[l] = (int)v.y;
            }
#pragma unroll
            for (int la = 0; la < DA; ++la)
#pragma unroll
                for (int lb = 0; lb < DB; ++lb) {
                    acc[0][0][la + lb] = __builtin_amdgcn_sdot4(a0[la], b0[lb], acc[0][0][la + lb], false);
                    acc[0][1][la + lb] = __builtin_amdgcn_sdot4(a0[la], b1[lb], acc[0][1][la + lb], false);
                    acc[1][0][la + lb] = __builtin_amdgcn_sdot4(a1[la], b0[lb], acc[1][0][la + lb], false);
                    acc[1][1][la + lb] = __builtin_amdgcn_sdot4(a1[la], b1[lb], acc[1][1][la + lb], false);
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t i = i0 + 2 * ty + r, j = j0 + 2 * tx + c;
            if (i < N && j < M) {
                Fr v = combine_diagonals<DA, DB>(acc[r][c]);
                st_fr(out + (int64_t)i * ors + (int64_t)j * ocs, v);
                if (SYM && bi != bj) st_fr(out + (int64_t)j * ors + (int64_t)i * ocs, v);
            }
        }
}

template <int DA, int DB>
static hipError_t gemm_dispatch(bool sym, const uint32_t* Ad, const uint32_t* Bd, uint32_t N,
                                uint32_t M, uint32_t kg, Fr* out, int64_t ors, int64_t ocs,
                                hipStream_t st) {
    uint32_t tn = (N + GT - 1) / GT, tm = (M + GT - 1) / GT;
    if (sym) {
        if (DA != DB || N != M) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_gemm_dot4<DA, DB, true>), dim3(tm * (tm + 1) / 2), dim3(256), 0, st,
                           Ad, Bd, N, M, kg, out, ors, ocs, tm);
    } else {
        hipLaunchKernelGGL((k_gemm_dot4<DA, DB, false>), dim3(tn * tm), dim3(256), 0, st, Ad, Bd,
                           N, M, kg, out, ors, ocs, tm);
    }
    return hipGetLastError();
}

bool gemm_digits_supported(int DA, int DB) {
    auto ok = [](int d) { return d == 5 || d == 8 || d == 9; };
    return ok(DA) && ok(DB);
}

hipError_t launch_gemm_digits(int DA, int DB, bool sym, const uint32_t* Ad, const uint32_t* Bd,
                              uint32_t N, uint32_t M, uint32_t kg, Fr* out, int64_t ors,
                              int64_t ocs, hipStream_t st) {
#define SVDW_G(a, b) \
    if (DA == a && DB == b) return gemm_dispatch<a, b>(sym, Ad, Bd, N, M, kg, out, ors, ocs, st);
    SVDW_G(5, 5) SVDW_G(5, 8) SVDW_G(5, 9) SVDW_G(8, 5) SVDW_G(8, 8) SVDW_G(8, 9)
    SVDW_G(9, 5) SVDW_G(9, 8) SVDW_G(9, 9)
#undef SVDW_G
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------- MFMA GEMM
// Same exact decomposition on the matrix cores: v_mfma_i32_16x16x64_i8 over
// balanced base-256 digit planes. Global digit layout: [row][kc][D][64 B]
// (kc = 64-k chunk; byte b = digit of X(row, 64 kc + b)), rows padded to 32.
// Fragment (one digit, 16 rows x 64 k): lane l holds row (l & 15), bytes
// [16 (l >> 4), +16) of the chunk; A and B use the same k mapping, so the
// product is independent of the hardware's k order inside the chunk.
// C/D (16x16 i32): col = lane & 15, row = 4 (lane >> 4) + reg.
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int MT = 32;        // block tile (2 x 2 waves of 16 x 16)
constexpr int LROW = 80;      // LDS bytes per (digit, row): 64 + 16 pad

// Digit planes chosen on the device from an operand's bit-length maximum (the
// engine's digits_for_bits + round_digits): 5, 8 or 9 planes, 0 = too wide for
// the digit GEMM (Montgomery fallback).
__device__ __forceinline__ int device_digits(const unsigned* __restrict__ bits) {
    const uint32_t b = *bits;
    const int need = b <= 7 ? 1 : (int)((b + 9) / 8);
    return need <= 5 ? 5 : need <= 8 ? 8 : need <= 9 ? 9 : 0;
}

__global__ __launch_bounds__(256) void k_to_digits_mf(const DView x, uint32_t rows, uint32_t kdim,
                                                      int D, uint32_t rows_pad, uint32_t kcn,
                                                      uint32_t* __restrict__ out,
                                                      const unsigned* __restrict__ dbits) {
    if (dbits) {
        D = device_digits(dbits);
        if (!D) return;
    }
    uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (uint64_t)rows_pad * kcn * 16) return;
    const uint32_t g = (uint32_t)(idx & 15);
    const uint64_t rk = idx >> 4;
    const uint32_t row = (uint32_t)(rk / kcn), kc = (uint32_t)(rk % kcn);
    uint32_t words[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    Fr zero = fr_zero();
    Fr half = fr_p();
    {
        uint32_t c = 0;
#pragma unroll
        for (int i = 7; i >= 0; --i) {
            uint32_t nw = (half.w[i] >> 1) | c;
            c = half.w[i] << 31;
            half.w[i] = nw;
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t k = kc * 64 + g * 4 + t;
        if (row >= rows || k >= kdim) continue;
        Fr v = view_load(x, zero, row, k);
        Fr tmp;
        bool neg = sub256(tmp, half, v) != 0;
        Fr mag = neg ? fr_sub(fr_zero(), v) : v;
        __int128 s = (__int128)(((unsigned __int128)mag.w[3] << 96) | ((unsigned __int128)mag.w[2] << 64) |
                                ((unsigned __int128)mag.w[1] << 32) | mag.w[0]);
        if (neg) s = -s;
#pragma unroll
        for (int l = 0; l < 9; ++l) {
            if (l < D) {
                int dg = (int)(uint32_t)(s & 0xff);
                if (dg >= 128) dg -= 256;
                s = (s - dg) >> 8;
                words[l] |= ((uint32_t)dg & 0xffu) << (8 * t);
            }
        }
    }
    uint32_t* o = out + rk * (uint64_t)D * 16 + g;
#pragma unroll
    for (int l = 0; l < 9; ++l)
        if (l < D) o[l * 16] = words[l];
}

hipError_t launch_to_digits_mf(const DView& x, uint32_t rows, uint32_t kdim, int D, uint32_t rows_pad,
                               uint32_t kcn, uint32_t* out, hipStream_t st, const unsigned* dbits) {
    uint64_t n = (uint64_t)rows_pad * kcn * 16;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_to_digits_mf, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, rows,
                       kdim, D, rows_pad, kcn, out, dbits);
    return hipGetLastError();
}

template <int DA, int DB>
__device__ __forceinline__ Fr combine_diag_reg(const v4i (&acc)[DA + DB - 1], int reg) {
    int a[DA + DB - 1];
#pragma unroll
    for (int d = 0; d < DA + DB - 1; ++d) a[d] = acc[d][reg];
    return combine_diagonals<DA, DB>(a);
}

template <int DA, int DB>
constexpr int gemm_lds_bytes() {
    return (DA + DB) * MT * LROW > MT * MT * 32 ? (DA + DB) * MT * LROW : MT * MT * 32;
}
template <int DA, int DB, bool SYM>
__device__ __forceinline__ void gemm_mfma_body(uint8_t* S, const uint8_t* __restrict__ Ad,
                                               const uint8_t* __restrict__ Bd, uint32_t N,
                                               uint32_t M, uint32_t kcn, Fr* __restrict__ out,
                                               int64_t ors, int64_t ocs, uint32_t tiles_m) {
    // one LDS array: operand slabs during the K loop, the output tile after it
    uint8_t* As = S;
    uint8_t* Bs = S + DA * MT * LROW;
    uint8_t* Ts = S;
    uint32_t bi, bj;
    if (SYM) {
        uint32_t b = blockIdx.x, r = 0, rowlen = tiles_m;
        while (b >= rowlen) { b -= rowlen; ++r; --rowlen; }
        bi = r; bj = r + b;
    } else {
        bi = blockIdx.x / tiles_m;
        bj = blockIdx.x % tiles_m;
    }
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wr = wave >> 1, wc = wave & 1;
    const uint32_t i0 = bi * MT, j0 = bj * MT;
    v4i acc[DA + DB - 1];
#pragma unroll
    for (int d = 0; d < DA + DB - 1; ++d) acc[d] = v4i{0, 0, 0, 0};

    const uint32_t frow = lane & 15, fk = (lane >> 4) * 16;
    for (uint32_t kc = 0; kc < kcn; ++kc) {
        // stage the A / B slabs: rows x D x 64 B, 16 B per thread-iteration
        for (uint32_t q = tid; q < (uint32_t)(MT * DA * 4); q += 256) {
            const uint32_t row = q / (DA * 4), rem = q % (DA * 4), l = rem >> 2, part = rem & 3;
            const uint4 v = *reinterpret_cast<const uint4*>(
                Ad + (((uint64_t)(i0 + row) * kcn + kc) * DA + l) * 64 + part * 16);
            *reinterpret_cast<uint4*>(As + (l * MT + row) * LROW + part * 16) = v;
        }
        for (uint32_t q = tid; q < (uint32_t)(MT * DB * 4); q += 256) {
            const uint32_t row = q / (DB * 4), rem = q % (DB * 4), l = rem >> 2, part = rem & 3;
            const uint4 v = *reinterpret_cast<const uint4*>(
                Bd + (((uint64_t)(j0 + row) * kcn + kc) * DB + l) * 64 + part * 16);
            *reinterpret_cast<uint4*>(Bs + (l * MT + row) * LROW + part * 16) = v;
        }
        __syncthreads();
        v4i bf[DB];
#pragma unroll
        for (int lb = 0; lb < DB; ++lb)
            bf[lb] = *reinterpret_cast<const v4i*>(Bs + (lb * MT + wc * 16 + frow) * LROW + fk);
#pragma unroll
        for (int la = 0; la < DA; ++la) {
            const v4i af = *reinterpret_cast<const v4i*>(As + (la * MT + wr * 16 + frow) * LROW + fk);
#pragma unroll
            for (int lb = 0; lb < DB; ++lb)
                acc[la + lb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[lb], acc[la + lb], 0, 0, 0);
        }
        __syncthreads();
    }
    // Epilogue: reduce the 17 diagonals to canonical Fr, stage the 32 x 32 cell
    // tile (32 KiB) in the (now free) operand LDS, then write whole 1 KiB tile
    // rows — and, for a symmetric off-diagonal tile, the transposed rows too —
    // as contiguous 16 B-per-lane stores.
    {
        const uint32_t tc = wc * 16 + (lane & 15);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const uint32_t tr = wr * 16 + (lane >> 4) * 4 + reg;
            Fr v = combine_diag_reg<DA, DB>(acc, reg);
            uint4* dst = reinterpret_cast<uint4*>(Ts + (tr * MT + tc) * 32);
            dst[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
            dst[1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
        }
    }
    __syncthreads();
    // direct tile: 32 rows x 64 half-cells; thread -> (row, half-cell)
    for (uint32_t q = tid; q < MT * 64; q += 256) {
        const uint32_t tr = q >> 6, hc = q & 63, tc = hc >> 1, h = hc & 1;
        const uint32_t row = i0 + tr, col = j0 + tc;
        if (row < N && col < M)
            reinterpret_cast<uint4*>(out + (int64_t)row * ors + (int64_t)col * ocs)[h] =
                reinterpret_cast<const uint4*>(Ts + (tr * MT + tc) * 32)[h];
    }
    if (SYM && bi != bj) {
        for (uint32_t q = tid; q < MT * 64; q += 256) {
            const uint32_t tc = q >> 6, hc = q & 63, tr = hc >> 1, h = hc & 1;   // out row = j
            const uint32_t row = j0 + tc, col = i0 + tr;
            if (row < M && col < N)
                reinterpret_cast<uint4*>(out + (int64_t)row * ors + (int64_t)col * ocs)[h] =
                    reinterpret_cast<const uint4*>(Ts + (tr * MT + tc) * 32)[h];
        }
    }
}

template <int DA, int DB, bool SYM>
__global__ __launch_bounds__(256) void k_gemm_mfma(const uint8_t* __restrict__ Ad,
                                                   const uint8_t* __restrict__ Bd, uint32_t N,
                                                   uint32_t M, uint32_t kcn, Fr* __restrict__ out,
                                                   int64_t ors, int64_t ocs, uint32_t tiles_m) {
    __shared__ __attribute__((aligned(16))) uint8_t S[gemm_lds_bytes<DA, DB>()];
    gemm_mfma_body<DA, DB, SYM>(S, Ad, Bd, N, M, kcn, out, ors, ocs, tiles_m);
}
// Digit counts read on the device (no host round trip for the operand bounds):
// every (DA, DB) pair is compiled in and the block branches uniformly.
template <bool SYM>
__global__ __launch_bounds__(256) void k_gemm_mfma_rt(const uint8_t* __restrict__ Ad,
                                                      const uint8_t* __restrict__ Bd, uint32_t N,
                                                      uint32_t M, uint32_t kcn, Fr* __restrict__ out,
                                                      int64_t ors, int64_t ocs, uint32_t tiles_m,
                                                      const unsigned* __restrict__ sa,
                                                      const unsigned* __restrict__ sb) {
    __shared__ __attribute__((aligned(16))) uint8_t S[gemm_lds_bytes<9, 9>()];
    const int DA = device_digits(sa), DB = SYM ? DA : device_digits(sb);
#define SVDW_RT(a, b) \
    if (DA == a && DB == b) { gemm_mfma_body<a, b, SYM>(S, Ad, Bd, N, M, kcn, out, ors, ocs, tiles_m); return; }
    if (SYM) {
        SVDW_RT(5, 5) SVDW_RT(8, 8) SVDW_RT(9, 9)
    } else {
        SVDW_RT(5, 5) SVDW_RT(5, 8) SVDW_RT(5, 9) SVDW_RT(8, 5) SVDW_RT(8, 8) SVDW_RT(8, 9)
        SVDW_RT(9, 5) SVDW_RT(9, 8) SVDW_RT(9, 9)
    }
#undef SVDW_RT
}
hipError_t launch_gemm_mfma_rt(bool sym, const uint8_t* Ad, const uint8_t* Bd, uint32_t N,
                               uint32_t M, uint32_t kcn, Fr* out, int64_t ors, int64_t ocs,
                               const unsigned* bits_a, const unsigned* bits_b, hipStream_t st) {
    uint32_t tn = (N + MT - 1) / MT, tm = (M + MT - 1) / MT;
    if (sym) {
        if (N != M) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_gemm_mfma_rt<true>, dim3(tm * (tm + 1) / 2), dim3(256), 0, st, Ad, Ad, N,
                           M, kcn, out, ors, ocs, tm, bits_a, bits_a);
    } else {
        hipLaunchKernelGGL(k_gemm_mfma_rt<false>, dim3(tn * tm), dim3(256), 0, st, Ad, Bd, N, M, kcn,
                           out, ors, ocs, tm, bits_a, bits_b);
    }
    return hipGetLastError();
}

template <int DA, int DB>
static hipError_t gemm_mfma_dispatch(bool sym, const uint8_t* Ad, const uint8_t* Bd, uint32_t N,
                                     uint32_t M, uint32_t kcn, Fr* out, int64_t ors, int64_t ocs,
                                     hipStream_t st) {
    uint32_t tn = (N + MT - 1) / MT, tm = (M + MT - 1) / MT;
    if (sym) {
        if (DA != DB || N != M) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_gemm_mfma<DA, DB, true>), dim3(tm * (tm + 1) / 2), dim3(256), 0, st,
                           Ad, Bd, N, M, kcn, out, ors, ocs, tm);
    } else {
        hipLaunchKernelGGL((k_gemm_mfma<DA, DB, false>), dim3(tn * tm), dim3(256), 0, st, Ad, Bd, N,
                           M, kcn, out, ors, ocs, tm);
    }
    return hipGetLastError();
}

hipError_t launch_gemm_mfma(int DA, int DB, bool sym, const uint8_t* Ad, const uint8_t* Bd,
                            uint32_t N, uint32_t M, uint32_t kcn, Fr* out, int64_t ors,
                            int64_t ocs, hipStream_t st) {
#define SVDW_G(a, b) \
    if (DA == a && DB == b) return gemm_mfma_dispatch<a, b>(sym, Ad, Bd, N, M, kcn, out, ors, ocs, st);
    SVDW_G(5, 5) SVDW_G(5, 8) SVDW_G(5, 9) SVDW_G(8, 5) SVDW_G(8, 8) SVDW_G(8, 9)
    SVDW_G(9, 5) SVDW_G(9, 8) SVDW_G(9, 9)
#undef SVDW_G
    return hipErrorInvalidValue;
}

// ------------------------------------------- multi-modular (CRT) exact GEMM
// c_s = A * Bt exactly for |A| < 2^ba, |B| < 2^bb (ba, bb <= 128): with n
// pairwise coprime moduli m_k <= 256 whose product Mtot exceeds 2^(ba+bb+lk+2),
// every residue product C mod m_k is one plain int8 GEMM of the balanced
// residue planes (|r| <= 128, K <= 2^17 keeps the i32 sums exact), and C is
// rebuilt from its n residues (crt_tables.hpp). ~19 int8 GEMMs at P = 63
// instead of 72 digit-pair products. n is decided on the device from the
// operand bit-length words, like the digit path.
__device__ __forceinline__ int crt_nmod(uint32_t ba, uint32_t bb, uint32_t lk) {
    if (ba > 128 || bb > 128) return 0;
    const uint32_t need = ba + bb + lk + 2;
    // lane k tests table entry k + 1 (one load per lane; a scalar loop of
    // dependent loads cost ~2 us per call, measured in the GEMM's block
    // prologue). Called with the whole wave active.
    const uint32_t lane = threadIdx.x & 63;
    const bool ok = lane < (uint32_t)kCrtMaxMod && c_crt_cum_bits[lane + 1] >= need;
    const unsigned long long m = __ballot(ok);
    return m ? __ffsll(m) : 0;
}

// Balanced residues bal = ((x + h) mod m) - h, h = floor(m / 2), in [-128, 127],
// of 4 consecutive-k elements x = +-|x| for moduli k < n: one u32 word (4 x
// int8) per plane at o[k * plane]. w: NW u32 words of |x| (< 2^(32 NW)); nm:
// all ones for x < 0. The sign costs one xor per word, since -|x| = ~|x| + 1 -
// 2^(32 NW), plus the AND of the modulus' (1 - 2^(32 NW)) mod m; the sum of the
// bytes times 256^i mod m is one v_dot4_u32_u8 per word and stays < 2^20,
// where the mul_hi quotient by ceil(2^32 / m) is exact.
template <int NW>
__device__ __forceinline__ void residues_emit(const uint32_t (&w)[4][4], const uint32_t (&nm)[4],
                                              uint32_t* __restrict__ o, uint64_t plane, int n) {
    uint32_t x[4][NW];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < NW; ++j) x[t][j] = w[t][j] ^ nm[t];
    for (int k = 0; k < n; ++k) {
        const uint32_t m = c_crt_mod[k], magic = c_crt_magic[k], h = m >> 1,
                       cn = c_crt_negc[NW - 2][k];
        uint32_t bal[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            uint32_t s0 = nm[t] & cn;
#pragma unroll
            for (int j = 0; j < NW; ++j) s0 = __builtin_amdgcn_udot4(x[t][j], c_crt_p256[k][j], s0, false);
            const uint32_t q = __umulhi(s0 + h, magic);
            bal[t] = s0 - __umul24(q, m);                      // (x + h) mod m - h, two's complement
        }
        const uint32_t lo = __builtin_amdgcn_perm(bal[1], bal[0], 0x0c0c0400u),
                       hi = __builtin_amdgcn_perm(bal[3], bal[2], 0x0c0c0400u);
        o[k * plane] = lo | (hi << 16);
    }
}
// NW words of |x| (|x| < 2^(32 NW)) from canonical Fr cells.
template <int NW>
__device__ __forceinline__ void residues_body(const DView& x, uint32_t rows, uint32_t kdim,
                                              uint32_t rows_pad, uint32_t kw,
                                              uint32_t* __restrict__ out, int n, uint32_t row,
                                              uint32_t kg, const Fr& half) {
    const Fr zero = fr_zero();
    uint32_t w[4][4], nm[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const uint32_t kk = kg * 4 + t;
        Fr v = zero;
        if (row < rows && kk < kdim) v = view_load(x, zero, row, kk);
        Fr tmp;
        const bool neg = sub256(tmp, half, v) != 0;
        const Fr mag = neg ? fr_sub(zero, v) : v;
        nm[t] = neg ? ~0u : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[t][j] = mag.w[j];
    }
    residues_emit<NW>(w, nm, out + (uint64_t)row * kw + kg, (uint64_t)rows_pad * kw, n);
}
// Balanced residue planes: out[k][row][kpad] int8 (= u32 words of 4 consecutive
// k), k < n; rows >= `rows` and columns >= kdim are zero.
__global__ __launch_bounds__(256) void k_to_residues(const DView x, uint32_t rows, uint32_t kdim,
                                                     uint32_t rows_pad, uint32_t kw,
                                                     uint32_t* __restrict__ out,
                                                     const unsigned* __restrict__ bits_a,
                                                     const unsigned* __restrict__ bits_b,
                                                     const unsigned* __restrict__ bits_c,
                                                     uint32_t lk) {
    // planes for the product (a, b) and, when bits_c is given, also for (c, c)
    int n = crt_nmod(*bits_a, *bits_b, lk);
    if (bits_c) n = max(n, crt_nmod(*bits_c, *bits_c, lk));
    if (!n) return;
    const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (uint64_t)rows_pad * kw) return;
    const uint32_t row = (uint32_t)(idx / kw), kg = (uint32_t)(idx % kw);
    Fr half = fr_p();
    {
        uint32_t c = 0;
#pragma unroll
        for (int i = 7; i >= 0; --i) {
            const uint32_t nw = (half.w[i] >> 1) | c;
            c = half.w[i] << 31;
            half.w[i] = nw;
        }
    }
    const uint32_t bmax = max(max(*bits_a, *bits_b), bits_c ? *bits_c : 0u);
    if (bmax <= 64)
        residues_body<2>(x, rows, kdim, rows_pad, kw, out, n, row, kg, half);
    else if (bmax <= 96)
        residues_body<3>(x, rows, kdim, rows_pad, kw, out, n, row, kg, half);
    else
        residues_body<4>(x, rows, kdim, rows_pad, kw, out, n, row, kg, half);
}
hipError_t launch_to_residues(const DView& x, uint32_t rows, uint32_t kdim, uint32_t rows_pad,
                              uint32_t kpad, uint32_t* out, const unsigned* bits_a,
                              const unsigned* bits_b, uint32_t lk, hipStream_t st,
                              const unsigned* bits_c) {
    const uint64_t n = (uint64_t)rows_pad * (kpad / 4);
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_to_residues, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, rows,
                       kdim, rows_pad, kpad / 4, out, bits_a, bits_b, bits_c, lk);
    return hipGetLastError();
}

// |x_q| and sign of ZkMatrix::new's quantization (quantize_body: round half away
// of |x| 2^P, u128 saturation, NaN -> 0, sign(x) < 0 -> p - x_q) as u32 words;
// nm = all ones when x_q is negative (-0.0 included: its residues are 0 either way).
__device__ __forceinline__ void quantized_words(double x, double scale, uint32_t (&w)[4], uint32_t& nm) {
    nm = signbit(x) && !isnan(x) ? ~0u : 0u;
    const double s = round(fabs(x) * scale);
    w[0] = w[1] = w[2] = w[3] = 0u;
    if (s >= 340282366920938463463374607431768211456.0) {
        w[0] = w[1] = w[2] = w[3] = 0xffffffffu;
    } else if (s > 0.0) {
        const uint64_t bits = __double_as_longlong(s);
        const int e = (int)((bits >> 52) & 0x7ff) - 1075;
        const uint64_t mant = (bits & 0xfffffffffffffull) | (1ull << 52);
        const unsigned __int128 v = e >= 0 ? ((unsigned __int128)mant << e) : (unsigned __int128)(mant >> -e);
        w[0] = (uint32_t)v; w[1] = (uint32_t)(v >> 32);
        w[2] = (uint32_t)(v >> 64); w[3] = (uint32_t)(v >> 96);
    }
}
// Residue planes straight from the f64 inputs of svd_witness (what k_to_residues
// computes from the quantized cells, without reading the 32 B cells back): up to
// kMaxResSegs matrices in one launch, segment s covering blocks [blk0[s], blk0[s+1]).
__global__ __launch_bounds__(256) void k_residues_f64(const ResSegs q, const unsigned* __restrict__ W,
                                                      double scale) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 1; k < kMaxResSegs; ++k) s += (uint32_t)k < q.nseg && blockIdx.x >= q.blk0[k];
    const ResSeg g = q.seg[s];
    int n = 0;
    uint32_t bmax = 0;
#pragma unroll
    for (int p = 0; p < 2; ++p)
        if (g.wa[p] >= 0) {
            const uint32_t ba = W[g.wa[p]], bb = W[g.wb[p]];
            const int np = crt_nmod(ba, bb, g.lk[p]);
            if (!np) return;                                   // too wide: no CRT product
            n = max(n, np);
            bmax = max(bmax, max(ba, bb));
        }
    if (!n) return;
    const uint64_t idx = (uint64_t)(blockIdx.x - q.blk0[s]) * blockDim.x + threadIdx.x;
    if (idx >= (uint64_t)g.rows_pad * g.kw) return;
    const uint32_t row = g.tr ? (uint32_t)(idx % g.rows_pad) : (uint32_t)(idx / g.kw),
                   kg = g.tr ? (uint32_t)(idx / g.rows_pad) : (uint32_t)(idx % g.kw);
    uint32_t w[4][4], nm[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const uint32_t kk = kg * 4 + t;
        const uint64_t at = g.tr ? (uint64_t)kk * g.ld + row : (uint64_t)row * g.ld + kk;
        const double x = row < g.rows && kk < g.cols ? g.in[at] : 0.0;
        quantized_words(x, scale, w[t], nm[t]);
    }
    uint32_t* o = g.out + (uint64_t)row * g.kw + kg;
    const uint64_t plane = (uint64_t)g.rows_pad * g.kw;
    if (bmax <= 64)
        residues_emit<2>(w, nm, o, plane, n);
    else if (bmax <= 96)
        residues_emit<3>(w, nm, o, plane, n);
    else
        residues_emit<4>(w, nm, o, plane, n);
}
hipError_t launch_residues_f64(const ResSegs& q0, const unsigned* W, int precision_bits,
                               hipStream_t st) {
    ResSegs q = q0;
    if (!q.nseg || q.nseg > (uint32_t)kMaxResSegs) return hipErrorInvalidValue;
    uint32_t blocks = 0;
    for (uint32_t k = 0; k < q.nseg; ++k) {
        ResSeg& g = q.seg[k];
        if (g.kw * 4 < g.cols || g.rows_pad < g.rows || g.ld < (g.tr ? g.rows : g.cols)) return hipErrorInvalidValue;
        q.blk0[k] = blocks;
        blocks += (uint32_t)(((uint64_t)g.rows_pad * g.kw + 255) / 256);
    }
    q.blk0[q.nseg] = blocks;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_residues_f64, dim3(blocks), dim3(256), 0, st, q, W,
                       (double)(1ull << precision_bits));
    return hipGetLastError();
}

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): an unrolled
// loop whose index is a compile-time constant in the body
template <int I, int N, class F>
__device__ __forceinline__ void static_for_impl(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for_impl<I + 1, N>(f);
    }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl<0, N>(f); }

static constexpr int CT = CT_TILE;     // CRT GEMM block tile (4 waves of 64 x 64)
// Staged operand rows are 64 B (one k-chunk) with the four 16 B parts XOR-swizzled
// by (row >> 2) & 3: the staging stores (4 rows x 4 parts per 16 lanes) and the
// fragment reads (16 rows x 1 part) both land on 16 distinct 4-bank groups.
static constexpr int CROW = 64;
static constexpr uint32_t kCrtTileBytes = CT * CT;             // residues of one (tile, modulus)
__device__ __forceinline__ uint32_t crt_lds(uint32_t row, uint32_t part) {
    return row * CROW + 16u * (part ^ ((row >> 2) & 3u));
}

// One (128 x 128 tile, modulus) per block: residues of C mod m_k as bytes
// R[k][row][rpad_m] (tile (bi, bj) of the product; SYM: A == B).
// Ar / Br: planes of astride / bstride rows (a row block of a larger operand is
// its planes from row r0 on with the full operand's stride); R is
// [mod][tiles_a * CT][tiles_m * CT]. One 64-k chunk per LDS round, the next
// chunk's global loads in flight under the current chunk's MFMAs.
// Software pipeline, one barrier per 64-k step: LDS is double-buffered (the
// next chunk is stored into the other buffer while this chunk's MFMAs run from
// fragments read before them), two chunks are in flight in registers behind
// that, and the next step's fragment reads overlap the MFMAs still in the
// pipe. (A single buffer with a store / barrier / read / MFMA / barrier chain
// per step took ~1 us per step, ~16 us per tile, against ~0.1 us of MFMA.)
constexpr int crt_lds_bytes() { return 4 * CT * CROW; }
// Residues of the 4 x 4 accumulator tiles of one wave, stored in MFMA order:
// R[mod][tile][wave][a][b][lane][reg] (one u32 per lane and (a, b): a wave store
// is 256 contiguous bytes); the combine reads the same order (crt_combine_elem).
__device__ __forceinline__ void crt_store_residues(const v4i (&acc)[4][4], uint8_t* __restrict__ R,
                                                   uint32_t nblk, uint32_t tile, int mod) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t m = c_crt_mod[mod], magic = c_crt_magic[mod], bias = c_crt_bias[mod];
    uint32_t* Rt = reinterpret_cast<uint32_t*>(R + ((uint64_t)mod * nblk + tile) * kCrtTileBytes) +
                   wave * 1024 + lane;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t r[4];
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                // |acc| <= K 2^14 <= 2^27, bias = m ceil(2^27 / m): x < 2^28 + 2^8,
                // where the quotient by magic = ceil(2^32 / m) is floor(x / m) or
                // one more (x (magic m - 2^32) < 2^32 m / 16), so x - q m is in
                // [-m, m) and min_u32(r, r + m) is the residue: five VALU
                // operations (the fp32 quotient with two corrections took twelve)
                const uint32_t x = (uint32_t)acc[a][b][reg] + bias;
                const uint32_t q = __umulhi(x, magic);
                const uint32_t rr = (uint32_t)((int)x - __mul24((int)q, (int)m));
                r[reg] = min(rr, rr + m);
            }
            Rt[(a * 4 + b) * 64] = __builtin_amdgcn_perm(r[1], r[0], 0x0c0c0400u) |
                                   (__builtin_amdgcn_perm(r[3], r[2], 0x0c0c0400u) << 16);
        }
}
__device__ __forceinline__ void crt_gemm_tile(const uint8_t* __restrict__ Ar, const uint8_t* __restrict__ Br,
                                              uint32_t astride, uint32_t bstride, uint32_t kpad,
                                              uint32_t nblk, uint32_t tile, uint8_t* __restrict__ R,
                                              uint32_t bi, uint32_t bj, int mod, uint8_t* __restrict__ S,
                                              uint64_t& tp1, uint64_t& tp2) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wr = wave >> 1, wc = wave & 1;
    const uint8_t* Ap = Ar + ((uint64_t)mod * astride + bi * CT) * kpad;
    const uint8_t* Bp = Br + ((uint64_t)mod * bstride + bj * CT) * kpad;
    // staging map: 512 x 16 B per operand chunk; thread -> (row, part) for q = tid, tid + 256
    const uint32_t r0 = tid >> 2, r1 = (tid + 256) >> 2, part = tid & 3;
    const uint32_t kcn = kpad / 64;
    v4i acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = v4i{0, 0, 0, 0};
    const uint32_t frow = lane & 15, fk = (lane >> 4) * 16;
    // Staging registers per chunk as named variables, loops spelled out by macro
    // (arrays or lambdas over them ended up in scratch). Chunk indices past the
    // end are clamped to the last chunk, so the loads stay unconditional; those
    // chunks are never stored or multiplied.
#define CRT_GLOAD(g, chunk)                                                                   \
    {                                                                                         \
        const uint64_t ko = (uint64_t)min((uint32_t)(chunk), kcn - 1) * 64 + part * 16;     \
        g##a0 = *reinterpret_cast<const uint4*>(Ap + (uint64_t)r0 * kpad + ko);             \
        g##a1 = *reinterpret_cast<const uint4*>(Ap + (uint64_t)r1 * kpad + ko);             \
        g##b0 = *reinterpret_cast<const uint4*>(Bp + (uint64_t)r0 * kpad + ko);             \
        g##b1 = *reinterpret_cast<const uint4*>(Bp + (uint64_t)r1 * kpad + ko);             \
    }
#define CRT_LSTORE(g, buf)                                                                    \
    {                                                                                         \
        uint8_t* Ac = S + (buf) * 2 * CT * CROW;                                              \
        uint8_t* Bc = Ac + CT * CROW;                                                         \
        *reinterpret_cast<uint4*>(Ac + crt_lds(r0, part)) = g##a0;                            \
        *reinterpret_cast<uint4*>(Ac + crt_lds(r1, part)) = g##a1;                            \
        *reinterpret_cast<uint4*>(Bc + crt_lds(r0, part)) = g##b0;                            \
        *reinterpret_cast<uint4*>(Bc + crt_lds(r1, part)) = g##b1;                            \
    }
#define CRT_FRAG(buf)                                                                         \
    {                                                                                         \
        const uint8_t* Ac = S + (buf) * 2 * CT * CROW;                                        \
        const uint8_t* Bc = Ac + CT * CROW;                                                   \
        _Pragma("unroll") for (int a = 0; a < 4; ++a)                                         \
            af[a] = *reinterpret_cast<const v4i*>(Ac + crt_lds(wr * 64 + a * 16 + frow, fk >> 4)); \
        _Pragma("unroll") for (int b = 0; b < 4; ++b)                                         \
            bf[b] = *reinterpret_cast<const v4i*>(Bc + crt_lds(wc * 64 + b * 16 + frow, fk >> 4)); \
    }
#define CRT_MMA()                                                                             \
    {                                                                                         \
        _Pragma("unroll") for (int a = 0; a < 4; ++a)                                         \
            _Pragma("unroll") for (int b = 0; b < 4; ++b)                                     \
                acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[b], acc[a][b], 0, 0, 0); \
    }
    // chunk c lives in register set g(c mod 4) until it is stored to LDS (at
    // step c - 1); four chunks in flight keep ~64 KB of loads outstanding per
    // CU, what an HBM / Infinity Cache latency needs (at 2 chunks a tile took
    // ~1 us per 64-k step, bound by bytes in flight, not by the MFMAs)
    uint4 g0a0, g0a1, g0b0, g0b1, g1a0, g1a1, g1b0, g1b1;
    uint4 g2a0, g2a1, g2b0, g2b1, g3a0, g3a1, g3b0, g3b1;
    v4i af[4], bf[4];
    CRT_GLOAD(g0, 0);
    CRT_GLOAD(g1, 1);
    CRT_GLOAD(g2, 2);
    CRT_GLOAD(g3, 3);
    CRT_LSTORE(g0, 0);
    CRT_GLOAD(g0, 4);
    __syncthreads();
    tp1 = wall_clock64();
    CRT_FRAG(0);
    // kcn is a multiple of 4 (kpad % 256 == 0): the steps are branch-free, so
    // the compiler's load counters see the four chunks in flight (a branch per
    // step made it drain every load before each LDS store). The last group's
    // stores and fragment reads of chunks >= kcn (clamped loads) are unused.
#define CRT_STEP(g, c)                                                                        \
    {                                                                                         \
        CRT_LSTORE(g, ((c) + 1) & 1);                    /* chunk c + 1 into the other buffer */ \
        CRT_GLOAD(g, (c) + 5);                           /* (c + 5) mod 4 = (c + 1) mod 4 */  \
        CRT_MMA();                                                                            \
        __syncthreads();                                                                      \
        CRT_FRAG(((c) + 1) & 1);                                                              \
    }
    for (uint32_t c0 = 0; c0 < kcn; c0 += 4) {
        CRT_STEP(g1, c0)
        CRT_STEP(g2, c0 + 1)
        CRT_STEP(g3, c0 + 2)
        CRT_STEP(g0, c0 + 3)
    }
    tp2 = wall_clock64();
#undef CRT_STEP
#undef CRT_GLOAD
#undef CRT_LSTORE
#undef CRT_FRAG
#undef CRT_MMA
    crt_store_residues(acc, R, nblk, tile, mod);
}


// Debug timeline of the GEMM's blocks (svdw_debug_trace): per real block its
// start and end on the 100 MHz wall clock and (XCC id << 16 | HW_ID).
__device__ unsigned long long* g_trace = nullptr;
hipError_t set_debug_trace(void* buf) {
    unsigned long long* p = (unsigned long long*)buf;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &p, sizeof p);
}
__device__ __forceinline__ void trace_block(uint64_t t0, uint64_t t1, uint64_t t2) {
    unsigned long long* tr = g_trace;
    if (!tr || threadIdx.x) return;
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    tr[5 * blockIdx.x] = t0;
    tr[5 * blockIdx.x + 1] = t1;
    tr[5 * blockIdx.x + 2] = t2;
    tr[5 * blockIdx.x + 3] = wall_clock64();
    tr[5 * blockIdx.x + 4] = ((unsigned long long)xcc << 32) | hw;
}


// tile t of a job (t < nblk; the sequence starts at tile0) -> its (row,
// column) tile (SYM: upper tiles row by row)
__device__ __forceinline__ void crt_tile_rc(const CrtJob& q, uint32_t t, uint32_t* bi, uint32_t* bj) {
    t += q.tile0;
    if (q.sym) {
        uint32_t r = 0, rest = t, rowlen = q.tiles_a;
        while (rest >= rowlen) { rest -= rowlen; ++r; --rowlen; }
        *bi = r; *bj = r + rest;
    } else {
        *bi = t / q.tiles_m;
        *bj = t - *bi * q.tiles_m;
    }
}
// The products of a CrtBatch in one launch, placed modulus-major per XCD: the
// work units (job, modulus < the job's device-decided count n, tile) are laid
// out job-major, modulus-major, and XCD x (blocks x, x + 8, ... on gfx950) takes
// the x-th eighth of them in order, so an XCD streams one modulus's residue
// planes through its own L2 while it computes that modulus's tiles, instead of
// every XCD reading strips of every plane. Blocks past the units exit at once
// (the grid is sized for n = kCrtMaxMod).
// (job, modulus, tile) unit u of the batch in the XCD-modulus-major order of
// the GEMM kernels; false for blocks past the units
__device__ __forceinline__ bool crt_unit(const CrtBatch& b, uint32_t blk, uint32_t* jo, uint32_t* mo,
                                         uint32_t* to) {
    uint32_t cnt[kMaxCrtJobs], total = 0;
#pragma unroll
    for (int j = 0; j < kMaxCrtJobs; ++j) {
        cnt[j] = 0;
        if ((uint32_t)j < b.njobs)
            cnt[j] = (uint32_t)crt_nmod(*b.job[j].bits_a, *b.job[j].bits_b, b.job[j].lk) * b.job[j].nblk;
        total += cnt[j];
    }
    const uint32_t per = (total + 7) / 8, k = blk >> 3;
    if (k >= per) return false;
    uint32_t u = (blk & 7) * per + k;
    if (u >= total) return false;
    uint32_t j = 0;
#pragma unroll
    for (int q = 0; q < kMaxCrtJobs - 1; ++q)
        if (j == (uint32_t)q && u >= cnt[q]) { u -= cnt[q]; ++j; }
    *jo = j;
    *mo = u / b.job[j].nblk;
    *to = u - *mo * b.job[j].nblk;
    return true;
}
__global__ __launch_bounds__(256) void k_gemm_crt_multi(const CrtBatch b) {
    __shared__ __attribute__((aligned(16))) uint8_t S[crt_lds_bytes()];
    const uint64_t t0 = wall_clock64();
    uint32_t j, mod, t;
    if (!crt_unit(b, blockIdx.x, &j, &mod, &t)) return;
    const CrtJob& q = b.job[j];
    uint32_t bi, bj;
    crt_tile_rc(q, t, &bi, &bj);
    uint64_t tp1 = 0, tp2 = 0;
    crt_gemm_tile(q.Ar, q.sym ? q.Ar : q.Br, q.astride, q.sym ? q.astride : q.bstride, q.kpad, q.nblk, t,
                  q.R, bi, bj, (int)mod, S, tp1, tp2);
    trace_block(t0, tp1, tp2);
}
// persistent CRT GEMM blocks per XCD label: two per CU (32 CUs per XCD)
static constexpr uint32_t kCrtPersPerXcd = 64;
// Operand row-tile bases and output place of one (job, modulus, tile) unit.
struct CrtUnitPtr {
    const uint8_t* Ap;
    const uint8_t* Bp;
    uint8_t* R;
    uint32_t nblk, t, mod;
};
__device__ __forceinline__ CrtUnitPtr crt_unit_ptr(const CrtBatch& b, const uint32_t (&cnt)[kMaxCrtJobs],
                                                   uint32_t u) {
    uint32_t j = 0;
#pragma unroll
    for (int q = 0; q < kMaxCrtJobs - 1; ++q)
        if (j == (uint32_t)q && u >= cnt[q]) { u -= cnt[q]; ++j; }
    const CrtJob& q = b.job[j];
    CrtUnitPtr o;
    o.mod = u / q.nblk;
    o.t = u - o.mod * q.nblk;
    o.nblk = q.nblk;
    o.R = q.R;
    uint32_t bi, bj;
    crt_tile_rc(q, o.t, &bi, &bj);
    o.Ap = q.Ar + ((uint64_t)o.mod * q.astride + bi * CT) * q.kpad;
    o.Bp = (q.sym ? q.Ar : q.Br) + ((uint64_t)o.mod * (q.sym ? q.astride : q.bstride) + bj * CT) * q.kpad;
    return o;
}
// The register-staged tile loop of crt_gemm_tile on a persistent grid: block b
// (XCD label b mod 8, slot b / 8 of nb8) takes the units lo + slot, lo + slot +
// nb8, ... of its XCD's eighth [lo, hi) of the batch's units (the order of
// k_gemm_crt_multi), and its chunk pipeline runs on across unit boundaries: the
// loads of the next unit's first chunks are in flight while the current unit's
// last chunks are multiplied and its residues reduced and stored, so a block's
// prologue (3.3 us per 128 x 128 x 1024 unit, gemmprobe timeline) is paid once
// instead of per unit. Needs one kpad for all jobs with at least 8 chunks (a
// load is then at most one unit ahead); launch_gemm_crt_multi checks.
__global__ __launch_bounds__(256, 2) void k_gemm_crt_pers(const CrtBatch b) {
    __shared__ __attribute__((aligned(16))) uint8_t S[crt_lds_bytes()];
    const uint64_t t0 = wall_clock64();
    uint32_t cnt[kMaxCrtJobs], total = 0;
#pragma unroll
    for (int j = 0; j < kMaxCrtJobs; ++j) {
        cnt[j] = 0;
        if ((uint32_t)j < b.njobs)
            cnt[j] = (uint32_t)crt_nmod(*b.job[j].bits_a, *b.job[j].bits_b, b.job[j].lk) * b.job[j].nblk;
        total += cnt[j];
    }
    const uint32_t per = (total + 7) / 8, x = blockIdx.x & 7, slot = blockIdx.x >> 3, nb8 = gridDim.x >> 3;
    const uint32_t lo = x * per, hi = min(lo + per, total);
    if (lo + slot >= hi) return;
    const uint32_t nunits = (hi - lo - slot + nb8 - 1) / nb8;
    const uint32_t kpad = b.job[0].kpad, kcn = kpad / 64;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wr = wave >> 1, wc = wave & 1;
    const uint32_t r0 = tid >> 2, r1 = (tid + 256) >> 2, part = tid & 3;
    const uint32_t frow = lane & 15, fk = (lane >> 4) * 16;
    const uint64_t o0 = (uint64_t)r0 * kpad + part * 16, o1 = (uint64_t)r1 * kpad + part * 16;
    CrtUnitPtr cur = crt_unit_ptr(b, cnt, lo + slot);
    CrtUnitPtr nxt = nunits > 1 ? crt_unit_ptr(b, cnt, lo + slot + nb8) : cur;
    v4i acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[a][q] = v4i{0, 0, 0, 0};
    // chunk ch of the current unit (ch >= kcn: chunk ch - kcn of the next one,
    // the current unit's last chunk when there is none)
#define CRP_GLOAD(g, ch)                                                                      \
    {                                                                                         \
        const uint32_t c_ = (ch);                                                             \
        const bool nx_ = c_ >= kcn;                                                           \
        const uint8_t* A_ = nx_ ? nxt.Ap : cur.Ap;                                            \
        const uint8_t* B_ = nx_ ? nxt.Bp : cur.Bp;                                            \
        const uint64_t ko = (uint64_t)(nx_ ? c_ - kcn : c_) * 64;                             \
        g##a0 = *reinterpret_cast<const uint4*>(A_ + o0 + ko);                                \
        g##a1 = *reinterpret_cast<const uint4*>(A_ + o1 + ko);                                \
        g##b0 = *reinterpret_cast<const uint4*>(B_ + o0 + ko);                                \
        g##b1 = *reinterpret_cast<const uint4*>(B_ + o1 + ko);                                \
    }
#define CRP_LSTORE(g, buf)                                                                    \
    {                                                                                         \
        uint8_t* Ac = S + (buf) * 2 * CT * CROW;                                              \
        uint8_t* Bc = Ac + CT * CROW;                                                         \
        *reinterpret_cast<uint4*>(Ac + crt_lds(r0, part)) = g##a0;                            \
        *reinterpret_cast<uint4*>(Ac + crt_lds(r1, part)) = g##a1;                            \
        *reinterpret_cast<uint4*>(Bc + crt_lds(r0, part)) = g##b0;                            \
        *reinterpret_cast<uint4*>(Bc + crt_lds(r1, part)) = g##b1;                            \
    }
#define CRP_FRAG(buf)                                                                         \
    {                                                                                         \
        const uint8_t* Ac = S + (buf) * 2 * CT * CROW;                                        \
        const uint8_t* Bc = Ac + CT * CROW;                                                   \
        _Pragma("unroll") for (int a = 0; a < 4; ++a)                                         \
            af[a] = *reinterpret_cast<const v4i*>(Ac + crt_lds(wr * 64 + a * 16 + frow, fk >> 4)); \
        _Pragma("unroll") for (int q = 0; q < 4; ++q)                                         \
            bf[q] = *reinterpret_cast<const v4i*>(Bc + crt_lds(wc * 64 + q * 16 + frow, fk >> 4)); \
    }
#define CRP_MMA()                                                                             \
    {                                                                                         \
        _Pragma("unroll") for (int a = 0; a < 4; ++a)                                         \
            _Pragma("unroll") for (int q = 0; q < 4; ++q)                                     \
                acc[a][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[q], acc[a][q], 0, 0, 0); \
    }
#define CRP_STEP(g, c)                                                                        \
    {                                                                                         \
        CRP_LSTORE(g, ((c) + 1) & 1);                                                         \
        CRP_GLOAD(g, (c) + 5);                                                                \
        CRP_MMA();                                                                            \
        __syncthreads();                                                                      \
        CRP_FRAG(((c) + 1) & 1);                                                              \
    }
    uint4 g0a0, g0a1, g0b0, g0b1, g1a0, g1a1, g1b0, g1b1;
    uint4 g2a0, g2a1, g2b0, g2b1, g3a0, g3a1, g3b0, g3b1;
    v4i af[4], bf[4];
    CRP_GLOAD(g0, 0);
    CRP_GLOAD(g1, 1);
    CRP_GLOAD(g2, 2);
    CRP_GLOAD(g3, 3);
    CRP_LSTORE(g0, 0);
    CRP_GLOAD(g0, 4);
    __syncthreads();
    const uint64_t tp1 = wall_clock64();
    CRP_FRAG(0);
    for (uint32_t k = 0; k < nunits; ++k) {
        if (k + 1 >= nunits) nxt = cur;
        // (the last unit's loads past its end re-read its first chunks: the
        // stores and fragment reads of those are never multiplied)
        for (uint32_t c0 = 0; c0 < kcn; c0 += 4) {
            CRP_STEP(g1, c0)
            CRP_STEP(g2, c0 + 1)
            CRP_STEP(g3, c0 + 2)
            CRP_STEP(g0, c0 + 3)
        }
        crt_store_residues(acc, cur.R, cur.nblk, cur.t, (int)cur.mod);
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = v4i{0, 0, 0, 0};
        cur = nxt;
        if (k + 2 < nunits) nxt = crt_unit_ptr(b, cnt, lo + slot + (k + 2) * nb8);
    }
    trace_block(t0, tp1, wall_clock64());
#undef CRP_STEP
#undef CRP_GLOAD
#undef CRP_LSTORE
#undef CRP_FRAG
#undef CRP_MMA
}
// 256 x 128 block tile: two vertically adjacent 128 x 128 tiles of the job's
// tile grid per (tile pair, modulus) unit, 4 waves of 128 x 64. Per 64-k step a
// wave reads 8 A and 4 B fragments (12 KiB) for 32 MFMAs: half the LDS bytes
// per MFMA of the 64 x 64 wave tiles (16 fragments for 16 MFMAs), which bound
// those near 40 % of the matrix-core rate. 48 KiB of LDS (two 24 KiB buffers),
// two chunks in flight in registers, two blocks per CU. Non-symmetric jobs of
// whole tile grids only (launch_gemm_crt_multi checks); a pair's second tile
// past the last tile row reads clamped rows and stores nothing. Residues go to
// the 128 x 128 tiles' places in the per-unit kernel's MFMA order, so the
// combine is unchanged: wave (wr, wc)'s accumulator rows a < 4 / a >= 4 are the
// per-unit kernel's waves 2 * 0 + wc / 2 * 1 + wc of tile 2 bi2 + wr.
static constexpr int CTW = 2 * CT;
constexpr int crt_wide_lds_bytes() { return 2 * (CTW + CT) * CROW; }
__device__ __forceinline__ uint32_t crt_npairs(const CrtJob& q) { return (q.tiles_a + 1) / 2 * q.tiles_m; }
__device__ __forceinline__ bool crt_unit_wide(const CrtBatch& b, uint32_t blk, uint32_t* jo, uint32_t* mo,
                                              uint32_t* po) {
    uint32_t cnt[kMaxCrtJobs], total = 0;
#pragma unroll
    for (int j = 0; j < kMaxCrtJobs; ++j) {
        cnt[j] = 0;
        if ((uint32_t)j < b.njobs)
            cnt[j] = (uint32_t)crt_nmod(*b.job[j].bits_a, *b.job[j].bits_b, b.job[j].lk) * crt_npairs(b.job[j]);
        total += cnt[j];
    }
    const uint32_t per = (total + 7) / 8, k = blk >> 3;
    if (k >= per) return false;
    uint32_t u = (blk & 7) * per + k;
    if (u >= total) return false;
    uint32_t j = 0;
#pragma unroll
    for (int q = 0; q < kMaxCrtJobs - 1; ++q)
        if (j == (uint32_t)q && u >= cnt[q]) { u -= cnt[q]; ++j; }
    const uint32_t np = crt_npairs(b.job[j]);
    *jo = j;
    *mo = u / np;
    *po = u - *mo * np;
    return true;
}
__global__ __launch_bounds__(256, 2) void k_gemm_crt_wide(const CrtBatch b) {
    __shared__ __attribute__((aligned(16))) uint8_t S[crt_wide_lds_bytes()];
    const uint64_t t0 = wall_clock64();
    uint32_t j, mod, pr;
    if (!crt_unit_wide(b, blockIdx.x, &j, &mod, &pr)) return;
    const CrtJob& q = b.job[j];
    const uint32_t bi2 = pr / q.tiles_m, bj = pr - bi2 * q.tiles_m;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wr = wave >> 1, wc = wave & 1;
    const uint32_t kpad = q.kpad, kcn = kpad / 64;
    const uint32_t rlast = q.tiles_a * CT - 1;            // staged A rows stay in the job's tile rows
    const uint8_t* Ap = q.Ar + (uint64_t)mod * q.astride * kpad;
    const uint8_t* Bp = q.Br + ((uint64_t)mod * q.bstride + bj * CT) * kpad;
    const uint32_t rr = tid >> 2, part = tid & 3;
    uint64_t ao[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ao[i] = (uint64_t)min(bi2 * CTW + rr + 64u * i, rlast) * kpad + part * 16;
    const uint64_t bo0 = (uint64_t)rr * kpad + part * 16, bo1 = (uint64_t)(rr + 64) * kpad + part * 16;
    const uint32_t frow = lane & 15, fp = lane >> 4;
    v4i acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = v4i{0, 0, 0, 0};
#define CRW_GLOAD(g, chunk)                                                                   \
    {                                                                                         \
        const uint64_t ko = (uint64_t)min((uint32_t)(chunk), kcn - 1) * 64;                   \
        g##a0 = *reinterpret_cast<const uint4*>(Ap + ao[0] + ko);                             \
        g##a1 = *reinterpret_cast<const uint4*>(Ap + ao[1] + ko);                             \
        g##a2 = *reinterpret_cast<const uint4*>(Ap + ao[2] + ko);                             \
        g##a3 = *reinterpret_cast<const uint4*>(Ap + ao[3] + ko);                             \
        g##b0 = *reinterpret_cast<const uint4*>(Bp + bo0 + ko);                               \
        g##b1 = *reinterpret_cast<const uint4*>(Bp + bo1 + ko);                               \
    }
#define CRW_LSTORE(g, buf)                                                                    \
    {                                                                                         \
        uint8_t* Ac = S + (buf) * (CTW + CT) * CROW;                                          \
        uint8_t* Bc = Ac + CTW * CROW;                                                        \
        *reinterpret_cast<uint4*>(Ac + crt_lds(rr, part)) = g##a0;                            \
        *reinterpret_cast<uint4*>(Ac + crt_lds(rr + 64, part)) = g##a1;                       \
        *reinterpret_cast<uint4*>(Ac + crt_lds(rr + 128, part)) = g##a2;                      \
        *reinterpret_cast<uint4*>(Ac + crt_lds(rr + 192, part)) = g##a3;                      \
        *reinterpret_cast<uint4*>(Bc + crt_lds(rr, part)) = g##b0;                            \
        *reinterpret_cast<uint4*>(Bc + crt_lds(rr + 64, part)) = g##b1;                       \
    }
#define CRW_FRAG(buf)                                                                         \
    {                                                                                         \
        const uint8_t* Ac = S + (buf) * (CTW + CT) * CROW;                                    \
        const uint8_t* Bc = Ac + CTW * CROW;                                                  \
        _Pragma("unroll") for (int a = 0; a < 8; ++a)                                         \
            af[a] = *reinterpret_cast<const v4i*>(Ac + crt_lds(wr * 128 + a * 16 + frow, fp)); \
        _Pragma("unroll") for (int c = 0; c < 4; ++c)                                         \
            bf[c] = *reinterpret_cast<const v4i*>(Bc + crt_lds(wc * 64 + c * 16 + frow, fp));  \
    }
#define CRW_MMA()                                                                             \
    {                                                                                         \
        _Pragma("unroll") for (int a = 0; a < 8; ++a)                                         \
            _Pragma("unroll") for (int c = 0; c < 4; ++c)                                     \
                acc[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[c], acc[a][c], 0, 0, 0); \
    }
    // chunk c + 1 into the other LDS buffer, chunk c + 3 into the registers it
    // came from, chunk c multiplied, then the fragments of chunk c + 1
#define CRW_STEP(g, c)                                                                        \
    {                                                                                         \
        CRW_LSTORE(g, ((c) + 1) & 1);                                                         \
        CRW_GLOAD(g, (c) + 3);                                                                \
        CRW_MMA();                                                                            \
        __syncthreads();                                                                      \
        CRW_FRAG(((c) + 1) & 1);                                                              \
    }
    uint4 g0a0, g0a1, g0a2, g0a3, g0b0, g0b1, g1a0, g1a1, g1a2, g1a3, g1b0, g1b1;
    v4i af[8], bf[4];
    CRW_GLOAD(g0, 0);
    CRW_GLOAD(g1, 1);
    CRW_LSTORE(g0, 0);
    CRW_GLOAD(g0, 2);
    __syncthreads();
    const uint64_t tp1 = wall_clock64();
    CRW_FRAG(0);
    // (kcn is a multiple of 4: whole pairs of steps)
    for (uint32_t c0 = 0; c0 < kcn; c0 += 2) {
        CRW_STEP(g1, c0)
        CRW_STEP(g0, c0 + 1)
    }
    const uint64_t tp2 = wall_clock64();
#undef CRW_STEP
#undef CRW_GLOAD
#undef CRW_LSTORE
#undef CRW_FRAG
#undef CRW_MMA
    const uint32_t ti = bi2 * 2 + wr;                       // this wave's 128 x 128 tile row
    if (ti < q.tiles_a) {
        const uint32_t m = c_crt_mod[mod], magic = c_crt_magic[mod], bias = c_crt_bias[mod];
        uint32_t* Rt = reinterpret_cast<uint32_t*>(q.R + ((uint64_t)mod * q.nblk + ti * q.tiles_m + bj) *
                                                            kCrtTileBytes) + lane;
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                uint32_t r[4];
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {           // (crt_store_residues' reduction)
                    const uint32_t x = (uint32_t)acc[a][c][reg] + bias;
                    const uint32_t qq = __umulhi(x, magic);
                    const uint32_t rv = (uint32_t)((int)x - __mul24((int)qq, (int)m));
                    r[reg] = min(rv, rv + m);
                }
                Rt[((a >> 2) * 2 + wc) * 1024 + ((a & 3) * 4 + c) * 64] =
                    __builtin_amdgcn_perm(r[1], r[0], 0x0c0c0400u) |
                    (__builtin_amdgcn_perm(r[3], r[2], 0x0c0c0400u) << 16);
            }
    }
    trace_block(t0, tp1, tp2);
}
// C from its n residues, written as canonical Fr to out[i*ors + j*ocs]: one
// element per thread in the GEMM's tile order (each block one 256-element
// stretch of a tile), so a wave reads 64 consecutive residue bytes per modulus
// (the n loads issued before the first use: one memory latency, not n) and
// writes four rows of 16 consecutive cells. C mod p = sum_k r_k E_k +
// q (-Mtot mod p), q = floor(sum_k r_k inv_k / m_k + 1/2) in f64 (|C| < Mtot / 4
// keeps it exact), accumulated in eight 64-bit accumulators, one per 32-bit
// word of E_k (each sum of n <= 40 products of an 8-bit residue and a 32-bit
// word stays below 2^46: no carries until the end), then one 9-word
// reduction. SYM: elements j >= i of the upper tiles (the GEMM computed upper
// and diagonal 128-tiles), each also stored at (j, i).
__device__ __forceinline__ void crt_combine_elem(const CrtJob& q, uint32_t cblk) {
    const int n = crt_nmod(*q.bits_a, *q.bits_b, q.lk);
    if (!n) return;
    // element e of tile t in the GEMM's MFMA order (wave, a, b, lane, reg)
    constexpr uint32_t BPT = kCrtTileBytes / 256;
    const uint32_t tl = cblk / BPT;
    const uint32_t e = (cblk - tl * BPT) * 256 + threadIdx.x;
    const uint32_t reg = e & 3, ln = (e >> 2) & 63, ab = (e >> 8) & 15, w = e >> 12;
    uint32_t bi, bj;
    crt_tile_rc(q, tl, &bi, &bj);
    const uint32_t i = bi * CT + (w >> 1) * 64 + (ab >> 2) * 16 + (ln >> 4) * 4 + reg;
    const uint32_t j = bj * CT + (w & 1) * 64 + (ab & 3) * 16 + (ln & 15);
    if (i >= q.N || j >= q.M || (q.sym && j < i)) return;
    const uint64_t plane = (uint64_t)q.nblk * kCrtTileBytes;
    const uint8_t* __restrict__ rp = q.R + (uint64_t)tl * kCrtTileBytes + e;
    uint32_t r[kCrtMaxMod];
#pragma unroll
    for (int k = 0; k < kCrtMaxMod; ++k) r[k] = k < n ? rp[k * plane] : 0u;
    const int off = n * (n - 1) / 2;
    // one 64-bit accumulator per 32-bit word of E_k (v_mad_u64_u32): r (8 bit)
    // x word (32 bit) summed over n <= 40 moduli stays below 2^46 -> no carries
    // until the end (half the VALU of 16-bit limbs with 24-bit products)
    uint64_t acc[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) acc[w] = 0;
    double sq = 0.0;
#pragma unroll
    for (int k = 0; k < kCrtMaxMod; ++k) {
        if (k < n) {                                       // (uniform)
            sq = fma((double)r[k], c_crt_frac[off + k], sq);
#pragma unroll
            for (int w = 0; w < 8; ++w) acc[w] += (uint64_t)r[k] * c_crt_ep[off + k][w];
        }
    }
    const uint32_t qq = (uint32_t)floor(sq + 0.5);         // < 2^14
    uint32_t x[9];
    uint64_t t = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        t += acc[w] + (uint64_t)qq * c_crt_nmp[n][w];       // < 2^47 + carry
        x[w] = (uint32_t)t;
        t >>= 32;
    }
    x[8] = (uint32_t)t;
    const Fr v = reduce9(x);
    // plain stores: the two 16 B halves of a cell (and, for the mirror, the
    // other lanes' cells of a line) meet in L2 and go out as whole lines (the
    // nontemporal form wrote x1.24 the cell bytes, r03_pmc_summary.json)
    st_fr(q.out + (int64_t)i * q.ors + (int64_t)j * q.ocs, v);
    if (q.sym && j > i) st_fr(q.out + (int64_t)j * q.ors + (int64_t)i * q.ocs, v);
}
// Combine blocks of a CrtBatch (cblocks in all, job j from cblk0[j]) dealt
// XCD-contiguously: XCD x takes a contiguous run of the row-major tile
// sequence, so the halves of a 128-byte residue line that neighbouring tiles
// read come through the same L2.
__global__ __launch_bounds__(256) void k_crt_combine_multi(const CrtBatch b, uint32_t cblocks) {
    const uint32_t per = (cblocks + 7) / 8, t = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (t >= cblocks) return;
    uint32_t j = 0;
    for (uint32_t k = 1; k < b.njobs; ++k) j += t >= b.job[k].cblk0;
    crt_combine_elem(b.job[j], t - b.job[j].cblk0);
}

size_t crt_scratch_bytes(uint32_t N, uint32_t M) {
    // kCrtMaxMod planes of whole 128 x 128 tiles
    const uint64_t a = ((uint64_t)N + CT - 1) / CT * CT, m = ((uint64_t)M + CT - 1) / CT * CT;
    return (size_t)(kCrtMaxMod * a * m);
}
// tile / block fields of a batch; units: GEMM blocks for n = kCrtMaxMod, cblocks: combine blocks
static hipError_t prep_crt_batch(CrtBatch& b, uint32_t& units, uint32_t& cblocks) {
    if (b.njobs < 1 || b.njobs > (uint32_t)kMaxCrtJobs) return hipErrorInvalidValue;
    units = 0;
    cblocks = 0;
    for (uint32_t j = 0; j < b.njobs; ++j) {
        CrtJob& q = b.job[j];
        q.tiles_a = (q.N + CT - 1) / CT;
        q.tiles_m = q.sym ? q.tiles_a : (q.M + CT - 1) / CT;
        // every staged row (tiles x CT) lies inside its operand's planes
        if (q.kpad % 256 || q.astride < q.tiles_a * CT || (!q.sym && q.bstride < q.tiles_m * CT))
            return hipErrorInvalidValue;
        if (q.sym && q.N != q.M) return hipErrorInvalidValue;
        q.nblk = q.sym ? q.tiles_a * (q.tiles_a + 1) / 2 : q.tiles_a * q.tiles_m;
        if (q.tcount) {
            if (q.tile0 + q.tcount > q.nblk) return hipErrorInvalidValue;
            q.nblk = q.tcount;
        } else if (q.tile0) {
            return hipErrorInvalidValue;
        }
        units += kCrtMaxMod * q.nblk;                    // upper bound: n = kCrtMaxMod
        q.cblk0 = cblocks;
        cblocks += q.nblk * (kCrtTileBytes / 256);
    }
    return hipSuccess;
}
hipError_t launch_gemm_crt_multi(const CrtBatch& b0, hipStream_t st) {
    CrtBatch b = b0;
    uint32_t units, cblocks;
    const hipError_t pe = prep_crt_batch(b, units, cblocks);
    if (pe != hipSuccess) return pe;
    const dim3 grid((units + 7) / 8 * 8);
    if (b.kern > 3) return hipErrorInvalidValue;
    // wide tiles: non-symmetric jobs over whole tile grids (kern 3: and at
    // least 64 tile pairs, ~1200 units at n = 19, two rounds of two blocks per
    // CU; gemmprobe: 2048^2 m.v^T 209 -> 186 us against the persistent kernel,
    // but 1024^2's 608 units 35 -> 37 us), else the persistent kernel (one
    // kpad of >= 8 chunks for every job), else the per-unit one
    bool wide = b.kern >= 2;
    uint32_t wunits = 0, pairs = 0;
    for (uint32_t j = 0; j < b.njobs; ++j) {
        const CrtJob& q = b.job[j];
        wide = wide && !q.sym && !q.tile0 && !q.tcount;
        pairs += (q.tiles_a + 1) / 2 * q.tiles_m;
    }
    wunits = kCrtMaxMod * pairs;
    if (b.kern == 3 && pairs < 64) wide = false;
    bool pers = b.kern >= 1 && b.job[0].kpad >= 512;
    for (uint32_t j = 1; j < b.njobs; ++j) pers = pers && b.job[j].kpad == b.job[0].kpad;
    if (wide)
        hipLaunchKernelGGL(k_gemm_crt_wide, dim3((wunits + 7) / 8 * 8), dim3(256), 0, st, b);
    else if (pers)
        hipLaunchKernelGGL(k_gemm_crt_pers, dim3(std::min<uint32_t>(grid.x, 8 * kCrtPersPerXcd)), dim3(256), 0,
                           st, b);
    else
        hipLaunchKernelGGL(k_gemm_crt_multi, grid, dim3(256), 0, st, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_crt_combine_multi, dim3((cblocks + 7) / 8 * 8), dim3(256), 0, st, b, cblocks);
    return hipGetLastError();
}

hipError_t launch_gemm_crt(bool sym, const uint8_t* Ar, const uint8_t* Br, uint32_t N, uint32_t M,
                           uint32_t astride, uint32_t bstride, uint32_t kpad, uint8_t* R, Fr* out,
                           int64_t ors, int64_t ocs, const unsigned* bits_a,
                           const unsigned* bits_b, uint32_t lk, hipStream_t st, uint32_t kern) {
    if (sym && (N != M || astride != bstride)) return hipErrorInvalidValue;
    CrtBatch b;
    memset(&b, 0, sizeof b);
    b.njobs = 1;
    b.kern = kern;
    CrtJob& q = b.job[0];
    q.Ar = Ar;
    q.Br = sym ? Ar : Br;
    q.R = R;
    q.out = out;
    q.bits_a = bits_a;
    q.bits_b = bits_b;
    q.ors = ors;
    q.ocs = ocs;
    q.astride = astride;
    q.bstride = bstride;
    q.kpad = kpad;
    q.N = N;
    q.M = M;
    q.lk = lk;
    q.sym = sym;
    return launch_gemm_crt_multi(b, st);
}

// -------------------------------------------------------- Montgomery GEMM
__global__ __launch_bounds__(256) void k_gemm_mont(const DView A, const DView B, uint32_t N,
                                                   uint32_t K, uint32_t M, Fr* out, int64_t ors,
                                                   int64_t ocs, const unsigned* __restrict__ sa,
                                                   const unsigned* __restrict__ sb, int crt_lk) {
    if (sa) {   // the digit (crt_lk < 0) or CRT GEMM already produced the product
        if (crt_lk < 0 ? (device_digits(sa) && device_digits(sb)) : crt_nmod(*sa, *sb, crt_lk) > 0)
            return;
    }
    uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (uint64_t)N * M) return;
    uint32_t i = (uint32_t)(e / M), j = (uint32_t)(e % M);
    Fr zero = fr_zero();
    Fr acc = fr_zero();
    for (uint32_t k = 0; k < K; ++k) {
        Fr a = view_load(A, zero, i, k);
        Fr b = view_load(B, zero, k, j);
        acc = fr_add(acc, mont_mul(a, b));   // a * b * R^-1
    }
    st_fr(out + (int64_t)i * ors + (int64_t)j * ocs, mont_mul(acc, fr_r2()));
}

hipError_t launch_gemm_mont(const DView& A, const DView& B, uint32_t N, uint32_t K, uint32_t M,
                            Fr* out, int64_t ors, int64_t ocs, hipStream_t st,
                            const unsigned* bits_a, const unsigned* bits_b, int crt_lk) {
    uint64_t n = (uint64_t)N * M;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gemm_mont, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A, B, N, K,
                       M, out, ors, ocs, bits_a, bits_b, crt_lk);
    return hipGetLastError();
}

// ---------------------------------------------------------- checker
// svdw_check_gates: the MockProver-style constraint check of a generated
// witness on the device (halo2-base's basic gate q * (a + b*c - d) = 0 at every
// enabled offset, and the lookup table [0, 2^lb)); copy constraints are not
// checked here. One thread per (unit, gate); counts via one atomic per wave.
// Checker kernels: grid-stride, per-thread counts reduced in LDS, one global
// atomic per block and counter (per-wave atomics on one address serialise).
__device__ __forceinline__ void block_flush(const uint32_t (&v)[4], unsigned long long* c0,
                                            unsigned long long* c1) {
    __shared__ unsigned long long s[4];
    if (threadIdx.x < 4) s[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (v[k]) atomicAdd(&s[k], (unsigned long long)v[k]);
    __syncthreads();
    if (threadIdx.x < 2 && c0 && s[threadIdx.x]) atomicAdd(c0 + threadIdx.x, s[threadIdx.x]);
    if (threadIdx.x >= 2 && threadIdx.x < 4 && c1 && s[threadIdx.x])
        atomicAdd(c1 + threadIdx.x - 2, s[threadIdx.x]);
}
static inline unsigned check_grid(uint64_t n) {
    const uint64_t b = (n + 255) / 256;
    return (unsigned)(b < 4096 ? b : 4096);
}
__global__ __launch_bounds__(256) void k_check_cells(const Fr* __restrict__ adv, uint64_t u0, uint64_t nunits,
                                                     uint32_t unit, uint32_t cols,
                                                     const uint32_t* __restrict__ words, uint32_t nw,
                                                     ChkView v0, ChkView v1, unsigned long long* cnt) {
    uint32_t v[4] = {0, 0, 0, 0};   // gates checked / failed, copies checked / failed
    const uint64_t n = nunits * nw;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
         idx += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t u = idx / nw;
        const uint32_t w = words[idx - u * nw];
        const Fr* q = adv + u * unit;
        if (chk_kind(w) == CHK_GATE) {
            const Fr* g = q + w;
            ++v[0];
            v[1] += !fr_eq(fr_add(ld_fr(g), fr_mul(ld_fr(g + 1), ld_fr(g + 2))), ld_fr(g + 3));
        } else if (chk_kind(w) == CHK_COPY) {
            ++v[2];
            v[3] += !fr_eq(ld_fr(q + chk_a(w)), ld_fr(q + chk_b(w)));
        } else {
            const ChkView vw = chk_a(w) ? v1 : v0;
            const uint64_t i = (u0 + u) / cols, j = (u0 + u) - i * cols;
            if (vw.ptr && i < vw.rows && j < vw.cols) {
                ++v[2];
                v[3] += !fr_eq(ld_fr(vw.ptr + (int64_t)i * vw.rs + (int64_t)j * vw.cs), ld_fr(q + chk_b(w)));
            }
        }
    }
    block_flush(v, cnt, cnt + 4);
}
hipError_t launch_check_cells(const Fr* adv, uint64_t u0, uint64_t nunits, uint32_t unit, uint32_t cols,
                              const uint32_t* words, uint32_t nw, ChkView v0, ChkView v1,
                              unsigned long long* cnt, hipStream_t st) {
    const uint64_t n = nunits * nw;
    if (!n) return hipSuccess;
    if (!cols) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_check_cells, dim3(check_grid(n)), dim3(256), 0, st, adv, u0,
                       nunits, unit, cols, words, nw, v0, v1, cnt);
    return hipGetLastError();
}
__global__ __launch_bounds__(256) void k_gate_bits(uint32_t* qb, uint64_t off, uint64_t n,
                                                   uint64_t unit, const uint8_t* __restrict__ ubits) {
    const uint64_t w = off / 32 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w * 32 >= off + n) return;
    uint32_t bits = 0;
    const uint64_t i0 = w * 32;
    uint64_t o = i0 >= off ? (i0 - off) % unit : 0;
    for (int b = 0; b < 32; ++b) {
        const uint64_t i = i0 + b;
        if (i >= off && i < off + n) {
            if (ubits[o]) bits |= 1u << b;
            if (++o == unit) o = 0;
        }
    }
    if (bits) atomicOr(qb + w, bits);
}
hipError_t launch_gate_bits(uint32_t* qb, uint64_t off, uint64_t n, uint64_t unit, const uint8_t* ubits,
                            hipStream_t st) {
    if (!n) return hipSuccess;
    if (!unit) return hipErrorInvalidValue;
    const uint64_t nw = (off + n + 31) / 32 - off / 32;
    hipLaunchKernelGGL(k_gate_bits, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, qb, off, n, unit,
                       ubits);
    return hipGetLastError();
}
// 4 selector bytes per thread
__global__ __launch_bounds__(256) void k_selectors(uint8_t* q, const uint32_t* __restrict__ qb,
                                                   uint64_t start, uint64_t len, uint64_t rows,
                                                   bool clear_last) {
    const uint64_t r0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (r0 >= rows) return;
    uint32_t v = 0;
    for (int b = 0; b < 4; ++b) {
        const uint64_t r = r0 + b;
        if (r < len && !(clear_last && r + 1 == len)) {
            const uint64_t i = start + r;
            v |= ((qb[i >> 5] >> (i & 31)) & 1u) << (8 * b);
        }
    }
    *reinterpret_cast<uint32_t*>(q + r0) = v;
}
hipError_t launch_selectors(uint8_t* q, const uint32_t* qb, uint64_t start, uint64_t len, uint64_t rows,
                            bool clear_last, hipStream_t st) {
    if ((rows & 3) || ((uintptr_t)q & 3)) return hipErrorInvalidValue;
    if (len && !qb) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_selectors, dim3((unsigned)((rows / 4 + 255) / 256)), dim3(256), 0, st, q, qb, start,
                       len, rows, clear_last);
    return hipGetLastError();
}
__global__ __launch_bounds__(256) void k_check_physical(const Fr* __restrict__ cols,
                                                        const uint8_t* __restrict__ q, uint64_t rows,
                                                        uint32_t ncols, unsigned long long* cnt) {
    uint32_t v[4] = {0, 0, 0, 0};
    const uint64_t n = rows * ncols;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
         idx += (uint64_t)gridDim.x * blockDim.x) {
        if (!q[idx]) continue;
        const uint64_t col = idx / rows, r = idx - col * rows;
        const Fr* g = cols + idx;
        ++v[0];
        v[1] += r + 3 >= rows ||
                !fr_eq(fr_add(ld_fr(g), fr_mul(ld_fr(g + 1), ld_fr(g + 2))), ld_fr(g + 3));
    }
    block_flush(v, cnt, nullptr);
}
// the break cell of column c (row bp[c]) == row 0 of column c + 1
__global__ __launch_bounds__(256) void k_check_breaks(const Fr* __restrict__ cols, uint64_t rows,
                                                      const uint64_t* __restrict__ bp, uint32_t nb,
                                                      unsigned long long* cnt) {
    uint32_t v[4] = {0, 0, 0, 0};
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nb; c += gridDim.x * blockDim.x) {
        ++v[0];
        v[1] += bp[c] >= rows || !fr_eq(ld_fr(cols + c * rows + bp[c]), ld_fr(cols + (c + 1) * rows));
    }
    block_flush(v, cnt, nullptr);
}
hipError_t launch_check_breaks(const Fr* cols, uint64_t rows, const uint64_t* bp, uint32_t nb,
                               unsigned long long* cnt, hipStream_t st) {
    if (!nb) return hipSuccess;
    hipLaunchKernelGGL(k_check_breaks, dim3((nb + 255) / 256), dim3(256), 0, st, cols, rows, bp, nb, cnt);
    return hipGetLastError();
}
hipError_t launch_check_physical(const Fr* cols, const uint8_t* q, uint64_t rows, uint32_t ncols,
                                 unsigned long long* cnt, hipStream_t st) {
    const uint64_t n = rows * ncols;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_check_physical, dim3(check_grid(n)), dim3(256), 0, st, cols, q, rows,
                       ncols, cnt);
    return hipGetLastError();
}
__global__ __launch_bounds__(256) void k_check_lookups(const Fr* __restrict__ lk, uint64_t n,
                                                       uint32_t lb, unsigned long long* cnt) {
    uint32_t v[4] = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const Fr x = ld_fr(lk + i);
        bool bad = false;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const int keep = (int)lb - 32 * w;
            const uint32_t m = keep >= 32 ? 0u : (keep <= 0 ? 0xffffffffu : ~((1u << keep) - 1u));
            bad |= (x.w[w] & m) != 0;
        }
        ++v[0];
        v[1] += bad;
    }
    block_flush(v, cnt, nullptr);
}
// Equality lists (svdw_check_equalities) on cell stores: pair i = (source | its
// store << 62, destination); store 2 is the external value `ext` (init_rand).
// Constants: 5 words per record, (destination, canonical value).
__global__ __launch_bounds__(256) void k_check_copies(const Fr* __restrict__ s0, const Fr* __restrict__ s1,
                                                      const Fr* __restrict__ dst,
                                                      const uint64_t* __restrict__ pairs, uint64_t n,
                                                      const Fr ext, unsigned long long* cnt) {
    uint32_t v[4] = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t src = pairs[2 * i], d = pairs[2 * i + 1];
        const uint32_t st = (uint32_t)(src >> 62);
        const uint64_t so = src & ((1ull << 62) - 1);
        const Fr a = st == 2 ? ext : ld_fr((st ? s1 : s0) + so);
        const Fr b = ld_fr(dst + d);
        ++v[0];
        v[1] += !fr_eq(a, b);
    }
    block_flush(v, cnt, nullptr);
}
__global__ __launch_bounds__(256) void k_check_consts(const Fr* __restrict__ dst,
                                                      const uint64_t* __restrict__ recs, uint64_t n,
                                                      unsigned long long* cnt) {
    uint32_t v[4] = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t* r = recs + 5 * i;
        const Fr b = ld_fr(dst + r[0]);
        Fr k;
#pragma unroll
        for (int w = 0; w < 4; ++w) { k.w[2 * w] = (uint32_t)r[1 + w]; k.w[2 * w + 1] = (uint32_t)(r[1 + w] >> 32); }
        ++v[0];
        v[1] += !fr_eq(k, b);
    }
    block_flush(v, cnt, nullptr);
}
hipError_t launch_check_copies(const Fr* s0, const Fr* s1, const Fr* dst, const uint64_t* pairs,
                               uint64_t n, const Fr& ext, unsigned long long* cnt, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_check_copies, dim3(check_grid(n)), dim3(256), 0, st, s0, s1, dst, pairs, n,
                       ext, cnt);
    return hipGetLastError();
}
// the copy source of a region's view (engine.cpp eq_src_cell, same cases)
__device__ __forceinline__ uint64_t eq_src_dev(const EqSrcDev& e, uint64_t i, uint64_t j, uint64_t t,
                                               unsigned* err) {
    if (e.kind == 2) {                          // EQS_CHAIN
        if (t == 0) return e.first | (uint64_t)e.first_phase << 62;
        return (e.off + (t - 1) * (uint64_t)e.rs) | (uint64_t)e.phase << 62;
    }
    if (e.kind == 1) {                          // EQS_MAT
        if (e.diag_phase >= 0 && i == j) return e.diag_off | (uint64_t)e.diag_phase << 62;
        if (i < e.rows && j < e.cols)
            return (uint64_t)((int64_t)e.off + (int64_t)i * e.rs + (int64_t)j * e.cs) | (uint64_t)e.phase << 62;
        if (e.pad_phase >= 0) return e.pad_off | (uint64_t)e.pad_phase << 62;
    }
    atomicOr(err, 1u);
    return 0;
}
__global__ __launch_bounds__(256) void k_eq_records(const EqRegionDev* __restrict__ R, uint32_t nreg,
                                                    uint64_t nitems, const uint32_t* __restrict__ words,
                                                    const Fr* __restrict__ konst, uint32_t phase,
                                                    uint64_t ext_off, uint64_t* __restrict__ copies,
                                                    uint64_t* __restrict__ consts, unsigned* __restrict__ err) {
    const uint64_t me = (uint64_t)phase << 62;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nitems;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = nreg;                 // region: the last with item0 <= g
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (R[mid].item0 <= g) lo = mid; else hi = mid;
        }
        const EqRegionDev& r = R[lo];
        const uint64_t e = g - r.item0;
        if (r.scan) {                               // [C(0), E(a_j), E(v_j), W(s_j), ...]
            const uint64_t i = e / r.L, j = e - i * r.L, base = r.off + i * r.unit;
            if (j == 0) {
                uint64_t* k = consts + 5 * (r.const0 + i);
                k[0] = base;
                k[1] = k[2] = k[3] = k[4] = 0;
            }
            uint64_t* c = copies + 2 * (r.copy0 + 2 * (i * r.L + j));
            c[0] = eq_src_dev(r.src[0], i, j, 0, err);
            c[1] = base + 1 + 3 * j;
            c[2] = eq_src_dev(r.src[1], 0, 0, j, err);
            c[3] = base + 2 + 3 * j;
            continue;
        }
        const uint64_t base = r.off + e * r.unit, i = e / r.cols, j = e - i * r.cols;
        uint64_t* c = copies + 2 * (r.copy0 + e * r.ncw);
        uint64_t* k = consts + 5 * (r.const0 + e * r.nkw);
        for (uint32_t q = 0; q < r.nw; ++q) {
            const uint32_t w = words[r.w0 + q], a = eq_a(w), at = eq_slot(w);
            switch (eq_kind(w)) {
            case EQ_CONST: {
                const Fr v = konst[r.k0 + a];
                k[0] = base + at;
                for (int t = 0; t < 4; ++t) k[1 + t] = (uint64_t)v.w[2 * t] | (uint64_t)v.w[2 * t + 1] << 32;
                k += 5;
                break;
            }
            case EQ_LOCAL: c[0] = (base + a) | me; c[1] = base + at; c += 2; break;
            case EQ_VIEW: c[0] = eq_src_dev(r.src[a], i, j, i, err); c[1] = base + at; c += 2; break;
            default: c[0] = ext_off | 2ull << 62; c[1] = base + at; c += 2; break;   // init_rand
            }
        }
    }
}
__device__ __forceinline__ uint64_t phys_dev(const uint64_t* st, uint32_t ncol, uint32_t k, uint64_t v) {
    uint32_t lo = 0, hi = ncol;                     // upper_bound(st, v) - 1
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (st[mid] <= v) lo = mid + 1; else hi = mid;
    }
    uint32_t col = lo ? lo - 1 : 0;
    if (col > 0 && v == st[col]) --col;             // break cell: its row in the column before
    return ((uint64_t)col << k) + (v - st[col]);
}
__global__ __launch_bounds__(256) void k_eq_phys(uint64_t* __restrict__ copies, uint64_t nc,
                                                 uint64_t* __restrict__ consts, uint64_t nk,
                                                 const uint64_t* __restrict__ s0, uint32_t n0,
                                                 const uint64_t* __restrict__ s1, uint32_t n1, uint32_t phase,
                                                 uint32_t k) {
    const uint64_t* sp = phase ? s1 : s0;
    const uint32_t np = phase ? n1 : n0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nc + nk;
         g += (uint64_t)gridDim.x * blockDim.x) {
        if (g < nc) {
            const uint64_t src = copies[2 * g];
            const uint32_t st = (uint32_t)(src >> 62);
            if (st < 2)
                copies[2 * g] = phys_dev(st ? s1 : s0, st ? n1 : n0, k, src & ((1ull << 62) - 1)) | (uint64_t)st << 62;
            copies[2 * g + 1] = phys_dev(sp, np, k, copies[2 * g + 1]);
        } else {
            consts[5 * (g - nc)] = phys_dev(sp, np, k, consts[5 * (g - nc)]);
        }
    }
}
hipError_t launch_eq_records(const EqRegionDev* regions, uint32_t nreg, uint64_t nitems,
                             const uint32_t* words, const Fr* konst, uint32_t phase, uint64_t ext_off,
                             uint64_t* copies, uint64_t* consts, unsigned* err, hipStream_t st) {
    if (!nitems || !nreg) return hipSuccess;
    hipLaunchKernelGGL(k_eq_records, dim3(check_grid(nitems)), dim3(256), 0, st, regions, nreg, nitems, words,
                       konst, phase, ext_off, copies, consts, err);
    return hipGetLastError();
}
hipError_t launch_eq_phys(uint64_t* copies, uint64_t nc, uint64_t* consts, uint64_t nk,
                          const uint64_t* start0, uint32_t ncol0, const uint64_t* start1, uint32_t ncol1,
                          uint32_t phase, uint32_t k, hipStream_t st) {
    if (!nc && !nk) return hipSuccess;
    hipLaunchKernelGGL(k_eq_phys, dim3(check_grid(nc + nk)), dim3(256), 0, st, copies, nc, consts, nk, start0,
                       ncol0, start1, ncol1, phase, k);
    return hipGetLastError();
}
hipError_t launch_check_consts(const Fr* dst, const uint64_t* recs, uint64_t n,
                               unsigned long long* cnt, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_check_consts, dim3(check_grid(n)), dim3(256), 0, st, dst, recs, n, cnt);
    return hipGetLastError();
}
hipError_t launch_check_lookups(const Fr* lk, uint64_t n, uint32_t lb, unsigned long long* cnt,
                                hipStream_t st) {
    if (!n) return hipSuccess;
    if ((n + 255) / 256 > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_check_lookups, dim3(check_grid(n)), dim3(256), 0, st, lk, n,
                       lb, cnt);
    return hipGetLastError();
}

// ------------------------------------------------------------ vectors
// grid (ceil(L / 256), 1 + kTabSlots): y = 0 the canonical copy, y = 1 + s the
// table slot s (one Montgomery product per thread).
__device__ __forceinline__ void tab_store(Fr* wc, Fr* tab, uint32_t L, uint32_t j, uint32_t y,
                                          const Fr& v, const ScaleTab& f) {
    if (y == 0) {
        if (wc) st_fr(wc + j, v);
        return;
    }
    const uint32_t s = y - 1;
    const Fr x = mont_mul(v, f.f[s]);
    Fr* base = tab + 2ull * s * L;
    st_fr(base + j, x);
    if (s < kTabSlots - 1) st_fr(base + L + j, fr_neg(x));
}
__global__ __launch_bounds__(256) void k_vec_prep(const DView w, uint32_t L, Fr* wc, Fr* tab,
                                                  const ScaleTab f) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= L) return;
    const Fr v = view_load(w, fr_zero(), 0, j);
    tab_store(wc, tab, L, j, blockIdx.y, v, f);
}
hipError_t launch_vec_prep(const DView& w, uint32_t L, Fr* wc, Fr* tab, const ScaleTab& f,
                           hipStream_t st) {
    if (!L) return hipSuccess;
    hipLaunchKernelGGL(k_vec_prep, dim3((L + 255) / 256, 1 + kTabSlots), dim3(256), 0, st, w, L, wc,
                       tab, f);
    return hipGetLastError();
}
// g^j from the host's three Montgomery tables (depth: three products, then the
// slot's): no per-element square-and-multiply chain.
__global__ __launch_bounds__(256) void k_gamma_prep(const GammaTab g, uint32_t L, Fr* wc, Fr* tab,
                                                    const ScaleTab f, const PowCells pc) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= L) return;
    const Fr v = fr_from_mont(mont_mul(mont_mul(g.t[j & 15], g.t[16 + ((j >> 4) & 15)]), g.t[32 + (j >> 8)]));
    tab_store(wc, tab, L, j, blockIdx.y, v, f);
    if (pc.one && blockIdx.y == 0 && j < pc.d) {          // v_j = gamma^j: v_0 is the one cell
        if (j == 0) st_fr(pc.one, v);
        if (j >= 1) {                                      // element j - 1: [0, v_(j-1), gamma, v_j]
            Fr* e = pc.pows + 4ull * (j - 1);
            st_fr(e, fr_zero());
            st_fr(e + 2, pc.gamma);
            st_fr(e + 3, v);
        }
        if (j + 1 < pc.d) st_fr(pc.pows + 4ull * j + 1, v); // v_j as element j's v_(i-1)
    }
}
hipError_t launch_gamma_prep(const GammaTab& g, uint32_t L, Fr* wc, Fr* tab, const ScaleTab& f,
                             hipStream_t st, const PowCells* pc) {
    if (!L) return hipSuccess;
    if ((L + 255) / 256 > g.nhi || g.nhi > (uint32_t)kGammaTab - 32) return hipErrorInvalidValue;
    PowCells p;
    memset(&p, 0, sizeof p);
    if (pc) {
        if (pc->d > L || !pc->d) return hipErrorInvalidValue;
        p = *pc;
    }
    hipLaunchKernelGGL(k_gamma_prep, dim3((L + 255) / 256, 1 + kTabSlots), dim3(256), 0, st, g, L,
                       wc, tab, f, p);
    return hipGetLastError();
}

// -------------------------------------------------------- row inner products
// One 256-thread block per row. Chunks of 256 terms: Montgomery products
// a_j * w_j, wave shuffle scan + cross-wave LDS combine (Fr addition is
// associative, so the prefix values are exact whatever the order), cells
// [a_j, w_j, s_j] staged in LDS and written as coalesced 16 B half-cells.
__device__ __forceinline__ Fr shfl_up_fr(const Fr& v, int d) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = (uint32_t)__shfl_up((int)v.w[i], d);
    return r;
}

// Row handled by block b of a row scan. Blocks are dealt round-robin to the 8
// XCDs (b % 8); give each XCD a contiguous run of rows so that a column-strided
// view (row r of a transposed matrix = column r) finds its neighbours' 128 B
// lines in the same L2 instead of every XCD fetching them separately.
__device__ __forceinline__ uint32_t scan_row(uint32_t b, uint32_t nb) {
    return (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
}

// Inclusive wave64 scan of Fr values with DPP lane moves (GFX9 row_shr 1/2/4/8
// inside 16-lane rows, then row_bcast:15 / row_bcast:31 across rows); lanes
// without a source receive 0 (bound_ctrl / row_mask), and adding 0 is a no-op.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ Fr dpp_fr(const Fr& v) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        r.w[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.w[i], CTRL, ROW_MASK, 0xf, true);
    return r;
}
__device__ __forceinline__ Fr wave_scan_fr(Fr s) {
    s = fr_add(s, dpp_fr<0x111, 0xf>(s));   // row_shr:1
    s = fr_add(s, dpp_fr<0x112, 0xf>(s));   // row_shr:2
    s = fr_add(s, dpp_fr<0x114, 0xf>(s));   // row_shr:4
    s = fr_add(s, dpp_fr<0x118, 0xf>(s));   // row_shr:8
    s = fr_add(s, dpp_fr<0x142, 0xa>(s));   // row_bcast:15 -> rows 1, 3
    s = fr_add(s, dpp_fr<0x143, 0xc>(s));   // row_bcast:31 -> rows 2, 3
    return s;
}

// Unreduced 9-word sums (values < 2^288, exact integers) for the scan network.
struct U9 {
    uint32_t w[9];
};
__device__ __forceinline__ U9 u9_from(const Fr& a) {
    U9 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = a.w[i];
    r.w[8] = 0;
    return r;
}
__device__ __forceinline__ U9 u9_add(const U9& a, const U9& b) {
    U9 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.w[i] = addc32(a.w[i], b.w[i], c);
    return r;
}
__device__ __forceinline__ U9 u9_sub(const U9& a, const U9& b) {   // a >= b
    U9 r;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.w[i] = subb32(a.w[i], b.w[i], br);
    return r;
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ U9 dpp_u9(const U9& v) {
    U9 r;
#pragma unroll
    for (int i = 0; i < 9; ++i)
        r.w[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.w[i], CTRL, ROW_MASK, 0xf, true);
    return r;
}
// inclusive wave scan without modular reduction (64 terms < 2^b -> < 2^(b+6))
__device__ __forceinline__ U9 wave_scan_u9(U9 s) {
    s = u9_add(s, dpp_u9<0x111, 0xf>(s));
    s = u9_add(s, dpp_u9<0x112, 0xf>(s));
    s = u9_add(s, dpp_u9<0x114, 0xf>(s));
    s = u9_add(s, dpp_u9<0x118, 0xf>(s));
    s = u9_add(s, dpp_u9<0x142, 0xa>(s));
    s = u9_add(s, dpp_u9<0x143, 0xc>(s));
    return s;
}

// T terms per thread, DPP scan. The cells go through a 24 KB LDS stage (768
// cells) in T rounds -- round q stages the 3T cells of threads [q*256/T,
// (q+1)*256/T) and the whole block writes them as coalesced 16 B half-cells --
// so four blocks fit a CU and N = 1024 rows run as one wave of blocks.
// NA < 8: |signed a| < 2^(32 NA) and wm = w * 2^(32 NA) (fr_mul_small_signed);
// NA = 8: wm is Montgomery form (any field elements).
// One launch serves up to kMaxScanJobs independent scans (blocks [blk0, blk0 + rows)
// of the grid belong to job q), so the scans of several verify_mul calls share
// one wave of blocks.
// Words of the small operand from a bit bound (host: scan_na): 8 = full Montgomery.
__device__ __forceinline__ int na_of_bits(uint32_t b) {
    if (b > 192) return 8;
    return b ? (int)((b + 31) / 32) : 1;
}
__device__ __forceinline__ int spec_na(const NaSpec& sp, const unsigned* __restrict__ W) {
    if (sp.wa == -2) return na_of_bits(sp.lk);            // host-known bound
    if (sp.wa < 0 || !W) return 8;
    uint32_t b = W[sp.wa];
    if (sp.wb >= 0) b += W[sp.wb] + sp.lk;
    return na_of_bits(b);
}
// the launch's na: the template's, or (NA = 0) the max over the jobs' specs
template <int NA>
__device__ __forceinline__ int batch_na(const ScanBatch& B) {
    if constexpr (NA != 0) {
        return NA;
    } else {
        int na = 1;
#pragma unroll
        for (int q = 0; q < kMaxScanJobs; ++q)
            if ((uint32_t)q < B.njobs) na = max(na, spec_na(B.job[q].spec, B.bitw));
        return na;
    }
}
__device__ __forceinline__ const Fr* tab_slot(const Fr* tab, uint32_t L, int na) {
    return tab + 2ull * (na >= 8 ? kTabSlots - 1 : na - 1) * L;
}
// a_j * w_j: |signed a| < 2^(32 NA): a negative value p - x has a non-zero top
// word; multiply |a| (NA words) by w * 2^(32 NA) or by its negation. NA = 8:
// Montgomery product with w's Montgomery form.
template <int NA>
__device__ __forceinline__ Fr scan_prod(const Fr& a, const Fr* __restrict__ wm,
                                        const Fr* __restrict__ wn, uint32_t j) {
    if constexpr (NA == 8) {
        return mont_mul(a, ld_fr(wm + j));
    } else {
        const bool neg = a.w[7] != 0;
        Fr mag = fr_zero();
        uint32_t br = 0;
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            const uint32_t t = subb32(p_word(q), a.w[q], br);
            mag.w[q] = neg ? t : a.w[q];
        }
        return mont_mul_small<NA>(mag, ld_fr((neg ? wn : wm) + j));
    }
}
template <int NA>
__device__ __forceinline__ Fr scan_prod_rt(int na, const Fr& a, const Fr* __restrict__ wm,
                                           const Fr* __restrict__ wn, uint32_t j) {
    if constexpr (NA != 0) {
        return scan_prod<NA>(a, wm, wn, j);
    } else {
        switch (na) {          // uniform over the launch
        case 1: return scan_prod<1>(a, wm, wn, j);
        case 2: return scan_prod<2>(a, wm, wn, j);
        case 3: return scan_prod<3>(a, wm, wn, j);
        case 4: return scan_prod<4>(a, wm, wn, j);
        case 5: return scan_prod<5>(a, wm, wn, j);
        case 6: return scan_prod<6>(a, wm, wn, j);
        default: return scan_prod<8>(a, wm, wn, j);
        }
    }
}

// scan_prod with the table entries already loaded (wmv = w * 2^(32 NA) or its
// Montgomery form for NA = 8, wnv = -wmv)
template <int NA>
__device__ __forceinline__ Fr scan_prod_v(const Fr& a, const Fr& wmv, const Fr& wnv) {
    if constexpr (NA == 8) {
        return mont_mul(a, wmv);
    } else {
        const bool neg = a.w[7] != 0;
        Fr mag = fr_zero(), wv;
        uint32_t br = 0;
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            const uint32_t t = subb32(p_word(q), a.w[q], br);
            mag.w[q] = neg ? t : a.w[q];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) wv.w[q] = neg ? wnv.w[q] : wmv.w[q];
        return mont_mul_small<NA>(mag, wv);
    }
}
template <int NA>
__device__ __forceinline__ Fr scan_prod_pre(int na, const Fr& a, const Fr& wmv, const Fr& wnv) {
    if constexpr (NA != 0) {
        return scan_prod_v<NA>(a, wmv, wnv);
    } else {
        switch (na) {          // uniform over the launch
        case 1: return scan_prod_v<1>(a, wmv, wnv);
        case 2: return scan_prod_v<2>(a, wmv, wnv);
        case 3: return scan_prod_v<3>(a, wmv, wnv);
        case 4: return scan_prod_v<4>(a, wmv, wnv);
        case 5: return scan_prod_v<5>(a, wmv, wnv);
        case 6: return scan_prod_v<6>(a, wmv, wnv);
        default: return scan_prod_v<8>(a, wmv, wnv);
        }
    }
}

template <int T, int NA>
__global__ __launch_bounds__(256) void k_matvec_scan_dpp(const ScanBatch B) {
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

// out[r] = sum_j A(r, j) w_j mod p for rows [0, R) (values only, no cells): the
// row-sharded witness needs every entry of b.g while it emits the b.g scan
// cells of its own rows only. One block per row; products as in the scan.
// Batched like the scans: job q owns blocks [blk0, blk0 + rows) of the grid.
template <int NA>
__global__ __launch_bounds__(256) void k_matvec_values(const ScanBatch B) {
    __shared__ U9 part[256];
    ScanJob J = B.job[0];
#pragma unroll
    for (int q = 1; q < kMaxScanJobs; ++q)
        if ((uint32_t)q < B.njobs && blockIdx.x >= B.job[q].blk0) J = B.job[q];
    const DView& A = J.A;
    const uint32_t L = J.L;
    const int na = batch_na<NA>(B);
    const Fr* __restrict__ wm = tab_slot(J.tab, J.tl, na);
    const Fr* __restrict__ wn = wm + J.tl;
    Fr* __restrict__ out = J.out;
    // rows dealt XCD-contiguously (as the scans): a transposed b's neighbouring
    // rows are neighbouring columns, one 128 B line per 4 rows in one L2
    const uint32_t lb = blockIdx.x - J.blk0;
    const uint32_t r = (J.blk0 & 7) ? lb : scan_row(lb, J.rows), tid = threadIdx.x;
    const Fr zero = fr_zero();
    U9 acc = u9_from(zero);
    for (uint32_t j = tid; j < L; j += 256) {
        const Fr a = view_load(A, zero, r, j);
        const Fr s = scan_prod_rt<NA>(na, a, wm, wn, j);
        acc = u9_add(acc, u9_from(s));                     // <= 2^13 terms of < p: < 2^267
    }
    part[tid] = acc;
    __syncthreads();
    for (uint32_t h = 128; h > 0; h >>= 1) {
        if (tid < h) part[tid] = u9_add(part[tid], part[tid + h]);
        __syncthreads();
    }
    if (tid == 0) st_fr(out + r, reduce9(part[0].w));
}
hipError_t launch_matvec_values(const ScanBatch& b0, int na, hipStream_t st) {
    ScanBatch b = b0;
    uint32_t blocks = 0;
    for (uint32_t q = 0; q < b.njobs; ++q) {
        if (b.job[q].L > 8192 || b.job[q].tl < b.job[q].L) return hipErrorInvalidValue;
        b.job[q].blk0 = blocks;
        blocks += b.job[q].L ? b.job[q].rows : 0;
        if (!b.job[q].L) b.job[q].rows = 0;
    }
    if (!blocks) return hipSuccess;
    const dim3 g(blocks), blk(256);
    switch (na) {
    case 0: hipLaunchKernelGGL(k_matvec_values<0>, g, blk, 0, st, b); break;
    case 1: hipLaunchKernelGGL(k_matvec_values<1>, g, blk, 0, st, b); break;
    case 2: hipLaunchKernelGGL(k_matvec_values<2>, g, blk, 0, st, b); break;
    case 3: hipLaunchKernelGGL(k_matvec_values<3>, g, blk, 0, st, b); break;
    case 4: hipLaunchKernelGGL(k_matvec_values<4>, g, blk, 0, st, b); break;
    case 5: hipLaunchKernelGGL(k_matvec_values<5>, g, blk, 0, st, b); break;
    case 6: hipLaunchKernelGGL(k_matvec_values<6>, g, blk, 0, st, b); break;
    default: hipLaunchKernelGGL(k_matvec_values<8>, g, blk, 0, st, b); break;
    }
    return hipGetLastError();
}

// b.g for b = X^T with X an f64 input of svd_witness (the row-sharded witness's
// b.g vector, every entry): (b.g)_i = sum_j q(X[j][i]) g^j, q = ZkMatrix::new's
// quantization done in registers (the cells of X need not exist on this rank).
// Column-parallel: thread = column i, block = (256 columns, one slice of
// rows), so every wave load is 2 KiB of one row of X (k_matvec_values reads a
// transposed view: one 32 B cell per lane, each from a different row). The
// slices' partial sums land in part[job][slice][C]; k_vec_prep_sum adds them.
__device__ __forceinline__ void quantize_mag(double x, double scale, Fr& mag, bool& neg) {
    const double s = round(fabs(x) * scale);
    mag = fr_zero();
    if (s >= 340282366920938463463374607431768211456.0) {
        mag.w[0] = mag.w[1] = mag.w[2] = mag.w[3] = 0xffffffffu;
    } else if (s > 0.0) {
        const uint64_t bits = __double_as_longlong(s);
        const int e = (int)((bits >> 52) & 0x7ff) - 1075;
        const uint64_t mant = (bits & 0xfffffffffffffull) | (1ull << 52);
        const unsigned __int128 v = e >= 0 ? ((unsigned __int128)mant << e) : (unsigned __int128)(mant >> -e);
        mag.w[0] = (uint32_t)v; mag.w[1] = (uint32_t)(v >> 32);
        mag.w[2] = (uint32_t)(v >> 64); mag.w[3] = (uint32_t)(v >> 96);
    }
    // -0.0 and negatives quantizing to 0 are the cell 0 (quantize_body)
    neg = signbit(x) && !isnan(x) && s > 0.0;
}
// Beside a saturating cell stream a memory round trip costs microseconds, so
// the kernel has three: the block's slice of the g table into LDS, every f64
// of the thread issued at once, the partial-sum store. Block = 32 columns x 8
// sub-slices of kColRows rows (one slice of 8 kColRows rows); the sub-slices
// are added in LDS, so a column has ceil(R / (8 kColRows)) partial sums.
template <int NA>
__device__ __forceinline__ U9 colsum_rows(const double (&x)[kColRows], uint32_t jl0, double scale,
                                          const Fr* sWm, const Fr* sWn) {
    U9 acc = u9_from(fr_zero());
#pragma unroll
    for (int t = 0; t < kColRows; ++t) {
        Fr mag;
        bool neg;
        quantize_mag(x[t], scale, mag, neg);
        const uint32_t jl = jl0 + t;
        Fr s;
        if constexpr (NA == 8) s = mont_mul(neg ? fr_neg(mag) : mag, sWm[jl]);
        else s = mont_mul_small<NA>(mag, neg ? sWn[jl] : sWm[jl]);
        acc = u9_add(acc, u9_from(s));                    // kColRows * 8 terms of < p
    }
    return acc;
}
__global__ __launch_bounds__(256) void k_colsum_f64(const ColBatch B, double scale) {
    constexpr uint32_t SR = 8 * kColRows;                 // rows per block
    __shared__ Fr sWm[SR], sWn[SR];
    __shared__ U9 sPart[256];
    const ColJob J = B.job[blockIdx.y];
    const uint32_t ncb = (J.C + 31) / 32, cb = blockIdx.x % ncb, sg = blockIdx.x / ncb;
    if (sg * SR >= J.R) return;                           // (grid sized for the longest job)
    const uint32_t tid = threadIdx.x, col = tid & 31, sub = tid >> 5;
    const uint32_t i = cb * 32 + col, jb = sg * SR, jl0 = sub * kColRows;
    int na = spec_na(J.spec, B.bitw);
    if (na > 4) na = 8;                                   // (quantized: <= 128 bits)
    const Fr* __restrict__ wm = tab_slot(B.tab, B.tl, na);
    const Fr* __restrict__ wn = wm + B.tl;
    double x[kColRows];
#pragma unroll
    for (int t = 0; t < kColRows; ++t) {
        const uint32_t j = jb + jl0 + t;
        x[t] = i < J.C && j < J.R ? J.x[(uint64_t)j * J.ld + i] : 0.0;
    }
    for (uint32_t k = tid; k < SR; k += 256) {            // rows past R read as 0 (x = 0 there)
        const uint32_t j = min(jb + k, J.R - 1);
        sWm[k] = ld_fr(wm + j);
        sWn[k] = na == 8 ? fr_zero() : ld_fr(wn + j);
    }
    __syncthreads();
    U9 acc;
    switch (na) {                                         // uniform over the launch
    case 1: acc = colsum_rows<1>(x, jl0, scale, sWm, sWn); break;
    case 2: acc = colsum_rows<2>(x, jl0, scale, sWm, sWn); break;
    case 3: acc = colsum_rows<3>(x, jl0, scale, sWm, sWn); break;
    case 4: acc = colsum_rows<4>(x, jl0, scale, sWm, sWn); break;
    default: acc = colsum_rows<8>(x, jl0, scale, sWm, sWn); break;
    }
    sPart[tid] = acc;
    __syncthreads();
    if (sub == 0 && i < J.C) {
#pragma unroll
        for (int k = 1; k < 8; ++k) acc = u9_add(acc, sPart[tid + 32 * k]);   // < 2^267 + 2^264
        st_fr(J.part + (uint64_t)sg * J.C + i, reduce9(acc.w));
    }
}
uint32_t colsum_slices(uint32_t R) { return (R + 8 * kColRows - 1) / (8 * kColRows); }
hipError_t launch_colsum_f64(const ColBatch& b, int precision_bits, hipStream_t st) {
    if (!b.njobs || b.njobs > (uint32_t)kMaxColJobs) return hipErrorInvalidValue;
    uint32_t blocks = 0;
    for (uint32_t q = 0; q < b.njobs; ++q) {
        const ColJob& j = b.job[q];
        if (!j.R || j.R > b.tl || j.R > 8192 || j.ld < j.C) return hipErrorInvalidValue;
        blocks = max(blocks, (j.C + 31) / 32 * colsum_slices(j.R));
    }
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_colsum_f64, dim3(blocks, b.njobs), dim3(256), 0, st, b,
                       (double)(1ull << precision_bits));
    return hipGetLastError();
}
// w_j = sum_s part[s L + j] -> canonical copy and scaled table (as k_vec_prep);
// a thread's loads are issued kColPartBatch at a time
__global__ __launch_bounds__(256) void k_vec_prep_sum(const Fr* __restrict__ part, uint32_t S, uint32_t L,
                                                      Fr* wc, Fr* tab, const ScaleTab f) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= L) return;
    Fr v = fr_zero();
    for (uint32_t s0 = 0; s0 < S; s0 += kColPartBatch) {
        Fr p[kColPartBatch];
#pragma unroll
        for (int s = 0; s < kColPartBatch; ++s)
            p[s] = s0 + s < S ? ld_fr(part + (uint64_t)(s0 + s) * L + j) : fr_zero();
#pragma unroll
        for (int s = 0; s < kColPartBatch; ++s) v = fr_add(v, p[s]);
    }
    tab_store(wc, tab, L, j, blockIdx.y, v, f);
}
// k_vec_prep_sum over the jobs of a batch (block x: job by blk0 ranges)
__global__ __launch_bounds__(256) void k_vec_prep_sum_multi(const VecPrepBatch b, const ScaleTab f) {
    uint32_t q = 0;
#pragma unroll
    for (int k = 1; k < kMaxColJobs; ++k) q += (uint32_t)k < b.njobs && blockIdx.x >= b.job[k].blk0;
    const Fr* part = b.job[0].part;
    uint32_t S = b.job[0].S, L = b.job[0].L, b0 = b.job[0].blk0;
    Fr* wc = b.job[0].wc;
    Fr* tab = b.job[0].tab;
#pragma unroll
    for (int k = 1; k < kMaxColJobs; ++k)                 // selects, not a dynamic index into the argument
        if (q == (uint32_t)k) {
            part = b.job[k].part; S = b.job[k].S; L = b.job[k].L; b0 = b.job[k].blk0; wc = b.job[k].wc;
            tab = b.job[k].tab;
        }
    const uint32_t j = (blockIdx.x - b0) * blockDim.x + threadIdx.x;
    if (j >= L) return;
    Fr v = fr_zero();
    for (uint32_t s0 = 0; s0 < S; s0 += kColPartBatch) {
        Fr p[kColPartBatch];
#pragma unroll
        for (int s = 0; s < kColPartBatch; ++s)
            p[s] = s0 + s < S ? ld_fr(part + (uint64_t)(s0 + s) * L + j) : fr_zero();
#pragma unroll
        for (int s = 0; s < kColPartBatch; ++s) v = fr_add(v, p[s]);
    }
    tab_store(wc, tab, L, j, blockIdx.y, v, f);
}
hipError_t launch_vec_prep_sum_multi(const VecPrepBatch& b0, const ScaleTab& f, hipStream_t st) {
    if (!b0.njobs || b0.njobs > (uint32_t)kMaxColJobs) return hipErrorInvalidValue;
    VecPrepBatch b = b0;
    uint32_t blocks = 0;
    for (uint32_t q = 0; q < b.njobs; ++q) {
        if (!b.job[q].S) return hipErrorInvalidValue;
        b.job[q].blk0 = blocks;
        blocks += (b.job[q].L + 255) / 256;
    }
    for (uint32_t q = b.njobs; q < (uint32_t)kMaxColJobs; ++q) b.job[q].blk0 = ~0u;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_vec_prep_sum_multi, dim3(blocks, 1 + kTabSlots), dim3(256), 0, st, b, f);
    return hipGetLastError();
}
hipError_t launch_vec_prep_sum(const Fr* part, uint32_t S, uint32_t L, Fr* wc, Fr* tab, const ScaleTab& f,
                               hipStream_t st) {
    if (!L) return hipSuccess;
    if (!S) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_vec_prep_sum, dim3((L + 255) / 256, 1 + kTabSlots), dim3(256), 0, st, part, S, L,
                       wc, tab, f);
    return hipGetLastError();
}

hipError_t launch_scan_batch(const ScanBatch& b0, int na, hipStream_t st) {
    ScanBatch b = b0;
    uint32_t blocks = 0;
    for (uint32_t q = 0; q < b.njobs; ++q) {
        if (b.job[q].tl < b.job[q].L) return hipErrorInvalidValue;
        b.job[q].blk0 = blocks;
        blocks += b.job[q].L ? b.job[q].rows : 0;
        if (!b.job[q].L) b.job[q].rows = 0;
    }
    if (!blocks) return hipSuccess;
    const dim3 g(blocks), blk(256);
    switch (na) {                      // two terms per thread (T = 2)
    case 0: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 0>), g, blk, 0, st, b); break;
    case 1: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 1>), g, blk, 0, st, b); break;
    case 2: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 2>), g, blk, 0, st, b); break;
    case 3: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 3>), g, blk, 0, st, b); break;
    case 4: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 4>), g, blk, 0, st, b); break;
    case 5: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 5>), g, blk, 0, st, b); break;
    case 6: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 6>), g, blk, 0, st, b); break;
    default: hipLaunchKernelGGL((k_matvec_scan_dpp<2, 8>), g, blk, 0, st, b); break;
    }
    return hipGetLastError();
}
hipError_t launch_matvec_scan(const DView& A, uint32_t r_begin, uint32_t r_end, uint32_t L,
                              const Fr* wc, const Fr* tab, uint32_t tl, Fr* out, int na, hipStream_t st) {
    if (r_end <= r_begin || !L) return hipSuccess;
    if (tl < L) return hipErrorInvalidValue;
    ScanBatch b;
    memset(&b, 0, sizeof b);
    b.njobs = 1;
    b.job[0] = ScanJob{A, wc, tab, tl, out, L, r_end - r_begin, 0, r_begin, NaSpec{-1, -1, 0, 0}};
    b.bitw = nullptr;
    return launch_scan_batch(b, na, st);
}

}  // namespace svdw
