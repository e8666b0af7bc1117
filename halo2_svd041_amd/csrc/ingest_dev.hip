// Device-side ingest of data/matrix.in (see ingest_dev.hpp). The host parser it
// mirrors is csrc/ingest.hpp (kParseSerde): same numbers, same value per number
// (serde_json 1.0's default path, examples/svd_example.rs:326-330).
//
// Pass 1: per 2 KiB chunk, the 2-state transfer (string state, bracket depth)
// of its bytes. Scan 1: every chunk's entry state. Pass 2: per chunk, counts of
// number tokens, row opens ('[' at depth 2) and depth-1 string starts. Scan 2:
// their offsets. Pass 3: positions, parsed values, depths and grammar flags of
// every number, row-open and depth-1 string positions, and the structural
// checks of the array bytes.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ingest_dev.hpp"

namespace svdw_ingest_dev {

static constexpr int kThreads = 256, kPer = kChunk / kThreads;   // 16 bytes per thread
static constexpr uint32_t kHalo = 256;   // bytes staged before and after a chunk

// The text as a block sees it: its chunk and halos staged in LDS (coalesced
// 16-byte loads), anything further out (long tokens or whitespace runs) read
// from global memory.
struct Txt {
    const uint8_t* g;
    const uint8_t* s;
    uint64_t lo, hi;
    __device__ __forceinline__ uint8_t operator[](uint64_t i) const { return i >= lo && i < hi ? s[i - lo] : g[i]; }
};
__device__ __forceinline__ Txt stage(const uint8_t* g, uint64_t n, uint8_t* sw) {
    const uint64_t c0 = (uint64_t)blockIdx.x * kChunk;
    const uint64_t lo = c0 >= kHalo ? c0 - kHalo : 0, hi = min(n, c0 + kChunk + kHalo);
    for (uint64_t k = threadIdx.x; 16 * k < hi - lo; k += blockDim.x) {
        const uint64_t off = lo + 16 * k;
        if (off + 16 <= hi && ((reinterpret_cast<uintptr_t>(g) + off) & 15) == 0) {
            *reinterpret_cast<uint4*>(sw + 16 * k) = *reinterpret_cast<const uint4*>(g + off);
        } else {
            for (uint64_t b = off; b < off + 16 && b < hi; ++b) sw[b - lo] = g[b];
        }
    }
    __syncthreads();
    return Txt{g, sw, lo, hi};
}
static_assert(kPer * kThreads == (int)kChunk, "chunk = threads x bytes per thread");

__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ bool num_char(uint8_t c) {
    return is_digit(c) || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-';
}
__device__ __forceinline__ bool is_alpha(uint8_t c) { return (c | 0x20) >= 'a' && (c | 0x20) <= 'z'; }
__device__ __forceinline__ bool is_ws(uint8_t c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }

__device__ __forceinline__ int fstate(const Xfer& x, int s) { return (x.f >> s) & 1; }
__device__ __forceinline__ Xfer xid() { return Xfer{2, 0, 0}; }
// a then b
__device__ __forceinline__ Xfer compose(const Xfer& a, const Xfer& b) {
    const int a0 = fstate(a, 0), a1 = fstate(a, 1);
    Xfer r;
    r.f = fstate(b, a0) | (fstate(b, a1) << 1);
    r.d0 = a.d0 + (a0 ? b.d1 : b.d0);
    r.d1 = a.d1 + (a1 ? b.d1 : b.d0);
    return r;
}
// a '"' at i ends a string only after an even run of backslashes (ingest.hpp str())
__device__ __forceinline__ bool escaped(const Txt& t, uint64_t i) {
    uint64_t k = 0;
    while (k < i && t[i - 1 - k] == '\\') ++k;
    return k & 1;
}
__device__ __forceinline__ Xfer byte_xfer(const Txt& t, uint64_t i, uint8_t c) {
    if (c == '"') return Xfer{1 | ((escaped(t, i) ? 1 : 0) << 1), 0, 0};
    if (c == '[' || c == '{') return Xfer{2, 1, 0};
    if (c == ']' || c == '}') return Xfer{2, -1, 0};
    return xid();
}
// Four bytes of the text from i (4-aligned): one LDS read inside the staged
// window (past the end: spaces).
__device__ __forceinline__ uint32_t word_at(const Txt& t, uint64_t n, uint64_t i) {
    if (i >= t.lo && i + 4 <= t.hi) return *reinterpret_cast<const uint32_t*>(t.s + (i - t.lo));
    uint32_t x = 0;
    for (int b = 0; b < 4; ++b) x |= (uint32_t)(i + b < n ? t[i + b] : ' ') << (8 * b);
    return x;
}
__device__ __forceinline__ Xfer thread_xfer(const Txt& t, uint64_t n, uint64_t b0) {
    Xfer x = xid();
    for (int wi = 0; wi < kPer / 4; ++wi) {
        const uint32_t w = word_at(t, n, b0 + 4 * wi);
#pragma unroll
        for (int b = 0; b < 4; ++b) x = compose(x, byte_xfer(t, b0 + 4 * wi + b, (uint8_t)(w >> (8 * b))));
    }
    return x;
}
// block-wide exclusive scan (in order) of the threads' transfers
__device__ __forceinline__ Xfer block_excl(Xfer x, Xfer* sx) {
    const int t = threadIdx.x;
    sx[t] = x;
    __syncthreads();
    for (int s = 1; s < kThreads; s <<= 1) {
        const Xfer y = t >= s ? compose(sx[t - s], sx[t]) : sx[t];
        __syncthreads();
        sx[t] = y;
        __syncthreads();
    }
    const Xfer r = t ? sx[t - 1] : xid();
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kThreads) void k_pass1(const uint8_t* __restrict__ text, uint64_t n,
                                                    Xfer* __restrict__ cx) {
    __shared__ Xfer sx[kThreads];
    __shared__ __attribute__((aligned(16))) uint8_t sw[kChunk + 2 * kHalo];
    const Txt t = stage(text, n, sw);
    const uint64_t b0 = (uint64_t)blockIdx.x * kChunk + (uint64_t)threadIdx.x * kPer;
    const Xfer x = thread_xfer(t, n, b0);
    const Xfer pre = block_excl(x, sx);
    if (threadIdx.x == kThreads - 1) cx[blockIdx.x] = compose(pre, x);
}

// one block: entry state of every chunk (and of the end, at entry[nchunks])
__global__ __launch_bounds__(1024) void k_scan1(const Xfer* __restrict__ cx, uint32_t nc,
                                                Entry* __restrict__ entry) {
    __shared__ Xfer sx[1024];
    const uint32_t t = threadIdx.x, per = (nc + 1023) / 1024;
    const uint32_t c0 = min(nc, t * per), c1 = min(nc, c0 + per);
    Xfer x = xid();
    for (uint32_t c = c0; c < c1; ++c) x = compose(x, cx[c]);
    sx[t] = x;
    __syncthreads();
    for (uint32_t s = 1; s < 1024; s <<= 1) {
        const Xfer y = t >= s ? compose(sx[t - s], sx[t]) : sx[t];
        __syncthreads();
        sx[t] = y;
        __syncthreads();
    }
    const Xfer pre = t ? sx[t - 1] : xid();
    int st = fstate(pre, 0), dp = pre.d0;            // from the start: outside, depth 0
    for (uint32_t c = c0; c < c1; ++c) {
        entry[c] = Entry{st, dp};
        dp += st ? cx[c].d1 : cx[c].d0;
        st = fstate(cx[c], st);
    }
    if (t == 1023) entry[nc] = Entry{fstate(sx[1023], 0), sx[1023].d0};
}

// This thread's entry (state, depth) inside its chunk.
__device__ __forceinline__ Entry thread_entry(const Txt& t, uint64_t n, const Entry* entry,
                                              Xfer* sx, uint64_t b0) {
    const Xfer pre = block_excl(thread_xfer(t, n, b0), sx);
    const Entry e = entry[blockIdx.x];
    return Entry{fstate(pre, e.state), e.depth + (e.state ? pre.d1 : pre.d0)};
}
// what a byte starts, given the state and depth before it
struct Kinds {
    bool num, row, key;
};
__device__ __forceinline__ Kinds kinds(uint8_t c, uint8_t p, int st, int dp) {
    Kinds k{false, false, false};
    if (st) return k;
    if (num_char(c)) {
        k.num = !num_char(p) && !is_alpha(p);         // (not the 'e' of true / false)
    } else if (c == '[') {
        k.row = dp == 2;
    } else if (c == '"') {
        k.key = dp == 1;
    }
    return k;
}
__device__ __forceinline__ void advance(const Txt& t, uint64_t i, uint8_t c, int& st, int& dp) {
    const Xfer x = byte_xfer(t, i, c);
    dp += st ? x.d1 : x.d0;
    st = fstate(x, st);
}

__global__ __launch_bounds__(kThreads) void k_pass2(const uint8_t* __restrict__ text, uint64_t n,
                                                    const Entry* __restrict__ entry,
                                                    Counts* __restrict__ cc) {
    __shared__ Xfer sx[kThreads];
    __shared__ uint32_t sn[kThreads], sr[kThreads], sk[kThreads];
    __shared__ __attribute__((aligned(16))) uint8_t sw[kChunk + 2 * kHalo];
    const Txt t = stage(text, n, sw);
    const uint64_t b0 = (uint64_t)blockIdx.x * kChunk + (uint64_t)threadIdx.x * kPer;
    Entry e = thread_entry(t, n, entry, sx, b0);
    uint32_t cn = 0, cr = 0, ck = 0;
    uint8_t p = b0 ? t[b0 - 1] : ' ';
    for (int wi = 0; wi < kPer / 4; ++wi) {
        const uint32_t w = word_at(t, n, b0 + 4 * wi);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint8_t c = (uint8_t)(w >> (8 * b));
            const Kinds kd = kinds(c, p, e.state, e.depth);
            cn += kd.num; cr += kd.row; ck += kd.key;
            advance(t, b0 + 4 * wi + b, c, e.state, e.depth);
            p = c;
        }
    }
    sn[threadIdx.x] = cn; sr[threadIdx.x] = cr; sk[threadIdx.x] = ck;
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sn[threadIdx.x] += sn[threadIdx.x + s];
            sr[threadIdx.x] += sr[threadIdx.x + s];
            sk[threadIdx.x] += sk[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) cc[blockIdx.x] = Counts{sn[0], sr[0], sk[0], 0};
}

__global__ __launch_bounds__(1024) void k_scan2(Counts* __restrict__ cc, uint32_t nc) {
    __shared__ uint32_t s[3][1024];
    const uint32_t t = threadIdx.x, per = (nc + 1023) / 1024;
    const uint32_t c0 = min(nc, t * per), c1 = min(nc, c0 + per);
    uint32_t a = 0, b = 0, k = 0;
    for (uint32_t c = c0; c < c1; ++c) { a += cc[c].num; b += cc[c].row; k += cc[c].key; }
    s[0][t] = a; s[1][t] = b; s[2][t] = k;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        uint32_t y[3];
        for (int q = 0; q < 3; ++q) y[q] = s[q][t] + (t >= d ? s[q][t - d] : 0u);
        __syncthreads();
        for (int q = 0; q < 3; ++q) s[q][t] = y[q];
        __syncthreads();
    }
    uint32_t on = t ? s[0][t - 1] : 0u, orr = t ? s[1][t - 1] : 0u, ok = t ? s[2][t - 1] : 0u;
    for (uint32_t c = c0; c < c1; ++c) {
        const Counts x = cc[c];
        cc[c] = Counts{on, orr, ok, 0};
        on += x.num; orr += x.row; ok += x.key;
    }
    if (t == 1023) cc[nc] = Counts{s[0][1023], s[1][1023], s[2][1023], 0};
}

// The previous non-whitespace byte before i (0 at the start).
__device__ __forceinline__ uint8_t prev_nonws(const Txt& t, uint64_t i, uint64_t* at = nullptr) {
    while (i > 0) {
        const uint8_t c = t[--i];
        if (!is_ws(c)) {
            if (at) *at = i;
            return c;
        }
    }
    return 0;
}

// One number token at i (ingest.hpp Parser::number, kParseSerde). Returns the
// error code (0: ok) and the value.
__device__ __forceinline__ uint32_t parse_number(const Txt& t, uint64_t n, uint64_t i,
                                                 const double* __restrict__ pow10, double* out,
                                                 uint64_t* end) {
    uint64_t p = i;
    const bool neg = t[p] == '-';
    if (neg) ++p;
    uint64_t sig = 0;
    bool over = false;
    const uint64_t d0 = p;
    while (p < n && is_digit(t[p])) {
        const uint64_t g = t[p] - '0';
        if (sig > (~0ull - g) / 10) over = true;
        sig = sig * 10 + g;
        ++p;
    }
    if (p == d0) { *end = p; return (uint32_t)kErrNumber; }
    int64_t fl = 0;
    if (p < n && t[p] == '.') {
        const uint64_t f0 = ++p;
        while (p < n && is_digit(t[p])) {
            const uint64_t g = t[p] - '0';
            if (sig > (~0ull - g) / 10) over = true;
            sig = sig * 10 + g;
            ++p;
        }
        if (p == f0) { *end = p; return (uint32_t)kErrNumber; }
        fl = (int64_t)(p - f0);
    }
    int64_t e10 = 0;
    if (p < n && (t[p] == 'e' || t[p] == 'E')) {
        ++p;
        bool en = false;
        if (p < n && (t[p] == '+' || t[p] == '-')) en = t[p++] == '-';
        const uint64_t e0 = p;
        while (p < n && is_digit(t[p])) {
            if (e10 < 100000) e10 = e10 * 10 + (t[p] - '0');
            ++p;
        }
        if (p == e0) { *end = p; return (uint32_t)kErrNumber; }
        if (en) e10 = -e10;
    }
    *end = p;
    if (p < n && num_char(t[p])) return (uint32_t)kErrNumber;    // e.g. "1.2.3", "1e5e"
    if (over) return (uint32_t)kErrOverflow;
    int64_t e = e10 - fl;
    double f = (double)sig;
    for (;;) {
        const int64_t ae = e < 0 ? -e : e;
        if (ae <= 308) {
            const double pw = pow10[ae];
            f = e >= 0 ? f * pw : f / pw;
            break;
        }
        if (f == 0.0) break;
        if (e >= 0) return (uint32_t)kErrRange;
        f /= 1e308;
        e += 308;
    }
    *out = neg ? -f : f;
    return 0;
}

// Structural check of a byte outside strings, given the depth before it.
// Inside member arrays (depth >= 2): JSON arrays of arrays of numbers -- each
// element after '[' or ',', each ',' / ']' after an element (1: an error the
// host keeps when it lies inside m, u, v or d; unknown members may hold
// anything). Object level (depth 0 / 1): the members' syntax (2: always an
// error). 0: fine.
__device__ __forceinline__ uint32_t struct_bad(const Txt& t, uint64_t i, int dp) {
    const uint8_t c = t[i];
    if (is_ws(c)) return 0;
    const uint8_t p = prev_nonws(t, i);
    if (dp >= 2) {
        if (num_char(c)) return 0;                   // tokens: parse_number + separators
        const bool elem_end = p == ']' || is_digit(p) || p == '.';
        if (c == '[') return (p == '[' || p == ',') ? 0 : 1;
        if (c == ']') return (p == '[' || elem_end) ? 0 : 1;
        if (c == ',') return elem_end ? 0 : 1;
        return 1;                                    // strings, objects, literals, ':'
    }
    const bool val_end = p == ']' || p == '}' || p == '"' || num_char(p) || is_alpha(p);
    if (dp == 0) return (c == '{' && p == 0) ? 0 : 2;   // one object, nothing around it
    if (dp < 0) return 2;
    // dp == 1: inside the top-level object
    if (c == ':') return p == '"' ? 0 : 2;
    if (c == ',') return val_end ? 0 : 2;
    if (c == '[' || c == '{') return p == ':' ? 0 : 2;
    if (c == '"') return (p == '{' || p == ',' || p == ':') ? 0 : 2;
    if (c == '}') return (p == '{' || val_end) ? 0 : 2;
    if (num_char(c) || is_alpha(c)) return (p == ':' || num_char(p) || is_alpha(p)) ? 0 : 2;
    return 2;
}

// Bytes of a walk that need a check against their neighbours: number tokens
// (parse + separators) and structural bytes outside strings (struct_bad).
__device__ __forceinline__ bool struct_candidate(uint8_t c, int dp) {
    return !is_ws(c) && !(dp >= 2 && num_char(c));
}
__device__ __forceinline__ int8_t clamp_depth(int dp) { return (int8_t)max(-1, min(dp, 127)); }

// Pass 3 walks each thread's bytes twice: counting, then writing row-open and
// key positions and collecting the block's number tokens and structural bytes
// (chunk offset, depth) in LDS in document order; the numbers are then parsed
// and the structural bytes checked one item per thread (a per-byte walk would
// run every thread's number parse on the whole wave).
__global__ __launch_bounds__(kThreads) void k_pass3(const uint8_t* __restrict__ text, uint64_t n,
                                                    const Entry* __restrict__ entry,
                                                    const Counts* __restrict__ off,
                                                    const double* __restrict__ pow10,
                                                    double* __restrict__ val, uint64_t* __restrict__ npos,
                                                    uint8_t* __restrict__ ndepth,
                                                    uint64_t* __restrict__ rpos, uint64_t* __restrict__ kpos,
                                                    unsigned long long* __restrict__ err) {
    __shared__ Xfer sx[kThreads];
    __shared__ uint32_t sn[kThreads], sr[kThreads], sk[kThreads], ss[kThreads];
    __shared__ __attribute__((aligned(16))) uint8_t sw[kChunk + 2 * kHalo];
    // a number token takes >= 2 bytes with its separator: <= kChunk / 2 per chunk
    __shared__ uint16_t lnum[kChunk / 2];
    __shared__ int8_t lnd[kChunk / 2];
    __shared__ uint16_t lst[kChunk];
    __shared__ int8_t lsd[kChunk];
    const Txt t = stage(text, n, sw);
    const uint64_t c0 = (uint64_t)blockIdx.x * kChunk;
    const uint64_t b0 = c0 + (uint64_t)threadIdx.x * kPer;
    const Entry e0 = thread_entry(t, n, entry, sx, b0);
    const uint8_t p0 = b0 ? t[b0 - 1] : ' ';
    Entry e = e0;
    uint32_t cn = 0, cr = 0, ck = 0, cs = 0;
    uint8_t p = p0;
    for (int wi = 0; wi < kPer / 4; ++wi) {
        const uint32_t w = word_at(t, n, b0 + 4 * wi);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t i = b0 + 4 * wi + b;
            const uint8_t c = (uint8_t)(w >> (8 * b));
            const Kinds kd = kinds(c, p, e.state, e.depth);
            cn += kd.num; cr += kd.row; ck += kd.key;
            cs += !e.state && i < n && struct_candidate(c, e.depth);
            advance(t, i, c, e.state, e.depth);
            p = c;
        }
    }
    sn[threadIdx.x] = cn; sr[threadIdx.x] = cr; sk[threadIdx.x] = ck; ss[threadIdx.x] = cs;
    __syncthreads();
    for (int s = 1; s < kThreads; s <<= 1) {
        const bool on = (int)threadIdx.x >= s;
        const uint32_t a = on ? sn[threadIdx.x - s] : 0u, b = on ? sr[threadIdx.x - s] : 0u,
                       c = on ? sk[threadIdx.x - s] : 0u, d = on ? ss[threadIdx.x - s] : 0u;
        __syncthreads();
        sn[threadIdx.x] += a; sr[threadIdx.x] += b; sk[threadIdx.x] += c; ss[threadIdx.x] += d;
        __syncthreads();
    }
    const uint32_t nb = sn[kThreads - 1], sb = ss[kThreads - 1];
    const Counts o = off[blockIdx.x];
    uint32_t jn = sn[threadIdx.x] - cn, js = ss[threadIdx.x] - cs;
    uint32_t ir = o.row + sr[threadIdx.x] - cr, ik = o.key + sk[threadIdx.x] - ck;
    e = e0;
    p = p0;
    for (int wi = 0; wi < kPer / 4; ++wi) {
        const uint32_t w = word_at(t, n, b0 + 4 * wi);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t i = b0 + 4 * wi + b;
            const uint8_t c = (uint8_t)(w >> (8 * b));
            const Kinds kd = kinds(c, p, e.state, e.depth);
            if (kd.num) { lnum[jn] = (uint16_t)(i - c0); lnd[jn] = clamp_depth(e.depth); ++jn; }
            if (kd.row) rpos[ir++] = i;
            if (kd.key) kpos[ik++] = i;
            if (!e.state && i < n && struct_candidate(c, e.depth)) { lst[js] = (uint16_t)(i - c0); lsd[js] = clamp_depth(e.depth); ++js; }
            advance(t, i, c, e.state, e.depth);
            p = c;
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += kThreads) {
        const uint64_t i = c0 + lnum[j];
        const int dp = lnd[j];
        double v = 0.0;
        uint64_t end = i;
        uint32_t code = parse_number(t, n, i, pow10, &v, &end);
        if (!code && dp >= 2) {
            // separators: after '[' or ',', before ',' or ']'
            const uint8_t p = prev_nonws(t, i);
            uint64_t q = end;
            while (q < n && is_ws(t[q])) ++q;
            const uint8_t nx = q < n ? t[q] : 0;
            if (!(p == '[' || p == ',') || !(nx == ',' || nx == ']')) code = (uint32_t)kErrSeparator;
        }
        const uint32_t at = o.num + j;
        val[at] = v;
        npos[at] = i;
        ndepth[at] = (uint8_t)(code ? 0x80u | code : (uint32_t)max(dp, 0));
    }
    for (uint32_t j = threadIdx.x; j < sb; j += kThreads) {
        const uint64_t i = c0 + lst[j];
        const uint32_t bad = struct_bad(t, i, lsd[j]);
        if (bad) {
            // structural errors: position list (bit 63: object level, always an
            // error; else the host keeps those inside m, u, v, d)
            const unsigned long long slot = atomicAdd(err, 1ull);
            if (slot < 255) err[1 + slot] = i | (bad == 2 ? (1ull << 63) : 0ull);
        }
    }
}

__device__ __forceinline__ uint32_t lower_bound(const uint64_t* a, uint32_t n, uint64_t x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__global__ void k_ranges(const uint64_t* __restrict__ npos, uint32_t nn, const uint64_t* __restrict__ rpos,
                         uint32_t nr, const uint64_t* __restrict__ q, uint32_t nq, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    out[2 * i] = lower_bound(npos, nn, q[i]);
    out[2 * i + 1] = lower_bound(rpos, nr, q[i]);
}
// err[0]: min over failures of (code << 48 | byte position)
__global__ __launch_bounds__(256) void k_validate(const uint8_t* __restrict__ nd, uint32_t lo, uint32_t hi,
                                                  uint32_t depth, const uint64_t* __restrict__ npos,
                                                  uint32_t nn, const uint64_t* __restrict__ rpos, uint32_t r0,
                                                  uint32_t rows, uint32_t cols,
                                                  unsigned long long* __restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (uint64_t)(hi - lo)) {
        const uint32_t k = lo + (uint32_t)i;
        const uint8_t d = nd[k];
        if (d & 0x80u) atomicMin(err, ((unsigned long long)(d & 0x7fu) << 48) | npos[k]);
        else if (d != depth) atomicMin(err, ((unsigned long long)kErrDepth << 48) | npos[k]);
    }
    if (i < rows) {
        const uint32_t first = lower_bound(npos, nn, rpos[r0 + i]);
        if (first != lo + (uint32_t)i * cols) atomicMin(err, ((unsigned long long)kErrRagged << 48) | rpos[r0 + i]);
    }
}

hipError_t launch_pass1(const uint8_t* text, uint64_t n, Xfer* chunk_x, hipStream_t st) {
    const uint64_t nc = (n + kChunk - 1) / kChunk;
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_pass1, dim3((uint32_t)nc), dim3(kThreads), 0, st, text, n, chunk_x);
    return hipGetLastError();
}
hipError_t launch_scan1(const Xfer* chunk_x, uint32_t nchunks, Entry* entry, hipStream_t st) {
    hipLaunchKernelGGL(k_scan1, dim3(1), dim3(1024), 0, st, chunk_x, nchunks, entry);
    return hipGetLastError();
}
hipError_t launch_pass2(const uint8_t* text, uint64_t n, const Entry* entry, Counts* chunk_c,
                        hipStream_t st) {
    const uint64_t nc = (n + kChunk - 1) / kChunk;
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_pass2, dim3((uint32_t)nc), dim3(kThreads), 0, st, text, n, entry, chunk_c);
    return hipGetLastError();
}
hipError_t launch_scan2(Counts* chunk_c, uint32_t nchunks, hipStream_t st) {
    hipLaunchKernelGGL(k_scan2, dim3(1), dim3(1024), 0, st, chunk_c, nchunks);
    return hipGetLastError();
}
hipError_t launch_pass3(const uint8_t* text, uint64_t n, const Entry* entry, const Counts* chunk_off,
                        const double* pow10, double* val, uint64_t* npos, uint8_t* ndepth,
                        uint64_t* rpos, uint64_t* kpos, unsigned long long* err, hipStream_t st) {
    const uint64_t nc = (n + kChunk - 1) / kChunk;
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_pass3, dim3((uint32_t)nc), dim3(kThreads), 0, st, text, n, entry, chunk_off,
                       pow10, val, npos, ndepth, rpos, kpos, err);
    return hipGetLastError();
}
hipError_t launch_ranges(const uint64_t* npos, uint32_t nn, const uint64_t* rpos, uint32_t nr,
                         const uint64_t* queries, uint32_t nq, uint32_t* out, hipStream_t st) {
    if (!nq) return hipSuccess;
    hipLaunchKernelGGL(k_ranges, dim3((nq + 63) / 64), dim3(64), 0, st, npos, nn, rpos, nr, queries, nq, out);
    return hipGetLastError();
}
hipError_t launch_validate(const uint8_t* ndepth, uint32_t lo, uint32_t hi, uint32_t depth,
                           const uint64_t* npos, uint32_t nn, const uint64_t* rpos, uint32_t r0,
                           uint32_t rows, uint32_t cols, unsigned long long* err, hipStream_t st) {
    const uint64_t work = std::max<uint64_t>(hi - lo, rows);
    if (!work) return hipSuccess;
    hipLaunchKernelGGL(k_validate, dim3((uint32_t)((work + 255) / 256)), dim3(256), 0, st, ndepth, lo, hi,
                       depth, npos, nn, rpos, r0, rows, cols, err);
    return hipGetLastError();
}

}  // namespace svdw_ingest_dev
