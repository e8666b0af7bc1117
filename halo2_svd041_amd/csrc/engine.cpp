// Host engine + C ABI (include/svdw.h) of the SVD-verify witness engine.
//
// Each reference function (src/matrix/mod.rs, src/svd/mod.rs) becomes:
//   1. a data-independent cell program built on the host by replaying the
//      halo2-base gadget sequence symbolically (PB below), and
//   2. one launch of the generic stage kernel over the elements, or the
//      dedicated GEMM / inner-product-row kernels.
// Offsets in the per-phase streams are known at enqueue time, so all work is
// asynchronous on the context's HIP stream. A context created with
// device = -1 is a "dry" planner: identical control flow, no device work,
// which is how svdw_plan_svd gets exact closed-form counts.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <array>
#include <functional>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/svdw.h"
#include "ingest.hpp"
#include "ingest_dev.hpp"
#include "kernels.hpp"

using namespace svdw;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
struct SvdwError {
    int code;
    std::string msg;
};
[[noreturn]] static void fail(int code, const std::string& msg) { throw SvdwError{code, msg}; }
static void hipck(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(SVDW_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
template <class F>
static int guarded(F&& f) {
    try {
        f();
        return SVDW_OK;
    } catch (const SvdwError& e) {
        g_err = e.msg;
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return SVDW_ENOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return SVDW_EINVAL;
    }
}
#define REQUIRE(cond, msg) \
    do {                   \
        if (!(cond)) fail(SVDW_EINVAL, msg); \
    } while (0)

// ------------------------------------------------------- host big integers
// Unsigned 256-bit integers (BigUint bounds of the range checks).
struct BigU {
    Fr v;
};
static BigU big_from_words(const uint64_t w[4]) {
    BigU b;
    for (int i = 0; i < 4; ++i) {
        b.v.w[2 * i] = (uint32_t)w[i];
        b.v.w[2 * i + 1] = (uint32_t)(w[i] >> 32);
    }
    return b;
}
static BigU big_from_u128(unsigned __int128 x) {
    BigU b;
    b.v = fr_zero();
    for (int i = 0; i < 4; ++i) b.v.w[i] = (uint32_t)(x >> (32 * i));
    return b;
}
static int big_bits(const BigU& b) {
    for (int i = 7; i >= 0; --i)
        if (b.v.w[i]) return 32 * i + 32 - __builtin_clz(b.v.w[i]);
    return 0;
}
static bool big_is_zero(const BigU& b) { return big_bits(b) == 0; }
static BigU big_pow2(uint32_t k) {     // k < 256
    BigU b;
    b.v = fr_zero();
    b.v.w[k / 32] = 1u << (k % 32);
    return b;
}
static BigU big_add_u32(const BigU& a, uint32_t s) {
    BigU r;
    Fr t = fr_from_u64(s);
    if (add256(r.v, a.v, t)) fail(SVDW_ERANGE, "bound overflows 256 bits");
    return r;
}
static BigU big_sub_u32(const BigU& a, uint32_t s) {
    BigU r;
    Fr t = fr_from_u64(s);
    if (sub256(r.v, a.v, t)) fail(SVDW_EINVAL, "bound underflow (bound must be >= 1)");
    return r;
}
static BigU big_shl1(const BigU& a) {
    BigU r;
    if (a.v.w[7] >> 31) fail(SVDW_ERANGE, "bound overflows 256 bits");
    for (int i = 7; i > 0; --i) r.v.w[i] = (a.v.w[i] << 1) | (a.v.w[i - 1] >> 31);
    r.v.w[0] = a.v.w[0] << 1;
    return r;
}
// biguint_to_fe: value mod p.
static Fr big_to_fr(const BigU& b) {
    Fr x = b.v, t;
    while (!sub256(t, x, fr_p())) x = t;   // at most a few subtractions (< 2^256)
    return x;
}
static Fr pow2_fr(uint32_t k) {
    Fr x = fr_from_u64(1);
    for (uint32_t i = 0; i < k; ++i) x = fr_add(x, x);
    return x;
}
static Fr fr_from_words(const uint64_t w[4]) { return big_to_fr(big_from_words(w)); }

// ------------------------------------------------------- program builder
// Replays halo2-base 0.4.1 gadgets on symbolic per-element values
// (SURVEY.md Appendix A); produces the micro-ops, cell and lookup slot ops.
struct PB {
    StageArgs a;
    uint32_t lb;
    // What MockProver checks on an element's C cells (svdw_check_gates), as
    // check words (kernels.hpp CHK_*): the offsets where halo2-base's
    // assign_region enables a basic gate a + b*c = d, and the copy constraints
    // -- a value's later cells against its first cell, a loaded value's first
    // cell against its source cell (view), range_check's last running sum
    // against the checked value (RangeChip::range_check's constrain_equal).
    std::vector<uint32_t> chk;
    // halo2-base's equality records of an element's cells (svdw_equalities), in
    // assign order: a Constant cell's (cell, value), an Existing cell's (source
    // cell, cell), range_check's constrain_equal(a, last running sum) -- as eq
    // words (kernels.hpp EQ_*): a constant slot, an earlier cell of the element,
    // the element's cell of a view (RegionChecks::esrc), or an external cell
    std::vector<uint32_t> eq;
    int kext = -1;            // constant slot holding an external cell's value (init_rand)
    bool vsrc[kMaxViews] = {true, true};   // false: the view holds values produced here
    static constexpr int EQ_AUTO = -1, EQ_WIT = -2;
    bool kconst = true;       // its constant-source cells are halo2-base Constants
    int8_t vload[kMaxV];      // view a value was loaded from (-1: computed)
    int16_t fullc[kMaxV];     // first cell holding the value in full (-1: none)
    void gate(uint32_t at) { chk.push_back(chk_gate(at)); }
    void copy_of(uint8_t v, uint32_t at) {    // cell `at` must equal value v's cell
        if (fullc[v] >= 0) chk.push_back(chk_copy((uint32_t)fullc[v], at));
        else if (vload[v] >= 0) chk.push_back(chk_view((uint32_t)vload[v], at));
    }
    explicit PB(uint32_t lookup_bits) : lb(lookup_bits) {
        memset(&a, 0, sizeof(a));
        memset(vload, -1, sizeof vload);
        for (auto& f : fullc) f = -1;
    }

    uint8_t newv() {
        if (a.nv >= (uint32_t)kMaxV) fail(SVDW_ERANGE, "stage needs too many element values");
        return (uint8_t)a.nv++;
    }
    uint8_t kidx(const Fr& c) {
        for (uint32_t k = 0; k < a.nk; ++k)
            if (fr_eq(a.K[k], c)) return (uint8_t)k;
        if (a.nk >= (uint32_t)kMaxK) fail(SVDW_ERANGE, "stage needs too many constants");
        a.K[a.nk] = c;
        return (uint8_t)a.nk++;
    }
    uint8_t K(const Fr& c) { return KSRC + kidx(c); }
    uint8_t K(uint64_t c) { return K(fr_from_u64(c)); }
    void op(uint8_t code, uint8_t dst, uint8_t x, uint8_t y, uint16_t p0 = 0, uint16_t p1 = 0) {
        if (a.nmo >= (uint32_t)kMaxMicro) fail(SVDW_ERANGE, "stage needs too many micro-ops");
        a.mo[a.nmo++] = MicroOp{code, dst, x, y, p0, p1};
    }
    static SlotOp slot(uint8_t src, uint32_t lo, uint32_t nbits) {
        if (nbits >= 256) nbits = 0;
        return SlotOp{src, (uint8_t)lo, (uint8_t)nbits, 0};
    }
    // cell `at` holds a copy of value v (QuantumCell::Existing of v's cell)
    void eq_of_value(uint8_t v, uint32_t at) {
        if (vload[v] >= 0 && vsrc[vload[v]]) eq.push_back(eq_word(EQ_VIEW, (uint32_t)vload[v], at));
        else if (fullc[v] >= 0) eq.push_back(eq_word(EQ_LOCAL, (uint32_t)fullc[v], at));
    }
    // eqk: EQ_AUTO -- a Constant for a constant slot (kconst), the external cell
    // for kext, an Existing copy for a value's full cell seen before (or loaded
    // from a source view), else a Witness; EQ_WIT: a Witness; >= 0: an Existing
    // copy of the element's cell eqk (range_check's last limb)
    void cell(uint8_t src, uint32_t lo = 0, uint32_t nbits = 0, int eqk = EQ_AUTO) {
        if (a.C >= (uint32_t)kMaxAdv) fail(SVDW_ERANGE, "stage has too many cells per element (raise lookup_bits)");
        const SlotOp s = slot(src, lo, nbits);
        if (eqk >= 0) {
            eq.push_back(eq_word(EQ_LOCAL, (uint32_t)eqk, a.C));
        } else if (eqk == EQ_AUTO) {
            if (src >= KSRC) {
                const int k = src - KSRC;
                if (k == kext) eq.push_back(eq_word(EQ_EXT, 0, a.C));
                else if (kconst) eq.push_back(eq_word(EQ_CONST, (uint32_t)k, a.C));
            } else if (s.lo == 0 && s.nbits == 0) {
                eq_of_value(src, a.C);
            }
        }
        if (src < KSRC && s.lo == 0 && s.nbits == 0) {      // the value itself: a copy or its first cell
            copy_of(src, a.C);
            if (fullc[src] < 0) fullc[src] = (int16_t)a.C;
        }
        a.adv[a.C++] = s;
    }
    void look(uint8_t src, uint32_t lo = 0, uint32_t nbits = 0) {
        if (a.L >= (uint32_t)kMaxLk) fail(SVDW_ERANGE, "stage has too many lookups per element (raise lookup_bits)");
        a.lk[a.L++] = slot(src, lo, nbits);
    }
    // --- element values
    uint8_t load(int view_idx) {
        uint8_t v = newv();
        op(MO_LOAD, v, (uint8_t)view_idx, 0);
        vload[v] = (int8_t)view_idx;
        return v;
    }
    uint8_t addk(uint8_t x, const Fr& k) {
        uint8_t t = newv();
        op(MO_ADDK, t, x, kidx(k));
        return t;
    }
    // --- GateChip
    uint8_t g_add_k(uint8_t x, const Fr& k) {       // add(x, Constant(k)): [x, k, 1, x+k]
        uint8_t t = addk(x, k);
        gate(a.C);
        cell(x); cell(K(k)); cell(K(1)); cell(t);
        return t;
    }
    uint8_t g_sub_k(uint8_t x, const Fr& k) {       // sub(x, Constant(k)): [x-k, k, 1, x]
        uint8_t d = addk(x, fr_neg(k));
        gate(a.C);
        cell(d); cell(K(k)); cell(K(1)); cell(x);
        return d;
    }
    uint8_t g_sub(uint8_t x, uint8_t y) {           // sub: [x-y, y, 1, x]
        uint8_t d = newv();
        op(MO_SUB, d, x, y);
        gate(a.C);
        cell(d); cell(y); cell(K(1)); cell(x);
        return d;
    }
    uint8_t g_mul(uint8_t x, uint8_t y) {           // mul: [0, x, y, x*y]
        uint8_t m = newv();
        op(MO_MUL, m, x, y);
        gate(a.C);
        cell(K(0)); cell(x); cell(y); cell(m);
        return m;
    }
    void g_is_equal(uint8_t x, uint8_t y) {         // sub + is_zero: 12 cells
        uint8_t d = g_sub(x, y);
        uint8_t z = newv();
        uint8_t inv = newv();
        (void)inv;
        op(MO_ISZERO, z, d, 0);
        gate(a.C);
        gate(a.C + 4);
        cell(z); cell(d); cell((uint8_t)(z + 1)); cell(K(1));
        cell(K(0)); cell(d); cell(z); cell(K(0));
    }
    // --- RangeChip::range_check
    void range_check(uint8_t v, uint32_t bits) {
        if (bits == 0) return;    // assert_is_const(a, 0): no cells
        if (bits > 254 + lb) fail(SVDW_ERANGE, "range_check bits too large");
        const uint32_t n = (bits + lb - 1) / lb, rem = bits % lb;
        uint8_t lsrc = v;
        uint32_t llo = 0, lnb = 0;
        int lastc = EQ_AUTO;                        // the last limb's cell (n > 1)
        if (n == 1) {
            look(v);
        } else {
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t lo = i * lb;
                uint8_t src = v;
                uint32_t slo = lo, snb = lb;
                if (lo >= 256) { src = K(0); slo = 0; snb = 0; }
                if (i == 0) {
                    lastc = (int)a.C;
                    cell(src, slo, snb, EQ_WIT);   // limbs are witnesses
                } else {
                    gate(a.C - 1);                  // [s_(i-1), l_i, 2^(i lb), s_i]
                    lastc = (int)a.C;
                    cell(src, slo, snb, EQ_WIT);
                    cell(K(pow2_fr(lo)));
                    cell(v, 0, (i + 1) * lb, EQ_WIT);   // running sum = v mod 2^((i+1) lb)
                    if (i + 1 == n && n * lb < 256) copy_of(v, a.C - 1);   // constrain_equal(a, sum)
                    if (i + 1 == n) eq_of_value(v, a.C - 1);
                }
                look(src, slo, snb);
                lsrc = src; llo = slo; lnb = snb;
            }
        }
        if (rem == 1) {                             // assert_bit: [0, l, l, l]
            gate(a.C);
            cell(K(0)); cell(lsrc, llo, lnb, lastc); cell(lsrc, llo, lnb, lastc); cell(lsrc, llo, lnb, lastc);
        } else if (rem > 1) {                       // mul(last, 2^(lb-rem)), looked up
            const uint32_t sh = lb - rem;
            uint8_t m = newv();
            if (n == 1) op(MO_FDBL, m, v, (uint8_t)sh);
            else if ((n - 1) * lb >= 256) op(MO_ADDK, m, v, kidx(fr_zero()));   // unreachable in practice
            else op(MO_LIMBSHL, m, v, (uint8_t)sh, (uint16_t)((n - 1) * lb), (uint16_t)lb);
            gate(a.C);
            cell(K(0)); cell(lsrc, llo, lnb, lastc); cell(K(pow2_fr(sh))); cell(m);
            look(m);
        }
    }
    // --- RangeChip::check_less_than(a, Constant(b), bits)
    void check_less_than_k(uint8_t x, const BigU& b, uint32_t bits) {
        Fr pw = pow2_fr(bits), bf = big_to_fr(b);
        uint8_t t3 = addk(x, pw);                  // a + 2^bits
        uint8_t t2 = addk(t3, fr_neg(bf));         // a + 2^bits - b
        gate(a.C);
        gate(a.C + 3);
        cell(t2); cell(K(bf)); cell(K(1)); cell(t3); cell(K(fr_neg(pw))); cell(K(1)); cell(x);
        range_check(t2, bits);
    }
    void check_big_less_than_safe(uint8_t x, const BigU& bnd) {
        uint32_t rb = (big_bits(bnd) + lb - 1) / lb * lb;
        range_check(x, rb);
        check_less_than_k(x, bnd, rb);
    }
    // RangeChip::div_mod(t, 2^p, nb) [ext halo2-base 0.4.1]: [r, 2^p, q, t], then
    // check_big_less_than_safe(q, 2^nb / 2^p + 1), check_big_less_than_safe(r, 2^p)
    uint8_t div_mod_pow2(uint8_t t, uint32_t p, uint32_t nb) {
        uint8_t q = newv();
        op(MO_SHR, q, t, 0, (uint16_t)p);
        uint8_t r = newv();
        op(MO_LIMBSHL, r, t, 0, 0, (uint16_t)p);
        gate(a.C);
        cell(r); cell(K(pow2_fr(p))); cell(q); cell(t);
        check_big_less_than_safe(q, big_add_u32(big_pow2(nb - p), 1));
        check_big_less_than_safe(r, big_pow2(p));
        return q;
    }
    // FixedPointChip041::signed_div_scale, parameterised (oracle/pyoracle.py
    // signed_div_scale; chip source unavailable, parity unpinned): add 2^s,
    // div_mod by 2^p on nb bits, subtract 2^(s-p). Returns the quotient value.
    uint8_t signed_div_scale(uint8_t x, uint32_t p, uint32_t s, uint32_t nb) {
        uint8_t t = g_add_k(x, pow2_fr(s));
        uint8_t q = div_mod_pow2(t, p, nb);
        return g_sub_k(q, pow2_fr(s - p));
    }
    // FixedPointChip041::qsqrt (ZkVector::norm / dist, src/matrix/mod.rs:124-131,
    // 156-164), parameterised (the chip's source is unavailable: PARITY UNPINNED;
    // oracle/pyoracle.py qsqrt): y = floor(sqrt(a 2^P)) for a fixed-point a in
    // [0, 2^nbits), as load_witness(y) with range_check(y, ny), t = mul(a, 2^P),
    // d = sub(t, mul(y, y)) and f = sub(mul(y, 2), d), both range-checked on nd
    // bits: 0 <= t - y^2 <= 2y, i.e. y^2 <= t < (y + 1)^2.
    uint8_t qsqrt(uint8_t x, uint32_t p, uint32_t nbits) {
        const uint32_t ny = (nbits + p + 1) / 2 + 1, nd = ny + 1;
        uint8_t t = newv();
        op(MO_FDBL, t, x, (uint8_t)p);                   // a 2^P (< 2^254: an integer)
        uint8_t y = newv();
        op(MO_ISQRT, y, t, 0);
        cell(y);                                          // load_witness(y)
        range_check(y, ny);
        gate(a.C);
        cell(K(0)); cell(x); cell(K(pow2_fr(p))); cell(t);   // mul(a, 2^P)
        uint8_t y2 = g_mul(y, y);
        uint8_t d = g_sub(t, y2);
        range_check(d, nd);
        uint8_t e = newv();
        op(MO_FDBL, e, y, 1);
        gate(a.C);
        cell(K(0)); cell(y); cell(K(2)); cell(e);          // mul(y, 2)
        uint8_t f = g_sub(e, d);
        range_check(f, nd);
        return y;
    }
    // check_abs_less_than (src/matrix/mod.rs:425-435)
    void check_abs_less_than(uint8_t x, const BigU& bnd) {
        if (big_is_zero(bnd)) fail(SVDW_EINVAL, "check_abs_less_than: bound must be >= 1");
        BigU nb = big_sub_u32(big_shl1(bnd), 1);
        uint8_t t = g_add_k(x, big_to_fr(big_sub_u32(bnd, 1)));
        check_big_less_than_safe(t, nb);
    }
};

// -------------------------------------------------------------- context
struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
};
struct Stream {
    Fr* adv = nullptr;
    uint64_t n = 0, cap = 0;
    Fr* lk = nullptr;
    uint64_t nl = 0, lcap = 0;
};
struct svdw_ctx {
    // SVDW_HOST_TRACE=1: host-side timestamps of svd_witness's enqueue points on
    // stderr (µs since the call started), to find host waits inside a call
    bool host_trace = false;
    std::chrono::steady_clock::time_point ht0;
    int device = -1;
    bool dry = true;
    hipStream_t st = nullptr;
    uint32_t P = 32, LB = 19;
    Stream ph[2];
    // Pipelined svd_witness ("pipeline", svd_witness_pipe): consecutive
    // witnesses alternate between two sets of cell streams (ph and alt), so call
    // j's product chain (st) runs beside call j - 1's HBM-bound stages (st2) and
    // row scans (st3) instead of after them. Call j's st first waits for call
    // j - 2's tail (tail_ev[parity]: its last work on st2 / st3), the last user
    // of this cell set and of this half of the bit-length words. Anything else
    // that touches the streams after a pipelined call settles first (settle).
    Stream alt[2];
    int pipeline = 1;                       // "pipeline": 1 on, 0 off
    bool in_pipe = false;                   // inside a pipelined svd_witness
    int pipe_par = 0;                       // this call's parity (cell set, bit words)
    hipEvent_t tail_ev[2][2] = {};          // [parity][st2, st3]
    bool tail_valid[2] = {false, false};
    bool tail_pending = false;              // the last pipelined call's tail not yet joined into st
    int tail_last = 0;
    size_t mem_total = 0;                   // device memory (hipMemGetInfo at create)
    // "lanes" 2: svdw_verify_mul_witness on its captured-graph path alternates
    // between two complete context states, this one and `lane` (own streams,
    // cells, scratch, graph). The states are exchanged (std::swap) at the start
    // of a call, so call j + 1 runs on the other state's streams beside call j
    // and the handle always holds the latest call's cells. sync, stream_wait,
    // stream_signal, graph_stats and destroy cover both; lane / lanes stay with
    // the handle.
    int lanes = 2;                          // (config 2, same box: 0.081 -> 0.058 ms per call)
    svdw_ctx* lane = nullptr;
    // svdw_stream_wait's event (the caller's stream), not yet waited on by
    // st2 / st3: st waits at once; the side streams inherit it through
    // after_previous or the captured graph's fork from st, and the pipelined
    // svd_witness (whose side streams do not wait for st) waits explicitly
    hipEvent_t xwait_side = nullptr;
    DBuf f64in, digA, digB, digC, w1c, w1t, w2c, w2t, bits, gpc, gtab, crtR, gbits, chk, chkg;
    DBuf gpc_alt, gtab_alt;                 // pipelined svd_witness: gamma tables of the other parity
    DBuf wbc[kMaxScanJobs], wbt[kMaxScanJobs];   // b.v per batched verify_mul (canonical, table)
    // gamma^j (canonical gpc, scaled table gtab, kernels.hpp kTabSlots) of the
    // current verify_mul calls: recomputed for every witness (a fresh challenge
    // each time). svd_witness queues it first thing on a side stream (gp_ev).
    Fr gp_gamma{};
    uint32_t gp_len = 0;
    hipEvent_t gp_ev = nullptr;
    hipStream_t gp_st = nullptr;            // the stream gp_ev was recorded on
    // verify_mul_witness: the one cell and gamma powers written by k_gamma_prep
    // (phase-1 offsets one_off / pows_off for d), so verify_mul does not launch them
    struct PowsPre {
        bool on = false;
        uint64_t one_off = 0, pows_off = 0;
        uint32_t d = 0;
    } pows_pre;             // gamma_prep queued ahead (svd_witness)
    // Device bit-length words of matrices written in this witness (svd_witness:
    // quantized m, u, v at dbitw[0..2]): the row scans decide their operand
    // width on the device from these (NaSpec), so the host never waits for them.
    struct DevBits { svdw_mat m; int16_t word; };
    std::vector<DevBits> dwords;
    const unsigned* dbitw = nullptr;
    // Known magnitude bounds of matrices written in this witness: cell (i, j) of
    // `m` satisfies |signed value| < 2^bits. Cleared with the streams.
    struct MatBits { svdw_mat m; uint32_t bits; };
    std::vector<MatBits> mbits;
    // products c_s = a * b (K = 2^lk-bounded inner dimension): |c_s| < 2^(bits_a + bits_b + lk)
    struct Prod { svdw_mat cs, a, b; uint32_t lk; };
    std::vector<Prod> prods;
    // svd_witness: bit lengths of quantized m, u, v travel to pinned host memory
    // behind ev_bits; the host waits for them only where the GEMM launches need
    // them (fetch_bits), with check stages already queued on the device.
    uint32_t* hbits = nullptr;
    hipEvent_t ev_bits = nullptr;
    bool bits_pending = false;
    uint32_t qbits[3] = {0, 0, 0};
    svdw_mat qmat[3] = {};
    // built-in event profiler (svdw_profile_*): one start/stop event pair per launch
    bool prof = false;
    std::string prof_filter;                // record only kernels whose name starts with this
    struct Rec {
        std::string name;
        double bytes, ops;
        hipEvent_t e0, e1;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    int gemm_impl = SVDW_GEMM_MFMA;         // svdw_set_gemm_impl
    // STAGE_* (4 KiB-aligned block store windows; "stage_rot" 1: phase B from a
    // block-dependent window on, tools/r6/place_ab.py over 8 placements of the
    // 1024^2 cell streams: 1.739-1.891 -> 1.728-1.825 ms, mean 1.815 -> 1.751)
    uint32_t stage_flags = STAGE_ALIGN | STAGE_ROT;
    uint32_t stage_elems = kStageElems;     // "stage_elems": elements per stage block (16..256)
    hipStream_t stream_id[3] = {};          // st, st2, st3 as created (st / st2 / st3 are swapped at times)
    int gemm_crt = 1;                       // "gemm_crt": multi-modular GEMM (else digits)
    // "gemm_kern": CRT GEMM kernel (CrtBatch::kern); -1: wide tiles or the
    // persistent grid for a product queued on its own (svdw_honest_prover_mat_mul,
    // gemm_solo; CrtBatch::kern 3), one block per unit inside the witness calls,
    // beside their stage kernels
    int gemm_kern = -1;
    bool gemm_solo = false;
    int res_wait = -1;                      // "res_wait": stages wait for the residue planes
    int place_trials = 6;                   // "place_trials": candidate placements of a new cell stream
    bool gemm_batched = false;              // this witness's products went out as one batch
    bool res_f64 = true;                    // "res_f64": CRT residue planes of m, u, v from the
                                            // f64 inputs, one launch (else from the cells)
    const double* svd_f64[3] = {nullptr, nullptr, nullptr};   // device f64 m, u, v of svd_witness
    int phase1_overlap = 1;                 // "phase1_overlap": 0 off, 1 on st2 behind the
                                            // GEMMs, 2 on st3 from quantization on
    bool prelaunched = false;               // this witness's products were queued on st2
    int prod_cell = 1;                      // "prod_cell": svd_witness's products (residues, GEMM,
                                            // combine) on the cell stream and the u / v bounds and
                                            // u.d beside them on st2 (1), not (0); -1: on row-sharded
                                            // ranks only. On by default: the product chain is the
                                            // critical path sharded, and unsharded it measured
                                            // 2.5 % faster at 1024^2 and 2048^2, neutral at 512^2
    bool prod_on_cell = false;              // this witness's products went on the cell stream
    uint32_t hold_us = 0;                   // "hold_us": timing aid, st spins this long first
    Fr ext_gamma{};                          // init_rand of the last verify_mul (equality source 2)
    uint64_t ext_off = 0;                    // its cell in the RLC context
    // ctx_rlc of the last svd_witness with rlc_prefix: [E(one), E(zero), W(gamma)]
    // and the phase-1 offsets of the two ctx_gate constants its first cells copy
    struct RlcTrace {
        uint32_t n = 0;
        Fr cells[3];
        uint64_t src[2];
    } rlc;
    bool rlc_prefix = false;                 // "rlc_prefix": svd_witness's phase 1 starts with the
                                             // ctx_gate cells of load_rlc_cache(.., 1)
    int p1_at = -1;                         // "p1_at": phase 1 on st3 (mode 2) enqueued after
                                            // phase-0 stage 0 / 1 / 2 (the u, v bounds), 3: at the
                                            // end; -1: auto (tools/shard_sim.py --opt p1_at=):
                                            // 0 on a rank of >= 4, 3 of 2-3, else 1
    std::function<void(const svdw_svd_payload&)> early_p1;   // that enqueue (svd_witness)
    // pipelined svd_witness: "dchk_at" the d checks on the cell stream behind
    // the products (0), on st2 with the bounds and u.d (1) or on st3 ahead of
    // phase 1 (2); "gamma_at" k_gamma_prep at the head of the cell stream (0) or
    // of st3 (1); -1: st3 on a row-sharded rank, whose cell stream (quantize ->
    // residues -> GEMM -> combine, then the diff on st2) is the step's chain
    // (8-way rank 0.331 -> 0.316-0.321 ms; 1024^2 / 512^2 +0.5 %, r5p / r5q)
    int dchk_at = 0, gamma_at = -1;
    // Host-side replays cached for repeated calls of the same shape: the dry
    // plan of svd_witness's stream sizes (key: N, M, config) and prelaunch's
    // product offsets (key: stream state at entry, operand views, bounds).
    std::vector<uint64_t> plan_key, plan_val, log_key, log_val;
    std::vector<hipEvent_t> gemm_done;      // their completion events (this witness)
    std::vector<hipEvent_t> wait_before_cs; // verify_mul_many: wait before the c_s scans
    // Row-block sharding of one witness: this context computes the
    // rows [R rank / world, R (rank + 1) / world) of every row-parallel stage
    // (R = that stage's row count) into the globally laid-out streams; shared
    // inputs (quantized operands, single constants, the Freivalds b.g values)
    // are computed in full. `owned` lists the cell ranges this rank is the
    // source of, for reassembly.
    uint32_t shard_rank = 0, shard_world = 1;
    struct Seg { uint32_t phase, lookup; uint64_t off, n; };
    std::vector<Seg> owned;
    DBuf bvfull[kMaxScanJobs];              // shard mode: full b.g values per verify_mul
    // svd_witness's quantized matrices and their device f64 inputs (u, v): a
    // row-sharded rank takes b.g of b = u^T, v^T from the f64 rows directly
    // (k_colsum_f64), not from cells. Cleared at the end of the witness.
    struct F64Src { svdw_mat m; const double* x; };
    // loaded regions whose f64 source is on the device for the current call:
    // launches read them through VIEW_F64 (quantized in registers) instead of
    // waiting for the quantized cells (f64_view)
    struct F64Region { uint32_t phase; uint64_t off, n; const double* x; };
    std::vector<F64Region> f64reg;
    bool f64_views = true;                  // "f64_views"
    std::vector<F64Src> f64src;
    DBuf colpart;
    DBuf qfold;                             // k_quantize_multi's fold counters + group maxima
    // second stream: GEMMs overlap the HBM-bound stages; third: phase 1
    hipStream_t st2 = nullptr;
    hipStream_t st3 = nullptr;
    hipStream_t st_cell = nullptr;          // the cell stream proper (st is swapped at times)
    hipEvent_t xev[4] = {};                 // svdw_stream_wait / _signal (caller's stream)
    // svdw_mark ring: slot k holds ticket t[k]'s events (one per stream of
    // both lanes), recorded on the context's own streams (no waits); it stays
    // with the handle when lanes exchange states (lane_switch)
    static constexpr int kMarks = 16;
    struct Marks {
        hipEvent_t ev[kMarks][6] = {};
        uint64_t t[kMarks] = {};
        uint8_t used[kMarks] = {};
        uint64_t seq = 0;
    } mk;
    bool overlap = true;
    struct PreGemm {
        uint64_t off;
        hipEvent_t ev;
        hipStream_t st;                     // the stream it was launched on
    };
    std::vector<PreGemm> pre;               // GEMMs launched ahead on st2, in append order
    hipStream_t pre_wait_st = nullptr;      // the last (stream, event) waited on for them
    hipEvent_t pre_wait_ev = nullptr;
    std::vector<svdw_region> layout;        // every appended region of the current witness
    // per region: gate offsets within one element's cells and cells per element
    // (program regions; empty otherwise; svdw_check_gates)
    std::vector<RegionChecks> layout_chk;
    // distinct constant cell values (halo2-base Constant / load_constant):
    // the fixed-column count of svdw_physical_layout
    std::set<std::array<uint32_t, 8>> consts;
    // svdw_physical_layout's plan: per phase, the virtual index of each advice
    // column's row 0 and each full column's break point
    struct Phys {
        bool valid = false;
        uint32_t k = 0, min_rows = 0;
        uint64_t R = 0;
        std::vector<uint64_t> start[2], bp[2];
    } phys;
    DBuf gateq[2];
    std::vector<uint64_t>* gemm_log = nullptr;   // dry run: offsets of honest_prover_mat_mul
    std::vector<hipEvent_t> deps;           // dependency events (no timing)
    size_t dep_next = 0;
    // Stage batches (BatchScope, "stage_batch"): stage launches on a stream with
    // an open batch are collected and issued as k_stage_multi launches when the
    // scope closes, when a stage reads cells a pending stage writes, or before
    // anything else is recorded or launched on that stream.
    struct Pending {
        StageArgs a;
        std::string name;
        double bytes;
    };
    // A batch holds groups issued in order, one k_stage_multi launch each: a
    // stage joins the group after the last one holding a stage whose cells it
    // reads, so a dependent stage (entries_in_desc_order's range checks of its
    // subtractions) defers only itself, not the independent stages after it.
    struct Batch {
        hipStream_t st;
        std::vector<std::vector<Pending>> groups;
        size_t last = 0;                   // group of the latest stage
    };
    std::vector<Batch> batches;
    bool stage_batch = true;
    bool stage_front = false;               // stage_launch: the stage goes ahead of the batch's groups
    // device ingest (svdw_parse_svd_input_device) scratch
    DBuf ing_x, ing_e, ing_c, ing_p10, ing_val, ing_npos, ing_nd, ing_rpos, ing_kpos, ing_err, ing_q;
    // device equality records (eq_gen_device)
    DBuf eq_cp, eq_ks, eq_reg, eq_w, eq_k, eq_err, eq_st;
    // ---- captured verify_mul_witness ("graph", vm_graph): the launch sequence of
    // a device-input call is captured once into a HIP graph (the second call of
    // a shape, when every buffer is sized) and replayed by later calls of the
    // same key; gamma enters only through k_gamma_prep, launched eagerly on st
    // ahead of the graph (gp_external), so the graph itself is gamma-free.
    int graph_vm = 1;                       // "graph": 0 off, 1 verify_mul_witness
    // "vm_linear": the captured verify_mul_witness runs on the context stream
    // alone (st2 = st3 = st while it is queued: a linear graph, no fork / join
    // events); concurrency comes from the two lanes instead. `linear` is set
    // while such a call is queued: stream_dep returns lin_ev (never recorded)
    // and dep_wait skips it.
    int vm_linear = 1;
    bool linear = false;
    hipEvent_t lin_ev = nullptr;
    bool capturing = false;                 // st is capturing: no allocation, no sync
    bool gp_external = false;               // verify_mul_witness: k_gamma_prep already queued
    const Fr* gp_ext_one = nullptr;         // the one cell it wrote (null: none)
    uint64_t epoch = 0;                     // bumped by every allocation / option change
    // (layout_chk index, eqk slot) of the constants that hold gamma (the
    // verify_mul gamma powers' init_rand), patched on replay
    std::vector<std::pair<size_t, int>> gamma_slots;
    struct VmGraph {
        std::vector<uint64_t> key, seen;    // replay key; the last eager call's key
        hipGraphExec_t exec = nullptr;
        // host state the captured call left behind (restored on replay)
        std::vector<svdw_region> layout;
        std::vector<RegionChecks> layout_chk;
        std::set<std::array<uint32_t, 8>> consts;
        std::vector<std::pair<size_t, int>> gamma_slots;
        std::vector<MatBits> mbits;
        std::vector<Prod> prods;
        std::vector<DevBits> dwords;
        const unsigned* dbitw = nullptr;
        uint64_t ext_off = 0;
        svdw_counts counts{};
        uint64_t replays = 0, captures = 0;
    } vmg;
};

static void flush_batch(svdw_ctx* c, hipStream_t s, hipStream_t waiter = nullptr, hipEvent_t then_wait = nullptr);
// debug logs (read once: getenv scans the environment)
static bool env_flag(const char* name) { const char* v = getenv(name); return v && *v && *v != '0'; }
static const bool g_batch_log = env_flag("SVDW_BATCH_LOG");
static const bool g_stage_log = env_flag("SVDW_STAGE_LOG");
static void sync(svdw_ctx* c) {
    if (c->dry) return;
    REQUIRE(!c->capturing, "internal: synchronisation during graph capture");
    hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");
    hipck(hipStreamSynchronize(c->st2), "hipStreamSynchronize");
    if (c->st3) hipck(hipStreamSynchronize(c->st3), "hipStreamSynchronize");
    c->tail_pending = false;
    if (c->lane) sync(c->lane);
}
// After a pipelined svd_witness its tail (st2, st3) is not joined into st:
// anything else queued on the context waits for it first.
static void settle(svdw_ctx* c) {
    if (c->dry || !c->tail_pending || c->in_pipe) return;
    for (int k = 0; k < 2; ++k)
        hipck(hipStreamWaitEvent(c->st, c->tail_ev[c->tail_last][k], 0), "hipStreamWaitEvent");
    c->tail_pending = false;
}
// Device bytes held by a set of cell streams (both phases, advice + lookups).
static double set_bytes(const Stream (&s)[2]) {
    return 32.0 * (double)(s[0].cap + s[0].lcap + s[1].cap + s[1].lcap);
}
// Free the pipeline's other cell set (after the work that may read it).
static void release_alt(svdw_ctx* c) {
    if (c->dry || set_bytes(c->alt) == 0) return;
    sync(c);
    for (auto& s : c->alt) {
        if (s.adv) hipck(hipFree(s.adv), "hipFree");
        if (s.lk) hipck(hipFree(s.lk), "hipFree");
        s = Stream{};
    }
    ++c->epoch;
}
// Dependency recorded on `from`; `to` waits for it (cross-stream dependency).
// The returned handle is waited on later with dep_wait. (Round 4 measured the
// alternative of stream values, hipStreamWriteValue32 / hipStreamWaitValue32,
// once its flag initialisation was ordered: the suite passed, but 512^2 went
// 0.417 -> 0.444 ms and 1024^2 2.078 -> 2.100 ms, 8-way ranks unchanged --
// HIP runs those waits and writes as kernels of their own -- so it was removed.)
static hipEvent_t stream_dep(svdw_ctx* c, hipStream_t from, hipStream_t to) {
    if (c->linear) {                                   // one stream: order is implicit
        flush_batch(c, from);
        return c->lin_ev;
    }
    if (c->dep_next == c->deps.size()) {
        hipEvent_t e;
        // same-device consumer only: agent-scope release, no system-scope writeback
        hipck(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice),
              "hipEventCreate");
        c->deps.push_back(e);
    }
    hipEvent_t e = c->deps[c->dep_next++];
    flush_batch(c, from);
    if (g_batch_log) fprintf(stderr, "dep %p -> %p\n", (void*)from, (void*)to);
    hipck(hipEventRecord(e, from), "hipEventRecord");
    if (to) hipck(hipStreamWaitEvent(to, e, 0), "hipStreamWaitEvent");
    return e;
}
// `s` waits for a dependency stream_dep returned (or any other event)
static void dep_wait(svdw_ctx* c, hipStream_t s, hipEvent_t e) {
    if (c->linear && e == c->lin_ev) return;
    hipck(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent");
}
// (Round 4 removed "gemm_priority", a high-priority second stream at 512 <=
// max(N, M) < 1024: +2 % in round 2's tools/ab.py runs, but bench.py at 512^2
// P=32 measured 0.68 ms with it and 0.41 ms without -- the stream created
// mid-run shares a hardware queue with the cell stream, GPU_MAX_HW_QUEUES = 4.)
static bool same_cells(const svdw_mat& a, const svdw_mat& b) {
    if (a.phase != b.phase || a.off != b.off) return false;
    return (a.rows == b.rows && a.cols == b.cols && a.rs == b.rs && a.cs == b.cs) ||
           (a.rows == b.cols && a.cols == b.rows && a.rs == b.cs && a.cs == b.rs);
}
static void reg_bits(svdw_ctx* c, const svdw_mat& m, uint32_t bits) {
    if (bits == ~0u) return;
    for (auto& r : c->mbits)
        if (same_cells(r.m, m)) { r.bits = bits; return; }
    c->mbits.push_back({m, bits});
}
static uint32_t bits_of(const svdw_ctx* c, const svdw_mat& m) {
    for (auto& r : c->mbits)
        if (same_cells(r.m, m)) return r.bits;
    for (auto& p : c->prods)
        if (same_cells(p.cs, m)) {
            const uint32_t ba = bits_of(c, p.a), bb = bits_of(c, p.b);
            if (ba != ~0u && bb != ~0u) return ba + bb + p.lk;
        }
    return ~0u;
}
static void fetch_bits(svdw_ctx* c) {
    if (!c->bits_pending) return;
    hipck(hipEventSynchronize(c->ev_bits), "hipEventSynchronize");
    // the words are final once the event has fired: read them now (no copy is
    // queued on st per witness, the device-side consumers read the words directly)
    hipck(hipMemcpy(c->hbits, c->dbitw, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost), "D2H");
    c->bits_pending = false;
    for (int i = 0; i < 3; ++i) {
        c->qbits[i] = c->hbits[i];
        reg_bits(c, c->qmat[i], c->qbits[i]);
    }
}
static bool sharded(const svdw_ctx* c) { return c->shard_world > 1; }
static void host_mark(svdw_ctx* c, const char* what) {
    if (!c->host_trace || c->dry) return;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c->ht0).count();
    fprintf(stderr, "[svdw host] %9.1f us  %s\n", us, what);
}
// rows of a row-parallel stage (R rows) that this rank computes / owns
static void shard_rows(const svdw_ctx* c, uint64_t R, uint64_t* r0, uint64_t* r1) {
    *r0 = R * c->shard_rank / c->shard_world;
    *r1 = R * (c->shard_rank + 1) / c->shard_world;
}
static void own(svdw_ctx* c, uint32_t phase, bool lookup, uint64_t off, uint64_t n) {
    if (sharded(c) && n) c->owned.push_back({phase, lookup ? 1u : 0u, off, n});
}
static void clear_streams(svdw_ctx* c) {
    c->owned.clear();
    c->layout.clear();
    c->layout_chk.clear();
    c->ext_off = 0;
    c->consts.clear();
    c->phys.valid = false;
    c->bits_pending = false;
    for (auto& s : c->ph) { s.n = 0; s.nl = 0; }
    c->mbits.clear();
    c->prods.clear();
    c->dwords.clear();
    c->dbitw = nullptr;
    c->gamma_slots.clear();
}
// RAII: brackets one kernel launch with HIP events on the context stream.
struct ProfScope {
    svdw_ctx* c;
    long idx = -1;
    static hipEvent_t ev(svdw_ctx* c) {
        if (!c->pool.empty()) {
            hipEvent_t e = c->pool.back();
            c->pool.pop_back();
            return e;
        }
        // timing-only events: skip the system-scope fence (cache writeback and
        // invalidate) a default event performs, which would perturb what it measures
        hipEvent_t e;
        hipck(hipEventCreateWithFlags(&e, hipEventDisableSystemFence), "hipEventCreate");
        return e;
    }
    hipStream_t s = nullptr;
    bool ext = false;                       // stage launches: events recorded by their dispatch
    // stage: the scope holds stage launches only (launch_stage*), which record
    // the events themselves (set_launch_events): no event records between the
    // launches, which cost a few us of stream time each
    ProfScope(svdw_ctx* cc, hipStream_t ss, const std::string& name, double bytes, double ops,
              bool batch = false, bool stage = false)
        : c(cc), s(ss) {
        if (!batch) flush_batch(c, s);      // earlier batched stages go first
        if (!c->prof || c->dry) return;
        if (!c->prof_filter.empty() && name.compare(0, c->prof_filter.size(), c->prof_filter) != 0)
            return;
        // every launch is tagged with its stream (@cell, @s2, @s3 as created), so a
        // bench can report the busiest stream's stage rate beside the all-stream one
        const char* tag = s == c->stream_id[0] ? "@cell" : s == c->stream_id[1] ? "@s2"
                          : s == c->stream_id[2] ? "@s3" : "";
        svdw_ctx::Rec r{name + tag, bytes, ops, ev(c), ev(c)};
        ext = stage;
        if (ext)
            set_launch_events(r.e0, r.e1);
        else
            hipck(hipEventRecord(r.e0, s), "hipEventRecord");
        c->recs.push_back(r);
        idx = (long)c->recs.size() - 1;
    }
    ~ProfScope() {
        if (idx < 0) return;
        if (ext && launch_events_used()) return;
        if (ext) (void)hipEventRecord(c->recs[idx].e0, s);       // nothing launched: an empty interval
        (void)hipEventRecord(c->recs[idx].e1, s);
    }
};

static void ensure_buf(svdw_ctx* c, DBuf& b, size_t bytes) {
    if (c->dry || b.cap >= bytes) return;
    REQUIRE(!c->capturing, "internal: allocation during graph capture");
    ++c->epoch;
    sync(c);
    if (b.p) hipck(hipFree(b.p), "hipFree");
    b.p = nullptr;
    size_t cap = std::max(bytes, b.cap + b.cap / 2);
    if (hipMalloc(&b.p, cap) != hipSuccess) {
        b.cap = 0;
        fail(SVDW_ENOMEM, "device allocation failed (scratch)");
    }
    b.cap = cap;
}
// The bit-length words out[0 .. nred) folded inside the quantize launch
// (BitFold) when its first nred segments carry block maxima laid out back to
// back from qs.blockmax[0]; else k_bits_reduce over `seg`, a launch of its own.
static void bits_words(svdw_ctx* c, QuantSegs& qs, uint32_t nred, const BitSegs& seg, unsigned* out,
                       bool* folded) {
    *folded = false;
    if (c->dry || !qs.nseg || qs.nseg < nred || nred > 3) return;
    for (uint32_t s = 0; s < nred; ++s)
        if (qs.blockmax[s] != qs.blockmax[0] + qs.blk0[s] || qs.blk0[s] != seg.begin[s]) return;
    const uint32_t nblk = qs.blk0[nred];
    if (!c->qfold.p) {
        ensure_buf(c, c->qfold, 256);
        // the counters start at zero, before the quantize launch on st (a
        // null-stream hipMemset is not ordered against it)
        hipck(hipMemsetAsync(c->qfold.p, 0, c->qfold.cap, c->st), "hipMemsetAsync");
    }
    BitFold& f = qs.fold;
    f.bm = qs.blockmax[0];
    f.cnt = (unsigned*)c->qfold.p;
    f.wout = out;
    f.nblk = nblk;
    f.nred = nred;
    for (uint32_t s = 0; s <= nred; ++s) f.b[s] = qs.blk0[s];
    *folded = true;
}
// Write rate of the stage kernel's store pattern over `cells` cells at buf: a
// stage of 61 constant cells per element (no loads, no micro-ops), one warm and
// one timed launch on the cell stream.
static double stage_store_rate(svdw_ctx* c, Fr* buf, uint64_t cells) {
    StageArgs a;
    memset(&a, 0, sizeof a);
    const uint32_t C = 61;
    const uint64_t ne = std::min<uint64_t>(cells / C, 1ull << 26);
    if (ne < 1024) return 0.0;
    a.out_adv = buf;
    a.e_begin = 0;
    a.e_end = (uint32_t)ne;
    a.cols = 1;
    a.C = C;
    a.nv = 1;
    a.nk = 1;
    a.flags = c->stage_flags;
    a.cdiv_magic = (uint32_t)(((1ull << 32) + C - 1) / C);
    for (uint32_t k = 0; k < C; ++k) a.adv[k] = SlotOp{(uint8_t)KSRC, (uint8_t)(8 * (k % 8)), 0, 0};
    a.K[0] = fr_from_u64(0x9e3779b97f4a7c15ull);
    hipEvent_t e0, e1;
    hipck(hipEventCreate(&e0), "hipEventCreate");
    hipck(hipEventCreate(&e1), "hipEventCreate");
    hipck(launch_stage(a, c->st), "k_stage (placement probe)");
    hipck(hipEventRecord(e0, c->st), "hipEventRecord");
    hipck(launch_stage(a, c->st), "k_stage (placement probe)");
    hipck(hipEventRecord(e1, c->st), "hipEventRecord");
    hipck(hipEventSynchronize(e1), "hipEventSynchronize");
    float ms = 0;
    hipck(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms > 0 ? 32.0 * C * ne / (ms * 1e-3) : 0.0;
}
// A new cell stream of >= 256 MiB with "place_trials" k > 1 (default 6): k
// buffers are allocated side by side (so they lie in different places of HBM),
// the stage store pattern is timed on each, and the fastest is kept. The same
// witness runs 1.73-2.03 ms per step depending on where its streams lie, and a
// fresh process's first placement is a slow one (fresh
// bench.py processes at 1024^2, one box: 2.010-2.014 ms without trials,
// 1.848-1.861 with 3, 1.721-1.767 with 6, tools/r6/r6pt3.sh).
// The trials need k times the stream in free memory (fewer when it is short:
// none at 4096^2) and a few ms once per allocation.
static Fr* place_cells(svdw_ctx* c, uint64_t cells) {
    const uint64_t bytes = cells * sizeof(Fr);
    int k = c->place_trials;
    if (k > 1 && bytes >= (256ull << 20)) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
        while (k > 1 && (double)k * bytes > 0.5 * (double)fr) --k;
    }
    Fr* best = nullptr;
    if (k <= 1 || bytes < (256ull << 20)) {
        if (hipMalloc((void**)&best, bytes) != hipSuccess) return nullptr;
        return best;
    }
    sync(c);
    std::vector<Fr*> cand;
    double br = -1.0;
    for (int i = 0; i < k; ++i) {
        Fr* p = nullptr;
        if (hipMalloc((void**)&p, bytes) != hipSuccess) break;
        cand.push_back(p);
        const double r = stage_store_rate(c, p, cells);
        if (c->host_trace) fprintf(stderr, "place_cells: %.2f GB candidate %d at %p: %.3f TB/s\n", bytes / 1e9, i,
                                   (void*)p, r / 1e12);
        if (r > br) {
            br = r;
            best = p;
        }
    }
    for (Fr* p : cand)
        if (p != best) hipck(hipFree(p), "hipFree");
    return best;
}
static void grow(svdw_ctx* c, Fr*& ptr, uint64_t used, uint64_t& cap, uint64_t need) {
    if (c->dry || need <= cap) return;
    REQUIRE(!c->capturing, "internal: allocation during graph capture");
    ++c->epoch;
    uint64_t ncap = std::max(need, cap + cap / 2);
    Fr* np = ptr ? nullptr : place_cells(c, ncap);
    if (!np && hipMalloc((void**)&np, ncap * sizeof(Fr)) != hipSuccess)
        fail(SVDW_ENOMEM, "device allocation failed (cell stream of " + std::to_string(ncap) + " cells)");
    if (ptr) {
        hipck(hipMemcpyAsync(np, ptr, used * sizeof(Fr), hipMemcpyDeviceToDevice, c->st), "copy");
        sync(c);
        hipck(hipFree(ptr), "hipFree");
    }
    ptr = np;
    cap = ncap;
}
// Append n advice and nl lookup cells to a phase; returns their offsets.
// Every cell region of a witness is appended here, in the reference's order;
// the layout table (svdw_layout) records what each region is: the gadget /
// function that appends it and its rows (row-parallel regions hold `rows`
// equal runs of cells).
static void append(svdw_ctx* c, uint32_t phase, uint64_t n, uint64_t nl, uint64_t* off,
                   uint64_t* loff, const char* tag, uint64_t rows = 1) {
    REQUIRE(phase < 2, "phase must be 0 or 1");
    settle(c);
    Stream& s = c->ph[phase];
    c->phys.valid = false;
    grow(c, s.adv, s.n, s.cap, s.n + n);
    grow(c, s.lk, s.nl, s.lcap, s.nl + nl);
    *off = s.n;
    if (loff) *loff = s.nl;
    svdw_region r;
    memset(&r, 0, sizeof r);
    r.phase = phase;
    r.off = s.n;
    r.n = n;
    r.loff = s.nl;
    r.nl = nl;
    r.rows = rows ? rows : 1;
    snprintf(r.tag, sizeof r.tag, "%s", tag);
    c->layout.push_back(r);
    c->layout_chk.emplace_back();
    s.n += n;
    s.nl += nl;
}
static Fr* cellp(svdw_ctx* c, uint32_t phase, uint64_t off) { return c->ph[phase].adv + off; }

// Device pointers into the cell streams (views) are taken while a gadget is
// being built; a stream reallocation in between would leave them pointing at
// the freed buffer. Every ABI entry point that appends after taking a view
// therefore sizes the streams first from a dry replay of itself (layouts are
// data independent), so nothing reallocates inside the call.
template <class F>
static void pregrow(svdw_ctx* c, F&& fn) {
    if (c->dry) return;
    svdw_ctx plan;
    plan.P = c->P;
    plan.LB = c->LB;
    for (int p = 0; p < 2; ++p) { plan.ph[p].n = c->ph[p].n; plan.ph[p].nl = c->ph[p].nl; }
    fn(&plan);
    for (int p = 0; p < 2; ++p) {
        grow(c, c->ph[p].adv, c->ph[p].n, c->ph[p].cap, plan.ph[p].n);
        grow(c, c->ph[p].lk, c->ph[p].nl, c->ph[p].lcap, plan.ph[p].nl);
    }
}

// --------------------------------------------------------------- views
// A dry context has no streams: its views carry a placeholder pointer that
// view_source decodes to (phase, offset) (never dereferenced: nothing launches).
static constexpr uintptr_t kDryBase = (uintptr_t)1 << 44;
static const Fr* dry_ptr(uint32_t phase, uint64_t off) {
    return reinterpret_cast<const Fr*>(kDryBase * (phase + 1) + off * sizeof(Fr));
}
static DView view_of(svdw_ctx* c, const svdw_mat& m) {
    DView v;
    memset(&v, 0, sizeof v);
    v.ptr = c->dry ? dry_ptr(m.phase, m.off) : cellp(c, m.phase, m.off);
    v.rs = m.rs;
    v.cs = m.cs;
    v.rows = m.rows;
    v.cols = m.cols;
    v.mode = VIEW_STRIDED;
    return v;
}
// A launch's view of loaded cells whose f64 source is registered for this call
// (f64reg): the same elements read from the f64 input and quantized in the
// kernel (VIEW_F64), so the launch does not wait for k_quantize_multi. The
// checker's copies of the views (note_gates) stay cell views.
static DView f64_view(const svdw_ctx* c, const DView& v) {
    if (!c->f64_views || c->f64reg.empty() || v.mode != VIEW_STRIDED || !v.ptr || !v.rows || !v.cols) return v;
    for (const auto& r : c->f64reg) {
        const Fr* base = c->ph[r.phase].adv + r.off;
        const int64_t o = v.ptr - base;
        const int64_t er = (int64_t)(v.rows - 1) * v.rs, ec = (int64_t)(v.cols - 1) * v.cs;
        const int64_t lo = o + std::min<int64_t>(er, 0) + std::min<int64_t>(ec, 0),
                      hi = o + std::max<int64_t>(er, 0) + std::max<int64_t>(ec, 0);
        if (lo < 0 || hi >= (int64_t)r.n) continue;
        DView f = v;
        f.ptr = reinterpret_cast<const Fr*>(r.x + o);
        f.mode = VIEW_F64;
        f._r0 = (uint8_t)c->P;
        return f;
    }
    return v;
}
static svdw_mat mat_of_vec(const svdw_vec& v) {   // len x 1 column
    return svdw_mat{v.phase, v.len, 1, v.off, v.stride, 0};
}
static void check_mat(const svdw_ctx* c, const svdw_mat& m) {
    REQUIRE(m.phase < 2, "matrix phase must be 0 or 1");
    REQUIRE(m.rows >= 1 && m.cols >= 1, "empty matrix");
    // every referenced cell must already exist
    int64_t lo = (int64_t)m.off, hi = (int64_t)m.off;
    int64_t er = (int64_t)(m.rows - 1) * m.rs, ec = (int64_t)(m.cols - 1) * m.cs;
    lo += std::min<int64_t>(er, 0) + std::min<int64_t>(ec, 0);
    hi += std::max<int64_t>(er, 0) + std::max<int64_t>(ec, 0);
    REQUIRE(lo >= 0 && (uint64_t)hi < c->ph[m.phase].n, "matrix view outside its phase stream");
}
static void check_vec(const svdw_ctx* c, const svdw_vec& v) { check_mat(c, mat_of_vec(v)); }

// ------------------------------------------------------- stage launches
// Appends the stage's cells for `nelem` elements; returns the advice offset.
// Launch a stage whose cells were appended at (off, loff) earlier.
static void stage_launch(svdw_ctx* c, uint32_t phase, PB& pb, uint32_t nelem, uint32_t cols,
                         uint64_t off, uint64_t loff, const char* tag) {
    StageArgs a = pb.a;
    uint32_t eb = 0, ee = nelem;
    if (sharded(c) && nelem) {
        const uint64_t cw = cols ? cols : 1, R = nelem / cw;
        uint64_t r0, r1;
        shard_rows(c, R, &r0, &r1);
        if (R > 1) {                                      // single cells: every rank
            eb = (uint32_t)(r0 * cw);
            ee = (uint32_t)(r1 * cw);
        }
    }
    if (g_stage_log) {
        uint32_t nmul = 0;
        for (uint32_t i = 0; i < a.nmo; ++i) nmul += a.mo[i].op == MO_MUL;
        const int sid = c->st == c->st_cell ? 1 : c->st == c->st2 ? 2 : c->st == c->st3 ? 3 : 0;
        fprintf(stderr, "stage %-28s elems %8u C %3u L %3u nv %2u nmo %2u muls %u nk %u  s%d\n", tag, ee - eb,
                a.C, a.L, a.nv, a.nmo, nmul, a.nk, sid);
        if (getenv("SVDW_STAGE_LOG")[0] == '2') {        // the slot ops too: (src lo nbits) per cell
            fprintf(stderr, "  slots");
            for (uint32_t k = 0; k < a.C + a.L; ++k) {
                const SlotOp& o = k < a.C ? a.adv[k] : a.lk[k - a.C];
                fprintf(stderr, " %u:%u:%u", o.src, o.lo, o.nbits);
            }
            fprintf(stderr, "\n");
        }
    }
    if (c->dry || ee <= eb) return;
    a.out_adv = cellp(c, phase, off);
    a.out_lk = a.L ? c->ph[phase].lk + loff : nullptr;
    for (int k = 0; k < kMaxViews; ++k) a.view[k] = f64_view(c, a.view[k]);
    a.e_begin = eb;
    a.e_end = ee;
    a.cols = cols ? cols : 1;
    a.flags = c->stage_flags;
    // small blocks overlap better with concurrent work, but a stage with field
    // multiplications / inversions keeps one element per thread of a full block
    bool heavy = false;
    for (uint32_t i = 0; i < a.nmo; ++i)
        heavy |= a.mo[i].op == MO_MUL || a.mo[i].op == MO_ISZERO || a.mo[i].op == MO_POWK;
    a.E = heavy ? kStageElems : c->stage_elems;
    // keep the block's LDS (element values) within 64 KiB: fewer elements per
    // block for stages with many values (signed_div_scale)
    while (a.E > 64 && stage_lds_bytes(a.nv ? a.nv : 1, a.E, a.C + a.L) > 65536) a.E -= 64;
    // 32-bit magics for fastdiv (divisor 1 is handled in the kernel)
    auto magic = [](uint64_t d) -> uint32_t { return d > 1 ? (uint32_t)(((1ull << 32) + d - 1) / d) : 0; };
    a.cdiv_magic = magic(a.C);
    a.ldiv_magic = magic(a.L);
    uint32_t loads = 0;
    for (uint32_t i = 0; i < a.nmo; ++i) loads += a.mo[i].op == MO_LOAD;
    const double bytes = 32.0 * (ee - eb) * ((double)a.C + a.L + loads);
    for (auto& b : c->batches) {
        if (b.st != c->st || !stage_multi_fits(a)) continue;
        // does this stage read cells that pending stage q writes?
        auto reads = [&](const svdw_ctx::Pending& q) {
            const char* w0 = reinterpret_cast<const char*>(q.a.out_adv);
            const char* w1 = w0 + sizeof(Fr) * (uint64_t)q.a.e_end * q.a.C;
            for (int k = 0; k < kMaxViews; ++k) {
                const DView& v = a.view[k];
                if (!v.ptr || v.mode == VIEW_DIAGK) continue;
                // the view's cells lie within [lo, hi) of ptr (signed strides, in cells)
                const int64_t dr = (int64_t)(v.rows ? v.rows - 1 : 0) * v.rs,
                              dc = (int64_t)(v.cols ? v.cols - 1 : 0) * v.cs;
                const int64_t lo = std::min<int64_t>(dr, 0) + std::min<int64_t>(dc, 0),
                              hi = std::max<int64_t>(dr, 0) + std::max<int64_t>(dc, 0) + 1;
                const char* p = reinterpret_cast<const char*>(v.ptr);
                if (p + lo * (int64_t)sizeof(Fr) < w1 && p + hi * (int64_t)sizeof(Fr) > w0) return true;
            }
            return false;
        };
        size_t g = 0;                                     // after the last group it depends on
        for (size_t k = 0; k < b.groups.size(); ++k)
            for (const auto& q : b.groups[k])
                if (reads(q)) g = k + 1;
        if (c->stage_front && g == 0) {                   // a launch of its own, ahead of the batch
            b.groups.insert(b.groups.begin(), std::vector<svdw_ctx::Pending>{});
            b.groups[0].push_back({a, std::string("k_stage:") + tag, bytes});
            b.last = 0;
            return;
        }
        if (g == b.groups.size()) b.groups.emplace_back();
        b.groups[g].push_back({a, std::string("k_stage:") + tag, bytes});
        b.last = g;
        return;
    }
    {
        ProfScope ps(c, c->st, std::string("k_stage:") + tag, bytes, 0, false, true);
        const StageArgs* one = &a;
        hipck(launch_stage_multi(&one, 1, c->st), "k_stage");
    }
}
// Issue a stream's pending batched stages (k_stage_multi; one program: k_stage).
// waiter: after the group holding the latest stage, `waiter` waits for s there
// (it needs that stage and what came before on s, not the later groups: those
// hold stages queued earlier that depend on other pending ones).
// then_wait: s waits for this event before the groups after that point.
static void flush_batch(svdw_ctx* c, hipStream_t s, hipStream_t waiter, hipEvent_t then_wait) {
    for (auto& b : c->batches) {
        if (b.st != s || b.groups.empty()) continue;
        std::vector<std::vector<svdw_ctx::Pending>> groups;
        groups.swap(b.groups);               // (cleared before launching: no re-entry)
        const size_t upto = b.last;
        for (size_t gi = 0; gi < groups.size(); ++gi) {
            const auto& grp = groups[gi];
            if (gi == upto + 1 && waiter) {
                stream_dep(c, s, waiter);
                waiter = nullptr;
                if (then_wait) dep_wait(c, s, then_wait);
            }
            if (grp.empty()) continue;
            std::vector<const StageArgs*> ps;
            double bytes = 0;
            for (const auto& q : grp) {
                ps.push_back(&q.a);
                bytes += q.bytes;
            }
            const std::string name = grp.size() == 1 ? grp[0].name : "k_stage:multi";
            if (g_batch_log) {
                fprintf(stderr, "batch stream %p group %zu/%zu (last %zu):", (void*)s, gi, groups.size(), upto);
                for (const auto& q : grp) fprintf(stderr, " %s", q.name.c_str());
                fprintf(stderr, "\n");
            }
            ProfScope pr(c, s, name, bytes, 0, true, true);
            hipck(launch_stage_multi(ps.data(), (int)ps.size(), s), "k_stage_multi");
        }
    }
    if (waiter) stream_dep(c, s, waiter);
}
// RAII: stage launches on the current stream between construction and end()
// are batched (k_stage_multi); nested scopes on the same stream join the outer
// one. Without end() (an exception) the pending stages are dropped.
struct BatchScope {
    svdw_ctx* c;
    hipStream_t st = nullptr;
    bool mine = false;
    explicit BatchScope(svdw_ctx* cc, hipStream_t on = nullptr) : c(cc) {
        if (c->dry || !c->stage_batch) return;
        if (!on) on = c->st;
        for (auto& b : c->batches)
            if (b.st == on) return;
        st = on;
        c->batches.push_back({st, {}});
        mine = true;
    }
    void end() {
        if (!mine) return;
        flush_batch(c, st);
        close();
    }
    void close() {
        for (size_t i = 0; i < c->batches.size(); ++i)
            if (c->batches[i].st == st) { c->batches.erase(c->batches.begin() + i); break; }
        mine = false;
    }
    ~BatchScope() { if (mine) close(); }
};
// shard ownership of a stage's cells: this rank's rows (single cells: the last rank)
static void stage_own(svdw_ctx* c, uint32_t phase, const PB& pb, uint32_t nelem, uint32_t cols,
                      uint64_t off, uint64_t loff) {
    if (!sharded(c) || !nelem) return;
    const uint64_t cw = cols ? cols : 1, R = nelem / cw;
    uint64_t r0, r1;
    shard_rows(c, R, &r0, &r1);
    own(c, phase, false, off + r0 * cw * pb.a.C, (r1 - r0) * cw * pb.a.C);
    own(c, phase, true, loff + r0 * cw * pb.a.L, (r1 - r0) * cw * pb.a.L);
}
static uint64_t f64_key(double x) {
    uint64_t k;
    memcpy(&k, &x, sizeof k);
    return k;
}
static void note_const(svdw_ctx* c, const Fr& v) {
    std::array<uint32_t, 8> w;
    for (int i = 0; i < 8; ++i) w[i] = v.w[i];
    c->consts.insert(w);
}
// the last appended region is `nelem` copies of pb's program: record its gates
// (views: the source cells as (phase, offset), strided views into the cell
// streams only -- the streams may move before the check)
// (phase, offset) of a view's cell 0 in the cell streams (dry placeholders too)
static bool view_source(const svdw_ctx* c, const Fr* ptr, uint32_t* phase, uint64_t* off) {
    if (!ptr) return false;
    if (c->dry) {
        const uintptr_t x = reinterpret_cast<uintptr_t>(ptr);
        if (x < kDryBase || x >= 3 * kDryBase) return false;
        *phase = (uint32_t)(x / kDryBase - 1);
        *off = (x % kDryBase) / sizeof(Fr);
        return true;
    }
    for (uint32_t p = 0; p < 2; ++p) {
        const Fr* base = c->ph[p].adv;
        if (base && ptr >= base && ptr < base + c->ph[p].n) {
            *phase = p;
            *off = (uint64_t)(ptr - base);
            return true;
        }
    }
    return false;
}
// equality source of a matrix / a vector chain (RegionChecks::EqSrc)
static RegionChecks::EqSrc eqsrc_mat(const svdw_mat& m) {
    RegionChecks::EqSrc e;
    e.kind = EQS_MAT;
    e.phase = m.phase; e.off = m.off; e.rs = m.rs; e.cs = m.cs; e.rows = m.rows; e.cols = m.cols;
    return e;
}
static RegionChecks::EqSrc eqsrc_chain(uint32_t first_phase, uint64_t first, uint32_t phase,
                                       uint64_t base, int64_t stride) {
    RegionChecks::EqSrc e;
    e.kind = EQS_CHAIN;
    e.first_phase = first_phase; e.first = first; e.phase = phase; e.off = base; e.rs = stride;
    return e;
}
static RegionChecks::EqSrc eqsrc_vec(const svdw_vec& v) {   // cells v.off + t v.stride
    return eqsrc_chain(v.phase, v.off, v.phase, v.off + v.stride, v.stride);
}
static void note_gates(svdw_ctx* c, const PB& pb, uint32_t cols = 1, size_t reg = ~size_t(0)) {
    RegionChecks& r = reg == ~size_t(0) ? c->layout_chk.back() : c->layout_chk.at(reg);
    r.eq = pb.eq;
    r.eqk.assign(pb.a.K, pb.a.K + pb.a.nk);
    for (int k = 0; k < kMaxViews; ++k) {             // the loaded values' source cells
        const DView& v = pb.a.view[k];
        uint32_t ph;
        uint64_t off;
        if (v.mode == VIEW_STRIDED && view_source(c, v.ptr, &ph, &off))
            r.esrc[k] = eqsrc_mat(svdw_mat{ph, v.rows, v.cols, off, v.rs, v.cs});
    }
    if (pb.kconst)
        for (uint32_t q = 0; q < pb.a.C; ++q)
            if (pb.a.adv[q].src >= KSRC && pb.a.adv[q].src - KSRC != pb.kext)
                note_const(c, pb.a.K[pb.a.adv[q].src - KSRC]);
    r.words = pb.chk;
    r.unit = pb.a.C;
    r.cols = cols ? cols : 1;
    for (int k = 0; k < kMaxViews; ++k) {
        const DView& v = pb.a.view[k];
        RegionChecks::Src& s = r.src[k];
        s.phase = -1;
        if (!v.ptr || v.mode != VIEW_STRIDED) continue;
        for (int p = 0; p < 2; ++p) {
            const Fr* base = c->ph[p].adv;
            if (base && v.ptr >= base && v.ptr < base + c->ph[p].n) {
                s = RegionChecks::Src{p, (uint64_t)(v.ptr - base), v.rs, v.cs, v.rows, v.cols};
                break;
            }
        }
    }
    // a view word whose source is not in the streams (host-known constants,
    // the gamma powers buffer) is dropped
    std::vector<uint32_t> keep;
    for (uint32_t w : r.words)
        if (chk_kind(w) != CHK_VIEW || r.src[chk_a(w)].phase >= 0) keep.push_back(w);
    r.words.swap(keep);
}
static uint64_t run_stage(svdw_ctx* c, uint32_t phase, PB& pb, uint32_t nelem, uint32_t cols,
                          const char* tag, uint64_t* loff_out = nullptr) {
    uint64_t off = 0, loff = 0;
    append(c, phase, (uint64_t)nelem * pb.a.C, (uint64_t)nelem * pb.a.L, &off, &loff, tag,
           cols ? nelem / cols : nelem);
    note_gates(c, pb, cols);
    stage_own(c, phase, pb, nelem, cols, off, loff);
    if (loff_out) *loff_out = loff;
    stage_launch(c, phase, pb, nelem, cols, off, loff, tag);
    return off;
}
static svdw_vec put_cell(svdw_ctx* c, uint32_t phase, const Fr& v, bool constant = false) {
    PB pb(c->LB);                                          // load_witness / load_constant
    pb.kconst = constant;
    pb.cell(pb.K(v));
    // Inside svd_witness (products queued ahead), a one-cell launch on the cell
    // stream would wait for a free CU behind the scans on st2 (15-35 us on the
    // critical path); it depends on nothing, so it goes on st2 itself (never
    // back onto the cell stream: with st and st2 exchanged, as for a pipelined
    // witness's diff and ids, it stays where it is).
    const bool aside = c->prelaunched && !c->dry && c->st2 != c->st_cell;
    if (aside) std::swap(c->st, c->st2);
    uint64_t off = 0;
    try {
        off = run_stage(c, phase, pb, 1, 1, "load_cell");
    } catch (...) {
        if (aside) std::swap(c->st, c->st2);
        throw;
    }
    if (aside) std::swap(c->st, c->st2);
    return svdw_vec{phase, 1, off, 1};
}

// ----------------------------------------------------- reference functions
// qs: collect the quantization into one k_quantize_multi launch (device inputs
// only) instead of launching it here.
// own_rows_only (row-sharded svd_witness, m): quantize only this rank's rows,
// the only rows of the matrix any of its stages read.
// own_rows_cols (row-sharded svd_witness, square u and v, b.g from the f64
// inputs): store only this rank's rows and its column block, the cells its
// stages (bounds, u.d, the a and b = X^T scans) read; the bit-length maxima
// still cover the whole matrix (the GEMM's B operand).
static svdw_mat zkmatrix_new(svdw_ctx* c, uint32_t phase, const double* data, uint32_t rows,
                             uint32_t cols, bool on_device, unsigned* blockmax = nullptr,
                             QuantSegs* qs = nullptr, bool own_rows_only = false,
                             bool own_rows_cols = false) {
    REQUIRE(rows >= 1 && cols >= 1, "ZkMatrix::new: empty matrix");
    REQUIRE(data || c->dry, "null data");
    uint64_t n = (uint64_t)rows * cols, off;
    append(c, phase, n, 0, &off, nullptr, "load", rows);
    uint64_t q0 = 0;                                      // first quantized value
    if (own_rows_only && sharded(c) && on_device && qs) {
        uint64_t r0, r1;
        shard_rows(c, rows, &r0, &r1);
        q0 = r0 * cols;
        n = (r1 - r0) * cols;
    }
    if (!c->dry && n) {
        const double* src = data + q0;
        if (!on_device) {
            ensure_buf(c, c->f64in, n * sizeof(double));
            hipck(hipMemcpyAsync(c->f64in.p, data, n * sizeof(double), hipMemcpyHostToDevice, c->st),
                  "H2D");
            src = (const double*)c->f64in.p;
        }
        if (qs && on_device && qs->nseg < (uint32_t)kMaxQuantSegs) {
            const uint32_t k = qs->nseg++;
            qs->in[k] = src;
            qs->out[k] = cellp(c, phase, off + q0);
            qs->blockmax[k] = blockmax;
            qs->n[k] = n;
            qs->keep[k] = QuantKeep{0, 0, 0, 0, 0};
            if (own_rows_cols && sharded(c) && rows == cols) {
                uint64_t r0, r1;
                shard_rows(c, rows, &r0, &r1);
                qs->keep[k] = QuantKeep{cols, (uint32_t)r0, (uint32_t)r1, (uint32_t)r0, (uint32_t)r1};
            }
            const uint32_t pb = qs->per_block ? qs->per_block : kQuantPerBlock;
            qs->blk0[k + 1] = qs->blk0[k] + (uint32_t)((n + pb - 1) / pb);
        } else {
            ProfScope ps(c, c->st, "k_quantize", 40.0 * n, 0);
            hipck(launch_quantize(src, n, cellp(c, phase, off), (int)c->P, blockmax, c->st),
                  "k_quantize");
        }
    }
    if (sharded(c)) {            // every rank quantizes all of it (operands of the products)
        uint64_t r0, r1;
        shard_rows(c, rows, &r0, &r1);
        own(c, phase, false, off + r0 * cols, (r1 - r0) * cols);
    }
    return svdw_mat{phase, rows, cols, off, (int64_t)cols, 1};
}

// ZkVector::entries_less_than
static void entries_less_than(svdw_ctx* c, const svdw_vec& d, uint32_t bits) {
    PB pb(c->LB);
    pb.a.view[0] = view_of(c, mat_of_vec(d));
    pb.range_check(pb.load(0), bits);
    run_stage(c, d.phase, pb, d.len, 1, "entries_less_than");
}
// ZkVector::entries_in_desc_order: all qsub(d_i, d_{i+1}) first, then range checks.
static void entries_in_desc_order(svdw_ctx* c, const svdw_vec& d, uint32_t bits) {
    REQUIRE(d.len >= 1, "entries_in_desc_order: empty vector");   // reference: 0..len-1 underflow
    if (d.len == 1) return;
    uint32_t n = d.len - 1;
    PB sb(c->LB);
    svdw_vec d1 = d;
    d1.off = d.off + d.stride;
    d1.len = n;
    svdw_vec d0 = d;
    d0.len = n;
    sb.a.view[0] = view_of(c, mat_of_vec(d0));
    sb.a.view[1] = view_of(c, mat_of_vec(d1));
    uint8_t x = sb.load(0), y = sb.load(1);
    sb.g_sub(x, y);
    uint64_t soff = run_stage(c, d.phase, sb, n, 1, "desc_order_sub");
    PB rb(c->LB);
    rb.a.view[0] = view_of(c, mat_of_vec(svdw_vec{d.phase, n, soff, 4}));
    rb.range_check(rb.load(0), bits);
    run_stage(c, d.phase, rb, n, 1, "desc_order_range");
}
static void check_mat_entries_bounded(svdw_ctx* c, const svdw_mat& a, const BigU& bnd) {
    PB pb(c->LB);
    pb.a.view[0] = view_of(c, a);
    pb.check_abs_less_than(pb.load(0), bnd);
    run_stage(c, a.phase, pb, a.rows * a.cols, a.cols, "check_mat_entries_bounded");
}
// check_mat_diff on arbitrary views (a may be zero-padded, b may be diagonal).
// a cell of the streams, for equality sources (phase -1: none)
struct EqCell {
    int phase = -1;
    uint64_t off = 0;
};
static void check_mat_diff_views(svdw_ctx* c, uint32_t phase, const DView& a, const DView& b,
                                 uint32_t rows, uint32_t cols, const BigU& tol,
                                 const Fr* diag_val = nullptr, EqCell pad_a = {},
                                 EqCell pad_b = {}, EqCell diag_b = {}) {
    PB pb(c->LB);
    pb.a.view[0] = a;
    pb.a.view[1] = b;
    uint8_t x = pb.load(0), y = pb.load(1);
    uint8_t dlt = pb.g_sub(x, y);
    pb.check_abs_less_than(dlt, tol);
    // pad / diag constants referenced by the views
    pb.a.view[0].pad_k = pb.kidx(fr_zero());
    pb.a.view[1].pad_k = pb.kidx(fr_zero());
    if (diag_val) pb.a.view[1].diag_k = pb.kidx(*diag_val);
    run_stage(c, phase, pb, rows * cols, cols, "check_mat_diff");
    // equality sources of the padded / diagonal entries: the zero padding
    // constant (check_svd_phase0), check_mat_id's zero and scalar_id cells
    RegionChecks& r = c->layout_chk.back();
    if (pad_a.phase >= 0) { r.esrc[0].pad_phase = pad_a.phase; r.esrc[0].pad_off = pad_a.off; }
    if (b.mode != VIEW_STRIDED) {
        r.esrc[1] = RegionChecks::EqSrc();
        r.esrc[1].kind = EQS_MAT;                         // no strided part: pad or diagonal
    }
    if (pad_b.phase >= 0) { r.esrc[1].pad_phase = pad_b.phase; r.esrc[1].pad_off = pad_b.off; }
    if (diag_b.phase >= 0) { r.esrc[1].diag_phase = diag_b.phase; r.esrc[1].diag_off = diag_b.off; }
}
// sid_val: the scalar's value when the host knows it (svd_witness's q^2): the
// stage then takes it as a constant and does not read sid's cell, which may
// still be in flight on another stream.
static void check_mat_id(svdw_ctx* c, const svdw_mat& a, const svdw_vec& sid, const BigU& tol,
                         const Fr* sid_val = nullptr) {
    const svdw_vec zero = put_cell(c, a.phase, fr_zero(), true);   // ctx.load_constant(F::ZERO)
    DView b;
    memset(&b, 0, sizeof b);
    b.mode = sid_val ? VIEW_DIAGK : VIEW_DIAG;
    b.ptr = c->dry || sid_val ? nullptr : cellp(c, sid.phase, sid.off);
    b.rows = a.rows;
    b.cols = a.cols;
    check_mat_diff_views(c, a.phase, view_of(c, a), b, a.rows, a.cols, tol, sid_val, EqCell{},
                         EqCell{(int)zero.phase, zero.off}, EqCell{(int)sid.phase, sid.off});
}
static svdw_mat mat_times_diag_mat(svdw_ctx* c, const svdw_mat& a, const svdw_vec& v) {
    REQUIRE(v.len <= a.cols, "mat_times_diag_mat: v longer than a's rows");
    PB pb(c->LB);
    pb.a.view[0] = view_of(c, a);
    pb.a.view[1] = view_of(c, svdw_mat{v.phase, a.rows, v.len, v.off, 0, v.stride});
    uint8_t x = pb.load(0), y = pb.load(1);
    pb.g_mul(x, y);
    uint64_t off = run_stage(c, a.phase, pb, a.rows * v.len, v.len, "mat_times_diag_mat");
    return svdw_mat{a.phase, a.rows, v.len, off + 3, (int64_t)4 * v.len, 4};
}

// signed_div_scale constants (svdw_div_scale; zero fields -> 3P, shift + 1)
struct DivScale {
    uint32_t s, nb;
};
static DivScale div_scale_of(const svdw_ctx* c, const svdw_div_scale* cfg) {
    DivScale d;
    d.s = cfg && cfg->shift_bits ? cfg->shift_bits : 3 * c->P;
    // the reference's cell counts (svdw.h); a shift alone >= 4P + 1 widens the div_mod
    d.nb = cfg && cfg->num_bits ? cfg->num_bits : std::max(4 * c->P + 1, d.s + 1);
    REQUIRE(d.s >= c->P && d.s < 254 && d.nb > d.s && d.nb <= 253 && d.nb - c->P <= 200,
            "signed_div_scale: need P <= shift_bits < num_bits <= 253, num_bits - P <= 200");
    return d;
}
// ZkMatrix::rescale_matrix (src/matrix/mod.rs:354-375): signed_div_scale of
// every entry of c_s, row-major; the result matrix is the final sub's cell 0.
static svdw_mat rescale_matrix(svdw_ctx* c, const svdw_mat& cs, DivScale d) {
    PB pb(c->LB);
    pb.a.view[0] = view_of(c, cs);
    pb.signed_div_scale(pb.load(0), c->P, d.s, d.nb);
    const uint32_t C = pb.a.C;
    uint64_t off = run_stage(c, cs.phase, pb, cs.rows * cs.cols, cs.cols, "rescale_matrix");
    return svdw_mat{cs.phase, cs.rows, cs.cols, off + C - 4, (int64_t)C * cs.cols, C};
}
static svdw_vec field_mat_vec_mul(svdw_ctx* c, uint32_t phase, const svdw_mat& a, const svdw_vec& v);
// ZkVector::inner_product (src/matrix/mod.rs:79-106): gate.inner_product(x, self)
// (the field_mat_vec_mul row layout with x as the row), then signed_div_scale.
static svdw_vec zkvector_inner_product(svdw_ctx* c, uint32_t phase, const svdw_vec& self,
                                       const svdw_vec& x, DivScale d) {
    REQUIRE(self.len == x.len && x.len >= 1, "ZkVector::inner_product: length mismatch");
    svdw_vec s = field_mat_vec_mul(c, phase, svdw_mat{x.phase, 1, x.len, x.off, 0, x.stride}, self);
    PB pb(c->LB);
    pb.a.view[0] = view_of(c, mat_of_vec(s));
    pb.signed_div_scale(pb.load(0), c->P, d.s, d.nb);
    const uint32_t C = pb.a.C;
    uint64_t off = run_stage(c, phase, pb, 1, 1, "signed_div_scale");
    return svdw_vec{phase, 1, off + C - 4, 1};
}
// ZkVector::_norm_square (src/matrix/mod.rs:112-119): self.inner_product(self).
static svdw_vec zkvector_norm_square(svdw_ctx* c, uint32_t phase, const svdw_vec& self, DivScale d) {
    return zkvector_inner_product(c, phase, self, self, d);
}
// ZkVector::_dist_square (src/matrix/mod.rs:135-148): diff_i = qsub(self_i, x_i)
// (FixedPointChip041::qsub = gate.sub [ext, inferred as for entries_in_desc_order]:
// cells [a - b, b, 1, a]), then diff._norm_square.
// qsqrt of a one-element vector (ZkVector::norm / dist's final step)
static svdw_vec qsqrt_vec(svdw_ctx* c, uint32_t phase, const svdw_vec& a, uint32_t nbits) {
    const uint32_t nb = nbits ? nbits : 2 * c->P;
    REQUIRE(nb >= 1 && nb + c->P <= 250, "qsqrt: need 1 <= sqrt_bits, sqrt_bits + P <= 250");
    PB pb(c->LB);
    pb.a.view[0] = view_of(c, mat_of_vec(a));
    pb.qsqrt(pb.load(0), c->P, nb);
    uint64_t off = run_stage(c, phase, pb, 1, 1, "qsqrt");
    return svdw_vec{phase, 1, off, 1};                   // y: the gadget's first cell
}
static svdw_vec zkvector_dist_square(svdw_ctx* c, uint32_t phase, const svdw_vec& self,
                                     const svdw_vec& x, DivScale d) {
    REQUIRE(self.len == x.len && x.len >= 1, "ZkVector::_dist_square: length mismatch");
    PB sb(c->LB);
    sb.a.view[0] = view_of(c, mat_of_vec(self));
    sb.a.view[1] = view_of(c, mat_of_vec(x));
    uint8_t a = sb.load(0), b = sb.load(1);
    sb.g_sub(a, b);
    const uint64_t soff = run_stage(c, phase, sb, self.len, 1, "qsub");
    const svdw_vec diff{phase, self.len, soff, 4};
    return zkvector_norm_square(c, phase, diff, d);
}
// ZkVector::mul (src/matrix/mod.rs:169-182): inner_product with each row of a
// (one row scan + one stage per row; config-1 plumbing, not the hot path).
static svdw_vec zkvector_mul(svdw_ctx* c, uint32_t phase, const svdw_vec& self, const svdw_mat& a,
                             DivScale d) {
    REQUIRE(a.cols == self.len, "ZkVector::mul: a.num_col != self.size()");
    svdw_vec first{}, prev{};
    for (uint32_t i = 0; i < a.rows; ++i) {
        svdw_vec row{a.phase, a.cols, a.off + (uint64_t)((int64_t)i * a.rs), a.cs};
        svdw_vec y = zkvector_inner_product(c, phase, self, row, d);
        if (i == 0) first = y;
        if (i == 1) first.stride = (int64_t)(y.off - prev.off);
        prev = y;
    }
    first.len = a.rows;
    return first;
}

// Balanced base-256 digits needed for |x| < 2^bits.
static int digits_for_bits(uint32_t bits) {
    for (int D = 1; D <= 16; ++D) {
        // max representable magnitude 127 * (256^D - 1) / 255 >= 2^bits - 1 ?
        long double maxv = 127.0L * (powl(256.0L, D) - 1.0L) / 255.0L;
        if (maxv >= powl(2.0L, bits) - 1.0L) return D;
    }
    return 99;
}
static int round_digits(int need) {
    if (need <= 5) return 5;
    if (need <= 8) return 8;
    if (need <= 9) return 9;
    return 0;
}
static bool is_transpose_of(const svdw_mat& b, const svdw_mat& a) {
    return a.phase == b.phase && a.off == b.off && a.rows == b.cols && a.cols == b.rows &&
           a.rs == b.cs && a.cs == b.rs;
}
static std::vector<uint32_t> maxbits_many(svdw_ctx* c, const std::vector<svdw_mat>& ms) {
    std::vector<uint32_t> out(ms.size(), 0);
    if (c->dry || ms.empty()) return out;
    settle(c);                                  // a pipelined witness's row scans read c->bits
    const size_t words = ms.size() * kMaxBitBlocks;
    ensure_buf(c, c->bits, words * sizeof(unsigned));
    std::vector<uint32_t> nb(ms.size());
    for (size_t i = 0; i < ms.size(); ++i) {
        const uint64_t n = (uint64_t)ms[i].rows * ms[i].cols;
        nb[i] = (uint32_t)std::min<uint64_t>((n + 255) / 256, kMaxBitBlocks);
        hipck(launch_maxbits(view_of(c, ms[i]), ms[i].rows, ms[i].cols,
                             (unsigned*)c->bits.p + i * kMaxBitBlocks, c->st), "k_maxbits");
    }
    std::vector<unsigned> h(words);
    hipck(hipMemcpyAsync(h.data(), c->bits.p, words * sizeof(unsigned), hipMemcpyDeviceToHost,
                         c->st), "D2H");
    sync(c);
    for (size_t i = 0; i < ms.size(); ++i)
        for (uint32_t b = 0; b < nb[i]; ++b) out[i] = std::max(out[i], h[i * kMaxBitBlocks + b]);
    return out;
}
// field_mat_mul (src/matrix/mod.rs:510-537) on stream `s`: c_s = a * b written
// as canonical cells at `out` (row-major). Exact: balanced base-256 digit planes
// + v_dot4c_i32_i8 when |entries| fit 9 digits, else Montgomery per MAC.
// With device bit-length words (sa, sb: one word each) the digit counts are
// read by the kernels themselves and the host needs no operand bounds.
// quantized: both operands are ZkMatrix::new cells (|x| < 2^128 by the u128
// saturation), so the CRT path always applies and no fallback is queued.
// CRT path residue reuse (prelaunched products of check_svd_phase0): b_cover
// makes b's planes (kept in digB) also valid for the product (b, b); a_from_b
// takes a's planes from digB (a is that b) instead of recomputing them.
// bbuf: where b's planes live (default digB); b_ready: they are already there
// (row-sharded v.v^T after m.v^T: same b, planes built with b_cover).
static void gemm_exec(svdw_ctx* c, hipStream_t s, const svdw_mat& a, const svdw_mat& b, Fr* out,
                      uint32_t bits_a, uint32_t bits_b, const unsigned* sa = nullptr,
                      const unsigned* sb = nullptr, bool quantized = false,
                      const unsigned* b_cover = nullptr, bool a_from_b = false,
                      DBuf* bbuf = nullptr, bool b_ready = false) {
    DBuf& BB = bbuf ? *bbuf : c->digB;
    const uint32_t N = a.rows, K = a.cols, M = b.cols;
    const bool sym = is_transpose_of(b, a);
    if (!sa && !sb && c->gemm_crt && c->gemm_impl == SVDW_GEMM_MFMA && bits_a <= 128 &&
        bits_b <= 128 && K <= 8192 && !c->dry) {
        // host-known bounds: hand them to the CRT kernels as device words
        // (stream-ordered memsets, one pair per stream)
        const int slot = s == c->st2 ? 2 : 0;
        ensure_buf(c, c->gbits, 4 * sizeof(unsigned));
        unsigned* w = (unsigned*)c->gbits.p + slot;
        hipck(hipMemsetD32Async((hipDeviceptr_t)w, bits_a, 1, s), "hipMemsetD32Async");
        hipck(hipMemsetD32Async((hipDeviceptr_t)(w + 1), bits_b, 1, s), "hipMemsetD32Async");
        sa = w;
        sb = w + 1;
    }
    if (sa && sb && c->gemm_crt && K <= 8192) {   // |acc| <= K 2^14 <= 2^27 (bias in k_gemm_crt)
        // multi-modular path: residue planes, one int8 GEMM per modulus, CRT
        uint32_t lk = 0;
        while ((1ull << lk) < K) ++lk;
        const uint32_t kpad = (K + 255) / 256 * 256;      // whole groups of four 64-k chunks
        const uint32_t rpa = (N + 127) / 128 * 128, rpb = (M + 127) / 128 * 128;
        ensure_buf(c, c->crtR, crt_scratch_bytes(N, M));
        const uint8_t* Ar;
        if (a_from_b && sym) {
            Ar = (const uint8_t*)BB.p;                    // planes of this operand already built
        } else {
            ensure_buf(c, c->digA, (size_t)kCrtMaxResidues * rpa * kpad);
            ProfScope ps(c, s, "k_to_residues", 32.0 * N * K, 0);
            hipck(launch_to_residues(view_of(c, a), N, K, rpa, kpad, (uint32_t*)c->digA.p, sa,
                                     sym ? sa : sb, lk, s), "k_to_residues");
            Ar = (const uint8_t*)c->digA.p;
        }
        const uint8_t* Br = Ar;
        if (!sym && !b_ready) {
            ensure_buf(c, BB, (size_t)kCrtMaxResidues * rpb * kpad);
            svdw_mat bt = b;   // Bt(j, k) = b(k, j)
            bt.rows = b.cols; bt.cols = b.rows; bt.rs = b.cs; bt.cs = b.rs;
            ProfScope ps(c, s, "k_to_residues", 32.0 * M * K, 0);
            hipck(launch_to_residues(view_of(c, bt), M, K, rpb, kpad, (uint32_t*)BB.p, sa, sb,
                                     lk, s, b_cover), "k_to_residues");
        }
        if (!sym) Br = (const uint8_t*)BB.p;
        {
            ProfScope ps(c, s, std::string("k_gemm_crt") + (sym ? ":s" : ""), 32.0 * N * M,
                         (double)N * M * K);
            hipck(launch_gemm_crt(sym, Ar, Br, N, M, rpa, sym ? rpa : rpb,
                                  kpad, (uint8_t*)c->crtR.p, out, M, 1, sa, sym ? sa : sb, lk, s,
                                  c->gemm_kern >= 0 ? (uint32_t)c->gemm_kern : (c->gemm_solo ? 3u : 0u)),
                  "k_gemm_crt");
        }
        if (!quantized)
            hipck(launch_gemm_mont(view_of(c, a), view_of(c, b), N, K, M, out, M, 1, s, sa,
                                   sym ? sa : sb, (int)lk), "k_gemm_mont");
        return;
    }
    if (sa && sb && K <= 8192) {
        const uint32_t kcn = (K + 63) / 64;
        const uint32_t npad = (N + 31) / 32 * 32, mpad = (M + 31) / 32 * 32;
        ensure_buf(c, c->digA, (size_t)npad * kcn * 9 * 64);
        {
            ProfScope ps(c, s, "k_to_digits_mf", 32.0 * N * K + 64.0 * npad * kcn * 9, 0);
            hipck(launch_to_digits_mf(view_of(c, a), N, K, 9, npad, kcn, (uint32_t*)c->digA.p, s, sa),
                  "k_to_digits_mf");
        }
        const uint8_t* Bd = (const uint8_t*)c->digA.p;
        if (!sym) {
            ensure_buf(c, c->digB, (size_t)mpad * kcn * 9 * 64);
            svdw_mat bt = b;   // Bt(j, k) = b(k, j)
            bt.rows = b.cols; bt.cols = b.rows; bt.rs = b.cs; bt.cs = b.rs;
            ProfScope ps(c, s, "k_to_digits_mf", 32.0 * M * K + 64.0 * mpad * kcn * 9, 0);
            hipck(launch_to_digits_mf(view_of(c, bt), M, K, 9, mpad, kcn, (uint32_t*)c->digB.p, s, sb),
                  "k_to_digits_mf");
            Bd = (const uint8_t*)c->digB.p;
        }
        {
            ProfScope ps(c, s, std::string("k_gemm_mfma:rt") + (sym ? "s" : ""),
                         32.0 * N * M, (double)N * M * K);
            hipck(launch_gemm_mfma_rt(sym, (const uint8_t*)c->digA.p, Bd, N, M, kcn, out, M, 1, sa,
                                      sym ? sa : sb, s), "k_gemm_mfma_rt");
        }
        hipck(launch_gemm_mont(view_of(c, a), view_of(c, b), N, K, M, out, M, 1, s, sa,
                               sym ? sa : sb), "k_gemm_mont");
        return;
    }
    int DA = round_digits(digits_for_bits(bits_a)), DB = round_digits(digits_for_bits(bits_b));
    const bool digits_ok = DA && DB && K <= 8192 && gemm_digits_supported(DA, DB);
    if (digits_ok && c->gemm_impl == SVDW_GEMM_MFMA) {
        const uint32_t kcn = (K + 63) / 64;
        const uint32_t npad = (N + 31) / 32 * 32, mpad = (M + 31) / 32 * 32;
        ensure_buf(c, c->digA, (size_t)npad * kcn * DA * 64);
        {
            ProfScope ps(c, s, "k_to_digits_mf", 32.0 * N * K + 64.0 * npad * kcn * DA, 0);
            hipck(launch_to_digits_mf(view_of(c, a), N, K, DA, npad, kcn, (uint32_t*)c->digA.p, s),
                  "k_to_digits_mf");
        }
        const uint8_t* Bd = (const uint8_t*)c->digA.p;
        if (!sym) {
            ensure_buf(c, c->digB, (size_t)mpad * kcn * DB * 64);
            svdw_mat bt = b;   // Bt(j, k) = b(k, j)
            bt.rows = b.cols; bt.cols = b.rows; bt.rs = b.cs; bt.cs = b.rs;
            ProfScope ps(c, s, "k_to_digits_mf", 32.0 * M * K + 64.0 * mpad * kcn * DB, 0);
            hipck(launch_to_digits_mf(view_of(c, bt), M, K, DB, mpad, kcn, (uint32_t*)c->digB.p, s),
                  "k_to_digits_mf");
            Bd = (const uint8_t*)c->digB.p;
        }
        ProfScope ps(c, s, std::string("k_gemm_mfma:") + std::to_string(DA) + "x" +
                               std::to_string(DB) + (sym ? "s" : ""),
                     64.0 * kcn * ((double)npad * DA + (sym ? 0.0 : (double)mpad * DB)) + 32.0 * N * M,
                     (double)N * M * K);
        hipck(launch_gemm_mfma(DA, DB, sym, (const uint8_t*)c->digA.p, Bd, N, M, kcn, out, M, 1, s),
              "k_gemm_mfma");
    } else if (digits_ok) {
        const uint32_t kg = ((K + 3) / 4 + 7) / 8 * 8;
        const uint32_t npad = (N + 31) / 32 * 32, mpad = (M + 31) / 32 * 32;
        ensure_buf(c, c->digA, (size_t)npad * kg * DA * 4);
        {
            ProfScope ps(c, s, "k_to_digits", 32.0 * N * K + 4.0 * npad * kg * DA, 0);
            hipck(launch_to_digits(view_of(c, a), N, K, DA, npad, kg, (uint32_t*)c->digA.p, s),
                  "k_to_digits");
        }
        const uint32_t* Bd = (const uint32_t*)c->digA.p;
        if (!sym) {
            ensure_buf(c, c->digB, (size_t)mpad * kg * DB * 4);
            svdw_mat bt = b;   // Bt(j, k) = b(k, j)
            bt.rows = b.cols; bt.cols = b.rows; bt.rs = b.cs; bt.cs = b.rs;
            ProfScope ps(c, s, "k_to_digits", 32.0 * M * K + 4.0 * mpad * kg * DB, 0);
            hipck(launch_to_digits(view_of(c, bt), M, K, DB, mpad, kg, (uint32_t*)c->digB.p, s),
                  "k_to_digits");
            Bd = (const uint32_t*)c->digB.p;
        }
        ProfScope ps(c, s, std::string("k_gemm_dot4:") + std::to_string(DA) + "x" +
                               std::to_string(DB) + (sym ? "s" : ""),
                     4.0 * kg * ((double)npad * DA + (sym ? 0.0 : (double)mpad * DB)) + 32.0 * N * M,
                     (double)N * M * K);
        hipck(launch_gemm_digits(DA, DB, sym, (const uint32_t*)c->digA.p, Bd, N, M, kg, out, M, 1, s),
              "k_gemm_dot4");
    } else {
        ProfScope ps(c, s, "k_gemm_mont", 32.0 * ((double)N * K + (double)K * M + (double)N * M),
                     (double)N * M * K);
        hipck(launch_gemm_mont(view_of(c, a), view_of(c, b), N, K, M, out, M, 1, s), "k_gemm_mont");
    }
}
// rows [r0, r1) of a matrix view
static svdw_mat row_block(const svdw_mat& a, uint64_t r0, uint64_t r1) {
    return svdw_mat{a.phase, (uint32_t)(r1 - r0), a.cols, a.off + r0 * a.rs, a.rs, a.cs};
}
// honest_prover_mat_mul (src/matrix/mod.rs:546-568). bits_a/bits_b: known bounds or ~0u.
// If the product was launched ahead on st2 (c->pre), only append and order st after it.
static svdw_mat honest_prover_mat_mul(svdw_ctx* c, uint32_t phase, const svdw_mat& a,
                                      const svdw_mat& b, uint32_t bits_a = ~0u,
                                      uint32_t bits_b = ~0u) {
    REQUIRE(a.cols == b.rows, "honest_prover_mat_mul: a.num_col != b.num_rows");
    const uint32_t N = a.rows, M = b.cols;
    uint64_t off;
    append(c, phase, (uint64_t)N * M, 0, &off, nullptr, "product", N);
    svdw_mat cs{phase, N, M, off, (int64_t)M, 1};
    if (c->gemm_log) c->gemm_log->push_back(off);
    uint64_t sr0 = 0, sr1 = N;                            // shard: rows of c_s computed here
    if (sharded(c)) {
        shard_rows(c, N, &sr0, &sr1);
        own(c, phase, false, off + sr0 * M, (sr1 - sr0) * M);
    }
    {   // |c_s| <= K * 2^bits_a * 2^bits_b, resolved when the operand bounds are known
        uint32_t lk = 0;
        while ((1ull << lk) < a.cols) ++lk;
        c->prods.push_back({cs, a, b, lk});
    }
    if (bits_a == ~0u) bits_a = bits_of(c, a);
    if (bits_b == ~0u) bits_b = bits_of(c, b);
    if (c->dry) return cs;
    if (!c->pre.empty()) {
        if (c->pre.front().off != off) fail(SVDW_EDEVICE, "internal: pre-launched GEMM offset mismatch");
        // (launched on this very stream: already ordered; the three batched
        // products share one event: one wait per stream)
        if (c->pre.front().st != c->st && !(c->pre_wait_st == c->st && c->pre_wait_ev == c->pre.front().ev)) {
            dep_wait(c, c->st, c->pre.front().ev);
            c->pre_wait_st = c->st;
            c->pre_wait_ev = c->pre.front().ev;
        }
        c->pre.erase(c->pre.begin());
        return cs;
    }
    const bool sym = is_transpose_of(b, a);
    if (bits_a == ~0u || bits_b == ~0u) {
        std::vector<svdw_mat> ms{a};
        if (!sym) ms.push_back(b);
        auto bb = maxbits_many(c, ms);
        bits_a = bb[0];
        bits_b = sym ? bb[0] : bb[1];
        reg_bits(c, a, bits_a);
        reg_bits(c, b, bits_b);
    }
    if (sharded(c)) {
        if (sr1 > sr0)
            gemm_exec(c, c->st, row_block(a, sr0, sr1), b, cellp(c, phase, off + sr0 * M), bits_a,
                      bits_b);
        return cs;
    }
    gemm_exec(c, c->st, a, b, cellp(c, phase, off), bits_a, bits_b);
    return cs;
}
// Words of the small operand for the row-scan products: |signed a| < 2^(32 na)
// when a's bound is known to the host, else 8 (full Montgomery).
static int scan_na(const svdw_ctx* c, const svdw_mat& a) {
    const uint32_t b = bits_of(c, a);
    if (b == ~0u || b > 192) return 8;
    return std::max(1, (int)((b + 31) / 32));
}
// The same bound as the device sees it: a quantized matrix's bit-length word, or
// a product of two of them (bits_a + bits_b + lk); wa = -1: unknown.
static NaSpec scan_spec(const svdw_ctx* c, const svdw_mat& a) {
    auto word = [&](const svdw_mat& m) -> int16_t {
        for (auto& r : c->dwords)
            if (same_cells(r.m, m)) return r.word;
        return -1;
    };
    const int16_t w = word(a);
    if (w >= 0) return NaSpec{w, -1, 0, 0};
    for (auto& p : c->prods)
        if (same_cells(p.cs, a)) {
            const int16_t wa = word(p.a), wb = word(p.b);
            if (wa >= 0 && wb >= 0) return NaSpec{wa, wb, (uint16_t)p.lk, 0};
        }
    return NaSpec{-1, -1, 0, 0};
}
// A scan job's bound for the device: host-known bits as a constant (wa = -2,
// bits in lk), else its device words (scan_spec).
static NaSpec job_spec(const svdw_ctx* c, const svdw_mat& a) {
    const uint32_t b = bits_of(c, a);
    if (b != ~0u) return NaSpec{-2, -1, (uint16_t)std::min(b, 65535u), 0};
    return scan_spec(c, a);
}
// na of a batch of scans: host-known (1..8), or 0 = decided on the device from
// the jobs' specs (job_spec), so the host needs no operand bounds
static int batch_na_host(const svdw_ctx* c, const svdw_mat* ms, int n) {
    int na = 1;
    bool host = true, dev = c->dbitw != nullptr;
    for (int i = 0; i < n; ++i) {
        if (bits_of(c, ms[i]) != ~0u) na = std::max(na, scan_na(c, ms[i]));
        else host = false;
        if (job_spec(c, ms[i]).wa == -1) dev = false;
    }
    if (host) return na;
    return dev ? 0 : 8;
}
// mont_mul(w, f[s]) = slot s of w's scaled table: w * 2^(32 (s + 1)) for s < 6,
// w's Montgomery form for s = 6 (kernels.hpp kTabSlots)
static ScaleTab scale_tab() {
    ScaleTab t;
    for (int s = 0; s < kTabSlots - 1; ++s) {
        Fr x = fr_zero();
        x.w[s + 1] = 1;                                    // 2^(32 (s + 1)) < p
        t.f[s] = mont_mul(x, fr_r2());
    }
    t.f[kTabSlots - 1] = fr_r2();
    return t;
}
// field_mat_vec_mul with the vector given as canonical copy + scaled table.
// the equality sources of an inner-product row region: a's row i, the vector w
static void note_scan(svdw_ctx* c, const svdw_mat& a, const RegionChecks::EqSrc& w) {
    RegionChecks& r = c->layout_chk.back();
    r.scan = true;
    r.unit = 3 * a.cols + 1;
    r.esrc[0] = eqsrc_mat(a);
    r.esrc[1] = w;
}
static svdw_vec matvec_rows(svdw_ctx* c, uint32_t phase, const svdw_mat& a, const Fr* wc,
                            const Fr* tab, uint32_t tl, int na, const RegionChecks::EqSrc& wsrc) {
    const uint32_t R = a.rows, L = a.cols;
    uint64_t off;
    append(c, phase, (uint64_t)R * (3ull * L + 1), 0, &off, nullptr, "scan", R);
    note_scan(c, a, wsrc);
    uint64_t r0 = 0, r1 = R;
    if (sharded(c)) {
        shard_rows(c, R, &r0, &r1);
        own(c, phase, false, off + r0 * (3ull * L + 1), (r1 - r0) * (3ull * L + 1));
    }
    if (!c->dry) {
        ProfScope ps(c, c->st, a.cs == 1 ? "k_matvec_scan:rows" : "k_matvec_scan:cols", 32.0 * (double)R * (4.0 * L + 1) + 64.0 * L, (double)R * L);
        hipck(launch_matvec_scan(view_of(c, a), (uint32_t)r0, (uint32_t)r1, L, wc, tab, tl,
                                 cellp(c, phase, off + r0 * (3ull * L + 1)), na,
                                 c->st), "k_matvec_scan");
    }
    return svdw_vec{phase, R, off + 3ull * L, (int64_t)(3ull * L + 1)};
}
// canonical copy into bc, scaled table into bt
static const Fr* vec_prep_view(svdw_ctx* c, const DView& w, uint32_t len, DBuf& bc, DBuf& bt) {
    ensure_buf(c, bc, (size_t)len * sizeof(Fr));
    ensure_buf(c, bt, tab_len(len) * sizeof(Fr));
    if (!c->dry) {
        ProfScope ps(c, c->st, "k_vec_prep", 32.0 * len * (2 + tab_len(1)), 0);
        hipck(launch_vec_prep(w, len, (Fr*)bc.p, (Fr*)bt.p, scale_tab(), c->st), "k_vec_prep");
    }
    return (const Fr*)bt.p;
}
static const Fr* vec_prep(svdw_ctx* c, const svdw_vec& v, DBuf& bc, DBuf& bt) {
    return vec_prep_view(c, view_of(c, svdw_mat{v.phase, 1, v.len, v.off, 0, v.stride}), v.len, bc, bt);
}
// the same from a device vector of len canonical values
static const Fr* vec_prep_ptr(svdw_ctx* c, const Fr* src, uint32_t len, DBuf& bc, DBuf& bt) {
    DView w;
    memset(&w, 0, sizeof w);
    w.ptr = src;
    w.rs = 0; w.cs = 1; w.rows = 1; w.cols = len;
    return vec_prep_view(c, w, len, bc, bt);
}
static svdw_vec field_mat_vec_mul(svdw_ctx* c, uint32_t phase, const svdw_mat& a,
                                  const svdw_vec& v) {
    REQUIRE(a.cols == v.len, "field_mat_vec_mul: a[0].len() != v.len()");
    const int na = scan_na(c, a);
    const Fr* tab = vec_prep(c, v, c->w1c, c->w1t);
    return matvec_rows(c, phase, a, (const Fr*)c->w1c.p, tab, v.len, na, eqsrc_vec(v));
}
// ZkMatrix::verify_mul (src/matrix/mod.rs:251-282) for several (a, b, c_s) triples
// with one gamma: cells are appended exactly as consecutive verify_mul calls
// would append them, then the row scans run as three batched launches (all
// c_s.v scans, all b.v scans, all a.(b.v) scans) so the rows of every call
// share one wave of blocks.
struct VMul {
    svdw_mat a, b, cs;
};
// v = (1, g, g^2, ...): canonical (gpc) + scaled table (gtab), on stream s. The
// powers come from three host-side Montgomery tables (g^a, g^(16 b), g^(256 c)):
// three products per element on the device instead of a square-and-multiply chain.
static void gamma_prep(svdw_ctx* c, uint32_t d, const Fr& gamma, hipStream_t s, const PowCells* pc = nullptr) {
    if (c->dry) return;
    REQUIRE(!c->capturing, "internal: gamma inside a captured graph");
    const uint32_t len = std::max(d, 1u);
    REQUIRE((len + 255) / 256 <= (uint32_t)kGammaTab - 32, "verify_mul: vector too long");
    ensure_buf(c, c->gpc, (size_t)len * sizeof(Fr));
    ensure_buf(c, c->gtab, tab_len(len) * sizeof(Fr));
    GammaTab g;
    memset(&g, 0, sizeof g);
    const Fr one = fr_to_mont(fr_from_u64(1)), gm = fr_to_mont(gamma);
    g.t[0] = one;
    for (int i = 1; i < 16; ++i) g.t[i] = mont_mul(g.t[i - 1], gm);
    const Fr g16 = mont_mul(g.t[15], gm);
    g.t[16] = one;
    for (int i = 1; i < 16; ++i) g.t[16 + i] = mont_mul(g.t[15 + i], g16);
    const Fr g256 = mont_mul(g.t[31], g16);
    g.nhi = (len + 255) / 256;
    g.t[32] = one;
    for (uint32_t i = 1; i < g.nhi; ++i) g.t[32 + i] = mont_mul(g.t[31 + i], g256);
    {
        ProfScope ps(c, s, "k_gamma_prep", 32.0 * len * (1 + tab_len(1)), 0);
        hipck(launch_gamma_prep(g, len, (Fr*)c->gpc.p, (Fr*)c->gtab.p, scale_tab(), s, pc),
              "k_gamma_prep");
    }
    c->gp_gamma = gamma;
    c->gp_len = len;
}
// gamma vector for verify_mul on c->st: the one queued ahead when it matches,
// else prepared here
static void ensure_gamma_vec(svdw_ctx* c, uint32_t d, const Fr& gamma) {
    if (c->dry) return;
    if (c->gp_ev && c->gp_len >= d && fr_eq(c->gp_gamma, gamma)) {
        if (c->gp_st != c->st) dep_wait(c, c->st, c->gp_ev);
        return;
    }
    gamma_prep(c, d, gamma, c->st);
    c->gp_ev = nullptr;
}
static void verify_mul_many(svdw_ctx* c, uint32_t phase, const VMul* vm, int n, const Fr& gamma) {
    REQUIRE(n >= 1 && n <= kMaxVerifyBatch, "internal: verify_mul batch size");
    c->ext_gamma = gamma;
    struct Plan {
        PB one, pows, eq;
        uint64_t one_off = 0, one_loff = 0, pows_off = 0, pows_loff = 0, eq_off = 0, eq_loff = 0;
        size_t eq_reg = 0;                // its layout region (views noted at launch)
        svdw_vec csv{}, bv{}, abv{};
        explicit Plan(uint32_t lb) : one(lb), pows(lb), eq(lb) {}
    };
    std::vector<Plan> pl;
    pl.reserve(n);
    uint32_t dmax = 0;
    auto scan_append = [&](const svdw_mat& a, const RegionChecks::EqSrc& w) {
        uint64_t off;
        append(c, phase, (uint64_t)a.rows * (3ull * a.cols + 1), 0, &off, nullptr, "scan", a.rows);
        note_scan(c, a, w);
        note_const(c, fr_zero());                             // inner_product's Constant(0)
        return svdw_vec{phase, a.rows, off + 3ull * a.cols, (int64_t)(3ull * a.cols + 1)};
    };
    // pass 1: the cell layout, in the reference's order
    for (int i = 0; i < n; ++i) {
        const svdw_mat &a = vm[i].a, &b = vm[i].b, &cs = vm[i].cs;
        REQUIRE(a.cols == b.rows, "verify_mul: a.num_col != b.num_rows");
        REQUIRE(cs.rows == a.rows, "verify_mul: c_s.len() != a.num_rows");
        REQUIRE(cs.cols == b.cols, "verify_mul: c_s[0].len() != b.num_col");
        const uint32_t d = cs.cols;
        dmax = std::max(dmax, d);
        pl.emplace_back(c->LB);
        Plan& p = pl.back();
        p.one.cell(p.one.K(fr_from_u64(1)));                  // load_witness(F::ONE)
        append(c, phase, p.one.a.C, 0, &p.one_off, &p.one_loff, "load_cell");
        note_gates(c, p.one);                                 // assert_is_const(one, 1)
        stage_own(c, phase, p.one, 1, 1, p.one_off, p.one_loff);
        if (d > 1) {                                          // v_i = mul(v_{i-1}, init_rand)
            uint8_t prev = p.pows.load(0), cur = p.pows.load(1);
            p.pows.gate(0);                               // mul(v_(i-1), init_rand)
            p.pows.kext = p.pows.kidx(gamma);             // gamma: a cell of the RLC context
            p.pows.vsrc[1] = false;                       // v_i: produced here
            note_const(c, fr_zero());
            p.pows.cell(p.pows.K(0)); p.pows.cell(prev); p.pows.cell(p.pows.K(gamma)); p.pows.cell(cur);
            append(c, phase, (uint64_t)(d - 1) * p.pows.a.C, 0, &p.pows_off, &p.pows_loff,
                   "verify_mul_gamma_pows");
            note_gates(c, p.pows);
            c->gamma_slots.emplace_back(c->layout_chk.size() - 1, p.pows.kext);
            // v_(i-1): the `one` cell, then the previous mul's output
            c->layout_chk.back().esrc[0] = eqsrc_chain(phase, p.one_off, phase, p.pows_off + 3, 4);
            stage_own(c, phase, p.pows, d - 1, 1, p.pows_off, p.pows_loff);
        }
        const RegionChecks::EqSrc gsrc = eqsrc_chain(phase, p.one_off, phase, p.pows_off + 3, 4);
        p.csv = scan_append(cs, gsrc);
        p.bv = scan_append(b, gsrc);
        p.abv = scan_append(a, eqsrc_vec(p.bv));
        if (sharded(c)) {                                 // this rank's rows of the three scans
            for (const auto& sv : {std::make_pair(cs, p.csv), std::make_pair(b, p.bv),
                                   std::make_pair(a, p.abv)}) {
                const uint64_t rowc = 3ull * sv.first.cols + 1, base = sv.second.off - 3ull * sv.first.cols;
                uint64_t r0, r1;
                shard_rows(c, sv.first.rows, &r0, &r1);
                own(c, phase, false, base + r0 * rowc, (r1 - r0) * rowc);
            }
        }
        uint8_t x = p.eq.load(0), y = p.eq.load(1);           // is_equal per row (result unused)
        p.eq.g_is_equal(x, y);
        append(c, phase, (uint64_t)a.rows * p.eq.a.C, (uint64_t)a.rows * p.eq.a.L, &p.eq_off,
               &p.eq_loff, "verify_mul_is_equal", a.rows);
        note_gates(c, p.eq);
        p.eq_reg = c->layout_chk.size() - 1;
        c->layout_chk.back().esrc[0] = eqsrc_mat(mat_of_vec(p.csv));
        c->layout_chk.back().esrc[1] = eqsrc_mat(mat_of_vec(p.abv));
        stage_own(c, phase, p.eq, a.rows, 1, p.eq_off, p.eq_loff);
    }
    if (c->dry) return;
    host_mark(c, "verify_mul layout");
    // pass 2: launches
    ensure_gamma_vec(c, dmax, gamma);
    const Fr* gpc = (const Fr*)c->gpc.p;
    const Fr* gtab = (const Fr*)c->gtab.p;
    // verify_mul_witness: k_gamma_prep already wrote the one cell and the powers
    const bool pre = c->pows_pre.on && n == 1 && pl[0].one_off == c->pows_pre.one_off &&
                     pl[0].pows_off == c->pows_pre.pows_off && vm[0].cs.cols == c->pows_pre.d &&
                     pl[0].one_loff == 0;
    c->pows_pre.on = false;
    // the one cells and gamma powers: read by no kernel of the call (gpc, not
    // these cells, feeds the scans), so a pipelined svd_witness launches them
    // after the scans, off the head of phase 1's stream
    auto pows_launch = [&] {
        if (pre) return;
        // (a captured graph must not hold gamma: the powers' launch carries it)
        for (int i = 0; i < n; ++i) REQUIRE(!c->capturing || vm[i].cs.cols <= 1, "internal: gamma inside a captured graph");
        BatchScope bs(c);                                 // the one cells and gamma powers: one launch
        for (int i = 0; i < n; ++i) {
            Plan& p = pl[i];
            const uint32_t d = vm[i].cs.cols;
            stage_launch(c, phase, p.one, 1, 1, p.one_off, p.one_loff, "load_cell");
            if (d > 1) {
                DView w;
                memset(&w, 0, sizeof w);
                w.ptr = gpc;
                w.rs = 1; w.cs = 0; w.rows = d; w.cols = 1;
                p.pows.a.view[0] = w;
                p.pows.a.view[1] = w;
                p.pows.a.view[1].ptr = gpc + 1;
                stage_launch(c, phase, p.pows, d - 1, 1, p.pows_off, p.pows_loff, "verify_mul_gamma_pows");
            }
        }
        bs.end();
    };
    const bool pows_late = c->in_pipe;
    if (!pows_late) pows_launch();
    // One scan launch over jobs (a_q against the vector wc_q / tab_q, cells at
    // v_q); operand widths host-known or read on the device (na 0).
    struct Scans {
        ScanBatch sb;
        svdw_mat ms[kMaxScanJobs];
        double bytes = 0, ops = 0;
        Scans() { memset(&sb, 0, sizeof sb); }
    };
    auto add_job = [&](Scans& S, const svdw_mat& a, const svdw_vec& v, const Fr* wc, const Fr* tab,
                       uint32_t tl) -> ScanJob& {
        REQUIRE(S.sb.njobs < (uint32_t)kMaxScanJobs, "internal: scan batch full");
        uint64_t r0 = 0, r1 = a.rows;                     // shard: this rank's rows
        const uint64_t rowc = 3ull * a.cols + 1, base = v.off - 3ull * a.cols;
        if (sharded(c)) shard_rows(c, a.rows, &r0, &r1);
        S.ms[S.sb.njobs] = a;
        ScanJob& j = S.sb.job[S.sb.njobs++];
        j = ScanJob{f64_view(c, view_of(c, a)), wc, tab, tl, cellp(c, phase, base + r0 * rowc),
                    a.cols, (uint32_t)(r1 - r0), 0, (uint32_t)r0, job_spec(c, a)};
        S.bytes += 32.0 * (r1 - r0) * (4.0 * a.cols + 1) + 64.0 * a.cols;
        S.ops += (double)(r1 - r0) * a.cols;
        return j;
    };
    auto launch = [&](Scans& S, const char* name) {
        S.sb.bitw = c->dbitw;
        S.sb.f = scale_tab();
        const int na = batch_na_host(c, S.ms, (int)S.sb.njobs);
        ProfScope ps(c, c->st, name, S.bytes, S.ops);
        hipck(launch_scan_batch(S.sb, na, c->st), "k_matvec_scan");
    };
    // b.g of job i: the b scan of the first job with the same b (m.v^T and
    // v.v^T share v^T) serves every later job with it
    int src[kMaxVerifyBatch];
    for (int i = 0; i < n; ++i) {
        src[i] = i;
        for (int k = 0; k < i; ++k)
            if (vm[k].b.phase == vm[i].b.phase && vm[k].b.off == vm[i].b.off &&
                vm[k].b.rows == vm[i].b.rows && vm[k].b.cols == vm[i].b.cols &&
                vm[k].b.rs == vm[i].b.rs && vm[k].b.cs == vm[i].b.cs) { src[i] = k; break; }
    }
    const Fr* wt[kMaxVerifyBatch];
    // b = X^T of an f64 input of svd_witness: X, else null
    auto f64_of = [&](const svdw_mat& b) -> const svdw_ctx::F64Src* {
        if (b.cols > 8192) return nullptr;
        for (auto& s : c->f64src)
            if (is_transpose_of(b, s.m) && s.m.rs == (int64_t)s.m.cols && s.m.cs == 1) return &s;
        return nullptr;
    };
    bool all_f64 = true;
    for (int i = 0; i < n && all_f64; ++i) all_f64 = f64_of(vm[i].b) != nullptr;
    // launch order != append order: the b and a.(b.g) scans need only the
    // operands, the c_s scans wait for the products when those run elsewhere
    Scans bs_, as_;
    auto add_b = [&](Scans& S, int i) -> ScanJob& { return add_job(S, vm[i].b, pl[i].bv, gpc, gtab, c->gp_len); };
    auto add_a = [&](Scans& S, int i) {
        add_job(S, vm[i].a, pl[i].abv, (const Fr*)c->wbc[src[i]].p, wt[i], vm[i].b.rows);
    };
    if (all_f64) {
        // every entry of b.g from the f64 rows of X (quantized in registers),
        // column-parallel and coalesced: one launch for the distinct b's, then
        // the slices' sums folded into each vector's table (k_vec_prep_sum);
        // the b and a.(b.g) scans are then independent: one launch
        ColBatch cb;
        memset(&cb, 0, sizeof cb);
        cb.tab = gtab;
        cb.tl = c->gp_len;
        cb.bitw = c->dbitw;
        int slot[kMaxVerifyBatch];
        size_t poff[kMaxVerifyBatch], ptot = 0;
        for (int i = 0; i < n; ++i) {
            if (src[i] != i) { slot[i] = slot[src[i]]; continue; }
            REQUIRE(cb.njobs < (uint32_t)kMaxColJobs, "internal: too many distinct b for k_colsum_f64");
            const svdw_ctx::F64Src* s = f64_of(vm[i].b);
            ColJob& j = cb.job[cb.njobs];
            j.x = s->x;
            j.R = s->m.rows;
            j.C = s->m.cols;
            j.ld = s->m.cols;
            j.spec = job_spec(c, vm[i].b);
            poff[cb.njobs] = ptot;
            ptot += (size_t)colsum_slices(j.R) * j.C;
            slot[i] = (int)cb.njobs++;
        }
        ensure_buf(c, c->colpart, ptot * sizeof(Fr));
        for (uint32_t q = 0; q < cb.njobs; ++q) cb.job[q].part = (Fr*)c->colpart.p + poff[q];
        {
            ProfScope ps(c, c->st, "k_colsum_f64", 0, 0);
            hipck(launch_colsum_f64(cb, (int)c->P, c->st), "k_colsum_f64");
        }
        // the distinct b's vectors in one launch
        VecPrepBatch vp;
        memset(&vp, 0, sizeof vp);
        double vbytes = 0;
        for (int i = 0; i < n; ++i) {
            if (src[i] != i) { wt[i] = wt[src[i]]; continue; }
            const uint32_t L = vm[i].b.rows;
            ensure_buf(c, c->wbc[i], (size_t)L * sizeof(Fr));
            ensure_buf(c, c->wbt[i], tab_len(L) * sizeof(Fr));
            REQUIRE(vp.njobs < (uint32_t)kMaxColJobs, "internal: too many distinct b for k_vec_prep_sum");
            vp.job[vp.njobs++] = VecPrepJob{cb.job[slot[i]].part, colsum_slices(cb.job[slot[i]].R), L,
                                            (Fr*)c->wbc[i].p, (Fr*)c->wbt[i].p, 0};
            vbytes += 32.0 * L * (2 + tab_len(1));
            wt[i] = (const Fr*)c->wbt[i].p;
        }
        {
            ProfScope ps(c, c->st, "k_vec_prep", vbytes, 0);
            hipck(launch_vec_prep_sum_multi(vp, scale_tab(), c->st), "k_vec_prep_sum_multi");
        }
        for (int i = 0; i < n; ++i) add_b(bs_, i);
        for (int i = 0; i < n; ++i) add_a(bs_, i);
        launch(bs_, "k_matvec_scan:ba");
    } else if (sharded(c)) {
        for (int i = 0; i < n; ++i) add_b(bs_, i);
        launch(bs_, "k_matvec_scan:b");
        // only this rank's rows of the b.g scans exist: every entry of b.g comes
        // from the values-only mat-vec instead (the distinct b's in one launch)
        ScanBatch vb;
        memset(&vb, 0, sizeof vb);
        svdw_mat vms[kMaxVerifyBatch];
        int nv = 0, slot[kMaxVerifyBatch];
        for (int i = 0; i < n; ++i) {
            if (src[i] != i) { slot[i] = slot[src[i]]; continue; }
            const svdw_mat b = vm[i].b;
            ensure_buf(c, c->bvfull[nv], (size_t)b.rows * sizeof(Fr));
            vb.job[nv] = ScanJob{f64_view(c, view_of(c, b)), nullptr, gtab, c->gp_len, (Fr*)c->bvfull[nv].p,
                                 b.cols, b.rows, 0, 0, job_spec(c, b)};
            vms[nv] = b;
            slot[i] = nv++;
        }
        vb.njobs = nv;
        vb.bitw = c->dbitw;
        {
            ProfScope ps(c, c->st, "k_matvec_values", 0, 0);
            hipck(launch_matvec_values(vb, batch_na_host(c, vms, nv), c->st), "k_matvec_values");
        }
        for (int i = 0; i < n; ++i)
            wt[i] = src[i] != i ? wt[src[i]]
                                : vec_prep_ptr(c, (const Fr*)c->bvfull[slot[i]].p, vm[i].b.rows,
                                               c->wbc[i], c->wbt[i]);
        for (int i = 0; i < n; ++i) add_a(as_, i);
        launch(as_, "k_matvec_scan:a");
    } else {
        // every row of b scanned: the b scan of each distinct b also writes b.g
        // as the a scan's vector (canonical + table) from its row totals
        for (int i = 0; i < n; ++i) {
            ScanJob& j = add_b(bs_, i);
            if (src[i] != i) continue;
            const uint32_t L = vm[i].b.rows;
            ensure_buf(c, c->wbc[i], (size_t)L * sizeof(Fr));
            ensure_buf(c, c->wbt[i], tab_len(L) * sizeof(Fr));
            j.pc = (Fr*)c->wbc[i].p;
            j.ptab = (Fr*)c->wbt[i].p;
            j.plen = L;
        }
        for (int i = 0; i < n; ++i) wt[i] = (const Fr*)c->wbt[src[i]].p;
        launch(bs_, "k_matvec_scan:b");
        for (int i = 0; i < n; ++i) add_a(as_, i);
        launch(as_, "k_matvec_scan:a");
    }
    host_mark(c, "verify_mul b, a scans queued");
    for (hipEvent_t ev : c->wait_before_cs)
        dep_wait(c, c->st, ev);
    // the c_s scans; each row's is_equal(c_s.g, a.(b.g)) cells from its row
    // total and the a scan's last cell (k_matvec_scan_dpp's eq epilogue)
    Scans cs_;
    for (int i = 0; i < n; ++i) {
        Plan& p = pl[i];
        ScanJob& j = add_job(cs_, vm[i].cs, p.csv, gpc, gtab, c->gp_len);
        j.eq_out = cellp(c, phase, p.eq_off);
        j.eq_y = cellp(c, p.abv.phase, p.abv.off);
        j.eq_ys = (uint32_t)p.abv.stride;
        p.eq.a.view[0] = view_of(c, mat_of_vec(p.csv));
        p.eq.a.view[1] = view_of(c, mat_of_vec(p.abv));
        note_gates(c, p.eq, 1, p.eq_reg);
    }
    launch(cs_, "k_matvec_scan:cs");
    if (pows_late) pows_launch();
}
static void verify_mul(svdw_ctx* c, uint32_t phase, const svdw_mat& a, const svdw_mat& b,
                       const svdw_mat& cs, const Fr& gamma) {
    VMul v{a, b, cs};
    verify_mul_many(c, phase, &v, 1, gamma);
}

// err_calc (src/svd/mod.rs:155-163). Host f64, built with -ffp-contract=off.
static void err_calc(uint32_t p, uint64_t size, double max_norm, double eps_svd, double eps_u,
                     double* es, double* eu) {
    volatile double precision = pow(2.0, -1.0 * ((double)p + 1.0));
    double s = (double)size;
    *es = precision * s * (1.0 + max_norm + eps_svd + precision) + s * max_norm * precision +
          pow(1.0 + eps_u, 0.5) * (max_norm + eps_svd) * eps_u + pow(1.0 + eps_u, 0.5) * eps_svd;
    *eu = eps_u + precision * s * (2.0 * (1.0 + eps_u) + precision);
}
// `(err * (2u128.pow(2P) as f64)).round() as u128`
static BigU scale_err(double err, uint32_t p) {
    double x = round(err * ldexp(1.0, 2 * (int)p));
    if (!(x > 0)) return big_from_u128(0);
    if (x >= 340282366920938463463374607431768211456.0) return big_from_u128(~(unsigned __int128)0);
    return big_from_u128((unsigned __int128)x);
}

// The three products of check_svd_phase0 (A[g] * B[g], B = transposes) on st2
// from residue planes built in one k_residues_f64 launch over svd_witness's f64
// inputs: m (this rank's rows) into digA, v into digB (covering m.v^T and
// v.v^T), u into digC. Planes of v and u carry 128 rows of slack so a row block
// (sharded rank) reads its A tiles as a slice of the full planes. log[g]: the
// products' stream offsets (dry replay); W: the device bit-length words of m, u, v.
static void prelaunch_products_f64(svdw_ctx* c, const svdw_mat (&A)[3], const svdw_mat (&B)[3],
                                   const std::vector<uint64_t>& log, uint32_t phase,
                                   unsigned* W, hipStream_t pst) {
    const uint32_t N = A[0].rows, M = A[0].cols;
    auto clog2 = [](uint32_t k) { uint32_t l = 0; while ((1ull << l) < k) ++l; return l; };
    auto ceil_to = [](uint32_t x, uint32_t a) { return (x + a - 1) / a * a; };
    const uint32_t lkM = clog2(M), lkN = clog2(N), kpM = ceil_to(M, 256), kpN = ceil_to(N, 256);
    uint64_t rr0[3], rr1[3];
    for (int g = 0; g < 3; ++g) {
        rr0[g] = 0; rr1[g] = A[g].rows;
        if (sharded(c)) shard_rows(c, A[g].rows, &rr0[g], &rr1[g]);
    }
    const uint32_t rows_m = (uint32_t)(rr1[0] - rr0[0]);
    const uint32_t rp_m = ceil_to(std::max(rows_m, 1u), 128), rp_v = ceil_to(M, 128) + 128,
                   rp_u = ceil_to(N, 128) + 128;
    ensure_buf(c, c->digA, (size_t)kCrtMaxResidues * rp_m * kpM);
    ensure_buf(c, c->digB, (size_t)kCrtMaxResidues * rp_v * kpM);
    ensure_buf(c, c->digC, (size_t)kCrtMaxResidues * rp_u * kpN);
    ResSegs q;
    memset(&q, 0, sizeof q);
    auto seg = [&](const double* in, uint32_t rows, uint32_t cols, uint32_t rp, uint32_t kp,
                   DBuf& out, std::initializer_list<std::array<int, 3>> pairs) {
        ResSeg& g = q.seg[q.nseg++];
        g.in = in; g.out = (uint32_t*)out.p;
        g.rows = rows; g.cols = cols; g.ld = cols; g.rows_pad = rp; g.kw = kp / 4;
        g.wa[0] = g.wa[1] = g.wb[0] = g.wb[1] = -1;
        int k = 0;
        for (auto& pr : pairs) { g.wa[k] = (int16_t)pr[0]; g.wb[k] = (int16_t)pr[1]; g.lk[k] = (uint32_t)pr[2]; ++k; }
    };
    if (rows_m) seg(c->svd_f64[0] + rr0[0] * M, rows_m, M, rp_m, kpM, c->digA, {{0, 2, (int)lkM}});
    seg(c->svd_f64[2], M, M, rp_v, kpM, c->digB, {{0, 2, (int)lkM}, {2, 2, (int)lkM}});
    seg(c->svd_f64[1], N, N, rp_u, kpN, c->digC, {{1, 1, (int)lkN}});
    {
        ProfScope ps(c, pst, "k_residues_f64",
                     8.0 * ((double)rows_m * M + (double)M * M + (double)N * N), 0);
        hipck(launch_residues_f64(q, W, (int)c->P, pst), "k_residues_f64");
    }
    // the stages beside the products wait for the residue planes, which then
    // run alone instead of beside the first (HBM-saturating) stages (same box:
    // 512^2 0.427 -> 0.422 ms, 1024^2 2.098 -> 2.072 ms, 8-way rank 0.36 -> 0.35)
    // ("res_wait" 0, pipelined with every load read from the f64 inputs: the
    // stages need nothing of this chain before the products, so st2 goes on
    // without waiting for the residue planes; -1: so on unsharded contexts,
    // tools/ab.py r6f: 512^2 0.378 -> 0.371 ms, 1024^2 2.035 -> 2.026 ms, while
    // the 8-way rank's chain is better served by the wait, 0.321 -> 0.327 ms)
    const bool rw = c->res_wait >= 0 ? c->res_wait != 0 : sharded(c);
    if (rw || !c->in_pipe || !c->f64_views || c->f64reg.empty())
        stream_dep(c, pst, pst != c->st ? c->st : c->st2);
    const uint8_t* P[3] = {(const uint8_t*)c->digA.p, (const uint8_t*)c->digC.p,
                           (const uint8_t*)c->digB.p};                 // A planes of m, u, v
    const uint32_t stride[3] = {rp_m, rp_u, rp_v}, kp[3] = {kpM, kpN, kpM}, lk[3] = {lkM, lkN, lkM};
    const int wa[3] = {0, 1, 2}, wb[3] = {2, 1, 2};
    // one launch each for the three GEMMs and combines (same box, tools/probes/probe_opts.sh:
    // 512^2 P=32 0.43 -> 0.41 ms, 1024^2 P=63 2.10 -> 2.07 ms; row-sharded ranks too)
    {
        // the three products in one GEMM launch and one combine launch (each its
        // own residue scratch): one step of the st2 chain instead of three
        CrtBatch b;
        memset(&b, 0, sizeof b);
        size_t rbytes[3], rtot = 0;
        for (int g = 0; g < 3; ++g) {
            rbytes[g] = crt_scratch_bytes(std::max<uint32_t>((uint32_t)(rr1[g] - rr0[g]), 1), B[g].cols);
            rtot += rbytes[g];
        }
        ensure_buf(c, c->crtR, rtot);
        size_t roff = 0;
        double bytes = 0, ops = 0;
        for (int g = 0; g < 3; ++g) {
            const uint32_t rows = (uint32_t)(rr1[g] - rr0[g]), cols = B[g].cols;
            if (rows) {
                const bool sym = !sharded(c) && g > 0;
                CrtJob& q = b.job[b.njobs++];
                q.Ar = P[g] + (g == 0 ? 0 : rr0[g] * (uint64_t)kp[g]);
                q.Br = g == 0 ? (const uint8_t*)c->digB.p : P[g];
                q.R = (uint8_t*)c->crtR.p + roff;
                q.out = cellp(c, phase, log[g] + rr0[g] * cols);
                q.bits_a = W + wa[g];
                q.bits_b = W + wb[g];
                q.ors = cols;
                q.ocs = 1;
                q.astride = stride[g];
                q.bstride = g == 0 ? rp_v : stride[g];
                q.kpad = kp[g];
                q.N = rows;
                q.M = cols;
                q.lk = lk[g];
                q.sym = sym;
                bytes += 32.0 * rows * cols;
                ops += (double)rows * cols * A[g].cols;
            }
            roff += rbytes[g];
        }
        c->gemm_batched = true;
        b.kern = c->gemm_kern >= 0 ? (uint32_t)c->gemm_kern : 0u;
        if (b.njobs) {
            ProfScope ps(c, pst, "k_gemm_crt:multi", bytes, ops);
            hipck(launch_gemm_crt_multi(b, pst), "k_gemm_crt_multi");
        }
        const hipEvent_t done = stream_dep(c, pst, nullptr);   // one completion point
        for (int g = 0; g < 3; ++g) {
            c->pre.push_back({log[g], done, pst});
            c->gemm_done.push_back(done);
        }
    }
}

// check_svd_phase0
static svdw_svd_payload check_svd_phase0(svdw_ctx* c, const svdw_mat& m, const svdw_mat& u,
                                         const svdw_mat& v, const svdw_vec& d, double err_svd,
                                         double err_u, uint32_t max_bits_d,
                                         const uint32_t* known_bits = nullptr,
                                         const unsigned* dev_bits = nullptr,
                                         bool dev_quantized = false) {
    REQUIRE(m.rows == u.rows, "check_svd_phase0: m.num_rows != u.num_rows");
    REQUIRE(m.cols == v.rows, "check_svd_phase0: m.num_col != v.num_rows");
    REQUIRE(u.rows == u.cols, "check_svd_phase0: u not square");
    REQUIRE(v.rows == v.cols, "check_svd_phase0: v not square");
    const uint32_t N = m.rows, M = m.cols, r = std::min(N, M);
    REQUIRE(d.len == r, "check_svd_phase0: d.len != min(N, M)");
    const uint32_t P = c->P;
    const uint32_t max_bits = max_bits_d + P;
    uint64_t n0[2], nl0[2];                               // stream state at entry (for the replay)
    for (int p = 0; p < 2; ++p) { n0[p] = c->ph[p].n; nl0[p] = c->ph[p].nl; }
    auto prelaunch = [&] {
        if (c->dry || !c->overlap || !known_bits || !c->pre.empty()) return;
        // The three products depend only on m, u, v: take their stream offsets
        // from a dry replay of this function and launch them now on st2, so the
        // integer GEMMs run under the HBM-bound check stages on st. Called after
        // the first check stage is queued, so the device is busy while the host
        // waits for the operand bit lengths.
        const bool on_device = dev_bits && c->gemm_impl == SVDW_GEMM_MFMA;
        if (!on_device) fetch_bits(c);
        // residue planes straight from svd_witness's f64 inputs (one launch for m,
        // u and v) when they are on the device and the CRT path applies
        const bool from_f64 = on_device && dev_quantized && c->res_f64 && c->gemm_crt &&
                              c->svd_f64[0] && c->svd_f64[1] && c->svd_f64[2] && N <= 8192 &&
                              M <= 8192;
        std::vector<uint64_t> key = {n0[0], n0[1], nl0[0], nl0[1], d.phase, d.len, d.off,
                                     (uint64_t)d.stride, f64_key(err_svd), f64_key(err_u), max_bits_d};
        for (const svdw_mat* x : {&m, &u, &v})
            key.insert(key.end(), {x->phase, x->rows, x->cols, x->off, (uint64_t)x->rs, (uint64_t)x->cs});
        std::vector<uint64_t> log;
        if (key == c->log_key) {
            log = c->log_val;
        } else {
            svdw_ctx plan;
            plan.P = c->P; plan.LB = c->LB;
            for (int p = 0; p < 2; ++p) { plan.ph[p].n = n0[p]; plan.ph[p].nl = nl0[p]; }
            plan.gemm_log = &log;
            check_svd_phase0(&plan, m, u, v, d, err_svd, err_u, max_bits_d, known_bits);
            REQUIRE(log.size() == 3, "internal: expected three products in check_svd_phase0");
            c->log_key = key;
            c->log_val = log;
        }
        svdw_mat ut = u, vt = v;
        std::swap(ut.rows, ut.cols); std::swap(ut.rs, ut.cs);
        std::swap(vt.rows, vt.cols); std::swap(vt.rs, vt.cs);
        // loads of m, u, v done: the quantization event when svd_witness recorded
        // one (the cell stream may already hold later stages), else st's position
        // products on the cell stream (prod_cell): already behind the loads there
        c->prod_on_cell = from_f64 && c->bits_pending && (c->prod_cell > 0 || (c->prod_cell < 0 && sharded(c)));
        hipStream_t pst = c->prod_on_cell ? c->st : c->st2;
        if (c->prod_on_cell) {
        } else if (c->bits_pending) {
            dep_wait(c, c->st2, c->ev_bits);
        } else {
            stream_dep(c, c->st, c->st2);
        }
        const svdw_mat A[3] = {m, u, v}, B[3] = {vt, ut, vt};
        const uint32_t ba[3] = {known_bits[0], known_bits[1], known_bits[2]};
        const uint32_t bb[3] = {known_bits[2], known_bits[1], known_bits[2]};
        (void)ba; (void)bb;
        const unsigned* sl[3] = {dev_bits, dev_bits ? dev_bits + 1 : nullptr,
                                 dev_bits ? dev_bits + 2 : nullptr};
        const unsigned* sa[3] = {sl[0], sl[1], sl[2]};
        const unsigned* sb[3] = {sl[2], sl[1], sl[2]};
        if (from_f64) {
            prelaunch_products_f64(c, A, B, log, m.phase, const_cast<unsigned*>(dev_bits), pst);   // (c->bits)
            c->prelaunched = true;
            host_mark(c, "products queued");
            return;
        }
        bool vplanes = false;                            // v's planes built (digB) on this rank
        for (int g = 0; g < 3; ++g) {
            // shard: rows [r0, r1) of the product only
            uint64_t r0 = 0, r1 = A[g].rows;
            if (sharded(c)) shard_rows(c, A[g].rows, &r0, &r1);
            const svdw_mat Ag = sharded(c) ? row_block(A[g], r0, r1) : A[g];
            Fr* outg = cellp(c, m.phase, log[g] + r0 * B[g].cols);
            // CRT: v's residue planes from m.v^T (covering v.v^T too) serve v.v^T:
            // as both operands unsharded (v.v^T symmetric), as the b operand when
            // the rows are sharded (u's planes go to digC so v's survive)
            const bool shd = sharded(c);
            if (r1 <= r0) {
                // nothing of this product on this rank
            } else if (on_device)
                gemm_exec(c, c->st2, Ag, B[g], outg, ~0u, ~0u, sa[g], sb[g], dev_quantized,
                          g == 0 ? sl[2] : nullptr, !shd && g == 2,
                          shd && g == 1 ? &c->digC : nullptr, shd && g == 2 && vplanes);
            else
                gemm_exec(c, c->st2, Ag, B[g], outg, ba[g], bb[g]);
            if (g == 0 && r1 > r0 && on_device) vplanes = true;
            c->pre.push_back({log[g], stream_dep(c, c->st2, nullptr), c->st2});
            c->gemm_done.push_back(c->pre.back().ev);
        }
        c->prelaunched = true;
        host_mark(c, "products queued");
    };
    prelaunch();
    // what goes aside on st2 (d checks, single constant cells) is read by no
    // later kernel: batched until the end of phase 0 (two launches)
    BatchScope aside(c, c->st2);
    if (!c->prelaunched) aside.close();
    {
        // The d checks (three latency-bound stages over r elements) depend on d
        // only: with the products queued ahead they go behind them on st2, off
        // the cell stream, which starts on the u / v bounds at once. Pipelined
        // (st2 then carries every stage of the call back to back, st3 phase 1),
        // on the cell stream behind the products, its least loaded stream.
        struct Swap {
            svdw_ctx* c;
            hipStream_t* other;
            Swap(svdw_ctx* cc, bool o, bool third) : c(cc), other(o ? (third ? &cc->st3 : &cc->st2) : nullptr) {
                if (other) std::swap(c->st, *other);
            }
            ~Swap() { if (other) std::swap(c->st, *other); }
            bool on() const { return other != nullptr; }
        };
        // (pipelined: where dchk_at puts them; st3 only when it exists)
        const int da = !c->in_pipe ? 1 : (c->dchk_at == 2 && !c->st3 ? 1 : c->dchk_at);
        Swap sw(c, c->overlap && known_bits && !c->dry && c->bits_pending && da != 0, da == 2);
        // d loaded -- unless every load these stages (and the bounds and u.d
        // queued behind them with the products on the cell stream) read comes
        // from the registered f64 inputs (f64_view): then st2 starts at once
        const bool from_f64 = c->f64_views && !c->f64reg.empty() && c->prod_on_cell;
        if (sw.on() && !from_f64) dep_wait(c, c->st, c->ev_bits);
        BatchScope bs(c);                   // (desc_order_range reads desc_order_sub: two launches)
        entries_less_than(c, d, max_bits);
        entries_in_desc_order(c, d, max_bits);
        bs.end();
        host_mark(c, "d checks queued");
    }
    // svd_witness's phase 1 on the third stream, enqueued as soon as the products
    // are (their offsets from the dry replay give the payload): with only the
    // first phase-0 stages queued ahead of it, the third stream starts early
    // instead of after the host has queued all of phase 0.
    auto early_phase1 = [&](int at) {
        const int p1_at = c->p1_at >= 0 ? c->p1_at
                                         : (!sharded(c) ? 1 : (c->shard_world >= 4 ? 0 : 3));
        if (!c->early_p1 || p1_at != at || !c->prelaunched || c->pre.size() != 3) return;
        svdw_mat t_u = u, t_v = v;
        std::swap(t_u.rows, t_u.cols); std::swap(t_u.rs, t_u.cs);
        std::swap(t_v.rows, t_v.cols); std::swap(t_v.rs, t_v.cs);
        const svdw_svd_payload pl{t_u, t_v, svdw_mat{m.phase, N, M, c->pre[0].off, (int64_t)M, 1},
                                  svdw_mat{m.phase, N, N, c->pre[1].off, (int64_t)N, 1},
                                  svdw_mat{m.phase, M, M, c->pre[2].off, (int64_t)M, 1}};
        // the products' bounds (|c_s| < 2^(bits_a + bits_b + lk)) before
        // honest_prover_mat_mul registers them: the c_s scans then size their
        // operand on the device (NaSpec) instead of falling back to full
        // Montgomery products (8-way shard rank: 81 -> 25 us)
        auto clog2 = [](uint32_t k) { uint32_t l = 0; while ((1ull << l) < k) ++l; return l; };
        c->prods.push_back({pl.m_times_vt, m, t_v, clog2(M)});
        c->prods.push_back({pl.u_times_ut, u, t_u, clog2(N)});
        c->prods.push_back({pl.v_times_vt, v, t_v, clog2(M)});
        auto f = std::move(c->early_p1);
        c->early_p1 = nullptr;
        f(pl);
    };
    early_phase1(0);
    // The u, v bounds and u.d read only the loaded matrices: one launch when
    // batched (stage_batch), after which phase 1 is queued (p1_at 1 or 2).
    // With the products on the cell stream they go on st2 instead (behind the
    // d checks, in the same batch), and the cell stream waits for them before
    // the diff, by when they are done.
    const bool pc = c->prod_on_cell && c->prelaunched;
    if (pc) std::swap(c->st, c->st2);
    BatchScope bs(c);
    const bool batched = bs.mine || pc;
    BigU unit = big_from_u128(((unsigned __int128)1 << P) + 1);
    check_mat_entries_bounded(c, u, unit);
    host_mark(c, "bounds(u) queued");
    if (!batched) early_phase1(1);
    check_mat_entries_bounded(c, v, unit);
    host_mark(c, "bounds(v) queued");
    if (!batched) early_phase1(2);
    svdw_mat ut = u, vt = v;
    std::swap(ut.rows, ut.cols); std::swap(ut.rs, ut.cs);
    std::swap(vt.rows, vt.cols); std::swap(vt.rs, vt.cs);
    DView udv;
    EqCell udpad;
    // products on the cell stream: u.d (all the diff needs from st2) in a launch
    // ahead of the bounds, so the cell stream waits for it alone (pipelined, the
    // diff follows on st2 itself: u.d shares the bounds' launch)
    if (r == M) {
        c->stage_front = pc && !c->in_pipe;
        const svdw_mat ud = mat_times_diag_mat(c, u, d);
        c->stage_front = false;
        udv = view_of(c, ud);
    } else {
        const svdw_vec z = put_cell(c, 0 + u.phase, fr_zero(), true);   // zero padding constant
        udpad = EqCell{(int)z.phase, z.off};
        svdw_mat ud = mat_times_diag_mat(c, u, d);
        udv = view_of(c, ud);
        udv.cols = r;                                     // columns >= N read as 0
    }
    udv.rows = N;
    bs.end();
    if (pc) {
        std::swap(c->st, c->st2);
        // the cell stream waits for u.d (and what precedes it on st2), not for
        // the d checks' dependent second group batched behind it; pipelined,
        // the diff is on st2 itself and st carries the next call: no wait
        flush_batch(c, c->st2, c->in_pipe ? nullptr : c->st);
    }
    if (batched) {
        host_mark(c, "bounds(u), bounds(v), u.d queued");
        early_phase1(1);
        early_phase1(2);
    }
    uint32_t bm = ~0u, bu = ~0u, bv = ~0u;
    if (known_bits && c->pre.empty()) {                  // products not launched ahead
        fetch_bits(c);
        bm = known_bits[0]; bu = known_bits[1]; bv = known_bits[2];
    }
    // products batched (one completion point): diff and the two ids in one launch;
    // pipelined (c->in_pipe), on st2 behind the bounds, so that st is free for
    // the next call's product chain (honest_prover_mat_mul's wait for the
    // products lands on st2)
    const bool dst2 = c->in_pipe && pc;
    if (dst2) std::swap(c->st, c->st2);
    BatchScope bs2(c);
    if (!c->gemm_batched) bs2.close();
    svdw_mat mvt = honest_prover_mat_mul(c, m.phase, m, vt, bm, bv);
    BigU es = scale_err(err_svd, P), eu = scale_err(err_u, P);
    host_mark(c, "u.d queued");
    check_mat_diff_views(c, m.phase, udv, view_of(c, mvt), N, M, es, nullptr, udpad);
    host_mark(c, "diff queued");
    Fr q = pow2_fr(P);
    const Fr qq = fr_mul(q, q);
    svdw_vec q2 = put_cell(c, m.phase, qq, true);
    svdw_mat uut = honest_prover_mat_mul(c, m.phase, u, ut, bu, bu);
    check_mat_id(c, uut, q2, eu, &qq);
    svdw_mat vvt = honest_prover_mat_mul(c, m.phase, v, vt, bv, bv);
    check_mat_id(c, vvt, q2, eu, &qq);
    bs2.end();
    if (dst2) std::swap(c->st, c->st2);
    aside.end();
    host_mark(c, "ids queued");
    return svdw_svd_payload{ut, vt, mvt, uut, vvt};
}
static void check_svd_phase1(svdw_ctx* c, const svdw_mat& m, const svdw_mat& u, const svdw_mat& v,
                             const svdw_svd_payload& pl, const Fr& g) {
    const VMul vm[3] = {{m, pl.v_t, pl.m_times_vt}, {u, pl.u_t, pl.u_times_ut},
                        {v, pl.v_t, pl.v_times_vt}};
    verify_mul_many(c, 1, vm, 3, g);
}

// A witness call's side streams start after everything queued on st (the
// previous call's work joins st at its end): without this, the next call's
// gamma tables (st3) and first stages (st2, f64 views need no load) could
// overwrite buffers the previous call's kernels still read.
static void after_previous(svdw_ctx* c) {
    if (c->dry) return;
    const hipEvent_t e = stream_dep(c, c->st, c->st2);
    if (c->st3) dep_wait(c, c->st3, e);
    c->xwait_side = nullptr;                      // (st waited for the caller's stream)
}
static svdw_counts svd_witness(svdw_ctx* c, const double* m, const double* u, const double* v,
                               const double* d, uint32_t N, uint32_t M, bool on_device,
                               const svdw_svd_config& cfg, const Fr& gamma) {
    REQUIRE(N >= 1 && M >= 1, "empty matrix");
    const uint32_t r = std::min(N, M);
    c->ht0 = std::chrono::steady_clock::now();
    host_mark(c, "svd_witness start");
    clear_streams(c);
    c->dep_next = 0;
    c->prelaunched = false;
    c->prod_on_cell = false;
    c->gemm_batched = false;
    c->gemm_done.clear();
    c->wait_before_cs.clear();
    c->pre.clear();
    c->pre_wait_st = nullptr;
    c->pre_wait_ev = nullptr;
    c->in_pipe = false;
    struct PipeGuard {                     // an exception inside a pipelined call: its
        svdw_ctx* c;                       // tail is whatever reached st2 / st3 -- join it
        ~PipeGuard() {
            if (!c->in_pipe) return;
            const int par = c->pipe_par;
            (void)hipEventRecord(c->tail_ev[par][0], c->st2);
            (void)hipEventRecord(c->tail_ev[par][1], c->st3);
            c->tail_valid[par] = true;
            c->tail_pending = true;
            c->tail_last = par;
            c->pipe_par ^= 1;
            c->in_pipe = false;
        }
    } pguard{c};
    if (!c->dry) {
        // exact sizes from the dry planner: no growth copies inside the step
        const std::vector<uint64_t> key = {N, M, cfg.max_bits_d, f64_key(cfg.max_norm),
                                           f64_key(cfg.eps_svd), f64_key(cfg.eps_u), c->rlc_prefix};
        if (key != c->plan_key) {
            svdw_ctx plan;
            plan.P = c->P; plan.LB = c->LB;
            plan.rlc_prefix = c->rlc_prefix;
            svd_witness(&plan, nullptr, nullptr, nullptr, nullptr, N, M, false, cfg, gamma);
            c->plan_key = key;
            c->plan_val = {plan.ph[0].n, plan.ph[0].nl, plan.ph[1].n, plan.ph[1].nl};
        }
        // Pipelined (svd_witness_pipe): device inputs on the f64 product path
        // with the products on the cell stream, and two cell sets that fit in
        // at most 60 % of the device memory (1024^2 P=63: 2 x 9.3 GB; 4096^2
        // P=63, 2 x 148 GB, runs unpipelined)
        const double wbytes = 32.0 * (double)(c->plan_val[0] + c->plan_val[1] + c->plan_val[2] + c->plan_val[3]);
        const bool qualifies = c->pipeline && on_device && c->overlap && c->res_f64 && c->gemm_crt &&
                               c->gemm_impl == SVDW_GEMM_MFMA && N <= 8192 && M <= 8192 &&
                               (c->prod_cell > 0 || (c->prod_cell < 0 && sharded(c)));
        // The other cell set must already hold this witness, or its growth must
        // fit in the device's free memory now (other contexts, the lane's state
        // and torch's allocations count) with 10 % of the device to spare for
        // scratch; else the call runs unpipelined and the set is released.
        bool fits = qualifies;
        if (qualifies) {
            const double need = wbytes - set_bytes(c->alt);
            if (need > 0) {
                size_t fr = 0, tot = 0;
                hipck(hipMemGetInfo(&fr, &tot), "hipMemGetInfo");
                fits = need + 0.1 * (double)tot <= (double)fr;
            }
        }
        if (qualifies && !fits) release_alt(c);
        c->in_pipe = fits;
        if (c->in_pipe) {
            // the other cell set (last written by call j - 2): every stream waits
            // for that call's tail, the last reader of these cells and bit words
            // (st2's first stages write cells that call's st3 scans read)
            for (int p = 0; p < 2; ++p) std::swap(c->ph[p], c->alt[p]);
            std::swap(c->gpc, c->gpc_alt);        // (call j - 1's scans still read the others)
            std::swap(c->gtab, c->gtab_alt);
            clear_streams(c);
            // (tail_ev[.][0] was recorded on st2, [.][1] on st3: a stream does not
            // wait for its own earlier work)
            if (c->tail_valid[c->pipe_par])
                for (hipStream_t t : {c->st, c->st2, c->st3})
                    for (int k = 0; k < 2; ++k)
                        if (t != (k ? c->st3 : c->st2))
                            hipck(hipStreamWaitEvent(t, c->tail_ev[c->pipe_par][k], 0), "hipStreamWaitEvent");
            if (c->xwait_side) {                  // the caller's stream (svdw_stream_wait)
                for (hipStream_t t : {c->st2, c->st3})
                    hipck(hipStreamWaitEvent(t, c->xwait_side, 0), "hipStreamWaitEvent");
                c->xwait_side = nullptr;
            }
        } else {
            settle(c);
            after_previous(c);
        }
        auto grow_set = [&] {
            for (int p = 0; p < 2; ++p) {
                grow(c, c->ph[p].adv, 0, c->ph[p].cap, c->plan_val[2 * p]);
                grow(c, c->ph[p].lk, 0, c->ph[p].lcap, c->plan_val[2 * p + 1]);
            }
        };
        if (!c->in_pipe) {
            grow_set();
        } else {
            try {
                grow_set();
            } catch (const SvdwError& e) {
                if (e.code != SVDW_ENOMEM) throw;
                // the other set could not be allocated after all: back to this
                // set, unpipelined (the waits already queued are harmless)
                for (int p = 0; p < 2; ++p) std::swap(c->ph[p], c->alt[p]);
                std::swap(c->gpc, c->gpc_alt);
                std::swap(c->gtab, c->gtab_alt);
                c->in_pipe = false;
                release_alt(c);
                clear_streams(c);
                settle(c);
                after_previous(c);
                grow_set();
            }
        }
    }
    // examples/svd_example.rs:183-184 run rlc.load_rlc_cache((ctx_gate, ctx_rlc), gate, 1)
    // on the phase-1 pair before check_svd_phase1. As recalled from axiom-eth's
    // RlcChip (un-vendored; parity unpinned), an empty cache loads gamma as
    // compute_rlc_fixed_len(ctx_rlc, [one, zero]) with one = ctx_gate.load_constant(1),
    // zero = ctx_gate.load_zero(): two constant cells at the head of ctx_gate (the
    // stream here); [E(one), E(zero), W(gamma)] go to ctx_rlc, whose cell 2 is init_rand.
    c->ext_off = 0;
    c->rlc.n = 0;
    if (c->rlc_prefix) {
        const svdw_vec one = put_cell(c, 1, fr_from_u64(1), true);
        const svdw_vec zero = put_cell(c, 1, fr_zero(), true);
        c->ext_off = 2;
        c->rlc.n = 3;
        c->rlc.cells[0] = fr_from_u64(1);
        c->rlc.cells[1] = fr_zero();
        c->rlc.cells[2] = gamma;
        c->rlc.src[0] = (uint64_t)one.phase << 62 | one.off;
        c->rlc.src[1] = (uint64_t)zero.phase << 62 | zero.off;
    }
    c->gp_ev = nullptr;
    if (!c->dry && c->hold_us) {       // every stream of the step waits for st's hold
        hipck(launch_hold(c->hold_us, c->st), "k_hold");
        stream_dep(c, c->st, c->st3);
        stream_dep(c, c->st, c->st2);  // (st2's first stages need no load with f64 views)
    }
    if (!c->dry) {
        // gamma^j depends on gamma only: queue it first, on its own stream, so it
        // runs beside quantization instead of on the phase-1 chain (pipelined: on
        // the cell stream, the least loaded one, into this parity's tables)
        const bool g3 = c->gamma_at == 1 || (c->gamma_at < 0 && sharded(c));
        hipStream_t gs = c->in_pipe && !(g3 && c->st3) ? c->st_cell : c->st3;
        gamma_prep(c, std::max(N, M), gamma, gs);
        c->gp_ev = stream_dep(c, gs, nullptr);
        c->gp_st = gs;
        host_mark(c, "gamma_prep queued");
    }
    unsigned* dbits = nullptr;
    // m: only this rank's rows are quantized on a row-sharded rank (zkmatrix_new)
    uint64_t mr0 = 0, mr1 = N;
    if (sharded(c) && on_device) shard_rows(c, N, &mr0, &mr1);
    // (host inputs go through launch_quantize, kQuantPerBlock values per block)
    const uint32_t qpb = on_device ? quant_per_block((mr1 - mr0) * M + (uint64_t)N * N + (uint64_t)M * M + r)
                                   : kQuantPerBlock;
    const uint32_t nbm = (uint32_t)(((mr1 - mr0) * M + qpb - 1) / qpb);
    const uint32_t nbu = (uint32_t)(((uint64_t)N * N + qpb - 1) / qpb);
    const uint32_t nbv = (uint32_t)(((uint64_t)M * M + qpb - 1) / qpb);
    if (!c->dry) {
        // [0, 3): bit-length maxima of m, u, v; from word 64: per-block maxima
        // (pipelined: a half per parity, call j - 1's row scans still read theirs)
        const size_t words = (64 + nbm + nbu + nbv + 63) / 64 * 64;
        ensure_buf(c, c->bits, 2 * words * sizeof(unsigned));
        dbits = (unsigned*)c->bits.p + (c->in_pipe ? c->pipe_par * words : 0);
    }
    QuantSegs qs;
    memset(&qs, 0, sizeof qs);
    qs.per_block = qpb;
    QuantSegs* qp = &qs;
    svdw_mat zm = zkmatrix_new(c, 0, m, N, M, on_device, dbits ? dbits + 64 : nullptr, qp, true);
    // (u, v: the rank's rows and column block only, when b.g comes from the f64
    // inputs and so do the products' residue planes: no kernel reads the rest;
    // the conditions of f64_of and of check_svd_phase0's from_f64 prelaunch)
    const bool part = sharded(c) && on_device && N <= 8192 && M <= 8192 && c->overlap && c->res_f64 &&
                      c->gemm_crt && c->gemm_impl == SVDW_GEMM_MFMA;
    svdw_mat zu = zkmatrix_new(c, 0, u, N, N, on_device, dbits ? dbits + 64 + nbm : nullptr, qp, false, part);
    svdw_mat zv = zkmatrix_new(c, 0, v, M, M, on_device, dbits ? dbits + 64 + nbm + nbu : nullptr, qp, false,
                               part);
    svdw_mat zdm = zkmatrix_new(c, 0, d, r, 1, on_device, nullptr, qp);
    BitSegs seg{};
    seg.begin[0] = 0;
    seg.begin[1] = nbm;
    seg.begin[2] = nbm + nbu;
    seg.begin[3] = nbm + nbu + nbv;
    bool folded = false;
    bits_words(c, qs, 3, seg, dbits, &folded);
    // (Round 4 measured the quantization beside the product chain instead: the
    // bit-length words from a read-only k_bits_f64 on st, the cells on st2; it
    // was 0.7-4 % slower at 1024^2, 512^2 and on 8-way ranks -- the words'
    // cross-block reduction costs what the cells' stores did -- and was removed.)
    if (qs.nseg) {
        ProfScope ps(c, c->st, "k_quantize", 40.0 * ((double)N * M + (double)N * N + (double)M * M + r), 0);
        hipck(launch_quantize_multi(qs, (int)c->P, c->st), "k_quantize_multi");
    }
    svdw_vec zd{0, r, zdm.off, 1};
    double es, eu;
    err_calc(c->P, std::max(N, M), cfg.max_norm, cfg.eps_svd, cfg.eps_u, &es, &eu);
    if (!c->dry) {   // operand bit lengths (GEMM digit counts): read lazily, see fetch_bits
        if (!folded) hipck(launch_bits_reduce(dbits + 64, seg, 3, dbits, c->st), "k_bits_reduce");
        flush_batch(c, c->st);
        hipck(hipEventRecord(c->ev_bits, c->st), "hipEventRecord");
        c->bits_pending = true;
        c->qmat[0] = zm; c->qmat[1] = zu; c->qmat[2] = zv;
        // the same words for the device-side choices (row-scan operand widths)
        c->dbitw = dbits;
        c->dwords = {{zm, 0}, {zu, 1}, {zv, 2}};
        host_mark(c, "quantize + bits queued");
    }
    // Phase 1 needs only the products (queued on st2 by check_svd_phase0), the
    // quantized operands and gamma: run it on st2 behind the GEMMs, concurrently
    // with the HBM-bound phase-0 checks still on st (its row scans are
    // VALU-bound), and join the streams afterwards.
    // Mode 2: on a third stream that starts after quantization; the b.g and
    // a.(b.g) scans run at once, the c_s.g scans wait for the products; queued
    // from inside check_svd_phase0 right after its first stage (p1_at).
    // Mode 1 on a row-sharded rank becomes mode 2: there the products are only a
    // row block, the st2 chain (products + phase 1) is the critical path and the
    // operand-only scans fit beside the products (tools/shard_sim.py, 8 ranks:
    // 0.62 -> 0.54 ms). So does a small witness (max(N, M) < 1024), where the
    // st2 chain is also the critical path (tools/ab.py: 512^2 P=32 0.559 ->
    // 0.454 ms, 768^2 P=63 1.328 -> 1.272 ms); from 1024 on it is neutral to
    // 1 % slower.
    const bool p1_small = std::max(N, M) < 1024;
    // (pipelined: st2 carries the diff and ids after the bounds, phase 1 goes to st3)
    const int p1mode = c->phase1_overlap == 1 && (sharded(c) || p1_small || c->in_pipe) ? 2 : c->phase1_overlap;
    bool p1_queued = false;
    auto queue_phase1 = [&](const svdw_svd_payload& pl, bool overlap) {
        const bool p1_overlap = p1mode && overlap;
        hipStream_t p1s = p1mode == 2 ? c->st3 : c->st2;
        // phase 1 beside the products (st3, or st2 while the products run on the
        // cell stream): it waits for the loads, and its c_s scans for the products
        if (p1_overlap && (p1s == c->st3 || c->prod_on_cell)) {
            dep_wait(c, p1s, c->ev_bits);
            c->wait_before_cs = c->gemm_done;
        }
        {
            struct Swap {
                svdw_ctx* c;
                hipStream_t* other;
                Swap(svdw_ctx* cc, hipStream_t* o) : c(cc), other(o) { if (other) std::swap(c->st, *other); }
                ~Swap() { if (other) std::swap(c->st, *other); }
            } sw(c, p1_overlap ? (p1s == c->st3 ? &c->st3 : &c->st2) : nullptr);
            check_svd_phase1(c, zm, zu, zv, pl, gamma);
        }
        c->wait_before_cs.clear();
        p1_queued = true;
        host_mark(c, "phase 1 (early) queued");
    };
    struct Clear {
        svdw_ctx* c;
        ~Clear() { c->early_p1 = nullptr; }
    } clr{c};
    if (p1mode == 2 && !c->dry) c->early_p1 = [&](const svdw_svd_payload& pl) { queue_phase1(pl, true); };
    struct F64 {
        svdw_ctx* c;
        ~F64() {
            c->svd_f64[0] = c->svd_f64[1] = c->svd_f64[2] = nullptr;
            c->f64src.clear();
            c->f64reg.clear();
        }
    } f64clr{c};
    if (on_device && !c->dry) {
        c->svd_f64[0] = m; c->svd_f64[1] = u; c->svd_f64[2] = v;
        c->f64src = {{zu, u}, {zv, v}};
        c->f64reg = {{zm.phase, zm.off, (uint64_t)N * M, m}, {zu.phase, zu.off, (uint64_t)N * N, u},
                     {zv.phase, zv.off, (uint64_t)M * M, v}, {zdm.phase, zdm.off, (uint64_t)r, d}};
    }
    svdw_svd_payload pl =
        check_svd_phase0(c, zm, zu, zv, zd, es, eu, cfg.max_bits_d, c->qbits, dbits, true);
    c->early_p1 = nullptr;
    const bool p1_overlap = p1mode && c->prelaunched && !c->dry;
    hipStream_t p1s = p1mode == 2 ? c->st3 : c->st2;
    host_mark(c, "phase 0 queued");
    if (!p1_queued) queue_phase1(pl, p1_overlap);
    host_mark(c, "phase 1 queued");
    if (c->in_pipe) {
        // no join into st: the next call's product chain starts on st while this
        // call's stages (st2) and row scans (st3) finish; they end at tail_ev
        const int par = c->pipe_par;
        flush_batch(c, c->st2);
        flush_batch(c, c->st3);
        hipck(hipEventRecord(c->tail_ev[par][0], c->st2), "hipEventRecord");
        hipck(hipEventRecord(c->tail_ev[par][1], c->st3), "hipEventRecord");
        c->tail_valid[par] = true;
        c->tail_pending = true;
        c->tail_last = par;
        c->pipe_par ^= 1;
        c->in_pipe = false;
        host_mark(c, "svd_witness end (pipelined)");
        return svdw_counts{c->ph[0].n, c->ph[1].n, c->ph[0].nl, c->ph[1].nl};
    }
    if (p1_overlap) stream_dep(c, p1s, c->st);
    // st2 also carries the d checks and single cells queued aside (and, with
    // phase 1 on st3, nothing else joins it): join it too
    if (c->prelaunched && !c->dry && !(p1_overlap && p1s == c->st2)) stream_dep(c, c->st2, c->st);
    host_mark(c, "svd_witness end");
    return svdw_counts{c->ph[0].n, c->ph[1].n, c->ph[0].nl, c->ph[1].nl};
}

// README.md:32-46 as one call: ZkMatrix::new(a), ZkMatrix::new(b), c_s =
// honest_prover_mat_mul(a, b) into phase 0, verify_mul(a, b, c_s, gamma) into
// phase 1 -- the modular calls' cells, enqueued without host waits: a and b
// quantized in one launch, the GEMM's modulus count and the row scans' operand
// widths decided on the device from the bit-length words, gamma^j prepared
// first on the side stream.
// verify_mul_witness's phase 1 opens with verify_mul's one cell and its d - 1
// gamma-power elements (verify_mul_many's first appends at phase-1 offsets 0
// and 1): k_gamma_prep writes them when the phase-1 stream holds them
static bool vm_pow_cells(svdw_ctx* c, uint32_t M, const Fr& gamma, PowCells* pc) {
    memset(pc, 0, sizeof *pc);
    if (M <= 1 || c->ph[1].cap < 1 + 4ull * (M - 1)) return false;
    pc->one = cellp(c, 1, 0);
    pc->pows = cellp(c, 1, 1);
    pc->d = M;
    pc->gamma = gamma;
    return true;
}
static svdw_counts verify_mul_witness(svdw_ctx* c, const double* a, const double* b, uint32_t N,
                                      uint32_t K, uint32_t M, bool on_device, const Fr& gamma) {
    REQUIRE(N >= 1 && K >= 1 && M >= 1, "empty matrix");
    REQUIRE(!sharded(c), "verify_mul_witness: not for row-sharded contexts");
    c->ht0 = std::chrono::steady_clock::now();
    host_mark(c, "verify_mul_witness start");
    clear_streams(c);
    c->dep_next = 0;
    settle(c);
    after_previous(c);
    c->prelaunched = false;
    c->prod_on_cell = false;
    c->gemm_batched = false;
    c->gemm_done.clear();
    c->wait_before_cs.clear();
    c->pre.clear();
    c->pre_wait_st = nullptr;
    c->pre_wait_ev = nullptr;
    if (!c->dry) {
        const std::vector<uint64_t> key = {0x766d77ull, N, K, M};      // sizes from the dry plan
        if (key != c->plan_key) {
            svdw_ctx plan;
            plan.P = c->P; plan.LB = c->LB;
            verify_mul_witness(&plan, nullptr, nullptr, N, K, M, false, gamma);
            c->plan_key = key;
            c->plan_val = {plan.ph[0].n, plan.ph[0].nl, plan.ph[1].n, plan.ph[1].nl};
        }
        for (int p = 0; p < 2; ++p) {
            grow(c, c->ph[p].adv, 0, c->ph[p].cap, c->plan_val[2 * p]);
            grow(c, c->ph[p].lk, 0, c->ph[p].lcap, c->plan_val[2 * p + 1]);
        }
    }
    c->ext_off = 0;
    c->gp_ev = nullptr;
    if (!c->dry && c->hold_us) {       // every stream of the step waits for st's hold
        hipck(launch_hold(c->hold_us, c->st), "k_hold");
        stream_dep(c, c->st, c->st3);
        stream_dep(c, c->st, c->st2);
    }
    host_mark(c, "plan + gamma_prep queued");
    unsigned* dbits = nullptr;
    const uint32_t qpb = on_device ? quant_per_block((uint64_t)N * K + (uint64_t)K * M) : kQuantPerBlock;
    const uint32_t nba = (uint32_t)(((uint64_t)N * K + qpb - 1) / qpb),
                   nbb = (uint32_t)(((uint64_t)K * M + qpb - 1) / qpb);
    c->pows_pre.on = false;
    if (!c->dry) {
        // phase 1 opens with verify_mul's one cell and its d - 1 gamma-power
        // elements (verify_mul_many's first appends): k_gamma_prep writes them
        PowCells pc;
        // (queued ahead: only if that launch wrote them where they are now)
        if (c->ph[1].n == 0 && vm_pow_cells(c, M, gamma, &pc) && (!c->gp_external || c->gp_ext_one == pc.one))
            c->pows_pre = {true, 0, 1, M};
        if (c->gp_external) {                         // queued on st ahead of the captured graph
            c->gp_gamma = gamma;
            c->gp_len = std::max(M, 1u);
        } else {
            gamma_prep(c, M, gamma, c->st3, pc.one ? &pc : nullptr);
        }
        c->gp_ev = stream_dep(c, c->st3, nullptr);
        c->gp_st = c->st3;
        ensure_buf(c, c->bits, (64 + nba + nbb) * sizeof(unsigned));
        dbits = (unsigned*)c->bits.p;
    }
    QuantSegs qs;
    memset(&qs, 0, sizeof qs);
    qs.per_block = qpb;
    QuantSegs* qp = on_device ? &qs : nullptr;
    const svdw_mat za = zkmatrix_new(c, 0, a, N, K, on_device, dbits ? dbits + 64 : nullptr, qp);
    const svdw_mat zb = zkmatrix_new(c, 0, b, K, M, on_device, dbits ? dbits + 64 + nba : nullptr, qp);
    BitSegs seg{};
    seg.begin[0] = 0;
    seg.begin[1] = nba;
    seg.begin[2] = nba + nbb;
    bool folded = false;
    bits_words(c, qs, 2, seg, dbits, &folded);
    // (quantization stays on the chain here: beside it on st2, config 2 measured
    // 0.091-0.096 -> 0.106 ms, host-bound, round 4)
    if (qs.nseg) {
        ProfScope ps(c, c->st, "k_quantize", 40.0 * ((double)N * K + (double)K * M), 0);
        hipck(launch_quantize_multi(qs, (int)c->P, c->st), "k_quantize_multi");
    }
    if (!c->dry) {
        if (!folded) hipck(launch_bits_reduce(dbits + 64, seg, 2, dbits, c->st), "k_bits_reduce");
        c->dbitw = dbits;
        c->dwords = {{za, 0}, {zb, 1}};
    }
    host_mark(c, "quantize queued");
    struct RegClear {
        svdw_ctx* c;
        ~RegClear() { c->f64reg.clear(); }
    } regclr{c};
    if (on_device && !c->dry)
        c->f64reg = {{za.phase, za.off, (uint64_t)N * K, a}, {zb.phase, zb.off, (uint64_t)K * M, b}};
    // c_s = a * b (honest_prover_mat_mul's cells), the CRT GEMM sized on the device
    uint64_t off;
    append(c, 0, (uint64_t)N * M, 0, &off, nullptr, "product", N);
    const svdw_mat cs{0, N, M, off, (int64_t)M, 1};
    {
        uint32_t lk = 0;
        while ((1ull << lk) < K) ++lk;
        c->prods.push_back({cs, za, zb, lk});
    }
    // device inputs: residue planes of a and b^T straight from the f64 inputs
    // (one launch), the GEMM and combine on st, and verify_mul on the third
    // stream from the loads on: its one / gamma-power cells and the b and a
    // scans run beside the product, only the c_s scans wait for it
    const bool f64 = on_device && !c->dry && c->res_f64 && c->gemm_crt && c->gemm_impl == SVDW_GEMM_MFMA &&
                     K <= 8192 && qs.nseg == 2;
    hipEvent_t loaded = nullptr;
    if (f64) {
        loaded = stream_dep(c, c->st, nullptr);
        uint32_t lk = 0;
        while ((1ull << lk) < K) ++lk;
        const uint32_t kpad = (K + 255) / 256 * 256, rpa = (N + 127) / 128 * 128, rpb = (M + 127) / 128 * 128;
        ensure_buf(c, c->digA, (size_t)kCrtMaxResidues * rpa * kpad);
        ensure_buf(c, c->digB, (size_t)kCrtMaxResidues * rpb * kpad);
        ensure_buf(c, c->crtR, crt_scratch_bytes(N, M));
        ResSegs q;
        memset(&q, 0, sizeof q);
        auto seg = [&](const double* in, uint32_t rows, uint32_t ld, uint32_t rp, DBuf& out, uint32_t tr) {
            ResSeg& g = q.seg[q.nseg++];
            g.in = in; g.out = (uint32_t*)out.p;
            g.rows = rows; g.cols = K; g.ld = ld; g.rows_pad = rp; g.kw = kpad / 4; g.tr = tr;
            g.wa[0] = 0; g.wb[0] = 1; g.lk[0] = lk;
            g.wa[1] = g.wb[1] = -1;
        };
        seg(a, N, K, rpa, c->digA, 0);
        seg(b, M, M, rpb, c->digB, 1);                    // b^T(j, k) = b[k * M + j]
        {
            ProfScope ps(c, c->st, "k_residues_f64", 8.0 * ((double)N * K + (double)K * M), 0);
            hipck(launch_residues_f64(q, dbits, (int)c->P, c->st), "k_residues_f64");
        }
        {
            ProfScope ps(c, c->st, "k_gemm_crt", 32.0 * N * M, (double)N * M * K);
            hipck(launch_gemm_crt(false, (const uint8_t*)c->digA.p, (const uint8_t*)c->digB.p, N, M, rpa, rpb,
                                  kpad, (uint8_t*)c->crtR.p, cellp(c, 0, off), M, 1, dbits, dbits + 1, lk,
                                  c->st, c->gemm_kern >= 0 ? (uint32_t)c->gemm_kern : 0u),
                  "k_gemm_crt");
        }
    } else if (!c->dry) {
        gemm_exec(c, c->st, za, zb, cellp(c, 0, off), ~0u, ~0u, dbits, dbits + 1, true);
    }
    host_mark(c, "product queued");
    const VMul vm{za, zb, cs};
    if (f64) {
        c->wait_before_cs = {stream_dep(c, c->st, nullptr)};
        dep_wait(c, c->st3, loaded);
        std::swap(c->st, c->st3);
        try {
            verify_mul_many(c, 1, &vm, 1, gamma);
        } catch (...) {
            std::swap(c->st, c->st3);
            c->wait_before_cs.clear();
            throw;
        }
        std::swap(c->st, c->st3);
        c->wait_before_cs.clear();
        stream_dep(c, c->st3, c->st);                     // join
    } else {
        verify_mul_many(c, 1, &vm, 1, gamma);
    }
    host_mark(c, "verify_mul_witness end");
    return svdw_counts{c->ph[0].n, c->ph[1].n, c->ph[0].nl, c->ph[1].nl};
}

// ---------------------------------------- captured verify_mul_witness (graph)
// A device-input verify_mul_witness enqueues ~20 HIP calls for a GPU step of
// ~70 us at 256^2 (BASELINE config 2), so the host bounds it. Every call of
// one key (shape, input pointers, buffer epoch) enqueues the same launches:
// nothing in it waits for the device, and gamma reaches the device only as
// k_gamma_prep's tables. So k_gamma_prep goes out eagerly on st (by value),
// the rest is captured once (on the second call of a key, when every buffer
// is sized) and replayed with one hipGraphLaunch; the host state the call
// leaves (layout, checks, counts) is restored from the capture, with gamma
// patched into the constants that hold it.
static void vmg_drop(svdw_ctx* c) {
    if (c->vmg.exec) (void)hipGraphExecDestroy(c->vmg.exec);
    c->vmg.exec = nullptr;
    c->vmg.key.clear();
}
static void vmg_snapshot(svdw_ctx* c, const svdw_counts& k) {
    auto& g = c->vmg;
    g.layout = c->layout;
    g.layout_chk = c->layout_chk;
    g.consts = c->consts;
    g.gamma_slots = c->gamma_slots;
    g.mbits = c->mbits;
    g.prods = c->prods;
    g.dwords = c->dwords;
    g.dbitw = c->dbitw;
    g.ext_off = c->ext_off;
    g.counts = k;
}
static svdw_counts vmg_restore(svdw_ctx* c, const Fr& gamma) {
    const auto& g = c->vmg;
    clear_streams(c);
    c->layout = g.layout;
    c->layout_chk = g.layout_chk;
    c->consts = g.consts;
    c->gamma_slots = g.gamma_slots;
    for (const auto& s : c->gamma_slots) c->layout_chk.at(s.first).eqk.at((size_t)s.second) = gamma;
    c->mbits = g.mbits;
    c->prods = g.prods;
    c->dwords = g.dwords;
    c->dbitw = g.dbitw;
    c->ext_off = g.ext_off;
    c->ext_gamma = gamma;
    c->ph[0].n = g.counts.advice0;
    c->ph[1].n = g.counts.advice1;
    c->ph[0].nl = g.counts.lookup0;
    c->ph[1].nl = g.counts.lookup1;
    return g.counts;
}
// Every scratch buffer of a state (release, footprint).
static std::vector<DBuf*> dbufs(svdw_ctx* c) {
    std::vector<DBuf*> v = {&c->f64in, &c->digA, &c->digB, &c->digC, &c->chk, &c->chkg, &c->gateq[0], &c->gateq[1],
                            &c->w1c, &c->w1t, &c->w2c, &c->w2t, &c->bits, &c->gpc, &c->gtab, &c->gpc_alt,
                            &c->gtab_alt, &c->crtR, &c->gbits, &c->colpart, &c->qfold, &c->ing_x, &c->ing_e,
                            &c->ing_c, &c->ing_p10, &c->ing_val, &c->ing_npos, &c->ing_nd, &c->ing_rpos,
                            &c->ing_kpos, &c->ing_err, &c->ing_q, &c->eq_cp, &c->eq_ks, &c->eq_reg, &c->eq_w,
                            &c->eq_k, &c->eq_err, &c->eq_st};
    for (int i = 0; i < kMaxScanJobs; ++i) {
        v.push_back(&c->wbc[i]);
        v.push_back(&c->wbt[i]);
        v.push_back(&c->bvfull[i]);
    }
    return v;
}
// Device bytes a state holds (cell sets and scratch).
static double state_bytes(svdw_ctx* c) {
    double b = set_bytes(c->ph) + set_bytes(c->alt);
    for (DBuf* d : dbufs(c)) b += (double)d->cap;
    return b;
}
// Every device object is released on its own (a state whose creation failed
// part-way holds some of them only).
static void ctx_release(svdw_ctx* c) {
    if (!c) return;
    if (c->lane) ctx_release(c->lane);
    if (!c->dry) {
        for (hipStream_t t : {c->st_cell ? c->st_cell : c->st, c->st2, c->st3})
            if (t) (void)hipStreamSynchronize(t);
        vmg_drop(c);
        for (auto& s : c->ph) { (void)hipFree(s.adv); (void)hipFree(s.lk); }
        for (auto& s : c->alt) { (void)hipFree(s.adv); (void)hipFree(s.lk); }
        for (auto& t : c->tail_ev)
            for (auto e : t)
                if (e) (void)hipEventDestroy(e);
        for (DBuf* b : dbufs(c))
            if (b->p) (void)hipFree(b->p);
        if (c->hbits) (void)hipHostFree(c->hbits);
        if (c->ev_bits) (void)hipEventDestroy(c->ev_bits);
        for (auto e : c->xev)
            if (e) (void)hipEventDestroy(e);
        for (auto& m : c->mk.ev)
            for (auto e : m)
                if (e) (void)hipEventDestroy(e);
        for (auto& r : c->recs) { (void)hipEventDestroy(r.e0); (void)hipEventDestroy(r.e1); }
        for (auto e : c->pool) (void)hipEventDestroy(e);
        for (auto e : c->deps) (void)hipEventDestroy(e);
        if (c->lin_ev) (void)hipEventDestroy(c->lin_ev);
        for (hipStream_t t : {c->st3, c->st2, c->st_cell ? c->st_cell : c->st})
            if (t) (void)hipStreamDestroy(t);
    }
    delete c;
}
// "lanes": may the next verify_mul_witness run on the other state? Yes when
// that state already holds as much device memory as this one (the calls have
// one shape), or when its growth to this one's footprint fits in free memory
// with 10 % of the device to spare; else the call stays on this state.
static bool lane_fits(svdw_ctx* c) {
    const double need = state_bytes(c) - (c->lane ? state_bytes(c->lane) : 0.0);
    if (need <= 0) return true;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
    return need + 0.1 * (double)tot <= (double)fr;
}
// Device state of a new context: its three streams, the pinned bit words, events.
static void ctx_init_device(svdw_ctx* c) {
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking);
    c->st_cell = c->st;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking);
    // the third stream exists from the start: one created lazily inside a
    // call would not wait for what st already waits for (svdw_stream_wait)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->st3, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->hbits, 64 * sizeof(uint32_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_bits, hipEventDisableTiming | hipEventReleaseToDevice);
    for (int k = 0; k < 4 && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&c->tail_ev[k / 2][k % 2], hipEventDisableTiming | hipEventReleaseToDevice);
    c->stream_id[0] = c->st;
    c->stream_id[1] = c->st2;
    c->stream_id[2] = c->st3;
    size_t mfree = 0;
    if (e == hipSuccess) e = hipMemGetInfo(&mfree, &c->mem_total);
    if (e != hipSuccess) fail(SVDW_EDEVICE, std::string("HIP device init failed: ") + hipGetErrorString(e));
}
// The settings (options, shard, profiler) of `s` onto the lane `d`; a change
// bumps the lane's epoch (its captured graph no longer applies).
static void copy_settings(svdw_ctx* d, const svdw_ctx* s) {
    const int64_t a[] = {s->gemm_impl, s->stage_flags, s->stage_elems, s->gemm_crt, s->gemm_kern, s->res_wait, s->place_trials, s->res_f64,
                         s->phase1_overlap, s->prod_cell, s->hold_us, s->rlc_prefix, s->p1_at, s->dchk_at, s->gamma_at,
                         s->f64_views, s->overlap, s->stage_batch, s->graph_vm, s->vm_linear, s->pipeline,
                         s->shard_rank, s->shard_world, s->prof, s->host_trace};
    const int64_t b[] = {d->gemm_impl, d->stage_flags, d->stage_elems, d->gemm_crt, d->gemm_kern, d->res_wait, d->place_trials, d->res_f64,
                         d->phase1_overlap, d->prod_cell, d->hold_us, d->rlc_prefix, d->p1_at, d->dchk_at, d->gamma_at,
                         d->f64_views, d->overlap, d->stage_batch, d->graph_vm, d->vm_linear, d->pipeline,
                         d->shard_rank, d->shard_world, d->prof, d->host_trace};
    if (!memcmp(a, b, sizeof a) && d->prof_filter == s->prof_filter) return;
    d->gemm_impl = s->gemm_impl; d->stage_flags = s->stage_flags; d->stage_elems = s->stage_elems;
    d->gemm_crt = s->gemm_crt; d->gemm_kern = s->gemm_kern; d->res_wait = s->res_wait; d->place_trials = s->place_trials; d->res_f64 = s->res_f64; d->phase1_overlap = s->phase1_overlap;
    d->prod_cell = s->prod_cell; d->hold_us = s->hold_us; d->rlc_prefix = s->rlc_prefix;
    d->p1_at = s->p1_at; d->f64_views = s->f64_views; d->overlap = s->overlap;
    d->dchk_at = s->dchk_at; d->gamma_at = s->gamma_at;
    d->stage_batch = s->stage_batch; d->graph_vm = s->graph_vm; d->pipeline = s->pipeline;
    d->vm_linear = s->vm_linear;
    d->shard_rank = s->shard_rank; d->shard_world = s->shard_world; d->prof = s->prof;
    d->host_trace = s->host_trace; d->prof_filter = s->prof_filter;
    ++d->epoch;
}
// "lanes": exchange this state with the lane's (created on first use).
static_assert(std::is_nothrow_move_constructible<svdw_ctx>::value && std::is_nothrow_move_assignable<svdw_ctx>::value, "svdw_ctx moves");
static void lane_switch(svdw_ctx* c) {
    if (!c->lane) {
        svdw_ctx* L = new svdw_ctx();
        L->P = c->P;
        L->LB = c->LB;
        L->device = c->device;
        L->dry = false;
        try {
            ctx_init_device(L);
        } catch (...) {
            ctx_release(L);
            throw;
        }
        c->lane = L;
    }
    svdw_ctx* L = c->lane;
    copy_settings(L, c);
    std::swap(*c, *L);
    std::swap(c->lane, L->lane);                  // (the handle keeps the lane and the option)
    std::swap(c->lanes, L->lanes);
    std::swap(c->mk, L->mk);
}
static hipEvent_t xevent(svdw_ctx* c, int i);
// caller: the caller's stream (svdw_verify_mul_witness_on), waited for by the
// state that runs the call (after the lane switch)
static svdw_counts verify_mul_witness_api(svdw_ctx* c, const double* a, const double* b, uint32_t N,
                                          uint32_t K, uint32_t M, bool on_device, const Fr& gamma,
                                          hipStream_t caller = nullptr, bool has_caller = false) {
    const bool plain = on_device && !c->dry && !c->prof && !c->hold_us && !sharded(c) && N >= 1 && K >= 1 &&
                       M >= 1;
    if (plain && c->lanes > 1 && lane_fits(c)) lane_switch(c);
    if (has_caller && !c->dry) {
        const hipEvent_t e = xevent(c, 0);
        hipck(hipEventRecord(e, caller), "hipEventRecord");
        hipck(hipStreamWaitEvent(c->st, e, 0), "hipStreamWaitEvent");
        c->xwait_side = e;                        // (st2 / st3: through st, see after_previous)
    }
    const bool usable = c->graph_vm && plain;
    if (!usable) {
        vmg_drop(c);
        c->vmg.seen.clear();
        return verify_mul_witness(c, a, b, N, K, M, on_device, gamma);
    }
    c->ht0 = std::chrono::steady_clock::now();
    settle(c);                     // (before any linear scope: it waits on tail events)
    struct Linear {                // vm_linear: every launch of the call on st
        svdw_ctx* c;
        hipStream_t s2 = nullptr, s3 = nullptr;
        bool on = false;
        explicit Linear(svdw_ctx* cc) : c(cc) {
            if (!c->vm_linear) return;
            if (!c->lin_ev) hipck(hipEventCreateWithFlags(&c->lin_ev, hipEventDisableTiming), "hipEventCreate");
            s2 = c->st2;
            s3 = c->st3;
            c->st2 = c->st3 = c->st;
            c->linear = on = true;
        }
        ~Linear() {
            if (!on) return;
            c->st2 = s2;
            c->st3 = s3;
            c->linear = false;
        }
    } lin{c};
    struct Flags {
        svdw_ctx* c;
        ~Flags() {
            c->gp_external = false;
            c->capturing = false;
            c->gp_ev = nullptr;
            c->pows_pre.on = false;
        }
    } flags{c};
    // gamma's tables (and the one / gamma-power cells when phase 1 holds them)
    // on st, ahead of everything the call queues. (Round 4 tried them on st3
    // beside the graph, the graph's scans waiting through an external event
    // node (hipEventWaitExternal): the runtime aborted in the capture/replay.)
    settle(c);
    PowCells pc;
    const bool pw = vm_pow_cells(c, M, gamma, &pc);
    gamma_prep(c, M, gamma, c->st, pw ? &pc : nullptr);
    host_mark(c, "vm: gamma_prep queued");
    c->gp_external = true;
    c->gp_ext_one = pw ? pc.one : nullptr;
    // (the cell set and gamma tables too: a pipelined svd_witness alternates between two)
    auto key_now = [&] {
        return std::vector<uint64_t>{N, K, M, (uint64_t)(uintptr_t)a, (uint64_t)(uintptr_t)b, c->epoch,
                                     (uint64_t)(uintptr_t)c->ph[0].adv, (uint64_t)(uintptr_t)c->ph[1].adv,
                                     (uint64_t)(uintptr_t)c->ph[0].lk, (uint64_t)(uintptr_t)c->ph[1].lk,
                                     (uint64_t)(uintptr_t)c->gpc.p, (uint64_t)(uintptr_t)c->gtab.p};
    };
    const std::vector<uint64_t> key = key_now();
    if (c->vmg.exec && key == c->vmg.key) {
        const svdw_counts k = vmg_restore(c, gamma);
        host_mark(c, "vm: host state restored");
        hipck(hipGraphLaunch(c->vmg.exec, c->st), "hipGraphLaunch");
        c->xwait_side = nullptr;                      // (its side streams fork from st)
        host_mark(c, "vm: graph launched");
        ++c->vmg.replays;
        return k;
    }
    if (key == c->vmg.seen) {
        vmg_drop(c);
        hipGraph_t graph = nullptr;
        hipck(hipStreamBeginCapture(c->st, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
        c->capturing = true;
        svdw_counts k{};
        try {
            k = verify_mul_witness(c, a, b, N, K, M, on_device, gamma);
            stream_dep(c, c->st2, c->st);                  // every forked stream joins st
            if (c->st3) stream_dep(c, c->st3, c->st);
        } catch (...) {
            // nothing captured ran: end the capture and run the call eagerly
            c->capturing = false;
            graph = nullptr;
            if (hipStreamEndCapture(c->st, &graph) == hipSuccess && graph) (void)hipGraphDestroy(graph);
            (void)hipGetLastError();
            c->vmg.seen.clear();
            return verify_mul_witness(c, a, b, N, K, M, on_device, gamma);
        }
        c->capturing = false;
        hipck(hipStreamEndCapture(c->st, &graph), "hipStreamEndCapture");
        hipGraphExec_t exec = nullptr;
        const hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        hipck(e, "hipGraphInstantiate");
        c->vmg.exec = exec;
        c->vmg.key = key;
        vmg_snapshot(c, k);
        hipck(hipGraphLaunch(exec, c->st), "hipGraphLaunch");
        ++c->vmg.captures;
        return k;
    }
    vmg_drop(c);
    const svdw_counts k = verify_mul_witness(c, a, b, N, K, M, on_device, gamma);
    c->vmg.seen = key_now();
    return k;
}

// ------------------------------------------------------ equality lists
// halo2-base's equality records of phase `phase` (svdw_equalities), in assign
// order, from the layout table: per region its element program's eq words
// (PB::eq) or the inner-product row pattern, with the source cells of the
// loaded values (RegionChecks::esrc). copies: (source | store << 62,
// destination) pairs, store 2 = the external init_rand cell; consts: (cell,
// 4 canonical words).
static uint64_t eq_src_cell(const RegionChecks::EqSrc& e, uint64_t i, uint64_t j, uint64_t t) {
    if (e.kind == EQS_CHAIN) {
        if (t == 0) return e.first | (uint64_t)e.first_phase << 62;
        return (e.off + (t - 1) * (uint64_t)e.rs) | (uint64_t)e.phase << 62;
    }
    if (e.kind == EQS_MAT) {
        if (e.diag_phase >= 0 && i == j) return e.diag_off | (uint64_t)e.diag_phase << 62;
        if (i < e.rows && j < e.cols)
            return (uint64_t)((int64_t)e.off + (int64_t)i * e.rs + (int64_t)j * e.cs) | (uint64_t)e.phase << 62;
        if (e.pad_phase >= 0) return e.pad_off | (uint64_t)e.pad_phase << 62;
    }
    fail(SVDW_EINVAL, "svdw_equalities: a region's copy source is not in the cell streams");
    return 0;
}
static void eq_lists(const svdw_ctx* c, uint32_t phase, std::vector<uint64_t>* copies,
                     std::vector<uint64_t>* consts) {
    auto konst = [&](uint64_t dst, const Fr& v) {
        consts->push_back(dst);
        for (int w = 0; w < 4; ++w) consts->push_back((uint64_t)v.w[2 * w] | (uint64_t)v.w[2 * w + 1] << 32);
    };
    const uint64_t me = (uint64_t)phase << 62;
    for (size_t k = 0; k < c->layout.size(); ++k) {
        const svdw_region& r = c->layout[k];
        const RegionChecks& rc = c->layout_chk[k];
        if (r.phase != phase || !r.n) continue;
        if (rc.scan) {                                    // [C(0), E(a_j), E(v_j), W(s_j), ...]
            const uint64_t R = r.rows, unit = r.n / R, L = (unit - 1) / 3;
            for (uint64_t i = 0; i < R; ++i) {
                const uint64_t base = r.off + i * unit;
                konst(base, fr_zero());
                for (uint64_t j = 0; j < L; ++j) {
                    copies->push_back(eq_src_cell(rc.esrc[0], i, j, 0));
                    copies->push_back(base + 1 + 3 * j);
                    copies->push_back(eq_src_cell(rc.esrc[1], 0, 0, j));
                    copies->push_back(base + 2 + 3 * j);
                }
            }
            continue;
        }
        if (rc.eq.empty() || !rc.unit) continue;
        const uint64_t unit = rc.unit, nel = r.n / unit, cols = rc.cols ? rc.cols : 1;
        for (uint64_t e = 0; e < nel; ++e) {
            const uint64_t base = r.off + e * unit, i = e / cols, j = e % cols;
            for (uint32_t w : rc.eq) {
                const uint32_t a = eq_a(w), at = eq_slot(w);
                switch (eq_kind(w)) {
                case EQ_CONST: konst(base + at, rc.eqk.at(a)); break;
                case EQ_LOCAL: copies->push_back((base + a) | me); copies->push_back(base + at); break;
                case EQ_VIEW:
                    copies->push_back(eq_src_cell(rc.esrc[a], i, j, i));
                    copies->push_back(base + at);
                    break;
                default:                                  // EQ_EXT: init_rand's RLC cell
                    copies->push_back(c->ext_off | 2ull << 62); copies->push_back(base + at); break;
                }
            }
        }
    }
}
// The same records generated on the device (k_eq_records) into c->eq_cp /
// c->eq_ks: per region its record counts are closed-form (elements x copy /
// constant words, or rows x 2L copies + rows constants for a scan), so every
// work item writes at a fixed offset and the order is eq_lists' order.
static EqSrcDev eqsrc_dev(const RegionChecks::EqSrc& e) {
    EqSrcDev d;
    memset(&d, 0, sizeof d);
    d.kind = e.kind; d.phase = (int32_t)e.phase; d.pad_phase = e.pad_phase; d.diag_phase = e.diag_phase;
    d.first_phase = (int32_t)e.first_phase; d.off = e.off; d.pad_off = e.pad_off; d.diag_off = e.diag_off;
    d.first = e.first; d.rs = e.rs; d.cs = e.cs; d.rows = e.rows; d.cols = e.cols;
    return d;
}
static void eq_gen_device(svdw_ctx* c, uint32_t phase, uint64_t* n_copies, uint64_t* n_consts) {
    std::vector<EqRegionDev> regs;
    std::vector<uint32_t> words;
    std::vector<Fr> konst;
    uint64_t items = 0, nc = 0, nk = 0;
    for (size_t k = 0; k < c->layout.size(); ++k) {
        const svdw_region& r = c->layout[k];
        const RegionChecks& rc = c->layout_chk[k];
        if (r.phase != phase || !r.n) continue;
        EqRegionDev d;
        memset(&d, 0, sizeof d);
        d.off = r.off;
        d.item0 = items;
        d.copy0 = nc;
        d.const0 = nk;
        d.src[0] = eqsrc_dev(rc.esrc[0]);
        d.src[1] = eqsrc_dev(rc.esrc[1]);
        if (rc.scan) {
            const uint64_t R = r.rows, unit = r.n / R, L = (unit - 1) / 3;
            REQUIRE(L >= 1, "internal: empty scan rows");
            d.scan = 1; d.unit = (uint32_t)unit; d.L = (uint32_t)L;
            d.nitems = R * L;
            nc += R * 2 * L;
            nk += R;
        } else {
            if (rc.eq.empty() || !rc.unit) continue;
            const uint64_t nel = r.n / rc.unit;
            d.unit = rc.unit;
            d.cols = rc.cols ? rc.cols : 1;
            d.w0 = (uint32_t)words.size();
            d.nw = (uint32_t)rc.eq.size();
            d.k0 = (uint32_t)konst.size();
            for (uint32_t w : rc.eq) (eq_kind(w) == EQ_CONST ? d.nkw : d.ncw) += 1;
            words.insert(words.end(), rc.eq.begin(), rc.eq.end());
            konst.insert(konst.end(), rc.eqk.begin(), rc.eqk.end());
            d.nitems = nel;
            nc += nel * d.ncw;
            nk += nel * d.nkw;
        }
        items += d.nitems;
        regs.push_back(d);
    }
    *n_copies = nc;
    *n_consts = nk;
    ensure_buf(c, c->eq_cp, std::max<uint64_t>(nc, 1) * 16);
    ensure_buf(c, c->eq_ks, std::max<uint64_t>(nk, 1) * 40);
    ensure_buf(c, c->eq_reg, std::max<size_t>(regs.size(), 1) * sizeof(EqRegionDev));
    ensure_buf(c, c->eq_w, std::max<size_t>(words.size(), 1) * 4);
    ensure_buf(c, c->eq_k, std::max<size_t>(konst.size(), 1) * sizeof(Fr));
    ensure_buf(c, c->eq_err, 4);
    hipStream_t s = c->st;
    if (!regs.empty())
        hipck(hipMemcpyAsync(c->eq_reg.p, regs.data(), regs.size() * sizeof(EqRegionDev), hipMemcpyHostToDevice, s), "H2D");
    if (!words.empty()) hipck(hipMemcpyAsync(c->eq_w.p, words.data(), words.size() * 4, hipMemcpyHostToDevice, s), "H2D");
    if (!konst.empty())
        hipck(hipMemcpyAsync(c->eq_k.p, konst.data(), konst.size() * sizeof(Fr), hipMemcpyHostToDevice, s), "H2D");
    hipck(hipMemsetAsync(c->eq_err.p, 0, 4, s), "memset");
    hipck(launch_eq_records((const EqRegionDev*)c->eq_reg.p, (uint32_t)regs.size(), items, (const uint32_t*)c->eq_w.p,
                            (const Fr*)c->eq_k.p, phase, c->ext_off, (uint64_t*)c->eq_cp.p, (uint64_t*)c->eq_ks.p,
                            (unsigned*)c->eq_err.p, s), "k_eq_records");
    unsigned err = 0;
    hipck(hipMemcpyAsync(&err, c->eq_err.p, 4, hipMemcpyDeviceToHost, s), "D2H");
    hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
    REQUIRE(!err, "svdw_equalities: a region's copy source is not in the cell streams");
}
// virtual cell -> column-major physical index (the first placement of a break cell)
static uint64_t phys_index(const svdw_ctx* c, uint32_t phase, uint64_t v) {
    const auto& st = c->phys.start[phase];
    size_t col = std::upper_bound(st.begin(), st.end(), v) - st.begin();
    REQUIRE(col > 0, "internal: cell before column 0");
    --col;
    if (col > 0 && v == st[col]) --col;                   // break cell: its row in the column before
    return ((uint64_t)col << c->phys.k) + (v - st[col]);
}

// ================================================================== C ABI
extern "C" {

const char* svdw_last_error(void) { return g_err.c_str(); }

int svdw_ctx_create(const svdw_params* p, svdw_ctx** out) {
    return guarded([&] {
        REQUIRE(p && out, "null argument");
        if (p->precision_bits < 1 || p->precision_bits > 63)
            fail(SVDW_ERANGE, "precision_bits must be in [1, 63] (src/svd/mod.rs:74 uses u64)");
        if (p->lookup_bits < 8 || p->lookup_bits > 63)
            fail(SVDW_ERANGE, "lookup_bits must be in [8, 63]");
        svdw_ctx* c = new svdw_ctx();
        c->P = p->precision_bits;
        c->LB = p->lookup_bits;
        c->device = p->device;
        c->dry = p->device < 0;
        if (const char* h = getenv("SVDW_HOST_TRACE")) c->host_trace = atoi(h) != 0;
        if (const char* g = getenv("SVDW_GEMM"))
            c->gemm_impl = (!strcmp(g, "valu") || !strcmp(g, "dot4")) ? SVDW_GEMM_VALU : SVDW_GEMM_MFMA;
        if (!c->dry) {
            try {
                ctx_init_device(c);
            } catch (...) {
                ctx_release(c);
                throw;
            }
        }
        *out = c;
    });
}
int svdw_ctx_destroy(svdw_ctx* c) {
    return guarded([&] { ctx_release(c); });
}
int svdw_ctx_reset(svdw_ctx* c) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        sync(c);
        clear_streams(c);
        c->pre.clear();
        c->pre_wait_st = nullptr;
        c->pre_wait_ev = nullptr;
    });
}
int svdw_reserve(svdw_ctx* c, uint32_t phase, uint64_t na, uint64_t nl) {
    return guarded([&] {
        REQUIRE(c && phase < 2, "bad argument");
        Stream& s = c->ph[phase];
        grow(c, s.adv, s.n, s.cap, na);
        grow(c, s.lk, s.nl, s.lcap, nl);
    });
}
// Stream-ordered hand-off with a caller's stream (e.g. torch's current stream):
// the context's streams wait for the work queued on `s` so far (inputs it is
// still writing, buffers it still reads), and `s` waits for the context's
// queued work (outputs it will read). No host wait either way.
static hipEvent_t xevent(svdw_ctx* c, int i) {
    if (!c->xev[i])
        hipck(hipEventCreateWithFlags(&c->xev[i], hipEventDisableTiming), "hipEventCreate");
    return c->xev[i];
}
// st waits at once; st2 / st3 inherit the wait from st where a call orders them
// after it, else wait themselves (xwait_side). With lanes, the lane's state too
// (the next verify_mul_witness runs there).
int svdw_stream_wait(svdw_ctx* c, void* stream) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        if (c->dry) return;
        const hipStream_t s = (hipStream_t)stream;
        const hipEvent_t e = xevent(c, 0);
        hipck(hipEventRecord(e, s), "hipEventRecord");
        for (svdw_ctx* x : {c, c->lane}) {
            if (!x) continue;
            hipck(hipStreamWaitEvent(x->st, e, 0), "hipStreamWaitEvent");
            x->xwait_side = e;
        }
    });
}
int svdw_stream_signal(svdw_ctx* c, void* stream) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        if (c->dry) return;
        const hipStream_t s = (hipStream_t)stream;
        for (svdw_ctx* x : {c, c->lane}) {
            if (!x) continue;
            int i = 1;
            for (hipStream_t t : {x->st, x->st2, x->st3}) {
                if (!t) continue;
                flush_batch(x, t);
                const hipEvent_t e = xevent(x, i++);
                hipck(hipEventRecord(e, t), "hipEventRecord");
                hipck(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent");
            }
        }
    });
}
int svdw_debug_trace(void* buf) {
    return guarded([&] { hipck(set_debug_trace(buf), "set_debug_trace"); });
}
int svdw_sync(svdw_ctx* c) {
    return guarded([&] { REQUIRE(c, "null ctx"); sync(c); });
}
// 1 when every launch queued on the context (both lanes) has completed, 0
// while some still runs; no host wait (hipStreamQuery).
int svdw_query(svdw_ctx* c) {
    int done = 1;
    const int rc = guarded([&] {
        REQUIRE(c, "null ctx");
        if (c->dry) return;
        for (svdw_ctx* x : {c, c->lane}) {
            if (!x) continue;
            for (hipStream_t t : {x->st, x->st2, x->st3}) {
                if (!t) continue;
                const hipError_t e = hipStreamQuery(t);
                if (e == hipErrorNotReady) {
                    done = 0;
                    return;
                }
                hipck(e, "hipStreamQuery");
            }
        }
    });
    return rc ? rc : done;
}
// Completion marks (svdw_mark / svdw_mark_done / svdw_mark_wait): an event on
// each stream of both lanes, recorded behind what is queued there (pending
// batched stages launched first), so no stream waits for anything. A slot is
// reused 16 marks later; a ticket whose slot holds a later mark is answered
// by that mark (later done implies earlier done; not done reads as 0).
int svdw_mark(svdw_ctx* c, uint64_t* ticket) {
    return guarded([&] {
        REQUIRE(c && ticket, "null argument");
        const uint64_t t = ++c->mk.seq;
        *ticket = t;
        if (c->dry) return;
        const int k = (int)(t % svdw_ctx::kMarks);
        int i = 0;
        for (svdw_ctx* x : {c, c->lane}) {
            if (!x) continue;
            for (hipStream_t st : {x->st, x->st2, x->st3}) {
                if (!st) continue;
                flush_batch(x, st);
                hipEvent_t& e = c->mk.ev[k][i++];
                if (!e) hipck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
                hipck(hipEventRecord(e, st), "hipEventRecord");
            }
        }
        c->mk.used[k] = (uint8_t)i;
        c->mk.t[k] = t;
    });
}
// the slot answering ticket t, or -1 (t not issued)
static int mark_slot(const svdw_ctx* c, uint64_t t) {
    if (!t || t > c->mk.seq) return -1;
    return (int)(t % svdw_ctx::kMarks);
}
int svdw_mark_done(svdw_ctx* c, uint64_t ticket) {
    int done = 1;
    const int rc = guarded([&] {
        REQUIRE(c, "null ctx");
        const int k = mark_slot(c, ticket);
        REQUIRE(k >= 0, "svdw_mark_done: ticket not issued");
        if (c->dry) return;
        for (int i = 0; i < c->mk.used[k]; ++i) {
            const hipError_t e = hipEventQuery(c->mk.ev[k][i]);
            if (e == hipErrorNotReady) {
                done = 0;
                return;
            }
            hipck(e, "hipEventQuery");
        }
    });
    return rc ? rc : done;
}
int svdw_mark_wait(svdw_ctx* c, uint64_t ticket) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        const int k = mark_slot(c, ticket);
        REQUIRE(k >= 0, "svdw_mark_wait: ticket not issued");
        if (c->dry) return;
        for (int i = 0; i < c->mk.used[k]; ++i) hipck(hipEventSynchronize(c->mk.ev[k][i]), "hipEventSynchronize");
    });
}
uint64_t svdw_advice_len(const svdw_ctx* c, uint32_t phase) { return c && phase < 2 ? c->ph[phase].n : 0; }
uint64_t svdw_lookup_len(const svdw_ctx* c, uint32_t phase) { return c && phase < 2 ? c->ph[phase].nl : 0; }
const void* svdw_advice_device_ptr(const svdw_ctx* c, uint32_t phase) { return c && phase < 2 ? c->ph[phase].adv : nullptr; }
const void* svdw_lookup_device_ptr(const svdw_ctx* c, uint32_t phase) { return c && phase < 2 ? c->ph[phase].lk : nullptr; }

static int copy_cells(svdw_ctx* c, uint32_t phase, uint64_t off, uint64_t n, uint64_t* out, bool lk) {
    return guarded([&] {
        REQUIRE(c && phase < 2 && out, "bad argument");
        REQUIRE(!c->dry, "planning context has no cells");
        const Stream& s = c->ph[phase];
        REQUIRE(off + n <= (lk ? s.nl : s.n), "copy range outside the stream");
        if (!n) return;
        settle(c);
        hipck(hipMemcpyAsync(out, (lk ? s.lk : s.adv) + off, n * sizeof(Fr), hipMemcpyDeviceToHost,
                             c->st), "D2H");
        sync(c);
    });
}
int svdw_copy_advice(svdw_ctx* c, uint32_t phase, uint64_t off, uint64_t n, uint64_t* out) {
    return copy_cells(c, phase, off, n, out, false);
}
int svdw_copy_lookup(svdw_ctx* c, uint32_t phase, uint64_t off, uint64_t n, uint64_t* out) {
    return copy_cells(c, phase, off, n, out, true);
}

int svdw_zkmatrix_new(svdw_ctx* c, uint32_t phase, const double* data, uint32_t rows,
                      uint32_t cols, int on_device, svdw_mat* out) {
    return guarded([&] {
        REQUIRE(c && out, "null argument");
        *out = zkmatrix_new(c, phase, data, rows, cols, on_device != 0);
    });
}
int svdw_zkvector_new(svdw_ctx* c, uint32_t phase, const double* data, uint32_t len, int on_device,
                      svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && out, "null argument");
        svdw_mat m = zkmatrix_new(c, phase, data, len, 1, on_device != 0);
        *out = svdw_vec{phase, len, m.off, 1};
    });
}
int svdw_transpose_matrix(const svdw_mat* a, svdw_mat* out) {
    return guarded([&] {
        REQUIRE(a && out, "null argument");
        svdw_mat t = *a;
        std::swap(t.rows, t.cols);
        std::swap(t.rs, t.cs);
        *out = t;
    });
}
int svdw_load_witness(svdw_ctx* c, uint32_t phase, const uint64_t value[4], svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && value && out, "null argument");
        *out = put_cell(c, phase, fr_from_words(value));
    });
}
int svdw_load_constant(svdw_ctx* c, uint32_t phase, const uint64_t value[4], svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && value && out, "null argument");
        *out = put_cell(c, phase, fr_from_words(value), true);
    });
}
int svdw_entries_less_than(svdw_ctx* c, const svdw_vec* d, uint32_t max_bits) {
    return guarded([&] {
        REQUIRE(c && d, "null argument");
        check_vec(c, *d);
        pregrow(c, [&](svdw_ctx* x) { entries_less_than(x, *d, max_bits); });
        entries_less_than(c, *d, max_bits);
    });
}
int svdw_entries_in_desc_order(svdw_ctx* c, const svdw_vec* d, uint32_t max_bits) {
    return guarded([&] {
        REQUIRE(c && d, "null argument");
        check_vec(c, *d);
        pregrow(c, [&](svdw_ctx* x) { entries_in_desc_order(x, *d, max_bits); });
        entries_in_desc_order(c, *d, max_bits);
    });
}
int svdw_check_mat_entries_bounded(svdw_ctx* c, const svdw_mat* a, const uint64_t bnd[4]) {
    return guarded([&] {
        REQUIRE(c && a && bnd, "null argument");
        check_mat(c, *a);
        pregrow(c, [&](svdw_ctx* x) { check_mat_entries_bounded(x, *a, big_from_words(bnd)); });
        check_mat_entries_bounded(c, *a, big_from_words(bnd));
    });
}
int svdw_check_mat_diff(svdw_ctx* c, const svdw_mat* a, const svdw_mat* b, const uint64_t tol[4]) {
    return guarded([&] {
        REQUIRE(c && a && b && tol, "null argument");
        check_mat(c, *a);
        check_mat(c, *b);
        REQUIRE(a->rows == b->rows && a->cols == b->cols, "check_mat_diff: shape mismatch");
        REQUIRE(a->phase == b->phase, "check_mat_diff: a and b in different phases");
        pregrow(c, [&](svdw_ctx* x) {
            check_mat_diff_views(x, a->phase, view_of(x, *a), view_of(x, *b), a->rows, a->cols,
                                 big_from_words(tol));
        });
        check_mat_diff_views(c, a->phase, view_of(c, *a), view_of(c, *b), a->rows, a->cols,
                             big_from_words(tol));
    });
}
int svdw_check_mat_id(svdw_ctx* c, const svdw_mat* a, const svdw_vec* sid, const uint64_t tol[4]) {
    return guarded([&] {
        REQUIRE(c && a && sid && tol, "null argument");
        check_mat(c, *a);
        check_vec(c, *sid);
        pregrow(c, [&](svdw_ctx* x) { check_mat_id(x, *a, *sid, big_from_words(tol)); });
        check_mat_id(c, *a, *sid, big_from_words(tol));
    });
}
int svdw_mat_times_diag_mat(svdw_ctx* c, const svdw_mat* a, const svdw_vec* v, svdw_mat* out) {
    return guarded([&] {
        REQUIRE(c && a && v && out, "null argument");
        check_mat(c, *a);
        check_vec(c, *v);
        pregrow(c, [&](svdw_ctx* x) { mat_times_diag_mat(x, *a, *v); });
        *out = mat_times_diag_mat(c, *a, *v);
    });
}
int svdw_rescale_matrix(svdw_ctx* c, const svdw_mat* cs, const svdw_div_scale* cfg, svdw_mat* out) {
    return guarded([&] {
        REQUIRE(c && cs && out, "null argument");
        check_mat(c, *cs);
        const DivScale d = div_scale_of(c, cfg);
        pregrow(c, [&](svdw_ctx* x) { rescale_matrix(x, *cs, d); });
        *out = rescale_matrix(c, *cs, d);
    });
}
int svdw_zkvector_inner_product(svdw_ctx* c, uint32_t phase, const svdw_vec* self, const svdw_vec* x,
                                const svdw_div_scale* cfg, svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && self && x && out, "null argument");
        REQUIRE(phase < 2, "phase must be 0 or 1");
        check_vec(c, *self);
        check_vec(c, *x);
        const DivScale d = div_scale_of(c, cfg);
        pregrow(c, [&](svdw_ctx* y) { zkvector_inner_product(y, phase, *self, *x, d); });
        *out = zkvector_inner_product(c, phase, *self, *x, d);
    });
}
int svdw_zkvector_norm_square(svdw_ctx* c, uint32_t phase, const svdw_vec* self,
                              const svdw_div_scale* cfg, svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && self && out, "null argument");
        REQUIRE(phase < 2, "phase must be 0 or 1");
        check_vec(c, *self);
        const DivScale d = div_scale_of(c, cfg);
        pregrow(c, [&](svdw_ctx* y) { zkvector_norm_square(y, phase, *self, d); });
        *out = zkvector_norm_square(c, phase, *self, d);
    });
}
int svdw_zkvector_norm(svdw_ctx* c, uint32_t phase, const svdw_vec* self, const svdw_div_scale* cfg,
                       uint32_t sqrt_bits, svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && self && out, "null argument");
        REQUIRE(phase < 2, "phase must be 0 or 1");
        check_vec(c, *self);
        const DivScale d = div_scale_of(c, cfg);
        auto f = [&](svdw_ctx* x) { return qsqrt_vec(x, phase, zkvector_norm_square(x, phase, *self, d), sqrt_bits); };
        pregrow(c, f);
        *out = f(c);
    });
}
int svdw_zkvector_dist(svdw_ctx* c, uint32_t phase, const svdw_vec* self, const svdw_vec* x,
                       const svdw_div_scale* cfg, uint32_t sqrt_bits, svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && self && x && out, "null argument");
        REQUIRE(phase < 2, "phase must be 0 or 1");
        check_vec(c, *self);
        check_vec(c, *x);
        const DivScale d = div_scale_of(c, cfg);
        auto f = [&](svdw_ctx* y) {
            return qsqrt_vec(y, phase, zkvector_dist_square(y, phase, *self, *x, d), sqrt_bits);
        };
        pregrow(c, f);
        *out = f(c);
    });
}
int svdw_zkvector_dist_square(svdw_ctx* c, uint32_t phase, const svdw_vec* self, const svdw_vec* x,
                              const svdw_div_scale* cfg, svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && self && x && out, "null argument");
        REQUIRE(phase < 2, "phase must be 0 or 1");
        check_vec(c, *self);
        check_vec(c, *x);
        const DivScale d = div_scale_of(c, cfg);
        pregrow(c, [&](svdw_ctx* y) { zkvector_dist_square(y, phase, *self, *x, d); });
        *out = zkvector_dist_square(c, phase, *self, *x, d);
    });
}
int svdw_zkvector_mul(svdw_ctx* c, uint32_t phase, const svdw_vec* self, const svdw_mat* a,
                      const svdw_div_scale* cfg, svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && self && a && out, "null argument");
        REQUIRE(phase < 2, "phase must be 0 or 1");
        check_vec(c, *self);
        check_mat(c, *a);
        const DivScale d = div_scale_of(c, cfg);
        pregrow(c, [&](svdw_ctx* y) { zkvector_mul(y, phase, *self, *a, d); });
        *out = zkvector_mul(c, phase, *self, *a, d);
    });
}
int svdw_honest_prover_mat_mul(svdw_ctx* c, uint32_t phase, const svdw_mat* a, const svdw_mat* b,
                               svdw_mat* out) {
    return guarded([&] {
        REQUIRE(c && a && b && out, "null argument");
        check_mat(c, *a);
        check_mat(c, *b);
        struct Solo {                        // a product queued on its own: the persistent GEMM
            svdw_ctx* c;
            ~Solo() { c->gemm_solo = false; }
        } solo{c};
        c->gemm_solo = true;
        *out = honest_prover_mat_mul(c, phase, *a, *b);
    });
}
int svdw_field_mat_vec_mul(svdw_ctx* c, uint32_t phase, const svdw_mat* a, const svdw_vec* v,
                           svdw_vec* out) {
    return guarded([&] {
        REQUIRE(c && a && v && out, "null argument");
        check_mat(c, *a);
        check_vec(c, *v);
        pregrow(c, [&](svdw_ctx* x) { field_mat_vec_mul(x, phase, *a, *v); });
        *out = field_mat_vec_mul(c, phase, *a, *v);
    });
}
int svdw_verify_mul(svdw_ctx* c, uint32_t phase, const svdw_mat* a, const svdw_mat* b,
                    const svdw_mat* cs, const uint64_t gamma[4]) {
    return guarded([&] {
        REQUIRE(c && a && b && cs && gamma, "null argument");
        check_mat(c, *a);
        check_mat(c, *b);
        check_mat(c, *cs);
        pregrow(c, [&](svdw_ctx* x) { verify_mul(x, phase, *a, *b, *cs, fr_from_words(gamma)); });
        verify_mul(c, phase, *a, *b, *cs, fr_from_words(gamma));
    });
}
int svdw_err_calc(uint32_t p, uint64_t size, double max_norm, double eps_svd, double eps_u,
                  double* es, double* eu) {
    return guarded([&] {
        REQUIRE(es && eu, "null argument");
        err_calc(p, size, max_norm, eps_svd, eps_u, es, eu);
    });
}
int svdw_check_svd_phase0(svdw_ctx* c, const svdw_mat* m, const svdw_mat* u, const svdw_mat* v,
                          const svdw_vec* d, double err_svd, double err_u, uint32_t max_bits_d,
                          svdw_svd_payload* out) {
    return guarded([&] {
        REQUIRE(c && m && u && v && d && out, "null argument");
        check_mat(c, *m); check_mat(c, *u); check_mat(c, *v); check_vec(c, *d);
        REQUIRE(m->phase == 0 && u->phase == 0 && v->phase == 0 && d->phase == 0,
                "check_svd_phase0 inputs must live in phase 0");
        pregrow(c, [&](svdw_ctx* x) {
            check_svd_phase0(x, *m, *u, *v, *d, err_svd, err_u, max_bits_d);
        });
        *out = check_svd_phase0(c, *m, *u, *v, *d, err_svd, err_u, max_bits_d);
    });
}
int svdw_check_svd_phase1(svdw_ctx* c, const svdw_mat* m, const svdw_mat* u, const svdw_mat* v,
                          const svdw_svd_payload* pl, const uint64_t gamma[4]) {
    return guarded([&] {
        REQUIRE(c && m && u && v && pl && gamma, "null argument");
        pregrow(c, [&](svdw_ctx* x) { check_svd_phase1(x, *m, *u, *v, *pl, fr_from_words(gamma)); });
        check_svd_phase1(c, *m, *u, *v, *pl, fr_from_words(gamma));
    });
}
int svdw_svd_witness(svdw_ctx* c, const double* m, const double* u, const double* v,
                     const double* d, uint32_t N, uint32_t M, int on_device,
                     const svdw_svd_config* cfg, const uint64_t gamma[4], svdw_counts* counts) {
    return guarded([&] {
        REQUIRE(c && cfg && gamma, "null argument");
        REQUIRE(c->dry || (m && u && v && d), "null input matrix");
        svdw_counts k = svd_witness(c, m, u, v, d, N, M, on_device != 0, *cfg, fr_from_words(gamma));
        if (counts) *counts = k;
    });
}
int svdw_verify_mul_witness(svdw_ctx* c, const double* a, const double* b, uint32_t N, uint32_t K,
                            uint32_t M, int on_device, const uint64_t gamma[4], svdw_counts* counts) {
    return guarded([&] {
        REQUIRE(c && gamma, "null argument");
        REQUIRE(c->dry || (a && b), "null input matrix");
        svdw_counts k = verify_mul_witness_api(c, a, b, N, K, M, on_device != 0, fr_from_words(gamma));
        if (counts) *counts = k;
    });
}
int svdw_verify_mul_witness_on(svdw_ctx* c, void* stream, const double* a, const double* b, uint32_t N,
                               uint32_t K, uint32_t M, const uint64_t gamma[4], svdw_counts* counts) {
    return guarded([&] {
        REQUIRE(c && gamma, "null argument");
        REQUIRE(c->dry || (a && b), "null input matrix");
        svdw_counts k = verify_mul_witness_api(c, a, b, N, K, M, true, fr_from_words(gamma), (hipStream_t)stream,
                                               true);
        if (counts) *counts = k;
    });
}
int svdw_parse_svd_input(const char* text, uint64_t len, int mode, svdw_input_dims* dims,
                         double* m, double* u, double* d, double* v) {
    return guarded([&] {
        REQUIRE(text && dims, "null argument");
        REQUIRE(mode == SVDW_PARSE_SERDE || mode == SVDW_PARSE_CORRECT, "parse mode: 0 or 1");
        svdw_ingest::SvdInput in;
        std::string err;
        svdw_ingest::Parser ps(text, len, mode);
        if (!ps.parse(in, err)) fail(SVDW_EINVAL, "svd input: " + err);
        REQUIRE(in.d.rows == 0 && in.m.rows && in.u.rows && in.v.rows,
                "svd input: m, u, v must be matrices and d a vector");
        *dims = svdw_input_dims{in.m.rows, in.m.cols, in.u.rows, in.u.cols, in.v.rows, in.v.cols,
                                in.d.cols};
        const std::pair<double*, const svdw_ingest::Array*> outs[4] = {
            {m, &in.m}, {u, &in.u}, {d, &in.d}, {v, &in.v}};
        for (const auto& o : outs)
            if (o.first) memcpy(o.first, o.second->v.data(), o.second->v.size() * sizeof(double));
    });
}
// Device ingest of data/matrix.in (ingest_dev.hip): three passes over the text
// on the device, then the few top-level keys and the arrays' number ranges on
// the host (small reads), then a device check of depths, separators and row
// lengths of m, u, v, d and device-to-device copies of their values.
namespace {
struct DevText {                  // small host reads of the device text
    svdw_ctx* c;
    const uint8_t* t;
    uint64_t n;
    std::vector<uint8_t> get(uint64_t at, uint64_t len) {
        len = std::min(len, at < n ? n - at : 0);
        std::vector<uint8_t> b(len);
        if (len) hipck(hipMemcpy(b.data(), t + at, len, hipMemcpyDeviceToHost), "D2H");
        return b;
    }
    // the string starting with the quote at `at`: its content (escapes as the
    // host parser reads them) and the position just past the closing quote
    bool str(uint64_t at, std::string* s, uint64_t* end) {
        uint64_t p = at + 1;
        bool esc = false;
        for (;;) {
            std::vector<uint8_t> b = get(p, 256);
            if (b.empty()) return false;
            for (size_t k = 0; k < b.size(); ++k, ++p) {
                if (esc) { s->push_back((char)b[k]); esc = false; continue; }
                if (b[k] == '\\') { esc = true; continue; }
                if (b[k] == '"') { *end = p + 1; return true; }
                s->push_back((char)b[k]);
            }
        }
    }
    int next_nonws(uint64_t at) {
        for (;;) {
            std::vector<uint8_t> b = get(at, 256);
            if (b.empty()) return -1;
            for (uint8_t x : b)
                if (!(x == ' ' || x == '\n' || x == '\r' || x == '\t')) return x;
            at += b.size();
        }
    }
};
}  // namespace
int svdw_parse_svd_input_device(svdw_ctx* c, const void* text, uint64_t len, int mode,
                                svdw_input_dims* dims, double* m, double* u, double* d, double* v) {
    namespace ig = svdw_ingest_dev;
    return guarded([&] {
        REQUIRE(c && text && dims, "null argument");
        REQUIRE(!c->dry, "device ingest needs a device context");
        REQUIRE(mode == SVDW_PARSE_SERDE,
                "device ingest: serde mode only (correct rounding: svdw_parse_svd_input)");
        REQUIRE(len > 0, "svd input: empty text");
        const uint8_t* t = (const uint8_t*)text;
        const uint64_t nc64 = (len + ig::kChunk - 1) / ig::kChunk;
        REQUIRE(nc64 < (1ull << 31), "svd input: text too large");
        const uint32_t nc = (uint32_t)nc64;
        hipStream_t s = c->st;
        sync(c);
        if (!c->ing_p10.p) {                       // serde's POW10 table (correctly rounded 10^k)
            std::vector<double> p10(309);
            char buf[16];
            for (int i = 0; i <= 308; ++i) { snprintf(buf, sizeof buf, "1e%d", i); p10[i] = strtod(buf, nullptr); }
            ensure_buf(c, c->ing_p10, sizeof(double) * 309);
            // on st, complete before p10 goes out of scope (a null-stream copy
            // is not ordered against the parse launches on st)
            hipck(hipMemcpyAsync(c->ing_p10.p, p10.data(), sizeof(double) * 309, hipMemcpyHostToDevice, s), "H2D");
            hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
        }
        ensure_buf(c, c->ing_x, sizeof(ig::Xfer) * nc);
        ensure_buf(c, c->ing_e, sizeof(ig::Entry) * (nc + 1));
        ensure_buf(c, c->ing_c, sizeof(ig::Counts) * (nc + 1));
        ig::Xfer* X = (ig::Xfer*)c->ing_x.p;
        ig::Entry* E = (ig::Entry*)c->ing_e.p;
        ig::Counts* C = (ig::Counts*)c->ing_c.p;
        hipck(ig::launch_pass1(t, len, X, s), "ingest pass 1");
        hipck(ig::launch_scan1(X, nc, E, s), "ingest scan 1");
        hipck(ig::launch_pass2(t, len, E, C, s), "ingest pass 2");
        hipck(ig::launch_scan2(C, nc, s), "ingest scan 2");
        ig::Entry fin;
        ig::Counts tot;
        hipck(hipMemcpyAsync(&fin, E + nc, sizeof fin, hipMemcpyDeviceToHost, s), "D2H");
        hipck(hipMemcpyAsync(&tot, C + nc, sizeof tot, hipMemcpyDeviceToHost, s), "D2H");
        hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
        REQUIRE(fin.state == 0, "svd input: unterminated string");
        REQUIRE(fin.depth == 0, "svd input: unbalanced brackets");
        const uint32_t nn = tot.num, nr = tot.row, nk = tot.key;
        ensure_buf(c, c->ing_val, sizeof(double) * std::max(nn, 1u));
        ensure_buf(c, c->ing_npos, sizeof(uint64_t) * std::max(nn, 1u));
        ensure_buf(c, c->ing_nd, std::max(nn, 1u));
        ensure_buf(c, c->ing_rpos, sizeof(uint64_t) * std::max(nr, 1u));
        ensure_buf(c, c->ing_kpos, sizeof(uint64_t) * std::max(nk, 1u));
        ensure_buf(c, c->ing_err, sizeof(uint64_t) * 264);
        unsigned long long* slist = (unsigned long long*)c->ing_err.p;          // [0] count, [1..255]
        unsigned long long* verr = slist + 256;
        hipck(hipMemsetAsync(slist, 0, sizeof(uint64_t), s), "memset");
        hipck(hipMemsetAsync(verr, 0xff, sizeof(uint64_t), s), "memset");
        hipck(ig::launch_pass3(t, len, E, C, (const double*)c->ing_p10.p, (double*)c->ing_val.p,
                               (uint64_t*)c->ing_npos.p, (uint8_t*)c->ing_nd.p, (uint64_t*)c->ing_rpos.p,
                               (uint64_t*)c->ing_kpos.p, slist, s), "ingest pass 3");
        std::vector<uint64_t> kpos(nk), sl(256);
        if (nk) hipck(hipMemcpyAsync(kpos.data(), c->ing_kpos.p, sizeof(uint64_t) * nk, hipMemcpyDeviceToHost, s), "D2H");
        hipck(hipMemcpyAsync(sl.data(), slist, sizeof(uint64_t) * 256, hipMemcpyDeviceToHost, s), "D2H");
        hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
        auto at = [](uint64_t p) { return " (at byte " + std::to_string(p) + ")"; };
        // members: depth-1 strings followed by ':' are keys (host parser: str, ws, ':')
        DevText dt{c, t, len};
        struct Member { uint64_t pos; std::string key; };
        std::vector<Member> mem;
        for (uint32_t j = 0; j < nk; ++j) {
            std::string k;
            uint64_t end = 0;
            REQUIRE(dt.str(kpos[j], &k, &end), "svd input: unterminated string" + at(kpos[j]));
            const int nx = dt.next_nonws(end);
            // a key follows '{' or ','; a string value follows ':' and is not followed by ':'
            std::vector<uint8_t> back = dt.get(kpos[j] >= 256 ? kpos[j] - 256 : 0, kpos[j] >= 256 ? 256 : kpos[j]);
            int pv = 0;
            for (size_t q = back.size(); q-- > 0;)
                if (!(back[q] == ' ' || back[q] == '\n' || back[q] == '\r' || back[q] == '\t')) { pv = back[q]; break; }
            if (pv == ':') {
                REQUIRE(nx != ':', "svd input: expected ',' or '}'" + at(end));
                continue;
            }
            REQUIRE(nx == ':', "svd input: expected ':'" + at(end));
            mem.push_back({kpos[j], k});
        }
        const uint64_t nsl = sl[0];
        REQUIRE(nsl <= 255, "svd input: too many structural irregularities for the device parser");
        for (const char* want : {"m", "u", "v", "d"}) {
            int cnt = 0;
            for (const auto& x : mem) cnt += x.key == want;
            REQUIRE(cnt <= 1, std::string("svd input: duplicate key \"") + want + "\"");
            REQUIRE(cnt == 1, "svd input: missing one of the keys m, u, v, d");
        }
        // number / row-open ranges of every member
        std::vector<uint64_t> q;
        for (const auto& x : mem) q.push_back(x.pos);
        q.push_back(len);
        ensure_buf(c, c->ing_q, (sizeof(uint64_t) + 2 * sizeof(uint32_t)) * q.size());
        uint32_t* rg = (uint32_t*)((uint64_t*)c->ing_q.p + q.size());
        hipck(hipMemcpyAsync(c->ing_q.p, q.data(), sizeof(uint64_t) * q.size(), hipMemcpyHostToDevice, s), "H2D");
        hipck(ig::launch_ranges((const uint64_t*)c->ing_npos.p, nn, (const uint64_t*)c->ing_rpos.p, nr,
                                (const uint64_t*)c->ing_q.p, (uint32_t)q.size(), rg, s), "ingest ranges");
        std::vector<uint32_t> r(2 * q.size());
        hipck(hipMemcpyAsync(r.data(), rg, sizeof(uint32_t) * r.size(), hipMemcpyDeviceToHost, s), "D2H");
        hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
        for (uint64_t k = 0; k < nsl; ++k) {       // structural errors: object level, or inside m/u/v/d
            const uint64_t p = sl[1 + k] & ~(1ull << 63);
            REQUIRE(!(sl[1 + k] >> 63), "svd input: malformed JSON object" + at(p));
            for (size_t j = 0; j < mem.size(); ++j) {
                const bool known = mem[j].key == "m" || mem[j].key == "u" || mem[j].key == "v" || mem[j].key == "d";
                REQUIRE(!(known && p >= q[j] && p < q[j + 1]), "svd input: malformed array" + at(p));
            }
        }
        struct Arr { uint32_t lo, hi, r0, rows, cols; };
        auto arr = [&](const char* key, bool matrix) {
            size_t j = 0;
            while (mem[j].key != key) ++j;
            Arr a{r[2 * j], r[2 * j + 2], r[2 * j + 1], r[2 * j + 3] - r[2 * j + 1], 0};
            const uint32_t total = a.hi - a.lo;
            if (matrix) {
                REQUIRE(a.rows >= 1, "svd input: m, u, v must be matrices and d a vector");
                REQUIRE(total % a.rows == 0, std::string("svd input: ragged matrix rows (") + key + ")");
                a.cols = total / a.rows;
            } else {
                REQUIRE(a.rows == 0, "svd input: m, u, v must be matrices and d a vector");
                a.cols = total;
            }
            hipck(ig::launch_validate((const uint8_t*)c->ing_nd.p, a.lo, a.hi, matrix ? 3 : 2,
                                      (const uint64_t*)c->ing_npos.p, nn, (const uint64_t*)c->ing_rpos.p,
                                      a.r0, a.rows, a.cols, verr, s), "ingest validate");
            return a;
        };
        const Arr am = arr("m", true), au = arr("u", true), av = arr("v", true), ad = arr("d", false);
        unsigned long long ve = 0;
        hipck(hipMemcpyAsync(&ve, verr, sizeof ve, hipMemcpyDeviceToHost, s), "D2H");
        hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
        if (ve != ~0ull) {
            static const char* what[] = {"", "expected a number", "significand beyond u64 (serde's overflow path is not emulated)",
                                         "number out of range", "expected ',' or ']'", "unexpected nesting",
                                         "ragged matrix rows"};
            const uint32_t code = (uint32_t)(ve >> 48);
            fail(SVDW_EINVAL, std::string("svd input: ") + (code < 7 ? what[code] : "malformed") +
                              at(ve & ((1ull << 48) - 1)));
        }
        *dims = svdw_input_dims{am.rows, am.cols, au.rows, au.cols, av.rows, av.cols, ad.cols};
        const std::pair<double*, const Arr*> outs[4] = {{m, &am}, {u, &au}, {d, &ad}, {v, &av}};
        for (const auto& o : outs)
            if (o.first && o.second->hi > o.second->lo)
                hipck(hipMemcpyAsync(o.first, (const double*)c->ing_val.p + o.second->lo,
                                     sizeof(double) * (o.second->hi - o.second->lo), hipMemcpyDeviceToDevice, s),
                      "D2D");
        hipck(hipStreamSynchronize(s), "hipStreamSynchronize");
    });
}
int svdw_set_shard(svdw_ctx* c, uint32_t rank, uint32_t world) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        REQUIRE(world >= 1 && rank < world, "svdw_set_shard: need rank < world");
        ++c->epoch;
        c->shard_rank = rank;
        c->shard_world = world;
        c->owned.clear();
    });
}
// The parts of [off, off + n) of a phase's advice (lookup) stream this context
// holds: all of it, or for a row-sharded rank the intersection with its owned
// segments (whole row blocks).
static std::vector<std::pair<uint64_t, uint64_t>> held(const svdw_ctx* c, uint32_t phase, bool lookup,
                                                       uint64_t off, uint64_t n) {
    std::vector<std::pair<uint64_t, uint64_t>> out;
    if (!n) return out;
    if (!sharded(c)) {
        out.emplace_back(off, n);
        return out;
    }
    for (const auto& o : c->owned) {
        if (o.phase != phase || (o.lookup != 0) != lookup) continue;
        const uint64_t b = std::max(off, o.off), e = std::min(off + n, o.off + o.n);
        if (b < e) out.emplace_back(b, e - b);
    }
    return out;
}
int svdw_check_gates(svdw_ctx* c, svdw_check_result* out) {
    return guarded([&] {
        REQUIRE(c && out, "null argument");
        REQUIRE(!c->dry, "svdw_check_gates needs a device context");
        sync(c);
        memset(out, 0, sizeof *out);
        ensure_buf(c, c->chk, 6 * sizeof(unsigned long long));
        unsigned long long* cnt = (unsigned long long*)c->chk.p;
        hipck(hipMemsetAsync(cnt, 0, 6 * sizeof(unsigned long long), c->st), "hipMemsetAsync");
        std::vector<uint32_t> scan_w;
        for (size_t k = 0; k < c->layout.size(); ++k) {
            const svdw_region& r = c->layout[k];
            const RegionChecks& rc = c->layout_chk[k];
            for (const auto& sg : held(c, r.phase, true, r.loff, r.nl))
                hipck(launch_check_lookups(c->ph[r.phase].lk + sg.first, sg.second, c->LB, cnt + 2, c->st),
                      "k_check_lookups");
            const std::vector<uint32_t>* w = &rc.words;
            uint64_t unit = rc.unit;
            uint32_t cols = rc.cols;
            if (!strcmp(r.tag, "scan") && r.rows) {         // rows [0, a0, v0, s0, a1, v1, s1, ...]
                unit = r.n / r.rows;
                cols = 1;
                scan_w.clear();
                for (uint64_t q = 0; q + 3 < unit; q += 3) scan_w.push_back(chk_gate((uint32_t)q));
                w = &scan_w;
            }
            if (w->empty() || !unit || !r.n) continue;
            ChkView v[kMaxViews];
            for (int q = 0; q < kMaxViews; ++q) {
                const RegionChecks::Src& s = rc.src[q];
                v[q] = s.phase < 0 ? ChkView{nullptr, 0, 0, 0, 0}
                                   : ChkView{c->ph[s.phase].adv + s.off, s.rs, s.cs, s.rows, s.cols};
            }
            const auto segs = held(c, r.phase, false, r.off, r.n);
            if (segs.empty()) continue;
            ensure_buf(c, c->chkg, w->size() * sizeof(uint32_t));
            hipck(hipMemcpyAsync(c->chkg.p, w->data(), w->size() * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, c->st), "H2D");
            for (const auto& sg : segs) {
                if ((sg.first - r.off) % unit || sg.second % unit)
                    fail(SVDW_EINVAL, "svdw_check_gates: owned segment is not whole elements");
                hipck(launch_check_cells(c->ph[r.phase].adv + sg.first, (sg.first - r.off) / unit,
                                         sg.second / unit, (uint32_t)unit, cols, (const uint32_t*)c->chkg.p,
                                         (uint32_t)w->size(), v[0], v[1], cnt, c->st), "k_check_cells");
            }
            hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");   // chkg is reused
        }
        unsigned long long h[6];
        hipck(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, c->st), "D2H");
        hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");
        out->gates_checked = h[0];
        out->gate_failures = h[1];
        out->lookups_checked = h[2];
        out->lookup_failures = h[3];
        out->copies_checked = h[4];
        out->copy_failures = h[5];
    });
}
// ------------------------------------------------- physical layout
// Virtual -> physical assignment of a phase's cells (halo2-base 0.4.1, recalled;
// oracle/pyoracle.py physical_layout): basic-gate advice columns of max_rows =
// 2^k - minimum_rows usable rows. A column ends at a cell whose gate would
// cross max_rows (q && row + 4 > max_rows) or at row max_rows - 1; that cell is
// repeated at row 0 of the next column (copy-constrained) and its selector is
// enabled there only.
namespace {
struct GateIndex {               // q(i): does a basic gate start at virtual cell i
    struct Reg {
        uint64_t off, n, unit;
        bool scan;
        std::vector<uint8_t> bit;    // per unit offset (program regions)
    };
    std::vector<Reg> regs;       // ascending offsets
    GateIndex(const svdw_ctx* c, uint32_t phase) {
        for (size_t k = 0; k < c->layout.size(); ++k) {
            const svdw_region& r = c->layout[k];
            if (r.phase != phase || !r.n) continue;
            if (!strcmp(r.tag, "scan") && r.rows) {
                regs.push_back(Reg{r.off, r.n, r.n / r.rows, true, {}});
                continue;
            }
            const RegionChecks& rc = c->layout_chk[k];
            Reg g{r.off, r.n, rc.unit, false, std::vector<uint8_t>(rc.unit, 0)};
            bool any = false;
            for (uint32_t w : rc.words)
                if (chk_kind(w) == CHK_GATE) g.bit[w] = 1, any = true;
            if (any && rc.unit) regs.push_back(std::move(g));
        }
    }
    bool q(uint64_t i) const {
        auto it = std::upper_bound(regs.begin(), regs.end(), i,
                                   [](uint64_t x, const Reg& r) { return x < r.off; });
        if (it == regs.begin()) return false;
        const Reg& r = *--it;
        if (i >= r.off + r.n) return false;
        const uint64_t o = (i - r.off) % r.unit;
        return r.scan ? (o % 3 == 0 && o + 3 < r.unit) : r.bit[o] != 0;
    }
};
}  // namespace
int svdw_physical_layout(svdw_ctx* c, uint32_t k, uint32_t minimum_rows, svdw_physical_params* out) {
    return guarded([&] {
        REQUIRE(c && out, "null argument");
        REQUIRE(k >= 3 && k <= 40, "svdw_physical_layout: k out of range");
        REQUIRE(!sharded(c), "svdw_physical_layout: the witness of a sharded context is partial");
        REQUIRE((1ull << k) > (uint64_t)minimum_rows + 4, "svdw_physical_layout: minimum_rows >= 2^k - 4");
        const uint64_t R = (1ull << k) - minimum_rows;
        auto& P = c->phys;
        P.valid = false;
        P.k = k;
        P.min_rows = minimum_rows;
        P.R = R;
        memset(out, 0, sizeof *out);
        out->k = k;
        out->minimum_rows = minimum_rows;
        out->max_rows = R;
        for (uint32_t ph = 0; ph < 2; ++ph) {
            const uint64_t T = c->ph[ph].n, TL = c->ph[ph].nl;
            P.start[ph].clear();
            P.bp[ph].clear();
            const GateIndex gi(c, ph);
            for (uint64_t s = 0; T && true;) {
                P.start[ph].push_back(s);
                // the first of rows R-3, R-2 (gate crossing max_rows) or R-1 (last row)
                uint64_t r = R - 3;
                for (; r < R - 1; ++r)
                    if (s + r < T && gi.q(s + r)) break;
                if (s + r >= T) break;                     // the phase ends in this column
                P.bp[ph].push_back(r);
                s += r;
            }
            out->num_advice[ph] = (uint32_t)((T + R - 1) / R);
            out->columns_used[ph] = (uint32_t)P.start[ph].size();
            out->num_lookup_advice[ph] = (uint32_t)((TL + R - 1) / R);
        }
        out->constants = c->consts.size();
        out->num_fixed = (uint32_t)((c->consts.size() + (1ull << k) - 1) >> k);
        P.valid = true;
    });
}
int svdw_break_points(const svdw_ctx* c, uint32_t phase, uint64_t* out, uint64_t cap, uint64_t* n) {
    return guarded([&] {
        REQUIRE(c && n && phase < 2, "bad argument");
        REQUIRE(c->phys.valid, "svdw_break_points: call svdw_physical_layout after the witness");
        const auto& b = c->phys.bp[phase];
        *n = b.size();
        for (uint64_t i = 0; i < cap && i < b.size() && out; ++i) out[i] = b[i];
    });
}
int svdw_assign_columns(svdw_ctx* c, uint32_t phase, void* advice, uint8_t* selectors, void* lookup) {
    return guarded([&] {
        REQUIRE(c && phase < 2, "bad argument");
        REQUIRE(!c->dry, "svdw_assign_columns needs a device context");
        REQUIRE(c->phys.valid, "svdw_assign_columns: call svdw_physical_layout after the witness");
        sync(c);
        const auto& P = c->phys;
        const uint64_t rows = 1ull << P.k, T = c->ph[phase].n, TL = c->ph[phase].nl;
        const size_t ncols = P.start[phase].size();
        REQUIRE(ncols <= (T + P.R - 1) / P.R,
                "NOT ENOUGH ADVICE COLUMNS IN PHASE (columns_used > num_advice: raise k)");
        if (selectors && T) {                              // q bits of the virtual stream
            const GateIndex gi(c, phase);
            const uint64_t nw = (T + 31) / 32;
            ensure_buf(c, c->gateq[phase], nw * 4);
            uint32_t* qb = (uint32_t*)c->gateq[phase].p;
            hipck(hipMemsetAsync(qb, 0, nw * 4, c->st), "hipMemsetAsync");
            for (const auto& r : gi.regs) {
                std::vector<uint8_t> bits(r.unit);
                for (uint64_t o = 0; o < r.unit; ++o)
                    bits[o] = r.scan ? (o % 3 == 0 && o + 3 < r.unit) : r.bit[o];
                ensure_buf(c, c->chkg, r.unit);
                hipck(hipMemcpyAsync(c->chkg.p, bits.data(), r.unit, hipMemcpyHostToDevice, c->st), "H2D");
                hipck(launch_gate_bits(qb, r.off, r.n, r.unit, (const uint8_t*)c->chkg.p, c->st),
                      "k_gate_bits");
                hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");   // chkg is reused
            }
        }
        for (size_t col = 0; col < ncols; ++col) {
            const uint64_t s = P.start[phase][col];
            const bool last = col + 1 == ncols;
            const uint64_t len = last ? T - s : P.bp[phase][col] + 1;
            if (advice) {
                Fr* dst = (Fr*)advice + col * rows;
                hipck(hipMemcpyAsync(dst, c->ph[phase].adv + s, len * sizeof(Fr), hipMemcpyDeviceToDevice,
                                     c->st), "D2D");
                if (len < rows)
                    hipck(hipMemsetAsync(dst + len, 0, (rows - len) * sizeof(Fr), c->st), "hipMemsetAsync");
            }
            if (selectors)
                hipck(launch_selectors(selectors + col * rows, (const uint32_t*)c->gateq[phase].p, s, len,
                                       rows, !last, c->st), "k_selectors");
        }
        if (lookup) {
            const uint64_t nl = (TL + P.R - 1) / P.R;
            for (uint64_t col = 0; col < nl; ++col) {
                const uint64_t s = col * P.R, len = std::min(P.R, TL - s);
                Fr* dst = (Fr*)lookup + col * rows;
                hipck(hipMemcpyAsync(dst, c->ph[phase].lk + s, len * sizeof(Fr), hipMemcpyDeviceToDevice,
                                     c->st), "D2D");
                hipck(hipMemsetAsync(dst + len, 0, (rows - len) * sizeof(Fr), c->st), "hipMemsetAsync");
            }
        }
        hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");
    });
}
int svdw_check_physical(svdw_ctx* c, uint32_t phase, const void* advice, const uint8_t* selectors,
                        uint32_t ncols, svdw_check_result* out) {
    return guarded([&] {
        REQUIRE(c && advice && selectors && out && phase < 2, "bad argument");
        REQUIRE(!c->dry, "svdw_check_physical needs a device context");
        REQUIRE(c->phys.valid, "svdw_check_physical: call svdw_physical_layout first");
        memset(out, 0, sizeof *out);
        settle(c);
        ensure_buf(c, c->chk, 6 * sizeof(unsigned long long));
        unsigned long long* cnt = (unsigned long long*)c->chk.p;
        hipck(hipMemsetAsync(cnt, 0, 6 * sizeof(unsigned long long), c->st), "hipMemsetAsync");
        hipck(launch_check_physical((const Fr*)advice, selectors, 1ull << c->phys.k, ncols, cnt, c->st),
              "k_check_physical");
        const auto& bp = c->phys.bp[phase];
        const uint32_t nb = (uint32_t)std::min<uint64_t>(bp.size(), ncols ? ncols - 1 : 0);
        if (nb) {
            ensure_buf(c, c->chkg, nb * sizeof(uint64_t));
            hipck(hipMemcpyAsync(c->chkg.p, bp.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, c->st),
                  "H2D");
            hipck(launch_check_breaks((const Fr*)advice, 1ull << c->phys.k, (const uint64_t*)c->chkg.p, nb,
                                      cnt + 4, c->st), "k_check_breaks");
        }
        unsigned long long h[6];
        hipck(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, c->st), "D2H");
        hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");
        out->gates_checked = h[0];
        out->gate_failures = h[1];
        out->copies_checked = h[4];
        out->copy_failures = h[5];
    });
}
int svdw_equalities(const svdw_ctx* c, uint32_t phase, uint64_t* copies, uint64_t copies_cap,
                    uint64_t* n_copies, uint64_t* consts, uint64_t consts_cap, uint64_t* n_consts) {
    return guarded([&] {
        REQUIRE(c && phase < 2 && n_copies && n_consts, "bad argument");
        if (!c->dry) {                       // generated on the device, copied out up to the caps
            svdw_ctx* m = const_cast<svdw_ctx*>(c);
            sync(m);
            eq_gen_device(m, phase, n_copies, n_consts);
            if (copies && copies_cap)
                hipck(hipMemcpy(copies, m->eq_cp.p, std::min(copies_cap, *n_copies) * 16, hipMemcpyDeviceToHost), "D2H");
            if (consts && consts_cap)
                hipck(hipMemcpy(consts, m->eq_ks.p, std::min(consts_cap, *n_consts) * 40, hipMemcpyDeviceToHost), "D2H");
            return;
        }
        std::vector<uint64_t> cp, cs;
        eq_lists(c, phase, &cp, &cs);
        *n_copies = cp.size() / 2;
        *n_consts = cs.size() / 5;
        if (copies) memcpy(copies, cp.data(), std::min<uint64_t>(copies_cap, cp.size() / 2) * 16);
        if (consts) memcpy(consts, cs.data(), std::min<uint64_t>(consts_cap, cs.size() / 5) * 40);
    });
}
int svdw_check_equalities(svdw_ctx* c, uint32_t phase, const void* columns0, const void* columns1,
                          svdw_eq_check* out) {
    return guarded([&] {
        REQUIRE(c && phase < 2 && out, "bad argument");
        REQUIRE(!c->dry, "svdw_check_equalities needs a device context");
        // a record's source and destination cells may lie in other ranks' rows,
        // which this context never wrote (svdw_check_gates checks a rank's own)
        REQUIRE(!sharded(c), "svdw_check_equalities: not on a row-sharded context (its streams hold "
                             "this rank's rows only; check the reassembled witness, or use svdw_check_gates)");
        const bool phys = columns0 || columns1;
        REQUIRE(!phys || (c->phys.valid && (phase == 0 ? columns0 != nullptr : columns0 && columns1)),
                "svdw_check_equalities: physical columns need svdw_physical_layout and phase 0's "
                "columns (and phase 1's for phase 1)");
        memset(out, 0, sizeof *out);
        sync(c);
        uint64_t nc = 0, nk = 0;
        eq_gen_device(c, phase, &nc, &nk);
        if (phys) {                          // records onto the assigned columns
            const auto& s0 = c->phys.start[0];
            const auto& s1 = c->phys.start[1];
            ensure_buf(c, c->eq_st, (s0.size() + s1.size() + 1) * sizeof(uint64_t));
            uint64_t* st = (uint64_t*)c->eq_st.p;
            if (!s0.empty()) hipck(hipMemcpyAsync(st, s0.data(), s0.size() * 8, hipMemcpyHostToDevice, c->st), "H2D");
            if (!s1.empty())
                hipck(hipMemcpyAsync(st + s0.size(), s1.data(), s1.size() * 8, hipMemcpyHostToDevice, c->st), "H2D");
            hipck(launch_eq_phys((uint64_t*)c->eq_cp.p, nc, (uint64_t*)c->eq_ks.p, nk, st, (uint32_t)s0.size(),
                                 st + s0.size(), (uint32_t)s1.size(), phase, c->phys.k, c->st), "k_eq_phys");
        }
        const Fr* s0 = phys ? (const Fr*)columns0 : c->ph[0].adv;
        const Fr* s1 = phys ? (const Fr*)columns1 : c->ph[1].adv;
        const Fr* dst = phase ? s1 : s0;
        ensure_buf(c, c->chk, 6 * sizeof(unsigned long long));
        unsigned long long* cnt = (unsigned long long*)c->chk.p;
        hipck(hipMemsetAsync(cnt, 0, 6 * sizeof(unsigned long long), c->st), "hipMemsetAsync");
        hipck(launch_check_copies(s0, s1, dst, (const uint64_t*)c->eq_cp.p, nc, c->ext_gamma, cnt, c->st),
              "k_check_copies");
        hipck(launch_check_consts(dst, (const uint64_t*)c->eq_ks.p, nk, cnt + 2, c->st), "k_check_consts");
        unsigned long long h[4];
        hipck(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, c->st), "D2H");
        hipck(hipStreamSynchronize(c->st), "hipStreamSynchronize");
        out->copies_checked = h[0];
        out->copy_failures = h[1];
        out->consts_checked = h[2];
        out->const_failures = h[3];
    });
}
int svdw_rlc_trace(const svdw_ctx* c, uint64_t* cells, uint64_t* copies, uint32_t* n) {
    return guarded([&] {
        REQUIRE(c && n, "null argument");
        *n = c->rlc.n;
        if (!c->rlc.n) return;
        REQUIRE(cells && copies, "null output");
        for (uint32_t k = 0; k < c->rlc.n; ++k)
            for (int w = 0; w < 4; ++w)
                cells[4 * k + w] = (uint64_t)c->rlc.cells[k].w[2 * w] | (uint64_t)c->rlc.cells[k].w[2 * w + 1] << 32;
        copies[0] = c->rlc.src[0];
        copies[1] = c->rlc.src[1];
    });
}
int svdw_layout(const svdw_ctx* c, svdw_region* out, uint64_t cap, uint64_t* n) {
    return guarded([&] {
        REQUIRE(c && n, "null argument");
        *n = c->layout.size();
        for (uint64_t i = 0; i < cap && i < c->layout.size(); ++i) out[i] = c->layout[i];
    });
}
int svdw_shard_segments(const svdw_ctx* c, svdw_segment* out, uint64_t cap, uint64_t* n) {
    return guarded([&] {
        REQUIRE(c && n, "null argument");
        *n = c->owned.size();
        for (uint64_t i = 0; i < c->owned.size() && i < cap && out; ++i)
            out[i] = svdw_segment{c->owned[i].phase, c->owned[i].lookup, c->owned[i].off,
                                  c->owned[i].n};
    });
}
int svdw_abi_version(void) { return SVDW_ABI_VERSION; }
int svdw_set_option(svdw_ctx* c, const char* name, int64_t value) {
    return guarded([&] {
        REQUIRE(c && name, "null argument");
        sync(c);
        ++c->epoch;                                  // a captured launch sequence may change
        const std::string n(name);
        if (n == "lanes") {                          // verify_mul_witness on two alternating states
            REQUIRE(value == 1 || value == 2, "lanes: 1 or 2");
            c->lanes = (int)value;
        } else if (n == "pipeline") {                // pipelined svd_witness (svd_witness)
            REQUIRE(value == 0 || value == 1, "pipeline: 0 or 1");
            c->pipeline = (int)value;
            if (!value) {                            // the other cell set is not needed any more
                release_alt(c);
                if (c->lane) release_alt(c->lane);
            }
        } else if (n == "vm_linear") {               // captured verify_mul_witness on one stream
            REQUIRE(value == 0 || value == 1, "vm_linear: 0 or 1");
            c->vm_linear = (int)value;
        } else if (n == "graph") {                   // captured verify_mul_witness (vm_graph)
            REQUIRE(value == 0 || value == 1, "graph: 0 or 1");
            c->graph_vm = (int)value;
        } else if (n == "gemm_impl") {
            REQUIRE(value == SVDW_GEMM_MFMA || value == SVDW_GEMM_VALU, "gemm_impl: 0 (mfma) or 1 (valu)");
            c->gemm_impl = (int)value;
        } else if (n == "stage_elems") {
            REQUIRE(value >= 16 && value <= 256 && value % 16 == 0,
                    "stage_elems: a multiple of 16 in [16, 256]");
            c->stage_elems = (uint32_t)value;
        } else if (n == "prod_cell") {
            REQUIRE(value >= -1 && value <= 1, "prod_cell: -1, 0 or 1");
            c->prod_cell = (int)value;
        } else if (n == "phase1_overlap") {
            REQUIRE(value >= 0 && value <= 2, "phase1_overlap: 0, 1 or 2");
            c->phase1_overlap = (int)value;
        } else if (n == "hold_us") {         // timing aid: GPU-only schedule of a witness
            REQUIRE(value >= 0 && value <= 100000, "hold_us: 0..100000");
            c->hold_us = (uint32_t)value;
        } else if (n == "rlc_prefix") {
            c->rlc_prefix = value != 0;
        } else if (n == "res_f64") {
            c->res_f64 = value != 0;
        } else if (n == "gemm_crt") {
            REQUIRE(value == 0 || value == 1, "gemm_crt: 0 or 1");
            c->gemm_crt = (int)value;
        } else if (n == "res_wait") {                // pipelined: st2 waits for the residue planes
            REQUIRE(value >= -1 && value <= 1, "res_wait: -1 (auto), 0 or 1");
            c->res_wait = (int)value;
        } else if (n == "place_trials") {            // cell streams >= 256 MiB: best of this many placements
            REQUIRE(value >= 0 && value <= 8, "place_trials: 0..8");
            c->place_trials = (int)value;
        } else if (n == "stage_rot") {               // phase B from a block-dependent window on
            REQUIRE(value == 0 || value == 1, "stage_rot: 0 or 1");
            c->stage_flags = value ? (c->stage_flags | STAGE_ROT) : (c->stage_flags & ~STAGE_ROT);
        } else if (n == "gemm_kern") {               // CRT GEMM kernel variant (bit-identical)
            REQUIRE(value >= -1 && value <= 2, "gemm_kern: -1 (auto), 0, 1 or 2");
            c->gemm_kern = (int)value;
        } else if (n == "stage_batch") {          // small independent stages share k_stage_multi launches
            c->stage_batch = value != 0;
        } else if (n == "f64_views") {
            c->f64_views = value != 0;
        } else if (n == "p1_at") {
            REQUIRE(value >= -1 && value <= 3, "p1_at: -1 (auto), 0, 1, 2 or 3");
            c->p1_at = (int)value;
        } else if (n == "dchk_at") {                 // pipelined: the d checks' stream
            REQUIRE(value >= 0 && value <= 2, "dchk_at: 0 (cell stream), 1 (st2) or 2 (st3)");
            c->dchk_at = (int)value;
        } else if (n == "gamma_at") {                // pipelined: k_gamma_prep's stream
            REQUIRE(value >= -1 && value <= 1, "gamma_at: -1 (auto), 0 (cell stream) or 1 (st3)");
            c->gamma_at = (int)value;
        } else if (n == "overlap") {
            c->overlap = value != 0;
        } else {
            fail(SVDW_EINVAL, "unknown option " + n);
        }
    });
}
int svdw_graph_stats(svdw_ctx* c, uint64_t* captures, uint64_t* replays) {
    return guarded([&] {
        REQUIRE(c && captures && replays, "null argument");
        *captures = c->vmg.captures + (c->lane ? c->lane->vmg.captures : 0);
        *replays = c->vmg.replays + (c->lane ? c->lane->vmg.replays : 0);
    });
}
int svdw_set_gemm_impl(svdw_ctx* c, int impl) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        REQUIRE(impl == SVDW_GEMM_MFMA || impl == SVDW_GEMM_VALU, "unknown GEMM implementation");
        sync(c);
        ++c->epoch;
        c->gemm_impl = impl;
    });
}
int svdw_profile_enable(svdw_ctx* c, int on) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        sync(c);
        for (auto& r : c->recs) { c->pool.push_back(r.e0); c->pool.push_back(r.e1); }
        c->recs.clear();
        c->prof = on != 0;
    });
}
int svdw_profile_filter(svdw_ctx* c, const char* prefix) {
    return guarded([&] {
        REQUIRE(c, "null ctx");
        c->prof_filter = prefix ? prefix : "";
    });
}
int svdw_profile_collect(svdw_ctx* c, svdw_kstat* out, uint32_t cap, uint32_t* n) {
    return guarded([&] {
        REQUIRE(c && n, "null argument");
        sync(c);
        std::vector<svdw_kstat> agg;
        for (auto& r : c->recs) {
            float ms = 0;
            hipck(hipEventElapsedTime(&ms, r.e0, r.e1), "hipEventElapsedTime");
            svdw_kstat* s = nullptr;
            for (auto& x : agg)
                if (r.name == x.name) s = &x;
            if (!s) {
                agg.emplace_back();
                s = &agg.back();
                memset(s, 0, sizeof(*s));
                snprintf(s->name, sizeof(s->name), "%s", r.name.c_str());
            }
            s->launches += 1;
            s->total_ms += ms;
            s->bytes += r.bytes;
            s->ops += r.ops;
            if (ms > s->max_ms) s->max_ms = ms;
            c->pool.push_back(r.e0);
            c->pool.push_back(r.e1);
        }
        c->recs.clear();
        *n = (uint32_t)agg.size();
        if (out)
            for (uint32_t i = 0; i < agg.size() && i < cap; ++i) out[i] = agg[i];
    });
}
int svdw_plan_svd(uint32_t N, uint32_t M, uint32_t p, uint32_t lb, const svdw_svd_config* cfg,
                  svdw_counts* counts) {
    return guarded([&] {
        REQUIRE(cfg && counts, "null argument");
        if (p < 1 || p > 63) fail(SVDW_ERANGE, "precision_bits must be in [1, 63]");
        if (lb < 8 || lb > 63) fail(SVDW_ERANGE, "lookup_bits must be in [8, 63]");
        svdw_ctx plan;
        plan.P = p;
        plan.LB = lb;
        *counts = svd_witness(&plan, nullptr, nullptr, nullptr, nullptr, N, M, false, *cfg, fr_zero());
    });
}

}  // extern "C"
