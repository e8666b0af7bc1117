// BN254 scalar field Fr for host and gfx950 device code.
//
// Representation: 8 x u32 little-endian limbs. In memory a canonical Fr is
// byte-identical to halo2curves' `Fr::to_repr()` (32-byte little endian),
// which is the cell format of every advice / lookup stream this engine
// writes. Montgomery form (x * 2^256 mod p) is used only inside products:
// mont_mul(a_canonical, b_montgomery) == a*b canonical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SVDW_HD __host__ __device__ __forceinline__

namespace svdw {

struct alignas(16) Fr {
    uint32_t w[8];
};

// p = 21888242871839275222246405745257275088548364400416034343698204186575808495617
#define SVDW_P_WORDS 0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u, \
                     0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u
#define SVDW_R2_WORDS 0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u, \
                      0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u
static constexpr uint32_t kPinv32 = 0xefffffffu;   // -p^-1 mod 2^32

SVDW_HD uint32_t p_word(int i) {
    constexpr uint32_t P[8] = {SVDW_P_WORDS};
    return P[i];
}

SVDW_HD Fr fr_zero() {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = 0;
    return r;
}
SVDW_HD Fr fr_from_u64(uint64_t x) {
    Fr r = fr_zero();
    r.w[0] = (uint32_t)x;
    r.w[1] = (uint32_t)(x >> 32);
    return r;
}
SVDW_HD Fr fr_p() {
    Fr r;
    constexpr uint32_t P[8] = {SVDW_P_WORDS};
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = P[i];
    return r;
}
SVDW_HD Fr fr_r2() {
    Fr r;
    constexpr uint32_t R2[8] = {SVDW_R2_WORDS};
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = R2[i];
    return r;
}
SVDW_HD bool fr_is_zero(const Fr& a) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x |= a.w[i];
    return x == 0;
}
SVDW_HD bool fr_eq(const Fr& a, const Fr& b) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x |= a.w[i] ^ b.w[i];
    return x == 0;
}

// Carry chains: __builtin_addc / __builtin_subc lower to v_add_co_u32 /
// v_addc_co_u32 (v_sub_co / v_subb_co) on gfx950, one instruction per word.
// The 64-bit "c += a + b; c >>= 32" idiom instead compiles to v_lshl_add_u64
// plus a v_mov per word to zero the high half (3-4x the instructions).
SVDW_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t& c) {
    unsigned co;
    const uint32_t r = __builtin_addc(a, b, c, &co);
    c = co;
    return r;
}
SVDW_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t& br) {
    unsigned bo;
    const uint32_t r = __builtin_subc(a, b, br, &bo);
    br = bo;
    return r;
}
// r = a - b over 256 bits; returns borrow.
SVDW_HD uint32_t sub256(Fr& r, const Fr& a, const Fr& b) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = subb32(a.w[i], b.w[i], br);
    return br;
}
// r = a + b over 256 bits; returns carry.
SVDW_HD uint32_t add256(Fr& r, const Fr& a, const Fr& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = addc32(a.w[i], b.w[i], c);
    return c;
}
// r = a - p over 256 bits; returns borrow.
SVDW_HD uint32_t sub_p(Fr& r, const Fr& a) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = subb32(a.w[i], p_word(i), br);
    return br;
}

// Canonical modular add/sub (inputs canonical, output canonical).
SVDW_HD Fr fr_add(const Fr& a, const Fr& b) {
    Fr s, t;
    uint32_t c = add256(s, a, b);
    uint32_t br = sub_p(t, s);
    // keep t if (carry) or (no borrow): s >= p
    bool use_t = c | (br ^ 1u);
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = use_t ? t.w[i] : s.w[i];
    return r;
}
SVDW_HD Fr fr_sub(const Fr& a, const Fr& b) {
    Fr d, t;
    uint32_t br = sub256(d, a, b);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t.w[i] = addc32(d.w[i], p_word(i), c);
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = br ? t.w[i] : d.w[i];
    return r;
}
SVDW_HD Fr fr_neg(const Fr& a) { return fr_sub(fr_zero(), a); }

// t + a*b + c as (lo, new carry c): one v_mad_u64_u32 (a*b + t < 2^64 - 2^32)
// and an add-with-carry of c.
SVDW_HD uint32_t mac32(uint32_t a, uint32_t b, uint32_t t, uint32_t& c) {
    const uint64_t pr = (uint64_t)a * b + t;
    uint32_t cy = 0;
    const uint32_t lo = addc32((uint32_t)pr, c, cy);
    c = (uint32_t)(pr >> 32) + cy;
    return lo;
}
// NR rounds of CIOS Montgomery multiplication, one per word of `a`:
// a * b * 2^(-32 NR) mod p for a < 2^(32 NR), b < p. Output canonical.
template <int NR>
SVDW_HD Fr mont_mul_rounds(const Fr& a, const Fr& b) {
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        uint32_t c = 0, cy = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = mac32(b.w[j], a.w[i], t[j], c);
        t[8] = addc32(t[8], c, cy);
        t[9] = cy;
        const uint32_t m = t[0] * kPinv32;
        c = 0;
        (void)mac32(m, p_word(0), t[0], c);               // low word cancels
#pragma unroll
        for (int j = 1; j < 8; ++j) t[j - 1] = mac32(m, p_word(j), t[j], c);
        cy = 0;
        t[7] = addc32(t[8], c, cy);
        t[8] = t[9] + cy;
    }
    Fr r, s;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = t[i];
    const uint32_t br = sub_p(s, r);
    const bool use_s = t[8] | (br ^ 1u);
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = use_s ? s.w[i] : r.w[i];
    return r;
}
// Montgomery product a*b*2^-256 mod p (CIOS, 32-bit limbs). Output canonical
// (< p) for inputs < p.
SVDW_HD Fr mont_mul(const Fr& a, const Fr& b) { return mont_mul_rounds<8>(b, a); }
// a * b * 2^(-32 NA) mod p for a < 2^(32 NA) (words >= NA of `a` ignored):
// CIOS with NA outer rounds, one per word of the small operand. Output < p.
template <int NA>
SVDW_HD Fr mont_mul_small(const Fr& a, const Fr& b) { return mont_mul_rounds<NA>(a, b); }
// a * b mod p for a canonical `a` whose signed value (a or a - p) has magnitude
// < 2^(32 NA), with bs = b * 2^(32 NA) mod p.
template <int NA>
SVDW_HD Fr fr_mul_small_signed(const Fr& a, const Fr& bs) {
    Fr n, d;
    sub256(n, fr_p(), a);                       // p - a
    const uint32_t neg = sub256(d, n, a);       // p - a < a: a is negative
    Fr mag;
#pragma unroll
    for (int i = 0; i < 8; ++i) mag.w[i] = neg ? n.w[i] : a.w[i];
    const Fr r = mont_mul_small<NA>(mag, bs);
    const Fr nr = fr_neg(r);
    Fr o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.w[i] = neg ? nr.w[i] : r.w[i];
    return o;
}
SVDW_HD Fr fr_to_mont(const Fr& a) { return mont_mul(a, fr_r2()); }
SVDW_HD Fr fr_from_mont(const Fr& a) { return mont_mul(a, fr_from_u64(1)); }
// Canonical product.
SVDW_HD Fr fr_mul(const Fr& a, const Fr& b) { return mont_mul(mont_mul(a, b), fr_r2()); }

// a^e for canonical a (square and multiply over the low `nbits` bits of e).
SVDW_HD Fr fr_pow_u64(const Fr& a, uint64_t e, int nbits = 64) {
    Fr am = fr_to_mont(a);
    Fr r = fr_to_mont(fr_from_u64(1));
    for (int i = nbits - 1; i >= 0; --i) {
        r = mont_mul(r, r);
        if ((e >> i) & 1) r = mont_mul(r, am);
    }
    return fr_from_mont(r);
}
// a^-1 (a^(p-2)); 0 -> 0.
SVDW_HD Fr fr_inv(const Fr& a) {
    Fr e = fr_p();
    e.w[0] -= 2;   // p - 2 (no borrow: low word is 0xf0000001)
    Fr am = fr_to_mont(a);
    Fr r = fr_to_mont(fr_from_u64(1));
    for (int wi = 7; wi >= 0; --wi) {
        // select chain instead of e.w[wi]: a runtime index would spill e to scratch
        uint32_t word = e.w[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) word = (wi == k) ? e.w[k] : word;
        for (int b = 31; b >= 0; --b) {
            r = mont_mul(r, r);
            if ((word >> b) & 1) r = mont_mul(r, am);
        }
    }
    return fr_from_mont(r);
}
// Signed two's-complement integer of `nw` 32-bit words (little endian, value
// |x| < 2^(32*nw - 1) < p) to canonical Fr.
template <int NW>
SVDW_HD Fr fr_from_signed_words(const uint32_t (&x)[NW]) {
    bool neg = (x[NW - 1] >> 31) & 1;
    Fr mag = fr_zero();
    uint64_t c = neg ? 1 : 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        uint32_t v = neg ? ~x[i] : x[i];
        c += v;
        mag.w[i] = (uint32_t)c;
        c >>= 32;
    }
    return neg ? fr_sub(fr_zero(), mag) : mag;
}

}  // namespace svdw
