/*
 * svdw_oracle.c — single-threaded C restatement of the reference's
 * SVD-verify witness path. TEST INFRASTRUCTURE ONLY: loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker
 * and the reported CPU baseline. Never linked into the product.
 *
 * Follows (reference repo paths):
 *   src/matrix/mod.rs:29-40    ZkVector::new         -> orc_load_vec
 *   src/matrix/mod.rs:185-215  entries_less_than / entries_in_desc_order
 *   src/matrix/mod.rs:230-252  ZkMatrix::new         -> orc_load_mat
 *   src/matrix/mod.rs:299-342  ZkMatrix::verify_mul  -> orc_verify_mul
 *   src/matrix/mod.rs:425-501  check_abs_less_than / check_mat_diff / check_mat_id /
 *                              check_mat_entries_bounded
 *   src/matrix/mod.rs:510-568  field_mat_mul (naive i-j-k, column-strided b)
 *                              / honest_prover_mat_mul
 *   src/matrix/mod.rs:574-627  field_mat_vec_mul / mat_times_diag_mat
 *   src/svd/mod.rs:32-163      check_svd_phase0 / check_svd_phase1 / err_calc
 *   halo2-base 0.4.1 [ext]     gate and range layouts
 *   zk_fixed_point_chip [ext]  quantization
 *
 * Like halo2curves, field values are kept in Montgomery form internally and
 * converted to canonical little-endian (to_repr) on output; every field
 * product in the GEMM is one Montgomery multiplication, as in the reference.
 * Pinning: see oracle/pyoracle.py header (counts README.md:67, KAT README.md:93).
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;   /* Montgomery form */

static const uint64_t P64[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull,
                                0xb85045b68181585dull, 0x30644e72e131a029ull};
static const uint64_t R2[4] = {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull,
                               0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull};
static const uint64_t PINV = 0xc2e1f593efffffffull;

/* ------------------------------------------------------------------ field */
static int geq_p(const uint64_t a[4]) {
    for (int i = 3; i >= 0; --i) {
        if (a[i] > P64[i]) return 1;
        if (a[i] < P64[i]) return 0;
    }
    return 1;
}
static void sub_p(uint64_t a[4]) {
    u128 br = 0;
    for (int i = 0; i < 4; ++i) {
        u128 t = (u128)a[i] - P64[i] - br;
        a[i] = (uint64_t)t;
        br = (t >> 64) & 1;
    }
}
static fe fe_add(fe a, fe b) {
    fe r; u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)a.v[i] + b.v[i]; r.v[i] = (uint64_t)c; c >>= 64; }
    if (c || geq_p(r.v)) sub_p(r.v);
    return r;
}
static fe fe_sub(fe a, fe b) {
    fe r; u128 br = 0;
    for (int i = 0; i < 4; ++i) {
        u128 t = (u128)a.v[i] - b.v[i] - br;
        r.v[i] = (uint64_t)t; br = (t >> 64) & 1;
    }
    if (br) {
        u128 c = 0;
        for (int i = 0; i < 4; ++i) { c += (u128)r.v[i] + P64[i]; r.v[i] = (uint64_t)c; c >>= 64; }
    }
    return r;
}
static fe fe_mul(fe a, fe b) {   /* CIOS Montgomery, 4x64 */
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a.v[j] * b.v[i] + t[j];
            t[j] = (uint64_t)c; c >>= 64;
        }
        c += t[4]; t[4] = (uint64_t)c; t[5] = (uint64_t)(c >> 64);
        uint64_t m = t[0] * PINV;
        c = (u128)m * P64[0] + t[0]; c >>= 64;
        for (int j = 1; j < 4; ++j) {
            c += (u128)m * P64[j] + t[j];
            t[j - 1] = (uint64_t)c; c >>= 64;
        }
        c += t[4]; t[3] = (uint64_t)c; t[4] = t[5] + (uint64_t)(c >> 64);
    }
    fe r; memcpy(r.v, t, 32);
    if (t[4] || geq_p(r.v)) sub_p(r.v);
    return r;
}
static fe fe_from_canon(const uint64_t c[4]) { fe a; memcpy(a.v, c, 32); fe r2; memcpy(r2.v, R2, 32); return fe_mul(a, r2); }
static void fe_to_canon(fe a, uint64_t out[4]) { fe one = {{1, 0, 0, 0}}; fe r = fe_mul(a, one); memcpy(out, r.v, 32); }
static fe fe_zero(void) { fe z = {{0, 0, 0, 0}}; return z; }
static fe fe_u128(u128 x) { uint64_t c[4] = {(uint64_t)x, (uint64_t)(x >> 64), 0, 0}; return fe_from_canon(c); }
static fe fe_one(void) { return fe_u128(1); }
static int fe_is_zero(fe a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3]); }
static int fe_eq(fe a, fe b) { return !memcmp(a.v, b.v, 32); }
static fe fe_pow2(unsigned k) { uint64_t c[4] = {0, 0, 0, 0}; c[k / 64] = 1ull << (k % 64); return fe_from_canon(c); }
static fe fe_inv(fe a) {  /* a^(p-2) */
    uint64_t e[4]; memcpy(e, P64, 32); e[0] -= 2;
    fe r = fe_one(), b = a;
    for (int i = 0; i < 256; ++i) {
        if ((e[i / 64] >> (i % 64)) & 1) r = fe_mul(r, b);
        b = fe_mul(b, b);
    }
    return r;
}

/* ------------------------------------------------- small unsigned bigints */
typedef struct { uint64_t v[4]; } big;   /* non-modular, < 2^256 */
static big big_u128(u128 x) { big b = {{(uint64_t)x, (uint64_t)(x >> 64), 0, 0}}; return b; }
static int big_bits(big b) {
    for (int i = 3; i >= 0; --i) if (b.v[i]) return 64 * i + 64 - __builtin_clzll(b.v[i]);
    return 0;
}
static big big_add_small(big b, int64_t s) {  /* b + s, s may be negative */
    u128 c = (u128)(uint64_t)s; uint64_t ext = s < 0 ? ~0ull : 0;
    big r;
    for (int i = 0; i < 4; ++i) {
        c += (u128)b.v[i] + (i ? ext : 0);
        r.v[i] = (uint64_t)c; c >>= 64;
    }
    return r;
}
static big big_shl1(big b) {
    big r;
    for (int i = 3; i > 0; --i) r.v[i] = (b.v[i] << 1) | (b.v[i - 1] >> 63);
    r.v[0] = b.v[0] << 1;
    return r;
}
static fe fe_big(big b) { return fe_from_canon(b.v); }  /* b < p assumed */

/* --------------------------------------------------------------- context */
typedef struct {
    fe *adv; size_t n, cap;
    fe *lk; size_t nl, lcap;
    int lb;
} octx;

static void ctx_init(octx *c, int lb) { memset(c, 0, sizeof *c); c->lb = lb; }
static void ctx_free(octx *c) { free(c->adv); free(c->lk); }
static size_t push(octx *c, fe v) {
    if (c->n == c->cap) { c->cap = c->cap ? 2 * c->cap : 1024; c->adv = (fe *)realloc(c->adv, c->cap * sizeof(fe)); }
    c->adv[c->n] = v;
    return c->n++;
}
static void push_lk(octx *c, fe v) {
    if (c->nl == c->lcap) { c->lcap = c->lcap ? 2 * c->lcap : 1024; c->lk = (fe *)realloc(c->lk, c->lcap * sizeof(fe)); }
    c->lk[c->nl++] = v;
}
#define VAL(c, i) ((c)->adv[(i)])

/* ------------------------------------------------ GateChip (halo2-base) */
static size_t g_add(octx *c, fe a, fe b) {            /* [a, b, 1, a+b] */
    push(c, a); push(c, b); push(c, fe_one());
    return push(c, fe_add(a, b));
}
static size_t g_sub(octx *c, fe a, fe b) {            /* [a-b, b, 1, a] */
    size_t r = push(c, fe_sub(a, b)); push(c, b); push(c, fe_one()); push(c, a);
    return r;
}
static size_t g_mul(octx *c, fe a, fe b) {            /* [0, a, b, a*b] */
    push(c, fe_zero()); push(c, a); push(c, b);
    return push(c, fe_mul(a, b));
}
/* inner_product with b not starting with Constant(1): [0, a0, b0, s0, ...] */
static size_t g_inner_product(octx *c, const size_t *a, size_t as, const fe *b, size_t n) {
    fe s = fe_zero();
    push(c, fe_zero());
    size_t last = 0;
    for (size_t i = 0; i < n; ++i) {
        fe av = VAL(c, a[i * as]);
        s = fe_add(s, fe_mul(av, b[i]));
        push(c, av); push(c, b[i]); last = push(c, s);
    }
    return last;
}
static void g_is_equal(octx *c, fe a, fe b) {
    size_t d = g_sub(c, a, b);
    fe x = VAL(c, d), z, inv;
    if (fe_is_zero(x)) { z = fe_one(); inv = fe_one(); } else { z = fe_zero(); inv = fe_inv(x); }
    push(c, z); push(c, x); push(c, inv); push(c, fe_one());
    push(c, fe_zero()); push(c, x); push(c, z); push(c, fe_zero());
}

/* ------------------------------------------------ RangeChip (halo2-base) */
static void range_check(octx *c, size_t a_idx, int range_bits) {
    const int lb = c->lb;
    if (range_bits == 0) return;               /* assert_is_const: no cells */
    int n = (range_bits + lb - 1) / lb, rem = range_bits % lb;
    fe last;
    if (n == 1) {
        last = VAL(c, a_idx);
        push_lk(c, last);
    } else {
        uint64_t cv[4]; fe_to_canon(VAL(c, a_idx), cv);
        const uint64_t mask = lb == 64 ? ~0ull : ((1ull << lb) - 1);
        /* inner_product(limbs, [1, 2^lb, ...]) with leading-1 elision */
        fe s = fe_zero();
        for (int i = 0; i < n; ++i) {
            int lo = i * lb, w = lo / 64, sh = lo % 64;
            uint64_t x = w < 4 ? cv[w] >> sh : 0;
            if (sh && w + 1 < 4) x |= cv[w + 1] << (64 - sh);
            x &= mask;
            fe limb = fe_u128(x);
            if (i == 0) { s = limb; push(c, limb); }
            else {
                s = fe_add(s, fe_mul(limb, fe_pow2((unsigned)lo)));
                push(c, limb); push(c, fe_pow2((unsigned)lo)); push(c, s);
            }
            push_lk(c, limb);
            last = limb;
        }
    }
    if (rem == 1) {
        push(c, fe_zero()); push(c, last); push(c, last); push(c, last);
    } else if (rem > 1) {
        size_t k = g_mul(c, last, fe_pow2((unsigned)(lb - rem)));
        push_lk(c, VAL(c, k));
    }
}
static void check_less_than(octx *c, fe a, fe b, int bits) {
    fe pw = fe_pow2((unsigned)bits), shift = fe_add(pw, a);
    size_t r = push(c, fe_sub(shift, b));
    push(c, b); push(c, fe_one()); push(c, shift);
    push(c, fe_sub(fe_zero(), pw)); push(c, fe_one()); push(c, a);
    range_check(c, r, bits);
}
static void check_big_less_than_safe(octx *c, size_t a_idx, big bnd) {
    int rb = (big_bits(bnd) + c->lb - 1) / c->lb * c->lb;
    range_check(c, a_idx, rb);
    check_less_than(c, VAL(c, a_idx), fe_big(bnd), rb);
}
/* src/matrix/mod.rs:425-435 */
static void check_abs_less_than(octx *c, fe x, big bnd) {
    big nb = big_add_small(big_shl1(bnd), -1);
    size_t t = g_add(c, x, fe_big(big_add_small(bnd, -1)));
    check_big_less_than_safe(c, t, nb);
}

/* ------------------------------------------------ quantization / err_calc */
static u128 f64_to_u128_sat(double x) {
    if (!(x > 0)) return 0;                    /* NaN, 0, negative */
    if (x >= 340282366920938463463374607431768211456.0) return ~(u128)0;
    return (u128)x;
}
static fe quantize(double x, int p) {
    int neg = !isnan(x) && signbit(x);
    u128 xq = f64_to_u128_sat(round(fabs(x) * ldexp(1.0, p)));  /* round(): ties away */
    fe q = fe_u128(xq);
    return neg ? fe_sub(fe_zero(), q) : q;
}
void orc_err_calc(int p, size_t size, double max_norm, double eps_svd, double eps_u,
                  double *err_svd, double *err_u) {   /* src/svd/mod.rs:155-163 */
    double precision = pow(2.0, -1.0 * ((double)p + 1.0));
    double s = (double)size;
    *err_svd = precision * s * (1.0 + max_norm + eps_svd + precision)
             + s * max_norm * precision
             + pow(1.0 + eps_u, 0.5) * (max_norm + eps_svd) * eps_u
             + pow(1.0 + eps_u, 0.5) * eps_svd;
    *err_u = eps_u + precision * s * (2.0 * (1.0 + eps_u) + precision);
}
static u128 scale_err(double err, int p) { return f64_to_u128_sat(round(err * ldexp(1.0, 2 * p))); }

/* ------------------------------------------------ matrix layer */
/* A ZkMatrix is rows x cols cell indices (Vec<Vec<AssignedValue>>). */
typedef struct { size_t *idx; size_t rows, cols; } omat;
static omat mat_alloc(size_t r, size_t cl) { omat m = {(size_t *)malloc(r * cl * sizeof(size_t)), r, cl}; return m; }
#define AT(m, i, j) ((m).idx[(i) * (m).cols + (j)])

static omat orc_load_mat(octx *c, const double *x, size_t r, size_t cl, int p) {
    omat m = mat_alloc(r, cl);
    for (size_t i = 0; i < r * cl; ++i) m.idx[i] = push(c, quantize(x[i], p));
    return m;
}
static omat transpose(omat a) {
    omat t = mat_alloc(a.cols, a.rows);
    for (size_t i = 0; i < a.cols; ++i)
        for (size_t j = 0; j < a.rows; ++j) AT(t, i, j) = AT(a, j, i);
    return t;
}
/* the rows a sampled witness computes of every row-parallel stage: [rb, re) */
typedef struct { size_t rb, re; } rwin;
static int in_win(rwin w, size_t i) { return i >= w.rb && i < w.re; }
/* field_mat_mul + load_witness (src/matrix/mod.rs:510-568), rows of the window */
static omat honest_prover_mat_mul(octx *c, omat a, omat b, rwin w) {
    omat cs = mat_alloc(a.rows, b.cols);
    for (size_t i = 0; i < a.rows; ++i)
        for (size_t j = 0; j < b.cols; ++j) {
            if (!in_win(w, i)) { AT(cs, i, j) = 0; continue; }
            fe e = fe_zero();
            for (size_t k = 0; k < a.cols; ++k)
                e = fe_add(e, fe_mul(VAL(c, AT(a, i, k)), VAL(c, AT(b, k, j))));
            AT(cs, i, j) = push(c, e);
        }
    return cs;
}
static void check_mat_diff_val(octx *c, omat a, const fe *bvals, omat b, rwin w, big tol) {
    for (size_t i = w.rb; i < a.rows && i < w.re; ++i)
        for (size_t j = 0; j < a.cols; ++j) {
            fe bv = bvals ? bvals[i == j ? 0 : 1] : VAL(c, AT(b, i, j));
            size_t d = g_sub(c, VAL(c, AT(a, i, j)), bv);
            check_abs_less_than(c, VAL(c, d), tol);
        }
}

/* ------------------------------------------------ SVD driver */
typedef struct {
    fe *adv; size_t n;   /* unused in API; kept for clarity */
} unused_t;

static void out_cells(octx *c, uint64_t **adv, size_t *na, uint64_t **lk, size_t *nl) {
    if (adv) {
        *adv = (uint64_t *)malloc((c->n ? c->n : 1) * 32);
        for (size_t i = 0; i < c->n; ++i) fe_to_canon(c->adv[i], *adv + 4 * i);
        *na = c->n;
    }
    if (lk) {
        *lk = (uint64_t *)malloc((c->nl ? c->nl : 1) * 32);
        for (size_t i = 0; i < c->nl; ++i) fe_to_canon(c->lk[i], *lk + 4 * i);
        *nl = c->nl;
    }
}

static void verify_mul(octx *c, octx *c0, omat a, omat b, omat cs, fe gamma, rwin w) {
    size_t d = cs.cols;
    fe *v = (fe *)malloc(d * sizeof(fe));
    { size_t k = push(c, fe_one()); v[0] = VAL(c, k); }      /* load_witness(1) */
    for (size_t i = 1; i < d; ++i) { size_t k = g_mul(c, v[i - 1], gamma); v[i] = VAL(c, k); }
    /* field_mat_vec_mul reads phase-0 cells (cross-context copies) */
    fe *csv = (fe *)malloc(cs.rows * sizeof(fe)), *bv = (fe *)malloc(b.rows * sizeof(fe));
    fe *abv = (fe *)malloc(a.rows * sizeof(fe));
    octx tmp; ctx_init(&tmp, c->lb);
#define IP_ROWS(M, VEC, OUT, W)                                                \
    for (size_t r = 0; r < (M).rows; ++r) {                                    \
        octx *dst = in_win((W), r) ? c : &tmp;                                 \
        tmp.n = 0;                                                             \
        fe s = fe_zero(); push(dst, fe_zero());                                \
        for (size_t j = 0; j < (M).cols; ++j) {                                \
            fe av = VAL(c0, AT(M, r, j));                                      \
            s = fe_add(s, fe_mul(av, (VEC)[j]));                               \
            push(dst, av); push(dst, (VEC)[j]); push(dst, s);                  \
        }                                                                      \
        (OUT)[r] = s;                                                          \
    }
    IP_ROWS(cs, v, csv, w)
    IP_ROWS(b, v, bv, w)
    IP_ROWS(a, bv, abv, w)
#undef IP_ROWS
    for (size_t r = w.rb; r < a.rows && r < w.re; ++r) g_is_equal(c, csv[r], abv[r]);
    ctx_free(&tmp);
    free(v); free(csv); free(bv); free(abv);
}

/*
 * Whole witness of examples/svd_example.rs:98-200 with the intended one-context
 * semantics. gamma: canonical 4x u64. row_begin / row_lim limit every
 * row-parallel stage to its rows [row_begin, row_begin + row_lim) (CPU-baseline
 * sampling, and the full-size parity of any row-sharded rank's rows; 0 /
 * SIZE_MAX = the full witness); every other region is computed in full.
 * Outputs are malloc'd canonical cells (4 x u64 each); free with orc_free.
 */
int orc_svd_witness(const double *m, const double *u, const double *v, const double *d,
                    size_t N, size_t M, int p, int lb, const uint64_t gamma_c[4],
                    double max_norm, double eps_svd, double eps_u, int max_bits_d,
                    size_t row_begin, size_t row_lim,
                    uint64_t **adv0, size_t *n0, uint64_t **lk0, size_t *nl0,
                    uint64_t **adv1, size_t *n1) {
    if (p < 1 || p > 63 || lb < 1 || lb > 63 || !N || !M) return -1;
    size_t r = N < M ? N : M;
    rwin w = {row_begin, row_lim > SIZE_MAX - row_begin ? SIZE_MAX : row_begin + row_lim};
    octx c0; ctx_init(&c0, lb);
    omat zm = orc_load_mat(&c0, m, N, M, p);
    omat zu = orc_load_mat(&c0, u, N, N, p);
    omat zv = orc_load_mat(&c0, v, M, M, p);
    size_t *zd = (size_t *)malloc(r * sizeof(size_t));
    for (size_t i = 0; i < r; ++i) zd[i] = push(&c0, quantize(d[i], p));
    double err_svd, err_u;
    orc_err_calc(p, N > M ? N : M, max_norm, eps_svd, eps_u, &err_svd, &err_u);

    /* --- check_svd_phase0 (src/svd/mod.rs:32-116) --- */
    int max_bits = max_bits_d + p;
    for (size_t i = 0; i < r; ++i) range_check(&c0, zd[i], max_bits);
    size_t *dd = (size_t *)malloc((r ? r : 1) * sizeof(size_t));
    for (size_t i = 0; i + 1 < r; ++i) dd[i] = g_sub(&c0, VAL(&c0, zd[i]), VAL(&c0, zd[i + 1]));
    for (size_t i = 0; i + 1 < r; ++i) range_check(&c0, dd[i], max_bits);
    big unit = big_u128(((u128)1 << p) + 1);
    for (size_t i = w.rb; i < N && i < w.re; ++i)
        for (size_t j = 0; j < N; ++j) check_abs_less_than(&c0, VAL(&c0, AT(zu, i, j)), unit);
    for (size_t i = w.rb; i < M && i < w.re; ++i)
        for (size_t j = 0; j < M; ++j) check_abs_less_than(&c0, VAL(&c0, AT(zv, i, j)), unit);
    omat ut = transpose(zu), vt = transpose(zv);
    omat ud = mat_alloc(N, M);
    size_t zero_idx = 0;
    if (r != M) zero_idx = push(&c0, fe_zero());
    for (size_t i = 0; i < N; ++i) {
        for (size_t j = 0; j < r; ++j)
            AT(ud, i, j) = in_win(w, i) ? g_mul(&c0, VAL(&c0, AT(zu, i, j)), VAL(&c0, zd[j])) : 0;
        for (size_t j = r; j < M; ++j) AT(ud, i, j) = zero_idx;
    }
    omat mvt = honest_prover_mat_mul(&c0, zm, vt, w);
    big tol_svd = big_u128(scale_err(err_svd, p)), tol_u = big_u128(scale_err(err_u, p));
    if (!big_bits(tol_svd) || !big_bits(tol_u)) return -2;
    check_mat_diff_val(&c0, ud, NULL, mvt, w, tol_svd);
    fe q = fe_pow2((unsigned)p);
    size_t q2i = push(&c0, fe_mul(q, q)); fe q2 = VAL(&c0, q2i);
    omat uut = honest_prover_mat_mul(&c0, zu, ut, w);
    fe idv[2] = {q2, fe_zero()};
    push(&c0, fe_zero());
    check_mat_diff_val(&c0, uut, idv, uut, w, tol_u);
    omat vvt = honest_prover_mat_mul(&c0, zv, vt, w);
    push(&c0, fe_zero());
    check_mat_diff_val(&c0, vvt, idv, vvt, w, tol_u);

    /* --- check_svd_phase1 (src/svd/mod.rs:127-144) --- */
    octx c1; ctx_init(&c1, lb);
    fe gamma = fe_from_canon(gamma_c);
    /* Phase-1 mat-vec rows read the phase-0 payload (cross-phase copies).
       In sampled mode the c_s rows outside the window were not computed (0). */
    verify_mul(&c1, &c0, zm, vt, mvt, gamma, w);
    verify_mul(&c1, &c0, zu, ut, uut, gamma, w);
    verify_mul(&c1, &c0, zv, vt, vvt, gamma, w);

    out_cells(&c0, adv0, n0, lk0, nl0);
    out_cells(&c1, adv1, n1, NULL, NULL);
    ctx_free(&c0); ctx_free(&c1);
    free(zm.idx); free(zu.idx); free(zv.idx); free(zd); free(dd);
    free(ut.idx); free(vt.idx); free(ud.idx); free(mvt.idx); free(uut.idx); free(vvt.idx);
    return 0;
}

/*
 * Matrix-multiplication recipe of README.md:32-46 (BASELINE config 2): phase 0
 * loads a (n x k) and b (k x m) with ZkMatrix::new (src/matrix/mod.rs:230-252),
 * then c_s = honest_prover_mat_mul(a, b) (:546-568); phase 1 runs
 * verify_mul(a, b, c_s, gamma) (:299-342). A dishonest prover is modelled by
 * bw != NULL: a third matrix (k x m) is loaded after b and c_s = a * bw, so
 * every row whose Freivalds sums differ gets non-trivial is_equal cells.
 */
int orc_verify_mul_witness(const double *a, const double *b, const double *bw, size_t n,
                           size_t k, size_t m, int p, const uint64_t gamma_c[4],
                           uint64_t **adv0, size_t *n0, uint64_t **adv1, size_t *n1) {
    if (p < 1 || p > 63 || !n || !k || !m) return -1;
    octx c0; ctx_init(&c0, 19);
    omat za = orc_load_mat(&c0, a, n, k, p);
    omat zb = orc_load_mat(&c0, b, k, m, p);
    omat zw = zb;
    if (bw) zw = orc_load_mat(&c0, bw, k, m, p);
    const rwin all = {0, (size_t)-1};
    omat cs = honest_prover_mat_mul(&c0, za, zw, all);
    octx c1; ctx_init(&c1, 19);
    verify_mul(&c1, &c0, za, zb, cs, fe_from_canon(gamma_c), all);
    out_cells(&c0, adv0, n0, NULL, NULL);
    out_cells(&c1, adv1, n1, NULL, NULL);
    ctx_free(&c0); ctx_free(&c1);
    free(za.idx); free(zb.idx); if (bw) free(zw.idx); free(cs.idx);
    return 0;
}

void orc_free(void *p) { free(p); }

/* Field KAT helpers for tests: canonical in/out. */
void orc_fe_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    fe_to_canon(fe_mul(fe_from_canon(a), fe_from_canon(b)), out);
}
void orc_fe_add(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    fe_to_canon(fe_add(fe_from_canon(a), fe_from_canon(b)), out);
}
void orc_fe_sub(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    fe_to_canon(fe_sub(fe_from_canon(a), fe_from_canon(b)), out);
}
void orc_fe_inv(const uint64_t a[4], uint64_t out[4]) { fe_to_canon(fe_inv(fe_from_canon(a)), out); }
void orc_quantize(double x, int p, uint64_t out[4]) { fe_to_canon(quantize(x, p), out); }
