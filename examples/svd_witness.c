/*
 * svd_witness.c — C caller of the engine, the witness part of the reference's
 * examples/svd_example.rs (do_zk_svd -> virtual_assign_phase0/1).
 *
 *   gcc examples/svd_witness.c -Iinclude -Lhalo2_svd041_amd -lsvdw -lm \
 *       -Wl,-rpath,$PWD/halo2_svd041_amd -o svd_witness
 *   ./svd_witness [N] [P]            (device 0; N x N input with known SVD)
 *   ./svd_witness data/matrix.in [P] (input-creator.py file, serde_json-default parse)
 *
 * Input: m = u diag(d) v with u, v signed permutations scaled by cos/sin
 * (Givens rotations), so u, v are exactly orthogonal up to f64 rounding.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "svdw.h"

#define CHECK(x)                                                        \
    do {                                                                \
        int rc_ = (x);                                                  \
        if (rc_ != SVDW_OK) {                                           \
            fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, svdw_last_error()); \
            return 1;                                                   \
        }                                                               \
    } while (0)

static void rotation(double* a, uint32_t n, double theta) {
    /* block-diagonal 2x2 rotations */
    for (uint32_t i = 0; i < n * n; ++i) a[i] = 0.0;
    for (uint32_t i = 0; i + 1 < n; i += 2) {
        double c = cos(theta * (i + 1)), s = sin(theta * (i + 1));
        a[i * n + i] = c; a[i * n + i + 1] = -s;
        a[(i + 1) * n + i] = s; a[(i + 1) * n + i + 1] = c;
    }
    if (n % 2) a[(n - 1) * n + n - 1] = 1.0;
}

static char* read_file(const char* path, long* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *len = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* buf = malloc((size_t)*len);
    if (buf && fread(buf, 1, (size_t)*len, f) != (size_t)*len) { free(buf); buf = NULL; }
    fclose(f);
    return buf;
}

int main(int argc, char** argv) {
    uint32_t N = 64, M = 64;
    uint32_t P = argc > 2 ? (uint32_t)atoi(argv[2]) : 42;
    double *u, *v, *m, *d;
    long len = 0;
    char* text = argc > 1 ? read_file(argv[1], &len) : NULL;
    if (text) {                          /* the reference example's input file */
        svdw_input_dims dims;
        CHECK(svdw_parse_svd_input(text, (uint64_t)len, SVDW_PARSE_SERDE, &dims, NULL, NULL, NULL, NULL));
        N = dims.m_rows; M = dims.m_cols;
        m = malloc(sizeof(double) * N * M); u = malloc(sizeof(double) * N * N);
        v = malloc(sizeof(double) * M * M); d = malloc(sizeof(double) * dims.d_len);
        CHECK(svdw_parse_svd_input(text, (uint64_t)len, SVDW_PARSE_SERDE, &dims, m, u, d, v));
        free(text);
    } else {                             /* synthetic N x N with a known SVD */
        if (argc > 1) N = M = (uint32_t)atoi(argv[1]);
        u = malloc(sizeof(double) * N * N);
        v = malloc(sizeof(double) * N * N);
        m = malloc(sizeof(double) * N * N);
        d = malloc(sizeof(double) * N);
        rotation(u, N, 0.3);
        rotation(v, N, 0.7);
        for (uint32_t i = 0; i < N; ++i) d[i] = 50.0 / (1.0 + i);
        for (uint32_t i = 0; i < N; ++i)
            for (uint32_t j = 0; j < N; ++j) {
                double s = 0;
                for (uint32_t k = 0; k < N; ++k) s += u[i * N + k] * d[k] * v[k * N + j];
                m[i * N + j] = s;
            }
    }
    svdw_params p = {0, P, 19};
    svdw_ctx* ctx = NULL;
    CHECK(svdw_ctx_create(&p, &ctx));
    svdw_svd_config cfg = {100.0, 1e-10, 1e-10, 30};
    uint64_t gamma[4] = {0x1234567890abcdefull, 0x0fedcba987654321ull, 0x1111ull, 0x0ull};
    svdw_counts cnt;
    CHECK(svdw_svd_witness(ctx, m, u, v, d, N, M, 0, &cfg, gamma, &cnt));
    CHECK(svdw_sync(ctx));
    printf("N=%u M=%u P=%u advice0=%llu advice1=%llu lookup0=%llu\n", N, M, P,
           (unsigned long long)cnt.advice0, (unsigned long long)cnt.advice1,
           (unsigned long long)cnt.lookup0);
    uint64_t cell[4];
    CHECK(svdw_copy_advice(ctx, 0, 0, 1, cell));   /* quantized m[0][0] */
    printf("advice0[0] = %016llx%016llx%016llx%016llx (m[0][0]=%.17g)\n",
           (unsigned long long)cell[3], (unsigned long long)cell[2],
           (unsigned long long)cell[1], (unsigned long long)cell[0], m[0]);
    /* README.md:93: "SVD should verify on matrix but fail on matrix-wrong" */
    svdw_check_result chk;
    CHECK(svdw_check_gates(ctx, &chk));
    const int ok = chk.gate_failures + chk.copy_failures + chk.lookup_failures == 0;
    printf("constraints: %llu gates (%llu failed), %llu copies (%llu failed), %llu lookups "
           "(%llu failed): SVD %s\n",
           (unsigned long long)chk.gates_checked, (unsigned long long)chk.gate_failures,
           (unsigned long long)chk.copies_checked, (unsigned long long)chk.copy_failures,
           (unsigned long long)chk.lookups_checked, (unsigned long long)chk.lookup_failures,
           ok ? "verifies" : "does NOT verify");
    CHECK(svdw_ctx_destroy(ctx));
    free(u); free(v); free(m); free(d);
    return 0;
}
