/*
 * svdw.h — C ABI of the MI355X-native SVD-verify witness engine.
 *
 * Drop-in boundary for the witness path of neilcouture/halo2-svd041: every
 * entry point replaces one reference function that appends BN254-Fr cells to
 * a halo2-base `Context` (citations: reference repo paths). Values are the
 * canonical little-endian 32-byte cells (halo2curves `Fr::to_repr`), stored
 * device-resident in per-phase advice / lookup streams owned by the context.
 * Handles (svdw_mat / svdw_vec) are plain views (offset + strides) into a
 * phase's advice stream, valid for the context's lifetime — the analogue of
 * `Vec<Vec<AssignedValue<F>>>` (src/matrix/mod.rs:219-223), with transpose a
 * stride swap (src/matrix/mod.rs:408-419).
 *
 * Errors: every call returns SVDW_OK or a negative code and never aborts; the
 * reference panics (assert!/assert_eq!) on the same conditions
 * (src/matrix/mod.rs:86,142,175,239,307-310,515,580,616; src/svd/mod.rs:50-61).
 * svdw_last_error() gives the thread-local message of the last failure.
 * Threading: one context = one `&mut Context` per phase; not thread safe.
 * Work is enqueued on the context's HIP stream; svdw_sync() waits for it.
 */
#ifndef SVDW_H
#define SVDW_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVDW_OK 0
#define SVDW_EINVAL -1   /* shape / argument mismatch (reference: assert! panic) */
#define SVDW_ERANGE -2   /* unsupported precision / lookup bits / bound */
#define SVDW_EDEVICE -3  /* HIP runtime error */
#define SVDW_ENOMEM -4

typedef struct svdw_ctx svdw_ctx;

typedef struct {
    int device;               /* HIP device ordinal (-1: host-only planning context) */
    uint32_t precision_bits;  /* FixedPointChip041 PRECISION_BITS, 1..63 */
    uint32_t lookup_bits;     /* RangeChip lookup_bits (LOOKUP_BITS env), 8..63 */
} svdw_params;

/* View of cells of one phase's advice stream:
 * cell(i, j) = stream[phase][off + i*rs + j*cs]. */
typedef struct {
    uint32_t phase;
    uint32_t rows, cols;
    uint64_t off;
    int64_t rs, cs;
} svdw_mat;

typedef struct {
    uint32_t phase;
    uint32_t len;
    uint64_t off;
    int64_t stride;
} svdw_vec;

/* check_svd_phase0's return tuple (src/svd/mod.rs:42-48,115). */
typedef struct {
    svdw_mat u_t, v_t, m_times_vt, u_times_ut, v_times_vt;
} svdw_svd_payload;

/* Constants of the example caller (examples/svd_example.rs:115-118,149,160). */
typedef struct {
    double max_norm;    /* MAX_NORM = 100.0 */
    double eps_svd;     /* EPS_SVD = 1e-10 */
    double eps_u;       /* EPS_U = 1e-10 */
    uint32_t max_bits_d;/* 30 */
} svdw_svd_config;

/* Cell totals of one SVD witness (phase 0 + phase 1). */
typedef struct {
    uint64_t advice0, advice1, lookup0, lookup1;
} svdw_counts;

/* ---------------------------------------------------------------- context */
int svdw_ctx_create(const svdw_params* params, svdw_ctx** out);
int svdw_ctx_destroy(svdw_ctx* ctx);
/* Drop all cells of both phases (allocations are kept). */
int svdw_ctx_reset(svdw_ctx* ctx);
/* Pre-size a phase's advice / lookup streams (cells). */
int svdw_reserve(svdw_ctx* ctx, uint32_t phase, uint64_t advice_cells, uint64_t lookup_cells);
int svdw_sync(svdw_ctx* ctx);
/* Stream ordering with the caller's own HIP stream (hipStream_t as void*; e.g.
 * torch.cuda.current_stream().cuda_stream). The context runs on streams of its
 * own and does NOT see work queued elsewhere: device memory an on_device call
 * reads (f64 inputs, device text) or writes (parse outputs) must be complete
 * / free when the call's work starts. Either synchronize the producing stream
 * first, or call svdw_stream_wait(ctx, producer) before the call: the
 * context's streams then wait (on the device, no host wait) for everything
 * queued on `stream` so far. svdw_stream_signal(ctx, consumer) after a call
 * makes `stream` wait for everything the context has queued (its outputs).
 * The Python layer (halo2_svd041_amd.zk) does both around every on-device call
 * with torch's current stream.
 *
 * Lifetime of device inputs. An on_device call returns before the device has
 * read its inputs: with "pipeline" (svd_witness) the call's stage kernels and
 * row scans read m, u, v, d straight from the f64 buffers after it returned,
 * and with "lanes" (verify_mul_witness) the call runs beside the next one. The
 * caller must keep every input buffer allocated and unmodified until the
 * call's work has completed: svdw_sync(), or svdw_query() returning 1, or any
 * stream ordered after svdw_stream_signal(ctx, stream) (a caching allocator
 * that frees on that stream). The Python layer holds a reference to every
 * device input tensor until a completion mark (svdw_mark, below) after its
 * call, or sync / reset / close, shows the work done. */
int svdw_stream_wait(svdw_ctx* ctx, void* stream);
/* 1 when everything queued on the context (both lanes) has completed, 0 while
 * some of it still runs (no host wait), < 0 on error. */
int svdw_query(svdw_ctx* ctx);
/* Completion marks: svdw_mark records how far the context's work is queued
 * (an event on each of its streams behind what is queued there; no stream
 * waits) and returns a ticket. svdw_mark_done(ticket) is 1 once everything
 * queued before the mark has completed, 0 while some of it runs (no host
 * wait), < 0 on error; svdw_mark_wait(ticket) waits for it on the host. The
 * last 16 marks are kept; an older ticket is answered by the mark that reused
 * its slot (done implies done; otherwise 0). (svdw_stream_signal onto a side
 * stream does the same job, but with 4 hardware queues per process that
 * stream may share a queue with one of the context's streams, whose later
 * work then waits behind the side stream's wait.) */
int svdw_mark(svdw_ctx* ctx, uint64_t* ticket);
int svdw_mark_done(svdw_ctx* ctx, uint64_t ticket);
int svdw_mark_wait(svdw_ctx* ctx, uint64_t ticket);
/* Debug: the CRT GEMM's block timeline into device buffer buf (3 u64 per block:
 * start and end on the 100 MHz wall clock, XCC id << 32 | HW_ID); null: off. */
int svdw_debug_trace(void* buf);
int svdw_stream_signal(svdw_ctx* ctx, void* stream);
const char* svdw_last_error(void);

/* ------------------------------------------------------ stream access */
uint64_t svdw_advice_len(const svdw_ctx* ctx, uint32_t phase);
uint64_t svdw_lookup_len(const svdw_ctx* ctx, uint32_t phase);
/* Device pointers to the canonical 32-byte cells (valid until the next append). */
const void* svdw_advice_device_ptr(const svdw_ctx* ctx, uint32_t phase);
const void* svdw_lookup_device_ptr(const svdw_ctx* ctx, uint32_t phase);
/* Copy cells [off, off+n) to host memory (4 x u64 little endian per cell); syncs. */
int svdw_copy_advice(svdw_ctx* ctx, uint32_t phase, uint64_t off, uint64_t n, uint64_t* out);
int svdw_copy_lookup(svdw_ctx* ctx, uint32_t phase, uint64_t off, uint64_t n, uint64_t* out);

/* ------------------------------------------- ZkMatrix / ZkVector (matrix/mod.rs) */
/* ZkMatrix::new (src/matrix/mod.rs:230-252): quantize + load_witness, row-major.
 * data: rows*cols f64 (host memory, or device memory if on_device). */
int svdw_zkmatrix_new(svdw_ctx* ctx, uint32_t phase, const double* data, uint32_t rows,
                      uint32_t cols, int on_device, svdw_mat* out);
/* ZkVector::new (src/matrix/mod.rs:29-40). */
int svdw_zkvector_new(svdw_ctx* ctx, uint32_t phase, const double* data, uint32_t len,
                      int on_device, svdw_vec* out);
/* ZkMatrix::transpose_matrix (src/matrix/mod.rs:408-419): no cells. */
int svdw_transpose_matrix(const svdw_mat* a, svdw_mat* out);
/* Context::load_witness / load_constant of one canonical value (halo2-base). */
int svdw_load_witness(svdw_ctx* ctx, uint32_t phase, const uint64_t value[4], svdw_vec* out);
int svdw_load_constant(svdw_ctx* ctx, uint32_t phase, const uint64_t value[4], svdw_vec* out);

/* ZkVector::entries_less_than (src/matrix/mod.rs:185-194). */
int svdw_entries_less_than(svdw_ctx* ctx, const svdw_vec* d, uint32_t max_bits);
/* ZkVector::entries_in_desc_order (src/matrix/mod.rs:199-215). */
int svdw_entries_in_desc_order(svdw_ctx* ctx, const svdw_vec* d, uint32_t max_bits);

/* check_mat_entries_bounded (src/matrix/mod.rs:490-501): |a_ij| < bnd.
 * bnd: unsigned 256-bit little endian (BigUint). */
int svdw_check_mat_entries_bounded(svdw_ctx* ctx, const svdw_mat* a, const uint64_t bnd[4]);
/* check_mat_diff (src/matrix/mod.rs:441-457): |a_ij - b_ij| < tol. */
int svdw_check_mat_diff(svdw_ctx* ctx, const svdw_mat* a, const svdw_mat* b,
                        const uint64_t tol[4]);
/* check_mat_id (src/matrix/mod.rs:461-483): |a_ij - scalar_id*I_ij| < tol. */
int svdw_check_mat_id(svdw_ctx* ctx, const svdw_mat* a, const svdw_vec* scalar_id,
                      const uint64_t tol[4]);
/* mat_times_diag_mat (src/matrix/mod.rs:610-627): a[i][j]*v[j], j < len(v). */
int svdw_mat_times_diag_mat(svdw_ctx* ctx, const svdw_mat* a, const svdw_vec* v, svdw_mat* out);
/* FixedPointChip041::signed_div_scale constants. The chip's source
 * (zk_fixed_point_chip, git HEAD) is not available offline, so its layout is
 * PARITY UNPINNED; the engine emits the parameterised construction
 *   add(x, 2^S) ; RangeChip::div_mod(t, 2^P, NB) ; sub(q, 2^(S-P))
 * (div_mod = [r, 2^P, q, t] + check_big_less_than_safe(q, 2^NB/2^P + 1)
 *  + check_big_less_than_safe(r, 2^P)), i.e. floor(x / 2^P) for |x| < 2^S.
 * Zero fields (or a null pointer) select S = 3P (the domain rescale_matrix's
 * doc states, src/matrix/mod.rs:350-353) and NB = max(4P + 1, S + 1) (NB = S + 1
 * is the tightest sound choice; a shift alone never makes the default NB
 * invalid). NB = 4P + 1 is the choice that reproduces the
 * reference's own cell counts: 90 cells per element at P = 32, LOOKUP_BITS = 12
 * ("#CONSTRAINTS = 90", src/matrix/mod.rs:102; "~94 (when lookup_bits = 12)",
 * :348) and 60-90 for P = 32 across LOOKUP_BITS 12-24, more for P > 32
 * (README.md:51: "60N^2 - 100N^2, depends on LB; higher for P>32"); NB = 3P + 1
 * gives 72 at P = 32, LB = 12. Both stay parity unpinned. */
typedef struct {
    uint32_t shift_bits;
    uint32_t num_bits;
} svdw_div_scale;
/* ZkMatrix::rescale_matrix (src/matrix/mod.rs:354-375): signed_div_scale of
 * every c_s entry, row-major, into c_s's phase; out = the quotient cells. */
int svdw_rescale_matrix(svdw_ctx* ctx, const svdw_mat* c_s, const svdw_div_scale* cfg,
                        svdw_mat* out);
/* ZkVector::inner_product (src/matrix/mod.rs:79-106): gate.inner_product(x, self)
 * then signed_div_scale; out = 1-element vector. */
int svdw_zkvector_inner_product(svdw_ctx* ctx, uint32_t phase, const svdw_vec* self,
                                const svdw_vec* x, const svdw_div_scale* cfg, svdw_vec* out);
/* ZkVector::_norm_square (src/matrix/mod.rs:112-119) = inner_product(self, self);
 * ZkVector::_dist_square (src/matrix/mod.rs:135-148): per-entry qsub (gate.sub)
 * then _norm_square of the differences. */
int svdw_zkvector_norm_square(svdw_ctx* ctx, uint32_t phase, const svdw_vec* self,
                              const svdw_div_scale* cfg, svdw_vec* out);
int svdw_zkvector_dist_square(svdw_ctx* ctx, uint32_t phase, const svdw_vec* self,
                              const svdw_vec* x, const svdw_div_scale* cfg, svdw_vec* out);
/* ZkVector::norm / dist (src/matrix/mod.rs:124-131, 156-164): _norm_square /
 * _dist_square then FixedPointChip041::qsqrt. The chip (zk_fixed_point_chip,
 * git HEAD) is not available, so qsqrt is a parameterised, constraint-checked
 * construction, PARITY UNPINNED: y = floor(sqrt(a 2^P)) for a in [0, 2^B)
 * (B = sqrt_bits, 0 -> 2P): load_witness(y), range_check(y, ny), t = mul(a, 2^P),
 * d = sub(t, mul(y, y)), range_check(d, ny + 1), f = sub(mul(y, 2), d),
 * range_check(f, ny + 1), ny = ceil((B + P) / 2) + 1; out = the y cell. */
int svdw_zkvector_norm(svdw_ctx* ctx, uint32_t phase, const svdw_vec* self, const svdw_div_scale* cfg,
                       uint32_t sqrt_bits, svdw_vec* out);
int svdw_zkvector_dist(svdw_ctx* ctx, uint32_t phase, const svdw_vec* self, const svdw_vec* x,
                       const svdw_div_scale* cfg, uint32_t sqrt_bits, svdw_vec* out);
/* ZkVector::mul (src/matrix/mod.rs:169-182): inner_product with every row of a. */
int svdw_zkvector_mul(svdw_ctx* ctx, uint32_t phase, const svdw_vec* self, const svdw_mat* a,
                      const svdw_div_scale* cfg, svdw_vec* out);
/* honest_prover_mat_mul (src/matrix/mod.rs:546-568): c_s = a*b over Fr, loaded row-major. */
int svdw_honest_prover_mat_mul(svdw_ctx* ctx, uint32_t phase, const svdw_mat* a,
                               const svdw_mat* b, svdw_mat* c_s);
/* field_mat_vec_mul (src/matrix/mod.rs:574-599): one inner_product per row of a;
 * out = the row results (last cell of each row block). */
int svdw_field_mat_vec_mul(svdw_ctx* ctx, uint32_t phase, const svdw_mat* a, const svdw_vec* v,
                           svdw_vec* out);
/* ZkMatrix::verify_mul (src/matrix/mod.rs:299-342), Freivalds with v = (1, g, g^2, ...);
 * gamma: canonical init_rand value (rlc.gamma_pow_cached()[0]). */
int svdw_verify_mul(svdw_ctx* ctx, uint32_t phase, const svdw_mat* a, const svdw_mat* b,
                    const svdw_mat* c_s, const uint64_t gamma[4]);

/* ------------------------------------------------------------ svd (svd/mod.rs) */
/* err_calc (src/svd/mod.rs:155-163). */
int svdw_err_calc(uint32_t p, uint64_t size, double max_norm, double eps_svd, double eps_u,
                  double* err_svd, double* err_u);
/* check_svd_phase0 (src/svd/mod.rs:32-116), appending to phase 0. */
int svdw_check_svd_phase0(svdw_ctx* ctx, const svdw_mat* m, const svdw_mat* u, const svdw_mat* v,
                          const svdw_vec* d, double err_svd, double err_u, uint32_t max_bits_d,
                          svdw_svd_payload* out);
/* check_svd_phase1 (src/svd/mod.rs:127-144), appending to phase 1. */
int svdw_check_svd_phase1(svdw_ctx* ctx, const svdw_mat* m, const svdw_mat* u, const svdw_mat* v,
                          const svdw_svd_payload* payload, const uint64_t gamma[4]);

/* Whole SVD-verify witness of examples/svd_example.rs:98-200 (intended
 * one-context semantics): reset, ZkMatrix::new(m,u,v), ZkVector::new(d),
 * err_calc(P, max(N,M), ...), check_svd_phase0 into phase 0, then
 * check_svd_phase1 into phase 1. m: N x M, u: N x N, v: M x M, d: min(N,M),
 * all row-major f64 (device memory if on_device). */
int svdw_svd_witness(svdw_ctx* ctx, const double* m, const double* u, const double* v,
                     const double* d, uint32_t N, uint32_t M, int on_device,
                     const svdw_svd_config* cfg, const uint64_t gamma[4], svdw_counts* counts);
/* The README.md:32-46 recipe as one call (BASELINE config 2): reset,
 * ZkMatrix::new(a) (N x K), ZkMatrix::new(b) (K x M), c_s =
 * honest_prover_mat_mul(a, b) into phase 0, ZkMatrix::verify_mul(a, b, c_s,
 * gamma) (src/matrix/mod.rs:299-342) into phase 1; the same cells as those four
 * modular calls, without host waits. a, b row-major f64 (device memory if
 * on_device). */
int svdw_verify_mul_witness(svdw_ctx* ctx, const double* a, const double* b, uint32_t N, uint32_t K,
                            uint32_t M, int on_device, const uint64_t gamma[4], svdw_counts* counts);
/* svdw_verify_mul_witness with device inputs, ordered after the work queued
 * so far on the caller's stream `stream` (svdw_stream_wait inside the call, on
 * the context state that runs it -- with "lanes" 2 the other one): one call
 * and one hand-off wait instead of two calls and a wait per state. */
int svdw_verify_mul_witness_on(svdw_ctx* ctx, void* stream, const double* a, const double* b, uint32_t N,
                               uint32_t K, uint32_t M, const uint64_t gamma[4], svdw_counts* counts);
/* Exact integer GEMM of honest_prover_mat_mul (the integer sum of quantized
 * products, reduced mod p once). Matrix-core paths (SVDW_GEMM_MFMA, default):
 *   - multi-modular / CRT (option "gemm_crt" 1, default): balanced residues
 *     modulo n pairwise coprime moduli <= 256 (n from the operand bit lengths:
 *     19 for m.v^T at P = 63), one int8 v_mfma_i32_16x16x64_i8 GEMM per
 *     modulus, CRT reconstruction; operands up to 2^128, K <= 8192;
 *   - balanced base-256 digit planes with i32 digit-pair diagonal sums
 *     ("gemm_crt" 0), operands up to ~2^71.
 * SVDW_GEMM_VALU: the digit planes on v_dot4c_i32_i8. All paths are
 * bit-identical; wider operands use a Montgomery GEMM. The environment
 * variable SVDW_GEMM=valu selects the VALU path at create. */
#define SVDW_GEMM_MFMA 0
#define SVDW_GEMM_VALU 1
int svdw_set_gemm_impl(svdw_ctx* ctx, int impl);
/* Options (svdw_set_option; 22 names; any other name is SVDW_EINVAL). Tuning
 * knobs, bit-identical results
 * for every value, defaults first:
 *   "gemm_impl" 0 | 1; "gemm_crt" 1 | 0 (CRT or digit-plane matrix-core GEMM);
 *   "overlap" 1 | 0 (the three check_svd_phase0 products run ahead on a second
 *   stream); "phase1_overlap" 1 | 2 | 0 (svd_witness: phase 1 runs on the
 *   second stream behind the products / on a third stream from quantization
 *   on, its c_s scans waiting for the products / after phase 0; 1 acts as 2 on
 *   a row-sharded context and when max(N, M) < 1024); "p1_at" -1 | 0 | 1 | 2 | 3
 *   (with phase 1 on the third stream: queued after the first 0 / 1 / 2
 *   phase-0 stages, 3 after all of phase 0; -1: 0 on a rank of a >= 4-way shard, 3 of a
 *   2-3-way shard, else 1);
 *   "stage_elems" 256 (elements per stage block, multiple of 16 in [16, 256]);
 *   "place_trials" 6 | 0..8 (a cell stream of >= 256 MiB allocated from now on
 *   is chosen among that many placements in HBM by timing the stage kernels'
 *   store pattern on each; 0 or 1: the first one);
 *   "stage_rot" 1 | 0 (a stage block writes its chunk of cells from a
 *   block-dependent 4 KiB window on, wrapping around, instead of from its
 *   start, so that blocks started together write different window offsets);
 *   "f64_views" 1 | 0 (svd_witness / verify_mul_witness with device inputs:
 *   stages and row scans read the loaded matrices from the f64 inputs,
 *   quantized in registers, instead of waiting for the quantized cells);
 *   "res_f64" 1 | 0 (svd_witness with inputs in HBM: the CRT residue planes of
 *   m, u, v built from the f64 inputs in one launch, or from the quantized cells);
 *   "stage_batch" 1 | 0 (independent stages share k_stage_multi launches: the
 *   u / v bounds and u.d, the d checks and constant cells, verify_mul's one cells
 *   and gamma powers, the is_equal rows; split automatically where a stage reads
 *   cells a pending one writes); "prod_cell" 1 | 0 | -1 (svd_witness with
 *   device inputs: the products on the cell stream and the u / v bounds and u.d
 *   beside them; -1 on row-sharded contexts only);
 *   "pipeline" 1 | 0 (svd_witness with device inputs on the f64 CRT product
 *   path with the products on the cell stream, when the second cell set is
 *   already allocated or its growth fits in the device's free memory with 10 %
 *   of the device to spare -- else the call runs unpipelined and the second set
 *   is released, as it is by "pipeline" 0: consecutive calls overlap -- a call returns with its
 *   u.d / bound / diff stages and its phase-1 row scans still running on the
 *   second and third streams, and the next call's gamma tables, quantization
 *   and products start on the cell stream beside them, into the other cell
 *   set and tables; any other call on the context, a copy and svdw_sync wait
 *   for that tail);
 *   "lanes" 2 | 1 (svdw_verify_mul_witness with device inputs: 2 alternates
 *   between two complete context states, exchanged behind the handle at each
 *   call, so consecutive calls run beside each other on separate streams; the
 *   handle always shows the latest call's cells; svdw_sync, stream_wait /
 *   _signal, graph_stats and destroy cover both states; a call stays on the
 *   current state when the other one would have to grow beyond the device's
 *   free memory less 10 % of the device);
 *   "graph" 1 | 0: svdw_verify_mul_witness with device inputs replays a HIP graph
 *   of its launch sequence. The second call of a key (N, K, M, the input
 *   pointers, no allocation or option change since) is captured, later calls
 *   of the key replay it with one hipGraphLaunch; k_gamma_prep (gamma's tables,
 *   and the one / gamma-power cells) is queued on the context stream ahead of
 *   the graph, so gamma is never part of it. Off while profiling or hold_us is
 *   set; "gamma_at" -1 | 0 | 1 and "dchk_at" 0 | 1 | 2 (pipelined svd_witness:
 *   k_gamma_prep at the head of the cell stream (0) or of the third stream (1;
 *   -1: the third on a row-sharded rank, else the cell stream); the d checks
 *   on the cell stream behind the products (0), on the second stream with the
 *   bounds and u.d (1) or on the third ahead of phase 1 (2)); "vm_linear" 1 | 0 (the captured sequence is queued on the context
 *   stream alone, a linear graph, instead of forking to the second stream);
 *   "gemm_kern" -1 | 0 | 1 | 2 (CRT GEMM: 0 one block per (128 x 128 tile,
 *   modulus) unit, 1 a persistent grid whose blocks' chunk pipelines run on
 *   across their units (jobs of one K >= 512), 2 256 x 128 tiles (non-symmetric
 *   products; others as 1); -1: for a product queued on its own
 *   (svdw_honest_prover_mat_mul) 2 from 64 tile pairs of 256 x 128 on, else 1,
 *   and 0 inside the witness calls);
 *   "res_wait" -1 | 0 | 1 (pipelined svd_witness reading its loads from the f64
 *   inputs: the second stream's stages wait for the residue planes (1) or not
 *   (0); -1: 1 on a row-sharded context, else 0).
 * Layout option (changes the phase-1 stream): "rlc_prefix" 0 | 1 (svd_witness:
 *   phase 1 starts with the two ctx_gate constant cells [1, 0] that
 *   examples/svd_example.rs:183's rlc.load_rlc_cache(.., 1) appends as recalled
 *   from axiom-eth's RlcChip, parity unpinned; init_rand is then RLC cell 2).
 * Test hook: "hold_us" 0 | us (svd_witness, verify_mul_witness: the step's
 *   streams wait behind a kernel spinning that long, so the GPU schedule is
 *   measured without host gaps and a missing cross-stream dependency shows).
 * Fixed since round 4 (measured, no longer options): products batched into one
 *   GEMM and one combine launch, residue planes before the stages beside them,
 *   the d checks and constant cells on the second stream, m, u, v, d quantized
 *   in one launch with the bit-length words folded inside it, b.g of a
 *   row-sharded rank from the f64 inputs, 4 KiB-aligned stage store windows,
 *   GEMM sizes decided on the device.
 * ABI version 2 removed the options ABI 1 had retired as no-ops ("bits_fold",
 *   "bounds_after", "colsum", "d_checks_aside", "dep_values", "fused_quantize",
 *   "gemm_batch", "gemm_priority", "gemm_rt", "prelaunch_at", "prod_blocks",
 *   "prod_first", "res_first", "stage_align", "stage_priority", "stage_probe",
 *   "stage_nt") and the persistent front streamer with its options
 *   ("stage_occ", "stage_front_all", and "stage_diag", a timing diagnostic
 *   whose cells were wrong): they are unknown names now (SVDW_EINVAL). */
int svdw_set_option(svdw_ctx* ctx, const char* name, int64_t value);
/* SVDW_ABI_VERSION of the library (callers compare it with the header's). */
#define SVDW_ABI_VERSION 2
int svdw_abi_version(void);
/* Captures and replays of the verify_mul_witness graph ("graph") so far. */
int svdw_graph_stats(svdw_ctx* ctx, uint64_t* captures, uint64_t* replays);

/* ----------------------------------------------------------- profiling */
/* Per-kernel statistics from HIP events recorded around every launch on the
 * context stream. bytes / ops: algorithmic HBM bytes / MACs of the launches
 * (cells x 32 B written + input cells read; GEMM MACs = N*M*K). */
typedef struct {
    char name[48];
    uint64_t launches;
    double total_ms, max_ms;
    double bytes, ops;
} svdw_kstat;
/* Enable (1) / disable (0) event recording; drops pending records. */
int svdw_profile_enable(svdw_ctx* ctx, int on);
/* Record only launches whose kernel name starts with `prefix` ("" / NULL = all):
 * each recorded launch adds two event packets to the stream. */
int svdw_profile_filter(svdw_ctx* ctx, const char* prefix);
/* Synchronize, aggregate pending records by kernel name (up to cap entries
 * written to out; *n = number of distinct names) and drop them. */
int svdw_profile_collect(svdw_ctx* ctx, svdw_kstat* out, uint32_t cap, uint32_t* n);

/* ---------------------------------------------- row-block sharding
 * One witness split over `world` contexts (one per GPU, no data exchange):
 * after svdw_set_shard(ctx, rank, world), svdw_svd_witness / check_svd_phase0/1
 * compute on this context only the rows [R*rank/world, R*(rank+1)/world) of
 * every row-parallel stage (R = the stage's row count: N or M), writing them
 * at their global offsets of full-size streams; the shared operands (quantized
 * m, u, v, d, single constants, the Freivalds b.g vector values) are computed
 * by every rank. svdw_shard_segments lists the cell ranges this rank is the
 * source of; over all ranks they tile every stream exactly once, so the global
 * witness is the union (a gather to one device, or kept sharded-resident).
 * Works on planning contexts too (segments without cells). world = 1: off. */
typedef struct {
    uint32_t phase;     /* 0 / 1 */
    uint32_t lookup;    /* 0: advice stream, 1: lookup stream */
    uint64_t off, n;    /* cells [off, off + n) */
} svdw_segment;
int svdw_set_shard(svdw_ctx* ctx, uint32_t rank, uint32_t world);
/* Virtual layout of the last witness: every cell region in append order (the
 * order halo2-base's Context receives them), tagged with the gadget / function
 * that appended it. rows > 1: the region is `rows` equal runs of cells, one per
 * row of a row-parallel stage (the unit of svdw_set_shard). Works on planning
 * contexts. Up to cap regions into out; *n = total count. */
typedef struct {
    uint32_t phase;
    uint32_t _pad;
    uint64_t off, n;      /* advice cells [off, off + n) */
    uint64_t loff, nl;    /* lookup cells [loff, loff + nl) */
    uint64_t rows;
    char tag[40];
} svdw_region;
int svdw_layout(const svdw_ctx* ctx, svdw_region* out, uint64_t cap, uint64_t* n);
/* ctx_rlc of the last svd_witness run with "rlc_prefix" 1: the RLC context of
 * examples/svd_example.rs:181-184 (rlc.load_rlc_cache((ctx_gate, ctx_rlc),
 * gate, 1); gamma_pow_cached()[0]), as recalled from axiom-eth's RlcChip
 * (un-vendored: PARITY UNPINNED). An empty cache loads gamma as
 * compute_rlc_fixed_len(ctx_rlc, [one, zero]): ctx_rlc holds
 * [E(one), E(zero), W(gamma)], whose cell 2 is the init_rand every phase-1
 * gamma cell copies. cells: 3 x 4 u64 (canonical LE); copies[k]: the source of
 * ctx_rlc cell k < 2 (phase << 62 | offset in that phase's advice stream, the
 * two ctx_gate constants at the head of phase 1). *n = 3, or 0 when the last
 * witness had no RLC prefix (cells / copies untouched). Host memory, no GPU. */
int svdw_rlc_trace(const svdw_ctx* ctx, uint64_t* cells, uint64_t* copies, uint32_t* n);

/* Constraint check of the last witness on the device, the MockProver-style
 * verification of an (unsharded) context: every halo2-base basic gate
 * a + b*c = d at the offsets the reference's gadgets enable (assign_region's
 * gate offsets; the row-scan inner products), every lookup cell against the
 * [0, 2^lookup_bits) table, and the copy constraints of the gadget blocks: a
 * value's repeated cells, a loaded operand against its source cell, and
 * range_check's last running sum against the checked value. Not checked: the
 * copies of the row scans' operands and of constant cells. An honest witness
 * has no failures; an SVD that violates a bound fails range-check copies
 * (README.md:93 "matrix-wrong", from P = 42 on). A row-sharded context
 * (svdw_set_shard) checks the cells it owns (svdw_shard_segments): summed over
 * the ranks, the counts equal those of the unsharded witness. */
typedef struct {
    uint64_t gates_checked, gate_failures;
    uint64_t lookups_checked, lookup_failures;
    uint64_t copies_checked, copy_failures;
} svdw_check_result;
int svdw_check_gates(svdw_ctx* ctx, svdw_check_result* out);

/* Virtual -> physical layout of the last witness (the
 * halo2-base 0.4.1 keygen assignment, restated from memory -- parity unpinned,
 * see DESIGN.md): basic-gate advice columns of max_rows = 2^k - minimum_rows
 * usable rows (BaseCircuitBuilder::calculate_params, src/scaffold/mod.rs:245-247
 * MINIMUM_ROWS default 20). A column breaks at the cell whose gate would cross
 * max_rows, or at row max_rows - 1; the break cell is repeated at row 0 of the
 * next column and its selector enabled there only. Lookup cells fill lookup
 * advice columns max_rows at a time. num_advice is calculate_params' estimate
 * ceil(cells / max_rows); columns_used is what the assignment needs (more than
 * num_advice: the reference's keygen panics "NOT ENOUGH ADVICE COLUMNS"). */
typedef struct {
    uint32_t k, minimum_rows;
    uint64_t max_rows;
    uint32_t num_advice[2], columns_used[2], num_lookup_advice[2];
    uint32_t num_fixed;
    uint64_t constants;    /* distinct constant cell values (fixed column cells) */
} svdw_physical_params;
int svdw_physical_layout(svdw_ctx* ctx, uint32_t k, uint32_t minimum_rows, svdw_physical_params* out);
/* each column but the last: the row of its break cell (halo2-base break_points) */
int svdw_break_points(const svdw_ctx* ctx, uint32_t phase, uint64_t* out, uint64_t cap, uint64_t* n);
/* Materialise phase `phase` on the device, column-major, 2^k rows per column
 * (rows past the used ones zero): advice = columns_used x 2^k cells, selectors
 * = columns_used x 2^k q_enable bytes, lookup = num_lookup_advice x 2^k cells;
 * any may be NULL. Fails with SVDW_ERANGE when columns_used > num_advice. */
int svdw_assign_columns(svdw_ctx* ctx, uint32_t phase, void* advice, uint8_t* selectors, void* lookup);
/* The basic gate at every enabled (column, row) of assigned columns, and each
 * break cell against row 0 of the next column (copies_*). */
int svdw_check_physical(svdw_ctx* ctx, uint32_t phase, const void* advice, const uint8_t* selectors,
                        uint32_t ncols, svdw_check_result* out);
/* Copy-constraint (equality) lists of phase `phase` of the last witness: the
 * records halo2-base 0.4.1's copy manager holds after the same calls, in assign
 * order -- every QuantumCell::Existing cell against its source cell, every
 * Constant cell (and assert_is_const) against its value, range_check's
 * constrain_equal(a, last running sum) -- so keygen / MockProver can run on
 * the engine's columns. Replaces Context's copy manager (advice_equalities,
 * constant_equalities) consumed by raw_synthesize_phase0/1
 * (src/utils/executor.rs:100-102,116-118; src/scaffold/mod.rs:93-106).
 * copies: 2 words per record, (source cell | source phase << 62, destination
 * cell of `phase`); source phase 2 = the external init_rand cell of verify_mul
 * (RLC context). consts: 5 words per record, (cell, 4 canonical LE words).
 * Works on dry (planner) contexts. Null buffers: counts only. */
int svdw_equalities(const svdw_ctx* ctx, uint32_t phase, uint64_t* copies, uint64_t copies_cap,
                    uint64_t* n_copies, uint64_t* consts, uint64_t consts_cap, uint64_t* n_consts);
typedef struct {
    uint64_t copies_checked, copy_failures;
    uint64_t consts_checked, const_failures;
} svdw_eq_check;
/* Check every equality record of `phase` on the device: on the virtual cell
 * streams (columns0 = columns1 = NULL), or on assigned physical columns
 * (svdw_assign_columns output of phase 0, and of phase 1 for phase 1), each
 * cell at its first placement. External sources compare with the last init_rand. */
int svdw_check_equalities(svdw_ctx* ctx, uint32_t phase, const void* columns0, const void* columns1,
                          svdw_eq_check* out);
/* Up to cap segments of the last witness into out; *n = total count. */
int svdw_shard_segments(const svdw_ctx* ctx, svdw_segment* out, uint64_t cap, uint64_t* n);

/* ------------------------------------------------------------ input ingest
 * Parse the example's input file (data/matrix.in of input-creator.py:23-44;
 * read by examples/svd_example.rs:326-330 with serde_json::from_str) into
 * row-major f64 arrays. mode SVDW_PARSE_SERDE reproduces serde_json's default
 * float parse (u64 significand x / / 10^|e| in f64; 1 ulp off correct rounding
 * on ~10 % of the values, which changes quantized cells), SVDW_PARSE_CORRECT
 * rounds correctly. Call with null arrays to get the shapes, then again with
 * arrays of those sizes. */
#define SVDW_PARSE_SERDE 0
#define SVDW_PARSE_CORRECT 1
typedef struct {
    uint32_t m_rows, m_cols, u_rows, u_cols, v_rows, v_cols, d_len;
} svdw_input_dims;
int svdw_parse_svd_input(const char* text, uint64_t len, int mode, svdw_input_dims* dims,
                         double* m, double* u, double* d, double* v);
/* The same parse of text already in device memory, on the context's device
 * (serde mode only): m, u, d, v are DEVICE pointers (null: dims only), ready for
 * svdw_svd_witness(on_device = 1). Replaces examples/svd_example.rs:326-330
 * (read_to_string + serde_json::from_str) for a file staged to HBM; the values
 * are identical to svdw_parse_svd_input's (SVDW_PARSE_SERDE) on every input, and
 * malformed text is rejected (SVDW_EINVAL). Synchronous. */
int svdw_parse_svd_input_device(svdw_ctx* ctx, const void* text, uint64_t len, int mode,
                                svdw_input_dims* dims, double* m, double* u, double* d, double* v);

/* Closed-form cell counts of svdw_svd_witness without touching a device. */
int svdw_plan_svd(uint32_t N, uint32_t M, uint32_t precision_bits, uint32_t lookup_bits,
                  const svdw_svd_config* cfg, svdw_counts* counts);

#ifdef __cplusplus
}
#endif
#endif /* SVDW_H */
