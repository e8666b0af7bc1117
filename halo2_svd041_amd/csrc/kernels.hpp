// Host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fr.hpp"
#include "prog.hpp"

namespace svdw {

// Row-scan operand width decided on the device: a job's matrix has |signed
// entries| < 2^bits with bits = W[wa] (ZkMatrix::new cells whose bit-length
// maximum is device word W[wa]) or W[wa] + W[wb] + lk (a product c_s = a * b
// with K <= 2^lk, like bits_of on the host); wa < 0: unknown (na = 8).
struct NaSpec {
    int16_t wa, wb;
    uint16_t lk, _r;
};
// Scaled-vector table of a length-L vector w: kTabSlots slots of 2L cells.
// Slot s < 6 (na = s + 1): w * 2^(32 na) mod p at [2sL, 2sL + L) and its
// negation at [2sL + L, 2sL + 2L); slot 6: w in Montgomery form at [12L, 13L).
static constexpr int kTabSlots = 7;
constexpr uint64_t tab_len(uint64_t L) { return 2ull * kTabSlots * L; }
// factors per slot: mont_mul(w, f[s]) is slot s's entry for a canonical w
struct ScaleTab {
    Fr f[kTabSlots];
};
// One row scan of a batched launch: rows [r_begin, r_begin + rows) of A (L
// columns) against w (canonical wc, scaled table tab), row i's 3L+1 cells at
// out + i*(3L+1). blk0 is set by launch_scan_batch.
// Row-end epilogues (zero fields: none):
//  pc / ptab: the row totals t_r (= A.w, every row of A scanned) as a vector of
//    length plen -- canonical copy pc[r] and scaled table ptab (k_vec_prep's), so
//    the next scan multiplies by it without a k_vec_prep launch;
//  eq_out: verify_mul's is_equal(t_r, y_r) row (12 cells, PB::g_is_equal's
//    [d, y, 1, x, z, d, inv, 1, 0, d, z, 0]) at eq_out + 12 r, y_r = eq_y[r eq_ys].
struct ScanJob {
    DView A;
    const Fr* wc;
    const Fr* tab;
    uint32_t tl;     // the table's length (slot stride, >= L: gamma tables serve shorter scans)
    Fr* out;
    uint32_t L, rows, blk0, r_begin;
    NaSpec spec;
    Fr* pc;
    Fr* ptab;
    uint32_t plen;
    uint32_t eq_ys;
    Fr* eq_out;
    const Fr* eq_y;
};
static constexpr int kMaxScanJobs = 8;
static constexpr int kMaxVerifyBatch = 4;   // verify_mul calls per batch (b and a scans share a launch)
struct ScanBatch {
    ScanJob job[kMaxScanJobs];
    uint32_t njobs;
    const unsigned* bitw;     // device bit-length words of the NaSpecs (na = 0 launches)
    ScaleTab f;               // slot factors for the pc / ptab epilogue
};
// gamma powers from host-side Montgomery tables: g^j = t[j & 15] t[16 + (j >> 4 & 15)]
// t[32 + (j >> 8)] (j < 256 * nhi)
static constexpr int kGammaTab = 96;
struct GammaTab {
    Fr t[kGammaTab];
    uint32_t nhi;
};

// Elements per block of the generic stage kernel (= block size; LDS: E * (nv * 32 + 16) B).
static constexpr int kStageElems = 256;

// ZkMatrix::new / ZkVector::new quantization (f64 -> Fr) of n contiguous values.
// blockmax (nullable, ceil(n / kQuantPerBlock) words): per-block max of bit-length(|x_q|).
hipError_t launch_quantize(const double* in, uint64_t n, Fr* out, int precision_bits,
                           unsigned* blockmax, hipStream_t st);
// Fold per-block maxima: out[s] = max(blockmax[begin[s] .. begin[s + 1])), s < nseg.
// One launch quantizing up to 4 matrices (m, u, v, d of the SVD witness):
// segment s covers blocks [blk0[s], blk0[s+1]) of kQuantPerBlock values.
// Segment k may store only part of its cells (keep[k].cols != 0: value i is
// element (i / cols, i % cols) and is stored when its row is in [rlo, rhi) or
// its column in [clo, chi)); its bit-length maxima still cover every value.
static constexpr int kMaxQuantSegs = 4;
struct QuantKeep {
    uint32_t cols, rlo, rhi, clo, chi;
};
// In-launch fold of the per-block bit-length maxima (what k_bits_reduce does in
// a launch of its own): blocks [0, nblk) publish bm[block] and arrive on the
// counters cnt[1 + (block & 7)], the last of each group on cnt[0] (all zero
// between launches, each reset by its last arrival); the last block folds
// segment s = blocks [b[s], b[s + 1]) into wout[s].
struct BitFold {
    unsigned* bm;
    unsigned* cnt;
    unsigned* wout;
    uint32_t nblk;
    uint32_t nred;                       // segments folded (<= 3)
    uint32_t b[4];
};
// Values per quantize block (16 per thread): few enough blocks for one wave of
// them at 1024^2, so the fold's arrival costs each block once. Launches of
// fewer than 2^21 values use 1024 per block (4 per thread): 256^2 x 2 is
// otherwise 32 blocks on 256 CUs.
static constexpr uint32_t kQuantPerBlock = 4096;
static constexpr uint32_t kQuantPerBlockSmall = 1024;
static inline uint32_t quant_per_block(uint64_t total_values) {
    return total_values < (1ull << 21) ? kQuantPerBlockSmall : kQuantPerBlock;
}
struct QuantSegs {
    const double* in[kMaxQuantSegs];
    Fr* out[kMaxQuantSegs];
    unsigned* blockmax[kMaxQuantSegs];
    uint64_t n[kMaxQuantSegs];
    QuantKeep keep[kMaxQuantSegs];
    uint32_t blk0[kMaxQuantSegs + 1];
    uint32_t nseg;
    uint32_t per_block;                  // values per block: kQuantPerBlock(Small); 0 = kQuantPerBlock
    BitFold fold;                        // fold.wout null: no in-launch fold
};
hipError_t launch_quantize_multi(const QuantSegs& q, int precision_bits, hipStream_t st);
// Witness checker (svdw_check_gates). A region is `nunits` repetitions of a
// `unit`-cell block (element u = row u / cols, column u % cols); check words:
//   CHK_GATE g      a + b*c = d on cells g..g+3
//   CHK_COPY i, j   cell i == cell j
//   CHK_VIEW k, j   view k's cell of the element == cell j (not counted outside the view)
// cnt[0..1] += gates checked / failed, cnt[4..5] += copies checked / failed;
// lookups: every cell < 2^lb -> cnt[0] += n, cnt[1] += failed.
enum : uint32_t { CHK_GATE = 0, CHK_COPY = 1, CHK_VIEW = 2 };
constexpr uint32_t chk_gate(uint32_t g) { return g; }
constexpr uint32_t chk_copy(uint32_t i, uint32_t j) { return (CHK_COPY << 30) | (i << 15) | j; }
constexpr uint32_t chk_view(uint32_t k, uint32_t j) { return (CHK_VIEW << 30) | (k << 15) | j; }
constexpr uint32_t chk_kind(uint32_t w) { return w >> 30; }
constexpr uint32_t chk_a(uint32_t w) { return (w >> 15) & 0x7fff; }
constexpr uint32_t chk_b(uint32_t w) { return w & 0x7fff; }
struct ChkView {
    const Fr* ptr;   // null: no view
    int64_t rs, cs;
    uint32_t rows, cols;
};
// the checks of one layout region (engine side)
struct RegionChecks {
    struct Src {
        int phase;     // -1: none
        uint64_t off;
        int64_t rs, cs;
        uint32_t rows, cols;
    };
    std::vector<uint32_t> words;
    uint32_t unit = 0, cols = 1;
    Src src[kMaxViews] = {{-1, 0, 0, 0, 0, 0}, {-1, 0, 0, 0, 0, 0}};
    // ---- equality lists (svdw_equalities): halo2-base's copy / constant
    // equalities of the region, per element in assign order (eq words, below),
    // with the source cells of the element's loaded values per view (esrc)
    std::vector<uint32_t> eq;
    struct EqSrc {
        int kind = 0;                 // EQS_NONE / EQS_MAT / EQS_CHAIN
        uint32_t phase = 0;           // EQS_MAT: cell (i, j) = off + i rs + j cs inside rows x cols,
        uint64_t off = 0;             //   else `pad`; diag >= 0 phase: (i == i) -> diag, else pad
        int64_t rs = 0, cs = 0;
        uint32_t rows = 0, cols = 0;
        int pad_phase = -1, diag_phase = -1;
        uint64_t pad_off = 0, diag_off = 0;
        // EQS_CHAIN (vector, index t = the element's row i, or the scan term j):
        // t == 0 -> (first_phase, first), else (phase, off + (t - 1) * rs)
        uint32_t first_phase = 0;
        uint64_t first = 0;
    } esrc[kMaxViews];
    std::vector<Fr> eqk;              // the program's constants (EQ_CONST values)
    bool scan = false;                // inner_product rows: [C(0), E(a_j), E(v_j), W(s_j), ...],
                                      // a = esrc[0] (row i, term j), v = esrc[1] (term j)
};
// equality words of an element program: kind << 24 | a << 12 | slot
enum : uint32_t { EQ_CONST = 0, EQ_LOCAL = 1, EQ_VIEW = 2, EQ_EXT = 3 };
enum : int { EQS_NONE = 0, EQS_MAT = 1, EQS_CHAIN = 2 };
constexpr uint32_t eq_word(uint32_t kind, uint32_t a, uint32_t slot) { return kind << 24 | a << 12 | slot; }
constexpr uint32_t eq_kind(uint32_t w) { return w >> 24; }
constexpr uint32_t eq_a(uint32_t w) { return (w >> 12) & 0xfff; }
constexpr uint32_t eq_slot(uint32_t w) { return w & 0xfff; }
// (u0: index in the region of the first unit at adv, for the view rows / columns)
hipError_t launch_check_cells(const Fr* adv, uint64_t u0, uint64_t nunits, uint32_t unit, uint32_t cols,
                              const uint32_t* words, uint32_t nw, ChkView v0, ChkView v1,
                              unsigned long long* cnt, hipStream_t st);
// Physical layout (svdw_assign_columns): qb |= the gate-start bits of a region
// (`unit`-periodic pattern ubits[unit]); a column's selector bytes from the bits
// (the last row of a full column cleared); the basic gate at every enabled
// (column, row), and each break cell against row 0 of the next column
// (cnt[0..1] gates, cnt[4..5] copies).
hipError_t launch_gate_bits(uint32_t* qb, uint64_t off, uint64_t n, uint64_t unit, const uint8_t* ubits,
                            hipStream_t st);
hipError_t launch_selectors(uint8_t* q, const uint32_t* qb, uint64_t start, uint64_t len, uint64_t rows,
                            bool clear_last, hipStream_t st);
hipError_t launch_check_physical(const Fr* cols, const uint8_t* q, uint64_t rows, uint32_t ncols,
                                 unsigned long long* cnt, hipStream_t st);
hipError_t launch_check_breaks(const Fr* cols, uint64_t rows, const uint64_t* bp, uint32_t nb,
                               unsigned long long* cnt, hipStream_t st);
// Equality lists: cnt[0..1] += pairs checked / failing (source store from the
// top two bits: s0, s1, or 2 = ext), constants checked / failing.
hipError_t launch_check_copies(const Fr* s0, const Fr* s1, const Fr* dst, const uint64_t* pairs,
                               uint64_t n, const Fr& ext, unsigned long long* cnt, hipStream_t st);
hipError_t launch_check_consts(const Fr* dst, const uint64_t* recs, uint64_t n,
                               unsigned long long* cnt, hipStream_t st);
hipError_t launch_check_lookups(const Fr* lk, uint64_t n, uint32_t lb, unsigned long long* cnt,
                                hipStream_t st);
// Equality records on the device (svdw_equalities / svdw_check_equalities): one
// work item per element of a program region (its eq words in order) or per
// (row, term) of an inner-product scan region; records land at closed-form
// offsets, so the lists come out in the host's assign order.
struct EqSrcDev {
    int32_t kind, phase, pad_phase, diag_phase, first_phase, _r;
    uint64_t off, pad_off, diag_off, first;
    int64_t rs, cs;
    uint32_t rows, cols;
};
struct EqRegionDev {
    uint64_t off, nitems, item0, copy0, const0;
    uint32_t scan, unit, cols, L;
    uint32_t w0, nw, ncw, nkw, k0, _r;
    EqSrcDev src[2];
};
// copies: (source | store << 62, destination) pairs; consts: (cell, 4 words);
// err: set to 1 when a copy source lies outside the cell streams.
hipError_t launch_eq_records(const EqRegionDev* regions, uint32_t nreg, uint64_t nitems,
                             const uint32_t* words, const Fr* konst, uint32_t phase, uint64_t ext_off,
                             uint64_t* copies, uint64_t* consts, unsigned* err, hipStream_t st);
// virtual cell -> column-major physical index, in place over the records
// (svdw_assign_columns' layout: start[phase][col] = the column's first cell)
hipError_t launch_eq_phys(uint64_t* copies, uint64_t nc, uint64_t* consts, uint64_t nk,
                          const uint64_t* start0, uint32_t ncol0, const uint64_t* start1, uint32_t ncol1,
                          uint32_t phase, uint32_t k, hipStream_t st);
static constexpr int kMaxBitSegs = 8;
struct BitSegs {
    uint32_t begin[kMaxBitSegs];
};
// Timing aid: a one-wave kernel spinning `us` microseconds on the device clock.
hipError_t launch_hold(uint32_t us, hipStream_t st);
hipError_t launch_bits_reduce(const unsigned* blockmax, const BitSegs& seg, uint32_t nseg,
                              unsigned* out, hipStream_t st);
// k_maxbits grid bound (= words written to `out`).
static constexpr uint32_t kMaxBitBlocks = 2048;
// Generic cell-program stage over elements [a.e_begin, a.e_end).
hipError_t launch_stage(const StageArgs& a, hipStream_t st);
// Independent stages (no stage reads another's cells) in as few k_stage_multi
// launches as their records fit (stage_record_bytes, kMultiBytes); n >= 1.
hipError_t launch_stage_multi(const StageArgs* const* progs, int n, hipStream_t st);
// The next stage launches of this thread (launch_stage*, until
// launch_events_used) record e0 at the first one's start and e1 at each one's
// end through their dispatch; launch_events_used says whether any launched.
void set_launch_events(hipEvent_t e0, hipEvent_t e1);
bool launch_events_used();
// does the record of `a` fit one k_stage_multi launch?
bool stage_multi_fits(const StageArgs& a);
// max over the view of bit-length(|signed(x)|): out[b] = max of block b
// (min(ceil(rows * cols / 256), kMaxBitBlocks) blocks).
hipError_t launch_maxbits(const DView& v, uint32_t rows, uint32_t cols, unsigned* out,
                          hipStream_t st);
// Balanced base-256 digit planes of X (rows x kdim): out[row][kg][D] int32 words,
// each packing the digit of 4 consecutive k. rows_pad/kg_pad are zero-filled.
hipError_t launch_to_digits(const DView& x, uint32_t rows, uint32_t kdim, int D,
                            uint32_t rows_pad, uint32_t kg_pad, uint32_t* out, hipStream_t st);
// c_s[i][j] = sum_k A[i][k] * Bt[j][k] exactly, written as canonical Fr to
// out[i*ors + j*ocs]. sym: A == Bt (upper tiles + mirror).
hipError_t launch_gemm_digits(int DA, int DB, bool sym, const uint32_t* Ad, const uint32_t* Bd,
                              uint32_t N, uint32_t M, uint32_t kg_pad, Fr* out, int64_t ors,
                              int64_t ocs, hipStream_t st);
bool gemm_digits_supported(int DA, int DB);
// Matrix-core variant: digit planes laid out [row][kc][D][64 B] (kc = 64-k chunks).
// dbits (nullable, one word): take D from this device-side bit-length maximum
// instead (5 / 8 / 9 planes; nothing written when wider than 9 digits).
hipError_t launch_to_digits_mf(const DView& x, uint32_t rows, uint32_t kdim, int D, uint32_t rows_pad,
                               uint32_t kcn, uint32_t* out, hipStream_t st,
                               const unsigned* dbits = nullptr);
hipError_t launch_gemm_mfma(int DA, int DB, bool sym, const uint8_t* Ad, const uint8_t* Bd,
                            uint32_t N, uint32_t M, uint32_t kcn, Fr* out, int64_t ors,
                            int64_t ocs, hipStream_t st);
// Same product with DA / DB decided on the device from bit-length words (planes
// laid out for those counts by launch_to_digits_mf with the same words); a
// no-op when either operand is wider than 9 digits.
hipError_t launch_gemm_mfma_rt(bool sym, const uint8_t* Ad, const uint8_t* Bd, uint32_t N,
                               uint32_t M, uint32_t kcn, Fr* out, int64_t ors, int64_t ocs,
                               const unsigned* bits_a, const unsigned* bits_b, hipStream_t st);
// Generic Montgomery GEMM (any field elements): out = A(NxK) * B(KxM). With
// bit-length words, a no-op unless an operand is too wide for the digit GEMM.
// crt_lk >= 0: the skip test is the CRT GEMM's (ceil(log2 K) = crt_lk).
hipError_t launch_gemm_mont(const DView& A, const DView& B, uint32_t N, uint32_t K, uint32_t M,
                            Fr* out, int64_t ors, int64_t ocs, hipStream_t st,
                            const unsigned* bits_a = nullptr, const unsigned* bits_b = nullptr,
                            int crt_lk = -1);
// Multi-modular exact GEMM (device-decided modulus count from bits_a / bits_b,
// no-op when an operand exceeds 128 bits). Residue planes of X: out =
// [kCrtMaxResidues][rows_pad][kpad] int8 (rows_pad % 128 == 0, kpad % 64 == 0).
// bits_c (nullable): also cover the product (c, c), so the planes can be reused.
hipError_t launch_to_residues(const DView& x, uint32_t rows, uint32_t kdim, uint32_t rows_pad,
                              uint32_t kpad, uint32_t* out, const unsigned* bits_a,
                              const unsigned* bits_b, uint32_t lk, hipStream_t st,
                              const unsigned* bits_c = nullptr);
// Residue planes of up to kMaxResSegs f64 matrices (row-major, row pitch ld),
// each as k_to_residues would build them from its quantized cells: planes
// [n][rows_pad][kw] u32 words (4 x int8 per word, kw * 4 >= cols), rows >= rows
// and k >= cols zero; n = max over the segment's pairs p (wa[p] >= 0) of the CRT
// modulus count of a product with operand bits W[wa[p]], W[wb[p]] and K <= 2^lk[p].
static constexpr int kMaxResSegs = 4;
// tr: element (row, k) is in[k * ld + row] (the planes of a transposed operand:
// b^T of verify_mul_witness's b), threads laid along rows so the reads coalesce.
struct ResSeg {
    const double* in;
    uint32_t* out;
    uint32_t rows, cols, ld, rows_pad, kw;
    int16_t wa[2], wb[2];
    uint32_t lk[2];
    uint32_t tr;
};
struct ResSegs {
    ResSeg seg[kMaxResSegs];
    uint32_t blk0[kMaxResSegs + 1];   // set by the launcher
    uint32_t nseg;
};
hipError_t launch_residues_f64(const ResSegs& q, const unsigned* W, int precision_bits,
                               hipStream_t st);
// c_s = A * Bt from residue planes Ar (plane stride astride rows, from the A rows'
// first row) and Br (bstride): N x M; R is the residue scratch
// (crt_scratch_bytes(N, M) bytes).
hipError_t launch_gemm_crt(bool sym, const uint8_t* Ar, const uint8_t* Br, uint32_t N, uint32_t M,
                           uint32_t astride, uint32_t bstride, uint32_t kpad, uint8_t* R, Fr* out,
                           int64_t ors, int64_t ocs, const unsigned* bits_a,
                           const unsigned* bits_b, uint32_t lk, hipStream_t st, uint32_t kern = 0);
// Debug: record the CRT GEMM's block timeline into buf (3 u64 per block; null: off).
hipError_t set_debug_trace(void* buf);
static constexpr int kCrtMaxResidues = 40;   // = kCrtMaxMod (crt_tables.hpp)
// Several CRT products in one GEMM launch and one combine launch (the three
// products of check_svd_phase0; launch_gemm_crt is the one-job case). The GEMM's
// (job, modulus, tile) units are placed modulus-major per XCD. Per job the caller sets Ar, Br,
// astride, bstride, kpad, R (its own residue scratch), out, ors, ocs, N, M,
// bits_a, bits_b, lk and sym (A == B: upper tiles + mirror); the launcher
// fills the tile and block fields.
static constexpr int kMaxCrtJobs = 3;
static constexpr uint32_t CT_TILE = 128;   // CRT GEMM output tile edge (kernels.hip CT)
struct CrtJob {
    const uint8_t* Ar;
    const uint8_t* Br;
    uint8_t* R;
    Fr* out;
    const unsigned* bits_a;
    const unsigned* bits_b;
    int64_t ors, ocs;
    uint32_t astride, bstride, kpad, N, M, lk, sym;
    uint32_t tiles_a, tiles_m, nblk, cblk0;
    // tiles [tile0, tile0 + tcount) of the job's tile sequence only (tcount 0:
    // all): a row block of a product (SYM: the upper tiles of rows of tiles
    // [b0, b1), whose mirrors land in later rows)
    uint32_t tile0, tcount;
};
struct CrtBatch {
    CrtJob job[kMaxCrtJobs];
    uint32_t njobs;
    // GEMM kernel (bit-identical): 0 one block per (tile, modulus) unit
    // (k_gemm_crt_multi), 1 a persistent grid whose blocks' chunk pipelines
    // run across their units (k_gemm_crt_pers; jobs of one kpad >= 512), 2
    // 256 x 128 tiles (k_gemm_crt_wide; non-symmetric whole jobs), 3 wide
    // from 64 tile pairs on, else persistent (products queued on their own)
    uint32_t kern;
};
// R sized crt_scratch_bytes per job
hipError_t launch_gemm_crt_multi(const CrtBatch& b, hipStream_t st);
// residue scratch R one CRT product of N x M needs
size_t crt_scratch_bytes(uint32_t N, uint32_t M);
// w (len L) from a view (row 0 / col j of a 1 x L view) -> canonical copy
// (w_canon nullable) and its scaled table (ScaleTab f: see kTabSlots).
hipError_t launch_vec_prep(const DView& w, uint32_t L, Fr* w_canon, Fr* tab, const ScaleTab& f,
                           hipStream_t st);
// w_j = gamma^j, j < L (L <= 256 * (kGammaTab - 32)): canonical copy and scaled table.
// verify_mul's `one` cell and gamma-power cells [0, v_(i-1), gamma, v_i],
// i = 1 .. d - 1, written by k_gamma_prep beside the table (one null: none).
struct PowCells {
    Fr* one;
    Fr* pows;
    uint32_t d;
    Fr gamma;     // canonical
};
hipError_t launch_gamma_prep(const GammaTab& g, uint32_t L, Fr* w_canon, Fr* tab, const ScaleTab& f,
                             hipStream_t st, const PowCells* pc = nullptr);
// Freivalds inner-product rows (GateChip::inner_product, 1+3L cells per row) for
// rows [r_begin, r_end) of A (R x L); row r's cells at out + (r - r_begin)*(3L+1):
// one block per row, two terms per thread, DPP wave scan, small-operand products
// when na < 8 (|signed A| < 2^(32 na), the table's slot na - 1), the table's
// Montgomery slot for na = 8.
hipError_t launch_matvec_scan(const DView& A, uint32_t r_begin, uint32_t r_end, uint32_t L,
                              const Fr* w_canon, const Fr* tab, uint32_t tl, Fr* out, int na, hipStream_t st);
// out[r] = sum_j A(r, j) w_j per job (job.tab = w's scaled table, job.out = the
// values, rows [0, job.rows)); one launch for all jobs. na as for the scans
// (0: from the jobs' NaSpecs and b.bitw on the device).
hipError_t launch_matvec_values(const ScanBatch& b, int na, hipStream_t st);
// b.g of b = X^T from svd_witness's f64 input X (R x C, row pitch ld), quantized
// in registers: part[s C + i] = sum over the rows j of slice s (colsum_slices(R)
// slices of 8 kColRows rows) of q(X[j][i]) g^j, with g's scaled table `tab`
// (length tl >= R) and the job's operand width from its NaSpec (bitw).
// k_vec_prep_sum then adds the S slices into the canonical vector and its table.
static constexpr int kMaxColJobs = 2;
static constexpr int kColRows = 16;       // rows per thread
static constexpr int kColPartBatch = 8;   // slice sums loaded together by k_vec_prep_sum
struct ColJob {
    const double* x;
    Fr* part;
    uint32_t R, C, ld;
    NaSpec spec;
};
struct ColBatch {
    ColJob job[kMaxColJobs];
    uint32_t njobs, tl;
    const Fr* tab;
    const unsigned* bitw;
};
uint32_t colsum_slices(uint32_t R);
hipError_t launch_colsum_f64(const ColBatch& b, int precision_bits, hipStream_t st);
hipError_t launch_vec_prep_sum(const Fr* part, uint32_t S, uint32_t L, Fr* w_canon, Fr* tab,
                               const ScaleTab& f, hipStream_t st);
// The same for up to kMaxColJobs vectors in one launch.
struct VecPrepJob {
    const Fr* part;
    uint32_t S, L;
    Fr* wc;
    Fr* tab;
    uint32_t blk0;                       // set by the launcher
};
struct VecPrepBatch {
    VecPrepJob job[kMaxColJobs];
    uint32_t njobs;
};
hipError_t launch_vec_prep_sum_multi(const VecPrepBatch& b, const ScaleTab& f, hipStream_t st);
// Up to kMaxScanJobs DPP row scans in one launch (two terms per thread; na
// shared by every job; na = 0: the max over the jobs' NaSpecs, read on the
// device from b.bitw, so the host needs no operand bounds).
hipError_t launch_scan_batch(const ScanBatch& b, int na, hipStream_t st);

}  // namespace svdw
