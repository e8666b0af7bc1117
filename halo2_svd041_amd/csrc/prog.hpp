// Cell programs: the data-independent layout of one element's block of
// advice / lookup cells for a gadget stage, as emitted by the generic
// streaming kernel (kernels.hip: k_stage).
//
// Every halo2-base 0.4.1 gadget used on the hot path (GateChip add / sub / mul
// / is_equal / assert_bit, RangeChip range_check / check_less_than /
// check_big_less_than_safe, and the reference's check_abs_less_than,
// src/matrix/mod.rs:425-435) appends, per element, a fixed number of cells
// whose values are simple functions of a few per-element field values:
//   * a handful of field values V[0..nv) computed per element by micro-ops
//     (load from a matrix view, +constant, -, *, limb<<shift, is_zero/inverse,
//     gamma^k), and
//   * for every cell: (V[src] >> lo) & (2^nbits - 1)  or a constant K[k].
// Range-check limbs are bit windows of the canonical value, and the running
// sums of the limb inner product are `value mod 2^(i*LB)`.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "fr.hpp"

namespace svdw {

// ------------------------------------------------------------------ views
// Matrix view over canonical Fr cells: X(i, j) = ptr[i*rs + j*cs] for
// i < rows && j < cols, else K[pad_k]. mode DIAG: X(i,j) = i==j ? *ptr : K[pad_k]
// (check_mat_id's implicit scalar_id * Id matrix, src/matrix/mod.rs:461-483).
// mode DIAGK: X(i,j) = i==j ? K[diag_k] : K[pad_k] (the same matrix when the
// diagonal scalar is a constant the host knows: no read of its cell).
// VIEW_F64: ptr is a row-major f64 input (svd_witness / verify_mul_witness
// device inputs) laid out like the loaded cells; element (i, j) is its
// ZkMatrix::new quantization at PRECISION_BITS = _r0, computed in registers.
enum : uint32_t { VIEW_STRIDED = 0, VIEW_DIAG = 1, VIEW_DIAGK = 2, VIEW_F64 = 3 };
struct DView {
    const Fr* ptr;
    int64_t rs, cs;
    uint32_t rows, cols;
    uint32_t mode;
    uint8_t pad_k, diag_k, _r0, _r1;
};

// ------------------------------------------------------------ micro-ops
enum : uint8_t {
    MO_LOAD = 1,     // V[dst] = view[a](i, j)
    MO_ADDK,         // V[dst] = V[a] + K[b]
    MO_SUB,          // V[dst] = V[a] - V[b]
    MO_MUL,          // V[dst] = V[a] * V[b]
    MO_LIMBSHL,      // V[dst] = ((V[a] >> p0) & (2^p1 - 1)) << b      (non-modular, < 2^128)
    MO_FDBL,         // V[dst] = V[a] * 2^b mod p
    MO_ISZERO,       // V[dst] = (V[a]==0), V[dst+1] = V[a]==0 ? 1 : V[a]^-1
    MO_POWK,         // V[dst] = K[a] ^ (e + p0)                         (verify_mul's gamma powers)
    MO_SHR,          // V[dst] = V[a] >> p0 (canonical value, full width; div_mod quotients)
    MO_ISQRT,        // V[dst] = floor(sqrt(V[a])) of the canonical value as an integer (< 2^256)
};
struct MicroOp {
    uint8_t op, dst, a, b;
    uint16_t p0, p1;
};

// ------------------------------------------------------------- slot ops
// value = (S >> lo) & (2^nbits - 1); nbits == 0 keeps all 256 bits.
// src < 0x80: element value V[src]; src >= 0x80: constant K[src - 0x80].
struct SlotOp {
    uint8_t src, lo, nbits, _pad;
};
static constexpr uint8_t KSRC = 0x80;

static constexpr uint32_t STAGE_ALIGN = 256;     // 4 KiB-aligned block store windows
static constexpr uint32_t STAGE_ROT = 512;       // blocks start phase B at a block-dependent window

static constexpr int kMaxViews = 2;
static constexpr int kMaxMicro = 16;
static constexpr int kMaxAdv = 160;
static constexpr int kMaxLk = 48;
static constexpr int kMaxK = 32;
static constexpr int kMaxV = 12;

// Kernel argument block of one stage launch (passed by value, < 4 KiB).
struct StageArgs {
    Fr* out_adv;          // cell 0 of element 0 of this stage
    Fr* out_lk;           // lookup cell 0 of element 0 (may be null if L == 0)
    uint32_t e_begin, e_end;   // element range processed by this launch
    uint32_t cols;        // element e -> (i, j) = (e / cols, e % cols)
    uint32_t C, L;        // advice / lookup cells per element
    uint32_t nv, nmo, nk;
    uint32_t flags;       // STAGE_* bits
    uint32_t cdiv_magic;  // ceil(2^32 / C) (C >= 2): x / C = mul_hi(x, magic) for x * C < 2^32
    uint32_t ldiv_magic;  // ceil(2^32 / L)
    uint32_t E;           // elements per block (<= 256 = block size); 0 -> 256
    DView view[kMaxViews];
    MicroOp mo[kMaxMicro];
    SlotOp adv[kMaxAdv];
    SlotOp lk[kMaxLk];
    Fr K[kMaxK];
};
static_assert(sizeof(StageArgs) < 4096, "kernel argument block too large");

// A batch of independent stages in one launch (k_stage_multi). Each program is
// a compact record in `data`: StageArgs up to `mo` (scalar fields and views,
// kRecHead bytes), then its nmo micro-ops, C + L slot ops and nk constants.
// Program p runs blocks [blk0[p], blk0[p + 1]).
static constexpr uint32_t kRecHead = (uint32_t)offsetof(StageArgs, mo);
static_assert(kRecHead % 8 == 0, "record head keeps 8-byte alignment");
constexpr uint32_t stage_record_bytes(uint32_t nmo, uint32_t C, uint32_t L, uint32_t nk) {
    return (kRecHead + 8 * nmo + 4 * (C + L) + 32 * nk + 7) / 8 * 8;
}
static constexpr int kMaxMulti = 16;
static constexpr uint32_t kMultiBytes = 3712;
struct StageMulti {
    uint32_t nprog;
    uint32_t blk0[kMaxMulti + 1];
    uint32_t off[kMaxMulti];
    uint32_t _pad;
    alignas(8) uint8_t data[kMultiBytes];
};
static_assert(sizeof(StageMulti) < 4096, "kernel argument block too large");

// Phase-B half-cell descriptor (one per slot and half, built per block in LDS):
// output words [4h, 4h+4) of a cell are alignbit(x[i+1], x[i], r) & mask[i]
// with x = the 5 LDS words from word `off` of the constants (bit 31 clear) or
// of the element's values (bit 31 set); the masks already clip the window to
// `nbits` and to the 256 bits of the source, so words read past the source
// value (up to 12) are masked off.
static constexpr uint32_t kHalfElem = 0x80000000u;
constexpr uint32_t half_desc(uint32_t off, uint32_t r, bool elem) {
    return off | (r << 16) | (elem ? kHalfElem : 0u);
}
static constexpr uint32_t kStageLdsPad = 64;   // over-read slack after the last table

// LDS words per element in a stage block: nv values of 8 words + 4 words of
// padding. Phase A reads / writes a value with ds_read/write_b128 at lane stride
// stage_elem_words(nv); a stride of 4 (mod 8) words puts the 16 lanes of one
// b128 pass on 16 distinct 4-bank groups (nv * 8 alone: 2- to 16-way conflicts).
constexpr uint32_t stage_elem_words(uint32_t nv) { return nv * 8 + 4; }

// Dynamic LDS of a stage block: constants, E elements' values, slot / micro-op
// tables, views, and per (slot, half) descriptors (4 B) + masks (16 B) for the
// C + L slots (constexpr: host and device).
constexpr uint32_t stage_lds_bytes(uint32_t nv, uint32_t E, uint32_t CL = kMaxAdv + kMaxLk) {
    return kMaxK * 32 + E * stage_elem_words(nv) * 4 + (kMaxAdv + kMaxLk) * 4 + kMaxMicro * 8 + kMaxViews * 48 +
           CL * 2 * 20 + kStageLdsPad;
}

}  // namespace svdw
