"""Pure-Python restatement of the reference's SVD-verify witness path.

TEST INFRASTRUCTURE ONLY. Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import anything under `oracle/`, and only
as the checker. The product path (`halo2_svd041_amd`) never imports this.

What it restates (all paths under the reference repo root):
  * halo2-base 0.4.1 gate/range layouts [ext crate, not vendored] as called from
    src/matrix/mod.rs and src/svd/mod.rs.
  * FixedPointChip041::quantization [ext crate], call sites
    src/matrix/mod.rs:36 and :245.
  * ZkVector / ZkMatrix / free functions of src/matrix/mod.rs:19-627.
  * check_svd_phase0 / check_svd_phase1 / err_calc of src/svd/mod.rs:32-163.

Pinning: the reference is Rust with un-vendored crates and cannot be built in
this image (no cargo/rustc, no crate sources).  This model is pinned by
(1) the closed-form cell-count coefficients published at README.md:67 and the
~9N^2 verify_mul count at README.md:51, reproduced exactly
(tests/test_oracle_pins.py), (2) the behavioural known-answer test of
README.md:93 (honest input satisfies every gate/copy/lookup; `matrix-wrong`
does not at P>=42), checked by `check_constraints`, and (3) inputs made by the
reference's own generator recipe (input-creator.py:23-49, seeded).  Cell
*values* are pinned through the gate equations, not through vectors emitted by
the reference binary ("values pinned by constraints").

Pure Python ints; meant for small shapes (N <= ~32).
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field
from typing import Optional, List, Sequence, Tuple

# BN254 scalar field modulus (halo2curves bn256::Fr).
P_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617


# ---------------------------------------------------------------------------
# Context / AssignedValue / QuantumCell  (halo2-base 0.4.1 [ext])
# ---------------------------------------------------------------------------
@dataclass
class Context:
    """Append-only virtual cell list of one phase (halo2-base `Context`).

    Besides the values it records what MockProver would check on the virtual
    layout: gate offsets (a + b*c = d at k..k+3), copy constraints (possibly
    across contexts), constant cells and the RangeChip lookup list.
    """
    phase: int = 0
    advice: List[int] = field(default_factory=list)
    lookups: List[int] = field(default_factory=list)      # values of looked-up cells
    lookup_idx: List[int] = field(default_factory=list)   # advice index of each lookup
    gates: List[int] = field(default_factory=list)
    copies: List[Tuple["AV", int]] = field(default_factory=list)
    consts: List[Tuple[int, int]] = field(default_factory=list)

    def get(self, i: int) -> "AV":
        return AV(self, i if i >= 0 else len(self.advice) + i)


@dataclass(frozen=True)
class AV:
    """AssignedValue: (context, offset)."""
    ctx: Context
    idx: int

    @property
    def value(self) -> int:
        return self.ctx.advice[self.idx]


# QuantumCell constructors
def E(av: AV):
    return ("E", av)


def C(val: int):
    return ("C", val % P_MOD)


def W(val: int):
    return ("W", val % P_MOD)


def qval(qc) -> int:
    kind, v = qc
    return v.value if kind == "E" else v


def assign_region(ctx: Context, cells, gate_offsets) -> int:
    base = len(ctx.advice)
    for kind, v in cells:
        i = len(ctx.advice)
        if kind == "E":
            ctx.advice.append(v.value)
            ctx.copies.append((v, i))
        elif kind == "C":
            ctx.advice.append(v)
            ctx.consts.append((i, v))
        else:
            ctx.advice.append(v)
    for g in gate_offsets:
        ctx.gates.append(base + g)
    return base


def load_witness(ctx: Context, v: int) -> AV:
    return ctx.get(assign_region(ctx, [W(v)], []))


def load_constant(ctx: Context, v: int) -> AV:
    return ctx.get(assign_region(ctx, [C(v)], []))


# ---------------------------------------------------------------------------
# GateChip — layouts per SURVEY.md Appendix A
# ---------------------------------------------------------------------------
def gate_add(ctx, a, b) -> AV:
    out = qval(a) + qval(b)
    return ctx.get(assign_region(ctx, [a, b, C(1), W(out)], [0]) + 3)


def gate_sub(ctx, a, b) -> AV:
    out = qval(a) - qval(b)
    return ctx.get(assign_region(ctx, [W(out), b, C(1), a], [0]))


def gate_mul(ctx, a, b) -> AV:
    out = qval(a) * qval(b)
    return ctx.get(assign_region(ctx, [C(0), a, b, W(out)], [0]) + 3)


def gate_inner_product(ctx, a: Sequence, b: Sequence) -> AV:
    """inner_product; b starting with Constant(1) elides the leading zero."""
    a, b = list(a), list(b)
    assert len(a) == len(b) and len(a) > 0
    if b[0][0] == "C" and b[0][1] == 1:
        s = qval(a[0])
        cells = [a[0]]
        pairs = zip(a[1:], b[1:])
    else:
        s = 0
        cells = [C(0)]
        pairs = zip(a, b)
    for ai, bi in pairs:
        s = (s + qval(ai) * qval(bi)) % P_MOD
        cells += [ai, bi, W(s)]
    ng = (len(cells) - 1) // 3
    base = assign_region(ctx, cells, [3 * i for i in range(ng)])
    return ctx.get(base + len(cells) - 1)


def gate_is_zero(ctx, a: AV) -> AV:
    x = a.value
    z, inv = (1, 1) if x == 0 else (0, pow(x, P_MOD - 2, P_MOD))
    base = assign_region(ctx, [W(z), E(a), W(inv), C(1), C(0), E(a), W(z), C(0)], [0, 4])
    ctx.copies.append((ctx.get(base), base + 6))
    return ctx.get(base + 6)


def gate_is_equal(ctx, a, b) -> AV:
    return gate_is_zero(ctx, gate_sub(ctx, a, b))


def gate_assert_bit(ctx, x: AV) -> None:
    assign_region(ctx, [C(0), E(x), E(x), E(x)], [0])


# ---------------------------------------------------------------------------
# RangeChip
# ---------------------------------------------------------------------------
class RangeChip:
    def __init__(self, lookup_bits: int):
        assert 1 <= lookup_bits <= 64
        self.lb = lookup_bits

    def add_cell_to_lookup(self, ctx, a: AV) -> None:
        ctx.lookups.append(a.value)
        ctx.lookup_idx.append(a.idx)

    def range_check(self, ctx, a: AV, range_bits: int) -> None:
        lb = self.lb
        if range_bits == 0:
            ctx.consts.append((a.idx, 0))
            return
        n = -(-range_bits // lb)
        rem = range_bits % lb
        if n == 1:
            self.add_cell_to_lookup(ctx, a)
            last = a
        else:
            v = a.value
            mask = (1 << lb) - 1
            limbs = [(v >> (lb * i)) & mask for i in range(n)]
            row = len(ctx.advice)
            acc = gate_inner_product(ctx, [W(x) for x in limbs],
                                     [C(1 << (lb * i)) for i in range(n)])
            ctx.copies.append((a, acc.idx))
            self.add_cell_to_lookup(ctx, ctx.get(row))
            for i in range(n - 1):
                self.add_cell_to_lookup(ctx, ctx.get(row + 1 + 3 * i))
            last = ctx.get(row + 1 + 3 * (n - 2))
        if rem == 1:
            gate_assert_bit(ctx, last)
        elif rem > 1:
            chk = gate_mul(ctx, E(last), C(1 << (lb - rem)))
            self.add_cell_to_lookup(ctx, chk)

    def check_less_than(self, ctx, a, b, num_bits: int) -> None:
        pw = 1 << num_bits
        shift = pw + qval(a)
        base = assign_region(ctx, [W(shift - qval(b)), b, C(1), W(shift), C(-pw), C(1), a], [0, 3])
        self.range_check(ctx, ctx.get(base), num_bits)

    def check_big_less_than_safe(self, ctx, a: AV, bnd: int) -> None:
        rb = -(-bnd.bit_length() // self.lb) * self.lb
        self.range_check(ctx, a, rb)
        self.check_less_than(ctx, E(a), C(bnd), rb)


# ---------------------------------------------------------------------------
# FixedPointChip041::quantization [ext]
# ---------------------------------------------------------------------------
U128_MAX = (1 << 128) - 1


def rust_round(x: float) -> float:
    """f64::round: ties away from zero."""
    if math.isnan(x) or math.isinf(x):
        return x
    t = math.trunc(x)
    if abs(x - t) >= 0.5:
        return t + math.copysign(1.0, x)
    return float(t)


def f64_to_u128_sat(x: float) -> int:
    """Rust `as u128`: NaN -> 0, negative -> 0, >= 2^128 -> u128::MAX."""
    if math.isnan(x) or x <= 0:
        return 0
    if x >= 2.0 ** 128:
        return U128_MAX
    return int(x)


def quantize(x: float, precision_bits: int) -> int:
    """x -> round(|x| 2^P) as u128; sign<0 (signum, so -0.0 too) -> p - x_q."""
    neg = (not math.isnan(x)) and math.copysign(1.0, x) < 0
    xq = f64_to_u128_sat(rust_round(abs(x) * float(1 << precision_bits)))
    return (P_MOD - xq) % P_MOD if neg else xq


def to_signed(v: int) -> int:
    return v - P_MOD if v > P_MOD // 2 else v


# ---------------------------------------------------------------------------
# src/matrix/mod.rs
# ---------------------------------------------------------------------------
def zkmatrix_new(ctx, p: int, m) -> List[List[AV]]:
    """ZkMatrix::new (src/matrix/mod.rs:230-252)."""
    cols = len(m[0])
    out = []
    for row in m:
        assert len(row) == cols
        out.append([load_witness(ctx, quantize(float(x), p)) for x in row])
    return out


def zkvector_new(ctx, p: int, v) -> List[AV]:
    """ZkVector::new (src/matrix/mod.rs:29-40)."""
    return [load_witness(ctx, quantize(float(x), p)) for x in v]


def transpose(a):
    """ZkMatrix::transpose_matrix (src/matrix/mod.rs:408-419): no cells."""
    return [list(col) for col in zip(*a)]


def check_abs_less_than(ctx, rc: RangeChip, x: AV, bnd: int) -> None:
    """src/matrix/mod.rs:425-435."""
    assert bnd >= 1
    t = gate_add(ctx, E(x), C(bnd - 1))
    rc.check_big_less_than_safe(ctx, t, 2 * bnd - 1)


def check_mat_diff(ctx, rc, a, b, tol: int) -> None:
    """src/matrix/mod.rs:441-457."""
    assert len(a) == len(b) and len(a[0]) == len(b[0])
    for i in range(len(a)):
        for j in range(len(a[0])):
            check_abs_less_than(ctx, rc, gate_sub(ctx, E(a[i][j]), E(b[i][j])), tol)


def check_mat_id(ctx, rc, a, scalar_id: AV, tol: int) -> None:
    """src/matrix/mod.rs:461-483."""
    zero = load_constant(ctx, 0)
    b = [[scalar_id if i == j else zero for j in range(len(a[0]))] for i in range(len(a))]
    check_mat_diff(ctx, rc, a, b, tol)


def check_mat_entries_bounded(ctx, rc, a, bnd: int) -> None:
    """src/matrix/mod.rs:490-501."""
    for row in a:
        for x in row:
            check_abs_less_than(ctx, rc, x, bnd)


def field_mat_mul(a, b) -> List[List[int]]:
    """src/matrix/mod.rs:510-537 (values only)."""
    assert len(a[0]) == len(b)
    av = [[x.value for x in r] for r in a]
    bv = [[x.value for x in r] for r in b]
    k, m = len(b), len(b[0])
    return [[sum(ar[t] * bv[t][j] for t in range(k)) % P_MOD for j in range(m)] for ar in av]


def honest_prover_mat_mul(ctx, a, b):
    """src/matrix/mod.rs:546-568."""
    return [[load_witness(ctx, x) for x in row] for row in field_mat_mul(a, b)]


def field_mat_vec_mul(ctx, a, v) -> List[AV]:
    """src/matrix/mod.rs:574-599: one inner_product per row."""
    assert len(a[0]) == len(v)
    return [gate_inner_product(ctx, [E(x) for x in row], [E(y) for y in v]) for row in a]


def mat_times_diag_mat(ctx, a, v):
    """src/matrix/mod.rs:610-627."""
    assert len(v) <= len(a[0])
    return [[gate_mul(ctx, E(a[i][j]), E(v[j])) for j in range(len(v))] for i in range(len(a))]


def entries_less_than(ctx, rc, d, max_bits: int) -> None:
    """ZkVector::entries_less_than (src/matrix/mod.rs:185-194)."""
    for x in d:
        rc.range_check(ctx, x, max_bits)


def entries_in_desc_order(ctx, rc, d, max_bits: int) -> None:
    """ZkVector::entries_in_desc_order (src/matrix/mod.rs:199-215); qsub = gate.sub."""
    diffs = [gate_sub(ctx, E(d[i]), E(d[i + 1])) for i in range(len(d) - 1)]
    for x in diffs:
        rc.range_check(ctx, x, max_bits)


def verify_mul(ctx, a, b, c_s, init_rand: AV) -> None:
    """ZkMatrix::verify_mul (src/matrix/mod.rs:299-342)."""
    assert len(a[0]) == len(b) and len(c_s) == len(a) and len(c_s[0]) == len(b[0])
    d = len(c_s[0])
    assert d >= 1
    one = load_witness(ctx, 1)
    ctx.consts.append((one.idx, 1))     # assert_is_const
    v = [one]
    for _ in range(1, d):
        v.append(gate_mul(ctx, E(v[-1]), E(init_rand)))
    cs_v = field_mat_vec_mul(ctx, c_s, v)
    b_v = field_mat_vec_mul(ctx, b, v)
    ab_v = field_mat_vec_mul(ctx, a, b_v)
    for i in range(len(cs_v)):
        gate_is_equal(ctx, E(cs_v[i]), E(ab_v[i]))  # result unconstrained (mod.rs:339-341)


# ---------------------------------------------------------------------------
# FixedPointChip041::signed_div_scale [ext, PARITY UNPINNED] and its callers
# ---------------------------------------------------------------------------
def div_scale_defaults(p: int, shift_bits: int = 0, num_bits: int = 0):
    """Default constants: the input domain |x| < 2^(3P) that rescale_matrix's
    doc comment states (src/matrix/mod.rs:350-353): shift 2^(3P); div_mod on
    4P+1 bits, the width that reproduces the reference's own counts (90 cells
    per element at P=32, LB=12: src/matrix/mod.rs:102 "#CONSTRAINTS = 90",
    :348 "~94"; README.md:51 60-100 N^2; include/svdw.h svdw_div_scale)."""
    s = shift_bits or 3 * p
    nb = num_bits or max(4 * p + 1, s + 1)      # (a shift alone >= 4P+1 widens the div_mod)
    assert p <= s < 254 and s < nb <= 253 and nb - p <= 200
    return s, nb


def range_div_mod(ctx, rc: RangeChip, a: AV, b: int, a_num_bits: int):
    """RangeChip::div_mod [ext halo2-base 0.4.1, recalled]: [r, C(b), q, a]
    (gate r + b*q = a), then check_big_less_than_safe(q, 2^nb / b + 1) and
    check_big_less_than_safe(r, b)."""
    q, r = divmod(a.value, b)
    base = assign_region(ctx, [W(r), C(b), W(q), E(a)], [0])
    rem, div = ctx.get(base), ctx.get(base + 2)
    rc.check_big_less_than_safe(ctx, div, (1 << a_num_bits) // b + 1)
    rc.check_big_less_than_safe(ctx, rem, b)
    return div, rem


def signed_div_scale(ctx, rc: RangeChip, a: AV, p: int, shift_bits: int = 0, num_bits: int = 0):
    """FixedPointChip041::signed_div_scale (called at src/matrix/mod.rs:104,369;
    src/matrix/test_matrix.rs:259). The chip's source (zk_fixed_point_chip git
    HEAD) is not available offline, so this is a parameterised restatement of
    the usual shift / div_mod / unshift construction: t = a + 2^S (add),
    (q, r) = div_mod(t, 2^P, nb), y = q - 2^(S-P) (sub). For |x| < 2^S the
    result is floor(x / 2^P) in signed encoding. Returns (y, r)."""
    s, nb = div_scale_defaults(p, shift_bits, num_bits)
    t = gate_add(ctx, E(a), C(1 << s))
    q, r = range_div_mod(ctx, rc, t, 1 << p, nb)
    y = gate_sub(ctx, E(q), C(1 << (s - p)))
    return y, r


def rescale_matrix(ctx, rc, c_s, p: int, shift_bits: int = 0, num_bits: int = 0):
    """ZkMatrix::rescale_matrix (src/matrix/mod.rs:354-375): row-major
    signed_div_scale of every entry; returns the quotient matrix."""
    return [[signed_div_scale(ctx, rc, x, p, shift_bits, num_bits)[0] for x in row] for row in c_s]


def zkvector_inner_product(ctx, rc, vec, x, p: int, shift_bits: int = 0, num_bits: int = 0) -> AV:
    """ZkVector::inner_product (src/matrix/mod.rs:79-106): gate.inner_product(x,
    self) then signed_div_scale."""
    assert len(vec) == len(x) and len(x) >= 1
    res_s = gate_inner_product(ctx, [E(a) for a in x], [E(b) for b in vec])
    return signed_div_scale(ctx, rc, res_s, p, shift_bits, num_bits)[0]


def zkvector_norm_square(ctx, rc, vec, p: int, shift_bits: int = 0, num_bits: int = 0) -> AV:
    """ZkVector::_norm_square (src/matrix/mod.rs:112-119): self.inner_product(self)."""
    return zkvector_inner_product(ctx, rc, vec, vec, p, shift_bits, num_bits)


def qsqrt(ctx, rc: RangeChip, a: AV, p: int, sqrt_bits: int = 0) -> AV:
    """FixedPointChip041::qsqrt [ext, PARITY UNPINNED: the chip's source is not
    available offline] as the engine's parameterised construction (include/svdw.h
    svdw_zkvector_norm): y = floor(sqrt(a 2^P)) for a in [0, 2^B), B = sqrt_bits
    or 2P; y^2 <= a 2^P < (y + 1)^2 enforced by two range-checked differences."""
    nb = sqrt_bits or 2 * p
    ny = (nb + p + 1) // 2 + 1
    y = load_witness(ctx, math.isqrt(a.value * (1 << p)))
    rc.range_check(ctx, y, ny)
    t = gate_mul(ctx, E(a), C(1 << p))
    y2 = gate_mul(ctx, E(y), E(y))
    d = gate_sub(ctx, E(t), E(y2))
    rc.range_check(ctx, d, ny + 1)
    e = gate_mul(ctx, E(y), C(2))
    f = gate_sub(ctx, E(e), E(d))
    rc.range_check(ctx, f, ny + 1)
    return y


def zkvector_norm(ctx, rc, vec, p: int, shift_bits: int = 0, num_bits: int = 0, sqrt_bits: int = 0) -> AV:
    """ZkVector::norm (src/matrix/mod.rs:124-131): qsqrt(_norm_square)."""
    return qsqrt(ctx, rc, zkvector_norm_square(ctx, rc, vec, p, shift_bits, num_bits), p, sqrt_bits)


def zkvector_dist(ctx, rc, vec, x, p: int, shift_bits: int = 0, num_bits: int = 0, sqrt_bits: int = 0) -> AV:
    """ZkVector::dist (src/matrix/mod.rs:156-164): qsqrt(_dist_square(x))."""
    return qsqrt(ctx, rc, zkvector_dist_square(ctx, rc, vec, x, p, shift_bits, num_bits), p, sqrt_bits)


def zkvector_dist_square(ctx, rc, vec, x, p: int, shift_bits: int = 0, num_bits: int = 0) -> AV:
    """ZkVector::_dist_square (src/matrix/mod.rs:135-148): diff_i = fpchip.qsub(self_i,
    x_i) [ext; gate.sub, as in entries_in_desc_order], then diff._norm_square."""
    assert len(vec) == len(x)
    diff = [gate_sub(ctx, E(a), E(b)) for a, b in zip(vec, x)]
    return zkvector_norm_square(ctx, rc, diff, p, shift_bits, num_bits)


def zkvector_mul(ctx, rc, vec, a, p: int, shift_bits: int = 0, num_bits: int = 0) -> List[AV]:
    """ZkVector::mul (src/matrix/mod.rs:169-182): inner_product with each row of a."""
    assert len(a[0]) == len(vec)
    return [zkvector_inner_product(ctx, rc, vec, row, p, shift_bits, num_bits) for row in a]


# ---------------------------------------------------------------------------
# src/svd/mod.rs
# ---------------------------------------------------------------------------
def err_calc(p: int, size: int, max_norm: float, eps_svd: float, eps_u: float):
    """src/svd/mod.rs:155-163, same f64 operation order; powf -> libm pow."""
    precision = math.pow(2.0, -1.0 * (float(p) + 1.0))
    s = float(size)
    err_svd = (precision * s * (1.0 + max_norm + eps_svd + precision)
               + s * max_norm * precision
               + math.pow(1.0 + eps_u, 0.5) * (max_norm + eps_svd) * eps_u
               + math.pow(1.0 + eps_u, 0.5) * eps_svd)
    err_u = eps_u + precision * s * (2.0 * (1.0 + eps_u) + precision)
    return err_svd, err_u


def scale_err(err: float, p: int) -> int:
    """`(err * (2u128.pow(2P) as f64)).round() as u128` (src/svd/mod.rs:99-102)."""
    return f64_to_u128_sat(rust_round(err * float(1 << (2 * p))))


@dataclass
class SvdPayload:
    u_t: list
    v_t: list
    m_times_vt: list
    u_times_ut: list
    v_times_vt: list


def check_svd_phase0(ctx, rc, p, m, u, v, d, err_svd, err_u, max_bits_d) -> SvdPayload:
    """src/svd/mod.rs:32-116."""
    N, M = len(m), len(m[0])
    r = min(N, M)
    assert len(u) == N and len(u[0]) == N and len(v) == M and len(v[0]) == M
    assert len(d) == r
    max_bits = max_bits_d + p
    entries_less_than(ctx, rc, d, max_bits)
    entries_in_desc_order(ctx, rc, d, max_bits)
    unit_bnd = (1 << p) + 1
    check_mat_entries_bounded(ctx, rc, u, unit_bnd)
    check_mat_entries_bounded(ctx, rc, v, unit_bnd)
    u_t, v_t = transpose(u), transpose(v)
    if r == M:
        ud = mat_times_diag_mat(ctx, u, d)
    else:
        zero = load_constant(ctx, 0)
        ud = mat_times_diag_mat(ctx, u, d)
        for row in ud:
            row.extend([zero] * (M - N))
    mvt = honest_prover_mat_mul(ctx, m, v_t)
    check_mat_diff(ctx, rc, ud, mvt, scale_err(err_svd, p))
    q2 = load_constant(ctx, (1 << p) * (1 << p))
    uut = honest_prover_mat_mul(ctx, u, u_t)
    check_mat_id(ctx, rc, uut, q2, scale_err(err_u, p))
    vvt = honest_prover_mat_mul(ctx, v, v_t)
    check_mat_id(ctx, rc, vvt, q2, scale_err(err_u, p))
    return SvdPayload(u_t, v_t, mvt, uut, vvt)


def check_svd_phase1(ctx, m, u, v, pl: SvdPayload, init_rand: AV) -> None:
    """src/svd/mod.rs:127-144."""
    verify_mul(ctx, m, pl.v_t, pl.m_times_vt, init_rand)
    verify_mul(ctx, u, pl.u_t, pl.u_times_ut, init_rand)
    verify_mul(ctx, v, pl.v_t, pl.v_times_vt, init_rand)


# ---------------------------------------------------------------------------
# Whole-witness driver: intended semantics of examples/svd_example.rs:98-200
# (m, u, v, d and check_svd_phase0 in ONE phase-0 context).
# gamma (init_rand) sits in its own RLC context: not part of the streams.
# ---------------------------------------------------------------------------
@dataclass
class SvdWitness:
    ctx0: Context
    ctx1: Context
    err_svd: float
    err_u: float
    rlc: Optional[Context] = None     # ctx_rlc (rlc_prefix: [E(one), E(zero), W(gamma)])


def load_rlc_cache_1(ctx_gate: Context, rlc: Context, gamma: int) -> AV:
    """rlc.load_rlc_cache((ctx_gate, ctx_rlc), gate, 1) then gamma_pow_cached()[0]
    (examples/svd_example.rs:183-184), as recalled from axiom-eth's RlcChip
    (un-vendored crate; PARITY UNPINNED): an empty cache loads gamma as
    compute_rlc_fixed_len(ctx_rlc, [one, zero]) = one * gamma + zero, with
    one = ctx_gate.load_constant(1) and zero = ctx_gate.load_zero() (a constant);
    the RLC trace [E(one), E(zero), W(gamma)] lives in ctx_rlc."""
    one = load_constant(ctx_gate, 1)
    zero = load_constant(ctx_gate, 0)
    return rlc.get(assign_region(rlc, [E(one), E(zero), W(gamma)], []) + 2)


def svd_witness(m, u, v, d, p: int, lookup_bits: int, gamma: int,
                max_norm: float = 100.0, eps_svd: float = 1e-10, eps_u: float = 1e-10,
                max_bits_d: int = 30, rlc_prefix: bool = False) -> SvdWitness:
    rc = RangeChip(lookup_bits)
    ctx0 = Context(phase=0)
    zm = zkmatrix_new(ctx0, p, m)
    zu = zkmatrix_new(ctx0, p, u)
    zv = zkmatrix_new(ctx0, p, v)
    zd = zkvector_new(ctx0, p, d)
    err_svd, err_u = err_calc(p, max(len(m), len(m[0])), max_norm, eps_svd, eps_u)
    pl = check_svd_phase0(ctx0, rc, p, zm, zu, zv, zd, err_svd, err_u, max_bits_d)
    rlc = Context(phase=1)
    ctx1 = Context(phase=1)
    g = load_rlc_cache_1(ctx1, rlc, gamma) if rlc_prefix else load_witness(rlc, gamma)
    check_svd_phase1(ctx1, zm, zu, zv, pl, g)
    return SvdWitness(ctx0, ctx1, err_svd, err_u, rlc)


# ---------------------------------------------------------------------------
# Constraint checker (MockProver-equivalent on the virtual layout)
# ---------------------------------------------------------------------------
def check_constraints(ctx: Context, lookup_bits: int) -> List[str]:
    a = ctx.advice
    bad = []
    for k in ctx.gates:
        if (a[k] + a[k + 1] * a[k + 2] - a[k + 3]) % P_MOD != 0:
            bad.append(f"gate@{k}")
    for src, i in ctx.copies:
        if src.value != a[i]:
            bad.append(f"copy->{i}")
    for i, c in ctx.consts:
        if a[i] != c % P_MOD:
            bad.append(f"const@{i}")
    lim = 1 << lookup_bits
    for idx, val in zip(ctx.lookup_idx, ctx.lookups):
        if val >= lim or a[idx] != val:
            bad.append(f"lookup@{idx}")
    return bad


# ---------------------------------------------------------------------------
# Virtual -> physical layout
# ---------------------------------------------------------------------------
# Restated from halo2-base 0.4.1 [ext, not on disk; recalled, parity unpinned]:
# BaseCircuitBuilder::calculate_params (max_rows = 2^k - minimum_rows, columns =
# ceil(cells / max_rows), called from src/utils/executor.rs:48-55 and
# src/scaffold/mod.rs:245-247 with MINIMUM_ROWS default 20), the keygen
# assignment of a phase's virtual cells to basic-gate advice columns (a column
# breaks at a cell whose gate would cross max_rows, or at row max_rows - 1; the
# break cell is repeated at row 0 of the next column, copy-constrained, and its
# selector is enabled only there), and the lookup-advice chunking (lookup cells
# in order, max_rows per column).
@dataclass
class Physical:
    k: int
    max_rows: int
    num_advice: int                 # calculate_params' estimate
    columns: List[List[int]]        # advice column values (used rows only)
    selectors: List[List[int]]      # q_enable per used row
    break_points: List[int]         # per column but the last: the row of its last cell
    lookup_columns: List[List[int]]
    num_lookup_advice: int
    num_fixed: int


def physical_layout(ctx: Context, k: int, minimum_rows: int = 20) -> Physical:
    R = (1 << k) - minimum_rows
    assert R >= 4
    q = set(ctx.gates)
    cols, sels, bps = [[]], [[]], []
    row = 0
    for i, v in enumerate(ctx.advice):
        cols[-1].append(v)
        sels[-1].append(0)
        if (i in q and row + 4 > R) or row >= R - 1:
            bps.append(row)
            row = 0
            cols.append([v])
            sels.append([0])
        if i in q:
            sels[-1][row] = 1
        row += 1
    if not ctx.advice:
        cols, sels = [], []
    lk = [ctx.lookups[j:j + R] for j in range(0, len(ctx.lookups), R)]
    distinct = len({c % P_MOD for _, c in ctx.consts})
    return Physical(k, R, -(-len(ctx.advice) // R), cols, sels, bps, lk,
                    -(-len(ctx.lookups) // R), -(-distinct // (1 << k)))


def cells_to_bytes(vals: Sequence[int]) -> bytes:
    """Canonical little-endian 32-byte cells (halo2curves Fr::to_repr)."""
    return b"".join(int(x).to_bytes(32, "little") for x in vals)


def f64_bits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]
