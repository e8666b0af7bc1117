"""BASELINE config 2: the matrix-multiplication recipe of README.md:32-46 as a
standalone workload -- phase 0 ZkMatrix::new(a), ZkMatrix::new(b),
c_s = honest_prover_mat_mul(a, b); phase 1 ZkMatrix::verify_mul(a, b, c_s, gamma)
(src/matrix/mod.rs:230-252, 546-568, 299-342).

CPU: the C oracle's recipe (oracle/svdw_oracle.c orc_verify_mul_witness) is pinned
against the Python restatement, honest and dishonest, and its cell counts against
the closed form of README.md:51 (~9 N^2 for verify_mul).
GPU: the full advice streams of the engine (modular C ABI) at 256 x 256, P=32
equal the C oracle's, for an honest c_s and for a c_s computed from a perturbed b
(then every is_equal row carries a non-zero difference and its inverse).
"""
import numpy as np
import pytest

import corc
import pyoracle as po
from conftest import P_MOD, gamma_for


def _inputs(n, k, m, seed):
    rs = np.random.RandomState(seed)
    a = rs.uniform(-1, 1, (n, k))
    b = rs.uniform(-1, 1, (k, m))
    bw = b.copy()
    bw[k // 2, m // 3] += 0.5              # one wrong entry of b: c_s wrong in one column
    return a, b, bw


def _ints(cells):
    c = cells.astype(object)
    return [int(r[0]) | int(r[1]) << 64 | int(r[2]) << 128 | int(r[3]) << 192 for r in c]


def vm_cells(n, k, m):
    """Phase-1 cells of verify_mul."""
    return 1 + 4 * (m - 1) + n * (3 * m + 1) + k * (3 * m + 1) + n * (3 * k + 1) + 12 * n


@pytest.mark.parametrize("wrong", [False, True])
@pytest.mark.parametrize("n,k,m,P", [(5, 7, 4, 32), (6, 6, 6, 63), (1, 3, 1, 42)])
def test_c_oracle_recipe_matches_python(n, k, m, P, wrong):
    a, b, bw = _inputs(n, k, m, seed=n * 100 + k * 10 + m)
    g = gamma_for(n + k + m)
    c0, c1 = corc.verify_mul_witness(a, b, P, g, b_wrong=bw if wrong else None)
    o0, o1, orlc = po.Context(phase=0), po.Context(phase=1), po.Context(phase=1)
    oa = po.zkmatrix_new(o0, P, a.tolist())
    ob = po.zkmatrix_new(o0, P, b.tolist())
    ow = po.zkmatrix_new(o0, P, bw.tolist()) if wrong else ob
    ocs = po.honest_prover_mat_mul(o0, oa, ow)
    po.verify_mul(o1, oa, ob, ocs, po.load_witness(orlc, g))
    assert _ints(c0) == o0.advice
    assert _ints(c1) == o1.advice
    assert len(c0) == n * k + k * m * (2 if wrong else 1) + n * m
    assert len(c1) == vm_cells(n, k, m)


def test_verify_mul_is_about_9n2_at_256():
    n = 256
    assert abs(vm_cells(n, n, n) / n ** 2 - 9) < 0.1          # README.md:51


def _is_equal_diffs(a1, n, k, m):
    """The n is_equal blocks close the phase-1 stream: [d, b, 1, a, z, d, inv, 1, 0, d, z, 0]."""
    blocks = _ints(a1[len(a1) - 12 * n:])
    return [(blk[0], blk[4], blk[6]) for blk in (blocks[12 * i:12 * i + 12] for i in range(n))]


@pytest.mark.gpu
@pytest.mark.parametrize("wrong", [False, True])
def test_config2_verify_mul_256_full_stream(gpu_ctx_factory, wrong):
    """BASELINE config 2 at full size: 256 x 256, PRECISION_BITS=32, bit-exact vs CPU."""
    import halo2_svd041_amd as hs
    n = k = m = 256
    P = 32
    a, b, bw = _inputs(n, k, m, seed=2)
    g = gamma_for(2)
    ctx = gpu_ctx_factory(P)
    za, zb = hs.ZkMatrix.new(ctx, a), hs.ZkMatrix.new(ctx, b)
    zw = hs.ZkMatrix.new(ctx, bw) if wrong else zb
    cs = hs.honest_prover_mat_mul(ctx, za, zw)
    hs.ZkMatrix.verify_mul(ctx, za, zb, cs, g)
    c0, c1 = corc.verify_mul_witness(a, b, P, g, b_wrong=bw if wrong else None)
    g0, g1 = ctx.advice(0), ctx.advice(1)
    assert g0.shape == c0.shape and g1.shape == c1.shape
    assert np.array_equal(g0, c0), "phase-0 advice differs from the C oracle"
    assert np.array_equal(g1, c1), "phase-1 advice differs from the C oracle"
    diffs = _is_equal_diffs(g1, n, k, m)
    if wrong:
        # a[i][k/2] != 0 for every row: every Freivalds row differs, is_zero = 0,
        # and the witness carries the inverse of the difference
        assert all(d != 0 and z == 0 and d * inv % P_MOD == 1 for d, z, inv in diffs)
    else:
        assert all(d == 0 and z == 1 for d, z, inv in diffs)
    chk = ctx.check_gates()
    assert chk["gate_failures"] == 0 and chk["lookup_failures"] == 0 and chk["copy_failures"] == 0


def test_fused_recipe_plans_like_the_modular_calls():
    """svdw_verify_mul_witness appends exactly the modular calls' cells (dry planner)."""
    import halo2_svd041_amd as hs
    for n, k, m, P in ((5, 7, 4, 32), (33, 17, 40, 63), (256, 256, 256, 32)):
        a, b, _ = _inputs(n, k, m, seed=n + k)
        with hs.Context(device=-1, precision_bits=P, lookup_bits=19) as c1, \
                hs.Context(device=-1, precision_bits=P, lookup_bits=19) as c2:
            got = hs.verify_mul_witness(c1, a, b, 7)
            za, zb = hs.ZkMatrix.new(c2, a), hs.ZkMatrix.new(c2, b)
            hs.ZkMatrix.verify_mul(c2, za, zb, hs.honest_prover_mat_mul(c2, za, zb), 7)
            assert got == {"advice0": c2.advice_len(0), "advice1": c2.advice_len(1),
                           "lookup0": c2.lookup_len(0), "lookup1": c2.lookup_len(1)}
            assert got["advice1"] == vm_cells(n, k, m)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,m,P,dev", [(256, 256, 256, 32, True), (256, 256, 256, 32, False),
                                         (45, 130, 37, 63, True), (1, 1, 1, 32, True)])
def test_fused_verify_mul_witness_full_stream(gpu_ctx_factory, n, k, m, P, dev):
    """The one-call recipe (svdw_verify_mul_witness: device-decided GEMM moduli and
    row-scan widths, no host waits) against the C oracle, full advice streams."""
    import torch
    import halo2_svd041_amd as hs
    a, b, _ = _inputs(n, k, m, seed=n + 3 * m)
    g = gamma_for(n + m)
    ctx = gpu_ctx_factory(P)
    if dev:
        ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
        hs.verify_mul_witness(ctx, ta, tb, g)
    else:
        hs.verify_mul_witness(ctx, a, b, g)
    c0, c1 = corc.verify_mul_witness(a, b, P, g)
    assert np.array_equal(ctx.advice(0), c0) and np.array_equal(ctx.advice(1), c1)
    chk = ctx.check_gates()
    assert chk["gate_failures"] == 0 and chk["lookup_failures"] == 0 and chk["copy_failures"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("pos", ["first", "middle", "last", "b_last"])
def test_bit_fold_outlier_block(gpu_ctx_factory, pos):
    """The operand bit-length words decide the GEMM's modulus count. One large
    entry in one quantize block (first / middle / last block of a, last of b)
    must reach the word through the in-launch fold: too few moduli would
    change c_s. 300 x 200 x 150 spans
    several 4096-value blocks; every run repeats twice (the fold's counter is
    reset by its last arrival)."""
    import torch
    import halo2_svd041_amd as hs
    n, k, m, P = 300, 200, 150, 63
    a, b, _ = _inputs(n, k, m, seed=11)
    a = a * 1e-3
    b = b * 1e-3
    big = 3.0e7                                     # 2^63 * 3e7 ~ 2^88 bits
    if pos == "first":
        a[0, 5] = big
    elif pos == "middle":
        a[n // 2, k // 3] = -big
    elif pos == "last":
        a[n - 1, k - 1] = big
    else:
        b[k - 1, m - 1] = -big
    g = gamma_for(n + m)
    ctx = gpu_ctx_factory(P)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    c0, c1 = corc.verify_mul_witness(a, b, P, g)
    for _ in range(2):
        ctx.reset()
        hs.verify_mul_witness(ctx, ta, tb, g)
        assert np.array_equal(ctx.advice(0), c0) and np.array_equal(ctx.advice(1), c1)


@pytest.mark.gpu
@pytest.mark.parametrize("pos", ["first", "last"])
def test_bit_fold_many_blocks(gpu_ctx_factory, pos):
    """A quantize launch of 2 103 blocks (4 096 values each; 4100 x 2100 a
    against a 2100 x 2 b): the fold's last block reads the block maxima in two
    rounds of 2 048. One outlier in the first or the last block."""
    import torch
    import halo2_svd041_amd as hs
    n, k, m, P = 4100, 2100, 2, 63
    rs = np.random.RandomState(21)
    a = rs.uniform(-1e-3, 1e-3, (n, k))
    b = rs.uniform(-1, 1, (k, m))
    a[(0, 7) if pos == "first" else (n - 1, k - 1)] = 3.0e7
    g = gamma_for(5)
    ctx = gpu_ctx_factory(P)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    c0, c1 = corc.verify_mul_witness(a, b, P, g)
    for _ in range(2):
        ctx.reset()
        hs.verify_mul_witness(ctx, ta, tb, g)
        assert np.array_equal(ctx.advice(0), c0) and np.array_equal(ctx.advice(1), c1)
