"""GPU parity: the HIP witness engine vs the CPU oracle restatement, bit-exact.

Every test calls the product through the C ABI (halo2_svd041_amd -> libsvdw.so)
and compares the full advice / lookup streams with oracle/svdw_oracle.c on the
same seeded inputs (input-creator.py recipe) and the same gamma.
"""
import numpy as np
import pytest

import corc
from conftest import gamma_for, gen_svd_input

pytestmark = pytest.mark.gpu


def _assert_streams(ctx, a0, l0, a1):
    g0, gl0, g1 = ctx.advice(0), ctx.lookups(0), ctx.advice(1)
    assert g0.shape == a0.shape, (g0.shape, a0.shape)
    assert g1.shape == a1.shape, (g1.shape, a1.shape)
    assert gl0.shape == l0.shape, (gl0.shape, l0.shape)
    for name, g, o in (("advice0", g0, a0), ("lookup0", gl0, l0), ("advice1", g1, a1)):
        bad = np.nonzero(np.any(g != o, axis=1))[0]
        assert bad.size == 0, f"{name}: {bad.size} cells differ, first at {bad[:8]}"


SHAPES = [
    (1, 1, 32), (2, 2, 63), (4, 4, 32), (4, 3, 63), (3, 4, 42), (6, 6, 42), (5, 7, 63),
    (8, 8, 32), (16, 16, 63), (33, 31, 32), (31, 33, 63), (40, 40, 40), (64, 64, 63),
]


@pytest.mark.parametrize("N,M,P", SHAPES)
def test_svd_witness_parity(gpu_ctx_factory, N, M, P):
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N * 1000 + M * 10 + P)
    g = gamma_for(N + M + P)
    ctx = gpu_ctx_factory(P)
    cnt = hs.svd_witness(ctx, m, u, v, d, g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    assert cnt["advice0"] == a0.shape[0] and cnt["advice1"] == a1.shape[0]
    _assert_streams(ctx, a0, l0, a1)


@pytest.mark.parametrize("lb", [8, 11, 13, 17, 24])
def test_lookup_bits_parity(gpu_ctx_factory, lb):
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(9, 7, seed=lb)
    g = gamma_for(lb)
    for P in (32, 63):
        ctx = gpu_ctx_factory(P, lb)
        hs.svd_witness(ctx, m, u, v, d, g)
        a0, l0, a1 = corc.svd_witness(m, u, v, d, P, lb, g)
        _assert_streams(ctx, a0, l0, a1)


def test_matrix_wrong_parity(gpu_ctx_factory):
    """input-creator.py:46-49 perturbation: witness still bit-exact."""
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(12, 12, seed=5)
    m = m.copy()
    m[3][7] += 1e-7
    for P in (32, 63):
        ctx = gpu_ctx_factory(P)
        hs.svd_witness(ctx, m, u, v, d, gamma_for(7))
        a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, gamma_for(7))
        _assert_streams(ctx, a0, l0, a1)


def test_garbage_inputs_parity(gpu_ctx_factory):
    """Non-SVD inputs: large, tiny, negative zero, ties, NaN, inf (quantization
    edges; non-zero Freivalds differences exercise the is_zero inverse path)."""
    import halo2_svd041_amd as hs
    rs = np.random.RandomState(11)
    N, M = 6, 5
    m = rs.standard_normal((N, M)) * 50
    u = rs.standard_normal((N, N))
    v = rs.standard_normal((M, M))
    d = np.abs(rs.standard_normal(min(N, M)))
    m[0, 0] = -0.0
    m[0, 1] = 0.5 / 2 ** 32          # exact tie at P=32
    m[0, 2] = -1.5 / 2 ** 32
    u[1, 1] = 1.0
    u[1, 2] = -1.0
    v[2, 2] = 3e5
    d[0] = 1e9
    for P in (32, 63):
        ctx = gpu_ctx_factory(P)
        g = gamma_for(99)
        hs.svd_witness(ctx, m, u, v, d, g)
        a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
        _assert_streams(ctx, a0, l0, a1)


@pytest.mark.parametrize("crt", [1, 0])
def test_generic_gemm_fallback_parity(gpu_ctx_factory, crt):
    """Operands too wide for the digit GEMM (|x| >= 2^72): the CRT GEMM takes them
    (up to 2^128), the digit path falls back to the Montgomery GEMM."""
    import halo2_svd041_amd as hs
    rs = np.random.RandomState(3)
    N = 5
    m = rs.uniform(-1, 1, (N, N)) * 2.0 ** 20
    m[0, 0] = 3.0e19                       # saturates to 2^128 - 1 at P = 63
    u, d, v = np.eye(N), np.ones(N), np.eye(N)
    ctx = gpu_ctx_factory(63)
    ctx.set_option("gemm_crt", crt)
    hs.svd_witness(ctx, m, u, v, d, 5)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, 63, 19, 5)
    _assert_streams(ctx, a0, l0, a1)


def test_modular_api_matches_whole_witness(gpu_ctx_factory):
    """ZkMatrix::new + check_svd_phase0/1 through the modular ABI == svd_witness."""
    import halo2_svd041_amd as hs
    N, M, P = 10, 13, 42
    m, u, d, v = gen_svd_input(N, M, seed=17)
    g = gamma_for(17)
    ctx = gpu_ctx_factory(P)
    zm = hs.ZkMatrix.new(ctx, m)
    zu = hs.ZkMatrix.new(ctx, u)
    zv = hs.ZkMatrix.new(ctx, v)
    zd = hs.ZkVector.new(ctx, d)
    es, eu = hs.err_calc(P, max(N, M), 100.0, 1e-10, 1e-10)
    pl = hs.check_svd_phase0(ctx, zm, zu, zv, zd, es, eu, 30)
    hs.check_svd_phase1(ctx, zm, zu, zv, pl, g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)
    whole = gpu_ctx_factory(P)                   # the device checker sees the same witness
    hs.svd_witness(whole, m, u, v, d, g)
    r, rw = ctx.check_gates(), whole.check_gates()
    assert r == rw and r["gate_failures"] + r["copy_failures"] + r["lookup_failures"] == 0, (r, rw)


@pytest.mark.parametrize("impl", ["mfma", "valu"])
@pytest.mark.parametrize("N,M,P", [(33, 47, 63), (64, 64, 32), (70, 65, 42), (96, 96, 63)])
def test_gemm_impls_parity(gpu_ctx_factory, impl, N, M, P):
    """Both exact GEMM paths (matrix cores / v_dot4) give the oracle's c_s cells."""
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N + 3 * M)
    g = gamma_for(N * 7)
    ctx = gpu_ctx_factory(P)
    ctx.set_gemm_impl(impl)
    hs.svd_witness(ctx, m, u, v, d, g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)


def test_honest_prover_mat_mul_k_beyond_chunks(gpu_ctx_factory):
    """Modular GEMM with K not a multiple of 64 / 32 and non-square shapes."""
    import halo2_svd041_amd as hs
    import pyoracle as po
    rs = np.random.RandomState(8)
    A = rs.uniform(-3, 3, (37, 131))
    B = rs.uniform(-3, 3, (131, 29))
    for impl in ("mfma", "valu"):
        ctx = gpu_ctx_factory(40)
        ctx.set_gemm_impl(impl)
        za, zb = hs.ZkMatrix.new(ctx, A), hs.ZkMatrix.new(ctx, B)
        c = hs.honest_prover_mat_mul(ctx, za, zb)
        got = c.values()
        qa = [[po.quantize(x, 40) for x in r] for r in A.tolist()]
        qb = [[po.quantize(x, 40) for x in r] for r in B.tolist()]
        for i in (0, 17, 36):
            for j in (0, 11, 28):
                want = sum(qa[i][k] * qb[k][j] for k in range(131)) % po.P_MOD
                assert int(got[i, j, 0]) | (int(got[i, j, 1]) << 64) | (int(got[i, j, 2]) << 128) \
                    | (int(got[i, j, 3]) << 192) == want


@pytest.mark.parametrize("kern,N,K,M", [(-1, 300, 700, 260), (2, 300, 700, 260), (-1, 2048, 1024, 1100),
                                         (1, 2048, 1024, 1100)])
def test_honest_prover_mat_mul_persistent(gpu_ctx_factory, kern, N, K, M):
    """svdw_honest_prover_mat_mul queued on its own: gemm_kern -1 runs the
    persistent CRT GEMM below 64 tile pairs of 256 x 128 (300 x 700 x 260: K =
    700 gives 12 chunks of 64, several units per block, the chunk pipeline
    crossing unit boundaries) and the wide-tile kernel from there on (2048 x
    1024 x 1100: 72 pairs, a partial last tile column); gemm_kern 2 forces the
    wide kernel on 3 tile rows (a pair whose second tile is past the end). Sampled
    entries against exact integer sums of the quantized operands, and the whole
    product against the per-unit kernel's (gemm_kern 0)."""
    import halo2_svd041_amd as hs
    import pyoracle as po
    rs = np.random.RandomState(9)
    A = rs.uniform(-3, 3, (N, K))
    B = rs.uniform(-3, 3, (K, M))
    outs = []
    for k in (kern, 0):
        ctx = gpu_ctx_factory(63)
        ctx.set_option("gemm_kern", k)
        za, zb = hs.ZkMatrix.new(ctx, A), hs.ZkMatrix.new(ctx, B)
        outs.append(hs.honest_prover_mat_mul(ctx, za, zb).values())
        ctx.close()
    assert np.array_equal(outs[0], outs[1])
    got = outs[0]
    rows, cols = (0, 129, N - 1), (0, 128, M - 1)
    qa = {i: [po.quantize(x, 63) for x in A[i].tolist()] for i in rows}
    qb = {j: [po.quantize(x, 63) for x in B[:, j].tolist()] for j in cols}
    for i in rows:
        for j in cols:
            want = sum(x * y for x, y in zip(qa[i], qb[j])) % po.P_MOD
            assert int(got[i, j, 0]) | (int(got[i, j, 1]) << 64) | (int(got[i, j, 2]) << 128) \
                | (int(got[i, j, 3]) << 192) == want


@pytest.mark.parametrize("N,M,P,world,device", [(260, 270, 32, 1, True), (257, 255, 63, 1, False),
                                                (300, 200, 32, 3, True), (513, 40, 32, 1, True)])
def test_crt_gemm_tiles_parity(gpu_ctx_factory, N, M, P, world, device):
    """The CRT GEMM's 128 x 128 output tiles across tile edges: shapes one past /
    one short of 256, a row-sharded rank whose row block is not a tile multiple,
    a tall product with a single column tile; device inputs (the batched f64
    residue path) and host inputs (one product per launch); every cell against
    the oracle."""
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N + M + 7)
    g = gamma_for(N + 7)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    ctxs = []
    counts = None
    for rank in range(world):
        ctx = gpu_ctx_factory(P)
        if world > 1:
            ctx.set_shard(rank, world)
        counts = hs.svd_witness(ctx, *(_on_device(m, u, v, d) if device else (m, u, v, d)), g)
        ctxs.append(ctx)
    if world == 1:
        _assert_streams(ctxs[0], a0, l0, a1)
        return
    got = _reassemble(ctxs, counts)
    for key, want in (((0, 0), a0), ((1, 0), a1), ((0, 1), l0)):
        bad = np.nonzero(np.any(got[key] != want, axis=1))[0]
        assert bad.size == 0, f"{key}: {bad.size} cells differ, first at {bad[:8]}"


@pytest.mark.parametrize("opts", [{"gemm_crt": 0}, {"stage_elems": 64}, {"stage_elems": 192},
                                  {"phase1_overlap": 0}, {"phase1_overlap": 2},
                                  {"overlap": 0},
                                  {"stage_batch": 0}, {"pipeline": 0}, {"pipeline": 0, "phase1_overlap": 2},
                                  {"gemm_impl": 1}, {"res_f64": 0}, {"f64_views": 0},
                                  {"gemm_kern": 0}, {"gemm_kern": 1}, {"gemm_kern": 2}, {"res_wait": 0},
                                  {"res_wait": 1}, {"stage_rot": 0}, {"stage_rot": 0, "pipeline": 0}])
def test_tuning_options_parity(gpu_ctx_factory, opts):
    """Every tuning knob of svdw_set_option leaves the witness bit-identical."""
    import halo2_svd041_amd as hs
    N, M, P = 45, 37, 63
    m, u, d, v = gen_svd_input(N, M, seed=4)
    g = gamma_for(4)
    ctx = gpu_ctx_factory(P)
    for k, val in opts.items():
        ctx.set_option(k, val)
    hs.svd_witness(ctx, m, u, v, d, g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)


def test_modular_verify_mul_parity(gpu_ctx_factory):
    """ZkMatrix::verify_mul through the ABI, twice (honest and wrong c_s), vs the
    Python restatement of src/matrix/mod.rs:299-342 on the same quantized cells."""
    import halo2_svd041_amd as hs
    import pyoracle as po
    rs = np.random.RandomState(21)
    P = 42
    A = rs.uniform(-3, 3, (5, 7))
    B = rs.uniform(-3, 3, (7, 4))
    W = rs.uniform(-50, 50, (5, 4))
    g = gamma_for(21)
    ctx = gpu_ctx_factory(P)
    za, zb, zw = hs.ZkMatrix.new(ctx, A), hs.ZkMatrix.new(ctx, B), hs.ZkMatrix.new(ctx, W)
    cs = hs.honest_prover_mat_mul(ctx, za, zb)
    hs.ZkMatrix.verify_mul(ctx, za, zb, cs, g)
    hs.ZkMatrix.verify_mul(ctx, za, zb, zw, g)
    o0, o1, orlc = po.Context(phase=0), po.Context(phase=1), po.Context(phase=1)
    oa, ob, ow = (po.zkmatrix_new(o0, P, x.tolist()) for x in (A, B, W))
    ocs = po.honest_prover_mat_mul(o0, oa, ob)
    gam = po.load_witness(orlc, g)
    po.verify_mul(o1, oa, ob, ocs, gam)
    po.verify_mul(o1, oa, ob, ow, gam)
    def ints(cells):
        return [int(r[0]) | int(r[1]) << 64 | int(r[2]) << 128 | int(r[3]) << 192 for r in cells]
    assert ints(ctx.advice(0)) == o0.advice
    assert ints(ctx.advice(1)) == o1.advice


def _reassemble(ctxs, counts):
    """Global streams from the ranks' owned segments (each cell exactly once)."""
    out = {(0, 0): np.zeros((counts["advice0"], 4), np.uint64),
           (1, 0): np.zeros((counts["advice1"], 4), np.uint64),
           (0, 1): np.zeros((counts["lookup0"], 4), np.uint64),
           (1, 1): np.zeros((counts["lookup1"], 4), np.uint64)}
    seen = {k: np.zeros(v.shape[0], np.int32) for k, v in out.items()}
    for ctx in ctxs:
        streams = {(0, 0): ctx.advice(0), (1, 0): ctx.advice(1),
                   (0, 1): ctx.lookups(0), (1, 1): ctx.lookups(1)}
        for phase, lookup, off, n in ctx.shard_segments():
            out[(phase, lookup)][off:off + n] = streams[(phase, lookup)][off:off + n]
            seen[(phase, lookup)][off:off + n] += 1
    for k, s in seen.items():
        assert np.all(s == 1), k
    return out


@pytest.mark.parametrize("N,M,P,world,crt", [(40, 33, 63, 2, 1), (33, 40, 32, 3, 1), (24, 24, 42, 5, 1),
                                              (40, 33, 63, 2, 0), (70, 70, 63, 8, 1)])
def test_row_sharded_witness_parity(gpu_ctx_factory, N, M, P, world, crt):
    """Row-block sharding (BASELINE config 4 layout): the union of the ranks'
    owned cells is the oracle's witness, bit for bit (CRT products, with v's
    residue planes reused by v.v^T on each rank; and the digit-plane GEMM)."""
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N * M + world)
    g = gamma_for(world)
    ctxs = []
    for rank in range(world):
        ctx = gpu_ctx_factory(P)
        ctx.set_option("gemm_crt", crt)
        ctx.set_shard(rank, world)
        counts = hs.svd_witness(ctx, m, u, v, d, g)
        ctxs.append(ctx)
    got = _reassemble(ctxs, counts)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    for key, want in (((0, 0), a0), ((1, 0), a1), ((0, 1), l0)):
        bad = np.nonzero(np.any(got[key] != want, axis=1))[0]
        assert bad.size == 0, f"{key}: {bad.size} cells differ, first at {bad[:8]}"


def test_row_sharded_matches_unsharded_256(gpu_ctx_factory):
    """BASELINE config 2/4 shape class at 256^2, P=63, 4 row blocks: sharded union ==
    the single-context witness (itself oracle-checked at the smaller sizes)."""
    import halo2_svd041_amd as hs
    N, P, world = 256, 63, 4
    m, u, d, v = gen_svd_input(N, N, seed=256)
    g = gamma_for(256)
    full = gpu_ctx_factory(P)
    counts = hs.svd_witness(full, m, u, v, d, g)
    ctxs = []
    for rank in range(world):
        ctx = gpu_ctx_factory(P)
        ctx.set_shard(rank, world)
        hs.svd_witness(ctx, m, u, v, d, g)
        ctxs.append(ctx)
    got = _reassemble(ctxs, counts)
    assert np.array_equal(got[(0, 0)], full.advice(0))
    assert np.array_equal(got[(1, 0)], full.advice(1))
    assert np.array_equal(got[(0, 1)], full.lookups(0))


def _ints(cells):
    return [int(r[0]) | int(r[1]) << 64 | int(r[2]) << 128 | int(r[3]) << 192 for r in cells]


@pytest.mark.parametrize("P,LB,S,NB,elems", [(32, 12, 0, 0, 256), (32, 19, 0, 0, 256), (63, 19, 0, 0, 256),
                                            (42, 16, 100, 110, 256), (40, 19, 120, 0, 256),
                                            (32, 12, 0, 0, 64), (63, 19, 0, 0, 128), (63, 12, 0, 0, 64),
                                            (32, 12, 96, 97, 64)])
def test_rescale_and_inner_product_parity(gpu_ctx_factory, P, LB, S, NB, elems):
    """rescale_matrix / ZkVector::inner_product / ZkVector::mul through the ABI vs
    the oracle's parameterised signed_div_scale (chip layout parity unpinned:
    both sides follow include/svdw.h's svdw_div_scale construction); advice and
    lookup streams must match cell for cell, the oracle's constraint checker
    must pass, and the quotients must be floor(c / 2^P)."""
    import halo2_svd041_amd as hs
    import pyoracle as po
    rs = np.random.RandomState(P + LB)
    A = rs.uniform(-9, 9, (6, 11))
    B = rs.uniform(-9, 9, (11, 7))
    x = rs.uniform(-50, 50, 11)
    ctx = gpu_ctx_factory(P, LB)
    ctx.set_option("stage_elems", elems)
    za, zb, zx = hs.ZkMatrix.new(ctx, A), hs.ZkMatrix.new(ctx, B), hs.ZkVector.new(ctx, x)
    cs = hs.honest_prover_mat_mul(ctx, za, zb)
    c = hs.ZkMatrix.rescale_matrix(ctx, cs, S, NB)
    ip = zx.inner_product(zx, 0, S, NB)
    y = zx.mul(za, 0, S, NB)
    o = po.Context(phase=0)
    rc = po.RangeChip(LB)
    oa, ob = po.zkmatrix_new(o, P, A.tolist()), po.zkmatrix_new(o, P, B.tolist())
    ox = po.zkvector_new(o, P, x.tolist())
    ocs = po.honest_prover_mat_mul(o, oa, ob)
    oc = po.rescale_matrix(o, rc, ocs, P, S, NB)
    oip = po.zkvector_inner_product(o, rc, ox, ox, P, S, NB)
    oy = po.zkvector_mul(o, rc, ox, oa, P, S, NB)
    assert po.check_constraints(o, LB) == []
    assert _ints(ctx.advice(0)) == o.advice
    assert _ints(ctx.lookups(0)) == o.lookups
    got = np.array(_ints(c.values().reshape(-1, 4))).reshape(6, 7)
    assert [[int(v) for v in r] for r in got] == [[e.value for e in r] for r in oc]
    for i in range(6):
        for j in range(7):
            assert po.to_signed(oc[i][j].value) == po.to_signed(ocs[i][j].value) >> P
    assert _ints(ip.values()) == [oip.value]
    assert _ints(y.values()) == [e.value for e in oy]


def _on_device(*xs):
    import torch
    dev = torch.device("cuda", 0)
    return [torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in xs]


@pytest.mark.parametrize("f64v", [1, 0])
@pytest.mark.parametrize("res", [1, 0])
@pytest.mark.parametrize("pipe", [1, 0])
@pytest.mark.parametrize("N,M,P", [(130, 97, 63), (64, 200, 32)])
def test_device_inputs_parity(gpu_ctx_factory, pipe, res, f64v, N, M, P):
    """The bench path: m, u, v, d already resident in HBM (torch float64 CUDA
    tensors), quantized in one fused launch; the CRT residue planes of
    m, u, v built from the f64 inputs in one launch (res 1) or from the
    quantized cells (res 0); the stages and row scans reading the loaded
    matrices through f64 views (f64v 1: quantized in registers, no wait for the
    cells) or the cells; pipelined (pipe) or not; witness vs the oracle."""
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N * M)
    g = gamma_for(N + M)
    ctx = gpu_ctx_factory(P)
    ctx.set_option("pipeline", pipe)
    ctx.set_option("res_f64", res)
    ctx.set_option("f64_views", f64v)
    dm, du, dv, dd = _on_device(m, u, v, d)
    hs.svd_witness(ctx, dm, du, dv, dd, g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)


@pytest.mark.parametrize("P", [32, 63])
def test_device_garbage_inputs_parity(gpu_ctx_factory, P):
    """Quantization edges through the f64 residue planes (device inputs): -0.0,
    ties, saturation to 2^128 - 1, +-inf, NaN, in the GEMM operands m, u, v."""
    import halo2_svd041_amd as hs
    rs = np.random.RandomState(12)
    N, M = 7, 6
    m = rs.standard_normal((N, M)) * 50
    u = rs.standard_normal((N, N))
    v = rs.standard_normal((M, M))
    d = np.abs(rs.standard_normal(min(N, M)))
    m[0, 0] = -0.0
    m[0, 1] = 0.5 / 2 ** 32
    m[0, 2] = -1.5 / 2 ** 32
    m[1, 0] = 3.0e19 if P == 63 else 1e30     # saturates to 2^128 - 1
    m[1, 1] = -np.inf
    m[1, 2] = np.nan
    u[2, 3] = np.inf
    v[3, 1] = -2.5 / 2 ** P
    g = gamma_for(98)
    ctx = gpu_ctx_factory(P)
    hs.svd_witness(ctx, *_on_device(m, u, v, d), g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)


@pytest.mark.parametrize("N,M,P,world", [(40, 33, 63, 2), (33, 40, 32, 3), (70, 70, 63, 8),
                                         (130, 97, 63, 3), (97, 130, 42, 5)])
def test_row_sharded_device_inputs_parity(gpu_ctx_factory, N, M, P, world):
    """Row-sharded ranks with device-resident inputs (the config-4 bench path):
    each rank's A operand planes are a row slice of the full f64 residue planes
    (u, v) or its own rows of m; the union of the owned cells is the oracle's
    witness."""
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N * M + 7 * world)
    g = gamma_for(world + 40)
    dm, du, dv, dd = _on_device(m, u, v, d)
    ctxs = []
    for rank in range(world):
        ctx = gpu_ctx_factory(P)
        ctx.set_shard(rank, world)
        counts = hs.svd_witness(ctx, dm, du, dv, dd, g)
        ctxs.append(ctx)
    got = _reassemble(ctxs, counts)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    for key, want in (((0, 0), a0), ((1, 0), a1), ((0, 1), l0)):
        bad = np.nonzero(np.any(got[key] != want, axis=1))[0]
        assert bad.size == 0, f"{key}: {bad.size} cells differ, first at {bad[:8]}"


@pytest.mark.parametrize("world,opts", [(1, {"prod_cell": 1}), (1, {"prod_cell": 1, "stage_batch": 0}),
                                        (1, {"prod_cell": 1, "p1_at": 1}), (1, {"prod_cell": 1, "hold_us": 50}),
                                        (3, {"prod_cell": 0}), (3, {"prod_cell": 1, "stage_batch": 0}),
                                        (4, {"prod_cell": 1, "pipeline": 0}), (1, {"pipeline": 0}),
                                        (5, {"prod_cell": 0}), (4, {"p1_at": 3}), (1, {"prod_cell": 0})])
def test_products_on_cell_stream_parity(gpu_ctx_factory, world, opts):
    """prod_cell: the products on the cell stream, the u / v bounds and u.d on
    st2 beside them (default on row-sharded ranks), with device inputs (the
    only path it applies to): bit-identical to the oracle, sharded or not."""
    import halo2_svd041_amd as hs
    N, M, P = 70, 53, 63
    m, u, d, v = gen_svd_input(N, M, seed=world + 90)
    g = gamma_for(world + 90)
    dm, du, dv, dd = _on_device(m, u, v, d)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    ctxs = []
    for rank in range(world):
        ctx = gpu_ctx_factory(P)
        if world > 1:
            ctx.set_shard(rank, world)
        for k, val in opts.items():
            ctx.set_option(k, val)
        counts = hs.svd_witness(ctx, dm, du, dv, dd, g)
        ctxs.append(ctx)
    if world == 1:
        _assert_streams(ctxs[0], a0, l0, a1)
        return
    got = _reassemble(ctxs, counts)
    for key, want in (((0, 0), a0), ((1, 0), a1), ((0, 1), l0)):
        bad = np.nonzero(np.any(got[key] != want, axis=1))[0]
        assert bad.size == 0, f"{key}: {bad.size} cells differ, first at {bad[:8]}"


@pytest.mark.parametrize("N,M,P,world,hold,opts", [
    (70, 53, 63, 1, 0, {}), (53, 70, 32, 1, 200, {}), (130, 97, 63, 4, 0, {}), (40, 33, 63, 1, 0, {}),
    (70, 53, 63, 1, 200, {"dchk_at": 1}), (53, 70, 32, 1, 200, {"dchk_at": 2, "gamma_at": 1}),
    (130, 97, 63, 4, 200, {"dchk_at": 2, "gamma_at": 1}), (97, 130, 63, 4, 0, {"dchk_at": 1, "gamma_at": 1})])
def test_pipelined_witnesses_parity(gpu_ctx_factory, N, M, P, world, hold, opts):
    """pipeline: consecutive svd_witness calls on one context overlap (a call
    returns with its stages and row scans still running; the next call's
    quantization and products start beside them, into the other cell set).
    Four calls of different inputs (and, between the second and third, a
    change of shape) queued back to back without a host wait; the last
    witness vs the oracle, then a non-pipelined call (check_svd_phase0 through
    the modular API would append cells: a verify_mul_witness) and a further
    pipelined witness, each vs the oracle. hold: every call's streams wait
    behind a spinning kernel, so a missing cross-call dependency shows. opts:
    the pipelined schedule's stream placements (dchk_at, gamma_at)."""
    import halo2_svd041_amd as hs
    ctx = gpu_ctx_factory(P)
    for k, val in opts.items():
        ctx.set_option(k, val)
    if world > 1:
        ctx.set_shard(world - 1, world)
    if hold:
        ctx.set_option("hold_us", hold)
    ins = []
    for k in range(4):
        n, m_ = (N, M) if k != 2 else (M, N)
        m, u, d, v = gen_svd_input(n, m_, seed=400 + 13 * k + N)
        ins.append((m, u, d, v, gamma_for(500 + k)))
    devs = [_on_device(m, u, v, d) for m, u, d, v, _ in ins]
    for (m, u, d, v, g), dv in zip(ins, devs):
        counts = hs.svd_witness(ctx, *dv, g)

    def check(m, u, d, v, g, counts):
        a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
        if world == 1:
            _assert_streams(ctx, a0, l0, a1)
            return
        streams = {(0, 0): ctx.advice(0), (1, 0): ctx.advice(1), (0, 1): ctx.lookups(0)}
        for phase, lookup, off, n in ctx.shard_segments():
            if (phase, lookup) not in streams:
                continue
            want = {(0, 0): a0, (1, 0): a1, (0, 1): l0}[(phase, lookup)]
            got = streams[(phase, lookup)]
            bad = np.nonzero(np.any(got[off:off + n] != want[off:off + n], axis=1))[0]
            assert bad.size == 0, f"{(phase, lookup)}: {bad.size} owned cells differ from {off}"

    check(*ins[3], counts)
    if world == 1:
        a = np.random.RandomState(3).standard_normal((9, 7))
        b = np.random.RandomState(4).standard_normal((7, 5))
        gv = gamma_for(77)
        hs.verify_mul_witness(ctx, *_on_device(a, b), gv)
        w0, w1 = corc.verify_mul_witness(a, b, P, gv)
        np.testing.assert_array_equal(ctx.advice(0, 0, w0.shape[0]), w0)
        np.testing.assert_array_equal(ctx.advice(1, 0, w1.shape[0]), w1)
    ctx.reset()
    counts = hs.svd_witness(ctx, *devs[1], ins[1][4])
    check(*ins[1], counts)


@pytest.mark.parametrize("N,M,P,row_lim,device,hold", [(1024, 1024, 63, 64, False, 0), (512, 512, 32, 128, False, 0),
                                                       (2048, 1024, 32, 24, False, 0), (1024, 1024, 63, 32, True, 0),
                                                       (2048, 1024, 32, 16, True, 0),
                                                       (1024, 1024, 63, 32, True, 3000),
                                                       (1024, 1024, 63, 32, True, -3000)])
def test_full_size_sampled_parity(gpu_ctx_factory, N, M, P, row_lim, device, hold):
    """BASELINE config sizes (1024^2 P=63 = the bench workload, 512^2 P=32,
    2048x1024 P=32): the GPU computes the whole witness; the C oracle computes
    the first row_lim rows of every row-parallel region and all other regions
    in full. Walking the engine's layout table (svdw_layout), every cell the
    oracle computed must equal the GPU's cell at its full-witness offset: the
    loads, d checks and gamma powers entirely, the first row_lim rows of every
    bound / product / diff / scan / is_equal region. hold: every stream of the
    witness waits behind a spinning kernel until the host has queued all of it,
    so a launch missing a cross-stream dependency runs ahead (the c_s scans
    beside products on another stream) and reads unwritten cells."""
    import halo2_svd041_amd as hs
    from conftest import walk_window
    m, u, d, v = gen_svd_input(N, M, seed=N + M + P)
    g = gamma_for(N * M)
    ctx = gpu_ctx_factory(P)
    if hold < 0:                                  # (and not pipelined)
        ctx.set_option("pipeline", 0)
        hold = -hold
    if hold:
        # a first witness of other inputs allocates every buffer (allocation
        # synchronises), so the witness below runs fully queued behind the hold;
        # a launch that ran ahead would read the first witness's cells
        # (twice: a pipelined context alternates between two cell sets)
        m2, u2, d2, v2 = gen_svd_input(N, M, seed=N + M + P + 1)
        for k in range(2):
            hs.svd_witness(ctx, *_on_device(m2, u2, v2, d2), gamma_for(N * M + 1 + k))
        ctx.sync()
        ctx.reset()
        ctx.set_option("hold_us", hold)
    if device:                                    # the bench path (inputs resident in HBM)
        hs.svd_witness(ctx, *_on_device(m, u, v, d), g)
    else:
        hs.svd_witness(ctx, m, u, v, d, g)
    ctx.sync()
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g, row_lim=row_lim)
    get = lambda ph, lk, off, n: (ctx.lookups if lk else ctx.advice)(ph, off, n)   # noqa: E731
    assert walk_window(ctx.layout(), get, {(0, 0): a0, (0, 1): l0, (1, 0): a1}, 0, row_lim) > 0


@pytest.mark.parametrize("shapes,P,row_begin,row_lim,hold", [
    (((1024, 1024),) * 3, 63, 500, 24, 0),
    (((1024, 1024),) * 3, 63, 1000, 24, 3000),
    (((512, 512), (512, 512), (2048, 1024)), 32, 300, 16, 0),
])
def test_pipelined_full_size_parity(gpu_ctx_factory, shapes, P, row_begin, row_lim, hold):
    """The bench's own regime at full size: device-input svd_witness calls
    queued back to back with no host wait, each with its own inputs and gamma
    (call j + 1's quantization, residues, GEMM and combine run beside call j's
    stage kernels and row scans, and call j + 2 reuses call j's cell set behind
    its tail events). The last witness is then walked against the C oracle in a
    row window away from the top rows: every load, d check and gamma power,
    and rows [row_begin, row_begin + row_lim) of every row-parallel region.
    hold: every call's streams also wait behind a spinning kernel, so each
    call's launches sit fully queued before any of them runs. The third case
    changes the shape inside the pipeline (two 512^2 then 2048 x 1024)."""
    import halo2_svd041_amd as hs
    from conftest import walk_window
    ctx = gpu_ctx_factory(P)
    if hold:
        ctx.set_option("hold_us", hold)
    ins = []
    for k, (N, M) in enumerate(shapes):
        m, u, d, v = gen_svd_input(N, M, seed=7000 + 31 * k + N + P)
        ins.append((m, u, d, v, gamma_for(7100 + k)))
    devs = [_on_device(m, u, v, d) for m, u, d, v, _ in ins]
    for (m, u, d, v, g), dv in zip(ins, devs):
        hs.svd_witness(ctx, *dv, g)                   # no host wait in between
    ctx.sync()
    m, u, d, v, g = ins[-1]
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g, row_lim=row_lim, row_begin=row_begin)
    get = lambda ph, lk, off, n: (ctx.lookups if lk else ctx.advice)(ph, off, n)   # noqa: E731
    assert walk_window(ctx.layout(), get, {(0, 0): a0, (0, 1): l0, (1, 0): a1}, row_begin, row_lim) > 0


def test_device_input_lifetime(gpu_ctx_factory):
    """Device inputs passed as temporaries (include/svdw.h, "Lifetime of device
    inputs"): the call returns while its kernels are still held behind a
    spinning kernel, the caller drops the tensors, and torch immediately
    allocates tensors of the same sizes and fills them with other values on its
    own stream (which does not wait for the engine). The Python layer keeps the
    inputs referenced until the work is done, so torch cannot hand out their
    memory: the witness still equals the oracle's for the original inputs."""
    import torch
    import halo2_svd041_amd as hs
    N, M, P = 192, 160, 63
    ctx = gpu_ctx_factory(P)
    m2, u2, d2, v2 = gen_svd_input(N, M, seed=91)
    for k in range(2):                                # every buffer allocated (both cell sets)
        hs.svd_witness(ctx, *_on_device(m2, u2, v2, d2), gamma_for(92 + k))
    ctx.sync()
    ctx.reset()
    ctx.set_option("hold_us", 20000)
    m, u, d, v = gen_svd_input(N, M, seed=93)
    g = gamma_for(94)
    hs.svd_witness(ctx, *_on_device(m, u, v, d), g)   # the tensors are temporaries
    dev = torch.device("cuda", 0)
    junk = [torch.full(x.shape, -1.0e30, dtype=torch.float64, device=dev) for x in (m, u, v, d)]
    assert not ctx.query()                            # the witness is still held
    ctx.sync()
    del junk
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)


@pytest.mark.parametrize("N,M", [(320, 300), (300, 520)])
def test_gemm_kern_full_streams(gpu_ctx_factory, N, M):
    """The persistent CRT GEMM (gemm_kern 1) and gemm_kern 2 (the batch holds
    the symmetric u.u^T and v.v^T, so it falls back to 1 as a whole; the wide
    kernel runs inside a witness on row-sharded ranks, test_full_size_shard_rank_parity)
    against the per-unit one (0,
    oracle-checked throughout this file) on pipelined device-input witnesses at
    K >= 300 (>= 8 chunks of 64: the persistent grid runs, its chunk pipeline
    crossing unit boundaries; 300 x 520 mixes kpads, where it falls back to
    the per-unit kernel): whole advice and lookup streams of both phases, two
    calls in a row."""
    import halo2_svd041_amd as hs
    P = 63
    outs = []
    for k in (0, 1, 2):
        ctx = gpu_ctx_factory(P)
        ctx.set_option("gemm_kern", k)
        for c in range(2):
            m, u, d, v = gen_svd_input(N, M, seed=4100 + c + N)
            hs.svd_witness(ctx, *_on_device(m, u, v, d), gamma_for(4200 + c))
        ctx.sync()
        outs.append((ctx.advice(0), ctx.lookups(0), ctx.advice(1)))
        ctx.close()
    for k, out in zip((1, 2), outs[1:]):
        for name, a, b in zip(("advice0", "lookup0", "advice1"), outs[0], out):
            assert a.shape == b.shape
            bad = np.nonzero(np.any(a != b, axis=1))[0]
            assert bad.size == 0, f"gemm_kern {k} {name}: {bad.size} cells differ, first at {bad[:8]}"


def test_place_trials_full_streams(gpu_ctx_factory):
    """place_trials 3 (6 by default): each cell stream of >= 256 MiB is chosen among three
    placements by timing the stage store pattern on each (the probe writes
    constant cells over the candidates). 1024^2 P=32 pipelined device-input
    witnesses, two calls (both cell sets), against a context without trials (0):
    whole advice and lookup streams of both phases."""
    import halo2_svd041_amd as hs
    N = M = 1024
    P = 32
    outs = []
    for k in (0, 3):
        ctx = gpu_ctx_factory(P)
        ctx.set_option("place_trials", k)
        for c in range(2):
            m, u, d, v = gen_svd_input(N, M, seed=4300 + c)
            hs.svd_witness(ctx, *_on_device(m, u, v, d), gamma_for(4400 + c))
        ctx.sync()
        outs.append((ctx.advice(0), ctx.lookups(0), ctx.advice(1)))
        ctx.close()
    for name, a, b in zip(("advice0", "lookup0", "advice1"), outs[0], outs[1]):
        assert a.shape == b.shape
        bad = np.nonzero(np.any(a != b, axis=1))[0]
        assert bad.size == 0, f"{name}: {bad.size} cells differ, first at {bad[:8]}"


def test_completion_marks(gpu_ctx_factory):
    """svdw_mark behind a held witness (hold_us: a spinning kernel at the head
    of the step) reads not-done until the work completes; svdw_mark_wait waits
    for it; 20 further marks reuse every slot of the 16-entry ring, and the
    oldest ticket is then answered by the mark that took its slot."""
    import ctypes as ct
    import halo2_svd041_amd as hs
    from halo2_svd041_amd import _lib
    L = _lib.lib()
    N, M, P = 64, 48, 63
    ctx = gpu_ctx_factory(P)
    m, u, d, v = gen_svd_input(N, M, seed=71)
    for k in range(2):
        hs.svd_witness(ctx, *_on_device(m, u, v, d), gamma_for(72 + k))
    ctx.sync()
    ctx.set_option("hold_us", 20000)
    hs.svd_witness(ctx, *_on_device(m, u, v, d), gamma_for(74))
    t = ct.c_uint64(0)
    assert L.svdw_mark(ctx.handle, ct.byref(t)) == 0
    first = t.value
    assert L.svdw_mark_done(ctx.handle, first) == 0
    assert L.svdw_mark_wait(ctx.handle, first) == 0
    assert L.svdw_mark_done(ctx.handle, first) == 1
    assert ctx.query()
    ctx.set_option("hold_us", 0)
    for _ in range(20):
        assert L.svdw_mark(ctx.handle, ct.byref(t)) == 0
    ctx.sync()
    assert L.svdw_mark_done(ctx.handle, first) == 1 and L.svdw_mark_done(ctx.handle, t.value) == 1


def test_held_inputs_bounded(gpu_ctx_factory):
    """back-to-back pipelined witnesses on fresh device tensors with
    no sync and no readback. The Python layer releases each call's inputs once a
    completion mark (svdw_mark) after that call has completed, so the held set stays bounded
    (HOLD_EVERY * (HOLD_CKPTS + 1) calls at most) instead of growing until the
    device is out of memory; the last witness still equals the oracle's."""
    import halo2_svd041_amd as hs
    N, M, P = 96, 80, 63
    ctx = gpu_ctx_factory(P)
    bound = 4 * ctx.HOLD_EVERY * (ctx.HOLD_CKPTS + 1)
    sizes = []
    for k in range(60):
        m, u, d, v = gen_svd_input(N, M, seed=1200 + k)
        g = gamma_for(1300 + k)
        hs.svd_witness(ctx, *_on_device(m, u, v, d), g)
        sizes.append(len(ctx._held))
        assert sizes[-1] <= bound, sizes
    assert min(sizes[40:]) < max(sizes), sizes         # entries are released while calls run
    ctx.sync()
    assert not ctx._held
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    _assert_streams(ctx, a0, l0, a1)


@pytest.mark.parametrize("rank,opts", [(0, {}), (3, {}), (7, {}),
                                       (3, {"overlap": 0, "phase1_overlap": 0}),
                                       (5, {"dchk_at": 2, "gamma_at": 1}), (6, {"dchk_at": 1}),
                                       (2, {"gemm_kern": 2})])
def test_full_size_shard_rank_parity(gpu_ctx_factory, rank, opts):
    """BASELINE config 4 (1024^2, P=63, row blocks over 8 GPUs), rank by rank at
    full size, cell for cell: the rank's witness on the GPU (svdw_set_shard, the
    bench's device-input path) against the C oracle's row window inside that
    rank's rows ([128 rank + 40, +16) of every row-parallel region; every other
    region in full), mapped through the layout table, on the cells the rank
    owns (svdw_shard_segments). Together with the
    owned-segment tiling (tests/test_shard_cpu.py) and the small-shape union
    tests, every rank's cells are value-checked, not just rank 0's."""
    import halo2_svd041_amd as hs
    from conftest import walk_window
    N, P, world, lim = 1024, 63, 8, 16
    m, u, d, v = gen_svd_input(N, N, seed=2 * N + P)
    g = gamma_for(N * N + 8)
    ctx = gpu_ctx_factory(P)
    for k, val in opts.items():
        ctx.set_option(k, val)
    ctx.set_shard(rank, world)
    hs.svd_witness(ctx, *_on_device(m, u, v, d), g)
    ctx.sync()
    rb = N * rank // world + 40
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g, row_lim=lim, row_begin=rb)
    # a row-sharded context writes (at least) the cells it owns: compare those
    owned = {}
    for ph, lk, off, n in ctx.shard_segments():
        owned.setdefault((ph, lk), []).append((off, off + n))
    get = lambda ph, lk, off, n: (ctx.lookups if lk else ctx.advice)(ph, off, n)   # noqa: E731
    want = {(0, 0): a0, (0, 1): l0, (1, 0): a1}
    compared = walk_window(ctx.layout(), get, want, rb, lim, owned)
    # the window's rows of every row-parallel region (all owned) were compared
    assert compared >= 0.9 * (a1.shape[0] - 3 * (1 + 4 * (N - 1))), compared


def _zkvector_inputs(N, M):
    """src/matrix/test_matrix.rs:51-97 (test_zkvector's deterministic inputs, M = 4
    there). Longer vectors repeat the first 8 entries' pattern (i -> i % 8) so
    every product stays inside signed_div_scale's |x| < 2^(3P) domain."""
    A = [[i + (j % 8) / 10.0 for j in range(M)] for i in range(N)]
    k = [i % 8 for i in range(M)]
    v1 = [(i + (i * i + 1) / 10.0) if i % 2 == 0 else (-i + (i * i + 1) / 10.0) for i in k]
    v2 = [((1.0 + i ** 3) / 10.0) * (1 if i % 2 == 0 else -1) for i in k]
    return A, v1, v2


@pytest.mark.parametrize("N,M,P,LB", [(5, 4, 32, 12), (5, 64, 32, 19)])
def test_zkvector_parity(gpu_ctx_factory, N, M, P, LB):
    """BASELINE config 1 (test_zkvector, src/matrix/test_matrix.rs:39-198, with a
    64-entry variant): inner_product, _norm_square, _dist_square, norm, dist and
    mul through the ABI on the reference's inputs; every advice / lookup cell
    equals the oracle's, its constraint checker passes, and the dequantised
    results are within fixed-point error of the f64 values the reference prints
    (norm / dist: qsqrt is the parameterised construction of include/svdw.h,
    parity unpinned -- the chip's source is unavailable)."""
    import halo2_svd041_amd as hs
    import pyoracle as po
    A, v1, v2 = _zkvector_inputs(N, M)
    ctx = gpu_ctx_factory(P, LB)
    za = hs.ZkMatrix.new(ctx, np.array(A))
    z1, z2 = hs.ZkVector.new(ctx, np.array(v1)), hs.ZkVector.new(ctx, np.array(v2))
    ip = z1.inner_product(z2)
    ns1, ns2 = z1._norm_square(), z2._norm_square()
    ds = z1._dist_square(z2)
    u1, u2 = z1.mul(za), z2.mul(za)
    n1, n2, dd = z1.norm(), z2.norm(), z1.dist(z2)
    o = po.Context(phase=0)
    rc = po.RangeChip(LB)
    oa = po.zkmatrix_new(o, P, A)
    o1, o2 = po.zkvector_new(o, P, v1), po.zkvector_new(o, P, v2)
    oip = po.zkvector_inner_product(o, rc, o1, o2, P)
    ons1, ons2 = po.zkvector_norm_square(o, rc, o1, P), po.zkvector_norm_square(o, rc, o2, P)
    ods = po.zkvector_dist_square(o, rc, o1, o2, P)
    ou1, ou2 = po.zkvector_mul(o, rc, o1, oa, P), po.zkvector_mul(o, rc, o2, oa, P)
    on1, on2 = po.zkvector_norm(o, rc, o1, P), po.zkvector_norm(o, rc, o2, P)
    odd = po.zkvector_dist(o, rc, o1, o2, P)
    assert po.check_constraints(o, LB) == []
    assert _ints(ctx.advice(0)) == o.advice
    assert _ints(ctx.lookups(0)) == o.lookups
    deq = lambda x: po.to_signed(x) / 2.0 ** P   # noqa: E731
    for got, want, f64 in ((ip, oip, sum(a * b for a, b in zip(v1, v2))),
                           (ns1, ons1, sum(a * a for a in v1)), (ns2, ons2, sum(b * b for b in v2)),
                           (ds, ods, sum((a - b) ** 2 for a, b in zip(v1, v2))),
                           (n1, on1, sum(a * a for a in v1) ** 0.5), (n2, on2, sum(b * b for b in v2) ** 0.5),
                           (dd, odd, sum((a - b) ** 2 for a, b in zip(v1, v2)) ** 0.5)):
        assert _ints(got.values()) == [want.value]
        assert abs(deq(want.value) - f64) <= 1e-6 * max(1.0, abs(f64))
    for got, want, vec in ((u1, ou1, v1), (u2, ou2, v2)):
        assert _ints(got.values()) == [e.value for e in want]
        for i in range(N):
            f64 = sum(A[i][j] * vec[j] for j in range(M))
            assert abs(deq(want[i].value) - f64) <= 1e-6 * max(1.0, abs(f64))


@pytest.mark.parametrize("N,M,LB,seed", [(5, 5, 12, 0), (5, 5, 19, 1), (64, 48, 19, 2)])
def test_field_mat_times_vec_parity(gpu_ctx_factory, N, M, LB, seed):
    """test_field_mat_times_vec (src/matrix/test_matrix.rs:201-265; P=32, entries
    uniform in (-100, 100), seeded here where the reference uses thread_rng):
    ZkMatrix::new, ZkVector::new, field_mat_vec_mul, then signed_div_scale of
    every entry (as rescale_matrix of the N x 1 result). Every cell equals the
    oracle's, its constraint checker and the device checker pass, and the
    dequantised results are within fixed-point error of the f64 product the
    reference prints."""
    import halo2_svd041_amd as hs
    import pyoracle as po
    from halo2_svd041_amd._lib import Mat
    P = 32
    rs = np.random.RandomState(seed)
    A = rs.uniform(-100.0, 100.0, (N, M))
    v1 = rs.uniform(-100.0, 100.0, M)
    ctx = gpu_ctx_factory(P, LB)
    za, zv = hs.ZkMatrix.new(ctx, A), hs.ZkVector.new(ctx, v1)
    s = hs.field_mat_vec_mul(ctx, za, zv)
    col = hs.ZkMatrix(ctx, Mat(s.vec.phase, s.vec.len, 1, s.vec.off, s.vec.stride, 1))
    q = hs.ZkMatrix.rescale_matrix(ctx, col)
    o = po.Context(phase=0)
    rc = po.RangeChip(LB)
    oa, ov = po.zkmatrix_new(o, P, A.tolist()), po.zkvector_new(o, P, v1.tolist())
    os_ = po.field_mat_vec_mul(o, oa, ov)
    oq = [po.signed_div_scale(o, rc, x, P)[0] for x in os_]
    assert po.check_constraints(o, LB) == []
    assert _ints(ctx.advice(0)) == o.advice
    assert _ints(ctx.lookups(0)) == o.lookups
    got = _ints(q.values().reshape(-1, 4))
    assert got == [x.value for x in oq]
    r = ctx.check_gates()
    assert r["gate_failures"] + r["copy_failures"] + r["lookup_failures"] == 0, r
    f64 = A @ v1
    for i in range(N):
        assert abs(po.to_signed(oq[i].value) / 2.0 ** P - f64[i]) <= 1e-6 * max(1.0, abs(f64[i]))
