"""Copy-constraint (equality) lists of the virtual witness (svdw_equalities,
SURVEY.md §8f rank 2), from the engine's dry planner, against the oracle's
Context.copies / Context.consts (oracle/pyoracle.py assign_region: every
Existing cell against its source, every Constant cell, assert_is_const and
range_check's constrain_equal), record for record in assign order.

Parity: the lists follow halo2-base 0.4.1's QuantumCell semantics as the
oracle restates them (recalled); the engine and the oracle must
agree exactly, including cross-phase sources (phase-1 rows copying phase-0
cells) and verify_mul's init_rand (an RLC-context cell, phase 2 here)."""
import pytest

import halo2_svd041_amd as hs
import pyoracle as po
from conftest import gamma_for, gen_svd_input


def _oracle_lists(w, octx):
    def phase_of(av):
        return 0 if av.ctx is w.ctx0 else (1 if av.ctx is w.ctx1 else 2)
    copies = [(phase_of(a), a.idx, dst) for a, dst in octx.copies]
    consts = [(i, v % po.P_MOD) for i, v in octx.consts]
    return copies, consts


@pytest.mark.parametrize("N,M,P,LB", [(4, 4, 32, 19), (5, 3, 63, 19), (3, 6, 42, 19), (6, 5, 63, 8),
                                      (1, 1, 32, 19), (7, 2, 40, 11), (4, 4, 32, 61), (2, 5, 63, 24)])
def test_svd_equalities_match_oracle(N, M, P, LB):
    m, u, d, v = gen_svd_input(N, M, seed=N * 10 + M + P + LB)
    g = gamma_for(LB)
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=LB)
    hs.svd_witness(ctx, m, u, v, d, g)
    w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), d.tolist(), P, LB, gamma=g)
    for ph, octx in ((0, w.ctx0), (1, w.ctx1)):
        cp, ks = ctx.equalities(ph)
        ocp, oks = _oracle_lists(w, octx)
        assert [tuple(int(x) for x in r) for r in cp] == ocp, ph
        assert ks == oks, ph
    ctx.close()


def test_equalities_cover_every_copy_kind():
    """Sanity on one witness: cross-phase sources, init_rand, constant cells,
    and every oracle constant value present."""
    m, u, d, v = gen_svd_input(4, 3, seed=5)
    ctx = hs.Context(device=-1, precision_bits=32, lookup_bits=19)
    hs.svd_witness(ctx, m, u, v, d, gamma_for(5))
    cp1, ks1 = ctx.equalities(1)
    assert (cp1[:, 0] == 0).any() and (cp1[:, 0] == 1).any() and (cp1[:, 0] == 2).any()
    cp0, ks0 = ctx.equalities(0)
    assert (cp0[:, 0] == 0).all()
    assert {v for _, v in ks0} >= {0, 1}
    ctx.close()


@pytest.mark.parametrize("n,k,m,P", [(5, 7, 4, 32), (6, 6, 6, 63), (1, 3, 1, 42)])
def test_modular_verify_mul_equalities(n, k, m, P):
    """BASELINE config 2's recipe through the modular API (ZkMatrix::new x2,
    honest_prover_mat_mul, verify_mul) on the dry planner vs the oracle."""
    import numpy as np
    rs = np.random.RandomState(n + k + m)
    a, b = rs.uniform(-1, 1, (n, k)), rs.uniform(-1, 1, (k, m))
    g = gamma_for(n * k * m)
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=19)
    za, zb = hs.ZkMatrix.new(ctx, a), hs.ZkMatrix.new(ctx, b)
    cs = hs.honest_prover_mat_mul(ctx, za, zb)
    hs.ZkMatrix.verify_mul(ctx, za, zb, cs, g)
    o0, o1, orlc = po.Context(phase=0), po.Context(phase=1), po.Context(phase=1)
    oa, ob = po.zkmatrix_new(o0, P, a.tolist()), po.zkmatrix_new(o0, P, b.tolist())
    po.verify_mul(o1, oa, ob, po.honest_prover_mat_mul(o0, oa, ob), po.load_witness(orlc, g))

    class W:
        ctx0, ctx1 = o0, o1
    for ph, octx in ((0, o0), (1, o1)):
        cp, ks = ctx.equalities(ph)
        ocp, oks = _oracle_lists(W, octx)
        assert [tuple(int(x) for x in r) for r in cp] == ocp, ph
        assert ks == oks, ph
    ctx.close()


@pytest.mark.parametrize("P,LB", [(32, 12), (63, 19)])
def test_rescale_and_inner_product_equalities(P, LB):
    """rescale_matrix / ZkVector::inner_product (the parameterised
    signed_div_scale of svdw_div_scale, layout parity unpinned) vs the oracle."""
    import numpy as np
    rs = np.random.RandomState(P + LB)
    A, B = rs.uniform(-9, 9, (3, 4)), rs.uniform(-9, 9, (4, 2))
    x, y = rs.uniform(-3, 3, 5), rs.uniform(-3, 3, 5)
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=LB)
    za, zb = hs.ZkMatrix.new(ctx, A), hs.ZkMatrix.new(ctx, B)
    cs = hs.honest_prover_mat_mul(ctx, za, zb)
    hs.ZkMatrix.rescale_matrix(ctx, cs)
    zx, zy = hs.ZkVector.new(ctx, x), hs.ZkVector.new(ctx, y)
    zx.inner_product(zy)
    zx.norm()
    zx.dist(zy)
    o0 = po.Context(phase=0)
    rc = po.RangeChip(LB)
    oa, ob = po.zkmatrix_new(o0, P, A.tolist()), po.zkmatrix_new(o0, P, B.tolist())
    po.rescale_matrix(o0, rc, po.honest_prover_mat_mul(o0, oa, ob), P)
    ox, oy = po.zkvector_new(o0, P, x.tolist()), po.zkvector_new(o0, P, y.tolist())
    po.zkvector_inner_product(o0, rc, ox, oy, P)         # zx.inner_product(zy): self = x
    po.zkvector_norm(o0, rc, ox, P)
    po.zkvector_dist(o0, rc, ox, oy, P)

    class W:
        ctx0, ctx1 = o0, None
    cp, ks = ctx.equalities(0)
    ocp, oks = _oracle_lists(W, o0)
    assert [tuple(int(v) for v in r) for r in cp] == ocp
    assert ks == oks
    ctx.close()


@pytest.mark.parametrize("N,M,P", [(4, 4, 32), (5, 3, 63)])
def test_rlc_prefix_equalities(N, M, P):
    """rlc_prefix: load_rlc_cache(.., 1)'s two ctx_gate constants head phase 1
    and init_rand is RLC cell 2 (recalled axiom-eth construction, parity
    unpinned): the lists shift with the stream and still match the oracle."""
    m, u, d, v = gen_svd_input(N, M, seed=3)
    g = gamma_for(9)
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=19)
    ctx.set_option("rlc_prefix", 1)
    hs.svd_witness(ctx, m, u, v, d, g)
    w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), d.tolist(), P, 19, gamma=g, rlc_prefix=True)
    for ph, octx in ((0, w.ctx0), (1, w.ctx1)):
        cp, ks = ctx.equalities(ph)
        ocp, oks = _oracle_lists(w, octx)
        assert [tuple(int(x) for x in r) for r in cp] == ocp, ph
        assert ks == oks, ph
    _, ks1 = ctx.equalities(1)
    assert ks1[:2] == [(0, 1), (1, 0)]
    ctx.close()
