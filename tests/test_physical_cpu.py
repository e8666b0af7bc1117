"""Virtual -> physical layout plan (svdw_physical_layout)
on the engine's dry planner, against the oracle's restatement
(oracle/pyoracle.py physical_layout) on the same witness.

Parity unpinned: the assignment rule is halo2-base 0.4.1's, which is not on
disk here (recalled). What these tests pin is that the engine
and the oracle agree on it, and the rule's invariants."""
import pytest

import halo2_svd041_amd as hs
import pyoracle as po
from conftest import gamma_for, gen_svd_input


def _both(N, M, P, g=3):
    m, u, d, v = gen_svd_input(N, M, seed=N * 10 + M + P)
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=19)
    hs.svd_witness(ctx, m, u, v, d, g)
    w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), d.tolist(), P, 19, gamma=g)
    return ctx, w


@pytest.mark.parametrize("N,M,P", [(4, 4, 32), (5, 3, 63), (3, 6, 42)])
@pytest.mark.parametrize("k", [6, 7, 9, 12])
def test_plan_matches_oracle(N, M, P, k):
    ctx, w = _both(N, M, P)
    p = ctx.physical_layout(k, 20)
    assert p["max_rows"] == (1 << k) - 20
    for ph, wc in ((0, w.ctx0), (1, w.ctx1)):
        o = po.physical_layout(wc, k, 20)
        assert ctx.break_points(ph) == o.break_points, ph
        assert p["columns_used"][ph] == len(o.columns)
        assert p["num_advice"][ph] == o.num_advice
        assert p["num_lookup_advice"][ph] == len(o.lookup_columns) == o.num_lookup_advice
    consts = {c % po.P_MOD for _, c in w.ctx0.consts} | {c % po.P_MOD for _, c in w.ctx1.consts}
    assert p["constants"] == len(consts)
    assert p["num_fixed"] == 1
    ctx.close()


@pytest.mark.parametrize("k", [6, 8, 10])
def test_oracle_layout_invariants(k):
    """Every enabled selector's gate lies inside its column and holds; removing
    each repeated break cell gives back the virtual stream; only the last
    column may be shorter than a break."""
    m, u, d, v = gen_svd_input(4, 4, seed=7)
    w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), d.tolist(), 32, 19, gamma=gamma_for(1))
    o = po.physical_layout(w.ctx0, k, 20)
    R = o.max_rows
    flat = []
    for c, (col, sel) in enumerate(zip(o.columns, o.selectors)):
        assert len(col) <= R
        if c + 1 < len(o.columns):
            assert len(col) == o.break_points[c] + 1 and col[-1] == o.columns[c + 1][0]
            assert sel[-1] == 0
        for r, q in enumerate(sel):
            if q:
                assert r + 4 <= R
                a, b, cc, dd = col[r:r + 4]
                assert (a + b * cc - dd) % po.P_MOD == 0
        flat += col if c + 1 == len(o.columns) else col[:-1]
    assert flat == w.ctx0.advice
    assert sum(map(sum, o.selectors)) == len(w.ctx0.gates)


def test_plan_errors():
    ctx = hs.Context(device=-1, precision_bits=32, lookup_bits=19)
    with pytest.raises(hs.SvdwError):
        ctx.physical_layout(4, 20)              # minimum_rows >= 2^k - 4
    with pytest.raises(hs.SvdwError):
        ctx.break_points(0)                     # no plan yet
    ctx.close()
