"""Oracle checks for the parameterised signed_div_scale (FixedPointChip041,
parity unpinned: the chip's source is unavailable offline; see include/svdw.h
svdw_div_scale). The construction must satisfy every gate / copy / lookup of
the oracle's constraint checker and compute floor(x / 2^P) on its domain."""
import random

import pytest

import pyoracle as po


@pytest.mark.parametrize("P,LB", [(32, 12), (32, 19), (42, 16), (63, 19)])
def test_signed_div_scale_floor_and_constraints(P, LB):
    rnd = random.Random(P * 100 + LB)
    ctx = po.Context()
    rc = po.RangeChip(LB)
    lim = 1 << (3 * P)
    xs = [rnd.randrange(-lim + 1, lim) for _ in range(40)]
    xs += [0, 1, -1, (1 << P) - 1, -(1 << P), lim - 1, -lim]
    for x in xs:
        a = po.load_witness(ctx, x % po.P_MOD)
        y, r = po.signed_div_scale(ctx, rc, a, P)
        assert po.to_signed(y.value) == x >> P
        assert r.value == x % (1 << P)
    assert po.check_constraints(ctx, LB) == []


def test_signed_div_scale_out_of_domain_fails_constraints():
    """|x| >= 2^S: the quotient bound check must fail (a lookup is out of range)."""
    P, LB = 32, 12
    ctx = po.Context()
    rc = po.RangeChip(LB)
    a = po.load_witness(ctx, (1 << (3 * P + 5)) % po.P_MOD)
    po.signed_div_scale(ctx, rc, a, P)
    assert po.check_constraints(ctx, LB) != []


def test_cells_per_element():
    """Cells per element of the default construction (documented in DESIGN.md)."""
    def cells(P, LB):
        ctx = po.Context()
        a = po.load_witness(ctx, 5)
        po.signed_div_scale(ctx, po.RangeChip(LB), a, P)
        return len(ctx.advice) - 1
    assert cells(32, 12) == 72
    assert cells(32, 19) == 54
    assert cells(63, 19) == 84
