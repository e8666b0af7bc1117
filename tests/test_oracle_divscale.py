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


@pytest.mark.parametrize("x", [1 << (4 * 32 + 1), -(1 << (3 * 32 + 5))])
def test_signed_div_scale_out_of_domain_fails_constraints(x):
    """x + 2^S outside [0, 2^NB) (NB = 4P + 1 by default): the quotient bound
    check must fail (a lookup is out of range)."""
    P, LB = 32, 12
    ctx = po.Context()
    rc = po.RangeChip(LB)
    a = po.load_witness(ctx, x % po.P_MOD)
    po.signed_div_scale(ctx, rc, a, P)
    assert po.check_constraints(ctx, LB) != []


def test_cells_per_element():
    """Cells per element of the default construction (S = 3P, NB = 4P + 1):
    90 at P = 32, LB = 12 as the reference states (src/matrix/mod.rs:102
    "#CONSTRAINTS = 90", :348 "~94 (when lookup_bits = 12)"), inside README.md:51's
    60-100 per element, and NB = S + 1 for comparison."""
    def cells(P, LB):
        ctx = po.Context()
        a = po.load_witness(ctx, 5)
        po.signed_div_scale(ctx, po.RangeChip(LB), a, P)
        return len(ctx.advice) - 1
    assert cells(32, 12) == 90
    assert cells(32, 16) == 78
    assert cells(32, 19) == 66
    assert cells(32, 24) == 60
    assert cells(63, 19) == 108

    def cells_nb(P, LB, nb):
        ctx = po.Context()
        a = po.load_witness(ctx, 5)
        po.signed_div_scale(ctx, po.RangeChip(LB), a, P, 3 * P, nb)
        return len(ctx.advice) - 1
    assert cells_nb(32, 12, 97) == 72


@pytest.mark.parametrize("P,LB", [(32, 12), (42, 16), (63, 19)])
def test_qsqrt_floor_and_constraints(P, LB):
    """qsqrt (ZkVector::norm / dist's last step; parameterised, parity unpinned):
    y = floor(sqrt(a 2^P)) on [0, 2^(2P)), every constraint of the gadget holds."""
    import math
    rnd = random.Random(P + LB)
    ctx = po.Context()
    rc = po.RangeChip(LB)
    xs = [0, 1, 2, 3, (1 << P), (1 << (2 * P)) - 1] + [rnd.randrange(0, 1 << (2 * P)) for _ in range(30)]
    for x in xs:
        y = po.qsqrt(ctx, rc, po.load_witness(ctx, x), P)
        assert y.value == math.isqrt(x << P)
    assert po.check_constraints(ctx, LB) == []


def test_qsqrt_wrong_root_fails_constraints():
    """A witness y one off the floor root breaks a range check (t - y^2 < 0 or > 2y)."""
    import math
    P, LB = 32, 12
    for delta in (1, -1):
        ctx = po.Context()
        rc = po.RangeChip(LB)
        a = po.load_witness(ctx, 12345678901)
        y = po.qsqrt(ctx, rc, a, P)
        good = math.isqrt(a.value << P)
        assert y.value == good
        # rebuild with a wrong y: replay the gadget's cells with y + delta
        ctx2 = po.Context()
        a2 = po.load_witness(ctx2, a.value)
        real = math.isqrt
        try:
            math.isqrt = lambda v, _r=real, _d=delta: _r(v) + _d
            po.qsqrt(ctx2, po.RangeChip(LB), a2, P)
        finally:
            math.isqrt = real
        assert po.check_constraints(ctx2, LB) != []


def test_shift_only_widens_default_num_bits():
    """A caller that sets shift_bits only (>= 4P + 1) gets NB = S + 1, not the
    invalid NB = 4P + 1 <= S: the default is max(4P + 1, S + 1) (engine and
    oracle alike; tests/test_abi_cpu.py checks the engine's dry planner)."""
    P, LB, S = 32, 12, 140
    assert po.div_scale_defaults(P, S) == (S, S + 1)
    assert po.div_scale_defaults(P) == (3 * P, 4 * P + 1)
    ctx = po.Context()
    rc = po.RangeChip(LB)
    for x in (0, 5, -7, (1 << 139) - 3, -(1 << 139)):
        a = po.load_witness(ctx, x % po.P_MOD)
        y, _ = po.signed_div_scale(ctx, rc, a, P, S)
        assert po.to_signed(y.value) == x >> P
    assert po.check_constraints(ctx, LB) == []
