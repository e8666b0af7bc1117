"""Seeded random sweep over shapes, precisions, lookup widths and gammas: the
whole witness (advice + lookup streams) bit-exact against the C oracle, and the
device constraint checker passes on every honest input. Tall, wide, square and
degenerate (1-row / 1-column) shapes; P over [32, 63]; LB over [10, 24]."""
import numpy as np
import pytest

import corc
from conftest import gamma_for, gen_svd_input

pytestmark = pytest.mark.gpu


def _cases(n=36, seed=2024):
    rs = np.random.RandomState(seed)
    out = []
    for i in range(n):
        N = int(rs.randint(4, 49) if rs.rand() < 0.7 else rs.randint(1, 4))
        M = int(rs.randint(4, 49) if rs.rand() < 0.7 else rs.randint(1, 4))
        out.append((N, M, int(rs.randint(32, 64)), int(rs.randint(10, 25)), int(rs.randint(1 << 30))))
    return out


@pytest.mark.parametrize("N,M,P,LB,seed", _cases())
def test_random_witness_parity(gpu_ctx_factory, N, M, P, LB, seed):
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=seed)
    g = gamma_for(seed)
    ctx = gpu_ctx_factory(P, LB)
    cnt = hs.svd_witness(ctx, m, u, v, d, g)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, LB, g)
    assert (cnt["advice0"], cnt["lookup0"], cnt["advice1"]) == (a0.shape[0], l0.shape[0], a1.shape[0])
    for name, got, ref in (("advice0", ctx.advice(0), a0), ("lookup0", ctx.lookups(0), l0),
                           ("advice1", ctx.advice(1), a1)):
        bad = np.nonzero(np.any(got != ref, axis=1))[0]
        assert bad.size == 0, f"{name}: {bad.size} cells differ, first at {bad[:8]}"
    r = ctx.check_gates()
    assert r["gate_failures"] == 0 and r["copy_failures"] == 0 and r["lookup_failures"] == 0, r
