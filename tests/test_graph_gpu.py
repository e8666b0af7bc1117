"""Captured verify_mul_witness (option "graph", engine.cpp verify_mul_witness_api).

The second device-input call of a key is captured into a HIP graph and later
calls replay it, with k_gamma_prep queued ahead of the graph. Every call's cells,
gate checks and equality records must be those of an eager call with the same
inputs and gamma: the full advice streams are compared with the C oracle
(oracle/svdw_oracle.c, README.md:32-46's recipe) after each call, and with a
graph-off context.
"""
import numpy as np
import pytest

import corc
from conftest import gamma_for


def _mats(n, k, m, seed):
    rs = np.random.RandomState(seed)
    return rs.uniform(-1, 1, (n, k)), rs.uniform(-1, 1, (k, m))


def _check_all(ctx, a, b, P, g):
    c0, c1 = corc.verify_mul_witness(a, b, P, g)
    assert np.array_equal(ctx.advice(0), c0), "phase-0 advice differs from the C oracle"
    assert np.array_equal(ctx.advice(1), c1), "phase-1 advice differs from the C oracle"
    chk = ctx.check_gates()
    assert chk["gate_failures"] == 0 and chk["lookup_failures"] == 0 and chk["copy_failures"] == 0
    eq = ctx.check_equalities(1)
    assert eq["copy_failures"] == 0 and eq["const_failures"] == 0 and eq["copies_checked"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,m,P", [(256, 256, 256, 32), (45, 130, 37, 63), (3, 2, 1, 32)])
def test_graph_replays_match_oracle(gpu_ctx_factory, n, k, m, P):
    """Five calls on the same input tensors (new values written in place) with a
    fresh gamma each: eager, then captured, then replayed (the checks between
    calls allocate their scratch on the first pass, which bumps the buffer
    epoch once: capture on call 3, replays on calls 4-5)."""
    import torch
    import halo2_svd041_amd as hs
    ctx = gpu_ctx_factory(P)
    ctx.set_option("lanes", 1)                        # (counts of one state's graph)
    ta = torch.empty((n, k), dtype=torch.float64, device="cuda:0")
    tb = torch.empty((k, m), dtype=torch.float64, device="cuda:0")
    for it in range(5):
        a, b = _mats(n, k, m, seed=100 * it + n)
        ta.copy_(torch.from_numpy(a))
        tb.copy_(torch.from_numpy(b))
        g = gamma_for(it + 7 * n)
        hs.verify_mul_witness(ctx, ta, tb, g)
        _check_all(ctx, a, b, P, g)
    assert ctx.graph_stats() == (1, 2)


@pytest.mark.gpu
def test_graph_pipelined_calls_keep_gamma_order(gpu_ctx_factory):
    """Replays queued back to back without a host sync: each call's gamma tables
    are written on the context stream after the previous graph has finished, so
    the last call's cells carry the last gamma only."""
    import torch
    import halo2_svd041_amd as hs
    n = k = m = 96
    P = 32
    a, b = _mats(n, k, m, seed=5)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    ctx = gpu_ctx_factory(P)
    ctx.set_option("lanes", 1)                        # (counts of one state's graph)
    for it in range(8):
        hs.verify_mul_witness(ctx, ta, tb, gamma_for(it))
    _check_all(ctx, a, b, P, gamma_for(7))
    cap, rep = ctx.graph_stats()
    assert cap == 1 and rep == 6


@pytest.mark.gpu
def test_graph_off_and_invalidation(gpu_ctx_factory):
    """Graph on / off give identical streams; an option change, a different shape
    or new input pointers drop the graph (the next calls recapture)."""
    import torch
    import halo2_svd041_amd as hs
    P = 32
    a, b = _mats(64, 40, 50, seed=9)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    on, off = gpu_ctx_factory(P), gpu_ctx_factory(P)
    for x in (on, off):
        x.set_option("lanes", 1)
    off.set_option("graph", 0)
    for it in range(4):
        g = gamma_for(40 + it)
        hs.verify_mul_witness(on, ta, tb, g)
        hs.verify_mul_witness(off, ta, tb, g)
        assert np.array_equal(on.advice(0), off.advice(0)) and np.array_equal(on.advice(1), off.advice(1))
        assert on.layout() == off.layout()
    assert on.graph_stats() == (1, 2) and off.graph_stats() == (0, 0)
    on.set_option("stage_batch", 1)                      # any option change: recapture
    for it in range(3):
        hs.verify_mul_witness(on, ta, tb, gamma_for(50 + it))
    assert on.graph_stats() == (2, 3)
    _check_all(on, a, b, P, gamma_for(52))
    a2, b2 = _mats(30, 40, 20, seed=3)                    # another shape, then back
    t2a, t2b = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a2, b2))
    hs.verify_mul_witness(on, t2a, t2b, gamma_for(60))
    _check_all(on, a2, b2, P, gamma_for(60))
    for it in range(3):
        hs.verify_mul_witness(on, ta, tb, gamma_for(61 + it))
        _check_all(on, a, b, P, gamma_for(61 + it))
    assert on.graph_stats() == (3, 4)


@pytest.mark.gpu
def test_graph_replay_after_svd_witness(gpu_ctx_factory):
    """A replay after another call on the same context: the captured graph's
    host state (layout, checks, constants, counts, product bounds) must be
    restored over whatever svd_witness left, with nothing reallocated in
    between (the svd witness runs first at the same sizes, so the second one
    grows nothing and the epoch, hence the graph, survives). A pipelined
    svd_witness alternates between two cell sets: two calls allocate both, and
    the graph replays only on the set it was captured on (part of its key)."""
    import torch
    import halo2_svd041_amd as hs
    from conftest import gen_svd_input
    P = 32
    a, b = _mats(64, 40, 50, seed=21)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    m, u, d, v = gen_svd_input(48, 40, seed=22)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device="cuda:0")
                      for x in (m, u, v, d))
    ctx = gpu_ctx_factory(P)
    ctx.set_option("lanes", 1)                        # (counts of one state's graph)
    for k in range(2):
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(69 + k))
    for it in range(3):                                   # eager, capture, replay
        hs.verify_mul_witness(ctx, ta, tb, gamma_for(71 + it))
    c0, c1 = corc.verify_mul_witness(a, b, P, gamma_for(73))   # (no checker here: its scratch
    assert np.array_equal(ctx.advice(0), c0) and np.array_equal(ctx.advice(1), c1)   # would bump the epoch)
    assert ctx.graph_stats() == (1, 1)
    for k in range(2):                                    # (back on the graph's cell set)
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(74))
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, gamma_for(74))
    assert np.array_equal(ctx.advice(0), a0) and np.array_equal(ctx.advice(1), a1)
    hs.verify_mul_witness(ctx, ta, tb, gamma_for(75))
    assert ctx.graph_stats() == (1, 2), "the svd witness reallocated: no replay was tested"
    _check_all(ctx, a, b, P, gamma_for(75))


@pytest.mark.gpu
def test_lanes_alternate_match_oracle(gpu_ctx_factory):
    """lanes 2: consecutive verify_mul_witness calls alternate between two
    complete context states (streams, cells, scratch, graph), exchanged behind
    the handle at each call, so the handle shows the latest call's cells. Ten
    calls with new values and gamma, each checked (cells, gates, equalities):
    each state captures on its third call and replays after."""
    import torch
    import halo2_svd041_amd as hs
    P, n, k, m = 32, 64, 48, 40
    ctx = gpu_ctx_factory(P)
    ctx.set_option("lanes", 2)
    ta = torch.empty((n, k), dtype=torch.float64, device="cuda:0")
    tb = torch.empty((k, m), dtype=torch.float64, device="cuda:0")
    for it in range(10):
        a, b = _mats(n, k, m, seed=300 + it)
        ta.copy_(torch.from_numpy(a))
        tb.copy_(torch.from_numpy(b))
        g = gamma_for(900 + it)
        hs.verify_mul_witness(ctx, ta, tb, g)
        _check_all(ctx, a, b, P, g)
    assert ctx.graph_stats() == (2, 4)


@pytest.mark.gpu
def test_lanes_back_to_back_then_svd(gpu_ctx_factory):
    """lanes 2 without a host wait between calls (call j + 1 runs beside call
    j on the other state's streams): the last call's witness matches the
    oracle; then an svd_witness and another verify_mul on the same handle."""
    import torch
    import halo2_svd041_amd as hs
    from conftest import gen_svd_input
    P = 32
    ctx = gpu_ctx_factory(P)
    ctx.set_option("lanes", 2)
    a, b = _mats(96, 80, 72, seed=41)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    for it in range(9):
        hs.verify_mul_witness(ctx, ta, tb, gamma_for(950 + it))
    c0, c1 = corc.verify_mul_witness(a, b, P, gamma_for(958))
    assert np.array_equal(ctx.advice(0), c0) and np.array_equal(ctx.advice(1), c1)
    assert ctx.graph_stats()[1] >= 2
    mm, u, d, v = gen_svd_input(40, 36, seed=43)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device="cuda:0")
                      for x in (mm, u, v, d))
    hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(960))
    a0, l0, a1 = corc.svd_witness(mm, u, v, d, P, 19, gamma_for(960))
    assert np.array_equal(ctx.advice(0), a0) and np.array_equal(ctx.advice(1), a1)
    hs.verify_mul_witness(ctx, ta, tb, gamma_for(961))
    _check_all(ctx, a, b, P, gamma_for(961))


@pytest.mark.gpu
def test_pipelined_svd_and_lanes_interleaved(gpu_ctx_factory):
    """svd_witness (pipelined, alternating cell sets and gamma tables) and
    verify_mul_witness (two lanes, captured graphs) interleaved on one handle,
    six rounds, with no host wait except where cells are read: the svd
    witness is read (and compared with the oracle) right after its call in
    rounds 2 and 5, the verify_mul witness right after its call in rounds 1
    and 4 (each read synchronises the handle; the other rounds run back to
    back), and the last svd witness again at the end."""
    import torch
    import halo2_svd041_amd as hs
    from conftest import gen_svd_input
    P = 32
    ctx = gpu_ctx_factory(P)
    a, b = _mats(72, 56, 48, seed=61)
    ta, tb = (torch.tensor(x, dtype=torch.float64, device="cuda:0") for x in (a, b))
    mm, u, d, v = gen_svd_input(44, 38, seed=62)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device="cuda:0")
                      for x in (mm, u, v, d))
    for r in range(6):
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(970 + r))
        if r in (2, 5):
            s0, sl0, s1 = corc.svd_witness(mm, u, v, d, P, 19, gamma_for(970 + r))
            assert np.array_equal(ctx.advice(0), s0) and np.array_equal(ctx.advice(1), s1), r
            assert np.array_equal(ctx.lookups(0), sl0), r
        hs.verify_mul_witness(ctx, ta, tb, gamma_for(980 + r))
        if r in (1, 4):
            c0, c1 = corc.verify_mul_witness(a, b, P, gamma_for(980 + r))
            assert np.array_equal(ctx.advice(0), c0) and np.array_equal(ctx.advice(1), c1), r
    hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(990))
    a0, l0, a1 = corc.svd_witness(mm, u, v, d, P, 19, gamma_for(990))
    assert np.array_equal(ctx.advice(0), a0) and np.array_equal(ctx.advice(1), a1)
    assert np.array_equal(ctx.lookups(0), l0)
