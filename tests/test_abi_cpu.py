"""C-ABI boundary checks that need no GPU: the HIP library loads and exports
every function include/svdw.h declares, the planning (dry) context gives the
exact cell counts of the oracle, host-side argument / shape errors map to the
documented codes, and err_calc matches the reference expression."""
import ctypes as ct
import os
import re

import numpy as np
import pytest

import corc
import halo2_svd041_amd as hs
from halo2_svd041_amd import _lib
from conftest import ROOT, gen_svd_input

HEADER = os.path.join(ROOT, "include", "svdw.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(svdw_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = ct.CDLL(_lib.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(declared_functions()) == set(_lib.SIGNATURES)


@pytest.mark.parametrize("N,M,P,LB", [(1, 1, 32, 19), (4, 4, 32, 19), (4, 3, 63, 19),
                                      (3, 4, 42, 19), (9, 9, 40, 13), (7, 5, 63, 8),
                                      (16, 24, 63, 17), (33, 17, 32, 63)])
def test_planner_counts_match_oracle(N, M, P, LB):
    m, u, d, v = gen_svd_input(N, M, seed=N + M)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, LB, 3)
    plan = hs.plan_svd(N, M, P, LB)
    assert plan == {"advice0": a0.shape[0], "advice1": a1.shape[0], "lookup0": l0.shape[0],
                    "lookup1": 0}


def test_planner_baseline_configs():
    """BASELINE.md §2 derived totals (Appendix B closed form)."""
    assert hs.plan_svd(512, 512, 32, 19) == {"advice0": 35406321, "advice1": 7107063,
                                             "lookup0": 6820859, "lookup1": 0}
    assert hs.plan_svd(1024, 1024, 63, 19) == {"advice0": 210803694, "advice1": 28369911,
                                               "lookup0": 50343930, "lookup1": 0}
    assert hs.plan_svd(2048, 1024, 32, 19) == {"advice0": 335578097, "advice1": 63006711,
                                               "lookup0": 65021947, "lookup1": 0}
    assert hs.plan_svd(256, 256, 32, 19)["advice0"] == 8855793


def test_planner_readme_coefficients_at_scale():
    """README.md:67 at N = 1000: advice 162 N^2 / 228 N^2 (+ O(N)), lookups 26 / 48 N^2."""
    for P, adv, lk in ((32, 162, 26), (63, 228, 48)):
        c = [hs.plan_svd(n, n, P, 19) for n in (992, 1000, 1008)]
        tot = [x["advice0"] + x["advice1"] for x in c]
        assert (tot[2] - 2 * tot[1] + tot[0]) / (2 * 64) == adv
        lks = [x["lookup0"] for x in c]
        assert (lks[2] - 2 * lks[1] + lks[0]) / (2 * 64) == lk


def test_err_calc_matches_oracle():
    for p, size in [(32, 512), (63, 1024), (42, 4)]:
        assert hs.err_calc(p, size, 100.0, 1e-10, 1e-10) == corc.err_calc(p, size)


def test_error_codes_on_planning_context():
    with pytest.raises(hs.SvdwError) as e:
        hs.Context(device=-1, precision_bits=64, lookup_bits=19)
    assert e.value.code == -2
    with pytest.raises(hs.SvdwError) as e:
        hs.Context(device=-1, precision_bits=32, lookup_bits=4)
    assert e.value.code == -2
    ctx = hs.Context(device=-1, precision_bits=32, lookup_bits=19)
    a = hs.ZkMatrix.new(ctx, np.zeros((3, 4)))
    b = hs.ZkMatrix.new(ctx, np.zeros((3, 4)))
    with pytest.raises(hs.SvdwError) as e:       # a.num_col != b.num_rows
        hs.honest_prover_mat_mul(ctx, a, b)
    assert e.value.code == -1
    with pytest.raises(hs.SvdwError) as e:       # check_mat_diff shape mismatch
        hs.check_mat_diff(ctx, a, a.transpose_matrix(), 5)
    assert e.value.code == -1
    with pytest.raises(hs.SvdwError) as e:       # bound must be >= 1
        hs.check_mat_entries_bounded(ctx, a, 0)
    assert e.value.code == -1
    c = hs.honest_prover_mat_mul(ctx, a, b.transpose_matrix())
    assert (c.num_rows, c.num_col) == (3, 3)
    assert ctx.advice_len(0) == 24 + 9
    ctx.close()


def test_dry_modular_api_counts():
    """Cell accounting of the modular API equals the whole-witness planner."""
    N, M, P = 6, 9, 42
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=19)
    m, u, d, v = gen_svd_input(N, M, seed=1)
    zm, zu, zv = hs.ZkMatrix.new(ctx, m), hs.ZkMatrix.new(ctx, u), hs.ZkMatrix.new(ctx, v)
    zd = hs.ZkVector.new(ctx, d)
    es, eu = hs.err_calc(P, max(N, M), 100.0, 1e-10, 1e-10)
    pl = hs.check_svd_phase0(ctx, zm, zu, zv, zd, es, eu, 30)
    hs.check_svd_phase1(ctx, zm, zu, zv, pl, 5)
    plan = hs.plan_svd(N, M, P, 19)
    assert ctx.advice_len(0) == plan["advice0"] and ctx.advice_len(1) == plan["advice1"]
    assert ctx.lookup_len(0) == plan["lookup0"]
    assert (pl.m_times_vt.num_rows, pl.m_times_vt.num_col) == (N, M)
    assert (pl.u_t.num_rows, pl.v_t.num_col) == (N, M)
    ctx.close()


def test_dry_rescale_shift_only():
    """rescale_matrix with shift_bits only (>= 4P + 1): accepted, and the cell
    count is the oracle's for NB = S + 1 (the default was 4P + 1)."""
    import pyoracle as po
    P, LB, S = 32, 12, 140
    ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=LB)
    a = hs.ZkMatrix.new(ctx, np.ones((2, 3)))
    b = hs.ZkMatrix.new(ctx, np.ones((3, 2)))
    cs = hs.honest_prover_mat_mul(ctx, a, b)
    n0 = ctx.advice_len(0)
    hs.ZkMatrix.rescale_matrix(ctx, cs, S)
    o = po.Context()
    po.signed_div_scale(o, po.RangeChip(LB), po.load_witness(o, 5), P, S)
    assert ctx.advice_len(0) - n0 == 4 * (len(o.advice) - 1)
    ctx.close()


def test_removed_options_are_rejected():
    """ABI version 2: the front streamer's options, among
    them "stage_diag" (a timing diagnostic that made the engine write wrong
    cells), and the no-ops retired in ABI 1 are unknown names (SVDW_EINVAL);
    live options still set."""
    L = _lib.lib()
    assert L.svdw_abi_version() == 2
    ctx = hs.Context(device=-1, precision_bits=63, lookup_bits=19)
    try:
        for name in ("stage_diag", "stage_occ", "stage_front_all", "stage_nt", "bits_fold",
                     "prod_first", "stage_probe"):
            assert L.svdw_set_option(ctx.handle, name.encode(), 1) == -1, name
            assert b"unknown option" in L.svdw_last_error()
        ctx.set_option("stage_elems", 128)
        ctx.set_option("pipeline", 0)
    finally:
        ctx.close()


def test_completion_marks_dry():
    """svdw_mark / svdw_mark_done / svdw_mark_wait on the planning context:
    tickets count up from 1, a dry context's marks are complete at once, and a
    ticket never issued is an error."""
    import ctypes as ct
    L = _lib.lib()
    ctx = hs.Context(device=-1, precision_bits=63, lookup_bits=19)
    try:
        t = ct.c_uint64(0)
        got = []
        for _ in range(3):
            assert L.svdw_mark(ctx.handle, ct.byref(t)) == 0
            got.append(t.value)
        assert got == [1, 2, 3]
        assert L.svdw_mark_done(ctx.handle, 2) == 1
        assert L.svdw_mark_wait(ctx.handle, 3) == 0
        assert L.svdw_mark_done(ctx.handle, 0) < 0
        assert L.svdw_mark_done(ctx.handle, 4) < 0
        assert b"not issued" in L.svdw_last_error()
    finally:
        ctx.close()
