"""svdw_check_equalities: every copy-constraint record of the witness
(svdw_equalities, the lists tests/test_equalities_cpu.py pins against the
oracle) checked on the device -- on the virtual cell streams and on the
assigned physical columns (svdw_assign_columns), where each record's cells sit
at their first placement. Honest witnesses satisfy every record; the
README.md:93 known answer (matrix-wrong) breaks some exactly when the oracle's
own constraint checker finds failing copies (P >= 42)."""
import numpy as np
import pytest

from conftest import gamma_for, gen_svd_input

pytestmark = pytest.mark.gpu


def _oracle_copy_failures(w):
    import pyoracle as po
    bad = po.check_constraints(w.ctx0, 19) + po.check_constraints(w.ctx1, 19)
    return sum(b.startswith("copy") or b.startswith("const") for b in bad)


@pytest.mark.parametrize("N,M,P", [(4, 4, 32), (6, 5, 63), (5, 7, 42), (1, 1, 32), (40, 33, 63)])
def test_equalities_hold_on_streams(gpu_ctx_factory, N, M, P):
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N * 3 + M + P)
    ctx = gpu_ctx_factory(P)
    hs.svd_witness(ctx, m, u, v, d, gamma_for(P + 1))
    for ph in (0, 1):
        cp, ks = ctx.equalities(ph)
        r = ctx.check_equalities(ph)
        assert r == {"copies_checked": len(cp), "copy_failures": 0,
                     "consts_checked": len(ks), "const_failures": 0}, (ph, r)


@pytest.mark.parametrize("P,expect_fail", [(32, False), (42, True), (63, True)])
def test_matrix_wrong_breaks_equalities(gpu_ctx_factory, P, expect_fail):
    import halo2_svd041_amd as hs
    import pyoracle as po
    m, u, d, v = gen_svd_input(6, 6, seed=11)
    m = m.copy()
    m[2][3] += 1e-7                        # input-creator.py:46-49
    ctx = gpu_ctx_factory(P)
    hs.svd_witness(ctx, m, u, v, d, 3)
    fails = sum(ctx.check_equalities(ph)["copy_failures"] for ph in (0, 1))
    w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), d.tolist(), P, 19, gamma=3)
    assert (fails > 0) == expect_fail == (_oracle_copy_failures(w) > 0)


@pytest.mark.parametrize("N,M,P,k", [(4, 4, 32, 7), (5, 3, 63, 9), (6, 6, 42, 11), (512, 512, 32, 22)])
def test_equalities_hold_on_physical_columns(gpu_ctx_factory, N, M, P, k):
    """Keygen's view: the records mapped through the break points onto the
    column-major advice columns of both phases (phase-1 records reach into
    phase 0's columns)."""
    import torch
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N + M + P)
    ctx = gpu_ctx_factory(P)
    hs.svd_witness(ctx, m, u, v, d, gamma_for(k))
    p = ctx.physical_layout(k, 20)
    if any(p["columns_used"][ph] > p["num_advice"][ph] for ph in (0, 1)):
        pytest.skip("plan needs more columns than the estimate")
    cols = [ctx.assign_columns(ph)[0] for ph in (0, 1)]
    torch.cuda.synchronize()
    for ph in (0, 1):
        virt = ctx.check_equalities(ph)
        phys = ctx.check_equalities(ph, cols[0], cols[1])
        assert phys == virt and phys["copy_failures"] == 0 and phys["const_failures"] == 0, (ph, phys)
        assert phys["copies_checked"] > 0


def test_shifted_columns_are_caught(gpu_ctx_factory):
    """The physical check really reads the columns: swapping two rows of an
    advice column breaks records."""
    import torch
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(5, 5, seed=2)
    ctx = gpu_ctx_factory(63)
    hs.svd_witness(ctx, m, u, v, d, gamma_for(2))
    ctx.physical_layout(9, 20)
    c0 = ctx.assign_columns(0)[0]
    c1 = ctx.assign_columns(1)[0]
    torch.cuda.synchronize()
    fails = lambda: sum(ctx.check_equalities(ph, c0, c1)["copy_failures"] for ph in (0, 1))
    assert fails() == 0
    c0[0, [1, 2]] = c0[0, [2, 1]]          # m[0][1], m[0][2]: sources of phase-1 scan copies
    torch.cuda.synchronize()
    assert fails() > 0


@pytest.mark.parametrize("N,M,P,rlc", [(6, 5, 63, 0), (33, 40, 32, 1), (128, 96, 63, 0)])
def test_device_records_equal_planner_lists(gpu_ctx_factory, N, M, P, rlc):
    """svdw_equalities on a device context generates the records on the GPU
    (k_eq_records); they equal the dry planner's host lists record for record
    (the lists tests/test_equalities_cpu.py pins against the oracle)."""
    import numpy as np
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N + 7 * M + P)
    g = gamma_for(N + M)
    ctx = gpu_ctx_factory(P)
    ctx.set_option("rlc_prefix", rlc)
    hs.svd_witness(ctx, m, u, v, d, g)
    with hs.Context(device=-1, precision_bits=P, lookup_bits=19) as dry:
        dry.set_option("rlc_prefix", rlc)
        hs.svd_witness(dry, m, u, v, d, g)
        for ph in (0, 1):
            cp_d, ks_d = ctx.equalities(ph)
            cp_h, ks_h = dry.equalities(ph)
            assert np.array_equal(cp_d, cp_h), ph
            assert ks_d == ks_h, ph


def test_full_size_equalities_on_device(gpu_ctx_factory):
    """1024^2 P=63 (29 M + 19 M copy records, 76 M constants): generated and
    checked on the device, every record holds."""
    import time
    import torch
    import halo2_svd041_amd as hs
    from bench import gen_input
    m, u, d, v = gen_input(1024, 1024, 0)
    dev = torch.device("cuda", 0)
    tm = [torch.tensor(x, dtype=torch.float64, device=dev) for x in (m, u, v, d)]
    ctx = gpu_ctx_factory(63)
    hs.svd_witness(ctx, *tm, gamma_for(1))
    t0 = time.perf_counter()
    r = [ctx.check_equalities(ph) for ph in (0, 1)]
    dt = time.perf_counter() - t0
    assert r[0]["copies_checked"] > 20_000_000 and r[0]["consts_checked"] > 50_000_000
    assert all(x["copy_failures"] == 0 and x["const_failures"] == 0 for x in r), r
    print(f"\nequality records at 1024^2: {sum(x['copies_checked'] + x['consts_checked'] for x in r) / 1e6:.1f} M "
          f"generated and checked on the device in {dt * 1e3:.1f} ms")
