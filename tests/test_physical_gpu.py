"""svdw_assign_columns: the physical advice / selector / lookup columns on the
device against the oracle's restatement (oracle/pyoracle.py physical_layout),
and at full size against the layout's own invariants (svdw_check_physical: the
basic gate at every enabled row of the physical columns, every break cell
repeated at row 0 of the next column). Parity of the rule itself unpinned
(halo2-base 0.4.1 recalled)."""
import numpy as np
import pytest

from conftest import gamma_for, gen_svd_input

pytestmark = pytest.mark.gpu


def _cells(vals, rows):
    out = np.zeros((rows, 32), dtype=np.uint8)
    for r, x in enumerate(vals):
        out[r] = np.frombuffer(int(x).to_bytes(32, "little"), dtype=np.uint8)
    return out


@pytest.mark.parametrize("N,M,P,k", [(4, 4, 32, 7), (5, 3, 63, 9), (6, 6, 42, 11)])
def test_columns_match_oracle(gpu_ctx_factory, N, M, P, k):
    import halo2_svd041_amd as hs
    import pyoracle as po
    m, u, d, v = gen_svd_input(N, M, seed=N + M + P)
    g = gamma_for(k)
    ctx = gpu_ctx_factory(P)
    hs.svd_witness(ctx, m, u, v, d, g)
    p = ctx.physical_layout(k, 20)
    w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), d.tolist(), P, 19, gamma=g)
    rows = 1 << k
    for ph, wc in ((0, w.ctx0), (1, w.ctx1)):
        o = po.physical_layout(wc, k, 20)
        if p["columns_used"][ph] > p["num_advice"][ph]:
            with pytest.raises(hs.SvdwError):
                ctx.assign_columns(ph)
            continue
        adv, sel, lk = ctx.assign_columns(ph)
        adv, sel, lk = adv.cpu().numpy(), sel.cpu().numpy(), lk.cpu().numpy()
        assert adv.shape[0] == len(o.columns) and lk.shape[0] == len(o.lookup_columns)
        for c, (col, q) in enumerate(zip(o.columns, o.selectors)):
            assert np.array_equal(adv[c], _cells(col, rows)), (ph, c)
            want = np.zeros(rows, dtype=np.uint8)
            want[:len(q)] = q
            assert np.array_equal(sel[c], want), (ph, c)
        for c, col in enumerate(o.lookup_columns):
            assert np.array_equal(lk[c], _cells(col, rows)), (ph, c)


@pytest.mark.parametrize("N,M,P,k", [(1024, 1024, 63, 24), (512, 512, 32, 22)])
def test_full_size_physical_columns(gpu_ctx_factory, N, M, P, k):
    """BASELINE sizes: every phase's columns assigned on the device; every enabled
    selector's gate holds on the physical columns, and their number equals the
    virtual witness's gates (svdw_check_gates); every break cell is repeated."""
    import torch
    import halo2_svd041_amd as hs
    m, u, d, v = gen_svd_input(N, M, seed=N + M + P)
    ctx = gpu_ctx_factory(P)
    hs.svd_witness(ctx, m, u, v, d, gamma_for(N * M))
    virt = ctx.check_gates()["gates_checked"]
    p = ctx.physical_layout(k, 20)
    gates = 0
    for ph in (0, 1):
        assert p["columns_used"][ph] <= p["num_advice"][ph], p
        adv, sel, lk = ctx.assign_columns(ph)
        torch.cuda.synchronize()
        r = ctx.check_physical(ph, adv, sel)
        assert r["gate_failures"] == 0 and r["copy_failures"] == 0, r
        assert r["copies_checked"] == p["columns_used"][ph] - 1
        gates += r["gates_checked"]
        nl = ctx.lookup_len(ph)
        if nl:                                   # lookup columns: the lookup stream in order
            R = p["max_rows"]
            got = lk[:, :R].reshape(-1, 32)[:nl]
            ref = ctx.lookups(ph, 0, nl)                 # [n, 4] u64 words
            assert np.array_equal(got.cpu().numpy().view("<u8"), ref)
        del adv, sel, lk
    assert gates == virt
