import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

P_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def gen_svd_input(N, M, seed):
    """input-creator.py:23-30 recipe with a seeded RandomState (same call order)."""
    rs = np.random.RandomState(seed)
    m = rs.uniform(-10, 10, size=(N, M))
    m = m / np.linalg.norm(m, ord=2) * rs.uniform(1, 100)
    U, D, V = np.linalg.svd(m)
    return m, U, D, V


def gamma_for(seed) -> int:
    """Fixed Fiat-Shamir stand-in: SHA-256("svdw-gamma-<seed>") mod p."""
    return int.from_bytes(hashlib.sha256(f"svdw-gamma-{seed}".encode()).digest(), "little") % P_MOD


def have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx_factory():
    if not have_gpu():
        pytest.skip("no HIP device")
    import halo2_svd041_amd as hs
    hs.zk.lib()  # raises loudly if libsvdw.so is missing
    ctxs = []

    def make(p, lb=19):
        c = hs.Context(device=0, precision_bits=p, lookup_bits=lb)
        ctxs.append(c)
        return c
    yield make
    for c in ctxs:
        c.close()


# Regions of a witness that the C oracle's sampled mode (row window) restricts to
# rows [row_begin, row_begin + row_lim); every other region it computes in full.
ROW_LIMITED = {"check_mat_entries_bounded", "mat_times_diag_mat", "product", "check_mat_diff",
               "scan", "verify_mul_is_equal"}


def walk_window(layout, get, want, row_begin, row_lim, owned=None):
    """Compare the cells of a full-size witness (get(phase, lookup, off, n) ->
    (n, 4) uint64, whole-witness offsets from the engine's layout table) with
    the C oracle's sampled witness `want` {(phase, lookup): cells}: every region
    in full, except the row-parallel ones (ROW_LIMITED), of which only the rows
    [row_begin, row_begin + row_lim) exist in `want`. owned: {(phase, lookup):
    [(begin, end), ...]} restricts the comparison to those cells (a row-sharded
    rank's). Returns the cells compared."""
    pos = {k: 0 for k in want}
    compared = 0
    for r in layout:
        ph, rows = r["phase"], r["rows"]
        limited = r["tag"] in ROW_LIMITED
        r0 = min(row_begin, rows) if limited else 0
        r1 = min(row_begin + row_lim, rows) if limited else rows
        for lk, off, n in ((0, r["off"], r["n"]), (1, r["loff"], r["nl"])):
            if not n or (ph, lk) not in want:
                continue
            unit = n // rows
            take = (r1 - r0) * unit
            got = get(ph, lk, off + r0 * unit, take)
            ref = want[(ph, lk)][pos[(ph, lk)]:pos[(ph, lk)] + take]
            diff = np.any(got != ref, axis=1)
            if owned is not None:
                keep = np.zeros(take, dtype=bool)
                a = off + r0 * unit
                for b0, b1 in owned.get((ph, lk), []):
                    lo, hi = max(b0, a), min(b1, a + take)
                    if lo < hi:
                        keep[lo - a:hi - a] = True
                diff &= keep
                compared -= take - int(keep.sum())
            bad = np.nonzero(diff)[0]
            assert bad.size == 0, (f"{r['tag']} phase {ph} {'lookup' if lk else 'advice'} rows "
                                   f"[{r0}, {r1}): {bad.size} of {take} cells differ, first at {bad[:6]}")
            pos[(ph, lk)] += take
            compared += take
    for k, w in want.items():                      # the walk consumed every oracle cell
        assert pos[k] == w.shape[0], (k, pos[k], w.shape[0])
    return compared
